set -o pipefail
mkdir -p gpurun_out/r17
L=awq-converter_amd/awq_quantizer/_lib
timeout -k 10 300 python scripts/kbench.py --sets opt-125m,llama3-8b-mlp --libs $L/libawq_hip.so,$L/variants/libawq_hip_triv.so --rounds 3 --iters 20 > gpurun_out/r17/kbench.log 2>&1 && grep -v '^{' gpurun_out/r17/kbench.log
LIBS=$L/libawq_hip.so,$L/variants/libawq_hip_triv.so SETS=opt-125m,llama3-8b-mlp bash scripts/gpu_pmc.sh r17/pmc
