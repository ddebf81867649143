set -o pipefail
mkdir -p gpurun_out/r28
L=awq-converter_amd/awq_quantizer/_lib
V=$L/variants/libawq_hip_
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r28/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r28/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/kbench.py --sets opt-125m,llama3-8b-mlp,k768,c1x64,c1 --libs $L/libawq_hip.so,${V}triv.so --blocks 0,nt --rounds 3 --iters 10 > gpurun_out/r28/kbench.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r28/kbench.log; [ $rc -eq 0 ] || exit $rc
for s in opt-125m llama3-8b-mlp; do timeout -k 10 200 python scripts/trace_waves.py --set $s --lib ${V}trace.so > gpurun_out/r28/trace_$s.log 2>&1 || exit 1; grep '^{' gpurun_out/r28/trace_$s.log | tail -4; done
