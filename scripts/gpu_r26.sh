set -o pipefail
mkdir -p gpurun_out/r26
timeout -k 10 600 python scripts/kbench.py --sets opt-125m,llama3-8b-mlp,k768,c1x64 --blocks 0,4096,8192,16384,32768,1000000 --rounds 3 --iters 10 > gpurun_out/r26/kbench.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r26/kbench.log; exit $rc
