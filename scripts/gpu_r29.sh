set -o pipefail
mkdir -p gpurun_out/r29
L=awq-converter_amd/awq_quantizer/_lib
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r29/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r29/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/kbench.py --sets opt-125m,llama3-8b-mlp,k768,c1x64,c1 --blocks 0,nt --rounds 3 --iters 10 > gpurun_out/r29/kbench.log 2>&1; rc=$?; grep -v '^{' gpurun_out/r29/kbench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r29/bench.json 2> gpurun_out/r29/bench.err; rc=$?; cat gpurun_out/r29/bench.json; exit $rc
