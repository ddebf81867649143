set -o pipefail
mkdir -p gpurun_out/r45
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_f16_fast.py tests/test_scale_search.py -m gpu -x -q > gpurun_out/r45/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r45/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/generic_bench.py --shape "256,4096;1024,4096;2048,4096;4096,4096;8192,4096;14336,4096" --dtypes bf16,f16 --iters 200 --small-tiles 0,1099511627776 > gpurun_out/r45/small.log 2>&1; rc=$?; grep '^{' gpurun_out/r45/small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c1 --no-cpu-baseline > gpurun_out/r45/bench_c1.json 2> gpurun_out/r45/bench_c1.err; rc=$?; cat gpurun_out/r45/bench_c1.json; exit $rc
