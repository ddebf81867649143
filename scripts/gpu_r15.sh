set -o pipefail
mkdir -p gpurun_out/r15
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r15/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r15/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --events step > gpurun_out/r15/bench_step.json 2> gpurun_out/r15/bench_step.err && cat gpurun_out/r15/bench_step.json
timeout -k 10 300 python bench.py --events span --no-cpu-baseline > gpurun_out/r15/bench_span.json 2>&1 && cat gpurun_out/r15/bench_span.json
bash scripts/profile_round.sh r15
