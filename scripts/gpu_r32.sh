set -o pipefail
mkdir -p gpurun_out/r32
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r32/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r32/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r32/bench.json 2> gpurun_out/r32/bench.err; rc=$?; cat gpurun_out/r32/bench.json; [ $rc -eq 0 ] || exit $rc
bash scripts/profile_round.sh r32 || exit $?
for w in c1 opt-350m llama3-8b; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r32/bench_$w.json 2>gpurun_out/r32/bench_$w.err || exit $?
  cat gpurun_out/r32/bench_$w.json
done
