set -o pipefail
mkdir -p gpurun_out/r23
bash scripts/profile_round.sh r23 || exit $?
for w in c1 opt-350m llama3-8b; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r23/bench_$w.json 2>gpurun_out/r23/bench_$w.err || exit $?
  cat gpurun_out/r23/bench_$w.json
done
timeout -k 10 300 python bench.py --events step --no-cpu-baseline > gpurun_out/r23/bench_step.json 2>/dev/null && cat gpurun_out/r23/bench_step.json
