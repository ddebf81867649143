set -o pipefail
# round refresh: smoke, GPU suite, bench (defaults), extra lines, rocprof + PMC
PROFILE=0 bash scripts/gpu_round.sh r80 && bash scripts/profile_round.sh r80 && \
for X in "--dtype f16" "--dtype f32" "--group-size 64" "--group-size 32"; do
  N=$(echo $X | tr -d ' -'); timeout -k 10 300 python bench.py $X --no-cpu-baseline > gpurun_out/r80/bench_$N.log 2>&1 || exit 1
  grep '^{"metric"' gpurun_out/r80/bench_$N.log | cut -c1-200
done
