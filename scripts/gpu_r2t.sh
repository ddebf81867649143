#!/bin/bash
# round 2: 70B inputs in one arena vs per-tensor allocations (kernel-only, same library),
# extra bench lines (dtypes, group size, other sets) at one wave per workgroup, and a
# cProfile of the CLI device thread on opt-350m
set -u
OUT=gpurun_out/r2t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python scripts/kbench.py --sets llama3-70b --rounds 3 --iters 10 > $OUT/kbench_70b_separate.log 2>&1 || exit $?
timeout -k 10 300 python scripts/kbench.py --sets llama3-70b --rounds 3 --iters 10 --arena > $OUT/kbench_70b_arena.log 2>&1 || exit $?
for A in "--workload llama3-8b" "--workload opt-125m --steps 200 --warmup 20" "--workload llama3-8b --dtype f16" "--workload llama3-8b --dtype f32" "--workload llama3-8b --group-size 64" "--workload llama3-8b --bits 8" "--workload llama3-8b --symmetric"; do
  N=$(echo $A | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py $A --no-cpu-baseline > $OUT/bench_$N.log 2>&1 || exit $?
done
W=/tmp/awq_cli_r2t
mkdir -p $W
AWQ_CLI_PROFILE=$OUT/cli_opt350m.prof timeout -k 10 300 python scripts/cli_bench.py --workload opt-350m --format packed --workdir $W --repeat 2 > $OUT/cli_opt350m.log 2>&1 || exit $?
python -c "
import pstats; p = pstats.Stats('$OUT/cli_opt350m.prof'); p.sort_stats('tottime').print_stats(25)" > $OUT/cli_opt350m_profile.txt 2>&1
rm -rf $W
echo done
