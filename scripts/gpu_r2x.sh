#!/bin/bash
# round 2: row-segment pass 2 per-half parameters (SPLIT 4 / 8 templates): parity, then
# throughput per group size and a groups-per-tile sweep at group size 100; activation-aware
# search with the sub-block summation orders: parity, timing, per-kernel rocprof stats
set -u
OUT=gpurun_out/r2x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rowgroup.py tests/test_gpu_group_sizes.py tests/test_act_search.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 300 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16,f16,f32 --group-sizes 100,48,96,60,200,300 > $OUT/gs_sweep.log 2>&1 || exit $?
for G in 8 16 32; do
  AWQ_RG_GPT=$G timeout -k 10 120 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16 --group-sizes 100,60,200 > $OUT/gpt$G.log 2>&1 || exit $?
done
timeout -k 10 300 python scripts/act_search_bench.py --tokens 512 --grid 20 > $OUT/act_search_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_act -o act -- python scripts/act_search_bench.py --tokens 512 --grid 20 --iters 2 > $OUT/act_prof.log 2>&1 || exit $?
echo done
