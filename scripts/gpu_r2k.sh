#!/bin/bash
# round 2: CLI end-to-end before/after the pinned asynchronous table uploads (same box,
# same model files): AWQ_PAGEABLE_TABLES=1 is the round-1 path
set -u
OUT=gpurun_out/r2k
mkdir -p $OUT
export TMPDIR=/tmp
W=/tmp/awq_cli_r2k
mkdir -p $W
for WL in opt-350m opt-125m; do
  for FMT in packed reference; do
    for PG in 1 0 1 0; do
      AWQ_PAGEABLE_TABLES=$PG timeout -k 10 300 python scripts/cli_bench.py --workload $WL --format $FMT --workdir $W/$WL --repeat 2 >> $OUT/cli_${WL}_${FMT}_pageable$PG.log 2>&1 || exit $?
    done
  done
done
rm -rf $W
echo done
