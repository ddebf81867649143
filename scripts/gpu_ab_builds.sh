#!/bin/bash
# A/B of two in-tree builds of libawq_hip.so on the row-segment shapes, alternating processes:
#   bash scripts/gpu_ab_builds.sh <tag> <lib_a> <lib_b> [rounds]
set -u
TAG=$1; A=$2; B=$3; N=${4:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
GB="python scripts/generic_bench.py --shape 14336,4096;4096,14336;8192,3000 --dtypes bf16,f16,f32 --group-sizes 100,48,200,96 --iters 30"
for i in $(seq 1 "$N"); do
  for L in "$A" "$B"; do
    timeout -k 10 200 $GB --lib "$L" >> "$OUT/ab_builds.log" 2>&1 || { echo "bench failed ($L)"; exit 1; }
  done
done
echo done
