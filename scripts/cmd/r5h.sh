# round 5: activation-aware loss kernel A/B (table prefetch, 8 elements per lane, occupancy)
# + the full GPU suite and smoke on the current tree
set -u
AB="python scripts/act_search_bench.py --iters 5"
steps=()
for rnd in 1 2; do
  for v in base pf1 pf2 epl8 w5 pf1w4 epl8pf2 epl8pf1; do
    steps+=("act_${v}_$rnd:120:$AB --lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_$v.so")
  done
done
bash scripts/gpu_run.sh r5h pytest smoke "${steps[@]}"
