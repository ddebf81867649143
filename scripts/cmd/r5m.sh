# round 5: act loss kernel with the LDS-DMA table ring (product) vs the register-load kernel
set -u
AB="python scripts/act_search_bench.py --iters 5"
L=awq-converter_amd/awq_quantizer/_lib/ab
steps=("pytest=tests/test_act_search.py")
for rnd in 1 2 3; do
  for dt in bf16 f16; do
    steps+=("a_lds_${dt}_$rnd:120:$AB --dtype $dt" "a_old_${dt}_$rnd:120:$AB --dtype $dt --lib $L/libawq_hip_actold.so")
  done
done
bash scripts/gpu_run.sh r5m "${steps[@]}"
