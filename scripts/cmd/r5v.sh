# round 5: act loss kernel with x_sq read from the LDS ring (hlds) vs held in VGPRs (product)
set -u
AB="python scripts/act_search_bench.py --iters 5"
L=awq-converter_amd/awq_quantizer/_lib/ab
steps=("t_hlds:300:AWQ_TEST_LIB=$L/libawq_hip_hlds.so python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_act_search.py")
for rnd in 1 2 3; do
  for dt in bf16 f16; do
    steps+=("a_prod_${dt}_$rnd:120:$AB --dtype $dt" "a_hlds_${dt}_$rnd:120:$AB --dtype $dt --lib $L/libawq_hip_hlds.so")
  done
done
bash scripts/gpu_run.sh r5v "${steps[@]}"
