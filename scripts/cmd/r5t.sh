# round 5: weight column sums — one-pass variants (column tile = gs, 256, 512) A/B, each lib
# checked against the oracle first
set -u
AB="python scripts/act_search_bench.py --iters 5 --groups gate_up,down,qkv"
L=awq-converter_amd/awq_quantizer/_lib/ab
steps=()
for v in wm1 wm2 wm3; do
  steps+=("t_$v:300:AWQ_TEST_LIB=$L/libawq_hip_$v.so python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_act_search.py -k weight_mean")
done
for rnd in 1 2; do
  for v in wm1 wm2 wm3; do steps+=("a_${v}_$rnd:120:$AB --lib $L/libawq_hip_$v.so"); done
done
bash scripts/gpu_run.sh r5t "${steps[@]}"
