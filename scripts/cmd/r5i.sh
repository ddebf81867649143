# round 5: clip-search instruction trims (alpha per lane, fp16 product + mixed fma, no SLP
# packing) and the act loss kernel without SLP packing: A/B of builds, outputs hashed
set -u
GB="python scripts/generic_bench.py --iters 20 --search 10 --dtypes bf16,f16 --group-sizes 128,32 --shape '14336,4096;4096,14336'"
AB="python scripts/act_search_bench.py --iters 5"
L=awq-converter_amd/awq_quantizer/_lib/ab
steps=()
for rnd in 1 2; do
  steps+=("s_base_$rnd:200:$GB")
  for v in al f16m alf16m alf16mns noslp; do
    steps+=("s_${v}_$rnd:200:$GB --lib $L/libawq_hip_$v.so")
  done
  steps+=("a_base_$rnd:120:$AB" "a_actnoslp_$rnd:120:$AB --lib $L/libawq_hip_actnoslp.so")
done
bash scripts/gpu_run.sh r5i "${steps[@]}"
