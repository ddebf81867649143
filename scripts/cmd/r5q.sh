# round 5: clip search on a group-contiguous copy of the tile (product) vs the round-4 layout
# (gcoff), a 6-wave budget and no scheduling barriers; bit-exactness first
set -u
GB="python scripts/generic_bench.py --iters 20 --search 10 --dtypes bf16,f16 --group-sizes 128,32 --shape '14336,4096;4096,14336'"
L=awq-converter_amd/awq_quantizer/_lib/ab
steps=("pytest=tests/test_scale_search.py tests/test_gpu_parity.py -k 'search'")
for rnd in 1 2; do
  steps+=("s_gc_$rnd:200:$GB")
  for v in gcoff gcw6 gcnosb; do steps+=("s_${v}_$rnd:200:$GB --lib $L/libawq_hip_$v.so"); done
done
steps+=("bench_search:400:python bench.py --mode search --workload llama3-8b --no-cpu-baseline")
bash scripts/gpu_run.sh r5q "${steps[@]}"
