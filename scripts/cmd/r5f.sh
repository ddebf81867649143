# round 5: clip-search candidate pairs (ILP) vs the single-candidate loop, A/B of builds
set -u
O=gpurun_out/r5f
mkdir -p $O
GB="python scripts/generic_bench.py --iters 20 --search 10 --dtypes bf16,f16 --group-sizes 128,32 --shape '14336,4096;4096,14336'"
steps=("pytest=tests/test_scale_search.py")
for rnd in 1 2; do
  for v in orig pair4 pair5 single pair6 single6; do
    steps+=("ab_${v}_$rnd:200:$GB --lib awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_$v.so")
  done
done
bash scripts/gpu_run.sh r5f "${steps[@]}"
