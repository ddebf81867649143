# counters for the next round's analysis: final row-segment kernel (long rows) and the
# streaming kernel on the same tensor at gs 128 (residency / issue comparison)
bash scripts/gpu_run.sh r4v \
 "pmc1:400:bash scripts/pmc_kernel.sh gpurun_out/r4v/pmc_rg_bf16_4096x14336 awq_rowgroup python scripts/generic_bench.py --iters 3 --group-sizes 100 --shape 4096,14336 --dtypes bf16" \
 "pmc2:400:bash scripts/pmc_kernel.sh gpurun_out/r4v/pmc_rg_f16_14336x4096 awq_rowgroup python scripts/generic_bench.py --iters 3 --group-sizes 100 --shape 14336,4096 --dtypes f16" \
 "pmc3:400:bash scripts/pmc_kernel.sh gpurun_out/r4v/pmc_fast_bf16_14336x4096 awq_fast_kernel python scripts/generic_bench.py --iters 3 --group-sizes 128 --shape 14336,4096 --dtypes bf16"
