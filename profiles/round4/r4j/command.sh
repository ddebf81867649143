AB="python scripts/generic_bench.py --iters 30 --group-sizes 100,60,76,124,52,100 --shape '4096,14336;8192,8192' --dtypes bf16,f16"
P="python scripts/generic_bench.py --iters 3 --group-sizes 100"
bash scripts/gpu_run.sh r4j "pytest=tests/test_gpu_rowgroup.py" \
 "abr:500:$AB --tunings rg_waves=0/rg_waves=1" \
 "pmc1:400:bash scripts/pmc_kernel.sh gpurun_out/r4j/pmc_rg_bf16_14336x4096 awq_rowgroup $P --shape 14336,4096 --dtypes bf16" \
 "pmc2:400:bash scripts/pmc_kernel.sh gpurun_out/r4j/pmc_rg_f16_14336x4096 awq_rowgroup $P --shape 14336,4096 --dtypes f16" \
 "pmc3:400:bash scripts/pmc_kernel.sh gpurun_out/r4j/pmc_rg_bf16_4096x14336 awq_rowgroup $P --shape 4096,14336 --dtypes bf16" \
 "pmc4:400:bash scripts/pmc_kernel.sh gpurun_out/r4j/pmc_rg_f16_4096x14336 awq_rowgroup $P --shape 4096,14336 --dtypes f16"
