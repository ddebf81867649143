GBL="python scripts/generic_bench.py --iters 30 --group-sizes 100,48,200,96,60 --shape '4096,14336' --dtypes bf16,f16"
P="python scripts/generic_bench.py --iters 3 --group-sizes 100"
bash scripts/gpu_run.sh r4g \
 "abk:500:$GBL --tunings rg_waves=0/rg_waves=2,rg_gpt=48/rg_waves=2,rg_gpt=32/rg_waves=2,rg_gpt=64/rg_gpt=16" \
 "pmc1:400:bash scripts/pmc_kernel.sh gpurun_out/r4g/pmc_rg_bf16_14336x4096 awq_rowgroup $P --shape 14336,4096 --dtypes bf16" \
 "pmc2:400:bash scripts/pmc_kernel.sh gpurun_out/r4g/pmc_rg_f16_14336x4096 awq_rowgroup $P --shape 14336,4096 --dtypes f16" \
 "pmc3:400:bash scripts/pmc_kernel.sh gpurun_out/r4g/pmc_rg_bf16_4096x14336 awq_rowgroup $P --shape 4096,14336 --dtypes bf16" \
 "pmc4:400:bash scripts/pmc_kernel.sh gpurun_out/r4g/pmc_rg_f16_4096x14336 awq_rowgroup $P --shape 4096,14336 --dtypes f16"
