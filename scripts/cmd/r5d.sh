# round 5: counters of the register-resident row-segment kernel vs the LDS-stage kernel
set -u
O=gpurun_out/r5d
GB="python scripts/generic_bench.py --iters 3 --dtypes bf16 --group-sizes 100"
bash scripts/gpu_run.sh r5d \
 "pmc_rr:400:bash scripts/pmc_kernel.sh $O/pmc_rr_14336x4096 awq_rowreg $GB --shape 14336,4096" \
 "pmc_rg:400:bash scripts/pmc_kernel.sh $O/pmc_rg_14336x4096 awq_rowgroup $GB --shape 14336,4096 --tunings rg_reg=1" \
 "pmc_rr2:400:bash scripts/pmc_kernel.sh $O/pmc_rr_4096x14336 awq_rowreg $GB --shape 4096,14336"
