# round 5: register-resident row segments, pass 1 by LDS atomics (3 KiB per wave)
set -u
O=gpurun_out/r5e
GB="python scripts/generic_bench.py --iters 30 --dtypes bf16,f16"
bash scripts/gpu_run.sh r5e \
 "pytest=tests/test_gpu_rowgroup.py -k 'rowreg or vs_oracle or special or full_size'" \
 "ab_gs100:300:$GB --shape '14336,4096;4096,14336' --group-sizes 100 --tunings 'default/rg_reg=1/rg_reg=0/rg_reg=1/default'" \
 "ab_other:400:$GB --shape '14336,4096;4096,14336;8192,3000' --group-sizes 48,60,96,124,200,36,500 --tunings 'default/rg_reg=1'" \
 "pmc_rr:400:bash scripts/pmc_kernel.sh $O/pmc_rr_14336x4096 awq_rowreg python scripts/generic_bench.py --iters 3 --dtypes bf16 --group-sizes 100 --shape 14336,4096"
