# round 5: register-resident row-segment kernel: parity + A/B + rocprof
set -u
O=gpurun_out/r5c
GB="python scripts/generic_bench.py --iters 30 --dtypes bf16,f16"
bash scripts/gpu_run.sh r5c \
 "pytest=tests/test_gpu_rowgroup.py" \
 "pytest=tests/test_gpu_parity.py tests/test_gpu_nan.py tests/test_gpu_padded_rows.py tests/test_gpu_odd_groups.py" \
 "ab_gs100:300:$GB --shape '14336,4096;4096,14336' --group-sizes 100 --tunings 'default/rg_reg=1/rg_reg=0/rg_reg=1/default'" \
 "ab_other:400:$GB --shape '14336,4096;4096,14336;8192,3000' --group-sizes 48,60,96,124,200,36,500 --tunings 'default/rg_reg=1'" \
 "trace:300:rocprofv3 --kernel-trace --stats -d $O/trace -o rr --output-format csv -- python scripts/generic_bench.py --iters 20 --dtypes bf16,f16 --shape '14336,4096;4096,14336' --group-sizes 100"
