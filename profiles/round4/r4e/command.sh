GB="python scripts/generic_bench.py --iters 30 --group-sizes 100,48,200,96,60,300 --shape '14336,4096;4096,14336;8192,3000' --dtypes bf16,f16"
RS="python scripts/generic_bench.py --iters 30 --group-sizes 100 --shape '14336,4096;4096,14336' --dtypes bf16,f16"
bash scripts/gpu_run.sh r4e pytest smoke \
 "init:200:python scripts/init_probe.py --runs 2" \
 "ab1:400:$GB --tunings rg_waves=0/rg_ldsdma=1" \
 "rsprof:300:rocprofv3 --kernel-trace --stats --kernel-include-regex awq_rowgroup -d gpurun_out/r4e/rs -o rs --output-format csv -- $RS"
