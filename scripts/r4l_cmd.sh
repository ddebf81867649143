AB="python scripts/generic_bench.py --iters 30 --group-sizes 100,96,200,52,100 --shape '14336,4096;4096,14336;8192,3000' --dtypes bf16,f16"
RS="python scripts/generic_bench.py --iters 30 --group-sizes 100 --shape '14336,4096;4096,14336' --dtypes bf16,f16"
bash scripts/gpu_run.sh r4l "pytest=tests/test_gpu_rowgroup.py" \
 "abu:500:$AB --tunings rg_p1u=0/rg_p1u=1" \
 "rsprof:300:rocprofv3 --kernel-trace --stats --kernel-include-regex awq_rowgroup -d gpurun_out/r4l/rs -o rs --output-format csv -- $RS"
[ $? -eq 0 ] && bash scripts/gpu_run.sh r4l_cli \
 "ref4:400:python scripts/cli_first_run.py --workload opt-350m --shards 3 --formats reference --runs 3 --trace" \
 "ref8:400:python scripts/cli_first_run.py --workload opt-350m --shards 3 --formats reference --runs 3 --trace --opts '{\"writers\": 8}'"
