GB="python scripts/generic_bench.py --iters 30 --group-sizes 100,48,200,96,60,300 --shape '14336,4096;4096,14336;8192,3000' --dtypes bf16,f16"
bash scripts/gpu_run.sh r4d pytest smoke \
 "ab1:400:$GB --tunings rg_waves=0/rg_ldsdma=1/rg_persist=1" \
 "ab2:400:$GB --tunings rg_persist=1/rg_ldsdma=1/rg_waves=0" \
 "cli350:600:python scripts/cli_first_run.py --workload opt-350m --shards 3 --formats packed,reference --runs 2 --trace" \
 "cli8b:900:python scripts/cli_first_run.py --workload llama3-8b --shards 4 --formats packed,reference --runs 1 --trace"
