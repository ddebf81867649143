# final tree: the driver's commands, then the row-segment gs-100 record (rocprof + counters) and a CLI check
RS="python scripts/generic_bench.py --iters 30 --group-sizes 100 --shape '14336,4096;4096,14336' --dtypes bf16,f16"
P="python scripts/generic_bench.py --iters 3 --group-sizes 100"
bash scripts/gpu_run.sh r4n \
 "driver_pytest:1200:python -m pytest tests -m gpu -x -q" smoke bench \
 "rsprof:300:rocprofv3 --kernel-trace --stats --kernel-include-regex awq_rowgroup -d gpurun_out/r4n/rs -o rs --output-format csv -- $RS" \
 "pmc1:400:bash scripts/pmc_kernel.sh gpurun_out/r4n/pmc_rg_bf16_14336x4096 awq_rowgroup $P --shape 14336,4096 --dtypes bf16" \
 "cli350:400:python scripts/cli_first_run.py --workload opt-350m --shards 3 --formats packed --runs 2 --trace" \
 "cli8b:600:python scripts/cli_first_run.py --workload llama3-8b --shards 4 --formats packed --runs 2 --trace"
