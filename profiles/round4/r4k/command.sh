# the driver's own commands first (GPUTEST: pytest -m gpu, then the smoke; BENCH: bench.py), then
# the process-first CLI record for profiles/round4/cli/
bash scripts/gpu_run.sh r4k \
 "driver_pytest:1200:python -m pytest tests -m gpu -x -q" smoke bench \
 "abr:500:python scripts/generic_bench.py --iters 30 --group-sizes 100,60,76,124,52 --shape '4096,14336;8192,8192;14336,4096' --dtypes bf16,f16 --tunings rg_waves=0/rg_waves=1" \
 "cli350:600:python scripts/cli_first_run.py --workload opt-350m --shards 3 --formats packed,reference --runs 3 --trace" \
 "cli8b:900:python scripts/cli_first_run.py --workload llama3-8b --shards 4 --formats packed --runs 3 --trace" \
 "cli8bref:900:python scripts/cli_first_run.py --workload llama3-8b --shards 4 --formats reference --runs 1 --trace"
