bash scripts/gpu_run.sh r4f pytest smoke \
 "init:200:python scripts/init_probe.py --runs 2" \
 "cli350:600:python scripts/cli_first_run.py --workload opt-350m --shards 3 --formats packed,reference --runs 2 --trace" \
 "cli8b:900:python scripts/cli_first_run.py --workload llama3-8b --shards 4 --formats packed --runs 2 --trace"
