bash scripts/gpu_run.sh r4t "pytest=tests/test_cli.py tests/test_dist_output.py" \
 "cli350:400:python scripts/cli_first_run.py --workload opt-350m --shards 3 --formats packed,reference --runs 3 --trace" \
 "cli8b:600:python scripts/cli_first_run.py --workload llama3-8b --shards 4 --formats packed --runs 2 --trace"
