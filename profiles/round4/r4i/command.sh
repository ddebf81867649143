C350="python scripts/cli_first_run.py --workload opt-350m --shards 3 --formats packed --runs 3 --trace"
bash scripts/gpu_run.sh r4i \
 "early:300:python scripts/early_probe.py --runs 3" \
 "cli350:400:$C350" \
 "cli350ne:400:$C350 --no-early"
