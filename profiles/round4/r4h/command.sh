C350="python scripts/cli_first_run.py --workload opt-350m --shards 3 --formats packed --runs 2 --trace"
C8B="python scripts/cli_first_run.py --workload llama3-8b --shards 4 --formats packed --runs 2 --trace"
bash scripts/gpu_run.sh r4h pytest \
 "d2h:120:python scripts/d2h_probe.py" \
 "d2ht:120:python scripts/d2h_probe.py --touch" \
 "cli350:400:$C350" \
 "cli350s32:400:$C350 --opts '{\"slot_bytes\": 33554432}'" \
 "cli8b:600:$C8B" \
 "cli8bs128:600:$C8B --opts '{\"slot_bytes\": 134217728}'" \
 "cli8bh:600:$C8B --opts '{\"host_ring_bytes\": 1811939328}'"
