C="python scripts/cli_first_run.py --workload opt-350m --shards 3 --formats packed --runs 3 --trace"
bash scripts/gpu_run.sh r4s "d:400:$C" "s32:400:$C --opts '{\"slot_bytes\": 33554432}'" "s48:400:$C --opts '{\"slot_bytes\": 50331648}'" "d2:400:$C"
