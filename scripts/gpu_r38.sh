set -o pipefail
mkdir -p gpurun_out/r38
AWQ_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r38/bench2.log 2>&1; rc=$?; grep '^{' gpurun_out/r38/bench2.log; tail -3 gpurun_out/r38/bench2.log; exit $rc
