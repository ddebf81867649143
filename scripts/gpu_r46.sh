set -o pipefail
mkdir -p gpurun_out/r46
timeout -k 10 600 python -m pytest tests/test_cli.py tests/test_distributed.py -m gpu -x -q > gpurun_out/r46/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r46/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 env AWQ_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r46/bench_n2_gloo.json 2> gpurun_out/r46/bench_n2_gloo.err; rc=$?; cat gpurun_out/r46/bench_n2_gloo.json; exit $rc
