set -o pipefail
mkdir -p gpurun_out/r42
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "stream_copy or fast_path_vs" > gpurun_out/r42/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r42/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r42/bench.json 2> gpurun_out/r42/bench.err; rc=$?; python -c "import json;d=json.load(open('gpurun_out/r42/bench.json'));print(d['value'], d['roofline'])"; exit $rc
