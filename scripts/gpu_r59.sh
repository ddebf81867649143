set -o pipefail
# bench at the new default (200 steps) + extra lines (fp16, fp32, gs 64) + rocprof/PMC
mkdir -p gpurun_out/r59
run() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > gpurun_out/r59/$name.log 2>&1; local rc=$?; grep -v '^\s*$' gpurun_out/r59/$name.log | tail -2 | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run bench 300 python bench.py
run bench_f16 200 python bench.py --dtype f16 --no-cpu-baseline
run bench_f32 200 python bench.py --dtype f32 --no-cpu-baseline
run bench_gs64 200 python bench.py --group-size 64 --no-cpu-baseline
run bench_llama8b 300 python bench.py --workload llama3-8b --steps 20 --warmup 3 --no-cpu-baseline
run rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r59/prof -o run --output-format csv -- python bench.py --no-cpu-baseline
