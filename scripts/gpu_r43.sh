set -o pipefail
mkdir -p gpurun_out/r43
df -h /tmp . | tee gpurun_out/r43/df.txt
free -g | tee -a gpurun_out/r43/df.txt
timeout -k 10 900 python bench.py --workload llama3-70b --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r43/bench_70b.json 2> gpurun_out/r43/bench_70b.err; rc=$?; cat gpurun_out/r43/bench_70b.json; tail -3 gpurun_out/r43/bench_70b.err; exit $rc
