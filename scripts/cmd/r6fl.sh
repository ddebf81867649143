#!/bin/bash
# round 6 final tree (after the search / act trims), part B: bench lines on the committed records (profiles/round6/pmc_traffic.json,
# pmc_valu.json: bench.py's defaults), kernel traces of the searches, dequantize vs its ceiling,
# smoke, full GPU suite
set -u
O=gpurun_out/r6fl
mkdir -p $O
SRCH="--mode search --workload llama3-8b"
ACT="--mode act"
bash scripts/gpu_run.sh r6fl \
 "bench:600:python bench.py " \
 "bench_f16:300:python bench.py --workload llama3-8b --dtype f16 --no-cpu-baseline" \
 "bench_search:400:python bench.py $SRCH " \
 "bench_act:400:python bench.py $ACT " \
 "trace_search:300:rocprofv3 --kernel-trace --stats --kernel-include-regex awq_fast_kernel -d $O/trace_search -o s --output-format csv -- python bench.py $SRCH --no-cpu-baseline " \
 "trace_act:300:rocprofv3 --kernel-trace --stats -d $O/trace_act -o act --output-format csv -- python bench.py $ACT --no-cpu-baseline " \
 "dq:300:python scripts/dq_ceiling_bench.py" \
 smoke \
 pytest || exit $?
# single-tensor kernels at settled clocks (row-segment gs 100, streaming gs 128, dequantize): the
# figures DESIGN §0 quotes
mkdir -p gpurun_out/r6fl && timeout -k 10 300 python scripts/generic_bench.py --shape "14336,4096;4096,14336;128256,4096" --dtypes bf16,f16 --group-sizes 128,100 --dequant --iters 20 --settle-ms 200 > gpurun_out/r6fl/single_settled.log 2>&1
echo single_settled rc=$?
