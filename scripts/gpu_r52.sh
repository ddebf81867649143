set -o pipefail
mkdir -p gpurun_out/r52
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-include-regex 'awq_fast_kernel' --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r52/sq -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-copy-ceiling > $R/gpurun_out/r52/sq.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-include-regex 'awq_fast_kernel' --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r52/sq8b -o run -- python3 $R/bench.py --workload llama3-8b --steps 3 --warmup 1 --no-cpu-baseline --no-copy-ceiling > $R/gpurun_out/r52/sq8b.log 2>&1 || exit $?
cd $R && python scripts/pmc_summary.py gpurun_out/r52/sq > gpurun_out/r52/sq.summary.json && python scripts/pmc_summary.py gpurun_out/r52/sq8b > gpurun_out/r52/sq8b.summary.json && find gpurun_out/r52 -name '*counter_collection.csv' -size +2M -delete; cat gpurun_out/r52/sq.summary.json
