set -o pipefail
mkdir -p gpurun_out/r48
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r48/prof -o act -- python3 $R/scripts/act_search_bench.py --tokens 512 --grid 20 --iters 2 --groups qkv,down > $R/gpurun_out/r48/prof.log 2>&1 || exit $?
find $R/gpurun_out/r48/prof -name "*stats*"
timeout -k 10 400 rocprofv3 --kernel-include-regex 'act_loss_kernel' --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r48/pmc -o act -- python3 $R/scripts/act_search_bench.py --tokens 512 --grid 20 --iters 1 --groups o > $R/gpurun_out/r48/pmc.log 2>&1 || exit $?
find $R/gpurun_out/r48/pmc -name "*.csv"
