#!/bin/bash
# Counter passes for ONE kernel of ONE workload (each pass its own rocprofv3 run, kernel-trace
# only, each under its own time limit), then a per-dispatch summary:
#   bash scripts/pmc_kernel.sh <out_dir> <kernel_regex> <program and args ...>
# passes: FETCH_SIZE | WRITE_SIZE | the SQ issue/wait breakdown | SQ instruction mix
# (gfx950 FETCH_SIZE reads half the bytes of a 16-B streaming load: pmc_breakdown.py doubles it).
set -u
OUT=$1; RX=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 100 rocprofv3 --kernel-include-regex "$RX" --pmc "$@" --output-format csv -d "$OUT/$name" -o p -- \
    "${PROG[@]}" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
PROG=("$@")
pass fetch FETCH_SIZE GRBM_GUI_ACTIVE
pass write WRITE_SIZE GRBM_GUI_ACTIVE
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pass mix SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM
python scripts/pmc_breakdown.py "$OUT" > "$OUT/summary.json" && find "$OUT" -name '*counter_collection.csv' -size +2M -delete
