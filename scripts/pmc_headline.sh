#!/bin/bash
# Counters of the headline kernel (awq_fast_kernel, Llama-3-70B set, the bench line) next to
# its memory-structure ceiling (awq_stream_ceiling_kernel, run by the same bench.py before
# the warmup): wave cycles, busy / wait cycles, instruction mix, and HBM traffic — each
# counter group in its own rocprofv3 --pmc run (kernel-trace only).
#   bash scripts/pmc_headline.sh <tag>          (on the GPU box, from the repo root)
set -u
TAG=${1:-pmc_headline}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
RX='awq_fast_kernel|awq_stream_ceiling_kernel'
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${WL_ARGS:-}"
step() { local name=$1; shift; echo "=== $name"; timeout -s KILL 240 rocprofv3 --kernel-include-regex "$RX" --pmc "$@" \
           --output-format csv -d "$OUT/$name" -o run -- $B > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc";
         [ $rc -eq 0 ] || exit $rc; python scripts/pmc_summary.py "$OUT/$name" > "$OUT/$name.summary.json";
         find "$OUT/$name" -name '*counter_collection.csv' -size +2M -delete; }
step sq_a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
step sq_b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS GRBM_GUI_ACTIVE
step fetch FETCH_SIZE GRBM_GUI_ACTIVE
step write WRITE_SIZE GRBM_GUI_ACTIVE
python scripts/pmc_headline.py "$OUT" > "$OUT/headline_counters.json" && cat "$OUT/headline_counters.json"
echo done
