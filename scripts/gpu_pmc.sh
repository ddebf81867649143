#!/bin/bash
# PMC passes (each counter group in its own rocprofv3 run, kernel-trace only; no sys/runtime trace).
set -u
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
LIBS=${LIBS:-awq-converter_amd/awq_quantizer/_lib/libawq_hip.so}
SETS=${SETS:-llama3-8b-mlp,opt-125m}
step() { local name=$1; shift; echo "=== $name"; timeout -k 10 400 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -2 "$OUT/$name.log"; case $rc in 0) ;; *) exit $rc;; esac;
  python scripts/pmc_summary.py "$OUT/$name" > "$OUT/$name.summary.json"; find "$OUT/$name" -name '*counter_collection.csv' -size +2M -delete; }
step fetch rocprofv3 --kernel-include-regex 'awq_fast_kernel' --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$OUT/fetch" -o run -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline
step write rocprofv3 --kernel-include-regex 'awq_fast_kernel' --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$OUT/write" -o run -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline
i=0
for LIB in ${LIBS//,/ }; do
  for SET in ${SETS//,/ }; do
    i=$((i+1))
    step sq_${i} rocprofv3 --kernel-include-regex 'awq_fast_kernel' --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU \
      --output-format csv -d "$OUT/sq_${i}" -o run -- python scripts/kbench.py --sets $SET --libs $LIB --rounds 1 --iters 4
    step sq2_${i} rocprofv3 --kernel-include-regex 'awq_fast_kernel' --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE \
      --output-format csv -d "$OUT/sq2_${i}" -o run -- python scripts/kbench.py --sets $SET --libs $LIB --rounds 1 --iters 4
    echo "sq_${i} = $LIB $SET" >> "$OUT/index.txt"
  done
done
echo done
