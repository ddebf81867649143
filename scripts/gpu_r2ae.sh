#!/bin/bash
# round 2: row-segment PMC per groups-per-tile (gs 100): VALU / SALU / LDS per wave and
# wave lifetimes, to tell instruction-bound from occupancy / latency-bound
set -u
OUT=gpurun_out/r2ae
mkdir -p $OUT
export TMPDIR=/tmp
for G in 16 24 48; do
  AWQ_RG_GPT=$G timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $OUT/pmc_gpt$G -o sq1 --output-format csv -- python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16 --group-sizes 100 --iters 3 > $OUT/pmc_gpt$G.log 2>&1 || exit $?
  AWQ_RG_GPT=$G timeout -s KILL 60 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc2_gpt$G -o sq2 --output-format csv -- python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16 --group-sizes 100 --iters 3 > $OUT/pmc2_gpt$G.log 2>&1 || exit $?
done
echo done
