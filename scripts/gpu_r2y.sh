#!/bin/bash
# round 2: row-segment stage loads all in flight, host 1/L, packed bf16 field chain
set -u
OUT=gpurun_out/r2y
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rowgroup.py tests/test_gpu_group_sizes.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
timeout -k 10 300 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16,f16,f32 --group-sizes 100,48,96,60,200,300 > $OUT/gs_sweep.log 2>&1 || exit $?
for G in 8 32; do
  AWQ_RG_GPT=$G timeout -k 10 120 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16 --group-sizes 100,60,200 > $OUT/gpt$G.log 2>&1 || exit $?
done
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $OUT/pmc -o sq1 --output-format csv -- python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16 --group-sizes 100 --iters 3 > $OUT/pmc1.log 2>&1 || exit $?
echo done
