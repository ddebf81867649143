#!/bin/bash
# round 2: row-segment pass 2 with wave-uniform branches (full sweeps unmasked, ballot tests)
set -u
OUT=gpurun_out/r2ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rowgroup.py tests/test_gpu_group_sizes.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit $?
AWQ_RG_GPT=64 timeout -k 10 300 python -u -m pytest tests/test_gpu_rowgroup.py -x -q --timeout 120 --timeout-method thread -k "bfloat16 and not special" > $OUT/pytest_gpt64.log 2>&1 || exit $?
timeout -k 10 300 python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16,f16,f32 --group-sizes 100,48,96,60,200,300 > $OUT/gs_default.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $OUT/pmc -o sq1 --output-format csv -- python scripts/generic_bench.py --shape 14336,4096 --dtypes bf16 --group-sizes 100 --iters 3 > $OUT/pmc1.log 2>&1 || exit $?
echo done
