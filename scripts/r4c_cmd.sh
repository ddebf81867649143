GB="python scripts/generic_bench.py --iters 30 --group-sizes 100,48,200,96 --shape '14336,4096;4096,14336' --dtypes bf16,f16"
bash scripts/gpu_run.sh r4c \
 "pytest=tests/test_gpu_rowgroup.py tests/test_gpu_nan.py tests/test_gpu_odd_groups.py tests/test_gpu_generic_span.py tests/test_gpu_padded_rows.py" \
 "ab1:300:$GB --tunings rg_waves=0/rg_p2reg=1/rg_ldsdma=1/rg_waves=1" \
 "ab2:300:$GB --tunings rg_ldsdma=1/rg_waves=1/rg_p2reg=1/rg_waves=0" \
 "dqab:200:python scripts/generic_bench.py --iters 30 --dequant --group-sizes 100,128,50 --shape 14336,4096 --dtypes bf16" \
 "ceiling:120:python scripts/ceiling_probe.py --mb 117.440512,469.762048,1073.741824" \
 "dqprobe:120:scripts/dq_probe" \
 "pin2:120:python scripts/pin_probe.py --sizes-mb 256 --methods twoalloc" \
 "cli350:600:python scripts/cli_first_run.py --workload opt-350m --shards 3 --formats packed,reference --runs 2" \
 "cli8b:900:python scripts/cli_first_run.py --workload llama3-8b --shards 4 --formats packed --runs 2"
