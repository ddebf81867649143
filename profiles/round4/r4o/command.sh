RS="python scripts/generic_bench.py --iters 30 --group-sizes 100 --shape '14336,4096;4096,14336' --dtypes bf16,f16"
bash scripts/gpu_run.sh r4o "pytest=tests/test_gpu_rowgroup.py tests/test_gpu_nan.py" \
 "abb:900:bash scripts/gpu_ab_builds.sh r4o awq-converter_amd/awq_quantizer/_lib/libawq_hip_prev.so awq-converter_amd/awq_quantizer/_lib/libawq_hip.so 2" \
 "rsprof:300:rocprofv3 --kernel-trace --stats --kernel-include-regex awq_rowgroup -d gpurun_out/r4o/rs -o rs --output-format csv -- $RS"
