GBL="python scripts/generic_bench.py --iters 30 --group-sizes 100,48,200,96,60 --shape '4096,14336' --dtypes bf16,f16"
bash scripts/gpu_run.sh r4g \
 "abk:500:$GBL --tunings rg_waves=0/rg_waves=2,rg_gpt=48/rg_waves=2,rg_gpt=32/rg_waves=2,rg_gpt=64/rg_gpt=16" \
 "prof:900:COMMIT=${COMMIT:-unknown} STEP_TIMEOUT=300 bash scripts/profile_round.sh r4g_prof"
