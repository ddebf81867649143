set -o pipefail
mkdir -p gpurun_out/r25
V=awq-converter_amd/awq_quantizer/_lib/variants/libawq_hip_
for s in llama3-8b-mlp opt-125m; do
    timeout -k 10 200 python scripts/trace_waves.py --set $s --lib ${V}trace.so > gpurun_out/r25/$s.log 2>&1 || { cat gpurun_out/r25/$s.log; exit 1; }
    echo "== $s"; grep '^{' gpurun_out/r25/$s.log | tail -6
done
