set -o pipefail
mkdir -p gpurun_out/r30
V=awq-converter_amd/awq_quantizer/_lib/variants/libawq_hip_
for s in opt-125m llama3-8b-mlp c1; do
  for v in trace tracetriv; do
    timeout -k 10 200 python scripts/trace_waves.py --set $s --lib ${V}$v.so > gpurun_out/r30/$s.$v.log 2>&1 || { tail -5 gpurun_out/r30/$s.$v.log; exit 1; }
    echo "== $s $v"; grep '^{' gpurun_out/r30/$s.$v.log | tail -2
  done
done
