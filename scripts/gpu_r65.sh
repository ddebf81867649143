set -o pipefail
# act-search loss kernel: hardware group params, fmin/fmax, DPP reductions, fp32 fast path
mkdir -p gpurun_out/r65
timeout -k 10 600 python -u -m pytest tests/test_act_search.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r65/pytest_act.log 2>&1; rc=$?; tail -3 gpurun_out/r65/pytest_act.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/act_search_bench.py > gpurun_out/r65/act_new.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r65/act_new.log | tail -6; [ $rc -eq 0 ] || exit $rc
AWQ_HIP_LIB=awq-converter_amd/awq_quantizer/_lib/variants/libawq_hip_prev.so timeout -k 10 300 python scripts/act_search_bench.py > gpurun_out/r65/act_prev.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r65/act_prev.log | tail -6; exit $rc
