# round 5: VALU probe, more instruction classes (integer min/max/bitwise, f16, perm, shifts),
# with the dual-issue counter pass
set -u
O=gpurun_out/r5y
mkdir -p $O
A="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU_ADD_F16 SQ_INSTS_VALU_MUL_F16 SQ_INSTS_VALU_FMA_F16 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU GRBM_GUI_ACTIVE"
bash scripts/gpu_run.sh r5y \
 "probe:300:scripts/valu_probe --ghz 2.4" \
 "probe_pmc_a:150:timeout -s KILL 140 rocprofv3 --pmc $A --output-format csv -d $O/probe_a -o p -- scripts/valu_probe" \
 "probe_pmc_b:150:timeout -s KILL 140 rocprofv3 --pmc $B --output-format csv -d $O/probe_b -o p -- scripts/valu_probe" \
 "classes:60:python scripts/valu_classes.py --probe-log $O/probe.log --pmc-a $O/probe_a --pmc-b $O/probe_b --out $O/valu_classes.json"
