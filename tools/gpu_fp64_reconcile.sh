# FP64 counter calibration + reconciliation on the GPU box:
#   cal: tools/flopcal (known instruction counts) under the FP64 counters
#   rec: tools/fp64_reconcile.py (all lanes, then one lane per wave) under the same counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r02_fp64}
mkdir -p $O
CTR="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU"
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d $O/cal -o run -- tools/flopcal > $O/cal.log 2>&1 || { echo CAL_FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d $O/rec -o run -- python3 tools/fp64_reconcile.py --out $O/rec_counts.json > $O/rec.log 2>&1 || { echo REC_FAILED; tail -20 $O/rec.log; exit 1; }
cat $O/rec_counts.json
echo FP64_OK
