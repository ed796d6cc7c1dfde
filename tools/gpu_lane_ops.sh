# Lane-op reconciliation on the GPU box (tools/lane_ops_reconcile.py): two PMC passes
# over tools/lane_ops_probe.py (production, counting and one-lane calls of the same samples), then
# the reconciliation into gpurun_out/<tag>/pmc_lane_ops.json.
# usage: bash tools/gpu_lane_ops.sh <tag> [spp]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-lane_ops}
SPP=${2:-8}
mkdir -p $O
P1="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_WAVES SQ_INSTS_SALU"
P2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $O/p1 -o run -- python3 tools/lane_ops_probe.py --spp $SPP --out $O/probe.json > $O/p1.log 2>&1 || { echo P1_FAILED; tail -20 $O/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d $O/p2 -o run -- python3 tools/lane_ops_probe.py --spp $SPP > $O/p2.log 2>&1 || { echo P2_FAILED; tail -20 $O/p2.log; exit 1; }
python3 tools/lane_ops_reconcile.py $O $O/probe.json $O/pmc_lane_ops.json || exit 1
echo LANE_OPS_OK
