# PMC probe of the render kernel on one bench step: the counter list, then LDS, instruction-mix and
# wait passes (one rocprofv3 run per pass).  usage: bash tools/gpu_pmc_probe.sh <outdir>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_probe}
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || echo "list rc $?"
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-modes"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  # keep only counters the list has (an unknown name fails the whole pass)
  ok=""
  for c in $grp; do grep -qw "$c" $O/counters.txt && ok="$ok $c"; done
  echo "pass $i:$ok"
  [ -z "$ok" ] && continue
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ok --output-format csv -d $O/p$i -o run -- python3 bench.py $ARGS > $O/p$i.log 2>&1 || { echo PASS_${i}_FAILED; tail -5 $O/p$i.log; exit 1; }
done <<'LIST'
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU
SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES
LIST
echo PMC_PROBE_OK
