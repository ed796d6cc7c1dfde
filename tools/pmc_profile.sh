#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only with kernel-trace) over bench.py.
# Usage (on the GPU box): bash tools/pmc_profile.sh <outdir> [bench args...]
# PMC_GROUPS (optional): counter groups separated by ';' (default: the roofline set below).
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:---steps 1 --warmup 1 --no-cpu-baseline --no-modes --no-configs --no-tiles}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/$OUT
DEFAULT="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU;SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_IOPS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY;FETCH_SIZE;WRITE_SIZE"
IFS=';' read -ra GROUPS_ <<< "${PMC_GROUPS:-$DEFAULT}"
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $R/$OUT/p$i -o run -- python3 $R/bench.py $ARGS > $R/$OUT/p$i.log 2>&1
done
