# r05g: PMC view of the first-segment split: per kernel VALU instructions, lane utilisation and
# wave-cycles waiting, one synced 1920x1080x512 call (after a warm one), split1 (the split) vs base (one kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05g
mkdir -p gpurun_out/$T
C="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
C2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
for v in split1 base; do
  if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
  YKGPU_LIB_OVERRIDE=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/$T/${v}_p1 -o run -- python3 tools/timeline_once.py 512 > gpurun_out/$T/${v}_p1.log 2>&1 || { echo PMC_FAILED $v; tail -5 gpurun_out/$T/${v}_p1.log; exit 1; }
  YKGPU_LIB_OVERRIDE=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C2 --output-format csv -d gpurun_out/$T/${v}_p2 -o run -- python3 tools/timeline_once.py 512 > gpurun_out/$T/${v}_p2.log 2>&1 || { echo PMC2_FAILED $v; tail -5 gpurun_out/$T/${v}_p2.log; exit 1; }
done
echo PMC_OK
