# r05n: short-lived warm-up waves (r05m's drain probe: as a render workgroup's waves leave, warm-up
# waves take their registers, and the next render workgroup waits ~0.27 ms per CU per launch for
# them): FP64 warm-up grids of 128 / 256 blocks per CU (8 / 4 slots per thread) and 1024 blocks of
# 1 slot per thread, against base (32 blocks per CU, ~32 slots per thread); the drain probe on w1s.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05n
mkdir -p gpurun_out/$T
timeout -k 10 600 python tools/abtime.py 512 base w128 w256 w1s > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_drainw1s.so timeout -k 10 120 python tools/drain_probe.py 512 "" gpurun_out/$T/drain_frame_w1s.json > gpurun_out/$T/drain_frame_w1s.log 2>&1 || { echo DRAIN_FAILED; tail -20 gpurun_out/$T/drain_frame_w1s.log; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/$T/drain_frame_w1s.json')); print({k: d[k] for k in ('call_ms','launches','cus','wave_idle_ms_per_cu','handover_ms_per_cu','bound_ms','bound_over_call')})"
