# r05m: four render waves per SIMD (1024-thread workgroups) at 96 / 104 / 112 VGPRs (the warm-up
# waves get what is left: 4 / 3 / 2 per SIMD) against base (768 threads, 128 VGPRs, 4 warm-up waves).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05m
mkdir -p gpurun_out/$T
timeout -k 10 600 python tools/abtime.py 512 base b1024v96 b1024v104 b1024v112 > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
# the per-launch drain, measured (diagnostic build): the frame and an 8-way row tile
L=$PWD/uecraytracing_amd/lib/abl/libykgpu_drain.so
YKGPU_LIB_OVERRIDE=$L timeout -k 10 120 python tools/drain_probe.py 512 "" gpurun_out/$T/drain_frame.json > gpurun_out/$T/drain_frame.log 2>&1 || { echo DRAIN_FAILED; tail -20 gpurun_out/$T/drain_frame.log; exit 1; }
YKGPU_LIB_OVERRIDE=$L timeout -k 10 120 python tools/drain_probe.py 512 0:135:8 gpurun_out/$T/drain_tile8.json > gpurun_out/$T/drain_tile8.log 2>&1 || { echo DRAIN8_FAILED; tail -20 gpurun_out/$T/drain_tile8.log; exit 1; }
python3 -c "
import json
for f in ('drain_frame','drain_tile8'):
    d=json.load(open('gpurun_out/$T/'+f+'.json')); print(f, {k: d[k] for k in ('call_ms','launches','cus','wave_idle_ms_per_cu','handover_ms_per_cu','bound_ms','bound_over_call')})"
