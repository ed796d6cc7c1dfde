# r05o: the render workgroup's waves leave together (YK_WG_HOLD: a barrier at the kernel's end, so
# the CU frees whole and the next launch's workgroup is not starved by warm-up workgroups taking the
# registers piecemeal, r05m/r05n drain probes), alone and with the 128-block warm-up grid (r05n:
# -0.25%); synced calls, the bench's steps; the drain probe on it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05o
mkdir -p gpurun_out/$T
timeout -k 10 600 python tools/abtime.py 512 base wgsync w128 wgsync128 > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_drainwg.so timeout -k 10 120 python tools/drain_probe.py 512 "" gpurun_out/$T/drain_frame_wg.json > gpurun_out/$T/drain_frame_wg.log 2>&1 || { echo DRAIN_FAILED; tail -20 gpurun_out/$T/drain_frame_wg.log; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/$T/drain_frame_wg.json')); print({k: d[k] for k in ('call_ms','launches','cus','wave_idle_ms_per_cu','handover_ms_per_cu','bound_ms','bound_over_call')})"
bash tools/gpu_bench_ab.sh r05o_bench base w128 wgsync || exit 1
