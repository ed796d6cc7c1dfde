# r05p: raw wave records of the drain probe (base build + diag), for the per-CU handover analysis
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05p
mkdir -p gpurun_out/$T
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_drain.so timeout -k 10 120 python tools/drain_probe.py 512 "" gpurun_out/$T/drain_frame.json > gpurun_out/$T/drain_frame.log 2>&1 || { echo DRAIN_FAILED; tail -20 gpurun_out/$T/drain_frame.log; exit 1; }
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_drain.so YKGPU_TIMELINE=1 timeout -k 10 120 python tools/timeline_once.py 512 > gpurun_out/$T/timeline.txt 2>&1 || { echo TL_FAILED; exit 1; }
echo OK
