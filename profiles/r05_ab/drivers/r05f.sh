# r05f: where the first-segment split's time goes: rocprofv3 kernel traces of one synced
# 1920x1080x512 call (after a warm one) with the split (base), without (split0), and with the
# primary kernel touching the next batch's records (touch, fixed: a real load consumed after the
# segment).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05f
mkdir -p gpurun_out/$T
for v in base split0 touch; do
  if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
  YKGPU_LIB_OVERRIDE=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/$v -o run -- python3 tools/timeline_once.py 512 > gpurun_out/$T/$v.log 2>&1 || { echo TRACE_FAILED $v; tail -20 gpurun_out/$T/$v.log; exit 1; }
  echo "== $v"; grep -E "^\{" gpurun_out/$T/$v.log
  python3 tools/kernel_durations.py gpurun_out/$T/$v/run_kernel_trace.csv
done
