# r06z: per-launch timelines (YKGPU_TIMELINE=1) of one synced 1920x1080x512 call, 32-spp (base)
# vs 64-spp (l64) frame launches: where the synced call loses what the back-to-back calls gain
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06z
mkdir -p gpurun_out/$T
for V in base l64; do
  if [ $V = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$V.so; fi
  YKGPU_LIB_OVERRIDE=$L timeout -k 10 200 python tools/timeline_once.py 512 > gpurun_out/$T/timeline_$V.txt 2>&1 || { tail -20 gpurun_out/$T/timeline_$V.txt; exit 1; }
  echo "== $V"; tail -3 gpurun_out/$T/timeline_$V.txt
done
