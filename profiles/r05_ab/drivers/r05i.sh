# r05i: fused first-segment render policies at 512 spp (after r05h: 2 producers +2.3%, 3 +4%, 4 +15%
# vs base; 32 spp: 3 producers -1.9%): 0/1/2 producer waves, queue threshold 8/16 chunks, producers
# that render bounces while the queue is long (fused3h); then per-launch timelines of base and fused1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05i
mkdir -p gpurun_out/$T
timeout -k 10 700 python tools/abtime.py 512 base fused0 fused1 fused2 fused2q8 fused2q16 fused3h > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
for v in base fused1; do
  if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
  YKGPU_LIB_OVERRIDE=$L timeout -k 10 120 python tools/timeline_once.py 512 > gpurun_out/$T/timeline_$v.txt 2>&1 || { echo TL_FAILED $v; tail -5 gpurun_out/$T/timeline_$v.txt; exit 1; }
done
echo TL_OK
