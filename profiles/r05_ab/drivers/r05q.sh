# r05q: sensitivity of the frame to the seed walks' cost: the warm-up walks every sample's seed
# twice (YK_WALK_SENS=1, +~80% warm-up VALU work) against base
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05q
mkdir -p gpurun_out/$T
timeout -k 10 400 python tools/abtime.py 512 base walk2 > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
for v in base walk2; do
  if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
  YKGPU_LIB_OVERRIDE=$L timeout -k 10 120 python tools/timeline_once.py 512 > gpurun_out/$T/timeline_$v.txt 2>&1 || { echo TL_FAILED $v; exit 1; }
done
echo TL_OK
