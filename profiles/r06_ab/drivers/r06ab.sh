# r06ab: renders waiting for the reduce of launch g - 2 (timelines r06z / r06aa): a colour ring of 3
# (cr3, l64cr3) and the reduce stream at the renders' priority (redp, l64redp), at 32- and 64-spp
# frame launches; synced A/B at 512 spp, bench A/B, synced timelines of cr3 and l64cr3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06ab
mkdir -p gpurun_out/$T
timeout -k 10 900 python tools/abtime.py 512 base cr3 redp l64 l64cr3 l64redp > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06ab_bench base cr3 redp l64 l64cr3 l64redp || exit 3
for V in cr3 l64cr3; do
  YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$V.so timeout -k 10 200 python tools/timeline_once.py 512 > gpurun_out/$T/timeline_$V.txt 2>&1 || { tail -20 gpurun_out/$T/timeline_$V.txt; exit 1; }
  echo "== $V"; tail -1 gpurun_out/$T/timeline_$V.txt
done
