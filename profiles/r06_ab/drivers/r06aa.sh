# r06aa: 64-spp frame launches with a slower synced ramp (YK_SCHED_SLOW: growth by half from 32
# spp, l64r: 4, 8, 16, 32, 48, 64...; from 16, l64r16: 4, 8, 16, 24, 36, 54, 64...) vs l64 and the
# 32-spp product; synced A/B at 512 spp, bench A/B, the synced timeline of l64r
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06aa
mkdir -p gpurun_out/$T
timeout -k 10 900 python tools/abtime.py 512 base l64 l64r l64r16 > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06aa_bench base l64 l64r l64r16 || exit 3
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_l64r.so timeout -k 10 200 python tools/timeline_once.py 512 > gpurun_out/$T/timeline_l64r.txt 2>&1 || { tail -20 gpurun_out/$T/timeline_l64r.txt; exit 1; }
tail -2 gpurun_out/$T/timeline_l64r.txt
