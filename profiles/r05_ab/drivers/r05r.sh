# r05r: the node visit's child-code read issued with the plane reads, before the first slab FMA
# (YK_CHILD_EARLY: a scheduling barrier after the seven LDS reads; production issues it ~25
# instructions later and waits for it at the visit's end) against base
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05r
mkdir -p gpurun_out/$T
timeout -k 10 400 python tools/abtime.py 512 base chearly > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r05r_bench base chearly || exit 1
