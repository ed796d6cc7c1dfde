# r05j: fused render diagnostics (2 and 3 producer waves: pauses, idle waits, dry consumer trips,
# regions by consumer waves) at 512 and 32 spp; the reduce stream at the render priority (redprio)
# vs base: synced calls and the bench's steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05j
mkdir -p gpurun_out/$T
for v in fused2d fused3d; do
  for s in 512 32; do
    YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so timeout -k 10 120 python tools/fused_diag.py $s > gpurun_out/$T/diag_${v}_$s.txt 2>&1 || { echo DIAG_FAILED $v; tail -5 gpurun_out/$T/diag_${v}_$s.txt; exit 1; }
    echo $v $s; tail -1 gpurun_out/$T/diag_${v}_$s.txt
  done
done
timeout -k 10 400 python tools/abtime.py 512 base redprio > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r05j_bench base redprio || exit 1
