# r05k: fused render with producer waves at issue priority 2 (3) while they render first segments
# (r05j: with 2 producers the bounce waves find the queue empty on ~15% of their trips, with 3 the
# producers wait on a full queue): 2/3/4 producers, and the diagnostics of 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05k
mkdir -p gpurun_out/$T
timeout -k 10 700 python tools/abtime.py 512 base fused2 fused2p fused3p fused4p fused3p3 > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_fused3pd.so timeout -k 10 120 python tools/fused_diag.py 512 > gpurun_out/$T/diag_fused3pd_512.txt 2>&1 || { echo DIAG_FAILED; tail -5 gpurun_out/$T/diag_fused3pd_512.txt; exit 1; }
tail -1 gpurun_out/$T/diag_fused3pd_512.txt
