# r06an: the FP64 visit loop in two copies, with and without the stack check (YK_VISIT_UNSWITCH,
# unsw: no uniform branch inside the loop, one taken branch per iteration instead of two): the
# parity suite on the variant, synced 512-spp A/B with image hashes, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06an
mkdir -p gpurun_out/$T
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_unsw.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/parity_unsw.log 2>&1 || { echo PARITY_FAILED; grep -E "FAILED|Error" gpurun_out/$T/parity_unsw.log | head; tail -30 gpurun_out/$T/parity_unsw.log; exit 1; }
tail -1 gpurun_out/$T/parity_unsw.log
timeout -k 10 900 python tools/abtime.py 512 base unsw > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06an_bench base unsw || exit 3
