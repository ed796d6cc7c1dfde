# r06ao: the leaves' root bounds in float (YK_LEAF_F32,
# lf32: 1/a, sqrt and the margins in float, U* a float; a lane out of float range takes the scan): the
# parity suite on the variant, synced 512-spp A/B with image hashes, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06ao
mkdir -p gpurun_out/$T
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_lf32.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/parity_lf32.log 2>&1 || { echo PARITY_FAILED; grep -E "FAILED|Error" gpurun_out/$T/parity_lf32.log | head; tail -30 gpurun_out/$T/parity_lf32.log; exit 1; }
tail -1 gpurun_out/$T/parity_lf32.log
timeout -k 10 900 python tools/abtime.py 512 base lf32 > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06ao_bench base lf32 || exit 3
