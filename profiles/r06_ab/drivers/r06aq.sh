# r06aq: the render at 120 VGPRs (v120: the third warm-up wave still fits, 3 x 120 + 3 x 48 = 504,
# the reduce wave no longer beside them) and the leaves' float root bounds at 120 VGPRs (lf32v120:
# profiles/r06_ab/shade/yk_leaf_f32.patch without its spills) against the product: parity of lf32v120,
# synced 512-spp A/B with image hashes, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06aq
mkdir -p gpurun_out/$T
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_lf32v120.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/parity_lf32v120.log 2>&1 || { echo PARITY_FAILED; grep -E "FAILED|Error" gpurun_out/$T/parity_lf32v120.log | head; tail -30 gpurun_out/$T/parity_lf32v120.log; exit 1; }
tail -1 gpurun_out/$T/parity_lf32v120.log
timeout -k 10 900 python tools/abtime.py 512 base v120 lf32v120 > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06aq_bench base v120 lf32v120 || exit 3
