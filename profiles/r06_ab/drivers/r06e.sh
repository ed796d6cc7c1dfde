# r06e: tiles in ~2^26-slot launches with rings deeper than a call (ctx->gev): GPU suite, then A/B
# against the round's start (r06base): the 8-/4-way tiles and the frame back to back (K = 8), and
# every rank's 8-way tile under columns and rows
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06e
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/$T/gpu_tests.log | head; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
CALLS=8 timeout -k 10 600 python tools/tile_ab.py r06base base > gpurun_out/$T/tile8_ab.txt 2>&1 || exit 1
TILE=1920:512:4:0:cols CALLS=8 timeout -k 10 600 python tools/tile_ab.py r06base base > gpurun_out/$T/tile4_ab.txt 2>&1 || exit 1
TILE=1920:512:1:0:cols CALLS=8 timeout -k 10 600 python tools/tile_ab.py r06base base > gpurun_out/$T/frame_ab.txt 2>&1 || exit 1
TILE=3840:1024:8:0:cols CALLS=6 timeout -k 10 600 python tools/tile_ab.py r06base base > gpurun_out/$T/c4tile8_ab.txt 2>&1 || exit 1
K=8 timeout -k 10 900 python tools/deal_ab.py cols rows > gpurun_out/$T/deal8.txt 2>&1 || exit 1
