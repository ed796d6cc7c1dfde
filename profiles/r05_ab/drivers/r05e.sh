# r05e: first-segment split (kPrimary coherent first segments + kBounce from hand-over records):
# the GPU suite on it, then A/B against the one-kernel path (split0): synced calls, the bench's
# back-to-back steps, the 8-way tile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05e
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error|error' gpurun_out/$T/gpu_tests.log | head -20; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
timeout -k 10 600 python tools/abtime.py 512 base split0 touch > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -5 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r05e_bench base split0 touch || exit 1
timeout -k 10 600 python tools/tile_ab.py base split0 touch > gpurun_out/$T/tile8.txt 2>&1 || { echo TILE_FAILED; exit 1; }
cat gpurun_out/$T/tile8.txt
