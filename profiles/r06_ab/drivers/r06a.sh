set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06a
timeout -k 10 300 python tools/tile_timeline.py 1920 512 8 0 cols 4 > gpurun_out/r06a/timeline_tile8.json 2> gpurun_out/r06a/timeline_tile8.txt || exit 1
timeout -k 10 300 python tools/tile_timeline.py 1920 512 1 0 cols 4 > gpurun_out/r06a/timeline_frame.json 2> gpurun_out/r06a/timeline_frame.txt || exit 1
timeout -k 10 600 python tools/tile_ab.py r05d r05v r05af r05ba > gpurun_out/r06a/tile8_ab.txt 2>&1 || exit 1
TILE=1920:512:4:0:cols timeout -k 10 600 python tools/tile_ab.py r05d r05ba > gpurun_out/r06a/tile4_ab.txt 2>&1 || exit 1
TILE=1920:512:1:0:cols CALLS=4 timeout -k 10 600 python tools/tile_ab.py r05d r05ba > gpurun_out/r06a/frame_ab.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06a/robust.log 2>&1 || { echo ROBUST_FAILED; tail -30 gpurun_out/r06a/robust.log; exit 1; }
tail -3 gpurun_out/r06a/robust.log
