# Wall time of the rank-0 row tile of an N-way split (what each rank renders at N GPUs), N = 1,2,4,8:
# single rows dealt cyclically and bands of 8 rows dealt cyclically (tiles.py's split).
# usage: bash tools/gpu_tiles.sh [variant ...]   (base = lib/libykgpu.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/tiles_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/tiles_tests.log; exit 1; }
tail -1 gpurun_out/tiles_tests.log
for spec in "0:1080:1" "0:540:2" "0:544:2:3" "0:270:4" "0:272:4:3" "0:135:8" "0:136:8:3"; do
  echo "== rows $spec"
  AB_ROWS=$spec AB_REPS=3 timeout -k 10 300 python -u tools/abtime.py 512 base "$@" 2>&1 | grep '^0 ' || exit 2
done
