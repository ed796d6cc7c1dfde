# GPU parity (parity + modes), then rank-0 tile wall times of 1/2/4/8-way banded splits for variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/tiles_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/tiles_tests.log; exit 1; }
tail -1 gpurun_out/tiles_tests.log
for spec in "0:1080:1" "0:544:2:3" "0:272:4:3" "0:136:8:3"; do
  echo "== rows $spec"
  AB_ROWS=$spec AB_REPS=3 timeout -k 10 300 python -u tools/abtime.py 512 base "$@" 2>&1 | grep '^0 ' || exit 2
done
