# r06aw: the in-tree build of the final tree as the driver will find it: the whole -m gpu suite and
# smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06aw
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke: ok')" > gpurun_out/$T/smoke.txt 2>&1 || { tail -20 gpurun_out/$T/smoke.txt; exit 2; }
tail -1 gpurun_out/$T/smoke.txt
