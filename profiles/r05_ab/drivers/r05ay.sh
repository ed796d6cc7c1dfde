# r05ay: the reduce split into two instances (yk_reduce_samples<ids>: the plain one as before the
# shared unwind) and the plain 24-byte colour store back for launches that keep the render's whole
# unwind: base (shared unwind for launches of >= 16 spp), ks1 (for every launch) and prev (before the
# shared unwind) on a whole config-4 frame and on config 3, synced, with image hashes; then the GPU
# suite on base.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05ay
mkdir -p gpurun_out/$T
AB_W=3840 AB_REPS=2 timeout -k 10 500 python tools/abtime.py 1024 base ks1 prev > gpurun_out/$T/ab1024_w3840.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab1024_w3840.txt; exit 1; }
cat gpurun_out/$T/ab1024_w3840.txt
AB_REPS=2 timeout -k 10 300 python tools/abtime.py 512 base ks1 prev > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
