# r06ac: 64-spp launches for in-flight calls only (YK_LAUNCH_SPP_OV, the rings sized for them; a
# synced call keeps 32): the GPU suite on the product, synced A/B at 512 spp (base = product vs
# ov32 = in-flight launches of 32 as before vs l64 = 64 for every call), bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06ac
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/$T/gpu_tests.log | head; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 900 python tools/abtime.py 512 base ov32 l64 > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06ac_bench base ov32 l64 || exit 3
