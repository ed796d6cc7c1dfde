# r06i: the deferred warm-up's aligned path (a lane's four walks = one pixel's samples when the
# grid-stride is a whole number of pixel passes: seed and position once per trip) vs the general
# path (align0): the GPU suite on the product, synced A/B at 512 spp, bench A/B; then the RCCL
# gather probe (tools/gather_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06i
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/$T/gpu_tests.log | head; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 900 python tools/abtime.py 512 base align0 > gpurun_out/$T/ab512.txt 2>&1 || exit 1
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06i_bench base align0 || exit 1
timeout -k 10 300 python tools/gather_probe.py > gpurun_out/$T/probe.txt 2>&1 || { tail -20 gpurun_out/$T/probe.txt; exit 1; }
HIPRIO=1 MASTER_PORT=29532 timeout -k 10 300 python tools/gather_probe.py > gpurun_out/$T/probe_hiprio.txt 2>&1 || { tail -20 gpurun_out/$T/probe_hiprio.txt; exit 1; }
grep -h '^{' gpurun_out/$T/probe.txt gpurun_out/$T/probe_hiprio.txt
