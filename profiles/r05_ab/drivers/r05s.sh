# r05s: the warm-up's thin-lens retries drawn after its grid-stride walks (YK_LENS_DEFER v2: the
# first candidate in line, the rejected queued in a per-wave ring of 512 and drawn 64 at a time at
# the kernel's end; a full ring hands the sample to the render; the main loop spill-free at 32
# VGPRs) against base: synced calls (image hash), the bench's steps, the GPU suite on it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05s
mkdir -p gpurun_out/$T
timeout -k 10 400 python tools/abtime.py 512 base ld2 > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r05s_bench base ld2 || exit 1
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_ld2.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error|error' gpurun_out/$T/gpu_tests.log | head -20; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
