# r05l: warm-up lens retries deferred to a per-wave ring (YK_LENS_DEFER): every sample draws its
# first thin-lens candidate in line, the rejected wait in a ring and get their next candidates 64
# at a time.  512-spp A/B (warm-up at 32 VGPRs with spills / 40 / uncapped 42) against base, the
# FP32 mode's image at 64 spp, then the GPU suite on ld32.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05l
mkdir -p gpurun_out/$T
timeout -k 10 600 python tools/abtime.py 512 base ld32 ld40 ld > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
AB_PREC=1 AB_REPS=1 timeout -k 10 300 python tools/abtime.py 64 base ld32 > gpurun_out/$T/ab64_f32.txt 2>&1 || { echo AB32_FAILED; tail -20 gpurun_out/$T/ab64_f32.txt; exit 1; }
cat gpurun_out/$T/ab64_f32.txt
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_ld32.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error|error' gpurun_out/$T/gpu_tests.log | head -20; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
