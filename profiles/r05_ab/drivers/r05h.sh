# r05h: the fused first-segment render (kMode 32: producer waves render coherent first segments
# and queue the survivors' records in LDS, the other waves render the bounces from the queue, one
# kernel per launch).  Image check at 32 spp against base, then 512-spp A/B over 2/3/4 producer
# waves, then the GPU suite with the fused library as the library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05h
mkdir -p gpurun_out/$T
AB_REPS=1 timeout -k 10 300 python tools/abtime.py 32 base fused3 > gpurun_out/$T/ab32.txt 2>&1 || { echo AB32_FAILED; tail -20 gpurun_out/$T/ab32.txt; exit 1; }
cat gpurun_out/$T/ab32.txt
timeout -k 10 600 python tools/abtime.py 512 base fused2 fused3 fused4 > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_fused3.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error|error' gpurun_out/$T/gpu_tests.log | head -20; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
