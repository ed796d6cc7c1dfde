# r06ax: the FP64 candidate list's tuple ids as 16-bit halves of two registers (YK_CAND_PACK, cpack:
# the shift-in one alignbit + one lshl_or instead of moves, two VGPRs freed), and with them the
# newest candidate's v_rsq_f64 kept for math::sqrt's start (YK_CAND_RSQ, cprsq: no spill once the
# ids are packed) against the product: parity of cprsq, synced 512-spp A/B with image hashes, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06ax
mkdir -p gpurun_out/$T
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_cprsq.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/parity_cprsq.log 2>&1 || { echo PARITY_FAILED; grep -E "FAILED|Error" gpurun_out/$T/parity_cprsq.log | head; tail -30 gpurun_out/$T/parity_cprsq.log; exit 1; }
tail -1 gpurun_out/$T/parity_cprsq.log
timeout -k 10 900 python tools/abtime.py 512 base cpack cprsq > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06ax_bench base cpack cprsq || exit 3
