# r06t: on the product (branch-free visit + fast unwind): slot claims from a kernel argument and a
# v_readlane (YK_CLAIM_ARGS), the FP64 slab pairs read by op_sel (YK_SLAB_PAIRS_F64: 116 instead of
# 128 VGPRs, room for a third warm-up wave per SIMD), and both; parity suite per variant, synced
# A/B at 512 spp, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06t
mkdir -p gpurun_out/$T
for V in claimrl slabp slabcrl; do
  YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/$T/parity_$V.log 2>&1 || { echo PARITY_FAILED $V; tail -30 gpurun_out/$T/parity_$V.log; exit 1; }
  echo $V; tail -1 gpurun_out/$T/parity_$V.log
done
timeout -k 10 900 python tools/abtime.py 512 base claimrl slabp slabcrl > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06t_bench base claimrl slabp slabcrl || exit 3
