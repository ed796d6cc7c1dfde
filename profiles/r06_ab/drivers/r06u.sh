# r06u: the render's registers against the warm-up's waves: slab pairs + claim args (slabcrl: 114
# VGPRs, three 48-VGPR warm-up waves per SIMD) vs the same capped at 112 and at 104 VGPRs
# (YK_SINGLE_VGPRS: 104 leaves room for a fourth warm-up wave; 16 B of spills); parity suite per
# variant, synced A/B at 512 spp, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06u
mkdir -p gpurun_out/$T
for V in slabcap104 slabcap112; do
  YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/$T/parity_$V.log 2>&1 || { echo PARITY_FAILED $V; tail -30 gpurun_out/$T/parity_$V.log; exit 1; }
  echo $V; tail -1 gpurun_out/$T/parity_$V.log
done
timeout -k 10 900 python tools/abtime.py 512 base slabcrl slabcap112 slabcap104 > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06u_bench base slabcrl slabcap112 slabcap104 || exit 3
