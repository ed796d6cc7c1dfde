# r06w: four render waves per SIMD (1024-thread workgroups) now that the render fits 112 VGPRs:
# 4 x 112 leave 64, one 48-VGPR warm-up wave per SIMD (b1024), or at 104 VGPRs two (b1024v104);
# the traversal stack then holds 10 checked entries (LDS); parity suite per variant, synced A/B at
# 512 spp, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06w
mkdir -p gpurun_out/$T
for V in b1024 b1024v104; do
  YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/$T/parity_$V.log 2>&1 || { echo PARITY_FAILED $V; tail -30 gpurun_out/$T/parity_$V.log; exit 1; }
  echo $V; tail -1 gpurun_out/$T/parity_$V.log
done
timeout -k 10 900 python tools/abtime.py 512 base b1024 b1024v104 > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06w_bench base b1024 b1024v104 || exit 3
