# r06x: the FP64 dielectric's 1/ior and Schlick r0 (both sides) precomputed on the host
# (YK_DIEL_PRE: two FP64 divisions fewer per trip with a glass hit), and 64-spp launches on the
# current build (YK_LAUNCH_SPP=64: 8 launches per frame); parity suite per variant, synced A/B at
# 512 spp, bench A/B (+ config 5, the glass scene, for dielpre)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06x
mkdir -p gpurun_out/$T
for V in dielpre l64; do
  YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/$T/parity_$V.log 2>&1 || { echo PARITY_FAILED $V; tail -30 gpurun_out/$T/parity_$V.log; exit 1; }
  echo $V; tail -1 gpurun_out/$T/parity_$V.log
done
timeout -k 10 900 python tools/abtime.py 512 base dielpre l64 > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06x_bench base dielpre l64 || exit 3
