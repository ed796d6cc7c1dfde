# r06q: branch-free visit variants after the r06o/r06p stall (YK_NODE_BF=2's cap check compared a
# below-the-base top unsigned; now signed): BF1 / BF2 (entry below the top as the loop variable,
# child codes from LDS address 0), the proven-depth stack without the overflow check
# (YK_STACK_EXACT), the candidate skip (YK_CAND_SKIP); parity suite per variant, synced A/B at
# 512 spp, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06q
mkdir -p gpurun_out/$T
for V in bf2c bf2x bf1x bf2xskip; do
  YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/$T/parity_$V.log 2>&1 || { echo PARITY_FAILED $V; tail -30 gpurun_out/$T/parity_$V.log; exit 1; }
  echo $V; tail -1 gpurun_out/$T/parity_$V.log
done
timeout -k 10 900 python tools/abtime.py 512 base nodebf bf2c bf2x bf1x bf2xskip > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06q_bench nodebf bf2c bf2x bf1x bf2xskip || exit 3
