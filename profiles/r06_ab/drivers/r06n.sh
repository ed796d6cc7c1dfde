# r06n: the FP64 node loop's stack reads: the branch-free visit (YK_NODE_BF: sentinel entry, the
# entry below the top read with the planes), the pop after a leaf read before the leaf's loads
# (YK_LEAF_POP), and both; parity suite per variant, synced A/B at 512 spp, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06n
mkdir -p gpurun_out/$T
for V in nodebf leafpop bfpop; do
  YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/parity_$V.log 2>&1 || { echo PARITY_FAILED $V; tail -30 gpurun_out/$T/parity_$V.log; exit 1; }
  echo $V; tail -1 gpurun_out/$T/parity_$V.log
done
timeout -k 10 900 python tools/abtime.py 512 base nodebf leafpop bfpop > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06n_bench base nodebf leafpop bfpop || exit 3
