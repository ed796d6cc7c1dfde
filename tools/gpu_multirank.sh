# N>1 rehearsal on one GPU (ranks share it, gloo): the contract's torchrun launch of bench.py at
# --gpus 2, 3 and 8 (NS overrides), and tools/multirank_check.py (assembled image == single render, byte for byte).
# usage: bash tools/gpu_multirank.sh <outdir>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/multirank}
mkdir -p $O
for N in ${NS:-2 3 8}; do
  YK_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 2 --warmup 1 \
    --no-cpu-baseline --no-modes > $O/bench_n$N.log 2>&1 || { echo BENCH_N${N}_FAILED; tail -20 $O/bench_n$N.log; exit 1; }
  grep '^{' $O/bench_n$N.log | tail -1 > $O/bench_n$N.json
  YK_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29600 + N)) tools/multirank_check.py 320 16 > $O/check_n$N.log 2>&1 || { echo CHECK_N${N}_FAILED; tail -20 $O/check_n$N.log; exit 1; }
done
echo MULTIRANK_OK
