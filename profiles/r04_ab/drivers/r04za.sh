cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04za &&
YK_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 7 --master-addr 127.0.0.1 --master-port 29607 tools/multirank_check.py 320 16 > gpurun_out/r04za/check_n7.log 2>&1 &&
YK_BENCH_BACKEND=gloo YK_DEAL=rows timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29603 tools/multirank_check.py 320 16 > gpurun_out/r04za/check_n3_rows.log 2>&1
