# r06d: the N-GPU partition: every rank's 8-way tile of config 3 under column
# bands, single rows and 8-row bands, timed like the contract loop (K = 8 and 20); then the bench
# with the like-for-like tile timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06d
mkdir -p gpurun_out/$T
K=8 timeout -k 10 900 python tools/deal_ab.py cols rows rows3 rows2 > gpurun_out/$T/deal8.txt 2>&1 || { tail -5 gpurun_out/$T/deal8.txt; exit 1; }
timeout -k 10 900 python bench.py --no-cpu-baseline --no-modes > gpurun_out/$T/bench.log 2>&1 || { tail -20 gpurun_out/$T/bench.log; exit 1; }
grep '^{' gpurun_out/$T/bench.log | tail -1 > gpurun_out/$T/bench.json
