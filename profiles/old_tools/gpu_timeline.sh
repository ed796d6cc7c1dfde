# rocprofv3 kernel trace of two bench steps → per-dispatch timeline of the last call.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=${1:-gpurun_out/tl}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-modes > $O/kt.log 2>&1 || { echo KT_FAILED; tail -5 $O/kt.log; exit 1; }
python3 tools/timeline.py $O/kt/run_kernel_trace.csv -1
