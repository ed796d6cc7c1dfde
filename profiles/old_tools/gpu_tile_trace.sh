set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in 1 2 4; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tt$n -o run -- python3 tools/tile_trace.py $n > gpurun_out/tt$n.log 2>&1 || exit 1
grep "N=" gpurun_out/tt$n.log
done
