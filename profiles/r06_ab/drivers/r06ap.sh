# r06ap: round-end evidence of the final tree (kernels ISA-identical to r06aj; host knobs added off):
# lane ops, the whole -m gpu suite, PMC passes, bench, kernel trace, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_lane_ops.sh r06ap_lane_ops || exit 1
cp gpurun_out/r06ap_lane_ops/pmc_lane_ops.json profiles/pmc_lane_ops.json
bash tools/gpu_round_end.sh r06ap || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke: ok')" > gpurun_out/r06ap/smoke.txt 2>&1 || { tail -20 gpurun_out/r06ap/smoke.txt; exit 3; }
tail -1 gpurun_out/r06ap/smoke.txt
