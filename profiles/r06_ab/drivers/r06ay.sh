# r06ay: round-end evidence of the final tree (the packed candidate ids adopted):
# lane ops, the whole -m gpu suite, PMC passes, bench, kernel trace, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_lane_ops.sh r06ay_lane_ops || exit 1
cp gpurun_out/r06ay_lane_ops/pmc_lane_ops.json profiles/pmc_lane_ops.json
bash tools/gpu_round_end.sh r06ay || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke: ok')" > gpurun_out/r06ay/smoke.txt 2>&1 || { tail -20 gpurun_out/r06ay/smoke.txt; exit 3; }
tail -1 gpurun_out/r06ay/smoke.txt
