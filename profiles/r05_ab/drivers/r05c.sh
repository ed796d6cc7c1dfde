# r05c: lane-op reconciliation probe; A/B of the tail-size claims (bench back-to-back steps and
# the 8-way config-3 tile, interleaved): base (64-slot tail claims below 2 x 512 slots per wave),
# claimtail0 (full claims to the end, round 4), ct128, ct64f4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05c
bash tools/gpu_lane_ops.sh r05c 8 > gpurun_out/r05c/lane_ops.log 2>&1 || { echo LANE_OPS_FAILED; tail -30 gpurun_out/r05c/lane_ops.log; exit 1; }
tail -45 gpurun_out/r05c/lane_ops.log
timeout -k 10 600 python tools/tile_ab.py base claimtail0 ct128 ct64f4 > gpurun_out/r05c/tile8_ab.txt 2>&1 || { echo TILE_AB_FAILED; tail -10 gpurun_out/r05c/tile8_ab.txt; exit 1; }
cat gpurun_out/r05c/tile8_ab.txt
bash tools/gpu_bench_ab.sh r05c_bench base claimtail0 ct128 ct64f4 || exit 1
