# Per-launch HIP-event timeline (YKGPU_TIMELINE=1) of one bench call of the current build.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tl_now
YKGPU_TIMELINE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes --steps 1 --warmup 1 > gpurun_out/tl_now/bench.log 2>&1 || exit 1
grep -h "launch\|call" gpurun_out/tl_now/bench.log | head -19
