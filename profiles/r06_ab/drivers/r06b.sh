# r06b: the synced first call of a tile (the ramp) vs first-launch sizes, and many back-to-back
# calls (the in-flight steady state) for the 8-way tile and the frame
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06b
mkdir -p gpurun_out/$T
TILE=1920:512:8:0:cols CALLS=1 timeout -k 10 600 python tools/tile_ab.py base knob knob@YKGPU_FIRST_LAUNCH=16 knob@YKGPU_FIRST_LAUNCH=32 knob@YKGPU_FIRST_LAUNCH=64 knob@YKGPU_FIRST_LAUNCH=32@YKGPU_SCHED_GROW=4 knob@YKGPU_FIRST_LAUNCH=8@YKGPU_SCHED_GROW=4 > gpurun_out/$T/tile8_synced.txt 2>&1 || exit 1
TILE=1920:512:1:0:cols CALLS=1 timeout -k 10 600 python tools/tile_ab.py base knob@YKGPU_FIRST_LAUNCH=8 > gpurun_out/$T/frame_synced.txt 2>&1 || exit 1
TILE=1920:512:8:0:cols CALLS=20 timeout -k 10 600 python tools/tile_ab.py base > gpurun_out/$T/tile8_b2b20.txt 2>&1 || exit 1
TILE=1920:512:8:0:cols CALLS=4 timeout -k 10 600 python tools/tile_ab.py base > gpurun_out/$T/tile8_b2b4.txt 2>&1 || exit 1
TILE=1920:512:1:0:cols CALLS=20 timeout -k 10 600 python tools/tile_ab.py base > gpurun_out/$T/frame_b2b20.txt 2>&1 || exit 1
