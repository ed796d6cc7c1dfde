# r06c: back-to-back call boundary on the timeline (previous call's launches printed too), and the
# first-segment split's touch variant rebuilt with the explicit bound + device assert, A/B once
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06c
mkdir -p gpurun_out/$T
timeout -k 10 300 python tools/tile_timeline.py 1920 512 8 0 cols 6 > gpurun_out/$T/timeline_tile8.json 2> gpurun_out/$T/timeline_tile8.txt || exit 1
timeout -k 10 300 python tools/tile_timeline.py 1920 512 1 0 cols 3 > gpurun_out/$T/timeline_frame.json 2> gpurun_out/$T/timeline_frame.txt || exit 1
AB_REPS=2 timeout -k 10 600 python tools/abtime.py 512 split6 touch6 > gpurun_out/$T/ab512_split6_touch6.txt 2>&1 || exit 1
