# Row-tile A/B at 512 spp: rank 0 of an 8-way and of a 4-way split (cyclic 8-row bands), then
# the full frame, for the given variants (tools/abtime.py).
# usage: bash tools/gpu_tiles_ab.sh <tag> <variant> ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/$T
AB_ROWS=0:135:8:3 timeout -k 10 600 python tools/abtime.py 512 "$@" > gpurun_out/$T/tile8.txt 2>&1 || exit 1
AB_ROWS=0:270:4:3 timeout -k 10 600 python tools/abtime.py 512 "$@" > gpurun_out/$T/tile4.txt 2>&1 || exit 2
timeout -k 10 600 python tools/abtime.py 512 "$@" > gpurun_out/$T/frame.txt 2>&1 || exit 3
for f in tile8 tile4 frame; do echo "== $f"; cat gpurun_out/$T/$f.txt; done
