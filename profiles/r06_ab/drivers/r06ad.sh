# r06ad (and r06ae, after the two-launch floor): in-flight tile launches of 2^27 slots (YK_LAUNCH_SLOTS_OV, s27) vs 2^26 (product): rank 0's
# row tile of config 3 at N = 8, 4, 2 (20 back-to-back calls) and of config 4 at N = 8 (6 calls),
# timed as the N-GPU bench's steps run them (tools/tile_ab.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06ad
mkdir -p gpurun_out/$T
for TL in 1920:512:8:0:rows 1920:512:4:0:rows 1920:512:2:0:rows; do
  TILE=$TL CALLS=20 timeout -k 10 600 python tools/tile_ab.py base s27 > gpurun_out/$T/tile_${TL//:/_}.txt 2>&1 || { tail -20 gpurun_out/$T/tile_${TL//:/_}.txt; exit 1; }
  echo "== $TL"; cat gpurun_out/$T/tile_${TL//:/_}.txt
done
TL=3840:1024:8:0:rows
TILE=$TL CALLS=6 timeout -k 10 600 python tools/tile_ab.py base s27 > gpurun_out/$T/tile_${TL//:/_}.txt 2>&1 || { tail -20 gpurun_out/$T/tile_${TL//:/_}.txt; exit 1; }
echo "== $TL"; cat gpurun_out/$T/tile_${TL//:/_}.txt
