# Wall time of every rank's tile of an N-way split in the bench's layout (8-row bands dealt
# cyclically, uecraytracing_amd/tiles.py tile_rows), each rank's tile rendered alone on one GPU:
# the load balance the N-GPU bench sees.  usage: bash tools/gpu_rank_tiles_banded.sh N
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
N=$1
for r in $(seq 0 $((N-1))); do
  # tiles.tile_rows(r, N, 1080): 135 bands of 8 rows, band b -> rank b mod N
  ROWS="$((r * 8)):$(( ((135 - r + N - 1) / N) * 8 )):$N:3"
  echo "== rank $r rows $ROWS"
  AB_ROWS=$ROWS AB_REPS=2 timeout -k 10 300 python -u tools/abtime.py 512 base 2>&1 | grep '^[01] ' || exit 2
done
