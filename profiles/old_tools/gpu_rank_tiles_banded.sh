# Wall time of every rank's tile of an N-way split in the bench's layout (8-row bands dealt
# cyclically, uecraytracing_amd/tiles.py tile_rows), each rank's tile rendered alone on one GPU:
# the load balance the N-GPU bench sees.  usage: bash tools/gpu_rank_tiles_banded.sh N [L]
# (L = row_band_log2, default 3: bands of 2^L rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
N=$1
L=${2:-3}
B=$((1 << L))
NB=$(( (1080 + B - 1) / B ))
for r in $(seq 0 $((N-1))); do
  # tiles.tile_rows(r, N, 1080, L): NB bands of B rows (1080 is a multiple of B for L <= 3),
  # band b -> rank b mod N
  ROWS="$((r * B)):$(( ((NB - r + N - 1) / N) * B )):$N:$L"
  echo "== rank $r rows $ROWS"
  AB_ROWS=$ROWS AB_REPS=2 timeout -k 10 300 python -u tools/abtime.py 512 base 2>&1 | grep '^[01] ' || exit 2
done
