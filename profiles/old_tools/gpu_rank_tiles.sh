# Wall time of every rank's tile of an N-way split (load balance across ranks).  usage: bash tools/gpu_rank_tiles.sh N
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
N=$1
R=$(( (1080 + N - 1) / N ))
for r in $(seq 0 $((N-1))); do
  C=$(( (1080 - r + N - 1) / N ))
  echo "== rows $r:$C:$N"
  AB_ROWS=$r:$C:$N AB_REPS=2 timeout -k 10 300 python -u tools/abtime.py 512 base 2>&1 | grep '^0 ' || exit 2
done
