set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for spec in "0:1080:1" "0:272:4:3"; do
  echo "== rows $spec"
  ROWS=$spec YKGPU_LIB_OVERRIDE=uecraytracing_amd/lib/abl/libykgpu_diag8.so timeout -k 10 300 python -u tools/phases.py final 128 || exit 1
done
