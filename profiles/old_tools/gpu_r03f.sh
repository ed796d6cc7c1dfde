set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03f
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_split.so timeout -k 10 200 python tools/timeline_once.py 512 > gpurun_out/r03f/tl_split.txt 2>&1 || exit 1
timeout -k 10 200 python tools/timeline_once.py 512 > gpurun_out/r03f/tl_base.txt 2>&1 || exit 2
grep -A20 "timed call" gpurun_out/r03f/tl_split.txt
grep -A20 "timed call" gpurun_out/r03f/tl_base.txt | tail -4
