cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04zc &&
for t in 1920:512:8:0:cols 1920:512:4:0:cols 1920:512:2:0:cols 3840:1024:8:0:cols; do TILE=$t CALLS=4 timeout -k 10 600 python tools/tile_ab.py base rule2; done > gpurun_out/r04zc/tiles.txt 2>&1 &&
TILE=1920:512:1:0:cols CALLS=4 timeout -k 10 400 python tools/tile_ab.py base rule2 > gpurun_out/r04zc/frame.txt 2>&1
