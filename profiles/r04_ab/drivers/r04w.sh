cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04w &&
DEPTH=200 YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_stamps.so timeout -k 10 300 python -u tools/phases.py glass 32 > gpurun_out/r04w/phases_glass.txt 2>&1
