cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04u &&
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_stamps.so timeout -k 10 300 python -u tools/phases.py final 32 > gpurun_out/r04u/phases_fp64.txt 2>&1 &&
PREC=1 YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_stamps.so timeout -k 10 300 python -u tools/phases.py final 32 > gpurun_out/r04u/phases_fp32.txt 2>&1
