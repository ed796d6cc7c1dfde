cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04o &&
AB_REPS=4 timeout -k 10 600 python tools/abtime.py 512 base base@YKGPU_FIRST_LAUNCH=2 base@YKGPU_FIRST_LAUNCH=1 base@YKGPU_FIRST_LAUNCH=2@YKGPU_SCHED_GROW=3 base@YKGPU_FIRST_LAUNCH=8 > gpurun_out/r04o/ab_synced_ramp.txt 2>&1
