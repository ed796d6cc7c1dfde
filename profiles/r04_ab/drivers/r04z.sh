cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
bash tools/gpu_round_end.sh r04z > gpurun_out/r04z.txt 2>&1 &&
NS="2 8" bash tools/gpu_multirank.sh gpurun_out/r04z_multirank >> gpurun_out/r04z.txt 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" >> gpurun_out/r04z.txt 2>&1
