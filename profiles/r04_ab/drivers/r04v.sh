cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04v &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04v/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r04v/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py --no-cpu-baseline --no-configs --no-tiles > gpurun_out/r04v/bench.log 2>&1
