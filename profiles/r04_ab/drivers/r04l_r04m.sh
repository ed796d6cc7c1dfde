cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04m &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "f32 or fp32 or FP32 or golden or modes or column or back_to_back" > gpurun_out/r04m/gpu_tests.log 2>&1 &&
AB_PREC=1 timeout -k 10 600 python tools/abtime.py 512 base nosplit > gpurun_out/r04m/ab_f32.txt 2>&1
