# r06ai: the FP64 visit's distances from tmin_lo scaled by 2^-24, the near FMAs clamping to [0, 1]
# in place of the max with tmin_lo (YK_NEAR_CLAMP, nclamp: 4 VALU fewer per visit): the GPU parity
# suite on the variant library (YKGPU_LIB_OVERRIDE), synced 512-spp A/B with image hashes, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06ai
mkdir -p gpurun_out/$T
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_nclamp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/parity_nclamp.log 2>&1 || { echo PARITY_FAILED; grep -E "FAILED|Error" gpurun_out/$T/parity_nclamp.log | head; tail -30 gpurun_out/$T/parity_nclamp.log; exit 1; }
tail -1 gpurun_out/$T/parity_nclamp.log
timeout -k 10 900 python tools/abtime.py 512 base nclamp > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06ai_bench base nclamp || exit 3
for f in gpurun_out/r06ai_bench/bench_*_0.log; do python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']
print('$f', 'visits/segment', r.get('node_visits_per_segment'), 'tests/segment', r.get('tests_per_segment'))"; done
