# r06p: which test the YK_NODE_BF=2 build stalls in (r06o: no output for 180 s after 54 parity tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06p
mkdir -p gpurun_out/$T
for V in nodebf bf2c; do
  echo "== $V"
  YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$V.so timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 60 --timeout-method thread -k "config2 or headline_geometry or bvh_matches" > gpurun_out/$T/parity_$V.log 2>&1
  rc=$?
  tail -5 gpurun_out/$T/parity_$V.log
  if [ $rc -ne 0 ]; then echo "rc=$rc"; grep -n "Timeout\|File \"" gpurun_out/$T/parity_$V.log | tail -20; exit 1; fi
done
