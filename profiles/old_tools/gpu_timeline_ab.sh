cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02ae
for v in base k4; do
  if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
  YKGPU_TIMELINE=1 YKGPU_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes --steps 1 --warmup 1 > gpurun_out/r02ae/bench_$v.log 2>&1 || exit 1
done
grep -h "launch\|call" gpurun_out/r02ae/bench_base.log | tail -22
echo ==; grep -h "launch\|call" gpurun_out/r02ae/bench_k4.log | tail -22
