# r06av: the render at 120 VGPRs with the kept discriminant (hd120) against the product (112 VGPRs):
# the whole bench line (modes, configs 4 and 5, tiles) of each, twice, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06av
mkdir -p gpurun_out/$T
for rnd in 0 1; do
  for v in base hd120; do
    if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
    YKGPU_LIB_OVERRIDE=$L timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/$T/bench_${v}_$rnd.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/bench_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${v}_$rnd.log') if l.startswith('{')][-1]); t=d['tiles']
print($rnd, '$v', d['value'], d['ms_per_step'], 'fp32', d['modes']['fp32_mt19937']['ms'], 'x128', d['modes']['fp64_xor128']['ms'], 'c5', d['configs']['config5']['ms'], 'c4', d['configs']['config4_rank0_of_8']['ms'], 'n8', t['config3_n8']['slowest_ms'], t['config3_n8']['slowest_over_ideal'], 'n4', t['config3_n4']['slowest_ms'], 'c4n8', t['config4_n8']['slowest_ms'])"
  done
done
