"""Wall time of one render of the headline workload (1920x1080, final scene, depth 50) in each
engine / precision mode (not the contract bench).  usage: python tools/modes_time.py [spp] [fp32_spp]"""
import sys
import time

sys.path.insert(0, '.')
import uecraytracing_amd as yk
from uecraytracing_amd.records import PRECISION_FP32, RNG_XOR128, make_params

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 512
spp32 = int(sys.argv[2]) if len(sys.argv) > 2 else 16
arr, cam = yk.build_scene("final", 42)
with yk.Renderer(0) as r:
    r.set_scene(arr, cam)
    for name, kw, s in [("mt19937/fp64", {}, spp), ("xor128/fp64", {"rng": RNG_XOR128}, spp),
                        ("mt19937/fp32", {"precision": PRECISION_FP32}, spp32),
                        ("xor128/fp32", {"precision": PRECISION_FP32, "rng": RNG_XOR128}, spp32),
                        ("mt19937/fp32 linear scan", {"precision": PRECISION_FP32, "flags": 2}, 16)]:
        p = make_params(1920, None, s, 50, 404, **kw)
        r.render(p)
        ts = []
        for _ in range(2):
            t = time.perf_counter()
            r.render(p)
            ts.append(time.perf_counter() - t)
        st = r.stats()
        dt = min(ts)
        print(f"{name}: spp {s}: {dt*1e3:.1f} ms, {st['samples']/dt/1e6:.0f} Msamples/s "
              f"(render kernels {st['kernel_ms']:.1f} ms, warm-ups {st['warmup_ms']:.1f} ms)", flush=True)
