"""Per-launch drain of the persistent render, measured.

usage: YKGPU_LIB_OVERRIDE=.../libykgpu_drain.so python tools/drain_probe.py [spp] [rows] [out.json]
(the library built with -DYK_DRAIN_DIAG: tools/build_def_variant.sh drain -DYK_DRAIN_DIAG)

Renders the headline workload (or a row tile "begin:count:stride") once warm, clears the wave
records, renders it again synced, and reads every FP64 render wave's start and end
(s_memrealtime, 10 ns) and its CU (HW_ID, XCC_ID).  Per launch:
* wave-idle: for each workgroup, the wave-time between a wave leaving the loop (no slot left for
  it) and its workgroup's last wave leaving (the workgroup holds the CU's LDS until then), summed,
  in CU-equivalents (/ waves per workgroup);
* handover: for each CU, the gap between its workgroup of this launch ending and the next
  workgroup (any later launch) starting on it — the CU idle, render-wise.
Their sum over the call, divided by the CU count, is what a render that continued into the next
launch's slots could win at most (it removes both)."""
import collections
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import uecraytracing_amd as yk  # noqa: E402
from uecraytracing_amd.records import make_params  # noqa: E402

L, B, W = 64, 512, 16


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    rows = tuple(int(v) for v in sys.argv[2].split(":")) if len(sys.argv) > 2 and sys.argv[2] else None
    out = sys.argv[3] if len(sys.argv) > 3 else None
    arr, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
    with yk.Renderer(0) as r:
        r.set_scene(arr, cam)
        lib = r._lib
        lib.ykgpu_diag_wave_times.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_size_t]
        p = make_params(1920, None, spp, 50, 404, rows=rows)
        r.render(p)
        assert lib.ykgpu_diag_wave_times_clear() == 0
        r.render(p)
        st = r.stats()
        n = L * B * W * 3
        buf = (ctypes.c_ulonglong * n)()
        assert lib.ykgpu_diag_wave_times(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(L, B, W, 3)
    if out:
        np.save(out.rsplit(".", 1)[0] + "_raw.npy", a[: st["launches"]])  # (launch, block, wave, {start, end, id})
    cus = collections.defaultdict(list)  # (xcc, se, cu) -> [(start, end, launch)]
    launches = []
    total_idle = total_gap = 0.0
    for c in range(L):
        blk = a[c]
        used = blk[:, :, 0] > 0
        if not used.any():
            continue
        t0 = blk[:, :, 0][used].min()
        idle = 0.0
        nwg = 0
        for b in range(B):
            m = used[b]
            if not m.any():
                continue
            nwg += 1
            ends = blk[b, m, 1].astype(np.float64)
            idle += float((ends.max() - ends).sum()) / m.sum()
            hw = int(blk[b, m, 2][0])
            key = (hw >> 32, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15)
            cus[key].append((float(blk[b, m, 0].min()), float(ends.max()), c))
        total_idle += idle
        launches.append({"launch": c, "workgroups": nwg, "wave_idle_cu_us": round(idle / 100.0, 1),
                         "span_ms": round(float(blk[:, :, 1][used].max() - t0) / 1e5, 3)})
    gaps = collections.defaultdict(float)
    for key, wgs in cus.items():
        wgs.sort()
        for (s0, e0, c0), (s1, e1, c1) in zip(wgs, wgs[1:]):
            if s1 > e0:
                gaps[c0] += s1 - e0
                total_gap += s1 - e0
    for d in launches:
        d["handover_cu_us"] = round(gaps[d["launch"]] / 100.0, 1)
    ncu = len(cus)
    res = {"spp": spp, "rows": rows, "call_ms": round(st["total_ms"], 3), "launches": len(launches), "cus": ncu,
           "wave_idle_ms_per_cu": round(total_idle / 1e5 / ncu, 4),
           "handover_ms_per_cu": round(total_gap / 1e5 / ncu, 4),
           "bound_ms": round((total_idle + total_gap) / 1e5 / ncu, 4),
           "per_launch": launches}
    res["bound_over_call"] = round(res["bound_ms"] / res["call_ms"], 4)
    js = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
