"""Lane-op reconciliation probe.  Run under rocprofv3 --pmc
(tools/gpu_lane_ops.sh).  Renders the bench workload's scene and image (final42, 1920x1080) at
`--spp` samples three times, synced, in this order:
  call A: the production instance (flags 0, all lanes);
  call B: the counting instance (YK_FLAG_COUNT_WORK, all lanes) — the work counters;
  call C: the counting instance with one lane per wave (COUNT_WORK | ONE_LANE): the per-wave-
          instruction counters then count exactly the instructions one lane executed.
The same samples (same seeds) every time.  The JSON carries call B's counters and the dispatch
layout, for tools/lane_ops_reconcile.py."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch  # noqa: F401  (torch's HIP runtime first, uecraytracing_amd/__init__.py)

    import uecraytracing_amd as yk
    from uecraytracing_amd.records import FLAG_COUNT_WORK, FLAG_ONE_LANE, image_height_for, make_params

    spheres, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
    W = a.width
    H = image_height_for(W)
    out = {"workload": f"final42_{W}x{H}x{a.spp}_d50", "calls": []}
    with yk.Renderer(0) as r:
        r.set_scene(spheres, cam)
        imgs = []
        for name, flags in (("A", 0), ("B", FLAG_COUNT_WORK), ("C", FLAG_COUNT_WORK | FLAG_ONE_LANE)):
            imgs.append(r.render(make_params(W, H, a.spp, 50, 404, flags=flags)))
            st = r.stats()
            out["calls"].append({"call": name, "flags": flags, "launches": st["launches"],
                                 **{k: st[k] for k in ("samples", "segments", "sphere_tests", "sqrt_calls",
                                                       "newton_calls", "newton_iters", "node_visits",
                                                       "linear_scans", "mt_fallbacks", "kernel_ms", "warmup_ms")},
                                 "work": st["work"]})
        out["images_equal"] = bool((imgs[0] == imgs[1]).all() and (imgs[1] == imgs[2]).all())
    js = json.dumps(out)
    if a.out:
        with open(a.out, "w") as f:
            f.write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
