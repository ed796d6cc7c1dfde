#!/usr/bin/env python3
"""Benchmark of the per-pixel sampling loop on MI355X (BASELINE.json metric).

One STEP = one full render of the headline configuration (BASELINE config 3): 1920x1080,
512 spp, max_depth 50, the ~485-sphere RTIOW final scene (seed 42), FP64 / mt19937, bit-exact to
the reference's arithmetic.  Inputs (scene, camera) are resident in HBM before the timed region;
the output RGB8 image is produced in HBM (rank 0 holds the assembled image).

N > 1 (one process per GPU, torchrun): the image's rows are dealt cyclically (row r → rank r mod N;
`--deal cols`: 8-column bands over every row, band b → rank b mod N), each rank
renders its tile into device memory, and the tiles are gathered to rank 0 over RCCL
(torch.distributed 'nccl') and de-interleaved on device — all inside the timed region.
The total image is fixed, so this is STRONG scaling.

Prints ONE JSON line on rank 0.  The `roofline` object is the dominant kernel's VALU roofline
(the path is neither HBM- nor MFMA-bound): algorithmic FP64 flops per launch (the
reference's expressions over the kernel's own work counters, uecraytracing_amd/flops.py) over the
launch duration = the union of the launches' HIP-event spans / launches (they overlap on two
streams, so a per-span average would count the overlap twice).  HBM and issue views sit beside
it.  The `cpu_baseline` is the CPU oracle restatement (oracle/yk_oracle.c, "port") on a strided
row subset of the same workload, on every CPU this job may use (the box's cgroup quota), rank 0
at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/sec at 1920x1080x512spp (~500 spheres); per-pixel RMSE vs CPU"
HBM_PEAK_GBPS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
SPHERE_RECORD_BYTES = 80      # yk_sphere (include/ykgpu.h): the scene a workgroup stages once

PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")
FP64_RECONCILE = os.path.join(ROOT, "profiles", "r02_fp64_reconcile.json")


def usable_cpus():
    """CPUs this process may run on: the affinity mask, capped by the cgroup CPU quota (the GPU
    box grants each one-GPU job 16 of the node's 256 logical CPUs), and the node's count."""
    node = os.cpu_count() or 1
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else node
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    if quota is not None:
        n = max(1, min(n, int(quota)))
    return n, node, quota


def fp64_reconcile_facts():
    """The committed FP64 counter reconciliation (tools/gpu_fp64_reconcile.sh), or None."""
    if not os.path.exists(FP64_RECONCILE):
        return None
    with open(FP64_RECONCILE) as f:
        rec = json.load(f)
    keep = ("workload", "implementation_model_vs_counter", "algorithmic_share_of_executed",
            "fp64_lane_utilization", "per_sample")
    out = {k: rec[k] for k in keep if k in rec}
    out["source"] = "profiles/r02_fp64_reconcile.json (tools/gpu_fp64_reconcile.sh)"
    out["calibration"] = rec.get("calibration", {}).get("finding")
    return out


def pmc_facts(workload=None):
    """Counter facts of the same workload from the committed rocprofv3 --pmc passes
    (tools/pmc_profile.sh + tools/pmc_summary.py → profiles/pmc_summary.json), or None."""
    if not os.path.exists(PMC_SUMMARY):
        return None
    with open(PMC_SUMMARY) as f:
        rec = json.load(f)
    if workload is not None and rec.get("workload") != workload:
        return None
    keep = ("source", "kernel", "workload", "mean_ms", "valu_pipe_util", "valu_lane_utilization",
            "SQ_WAIT_ANY_frac", "SQ_WAIT_INST_ANY_frac", "hbm_bytes_per_launch", "hbm_bytes_per_sample",
            "fp64_flops_hw_per_launch")
    return {k: rec[k] for k in keep if k in rec}


PMC_LANE_OPS = os.path.join(ROOT, "profiles", "pmc_lane_ops.json")
PMC_HBM = os.path.join(ROOT, "profiles", "pmc_hbm.json")
HBM_MEASURED_GBPS = 6290.0    # MI355X_MICROARCH.md chip table: float4 copy, measured


def hbm_measured(samples_per_step, ms_per_step, alg_bytes_per_sample, path=PMC_HBM):
    """The step's HBM traffic from the PMC counters (north_star "rocprof
    achieved-HBM-GB/s against the chip's peak"): every kernel of a launch — render, warm-up,
    reduce — in bytes per sample (tools/pmc_hbm.py over tools/pmc_profile.sh's FETCH_SIZE and
    WRITE_SIZE passes of the same build), times the step's samples over the step's time.  None
    without the committed summary."""
    if not os.path.exists(path):
        return None
    with open(path) as f:
        rec = json.load(f)
    bps = rec["bytes_per_sample"]
    gbps = bps * samples_per_step / (ms_per_step * 1e-3) / 1e9
    return {
        "achieved": round(gbps, 2), "unit": "GB/s",
        "peak": HBM_PEAK_GBPS, "frac": round(gbps / HBM_PEAK_GBPS, 5),
        "peak_measured": HBM_MEASURED_GBPS, "frac_of_measured": round(gbps / HBM_MEASURED_GBPS, 5),
        "bytes_per_sample": round(bps, 3),
        "bytes_per_sample_by_kernel": {k: round(v["bytes_per_sample"], 3) for k, v in rec["kernels"].items()},
        "traffic_per_step": round(bps * samples_per_step),
        "traffic_over_algorithmic": round(bps / alg_bytes_per_sample, 1),
        "source": f"{os.path.relpath(path, ROOT)} ({rec['source']}); GB/s = bytes per sample x the "
                  f"step's samples / ms_per_step",
    }


def pmc_lane_ops():
    """The committed reconciliation of the lane-op model with the PMC counters
    (tools/lane_ops_reconcile.py), or None."""
    if not os.path.exists(PMC_LANE_OPS):
        return None
    with open(PMC_LANE_OPS) as f:
        return json.load(f)


def _run_harness(harness, mode, arg, W, H, spp, depth, seed0, nproc, timeout_s):
    """oracle/_ref/ref_harness as `nproc` processes over interleaved rows (YK_REF_ROWS = k:nproc,
    row y → process y mod nproc), the image assembled from their row sets; wall clock from the
    first start to the last exit.  Raises on a non-zero exit or on the time limit (every process
    is killed first)."""
    import subprocess
    import tempfile

    import numpy as np
    with tempfile.TemporaryDirectory() as td:
        paths = [os.path.join(td, f"h{k}.rgb") for k in range(nproc)]
        t = time.perf_counter()
        procs = [subprocess.Popen([harness, mode, arg, str(W), str(H), str(spp), str(depth), str(seed0), paths[k]],
                                  env=dict(os.environ, YK_REF_ROWS=f"{k}:{nproc}"),
                                  stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
                 for k in range(nproc)]
        try:
            for pr in procs:
                left = max(0.1, timeout_s - (time.perf_counter() - t))
                _, err = pr.communicate(timeout=left)
                if pr.returncode != 0:
                    raise RuntimeError(f"ref_harness exit {pr.returncode}: {err.decode(errors='replace')[-300:]}")
        finally:
            for pr in procs:
                if pr.poll() is None:
                    pr.kill()
                    pr.wait()
        dt = time.perf_counter() - t
        img = np.zeros((H, W, 3), np.uint8)
        for k in range(nproc):
            img[k::nproc] = np.fromfile(paths[k], np.uint8).reshape(H, W, 3)[k::nproc]
    return img, dt


def reference_calibration(seed0, nthreads, W=160, spp=32, depth=50, W_all=640, timeout_s=120.0):
    """The reference's own loop beside the port on this host (north_star: "the reference CPU loop
    timed on the node's own host cores ... core count stated").  oracle/_ref/ref_harness is the
    reference's headers (ray_color, hittable_list, sphere, mt19937, generate_canonical, math::sqrt)
    and its per-pixel loop (source.cpp:122-172) with the constexpr seed, -O2 (oracle/Makefile;
    built only where /root/reference exists, the binary travels with the tree).  The 485-sphere
    scene does not compile through the reference's tuple API, so it renders the
    reference's own 4-sphere world (source.cpp:103-112) and the 48-sphere slice of the final scene
    (tests/golden/final48.yks, through the harness's scene-file tuple).
      one_core:  W x H x spp on one thread each, harness and port (oracle/yk_oracle.c);
      all_cores: W_all x H x spp with the harness as `nthreads` processes over interleaved rows
                 (the reference's own `par` mode does not run, source.cpp:17-19,85-96, SURVEY
                 finding 8) and the port on `nthreads` threads.
    Both images are compared; a failure or a time-out is recorded, never raised (a side
    measurement must not cost the bench line)."""
    import numpy as np

    import golden_data
    import oracle_lib
    import refscenes
    from uecraytracing_amd.records import image_height_for, make_params
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return {"skipped": "oracle/_ref/ref_harness absent (built from /root/reference by oracle/Makefile)"}
    final48 = os.path.join(ROOT, "tests", "golden", "final48.yks")
    scenes = (("ref4", "render", "ref4", lambda: (refscenes.ref4(), refscenes.reference_camera())),
              ("final48", "render_file", final48, lambda: golden_data.read_scene_file(final48)))
    out = {"method": f"one_core: {W}x{image_height_for(W)}x{spp}, one thread each; all_cores: "
                     f"{W_all}x{image_height_for(W_all)}x{spp}, the harness as {nthreads} processes over "
                     f"interleaved rows, the port on {nthreads} threads; depth {depth}, seed0 {seed0}, wall "
                     f"clock; harness = the reference's headers and loop (-O2), port = oracle/yk_oracle.c (-O2)",
           "cores": nthreads}
    mismatch = []
    for leg, w, nt in (("one_core", W, 1), ("all_cores", W_all, nthreads)):
        h = image_height_for(w)
        n = w * h * spp
        res = {}
        for name, mode, arg, scene_fn in scenes:
            try:
                scene = scene_fn()
                h_rgb, dt_h = _run_harness(harness, mode, arg, w, h, spp, depth, seed0, nt, timeout_s)
                t = time.perf_counter()
                p_rgb, _, _, _ = oracle_lib.render(scene[0], scene[1], make_params(w, h, spp, depth, seed0),
                                                   nthreads=nt)
                dt_p = time.perf_counter() - t
                eq = bool((h_rgb == p_rgb).all())
                if not eq:
                    mismatch.append(f"{leg}/{name}")
                res[name] = {"spheres": len(scene[0]), "harness_msps": round(n / dt_h / 1e6, 4),
                             "port_msps": round(n / dt_p / 1e6, 4), "port_over_harness": round(dt_h / dt_p, 3),
                             "harness_s": round(dt_h, 2), "port_s": round(dt_p, 2), "images_equal": eq}
            except Exception as e:  # noqa: BLE001 (recorded, never fatal)
                res[name] = {"error": f"{type(e).__name__}: {e}"[:400]}
        out[leg] = res
    fin = out["all_cores"].get("final48", {})
    if "harness_msps" in fin:
        out["harness_msps_all_cores"] = fin["harness_msps"]
    out["images_equal"] = not mismatch
    if mismatch:
        out["IMAGES_DIFFER"] = mismatch
    return out


def other_configs(ren, stream, seed0, nthreads, peak_tf, deal):
    """BASELINE configs 4 and 5 on this GPU, after the contract line's timed region (rank 0, N=1):
    config 5 = 1920x1080x4096, max_depth 200, the dielectric-heavy glass scene, whole frame (the
    active-ray compaction stress); config 4 = 3840x2160x1024 on the final scene, rank 0's tile of
    the 8-GPU split under `deal` (tiles.py: every 8th 8-column band, or every 8th row: what one GPU
    renders in the driver's 8-GPU run).  Each:
    one warm call, one timed call (HIP events around the call on the bench stream), the roofline
    from a counting call, and the timed image's rows compared with the CPU oracle."""
    import numpy as np
    import torch

    import uecraytracing_amd as yk
    from uecraytracing_amd import flops
    from uecraytracing_amd.records import image_height_for, make_params
    from uecraytracing_amd.tiles import rank_tile, tile_image_cols
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    out = {}
    cases = (("config5", "glass", 1920, 4096, 200, None, (17, 1061)),
             ("config4_rank0_of_8", "final", 3840, 1024, 50, (0, 8),
              (0, 134, 269) if deal == "rows" else (0, 1079, 2159)))
    for name, scene, W, spp, depth, split, cmp_rows in cases:
        scene_file = os.path.join(yk.SCENE_DIR, f"{scene}_seed42.yks")
        spheres, cam = yk.read_scene(scene_file)
        ren.set_scene(spheres, cam)
        H = image_height_for(W)
        tk = rank_tile(split[0], split[1], H, W, deal) if split else {"rows": (0, H, 1, 0)}
        rows = tk["rows"]
        p = make_params(W, H, spp, depth, seed0, flags=0, **tk)
        Wt = p.tile_width()
        xs = (tile_image_cols(split[0], split[1], W) if split and tk.get("cols") else list(range(W)))
        tile = torch.empty((rows[1], Wt, 3), dtype=torch.uint8, device=torch.device("cuda", ren.device))
        with torch.cuda.stream(stream):
            ren.render_async(p, tile.data_ptr(), stream.cuda_stream)  # warm call (allocations)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            ren.render_async(p, tile.data_ptr(), stream.cuda_stream)
            e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        tst = ren.stats()
        img = tile.cpu().numpy()
        ren.render_async(make_params(W, H, spp, depth, seed0, flags=1, **tk), tile.data_ptr(),
                         stream.cuda_stream)
        torch.cuda.synchronize()
        st = ren.stats()
        n = rows[1] * Wt * spp
        launches = max(1, tst["launches"])
        launch_ms = tst["render_busy_ms"] / launches
        alg = flops.algorithmic(st)
        ach = alg / launches / (launch_ms * 1e-3) / 1e12
        # parity: tile rows cmp_rows (their image rows y) against the oracle at full spp
        ys = [rows[0] + t * rows[2] for t in cmp_rows]
        cpu = np.concatenate([oracle_lib.render(spheres, cam, make_params(W, H, spp, depth, seed0, rows=(y, 1, 1)),
                                                nthreads=nthreads)[0][:, xs] for y in ys])
        gpu = img[list(cmp_rows)]
        out[name] = {
            "workload": f"{W}x{H}x{spp}spp, max_depth {depth}, {os.path.relpath(scene_file, ROOT)} "
                        f"({len(spheres)} spheres), seed0 {seed0}, mt19937 + FP64"
                        + ((f", rows {rows[0]}::{rows[2]} ({rows[1]} rows = rank {split[0]} of {split[1]})"
                            if deal == "rows" else
                            f", 8-column bands {split[0]}::{split[1]} ({Wt} columns x {H} rows = rank "
                            f"{split[0]} of {split[1]})") if split else ""),
            "value": round(n / (ms * 1e-3) / 1e6, 3), "unit": "Msamples/s", "ms": round(ms, 3),
            "samples": n, "launches": launches,
            "roofline": {"bound": "valu", "achieved": round(ach, 4), "peak": peak_tf, "unit": "TFLOP/s",
                         "frac": round(ach / peak_tf, 5), "launch_ms": round(launch_ms, 4),
                         "algorithmic_flops_per_launch": round(alg / launches)},
            "segments_per_sample": round(st["segments"] / max(1, st["samples"]), 4),
            "mt_fallback_samples": st["mt_fallbacks"],
            "device_bytes": tst["device_bytes"],
            "call_bytes": tst["call_bytes"],
            "parity_vs_cpu": {"image_rows_compared": ys, "bytes_differing": int((gpu != cpu).sum()),
                              "max_abs_levels": int(np.abs(gpu.astype(int) - cpu.astype(int)).max())},
        }
    return out


def rank_tiles(ren, stream, seed0, frame, deal, steps, warmup):
    """The N-GPU bound on this GPU: every rank's tile of the N-way
    split under `deal` (8-column bands or single rows, tiles.py) rendered ALONE, timed exactly as
    the contract loop times the frame — `warmup` untimed calls, a synchronisation, then `steps`
    calls back to back (HIP events on the bench stream) — for config 3 at N = 2, 4, 8 and config
    4's eight tiles, and the other dealing at N = 8 for comparison.  Like with like: the first
    timed call starts synced (its launches ramp up) and the rest start while the
    previous call still runs, in the frame's steps and in the tiles' alike; a tile timed over fewer
    calls than the frame would carry a larger share of that first call (VERDICT r5's 1.086 was 4
    tile calls against 20 frame steps; profiles/r06b).  The slowest tile bounds the N-GPU step
    before the gather; `speedup_bound` = the single-GPU frame / the slowest tile.  `in_flight`
    figures leave the first call out (ms per call between the ends of calls 1 and K).
    frame: {"ms", "in_flight_ms"} of the contract loop (config 3)."""
    import torch

    import uecraytracing_amd as yk
    from uecraytracing_amd.records import image_height_for, make_params
    from uecraytracing_amd.tiles import rank_tile

    def call_ms(p, out, calls):
        # the contract loop's structure: warm-up calls, a sync, `calls` back-to-back calls; an
        # event on the stream after each call fires when that call's image is complete
        with torch.cuda.stream(stream):
            for _ in range(max(1, warmup)):
                ren.render_async(p, out.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        with torch.cuda.stream(stream):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(calls + 1)]
            ev[0].record(stream)
            for k in range(calls):
                ren.render_async(p, out.data_ptr(), stream.cuda_stream)
                ev[k + 1].record(stream)
        torch.cuda.synchronize()
        total = ev[0].elapsed_time(ev[calls]) / calls
        inflight = ev[1].elapsed_time(ev[calls]) / (calls - 1) if calls > 1 else total
        return total, inflight

    out = {"deal": deal, "steps": steps, "warmup": warmup,
           "method": "per tile: `warmup` calls, a sync, `steps` back-to-back calls (the contract loop's "
                     "structure); ms per call; in_flight = calls 2..K"}
    other = "rows" if deal == "cols" else "cols"
    for cfg, W, spp, ns in (("config3", 1920, 512, (2, 4, 8)), ("config4", 3840, 1024, (8,))):
        spheres, cam = yk.read_scene(os.path.join(yk.SCENE_DIR, "final_seed42.yks"))
        ren.set_scene(spheres, cam)
        H = image_height_for(W)
        # config 4's frame takes ~1.3 s per call: at most 6 calls for it and its tiles alike
        k = steps if cfg == "config3" else min(steps, 6)
        buf = torch.empty((H, W, 3), dtype=torch.uint8, device=torch.device("cuda", ren.device))
        if cfg == "config3":
            full, full_if = frame["ms"], frame["in_flight_ms"]
        else:
            full, full_if = call_ms(make_params(W, H, spp, 50, seed0, flags=0), buf, k)
        # the bench's dealing at every N; the other dealing at N = 8 for comparison
        for n, d in [(n, deal) for n in ns] + [(8, other)]:
            ms = [call_ms(make_params(W, H, spp, 50, seed0, flags=0, **rank_tile(r, n, H, W, d)), buf, k)
                  for r in range(n)]
            tot = [m[0] for m in ms]
            inf = [m[1] for m in ms]
            out[f"{cfg}_n{n}" + ("" if d == deal else f"_{d}")] = {
                "calls": k, "tile_ms": [round(m, 3) for m in tot], "slowest_ms": round(max(tot), 3),
                "frame_ms": round(full, 3), "speedup_bound": round(full / max(tot), 3),
                "slowest_over_ideal": round(max(tot) / (full / n), 4),
                "in_flight": {"tile_ms": [round(m, 3) for m in inf], "frame_ms": round(full_if, 3),
                              "slowest_over_ideal": round(max(inf) / (full_if / n), 4)}}
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the driver's own run: --steps 20 --warmup 5 (BENCH_r05.json); the per-rank tiles are timed over
    # the same number of calls (rank_tiles)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--spp", type=int, default=512)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--scene", default="final")
    ap.add_argument("--scene-seed", type=int, default=42)
    ap.add_argument("--seed0", type=int, default=404)
    ap.add_argument("--cpu-row-step", type=int, default=45,
                    help="CPU baseline renders every k-th row at full spp")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: every CPU this job may use)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-modes", action="store_true",
                    help="skip the one-call timings of the FP32 and xor128 modes (rank 0, N=1)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the BASELINE config 4 / 5 measurements (rank 0, N=1)")
    ap.add_argument("--deal", choices=("cols", "rows"), default=None,
                    help="N-GPU split: single rows (default, tiles.DEAL) or 8-column bands over every row")
    ap.add_argument("--no-tiles", action="store_true",
                    help="skip the per-rank tile timings of the N-GPU splits (rank 0, N=1)")
    return ap.parse_args()


def main():
    args = parse()
    if args.deal is None:
        from uecraytracing_amd.tiles import DEAL
        args.deal = DEAL
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist

    import uecraytracing_amd as yk
    from uecraytracing_amd import flops
    from uecraytracing_amd.records import image_height_for, make_params
    from uecraytracing_amd.tiles import BAND_LOG2, COL_BAND_LOG2, TileGather, rank_tile

    # one process per GPU; YK_BENCH_BACKEND=gloo (rehearsal only) lets several ranks share a GPU
    backend = os.environ.get("YK_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    dev = torch.device("cuda", local)

    W, spp, depth = args.width, args.spp, args.depth
    H = image_height_for(W)
    # the committed scene file of the config when there is one (identical to the seeded
    # generator's output, tests/test_scene_files.py), else the generator
    scene_file = os.path.join(yk.SCENE_DIR, f"{args.scene}_seed{args.scene_seed}.yks")
    if os.path.exists(scene_file):
        spheres, cam = yk.read_scene(scene_file)
    else:
        scene_file = None
        spheres, cam = yk.build_scene(args.scene, args.scene_seed)
    tk = rank_tile(rank, world, H, W, args.deal)  # this rank's rows (and columns): tiles.py
    params = make_params(W, H, spp, depth, args.seed0, flags=0, **tk)  # production instance
    pix_mine = params.row_count * params.tile_width()

    ren = yk.Renderer(local)
    # world + camera uploaded to HBM before any timing (the contract: inputs resident when the
    # timed region starts); SURVEY §8(d) counts the upload in the render call, so its cost (host
    # BVH builds + H2D copies, per rank) is timed here and reported beside the step
    up = []
    for _ in range(3):
        t = time.perf_counter()
        ren.set_scene(spheres, cam)
        up.append((time.perf_counter() - t) * 1e3)
    scene_upload_ms = sorted(up)[1]
    stream = torch.cuda.Stream(device=dev)
    tg = TileGather(rank, world, H, W, dev, deal=args.deal)  # tile, gather buffers and the assembled image
    ev = []

    def step(timed):
        with torch.cuda.stream(stream):
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            ren.render_async(params, tg.tile.data_ptr(), stream.cuda_stream)
            if timed:
                e1.record(stream)
                ev.append((e0, e1))
            tg.gather()  # RCCL gather to rank 0 + de-interleave (world > 1)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    call_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    # ms per step after the first (which starts synced): between the ends of steps 1
    # and K on the bench stream (HIP events; e1 of a step fires when its image is complete)
    step_in_flight_ms = (ev[0][1].elapsed_time(ev[-1][1]) / (len(ev) - 1)) if len(ev) > 1 else call_ms
    tst = ren.stats()  # per-kernel event timings of the last timed step (same stream)
    launches = max(1, tst["launches"])
    # work counters: one more launch of the same workload with the counting instance, after the
    # timed region (the work is deterministic, so its counts are the timed launches' counts)
    ren.render_async(make_params(W, H, spp, depth, args.seed0, flags=1, **tk),
                     tg.tile.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    st = ren.stats()
    total_samples = W * H * spp
    value = total_samples * args.steps / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    # Roofline of the dominant kernel, yk_render_persistent (`launches` launches per step).
    # Launch c + 1 starts on the CUs launch c's draining blocks free (two streams), so spans
    # overlap: the per-launch duration is the UNION of the spans / launches, never their sum.
    # Back-to-back steps also overlap each other: a step's first renders are enqueued
    # (their start events fire) while the previous step's last ones still hold the CUs, so the
    # union can exceed the step; the renders then run through the whole step period, which bounds
    # the per-step render time.
    busy_ms = tst["render_busy_ms"]
    clamped = busy_ms > ms_per_step
    launch_ms = min(busy_ms, ms_per_step) / launches
    # the FP64 VALU peak measured on this chip (tools/ubench.hip → profiles/r03_ubench.jsonl)
    peak_tf, peak_ev = flops.fp64_valu_peak()
    alg = flops.algorithmic(st)       # FP64 flops of the reference's expressions, per step
    impl = flops.implementation(st)   # counter-weighted FP64 operations the kernel executes
    achieved_tf = alg / launches / (launch_ms * 1e-3) / 1e12
    impl_tf = impl / launches / (launch_ms * 1e-3) / 1e12
    # SURVEY §8(d) algorithmic HBM bytes: the RGB8 image once, the scene once per workgroup
    scene_bytes = len(spheres) * SPHERE_RECORD_BYTES
    hbm_step = pix_mine * 3 + launches * tst["grid_blocks"] * scene_bytes
    hbm_gbps = hbm_step / launches / (launch_ms * 1e-3) / 1e9
    workload = f"{args.scene}{args.scene_seed}_{W}x{H}x{spp}_d{depth}_n{world}"
    facts = pmc_facts(workload)
    traffic = facts.get("hbm_bytes_per_launch") if facts else None
    # per SAMPLE, so that the ratio compares like with like (the PMC passes profile synced calls,
    # whose launches are smaller on average than the bench's back-to-back ones)
    traffic_ps = facts.get("hbm_bytes_per_sample") if facts else None
    alg_ps = hbm_step / (pix_mine * spp)
    # The VALU lane-op roofline of the path's whole work (flops.py: FP64 flops + the RNG's
    # integer ops, by kernel): the seed walks (yk_mt_warmup) and the paths (yk_render_persistent)
    # share every SIMD, so the STEP figure (both kernels' work over the step) is the path's; each
    # kernel's own figure divides by its own per-launch span
    costs, costs_src = flops.issue_costs()
    lo = flops.lane_ops(st)
    both = {k: lo["warmup"][k] + lo["render"][k] for k in lo["render"]}
    per_l = lambda d: {k: v / launches for k, v in d.items()}
    valu_ops = {
        "render": dict(flops.lane_op_roofline(per_l(lo["render"]), launch_ms * 1e-3, costs),
                       kernel="yk_render_persistent", per="launch", seconds_source="launch_ms"),
        "warmup": dict(flops.lane_op_roofline(per_l(lo["warmup"]), tst["warmup_ms"] / launches * 1e-3, costs),
                       kernel="yk_mt_warmup", per="launch",
                       seconds_source="the step's warm-up HIP-event spans / launches"),
        "step": dict(flops.lane_op_roofline(both, ms_per_step * 1e-3, costs), per="step",
                     seconds_source="ms_per_step (both kernels share the SIMDs)"),
        "issue_cycles_per_wave_instr": costs, "issue_cycles_source": costs_src,
        "per_sample": {k: round(v / st["samples"], 2) for k, v in both.items()},
        "counted": {"words_drawn": st["work"][5], "words_drawn_by_warmup": st["work"][6],
                    "mt_twists": st["work"][7], "mt_fallback_samples": st["mt_fallbacks"]},
        "algorithmic": "the reference's operators for the work done (uecraytracing_amd/flops.py lane_ops): "
                       "FP64 flops + per sample the 397-step seeding walk (4 ops/step) + per engine word "
                       "21 integer ops (next seeding step, twisted word, tempering) and 3 FP64 (canonical) "
                       "+ the full engine's seeding and twists past draw 227",
        "reconcile": pmc_lane_ops(),
    }
    issue = None
    if facts and "valu_pipe_util" in facts and "valu_lane_utilization" in facts:
        issue = {"valu_busy": round(facts["valu_pipe_util"], 4),
                 "lane_utilization": round(facts["valu_lane_utilization"], 4),
                 "busy_x_lanes": round(facts["valu_pipe_util"] * facts["valu_lane_utilization"], 4),
                 "source": "PMC (profiles/pmc_summary.json): VALU busy = SQ_INSTS_VALU x 2 cycles "
                           "(SIMD-32) / GRBM_GUI_ACTIVE per XCD; lanes = SQ_THREAD_CYCLES_VALU / "
                           "(64 SQ_ACTIVE_INST_VALU)"}

    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"BASELINE config 3: {W}x{H}x{spp}spp, max_depth {depth}, RTIOW final "
                        f"scene ({len(spheres)} spheres, generator seed {args.scene_seed}), "
                        f"seed0 {args.seed0}, mt19937 + FP64 bit-exact",
            "image": f"{W}x{H}", "spp": spp, "max_depth": depth, "spheres": len(spheres),
            "scene_file": os.path.relpath(scene_file, ROOT) if scene_file else None,
            "partition": ((f"rows dealt cyclically in bands of {1 << BAND_LOG2}" if BAND_LOG2 else
                           "single rows dealt cyclically (row r -> rank r mod N)") if args.deal == "rows" else
                          f"columns dealt cyclically in bands of {1 << COL_BAND_LOG2} (every row)")
                         + f" over {world} GPU(s), "
                         + ("RCCL gather to rank 0" if backend == "nccl" else
                            f"{backend} gather to rank 0 through the host (rehearsal: ranks share a GPU)"),
        },
        "ms_per_step_in_flight": round(step_in_flight_ms, 3),
        "scene_upload_ms": round(scene_upload_ms, 3),
        "value_incl_scene_upload": round(total_samples * args.steps
                                         / (elapsed + args.steps * scene_upload_ms * 1e-3) / 1e6, 3),
        # the path is VALU-bound (FP64 vector arithmetic under divergence), neither
        # HBM- nor MFMA-bound; the HBM view is a sub-object
        "roofline": {
            "bound": "valu",
            "achieved": round(achieved_tf, 4),
            "peak": peak_tf,
            "unit": "TFLOP/s",
            "frac": round(achieved_tf / peak_tf, 5),
            "peak_evidence": peak_ev,
            "frac_of_spec": round(achieved_tf / flops.SPEC_FP64_VALU_TFLOPS, 5),
            "traffic": traffic,
            "kernel": "yk_render_persistent",
            "launches_per_step": launches,
            "launch_ms": round(launch_ms, 4),
            "launch_ms_source": "min(union of the step's render HIP-event spans (render_busy_ms), the step "
                                "period) / launches; the rocprofv3 kernel-trace union per dispatch is in "
                                "profiles/<tag>_kernel_union.json",
            "algorithmic_flops_per_launch": round(alg / launches),
            "algorithmic": f"FP64 flops of the reference's expressions, {flops.algorithmic_terms()}, "
                           f"over the kernel's work counters: {alg:.5g} per step / {launches} launches",
            "implementation": {
                "flops_per_launch": round(impl / launches),
                "achieved": round(impl_tf, 4),
                "frac": round(impl_tf / peak_tf, 5),
                "note": "FP64 operations the kernel executes (divisions as rcp+FMA sequences, "
                        "math::sqrt's start and steps, the BVH's root bounds), weighted as "
                        "SQ_INSTS_VALU_FLOPS_FP64 weighs them (uecraytracing_amd/flops.py)",
                "counter_check": fp64_reconcile_facts(),
            },
            "issue": issue,
            "hbm": {"algorithmic_bytes_per_launch": round(hbm_step / launches),
                    "algorithmic_achieved": round(hbm_gbps, 4), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "algorithmic_frac": round(hbm_gbps / HBM_PEAK_GBPS, 7),
                    # the whole step's PMC-measured traffic (render + warm-up + reduce) as GB/s
                    "measured": hbm_measured(pix_mine * spp, ms_per_step, alg_ps),
                    "render_kernel_traffic_per_launch": traffic,
                    "render_kernel_traffic_per_sample": round(traffic_ps, 3) if traffic_ps else None,
                    "algorithmic_bytes_per_sample": round(alg_ps, 4),
                    "render_kernel_traffic_over_algorithmic": round(traffic_ps / alg_ps, 1) if traffic_ps else None,
                    "device_bytes": tst["device_bytes"], "call_bytes": tst["call_bytes"],
                    "algorithmic": f"SURVEY §8(d): the RGB8 image ({pix_mine * 3} B) once per "
                                   f"step + the scene ({scene_bytes} B) once per workgroup "
                                   f"({tst['grid_blocks']} per launch); render_kernel_traffic = PMC FETCH_SIZE "
                                   f"x2 + WRITE_SIZE of yk_render_persistent alone (scratch: the start "
                                   f"records, the colour records, MT fallback state); `measured` adds "
                                   f"the warm-up and reduce kernels: the step's traffic"},
            # the union of the step's render spans can exceed the step (a step's first renders are
            # enqueued while the previous step's still run): then launch_ms is the step / launches
            "launch_ms_unclamped": round(busy_ms / launches, 4),
            "launch_ms_clamped_to_step": bool(clamped),
            "valu_ops": valu_ops,
            # render = the launches' spans summed (they overlap); render_busy = their union
            "step_breakdown_ms": {"render_spans_summed": round(tst["kernel_ms"], 3),
                                  "render_busy": round(busy_ms, 3),
                                  "mt_warmup": round(tst["warmup_ms"], 3),
                                  "reduce": round(tst["resolve_ms"], 3), "call": round(call_ms, 3)},
            "pmc": facts,
            "segments_per_sample": round(st["segments"] / max(1, st["samples"]), 4),
            "tests_per_segment": round(st["sphere_tests"] / max(1, st["segments"]), 2),
            "node_visits_per_segment": round(st["node_visits"] / max(1, st["segments"]), 2),
        },
        "cpu_baseline": None,
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import numpy as np

        import oracle_lib

        rows = list(range(0, H, args.cpu_row_step))
        usable, node_cpus, quota = usable_cpus()
        nthreads = args.cpu_threads or usable
        cp = make_params(W, H, spp, depth, args.seed0,
                         rows=(0, len(rows), args.cpu_row_step))
        t = time.perf_counter()
        cpu_rgb, _, _, _ = oracle_lib.render(spheres, cam, cp, nthreads=nthreads)
        dt = time.perf_counter() - t
        n = len(rows) * W * spp
        gpu_rows = tg.image[::args.cpu_row_step].cpu().numpy()
        diff = (gpu_rows.astype(np.float64) - cpu_rgb.astype(np.float64)) / 255.0
        result["cpu_baseline"] = {
            "value": round(n / dt / 1e6, 4),
            "unit": "Msamples/s",
            "cores": nthreads,
            "kind": "port",
            "sample": f"{len(rows)} rows (every {args.cpu_row_step}th) x {W} px x {spp} spp = "
                      f"{n} samples of the same workload, {dt:.1f} s, oracle/yk_oracle.c "
                      f"(-O2, {nthreads} threads)",
            "host": {"node_logical_cpus": node_cpus, "cgroup_cpu_quota": quota,
                     "threads_used": nthreads,
                     "note": "threads = every CPU this job may use (affinity capped by the cgroup "
                             "quota); the node's other CPUs belong to other jobs"},
        }
        # SURVEY §8(d) variants: the same port on ONE core (one row), and the reference's
        # as-shipped cost model (a random_device seed per sample, source.cpp:159) on all threads
        r1 = make_params(W, H, spp, depth, args.seed0, rows=(H // 2, 1, 1))
        t = time.perf_counter()
        oracle_lib.render(spheres, cam, r1, nthreads=1)
        dt1 = time.perf_counter() - t
        rows_as = list(range(0, H, args.cpu_row_step * 4))
        ra = make_params(W, H, spp, depth, args.seed0, rows=(0, len(rows_as), args.cpu_row_step * 4))
        t = time.perf_counter()
        oracle_lib.render_as_shipped(spheres, cam, ra, nthreads=nthreads)
        dta = time.perf_counter() - t
        result["cpu_baseline"]["variants"] = {
            "port_1_core": {"value": round(W * spp / dt1 / 1e6, 4), "cores": 1,
                            "sample": f"row {H // 2} x {W} px x {spp} spp, {dt1:.1f} s"},
            "as_shipped_cost_model": {
                "value": round(len(rows_as) * W * spp / dta / 1e6, 4), "cores": nthreads,
                "sample": f"{len(rows_as)} rows (every {args.cpu_row_step * 4}th) x {W} px x {spp} spp, "
                          f"{dta:.1f} s; a random_device seed per sample as in the runtime build "
                          f"(source.cpp:159), so not reproducible"},
        }
        cal = reference_calibration(args.seed0, nthreads)
        result["cpu_baseline"]["reference_calibration"] = cal
        fin = cal.get("all_cores", {}).get("final48", {})
        if "harness_msps" in fin:
            # the reference's own loop on every usable core (the 48-sphere slice: the 485-sphere
            # scene does not compile through its tuple API), beside the port on the same cores
            result["cpu_baseline"]["variants"]["reference_loop_all_cores"] = {
                "value": fin["harness_msps"], "cores": nthreads, "kind": "reference",
                "port_same_cores_same_scene": fin["port_msps"],
                "port_over_reference": fin["port_over_harness"], "images_equal": fin["images_equal"],
                "sample": cal["method"].split("; all_cores: ")[1].split(";")[0] + ", tests/golden/final48.yks"}
        result["parity_vs_cpu"] = {
            "rows_compared": len(rows),
            "rmse": float(np.sqrt(np.mean(diff ** 2))),
            "max_abs_levels": int(np.abs(gpu_rows.astype(int) - cpu_rgb.astype(int)).max()),
            "bytes_differing": int((gpu_rows != cpu_rgb).sum()),
        }

    if rank == 0 and world == 1 and not args.no_modes:
        # The reference's other arithmetic and engine on the same workload, after everything
        # above: render<float> (its own tree) and the yk::xor128 engine.  Each is
        # bit-exact against the reference in its own mode; neither is the contract's `value`.
        from uecraytracing_amd.records import PRECISION_FP32, RNG_XOR128
        scratch = torch.empty_like(tg.tile)
        modes = {}
        for name, kw in (("fp32_mt19937", {"precision": PRECISION_FP32}), ("fp64_xor128", {"rng": RNG_XOR128})):
            mp = make_params(W, H, spp, depth, args.seed0, **tk, **kw)
            ren.render_async(mp, scratch.data_ptr(), stream.cuda_stream)  # warm-up call
            torch.cuda.synchronize()
            t = time.perf_counter()
            ren.render_async(mp, scratch.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            modes[name] = {"value": round(total_samples / dt / 1e6, 3), "unit": "Msamples/s",
                           "ms": round(dt * 1e3, 3)}
        result["modes"] = modes

    if rank == 0 and world == 1 and not args.no_configs:
        result["configs"] = other_configs(ren, stream, args.seed0, args.cpu_threads or usable_cpus()[0], peak_tf,
                                          args.deal)

    if rank == 0 and world == 1 and not args.no_tiles and (W, spp, depth, args.scene) == (1920, 512, 50, "final"):
        result["tiles"] = rank_tiles(ren, stream, args.seed0, {"ms": ms_per_step, "in_flight_ms": step_in_flight_ms},
                                     args.deal, args.steps, args.warmup)

    if rank == 0:
        print(json.dumps(result), flush=True)
    ren.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
