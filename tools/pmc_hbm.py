"""HBM bytes per sample of each kernel of a launch, from tools/pmc_profile.sh's passes (VERDICT r5
item 3: the step's measured HBM traffic, not only the render kernel's).

Per kernel: bytes = FETCH_SIZE x 2 x 1024 (gfx950 reports half of a wide streaming read,
MI355X_MICROARCH.md §HBM; the factor is applied to every read as the render's summary always
did) + WRITE_SIZE x 1024, summed over the kernel's dispatches in the pass that holds the counter;
frames = dispatches / launches per frame (each bench run renders whole frames: the warm-up step,
the timed step, the counting call — the production render instance is not used by the counting
call, so it sees two frames where the warm-up and reduce kernels see three); per sample = bytes /
(frames x samples per frame).
usage: python tools/pmc_hbm.py <pmc dir> <samples per frame> <launches per frame> [out.json] [tag]"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = {  # name in the line → substring of the kernel name
    "render": "yk_render_persistent<true, 0>",
    "warmup": "yk_mt_warmup",
    "reduce": "yk_reduce_samples",
}


def summarise(d, samples_per_frame, launches_per_frame):
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] not in ("FETCH_SIZE", "WRITE_SIZE"):
                continue
            for k, sub in KERNELS.items():
                if sub in r["Kernel_Name"]:
                    tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
                    disp[(k, r["Counter_Name"])].add((f, r["Dispatch_Id"]))
    out = {"source": f"rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE passes, {d}",
           "samples_per_frame": samples_per_frame, "launches_per_frame": launches_per_frame,
           "bytes": "FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024 (MI355X_MICROARCH.md: FETCH_SIZE reads "
                    "half of a wide streaming read on gfx950)", "kernels": {}}
    total = 0.0
    for k, sub in KERNELS.items():
        row = {"kernel": sub}
        for c, scale in (("FETCH_SIZE", 2048.0), ("WRITE_SIZE", 1024.0)):
            n = len(disp[(k, c)])
            if n == 0:
                raise SystemExit(f"no {c} dispatches of {sub} in {d}")
            frames = n / launches_per_frame
            row[c.lower().replace("_size", "") + "_bytes_per_sample"] = tot[(k, c)] * scale / (frames * samples_per_frame)
            row["frames_" + c.lower()] = frames
        row["bytes_per_sample"] = row["fetch_bytes_per_sample"] + row["write_bytes_per_sample"]
        total += row["bytes_per_sample"]
        out["kernels"][k] = row
    out["bytes_per_sample"] = total
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1], int(float(sys.argv[2])), int(sys.argv[3]))
    js = json.dumps(res, indent=1)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(js + "\n")
    print(js)
