"""Per-launch duration of a kernel from a rocprofv3 kernel trace, counting overlap once.

The render launches alternate between two streams and overlap (launch c + 1 starts on the CUs
launch c's draining blocks free), so rocprofv3's per-dispatch average counts the overlapped time
twice.  This reports, for the dispatches whose name contains the substring: the plain average
span (what --stats prints), the UNION of the spans, and union / dispatches — the figure bench.py
divides by (`roofline.launch_ms`).
usage: python tools/kernel_union.py <run_kernel_trace.csv> [kernel-substring[|substring...]] [out.json]
                                    [spp_total spp_per_launch [last_launches]]
With spp_total (every sample per pixel the traced run rendered with this kernel) and the bench's
launch size, also union_per_launch_equiv_ms = union / (spp_total / spp_per_launch): the traced
run mixes synced calls (launches of 4, 8, 16, 32 spp) and back-to-back ones (64 each, round 6), so
this is the figure comparable with the bench's per-launch launch_ms.
With last_launches, also union_last_call_per_launch_ms: the union of the last that many dispatches
(the traced run's last call, started in flight, its last launch draining alone) / that many.
Several substrings ('|'-separated) take the union of all their dispatches (kernels that share a
launch); "launches" = the dispatches of the LAST substring (one per launch).
"""
import csv
import json
import sys


def main():
    path = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "yk_render_persistent<true, 0>"
    names = kern.split("|")
    rows = list(csv.DictReader(open(path)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                for r in rows if any(k in r["Kernel_Name"] for k in names))
    launches = sum(1 for r in rows if names[-1] in r["Kernel_Name"])
    if not iv:
        raise SystemExit(f"no dispatch of {kern!r} in {path}")
    union = 0
    cur_s, cur_e = iv[0]
    for s, e in iv[1:]:
        if s > cur_e:
            union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    spans = sum(e - s for s, e in iv)
    out = {"trace": path, "kernel": kern, "dispatches": len(iv), "launches": launches,
           "avg_span_ms": spans / len(iv) / 1e6, "union_ms": union / 1e6,
           "union_per_dispatch_ms": union / max(1, launches) / 1e6,
           "overlap_fraction_of_spans": 1 - union / spans}
    if len(sys.argv) > 5:
        spp_total, per = float(sys.argv[4]), float(sys.argv[5])
        out["spp_total"], out["spp_per_launch"] = spp_total, per
        out["union_per_launch_equiv_ms"] = union / (spp_total / per) / 1e6
    if len(sys.argv) > 6:
        n = int(sys.argv[6])
        last = iv[-n:]
        u, (cs, ce) = 0, last[0]
        for s_, e_ in last[1:]:
            if s_ > ce:
                u, cs, ce = u + ce - cs, s_, e_
            else:
                ce = max(ce, e_)
        u += ce - cs
        out["last_launches"] = n
        out["union_last_call_per_launch_ms"] = u / n / 1e6
    js = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
