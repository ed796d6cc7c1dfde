"""Per-launch union of the render spans of configs 4 and 5 from the kernel trace of
`rocprofv3 --kernel-trace -- python3 tools/configs45.py c4 c5`: each config renders a warm call and
a timed call with the production instance (then a counting call, another instance), so the
production dispatches come as [c4 warm, c4 timed, c5 warm, c5 timed]; the timed call's union of
spans / its launches is the figure bench.py reports as the configs' roofline.launch_ms.
usage: python tools/configs45_union.py <run_kernel_trace.csv> <out.json> [n_c4 n_c5]"""
import csv
import json
import sys

KERNEL = "yk_render_persistent<true, 0>"


def union(iv):
    iv = sorted(iv)
    tot, (cs, ce) = 0, iv[0]
    for s, e in iv[1:]:
        if s > ce:
            tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + ce - cs


def main():
    path, out = sys.argv[1], sys.argv[2]
    n4, n5 = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (32, 129)
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path))
                   if KERNEL in r["Kernel_Name"]))
    if len(rows) != 2 * (n4 + n5):
        raise SystemExit(f"{len(rows)} dispatches of {KERNEL}, expected {2 * (n4 + n5)}")
    res = {}
    for name, lo, n in (("config4_rank0_of_8", n4, n4), ("config5", 2 * n4 + n5, n5)):
        iv = rows[lo:lo + n]
        u = union(iv)
        res[name] = {"trace": f"{path} (tools/configs45.py c4 c5 under rocprofv3 --kernel-trace)", "kernel": KERNEL,
                     "timed_call_dispatches": n, "union_ms": u / 1e6, "union_per_dispatch_ms": u / n / 1e6,
                     "avg_span_ms": sum(e - s for s, e in iv) / n / 1e6}
    js = json.dumps(res, indent=1)
    open(out, "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
