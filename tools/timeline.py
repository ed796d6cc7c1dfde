"""Per-dispatch timeline of one render call from a rocprofv3 kernel trace (run_kernel_trace.csv):
the warm-up, render and reduce dispatches with start/end relative to the first, and the idle gaps
of the render stream.  usage: python tools/timeline.py <kernel_trace.csv> [call index]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
want = int(sys.argv[2]) if len(sys.argv) > 2 else -1
# calls: a call starts with a warm-up that follows a reduce with ra.last (group by gaps > 5 ms)
kinds = {"yk_mt_warmup": "W", "yk_render_persistent": "R", "yk_render_counting": "R", "yk_render_f32": "R", "yk_reduce_samples": "S"}
ev = []
for r in rows:
    k = next((v for n, v in kinds.items() if n in r["Kernel_Name"]), None)
    if k:
        ev.append((k, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
calls, cur = [], []
for e in ev:
    if cur and e[0] == "W" and e[1] > max(x[2] for x in cur) + 1_000_000:
        calls.append(cur)
        cur = []
    cur.append(e)
calls.append(cur)
c = calls[want]
t0 = c[0][1]
for k, a, b in c:
    print(f"{k} {(a - t0) / 1e6:9.3f} {(b - t0) / 1e6:9.3f} {(b - a) / 1e6:8.3f}")
r = sorted((a, b) for k, a, b in c if k == "R")
busy, end = 0, r[0][0]
for a, b in r:
    busy += max(0, b - max(a, end))
    end = max(end, b)
print(f"call {(max(x[2] for x in c) - t0) / 1e6:.3f} ms, render union {busy / 1e6:.3f} ms, first render at "
      f"{(r[0][0] - t0) / 1e6:.3f} ms, last render end {(end - t0) / 1e6:.3f} ms")
