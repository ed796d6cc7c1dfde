"""Per-kernel dispatch durations from a rocprofv3 kernel trace (diagnostic): count, mean and total ms
per kernel name (template arguments kept), in dispatch order of first appearance.
usage: python tools/kernel_durations.py <run_kernel_trace.csv>"""
import collections
import csv
import re
import sys

agg = collections.OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    name = re.sub(r"\(anonymous namespace\)::|\(\(anonymous namespace\)::\w+\)$|^void ", "", r["Kernel_Name"])
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    agg.setdefault(name, []).append(d)
for k, v in agg.items():
    print(f"{len(v):5d} x {sum(v) / len(v):8.3f} ms = {sum(v):9.3f} ms  {k}")
