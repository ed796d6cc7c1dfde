"""Per-function comparison of two gfx950 device assembly files (hipcc --cuda-device-only -S):
which kernels' instruction streams are identical after normalising local labels.  Used to show
that a source cleanup left the compiled kernels unchanged.
usage: python tools/isa_diff.py before.s after.s"""
import re
import sys


def funcs(path):
    out, cur = {}, None
    for line in open(path).read().split("\n"):
        m = re.match(r"^(_Z\S+):\s", line + " ")
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur:
            if line.startswith(".Lfunc_end"):
                cur = None
                continue
            line = re.sub(r"\.LBB\d+_\d+", "L", line)
            line = re.sub(r"\s*;.*$", "", line)  # trailing comments (basic-block numbers)
            if line.strip().startswith(";"):
                continue
            out[cur].append(line)
    return out


a, b = funcs(sys.argv[1]), funcs(sys.argv[2])
diff = 0
for k in sorted(set(a) | set(b)):
    if k not in a or k not in b:
        print("ONLY", "before" if k in a else "after", k)
        diff += 1
        continue
    same = a[k] == b[k]
    diff += not same
    print("SAME" if same else "DIFF", len(a[k]), len(b[k]), k)
sys.exit(1 if diff else 0)
