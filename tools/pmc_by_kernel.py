"""Per-kernel PMC summary of a tools/timeline_once.py run (two identical calls: a warm one, then the
timed one) — the second half of each kernel's dispatches, merged over the --pmc pass directories.

usage: python tools/pmc_by_kernel.py <samples> <out.json> <label>=<dir>[,<dir>...] ...

Per kernel: SQ_INSTS_VALU per sample, VALU lane utilisation (SQ_THREAD_CYCLES_VALU /
(64 SQ_ACTIVE_INST_VALU)), waves, and wave-cycles (SQ_WAVE_CYCLES) split into issuing
(SQ_ACTIVE_INST_ANY) and waiting (SQ_WAIT_ANY) — whatever counters the passes hold.
Used for the first-segment split A/B (profiles/r05_ab/split/)."""
import collections
import csv
import json
import os
import sys


def kernels(dirs):
    per = collections.defaultdict(lambda: collections.OrderedDict())
    for d in dirs:
        rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
        disp = collections.OrderedDict()
        for r in rows:
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            k = (name.split("(")[0], int(r["Dispatch_Id"]))
            disp.setdefault(k, {})[r["Counter_Name"]] = float(r["Counter_Value"])
        byk = collections.defaultdict(list)
        for (name, _), c in disp.items():
            byk[name].append(c)
        for name, cs in byk.items():
            timed = cs[len(cs) // 2:]
            acc = per[name]
            acc["dispatches"] = len(timed)
            for c in timed:
                for ctr, v in c.items():
                    acc[ctr] = acc.get(ctr, 0.0) + v
    return per


def summary(per, samples):
    out = {}
    for name, c in per.items():
        if "rocclr" in name:
            continue
        s = {"dispatches": c["dispatches"]}
        if "SQ_INSTS_VALU" in c:
            s["valu_wave_instr_per_sample"] = round(c["SQ_INSTS_VALU"] / samples, 3)
        if "SQ_THREAD_CYCLES_VALU" in c and c.get("SQ_ACTIVE_INST_VALU"):
            s["valu_lane_utilization"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"]), 4)
        for k in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                  "SQ_ACTIVE_INST_ANY", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU",
                  "SQ_INSTS_SMEM", "SQ_WAIT_INST_LDS", "SQ_INST_CYCLES_VMEM_RD"):
            if k in c:
                s[k] = c[k]
        if c.get("SQ_WAVE_CYCLES"):
            for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"):
                if k in c:
                    s[k.lower() + "_share_of_wave_cycles"] = round(c[k] / c["SQ_WAVE_CYCLES"], 4)
        out[name] = s
    return out


def main():
    samples = float(sys.argv[1])
    out = sys.argv[2]
    res = {"samples_per_call": samples, "source": "rocprofv3 --pmc over tools/timeline_once.py (timed call)"}
    for arg in sys.argv[3:]:
        label, dirs = arg.split("=", 1)
        res[label] = summary(kernels(dirs.split(",")), samples)
    js = json.dumps(res, indent=1)
    open(out, "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
