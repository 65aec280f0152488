"""Per-kernel-family device time per step (mean over three timed steps) by
stream, from a rocprofv3 kernel trace of bench.py.
usage: step_families.py run_kernel_trace.csv [other_trace.csv]  (two: side by side)"""
import collections
import csv
import re
import sys


def families(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "weight_prep_batch" in r["Kernel_Name"]]
    tot, cnt = collections.Counter(), collections.Counter()
    steps = (-4, -3, -2)
    for k in steps:
        for r in rows[ends[k - 1]:ends[k]]:
            n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", r["Kernel_Name"])
            n = re.sub(r"\(anonymous namespace\)::", "", n).replace("void ", "")
            m = re.match(r"[A-Za-z_]+", n)
            key = (m.group(0) if m else n[:20], r["Stream_Id"])
            tot[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / len(steps)
            cnt[key] += 1 / len(steps)
    wall = sum(int(rows[ends[k]]["Start_Timestamp"]) - int(rows[ends[k - 1]]["Start_Timestamp"]) for k in steps)
    return tot, cnt, wall / 1e3 / len(steps)


ts = [families(p) for p in sys.argv[1:]]
keys = sorted(set().union(*[t[0] for t in ts]), key=lambda k: -max(t[0].get(k, 0) for t in ts))
print("step wall (us): " + "  ".join(f"{t[2]:8.1f}" for t in ts))
for k in keys:
    print("  ".join(f"{t[0].get(k, 0):8.1f} {t[1].get(k, 0):4.0f}x" for t in ts) + f"  s{k[1]} {k[0]}")
