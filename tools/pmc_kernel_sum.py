"""Per-dispatch averages of every PMC counter in a rocprofv3 counter_collection.csv
for the kernels whose name contains a substring (one line per counter).
usage: pmc_kernel_sum.py <counter_collection.csv> <kernel substring> [label]"""
import collections
import csv
import sys

path, sub = sys.argv[1], sys.argv[2]
label = sys.argv[3] if len(sys.argv) > 3 else sub
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for r in csv.DictReader(open(path)):
    if sub not in r["Kernel_Name"]:
        continue
    tot[r["Counter_Name"]] += float(r["Counter_Value"])
    disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for c in sorted(tot):
    n = len(disp[c])
    print(f"{label:24s} {c:28s} per dispatch {tot[c] / n:14.4g}  ({n} dispatches)")
