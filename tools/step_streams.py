"""Per-stream busy time, idle time and main-stream gaps of one timed step of a
rocprofv3 kernel trace (CSV) of bench.py, plus the step's first and last
launches.  usage: step_streams.py run_kernel_trace.csv [step_index]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else -3
# a step starts with its batched compute-dtype weight refresh (SemiStep)
ends = [i for i, r in enumerate(rows) if "weight_prep_batch" in r["Kernel_Name"]]
step = rows[ends[k - 1]:ends[k]]
t0 = int(step[0]["Start_Timestamp"])
t1 = int(rows[ends[k]]["Start_Timestamp"])
print(f"one step (weight refresh to the next step's): wall {(t1 - t0) / 1e3:.1f} us, {len(step)} launches")
by = collections.defaultdict(list)
for r in step:
    by[r["Stream_Id"]].append(r)
for sid, rs in sorted(by.items()):
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e3
    span = (max(int(r["End_Timestamp"]) for r in rs) - int(rs[0]["Start_Timestamp"])) / 1e3
    print(f"  stream {sid}: {len(rs):3d} launches, busy {busy:7.1f} us over a span of {span:7.1f} us")
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
u, (cs, ce) = 0, iv[0]
for s, e in iv[1:]:
    if s > ce:
        u += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
u += ce - cs
print(f"  any stream busy {u / 1e3:.1f} us, all idle {(t1 - t0 - u) / 1e3:.1f} us")
# the all-idle intervals (no kernel of any stream running), largest first, with
# the kernel that ended before and the one that started after
idle = []
cs, ce, last = iv[0][0], iv[0][1], None
ends_at = {}
for r in step:
    ends_at.setdefault(int(r["End_Timestamp"]), r["Kernel_Name"])
for s, e in iv[1:] + [(t1, t1)]:
    if s > ce:
        before = max((r for r in step if int(r["End_Timestamp"]) <= s), key=lambda r: int(r["End_Timestamp"]))
        after = min((r for r in rows if int(r["Start_Timestamp"]) >= s), key=lambda r: int(r["Start_Timestamp"]),
                    default=None)
        idle.append(((s - ce) / 1e3, (ce - t0) / 1e3, before["Kernel_Name"][:40],
                     after["Kernel_Name"][:40] if after else "-"))
        cs, ce = s, e
    else:
        ce = max(ce, e)
idle.sort(reverse=True)
print(f"  all-idle intervals: {len(idle)}, largest:")
for g in idle[:8]:
    print("    %7.1f us at %8.1f  %s -> %s" % g)
main = max(by.values(), key=len)
gaps = sorted(((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3, a["Kernel_Name"][:48],
               b["Kernel_Name"][:48]) for a, b in zip(main, main[1:]))[::-1]
print(f"  main-stream gaps: {sum(g for g, _, _ in gaps):.1f} us; largest:")
for g in gaps[:5]:
    print("    %7.1f us  %s -> %s" % g)


def show(rs):
    for r in rs:
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:64]
        print(f"  {s:8.1f} {e:8.1f} {e - s:7.1f}  stream {r['Stream_Id']}  {n}")


print("first launches:")
show(step[:10])
print("last launches:")
show(step[-12:])
