"""Per-step kernel timeline from a rocprofv3 results .db (SQLite).

usage: python tools/db_steps.py <run_results.db> [--step -2] [--family]
Steps are delimited by the AdamW launch (one per optimizer step).  Prints
each kernel of the chosen step with its duration, grid and the idle gap
before it, and the step's wall time vs the sum of kernel time.
"""
import argparse, collections, re, sqlite3


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    m = re.search(r"(conv_glds_kernel|conv_gemm_kernel)<(\d+), ([^>]*)>", n)
    if m:
        return f"{m.group(1)}<{'fdw'[int(m.group(2))]},{m.group(3).replace(' ', '')}>"
    return n.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--family", action="store_true")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, grid_y, workgroup_x, stream_id from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if "adamw" in r[0] and "sched" not in r[0]]
    i0, i1 = ends[a.step - 1] + 1, ends[a.step] + 1
    step = rows[i0:i1]
    wall = (step[-1][2] - rows[i0 - 1][2]) / 1e3
    busy = sum((r[2] - r[1]) for r in step) / 1e3
    fam = collections.defaultdict(lambda: [0.0, 0])
    prev_end = rows[i0 - 1][2]
    for r in step:
        d = (r[2] - r[1]) / 1e3
        gap = (r[1] - prev_end) / 1e3
        prev_end = max(prev_end, r[2])
        k = short(r[0])
        key = re.sub(r"<.*", "", k) if a.family else k
        fam[key][0] += d
        fam[key][1] += 1
        if not a.family:
            print(f"{d:8.1f}us gap {gap:6.1f} s{r[6]} grid {r[3] // max(1, r[5]):6d}x{r[4]:<3d} {k}")
    print(f"step wall {wall:.1f} us, kernel busy {busy:.1f} us")
    for k, (t, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        print(f"{t:9.1f}us {n:4d}x  {k}")


if __name__ == "__main__":
    main()
