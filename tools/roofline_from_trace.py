"""Recompute bench.py's conv-family roofline fraction from a rocprofv3 kernel
trace of `python bench.py --profile-leg {full,production} --steps K`.

The leg's last step is the last instrumented one (the launches from the last
`weight_prep_batch` launch -- every step's head -- to the end of the trace).
Its conv-family kernel durations are summed (the same launches bench.py's
HIP-event brackets time: conv_glds / conv_gemm / conv_halo* / conv_stem* and
the wgrad slab reduces), and

    frac = conv TFLOP per step / summed duration / peak

with the TFLOP of the workload (3.1895 for the config-3 step).
Also prints per-kernel rows so the dominant kernel's average launch duration
can be compared with the line's.

usage: roofline_from_trace.py <kernel_trace.csv> [--tflop 3.1895] [--peak 2500] [--out f.txt]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\((?![^<]*>).*", "", name)
    return name[:80]


def is_conv(n):
    return any(k in n for k in ("conv_glds_kernel", "conv_gemm_kernel", "conv_halo", "conv_stem", "wgrad_reduce"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tflop", type=float, default=3.1895)
    ap.add_argument("--peak", type=float, default=2500.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    heads = [i for i, r in enumerate(rows) if "weight_prep_batch" in r["Kernel_Name"]]
    step = rows[heads[-1]:]
    agg = collections.OrderedDict()
    tot = 0.0
    n = 0
    for r in step:
        if not is_conv(r["Kernel_Name"]):
            continue
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        d = agg.setdefault(short(r["Kernel_Name"]), [0, 0.0])
        d[0] += 1
        d[1] += us
        tot += us
        n += 1
    ach = a.tflop / (tot * 1e-6)
    lines = [f"# conv-family launches of the last step of {a.label or a.trace} (rocprofv3 kernel trace)",
             f"# {n} launches, {tot:.1f} us; {a.tflop} TFLOP / {tot:.1f} us = {ach:.1f} TFLOP/s = "
             f"frac {ach / a.peak:.4f} of {a.peak:.0f}",
             f"{'kernel':82s} {'n':>3s} {'us':>8s} {'avg_us':>8s}"]
    for k, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"{k:82s} {c:3d} {us:8.1f} {us / c:8.1f}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
