"""Isolated BN-backward passes (reduce / finalize / apply of ssip_bn_bwd with
mask bits, as the train step's block-output BNs) on the ResNet-18 batch-256
geometries; run under rocprofv3 --kernel-trace to get per-kernel durations:

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bnb -o run -- python tools/time_bn_bwd.py
  python tools/time_bn_bwd.py --trace gpurun_out/bnb/run_kernel_trace.csv   (host: per-kernel us and GB/s)
"""
import argparse
import collections
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))

GEOMS = [("l1", 256 * 56 * 56, 64), ("l2", 256 * 28 * 28, 128), ("l3", 256 * 14 * 14, 256), ("l4", 256 * 7 * 7, 512)]
ITERS = 10


def run():
    import torch
    from ssip import ops
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    for nm, M, C in GEOMS:
        dz = torch.randn(M, C, device=dev).to(bf)
        y = torch.randn(M, C, device=dev).to(bf)
        mb = torch.randint(0, 256, (M * C // 8,), device=dev, dtype=torch.uint8)
        mean, invstd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        gamma = torch.ones(C, device=dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        part = torch.empty(ops.bn_bwd_partial_floats(M, C), device=dev)
        coef = torch.empty(3 * C, device=dev)
        dy = torch.empty_like(dz)
        for _ in range(ITERS):
            ops.bn_bwd(M, C, dz, None, y, mean, invstd, gamma, dg, db, False, dy, None, part, coef, mbits=mb)
        torch.cuda.synchronize()


def report(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "bn_bwd" in r["Kernel_Name"]]
    per = 3 * ITERS
    for gi, (nm, M, C) in enumerate(GEOMS):
        seg = rows[gi * per:(gi + 1) * per]
        by = collections.defaultdict(list)
        for r in seg:
            k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("_ZN12_GLOBAL__N_1", "")
            by[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        t = M * C * 2
        for k, v in by.items():
            us = sorted(v)[len(v) // 2]
            nbytes = 2 * t + M * C / 8 if "reduce" in k else (3 * t + M * C / 8 if "apply" in k else 0)
            bw = f"{nbytes / us / 1e6:6.2f} TB/s" if nbytes else ""
            print(f"{nm} M={M:7d} C={C:3d}  {k[:40]:40s} {us:7.1f} us  {bw}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", default=None)
    a = ap.parse_args()
    if a.trace:
        report(a.trace)
    else:
        run()
