"""Isolated BN forward elementwise passes (ssip_bn_apply without / with the
residual + mask bits, ssip_bn_apply2) on the ResNet-18 batch-256 block
geometries; run under rocprofv3 --kernel-trace for per-kernel durations:

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bna -o run -- python tools/time_bn_apply.py
  python tools/time_bn_apply.py --trace gpurun_out/bna/run_kernel_trace.csv   (host: per-kernel us and TB/s)
"""
import argparse
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))

GEOMS = [("l1", 256 * 56 * 56, 64), ("l2", 256 * 28 * 28, 128), ("l3", 256 * 14 * 14, 256), ("l4", 256 * 7 * 7, 512)]
VARIANTS = [("plain", 2), ("res+bits", 3), ("dual+bits", 3)]  # (name, bf16 tensors moved)
ITERS = 10


def run():
    import torch
    from ssip import ops
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    for nm, M, C in GEOMS:
        y = torch.randn(M, C, device=dev).to(bf)
        r = torch.randn(M, C, device=dev).to(bf)
        z = torch.empty_like(y)
        mb = torch.empty(M * C // 8, device=dev, dtype=torch.uint8)
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
        for _ in range(ITERS):
            ops.bn_apply(M, C, y, sc, sh, None, True, z)
        for _ in range(ITERS):
            ops.bn_apply(M, C, y, sc, sh, r, True, z, mb)
        for _ in range(ITERS):
            ops.bn_apply2(M, C, y, sc, sh, r, sc, sh, True, z, mb)
        torch.cuda.synchronize()


def report(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "bn_apply" in r["Kernel_Name"]]
    i = 0
    for nm, M, C in GEOMS:
        for vn, nt in VARIANTS:
            seg = rows[i:i + ITERS]
            i += ITERS
            us = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in seg)[ITERS // 2]
            nbytes = nt * M * C * 2 + (M * C / 8 if "bits" in vn else 0)
            print(f"{nm} M={M:7d} C={C:3d}  {vn:10s} {us:7.1f} us  {nbytes / us / 1e6:5.2f} TB/s")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", default=None)
    a = ap.parse_args()
    if a.trace:
        report(a.trace)
    else:
        run()
