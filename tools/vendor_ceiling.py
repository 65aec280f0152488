"""Calibrate the conv kernels against the vendor libraries on the same shapes.

For each ResNet-18 batch-256 3x3 shape, time (HIP events, random bf16 data):
  gemm  : the same M x N x K as a PLAIN bf16 GEMM (torch.matmul -> hipBLASLt),
          i.e. no im2col, the best case a library reaches for that volume;
  miopen: torch conv2d, channels_last bf16 (MIOpen), forward;
  ssip  : our forward (planner's choice).
Measurement only: nothing here is on the product path.
usage (GPU box): python tools/vendor_ceiling.py [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from ssip import ops  # noqa: E402
from tune_conv import shapes, time_fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    part = torch.empty(8 << 20, dtype=torch.float32, device=dev)
    torch.backends.cudnn.benchmark = True
    print(f"{'shape':9s} {'M':>8s} {'N':>5s} {'K':>5s} {'gemm':>16s} {'miopen':>16s} {'ssip':>16s}", flush=True)
    for nm, g in shapes(a.batch):
        if g.R != 3:
            continue
        M, N, K = g.N * g.P * g.Q, g.K, g.R * g.S * g.C
        fl = 2.0 * M * N * K
        A = torch.randn(M, K, device=dev).to(bf)
        B = torch.randn(K, N, device=dev).to(bf)
        C = torch.empty(M, N, device=dev, dtype=bf)
        t_g = time_fn(lambda: torch.matmul(A, B, out=C), a.iters)
        del A, B, C
        x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
        w = (torch.randn(g.K, g.R, g.S, g.C, device=dev) * 0.05).to(bf)
        xc = x.permute(0, 3, 1, 2)  # NCHW view of NHWC memory = channels_last
        wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        try:
            t_m = time_fn(lambda: F.conv2d(xc, wc, stride=g.stride, padding=g.pad), a.iters)
        except RuntimeError as e:  # MIOpen may lack a bf16 solver for a shape
            print(f"  miopen {nm}: {str(e)[:80]}", flush=True)
            t_m = float("nan")
        y = torch.empty(g.N, g.P, g.Q, g.K, device=dev, dtype=bf)
        t_s = time_fn(lambda: ops.conv_fwd(g, x, w, y, part), a.iters)
        cell = lambda t: f"{t:7.1f}us {fl / t / 1e6:5.0f}TF"
        print(f"{nm:9s} {M:8d} {N:5d} {K:5d} {cell(t_g):>16s} {cell(t_m):>16s} {cell(t_s):>16s}", flush=True)
        del x, w, y
    # a large square GEMM for the library's own best rate on this box
    for n in (4096, 8192):
        A = torch.randn(n, n, device=dev).to(bf)
        B = torch.randn(n, n, device=dev).to(bf)
        C = torch.empty(n, n, device=dev, dtype=bf)
        t = time_fn(lambda: torch.matmul(A, B, out=C), a.iters)
        print(f"square {n}: {t:8.1f} us {2.0 * n ** 3 / t / 1e6:6.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
