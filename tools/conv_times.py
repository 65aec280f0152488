"""Per-launch times of the planner's choice for every ResNet-18 conv shape and
pass (fwd / dgrad / wgrad) at one batch, HIP events, random bf16 data; for
A/B of two builds on one box (run it once per SSIP_LIB).  Timing only.
usage (GPU box): python tools/conv_times.py [--batch 256] [--iters 20] [--modes fdw]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from ssip import ops  # noqa: E402
from tune_conv import shapes, time_fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--modes", default="fdw")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    part = torch.empty(16 << 20, device=dev)
    wsp = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    total = 0.0
    for name, g in shapes(a.batch):
        x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
        w = (torch.randn(g.K, g.R, g.S, g.C, device=dev) * 0.05).to(bf)
        wc = w.permute(3, 1, 2, 0).contiguous()
        y = torch.empty(g.N, g.P, g.Q, g.K, device=dev, dtype=bf)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.empty(g.K, g.C, g.R, g.S, device=dev)
        fns = {"f": ("fwd", lambda: ops.conv_fwd(g, x, w, y, part)),
               "d": ("dgrad", lambda: ops.conv_dgrad(g, dy, wc, dx)),
               "w": ("wgrad", lambda: ops.conv_wgrad(g, dy, x, dw, False, wsp))}
        for m in a.modes:
            mode, fn = fns[m]
            if m == "d" and g.stride != 1:
                continue  # stride-2 dgrads run fused with the downsample in the step
            t = time_fn(fn, a.iters)
            total += t
            print(f"{name:10s} {mode:5s} {t:7.1f} us {g.flops() / t / 1e6:6.0f} TF/s  {ops.conv_kernel_name(mode, g, bf)}",
                  flush=True)
    print(f"sum {total:.1f} us", flush=True)


if __name__ == "__main__":
    main()
