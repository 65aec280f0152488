"""Wgrad tile / ring / grid lab (GPU box): every layer 2-4 wgrad of the
ResNet-18 batch-256 step, for each LDS-DMA configuration given, at the full
grid (budget 0) and at the side stream's one-workgroup-per-CU budget
(ssip_conv_wgrad_budget, what the production step runs).  Times include the
slab reduce; results are checked against the default plan's dW.

usage: python tools/wgrad_lab.py [--cfg 'bm,bn,wm,wn,st;...'] [--budgets 0,256] [--iters 20]
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
    ap.add_argument("--cfg", default="default;128,128,4,2,3;256,128,4,2,2;128,256,2,4,2;256,256,4,2,2;256,256,4,4,2")
    ap.add_argument("--budgets", default="0,256")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="l2.3x3s2,l2.3x3,l3.3x3s2,l3.3x3,l4.3x3s2,l4.3x3")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    ws = torch.empty(768 << 20, dtype=torch.uint8, device=dev)
    want = args.shapes.split(",")
    cfgs = args.cfg.split(";")
    budgets = [int(b) for b in args.budgets.split(",")]
    tot = {}
    for nm, g in shapes(256):
        if nm not in want:
            continue
        x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
        dy = torch.randn(g.N, g.P, g.Q, g.K, device=dev).to(bf)
        ref = torch.empty(g.K, g.C, g.R, g.S, device=dev)
        os.environ.pop("SSIP_CONV_FORCE", None)
        ops.conv_wgrad(g, dy, x, ref, False, ws)
        torch.cuda.synchronize()
        for b in budgets:
            line = f"{nm:9s} b{b:<4d}"
            for c in cfgs:
                if c == "default":
                    os.environ.pop("SSIP_CONV_FORCE", None)
                else:
                    os.environ["SSIP_CONV_FORCE"] = "w," + c
                dw = torch.empty_like(ref)
                try:
                    ops.conv_wgrad(g, dy, x, dw, False, ws, max_workgroups=b)
                    torch.cuda.synchronize()
                except RuntimeError as e:
                    line += f" | {c}: n/a ({str(e)[:40]})"
                    continue
                err = ((dw - ref).abs().max() / ref.abs().max()).item()
                us = time_fn(lambda: ops.conv_wgrad(g, dy, x, dw, False, ws, max_workgroups=b), args.iters)
                tf = g.flops() / us / 1e6
                tot[(b, c)] = tot.get((b, c), 0.0) + us
                line += f" | {c}: {us:6.1f}us {tf:5.0f}TF{' ERR %.1e' % err if err > 1e-3 else ''}"
            print(line, flush=True)
    os.environ.pop("SSIP_CONV_FORCE", None)
    for b in budgets:
        print(f"total b{b}: " + "  ".join(f"{c}={tot.get((b, c), 0):.1f}" for c in cfgs), flush=True)


if __name__ == "__main__":
    main()
