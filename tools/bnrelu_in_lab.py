"""Layer-1 convs with the BN+ReLU below applied in their LDS tile (ABI 13)
vs the plain convs over a materialised input, HIP events, batch 256 (fwd,
wgrad at the full grid and at the side stream's half-CU budget).  Timing only.
usage (GPU box): python tools/bnrelu_in_lab.py [--iters 30]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from ssip import ops  # noqa: E402
from ssip.ops import ConvGeom  # noqa: E402
from tune_conv import time_fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N = a.batch
    g = ConvGeom(N, 56, 56, 64, 64, 3, 3, 1, 1, 64, 3)
    y = torch.randn(N, 56, 56, 64, device=dev).to(torch.bfloat16)
    sc = torch.rand(64, device=dev) + 0.5
    sh = torch.randn(64, device=dev) * 0.2
    x = torch.empty_like(y)
    ops.bn_apply(N * 56 * 56, 64, y, sc, sh, None, True, x)
    w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(torch.bfloat16)
    out = torch.empty_like(y)
    part = torch.empty(ops.conv_fwd_partial_floats(g), device=dev)
    dy = torch.randn_like(y)
    dw = torch.empty(64, 64, 3, 3, device=dev)
    half = torch.cuda.get_device_properties(dev).multi_processor_count // 2
    ws = torch.empty(max(ops.conv_wgrad_workspace_bytes(g, 0), ops.conv_wgrad_workspace_bytes(g, half)), device=dev,
                     dtype=torch.uint8)
    cases = [
        ("fwd plain", lambda: ops.conv_fwd(g, x, w, out, part)),
        ("fwd bnrelu_in", lambda: ops.conv_fwd_bnrelu_in(g, y, sc, sh, w, out, part)),
        ("wgrad plain full", lambda: ops.conv_wgrad(g, dy, x, dw, False, ws)),
        ("wgrad bnrelu_in full", lambda: ops.conv_wgrad_bnrelu_in(g, dy, y, sc, sh, dw, False, ws)),
        (f"wgrad plain budget {half}", lambda: ops.conv_wgrad(g, dy, x, dw, False, ws, max_workgroups=half)),
        (f"wgrad bnrelu_in budget {half}",
         lambda: ops.conv_wgrad_bnrelu_in(g, dy, y, sc, sh, dw, False, ws, max_workgroups=half)),
        ("bn_apply (the pass it replaces)", lambda: ops.bn_apply(N * 56 * 56, 64, y, sc, sh, None, True, x)),
    ]
    for name, fn in cases:
        print(f"{name:34s} {time_fn(fn, a.iters):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
