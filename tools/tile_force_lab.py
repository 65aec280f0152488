"""Tile lab (GPU box): the planner's LDS-DMA tile vs forced alternatives
(SSIP_CONV_FORCE) for ResNet-18 batch-256 fwd / dgrad shapes, alternated
HIP-event timing, results compared with the default plan's (bitwise where the
k-order is the same: every fwd / dgrad tile walks the same k-steps).

usage: python tools/tile_force_lab.py [--cfg '256,128,4,2,2;...'] [--shapes l2.3x3,...] [--modes fd]
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
    ap.add_argument("--cfg", default="256,128,4,2,2")
    ap.add_argument("--shapes", default="l2.3x3s2,l2.3x3,l3.3x3s2,l4.3x3s2,l4.3x3")
    ap.add_argument("--modes", default="fd")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    torch.manual_seed(0)
    part = torch.empty(16 << 20, device=dev)
    want = a.shapes.split(",")
    for nm, g in shapes(a.batch):
        if nm not in want:
            continue
        x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
        w = (torch.randn(g.K, g.R, g.S, g.C, device=dev) * 0.05).to(bf)
        wc = w.permute(3, 1, 2, 0).contiguous()
        y = torch.empty(g.N, g.P, g.Q, g.K, device=dev, dtype=bf)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        for m in a.modes:
            if m == "d" and g.stride != 1:
                continue
            mode = "fwd" if m == "f" else "dgrad"
            out = y if m == "f" else dx
            fn = (lambda: ops.conv_fwd(g, x, w, y, part)) if m == "f" else (lambda: ops.conv_dgrad(g, dy, wc, dx))
            os.environ.pop("SSIP_CONV_FORCE", None)
            base_name = ops.conv_kernel_name(mode, g, bf)
            fn()
            torch.cuda.synchronize()
            ref = out.clone()
            line = f"{nm:9s} {mode:5s} default {base_name}"
            res = []
            for c in a.cfg.split(";"):
                os.environ["SSIP_CONV_FORCE"] = f"{m},{c}"
                try:
                    kn = ops.conv_kernel_name(mode, g, bf)
                    out.zero_()
                    fn()
                    torch.cuda.synchronize()
                except RuntimeError as e:
                    res.append((c, None, str(e)[:60]))
                    continue
                same = torch.equal(out.view(torch.int16), ref.view(torch.int16))
                td, tf = [], []
                for _ in range(a.rounds):
                    os.environ.pop("SSIP_CONV_FORCE", None)
                    td.append(time_fn(fn, a.iters))
                    os.environ["SSIP_CONV_FORCE"] = f"{m},{c}"
                    tf.append(time_fn(fn, a.iters))
                res.append((c, (min(td), min(tf), same), kn))
            os.environ.pop("SSIP_CONV_FORCE", None)
            print(line, flush=True)
            for c, r, kn in res:
                if r is None:
                    print(f"    {c}: {kn}", flush=True)
                else:
                    td, tf, same = r
                    print(f"    {c:16s} default {td:7.1f} us  forced {tf:7.1f} us ({(tf / td - 1) * 100:+5.1f} %) "
                          f"{g.flops() / tf / 1e6:5.0f} TF/s  bits {'same' if same else 'differ'}  {kn}", flush=True)


if __name__ == "__main__":
    main()
