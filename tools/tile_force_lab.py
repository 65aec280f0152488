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
    ap.add_argument("--r50", action="store_true", help="ResNet-50 1x1 shapes at 512^2 (BASELINE config 5)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    torch.manual_seed(0)
    part = torch.empty(16 << 20, device=dev)
    want = a.shapes.split(",")
    if a.r50:
        # name, H, C, K (1x1, stride 1) at 512^2: layer1 128^2, layer2 64^2, layer3 32^2, layer4 16^2
        r50 = [("l1.conv1a", 128, 64, 64), ("l1.conv1", 128, 256, 64), ("l1.conv3", 128, 64, 256),
               ("l2.conv1", 64, 512, 128), ("l2.conv3", 64, 128, 512), ("l3.conv1", 32, 1024, 256),
               ("l3.conv3", 32, 256, 1024), ("l4.conv1", 16, 2048, 512), ("l4.conv3", 16, 512, 2048)]
        shape_list = [(nm, ops.ConvGeom(a.batch, H, H, C, K, 1, 1, 1, 0, C, 1)) for nm, H, C, K in r50]
        want = [nm for nm, _ in shape_list]
    else:
        shape_list = shapes(a.batch)
    for nm, g in shape_list:
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
