"""Stagger lab (GPU box): every ResNet-18 batch-256 conv the LDS-DMA ring
kernel runs (fwd, stride-1 dgrad, fused stride-2 dgrad + downsample, wgrad at
the full grid and at the side stream's 256-workgroup budget), with
SSIP_STAGGER off and on: outputs must be the same bits, times alternate
A/B/A/B over HIP events.  Timing + bitwise check only.

usage: python tools/stagger_lab.py [--on 7] [--rounds 4] [--iters 20] [--shapes l2.3x3,...]
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
    ap.add_argument("--on", default="7", help="SSIP_STAGGER value for the B side")
    ap.add_argument("--off", default="0", help="SSIP_STAGGER value for the A side")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--shapes", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    torch.manual_seed(0)
    part = torch.empty(16 << 20, device=dev)
    wsp = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    want = set(args.shapes.split(",")) if args.shapes else None
    geo = dict(shapes(args.batch))
    cases = []
    for nm, g in shapes(args.batch):
        if nm == "l1.3x3" or (want and nm not in want):
            continue  # layer 1 runs the halo kernels
        x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
        w = (torch.randn(g.K, g.R, g.S, g.C, device=dev) * 0.05).to(bf)
        wc = w.permute(3, 1, 2, 0).contiguous()
        y = torch.empty(g.N, g.P, g.Q, g.K, device=dev, dtype=bf)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.empty(g.K, g.C, g.R, g.S, device=dev)
        if not nm.endswith(".ds"):
            cases.append((nm, "fwd", 0, g.flops(), y, lambda g=g, x=x, w=w, y=y: ops.conv_fwd(g, x, w, y, part)))
        if g.stride == 1:
            cases.append((nm, "dgrad", 0, g.flops(), dx,
                          lambda g=g, dy=dy, wc=wc, dx=dx: ops.conv_dgrad(g, dy, wc, dx)))
        elif g.R == 3:
            gds = geo[nm.split(".")[0] + ".ds"]
            wds = (torch.randn(gds.C, gds.K, device=dev) * 0.05).to(bf)
            dyds = torch.randn_like(y)
            cases.append((nm, "dgrad+ds", 0, g.flops() + gds.flops(), dx,
                          lambda g=g, gds=gds, dy=dy, wc=wc, dyds=dyds, wds=wds, dx=dx:
                          ops.conv_dgrad_ds(g, dy, wc, gds, dyds, wds, dx)))
        for b in (0, 256):
            cases.append((nm, "wgrad", b, g.flops(), dw,
                          lambda g=g, dy=dy, x=x, dw=dw, b=b: ops.conv_wgrad(g, dy, x, dw, False, wsp, b)))
    tot = {"A": 0.0, "B": 0.0}
    for nm, mode, b, fl, out, fn in cases:
        res = {}
        for side, val in (("A", args.off), ("B", args.on)):
            os.environ["SSIP_STAGGER"] = val
            out.zero_()
            fn()
            torch.cuda.synchronize()
            res[side] = out.clone()
        same = torch.equal(res["A"].view(torch.int16) if res["A"].dtype == bf else res["A"].view(torch.int32),
                           res["B"].view(torch.int16) if res["B"].dtype == bf else res["B"].view(torch.int32))
        ts = {"A": [], "B": []}
        for _ in range(args.rounds):
            for side, val in (("A", args.off), ("B", args.on)):
                os.environ["SSIP_STAGGER"] = val
                ts[side].append(time_fn(fn, args.iters))
        ta, tb = min(ts["A"]), min(ts["B"])
        tot["A"] += ta
        tot["B"] += tb
        os.environ["SSIP_STAGGER"] = args.on
        kn = ops.conv_kernel_name("wgrad" if mode == "wgrad" else ("dgrad" if "dgrad" in mode else "fwd"),
                                  geo[nm], bf, b)
        print(f"{nm:9s} {mode:8s} b{b:<4d} off {ta:7.1f} us  on {tb:7.1f} us  ({(tb / ta - 1) * 100:+5.1f} %)  "
              f"{fl / tb / 1e6:5.0f} TF/s  bits {'same' if same else 'DIFFER'}  {kn}", flush=True)
        if not same:
            print("BITWISE MISMATCH", nm, mode, b, flush=True)
            sys.exit(1)
    print(f"sum off {tot['A']:.1f} us  on {tot['B']:.1f} us  ({(tot['B'] / tot['A'] - 1) * 100:+.1f} %)", flush=True)


if __name__ == "__main__":
    main()
