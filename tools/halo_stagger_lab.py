"""Layer-1 halo conv stagger lab (GPU box): every conv_halo_kernel form the
ResNet-18 step runs (forward with BN records, forward with bn1's BN+ReLU
formed in LDS, dgrad, dgrad + residual, dgrad + BN-backward reduction) at
batch 256 and 128, with SSIP_HALO_STAGGER off and on: outputs and BN records
must be the same bits; times alternate A/B over HIP events.

usage: python tools/halo_stagger_lab.py [--on 1] [--rounds 3] [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from ssip import ops  # noqa: E402
from tune_conv import time_fn  # noqa: E402

ENV = "SSIP_HALO_STAGGER"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--on", default="1")
    ap.add_argument("--off", default="0")
    ap.add_argument("--env", default=ENV)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batches", default="256,128")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    torch.manual_seed(0)
    tot = {"A": 0.0, "B": 0.0}
    for n in [int(b) for b in a.batches.split(",")]:
        g = ops.ConvGeom(n, 56, 56, 64, 64, 3, 3, 1, 1, 64, 3)
        x = torch.randn(n, 56, 56, 64, device=dev).to(bf)
        w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(bf)
        wc = w.permute(3, 1, 2, 0).contiguous()
        y = torch.empty(n, 56, 56, 64, device=dev, dtype=bf)
        dx = torch.empty_like(x)
        part = torch.zeros(ops.conv_fwd_partial_floats(g), device=dev)
        dpart = torch.zeros(ops.conv_dgrad_bn_partial_floats(g), device=dev)
        add = torch.randn_like(dx)
        yb = torch.randn_like(dx)
        sc, sh = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.3
        mean, inv = torch.randn(64, device=dev) * 0.1, torch.rand(64, device=dev) + 0.5
        cases = [
            ("fwd", (y, part), lambda: ops.conv_fwd(g, x, w, y, part)),
            ("fwd_bnrelu_in", (y, part), lambda: ops.conv_fwd_bnrelu_in(g, x, sc, sh, w, y, part)),
            ("dgrad", (dx,), lambda: ops.conv_dgrad(g, y, wc, dx)),
            ("dgrad+add", (dx,), lambda: ops.conv_dgrad(g, y, wc, dx, add)),
            ("dgrad_bn", (dx, dpart), lambda: ops.conv_dgrad_bn(g, y, wc, None, None, yb, mean, inv, dx, dpart,
                                                                 mscale=sc, mshift=sh)),
        ]
        print(f"batch {n}: {ops.conv_kernel_name('fwd', g, bf)} / {ops.conv_kernel_name('dgrad', g, bf)}",
              flush=True)
        for name, outs, fn in cases:
            res = {}
            for side, val in (("A", a.off), ("B", a.on)):
                os.environ[a.env] = val
                for o in outs:
                    o.zero_()
                fn()
                torch.cuda.synchronize()
                res[side] = [o.clone() for o in outs]
            same = all(torch.equal(p.view(torch.int16) if p.dtype == bf else p.view(torch.int32),
                                   q.view(torch.int16) if q.dtype == bf else q.view(torch.int32))
                       for p, q in zip(res["A"], res["B"]))
            ts = {"A": [], "B": []}
            for _ in range(a.rounds):
                for side, val in (("A", a.off), ("B", a.on)):
                    os.environ[a.env] = val
                    ts[side].append(time_fn(fn, a.iters))
            ta, tb = min(ts["A"]), min(ts["B"])
            tot["A"] += ta
            tot["B"] += tb
            print(f"  {name:14s} off {ta:7.1f} us  on {tb:7.1f} us  ({(tb / ta - 1) * 100:+5.1f} %)  "
                  f"bits {'same' if same else 'DIFFER'}", flush=True)
            if not same:
                print("BITWISE MISMATCH", n, name, flush=True)
                sys.exit(1)
    os.environ.pop(a.env, None)
    print(f"sum off {tot['A']:.1f} us  on {tot['B']:.1f} us  ({(tot['B'] / tot['A'] - 1) * 100:+.1f} %)", flush=True)


if __name__ == "__main__":
    main()
