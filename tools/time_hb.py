"""A/B of the row-balanced halo kernel (SSIP_HB=1) against the default
planner on the ResNet-18 3x3 stride-1 convs, interleaved in one process.
usage (GPU box): python tools/time_hb.py [--iters 20] [--rounds 3]"""
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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="l2.3x3,l3.3x3,l4.3x3")
    ap.add_argument("--dbg", default="", help="comma-separated SSIP_HB_DBG values timed as extra hb variants")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    part = torch.empty(8 << 20, dtype=torch.float32, device=dev)
    for batch in (256, 128):
        shp = dict(shapes(batch))
        for nm in a.shapes.split(","):
            g = shp[nm]
            x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
            w = (torch.randn(g.K, g.R, g.S, g.C, device=dev) * 0.05).to(bf)
            wc = w.permute(3, 1, 2, 0).contiguous()
            y = torch.empty(g.N, g.P, g.Q, g.K, device=dev, dtype=bf)
            dy = torch.randn_like(y)
            dx = torch.empty_like(x)
            for mode, fn in (("f", lambda: ops.conv_fwd(g, x, w, y, part)), ("d", lambda: ops.conv_dgrad(g, dy, wc, dx))):
                if batch == 128 and mode == "d":
                    continue
                variants = ["0", "1"] + ["1d" + d for d in a.dbg.split(",") if d]
                res = {v: [] for v in variants}
                names = {}
                for _ in range(a.rounds):
                    for v in variants:
                        os.environ["SSIP_HB"] = v[0]
                        os.environ["SSIP_HB_DBG"] = v[2:] if len(v) > 1 else "0"
                        names[v] = ops.conv_kernel_name("fwd" if mode == "f" else "dgrad", g, bf)
                        res[v].append(time_fn(fn, a.iters))
                os.environ["SSIP_HB_DBG"] = "0"
                t0, t1 = sorted(res["0"])[a.rounds // 2], sorted(res["1"])[a.rounds // 2]
                print(f"bs{batch} {nm:7s} {mode}  default {t0:7.1f} us ({g.flops() / t0 / 1e6:5.0f} TF/s) {names['0']:28s}"
                      f"  hb {t1:7.1f} us ({g.flops() / t1 / 1e6:5.0f} TF/s) {names['1']}" +
                      "".join(f"  dbg{v[2:]} {sorted(res[v])[a.rounds // 2]:7.1f}" for v in variants[2:]), flush=True)


if __name__ == "__main__":
    main()
