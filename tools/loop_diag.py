"""k-loop ablations of conv_glds_kernel (timing only; results are wrong).

For each SSIP_LOOP_DIAG value (a separate process each: the library reads the
variable once) time the 2-stage 128x128 (8 waves, 4x2) and 256x256 kernels on
the ResNet-18 batch-256 3x3 shapes:
  0 full loop, 1 no MFMAs, 2 no fragment reads, 4 no LDS-DMA issue,
  8 no barrier (plus sums of those bits).
usage (GPU box): python tools/loop_diag.py [--diags 0,1,2,4,8] [--iters 20]
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [("l2.3x3", "f", "128,128,4,2,2"), ("l2.3x3", "d", "128,128,4,2,2"), ("l3.3x3", "f", "256,256,4,2,2"),
         ("l3.3x3", "f", "128,128,4,2,2"), ("l3.3x3", "d", "128,128,4,2,2"), ("l4.3x3", "f", "128,128,4,2,2"),
         ("l2.3x3", "w", "128,128,4,2,2"), ("l3.3x3", "w", "128,128,4,2,2")]


def child(iters):
    sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import torch
    from ssip import ops
    from tune_conv import shapes, time_fn
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    ws = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    part = torch.empty(8 << 20, dtype=torch.float32, device=dev)
    shp = dict(shapes(256))
    for nm, mode, cfg in CASES:
        g = shp[nm]
        x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
        w = (torch.randn(g.K, g.R, g.S, g.C, device=dev) * 0.05).to(bf)
        wc = w.permute(3, 1, 2, 0).contiguous()
        y = torch.empty(g.N, g.P, g.Q, g.K, device=dev, dtype=bf)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.empty(g.K, g.C, g.R, g.S, device=dev, dtype=torch.float32)
        fn = {"f": lambda: ops.conv_fwd(g, x, w, y, part), "d": lambda: ops.conv_dgrad(g, dy, wc, dx),
              "w": lambda: ops.conv_wgrad(g, dy, x, dw, False, ws)}[mode]
        os.environ["SSIP_CONV_FORCE"] = mode + "," + cfg
        try:
            t = time_fn(fn, iters)
            print(f"{os.environ.get('SSIP_LOOP_DIAG', '0'):>3s} {nm:8s} {mode} {cfg:14s} {t:8.1f} us "
                  f"{g.flops() / t / 1e6:6.0f} TF/s", flush=True)
        except RuntimeError as e:
            print(f"{nm} {mode} {cfg}: {str(e)[:80]}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--diags", default="0,1,2,4,8,3,5,6,12")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a.iters)
        return
    for d in a.diags.split(","):
        env = dict(os.environ, SSIP_LOOP_DIAG=d)
        r = subprocess.run([sys.executable, __file__, "--child", "--iters", str(a.iters)], env=env, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
