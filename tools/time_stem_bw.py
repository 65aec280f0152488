"""Time the fused stem backward wgrad (ssip_stem_bwd_wgrad: BN-backward apply
through the max-pool formed per tile in LDS + the stem wgrad) at the bench
geometry, under SSIP_STEM_DIAG ablations (the library reads it once per
process, so each variant is its own process):
  0 = as shipped, 1 = no dy pass, 2 = no MFMAs, 4 = zero-extent loads (no memory traffic)

usage (GPU box):  python tools/time_stem_bw.py [--batch 256]   (spawns one child per variant)
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))


def child(batch, iters):
    import torch
    from ssip import ops
    dev = torch.device("cuda", 0)
    N, H, P, P2 = batch, 230, 112, 56
    g = ops.ConvGeom(N, H, H, 4, 64, 7, 8, 2, 0, 3, 7)
    bf = torch.bfloat16
    torch.manual_seed(0)
    x = torch.randn(N, H, H, 4, device=dev).to(bf)
    y = torch.randn(N, P, P, 64, device=dev).to(bf)
    dp = torch.randn(N, P2, P2, 64, device=dev).to(bf)
    ix = torch.randint(0, 9, (N, P2, P2, 64), device=dev, dtype=torch.uint8)
    sc, sh = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.1
    coef = torch.randn(3 * 64, device=dev)
    dw = torch.zeros(64, 3, 7, 7, device=dev)
    ws = torch.empty(64 << 20, device=dev, dtype=torch.uint8)
    fn = lambda: ops.stem_bwd_wgrad(g, dp, ix, y, x, sc, sh, coef, dw, False, ws)  # noqa: E731
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    flops = 2.0 * N * P * P * 64 * 147
    print(f"SSIP_STEM_DIAG={os.environ.get('SSIP_STEM_DIAG', '0')}: {us:7.1f} us  {flops / us / 1e6:6.1f} TF/s  "
          f"dw sum {dw.double().sum().item():.10e} abs {dw.double().abs().sum().item():.10e}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--diags", default="0,8,1,2,3")
    args = ap.parse_args()
    if args.child:
        return child(args.batch, args.iters)
    for d in args.diags.split(","):
        env = dict(os.environ, SSIP_STEM_DIAG=d)
        r = subprocess.run([sys.executable, __file__, "--child", "--batch", str(args.batch), "--iters",
                            str(args.iters)], env=env, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
