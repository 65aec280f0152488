"""Layer-1 halo conv lab (GPU box): the 3x3 / stride-1 / 64-channel forward and
dgrad of ResNet-18 layer 1 (conv_halo_kernel) at batch 256 and 128, timed
with HIP events, per SSIP_HALO_DIAG ablation (timing only, results wrong):
0 full, 16 epilogue not deferred (results right), 4 no input-row DMA after the first
tile, 8 no BN statistics (bits combine).  Speed of light per launch:
max(FLOPs / 2.5 PF, (x + y bytes) / 8 TB/s).

usage: python tools/halo_lab.py [--diags 0,1,2,3,4,8,12] [--iters 20]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--diags", default="0,16,4,8,12")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--stem-diags", default="0", help="SSIP_STEM_DIAG values: 1 no stores, 8 no BN statistics")
    ap.add_argument("--batches", default="256,128")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    part = torch.empty(16 << 20, device=dev)
    for n in [int(b) for b in a.batches.split(",")]:
        g = ops.ConvGeom(n, 56, 56, 64, 64, 3, 3, 1, 1, 64, 3)
        x = torch.randn(n, 56, 56, 64, device=dev).to(bf)
        w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(bf)
        wc = w.permute(3, 1, 2, 0).contiguous()
        y = torch.empty(n, 56, 56, 64, device=dev, dtype=bf)
        dx = torch.empty_like(x)
        sol = max(g.flops() / 2.5e15, 2 * x.numel() * 2 / 8e12) * 1e6
        print(f"batch {n}: {ops.conv_kernel_name('fwd', g, bf)} / {ops.conv_kernel_name('dgrad', g, bf)}; "
              f"SoL {sol:.1f} us", flush=True)
        for dg in a.diags.split(","):
            os.environ["SSIP_HALO_DIAG"] = dg
            tf = time_fn(lambda: ops.conv_fwd(g, x, w, y, part), a.iters)
            td = time_fn(lambda: ops.conv_dgrad(g, y, wc, dx), a.iters)
            print(f"  diag {dg}: fwd {tf:6.1f} us ({sol / tf:.2f} SoL, {g.flops() / tf / 1e6:4.0f} TF/s)"
                  f"  dgrad {td:6.1f} us ({sol / td:.2f} SoL)", flush=True)
        os.environ.pop("SSIP_HALO_DIAG", None)
        # the step's other two dgrad forms: + residual gradient, and the fused
        # BN-backward reduction of the BN+ReLU below (mask from its affine)
        add = torch.randn_like(dx)
        yb = torch.randn_like(dx)
        mean, inv = torch.randn(64, device=dev) * 0.1, torch.rand(64, device=dev) + 0.5
        msc, msh = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.1
        dpart = torch.empty(ops.conv_dgrad_bn_partial_floats(g), device=dev)
        ta = time_fn(lambda: ops.conv_dgrad(g, y, wc, dx, add), a.iters)
        tb = time_fn(lambda: ops.conv_dgrad_bn(g, y, wc, None, None, yb, mean, inv, dx, dpart, mscale=msc,
                                                mshift=msh), a.iters)
        print(f"  dgrad + residual {ta:6.1f} us   dgrad + BN-backward reduce (affine mask) {tb:6.1f} us", flush=True)
        # the stem conv (conv_stem_halo_kernel): pre-padded 230x230x4 image, 7x7/2 -> 112x112x64
        gs = ops.ConvGeom(n, 230, 230, 4, 64, 7, 8, 2, 0, 3, 7)
        xs = torch.randn(n, 230, 230, 4, device=dev).to(bf)
        ws_ = (torch.randn(64, 7, 8, 4, device=dev) * 0.05).to(bf)
        ys = torch.empty(n, 112, 112, 64, device=dev, dtype=bf)
        ssol = max(gs.flops() / 2.5e15, (xs.numel() + ys.numel()) * 2 / 8e12) * 1e6
        for sd in a.stem_diags.split(","):
            os.environ["SSIP_STEM_DIAG"] = sd
            t = time_fn(lambda: ops.conv_fwd(gs, xs, ws_, ys, part), a.iters)
            print(f"  stem {ops.conv_kernel_name('fwd', gs, bf)} diag {sd}: {t:6.1f} us ({ssol / t:.2f} of SoL "
                  f"{ssol:.1f} us)", flush=True)
        os.environ.pop("SSIP_STEM_DIAG", None)
        sc = torch.rand(64, device=dev) + 0.5
        sh = torch.randn(64, device=dev) * 0.1
        pool = torch.empty(n, 56, 56, 64, device=dev, dtype=bf)
        pidx = torch.empty(n, 56, 56, 64, device=dev, dtype=torch.uint8)
        ymx = torch.empty_like(pool)
        tp = time_fn(lambda: ops.stem_bn_pool_fwd(n, 112, 112, 64, 3, 2, 1, ys, sc, sh, pool, pidx, ymx), a.iters)
        print(f"  stem_bn_pool_fwd (unfused pool pass): {tp:6.1f} us", flush=True)
        ta = time_fn(lambda: ops.bn_apply(n * 56 * 56, 64, ymx, sc, sh, None, True, pool), a.iters)
        print(f"  pooled bn_apply: {ta:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
