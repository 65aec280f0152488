"""Stem BN -> ReLU -> max-pool forward: the generic kernel (rows 0) vs the
k3s2 kernel at several pooled-rows-per-workgroup values, HIP events, batch
256 with ymax (train forward) and 128 without (weak forward).  Timing only.
usage (GPU box): python tools/pool_lab.py [--rows 0,4,2,8] [--iters 30]"""
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
    ap.add_argument("--rows", default="0,4,2,8")
    ap.add_argument("--lds", default="0", help="SSIP_POOL_LDS values (ymax from the thread's LDS slots)")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for N, with_ymax in ((256, True), (128, False)):
        H = W = 112
        y = torch.randn(N, H, W, 64, device=dev).to(torch.bfloat16)
        scale = torch.rand(64, device=dev) + 0.5
        shift = torch.randn(64, device=dev) * 0.2
        pool = torch.empty(N, 56, 56, 64, device=dev, dtype=torch.bfloat16)
        idx = torch.empty(N, 56, 56, 64, device=dev, dtype=torch.uint8)
        ymax = torch.empty_like(pool) if with_ymax else None
        nbytes = y.numel() * 2 + pool.numel() * (2 + 1 + (2 if with_ymax else 0))
        for lds in a.lds.split(","):
            os.environ["SSIP_POOL_LDS"] = lds
            for r in a.rows.split(","):
                os.environ["SSIP_POOL_ROWS"] = r
                t = time_fn(lambda: ops.stem_bn_pool_fwd(N, H, W, 64, 3, 2, 1, y, scale, shift, pool, idx, ymax),
                            a.iters)
                print(f"N={N:3d} ymax={int(with_ymax)} lds={lds} rows={r:>2s} {t:7.1f} us "
                      f"{nbytes / t / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
