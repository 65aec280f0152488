"""Split a conv's time into per-k-step and per-tile cost: time the same
output shape with the input channels (so the k-loop) scaled 1x/2x/4x, with
and without the BN-statistics epilogue.  Runs on the GPU box."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from ssip import ops  # noqa: E402
from tune_conv import time_fn  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
part = torch.empty(16 << 20, device=dev)
for (H, K) in [(56, 64), (28, 128), (14, 256), (7, 512)]:
    for C in [K // 2, K, 2 * K, 4 * K]:
        if C < 64:
            continue
        g = ops.ConvGeom(256, H, H, C, K, 3, 3, 1, 1, C, 3)
        x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
        w = (torch.randn(g.K, g.R, g.S, g.C, device=dev) * 0.05).to(bf)
        y = torch.empty(g.N, g.P, g.Q, g.K, device=dev, dtype=bf)
        t1 = time_fn(lambda: ops.conv_fwd(g, x, w, y, part), 10)
        t0 = time_fn(lambda: ops.conv_fwd(g, x, w, y, None), 10)
        ks = 9 * C // 64
        print(f"H={H:3d} K={K:4d} C={C:5d} ksteps={ks:4d}  stats {t1:8.1f}us  nostats {t0:8.1f}us  "
              f"{g.flops() / t1 / 1e6:7.0f} TF/s", flush=True)
