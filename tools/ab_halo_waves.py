"""A/B of the conv_halo_kernel wave layouts (SSIP_HALO_WAVES = 8: 8 waves of
64x32, 16: 16 waves of 32x32) on layer1 fwd (with BN records) and dgrad
(with the residual add), interleaved in one process.  GPU box."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from ssip import ops  # noqa: E402
from tune_conv import time_fn  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
g = ops.ConvGeom(256, 56, 56, 64, 64, 3, 3, 1, 1, 64, 3)
x = torch.randn(256, 56, 56, 64, device=dev).to(bf)
w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(bf)
y = torch.empty_like(x)
add = torch.randn_like(x)
part = torch.empty(ops.conv_fwd_partial_floats(g), device=dev)
res = {}
for rep in range(3):
    for wv in ("8", "16"):
        os.environ["SSIP_HALO_WAVES"] = wv
        res.setdefault(("f", wv), []).append(time_fn(lambda: ops.conv_fwd(g, x, w, y, part), 20))
        res.setdefault(("d", wv), []).append(time_fn(lambda: ops.conv_dgrad(g, x, w, y, add), 20))
for (m, wv), ts in sorted(res.items()):
    print(f"{m} waves {wv:>2s}: " + " ".join(f"{t:6.1f}" for t in ts) + f"  min {min(ts):6.1f} us", flush=True)
