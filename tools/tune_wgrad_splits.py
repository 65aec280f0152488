"""Time the wgrad (+ its slab reduce) per ResNet-18 shape for several split
targets (SSIP_WGRAD_BLOCKS) on the GPU box."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from ssip import ops  # noqa: E402
from tune_conv import shapes, time_fn  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
ws = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
targets = ["model", 512, 1024, "model2"]  # "model": the planner's own choice (SSIP_WGRAD_BLOCKS unset)
tot = {t: 0.0 for t in targets}
for nm, g in shapes(256):
    x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
    dy = torch.randn(g.N, g.P, g.Q, g.K, device=dev).to(bf)
    dw = torch.empty(g.K, g.C, g.R, g.S, device=dev)
    line = f"{nm:9s}"
    for t in targets:
        if str(t).startswith("model"):
            os.environ.pop("SSIP_WGRAD_BLOCKS", None)
        else:
            os.environ["SSIP_WGRAD_BLOCKS"] = str(t)
        us = time_fn(lambda: ops.conv_wgrad(g, dy, x, dw, False, ws), 20)
        tot[t] += us
        line += f"  {t}:{us:6.1f}"
    print(line, flush=True)
print("total", {t: round(v, 1) for t, v in tot.items()})
