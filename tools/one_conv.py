"""Run one ResNet-18 conv shape/mode N times (for rocprofv3 PMC passes).
usage: one_conv.py <shape-name> <f|d|w> [iters]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from ssip import ops  # noqa: E402
from tune_conv import shapes  # noqa: E402

name, mode = sys.argv[1], sys.argv[2]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = torch.device("cuda:0")
bf = torch.bfloat16
g = dict(shapes(256))[name]
x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
w = (torch.randn(g.K, g.R, g.S, g.C, device=dev) * 0.05).to(bf)
wc = w.permute(3, 1, 2, 0).contiguous()
y = torch.empty(g.N, g.P, g.Q, g.K, device=dev, dtype=bf)
dy = torch.randn_like(y)
dx = torch.empty_like(x)
dw = torch.empty(g.K, g.C, g.R, g.S, device=dev)
ws = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
part = torch.empty(8 << 20, device=dev)
fn = {"f": lambda: ops.conv_fwd(g, x, w, y, part), "d": lambda: ops.conv_dgrad(g, dy, wc, dx),
      "w": lambda: ops.conv_wgrad(g, dy, x, dw, False, ws)}[mode]
for _ in range(iters):
    fn()
torch.cuda.synchronize()
print("done", name, mode, g.flops() / 1e9, "GFLOP")
