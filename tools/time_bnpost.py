"""Isolated timing: dgrad vs dgrad fused with the BN-backward reduction vs the
separate bn_bwd passes, on ResNet-18 shapes (GPU box)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from ssip import ops  # noqa: E402
from tune_conv import shapes, time_fn  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
for nm, g in shapes(256):
    if g.stride != 1:
        continue
    dy = torch.randn(g.N, g.P, g.Q, g.K, device=dev).to(bf)
    wc = (torch.randn(g.C, g.R, g.S, g.K, device=dev) * 0.05).to(bf)
    dx = torch.empty(g.N, g.H, g.W, g.C, device=dev, dtype=bf)
    z = torch.relu(torch.randn_like(dx))
    y = torch.randn_like(dx)
    add = torch.randn_like(dx)
    mean = torch.zeros(g.C, device=dev)
    invstd = torch.ones(g.C, device=dev)
    part = torch.empty(ops.conv_dgrad_bn_partial_floats(g), device=dev)
    M = g.N * g.H * g.W
    bpart = torch.empty(ops.bn_bwd_partial_floats(M, g.C), device=dev)
    coef = torch.empty(3 * g.C, device=dev)
    dyo = torch.empty_like(dx)
    t_d = time_fn(lambda: ops.conv_dgrad(g, dy, wc, dx), 20)
    t_da = time_fn(lambda: ops.conv_dgrad(g, dy, wc, dx, add), 20)
    t_f = time_fn(lambda: ops.conv_dgrad_bn(g, dy, wc, None, z, y, mean, invstd, dx, part), 20)
    t_fa = time_fn(lambda: ops.conv_dgrad_bn(g, dy, wc, add, z, y, mean, invstd, dx, part), 20)
    t_bn = time_fn(lambda: ops.bn_bwd(M, g.C, dx, z, y, mean, invstd, None, None, None, False, dyo, None, bpart,
                                      coef), 20)
    t_bnp = time_fn(lambda: ops.bn_bwd_from_partials(M, g.C, ops.conv_dgrad_bn_partial_tiles(g, bf), part, dx, y,
                                                     mean, invstd, None, None, None, False, dyo, coef), 20)
    print(f"{nm:9s} dgrad {t_d:6.1f} +add {t_da:6.1f} | fused {t_f:6.1f} +add {t_fa:6.1f} | "
          f"bn_bwd(full) {t_bn:6.1f} from_partials {t_bnp:6.1f} | separate {t_d + t_bn:6.1f} fused {t_f + t_bnp:6.1f}",
          flush=True)
