"""CPU: the library's kernel choice for a conv geometry and the BatchNorm
record sizing derived from it agree on every call (host planning only, no
device).  A persistent forward kernel (halo) writes one record per
(channel, workgroup, wave row): G * 8 per channel; the partial buffer the
engine allocates (ssip_conv_fwd_partial_floats) must hold every record the
launched kernel writes, on the first call and on repeated (cached) calls.
Regression: a persistent kernel's plan cache once answered a repeated call
differently from the first one (layer-4 shapes), and the forward overran its
records (that kernel, conv_hb, is now on the r3-variants branch only)."""
import re

import pytest
import torch

from ssip import ops
from ssip.ops import ConvGeom

DT = torch.bfloat16

# ResNet-18 (224^2) and ResNet-50 (512^2) 3x3 / stride-1 and stride-2 convs, batch 128 / 256 / odd
SHAPES = [(C, H, K, st) for (C, H, K) in [(64, 56, 64), (128, 28, 128), (256, 14, 256), (512, 7, 512),
                                          (128, 64, 128), (256, 32, 256), (512, 16, 512), (64, 128, 64)]
          for st in (1,)] + [(64, 56, 128, 2), (128, 28, 256, 2), (256, 14, 512, 2)]


@pytest.mark.parametrize("n", [256, 128, 5])
@pytest.mark.parametrize("C,H,K,st", SHAPES)
def test_fwd_records_fit(n, C, H, K, st):
    g = ConvGeom(n, H, H, C, K, 3, 3, st, 1, C, 3)
    names = {ops._lib.lib() and ops.conv_kernel_name("fwd", g, DT) for _ in range(3)}
    assert len(names) == 1, names
    name = names.pop()
    tiles = {int(ops._lib.lib().ssip_conv_fwd_partial_tiles(g.desc(), ops._DT[DT])) for _ in range(3)}
    assert len(tiles) == 1
    t = tiles.pop()
    m = re.search(r"G=(\d+)", name)
    if name.startswith("halo<"):
        assert m and t == int(m.group(1)) * 8, (name, t)
    floats = int(ops._lib.lib().ssip_conv_fwd_partial_floats(g.desc()))
    assert floats >= t * K * 3, (name, t, floats)


@pytest.mark.parametrize("C,H,K,st", SHAPES)
def test_dgrad_choice_stable(C, H, K, st):
    g = ConvGeom(256, H, H, C, K, 3, 3, st, 1, C, 3)
    names = {ops.conv_kernel_name("dgrad", g, DT) for _ in range(3)}
    assert len(names) == 1, names
