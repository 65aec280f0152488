"""GPU: a downsampling block's conv1 (3x3 / stride 2) and 1x1 / stride-2
downsample forwards in one launch (ssip_conv_fwd_ds: the downsample's tiles
are extra workgroups of the conv's grid running only its tap-(1,1) k-steps)
against the two separate launches (SSIP_NO_FWD_DSFUSE=1): outputs and BN
partial records bit for bit (the same per-element k order, the same M-tiles),
at the ResNet-18 layer2-4 geometries, batch 256 (train) and 128 (weak view),
plus the whole-engine forward with the fusion on and off."""
import os

import pytest
import torch

from ssip import ops
from ssip.ops import ConvGeom

pytestmark = pytest.mark.gpu
DT = torch.bfloat16
BLOCKS = [("l2.0", 64, 56, 128), ("l3.0", 128, 28, 256), ("l4.0", 256, 14, 512)]


@pytest.mark.parametrize("n", [256, 128])
@pytest.mark.parametrize("name,C,H,K", BLOCKS, ids=[b[0] for b in BLOCKS])
def test_fwd_ds_fused_equals_separate(dev, name, C, H, K, n):
    g = ConvGeom(n, H, H, C, K, 3, 3, 2, 1, C, 3)
    gd = ConvGeom(n, H, H, C, K, 1, 1, 2, 0, C, 1)
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(n, H, H, C, generator=gen).to(DT).to(dev)
    w = (torch.randn(K, 3, 3, C, generator=gen) * 0.05).to(DT).to(dev)
    wd = (torch.randn(K, 1, 1, C, generator=gen) * 0.1).to(DT).to(dev)
    out = {}
    for fuse in ("1", "0"):
        if fuse == "0":
            os.environ["SSIP_NO_FWD_DSFUSE"] = "1"
        try:
            y = torch.empty(n, g.P, g.Q, K, device=dev, dtype=DT)
            yd = torch.empty_like(y)
            p = torch.full((ops.conv_fwd_partial_floats(g),), float("nan"), device=dev)
            pd = torch.full((ops.conv_fwd_partial_floats(gd),), float("nan"), device=dev)
            ops.conv_fwd_ds(g, x, w, y, p, gd, wd, yd, pd)
            tiles = (int(ops._lib.lib().ssip_conv_fwd_partial_tiles(g.desc(), 1)),
                     int(ops._lib.lib().ssip_conv_fwd_ds_partial_tiles(g.desc(), gd.desc(), 1)))
            torch.cuda.synchronize()
            out[fuse] = (y, yd, p[: tiles[0] * K * 3], pd[: tiles[1] * K * 3], tiles)
        finally:
            os.environ.pop("SSIP_NO_FWD_DSFUSE", None)
    (y1, yd1, p1, pd1, t1), (y0, yd0, p0, pd0, t0) = out["1"], out["0"]
    assert t1 == t0, (t1, t0)
    assert torch.equal(y1, y0) and torch.equal(yd1, yd0)
    assert torch.equal(p1, p0) and torch.equal(pd1, pd0)
    assert not torch.isnan(pd1).any()


def test_engine_forward_with_and_without_fusion(dev, monkeypatch):
    """The ResNet-18 train forward (batch 32, 224x224, bf16) with the fused
    block forwards equals the unfused engine bit for bit (logits and BN
    running statistics)."""
    from ssip import SSIPResNet, replace_fc
    from ssip import resnet as R

    res = []
    for off in (False, True):
        monkeypatch.setattr(R, "_NO_FWD_DS", off)
        torch.manual_seed(0)
        m = replace_fc(SSIPResNet("resnet18", 1000, dtype="bf16"), 2).to(dev).train()
        x = torch.randn(32, 3, 224, 224, generator=torch.Generator().manual_seed(1)).to(dev)
        with torch.no_grad():
            z = m(x)
        torch.cuda.synchronize()
        res.append((z.cpu(), [b.cpu().clone() for b in m.buffers()]))
    assert torch.equal(res[0][0], res[1][0])
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))
