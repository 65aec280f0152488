"""GPU: the batched compute-dtype weight refresh (ssip_weight_prep_batch, the
64 x 64 tap-slice kernel) equals the one-item elementwise conversion
(ssip_weight_prep) bit for bit, for ResNet-18 / ResNet-50 conv
shapes including the 7x7 stem's channel / tap padding, with and without the
per-output-channel factor of a folded eval BatchNorm."""
import pytest
import torch

from ssip import ops

pytestmark = pytest.mark.gpu

DT = torch.bfloat16

# (K, C, R, S, Cp, Sp)
SHAPES = [(64, 3, 7, 7, 4, 8), (64, 64, 3, 3, 64, 3), (128, 64, 3, 3, 64, 3), (128, 64, 1, 1, 64, 1),
          (256, 128, 3, 3, 128, 3), (512, 512, 3, 3, 512, 3), (2048, 512, 1, 1, 512, 1), (100, 70, 3, 3, 70, 3)]


@pytest.mark.parametrize("scaled", [False, True, "negative"])
def test_weight_prep_batch_matches_single(dev, scaled):
    """"negative": scales of both signs (a folded BN with gamma < 0) -- the
    channel / tap padding must stay +0.0, as the elementwise kernel stores it."""
    g = torch.Generator().manual_seed(7)
    items, want = [], []
    for (K, C, R, S, Cp, Sp) in SHAPES:
        w = torch.randn(K, C, R, S, generator=g).to(dev)
        ks = (torch.rand(K, generator=g) + 0.5).to(dev) if scaled else None
        if scaled == "negative":
            ks = ks * torch.where(torch.arange(K, device=dev) % 2 == 0, -1.0, 1.0)
        krsc = torch.full((K, R, Sp, Cp), float("nan"), device=dev, dtype=DT)
        crsk = torch.full((Cp, R, Sp, K), float("nan"), device=dev, dtype=DT)
        items.append((w, Cp, Sp, krsc, crsk, ks))
        # reference: the elementwise one-item kernel on the (scaled) fp32 weight
        ref_w = w * ks.view(K, 1, 1, 1) if scaled else w
        rk = torch.empty_like(krsc)
        rc = torch.empty_like(crsk)
        ops.weight_prep(ref_w.contiguous(), DT, Cp, Sp, rk, rc)
        want.append((rk, rc))
    ops.weight_prep_batch(items, DT)
    torch.cuda.synchronize()
    for (w, Cp, Sp, krsc, crsk, ks), (rk, rc), shp in zip(items, want, SHAPES):
        assert torch.equal(krsc.view(torch.int16), rk.view(torch.int16)), shp
        assert torch.equal(crsk.view(torch.int16), rc.view(torch.int16)), shp


def test_weight_prep_batch_krsc_only(dev):
    """Items without a CRSK output (need_t=False, eval folding)."""
    g = torch.Generator().manual_seed(8)
    w = torch.randn(128, 64, 3, 3, generator=g).to(dev)
    krsc = torch.empty((128, 3, 3, 64), device=dev, dtype=DT)
    ops.weight_prep_batch([(w, 64, 3, krsc, None)], DT)
    rk = torch.empty_like(krsc)
    ops.weight_prep(w, DT, 64, 3, rk, None)
    torch.cuda.synchronize()
    assert torch.equal(krsc.view(torch.int16), rk.view(torch.int16))
