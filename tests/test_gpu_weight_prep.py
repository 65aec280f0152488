"""Batched compute-dtype weight preparation (ssip_weight_prep_batch): the
whole-tap tile kernel against a host restatement of the two layouts, bit for
bit, on every ResNet-18 conv shape (3x3 over 64-512 channels, the 1x1/2
downsamples, the 7x7 stem padded to C 4 / S 8), with and without the folded
eval-BN scale, both dtypes, in one launch as the train step issues it.

Layouts (include/ssip.h ssip_wprep): w_krsc[K][R][Sp][Cp], w_crsk[Cp][R][Sp][K]
from the fp32 torchvision KCRS master (src/training/common.py:299-304's
resnet18 conv weights), zero in the padded channels / columns; with kscale the
value is fp32(w * kscale[k]) before the dtype conversion.
"""
import pytest
import torch

from ssip import ops

pytestmark = pytest.mark.gpu

# (K, C, R, S, Cp, Sp): every distinct ResNet-18 conv, plus a K that is not a
# multiple of 64 and a 1x1 with C > 64
SHAPES = [(64, 3, 7, 7, 4, 8), (64, 64, 3, 3, 64, 3), (128, 64, 3, 3, 64, 3), (128, 128, 3, 3, 128, 3),
          (128, 64, 1, 1, 64, 1), (256, 128, 3, 3, 128, 3), (256, 256, 3, 3, 256, 3), (256, 128, 1, 1, 128, 1),
          (512, 256, 3, 3, 256, 3), (512, 512, 3, 3, 512, 3), (512, 256, 1, 1, 256, 1), (96, 192, 1, 1, 192, 1)]


def _host(w, Cp, Sp, ksc, dt):
    K, C, R, S = w.shape
    v = w * ksc.view(K, 1, 1, 1) if ksc is not None else w
    full = torch.zeros(K, Cp, R, Sp)
    full[:, :C, :, :S] = v
    full = full.to(dt)
    return full.permute(0, 2, 3, 1).contiguous(), full.permute(1, 2, 3, 0).contiguous()


@pytest.mark.parametrize("dtname", ["bf16", "f32"])
@pytest.mark.parametrize("fold", [False, True])
def test_weight_prep_batch_exact(dev, dtname, fold):
    dt = torch.bfloat16 if dtname == "bf16" else torch.float32
    gen = torch.Generator().manual_seed(5)
    items, want = [], []
    for K, C, R, S, Cp, Sp in SHAPES:
        w = torch.randn(K, C, R, S, generator=gen)
        ksc = (torch.rand(K, generator=gen) + 0.5) if fold else None
        krsc = torch.full((K, R, Sp, Cp), float("nan"), device=dev, dtype=dt)
        crsk = torch.full((Cp, R, Sp, K), float("nan"), device=dev, dtype=dt)
        items.append((w.to(dev), Cp, Sp, krsc, crsk, ksc.to(dev) if ksc is not None else None))
        want.append(_host(w, Cp, Sp, ksc, dt))
    ops.weight_prep_batch(items, dt)
    torch.cuda.synchronize()
    for (K, C, R, S, Cp, Sp), it, (hk, hc) in zip(SHAPES, items, want):
        assert torch.equal(it[3].cpu(), hk), (K, C, R, S, "krsc")
        assert torch.equal(it[4].cpu(), hc), (K, C, R, S, "crsk")


def test_weight_prep_batch_one_output(dev):
    """Only one of the two outputs requested (the eval fold asks for KRSC only)."""
    dt = torch.bfloat16
    w = torch.randn(256, 128, 3, 3, generator=torch.Generator().manual_seed(6))
    hk, hc = _host(w, 128, 3, None, dt)
    krsc = torch.empty((256, 3, 3, 128), device=dev, dtype=dt)
    crsk = torch.empty((128, 3, 3, 256), device=dev, dtype=dt)
    ops.weight_prep_batch([(w.to(dev), 128, 3, krsc, None)], dt)
    ops.weight_prep_batch([(w.to(dev), 128, 3, None, crsk)], dt)
    torch.cuda.synchronize()
    assert torch.equal(krsc.cpu(), hk)
    assert torch.equal(crsk.cpu(), hc)
