"""GPU parity of the stem's BN -> ReLU -> 3x3/2 max-pool forward kernel for
the ResNet stem's shape class (bf16, C = 64, pad 1, even H and W: the
VALU-lean `stem_bn_pool_fwd_k3s2_kernel`, csrc/stem.hip) against the generic
kernel (SSIP_POOL_ROWS=0) and against ssip_bn_apply + ssip_maxpool_fwd.

Pooled values, argmax bytes and ymax must be bit-identical, including ties
(ReLU zeros everywhere, equal values), negative scales, -0.0, +-inf and NaN
inputs (NaN maps to 0 as in ssip_bn_apply), pooled heights that are not a
multiple of the rows-per-workgroup walk, and the padding column / row."""
import pytest
import torch

from ssip import ops

pytestmark = pytest.mark.gpu

SHAPES = [
    (2, 112, 112),  # the stem at 224^2
    (3, 18, 22),    # 9 pooled rows: a remainder for every rows-per-workgroup value
    (1, 8, 128),    # 64 pooled columns: 512 threads
    (1, 6, 260),    # 130 pooled columns: three column groups, the last partial
    (2, 2, 2),      # one pooled pixel, every window clipped
]


def _run(monkeypatch, rows, N, H, W, y, scale, shift, with_ymax, lds=0):
    monkeypatch.setenv("SSIP_POOL_ROWS", str(rows))
    monkeypatch.setenv("SSIP_POOL_LDS", str(lds))
    P, Q = H // 2, W // 2
    dev = y.device
    pool = torch.full((N, P, Q, 64), 3.0, device=dev, dtype=torch.bfloat16)
    idx = torch.full((N, P, Q, 64), 77, device=dev, dtype=torch.uint8)
    ymax = torch.full_like(pool, 5.0) if with_ymax else None
    ops.stem_bn_pool_fwd(N, H, W, 64, 3, 2, 1, y, scale, shift, pool, idx, ymax)
    torch.cuda.synchronize()
    return pool, idx, ymax


def _inputs(N, H, W, dev, seed, special):
    g = torch.Generator(device="cpu").manual_seed(seed)
    y = torch.randn(N, H, W, 64, generator=g).to(torch.bfloat16)
    if special:
        # coarse values: many exact ties after BN + rounding
        y = (y * 2).round().to(torch.bfloat16) / 2
        flat = y.view(-1)
        n = flat.numel()
        pick = torch.randperm(n, generator=g)
        flat[pick[: n // 50]] = float("nan")
        flat[pick[n // 50: n // 25]] = float("inf")
        flat[pick[n // 25: 3 * n // 50]] = float("-inf")
        flat[pick[3 * n // 50: n // 10]] = -0.0
    scale = (torch.rand(64, generator=g) + 0.25) * torch.where(torch.rand(64, generator=g) < 0.25, -1.0, 1.0)
    shift = torch.randn(64, generator=g) * 0.5
    if special:
        scale[:4] = 0.0   # every y -> shift: all nine taps tie
        shift[:2] = 0.0   # ... at exactly zero
        shift[2:4] = -1.0
    return y.to(dev), scale.to(dev), shift.to(dev)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("special", [False, True])
def test_k3s2_equals_generic(dev, monkeypatch, shape, special):
    N, H, W = shape
    y, scale, shift = _inputs(N, H, W, dev, 5, special)
    ref = _run(monkeypatch, 0, N, H, W, y, scale, shift, True)
    for rows in (4, 3, 1, 8):
        for lds in (0, 1):
            got = _run(monkeypatch, rows, N, H, W, y, scale, shift, True, lds)
            for a, b in zip(got, ref):
                assert torch.equal(a.view(torch.uint8), b.view(torch.uint8)), (rows, lds)
        p2, i2, _ = _run(monkeypatch, rows, N, H, W, y, scale, shift, False)
        assert torch.equal(p2.view(torch.uint8), ref[0].view(torch.uint8))
        assert torch.equal(i2, ref[1])
        # a no-grad forward: no argmax bytes, the same pooled values
        monkeypatch.setenv("SSIP_POOL_ROWS", str(rows))
        p3 = torch.full_like(ref[0], 3.0)
        ops.stem_bn_pool_fwd(N, H, W, 64, 3, 2, 1, y, scale, shift, p3, None, None)
        torch.cuda.synchronize()
        assert torch.equal(p3.view(torch.uint8), ref[0].view(torch.uint8))


@pytest.mark.parametrize("special", [False, True])
def test_k3s2_equals_apply_then_maxpool(dev, monkeypatch, special):
    N, H, W = 2, 24, 20
    y, scale, shift = _inputs(N, H, W, dev, 6, special)
    z = torch.empty_like(y)
    ops.bn_apply(N * H * W, 64, y, scale, shift, None, True, z)
    pool_r = torch.empty(N, H // 2, W // 2, 64, device=dev, dtype=torch.bfloat16)
    idx_r = torch.empty(N, H // 2, W // 2, 64, device=dev, dtype=torch.uint8)
    ops.maxpool_fwd(N, H, W, 64, 3, 2, 1, z, pool_r, idx_r)
    pool, idx, _ = _run(monkeypatch, 4, N, H, W, y, scale, shift, True)
    assert torch.equal(pool.view(torch.uint8), pool_r.view(torch.uint8))
    assert torch.equal(idx, idx_r)
