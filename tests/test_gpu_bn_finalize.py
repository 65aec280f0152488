"""BatchNorm finalize (forward statistics and backward coefficients) over
record counts either side of the split point (more than 2048 records per
channel are merged by several 256-thread workgroups plus a one-wave merge
pass).  Reference: the same records merged on the host in float64 (Chan's
pairwise formula for {count, sum, M2}; plain sums for the backward), i.e. the
batch mean / biased variance torchvision's BatchNorm2d uses
(src/training/common.py:380 `model(inputs)` in train mode).  Tolerance:
rel 1e-6 on mean / invstd (fp64 merge, fp32 output rounding)."""
import numpy as np
import pytest
import torch

from ssip import ops

pytestmark = pytest.mark.gpu


def _records(C, tiles, seed, empty_every=0):
    rng = np.random.default_rng(seed)
    n = rng.integers(1, 300, size=(C, tiles)).astype(np.float64)
    if empty_every:
        n[:, ::empty_every] = 0.0
    mu = rng.normal(0.7, 2.0, size=(C, 1)) + rng.normal(0, 0.3, size=(C, tiles))
    m2 = n * rng.uniform(0.5, 4.0, size=(C, tiles))
    rec = np.stack([n, n * mu, m2], -1).astype(np.float32)
    rec[n == 0] = 0.0
    return rec


def _host_stats(rec):
    r = rec.astype(np.float64)
    n, s, m2 = r[..., 0], r[..., 1], r[..., 2]
    N = n.sum(1)
    mean = s.sum(1) / N
    with np.errstate(invalid="ignore", divide="ignore"):
        mt = np.where(n > 0, s / np.where(n > 0, n, 1), 0.0)
    M2 = m2.sum(1) + (n * (mt - mean[:, None]) ** 2).sum(1)
    return N, mean, M2 / N


@pytest.mark.parametrize("C,tiles,empty", [(64, 1, 0), (64, 513, 0), (64, 2048, 0), (64, 2049, 0), (128, 5000, 7),
                                           (64, 18816, 0), (8, 140000, 0)])
def test_bn_finalize_split(dev, C, tiles, empty):
    rec = _records(C, tiles, seed=tiles + C, empty_every=empty)
    N, mean, var = _host_stats(rec)
    extra = ops.bn_finalize_scratch_floats(C, tiles)
    assert (extra > 0) == (tiles > 2048)
    part = torch.full((C * tiles * 3 + extra,), float("nan"), device=dev)
    part[:C * tiles * 3] = torch.from_numpy(rec.reshape(-1)).to(dev)
    keep = part[:C * tiles * 3].clone()
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev)
    rm = torch.randn(C, device=dev)
    rv = torch.rand(C, device=dev) + 0.5
    rm0, rv0 = rm.clone(), rv.clone()
    st = torch.empty(4, C, device=dev)
    ops.bn_finalize(C, tiles, part, gamma, beta, rm, rv, 0.1, 1e-5, True, st[0], st[1], st[2], st[3])
    torch.cuda.synchronize()
    assert torch.equal(part[:C * tiles * 3], keep)  # the records are not modified
    invstd = 1.0 / np.sqrt(var + 1e-5)
    got = st.double().cpu().numpy()
    np.testing.assert_allclose(got[0], mean, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(got[1], invstd, rtol=1e-6)
    g = gamma.double().cpu().numpy()
    np.testing.assert_allclose(got[2], g * invstd, rtol=1e-6)
    np.testing.assert_allclose(got[3], beta.double().cpu().numpy() - mean * g * invstd, rtol=1e-5, atol=1e-5)
    unb = var * N / (N - 1)
    np.testing.assert_allclose(rm.double().cpu().numpy(), 0.9 * rm0.double().cpu().numpy() + 0.1 * mean,
                               rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(rv.double().cpu().numpy(), 0.9 * rv0.double().cpu().numpy() + 0.1 * unb, rtol=1e-6)
    # deterministic: a second call gives identical bits
    st2 = torch.empty_like(st)
    ops.bn_finalize(C, tiles, part, gamma, beta, rm, rv, 0.1, 1e-5, False, st2[0], st2[1], st2[2], st2[3])
    torch.cuda.synchronize()
    assert torch.equal(st, st2)


@pytest.mark.parametrize("tiles", [512, 513, 2049, 9408])
def test_bn_bwd_from_partials_split(dev, tiles):
    """[C][tiles][2] sums of dout and dout*xhat (the dgrad-fused BN reduction)
    -> dgamma / dbeta and dy = dBN(dout), split finalize included."""
    C, M = 64, 4096
    rng = np.random.default_rng(tiles)
    p = rng.normal(0, 1, size=(C, tiles, 2)).astype(np.float32)
    sums = p.astype(np.float64).sum(1)  # [C][2]
    extra = 0 if tiles <= 2048 else 2 + C * 64 * 4
    part = torch.full((tiles * C * 2 + extra,), float("nan"), device=dev)
    part[:tiles * C * 2] = torch.from_numpy(p.reshape(-1)).to(dev)
    dout = torch.randn(M, C, device=dev)
    y = torch.randn(M, C, device=dev)
    mean = torch.randn(C, device=dev) * 0.1
    invstd = torch.rand(C, device=dev) + 0.5
    gamma = torch.rand(C, device=dev) + 0.5
    dg = torch.empty(C, device=dev)
    db = torch.empty(C, device=dev)
    dy = torch.empty_like(dout)
    coef = torch.empty(3 * C, device=dev)
    ops.bn_bwd_from_partials(M, C, tiles, part, dout, y, mean, invstd, gamma, dg, db, False, dy, coef)
    torch.cuda.synchronize()
    np.testing.assert_allclose(db.double().cpu().numpy(), sums[:, 0], rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(dg.double().cpu().numpy(), sums[:, 1], rtol=1e-6, atol=1e-5)
    g, i, m = (t.double().cpu().numpy() for t in (gamma, invstd, mean))
    A = g * i
    k0 = -A * sums[:, 0] / M
    k1 = -A * sums[:, 1] / M * i
    ref = A * dout.double().cpu().numpy() + k1 * y.double().cpu().numpy() + (k0 - k1 * m)
    np.testing.assert_allclose(dy.double().cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
