"""GPU parity at BASELINE config 5's own geometry beyond the bottleneck convs
(those are tests/test_gpu_r50_geometry.py): ResNet-50, 512x512 input, batch
128 per GPU (reference model boundary: src/training/common.py:299-304).

  * stem 7x7/2 conv on the pre-padded 518x518 NHWC4 image, forward and
    weight gradient, through the kernels this geometry selects (asserted by
    name: the LDS-DMA stem kernels -- the persistent stem kernels are
    224-only); fp64 reference on sampled outputs (forward: 4,096 pixels x 64
    channels) and on full reductions (wgrad: 16 output channels x 3 x 7 x 7
    over all 8,388,608 output pixels);
  * stem BN -> ReLU -> 3x3/2 max-pool forward and its backward through the
    unfused path config 5 takes (ssip_stem_bwd_wgrad_supported is 0 here,
    conv.hip's fused stem backward needs Q = 112): pooled values vs the
    window max, argmax bytes consistent with them, dy / dgamma / dbeta vs
    fp64 with the kernel's own routing of each window's gradient;
  * BatchNorm at layer-1 size, M = 128 * 128 * 128 = 2,097,152 rows x 256
    channels: bn_finalize over 16,384 tile records, bn_apply (+ residual,
    + ReLU, mask bits), bn_bwd (mask from the bits) vs fp64.

Tolerances: bf16 outputs |y - ref| <= 2^-8 |ref| + 1e-4 max|ref| (one bf16
rounding of an fp32 result); fp32 reductions (weight gradients, dgamma,
dbeta, batch statistics) rel <= 2e-4 of the largest element; mask bits and
argmax consistency exact.  The bf16 ResNet-50 semi step at 512x512 against
the fp64 oracle is in tests/test_gpu_semi_step.py.
"""
import pytest
import torch

from ssip import ops
from ssip.ops import ConvGeom

pytestmark = pytest.mark.gpu
N, S = 128, 512
DT = torch.bfloat16


def _check_bf16(got, ref, what):
    got, ref = got.double(), ref.double()
    bound = ref.abs() * 2.0 ** -8 + 1e-4 * ref.abs().max()
    over = ((got - ref).abs() - bound).max().item()
    assert over <= 0, f"{what}: worst element exceeds the bf16 rounding bound by {over:.3e}"


def _rel(got, ref):
    got, ref = got.double(), ref.double()
    return ((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()


def _stem_geom():
    return ConvGeom(N, S + 6, S + 6, 4, 64, 7, 8, 2, 0, 3, 7)


@pytest.fixture(scope="module")
def stem_io():
    """The stem's operands at config 5: pre-padded bf16 NHWC4 input, bf16
    weights (real KCRS and the kernel's KRSC), and the forward output."""
    dev = torch.device("cuda", 0)
    g = _stem_geom()
    gen = torch.Generator(device="cuda").manual_seed(501)
    x = torch.randn(N, 3, S, S, device=dev, generator=gen).to(DT).float()
    xh = ops.nchw_to_nhwc(x, 4, DT, pad=3)  # [N, 518, 518, 4], channel 3 and the border zero
    del x
    w = (torch.randn(64, 3, 7, 7, device=dev, generator=gen) * 0.1).to(DT).float()
    krsc = torch.empty((64, 7, 8, 4), device=dev, dtype=DT)
    ops.weight_prep(w, DT, 4, 8, krsc, None)
    y = torch.empty((N, g.P, g.Q, 64), device=dev, dtype=DT)
    part = torch.empty(ops.conv_fwd_partial_floats(g), device=dev)
    ops.conv_fwd(g, xh, krsc, y, part)
    torch.cuda.synchronize()
    return g, xh, w, y


def test_c5_stem_fwd(dev, stem_io):
    g, xh, w, y = stem_io
    assert (g.P, g.Q) == (256, 256)
    assert ops.conv_kernel_name("fwd", g, DT).startswith("glds<fwd,"), ops.conv_kernel_name("fwd", g, DT)
    gen = torch.Generator(device="cuda").manual_seed(502)
    idx = torch.randint(0, N * g.P * g.Q, (4096,), device="cuda", generator=gen)
    n, p, q = idx // (g.P * g.Q), (idx // g.Q) % g.P, idx % g.Q
    rows = torch.stack([xh[n, 2 * p + r, 2 * q + s, :3].double() for r in range(7) for s in range(7)], 1)
    ref = rows.reshape(4096, 147) @ w.double().permute(0, 2, 3, 1).reshape(64, 147).T
    _check_bf16(y[n, p, q], ref, "stem fwd 512")


def test_c5_stem_wgrad(dev, stem_io):
    g, xh, _, _ = stem_io
    assert ops.conv_kernel_name("wgrad", g, DT).startswith("glds<wgrad,"), ops.conv_kernel_name("wgrad", g, DT)
    gen = torch.Generator(device="cuda").manual_seed(503)
    dy = (torch.randn(N, g.P, g.Q, 64, device=dev, generator=gen) * 1e-2).to(DT)
    ws = torch.empty(ops.conv_wgrad_workspace_bytes(g), device=dev, dtype=torch.uint8)
    dw = torch.full((64, 3, 7, 7), float("nan"), device=dev)
    ops.conv_wgrad(g, dy, xh, dw, False, ws)
    ks = torch.randperm(64, generator=torch.Generator().manual_seed(504))[:16].to(dev)
    dys = dy[..., ks].double().reshape(-1, 16)
    ref = torch.empty(16, 3, 7, 7, device=dev, dtype=torch.float64)
    for r in range(7):
        for s in range(7):
            xs = xh[:, r: r + 2 * (g.P - 1) + 1: 2, s: s + 2 * (g.Q - 1) + 1: 2, :3].double().reshape(-1, 3)
            ref[:, :, r, s] = dys.T @ xs
    torch.cuda.synchronize()
    assert _rel(dw[ks], ref) <= 2e-4


def test_c5_stem_bn_pool_fwd_bwd(dev, stem_io):
    """The stem's BN -> ReLU -> max-pool forward and the unfused backward
    (ssip_stem_pool_bn_bwd: pooled-grid reduction with ymax, then the apply
    pass that materialises dy for the LDS-DMA stem wgrad) at 256x256 x 64."""
    g, _, _, y = stem_io
    assert not ops.stem_bwd_wgrad_supported(g, DT)  # config 5 takes this path
    C, H, W = 64, g.P, g.Q
    P, Q = H // 2, W // 2
    gen = torch.Generator(device="cuda").manual_seed(505)
    mean = torch.randn(C, device=dev, generator=gen) * 0.1
    invstd = torch.rand(C, device=dev, generator=gen) + 0.5
    gamma = torch.rand(C, device=dev, generator=gen) + 0.5
    beta = torch.randn(C, device=dev, generator=gen) * 0.1
    scale = gamma * invstd
    shift = beta - mean * scale
    pool = torch.empty(N, P, Q, C, device=dev, dtype=DT)
    idx = torch.empty(N, P, Q, C, device=dev, dtype=torch.uint8)
    ymax = torch.empty_like(pool)
    ops.stem_bn_pool_fwd(N, H, W, C, 3, 2, 1, y, scale, shift, pool, idx, ymax)
    # z = relu(fma(y, scale, shift)) rounded as the kernel stores it; the pool is its window max
    z32 = (y.double() * scale.double() + shift.double()).float()
    zb = torch.relu(z32).to(DT)
    zmax = torch.nn.functional.max_pool2d(zb.float().permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert ((pool.float() - zmax).abs() <= zmax.abs() * 2.0 ** -7).all()
    # the argmax byte names a window element holding the pooled value
    ii = torch.arange(P, device=dev).view(1, P, 1, 1)
    jj = torch.arange(Q, device=dev).view(1, 1, Q, 1)
    hh = 2 * ii - 1 + (idx.long() // 3)
    ww = 2 * jj - 1 + (idx.long() % 3)
    assert bool(((hh >= 0) & (hh < H) & (ww >= 0) & (ww < W)).all())
    nn_ = torch.arange(N, device=dev).view(N, 1, 1, 1)
    cc = torch.arange(C, device=dev).view(1, 1, 1, C)
    flat = ((nn_ * H + hh) * W + ww) * C + cc
    del hh, ww
    assert torch.equal(zb.reshape(-1)[flat.reshape(-1)].view(N, P, Q, C), pool)
    assert torch.equal(y.reshape(-1)[flat.reshape(-1)].view(N, P, Q, C), ymax)
    del zb, zmax
    # backward through the unfused path, vs fp64 with the kernel's own routing
    dpool = (torch.randn(N, P, Q, C, device=dev, generator=gen) * 1e-2).to(DT)
    dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
    part = torch.empty(ops.stem_pool_bn_bwd_partial_floats(N, H, W, C), device=dev)
    coef = torch.empty(3 * C, device=dev)
    dyo = torch.empty_like(y)
    ops.stem_pool_bn_bwd(N, H, W, C, 3, 2, 1, dpool, idx, y, mean, invstd, scale, shift, gamma, dg, db, False, dyo,
                         part, coef, ymax)
    M = N * H * W
    da = torch.zeros(M * C, device=dev, dtype=torch.float64)
    da.index_put_((flat.reshape(-1),), dpool.double().reshape(-1), accumulate=True)
    del flat
    dz = da.view(N, H, W, C) * (z32 > 0)
    del da, z32
    xhat = (y.double() - mean.double()) * invstd.double()
    db_ref = dz.sum((0, 1, 2))
    dg_ref = (dz * xhat).sum((0, 1, 2))
    dy_ref = (gamma * invstd).double() * (dz - db_ref / M - xhat * (dg_ref / M))
    del dz, xhat
    torch.cuda.synchronize()
    assert _rel(db, db_ref) <= 2e-4
    assert _rel(dg, dg_ref) <= 2e-4
    _check_bf16(dyo, dy_ref, "stem BN-pool backward dy")


def test_c5_bn_layer1_size(dev):
    """BatchNorm passes at ResNet-50 layer-1 size (bottleneck output, 256
    channels at 128x128, batch 128): 2,097,152 rows."""
    C, M, T = 256, N * 128 * 128, 128
    tiles = M // T
    gen = torch.Generator(device="cuda").manual_seed(506)
    y = (torch.randn(M, C, device=dev, generator=gen) * 2
         + torch.linspace(-1, 1, C, device=dev)).to(DT)
    res = torch.randn(M, C, device=dev, generator=gen).to(DT)
    gamma = torch.rand(C, device=dev, generator=gen) + 0.5
    beta = torch.randn(C, device=dev, generator=gen) * 0.1
    # forward statistics from per-(channel, 128-row tile) {count, sum, M2} records, as the conv epilogue emits
    yt = y.view(tiles, T, C).double()
    tsum = yt.sum(1)
    tm2 = ((yt - (tsum / T).unsqueeze(1)) ** 2).sum(1)
    del yt
    part = torch.stack([torch.full_like(tsum, T), tsum, tm2], 2).permute(1, 0, 2).contiguous().float()  # [C][tiles][3]
    del tsum, tm2
    scratch = torch.empty(C * tiles * 3 + ops.bn_finalize_scratch_floats(C, tiles), device=dev)
    scratch[: part.numel()].copy_(part.reshape(-1))
    del part
    stats = torch.empty(4, C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    ops.bn_finalize(C, tiles, scratch, gamma, beta, rm, rv, 0.1, 1e-5, True, stats[0], stats[1], stats[2], stats[3])
    yd = y.double()
    mu = yd.mean(0)
    var = yd.var(0, unbiased=False)
    torch.cuda.synchronize()
    assert _rel(stats[0], mu) <= 2e-4
    assert _rel(stats[1], 1.0 / torch.sqrt(var + 1e-5)) <= 2e-4
    assert _rel(rv, 0.9 + 0.1 * yd.var(0, unbiased=True)) <= 2e-4
    # apply: z = relu(bn(y) + res), with the ReLU mask bits
    mean, invstd, scale, shift = stats[0], stats[1], stats[2], stats[3]
    z = torch.empty_like(y)
    mbits = torch.empty(M * C // 8, device=dev, dtype=torch.uint8)
    ops.bn_apply(M, C, y, scale, shift, res, True, z, mbits)
    zref = torch.relu(yd * scale.double() + shift.double() + res.double())
    _check_bf16(z, zref, "bn_apply 2M rows")
    del zref
    pos = (z.view(-1) > 0).view(-1, 8).to(torch.uint8)
    want = (pos << torch.arange(8, device=dev, dtype=torch.uint8)).sum(1, dtype=torch.uint8)
    assert torch.equal(want, mbits)
    del pos, want
    # backward with the mask from the bits
    dz = (torch.randn(M, C, device=dev, generator=gen) * 1e-2).to(DT)
    dgam, dbet = torch.empty(C, device=dev), torch.empty(C, device=dev)
    dy, dpre = torch.empty_like(y), torch.empty_like(y)
    pb = torch.empty(ops.bn_bwd_partial_floats(M, C), device=dev)
    coef = torch.empty(3 * C, device=dev)
    ops.bn_bwd(M, C, dz, None, y, mean, invstd, gamma, dgam, dbet, False, dy, dpre, pb, coef, mbits=mbits)
    g = dz.double() * (z > 0)
    assert torch.equal(dpre, g.to(DT))
    xhat = (yd - mean.double()) * invstd.double()
    db_ref = g.sum(0)
    dg_ref = (g * xhat).sum(0)
    dy_ref = (gamma * invstd).double() * (g - db_ref / M - xhat * (dg_ref / M))
    torch.cuda.synchronize()
    assert _rel(dbet, db_ref) <= 2e-4
    assert _rel(dgam, dg_ref) <= 2e-4
    _check_bf16(dy, dy_ref, "bn_bwd 2M rows")
