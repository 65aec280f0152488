"""GPU parity: implicit-GEMM conv fwd / dgrad / wgrad and BN statistics vs
torch CPU float64 (the oracle for a floating-point kernel).
Tolerances: f32 path rel-err <= 2e-5 of max|ref|; bf16 path compares against
the f64 result on bf16-rounded operands, rel-err <= 1e-2 (output rounding)."""
import pytest
import torch
import torch.nn.functional as F

from ssip import ops
from ssip.ops import ConvGeom

pytestmark = pytest.mark.gpu

SHAPES = [
    # N, C, H, W, K, R, stride, pad
    (2, 64, 16, 16, 64, 3, 1, 1),
    (2, 64, 16, 16, 128, 3, 2, 1),
    (2, 128, 15, 15, 256, 1, 2, 0),
    (2, 64, 15, 13, 128, 3, 2, 1),  # odd H/W: unequal stride-2 dgrad phases
    (3, 64, 7, 7, 192, 3, 1, 1),
    (2, 3, 32, 32, 64, 7, 2, 3),   # stem (C padded to 4, S to 8)
    (1, 256, 7, 7, 512, 3, 1, 1),
    # stem on a pre-padded image (pad-0 conv over H+6 x W+6; the engine's layout)
    (2, 3, 32, 32, 64, 7, 2, 3, True),
    (3, 3, 56, 40, 64, 7, 2, 3, True),
]


def _unpack(shape):
    N, C, H, W, K, R, st, pd, *rest = shape
    return N, C, H, W, K, R, st, pd, bool(rest and rest[0])


def _geom(N, C, H, W, K, R, st, pd, pre=False):
    stem = C == 3
    if pre:  # the input carries the conv padding as a zero border
        H, W, pd = H + 2 * pd, W + 2 * pd, 0
    return ConvGeom(N=N, H=H, W=W, C=4 if stem else C, K=K, R=R, S=8 if stem else R, stride=st, pad=pd,
                    c_real=C, s_real=R)


def _to_nhwc(x, Cp, dt, dev, pad=0):
    return ops.nchw_to_nhwc(x.to(dev), Cp, dt, pad=pad)


def _relerr(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtname", ["f32", "bf16"])
def test_conv_fwd(dev, shape, dtname):
    torch.manual_seed(0)
    N, C, H, W, K, R, st, pd, pre = _unpack(shape)
    dt = torch.float32 if dtname == "f32" else torch.bfloat16
    g = _geom(*_unpack(shape))
    x = torch.randn(N, C, H, W)
    w = torch.randn(K, C, R, R) * 0.1
    if dt == torch.bfloat16:
        x = x.bfloat16().float()
        w = w.bfloat16().float()
    ref = F.conv2d(x.double(), w.double(), stride=st, padding=pd).permute(0, 2, 3, 1)
    xh = _to_nhwc(x, g.C, dt, dev, pd if pre else 0)
    krsc = torch.empty((K, R, g.S, g.C), device=dev, dtype=dt)
    ops.weight_prep(w.to(dev), dt, g.C, g.S, krsc, None)
    y = torch.empty((N, g.P, g.Q, K), device=dev, dtype=dt)
    part = torch.empty(ops.conv_fwd_partial_floats(g), device=dev)
    ops.conv_fwd(g, xh, krsc, y, part)
    torch.cuda.synchronize()
    assert y.shape[1:3] == ref.shape[1:3]
    tol = 2e-5 if dt == torch.float32 else 1e-2
    assert _relerr(y.cpu(), ref) < tol
    # BN statistics from the partials
    stats = torch.empty((4, K), device=dev)
    gamma = torch.ones(K, device=dev)
    beta = torch.zeros(K, device=dev)
    rm = torch.zeros(K, device=dev)
    rv = torch.ones(K, device=dev)
    ops.bn_finalize(K, ops.conv_fwd_partial_tiles(g, dt), part, gamma, beta, rm, rv, 0.1, 1e-5, True, stats[0], stats[1],
                    stats[2], stats[3])
    torch.cuda.synchronize()
    r = ref.reshape(-1, K)
    mean = r.mean(0)
    var = r.var(0, unbiased=False)
    tol_s = 1e-5 if dt == torch.float32 else 1e-2
    assert _relerr(stats[0].cpu(), mean) < tol_s * 10
    assert _relerr((1 / stats[1].cpu().double() ** 2 - 1e-5), var) < tol_s * 10
    assert _relerr(rv.cpu(), 0.9 + 0.1 * r.var(0, unbiased=True)) < tol_s * 10


@pytest.mark.parametrize("shape", [s for s in SHAPES if s[1] != 3 and len(s) == 8])
@pytest.mark.parametrize("dtname", ["f32", "bf16"])
def test_conv_dgrad(dev, shape, dtname):
    torch.manual_seed(1)
    N, C, H, W, K, R, st, pd = shape
    dt = torch.float32 if dtname == "f32" else torch.bfloat16
    g = _geom(*shape)
    w = torch.randn(K, C, R, R) * 0.1
    dy = torch.randn(N, K, g.P, g.Q)
    add = torch.randn(N, C, H, W)
    if dt == torch.bfloat16:
        w, dy, add = w.bfloat16().float(), dy.bfloat16().float(), add.bfloat16().float()
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.double(), dy.double(), stride=st, padding=pd)
    ref = (ref + add.double()).permute(0, 2, 3, 1)
    crsk = torch.empty((C, R, R, K), device=dev, dtype=dt)
    ops.weight_prep(w.to(dev), dt, C, R, None, crsk)
    dyh = _to_nhwc(dy, K, dt, dev)
    addh = _to_nhwc(add, C, dt, dev)
    dx = torch.empty((N, H, W, C), device=dev, dtype=dt)
    ops.conv_dgrad(g, dyh, crsk, dx, addh)
    torch.cuda.synchronize()
    tol = 2e-5 if dt == torch.float32 else 1e-2
    assert _relerr(dx.cpu(), ref) < tol


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dtname", ["f32", "bf16"])
def test_conv_wgrad(dev, shape, dtname):
    torch.manual_seed(2)
    N, C, H, W, K, R, st, pd, pre = _unpack(shape)
    dt = torch.float32 if dtname == "f32" else torch.bfloat16
    g = _geom(*_unpack(shape))
    x = torch.randn(N, C, H, W)
    dy = torch.randn(N, K, g.P, g.Q)
    if dt == torch.bfloat16:
        x, dy = x.bfloat16().float(), dy.bfloat16().float()
    ref = torch.nn.grad.conv2d_weight(x.double(), (K, C, R, R), dy.double(), stride=st, padding=pd)
    xh = _to_nhwc(x, g.C, dt, dev, pd if pre else 0)
    dyh = _to_nhwc(dy, K, dt, dev)
    dw = torch.full((K, C, R, R), 7.0, device=dev)
    ws = torch.empty(ops.conv_wgrad_workspace_bytes(g), device=dev, dtype=torch.uint8)
    ops.conv_wgrad(g, dyh, xh, dw, False, ws)
    torch.cuda.synchronize()
    tol = 2e-5 if dt == torch.float32 else 1e-4
    assert _relerr(dw.cpu(), ref) < tol
    # accumulate mode adds on top
    ops.conv_wgrad(g, dyh, xh, dw, True, ws)
    torch.cuda.synchronize()
    assert _relerr(dw.cpu(), 2 * ref) < tol


def _mask_bits(m_nhwc):
    """bit j of byte i = element 8i + j of the NHWC-flat mask (ssip_bn_apply's layout)"""
    f = m_nhwc.reshape(-1, 8).to(torch.int32)
    return (f << torch.arange(8, dtype=torch.int32)).sum(1).to(torch.uint8)


@pytest.mark.parametrize("shape", [s for s in SHAPES if s[1] != 3 and len(s) == 8] + [(4, 64, 28, 28, 64, 3, 1, 1)])
@pytest.mark.parametrize("dtname", ["f32", "bf16"])
@pytest.mark.parametrize("with_add", [False, True])
@pytest.mark.parametrize("mask", ["z", "bits", "affine"])
def test_conv_dgrad_bn_fused(dev, shape, dtname, with_add, mask):
    """dgrad epilogue fused with the ReLU mask and the BN-backward partial
    sums of the layer below: dpre = (dgrad + add) * relu_mask,
    sum(dpre), sum(dpre * (y - mean) * invstd) per channel ([C][tiles][2]).
    The mask from z > 0, from the forward's mask bits, or from
    fma(y, scale, shift) > 0; bf16 3x3 / stride-1 / 64-channel shapes run the
    halo kernel (which takes bits or the affine)."""
    torch.manual_seed(3)
    N, C, H, W, K, R, st, pd = shape
    dt = torch.float32 if dtname == "f32" else torch.bfloat16
    g = _geom(*shape)
    halo = ops.conv_kernel_name("dgrad", g, dt).startswith("halo")
    w = torch.randn(K, C, R, R) * 0.1
    dy = torch.randn(N, K, g.P, g.Q)
    add = torch.randn(N, C, H, W)
    y = torch.randn(N, C, H, W) * 2 + 0.5
    z = torch.relu(torch.randn(N, C, H, W))
    if dt == torch.bfloat16:
        w, dy, add, y, z = (t.bfloat16().float() for t in (w, dy, add, y, z))
    mean = torch.randn(C) * 0.1
    invstd = torch.rand(C) + 0.5
    msc = torch.randn(C)
    msh = torch.randn(C) * 0.5
    if mask == "affine":
        keep = (y.double() * msc.double()[None, :, None, None] + msh.double()[None, :, None, None]) > 0
    else:
        keep = z > 0
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.double(), dy.double(), stride=st, padding=pd)
    if with_add:
        ref = ref + add.double()
    if dt == torch.bfloat16:  # the stored dgrad (+ add) is bf16 before the mask and the sums
        ref = ref.float().bfloat16().double()
    ref = ref * keep.double()
    xhat = (y.double() - mean.double()[None, :, None, None]) * invstd.double()[None, :, None, None]
    sum_d = ref.sum((0, 2, 3))
    sum_dx = (ref * xhat).sum((0, 2, 3))
    crsk = torch.empty((C, R, R, K), device=dev, dtype=dt)
    ops.weight_prep(w.to(dev), dt, C, R, None, crsk)
    dpre = torch.empty((N, H, W, C), device=dev, dtype=dt)
    part = torch.full((ops.conv_dgrad_bn_partial_floats(g),), float("nan"), device=dev)
    zh = _to_nhwc(z, C, dt, dev) if mask == "z" else None
    bits = _mask_bits(keep.permute(0, 2, 3, 1).contiguous()).to(dev) if mask == "bits" else None
    sc, sh = (msc.to(dev), msh.to(dev)) if mask == "affine" else (None, None)
    args = (g, _to_nhwc(dy, K, dt, dev), crsk, _to_nhwc(add, C, dt, dev) if with_add else None, zh,
            _to_nhwc(y, C, dt, dev), mean.to(dev), invstd.to(dev), dpre, part)
    if halo and mask == "z":
        with pytest.raises(RuntimeError, match="halo kernel takes mask bits"):
            ops.conv_dgrad_bn(*args)
        return
    ops.conv_dgrad_bn(*args, mask_bits=bits, mscale=sc, mshift=sh)
    torch.cuda.synchronize()
    tol = 2e-5 if dt == torch.float32 else 1e-2
    assert _relerr(dpre.cpu(), ref.permute(0, 2, 3, 1)) < tol
    tiles = ops.conv_dgrad_bn_partial_tiles(g, dt)
    p = part[: tiles * C * 2].view(C, tiles, 2).double().sum(1).cpu()
    tol_s = 1e-4 if dt == torch.float32 else 2e-2
    assert _relerr(p[:, 0], sum_d) < tol_s
    assert _relerr(p[:, 1], sum_dx) < tol_s


@pytest.mark.parametrize("shape", [(16, 64, 28, 28, 128, 3, 1, 1), (8, 128, 14, 14, 256, 1, 2, 0),
                                   (4, 3, 64, 64, 64, 7, 2, 3, True)])
def test_conv_wgrad_many_splits(dev, shape):
    """bf16 wgrad with many split-K slabs (grouped vectorised slab reduction)
    against the fp64 reference; three back-to-back launches give identical
    bits (fixed summation order)."""
    torch.manual_seed(4)
    N, C, H, W, K, R, st, pd, pre = _unpack(shape)
    dt = torch.bfloat16
    g = _geom(*_unpack(shape))
    x = torch.randn(N, C, H, W).bfloat16().float()
    dy = torch.randn(N, K, g.P, g.Q).bfloat16().float()
    ref = torch.nn.grad.conv2d_weight(x.double(), (K, C, R, R), dy.double(), stride=st, padding=pd)
    xh = _to_nhwc(x, g.C, dt, dev, pd if pre else 0)
    dyh = _to_nhwc(dy, K, dt, dev)
    ws = torch.empty(ops.conv_wgrad_workspace_bytes(g), device=dev, dtype=torch.uint8)
    outs = []
    for _ in range(3):
        dw = torch.full((K, C, R, R), 7.0, device=dev)
        ops.conv_wgrad(g, dyh, xh, dw, False, ws)
        torch.cuda.synchronize()
        outs.append(dw.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert _relerr(outs[0], ref) < 1e-4


def test_conv_dgrad_in_place_add_skips_empty_phases(dev):
    """1x1 stride-2 dgrad accumulated in place (dx_add is dx, as the engine
    adds the downsample branch): 3 of 4 output phases receive no tap and are
    left untouched; the result equals ref + the old dx."""
    torch.manual_seed(5)
    N, C, H, W, K, R, st, pd = 2, 128, 15, 15, 256, 1, 2, 0
    dt = torch.bfloat16
    g = _geom(N, C, H, W, K, R, st, pd)
    w = (torch.randn(K, C, R, R) * 0.1).bfloat16().float()
    dy = torch.randn(N, K, g.P, g.Q).bfloat16().float()
    add = torch.randn(N, C, H, W).bfloat16().float()
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.double(), dy.double(), stride=st, padding=pd)
    ref = (ref + add.double()).permute(0, 2, 3, 1)
    crsk = torch.empty((C, R, R, K), device=dev, dtype=dt)
    ops.weight_prep(w.to(dev), dt, C, R, None, crsk)
    dyh = _to_nhwc(dy, K, dt, dev)
    dx = _to_nhwc(add, C, dt, dev)
    ops.conv_dgrad(g, dyh, crsk, dx, dx)
    torch.cuda.synchronize()
    assert _relerr(dx.cpu(), ref) < 1e-2
