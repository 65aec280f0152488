"""GPU parity of the halo-resident 3x3 conv path (conv_halo_kernel: ResNet
layer1's forward convs and stride-1 dgrads with 64 reduction channels).

Each MFMA k-step is one weight tap's 64 channels in tap order, as in the
implicit-GEMM kernel, so y / dx must equal that path's output bit for bit
(SSIP_HALO=0 selects it).  Against torch float64 on the bf16-rounded
operands: rel-err <= 1e-2 (output rounding).  The BN statistics come from
per-workgroup merged records and are checked through ssip_bn_finalize
(mean / biased var rel-err <= 1e-3)."""
import pytest
import torch
import torch.nn.functional as F

from ssip import ops
from ssip.ops import ConvGeom

pytestmark = pytest.mark.gpu

SHAPES = [
    # N, C(=64), H, W, K
    (2, 64, 56, 56, 64),    # layer1 (TR = 4 rows of 56)
    (3, 64, 28, 28, 128),   # two 64-column panels, TR = 7
    (2, 64, 16, 16, 64),    # TR = 16: the whole image in one tile
    (5, 64, 56, 56, 64),    # tiles not a multiple of the workgroup count
]


def _relerr(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


def _stats(g, part, dt, dev):
    K = g.K
    stats = torch.empty((4, K), device=dev)
    ops.bn_finalize(K, ops.conv_fwd_partial_tiles(g, dt), part, torch.ones(K, device=dev),
                    torch.zeros(K, device=dev), torch.zeros(K, device=dev), torch.ones(K, device=dev), 0.1, 1e-5,
                    True, stats[0], stats[1], stats[2], stats[3])
    torch.cuda.synchronize()
    return stats[0].cpu(), (1 / stats[1].cpu().double() ** 2 - 1e-5)


@pytest.mark.parametrize("shape", SHAPES)
def test_halo_fwd(dev, shape, monkeypatch):
    torch.manual_seed(10)
    N, C, H, W, K = shape
    dt = torch.bfloat16
    g = ConvGeom(N, H, W, C, K, 3, 3, 1, 1, C, 3)
    x = torch.randn(N, C, H, W).bfloat16().float()
    w = (torch.randn(K, C, 3, 3) * 0.1).bfloat16().float()
    ref = F.conv2d(x.double(), w.double(), padding=1).permute(0, 2, 3, 1)
    xh = ops.nchw_to_nhwc(x.to(dev), C, dt)
    krsc = torch.empty((K, 3, 3, C), device=dev, dtype=dt)
    ops.weight_prep(w.to(dev), dt, C, 3, krsc, None)

    monkeypatch.delenv("SSIP_HALO", raising=False)
    y = torch.empty((N, H, W, K), device=dev, dtype=dt)
    part = torch.full((ops.conv_fwd_partial_floats(g),), float("nan"), device=dev)
    ops.conv_fwd(g, xh, krsc, y, part)
    mean_h, var_h = _stats(g, part, dt, dev)

    monkeypatch.setenv("SSIP_HALO", "0")
    y0 = torch.empty_like(y)
    part0 = torch.empty(ops.conv_fwd_partial_floats(g), device=dev)
    ops.conv_fwd(g, xh, krsc, y0, part0)
    mean_0, var_0 = _stats(g, part0, dt, dev)
    torch.cuda.synchronize()

    assert torch.equal(y, y0)
    assert _relerr(y.cpu(), ref) < 1e-2
    r = ref.reshape(-1, K)
    assert _relerr(mean_h, r.mean(0)) < 1e-3
    assert _relerr(var_h, r.var(0, unbiased=False)) < 1e-3
    assert _relerr(mean_h, mean_0.double()) < 1e-4
    assert _relerr(var_h, var_0) < 1e-4


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("add", ["none", "separate", "in_place"])
def test_halo_dgrad(dev, shape, add, monkeypatch):
    torch.manual_seed(11)
    N, Cr, H, W, Kc = shape
    # dgrad of a conv with C_in = Kc (the output columns) and K_out = 64 (the reduction)
    C, K = Kc, 64
    dt = torch.bfloat16
    g = ConvGeom(N, H, W, C, K, 3, 3, 1, 1, C, 3)
    w = (torch.randn(K, C, 3, 3) * 0.1).bfloat16().float()
    dy = torch.randn(N, K, H, W).bfloat16().float()
    addt = torch.randn(N, C, H, W).bfloat16().float()
    ref = torch.nn.grad.conv2d_input((N, C, H, W), w.double(), dy.double(), padding=1)
    if add != "none":
        ref = ref + addt.double()
    ref = ref.permute(0, 2, 3, 1)
    crsk = torch.empty((C, 3, 3, K), device=dev, dtype=dt)
    ops.weight_prep(w.to(dev), dt, C, 3, None, crsk)
    dyh = ops.nchw_to_nhwc(dy.to(dev), K, dt)
    addh = ops.nchw_to_nhwc(addt.to(dev), C, dt)

    def run():
        if add == "in_place":
            dx = addh.clone()
            ops.conv_dgrad(g, dyh, crsk, dx, dx)
        else:
            dx = torch.empty((N, H, W, C), device=dev, dtype=dt)
            ops.conv_dgrad(g, dyh, crsk, dx, addh if add == "separate" else None)
        torch.cuda.synchronize()
        return dx

    monkeypatch.delenv("SSIP_HALO", raising=False)
    dx = run()
    monkeypatch.setenv("SSIP_HALO", "0")
    dx0 = run()
    assert torch.equal(dx, dx0)
    assert _relerr(dx.cpu(), ref) < 1e-2


def test_halo_partial_tiles_is_workgroup_count(dev, monkeypatch):
    """The BN record count of a halo forward is its workgroup count and fits
    the buffer sized by ssip_conv_fwd_partial_floats."""
    monkeypatch.delenv("SSIP_HALO", raising=False)
    g = ConvGeom(256, 56, 56, 64, 64, 3, 3, 1, 1, 64, 3)
    tiles = ops.conv_fwd_partial_tiles(g, torch.bfloat16)
    assert 1 <= tiles <= 256 * 56 // 4
    assert tiles * 64 * 3 <= ops.conv_fwd_partial_floats(g)
    monkeypatch.setenv("SSIP_HALO", "0")
    assert ops.conv_fwd_partial_tiles(g, torch.bfloat16) == -(-256 * 56 * 56 // 128)


@pytest.mark.parametrize("shape", [(2, 56, 56), (3, 16, 16), (5, 56, 56)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_halo_wgrad(dev, shape, accumulate, monkeypatch):
    """conv_halo_wgrad_kernel (C = K = 64, 3x3/s1/p1): fp32 dW against torch
    float64 on the bf16 operands (rel-err <= 1e-4, the implicit-GEMM path's
    bound) and against that path itself (the k-order differs: not bitwise)."""
    torch.manual_seed(12)
    N, H, W = shape
    C = K = 64
    dt = torch.bfloat16
    g = ConvGeom(N, H, W, C, K, 3, 3, 1, 1, C, 3)
    x = torch.randn(N, C, H, W).bfloat16().float()
    dy = torch.randn(N, K, H, W).bfloat16().float()
    ref = torch.nn.grad.conv2d_weight(x.double(), (K, C, 3, 3), dy.double(), padding=1)
    xh = ops.nchw_to_nhwc(x.to(dev), C, dt)
    dyh = ops.nchw_to_nhwc(dy.to(dev), K, dt)
    ws = torch.empty(ops.conv_wgrad_workspace_bytes(g), device=dev, dtype=torch.uint8)
    base = torch.randn(K, C, 3, 3, device=dev)

    def run():
        dw = base.clone()
        ops.conv_wgrad(g, dyh, xh, dw, accumulate, ws)
        torch.cuda.synchronize()
        return dw.cpu().double()

    monkeypatch.delenv("SSIP_HALO", raising=False)
    dw = run()
    monkeypatch.setenv("SSIP_HALO", "0")
    dw0 = run()
    want = ref + (base.cpu().double() if accumulate else 0)
    assert _relerr(dw, want) < 1e-4
    assert _relerr(dw, dw0) < 1e-5


@pytest.mark.parametrize("accumulate", [False, True])
def test_stem_bwd_wgrad_fused(dev, accumulate):
    """ssip_stem_bwd_wgrad (dy formed per tile in LDS) against the unfused
    ssip_stem_pool_bn_bwd apply pass + ssip_conv_wgrad on the same inputs
    (224x224 geometry, batch 2).  dy is the same bf16 expression; only
    fused-multiply-add contraction may differ -> dW rel-err <= 2e-3."""
    torch.manual_seed(13)
    N, C = 2, 64
    dt = torch.bfloat16
    g = ConvGeom(N, 230, 230, 4, C, 7, 8, 2, 0, 3, 7)
    assert ops.stem_bwd_wgrad_supported(g, dt)
    x = torch.randn(N, 230, 230, 4, device=dev).to(dt)
    x[..., 3] = 0
    y = torch.randn(N, 112, 112, C, device=dev).to(dt)
    mean = torch.randn(C, device=dev) * 0.1
    invstd = torch.rand(C, device=dev) + 0.5
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev) * 0.1
    scale = gamma * invstd
    shift = beta - mean * scale
    pool = torch.empty(N, 56, 56, C, device=dev, dtype=dt)
    idx = torch.empty(N, 56, 56, C, device=dev, dtype=torch.uint8)
    ymax = torch.empty_like(pool)
    ops.stem_bn_pool_fwd(N, 112, 112, C, 3, 2, 1, y, scale, shift, pool, idx, ymax)
    dpool = torch.randn(N, 56, 56, C, device=dev).to(dt)
    part = torch.empty(ops.stem_pool_bn_bwd_partial_floats(N, 112, 112, C), device=dev)
    ws = torch.empty(ops.conv_wgrad_workspace_bytes(g), device=dev, dtype=torch.uint8)
    base = torch.randn(C, 3, 7, 7, device=dev)

    # unfused
    dg, db, coef = torch.empty(C, device=dev), torch.empty(C, device=dev), torch.empty(3 * C, device=dev)
    dy = torch.empty_like(y)
    ops.stem_pool_bn_bwd(N, 112, 112, C, 3, 2, 1, dpool, idx, y, mean, invstd, scale, shift, gamma, dg, db, False, dy,
                         part, coef, ymax)
    dw0 = base.clone()
    ops.conv_wgrad(g, dy, x, dw0, accumulate, ws)
    # fused
    dg2, db2, coef2 = torch.empty(C, device=dev), torch.empty(C, device=dev), torch.empty(3 * C, device=dev)
    ops.stem_pool_bn_bwd(N, 112, 112, C, 3, 2, 1, dpool, idx, y, mean, invstd, scale, shift, gamma, dg2, db2, False,
                         None, part, coef2, ymax)
    dw = base.clone()
    ops.stem_bwd_wgrad(g, dpool, idx, y, x, scale, shift, coef2, dw, accumulate, ws)
    torch.cuda.synchronize()
    assert torch.equal(coef, coef2) and torch.equal(dg, dg2) and torch.equal(db, db2)
    assert _relerr(dw.cpu(), dw0.cpu()) < 2e-3
