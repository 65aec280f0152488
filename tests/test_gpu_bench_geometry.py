"""GPU parity at the benchmarked geometry: every conv of the ResNet-18 train
step at batch 256, 224x224 (bench.py's workload), through the production
kernel that geometry selects (asserted by name via ssip_conv_kernel_name).

Oracle: torch CPU float32 convolution on the bf16-rounded operands (the
"plain PyTorch fp32 reference" of a floating-point kernel).
Tolerances, per element (bf16 outputs are an fp32 accumulation rounded once
to bf16, so the error is at most half a bf16 ulp = 2^-8 |value| plus the
fp32 summation-order difference):
    |y - ref| <= 2^-8 |ref| + 1e-4 max|ref|
(dgrad + residual add: + 2^-8 |dgrad|, the second rounding, see _check_bf16)
fp32 weight gradients (reductions over up to 802,816 rows):
    max|dw - ref| <= 1e-4 max|ref|
BN statistics from the forward's partial records: rel 1e-3.
"""
import pytest
import torch
import torch.nn.functional as F

from ssip import ops
from ssip.ops import ConvGeom

pytestmark = pytest.mark.gpu

N = 256
# name, (C, H, K, R, stride, pad), expected kernel per pass (prefix match)
CONVS = [
    ("l1.3x3", (64, 56, 64, 3, 1, 1), {"fwd": "halo<fwd", "dgrad": "halo<dgrad", "wgrad": "halo_wgrad<"}),
    ("l2.0.conv1", (64, 56, 128, 3, 2, 1), {"fwd": "glds<fwd,128x128", "dgrad": "glds<dgrad,128x64,4x2,2,phased",
                                            "wgrad": "glds<wgrad,128x128", "budget": "glds<wgrad,128x256,2x4,2"}),
    ("l2.3x3", (128, 28, 128, 3, 1, 1), {"fwd": "glds<fwd,128x128", "dgrad": "glds<dgrad,128x128",
                                         "wgrad": "glds<wgrad,128x128", "budget": "glds<wgrad,128x256,2x4,2"}),
    ("l2.ds", (64, 56, 128, 1, 2, 0), {"fwd": "glds<fwd", "dgrad": "glds<dgrad", "wgrad": "glds<wgrad"}),
    ("l3.0.conv1", (128, 28, 256, 3, 2, 1), {"fwd": "glds<fwd", "dgrad": "glds<dgrad,128x128,4x2,2,phased",
                                             "wgrad": "glds<wgrad", "budget": "glds<wgrad,128x256,2x4,2"}),
    ("l3.3x3", (256, 14, 256, 3, 1, 1), {"fwd": "glds<fwd,256x256,4x2,2", "dgrad": "glds<dgrad,256x256,4x2,2",
                                         "wgrad": "glds<wgrad,128x128", "budget": "glds<wgrad,256x256,4x2,2"}),
    ("l3.ds", (128, 28, 256, 1, 2, 0), {"fwd": "glds<fwd", "dgrad": "glds<dgrad", "wgrad": "glds<wgrad"}),
    ("l4.0.conv1", (256, 14, 512, 3, 2, 1), {"fwd": "glds<fwd", "dgrad": "glds<dgrad,128x128,4x2,2,phased",
                                             "wgrad": "glds<wgrad", "budget": "glds<wgrad,256x256,4x2,2"}),
    ("l4.3x3", (512, 7, 512, 3, 1, 1), {"fwd": "glds<fwd", "dgrad": "glds<dgrad", "wgrad": "glds<wgrad",
                                        "budget": "glds<wgrad,256x256,4x2,2"}),
    ("l4.ds", (256, 14, 512, 1, 2, 0), {"fwd": "glds<fwd", "dgrad": "glds<dgrad", "wgrad": "glds<wgrad"}),
]
DT = torch.bfloat16


def _geom(C, H, K, R, st, pd, n=N):
    return ConvGeom(n, H, H, C, K, R, R, st, pd, C, R)


def _check_bf16(out_nhwc, ref_nchw, what, pre_add=None):
    """pre_add: the dgrad term of a dgrad+add output.  The kernels round the
    dgrad accumulator to bf16 and then add the bf16 residual gradient with one
    more rounding (as a bf16 torch autograd graph does: dgrad output, then the
    add), so that output may carry one half-ulp of each: 2^-8 (|dgrad| + |sum|)."""
    ref = ref_nchw.permute(0, 2, 3, 1).float()
    got = out_nhwc.float().cpu()
    bound = ref.abs() * 2.0 ** -8 + 1e-4 * ref.abs().max()
    if pre_add is not None:
        bound = bound + pre_add.permute(0, 2, 3, 1).float().abs() * 2.0 ** -8
    over = ((got - ref).abs() - bound).max().item()
    assert over <= 0, f"{what}: worst element exceeds the bf16 rounding bound by {over:.3e}"


def _rnd(t):
    return t.bfloat16().float()


@pytest.mark.parametrize("n", [N, 128], ids=["bs256", "weak128"])
@pytest.mark.parametrize("name,shape,kern", CONVS, ids=[c[0] for c in CONVS])
def test_fwd_bs256(dev, name, shape, kern, n):
    """n = 128: the weak (pseudo-label) forward's batch in the step."""
    C, H, K, R, st, pd = shape
    g = _geom(*shape, n=n)
    if n == N:
        assert ops.conv_kernel_name("fwd", g, DT).startswith(kern["fwd"]), ops.conv_kernel_name("fwd", g, DT)
    gen = torch.Generator().manual_seed(100)
    x = _rnd(torch.randn(n, C, H, H, generator=gen))
    w = _rnd(torch.randn(K, C, R, R, generator=gen) * (2.0 / (C * R * R)) ** 0.5)
    ref = F.conv2d(x, w, stride=st, padding=pd)
    xh = ops.nchw_to_nhwc(x.to(dev), C, DT)
    krsc = torch.empty((K, R, R, C), device=dev, dtype=DT)
    ops.weight_prep(w.to(dev), DT, C, R, krsc, None)
    y = torch.empty((n, g.P, g.Q, K), device=dev, dtype=DT)
    part = torch.full((ops.conv_fwd_partial_floats(g),), float("nan"), device=dev)
    ops.conv_fwd(g, xh, krsc, y, part)
    stats = torch.empty((4, K), device=dev)
    rm, rv = torch.zeros(K, device=dev), torch.ones(K, device=dev)
    ops.bn_finalize(K, ops.conv_fwd_partial_tiles(g, DT), part, torch.ones(K, device=dev), torch.zeros(K, device=dev),
                    rm, rv, 0.1, 1e-5, True, stats[0], stats[1], stats[2], stats[3])
    torch.cuda.synchronize()
    _check_bf16(y, ref, f"{name} fwd")
    r = ref.double().permute(0, 2, 3, 1).reshape(-1, K)
    mean, var = r.mean(0), r.var(0, unbiased=False)
    m_got = stats[0].cpu().double()
    v_got = 1.0 / stats[1].cpu().double() ** 2 - 1e-5
    assert ((m_got - mean).abs().max() / var.sqrt().max()).item() < 1e-3, name
    assert ((v_got - var).abs().max() / var.max()).item() < 1e-3, name


@pytest.mark.parametrize("name,shape,kern", CONVS, ids=[c[0] for c in CONVS])
def test_dgrad_bs256(dev, name, shape, kern):
    C, H, K, R, st, pd = shape
    g = _geom(*shape)
    assert ops.conv_kernel_name("dgrad", g, DT).startswith(kern["dgrad"]), ops.conv_kernel_name("dgrad", g, DT)
    gen = torch.Generator().manual_seed(101)
    w = _rnd(torch.randn(K, C, R, R, generator=gen) * (2.0 / (K * R * R)) ** 0.5)
    dy = _rnd(torch.randn(N, K, g.P, g.Q, generator=gen))
    add = _rnd(torch.randn(N, C, H, H, generator=gen))
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w, dy, stride=st, padding=pd)
    crsk = torch.empty((C, R, R, K), device=dev, dtype=DT)
    ops.weight_prep(w.to(dev), DT, C, R, None, crsk)
    dyh = ops.nchw_to_nhwc(dy.to(dev), K, DT)
    dx = torch.empty((N, H, H, C), device=dev, dtype=DT)
    ops.conv_dgrad(g, dyh, crsk, dx, None)
    # in-place accumulation (the engine adds the downsample branch into dx)
    dx2 = ops.nchw_to_nhwc(add.to(dev), C, DT)
    ops.conv_dgrad(g, dyh, crsk, dx2, dx2)
    torch.cuda.synchronize()
    _check_bf16(dx, ref, f"{name} dgrad")
    _check_bf16(dx2, ref + add, f"{name} dgrad+add", pre_add=ref)


@pytest.mark.parametrize("name,shape,kern", CONVS, ids=[c[0] for c in CONVS])
def test_wgrad_bs256(dev, name, shape, kern):
    C, H, K, R, st, pd = shape
    g = _geom(*shape)
    assert ops.conv_kernel_name("wgrad", g, DT).startswith(kern["wgrad"]), ops.conv_kernel_name("wgrad", g, DT)
    gen = torch.Generator().manual_seed(102)
    x = _rnd(torch.relu(torch.randn(N, C, H, H, generator=gen)))
    dy = _rnd(torch.randn(N, K, g.P, g.Q, generator=gen) * 1e-2)
    ref = torch.nn.grad.conv2d_weight(x, (K, C, R, R), dy, stride=st, padding=pd)
    xh = ops.nchw_to_nhwc(x.to(dev), C, DT)
    dyh = ops.nchw_to_nhwc(dy.to(dev), K, DT)
    ws = torch.empty(ops.conv_wgrad_workspace_bytes(g), device=dev, dtype=torch.uint8)
    base = torch.randn(K, C, R, R, device=dev)
    dw = torch.full((K, C, R, R), float("nan"), device=dev)
    ops.conv_wgrad(g, dyh, xh, dw, False, ws)
    dwa = base.clone()
    ops.conv_wgrad(g, dyh, xh, dwa, True, ws)
    # side-stream grids (ssip_conv_wgrad_budget): the engine's own choice (one
    # workgroup per CU; half the CUs for the persistent layer-1 wgrad), and a
    # small odd cap (uneven persistent tile ranges / one split): the same
    # result up to the split / slab sum's fp32 order
    from ssip.resnet import _side_wgrad_budget

    budgets = (_side_wgrad_budget(g, DT, dev), 7)
    if "budget" in kern:  # the side stream's production kernel (round 6: 8-wave wide tiles on 62 % of the CUs)
        assert ops.conv_kernel_name("wgrad", g, DT, budgets[0]).startswith(kern["budget"]), \
            ops.conv_kernel_name("wgrad", g, DT, budgets[0])
    dwb = []
    for b in budgets:
        dwb.append(torch.full((K, C, R, R), float("nan"), device=dev))
        wsb = torch.empty(ops.conv_wgrad_workspace_bytes(g, b), device=dev, dtype=torch.uint8)
        ops.conv_wgrad(g, dyh, xh, dwb[-1], False, wsb, max_workgroups=b)
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    assert (dw.cpu() - ref).abs().max().item() <= 1e-4 * scale, name
    assert (dwa.cpu() - base.cpu() - ref).abs().max().item() <= 1e-4 * scale + 1e-6 * base.abs().max().item(), name
    for b, d in zip(budgets, dwb):
        assert (d.cpu() - ref).abs().max().item() <= 1e-4 * scale, (name, b)


def test_stem_bs256(dev):
    """The 7x7/2 stem on the pre-padded NHWC4 image at batch 256: forward
    (stem_halo) and wgrad (stem_wgrad), and the fused BN-backward + wgrad
    (ssip_stem_bwd_wgrad) against the unfused apply pass + wgrad."""
    C, K = 3, 64
    g = ConvGeom(N, 230, 230, 4, K, 7, 8, 2, 0, 3, 7)
    assert ops.conv_kernel_name("fwd", g, DT).startswith("stem_halo<")
    assert ops.conv_kernel_name("wgrad", g, DT).startswith("stem_wgrad<")
    gen = torch.Generator().manual_seed(103)
    x = _rnd(torch.randn(N, C, 224, 224, generator=gen))
    w = _rnd(torch.randn(K, C, 7, 7, generator=gen) * 0.1)
    ref = F.conv2d(x, w, stride=2, padding=3)
    xh = ops.nchw_to_nhwc(x.to(dev), 4, DT, pad=3)
    krsc = torch.empty((K, 7, 8, 4), device=dev, dtype=DT)
    ops.weight_prep(w.to(dev), DT, 4, 8, krsc, None)
    y = torch.empty((N, 112, 112, K), device=dev, dtype=DT)
    part = torch.empty(ops.conv_fwd_partial_floats(g), device=dev)
    ops.conv_fwd(g, xh, krsc, y, part)
    torch.cuda.synchronize()
    _check_bf16(y, ref, "stem fwd")
    dy = _rnd(torch.randn(N, K, 112, 112, generator=gen) * 1e-2)
    ref_w = torch.nn.grad.conv2d_weight(x, (K, C, 7, 7), dy, stride=2, padding=3)
    ws = torch.empty(ops.conv_wgrad_workspace_bytes(g), device=dev, dtype=torch.uint8)
    dw = torch.empty(K, C, 7, 7, device=dev)
    ops.conv_wgrad(g, ops.nchw_to_nhwc(dy.to(dev), K, DT), xh, dw, False, ws)
    torch.cuda.synchronize()
    assert (dw.cpu() - ref_w).abs().max().item() <= 1e-4 * ref_w.abs().max().item()

    # fused stem backward tail vs unfused, same inputs (rel 2e-3: fma contraction only)
    assert ops.stem_bwd_wgrad_supported(g, DT)
    mean = torch.randn(K, device=dev) * 0.1
    invstd = torch.rand(K, device=dev) + 0.5
    gamma = torch.rand(K, device=dev) + 0.5
    scale = gamma * invstd
    shift = torch.randn(K, device=dev) * 0.1 - mean * scale
    pool = torch.empty(N, 56, 56, K, device=dev, dtype=DT)
    idx = torch.empty(N, 56, 56, K, device=dev, dtype=torch.uint8)
    ymax = torch.empty_like(pool)
    ops.stem_bn_pool_fwd(N, 112, 112, K, 3, 2, 1, y, scale, shift, pool, idx, ymax)
    dpool = (torch.randn(N, 56, 56, K, device=dev) * 1e-2).to(DT)
    sp = torch.empty(ops.stem_pool_bn_bwd_partial_floats(N, 112, 112, K), device=dev)
    dg, db, coef = torch.empty(K, device=dev), torch.empty(K, device=dev), torch.empty(3 * K, device=dev)
    dyb = torch.empty_like(y)
    ops.stem_pool_bn_bwd(N, 112, 112, K, 3, 2, 1, dpool, idx, y, mean, invstd, scale, shift, gamma, dg, db, False, dyb,
                         sp, coef, ymax)
    dw0 = torch.empty(K, C, 7, 7, device=dev)
    ops.conv_wgrad(g, dyb, xh, dw0, False, ws)
    dg2, db2, coef2 = torch.empty(K, device=dev), torch.empty(K, device=dev), torch.empty(3 * K, device=dev)
    ops.stem_pool_bn_bwd(N, 112, 112, K, 3, 2, 1, dpool, idx, y, mean, invstd, scale, shift, gamma, dg2, db2, False,
                         None, sp, coef2, ymax)
    dw1 = torch.empty(K, C, 7, 7, device=dev)
    ops.stem_bwd_wgrad(g, dpool, idx, y, xh, scale, shift, coef2, dw1, False, ws)
    torch.cuda.synchronize()
    assert torch.equal(coef, coef2) and torch.equal(dg, dg2) and torch.equal(db, db2)
    assert (dw1 - dw0).abs().max().item() <= 2e-3 * dw0.abs().max().item()
    # the fused kernel (conv_stem_bwd_wgrad2: dy formed per tile in LDS, never
    # stored) directly against torch's fp32 weight gradient of the materialised
    # bf16 dy: the unfused wgrad reads exactly that dy (1e-4, summation order);
    # the fused one forms the same bf16 values with the same coefficients, up to
    # fma contraction in a few elements (2e-3)
    ref_w1 = torch.nn.grad.conv2d_weight(x, (K, C, 7, 7), dyb.float().permute(0, 3, 1, 2).cpu(), stride=2, padding=3)
    scale_w1 = ref_w1.abs().max().item()
    assert (dw0.cpu() - ref_w1).abs().max().item() <= 1e-4 * scale_w1
    assert (dw1.cpu() - ref_w1).abs().max().item() <= 2e-3 * scale_w1


def _bn_affine(C, gen):
    """A BatchNorm affine of both signs (scale = gamma * invstd, shift = beta - mean * scale)."""
    scale = (torch.rand(C, generator=gen) + 0.25) * torch.where(torch.rand(C, generator=gen) < 0.2, -1.0, 1.0)
    shift = torch.randn(C, generator=gen) * 0.5
    return scale, shift


def _bnrelu_ref(y, scale, shift):
    """bf16(relu(fma_f32(y, scale, shift))), NCHW: ssip_bn_apply's arithmetic.
    The product of a bf16 y and an fp32 scale is exact in fp64 and the sum is
    rounded to fp64 once, so rounding that to fp32 is the fp32 fma (up to a
    double-rounding case of probability ~2^-29); then one RNE rounding to bf16."""
    z = (y.double() * scale.double()[None, :, None, None] + shift.double()[None, :, None, None]).float()
    return torch.relu(z).bfloat16().float()


@pytest.mark.parametrize("n", [N, 128], ids=["bs256", "weak128"])
def test_bnrelu_in_fwd_bench_geometry(dev, n):
    """ABI 13's layer-1 forward with bn1's BN+ReLU formed in the conv's LDS
    tile (the step's layer1.x.conv2 at batch 256; the weak forward's 128),
    against torch fp32 conv2d of relu(bn(y1)) on bf16-rounded operands, plus
    its BN statistics and the optional z_out."""
    C = K = 64
    H = 56
    g = _geom(C, H, K, 3, 1, 1, n=n)
    assert ops.conv_bnrelu_in_supported(g, DT)
    assert ops.conv_kernel_name("fwd", g, DT).startswith("halo<fwd"), ops.conv_kernel_name("fwd", g, DT)
    gen = torch.Generator().manual_seed(104)
    y1 = _rnd(torch.randn(n, C, H, H, generator=gen))
    scale, shift = _bn_affine(C, gen)
    w = _rnd(torch.randn(K, C, 3, 3, generator=gen) * (2.0 / (C * 9)) ** 0.5)
    z = _bnrelu_ref(y1, scale, shift)
    ref = F.conv2d(z, w, stride=1, padding=1)
    yh = ops.nchw_to_nhwc(y1.to(dev), C, DT)
    krsc = torch.empty((K, 3, 3, C), device=dev, dtype=DT)
    ops.weight_prep(w.to(dev), DT, C, 3, krsc, None)
    out = torch.empty((n, H, H, K), device=dev, dtype=DT)
    part = torch.full((ops.conv_fwd_partial_floats(g),), float("nan"), device=dev)
    zo = torch.empty_like(yh)
    ops.conv_fwd_bnrelu_in(g, yh, scale.to(dev), shift.to(dev), krsc, out, part, z_out=zo)
    stats = torch.empty((4, K), device=dev)
    rm, rv = torch.zeros(K, device=dev), torch.ones(K, device=dev)
    ops.bn_finalize(K, ops.conv_fwd_partial_tiles(g, DT), part, torch.ones(K, device=dev), torch.zeros(K, device=dev),
                    rm, rv, 0.1, 1e-5, True, stats[0], stats[1], stats[2], stats[3])
    torch.cuda.synchronize()
    _check_bf16(out, ref, f"bnrelu_in fwd n={n}")
    # z_out: the transformed input itself, bit for bit
    assert torch.equal(zo.float().cpu(), z.permute(0, 2, 3, 1))
    r = ref.double().permute(0, 2, 3, 1).reshape(-1, K)
    mean, var = r.mean(0), r.var(0, unbiased=False)
    assert ((stats[0].cpu().double() - mean).abs().max() / var.sqrt().max()).item() < 1e-3
    assert ((1.0 / stats[1].cpu().double() ** 2 - 1e-5 - var).abs().max() / var.max()).item() < 1e-3


def test_bnrelu_in_wgrad_bench_geometry(dev):
    """ABI 13's layer-1 weight gradient with the input relu(bn(y1)) formed in
    LDS, at batch 256: the full grid and the step's side-stream budget (half the
    CUs), fresh and accumulating, against torch fp32 conv2d_weight."""
    from ssip.resnet import _side_wgrad_budget

    C = K = 64
    H = 56
    g = _geom(C, H, K, 3, 1, 1)
    assert ops.conv_bnrelu_in_supported(g, DT)
    assert ops.conv_kernel_name("wgrad", g, DT).startswith("halo_wgrad<"), ops.conv_kernel_name("wgrad", g, DT)
    gen = torch.Generator().manual_seed(105)
    y1 = _rnd(torch.randn(N, C, H, H, generator=gen))
    scale, shift = _bn_affine(C, gen)
    dy = _rnd(torch.randn(N, K, H, H, generator=gen) * 1e-2)
    z = _bnrelu_ref(y1, scale, shift)
    ref = torch.nn.grad.conv2d_weight(z, (K, C, 3, 3), dy, stride=1, padding=1)
    yh = ops.nchw_to_nhwc(y1.to(dev), C, DT)
    dyh = ops.nchw_to_nhwc(dy.to(dev), K, DT)
    sc, sh = scale.to(dev), shift.to(dev)
    scale_max = ref.abs().max().item()
    base = torch.randn(K, C, 3, 3, device=dev)
    for b in (0, _side_wgrad_budget(g, DT, dev)):
        ws = torch.empty(ops.conv_wgrad_workspace_bytes(g, b), device=dev, dtype=torch.uint8)
        dw = torch.full((K, C, 3, 3), float("nan"), device=dev)
        ops.conv_wgrad_bnrelu_in(g, dyh, yh, sc, sh, dw, False, ws, max_workgroups=b)
        dwa = base.clone()
        ops.conv_wgrad_bnrelu_in(g, dyh, yh, sc, sh, dwa, True, ws, max_workgroups=b)
        torch.cuda.synchronize()
        assert (dw.cpu() - ref).abs().max().item() <= 1e-4 * scale_max, b
        assert (dwa.cpu() - base.cpu() - ref).abs().max().item() <= 1e-4 * scale_max + 1e-6 * base.abs().max().item(), b


@pytest.mark.parametrize("n,ymax", [(N, True), (128, False)], ids=["bs256_ymax", "weak128"])
def test_stem_pool_k3s2_bench_geometry(dev, n, ymax):
    """The stem's BN+ReLU+3x3/2 max-pool (stem_bn_pool_fwd_k3s2) at 112^2:
    batch 256 with argmax + ymax (the train forward), batch 128 without ymax
    (the weak forward), against torch fp32 max_pool2d of relu(bn(y)) --
    pooled values exact, argmax = torch's window index, ymax = y there."""
    C, H = 64, 112
    want = f"stem_bn_pool_fwd_k3s2<{2 if ymax else 0}>"
    assert ops.stem_bn_pool_kernel_name(DT, n, H, H, C, 3, 2, 1, ymax) == want
    gen = torch.Generator().manual_seed(106)
    y = _rnd(torch.randn(n, C, H, H, generator=gen))
    scale, shift = _bn_affine(C, gen)
    z = _bnrelu_ref(y, scale, shift)
    ref, ridx = F.max_pool2d(z, 3, 2, 1, return_indices=True)
    yh = ops.nchw_to_nhwc(y.to(dev), C, DT)
    P = 56
    out = torch.empty(n, P, P, C, device=dev, dtype=DT)
    idx = torch.empty(n, P, P, C, device=dev, dtype=torch.uint8)
    ym = torch.empty(n, P, P, C, device=dev, dtype=DT) if ymax else None
    ops.stem_bn_pool_fwd(n, H, H, C, 3, 2, 1, yh, scale.to(dev), shift.to(dev), out, idx, ym)
    torch.cuda.synchronize()
    got = out.float().cpu().permute(0, 3, 1, 2)
    assert torch.equal(got, ref)
    # argmax bytes (window tap t = 3 dr + ds) -> the flat input index torch
    # returns; both take the first maximum in window order
    t = idx.long().cpu().permute(0, 3, 1, 2)
    pr = torch.arange(P).view(1, 1, P, 1)
    pc = torch.arange(P).view(1, 1, 1, P)
    flat = (2 * pr - 1 + t // 3) * H + (2 * pc - 1 + t % 3)
    assert torch.equal(flat, ridx)
    if ymax:
        yv = y.reshape(n, C, H * H).gather(2, ridx.reshape(n, C, -1)).reshape(n, C, P, P)
        assert torch.equal(ym.float().cpu().permute(0, 3, 1, 2), yv)
