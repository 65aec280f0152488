"""GPU parity of the downsampling-block fusions (ABI 5):

* ssip_conv_dgrad_ds: conv1 (3x3/2) and downsample (1x1/2) input gradients of
  a BasicBlock in one phase-split launch, at the benchmarked batch (256) and at
  a ragged small batch, vs torch CPU fp32 on the bf16-rounded operands; the
  f32 dtype takes the two-launch path and is held to the f32 bound.
* ssip_bn_apply2: relu(bn2(y2) + bn_ds(y_ds)) vs the unfused apply pair
  (f32: bit-identical, same fma sequence) and vs torch fp64.
* ssip_bn_bwd_dual: its backward vs torch fp64 autograd of the same graph.

Reference semantics: torchvision BasicBlock.forward (out = bn2(conv2(..)) +
downsample(x); relu), used by the reference at src/training/common.py:380-382.
Tolerances are written at each assert (bf16 bound as in
tests/test_gpu_bench_geometry.py).
"""
import pytest
import torch
import torch.nn.functional as F

from ssip import ops
from ssip.ops import ConvGeom

pytestmark = pytest.mark.gpu

DT = torch.bfloat16
# (C, H, K) of the stride-2 blocks of ResNet-18
BLOCKS = [("l2", 64, 56, 128), ("l3", 128, 28, 256), ("l4", 256, 14, 512)]


def _rnd(t):
    return t.bfloat16().float()


def _check(out_nhwc, ref_nchw, what, rel_ulp):
    ref = ref_nchw.permute(0, 2, 3, 1).double()
    got = out_nhwc.double().cpu()
    bound = ref.abs() * rel_ulp + 1e-4 * ref.abs().max()
    over = ((got - ref).abs() - bound).max().item()
    assert over <= 0, f"{what}: worst element exceeds the rounding bound by {over:.3e}"


@pytest.mark.parametrize("n", [256, 3], ids=["bs256", "n3"])
@pytest.mark.parametrize("dtname", ["bf16", "f32"])
@pytest.mark.parametrize("name,C,H,K", BLOCKS, ids=[b[0] for b in BLOCKS])
def test_conv_dgrad_ds(dev, name, C, H, K, dtname, n):
    if dtname == "f32" and n == 256:
        pytest.skip("f32 runs the unfused pair; covered at n=3")
    dt = DT if dtname == "bf16" else torch.float32
    g = ConvGeom(n, H, H, C, K, 3, 3, 2, 1, C, 3)
    gds = ConvGeom(n, H, H, C, K, 1, 1, 2, 0, C, 1)
    gen = torch.Generator().manual_seed(7)
    w = _rnd(torch.randn(K, C, 3, 3, generator=gen) * (2.0 / (K * 9)) ** 0.5)
    wds = _rnd(torch.randn(K, C, 1, 1, generator=gen) * (2.0 / K) ** 0.5)
    dy = _rnd(torch.randn(n, K, g.P, g.Q, generator=gen))
    dyds = _rnd(torch.randn(n, K, g.P, g.Q, generator=gen))
    ref = (torch.nn.grad.conv2d_input((n, C, H, H), w, dy, stride=2, padding=1) +
           torch.nn.grad.conv2d_input((n, C, H, H), wds, dyds, stride=2, padding=0))
    crsk = torch.empty((C, 3, 3, K), device=dev, dtype=dt)
    ops.weight_prep(w.to(dev), dt, C, 3, None, crsk)
    cds = torch.empty((C, 1, 1, K), device=dev, dtype=dt)
    ops.weight_prep(wds.to(dev), dt, C, 1, None, cds)
    dx = torch.full((n, H, H, C), float("nan"), device=dev, dtype=dt)
    ops.conv_dgrad_ds(g, ops.nchw_to_nhwc(dy.to(dev), K, dt), crsk, gds, ops.nchw_to_nhwc(dyds.to(dev), K, dt),
                      cds, dx)
    torch.cuda.synchronize()
    # bf16: one fp32 accumulation over both operands, rounded once (half an ulp, 2^-8);
    # f32: summation order only
    _check(dx, ref, f"{name} dgrad_ds {dtname}", 2.0 ** -8 if dt == DT else 1e-5)


@pytest.mark.parametrize("dtname", ["f32", "bf16"])
def test_bn_apply2(dev, dtname):
    dt = DT if dtname == "bf16" else torch.float32
    torch.manual_seed(1)
    M, C = 3 * 14 * 14 + 5, 256
    y, y2 = torch.randn(M, C), torch.randn(M, C)
    sc, sh = torch.rand(C) + 0.5, torch.randn(C) * 0.2
    sc2, sh2 = torch.randn(C), torch.randn(C) * 0.2
    yh, y2h = y.to(dev, dt), y2.to(dev, dt)
    z = torch.empty_like(yh)
    ops.bn_apply2(M, C, yh, sc.to(dev), sh.to(dev), y2h, sc2.to(dev), sh2.to(dev), True, z)
    # unfused: ident = bn_ds(y2) (stored), then relu(bn2(y) + ident)
    ident = torch.empty_like(yh)
    ops.bn_apply(M, C, y2h, sc2.to(dev), sh2.to(dev), None, False, ident)
    z2 = torch.empty_like(yh)
    ops.bn_apply(M, C, yh, sc.to(dev), sh.to(dev), ident, True, z2)
    torch.cuda.synchronize()
    if dt == torch.float32:
        assert torch.equal(z, z2), "f32: the fused pass runs the same fma / add sequence"
    ref = torch.relu(yh.double().cpu() * sc.double() + sh.double() + y2h.double().cpu() * sc2.double() + sh2.double())
    tol = 1e-6 if dt == torch.float32 else 2.0 ** -8
    assert ((z.double().cpu() - ref).abs() - tol * ref.abs() - 1e-6).max().item() <= 0


@pytest.mark.parametrize("dtname", ["f32", "bf16"])
def test_bn_bwd_dual(dev, dtname):
    dt = DT if dtname == "bf16" else torch.float32
    torch.manual_seed(2)
    N, C, H = 4, 128, 9
    M = N * H * H
    ya = torch.randn(N, C, H, H) * 2 + 0.3
    yb = torch.randn(N, C, H, H) - 0.2
    g = torch.randn(N, C, H, H)
    if dt == DT:
        ya, yb, g = _rnd(ya), _rnd(yb), _rnd(g)
    ga, ba = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    gb, bb = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    yad, ybd = ya.double().requires_grad_(), yb.double().requires_grad_()
    gad, bad_ = ga.double().requires_grad_(), ba.double().requires_grad_()
    gbd, bbd = gb.double().requires_grad_(), bb.double().requires_grad_()
    out = torch.relu(F.batch_norm(yad, None, None, gad, bad_, training=True, eps=1e-5) +
                     F.batch_norm(ybd, None, None, gbd, bbd, training=True, eps=1e-5))
    out.backward(g.double())

    def nhwc(t):
        return t.permute(0, 2, 3, 1).reshape(M, C).contiguous()

    def stats(y):
        yd = nhwc(y).double()
        mean, var = yd.mean(0), yd.var(0, unbiased=False)
        return mean.float().to(dev), (1.0 / (var + 1e-5).sqrt()).float().to(dev)

    ma, ia = stats(ya)
    mb, ib = stats(yb)
    # the forward output (mask source) from the fused apply with batch-stat coefficients
    sca, sha = ga.to(dev) * ia, ba.to(dev) - ma * ga.to(dev) * ia
    scb, shb = gb.to(dev) * ib, bb.to(dev) - mb * gb.to(dev) * ib
    yah, ybh = nhwc(ya).to(dev, dt), nhwc(yb).to(dev, dt)
    z = torch.empty_like(yah)
    ops.bn_apply2(M, C, yah, sca, sha, ybh, scb, shb, True, z)
    gh = nhwc(g).to(dev, dt)
    dga, dba, dgb, dbb = (torch.full((C,), float("nan"), device=dev) for _ in range(4))
    dya, dyb = torch.empty_like(yah), torch.empty_like(ybh)
    part = torch.empty(ops.bn_bwd_dual_partial_floats(M, C), device=dev)
    coef = torch.empty(6 * C, device=dev)
    ops.bn_bwd_dual(M, C, gh, z, yah, ma, ia, ga.to(dev), dga, dba, ybh, mb, ib, gb.to(dev), dgb, dbb, False, dya, dyb,
                    part, coef)
    torch.cuda.synchronize()

    def rel(a, b):
        return ((a.double().cpu() - b.double()).abs().max() / b.double().abs().max()).item()

    tol = 1e-4 if dt == torch.float32 else 5e-2  # bf16: mask flips at near-zero outputs + bf16 dy
    assert rel(dga, gad.grad) < tol and rel(dba, bad_.grad) < tol
    assert rel(dgb, gbd.grad) < tol and rel(dbb, bbd.grad) < tol
    assert rel(dya, nhwc(yad.grad)) < tol and rel(dyb, nhwc(ybd.grad)) < tol
    # accumulate mode adds the same sums again
    ops.bn_bwd_dual(M, C, gh, z, yah, ma, ia, ga.to(dev), dga, dba, ybh, mb, ib, gb.to(dev), dgb, dbb, True, dya, dyb,
                    part, coef)
    torch.cuda.synchronize()
    assert rel(dgb, 2 * gbd.grad) < tol and rel(dba, 2 * bad_.grad) < tol


@pytest.mark.parametrize("dtname", ["f32", "bf16"])
def test_relu_mask_bits(dev, dtname):
    """ssip_bn_apply(2)'s mask bits (bit j of byte i = z[8i+j] > 0) and the
    backward passes that read them instead of z: the same outputs, bit for bit."""
    dt = DT if dtname == "bf16" else torch.float32
    torch.manual_seed(3)
    M, C = 2 * 7 * 7 + 3, 64
    y, y2, r = (torch.randn(M, C, device=dev).to(dt) for _ in range(3))
    sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.3
    sc2, sh2 = torch.randn(C, device=dev), torch.randn(C, device=dev) * 0.3
    z, bits = torch.empty_like(y), torch.empty(M * C // 8, device=dev, dtype=torch.uint8)
    ops.bn_apply(M, C, y, sc, sh, r, True, z, bits)
    z2, bits2 = torch.empty_like(y), torch.empty_like(bits)
    ops.bn_apply2(M, C, y, sc, sh, y2, sc2, sh2, True, z2, bits2)
    torch.cuda.synchronize()
    w = (2 ** torch.arange(8, device=dev)).to(torch.int32)
    for zz, bb in ((z, bits), (z2, bits2)):
        want = ((zz.float() > 0).reshape(-1, 8).to(torch.int32) * w).sum(1).to(torch.uint8)
        assert torch.equal(bb, want)
    dz = torch.randn(M, C, device=dev).to(dt)
    mean, invstd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    gamma = torch.rand(C, device=dev) + 0.5
    outs = []
    for zm, mb in ((z, None), (None, bits)):
        dg, db, dy, dpre = torch.empty(C, device=dev), torch.empty(C, device=dev), torch.empty_like(y), torch.empty_like(y)
        part = torch.empty(ops.bn_bwd_partial_floats(M, C), device=dev)
        coef = torch.empty(3 * C, device=dev)
        ops.bn_bwd(M, C, dz, zm, y, mean, invstd, gamma, dg, db, False, dy, dpre, part, coef, mbits=mb)
        outs.append((dg, db, dy, dpre))
    for zm, mb in ((z2, None), (None, bits2)):
        t = [torch.empty(C, device=dev) for _ in range(4)]
        dya, dyb = torch.empty_like(y), torch.empty_like(y)
        part = torch.empty(ops.bn_bwd_dual_partial_floats(M, C), device=dev)
        coef = torch.empty(6 * C, device=dev)
        ops.bn_bwd_dual(M, C, dz, zm, y, mean, invstd, gamma, t[0], t[1], y2, mean, invstd, gamma, t[2], t[3], False,
                        dya, dyb, part, coef, mbits=mb)
        outs.append(tuple(t) + (dya, dyb))
    torch.cuda.synchronize()
    for a, b in ((outs[0], outs[1]), (outs[2], outs[3])):
        for x, y_ in zip(a, b):
            assert torch.equal(x, y_)
