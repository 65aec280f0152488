"""GPU parity of the non-GEMM kernels vs torch CPU float64 autograd:
BatchNorm train forward/backward (+ReLU, +residual), max-pool, global
average pool + fc, cross-entropy, pseudo-label selection, consistency loss,
AdamW.  Tolerances: f32 rel-max 1e-5 (1e-4 for reductions over >1e4
elements), bf16 rel-max 2e-2; max-pool indices and pseudo-label picks exact."""
import pytest
import torch
import torch.nn.functional as F

from ssip import ops

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("dtname", ["f32", "bf16"])
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_bn_train_fwd_bwd(dev, dtname, relu, res):
    torch.manual_seed(0)
    dt = torch.float32 if dtname == "f32" else torch.bfloat16
    N, C, H, W = 4, 64, 10, 10
    y = (torch.randn(N, C, H, W) * 2 + 0.5)
    r = torch.randn(N, C, H, W)
    g = torch.randn(N, C, H, W)
    gamma = torch.rand(C) + 0.5
    beta = torch.randn(C) * 0.1
    if dt == torch.bfloat16:
        y, r, g = y.bfloat16().float(), r.bfloat16().float(), g.bfloat16().float()
    yd = y.double().requires_grad_()
    gd = gamma.double().requires_grad_()
    bd = beta.double().requires_grad_()
    out = F.batch_norm(yd, None, None, gd, bd, training=True, eps=1e-5)
    if res:
        out = out + r.double()
    if relu:
        out = torch.relu(out)
    out.backward(g.double())
    # device path: stats from a fake single-tile partial set computed on the host
    M = N * H * W
    ym = _nhwc(y).reshape(M, C)
    part = torch.stack([torch.full((C,), float(M)), ym.double().sum(0).float(),
                        ((ym.double() - ym.double().mean(0)) ** 2).sum(0).float()], 1)  # [C][3] (1 tile)
    part = part.reshape(C, 1, 3).contiguous().to(dev)
    stats = torch.empty(4, C, device=dev)
    rm = torch.zeros(C, device=dev)
    rv = torch.ones(C, device=dev)
    ops.bn_finalize(C, 1, part, gamma.to(dev), beta.to(dev), rm, rv, 0.1, 1e-5, True, stats[0], stats[1], stats[2],
                    stats[3])
    yh = _nhwc(y).to(dev, dt)
    rh = _nhwc(r).to(dev, dt) if res else None
    z = torch.empty_like(yh)
    ops.bn_apply(M, C, yh, stats[2], stats[3], rh, relu, z)
    torch.cuda.synchronize()
    tol = 1e-5 if dt == torch.float32 else 2e-2
    assert _rel(z.cpu(), _nhwc(out.detach())) < tol
    gh = _nhwc(g).to(dev, dt)
    dgam = torch.empty(C, device=dev)
    dbet = torch.empty(C, device=dev)
    dy = torch.empty_like(yh)
    dpre = torch.empty_like(yh)
    part_b = torch.empty(ops.bn_bwd_partial_floats(M, C), device=dev)
    coef = torch.empty(3 * C, device=dev)
    ops.bn_bwd(M, C, gh, z if relu else None, yh, stats[0], stats[1], gamma.to(dev), dgam, dbet, False, dy, dpre,
               part_b, coef)
    torch.cuda.synchronize()
    tolb = 1e-4 if dt == torch.float32 else 5e-2
    assert _rel(dgam, gd.grad) < tolb
    assert _rel(dbet, bd.grad) < tolb
    assert _rel(dy.cpu(), _nhwc(yd.grad)) < tolb
    if relu:
        mask = (_nhwc(out.detach()) > 0)
        assert _rel(dpre.cpu(), _nhwc(g) * mask) < tol
    # accumulate mode
    ops.bn_bwd(M, C, gh, z if relu else None, yh, stats[0], stats[1], gamma.to(dev), dgam, dbet, True, dy, None,
               part_b, coef)
    torch.cuda.synchronize()
    assert _rel(dgam, 2 * gd.grad) < tolb


@pytest.mark.parametrize("dtname", ["f32", "bf16"])
def test_maxpool(dev, dtname):
    torch.manual_seed(0)
    dt = torch.float32 if dtname == "f32" else torch.bfloat16
    N, C, H, W = 2, 64, 17, 16
    x = torch.relu(torch.randn(N, C, H, W))  # many ties at 0, like the stem
    x = x.to(dt).float()
    xd = x.double().requires_grad_()
    y = F.max_pool2d(xd, 3, 2, 1)
    g = torch.randn_like(y).to(dt).double()
    y.backward(g)
    xh = _nhwc(x).to(dev, dt)
    P, Q = y.shape[2], y.shape[3]
    yh = torch.empty(N, P, Q, C, device=dev, dtype=dt)
    idx = torch.empty(N, P, Q, C, device=dev, dtype=torch.uint8)
    ops.maxpool_fwd(N, H, W, C, 3, 2, 1, xh, yh, idx)
    dx = torch.empty_like(xh)
    ops.maxpool_bwd(N, H, W, C, 3, 2, 1, _nhwc(g.float()).to(dev, dt), idx, dx)
    torch.cuda.synchronize()
    assert torch.equal(yh.cpu().float(), _nhwc(y.detach()).float())
    tol = 1e-6 if dt == torch.float32 else 1e-2
    assert _rel(dx.cpu(), _nhwc(xd.grad)) < tol


@pytest.mark.parametrize("dtname", ["f32", "bf16"])
def test_avgpool_fc(dev, dtname):
    torch.manual_seed(0)
    dt = torch.float32 if dtname == "f32" else torch.bfloat16
    B, C, H, W, J = 5, 512, 7, 7, 2
    z = torch.randn(B, C, H, W).to(dt).float()
    w = torch.randn(J, C) * 0.05
    b = torch.randn(J)
    zd = z.double().requires_grad_()
    wd = w.double().requires_grad_()
    bd = b.double().requires_grad_()
    feat = zd.mean((2, 3))
    logits = feat @ wd.t() + bd
    gl = torch.randn(B, J).double()
    logits.backward(gl)
    zh = _nhwc(z).to(dev, dt)
    f = torch.empty(B, C, device=dev)
    lo = torch.empty(B, J, device=dev)
    ops.avgpool_fc_fwd(B, H * W, C, J, zh, w.to(dev), b.to(dev), f, lo)
    dz = torch.empty_like(zh)
    dw = torch.empty(J, C, device=dev)
    db = torch.empty(J, device=dev)
    ops.avgpool_fc_bwd(dt, B, H * W, C, J, gl.float().to(dev), w.to(dev), f, dz, dw, db, False)
    torch.cuda.synchronize()
    assert _rel(f, feat) < 1e-5
    assert _rel(lo, logits) < 1e-5
    assert _rel(dw, wd.grad) < 1e-5
    assert _rel(db, bd.grad) < 1e-5
    assert _rel(dz.cpu(), _nhwc(zd.grad)) < (1e-5 if dt == torch.float32 else 1e-2)


def test_cross_entropy_and_select(dev):
    torch.manual_seed(0)
    z = torch.randn(300, 2) * 3
    y = torch.randint(0, 2, (300,))
    zd = z.double().requires_grad_()
    loss = F.cross_entropy(zd, y)
    loss.backward()
    l, dl, pred = ops.cross_entropy(z.to(dev), y.to(dev))
    torch.cuda.synchronize()
    assert abs(l.item() - loss.item()) < 1e-5 * max(1.0, abs(loss.item()))
    assert _rel(dl, zd.grad) < 1e-5
    assert torch.equal(pred.cpu(), z.argmax(1))
    probs, conf, p2, keep, pos = ops.softmax_select(z.to(dev), 0.7, 0)
    torch.cuda.synchronize()
    pr = torch.softmax(z, 1)
    c, a = pr.max(1)
    assert _rel(probs, pr) < 1e-6
    assert torch.equal(p2.cpu(), a)
    assert torch.equal(keep.cpu().bool(), c >= 0.7)
    assert _rel(pos, pr[:, 0]) < 1e-6


def test_semi_loss(dev):
    torch.manual_seed(1)
    zl = torch.randn(16, 2)
    yl = torch.randint(0, 2, (16,))
    zw = torch.randn(24, 2) * 2
    zs = torch.randn(24, 2)
    tau, lam = 0.7, 1.0
    zld = zl.double().requires_grad_()
    zsd = zs.double().requires_grad_()
    pw = torch.softmax(zw.double(), 1)
    conf, pseudo = pw.max(1)
    mask = (conf >= tau).double()
    lu = (F.cross_entropy(zsd, pseudo, reduction="none") * mask).mean()
    ll = F.cross_entropy(zld, yl)
    tot = ll + lam * lu
    tot.backward()
    out, dzl, dzs, ps, mk = ops.semi_loss(zl.to(dev), yl.to(dev), zw.to(dev), zs.to(dev), tau, lam)
    torch.cuda.synchronize()
    o = out.cpu()
    assert abs(o[0].item() - tot.item()) < 1e-5
    assert abs(o[3].item() - mask.sum().item()) < 0.5
    assert torch.equal(ps.cpu(), pseudo)
    assert _rel(dzl, zld.grad) < 1e-5
    assert _rel(dzs, zsd.grad) < 1e-5


def test_adamw_matches_torch(dev):
    torch.manual_seed(0)
    p0 = torch.randn(1000)
    grads = [torch.randn(1000) for _ in range(3)]
    ref = p0.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=1e-3, weight_decay=1e-2)
    p = p0.clone().to(dev)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for t, g in enumerate(grads, 1):
        ref.grad = g.clone()
        opt.step()
        ops.adamw(p, g.to(dev), m, v, 1e-3, 0.9, 0.999, 1e-8, 1e-2, t)
    torch.cuda.synchronize()
    assert _rel(p, ref.detach()) < 1e-6


def test_adamw_device_schedule_fused_advance(dev):
    """ssip_adamw_dev with advance=1 (ABI 8: the first update launch of a step
    advances t and the bias corrections itself) equals the separate
    ssip_adamw_sched_step + ssip_adamw_dev(advance=0) launches bit for bit,
    through ssip.optim.AdamW's device schedule over 5 steps with several
    launches per step (two arena runs, a loose parameter, a second group, and
    a step split around one parameter as SemiStep does); both stay within
    fp32 rounding of torch.optim.AdamW and count t like it."""
    from ssip.arena import ParamArena
    from ssip.optim import AdamW

    torch.manual_seed(0)
    shapes = [(300,), (17, 5), (1000,), (64,)]
    base = [torch.randn(s) for s in shapes]
    grads = [[torch.randn(s) for s in shapes] for _ in range(5)]
    # reference: torch AdamW on the CPU
    ref = [torch.nn.Parameter(b.clone()) for b in base]
    topt = torch.optim.AdamW([{"params": [ref[0], ref[2]]}, {"params": [ref[1], ref[3]], "lr": 5e-4}], lr=1e-3,
                             weight_decay=1e-2)
    for gs in grads:
        for p, g in zip(ref, gs):
            p.grad = g.clone()
        topt.step()
    # fused path (AdamW.use_device_schedule)
    ps = [torch.nn.Parameter(b.clone().to(dev)) for b in base]
    arena = ParamArena(ps[:3])
    opt = AdamW([ps[0], ps[2]], lr=1e-3, weight_decay=1e-2, arena=arena)
    opt.add_param_group({"params": [ps[1], ps[3]], "lr": 5e-4})  # ps[3] is not in the arena
    opt.use_device_schedule()
    for t, gs in enumerate(grads):
        for p, g in zip(ps, gs):
            p.grad = arena.grad_view(p) if arena.owns(p) else torch.empty_like(p)
            p.grad.copy_(g.to(dev))
        if t == 2:  # split step: everything but ps[0], then ps[0] alone
            opt.step(skip={id(ps[0])}, join_pending=False)
            opt.step(only={id(ps[0])}, sched_step=False)
        else:
            opt.step()
    # the separate schedule launch, by hand
    qs = [b.clone().to(dev) for b in base]
    mv = [(torch.zeros_like(q), torch.zeros_like(q)) for q in qs]
    scheds = [torch.tensor([lr] + [0.0] * 6, dtype=torch.float64, device=dev) for lr in (1e-3, 5e-4)]
    for gs in grads:
        for gi, idx in ((0, (0, 2)), (1, (1, 3))):
            ops.adamw_sched_step(scheds[gi], 0.9, 0.999)
            for k in idx:
                ops.adamw_dev(qs[k], gs[k].to(dev).reshape(-1).reshape(qs[k].shape), mv[k][0], mv[k][1], scheds[gi],
                              0.9, 0.999, 1e-8, 1e-2)
    torch.cuda.synchronize()
    assert opt.device_step_count(0) == 5 and opt.device_step_count(1) == 5
    for k in range(4):
        assert torch.equal(ps[k].detach().cpu(), qs[k].cpu()), k
        assert _rel(ps[k].detach(), ref[k].detach()) < 1e-6, k


@pytest.mark.parametrize("off", [0, 1, 2, 3])
def test_adamw_vector_body_bitwise(dev, off):
    """The AdamW kernels' 16-B vector body with its scalar head and tail (an
    arena run at any element offset) equals the all-scalar path (taken when
    the gradient's 16-B alignment differs from the parameter's) bit for bit,
    for the device-schedule and the host-schedule kernels, and torch.optim.AdamW
    to fp32 rounding, over 3 steps."""
    n = 40_003
    torch.manual_seed(4)
    base = torch.randn(n + 8)
    grads = [torch.randn(n) for _ in range(3)]

    def run(goff, dev_sched):
        P = base.clone().to(dev)
        M, V, G = (torch.zeros(n + 8, device=dev) for _ in range(3))
        p, m, v, g = P[off:off + n], M[off:off + n], V[off:off + n], G[goff:goff + n]
        sched = torch.tensor([1e-3] + [0.0] * 6, dtype=torch.float64, device=dev)
        for t, gr in enumerate(grads, 1):
            g.copy_(gr.to(dev))
            if dev_sched:
                ops.adamw_dev(p, g, m, v, sched, 0.9, 0.999, 1e-8, 1e-2, advance=True)
            else:
                ops.adamw(p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 1e-2, t)
        torch.cuda.synchronize()
        return p.cpu()

    ref = torch.nn.Parameter(base[off:off + n].clone())
    topt = torch.optim.AdamW([ref], lr=1e-3, weight_decay=1e-2)
    for gr in grads:
        ref.grad = gr.clone()
        topt.step()
    for dev_sched in (True, False):
        vec, sca = run(off, dev_sched), run(off + 1, dev_sched)
        assert torch.equal(vec, sca), dev_sched
        assert _rel(vec, ref.detach()) < 1e-6, dev_sched


@pytest.mark.parametrize("n", [5, 3 * 256 + 10])
def test_adamw_dev_advance_small_n(dev, n):
    """An advancing ssip_adamw_dev launch whose threads own at most one
    element (n < 256 * workgroups: most waves of a workgroup have no element
    and finish at once) advances t exactly once per launch, and every element
    is updated with that launch's bias corrections (the arrival
    count must wait for every wave's schedule read).  40 steps vs torch."""
    torch.manual_seed(3)
    p0 = torch.randn(n)
    ref = torch.nn.Parameter(p0.clone())
    topt = torch.optim.AdamW([ref], lr=1e-3, weight_decay=1e-2)
    p = p0.clone().to(dev)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    sched = torch.tensor([1e-3] + [0.0] * 6, dtype=torch.float64, device=dev)
    for _ in range(40):
        g = torch.randn(n)
        ref.grad = g.clone()
        topt.step()
        ops.adamw_dev(p, g.to(dev), m, v, sched, 0.9, 0.999, 1e-8, 1e-2, advance=True)
    torch.cuda.synchronize()
    s = sched.cpu()
    assert s[1].item() == 40.0 and s[4].item() == 0.0
    assert _rel(p, ref.detach()) < 1e-6


@pytest.mark.parametrize("dtname", ["f32", "bf16"])
def test_weight_prep_batch_layouts(dev, dtname):
    """Batched prep == the per-tensor layouts (exact): KRSC / CRSK, zero
    padding of the stem (C 3->4, S 7->8), ragged K/C (not multiples of 64)."""
    dt = torch.float32 if dtname == "f32" else torch.bfloat16
    torch.manual_seed(0)
    shapes = [(64, 3, 7, 7, 4, 8), (128, 64, 3, 3, 64, 3), (96, 40, 1, 1, 40, 1), (512, 256, 3, 3, 256, 3)]
    items, refs = [], []
    for K, C, R, S, Cp, Sp in shapes:
        w = torch.randn(K, C, R, S)
        pad = torch.zeros(K, Cp, R, Sp)
        pad[:, :C, :, :S] = w
        krsc_ref = pad.permute(0, 2, 3, 1).contiguous().to(dt)
        crsk_ref = pad.permute(1, 2, 3, 0).contiguous().to(dt)
        krsc = torch.full((K, R, Sp, Cp), float("nan"), device=dev, dtype=dt)
        crsk = torch.full((Cp, R, Sp, K), float("nan"), device=dev, dtype=dt)
        items.append((w.to(dev), Cp, Sp, krsc, crsk))
        refs.append((krsc_ref, crsk_ref, krsc, crsk))
    ops.weight_prep_batch(items, dt)
    torch.cuda.synchronize()
    for krsc_ref, crsk_ref, krsc, crsk in refs:
        assert torch.equal(krsc.cpu(), krsc_ref)
        assert torch.equal(crsk.cpu(), crsk_ref)


def test_weight_cache_follows_optimizer(dev):
    """The compute-dtype weight copies are refreshed after every optimizer
    step (version counter) and reused between steps."""
    from ssip import SSIPResNet
    from ssip.optim import AdamW
    torch.manual_seed(0)
    m = SSIPResNet("resnet18", num_classes=2, dtype="fp32").to(dev)
    arena = m.flatten_parameters()
    x = torch.randn(2, 3, 32, 32, device=dev)
    out = m(x)
    key = (id(m.conv1), m.compute_dtype)
    before = m._prep[key][0].clone()
    out.sum().backward()
    opt = AdamW(m.parameters(), lr=1e-2, arena=arena)
    opt.step()
    v = m.conv1.weight._version
    assert m._prep[key][2] != v
    m(x)
    assert m._prep[key][2] == v
    w = m.conv1.weight.detach()
    exp = torch.zeros(64, 7, 8, 4, device=dev)
    exp[:, :, :7, :3] = w.permute(0, 2, 3, 1)
    assert torch.equal(m._prep[key][0], exp)
    assert not torch.equal(before, exp)


@pytest.mark.parametrize("dtname", ["f32", "bf16"])
def test_stem_bn_pool_fused_matches_unfused(dev, dtname):
    """Fused stem BN->ReLU->max-pool forward is bit-identical to bn_apply +
    maxpool_fwd (values and argmax bytes); the fused backward matches
    maxpool_bwd + bn_bwd (f32 1e-5, bf16 2e-2: the unfused path rounds the
    scattered gradient to bf16 before the BN backward, the fused one keeps f32)."""
    dt = torch.float32 if dtname == "f32" else torch.bfloat16
    torch.manual_seed(0)
    N, H, W, C, k, s, pd = 3, 20, 18, 64, 3, 2, 1
    M = N * H * W
    y = torch.randn(N, H, W, C, device=dev).to(dt)
    mean = torch.randn(C, device=dev) * 0.1
    invstd = torch.rand(C, device=dev) + 0.5
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev) * 0.1
    scale = gamma * invstd
    shift = beta - mean * scale
    P, Q = (H + 2 * pd - k) // s + 1, (W + 2 * pd - k) // s + 1
    # unfused reference path
    z = torch.empty_like(y)
    ops.bn_apply(M, C, y, scale, shift, None, True, z)
    pool_r = torch.empty(N, P, Q, C, device=dev, dtype=dt)
    idx_r = torch.empty(N, P, Q, C, device=dev, dtype=torch.uint8)
    ops.maxpool_fwd(N, H, W, C, k, s, pd, z, pool_r, idx_r)
    # fused
    pool = torch.empty_like(pool_r)
    idx = torch.empty_like(idx_r)
    ymax = torch.empty_like(pool_r)
    ops.stem_bn_pool_fwd(N, H, W, C, k, s, pd, y, scale, shift, pool, idx, ymax)
    torch.cuda.synchronize()
    assert torch.equal(pool.cpu(), pool_r.cpu())
    assert torch.equal(idx.cpu(), idx_r.cpu())
    # ymax = y at each window's argmax (torch's first-max order)
    Hp, Wp = P, Q
    yp = torch.nn.functional.pad(y.float().permute(0, 3, 1, 2), (pd, pd, pd, pd))
    win = yp.unfold(2, k, s).unfold(3, k, s)[:, :, :Hp, :Wp].reshape(N, C, Hp, Wp, k * k)
    want = torch.gather(win, 4, idx.permute(0, 3, 1, 2).long().unsqueeze(-1)).squeeze(-1).permute(0, 2, 3, 1)
    assert torch.equal(ymax.float().cpu(), want.cpu())
    # backward
    dpool = torch.randn(N, P, Q, C, device=dev).to(dt)
    dz = torch.empty_like(y)
    ops.maxpool_bwd(N, H, W, C, k, s, pd, dpool, idx_r, dz)
    dy_r = torch.empty_like(y)
    dg_r = torch.empty(C, device=dev)
    db_r = torch.empty(C, device=dev)
    part = torch.empty(ops.bn_bwd_partial_floats(M, C), device=dev)
    coef = torch.empty(3 * C, device=dev)
    ops.bn_bwd(M, C, dz, z, y, mean, invstd, gamma, dg_r, db_r, False, dy_r, None, part, coef)
    dy = torch.empty_like(y)
    dg = torch.empty(C, device=dev)
    db = torch.empty(C, device=dev)
    part2 = torch.empty(ops.stem_pool_bn_bwd_partial_floats(N, H, W, C), device=dev)
    coef2 = torch.empty(3 * C, device=dev)
    tol = 1e-5 if dt == torch.float32 else 2e-2
    for ym in (None, ymax):  # full-resolution gather reduction / pooled-grid reduction
        ops.stem_pool_bn_bwd(N, H, W, C, k, s, pd, dpool, idx, y, mean, invstd, scale, shift, gamma, dg, db, False,
                             dy, part2, coef2, ym)
        torch.cuda.synchronize()
        assert _rel(dy, dy_r) < tol
        assert _rel(dg, dg_r) < tol
        assert _rel(db, db_r) < tol


@pytest.mark.parametrize("dtname", ["f32", "bf16"])
def test_bn_relu_bwd_affine_mask_matches_z_mask(dev, dtname):
    """ssip_bn_relu_bwd (mask from fma(y, scale, shift) > 0) is bit-identical to
    ssip_bn_bwd with the stored ReLU output as the mask."""
    dt = torch.float32 if dtname == "f32" else torch.bfloat16
    torch.manual_seed(1)
    M, C = 3000, 128
    y = torch.randn(M, C, device=dev).to(dt)
    dz = torch.randn(M, C, device=dev).to(dt)
    mean = torch.randn(C, device=dev) * 0.1
    invstd = torch.rand(C, device=dev) + 0.5
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev) * 0.1
    scale = gamma * invstd
    shift = beta - mean * scale
    z = torch.empty_like(y)
    ops.bn_apply(M, C, y, scale, shift, None, True, z)
    outs = []
    for affine in (False, True):
        dy = torch.empty_like(y)
        dg = torch.empty(C, device=dev)
        db = torch.empty(C, device=dev)
        part = torch.empty(ops.bn_bwd_partial_floats(M, C), device=dev)
        coef = torch.empty(3 * C, device=dev)
        if affine:
            ops.bn_relu_bwd(M, C, dz, y, mean, invstd, scale, shift, gamma, dg, db, False, dy, part, coef)
        else:
            ops.bn_bwd(M, C, dz, z, y, mean, invstd, gamma, dg, db, False, dy, None, part, coef)
        outs.append((dy.cpu(), dg.cpu(), db.cpu()))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)

