"""GPU parity at BASELINE config 5's geometry: every distinct conv of the
ResNet-50 train step at 512x512, batch 128 per GPU (bottleneck 1x1 convs with
64-2048 channels, 3x3 convs at 128^2 / 64^2 / 32^2 / 16^2, the stride-2 3x3
convs and the 1x1 / stride-2 downsamples), forward, data gradient and weight
gradient, each through the production kernel that geometry selects (its name
is asserted to be an LDS-DMA / halo kernel, not the register-staged fallback).

Operands are bf16-rounded random tensors generated on the device; the oracle
is a float64 reference of the same op on those operands (torch matmul on the
device), evaluated on a sample of the outputs so every shape runs in well
under a second:
  fwd   : 4,096 random output pixels x all K channels (their im2col rows)
  dgrad : 4,096 random input pixels x all C channels (their dy neighbourhoods)
  wgrad : 8 output channels x all (c, r, s), full reduction over N*P*Q rows
Tolerances (as tests/test_gpu_bench_geometry.py): bf16 outputs
|y - ref| <= 2^-8 |ref| + 1e-4 max|ref| (one bf16 rounding of an fp32
accumulation); fp32 weight gradients max|dw - ref| <= 2e-4 max|ref|
(reductions over up to 2,097,152 rows, fp32 accumulation in another order).
"""
import pytest
import torch

from ssip import ops
from ssip.ops import ConvGeom

pytestmark = pytest.mark.gpu
N = 128
DT = torch.bfloat16
SAMPLES = 4096
# (C, H, K, R, stride, pad): the ResNet-50 v1.5 convs at 512x512 input (stem
# and max-pool: 128x128 into layer1)
CONVS = [
    ("l1.c1.in64", (64, 128, 64, 1, 1, 0)), ("l1.c2", (64, 128, 64, 3, 1, 1)),
    ("l1.c3/ds", (64, 128, 256, 1, 1, 0)), ("l1.c1", (256, 128, 64, 1, 1, 0)),
    ("l2.0.c1", (256, 128, 128, 1, 1, 0)), ("l2.0.c2s2", (128, 128, 128, 3, 2, 1)),
    ("l2.c3", (128, 64, 512, 1, 1, 0)), ("l2.0.ds", (256, 128, 512, 1, 2, 0)),
    ("l2.c1", (512, 64, 128, 1, 1, 0)), ("l2.c2", (128, 64, 128, 3, 1, 1)),
    ("l3.0.c1", (512, 64, 256, 1, 1, 0)), ("l3.0.c2s2", (256, 64, 256, 3, 2, 1)),
    ("l3.c3", (256, 32, 1024, 1, 1, 0)), ("l3.0.ds", (512, 64, 1024, 1, 2, 0)),
    ("l3.c1", (1024, 32, 256, 1, 1, 0)), ("l3.c2", (256, 32, 256, 3, 1, 1)),
    ("l4.0.c1", (1024, 32, 512, 1, 1, 0)), ("l4.0.c2s2", (512, 32, 512, 3, 2, 1)),
    ("l4.c3", (512, 16, 2048, 1, 1, 0)), ("l4.0.ds", (1024, 32, 2048, 1, 2, 0)),
    ("l4.c1", (2048, 16, 512, 1, 1, 0)), ("l4.c2", (512, 16, 512, 3, 1, 1)),
]


def _geom(C, H, K, R, st, pd):
    return ConvGeom(N, H, H, C, K, R, R, st, pd, C, R)


def _production(mode, g):
    name = ops.conv_kernel_name(mode, g, DT)
    assert name.startswith(("glds<", "halo<", "halo_wgrad<")), name
    return name


def _rand(shape, gen, scale=1.0):
    return (torch.randn(shape, device="cuda", generator=gen) * scale).to(DT)


def _check(got, ref, what):
    got, ref = got.double(), ref.double()
    bound = ref.abs() * 2.0 ** -8 + 1e-4 * ref.abs().max()
    over = ((got - ref).abs() - bound).max().item()
    assert over <= 0, f"{what}: worst element exceeds the bf16 rounding bound by {over:.3e}"


def _pixels(gen, n, h, w, count):
    idx = torch.randint(0, n * h * w, (count,), device="cuda", generator=gen)
    return idx // (h * w), (idx // w) % h, idx % w


@pytest.mark.parametrize("name,shape", CONVS, ids=[c[0] for c in CONVS])
def test_r50_fwd(dev, name, shape):
    C, H, K, R, st, pd = shape
    g = _geom(*shape)
    _production("fwd", g)
    gen = torch.Generator(device="cuda").manual_seed(11)
    x = _rand((N, H, H, C), gen)
    w = _rand((K, R, R, C), gen, (2.0 / (C * R * R)) ** 0.5)  # KRSC = the kernel's B operand
    y = torch.empty((N, g.P, g.Q, K), device=dev, dtype=DT)
    part = torch.empty(ops.conv_fwd_partial_floats(g), device=dev)
    ops.conv_fwd(g, x, w, y, part)
    n, p, q = _pixels(gen, N, g.P, g.Q, SAMPLES)
    xp = torch.nn.functional.pad(x.double(), (0, 0, pd, pd, pd, pd))
    rows = torch.stack([xp[n, p * st + r, q * st + s] for r in range(R) for s in range(R)], 1)  # [S, R*R, C]
    ref = rows.reshape(SAMPLES, -1) @ w.double().reshape(K, -1).T
    torch.cuda.synchronize()
    _check(y[n, p, q], ref, f"{name} fwd")


@pytest.mark.parametrize("name,shape", CONVS, ids=[c[0] for c in CONVS])
def test_r50_dgrad(dev, name, shape):
    C, H, K, R, st, pd = shape
    g = _geom(*shape)
    _production("dgrad", g)
    gen = torch.Generator(device="cuda").manual_seed(12)
    w = _rand((K, R, R, C), gen, (2.0 / (K * R * R)) ** 0.5)
    dy = _rand((N, g.P, g.Q, K), gen)
    crsk = w.permute(3, 1, 2, 0).contiguous()  # the dgrad's B operand [C][R][S][K]
    dx = torch.empty((N, H, H, C), device=dev, dtype=DT)
    ops.conv_dgrad(g, dy, crsk, dx, None)
    n, h, ww = _pixels(gen, N, H, H, SAMPLES)
    ref = torch.zeros(SAMPLES, C, device=dev, dtype=torch.float64)
    dyd, wd = dy.double(), w.double()
    for r in range(R):
        for s in range(R):
            ph, pw = h + pd - r, ww + pd - s
            ok = (ph % st == 0) & (pw % st == 0) & (ph >= 0) & (pw >= 0) & (ph // st < g.P) & (pw // st < g.Q)
            pi, qi = torch.where(ok, ph // st, 0), torch.where(ok, pw // st, 0)
            ref += (dyd[n, pi, qi] * ok[:, None]) @ wd[:, r, s, :]
    torch.cuda.synchronize()
    _check(dx[n, h, ww], ref, f"{name} dgrad")


@pytest.mark.parametrize("name,shape", CONVS, ids=[c[0] for c in CONVS])
def test_r50_wgrad(dev, name, shape):
    C, H, K, R, st, pd = shape
    g = _geom(*shape)
    _production("wgrad", g)
    gen = torch.Generator(device="cuda").manual_seed(13)
    x = torch.relu(_rand((N, H, H, C), gen))
    dy = _rand((N, g.P, g.Q, K), gen, 1e-2)
    ws = torch.empty(ops.conv_wgrad_workspace_bytes(g), device=dev, dtype=torch.uint8)
    dw = torch.full((K, C, R, R), float("nan"), device=dev)
    ops.conv_wgrad(g, dy, x, dw, False, ws)
    ks = torch.randperm(K, generator=torch.Generator().manual_seed(14))[:8].to(dev)
    xp = torch.nn.functional.pad(x.double(), (0, 0, pd, pd, pd, pd))
    dys = dy.double()[..., ks].reshape(-1, 8)  # [N*P*Q, 8]
    ref = torch.empty(8, C, R, R, device=dev, dtype=torch.float64)
    for r in range(R):
        for s in range(R):
            xs = xp[:, r: r + st * (g.P - 1) + 1: st, s: s + st * (g.Q - 1) + 1: st, :].reshape(-1, C)
            ref[:, :, r, s] = dys.T @ xs
    torch.cuda.synchronize()
    got = dw[ks].double()
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() <= 2e-4 * scale, name
