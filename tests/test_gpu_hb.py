"""GPU parity of the row-balanced halo kernel (conv_hb_kernel, SSIP_HB=1):
the 3x3 / stride-1 convs of ResNet layers 2-4 at the benchmarked batch
(256; 128 for the weak forward), forward with its BatchNorm records and
dgrad with and without the in-place residual-gradient add, plus ragged
geometries (units that do not divide over the workgroups, tiles crossing
images).  Oracle and bounds as tests/test_gpu_bench_geometry.py: torch CPU
float32 on the bf16-rounded operands, |y - ref| <= 2^-8 |ref| + 1e-4 max|ref|.
"""
import os

import pytest
import torch
import torch.nn.functional as F

from ssip import ops
from test_gpu_bench_geometry import DT, _check_bf16, _geom, _rnd

pytestmark = pytest.mark.gpu

SHAPES = [("l2.3x3", (128, 28, 128, 3, 1, 1)), ("l3.3x3", (256, 14, 256, 3, 1, 1)),
          ("l4.3x3", (512, 7, 512, 3, 1, 1))]
RAGGED = [("r1", 3, (128, 9, 128, 3, 1, 1)), ("r2", 5, (192, 13, 256, 3, 1, 1)), ("r3", 2, (64 * 3, 30, 128, 3, 1, 1))]


@pytest.fixture
def hb():
    old = os.environ.get("SSIP_HB")
    os.environ["SSIP_HB"] = "1"
    yield
    if old is None:
        os.environ.pop("SSIP_HB")
    else:
        os.environ["SSIP_HB"] = old


def _fwd(dev, g, C, K, n, H, seed):
    gen = torch.Generator().manual_seed(seed)
    x = _rnd(torch.randn(n, C, H, H, generator=gen))
    w = _rnd(torch.randn(K, C, 3, 3, generator=gen) * (2.0 / (C * 9)) ** 0.5)
    ref = F.conv2d(x, w, stride=1, padding=1)
    xh = ops.nchw_to_nhwc(x.to(dev), C, DT)
    krsc = torch.empty((K, 3, 3, C), device=dev, dtype=DT)
    ops.weight_prep(w.to(dev), DT, C, 3, krsc, None)
    y = torch.empty((n, H, H, K), device=dev, dtype=DT)
    part = torch.full((ops.conv_fwd_partial_floats(g),), float("nan"), device=dev)
    ops.conv_fwd(g, xh, krsc, y, part)
    stats = torch.empty((4, K), device=dev)
    rm, rv = torch.zeros(K, device=dev), torch.ones(K, device=dev)
    ops.bn_finalize(K, ops.conv_fwd_partial_tiles(g, DT), part, torch.ones(K, device=dev), torch.zeros(K, device=dev),
                    rm, rv, 0.1, 1e-5, True, stats[0], stats[1], stats[2], stats[3])
    torch.cuda.synchronize()
    return y, ref, stats


def _check_stats(ref, stats, K, what):
    r = ref.double().permute(0, 2, 3, 1).reshape(-1, K)
    mean, var = r.mean(0), r.var(0, unbiased=False)
    m_got = stats[0].cpu().double()
    v_got = 1.0 / stats[1].cpu().double() ** 2 - 1e-5
    assert ((m_got - mean).abs().max() / var.sqrt().max()).item() < 1e-3, what
    assert ((v_got - var).abs().max() / var.max()).item() < 1e-3, what


def _dgrad(dev, g, C, K, n, H, seed):
    gen = torch.Generator().manual_seed(seed)
    w = _rnd(torch.randn(K, C, 3, 3, generator=gen) * (2.0 / (K * 9)) ** 0.5)
    dy = _rnd(torch.randn(n, K, H, H, generator=gen))
    add = _rnd(torch.randn(n, C, H, H, generator=gen))
    ref = torch.nn.grad.conv2d_input((n, C, H, H), w, dy, stride=1, padding=1)
    crsk = torch.empty((C, 3, 3, K), device=dev, dtype=DT)
    ops.weight_prep(w.to(dev), DT, C, 3, None, crsk)
    dyh = ops.nchw_to_nhwc(dy.to(dev), K, DT)
    dx = torch.empty((n, H, H, C), device=dev, dtype=DT)
    ops.conv_dgrad(g, dyh, crsk, dx, None)
    dx2 = ops.nchw_to_nhwc(add.to(dev), C, DT)
    ops.conv_dgrad(g, dyh, crsk, dx2, dx2)
    torch.cuda.synchronize()
    return dx, dx2, ref, add


@pytest.mark.parametrize("n", [256, 128], ids=["bs256", "weak128"])
@pytest.mark.parametrize("name,shape", SHAPES, ids=[s[0] for s in SHAPES])
def test_hb_fwd(dev, hb, name, shape, n):
    C, H, K = shape[0], shape[1], shape[2]
    g = _geom(*shape, n=n)
    assert ops.conv_kernel_name("fwd", g, DT).startswith("hb<fwd"), ops.conv_kernel_name("fwd", g, DT)
    y, ref, stats = _fwd(dev, g, C, K, n, H, 200)
    _check_bf16(y, ref, f"{name} hb fwd")
    _check_stats(ref, stats, K, f"{name} hb fwd stats")


@pytest.mark.parametrize("name,shape", SHAPES, ids=[s[0] for s in SHAPES])
def test_hb_dgrad(dev, hb, name, shape):
    C, H, K = shape[0], shape[1], shape[2]
    g = _geom(*shape, n=256)
    assert ops.conv_kernel_name("dgrad", g, DT).startswith("hb<dgrad"), ops.conv_kernel_name("dgrad", g, DT)
    dx, dx2, ref, add = _dgrad(dev, g, C, K, 256, H, 201)
    _check_bf16(dx, ref, f"{name} hb dgrad")
    _check_bf16(dx2, ref + add, f"{name} hb dgrad+add", pre_add=ref)


@pytest.mark.parametrize("name,n,shape", RAGGED, ids=[s[0] for s in RAGGED])
def test_hb_ragged(dev, hb, name, n, shape):
    """Geometries whose pixel count does not split evenly: ragged last tiles,
    tiles crossing image boundaries, column blocks split across workgroups."""
    C, H, K = shape[0], shape[1], shape[2]
    g = _geom(*shape, n=n)
    assert ops.conv_kernel_name("fwd", g, DT).startswith("hb<fwd"), ops.conv_kernel_name("fwd", g, DT)
    y, ref, stats = _fwd(dev, g, C, K, n, H, 202)
    _check_bf16(y, ref, f"{name} hb fwd")
    _check_stats(ref, stats, K, f"{name} hb fwd stats")
    gd = _geom(K, H, C, 3, 1, 1, n=n)  # dgrad of a conv with K in, C out: reduction over C (>= 128)
    assert ops.conv_kernel_name("dgrad", gd, DT).startswith("hb<dgrad"), ops.conv_kernel_name("dgrad", gd, DT)
    dx, dx2, ref2, add = _dgrad(dev, gd, K, C, n, H, 203)
    _check_bf16(dx, ref2, f"{name} hb dgrad")
    _check_bf16(dx2, ref2 + add, f"{name} hb dgrad+add", pre_add=ref2)
