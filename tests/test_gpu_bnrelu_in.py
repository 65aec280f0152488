"""GPU parity of the convs that take relu(bn(y)) of the layer below as their
input, formed in their LDS tile (ssip_conv_fwd_bnrelu_in /
ssip_conv_wgrad_bnrelu_in, ABI 13: the layer-1 halo kernels).

The transform repeats ssip_bn_apply's arithmetic (fma, ReLU, one bf16
rounding) on the halo tile's in-image pixels only -- the zero padding stays
zero -- so the output, the BN-statistics records and the weight gradient must
equal ssip_bn_apply followed by the plain conv bit for bit.  Scales of both
signs and shifts that push part of every channel below zero are drawn."""
import pytest
import torch

from ssip import ops
from ssip.ops import ConvGeom

pytestmark = pytest.mark.gpu

SHAPES = [
    # N, H, W (C = K = 64)
    (2, 56, 56),   # layer 1, TR = 4
    (5, 56, 56),   # tiles not a multiple of the workgroup count
    (2, 16, 16),   # one tile per image
    (3, 28, 28),   # TR = 7
]


def _inputs(N, H, W, dev, seed):
    torch.manual_seed(seed)
    g = ConvGeom(N, H, W, 64, 64, 3, 3, 1, 1, 64, 3)
    y_in = torch.randn(N, H, W, 64, device=dev).to(torch.bfloat16)
    scale = (torch.rand(64, device=dev) + 0.25) * torch.where(torch.rand(64, device=dev) < 0.2, -1.0, 1.0)
    shift = torch.randn(64, device=dev) * 0.5
    w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(torch.bfloat16)
    x = torch.empty_like(y_in)
    ops.bn_apply(N * H * W, 64, y_in, scale, shift, None, True, x)
    return g, y_in, scale, shift, w, x


@pytest.mark.parametrize("shape", SHAPES)
def test_fwd_bnrelu_in_equals_apply_then_conv(dev, shape):
    N, H, W = shape
    g, y_in, scale, shift, w, x = _inputs(N, H, W, dev, 21)
    assert ops.conv_bnrelu_in_supported(g, torch.bfloat16)
    assert ops.conv_kernel_name("fwd", g, torch.bfloat16).startswith("halo")
    nparts = ops.conv_fwd_partial_floats(g)
    ref_y = torch.empty(N, H, W, 64, device=dev, dtype=torch.bfloat16)
    ref_p = torch.zeros(nparts, device=dev)
    ops.conv_fwd(g, x, w, ref_y, ref_p)
    out_y = torch.full_like(ref_y, 7.0)
    out_p = torch.zeros(nparts, device=dev)
    ops.conv_fwd_bnrelu_in(g, y_in, scale, shift, w, out_y, out_p)
    torch.cuda.synchronize()
    assert torch.equal(out_y.view(torch.int16), ref_y.view(torch.int16))
    n = ops.conv_fwd_partial_tiles(g, torch.bfloat16) * 64 * 3
    assert torch.equal(out_p[:n], ref_p[:n])
    # z_out: the BN+ReLU output written by the conv, = bn_apply's, bit for bit;
    # the conv's own outputs unchanged
    z = torch.full_like(x, 9.0)
    out2 = torch.full_like(ref_y, 7.0)
    out_p2 = torch.zeros(nparts, device=dev)
    ops.conv_fwd_bnrelu_in(g, y_in, scale, shift, w, out2, out_p2, z_out=z)
    torch.cuda.synchronize()
    assert torch.equal(z.view(torch.int16), x.view(torch.int16))
    assert torch.equal(out2.view(torch.int16), ref_y.view(torch.int16))
    assert torch.equal(out_p2[:n], ref_p[:n])
    # the input tensor itself is not modified
    x2 = torch.empty_like(x)
    ops.bn_apply(N * H * W, 64, y_in, scale, shift, None, True, x2)
    assert torch.equal(x2.view(torch.int16), x.view(torch.int16))


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("budget", [0, 96])
def test_wgrad_bnrelu_in_equals_apply_then_wgrad(dev, shape, budget):
    N, H, W = shape
    g, y_in, scale, shift, w, x = _inputs(N, H, W, dev, 22)
    dy = torch.randn(N, H, W, 64, device=dev).to(torch.bfloat16)
    ws = torch.empty(ops.conv_wgrad_workspace_bytes(g, budget), device=dev, dtype=torch.uint8)
    ref = torch.empty(64, 64, 3, 3, device=dev)
    ops.conv_wgrad(g, dy, x, ref, False, ws, max_workgroups=budget)
    out = torch.full_like(ref, 3.0)
    ops.conv_wgrad_bnrelu_in(g, dy, y_in, scale, shift, out, False, ws, max_workgroups=budget)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    # accumulate
    acc = ref.clone()
    ops.conv_wgrad_bnrelu_in(g, dy, y_in, scale, shift, acc, True, ws, max_workgroups=budget)
    ref2 = ref.clone()
    ops.conv_wgrad(g, dy, x, ref2, True, ws, max_workgroups=budget)
    torch.cuda.synchronize()
    assert torch.equal(acc, ref2)


def test_bnrelu_in_rejects_other_geometries(dev):
    g = ConvGeom(2, 28, 28, 64, 128, 3, 3, 1, 1, 64, 3)  # a halo forward, but no halo wgrad (K = 128)
    assert not ops.conv_bnrelu_in_supported(g, torch.bfloat16)
    y_in = torch.zeros(2, 28, 28, 64, device=dev, dtype=torch.bfloat16)
    s = torch.ones(64, device=dev)
    w = torch.zeros(128, 3, 3, 64, device=dev, dtype=torch.bfloat16)
    y = torch.empty(2, 28, 28, 128, device=dev, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops.conv_fwd_bnrelu_in(g, y_in, s, s, w, y, None)
