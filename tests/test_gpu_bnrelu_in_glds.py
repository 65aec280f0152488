"""GPU: the BN+ReLU-in convs on the LDS-DMA ring kernel (ssip_conv_fwd_bnrelu_in
/ ssip_conv_wgrad_bnrelu_in beyond the layer-1 halo geometry, round 6): the
ResNet-50 bottleneck's conv3 (1x1, stride 1) over relu(bn2(y2)) at BASELINE
config 5's geometry (512^2 input, batch 128 per GPU: the train forward's 64 +
64 images), and the 3x3 / stride-1 form (SSIP_BNRELU_GLDS bit 1) at ResNet-18
layer 2's batch-256 geometry.

Checked two ways:
  * bit for bit against ssip_bn_apply + the plain conv (outputs, BN partial
    records, weight gradient; the transform is bn_apply's arithmetic and the
    plan / k-order are the same);
  * against torch fp32 (conv2d / conv2d_weight) of bf16(relu(fma_f32(y, scale,
    shift))) on the CPU, at the bf16 rounding bound of test_gpu_bench_geometry
    (outputs) and 1e-4 max|ref| (weight gradients, fp32).
Reference model boundary: reference src/training/common.py:299-304 (the
torchvision model), the step at :380-382."""
import sys
from pathlib import Path

import pytest
import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).parent))
from ssip import ops  # noqa: E402
from ssip.ops import ConvGeom  # noqa: E402
from test_gpu_bench_geometry import _bn_affine, _bnrelu_ref, _check_bf16, _rnd  # noqa: E402

pytestmark = pytest.mark.gpu
DT = torch.bfloat16

# name, N, H, C, K, R (stride 1; pad (R - 1) / 2), SSIP_BNRELU_GLDS value
CASES = [
    ("r50.l1.conv3", 64, 128, 64, 256, 1, "1"),
    ("r50.l2.conv3", 128, 64, 128, 512, 1, "1"),
    ("r50.l3.conv3", 128, 32, 256, 1024, 1, "1"),
    ("r50.l4.conv3", 128, 16, 512, 2048, 1, "1"),
    ("r18.l2.conv2", 256, 28, 128, 128, 3, "3"),
]


@pytest.mark.parametrize("name,N,H,C,K,R,env", CASES, ids=[c[0] for c in CASES])
def test_glds_bnrelu_in_matches_apply_then_conv_and_torch(dev, monkeypatch, name, N, H, C, K, R, env):
    monkeypatch.setenv("SSIP_BNRELU_GLDS", env)
    # every shape, also those below the production row threshold
    monkeypatch.setenv("SSIP_BNRELU_GLDS_MINM", "0")
    # the plain wgrad on the budget's plain tiles, as the INBN form plans (the
    # wide SSIP_WGRAD_BIG tiles have no INBN form): the same splits, same bits
    monkeypatch.setenv("SSIP_WGRAD_BIG", "0")
    pd = (R - 1) // 2
    g = ConvGeom(N, H, H, C, K, R, R, 1, pd, C, R)
    assert ops.conv_bnrelu_in_supported(g, DT), name
    assert ops.conv_kernel_name("fwd", g, DT).startswith("glds<"), ops.conv_kernel_name("fwd", g, DT)
    gen = torch.Generator().manual_seed(200 + C)
    y = _rnd(torch.randn(N, C, H, H, generator=gen))
    scale, shift = _bn_affine(C, gen)
    w = _rnd(torch.randn(K, C, R, R, generator=gen) * (2.0 / (C * R * R)) ** 0.5)
    dy = _rnd(torch.randn(N, K, H, H, generator=gen) * 1e-2)
    yh = ops.nchw_to_nhwc(y.to(dev), C, DT)
    sc, sh = scale.to(dev), shift.to(dev)
    krsc = torch.empty((K, R, R, C), device=dev, dtype=DT)
    ops.weight_prep(w.to(dev), DT, C, R, krsc, None)
    dyh = ops.nchw_to_nhwc(dy.to(dev), K, DT)
    nparts = ops.conv_fwd_partial_floats(g)

    # fused: the conv over y with the transform in its ring
    out = torch.empty((N, H, H, K), device=dev, dtype=DT)
    part = torch.zeros(nparts, device=dev)
    ops.conv_fwd_bnrelu_in(g, yh, sc, sh, krsc, out, part)
    # 1x1: the same launch with z_out (the n-tile-0 workgroups store each
    # transformed piece: z must be bn_apply's output, bit for bit)
    zo = None
    if R == 1:
        zo = torch.full_like(yh, float("nan"))
        out_z, part_z = torch.empty_like(out), torch.zeros(nparts, device=dev)
        ops.conv_fwd_bnrelu_in(g, yh, sc, sh, krsc, out_z, part_z, z_out=zo)
    # apply pass + plain conv
    z = torch.empty_like(yh)
    ops.bn_apply(N * H * H, C, yh, sc, sh, None, True, z)
    out2 = torch.empty_like(out)
    part2 = torch.zeros(nparts, device=dev)
    ops.conv_fwd(g, z, krsc, out2, part2)
    from ssip.resnet import _side_wgrad_budget

    dws = {}
    for b in (0, _side_wgrad_budget(g, DT, dev)):
        ws = torch.empty(ops.conv_wgrad_workspace_bytes(g, b), device=dev, dtype=torch.uint8)
        d1 = torch.full((K, C, R, R), float("nan"), device=dev)
        ops.conv_wgrad_bnrelu_in(g, dyh, yh, sc, sh, d1, False, ws, max_workgroups=b)
        d2 = torch.full((K, C, R, R), float("nan"), device=dev)
        ops.conv_wgrad(g, dyh, z, d2, False, ws, b)
        dws[b] = (d1, d2)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), out2.view(torch.int16)), name
    assert torch.equal(part, part2), name
    if zo is not None:
        assert torch.equal(zo.view(torch.int16), z.view(torch.int16)), name
        assert torch.equal(out_z.view(torch.int16), out.view(torch.int16)) and torch.equal(part_z, part), name
    for b, (d1, d2) in dws.items():
        assert torch.equal(d1, d2), (name, b)
    # vs torch fp32 on the same bf16 operands
    zr = _bnrelu_ref(y, scale, shift)
    assert torch.equal(z.float().cpu().permute(0, 3, 1, 2), zr), name
    ref = F.conv2d(zr, w, padding=pd)
    _check_bf16(out, ref, f"{name} fwd")
    refw = torch.nn.grad.conv2d_weight(zr, (K, C, R, R), dy, padding=pd)
    scale_w = refw.abs().max().item()
    for b, (d1, _) in dws.items():
        assert (d1.cpu() - refw).abs().max().item() <= 1e-4 * scale_w, (name, b)
