"""Eval-mode BatchNorm folded into the convs: ssip_conv_fwd_bias
(y = act(conv(x, w * s) + bias (+ residual))) per kernel family against torch,
and the folded eval forward of the whole network against the unfolded one and
the fp64 oracle, including the refresh after the running statistics change.

Reference semantics: torchvision BatchNorm2d in eval mode (running statistics)
inside model(inputs) at src/training/common.py:333 (evaluate_on_loader),
semi_supervised.py:59 (pseudo-labels) and feature_extraction.py:291.
Tolerances at each assert: f32 rel 1e-5 per op / 1e-4 whole net vs fp64;
bf16 per op: half an ulp of the stored output plus the residual's rounding.
"""
import pytest
import torch
import torch.nn.functional as F

from oracle.torchvision_restate.torchvision import models as tvm
from ssip import SSIPResNet, replace_fc, ops, resnet
from ssip.ops import ConvGeom

pytestmark = pytest.mark.gpu

# name, (N, C, H, K, R, stride, pad), kernel prefix (bf16)
SHAPES = [
    ("l1.halo", (8, 64, 56, 64, 3, 1, 1), "halo<fwd"),
    ("l2.3x3", (16, 128, 28, 128, 3, 1, 1), "glds<fwd"),
    ("l3.s2", (16, 128, 28, 256, 3, 2, 1), "glds<fwd"),
    ("l4.ds", (8, 256, 14, 512, 1, 2, 0), "glds<fwd"),
]


@pytest.mark.parametrize("dtname", ["bf16", "f32"])
@pytest.mark.parametrize("res,relu", [(True, True), (False, True), (False, False)])
@pytest.mark.parametrize("name,shape,kern", SHAPES, ids=[s[0] for s in SHAPES])
def test_conv_fwd_bias(dev, name, shape, kern, res, relu, dtname):
    dt = torch.bfloat16 if dtname == "bf16" else torch.float32
    N, C, H, K, R, st, pd = shape
    g = ConvGeom(N, H, H, C, K, R, R, st, pd, C, R)
    if dt == torch.bfloat16:
        assert ops.conv_kernel_name("fwd", g, dt).startswith(kern), ops.conv_kernel_name("fwd", g, dt)
    gen = torch.Generator().manual_seed(11)
    x = torch.randn(N, C, H, H, generator=gen).to(dt).float()
    w = torch.randn(K, C, R, R, generator=gen) * (2.0 / (C * R * R)) ** 0.5
    s = torch.rand(K, generator=gen) + 0.5
    b = torch.randn(K, generator=gen) * 0.3
    r = torch.randn(N, K, g.P, g.Q, generator=gen).to(dt).float()
    krsc = torch.empty((K, R, R, C), device=dev, dtype=dt)
    ops.weight_prep_batch([(w.to(dev), C, R, krsc, None, s.to(dev))], dt)
    wf = (w * s.view(K, 1, 1, 1)).to(dt).float()  # the folded weight as the kernel stores it
    ref = F.conv2d(x.double(), wf.double(), stride=st, padding=pd) + b.double().view(1, K, 1, 1)
    pre = ref.clone()
    if res:
        ref = ref + r.double()
    if relu:
        ref = ref.clamp_min(0)
    y = torch.full((N, g.P, g.Q, K), float("nan"), device=dev, dtype=dt)
    ops.conv_fwd_bias(g, ops.nchw_to_nhwc(x.to(dev), C, dt), krsc, b.to(dev),
                      ops.nchw_to_nhwc(r.to(dev), K, dt) if res else None, relu, y)
    torch.cuda.synchronize()
    got = y.double().cpu()
    refh = ref.permute(0, 2, 3, 1)
    preh = pre.permute(0, 2, 3, 1).abs()
    if dt == torch.float32:
        bound = 1e-5 * refh.abs().max() + 0 * refh
    else:  # conv+bias rounded once, + residual rounded again
        bound = 2.0 ** -8 * (refh.abs() + (preh if res else 0)) + 1e-4 * refh.abs().max()
    over = ((got - refh).abs() - bound).max().item()
    assert over <= 0, f"{name}: exceeds the bound by {over:.3e}"


def _pair(dtype):
    torch.manual_seed(0)
    ref = tvm.resnet18()
    ref.fc = torch.nn.Linear(512, 2)
    for m in ref.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.1, 0.1)
    mine = SSIPResNet("resnet18", num_classes=1000, dtype=dtype)
    replace_fc(mine, 2)
    mine.load_state_dict(ref.state_dict())
    return ref.eval(), mine


@pytest.mark.parametrize("dtname", ["fp32", "bf16"])
def test_folded_eval_forward(dev, dtname, monkeypatch):
    ref, mine = _pair(dtname)
    mine = mine.to(dev).eval()
    x = torch.randn(6, 3, 112, 112)
    with torch.no_grad():
        want = ref.double()(x.double())
        folded = mine(x.to(dev))
        monkeypatch.setattr(resnet, "_FOLD_EVAL_BN", False)
        plain = mine(x.to(dev))
        monkeypatch.setattr(resnet, "_FOLD_EVAL_BN", True)
    rel = lambda a, b: ((a.double().cpu() - b.double().cpu()).abs().max() / b.double().cpu().abs().max()).item()
    if dtname == "fp32":
        assert rel(folded, want) < 1e-4 and rel(folded, plain) < 1e-5
    else:
        assert rel(folded, want) < 5e-2 and rel(plain, want) < 5e-2

    # a train-mode forward updates the running statistics on the device: the
    # folded copies must follow (model._bn_epoch), as must a state_dict load
    mine.train()
    with torch.no_grad():
        mine(torch.randn(4, 3, 112, 112).to(dev))
    mine.eval()
    with torch.no_grad():
        folded2 = mine(x.to(dev))
        monkeypatch.setattr(resnet, "_FOLD_EVAL_BN", False)
        plain2 = mine(x.to(dev))
        monkeypatch.setattr(resnet, "_FOLD_EVAL_BN", True)
    assert rel(plain2, plain) > 1e-6, "running statistics did not change"
    tol = 1e-5 if dtname == "fp32" else 5e-2
    assert rel(folded2, plain2) < tol
    mine.load_state_dict(ref.state_dict())
    with torch.no_grad():
        folded3 = mine(x.to(dev))
    assert rel(folded3, folded) < (1e-6 if dtname == "fp32" else 1e-3)
