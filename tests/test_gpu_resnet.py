"""GPU parity of the whole ResNet train step (forward, CE, backward, BN
running stats) against the oracle torchvision restatement on CPU.
Tolerances (relative to max |ref| per tensor): f32 path 1e-4 on logits and
1e-3 on gradients; bf16 path 5e-2 on logits and 1e-1 on gradients."""
import copy

import pytest
import torch

from oracle.torchvision_restate.torchvision import models as tvm
from ssip import SSIPResNet, replace_fc

pytestmark = pytest.mark.gpu


def _relerr(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _pair(arch="resnet18", ncls=2, seed=0, dtype="fp32"):
    torch.manual_seed(seed)
    ref = tvm.resnet18() if arch == "resnet18" else tvm.resnet50()
    ref.fc = torch.nn.Linear(ref.fc.in_features, ncls)
    torch.manual_seed(seed)
    mine = SSIPResNet(arch, num_classes=1000, dtype=dtype)
    replace_fc(mine, ncls)
    return ref, mine


def test_init_matches_torchvision_restatement():
    ref, mine = _pair()
    sd_r, sd_m = ref.state_dict(), mine.state_dict()
    assert list(sd_r.keys()) == list(sd_m.keys())
    for k in sd_r:
        assert torch.equal(sd_r[k], sd_m[k]), k


def _cos(a, b):
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


def _rel_l2(a, b):
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _bf16_step_check(arch, seed, x, y, dev, grad_floor=2e-2):
    """bf16 engine train step vs the float64 oracle, every tolerance derived
    from the same oracle run under bf16-storage emulation (oracle/bf16_emulate:
    bf16 conv inputs / weights / outputs and activation gradients, the
    engine's rounding points).  At random init a bf16 ResNet is chaotic in its
    ReLU masks (a CPU probe: perturbing the emulated run's input by 1e-6 moves
    its gradient errors as much as bf16 itself), so per-tensor gradients of
    ANY bf16 implementation are far from fp64 (median rel-L2 0.34 for R18,
    1.2 for R50): the bound is statistical, "no worse than the emulation":
      logits       max-abs err <= max(2 * emulated, 1e-3 max|ref|)
      gradients    median rel-L2 <= max(2 * emulated median, grad_floor),
                   worst  rel-L2 <= max(3 * emulated worst, grad_floor)
      BN running   max-abs err <= max(3 * emulated, 1e-3 max|ref|)
    The tight bf16 checks are per op (test_gpu_conv.py, test_gpu_bench_geometry.py)."""
    import statistics

    from oracle.bf16_emulate import emulate_bf16

    ref, mine = _pair(arch=arch, seed=seed, dtype="bf16")
    mine = mine.to(dev).train()
    outs = {}
    for kind in ("f64", "emu"):
        m = copy.deepcopy(ref).double().train()
        if kind == "emu":
            emulate_bf16(m)
        o = m(x.double())
        torch.nn.functional.cross_entropy(o, y).backward()
        outs[kind] = (o.detach(), {n: p.grad.clone() for n, p in m.named_parameters()},
                      {n: b.clone() for n, b in m.named_buffers()})
    out_m = mine(x.to(dev))
    torch.nn.functional.cross_entropy(out_m, y.to(dev)).backward()
    torch.cuda.synchronize()
    (o64, g64, b64), (oem, gem, bem) = outs["f64"], outs["emu"]
    err = (out_m.detach().cpu().double() - o64).abs().max().item()
    tol = max(2 * (oem - o64).abs().max().item(), 1e-3 * o64.abs().max().item())
    print(f"{arch} logits: gpu {err:.3e}, bound {tol:.3e}")
    assert err <= tol, (err, tol)
    e_gpu, e_emu = [], []
    for name, p in mine.named_parameters():
        assert p.grad is not None, name
        e_gpu.append(_rel_l2(p.grad, g64[name]))
        e_emu.append(_rel_l2(gem[name], g64[name]))
    med_g, med_e = statistics.median(e_gpu), statistics.median(e_emu)
    print(f"{arch} gradient rel-L2: gpu median {med_g:.3e} worst {max(e_gpu):.3e}; "
          f"emulated median {med_e:.3e} worst {max(e_emu):.3e}")
    assert med_g <= max(2 * med_e, grad_floor)
    assert max(e_gpu) <= max(3 * max(e_emu), grad_floor)
    for n, b in mine.named_buffers():
        if b.dtype.is_floating_point:
            eg = (b.detach().cpu().double() - b64[n]).abs().max().item()
            ee = (bem[n] - b64[n]).abs().max().item()
            assert eg <= max(3 * ee, 1e-3 * b64[n].abs().max().item()), n
        else:
            assert torch.equal(b.cpu(), b64[n]), n


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_train_step_matches_oracle(dev, dtype):
    """Whole train step vs the float64 oracle.

    fp32: logits and the fc gradients are checked tightly.  Trunk gradients
    pass through ReLU masks: at batch 8 x 3x3 (layer4) a single
    pre-activation within ~1e-5 of zero that lands on the other side of the
    mask moves a channel's sum by 1/72, so the trunk is checked by cosine
    similarity plus a loose max-error bound (cos > 0.9999, rel-max < 0.1).
    bf16: tolerances derived from the bf16-storage emulation of the oracle
    (_bf16_step_check)."""
    torch.manual_seed(123)
    x = torch.randn(8, 3, 96, 96)
    y = torch.tensor([0, 1, 1, 0, 1, 0, 0, 1])
    if dtype == "bf16":
        _bf16_step_check("resnet18", 0, x, y, dev)
        return
    ref, mine = _pair(dtype=dtype)
    ref64 = copy.deepcopy(ref).double()
    mine = mine.to(dev)
    for m in (ref64, mine):
        m.train()
    out_64 = ref64(x.double())
    torch.nn.functional.cross_entropy(out_64, y).backward()
    out_m = mine(x.to(dev))
    torch.nn.functional.cross_entropy(out_m, y.to(dev)).backward()
    torch.cuda.synchronize()
    named_64 = dict(ref64.named_parameters())
    assert _relerr(out_m, out_64) < 1e-4
    for n in ("fc.weight", "fc.bias"):
        assert _relerr(dict(mine.named_parameters())[n].grad, named_64[n].grad) < 1e-4
    for name, p in mine.named_parameters():
        assert p.grad is not None, name
        assert _cos(p.grad, named_64[name].grad) > 0.9999, name
        assert _relerr(p.grad, named_64[name].grad) < 0.1, name
    for (n1, b1), (n2, b2) in zip(ref64.named_buffers(), mine.named_buffers()):
        assert n1 == n2
        if b1.dtype.is_floating_point:
            assert _relerr(b2, b1) < 1e-4, n1
        else:
            assert torch.equal(b1, b2.cpu()), n1


def test_resnet18_bf16_224_bs32(dev):
    """bf16 train step at the benchmark's image size (224x224), batch 32."""
    torch.manual_seed(7)
    x = torch.randn(32, 3, 224, 224)
    y = torch.randint(0, 2, (32,))
    _bf16_step_check("resnet18", 1, x, y, dev)


def test_resnet50_bf16_train_step(dev):
    """BASELINE config 5's backbone in bf16 (the throughput dtype): batch 8
    at 128x128 against the float64 oracle, emulation-derived tolerances."""
    torch.manual_seed(11)
    x = torch.randn(8, 3, 128, 128)
    y = torch.tensor([0, 1, 1, 0, 1, 0, 0, 1])
    _bf16_step_check("resnet50", 3, x, y, dev)


def test_eval_and_embedding(dev):
    ref, mine = _pair()
    # make running stats non-trivial
    for m in list(ref.modules()):
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.5, 1.5)
    mine.load_state_dict(ref.state_dict())
    mine = mine.to(dev).eval()
    ref.eval()
    x = torch.randn(5, 3, 96, 96)
    with torch.no_grad():
        lr = ref(x)
        lm = mine(x.to(dev))
        fr = torch.nn.Sequential(*list(ref.children())[:-1])(x).flatten(1)
        mine.embedding_only = True
        fm = mine(x.to(dev)).flatten(1)
        mine.embedding_only = False
    assert _relerr(lm, lr) < 1e-4
    assert _relerr(fm, fr) < 1e-4


def test_frozen_backbone_only_fc_grads(dev):
    ref, mine = _pair()
    mine = mine.to(dev).train()
    for n, p in mine.named_parameters():
        if not n.startswith("fc"):
            p.requires_grad = False
    for n, p in ref.named_parameters():
        if not n.startswith("fc"):
            p.requires_grad = False
    x = torch.randn(3, 3, 64, 64)
    y = torch.tensor([1, 0, 1])
    torch.nn.functional.cross_entropy(ref(x), y).backward()
    torch.nn.functional.cross_entropy(mine(x.to(dev)), y.to(dev)).backward()
    for n, p in mine.named_parameters():
        if n.startswith("fc"):
            assert _relerr(p.grad, dict(ref.named_parameters())[n].grad) < 1e-3
        else:
            assert p.grad is None
    # running stats still updated in frozen-backbone train mode (reference quirk)
    assert _relerr(mine.bn1.running_mean, ref.bn1.running_mean) < 1e-3


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fused_bn_backward_path_matches(dev, dtype, monkeypatch):
    """The dgrad-epilogue BN-backward fusion (ssip_conv_dgrad_bn +
    ssip_bn_bwd_from_partials) gives the same gradients as the separate
    reduction pass (only the summation order differs)."""
    import ssip.resnet as R
    torch.manual_seed(5)
    x = torch.randn(4, 3, 64, 64)
    y = torch.randint(0, 2, (4,))
    grads = []
    # "0": separate reduce passes; "1": fused wherever possible; "": the
    # default policy (fused on the halo dgrads only)
    for fuse in ("0", "1", ""):
        monkeypatch.setattr(R, "_FUSE_BN_BWD", fuse)
        _, mine = _pair(dtype=dtype)
        mine = mine.to(dev).train()
        out = mine(x.to(dev))
        torch.nn.functional.cross_entropy(out.float(), y.to(dev)).backward()
        torch.cuda.synchronize()
        grads.append({k: p.grad.detach().cpu().clone() for k, p in mine.named_parameters()})
    tol = 1e-4 if dtype == "fp32" else 5e-2
    for gr in grads[1:]:
        for k in grads[0]:
            assert _cos(grads[0][k], gr[k]) > (0.99999 if dtype == "fp32" else 0.99), k
            assert _relerr(gr[k], grads[0][k]) < tol, k


def test_resnet50_train_step_matches_oracle(dev):
    """BASELINE config 5's backbone (Bottleneck blocks, 1x1 convs, stride-2
    in the 3x3) through the same engine: fp32 train step vs the float64
    torchvision restatement (same tolerances as the ResNet-18 test)."""
    ref, mine = _pair(arch="resnet50", ncls=2, seed=3)
    ref64 = copy.deepcopy(ref).double()
    ref32 = copy.deepcopy(ref)
    mine = mine.to(dev)
    for m in (ref64, ref32, mine):
        m.train()
    torch.manual_seed(9)
    x = torch.randn(4, 3, 64, 64)
    y = torch.tensor([0, 1, 1, 0])
    out_64 = ref64(x.double())
    torch.nn.functional.cross_entropy(out_64, y).backward()
    torch.nn.functional.cross_entropy(ref32(x), y).backward()
    out_m = mine(x.to(dev))
    torch.nn.functional.cross_entropy(out_m, y.to(dev)).backward()
    torch.cuda.synchronize()
    assert _relerr(out_m, out_64) < 1e-4
    named_64 = dict(ref64.named_parameters())
    named_32 = dict(ref32.named_parameters())
    # 53 ReLU masks deep with BN over 16 values per channel in layer4 (2x2 at
    # batch 4), some gradients are ill-conditioned in fp32 itself: the CPU
    # fp32 restatement reaches only cos 0.9994 vs fp64 on layer4.1.bn1.bias.
    # Bound the HIP fp32 path's angle to fp64 by 4x the CPU fp32 one (floor 1e-3).
    for name, p in mine.named_parameters():
        assert p.grad is not None, name
        cpu_err = 1.0 - _cos(named_32[name].grad, named_64[name].grad)
        assert 1.0 - _cos(p.grad, named_64[name].grad) <= max(1e-3, 4.0 * cpu_err), name
