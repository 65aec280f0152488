"""ResNet-18/50 on the ssip HIP kernels, behind the torchvision module API.

Reference boundary: `create_model` (src/training/common.py:299-304) returns a
torchvision ``resnet18`` whose ``fc`` is replaced by ``nn.Linear(512, C)``;
the train loop calls ``model(inputs)`` with f32 NCHW batches
(common.py:380), ``loss.backward()`` (:382) and ``optimizer.step()``
(:383); checkpoints are ``model.state_dict()`` (:418-424) with torchvision
key names; feature extraction uses ``children()[:-1]`` = everything up to
the global average pool (src/feature_extraction.py:210-227).

Design (MI355X-first):
  * The nn.Module tree below is a *parameter container* that mirrors
    torchvision's construction order exactly (same RNG consumption, same
    state_dict keys/shapes), so seeded initialisation and checkpoints are
    interchangeable with torchvision's.  Its submodules are never called.
  * ``forward`` runs the whole network as ONE autograd node whose forward
    and backward are sequences of C-ABI launches (libssip_hip.so) on NHWC
    activations in bf16 or f32; weight gradients are written straight into
    ``param.grad`` (views into one flat fp32 arena when the model is
    flattened for the fused optimizer / RCCL all-reduce).
  * BatchNorm semantics follow torch: train mode uses batch statistics and
    updates running stats (also in the frozen-backbone stage,
    src/training/semi_supervised.py:260-285), eval mode uses running stats.
"""
from __future__ import annotations

import os

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import ops
from .ops import ConvGeom

# ---------------------------------------------------------------------------
# parameter containers (torchvision-compatible structure and init order)
# ---------------------------------------------------------------------------


def _conv3x3(i, o, stride=1):
    return nn.Conv2d(i, o, kernel_size=3, stride=stride, padding=1, bias=False)


def _conv1x1(i, o, stride=1):
    return nn.Conv2d(i, o, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def stages(self):
        return [(self.conv1, self.bn1), (self.conv2, self.bn2)]

    def forward(self, x):  # pragma: no cover - containers are never executed
        raise RuntimeError("ssip blocks are parameter containers; call the top-level model")


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        width = planes
        self.conv1 = _conv1x1(inplanes, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = _conv3x3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = _conv1x1(width, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def stages(self):
        return [(self.conv1, self.bn1), (self.conv2, self.bn2), (self.conv3, self.bn3)]

    def forward(self, x):  # pragma: no cover
        raise RuntimeError("ssip blocks are parameter containers; call the top-level model")


ARCHS = {
    "resnet18": (BasicBlock, [2, 2, 2, 2]),
    "resnet34": (BasicBlock, [3, 4, 6, 3]),
    "resnet50": (Bottleneck, [3, 4, 6, 3]),
}

_DTYPES = {"fp32": torch.float32, "f32": torch.float32, "float32": torch.float32,
           "bf16": torch.bfloat16, "bfloat16": torch.bfloat16}


STEM_PAD = 3  # torchvision conv1 padding; the input producers pre-apply it
# dgrad epilogue + BN-backward reduction fusion (ssip_conv_dgrad_bn); see _backward.
# Default: where the dgrad runs on the halo kernel (layer 1: 3x3 / stride 1 / 64
# channels) and the BN below has no residual add; SSIP_FUSE_BN_BWD=halo: every
# halo dgrad, =1 everywhere, =0 nowhere.
_FUSE_BN_BWD = os.environ.get("SSIP_FUSE_BN_BWD", "")
_fuse_cache: dict = {}


def _fuse_bn_bwd(g: ConvGeom, dt: torch.dtype, residual: bool = False) -> bool:
    """residual: the BN below ends a block (mask bits + the identity gradient add)."""
    if _FUSE_BN_BWD in ("0", "1"):
        return _FUSE_BN_BWD == "1"
    if residual and _FUSE_BN_BWD != "halo":
        return False
    key = (g, dt)
    v = _fuse_cache.get(key)
    if v is None:
        v = _fuse_cache[key] = ops.conv_kernel_name("dgrad", g, dt).startswith("halo")
    return v


@dataclass
class DeviceImages:
    """A batch already in the stem's NHWC4 layout and the engine dtype
    (produced by ``ssip.augment``): skips the NCHW->NHWC conversion.

    ``buf`` is [B, H+2*pad, W+2*pad, 4] with a zero border of ``pad`` pixels:
    with pad == 3 (the stem conv's own padding) the stem runs as a pad-0 conv
    whose 16-byte pixel-pair loads are aligned and never straddle the border.
    """

    buf: torch.Tensor
    pad: int = 0

    @property
    def nhwc4(self) -> torch.Tensor:
        """The unpadded [B, H, W, 4] image (a view)."""
        p = self.pad
        if p == 0:
            return self.buf
        return self.buf[:, p:self.buf.shape[1] - p, p:self.buf.shape[2] - p, :]

    def __len__(self):
        return self.buf.shape[0]


class _Identity(nn.Module):
    def forward(self, x):
        return x


# ---------------------------------------------------------------------------
# saved forward state
# ---------------------------------------------------------------------------
@dataclass
class _ConvRec:
    geom: ConvGeom
    conv: nn.Conv2d
    bn: nn.BatchNorm2d
    x: torch.Tensor          # conv input  [N,H,W,C]
    y: torch.Tensor          # conv output [N,P,Q,K] (pre-BN)
    stats: torch.Tensor      # [4, K] mean, invstd, scale, shift
    z: Optional[torch.Tensor] = None   # post BN(+add)+ReLU output (mask source)
    zbits: Optional[torch.Tensor] = None  # its ReLU mask, one bit per element (the backward reads this, not z)
    # x is y of the BN+ReLU below and this conv forms relu(x * scale + shift)
    # in its LDS tile (ssip_conv_*_bnrelu_in): (scale, shift)
    in_bn: Optional[Tuple[torch.Tensor, torch.Tensor]] = None


@dataclass
class _Saved:
    dtype: torch.dtype
    N: int
    stem: _ConvRec = None
    pool_out: torch.Tensor = None
    pool_idx: torch.Tensor = None
    pool_ymax: torch.Tensor = None  # pre-BN y at each max-pool window's argmax (stem backward)
    pool_hw: Tuple[int, int] = (0, 0)
    blocks: List[Tuple[List[_ConvRec], Optional[_ConvRec], torch.Tensor]] = field(default_factory=list)
    feat: torch.Tensor = None
    logits: Optional[torch.Tensor] = None
    last: torch.Tensor = None
    last_pq: int = 0


class SSIPResNet(nn.Module):
    """torchvision-compatible ResNet whose compute runs on libssip_hip.so."""

    def __init__(self, arch: str = "resnet18", num_classes: int = 1000, dtype: str = "fp32"):
        super().__init__()
        block, layers = ARCHS[arch]
        self.arch = arch
        self.inplanes = 64
        self.dilation = 1
        self.groups = 1
        self.base_width = 64
        self.conv1 = nn.Conv2d(3, self.inplanes, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(self.inplanes)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        self.compute_dtype = _DTYPES[dtype]
        self.bn_update_running = True   # may be switched off for no-update batch-stat passes
        # (id(conv), dtype) -> [krsc, crsk or None, weight version they were made from]
        self._prep: Dict[Tuple[int, torch.dtype], list] = {}
        # (id(conv), dtype) -> [krsc with the eval BN folded in, bias, state stamp]
        self._fold: Dict[Tuple[int, torch.dtype], list] = {}
        self._bn_epoch = 0
        self._arena = None
        self.embedding_only = False
        # the CPU device was asked for (src.feature_extraction --device cpu):
        # a CPU model's eval forward runs ssip/host.py instead of raising
        self.host_execution = False
        # backward tail (single process, SemiStep): leave the stem wgrad (the
        # last kernel of the backward, on the wgrad side stream) unjoined; the
        # main stream only waits for the wgrads before it, so the optimizer
        # and the compute-dtype weight refresh of every other parameter overlap
        # it.  The caller must ops.wait_stream(main, model.take_pending_side())
        # before it reads conv1.weight.grad.
        self.defer_stem_wgrad_join = False
        self._pending_side = None
        # (single process, SemiStep) called once the backward has enqueued every
        # gradient of the blocks from `early_update_block` up and of the head:
        # early_update(stream that holds the last of those wgrads)
        self.early_update = None
        self.early_update_block = -1

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                _conv1x1(self.inplanes, planes * block.expansion, stride),
                nn.BatchNorm2d(planes * block.expansion),
            )
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    # ------------------------------------------------------------------
    def set_compute_dtype(self, dtype: str) -> "SSIPResNet":
        self.compute_dtype = _DTYPES[dtype]
        self._prep.clear()
        self._fold.clear()
        return self

    def blocks(self):
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            for b in layer:
                yield b

    def _apply(self, fn, *args, **kwargs):
        self._prep.clear()
        self._fold.clear()
        self._arena = None
        return super()._apply(fn, *args, **kwargs)

    # ------------------------------------------------------------------
    # flat parameter arena (fused optimizer / bucketed all-reduce)
    # ------------------------------------------------------------------
    def flatten_parameters(self):
        """Re-home every parameter (and its grad) into one contiguous fp32
        buffer, in ``named_parameters()`` order.  Idempotent."""
        from .arena import ParamArena

        if self._arena is None or not self._arena.valid():
            self._arena = ParamArena(list(self.parameters()))
        return self._arena

    def take_pending_side(self):
        """The side stream whose stem wgrad the last backward left unjoined
        (defer_stem_wgrad_join), or None; clears it."""
        s, self._pending_side = self._pending_side, None
        if self._arena is not None and self._arena.pending_side is s:
            self._arena.pending_side = None
        return s

    def join_pending_side(self) -> None:
        """The current stream waits for a stem wgrad left unjoined (no-op otherwise)."""
        s = self.take_pending_side()
        if s is not None:
            ops.wait_stream(torch.cuda.current_stream(s.device), s)

    def prepare_weights(self, need_t: bool = True, force: bool = False) -> None:
        """Refresh the compute-dtype conv weight copies now (one launch) so a
        later forward on another stream only reads them.  force: refresh all
        of them regardless of version (a captured step must always contain
        the refresh)."""
        _prepare_weights(self, need_t, force)

    # ------------------------------------------------------------------
    def forward(self, x):
        # a previous backward's deferred stem wgrad still writes conv1's grad
        self.join_pending_side()
        if isinstance(x, DeviceImages):
            images, pad = x.buf, x.pad
            if pad not in (0, self.conv1.padding[0]):
                images, pad = x.nhwc4, 0
            if images.dtype != self.compute_dtype or not images.is_contiguous():
                images = images.to(self.compute_dtype).contiguous()
        else:
            dev = self.conv1.weight.device
            if dev.type != "cuda":
                if self.host_execution:
                    # the frozen eval pass on the CPU, asked for explicitly
                    # (feature extraction --device cpu): ssip/host.py
                    from .host import host_forward

                    return host_forward(self, x)
                raise RuntimeError("SSIPResNet runs on the HIP device only; call model.to('cuda') first")
            x = x.to(dev, non_blocking=True)
            if x.dim() != 4 or x.shape[1] != 3:
                raise ValueError(f"expected a [B,3,H,W] batch, got {tuple(x.shape)}")
            pad = self.conv1.padding[0]
            images = ops.nchw_to_nhwc(x, 4, self.compute_dtype, pad=pad)
        params = [p for p in self.parameters()]
        if not (torch.is_grad_enabled() and any(p.requires_grad for p in params)):
            # inference (eval, pseudo-labelling, weak view, extraction): no autograd node, nothing saved
            sv = _forward(self, images, train=self.training, save=False, in_pad=pad)
            return sv.feat.view(sv.N, -1, 1, 1) if self.embedding_only else sv.logits
        return _NetFn.apply(self, images, pad, *params)


class _NetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model: SSIPResNet, images: torch.Tensor, in_pad: int, *params):
        train = model.training
        saved = _forward(model, images, train=train, save=train, in_pad=in_pad)
        ctx.model = model
        ctx.saved = saved
        out = saved.feat.view(saved.N, -1, 1, 1) if model.embedding_only else saved.logits
        if model.embedding_only:
            ctx.mark_non_differentiable(out)
        return out

    @staticmethod
    def backward(ctx, dlogits):
        model: SSIPResNet = ctx.model
        saved: _Saved = ctx.saved
        if saved is None or saved.stem is None or not model.training:
            raise RuntimeError("ssip: backward requires a train-mode forward with trainable parameters")
        _backward(model, saved, dlogits.contiguous().float())
        ctx.saved = None
        return (None, None, None) + (None,) * len(list(model.parameters()))


# ---------------------------------------------------------------------------
# forward engine
# ---------------------------------------------------------------------------
def _geom(conv: nn.Conv2d, N: int, H: int, W: int, in_pad: int = 0) -> ConvGeom:
    """in_pad: the input already carries a zero border of the conv's own
    padding (H, W include it) -> a pad-0 conv over the padded image."""
    K, C, R, S = conv.weight.shape
    stem = C == 3
    pad = conv.padding[0]
    if in_pad:
        assert in_pad == pad, "pre-padded input must carry exactly the conv padding"
        pad = 0
    return ConvGeom(N=N, H=H, W=W, C=4 if stem else C, K=K, R=R, S=8 if stem else S,
                    stride=conv.stride[0], pad=pad, c_real=C, s_real=S)


def _prepare_weights(model: SSIPResNet, need_t: bool, force: bool = False) -> None:
    """Refresh the compute-dtype KRSC (forward) and CRSK (data-gradient)
    copies of every conv weight whose fp32 master changed since the last
    refresh (torch version counter; ssip.optim.AdamW bumps it), in one
    batched launch — once per optimizer step, not once per forward."""
    dt = model.compute_dtype
    items = []
    for conv in model.modules():
        if not isinstance(conv, nn.Conv2d):
            continue
        w = conv.weight
        key = (id(conv), dt)
        ent = model._prep.get(key)
        if not force and ent is not None and ent[2] == w._version and (ent[1] is not None or not need_t):
            continue
        g = _geom(conv, 1, 1, 1)
        if ent is None or (need_t and ent[1] is None):
            krsc = torch.empty((g.K, g.R, g.S, g.C), device=w.device, dtype=dt)
            crsk = torch.empty((g.C, g.R, g.S, g.K), device=w.device, dtype=dt) if need_t else None
        else:
            krsc, crsk = ent[0], ent[1]
        model._prep[key] = [krsc, crsk, w._version]
        items.append((w.detach(), g.C, g.S, krsc, crsk))
    if items:
        ops.weight_prep_batch(items, dt)


def _prepped(model: SSIPResNet, conv: nn.Conv2d, g: ConvGeom, need_t: bool):
    ent = model._prep.get((id(conv), model.compute_dtype))
    if ent is None or ent[2] != conv.weight._version or (need_t and ent[1] is None):
        _prepare_weights(model, need_t)
        ent = model._prep[(id(conv), model.compute_dtype)]
    return ent


def _conv_bn(model: SSIPResNet, conv, bn, x: torch.Tensor, N, H, W, train: bool, save: bool,
             update_running: bool, in_pad: int = 0, in_bn=None) -> _ConvRec:
    """in_bn = (scale, shift): x is the pre-BN y of the BN+ReLU below, applied
    inside the conv (train mode, _bnrelu_in_ok geometries)."""
    g = _geom(conv, N, H, W, in_pad)
    dt = model.compute_dtype
    krsc = _prepped(model, conv, g, need_t=save)[0]
    y = torch.empty((N, g.P, g.Q, g.K), device=x.device, dtype=dt)
    stats = torch.empty((4, g.K), device=x.device, dtype=torch.float32)
    if train:
        nparts = ops.conv_fwd_partial_floats(g)
        partial = torch.empty(nparts, device=x.device, dtype=torch.float32)
        if in_bn is not None:
            # z_out: the halo forward writes it under SSIP_BNRELU_Z; a 1x1 conv
            # on the LDS-DMA ring always does (its in-ring wgrad transform sits
            # on the side stream's one-workgroup-per-CU grid and costs more
            # than the stores: profiles/r6_bnrelu_in_glds_lab.txt)
            one = g.R == 1 and g.S == 1
            z = torch.empty_like(x) if (save and (_BNRELU_Z or one)) else None
            ops.conv_fwd_bnrelu_in(g, x, in_bn[0], in_bn[1], krsc, y, partial, z_out=z)
            if z is not None:
                # the conv wrote relu(bn(x)) as it formed its tiles: the weight
                # gradient takes it as a plain input
                x, in_bn = z, None
        else:
            ops.conv_fwd(g, x, krsc, y, partial)
        ops.bn_finalize(g.K, ops.conv_fwd_partial_tiles(g, dt), partial, bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                        bn.running_var, bn.momentum if bn.momentum is not None else 0.1, bn.eps,
                        update_running, stats[0], stats[1], stats[2], stats[3])
    else:
        ops.conv_fwd(g, x, krsc, y, None)
        ops.bn_eval_coeffs(g.K, bn.weight.detach(), bn.bias.detach(), bn.running_mean, bn.running_var, bn.eps,
                           stats[0], stats[1], stats[2], stats[3])
    return _ConvRec(geom=g, conv=conv, bn=bn, x=x, y=y, stats=stats, in_bn=in_bn)


# BN+ReLU of a block's first conv applied inside its second conv (layer 1's
# halo geometry: ssip_conv_fwd_bnrelu_in / ssip_conv_wgrad_bnrelu_in) instead
# of a separate apply pass (SSIP_BNRELU_IN=0: the apply pass)
_BNRELU_IN = os.environ.get("SSIP_BNRELU_IN", "1") != "0"
# SSIP_BNRELU_Z=1: with a backward to follow, the conv also writes the BN+ReLU
# output (each row once, from the tiles it forms) so its weight gradient is the
# plain halo wgrad (the in-tile transform makes that one 50-100 us longer
# beside the main stream's layer-1 backward).  Measured 6.216 vs 6.196 ms
# (4 + 4): the forward's extra 103 MB of stores cost more.  Off by default.
_BNRELU_Z = os.environ.get("SSIP_BNRELU_Z", "0") == "1"


def _bnrelu_in_ok(conv, N: int, H: int, W: int, dtype) -> bool:
    return _BNRELU_IN and ops.conv_bnrelu_in_supported(_geom(conv, N, H, W), dtype)


def _conv_bn_ds(model: SSIPResNet, conv, bn, ds_conv, ds_bn, x: torch.Tensor, N, H, W, train: bool, save: bool,
                update_running: bool) -> Tuple[_ConvRec, _ConvRec]:
    """_conv_bn of a downsampling block's conv1 and of its 1x1 downsample in
    one fused launch (ops.conv_fwd_ds): same input, same output grid."""
    g = _geom(conv, N, H, W)
    gd = _geom(ds_conv, N, H, W)
    dt = model.compute_dtype
    krsc = _prepped(model, conv, g, need_t=save)[0]
    kds = _prepped(model, ds_conv, gd, need_t=save)[0]
    recs = []
    ys, parts, stats = [], [], []
    for gg in (g, gd):
        ys.append(torch.empty((N, gg.P, gg.Q, gg.K), device=x.device, dtype=dt))
        stats.append(torch.empty((4, gg.K), device=x.device, dtype=torch.float32))
        parts.append(torch.empty(ops.conv_fwd_partial_floats(gg), device=x.device, dtype=torch.float32)
                     if train else None)
    ops.conv_fwd_ds(g, x, krsc, ys[0], parts[0], gd, kds, ys[1], parts[1])
    tiles = (ops.conv_fwd_partial_tiles(g, dt), ops.conv_fwd_ds_partial_tiles(g, gd, dt))
    for gg, c, b, y, part, st, nt in zip((g, gd), (conv, ds_conv), (bn, ds_bn), ys, parts, stats, tiles):
        if train:
            ops.bn_finalize(gg.K, nt, part, b.weight.detach(), b.bias.detach(), b.running_mean, b.running_var,
                            b.momentum if b.momentum is not None else 0.1, b.eps, update_running, st[0], st[1],
                            st[2], st[3])
        else:
            ops.bn_eval_coeffs(gg.K, b.weight.detach(), b.bias.detach(), b.running_mean, b.running_var, b.eps,
                               st[0], st[1], st[2], st[3])
        recs.append(_ConvRec(geom=gg, conv=c, bn=b, x=x, y=y, stats=st))
    return recs[0], recs[1]


def _fwd_ds_fusable(blk, N: int, H: int, W: int) -> bool:
    """BasicBlock conv1 (3x3, pad 1, stride s) + downsample (1x1, stride s): ops.conv_fwd_ds."""
    if _NO_FWD_DS or blk.downsample is None or not isinstance(blk, BasicBlock):
        return False
    g = _geom(blk.conv1, N, H, W)
    gd = _geom(blk.downsample[0], N, H, W)
    return (g.R, g.S, g.pad, gd.R, gd.S, gd.pad, gd.stride) == (3, 3, 1, 1, 1, 0, g.stride) and \
        (g.P, g.Q, g.K, g.C) == (gd.P, gd.Q, gd.K, gd.C)


_NO_FWD_DS = os.environ.get("SSIP_NO_FWD_DSFUSE") == "1"


def _forward(model: SSIPResNet, images: torch.Tensor, train: bool, save: bool, in_pad: int = 0) -> _Saved:
    N, H, W, C4 = images.shape
    dt = model.compute_dtype
    upd = train and model.bn_update_running
    sv = _Saved(dtype=dt, N=N)
    dev = images.device
    _prepare_weights(model, need_t=save)
    # stem: conv 7x7/2 -> BN -> ReLU -> maxpool 3x3/2
    rec = _conv_bn(model, model.conv1, model.bn1, images, N, H, W, train, save, upd, in_pad)
    g = rec.geom
    mp = model.maxpool
    k, s, pd = mp.kernel_size, mp.stride, mp.padding
    Hp = (g.P + 2 * pd - k) // s + 1
    Wp = (g.Q + 2 * pd - k) // s + 1
    pool = torch.empty((N, Hp, Wp, g.K), device=dev, dtype=dt)
    # (argmax bytes only for a backward: the weak forward writes none)
    idx = torch.empty((N, Hp, Wp, g.K), device=dev, dtype=torch.uint8) if save else None
    # BN -> ReLU -> max-pool in one pass over y (the full-resolution z is never
    # stored).  (Round 5 measured the window selection inside the stem conv --
    # conv rows 2p-1..2p+1 per pooled row, BN + ReLU after on the pooled grid,
    # no y read -- at 429 us vs 164 + 180 for the two kernels: the per-element
    # selection and statistics VALU work inside the conv costs more than the
    # y read it saves; profiles/r5_stem_pool_lab.txt)
    ymax = torch.empty((N, Hp, Wp, g.K), device=dev, dtype=dt) if save else None
    ops.stem_bn_pool_fwd(N, g.P, g.Q, g.K, k, s, pd, rec.y, rec.stats[2], rec.stats[3], pool, idx, ymax)
    if save:
        sv.stem, sv.pool_out, sv.pool_idx, sv.pool_hw = rec, pool, idx, (g.P, g.Q)
        sv.pool_ymax = ymax
    x, Hc, Wc = pool, Hp, Wp
    fold = not train and _FOLD_EVAL_BN
    if fold:
        _prepare_folded(model)
    for blk in model.blocks():
        if fold:
            # eval mode: each conv carries its BN as scaled weights + bias, and the
            # ReLU / residual add run in the conv epilogue (no BN passes)
            ident = x
            if blk.downsample is not None:
                gd = _geom(blk.downsample[0], N, Hc, Wc)
                kr, b = model._fold[(id(blk.downsample[0]), dt)][:2]
                ident = torch.empty((N, gd.P, gd.Q, gd.K), device=dev, dtype=dt)
                ops.conv_fwd_bias(gd, x, kr, b, None, False, ident)
            z, h, w = x, Hc, Wc
            stages = blk.stages()
            for i, (conv, bn) in enumerate(stages):
                g = _geom(conv, N, h, w)
                kr, b = model._fold[(id(conv), dt)][:2]
                out = torch.empty((N, g.P, g.Q, g.K), device=dev, dtype=dt)
                ops.conv_fwd_bias(g, z, kr, b, ident if i == len(stages) - 1 else None, True, out)
                z, h, w = out, g.P, g.Q
            x, Hc, Wc = z, h, w
            continue
        recs = []
        z = x
        h, w = Hc, Wc
        stages = blk.stages()
        ds = None
        fuse_ds = _fwd_ds_fusable(blk, N, Hc, Wc)
        in_bn = None
        for i, (conv, bn) in enumerate(stages):
            if i == 0 and fuse_ds:
                r, ds = _conv_bn_ds(model, conv, bn, blk.downsample[0], blk.downsample[1], z, N, h, w, train, save,
                                    upd)
            else:
                r = _conv_bn(model, conv, bn, z, N, h, w, train, save, upd, in_bn=in_bn)
            in_bn = None
            h, w = r.geom.P, r.geom.Q
            if i < len(stages) - 1:
                if train and _bnrelu_in_ok(stages[i + 1][0], N, h, w, dt):
                    # the next conv applies this BN+ReLU itself; its input and
                    # its wgrad's stay the pre-BN y (the backward's mask comes
                    # from y and the affine, so z is never needed)
                    z, in_bn = r.y, (r.stats[2], r.stats[3])
                else:
                    zz = torch.empty_like(r.y)
                    ops.bn_apply(N * h * w, r.geom.K, r.y, r.stats[2], r.stats[3], None, True, zz)
                    r.z = zz
                    z = zz
            recs.append(r)
        last = recs[-1]
        out = torch.empty_like(last.y)
        # the backward masks with 1 bit per element instead of re-reading out
        bits = torch.empty(out.numel() // 8, device=dev, dtype=torch.uint8) if save else None
        if blk.downsample is not None:
            # out = relu(bn2(y2) + bn_ds(y_ds)): the downsample's BN is formed in
            # registers by the same pass (its output is never stored)
            if ds is None:
                ds = _conv_bn(model, blk.downsample[0], blk.downsample[1], x, N, Hc, Wc, train, save, upd)
            ops.bn_apply2(N * h * w, last.geom.K, last.y, last.stats[2], last.stats[3], ds.y, ds.stats[2],
                          ds.stats[3], True, out, bits)
        else:
            ops.bn_apply(N * h * w, last.geom.K, last.y, last.stats[2], last.stats[3], x, True, out, bits)
        last.z = out
        last.zbits = bits
        if save:
            sv.blocks.append((recs, ds, x))
        x, Hc, Wc = out, h, w
    C = x.shape[-1]
    feat = torch.empty((N, C), device=dev, dtype=torch.float32)
    if model.embedding_only:
        ops.avgpool_fc_fwd(N, Hc * Wc, C, 0, x, None, None, feat, None)
        sv.logits = None
    else:
        J = model.fc.out_features
        logits = torch.empty((N, J), device=dev, dtype=torch.float32)
        ops.avgpool_fc_fwd(N, Hc * Wc, C, J, x, model.fc.weight.detach(), model.fc.bias.detach(), feat, logits)
        sv.logits = logits
    sv.feat = feat
    sv.last, sv.last_pq = x, Hc * Wc
    if train and upd:
        _bump_batches_tracked(model)
        model._bn_epoch += 1  # running statistics changed on the device: folded eval weights are stale
    return sv


# eval-mode BatchNorm folded into the convs (SSIP_NO_BN_FOLD=1: separate BN passes, for A/B)
_FOLD_EVAL_BN = os.environ.get("SSIP_NO_BN_FOLD") != "1"


def _prepare_folded(model: SSIPResNet) -> None:
    """Refresh the eval-mode folded copies of every block conv: w' = w * s[k]
    (s = gamma / sqrt(running_var + eps)) in the compute dtype, bias = beta -
    running_mean * s.  One coefficient launch per stale BN plus one batched
    weight launch; reused until a weight, a BN parameter or the running
    statistics change (torch version counters, and model._bn_epoch for the
    device-side running-stat updates of a train-mode forward)."""
    dt = model.compute_dtype
    items = []
    for blk in model.blocks():
        pairs = list(blk.stages()) + ([(blk.downsample[0], blk.downsample[1])] if blk.downsample is not None else [])
        for conv, bn in pairs:
            w = conv.weight
            stamp = (w._version, bn.weight._version, bn.bias._version, bn.running_mean._version,
                     bn.running_var._version, model._bn_epoch)
            key = (id(conv), dt)
            ent = model._fold.get(key)
            if ent is not None and ent[2] == stamp:
                continue
            K, C, R, S = w.shape
            if ent is None:
                ent = [torch.empty((K, R, S, C), device=w.device, dtype=dt),
                       torch.empty(K, device=w.device, dtype=torch.float32), None]
                model._fold[key] = ent
            scale = torch.empty(K, device=w.device, dtype=torch.float32)
            ops.bn_eval_coeffs(K, bn.weight.detach(), bn.bias.detach(), bn.running_mean, bn.running_var, bn.eps,
                               None, None, scale, ent[1])
            ent[2] = stamp
            items.append((w.detach(), C, S, ent[0], None, scale))
    if items:
        ops.weight_prep_batch(items, dt)


def _bump_batches_tracked(model: SSIPResNet):
    """num_batches_tracked += 1 on every BN layer (torch's train-mode BN), one launch."""
    t = getattr(model, "_nbt", None)
    if t is None or (t and t[0].device != model.conv1.weight.device):
        t = [m.num_batches_tracked for m in model.modules()
             if isinstance(m, nn.BatchNorm2d) and m.num_batches_tracked is not None]
        model._nbt = t
    if t and t[0].is_cuda:
        ops.counters_add(t, 1)
    else:
        torch._foreach_add_(t, 1)


# ---------------------------------------------------------------------------
# backward engine
# ---------------------------------------------------------------------------
def _grad_target(p: torch.Tensor, arena) -> Tuple[torch.Tensor, bool]:
    """Tensor to write p's gradient into, and whether to accumulate."""
    if p.grad is None:
        if arena is not None and arena.owns(p):
            p.grad = arena.grad_view(p)
        else:
            p.grad = torch.empty_like(p)
        return p.grad, False
    return p.grad, True


# Weight gradients sit off the backward's critical path (dout -> BN backward ->
# dgrad -> next dout): they run on a second stream, forked from the main one
# before each wgrad and joined at the end of the backward, so the HBM- and
# latency-bound BN-backward passes and finalize launches overlap with them.
# WGRAD_SIDE_STREAM = False serialises everything on the current stream.
WGRAD_SIDE_STREAM = os.environ.get("SSIP_WGRAD_STREAM", "1") != "0"
# measurement only (bench.py's production roofline leg): keep the side
# stream's wgrad grid budgets when everything runs serialised on one stream
WGRAD_BUDGET_SERIAL = False
_side_streams = {}


_cus = {}


def _cu_count(dev: torch.device) -> int:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    n = _cus.get(idx)
    if n is None:
        n = _cus[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return n


_side_budgets = {}


_HALO_WG_FRAC = float(os.environ.get("SSIP_HALO_WG_FRAC", "0.5"))  # share of the CUs for the layer-1 wgrad


_LAST_WG_FULL = os.environ.get("SSIP_LAST_WG_FULL", "0") == "1"


def _side_wgrad_budget(g, dtype, dev: torch.device) -> int:
    """Grid cap of a wgrad on the side stream, beside the main stream's dgrad /
    BN-backward chain (ssip_conv_wgrad_budget): the split-K LDS-DMA wgrads one
    workgroup per CU (SSIP_WGRAD_BLOCKS sweep: 6.431 ms at 256 vs 6.490
    uncapped), the persistent layer-1 wgrad -- one workgroup per CU holding all
    of its LDS, so a main-stream kernel cannot start beside it -- half the CUs
    (6.551 vs 6.650 ms at 100 %, 6.567 at 62 %, 6.637 at 37 %; 3 alternated
    runs each, tools/gpu_r4_halo.sh)."""
    key = (g, dtype, dev.index)
    b = _side_budgets.get(key)
    if b is None:
        cus = _cu_count(dev)
        halo = ops.conv_kernel_name("wgrad", g, dtype).startswith("halo_wgrad")
        b = _side_budgets[key] = int(cus * _HALO_WG_FRAC) if halo else cus
    return b


def _wgrad_stream(dev: torch.device):
    if not WGRAD_SIDE_STREAM or dev.type != "cuda":
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _side_streams.get(idx)
    if st is None:
        st = _side_streams[idx] = torch.cuda.Stream(device=idx)
    return st


def _stage_params(model: SSIPResNet):
    """(trunk parameters, per-stage parameter lists: stem, then each block),
    cached on the model (the module tree is fixed; requires_grad is read
    from the parameters at every call)."""
    st = getattr(model, "_stage_params_cache", None)
    if st is None:
        stages = [[model.conv1, model.bn1]] + [[m for m in b.modules() if m is not b] for b in model.blocks()]
        per = [[p for m in mods for p in m.parameters(recurse=False)] for mods in stages]
        st = ([p for ps in per for p in ps], per)
        object.__setattr__(model, "_stage_params_cache", st)
    return st


def _backward(model: SSIPResNet, sv: _Saved, dlogits: torch.Tensor):
    side = _wgrad_stream(dlogits.device)
    if side is None:
        _backward_impl(model, sv, dlogits, None, None)
        return
    main = torch.cuda.current_stream(dlogits.device)
    model._pending_side = None
    deferred = False
    try:
        deferred = _backward_impl(model, sv, dlogits, main, side)
    finally:
        if deferred:
            model._pending_side = side
            if model._arena is not None:
                model._arena.pending_side = side  # AdamW.step / zero_grad join it
        else:
            ops.wait_stream(main, side)


def _backward_impl(model: SSIPResNet, sv: _Saved, dlogits: torch.Tensor, main, side):
    dt = sv.dtype
    N = sv.N
    arena = model._arena if (model._arena is not None and model._arena.valid()) else None
    dev = dlogits.device
    fc = model.fc
    C = sv.last.shape[-1]
    J = fc.out_features
    # which stages need input gradients: anything downstream of the first trainable layer
    trunk_params, stage_params = _stage_params(model)
    trunk_trainable = any(p.requires_grad for p in trunk_params)
    fc_w = fc.weight
    dw = db = None
    accw = accb = False
    if fc_w.requires_grad:
        dw, accw = _grad_target(fc_w, arena)
    if fc.bias is not None and fc.bias.requires_grad:
        db, accb = _grad_target(fc.bias, arena)
    user_hook = getattr(model, "grad_ready_hook", None)
    hook = None
    if user_hook is not None and side is None:
        def hook(params):
            ops.host_callback(user_hook, params)
    elif user_hook is not None:
        def _on_side(params):
            # the hook's consumers (gradient buckets) order themselves after
            # the current stream: make that the side stream, joined to main
            side.wait_stream(main)
            with torch.cuda.stream(side):
                user_hook(params)

        def hook(params):
            ops.host_callback(_on_side, params)
    if not trunk_trainable:
        if dw is not None:
            ops.avgpool_fc_bwd(dt, N, sv.last_pq, C, J, dlogits, fc_w.detach(), sv.feat, None, dw,
                               db, accw)
        if hook is not None:
            hook(list(fc.parameters()))
        return
    dz = torch.empty_like(sv.last)
    if dw is not None and db is not None and accw != accb:
        raise RuntimeError("ssip: fc weight/bias grads must both be fresh or both accumulate")
    ops.avgpool_fc_bwd(dt, N, sv.last_pq, C, J, dlogits, fc_w.detach(), sv.feat, dz, dw, db, accw)
    if hook is not None:
        hook(list(fc.parameters()))

    # earliest trainable stage decides where dgrad can stop
    first_trainable = None
    for i, ps in enumerate(stage_params):
        if any(p.requires_grad for p in ps):
            first_trainable = i
            break

    ws_bytes = 0
    budgeted = side is not None or WGRAD_BUDGET_SERIAL
    for r in [r for recs, ds, _ in sv.blocks for r in recs + ([ds] if ds is not None else [])] + [sv.stem]:
        ws_bytes = max(ws_bytes, ops.conv_wgrad_workspace_bytes(r.geom))
        if budgeted:  # the side stream's grids may take more split slabs (ABI 12)
            ws_bytes = max(ws_bytes, ops.conv_wgrad_workspace_bytes(r.geom, _side_wgrad_budget(r.geom, dt, dev)))
    workspace = torch.empty(ws_bytes, device=dev, dtype=torch.uint8)
    coef_buf = torch.empty(6 * 2048, device=dev, dtype=torch.float32)

    def bn_grads(rec: _ConvRec):
        bn = rec.bn
        dgam = dbet = None
        acc = False
        if bn.weight.requires_grad:
            dgam, acc = _grad_target(bn.weight, arena)
        if bn.bias.requires_grad:
            dbet, acc2 = _grad_target(bn.bias, arena)
            if dgam is not None and acc2 != acc:
                raise RuntimeError("ssip: BN weight/bias grads must both be fresh or both accumulate")
            acc = acc2
        return dgam, dbet, acc

    def bn_backward(rec: _ConvRec, dzin, zmask, dpre=None, mbits=None):
        """BN(+ReLU) backward with its own reduction pass; the ReLU mask from
        zmask (z > 0) or from the forward's mask bits."""
        g = rec.geom
        M = N * g.P * g.Q
        dgam, dbet, acc = bn_grads(rec)
        dy = torch.empty_like(rec.y)
        partial = torch.empty(ops.bn_bwd_partial_floats(M, g.K), device=dev, dtype=torch.float32)
        ops.bn_bwd(M, g.K, dzin, zmask, rec.y, rec.stats[0], rec.stats[1], rec.bn.weight.detach(), dgam, dbet, acc,
                   dy, dpre, partial, coef_buf[: 3 * g.K], mbits)
        return dy

    def bn_relu_backward(rec: _ConvRec, dzin):
        """BN+ReLU (no residual) backward; the mask comes from y and the BN
        affine, so z is not read."""
        g = rec.geom
        M = N * g.P * g.Q
        dgam, dbet, acc = bn_grads(rec)
        dy = torch.empty_like(rec.y)
        partial = torch.empty(ops.bn_bwd_partial_floats(M, g.K), device=dev, dtype=torch.float32)
        ops.bn_relu_bwd(M, g.K, dzin, rec.y, rec.stats[0], rec.stats[1], rec.stats[2], rec.stats[3],
                        rec.bn.weight.detach(), dgam, dbet, acc, dy, partial, coef_buf[: 3 * g.K])
        return dy

    def bn_backward_fused(rec: _ConvRec, dpre, partial, tiles):
        """BN backward whose reduction came out of the dgrad epilogue that
        produced dpre (already ReLU-masked)."""
        g = rec.geom
        M = N * g.P * g.Q
        dgam, dbet, acc = bn_grads(rec)
        dy = torch.empty_like(rec.y)
        ops.bn_bwd_from_partials(M, g.K, tiles, partial, dpre, rec.y, rec.stats[0], rec.stats[1],
                                 rec.bn.weight.detach(), dgam, dbet, acc, dy, coef_buf[: 3 * g.K])
        return dy

    def bn_backward_dual(rec_a: _ConvRec, rec_b: _ConvRec, dzin, zmask, mbits=None):
        """Backward of z = relu(BN_a(y_a) + BN_b(y_b)) in one reduction and one
        apply pass (the masked gradient that feeds both is never stored);
        None when the two BNs' gradients do not both accumulate or both start fresh."""
        g = rec_a.geom
        M = N * g.P * g.Q
        ga, ba, acc_a = bn_grads(rec_a)
        gb, bb, acc_b = bn_grads(rec_b)
        if (ga is not None or ba is not None) and (gb is not None or bb is not None) and acc_a != acc_b:
            return None
        acc = acc_a if (ga is not None or ba is not None) else acc_b
        dya = torch.empty_like(rec_a.y)
        dyb = torch.empty_like(rec_b.y)
        partial = torch.empty(ops.bn_bwd_dual_partial_floats(M, g.K), device=dev, dtype=torch.float32)
        ops.bn_bwd_dual(M, g.K, dzin, zmask, rec_a.y, rec_a.stats[0], rec_a.stats[1], rec_a.bn.weight.detach(), ga,
                        ba, rec_b.y, rec_b.stats[0], rec_b.stats[1], rec_b.bn.weight.detach(), gb, bb, acc, dya, dyb,
                        partial, coef_buf[: 6 * g.K], mbits)
        return dya, dyb

    def conv_wgrad(rec: _ConvRec, dy, last: bool = False):
        w = rec.conv.weight
        if not w.requires_grad:
            return
        tgt, acc = _grad_target(w, arena)
        if rec.in_bn is not None:
            budget = _side_wgrad_budget(rec.geom, dy.dtype, dev) if (side is not None or WGRAD_BUDGET_SERIAL) else 0
            if last and _LAST_WG_FULL:
                budget = 0
            if side is not None:
                ops.wait_stream(side, main)
            with torch.cuda.stream(side if side is not None else main):
                ops.conv_wgrad_bnrelu_in(rec.geom, dy, rec.x, rec.in_bn[0], rec.in_bn[1], tgt, acc, workspace,
                                         max_workgroups=budget)
            if side is not None:
                dy.record_stream(side)
            return
        if side is None:
            ops.conv_wgrad(rec.geom, dy, rec.x, tgt, acc, workspace,
                           max_workgroups=_side_wgrad_budget(rec.geom, dy.dtype, dev) if WGRAD_BUDGET_SERIAL else 0)
            return
        # (round 5: holding a block's wgrads behind one event at its end -- 8
        # event records instead of 19 -- made the step 3 % slower: the side
        # stream idles while they wait)
        ops.wait_stream(side, main)
        with torch.cuda.stream(side):
            ops.conv_wgrad(rec.geom, dy, rec.x, tgt, acc, workspace,
                           max_workgroups=0 if (last and _LAST_WG_FULL) else _side_wgrad_budget(rec.geom, dy.dtype, dev))
        dy.record_stream(side)

    def conv_dgrad(rec: _ConvRec, dy, out, add=None):
        crsk = _prepped_t(model, rec)[1]
        ops.conv_dgrad(rec.geom, dy, crsk, out, add)

    def conv_dgrad_bn(rec: _ConvRec, dy, below: _ConvRec, out, add=None, residual: bool = False):
        """dgrad of `rec` fused with the ReLU mask + BN-backward reduction of
        `below` (the BN+ReLU whose output is rec's input): the mask from the
        forward's mask bits where `below` ends a block (its ReLU follows the
        residual add), else from y and below's BN affine.  Only where
        _fuse_bn_bwd says so (the halo dgrads by default: the implicit-GEMM
        epilogue costs more than the reduce pass it replaces)."""
        if not _fuse_bn_bwd(rec.geom, dt, residual):
            conv_dgrad(rec, dy, out, add)
            return None
        crsk = _prepped_t(model, rec)[1]
        partial = torch.empty(ops.conv_dgrad_bn_partial_floats(rec.geom), device=dev, dtype=torch.float32)
        if residual:
            zm, bits, msc, msh = (None, below.zbits, None, None) if below.zbits is not None else (below.z, None, None, None)
        else:
            zm, bits, msc, msh = None, None, below.stats[2], below.stats[3]
        ops.conv_dgrad_bn(rec.geom, dy, crsk, add, zm, below.y, below.stats[0], below.stats[1], out, partial,
                          mask_bits=bits, mscale=msc, mshift=msh)
        return out, partial, ops.conv_dgrad_bn_partial_tiles(rec.geom, dt)

    nblocks = len(sv.blocks)
    blocks = list(model.blocks())
    pending = None  # (dpre, partial, tiles) of the current block's last BN, from the block above
    for bi in range(nblocks - 1, -1, -1):
        recs, ds, xin = sv.blocks[bi]
        stage_idx = bi + 1
        need_dx = first_trainable is not None and first_trainable < stage_idx
        below = sv.blocks[bi - 1][0][-1] if bi > 0 else None  # BN+ReLU producing this block's input
        last = recs[-1]
        dual = None
        zm, zb = (None, last.zbits) if last.zbits is not None else (last.z, None)
        if pending is None and ds is not None:
            dual = bn_backward_dual(last, ds, dz, zm, zb)
        dpre = None
        if dual is not None:
            dy, dy_ds = dual
        else:
            if pending is None:
                dpre = torch.empty_like(last.y)
                dy = bn_backward(last, dz, zm, dpre, zb)
            else:
                dpre, part, tiles = pending
                dy = bn_backward_fused(last, dpre, part, tiles)
            dy_ds = bn_backward(ds, dpre, None) if ds is not None else None
        pending = None
        # main path, last conv back to the first
        ds_dgrad_done = False
        g_cur = dy
        dxin = None
        for i in range(len(recs) - 1, -1, -1):
            r = recs[i]
            # the trunk's last wgrad (the first block's first conv) runs beside
            # only the stem's BN-backward reduction
            conv_wgrad(r, g_cur, last=(bi == 0 and i == 0 and ds is None))
            if i > 0:
                dzp = torch.empty_like(r.x)
                fused = conv_dgrad_bn(r, g_cur, recs[i - 1], dzp)
                if fused is None:
                    g_cur = bn_relu_backward(recs[i - 1], dzp)
                else:
                    g_cur = bn_backward_fused(recs[i - 1], *fused)
            elif need_dx:
                dxin = torch.empty_like(xin)
                if ds is None and below is not None:
                    pending = conv_dgrad_bn(r, g_cur, below, dxin, dpre, residual=True)
                elif ds is None:
                    conv_dgrad(r, g_cur, dxin, dpre)
                elif _ds_dgrad_fusable(r.geom, ds.geom) and (below is None or not _fuse_bn_bwd(ds.geom, dt, True)):
                    # conv1's and the downsample's input gradients in one launch
                    ops.conv_dgrad_ds(r.geom, g_cur, _prepped_t(model, r)[1], ds.geom, dy_ds,
                                      _prepped_t(model, ds)[1], dxin)
                    ds_dgrad_done = True
                else:
                    conv_dgrad(r, g_cur, dxin)
        if ds is not None:
            conv_wgrad(ds, dy_ds)
            if dxin is not None and not ds_dgrad_done:
                if below is not None:
                    pending = conv_dgrad_bn(ds, dy_ds, below, dxin, dxin, residual=True)
                else:
                    conv_dgrad(ds, dy_ds, dxin, dxin)
        if hook is not None:
            hook(list(blocks[bi].parameters()))
        if model.early_update is not None and bi == model.early_update_block:
            model.early_update(side if side is not None else main)
        dz = dxin
        if dz is None:
            return
    # stem: maxpool backward -> BN/ReLU backward -> conv1 wgrad
    stem = sv.stem
    P1, Q1 = sv.pool_hw
    mp = model.maxpool
    # max-pool backward + ReLU mask + BN backward straight from the pooled gradient
    C1 = stem.geom.K
    dgam, dbet, acc = bn_grads(stem)
    partial = torch.empty(ops.stem_pool_bn_bwd_partial_floats(N, P1, Q1, C1), device=dev, dtype=torch.float32)
    w1 = stem.conv.weight
    # the stem wgrad forms the BN-backward dy per tile in LDS (no full-resolution
    # dy pass) where the geometry allows: ssip_stem_bwd_wgrad
    fused = (w1.requires_grad and (mp.kernel_size, mp.stride, mp.padding) == (3, 2, 1)
             and ops.stem_bwd_wgrad_supported(stem.geom, dt))
    defer = bool(fused and side is not None and hook is None and model.defer_stem_wgrad_join)
    dy1 = None if fused else torch.empty_like(stem.y)
    coef1 = coef_buf[: 3 * C1] if not fused else torch.empty(3 * C1, device=dev, dtype=torch.float32)
    ops.stem_pool_bn_bwd(N, P1, Q1, C1, mp.kernel_size, mp.stride, mp.padding, dz, sv.pool_idx, stem.y,
                         stem.stats[0], stem.stats[1], stem.stats[2], stem.stats[3], stem.bn.weight.detach(), dgam,
                         dbet, acc, dy1, partial, coef1, sv.pool_ymax)
    if fused:
        tgt, acc_w = _grad_target(w1, arena)
        args = (stem.geom, dz, sv.pool_idx, stem.y, stem.x, stem.stats[2], stem.stats[3], coef1, tgt, acc_w,
                workspace)
        if side is None:
            ops.stem_bwd_wgrad(*args)
        else:
            ops.wait_stream(side, main)
            if defer:
                # main waits for every wgrad queued so far, not for this one
                ops.wait_stream(main, side)
            with torch.cuda.stream(side):
                ops.stem_bwd_wgrad(*args)
            # every tensor the side-stream kernel reads or writes was allocated
            # on main: keep the caching allocator from handing any of them to a
            # main-stream allocation before the join (deferred: after this returns)
            for t in (dz, sv.pool_idx, stem.y, stem.x, stem.stats, coef1, workspace):
                t.record_stream(side)
    else:
        defer = False
        conv_wgrad(stem, dy1)
    if hook is not None:
        hook([model.conv1.weight, model.bn1.weight, model.bn1.bias])
    return defer



def _ds_dgrad_fusable(g: ConvGeom, gds: ConvGeom) -> bool:
    """conv1 and the downsample of a block read the same input and produce the
    same output grid (BasicBlock): ssip_conv_dgrad_ds takes both."""
    return (gds.R == 1 and gds.S == 1 and gds.pad == 0 and gds.stride == g.stride
            and (g.N, g.H, g.W, g.C, g.K, g.P, g.Q) == (gds.N, gds.H, gds.W, gds.C, gds.K, gds.P, gds.Q))


def _prepped_t(model: SSIPResNet, rec: _ConvRec):
    return _prepped(model, rec.conv, rec.geom, need_t=True)


# ---------------------------------------------------------------------------
# factory helpers
# ---------------------------------------------------------------------------
def resnet(arch: str = "resnet18", num_classes: int = 1000, dtype: str = "fp32") -> SSIPResNet:
    return SSIPResNet(arch, num_classes=num_classes, dtype=dtype)


def replace_fc(model: SSIPResNet, num_classes: int) -> SSIPResNet:
    """`model.fc = nn.Linear(in_features, num_classes)` as create_model does
    (src/training/common.py:299-304) — consumes the torch RNG identically."""
    model.fc = nn.Linear(model.fc.in_features, num_classes)
    return model
