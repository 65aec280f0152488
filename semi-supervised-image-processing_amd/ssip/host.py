"""Host (CPU) execution of the frozen extraction pass, for the reference's
`--device cpu` (BASELINE config 1: `python -m src.feature_extraction
--device cpu --batch-size 32`; /root/reference/src/feature_extraction.py:
519-522 parses the flag, :542 builds the device, :184-207 the transform,
:210-227 the model, :289-293 the batched forward).

This is not a fallback: it runs only when the caller asks for the CPU
device, and the HIP path never routes here (SSIPResNet.forward on a CUDA
model calls the C ABI; on a CPU model without `host_forward` it raises).
It executes the product's own module tree -- the same SSIPResNet parameters
and buffers, the same eval-mode semantics -- with torch's CPU operators,
and the transform with the Pillow calls torchvision makes for a PIL image:

  Resize(256)     short side -> 256, long side int(256 * long / short),
                  Image.BILINEAR (torchvision functional_pil.resize)
  CenterCrop(224) top = int(round((h - 224) / 2)), left likewise
  ToTensor        uint8 HWC -> float CHW / 255
  Normalize       (t - mean) / std per channel
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch
import torch.nn.functional as F
from PIL import Image


def pil_extraction_transform(img: Image.Image, resize: int, crop: int, mean: Sequence[float],
                             std: Sequence[float]) -> torch.Tensor:
    """The reference's build_transform() on one PIL image -> float32 [3, crop, crop]."""
    w, h = img.size
    short, long = (w, h) if w <= h else (h, w)
    ns, nl = resize, int(resize * long / short)
    ow, oh = (ns, nl) if w <= h else (nl, ns)
    if (ow, oh) != (w, h):
        img = img.resize((ow, oh), Image.BILINEAR)
    top = int(round((oh - crop) / 2.0))
    left = int(round((ow - crop) / 2.0))
    img = img.crop((left, top, left + crop, top + crop))
    a = np.array(img, np.uint8, copy=True)
    if a.ndim == 2:
        a = a[:, :, None]
    t = torch.from_numpy(a).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    m = torch.as_tensor(mean, dtype=torch.float32).view(-1, 1, 1)
    s = torch.as_tensor(std, dtype=torch.float32).view(-1, 1, 1)
    return t.sub(m).div(s)


def _bn_eval(x: torch.Tensor, bn) -> torch.Tensor:
    return F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)


def _block(blk, x: torch.Tensor) -> torch.Tensor:
    """BasicBlock / Bottleneck in eval mode (torchvision's order of operations)."""
    idt = x
    convs = [(m, getattr(blk, "bn" + m[4:])) for m in ("conv1", "conv2", "conv3") if hasattr(blk, m)]
    out = x
    for i, (cname, bn) in enumerate(convs):
        conv = getattr(blk, cname)
        out = F.conv2d(out, conv.weight, None, conv.stride, conv.padding)
        out = _bn_eval(out, bn)
        if i < len(convs) - 1:
            out = F.relu(out)
    if blk.downsample is not None:
        ds_conv, ds_bn = blk.downsample[0], blk.downsample[1]
        idt = _bn_eval(F.conv2d(x, ds_conv.weight, None, ds_conv.stride, ds_conv.padding), ds_bn)
    return F.relu(out + idt)


@torch.no_grad()
def host_forward(model, x: torch.Tensor) -> torch.Tensor:
    """Eval-mode forward of an SSIPResNet whose parameters live on the CPU:
    [B,3,H,W] float32 -> the avgpool output [B, C, 1, 1] when
    model.embedding_only (the reference's children()[:-1]), else logits."""
    if model.training:
        raise RuntimeError("ssip host execution is the frozen eval pass only (feature extraction --device cpu)")
    c1 = model.conv1
    x = F.conv2d(x.to(torch.float32), c1.weight, None, c1.stride, c1.padding)
    x = F.relu(_bn_eval(x, model.bn1))
    x = F.max_pool2d(x, 3, 2, 1)
    for blk in model.blocks():
        x = _block(blk, x)
    feat = F.adaptive_avg_pool2d(x, (1, 1))
    if model.embedding_only:
        return feat
    return F.linear(feat.flatten(1), model.fc.weight, model.fc.bias)
