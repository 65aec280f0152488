"""The semi-supervised train step (north-star config 3/4): labelled batch +
unlabelled batch with a weak and a strong view and a FixMatch-style
consistency loss, entirely on the device.

Reference pieces it is built from (SURVEY.md §8a row a23 — the reference
itself trains offline pseudo-labels, it has no joint step):
  weak view     = the reference train transform (common.py:101-109)
  pseudo-label  = softmax -> max -> keep if >= tau (semi_supervised.py:57-66)
  loss          = nn.CrossEntropyLoss (semi_supervised.py:111)
  optimizer     = AdamW(lr, wd) (semi_supervised.py:115-122)

Step (per rank, B_l labelled + B_u unlabelled uint8 images resident in HBM):
  1. GPU augment: weak(labelled), weak(unlabelled), strong(unlabelled)
  2. weak forward over the unlabelled weak view: train-mode BN batch
     statistics, no running-stat update, no grad (pseudo-label source),
     on a second HIP stream, overlapping step 3
  3. one train forward over [labelled ; strong] (B_l + B_u images)
  4. ssip_semi_loss: CE(labelled) + lambda * mean_u[mask * CE(strong, pseudo)]
  5. backward (+ bucketed RCCL all-reduce when world > 1)
  6. fused AdamW over the flat arena
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch

from . import ops
from .augment import GpuTransform, draw_params_batch
from .optim import AdamW
from .resnet import DeviceImages, SSIPResNet


@dataclass
class StepStats:
    loss: torch.Tensor        # [4] total, L_l, L_u, mask count (device)


class SemiStep:
    def __init__(self, model: SSIPResNet, lr: float = 1e-4, weight_decay: float = 1e-4, tau: float = 0.7,
                 lambda_u: float = 1.0, image_size: int = 224, bucketer=None, seed: int = 0):
        self.model = model
        self.arena = model.flatten_parameters()
        self.opt = AdamW(model.parameters(), lr=lr, weight_decay=weight_decay, arena=self.arena)
        self.tau, self.lambda_u = tau, lambda_u
        self.size = image_size
        self.tf = GpuTransform(image_size, model.compute_dtype, "resize")
        self.bucketer = bucketer
        self.gen = torch.Generator().manual_seed(seed)
        if bucketer is not None:
            model.grad_ready_hook = bucketer.mark_ready
        self.overlap = True   # weak forward on a second HIP stream
        self._side = None

    def _side_stream(self, dev):
        if self._side is None:
            self._side = torch.cuda.Stream(device=dev)
        return self._side

    def draw_params(self, Bl: int, Bu: int):
        """Per-sample view parameters (host RNG, like a DataLoader worker)."""
        s = self.size
        return (draw_params_batch(Bl, s, False, self.gen).pin_memory(),
                draw_params_batch(Bu, s, False, self.gen).pin_memory(),
                draw_params_batch(Bu, s, True, self.gen).pin_memory())

    def __call__(self, x_l: torch.Tensor, y_l: torch.Tensor, x_u: torch.Tensor, params=None) -> StepStats:
        """x_l [Bl,H,W,3] u8, y_l [Bl] int64, x_u [Bu,H,W,3] u8 — all on the device."""
        m = self.model
        Bl, Bu = x_l.shape[0], x_u.shape[0]
        dev = x_l.device
        if params is None:
            params = self.draw_params(Bl, Bu)
        pl, pw, ps = (p.to(dev, non_blocking=True) for p in params)
        main = torch.cuda.current_stream(dev)
        S = self.size
        P = self.tf.pad
        m.train()
        # compute-dtype weights for both forwards, refreshed once, before the fork
        m.prepare_weights(need_t=True)
        # 2. weak view + weak forward on a side stream (batch-stat BN, no
        #    running update, no grad): it only meets the train forward at the
        #    loss, so the two latency-bound forwards overlap on the chip
        side = self._side_stream(dev) if self.overlap else main
        side.wait_stream(main)
        m.bn_update_running = False
        with torch.cuda.stream(side), torch.no_grad():
            xw = self.tf(x_u, pw)
            zw = m(xw)
        m.bn_update_running = True
        # 1+3. [labelled weak ; unlabelled strong] views and the joint train forward
        x_ls = torch.empty((Bl + Bu, S + 2 * P, S + 2 * P, 4), device=dev, dtype=m.compute_dtype)
        self.tf(x_l, pl, out=x_ls[:Bl])
        self.tf(x_u, ps, out=x_ls[Bl:])
        self.opt.zero_grad(set_to_none=True)
        if self.bucketer is not None:
            self.bucketer.reset()
        logits = m(DeviceImages(x_ls, P))
        if side is not main:
            main.wait_stream(side)
            zw.record_stream(main)
        # 4. loss + dlogits in one launch
        out, dzl, dzs, pseudo, mask = ops.semi_loss(logits[:Bl].detach().contiguous(), y_l,
                                                    zw.contiguous(), logits[Bl:].detach().contiguous(),
                                                    self.tau, self.lambda_u)
        # 5. backward
        logits.backward(torch.cat([dzl, dzs], 0))
        scale = self.bucketer.finish() if self.bucketer is not None else 1.0
        # 6. optimizer
        self.opt.step(grad_scale=scale)
        return StepStats(loss=out)
