"""Flat fp32 parameter/gradient arena.

All parameters of a model are re-homed into ONE contiguous device buffer
(``flat``) and their gradients into a parallel buffer (``grad``), in
``parameters()`` order.  This gives the fused AdamW kernel a single launch
over the whole model and lets data-parallel training all-reduce gradients
as a few large RCCL buckets instead of one call per tensor.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch


class ParamArena:
    def __init__(self, params: List[torch.nn.Parameter]):
        if not params:
            raise ValueError("ParamArena: no parameters")
        dev = params[0].device
        for p in params:
            if p.dtype != torch.float32 or p.device != dev:
                raise TypeError("ParamArena: all parameters must be fp32 on one device")
        self.params = list(params)
        total = sum(p.numel() for p in params)
        # padded to 64 floats: gradient buckets end on a 16-B multiple (RCCL
        # 2.26's ncclPreMulSum leaves a count % 4 tail unscaled, ssip/dist.py)
        self.padded = -(-total // 64) * 64
        self.flat = torch.zeros(self.padded, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(self.padded, device=dev, dtype=torch.float32)
        self.offsets: Dict[int, Tuple[int, int]] = {}
        off = 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                self.flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + n].view_as(p)
                if p.grad is not None:
                    self.grad[off:off + n].copy_(p.grad.reshape(-1))
                    p.grad = self.grad[off:off + n].view_as(p)
                self.offsets[id(p)] = (off, n)
                off += n
        self.numel = total
        # a side stream still writing into ``grad`` (the deferred stem wgrad of
        # SSIPResNet's backward); every consumer of the gradients or of the
        # parameters joins it first (join_pending)
        self.pending_side = None

    def join_pending(self) -> None:
        """Make the current stream wait for a side stream the last backward
        left unjoined, and forget it."""
        s, self.pending_side = self.pending_side, None
        if s is not None:
            from . import ops

            ops.wait_stream(torch.cuda.current_stream(s.device), s)

    def owns(self, p: torch.Tensor) -> bool:
        ent = self.offsets.get(id(p))
        if ent is None:
            return False
        return p.data_ptr() == self.flat.data_ptr() + 4 * ent[0]

    def valid(self) -> bool:
        return all(self.owns(p) for p in self.params)

    def span(self, p: torch.Tensor) -> Tuple[int, int]:
        return self.offsets[id(p)]

    def grad_view(self, p: torch.Tensor) -> torch.Tensor:
        off, n = self.offsets[id(p)]
        return self.grad[off:off + n].view_as(p)

    def attach_grads(self) -> None:
        """Point every param.grad at its arena slot (zeroed)."""
        self.grad.zero_()
        for p in self.params:
            p.grad = self.grad_view(p)
