"""Fused AdamW (torch.optim.AdamW semantics) on the flat parameter arena.

Drop-in for ``optim.AdamW(params, lr, weight_decay)`` as built by the
reference (src/training/semi_supervised.py:115-122, 265-272, 291-298;
src/training/supervised.py:71-78).  Parameters that live in a
``ParamArena`` are updated by ONE ``ssip_adamw`` launch per contiguous run
of trainable parameters; any other parameter gets its own launch.  The
state layout (``step``, ``exp_avg``, ``exp_avg_sq`` per parameter) and
``param_groups`` match torch's, so ``ReduceLROnPlateau`` and
``state_dict()`` work unchanged.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Tuple

import torch
from torch.autograd.graph import increment_version

from . import ops


class AdamW(torch.optim.Optimizer):
    def __init__(self, params: Iterable, lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 1e-2, arena=None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.arena = arena
        self._flat_state = None  # (exp_avg_flat, exp_avg_sq_flat) parallel to arena.flat
        self._runs_cache: Dict[int, List[Tuple[int, int, List[torch.Tensor]]]] = {}
        self._sched = None     # per group: fp64 device tensor {lr, t, lr/(1-b1^t), sqrt(1-b2^t), ...}
        self._sched_lr = None
        self._sched_betas = None
        # data parallelism (src/training/distributed.attach_grad_allreduce): a
        # GradBucketer whose all-reduces step() waits for, averaging by 1/world
        self.dp_bucketer = None

    def zero_grad(self, set_to_none: bool = True) -> None:
        if self.arena is not None:
            self.arena.join_pending()  # a deferred stem wgrad may still write the arena's grads
        super().zero_grad(set_to_none=set_to_none)
        if self.dp_bucketer is not None:
            self.dp_bucketer.reset()

    def use_device_schedule(self) -> None:
        """Keep lr and the step count on the device (``ssip_adamw_dev``, whose
        first launch of a step advances them): ``step()`` then enqueues kernels only — no host
        scalar changes per step, so it can run inside a captured hipGraph.
        All parameters of a group advance together (torch keeps one count per
        parameter; they agree whenever every parameter has a gradient)."""
        if self._sched is not None:
            return
        self._ensure_flat_state()
        dev = self.param_groups[0]["params"][0].device
        self._sched, self._sched_lr, self._sched_betas = [], [], []
        for group in self.param_groups:
            t = 0.0
            for p in group["params"]:
                st = self.state.get(p)
                if st and "step" in st:
                    t = float(st["step"])
                    break
            # {lr, t, lr/(1-b1^t), sqrt(1-b2^t), arrival counter of the advancing launch,
            #  staged 1-b1^(t+1), sqrt(1-b2^(t+1)) (0: not staged yet)}
            self._sched.append(torch.tensor([group["lr"], t, 0.0, 0.0, 0.0, 0.0, 0.0], dtype=torch.float64,
                                            device=dev))
            self._sched_lr.append(group["lr"])
            self._sched_betas.append(tuple(group["betas"]))

    def _ensure_flat_state(self):
        if self.arena is not None and self._flat_state is None:
            self._flat_state = (torch.zeros_like(self.arena.flat), torch.zeros_like(self.arena.flat))

    def _runs(self, gi: int, params: List[torch.Tensor]):
        """Group arena-resident params of a group into contiguous runs."""
        spans = []
        loose = []
        for p in params:
            if self.arena is not None and self.arena.owns(p) and p.grad is not None and \
                    p.grad.data_ptr() == self.arena.grad_view(p).data_ptr():
                off, n = self.arena.span(p)
                spans.append((off, n, p))
            else:
                loose.append(p)
        spans.sort(key=lambda t: t[0])
        runs: List[Tuple[int, int, List[torch.Tensor]]] = []
        for off, n, p in spans:
            if runs and runs[-1][0] + runs[-1][1] == off:
                o0, n0, ps = runs[-1]
                runs[-1] = (o0, n0 + n, ps + [p])
            else:
                runs.append((off, n, [p]))
        return runs, loose

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0, only=None, skip=None, sched_step: bool = True,
             join_pending: bool = True):
        """One AdamW update.  ``only`` / ``skip``: sets of id(param) restricting
        the update to a subset (a step split around a pending gradient, see
        SemiStep); the later parts of a split pass ``sched_step=False`` so the
        device schedule advances once per step.  Any gradient a side stream is
        still writing (a deferred stem wgrad) is joined first unless the caller
        updates only the other parameters (``join_pending=False``)."""
        if join_pending and self.arena is not None:
            self.arena.join_pending()
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self.dp_bucketer is not None:
            grad_scale = grad_scale * self.dp_bucketer.finish()
        self._ensure_flat_state()
        for gi, group in enumerate(self.param_groups):
            b1, b2 = group["betas"]
            params = [p for p in group["params"] if p.grad is not None and (only is None or id(p) in only)
                      and (skip is None or id(p) not in skip)]
            if not params:
                continue
            runs, loose = self._runs(gi, params)
            if self._sched is not None:
                self._step_device(gi, group, params, runs, loose, grad_scale, sched_step)
                continue
            # per-parameter state (views into the flat state for arena params)
            for p in params:
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    if self._flat_state is not None and self.arena.owns(p):
                        off, n = self.arena.span(p)
                        st["exp_avg"] = self._flat_state[0][off:off + n].view_as(p)
                        st["exp_avg_sq"] = self._flat_state[1][off:off + n].view_as(p)
                    else:
                        st["exp_avg"] = torch.zeros_like(p)
                        st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
            for off, n, ps in runs:
                step = int(self.state[ps[0]]["step"].item())
                ops.adamw(self.arena.flat[off:off + n], self.arena.grad[off:off + n],
                          self._flat_state[0][off:off + n], self._flat_state[1][off:off + n],
                          group["lr"], b1, b2, group["eps"], group["weight_decay"], step, grad_scale)
            for p in loose:
                st = self.state[p]
                ops.adamw(p.data, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"], group["lr"], b1, b2,
                          group["eps"], group["weight_decay"], int(st["step"].item()), grad_scale)
            # the kernels write through raw pointers: tell torch (and the
            # model's compute-dtype weight cache) that these tensors changed
            increment_version(params)
        return loss

    def _init_state(self, p):
        st = self.state[p]
        if len(st) == 0:
            st["step"] = torch.tensor(0.0)
            if self._flat_state is not None and self.arena.owns(p):
                off, n = self.arena.span(p)
                st["exp_avg"] = self._flat_state[0][off:off + n].view_as(p)
                st["exp_avg_sq"] = self._flat_state[1][off:off + n].view_as(p)
            else:
                st["exp_avg"] = torch.zeros_like(p)
                st["exp_avg_sq"] = torch.zeros_like(p)
        return st

    def _step_device(self, gi, group, params, runs, loose, grad_scale, sched_step=True):
        b1, b2 = group["betas"]
        sched = self._sched[gi]
        if group["lr"] != self._sched_lr[gi]:  # an LR scheduler moved it (host decision, eager only)
            sched[0].fill_(group["lr"])
            self._sched_lr[gi] = group["lr"]
        if tuple(group["betas"]) != self._sched_betas[gi]:
            # the advancing launch reads bias corrections the previous step
            # staged with the old betas (slots 5-6): drop them, so it
            # evaluates the corrections from this step's betas (torch reads
            # the betas at every step)
            sched[5:7].zero_()
            self._sched_betas[gi] = tuple(group["betas"])
        for p in params:
            self._init_state(p)
        # the first update launch of the step advances the schedule itself
        # (ssip_adamw_dev advance=1); later launches read the advanced values
        adv = sched_step
        for off, n, ps in runs:
            ops.adamw_dev(self.arena.flat[off:off + n], self.arena.grad[off:off + n],
                          self._flat_state[0][off:off + n], self._flat_state[1][off:off + n], sched,
                          b1, b2, group["eps"], group["weight_decay"], grad_scale, advance=adv)
            adv = False
        for p in loose:
            st = self.state[p]
            ops.adamw_dev(p.data, p.grad.contiguous(), st["exp_avg"], st["exp_avg_sq"], sched, b1, b2,
                          group["eps"], group["weight_decay"], grad_scale, advance=adv)
            adv = False
        increment_version(params)

    def device_step_count(self, gi: int = 0) -> int:
        """The device-side step count (syncs)."""
        return int(self._sched[gi][1].item()) if self._sched is not None else -1
