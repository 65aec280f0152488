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

import os
from dataclasses import dataclass
from typing import List, Optional

import torch

from . import ops
from .augment import GpuTransform, draw_params_batch
from .optim import AdamW
from .resnet import DeviceImages, SSIPResNet


# the weight refresh on the side stream beside the train views' augment
# (SSIP_PREP_SIDE=0: on main ahead of both; round 4 re-measured it, 3 + 3
# alternated runs on one box: 6.403 vs 6.416 ms/step, each pair in its favour)
_PREP_SIDE = os.environ.get("SSIP_PREP_SIDE", "1") != "0"


@dataclass
class StepStats:
    # [4] total, L_l, L_u, mask count (device).  In plan mode every replay
    # writes the same buffer: clone it to keep a step's value past the next step.
    loss: torch.Tensor


def _common_base(params):
    """The tensor the view parameters are consecutive row ranges of, or None."""
    b = params[0]._base
    if b is None or not b.is_contiguous() or b.dim() != 2:
        return None
    o = 0
    for p in params:
        if p._base is not b or p.data_ptr() != b[o:].data_ptr():
            return None
        o += p.shape[0]
    return b if o == b.shape[0] else None


# SSIP_EARLY_ADAMW=1: AdamW of the head and layers 2-4 on its own stream as
# soon as their gradients are final (during the layer-1 backward) instead of
# in the step's tail beside the stem wgrad, where both are HBM-bound (single
# process only: with a process group the all-reduce of every bucket comes
# first).  Bit-identical updates; measured 5.879 vs 5.849 ms (4 + 4): the
# layer-1 backward loses more to it than the tail gains.  Off by default.
_EARLY_ADAMW = os.environ.get("SSIP_EARLY_ADAMW", "0") == "1"


class SemiStep:
    """One call = one optimizer step.

    graph=True: the first ``eager_warmup`` calls run eagerly; the next call
    captures steps 1-5 (augment -> weak forward -> train forward -> loss ->
    backward, ~260 kernel launches) into one hipGraph via torch.cuda.graph,
    and every call from then on copies its inputs into the graph's static
    buffers and replays it: no per-kernel host launch cost, no host gaps.
    AdamW runs after the replay with its schedule on the device
    (``AdamW.use_device_schedule``); with world > 1 the gradient buckets are
    all-reduced between the replay and AdamW (ROCm has no external event
    nodes, so a bucket cannot be released from inside the graph; ``--eager``
    keeps the in-backward overlap instead).
    """

    def __init__(self, model: SSIPResNet, lr: float = 1e-4, weight_decay: float = 1e-4, tau: float = 0.7,
                 lambda_u: float = 1.0, image_size: int = 224, bucketer=None, seed: int = 0, graph: bool = False,
                 eager_warmup: int = 2, plan: bool = False):
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
        self.graph = graph
        self.eager_warmup = eager_warmup
        self._calls = 0
        self._g = None
        if graph and plan:
            raise ValueError("SemiStep: graph and plan are alternatives")
        self.plan = plan
        self._plan = None
        self._static_pbase = None
        # launch-plan replays the host may have enqueued ahead of the device:
        # with no bound the host fills HIP's queue, blocks, and resumes only
        # after the device has drained most of it -- the device then idles
        # ~0.3 ms per step (MI355X, ROCm 7.2: 6.95 vs 6.55 ms/step at 2,
        # tools/ab_inflight.sh).  0 = unbounded.
        self.max_inflight = int(os.environ.get("SSIP_MAX_INFLIGHT", "2"))
        self._inflight = []
        # pinned staging of the per-step view parameters: a ring reused across
        # steps (a fresh pin_memory() per step can allocate page-locked memory,
        # which stalls the device queue), each slot reusable once the H2D copy
        # that read it has run (its event)
        self._pin_ring = []   # [(pinned buffer, event or None)]
        self._pin_next = 0
        if graph or plan:
            self.opt.use_device_schedule()
        # single process, no graph capture: the optimizer overlaps the stem
        # wgrad at the end of the backward (a graph capture needs every forked
        # stream joined; a gradient bucketer reduces conv1's gradient itself)
        # (scoped to this step's own backward: _fwd_bwd sets the model flag and
        # clears it, so another trainer of the same model never defers)
        self._defer = bucketer is None and not graph and os.environ.get("SSIP_DEFER_STEM") != "0"
        self._upd = None          # the early AdamW's stream
        self._early_ids = None
        self._early_done = False

    def _side_stream(self, dev):
        if self._side is None:
            self._side = torch.cuda.Stream(device=dev)
        return self._side

    def draw_params(self, Bl: int, Bu: int):
        """Per-sample view parameters (host RNG, like a DataLoader worker):
        (labelled weak, unlabelled weak, unlabelled strong) as views of one
        pinned buffer, so a step moves them to the device in one copy."""
        s = self.size
        parts = (draw_params_batch(Bl, s, False, self.gen), draw_params_batch(Bu, s, False, self.gen),
                 draw_params_batch(Bu, s, True, self.gen))
        rows = sum(p.shape[0] for p in parts)
        buf = self._pinned(rows, parts[0].shape[1:], parts[0].dtype)
        torch.cat(parts, out=buf)
        return (buf[:Bl], buf[Bl:Bl + Bu], buf[Bl + Bu:])

    def _pinned(self, rows, tail, dtype) -> torch.Tensor:
        """The next slot of the pinned ring, waited for and sized to [rows, *tail]."""
        R = 4
        if len(self._pin_ring) < R:
            self._pin_ring = [(None, None)] * R
        i = self._pin_next
        self._pin_next = (i + 1) % R
        buf, ev = self._pin_ring[i]
        if ev is not None:
            ev.synchronize()
        if buf is None or buf.shape != (rows,) + tuple(tail) or buf.dtype != dtype:
            buf = torch.empty((rows,) + tuple(tail), dtype=dtype).pin_memory()
        self._pin_ring[i] = (buf, None)
        return buf

    def _pinned_read(self, *ts) -> None:
        """Mark every ring slot that holds (part of) a host tensor in ts as read
        by the current stream's latest copy: the slot is handed out again only
        after that copy has run.  Called after every non_blocking copy out of
        the ring (eager, plan and graph paths alike)."""
        for i, (buf, _) in enumerate(self._pin_ring):
            if buf is None:
                continue
            lo, hi = buf.data_ptr(), buf.data_ptr() + buf.numel() * buf.element_size()
            if any(t is not None and t.device.type == "cpu" and lo <= t.data_ptr() < hi for t in ts):
                ev = torch.cuda.Event()
                ev.record()
                self._pin_ring[i] = (buf, ev)

    def input_slots(self):
        """The device buffers a recorded plan reads its batch from
        (x_l, y_l, x_u): an input pipeline that writes the next batch here
        spares the step its copy-in.  None before the plan is recorded."""
        return None if self._plan is None else self._static[:3]

    # the three pieces of steps 1-5; each runs on the current stream and is
    # capturable (no host sync, no host-side value that changes per step)
    def _weak(self, x_u, pw) -> torch.Tensor:
        """weak view + weak forward (batch-stat BN, no running update, no grad)."""
        m = self.model
        m.bn_update_running = False
        with torch.no_grad():
            zw = m(self.tf(x_u, pw))
        m.bn_update_running = True
        return zw

    def _train_views(self, x_l, x_u, pl, ps) -> torch.Tensor:
        """[labelled weak ; unlabelled strong] views of the joint train forward."""
        m = self.model
        Bl, Bu = x_l.shape[0], x_u.shape[0]
        S, P = self.size, self.tf.pad
        x_ls = torch.empty((Bl + Bu, S + 2 * P, S + 2 * P, 4), device=x_l.device, dtype=m.compute_dtype)
        self.tf(x_l, pl, out=x_ls[:Bl])
        self.tf(x_u, ps, out=x_ls[Bl:])
        return x_ls

    def _train_fwd(self, x_l, x_u, pl, ps, x_ls=None) -> torch.Tensor:
        """The joint train forward (views formed here unless given)."""
        m = self.model
        if x_ls is None:
            x_ls = self._train_views(x_l, x_u, pl, ps)
        self.opt.zero_grad(set_to_none=True)
        if self.bucketer is not None:
            self.bucketer.reset()
        return m(DeviceImages(x_ls, self.tf.pad))

    def _loss_bwd(self, logits, y_l, zw) -> torch.Tensor:
        """loss + dlogits in one launch, then the backward."""
        Bl = y_l.shape[0]
        dz = torch.empty_like(logits, dtype=torch.float32)
        out, dzl, dzs, pseudo, mask = ops.semi_loss(logits[:Bl].detach().contiguous(), y_l, zw.contiguous(),
                                                    logits[Bl:].detach().contiguous(), self.tau, self.lambda_u, dz=dz)
        self.last = {"zw": zw, "logits": logits.detach(), "pseudo": pseudo, "mask": mask}  # device tensors
        logits.backward(dz)
        return out

    def _fwd_bwd(self, x_l, y_l, x_u, pl, pw, ps) -> torch.Tensor:
        """Steps 1-5, eager: the weak forward on a side stream overlaps the
        train forward (they only meet at the loss)."""
        m = self.model
        dev = x_l.device
        main = torch.cuda.current_stream(dev)
        m.train()
        side = self._side_stream(dev) if self.overlap else main
        if side is not main and _PREP_SIDE:
            # the compute-dtype weight refresh for both forwards on the side
            # stream, beside the train views' augment on main; main waits for
            # the refresh (not for the weak forward queued after it)
            ops.wait_stream(side, main)
            with torch.cuda.stream(side):
                m.prepare_weights(need_t=True)
            x_ls = self._train_views(x_l, x_u, pl, ps)
            ops.wait_stream(main, side)
            with torch.cuda.stream(side):
                zw = self._weak(x_u, pw)
            logits = self._train_fwd(x_l, x_u, pl, ps, x_ls)
        else:
            # compute-dtype weights for both forwards, refreshed once, before the fork
            m.prepare_weights(need_t=True)
            if side is not main:
                ops.wait_stream(side, main)
            with torch.cuda.stream(side):
                zw = self._weak(x_u, pw)
            logits = self._train_fwd(x_l, x_u, pl, ps)
        if side is not main:
            ops.wait_stream(main, side)
            zw.record_stream(main)
        m.defer_stem_wgrad_join = self._defer
        self._early_done = False
        if self._early_ok(main, side):
            m.early_update = self._early_update
            m.early_update_block = len(m.layer1)
        try:
            return self._loss_bwd(logits, y_l, zw)
        finally:
            m.defer_stem_wgrad_join = False
            m.early_update = None

    def __call__(self, x_l: torch.Tensor, y_l: torch.Tensor, x_u: torch.Tensor, params=None) -> StepStats:
        """x_l [Bl,H,W,3] u8, y_l [Bl] int64, x_u [Bu,H,W,3] u8 — all on the device."""
        Bl, Bu = x_l.shape[0], x_u.shape[0]
        dev = x_l.device
        if params is None:
            params = self.draw_params(Bl, Bu)
        self._calls += 1
        if self.graph and self._calls > self.eager_warmup:
            return self._replay(x_l, y_l, x_u, params)
        if self.plan and self._calls > self.eager_warmup:
            return self._plan_step(x_l, y_l, x_u, params)
        return self._eager_step(x_l, y_l, x_u, params)

    def _eager_step(self, x_l, y_l, x_u, params) -> StepStats:
        dev = x_l.device
        pl, pw, ps = (p.to(dev, non_blocking=True) for p in params)
        self._pinned_read(*params)
        out = self._fwd_bwd(x_l, y_l, x_u, pl, pw, ps)
        scale = self.bucketer.finish() if self.bucketer is not None else 1.0
        # 6. optimizer
        self._optimizer_step(scale)
        return StepStats(loss=out)

    def _dev_params(self, params, dev):
        """Device copies of the view parameters; views of one device buffer
        when the host ones are views of one buffer (one copy per replay)."""
        base = _common_base(params)
        self._static_pbase = None
        if base is None:
            return tuple(p.to(dev) for p in params)
        self._static_pbase = base.to(dev)
        out, o = [], 0
        for p in params:
            out.append(self._static_pbase[o:o + p.shape[0]])
            o += p.shape[0]
        return tuple(out)

    def _early_ok(self, main, side) -> bool:
        m = self.model
        return (_EARLY_ADAMW and self.bucketer is None and getattr(self.opt, "dp_bucketer", None) is None
                and side is not main and self._defer and hasattr(m, "layer1")
                and len(list(m.blocks())) > len(m.layer1))

    def _early_params(self):
        """ids of the head's and of layers 2-4's parameters (cached)."""
        if self._early_ids is None:
            m = self.model
            blocks = list(m.blocks())
            ps = [p for b in blocks[len(m.layer1):] for p in b.parameters()] + list(m.fc.parameters())
            self._early_ids = {id(p) for p in ps}
        return self._early_ids

    def _early_update(self, stream) -> None:
        """AdamW of _early_params on the update stream, after `stream` (which
        already waited for the main stream's BN gradients of those layers)."""
        dev = stream.device
        if self._upd is None:
            self._upd = torch.cuda.Stream(device=dev)
        ops.wait_stream(self._upd, stream)
        with torch.cuda.stream(self._upd):
            self.opt.step(grad_scale=1.0, only=self._early_params(), join_pending=False)
        self._early_done = True

    def _optimizer_step(self, scale: float) -> None:
        """AdamW; with the stem wgrad still running on the side stream
        (defer_stem_wgrad_join) every other parameter is enqueued first, with
        no join on the side stream, then conv1.  (On MI355X the stem wgrad
        holds every SIMD's register file, so the first update is dispatched
        as it drains rather than beside it: profiles/r2_step_streams.txt.)"""
        m = self.model
        late = {id(m.conv1.weight)}
        # (the stem wgrad on main with the other updates on the side stream,
        # round 3's SSIP_STEM_MAIN: 6.399 vs 6.395 ms/step over 3 + 3 alternated
        # runs, no gain -- the simpler layout stays)
        pend = m.take_pending_side()
        early = self._early_done
        self._early_done = False
        if early:
            # the early launch advanced the device schedule: the rest follow it
            ops.wait_stream(torch.cuda.current_stream(), self._upd)
            late_or_early = late | self._early_params()
            if pend is None:
                self.opt.step(grad_scale=scale, skip=self._early_params(), sched_step=False)
                return
            self.opt.step(grad_scale=scale, skip=late_or_early, join_pending=False, sched_step=False)
            ops.wait_stream(torch.cuda.current_stream(), pend)
            self.opt.step(grad_scale=scale, only=late, sched_step=False)
            return
        if pend is None:
            self.opt.step(grad_scale=scale)
            return
        self.opt.step(grad_scale=scale, skip=late, join_pending=False)
        ops.wait_stream(torch.cuda.current_stream(), pend)
        self.opt.step(grad_scale=scale, only=late, sched_step=False)

    # ------------------------------------------------------------------
    # launch-plan path (ssip/plan.py): record one step, replay it from C++
    # ------------------------------------------------------------------
    def _finish_buckets(self):
        self.bucketer.finish()

    def _plan_step(self, x_l, y_l, x_u, params) -> StepStats:
        """Steps 1-6 replayed from the recorded plan: the same launches on the
        same streams (weak forward and wgrads still overlap), with the gradient
        buckets' all-reduces launched between plan segments."""
        from torch.autograd.graph import increment_version

        from .plan import Plan

        dev = x_l.device
        if self._plan is None:
            self._static = (x_l.clone(), y_l.clone(), x_u.clone()) + self._dev_params(params, dev)
            plan = Plan()
            scale = self.bucketer.grad_scale() if self.bucketer is not None else 1.0
            with plan:
                out = self._fwd_bwd(*self._static)
                if self.bucketer is not None:
                    ops.host_callback(self._finish_buckets)
                self._optimizer_step(scale)
            self._plan, self._plan_out = plan, out
            return StepStats(loss=out)
        # the plan replays fixed buffers: a batch of another shape (a short last
        # batch) or dtype runs as an eager step instead
        rec = self._static
        if any(a.shape != b.shape or a.dtype != b.dtype
               for a, b in zip((x_l, y_l, x_u) + tuple(params), rec)) or len(params) != len(rec) - 3:
            return self._eager_step(x_l, y_l, x_u, params)
        for dst, src in zip(self._static[:3], (x_l, y_l, x_u)):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src, non_blocking=True)
        base = _common_base(params)
        if base is not None and self._static_pbase is not None and base.shape == self._static_pbase.shape:
            self._static_pbase.copy_(base, non_blocking=True)
        else:
            for dst, src in zip(self._static[3:], params):
                dst.copy_(src, non_blocking=True)
        self._pinned_read(*params)
        if self.bucketer is not None:
            self.bucketer.reset()
        if self.max_inflight > 0:
            while len(self._inflight) >= self.max_inflight:
                self._inflight.pop(0).synchronize()
        self._plan.replay()
        if self.max_inflight > 0:
            ev = torch.cuda.Event()
            ev.record()
            self._inflight.append(ev)
        # the replay's AdamW changed the weights behind torch's back: bump the
        # versions so an eager forward afterwards refreshes its weight copies
        increment_version(list(self.model.parameters()))
        return StepStats(loss=self._plan_out)

    # ------------------------------------------------------------------
    # hipGraph path
    # ------------------------------------------------------------------
    def _replay(self, x_l, y_l, x_u, params) -> StepStats:
        if self._g is None:
            self._capture(x_l, y_l, x_u, params)
        else:
            for dst, src in zip(self._static, (x_l, y_l, x_u) + tuple(params)):
                if dst.data_ptr() != src.data_ptr():
                    dst.copy_(src, non_blocking=True)
            self._pinned_read(*params)
        self._g.replay()
        if self.bucketer is not None:
            self.bucketer.launch_after_graph()
            scale = self.bucketer.finish()
        else:
            scale = 1.0
        self.opt.step(grad_scale=scale)
        # the next replay reads the compute-dtype weights: refresh them now
        self.model.prepare_weights(need_t=True, force=True)
        return StepStats(loss=self._g_out)

    def _capture(self, x_l, y_l, x_u, params):
        """One graph for steps 1-5.  The weak and train forwards are captured
        from two streams, but HIP executes graph nodes (and separately launched
        graphs) one after another, so they run back to back; splitting the
        step into per-stream graphs, or launching the weak forward eagerly
        beside the replay, measured no faster on MI355X."""
        dev = x_l.device
        m = self.model
        m.train()
        self._static = (x_l.clone(), y_l.clone(), x_u.clone()) + tuple(p.to(dev) for p in params)
        m.prepare_weights(need_t=True, force=True)
        torch.cuda.synchronize(dev)
        if self.bucketer is not None:
            self.bucketer.capture_mode = True
        g = torch.cuda.CUDAGraph()
        # thread-local capture: with a process group, RCCL's watchdog thread
        # queries its collectives' events while this thread captures (global
        # mode turns that into a fatal capture error in the watchdog)
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self._g_out = self._fwd_bwd(*self._static)
            if self.bucketer is not None:
                self.bucketer.end_capture()
        if self.bucketer is not None:
            self.bucketer.capture_mode = False
        self._g = g
