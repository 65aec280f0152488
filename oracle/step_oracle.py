"""ORACLE (test infrastructure / CPU baseline only): the semi-supervised
train step restated on the CPU in plain torch fp32 — the same algorithm as
ssip.semi_step.SemiStep, with the reference's own pieces:

  views     torchvision train transform on PIL images (Resize -> flip ->
            rotate -> ToTensor -> Normalize, src/training/common.py:96-119),
            strong view = the same ops with a +-30 deg rotation plus
            brightness/contrast jitter and a cutout square
  model     torchvision resnet18 / resnet50 (restated in oracle/torchvision_restate)
  loss      nn.CrossEntropyLoss (src/training/semi_supervised.py:111) on the
            labelled half + masked CE on the strong view with pseudo-labels
            softmax/max/>=tau (semi_supervised.py:57-66)
  optimizer torch.optim.AdamW(lr=1e-4, wd=1e-4)

Used by bench.py's `cpu_baseline` leg (timed on the GPU box's host cores).
"""
from __future__ import annotations

import sys
import time
from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F
from PIL import Image

from .torchvision_restate.torchvision import models as tvm
from .torchvision_restate.torchvision import transforms as T

MEAN = [0.485, 0.456, 0.406]
STD = [0.229, 0.224, 0.225]


def _view(img: Image.Image, size: int, degrees: float, strong: bool, g: torch.Generator) -> torch.Tensor:
    img = img.resize((size, size), Image.BILINEAR) if img.size != (size, size) else img
    if torch.rand(1, generator=g) < 0.5:
        img = img.transpose(Image.FLIP_LEFT_RIGHT)
    ang = float(torch.empty(1).uniform_(-degrees, degrees, generator=g).item())
    img = img.rotate(ang, Image.NEAREST, expand=False, fillcolor=(0, 0, 0))
    t = T.ToTensor()(img)
    if strong:
        u = torch.rand(4, generator=g)
        b = 1.0 + 0.4 * (2 * float(u[0]) - 1)
        c = 1.0 + 0.4 * (2 * float(u[1]) - 1)
        t = ((t * b - 0.5) * c + 0.5).clamp(0, 1)
        side = int(0.25 * size)
        x0 = int(float(u[2]) * (size - side))
        y0 = int(float(u[3]) * (size - side))
        t[:, y0:y0 + side, x0:x0 + side] = 0.5
    return T.Normalize(MEAN, STD)(t)


def view_from_draw(img: Image.Image, size: int, flip: bool, angle, brightness: float = 1.0, contrast: float = 1.0,
                   cutout=None) -> torch.Tensor:
    """One view with explicit per-sample parameters (what ssip's GPU
    transform receives): Resize -> flip -> rotate(NEAREST) -> ToTensor ->
    brightness/contrast (clamped) -> cutout (0.5) -> Normalize."""
    img = img.resize((size, size), Image.BILINEAR) if img.size != (size, size) else img
    if flip:
        img = img.transpose(Image.FLIP_LEFT_RIGHT)
    if angle is not None:
        img = img.rotate(angle, Image.NEAREST, expand=False, fillcolor=(0, 0, 0))
    t = T.ToTensor()(img)
    if brightness != 1.0 or contrast != 1.0:
        t = ((t * brightness - 0.5) * contrast + 0.5).clamp(0, 1)
    if cutout is not None:
        x0, y0, x1, y1 = cutout
        t[:, y0:y1, x0:x1] = 0.5
    return T.Normalize(MEAN, STD)(t)


def semi_step_reference(model, opt, x_l: np.ndarray, y_l: torch.Tensor, x_u: np.ndarray, draws_l, draws_w, draws_s,
                        size: int, tau: float, lambda_u: float, pseudo_override=None, out: dict = None) -> torch.Tensor:
    """One joint step with explicit view parameters (draws: (flip, angle,
    brightness, contrast, cutout) tuples).  Returns [total, L_l, L_u, mask count].

    pseudo_override: use these pseudo-labels instead of the weak view's argmax
    (a parity test pins near-tied samples to the device's picks); out (dict):
    receives the weak logits 'zw', the joint logits 'z' and the pseudo-labels."""
    xl = torch.stack([view_from_draw(Image.fromarray(a), size, *d) for a, d in zip(x_l, draws_l)])
    xw = torch.stack([view_from_draw(Image.fromarray(a), size, *d) for a, d in zip(x_u, draws_w)])
    xs = torch.stack([view_from_draw(Image.fromarray(a), size, *d) for a, d in zip(x_u, draws_s)])
    dt = next(model.parameters()).dtype
    xl, xw, xs = xl.to(dt), xw.to(dt), xs.to(dt)
    bns = [b for b in model.modules() if isinstance(b, torch.nn.BatchNorm2d)]
    model.train()
    with torch.no_grad():
        saved = [(b.running_mean.clone(), b.running_var.clone(), b.num_batches_tracked.clone()) for b in bns]
        zw = model(xw)
        for b, (rm, rv, nb) in zip(bns, saved):
            b.running_mean.copy_(rm)
            b.running_var.copy_(rv)
            b.num_batches_tracked.copy_(nb)
    conf, pseudo = torch.softmax(zw, 1).max(1)
    if pseudo_override is not None:
        pseudo = pseudo_override.to(pseudo.device, pseudo.dtype)
    mask = (conf >= tau).to(dt)
    opt.zero_grad(set_to_none=True)
    z = model(torch.cat([xl, xs], 0))
    if out is not None:
        out.update(zw=zw.detach(), z=z.detach(), pseudo=pseudo)
    Bl = xl.shape[0]
    l_l = F.cross_entropy(z[:Bl], y_l)
    l_u = (F.cross_entropy(z[Bl:], pseudo, reduction="none") * mask).mean()
    loss = l_l + lambda_u * l_u
    loss.backward()
    opt.step()
    return torch.stack([loss.detach(), l_l.detach(), l_u.detach(), mask.sum()])


class CpuSemiStep:
    """The CPU step.  Views are made the way the reference's loaders make them:
    on `workers` background workers (TrainingConfig.num_workers = 2,
    common.py:54, 256-292), one step ahead of the model compute -- the
    parameters are drawn in order on the calling thread (deterministic), the
    Pillow work runs in a thread pool (Pillow releases the GIL) while the
    previous step computes.  workers=0: views made synchronously."""

    def __init__(self, seed: int = 42, tau: float = 0.7, lambda_u: float = 1.0, size: int = 224,
                 arch: str = "resnet18", workers: int = 2):
        torch.manual_seed(seed)
        self.model = getattr(tvm, arch)()
        self.model.fc = torch.nn.Linear(self.model.fc.in_features, 2)
        self.opt = torch.optim.AdamW(self.model.parameters(), lr=1e-4, weight_decay=1e-4)
        self.tau, self.lambda_u, self.size = tau, lambda_u, size
        self.g = torch.Generator().manual_seed(seed)
        self.workers = workers
        self._pool = None
        self._next = None

    def _draw(self, n: int, degrees: float, strong: bool):
        out = []
        for _ in range(n):
            flip = bool(torch.rand(1, generator=self.g) < 0.5)
            ang = float(torch.empty(1).uniform_(-degrees, degrees, generator=self.g).item())
            extra = None
            if strong:
                u = torch.rand(4, generator=self.g)
                side = int(0.25 * self.size)
                x0 = int(float(u[2]) * (self.size - side))
                y0 = int(float(u[3]) * (self.size - side))
                extra = (1.0 + 0.4 * (2 * float(u[0]) - 1), 1.0 + 0.4 * (2 * float(u[1]) - 1),
                         (x0, y0, x0 + side, y0 + side))
            out.append((flip, ang) + (extra if extra is not None else (1.0, 1.0, None)))
        return out

    def _views(self, x_l: np.ndarray, x_u: np.ndarray):
        S = self.size
        dl, dw, ds = self._draw(len(x_l), 10.0, False), self._draw(len(x_u), 10.0, False), \
            self._draw(len(x_u), 30.0, True)
        jobs = [(a, d) for a, d in zip(x_l, dl)] + [(a, d) for a, d in zip(x_u, dw)] + \
               [(a, d) for a, d in zip(x_u, ds)]

        def make(job):
            a, d = job
            return view_from_draw(Image.fromarray(a), S, *d)

        def run():
            if self._pool is None:
                return [make(j) for j in jobs]
            # the workers split the step's views (a DataLoader worker builds whole batches)
            k = -(-len(jobs) // self.workers)
            parts = [self._pool.submit(lambda js=jobs[i:i + k]: [make(j) for j in js])
                     for i in range(0, len(jobs), k)]
            return [v for p in parts for v in p.result()]

        def stack():
            v = run()
            nl, nu = len(x_l), len(x_u)
            return torch.stack(v[:nl]), torch.stack(v[nl:nl + nu]), torch.stack(v[nl + nu:])

        return stack

    def __call__(self, x_l: np.ndarray, y_l: torch.Tensor, x_u: np.ndarray) -> float:
        from concurrent.futures import ThreadPoolExecutor

        if self.workers > 0 and self._pool is None:
            self._pool = ThreadPoolExecutor(self.workers + 1)
        if self._next is None:
            cur = self._views(x_l, x_u)()
        else:
            cur = self._next.result()
        if self._pool is not None:  # the next step's views while this one computes
            self._next = self._pool.submit(self._views(x_l, x_u))
        xl, xw, xs = cur
        m = self.model
        m.train()
        with torch.no_grad():
            # weak view: batch statistics without touching the running stats
            saved = [(b.running_mean.clone(), b.running_var.clone(), b.num_batches_tracked.clone())
                     for b in m.modules() if isinstance(b, torch.nn.BatchNorm2d)]
            zw = m(xw)
            for b, (rm, rv, nb) in zip([b for b in m.modules() if isinstance(b, torch.nn.BatchNorm2d)], saved):
                b.running_mean.copy_(rm)
                b.running_var.copy_(rv)
                b.num_batches_tracked.copy_(nb)
        conf, pseudo = torch.softmax(zw, 1).max(1)
        mask = (conf >= self.tau).float()
        self.opt.zero_grad(set_to_none=True)
        z = m(torch.cat([xl, xs], 0))
        Bl = xl.shape[0]
        loss = F.cross_entropy(z[:Bl], y_l) + self.lambda_u * (
            F.cross_entropy(z[Bl:], pseudo, reduction="none") * mask).mean()
        loss.backward()
        self.opt.step()
        return float(loss.detach())

    def close(self):
        if self._next is not None:
            self._next.result()
            self._next = None
        if self._pool is not None:
            self._pool.shutdown()
            self._pool = None


def time_cpu_step(Bl: int = 128, Bu: int = 128, steps: int = 5, warmup: int = 2, threads: int = 16,
                  seed: int = 0, arch: str = "resnet18", size: int = 224, budget_s: float = 0.0,
                  workers: int = 2) -> Dict:
    """Images/sec of the CPU step (warm-up steps, then
    the MEDIAN of the timed steps) on a bounded sample of steps x (Bl + Bu)
    images of the workload's own architecture and image size.  budget_s > 0
    stops the timed steps once that much wall time has gone into them (at
    least 3 are timed); the count actually timed is reported."""
    import statistics

    torch.set_num_threads(threads)
    rng = np.random.default_rng(seed)
    x_l = rng.integers(0, 256, (Bl, size, size, 3), dtype=np.uint8)
    x_u = rng.integers(0, 256, (Bu, size, size, 3), dtype=np.uint8)
    y_l = torch.from_numpy(rng.integers(0, 2, Bl))
    step = CpuSemiStep(arch=arch, size=size, workers=workers)
    for i in range(warmup):
        t0 = time.perf_counter()
        step(x_l, y_l, x_u)
        # one progress line per step on stderr: a multi-minute baseline must not look hung
        print(f"cpu_baseline warm-up {i + 1}/{warmup}: {time.perf_counter() - t0:.2f} s", file=sys.stderr, flush=True)
    times = []
    for i in range(steps):
        t0 = time.perf_counter()
        step(x_l, y_l, x_u)
        times.append(time.perf_counter() - t0)
        print(f"cpu_baseline step {i + 1}/{steps}: {times[-1]:.2f} s", file=sys.stderr, flush=True)
        if budget_s > 0 and len(times) >= 3 and sum(times) >= budget_s:
            break
    step.close()
    dt = statistics.median(times)
    return {"value": (Bl + Bu) / dt, "step_s": dt, "threads": torch.get_num_threads(), "step_times_s": times,
            "steps_timed": len(times), "warmup": warmup,
            "sample": f"median of {len(times)} timed steps after {warmup} warm-up, each {Bl} labelled + {Bu} "
                      f"unlabelled {size}x{size} uint8 images: PIL weak/strong views (on {workers} background "
                      f"workers one step ahead, as the reference's num_workers=2 loaders) + torch fp32 {arch} weak "
                      f"forward + joint fwd/bwd + AdamW (oracle/step_oracle.py)"}
