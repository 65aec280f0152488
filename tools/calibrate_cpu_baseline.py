"""Calibrate the CPU baseline (oracle/step_oracle.py) against the REFERENCE's
own `train_model` in the build container ("the restatement
and the reference train_model must agree within ~5 % on this container").
Build container only: imports /root/reference.

  (a) the reference's train_model (src/training/common.py:345-432) over
      batches of 256 synthetic 224x224 fp32 images, torch fp32 on the host
      threads: seconds per optimizer step (timestamps at each optimizer.step,
      the first step excluded)
  (b) the same step through the oracle's restated model (oracle/torchvision_
      restate resnet18 + AdamW + CE, oracle/step_oracle.py's machinery):
      seconds per step -- (a) and (b) must agree within ~5 %
  (c) the bench's cpu_baseline step (CpuSemiStep: 128 labelled + 128
      unlabelled uint8 images, PIL views on 2 background workers, weak
      forward + joint fwd/bwd + AdamW) on the same threads, for the record:
      its images/s is the number bench.py reports on the GPU box's cores

usage: python tools/calibrate_cpu_baseline.py [--threads 8] [--steps 4] [--out profiles/r5_cpu_calibration.txt]
"""
import argparse
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r5_cpu_calibration.txt"))
    a = ap.parse_args()
    if not REF.exists():
        sys.exit("calibrate_cpu_baseline: /root/reference not present (build container only)")
    sys.path.insert(0, str(ROOT / "oracle" / "torchvision_restate"))
    sys.path.insert(0, str(REF / "src"))
    sys.path.insert(0, str(ROOT))
    import numpy as np
    import torch
    from torch.utils.data import DataLoader

    from training import common as C  # reference module
    from oracle.step_oracle import time_cpu_step
    from oracle.torchvision_restate.torchvision import models as tvm

    torch.set_num_threads(a.threads)
    B = a.batch
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, 3, 224, 224, generator=g)
    y = torch.randint(0, 2, (B,), generator=g)

    # (a) the reference's train_model, one epoch of steps+1 batches (the first one is warm-up)
    torch.manual_seed(42)
    model = C.create_model(2, pretrained=False)
    opt = torch.optim.AdamW((p for p in model.parameters() if p.requires_grad), lr=1e-4, weight_decay=1e-4)
    stamps = []
    real_step = opt.step

    def timed_step(*args, **kw):
        out = real_step(*args, **kw)
        stamps.append(time.perf_counter())
        return out

    opt.step = timed_step
    train = DataLoader([(x[i], int(y[i])) for i in range(B)] * (a.steps + 1), batch_size=B, shuffle=False)
    val = DataLoader([(x[i], int(y[i])) for i in range(8)], batch_size=8)
    C.train_model(model, train, val, torch.nn.CrossEntropyLoss(), opt, torch.device("cpu"), num_epochs=1)
    ref_steps = [t1 - t0 for t0, t1 in zip(stamps, stamps[1:])]
    ref_s = statistics.median(ref_steps)

    # (b) the oracle's restated model, the same step
    torch.manual_seed(42)
    m2 = tvm.resnet18()
    m2.fc = torch.nn.Linear(512, 2)
    opt2 = torch.optim.AdamW(m2.parameters(), lr=1e-4, weight_decay=1e-4)
    m2.train()
    ts = []
    for i in range(a.steps + 1):
        t0 = time.perf_counter()
        opt2.zero_grad(set_to_none=True)
        loss = torch.nn.functional.cross_entropy(m2(x), y)
        loss.backward()
        opt2.step()
        float(loss)
        ts.append(time.perf_counter() - t0)
    ora_s = statistics.median(ts[1:])

    # (c) the bench's semi step restatement
    c = time_cpu_step(Bl=B // 2, Bu=B - B // 2, steps=a.steps, warmup=1, threads=a.threads)

    lines = [
        "# CPU baseline calibration (tools/calibrate_cpu_baseline.py, build container, "
        f"{a.threads} threads, torch {torch.__version__})",
        f"(a) reference train_model, bs {B} fp32 224x224, per optimizer step: median {ref_s:.3f} s over "
        f"{len(ref_steps)} steps = {B / ref_s:.1f} images/s  (steps: {', '.join(f'{t:.2f}' for t in ref_steps)})",
        f"(b) oracle restatement of the same step: median {ora_s:.3f} s over {a.steps} = {B / ora_s:.1f} images/s  "
        f"(steps: {', '.join(f'{t:.2f}' for t in ts[1:])})",
        f"    (b) / (a) time ratio = {ora_s / ref_s:.3f}  (SURVEY 8(d): agree within ~5 %)",
        f"(c) bench cpu_baseline step (CpuSemiStep, {B // 2} + {B - B // 2}, views on 2 background workers): "
        f"median {c['step_s']:.3f} s = {c['value']:.1f} images/s; its model work is a 128-image weak forward "
        f"(~1/6 of a 256-image train step) on top of (b)'s step: expected ~{7 / 6 * ora_s:.2f} s",
    ]
    txt = "\n".join(lines)
    print(txt)
    Path(a.out).write_text(txt + "\n")


if __name__ == "__main__":
    main()
