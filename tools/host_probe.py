"""Host-side cost of one plan-replayed SemiStep (bench.py's headline loop):
per-step host time of step() (draw_params + input/param copies + C++ replay)
against the device time per step, to see whether the host keeps ahead.

usage (GPU box): python tools/host_probe.py [--steps 30]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
import torch  # noqa: E402

from ssip import SSIPResNet, replace_fc  # noqa: E402
from ssip.semi_step import SemiStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
    torch.manual_seed(42)
    model = replace_fc(SSIPResNet("resnet18", 1000, dtype="bf16"), 2).to(dev).train()
    step = SemiStep(model, lr=1e-4, weight_decay=1e-4, tau=0.7, image_size=224, plan=True)
    g = torch.Generator().manual_seed(1000)
    x_l = torch.randint(0, 256, (128, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
    x_u = torch.randint(0, 256, (128, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
    y_l = torch.randint(0, 2, (128,), generator=g).to(dev)
    for _ in range(5):
        step(x_l, y_l, x_u)
    slots = step.input_slots()
    if slots is not None:
        for d, s in zip(slots, (x_l, y_l, x_u)):
            d.copy_(s)
        x_l, y_l, x_u = slots
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        h0 = time.perf_counter()
        step(x_l, y_l, x_u)
        host.append(time.perf_counter() - h0)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    host.sort()
    print(f"steps {a.steps}: wall {t_all / a.steps * 1e3:.3f} ms/step, host enqueue {t_enq / a.steps * 1e3:.3f} ms/step "
          f"(median {host[len(host) // 2] * 1e3:.3f}, max {host[-1] * 1e3:.3f})")
    # host pieces
    t = time.perf_counter()
    for _ in range(50):
        step.draw_params(128, 128)
    print(f"draw_params {(time.perf_counter() - t) / 50 * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
