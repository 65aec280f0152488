"""Per-launch conv durations of one single-stream train step (bench.py's
roofline leg: every conv launch bracketed by HIP events), in launch order.

usage (GPU box):  python tools/conv_breakdown.py [--batch 256]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
import torch  # noqa: E402

from ssip import SSIPResNet, ops, replace_fc  # noqa: E402
from ssip import resnet as resnet_mod  # noqa: E402
from ssip.semi_step import SemiStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=3, help="timed steps (per-launch median)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model = replace_fc(SSIPResNet("resnet18", 1000, dtype="bf16"), 2).to(dev).train()
    step = SemiStep(model, lr=1e-4, weight_decay=1e-4, tau=0.7, image_size=224, plan=False)
    step.overlap = False
    resnet_mod.WGRAD_SIDE_STREAM = False
    g = torch.Generator().manual_seed(1000)
    B = args.batch
    x_l = torch.randint(0, 256, (B // 2, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
    x_u = torch.randint(0, 256, (B - B // 2, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
    y_l = torch.randint(0, 2, (B // 2,), generator=g).to(dev)
    for _ in range(3):
        step(x_l, y_l, x_u)
    runs = []
    for _ in range(args.steps):
        t = ops.ConvTimer()
        ops.set_conv_timer(t)
        step(x_l, y_l, x_u)
        ops.set_conv_timer(None)
        torch.cuda.synchronize()
        runs.append([(k, f, s.elapsed_time(e) * 1e3) for k, f, _, s, e in t.records])
    tot_f = tot_us = 0.0
    by_kind = {}
    for i, (k, f, _) in enumerate(runs[0]):
        us = sorted(r[i][2] for r in runs)[len(runs) // 2]
        tot_f += f
        tot_us += us
        d = by_kind.setdefault(k, [0.0, 0.0, 0])
        d[0] += f
        d[1] += us
        d[2] += 1
        print(f"{i:3d} {k:6s} {f / 1e9:8.2f} GFLOP {us:8.1f} us {f / us / 1e6:7.1f} TF/s", flush=True)
    for k, (f, us, n) in by_kind.items():
        print(f"{k:6s} n={n:3d} {f / 1e12:.3f} TFLOP {us:8.1f} us {f / us / 1e6:7.1f} TF/s")
    print(f"total {tot_f / 1e12:.4f} TFLOP {tot_us:.1f} us {tot_f / tot_us / 1e6:.1f} TF/s "
          f"frac {tot_f / tot_us / 1e6 / 2500:.4f}")


if __name__ == "__main__":
    main()
