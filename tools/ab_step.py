"""In-process A/B of whole train steps under environment variants (the
library reads its SSIP_* tuning variables at every call, plan replays
included), interleaved in rounds so clock / box drift hits every variant
alike (cdna_hip_programming.md 5.4 rule 24).

usage (GPU box):  python tools/ab_step.py "A:" "B:SSIP_FOO=1,SSIP_BAR=2" [--rounds 7 --steps 10]
prints the median and min ms/step per variant.
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
import torch  # noqa: E402

from ssip import SSIPResNet, replace_fc  # noqa: E402
from ssip.semi_step import SemiStep  # noqa: E402


def parse_variant(s):
    name, _, rest = s.partition(":")
    env = {}
    for kv in filter(None, rest.split(",")):
        k, _, v = kv.partition("=")
        env[k] = v
    return name, env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--plan", type=int, default=1)
    args = ap.parse_args()
    variants = [parse_variant(v) for v in args.variants]
    keys = sorted({k for _, e in variants for k in e})
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model = replace_fc(SSIPResNet("resnet18", 1000, dtype="bf16"), 2).to(dev).train()
    step = SemiStep(model, lr=1e-4, weight_decay=1e-4, tau=0.7, image_size=224, plan=bool(args.plan))
    g = torch.Generator().manual_seed(1000)
    B = args.batch
    x_l = torch.randint(0, 256, (B // 2, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
    x_u = torch.randint(0, 256, (B - B // 2, 224, 224, 3), generator=g, dtype=torch.uint8).to(dev)
    y_l = torch.randint(0, 2, (B // 2,), generator=g).to(dev)

    def set_env(env):
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(env)

    for _, env in variants:  # warm every variant (plans, workspaces)
        set_env(env)
        for _ in range(3):
            step(x_l, y_l, x_u)
    torch.cuda.synchronize()
    times = {n: [] for n, _ in variants}
    for r in range(args.rounds):
        order = variants if r % 2 == 0 else variants[::-1]
        for name, env in order:
            set_env(env)
            step(x_l, y_l, x_u)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step(x_l, y_l, x_u)
            torch.cuda.synchronize()
            times[name].append((time.perf_counter() - t0) * 1e3 / args.steps)
        print(f"round {r}: " + "  ".join(f"{n} {times[n][-1]:.3f}" for n, _ in variants), flush=True)
    for name, _ in variants:
        t = times[name]
        print(f"{name:12s} median {statistics.median(t):.3f} ms/step  min {min(t):.3f}")


if __name__ == "__main__":
    main()
