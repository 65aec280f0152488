"""Per-launch time of the device-schedule AdamW over a ResNet-18-sized arena
(11.69 M fp32 parameters: 28 B / element moved), HIP events, alone on the GPU.

usage (GPU box):  python tools/time_adamw.py   (SSIP_LIB=<path> for another build)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
import torch  # noqa: E402

from ssip import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n = 11_689_512
    p, g, m, v = (torch.randn(n, device=dev) for _ in range(4))
    v.abs_()
    sched = torch.tensor([1e-3] + [0.0] * 6, dtype=torch.float64, device=dev)
    for _ in range(5):
        ops.adamw_dev(p, g, m, v, sched, 0.9, 0.999, 1e-8, 1e-2, advance=True)
    ts = []
    for _ in range(50):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        ops.adamw_dev(p, g, m, v, sched, 0.9, 0.999, 1e-8, 1e-2, advance=True)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    med = ts[len(ts) // 2]
    print(f"adamw_dev n={n}: median {med:.1f} us, min {ts[0]:.1f} us, {n * 28 / med / 1e6:.2f} TB/s "
          f"(lib {os.environ.get('SSIP_LIB', 'in-tree')})")
    # variants and references on the same box: a 2-read 1-write torch pass, torch's fused AdamW
    def timed(fn, reps=30):
        for _ in range(3):
            fn()
        out = []
        for _ in range(reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            out.append(s.elapsed_time(e) * 1e3)
        out.sort()
        return out[len(out) // 2]
    t_na = timed(lambda: ops.adamw_dev(p, g, m, v, sched, 0.9, 0.999, 1e-8, 1e-2, advance=False))
    print(f"adamw_dev advance=0: {t_na:.1f} us, {n * 28 / t_na / 1e6:.2f} TB/s")
    t_h = timed(lambda: ops.adamw(p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 1e-2, 7))
    print(f"adamw (host schedule): {t_h:.1f} us, {n * 28 / t_h / 1e6:.2f} TB/s")
    o = torch.empty_like(p)
    t_add = timed(lambda: torch.add(p, g, out=o))
    print(f"torch.add (2R 1W) n={n}: {t_add:.1f} us, {n * 12 / t_add / 1e6:.2f} TB/s")
    try:
        tp = torch.nn.Parameter(p.clone())
        tp.grad = g.clone()
        opt = torch.optim.AdamW([tp], lr=1e-3, weight_decay=1e-2, fused=True)
        t_f = timed(opt.step)
        print(f"torch AdamW(fused=True) n={n}: {t_f:.1f} us, {n * 28 / t_f / 1e6:.2f} TB/s")
    except Exception as ex:  # fused AdamW may be unavailable on this build
        print("torch fused AdamW unavailable:", ex)


if __name__ == "__main__":
    main()
