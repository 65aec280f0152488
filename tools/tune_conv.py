"""Time every conv kernel configuration on the ResNet-18 train-step shapes.

Runs on the GPU box:  python tools/tune_conv.py [--batch 256] [--out gpurun_out/tune.json]
Each configuration is selected with SSIP_CONV_FORCE (see csrc/conv.hip
apply_force); "default" is the planner's own choice.
"""
import argparse, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
import torch  # noqa: E402
from ssip import ops  # noqa: E402

# the configurations the library instantiates (csrc/conv.hip SSIP_GLDS_FD / SSIP_GLDS_WG;
# round 3's wider sets are on the r3-variants branch) and the register-staged kernel (stages 0)
FD = [(128, 128, 4, 2, 2), (128, 64, 4, 2, 2), (256, 256, 4, 2, 2), (128, 128, 4, 4, 3), (128, 128, 2, 2, 0),
      (256, 128, 4, 2, 0)]
WG = [(128, 128, 4, 2, 2), (64, 128, 2, 4, 2), (128, 128, 2, 2, 0)]


def shapes(n):
    # (name, H, C, K, R, stride, pad)
    out = [("l1.3x3", 56, 64, 64, 3, 1, 1),
           ("l2.3x3s2", 56, 64, 128, 3, 2, 1), ("l2.3x3", 28, 128, 128, 3, 1, 1), ("l2.ds", 56, 64, 128, 1, 2, 0),
           ("l3.3x3s2", 28, 128, 256, 3, 2, 1), ("l3.3x3", 14, 256, 256, 3, 1, 1), ("l3.ds", 28, 128, 256, 1, 2, 0),
           ("l4.3x3s2", 14, 256, 512, 3, 2, 1), ("l4.3x3", 7, 512, 512, 3, 1, 1), ("l4.ds", 14, 256, 512, 1, 2, 0)]
    return [(nm, ops.ConvGeom(n, H, H, C, K, R, R, s, p, C, R)) for nm, H, C, K, R, s, p in out]


def time_fn(fn, iters):
    for _ in range(3):
        fn()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/tune.json")
    ap.add_argument("--modes", default="fdw", help="passes to tune: any of f, d, w")
    ap.add_argument("--shapes", default="", help="comma-separated shape names (default: all)")
    ap.add_argument("--wg", default="", help="wgrad configs 'bm,bn,wm,wn,st;...' (default: the built-in list)")
    ap.add_argument("--fd", default="", help="fwd/dgrad configs 'bm,bn,wm,wn,st;...' (default: the built-in list)")
    ap.add_argument("--no-check", action="store_true", help="skip the result check")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    ws = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
    part = torch.empty(8 << 20, dtype=torch.float32, device=dev)
    res = []
    wg_cfgs = [tuple(int(v) for v in c.split(",")) for c in args.wg.split(";") if c] or WG
    fd_cfgs = [tuple(int(v) for v in c.split(",")) for c in args.fd.split(";") if c] or FD
    want = set(args.shapes.split(",")) if args.shapes else None
    for nm, g in shapes(args.batch):
        if want is not None and nm not in want:
            continue
        x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
        w = (torch.randn(g.K, g.R, g.S, g.C, device=dev) * 0.05).to(bf)
        wc = w.permute(3, 1, 2, 0).contiguous()
        y = torch.empty(g.N, g.P, g.Q, g.K, device=dev, dtype=bf)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.empty(g.K, g.C, g.R, g.S, device=dev, dtype=torch.float32)
        runs = {
            "f": (fd_cfgs, lambda: ops.conv_fwd(g, x, w, y, part), y),
            "d": (fd_cfgs, lambda: ops.conv_dgrad(g, dy, wc, dx), dx),
            "w": (wg_cfgs, lambda: ops.conv_wgrad(g, dy, x, dw, False, ws), dw),
        }
        for mode, (cfgs, fn, out) in runs.items():
            if mode not in args.modes:
                continue
            os.environ.pop("SSIP_CONV_FORCE", None)
            t_def = time_fn(fn, args.iters)
            ref = out.float().clone()
            scale = ref.abs().max().item()
            best = ("default", t_def)
            row = {"shape": nm, "mode": mode, "default_us": t_def, "tf": g.flops() / t_def / 1e6, "cfg": {}}
            for c in cfgs:
                os.environ["SSIP_CONV_FORCE"] = mode + "," + ",".join(map(str, c))
                try:
                    t = time_fn(fn, args.iters)
                except RuntimeError as e:  # configuration not valid for this shape
                    row["cfg"][str(c)] = str(e)[:60]
                    continue
                err = 0.0 if args.no_check else (out.float() - ref).abs().max().item() / scale
                if not err < 2e-2:
                    row["cfg"][str(c)] = f"MISMATCH rel err {err:.3g}"
                    print(f"  {nm} {mode} {c}: MISMATCH rel err {err:.3g}", flush=True)
                    continue
                row["cfg"][str(c)] = t
                if t < best[1]:
                    best = (str(c), t)
            os.environ.pop("SSIP_CONV_FORCE", None)
            row["best"], row["best_us"] = best
            res.append(row)
            print(f"{nm:9s} {mode} default {t_def:7.1f}us ({row['tf']:5.0f} TF/s)  best {best[0]:22s} "
                  f"{best[1]:7.1f}us ({g.flops() / best[1] / 1e6:5.0f} TF/s)", flush=True)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
