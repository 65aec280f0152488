"""One conv launch set for PMC passes over the conv k-loop:
layer3's 3x3 forward at batch 256, `--iters` launches of the planner's
choice (or SSIP_CONV_FORCE), with the operand fill on or off (SSIP_DIAG=3:
zero-extent buffer resources, the same instruction stream with no L2/HBM
traffic; results wrong).

usage (GPU box, one rocprofv3 pass per counter set):
  SSIP_DIAG=3 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS ... -d gpurun_out/x -o run -- \
      python tools/pmc_conv_loop.py [--shape l3.3x3] [--iters 5]
post-process (host): python tools/pmc_conv_loop.py --summarize <run_counter_collection.csv> ...
"""
import argparse
import collections
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(shape, iters):
    sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import torch
    from ssip import ops
    from tune_conv import shapes
    dev = torch.device("cuda:0")
    g = dict(shapes(256))[shape]
    bf = torch.bfloat16
    x = torch.randn(g.N, g.H, g.W, g.C, device=dev).to(bf)
    w = (torch.randn(g.K, g.R, g.S, g.C, device=dev) * 0.05).to(bf)
    y = torch.empty(g.N, g.P, g.Q, g.K, device=dev, dtype=bf)
    part = torch.empty(8 << 20, dtype=torch.float32, device=dev)
    for _ in range(iters):
        ops.conv_fwd(g, x, w, y, part)
    torch.cuda.synchronize()
    print(f"{shape} fwd x{iters} SSIP_DIAG={os.environ.get('SSIP_DIAG', '0')} "
          f"force={os.environ.get('SSIP_CONV_FORCE', '-')}", flush=True)


def summarize(paths):
    """Totals of every counter over the conv_glds dispatches of each file."""
    for p in paths:
        acc = collections.defaultdict(list)
        name = ""
        for r in csv.DictReader(open(p)):
            if "conv_glds" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"]
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f"# {p}\n#   {name[:110]}")
        for k, v in sorted(acc.items()):
            # a counter row per (dispatch, dimension instance): sum per dispatch
            print(f"  {k:28s} total {sum(v):.6g}  rows {len(v)}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="l3.3x3")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--summarize", nargs="*")
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize)
    else:
        run(a.shape, a.iters)


if __name__ == "__main__":
    main()
