"""Layer-1 halo forward phase stamps (GPU box): runs
conv_halo_kernel's STAMP instance (SSIP_HALO_DIAG=128, s_memtime after each
tile's barrier, after its k-loop's vmcnt(0) and after its epilogue, per wave)
at batch 256 and prints where a tile's cycles go: the k-loop (18 k-steps of
8 MFMAs per wave, 2 waves per SIMD: 4,608 MFMA cycles per SIMD if the matrix
pipe never idles), the epilogue (BN statistics + stores) and the barrier wait.

usage: python tools/halo_stamp_lab.py [--batch 256] [--out f.txt]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from ssip import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default=None)
    ap.add_argument("--label", default="")
    ap.add_argument("--diags", default="0", help="extra SSIP_HALO_DIAG bits per run (with 128): 1 no stores, "
                    "2 no MFMAs, 4 no input DMA after the first tile, 8 no BN statistics")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    n = a.batch
    g = ops.ConvGeom(n, 56, 56, 64, 64, 3, 3, 1, 1, 64, 3)
    x = torch.randn(n, 56, 56, 64, device=dev).to(bf)
    w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(bf)
    y = torch.empty(n, 56, 56, 64, device=dev, dtype=bf)
    part = torch.empty(16 << 20, device=dev)
    path = os.path.join(ROOT, "gpurun_out", "halo_stamps.bin")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    os.environ["SSIP_HALO_STAMP_OUT"] = path
    for _ in range(20):
        ops.conv_fwd(g, x, w, y, part)
    lines = [f"# conv_halo_kernel fwd batch {n}, 8 waves per workgroup, s_memtime cycles {a.label}"]
    for dg in a.diags.split(","):
        if os.path.exists(path):
            os.remove(path)
        os.environ["SSIP_HALO_DIAG"] = str(128 | int(dg))
        for _ in range(5):
            ops.conv_fwd(g, x, w, y, part)
        torch.cuda.synchronize()
        os.environ.pop("SSIP_HALO_DIAG")
        st = np.fromfile(path, dtype=np.uint64).astype(np.int64).reshape(-1, 8, 32, 3)
        lines.append(f"-- ablation bits {dg} (1 no stores, 2 no MFMAs, 4 no input DMA after the first tile, "
                     f"8 no BN statistics)")
        lines += breakdown(st)
    txt = "\n".join(lines)
    print(txt, flush=True)
    if a.out:
        open(a.out, "w").write(txt + "\n")


def breakdown(st):
    G = st.shape[0]
    lines = []
    ntile = (st[:, 0, :, 0] != 0).sum(axis=1)
    kl, ep, bw, tot = [], [], [], []
    for wg in range(G):
        t = ntile[wg]
        s = st[wg, :, :t, :]
        kl.append(s[:, :, 1] - s[:, :, 0])
        ep.append(s[:, :, 2] - s[:, :, 1])
        bw.append(s[:, 1:, 0] - s[:, :-1, 2])
        tot.append(s[:, -1, 2].max() - s[:, 0, 0].min())
    kl = np.concatenate([k.ravel() for k in kl])
    ep = np.concatenate([k.ravel() for k in ep])
    bw = np.concatenate([k.ravel() for k in bw])
    per_tile = np.median(np.array(tot) / ntile)
    lines.append(f"tiles per workgroup {ntile.min()}-{ntile.max()}; workgroup span per tile (median) {per_tile:.0f} cycles")
    for nm, v in (("k-loop (barrier exit -> vmcnt(0))", kl), ("epilogue (stats + stores)", ep),
                  ("barrier wait + next-tile head", bw)):
        lines.append(f"{nm:36s} median {np.median(v):7.0f}  p10 {np.percentile(v, 10):7.0f}  "
                     f"p90 {np.percentile(v, 90):7.0f} cycles")
    lines.append(f"ideal k-loop per tile at 2 waves per SIMD with the matrix pipe never idle: 4608 cycles ({G} WGs)")
    return lines


if __name__ == "__main__":
    main()
