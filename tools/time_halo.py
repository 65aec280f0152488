"""Time the halo-resident 3x3 conv path against the implicit-GEMM kernels on
the ResNet-18 layer1 shapes (train batch 256, weak batch 128).  GPU box:
python tools/time_halo.py"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semi-supervised-image-processing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402
from ssip import ops  # noqa: E402
from tune_conv import time_fn  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
for N in (256, 128):
    g = ops.ConvGeom(N, 56, 56, 64, 64, 3, 3, 1, 1, 64, 3)
    x = torch.randn(N, 56, 56, 64, device=dev).to(bf)
    w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(bf)
    y = torch.empty_like(x)
    add = torch.randn_like(x)
    part = torch.empty(ops.conv_fwd_partial_floats(g), device=dev)
    res = {}
    for halo in ("1", "0"):
        os.environ["SSIP_HALO"] = halo
        res[("f", halo)] = time_fn(lambda: ops.conv_fwd(g, x, w, y, part), 20)
        res[("d", halo)] = time_fn(lambda: ops.conv_dgrad(g, x, w, y, add), 20)
    for waves in ("4",):
        os.environ["SSIP_HALO"] = "1"
        os.environ["SSIP_HALO_WAVES"] = waves
        res[("f", "w" + waves)] = time_fn(lambda: ops.conv_fwd(g, x, w, y, part), 20)
        res[("d", "w" + waves)] = time_fn(lambda: ops.conv_dgrad(g, x, w, y, add), 20)
        del os.environ["SSIP_HALO_WAVES"]
    fl = g.flops()
    for (m, k), t in res.items():
        print(f"N={N:3d} {m} {'halo8' if k == '1' else 'gemm' if k == '0' else 'halo' + k[1:]:6s} {t:8.1f} us "
              f"{fl / t / 1e6:7.0f} TF/s", flush=True)

# ablations of the halo kernel (SSIP_HALO_DBG: 1 = no MFMA, 2 = no epilogue)
g = ops.ConvGeom(256, 56, 56, 64, 64, 3, 3, 1, 1, 64, 3)
x = torch.randn(256, 56, 56, 64, device=dev).to(bf)
w = (torch.randn(64, 3, 3, 64, device=dev) * 0.05).to(bf)
y = torch.empty_like(x)
part = torch.empty(ops.conv_fwd_partial_floats(g), device=dev)
os.environ["SSIP_HALO"] = "1"
for dbg in ("0", "1", "2"):
    os.environ["SSIP_HALO_DBG"] = dbg
    t = time_fn(lambda: ops.conv_fwd(g, x, w, y, part), 20)
    t2 = time_fn(lambda: ops.conv_fwd(g, x, w, y, None), 20)
    print(f"ablation dbg={dbg}: stats {t:8.1f} us   nostats {t2:8.1f} us", flush=True)
os.environ["SSIP_HALO_DBG"] = "0"

# stem: 7x7 / stride 2 over the pre-padded NHWC4 image (conv_stem_halo_kernel vs the C4 GEMM path)
for N in (256, 128):
    g = ops.ConvGeom(N, 230, 230, 4, 64, 7, 8, 2, 0, 3, 7)
    x = torch.randn(N, 230, 230, 4, device=dev).to(bf)
    w = (torch.randn(64, 7, 8, 4, device=dev) * 0.05).to(bf)
    y = torch.empty(N, 112, 112, 64, device=dev, dtype=bf)
    part = torch.empty(ops.conv_fwd_partial_floats(g), device=dev)
    for halo in ("1", "0"):
        os.environ["SSIP_HALO"] = halo
        t = time_fn(lambda: ops.conv_fwd(g, x, w, y, part), 20)
        print(f"stem N={N} {'halo' if halo == '1' else 'gemm'} {t:8.1f} us {g.flops() / t / 1e6:7.0f} TF/s", flush=True)
os.environ["SSIP_HALO"] = "1"

# layer1 wgrad: conv_halo_wgrad_kernel vs the implicit-GEMM split-K path (incl. the slab reduce)
for N in (256,):
    g = ops.ConvGeom(N, 56, 56, 64, 64, 3, 3, 1, 1, 64, 3)
    x = torch.randn(N, 56, 56, 64, device=dev).to(bf)
    dy = torch.randn(N, 56, 56, 64, device=dev).to(bf)
    dw = torch.empty(64, 64, 3, 3, device=dev)
    ws = torch.empty(ops.conv_wgrad_workspace_bytes(g), device=dev, dtype=torch.uint8)
    for halo in ("1", "0"):
        os.environ["SSIP_HALO"] = halo
        t = time_fn(lambda: ops.conv_wgrad(g, dy, x, dw, False, ws), 20)
        print(f"wgrad N={N} {'halo' if halo == '1' else 'gemm'} {t:8.1f} us {g.flops() / t / 1e6:7.0f} TF/s", flush=True)
os.environ["SSIP_HALO"] = "1"

# stem wgrad: conv_stem_wgrad_kernel vs the implicit-GEMM split-K path (incl. the slab reduce)
g = ops.ConvGeom(256, 230, 230, 4, 64, 7, 8, 2, 0, 3, 7)
x = torch.randn(256, 230, 230, 4, device=dev).to(bf)
dy = torch.randn(256, 112, 112, 64, device=dev).to(bf)
dw = torch.empty(64, 3, 7, 7, device=dev)
ws = torch.empty(ops.conv_wgrad_workspace_bytes(g), device=dev, dtype=torch.uint8)
for halo in ("1", "0"):
    os.environ["SSIP_HALO"] = halo
    t = time_fn(lambda: ops.conv_wgrad(g, dy, x, dw, False, ws), 10)
    print(f"stem wgrad {'halo' if halo == '1' else 'gemm'} {t:8.1f} us {g.flops() / t / 1e6:7.0f} TF/s", flush=True)
os.environ["SSIP_HALO"] = "1"
