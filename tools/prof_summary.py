"""Summarise a rocprofv3 kernel trace (CSV): kernel time by family for one
train step (the launches between two AdamW updates; default: the third
from last, a timed graph-replayed step of bench.py).

usage: prof_summary.py run_kernel_trace.csv [step_index]
"""
import collections
import csv
import sys

path = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else -3
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))


def family(n):
    if "conv_halo_wgrad_kernel" in n or "conv_stem_wgrad_kernel" in n:
        return "conv_wgrad"
    if "conv_stem_bwd_wgrad_kernel" in n:
        return "conv_wgrad (stem, fused BN-backward apply)"
    if "conv_stem_halo_kernel" in n:
        return "conv_fwd"
    if "conv_halo_kernel" in n:
        return "conv_halo (layer1 fwd + dgrad)"
    for key in ("conv_gemm_kernel<", "conv_glds_kernel<"):
        if key in n:
            mode = n.split(key)[1][0]
            return {"0": "conv_fwd", "1": "conv_dgrad", "2": "conv_wgrad"}[mode]
    for key in ["wgrad_reduce", "bn_apply", "bn_bwd_apply", "bn_bwd_reduce", "bn_bwd_finalize", "bn_finalize",
                "stem_bn_pool_fwd", "stem_pool_bn_bwd_reduce", "stem_pool_bn_bwd_apply", "maxpool_fwd",
                "maxpool_bwd", "augment", "weight_prep", "adamw", "avgpool_fc_fwd", "avgpool_fc_bwd",
                "fc_bwd_weight", "semi_loss", "cross_entropy", "nchw_to_nhwc"]:
        if key in n:
            return key
    return "other:" + n[:50]


ends = [i for i, r in enumerate(rows) if "weight_prep_batch" in r["Kernel_Name"] and
        (i == 0 or "weight_prep_batch" not in rows[i - 1]["Kernel_Name"])]  # the step head (1-2 launches)
step = rows[ends[k - 1] + 1:ends[k] + 1]
t0 = int(rows[ends[k - 1]]["End_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in step)
fam = collections.defaultdict(lambda: [0.0, 0])
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    f = fam[family(r["Kernel_Name"])]
    f[0] += d
    f[1] += 1
tot = sum(v[0] for v in fam.values())
print(f"one step: wall {(t1 - t0) / 1e3:.1f} us, {len(step)} launches, kernel time {tot:.1f} us")
for key, (t, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
    print(f"{t:9.1f} us {100 * t / tot:5.1f}%  n={n:4d}  {key}")
conv = sum(v[0] for key, v in fam.items() if key.startswith("conv_") or key == "wgrad_reduce")
print(f"conv family (fwd+dgrad+wgrad+wgrad_reduce): {conv:.1f} us")
