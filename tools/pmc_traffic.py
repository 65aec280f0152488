"""HBM traffic per train step from rocprofv3 PMC passes (MI355X_MICROARCH.md
HBM section): FETCH_SIZE and WRITE_SIZE collected in SEPARATE runs (they do
not fit one TCC pass); FETCH_SIZE doubled (gfx950 tallies 128-B requests at
64 B); values are KiB per dispatch.

usage: pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv [out.json [workload-key]]
(workload-key: bench.py's `_workload` string for the profiled command, e.g.
"semi_consistency_resnet18_224 bs256 labeled128 bf16"; bench.py only reports
the traffic of a file whose key matches its own run)
Groups dispatches of the last complete step (between the last two AdamW
launches) by kernel family and prints bytes per step.
"""
import collections, csv, json, sys


def family(n):
    # every conv kernel (conv_glds / conv_gemm / conv_halo / conv_stem_halo /
    # conv_halo_wgrad / conv_stem_wgrad / conv_stem_bwd_wgrad2 -- round 4's list
    # missed the last one's "2" and counted it under "stem")
    if "conv_" in n and "_kernel" in n:
        return "conv"
    if "wgrad_reduce" in n:
        return "conv"  # the wgrad split-K reduce belongs to the conv family (as in bench.py's roofline)
    for k in ("stem_", "bn_", "maxpool", "augment", "adamw", "avgpool", "weight_prep", "semi_loss"):
        if k in n:
            return k.rstrip("_")
    return "other"


def short(n):
    import re
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    return re.sub(r"\((?![^<]*>).*", "", n)[:70]


KERN = {}


def per_step(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r.get("Counter_Name", counter) == counter]
    idx = [i for i, r in enumerate(rows) if "weight_prep_batch" in r["Kernel_Name"] and
           (i == 0 or "weight_prep_batch" not in rows[i - 1]["Kernel_Name"])]  # the step head (1-2 launches)
    a, b = idx[-2], idx[-1]
    fam = collections.Counter()
    kern = KERN.setdefault(counter, collections.Counter())
    for r in rows[a + 1:b + 1]:
        v = float(r["Counter_Value"]) * 1024.0
        fam[family(r["Kernel_Name"])] += v
        kern[short(r["Kernel_Name"])] += v
    return fam


fetch = per_step(sys.argv[1], "FETCH_SIZE")
write = per_step(sys.argv[2], "WRITE_SIZE")
out = {}
for k in sorted(set(fetch) | set(write)):
    rd = 2.0 * fetch.get(k, 0.0)
    wr = write.get(k, 0.0)
    out[k] = {"read_bytes": rd, "write_bytes": wr, "total_bytes": rd + wr}
    print(f"{k:12s} read {rd / 1e9:8.3f} GB  write {wr / 1e9:8.3f} GB  total {(rd + wr) / 1e9:8.3f} GB per step")
# per-kernel bytes of the BN family (the per-pass breakdown VERDICT r5 item 3 asks for)
bnk = {}
for k in sorted(set(KERN.get("FETCH_SIZE", {})) | set(KERN.get("WRITE_SIZE", {}))):
    if family(k) != "bn":
        continue
    rd = 2.0 * KERN["FETCH_SIZE"].get(k, 0.0)
    wr = KERN["WRITE_SIZE"].get(k, 0.0)
    bnk[k] = {"read_bytes": rd, "write_bytes": wr, "total_bytes": rd + wr}
for k, v in sorted(bnk.items(), key=lambda kv: -kv[1]["total_bytes"]):
    print(f"  bn pass {k:70s} {v['total_bytes'] / 1e9:8.3f} GB")
out["bn_kernels"] = bnk
if len(sys.argv) > 4:
    out["_workload"] = sys.argv[4]
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
