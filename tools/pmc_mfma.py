"""MFMA utilisation per kernel from one rocprofv3 --pmc pass
(SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE, SQ_WAVE_CYCLES, SQ_WAIT_ANY,
SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_BUSY_CYCLES; tools/gpu_r2.sh mfma).

  MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (kernel-trace duration x SCLK x 256 CUs x 4 SIMDs)
  (SCLK: --sclk-mhz, the bench line's `sclk.mean_mhz` of the same box; the
  chip's ceiling is 2,400 MHz).  Round 4 normalised by GRBM_GUI_ACTIVE / 8,
  which reads 2.5-10 "GHz" over short or lightly loaded dispatches -- above the
  chip's clock, so it over-counts cycles and biased those rows low; the
  GUI-based figure is kept as a column (gui_mfma) for comparison.

SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe cycles per SIMD (16 per
v_mfma_f32_16x16x32_bf16), so MFMA busy is the fraction of the chip's SIMD
cycles inside the dispatch spent in MFMAs -- the "MFMA utilisation" the north
star asks for.  Dispatches of the last complete step (between the last two
AdamW launches) are grouped by kernel.

usage: pmc_mfma.py run_counter_collection.csv [out.txt] [--sclk-mhz 2335]
"""
import collections
import csv
import re
import sys

CUS, SIMDS, XCDS = 256, 4, 8


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\((?![^<]*>).*", "", name)  # drop the argument list, keep template args
    return name[:80]


def family(n):
    if any(k in n for k in ("conv_glds_kernel", "conv_gemm_kernel", "conv_halo", "conv_stem", "wgrad_reduce")):
        return "conv"
    for k in ("bn_", "stem_", "augment", "adamw", "avgpool", "weight_prep"):
        if k in n:
            return k.rstrip("_")
    return "other"


argv = list(sys.argv[1:])
SCLK_MHZ = 2400.0
if "--sclk-mhz" in argv:
    i = argv.index("--sclk-mhz")
    SCLK_MHZ = float(argv[i + 1])
    del argv[i:i + 2]
rows = list(csv.DictReader(open(argv[0])))
disp = collections.OrderedDict()
for r in rows:
    d = disp.setdefault(r["Dispatch_Id"], {"name": r["Kernel_Name"], "t": (int(r["Start_Timestamp"]),
                                                                          int(r["End_Timestamp"]))})
    d[r["Counter_Name"]] = float(r["Counter_Value"])
ds = list(disp.values())
HAVE_COEXEC = any("SQ_VALU_MFMA_COEXEC_CYCLES" in d for d in ds)
idx = [i for i, d in enumerate(ds) if "weight_prep_batch" in d["name"] and
       (i == 0 or "weight_prep_batch" not in ds[i - 1]["name"])]  # the step head (1-2 launches)
step = ds[idx[-2] + 1: idx[-1] + 1]
agg = collections.defaultdict(lambda: collections.Counter())
fam = collections.defaultdict(lambda: collections.Counter())
for d in step:
    dur = (d["t"][1] - d["t"][0]) * 1e-9
    for tgt in (agg[short(d["name"])], fam[family(d["name"])]):
        tgt["n"] += 1
        tgt["dur"] += dur
        tgt["gui"] += d.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                  "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES", "SQ_VALU_MFMA_COEXEC_CYCLES"):
            tgt[c] += d.get(c, 0.0)

lines = ["# MFMA busy per kernel, one step of `bench.py` (rocprofv3 --pmc, profiled clocks run lower than",
         f"# unprofiled: MI355X_MICROARCH.md DVFS item 2).  mfma = MFMA_BUSY / (trace duration * {SCLK_MHZ:.0f} MHz"
         " * 1024 SIMDs);",
         "# gui_mfma = MFMA_BUSY / (GUI_ACTIVE/8 * 1024 SIMDs) (round 4's normalisation; guiGHz = GUI_ACTIVE/8 / us);",
         "# wait/inst = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY as fractions of SQ_WAVE_CYCLES;",
         "# coexec = SQ_VALU_MFMA_COEXEC_CYCLES (vector and matrix instructions executing together) normalised as mfma",
         "# (blank when the pass did not collect it)",
         f"{'kernel':82s} {'n':>3s} {'us':>8s} {'mfma':>6s} {'guiGHz':>6s} {'gui_mfma':>8s} {'wait':>5s} {'winst':>5s}"
         f" {'active':>6s} {'coexec':>6s}"]


def fmt(k, v):
    wc = max(v["SQ_WAVE_CYCLES"], 1.0)
    util = v["SQ_VALU_MFMA_BUSY_CYCLES"] / max(v["dur"] * SCLK_MHZ * 1e6 * CUS * SIMDS, 1.0)
    gutil = v["SQ_VALU_MFMA_BUSY_CYCLES"] / max(v["gui"] * CUS * SIMDS, 1.0)
    ghz = v["gui"] / max(v["dur"], 1e-12) / 1e9
    co = v["SQ_VALU_MFMA_COEXEC_CYCLES"] / max(v["dur"] * SCLK_MHZ * 1e6 * CUS * SIMDS, 1.0)
    cos = f"{co:6.1%}" if HAVE_COEXEC else ""
    return (f"{k:82s} {int(v['n']):3d} {v['dur'] * 1e6:8.1f} {util:6.1%} {ghz:6.2f} {gutil:8.1%} "
            f"{v['SQ_WAIT_ANY'] / wc:5.2f} {v['SQ_WAIT_INST_ANY'] / wc:5.2f} {v['SQ_ACTIVE_INST_ANY'] / wc:6.2f} {cos}")


for k, v in sorted(agg.items(), key=lambda kv: -kv[1]["dur"]):
    lines.append(fmt(k, v))
lines.append("# by family")
for k, v in sorted(fam.items(), key=lambda kv: -kv[1]["dur"]):
    lines.append(fmt(k, v))
txt = "\n".join(lines)
print(txt)
if len(argv) > 1:
    open(argv[1], "w").write(txt + "\n")
