"""CPU checks of the measurement post-processors the committed profiles come
from: tools/roofline_from_trace.py (the conv-family fraction recomputed from a
rocprofv3 kernel trace of one bench leg) and tools/pmc_traffic.py (HBM bytes
per step from separate FETCH_SIZE / WRITE_SIZE passes: FETCH doubled for
gfx950, KiB per dispatch, grouped by family over the last complete step).
Synthetic CSVs with the rocprofv3 column names; expected values by hand."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, header, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=header)
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_roofline_from_trace(tmp_path):
    # two steps; only the last (from the last weight_prep_batch launch) counts
    names = ["weight_prep_batch_kernel", "void conv_glds_kernel<0, 128, 128, 4, 2, 2>(ConvArgs)",
             "bn_apply_kernel", "void conv_halo_kernel<4, 2>(HaloArgs)", "wgrad_reduce_kernel(float const*)"]
    durs = [5000, 40000, 9000, 20000, 1000]  # ns
    rows, t = [], 0
    for _ in range(2):
        for n, d in zip(names, durs):
            rows.append({"Kernel_Name": n, "Start_Timestamp": t, "End_Timestamp": t + d})
            t += d + 500
    p = tmp_path / "trace.csv"
    _write(p, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"], rows)
    out = tmp_path / "leg.txt"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline_from_trace.py"), str(p), "--tflop",
                        "0.0305", "--out", str(out)], capture_output=True, text=True, check=True)
    conv_us = (40000 + 20000 + 1000) / 1e3  # conv_glds + conv_halo + wgrad_reduce of the last step
    ach = 0.0305 / (conv_us * 1e-6)
    head = out.read_text().splitlines()[1]
    assert "3 launches" in head and f"{conv_us:.1f} us" in head
    assert f"frac {ach / 2500:.4f}" in head, (head, r.stdout)


def test_pmc_traffic(tmp_path):
    def rows(counter, vals):
        out, d = [], 0
        for _ in range(2):  # two steps, then a third head closing the second
            for n, v in vals:
                out.append({"Dispatch_Id": d, "Kernel_Name": n, "Counter_Name": counter, "Counter_Value": v})
                d += 1
        out.append({"Dispatch_Id": d, "Kernel_Name": "weight_prep_batch_kernel", "Counter_Name": counter,
                    "Counter_Value": 0})
        return out
    step = [("weight_prep_batch_kernel", 1.0), ("void conv_glds_kernel<0>(ConvArgs)", 100.0),
            ("bn_apply_kernel<__bf16>", 30.0), ("adamw_dev_kernel", 5.0)]
    hdr = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"]
    fe, wr = tmp_path / "fetch.csv", tmp_path / "write.csv"
    _write(fe, hdr, rows("FETCH_SIZE", step))
    _write(wr, hdr, rows("WRITE_SIZE", [(n, v / 2) for n, v in step]))
    out = tmp_path / "traffic.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(fe), str(wr), str(out),
                    "key bs1"], capture_output=True, text=True, check=True)
    d = json.load(open(out))
    kib = 1024.0
    assert d["conv"]["read_bytes"] == 2 * 100 * kib and d["conv"]["write_bytes"] == 50 * kib
    assert d["bn"]["total_bytes"] == 2 * 30 * kib + 15 * kib
    assert d["adamw"]["read_bytes"] == 2 * 5 * kib
    assert d["_workload"] == "key bs1"
    assert sum(v["total_bytes"] for v in d["bn_kernels"].values()) == d["bn"]["total_bytes"]
