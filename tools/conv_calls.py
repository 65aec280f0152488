"""Per-launch conv kernel durations for one train step of a rocprofv3 kernel trace.
Usage: conv_calls.py trace.csv [trace2.csv]  (two traces are printed side by side)."""
import csv, sys

def tag(n):
    for k in ('conv_gemm_kernelILi', 'conv_glds_kernelILi', 'conv_glds_kernel<'):
        if k in n:
            return ('old ' if 'gemm' in k else 'glds') + n.split(k)[1][:30]
    return 'reduce' if 'wgrad_reduce' in n else None

def calls(path):
    rows = list(csv.DictReader(open(path)))
    idx = [i for i, r in enumerate(rows) if 'adamw' in r['Kernel_Name']]
    a, b = idx[-3], idx[-2]
    out = []
    for r in rows[a + 1:b + 1]:
        t = tag(r['Kernel_Name'])
        if t:
            d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
            out.append((d, int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']), int(r['Grid_Size_Y']),
                        int(r['Workgroup_Size_X']), t))
    return out

A = calls(sys.argv[1])
B = calls(sys.argv[2]) if len(sys.argv) > 2 else None
ta = tb = 0.0
for i, (d, gx, gy, wg, t) in enumerate(A):
    ta += d
    line = f"{d:8.1f}us grid={gx},{gy} wg={wg} {t}"
    if B:
        d2, gx2, gy2, wg2, t2 = B[i]
        tb += d2
        line += f"   | {d2:8.1f}us grid={gx2},{gy2} wg={wg2} {t2}   ratio={d/d2:5.2f}"
    print(line)
print(f"total {ta:.1f}us" + (f"  vs {tb:.1f}us" if B else ""))
