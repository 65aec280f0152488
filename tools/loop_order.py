"""Print the k-loop of a kernel from hipcc device assembly as a compressed
instruction-class sequence (MFMA / ds_read / LDS-DMA / waits / barrier),
to see how a schedule interleaves them.
usage: python tools/loop_order.py file.s <mangled-symbol-prefix>"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
start = [i for i, l in enumerate(lines) if l.startswith(sys.argv[2]) and l.split(":")[0].endswith(("", ))][0]
end = start
while not lines[end].strip().startswith(".Lfunc_end"):
    end += 1
body = lines[start:end]
# the loop with the most MFMAs: a label that a later branch jumps back to
best = None
for k, l in enumerate(body):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if not m:
        continue
    back = [j for j in range(k + 1, len(body)) if "s_cbranch" in body[j] and m.group(1) in body[j]]
    if back:
        n = sum(1 for l2 in body[k:back[-1]] if "v_mfma" in l2)
        if best is None or n > best[0]:
            best = (n, k, back[-1])
_, a, b = best
seq = []
for l in body[a:b + 1]:
    t = l.strip().split()
    if not t:
        continue
    op = t[0]
    if op.startswith("v_mfma"):
        k = "M"
    elif op.startswith("ds_read"):
        k = "R"
    elif op.startswith(("buffer_load", "global_load")) and "lds" in l:
        k = "D"
    elif op == "s_waitcnt":
        k = "w(" + t[1] + ")"
    elif op == "s_barrier":
        k = "BAR"
    else:
        continue
    seq.append(k)
out = []
for k in seq:
    if out and out[-1][0] == k:
        out[-1][1] += 1
    else:
        out.append([k, 1])
print(" ".join(f"{k}{n}" if n > 1 else k for k, n in out))
