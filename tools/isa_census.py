"""Instruction census of a kernel's main loop from hipcc device assembly
(static counts: a branch's instructions count once per loop body).

usage (host, no GPU):
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics --cuda-device-only -S \
      semi-supervised-image-processing_amd/csrc/conv.hip -o /tmp/conv.s
  python tools/isa_census.py /tmp/conv.s 'conv_glds_kernel<0, 128, 128, 4, 2, 2, false, false, false>' ...

For each kernel: register / LDS / occupancy figures from the compiler's
resource comments, then every loop (a label that a later branch jumps back
to), innermost first, with its instruction counts by class.  The loop with
the most MFMAs is the k-loop; its counts per MFMA are what bounds the issue
stream (MI355X_MICROARCH.md, per-instruction cycle constants).
"""
import re
import subprocess
import sys
from collections import Counter, OrderedDict

CLASSES = [
    ("mfma", re.compile(r"^v_mfma")),
    ("ds_read", re.compile(r"^ds_read")),
    ("ds_write", re.compile(r"^ds_write")),
    ("lds_dma", re.compile(r"^(buffer|global)_load\S*\b.*\blds\b")),
    ("vmem_load", re.compile(r"^(buffer|global|flat)_load")),
    ("vmem_store", re.compile(r"^(buffer|global|flat)_store")),
    ("s_waitcnt", re.compile(r"^s_waitcnt")),
    ("s_barrier", re.compile(r"^s_barrier")),
    ("s_nop", re.compile(r"^s_nop")),
    ("s_setprio", re.compile(r"^s_setprio")),
    ("branch", re.compile(r"^s_(cbranch|branch)")),
    ("salu", re.compile(r"^s_")),
    ("valu", re.compile(r"^v_")),
]


def classify(op_line: str) -> str:
    for name, rx in CLASSES:
        if rx.search(op_line):
            return name
    return "other"


def demangle_all(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return dict(zip(names, out))


def functions(path):
    """{mangled name: [lines]} of every function body in the .s file."""
    funcs = OrderedDict()
    cur = None
    with open(path) as f:
        for line in f:
            m = re.match(r"^(_Z\w+):", line)
            if m:
                cur = m.group(1)
                funcs[cur] = []
                continue
            if cur is not None:
                if line.startswith(".Lfunc_end"):
                    cur = None
                    continue
                funcs[cur].append(line.rstrip("\n"))
    return funcs


def resources(path, mangled):
    """The compiler's resource comments for one kernel (after its body)."""
    res = {}
    with open(path) as f:
        text = f.read()
    i = text.find(f".Lfunc_end")  # cheap: find the kernel's own block below
    i = text.find(mangled + ":")
    j = text.find(".Lfunc_end", i)
    blk = text[j:j + 4000]
    for key in ("NumVgprs", "NumAgprs", "TotalNumVgprs", "NumSgprs", "ScratchSize", "Occupancy",
                "LDSByteSize"):
        m = re.search(rf";\s*{key}:\s*(\d+)", blk)
        if m:
            res[key] = int(m.group(1))
    return res


def loops(lines):
    """[(label, start, end)] for every backward branch target."""
    pos = {}
    out = []
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            pos[m.group(1)] = i
        m = re.match(r"^\s+s_c?branch\w*\s+(\.LBB\w+)", l)
        if m and m.group(1) in pos and pos[m.group(1)] < i:
            out.append((m.group(1), pos[m.group(1)], i))
    return out


def census(lines, a, b):
    c = Counter()
    waits = Counter()
    for l in lines[a:b + 1]:
        s = l.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        op = s.split()[0]
        k = classify(s)
        c[k] += 1
        if op == "s_waitcnt":
            waits[s.split(None, 1)[1].split(";")[0].strip()] += 1
    return c, waits


def main():
    global flags
    path = sys.argv[1]
    flags = [a for a in sys.argv[2:] if a.startswith("-")]
    wants = [a for a in sys.argv[2:] if not a.startswith("-")]
    funcs = functions(path)
    dm = demangle_all(list(funcs))
    for want in wants:
        hits = [m for m in funcs if want in dm[m]]
        if not hits:
            print(f"== {want}: not found")
            continue
        for m in hits:
            lines = funcs[m]
            name = dm[m].replace('(anonymous namespace)::', '')
            print(f"== {name[:name.find('>(') + 1] if '>(' in name else name}")
            print(f"   resources: {resources(path, m)}")
            ls = loops(lines)
            ls.sort(key=lambda t: t[2] - t[1])
            best = None
            for lab, s, e in ls:
                c, w = census(lines, s, e)
                if c["mfma"] == 0:
                    continue
                # the k-loop: most MFMAs; among back edges to the same header
                # (a rotated loop's continue paths), the widest span, so the
                # conditionally issued loads are counted too
                if best is None or c["mfma"] > best[0]["mfma"] or (
                        c["mfma"] == best[0]["mfma"] and lab == best[2] and e - s > best[4] - best[3]):
                    best = (c, w, lab, s, e)
            if best is None:
                print("   no MFMA loop")
                continue
            if "-v" in flags:
                for lab, s_, e_ in ls:
                    c_, w_ = census(lines, s_, e_)
                    if c_["mfma"]:
                        print(f"   loop {lab} lines {s_}-{e_}: " + ", ".join(f"{k} {v}" for k, v in c_.items()))
            c, w, lab, s, e = best
            n = c["mfma"]
            tot = sum(c.values())
            print(f"   k-loop {lab}: lines {s}-{e}, {tot} instructions, {n} MFMA")
            for k, _ in CLASSES + [("other", None)]:
                if c[k]:
                    print(f"     {k:10s} {c[k]:5d}   {c[k] / n:6.2f} per MFMA")
            print(f"     waits: {dict(w)}")


if __name__ == "__main__":
    main()
