"""Per-kernel PMC counter averages from a rocprofv3 --pmc results .db.
usage: python tools/pmc_db.py <pmc_results.db> [kernel-substring]"""
import collections, sqlite3, sys

c = sqlite3.connect(sys.argv[1])
sub = sys.argv[2] if len(sys.argv) > 2 else "conv_glds"
cols = [r[1] for r in c.execute("pragma table_info('counters_collection')")]
kcol = "kernel_name" if "kernel_name" in cols else [x for x in cols if "name" in x.lower() and "counter" not in x.lower()][0]
rows = c.execute(f"select {kcol}, counter_name, value, dispatch_id from counters_collection").fetchall()
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for k, cn, v, d in rows:
    if sub in k:
        acc[k[:90]][cn].append(v)
for k, d in acc.items():
    print(k)
    for cn, vs in sorted(d.items()):
        print(f"   {cn:28s} {sum(vs) / len(vs):16.4g}  (n={len(vs)})")
