"""Summarise a rocprofv3 --kernel-trace CSV per kernel, separating launches shorter than min_us
(default 8): the no-op launches of a captured iteration batch after convergence (they exit at
entry, ~4-5 us) -- and genuinely short launches such as the one-block top round of a sweep.
Usage: prof_summary.py kernel_trace.csv [min_us]"""
import collections
import csv
import sys

path = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
rows = list(csv.DictReader(open(path)))
agg = collections.defaultdict(lambda: [0, 0.0, 0, 0.0])
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:110]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg[name]
    if d >= min_us:
        a[0] += 1
        a[1] += d
    else:
        a[2] += 1
        a[3] += d
print(f"{'kernel':110s} {'live':>6s} {'avg_us':>9s} {'total_ms':>9s} {'skipped':>7s} {'skip_ms':>8s}")
for k, (n, t, ns, ts) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:110s} {n:6d} {t / max(n, 1):9.1f} {t / 1e3:9.2f} {ns:7d} {ts / 1e3:8.2f}")
