"""Kernel statistics CSV from a rocprofv3 database (`rocprofv3 --kernel-trace --stats` without
`--output-format csv` writes <dir>/<name>_results.db, the rocpd sqlite schema).

    python tools/rocpd_stats.py <results.db> <out.csv> [--skip N]

Columns follow rocprofv3's kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs) plus SteadyAverageNs: the mean over each kernel's calls after its first N (the
bench's warmup launches, which run before the clock has ramped).
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main(db, out, skip=0):
    c = sqlite3.connect(db)
    durs = defaultdict(list)
    for name, start, dur in c.execute("select name, start, duration from kernels order by start"):
        durs[name].append(float(dur))
    total = sum(sum(v) for v in durs.values())
    rows = []
    for name, v in durs.items():
        steady = v[skip:] if len(v) > skip else v
        rows.append(dict(Name=name, Calls=len(v), TotalDurationNs=sum(v),
                         AverageNs=sum(v) / len(v), Percentage=100.0 * sum(v) / total,
                         MinNs=min(v), MaxNs=max(v),
                         SteadyAverageNs=sum(steady) / len(steady)))
    rows.sort(key=lambda r: -r["TotalDurationNs"])
    with open(out, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    for r in rows[:3]:
        print(f"{r['Name'][:70]:70s} {r['Calls']:4d} avg {r['AverageNs'] / 1e3:9.1f} us "
              f"steady {r['SteadyAverageNs'] / 1e3:9.1f} us")


if __name__ == "__main__":
    a = sys.argv[1:]
    skip = 0
    if "--skip" in a:
        i = a.index("--skip")
        skip = int(a[i + 1])
        del a[i:i + 2]
    main(a[0], a[1], skip)
