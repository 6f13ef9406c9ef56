#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per-kernel totals and per-step share.

Input: the ``*_kernel_stats.csv`` of ``--stats --output-format csv`` or the ``*_results.db``
(rocpd SQLite, the default output format of rocprofv3 in ROCm 7).
usage: prof_summary.py <csv|db> [steps] [--skip-init]
"""
import csv
import sqlite3
import sys


def _rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        q = "select name, count(*), sum(duration), avg(duration) from kernels group by name"
        return [(n, int(k), float(t), float(a)) for n, k, t, a in c.execute(q)]
    r = list(csv.DictReader(open(path)))
    return [(x["Name"], int(x["Calls"]), float(x["TotalDurationNs"]), float(x["AverageNs"])) for x in r]


def main(path, steps=None, top=30):
    rows = _rows(path)
    tot = sum(t for _, _, t, _ in rows)
    lines = []
    for name, calls, t, avg in sorted(rows, key=lambda x: -x[2])[:top]:
        per = f" {t / 1e3 / steps:8.1f}us/step" if steps else ""
        lines.append(f"{t / 1e6:9.3f}ms {calls:6d} calls {avg / 1e3:8.2f}us avg {100 * t / tot:5.1f}%{per}  {name[:120]}")
    lines.append(f"total kernel time {tot / 1e6:.3f} ms")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
