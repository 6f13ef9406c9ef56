#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV: per-kernel totals and per-step share."""
import csv
import sys


def main(path, steps=None, top=30):
    r = list(csv.DictReader(open(path)))
    tot = sum(float(x["TotalDurationNs"]) for x in r)
    lines = []
    for x in sorted(r, key=lambda x: -float(x["TotalDurationNs"]))[:top]:
        t = float(x["TotalDurationNs"])
        per = f" {t / 1e3 / steps:8.1f}us/step" if steps else ""
        lines.append(f"{t / 1e6:9.3f}ms {int(x['Calls']):6d} calls {float(x['AverageNs']) / 1e3:8.2f}us avg "
                     f"{100 * t / tot:5.1f}%{per}  {x['Name'][:120]}")
    lines.append(f"total kernel time {tot / 1e6:.3f} ms")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
