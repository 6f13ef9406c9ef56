#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per kernel (substring filter): pmc_summary.py <csv...> [--kernel S]"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
filt = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "fm_gemm_kernel"
vals = defaultdict(list)
meta = {}
for path in args:
    if path == filt:
        continue
    for row in csv.DictReader(open(path)):
        if filt not in row["Kernel_Name"]:
            continue
        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        meta = {k: row[k] for k in ("VGPR_Count", "Accum_VGPR_Count", "LDS_Block_Size", "Grid_Size", "Workgroup_Size")}
        meta["dur_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
print(meta)
for k, v in sorted(vals.items()):
    print(f"{k:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
