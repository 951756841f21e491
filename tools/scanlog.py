#!/usr/bin/env python3
"""Kernel-by-kernel log of one steady-state scan from a rocprofv3 kernel trace: start / end relative to the scan's
first fe_keys, queue, grid size.  usage: scanlog.py run_kernel_trace.csv [scan_index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else 20
fk = [i for i, r in enumerate(rows) if "fe_keys" in r["Kernel_Name"]]
a, b = fk[which], fk[which + 1]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[max(a - 3, 0):b + 2]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"].replace("floam::(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} dur {(e - s) / 1e3:6.1f} q{r['Queue_Id']} "
          f"g{r['Grid_Size_X']:>8s} {n[:60]}")
