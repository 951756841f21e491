#!/usr/bin/env python3
"""Per-scan kernel timeline from a rocprofv3 kernel trace (run_kernel_trace.csv): one steady-state scan of the
bench (between two fe_keys launches), with the GPU idle gaps, grouped into phases."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else 20
fk = [i for i, r in enumerate(rows) if "fe_keys" in r["Kernel_Name"]]
a, b = fk[which], fk[which + 1]
t0 = int(rows[a]["Start_Timestamp"])
prev = t0
busy = 0
groups = {}
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    name = r["Kernel_Name"].replace("floam::(anonymous namespace)::", "")
    name = name.split("(")[0].replace("void ", "")
    if "rocprim" in name:
        name = "rocprim::" + name.split("detail::")[-1][:40]
    if "-v" in sys.argv:
        print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:6.1f} {name[:70]}")
    g = groups.setdefault(name, [0, 0.0, 0.0])
    g[0] += 1
    g[1] += (e - s) / 1e3
    g[2] += (s - prev) / 1e3
    prev = e
wall = (int(rows[b]["Start_Timestamp"]) - t0) / 1e3
print(f"scan wall {wall:.1f} us, kernels {b - a}, busy {busy / 1e3:.1f} us, idle {wall - busy / 1e3:.1f} us")
for k, v in sorted(groups.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k[:60]:60s} x{v[0]:3d} {v[1]:8.1f} us (+gaps {v[2]:6.1f})")
