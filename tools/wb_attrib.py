#!/usr/bin/env python3
"""Own HBM write bytes of the kernels bracketed by FLOAM_PROF_WB=1 (floam_amd/csrc/profwb.hpp): from a rocprofv3
`--pmc WRITE_SIZE` (or FETCH_SIZE) counter CSV, every dispatch X that sits between two `l2_writeback` dispatches
is charged WRITE_SIZE(X) + WRITE_SIZE(the write-back after it) — the lines X dirtied and left in L2 are written back
by that dispatch, and the write-back before it left no earlier kernel's dirty lines to be evicted during X.
Usage: python tools/wb_attrib.py <run_counter_collection.csv> [COUNTER] [--json out.json]"""
import collections
import csv
import json
import sys


def main():
    path = sys.argv[1]
    counter = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "WRITE_SIZE"
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    per = {}
    for r in rows:   # (a dispatch may carry one row per counter instance: sum them)
        d = int(r["Dispatch_Id"])
        name, v = r["Kernel_Name"], float(r["Counter_Value"])
        if d in per:
            per[d] = (name, per[d][1] + v)
        else:
            per[d] = (name, v)
    seq = [per[d] for d in sorted(per)]
    own = collections.defaultdict(list)
    during = collections.defaultdict(list)
    after = collections.defaultdict(list)
    for i in range(1, len(seq) - 1):
        if "l2_writeback" in seq[i - 1][0] and "l2_writeback" in seq[i + 1][0] and "l2_writeback" not in seq[i][0]:
            name = seq[i][0]
            during[name].append(seq[i][1] * 1024.0)
            after[name].append(seq[i + 1][1] * 1024.0)
            own[name].append((seq[i][1] + seq[i + 1][1]) * 1024.0)
    out = {}
    for name in own:
        n = len(own[name])
        out[name] = {"dispatches": n, "during_bytes": sum(during[name]) / n, "writeback_after_bytes": sum(after[name]) / n,
                     "own_bytes": sum(own[name]) / n}
        print(f"{name[:70]:70s} n={n:4d} during {out[name]['during_bytes'] / 1e6:8.3f} MB  after "
              f"{out[name]['writeback_after_bytes'] / 1e6:8.3f} MB  own {out[name]['own_bytes'] / 1e6:8.3f} MB")
    if "--json" in sys.argv:
        json.dump({"counter": counter, "unit": "bytes per dispatch (KiB x 1024)", "kernels": out},
                  open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
