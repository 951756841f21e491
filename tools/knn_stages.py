#!/usr/bin/env python3
"""Per-round-trip read attribution of the kNN search: from a rocprofv3
`--pmc FETCH_SIZE` (or WRITE_SIZE) counter CSV of `FLOAM_KNN_STAGES=1 python bench.py` (the roofline replay runs
knn_stage_launch: the search cut after 1..4 of its dependent round trips, each launch after an L2 eviction, then the
real search after one more), the average bytes per launch of each variant.  FETCH_SIZE is in KiB and doubled (the
gfx950 16-B/lane read correction, MI355X_MICROARCH.md), as in profiles/*/hbm_traffic.json.
Usage: python tools/knn_stages.py run_counter_collection.csv [COUNTER] [--json out.json]"""
import collections
import csv
import json
import re
import sys


def main():
    path = sys.argv[1]
    counter = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "FETCH_SIZE"
    per = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        d = int(r["Dispatch_Id"])
        v = float(r["Counter_Value"])
        per[d] = (r["Kernel_Name"], per[d][1] + v if d in per else v)
    seq = [per[d] for d in sorted(per)]
    scale = 1024.0 * (2.0 if counter == "FETCH_SIZE" else 1.0)
    by = collections.defaultdict(list)
    for i in range(1, len(seq)):
        if "l2_evict" in seq[i - 1][0] and "knn_kernel" in seq[i][0]:
            m = re.search(r"knn_kernel<([^>]*)>", seq[i][0])
            args = m.group(1).split(",") if m else []
            stop = int(args[5]) if len(args) > 5 else 0
            by[stop].append(seq[i][1] * scale)
    names = {1: "query load + transform", 2: "+ coarse probes (fine-block ranges)", 3: "+ stage-1 candidate loads",
             4: "+ stage 2", 0: "+ neighbour gathers and outputs (the real search)"}
    out, prev = {}, 0.0
    for stop in (1, 2, 3, 4, 0):
        if not by[stop]:
            continue
        avg = sum(by[stop]) / len(by[stop])
        out[str(stop)] = {"stage": names[stop], "launches": len(by[stop]), "bytes": avg, "added": avg - prev}
        print(f"{names[stop]:52s} n={len(by[stop]):4d}  {avg / 1e6:7.3f} MB  (+{(avg - prev) / 1e6:6.3f} MB)")
        prev = avg
    if "--json" in sys.argv:
        json.dump({"counter": counter, "stages": out}, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
