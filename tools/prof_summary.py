#!/usr/bin/env python3
"""Condense one GPU session's rocprofv3 output into files worth committing under profiles/<tag>/.

Inputs (written by tools/gpu_round.sh on the GPU box):
  <run>/prof_trace/run_kernel_stats.csv     rocprofv3 --kernel-trace --stats (no counters)
  <run>/prof_trace/run_kernel_trace.csv     per-dispatch trace of the same command
  <run>/prof_fetch/run_counter_collection.csv   --pmc FETCH_SIZE pass (own run)
  <run>/prof_write/run_counter_collection.csv   --pmc WRITE_SIZE pass (own run)

Outputs:
  profiles/<tag>/kernel_stats.csv   the rocprofv3 --stats summary, verbatim
  profiles/<tag>/summary.md         per-kernel table (calls, avg us, HBM bytes per launch) + bench line
  profiles/<tag>/hbm_traffic.json   per-kernel PMC bytes per launch, read by bench.py for roofline.traffic

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md § HBM: FETCH_SIZE and WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE
is taken as is.  Counter passes are separate runs of the same command (FETCH_SIZE and WRITE_SIZE do not fit one
pass).
"""
import argparse
import collections
import csv
import json
import os
import shutil


def short(name, n=64):
    name = name.replace("floam::(anonymous namespace)::", "").replace("rocprim::ROCPRIM_400200_NS::detail::", "rocprim::")
    return name if len(name) <= n else name[: n - 1] + "…"


def counters(path, counter, last=0):
    """Average KiB per dispatch of each kernel; with last > 0, over its last `last` dispatches only (the bench's
    timed region is the tail of the run)."""
    per = collections.defaultdict(list)
    if not os.path.exists(path):
        return {}
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    for r in rows:
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v[-last:] if last else v) / len(v[-last:] if last else v) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run", help="gpurun_out/<tag> directory")
    ap.add_argument("tag")
    ap.add_argument("--last", type=int, default=240,
                    help="dispatches per kernel averaged for hbm_traffic.json (the timed tail; default = 60 scans x 4 "
                         "solves)")
    ap.add_argument("--config", default="c3", help="bench config the profiled run used (bench.py keys traffic by it)")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles"))
    args = ap.parse_args()
    out = os.path.join(args.out, args.tag)
    os.makedirs(out, exist_ok=True)
    stats_csv = os.path.join(args.run, "prof_trace", "run_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(out, "kernel_stats.csv"))
    stats = list(csv.DictReader(open(stats_csv)))
    fetch = counters(os.path.join(args.run, "prof_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(args.run, "prof_write", "run_counter_collection.csv"), "WRITE_SIZE")
    fetch_t = counters(os.path.join(args.run, "prof_fetch", "run_counter_collection.csv"), "FETCH_SIZE", args.last)
    write_t = counters(os.path.join(args.run, "prof_write", "run_counter_collection.csv"), "WRITE_SIZE", args.last)
    bench = None
    bpath = os.path.join(args.run, "bench.json")
    if os.path.exists(bpath) and os.path.getsize(bpath):
        bench = json.loads(open(bpath).read().strip().splitlines()[-1])

    traffic = {}
    lines = [f"# rocprofv3 summary — {args.tag}", "",
             f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --cpu-baseline-seconds 0` ({args.config}, 8 warm-up + "
             "60 timed scans, then the same 68 scans replayed with per-launch events for the roofline; all dispatches of the run, map prefill included).  HBM bytes: separate "
             "`--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` runs of the same command; FETCH_SIZE doubled (gfx950 16-B/lane "
             "read correction), KiB → bytes.", "",
             "| kernel | calls | total us | avg us | % | HBM read B/launch | HBM write B/launch |",
             "|---|---|---|---|---|---|---|"]
    for r in stats:
        name = r["Name"]
        f = fetch.get(name)
        w = write.get(name)
        rd = None if f is None else 2.0 * f * 1024.0
        wr = None if w is None else w * 1024.0
        if name in fetch_t or name in write_t:
            rt = 2.0 * fetch_t.get(name, 0.0) * 1024.0
            wt = write_t.get(name, 0.0) * 1024.0
            traffic[name] = {"read_bytes": rt, "write_bytes": wt, "total_bytes": rt + wt}
        lines.append(f"| `{short(name)}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e3:.1f} | "
                     f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['Percentage']):.2f} | "
                     f"{'' if rd is None else f'{rd:,.0f}'} | {'' if wr is None else f'{wr:,.0f}'} |")
    if bench:
        lines += ["", "## bench line of the same session (un-profiled run)", "", "```json", json.dumps(bench), "```"]
    open(os.path.join(out, "summary.md"), "w").write("\n".join(lines) + "\n")
    json.dump({"source": f"profiles/{args.tag}", "config": args.config, "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate runs; "
               f"FETCH_SIZE x2 (gfx950), KiB->B; average over the kernel's last {args.last} dispatches (timed tail)",
               "kernels": traffic},
              open(os.path.join(out, "hbm_traffic.json"), "w"), indent=1)
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main()
