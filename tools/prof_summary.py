#!/usr/bin/env python3
"""Condense one GPU session's rocprofv3 output into files worth committing under profiles/<tag>/.

Inputs (written by tools/gpu_prof.sh on the GPU box):
  <run>/prof_trace/run_kernel_trace.csv     rocprofv3 --kernel-trace --stats (no counters), per dispatch
  <run>/prof_trace/run_kernel_stats.csv     the --stats summary of the same run (whole process)
  <run>/prof_fetch/run_counter_collection.csv   --pmc FETCH_SIZE pass (own run)
  <run>/prof_write/run_counter_collection.csv   --pmc WRITE_SIZE pass (own run)

The bench marks its timed region with two `floam_profile_marker` dispatches on the library stream
(floam_profile_mark, bench.py).  Every table here is restricted to that region: kernel-trace dispatches that start
after the first marker ends and end before the second starts (all streams), and counter rows whose Dispatch_Id lies
between the two markers' dispatch ids.  Runs without markers fall back to the whole trace (noted in the summary).

Outputs:
  profiles/<tag>/kernel_stats.csv   per-kernel calls / total / avg / min / max over the timed region
  profiles/<tag>/kernel_stats_whole_run.csv   the rocprofv3 --stats summary, verbatim (prefill, replay included)
  profiles/<tag>/summary.md         per-kernel table (calls per scan, avg us, HBM bytes per launch) + bench line
  profiles/<tag>/hbm_traffic.json   per-kernel PMC bytes per launch (timed region), read by bench.py's roofline,
                                    with the profiled tree's device-code hash (code_hash.txt), steps and a timestamp

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md § HBM: FETCH_SIZE and WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE
is taken as is.  Counter passes are separate runs of the same command (FETCH_SIZE and WRITE_SIZE do not fit one
pass).
"""
import argparse
import collections
import csv
import datetime
import json
import os
import shutil

MARKER = "floam_profile_marker"


def short(name, n=64):
    name = name.replace("floam::(anonymous namespace)::", "").replace("rocprim::ROCPRIM_400200_NS::detail::", "rocprim::")
    return name if len(name) <= n else name[: n - 1] + "…"


def trace_region(path):
    """(rows in the timed region, marked?) of a kernel_trace.csv."""
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["_s"], r["_e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["_s"])
    marks = [r for r in rows if MARKER in r["Kernel_Name"]]
    if len(marks) < 2:
        return rows, False, None
    t0, t1 = marks[0]["_e"], marks[1]["_s"]
    return [r for r in rows if r["_s"] >= t0 and r["_e"] <= t1 and MARKER not in r["Kernel_Name"]], True, (t0, t1)


def counters(path, counter):
    """Average KiB per dispatch of each kernel over the timed region (between the markers' dispatch ids)."""
    if not os.path.exists(path):
        return {}, False
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    marks = sorted(int(r["Dispatch_Id"]) for r in rows if MARKER in r["Kernel_Name"])
    marked = len(marks) >= 2
    per = collections.defaultdict(list)
    for r in rows:
        d = int(r["Dispatch_Id"])
        if MARKER in r["Kernel_Name"] or (marked and not marks[0] < d < marks[1]):
            continue
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}, marked


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run", help="gpurun_out/<tag> directory")
    ap.add_argument("tag")
    ap.add_argument("--config", default="c3", help="bench config the profiled run used (bench.py keys traffic by it)")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed scans of the profiled bench run (default: the session's bench.json steps, else 60)")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles"))
    args = ap.parse_args()
    out = os.path.join(args.out, args.tag)
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(args.run, "prof_trace", "run_kernel_stats.csv"),
                os.path.join(out, "kernel_stats_whole_run.csv"))
    bpath = os.path.join(args.run, "bench.json")
    if args.steps is None:
        args.steps = 60
        if os.path.exists(bpath) and os.path.getsize(bpath):
            args.steps = int(json.loads(open(bpath).read().strip().splitlines()[-1]).get("steps", 60))
    rows, marked, span = trace_region(os.path.join(args.run, "prof_trace", "run_kernel_trace.csv"))
    per = collections.defaultdict(list)
    for r in rows:
        per[r["Kernel_Name"]].append((r["_e"] - r["_s"]) / 1e3)
    total = sum(sum(v) for v in per.values())
    stats = sorted(per.items(), key=lambda kv: -sum(kv[1]))
    with open(os.path.join(out, "kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "CallsPerScan", "TotalUs", "AvgUs", "MinUs", "MaxUs", "Percentage"])
        for name, d in stats:
            w.writerow([name, len(d), f"{len(d) / args.steps:.2f}", f"{sum(d):.1f}", f"{sum(d) / len(d):.2f}",
                        f"{min(d):.2f}", f"{max(d):.2f}", f"{100 * sum(d) / total:.2f}"])
    fetch, fm = counters(os.path.join(args.run, "prof_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write, wm = counters(os.path.join(args.run, "prof_write", "run_counter_collection.csv"), "WRITE_SIZE")
    bench = None
    bpath = os.path.join(args.run, "bench.json")
    if os.path.exists(bpath) and os.path.getsize(bpath):
        bench = json.loads(open(bpath).read().strip().splitlines()[-1])
    region = (f"the timed region only ({args.steps} scans between the bench's two `{MARKER}` dispatches, "
              f"{(span[1] - span[0]) / 1e6:.2f} ms of trace)" if marked else
              "the WHOLE run (no markers found: prefill and replay included)")
    lines = [f"# rocprofv3 summary — {args.tag}", "",
             f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --cpu-baseline-seconds 0 --no-secondary` "
             f"({args.config}).  Dispatches of {region}.  HBM bytes: separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` "
             "runs of the same command, restricted the same way by dispatch id "
             f"({'marked' if fm and wm else 'unmarked'}); FETCH_SIZE doubled (gfx950 16-B/lane read correction), "
             "KiB → bytes.  Kernel time sums over all streams (the feature extraction overlaps the odometry).", "",
             "| kernel | calls | per scan | total us | avg us | min us | max us | % | HBM read B/launch | HBM write B/launch |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    traffic = {}
    for name, d in stats:
        f = fetch.get(name)
        wv = write.get(name)
        rd = None if f is None else 2.0 * f * 1024.0
        wr = None if wv is None else wv * 1024.0
        if rd is not None or wr is not None:
            traffic[name] = {"read_bytes": rd or 0.0, "write_bytes": wr or 0.0, "total_bytes": (rd or 0.0) + (wr or 0.0)}
        lines.append(f"| `{short(name)}` | {len(d)} | {len(d) / args.steps:.2f} | {sum(d):.1f} | {sum(d) / len(d):.2f} | "
                     f"{min(d):.2f} | {max(d):.2f} | {100 * sum(d) / total:.2f} | "
                     f"{'' if rd is None else f'{rd:,.0f}'} | {'' if wr is None else f'{wr:,.0f}'} |")
    lines += ["", f"Kernel time per scan (all streams): {total / args.steps:.1f} us; dispatches per scan: "
              f"{sum(len(d) for d in per.values()) / args.steps:.2f}"]
    if bench:
        lines += ["", "## bench line of the same session (un-profiled run)", "", "```json", json.dumps(bench), "```"]
    open(os.path.join(out, "summary.md"), "w").write("\n".join(lines) + "\n")
    chash = None
    hpath = os.path.join(args.run, "code_hash.txt")
    if os.path.exists(hpath):
        chash = open(hpath).read().strip() or None
    json.dump({"source": f"profiles/{args.tag}", "config": args.config, "steps": args.steps, "code_hash": chash,
               "created": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
               "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate runs; FETCH_SIZE x2 (gfx950), KiB->B; "
                         "average over the dispatches of the timed region (between the bench's marker dispatches)",
               "kernels": traffic},
              open(os.path.join(out, "hbm_traffic.json"), "w"), indent=1)
    print("\n".join(lines[:50]))


if __name__ == "__main__":
    main()
