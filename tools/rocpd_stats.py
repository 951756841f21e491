#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (kernel trace) as a per-kernel stats table.

Usage: python tools/rocpd_stats.py <run_results.db> [--csv out.csv] [--since-dispatch N]
Columns: kernel, calls, total_us, avg_us, min_us, max_us, pct, vgpr, sgpr, lds, scratch.
"""
import argparse
import collections
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default="")
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    con = sqlite3.connect(args.db)
    cur = con.cursor()
    rows = cur.execute(
        "select s.display_name, d.end - d.start, s.arch_vgpr_count, s.accum_vgpr_count, s.sgpr_count, "
        "d.group_segment_size, d.private_segment_size "
        "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
    agg = collections.OrderedDict()
    for name, dur, vg, ag, sg, lds, scr in rows:
        a = agg.setdefault(name, {"n": 0, "tot": 0, "min": 1 << 62, "max": 0, "vgpr": vg + (ag or 0), "sgpr": sg,
                                  "lds": lds, "scratch": scr})
        a["n"] += 1
        a["tot"] += dur
        a["min"] = min(a["min"], dur)
        a["max"] = max(a["max"], dur)
    total = sum(a["tot"] for a in agg.values()) or 1
    items = sorted(agg.items(), key=lambda kv: -kv[1]["tot"])
    hdr = "kernel,calls,total_us,avg_us,min_us,max_us,pct,vgpr,sgpr,lds_bytes,scratch_bytes"
    lines = [hdr]
    for name, a in items:
        short = name if len(name) < 90 else name[:87] + "..."
        lines.append(f"\"{short}\",{a['n']},{a['tot'] / 1e3:.1f},{a['tot'] / a['n'] / 1e3:.2f},{a['min'] / 1e3:.2f},"
                     f"{a['max'] / 1e3:.2f},{100.0 * a['tot'] / total:.1f},{a['vgpr']},{a['sgpr']},{a['lds']},"
                     f"{a['scratch']}")
    out = "\n".join(lines[: args.top + 1])
    print(out)
    if args.csv:
        with open(args.csv, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    sys.exit(main())


def per_scan(db, marker="fe_keys", last=10):
    """Per-scan kernel-time breakdown over the last `last` scans, using `marker` dispatches as scan starts."""
    con = sqlite3.connect(db)
    rows = con.execute(
        "select s.display_name, d.start, d.end from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
        "on d.kernel_id = s.id order by d.start").fetchall()
    starts = [r[1] for r in rows if marker in r[0]]
    if len(starts) < last + 1:
        last = len(starts) - 1
    t0, t1 = starts[-last - 1], rows[-1][2]
    agg = collections.Counter()
    cnt = collections.Counter()
    busy = 0
    for name, s, e in rows:
        if s >= t0:
            short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
            agg[short] += e - s
            cnt[short] += 1
            busy += e - s
    n = last + 1
    print(f"scans={n} wall/scan={(t1 - t0) / n / 1e3:.1f}us kernel-busy/scan={busy / n / 1e3:.1f}us "
          f"dispatches/scan={sum(cnt.values()) / n:.0f}")
    for k, v in agg.most_common(25):
        print(f"  {v / n / 1e3:8.1f}us/scan  {cnt[k] / n:5.1f}x  {k}")
