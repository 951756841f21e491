"""Main-stream timeline of steady-state scans from a rocprofv3 --kernel-trace CSV.

Usage: python tools/timeline.py gpurun_out/tl/p/.../run_kernel_trace.csv [scans]
Prints, for one steady-state scan of the stream that runs knn_kernel, every kernel with its duration and the idle
gap before it, then the per-scan period / busy / idle totals averaged over the last `scans` scans.
"""
import csv
import sys


def short(name):
    n = name.replace("floam::(anonymous namespace)::", "").replace("floam::", "").replace("void ", "")
    return n.split("(")[0][:34]


def main():
    path = sys.argv[1]
    nscan = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rows = list(csv.DictReader(open(path)))
    sid = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    for r in rows:
        r["s"] = int(r["Start_Timestamp"])
        r["e"] = int(r["End_Timestamp"])
        r["n"] = short(r["Kernel_Name"])
    marks = sorted(r["s"] for r in rows if "floam_profile_marker" in r["Kernel_Name"])
    if len(marks) >= 2:   # the bench's timed region only (its replays follow the second marker)
        rows = [r for r in rows if marks[0] < r["s"] < marks[1]]
    main_stream = next(r[sid] for r in rows if r["n"].startswith("knn_kernel"))
    ms = sorted((r for r in rows if r[sid] == main_stream), key=lambda r: r["s"])
    # a scan ends with gather_status (writeback + KeyFrameUpdate) followed by the map update
    ends = [i for i, r in enumerate(ms) if r["n"] == "gather_status"]
    if len(ends) < nscan + 2:
        nscan = max(1, len(ends) - 2)
    # timed scans sit before the replay; take the last nscan full scans of the first half of the run
    half = ends[: len(ends) // 2] if len(ends) > 2 * nscan + 4 else ends
    sel = half[-nscan - 1:]
    periods, busy = [], []
    for a, b in zip(sel[:-1], sel[1:]):
        seg = ms[a + 1: b + 1]
        t0, t1 = ms[a]["e"], ms[b]["e"]
        periods.append((t1 - t0) / 1e3)
        busy.append(sum(r["e"] - r["s"] for r in seg) / 1e3)
    a, b = sel[-2], sel[-1]
    prev = ms[a]["e"]
    print(f"{'kernel':36s} {'dur us':>8s} {'gap us':>8s}")
    for r in ms[a + 1: b + 1]:
        print(f"{r['n']:36s} {(r['e'] - r['s']) / 1e3:8.2f} {(r['s'] - prev) / 1e3:8.2f}")
        prev = r["e"]
    others = {}
    for r in rows:
        if r[sid] != main_stream and ms[a]["e"] <= r["s"] <= ms[b]["e"]:
            others.setdefault(r[sid], []).append((r["n"], (r["e"] - r["s"]) / 1e3))
    for s, ks in others.items():
        print(f"stream {s}: {len(ks)} kernels, {sum(k[1] for k in ks):.1f} us: " +
              ", ".join(f"{n} {d:.1f}" for n, d in ks))
    n = len(periods)
    print(f"scans {n}: period {sum(periods) / n:.1f} us, main-stream busy {sum(busy) / n:.1f} us, "
          f"idle {(sum(periods) - sum(busy)) / n:.1f} us, launches {b - a}")


if __name__ == "__main__":
    main()
