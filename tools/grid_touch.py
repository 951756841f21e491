#!/usr/bin/env python3
"""How much of the kNN hash grid a keyframe changes (incremental grid vs rebuild).

Runs the oracle on the bench's C3 sequence (same scans, same prefilled map) and, after every update that changed
the maps, compares the new corner / surf maps with the previous ones cell by cell on the grid's 1-m coarse cells
(grid.hpp): a coarse cell is "touched" when its multiset of float points differs.  An in-place grid update has to
rewrite at least the touched cells' point ranges (and every point's map index after the first insertion, unless the
tie-break key changes); the rebuild rewrites all of them.  CPU only (oracle/), diagnostic.
Usage: python tools/grid_touch.py [--config c3] [--scans 20]"""
import argparse
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from floam_amd import synth  # noqa: E402


def cells(m):
    xyz = m[["x", "y", "z"]] if m.dtype.names else m[:, :3]
    a = np.stack([xyz["x"], xyz["y"], xyz["z"]], 1).astype(np.float32) if m.dtype.names else xyz.astype(np.float32)
    c = np.floor(a.astype(np.float64)).astype(np.int64)
    return a, c


def by_cell(m):
    a, c = cells(m)
    d = collections.defaultdict(list)
    for p, k in zip(map(tuple, a.tolist()), map(tuple, c.tolist())):
        d[k].append(p)
    return {k: sorted(v) for k, v in d.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--scans", type=int, default=20)
    a = ap.parse_args()
    R = synth.lidar_model(a.config).rings

    def fe(raw, R_):
        e, s, _ = oracle.feature_extraction(raw, R_, 0.5, 90.0, canonical=True)
        return e, s

    mapE, mapS = synth.prefill_map(a.config, fe, synth.MAP_PREFILL.get(a.config, 0))
    oracle.reset_process_statics()
    ref = oracle.Odometry(R, 0.1, 0.5, 90.0, 0.1, "cauchy", stable_voxel=True)
    ref.init_map(mapE, mapS)
    prev = [by_cell(ref.map(0)), by_cell(ref.map(1))]
    tot = collections.defaultdict(float)
    for k in range(1, a.scans + 1):
        e, s = fe(synth.generate_scan(a.config, k), R)
        ref.update_selector(e, s, True)
        cur = [by_cell(ref.map(0)), by_cell(ref.map(1))]
        row = []
        for w in range(2):
            P, C = prev[w], cur[w]
            keys = set(P) | set(C)
            touched = [q for q in keys if P.get(q) != C.get(q)]
            npts = sum(len(v) for v in C.values())
            tpts = sum(len(C.get(q, [])) for q in touched)
            # points whose exact coordinates survive (same float triple somewhere in the map)
            ps = set(p for v in P.values() for p in v)
            kept = sum(1 for v in C.values() for p in v if p in ps)
            row.append((len(C), len(touched), npts, tpts, kept))
        changed = any(r[1] for r in row)
        if k > 2 and changed:   # the first updates replace the raw prefill (Q8), not the steady state
            for w in range(2):
                nc, tc, npts, tp, kept = row[w]
                tot[f"cells{w}"] += nc
                tot[f"touched{w}"] += tc
                tot[f"pts{w}"] += npts
                tot[f"tpts{w}"] += tp
                tot[f"kept{w}"] += kept
            tot["n"] += 1
        print(f"scan {k:3d} changed={int(changed)} " + "  ".join(
            f"{'corner' if w == 0 else 'surf'}: cells {r[0]} touched {r[1]} ({100 * r[1] / max(r[0], 1):.1f}%) "
            f"pts {r[2]} in touched cells {r[3]} ({100 * r[3] / max(r[2], 1):.1f}%) unchanged pts {r[4]}"
            for w, r in enumerate(row)), flush=True)
        prev = cur
    if tot["n"]:
        for w in range(2):
            print(f"{'corner' if w == 0 else 'surf'} over {int(tot['n'])} steady keyframes: touched cells "
                  f"{100 * tot[f'touched{w}'] / tot[f'cells{w}']:.1f}%, points in touched cells "
                  f"{100 * tot[f'tpts{w}'] / tot[f'pts{w}']:.1f}%, points with unchanged coordinates "
                  f"{100 * tot[f'kept{w}'] / tot[f'pts{w}']:.1f}%")


if __name__ == "__main__":
    main()
