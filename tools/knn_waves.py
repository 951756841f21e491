#!/usr/bin/env python3
"""Per-wave timeline of the latest kNN launch (FLOAM_KNN_WAVES dump, odom_kernels.hip knn_block): start | edge << 62 |
holds queries << 61 | XCC << 56, end (100 MHz).  Usage: knn_waves.py waves.bin"""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 2)
ok = a[:, 1] != 0
a = a[ok]
st = (a[:, 0] & np.uint64((1 << 56) - 1)).astype(np.int64)
en = a[:, 1].astype(np.int64)
edge = ((a[:, 0] >> np.uint64(62)) & np.uint64(1)).astype(bool)
work = ((a[:, 0] >> np.uint64(61)) & np.uint64(1)).astype(bool)
xcc = ((a[:, 0] >> np.uint64(56)) & np.uint64(15)).astype(int)
last = st.max()
m = st > last - 20000          # the latest launch only (older launches' rows are stale)
st, en, edge, work, xcc = st[m], en[m], edge[m], work[m], xcc[m]
t0 = st.min()
st, en = (st - t0) / 100.0, (en - t0) / 100.0
life = en - st
print(f"waves {len(st)} (edge {edge.sum()}, holding queries {work.sum()}), launch span {en.max():.2f} us")
for lab, mm in (("edge work", edge & work), ("surf work", ~edge & work), ("empty", ~work)):
    if mm.sum() == 0:
        continue
    print(f"{lab:10s} n {mm.sum():5d} start p0/50/90/100 {np.percentile(st[mm], [0, 50, 90, 100]).round(2)} "
          f"life p10/50/90/99/100 {np.percentile(life[mm], [10, 50, 90, 99, 100]).round(2)} "
          f"end p50/90/99/100 {np.percentile(en[mm], [50, 90, 99, 100]).round(2)}")
print("per XCC (work waves): end p50 / p99 / max")
for x in range(8):
    mm = work & (xcc == x)
    if mm.sum():
        print(f"  xcc {x}: n {mm.sum():5d} end {np.percentile(en[mm], 50):6.2f} {np.percentile(en[mm], 99):6.2f} "
              f"{en[mm].max():6.2f}  life p50 {np.percentile(life[mm], 50):5.2f}")
print("alive waves over time (work / empty):")
for t in np.arange(0, en.max() + 1.0, 1.0):
    a_w = ((st <= t) & (en > t) & work).sum()
    a_e = ((st <= t) & (en > t) & ~work).sum()
    print(f"  {t:5.1f} us  {a_w:5d} {a_e:5d}")
# the 20 latest-ending work waves
idx = np.argsort(-en * work)[:20]
print("latest-ending work waves (start, life, end, edge, xcc):")
for i in idx:
    print(f"  {st[i]:6.2f} {life[i]:6.2f} {en[i]:6.2f} {int(edge[i])} {xcc[i]}")
