#!/usr/bin/env python3
"""Per-wave timeline of the last kNN launch (FLOAM_KNN_TRACE dump: 2 x u64 per wave, bit 63 of the start = the
wave's block held queries).  Usage: knn_trace.py knn.bin"""
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 2)
idx = np.arange(len(a))
valid = a[:, 1] != 0
had = (a[:, 0] >> np.uint64(63)).astype(bool)
st = (a[:, 0] & np.uint64((1 << 63) - 1)).astype(np.int64)
en = a[:, 1].astype(np.int64)
last = en[valid].max()
m = valid & (st > last - 100 * 100)   # this launch only (older launches left stale words)
st, en, had, idx = st[m], en[m], had[m], idx[m]
t0 = st.min()
st, en = (st - t0) / 100.0, (en - t0) / 100.0
print("waves", len(st), "with work", int(had.sum()), "span us", en.max())
for lab, mm in (("work", had), ("empty", ~had)):
    if mm.sum() == 0:
        continue
    life = en[mm] - st[mm]
    print(lab, "start pct", np.percentile(st[mm], [0, 10, 50, 90, 100]).round(2), "life", np.percentile(life, [10, 50, 90, 99, 100]).round(2),
          "end", np.percentile(en[mm], [50, 90, 99, 100]).round(2))
for t in np.arange(0, en.max() + 1, 1.5):
    print(f"{t:5.1f} work {((st <= t) & (en > t) & had).sum():6d} empty {((st <= t) & (en > t) & ~had).sum():5d}")
