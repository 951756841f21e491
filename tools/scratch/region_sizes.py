"""CPU only: sizes of the map-merge regions a bucket = tile merge would see (scan voxels of bucket b + the map points
between its splitters), on the bench sequence with the oracle; splitters at the previous scan's quantiles."""
import sys
import numpy as np
sys.path.insert(0, ".")
import oracle
from floam_amd import synth

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
R = synth.lidar_model(cfg).rings
RES = 0.1


def cpu_fe(raw, R_):
    e, s, _ = oracle.feature_extraction(raw, R_, 0.5, 90.0, canonical=True)
    return e, s


def quat_mat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def keys(p, leaf):   # lexicographic (z, y, x) cell order as one sortable integer
    c = np.floor(p / leaf).astype(np.int64) + (1 << 20)
    return (c[:, 2] << 42) | (c[:, 1] << 21) | c[:, 0]


mapE, mapS = synth.prefill_map(cfg, cpu_fe, synth.MAP_PREFILL.get(cfg, 0))
oracle.reset_process_statics()
ref = oracle.Odometry(R, 0.1, 0.5, 90.0, RES, "Cauchy", stable_voxel=True)
ref.init_map(mapE, mapS)
prev = None
for k in range(1, n + 1):
    e, s = cpu_fe(synth.generate_scan(cfg, k), R)
    ref.update_selector(e, s, True)
    q, t = ref.pose()
    Rm = quat_mat(q)
    jobs = []
    for j, (cloud, leaf) in enumerate(((e, RES), (s, 2 * RES))):
        p = np.stack([cloud["x"], cloud["y"], cloud["z"]], 1).astype(np.float64) @ Rm.T + t
        sk = np.unique(keys(p, leaf))            # the scan's voxels (one key each)
        m = ref.map(j)
        mk = np.sort(keys(np.stack([m["x"], m["y"], m["z"]], 1).astype(np.float64), leaf))
        jobs.append((sk, mk))
    # one key space: job bit on top
    sk = np.concatenate([jobs[0][0], jobs[1][0] + (1 << 62)])
    mk = np.concatenate([jobs[0][1], jobs[1][1] + (1 << 62)])
    sk = np.sort(sk); mk = np.sort(mk)
    if prev is not None:
        spl = prev[((np.arange(1, 255) * len(prev)) // 255)]
        bs = np.searchsorted(spl, sk, side="right")
        bm = np.searchsorted(spl, mk, side="right")
        cs = np.bincount(bs, minlength=255); cm = np.bincount(bm, minlength=255)
        tot = cs + cm
        print(f"scan {k}: scan voxels {len(sk)}, map {len(mk)}; region mean {tot.mean():.0f} max {tot.max()} "
              f"p99 {np.percentile(tot, 99):.0f}; >2048: {(tot > 2048).sum()}, >1024: {(tot > 1024).sum()}; "
              f"scan part max {cs.max()}, map part max {cm.max()} (bucket {cm.argmax()})")
    prev = sk
