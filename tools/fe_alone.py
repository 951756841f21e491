"""featureExtraction alone on C3 scans (diagnostic): wall-clock scans/s of the asynchronous extraction with 3
rotating output buffers (as bench.py's secondary), and the host time spent issuing each call.  Run under
rocprofv3 --kernel-trace for the kernels' own durations without the odometry beside them."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import floam_amd  # noqa: E402
from floam_amd import _ffi, synth  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    steps, warm = 60, 8
    R = synth.lidar_model(cfg).rings
    params = floam_amd.LidarParams(num_lines=R, scan_period=0.1, vertical_angle=2.0, max_distance=90.0,
                                   min_distance=0.5)
    d_raw = [floam_amd.DeviceCloud(synth.generate_scan(cfg, k)) for k in range(1, steps + warm + 1)]
    bufs = [(floam_amd.DeviceCloud(), floam_amd.DeviceCloud()) for _ in range(3)]
    L = _ffi.load()
    fe = floam_amd.LaserProcessingClass(asynchronous=True)
    fe.init(params)
    host = 0.0

    def extract(k):
        nonlocal host
        t = time.perf_counter()
        e, s = bufs[k % 3]
        e.clear()
        s.clear()
        fe.featureExtraction(d_raw[k], e, s)
        host += time.perf_counter() - t

    for k in range(warm):
        extract(k)
    _ffi.check(L.floam_device_synchronize(0))
    host = 0.0
    t0 = time.perf_counter()
    for k in range(warm, warm + steps):
        extract(k)
    _ffi.check(L.floam_device_synchronize(0))
    dt = time.perf_counter() - t0
    fe.close()
    print(f"{cfg}: featureExtraction alone {steps / dt:.1f} scans/s, host issue {1e6 * host / steps:.1f} us per call")


if __name__ == "__main__":
    main()
