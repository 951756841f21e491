"""bench.py's roofline bookkeeping (CPU): the committed PMC profile a bench line cites is chosen by the device-code
hash it recorded, then by its step count and time stamp — never by directory-name order — and its
rocprof average for the kernel comes with it."""
import json
import os

import bench


def _profile(root, tag, config, code_hash, steps, created, total, avg_us):
    d = root / "profiles" / tag
    d.mkdir(parents=True)
    doc = {"source": f"profiles/{tag}", "config": config, "steps": steps, "code_hash": code_hash,
           "kernels": {"knn_kernel<16, 2, 6, 3, 0>": {"read_bytes": total, "write_bytes": 0.0, "total_bytes": total}}}
    if created is not None:
        doc["created"] = created
    (d / "hbm_traffic.json").write_text(json.dumps(doc))
    (d / "kernel_stats.csv").write_text("Name,Calls,CallsPerScan,TotalUs,AvgUs,MinUs,MaxUs,Percentage\n"
                                        f"\"knn_kernel<16, 2, 6, 3, 0>\",80,4.00,1.0,{avg_us},1.0,1.0,10.0\n")


def test_traffic_profile_chosen_by_code_hash(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "code_hash", lambda: "cafe")
    _profile(tmp_path, "r05u", "c3", None, 60, None, 1.0e6, 25.0)            # older, no hash (sorts last by name)
    _profile(tmp_path, "r06a", "c3", "beef", 20, "2026-10-18T10:00:00Z", 2.0e6, 23.0)   # other code
    _profile(tmp_path, "r06b", "c3", "cafe", 60, "2026-10-18T09:00:00Z", 3.0e6, 22.0)   # this code, other steps
    _profile(tmp_path, "r06c", "c3", "cafe", 20, "2026-10-18T08:00:00Z", 4.0e6, 21.5)   # this code and steps
    _profile(tmp_path, "r06d", "c5", "cafe", 20, "2026-10-18T11:00:00Z", 5.0e6, 40.0)   # other config
    t = bench.hbm_traffic("knn_kernel<", "c3", 20)
    assert t["source"] == os.path.join("profiles", "r06c", "hbm_traffic.json")
    assert t["bytes"] == 4000000 and t["rocprof_avg_us"] == 21.5
    assert t["code_match"] and t["steps_match"]
    t = bench.hbm_traffic("knn_kernel<", "c3", 60)   # the steps decide among this code's profiles
    assert t["source"].endswith(os.path.join("r06b", "hbm_traffic.json"))
    monkeypatch.setattr(bench, "code_hash", lambda: "dead")   # no profile of this code: the newest of the config
    t = bench.hbm_traffic("knn_kernel<", "c3", 20)
    assert t["source"].endswith(os.path.join("r06a", "hbm_traffic.json")) and not t["code_match"]
    assert bench.hbm_traffic("knn_kernel<", "c2", 20) is None


def test_code_hash_tracks_device_sources():
    h = bench.code_hash()
    assert len(h) == 16 and int(h, 16) >= 0
    assert bench.code_hash() == h   # deterministic
