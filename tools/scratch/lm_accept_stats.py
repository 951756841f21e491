"""CPU only: per-solve LM iterations / successful steps of the oracle on the bench sequence (C3 by default), to see
how often a candidate is rejected (the speculative reject-step question)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import oracle
from floam_amd import synth

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
R = synth.lidar_model(cfg).rings


def cpu_fe(raw, R_):
    e, s, _ = oracle.feature_extraction(raw, R_, 0.5, 90.0, canonical=True)
    return e, s


mapE, mapS = synth.prefill_map(cfg, cpu_fe, synth.MAP_PREFILL.get(cfg, 0))
oracle.reset_process_statics()
ref = oracle.Odometry(R, 0.1, 0.5, 90.0, 0.4, "Cauchy", stable_voxel=True)
ref.init_map(mapE, mapS)
it = succ = solves = 0
for k in range(1, n + 1):
    e, s = cpu_fe(synth.generate_scan(cfg, k), R)
    ref.update_selector(e, s, True)
    for t in ref.traces():
        solves += 1
        it += t["iterations"]
        succ += t["successful"]
        print(k, t["iterations"], t["successful"], round(t["initial_cost"], 4), round(t["final_cost"], 4))
    ref.clear_traces()
print(f"{solves} solves: {it} iterations, {succ} successful (incl. iteration zero)")
