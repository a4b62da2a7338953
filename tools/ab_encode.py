"""A/B the map-encode kernel variants on the bench workload (65536 envs, HARD) and check they
produce identical observations."""
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gym-eldorado_amd"))
import numpy as np
import city_of_gold as cg
n = 65536
env = cg.vec.get_vec_env(n)()
env.reset(12345, 4, 3, cg.HARD, 100000, False)
ref = None
out = {}
for v in (0, 1, 2, 0, 1, 2):
    ms = env.time_encode(30, v)
    env.sync_host()
    m = env.observations["shared"]["map"][::997].copy()
    if ref is None:
        ref = m
    assert np.array_equal(ref, m), f"variant {v} changed the output"
    out.setdefault(v, []).append(ms)
for v, ms in out.items():
    best = min(ms)
    print(json.dumps({"variant": v, "ms": best, "GBps": 18432 * n / (best / 1e3) / 1e9}))
