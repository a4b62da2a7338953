"""Experiment: envs per 64-lane wave (COG_ROLLOUT_NL) against shard size.  Prints, per (n, NL),
the rollout's device us/step in 1,000-step launches and the wall us/step of one 20-step call."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("COG_PKG_ROOT") or os.path.join(ROOT, "gym-eldorado_amd"))
import city_of_gold as cg  # noqa: E402


def run(n, nl):
    os.environ["COG_ROLLOUT_NL"] = str(nl)
    env = cg.vec.get_vec_env(n)(device=0)
    smp = cg.vec.get_vec_sampler(n)(12345, device=0)
    env.reset(12345, 4, 3, cg.HARD, 100000, False)
    r = cg.vec.get_runner(n)(env, smp, None, device_views=True)
    r.set_chunk(1000)
    r.rollout(200)
    r.sync()
    r.set_timing(True)
    r.rollout(2000)
    ms, done = r.kernel_time()
    r.set_timing(False)
    us_k = ms * 1e3 / max(done, 1)
    r.set_chunk(20)
    best = 1e9
    for _ in range(10):
        r.sync()
        t0 = time.perf_counter()
        r.rollout(20)
        r.sync()
        best = min(best, time.perf_counter() - t0)
    print(f"n={n:6d} NL={nl:2d}  us/step(1000)={us_k:6.3f}  G/s={n/us_k/1e3:6.2f}   "
          f"20-step wall us/step={best/20*1e6:6.3f}  G/s={n*20/best/1e9:6.2f}", flush=True)
    del r, smp, env


for n in [int(x) for x in sys.argv[1].split(",")]:
    for nl in [int(x) for x in sys.argv[2].split(",")]:
        run(n, nl)
