"""Diagnostic: steady full dynamics (stored masks, max_steps 100,000) at 65,536 envs with each
rollout kernel ($COG_ROLLOUT is read once per process: one kernel per run).
    COG_ROLLOUT=wave|pipe|duo python tools/fd_kinds.py [envs]
$COG_PKG: the directory holding the city_of_gold package to load (a same-box A/B against another
engine build; default gym-eldorado_amd)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("COG_PKG") or os.path.join(ROOT, "gym-eldorado_amd"))
import city_of_gold as cg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
env = cg.vec.get_vec_env(n)(device=0)
smp = cg.vec.get_vec_sampler(n)(12345, device=0)
env.reset(12345, 4, 3, cg.HARD, 100000, False)
r = cg.vec.get_runner(n)(env, smp, None, device_views=True, stored_masks=True)
r.set_chunk(1000)
r.rollout(200)
r.sync()
r.set_timing(True)
t0 = time.perf_counter()
r.rollout(2000)
r.sync()
wall = time.perf_counter() - t0
ms, k = r.kernel_time()
print("%s%s n=%d  %.3f us/step wall, %.3f us/step device  %.3g env-steps/s" % (
    os.environ.get("COG_ROLLOUT", "auto"), " [%s]" % os.environ["COG_PKG"] if os.environ.get("COG_PKG") else "", n, wall / 2000 * 1e6, ms * 1e3 / max(k, 1), n * 2000 / wall))
