"""Diagnostic: the rollout kernels launch by launch against the oracle; prints the first launch,
env and field that differ (run on the GPU box; COG_ROLLOUT selects the kernels).
    python tools/dbg_duo.py [n] [chunk] [launches] [stored 0|1] [max_steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "gym-eldorado_amd"), os.path.join(ROOT, "oracle"), ROOT):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import city_of_gold as cg  # noqa: E402
import pyoracle as po  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 5
launches = int(sys.argv[3]) if len(sys.argv) > 3 else 60
stored = int(sys.argv[4]) if len(sys.argv) > 4 else 1
max_steps = int(sys.argv[5]) if len(sys.argv) > 5 else 25
seed = 31337
env = cg.vec.get_vec_env(n)()
smp = cg.vec.get_vec_sampler(n)(seed)
env.reset(seed, 4, 3, cg.HARD, max_steps, False)
runner = cg.vec.get_runner(n)(env, smp, None, stored_masks=bool(stored), device_views=True)
runner.set_chunk(chunk)
orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
orc.reset(seed, 4, 3, 2, max_steps)
print("kind", os.environ.get("COG_ROLLOUT", "duo"), "n", n, "chunk", chunk, "stored", stored)
for L in range(launches):
    runner.rollout(chunk)
    runner.sync()
    env.sync_host()
    dones = np.zeros(n, bool)
    for _ in range(chunk):
        osm.sample(po.stored_masks(orc) if stored else orc.selected_action_masks)
        orc.step(osm.actions)
        dones |= orc.dones
    bad = None
    for nm in ("observations", "selected_action_masks", "infos"):
        for (leaf, x), (_, y) in zip(po.leaves(getattr(env, nm)), po.leaves(getattr(orc, nm))):
            ne = (x != y).reshape(n, -1).any(1)
            if ne.any():
                bad = (nm, leaf, np.nonzero(ne)[0][:8])
                break
        if bad:
            break
    if bad is None:
        for nm in ("rewards", "dones", "agent_selection"):
            a, b = getattr(env, nm), getattr(orc, nm)
            ne = (a != b).reshape(n, -1).any(1)
            if ne.any():
                bad = (nm, "", np.nonzero(ne)[0][:8])
                break
    if bad:
        e = int(bad[2][0])
        print(f"launch {L} (steps {L * chunk}..{(L + 1) * chunk - 1}): {bad[0]}.{bad[1]} differs, envs {bad[2]}; "
              f"env {e} had an episode end in this launch: {bool(dones[e])}")
        if bad[0] == "observations":
            x = env.observations[e]
            y = orc.observations[e]
            for leaf, a in po.leaves(x[None]):
                b = dict(po.leaves(y[None]))[leaf]
                if not np.array_equal(a, b):
                    print("  ", leaf, "engine", a.ravel()[:24], "\n   ", leaf, "oracle", b.ravel()[:24])
        print("engine agent", env.agent_selection[e], "oracle", orc.agent_selection[e], "dones", env.dones[e], orc.dones[e])
        sys.exit(1)
print("all launches equal")
