"""Diagnostic: step engine and oracle side by side (stored-mask driver) and print the first
differing fields with values."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "gym-eldorado_amd"), os.path.join(R, "oracle")]
import numpy as np
import city_of_gold as cg, pyoracle as po
seed, n, diff, ms, steps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
npl = int(sys.argv[6]) if len(sys.argv) > 6 else 4
env, smp = cg.vec.get_vec_env(n)(), cg.vec.get_vec_sampler(n)(seed)
orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
env.reset(seed, npl, 3, cg.Difficulty(diff), ms, False); orc.reset(seed, npl, 3, diff, ms)
prev_act = None
for t in range(steps):
    smp.sample(po.stored_masks(env)); osm.sample(po.stored_masks(orc))
    a_e, a_o = smp.get_actions().copy(), osm.actions.copy()
    if po.named_equal(a_e, a_o):
        print("actions differ at", t); break
    pre_obs = env.observations.copy()
    env.step(smp.get_actions()); orc.step(osm.actions)
    bad = []
    for i in range(n):
        for nm in ("observations", "selected_action_masks", "infos", "rewards", "dones", "agent_selection"):
            x, y = getattr(env, nm)[i:i+1], getattr(orc, nm)[i:i+1]
            d = po.named_equal(x, y) if x.dtype.names else (None if np.array_equal(x, y) else nm)
            if d: bad.append((i, nm, d))
    if bad:
        print("step", t, "diffs:", bad[:6])
        i = bad[0][0]
        print(" action", a_e[i], "agent before?", "agent now", env.agent_selection[i], orc.agent_selection[i])
        for (ii, nm, d) in bad[:4]:
            if ii != i: continue
            parts = d.split(".")
            x, y = getattr(env, nm)[i], getattr(orc, nm)[i]
            for p in parts:
                x, y = x[p], y[p]
            print("  ", nm, d, "\n    eng", np.asarray(x).astype(int).ravel()[:96].tolist(), "\n    orc", np.asarray(y).astype(int).ravel()[:96].tolist())
        print(" orc dbg", orc.debug_state(i)[:14])
        pd = pre_obs[i]["player_data"]["obs"]
        for p in range(npl):
            print("  before step, player", p, {f: np.asarray(pd[p][f]).astype(int).tolist() for f in pd.dtype.names})
        print("  before: phase", int(pre_obs[i]["shared"]["phase"]), "res", pre_obs[i]["shared"]["resources"].tolist())
        break
else:
    print("no divergence in", steps, "steps")
