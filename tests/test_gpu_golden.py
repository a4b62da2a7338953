"""GPU: the HIP engine against digests produced by the UNMODIFIED reference core
(tests/golden/, oracle/gen_golden.py), the reference test KATs, the C1 config and
size-independent properties at the BASELINE sizes.  Bit-exact over named fields."""
import json
import os

import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")

with open(os.path.join(GOLD, "ref_traces.json")) as _f:
    SETS = json.load(_f)["sets"]
DIGESTS = np.load(os.path.join(GOLD, "ref_trace_digests.npz"))


def digest_env(e, actions, i):
    s = slice(i, i + 1)
    return po.step_digest(e.observations[s], e.selected_action_masks[s], e.rewards[s], e.dones[s],
                          e.agent_selection[s], e.infos[s], actions[s])


def masks_of(env, mode):
    return env.selected_action_masks if mode == "sel" else po.stored_masks(env)


@pytest.mark.parametrize("st", SETS, ids=[s["name"] for s in SETS])
def test_engine_matches_reference_traces(cg, st):
    """Host API path: sampler.sample(masks) + env.step(actions), every step checked."""
    idx = [e["index"] for e in st["envs"]]
    steps = [e["steps"] for e in st["envs"]]
    n = max(idx) + 1
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(st["sampler_seed"])
    env.reset(st["seed"], st["n_players"], st["n_pieces"], cg.Difficulty(st["difficulty"]), st["max_steps"], False)
    ref = [DIGESTS[f"{st['name']}__{k}"] for k in range(len(idx))]
    horizon = min(max(steps), 6000)
    acts = smp.get_actions()
    for t in range(horizon + 1):
        for k, i in enumerate(idx):
            if t <= steps[k]:
                assert digest_env(env, acts, i) == ref[k][t].tobytes(), \
                    f"{st['name']}: env {i} differs from the reference at step {t}"
        if t == horizon:
            break
        smp.sample(masks_of(env, st["mode"]))
        env.step(acts)


@pytest.mark.parametrize("name", ["stored_hard_ms30", "C3shape_sel_hard"])
def test_runner_fused_matches_reference(cg, name):
    """Runner path: one fused on-device sample+step kernel per step, host views at sync."""
    st = next(s for s in SETS if s["name"] == name)
    idx = [e["index"] for e in st["envs"]]
    steps = [e["steps"] for e in st["envs"]]
    n = max(idx) + 1
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(st["sampler_seed"])
    env.reset(st["seed"], 4, st["n_pieces"], cg.Difficulty(st["difficulty"]), st["max_steps"], False)
    runner = cg.vec.get_runner(n)(env, smp, 4, stored_masks=(st["mode"] == "sto"))
    ref = [DIGESTS[f"{name}__{k}"] for k in range(len(idx))]
    acts = runner.get_actions()
    for t in range(1, min(max(steps), 800) + 1):
        runner.sample()
        runner.step_sync()
        for k, i in enumerate(idx):
            if t <= steps[k]:
                assert digest_env(env, acts, i) == ref[k][t].tobytes(), f"{name}: env {i} step {t}"


def test_engine_matches_reference_maps(cg):
    with open(os.path.join(GOLD, "ref_maps.json")) as f:
        entries = json.load(f)["entries"]
    zero = np.zeros(256, dtype=po.ACTION)               # one (all-zero) action record per env
    groups = {}
    for diff, npc, seed, hexd in entries:
        groups.setdefault((diff, npc), {})[seed] = hexd
    for (diff, npc), by_seed in groups.items():
        for lo in (0, 4096, 63744, 70000):
            env = cg.vec.get_vec_env(256)()
            env.reset(lo, 4, npc, cg.Difficulty(diff), 100000, False)
            for i in range(256):
                if lo + i in by_seed:
                    assert digest_env(env, zero, i).hex() == by_seed[lo + i], f"map seed={lo + i} diff={diff}"


def test_sampler_kat(cg):
    z = np.load(os.path.join(GOLD, "ref_sampler_kat.npz"))
    masks = z["masks"].view(po.MASK).reshape(3, -1)
    acts = z["actions"].view(po.ACTION).reshape(3, -1)
    s = cg.vec.get_vec_sampler(masks.shape[1])(int(z["seed"][0]))
    for k in range(3):
        s.sample(masks[k])
        assert po.named_equal(s.get_actions(), acts[k]) is None


def test_kat_natural_end(cg):
    """test_environment.cpp:106-130 with the values the reference produces here."""
    env = cg.vec.get_vec_env(1)()
    smp = cg.vec.get_vec_sampler(1)(42)
    env.reset(54321, 4, 1, cg.EASY, 100000, False)
    steps = 0
    while True:
        smp.sample(po.stored_masks(env))
        env.step(smp.get_actions())
        steps += 1
        if env.dones[0]:
            break
    ai = env.infos[0]["agent_infos"]
    assert env.infos[0]["total_length"] == 921 and steps == 37627
    assert list(ai["returns"]) == [-1.0, 3.0, -1.0, -1.0]


def test_kat_errors(cg):
    env = cg.vec.get_vec_env(1)()
    env.reset(124, 3, 3, cg.EASY, 200, False)
    with pytest.raises(RuntimeError, match="generate map"):
        env.reset(123, 3, 4, cg.EASY, 200, False)      # test_environment.cpp:77-79
    with pytest.raises(ValueError):
        env.step(np.zeros(2, dtype=cg.ActionData))      # wrong length: ValueError, not OOB read
    with pytest.raises(ValueError):
        env.step(np.zeros(1, dtype=np.uint8))


def test_c1_config_against_oracle(cg):
    """C1: n=1, 2 players, EASY, seed 0; 20,000 steps, both driver modes (oracle-pinned:
    EASY generation cannot run on the libstdc++-11 reference build)."""
    for mode in ("sel", "sto"):
        env, smp = cg.vec.get_vec_env(1)(), cg.vec.get_vec_sampler(1)(0)
        orc, osm = po.OracleVec(1), po.OracleSampler(1, 0)
        env.reset(0, 2, 3, cg.EASY, 100000, False)
        orc.reset(0, 2, 3, 0, 100000)
        for t in range(20000 if mode == "sel" else 8000):
            smp.sample(masks_of(env, mode))
            osm.sample(masks_of(orc, mode))
            env.step(smp.get_actions())
            orc.step(osm.actions)
            if t % 97 == 0 or env.dones[0]:
                assert digest_env(env, smp.get_actions(), 0) == digest_env(orc, osm.actions, 0), f"{mode} {t}"
        assert digest_env(env, smp.get_actions(), 0) == digest_env(orc, osm.actions, 0)


@pytest.mark.parametrize("n,diff", [(8192, 1), (65536, 2)])
def test_baseline_sizes_independence(cg, n, diff):
    """C3/C4-size batches: every env i of the device batch equals a 1-env oracle run seeded
    seed+i (checked on a random subset), after device-only rollouts through the fused runner."""
    steps = 300
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(12345)
    env.reset(12345, 4, 3, cg.Difficulty(diff), 100000, False)
    runner = cg.vec.get_runner(n)(env, smp, None, device_views=True)
    runner.rollout(steps)
    runner.sync()
    env.sync_host()
    acts = smp.get_actions()
    rng = np.random.default_rng(n)
    pick = np.unique(np.concatenate([[0, n - 1], rng.choice(n, 48, replace=False)]))
    for i in pick:
        o, s = po.OracleVec(1), po.OracleSampler(1, 12345 + int(i))
        o.reset(12345 + int(i), 4, 3, diff, 100000)
        for _ in range(steps):
            s.sample(o.selected_action_masks)
            o.step(s.actions)
        for nm in ("observations", "selected_action_masks", "infos"):
            assert po.named_equal(getattr(env, nm)[i:i + 1], getattr(o, nm)) is None, f"env {i} {nm}"
        assert env.agent_selection[i] == o.agent_selection[0]
    # the host actions view is refreshed by the runner only in host mode; device mode keeps HBM
    del acts


def test_stored_mode_many_resets_against_oracle(cg):
    """Full dynamics at 1024 envs with frequent auto-resets (moves, shop, specials), all envs."""
    n, steps = 1024, 400
    env, smp = cg.vec.get_vec_env(n)(), cg.vec.get_vec_sampler(n)(3)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, 3)
    env.reset(31337, 4, 3, cg.HARD, 25, False)
    orc.reset(31337, 4, 3, 2, 25)
    runner = cg.vec.get_runner(n)(env, smp, None, stored_masks=True)
    resets = 0
    for t in range(steps):
        runner.sample()
        runner.step_sync()
        osm.sample(po.stored_masks(orc))
        orc.step(osm.actions)
        resets += int(env.dones.sum())
    for nm in ("observations", "selected_action_masks", "infos"):
        assert po.named_equal(getattr(env, nm), getattr(orc, nm)) is None, nm
    assert np.array_equal(env.rewards, orc.rewards) and np.array_equal(env.agent_selection, orc.agent_selection)
    assert resets > n // 4
    haz, per = env.hazards()
    assert np.array_equal(per, orc.flags())
