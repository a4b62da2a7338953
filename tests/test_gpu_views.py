"""GPU: the host views are honest about writes.

The reference's views alias the live engine state (include/pybind/common.h:98-101): a write into
`selected_action_masks` changes the deck's mask that `step` reads (src/player.cpp:16-27).  Here
the env's records live in HBM and the numpy views are pinned copies the engine never reads back,
so the env's output views are read-only: an in-place write raises instead of being silently
lost.  Inputs stay writable and are honoured: the sampler's actions view (the argument of
env.step), and masks a caller edits in a copy before `sampler.sample(masks)` -- both checked
against the C oracle fed the same edited bytes.  Also: the sampler handed the env's own mask view
while an asynchronous runner.step() is still in flight reads the masks after that step (the
sampler's stream waits for the env's), as the same calls with a sync in between do.
"""
import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu


def make(cg, n, seed, max_steps=100000):
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, 4, 3, cg.HARD, max_steps, False)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
    orc.reset(seed, 4, 3, 2, max_steps)
    return env, smp, orc, osm


def test_env_output_views_are_read_only(cg):
    n = 64
    env, smp, _, _ = make(cg, n, 5)
    runner = cg.vec.get_runner(n)(env, smp, None)
    views = {"observations": env.observations, "selected_action_masks": env.selected_action_masks,
             "infos": env.infos, "rewards": env.rewards, "dones": env.dones,
             "agent_selection": env.agent_selection, "runner.get_action_masks": runner.get_action_masks(),
             "runner.get_actions": runner.get_actions()}
    for nm, v in views.items():
        assert not v.flags.writeable, nm
    with pytest.raises(ValueError):
        env.selected_action_masks["play"][:, 1] = False
    with pytest.raises(ValueError):
        env.observations["shared"]["phase"][0] = 2
    with pytest.raises(ValueError):
        env.rewards[0, 0] = 1.0
    with pytest.raises(ValueError):
        cg.ActionMask(env.selected_action_masks[3, ...]).play = np.zeros(22, bool)   # record views too
    assert smp.get_actions().flags.writeable                 # an input of env.step


def test_edited_inputs_are_honoured(cg):
    """Masks edited in a copy and actions edited in the sampler's view reach the engine exactly as
    the oracle takes the same bytes."""
    n, seed = 128, 77
    env, smp, orc, osm = make(cg, n, seed)
    acts = smp.get_actions()
    rng = np.random.default_rng(1)
    for t in range(60):
        masks = env.selected_action_masks.copy()             # a caller's own masks, edited
        omasks = orc.selected_action_masks.copy()
        drop = rng.random(n) < 0.5
        masks["play"][drop, 0] = False                       # forbid passing for half the envs (where
        omasks["play"][drop, 0] = False                      # a card is playable the sample still succeeds)
        keep = masks["play"].any(axis=1)
        masks["play"][~keep, 0] = True
        omasks["play"][~keep, 0] = True
        smp.sample(masks)
        osm.sample(omasks)
        assert po.named_equal(acts, osm.actions) is None, f"sample of edited masks differs at step {t}"
        if t % 3 == 0:                                       # an edited action: pass instead
            acts["play"][::7] = 0
            osm.actions["play"][::7] = 0
        env.step(acts)
        orc.step(osm.actions)
        for nm in ("observations", "selected_action_masks", "infos"):
            bad = po.named_equal(getattr(env, nm), getattr(orc, nm))
            assert bad is None, f"step {t}: {nm}.{bad} differs from the oracle"
        assert np.array_equal(env.agent_selection, orc.agent_selection)


def test_sampler_on_env_view_orders_after_async_step(cg):
    """runner.sample(); runner.step() (asynchronous, publishes itself); then sampler.sample on the
    env's own mask view without a sync: the sampler reads the masks after that step."""
    n, seed = 256, 31
    env, smp, orc, osm = make(cg, n, seed)
    smp2 = cg.vec.get_vec_sampler(n)(1000)
    osm2 = po.OracleSampler(n, 1000)
    runner = cg.vec.get_runner(n)(env, smp, None)
    masks = env.selected_action_masks
    for t in range(40):
        runner.sample()
        runner.step()                                        # in flight
        smp2.sample(masks)                                   # the env's own view: HBM, ordered
        osm.sample(orc.selected_action_masks)
        orc.step(osm.actions)
        osm2.sample(orc.selected_action_masks)
        runner.sync()
        assert po.named_equal(smp2.get_actions(), osm2.actions) is None, f"step {t}: sampled before the step"
        bad = po.named_equal(env.selected_action_masks, orc.selected_action_masks)
        assert bad is None, f"step {t}: {bad}"


def test_speculative_sample_exact(cg):
    """The reference host loop `sampler.sample(env.selected_action_masks); env.step(actions)`
    (benchmarks.py:47-51) takes the sample the step computed speculatively (cog_abi.cpp
    SamplerSpec): actions, sampler state and views stay bit-exact with the oracle through hits and
    through everything that must void the speculation -- another sampler stepping the env, a
    sample of other masks, a reset, an episode end, a runner step."""
    n, seed = 256, 4711
    env, smp, orc, osm = make(cg, n, seed, max_steps=25)
    other = cg.vec.get_vec_sampler(n)(999)
    oother = po.OracleSampler(n, 999)
    masks, acts = env.selected_action_masks, smp.get_actions()

    def check(t, what):
        for nm in ("observations", "selected_action_masks", "infos"):
            bad = po.named_equal(getattr(env, nm), getattr(orc, nm))
            assert bad is None, f"{what} step {t}: {nm}.{bad}"
        assert np.array_equal(env.dones, orc.dones) and np.array_equal(env.agent_selection, orc.agent_selection)

    ended, ended_prev, hits = 0, False, 0
    for t in range(400):
        if t == 150:                                         # another sampler steps the env once
            other.sample(masks)
            oother.sample(orc.selected_action_masks)
            env.step(other.get_actions())
            orc.step(oother.actions)
        if t == 300:                                         # a reset voids the speculation
            env.reset(seed + 1, 4, 3, cg.HARD, 25, False)
            orc.reset(seed + 1, 4, 3, 2, 25)
        # the speculation is taken exactly when the step before was a self-publishing host step
        # (not the first step after a reset: t = 0, 300), nothing touched the env since (t = 150,
        # 300), no episode ended in it, and the sample reads the env's own mask view
        expect = t not in (0, 1, 150, 300, 301) and t % 97 != 5 and not ended_prev
        before = smp.spec_stats()
        if t % 97 == 5:                                      # a sample of a copy of the masks
            smp.sample(masks.copy())
        else:
            smp.sample(masks)
        after = smp.spec_stats()
        assert after[0] == before[0] + 1
        assert after[1] - before[1] == int(expect), f"step {t}: speculative sample taken {after[1] - before[1]}, expected {int(expect)}"
        hits += after[1] - before[1]
        osm.sample(orc.selected_action_masks)
        assert po.named_equal(acts, osm.actions) is None, f"sample at step {t}"
        env.step(acts)
        orc.step(osm.actions)
        check(t, "host loop")
        ended_prev = bool(orc.dones.any())
        ended += int(orc.dones.sum())
    assert ended > 0, "no episode ended: the test lost a case"
    assert hits >= 50, f"only {hits} speculative samples taken"


def test_device_record_writes_taken_after_invalidate(cg):
    """Writes into the device records (DLPack views) are taken by the next step after
    env.invalidate_device(), as the reference's views alias its live state
    (include/pybind/common.h:97-101): the selected ActionMask is the deck's live mask
    (player.cpp:16-27, environment.cpp:31-37), a player's stored mask is what its next turn loads
    (environment.cpp:62-63), the decks are the Deck's piles, and Info steps_taken counts on from
    the record (environment.cpp:97).  The oracle is fed the same bytes; then 40 more steps through
    the runner's device loop (the trio) must equal it everywhere."""
    import torch
    n, seed = 256, 9090
    env, smp, orc, osm = make(cg, n, seed)
    run = cg.vec.get_runner(n)(env, smp, None, device_views=True)
    run.set_chunk(20)
    run.rollout(40)
    run.sync()
    po.run_threaded(orc, osm, 40, po.host_threads())
    t = cg.device_tensors(env)
    sel, obs, info = t["selected_action_masks"], t["observations"], t["infos"]
    ag = orc.agent_selection.copy()
    edits = []                                               # (tensor name, env, byte offset, value)
    for i in range(32):                                      # the selected mask: pass only
        edits += [("sel", i, 0, 1)] + [("sel", i, b, 0) for b in range(1, 22)]
    p40 = (int(ag[40]) + 1) % 4                              # a deck: one more Explorer in the discard
    off40 = 16192 + 256 * p40 + 84
    edits.append(("obs", 40, off40, int(orc.observations.view(np.uint8).reshape(n, -1)[40, off40]) + 1))
    p50 = (int(ag[50]) + 1) % 4                              # the next player's stored mask: pass only
    for b in range(22):
        edits.append(("obs", 50, 16192 + 256 * p50 + 128 + b, 1 if b == 0 else 0))
    edits.append(("info", 7, 4 + 32 * int(ag[7]), 200))     # Info steps_taken of the acting player
    host = {"sel": orc.selected_action_masks.view(np.uint8).reshape(n, -1),
            "obs": orc.observations.view(np.uint8).reshape(n, -1),
            "info": orc.infos.view(np.uint8).reshape(n, -1)}
    dev = {"sel": sel, "obs": obs, "info": info}
    for nm, i, off, v in edits:
        dev[nm][i, off] = v                                  # (on torch's current stream)
        host[nm][i, off] = v
    env.invalidate_device()                                  # (ordered after those writes)
    run.rollout(40)
    run.sync()
    env.sync_host()
    po.run_threaded(orc, osm, 40, po.host_threads())
    for nm in ("observations", "selected_action_masks", "infos"):
        bad = po.named_equal(getattr(env, nm), getattr(orc, nm))
        assert bad is None, f"{nm}.{bad} differs from the oracle fed the same edits"
    for nm in ("rewards", "dones", "agent_selection"):
        assert np.array_equal(getattr(env, nm), getattr(orc, nm)), nm
    acts = torch.from_dlpack(smp.dlpack()).cpu().numpy().view(po.ACTION).reshape(n)
    assert po.named_equal(acts, osm.actions) is None
    # the edits mattered: pass-only envs passed, env 7 counted on from 200
    assert int(orc.infos["agent_infos"]["steps_taken"][7].max()) >= 200
