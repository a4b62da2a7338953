"""GPU: the BASELINE configurations at their own sizes (BASELINE.json configs),
against the C oracle on the same seeds.  The engine's wave-uniform fast paths (the play/pass
short path, the narrow/wide deck ballot, the sampler's head ballot) depend on which envs share
a wave, so the configs run at the sizes they are quoted on.  Bit-exact over named fields.

  C2          n=256, 4p, EASY: 10,000 selected-mask steps through the runner's device loop, all
              256 envs checked at checkpoints; and 1,000 steps of the reference's host loop
              (sampler.sample(masks); env.step(actions)) with every env checked every step
  C4 shard    n=8,192, 4p, HARD (the last of the 8 shards of 65,536: start piece B region), host
              views refreshed every step by runner.sample(); runner.step_sync(), all envs checked
  full dyn.   stored-mask driver (moves, shop, specials) with auto-resets and device map
              generation inside the rollout: all 8,192 envs of a C3-size batch (MEDIUM), and 256
              envs of a C5-size batch (65,536, HARD) against 1-env-per-seed oracle runs
"""
import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu
FIELDS = ("observations", "selected_action_masks", "infos")


def assert_equal(env, orc, lo=0, hi=None, what=""):
    hi = env.agent_selection.shape[0] if hi is None else hi
    for nm in FIELDS:
        bad = po.named_equal(getattr(env, nm)[lo:hi], getattr(orc, nm))
        assert bad is None, f"{what}: {nm}.{bad} differs from the oracle"
    for nm in ("rewards", "dones", "agent_selection"):
        assert np.array_equal(getattr(env, nm)[lo:hi], getattr(orc, nm)), f"{what}: {nm} differs"


def test_C2_n256_easy_rollout_10000_steps(cg):
    n, seed, steps, every = 256, 12345, 10000, 1000
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, 4, 3, cg.EASY, 100000, False)
    runner = cg.vec.get_runner(n)(env, smp, None, device_views=True)
    runner.set_chunk(250)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
    orc.reset(seed, 4, 3, 0, 100000)
    for t in range(0, steps, every):
        runner.rollout(every)
        runner.sync()
        env.sync_host()
        for _ in range(every):
            osm.sample(orc.selected_action_masks)
            orc.step(osm.actions)
        assert_equal(env, orc, what=f"C2 step {t + every}")
    assert np.array_equal(env.hazards()[1], orc.flags())


def test_C2_n256_easy_host_loop_every_step(cg):
    n, seed = 256, 777
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, 4, 3, cg.EASY, 100000, False)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
    orc.reset(seed, 4, 3, 0, 100000)
    masks, acts = env.selected_action_masks, smp.get_actions()
    for t in range(1000):
        smp.sample(masks)
        env.step(acts)
        osm.sample(orc.selected_action_masks)
        orc.step(osm.actions)
        assert po.named_equal(acts, osm.actions) is None, f"C2 host loop: actions differ at step {t}"
        assert_equal(env, orc, what=f"C2 host loop step {t}")


def test_C4_shard_n8192_hard_host_views_every_step(cg):
    from city_of_gold.shard import shard, shard_seed
    lo, hi = shard(65536, 7, 8)                            # the 8th GPU's shard of C4
    n, base = hi - lo, shard_seed(12345, lo)
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(12345, first_index=lo)
    env.reset(base, 4, 3, cg.HARD, 100000, False)
    runner = cg.vec.get_runner(n)(env, smp, 8)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, 12345, lo)
    orc.reset(base, 4, 3, 2, 100000)
    acts = runner.get_actions()
    sub = slice(0, n, 37)                                  # a strided subset checked every step
    for t in range(1, 201):
        runner.sample()
        runner.step_sync()
        osm.sample(orc.selected_action_masks)
        orc.step(osm.actions)
        assert po.named_equal(acts[sub], osm.actions[sub]) is None, f"C4 shard actions step {t}"
        for nm in ("selected_action_masks", "infos"):
            assert po.named_equal(getattr(env, nm)[sub], getattr(orc, nm)[sub]) is None, f"C4 shard {nm} step {t}"
        for f in ("phase", "current_resources", "shop"):
            assert np.array_equal(env.observations["shared"][f][sub], orc.observations["shared"][f][sub]), (f, t)
        if t % 50 == 0:
            assert_equal(env, orc, what=f"C4 shard step {t}")
    starts = orc.observations["shared"]["map"][:, :, :, 6].reshape(n, -1).sum(1)
    assert starts.min() > 0                                # every env has its end hexes


def test_full_dynamics_resets_C3_size_all_envs(cg):
    n, seed, steps = 8192, 4242, 240
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, 4, 3, cg.MEDIUM, 30, False)
    runner = cg.vec.get_runner(n)(env, smp, None, device_views=True, stored_masks=True)
    runner.set_chunk(60)
    runner.rollout(steps)
    runner.sync()
    env.sync_host()
    orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
    orc.reset(seed, 4, 3, 1, 30)
    resets = 0
    for _ in range(steps):
        osm.sample(po.stored_masks(orc))
        orc.step(osm.actions)
        resets += int(orc.dones.sum())
    assert resets > n // 2                                 # auto-resets happened inside launches
    assert_equal(env, orc, what="C3-size full dynamics")
    assert np.array_equal(env.hazards()[1], orc.flags())


@pytest.mark.parametrize("block", [(0, 128), (65536 - 128, 65536)], ids=["first128", "last128"])
def test_full_dynamics_resets_C5_size_subsets(cg, block):
    n, seed, steps = 65536, 90001, 200
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, 4, 3, cg.HARD, 30, False)
    runner = cg.vec.get_runner(n)(env, smp, None, device_views=True, stored_masks=True)
    runner.set_chunk(100)
    runner.rollout(steps)
    runner.sync()
    env.sync_host()
    lo, hi = block
    orc, osm = po.OracleVec(hi - lo), po.OracleSampler(hi - lo, seed + lo)
    orc.reset(seed + lo, 4, 3, 2, 30)                      # env i == a batch seeded seed + i
    resets = 0
    for _ in range(steps):
        osm.sample(po.stored_masks(orc))
        orc.step(osm.actions)
        resets += int(orc.dones.sum())
    assert resets > (hi - lo) // 2
    assert_equal(env, orc, lo, hi, what=f"C5-size full dynamics envs [{lo}, {hi})")


def test_full_dynamics_beyond_4gib_of_observations(cg):
    """Maximum sizes: 262,144 envs hold 4.5 GB of ObsData, so the records of the envs past
    249,475 lie beyond 2^32 bytes of the observation buffer (and of the map-generation grids):
    any 32-bit truncation of a record offset would show there.  Full dynamics (stored masks,
    auto-resets with device map generation) through the device loop; the last 128 envs are
    read through the DLPack device views and checked against 1-env-per-seed oracle runs."""
    n, seed, steps = 262144, 31337, 300
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, 4, 3, cg.HARD, 30, False)
    runner = cg.vec.get_runner(n)(env, smp, None, device_views=True, stored_masks=True)
    runner.set_chunk(60)
    runner.rollout(steps)
    runner.sync()
    lo, hi = n - 128, n
    assert lo * 17216 > 2 ** 32
    t = cg.device_tensors(env)
    got = {nm: t[nm][lo:hi].cpu().numpy() for nm in ("observations", "selected_action_masks", "infos",
                                                     "rewards", "dones", "agent_selection")}
    orc, osm = po.OracleVec(hi - lo), po.OracleSampler(hi - lo, seed + lo)
    orc.reset(seed + lo, 4, 3, 2, 30)                      # env i == a batch seeded seed + i
    resets = 0
    for _ in range(steps):
        osm.sample(po.stored_masks(orc))
        orc.step(osm.actions)
        resets += int(orc.dones.sum())
    assert resets > (hi - lo) // 2
    for nm, dt in (("observations", po.OBS), ("selected_action_masks", po.MASK), ("infos", po.INFO)):
        bad = po.named_equal(np.ascontiguousarray(got[nm]).view(dt).reshape(hi - lo), getattr(orc, nm))
        assert bad is None, f"envs past 4 GiB: {nm}.{bad} differs from the oracle"
    assert np.array_equal(got["rewards"], orc.rewards)
    assert np.array_equal(got["dones"].view(np.bool_), orc.dones)
    assert np.array_equal(got["agent_selection"], orc.agent_selection)


@pytest.mark.parametrize("n", [24576, 4096], ids=["n24576", "n4096"])
@pytest.mark.parametrize("stored,players", [(True, 4), (False, 4), (False, 2), (False, 3)],
                         ids=["stored_4p", "selected_4p", "selected_2p", "selected_3p"])
def test_episode_ends_in_the_two_wave_rollouts(cg, n, stored, players):
    """The multi-wave rollouts by rollout_kind: 16,385-32,768 envs run the two-wave pipe, smaller
    batches the duo, and with the selected masks and >= 3 players both sizes run the trio (its
    deferred turn end).  Episode ends inside their launches go to the fix-up pass (in the pipe
    kernel, after the storing wave's last stores; k_env_fixup after the duo and the trio), which
    completes them (finish, auto-reset with map generation) and runs the env's remaining steps.
    Episodes of 30 turns, so most envs end inside the launches; the first and the last 128 envs
    against 1-env-seeded oracle batches."""
    want = "trio" if not stored and players >= 3 else ("pipe" if n > 16384 else "duo")
    assert cg._city_of_gold.rollout_kind(n, players, stored) == want
    seed, steps = (777 if stored else 778) + n + 10 * players, 150
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, players, 3, cg.MEDIUM, 30, False)
    runner = cg.vec.get_runner(n)(env, smp, None, device_views=True, stored_masks=stored)
    runner.set_chunk(50)
    runner.rollout(steps)
    runner.sync()
    env.sync_host()
    for lo, hi in ((0, 128), (n - 128, n)):
        orc, osm = po.OracleVec(hi - lo), po.OracleSampler(hi - lo, seed + lo)
        orc.reset(seed + lo, players, 3, 1, 30)
        resets = 0
        for _ in range(steps):
            osm.sample(po.stored_masks(orc) if stored else orc.selected_action_masks)
            orc.step(osm.actions)
            resets += int(orc.dones.sum())
        assert resets > 0, "no episode ended inside the launches"
        assert_equal(env, orc, lo, hi, what=f"{n}-env {want} rollout envs [{lo}, {hi}) ({'stored' if stored else 'selected'}, {players}p)")
