"""GPU: `city_of_gold.cog_env`, the single-environment API (reference src/pybind/single_env.cpp,
include/environment.h), driven the way the reference's own unit tests drive it
(src/tests/test_environment.cpp:8-130).  The sampler there is `action_sampler` on the acting
player's stored mask; here it is the vec sampler of one env, seed 42 -- the driver that produced
the KAT values (499 steps to total_length 100; 37,627 steps to 921)."""
import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu


def bound_env(cg, *params):
    env = cg.cog_env(*params) if params else cg.cog_env()
    obs, info = np.zeros(1, dtype=cg.ObsData), np.zeros(1, dtype=cg.Info)
    rewards, mask = np.zeros(4, dtype=np.float32), np.zeros(1, dtype=cg.ActionMask)
    env.init(obs, info, rewards, mask)
    return env, obs, info, rewards, mask


def run_until_done(cg, env, obs, limit):
    smp = cg.vec.get_vec_sampler(1)(42)
    steps = 0
    while True:                                            # test_environment.cpp:95-100
        ag = env.agent_selection
        smp.sample(np.ascontiguousarray(obs[0]["player_data"][ag]["action_mask"]).reshape(1))
        env.step(smp.get_actions())
        steps += 1
        if env.get_done() or steps >= limit:
            return steps


def test_constructor(cg):
    env = cg.cog_env()                                     # :8-11
    assert env.get_n_players() == 4 and env.get_n_pieces() == 3 and env.get_max_steps() == 100000


def test_reset_reinitializes(cg):
    env, obs, *_ = bound_env(cg)                           # :14-65
    env.reset(123, 3, 8, cg.MEDIUM, 200, False)
    first = obs[0]["shared"]["map"].copy()
    assert first.any()
    env.reset(123, 3, 8, cg.MEDIUM, 200, False)
    assert np.array_equal(obs[0]["shared"]["map"], first)  # same seed: same map
    env.reset(124, 3, 8, cg.MEDIUM, 200, False)
    assert not np.array_equal(obs[0]["shared"]["map"], first)
    params = (env.get_seed(), env.get_n_players(), env.get_n_pieces(), env.get_difficulty(),
              env.get_max_steps(), env.get_render())
    env.reset()                                            # keeps the parameters
    assert (env.get_seed(), env.get_n_players(), env.get_n_pieces(), env.get_difficulty(),
            env.get_max_steps(), env.get_render()) == params


def test_too_many_easy_pieces(cg):
    env, *_ = bound_env(cg)                                # :68-80
    env.reset(124, 3, 3, cg.EASY, 200, False)
    with pytest.raises(RuntimeError):
        env.reset(123, 3, 4, cg.EASY, 200, False)


def test_ends_at_max_steps(cg):
    env, obs, info, *_ = bound_env(cg)                     # :83-103
    env.reset(54321, 4, 5, cg.MEDIUM, 100, False)
    steps = run_until_done(cg, env, obs, 10000)
    assert env.get_done() and info[0]["total_length"] == 100 and steps == 499


def test_natural_end_and_dead_steps(cg):
    env, obs, info, rewards, mask = bound_env(cg)          # :106-130
    env.reset(54321, 4, 1, cg.EASY, 100000, False)
    steps = run_until_done(cg, env, obs, 100000)
    assert env.get_done() and info[0]["total_length"] == 921 and steps == 37627
    returns = list(info[0]["agent_infos"]["returns"])
    assert returns == [-1.0, 3.0, -1.0, -1.0] and sum(returns) == 0.0
    assert np.array_equal(rewards, np.array(returns, dtype=np.float32))
    # cog_env::step on a finished episode is a dead step (environment.cpp:92-95): no auto-reset
    before = (obs.tobytes(), info.tobytes(), mask.tobytes())
    env.step((1, 0, 0, 0, 0))
    env.step(np.zeros(1, dtype=cg.ActionData))
    assert env.get_done()
    for a, b in zip((obs, info, mask), before):
        assert a.tobytes() == b
    env.reset(54321, 4, 1, cg.EASY, 100000, False)         # reset starts a new episode (and,
    assert not env.get_done()                              # as cog_env::reset, leaves Info as is)
    assert info[0]["total_length"] == 921
    # The second episode is not the first again: reset keeps the shop's n_in_market (Q12).
    # The oracle, reset the same way after the same episode, pins it step by step.
    orc, osm = po.OracleVec(1), po.OracleSampler(1, 42)
    orc.reset(54321, 4, 1, 0, 100000)
    for _ in range(37627):
        osm.sample(po.stored_masks(orc))
        orc.step(osm.actions)
    orc.reset(54321, 4, 1, 0, 100000)
    osm, smp = po.OracleSampler(1, 42), cg.vec.get_vec_sampler(1)(42)
    for t in range(3000):
        ag = env.agent_selection
        smp.sample(np.ascontiguousarray(obs[0]["player_data"][ag]["action_mask"]).reshape(1))
        osm.sample(po.stored_masks(orc))
        env.step(smp.get_actions())
        orc.step(osm.actions)
        assert po.named_equal(obs, orc.observations) is None, f"step {t}"
        assert po.named_equal(mask, orc.selected_action_masks) is None, f"step {t}"


def test_reference_unit_loop_with_record_classes(cg):
    """test_environment.cpp:83-102 verbatim in Python: the record classes (single_env.cpp:34-85),
    action_sampler() with its default seed 42 (common.cpp:25-27, sampler.h:9-12) on the acting
    player's stored mask, cog_env.init() binding the records."""
    sampler = cg.action_sampler()
    observation, mask, info = cg.ObsData(), cg.ActionMask(), cg.Info()
    rewards = np.zeros(4, dtype=np.float32)
    assert mask.play[0] and not mask.play[1:].any() and mask.move[0]     # ActionMask() defaults
    env = cg.cog_env()
    env.init(observation, info, rewards, mask)
    env.reset(54321, 4, 5, cg.MEDIUM, 100, False)
    steps = 0
    while True:
        current_agent = env.agent_selection
        act = sampler.sample(observation.player_data[current_agent].action_mask)
        assert isinstance(act, cg.ActionData)
        env.step(act)
        steps += 1
        if env.get_done():
            break
    assert env.get_info().total_length == 100 and steps == 499
    assert info["total_length"] == 100                     # the bound record was updated
    assert observation.shared.map.shape == (48, 48, 7) and observation.shared.phase in (0, 1, 2)
    assert len(observation.player_data) == 4
    deck = observation.player_data[0].obs
    assert int(deck.draw.sum() + deck.hand.sum() + deck.active.sum() + deck.discard.sum()) >= 8


def test_action_sampler_matches_vec_sampler(cg):
    """action_sampler(seed).sample(mask) == vec_sampler(1)(seed) on the same masks."""
    rng = np.random.default_rng(1)
    a, v = cg.action_sampler(99), cg.vec.get_vec_sampler(1)(99)
    for _ in range(50):
        m = cg.ActionMask()
        for head, k in (("play", 22), ("play_special", 22), ("remove", 22), ("move", 7), ("get_from_shop", 19)):
            bits = rng.random(k) < 0.3
            bits[0] = True
            setattr(m, head, bits)
        act = a.sample(m)
        v.sample(m.record.reshape(1))
        assert act == v.get_actions()[0]
        rec = cg.ActionData(play=act.play)
        assert rec.play == act.play and np.dtype(cg.ActionData).itemsize == 64
