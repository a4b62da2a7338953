"""GPU: the reference's own Python tests, pytest/test_vec_env.py:161-171.  Each one is
run_test(10000, 16, 123456) (:74-113): reset(seed, 4 players, 3 pieces, EASY, 100000), then
10,000 x (sample(selected_action_masks); step(actions)).  The three tests differ only in the driver:
sequential (env.step + sampler.sample), the 4-thread async runner (runner.sample/step) and the
4-thread sync runner (runner.sample/step_sync).

The reference's tests only check that nothing crashes.  Here the three drivers must also end in
byte-identical states, equal to the oracle's run of the same loop.  EASY maps with more than one
travel piece take the past-the-end erase of map.cpp:727.  Its result follows the GCC >= 13
semantics both here and in the oracle, so that part of the parity is pinned by the
oracle alone."""
import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu

STEPS, N, SEED = 10000, 16, 123456
FIELDS = ("observations", "selected_action_masks", "rewards", "dones", "agent_selection", "infos")


def run_test(cg, threaded=False, threads=None, sync=False):
    """run_test of the reference (pytest/test_vec_env.py:74-113), returning the final state."""
    envs = cg.vec.get_vec_env(N)()
    samplers = cg.vec.get_vec_sampler(N)(SEED)
    runner = None
    if threaded:
        runner = cg.vec.get_runner(N)(envs, samplers, threads)
        step_fun = (lambda _: runner.step_sync()) if sync else (lambda _: runner.step())
        sample_fun = lambda _: runner.sample()
        envs = runner.get_envs()
    else:
        step_fun = envs.step
        sample_fun = samplers.sample
    assert not ((not threaded) and sync)
    envs.reset(SEED, 4, 3, cg.Difficulty.EASY, 100000, False)
    actions = samplers.get_actions()
    player_masks = envs.selected_action_masks
    for _ in range(STEPS):
        sample_fun(player_masks)
        step_fun(actions)
    if threaded:
        runner.sync()
    state = {nm: np.array(getattr(envs, nm), copy=True) for nm in FIELDS}
    state["flags"] = envs.hazards()[1].copy()
    return state


@pytest.fixture(scope="module")
def oracle_state():
    orc, osm = po.OracleVec(N), po.OracleSampler(N, SEED)
    orc.reset(SEED, 4, 3, 0, 100000)
    for _ in range(STEPS):
        osm.sample(orc.selected_action_masks)
        orc.step(osm.actions)
    state = {nm: np.array(getattr(orc, nm), copy=True) for nm in FIELDS}
    state["flags"] = orc.flags().copy()
    return state


def assert_state(got, want, tag):
    for nm in FIELDS:
        a, b = got[nm], want[nm]
        if a.dtype.names:
            assert po.named_equal(a, b) is None, f"{tag}: {nm}.{po.named_equal(a, b)}"
        else:
            assert np.array_equal(a, b), f"{tag}: {nm}"
    assert np.array_equal(got["flags"], want["flags"]), f"{tag}: hazard flags"


def test_sequential(cg, oracle_state):
    assert_state(run_test(cg), oracle_state, "sequential")


def test_async(cg, oracle_state):
    assert_state(run_test(cg, True, 4), oracle_state, "async")


def test_sync(cg, oracle_state):
    assert_state(run_test(cg, True, 4, True), oracle_state, "sync")
