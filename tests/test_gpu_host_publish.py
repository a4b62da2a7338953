"""GPU: host-visible steps that publish their own changes (k_env_step_pub) -- the reference's host
loop `sampler.sample(masks); env.step(actions)` (include/pybind/vectorized.h:60-68,118-125) with
the numpy views checked against the C oracle after every step, where the direct path meets what
it does not cover itself: episode ends and auto-resets (the ended envs' records published by
comparison, the regenerated maps through the dirty list), device-only work in between (runner
rollouts on device views, after which the next host step publishes by comparison again),
env.reset(), staged (non-pinned) actions, and handles of two shards.  Bit-exact over named fields.
"""
import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu
FIELDS = ("observations", "selected_action_masks", "infos")


def assert_equal(env, orc, what):
    for nm in FIELDS:
        bad = po.named_equal(getattr(env, nm), getattr(orc, nm))
        assert bad is None, f"{what}: {nm}.{bad} differs from the oracle"
    for nm in ("rewards", "dones", "agent_selection"):
        assert np.array_equal(getattr(env, nm), getattr(orc, nm)), f"{what}: {nm} differs"


def host_steps(env, smp, orc, osm, steps, what, staged=False):
    masks, acts = env.selected_action_masks, smp.get_actions()
    for t in range(steps):
        smp.sample(masks)
        env.step(acts.copy() if staged else acts)
        osm.sample(orc.selected_action_masks)
        orc.step(osm.actions)
        assert po.named_equal(acts, osm.actions) is None, f"{what}: actions differ at step {t}"
        assert_equal(env, orc, f"{what} step {t}")


def make(cg, n, seed, difficulty, max_steps, device=None):
    env = cg.vec.get_vec_env(n)(device=device) if device is not None else cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed, device=device) if device is not None else cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, 4, 3, difficulty, max_steps, False)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
    orc.reset(seed, 4, 3, {cg.EASY: 0, cg.MEDIUM: 1, cg.HARD: 2}[difficulty], max_steps)
    return env, smp, orc, osm


def test_host_loop_with_episode_ends_every_step(cg):
    # max_steps 25: every env ends and auto-resets every 25 of its turns' steps
    env, smp, orc, osm = make(cg, 256, 4242, cg.EASY, 25)
    host_steps(env, smp, orc, osm, 400, "C2 resets")
    assert int((orc.infos["total_length"] != 0).sum()) > 0, "no episode ended: the test lost its point"
    assert np.array_equal(env.hazards()[1], orc.flags())


def test_host_loop_interleaved_with_device_work(cg):
    n, seed = 256, 99
    env, smp, orc, osm = make(cg, n, seed, cg.MEDIUM, 40)
    runner_d = cg.vec.get_runner(n)(env, smp, None, device_views=True)    # sync() leaves the views
    runner_h = cg.vec.get_runner(n)(env, smp, None)                       # sync() publishes
    for r in (runner_d, runner_h):
        r.set_chunk(7)

    def device_steps(r, k):
        r.rollout(k)
        r.sync()
        if r is runner_d:
            env.sync_host()                           # (device views: the host views on request)
        for _ in range(k):
            osm.sample(orc.selected_action_masks)
            orc.step(osm.actions)
        assert_equal(env, orc, f"after rollout({k})")

    host_steps(env, smp, orc, osm, 30, "phase 1")
    device_steps(runner_d, 13)                        # device-only work, then a full refresh
    host_steps(env, smp, orc, osm, 30, "after a device-view rollout")
    device_steps(runner_h, 11)                        # device work published by comparison
    host_steps(env, smp, orc, osm, 30, "after a host-view rollout")
    device_steps(runner_h, 1)
    host_steps(env, smp, orc, osm, 3, "after one device step", staged=True)
    env.reset()                                       # reset_default: same parameters, rngs continue
    orc.reset_default()
    assert_equal(env, orc, "after reset()")
    host_steps(env, smp, orc, osm, 40, "after reset()")


def test_host_loop_two_shards(cg):
    # one handle, two shards (both on GPU 0 here), ragged 150 + 151, with resets
    env, smp, orc, osm = make(cg, 301, 5150, cg.HARD, 30, device=[0, 0])
    host_steps(env, smp, orc, osm, 120, "two shards")


SPIN_OFF_SCRIPT = r"""
import hashlib, sys
sys.path.insert(0, sys.argv[1])
import city_of_gold as cg
n, seed = 256, 31337
env = cg.vec.get_vec_env(n)()
smp = cg.vec.get_vec_sampler(n)(seed)
env.reset(seed, 4, 3, cg.EASY, 25, False)
masks, acts = env.selected_action_masks, smp.get_actions()
h = hashlib.sha256()
for _ in range(60):
    smp.sample(masks)
    env.step(acts)
    for a in (acts, env.observations, env.selected_action_masks, env.infos, env.rewards, env.dones,
              env.agent_selection):
        h.update(a.tobytes())
print(h.hexdigest())
"""


def test_completion_without_spin_same_bytes(cg, tmp_path):
    """COG_SPIN_US=0 (every call ends on hipStreamSynchronize, as in round 2) gives the bytes the
    default completion-word path gives, through the same host loop with episode ends."""
    import hashlib
    import os
    import subprocess
    import sys
    pkg = os.path.dirname(os.path.dirname(cg.__file__))
    n, seed = 256, 31337
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, 4, 3, cg.EASY, 25, False)
    masks, acts = env.selected_action_masks, smp.get_actions()
    h = hashlib.sha256()
    for _ in range(60):
        smp.sample(masks)
        env.step(acts)
        for a in (acts, env.observations, env.selected_action_masks, env.infos, env.rewards, env.dones,
                  env.agent_selection):
            h.update(a.tobytes())
    script = tmp_path / "spin_off.py"
    script.write_text(SPIN_OFF_SCRIPT)
    run = subprocess.run([sys.executable, str(script), pkg], capture_output=True, text=True, timeout=150,
                         env=dict(os.environ, COG_SPIN_US="0", COG_NO_TORCH="1"))
    assert run.returncode == 0, run.stderr[-2000:]
    assert run.stdout.strip().splitlines()[-1] == h.hexdigest()


def test_runner_host_steps_publish_themselves(cg):
    """runner.sample(); runner.step_sync() with host views (the C4 host loop) takes the direct
    publish, sampled actions included; a sample() queued after a direct step, two steps before one
    sync(), and env.step() between runner steps still leave every view as the reference's."""
    n, seed = 512, 2024
    env, smp, orc, osm = make(cg, n, seed, cg.MEDIUM, 30)
    runner = cg.vec.get_runner(n)(env, smp, None)
    acts = runner.get_actions()

    def ref_step():
        osm.sample(orc.selected_action_masks)
        orc.step(osm.actions)

    for t in range(60):                                    # the C4 loop, with episode ends
        runner.sample()
        runner.step_sync()
        ref_step()
        assert po.named_equal(acts, osm.actions) is None, f"runner loop: actions differ at step {t}"
        assert_equal(env, orc, f"runner loop step {t}")
    runner.sample()                                        # step, then a sample before the sync
    runner.step()
    runner.sample()
    runner.sync()
    ref_step()
    osm.sample(orc.selected_action_masks)
    assert po.named_equal(acts, osm.actions) is None, "the sample after a direct step is not in the view"
    assert_equal(env, orc, "step + sample + sync")
    runner.step()                                          # steps with those actions, then one more
    orc.step(osm.actions)
    runner.sample()
    runner.step()
    runner.sync()
    ref_step()
    assert_equal(env, orc, "two steps, one sync")
    host_steps(env, smp, orc, osm, 5, "env.step between runner steps")
    for t in range(5):
        runner.sample()
        runner.step_sync()
        ref_step()
        assert_equal(env, orc, f"runner after env.step, step {t}")
