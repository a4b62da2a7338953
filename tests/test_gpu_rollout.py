"""GPU: the persistent rollout kernel (runner.set_chunk(K > 1): K x (sample; step) per launch, state
kept on-chip between steps, every step's outputs stored) against the oracle and against one
launch per step.  Bit-exact over named fields."""
import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu


def run(cg, n, seed, n_players, diff, max_steps, steps, chunk, stored):
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, n_players, 3, cg.Difficulty(diff), max_steps, False)
    runner = cg.vec.get_runner(n)(env, smp, None, stored_masks=stored, device_views=True)
    runner.set_chunk(chunk)
    runner.rollout(steps)
    runner.sync()
    env.sync_host()
    return env, smp, runner


@pytest.mark.parametrize("chunk", [5, 64])
def test_rollout_stored_resets_against_oracle(cg, chunk):
    """Full dynamics (moves, shop, specials) with many auto-resets inside one launch."""
    n, steps = 1024, 300
    env, smp, _ = run(cg, n, 31337, 4, 2, 25, steps, chunk, True)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, 31337)
    orc.reset(31337, 4, 3, 2, 25)
    for _ in range(steps):
        osm.sample(po.stored_masks(orc))
        orc.step(osm.actions)
    for nm in ("observations", "selected_action_masks", "infos"):
        assert po.named_equal(getattr(env, nm), getattr(orc, nm)) is None, nm
    assert np.array_equal(env.rewards, orc.rewards)
    assert np.array_equal(env.dones, orc.dones)
    assert np.array_equal(env.agent_selection, orc.agent_selection)
    haz, per = env.hazards()
    assert np.array_equal(per, orc.flags())


@pytest.mark.parametrize("n_players", [2, 3])
def test_rollout_fewer_players_against_oracle(cg, n_players):
    n, steps = 512, 200
    env, smp, _ = run(cg, n, 4242, n_players, 1, 100000, steps, 50, False)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, 4242)
    orc.reset(4242, n_players, 3, 1, 100000)
    for _ in range(steps):
        osm.sample(orc.selected_action_masks)
        orc.step(osm.actions)
    for nm in ("observations", "selected_action_masks", "infos"):
        assert po.named_equal(getattr(env, nm), getattr(orc, nm)) is None, nm
    assert np.array_equal(env.agent_selection, orc.agent_selection)


def test_rollout_equals_per_step_launches_at_c5_size(cg):
    """C5 shape (65,536 envs, 4p, HARD): chunked rollout == one launch per step, byte for byte
    over every device buffer a step writes."""
    n, steps = 65536, 120
    a, sa, _ = run(cg, n, 12345, 4, 2, 100000, steps, 40, False)
    b, sb, _ = run(cg, n, 12345, 4, 2, 100000, steps, 1, False)
    for nm in ("observations", "selected_action_masks", "infos", "rewards", "dones", "agent_selection"):
        assert np.array_equal(getattr(a, nm).view(np.uint8), getattr(b, nm).view(np.uint8)), nm


def test_rollout_interleaves_with_host_steps(cg):
    """A chunked rollout, then host-API sample/step, then a rollout again: one consistent state."""
    n = 256
    env, smp, runner = run(cg, n, 99, 4, 2, 40, 37, 16, True)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, 99)
    orc.reset(99, 4, 3, 2, 40)
    for _ in range(37):
        osm.sample(po.stored_masks(orc))
        orc.step(osm.actions)
    for _ in range(5):                                     # host API in between
        smp.sample(po.stored_masks(env))
        osm.sample(po.stored_masks(orc))
        env.step(smp.get_actions())
        orc.step(osm.actions)
    runner.rollout(29)
    runner.sync()
    env.sync_host()
    for _ in range(29):
        osm.sample(po.stored_masks(orc))
        orc.step(osm.actions)
    for nm in ("observations", "selected_action_masks", "infos"):
        assert po.named_equal(getattr(env, nm), getattr(orc, nm)) is None, nm


@pytest.mark.parametrize("n,chunk", [(1, 7), (100, 33), (130, 1000)])
def test_rollout_ragged_batches_against_oracle(cg, n, chunk):
    """Batches that leave the last wave partly empty (and a chunk larger than the run), with
    episodes short enough that lanes park and resume inside one launch."""
    steps = 150
    env, smp, _ = run(cg, n, 2024 + n, 4, 2, 30, steps, chunk, True)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, 2024 + n)
    orc.reset(2024 + n, 4, 3, 2, 30)
    for _ in range(steps):
        osm.sample(po.stored_masks(orc))
        orc.step(osm.actions)
    for nm in ("observations", "selected_action_masks", "infos"):
        assert po.named_equal(getattr(env, nm), getattr(orc, nm)) is None, nm
    assert np.array_equal(env.rewards, orc.rewards)
    assert np.array_equal(env.dones, orc.dones)
    assert np.array_equal(env.agent_selection, orc.agent_selection)


@pytest.mark.parametrize("n,chunk,players", [(1, 7, 4), (100, 33, 3), (130, 1000, 4), (200, 20, 3)])
def test_trio_ragged_batches_with_episode_ends(cg, n, chunk, players):
    """The trio rollout (selected masks, >= 3 players) on batches that leave its last workgroup's
    waves partly empty, with max_steps 30 turns so that lanes finish inside launches (parked for
    k_env_fixup: finish, auto-reset, the rest of the launch) -- every named field against the
    oracle."""
    assert cg._city_of_gold.rollout_kind(n, players, False) == "trio"
    steps = 180
    env, smp, _ = run(cg, n, 7070 + n, players, 2, 30, steps, chunk, False)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, 7070 + n)
    orc.reset(7070 + n, players, 3, 2, 30)
    for _ in range(steps):
        osm.sample(orc.selected_action_masks)
        orc.step(osm.actions)
    for nm in ("observations", "selected_action_masks", "infos"):
        assert po.named_equal(getattr(env, nm), getattr(orc, nm)) is None, nm
    assert np.array_equal(env.rewards, orc.rewards)
    assert np.array_equal(env.dones, orc.dones)
    assert np.array_equal(env.agent_selection, orc.agent_selection)


def test_rollout_zero_steps_and_empty_batch(cg):
    env, smp, runner = run(cg, 64, 5, 4, 2, 100000, 0, 10, False)   # rollout(0): nothing runs
    before = env.observations.copy()
    runner.rollout(0)
    runner.sync()
    env.sync_host()
    assert po.named_equal(env.observations, before) is None
    e0 = cg.vec.get_vec_env(0)()
    s0 = cg.vec.get_vec_sampler(0)(1)
    r0 = cg.vec.get_runner(0)(e0, s0, None, device_views=True)
    r0.set_chunk(8)
    r0.rollout(20)
    r0.sync()


REDO_SCRIPT = r'''
import sys
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import numpy as np
import city_of_gold as cg
import pyoracle as po
n, seed, steps = int(sys.argv[3]), 4242, 60
env = cg.vec.get_vec_env(n)(device=0)
smp = cg.vec.get_vec_sampler(n)(seed, device=0)
env.reset(seed, 4, 3, cg.HARD, int(sys.argv[4]), False)
run = cg.vec.get_runner(n)(env, smp, None, device_views=True)
run.set_chunk(20)
run.rollout(steps)
run.sync()
env.sync_host()
orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
orc.reset_threaded(seed, 4, 3, 2, int(sys.argv[4]))
po.run_threaded(orc, osm, steps, po.host_threads())
for nm in ("observations", "selected_action_masks", "infos"):
    bad = po.named_equal(getattr(env, nm), getattr(orc, nm))
    assert bad is None, f"{nm}.{bad} differs from the oracle"
for nm in ("rewards", "dones", "agent_selection"):
    assert np.array_equal(getattr(env, nm), getattr(orc, nm)), nm
print("OK", int(orc.infos["total_length"].astype(bool).sum()))
'''


PARK_NOFIX_SCRIPT = r'''
import sys
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import numpy as np
import city_of_gold as cg
import pyoracle as po
n, j, seed, steps = int(sys.argv[3]), int(sys.argv[4]), 4242, 20
FIELDS = ("observations", "selected_action_masks", "infos", "rewards", "dones", "agent_selection")


def check(env, orc, keep, what):
    for nm in FIELDS:
        a, b = getattr(env, nm)[keep], getattr(orc, nm)[keep]
        bad = po.named_equal(a, b) if a.dtype.names else (None if np.array_equal(a, b) else nm)
        assert bad is None, f"{what}: {nm}.{bad} differs from the oracle"


env = cg.vec.get_vec_env(n)(device=0)
smp = cg.vec.get_vec_sampler(n)(seed, device=0)
env.reset(seed, 4, 3, cg.HARD, 100000, False)
run = cg.vec.get_runner(n)(env, smp, None, device_views=True)
run.set_chunk(steps)
run.rollout(steps)                        # lean_clock 0 + 20 < max_steps: launched without k_env_fixup
try:
    run.sync()
    err = None
except RuntimeError as e:
    err = str(e)
assert err is not None and "without its fix-up" in err, f"no F_PARK_NOFIX error: {err!r}"
env.sync_host()
orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
orc.reset_threaded(seed, 4, 3, 2, 100000)
po.run_threaded(orc, osm, steps, po.host_threads())
others = np.ones(n, bool)
others[j] = False
check(env, orc, others, "the other envs after the launch")
one, one_s = po.OracleVec(1), po.OracleSampler(1, seed, j)   # env j: a 1-env batch seeded seed + j
one.reset(seed + j, 4, 3, 2, 100000)
for _ in range(7):                                           # parked before its step 7
    one_s.sample(one.selected_action_masks)
    one.step(one_s.actions)
for nm in FIELDS:
    a, b = getattr(env, nm)[j:j + 1], getattr(one, nm)
    assert (po.named_equal(a, b) if a.dtype.names else (None if np.array_equal(a, b) else nm)) is None, \
        f"the parked env {j}: {nm} is not its state before step 7"
del run, smp
# the handle recovers: a reset, then launches that never reach step 7 (5-step launches).  The
# oracles go on from their own states (a reset leaves Info alone, environment.cpp:42-77: its
# steps_taken counts on), env j's from its 7 steps
seed2 = 777
smp = cg.vec.get_vec_sampler(n)(seed2, device=0)
env.reset(seed2, 4, 3, cg.HARD, 100000, False)
run = cg.vec.get_runner(n)(env, smp, None, device_views=True)
run.set_chunk(5)
run.rollout(steps)
run.sync()
env.sync_host()
osm = po.OracleSampler(n, seed2)
orc.reset_threaded(seed2, 4, 3, 2, 100000)
po.run_threaded(orc, osm, steps, po.host_threads())
check(env, orc, others, "after the reset")
one_s = po.OracleSampler(1, seed2, j)
one.reset(seed2 + j, 4, 3, 2, 100000)
for _ in range(steps):
    one_s.sample(one.selected_action_masks)
    one.step(one_s.actions)
for nm in FIELDS:
    a, b = getattr(env, nm)[j:j + 1], getattr(one, nm)
    assert (po.named_equal(a, b) if a.dtype.names else (None if np.array_equal(a, b) else nm)) is None, \
        f"env {j} after the reset: {nm}"
print("OK", err)
'''


@pytest.mark.parametrize("n", [4096, 40960])
def test_trio_park_without_fixup_is_an_error(cg, tmp_path, n):
    """The no-fix-up guard.  A trio launch that the host cleared with lean_clock (no env can park,
    so k_env_fixup is not launched: cog_abi.cpp runner_launch_fused) must turn a park it meets
    all the same into an error (F_PARK_NOFIX), never leave it unprocessed in silence.  The test hook
    COG_DEBUG_PARK_NOFIX=7:j parks env j before step 7 of such a launch: runner.sync() raises
    RuntimeError naming the missing fix-up, every other env equals the oracle after the launch,
    env j holds its state before step 7 (a 1-env oracle seeded seed + j), and a reset of the same
    handle runs clean afterwards.  4,096 envs (one workgroup per CU: the LAT form) and 40,960 (640
    workgroups, two per CU)."""
    import os
    import subprocess
    import sys
    assert cg._city_of_gold.rollout_kind(n) == "trio"
    pkg = os.path.dirname(os.path.dirname(cg.__file__))
    oracle_dir = os.path.join(os.path.dirname(pkg), "oracle")
    script = tmp_path / "park_nofix.py"
    script.write_text(PARK_NOFIX_SCRIPT)
    j = n // 2 + 37
    r = subprocess.run([sys.executable, str(script), pkg, oracle_dir, str(n), str(j)], capture_output=True,
                       text=True, timeout=240, env=dict(os.environ, COG_DEBUG_PARK_NOFIX=f"7:{j}"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.strip().splitlines()[-1].startswith("OK")


@pytest.mark.parametrize("max_steps", [100000, 12])
def test_trio_deferred_turn_end_redo_path(cg, tmp_path, max_steps):
    """The trio rollout's deferred turn end (selected masks, >= 3 players: the drawing wave runs the
    turn end's discard + draws with the env rng) parks an env whose action would draw from the env
    rng inside a step (kParkRedo), and k_env_fixup runs that step and the rest with the full step.
    The canonical loop never takes such an action, so the test hook COG_DEBUG_REDO_STEP=7 parks
    every env at step 7 of each 20-step launch; 4,096 envs (the trio) against the oracle, with and
    without episode ends (max_steps 12: parks for finished episodes in the same launches)."""
    import os
    import subprocess
    import sys
    assert cg._city_of_gold.rollout_kind(4096) == "trio"
    pkg = os.path.dirname(os.path.dirname(cg.__file__))
    oracle_dir = os.path.join(os.path.dirname(pkg), "oracle")
    script = tmp_path / "redo.py"
    script.write_text(REDO_SCRIPT)
    r = subprocess.run([sys.executable, str(script), pkg, oracle_dir, "4096", str(max_steps)], capture_output=True,
                       text=True, timeout=240, env=dict(os.environ, COG_DEBUG_REDO_STEP="7"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.strip().splitlines()[-1].startswith("OK")


@pytest.mark.parametrize("n", [4096, 40960])
def test_trio_compact_decks_across_drivers(cg, n):
    """A trio launch starts from the compact deck image the previous trio launch (and its fix-up)
    left (DevState::cdeck / cwide), which holds only while trio launches alone wrote decks.  Here
    full-dynamics launches (moves and purchases: decks with types >= 8, which the compact form
    cannot hold, so those envs park at step 0 of every trio launch) alternate with selected-mask
    trio launches of 20 steps, and the result must equal the oracle running the same drivers.
    4,096 envs: the LAT trio and the duo; 40,960: two trio workgroups per CU and the one-wave
    kernel."""
    seed = 2468
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, 4, 3, cg.Difficulty(2), 100000, False)
    sel = cg.vec.get_runner(n)(env, smp, None, device_views=True)
    sto = cg.vec.get_runner(n)(env, smp, None, stored_masks=True, device_views=True)
    sel.set_chunk(20)
    sto.set_chunk(50)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
    orc.reset(seed, 4, 3, 2, 100000)
    for kind, k in (("sel", 40), ("sto", 150), ("sel", 60), ("sto", 50), ("sel", 40)):
        (sel if kind == "sel" else sto).rollout(k)
        for _ in range(k):
            osm.sample(orc.selected_action_masks if kind == "sel" else po.stored_masks(orc))
            orc.step(osm.actions)
    sel.sync()
    sto.sync()
    env.sync_host()
    for nm in ("observations", "selected_action_masks", "infos"):
        bad = po.named_equal(getattr(env, nm), getattr(orc, nm))
        assert bad is None, f"{nm}.{bad} differs from the oracle"
    for nm in ("rewards", "dones", "agent_selection"):
        assert np.array_equal(getattr(env, nm), getattr(orc, nm)), nm
    piles = np.ascontiguousarray(orc.observations["player_data"]["obs"]).view(np.uint8).reshape(n, 4, 5, 21)
    wide = int((piles[:, :, :, 8:] != 0).any(axis=(1, 2, 3)).sum())   # (draw, hand, active, played, discard)
    assert wide > 0, "no deck holds a type >= 8: the test lost its case"
