"""GPU parity: the HIP engine (through the pybind11 module over the C ABI) against the C oracle
on identical seeds.  Bit-exact over every named field.  Oracle = checker only."""
import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu


def assert_same(env, orc, tag=""):
    for nm in ("observations", "selected_action_masks", "rewards", "dones", "agent_selection", "infos"):
        a, b = getattr(env, nm), getattr(orc, nm)
        if a.dtype.names:
            d = po.named_equal(a, b)
            if d is not None:
                bad = np.nonzero([po.named_equal(a[i:i + 1], b[i:i + 1]) is not None for i in range(len(a))])[0]
                raise AssertionError(f"{tag}: {nm}.{d} differs (envs {bad[:10]})")
        else:
            assert np.array_equal(a, b), f"{tag}: {nm} differs at {np.nonzero(a != b)[0][:10]}"


def test_sampler_random_masks(cg):
    n = 4096
    rng = np.random.default_rng(7)
    masks = np.zeros(n, dtype=po.MASK)
    raw = masks.view(np.uint8).reshape(n, 128)
    raw[:, :92] = rng.random((n, 92)) < 0.3
    raw[:7, :] = 0                                                  # empty heads -> 0, no draw
    s = cg.vec.get_vec_sampler(n)(123)
    o = po.OracleSampler(n, 123)
    for _ in range(3):
        s.sample(masks)
        o.sample(masks)
        assert po.named_equal(s.get_actions(), o.actions) is None


@pytest.mark.parametrize("diff", [0, 1, 2])
def test_reset_parity(cg, diff):
    n = 512
    env = cg.vec.get_vec_env(n)()
    orc = po.OracleVec(n)
    for seed in (0, 4096 * diff + 1, 63744, 70000):
        env.reset(seed, 4, 3, cg.Difficulty(diff), 100000, False)
        orc.reset(seed, 4, 3, diff, 100000)
        assert_same(env, orc, f"reset seed={seed} diff={diff}")
        haz, per = env.hazards()
        assert np.array_equal(per, orc.flags()), "hazard flags differ"


@pytest.mark.parametrize("mode", ["sel", "sto"])
def test_rollout_parity(cg, mode):
    n, steps = 256, 300
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(99)
    orc = po.OracleVec(n)
    osm = po.OracleSampler(n, 99)
    env.reset(12345, 4, 3, cg.HARD, 30 if mode == "sto" else 100000, False)
    orc.reset(12345, 4, 3, 2, 30 if mode == "sto" else 100000)
    assert_same(env, orc, "reset")
    for t in range(steps):
        m_env = env.selected_action_masks if mode == "sel" else po.stored_masks(env)
        m_orc = orc.selected_action_masks if mode == "sel" else po.stored_masks(orc)
        smp.sample(m_env)
        osm.sample(m_orc)
        assert po.named_equal(smp.get_actions(), osm.actions) is None, f"actions differ at {t}"
        env.step(smp.get_actions())
        orc.step(osm.actions)
        assert_same(env, orc, f"{mode} step {t}")


def test_sampler_draws_at_the_rejection_boundary(cg):
    """Sampler states whose j-th draw lands within 31 of the top of the range, where a head's
    draw may be rejected: the engine's sequential fallback path against the oracle."""
    P, RANGE = 2 ** 31 - 1, 2147483645
    inv = pow(16807, -1, P)
    rng = np.random.default_rng(11)
    raw = np.zeros((1, 128), dtype=np.uint8)
    raw[0, :92] = rng.random(92) < 0.5
    raw[0, [0, 22, 44, 66, 73]] = 1                       # every head has candidates
    masks = raw.view(po.MASK).reshape(1)
    for j in (0, 1, 4):                                  # which draw hits the boundary
        for r in range(RANGE - 34, RANGE + 1):
            x = (r + 1) * inv % P                        # state before the draw giving r
            for _ in range(j):
                x = x * inv % P                          # ... j draws earlier
            s, o = cg.vec.get_vec_sampler(1)(x), po.OracleSampler(1, x)
            for _ in range(2):
                s.sample(masks)
                o.sample(masks)
                assert po.named_equal(s.get_actions(), o.actions) is None, (j, r)


@pytest.mark.parametrize("seed", [5, 77])
def test_arbitrary_in_range_actions_against_oracle(cg, seed):
    """Host actions drawn at random within each head's range, masks ignored: cards played that
    are not in hand (u8 wrap-around), any card type including >= 8 (the deck's wide flag and the
    narrow/wide pile scans), moves into any neighbour, purchases whatever the coins.  The
    reference defines these byte by byte (only indices past a head are out of bounds), so the
    engine must match the oracle on every named field and on the hazard flags."""
    n, steps = 256, 400
    rng = np.random.default_rng(seed)
    env = cg.vec.get_vec_env(n)()
    orc = po.OracleVec(n)
    env.reset(seed, 4, 3, cg.HARD, 60, False)
    orc.reset(seed, 4, 3, 2, 60)
    top = (21, 21, 21, 6, 18)
    for t in range(steps):
        a = np.zeros(n, dtype=po.ACTION)
        head = rng.integers(0, 6, size=n)                # one head per env (5: pass), sometimes two
        for k, nm in enumerate(po.ACTION.names):
            v = rng.integers(1, top[k] + 1, size=n).astype(np.uint8)
            pick = (head == k) | (rng.random(n) < 0.05)
            a[nm] = np.where(pick, v, 0)
        env.step(a)
        orc.step(a)
        assert_same(env, orc, f"seed {seed} step {t}")
    haz, per = env.hazards()
    assert np.array_equal(per, orc.flags()), "hazard flags differ"
