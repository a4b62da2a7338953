"""GPU: the EXACT workloads bench.py times, every env against the C oracle.

For the N=1 headline batch (65,536 envs, 4 players, HARD, seeds 12345 + i) and for the last
rank's shard at N = 2, 4 and 8 (`shard(65536, N-1, N)`: 32,768 / 16,384 / 8,192 envs, seeds
12345 + global index: `make(..., first=lo)`), the engine is built by bench.py's own `make()`
and driven by `runner.rollout` in the two launch shapes the bench uses:
  - chunk 20: a 5-step launch (the driver's `--warmup 5`), then 20-step launches (`--steps 20`);
  - chunk 1000: 205 steps, then one 1,000-step launch (bench's default shape).
The kernels are the bench's (cog_engine.hip rollout_kind): the trio rollout at every one of these
sizes (k_env_rollout_trio + k_env_fixup: the deferred turn end); at 65,536 its 1,024 workgroups
run in two rounds.
After 1,205 steps ALL envs are compared with a threaded oracle run of the reference runner loop
(`sample(selected_action_masks); step(actions)`, benchmarks/benchmarks.py:47-51,
include/runner.h:33-62): every named field of ObsData / ActionMask / Info, rewards, dones,
agent_selection, the sampled actions and the per-env hazard flags.  Bit-exact.

Every env the reference itself can run (all but the erase-past maps, map.cpp:727) is also compared
with the reference: tests/golden/ref_workloads.npz holds the final-state digests the unmodified
reference core produced for each of them (oracle/gen_golden.py --workloads: 53,752 of the 65,536
envs of the timed workload after 1,205 steps; 2,738 of the 8,192 envs of C3).  The hazard envs are
pinned by the oracle only."""
import os

import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu

N_TOTAL, SEED, STEPS = 65536, 12345, 1205
SHARDS = [(1, 0), (2, 1), (4, 3), (8, 7)]          # (world, rank): the N=1 batch and last-rank shards
FIELDS = ("observations", "selected_action_masks", "infos")

_oracle_cache = {}
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_workloads.npz")


def ref_digests(name, n_total):
    """(safe mask over the workload's envs, reference digests of the safe envs in env order)."""
    z = np.load(GOLDEN)
    safe = np.unpackbits(z[f"{name}_safe"])[:n_total].astype(bool)
    return safe, z[f"{name}_digests"]


def assert_reference_digests(env, smp_actions, name, n_total, lo, hi, what):
    """The engine's final state of envs lo..hi-1 of workload `name` against the reference's
    digests, for every env in that range the reference ran."""
    safe, dig = ref_digests(name, n_total)
    pos = np.cumsum(safe) - 1                            # row of env g in `dig` (when safe)
    idx = np.nonzero(safe[lo:hi])[0]
    assert idx.size > 0
    got = po.batch_digest(env.observations[idx], env.selected_action_masks[idx], env.rewards[idx],
                          env.dones[idx], env.agent_selection[idx], env.infos[idx], smp_actions[idx])
    want = dig[pos[lo + idx]]
    bad = np.nonzero((got != want).any(1))[0]
    assert bad.size == 0, f"{what}: env {lo + int(idx[bad[0]])} differs from the reference's digest"
    return idx.size


def oracle_after(world, rank):
    """The oracle state after STEPS steps of the shard (cached: two chunk shapes share it)."""
    key = (world, rank)
    if key not in _oracle_cache:
        from city_of_gold.shard import shard, shard_seed
        _oracle_cache.clear()                        # keep one shard's oracle (1.1 GB at N=1)
        lo, hi = shard(N_TOTAL, rank, world)
        n, base = hi - lo, shard_seed(SEED, lo)
        orc, osm = po.OracleVec(n), po.OracleSampler(n, SEED, lo)
        orc.reset_threaded(base, 4, 3, 2, 100000)
        po.run_threaded(orc, osm, STEPS, po.host_threads())
        _oracle_cache[key] = (orc, osm)
    return _oracle_cache[key]


def first_bad_env(a, b):
    """(env index, leaf) of the first difference between two record arrays, or None."""
    from pyoracle import leaves
    for (nm, x), (_, y) in zip(leaves(a), leaves(b)):
        ne = (x != y).reshape(x.shape[0], -1).any(1)
        if ne.any():
            return int(np.argmax(ne)), nm
    return None


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,rank,chunk", [(w, r, c) for w, r in SHARDS for c in (20, 1000)],
                         ids=[f"{nm}_chunk{c}" for nm in ("n65536_N1", "n32768_N2_rank1", "n16384_N4_rank3",
                                                          "n8192_N8_rank7") for c in (20, 1000)])
def test_timed_workload_all_envs_vs_oracle(cg, world, rank, chunk):
    import torch

    import bench
    from city_of_gold.shard import shard
    lo, hi = shard(N_TOTAL, rank, world)
    n = hi - lo
    env, smp, runner = bench.make(cg, n, SEED, 0, first=lo)   # bench.py's own construction
    runner.set_chunk(chunk)
    first = 5 if chunk == 20 else 205
    runner.rollout(first)
    runner.rollout(STEPS - first)                         # (STEPS - first) / chunk full launches
    runner.sync()
    env.sync_host()
    acts = torch.from_dlpack(smp.dlpack()).cpu().numpy().view(po.ACTION).reshape(n)
    orc, osm = oracle_after(world, rank)
    what = f"{n} envs (global {lo}..{hi - 1}), chunk {chunk}, {STEPS} steps"
    for nm in FIELDS:
        bad = first_bad_env(getattr(env, nm), getattr(orc, nm))
        assert bad is None, f"{what}: {nm}.{bad[1]} of env {bad[0]} differs from the oracle"
    bad = first_bad_env(acts, osm.actions)
    assert bad is None, f"{what}: sampled action {bad[1]} of env {bad[0]} differs"
    for nm in ("rewards", "dones", "agent_selection"):
        assert np.array_equal(getattr(env, nm), getattr(orc, nm)), f"{what}: {nm} differs"
    assert np.array_equal(env.hazards()[1], orc.flags()), f"{what}: hazard flags differ"
    pinned = assert_reference_digests(env, acts, "c5", N_TOTAL, lo, hi, what)
    assert pinned == int((orc.flags() & po.REF_UNSAFE == 0).sum())
    steps_taken = env.infos["agent_infos"]["steps_taken"].astype(np.int64).sum()
    assert steps_taken > 0
    del runner, smp, env


@pytest.mark.timeout(600)
def test_C3_selected_all_envs_vs_oracle_and_reference(cg):
    """BASELINE config C3 at its own size and mode: 8,192 envs, 4 players, MEDIUM, seed 12345,
    sampler seeds the same, the runner's device loop over the selected masks (bench.make,
    device views), 1,000 steps in 20-step launches.  All envs against the oracle; the 2,738 the
    reference can run against its own final-state digests."""
    import torch

    import bench
    n, steps = 8192, 1000
    env, smp, runner = bench.make(cg, n, SEED, 0, difficulty=cg.MEDIUM)
    runner.set_chunk(20)
    runner.rollout(steps)
    runner.sync()
    env.sync_host()
    acts = torch.from_dlpack(smp.dlpack()).cpu().numpy().view(po.ACTION).reshape(n)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, SEED)
    orc.reset_threaded(SEED, 4, 3, 1, 100000)
    po.run_threaded(orc, osm, steps, po.host_threads())
    what = f"C3 {n} envs MEDIUM selected, {steps} steps"
    for nm in FIELDS:
        bad = first_bad_env(getattr(env, nm), getattr(orc, nm))
        assert bad is None, f"{what}: {nm}.{bad[1]} of env {bad[0]} differs from the oracle"
    bad = first_bad_env(acts, osm.actions)
    assert bad is None, f"{what}: sampled action {bad[1]} of env {bad[0]} differs"
    for nm in ("rewards", "dones", "agent_selection"):
        assert np.array_equal(getattr(env, nm), getattr(orc, nm)), f"{what}: {nm} differs"
    assert np.array_equal(env.hazards()[1], orc.flags()), f"{what}: hazard flags differ"
    assert assert_reference_digests(env, acts, "c3", n, 0, n, what) == 2738
    del runner, smp, env


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,rank", [(8, 7), (1, 0)], ids=["n8192_N8_rank7", "n65536_N1"])
def test_reference_horizon_10200_steps_vs_oracle(cg, world, rank):
    """The reference benchmark's own horizon (benchmarks.py:5: 200 warm-up + 10,000 timed steps) on
    the N=8 shard (8,192 envs, global 57,344..65,535) and on the whole N=1 batch (65,536 envs) of
    the timed workload (4 players, HARD), the trio rollout in 1,000-step launches: every env
    against the threaded C oracle after 10,200 steps (far past every test above)."""
    import torch

    import bench
    from city_of_gold.shard import shard, shard_seed
    lo, hi = shard(N_TOTAL, rank, world)
    n, base, steps = hi - lo, shard_seed(SEED, lo), 10200
    assert cg._city_of_gold.rollout_kind(n, 4, False) == "trio"
    env, smp, runner = bench.make(cg, n, SEED, 0, first=lo)
    runner.set_chunk(1000)
    runner.rollout(steps)
    runner.sync()
    env.sync_host()
    acts = torch.from_dlpack(smp.dlpack()).cpu().numpy().view(po.ACTION).reshape(n)
    orc, osm = po.OracleVec(n), po.OracleSampler(n, SEED, lo)
    orc.reset_threaded(base, 4, 3, 2, 100000)
    po.run_threaded(orc, osm, steps, po.host_threads())
    what = f"{n} envs (global {lo}..{hi - 1}), {steps} steps"
    for nm in FIELDS:
        bad = first_bad_env(getattr(env, nm), getattr(orc, nm))
        assert bad is None, f"{what}: {nm}.{bad[1]} of env {bad[0]} differs from the oracle"
    bad = first_bad_env(acts, osm.actions)
    assert bad is None, f"{what}: sampled action {bad[1]} of env {bad[0]} differs"
    for nm in ("rewards", "dones", "agent_selection"):
        assert np.array_equal(getattr(env, nm), getattr(orc, nm)), f"{what}: {nm} differs"
    assert np.array_equal(env.hazards()[1], orc.flags()), f"{what}: hazard flags differ"
    del runner, smp, env
