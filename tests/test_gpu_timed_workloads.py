"""GPU: the EXACT workloads bench.py times, every env against the C oracle.

For the N=1 headline batch (65,536 envs, 4 players, HARD, seeds 12345 + i) and for the last
rank's shard at N = 2, 4 and 8 (`shard(65536, N-1, N)`: 32,768 / 16,384 / 8,192 envs, seeds
`shard_seed(12345, lo)` = 12345 + global index), the engine is built by bench.py's own `make()`
and driven by `runner.rollout` in the two launch shapes the bench uses:
  - chunk 20: a 5-step launch (the driver's `--warmup 5`), then 20-step launches (`--steps 20`);
  - chunk 1000: 205 steps, then one 1,000-step launch (bench's default shape).
The kernels are the bench's (cog_engine.hip rollout_kind): 16,384 and 8,192 envs the duo rollout
(k_env_rollout_duo + k_env_fixup), 32,768 the two-wave k_env_rollout_pipe, 65,536 k_env_rollout.
After 1,205 steps ALL envs are compared with a threaded oracle run of the reference runner loop
(`sample(selected_action_masks); step(actions)`, benchmarks/benchmarks.py:47-51,
include/runner.h:33-62): every named field of ObsData / ActionMask / Info, rewards, dones,
agent_selection, the sampled actions and the per-env hazard flags.  Bit-exact."""
import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu

N_TOTAL, SEED, STEPS = 65536, 12345, 1205
SHARDS = [(1, 0), (2, 1), (4, 3), (8, 7)]          # (world, rank): the N=1 batch and last-rank shards
FIELDS = ("observations", "selected_action_masks", "infos")

_oracle_cache = {}


def oracle_after(world, rank):
    """The oracle state after STEPS steps of the shard (cached: two chunk shapes share it)."""
    key = (world, rank)
    if key not in _oracle_cache:
        from city_of_gold.shard import shard, shard_seed
        _oracle_cache.clear()                        # keep one shard's oracle (1.1 GB at N=1)
        lo, hi = shard(N_TOTAL, rank, world)
        n, base = hi - lo, shard_seed(SEED, lo)
        orc, osm = po.OracleVec(n), po.OracleSampler(n, base)
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
    from city_of_gold.shard import shard, shard_seed
    lo, hi = shard(N_TOTAL, rank, world)
    n, base = hi - lo, shard_seed(SEED, lo)
    env, smp, runner = bench.make(cg, n, base, 0)           # bench.py's own construction
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
    steps_taken = env.infos["agent_infos"]["steps_taken"].astype(np.int64).sum()
    assert steps_taken > 0
    del runner, smp, env
