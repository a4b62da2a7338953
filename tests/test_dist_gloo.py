"""CPU, world_size 2 over gloo: the multi-GPU path shards envs by index with no data-path
collective.  Each rank steps its shard (C oracle standing in for its GPU) with global-index
seeds; the gathered per-env digests must equal a single-process run of the whole batch.
Also exercises bench.py's timing barrier / max / sum helpers."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N_TOTAL, STEPS, SEED = 20, 120, 4242


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def digests(vec, smp, lo, hi):
    import pyoracle as po
    return [po.step_digest(vec.observations[i:i + 1], vec.selected_action_masks[i:i + 1],
                           vec.rewards[i:i + 1], vec.dones[i:i + 1], vec.agent_selection[i:i + 1],
                           vec.infos[i:i + 1], smp.actions[i:i + 1]) for i in range(lo, hi)]


def rollout(n, seed, steps, first=0, sampler_seed=None):
    """Envs [first, first + n) of a batch seeded `seed`: env reset seed (u32)(seed + first)
    (shard_seed), sampler seeds seed + first + i unwrapped (first_index); sampler_seed replaces
    the sampler's (seed, first) by (sampler_seed, 0) -- the wrapped base a rank used to pass."""
    import pyoracle as po
    from city_of_gold.shard import shard_seed
    vec = po.OracleVec(n)
    smp = po.OracleSampler(n, seed, first) if sampler_seed is None else po.OracleSampler(n, sampler_seed)
    vec.reset(shard_seed(seed, first), 4, 3, 2, 30)
    for _ in range(steps):
        smp.sample(po.stored_masks(vec))
        vec.step(smp.actions)
    return digests(vec, smp, 0, n)


def worker(rank, world, port, root, q, n_total=N_TOTAL, seed=SEED, steps=STEPS):
    import sys
    for p in (os.path.join(root, "gym-eldorado_amd"), os.path.join(root, "oracle"), root):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    from city_of_gold.shard import shard
    d = bench.Dist(world)
    lo, hi = shard(n_total, rank, world)
    mine = rollout(hi - lo, seed, steps, first=lo)
    gathered = [None] * world
    d.dist.all_gather_object(gathered, (lo, [x.hex() for x in mine]))
    class _Runner:                                         # (no GPU: sync() stands in for the engine's)
        calls = 0

        def sync(self):
            _Runner.calls += 1
    r = _Runner()
    d.barrier_sync(r)                                      # the bench's timed-region helpers
    d.sync(r)
    d.barrier()
    assert _Runner.calls == 3
    mx = d.max(float(rank + 1))
    tot = d.sum(float(hi - lo))
    if rank == 0:
        q.put((gathered, mx, tot))
    d.close()


def run_two_ranks(n_total, seed, steps):
    """gloo world 2: the gathered per-env digests of both ranks' shards, in global order"""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, root, q, n_total, seed, steps)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, mx, tot = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert mx == 2.0 and tot == n_total
    merged = []
    for lo, ds in sorted(gathered):
        merged.extend(ds)
    return merged


@pytest.mark.timeout(300)
def test_two_rank_shards_equal_single_process():
    merged = run_two_ranks(N_TOTAL, SEED, STEPS)
    assert merged == [x.hex() for x in rollout(N_TOTAL, SEED, STEPS)]


@pytest.mark.timeout(300)
def test_two_rank_shards_seed_exact_past_u32():
    """Base seed 2^32 - 1,000 over 2,000 envs: rank 1's envs have seed + global index >= 2^32.  The
    env seeds wrap (vec_environment.h:41, u32 parameter), the sampler seeds do not
    (vec_sampler.h:9-13, size_t): the shards sampled with (seed, first_index=lo) equal the whole
    batch, and the wrapped sampler base (seed + lo) & 0xffffffff -- what ranks passed before --
    does not."""
    n_total, seed, steps = 2000, 2 ** 32 - 1000, 40
    merged = run_two_ranks(n_total, seed, steps)
    full = [x.hex() for x in rollout(n_total, seed, steps)]
    assert merged == full
    lo = n_total // 2
    from city_of_gold.shard import shard_seed
    wrapped = [x.hex() for x in rollout(n_total - lo, seed, steps, first=lo, sampler_seed=shard_seed(seed, lo))]
    assert wrapped != full[lo:], "the wrapped sampler base should sample differently (the test's control)"


def test_shard_blocks():
    from city_of_gold.shard import shard
    assert [shard(10, r, 3) for r in range(3)] == [(0, 3), (3, 6), (6, 10)]
    assert sum(h - l for l, h in (shard(65536 * 8, r, 8) for r in range(8))) == 65536 * 8


def test_bench_roofline_store_model():
    """bench.roofline: HBM by the counter-measured bytes of the launch's own shape (envs, steps per
    launch, rollout kind) over the launch time, frac <= 1 for any real traffic; SURVEY 8d's 800
    B/env-step as a labelled equivalent; round 3's store model; the limiter's busy fraction from a
    stamps profile of the shape; nulls (with a note) for a shape or kernel the profile did not
    measure."""
    import bench
    n, k, launch = 65536, 20, 100e-6
    prof = {"store_costs": {"c_hit_s": 5e-12, "c_miss_s": 16e-12},
            "rollouts": {"65536:20": {"kind": "trio", "envs": n, "chunk": k, "bytes_per_launch": 3.6e8,
                                      "l2_per_launch": {"writes": 8.0e6, "hits": 4.5e6, "misses": 3.5e6},
                                      "per_wave_step": {"valu": 1000.0}},
                         "8192:20": {"kind": "duo", "envs": 8192, "chunk": k, "bytes_per_launch": 2.0e7,
                                     "companion": {"bytes_per_launch": 1.0e6},
                                     "l2_per_launch": {"writes": 1.0e6, "hits": 1.0e6, "misses": 1.0e4}}}}
    stamps = {"shapes": {"65536": {"busy_ticks_per_step": 3000.0, "wait_ticks_per_step": 600.0,
                                   "ticks_per_step": 3600.0, "busy_frac": 3000.0 / 3600.0}}}
    r = bench.roofline(prof, n, k, launch, "trio", stamps)
    alg = 800 * n * k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0 and r["traffic"] == 3.6e8
    assert abs(r["achieved"] - 3.6e8 / launch / 1e9) < 1e-9 * r["achieved"]
    assert abs(r["frac"] - r["achieved"] / 8000.0) < 1e-12 and 0 < r["frac"] <= 1
    assert abs(r["survey_8d_equivalent"]["GBs"] - alg / launch / 1e9) < 1e-6
    assert r["limiter"]["busy_frac"] == 3000.0 / 3600.0
    t_store = 4.5e6 * 5e-12 + 3.5e6 * 16e-12
    assert abs(r["store_model"]["frac"] - t_store / launch) < 1e-12
    assert abs(r["env_steps_per_s"] - n * k / launch) < 1e-6 * r["env_steps_per_s"]
    assert r["valu_issue"]["valu_per_wave_step"] == 1000.0 and r["kernel"].startswith("k_env_rollout_trio")
    issue = {"two_per_cu": {"per_step_instructions": 600, "mix": {"valu": 200, "salu": 400},
                            "ticks_per_step_issue": 1800.0, "ticks_per_step_dependent": 5400.0},
             "lat": {"per_step_instructions": 500, "mix": {"valu": 100, "salu": 400},
                     "ticks_per_step_issue": 900.0, "ticks_per_step_dependent": 4000.0}}
    ri = bench.roofline(prof, n, k, launch, "trio", stamps, issue)     # 65,536 envs: two per CU
    assert ri["limiter"]["issue_frac"] == 1800.0 / 3000.0 and ri["limiter"]["dependent_chain_frac"] == 5400.0 / 3000.0
    assert ri["limiter"]["issue"]["kernel_form"] == "two_per_cu"
    assert "issue_frac" not in r["limiter"]                          # (no issue profile given)
    small = bench.roofline(prof, 8192, k, 50e-6, "duo")            # its own entry, not the 65,536 one
    assert small["traffic"] == 2.1e7 and small["kernel"].startswith("k_env_rollout_duo")
    assert "busy_frac" not in small["limiter"]
    assert abs(small["store_model"]["frac"] - (1.0e6 * 5e-12 + 1.0e4 * 16e-12) / 50e-6) < 1e-12
    for other in (bench.roofline(prof, 16384, k, launch, "duo"),       # shape not profiled
                  bench.roofline(prof, 8192, k, launch, "pipe"),       # profiled with another kernel
                  bench.roofline(prof, n, 1000, launch, "trio")):      # another launch length
        assert other["traffic"] is None and other["store_model"] is None and "traffic unknown" in other["note"]
        assert other["frac"] is None and other["survey_8d_equivalent"]["x_peak"] > 0
