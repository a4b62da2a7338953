"""Index sharding of a global env batch across ranks / GPUs (no collectives needed).

Environments are independent (env i of an N batch == a 1-env batch seeded seed+i),
so a global batch of n_total envs is split into contiguous blocks, exactly like the reference
runner splits envs across worker threads (reference include/runner.h:36-38: block size
n // workers, the last worker takes the remainder).  Rank r steps its block with env seeds
seed + global_index and sampler seeds sampler_seed + global_index, so results are invariant to
the number of ranks:

    lo, hi = shard(n_total, rank, world)
    env.reset(shard_seed(seed, lo), ...)                          # (u32)(seed + lo + i)
    smp = cg.vec.get_vec_sampler(hi - lo)(seed, first_index=lo)   # seed + lo + i, not wrapped

The two seeds wrap differently in the reference: the env's sum is truncated to u32 by
cog_env::reset's parameter (vec_environment.h:41), the sampler's is a size_t
(vec_sampler.h:9-13), so a sampler must not be given the wrapped base shard_seed(seed, lo).
"""
from __future__ import annotations


def shard(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """[lo, hi) of the envs rank `rank` of `world` owns."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    block = n_total // world
    lo = rank * block
    hi = lo + block if rank < world - 1 else n_total
    return lo, hi


def shard_seed(seed: int, lo: int) -> int:
    """Env reset seed of a shard whose first env has global index lo (u32 wrap like
    vec_environment.h:41).  Samplers take (seed, first_index=lo) instead."""
    return (seed + lo) & 0xFFFFFFFF
