"""city_of_gold -- MI355X-native drop-in for the reference `city_of_gold` pybind11 module.

Same surface as the reference (src/pybind/common.cpp:5-37, src/pybind/vectorized.cpp:8-21,
include/pybind/vectorized.h:163-275):

    import city_of_gold as cg
    envs = cg.vec.get_vec_env(N)()           # class vec_cog_env_N
    samplers = cg.vec.get_vec_sampler(N)(seed)
    runner = cg.vec.get_runner(N)(envs, samplers, n_threads)
    envs.reset(seed, 4, 3, cg.Difficulty.EASY, 100000, False)

Differences, all additive: any N is accepted (the reference stops at 256 and only offers
N in {0..8, 16, 32, ..., 256}); input arrays are length/record-size checked (ValueError instead
of an out-of-bounds read); views keep their owner alive.  Runners accept two extra keyword
arguments: device_views=True keeps outputs in HBM (no per-sync host copy) and
stored_masks=True samples from the current agent's stored mask (full game dynamics); samplers
accept first_index= for a rank's block of a larger batch (city_of_gold.shard).

All computation runs in libcog_hip.so on a gfx950 GPU.  There is no CPU fallback: creating an
environment without a usable device raises RuntimeError.
"""
from __future__ import annotations

import os
import sys
import types

# torch (ROCm) and this engine load the same HIP runtime (SONAME libamdhip64.so.7).  torch rejects
# a runtime another library has already brought up ("No HIP GPUs are available"), while the
# engine is happy with torch's, so when torch is installed its GPU side is brought up first.
# COG_NO_TORCH=1 skips this (torch interop, e.g. device_tensors, then needs torch initialised
# before the first environment is created).
if not os.environ.get("COG_NO_TORCH"):
    try:
        import torch as _torch
        if _torch.cuda.is_available():
            _torch.cuda.init()
    except Exception:
        pass

from . import _city_of_gold as _C

Difficulty = _C.Difficulty
EASY, MEDIUM, HARD = _C.EASY, _C.MEDIUM, _C.HARD
# record classes (single_env.cpp:34-85); each also acts as its numpy dtype (np.zeros(n, dtype=cg.ActionData))
from .records import (ActionData, ActionMask, DeckObs, Info, ObsData, PlayerData, PlayerObservation,  # noqa: E402
                      SharedObservation, action_sampler)
device_count = _C.device_count

VEC_ENV_CLS = "vec_cog_env_"
VEC_SAMPLER_CLS = "vec_sampler_"
VEC_RUNNER_CLS = "vec_runner_"

vec = types.ModuleType("city_of_gold.vec", "Vectorized utilities")
# Q28: the reference binds samplers into `vec.env` and envs into `vec.sampler`
# (include/pybind/vectorized.h:260-273, call order vs. parameter names); the getters are right.
vec.env = types.ModuleType("city_of_gold.vec.env", "Vectorized environments")
vec.sampler = types.ModuleType("city_of_gold.vec.sampler", "Vectorized action samplers")
vec.runner = types.ModuleType("city_of_gold.vec.runner", "Vectorized runners")
for _m in (vec, vec.env, vec.sampler, vec.runner):
    sys.modules[_m.__name__] = _m


def _check_n(n):
    if isinstance(n, bool) or not isinstance(n, int) or n < 0:
        raise TypeError("number of environments must be a non-negative int")
    return int(n)


def _make_env_cls(n):
    def __init__(self, device=None):
        _C.VecEnvBase.__init__(self, n, device)

    def step_device(self, d_actions, stream=None):
        """step() with ActionData records in device memory (a torch tensor's data_ptr()),
        ordered after torch's current stream, or after `stream` (a hipStream_t handle, 0 = the
        null stream; -1: no ordering)."""
        if stream is None:
            # torch's current stream ON THE ENV'S DEVICE (a stream of another GPU cannot order it)
            stream = stream_handle(_C.VecEnvBase.shard_info(self, 0)[2])
        _C.VecEnvBase.step_device(self, d_actions, -1 if stream is None else int(stream))

    def invalidate_device(self, stream=None):
        """After writing device records (device_tensors / DLPack views): the next step takes them
        as written, as the reference's views alias its live state.  Ordered after torch's current
        stream on the env's device (or after `stream`, a hipStream_t handle; -1: no ordering)."""
        if stream is None and self.num_shards == 1:
            stream = stream_handle(_C.VecEnvBase.shard_info(self, 0)[2])
        _C.VecEnvBase.invalidate_device(self, -1 if stream is None else int(stream))

    doc = (f"Vectorized city of gold environment for {n} environments.\n\n"
           "reset() must be called first to initialize the environments before stepping.")
    return type(VEC_ENV_CLS + str(n), (_C.VecEnvBase,), {"__init__": __init__, "__doc__": doc,
                                                         "step_device": step_device,
                                                         "invalidate_device": invalidate_device,
                                                         "__module__": "city_of_gold.vec.sampler"})


def _make_sampler_cls(n):
    def __init__(self, seed=None, device=None, *, first_index=0):
        """first_index (an addition): the batch is envs [first_index, first_index + n) of a larger
        one (a rank's shard, city_of_gold.shard), so sampler i is seeded seed + first_index + i
        unwrapped, as in the whole batch (vec_sampler.h:9-13)."""
        _C.VecSamplerBase.__init__(self, n, seed, device, first_index)

    return type(VEC_SAMPLER_CLS + str(n), (_C.VecSamplerBase,), {"__init__": __init__,
                                                                 "__module__": "city_of_gold.vec.env"})


def _make_runner_cls(n):
    def __init__(self, env, sampler, n_threads=None, device_views=False, stored_masks=False):
        if env.num_envs != n:
            raise ValueError(f"runner for {n} envs got an env batch of {env.num_envs}")
        _C.RunnerBase.__init__(self, env, sampler, n_threads, device_views, stored_masks)

    return type(VEC_RUNNER_CLS + str(n), (_C.RunnerBase,), {"__init__": __init__,
                                                            "__module__": "city_of_gold.vec.runner"})


def _getter(module, prefix, factory):
    def get(n):
        n = _check_n(n)
        name = prefix + str(n)
        cls = getattr(module, name, None)
        if cls is None:
            cls = factory(n)
            setattr(module, name, cls)
        return cls

    return get


DEVICE_VIEWS = ("observations", "selected_action_masks", "rewards", "dones", "agent_selection", "infos")


def device_tensors(env, sampler=None, shard=None):
    """Shard `shard`'s device views (and the sampler's device actions) as torch tensors, zero
    copy via DLPack: rows are records, as uint8 bytes (rewards: float32 (N, 4)).  They alias the
    engine state, which the engine updates on its own HIP stream (env.stream(shard)): before
    reading them on a torch stream, order that stream after the engine with
    env.signal_stream(stream_handle(), shard) (or runner.sync()); before the engine consumes
    tensors torch wrote, env.wait_stream(stream_handle(), shard) (step_device(ptr) does that
    itself with torch's current stream).  The reference's docs suggest TensorDict over copies of
    the numpy views (docs/source/index.rst:20-26); these need no copy."""
    import torch
    if shard is None:
        if env.num_shards > 1:
            raise ValueError(f"device_tensors of a {env.num_shards}-shard env: pass shard=k "
                             "(each shard's views live on its own GPU)")
        shard = 0
    out = {nm: torch.from_dlpack(env.dlpack(nm, shard)) for nm in DEVICE_VIEWS}
    if sampler is not None:
        out["actions"] = torch.from_dlpack(sampler.dlpack()) if sampler.num_shards == 1 else None
    return out


def stream_handle(device=None):
    """torch's current HIP stream on `device` as an int handle (0 is the null stream, torch's
    default), the stream argument of step_device / wait_stream / signal_stream; None without
    torch."""
    try:
        import torch
        if torch.cuda.is_available():
            return int(torch.cuda.current_stream(device).cuda_stream)
    except Exception:
        pass
    return None


from .single import cog_env  # noqa: E402  (src/pybind/single_env.cpp: the single-env API)

get_vec_env = _getter(vec.sampler, VEC_ENV_CLS, _make_env_cls)
get_vec_sampler = _getter(vec.env, VEC_SAMPLER_CLS, _make_sampler_cls)
get_runner = _getter(vec.runner, VEC_RUNNER_CLS, _make_runner_cls)
vec.get_vec_env, vec.get_vec_sampler, vec.get_runner = get_vec_env, get_vec_sampler, get_runner

# pre-create the reference's instantiations (vectorized.h:260-267: 0..8, 16, 32, ..., 256)
for _n in list(range(0, 9)) + [16, 32, 64, 128, 256]:
    get_vec_env(_n), get_vec_sampler(_n), get_runner(_n)
del _n, _m

__all__ = ["vec", "Difficulty", "EASY", "MEDIUM", "HARD", "ObsData", "ActionMask", "ActionData", "Info",
           "DeckObs", "SharedObservation", "PlayerData", "PlayerObservation", "action_sampler", "get_vec_env",
           "get_vec_sampler", "get_runner", "device_count", "device_tensors", "stream_handle", "cog_env"]
