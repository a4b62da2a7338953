"""GPU: INTEGRATION.md section 3 end to end -- the raw C ABI (include/cog.h) driven through ctypes
with no pybind module in between, the way a consumer without a compiler binds it.  Create, reset,
then the reference's loop (`sample(selected_action_masks); step(actions)`, benchmarks.py:47-51)
through cog_sampler_sample / cog_env_step on the persistent host views, every view compared with
the C oracle after every step; a runner rollout through cog_runner_* at the end."""
import ctypes as C
import os

import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "gym-eldorado_amd", "city_of_gold", "libcog_hip.so")


class Views(C.Structure):                                  # cog_env_views (include/cog.h)
    _fields_ = [("n_envs", C.c_size_t)] + [(f, C.c_void_p) for f in (
        "observations", "selected_action_masks", "rewards", "dones", "agent_selection", "infos",
        "d_observations", "d_selected_action_masks", "d_rewards", "d_dones", "d_agent_selection", "d_infos")]


def view(ptr, dtype, shape):
    n = int(np.prod(shape)) * dtype.itemsize
    return np.frombuffer((C.c_uint8 * n).from_address(ptr), dtype=dtype).reshape(shape)


def lib():
    L = C.CDLL(LIB)
    L.cog_last_error.restype = C.c_char_p
    L.cog_env_create.argtypes = [C.c_size_t, C.c_int, C.POINTER(C.c_void_p)]
    L.cog_env_reset.argtypes = [C.c_void_p, C.c_uint32, C.c_uint8, C.c_uint8, C.c_int, C.c_uint32, C.c_int]
    L.cog_env_get_views.argtypes = [C.c_void_p, C.POINTER(Views)]
    L.cog_env_step.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.cog_env_destroy.argtypes = [C.c_void_p]
    L.cog_sampler_create.argtypes = [C.c_size_t, C.c_uint64, C.c_int, C.POINTER(C.c_void_p)]
    L.cog_sampler_sample.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.cog_sampler_actions.restype = C.c_void_p
    L.cog_sampler_actions.argtypes = [C.c_void_p]
    L.cog_sampler_destroy.argtypes = [C.c_void_p]
    L.cog_runner_create.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.POINTER(C.c_void_p)]
    L.cog_runner_rollout.argtypes = [C.c_void_p, C.c_int]
    L.cog_runner_sync.argtypes = [C.c_void_p]
    L.cog_runner_destroy.argtypes = [C.c_void_p]
    return L


def test_ctypes_abi_reference_loop_vs_oracle():
    L = lib()
    n, seed, steps = 1024, 12345, 60
    env, smp, run = C.c_void_p(), C.c_void_p(), C.c_void_p()
    assert L.cog_env_create(n, 0, C.byref(env)) == 0, L.cog_last_error()
    assert L.cog_env_reset(env, seed, 4, 3, 2, 100000, 0) == 0, L.cog_last_error()
    assert L.cog_sampler_create(n, seed, 0, C.byref(smp)) == 0, L.cog_last_error()
    v = Views()
    assert L.cog_env_get_views(env, C.byref(v)) == 0 and v.n_envs == n
    obs = view(v.observations, po.OBS, (n,))
    sel = view(v.selected_action_masks, po.MASK, (n,))
    rew = view(v.rewards, np.dtype("<f4"), (n, 4))
    dones = view(v.dones, np.dtype("?"), (n,))
    agent = view(v.agent_selection, np.dtype("u1"), (n,))
    infos = view(v.infos, po.INFO, (n,))
    acts = view(L.cog_sampler_actions(smp), po.ACTION, (n,))
    orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
    orc.reset(seed, 4, 3, 2, 100000)
    assert po.named_equal(obs, orc.observations) is None
    for t in range(steps):
        assert L.cog_sampler_sample(smp, v.selected_action_masks, n) == 0, L.cog_last_error()
        osm.sample(orc.selected_action_masks)
        assert po.named_equal(acts, osm.actions) is None, f"actions differ at step {t}"
        assert L.cog_env_step(env, L.cog_sampler_actions(smp), n) == 0, L.cog_last_error()
        orc.step(osm.actions)
        for nm, a, b in (("observations", obs, orc.observations), ("selected_action_masks", sel,
                         orc.selected_action_masks), ("infos", infos, orc.infos)):
            bad = po.named_equal(a, b)
            assert bad is None, f"{nm}.{bad} differs from the oracle at step {t}"
        assert np.array_equal(rew, orc.rewards) and np.array_equal(dones, orc.dones)
        assert np.array_equal(agent, orc.agent_selection)
    # the runner: 100 more steps in one call, host views refreshed by the sync (flags 0)
    assert L.cog_runner_create(env, smp, 0, 0, C.byref(run)) == 0, L.cog_last_error()
    assert L.cog_runner_rollout(run, 100) == 0 and L.cog_runner_sync(run) == 0, L.cog_last_error()
    po.run_threaded(orc, osm, 100, po.host_threads())
    assert po.named_equal(obs, orc.observations) is None
    assert po.named_equal(acts, osm.actions) is None
    L.cog_runner_destroy(run)
    L.cog_sampler_destroy(smp)
    L.cog_env_destroy(env)
