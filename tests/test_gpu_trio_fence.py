"""GPU: the trio rollout with its progress counters published by workgroup-scope release stores
(libcog_hip_fence.so, -DCOG_TRIO_FENCE) against the C oracle, beside the product's relaxed form.

The product's trio (cog_engine.hip cnt_store) publishes each wave's LDS records with a
wavefront-scope fence and a relaxed LDS store of the counter: correct because one wave's LDS
instructions complete in issue order, which the compiler fence preserves.  The fence build is
the conservative form of the same kernel.  Both run the bench's loop on the same seeds -- 4,096
envs (one workgroup per CU: the LAT form) and 40,960 (640 workgroups, two per CU) in 20-step
launches with episode ends (max_steps 15) -- and both must equal the oracle byte for byte, so a
toolchain change that reorders the relaxed form's LDS stores surfaces here as a parity failure
of one build and not the other.  Driven through the C ABI by ctypes in a
subprocess, so the fence library never shares a process with the product's."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "gym-eldorado_amd", "city_of_gold")

SCRIPT = r'''
import ctypes as C, os, sys
import numpy as np
sys.path[:0] = [sys.argv[1]]
import pyoracle as po
lib_path, n, max_steps, steps = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), 60
L = C.CDLL(lib_path)
L.cog_last_error.restype = C.c_char_p
vp = C.c_void_p
L.cog_env_create.argtypes = [C.c_size_t, C.c_int, C.POINTER(vp)]
L.cog_env_reset.argtypes = [vp, C.c_uint32, C.c_uint8, C.c_uint8, C.c_int, C.c_uint32, C.c_int]
L.cog_sampler_create.argtypes = [C.c_size_t, C.c_uint64, C.c_int, C.POINTER(vp)]
L.cog_sampler_actions.restype = vp
L.cog_sampler_actions.argtypes = [vp]
L.cog_runner_create.argtypes = [vp, vp, C.c_size_t, C.c_uint32, C.POINTER(vp)]
L.cog_runner_set_chunk.argtypes = [vp, C.c_int]
L.cog_runner_rollout.argtypes = [vp, C.c_int]
L.cog_runner_sync.argtypes = [vp]
for f in ("cog_runner_destroy", "cog_sampler_destroy", "cog_env_destroy"):
    getattr(L, f).argtypes = [vp]


class Views(C.Structure):
    _fields_ = [("n_envs", C.c_size_t)] + [(f, vp) for f in (
        "observations", "selected_action_masks", "rewards", "dones", "agent_selection", "infos",
        "d_observations", "d_selected_action_masks", "d_rewards", "d_dones", "d_agent_selection", "d_infos")]


L.cog_env_get_views.argtypes = [vp, C.POINTER(Views)]


def view(ptr, dtype, shape):
    k = int(np.prod(shape)) * dtype.itemsize
    return np.frombuffer((C.c_uint8 * k).from_address(ptr), dtype=dtype).reshape(shape)


def ok(rc):
    assert rc == 0, L.cog_last_error()


seed = 4242
env, smp, run = vp(), vp(), vp()
ok(L.cog_env_create(n, 0, C.byref(env)))
ok(L.cog_env_reset(env, seed, 4, 3, 2, max_steps, 0))
ok(L.cog_sampler_create(n, seed, 0, C.byref(smp)))
v = Views()
ok(L.cog_env_get_views(env, C.byref(v)))                     # host views: sync() refreshes them
ok(L.cog_runner_create(env, smp, 0, 0, C.byref(run)))        # (and the sampler's actions view)
ok(L.cog_runner_set_chunk(run, 20))
ok(L.cog_runner_rollout(run, steps))
ok(L.cog_runner_sync(run))
orc, osm = po.OracleVec(n), po.OracleSampler(n, seed)
orc.reset_threaded(seed, 4, 3, 2, max_steps)
po.run_threaded(orc, osm, steps, po.host_threads())
for nm, dt in (("observations", po.OBS), ("selected_action_masks", po.MASK), ("infos", po.INFO)):
    bad = po.named_equal(view(getattr(v, nm), dt, (n,)), getattr(orc, nm))
    assert bad is None, f"{nm}.{bad} differs from the oracle"
assert np.array_equal(view(v.rewards, np.dtype("<f4"), (n, 4)), orc.rewards)
assert np.array_equal(view(v.dones, np.dtype("?"), (n,)), orc.dones)
assert np.array_equal(view(v.agent_selection, np.dtype("u1"), (n,)), orc.agent_selection)
assert po.named_equal(view(L.cog_sampler_actions(smp), po.ACTION, (n,)), osm.actions) is None
ended = int(orc.infos["total_length"].astype(bool).sum())
L.cog_runner_destroy(run); L.cog_sampler_destroy(smp); L.cog_env_destroy(env)
print("OK", ended)
'''


@pytest.mark.parametrize("lib", ["libcog_hip_fence.so", "libcog_hip.so"])
@pytest.mark.parametrize("n", [4096, 40960])
def test_trio_counter_publication_forms_vs_oracle(tmp_path, lib, n):
    path = os.path.join(LIBDIR, lib)
    assert os.path.exists(path), f"{lib} not built (gym-eldorado_amd/build_ext.py)"
    script = tmp_path / "fence.py"
    script.write_text(SCRIPT)
    r = subprocess.run([sys.executable, str(script), os.path.join(ROOT, "oracle"), path, str(n), "15"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    last = r.stdout.strip().splitlines()[-1]
    assert last.startswith("OK") and int(last.split()[1]) > 0, "no episode ended: the test lost a case"
