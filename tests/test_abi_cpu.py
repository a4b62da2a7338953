"""CPU: the C-ABI library loads and exports every symbol include/*.h declares; the Python
mirror imports, mirrors the reference names/dtypes and fails loudly without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

import pyoracle as po

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "gym-eldorado_amd", "city_of_gold", "libcog_hip.so")


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "cog.h")).read()
    return sorted(set(re.findall(r"COG_API\s+[\w\s\*]+?\b(cog_\w+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for must in ("cog_env_create", "cog_env_reset", "cog_env_step", "cog_sampler_sample",
                 "cog_runner_step", "cog_runner_sync", "cog_last_error"):
        assert must in syms


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"libcog_hip.so lacks {missing}"


def test_abi_version_and_no_device():
    lib = ctypes.CDLL(LIB)
    assert lib.cog_abi_version() == 1
    n = ctypes.c_int(-1)
    assert lib.cog_device_count(ctypes.byref(n)) == 0
    if n.value == 0:
        h = ctypes.c_void_p()
        rc = lib.cog_env_create(ctypes.c_size_t(4), 0, ctypes.byref(h))
        assert rc == -4 and not h.value                # COG_ERR_NODEVICE: no CPU fallback
        lib.cog_last_error.restype = ctypes.c_char_p
        assert b"no HIP device" in lib.cog_last_error()


def test_python_surface(cg):
    assert cg.vec.get_vec_env(16).__name__ == "vec_cog_env_16"
    assert cg.vec.get_vec_sampler(16).__name__ == "vec_sampler_16"
    assert cg.vec.get_runner(16).__name__ == "vec_runner_16"
    assert cg.vec.get_vec_env(65536).__name__ == "vec_cog_env_65536"   # beyond the reference cap
    # Q28 placement: samplers live in vec.env, envs in vec.sampler
    assert hasattr(cg.vec.env, "vec_sampler_256") and hasattr(cg.vec.sampler, "vec_cog_env_256")
    assert int(cg.Difficulty.HARD) == 2 and cg.EASY == cg.Difficulty.EASY


def test_dtypes_match_reference_layout(cg):
    assert np.dtype(cg.ObsData) == po.OBS and np.dtype(cg.ActionMask) == po.MASK
    assert np.dtype(cg.ActionData) == po.ACTION and np.dtype(cg.Info) == po.INFO
    assert cg.ObsData.dtype.itemsize == 17216 and cg.ActionMask.dtype.itemsize == 128
    assert cg.ObsData.dtype["player_data"].base["action_mask"]["play"] == np.dtype(("?", (22,)))


def dtype_offset(dt, path):
    """Byte offset of a dotted numpy field path ("player_data[1].obs.hand") in dtype dt."""
    off = 0
    for part in path.split("."):
        m = re.fullmatch(r"(\w+)(?:\[(\d+)\])?", part)
        sub, o = dt.fields[m.group(1)][:2]
        off += o
        if m.group(2) is not None:
            off += int(m.group(2)) * sub.base.itemsize
            sub = sub.base
        dt = sub
    return off


def test_field_offsets_match_the_reference_build(cg):
    """Every named field's offset in the module's dtypes against offsetof-style addresses taken
    in a build of the unmodified reference headers (oracle/ref_harness.cpp, oracle/_ref)."""
    if not po.ref_available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    lay = po.ref_layout()
    assert len(lay) >= 40
    for name, ref_off in lay.items():
        rec, path = name.split(".", 1)
        assert dtype_offset(np.dtype(getattr(cg, rec)), path) == ref_off, name


def test_no_gpu_fails_loudly(cg):
    if cg.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(RuntimeError, match="no HIP device"):
        cg.vec.get_vec_env(4)()
    with pytest.raises(RuntimeError):
        cg.vec.get_vec_sampler(4)(0)


def test_default_device_order(cg, monkeypatch):
    """device=None: COG_DEVICES, else COG_DEVICE, else LOCAL_RANK, else GPU 0 -- never an implicit
    split over every visible GPU; bench.device_of follows the same order."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    for k in ("COG_DEVICES", "COG_DEVICE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    dd = cg._city_of_gold.default_devices
    assert dd() == [0]
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert dd() == [3]
    d = type("D", (), {"local": 3})()
    assert bench.device_of(d) == 3
    monkeypatch.setenv("COG_DEVICE", "1")
    assert dd() == [1] and bench.device_of(d) == 1
    monkeypatch.setenv("COG_DEVICES", "0,2")
    assert dd() == [0, 2]
    monkeypatch.setenv("COG_DEVICES", "0,x")
    with pytest.raises(ValueError):
        dd()


def test_rollout_kind_selection():
    """cog_rollout_kind (a host-only query, no device needed): the selected-mask loop with >= 3
    players takes the trio rollout at every shard size; the stored masks and 2-player batches keep
    round 3's kernels by size (duo <= 16,384, pipe <= 32,768, wave above: cog_engine.hip
    rollout_kind)."""
    if os.environ.get("COG_ROLLOUT") or os.environ.get("COG_TRIO"):
        pytest.skip("rollout kind forced by the environment")
    lib = ctypes.CDLL(LIB)
    kind = lambda n, p, stored: lib.cog_rollout_kind(ctypes.c_size_t(n), p, stored)   # noqa: E731
    TRIO, DUO, WAVE, PIPE = 3, 0, 1, 2
    for n in (64, 4096, 8192, 16384, 32768, 53752, 65536, 131072):
        assert kind(n, 4, 0) == TRIO and kind(n, 3, 0) == TRIO
    for p, stored in ((2, 0), (4, 1), (3, 1)):
        assert kind(8192, p, stored) == DUO and kind(16384, p, stored) == DUO
        assert kind(24576, p, stored) == PIPE and kind(32768, p, stored) == PIPE
        assert kind(65536, p, stored) == WAVE
