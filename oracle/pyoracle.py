"""TEST INFRASTRUCTURE ONLY -- ctypes wrappers around the C oracle (oracle/liboracle.so) and,
in the dev container, the reference core build (oracle/_ref/libref.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
The product package (gym-eldorado_amd/city_of_gold) never does.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref.so")

# ---- numpy records mirroring reference include/api.h:67-161 (field order as registered by
# ---- PYBIND11_NUMPY_DTYPE at src/pybind/common.cpp:8-20; pybind11 orders fields by offset) -
DECK = np.dtype({"names": ["draw", "hand", "active", "played", "discard"],
                 "formats": [("u1", (21,))] * 5, "offsets": [0, 21, 42, 63, 84], "itemsize": 105})
MASK = np.dtype({"names": ["play", "play_special", "remove", "move", "get_from_shop"],
                 "formats": [("?", (22,)), ("?", (22,)), ("?", (22,)), ("?", (7,)), ("?", (19,))],
                 "offsets": [0, 22, 44, 66, 73], "itemsize": 128})
PLAYER = np.dtype({"names": ["obs", "action_mask"], "formats": [DECK, MASK],
                   "offsets": [0, 128], "itemsize": 256})
SHARED = np.dtype({"names": ["map", "phase", "current_resources", "shop"],
                   "formats": [("u1", (48, 48, 7)), "u1", ("<f4", (3,)), ("u1", (18,))],
                   "offsets": [0, 16128, 16132, 16144], "itemsize": 16164})
OBS = np.dtype({"names": ["shared", "player_data"], "formats": [SHARED, (PLAYER, (4,))],
                "offsets": [0, 16192], "itemsize": 17216})
ACTION = np.dtype({"names": ["play", "play_special", "remove", "move", "get_from_shop"],
                   "formats": ["u1"] * 5, "offsets": [0, 1, 2, 3, 4], "itemsize": 64})
AGENT_INFO = np.dtype({"names": ["steps_taken", "returns", "travelled_hexes", "cards_added",
                                 "cards_removed", "n_machete_uses", "n_paddle_uses", "n_coin_uses",
                                 "n_card_uses"],
                       "formats": ["u1", "<f4", "<u4", "u1", "u1", "<u4", "<u4", "<u4", "<u4"],
                       "offsets": [0, 4, 8, 12, 13, 16, 20, 24, 28], "itemsize": 32})
INFO = np.dtype({"names": ["total_length", "agent_infos"], "formats": ["<u4", (AGENT_INFO, (4,))],
                 "offsets": [0, 4], "itemsize": 192})

F_MAPGEN_FAIL, F_ERASE_PAST, F_Q9_OOB, F_Q24_CLAMP = 0x01, 0x02, 0x04, 0x08
F_GRID_OVER, F_OOB_LOOKUP, F_SCAN_OVER, F_B_START_LT4 = 0x10, 0x20, 0x40, 0x80
# seeds with any of these cannot be run by the reference built against libstdc++ 11
REF_UNSAFE = F_ERASE_PAST | F_Q9_OOB | F_GRID_OVER | F_OOB_LOOKUP | F_SCAN_OVER | F_B_START_LT4 | F_Q24_CLAMP


def leaves(a, prefix=""):
    """Every leaf field of a structured array, padding excluded."""
    if a.dtype.names is None:
        yield prefix, np.ascontiguousarray(a)
        return
    for n in a.dtype.names:
        yield from leaves(a[n], prefix + "." + n if prefix else n)


def digest_update(h, a):
    for n, x in leaves(a):
        h.update(n.encode())
        h.update(x.tobytes())


def step_digest(obs, sel, rewards, dones, agent_sel, infos, actions, nbytes=8):
    h = hashlib.sha256()
    for a in (obs, sel, rewards, dones, agent_sel, infos, actions):
        digest_update(h, a)
    return h.digest()[:nbytes]


def batch_digest(obs, sel, rewards, dones, agent_sel, infos, actions, nbytes=8, chunk=2048):
    """step_digest of every env of a batch at once: row i equals step_digest(obs[i:i+1], ...,
    actions[i:i+1]) (the same leaf names and leaf bytes, in the same order, hashed as one stream).
    Returns uint8[n, nbytes]."""
    arrays = (obs, sel, rewards, dones, agent_sel, infos, actions)
    n = obs.shape[0]
    out = np.zeros((n, nbytes), dtype=np.uint8)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        parts = []
        for a in arrays:
            for nm, x in leaves(a[lo:hi]):
                name = np.frombuffer(nm.encode(), dtype=np.uint8)
                parts.append(np.broadcast_to(name, (hi - lo, name.size)))
                parts.append(np.ascontiguousarray(x).reshape(hi - lo, -1).view(np.uint8))
        rows = np.concatenate(parts, axis=1)
        for j in range(hi - lo):
            out[lo + j] = np.frombuffer(hashlib.sha256(rows[j].tobytes()).digest()[:nbytes], dtype=np.uint8)
    return out


def named_equal(a, b):
    """Compare two structured arrays field by field; return the first differing leaf or None."""
    for (n, x), (_, y) in zip(leaves(a), leaves(b)):
        if not np.array_equal(x, y):
            return n
    return None


def _view(ptr, dtype, shape):
    n = int(np.prod(shape)) * dtype.itemsize
    buf = (C.c_uint8 * n).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype).reshape(shape)


class _Lib:
    _oracle = None
    _ref = None

    @classmethod
    def oracle(cls):
        if cls._oracle is None:
            lib = C.CDLL(ORACLE_SO)
            vp, sz = C.c_void_p, C.c_size_t
            lib.orc_create.restype = vp
            lib.orc_create.argtypes = [sz]
            lib.orc_destroy.argtypes = [vp]
            lib.orc_reset.argtypes = [vp, C.c_uint32, C.c_uint8, C.c_uint8, C.c_int, C.c_uint32]
            lib.orc_reset_default.argtypes = [vp]
            lib.orc_reset_threaded.argtypes = [vp, C.c_uint32, C.c_uint8, C.c_uint8, C.c_int, C.c_uint32, C.c_int]
            lib.orc_step.argtypes = [vp, vp]
            lib.orc_step_range.argtypes = [vp, vp, sz, sz]
            for f in ("orc_obs", "orc_sel", "orc_rewards", "orc_dones", "orc_agent_sel", "orc_infos"):
                getattr(lib, f).restype = vp
                getattr(lib, f).argtypes = [vp]
            lib.orc_flags.restype = C.c_uint32
            lib.orc_flags.argtypes = [vp, sz]
            lib.orc_clear_flags.argtypes = [vp]
            lib.orc_debug_state.argtypes = [vp, sz, C.POINTER(C.c_uint32), sz]
            lib.orc_sampler_create.restype = vp
            lib.orc_sampler_create.argtypes = [sz, C.c_uint32]
            lib.orc_sampler_create_at.restype = vp
            lib.orc_sampler_create_at.argtypes = [sz, C.c_uint32, C.c_uint64]
            lib.orc_sampler_destroy.argtypes = [vp]
            lib.orc_sample.argtypes = [vp, vp]
            lib.orc_sampler_actions.restype = vp
            lib.orc_sampler_actions.argtypes = [vp]
            lib.orc_run_threaded.restype = C.c_double
            lib.orc_run_threaded.argtypes = [vp, vp, C.c_int, C.c_int]
            cls._oracle = lib
        return cls._oracle

    @classmethod
    def ref(cls):
        if cls._ref is None:
            lib = C.CDLL(REF_SO)
            vp = C.c_void_p
            lib.ref_create.restype = vp
            lib.ref_destroy.argtypes = [vp]
            lib.ref_reset.argtypes = [vp, C.c_uint32, C.c_uint8, C.c_uint8, C.c_int, C.c_uint32]
            lib.ref_reset_default.argtypes = [vp]
            lib.ref_step.argtypes = [vp, vp]
            for f in ("ref_obs", "ref_sel", "ref_rewards", "ref_dones", "ref_agent", "ref_infos"):
                getattr(lib, f).restype = vp
                getattr(lib, f).argtypes = [vp]
            lib.ref_sizeof.restype = C.c_size_t
            lib.ref_sizeof.argtypes = [C.c_int]
            lib.ref_sampler_create.restype = vp
            lib.ref_sampler_create.argtypes = [C.c_uint32]
            lib.ref_sampler_destroy.argtypes = [vp]
            lib.ref_sample.argtypes = [vp, vp]
            lib.ref_sampler_actions.restype = vp
            lib.ref_sampler_actions.argtypes = [vp]
            lib.ref_layout_name.restype = C.c_char_p
            lib.ref_layout_name.argtypes = [C.c_int]
            lib.ref_layout_offset.restype = C.c_size_t
            lib.ref_layout_offset.argtypes = [C.c_int]
            lib.ref_run_selected.restype = C.c_int
            lib.ref_run_selected.argtypes = [vp, vp, C.c_int]
            cls._ref = lib
        return cls._ref


def ref_available():
    return os.path.exists(REF_SO)


class OracleVec:
    """vec_cog_env<N> restated in C (any N)."""

    def __init__(self, n):
        self.lib = _Lib.oracle()
        self.n = n
        self.h = self.lib.orc_create(n)
        L = self.lib
        self.observations = _view(L.orc_obs(self.h), OBS, (n,))
        self.selected_action_masks = _view(L.orc_sel(self.h), MASK, (n,))
        self.rewards = _view(L.orc_rewards(self.h), np.dtype("<f4"), (n, 4))
        self.dones = _view(L.orc_dones(self.h), np.dtype("?"), (n,))
        self.agent_selection = _view(L.orc_agent_sel(self.h), np.dtype("u1"), (n,))
        self.infos = _view(L.orc_infos(self.h), INFO, (n,))

    def reset(self, seed, n_players=4, n_pieces=3, difficulty=0, max_steps=100000):
        if self.lib.orc_reset(self.h, seed & 0xFFFFFFFF, n_players, n_pieces, int(difficulty), max_steps):
            raise RuntimeError("Failed to generate map in specified maximum number of attempts")

    def reset_threaded(self, seed, n_players=4, n_pieces=3, difficulty=0, max_steps=100000, threads=None):
        """reset() split over `threads` host threads (bit-identical: envs are independent)."""
        threads = threads or host_threads()
        if self.lib.orc_reset_threaded(self.h, seed & 0xFFFFFFFF, n_players, n_pieces, int(difficulty),
                                       max_steps, threads):
            raise RuntimeError("Failed to generate map in specified maximum number of attempts")

    def reset_default(self):
        if self.lib.orc_reset_default(self.h):
            raise RuntimeError("Failed to generate map in specified maximum number of attempts")

    def step(self, actions):
        actions = np.ascontiguousarray(actions, dtype=ACTION)
        if self.lib.orc_step(self.h, actions.ctypes.data):
            raise RuntimeError("Failed to generate map in specified maximum number of attempts")

    def flags(self, i=None):
        if i is None:
            return np.array([self.lib.orc_flags(self.h, k) for k in range(self.n)], dtype=np.uint32)
        return self.lib.orc_flags(self.h, i)

    def clear_flags(self):
        self.lib.orc_clear_flags(self.h)

    def debug_state(self, i):
        out = (C.c_uint32 * 64)()
        k = self.lib.orc_debug_state(self.h, i, out, 64)
        return list(out[:k])

    def __del__(self):
        try:
            self.lib.orc_destroy(self.h)
        except Exception:
            pass


class OracleSampler:
    """vec_action_sampler(seed): sampler i seeded seed + first + i in size_t (vec_sampler.h:9-13);
    first is the global index of env 0 when the batch is one rank's block of a larger batch."""
    def __init__(self, n, seed, first=0):
        self.lib = _Lib.oracle()
        self.n = n
        self.h = self.lib.orc_sampler_create_at(n, seed & 0xFFFFFFFF, first)
        self.actions = _view(self.lib.orc_sampler_actions(self.h), ACTION, (n,))

    def get_actions(self):
        return self.actions

    def sample(self, masks):
        masks = np.ascontiguousarray(masks, dtype=MASK)
        self.lib.orc_sample(self.h, masks.ctypes.data)

    def __del__(self):
        try:
            self.lib.orc_sampler_destroy(self.h)
        except Exception:
            pass


def ref_layout():
    """{"ObsData.player_data[0].action_mask.play": offset, ...} from the reference build."""
    L = _Lib.ref()
    return {L.ref_layout_name(k).decode(): int(L.ref_layout_offset(k)) for k in range(L.ref_layout_count())}


def ref_available():
    return os.path.exists(REF_SO)


def host_threads():
    """Worker threads for oracle runs: this process's CPU share (OMP_NUM_THREADS caps it on the
    GPU box, where os.cpu_count() reports the whole machine)."""
    try:
        allowed = len(os.sched_getaffinity(0))
    except Exception:
        allowed = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", allowed) or allowed)
    return max(1, min(allowed, share))


def run_threaded(vec: OracleVec, sampler: OracleSampler, steps: int, n_threads: int) -> float:
    return _Lib.oracle().orc_run_threaded(vec.h, sampler.h, steps, n_threads)


class RefVec1:
    """The reference's own vec_cog_env<1> (dev container only; screened seeds only)."""

    def __init__(self):
        self.lib = _Lib.ref()
        L = self.lib
        assert L.ref_sizeof(0) == 17216 and L.ref_sizeof(1) == 128 and L.ref_sizeof(3) == 192
        self.h = L.ref_create()
        self.observations = _view(L.ref_obs(self.h), OBS, (1,))
        self.selected_action_masks = _view(L.ref_sel(self.h), MASK, (1,))
        self.rewards = _view(L.ref_rewards(self.h), np.dtype("<f4"), (1, 4))
        self.dones = _view(L.ref_dones(self.h), np.dtype("?"), (1,))
        self.agent_selection = _view(L.ref_agent(self.h), np.dtype("u1"), (1,))
        self.infos = _view(L.ref_infos(self.h), INFO, (1,))

    def reset(self, seed, n_players=4, n_pieces=3, difficulty=0, max_steps=100000):
        if self.lib.ref_reset(self.h, seed & 0xFFFFFFFF, n_players, n_pieces, int(difficulty), max_steps):
            raise RuntimeError("Failed to generate map in specified maximum number of attempts")

    def step(self, actions):
        actions = np.ascontiguousarray(actions, dtype=ACTION)
        if self.lib.ref_step(self.h, actions.ctypes.data):
            raise RuntimeError("Failed to generate map in specified maximum number of attempts")

    def run_selected(self, sampler, steps):
        """`steps` x (sampler.sample(selected_action_masks); step(actions)) inside the reference."""
        if self.lib.ref_run_selected(self.h, sampler.h, int(steps)):
            raise RuntimeError("Failed to generate map in specified maximum number of attempts")

    def __del__(self):
        try:
            self.lib.ref_destroy(self.h)
        except Exception:
            pass


class RefSampler1:
    def __init__(self, seed):
        self.lib = _Lib.ref()
        self.h = self.lib.ref_sampler_create(seed & 0xFFFFFFFF)
        self.actions = _view(self.lib.ref_sampler_actions(self.h), ACTION, (1,))

    def get_actions(self):
        return self.actions

    def sample(self, masks):
        masks = np.ascontiguousarray(masks, dtype=MASK)
        self.lib.ref_sample(self.h, masks.ctypes.data)

    def __del__(self):
        try:
            self.lib.ref_sampler_destroy(self.h)
        except Exception:
            pass


def stored_masks(env):
    """Full-dynamics driver mask: the current agent's stored mask (test_environment.cpp:97-98)."""
    n = env.agent_selection.shape[0]
    return env.observations["player_data"]["action_mask"][np.arange(n), env.agent_selection].copy()
