"""Record classes and the single masked sampler of the reference module.

The reference binds its POD records as classes (src/pybind/single_env.cpp:34-85): `ObsData`
(shared, player_data), `SharedObservation` (phase, map, shop, resources), `PlayerData`
(action_mask, obs), `ActionMask` (play, play_special, remove, move, get_from_shop),
`PlayerObservation` (draw, hand, played, discard) and `ActionData` (five read-write fields),
plus `action_sampler(seed)` with `.sample(mask) -> ActionData` (src/pybind/common.cpp:25-27,
include/sampler.h:9-79).

Here every record class is a view of one numpy structured record with the reference's byte
layout (the dtypes registered at common.cpp:8-20), so a record and the structured-array views
of the vec API share memory and convert both ways:

    rec = cg.ObsData()                     # a fresh zeroed record (additive: the reference has
                                           # no py::init for its records)
    rec = cg.ObsData(env.observations[3, ...])   # a view of env 3's record (a 0-d view; a
                                                 # structured scalar env.observations[3] is copied)
    rec.player_data[1].action_mask.play    # numpy view, writable by assignment like bind_array
    np.zeros(8, dtype=cg.ActionData)       # the classes also act as their numpy dtype

`action_sampler` draws on the GPU (a batch of one of the engine's sampler kernel): the engine
has no CPU path.
"""
from __future__ import annotations

import numpy as np

from . import _city_of_gold as _C


class _Record:
    """One record of `dtype`: a 0-d view of a structured array (shares memory with it)."""

    dtype: np.dtype = None
    __slots__ = ("_a",)

    def __init__(self, rec=None):
        if rec is None:
            a = np.zeros((), dtype=self.dtype)
            self._init_fresh(a)
        else:
            if isinstance(rec, _Record):
                rec = rec._a
            a = np.asarray(rec) if not isinstance(rec, np.void) else np.asarray(rec).copy()
            if a.dtype != self.dtype or a.size != 1:
                raise ValueError(f"expected one {type(self).__name__} record")
            a = a.reshape(())
        object.__setattr__(self, "_a", a)

    def _init_fresh(self, a):
        pass

    @property
    def record(self):
        """The numpy structured record (0-d array view) behind this object."""
        return self._a

    def __getitem__(self, field):          # structured-record indexing: rec["total_length"]
        return self._a[field]

    def _arr(self, name):
        return self._a[name]

    def _set(self, name, value):
        dst = self._a[name]
        v = np.asarray(value)
        if v.size != dst.size:
            raise RuntimeError("Invalid array size")       # bind_array's setter (common.h:27-29)
        dst[...] = v.reshape(dst.shape)

    def __repr__(self):
        return f"{type(self).__name__}({self._a!r})"


def _array_prop(name, doc=None):
    return property(lambda self: self._arr(name), lambda self, v: self._set(name, v), doc=doc)


def _mask_defaults(a):
    """ActionMask() (api.h:101-118): index 0 of every head set, the rest clear."""
    for head in ("play", "play_special", "remove", "move", "get_from_shop"):
        a[head][...] = False
        a[head][..., 0] = True


class ActionMask(_Record):
    """api.h:95-119; the reference's class has array properties play, play_special, remove,
    move, get_from_shop (single_env.cpp:62-72)."""

    dtype = _C.ActionMask
    __slots__ = ()

    def _init_fresh(self, a):
        _mask_defaults(a)

    play = _array_prop("play")
    play_special = _array_prop("play_special")
    remove = _array_prop("remove")
    move = _array_prop("move")
    get_from_shop = _array_prop("get_from_shop")


class PlayerObservation(_Record):
    """DeckObs (api.h:67-82), bound as PlayerObservation (single_env.cpp:74-82)."""

    dtype = _C.DeckObs
    __slots__ = ()
    draw = _array_prop("draw")
    hand = _array_prop("hand")
    active = _array_prop("active")           # additive: the reference does not bind `active`
    played = _array_prop("played")
    discard = _array_prop("discard")


DeckObs = PlayerObservation


class PlayerData(_Record):
    """api.h:121-124 (single_env.cpp:56-60)."""

    dtype = _C.ObsData.fields["player_data"][0].base
    __slots__ = ()

    def _init_fresh(self, a):
        _mask_defaults(a["action_mask"])

    @property
    def action_mask(self):
        return ActionMask(self._a["action_mask"])

    @property
    def obs(self):
        return PlayerObservation(self._a["obs"])


class SharedObservation(_Record):
    """api.h:88-93 (single_env.cpp:41-54): phase (read-only), map, shop, resources."""

    dtype = _C.ObsData.fields["shared"][0]
    __slots__ = ()

    @property
    def phase(self):
        return int(self._a["phase"])

    map = _array_prop("map")
    shop = _array_prop("shop")
    resources = _array_prop("current_resources")
    current_resources = resources


class ObsData(_Record):
    """api.h:126-129 (single_env.cpp:34-39): shared, player_data."""

    dtype = _C.ObsData
    __slots__ = ()

    def _init_fresh(self, a):
        _mask_defaults(a["player_data"]["action_mask"])

    @property
    def shared(self):
        return SharedObservation(self._a["shared"])

    @property
    def player_data(self):
        return tuple(PlayerData(self._a["player_data"][p]) for p in range(4))


class ActionData(_Record):
    """api.h:131-144 (single_env.cpp:80-85): five read-write u8 fields."""

    dtype = _C.ActionData
    __slots__ = ()

    def __init__(self, rec=None, **fields):
        super().__init__(rec)
        for k, v in fields.items():
            setattr(self, k, v)

    def _field(name):
        def get(self):
            return int(self._a[name])

        def set_(self, v):
            self._a[name] = v

        return property(get, set_)

    play = _field("play")
    play_special = _field("play_special")
    remove = _field("remove")
    move = _field("move")
    get_from_shop = _field("get_from_shop")
    del _field

    def __eq__(self, other):
        if isinstance(other, ActionData):
            other = other._a
        return all(int(self._a[k]) == int(np.asarray(other)[k]) for k in self.dtype.names)

    def __hash__(self):
        return hash(tuple(int(self._a[k]) for k in self.dtype.names))

    def as_tuple(self):
        return tuple(int(self._a[k]) for k in self.dtype.names)


class Info(_Record):
    """api.h:146-161 (numpy dtype only in the reference, common.cpp:17-19)."""

    dtype = _C.Info
    __slots__ = ()

    @property
    def total_length(self):
        return int(self._a["total_length"])

    @property
    def agent_infos(self):
        return self._a["agent_infos"]


def mask_record(mask):
    """An ActionMask record (object, structured record or (1,) array) as a (1,) structured array."""
    if isinstance(mask, _Record):
        mask = mask.record
    a = np.asarray(mask)
    if a.dtype != _C.ActionMask or a.size != 1:
        raise ValueError("expected one ActionMask record")
    return np.ascontiguousarray(a.reshape(1))


class action_sampler:
    """action_sampler(seed=42) (sampler.h:9-12, common.cpp:25-27): `sample(mask)` draws one
    uniform choice per head over the set bits of `mask` (sampler.h:14-79) and returns an
    ActionData.  The draws run on the GPU: a batch of one of the engine's sampler."""

    def __init__(self, seed=42, device=None):
        self._s = _C.VecSamplerBase(1, int(seed) & 0xFFFFFFFF, device)

    def sample(self, mask):
        self._s.sample(mask_record(mask))
        return ActionData(self._s.get_actions()[0:1].copy())

    def __repr__(self):
        return "action_sampler()"
