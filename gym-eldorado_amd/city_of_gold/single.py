"""`city_of_gold.cog_env`: the reference's single-environment binding (src/pybind/single_env.cpp:
12-32 over include/environment.h:47-76) on the same HIP engine, as a batch of one.

Differences from the vec env it is built on, all from the reference's cog_env:
  - no auto-reset: a finished episode stays done and later steps are dead steps
    (environment.cpp:91-95) until reset();
  - reset() without arguments keeps the parameters and continues the rng stream
    (environment.cpp:42-63);
  - init(observations, info, rewards, selected_action_masks) binds the caller's records, which
    every reset/step then updates (environment.cpp:25-40).

Additive: init() is optional (the env's own record views are then used: `observations`,
`infos`, `rewards`, `selected_action_masks`), step() takes an ActionData record or a 5-tuple,
and get_map() returns the (48, 48, 7) map observation.  Like the reference, everything runs
synchronously on the calling thread.  The reference's Python cannot create the records init()
needs (ObsData and ActionMask have no py::init), so this class is the usable form of that API.
"""
from __future__ import annotations

import numpy as np

from . import _city_of_gold as _C
from .records import Info, _Record

DEFAULTS = dict(n_players=4, n_pieces=3, difficulty=_C.Difficulty.EASY, max_steps=100000, render=False)


class cog_env:
    def __init__(self, seed=None, n_players=4, n_pieces=3, difficulty=_C.Difficulty.EASY,
                 max_steps=100000, render=False, device=None):
        self._v = _C.VecEnvBase(1, device)
        self._v.set_autoreset(False)
        if seed is None:
            seed = int(np.random.SeedSequence().entropy) & 0xFFFFFFFF   # std::random_device
        self._params = (int(seed) & 0xFFFFFFFF, int(n_players), int(n_pieces), _C.Difficulty(int(difficulty)),
                        int(max_steps), bool(render))
        self._bound = None
        self._reset_done = False
        self._done = False

    # ---- environment.h:50-56 -----------------------------------------------------------------
    def init(self, observations, info, rewards, selected_action_masks):
        def rec(a, dtype, what):
            if isinstance(a, _Record):
                a = a.record
            a = np.asarray(a)
            if a.dtype != dtype or a.size != 1:
                raise ValueError(f"{what}: expected one {dtype} record")
            return a.reshape(1)
        rw = np.asarray(rewards)
        if rw.dtype != np.float32 or rw.size != 4:
            raise ValueError("rewards: expected 4 float32")
        self._bound = (rec(observations, _C.ObsData, "observations"), rec(info, _C.Info, "info"),
                       rw.reshape(4), rec(selected_action_masks, _C.ActionMask, "selected_action_masks"))
        if self._reset_done:
            self._publish()

    def reset(self, *args):
        if args:
            if len(args) != 6:
                raise TypeError("reset() takes no arguments or (seed, n_players, n_pieces, difficulty, max_steps, render)")
            seed, n_players, n_pieces, difficulty, max_steps, render = args
            self._params = (int(seed) & 0xFFFFFFFF, int(n_players), int(n_pieces), _C.Difficulty(int(difficulty)),
                            int(max_steps), bool(render))
            self._v.reset(*self._params)
        elif not self._reset_done:
            self._v.reset(*self._params)      # first reset: the constructor's parameters and seed
        else:
            self._v.reset()                   # keep the parameters, continue the rng stream
        self._reset_done = True
        self._done = False                    # reset() clears done (environment.cpp:54)
        self._publish()

    def step(self, action):
        a = np.zeros(1, dtype=_C.ActionData)
        if isinstance(action, _Record):
            action = action.record
        if isinstance(action, np.ndarray) or isinstance(action, np.void):
            src = np.asarray(action).reshape(-1)
            if src.dtype != _C.ActionData or src.size != 1:
                raise ValueError("action: expected one ActionData record")
            a[:] = src
        else:
            play, play_special, remove, move, get_from_shop = action
            a["play"], a["play_special"], a["remove"], a["move"], a["get_from_shop"] = \
                play, play_special, remove, move, get_from_shop
        self._v.step(a)
        self._done = bool(self._v.dones[0])  # without auto-reset dones[0] is the env's done flag
        self._publish()

    def render(self):
        if self._params[5]:
            print("game over" if self.get_done() else self._describe())
        else:
            print("You are calling render method without specifying any render mode.")

    # ---- accessors (environment.h:58-76, single_env.cpp:17-32) ---------------------------------
    @property
    def agent_selection(self):
        return int(self._v.agent_selection[0])

    def get_seed(self):
        return self._params[0]

    def get_n_players(self):
        return self._params[1]

    def get_n_pieces(self):
        return self._params[2]

    def get_difficulty(self):
        return self._params[3]

    def get_max_steps(self):
        return self._params[4]

    def get_render(self):
        return self._params[5]

    def get_done(self):
        return self._done

    def get_info(self):
        return Info(self._v.infos[0:1].copy())

    def get_map(self):
        return self._v.observations[0]["shared"]["map"]

    @property
    def observations(self):
        return self._v.observations[0]

    @property
    def infos(self):
        return self._v.infos[0]

    @property
    def rewards(self):
        return self._v.rewards[0]

    @property
    def selected_action_masks(self):
        return self._v.selected_action_masks[0]

    def hazards(self):
        return self._v.hazards()

    # ---- internals ---------------------------------------------------------------------------
    def _publish(self):
        if self._bound is None:
            return
        obs, info, rew, sel = self._bound
        obs[...] = self._v.observations
        info[...] = self._v.infos
        rew[...] = self._v.rewards[0]
        sel[...] = self._v.selected_action_masks

    def _describe(self):
        o = self._v.observations[0]
        ag = self.agent_selection
        deck = o["player_data"][ag]["obs"]
        return (f"currently playing: {ag}\nphase: {int(o['shared']['phase'])}  resources: "
                f"{o['shared']['current_resources'].tolist()}\nshop: {o['shared']['shop'].tolist()}\n"
                f"draw {deck['draw'].tolist()}\nhand {deck['hand'].tolist()}\n"
                f"active {deck['active'].tolist()}\nplayed {deck['played'].tolist()}\n"
                f"discard {deck['discard'].tolist()}")
