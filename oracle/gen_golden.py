"""Generate tests/golden/ fixtures from the reference core compiled in this container
(oracle/_ref/libref.so = unmodified /root/reference/src/*.cpp + include/*.h + ref_harness.cpp).

TEST INFRASTRUCTURE ONLY; needs /root/reference (dev container), never runs on the GPU box.

Every run is first screened with the C oracle: the reference built against the image's
libstdc++ 11 aborts where map generation erases past the end of valid_indices (map.cpp:727,
needs GCC>=13) or where 2/3-player B-start maps overflow player_locations (map.cpp:347-352).
Reference runs stop one step before the first such hazard.  While generating, the oracle is
compared with the reference at every step (any disagreement aborts generation).

Digest per step (8 bytes): SHA-256 prefix over the named leaf fields (padding excluded) of
observations, selected_action_masks, rewards, dones, agent_selection, infos, actions
(SURVEY App. B.3), for ONE env.  Batch runs are compared env by env (envs are independent:
env i of a batch == a 1-env batch seeded seed+i, sampler seeded sseed+i).

    python oracle/gen_golden.py            # writes tests/golden/*.npz and *.json
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import pyoracle as po  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def digest_env(e, actions):
    return po.step_digest(e.observations, e.selected_action_masks, e.rewards, e.dones,
                          e.agent_selection, e.infos, actions)


def masks_of(e, mode):
    return e.selected_action_masks if mode == "sel" else po.stored_masks(e)


def screen(seed, np_, npc, diff, max_steps, sseed, mode, steps):
    """Number of steps the reference can run safely (-1: not even the reset)."""
    o = po.OracleVec(1)
    s = po.OracleSampler(1, sseed)
    try:
        o.reset(seed, np_, npc, diff, max_steps)
    except RuntimeError:
        return -1
    if o.flags(0) & po.REF_UNSAFE:
        return -1
    for t in range(steps):
        s.sample(masks_of(o, mode))
        o.step(s.actions)
        if o.flags(0) & po.REF_UNSAFE:
            return t
    return steps


def ref_trace(seed, np_, npc, diff, max_steps, sseed, mode, steps):
    """Reference digests for t = 0..steps (t=0 right after reset), oracle-checked."""
    r, rs = po.RefVec1(), po.RefSampler1(sseed)
    o, os_ = po.OracleVec(1), po.OracleSampler(1, sseed)
    r.reset(seed, np_, npc, diff, max_steps)
    o.reset(seed, np_, npc, diff, max_steps)
    out = [digest_env(r, rs.actions)]
    resets = 0
    for t in range(steps):
        rs.sample(masks_of(r, mode))
        os_.sample(masks_of(o, mode))
        r.step(rs.actions)
        o.step(os_.actions)
        resets += int(r.dones[0])
        d = digest_env(r, rs.actions)
        if d != digest_env(o, os_.actions):
            raise SystemExit(f"oracle != reference: seed={seed} diff={diff} mode={mode} step={t}")
        out.append(d)
    return out, resets


def traces():
    sets = []
    # name, seed, n_players, n_pieces, difficulty, max_steps, sampler seed, mode, steps, n_envs
    specs = [
        ("C2shape_sel_medium", 12345, 4, 3, 1, 100000, 12345, "sel", 1000, 16),
        ("C3shape_sel_hard", 12345, 4, 3, 2, 100000, 12345, "sel", 1000, 16),
        ("stored_hard_ms30", 7, 4, 3, 2, 30, 7, "sto", 1500, 16),
        ("stored_medium_ms40_bstart", 70000, 4, 3, 1, 40, 70000, "sto", 1500, 16),
        ("c1like_2p_medium_sel", 0, 2, 3, 1, 100000, 0, "sel", 20000, 1),
        ("c1like_2p_medium_sto", 0, 2, 3, 1, 100000, 0, "sto", 5000, 1),
        ("p3_hard_sto_ms60", 300, 3, 3, 2, 60, 300, "sto", 1500, 8),
    ]
    for name, seed, np_, npc, diff, ms, sseed, mode, steps, n in specs:
        envs = []
        i = 0
        while len(envs) < n and i < 64 * n:
            L = screen(seed + i, np_, npc, diff, ms, sseed + i, mode, steps)
            if L > 0:
                dig, resets = ref_trace(seed + i, np_, npc, diff, ms, sseed + i, mode, L)
                envs.append(dict(index=i, steps=L, resets=resets,
                                 digests=np.frombuffer(b"".join(dig), dtype=np.uint8).reshape(-1, 8)))
            i += 1
        tot = sum(e["steps"] for e in envs)
        print(f"{name}: {len(envs)} envs, {tot} reference steps, {sum(e['resets'] for e in envs)} resets")
        sets.append(dict(name=name, seed=seed, n_players=np_, n_pieces=npc, difficulty=diff, max_steps=ms,
                         sampler_seed=sseed, mode=mode, envs=envs))
    return sets


def maps():
    """Reset-only digests for every hazard-free seed of the survey's map sets."""
    out = []
    for diff in (0, 1, 2):
        for npc in ((1, 3) if diff == 0 else (3, 5)):
            for lo in (0, 4096, 63744, 70000):
                for s in range(lo, lo + 256):
                    if screen(s, 4, npc, diff, 100000, s, "sel", 0) < 0:
                        continue
                    r = po.RefVec1()
                    r.reset(s, 4, npc, diff, 100000)
                    o = po.OracleVec(1)
                    o.reset(s, 4, npc, diff, 100000)
                    zero = np.zeros(1, dtype=po.ACTION)
                    d = digest_env(r, zero)
                    if d != digest_env(o, zero):
                        raise SystemExit(f"map mismatch seed={s} diff={diff} npc={npc}")
                    out.append((diff, npc, s, d.hex()))
    print(f"maps: {len(out)} hazard-free reference maps")
    return out


def sampler_kat():
    rng = np.random.default_rng(2024)
    n = 256
    masks = np.zeros((3, n), dtype=po.MASK)
    raw = masks.view(np.uint8).reshape(3, n, 128)
    raw[:, :, :92] = rng.random((3, n, 92)) < 0.35
    raw[:, :5, :] = 0
    acts = np.zeros((3, n), dtype=po.ACTION)
    for i in range(n):
        rs = po.RefSampler1(99 + i)
        for k in range(3):
            rs.sample(masks[k, i:i + 1])
            acts[k, i] = rs.actions[0]
    return masks, acts


# Whole workloads pinned by the reference: final-state digests of every env the reference can run
# (name, n_envs, n_players, n_pieces, difficulty, seed, steps).  c5: bench.py's timed workload
# (65,536 envs, seeds 12345 + i, sampler seeds the same; 5 warm-up + 1,200 steps, the length
# tests/test_gpu_timed_workloads.py drives); c3: BASELINE config C3 at its own size.
WORKLOADS = [("c5", 65536, 4, 3, 2, 12345, 1205), ("c3", 8192, 4, 3, 1, 12345, 1000)]


def _ref_final_digests(job):
    """Worker: the reference's own loop (ref_run_selected) for each listed env, digest at the end."""
    seed0, idx, np_, npc, diff, steps = job
    out = np.zeros((len(idx), 8), dtype=np.uint8)
    for k, i in enumerate(idx):
        r, s = po.RefVec1(), po.RefSampler1(seed0 + int(i))
        r.reset(seed0 + int(i), np_, npc, diff, 100000)
        r.run_selected(s, steps)
        out[k] = np.frombuffer(digest_env(r, s.actions), dtype=np.uint8)
    return out


def workloads():
    """Per workload: the oracle runs the whole batch (threaded) to find the envs the reference can
    run (hazard flags), the reference runs each of those from its seed, and both final states'
    digests must agree env by env (any difference aborts)."""
    from multiprocessing import Pool
    arrays, meta = {}, []
    for name, n, np_, npc, diff, seed, steps in WORKLOADS:
        o, s = po.OracleVec(n), po.OracleSampler(n, seed)
        o.reset_threaded(seed, np_, npc, diff, 100000)
        po.run_threaded(o, s, steps, po.host_threads())
        flags = o.flags()
        safe = (flags & po.REF_UNSAFE) == 0
        idx = np.nonzero(safe)[0].astype(np.uint32)
        odig = po.batch_digest(o.observations[idx], o.selected_action_masks[idx], o.rewards[idx], o.dones[idx],
                               o.agent_selection[idx], o.infos[idx], s.actions[idx])
        del o, s
        jobs = [(seed, part, np_, npc, diff, steps) for part in np.array_split(idx, 64)]
        with Pool(max(1, (os.cpu_count() or 2) - 1)) as pool:
            rdig = np.concatenate(pool.map(_ref_final_digests, jobs))
        bad = np.nonzero((rdig != odig).any(1))[0]
        if bad.size:
            raise SystemExit(f"{name}: oracle != reference at env {int(idx[bad[0]])} after {steps} steps")
        arrays[f"{name}_safe"] = np.packbits(safe)
        arrays[f"{name}_digests"] = rdig
        meta.append(dict(name=name, n_envs=n, n_players=np_, n_pieces=npc, difficulty=diff, seed=seed,
                         sampler_seed=seed, steps=steps, mode="sel", ref_envs=int(idx.size),
                         oracle_only_envs=int(n - idx.size)))
        print(f"{name}: {idx.size} of {n} envs pinned by the reference after {steps} steps "
              f"({n - idx.size} hazard envs: oracle only)")
    np.savez(os.path.join(OUT, "ref_workloads.npz"), **arrays)
    with open(os.path.join(OUT, "ref_workloads.json"), "w") as f:
        json.dump(dict(source="oracle/_ref (unmodified reference core) via oracle/gen_golden.py --workloads",
                       digest="sha256[:8] per env over named leaves of obs, sel, rewards, dones, agent_sel, "
                              "infos, actions after `steps` x (sample(selected masks); step) from reset",
                       arrays="<name>_safe: packbits of the envs the reference ran; <name>_digests: "
                              "uint8[ref_envs, 8] in env order",
                       workloads=meta), f, indent=0)


def main():
    assert po.ref_available(), "build the reference first: make -C oracle ref"
    os.makedirs(OUT, exist_ok=True)
    if "--workloads" in sys.argv:
        workloads()
        return
    t = traces()
    arrays = {}
    for st in t:
        for k, e in enumerate(st["envs"]):
            arrays[f"{st['name']}__{k}"] = e.pop("digests")
    np.savez(os.path.join(OUT, "ref_trace_digests.npz"), **arrays)
    with open(os.path.join(OUT, "ref_traces.json"), "w") as f:
        json.dump(dict(source="oracle/_ref (unmodified reference core) via oracle/gen_golden.py",
                       digest="sha256[:8] over named leaves of obs, sel, rewards, dones, agent_sel, infos, actions",
                       digests_file="ref_trace_digests.npz (key <set>__<k>, uint8[steps+1, 8])",
                       sets=t), f, indent=0)
    m = maps()
    with open(os.path.join(OUT, "ref_maps.json"), "w") as f:
        json.dump(dict(source="oracle/_ref via oracle/gen_golden.py", entries=m), f)
    masks, acts = sampler_kat()
    np.savez_compressed(os.path.join(OUT, "ref_sampler_kat.npz"), masks=masks.view(np.uint8),
                        actions=acts.view(np.uint8), seed=np.array([99]))
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
