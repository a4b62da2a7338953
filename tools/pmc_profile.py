"""Per-launch PMC profile of the bench kernels from tools/pmc_passes.sh captures, with the gfx950
corrections of MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reports half the bytes of wide (16 B/lane) reads, so it is doubled; WRITE_SIZE is
exact for 16-B-per-lane stores.  SQ counters are summed over the XCD instances of a dispatch;
SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles.  Writes profiles/pmc_profile.json,
stamped with the hash of the engine source so that bench.py uses it only for the kernel version
it measures.

    python tools/pmc_profile.py <dir of the K-step capture>:<K>[:<envs>] [<dir>:<K>[:<envs>] ...]  [--envs 65536]
                                [--coeff <tools/store_coeff.sh output dir> | --coeff keep]

The first capture gives the per-wave-step instruction and cycle counts (use a long K); every
capture gives the rollout's HBM bytes and L2 write hits / misses per launch at its K.  --coeff adds
the store costs of bench.py's store roofline: seconds per L2-hitting and per L2-missing scattered
16-B store, solved from tools/storeprobe's packed and spread patterns (their times and their
counter-measured hits / misses).
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pmc_summary  # noqa: E402

ROLLOUT = "void cog::k_env_rollout<0, 64"             # (prefix: <0, 64> or <0, 64, WPG>)
STEP = "void cog::k_env_step<0>"
ENCODE = "void cog::k_encode_lds<true>"


def engine_hash():
    h = hashlib.sha256()
    for f in ("cog_engine.hip", "cog_engine.h", "cog_tables.h", "cog_rng.h"):
        with open(os.path.join(ROOT, "gym-eldorado_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def summary(d):
    tmp = os.path.join(d, "summary.json")
    pmc_summary.main(d, tmp, quiet=True)
    with open(tmp) as f:
        return json.load(f)


def traffic(k):
    if "FETCH_SIZE" not in k or "WRITE_SIZE" not in k:
        return None
    return 2.0 * k["FETCH_SIZE"] * 1024 + k["WRITE_SIZE"] * 1024


def store_costs(d):
    """Seconds per scattered 16-B store that hits / misses L2, from the packed and spread launches
    of tools/storeprobe (coeff mode): t = hits x c_hit + misses x c_miss for each pattern."""
    with open(os.path.join(d, "coeff.json")) as f:
        c = json.loads(f.read().strip().splitlines()[-1])
    res = summary(os.path.join(d, "pmc"))
    pk = {k: v for k, v in res.items() if k.startswith("void k_store<1, 0, false>")}
    sp = {k: v for k, v in res.items() if k.startswith("void k_store<1, 0, true>")}
    (p,), (q,) = pk.values(), sp.values()
    tp, ts = c["packed_us"] * 1e-6, c["spread_us"] * 1e-6
    a11, a12, a21, a22 = p["TCC_HIT_sum"], p["TCC_MISS_sum"], q["TCC_HIT_sum"], q["TCC_MISS_sum"]
    det = a11 * a22 - a12 * a21
    c_hit = (tp * a22 - a12 * ts) / det
    c_miss = (a11 * ts - a21 * tp) / det
    return {"c_hit_s": c_hit, "c_miss_s": c_miss, "probe": c,
            "packed": {"hits": a11, "misses": a12}, "spread": {"hits": a21, "misses": a22},
            "note": "tools/storeprobe.hip coeff mode on MI355X: 65,536 envs of 17,216-B records, 6 scattered "
                    "16-B stores per env-step into the record tails, 200 steps; packed = lines within L2, "
                    "spread = lines beyond an XCD's 4 MiB L2; t = hits x c_hit + misses x c_miss solved "
                    "from both"}


ROLLOUT_ANY = "void cog::k_env_rollout"                 # wave, pipe and duo kernels
COMPANION = "void cog::k_env_fixup"                    # the duo's fix-up launch (same batch)


def kind_of(name):
    return "duo" if "_duo" in name else "trio" if "_trio" in name else "pipe" if "_pipe" in name else "wave"


def rollout_entry(res, envs, k):
    """The rollout kernel of one capture (the one with the most dispatches x duration is the only
    k_env_rollout* name in a capture of one shard size): counter HBM bytes, L2 writes / hits /
    misses and per-wave-step issue counts, per launch of k steps over `envs` envs."""
    names = [n for n in res if n.startswith(ROLLOUT_ANY)]
    if not names:
        return None
    name = names[0]
    r = res[name]
    waves = (envs + 63) // 64                           # stepping waves (the duo / pipe: one per 64 envs)
    per = lambda c: r[c] / waves / k if c in r else None   # noqa: E731
    e = {"kernel": name, "kind": kind_of(name), "envs": envs, "chunk": k, "dispatches": r["dispatches"],
         "bytes_per_launch": traffic(r)}
    comp = next((v for n, v in res.items() if n.startswith(COMPANION)), None)
    if comp is not None and traffic(comp) is not None:
        e["companion"] = {"kernel": COMPANION, "bytes_per_launch": traffic(comp)}
    if "TCC_WRITE_sum" in r and "TCC_HIT_sum" in r:
        e["l2_per_launch"] = {"writes": r["TCC_WRITE_sum"], "hits": r["TCC_HIT_sum"], "misses": r["TCC_MISS_sum"],
                              "fabric_write_requests": r.get("TCC_EA0_WRREQ_sum")}
    if "SQ_INSTS_VALU" in r:
        e["per_wave_step"] = {"note": "counts over every wave of the launch (stepping and storing waves) / "
                                      "(envs / 64) / steps",
                              "valu": per("SQ_INSTS_VALU"), "salu": per("SQ_INSTS_SALU"), "lds": per("SQ_INSTS_LDS"),
                              "vmem_wr": per("SQ_INSTS_VMEM_WR"), "active_inst_any": per("SQ_ACTIVE_INST_ANY"),
                              "wait_any": per("SQ_WAIT_ANY"), "wave_cycles": per("SQ_WAVE_CYCLES")}
    if e["bytes_per_launch"] is not None:
        e["bytes_per_env_step"] = e["bytes_per_launch"] / envs / k
    return e


def main(specs, envs=65536, coeff=None):
    """specs: <capture dir>:<K>[:<envs>] -- the first spec at the default envs gives the legacy
    `k_env_rollout` block (per-wave-step counts of the N=1 kernel) and the k_env_step / k_encode
    figures; every spec adds a `rollouts` entry keyed "<envs>:<K>" (the bench's roofline at any
    shard size takes the entry of its own launch shape, or none)."""
    waves = (envs + 63) // 64
    out = {"engine_sha": engine_hash(), "sources": specs,
           "method": "bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (gfx950 corrections), mean per "
                     "dispatch; per-wave-step counts = counter / waves / steps per launch"}
    ro = {"envs_per_launch": envs, "bytes_per_step_launch": {}}
    rollouts = {}
    first = True
    for spec in specs:
        parts = spec.split(":")
        d, k = parts[0], int(parts[1])
        n = int(parts[2]) if len(parts) > 2 else envs
        res = summary(d)
        e = rollout_entry(res, n, k)
        if e:
            rollouts[f"{n}:{k}"] = e
        if n != envs:
            continue
        r = next((v for kk, v in res.items() if kk.startswith(ROLLOUT)), None)
        if r:
            b = traffic(r)
            if b is not None:
                ro["bytes_per_step_launch"][str(k)] = b
            if "TCC_WRITE_sum" in r and "TCC_HIT_sum" in r:
                ro.setdefault("l2_per_launch", {})[str(k)] = {
                    "writes": r["TCC_WRITE_sum"], "hits": r["TCC_HIT_sum"], "misses": r["TCC_MISS_sum"],
                    "fabric_write_requests": r.get("TCC_EA0_WRREQ_sum")}
            if first:
                per = lambda c: r[c] / waves / k if c in r else None   # noqa: E731
                ro.update(steps_per_launch=k, valu_per_wave_step=per("SQ_INSTS_VALU"),
                          salu_per_wave_step=per("SQ_INSTS_SALU"), lds_per_wave_step=per("SQ_INSTS_LDS"),
                          vmem_wr_per_wave_step=per("SQ_INSTS_VMEM_WR"),
                          active_inst_any_per_wave_step=per("SQ_ACTIVE_INST_ANY"),
                          wait_any_per_wave_step=per("SQ_WAIT_ANY"), wait_inst_any_per_wave_step=per("SQ_WAIT_INST_ANY"),
                          wave_cycles_per_wave_step=per("SQ_WAVE_CYCLES"),
                          per_env_step=(b / envs / k) if b is not None else None,
                          l2_hit=r.get("TCC_HIT_sum", 0) / max(1.0, r.get("TCC_HIT_sum", 0) + r.get("TCC_MISS_sum", 0)),
                          gui_active=r.get("GRBM_GUI_ACTIVE"))
        if first:
            for name, short in ((STEP, "k_env_step"), (ENCODE, "k_encode")):
                kk = res.get(name)
                if kk:
                    out[short] = {"envs_per_launch": envs, "bytes_per_launch": traffic(kk),
                                  "valu_per_wave": kk.get("SQ_INSTS_VALU", 0) / max(1, kk.get("SQ_WAVES", 1)),
                                  "dispatches": kk["dispatches"]}
                    if "TCC_HIT_sum" in kk:
                        out[short]["l2_per_launch"] = {"writes": kk.get("TCC_WRITE_sum"), "hits": kk["TCC_HIT_sum"],
                                                       "misses": kk["TCC_MISS_sum"],
                                                       "fabric_write_requests": kk.get("TCC_EA0_WRREQ_sum")}
        first = False
    out["k_env_rollout"] = ro
    out["rollouts"] = rollouts
    if coeff == "keep":                     # the store costs are the probe's, not the engine's: carry them over
        with open(os.path.join(ROOT, "profiles", "pmc_profile.json")) as f:
            prev = json.load(f).get("store_costs")
        if prev:
            out["store_costs"] = prev
    elif coeff:
        out["store_costs"] = store_costs(coeff)
    with open(os.path.join(ROOT, "profiles", "pmc_profile.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    if not [x for x in a if ":" in x]:
        sys.exit(__doc__)
    envs = 65536
    if "--envs" in a:
        i = a.index("--envs")
        envs = int(a[i + 1])
        del a[i:i + 2]
    coeff = None
    if "--coeff" in a:
        i = a.index("--coeff")
        coeff = a[i + 1]
        del a[i:i + 2]
    main(a, envs, coeff)
