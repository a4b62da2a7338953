"""Per-launch PMC profile of the bench kernels from tools/pmc_passes.sh captures, with the gfx950
corrections of MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reports half the bytes of wide (16 B/lane) reads, so it is doubled; WRITE_SIZE is
exact for 16-B-per-lane stores.  SQ counters are summed over the XCD instances of a dispatch;
SQ_*_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles.  Writes profiles/pmc_profile.json,
stamped with the hash of the engine source so that bench.py uses it only for the kernel version
it measures.

    python tools/pmc_profile.py <dir of the K-step capture>:<K> [<dir>:<K> ...]  [--envs 65536]

The first capture gives the per-wave-step instruction and cycle counts (use a long K); every
capture gives the rollout's HBM bytes per launch at its K.
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pmc_summary  # noqa: E402

ROLLOUT = "void cog::k_env_rollout<0, 64>"
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


def main(specs, envs=65536):
    waves = (envs + 63) // 64
    out = {"engine_sha": engine_hash(), "sources": specs,
           "method": "bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (gfx950 corrections), mean per "
                     "dispatch; per-wave-step counts = counter / waves / steps per launch"}
    ro = {"envs_per_launch": envs, "bytes_per_step_launch": {}}
    for j, spec in enumerate(specs):
        d, k = spec.rsplit(":", 1)
        k = int(k)
        res = summary(d)
        r = res.get(ROLLOUT)
        if r:
            b = traffic(r)
            if b is not None:
                ro["bytes_per_step_launch"][str(k)] = b
            if j == 0:
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
        if j == 0:
            for name, short in ((STEP, "k_env_step"), (ENCODE, "k_encode")):
                kk = res.get(name)
                if kk:
                    out[short] = {"envs_per_launch": envs, "bytes_per_launch": traffic(kk),
                                  "valu_per_wave": kk.get("SQ_INSTS_VALU", 0) / max(1, kk.get("SQ_WAVES", 1)),
                                  "dispatches": kk["dispatches"]}
    out["k_env_rollout"] = ro
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
    main(a, envs)
