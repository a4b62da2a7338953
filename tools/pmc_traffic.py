"""HBM traffic per launch of the bench kernels from a tools/pmc_passes.sh capture, with the gfx950
corrections of MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reports half the bytes of wide (16 B/lane) reads, so it is doubled; WRITE_SIZE is
exact for 16-B-per-lane stores.  Writes profiles/pmc_traffic.json, stamped with the hash of the
engine source so that bench.py reports `traffic` only for the kernel version it measures.

    python tools/pmc_traffic.py gpurun_out/<tag>/pmc [envs_per_launch] [rollout steps per launch]
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pmc_summary  # noqa: E402

# kernel -> (short name, steps per launch key)
KERNELS = {"void cog::k_env_rollout<0, false>": "k_env_rollout", "void cog::k_env_step<0>": "k_env_step",
           "void cog::k_encode_lds<true>": "k_encode"}


def engine_hash():
    h = hashlib.sha256()
    for f in ("cog_engine.hip", "cog_engine.h", "cog_tables.h", "cog_rng.h"):
        with open(os.path.join(ROOT, "gym-eldorado_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def main(d, envs=65536, chunk=1000):
    tmp = os.path.join(d, "summary.json")
    pmc_summary.main(d, tmp, quiet=True)
    with open(tmp) as f:
        res = json.load(f)
    out = {"source": d, "engine_sha": engine_hash(),
           "method": "bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (gfx950 corrections), mean per dispatch"}
    for k, short in KERNELS.items():
        if k not in res or "FETCH_SIZE" not in res[k] or "WRITE_SIZE" not in res[k]:
            continue
        rd = 2.0 * res[k]["FETCH_SIZE"] * 1024
        wr = res[k]["WRITE_SIZE"] * 1024
        spl = chunk if short == "k_env_rollout" else 1
        out[short] = {"envs_per_launch": envs, "steps_per_launch": spl, "read_bytes": rd, "write_bytes": wr, "bytes_per_launch": rd + wr,
                      "dispatches": res[k]["dispatches"],
                      "l2_hit": res[k].get("TCC_HIT_sum", 0) / max(1.0, res[k].get("TCC_HIT_sum", 0) + res[k].get("TCC_MISS_sum", 0))}
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 65536, int(sys.argv[3]) if len(sys.argv) > 3 else 1000)
