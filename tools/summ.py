"""One-screen summary of a gpu_r03.sh output directory (bench.json, bench_driver.json)."""
import json
import os
import sys

d = sys.argv[1]


def load(name):
    try:
        with open(os.path.join(d, name)) as f:
            return json.loads(f.read().strip().splitlines()[-1])
    except Exception:
        return None


b = load("bench.json")
if b:
    r = b["roofline"]
    print("bench   %.4g env-steps/s  %.3f us/step  kernel %.3f ms/launch  frac %s" %
          (b["value"], b["ms_per_step"] * 1e3, r["kernel_ms"], r.get("frac")))
    for k in ("shard_sizes", "per_launch", "encode", "reset", "time_reset_C2", "peakmem", "full_dynamics"):
        if k in b:
            print(k, json.dumps(b[k])[:400])
    if "host_loop" in b:
        for k, v in b["host_loop"].items():
            print("host_loop", k, "%.4g" % v["value"], "%.4f ms/step" % v["ms_per_step"])
    if b.get("cpu_baseline"):
        print("cpu", b["cpu_baseline"]["value"], b["cpu_baseline"]["cores"])
b = load("bench_driver.json")
if b:
    print("driver  %.4g env-steps/s  %.3f us/step" % (b["value"], b["ms_per_step"] * 1e3))
