"""profiles/stamps_profile.json from tools/duoprobe (built with -DCOG_STAMPS) runs with PROBE_JSON=1:
the trio stepping wave's s_memtime ticks per step, split into its own work (busy) and its waits on
the other waves' progress counters, per shard size, stamped with the engine source hash so that
bench.py attaches it (roofline.limiter) only to the engine it measured.

    python tools/stamps_profile.py <duoprobe output file> [...] > profiles/stamps_profile.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pmc_profile import engine_hash  # noqa: E402

shapes = {}
for path in sys.argv[1:]:
    for line in open(path):
        if line.startswith("STAMPS_JSON "):
            d = json.loads(line[len("STAMPS_JSON "):])
            shapes[str(d["envs"])] = d
print(json.dumps({"engine_sha": engine_hash(), "shapes": shapes,
                  "note": "trio stepping wave, median over waves, ticks per step (s_memtime) of a "
                          "-DCOG_STAMPS build of this engine source in launches of steps_per_launch steps; "
                          "busy = its own work, wait = its progress-counter waits"}, indent=1))
