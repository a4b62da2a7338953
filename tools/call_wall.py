"""Wall time of the driver's call shape -- runner.rollout(20); torch.cuda.synchronize() -- median and
min over 200 calls, per shard size; run once with $COG_NO_GRAPH set and once without (graph A/B)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import city_of_gold as cg  # noqa: E402
import torch  # noqa: E402

out = {"graph": os.environ.get("COG_NO_GRAPH") is None}
for n in (8192, 65536):
    env, smp, runner = bench.make(cg, n, bench.SEED, 0)
    runner.set_chunk(20)
    runner.rollout(100)
    torch.cuda.synchronize(0)
    v = []
    for _ in range(200):
        t0 = time.perf_counter()
        runner.rollout(20)
        torch.cuda.synchronize(0)
        v.append(time.perf_counter() - t0)
    sub = []
    for _ in range(50):                                   # host submission alone
        t0 = time.perf_counter()
        runner.rollout(20)
        sub.append(time.perf_counter() - t0)
        torch.cuda.synchronize(0)
    runner.sync()
    out[n] = {"median_us": round(statistics.median(v) * 1e6, 1), "min_us": round(min(v) * 1e6, 1),
              "submit_median_us": round(statistics.median(sub) * 1e6, 1)}
    del runner, smp, env
print(json.dumps(out))
