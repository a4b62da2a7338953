"""C2 host loop (sampler.sample(masks); env.step(actions), 256 EASY envs) A/B: the sampler reading the
env's own mask view in HBM (default) against over PCIe ($COG_NO_HBM_MASKS, read at each call)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import city_of_gold as cg  # noqa: E402

out = {}
for rep in range(3):
    for tag in ("hbm", "pcie"):
        if tag == "pcie":
            os.environ["COG_NO_HBM_MASKS"] = "1"
        else:
            os.environ.pop("COG_NO_HBM_MASKS", None)
        r = bench.host_loop(cg, 256, cg.EASY, 0, 2000, False)
        out.setdefault(tag, []).append(round(r["ms_per_step"] * 1e3, 2))
print(json.dumps({"C2_us_per_pair": out}))
