"""C2 host loop (sampler.sample(masks); env.step(actions), 256 EASY envs) A/B: the sampler reading the
env's own mask view in HBM (default) against over PCIe ($COG_NO_HBM_MASKS, read at each call); and
the pair's latency split (sample() alone, step() alone, in loops of their own)."""
import json
import os
import sys
import time

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
os.environ.pop("COG_NO_HBM_MASKS", None)
n = 256
env = cg.vec.get_vec_env(n)(device=0)
smp = cg.vec.get_vec_sampler(n)(bench.SEED, device=0)
env.reset(bench.SEED, bench.N_PLAYERS, bench.N_PIECES, cg.EASY, bench.MAX_STEPS, False)
masks, acts = env.selected_action_masks, smp.get_actions()
split = {}
for name, fn in (("sample", lambda: smp.sample(masks)), ("step", lambda: env.step(acts)),
                 ("pair", lambda: (smp.sample(masks), env.step(acts)))):
    for _ in range(50):
        fn()
    t0 = time.perf_counter()
    for _ in range(2000):
        fn()
    split[name] = round((time.perf_counter() - t0) / 2000 * 1e6, 2)
print(json.dumps({"C2_us_per_pair": out, "split_us": split}))
