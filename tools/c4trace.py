"""Diagnostic: the C4 shard's host loop (runner.sample(); runner.step_sync(), 8,192 envs, host
views) for a rocprofv3 kernel trace: which kernels run per step and how long each takes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-eldorado_amd"))
import city_of_gold as cg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
env = cg.vec.get_vec_env(n)()
smp = cg.vec.get_vec_sampler(n)(12345)
env.reset(12345, 4, 3, cg.HARD, 100000, False)
runner = cg.vec.get_runner(n)(env, smp, None)
env.observations                                          # host views live
for _ in range(200):
    runner.sample()
    runner.step_sync()
print("ok", n)
