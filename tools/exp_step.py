"""Per-launch step kernel (k_env_step<selected>, the runner's chunk-1 path): device us per launch
(HIP events over 500 back-to-back launches) at the given env counts."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-eldorado_amd"))
import city_of_gold as cg  # noqa: E402

for n in [int(x) for x in sys.argv[1].split(",")]:
    env = cg.vec.get_vec_env(n)(device=0)
    smp = cg.vec.get_vec_sampler(n)(12345, device=0)
    env.reset(12345, 4, 3, cg.HARD, 100000, False)
    r = cg.vec.get_runner(n)(env, smp, None, device_views=True)
    r.set_chunk(1)
    r.rollout(100)
    r.sync()
    r.set_timing(True)
    r.rollout(500)
    ms, done = r.kernel_time()
    r.set_timing(False)
    print(f"k_env_step n={n:6d}  {ms * 1e3 / max(done, 1):7.2f} us/launch", flush=True)
    del r, smp, env
