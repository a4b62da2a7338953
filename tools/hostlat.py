"""Diagnostic only: where the host time of a 20-step rollout call goes (bench's timed region).

    python tools/hostlat.py [envs] [K]

Prints medians over repeated calls of: the time rollout(K) takes to return (host launch path),
rollout + torch.cuda.synchronize() (the bench's timed region), rollout + runner.sync() (stream
sync), the device time of the launch (HIP events), and torch's own floor: a 1-element torch
kernel + torch.cuda.synchronize().
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-eldorado_amd"))
import torch  # noqa: E402

import city_of_gold as cg  # noqa: E402


def med(f, reps=30):
    v = []
    for _ in range(reps):
        v.append(f())
    return statistics.median(v) * 1e6


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    torch.cuda.set_device(0)
    env = cg.vec.get_vec_env(n)(device=0)
    smp = cg.vec.get_vec_sampler(n)(12345, device=0)
    env.reset(12345, 4, 3, cg.HARD, 100000, False)
    r = cg.vec.get_runner(n)(env, smp, None, device_views=True)
    r.set_chunk(k)
    r.rollout(5 * k)
    torch.cuda.synchronize()

    def call_only():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.rollout(k)
        t = time.perf_counter() - t0
        torch.cuda.synchronize()
        return t

    def torch_sync():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.rollout(k)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def stream_sync():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.rollout(k)
        r.sync()
        return time.perf_counter() - t0

    x = torch.zeros(1, device="cuda")

    def torch_floor():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def idle_sync():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    res = {}
    for name, f in (("rollout returns", call_only), ("rollout + torch.cuda.synchronize", torch_sync),
                    ("rollout + runner.sync", stream_sync), ("torch add_ + synchronize", torch_floor),
                    ("idle torch.cuda.synchronize", idle_sync)):
        res[name] = med(f)
    r.set_timing(True)
    r.rollout(30 * k)
    ms, launches = r.kernel_time()
    r.set_timing(False)
    res["device (HIP events per launch)"] = ms * 1e3 / max(launches, 1)
    for name, v in res.items():
        print(f"n={n} K={k}  {name:40s} {v:8.1f} us")


if __name__ == "__main__":
    main()
