#!/usr/bin/env python3
"""Benchmark of the MI355X City-of-Gold engine (driver contract: one JSON line on rank 0).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--chunk C]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json metric "env-steps/sec at n_envs=65536, 4 players"; config C5): each
rank owns 65,536 independent environments (4 players, HARD, n_pieces=3, max_steps=100000,
env seeds 12345 + global index, sampler seeds the same) resident in its GPU's HBM.  One step =
the reference loop `sample(selected_action_masks); step(actions)` (benchmarks/benchmarks.py:
47-51) for every env, run by the runner's on-device loop: a persistent kernel performs C steps
per launch (default 1000), keeping each env's state on-chip between steps and storing every
step's outputs (ObsData / ActionMask / Info records, rewards, dones, agent_selection, sampled
actions, sampler state) in place in HBM -- the same bytes a one-launch-per-step run leaves
(tests/test_gpu_rollout.py).  No host round-trip.  Environments shard by index across ranks
with no collective on the data path (weak scaling); the only collectives are the timing
barrier and the max/sum of scalars.

Also reported:
  roofline      the dominant kernel (k_env_rollout): algorithmic bytes per launch from SURVEY
                8d's per-env-step table, split into its reads (419 B: needed once per launch,
                the state then stays on-chip) and its writes (381 B: every step) ->
                n x (419 + C x 381) B per launch / average launch time (HIP events on the
                runner's stream); traffic = PMC HBM bytes per launch (rocprofv3 --pmc, gfx950
                corrections) measured on this exact engine source, else null.
  per_launch    the same workload with one kernel launch per step (k_env_step<selected>):
                throughput, kernel time and its roofline at the full 800 B/env-step.
  encode        the map-observation encode kernel (k_encode, reset path): 18,432 B/env.
  cpu_baseline  the C oracle (port of the reference) on the host cores in the reference
                ThreadedRunner shape, bounded sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-eldorado_amd"))

N_ENVS_PER_GPU = 65536
SEED = 12345
N_PLAYERS, N_PIECES, MAX_STEPS = 4, 3, 100000
STEP_BYTES = 800            # algorithmic bytes per env-step ...
STEP_READ_BYTES = 419       # ... of which reads: mask 92, sampler rng 4, action 5, selected mask 92,
                            # deck 105, phase/res/shop 31, 6 neighbour features 42, scalars 48
STEP_WRITE_BYTES = 381      # ... and writes: action 5, rng 4, selected mask 92, deck 105, stored
                            # mask 92, phase/res/shop 31, scalars 48, done/agent/info 4
ENCODE_BYTES = 18432        # algorithmic bytes per encoded env (16,128 written + 2,304 read)
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "env-steps/sec at n_envs=65536, 4 players; bit-exact vs C++ ref"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--envs", type=int, default=N_ENVS_PER_GPU, help="envs per GPU")
    ap.add_argument("--chunk", type=int, default=1000, help="rollout steps per kernel launch")
    ap.add_argument("--no-per-launch", action="store_true", help="skip the one-launch-per-step line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline wall time")
    ap.add_argument("--profile-steps", type=int, default=0,
                    help="only run warmup + this many steps (for rocprofv3 captures); no JSON checks")
    return ap.parse_args()


class Dist:
    def __init__(self, gpus):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.torch = None
        self.pg = False
        if self.world > 1:
            import torch
            import torch.distributed as dist
            self.torch = torch
            if torch.cuda.is_available():
                torch.cuda.set_device(self.local)
            dist.init_process_group("gloo")      # timing barrier / max only: no data-path collective
            self.dist = dist
            self.pg = True
        else:
            try:
                import torch
                if torch.cuda.is_available():
                    self.torch = torch
            except Exception:
                self.torch = None

    def barrier_sync(self, runner):
        runner.sync()
        if self.torch is not None and self.torch.cuda.is_available():
            self.torch.cuda.synchronize()
        if self.pg:
            self.dist.barrier()

    def max(self, x):
        if not self.pg:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        if not self.pg:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.pg:
            self.dist.destroy_process_group()


def load_pmc_traffic(kernel, steps_per_launch):
    """Per-launch HBM bytes for `kernel` measured by rocprofv3 --pmc (profiles/pmc_traffic.json,
    written by tools/pmc_traffic.py); None unless measured on this exact engine source with the
    same envs and steps per launch."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from pmc_traffic import engine_hash
        with open(p) as f:
            d = json.load(f)
        e = d.get(kernel)
        if (e and e.get("envs_per_launch") == N_ENVS_PER_GPU and e.get("steps_per_launch", 1) == steps_per_launch
                and d.get("engine_sha") == engine_hash()):
            return float(e["bytes_per_launch"])
    except Exception:
        pass
    return None


def cpu_baseline(seconds):
    """C oracle in the reference runner shape on this host's cores (bounded sample)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po

    try:
        allowed = len(os.sched_getaffinity(0))
    except Exception:
        allowed = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", allowed) or allowed)
    cores = max(1, min(allowed, share) - 1)            # nproc collapses: leave one
    n = 256                                            # the reference cap; per-env cost is N-independent
    vec = po.OracleVec(n)
    smp = po.OracleSampler(n, SEED)
    vec.reset(SEED, N_PLAYERS, N_PIECES, 2, MAX_STEPS)
    best = None
    for threads in sorted({1, max(1, cores // 2), cores}):
        po.run_threaded(vec, smp, 50, threads)                     # warm-up
        probe = 400
        t = po.run_threaded(vec, smp, probe, threads)
        steps = max(probe, int(probe * (seconds / 3.0) / max(t, 1e-6)))
        t = po.run_threaded(vec, smp, steps, threads)
        rate = n * steps / t
        if best is None or rate > best[0]:
            best = (rate, threads, steps)
    rate, threads, steps = best
    return {"value": rate, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} envs (first {n} of the workload: 4p HARD seed {SEED}) x {steps} steps of "
                      f"sample(selected masks)+step, C oracle, {threads} pinned worker threads "
                      f"(best of thread counts {sorted({1, max(1, cores // 2), cores})})"}


def main():
    args = parse()
    d = Dist(args.gpus)
    import city_of_gold as cg

    n = args.envs
    base = SEED + d.rank * n                              # env i of rank r = global index r*n + i
    env = cg.vec.get_vec_env(n)(device=d.local)
    smp = cg.vec.get_vec_sampler(n)(base, device=d.local)
    t0 = time.time()
    env.reset(base, N_PLAYERS, N_PIECES, cg.HARD, MAX_STEPS, False)
    reset_s = time.time() - t0
    runner = cg.vec.get_runner(n)(env, smp, None, device_views=True)
    chunk = max(1, args.chunk)
    runner.set_chunk(chunk)

    runner.rollout(args.warmup)
    d.barrier_sync(runner)

    if args.profile_steps:                                # rocprofv3 captures: both kernels
        runner.rollout(args.profile_steps)
        d.barrier_sync(runner)
        runner.set_chunk(1)
        runner.rollout(min(args.profile_steps, 500))
        d.barrier_sync(runner)
        if d.rank == 0:
            print(json.dumps({"profile_steps": args.profile_steps, "envs": n, "chunk": chunk}))
        d.close()
        return

    # ---- timed region: exactly K steps --------------------------------------------------
    d.barrier_sync(runner)
    t0 = time.perf_counter()
    runner.rollout(args.steps)
    d.barrier_sync(runner)
    wall = time.perf_counter() - t0
    wall_max = d.max(wall)
    total_env_steps = d.sum(float(n) * args.steps)
    value = total_env_steps / wall_max

    # ---- kernel timing for the roofline: HIP events on the runner's stream bracketing one
    # batch of back-to-back launches (the per-launch average rocprofv3's kernel trace reports)
    def kernel_time(steps_per_launch, launches):
        runner.set_chunk(steps_per_launch)
        runner.set_timing(True)
        runner.rollout(steps_per_launch * launches)
        ms, steps_done = runner.kernel_time()
        runner.set_timing(False)
        return ms / 1e3 / max(steps_done, 1) * steps_per_launch       # seconds per launch

    k_chunk = min(chunk, args.steps)
    launch_s = kernel_time(k_chunk, max(1, min(args.steps, 2 * k_chunk) // k_chunk))
    alg_bytes = n * (STEP_READ_BYTES + k_chunk * STEP_WRITE_BYTES)
    achieved = alg_bytes / launch_s / 1e9
    traffic = load_pmc_traffic("k_env_rollout", k_chunk)

    per_launch = None
    if not args.no_per_launch:
        pl_steps = min(args.steps, 2000)
        d.barrier_sync(runner)
        runner.set_chunk(1)
        t1 = time.perf_counter()
        runner.rollout(pl_steps)
        d.barrier_sync(runner)
        pl_wall = d.max(time.perf_counter() - t1)
        pl_kern = kernel_time(1, pl_steps)
        pl_ach = STEP_BYTES * n / pl_kern / 1e9
        per_launch = {"kernel": "k_env_step<selected>", "value": d.sum(float(n) * pl_steps) / pl_wall,
                      "ms_per_step": pl_wall / pl_steps * 1e3, "kernel_ms": pl_kern * 1e3,
                      "roofline": {"bound": "hbm", "achieved": pl_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": pl_ach / HBM_PEAK_GBS, "traffic": load_pmc_traffic("k_env_step", 1),
                                   "algorithmic_bytes_per_launch": STEP_BYTES * n}}
    runner.set_chunk(chunk)

    enc_ms = env.time_encode(20)
    enc_gbs = ENCODE_BYTES * n / (enc_ms / 1e3) / 1e9

    # parity guard on the benchmarked state: no hazard / error in any env
    haz, _ = env.hazards()

    if d.rank == 0:
        cpu = None
        if d.world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_seconds)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": d.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (procedurally generated maps from seeds; uniform masked random actions)",
            "steps_per_launch": chunk,
            "config": {
                "workload": "C5: 65536 envs/GPU, 4 players, HARD, n_pieces=3, max_steps=100000, "
                            "on-device masked sampler over selected_action_masks + step, persistent "
                            "rollout kernel, every step's AoS outputs stored in HBM",
                "n_envs_per_gpu": n,
                "n_envs_total": n * d.world,
                "seed": SEED,
                "parallelism": f"env-sharded x{d.world}, no collectives",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_env_rollout<selected, lean> + fix-up",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel_ms": launch_s * 1e3,
                "steps_per_launch": k_chunk,
                "algorithmic_bytes_per_launch": alg_bytes,
            },
            "per_launch": per_launch,
            "encode": {
                "kernel": "k_encode",
                "ms": enc_ms,
                "achieved": enc_gbs,
                "unit": "GB/s",
                "frac": enc_gbs / HBM_PEAK_GBS,
                "algorithmic_bytes_per_launch": ENCODE_BYTES * n,
            },
            "reset_s": reset_s,
            "hazards_or": int(haz),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    d.close()


if __name__ == "__main__":
    main()
