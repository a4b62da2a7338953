#!/usr/bin/env python3
"""Benchmark of the MI355X City-of-Gold engine (driver contract: one JSON line on rank 0).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--chunk C]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Headline workload (BASELINE.json metric "env-steps/sec at n_envs=65536, 4 players"; configs
C4/C5): 65,536 environments IN TOTAL, split by index across the N ranks (8,192 per GPU at N=8:
strong scaling), 4 players, HARD, n_pieces=3, max_steps=100000, env seeds 12345 + global index,
sampler seeds the same, everything resident in HBM.  One step = the reference loop
`sample(selected_action_masks); step(actions)` (benchmarks/benchmarks.py:47-51) for every env,
run by the runner's on-device loop: one persistent kernel performs min(C, K) steps per launch,
keeping each env's state on-chip between steps and storing every step's outputs (ObsData /
ActionMask / Info records, rewards, dones, agent_selection, sampled actions) in place in HBM --
the bytes a one-launch-per-step run leaves (tests/test_gpu_rollout.py).  No host round-trip
(C5).  No collective on the data path; the only collectives are the timing barrier and the
max/sum of scalars (gloo).

Also reported (rank 0; the extra lines only at N=1, so a scaling run stays short):
  roofline       the dominant kernel (the trio rollout) against HBM by the bytes it moves (PMC
                 counters of the same launch shape: FETCH x 2 + WRITE, gfx950 corrections), the
                 limiter that applies (the stepping wave's instruction stream, busy fraction from
                 phase stamps), SURVEY 8d's 800 B/env-step as a labelled equivalent, round 3's L2
                 store model as a record and `valu_issue` the VALU rate against the SIMDs' peak.
  shard_sizes    rollout us/step at the N=1 batch (65,536 on one GPU) and the N=8 shard (8,192)
  per_launch     one kernel launch per step (k_env_step<selected>)
  host_loop      the reference's numpy loop through the host API at C2 (256, EASY) and the C4
                 shard (8,192, HARD, runner.sample(); runner.step_sync()), D2H bytes per step
  full_dynamics  stored-mask driver (moves, shop, specials), max_steps 30: auto-resets with
                 device map generation inside the rollout; full_dynamics_steady the same driver
                 with max_steps 100,000 (no constant resets), 1,000-step launches
  reset, sample  time_reset / time_sample equivalents (benchmarks/benchmarks.py:53-69); reset()
                 without arguments beside reset(seed, ...); time_reset_C2 the asv shape (256 EASY)
  peakmem        asv peakmem_runner: device and host bytes of a runner with host views
  asv_grid       asv time_run / time_sample (benchmarks.py:47-57) at N in {1, 8, 64, 256, 8192} x
                 {sequential, async, sync}, 10,000 steps each, EASY; the N where each mode passes
                 cpu_baseline
  encode         the map-observation encode kernel (reset path), 18,432 B/env, beside a measured
                 device copy peak
  cpu_baseline   the C oracle (port of the reference) on the host cores in the reference
                 ThreadedRunner shape, bounded sample (rank 0, N=1 only)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-eldorado_amd"))

N_ENVS_TOTAL = 65536
N_SHARD8 = N_ENVS_TOTAL // 8
SEED = 12345
N_PLAYERS, N_PIECES, MAX_STEPS = 4, 3, 100000
STEP_BYTES = 800            # algorithmic bytes per env-step of sample + step
WRITEBACK_BYTES = 1234      # D2H / write-back bytes per env-step (C4)
ENCODE_BYTES = 18432        # per encoded env (16,128 written + 2,304 read)
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
N_SIMD, CLOCK_HZ, VALU_CYC = 1024, 2.4e9, 2.0   # 256 CUs x 4 SIMD-32; wave64 VALU = 2 cycles
N_CU = 256                  # the trio's one-workgroup-per-CU (LAT) form up to N_CU workgroups of 64 envs
METRIC = "env-steps/sec at n_envs=65536, 4 players; bit-exact vs C++ ref"
HAZ_ERASE_PAST = 0x02       # map.cpp:727 erase past the end: GCC>=13 libstdc++ semantics (oracle-pinned)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--envs-total", type=int, default=N_ENVS_TOTAL, help="envs over all ranks")
    ap.add_argument("--chunk", type=int, default=1000, help="rollout steps per kernel launch")
    ap.add_argument("--no-extras", action="store_true", help="headline + roofline only")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-asv", action="store_true", help="skip the asv time_run / time_sample grid extra")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline wall time")
    ap.add_argument("--profile-steps", type=int, default=0,
                    help="only run warmup + this many rollout steps (rocprofv3 captures); no JSON checks")
    return ap.parse_args()


class Dist:
    def __init__(self, gpus):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.torch = None
        self.pg = False
        self.device = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            self.torch = torch
            dist.init_process_group("gloo")      # timing barrier / max only: no data-path collective
            self.dist = dist
            self.pg = True
        else:
            try:
                import torch
                self.torch = torch
            except Exception:
                self.torch = None

    def sync(self, runner):
        """torch.cuda.synchronize() of THIS rank's GPU (every stream of it, the engine's included)."""
        t = self.torch
        if t is not None and t.cuda.is_available():
            t.cuda.synchronize(self.device)
        else:
            runner.sync()

    def barrier(self):
        if self.pg:
            self.dist.barrier()

    def barrier_sync(self, runner, check=True):
        """sync(), the runner's error check (check=False: left to the caller) and the barrier."""
        self.sync(runner)
        if check:
            runner.sync()
        self.barrier()

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


def device_of(d):
    """This rank's GPU: LOCAL_RANK, unless COG_DEVICE pins it (several ranks on one GPU) -- the
    order the library's default device follows (pybind_module.cpp default_devices)."""
    v = os.environ.get("COG_DEVICE")
    return int(v) if v else d.local


def bind_device(d, dev):
    """Make `dev` torch's current device, so that synchronize() and the timing events of this
    rank cover the GPU its engine runs on (not GPU 0)."""
    d.device = dev
    t = d.torch
    if t is not None and t.cuda.is_available():
        t.cuda.set_device(dev)


def load_profile():
    """profiles/pmc_profile.json (tools/pmc_profile.py) when it was measured on this exact engine
    source; else None."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from pmc_profile import engine_hash
        with open(os.path.join(ROOT, "profiles", "pmc_profile.json")) as f:
            p = json.load(f)
        return p if p.get("engine_sha") == engine_hash() else None
    except Exception:
        return None


def make(cg, n, seed, device, difficulty=None, max_steps=MAX_STEPS, device_views=True, stored=False, first=0):
    """The batch of global envs [first, first + n) of a run seeded `seed`: env i reset with
    (u32)(seed + first + i) (vec_environment.h:41), sampler i seeded seed + first + i unwrapped
    (vec_sampler.h:9-13), so that a rank's shard equals the same envs of one unsharded batch."""
    from city_of_gold.shard import shard_seed
    env = cg.vec.get_vec_env(n)(device=device)
    smp = cg.vec.get_vec_sampler(n)(seed, device=device, first_index=first)
    env.reset(shard_seed(seed, first), N_PLAYERS, N_PIECES, cg.HARD if difficulty is None else difficulty,
              max_steps, False)
    runner = cg.vec.get_runner(n)(env, smp, None, device_views=device_views, stored_masks=stored)
    return env, smp, runner


def kernel_time(runner, steps_per_launch, launches):
    """Seconds per launch: HIP events on the runner's stream around `launches` back-to-back
    launches of `steps_per_launch` steps (the per-launch average rocprofv3's kernel trace gives)."""
    runner.set_chunk(steps_per_launch)
    runner.set_timing(True)
    runner.rollout(steps_per_launch * launches)
    ms, steps_done = runner.kernel_time()
    runner.set_timing(False)
    return ms / 1e3 / max(steps_done, 1) * steps_per_launch


def us_per_step(cg, n, device, steps=1000):
    env, smp, runner = make(cg, n, SEED, device)
    runner.set_chunk(steps)
    runner.rollout(200)
    runner.sync()
    t = kernel_time(runner, steps, 2)
    del runner, smp, env
    return t / steps * 1e6


def host_loop(cg, n, difficulty, device, steps, use_runner):
    """The reference's loop through the host API with numpy views every step."""
    env = cg.vec.get_vec_env(n)(device=device)
    smp = cg.vec.get_vec_sampler(n)(SEED, device=device)
    env.reset(SEED, N_PLAYERS, N_PIECES, difficulty, MAX_STEPS, False)
    masks, acts = env.selected_action_masks, smp.get_actions()
    runner = cg.vec.get_runner(n)(env, smp, None) if use_runner else None

    def one():
        if runner is not None:
            runner.sample()
            runner.step_sync()
        else:
            smp.sample(masks)
            env.step(acts)
    for _ in range(20):
        one()
    s0, h0 = smp.spec_stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    wall = time.perf_counter() - t0
    s1, h1 = smp.spec_stats()
    split = None
    if runner is None:                                    # the two calls timed apart (per call, mean)
        ts = tt = 0.0
        for _ in range(steps):
            a = time.perf_counter()
            smp.sample(masks)
            b = time.perf_counter()
            env.step(acts)
            ts += b - a
            tt += time.perf_counter() - b
        split = {"sample_us": ts / steps * 1e6, "step_us": tt / steps * 1e6,
                 "speculative_samples": (h1 - h0) / max(1, s1 - s0),
                 "note": "sample(): the speculative sample the step before computed (a host copy) when "
                         "speculative_samples = 1; step(): one k_env_step_pub launch (the step, its "
                         "publish into the pinned views, the next sample) + its completion word"}
    # bytes of host-visible records refreshed per env-step: ObsData tail (1,088) + selected mask,
    # info, rewards, done, agent (338) + actions (64).  An upper bound of what crosses PCIe:
    # k_publish stores only the 16-B granules that changed since the last refresh, and the
    # sampler reads the env's pinned mask view in place
    d2h = 1088 + 128 + 192 + 16 + 2 + 64
    h2d = 0 if use_runner else 64 + 128
    return {"value": n * steps / wall, "unit": "env-steps/s", "ms_per_step": wall / steps * 1e3,
            "envs": n, "steps": steps, "d2h_bytes_per_env_step": d2h, "h2d_bytes_per_env_step": h2d,
            "survey_8d_writeback_bytes": WRITEBACK_BYTES,
            "view_refresh_GBs_nominal": n * (d2h + h2d) * steps / wall / 1e9,
            "note": "d2h/h2d bytes are the records refreshed per env-step (upper bound): k_publish "
                    "moves only the changed 16-B granules over PCIe",
            "loop": "runner.sample(); runner.step_sync()" if use_runner else "sampler.sample(masks); env.step(actions)",
            "split": split}


def time_reset_c2(cg, dev, calls=100):
    """asv time_reset at the reference's own shape (benchmarks.py:58-62): a 256-env EASY batch,
    `envs.reset()` without arguments, sequential mode, numpy views live."""
    n = 256
    env = cg.vec.get_vec_env(n)(device=dev)
    env.reset(SEED, N_PLAYERS, N_PIECES, cg.EASY, MAX_STEPS, False)
    env.observations                                      # host views live, as in the reference
    env.reset()
    t1 = time.perf_counter()
    for _ in range(calls):
        env.reset()
    s = (time.perf_counter() - t1) / calls
    del env
    return {"envs": n, "calls": calls, "ms_per_call": s * 1e3, "resets_per_s": n / s,
            "note": "vec_cog_env_256.reset() x calls (asv TimeEnvs.time_reset, sequential)"}


ASV_NS = (1, 8, 64, 256, 8192)
ASV_MODES = ("sequential", "async", "sync")
ASV_STEPS = 10000                  # benchmarks.py:5 N_STEPS


def asv_setup(cg, n, mode, dev):
    """TimeEnvs.setup (benchmarks/benchmarks.py:16-45) for (n, seed 12345, mode): the sample / step /
    end / sync callables of one mode, EASY maps, 4 players, 3 pieces.  The GPU runner has no thread
    count (its work runs on the device's stream), so `threads` is 1 throughout."""
    env = cg.vec.get_vec_env(n)(device=dev)
    env.reset(SEED, N_PLAYERS, N_PIECES, cg.EASY, MAX_STEPS, False)
    smp = cg.vec.get_vec_sampler(n)(SEED, device=dev)
    acts, am = smp.get_actions(), env.selected_action_masks
    if mode == "sequential":
        return (env, smp), (lambda: smp.sample(am)), (lambda: env.step(acts)), (lambda: None), (lambda: None)
    runner = cg.vec.get_runner(n)(env, smp, 1)
    if mode == "sync":
        return (env, smp, runner), runner.sample, runner.step_sync, (lambda: None), runner.sync
    return (env, smp, runner), runner.sample, runner.step, runner.sync, (lambda: None)


def asv_grid(cg, dev, cpu_value=None, steps=ASV_STEPS):
    """asv TimeEnvs.time_run and time_sample (benchmarks/benchmarks.py:47-57) over N in ASV_NS and
    the three modes, exactly as the reference defines them: sequential = sampler.sample(masks);
    env.step(actions) per step; async = runner.sample(); runner.step() per step, one runner.sync()
    at the end; sync = runner.sample(); runner.step_sync() per step.  time_sample: the sample call
    (+ sync() in sync mode) per step.  env-steps/s = N x steps / wall.  `crossover`: per mode, the
    smallest N of the grid whose time_run rate passes the CPU baseline (cpu_value, env-steps/s)."""
    out = {"steps": steps, "threads": 1, "Ns": list(ASV_NS), "time_run": {}, "time_sample": {}}
    for mode in ASV_MODES:
        out["time_run"][mode], out["time_sample"][mode] = {}, {}
        for n in ASV_NS:
            keep, sample, step, end, sync = asv_setup(cg, n, mode, dev)
            for _ in range(20):                              # warm-up (not in asv: its own repeats)
                sample()
                step()
            end()
            t0 = time.perf_counter()
            for _ in range(steps):
                sample()
                step()
            end()
            run = time.perf_counter() - t0
            t0 = time.perf_counter()
            for _ in range(steps):
                sample()
                sync()
            end()
            smp_s = time.perf_counter() - t0
            out["time_run"][mode][str(n)] = {"s": run, "us_per_step": run / steps * 1e6,
                                             "env_steps_per_s": n * steps / run}
            out["time_sample"][mode][str(n)] = {"s": smp_s, "us_per_call": smp_s / steps * 1e6,
                                                "samples_per_s": n * steps / smp_s}
            del keep, sample, step, end, sync
    if cpu_value:
        out["cpu_baseline_env_steps_per_s"] = cpu_value
        out["crossover"] = {m: next((n for n in ASV_NS if out["time_run"][m][str(n)]["env_steps_per_s"] > cpu_value),
                                    None) for m in ASV_MODES}
        out["crossover_note"] = ("smallest N of the grid whose time_run rate passes cpu_baseline (the C port in the "
                                 "reference ThreadedRunner shape, best thread count); null: none of the grid")
    return out


def rss_bytes():
    try:
        with open("/proc/self/statm") as f:
            return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
    except Exception:
        return None


def peakmem(cg, d, n, dev):
    """asv peakmem_runner (benchmarks/benchmarks.py:65-69): the memory a runner holds after one
    sample + step + sync, here with the reference's host views (numpy) live.  Device bytes are the
    drop in free HBM (hipMemGetInfo) over env + sampler + runner construction and the first
    step; host bytes the resident-set growth of this process (pinned views included)."""
    t = d.torch
    if t is None or not t.cuda.is_available():
        return None
    t.cuda.synchronize(dev)
    free0 = t.cuda.mem_get_info(dev)[0]
    rss0 = rss_bytes()
    env = cg.vec.get_vec_env(n)(device=dev)
    smp = cg.vec.get_vec_sampler(n)(SEED, device=dev)
    env.reset(SEED, N_PLAYERS, N_PIECES, cg.HARD, MAX_STEPS, False)
    runner = cg.vec.get_runner(n)(env, smp, None)
    views = (env.observations, env.selected_action_masks, env.infos, runner.get_actions())
    runner.sample()
    runner.step_sync()
    t.cuda.synchronize(dev)
    dev_bytes = free0 - t.cuda.mem_get_info(dev)[0]
    rss1 = rss_bytes()
    host = (rss1 - rss0) if rss0 is not None and rss1 is not None else None
    del views, runner, smp, env
    # pinned host views: ObsData + selected mask + Info + rewards + done + agent + actions
    pinned = n * (17216 + 128 + 192 + 16 + 1 + 1 + 64)
    return {"envs": n, "device_bytes": dev_bytes, "device_bytes_per_env": dev_bytes / n,
            "host_rss_growth_bytes": host, "host_pinned_view_bytes": pinned,
            "host_pinned_bytes_per_env": pinned / n,
            "note": "device: free-HBM drop (granularity of the HIP allocator included); host: RSS growth "
                    "of the process over the same span, the pinned numpy views included"}


def copy_peak_gbs(d):
    """A device-to-device copy of 2 GiB (torch), read + write bytes per second."""
    t = d.torch
    if t is None or not t.cuda.is_available():
        return None
    dev = t.device("cuda", device_of(d))
    a = t.empty(1 << 31, dtype=t.uint8, device=dev)
    b = t.empty_like(a)
    b.copy_(a)
    e0, e1 = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    s = e0.elapsed_time(e1) / 1e3 / 5
    del a, b
    return 2.0 * (1 << 31) / s / 1e9


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
    counts = sorted({1, max(1, cores // 2), cores})
    for threads in counts:
        po.run_threaded(vec, smp, 50, threads)                     # warm-up
        probe = 400
        t = po.run_threaded(vec, smp, probe, threads)
        steps = max(probe, int(probe * (seconds / len(counts)) / max(t, 1e-6)))
        t = po.run_threaded(vec, smp, steps, threads)
        rate = n * steps / t
        if best is None or rate > best[0]:
            best = (rate, threads, steps)
    rate, threads, steps = best
    out = {"value": rate, "unit": "env-steps/s", "cores": threads, "kind": "port",
           "sample": f"{n} envs (the first {n} of the workload: 4p HARD seed {SEED}) x {steps} steps of "
                     f"sample(selected masks)+step, C oracle, {threads} pinned worker threads "
                     f"(best of thread counts {counts})"}
    try:                                               # the port's speed against the reference
        cal = json.load(open(os.path.join(ROOT, "profiles", "calibration.json")))   # core's, same cores
        out["port_over_reference"] = cal["port_over_reference"]
        out["calibration"] = ("oracle/calibrate.py in the dev container (the reference cannot run on the "
                              "GPU box): " + cal["workload"] + "; median of " + str(len(cal["ratios"])) +
                              " interleaved reps " + ", ".join("%.2f" % x for x in cal["ratios"]))
    except Exception:
        pass
    return out


KERNEL_LABEL = {"wave": "k_env_rollout<selected>", "pipe": "k_env_rollout_pipe<selected>",
                "duo": "k_env_rollout_duo<selected> + k_env_fixup<selected>",
                "trio": "k_env_rollout_trio<selected> + k_env_fixup<selected>"}


def roofline(prof, n, k_chunk, launch_s, kind="trio", stamps=None, issue=None):
    """The dominant kernel -- the persistent rollout that runs a shard of n envs (`kind`: trio, wave,
    pipe or duo, cog_rollout_kind) -- against HBM, by the bytes it really moves: `traffic` is the HBM
    bytes of one launch of this exact engine source AT THIS LAUNCH SHAPE (n envs, k steps per launch,
    same kernel) from a rocprofv3 --pmc pass (profiles/pmc_profile.json `rollouts`: FETCH_SIZE x 2 +
    WRITE_SIZE, the gfx950 corrections of MI355X_MICROARCH.md), achieved = traffic / the launch time
    (HIP events on the runner's stream, live), peak = 8 TB/s, frac = achieved / peak -- reproducible
    from pmc_profile.json and the rocprofv3 kernel trace of the same command.

    The HBM roofline is not what limits this kernel (frac ~0.4): `limiter` names the bound that
    applies, the stepping wave's dependent instruction stream, with its busy fraction
    from the s_memtime phase stamps of a diagnostic build of the same source (profiles/
    stamps_profile.json: the share of a step the stepping wave spends issuing its own step rather
    than waiting for the other waves' progress counters) when one matches this engine.
    `survey_8d_equivalent` is SURVEY 8d's 800 algorithmic bytes per env-step over the same time: the
    bytes a one-launch-per-step sample + step would move; the rollout keeps each env's state on chip
    between steps, so that figure exceeds the HBM peak and is no roofline.  store_model: round 3's L2
    store-cost model of the same launch (a record).  No profile of this engine at this shape:
    traffic, achieved and frac are null."""
    alg = STEP_BYTES * n * k_chunk
    out = {"bound": "hbm", "kernel": KERNEL_LABEL.get(kind, kind), "rollout_kind": kind, "unit": "GB/s",
           "achieved": None, "peak": HBM_PEAK_GBS, "frac": None, "traffic": None,
           "env_steps_per_s": n * k_chunk / launch_s, "kernel_ms": launch_s * 1e3, "steps_per_launch": k_chunk,
           "envs_per_launch": n,
           "survey_8d_equivalent": {"bytes_per_env_step": STEP_BYTES, "bytes_per_launch": alg,
                                    "GBs": alg / launch_s / 1e9, "x_peak": alg / launch_s / 1e9 / HBM_PEAK_GBS,
                                    "note": "SURVEY 8d's algorithmic bytes of a one-launch-per-step sample + step; "
                                            "the rollout keeps the state on chip, so this is no roofline"},
           "limiter": {"kind": "issue: the stepping wave's dependent instruction stream (DESIGN.md 6)"},
           "store_model": None,
           "note": "achieved / frac: the HBM bytes this launch moves (PMC counters of this engine source at this "
                   "launch shape) / the live launch time; the kernel is limited by the stepping wave (limiter)"}
    waves = (n + 63) // 64
    valu_peak = N_SIMD * CLOCK_HZ / VALU_CYC                # wave64 VALU instructions per second
    e = ((prof or {}).get("rollouts") or {}).get("%d:%d" % (n, k_chunk))
    if e and e.get("kind") != kind:
        e = None                                          # profiled with another rollout kernel
    sc = (prof or {}).get("store_costs")
    l2 = (e or {}).get("l2_per_launch")
    if l2 and sc:
        t_store = l2["hits"] * sc["c_hit_s"] + l2["misses"] * sc["c_miss_s"]
        out["store_model"] = {"t_store_s": t_store, "frac": t_store / launch_s, "peak_env_steps_per_s": n * k_chunk / t_store,
                              "l2_write_requests_per_env_step": l2["writes"] / n / k_chunk,
                              "l2_hits_per_launch": l2["hits"], "l2_misses_per_launch": l2["misses"],
                              "l2_hit_rate": l2["hits"] / max(1.0, l2["hits"] + l2["misses"]),
                              "fabric_write_requests_per_launch": l2.get("fabric_write_requests"),
                              "c_hit_s": sc["c_hit_s"], "c_miss_s": sc["c_miss_s"]}
    if not e:
        out["note"] += "; no PMC profile of this engine source at %d envs x %d steps (%s; tools/pmc_profile.py): " \
                       "traffic unknown" % (n, k_chunk, kind)
    if e and e.get("bytes_per_launch") is not None:
        tr = e["bytes_per_launch"] + ((e.get("companion") or {}).get("bytes_per_launch") or 0.0)
        out["traffic"] = tr
        out["achieved"] = tr / launch_s / 1e9
        out["frac"] = tr / launch_s / 1e9 / HBM_PEAK_GBS
        out["counter_bytes_per_env_step"] = tr / n / k_chunk
    st = ((stamps or {}).get("shapes") or {}).get(str(n))
    if st:
        out["limiter"].update({k: st[k] for k in ("busy_ticks_per_step", "wait_ticks_per_step", "ticks_per_step",
                                                  "busy_frac", "steps_per_launch") if k in st})
        out["limiter"]["source"] = "profiles/stamps_profile.json (tools/duoprobe.cpp -DCOG_STAMPS, same engine source)"
    form = "lat" if (n + 63) // 64 <= N_CU else "two_per_cu"     # (cog_engine.hip launch_rollout's trio_jt)
    ip = (issue or {}).get(form)
    if st and ip and ip.get("ticks_per_step_issue") and kind == "trio":
        busy = st["busy_ticks_per_step"]
        out["limiter"]["issue_frac"] = ip["ticks_per_step_issue"] / busy
        out["limiter"]["dependent_chain_frac"] = ip["ticks_per_step_dependent"] / busy
        out["limiter"]["issue"] = {
            "per_step_instructions": ip["per_step_instructions"], "mix": ip["mix"], "kernel_form": form,
            "issue_ticks_per_step": ip["ticks_per_step_issue"], "dependent_ticks_per_step": ip["ticks_per_step_dependent"],
            "busy_ticks_per_step": busy,
            "note": "issue_frac = the stepping wave's per-step instructions (static count of its step loop without the "
                    "spin waits or the never-taken sampling fallback: an upper bound of what it issues) x a lone "
                    "wave's cost per instruction of each kind when it has independent work (tools/chainprobe.hip) "
                    "/ its measured busy ticks per step: near 1 = issue-bound, the chain at its floor; "
                    "dependent_chain_frac: the same with every instruction waiting for the one before "
                    "(profiles/issue_profile.json, tools/issue_frac.py, same engine source)"}
    pw = (e or {}).get("per_wave_step") or {}
    if pw.get("valu"):
        achieved = pw["valu"] * waves * k_chunk / launch_s
        out["valu_issue"] = {
            "achieved": achieved, "peak": valu_peak, "frac": achieved / valu_peak, "unit": "VALU wave-instr/s",
            "valu_per_wave_step": pw["valu"], "salu_per_wave_step": pw.get("salu"),
            "issue_quads_per_wave_step": pw.get("active_inst_any"), "wait_quads_per_wave_step": pw.get("wait_any"),
            "wave_quads_per_wave_step": pw.get("wave_cycles"),
            "note": "peak = 1,024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU; per 64-env wave and step (the duo / trio / "
                    "pipe: every wave of the workgroup); chip-wide, not the critical path (limiter)"}
    return out


def load_stamps(name="stamps_profile.json"):
    """profiles/<name> (stamps_profile.json, issue_profile.json) when it was measured on this exact
    engine source; else None."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from pmc_profile import engine_hash
        with open(os.path.join(ROOT, "profiles", name)) as f:
            p = json.load(f)
        return p if p.get("engine_sha") == engine_hash() else None
    except Exception:
        return None


def main():
    args = parse()
    d = Dist(args.gpus)
    import city_of_gold as cg
    from city_of_gold.shard import shard

    dev = device_of(d)
    bind_device(d, dev)
    lo, hi = shard(args.envs_total, d.rank, d.world)       # env i of rank r = global index lo + i
    n = hi - lo
    t0 = time.time()
    env, smp, runner = make(cg, n, SEED, dev, first=lo)
    setup_s = time.time() - t0
    chunk = max(1, min(args.chunk, max(args.steps, 1)))
    runner.set_chunk(chunk)

    runner.rollout(args.warmup)
    d.barrier_sync(runner)

    if args.profile_steps:                                # rocprofv3 captures: the rollout at
        runner.set_chunk(min(args.chunk, args.profile_steps))   # K steps per launch, then 200
        runner.rollout(args.profile_steps)                 # one-launch-per-step k_env_step's
        d.barrier_sync(runner)
        runner.set_chunk(1)
        runner.rollout(200)
        d.barrier_sync(runner)
        if d.rank == 0:
            print(json.dumps({"profile_steps": args.profile_steps, "envs": n, "chunk": args.chunk}))
        d.close()
        return

    # ---- timed region: exactly K steps --------------------------------------------------
    # Every rank starts its clock after the barrier and a synchronize, and stops it after its
    # own torch.cuda.synchronize(); the job's time is the max over ranks.  The closing barrier
    # runs after the clock: a gloo barrier takes 0.08 ms at 2 ranks and 0.4 ms at 8 (measured on
    # the CPU container), several times the 20-step rollout it would otherwise be added to.
    d.barrier_sync(runner)
    t0 = time.perf_counter()
    runner.rollout(args.steps)
    d.sync(runner)
    wall = time.perf_counter() - t0
    d.barrier()
    runner.sync()                                          # raises on an engine error
    wall_max = d.max(wall)
    total_env_steps = d.sum(float(n) * args.steps)
    value = total_env_steps / wall_max

    # ---- roofline of the dominant kernel at the timed launch length -----------------------
    k_chunk = min(chunk, args.steps)
    launch_s = kernel_time(runner, k_chunk, max(3, min(20, 4000 // max(k_chunk, 1))))
    prof = load_profile()
    roof = roofline(prof, n, k_chunk, launch_s, cg._city_of_gold.rollout_kind(n, N_PLAYERS, False), load_stamps(),
                    load_stamps("issue_profile.json"))

    haz, per = env.hazards()
    n_erase = int(((per & HAZ_ERASE_PAST) != 0).sum())
    n_any = int((per != 0).sum())
    n_erase, n_any = int(d.sum(n_erase)), int(d.sum(n_any))

    extras = {}
    if d.world == 1 and not args.no_extras:
        runner.set_chunk(chunk)
        extras["shard_sizes"] = {"us_per_step_at_%d" % n: launch_s / k_chunk * 1e6 if k_chunk >= 1000 else
                                 us_per_step(cg, n, dev),
                                 "us_per_step_at_%d" % N_SHARD8: us_per_step(cg, N_SHARD8, dev),
                                 "note": "rollout device time per step, 1,000-step launches; every shard size "
                                         "takes the trio rollout (4 waves per 64 envs: stepping, drawing and two "
                                         "storing waves; the N=8 shard of 8,192 envs is 128 workgroups, 65,536 "
                                         "envs are 1,024 in two rounds of two per CU)"}
        # one kernel launch per step (the runner's step() path)
        pl_steps = 500
        runner.set_chunk(1)
        d.barrier_sync(runner)
        t1 = time.perf_counter()
        runner.rollout(pl_steps)
        d.barrier_sync(runner)
        pl_wall = time.perf_counter() - t1
        pl_kern = kernel_time(runner, 1, pl_steps)
        ks = (prof or {}).get("k_env_step") or {}
        tr = ks.get("bytes_per_launch")
        extras["per_launch"] = {"kernel": "k_env_step<selected>", "value": n * pl_steps / pl_wall,
                                "ms_per_step": pl_wall / pl_steps * 1e3, "kernel_us": pl_kern * 1e6,
                                "hbm": {"survey_8d_GBs": STEP_BYTES * n / pl_kern / 1e9,
                                        "survey_8d_frac": STEP_BYTES * n / pl_kern / 1e9 / HBM_PEAK_GBS,
                                        "traffic": tr,
                                        "counter_frac": (tr / pl_kern / 1e9 / HBM_PEAK_GBS) if tr else None}}
        l2, sc = ks.get("l2_per_launch"), (prof or {}).get("store_costs")
        if l2 and sc and ks.get("envs_per_launch") == n:       # the store bound (roofline() above)
            t_store = l2["hits"] * sc["c_hit_s"] + l2["misses"] * sc["c_miss_s"]
            extras["per_launch"]["l2_store"] = {"t_store_us": t_store * 1e6, "frac": t_store / pl_kern,
                                                "l2_write_requests_per_env": (l2.get("writes") or 0) / n,
                                                "l2_hits": l2["hits"], "l2_misses": l2["misses"]}
        runner.set_chunk(chunk)
        enc_ms = env.time_encode(20)
        enc_gbs = ENCODE_BYTES * n / (enc_ms / 1e3) / 1e9
        cp_torch = copy_peak_gbs(d)
        cp = cg._city_of_gold.time_copy(dev, 1 << 31, 5)
        mix = cg._city_of_gold.time_stream_mix(dev, 1 << 28, 5)   # 256 MiB read, 1.75 GiB written
        extras["encode"] = {"kernel": "k_encode", "ms": enc_ms, "achieved": enc_gbs, "unit": "GB/s",
                            "frac": enc_gbs / HBM_PEAK_GBS, "copy_peak_GBs": cp,
                            "frac_of_copy_peak": enc_gbs / cp if cp else None,
                            "mix_peak_GBs": mix, "frac_of_mix_peak": enc_gbs / mix if mix else None,
                            "mix_peak_note": "a coalesced stream with the encode's read:write mix (16 B read, "
                                             "112 B written per work-item), the faster of plain and "
                                             "non-temporal stores: the peak of a kernel shaped like the encode",
                            "copy_peak_note": "the engine's copy kernel (16-B loads/stores, plain or non-temporal, 8 or 32 waves per CU: the fastest), "
                                              "2 x 2 GiB buffers, read + write bytes); torch's copy_ in the "
                                              "same run: %.0f GB/s" % cp_torch if cp_torch else "",
                            "algorithmic_bytes_per_launch": ENCODE_BYTES * n}
        del runner, smp, env
        # full dynamics: stored masks (moves, shop, specials), episodes of 30 turns -> auto-resets
        env, smp, runner = make(cg, n, SEED, dev, max_steps=30, stored=True, first=lo)
        runner.set_chunk(500)
        runner.rollout(200)
        d.barrier_sync(runner)
        fd_steps = 1000
        t1 = time.perf_counter()
        runner.rollout(fd_steps)
        d.barrier_sync(runner)
        fd_wall = time.perf_counter() - t1
        env.sync_host()
        resets = int(env.infos["total_length"].astype(bool).sum())
        extras["full_dynamics"] = {"value": n * fd_steps / fd_wall, "unit": "env-steps/s",
                                   "ms_per_step": fd_wall / fd_steps * 1e3, "steps": fd_steps,
                                   "workload": f"{n} envs, 4p HARD, max_steps 30, stored-mask sampler, "
                                               "500-step launches, auto-reset with device map generation",
                                   "envs_with_a_finished_episode": resets}
        del runner, smp, env
        # full dynamics without the constant resets: stored masks, max_steps 100,000 (episodes of the
        # reference harness's length), 1,000-step launches -- the general step's own rate
        env, smp, runner = make(cg, n, SEED, dev, stored=True, first=lo)
        runner.set_chunk(1000)
        runner.rollout(200)
        d.barrier_sync(runner)
        fs_steps = 2000
        t1 = time.perf_counter()
        runner.rollout(fs_steps)
        d.barrier_sync(runner)
        fs_wall = time.perf_counter() - t1
        fs_kern = kernel_time(runner, 1000, 2)
        extras["full_dynamics_steady"] = {
            "value": n * fs_steps / fs_wall, "unit": "env-steps/s", "ms_per_step": fs_wall / fs_steps * 1e3,
            "steps": fs_steps, "kernel_us_per_step": fs_kern / 1000 * 1e6,
            "rollout_kind": cg._city_of_gold.rollout_kind(n, N_PLAYERS, True),
            "workload": f"{n} envs, 4p HARD, max_steps 100000, stored-mask sampler (moves, purchases, specials: "
                        "test_environment.cpp:95-101's driver), 1,000-step launches"}
        # time_reset / time_sample (benchmarks/benchmarks.py:53-69)
        t1 = time.perf_counter()
        reps = 5
        for r in range(reps):
            env.reset(SEED + r, N_PLAYERS, N_PIECES, cg.HARD, MAX_STEPS, False)
        rs = (time.perf_counter() - t1) / reps
        masks = env.selected_action_masks
        smp.sample(masks)
        t1 = time.perf_counter()
        for _ in range(20):
            smp.sample(masks)
        ss = (time.perf_counter() - t1) / 20
        t1 = time.perf_counter()
        for r in range(reps):
            env.reset()                                   # reset_default: same params, rng continues
        rd = (time.perf_counter() - t1) / reps
        extras["reset"] = {"envs": n, "s_per_reset_call": rs, "resets_per_s": n / rs,
                           "note": "env.reset(seed, 4, 3, HARD, ...): device map generation + encode + "
                                   "host views refresh (1.1 GB D2H of ObsData)",
                           "reset_default": {"s_per_call": rd, "resets_per_s": n / rd,
                                             "note": "env.reset() without arguments, the form asv time_reset "
                                                     "times (benchmarks.py:58-62): parameters kept, each env's "
                                                     "rng continues"}}
        extras["sample"] = {"envs": n, "ms_per_call": ss * 1e3, "samples_per_s": n / ss,
                            "note": "sampler.sample(host masks): H2D masks, sampler kernel, D2H actions"}
        del runner, smp, env
        extras["host_loop"] = {
            "C2": host_loop(cg, 256, cg.EASY, dev, 300, False),
            "C4_shard": host_loop(cg, N_SHARD8, cg.HARD, dev, 100, True)}
        extras["time_reset_C2"] = time_reset_c2(cg, dev)
        extras["peakmem"] = peakmem(cg, d, n, dev)
        if not args.no_asv:
            extras["asv_grid"] = asv_grid(cg, dev)

    if d.rank == 0:
        cpu = None
        if d.world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_seconds)
            g = extras.get("asv_grid")
            if g:                                          # the crossover N against the same baseline
                ref = cpu["value"]
                g["cpu_baseline_env_steps_per_s"] = ref
                g["crossover"] = {m: next((n for n in ASV_NS if g["time_run"][m][str(n)]["env_steps_per_s"] > ref),
                                          None) for m in ASV_MODES}
                g["crossover_note"] = ("smallest N of the grid whose time_run rate passes cpu_baseline (the C port "
                                       "in the reference ThreadedRunner shape, best thread count); null: none")
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": d.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (procedurally generated maps from seeds; uniform masked random actions)",
            "steps_per_launch": chunk,
            "config": {
                "workload": "C5: 65,536 envs in total over the ranks, 4 players, HARD, n_pieces=3, "
                            "max_steps=100000, on-device masked sampler over selected_action_masks + step, "
                            "persistent rollout kernel, every step's AoS outputs stored in HBM",
                "n_envs_total": args.envs_total,
                "n_envs_per_gpu": n,
                "seed": SEED,
                "parallelism": f"env-sharded x{d.world} by index (runner.h:33-38 block split), no collectives",
            },
            "roofline": roof,
            "parity": {"hazard_envs": n_any, "erase_past_envs": n_erase,
                       "reference_pinned_envs": int(total_env_steps / max(args.steps, 1)) - n_any,
                       "note": "tests/test_gpu_timed_workloads.py runs this workload (and each N's last "
                               "shard) for 1,205 steps and compares every env with the C oracle; the "
                               "reference_pinned_envs (every env without a hazard flag) are also compared "
                               "with final-state digests the unmodified reference core produced "
                               "(tests/golden/ref_workloads.npz). The hazard envs -- chiefly erase_past: "
                               "map.cpp:727's past-the-end erase, GCC>=13 libstdc++ semantics, which the "
                               "image's libstdc++ 11 cannot run -- are pinned by the C oracle only (DESIGN.md 3)"},
            "timing": "per rank: clock started after barrier + synchronize, stopped after the rank's own "
                      "torch.cuda.synchronize(); value uses the max over ranks; the closing barrier runs "
                      "after the clock",
            "setup_s": setup_s,
            "cpu_baseline": cpu,
        }
        out.update(extras)
        print(json.dumps(out), flush=True)
    d.close()


if __name__ == "__main__":
    main()
