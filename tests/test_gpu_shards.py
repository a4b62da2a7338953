"""GPU: multi-device handles and the multi-process path with the real engine.

A handle may span several GPUs of one process (cog_env_create_multi: contiguous shards, the
reference runner's block split runner.h:33-38).  Seeds are seed + global index, so any shard
layout must give the bytes of a one-shard run; on a one-GPU box the shards share the GPU (one
stream each), which exercises the same host code.  The torchrun test runs two ranks with the
engine (COG_DEVICES pins both ranks to GPU 0) and compares their gathered shards with a
single-process run; the last test runs bench.py itself under torchrun."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import pyoracle as po

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("observations", "selected_action_masks", "infos", "rewards", "dones", "agent_selection")


def same(a, b, what):
    for nm in FIELDS:
        x, y = getattr(a, nm), getattr(b, nm)
        if x.dtype.names:
            assert po.named_equal(x, y) is None, f"{what}: {nm}"
        else:
            assert np.array_equal(x, y), f"{what}: {nm}"


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]], ids=["2shards", "3shards"])
def test_sharded_handle_equals_single(cg, devices):
    n, seed = 1000, 31
    one, many = cg.vec.get_vec_env(n)(device=0), cg.vec.get_vec_env(n)(device=devices)
    assert one.num_shards == 1 and many.num_shards == len(devices)
    firsts = [many.shard_info(k)[0] for k in range(many.num_shards)]
    counts = [many.shard_info(k)[1] for k in range(many.num_shards)]
    assert firsts[0] == 0 and sum(counts) == n and counts[:-1] == [n // len(devices)] * (len(devices) - 1)
    s1, sm = cg.vec.get_vec_sampler(n)(seed, device=0), cg.vec.get_vec_sampler(n)(seed, device=devices)
    for e in (one, many):
        e.reset(seed, 4, 3, cg.HARD, 25, False)
    same(one, many, "after reset")
    # host API: sample(masks) + step(actions)
    for t in range(30):
        s1.sample(po.stored_masks(one))
        sm.sample(po.stored_masks(many))
        assert po.named_equal(s1.get_actions(), sm.get_actions()) is None
        one.step(s1.get_actions())
        many.step(sm.get_actions())
        same(one, many, f"host step {t}")
    # runner: host-view steps, then device-only rollouts with resets across the shards
    r1 = cg.vec.get_runner(n)(one, s1, None, stored_masks=True)
    rm = cg.vec.get_runner(n)(many, sm, None, stored_masks=True)
    for t in range(20):
        for r in (r1, rm):
            r.sample()
            r.step_sync()
        same(one, many, f"runner step {t}")
    d1 = cg.vec.get_runner(n)(one, s1, None, device_views=True, stored_masks=True)
    dm = cg.vec.get_runner(n)(many, sm, None, device_views=True, stored_masks=True)
    for r in (d1, dm):
        r.set_chunk(40)
        r.rollout(300)
        r.sync()
    one.sync_host()
    many.sync_host()
    same(one, many, "after device rollouts")
    assert int(one.dones.sum()) >= 0 and one.infos["total_length"].any()
    # a runner needs the same shards on both sides
    with pytest.raises(ValueError):
        cg.vec.get_runner(n)(many, s1, None)
    assert np.array_equal(one.hazards()[1], many.hazards()[1])


def test_sharded_device_views(cg):
    import torch
    n = 300
    env = cg.vec.get_vec_env(n)(device=[0, 0])
    env.reset(5, 4, 3, cg.HARD, 100000, False)
    for k in range(2):
        first, count, dev = env.shard_info(k)
        t = cg.device_tensors(env, shard=k)
        assert t["observations"].shape == (count, 17216) and t["observations"].device.index == dev
        torch.cuda.synchronize()
        host = env.observations[first:first + count].view(np.uint8).reshape(count, -1)
        assert np.array_equal(t["observations"].cpu().numpy(), host)


WORKER = r"""
import json, os, sys
sys.path[:0] = [os.path.join(ROOT, "gym-eldorado_amd"), os.path.join(ROOT, "oracle")]
import torch.distributed as dist
import city_of_gold as cg
from city_of_gold.shard import shard, shard_seed
import pyoracle as po
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
lo, hi = shard(N, rank, world)
env = cg.vec.get_vec_env(hi - lo)()                  # device from LOCAL_RANK / COG_DEVICES
smp = cg.vec.get_vec_sampler(hi - lo)(SEED, first_index=lo)
env.reset(shard_seed(SEED, lo), 4, 3, cg.HARD, 30, False)
r = cg.vec.get_runner(hi - lo)(env, smp, None, device_views=True, stored_masks=True)
r.set_chunk(50)
r.rollout(STEPS)
r.sync()
env.sync_host()
dig = [po.step_digest(env.observations[i:i + 1], env.selected_action_masks[i:i + 1], env.rewards[i:i + 1],
                      env.dones[i:i + 1], env.agent_selection[i:i + 1], env.infos[i:i + 1],
                      env.selected_action_masks[i:i + 1]).hex() for i in range(hi - lo)]
out = [None] * world
dist.all_gather_object(out, (lo, dig))
if rank == 0:
    with open(OUT, "w") as f:
        json.dump(out, f)
dist.destroy_process_group()
"""


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def torchrun(args, env_extra, timeout):
    env = dict(os.environ, COG_DEVICES="0", COG_DEVICE="0", **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port())] + args
    return subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(240)
def test_torchrun_two_ranks_engine_shards(cg, tmp_path):
    n, seed, steps = 2048, 555, 150
    script = tmp_path / "worker.py"
    out = tmp_path / "gathered.json"
    script.write_text(f"ROOT = {ROOT!r}; N = {n}; SEED = {seed}; STEPS = {steps}; OUT = {str(out)!r}\n" + WORKER)
    p = torchrun([str(script)], {}, 200)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    gathered = json.load(open(out))
    env = cg.vec.get_vec_env(n)(device=0)
    smp = cg.vec.get_vec_sampler(n)(seed, device=0)
    env.reset(seed, 4, 3, cg.HARD, 30, False)
    r = cg.vec.get_runner(n)(env, smp, None, device_views=True, stored_masks=True)
    r.set_chunk(50)
    r.rollout(steps)
    r.sync()
    env.sync_host()
    full = [po.step_digest(env.observations[i:i + 1], env.selected_action_masks[i:i + 1], env.rewards[i:i + 1],
                           env.dones[i:i + 1], env.agent_selection[i:i + 1], env.infos[i:i + 1],
                           env.selected_action_masks[i:i + 1]).hex() for i in range(n)]
    merged = []
    for lo, ds in sorted((lo, ds) for lo, ds in gathered):
        merged.extend(ds)
    assert merged == full


@pytest.mark.timeout(240)
def test_bench_under_torchrun_two_ranks(cg):
    p = torchrun(["bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5", "--envs-total", "4096"], {}, 200)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["steps"] == 20 and d["scaling"] == "strong"
    assert d["config"]["n_envs_total"] == 4096 and d["config"]["n_envs_per_gpu"] == 2048
    assert d["value"] > 0 and d["cpu_baseline"] is None
