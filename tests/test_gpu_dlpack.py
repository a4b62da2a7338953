"""GPU: the device views as torch tensors through DLPack (city_of_gold.device_tensors), the
zero-copy device consumer path of SURVEY §8f rank 2, and stepping from device-resident actions
(env.step_device).  The tensors must alias the engine's HBM records byte for byte."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def make(cg, n, seed):
    env = cg.vec.get_vec_env(n)()
    smp = cg.vec.get_vec_sampler(n)(seed)
    env.reset(seed, 4, 3, cg.HARD, 100000, False)
    return env, smp


def test_device_tensors_alias_engine_state(cg):
    import torch
    n = 512
    env, smp = make(cg, n, 77)
    runner = cg.vec.get_runner(n)(env, smp, None, device_views=True)
    runner.set_chunk(16)
    runner.rollout(48)
    runner.sync()
    env.sync_host()
    t = cg.device_tensors(env, smp)
    ptrs = env.device_pointers()
    for nm in cg.DEVICE_VIEWS:
        assert t[nm].is_cuda and t[nm].data_ptr() == ptrs[nm], nm
    assert t["observations"].shape == (n, 17216) and t["observations"].dtype == torch.uint8
    assert t["rewards"].shape == (n, 4) and t["rewards"].dtype == torch.float32
    assert t["dones"].shape == (n,) and t["actions"].shape == (n, 64)
    torch.cuda.synchronize()
    for nm in ("observations", "selected_action_masks", "infos"):
        host = getattr(env, nm).view(np.uint8).reshape(n, -1)
        assert np.array_equal(t[nm].cpu().numpy(), host), nm
    assert np.array_equal(t["rewards"].cpu().numpy(), env.rewards)
    assert np.array_equal(t["dones"].cpu().numpy(), env.dones.view(np.uint8))
    assert np.array_equal(t["agent_selection"].cpu().numpy(), env.agent_selection)
    assert t["actions"].data_ptr() == smp.device_actions()   # (its host view is not refreshed
                                                            # by a device-views runner)
    del runner, env, smp                                  # the tensors keep the engine alive
    assert int(t["observations"][:, 16128].sum().item()) >= 0


def test_step_device_equals_host_step(cg):
    """Actions sampled into a torch tensor and stepped from HBM == the same actions from the host."""
    import torch
    n = 256
    a, _ = make(cg, n, 5)
    b, _ = make(cg, n, 5)
    g = torch.Generator().manual_seed(3)
    for _ in range(40):
        masks = a.selected_action_masks.view(np.uint8).reshape(n, 128)[:, :92].astype(bool)
        acts = np.zeros(n, dtype=cg.ActionData)
        play = masks[:, :22]                                 # a random legal play (or pass)
        r = torch.rand((n, 22), generator=g).numpy() * play
        acts["play"] = r.argmax(1).astype(np.uint8)
        d_acts = torch.from_numpy(acts.view(np.uint8).reshape(n, 64).copy()).cuda()
        torch.cuda.synchronize()
        a.step_device(d_acts.data_ptr())
        b.step(acts)
        a.sync_host()
        for nm in ("observations", "selected_action_masks", "infos"):
            assert np.array_equal(getattr(a, nm).view(np.uint8), getattr(b, nm).view(np.uint8)), nm


def test_step_device_orders_after_torch_stream(cg):
    """No torch.cuda.synchronize(): the actions are written on torch's current stream behind a
    long matmul chain, then step_device() is called at once; it must order its kernel after that
    stream (event + stream wait), not read the tensor's old (all-pass) contents."""
    import torch
    n = 4096
    a, _ = make(cg, n, 9)
    b, _ = make(cg, n, 9)
    masks = a.selected_action_masks.view(np.uint8).reshape(n, 128)[:, :22].astype(bool)
    acts = np.zeros(n, dtype=cg.ActionData)
    acts["play"] = np.where(masks[:, 1:].any(1), masks[:, 1:].argmax(1) + 1, 0).astype(np.uint8)
    assert (acts["play"] > 0).sum() > n // 2
    src = torch.from_numpy(acts.view(np.uint8).reshape(n, 64).copy()).pin_memory()
    d_acts = torch.zeros((n, 64), dtype=torch.uint8, device="cuda")
    m = torch.randn(4096, 4096, device="cuda")
    torch.cuda.synchronize()
    for _ in range(30):                                    # ~tens of ms of work on torch's stream
        m = torch.tanh(m @ m)
    d_acts.copy_(src, non_blocking=True)                  # queued behind the matmuls
    a.step_device(d_acts.data_ptr())                      # orders after torch's current stream
    b.step(acts)
    for nm in ("observations", "selected_action_masks", "infos"):
        assert np.array_equal(getattr(a, nm).view(np.uint8), getattr(b, nm).view(np.uint8)), nm
    del m


def test_signal_stream_orders_torch_reads_after_rollout(cg):
    """A device-views rollout is asynchronous; env.signal_stream(torch stream) makes torch's
    later reads wait for it without runner.sync()."""
    import torch
    n = 4096
    env, smp = make(cg, n, 13)
    runner = cg.vec.get_runner(n)(env, smp, None, device_views=True)
    runner.set_chunk(1000)
    t = cg.device_tensors(env)
    runner.rollout(3000)                                   # milliseconds of device work
    env.signal_stream(cg.stream_handle())
    snap = t["selected_action_masks"].clone()              # on torch's stream, after the rollout
    dn = t["infos"].clone()
    runner.sync()
    env.sync_host()
    assert np.array_equal(snap.cpu().numpy(), env.selected_action_masks.view(np.uint8).reshape(n, -1))
    assert np.array_equal(dn.cpu().numpy(), env.infos.view(np.uint8).reshape(n, -1))
