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
