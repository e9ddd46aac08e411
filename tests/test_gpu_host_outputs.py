"""GPU tests of the host delivery of step outputs (ch_outputs_to_host, cattleherd.env.HostOutputs: the batched SB3
VecEnv's and RLlib dict surface's source of numpy arrays) and of the runtime's buffer / error bookkeeping
(ADVICE r3): every delivered array equals the device buffer it comes from, bit for bit, including the envs that
auto-reset (compacted on the device, ascending) when more of them end in one step than the speculative first copy
holds; a new obs_out tensor at a recycled address is written in full; a full reset does not swallow a device error
nobody has seen."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check_delivery(b, h):
    import torch
    torch.cuda.synchronize()
    assert np.array_equal(h["obs"], b.obs.cpu().numpy())
    assert np.array_equal(h["reward"], b.reward.cpu().numpy(), equal_nan=True)
    assert np.array_equal(h["terminated"], b.terminated.cpu().numpy())
    assert np.array_equal(h["truncated"], b.truncated.cpu().numpy())
    rs = b.reset_happened.cpu().numpy()
    assert np.array_equal(h["reset_happened"], rs)
    idx = np.nonzero(rs)[0]
    assert np.array_equal(h["ended_env"], idx)
    assert np.array_equal(h["ended_obs"], b.terminal_obs.cpu().numpy()[idx])
    assert np.array_equal(h["ended_stats"], b.episode_stats.cpu().numpy()[idx])
    if "agent_active" in h:
        assert np.array_equal(h["agent_active"], b.agent_active.cpu().numpy())
    return len(idx)


@pytest.mark.parametrize("mode,E,n,m,level", [("ctde", 512, 4, 16, 2), ("marl", 256, 4, 32, 2), ("ctde", 300, 2, 8, 7)])
def test_outputs_to_host_equal_device_buffers(mode, E, n, m, level):
    from cattleherd.env import HerdBatch
    b = HerdBatch(E, n, m, mode=mode, curriculum_level=level, compat=mode == "marl" or n > 2)
    b.reset()
    host = b.host_outputs(ring=2, ended=True, agents=mode == "marl")
    ended = 0
    for _ in range(120):
        b.step(random_actions=True, autoreset=True, terminal_obs=True)
        ended += _check_delivery(b, host.fetch())
    assert ended > 0 or mode == "marl"
    # every env ends in the same step (more than the 64 of the first copy): CTDE at its time limit; MARL (whose
    # episodes do not end on truncation, marl_wrapper.py:113-117) with the drones around the herd centroid at level 2
    s = b.get_state()
    if mode == "ctde":
        b.set_state({"step_counter": np.full(E, 10 ** 6)})
    else:
        c = s["cow_pos"].mean(1)
        for k in range(n):
            s["drone_pos"][:, k, 0] = c[:, 0] + 0.3 * (k - (n - 1) / 2)
            s["drone_pos"][:, k, 1] = c[:, 1]
            s["drone_pos"][:, k, 2] = 0.45
        s["drone_vel"][:] = 0
        b.set_state({k: s[k] for k in ("drone_pos", "drone_vel")})
    b.step(actions=b.actions * 0, autoreset=True, terminal_obs=True)
    k = _check_delivery(b, host.fetch())
    assert k == E if mode == "ctde" else k > 64, k
    b.close()


def test_vec_env_numpy_step_matches_tensor_step():
    """CattleHerdVecEnv.step (numpy in, pinned delivery out) and the same batch stepped with the same actions
    through the tensor path give the same observations, rewards, dones and terminal observations; the array a step
    returns stays valid through the next step (two pinned buffers in turn)."""
    import torch
    from cattleherd.env import HerdBatch
    from cattleherd.vec_env import CattleHerdVecEnv
    E, n, m = 256, 4, 16
    venv = CattleHerdVecEnv(E, num_drones=n, num_cattle=m, curriculum_level=2)
    twin = HerdBatch(E, n, m, mode="ctde", curriculum_level=2)
    o0 = venv.reset()
    twin.reset()
    assert np.array_equal(o0, twin.obs.cpu().numpy())
    rng = np.random.default_rng(3)
    prev, prev_copy, ends = None, None, 0
    for _ in range(150):
        a = rng.uniform(-1, 1, (E, n, 4)).astype(np.float32)
        obs, rew, dones, infos = venv.step(a)
        if prev is not None:
            assert np.array_equal(prev, prev_copy)   # the previous step's array is untouched
        o, r, te, tr = twin.step(torch.from_numpy(a).to(twin.device), autoreset=True, terminal_obs=True)
        assert np.array_equal(obs, o.cpu().numpy())
        assert np.array_equal(rew, r[:, 0].cpu().numpy(), equal_nan=True)
        assert np.array_equal(dones, (te[:, 0] | tr[:, 0]).bool().cpu().numpy())
        tob = twin.terminal_obs.cpu().numpy()
        for e in np.nonzero(dones)[0]:
            ends += 1
            assert np.array_equal(infos[e]["terminal_observation"], tob[e])
            assert infos[e]["TimeLimit.truncated"] == bool(tr[e, 0] and not te[e, 0])
        for e in np.nonzero(~dones)[0][:8]:
            assert set(infos[e]) == {"answer"}
        prev, prev_copy = obs, obs.copy()
    assert ends > 0
    venv.close()
    twin.close()


def test_obs_out_new_tensor_at_recycled_address_is_written_in_full():
    """A step into obs_out B after a step into obs_out A: if B is a new tensor (even at A's recycled address,
    holding other data), every block is written in full -- equal to a twin batch stepping into its own buffer."""
    import torch
    from cattleherd.env import HerdBatch
    E, n, m = 256, 4, 16
    b = HerdBatch(E, n, m, mode="ctde")
    twin = HerdBatch(E, n, m, mode="ctde")
    for x in (b, twin):
        x.reset()
    a = torch.empty((E, 12, 86), dtype=torch.float32, device=b.device)
    addr = a.data_ptr()
    b.step(random_actions=True, obs_out=a)
    twin.step(random_actions=True)
    torch.cuda.synchronize()
    assert torch.equal(a, twin.obs)
    del a
    c = torch.full((E, 12, 86), 7.0, dtype=torch.float32, device=b.device)   # the caching allocator's recycled block
    recycled = c.data_ptr() == addr
    b.step(random_actions=True, obs_out=c)
    twin.step(random_actions=True)
    torch.cuda.synchronize()
    assert torch.equal(c, twin.obs), f"recycled address: {recycled}"
    # the same tensor again: only the changing entries are stored, the constant bytes are still right
    b.step(random_actions=True, obs_out=c)
    twin.step(random_actions=True)
    torch.cuda.synchronize()
    assert torch.equal(c, twin.obs)
    b.close()
    twin.close()


def test_full_reset_reports_an_unseen_device_error():
    """A device error nobody has read (no ch_sync / ch_metrics / ch_get_state since the failing step) is not
    cleared silently by a full reset: the reset happens and returns CH_ERR_DEVICE; after that the handle is clean.
    An error already reported is cleared by the full reset without another report."""
    from cattleherd import _lib
    from cattleherd.env import HerdBatch
    b = HerdBatch(256, 4, 16, mode="ctde")
    b.reset()
    assert _lib.lib().ch__set_phase_mask(b.handle, ctypes.c_int32(64)) == 0
    b.step(random_actions=True)
    assert _lib.lib().ch__set_phase_mask(b.handle, ctypes.c_int32(0)) == 0
    with pytest.raises(_lib.ChError) as ei:
        b.reset()
    assert ei.value.code == _lib.CH_ERR_DEVICE and "never reported" in str(ei.value)
    b.sync()
    b.step(random_actions=True)
    b.sync()
    # seen first, then reset: no second report
    assert _lib.lib().ch__set_phase_mask(b.handle, ctypes.c_int32(64)) == 0
    b.step(random_actions=True)
    assert _lib.lib().ch__set_phase_mask(b.handle, ctypes.c_int32(0)) == 0
    with pytest.raises(_lib.ChError):
        b.sync()
    b.reset()
    b.sync()
    b.close()
