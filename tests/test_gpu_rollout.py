"""GPU tests of the on-device PPO rollout buffer (cattleherd.rollout; ch_rollout_*), against plain torch
/ NumPy restatements of SB3 2.7's collect_rollouts, DiagGaussianDistribution and
compute_returns_and_advantage (SB3 is not installed: parity unpinned to its source; the reference's PPO
setup is CTDECattleHerder.py:107-127).  Tolerances: log-probabilities 1e-5 relative (float32 sums in a
different order than torch's), values / bootstrapped rewards 1e-5 (MFMA vs torch matmul), GAE 2e-6
against the float32 NumPy recursion fed with the buffer's own rewards and values."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _gae_numpy(rewards, values, episode_starts, last_values, dones, gamma, lam):
    """RolloutBuffer.compute_returns_and_advantage (float32 arrays, NumPy >= 2 scalar promotion)."""
    T = rewards.shape[0]
    adv = np.zeros_like(rewards)
    last = np.zeros_like(rewards[0])
    for step in reversed(range(T)):
        if step == T - 1:
            nnt = np.float32(1.0) - dones.astype(np.float32)
            nv = last_values
        else:
            nnt = np.float32(1.0) - episode_starts[step + 1]
            nv = values[step + 1]
        delta = rewards[step] + gamma * nv * nnt - values[step]
        last = delta + gamma * lam * nnt * last
        adv[step] = last
    return adv, adv + values


@pytest.mark.parametrize("E,n,m,compat,level", [(512, 4, 16, True, 2), (4096, 2, 8, False, 7)],
                         ids=["4x16_level2", "configs2_training"])
def test_rollout_buffer_matches_sb3_semantics(E, n, m, compat, level):
    """configs[2]'s training leg is the second case: 4096 envs x (2 drones, 8 cattle), NaN-safe rewards
    (compat = 0; with the reference's quirk every 2-drone CTDE reward is NaN, CattleAviary.py:234-246), the
    driver's default curriculum level 7 (80 s episodes, CTDECattleHerder.py:91-127)."""
    import torch
    from cattleherd.env import HerdBatch
    from cattleherd.policy import DevicePolicy
    from cattleherd.rollout import DeviceRolloutBuffer
    T = 40
    A = 4 * n                        # the CTDE action space is Box((NUM_DRONES, 4)), flattened by SB3
    sc = 4800 - 30 + (np.arange(E) % 60)   # half the envs reach the 80 s time limit inside the rollout

    def make():
        bb = HerdBatch(E, n, m, mode="ctde", curriculum_level=level, compat=compat)
        bb.reset()
        bb.set_state({"step_counter": sc})
        return bb
    b = make()
    actor = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, A], seed=1), "tanh", None)
    critic = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 1], seed=2), "tanh", None)
    log_std = torch.full((A,), -1.0, device=b.device)
    rb = DeviceRolloutBuffer(b, T)
    assert rb.act_dim == A
    rb.collect(actor, critic, log_std, seed=123)
    torch.cuda.synchronize()
    obs = rb.obs.cpu()
    # 1. log-probabilities and values of the stored samples under the torch reference forward
    mean = actor.reference(rb.obs.view(T * E, -1)).view(T, E, A)
    std = torch.exp(log_std)
    want_lp = torch.distributions.Normal(mean, std).log_prob(rb.actions).sum(-1)
    assert torch.allclose(rb.log_probs, want_lp, rtol=1e-5, atol=1e-4)
    want_v = critic.reference(rb.obs.view(T * E, -1)).view(T, E)
    assert torch.allclose(rb.values, want_v, rtol=1e-5, atol=1e-5)
    eps = (rb.actions - mean) / std
    assert abs(float(eps.mean())) < 0.02 and abs(float(eps.std()) - 1.0) < 0.02   # standard normal noise
    # 2. episode starts: first step all ones (after reset), then the previous step's dones
    es = rb.episode_starts.cpu().numpy()
    assert np.all(es[0] == 1.0)
    # 3. the same rollout replayed step by step on a twin batch with the stored (clipped) actions
    b2 = make()
    rew, dn, tl = [], [], []
    for t in range(T):
        assert torch.equal(b2.obs.view(E, -1).cpu(), obs[t]), t
        a = rb.actions[t].clamp(-1.0, 1.0).view(E, n, 4)
        _, r, te, tr = b2.step(a, autoreset=True, terminal_obs=True)
        tv = critic.reference(b2.terminal_obs.view(E, -1))[:, 0]
        te, tr = te[:, 0].bool(), tr[:, 0].bool()
        rr = r[:, 0].clone()
        rr[tr & ~te] += 0.99 * tv[tr & ~te]
        rew.append(rr.cpu().numpy()); dn.append((te | tr).cpu().numpy()); tl.append((tr & ~te).cpu().numpy())
    rew, dn = np.array(rew), np.array(dn)
    if not compat:
        assert np.isfinite(rb.rewards.cpu().numpy()).all()
    assert np.allclose(rb.rewards.cpu().numpy(), rew, rtol=1e-5, atol=1e-5)   # V(terminal) MFMA vs torch
    assert np.array_equal(es[1:], dn[:-1].astype(np.float32))
    assert dn.any() and np.array(tl).any()
    # 4. GAE bit for bit against the float32 recursion, from the device's V(last obs) (itself held to torch
    # at the values' tolerance: the MFMA and torch sum the 1032 products in different orders)
    last_v_ref = critic.reference(b2.obs.view(E, -1))[:, 0]
    assert torch.allclose(rb.value[:, 0], last_v_ref, rtol=1e-5, atol=1e-5)
    last_v = rb.value[:, 0].cpu().numpy()
    adv, ret = _gae_numpy(rb.rewards.cpu().numpy(), rb.values.cpu().numpy(), es, last_v, dn[-1],
                          0.99, 0.95)
    assert np.allclose(rb.advantages.cpu().numpy(), adv, rtol=2e-6, atol=2e-6)
    assert np.allclose(rb.returns.cpu().numpy(), ret, rtol=2e-6, atol=2e-6)
    b.close()
    b2.close()


@pytest.mark.parametrize("T", [5, 13, 16, 24, 32])
@pytest.mark.parametrize("path", [0, 2, 1], ids=["epilogues", "store_kernel", "copy_each"])
def test_native_collect_equals_python_loop(T, path):
    """ch_rollout_collect (the loop in C++) and collect_steps (the same kernels launched from Python) fill
    identical buffers, across auto-resets and truncation bootstraps: rollouts shorter than the deferred bootstrap's
    16-step flush period (kTvEvery, ch_api.cpp), crossing it, and ending exactly on a flush (16, 32), on each of the
    collection's paths (the store folded into the
    forward epilogues, the stand-alone store kernel, every observation copied into the buffer)."""
    import ctypes
    import torch
    from cattleherd import _lib
    from cattleherd.env import HerdBatch
    from cattleherd.policy import DevicePolicy
    from cattleherd.rollout import DeviceRolloutBuffer
    E, n, m = 256, 4, 16
    sc = 4800 - T // 2 + (np.arange(E) % T)   # truncations at every step of the rollout
    bufs = []
    for native in (True, False):
        b = HerdBatch(E, n, m, mode="ctde", curriculum_level=2)
        b.reset()
        b.set_state({"step_counter": sc})
        assert _lib.lib().ch__set_rollout_path(b.handle, ctypes.c_int32(path)) == 0
        actor = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 4 * n], seed=1), "tanh", None)
        critic = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 1], seed=2), "tanh", None)
        rb = DeviceRolloutBuffer(b, T)
        log_std = torch.full((4 * n,), -1.0, device=b.device)
        (rb.collect if native else rb.collect_steps)(actor, critic, log_std, seed=9)
        torch.cuda.synchronize()
        bufs.append({k: getattr(rb, k).cpu() for k in ("obs", "actions", "rewards", "episode_starts", "values",
                                                        "log_probs", "advantages", "returns")})
        assert rb.episode_starts[1:].sum() > 0
        b.close()
    for k in bufs[0]:
        assert torch.equal(bufs[0][k], bufs[1][k]), k


@pytest.mark.parametrize("T", [6, 24])
def test_fused_step_actor_is_bit_identical(T):
    """ch_rollout_collect with the actor forward fused into the step kernel (k_step2_actor: configs[3]'s geometry,
    4096 envs, the workgroup's 16 observation rows read back right after it wrote them) fills the same buffers as
    the separate actor + critic launch, across auto-resets and the deferred truncation bootstrap's flush; the fused
    kernel is the one that ran (T - 1 fused steps per collection)."""
    import ctypes
    import torch
    from cattleherd import _lib
    from cattleherd.env import HerdBatch
    from cattleherd.policy import DevicePolicy
    from cattleherd.rollout import DeviceRolloutBuffer
    L = _lib.lib()
    L.ch__rollout_fused_steps.restype = ctypes.c_int64
    E, n, m = 4096, 4, 16
    sc = 4800 - T // 2 + (np.arange(E) % T)
    bufs = []
    for path in (8, 4):
        b = HerdBatch(E, n, m, mode="ctde", curriculum_level=2)
        b.reset()
        b.set_state({"step_counter": sc})
        assert L.ch__set_rollout_path(b.handle, ctypes.c_int32(path)) == 0
        actor = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 4 * n], seed=1), "tanh", None)
        critic = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 1], seed=2), "tanh", None)
        rb = DeviceRolloutBuffer(b, T)
        log_std = torch.full((4 * n,), -1.0, device=b.device)
        rb.collect(actor, critic, log_std, seed=9)
        torch.cuda.synchronize()
        assert L.ch__rollout_fused_steps(b.handle) == (T - 1 if path == 4 else 0)
        bufs.append({k: getattr(rb, k).cpu() for k in ("obs", "actions", "rewards", "episode_starts", "values",
                                                        "log_probs", "advantages", "returns")})
        bufs[-1]["env_obs"] = b.obs.cpu()
        assert rb.episode_starts[1:].sum() > 0
        b.close()
    for k in bufs[0]:
        assert torch.equal(bufs[0][k], bufs[1][k]), k


def test_fused_actor_critic_is_bit_identical():
    """The SB3 actor and critic packed as one net (layer 1 stacked, layers 2-3 block-diagonal; one forward per
    step reads the observation once): its two heads equal the separate nets' forwards bit for bit -- the
    reference's trained model-v16-6 on oracle observations and random nets on a batch -- and a native collection
    with it fills the same buffers as with the separate nets."""
    import torch
    from cattleherd.env import HerdBatch
    from cattleherd.policy import DevicePolicy
    from cattleherd.rollout import DeviceRolloutBuffer
    from helpers import load
    d = load("policy_ctde_v16_6.npz")
    sd = {k.replace("__", "."): torch.tensor(d[k]) for k in d.files if "__" in k}
    actor, critic = DevicePolicy.sb3_actor(sd, clip=False), DevicePolicy.sb3_critic(sd)
    fused = DevicePolicy.sb3_actor_critic(sd)
    x = torch.tensor(d["obs"], device=fused.device).reshape(len(d["obs"]), -1)
    y = fused.forward(x)
    assert torch.equal(y[:, :48], actor.forward(x)) and torch.equal(y[:, 48:], critic.forward(x))
    E, T, n, m = 1024, 24, 4, 16
    sc = 4800 - 12 + (np.arange(E) % 24)
    bufs = []
    for use_fused in (False, True):
        b = HerdBatch(E, n, m, mode="ctde", curriculum_level=7)
        b.reset()
        b.set_state({"step_counter": sc})
        rb = DeviceRolloutBuffer(b, T, act_dim=48)
        log_std = torch.full((48,), -1.0, device=b.device)
        if use_fused:
            rb.collect(fused, None, log_std, seed=4)
        else:
            rb.collect(actor, critic, log_std, seed=4)
        torch.cuda.synchronize()
        bufs.append({k: getattr(rb, k).cpu() for k in ("obs", "actions", "rewards", "episode_starts", "values",
                                                        "log_probs", "advantages", "returns")})
        assert rb.episode_starts[1:].sum() > 0
        b.close()
    for k in bufs[0]:
        assert torch.equal(bufs[0][k], bufs[1][k]), k


def test_block_diagonal_skip_is_exact():
    """ch_mlp.split_out / split_in: the kernel skips a block-diagonal layer's zero blocks; the outputs equal the
    dense forward of the same weights bit for bit (random nets, packed and raw weights, several row counts)."""
    import torch
    from cattleherd.policy import DevicePolicy
    actor = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 48], seed=5), "tanh", None)
    critic = DevicePolicy(DevicePolicy.random_layers([12 * 86, 128, 128, 1], seed=6), "tanh", None)
    fused = DevicePolicy.fuse(actor, critic)
    assert fused.splits == {1: (128, 128), 2: (48, 128)}
    dense = DevicePolicy(list(zip(fused.weights, fused.biases)), "tanh", None)
    g = torch.Generator().manual_seed(7)
    for rows in (1, 100, 4096):
        x = torch.randn(rows, 12 * 86, generator=g) * 0.3
        x[:, 4 * 86:] = 0.0
        yb, yd = fused.forward(x), dense.forward(x)
        assert torch.equal(yb, yd), rows
        assert torch.equal(yb[:, :48], actor.forward(x)) and torch.equal(yb[:, 48:], critic.forward(x))
        for net in (fused, dense):
            net._net.packed = None          # the raw nn.Linear weight path
        assert torch.equal(fused.forward(x), yb) and torch.equal(dense.forward(x), yd)
        for net in (fused, dense):
            net._net.packed = net._packed.data_ptr()
