"""GPU test of the DTDE (RLlib) per-agent rollout collection (cattleherd.rollout.DeviceMarlRolloutBuffer,
ch_marl_rollout_collect) at configs[4]'s size, 4096 envs x (4 drones, 32 cattle), against plain torch / NumPy
restatements of RLlib PPO's sampling and GAE (RLlib is not installed: parity unpinned to its source; the
reference's setup is DTDECattleHerder.py:62-97 with one shared policy, the wrapper's drop-out and "__all__" are
rllib_envs/marl_wrapper.py:77-119) and a replay of the stored actions on a twin batch.

Tolerances: log-probabilities 1e-5 relative (float32 sums in another order than torch's), values 1e-5 (MFMA vs
torch matmul), the observations, rewards, flags and masks of the replay exact, GAE 2e-6 against the float32
recursion fed with the buffer's own rewards and values."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def gae_marl_numpy(rew, val, mask, term, last_v, gamma, lam):
    """Per-agent GAE in float32: a trajectory ends where the agent terminates; masked rows are 0."""
    T = rew.shape[0]
    g, gl = np.float32(gamma), np.float32(np.float64(gamma) * np.float64(lam))
    adv = np.zeros_like(rew)
    last = np.zeros_like(rew[0])
    nv = last_v.astype(np.float32).copy()
    for t in reversed(range(T)):
        m = mask[t] != 0
        nnt = np.where(term[t] != 0, np.float32(0), np.float32(1)).astype(np.float32)
        delta = (rew[t] + (g * nv) * nnt) - val[t]
        cur = delta + (gl * nnt) * last
        adv[t] = np.where(m, cur, np.float32(0))
        last = np.where(m, cur, np.float32(0)).astype(np.float32)
        nv = np.where(m, val[t], np.float32(0)).astype(np.float32)
    return adv, np.where(mask != 0, adv + val, np.float32(0)).astype(np.float32)


def _make(E, n, m, near):
    from cattleherd.env import HerdBatch
    b = HerdBatch(E, n, m, mode="marl", curriculum_level=2, min_drones=n, max_drones=n)
    b.reset()
    s = b.get_state()
    # the `near` envs start with their drone centroid 0.45 m from the herd centroid: at level 2 (approach_min 0.6,
    # curriculum_learning.py) every agent terminates and the env ends.  Half of them are n + 2 successes short of level
    # 3 (approach_min 0.3, 100 successes): env.step's n reward calls and the wrapper's reward call for agent 0 count
    # n + 1 (MARLCattleAviary._computeReward counts a success per call), agent 0's terminated call is still at level 2,
    # agent 1's reward call moves the env to level 3 -- agent 0 alone drops out (marl_wrapper.py:104-113)
    c = s["cow_pos"].mean(1)
    for k in range(n):
        s["drone_pos"][near, k, 0] = c[near, 0] + 0.5 * (k - (n - 1) / 2)
        s["drone_pos"][near, k, 1] = c[near, 1] + 0.45
    tally = s["tally"].copy()
    tally[near & (np.arange(E) % 2 == 0)] = 100 - n - 2
    b.set_state({"drone_pos": s["drone_pos"], "tally": tally})
    return b


GOLD = "tests/golden/policy_marl_rllib.npz"


def _trained():
    """The reference's trained RLlib weights (simulator/policy_weights.pkl, via tests/golden/make_policy_marl_golden)."""
    import os
    from cattleherd.policy import DevicePolicy
    d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), GOLD))
    w = {k.replace("__", "."): d[k] for k in d.files if "__" in k}
    return DevicePolicy.rllib_policy(w), DevicePolicy.rllib_value(w)


def _log_std(out, A=4):
    """RLlib's MLP head clamps the DiagGaussian log_std half to [-20, 20] (log_std_clip_param)."""
    return out[..., A:].clamp(-20.0, 20.0)


@pytest.mark.parametrize("weights", ["random", "trained"])
def test_marl_rollout_matches_rllib_semantics_configs4(weights):
    import torch
    from cattleherd.policy import DevicePolicy
    from cattleherd.rollout import DeviceMarlRolloutBuffer
    E, n, m, T = 4096, 4, 32, 16
    rows = E * n
    near = np.arange(E) % 3 == 0
    b = _make(E, n, m, near)
    if weights == "trained":
        policy, value = _trained()
    else:
        policy = DevicePolicy(DevicePolicy.random_layers([86, 256, 256, 8], seed=1), "tanh", None)
        value = DevicePolicy(DevicePolicy.random_layers([86, 256, 256, 1], seed=2), "tanh", None)
    rb = DeviceMarlRolloutBuffer(b, T)
    rb.collect(policy, value, seed=11)
    torch.cuda.synchronize()
    mask = rb.agent_mask.cpu().numpy()
    mb = torch.from_numpy(mask != 0).to(b.device)
    assert mask[0].all()
    # 1. log-probabilities and values of the stored samples under the torch forward, on the live rows
    out = policy.reference(rb.obs.view(T * rows, 86)).view(T, rows, 8)
    mean, log_std = out[..., :4], _log_std(out)
    std = torch.exp(log_std)
    want_lp = torch.distributions.Normal(mean, std).log_prob(rb.actions).sum(-1)
    assert torch.allclose(rb.log_probs[mb], want_lp[mb], rtol=1e-5, atol=1e-4)
    want_v = value.reference(rb.obs.view(T * rows, 86)).view(T, rows)
    assert torch.allclose(rb.values[mb], want_v[mb], rtol=1e-5, atol=1e-5)
    eps = ((rb.actions - mean) / std)[mb]
    assert abs(float(eps.mean())) < 0.02 and abs(float(eps.std()) - 1.0) < 0.02   # standard normal noise
    off = ~mb
    for t_ in (rb.log_probs, rb.values, rb.rewards, rb.advantages, rb.returns):
        assert float(t_[off].abs().max()) == 0.0 if off.any() else True
    # 2. the same rollout replayed on a twin batch with the stored actions, clipped, 0 for agents not live
    b2 = _make(E, n, m, near)
    obs = rb.obs.cpu()
    for t in range(T):
        assert torch.equal(b2.obs.view(rows, 86).cpu(), obs[t]), t
        a = (rb.actions[t].clamp(-1.0, 1.0) * mb[t, :, None]).view(E, n, 4)
        _, r, te, tr = b2.step(a, autoreset=True, terminal_obs=False)
        mt = mask[t] != 0
        assert np.array_equal(rb.rewards[t].cpu().numpy()[mt], r.view(-1).cpu().numpy()[mt], equal_nan=True), t
        assert np.array_equal(rb.terminated[t].cpu().numpy()[mt], te.view(-1).cpu().numpy()[mt]), t
        assert np.array_equal(rb.truncated[t].cpu().numpy()[mt], tr.view(-1).cpu().numpy()[mt]), t
        if t + 1 < T:   # the next step's agents: the survivors, or the new episode's
            assert np.array_equal(mask[t + 1], b2.agent_active.view(-1).cpu().numpy()), t
    assert torch.allclose(rb.last_values, value.reference(b2.obs.view(rows, 86))[:, 0], rtol=1e-5, atol=1e-5)
    # coverage: episodes ended (every agent terminated, env reset) and single agents dropped out
    term = rb.terminated.cpu().numpy()
    ended_env = term.reshape(T, E, n).all(axis=2) & mask.reshape(T, E, n).all(axis=2)
    dropped = (mask[:-1] != 0) & (mask[1:] == 0)
    assert ended_env.any() and dropped.any()
    # 3. GAE against the float32 recursion from the buffer's own rewards, values and the device's last values
    adv, ret = gae_marl_numpy(rb.rewards.cpu().numpy(), rb.values.cpu().numpy(), mask, term,
                              rb.last_values.cpu().numpy(), 0.99, 1.0)
    assert np.allclose(rb.advantages.cpu().numpy(), adv, rtol=2e-6, atol=2e-6, equal_nan=True)
    assert np.allclose(rb.returns.cpu().numpy(), ret, rtol=2e-6, atol=2e-6, equal_nan=True)
    b.close()
    b2.close()


def test_marl_rollout_gae_lambda_and_cpu_restatement_agree_on_a_small_case():
    """gamma / lambda other than RLlib's defaults reach the device recursion (E = 64, 3 drones x 8 cattle)."""
    import torch
    from cattleherd.policy import DevicePolicy
    from cattleherd.rollout import DeviceMarlRolloutBuffer
    E, n, m, T = 64, 3, 8, 9
    b = _make(E, n, m, np.arange(E) % 2 == 0)
    policy = DevicePolicy(DevicePolicy.random_layers([86, 64, 8], seed=3), "tanh", None)
    value = DevicePolicy(DevicePolicy.random_layers([86, 64, 1], seed=4), "tanh", None)
    rb = DeviceMarlRolloutBuffer(b, T, gamma=0.97, gae_lambda=0.9)
    rb.collect(policy, value, seed=2)
    torch.cuda.synchronize()
    mask, term = rb.agent_mask.cpu().numpy(), rb.terminated.cpu().numpy()
    adv, ret = gae_marl_numpy(rb.rewards.cpu().numpy(), rb.values.cpu().numpy(), mask, term,
                              rb.last_values.cpu().numpy(), 0.97, 0.9)
    assert np.allclose(rb.advantages.cpu().numpy(), adv, rtol=2e-6, atol=2e-6, equal_nan=True)
    assert np.allclose(rb.returns.cpu().numpy(), ret, rtol=2e-6, atol=2e-6, equal_nan=True)
    assert (term != 0).any()
    b.close()


def test_marl_rollout_clamps_log_std_like_rllib():
    """A policy whose log_std outputs leave [-20, 20]: the samples and log-probabilities use the clamped values (RLlib's
    MLP head, log_std_clip_param 20; the trained weights carry pi.log_std_clip_param_const = 20)."""
    import torch
    from cattleherd.policy import DevicePolicy
    from cattleherd.rollout import DeviceMarlRolloutBuffer
    E, n, m, T = 64, 3, 8, 3
    b = _make(E, n, m, np.zeros(E, bool))
    w = torch.zeros(8, 86)   # outputs = the bias exactly, on the device and in torch
    bias = torch.tensor([0.1, -0.2, 0.3, 0.0, 30.0, -30.0, 25.0, -1.0])
    policy = DevicePolicy([(w, bias)], "tanh", None)
    value = DevicePolicy(DevicePolicy.random_layers([86, 16, 1], seed=5), "tanh", None)
    rb = DeviceMarlRolloutBuffer(b, T)
    rb.collect(policy, value, seed=3)
    torch.cuda.synchronize()
    mb = rb.agent_mask != 0
    out = policy.reference(rb.obs.view(T * E * n, 86)).view(T, E * n, 8)
    mean, std = out[..., :4], torch.exp(_log_std(out))
    eps = (rb.actions.double() - mean) / std
    assert float(eps[mb][:, [0, 2]].abs().max()) < 7.0   # the e^20 columns: unclamped e^30 / e^25 would give e^10 / e^5 x eps
    want_lp = torch.distributions.Normal(mean, std).log_prob(rb.actions.double()).sum(-1)
    assert torch.allclose(rb.log_probs[mb].double(), want_lp[mb], rtol=1e-5, atol=1e-3)
    b.close()
