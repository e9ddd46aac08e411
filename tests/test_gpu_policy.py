"""On-device policy forward (csrc/ch_policy.hip) against torch.

Tolerances: the kernel multiplies in f32 on the matrix cores (each output a k-ordered f32 fma
chain); torch's CPU/GPU GEMMs sum in other orders.  Outputs are compared with an fp64 torch
forward of the same weights at atol 2e-5 + rtol 2e-5 (f32 rounding over K <= 1032 terms of
|w x| ~ 1e-2), and with the reference model's own fp32 outputs (golden file) at the same bar.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = "tests/golden/policy_ctde_v16_6.npz"


def _sd(d):
    import torch
    return {k.replace("__", "."): torch.tensor(d[k]) for k in d.files if "__" in k}


def _ref64(pol, x):
    import torch
    h = x.double().cpu().reshape(-1, pol.dims[0])
    for i, (w, b) in enumerate(zip(pol.weights, pol.biases)):
        h = h @ w.double().cpu().t()
        if b is not None:
            h = h + b.double().cpu()
        if i < len(pol.weights) - 1:
            h = torch.tanh(h) if pol.hidden_act == "tanh" else (torch.relu(h) if pol.hidden_act == "relu" else h)
    if pol.clip is not None:
        h = h.clamp(*pol.clip)
    return h


def _close(a, b, tol=2e-5):
    a = a.double().cpu()
    b = b.double().cpu()
    err = ((a - b).abs() - tol * b.abs()).max().item()
    return err <= tol, err


def test_sb3_actor_and_critic_match_reference_model():
    """model-v16-6 (the reference's trained CTDE PPO policy): deterministic actions and values."""
    import os
    import torch
    from cattleherd.policy import DevicePolicy
    d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), GOLD))
    sd = _sd(d)
    actor, critic = DevicePolicy.sb3_actor(sd), DevicePolicy.sb3_critic(sd)
    x = torch.tensor(d["obs"]).reshape(len(d["obs"]), -1)
    a = actor.forward(x)
    v = critic.forward(x)
    torch.cuda.synchronize()
    ok, err = _close(a, torch.tensor(d["actions"]))
    assert ok, err
    ok, err = _close(v[:, 0], torch.tensor(d["values"]))
    assert ok, err
    assert (a.abs() <= 1).all()


def test_rllib_policy_and_value_match_reference_weights():
    """The reference's trained RLlib PPO weights (simulator/policy_weights.pkl, read data-only by
    tests/golden/make_policy_marl_golden.py): pi logits (mean, log_std) and values on oracle MARL observations, against
    the fp32 torch outputs in the fixture and an fp64 forward, at 2e-5."""
    import os
    import torch
    from cattleherd.policy import DevicePolicy
    d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "tests/golden/policy_marl_rllib.npz"))
    w = {k.replace("__", "."): d[k] for k in d.files if "__" in k}
    pol, val = DevicePolicy.rllib_policy(w), DevicePolicy.rllib_value(w)
    assert pol.dims == [86, 256, 256, 8] and val.dims == [86, 256, 256, 1]
    x = torch.tensor(d["obs"])
    lg = pol.forward(x)
    v = val.forward(x)
    torch.cuda.synchronize()
    assert float(lg[:, 4:].abs().max()) < 20.0    # inside RLlib's log_std clamp: the head output is the logits
    ok, err = _close(lg, torch.tensor(d["logits"]))
    assert ok, err
    ok, err = _close(v[:, 0], torch.tensor(d["values"]))
    assert ok, err
    ok, err = _close(lg, _ref64(pol, x))
    assert ok, err


@pytest.mark.parametrize("dims,act,rows", [((1032, 128, 128, 48), "tanh", 4096), ((86, 256, 256, 8), "tanh", 4095),
                                           ((50, 16, 3), "relu", 17), ((1032, 128, 128, 1), "tanh", 1),
                                           ((7, 200, 33, 250, 5), "none", 100)])
def test_mlp_forward_vs_fp64(dims, act, rows):
    import torch
    from cattleherd.policy import DevicePolicy
    pol = DevicePolicy(DevicePolicy.random_layers(dims, seed=len(dims) + rows), act,
                       (-1.0, 1.0) if dims[-1] == 48 else None)
    g = torch.Generator().manual_seed(rows)
    x = torch.randn(rows, dims[0], generator=g)
    y = pol.forward(x)
    torch.cuda.synchronize()
    assert y.shape == (rows, dims[-1])
    ok, err = _close(y, _ref64(pol, x))
    assert ok, err


@pytest.mark.parametrize("mode,n,m", [("ctde", 4, 16), ("marl", 4, 16), ("ctde", 6, 8)])
def test_policy_forward_on_batch_skips_dead_rows_exactly(mode, n, m):
    """ch_policy_forward multiplies only the live part of each observation; the result equals the
    full-width forward of the same buffer (the skipped products are 0 * w)."""
    import torch
    from cattleherd.env import HerdBatch
    from cattleherd.policy import DevicePolicy
    b = HerdBatch(1000, n, m, mode=mode, min_drones=2, max_drones=n)
    dims = (12 * 86, 128, 128, 48) if mode == "ctde" else (86, 256, 256, 8)
    pol = DevicePolicy(DevicePolicy.random_layers(dims, seed=3), "tanh", (-1.0, 1.0))
    b.reset()
    for t in range(30):
        a = pol.act(b)
        full = pol.forward(b.obs)
        part = pol.forward_batch(b)
        torch.cuda.synchronize()
        assert torch.equal(part + 0.0, full + 0.0), t
        assert a.shape == (1000, n, 4)
        b.step(a, autoreset=True)
    torch.cuda.synchronize()
    ok, err = _close(pol.forward_batch(b), _ref64(pol, b.obs))
    assert ok, err
    b.close()


def test_policy_rollout_matches_host_policy_loop():
    """A device-policy rollout equals stepping the same batch with actions from the torch forward of
    each step's observation (to the forward's tolerance; actions are compared, the env runs on)."""
    import os
    import torch
    from cattleherd.env import HerdBatch
    from cattleherd.policy import DevicePolicy
    d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), GOLD))
    actor = DevicePolicy.sb3_actor(_sd(d))
    b = HerdBatch(512, 4, 16)
    b.reset()
    worst = 0.0
    for t in range(60):
        a = actor.act(b).contiguous()
        ref = actor.reference(b.obs).view(512, 12, 4)[:, :4]
        torch.cuda.synchronize()
        worst = max(worst, (a - ref).abs().max().item())
        b.step(a, autoreset=True)
    assert worst < 5e-5, worst
    b.close()


@pytest.mark.parametrize("dims,rows", [((1032, 128, 128, 1), 4096), ((86, 256, 256, 8), 1000)])
def test_masked_forward_computes_selected_rows_only(dims, rows):
    """ch_mlp_forward_masked: selected rows equal the unmasked forward bit for bit, the others keep what
    the output buffer held; an all-zero mask writes nothing (the rollout's terminal-value forward)."""
    import torch
    from cattleherd.policy import DevicePolicy
    pol = DevicePolicy(DevicePolicy.random_layers(dims, seed=5), "tanh", None)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(rows, dims[0], generator=g).cuda()
    full = pol.forward(x)
    mask = (torch.rand(rows, generator=g) < 0.02).to(torch.uint8).cuda()
    mask[3] = 1
    out = torch.full((rows, dims[-1]), 123.0, device="cuda")
    pol.forward(x, out, row_mask=mask)
    none = torch.full((rows, dims[-1]), -7.0, device="cuda")
    pol.forward(x, none, row_mask=torch.zeros(rows, dtype=torch.uint8, device="cuda"))
    torch.cuda.synchronize()
    sel = mask.bool()
    assert torch.equal(out[sel], full[sel])
    assert torch.all(out[~sel] == 123.0)
    assert torch.all(none == -7.0)


def test_weight_updates_are_seen_by_forward_and_collect():
    """DevicePolicy over nn.Linear parameters (used in place) sees every kind of weight update: an optimizer step
    and a write through ``.data`` (which does not move the tensor's version counter) -- forward() and a rollout
    collection both match the torch forward of the updated weights.  With cache_packed=True a ``.data`` write needs
    an explicit pack() (documented), after which it matches too."""
    import torch
    from cattleherd.env import HerdBatch
    from cattleherd.policy import DevicePolicy
    from cattleherd.rollout import DeviceRolloutBuffer
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)

    def mlp(out):
        return [torch.nn.Linear(1032, 128).to(dev), torch.nn.Linear(128, 128).to(dev), torch.nn.Linear(128, out).to(dev)]
    la, lc = mlp(16), mlp(1)
    actor = DevicePolicy([(l.weight, l.bias) for l in la], "tanh", None)
    critic = DevicePolicy([(l.weight, l.bias) for l in lc], "tanh", None)
    assert actor.weights[0] is la[0].weight
    x = torch.randn(300, 1032, device=dev) * 0.3
    y0 = actor.forward(x)
    assert torch.allclose(y0, actor.reference(x), rtol=1e-5, atol=1e-5)
    # 1. an optimizer step on the parameters
    opt = torch.optim.SGD([p for l in la for p in l.parameters()], lr=0.02)
    h = x
    for i, l in enumerate(la):
        h = l(h)
        if i < 2:
            h = torch.tanh(h)
    h.square().sum().backward()
    opt.step()
    y1 = actor.forward(x)
    assert not torch.allclose(y1, y0, rtol=1e-3, atol=1e-3)
    assert torch.allclose(y1, actor.reference(x), rtol=1e-4, atol=1e-4)
    # 2. a write through .data (no version bump)
    v0 = la[1].weight._version
    la[1].weight.data.copy_(torch.randn_like(la[1].weight) * 0.05)
    assert la[1].weight._version == v0
    y2 = actor.forward(x)
    assert not torch.allclose(y2, y1, rtol=1e-3, atol=1e-3)
    assert torch.allclose(y2, actor.reference(x), rtol=1e-4, atol=1e-4)
    # 3. a collection after a .data write into the critic: the stored values are V under the new weights
    E, T = 256, 6
    b = HerdBatch(E, 4, 16, mode="ctde")
    b.reset()
    rb = DeviceRolloutBuffer(b, T, act_dim=16)
    log_std = torch.full((16,), -1.0, device=dev)
    rb.collect(actor, critic, log_std, seed=3)
    lc[0].weight.data.mul_(1.5)
    rb.collect(actor, critic, log_std, seed=4)
    torch.cuda.synchronize()
    want = critic.reference(rb.obs.view(T * E, -1)).view(T, E)
    assert torch.allclose(rb.values, want, rtol=1e-5, atol=1e-5)
    # 4. cache_packed=True: packed once; a .data write is seen after pack()
    cached = DevicePolicy([(l.weight, l.bias) for l in la], "tanh", None, cache_packed=True)
    y3 = cached.forward(x)
    la[2].weight.data.mul_(-1.0)
    cached.pack()
    assert torch.allclose(cached.forward(x), cached.reference(x), rtol=1e-4, atol=1e-4)
    assert not torch.allclose(cached.forward(x), y3, rtol=1e-3, atol=1e-3)
    b.close()
