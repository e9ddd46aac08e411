"""The PPO update over a device rollout buffer (cattleherd.ppo, configs[2]'s training half; the CTDE driver's
hyper-parameters, simulator/CTDECattleHerder.py:107-127).  SB3 is not installed, so its PPO.train is restated
(parity unpinned); these tests hold the restatement's pieces to torch.distributions and the HIP-graph path to the
eager one.

Tolerances: the graph replays the eager path's kernels on the same minibatches, so parameters agree to 1e-6
(Adam's division amplifies last-bit differences of the reductions if any); the log-probability and entropy equal
torch.distributions.Normal's at 1e-5."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _collect(E=64, T=8, seed=1):
    from cattleherd.env import HerdBatch
    from cattleherd.ppo import SB3ActorCritic
    from cattleherd.rollout import DeviceRolloutBuffer
    b = HerdBatch(E, 2, 8, mode="ctde", compat=False)
    b.reset()
    model = SB3ActorCritic(obs_dim=b.obs_rows * 86, act_dim=48, device=b.device, seed=0)
    actor, critic, log_std = model.device_nets()
    rb = DeviceRolloutBuffer(b, T, act_dim=48)
    rb.collect(actor, critic, log_std, seed=seed)
    return b, model, rb


def test_evaluate_actions_matches_torch_distributions():
    import torch
    b, model, rb = _collect()
    obs = rb.obs.view(-1, rb.obs.shape[-1])
    act = rb.actions.view(-1, 48)
    with torch.no_grad():
        v, lp, ent = model.evaluate_actions(obs, act)
        mean = model.action_net(model.policy_net(obs))
        dist = torch.distributions.Normal(mean, torch.exp(model.log_std).expand_as(mean))
        assert torch.allclose(lp, dist.log_prob(act).sum(-1), rtol=1e-5, atol=1e-4)
        assert torch.allclose(ent, dist.entropy().sum(-1), rtol=1e-5, atol=1e-5)
        # the buffer's log-probs and values came from the device forwards of the same weights
        assert torch.allclose(rb.log_probs.view(-1), lp, rtol=1e-4, atol=1e-3)
        assert torch.allclose(rb.values.view(-1), v, rtol=1e-4, atol=1e-4)
    b.close()


def test_graph_update_equals_eager_update():
    import torch
    from cattleherd.ppo import PPOUpdate, SB3ActorCritic
    b, model, rb = _collect()
    init = [p.detach().clone() for p in model.parameters()]
    results = []
    for graph in (False, True):
        m = SB3ActorCritic(obs_dim=b.obs_rows * 86, act_dim=48, device=b.device, seed=0)
        with torch.no_grad():
            for p, q in zip(m.parameters(), init):
                p.copy_(q)
        upd = PPOUpdate(m, batch_size=16, n_epochs=2, graph=graph, steps_per_graph=8, seed=5)
        steps = upd.train(rb)
        torch.cuda.synchronize()
        assert steps == 2 * (rb.obs.shape[0] * rb.obs.shape[1]) // 16
        results.append([p.detach().clone() for p in m.parameters()])
        if graph:
            assert upd._graphs, "the graph path was not taken"
    for a, g, p0 in zip(*results, init):
        assert torch.allclose(a, g, rtol=1e-6, atol=1e-6)
        assert not torch.equal(a, p0)   # the update moved every parameter
    b.close()


def test_update_weights_reach_the_next_collection():
    """device_nets() share storage with the torch parameters: after train() the next collection's values are the
    updated critic's."""
    import torch
    from cattleherd.ppo import PPOUpdate
    b, model, rb = _collect()
    upd = PPOUpdate(model, batch_size=64, n_epochs=1, graph=False)
    upd.train(rb)
    actor, critic, log_std = model.device_nets()
    rb.collect(actor, critic, log_std, seed=2)
    torch.cuda.synchronize()
    with torch.no_grad():
        v, _, _ = model.evaluate_actions(rb.obs.view(-1, rb.obs.shape[-1]), rb.actions.view(-1, 48))
    assert np.allclose(rb.values.view(-1).cpu().numpy(), v.cpu().numpy(), rtol=1e-4, atol=1e-4)
    b.close()
