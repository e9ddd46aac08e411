"""The PPO update of the CTDE driver over a device rollout buffer: configs[2]'s training half, for the end-to-end
training rate (collection + update) beside the collection-only rate.

The driver trains ``PPO("MlpPolicy", learning_rate=3e-4, n_steps=2048, batch_size=64, n_epochs=10, gamma=0.99,
gae_lambda=0.95, clip_range=0.1, ent_coef=0.1, vf_coef=0.7, max_grad_norm=0.5, policy_kwargs=dict(log_std_init=-1,
ortho_init=False, net_arch=[dict(pi=[128, 128], vf=[128, 128])]))`` (``simulator/CTDECattleHerder.py:107-127``).
``SB3ActorCritic`` is that ActorCriticPolicy (flatten -> separate tanh MLPs -> ``action_net`` / ``value_net``, a free
``log_std``) with SB3's parameter names; ``device_nets()`` hands the rollout kernels the same storage, so every
optimizer step is seen by the next collection (``DevicePolicy`` re-packs before each forward).  ``PPOUpdate.train``
restates SB3 2.x ``PPO.train``: ``n_epochs`` passes over a fresh permutation of the buffer in minibatches of
``batch_size``, per-minibatch advantage normalisation, the clipped surrogate, MSE value loss, entropy bonus, Adam
(eps 1e-5, SB3's ActorCriticPolicy default), ``clip_grad_norm_``.  SB3 is not installed: parity unpinned to its
source (no logging statistics, and the permutation comes from torch's generator, not NumPy's).

With ``graph=True`` each run of ``steps_per_graph`` minibatch steps is one captured HIP graph (static index buffer,
capturable Adam): the update of a 64-row minibatch is ~60 small kernels, so launch overhead, not arithmetic, is
what an eager loop would measure.
"""
import math


def _torch():
    import torch
    return torch


class SB3ActorCritic:
    """SB3 ``ActorCriticPolicy`` for a flat Box observation: ``mlp_extractor.policy_net`` / ``value_net`` (Linear +
    Tanh, widths ``pi`` / ``vf``), ``action_net``, ``value_net``, ``log_std`` (initialised to ``log_std_init``;
    ``ortho_init=False``: torch's default Linear initialisation)."""

    def __init__(self, obs_dim=1032, act_dim=48, pi=(128, 128), vf=(128, 128), log_std_init=-1.0, device=None,
                 seed=0):
        torch = _torch()
        nn = torch.nn
        g = torch.manual_seed(seed)  # noqa: F841  (default nn.Linear init draws from the global generator)
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())

        def mlp(widths):
            layers, d = [], obs_dim
            for w in widths:
                layers += [nn.Linear(d, w), nn.Tanh()]
                d = w
            return nn.Sequential(*layers), d

        self.policy_net, dpi = mlp(pi)
        self.value_net_mlp, dvf = mlp(vf)
        self.action_net = nn.Linear(dpi, act_dim)
        self.value_net = nn.Linear(dvf, 1)
        self.log_std = nn.Parameter(torch.ones(act_dim) * log_std_init)
        self.modules = nn.ModuleList([self.policy_net, self.value_net_mlp, self.action_net, self.value_net]).to(dev)
        self.log_std.data = self.log_std.data.to(dev)
        self.device, self.obs_dim, self.act_dim = dev, obs_dim, act_dim

    def parameters(self):
        return list(self.modules.parameters()) + [self.log_std]

    def state_dict_sb3(self):
        """SB3's names -> the live tensors (no copies)."""
        sd = {}
        for i, m in enumerate(self.policy_net):
            if hasattr(m, "weight"):
                sd[f"mlp_extractor.policy_net.{i}.weight"], sd[f"mlp_extractor.policy_net.{i}.bias"] = m.weight, m.bias
        for i, m in enumerate(self.value_net_mlp):
            if hasattr(m, "weight"):
                sd[f"mlp_extractor.value_net.{i}.weight"], sd[f"mlp_extractor.value_net.{i}.bias"] = m.weight, m.bias
        sd["action_net.weight"], sd["action_net.bias"] = self.action_net.weight, self.action_net.bias
        sd["value_net.weight"], sd["value_net.bias"] = self.value_net.weight, self.value_net.bias
        sd["log_std"] = self.log_std
        return sd

    def device_nets(self):
        """(actor mean, critic) DevicePolicy over the same storage (``.data``: no autograd), and the log_std tensor."""
        from .policy import DevicePolicy
        sd = {k: v.data for k, v in self.state_dict_sb3().items()}
        return DevicePolicy.sb3_actor(sd, clip=False), DevicePolicy.sb3_critic(sd), self.log_std.data

    def evaluate_actions(self, obs, actions):
        """SB3 ``evaluate_actions`` with a DiagGaussian: values, summed log-probabilities, summed entropies."""
        torch = _torch()
        mean = self.action_net(self.policy_net(obs))
        values = self.value_net(self.value_net_mlp(obs))
        log_std = self.log_std.expand_as(mean)
        var = torch.exp(2.0 * log_std)
        log_prob = (-((actions - mean) ** 2) / (2.0 * var) - log_std - math.log(math.sqrt(2.0 * math.pi))).sum(-1)
        entropy = (0.5 + 0.5 * math.log(2.0 * math.pi) + log_std).sum(-1)
        return values.flatten(), log_prob, entropy


class PPOUpdate:
    """SB3 ``PPO.train`` over a ``DeviceRolloutBuffer`` (defaults: the CTDE driver's hyper-parameters)."""

    def __init__(self, model, learning_rate=3e-4, n_epochs=10, batch_size=64, clip_range=0.1, ent_coef=0.1,
                 vf_coef=0.7, max_grad_norm=0.5, normalize_advantage=True, graph=True, steps_per_graph=32, seed=0):
        torch = _torch()
        self.model = model
        self.n_epochs, self.batch_size = int(n_epochs), int(batch_size)
        self.clip_range, self.ent_coef, self.vf_coef = float(clip_range), float(ent_coef), float(vf_coef)
        self.max_grad_norm, self.normalize_advantage = float(max_grad_norm), bool(normalize_advantage)
        self.graph, self.steps_per_graph = bool(graph), int(steps_per_graph)
        self.opt = torch.optim.Adam(model.parameters(), lr=learning_rate, eps=1e-5, capturable=self.graph)
        self.gen = torch.Generator(device=model.device).manual_seed(seed)
        self._graphs = {}
        self.sgd_steps = 0

    def _loss(self, obs, actions, old_log_prob, advantages, returns):
        torch = _torch()
        values, log_prob, entropy = self.model.evaluate_actions(obs, actions)
        if self.normalize_advantage and advantages.shape[0] > 1:
            advantages = (advantages - advantages.mean()) / (advantages.std() + 1e-8)
        ratio = torch.exp(log_prob - old_log_prob)
        pl = -torch.min(advantages * ratio, advantages * torch.clamp(ratio, 1 - self.clip_range, 1 + self.clip_range)).mean()
        vl = torch.nn.functional.mse_loss(returns, values)
        return pl + self.ent_coef * (-torch.mean(entropy)) + self.vf_coef * vl

    def _sgd(self, data, idx):
        """One minibatch step: gather, loss, backward, clip, Adam (every op on the device, no host sync)."""
        torch = _torch()
        obs, act, lp, adv, ret = (t.index_select(0, idx) for t in data)
        loss = self._loss(obs, act, lp, adv, ret)
        self.opt.zero_grad(set_to_none=False)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.max_grad_norm)
        self.opt.step()
        return loss

    def _flat(self, rb):
        T, E = rb.T, rb.batch.n_envs
        n = T * E
        return (rb.obs.view(n, -1), rb.actions.view(n, -1), rb.log_probs.view(n), rb.advantages.view(n),
                rb.returns.view(n))

    def _graph_for(self, rb, data):
        """A captured run of steps_per_graph minibatch steps over `data`'s storage, reading indices from a static
        [steps_per_graph, batch_size] buffer."""
        torch = _torch()
        key = (id(rb), tuple(t.data_ptr() for t in data))
        g = self._graphs.get(key)
        if g is not None:
            return g
        k, bs = self.steps_per_graph, self.batch_size
        idx = torch.zeros((k, bs), dtype=torch.long, device=self.model.device)
        for p in self.model.parameters():      # gradients exist before capture (zero_grad keeps them)
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        # warm up the captured ops on a side stream (the graph recipe), then undo those steps: the warm-up must not
        # train the model
        saved = [p.detach().clone() for p in self.model.parameters()]
        saved_state = {id(p): {n: (v.clone() if torch.is_tensor(v) else v) for n, v in st.items()}
                       for p, st in self.opt.state.items()}
        s = torch.cuda.Stream(device=self.model.device)
        s.wait_stream(torch.cuda.current_stream(self.model.device))
        with torch.cuda.stream(s):
            for _ in range(2):
                self._sgd(data, idx[0])
        torch.cuda.current_stream(self.model.device).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for j in range(k):
                self._sgd(data, idx[j])
        with torch.no_grad():
            for p, v in zip(self.model.parameters(), saved):
                p.copy_(v)
            for p, st in self.opt.state.items():
                old = saved_state.get(id(p))
                for n, v in st.items():
                    if torch.is_tensor(v):
                        if old is None:
                            v.zero_()            # state the warm-up created: a fresh Adam (step 0, zero moments)
                        else:
                            v.copy_(old[n])
        g = (graph, idx)
        self._graphs[key] = g
        return g

    def train(self, rb):
        """n_epochs passes over the whole buffer; returns the number of minibatch steps taken."""
        torch = _torch()
        data = self._flat(rb)
        n = data[0].shape[0]
        bs = self.batch_size
        nb = (n + bs - 1) // bs
        steps = 0
        for _ in range(self.n_epochs):
            perm = torch.randperm(n, device=self.model.device, generator=self.gen)
            full = n // bs
            j = 0
            if self.graph and full >= self.steps_per_graph:
                graph, idx = self._graph_for(rb, data)
                k = self.steps_per_graph
                while j + k <= full:
                    idx.copy_(perm[j * bs:(j + k) * bs].view(k, bs))
                    graph.replay()
                    j += k
            while j < nb:     # the rest (and a last partial minibatch, as SB3's RolloutBuffer.get yields it)
                self._sgd(data, perm[j * bs:min((j + 1) * bs, n)])
                j += 1
            steps += nb
        self.sgd_steps += steps
        return steps
