"""On-device PPO rollout collection for the CTDE driver.

The reference trains with stable_baselines3 PPO (simulator/CTDECattleHerder.py:107-150: n_steps 2048,
gamma 0.99, gae_lambda 0.95, MlpPolicy with log_std_init -1).  Each of its rollout steps copies the
(n_envs, 12, 86) observations to the host, runs the policy, steps the SubprocVecEnv and appends to a numpy
RolloutBuffer.  ``DeviceRolloutBuffer.collect`` keeps all of it on the GPU: actor and critic forwards
(``ch_policy_forward``, f32 MFMA), the Gaussian sample / log-probability / buffer store
(``ch_rollout_store``), the env step (``ch_step``), the truncation bootstrap with V(terminal_observation)
and the episode starts (``ch_rollout_post``), and finally GAE (``ch_rollout_gae``).  The tensors then feed
a torch PPO update directly.

Semantics restated from SB3 2.7 (OnPolicyAlgorithm.collect_rollouts, RolloutBuffer,
DiagGaussianDistribution); SB3 is not installed here, so the restatement is "parity unpinned" to its
source.  The noise comes from Philox (seeded), not torch's generator.
"""
import ctypes

from . import _lib as L


class ChRollout(ctypes.Structure):
    _fields_ = [("n_steps", ctypes.c_int32), ("act_dim", ctypes.c_int32)] + \
        [(k, ctypes.c_void_p) for k in ("obs", "actions", "rewards", "episode_starts", "values", "log_probs",
                                        "advantages", "returns", "last_episode_starts")]


class ChRolloutIO(ctypes.Structure):
    _fields_ = [("step", ctypes.POINTER(L.ChStepIO))] + \
        [(k, ctypes.c_void_p) for k in ("mean", "value", "terminal_value", "env_actions")]


def _bind():
    lib = L.lib()
    vp, i32, u64, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64, ctypes.c_float
    P = ctypes.POINTER(ChRollout)
    lib.ch_rollout_store.argtypes = [vp, P, i32, vp, vp, vp, vp, u64, vp, vp]
    lib.ch_rollout_post.argtypes = [vp, P, i32, vp, vp, vp, vp, f32, vp]
    lib.ch_rollout_gae.argtypes = [vp, P, vp, f32, f32, vp]
    lib.ch_rollout_collect.argtypes = [vp, P, ctypes.POINTER(ChRolloutIO), ctypes.POINTER(L.ChMlp),
                                       ctypes.POINTER(L.ChMlp), vp, u64, f32, f32, i32, vp]
    for f in (lib.ch_rollout_store, lib.ch_rollout_post, lib.ch_rollout_gae, lib.ch_rollout_collect):
        f.restype = ctypes.c_int
    return lib


class DeviceRolloutBuffer:
    def __init__(self, batch, n_steps, act_dim=None, gamma=0.99, gae_lambda=0.95):
        if batch.mode != L.CH_MODE_CTDE:
            raise ValueError("the SB3 rollout buffer is for CTDE batches")
        torch = batch.torch
        self.batch, self.T, self.gamma, self.gae_lambda = batch, int(n_steps), float(gamma), float(gae_lambda)
        E, od = batch.n_envs, batch.obs_rows * 86
        self.act_dim = int(act_dim or batch.num_drones * 4)
        z = dict(dtype=torch.float32, device=batch.device)
        self.obs = torch.zeros((self.T, E, od), **z)
        self.actions = torch.zeros((self.T, E, self.act_dim), **z)
        for k in ("rewards", "episode_starts", "values", "log_probs", "advantages", "returns"):
            setattr(self, k, torch.zeros((self.T, E), **z))
        self.last_episode_starts = torch.ones(E, **z)          # SB3: _last_episode_starts = ones after reset
        self.env_actions = torch.zeros((E, batch.num_drones, 4), **z)
        self.value = torch.zeros((E, 1), **z)
        self.mean = torch.zeros((E, self.act_dim), **z)
        self.mean_fused = None   # [E, act_dim + 1]: a fused actor-critic's output (collect(critic=None))
        self.terminal_value = torch.zeros((E, 1), **z)
        rb = ChRollout()
        rb.n_steps, rb.act_dim = self.T, self.act_dim
        for k in ("obs", "actions", "rewards", "episode_starts", "values", "log_probs", "advantages", "returns",
                  "last_episode_starts"):
            setattr(rb, k, getattr(self, k).data_ptr())
        self._rb = rb
        self._lib = _bind()

    def collect(self, actor, critic, log_std, seed=0, bootstrap_truncated=True):
        """SB3 collect_rollouts for n_steps steps of every env, on the device, in one native call
        (ch_rollout_collect: the loop of collect_steps below runs in C++).  ``actor``: DevicePolicy of the
        action mean (no clip: SB3's action_net output), ``critic``: DevicePolicy of V, ``log_std``:
        float32 [act_dim] device tensor.  ``critic=None``: ``actor`` is a fused actor-critic
        (DevicePolicy.sb3_actor_critic / fuse, output [mean, value]) and one forward per step serves both."""
        b, lib = self.batch, self._lib
        torch = b.torch
        log_std = log_std.to(device=b.device, dtype=torch.float32).contiguous()
        for net in (actor, critic):
            if net is not None:
                net._ensure_packed()
        io = ChRolloutIO()
        io.step = ctypes.pointer(b._io)
        if critic is None:
            if actor.dims[-1] != self.act_dim + 1:
                raise ValueError(f"a fused actor-critic must output act_dim + 1 = {self.act_dim + 1} columns")
            if self.mean_fused is None:
                self.mean_fused = torch.zeros((b.n_envs, self.act_dim + 1), dtype=torch.float32, device=b.device)
                self.terminal_fused = torch.zeros((b.n_envs, self.act_dim + 1), dtype=torch.float32, device=b.device)
            io.mean, io.terminal_value = self.mean_fused.data_ptr(), self.terminal_fused.data_ptr()
        else:
            io.mean, io.value = self.mean.data_ptr(), self.value.data_ptr()
            io.terminal_value = self.terminal_value.data_ptr()
        io.env_actions = self.env_actions.data_ptr()
        keep = b._io.terminal_obs
        b._io.terminal_obs = b.terminal_obs.data_ptr()
        try:
            L.check(lib.ch_rollout_collect(b.handle, ctypes.byref(self._rb), ctypes.byref(io), ctypes.byref(actor._net),
                                           None if critic is None else ctypes.byref(critic._net), log_std.data_ptr(),
                                           int(seed), self.gamma, self.gae_lambda, int(bool(bootstrap_truncated)),
                                           b._stream()), b.handle)
        finally:
            b._io.terminal_obs = keep
        return self

    def collect_steps(self, actor, critic, log_std, seed=0, bootstrap_truncated=True):
        """The same collection driven from Python one kernel at a time (the reference loop the native
        call restates; kept for the parity test)."""
        b, lib, rb = self.batch, self._lib, ctypes.byref(self._rb)
        torch = b.torch
        log_std = log_std.to(device=b.device, dtype=torch.float32).contiguous()
        for t in range(self.T):
            actor.forward_batch(b, self.mean)
            critic.forward_batch(b, self.value)
            L.check(lib.ch_rollout_store(b.handle, rb, t, b.obs.data_ptr(), self.mean.data_ptr(), self.value.data_ptr(),
                                         log_std.data_ptr(), int(seed), self.env_actions.data_ptr(), b._stream()),
                    b.handle)
            b.step(self.env_actions, autoreset=True, terminal_obs=True)
            tv = None
            if bootstrap_truncated:
                # V(terminal obs) only for the envs that just reset (the only rows ch_rollout_post reads)
                critic.forward(b.terminal_obs.view(b.n_envs, -1), self.terminal_value, row_mask=b.reset_happened)
                tv = self.terminal_value.data_ptr()
            L.check(lib.ch_rollout_post(b.handle, rb, t, b.reward.data_ptr(), b.terminated.data_ptr(),
                                        b.truncated.data_ptr(), tv, self.gamma, b._stream()), b.handle)
        critic.forward_batch(b, self.value)
        L.check(lib.ch_rollout_gae(b.handle, rb, self.value.data_ptr(), self.gamma, self.gae_lambda, b._stream()),
                b.handle)
        return self


class ChMarlRollout(ctypes.Structure):
    _fields_ = [("n_steps", ctypes.c_int32), ("act_dim", ctypes.c_int32)] + \
        [(k, ctypes.c_void_p) for k in ("obs", "actions", "log_probs", "values", "rewards", "agent_mask", "terminated",
                                        "truncated", "advantages", "returns", "last_values")]


class ChMarlRolloutIO(ctypes.Structure):
    _fields_ = [("step", ctypes.POINTER(L.ChStepIO))] + \
        [(k, ctypes.c_void_p) for k in ("policy_out", "value_out", "env_actions")]


class DeviceMarlRolloutBuffer:
    """On-device rollout collection for the DTDE driver (SURVEY §8(f)2's RLlib half): RLlib PPO with one shared
    policy over every agent of every ``RLlibMultiAgentWrapper`` env (simulator/DTDECattleHerder.py:62-97:
    ``policies = {"shared_policy"}``, gamma 0.99; GAE lambda is RLlib PPO's default 1.0), the wrapper's agent
    drop-out and ``"__all__"`` (rllib_envs/marl_wrapper.py:77-119) handled per agent row.

    Rows are agents (``E * N``, row ``e * N + i`` = ``agent_i`` of env ``e``); every buffer is ``[T, rows, ...]``:
    ``obs`` (86 floats), ``actions`` (unclipped samples), ``log_probs``, ``values``, ``rewards``, ``agent_mask``
    (the agent was live at the step's start: its key was in the wrapper's dicts), ``terminated``, ``truncated``,
    ``advantages``, ``returns``; ``last_values`` = V(obs after the last step).  ``collect`` is one native call
    (ch_marl_rollout_collect): per step the policy and value forwards (f32 MFMA), the Gaussian sample /
    log-probability / store, ch_step with auto-reset; then GAE per agent (a trajectory ends where the agent
    terminates).  RLlib is not installed: its defaults are restated ("parity unpinned" to its source)."""

    def __init__(self, batch, n_steps, act_dim=4, gamma=0.99, gae_lambda=1.0):
        if batch.mode != L.CH_MODE_MARL:
            raise ValueError("the per-agent rollout buffer is for MARL batches")
        torch = batch.torch
        self.batch, self.T, self.gamma, self.gae_lambda = batch, int(n_steps), float(gamma), float(gae_lambda)
        self.act_dim = int(act_dim)
        self.rows = rows = batch.n_envs * batch.num_drones
        f32, u8 = dict(dtype=torch.float32, device=batch.device), dict(dtype=torch.uint8, device=batch.device)
        self.obs = torch.zeros((self.T, rows, 86), **f32)
        self.actions = torch.zeros((self.T, rows, self.act_dim), **f32)
        for k in ("log_probs", "values", "rewards", "advantages", "returns"):
            setattr(self, k, torch.zeros((self.T, rows), **f32))
        for k in ("agent_mask", "terminated", "truncated"):
            setattr(self, k, torch.zeros((self.T, rows), **u8))
        self.last_values = torch.zeros(rows, **f32)
        self.policy_out = torch.zeros((rows, 2 * self.act_dim), **f32)
        self.value_out = torch.zeros((rows, 1), **f32)
        self.env_actions = torch.zeros((batch.n_envs, batch.num_drones, 4), **f32)
        rb = ChMarlRollout()
        rb.n_steps, rb.act_dim = self.T, self.act_dim
        for k in ("obs", "actions", "log_probs", "values", "rewards", "agent_mask", "terminated", "truncated",
                  "advantages", "returns", "last_values"):
            setattr(rb, k, getattr(self, k).data_ptr())
        self._rb = rb
        lib = L.lib()
        vp = ctypes.c_void_p
        lib.ch_marl_rollout_collect.argtypes = [vp, ctypes.POINTER(ChMarlRollout), ctypes.POINTER(ChMarlRolloutIO),
                                                ctypes.POINTER(L.ChMlp), ctypes.POINTER(L.ChMlp), ctypes.c_uint64,
                                                ctypes.c_float, ctypes.c_float, vp]
        lib.ch_marl_rollout_collect.restype = ctypes.c_int
        self._lib = lib

    def collect(self, policy, value, seed=0):
        """RLlib PPO sampling for n_steps steps of every env and agent, on the device, in one native call.
        ``policy``: DevicePolicy 86 -> ... -> 2 * act_dim (mean, log_std: RLlib's DiagGaussian inputs), ``value``:
        DevicePolicy 86 -> ... -> 1 (RLlib PPO's separate value branch, vf_share_layers=False)."""
        b = self.batch
        for net in (policy, value):
            net._ensure_packed()
        io = ChMarlRolloutIO()
        io.step = ctypes.pointer(b._io)
        io.policy_out, io.value_out, io.env_actions = (self.policy_out.data_ptr(), self.value_out.data_ptr(),
                                                       self.env_actions.data_ptr())
        L.check(self._lib.ch_marl_rollout_collect(b.handle, ctypes.byref(self._rb), ctypes.byref(io),
                                                  ctypes.byref(policy._net), ctypes.byref(value._net), int(seed),
                                                  self.gamma, self.gae_lambda, b._stream()), b.handle)
        return self
