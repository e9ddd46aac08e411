"""On-device policy forward: the reference's trained MLPs on the matrix cores.

The CTDE driver trains ``PPO("MlpPolicy", net_arch=dict(pi=[128, 128], vf=[128, 128]))`` on the
flattened (12, 86) observation (``simulator/CTDECattleHerder.py:106-127``) and rolls it out with
``model.predict(obs, deterministic=True)`` (203): actor MLP -> ``action_net`` -> ``np.clip`` to the
[-1, 1] action box.  ``DevicePolicy`` runs that forward for every env of a ``HerdBatch`` in one HIP
launch (``csrc/ch_policy.hip``, f32 MFMA), so a rollout never leaves the GPU.

Weights come from an SB3 model zip (``policy.pth`` read with ``torch.load(weights_only=True)``,
nothing unpickled), from a state dict, or are random-initialised with the same architecture.
"""
import ctypes
import io
import zipfile

from . import _lib as L

_ACTS = {"none": L.CH_ACT_NONE, "tanh": L.CH_ACT_TANH, "relu": L.CH_ACT_RELU}


def load_sb3_state_dict(path):
    """``policy.pth`` of an SB3 model zip as a tensor dict (weights only; the zip's pickled
    ``data`` entry is never deserialised)."""
    import torch
    with zipfile.ZipFile(path) as z:
        return torch.load(io.BytesIO(z.read("policy.pth")), weights_only=True, map_location="cpu")


def _first(x):
    import numpy as np
    return np.asarray(x.cpu() if hasattr(x, "cpu") else x).reshape(-1)[0]


class DevicePolicy:
    """A dense MLP (1-4 layers, widths <= 256) evaluated by ``ch_mlp_forward``.

    ``layers``: list of (weight [out, in], bias [out] or None) tensors in ``nn.Linear`` layout (device float32
    contiguous tensors are used in place, so a torch optimizer updating them updates this policy);
    ``hidden_act`` after every layer but the last; ``clip`` = (lo, hi) or None on the output.

    The kernel reads the weights from a packed copy in its operand layout (biases are read in place).
    ``cache_packed=False`` (default) re-packs before every forward and collection, so any update of the weights
    -- ``optimizer.step()``, ``param.data.copy_()``, a Polyak average through ``.data`` -- is seen.
    ``cache_packed=True`` re-packs only when a weight tensor's version counter moves (``optimizer.step()`` and
    other in-place ops on the tensors themselves bump it; writes through ``.data`` or another alias do not): for
    frozen weights, e.g. rolling out a trained model; call ``pack()`` after any other update."""

    def __init__(self, layers, hidden_act="tanh", clip=None, device=None, splits=None, cache_packed=False):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("DevicePolicy needs a ROCm GPU; there is no CPU fallback")
        if not 1 <= len(layers) <= 4:
            raise ValueError("1..4 layers")
        self.torch = torch
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.weights, self.biases = [], []
        dims = [int(layers[0][0].shape[1])]
        for w, b in layers:
            w = torch.as_tensor(w, dtype=torch.float32).to(self.device).contiguous()
            if w.shape[1] != dims[-1] or w.shape[0] > 256:
                raise ValueError(f"layer shape {tuple(w.shape)} does not chain (widths <= 256)")
            self.weights.append(w)
            self.biases.append(None if b is None else torch.as_tensor(b, dtype=torch.float32).to(self.device).contiguous())
            dims.append(int(w.shape[0]))
        self.dims = dims
        self.hidden_act = hidden_act
        self.clip = clip
        net = L.ChMlp()
        net.n_layers = len(layers)
        for i, d in enumerate(dims):
            net.dims[i] = d
        for i in range(len(layers)):
            net.weight[i] = self.weights[i].data_ptr()
            net.bias[i] = self.biases[i].data_ptr() if self.biases[i] is not None else None
        net.hidden_act = _ACTS[hidden_act]
        net.clip = 1 if clip is not None else 0
        net.lo, net.hi = (clip if clip is not None else (0.0, 0.0))
        # block-diagonal layers {layer: (split_out, split_in)}: the kernel skips the zero blocks (ch_mlp.split_*)
        for i, (so, si) in (splits or {}).items():
            net.split_out[i], net.split_in[i] = int(so), int(si)
        self.splits = dict(splits or {})
        self._net = net
        # the weights in the kernel's operand layout (ch_mlp_pack): the forward reads this copy (and the biases in
        # place); re-packed before every forward, or with cache_packed only when a weight tensor's version moved
        self.cache_packed = bool(cache_packed)
        n = L.lib().ch_mlp_packed_size(ctypes.byref(net))
        self._packed = torch.empty(max(int(n), 4), dtype=torch.float32, device=self.device)
        self._packed_at = None
        net.packed = self._packed.data_ptr()

    def _versions(self):
        return tuple(w._version for w in self.weights)

    def pack(self):
        """Re-pack the weights now (on the current stream)."""
        L.check(L.lib().ch_mlp_pack(ctypes.byref(self._net), ctypes.c_void_p(self._packed.data_ptr()), self._stream()))
        self._packed_at = self._versions()

    def _ensure_packed(self):
        if not self.cache_packed or self._packed_at != self._versions():
            self.pack()

    # ---- constructors for the reference's models ------------------------------------------------
    @classmethod
    def sb3_actor(cls, state_dict, device=None, clip=True, cache_packed=False):
        """Deterministic SB3 ActorCriticPolicy action: policy_net (tanh) -> action_net, clipped to [-1, 1]
        (``clip=False``: the Gaussian mean, for stochastic rollouts, cattleherd.rollout)."""
        sd = state_dict
        layers = [(sd["mlp_extractor.policy_net.0.weight"], sd["mlp_extractor.policy_net.0.bias"]),
                  (sd["mlp_extractor.policy_net.2.weight"], sd["mlp_extractor.policy_net.2.bias"]),
                  (sd["action_net.weight"], sd["action_net.bias"])]
        return cls(layers, "tanh", (-1.0, 1.0) if clip else None, device, cache_packed=cache_packed)

    @classmethod
    def sb3_critic(cls, state_dict, device=None, cache_packed=False):
        """SB3 ActorCriticPolicy.predict_values: value_net on the tanh value MLP."""
        sd = state_dict
        layers = [(sd["mlp_extractor.value_net.0.weight"], sd["mlp_extractor.value_net.0.bias"]),
                  (sd["mlp_extractor.value_net.2.weight"], sd["mlp_extractor.value_net.2.bias"]),
                  (sd["value_net.weight"], sd["value_net.bias"])]
        return cls(layers, "tanh", None, device, cache_packed=cache_packed)

    @classmethod
    def rllib_policy(cls, weights, device=None, cache_packed=False):
        """The DTDE driver's RLlib PPO policy (``DTDECattleHerder.py:62-97``; the trained weights
        ``simulator/policy_weights.pkl`` = ``algo.get_weights()[policy]``, ``simulator/test.py:19-30``): the actor
        encoder Linear(86, 256) tanh Linear(256, 256) tanh, then ``pi`` Linear(256, 2A) = DiagGaussian (mean, log_std).
        The log_std half's clamp to [-20, 20] (``pi.log_std_clip_param_const``) is applied where the rollout reads it
        (``k_marl_store``); ``weights``: name -> array, RLlib's own key names."""
        w = weights
        layers = [(w["encoder.actor_encoder.net.mlp.0.weight"], w["encoder.actor_encoder.net.mlp.0.bias"]),
                  (w["encoder.actor_encoder.net.mlp.2.weight"], w["encoder.actor_encoder.net.mlp.2.bias"]),
                  (w["pi.net.mlp.0.weight"], w["pi.net.mlp.0.bias"])]
        clip = w.get("pi.log_std_clip_param_const")
        if clip is not None and abs(float(_first(clip)) - 20.0) > 0:
            raise ValueError("k_marl_store clamps log_std to RLlib's default 20; these weights carry "
                             f"log_std_clip_param {float(_first(clip))}")
        return cls(layers, "tanh", None, device, cache_packed=cache_packed)

    @classmethod
    def rllib_value(cls, weights, device=None, cache_packed=False):
        """The RLlib PPO value branch: critic encoder (the actor's shape, its own weights: vf_share_layers False)
        and ``vf`` Linear(256, 1)."""
        w = weights
        layers = [(w["encoder.critic_encoder.net.mlp.0.weight"], w["encoder.critic_encoder.net.mlp.0.bias"]),
                  (w["encoder.critic_encoder.net.mlp.2.weight"], w["encoder.critic_encoder.net.mlp.2.bias"]),
                  (w["vf.net.mlp.0.weight"], w["vf.net.mlp.0.bias"])]
        return cls(layers, "tanh", None, device, cache_packed=cache_packed)

    @classmethod
    def sb3_actor_critic(cls, state_dict, device=None):
        """SB3 ActorCriticPolicy's two MLPs as one net with both heads (output [mean (A), value]): layer 1
        stacked (policy_net.0 over value_net.0: the observation is read once), layers 2 and 3 block-diagonal.
        Every output is the same f32 MFMA fma chain as the separate nets' (the other head's blocks add +-0),
        so the mean and the value are bit-identical to sb3_actor(clip=False) and sb3_critic."""
        import torch
        sd = {k: torch.as_tensor(v, dtype=torch.float32) for k, v in state_dict.items()}
        aw = [sd["mlp_extractor.policy_net.0.weight"], sd["mlp_extractor.policy_net.2.weight"], sd["action_net.weight"]]
        ab = [sd["mlp_extractor.policy_net.0.bias"], sd["mlp_extractor.policy_net.2.bias"], sd["action_net.bias"]]
        cw = [sd["mlp_extractor.value_net.0.weight"], sd["mlp_extractor.value_net.2.weight"], sd["value_net.weight"]]
        cb = [sd["mlp_extractor.value_net.0.bias"], sd["mlp_extractor.value_net.2.bias"], sd["value_net.bias"]]
        layers = [(torch.cat([aw[0], cw[0]], 0), torch.cat([ab[0], cb[0]], 0))]
        for i in (1, 2):
            layers.append((torch.block_diag(aw[i], cw[i]), torch.cat([ab[i], cb[i]], 0)))
        splits = {i: (int(aw[i].shape[0]), int(aw[i].shape[1])) for i in (1, 2)}
        net = cls(layers, "tanh", None, device, splits=splits)
        net.heads = (int(aw[2].shape[0]), int(cw[2].shape[0]))
        return net

    @classmethod
    def fuse(cls, actor, critic):
        """The same packing from two DevicePolicy MLPs of equal depth (e.g. random-initialised ones)."""
        import torch
        if len(actor.weights) != len(critic.weights) or actor.hidden_act != critic.hidden_act:
            raise ValueError("actor and critic must have the same depth and activation")
        layers = []
        for i, (aw, ab, cw, cb) in enumerate(zip(actor.weights, actor.biases, critic.weights, critic.biases)):
            w = torch.cat([aw, cw], 0) if i == 0 else torch.block_diag(aw, cw)
            z = lambda w_, b_: b_ if b_ is not None else torch.zeros(w_.shape[0], device=w_.device)  # noqa: E731
            layers.append((w, torch.cat([z(aw, ab), z(cw, cb)], 0)))
        splits = {i: (int(actor.weights[i].shape[0]), int(actor.weights[i].shape[1])) for i in range(1, len(layers))}
        net = cls(layers, actor.hidden_act, None, actor.device, splits=splits)
        net.heads = (actor.dims[-1], critic.dims[-1])
        return net

    @staticmethod
    def random_layers(dims, seed=0):
        """nn.Linear default initialisation (uniform +-1/sqrt(fan_in)) for the given widths."""
        import torch
        g = torch.Generator().manual_seed(seed)
        out = []
        for i in range(len(dims) - 1):
            bound = 1.0 / dims[i] ** 0.5
            w = (torch.rand(dims[i + 1], dims[i], generator=g) * 2 - 1) * bound
            b = (torch.rand(dims[i + 1], generator=g) * 2 - 1) * bound
            out.append((w, b))
        return out

    # ---- forward ---------------------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def forward(self, x, out=None, row_mask=None):
        """y[rows, dims[-1]] = MLP(x[rows, dims[0]]) on the device (x float32, contiguous).  ``row_mask``
        (uint8/bool [rows] device tensor): only the selected rows are computed and written
        (ch_mlp_forward_masked)."""
        torch = self.torch
        self._ensure_packed()
        x = x.to(device=self.device, dtype=torch.float32).contiguous()
        rows = x.numel() // self.dims[0]
        if x.numel() != rows * self.dims[0]:
            raise ValueError(f"input has {x.numel()} floats, not a multiple of {self.dims[0]}")
        if out is None:
            out = torch.empty((rows, self.dims[-1]), dtype=torch.float32, device=self.device)
        if row_mask is not None:
            m = row_mask.to(device=self.device, dtype=torch.uint8).contiguous()
            if m.numel() != rows:
                raise ValueError(f"row_mask has {m.numel()} entries, not {rows}")
            self._mask_keep = m
            L.check(L.lib().ch_mlp_forward_masked(ctypes.byref(self._net), ctypes.c_void_p(x.data_ptr()), rows,
                                                  ctypes.c_void_p(m.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                                  self._stream()))
            return out
        L.check(L.lib().ch_mlp_forward(ctypes.byref(self._net), ctypes.c_void_p(x.data_ptr()), rows,
                                       ctypes.c_void_p(out.data_ptr()), self._stream()))
        return out

    def forward_batch(self, batch, out=None):
        """The forward on a HerdBatch's current observations (one row per env for CTDE, per agent for
        MARL), skipping the input columns past each env's NUM_DRONES."""
        torch = self.torch
        self._ensure_packed()
        rows = batch.n_envs if batch.mode == L.CH_MODE_CTDE else batch.n_envs * batch.num_drones
        if out is None:
            out = torch.empty((rows, self.dims[-1]), dtype=torch.float32, device=self.device)
        L.check(L.lib().ch_policy_forward(batch.handle, ctypes.byref(self._net), ctypes.c_void_p(batch.obs.data_ptr()),
                                          ctypes.c_void_p(out.data_ptr()), self._stream()), batch.handle)
        return out

    def act(self, batch, out=None):
        """Deterministic actions [E, N, 4] for the batch's observations (SB3 predict semantics: the
        first NUM_DRONES rows of the (12, 4) action; for MARL the first 4 of each agent's outputs)."""
        y = self.forward_batch(batch, out)
        n = batch.num_drones
        if batch.mode == L.CH_MODE_CTDE:
            return y.view(batch.n_envs, -1, 4)[:, :n, :]
        return y.view(batch.n_envs, n, -1)[:, :, :4]

    def reference(self, x):
        """Plain torch float32 forward of the same network (test oracle for the MFMA kernel)."""
        torch = self.torch
        h = x.to(device=self.device, dtype=torch.float32).reshape(-1, self.dims[0])
        for i, (w, b) in enumerate(zip(self.weights, self.biases)):
            h = h @ w.t()
            if b is not None:
                h = h + b
            if i < len(self.weights) - 1:
                h = {"tanh": torch.tanh, "relu": torch.relu, "none": lambda t: t}[self.hidden_act](h)
        if self.clip is not None:
            h = h.clamp(self.clip[0], self.clip[1])
        return h
