"""HerdBatch: E cattle-herding environments resident in HBM, stepped by one HIP launch per step.

This is the product-side host object over the C ABI (include/cattleherd.h).  It owns the device
buffers the kernels write (torch tensors, so a torch policy can read observations in place) and
exposes reset/step/get_state/set_state/metrics.  The Gymnasium, SB3-VecEnv and RLlib adapters in
``gym_pybullet_drones`` and ``cattleherd.vec_env`` are thin layers over it.

Reference: one ``CattleAviary`` (sb3_envs/CattleAviary.py) / ``MARLCattleAviary``
(rllib_envs/MARLCattleAviary.py) per OS process; here one HerdBatch holds all of a GPU's envs.
"""
import ctypes

import numpy as np

from . import _lib as L

DRONE_COMPS = 26   # ... pid_int_rpy[3], qlag[4] (the cached link frame, ch_config.link_lag)
CATTLE_COMPS = 4
PHYS_COMPS = 7   # last_clipped_action[4], DYN rpy_rates[3]
ENV_INTS = ("n", "step_counter", "step_counter_A", "has_prev", "level", "tally", "spawn_index", "active_mask",
            "episode", "step_index")


class HerdBatch:
    def __init__(self, n_envs, num_drones, num_cattle, mode="ctde", device=None, compat=True, precision="f64",
                 min_drones=None, max_drones=None, curriculum_level=None, seed=0x5EED, env_id_offset=0,
                 damping=0.04, torque_world=True, gyro=True, ctrl_freq=60, pyb_freq=240, spawn_table=None,
                 marl_wrapper=True, physics="pyb", eval_metrics=True, link_lag=True):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("HerdBatch needs a ROCm GPU (torch.cuda.is_available() is False); there is no CPU "
                               "fallback for the product path")
        self.torch = torch
        self.mode = {"ctde": L.CH_MODE_CTDE, "marl": L.CH_MODE_MARL}[mode] if isinstance(mode, str) else int(mode)
        dev_index = torch.cuda.current_device() if device is None else int(device)
        cfg = L.default_config(self.mode, num_drones, num_cattle)
        cfg.compat = int(bool(compat))
        cfg.precision = {"f64": L.CH_PREC_F64, "f32": L.CH_PREC_F32}[precision]
        cfg.min_drones = -1 if min_drones is None else int(min_drones)
        cfg.max_drones = -1 if max_drones is None else int(max_drones)
        cfg.curriculum_level = -1 if curriculum_level is None else int(curriculum_level)
        cfg.seed = int(seed)
        cfg.env_id_offset = int(env_id_offset)
        cfg.damping = float(damping)
        cfg.torque_world = int(bool(torque_world))
        cfg.gyro = int(bool(gyro))
        cfg.marl_wrapper = int(bool(marl_wrapper))
        cfg.ctrl_freq = int(ctrl_freq)
        cfg.pyb_freq = int(pyb_freq)
        # Physics enum by name ("pyb", "dyn", "pyb_gnd", ...), by value, or an object with .value / .name
        if hasattr(physics, "value"):
            physics = physics.value
        cfg.physics = L.PHYSICS[physics.lower()] if isinstance(physics, str) else int(physics)
        cfg.eval_metrics = int(bool(eval_metrics))
        cfg.link_lag = int(bool(link_lag))
        self._table = None
        if spawn_table is not None:
            self._table = np.ascontiguousarray(spawn_table, np.float64)
            cfg.spawn_table = self._table.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
            cfg.spawn_scenarios, cfg.spawn_cows = self._table.shape[0], self._table.shape[1]
        self.cfg = cfg
        self.handle = ctypes.c_void_p()
        torch.cuda.set_device(dev_index)
        L.check(L.lib().ch_create(ctypes.byref(cfg), int(n_envs), dev_index, ctypes.byref(self.handle)))
        E, R, C, K = ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        L.check(L.lib().ch_shape(self.handle, ctypes.byref(E), ctypes.byref(R), ctypes.byref(C), ctypes.byref(K)),
                self.handle)
        self.n_envs, self.obs_rows, self.obs_cols, self.reward_cols = E.value, R.value, C.value, K.value
        self.num_drones, self.num_cattle = num_drones, num_cattle
        self.device = torch.device("cuda", dev_index)
        z = dict(device=self.device)
        self.obs = torch.zeros((self.n_envs, self.obs_rows, 86), dtype=torch.float32, **z)
        self.terminal_obs = torch.zeros_like(self.obs)
        self.reward = torch.zeros((self.n_envs, self.reward_cols), dtype=torch.float32, **z)
        self.terminated = torch.zeros((self.n_envs, self.reward_cols), dtype=torch.uint8, **z)
        self.truncated = torch.zeros_like(self.terminated)
        self.agent_active = torch.zeros((self.n_envs, num_drones), dtype=torch.uint8, **z)
        self.reset_happened = torch.zeros(self.n_envs, dtype=torch.uint8, **z)
        self.actions = torch.zeros((self.n_envs, num_drones, 4), dtype=torch.float32, **z)
        # per env: return and length of the last episode that ended (rows rewritten only where one ends)
        self.episode_stats = torch.zeros((self.n_envs, 2), dtype=torch.float64, **z)
        # the step io block: output pointers are fixed for the life of the batch, so a step only
        # rewrites the action pointers and flags (keeps the per-step host cost to one ctypes call)
        self._io = L.ChStepIO()
        self._io.obs = self.obs.data_ptr()
        self._io.reward = self.reward.data_ptr()
        self._io.terminated = self.terminated.data_ptr()
        self._io.truncated = self.truncated.data_ptr()
        self._io.agent_active = self.agent_active.data_ptr()
        self._io.reset_happened = self.reset_happened.data_ptr()
        self._io.episode_stats = self.episode_stats.data_ptr()
        self._io_ref = ctypes.byref(self._io)
        self._ch_step = L.lib().ch_step
        self._raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        self._dev_index = dev_index
        self._actions_ptr = self.actions.data_ptr()
        self._terminal_ptr = self.terminal_obs.data_ptr()
        self._last_obs_out = None   # weakref of the last obs_out tensor stepped into

    # ------------------------------------------------------------------------------------------
    def _stream(self):
        if self._raw_stream is not None:
            return ctypes.c_void_p(self._raw_stream(self._dev_index))
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def reset(self, mask=None, num_drones=None, cow_vel=None):
        """BaseAviary.reset for the envs selected by ``mask`` (bool/uint8 [E] device tensor; None = all).

        ``num_drones`` (int [E]) and ``cow_vel`` (float64 [E, num_cattle, 2]) replace the device's Philox
        draws of those resets -- e.g. cattleherd.seeded.ReferenceResetRNG's replay of the reference's own
        seeded draws (ch_reset_with)."""
        m = None
        if mask is not None:
            mask = mask.to(device=self.device, dtype=self.torch.uint8).contiguous()
            m = ctypes.c_void_p(mask.data_ptr())
        obs = ctypes.c_void_p(self.obs.data_ptr())
        if num_drones is None and cow_vel is None:
            L.check(L.lib().ch_reset(self.handle, m, obs, self._stream()), self.handle)
            return self.obs
        nd = None if num_drones is None else np.ascontiguousarray(np.broadcast_to(num_drones, (self.n_envs,)), np.int32)
        cv = None
        if cow_vel is not None:
            cv = np.ascontiguousarray(np.broadcast_to(cow_vel, (self.n_envs, self.num_cattle, 2)), np.float64)
        L.check(L.lib().ch_reset_with(self.handle, m, None if nd is None else nd.ctypes.data,
                                      None if cv is None else cv.ctypes.data, obs, self._stream()), self.handle)
        return self.obs

    def step(self, actions=None, autoreset=True, random_actions=False, terminal_obs=True, obs_out=None):
        """BaseAviary.step for every env.  ``actions``: float32 [E, num_drones, 4] device tensor.

        ``self.obs`` is overwritten in place and is read-only to the caller: the step kernel stores only
        the entries that change (own state, neighbours, cattle), the constant-zero bytes of each block
        (rows >= NUM_DRONES, the action-buffer block) stay from the last full write.  After writing
        into ``self.obs``, call ``invalidate_obs()`` so the next step rewrites every block in full.
        ``obs_out`` (float32 [E, obs_rows, 86] device tensor, 16-byte aligned): write this step's
        observations there instead of ``self.obs`` (a switch of buffers makes the next step write every
        block in full, ch_api.cpp note_obs_buffer)."""
        io = self._io
        if obs_out is not None:
            if (obs_out.dtype != self.torch.float32 or obs_out.device != self.device or not obs_out.is_contiguous()
                    or tuple(obs_out.shape) != tuple(self.obs.shape)):
                raise ValueError(f"obs_out must be a contiguous float32 {tuple(self.obs.shape)} tensor on {self.device}")
            # The kernels recognise the buffer holding an env's constant-zero bytes by its address.  A new tensor can
            # reuse the address of one written earlier (torch's caching allocator) while holding other data, so any
            # tensor other than the last obs_out makes the next step write every block in full.
            last = self._last_obs_out() if self._last_obs_out is not None else None
            if last is not obs_out:
                self.invalidate_obs()
                import weakref
                self._last_obs_out = weakref.ref(obs_out)
            io.obs = obs_out.data_ptr()
            try:
                _, rew, te, tr = self.step(actions, autoreset, random_actions, terminal_obs)
            finally:
                io.obs = self.obs.data_ptr()
            return obs_out, rew, te, tr
        flags = (L.CH_STEP_AUTORESET if autoreset else 0) | (L.CH_STEP_RANDOM_ACTIONS if random_actions else 0)
        if random_actions:
            io.actions = None
            io.actions_out = self._actions_ptr
        else:
            if actions is None:
                actions = self.actions
            if actions.dtype != self.torch.float32 or actions.device != self.device or not actions.is_contiguous():
                actions = actions.to(device=self.device, dtype=self.torch.float32).contiguous()
            if tuple(actions.shape) != (self.n_envs, self.num_drones, 4):
                raise ValueError(f"actions must have shape {(self.n_envs, self.num_drones, 4)}, got {tuple(actions.shape)}")
            self._keep = actions
            io.actions = actions.data_ptr()
            io.actions_out = None
        io.terminal_obs = self._terminal_ptr if (terminal_obs and autoreset) else None
        io.flags = flags
        rc = self._ch_step(self.handle, self._io_ref, self._stream())
        if rc:
            L.check(rc, self.handle)
        return self.obs, self.reward, self.terminated, self.truncated

    def step_n(self, n_steps, actions=None, autoreset=True, random_actions=True):
        """``n_steps`` calls of ``step(..., terminal_obs=False)`` with the same arguments, in one ``ch_step_n``: the
        first step is one launch, the other ``n_steps - 1`` run in one launch in which every workgroup steps its envs
        back to back (the BASELINE geometries; one launch per step elsewhere).  Random actions are drawn per step on
        the device.  Returns the last step's outputs."""
        io = self._io
        flags = (L.CH_STEP_AUTORESET if autoreset else 0) | (L.CH_STEP_RANDOM_ACTIONS if random_actions else 0)
        if random_actions:
            io.actions = None
            io.actions_out = self._actions_ptr
        else:
            if actions is None:
                actions = self.actions
            if actions.dtype != self.torch.float32 or actions.device != self.device or not actions.is_contiguous():
                actions = actions.to(device=self.device, dtype=self.torch.float32).contiguous()
            if tuple(actions.shape) != (self.n_envs, self.num_drones, 4):
                raise ValueError(f"actions must have shape {(self.n_envs, self.num_drones, 4)}, got {tuple(actions.shape)}")
            self._keep = actions
            io.actions = actions.data_ptr()
            io.actions_out = None
        io.terminal_obs = None
        io.flags = flags
        L.check(L.lib().ch_step_n(self.handle, self._io_ref, int(n_steps), self._stream()), self.handle)
        return self.obs, self.reward, self.terminated, self.truncated

    def host_outputs(self, ring=2, ended=True, agents=False):
        """A HostOutputs over this batch: pinned host buffers the last step's outputs are delivered into
        (ch_outputs_to_host), ``ring`` sets of them used in turn."""
        return HostOutputs(self, ring=ring, ended=ended, agents=agents)

    def step_policy(self, policy, autoreset=True, terminal_obs=False):
        """One step with the actions of an on-device policy (cattleherd.policy.DevicePolicy) for the
        current observations: the SB3 ``model.predict(obs, deterministic=True)`` + ``env.step`` loop
        of CTDECattleHerder.py:202-204 without leaving the GPU."""
        return self.step(policy.act(self), autoreset=autoreset, terminal_obs=terminal_obs)

    def invalidate_obs(self):
        """The caller modified ``self.obs``: the next step writes every observation block in full."""
        L.check(L.lib().ch__obs_invalidate(self.handle, self._stream()), self.handle)

    def capture_rollout(self, steps, autoreset=True, terminal_obs=False):
        """Capture ``steps`` random-action steps into a HIP graph (torch.cuda.CUDAGraph); ``replay()``
        then runs them with one launch from the host.  Every launch parameter is constant across steps
        (the Philox counter lives in the env state) and the state-dependent switches (Euler cache,
        observation bytes) are per-env device flags the kernel reads at run time, so a replay is exactly
        ``steps`` calls of ``step(random_actions=True)``, also after reset()/set_state()/invalidate_obs()
        and after steps into another observation buffer (``obs_out``: the switch raises the flags).
        Nothing runs at capture time."""
        torch = self.torch
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            with torch.cuda.graph(graph, stream=side):
                for _ in range(steps):
                    self.step(random_actions=True, autoreset=autoreset, terminal_obs=terminal_obs)
        torch.cuda.current_stream(self.device).wait_stream(side)
        return graph

    # ------------------------------------------------------------------------------------------
    def state_size(self):
        nd, ni = ctypes.c_int64(), ctypes.c_int64()
        L.check(L.lib().ch_state_size(self.handle, ctypes.byref(nd), ctypes.byref(ni)), self.handle)
        return nd.value, ni.value

    def get_state_raw(self):
        nd, ni = self.state_size()
        d = np.zeros(nd, np.float64)
        i = np.zeros(ni, np.int32)
        L.check(L.lib().ch_get_state(self.handle, d.ctypes.data, i.ctypes.data, self._stream()), self.handle)
        return d, i

    def env_ints(self):
        """The per-env integer scalars only (ENV_INTS rows, numpy int32 [E] each): one small copy instead
        of the whole state (NUM_DRONES, step counters, curriculum level, ...)."""
        nd, ni = self.state_size()
        i = np.zeros(ni, np.int32)
        L.check(L.lib().ch_get_state(self.handle, None, i.ctypes.data, self._stream()), self.handle)
        iv = i.reshape(len(ENV_INTS), self.n_envs)
        return {name: iv[k].copy() for k, name in enumerate(ENV_INTS)}

    def set_state_raw(self, d, i):
        d = np.ascontiguousarray(d, np.float64)
        i = np.ascontiguousarray(i, np.int32)
        L.check(L.lib().ch_set_state(self.handle, d.ctypes.data, i.ctypes.data, self._stream()), self.handle)

    def get_state(self):
        """SoA state as a dict of numpy arrays with a leading env axis (keys as in tests/golden)."""
        d, ints = self.get_state_raw()
        E, N, M = self.n_envs, self.num_drones, self.num_cattle
        nd, nc = DRONE_COMPS * E * N, CATTLE_COMPS * E * M
        dr = d[:nd].reshape(DRONE_COMPS, E, N)
        ca = d[nd:nd + nc].reshape(CATTLE_COMPS, E, M)
        er = d[nd + nc:nd + nc + 2 * E].reshape(2, E)
        ph = d[nd + nc + 2 * E:].reshape(PHYS_COMPS, E, N)
        iv = ints.reshape(len(ENV_INTS), E)
        s = {"last_rpm": ph[0:4].transpose(1, 2, 0), "rpy_rates": ph[4:7].transpose(1, 2, 0),
             "drone_pos": dr[0:3].transpose(1, 2, 0), "drone_quat": dr[3:7].transpose(1, 2, 0),
             "drone_vel": dr[7:10].transpose(1, 2, 0), "drone_angv": dr[10:13].transpose(1, 2, 0),
             "pid_last_rpy": dr[13:16].transpose(1, 2, 0), "pid_int_pos": dr[16:19].transpose(1, 2, 0),
             "pid_int_rpy": dr[19:22].transpose(1, 2, 0), "drone_qlag": dr[22:26].transpose(1, 2, 0),
             "cow_pos": ca[0:2].transpose(1, 2, 0), "cow_vel": ca[2:4].transpose(1, 2, 0),
             "prev_cent": er[0].copy(), "clock": er[1].copy()}
        for k, name in enumerate(ENV_INTS):
            s[name] = iv[k].copy()
        s["active"] = ((s["active_mask"][:, None] >> np.arange(N)[None, :]) & 1).astype(np.uint8)
        return {k: np.ascontiguousarray(v) for k, v in s.items()}

    def set_state(self, s):
        """Inverse of get_state; any key left out keeps its current value."""
        d, ints = self.get_state_raw()
        E, N, M = self.n_envs, self.num_drones, self.num_cattle
        nd, nc = DRONE_COMPS * E * N, CATTLE_COMPS * E * M
        dr = d[:nd].reshape(DRONE_COMPS, E, N)
        ca = d[nd:nd + nc].reshape(CATTLE_COMPS, E, M)
        er = d[nd + nc:nd + nc + 2 * E].reshape(2, E)
        ph = d[nd + nc + 2 * E:].reshape(PHYS_COMPS, E, N)
        iv = ints.reshape(len(ENV_INTS), E)
        for key, lo, hi in (("last_rpm", 0, 4), ("rpy_rates", 4, 7)):
            if key in s:
                ph[lo:hi] = np.asarray(s[key], np.float64)[:, :N, :].transpose(2, 0, 1)
        if "drone_quat" in s and "drone_qlag" not in s:
            # a state from elsewhere (fixtures, the oracle's older dumps): the links' cached frame is the attitude
            # itself, as right after loadURDF
            s = dict(s, drone_qlag=s["drone_quat"])
        for key, lo, hi in (("drone_pos", 0, 3), ("drone_quat", 3, 7), ("drone_vel", 7, 10), ("drone_angv", 10, 13),
                            ("pid_last_rpy", 13, 16), ("pid_int_pos", 16, 19), ("pid_int_rpy", 19, 22),
                            ("drone_qlag", 22, 26)):
            if key in s:
                dr[lo:hi] = np.asarray(s[key], np.float64)[:, :N, :].transpose(2, 0, 1)
        for key, lo, hi in (("cow_pos", 0, 2), ("cow_vel", 2, 4)):
            if key in s:
                ca[lo:hi] = np.asarray(s[key], np.float64)[:, :M, :].transpose(2, 0, 1)
        if "prev_cent" in s:
            er[0] = np.nan_to_num(np.asarray(s["prev_cent"], np.float64), nan=0.0)
        if "clock" in s:
            er[1] = s["clock"]
        if "active" in s and "active_mask" not in s:
            a = np.asarray(s["active"]).astype(np.int64)[:, :N]
            s = dict(s, active_mask=(a << np.arange(N)[None, :]).sum(1))
        for k, name in enumerate(ENV_INTS):
            if name in s:
                iv[k] = np.asarray(s[name]).astype(np.int64)
        self.set_state_raw(d, ints)

    def metrics(self, reset=False):
        """Rollout metric sums (L.METRIC_NAMES) as float64 numpy: one device reduction, a 72-byte copy
        and a stream sync; raises if a step kernel recorded a device error."""
        out = np.zeros(len(L.METRIC_NAMES), np.float64)
        L.check(L.lib().ch_metrics(self.handle, out.ctypes.data, int(bool(reset)), self._stream()), self.handle)
        return out

    def metrics_device(self, reset=False, out=None):
        """The same sums into a float64 device tensor on the current stream, no host sync (the input of
        the end-of-rollout RCCL all-reduce)."""
        if out is None:
            out = self.torch.empty(len(L.METRIC_NAMES), dtype=self.torch.float64, device=self.device)
        L.check(L.lib().ch_metrics_device(self.handle, ctypes.c_void_p(out.data_ptr()), int(bool(reset)),
                                          self._stream()), self.handle)
        return out

    def eval_distances(self):
        """update_evaluation_metrics' per-drone episode distance (BaseAviary.py:1415-1426), numpy
        float64 [E, num_drones]; the reference's 2-vector holds this value in both components."""
        out = np.zeros((self.n_envs, self.num_drones), np.float64)
        L.check(L.lib().ch_get_eval(self.handle, out.ctypes.data, self._stream()), self.handle)
        return out

    def sync(self):
        """Wait for this batch's stream; raises ChError if a step kernel recorded a device error."""
        L.check(L.lib().ch_sync(self.handle, self._stream()), self.handle)

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            L.lib().ch_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostOutputs:
    """Pinned host copies of a HerdBatch's step outputs, filled by one ``ch_outputs_to_host`` call per step.

    This is what SubprocVecEnv.step_wait gathers from its workers (CTDECattleHerder.py:91-99) and what
    RLlibMultiAgentWrapper.step builds its dicts from (marl_wrapper.py:97-119).  ``ring`` sets of buffers are
    used in turn, so the arrays of the last ``ring - 1`` deliveries stay valid while the next one is filled
    (SB3's collect_rollouts reads the previous step's observation after the next env.step).  The observation
    copy moves only the first num_drones rows of every block; the rest of a CTDE block is always zero and the
    host buffers are zeroed once here."""

    def __init__(self, batch, ring=2, ended=True, agents=False):
        import torch
        self.batch, self.ring, self._k = batch, max(1, int(ring)), -1
        E, R, K, N = batch.n_envs, batch.obs_rows, batch.reward_cols, batch.num_drones
        pin = dict(pin_memory=True)
        self._sets = []
        for _ in range(self.ring):
            s = {"obs": torch.zeros((E, R, 86), dtype=torch.float32, **pin),
                 "reward": torch.zeros((E, K), dtype=torch.float32, **pin),
                 "terminated": torch.zeros((E, K), dtype=torch.uint8, **pin),
                 "truncated": torch.zeros((E, K), dtype=torch.uint8, **pin),
                 "reset_happened": torch.zeros(E, dtype=torch.uint8, **pin)}
            if agents:
                s["agent_active"] = torch.zeros((E, N), dtype=torch.uint8, **pin)
            if ended:
                s["ended_env"] = torch.zeros(E, dtype=torch.int64, **pin)
                s["ended_obs"] = torch.zeros((E, R, 86), dtype=torch.float32, **pin)
                s["ended_stats"] = torch.zeros((E, 2), dtype=torch.float64, **pin)
            out = L.ChHostOut()
            for k, t in s.items():
                setattr(out, k, t.data_ptr())
            self._sets.append((s, {k: t.numpy() for k, t in s.items()}, out))
        self.ended = ended

    def fetch(self):
        """Deliver the last step's outputs (synchronises the batch's stream).  Returns a dict of numpy arrays
        (views of this delivery's pinned buffers): obs, reward, terminated, truncated, reset_happened
        (+ agent_active) and, for the envs that auto-reset in the step, ``ended_env`` (ascending),
        ``ended_obs`` (their terminal observations) and ``ended_stats`` (episode return, length)."""
        b = self.batch
        self._k = (self._k + 1) % self.ring
        _, arrs, out = self._sets[self._k]
        L.check(L.lib().ch_outputs_to_host(b.handle, b._io_ref, ctypes.byref(out), b._stream()), b.handle)
        res = dict(arrs)
        if self.ended:
            n = int(out.ended_count)
            res["ended_env"], res["ended_obs"], res["ended_stats"] = (arrs["ended_env"][:n], arrs["ended_obs"][:n],
                                                                      arrs["ended_stats"][:n])
        return res
