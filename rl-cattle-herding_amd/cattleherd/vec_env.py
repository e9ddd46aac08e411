"""SB3-style vectorised env over one HerdBatch: all envs of a GPU behind the VecEnv interface.

Drop-in for ``make_vec_env(CattleAviary, n_envs=..., vec_env_cls=SubprocVecEnv)``
(simulator/CTDECattleHerder.py:91-97): ``CattleHerdVecEnv(n_envs, num_drones=..., num_cattle=...)``
returns numpy observations ``(E, 12, 86)`` (by default a view of one of ``obs_ring`` = 2 pinned host buffers used in
turn, valid until ``obs_ring`` more steps have run -- SB3's collect_rollouts needs one; ``copy_obs=True`` returns a
fresh array, SubprocVecEnv's semantics, at the cost of a 17 MB host copy per step at 4096 envs), rewards ``(E,)``,
dones ``(E,)`` and a fresh list of per-env infos (dicts the step never changes afterwards) with
SB3's ``terminal_observation`` / ``TimeLimit.truncated`` keys and, as the Monitor that ``make_vec_env``
wraps around every env (CTDECattleHerder.py:91-99) adds, ``episode = {"r", "l", "t"}`` for each episode that
ends, auto-resetting finished envs inside the step launch.  ``step_tensors`` is the zero-copy path for
on-device policies.

If stable_baselines3 is importable the class derives from its VecEnv; otherwise it implements the
same methods (duck-typed).
"""
import time

import numpy as np

from .env import HerdBatch
from .spaces import CURRICULUM, DEFAULT_LEVEL, check_supported, ctde_action_space, ctde_observation_space

try:  # pragma: no cover
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _VecEnvBase
except Exception:  # noqa: BLE001
    _VecEnvBase = object


class CattleHerdVecEnv(_VecEnvBase):
    def __init__(self, n_envs, num_drones=2, num_cattle=1, obs="cokin", act="vel", drone_model="cf2x",
                 physics="pyb", device=None, copy_obs=False, obs_ring=2, **batch_kw):
        check_supported(drone_model, physics, obs, act)
        self.batch = HerdBatch(n_envs, num_drones, num_cattle, mode="ctde", device=device, physics=physics,
                               **batch_kw)
        self.num_envs = n_envs
        self.num_drones = num_drones
        self.observation_space = ctde_observation_space()
        self.action_space = ctde_action_space(num_drones)
        self.render_mode = None
        self._actions = None
        self._attrs = {"EPISODE_LEN_SEC": self._episode_len(), "CTRL_FREQ": self.batch.cfg.ctrl_freq,
                       "CTRL_TIMESTEP": 1.0 / self.batch.cfg.ctrl_freq, "NUM_DRONES": num_drones,
                       "is_evaluating": False}
        self._t_start = time.time()
        # host delivery: pinned buffers filled by one ch_outputs_to_host per step (two sets used in turn, so the
        # observation array returned by a step stays valid through the next step, as SB3's collect_rollouts needs)
        if obs_ring < 2:
            raise ValueError("obs_ring must be >= 2 (collect_rollouts keeps the previous step's observations)")
        self._host = self.batch.host_outputs(ring=int(obs_ring), ended=True)
        self._copy_obs = bool(copy_obs)
        # _computeInfo's {"answer": 42} per env (CattleAviary.py): every step builds a new dict for every env (the envs
        # that ended also get terminal_observation, TimeLimit.truncated, episode), so infos a caller keeps or mutates do
        # not change under later steps (SubprocVecEnv hands out fresh dicts too)
        if _VecEnvBase is not object:  # SB3 bookkeeping
            _VecEnvBase.__init__(self, n_envs, self.observation_space, self.action_space)

    def _episode_len(self):
        lvl = self.batch.cfg.curriculum_level
        return CURRICULUM[DEFAULT_LEVEL["ctde"] if lvl < 0 else lvl][2]

    # ---- VecEnv API --------------------------------------------------------------------------
    def reset(self):
        return self.batch.reset().cpu().numpy()

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        """SubprocVecEnv.step_wait over the batch: one launch, then one ch_outputs_to_host (the first num_drones rows
        of every observation block, reward and flags, and the terminal observations / episode statistics of the
        envs that auto-reset, compacted on the device) into pinned buffers and a stream sync."""
        a = self._actions
        torch = self.batch.torch
        if not isinstance(a, torch.Tensor):
            # numpy actions through a pinned staging buffer (the previous step's copy out of it has completed: the
            # delivery below synchronises the stream)
            if getattr(self, "_act_pin", None) is None:
                self._act_pin = torch.zeros((self.num_envs, self.num_drones, 4), dtype=torch.float32)
                if str(self.batch.device).startswith("cuda"):   # (the CPU tests' stand-in batch has no device)
                    self._act_pin = self._act_pin.pin_memory()
                self._act_np = self._act_pin.numpy()
            np.copyto(self._act_np, np.asarray(a, np.float32).reshape(self.num_envs, -1, 4)[:, :self.num_drones])
            a = self._act_pin.to(self.batch.device, non_blocking=True)
        self.batch.step(a, autoreset=True, terminal_obs=True)
        h = self._host.fetch()
        rew_np = h["reward"][:, 0].copy()
        te_np = h["terminated"][:, 0].astype(bool)
        tr_np = h["truncated"][:, 0].astype(bool)
        dones = te_np | tr_np
        infos = [{"answer": 42} for _ in range(self.num_envs)]   # fresh dicts every step (SubprocVecEnv semantics)
        idx = h["ended_env"]
        if len(idx):
            # Monitor.step: the episode's summed float64 reward and length, kept on the device by the step kernel
            # (ch_step_io.episode_stats), and the wall time since the Monitor started
            t = round(time.time() - self._t_start, 6)
            term_obs, stats = h["ended_obs"], h["ended_stats"]
            for k, e in enumerate(idx.tolist()):
                infos[e] = {"answer": 42, "terminal_observation": term_obs[k].copy(),
                            "TimeLimit.truncated": bool(tr_np[e] and not te_np[e]),
                            "episode": {"r": round(float(stats[k, 0]), 6), "l": int(stats[k, 1]), "t": t}}
        return (h["obs"].copy() if self._copy_obs else h["obs"]), rew_np, dones, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def step_tensors(self, actions):
        """Zero-copy: device tensors in and out (obs (E,12,86), reward (E,1), terminated, truncated)."""
        return self.batch.step(actions, autoreset=True, terminal_obs=True)

    def close(self):
        self.batch.close()

    def seed(self, seed=None):
        return [None] * self.num_envs

    def get_attr(self, attr_name, indices=None):
        n = len(self._indices(indices))
        if attr_name in self._attrs:
            return [self._attrs[attr_name]] * n
        return [getattr(self, attr_name)] * n

    def set_attr(self, attr_name, value, indices=None):
        self._attrs[attr_name] = value

    def env_method(self, method_name, *args, indices=None, **kwargs):
        return [getattr(self, method_name)(*args, **kwargs) for _ in self._indices(indices)]

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._indices(indices))

    def get_images(self):
        return [None] * self.num_envs

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices
