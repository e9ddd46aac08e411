"""SB3-style vectorised env over one HerdBatch: all envs of a GPU behind the VecEnv interface.

Drop-in for ``make_vec_env(CattleAviary, n_envs=..., vec_env_cls=SubprocVecEnv)``
(simulator/CTDECattleHerder.py:91-97): ``CattleHerdVecEnv(n_envs, num_drones=..., num_cattle=...)``
returns numpy observations ``(E, 12, 86)``, rewards ``(E,)``, dones ``(E,)`` and per-env infos with
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
                 physics="pyb", device=None, **batch_kw):
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
        a = self._actions
        torch = self.batch.torch
        if not isinstance(a, torch.Tensor):
            a = np.asarray(a, np.float32).reshape(self.num_envs, -1, 4)[:, :self.num_drones]
            a = torch.from_numpy(np.ascontiguousarray(a)).to(self.batch.device)
        obs, rew, te, tr = self.batch.step(a, autoreset=True, terminal_obs=True)
        obs_np = obs.cpu().numpy()
        rew_np = rew[:, 0].cpu().numpy().astype(np.float32)
        te_np = te[:, 0].cpu().numpy().astype(bool)
        tr_np = tr[:, 0].cpu().numpy().astype(bool)
        dones = te_np | tr_np
        infos = [{"answer": 42} for _ in range(self.num_envs)]
        idx = np.nonzero(dones)[0]
        if len(idx):
            term_obs = self.batch.terminal_obs[idx].cpu().numpy()
            # Monitor.step: the episode's summed float64 reward and length, kept on the device by the step
            # kernel (ch_step_io.episode_stats), and the wall time since the Monitor started
            stats = self.batch.episode_stats[idx].cpu().numpy()
            t = round(time.time() - self._t_start, 6)
            for k, e in enumerate(idx):
                infos[e]["terminal_observation"] = term_obs[k]
                infos[e]["TimeLimit.truncated"] = bool(tr_np[e] and not te_np[e])
                infos[e]["episode"] = {"r": round(float(stats[k, 0]), 6), "l": int(stats[k, 1]), "t": t}
        return obs_np, rew_np, dones, infos

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
