"""MARLCattleAviary on the MI355X HIP path — drop-in for the reference's DTDE env
(reference: gym_pybullet_drones/rllib_envs/MARLCattleAviary.py, constructor at :14-105).

``reset() -> ({i: obs_i}, {"__all__": {}})`` and ``step(actions[N, 4]) -> (obs, reward, done, truncated,
info)`` dicts keyed by drone index with ``"__all__"`` entries, exactly the bare env.step dicts of
rllib_envs/BaseAviary.py:425-431 (ch_config.marl_wrapper = 0).  RLlib drivers use
``marl_wrapper.RLlibMultiAgentWrapper``, which runs the wrapper's own per-agent semantics on device.
"""
import numpy as np

from cattleherd.env import HerdBatch
from cattleherd.spaces import (CURRICULUM, ActionType, DroneModel, ObservationType, Physics, agent_action_space,
                               agent_observation_space, check_supported)


class MARLCattleAviary:
    def __init__(self, drone_model: DroneModel = DroneModel.CF2X, num_drones: int = 2, num_cattle: int = 1,
                 neighbourhood_radius: float = np.inf, initial_xyzs=None, initial_rpys=None,
                 physics: Physics = Physics.PYB, pyb_freq: int = 240, ctrl_freq: int = 60, gui=False, record=False,
                 obs: ObservationType = ObservationType.COKIN, act: ActionType = ActionType.VEL, *,
                 curriculum_level: int = 0, device=None, compat: bool = True, precision: str = "f64",
                 min_drones=None, max_drones=None, seed: int = 0x5EED, env_id: int = 0, _wrapper_semantics=False):
        check_supported(drone_model, physics, obs, act)
        if pyb_freq % ctrl_freq != 0:
            raise ValueError("[ERROR] in BaseAviary.__init__(), pyb_freq is not divisible by env_freq.")
        lo, hi, ep = CURRICULUM[curriculum_level]
        self.MIN_NUM_DRONES = min(lo, num_drones) if min_drones is None else int(min_drones)
        self.MAX_NUM_DRONES = min(hi, num_drones) if max_drones is None else int(max_drones)
        self.CTRL_FREQ, self.PYB_FREQ = ctrl_freq, pyb_freq
        self.CTRL_TIMESTEP = 1.0 / ctrl_freq
        self.EPISODE_LEN_SEC = ep
        self.NUM_CATTLE = num_cattle
        self.is_evaluating = False
        self.batch = HerdBatch(1, num_drones, num_cattle, mode="marl", device=device, compat=compat,
                               precision=precision, min_drones=self.MIN_NUM_DRONES, max_drones=self.MAX_NUM_DRONES,
                               curriculum_level=curriculum_level, seed=seed, env_id_offset=env_id,
                               ctrl_freq=ctrl_freq, pyb_freq=pyb_freq, physics=physics, marl_wrapper=_wrapper_semantics)
        self._num_drones_ctor = num_drones
        self.NUM_DRONES = min(self.MAX_NUM_DRONES, num_drones)
        self.action_space = agent_action_space()
        self.observation_space = agent_observation_space()
        self._last = None

    def _n(self):
        s = self.batch.get_state()
        self.NUM_DRONES = int(s["n"][0])
        return self.NUM_DRONES

    def reset(self, seed=None, options=None):
        obs = self.batch.reset()[0].cpu().numpy()
        n = self._n()
        self._last = obs
        return {i: obs[i] for i in range(n)}, {"__all__": {}}

    def _step_arrays(self, action):
        a = np.zeros((1, self._num_drones_ctor, 4), np.float32)
        act = np.asarray(action, np.float32).reshape(-1, 4)
        k = min(len(act), self._num_drones_ctor)
        a[0, :k] = act[:k]
        torch = self.batch.torch
        obs, rew, te, tr = self.batch.step(torch.from_numpy(a).to(self.batch.device), autoreset=False)
        self._last = obs[0].cpu().numpy()
        return (self._last, rew[0].cpu().numpy().astype(np.float64), te[0].cpu().numpy().astype(bool),
                tr[0].cpu().numpy().astype(bool))

    def step(self, action):
        n = self.NUM_DRONES
        obs, rew, te, tr = self._step_arrays(action)
        o = {i: obs[i] for i in range(n)}
        r = {i: float(rew[i]) for i in range(n)}
        d = {i: bool(te[i]) for i in range(n)}
        d["__all__"] = all(d.values())
        t = {i: bool(tr[i]) for i in range(n)}
        t["__all__"] = all(t.values())
        info = {i: {"answer": 42} for i in range(n)}
        return o, r, d, t, info

    def _computeObs(self, drone_id):
        return self._last[drone_id]

    def _computeInfo(self, drone_id):
        return {"answer": 42}

    def close(self):
        self.batch.close()
