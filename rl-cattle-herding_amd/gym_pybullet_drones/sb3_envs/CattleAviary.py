"""CattleAviary on the MI355X HIP path — drop-in for the reference's CTDE env
(reference: gym_pybullet_drones/sb3_envs/CattleAviary.py, constructor at :14-105).

Same constructor keywords, ``reset(seed, options) -> (obs, info)``,
``step(action) -> (obs, reward, terminated, truncated, info)``, (12, 86) float32 observations and the
attributes the drivers read (EPISODE_LEN_SEC, CTRL_FREQ, CTRL_TIMESTEP, NUM_DRONES, is_evaluating,
evaluation_save, action_space, observation_space).  One instance = one env (E = 1) for
Gymnasium / SB3 ``DummyVecEnv`` / ``evaluate_policy`` use; for throughput use the batched
``cattleherd.vec_env.CattleHerdVecEnv`` (a one-line ``vec_env_cls`` swap).
"""
import numpy as np

from cattleherd.evaluation import EvalTracker, Evaluator
from cattleherd.seeded import ReferenceResetRNG
from cattleherd.env import HerdBatch
from cattleherd.spaces import (CURRICULUM, ActionType, DroneModel, ObservationType, Physics, check_supported,
                               ctde_action_space, ctde_observation_space)

try:  # pragma: no cover
    import gymnasium as _gym
    _EnvBase = _gym.Env
except Exception:  # noqa: BLE001
    _EnvBase = object


class CattleAviary(_EnvBase):
    """Multi-agent RL problem: drones herding cattle (CTDE, one policy over a (12, 86) observation)."""

    def __init__(self, drone_model: DroneModel = DroneModel.CF2X, num_drones: int = 2, num_cattle: int = 1,
                 neighbourhood_radius: float = np.inf, initial_xyzs=None, initial_rpys=None,
                 physics: Physics = Physics.PYB, pyb_freq: int = 240, ctrl_freq: int = 60, gui=False, record=False,
                 obs: ObservationType = ObservationType.COKIN, act: ActionType = ActionType.VEL, *,
                 curriculum_level: int = 7, device=None, compat: bool = True, precision: str = "f64",
                 min_drones=None, max_drones=None, seed: int = 0x5EED, env_id: int = 0,
                 reference_rng_seed=None):
        check_supported(drone_model, physics, obs, act)
        if pyb_freq % ctrl_freq != 0:
            raise ValueError("[ERROR] in BaseAviary.__init__(), pyb_freq is not divisible by env_freq.")
        lo, hi, ep = CURRICULUM[curriculum_level]
        # the reference draws NUM_DRONES in the curriculum's [min, max] but sizes its controllers by
        # num_drones (BaseRLAviary.py:80); clip the range so every draw is runnable
        self.MIN_NUM_DRONES = min(lo, num_drones) if min_drones is None else int(min_drones)
        self.MAX_NUM_DRONES = min(hi, num_drones) if max_drones is None else int(max_drones)
        self.CTRL_FREQ, self.PYB_FREQ = ctrl_freq, pyb_freq
        self.CTRL_TIMESTEP, self.PYB_TIMESTEP = 1.0 / ctrl_freq, 1.0 / pyb_freq
        self.PYB_STEPS_PER_CTRL = pyb_freq // ctrl_freq
        self.EPISODE_LEN_SEC = ep
        self.NUM_CATTLE = num_cattle
        self.DRONE_TARGET_ALTITUDE = 0.45
        self.GUI, self.RECORD = bool(gui), bool(record)
        self.batch = HerdBatch(1, num_drones, num_cattle, mode="ctde", device=device, compat=compat,
                               precision=precision, min_drones=self.MIN_NUM_DRONES, max_drones=self.MAX_NUM_DRONES,
                               curriculum_level=curriculum_level, seed=seed, env_id_offset=env_id,
                               ctrl_freq=ctrl_freq, pyb_freq=pyb_freq, physics=physics)
        self._num_drones_ctor = num_drones
        # seed-exact resets: the draws a reference env makes after `random.seed(s); np.random.seed(s)`
        # (cattleherd/seeded.py; the curriculum's own [min, max] drone range, as the reference draws it)
        self._ref_rng = None if reference_rng_seed is None else ReferenceResetRNG(reference_rng_seed, lo, hi, num_cattle)
        self.NUM_DRONES = num_drones
        self.action_space = ctde_action_space(num_drones)
        self.observation_space = ctde_observation_space()
        self.eval_system = Evaluator()
        self._tracker = EvalTracker(self.eval_system)
        self._is_evaluating = False
        self._needs_reset = True

    @property
    def is_evaluating(self):
        return self._is_evaluating

    @is_evaluating.setter
    def is_evaluating(self, on):
        """Logging starts with the next step; the cattle velocities it logs are this step's read-back."""
        self._is_evaluating = bool(on)
        if self._is_evaluating and not self._needs_reset:
            self._tracker.set_step_start(self.batch.get_state())

    # ------------------------------------------------------------------------------------------
    def _sync_counts(self, ints=None):
        ints = self.batch.env_ints() if ints is None else ints
        self.NUM_DRONES = int(ints["n"][0])
        self.step_counter = int(ints["step_counter"][0])
        self.step_counter_A = int(ints["step_counter_A"][0])
        return ints

    def reset(self, seed: int = None, options: dict = None):
        """BaseAviary.reset (sb3_envs/BaseAviary.py:280-331); ``seed`` is ignored like the reference's."""
        if self._ref_rng is not None:
            scA = getattr(self, "step_counter_A", 0)   # steps of the episode that ends (its flocking draws)
            n, vel = self._ref_rng.reset(scA)
            if n > self._num_drones_ctor:   # the reference indexes controllers sized by num_drones (BaseRLAviary.py:80)
                raise IndexError(f"NUM_DRONES draw {n} exceeds num_drones={self._num_drones_ctor}")
            obs = self.batch.reset(num_drones=[n], cow_vel=vel[None])
        else:
            obs = self.batch.reset()
        s = self.batch.get_state()
        self._sync_counts(s)
        self._tracker.on_reset(s, self.NUM_DRONES)
        self._needs_reset = False
        return obs[0].cpu().numpy(), {"answer": 42}

    def step(self, action):
        """BaseAviary.step (sb3_envs/BaseAviary.py:335-465) for this env; no auto-reset (Gymnasium).
        While ``is_evaluating``: the reference's logging (update_evaluation_metrics, and the time-out
        evaluation_episode_trigger of _computeTruncated), see cattleherd.evaluation."""
        if self._needs_reset:
            self.reset()
        sc_before, n = self.step_counter, self.NUM_DRONES
        a = np.zeros((1, self._num_drones_ctor, 4), np.float32)
        act = np.asarray(action, np.float32).reshape(-1, 4)
        k = min(len(act), self._num_drones_ctor)
        a[0, :k] = act[:k]
        torch = self.batch.torch
        obs, rew, te, tr = self.batch.step(torch.from_numpy(a).to(self.batch.device), autoreset=False)
        # one device-to-host copy for the observation, reward and both flags (instead of four syncs)
        nobs = obs[0].numel()
        out = torch.cat((obs[0].reshape(-1), rew[0, :1], te[0, :1].float(), tr[0, :1].float())).cpu().numpy()
        obs_np = out[:nobs].reshape(obs.shape[1:])
        reward = float(out[nobs])
        terminated, truncated = bool(out[nobs + 1]), bool(out[nobs + 2])
        if self._is_evaluating:
            s = self.batch.get_state()
            self._tracker.after_step(s, self.batch.eval_distances()[0], n, self.NUM_CATTLE, sc_before, self.CTRL_FREQ,
                                     self.EPISODE_LEN_SEC)
            self._sync_counts(s)
        else:
            self._sync_counts()
        return obs_np, reward, terminated, truncated, {"answer": 42}

    def evaluation_save(self, save_path="evaluation_data.pkl"):
        """evaluation.py:73-94 schema."""
        self.eval_system.save_evaluation_data(save_path)

    def close(self):
        self.batch.close()

    def render(self, mode="human", close=False):
        s = self.batch.get_state()
        for i in range(int(s["n"][0])):
            p = s["drone_pos"][0, i]
            print(f"[INFO] CattleAviary.render() ——— drone {i} ——— x {p[0]:+06.2f}, y {p[1]:+06.2f}, z {p[2]:+06.2f}")
