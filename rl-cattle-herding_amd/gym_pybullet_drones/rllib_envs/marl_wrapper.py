"""RLlibMultiAgentWrapper on the MI355X HIP path — drop-in for the reference's
(reference: gym_pybullet_drones/rllib_envs/marl_wrapper.py:8-125).

Agent ids ``agent_i``, per-agent Box(86,) observation / Box(4,) action spaces,
``reset(*, seed, options) -> (obs, infos)`` and ``step(action_dict) -> (obs, rewards, dones, truncs,
infos)`` with ``"__all__"``.  The wrapper's per-agent recomputation after env.step, the removal of
finished agents and the ``"__all__"`` rule (all agents terminated; truncation does not end the
episode) run inside the HIP step launch (ch_config.marl_wrapper = 1), so the dicts are identical to
the reference's.
"""
import inspect
from typing import Any, Dict

import numpy as np

from gym_pybullet_drones.rllib_envs.MARLCattleAviary import MARLCattleAviary

# the reference's failure-detection hook (marl_wrapper.py:87-95): an exception out of env.step() is appended, with
# its traceback, to this file on the env runner, then re-raised
EXC_LOG = "/tmp/env_worker_exc.log"

try:  # pragma: no cover
    from ray.rllib.env import MultiAgentEnv as _MAEnvBase
except Exception:  # noqa: BLE001
    _MAEnvBase = object


class RLlibMultiAgentWrapper(_MAEnvBase):
    def __init__(self, env_config: Dict[str, Any]):
        if _MAEnvBase is not object:
            super().__init__()
        cfg = dict(env_config) if env_config is not None else {}
        params = set(inspect.signature(MARLCattleAviary.__init__).parameters)
        cfg.setdefault("gui", False)
        filtered = {k: v for k, v in cfg.items() if k in params and not k.startswith("_")}
        ignored = set(cfg) - set(filtered)
        try:
            self.env = MARLCattleAviary(**filtered, _wrapper_semantics=True)
        except Exception as e:
            msg = f"Failed to create MARLCattleAviary in RLlib wrapper: {e}"
            if ignored:
                msg += f" (ignored unsupported keys: {sorted(ignored)})"
            raise RuntimeError(msg) from e
        self._set_agents()

    def _set_agents(self):
        self.possible_agents = [f"agent_{i}" for i in range(self.env.NUM_DRONES)]
        self.agents = self.possible_agents.copy()
        self.action_space = {aid: self.env.action_space for aid in self.possible_agents}
        self.observation_space = {aid: self.env.observation_space for aid in self.possible_agents}

    def get_action_space(self, agent_id):
        return self.env.action_space

    def get_observation_space(self, agent_id):
        return self.env.observation_space

    def reset(self, *, seed=None, options=None):
        self.env.reset(seed=seed, options=options)
        self._set_agents()
        obs = {f"agent_{i}": self.env._computeObs(i) for i in range(self.env.NUM_DRONES)}
        infos = {f"agent_{i}": {} for i in range(self.env.NUM_DRONES)}
        return obs, infos

    def step(self, action_dict: Dict[str, np.ndarray]):
        n = self.env.NUM_DRONES
        actions = np.zeros((n, 4), dtype=np.float32)
        for i, aid in enumerate(self.possible_agents):
            if aid in action_dict and aid in self.agents:
                actions[i] = np.asarray(action_dict[aid], dtype=np.float32)
        try:
            obs_a, rew_a, te_a, tr_a = self.env._step_arrays(actions)
        except Exception:
            import traceback
            with open(EXC_LOG, "a") as fh:
                fh.write("=== Exception in env.step() ===\n")
                fh.write(traceback.format_exc())
                fh.write("\n")
            raise
        obs, rewards, dones, truncs, infos = {}, {}, {}, {}, {}
        for aid in list(self.agents):
            i = int(aid.split("_")[1])
            obs[aid] = obs_a[i]
            rewards[aid] = float(rew_a[i])
            dones[aid] = bool(te_a[i])
            truncs[aid] = bool(tr_a[i])
            infos[aid] = {"answer": 42}
        self.agents = [aid for aid in self.agents if not dones.get(aid, False)]
        dones["__all__"] = len(self.agents) == 0
        truncs["__all__"] = len(self.agents) == 0
        return obs, rewards, dones, truncs, infos

    def render(self, mode="human"):
        return None

    def close(self):
        return self.env.close()
