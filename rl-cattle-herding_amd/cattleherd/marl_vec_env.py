"""Batched RLlib multi-agent surface: ``num_envs`` RLlibMultiAgentWrapper envs in one HerdBatch.

The reference runs its DTDE driver with one ``RLlibMultiAgentWrapper(MARLCattleAviary)`` per RLlib env
runner slot (simulator/DTDECattleHerder.py:81; the wrapper is rllib_envs/marl_wrapper.py:8-125).  Here all of
a GPU's envs live in one ``HerdBatch(mode="marl", marl_wrapper=True)``: the step kernel already runs the
wrapper's per-agent recomputation, the agent drop-out and the ``"__all__"`` rule (marl_wrapper.py:97-119), and
an env whose agents have all terminated is reset inside the same launch.

Two surfaces over the same launch:

* ``step_tensors(actions)`` -- zero-copy device tensors: per-agent observations ``(E, N, 86)``, rewards,
  terminated, truncated ``(E, N)``, the agent mask the step started with (the wrapper's ``self.agents``,
  which decides which keys its dicts carry), the mask after it, ``__all__`` per env and the envs reset.
* ``step(action_dicts)`` -- the wrapper's dicts, one per env: ``obs / rewards / dones / truncs / infos``
  keyed ``"agent_i"`` for the agents live at the start of the step, plus ``"__all__"`` (all agents
  terminated; truncation does not end the episode, marl_wrapper.py:113-117).  An env that ended is already
  reset on the device (its dicts hold the episode's last observations, as the wrapper's would);
  ``reset_at(e)`` returns what the driver's ``reset()`` of that env would return, without another launch.
"""
import numpy as np

from .env import HerdBatch
from .spaces import (CURRICULUM, DEFAULT_LEVEL, agent_action_space, agent_observation_space, check_supported)


class CattleHerdMultiAgentVecEnv:
    def __init__(self, num_envs, env_config=None, device=None, **batch_kw):
        cfg = dict(env_config or {})
        num_drones = int(cfg.get("num_drones", 2))
        num_cattle = int(cfg.get("num_cattle", 1))
        level = int(cfg.get("curriculum_level", DEFAULT_LEVEL["marl"]))
        check_supported(cfg.get("drone_model", "cf2x"), cfg.get("physics", "pyb"), cfg.get("obs", "cokin"),
                        cfg.get("act", "vel"))
        lo, hi, ep = CURRICULUM[level]
        # the drone-count range MARLCattleAviary draws from, clipped to the constructor's num_drones (the
        # reference sizes its controllers by it, BaseRLAviary.py:80)
        mn = min(lo, num_drones) if cfg.get("min_drones") is None else int(cfg["min_drones"])
        mx = min(hi, num_drones) if cfg.get("max_drones") is None else int(cfg["max_drones"])
        self.batch = HerdBatch(num_envs, num_drones, num_cattle, mode="marl", device=device, marl_wrapper=True,
                               curriculum_level=level, min_drones=mn, max_drones=mx,
                               physics=cfg.get("physics", "pyb"), **batch_kw)
        self.num_envs, self.num_drones, self.EPISODE_LEN_SEC = num_envs, num_drones, ep
        self.action_space, self.observation_space = agent_action_space(), agent_observation_space()
        self._ids = np.array([f"agent_{i}" for i in range(num_drones)], dtype=object)
        self._before = None     # (E, N) bool device tensor: the wrapper's self.agents of every env
        self._active = None     # its host copy (the dict path)
        self._n = None          # (E,) NUM_DRONES of every env's episode
        self._reset_obs, self._reset_envs = None, set()

    # ---- reset -----------------------------------------------------------------------------------
    def reset(self, *, seed=None, options=None):
        """Every env's RLlibMultiAgentWrapper.reset (marl_wrapper.py:64-75): lists of obs dicts and info dicts
        with the agents of the new episodes."""
        obs = self.batch.reset().cpu().numpy()
        self.refresh_agents()
        self._reset_obs, self._reset_envs = obs, set(range(self.num_envs))
        return ([self._obs_dict(obs[e], self._n[e]) for e in range(self.num_envs)],
                [{self._ids[i]: {} for i in range(self._n[e])} for e in range(self.num_envs)])

    def refresh_agents(self):
        """Re-read every env's live agents and NUM_DRONES from the device state (after ``batch.set_state``)."""
        b = self.batch
        ints = b.env_ints()
        self._active = (ints["active_mask"][:, None] >> np.arange(self.num_drones)[None, :]) & 1 == 1
        self._active &= np.arange(self.num_drones)[None, :] < ints["n"][:, None]
        self._n = ints["n"].astype(np.int64)
        self._before = b.torch.from_numpy(self._active).to(b.device)

    def _obs_dict(self, obs_e, n):
        return {self._ids[i]: obs_e[i] for i in range(n)}

    def possible_agents(self, e):
        """The wrapper's possible_agents of env ``e`` (agent_0 .. agent_{NUM_DRONES-1} of its episode)."""
        return list(self._ids[:self._n[e]])

    def agents(self, e):
        """The wrapper's agents of env ``e``: the live agents the next step's dicts are keyed by."""
        return list(self._ids[np.nonzero(self._active[e])[0]])

    # ---- step ------------------------------------------------------------------------------------
    def step_tensors(self, actions):
        """One launch for every env (actions float32 [E, N, 4] device tensor; the actions of agents that are not
        live are ignored, marl_wrapper.py:80-84).  Returns a dict of device tensors: ``obs`` [E, N, 86] (the
        episode's last observation where the env ended), ``reward`` [E, N] (NaN for agents not live at the
        start), ``terminated``, ``truncated`` [E, N] bool, ``agents_before`` [E, N] (the wrapper's agents the
        step started with: its dicts carry these keys), ``agents`` [E, N] (the next step's: the survivors, or
        the new episode's where the env was reset) and ``all_done`` [E] (``"__all__"``: every agent
        terminated; those envs are reset in the same launch, their new observations in ``self.batch.obs``).
        ``reward``, ``terminated``, ``truncated`` and ``all_done`` are views of the batch's output buffers: valid
        until the next step."""
        b = self.batch
        torch = b.torch
        if self._before is None:
            raise RuntimeError("call reset() first")
        before = self._before
        b.step(actions, autoreset=True, terminal_obs=True)
        # the uint8 flag buffers reinterpreted as bool (no copy); agent_active is rewritten by the next step
        reset = b.reset_happened.view(torch.bool)
        self._before = b.agent_active.view(torch.bool).clone()
        return {"obs": torch.where(reset[:, None, None], b.terminal_obs, b.obs), "reward": b.reward,
                "terminated": b.terminated.view(torch.bool), "truncated": b.truncated.view(torch.bool),
                "agents_before": before, "agents": self._before, "all_done": reset}

    def step(self, action_dicts):
        """RLlibMultiAgentWrapper.step (marl_wrapper.py:77-119) for every env: ``action_dicts`` is a list of
        {agent_id: action} dicts (or an array [E, N, 4]); returns lists of per-env obs, rewards, dones, truncs
        and infos dicts keyed by the agents live at the start of the step, with ``"__all__"``."""
        b = self.batch
        torch = b.torch
        if isinstance(action_dicts, (list, tuple)):
            a = np.zeros((self.num_envs, self.num_drones, 4), np.float32)
            for e, d in enumerate(action_dicts):
                for aid, act in d.items():
                    a[e, int(str(aid).split("_")[1])] = np.asarray(act, np.float32)
            acts = torch.from_numpy(a).to(b.device)
        else:
            acts = torch.as_tensor(np.asarray(action_dicts, np.float32), device=b.device)
        live = self._active
        out = self.step_tensors(acts)
        obs = out["obs"].cpu().numpy()
        rew = out["reward"].cpu().numpy().astype(np.float64)
        te = out["terminated"].cpu().numpy()
        tr = out["truncated"].cpu().numpy()
        ended = out["all_done"].cpu().numpy()
        self._active = out["agents"].cpu().numpy()
        obs_l, rew_l, done_l, trunc_l, info_l = [], [], [], [], []
        for e in range(self.num_envs):
            idx = np.nonzero(live[e])[0]
            keys = self._ids[idx]
            obs_l.append(dict(zip(keys, obs[e, idx])))
            rew_l.append(dict(zip(keys, rew[e, idx].tolist())))
            d = dict(zip(keys, te[e, idx].tolist()))
            t = dict(zip(keys, tr[e, idx].tolist()))
            # the agents that terminated drop out (marl_wrapper.py:113); __all__ when none is left (116-117),
            # which is exactly when the kernel reset the env
            d["__all__"] = t["__all__"] = bool(ended[e])
            done_l.append(d)
            trunc_l.append(t)
            info_l.append({k: {"answer": 42} for k in keys})
        self._reset_envs = set(np.nonzero(ended)[0].tolist())
        if self._reset_envs:
            self._n = np.where(ended, self._active.sum(1), self._n)   # every agent of a new episode is live
            self._reset_obs = b.obs.cpu().numpy()
        return obs_l, rew_l, done_l, trunc_l, info_l

    def reset_at(self, e):
        """What RLlibMultiAgentWrapper.reset returns for env ``e`` after its episode ended (``"__all__"`` in the
        last step): the device already reset it in that step's launch."""
        if e not in self._reset_envs:
            raise ValueError(f"env {e} did not finish an episode in the last step")
        n = int(self._n[e])
        return self._obs_dict(self._reset_obs[e], n), {self._ids[i]: {} for i in range(n)}

    def close(self):
        self.batch.close()
