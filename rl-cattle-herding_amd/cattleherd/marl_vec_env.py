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

    def _builders(self):
        """Per agent count: functions that build one dict per env from per-agent columns with a dict display (the
        fastest way CPython builds a small dict), for the envs whose agents are all live."""
        if getattr(self, "_mk", None) is None:
            ks = ", ".join(f"{str(k)!r}: a{i}" for i, k in enumerate(self._ids))
            args = ", ".join(f"a{i}" for i in range(self.num_drones))
            cols = ", ".join(f"c{i}" for i in range(self.num_drones))
            self._mk = eval(f"lambda {cols}: [{{{ks}}} for {args}, in zip({cols})]")   # noqa: S307 (built from agent ids)
            self._mk_all = eval(f"lambda {cols}, al: [{{{ks}, '__all__': z}} for {args}, z in zip({cols}, al)]")   # noqa: S307
        return self._mk, self._mk_all

    def step(self, action_dicts):
        """RLlibMultiAgentWrapper.step (marl_wrapper.py:77-119) for every env: ``action_dicts`` is a list of
        {agent_id: action} dicts (or an array [E, N, 4]); returns lists of per-env obs, rewards, dones, truncs
        and infos dicts keyed by the agents live at the start of the step, with ``"__all__"``.

        One launch, one ch_outputs_to_host into pinned buffers (observations, rewards, flags, the agent masks and
        the envs reset, with their terminal observations compacted on the device), then the dicts: built from
        per-agent columns for the envs whose agents were all live, trimmed to the live agents elsewhere.  The
        observation arrays are views of one fresh copy per step.  Every agent's info is the reference's
        ``{"answer": 42}`` (_computeInfo): one dict per step shared by all agents of all envs."""
        b = self.batch
        torch = b.torch
        E, N = self.num_envs, self.num_drones
        if isinstance(action_dicts, (list, tuple)):
            a = np.zeros((E, N, 4), np.float32)
            for e, d in enumerate(action_dicts):
                for aid, act in d.items():
                    a[e, int(str(aid).split("_")[1])] = np.asarray(act, np.float32)
            acts = torch.from_numpy(a).to(b.device, non_blocking=True)
        else:
            acts = torch.as_tensor(np.asarray(action_dicts, np.float32)).to(b.device, non_blocking=True)
        live = self._active
        if self._before is None:
            raise RuntimeError("call reset() first")
        b.step(acts, autoreset=True, terminal_obs=True)
        self._before = b.agent_active.view(torch.bool).clone()
        if getattr(self, "_host", None) is None:
            self._host = b.host_outputs(ring=2, ended=True, agents=True)
        h = self._host.fetch()
        obs = h["obs"].copy()
        ended_env = h["ended_env"]
        ended = h["reset_happened"].astype(bool)
        if len(ended_env):
            # the dicts carry the episode's last observation; reset_at() hands out the new episode's
            self._reset_obs = {int(e): obs[e].copy() for e in ended_env}
            obs[ended_env] = h["ended_obs"]
        self._reset_envs = set(self._reset_obs) if len(ended_env) else set()
        mk, mk_all = self._builders()
        al = ended.tolist()
        obs_l = mk(*[list(obs[:, i]) for i in range(N)])
        rew_l = mk(*h["reward"].astype(np.float64).T.tolist())
        done_l = mk_all(*h["terminated"].astype(bool).T.tolist(), al)
        trunc_l = mk_all(*h["truncated"].astype(bool).T.tolist(), al)
        info = {"answer": 42}
        info_l = mk(*([[info] * E] * N))
        # envs with agents that were not live at the start of the step: only the live agents' keys
        part = np.nonzero(~live.all(axis=1))[0]
        if len(part):
            ids = self._ids
            for e in part.tolist():
                for i in np.nonzero(~live[e])[0].tolist():
                    k = ids[i]
                    for dl in (obs_l, rew_l, done_l, trunc_l, info_l):
                        del dl[e][k]
        self._active = h["agent_active"].astype(bool)
        if len(ended_env):
            self._n = np.where(ended, self._active.sum(1), self._n)   # every agent of a new episode is live
        return obs_l, rew_l, done_l, trunc_l, info_l

    def reset_at(self, e):
        """What RLlibMultiAgentWrapper.reset returns for env ``e`` after its episode ended (``"__all__"`` in the
        last step): the device already reset it in that step's launch."""
        if e not in self._reset_envs:
            raise ValueError(f"env {e} did not finish an episode in the last step")
        n = int(self._n[e])
        obs = self._reset_obs[e] if isinstance(self._reset_obs, dict) else self._reset_obs[e]
        return self._obs_dict(obs, n), {self._ids[i]: {} for i in range(n)}

    def close(self):
        self.batch.close()
