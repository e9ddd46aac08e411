"""Test-only stand-in for cattleherd.env.HerdBatch backed by the CPU oracle.

Lets the CPU test suite exercise the host-side adapters (Gymnasium env, SB3 VecEnv, RLlib wrapper:
dict packing, agent bookkeeping, info keys, auto-reset plumbing) without a GPU.  It is injected by
monkeypatching in tests only; the product path never sees it.
"""
import numpy as np
import torch

import oracle as O
from helpers import stack


class _Cfg:
    def __init__(self, ctrl_freq, curriculum_level):
        self.ctrl_freq = ctrl_freq
        self.curriculum_level = -1 if curriculum_level is None else curriculum_level


class FakeBatch:
    def __init__(self, n_envs, num_drones, num_cattle, mode="ctde", device=None, compat=True, precision="f64",
                 min_drones=None, max_drones=None, curriculum_level=None, seed=0x5EED, env_id_offset=0,
                 damping=0.04, torque_world=True, gyro=True, ctrl_freq=60, pyb_freq=240, spawn_table=None,
                 marl_wrapper=True, physics="pyb"):
        from cattleherd._lib import PHYSICS, spawn_table as st
        self.torch = torch
        self.device = torch.device("cpu")
        self.mode = 0 if mode == "ctde" else 1
        table = st(num_cattle) if spawn_table is None else spawn_table
        self.envs = [O.Env(self.mode, num_drones, num_cattle, table, min_drones=min_drones, max_drones=max_drones,
                           start_level=curriculum_level, compat=compat, seed=seed, env_id=env_id_offset + e,
                           ctrl_freq=ctrl_freq, pyb_freq=pyb_freq, marl_wrapper=marl_wrapper,
                           physics=PHYSICS[getattr(physics, "value", physics)])
                     for e in range(n_envs)]
        self.cfg = _Cfg(ctrl_freq, curriculum_level)
        self.n_envs, self.num_drones, self.num_cattle = n_envs, num_drones, num_cattle
        self.obs_rows = 12 if self.mode == 0 else num_drones
        self.reward_cols = 1 if self.mode == 0 else num_drones
        E, R, K = n_envs, self.obs_rows, self.reward_cols
        self.obs = torch.zeros((E, R, 86))
        self.terminal_obs = torch.zeros_like(self.obs)
        self.reward = torch.zeros((E, K))
        self.terminated = torch.zeros((E, K), dtype=torch.uint8)
        self.truncated = torch.zeros((E, K), dtype=torch.uint8)
        self.agent_active = torch.zeros((E, num_drones), dtype=torch.uint8)
        self.actions = torch.zeros((E, num_drones, 4))
        self.reset_happened = torch.zeros(E, dtype=torch.uint8)
        self.episode_stats = torch.zeros((E, 2), dtype=torch.float64)   # as ch_step_io.episode_stats
        self._ret, self._len = np.zeros(E), np.zeros(E)
        self.step_index = 0

    def reset(self, mask=None):
        for e, env in enumerate(self.envs):
            if mask is None or bool(mask[e]):
                self.obs[e] = torch.from_numpy(env.reset())
        return self.obs

    def step(self, actions=None, autoreset=True, random_actions=False, terminal_obs=True):
        for e, env in enumerate(self.envs):
            a = env.random_actions(self.step_index) if random_actions else actions[e].cpu().numpy()
            self.actions[e] = torch.from_numpy(np.asarray(a, np.float32))
            o, r, te, tr, done, tobs = env.step(a, autoreset=autoreset)
            self.obs[e] = torch.from_numpy(o)
            self.reward[e] = torch.from_numpy(r.astype(np.float32))
            self.terminated[e] = torch.from_numpy(te)
            self.truncated[e] = torch.from_numpy(tr)
            self.agent_active[e] = torch.from_numpy(env.get_state()["active"][:self.num_drones])
            self._ret[e] += float(np.sum(r[np.isfinite(r)])) if self.mode else float(r[0])
            self._len[e] += 1
            if done:
                self.episode_stats[e, 0], self.episode_stats[e, 1] = self._ret[e], self._len[e]
                self._ret[e], self._len[e] = 0.0, 0.0
            self.reset_happened[e] = int(done and autoreset)
            if done and autoreset:
                self.terminal_obs[e] = torch.from_numpy(tobs)
        self.step_index += 1
        return self.obs, self.reward, self.terminated, self.truncated

    def get_state(self):
        s = stack([env.get_state() for env in self.envs])
        s["drone_pos"] = s["drone_pos"][:, :self.num_drones]
        return s

    def set_state(self, s):
        for e, env in enumerate(self.envs):
            env.set_state({k: np.asarray(v)[e] for k, v in s.items()})

    def env_ints(self):
        s = stack([env.get_state() for env in self.envs])
        out = {k: np.asarray(s[k], np.int64) for k in ("n", "step_counter", "step_counter_A")}
        act = np.asarray(s["active"], np.int64)[:, :self.num_drones]
        out["active_mask"] = (act << np.arange(self.num_drones)[None, :]).sum(1)
        return out

    def eval_distances(self):
        return np.stack([env.get_state()["eval_dist"][:self.num_drones] for env in self.envs])

    def invalidate_obs(self):
        pass

    def host_outputs(self, ring=2, ended=True, agents=False):
        return _FakeHostOutputs(self)

    def metrics(self, reset=False):
        return np.zeros(8)

    def close(self):
        pass


class _FakeHostOutputs:
    """HostOutputs.fetch() of the CPU stand-in: the same dict of numpy arrays, the reset envs listed ascending."""

    def __init__(self, batch):
        self.b = batch

    def fetch(self):
        b = self.b
        idx = np.nonzero(b.reset_happened.numpy())[0]
        return {"obs": b.obs.numpy().astype(np.float32), "reward": b.reward.numpy().astype(np.float32),
                "terminated": b.terminated.numpy().copy(), "truncated": b.truncated.numpy().copy(),
                "reset_happened": b.reset_happened.numpy().copy(), "agent_active": b.agent_active.numpy().copy(),
                "ended_env": idx.astype(np.int64), "ended_obs": b.terminal_obs.numpy()[idx].astype(np.float32),
                "ended_stats": b.episode_stats.numpy()[idx].copy()}
