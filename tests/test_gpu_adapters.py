"""GPU tests of the drop-in surfaces over the real HIP batch (libcattleherd.so through HerdBatch):
the RLlib wrapper dicts (rllib_envs/marl_wrapper.py:77-119), the Gymnasium CattleAviary contract
(sb3_envs/CattleAviary.py:14-28, BaseAviary.py:280-465) and the SB3 VecEnv auto-reset semantics the
CTDE driver relies on (CTDECattleHerder.py:91-99, 185-220: terminal_observation, TimeLimit.truncated),
each replayed against the reference's own golden rollouts with state injection.

Tolerances as in test_gpu_parity.py: float32 outputs rtol 1e-6 / atol 1e-7, rewards (float32 buffer)
rtol 1e-6, flags and agent ids exact."""
import numpy as np
import pytest

from helpers import close, load, stack, state_at

pytestmark = pytest.mark.gpu

_SKIP = ("m", "ctor_level", "episode_len")


def _inject(batch, states):
    s = stack(states)
    batch.set_state({k: v for k, v in s.items() if k not in _SKIP})


def test_rllib_wrapper_replays_reference_dicts_on_gpu():
    """marl_roll_n3_m8_l0.npz through RLlibMultiAgentWrapper on the GPU: agent ids, per-agent obs,
    rewards, dones, truncs and __all__ (incl. finished agents dropping out), state injected before
    every step."""
    from gym_pybullet_drones.rllib_envs.marl_wrapper import RLlibMultiAgentWrapper
    d = load("marl_roll_n3_m8_l0.npz")
    s0 = state_at(d, "state_", 0)
    n = int(s0["n"])
    w = RLlibMultiAgentWrapper({"num_drones": n, "num_cattle": int(s0["m"]), "obs": "cokin", "act": "vel",
                                "gui": False, "record": False})
    obs, infos = w.reset()
    assert sorted(obs) == [f"agent_{i}" for i in range(n)] and all(v == {} for v in infos.values())
    assert w.get_observation_space("agent_0").shape == (86,) and w.get_action_space("agent_0").shape == (4,)
    T = len(d["action"])
    for t in range(T):
        st = state_at(d, "state_", t)
        _inject(w.env.batch, [st])
        w.agents = [f"agent_{i}" for i in range(n) if st["active"][i]]
        o, r, dn, tr, inf = w.step({f"agent_{i}": d["action"][t][i] for i in range(n)})
        act = [i for i in range(n) if st["active"][i]]
        assert sorted(o) == [f"agent_{i}" for i in act], t
        for i in act:
            assert close(o[f"agent_{i}"], d["obs"][t][i], 1e-6, 1e-7)[0], (t, i)
            assert close([r[f"agent_{i}"]], [d["reward"][t][i]], 1e-6, 1e-6)[0], (t, i)
            assert dn[f"agent_{i}"] == bool(d["terminated"][t][i]) and tr[f"agent_{i}"] == bool(d["truncated"][t][i])
        assert dn["__all__"] == bool(d["all_done"][t]) and tr["__all__"] == dn["__all__"], t
    assert T >= 100


def test_gym_cattle_aviary_replays_reference_rollout_on_gpu():
    """ctde_roll_n4_m16_l7.npz through the Gymnasium CattleAviary (E = 1): every step from the
    fixture state with the fixture action; obs (12, 86) float32, reward float, flags bool, info."""
    from gym_pybullet_drones.sb3_envs.CattleAviary import CattleAviary
    d = load("ctde_roll_n4_m16_l7.npz")
    env = CattleAviary(num_drones=4, num_cattle=16)
    assert env.EPISODE_LEN_SEC == 80 and env.CTRL_FREQ == 60 and env.action_space.shape == (4, 4)
    obs, info = env.reset(seed=42, options={})
    assert obs.shape == (12, 86) and obs.dtype == np.float32 and info == {"answer": 42}
    for t in range(0, len(d["action"]), 7):
        _inject(env.batch, [state_at(d, "state_", t)])
        env.batch.invalidate_obs()
        o, r, te, tr, inf = env.step(d["action"][t])
        assert isinstance(r, float) and isinstance(te, bool) and isinstance(tr, bool) and inf == {"answer": 42}
        assert close(o, d["obs"][t], 1e-6, 1e-7)[0], t
        assert close([r], [d["reward"][t]], 1e-6, 1e-6)[0], t
        assert te == bool(d["terminated"][t]) and tr == bool(d["truncated"][t]), t
    env.close()


@pytest.mark.parametrize("fname", ["ctde_roll_n4_m16_l7.npz", "ctde_roll_n3_m4_l7_timelimit.npz"])
def test_vec_env_autoreset_matches_reference_on_gpu(fname):
    """CattleHerdVecEnv with one env per fixture step (env t starts from state t): rewards, dones =
    terminated | truncated, SB3's terminal_observation = the reference's pre-reset obs,
    TimeLimit.truncated, and the auto-reset observation = the reference's reset obs."""
    import torch
    from cattleherd.vec_env import CattleHerdVecEnv
    d = load(fname)
    T = len(d["action"])
    s0 = state_at(d, "state_", 0)
    n, m = int(s0["n"]), int(s0["m"])
    venv = CattleHerdVecEnv(T, num_drones=n, num_cattle=m, min_drones=n, max_drones=n)
    venv.reset()
    _inject(venv.batch, [state_at(d, "state_", t) for t in range(T)])
    obs, rew, dones, infos = venv.step(d["action"].astype(np.float32))
    torch.cuda.synchronize()
    want_done = d["terminated"].astype(bool) | d["truncated"].astype(bool)
    assert np.array_equal(dones, want_done)
    assert close(rew, d["reward"], 1e-6, 1e-6)[0]
    resets = list(d["reset_at"])
    assert sorted(np.nonzero(dones)[0].tolist()) == sorted(resets)
    for k, t in enumerate(resets):
        assert close(infos[t]["terminal_observation"], d["obs"][t], 1e-6, 1e-7)[0], t
        assert infos[t]["TimeLimit.truncated"] == bool(d["truncated"][t] and not d["terminated"][t])
        assert close(obs[t], d["reset_obs"][k], 1e-6, 1e-7)[0], t
    keep = [t for t in range(T) if t not in resets]
    assert close(obs[keep], d["obs"][keep], 1e-6, 1e-7)[0]
    assert all("terminal_observation" not in infos[t] for t in keep)
    venv.close()


def test_vec_env_random_rollout_infos_on_gpu():
    """A random-action rollout of the batched VecEnv on the GPU: shapes, auto-resets with SB3 info
    keys, and the driver-facing attributes (get_attr / env_is_wrapped)."""
    from cattleherd.vec_env import CattleHerdVecEnv
    venv = CattleHerdVecEnv(64, num_drones=4, num_cattle=16)
    obs = venv.reset()
    assert obs.shape == (64, 12, 86)
    rng = np.random.default_rng(0)
    saw = 0
    for _ in range(120):
        obs, rew, dones, infos = venv.step(rng.uniform(-1, 1, (64, 4, 4)).astype(np.float32))
        assert obs.shape == (64, 12, 86) and rew.shape == (64,) and dones.shape == (64,)
        for e in np.nonzero(dones)[0]:
            saw += 1
            assert infos[e]["terminal_observation"].shape == (12, 86)
            assert "TimeLimit.truncated" in infos[e]
    assert saw > 0
    assert venv.get_attr("EPISODE_LEN_SEC") == [80] * 64 and venv.env_is_wrapped(object) == [False] * 64
    venv.close()


@pytest.mark.parametrize("n,m,compat", [(4, 16, True), (2, 8, False)])
def test_vec_env_monitor_episode_info_on_gpu(n, m, compat):
    """SB3 Monitor's info["episode"] (make_vec_env wraps every env in one, CTDECattleHerder.py:91-99) from the
    batched VecEnv: for every env that ends an episode, "l" is the number of steps since its last reset and "r"
    the sum of the rewards it returned (the device sums the float64 rewards, the host here the float32 ones it
    received: rtol 1e-6), "t" the seconds since the env started, non-decreasing."""
    from cattleherd.vec_env import CattleHerdVecEnv
    E = 256
    venv = CattleHerdVecEnv(E, num_drones=n, num_cattle=m, compat=compat)
    venv.reset()
    rng = np.random.default_rng(1)
    ret, length = np.zeros(E), np.zeros(E, np.int64)
    seen, last_t = 0, 0.0
    for _ in range(400):
        obs, rew, dones, infos = venv.step(rng.uniform(-1, 1, (E, n, 4)).astype(np.float32))
        ret += rew.astype(np.float64)
        length += 1
        for e in range(E):
            if dones[e]:
                ep = infos[e]["episode"]
                assert set(ep) == {"r", "l", "t"} and ep["l"] == length[e], (e, ep, length[e])
                assert np.isclose(ep["r"], ret[e], rtol=1e-6, atol=1e-5), (e, ep["r"], ret[e])
                assert ep["t"] >= last_t
                last_t = ep["t"]
                ret[e], length[e] = 0.0, 0
                seen += 1
            else:
                assert "episode" not in infos[e]
    assert seen > 50, seen
    venv.close()
