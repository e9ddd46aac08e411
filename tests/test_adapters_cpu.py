"""CPU tests of the host-side adapters (drop-in surfaces) over an oracle-backed FakeBatch:
the reference's RLlib wrapper dicts (marl_wrapper.py:77-119), the Gymnasium CattleAviary
reset/step contract (sb3_envs/BaseAviary.py:280-465) and the SB3 VecEnv auto-reset info keys."""
import numpy as np
import pytest

from fake_batch import FakeBatch
from helpers import close, load, state_at


@pytest.fixture
def patched(monkeypatch):
    import importlib
    ve = importlib.import_module("cattleherd.vec_env")
    ma = importlib.import_module("gym_pybullet_drones.rllib_envs.MARLCattleAviary")
    ca = importlib.import_module("gym_pybullet_drones.sb3_envs.CattleAviary")
    for mod in (ca, ma, ve):
        monkeypatch.setattr(mod, "HerdBatch", FakeBatch)
    return ca, ma, ve


def test_rllib_wrapper_reproduces_reference_dicts(patched):
    """Replay the golden RLlib wrapper rollout: same agent ids, rewards, dones, truncs, __all__."""
    from gym_pybullet_drones.rllib_envs.marl_wrapper import RLlibMultiAgentWrapper
    d = load("marl_roll_n3_m8_l0.npz")
    s0 = state_at(d, "state_", 0)
    n = int(s0["n"])
    w = RLlibMultiAgentWrapper({"num_drones": n, "num_cattle": int(s0["m"]), "obs": "cokin", "act": "vel",
                                "gui": False, "record": False, "unknown_key": 1})
    obs, infos = w.reset()
    assert sorted(obs) == [f"agent_{i}" for i in range(n)] and all(v == {} for v in infos.values())
    assert w.get_observation_space("agent_0").shape == (86,) and w.get_action_space("agent_0").shape == (4,)
    w.env.batch.set_state({k: np.asarray(v)[None] for k, v in s0.items() if k not in ("m", "ctor_level", "episode_len")})
    for t in range(40):
        st = state_at(d, "state_", t)
        o, r, dn, tr, inf = w.step({f"agent_{i}": d["action"][t][i] for i in range(n)})
        act = [i for i in range(n) if st["active"][i]]
        assert sorted(o) == [f"agent_{i}" for i in act]
        for i in act:
            assert close(o[f"agent_{i}"], d["obs"][t][i], 1e-6, 1e-7)[0]
            assert close([r[f"agent_{i}"]], [d["reward"][t][i]], 1e-6, 1e-6)[0]  # float32 reward buffer
            assert dn[f"agent_{i}"] == bool(d["terminated"][t][i]) and tr[f"agent_{i}"] == bool(d["truncated"][t][i])
        assert dn["__all__"] == bool(d["all_done"][t]) and tr["__all__"] == dn["__all__"]


def test_marl_env_bare_dicts(patched):
    """MARLCattleAviary.step returns the bare env.step dicts keyed by drone index with __all__."""
    _, ma, _ = patched
    env = ma.MARLCattleAviary(num_drones=3, num_cattle=8)
    obs, info = env.reset()
    assert sorted(obs) == [0, 1, 2] and info == {"__all__": {}}
    o, r, d, t, i = env.step(np.zeros((3, 4), np.float32))
    assert set(d) == {0, 1, 2, "__all__"} and set(t) == {0, 1, 2, "__all__"}
    assert d["__all__"] == all(d[k] for k in range(3))


def test_gym_cattle_aviary_contract(patched):
    """reset → (obs (12,86) float32, {'answer': 42}); step → 5-tuple; 2 drones → NaN reward quirk."""
    ca, _, _ = patched
    env = ca.CattleAviary(num_drones=4, num_cattle=16)
    assert env.EPISODE_LEN_SEC == 80 and env.CTRL_FREQ == 60 and env.action_space.shape == (4, 4)
    obs, info = env.reset(seed=42, options={})
    assert obs.shape == (12, 86) and obs.dtype == np.float32 and info == {"answer": 42}
    assert env.NUM_DRONES == 4
    o, r, te, tr, inf = env.step(np.zeros((4, 4), np.float32))
    assert isinstance(r, float) and isinstance(te, bool) and isinstance(tr, bool) and inf == {"answer": 42}
    env2 = ca.CattleAviary(num_drones=2, num_cattle=8)
    env2.reset()
    _, r2, _, _, _ = env2.step(np.zeros((2, 4), np.float32))
    assert np.isnan(r2)


def test_gym_cattle_aviary_unsupported_options(patched):
    ca, _, _ = patched
    with pytest.raises(NotImplementedError):
        ca.CattleAviary(num_drones=4, num_cattle=4, act="rpm")
    with pytest.raises(ValueError):
        ca.CattleAviary(num_drones=4, num_cattle=4, pyb_freq=250)


def test_vec_env_autoreset_infos(patched):
    """SB3 VecEnv semantics: done = terminated | truncated, auto-reset inside step, terminal_observation
    and TimeLimit.truncated in infos."""
    _, _, ve = patched
    venv = ve.CattleHerdVecEnv(4, num_drones=4, num_cattle=16)
    obs = venv.reset()
    assert obs.shape == (4, 12, 86)
    rng = np.random.default_rng(0)
    saw_done = False
    for _ in range(150):
        obs, rew, dones, infos = venv.step(rng.uniform(-1, 1, (4, 4, 4)).astype(np.float32))
        assert obs.shape == (4, 12, 86) and rew.shape == (4,) and dones.shape == (4,)
        for e in np.nonzero(dones)[0]:
            saw_done = True
            assert infos[e]["terminal_observation"].shape == (12, 86)
            assert "TimeLimit.truncated" in infos[e]
    assert saw_done
    assert venv.get_attr("EPISODE_LEN_SEC") == [80] * 4 and venv.env_is_wrapped(object) == [False] * 4


def test_vec_env_outputs_kept_across_steps(patched):
    """A caller (callback, wrapper, user loop) that keeps a step's infos -- and, with copy_obs=True, its
    observations -- sees them unchanged after later steps, as with SubprocVecEnv's fresh arrays and dicts; with the
    default ring of pinned buffers the observations stay valid for obs_ring - 1 more steps (SB3's collect_rollouts
    keeps the previous step's)."""
    import copy
    _, _, ve = patched
    rng = np.random.default_rng(1)
    for copy_obs in (True, False):
        venv = ve.CattleHerdVecEnv(4, num_drones=4, num_cattle=16, copy_obs=copy_obs, obs_ring=3)
        venv.reset()
        kept = []
        for t in range(12):
            obs, rew, dones, infos = venv.step(rng.uniform(-1, 1, (4, 4, 4)).astype(np.float32))
            kept.append((obs, obs.copy(), infos, copy.deepcopy(infos)))
            if dones.any():   # a step where infos carry terminal observations
                assert any("terminal_observation" in d for d in infos)
        for t, (obs, snap, infos, isnap) in enumerate(kept):
            assert len(infos) == 4
            for d, ds in zip(infos, isnap):
                assert d.keys() == ds.keys()
                for k in d:
                    assert np.array_equal(d[k], ds[k]) if k == "terminal_observation" else d[k] == ds[k]
            if copy_obs or t >= len(kept) - 2:   # ring of 3: this step and the two before it
                assert np.array_equal(obs, snap), t
        # no info dict is shared between envs or steps: mutating one leaks nowhere
        ids = [id(d) for _, _, infos, _ in kept for d in infos]
        assert len(set(ids)) == len(ids)
        kept[0][2][0]["mutated"] = True
        _, _, _, infos = venv.step(rng.uniform(-1, 1, (4, 4, 4)).astype(np.float32))
        assert all("mutated" not in d for d in infos)
    with pytest.raises(ValueError):
        ve.CattleHerdVecEnv(4, num_drones=4, num_cattle=16, obs_ring=1)


def test_physics_argument_reaches_the_batch(patched):
    """CattleAviary(physics=Physics.DYN) selects the explicit model (BaseAviary.py:1043-1118): no
    p.stepSimulation, so the cattle keep their positions; PYB moves them at their velocity."""
    ca, _, ve = patched
    from cattleherd.spaces import Physics
    moved = {}
    for ph in (Physics.DYN, Physics.PYB):
        env = ca.CattleAviary(num_drones=4, num_cattle=8, physics=ph)
        env.reset()
        p0 = env.batch.get_state()["cow_pos"].copy()
        env.step(np.zeros((4, 4), np.float32))
        moved[ph] = float(np.abs(env.batch.get_state()["cow_pos"] - p0).max())
    assert moved[Physics.DYN] == 0.0 and moved[Physics.PYB] > 0.0
    venv = ve.CattleHerdVecEnv(2, num_drones=4, num_cattle=8, physics="pyb_gnd_drag_dw")
    assert venv.reset().shape == (2, 12, 86)
    with pytest.raises(ValueError):
        ca.CattleAviary(num_drones=4, num_cattle=8, physics="rk4")


def test_rllib_wrapper_logs_step_exceptions(patched, tmp_path, monkeypatch):
    """The wrapper's failure-detection hook (marl_wrapper.py:87-95): an exception out of env.step() is appended
    with its traceback to the env-worker log, then re-raised; a good step writes nothing."""
    from gym_pybullet_drones.rllib_envs import marl_wrapper as mw
    log = tmp_path / "env_worker_exc.log"
    monkeypatch.setattr(mw, "EXC_LOG", str(log))
    w = mw.RLlibMultiAgentWrapper({"num_drones": 3, "num_cattle": 8})
    w.reset()
    w.step({f"agent_{i}": np.zeros(4, np.float32) for i in range(3)})
    assert not log.exists()

    def boom(actions):
        raise FloatingPointError("device step failed")
    monkeypatch.setattr(w.env, "_step_arrays", boom)
    for _ in range(2):
        with pytest.raises(FloatingPointError):
            w.step({"agent_0": np.zeros(4, np.float32)})
    text = log.read_text()
    assert text.count("=== Exception in env.step() ===") == 2 and "FloatingPointError: device step failed" in text
