"""Replay of the reference's MARL rollouts (tests/golden/marl_roll_*.npz: RLlibMultiAgentWrapper.step,
rllib_envs/marl_wrapper.py:77-119, run by make_golden.py) through the batched multi-agent surface, one env per
fixture step -- shared by the CPU test (oracle-backed FakeBatch) and the GPU test (the HIP batch)."""
import numpy as np

from helpers import close, load, stack, state_at

_SKIP = ("m", "ctor_level", "episode_len")


def replay_marl_fixture(fname):
    from cattleherd.marl_vec_env import CattleHerdMultiAgentVecEnv
    d = load(fname)
    T = len(d["action"])
    s0 = state_at(d, "state_", 0)
    n, m = int(s0["n"]), int(s0["m"])
    venv = CattleHerdMultiAgentVecEnv(T, {"num_drones": n, "num_cattle": m, "curriculum_level": int(d["level"]),
                                          "min_drones": n, "max_drones": n})
    obs0, infos0 = venv.reset()
    assert len(obs0) == T and sorted(obs0[0]) == [f"agent_{i}" for i in range(n)]
    assert all(v == {} for v in infos0[0].values())
    states = [state_at(d, "state_", t) for t in range(T)]
    s = stack(states)
    venv.batch.set_state({k: v for k, v in s.items() if k not in _SKIP})
    venv.refresh_agents()
    acts = [{f"agent_{i}": d["action"][t][i] for i in range(n)} for t in range(T)]
    o, r, dn, tr, inf = venv.step(acts)
    dropped = 0
    for t in range(T):
        live = [i for i in range(n) if states[t]["active"][i]]
        dropped += n - len(live)
        assert sorted(o[t]) == [f"agent_{i}" for i in live], t
        for i in live:
            a = f"agent_{i}"
            assert close(o[t][a], d["obs"][t][i], 1e-6, 1e-7)[0], (t, i)
            assert close([r[t][a]], [d["reward"][t][i]], 1e-6, 1e-6)[0], (t, i)
            assert dn[t][a] == bool(d["terminated"][t][i]) and tr[t][a] == bool(d["truncated"][t][i]), (t, i)
            assert inf[t][a] == {"answer": 42}
        assert dn[t]["__all__"] == bool(d["all_done"][t]) and tr[t]["__all__"] == dn[t]["__all__"], t
        # the next step's agents: the survivors
        assert venv.agents(t) == [f"agent_{i}" for i in live if not d["terminated"][t][i]], t
    venv.close()
    return dropped
