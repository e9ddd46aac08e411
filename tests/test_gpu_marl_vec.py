"""GPU tests of the batched RLlib multi-agent surface (cattleherd.marl_vec_env.CattleHerdMultiAgentVecEnv, the
configs[4] path): per-env wrapper dicts against the reference's own MARL rollouts (rllib_envs/marl_wrapper.py:
77-119 run by tests/golden/make_golden.py), one env per fixture step, and the episode end -- "__all__", the
in-launch reset and reset_at -- against the fp64 oracle.  Tolerances as in test_gpu_parity.py: observations rtol
1e-6 / atol 1e-7 (the f32 output cast), rewards rtol 1e-6 (the f32 buffer), flags and agent ids exact."""
import numpy as np
import pytest

from helpers import close, oracle_view
from marl_replay import replay_marl_fixture

pytestmark = pytest.mark.gpu

_SKIP = ("m", "ctor_level", "episode_len")


@pytest.mark.parametrize("fname", ["marl_roll_n3_m8_l0.npz", "marl_roll_n4_m16_l4.npz"])
def test_marl_vec_env_dicts_replay_reference(fname):
    """Env t of the batch starts from the fixture's state t (its live agents included) and takes action t:
    every env's dicts carry the agents live at the start, the reference's obs / reward / done / trunc per
    agent, and "__all__"."""
    replay_marl_fixture(fname)


def test_marl_vec_env_episode_end_and_reset_at_vs_oracle():
    """Level 2 ends an episode when the drone centroid reaches the herd's (CattleAviary curriculum, terminated
    for every agent at once): half the envs get their drones placed around their herd centroid after a random
    rollout.  Those envs report "__all__", their dicts hold the episode's last observations, reset_at gives the
    new episode, all equal to the oracle stepping the same state with the wrapper semantics and auto-reset."""
    import torch
    import oracle as O
    from cattleherd._lib import spawn_table
    from cattleherd.marl_vec_env import CattleHerdMultiAgentVecEnv
    E, n, m = 64, 3, 8
    venv = CattleHerdMultiAgentVecEnv(E, {"num_drones": n, "num_cattle": m, "curriculum_level": 2,
                                          "min_drones": n, "max_drones": n})
    venv.reset()
    rng = np.random.default_rng(5)
    for _ in range(20):
        venv.step_tensors(torch.tensor(rng.uniform(-1, 1, (E, n, 4)).astype(np.float32), device=venv.batch.device))
    s = venv.batch.get_state()
    close_envs = np.arange(0, E, 2)
    for e in close_envs:
        c = s["cow_pos"][e].mean(0)
        for k, dx in enumerate((-0.6, 0.0, 0.6)):
            s["drone_pos"][e, k] = (c[0] + dx, c[1], 0.45)
            s["drone_vel"][e, k] = 0
    venv.batch.set_state(s)
    venv.refresh_agents()
    acts = rng.uniform(-0.05, 0.05, (E, n, 4)).astype(np.float32)
    g = venv.batch.get_state()
    o, r, dn, tr, inf = venv.step(acts)
    table = spawn_table(m)
    ended = 0
    for e in range(E):
        env = O.Env(1, n, m, table, env_id=e, start_level=2)
        env.set_state(oracle_view(g, e, O.NMAX))
        env.st.episode = int(g["episode"][e])
        want_o, want_r, want_te, want_tr, done, tobs = env.step(acts[e], autoreset=True)
        assert dn[e]["__all__"] == done, e
        last = tobs if done else want_o
        for i in range(n):
            a = f"agent_{i}"
            assert close(o[e][a], last[i], 1e-6, 1e-7)[0], (e, i)
            assert close([r[e][a]], [want_r[i]], 1e-6, 1e-6)[0], (e, i)
            assert dn[e][a] == bool(want_te[i]) and tr[e][a] == bool(want_tr[i]), (e, i)
        if done:
            ended += 1
            ro, ri = venv.reset_at(e)
            assert sorted(ro) == [f"agent_{i}" for i in range(n)] and all(v == {} for v in ri.values())
            for i in range(n):
                assert close(ro[f"agent_{i}"], want_o[i], 1e-6, 1e-7)[0], (e, i)
            assert venv.agents(e) == [f"agent_{i}" for i in range(n)]
        else:
            with pytest.raises(ValueError):
                venv.reset_at(e)
    assert ended >= len(close_envs) // 2, ended
    venv.close()
