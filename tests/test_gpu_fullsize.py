"""Parity at the BASELINE sizes themselves (-m gpu): configs[3]'s 4096 envs x (4 drones, 16 cattle) after
a long random rollout, spot-checked env by env against the fp64 oracle for one step, and configs[0]'s single
env with one drone and 4 cattle (the reference's CPU case; compat = 0, since one drone in compat mode is the
reference's own ValueError), stepped in lockstep with the oracle.  Tolerances as in test_gpu_parity.py: obs
rtol 1e-6 / atol 1e-7 (the f32 output cast), reward rtol 1e-6, state 1e-9, flags exact."""
import numpy as np
import pytest

from helpers import close, oracle_view as _oracle_view

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,m,compat", [(4, 16, True), (2, 8, True), (2, 8, False)],
                         ids=["configs3", "configs2_compat", "configs2_training"])
def test_full_size_spot_parity(n, m, compat):
    """4096 envs, 300 device-drawn random steps with auto-reset, then one step with host actions; 64 envs
    (a fixed random sample, incl. the first and last workgroup) re-run that step on the oracle from the
    device state before it.  configs[3]'s (4, 16) and configs[2]'s (2, 8) -- the latter with the reference's
    quirks (compat: the 2-drone CTDE reward is NaN on every step, CattleAviary.py:234-246) and NaN-safe as its
    PPO training leg runs it (compat = 0: finite rewards)."""
    import torch
    import oracle as O
    from cattleherd._lib import spawn_table
    from cattleherd.env import HerdBatch
    E = 4096
    b = HerdBatch(E, n, m, compat=compat)
    b.reset()
    for _ in range(300):
        b.step(random_actions=True, autoreset=True)
    torch.cuda.synchronize()
    g = b.get_state()
    rng = np.random.default_rng(11)
    pick = np.unique(np.concatenate([[0, 1, 15, 16, E - 16, E - 1], rng.choice(E, 58, replace=False)]))
    acts = rng.uniform(-1, 1, (E, n, 4)).astype(np.float32)
    # no terminal observation requested: the workgroups take the sync-free auto-reset path
    obs, rew, te, tr = b.step(torch.tensor(acts, device=b.device), autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    obs, rew, te, tr = obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy(), tr.cpu().numpy()
    resets = np.nonzero(b.reset_happened.cpu().numpy())[0]
    assert len(resets) >= 4, "the checked step should auto-reset some envs"
    pick = np.unique(np.concatenate([pick, resets[:24]]))
    after = b.get_state()
    table = spawn_table(m)
    if compat and n == 2:
        assert np.isnan(rew).all()
    else:
        assert np.isfinite(rew).all()
    for e in pick:
        env = O.Env(0, n, m, table, env_id=int(e), compat=compat)
        env.set_state(_oracle_view(g, e, O.NMAX))
        env.st.episode = int(g["episode"][e])   # (set_state leaves the reset counter to the env's own resets)
        o, r, t1, t2, done, _ = env.step(acts[e], autoreset=True)
        assert close(obs[e], np.asarray(o).reshape(obs[e].shape), 1e-6, 1e-7)[0], e
        assert close(rew[e], np.asarray(r, np.float32).reshape(rew[e].shape), 1e-6, 1e-6)[0], e
        assert np.array_equal(te[e], np.asarray(t1).reshape(te[e].shape)), e
        assert np.array_equal(tr[e], np.asarray(t2).reshape(tr[e].shape)), e
        want = env.get_state()
        for k in ("drone_pos", "drone_quat", "drone_vel", "drone_angv"):
            assert close(after[k][e][:n], want[k][:n], 1e-9, 1e-9)[0], (e, k)
        assert close(after["cow_pos"][e], want["cow_pos"][:m], 1e-12, 1e-13)[0], e
        assert close(after["cow_vel"][e], want["cow_vel"][:m], 1e-9, 1e-12)[0], e
        assert int(after["step_counter"][e]) == int(want["step_counter"]), e
    assert len(pick) >= 60
    b.close()


@pytest.mark.parametrize("physics,precision", [("pyb", "f64"), ("pyb_gnd_drag_dw", "f64"), ("pyb", "f32")])
def test_sync_free_reset_path_equals_synced_path(physics, precision):
    """At configs[3]'s size the step kernel rebuilds auto-reset envs without a cow-wave sync when no terminal
    observation is requested, and through the drained, synced path when one is: 150 steps of both from the
    same start give bit-identical observations, rewards, flags and state, step by step (default physics and
    the all-effects variant, whose carried rpm / body rates a reset also clears)."""
    import torch
    from cattleherd.env import HerdBatch
    E, n, m = 4096, 4, 16
    hs = [HerdBatch(E, n, m, physics=physics, precision=precision), HerdBatch(E, n, m, physics=physics, precision=precision)]
    for h in hs:
        h.reset()
    nres = 0
    for t in range(150):
        hs[0].step(random_actions=True, autoreset=True, terminal_obs=True)
        hs[1].step(random_actions=True, autoreset=True, terminal_obs=False)
        for x, y in ((hs[0].obs, hs[1].obs), (hs[0].reward, hs[1].reward), (hs[0].terminated, hs[1].terminated),
                     (hs[0].truncated, hs[1].truncated), (hs[0].reset_happened, hs[1].reset_happened)):
            assert np.array_equal(x.cpu().numpy(), y.cpu().numpy(), equal_nan=x.dtype.is_floating_point), t
        nres += int(hs[0].reset_happened.sum())
    s0, s1 = hs[0].get_state(), hs[1].get_state()
    for k in s0:
        assert np.array_equal(np.asarray(s0[k]), np.asarray(s1[k]), equal_nan=np.asarray(s0[k]).dtype.kind == "f"), k
    assert nres > 500, nres
    for h in hs:
        h.close()


def test_configs0_one_env_one_drone_lockstep():
    """configs[0]: 1 env x (1 drone, 4 cattle), compat = 0 (NaN-safe spacing terms with a single drone),
    240 device-drawn random steps with auto-reset, the oracle taking the device state before every step."""
    import torch
    import oracle as O
    from cattleherd._lib import spawn_table
    from cattleherd.env import HerdBatch
    n, m, T = 1, 4, 240
    b = HerdBatch(1, n, m, compat=False)
    b.reset()
    table = spawn_table(m)
    env = O.Env(0, n, m, table, env_id=0, compat=False)
    o0 = env.reset()
    assert close(b.obs.cpu().numpy()[0], np.asarray(o0).reshape(12, 86), 1e-6, 1e-7)[0]
    for t in range(T):
        g = b.get_state()
        env.set_state(_oracle_view(g, 0, O.NMAX))
        env.st.episode = int(g["episode"][0])
        b.step(random_actions=True, autoreset=True)
        torch.cuda.synchronize()
        a = env.random_actions(t)
        assert np.array_equal(a, b.actions.cpu().numpy()[0]), t
        o, r, te, tr, done, _ = env.step(a, autoreset=True)
        assert close(b.obs.cpu().numpy()[0], np.asarray(o).reshape(12, 86), 1e-6, 1e-7)[0], t
        rr = b.reward.cpu().numpy()[0]
        assert np.isfinite(rr).all(), t
        assert close(rr, np.asarray(r, np.float32).reshape(rr.shape), 1e-6, 1e-6)[0], t
        assert bool(b.terminated.cpu().numpy()[0][0]) == bool(np.asarray(te).ravel()[0]), t
        assert bool(b.truncated.cpu().numpy()[0][0]) == bool(np.asarray(tr).ravel()[0]), t
    b.close()
