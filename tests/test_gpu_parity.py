"""GPU parity tests: the HIP path (libcattleherd.so via its C ABI) against the reference's golden
vectors and against the CPU oracle on identical seeded inputs.

Tolerances (stated per north_star's fp32 bar, tighter for the fp64 path):
  fp64 path: obs (float32 outputs) rtol 1e-6 / atol 1e-7; reward (float32 output buffer) rtol 1e-6;
             next state rtol 1e-9 (measured: <= 5e-14 abs vs the reference); flags exact.
             240-step rollouts run in lockstep (the oracle takes the device state before each step:
             1-ulp libm differences between ocml and glibc would otherwise grow through the closed
             loop to ~1e-3 m): actions / flags / resets exact, obs / reward / state as above.
  fp32 path: obs / reward / state rtol 1e-4 (the north_star's 1e-4 relative), flags on >= 99 %.
"""
import numpy as np
import pytest

from helpers import close, load, rollout_files, stack, state_at

pytestmark = pytest.mark.gpu


def _batch(mode, n, m, E, ctor_level, **kw):
    from cattleherd.env import HerdBatch
    return HerdBatch(E, n, m, mode="ctde" if mode == 0 else "marl", curriculum_level=ctor_level, **kw)


def _inject(b, states):
    s = stack(states)
    s = {k: v for k, v in s.items() if k not in ("m", "ctor_level", "episode_len")}
    b.set_state(s)


@pytest.mark.parametrize("fname", rollout_files())
def test_rollout_fixture_parity(fname):
    """Every step of each golden rollout, batched: env t starts from fixture state t and takes
    fixture action t; one launch steps them all."""
    import torch
    d = load(fname)
    mode = 0 if fname.startswith("ctde") else 1
    T = len(d["action"])
    states = [state_at(d, "state_", t) for t in range(T)]
    n, m, lvl = int(states[0]["n"]), int(states[0]["m"]), int(states[0]["ctor_level"])
    physics = int(d["physics"]) if "physics" in d.files else 0   # Physics enum (BaseAviary.py:420-450)
    b = _batch(mode, n, m, T, lvl, physics=physics)
    b.reset()
    _inject(b, states)
    acts = torch.tensor(d["action"], device=b.device)
    obs, rew, te, tr = b.step(acts, autoreset=False)
    torch.cuda.synchronize()
    obs, rew, te, tr = obs.cpu().numpy(), rew.cpu().numpy(), te.cpu().numpy(), tr.cpu().numpy()
    if mode == 0:
        assert close(obs, d["obs"], 1e-6, 1e-7)[0]
        assert close(rew[:, 0], d["reward"], 1e-6, 1e-6)[0]
        assert np.array_equal(te[:, 0], d["terminated"]) and np.array_equal(tr[:, 0], d["truncated"])
    else:
        act = np.stack([s["active"][:n] for s in states]).astype(bool)
        assert close(obs[act], d["obs"][act], 1e-6, 1e-7)[0]
        assert close(rew[act], d["reward"][act], 1e-6, 1e-6)[0]
        assert np.array_equal(te[act], d["terminated"][act]) and np.array_equal(tr[act], d["truncated"][act])
    g = b.get_state()
    resets = set(d["reset_at"].tolist())
    idx = [t for t in range(T - 1) if t not in resets]
    nxt = stack([states[t + 1] for t in idx])
    for k in ("drone_pos", "drone_quat", "drone_vel", "drone_angv", "pid_int_rpy", "pid_int_pos", "pid_last_rpy",
              "drone_qlag"):
        assert close(g[k][idx, :n], nxt[k][:, :n], 1e-9, 1e-12)[0], k
    if physics:
        assert close(g["last_rpm"][idx, :n], nxt["last_rpm"][:, :n], 1e-9, 1e-9)[0]
        assert close(g["rpy_rates"][idx, :n], nxt["rpy_rates"][:, :n], 1e-9, 1e-12)[0]
    assert close(g["cow_pos"][idx, :m], nxt["cow_pos"][:, :m], 1e-12, 1e-13)[0]
    assert close(g["cow_vel"][idx, :m], nxt["cow_vel"][:, :m], 1e-12, 1e-14)[0]
    for k in ("step_counter", "step_counter_A", "level", "tally"):
        assert np.array_equal(g[k][idx], nxt[k]), k
    b.close()


def _oracle_states(mode, n, m, E, table, steps, seed, level, compat=True, physics=0):
    """E oracle envs, each advanced a different number of random steps (diverse states)."""
    import oracle as O
    envs, states = [], []
    rng = np.random.default_rng(seed)
    for e in range(E):
        env = O.Env(mode, n, m, table, start_level=level, env_id=e, compat=compat, physics=physics)
        env.reset()
        for t in range(int(rng.integers(0, steps))):
            env.step(rng.uniform(-1, 1, (n, 4)).astype(np.float32), autoreset=True)
        envs.append(env)
        states.append(env.get_state())
    return envs, states


@pytest.mark.parametrize("mode,n,m,level,compat", [
    (0, 4, 16, 7, True), (0, 2, 8, 7, True), (0, 12, 16, 7, True), (0, 5, 16, 0, True), (0, 4, 16, 4, True),
    (0, 3, 4, 2, True), (0, 2, 8, 7, False), (1, 3, 8, 0, True), (1, 4, 32, 0, True), (1, 4, 16, 6, True),
    (1, 6, 16, 1, False), (0, 4, 32, 7, True), (0, 8, 64, 7, True)])
def test_step_vs_oracle(mode, n, m, level, compat):
    """One GPU launch over E diverse states vs the oracle stepping each state (no auto-reset)."""
    import torch
    from cattleherd._lib import spawn_table
    table = spawn_table(m)
    E = 48
    envs, states = _oracle_states(mode, n, m, E, table, 160, seed=n * 100 + m + level, level=level, compat=compat)
    b = _batch(mode, n, m, E, level, compat=compat)
    b.reset()
    b.set_state(stack([{k: v for k, v in s.items() if k != "episode"} for s in states]))
    rng = np.random.default_rng(7)
    acts = rng.uniform(-1, 1, (E, n, 4)).astype(np.float32)
    obs, rew, te, tr = b.step(torch.tensor(acts, device=b.device), autoreset=False)
    torch.cuda.synchronize()
    ref = [env.step(acts[e], autoreset=False) for e, env in enumerate(envs)]
    R = b.obs_rows
    assert close(obs.cpu().numpy(), np.stack([r[0] for r in ref]).reshape(E, R, 86), 1e-6, 1e-7)[0]
    K = b.reward_cols
    rr = np.stack([r[1] for r in ref]).reshape(E, K)
    assert close(rew.cpu().numpy(), rr.astype(np.float32), 1e-6, 1e-6)[0]
    assert np.array_equal(te.cpu().numpy(), np.stack([r[2] for r in ref]).reshape(E, K))
    assert np.array_equal(tr.cpu().numpy(), np.stack([r[3] for r in ref]).reshape(E, K))
    g = b.get_state()
    want = stack([env.get_state() for env in envs])
    for k in ("drone_pos", "drone_quat", "drone_vel", "drone_angv", "pid_int_rpy", "pid_int_pos", "pid_last_rpy",
              "drone_qlag"):
        assert close(g[k][:, :n], want[k][:, :n], 1e-9, 1e-12)[0], k
    assert close(g["cow_pos"], want["cow_pos"][:, :m], 1e-12, 1e-13)[0]
    assert close(g["cow_vel"], want["cow_vel"][:, :m], 1e-12, 1e-14)[0]
    for k in ("step_counter", "step_counter_A", "level", "tally", "has_prev", "spawn_index"):
        assert np.array_equal(g[k], want[k]), k
    assert close(g["clock"], want["clock"], 1e-12, 1e-12)[0]
    if mode == 1:
        assert np.array_equal(g["active"][:, :n], want["active"][:, :n])
    b.close()


PHYSICS_CASES = [(1, 0, 4, 16), (2, 0, 4, 16), (3, 0, 4, 16), (4, 0, 6, 8), (5, 0, 4, 16), (5, 1, 4, 16),
                 (1, 1, 3, 8), (5, 0, 12, 16)]


@pytest.mark.parametrize("physics,mode,n,m", PHYSICS_CASES)
def test_physics_variant_step_vs_oracle(physics, mode, n, m):
    """Physics variants (DYN 1, PYB_GND 2, PYB_DRAG 3, PYB_DW 4, PYB_GND_DRAG_DW 5;
    BaseAviary.py:420-450, 943-1118): one launch over E diverse oracle states, including the
    carried last_clipped_action and DYN body rates, vs the oracle stepping each state."""
    import torch
    from cattleherd._lib import spawn_table
    table = spawn_table(m)
    E = 48
    level = 7 if mode == 0 else 0
    envs, states = _oracle_states(mode, n, m, E, table, 160, seed=physics * 1000 + n * 100 + m, level=level,
                                  physics=physics)
    b = _batch(mode, n, m, E, level, physics=physics)
    b.reset()
    b.set_state(stack([{k: v for k, v in s.items() if k != "episode"} for s in states]))
    rng = np.random.default_rng(11)
    acts = rng.uniform(-1, 1, (E, n, 4)).astype(np.float32)
    obs, rew, te, tr = b.step(torch.tensor(acts, device=b.device), autoreset=False)
    torch.cuda.synchronize()
    ref = [env.step(acts[e], autoreset=False) for e, env in enumerate(envs)]
    R, K = b.obs_rows, b.reward_cols
    assert close(obs.cpu().numpy(), np.stack([r[0] for r in ref]).reshape(E, R, 86), 1e-6, 1e-7)[0]
    assert close(rew.cpu().numpy(), np.stack([r[1] for r in ref]).reshape(E, K).astype(np.float32), 1e-6, 1e-6)[0]
    assert np.array_equal(te.cpu().numpy(), np.stack([r[2] for r in ref]).reshape(E, K))
    assert np.array_equal(tr.cpu().numpy(), np.stack([r[3] for r in ref]).reshape(E, K))
    g = b.get_state()
    want = stack([env.get_state() for env in envs])
    for k in ("drone_pos", "drone_quat", "drone_vel", "drone_angv", "pid_int_rpy", "pid_int_pos", "pid_last_rpy",
              "rpy_rates", "drone_qlag"):
        assert close(g[k][:, :n], want[k][:, :n], 1e-9, 1e-12)[0], k
    assert close(g["last_rpm"][:, :n], want["last_rpm"][:, :n], 1e-12, 1e-9)[0]
    assert close(g["cow_pos"], want["cow_pos"][:, :m], 1e-12, 1e-13)[0]
    assert close(g["cow_vel"], want["cow_vel"][:, :m], 1e-12, 1e-14)[0]
    b.close()


def _oracle_view(g, e, nmax):
    """Env e of a HerdBatch.get_state() dict in the oracle's NMAX-padded layout."""
    out = {}
    for k, v in g.items():
        x = np.asarray(v[e])
        if k in ("drone_pos", "drone_quat", "drone_vel", "drone_angv", "pid_last_rpy", "pid_int_pos", "pid_int_rpy",
                 "last_rpm", "rpy_rates", "active", "drone_qlag"):
            pad = np.zeros((nmax,) + x.shape[1:], x.dtype)
            pad[:x.shape[0]] = x
            if k in ("drone_quat", "drone_qlag"):
                pad[x.shape[0]:, 3] = 1
            x = pad
        out[k] = x
    return out


@pytest.mark.parametrize("physics,mode,n,m", [("pyb", 0, 4, 16), ("pyb", 1, 4, 16), ("pyb", 0, 2, 8),
                                               ("dyn", 0, 4, 16), ("dyn_rk4", 0, 4, 16), ("dyn_rk4", 0, 2, 8),
                                               ("pyb_gnd_drag_dw", 0, 4, 16),
                                               ("pyb_gnd_drag_dw", 1, 3, 8)])
def test_random_rollout_with_autoreset_vs_oracle(physics, mode, n, m):
    """240 lockstep steps of device Philox actions with in-kernel auto-reset: before every step the
    oracle envs take the device state, so the 1-ulp ocml/glibc transcendental differences cannot
    grow through the closed loop (free-running, they reach ~1e-3 m in drone position after 240
    steps), then both step.  Actions, flags and reset timing exact; obs / reward to the per-step
    tolerances; the carried physics-variant state zeroed on reset."""
    import torch
    import oracle as O
    from cattleherd._lib import PHYSICS, spawn_table
    E, T = 16, 240
    ph = PHYSICS[physics]
    table = spawn_table(m)
    b = _batch(mode, n, m, E, None, physics=physics)
    b.reset()
    envs = [O.Env(mode, n, m, table, env_id=e, physics=ph) for e in range(E)]
    o0 = np.stack([env.reset() for env in envs])
    assert close(b.obs.cpu().numpy(), o0, 1e-6, 1e-7)[0]
    if mode == 1:
        # a MARL episode ends only when every agent has terminated (marl_wrapper.py:113-117): half the envs start with
        # their drones 0.8 m apart and the level-0 spacing clock just short of its 10 s hold (curriculum_learning.py:13-34)
        # so that auto-resets happen inside the rollout whatever the physics does with random actions
        s = b.get_state()
        ev = np.arange(E) % 2 == 0
        s["drone_pos"][ev, :, 0] = 0.8 * np.arange(n)[None, :]
        s["drone_pos"][ev, :, 1] = 0.0
        s["clock"][ev] = 10.0 - 3.0 / 60
        b.set_state({"drone_pos": s["drone_pos"], "clock": s["clock"]})
    R, K = b.obs_rows, b.reward_cols
    resets = 0
    for t in range(T):
        g = b.get_state()
        for e, env in enumerate(envs):
            env.set_state(_oracle_view(g, e, O.NMAX))
        b.step(random_actions=True, autoreset=True)
        torch.cuda.synchronize()
        acts = b.actions.cpu().numpy()
        ref = []
        for e, env in enumerate(envs):
            a = env.random_actions(t)
            assert np.array_equal(a, acts[e]), (t, e)
            ref.append(env.step(a, autoreset=True))
        assert close(b.obs.cpu().numpy(), np.stack([r[0] for r in ref]).reshape(E, R, 86), 1e-6, 1e-7)[0], t
        want_r = np.stack([r[1] for r in ref]).reshape(E, K).astype(np.float32)
        assert close(b.reward.cpu().numpy(), want_r, 1e-6, 1e-6)[0], t
        assert np.array_equal(b.terminated.cpu().numpy(), np.stack([r[2] for r in ref]).reshape(E, K)), t
        assert np.array_equal(b.truncated.cpu().numpy(), np.stack([r[3] for r in ref]).reshape(E, K)), t
        dn = np.array([bool(r[4]) for r in ref])
        assert np.array_equal(b.reset_happened.cpu().numpy().astype(bool), dn), t
        resets += int(dn.sum())
        if dn.any() and ph:
            st = b.get_state()
            assert np.all(st["last_rpm"][dn] == 0) and np.all(st["rpy_rates"][dn] == 0)
    st = b.get_state()
    want = stack([env.get_state() for env in envs])
    assert resets > 0
    assert np.array_equal(st["episode"], want["episode"])
    assert np.array_equal(st["spawn_index"], want["spawn_index"])
    # last_clipped_action / rpy_rates are carried only under the variants that read them (PYB: unused)
    for k in ("drone_pos", "drone_quat", "drone_vel", "drone_qlag") + (("last_rpm", "rpy_rates") if ph else ()):
        assert close(st[k][:, :n], want[k][:, :n], 1e-9, 1e-9)[0], k
    assert close(st["cow_pos"], want["cow_pos"][:, :m], 1e-12, 1e-13)[0]
    # update_evaluation_metrics' per-drone distance, accumulated on the device every step (BaseAviary.py:1415-1426)
    assert close(b.eval_distances(), np.stack([env.get_state()["eval_dist"][:n] for env in envs]), 1e-9, 1e-12)[0]
    b.close()


def test_reset_parity_and_spawn():
    """ch_reset: spawn scenario (env_id+2) mod 100 on the first reset, start layout, Philox cattle
    velocities identical to the oracle's."""
    import torch
    import oracle as O
    from cattleherd._lib import spawn_table
    for n, m in ((4, 16), (7, 16), (3, 32)):
        table = spawn_table(m)
        E = 130
        b = _batch(0, n, m, E, None)
        obs = b.reset()
        torch.cuda.synchronize()
        envs = [O.Env(0, n, m, table, env_id=e) for e in range(E)]
        o = np.stack([env.reset() for env in envs])
        assert close(obs.cpu().numpy(), o, 1e-6, 1e-7)[0]
        st = b.get_state()
        assert np.array_equal(st["spawn_index"], (np.arange(E) + 2) % 100)
        want = stack([env.get_state() for env in envs])
        assert close(st["cow_vel"], want["cow_vel"][:, :m], 1e-15, 1e-15)[0]
        assert np.array_equal(st["cow_pos"], want["cow_pos"][:, :m])
        b.close()


def test_f32_throughput_mode_error_budget():
    """CH_PREC_F32 (throughput mode) holds the positions, the centroids, prev_cent_dists and the observation
    offsets in f64 beside the f32 state (StepParams::pos64): the approach term -- a difference of two centroid
    distances divided by the 0.0083 m max step (CattleAviary.py:289-300) -- no longer amplifies f32 rounding.
    One step from diverse oracle states (tests/diag/f32_probe.py over 256 states, profiles/r03/f32_probe.log):
    rewards within 1e-4 relative (measured max abs 1.5e-7, median relative 9e-8) with a 1e-6 floor for rewards
    near zero; observations within 1e-4 relative with a 1e-6 floor, and the body rates (columns 7-9) within
    1e-4 relative down to 1e-8 (the yaw rate, column 9, 3e-4 under the cached link frame): the attitude loop's torque mix, the motor speeds, the body torque and the
    angular-velocity update run in f64 (ch_device.h pid_vel / drone_substep; in f32 they left 2.5e-4 relative
    on rates of ~3e-3 rad/s, tools/f32_emu.py); terminated / truncated flags identical; the state round trip
    keeps the f64 positions."""
    import torch
    from cattleherd._lib import spawn_table
    n, m, E = 4, 16, 64
    table = spawn_table(m)
    envs, states = _oracle_states(0, n, m, E, table, 120, seed=3, level=7)
    b = _batch(0, n, m, E, 7, precision="f32")
    b.reset()
    st = stack([{k: v for k, v in s.items() if k != "episode"} for s in states])
    b.set_state(st)
    back = b.get_state()
    assert np.array_equal(back["drone_pos"], st["drone_pos"][:, :n])
    assert np.array_equal(back["cow_pos"], st["cow_pos"][:, :m])
    assert np.array_equal(back["prev_cent"], np.nan_to_num(np.asarray(st["prev_cent"], np.float64), nan=0.0))
    acts = np.random.default_rng(1).uniform(-1, 1, (E, n, 4)).astype(np.float32)
    obs, rew, te, tr = b.step(torch.tensor(acts, device=b.device), autoreset=False)
    torch.cuda.synchronize()
    ref = [env.step(acts[e], autoreset=False) for e, env in enumerate(envs)]
    ro = np.stack([r[0] for r in ref])
    # every column but the yaw rate within 1e-4 relative with a 1e-6 floor
    o = obs.cpu().numpy()
    cols = [c for c in range(86) if c != 9]
    ok, worst = close(o[..., cols], ro[..., cols], 1e-4, 1e-6)
    assert ok, worst
    # roll / pitch rates (torque mix and angular-velocity update carried in f64) within 1e-4 relative down to 1e-8;
    # the yaw rate within 3e-4: Bullet's cached link frame (link_lag) couples it to the roll / pitch torques, and every
    # f32 piece of the PID feeds that coupling (tools/f32_emu.py, tests/test_f32_emulation.py)
    ok, worst = close(o[..., 7:9], ro[..., 7:9], 1e-4, 1e-8)
    assert ok, worst
    ok, worst = close(o[..., 9], ro[..., 9], 3e-4, 1e-8)
    assert ok, worst
    # against each column's scale (max |ref| over the batch) every observation column, the yaw rate included, is within
    # 1e-4: the body-rate errors are ~2e-5 rad/s on rates of up to ~6 rad/s; elementwise they exceed 1e-4 only where a
    # rate crosses zero (tools/f32_emu.py: 1e-4 elementwise on the yaw rate needs the PID and the quaternion state in
    # f64)
    scale = np.maximum(np.abs(ro).max(axis=(0, 1)), 1e-6)
    err = (np.abs(o.astype(np.float64) - ro) / scale).max(axis=(0, 1))
    assert err.max() <= 1e-4, (int(err.argmax()), float(err.max()))
    rr = np.array([r[1][0] for r in ref])
    assert close(rew.cpu().numpy()[:, 0], rr, 1e-4, 1e-6)[0], np.max(np.abs(rew.cpu().numpy()[:, 0] - rr))
    assert np.array_equal(te.cpu().numpy()[:, 0].astype(bool), np.array([r[2][0] for r in ref], bool))
    assert np.array_equal(tr.cpu().numpy()[:, 0].astype(bool), np.array([r[3][0] for r in ref], bool))
    b.close()


def test_full_size_properties():
    """BASELINE size (4096 envs x (4 drones, 16 cattle)): determinism across handles, sharding
    invariance (env_id_offset), unit quaternions, cattle speed cap, counters, finite obs."""
    import torch
    E, n, m, T = 4096, 4, 16, 64
    a = _batch(0, n, m, E, None)
    b2 = _batch(0, n, m, E, None)
    sh = _batch(0, n, m, E // 2, None, env_id_offset=E // 2)
    for h in (a, b2, sh):
        h.reset()
    for t in range(T):
        for h in (a, b2, sh):
            h.step(random_actions=True, autoreset=True)
    torch.cuda.synchronize()
    assert torch.equal(a.obs, b2.obs) and torch.equal(a.reward, b2.reward)
    assert torch.equal(a.obs[E // 2:], sh.obs)
    s = a.get_state()
    q = np.linalg.norm(s["drone_quat"], axis=-1)
    assert np.all(np.abs(q - 1) < 1e-12)
    sp = np.linalg.norm(s["cow_vel"], axis=-1)
    assert np.all(sp <= 0.2 + 1e-12)
    assert np.all(s["step_counter_A"] <= T) and np.all(s["step_counter"] % 4 == 0)
    assert torch.isfinite(a.obs).all()
    met = a.metrics()
    assert met[0] == E * T
    for h in (a, b2, sh):
        h.close()


@pytest.mark.parametrize("mode,n,m,E,geom", [(0, 4, 16, 4096, None), (0, 2, 8, 1024, None), (1, 4, 32, 600, None),
                                             (0, 12, 16, 300, None), (1, 3, 8, 257, None), (0, 8, 64, 40, None),
                                             (0, 4, 16, 1000, (4, 128)), (0, 4, 16, 999, (2, 128)),
                                             (0, 4, 16, 1001, (8, 256)), (0, 4, 16, 1003, (16, 512)), (1, 5, 16, 333, (3, 128)),
                                             (0, 2, 8, 700, (1, 256)),
                                             # per-wave env tables (> 16 cows): configs[4] at full size and
                                             # other geometries, CTDE and MARL
                                             (1, 4, 32, 4096, None), (1, 4, 32, 1000, (8, 512)), (1, 4, 32, 999, (4, 256)),
                                             (0, 4, 32, 1001, (8, 256)), (1, 3, 24, 513, (16, 512)), (0, 2, 20, 300, (2, 128)),
                                             # physics variants (BaseAviary.py:420-450): DYN, GND, DRAG, DW, all
                                             (0, 4, 16, 4096, "dyn"), (0, 4, 16, 1000, "pyb_gnd"),
                                             (0, 4, 16, 1000, "pyb_drag"), (0, 6, 8, 1000, "pyb_dw"),
                                             (0, 4, 16, 4096, "pyb_gnd_drag_dw"), (1, 4, 16, 333, "pyb_gnd_drag_dw"),
                                             (1, 3, 8, 257, "dyn"), (0, 4, 16, 1000, "dyn_rk4"), (1, 4, 32, 300, "dyn_rk4"),
                                             # f32 mode (f64 positions, centroids and prev_cent beside the f32 state)
                                             (0, 4, 16, 4096, "f32"), (1, 4, 32, 1000, "f32"), (0, 2, 8, 1000, "f32")])
def test_step_kernels_v1_v2_bit_identical(mode, n, m, E, geom):
    """The role-split v2 step kernel (ch_step.hip, the default) and the team-per-env v1 kernel
    (ch_kernels.hip) compute the same arithmetic in the same order: 150 random-action steps with
    auto-reset and terminal observations must agree bit for bit (incl. the alpha pair table)."""
    import ctypes
    import torch
    from cattleherd import _lib
    precision = "f32" if geom == "f32" else "f64"
    physics = geom if isinstance(geom, str) and geom != "f32" else "pyb"
    geom = None if isinstance(geom, str) else geom
    hs = [_batch(mode, n, m, E, None, physics=physics, precision=precision) for _ in range(2)]
    assert _lib.lib().ch__set_kernel(hs[0].handle, ctypes.c_int32(1)) == 0
    assert _lib.lib().ch__set_kernel(hs[1].handle, ctypes.c_int32(2)) == 0
    if geom is not None:
        assert _lib.lib().ch__set_geometry(hs[1].handle, ctypes.c_int32(geom[0]), ctypes.c_int32(geom[1])) == 0
    for h in hs:
        h.reset()
    for t in range(150):
        outs = []
        for h in hs:
            h.step(random_actions=True, autoreset=True, terminal_obs=True)
            outs.append([x.clone() for x in (h.obs, h.reward, h.terminated, h.truncated, h.terminal_obs,
                                             h.reset_happened, h.agent_active)])
        torch.cuda.synchronize()
        for a, b in zip(*outs):
            assert torch.equal(torch.nan_to_num(a.float(), nan=7.0), torch.nan_to_num(b.float(), nan=7.0)), t
    s1, s2 = hs[0].get_state(), hs[1].get_state()
    for k in s1:
        assert np.array_equal(np.nan_to_num(s1[k]), np.nan_to_num(s2[k])), k
    assert np.array_equal(hs[0].metrics(), hs[1].metrics(), equal_nan=True)
    assert np.array_equal(hs[0].eval_distances(), hs[1].eval_distances())
    for h in hs:
        h.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode,n,m", [(0, 4, 16), (1, 4, 16), (0, 6, 8)])
def test_obs_constant_bytes_sparse_writes(mode, n, m):
    """The v2 step stores only the observation entries that change; the constant-zero bytes of each
    block (rows >= NUM_DRONES, the action-buffer block) stay from the last full write (ch_api.cpp
    obs_zero_ptr).  With NUM_DRONES drawn per episode the dead rows move at every reset; a caller that
    scribbles over obs and calls invalidate_obs(), and a set_state(), must both get full blocks again.
    Compared bit for bit with the v1 kernel, which writes every block in full each step."""
    import ctypes
    import torch
    from cattleherd import _lib
    E = 777
    hs = [_batch(mode, n, m, E, None, min_drones=2, max_drones=n) for _ in range(2)]
    assert _lib.lib().ch__set_kernel(hs[0].handle, ctypes.c_int32(1)) == 0
    assert _lib.lib().ch__set_kernel(hs[1].handle, ctypes.c_int32(2)) == 0
    for h in hs:
        h.reset()
    resets = 0
    for t in range(200):
        if t == 60:
            hs[1].obs.fill_(3.0)
            hs[1].invalidate_obs()
        if t == 120:
            d, i = hs[1].get_state_raw()
            hs[1].obs.fill_(-1.0)
            hs[1].set_state_raw(d, i)
        outs = []
        for h in hs:
            h.step(random_actions=True, autoreset=True, terminal_obs=True)
            outs.append([x.clone() for x in (h.obs, h.reward, h.terminated, h.truncated, h.terminal_obs,
                                             h.reset_happened)])
        torch.cuda.synchronize()
        resets += int(outs[0][5].sum())
        for a, b in zip(*outs):
            assert torch.equal(torch.nan_to_num(a.float(), nan=7.0), torch.nan_to_num(b.float(), nan=7.0)), t
    assert resets > 0
    for h in hs:
        h.close()
