"""Generate the golden vectors under ``tests/golden/`` from the reference's OWN Python code.

Run in this container only (``python tests/golden/make_golden.py``); the reference is read-only at
``/root/reference`` and never travels.  The stubs in ``refstubs.py`` stand in for the packages the
reference imports but this image lacks (pybullet, gymnasium, ray).  Every fixture records the inputs
and the outputs of a reference function (file:line cited per fixture below); nothing of the
reference's source text is stored.

Fixtures
--------
flock.npz          ``BaseAviary._flockingStep`` (sb3_envs/BaseAviary.py:1352-1400) → flockUtils.py
                   ``_flocking`` / ``_global_clustering`` / ``_local_clustering`` on random herds.
effectiveness.npz  ``evaluate_herding_effectiveness`` (utils/evaluation.py:100-138).
pid.npz            ``DSLPIDControl.computeControl`` sequences (control/DSLPIDControl.py:82-259).
spacing.npz        ``SimpleSpacingReward`` / ``DroneSpacingRewardFunction`` / ``CattleSpacingRewardFunction``
                   (sb3_envs/CattleAviary.py:572-679) per curriculum level.
task_ctde.npz      ``_computeReward`` → ``_computeTerminated`` → ``_computeTruncated`` in env.step order
                   (sb3_envs/BaseAviary.py:458-460, CattleAviary.py:213-552) on synthetic states, all levels.
task_marl.npz      the RLlib wrapper's per-agent call sequence (marl_wrapper.py:77-119 over
                   MARLCattleAviary.py:110-383) on synthetic states, all levels.
ctde_roll_*.npz    whole ``CattleAviary.step`` rollouts incl. auto-resets (stub physics in the loop);
                   ``*_dyn`` / ``*_pyb_gnd`` / ``*_pyb_drag`` / ``*_pyb_dw`` / ``*_pyb_gnd_drag_dw``: the physics
                   variants (BaseAviary.py:420-450, 943-1118), ``--physics`` regenerates only these.
marl_roll_*.npz    whole ``RLlibMultiAgentWrapper.step`` rollouts.
reset.npz          ``reset`` bookkeeping: spawn-index sequence, drone initial positions, cattle spawn table.
"""
import contextlib
import io
import math
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refstubs  # noqa: E402

refstubs.install()
warnings.filterwarnings("ignore")

QUIET = contextlib.redirect_stdout(io.StringIO())


def quiet():
    return contextlib.redirect_stdout(io.StringIO())


with quiet():
    import gym_pybullet_drones.sb3_envs.CattleAviary as CA_mod  # noqa: E402
    import gym_pybullet_drones.rllib_envs.MARLCattleAviary as MA_mod  # noqa: E402
    from gym_pybullet_drones.rllib_envs.marl_wrapper import RLlibMultiAgentWrapper  # noqa: E402
    from gym_pybullet_drones.control.DSLPIDControl import DSLPIDControl  # noqa: E402
    from gym_pybullet_drones.utils.enums import DroneModel  # noqa: E402
    from gym_pybullet_drones.utils.evaluation import evaluate_herding_effectiveness  # noqa: E402
    from gym_pybullet_drones.utils.curriculum_learning import CurriculumLearning  # noqa: E402

W = refstubs.WORLD
NMAX, MMAX = 12, 32


def make_ctde(n, m, level=7, physics=None):
    orig = CA_mod.CurriculumLearning
    CA_mod.CurriculumLearning = lambda _lvl: CurriculumLearning(level)
    try:
        with quiet():
            kw = {} if physics is None else {"physics": physics}
            env = CA_mod.CattleAviary(num_drones=n, num_cattle=m, **kw)
    finally:
        CA_mod.CurriculumLearning = orig
    env.MIN_NUM_DRONES = env.MAX_NUM_DRONES = n
    env._ctor_level = level
    return env


def make_marl(n, m, level=0):
    orig = MA_mod.CurriculumLearning
    MA_mod.CurriculumLearning = lambda _lvl: CurriculumLearning(level)
    try:
        with quiet():
            env = MA_mod.MARLCattleAviary(num_drones=n, num_cattle=m)
    finally:
        MA_mod.CurriculumLearning = orig
    env.MIN_NUM_DRONES = env.MAX_NUM_DRONES = n
    env._ctor_level = level
    return env


# --------------------------------------------------------------------------------------
# State capture / injection (stub world bodies are the physics state)
# --------------------------------------------------------------------------------------

def capture(env, marl_agents=None, physics_state=False):
    n, m = env.NUM_DRONES, env.NUM_CATTLE
    s = {
        "n": n, "m": m,
        "drone_pos": np.zeros((NMAX, 3)), "drone_quat": np.zeros((NMAX, 4)),
        "drone_vel": np.zeros((NMAX, 3)), "drone_angv": np.zeros((NMAX, 3)),
        "pid_last_rpy": np.zeros((NMAX, 3)), "pid_int_pos": np.zeros((NMAX, 3)),
        "pid_int_rpy": np.zeros((NMAX, 3)), "drone_qlag": np.zeros((NMAX, 4)),
        "cow_pos": np.zeros((MMAX, 2)), "cow_vel": np.zeros((MMAX, 2)),
        "step_counter": env.step_counter, "step_counter_A": env.step_counter_A,
        "prev_cent": np.nan if env.prev_cent_dists is None else float(env.prev_cent_dists),
        "has_prev": 0 if env.prev_cent_dists is None else 1,
        "clock": float(env.drone_spacing_clock), "level": env.curriculum.curriculum_level,
        "tally": env.curriculum.curriculum_success_tally, "spawn_index": env.Cattle_Spawn_Index,
        "active": np.zeros(NMAX, dtype=np.uint8),
        "ctor_level": getattr(env, "_ctor_level", -1), "episode_len": float(env.EPISODE_LEN_SEC),
    }
    for i in range(n):
        b = W.bodies[int(env.DRONE_IDS[i])]
        s["drone_pos"][i], s["drone_quat"][i] = b.pos, b.quat
        s["drone_vel"][i], s["drone_angv"][i] = b.vel, b.angv
        s["drone_qlag"][i] = b.cached
        c = env.ctrl[i]
        s["pid_last_rpy"][i], s["pid_int_pos"][i], s["pid_int_rpy"][i] = c.last_rpy, c.integral_pos_e, c.integral_rpy_e
    for j in range(m):
        b = W.bodies[int(env.CATTLE_IDS[j])]
        s["cow_pos"][j] = b.pos[:2]
        s["cow_vel"][j] = b.vel[:2]
    if physics_state:
        # BaseAviary.step's per-drone physics-variant state: last_clipped_action (drag, 450) and
        # the DYN body rates (581-582, 1043-1075)
        s["last_rpm"] = np.zeros((NMAX, 4))
        s["rpy_rates"] = np.zeros((NMAX, 3))
        s["last_rpm"][:n] = env.last_clipped_action
        if hasattr(env, "rpy_rates"):
            s["rpy_rates"][:n] = env.rpy_rates
    if marl_agents is not None:
        for a in marl_agents:
            s["active"][int(a.split("_")[1])] = 1
    else:
        s["active"][:n] = 1
    return s


def sync_readback(env):
    """Refresh the env's cached kinematics from the world (what _updateAndStoreKinematicInformation does)."""
    with quiet():
        env._updateAndStoreKinematicInformation()


def stack_states(states):
    out = {}
    for k in states[0]:
        out[k] = np.stack([np.asarray(s[k]) for s in states])
    return out


# --------------------------------------------------------------------------------------
# Fixtures
# --------------------------------------------------------------------------------------

def gen_flock(rng):
    """Reference: sb3_envs/BaseAviary.py:1352-1400 (+ utils/flockUtils.py:116-382)."""
    env = make_ctde(4, 16)
    cases = []
    ms = [1, 2, 3, 4, 5, 8, 12, 16, 24, 32]
    for it in range(240):
        m = ms[it % len(ms)]
        n = 1 + (it * 7) % 12
        spread = rng.uniform(0.3, 4.0)
        center = rng.uniform(-10, 10, 2)
        cow_pos = center + rng.uniform(-spread, spread, (m, 2))
        ang = rng.uniform(-np.pi, np.pi, m)
        sp = rng.uniform(0, 0.25, m)
        cow_vel = np.stack([np.cos(ang) * sp, np.sin(ang) * sp], 1)
        # drones: mix of far, beta range (<= 1 m), predator range (<= 1.1 m)
        dpos = []
        for k in range(n):
            mode = rng.integers(0, 3)
            if mode == 0:
                dpos.append(center + rng.uniform(-8, 8, 2))
            else:
                c = cow_pos[rng.integers(0, m)]
                r = rng.uniform(0.15, 1.05 if mode == 1 else 3.0)
                a = rng.uniform(-np.pi, np.pi)
                dpos.append(c + r * np.array([np.cos(a), np.sin(a)]))
        dpos = np.array(dpos)
        # inject into env + world
        W.reset()
        env.NUM_DRONES, env.NUM_CATTLE = n, m
        env.DRONE_IDS = np.array([W.add("drone", [dpos[k, 0], dpos[k, 1], 0.45], [0, 0, 0, 1]) for k in range(n)])
        env.CATTLE_IDS = [W.add("cow", [cow_pos[j, 0], cow_pos[j, 1], 0.1], [0, 0, 0, 1]) for j in range(m)]
        for j in range(m):
            W.bodies[env.CATTLE_IDS[j]].vel = [cow_vel[j, 0], cow_vel[j, 1], 0.0]
        env.pos = np.zeros((n, 3)); env.quat = np.zeros((n, 4)); env.rpy = np.zeros((n, 3))
        env.vel = np.zeros((n, 3)); env.ang_v = np.zeros((n, 3))
        env.cattle_pos = np.zeros((m, 3)); env.cattle_quat = np.zeros((m, 4)); env.cattle_rpy = np.zeros((m, 3))
        env.cattle_vel = np.zeros((m, 3)); env.cattle_ang_v = np.zeros((m, 3))
        env.last_clipped_action = np.zeros((n, 4))
        if hasattr(env, "_vel_drift"):
            del env._vel_drift
        sync_readback(env)
        with quiet():
            env._flockingStep()
        new_vel = np.array([W.bodies[c].vel[:2] for c in env.CATTLE_IDS])
        cases.append((n, m, cow_pos, cow_vel, dpos, new_vel))
    K = len(cases)
    out = {"n": np.array([c[0] for c in cases]), "m": np.array([c[1] for c in cases]),
           "cow_pos": np.zeros((K, MMAX, 2)), "cow_vel": np.zeros((K, MMAX, 2)),
           "drone_pos": np.zeros((K, NMAX, 2)), "new_vel": np.zeros((K, MMAX, 2))}
    for i, (n, m, cp, cv, dp, nv) in enumerate(cases):
        out["cow_pos"][i, :m], out["cow_vel"][i, :m] = cp, cv
        out["drone_pos"][i, :n], out["new_vel"][i, :m] = dp, nv
    np.savez_compressed(os.path.join(HERE, "flock.npz"), **out)
    print("flock", K, "cases; predator-range fraction",
          np.mean([np.any(np.linalg.norm(c[4][:, None] - c[2][None], axis=-1) <= 1.1) for c in cases]))


def gen_effectiveness(rng):
    """Reference: utils/evaluation.py:100-138, 271-273."""
    cases = []
    for it in range(300):
        n = 1 + it % 12
        m = 1 + (it * 5) % 32
        if it % 10 == 0:   # lattice points hit edges / vertices exactly
            dp = rng.integers(-3, 4, (n, 2)).astype(np.float64)
            cp = rng.integers(-3, 4, (m, 2)).astype(np.float64)
        else:
            dp = rng.uniform(-3, 3, (n, 2))
            cp = rng.uniform(-3, 3, (m, 2))
        eff = evaluate_herding_effectiveness(cp, dp)
        cases.append((n, m, dp, cp, eff))
    K = len(cases)
    out = {"n": np.array([c[0] for c in cases]), "m": np.array([c[1] for c in cases]),
           "drone_pos": np.zeros((K, NMAX, 2)), "cow_pos": np.zeros((K, MMAX, 2)),
           "eff": np.array([c[4] for c in cases], dtype=np.float64)}
    for i, (n, m, dp, cp, _) in enumerate(cases):
        out["drone_pos"][i, :n], out["cow_pos"][i, :m] = dp, cp
    np.savez_compressed(os.path.join(HERE, "effectiveness.npz"), **out)
    print("effectiveness", K, "cases; nonzero", np.count_nonzero(out["eff"]))


def gen_pid(rng):
    """Reference: control/DSLPIDControl.py:82-259 (VEL targets as BaseRLAviary.py:185-222 builds them)."""
    seqs, T = 24, 40
    rec = {k: [] for k in ("pos", "quat", "vel", "angv", "target_pos", "target_rpy", "target_vel", "rpm",
                           "last_rpy", "int_pos", "int_rpy")}
    for s in range(seqs):
        with quiet():
            c = DSLPIDControl(drone_model=DroneModel.CF2X)
        for t in range(T):
            pos = np.array([rng.uniform(-5, 5), rng.uniform(-5, 5), rng.uniform(0.2, 0.7)])
            rpy = rng.normal(0, 0.15 if s % 3 else 0.6, 3)
            rpy[2] = rng.uniform(-np.pi, np.pi)
            quat = np.array(refstubs.getQuaternionFromEuler(rpy))
            vel = rng.normal(0, 0.8, 3)
            angv = rng.normal(0, 2.0, 3)
            a = rng.uniform(-1, 1, 4)
            hn = np.linalg.norm(a[:2])
            vu = a[:2] / hn if hn != 0 else np.zeros(2)
            tv = np.array([vu[0], vu[1], 0.0]) * (2.5 * abs(a[3]))
            tp = np.array([pos[0], pos[1], 0.45])
            tr = np.array([0.0, 0.0, refstubs.getEulerFromQuaternion(quat)[2]])
            with quiet():
                rpm, _, _ = c.computeControl(control_timestep=1 / 60, cur_pos=pos, cur_quat=quat, cur_vel=vel,
                                             cur_ang_vel=angv, target_pos=tp, target_rpy=tr, target_vel=tv)
            for k, v in (("pos", pos), ("quat", quat), ("vel", vel), ("angv", angv), ("target_pos", tp),
                         ("target_rpy", tr), ("target_vel", tv), ("rpm", rpm), ("last_rpy", c.last_rpy),
                         ("int_pos", c.integral_pos_e), ("int_rpy", c.integral_rpy_e)):
                rec[k].append(np.array(v, dtype=np.float64))
    out = {k: np.array(v).reshape(seqs, T, -1) for k, v in rec.items()}
    np.savez_compressed(os.path.join(HERE, "pid.npz"), **out)
    print("pid", seqs, "x", T, "calls")


def gen_spacing():
    """Reference: sb3_envs/CattleAviary.py:572-679 (identical in MARLCattleAviary.py:402-509)."""
    r = np.concatenate([[0.0, 0.3, 0.56, 0.64, 0.72, 0.8, 0.88, 0.96, 1.04, 1.3, 1.5, 5.0, 7.0, 1e9, np.inf],
                        np.linspace(0.0, 9.0, 181)])
    out = {"r": r}
    for lvl in range(8):
        env = make_ctde(4, 4, level=lvl)
        out[f"simple_{lvl}"] = np.array([env.SimpleSpacingReward(x) for x in r])
        out[f"complex_{lvl}"] = np.array([env.DroneSpacingRewardFunction(x) for x in r])
    env = make_ctde(4, 4)
    out["cattle"] = np.array([env.CattleSpacingRewardFunction(x) for x in r])
    np.savez_compressed(os.path.join(HERE, "spacing.npz"), **out)
    print("spacing", len(r))


def _synthetic_layout(rng, n, m, kind):
    """Drone xyz and cow xy placements that exercise each termination/truncation branch."""
    herd_c = rng.uniform(-6, 6, 2)
    cows = herd_c + rng.uniform(-1.5, 1.5, (m, 2))
    if kind == "ring":          # drones around the herd in index order → effectiveness > 0
        rad = rng.uniform(1.0, 3.0)
        ang = np.sort(rng.uniform(0, 2 * np.pi, n)) if rng.random() < 0.5 else np.linspace(0, 2 * np.pi, n, endpoint=False)
        xy = herd_c + rad * np.stack([np.cos(ang), np.sin(ang)], 1)
    elif kind == "spaced":      # nearest neighbour ≈ 0.8 m (level 0/1/5 windows)
        d = rng.uniform(0.5, 1.1)
        xy = herd_c + np.stack([np.arange(n) * d, np.zeros(n)], 1) + rng.normal(0, 0.02, (n, 2))
    elif kind == "close":       # centroid distance below approach thresholds
        xy = cows.mean(0) + rng.normal(0, 0.6, (n, 2))
    elif kind == "far":         # mission boundary / isolation
        xy = herd_c + rng.uniform(-20, 20, (n, 2))
    else:                       # generic
        xy = herd_c + rng.uniform(-5, 5, (n, 2))
    z = 0.45 + rng.normal(0, 0.12, n)
    return np.concatenate([xy, z[:, None]], 1), cows


def _inject(env, dxyz, cows, cow_vel=None):
    n, m = len(dxyz), len(cows)
    for i in range(n):
        b = W.bodies[int(env.DRONE_IDS[i])]
        b.pos = list(dxyz[i])
    for j in range(m):
        b = W.bodies[int(env.CATTLE_IDS[j])]
        b.pos = [cows[j, 0], cows[j, 1], 0.1]
        if cow_vel is not None:
            b.vel = [cow_vel[j, 0], cow_vel[j, 1], 0.0]
    sync_readback(env)


def gen_task_ctde(rng):
    """env.step's reward → terminated → truncated sequence (sb3_envs/BaseAviary.py:458-460)."""
    states_in, states_out, rew, term, trunc = [], [], [], [], []
    kinds = ["ring", "spaced", "close", "far", "generic"]
    for lvl in range(8):
        for n in (3, 4, 5, 8, 12):
            m = (4, 8, 16)[n % 3]
            env = make_ctde(n, m, level=lvl)
            with quiet():
                env.reset()
            for it in range(12):
                kind = kinds[it % len(kinds)]
                dxyz, cows = _synthetic_layout(rng, n, m, kind)
                _inject(env, dxyz, cows)
                if it % 4 == 0:
                    env.prev_cent_dists = None
                env.step_counter = int(rng.choice([0, 4 * 300, 4 * 1201, 4 * 1202]))
                if lvl in (0, 1) and it % 3 == 1:
                    env.drone_spacing_clock = env.curriculum.current_curriculum["drone_spacing_hold_timer"] - 1 / 240
                if it % 5 == 4:   # near the tally threshold so a level-up happens inside the call sequence
                    env.curriculum.curriculum_success_tally = env.curriculum.current_curriculum["required_tally"] - 1
                s0 = capture(env)
                with quiet():
                    r = env._computeReward()
                    te = env._computeTerminated()
                    tr = env._computeTruncated()
                states_in.append(s0)
                states_out.append(capture(env))
                rew.append(r); term.append(te); trunc.append(tr)
    out = {"in_" + k: v for k, v in stack_states(states_in).items()}
    out.update({"out_" + k: v for k, v in stack_states(states_out).items()})
    out.update(reward=np.array(rew), terminated=np.array(term, dtype=np.uint8), truncated=np.array(trunc, dtype=np.uint8))
    np.savez_compressed(os.path.join(HERE, "task_ctde.npz"), **out)
    print("task_ctde", len(rew), "cases; term", int(np.sum(term)), "trunc", int(np.sum(trunc)),
          "nan rewards", int(np.isnan(rew).sum()))


def gen_task_marl(rng):
    """The wrapper's per-agent sequence after env.step (marl_wrapper.py:104-117) — the env.step half
    (rllib_envs/BaseAviary.py:425-431) is reproduced too because its calls have side effects."""
    states_in, states_out = [], []
    rew, done, trunc = [], [], []
    kinds = ["ring", "spaced", "close", "far", "generic"]
    for lvl in range(8):
        for n in (3, 4, 6):
            m = (8, 16)[n % 2]
            env = make_marl(n, m, level=lvl)
            with quiet():
                w = RLlibMultiAgentWrapper.__new__(RLlibMultiAgentWrapper)
                w.env = env
                w.reset()
            for it in range(10):
                kind = kinds[it % len(kinds)]
                dxyz, cows = _synthetic_layout(rng, n, m, kind)
                _inject(env, dxyz, cows)
                if it % 4 == 0:
                    env.prev_cent_dists = None
                env.step_counter = int(rng.choice([0, 600, 2399, 2400, 2401]))
                if lvl in (0, 1) and it % 3 == 1:
                    env.drone_spacing_clock = env.curriculum.current_curriculum["drone_spacing_hold_timer"] - 3 / 60
                if it % 5 == 4:
                    env.curriculum.curriculum_success_tally = env.curriculum.current_curriculum["required_tally"] - 1
                w.agents = [a for a in w.possible_agents if rng.random() < 0.85] or [w.possible_agents[0]]
                s0 = capture(env, w.agents)
                with quiet():
                    # env.step's own dict construction (side effects only)
                    for i in range(env.NUM_DRONES):
                        env._computeReward(i)
                    for i in range(env.NUM_DRONES):
                        env._computeTerminated(i)
                    for i in range(env.NUM_DRONES):
                        env._computeTruncated(i)
                    env.step_counter += 1   # rllib_envs/BaseAviary.py:436, before the wrapper's calls
                    # the wrapper's recomputation (returned values)
                    r = np.full(NMAX, np.nan); d = np.zeros(NMAX, np.uint8); t = np.zeros(NMAX, np.uint8)
                    for aid in list(w.agents):
                        idx = int(aid.split("_")[1])
                        r[idx] = float(env._computeReward(idx))
                        d[idx] = bool(env._computeTerminated(idx))
                        t[idx] = bool(env._computeTruncated(idx))
                    w.agents = [a for a in w.agents if not d[int(a.split("_")[1])]]
                states_in.append(s0)
                states_out.append(capture(env, w.agents))
                rew.append(r); done.append(d); trunc.append(t)
    out = {"in_" + k: v for k, v in stack_states(states_in).items()}
    out.update({"out_" + k: v for k, v in stack_states(states_out).items()})
    out.update(reward=np.array(rew), terminated=np.array(done), truncated=np.array(trunc))
    np.savez_compressed(os.path.join(HERE, "task_marl.npz"), **out)
    print("task_marl", len(rew), "cases; done", int(np.sum(done)), "trunc", int(np.sum(trunc)))


def gen_ctde_rollout(rng, n, m, steps, level=7, tag=None, hover=False):
    """Whole CattleAviary.step (sb3_envs/BaseAviary.py:335-465) with SB3-style auto-reset."""
    env = make_ctde(n, m, level=level)
    with quiet():
        obs, _ = env.reset()
    rec = {"state": [], "action": [], "obs": [], "reward": [], "terminated": [], "truncated": [],
           "reset_state": [], "reset_obs": [], "reset_at": []}
    rec["init_state"] = capture(env)
    rec["init_obs"] = obs
    for t in range(steps):
        a = (rng.uniform(-1, 1, (n, 4)) * (0.15 if hover else 1.0)).astype(np.float32)
        rec["state"].append(capture(env))
        with quiet():
            obs, r, te, tr, _ = env.step(a)
        rec["action"].append(a); rec["obs"].append(obs); rec["reward"].append(r)
        rec["terminated"].append(te); rec["truncated"].append(tr)
        if te or tr:
            with quiet():
                obs0, _ = env.reset()
            rec["reset_at"].append(t)
            rec["reset_state"].append(capture(env))
            rec["reset_obs"].append(obs0)
    out = {"action": np.array(rec["action"]), "obs": np.array(rec["obs"]), "reward": np.array(rec["reward"]),
           "terminated": np.array(rec["terminated"], np.uint8), "truncated": np.array(rec["truncated"], np.uint8),
           "reset_at": np.array(rec["reset_at"], np.int64), "init_obs": rec["init_obs"],
           "level": np.int64(level)}
    out.update({"state_" + k: v for k, v in stack_states(rec["state"]).items()})
    out.update({"init_" + k: np.asarray(v) for k, v in rec["init_state"].items()})
    if rec["reset_state"]:
        out.update({"reset_" + k: v for k, v in stack_states(rec["reset_state"]).items()})
        out["reset_obs"] = np.array(rec["reset_obs"])
    name = tag or f"ctde_roll_n{n}_m{m}_l{level}"
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, steps, "steps; resets at", rec["reset_at"][:6], "nan rewards", int(np.isnan(out["reward"]).sum()))


def gen_eval(rng, n=3, m=4, level=2, steps=1300):
    """The evaluation logger with ``is_evaluating = True``: BaseAviary.update_evaluation_metrics
    (sb3_envs/BaseAviary.py:1406-1435) every step, evaluation_episode_trigger (1439-1450) from
    _computeTruncated at the time limit (CattleAviary.py:545-548, twice per step), reset between
    episodes, and the evaluator's lists exactly as save_evaluation_data (utils/evaluation.py:73-94)
    would pickle them -- aliasing included: the distance rows reference the env's list of arrays,
    which update_evaluation_metrics mutates in place.  Level 2 (40 s, terminates only on approach)
    with hover actions runs two full episodes into the time limit."""
    env = make_ctde(n, m, level=level)
    env.is_evaluating = True
    with quiet():
        env.reset()
    rec = {"state": [], "action": [], "reset_at": [], "reset_state": []}
    for t in range(steps):
        a = (rng.uniform(-1, 1, (n, 4)) * 0.15).astype(np.float32)
        rec["state"].append(capture(env))
        with quiet():
            _, _, te, tr, _ = env.step(a)
        rec["action"].append(a)
        if te or tr:
            with quiet():
                env.reset()
            rec["reset_at"].append(t)
            rec["reset_state"].append(capture(env))
    ev = env.eval_system
    out = {"action": np.array(rec["action"]), "reset_at": np.array(rec["reset_at"], np.int64),
           "level": np.int64(level)}
    out.update({"state_" + k: v for k, v in stack_states(rec["state"]).items()})
    out.update({"reset_" + k: v for k, v in stack_states(rec["reset_state"]).items()})
    # episode level
    out["ev_distances"] = np.array([np.array([np.asarray(d, np.float64) for d in ep]) for ep in ev.total_drone_distances])
    out["ev_num_drones"] = np.array(ev.total_number_of_drones, np.int64)
    out["ev_time_taken"] = np.array(ev.total_time_taken, np.float64)
    out["ev_effectiveness"] = np.array(ev.total_effectiveness, np.float64)
    # step level, concatenated over episodes with their lengths
    lens = [len(x) for x in ev.time_per_step]
    out["ev_steps_per_episode"] = np.array(lens, np.int64)
    cat = lambda lists: [row for ep in lists for row in ep]  # noqa: E731
    out["ev_time_per_step"] = np.array(cat(ev.time_per_step), np.float64)
    out["ev_effectiveness_per_step"] = np.array(cat(ev.effectiveness_per_step), np.float64)
    out["ev_distances_per_step"] = np.array([np.array([np.asarray(d, np.float64) for d in row])
                                             for row in cat(ev.drone_distances_per_step)])
    for key, src in (("drone_poses", ev.drone_poses_per_step), ("cattle_poses", ev.cattle_poses_per_step),
                     ("drone_vel", ev.drone_vel_per_step), ("cattle_vel", ev.cattle_vel_per_step)):
        out[f"ev_{key}_per_step"] = np.array(cat(src), np.float64)
    np.savez_compressed(os.path.join(HERE, "eval_ctde.npz"), **out)
    print("eval_ctde", steps, "steps; resets at", rec["reset_at"], "episodes", len(lens), "lengths", lens)


def gen_reset_seeded(seeds=(7, 20251031), schedule=(0, 3, 10, 1, 7, 0, 4)):
    """The reference's own random draws for resets under seeded global RNGs: ``random.seed(s);
    np.random.seed(s)`` then ``CattleAviary(num_drones=12, num_cattle=16)`` at curriculum level 7 (the CTDE
    driver's setup), reset, ``schedule[k]`` steps, reset, ...  Draw sites: NUM_DRONES =
    random.randint(min, max) (sb3_envs/BaseAviary.py:242 at construction, 307 per reset), per cow a yaw and
    a velocity angle np.pi * (2 np.random.rand() - 1) (617, 631), and per flocking step the drift noise
    np.random.normal(0, 0.02, (M, 2)) (1373; once an initial np.random.uniform(-0.1, 0.1, (M, 2)), 1366).
    The actions come from a separate generator, so only the env consumes the global streams."""
    import random
    out = {"seeds": np.array(seeds, np.int64), "schedule": np.array(schedule, np.int64)}
    for si, seed in enumerate(seeds):
        random.seed(seed)
        np.random.seed(seed)
        orig = CA_mod.CurriculumLearning
        CA_mod.CurriculumLearning = lambda _lvl: CurriculumLearning(7)
        try:
            with quiet():
                env = CA_mod.CattleAviary(num_drones=12, num_cattle=16)
        finally:
            CA_mod.CurriculumLearning = orig
        arng = np.random.default_rng(1000 + si)
        rec = {"n": [], "cow_pos": [], "cow_vel": [], "drone_pos": [], "spawn_index": [], "scA_before": []}
        out[f"s{si}_ctor_n"] = np.int64(env.NUM_DRONES)
        for k, steps in enumerate(schedule):
            rec["scA_before"].append(env.step_counter_A)
            with quiet():
                env.reset()
            c = capture(env)
            rec["n"].append(c["n"]); rec["cow_pos"].append(c["cow_pos"][:16]); rec["cow_vel"].append(c["cow_vel"][:16])
            rec["drone_pos"].append(c["drone_pos"]); rec["spawn_index"].append(c["spawn_index"])
            for _ in range(steps):
                a = arng.uniform(-1, 1, (12, 4)).astype(np.float32)
                with quiet():
                    env.step(a)
        for key, v in rec.items():
            out[f"s{si}_{key}"] = np.array(v)
    np.savez_compressed(os.path.join(HERE, "reset_seeded.npz"), **out)
    print("reset_seeded", {k: out[k].tolist() for k in out if k.endswith("_n")})


PHYSICS_IDS = {"pyb": 0, "dyn": 1, "pyb_gnd": 2, "pyb_drag": 3, "pyb_dw": 4, "pyb_gnd_drag_dw": 5}


def gen_physics_rollout(rng, physics, n, m, steps, scale=1.0, tag=None, stack=None):
    """CattleAviary.step under a physics variant (sb3_envs/BaseAviary.py:420-450): DYN explicit
    dynamics (1043-1118), ground effect (943-980), drag (982-1011), downwash (1013-1041).  The
    captured state carries last_clipped_action and rpy_rates; J_INV is stored to pin its value."""
    from gym_pybullet_drones.utils.enums import Physics
    env = make_ctde(n, m, physics=Physics(physics))
    with quiet():
        obs, _ = env.reset()
    if stack is not None:   # drones stacked (dz, dxy per index) so the downwash / ground terms are large
        z0, dz, dxy = stack
        xyz = np.array([[dxy * i, 0.0, z0 + dz * i] for i in range(n)])
        cows = np.array([W.bodies[int(env.CATTLE_IDS[j])].pos[:2] for j in range(m)])
        _inject(env, xyz, cows)
    rec = {"state": [], "action": [], "obs": [], "reward": [], "terminated": [], "truncated": [], "reset_at": []}
    for t in range(steps):
        a = (rng.uniform(-1, 1, (n, 4)) * scale).astype(np.float32)
        rec["state"].append(capture(env, physics_state=True))
        with quiet():
            obs, r, te, tr, _ = env.step(a)
        rec["action"].append(a); rec["obs"].append(obs); rec["reward"].append(r)
        rec["terminated"].append(te); rec["truncated"].append(tr)
        if te or tr:
            with quiet():
                env.reset()
            rec["reset_at"].append(t)
    out = {"action": np.array(rec["action"]), "obs": np.array(rec["obs"]), "reward": np.array(rec["reward"]),
           "terminated": np.array(rec["terminated"], np.uint8), "truncated": np.array(rec["truncated"], np.uint8),
           "reset_at": np.array(rec["reset_at"], np.int64), "level": np.int64(7),
           "physics": np.int64(PHYSICS_IDS[physics]), "j_inv": np.asarray(env.J_INV),
           "gnd_eff_h_clip": np.float64(env.GND_EFF_H_CLIP)}
    out.update({"state_" + k: v for k, v in stack_states(rec["state"]).items()})
    name = tag or f"ctde_roll_n{n}_m{m}_l7_{physics}"
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, steps, "steps; resets at", rec["reset_at"][:6])


def gen_physics():
    rng = np.random.default_rng(20251107)
    np.random.seed(777)
    import random
    random.seed(777)
    gen_physics_rollout(rng, "dyn", 4, 8, 200)
    gen_physics_rollout(rng, "pyb_gnd", 4, 8, 200)
    gen_physics_rollout(rng, "pyb_drag", 4, 8, 200)
    gen_physics_rollout(rng, "pyb_dw", 5, 8, 200)
    gen_physics_rollout(rng, "pyb_gnd_drag_dw", 6, 16, 200)
    gen_physics_rollout(rng, "pyb_dw", 4, 8, 60, scale=0.2, stack=(0.27, 0.12, 0.25),
                        tag="ctde_roll_n4_m8_l7_pyb_dw_stacked")
    gen_physics_rollout(rng, "pyb_gnd_drag_dw", 3, 8, 60, scale=0.2, stack=(0.19, 0.1, 0.22),
                        tag="ctde_roll_n3_m8_l7_pyb_gnd_drag_dw_low")


def gen_marl_rollout(rng, n, m, steps, level=0, tag=None):
    """Whole RLlibMultiAgentWrapper.step (marl_wrapper.py:77-119) — no auto-reset unless __all__."""
    env = make_marl(n, m, level=level)
    with quiet():
        w = RLlibMultiAgentWrapper.__new__(RLlibMultiAgentWrapper)
        w.env = env
        obs, _ = w.reset()
    N = env.NUM_DRONES
    rec = {k: [] for k in ("state", "action", "obs", "reward", "terminated", "truncated", "all_done",
                           "reset_state", "reset_obs", "reset_at")}
    rec["init_state"] = capture(env, w.agents)
    rec["init_obs"] = np.array([obs[f"agent_{i}"] for i in range(N)])
    for t in range(steps):
        a = rng.uniform(-1, 1, (N, 4)).astype(np.float32)
        rec["state"].append(capture(env, w.agents))
        with quiet():
            o, r, d, tr, _ = w.step({f"agent_{i}": a[i] for i in range(N)})
        ob = np.zeros((N, 86), np.float32); rr = np.full(N, np.nan); dd = np.zeros(N, np.uint8); tt = np.zeros(N, np.uint8)
        for aid in o:
            i = int(aid.split("_")[1])
            ob[i], rr[i], dd[i], tt[i] = o[aid], r[aid], d[aid], tr[aid]
        rec["action"].append(a); rec["obs"].append(ob); rec["reward"].append(rr)
        rec["terminated"].append(dd); rec["truncated"].append(tt); rec["all_done"].append(d["__all__"])
        if d["__all__"]:
            with quiet():
                obs, _ = w.reset()
            rec["reset_at"].append(t)
            rec["reset_state"].append(capture(env, w.agents))
            rec["reset_obs"].append(np.array([obs[f"agent_{i}"] for i in range(N)]))
    out = {k: np.array(rec[k]) for k in ("action", "obs", "reward", "terminated", "truncated")}
    out["all_done"] = np.array(rec["all_done"], np.uint8)
    out["reset_at"] = np.array(rec["reset_at"], np.int64)
    out["init_obs"] = rec["init_obs"]
    out["level"] = np.int64(level)
    out.update({"state_" + k: v for k, v in stack_states(rec["state"]).items()})
    out.update({"init_" + k: np.asarray(v) for k, v in rec["init_state"].items()})
    if rec["reset_state"]:
        out.update({"reset_" + k: v for k, v in stack_states(rec["reset_state"]).items()})
        out["reset_obs"] = np.array(rec["reset_obs"])
    name = tag or f"marl_roll_n{n}_m{m}_l{level}"
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, steps, "steps; agents done", int(out["terminated"].sum()), "trunc", int(out["truncated"].sum()))


def gen_reset():
    """reset bookkeeping: BaseAviary.py:251-331, 547-637; spawn table config/cattle_positions.yaml."""
    env = make_ctde(5, 16)
    idx, dpos, cows = [], [], []
    for _ in range(105):
        with quiet():
            env.reset()
        s = capture(env)
        idx.append(s["spawn_index"])
        dpos.append(s["drone_pos"][:5].copy())
        cows.append(s["cow_pos"][:16].copy())
    init_pos = {}
    for n in range(1, 13):
        with quiet():
            init_pos[n] = env.initialize_drone_positions(num_drones=n)
    out = {"spawn_index": np.array(idx), "drone_pos_n5": np.array(dpos), "cow_pos": np.array(cows),
           "spawn_table": np.array([[[c["x"], c["y"]] for c in sim["cows"]] for sim in env.cattle_spawn_data["simulations"]])}
    for n, v in init_pos.items():
        out[f"init_pos_n{n}"] = v
    np.savez_compressed(os.path.join(HERE, "reset.npz"), **out)
    print("reset: spawn index sequence", idx[:5], "...", out["spawn_table"].shape)


def main():
    rng = np.random.default_rng(20251031)
    np.random.seed(12345)          # the reference's own draws use numpy's global legacy RNG
    import random
    random.seed(12345)
    gen_flock(rng)
    gen_effectiveness(rng)
    gen_pid(rng)
    gen_spacing()
    gen_task_ctde(rng)
    gen_task_marl(rng)
    gen_reset()
    gen_ctde_rollout(rng, 4, 16, 400)
    gen_ctde_rollout(rng, 2, 8, 120)
    gen_ctde_rollout(rng, 3, 4, 1210, hover=True, tag="ctde_roll_n3_m4_l7_timelimit")
    gen_ctde_rollout(rng, 12, 16, 150)
    gen_ctde_rollout(rng, 5, 16, 300, level=4)
    gen_marl_rollout(rng, 3, 8, 300, level=0)
    gen_marl_rollout(rng, 4, 16, 200, level=4)


if __name__ == "__main__":
    if "--physics" in sys.argv:   # the physics-variant fixtures only (own seeds)
        gen_physics()
    elif "--reset-seeded" in sys.argv:   # reset_seeded.npz only (seeds its own global RNGs)
        gen_reset_seeded()
    elif "--eval" in sys.argv:   # eval_ctde.npz only, own seed
        np.random.seed(12345)
        import random
        random.seed(12345)
        gen_eval(np.random.default_rng(20261017))
    elif "--task-marl" in sys.argv:   # task_marl.npz only, own seed (regenerated for the step_counter order)
        np.random.seed(12345)
        gen_task_marl(np.random.default_rng(20261016))
    else:
        main()
        gen_physics()
