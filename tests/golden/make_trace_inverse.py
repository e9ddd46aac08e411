"""Pin the drone rigid body to real PyBullet: action inversion of the recorded evaluation trace.

Generator-side (run in this container; writes ``trace_inverse.npz``).  It reads only the committed fixture
``trace_eval.npz`` (the real-PyBullet trace ``simulator/evaluation_data.pkl`` sliced by ``extract_trace.py``) and
the oracle -- nothing from ``/root/reference``.

The trace was written by ``evaluate_policy(model, test_env_nogui, n_eval_episodes=5)`` with a deterministic SB3
policy (reference ``simulator/CTDECattleHerder.py:169-185``, ``utils/evaluation.py:73-94``): 3 drones, 16 cattle,
drone and cattle xy position and velocity after every control step, real Bullet in the loop.  The policy that
drove it is not among the shipped checkpoints (``make_trace_policy_search.py`` -> ``trace_policy_search.json``,
DESIGN.md §3), so the actions are recovered instead:

* ``seg0`` is the first evaluation episode of a fresh env -- drones at rest at (1.75 i, 0, 0.45), identity
  attitude, PID state zero (the controllers are created in the constructor and never reset,
  ``sb3_envs/BaseRLAviary.py:80``), cattle at ``pos[0] - vel[0] / 60``.  ``seg1`` starts after earlier episodes whose
  PID state carries over unknown, so it is not replayed.
* **Model test (float64 targets).**  A VEL action reaches the physics only through the PID's target velocity
  ``SPEED_LIMIT |a3| (a0, a1) / |(a0, a1)|`` (``BaseRLAviary.py:185-222``; z and yaw targets do not depend on it), so
  step by step and drone by drone the two target components are solved in float64 -- the oracle's test hook
  ``och__set_target_vel`` bypasses the float32 action row -- by least squares on the oracle's drone xy velocity AND
  position after the step against the trace's.  The drones do not interact under ``Physics.PYB``, so each
  drone-step is 2 unknowns against 4 recorded numbers: the residual tests the physics model, not a fit of it.  Run
  under the shipped model (Bullet's cached link frame, ``link_lag=1``) and its alternatives (``MODELS``).
* **Realisable actions.**  The shipped model's float64 targets are then realised as float32 triples (a0, a1, a3)
  -- the action's real degrees of freedom, with ``_preprocessAction``'s float32 normalisation and scale -- by an
  ulp-neighbourhood search (target error <= ~4e-8 m/s), and replayed through the unmodified step.  The fixture
  keeps the steps of that replay up to ``KEEP`` and its per-step residuals.

    python tests/golden/make_trace_inverse.py [steps]
"""
import ctypes
import os
import sys

import numpy as np
from scipy.optimize import least_squares

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
import oracle as O  # noqa: E402

N, M = 3, 16
SL32 = np.float32(0.3 * 30.0 * 1000.0 / 3600.0)   # SPEED_LIMIT as the float32 product sees it (ch_oracle.c och_step)

# model name -> (Env keywords, oracle model-flag bits).  torque_world = 2: the z torque in the world frame even under
# the cached link frame (PyBullet's LINK_FRAME torque quirk on a base, SURVEY.md:261); flag bit 0: a
# velocity-product term m w x v in the base's linear acceleration (a body-frame spatial-acceleration slip)
MODELS = {"lag": (dict(link_lag=1, torque_world=0), 0),
          "nolag": (dict(link_lag=0), 0),
          "lag_nogyro": (dict(link_lag=1, torque_world=0, gyro=False), 0),
          "lag_nodamp": (dict(link_lag=1, torque_world=0, damping=0.0), 0),
          "lag_worldtz": (dict(link_lag=1, torque_world=2), 0),
          "lag_wxv": (dict(link_lag=1, torque_world=0), 1)}
KEEP = 14


def initial_state(env, tr):
    s = env.get_state()
    for i in range(O.NMAX):
        s["drone_pos"][i] = [1.75 * i, 0.0, 0.45] if i < N else [0.0, 0.0, 0.0]
        s["drone_quat"][i] = [0, 0, 0, 1]
        s["drone_qlag"][i] = [0, 0, 0, 1]
        for k in ("drone_vel", "drone_angv", "pid_last_rpy", "pid_int_pos", "pid_int_rpy"):
            s[k][i] = 0.0
    cp = np.zeros((O.MMAX, 2))
    cv = np.zeros((O.MMAX, 2))
    cp[:M] = tr["seg0_cattle_pos"][0] - tr["seg0_cattle_vel"][0] / 60.0
    cv[:M] = tr["seg0_cattle_vel"][0]
    s.update(n=N, cow_pos=cp, cow_vel=cv, step_counter=0, step_counter_A=0, has_prev=0, clock=0.0,
             active=np.array([1] * N + [0] * (O.NMAX - N), np.uint8))
    env.set_state(s)


class Stepper:
    """One env of the oracle; evaluates candidate targets on copies of its state."""

    def __init__(self, kw, tr):
        self.env = O.Env(0, N, M, np.zeros((100, 16, 2)), **kw)
        initial_state(self.env, tr)
        self.L = O.lib()
        self.tmp = O.State()
        self.o = np.zeros((12, 86), np.float32)
        self.r = np.zeros(1)
        self.te = np.zeros(1, np.uint8)
        self.tru = np.zeros(1, np.uint8)

    def trial(self, acts):
        ctypes.memmove(ctypes.byref(self.tmp), ctypes.byref(self.env.st), ctypes.sizeof(O.State))
        a = np.ascontiguousarray(acts, np.float32)
        self.L.och_step(ctypes.byref(self.env.cfg), ctypes.byref(self.tmp), O._fp(a), O._fp(self.o), O._dp(self.r),
                        O._u8(self.te), O._u8(self.tru), None, 0)
        return self.tmp

    def commit(self, acts):
        self.env.step(acts, autoreset=False)


def _stats(g):
    q = g["drone_quat"][:N]
    tilt = np.degrees(np.arccos(np.clip(1 - 2 * (q[:, 0] ** 2 + q[:, 1] ** 2), -1, 1)))
    return np.hypot(g["drone_vel"][:N, 0], g["drone_vel"][:N, 1]).max(), tilt.max()


def fit_targets(name, tr, K, log=print):
    """Per step and drone the float64 target velocity (2 unknowns, bounded by SPEED_LIMIT) that best reproduces the
    trace's xy velocity and position after the step; returns targets [K, N, 2] and per-step max residuals."""
    kw, flags = MODELS[name]
    L = O.lib()
    L.och__set_target_vel.argtypes = [ctypes.c_void_p]
    L.och__set_model_flags(flags)
    tv, tp = tr["seg0_drone_vel"], tr["seg0_drone_pos"]
    st = Stepper(kw, tr)
    over = np.zeros(3 * O.NMAX)
    L.och__set_target_vel(over.ctypes.data)
    zero = np.zeros((N, 4), np.float32)
    targets, dvs, dps, speeds, tilts = [], [], [], [], []
    try:
        for t in range(K):
            for i in range(N):
                def res(x, i=i):
                    over[3 * i], over[3 * i + 1] = x
                    s = st.trial(zero)
                    return np.concatenate([(np.array([s.dv[i][0], s.dv[i][1]]) - tv[t, i]) * 1e4,
                                           (np.array([s.dp[i][0], s.dp[i][1]]) - tp[t, i]) * 6e5])
                best = None
                starts = [over[3 * i:3 * i + 2].copy()] + [
                    float(SL32) * np.array([r * np.cos(f), r * np.sin(f)]) for r in (0.1, 0.5, 0.95)
                    for f in np.linspace(-np.pi, np.pi, 13)[:-1]]
                for s0 in starts:
                    sol = least_squares(res, np.clip(s0, -2.5, 2.5), bounds=([-2.5, -2.5], [2.5, 2.5]), xtol=1e-15,
                                        ftol=1e-15, gtol=1e-15, diff_step=1e-7, max_nfev=200)
                    if best is None or sol.cost < best.cost:
                        best = sol
                    if best.cost < 1e-16:
                        break
                over[3 * i], over[3 * i + 1] = best.x
            st.commit(zero)
            g = st.env.get_state()
            targets.append(over[:3 * N].reshape(N, 3)[:, :2].copy())
            dvs.append(np.abs(g["drone_vel"][:N, :2] - tv[t]).max())
            dps.append(np.abs(g["drone_pos"][:N, :2] - tp[t]).max())
            sp, ti = _stats(g)
            speeds.append(sp)
            tilts.append(ti)
            log(f"  {name:11s} step {t:3d}: |dv| {dvs[-1]:.2e}  |dp| {dps[-1]:.2e}  speed {sp:.3f} m/s  tilt {ti:.1f} deg")
    finally:
        L.och__set_target_vel(None)
        L.och__set_model_flags(0)
    return np.array(targets), np.array(dvs), np.array(dps), np.array(speeds), np.array(tilts)


def target_of(a):
    """_preprocessAction's float32 target velocity (x, y) of an action row (a0, a1, a3) (ch_oracle.c och_step)."""
    hx, hy, a3 = np.float32(a[0]), np.float32(a[1]), np.float32(a[2])
    hn = np.sqrt(np.float32(hx * hx + hy * hy))
    ux, uy = (hx / hn, hy / hn) if hn != 0 else (np.float32(0), np.float32(0))
    sc = np.float32(SL32 * np.abs(a3))
    return np.array([float(ux) * float(sc), float(uy) * float(sc)])


def realise(target, rng):
    """A float32 triple (a0, a1, a3) in [-1, 1] whose target velocity is closest to `target`: the direction at
    several scales (the normalisation makes them equivalent up to rounding) and random ulp steps of all three."""
    r = float(np.hypot(*target))
    best, be = None, np.inf
    for scale in (1.0, 0.9, 0.75, 0.6, 0.5, 0.33, 0.25):
        base = np.array([target[0] / r * scale, target[1] / r * scale, r / float(SL32)], np.float32)
        for j in range(401):
            c = base.copy()
            if j:
                for k, d in enumerate(rng.integers(-6, 7, 3)):
                    for _ in range(abs(int(d))):
                        c[k] = np.nextafter(c[k], np.float32(np.sign(d) * 2.0))
            e = np.abs(target_of(c) - target).max()
            if e < be:
                be, best = e, c
    return best, be


def replay(acts, tr, kw=MODELS["lag"][0], flags=0):
    O.lib().och__set_model_flags(flags)
    st = Stepper(kw, tr)
    dv, dp = [], []
    for t in range(len(acts)):
        st.commit(acts[t])
        g = st.env.get_state()
        dv.append(np.abs(g["drone_vel"][:N, :2] - tr["seg0_drone_vel"][t]).max())
        dp.append(np.abs(g["drone_pos"][:N, :2] - tr["seg0_drone_pos"][t]).max())
    O.lib().och__set_model_flags(0)
    return np.array(dv), np.array(dp)


def main(K=16, out=os.path.join(HERE, "trace_inverse.npz")):
    tr = np.load(os.path.join(HERE, "trace_eval.npz"))
    arrays = {}
    for name in MODELS:
        targets, dv, dp, sp, ti = fit_targets(name, tr, K)
        arrays[name + "_dv"], arrays[name + "_dp"] = dv, dp
        if name == "lag":
            arrays["speed"], arrays["tilt_deg"], lag_targets = sp, ti, targets
    rng = np.random.default_rng(0)
    acts = np.zeros((K, N, 4), np.float32)
    rerr = 0.0
    for t in range(K):
        for i in range(N):
            a, e = realise(lag_targets[t, i], rng)
            acts[t, i] = [a[0], a[1], 0.0, a[2]]
            rerr = max(rerr, e)
    rdv, rdp = replay(acts, tr)
    keep = min(KEEP, K)
    for name, (kw, flags) in MODELS.items():   # the same float32 actions through every model (no refit)
        d1, p1 = replay(acts[:keep], tr, kw, flags)
        arrays[name + "_replay_dv"], arrays[name + "_replay_dp"] = d1, p1
    np.savez_compressed(out, actions=acts[:keep], steps=keep, trace_vel=tr["seg0_drone_vel"][:keep],
                        trace_pos=tr["seg0_drone_pos"][:keep], cattle_pos0=tr["seg0_cattle_pos"][0],
                        cattle_vel0=tr["seg0_cattle_vel"][0], replay_dv=rdv[:keep], replay_dp=rdp[:keep],
                        target_realisation_err=rerr, fit_steps=K, **arrays)
    print(f"kept {keep} steps; float32 realisation error {rerr:.1e} m/s")
    for t in range(K):
        print(f"step {t:2d}: speed {arrays['speed'][t]:.3f} tilt {arrays['tilt_deg'][t]:5.1f}  float64 fit "
              + "  ".join(f"{n} {arrays[n + '_dv'][t]:.1e}" for n in MODELS)
              + f"  | float32 replay {rdv[t]:.1e} / {rdp[t]:.1e}")


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
