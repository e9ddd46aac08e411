"""Pin the drone rigid body to real PyBullet: action inversion of the recorded evaluation trace.

Generator-side (run in this container; writes ``trace_inverse.npz``).  It reads only the committed fixture
``trace_eval.npz`` (the real-PyBullet trace ``simulator/evaluation_data.pkl`` sliced by ``extract_trace.py``) and
the oracle -- nothing from ``/root/reference``.

The trace was written by ``evaluate_policy(model, test_env_nogui, n_eval_episodes=5)`` with a deterministic SB3
policy (reference ``simulator/CTDECattleHerder.py:169-185``, ``utils/evaluation.py:73-94``): 3 drones, 16 cattle,
drone and cattle xy position and velocity after every control step, real Bullet in the loop.  The policy that
drove it is not among the shipped checkpoints: none of the 19 (of 82) with a 3 x 86 input reproduces even the sign
pattern of the first step's drone velocities (``make_trace_policy_search.py`` -> ``trace_policy_search.json``,
DESIGN.md §3).  So the actions are recovered instead:

* ``seg0`` is the first evaluation episode of a fresh env -- drones at rest at (1.75 i, 0, 0.45), identity
  attitude, PID state zero (the controllers are created in the constructor and never reset,
  ``sb3_envs/BaseRLAviary.py:80``), cattle at ``pos[0] - vel[0] / 60`` (no flocking step on step 1).  ``seg1``
  starts after earlier episodes whose PID state carries over unknown, so it is not replayed.
* Step by step and drone by drone, the VEL action (a0, a1, 0, a3) is solved (float32, as the env reads it) by
  least squares on the oracle's drone xy velocity AND position after the step against the trace's.  The drones
  do not interact under ``Physics.PYB``, so each drone-step is 2 unknowns against 4 recorded numbers: the
  residual left is a test of the physics model (over a control step the position integrates the velocity of
  four substeps, i.e. the intra-step profile of thrust direction, attitude and damping), not a fit of it.

Run under the model with Bullet's cached link frame (``link_lag=1``, the default) and under its alternatives --
the rounds 1-4 model (``link_lag=0``), no gyroscopic term, no damping -- the residuals differ by orders of
magnitude (printed, stored).  The fixture keeps the ``link_lag=1`` actions of the steps whose
position residual stays below ``POS_TOL``; the float32 rounding of the recovered actions is what limits it
(a float64 target-velocity fit holds ~1e-11 for ten steps).

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
POS_TOL = 1e-9


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


def action_of(x):
    """A VEL action with target velocity 2.5 (x, y) (|(x, y)| <= 1): direction (x, y), speed |a3| = |(x, y)|."""
    x = np.asarray(x, np.float64)
    r = float(np.hypot(x[0], x[1]))
    if r > 1.0:
        x = x / r
        r = 1.0
    return np.array([x[0], x[1], 0.0, r], np.float32)


class Stepper:
    """One env of the oracle; evaluates candidate actions on copies of its state."""

    def __init__(self, model, tr):
        table = np.zeros((100, 16, 2))
        self.env = O.Env(0, N, M, table, **model)
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


def invert(model, tr, K, log=print):
    tv, tp = tr["seg0_drone_vel"], tr["seg0_drone_pos"]
    st = Stepper(model, tr)
    acts = np.zeros((N, 4), np.float32)
    guess = np.zeros((N, 2))
    out_a, out_v, out_p = [], [], []
    for t in range(K):
        for i in range(N):
            def res(x, i=i):
                a = acts.copy()
                a[i] = action_of(x)
                s = st.trial(a)
                return np.concatenate([(np.array([s.dv[i][0], s.dv[i][1]]) - tv[t, i]) * 1e4,
                                       (np.array([s.dp[i][0], s.dp[i][1]]) - tp[t, i]) * 6e5])
            best = None
            starts = [guess[i]] + [np.array([r * np.cos(f), r * np.sin(f)]) for r in (0.1, 0.5, 0.95)
                                   for f in np.linspace(-np.pi, np.pi, 13)[:-1]]
            for s0 in starts:
                sol = least_squares(res, s0, bounds=([-1, -1], [1, 1]), xtol=1e-15, ftol=1e-15, gtol=1e-15,
                                    diff_step=1e-5, max_nfev=200)
                if best is None or sol.cost < best.cost:
                    best = sol
                if best.cost < 1e-14:
                    break
            guess[i] = best.x
            acts[i] = action_of(best.x)
        st.commit(acts)
        g = st.env.get_state()
        v = g["drone_vel"][:N, :2].copy()
        p = g["drone_pos"][:N, :2].copy()
        out_a.append(acts.copy()); out_v.append(v); out_p.append(p)
        log(f"  step {t:3d}: |dv| max {np.abs(v - tv[t]).max():.2e}  |dp| max {np.abs(p - tp[t]).max():.2e}")
    return np.array(out_a), np.array(out_v), np.array(out_p)


MODELS = {"lag": dict(link_lag=1), "nolag": dict(link_lag=0), "lag_nogyro": dict(link_lag=1, gyro=False),
          "lag_nodamp": dict(link_lag=1, damping=0.0)}


def main(K=9, out=os.path.join(HERE, "trace_inverse.npz")):
    tr = np.load(os.path.join(HERE, "trace_eval.npz"))
    arrays = {}
    for name, kw in MODELS.items():
        print(name, kw)
        a, v, p = invert(kw, tr, K)
        arrays[name + "_dv"] = np.abs(v - tr["seg0_drone_vel"][:K]).reshape(K, -1).max(1)
        arrays[name + "_dp"] = np.abs(p - tr["seg0_drone_pos"][:K]).reshape(K, -1).max(1)
        if name == "lag":
            acts = a
    dp = arrays["lag_dp"]
    keep = int(np.argmax(dp > POS_TOL)) if (dp > POS_TOL).any() else K
    np.savez_compressed(out, actions=acts[:keep], steps=keep, trace_vel=tr["seg0_drone_vel"][:keep],
                        trace_pos=tr["seg0_drone_pos"][:keep], cattle_pos0=tr["seg0_cattle_pos"][0],
                        cattle_vel0=tr["seg0_cattle_vel"][0], **arrays)
    print(f"kept {keep} steps")
    for name in MODELS:
        print(f"{name:11s} max |dv| {arrays[name + '_dv'][:keep].max():.2e}  max |dp| {arrays[name + '_dp'][:keep].max():.2e}")


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
