"""Shared test helpers: golden-fixture loading and state conversion."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name))


def rollout_files():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "*_roll_*.npz")))


def state_at(d, prefix, i):
    """One state dict (no env axis) from a stacked fixture."""
    out = {}
    for k in d.files:
        if k.startswith(prefix) and k != prefix + "obs":
            v = d[k]
            out[k[len(prefix):]] = v[i] if v.ndim > 0 else v
    return out


def stack(states):
    return {k: np.stack([np.asarray(s[k]) for s in states]) for k in states[0]}


def oracle_view(g, e, nmax):
    """Env ``e`` of a HerdBatch.get_state() dict as an oracle Env.set_state() dict: per-drone arrays padded to
    the oracle's ``nmax`` drones (identity quaternions, inactive) -- the device state before a step."""
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


def close(a, b, rtol, atol):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    both_nan = np.isnan(a) & np.isnan(b)
    ok = np.isclose(a, b, rtol=rtol, atol=atol) | both_nan
    return bool(np.all(ok)), (float(np.max(np.abs(np.where(both_nan, 0, a - b)))) if a.size else 0.0)


def trace_seg0_state(nmax=12, mmax=64):
    """The state the recorded real-PyBullet trace's first evaluation episode starts from (trace_inverse.npz; see
    tests/golden/make_trace_inverse.py): 3 drones at rest at (1.75 i, 0, 0.45) with identity attitude and cached
    link frame, PID state zero, the 16 cows at pos[0] - vel[0] / 60 with vel[0]; counters at a fresh reset."""
    t = load("trace_inverse.npz")
    s = {k: np.zeros((nmax, w)) for k, w in (("drone_pos", 3), ("drone_quat", 4), ("drone_qlag", 4), ("drone_vel", 3),
                                             ("drone_angv", 3), ("pid_last_rpy", 3), ("pid_int_pos", 3),
                                             ("pid_int_rpy", 3))}
    for i in range(3):
        s["drone_pos"][i] = [1.75 * i, 0.0, 0.45]
    s["drone_quat"][:, 3] = 1.0
    s["drone_qlag"][:, 3] = 1.0
    cp, cv = np.zeros((mmax, 2)), np.zeros((mmax, 2))
    cp[:16] = t["cattle_pos0"] - t["cattle_vel0"] / 60.0
    cv[:16] = t["cattle_vel0"]
    s.update(n=3, cow_pos=cp, cow_vel=cv, step_counter=0, step_counter_A=0, has_prev=0, prev_cent=np.nan, clock=0.0,
             level=7, tally=0, spawn_index=2, active=np.array([1, 1, 1] + [0] * (nmax - 3), np.uint8))
    return s
