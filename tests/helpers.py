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
                 "last_rpm", "rpy_rates", "active"):
            pad = np.zeros((nmax,) + x.shape[1:], x.dtype)
            pad[:x.shape[0]] = x
            if k == "drone_quat":
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
