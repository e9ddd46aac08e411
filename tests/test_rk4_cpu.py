"""CPU tests of the RK4 integrator option (north_star's "RK4 attitude/position update"; not a reference
path -- the reference has Bullet's semi-implicit step (PYB) and explicit Euler (DYN,
sb3_envs/BaseAviary.py:1043-1118)).  The oracle's RK4 integrates the DYN equations of motion; held to its
order of accuracy: halving the substep divides the error by ~16 (explicit Euler DYN: by ~2), measured
against a 256x finer RK4 solution of the same ODE, and it agrees with DYN as dt -> 0."""
import ctypes

import numpy as np


def _integrate(y0, rpm, dt, steps, rk4):
    import oracle as O
    L = O.lib()
    L.och_dyn_integrate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_int64, ctypes.c_int]
    y = np.ascontiguousarray(y0, np.float64).copy()
    r = np.ascontiguousarray(rpm, np.float64)
    L.och_dyn_integrate(y.ctypes.data, r.ctypes.data, dt, int(steps), int(rk4))
    return y


def _y0():
    q = np.array([0.05, -0.03, 0.2, 1.0])
    q /= np.linalg.norm(q)
    # p, v, q, body rates, (world rates out)
    return np.concatenate([[0.3, -0.2, 0.45], [0.4, -0.1, 0.05], q, [1.5, -2.0, 3.0], [0, 0, 0]])


def _err(a, b):
    return float(np.max(np.abs(a[:13] - b[:13])))


def test_rk4_is_fourth_order_and_dyn_first_order():
    rpm = np.array([14700.0, 14300.0, 14650.0, 14200.0])   # uneven: body torques and a spinning attitude
    T, base = 0.05, 1.0 / 240
    ref = _integrate(_y0(), rpm, base / 256, int(round(T / (base / 256))), 1)
    errs = {rk: [] for rk in (0, 1)}
    for k in range(4):
        dt = base / 2 ** k
        for rk in (0, 1):
            errs[rk].append(_err(_integrate(_y0(), rpm, dt, int(round(T / dt)), rk), ref))
    r4 = [errs[1][k] / errs[1][k + 1] for k in range(3)]
    r1 = [errs[0][k] / errs[0][k + 1] for k in range(3)]
    assert all(12.0 < r < 20.0 for r in r4), (r4, errs[1])
    assert all(1.6 < r < 2.5 for r in r1), (r1, errs[0])
    assert errs[1][0] < 1e-3 * errs[0][0]


def test_rk4_keeps_unit_quaternion_and_world_rates():
    rpm = np.array([14700.0, 14300.0, 14650.0, 14200.0])
    y = _integrate(_y0(), rpm, 1.0 / 240, 240, 1)
    q = y[6:10]
    assert abs(np.linalg.norm(q) - 1.0) < 1e-15
    x, yy, z, w = q
    # world angular velocity = R(q) w_b (pybullet matrix convention, ch_oracle.c och_matrix_from_quat)
    R = np.array([[1 - 2 * (yy * yy + z * z), 2 * (x * yy - z * w), 2 * (x * z + yy * w)],
                  [2 * (x * yy + z * w), 1 - 2 * (x * x + z * z), 2 * (yy * z - x * w)],
                  [2 * (x * z - yy * w), 2 * (yy * z + x * w), 1 - 2 * (x * x + yy * yy)]])
    assert np.allclose(y[13:16], R @ y[10:13], rtol=1e-12, atol=1e-12)
