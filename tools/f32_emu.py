"""Host emulation of the f32 throughput mode's drone path (ch_device.h pid_vel + drone_substep, PYB body wrench),
to find which pieces must be carried in f64 for the body rates (obs columns 7-9) to hold 1e-4 relative.

Every section is evaluated in the precision named by a policy (f32 = numpy float32 arithmetic, one rounding per
operation as the kernel's -ffp-contract=off code; f64 = float64) from oracle states (tests/diag/f32_probe.py's
draw), and the angular velocity after one control step is compared with the fp64 oracle's.

  python tools/f32_emu.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

KG, KMASS, KKF, KKM = 9.8, 0.027, 3.16e-10, 7.94e-12
KJ = (1.4e-5, 1.4e-5, 2.17e-5)
PWS, PWC = 0.2685, 4070.3


def quat_to_mat(q, t):
    x, y, z, w = (t(q[..., i]) for i in range(4))
    d = x * x + y * y + z * z + w * w
    s = t(2.0) / d
    xs, ys, zs = x * s, y * s, z * s
    wx, wy, wz, xx, xy, xz = w * xs, w * ys, w * zs, x * xs, x * ys, x * zs
    yy, yz, zz = y * ys, y * zs, z * zs
    one = t(1.0)
    return [one - (yy + zz), xy - wz, xz + wy, xy + wz, one - (xx + zz), yz - wx, xz - wy, yz + wx, one - (xx + yy)]


def euler(q, t):
    x, y, z, w = (t(q[..., i]) for i in range(4))
    sarg = t(-2.0) * (x * z - w * y)
    r = np.arctan2(t(2) * (y * z + w * x), w * w - x * x - y * y + z * z)
    p = np.arcsin(sarg)
    yw = np.arctan2(t(2) * (x * y + w * z), w * w + x * x - y * y - z * z)
    return [t(r), t(p), t(yw)]


def pid(pos, q, vel, rpy, tv, pidst, dt_ctrl, pol):
    """pid_vel: returns rpm (in pol['mix'] precision) and the updated pid state."""
    t = pol["pos"]
    dt = t(dt_ctrl)
    pe = [t(pos[..., 0]) * 0 + t(0), t(0) * t(pos[..., 1]), t(0.45) - t(pos[..., 2])]
    pe[0] = t(pos[..., 0]) - t(pos[..., 0]); pe[1] = t(pos[..., 1]) - t(pos[..., 1])
    ve = [t(tv[i]) - t(vel[..., i]) for i in range(3)]
    ip = [np.clip(t(pidst[:, 3 + i]) + pe[i] * dt, t(-2.), t(2.)) for i in range(3)]
    ip[2] = np.clip(ip[2], t(-0.15), t(.15))
    PF, IF, DF = (.4, .4, 1.25), (.05, .05, .05), (.2, .2, .5)
    T = [t(PF[i]) * pe[i] + t(IF[i]) * ip[i] + t(DF[i]) * ve[i] for i in range(3)]
    T[2] = T[2] + t(KG * KMASS)
    Rm = quat_to_mat(q, t)
    sc = T[0] * Rm[2] + T[1] * Rm[5] + T[2] * Rm[8]
    sc = np.where(sc > 0, sc, t(0))
    thrust = (np.sqrt(sc / (t(4) * t(KKF))) - t(PWC)) / t(PWS)
    ta = pol["att"]
    T = [ta(x) for x in T]
    Rm = quat_to_mat(q, ta)
    tn = np.sqrt(T[0] * T[0] + T[1] * T[1] + T[2] * T[2])
    z = [T[i] / tn for i in range(3)]
    yaw = ta(rpy[2])
    xc = [np.cos(yaw), np.sin(yaw), ta(0)]
    yt = [z[1] * xc[2] - z[2] * xc[1], z[2] * xc[0] - z[0] * xc[2], z[0] * xc[1] - z[1] * xc[0]]
    yn = np.sqrt(yt[0] * yt[0] + yt[1] * yt[1] + yt[2] * yt[2])
    y = [yt[i] / yn for i in range(3)]
    x = [y[1] * z[2] - y[2] * z[1], y[2] * z[0] - y[0] * z[2], y[0] * z[1] - y[1] * z[0]]
    Rt = [x[0], y[0], z[0], x[1], y[1], z[1], x[2], y[2], z[2]]

    def E(i, j):
        a = ta(0); b = ta(0)
        for k in range(3):
            a = a + Rt[k * 3 + i] * Rm[k * 3 + j]
            b = b + Rm[k * 3 + i] * Rt[k * 3 + j]
        return a - b
    rot_e = [E(2, 1), E(0, 2), E(1, 0)]
    td = pol["rate"]
    dtd = td(dt_ctrl)
    rates_e = [td(0) - (td(rpy[i]) - td(pidst[:, i])) / dtd for i in range(3)]
    ir = [np.clip(ta(pidst[:, 6 + i]) - rot_e[i] * ta(dt_ctrl), ta(-1500.), ta(1500.)) for i in range(3)]
    ir[0] = np.clip(ir[0], ta(-1), ta(1)); ir[1] = np.clip(ir[1], ta(-1), ta(1))
    tm = pol["mix"]
    PT, IT, DT = (70000., 70000., 60000.), (0., 0., 500.), (20000., 20000., 12000.)
    tt = [np.clip(-tm(PT[i]) * tm(rot_e[i]) + tm(DT[i]) * tm(rates_e[i]) + tm(IT[i]) * tm(ir[i]), tm(-3200), tm(3200))
          for i in range(3)]
    MIX = ((-.5, -.5, -1), (-.5, .5, 1), (.5, .5, -1), (.5, -.5, 1))
    rpm = []
    for k in range(4):
        pwm = tm(thrust) + (tm(MIX[k][0]) * tt[0] + tm(MIX[k][1]) * tt[1] + tm(MIX[k][2]) * tt[2])
        pwm = np.clip(pwm, tm(20000), tm(65535))
        rpm.append(tm(PWS) * pwm + tm(PWC))
    return rpm


def substep(q, v, w, rpm, dt_, pol, ql):
    """pol keys: sub (state precision), wrench (prop forces / torques), wb, damp, gyro, ab, aw, wup (each piece of
    the body-rate update; default = wrench).  ql: Bullet's cached link frame (ch_device.h drone_substep, link_lag)."""
    t = pol["sub"]
    tw = pol["wrench"]
    P = lambda k: pol.get(k, tw)  # noqa: E731
    M = quat_to_mat(q, t)
    Ml = quat_to_mat(ql, t)
    r = [tw(x) for x in rpm]
    Mw = [tw(x) for x in M]
    Mlw = [tw(x) for x in Ml]
    tq = [r[i] * r[i] * tw(KKM) for i in range(4)]
    tz = -tq[0] + tq[1] - tq[2] + tq[3]
    f = [r[i] * r[i] * tw(KKF) for i in range(4)]
    Tt = ((f[0] + f[1]) + f[2]) + f[3]
    F = [t(Mlw[2] * Tt), t(Mlw[5] * Tt), t(Mlw[8] * Tt)]
    u = [(Mw[0 + i] * Mlw[2] + Mw[3 + i] * Mlw[5]) + Mw[6 + i] * Mlw[8] for i in range(3)]
    sy = tw(0.028) * (((-f[0] - f[1]) + f[2]) + f[3])
    sx = tw(0.028) * (((-f[0] + f[1]) + f[2]) - f[3])
    tb = [sy * u[2] + u[0] * tz, sx * u[2] + u[1] * tz, (-sx * u[1] - sy * u[0]) + u[2] * tz]
    F[2] = F[2] + t(-KMASS * KG)
    k = t(0.04)
    vv = [t(x) for x in v]
    sp = np.sqrt(vv[0] * vv[0] + vv[1] * vv[1] + vv[2] * vv[2])
    F = [F[i] - t(KMASS) * vv[i] * (k + k * sp) for i in range(3)]
    a_ = P("wb")
    wb = [a_(M[0 + i]) * a_(w[0]) + a_(M[3 + i]) * a_(w[1]) + a_(M[6 + i]) * a_(w[2]) for i in range(3)]
    a_ = P("damp")
    J = [a_(x) for x in KJ]
    kw = a_(0.04)
    wbd = [a_(x) for x in wb]
    sw = np.sqrt(wbd[0] * wbd[0] + wbd[1] * wbd[1] + wbd[2] * wbd[2])
    dmp = [J[i] * wbd[i] * (kw + kw * sw) for i in range(3)]
    a_ = P("gyro")
    J = [a_(x) for x in KJ]
    wbg = [a_(x) for x in wb]
    Jw = [J[i] * wbg[i] for i in range(3)]
    g = [wbg[1] * Jw[2] - wbg[2] * Jw[1], wbg[2] * Jw[0] - wbg[0] * Jw[2], wbg[0] * Jw[1] - wbg[1] * Jw[0]]
    a_ = P("ab")
    tb = [a_(tb[i]) - a_(dmp[i]) for i in range(3)]
    tb = [tb[i] - a_(g[i]) for i in range(3)]
    ab = [tb[i] / a_(KJ[i]) for i in range(3)]
    dt = t(dt_)
    nv = [vv[i] + F[i] / t(KMASS) * dt for i in range(3)]
    nw = []
    for i in range(3):
        a_ = P("aw")
        aw = a_(M[i * 3 + 0]) * a_(ab[0]) + a_(M[i * 3 + 1]) * a_(ab[1]) + a_(M[i * 3 + 2]) * a_(ab[2])
        a_ = P("wup")
        nw.append(pol["wstate"](a_(w[i]) + a_(aw) * a_(dt_)))
    ws = [t(x) for x in nw]
    fang = np.sqrt(ws[0] * ws[0] + ws[1] * ws[1] + ws[2] * ws[2])
    s = np.sin(t(0.5) * fang * dt) / np.where(fang > 0, fang, t(1))
    s = np.where(fang < t(0.001), t(0.5) * dt - (dt * dt * dt) * t(0.020833333333) * fang * fang, s)
    ch = np.cos(t(0.5) * fang * dt)
    a = [ws[0] * s, ws[1] * s, ws[2] * s, ch]
    qq = [t(q[..., i]) for i in range(4)]
    o = [a[3] * qq[0] + a[0] * qq[3] + a[1] * qq[2] - a[2] * qq[1],
         a[3] * qq[1] + a[1] * qq[3] + a[2] * qq[0] - a[0] * qq[2],
         a[3] * qq[2] + a[2] * qq[3] + a[0] * qq[1] - a[1] * qq[0],
         a[3] * qq[3] - a[0] * qq[0] - a[1] * qq[1] - a[2] * qq[2]]
    n = np.sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2] + o[3] * o[3])
    nq = np.stack([o[i] / n for i in range(4)], -1)
    return nq, nv, nw, np.stack(qq, -1)


def run(states, acts, pol, n):
    S = lambda k: np.concatenate([np.asarray(s[k])[:n] for s in states])  # noqa: E731
    st = pol["state"]
    pos, q, vel, w = S("drone_pos"), st(S("drone_quat")), st(S("drone_vel")), st(S("drone_angv"))
    ql = st(S("drone_qlag"))
    pidst = np.concatenate([S("pid_last_rpy"), S("pid_int_pos"), S("pid_int_rpy")], 1)
    pidst = st(pidst)
    a = acts.reshape(-1, 4).astype(np.float32)
    hn = np.sqrt(a[:, 0] * a[:, 0] + a[:, 1] * a[:, 1])
    ux = np.where(hn != 0, a[:, 0] / np.where(hn != 0, hn, 1), 0).astype(np.float32)
    uy = np.where(hn != 0, a[:, 1] / np.where(hn != 0, hn, 1), 0).astype(np.float32)
    sc = np.float32(0.3 * 30.0 * (1000.0 / 3600.0)) * np.abs(a[:, 3])
    tv = [ux.astype(np.float64) * sc, uy.astype(np.float64) * sc, 0.0 * sc.astype(np.float64)]
    rpy = euler(q, pol["euler"])
    rpm = pid(pos, q, vel, rpy, tv, pidst, 1 / 60, pol)
    v = [vel[:, i] for i in range(3)]
    ww = [w[:, i] for i in range(3)]
    wc = pol.get("wcarry", st)
    for _ in range(4):
        q, v, ww, ql = substep(q, v, ww, rpm, 1 / 240, pol, ql)
        q = st(q); v = [st(x) for x in v]; ww = [wc(x) for x in ww]
    ww = [st(x) for x in ww]
    return np.stack([np.asarray(x, np.float64) for x in ww], 1)


def draw(E=256, seed=3):
    """E oracle envs after 0-119 random steps (tests/diag/f32_probe.py's draw), one random action row each, and the
    fp64 oracle's angular velocity after that step."""
    import oracle as O
    from cattleherd._lib import spawn_table
    n, m = 4, 16
    table = spawn_table(m)
    rng = np.random.default_rng(seed)
    envs, states = [], []
    for e in range(E):
        env = O.Env(0, n, m, table, start_level=7, env_id=e)
        env.reset()
        for _ in range(int(rng.integers(0, 120))):
            env.step(rng.uniform(-1, 1, (n, 4)).astype(np.float32), autoreset=True)
        envs.append(env)
        states.append(env.get_state())
    acts = np.random.default_rng(1).uniform(-1, 1, (E, n, 4)).astype(np.float32)
    for e, env in enumerate(envs):
        env.step(acts[e], autoreset=False)
    ref = np.concatenate([np.asarray(env.get_state()["drone_angv"])[:n] for env in envs])
    return states, acts, ref, n


def policies():
    f32, f64 = np.float32, np.float64
    base = dict(state=f32, pos=f32, euler=f32, att=f32, rate=f32, mix=f32, sub=f32, wrench=f32, wstate=f32)
    mw = {**base, "mix": f64, "wrench": f64}
    pols = {
        "all f64": {k: f64 for k in base},
        "all f32 (before round 4)": base,
        "f64 mix": {**base, "mix": f64},
        "f64 wrench": {**base, "wrench": f64},
        "f64 mix+wrench": mw,
        "f64 mix + prop torque only": {**mw, "wb": f32, "damp": f32, "gyro": f32, "ab": f32, "aw": f32, "wup": f32},
    }
    for piece in ("wb", "damp", "gyro", "ab", "aw", "wup"):
        pols[f"f64 mix+wrench but {piece} f32"] = {**mw, piece: f32}
    pols["f64 mix+wrench but wb, damp, gyro f32"] = {**mw, "wb": f32, "damp": f32, "gyro": f32}
    # what ch_device.h does since round 4: torque mix + motor speeds (pid_vel), prop forces / torque, world angular
    # acceleration and the angular-velocity update (drone_substep) in f64
    pols["kernel (round 4)"] = {**mw, "wb": f32, "damp": f32, "gyro": f32, "ab": f32}
    pols["f64 mix+wrench but wb, damp, gyro, aw f32"] = {**mw, "wb": f32, "damp": f32, "gyro": f32, "aw": f32}
    # round 6: with Bullet's cached link frame the yaw rate couples to the roll / pitch torques; what 1e-4 elementwise
    # on the yaw rate would take (the yaw column of main()'s output)
    kern = pols["kernel (round 4)"]
    pid64 = {**kern, "pos": f64, "euler": f64, "att": f64, "rate": f64}
    pols["kernel + PID all f64"] = pid64
    pols["kernel + PID all f64 + state f64"] = {**pid64, "state": f64}
    return pols


def errors(pol, d):
    """(max abs, max relative with a 1e-6 floor, the yaw rate's max relative with the test's 1e-8 floor) of the body
    rates as the f32 observation holds them."""
    states, acts, ref, n = d
    g32 = run(states, acts, pol, n).astype(np.float32).astype(np.float64)
    r32 = ref.astype(np.float32).astype(np.float64)
    diff = np.abs(g32 - r32)
    return (float(diff.max()), float((diff / np.maximum(np.abs(ref), 1e-6)).max()),
            float((diff[:, 2] / (1e-8 + np.abs(ref[:, 2]))).max()))


def main():
    d = draw()
    for name, pol in policies().items():
        a, r, y = errors(pol, d)
        print(f"{name:42s} max abs {a:.3e}  max rel (1e-6 floor) {r:.3e}  yaw rel (1e-8 floor) {y:.3e}")


if __name__ == "__main__":
    main()
