// ch_device.h — device-side math of the batched cattle-herding step (gfx950, HIP).
//
// Each function restates one piece of the reference's env.step() (paths relative to
// gym_pybullet_drones/ in BenCooper305/RL-Cattle-Herding).  Templated on the state precision R
// (double = the reference's arithmetic; float = throughput mode).  Operation order follows the
// reference so that, with -ffp-contract=off, the fp64 path reproduces the CPU oracle to the last
// few ulps (transcendentals differ by <= 1 ulp between ocml and glibc).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "ch_internal.h"

namespace ch {

// ---- constants: assets/cf2x.urdf:5-12, BaseAviary.py:97-173, DSLPIDControl.py:37-53 ----------
constexpr double kG = 9.8, kMass = 0.027, kKF = 3.16e-10, kKM = 7.94e-12;
constexpr double kJx = 1.4e-5, kJy = 1.4e-5, kJz = 2.17e-5;
constexpr double kTargetAlt = 0.45;
constexpr double kPwmScale = 0.2685, kPwmConst = 4070.3, kMinPwm = 20000, kMaxPwm = 65535;
constexpr double kMaxSpeedKmh = 30.0;
constexpr double kMaxVelCattle = 0.2;                       // BaseAviary.py:579
constexpr double kMissionBoundary = 15, kMaxFormation = 8, kCollision = 0.2;  // CattleAviary.py:94-97
constexpr double kPi = 3.14159265358979323846;

// curriculum_learning.py:10-194
__constant__ static const Level kLevels[8] = {
    {0.8, 0.3, 10, 0.0, 0, 0.0, 0.0, 3, 3, 40, 1, 0, 0, 0, 0, 0.0, 100},
    {0.8, 0.2, 25, 0.0, 0, 0.0, 0.0, 4, 4, 40, 0, 1, -0.5, 0, 0, 0.0, 300},
    {0.8, 0.2, 15, 0.6, 0, 0.0, 0.0, 4, 4, 40, 0, 0.8, 0, 1, 0, 0.0, 100},
    {0.8, 0.2, 15, 0.3, 0, 0.0, 0.0, 4, 4, 40, 0, 0.8, -0.5, 1, 0, 0.0, 400},
    {0.8, 0.2, 15, 0.3, 20, 0.0, 0.0, 4, 4, 80, 0, 0.7, -0.0, 0.8, 1, 0.0, 600},
    {0.8, 0.2, 15, 0.3, 50, 0.8, 0.1, 4, 4, 40, 0, 0.7, -0.5, 0.6, 1, 0.8, 600},
    {0.8, 0.3, 15, 0.2, 50, 0.0, 0.0, 4, 12, 80, 0.7, 0.0, -0.0, 0.8, 1, 0.0, 600},
    {0.8, 0.3, 15, 0.2, 50, 0.0, 0.0, 4, 12, 80, 0.0, 0.0, -0.0, 1, 1, 0.0, 600},
};

// Heavy libm entry points go through one out-of-line copy each (CH_NOINLINE_MATH) instead of being
// inlined at every call site: the fused step kernel is otherwise ~11k instructions and thrashes the
// shared instruction cache.
#ifdef CH_NOINLINE_MATH
#define CH_MATH_ATTR __device__ __noinline__
#else
#define CH_MATH_ATTR __device__ __forceinline__
#endif
template <class R> CH_MATH_ATTR R m_atan2(R y, R x) { return atan2(y, x); }
template <class R> CH_MATH_ATTR R m_asin(R x) { return asin(x); }
template <class R> CH_MATH_ATTR R m_exp(R x) { return exp(x); }
template <class R> CH_MATH_ATTR R m_cos(R x) { return cos(x); }
template <class R> CH_MATH_ATTR R m_sin(R x) { return sin(x); }
template <class R> CH_MATH_ATTR R m_pow(R x, R y) { return pow(x, y); }
// sin and cos of one argument share the range reduction
template <class R> CH_MATH_ATTR void m_sincos(R x, R* s, R* c) {
    if constexpr (sizeof(R) == 8) sincos(x, s, c);
    else sincosf(x, s, c);
}

// sin and cos of 0 <= x <= pi/4 with no argument reduction: the fdlibm __kernel_sin / __kernel_cos
// polynomials (their published coefficients; |x| < 0.3 and the x/4 split of __kernel_cos as selects).
// <= 1 ulp, like libm: tools/sincos_check.c measures them against glibc (max 1 ulp over 2e7
// arguments in [0, pi/8]).  About 25 VALU instead of ~70 for the reducing libm sequence.
template <class R> __device__ __forceinline__ void sincos_small(R x, R* s, R* c) {
    if constexpr (sizeof(R) == 8) {
        const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                     S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                     S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
        const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                     C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                     C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
        const double z = x * x, v = z * x;
        const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
        *s = x + v * (S1 + z * r);
        const double rc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
        const int ix = __double2hiint(x) & 0x7fffffff;
        // |x| >= 0.3: cos = (1 - qx) - ((z/2 - qx) - z r) with qx = x/4 rounded down to its high word
        const double qx = ix > 0x3fe90000 ? 0.28125 : __hiloint2double(ix - 0x00200000, 0);
        const double big = (1.0 - qx) - ((0.5 * z - qx) - (z * rc - 0.0));
        const double small = 1.0 - (0.5 * z - (z * rc - 0.0));
        *c = ix < 0x3FD33333 ? small : big;
    } else {
        sincosf(x, s, c);
    }
}

// x / c, correctly rounded, for a divisor whose reciprocal folds to a constant (or is loop-invariant):
// q = RN(x * RN(1/c)), the residual x - q c exactly by fma, and one fma correction give RN(x / c)
// (Markstein's correction step; 2.9e8 random operands over this file's divisors and random
// divisors reproduce IEEE division bit for bit, tools/div_check.c).  A zero or NaN residual means
// q is already exact (keeps -0) or x was infinite/NaN, and q is returned.  6 instructions instead
// of the 11-12 of the IEEE division sequence.
template <class R> __device__ __forceinline__ R divc(R x, R c) {
    const R rc = R(1) / c;
    const R q = x * rc;
    const R r = fma(-q, c, x);
    const R q2 = fma(r, rc, q);
    bool keep;
    if constexpr (sizeof(R) == 8) keep = __builtin_amdgcn_class(r, 1 | 2 | 32 | 64);   // NaN or +-0
    else keep = __builtin_amdgcn_classf(r, 1 | 2 | 32 | 64);
    return keep ? q : q2;
}

// d ** 3 of the predator term (flockUtils.py:343-348, np.power -> libm pow): the cube in double-word
// arithmetic rounded once, i.e. correctly rounded like pow (<= 0.52 ulp) up to double-rounding ties,
// in 8 instructions instead of pow's log/exp pair
template <class R> __device__ __forceinline__ R cube(R x) {
    const R h = x * x, l = fma(x, x, -h);   // x^2 = h + l exactly
    const R c = h * x, cl = fma(h, x, -c);  // h x = c + cl exactly
    return c + (cl + l * x);
}

template <class R> __device__ __forceinline__ R clip(R x, R lo, R hi) { return x < lo ? lo : (x > hi ? hi : x); }
template <class R> __device__ __forceinline__ R norm2(R x, R y) { return sqrt(x * x + y * y); }

// ---- pybullet.c quaternion conventions (x, y, z, w) ------------------------------------------
template <class R> __device__ __forceinline__ void quat_to_mat(const R q[4], R M[9]) {
    R x = q[0], y = q[1], z = q[2], w = q[3];
    R d = x * x + y * y + z * z + w * w, s = R(2.0) / d;
    R xs = x * s, ys = y * s, zs = z * s;
    R wx = w * xs, wy = w * ys, wz = w * zs, xx = x * xs, xy = x * ys, xz = x * zs;
    R yy = y * ys, yz = y * zs, zz = z * zs;
    M[0] = R(1.0) - (yy + zz); M[1] = xy - wz; M[2] = xz + wy;
    M[3] = xy + wz; M[4] = R(1.0) - (xx + zz); M[5] = yz - wx;
    M[6] = xz - wy; M[7] = yz + wx; M[8] = R(1.0) - (xx + yy);
}

// the third column of quat_to_mat(q) (the body z axis in the world frame), the same operations
template <class R> __device__ __forceinline__ void quat_to_zcol(const R q[4], R Z[3]) {
    R x = q[0], y = q[1], z = q[2], w = q[3];
    R d = x * x + y * y + z * z + w * w, s = R(2.0) / d;
    R xs = x * s, ys = y * s, zs = z * s;
    R wx = w * xs, wy = w * ys, xx = x * xs, xz = x * zs;
    R yy = y * ys, yz = y * zs;
    Z[0] = xz + wy; Z[1] = yz - wx; Z[2] = R(1.0) - (xx + yy);
}

template <class R> __device__ __forceinline__ void quat_to_euler(const R q[4], R rpy[3]) {
    R x = q[0], y = q[1], z = q[2], w = q[3];
    R sqx = x * x, sqy = y * y, sqz = z * z, squ = w * w;
    R sarg = R(-2.0) * (x * z - w * y);
    if (sarg <= R(-0.99999)) {
        rpy[0] = 0; rpy[1] = R(-0.5 * kPi); rpy[2] = R(2) * m_atan2(x, -y);
    } else if (sarg >= R(0.99999)) {
        rpy[0] = 0; rpy[1] = R(0.5 * kPi); rpy[2] = R(2) * m_atan2(-x, y);
    } else {
        rpy[0] = m_atan2(R(2) * (y * z + w * x), squ - sqx - sqy + sqz);
        rpy[1] = m_asin(sarg);
        rpy[2] = m_atan2(R(2) * (x * y + w * z), squ + sqx - sqy - sqz);
    }
}

// one angle of quat_to_euler (c = 0 roll, 1 pitch, 2 yaw), the same operations: the step's Euler pass spreads the
// three transcendentals of a drone over three lanes
template <class R> __device__ __forceinline__ R quat_to_euler_c(const R q[4], int c) {
    R x = q[0], y = q[1], z = q[2], w = q[3];
    R sqx = x * x, sqy = y * y, sqz = z * z, squ = w * w;
    R sarg = R(-2.0) * (x * z - w * y);
    const bool lo = sarg <= R(-0.99999), hi = !lo && sarg >= R(0.99999);
    if (c == 1) return lo ? R(-0.5 * kPi) : (hi ? R(0.5 * kPi) : m_asin(sarg));
    R ya, xa;
    if (lo) { ya = x; xa = -y; }
    else if (hi) { ya = -x; xa = y; }
    else if (c == 0) { ya = R(2) * (y * z + w * x); xa = squ - sqx - sqy + sqz; }
    else { ya = R(2) * (x * y + w * z); xa = squ + sqx - sqy - sqz; }
    const R r = m_atan2(ya, xa);
    return (lo || hi) ? (c == 0 ? R(0) : R(2) * r) : r;
}

// ---- DSLPIDControl.computeControl for a VEL target (DSLPIDControl.py:82-259,
//      BaseRLAviary.py:185-222).  pid[9] = last_rpy[3], integral_pos_e[3], integral_rpy_e[3].
// The torque mix and the motor speeds are f64 in either precision: the f32 mode's body rates come from the
// small differences of four ~14 k rpm (the torques of the attitude loop, a few hundred pwm on ~40 k), which
// f32 resolves to only ~1e-3 relative (tools/f32_emu.py); for R = double nothing changes.
template <class R>
__device__ __forceinline__ void pid_vel(const R pos[3], const R q[4], const R vel[3], const R Rm[9], const R rpy[3],
                                        const float act[4], R dt, R pid[9], double rpm[4], double* dbg = nullptr) {
    // _preprocessAction VEL branch: the float32 action row keeps the unit vector in float32;
    // SPEED_LIMIT * abs(a[3]) is float32 under NumPy >= 2 (DESIGN.md "Numerics").
    const double speed_limit = 0.3 * kMaxSpeedKmh * (1000.0 / 3600.0);
    float hx = act[0], hy = act[1];
    // plain sqrtf / '/' lower to the correctly rounded sequences (v_sqrt_f32 + fma refinement,
    // v_div_scale/fmas/fixup); __fsqrt_rn lowers to the bare 1-ulp v_sqrt_f32 on gfx950
    float hn = sqrtf(hx * hx + hy * hy);
    float ux = 0.0f, uy = 0.0f;
    if (hn != 0.0f) { ux = hx / hn; uy = hy / hn; }
    float sc = (float)speed_limit * fabsf(act[3]);
    const R tv[3] = {R((double)ux * (double)sc), R((double)uy * (double)sc), R(0.0 * (double)sc)};
    const R tp[3] = {pos[0], pos[1], R(kTargetAlt)};
    const R yaw = rpy[2];

    const R P_FOR[3] = {R(.4), R(.4), R(1.25)}, I_FOR[3] = {R(.05), R(.05), R(.05)}, D_FOR[3] = {R(.2), R(.2), R(.5)};
    R pe[3], ve[3], T[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        pe[i] = tp[i] - pos[i];
        ve[i] = tv[i] - vel[i];
        pid[3 + i] = clip(pid[3 + i] + pe[i] * dt, R(-2.), R(2.));
    }
    pid[5] = clip(pid[5], R(-0.15), R(.15));
#pragma unroll
    for (int i = 0; i < 3; ++i) T[i] = P_FOR[i] * pe[i] + I_FOR[i] * pid[3 + i] + D_FOR[i] * ve[i];
    T[2] += R(kG * kMass);
    R scalar = T[0] * Rm[2] + T[1] * Rm[5] + T[2] * Rm[8];
    if (!(scalar > R(0))) scalar = 0;
    R thrust = divc(sqrt(divc(scalar, R(4) * R(kKF))) - R(kPwmConst), R(kPwmScale));
    R tn = sqrt(T[0] * T[0] + T[1] * T[1] + T[2] * T[2]);
    R z[3] = {divc(T[0], tn), divc(T[1], tn), divc(T[2], tn)};
    R sy, cy;
    m_sincos(yaw, &sy, &cy);
    R xc[3] = {cy, sy, R(0)};
    R yt[3] = {z[1] * xc[2] - z[2] * xc[1], z[2] * xc[0] - z[0] * xc[2], z[0] * xc[1] - z[1] * xc[0]};
    R yn = sqrt(yt[0] * yt[0] + yt[1] * yt[1] + yt[2] * yt[2]);
    R y[3] = {divc(yt[0], yn), divc(yt[1], yn), divc(yt[2], yn)};
    R x[3] = {y[1] * z[2] - y[2] * z[1], y[2] * z[0] - y[0] * z[2], y[0] * z[1] - y[1] * z[0]};
    // target rotation columns x, y, z; rot_e from (Rt^T R - R^T Rt)
    const R Rt[9] = {x[0], y[0], z[0], x[1], y[1], z[1], x[2], y[2], z[2]};
    auto E = [&](int i, int j) {
        R a = 0, b = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) { a += Rt[k * 3 + i] * Rm[k * 3 + j]; b += Rm[k * 3 + i] * Rt[k * 3 + j]; }
        return a - b;
    };
    const R rot_e[3] = {E(2, 1), E(0, 2), E(1, 0)};
    const R P_TOR[3] = {R(70000.), R(70000.), R(60000.)}, I_TOR[3] = {R(.0), R(.0), R(500.)},
            D_TOR[3] = {R(20000.), R(20000.), R(12000.)};
    R rates_e[3];
    double tt[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        rates_e[i] = R(0.0) - divc(rpy[i] - pid[i], dt);
        pid[i] = rpy[i];
        pid[6 + i] = clip(pid[6 + i] - rot_e[i] * dt, R(-1500.), R(1500.));
    }
    pid[6] = clip(pid[6], R(-1.), R(1.));
    pid[7] = clip(pid[7], R(-1.), R(1.));
#pragma unroll
    for (int i = 0; i < 3; ++i)
        tt[i] = clip(-double(P_TOR[i]) * double(rot_e[i]) + double(D_TOR[i]) * double(rates_e[i]) +
                     double(I_TOR[i]) * double(pid[6 + i]), -3200.0, 3200.0);
    const double MIX[4][3] = {{-.5, -.5, -1}, {-.5, .5, 1}, {.5, .5, -1}, {.5, -.5, 1}};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        double pwm = double(thrust) + (MIX[k][0] * tt[0] + MIX[k][1] * tt[1] + MIX[k][2] * tt[2]);
        pwm = clip(pwm, kMinPwm, kMaxPwm);
        rpm[k] = kPwmScale * pwm + kPwmConst;
    }
    if (dbg) {
        dbg[0] = tv[0]; dbg[1] = tv[1]; dbg[2] = tv[2];
        dbg[3] = T[0]; dbg[4] = T[1]; dbg[5] = T[2];
        dbg[6] = rot_e[0]; dbg[7] = rot_e[1]; dbg[8] = rot_e[2];
        dbg[9] = thrust;
        dbg[10] = rpm[0]; dbg[11] = rpm[1]; dbg[12] = rpm[2]; dbg[13] = rpm[3];
        dbg[14] = (double)hn; dbg[15] = (double)sc;
    }
    (void)q;
}

// ---- _physics (BaseAviary.py:907-939) + one p.stepSimulation substep (448): btMultiBody model ----
struct NoExtraForces {
    template <class R> __device__ __forceinline__ void operator()(const R*, const R*, R*, R*) const {}
};
// `extra(M, Ml, F, Tw)` adds the physics-variant link forces (BaseAviary.py:424-445) after the motor
// model and before gravity, in the reference's applyExternalForce order.
// pacc (f32 mode): the position accumulates in f64 -- p + (v dt), f32 increment and f64 sum -- and p is its rounded copy
template <class R> __device__ __forceinline__ void pos_add(R p[3], double* pacc, int i, R d) {
    if (pacc) { pacc[i] = pacc[i] + (double)d; p[i] = R(pacc[i]); }
    else p[i] = p[i] + d;
}
// The prop torques (differences of four ~0.07 N forces), the world-frame angular acceleration and the
// angular-velocity update are f64 in either precision (W = double; see pid_vel): f32 there left 1e-4 relative
// errors on the body rates (tools/f32_emu.py: each of the three is needed; the damping and gyroscopic terms and
// the body-frame division are not).  For R = double this is the same arithmetic.
//
// ql != nullptr (ch_config.link_lag, the default): Bullet's cached link frame.  PyBullet's applyExternalForce /
// applyExternalTorque with LINK_FRAME on a multibody link rotate the link-frame vector by the link's cached world
// transform, which a link without a collision shape (the cf2x prop links and center_of_mass_link) gets only from the
// forward kinematics at the start of the previous stepSimulation: the base attitude one substep old (ql, carried in
// the state as drone components 22-25).  The force acts at the link's current centre of mass, so the lever arms turn
// with the current attitude.  Body frame, u = M^T ql_z: torque sum_i f_i (r_i x u) + u tz, force ql_z sum f.  Pinned
// by the real-PyBullet trace (oracle/ch_oracle.c drone_substep, the same operation order).
// extra(M, Ml, F, Tw): M the current attitude, Ml the cached link frame (== M without link_lag).
// torque_world acts only without the cached frame: under it the z torque (on link 4) turns with Ml like the forces;
// the trace rejects a world-frame z torque there (make_trace_inverse.py model lag_worldtz).
template <class R, class X = NoExtraForces>
__device__ __forceinline__ void drone_substep(R p[3], R q[4], R v[3], R w[3], const double rpm[4], R dt, R damping,
                                              bool torque_world, bool gyro, const X& extra = X(),
                                              double* pacc = nullptr, R* ql = nullptr, R* zl = nullptr,
                                              bool lag = false) {
    // (ql / zl are only dereferenced when lag: a conditional pointer to the caller's arrays would keep them out of
    // registers).  zl = the z axis of ql's frame (quat_to_zcol(ql) before the first substep; afterwards the previous
    // substep's M column, the same numbers), which is all the PYB wrench reads of it.
    using W = double;
    const R PX[4] = {R(0.028), R(-0.028), R(-0.028), R(0.028)}, PY[4] = {R(-0.028), R(-0.028), R(0.028), R(0.028)};
    R M[9], Ml[9];
    quat_to_mat(q, M);
    const bool body = std::is_same<X, NoExtraForces>::value && (torque_world || lag);
    if (lag && body) {
        Ml[2] = zl[0]; Ml[5] = zl[1]; Ml[8] = zl[2];
    } else if (lag) {
        quat_to_mat(ql, Ml);
    } else {
#pragma unroll
        for (int i = 0; i < 9; ++i) Ml[i] = M[i];
    }
    R F[3] = {0, 0, 0}, Tw[3] = {0, 0, 0}, tb[3];
    const W t0 = rpm[0] * rpm[0] * W(kKM), t1 = rpm[1] * rpm[1] * W(kKM), t2 = rpm[2] * rpm[2] * W(kKM),
            t3 = rpm[3] * rpm[3] * W(kKM);
    const W tz = (-t0 + t1 - t2 + t3);
    // PYB (no variant forces): the prop wrench in closed form in the body frame (the oracle's drone_substep, same
    // operation order).  Cached link frame: force ql_z sum f, torque above.  World-frame motor torque (rounds 1-4
    // model): torque (sum py f, -sum px f, 0) plus R^T e_z tz; force R e_z sum f.  Other cases accumulate per-link
    // world forces (variants add theirs).
    if (body && lag) {
        W f[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) f[i] = rpm[i] * rpm[i] * W(kKF);
        const W T = ((f[0] + f[1]) + f[2]) + f[3];
        F[0] = R(W(Ml[2]) * T); F[1] = R(W(Ml[5]) * T); F[2] = R(W(Ml[8]) * T);
        W u[3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
            u[i] = (W(M[0 + i]) * W(Ml[2]) + W(M[3 + i]) * W(Ml[5])) + W(M[6 + i]) * W(Ml[8]);
        const W sy = W(0.028) * (((-f[0] - f[1]) + f[2]) + f[3]);   // sum_i f_i r_iy
        const W sx = W(0.028) * (((-f[0] + f[1]) + f[2]) - f[3]);   // -sum_i f_i r_ix
        tb[0] = R(sy * u[2] + u[0] * tz);
        tb[1] = R(sx * u[2] + u[1] * tz);
        tb[2] = R((-sx * u[1] - sy * u[0]) + u[2] * tz);
    } else if (body) {
        W f[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) f[i] = rpm[i] * rpm[i] * W(kKF);
        const W T = ((f[0] + f[1]) + f[2]) + f[3];
        F[0] = R(W(M[2]) * T); F[1] = R(W(M[5]) * T); F[2] = R(W(M[8]) * T);
        tb[0] = R(W(0.028) * (((-f[0] - f[1]) + f[2]) + f[3]) + W(M[6]) * tz);
        tb[1] = R(W(0.028) * (((-f[0] + f[1]) + f[2]) - f[3]) + W(M[7]) * tz);
        tb[2] = R(W(M[8]) * tz);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            R f = R(rpm[i] * rpm[i] * W(kKF));
            R fw[3] = {Ml[2] * f, Ml[5] * f, Ml[8] * f};
            R rw[3] = {M[0] * PX[i] + M[1] * PY[i], M[3] * PX[i] + M[4] * PY[i], M[6] * PX[i] + M[7] * PY[i]};
            R t[3] = {rw[1] * fw[2] - rw[2] * fw[1], rw[2] * fw[0] - rw[0] * fw[2], rw[0] * fw[1] - rw[1] * fw[0]};
#pragma unroll
            for (int k = 0; k < 3; ++k) { F[k] += fw[k]; Tw[k] += t[k]; }
        }
        const R tzr = R(tz);
        if (torque_world && !lag) Tw[2] += tzr;
        else { Tw[0] += Ml[2] * tzr; Tw[1] += Ml[5] * tzr; Tw[2] += Ml[8] * tzr; }
        extra(M, Ml, F, Tw);
    }
    F[2] += R(-kMass * kG);
    const R k = damping;
    if (k != R(0)) {
        R sp = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
#pragma unroll
        for (int i = 0; i < 3; ++i) F[i] -= R(kMass) * v[i] * (k + k * sp);
    }
    R wb[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        wb[i] = M[0 + i] * w[0] + M[3 + i] * w[1] + M[6 + i] * w[2];
        if (!body) tb[i] = M[0 + i] * Tw[0] + M[3 + i] * Tw[1] + M[6 + i] * Tw[2];
    }
    const R J[3] = {R(kJx), R(kJy), R(kJz)};
    if (k != R(0)) {
        R sw = sqrt(wb[0] * wb[0] + wb[1] * wb[1] + wb[2] * wb[2]);
#pragma unroll
        for (int i = 0; i < 3; ++i) tb[i] -= J[i] * wb[i] * (k + k * sw);
    }
    if (gyro) {
        R Jw[3] = {J[0] * wb[0], J[1] * wb[1], J[2] * wb[2]};
        R g[3] = {wb[1] * Jw[2] - wb[2] * Jw[1], wb[2] * Jw[0] - wb[0] * Jw[2], wb[0] * Jw[1] - wb[1] * Jw[0]};
#pragma unroll
        for (int i = 0; i < 3; ++i) tb[i] -= g[i];
    }
    R ab[3] = {divc(tb[0], J[0]), divc(tb[1], J[1]), divc(tb[2], J[2])};
    const W ab0 = W(ab[0]), ab1 = W(ab[1]), ab2 = W(ab[2]), dtw = W(dt);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const W aw = W(M[i * 3 + 0]) * ab0 + W(M[i * 3 + 1]) * ab1 + W(M[i * 3 + 2]) * ab2;
        v[i] = v[i] + divc(F[i], R(kMass)) * dt;
        w[i] = R(W(w[i]) + aw * dtw);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) pos_add(p, pacc, i, v[i] * dt);
    if (lag) {   // the next substep's cached link frame: this substep's starting attitude
#pragma unroll
        for (int i = 0; i < 4; ++i) ql[i] = q[i];
        zl[0] = M[2]; zl[1] = M[5]; zl[2] = M[8];
    }
    // btMultiBody::stepPositionsMultiDof exponential-map quaternion update (base body)
    R fang = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    if (fang * dt > R(0.5 * (0.5 * kPi))) fang = R(0.5 * (0.5 * kPi)) / dt;
    // sin(0.5 fang dt) and cos(fang dt 0.5): the same double (a factor 0.5 commutes with rounding)
    R sh, ch;
    sincos_small(R(0.5) * fang * dt, &sh, &ch);   // 0 <= argument <= pi/8 after the clamp
    R s;
    if (fang < R(0.001)) s = R(0.5) * dt - (dt * dt * dt) * R(0.020833333333) * fang * fang;
    else s = sh / fang;
    R a[4] = {w[0] * s, w[1] * s, w[2] * s, ch};
    R o[4] = {a[3] * q[0] + a[0] * q[3] + a[1] * q[2] - a[2] * q[1],
              a[3] * q[1] + a[1] * q[3] + a[2] * q[0] - a[0] * q[2],
              a[3] * q[2] + a[2] * q[3] + a[0] * q[1] - a[1] * q[0],
              a[3] * q[3] - a[0] * q[0] - a[1] * q[1] - a[2] * q[2]};
    R n = sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2] + o[3] * o[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = divc(o[i], n);   // one reciprocal, four corrected quotients
}

// ---- physics variants (BaseAviary.py:420-450, 943-1118); cf2x.urdf:5 coefficients ----------------
constexpr double kGndCoeff = 11.36859, kPropRadius = 2.31348e-2, kArm = 0.0397;
constexpr double kDragXY = 9.1785e-7, kDragZ = 10.311e-7;
constexpr double kDw1 = 2267.18, kDw2 = .16, kDw3 = -.11;

// |roll| < pi/2 and |pitch| < pi/2 of getEulerFromQuaternion(q) (quat_to_euler), without its atan2/asin:
// off the gimbal-lock branches |asin(sarg)| < pi/2 always, and |atan2(Y, X)| < fl(pi/2) exactly when
// X > 0 unless |Y| / X is so large that atan2 rounds to fl(pi/2) (then atan2 decides, as it does for the
// X = +0, Y = 0 corner); NaN fails every test like the reference's comparison.
template <class R> __device__ __forceinline__ bool upright(const R q[4]) {
    const R x = q[0], y = q[1], z = q[2], w = q[3];
    const R sarg = R(-2.0) * (x * z - w * y);
    if (!(sarg > R(-0.99999) && sarg < R(0.99999))) return false;
    const R Y = R(2) * (y * z + w * x), X = w * w - x * x - y * y + z * z;
    if (X > R(0) && fabs(Y) <= X * R(1e12)) return true;
    if (!(X >= R(0))) return false;
    return fabs(m_atan2(Y, X)) < R(kPi / 2);
}

// _groundEffect (943-980): per-prop thrust boost below the clip height, skipped when tilted past 90 deg;
// each force is applied at its prop link (LINK_FRAME +z) so it also adds a torque about the COM.
template <class R>
__device__ __forceinline__ void ground_effect(const R p[3], const R q[4], const R M[9], const R rpm[4], R h_clip,
                                              R F[3], R Tw[3]) {
    const R PX[4] = {R(0.028), R(-0.028), R(-0.028), R(0.028)}, PY[4] = {R(-0.028), R(-0.028), R(0.028), R(0.028)};
    if (!upright(q)) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        R h = p[2] + (M[6] * PX[i] + M[7] * PY[i]);   // prop link COM height
        if (h < h_clip) h = h_clip;
        const R r = R(kPropRadius) / (R(4) * h);
        const R g = rpm[i] * rpm[i] * R(kKF) * R(kGndCoeff) * (r * r);
        const R fw[3] = {M[2] * g, M[5] * g, M[8] * g};
        const R rw[3] = {M[0] * PX[i] + M[1] * PY[i], M[3] * PX[i] + M[4] * PY[i], M[6] * PX[i] + M[7] * PY[i]};
        F[0] += fw[0]; F[1] += fw[1]; F[2] += fw[2];
        Tw[0] += rw[1] * fw[2] - rw[2] * fw[1];
        Tw[1] += rw[2] * fw[0] - rw[0] * fw[2];
        Tw[2] += rw[0] * fw[1] - rw[1] * fw[0];
    }
}

// _drag (982-1011): rotor drag from the previous substep's rpm (last_clipped_action), in the body
// frame, applied at the COM link
// (Mv: the frame the link-frame force is rotated by -- the cached link frame, or the current attitude once
// _groundEffect's getLinkStates has refreshed it)
template <class R>
__device__ __forceinline__ void rotor_drag(const R v[3], const R M[9], const R Mv[9], const R last_rpm[4], R F[3]) {
    R sum = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) sum += (R(2 * kPi) * last_rpm[i]) / R(60);
    const R dv[3] = {(R(-kDragXY) * sum) * v[0], (R(-kDragXY) * sum) * v[1], (R(-kDragZ) * sum) * v[2]};
    R b[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) b[k] = M[0 + k] * dv[0] + M[3 + k] * dv[1] + M[6 + k] * dv[2];
#pragma unroll
    for (int k = 0; k < 3; ++k) F[k] += Mv[3 * k + 0] * b[0] + Mv[3 * k + 1] * b[1] + Mv[3 * k + 2] * b[2];
}

// _downwash (1013-1041): one term per drone above (dz > 0) within 10 m horizontally; `o` is that
// drone's position at the start of the substep
template <class R>
__device__ __forceinline__ void downwash_term(const R me[3], const R o[3], const R M[9], R F[3]) {
    const R dz = o[2] - me[2];
    const R ex = o[0] - me[0], ey = o[1] - me[1];
    const R dxy = sqrt(ex * ex + ey * ey);
    if (dz > R(0) && dxy < R(10)) {
        const R r = R(kPropRadius) / (R(4) * dz);
        const R alpha = R(kDw1) * (r * r);
        const R beta = R(kDw2) * dz + R(kDw3);
        const R u = dxy / beta;
        const R fz = -alpha * m_exp(R(-.5) * (u * u));
        F[0] += M[2] * fz; F[1] += M[5] * fz; F[2] += M[8] * fz;
    }
}

// Physics.DYN: _dynamics (1043-1102) + _integrateQ (1104-1118).  Explicit Euler on the body rates rr
// (persistent rpy_rates); the stored angular velocity is rotation(old quat) @ rr.
template <class R>
__device__ __forceinline__ void dyn_substep(R p[3], R q[4], R v[3], R w[3], R rr[3], const R rpm[4], R dt,
                                            double* pacc = nullptr) {
    R M[9];
    quat_to_mat(q, M);
    R f[4], z[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { f[i] = rpm[i] * rpm[i] * R(kKF); z[i] = rpm[i] * rpm[i] * R(kKM); }
    const R T = f[0] + f[1] + f[2] + f[3];
    const R fw[3] = {M[2] * T, M[5] * T, M[8] * T - R(kG * kMass)};
    const R zt = -z[0] + z[1] - z[2] + z[3];
    const R ls = R(kArm) / sqrt(R(2));
    const R xt = (f[0] + f[1] - f[2] - f[3]) * ls, yt = (-f[0] + f[1] + f[2] - f[3]) * ls;
    const R J[3] = {R(kJx), R(kJy), R(kJz)};
    const R Jr[3] = {J[0] * rr[0], J[1] * rr[1], J[2] * rr[2]};
    const R c[3] = {rr[1] * Jr[2] - rr[2] * Jr[1], rr[2] * Jr[0] - rr[0] * Jr[2], rr[0] * Jr[1] - rr[1] * Jr[0]};
    const R tq[3] = {xt - c[0], yt - c[1], zt - c[2]};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        v[i] = v[i] + dt * (fw[i] / R(kMass));
        rr[i] = rr[i] + dt * ((R(1) / J[i]) * tq[i]);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) pos_add(p, pacc, i, dt * v[i]);
    const R on = sqrt(rr[0] * rr[0] + rr[1] * rr[1] + rr[2] * rr[2]);
    if (!(fabs(on) <= R(1e-8))) {   // np.isclose(omega_norm, 0): atol 1e-8
        R si, co;
        m_sincos(on * dt / R(2), &si, &co);
        const R k = R(2) / on;
        const R P = rr[0], Q = rr[1], Z = rr[2];
        const R L[4][4] = {{0, Z, -Q, P}, {-Z, 0, P, Q}, {Q, -P, 0, Z}, {-P, -Q, -Z, 0}};
        R o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            R m[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) m[j] = (i == j ? co : R(0)) + (k * (L[i][j] * R(.5))) * si;
            o[i] = m[0] * q[0] + m[1] * q[1] + m[2] * q[2] + m[3] * q[3];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) q[i] = o[i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) w[i] = M[3 * i + 0] * rr[0] + M[3 * i + 1] * rr[1] + M[3 * i + 2] * rr[2];
}

// RK4 option (CH_PHYS_DYN_RK4; north_star, not a reference path): the DYN equations of motion
// (_dynamics, BaseAviary.py:1043-1102; _integrateQ's L, 1104-1118) as an ODE in (p, v, q, w_b), classic
// four-stage Runge-Kutta over one substep at constant rpm, q renormalised, world rates R(q_new) w_b.
// Same operations in the same order as the oracle's rk4_substep (ch_oracle.c).
template <class R>
__device__ __forceinline__ void dyn_deriv(const R q[4], const R v[3], const R rr[3], const R rpm[4], R dp[3], R dv[3],
                                          R dq[4], R drr[3]) {
    R M[9];
    quat_to_mat(q, M);
    R f[4], z[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { f[i] = rpm[i] * rpm[i] * R(kKF); z[i] = rpm[i] * rpm[i] * R(kKM); }
    const R T = f[0] + f[1] + f[2] + f[3];
    const R fw[3] = {M[2] * T, M[5] * T, M[8] * T - R(kG * kMass)};
    const R zt = -z[0] + z[1] - z[2] + z[3];
    const R ls = R(kArm) / sqrt(R(2));
    const R xt = (f[0] + f[1] - f[2] - f[3]) * ls, yt = (-f[0] + f[1] + f[2] - f[3]) * ls;
    const R J[3] = {R(kJx), R(kJy), R(kJz)};
    const R Jr[3] = {J[0] * rr[0], J[1] * rr[1], J[2] * rr[2]};
    const R c[3] = {rr[1] * Jr[2] - rr[2] * Jr[1], rr[2] * Jr[0] - rr[0] * Jr[2], rr[0] * Jr[1] - rr[1] * Jr[0]};
    const R tq[3] = {xt - c[0], yt - c[1], zt - c[2]};
#pragma unroll
    for (int i = 0; i < 3; ++i) { dp[i] = v[i]; dv[i] = fw[i] / R(kMass); drr[i] = (R(1) / J[i]) * tq[i]; }
    const R P = rr[0], Q = rr[1], Z = rr[2];
    const R L[4][4] = {{0, Z, -Q, P}, {-Z, 0, P, Q}, {Q, -P, 0, Z}, {-P, -Q, -Z, 0}};
#pragma unroll
    for (int i = 0; i < 4; ++i) dq[i] = R(0.5) * (L[i][0] * q[0] + L[i][1] * q[1] + L[i][2] * q[2] + L[i][3] * q[3]);
}
template <class R>
__device__ __forceinline__ void rk4_substep(R p[3], R q[4], R v[3], R w[3], R rr[3], const R rpm[4], R dt,
                                            double* pacc = nullptr) {
    R kp[4][3], kv[4][3], kq[4][4], kr[4][3];
    const R a[4] = {R(0), R(0.5) * dt, R(0.5) * dt, dt};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        R yv[3], yq[4], yr[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            yv[i] = s ? v[i] + a[s] * kv[s - 1][i] : v[i];
            yr[i] = s ? rr[i] + a[s] * kr[s - 1][i] : rr[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) yq[i] = s ? q[i] + a[s] * kq[s - 1][i] : q[i];
        dyn_deriv(yq, yv, yr, rpm, kp[s], kv[s], kq[s], kr[s]);
    }
    const R h6 = dt / R(6.0);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        pos_add(p, pacc, i, h6 * (((kp[0][i] + R(2) * kp[1][i]) + R(2) * kp[2][i]) + kp[3][i]));
        v[i] = v[i] + h6 * (((kv[0][i] + R(2) * kv[1][i]) + R(2) * kv[2][i]) + kv[3][i]);
        rr[i] = rr[i] + h6 * (((kr[0][i] + R(2) * kr[1][i]) + R(2) * kr[2][i]) + kr[3][i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = q[i] + h6 * (((kq[0][i] + R(2) * kq[1][i]) + R(2) * kq[2][i]) + kq[3][i]);
    const R qn = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = q[i] / qn;
    R M[9];
    quat_to_mat(q, M);
#pragma unroll
    for (int i = 0; i < 3; ++i) w[i] = M[3 * i + 0] * rr[0] + M[3 * i + 1] * rr[1] + M[3 * i + 2] * rr[2];
}

// Physics variants (BaseAviary.py:420-450) for the drone on this lane, all substeps of one control
// step.  `base` is the lane of the env's drone 0, `nsh` a wave-uniform bound (>= n) on its drones and
// n its live drones; lr / rr carry last_clipped_action and the DYN body rates in and out.  The
// downwash term reads the other drones' substep-start positions by cross-lane shuffle: the loop bound
// is wave-uniform, so every lane of the branch joins each shuffle.
template <class R>
__device__ __forceinline__ void variant_substeps(const StepParams<R>& p, int base, int nsh, int n, R pos[3], R q[4],
                                                 R v[3], R w[3], const double rpm_w[4], R lr[4], R rr[3],
                                                 double* pacc = nullptr, R* ql = nullptr, R* zl = nullptr,
                                                 bool lag = false) {
    // the variants' terms in the state precision; the PYB wrench takes the f64 speeds (drone_substep)
    const R rpm[4] = {R(rpm_w[0]), R(rpm_w[1]), R(rpm_w[2]), R(rpm_w[3])};
    const int ph = p.physics;
    const bool gnd = ph == CH_PHYS_PYB_GND || ph == CH_PHYS_PYB_GND_DRAG_DW;
    const bool drag = ph == CH_PHYS_PYB_DRAG || ph == CH_PHYS_PYB_GND_DRAG_DW;
    const bool dw = ph == CH_PHYS_PYB_DW || ph == CH_PHYS_PYB_GND_DRAG_DW;
    const R h_clip = R(p.gnd_h_clip);
    for (int s = 0; s < p.substeps; ++s) {
        if (ph == CH_PHYS_DYN) {
            dyn_substep(pos, q, v, w, rr, rpm, R(p.dt), pacc);
        } else if (ph == CH_PHYS_DYN_RK4) {
            rk4_substep(pos, q, v, w, rr, rpm, R(p.dt), pacc);
        } else {
            // extra() runs before drone_substep moves the body: pos/q/v are the substep-start state.  _groundEffect
            // reads p.getLinkStates(computeForwardKinematics=1) (BaseAviary.py:958-963), which refreshes the cached
            // link transforms: its forces and the drag / downwash applied after it rotate by the current attitude M;
            // without it drag and downwash use the cached frame Ml (== M without link_lag)
            auto extra = [&](const R* M, const R* Ml, R* F, R* Tw) {
                const R* Mv = gnd ? M : Ml;
                if (gnd) ground_effect(pos, q, M, rpm, h_clip, F, Tw);
                if (drag) rotor_drag(v, M, Mv, lr, F);
                if (dw) {
                    for (int i = 0; i < nsh; ++i) {
                        const R o[3] = {__shfl(pos[0], base + i, 64), __shfl(pos[1], base + i, 64),
                                        __shfl(pos[2], base + i, 64)};
                        if (i < n) downwash_term(pos, o, Mv, F);
                    }
                }
            };
            drone_substep(pos, q, v, w, rpm_w, R(p.dt), R(p.damping), p.torque_world != 0, p.gyro != 0, extra, pacc,
                          ql, zl, lag);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) lr[c] = rpm[c];   // last_clipped_action (BaseAviary.py:450)
    }
}

// ---- flocking: MathematicalFlock (flockUtils.py:11-382) ----------------------------------------
constexpr double kEps = 0.1, kH = 0.2;
template <class R> __device__ __forceinline__ R sigma_norm_n(R n) { return divc(sqrt(R(1) + R(kEps) * (n * n)) - R(1), R(kEps)); }
// cos(x) for 0 <= x <= pi (the bump's argument): x = n pi/2 + r with n = round(x / (pi/2)) in {0, 1, 2} and
// |r| <= pi/4 (Cody-Waite: pi/2 in four parts, each product exact), then the fdlibm kernels
// (sincos_small): cos r, -sin r, -cos r.  <= 1 ulp like libm (tools/sincos_check.c), without the generic
// reduction of the libm entry point.
template <class R> __device__ __forceinline__ R cos_0pi(R x) {
    if constexpr (sizeof(R) == 8) {
        const double PIO2_1 = 1.57079632673412561417e+00, PIO2_2 = 6.07710050630396597660e-11,
                     PIO2_3 = 2.02226624871116645580e-21,
                     PIO2_3T = 8.47842766036889956997e-32;   // fdlibm pio2_1, pio2_2, pio2_3, pio2_3t
        const double n = rint(x * 6.36619772367581382433e-01);
        const double r = (((x - n * PIO2_1) - n * PIO2_2) - n * PIO2_3) - n * PIO2_3T;
        double s, c;
        sincos_small(fabs(r), &s, &c);
        s = r < 0 ? -s : s;
        return n == 0.0 ? c : (n == 1.0 ? -s : -c);
    } else {
        return cosf(x);
    }
}
// sin and cos of -pi <= x <= pi (a reset's cattle velocity angle, BaseAviary.py:631-632): the same
// reduction by pi/2 (quadrant n in -2..2) and fdlibm kernels; <= 1 ulp (tools/sincos_check.c)
__device__ __forceinline__ void sincos_pi(double x, double* s, double* c) {
    const double PIO2_1 = 1.57079632673412561417e+00, PIO2_2 = 6.07710050630396597660e-11,
                 PIO2_3 = 2.02226624871116645580e-21, PIO2_3T = 8.47842766036889956997e-32;
    const double n = rint(x * 6.36619772367581382433e-01);
    const double r = (((x - n * PIO2_1) - n * PIO2_2) - n * PIO2_3) - n * PIO2_3T;
    double sr, cr;
    sincos_small(fabs(r), &sr, &cr);
    sr = r < 0 ? -sr : sr;
    const int q = (int)n & 3;
    *s = q == 0 ? sr : (q == 1 ? cr : (q == 2 ? -sr : -cr));
    *c = q == 0 ? cr : (q == 1 ? -sr : (q == 2 ? -cr : sr));
}
template <class R> __device__ __forceinline__ R bump(R z) {
    if (z < R(0)) return R(0);
    if (z < R(kH)) return R(1);
#ifdef CH_OCML_COS
    if (z <= R(1)) return (R(1) + m_cos(divc(R(kPi) * (z - R(kH)), R(1) - R(kH)))) / R(2);
#else
    if (z <= R(1)) return (R(1) + cos_0pi(divc(R(kPi) * (z - R(kH)), R(1) - R(kH)))) / R(2);
#endif
    return R(0);
}
template <class R> __device__ __forceinline__ R sigma_1(R z) { return z / sqrt(R(1) + z * z); }

// gradient (phi_alpha * n_ij) and velocity-consensus (a_ij * (pj - pi)) contributions of one
// neighbour (flockUtils.py:327-337, 41-49, 365-374); ra = sigma_norm(r), da = sigma_norm(d)
template <class R>
__device__ __forceinline__ void pair_terms(R qix, R qiy, R pix, R piy, R qjx, R qjy, R pjx, R pjy, R ra, R da,
                                           R& gx, R& gy, R& cx, R& cy) {
    R zx = qjx - qix, zy = qjy - qiy;
    R n = sqrt(zx * zx + zy * zy);
    R den = sqrt(R(1) + R(kEps) * (n * n));
    R sn = divc(den - R(1), R(kEps));
    R b = bump(divc(sn, ra));
    R zz = sn - da;
    R ph = b * ((R(5.0 + 5.0) * sigma_1(zz + R(0.0)) + R(5.0 - 5.0)) / R(2));
    gx += ph * (zx / den);
    gy += ph * (zy / den);
    cx += b * (pjx - pix);
    cy += b * (pjy - piy);
}

// same as pair_terms with the neighbour offset z = qj - qi and its norm already at hand; returns the bump
template <class R>
__device__ __forceinline__ R pair_terms_n(R n, R zx, R zy, R pix, R piy, R pjx, R pjy, R ra, R da, R& gx, R& gy,
                                          R& cx, R& cy) {
    R den = sqrt(R(1) + R(kEps) * (n * n));
    R sn = divc(den - R(1), R(kEps));
    R b = bump(divc(sn, ra));
    R zz = sn - da;
    R ph = b * ((R(5.0 + 5.0) * sigma_1(zz + R(0.0)) + R(5.0 - 5.0)) / R(2));
    gx += ph * (zx / den);
    gy += ph * (zy / den);
    cx += b * (pjx - pix);
    cy += b * (pjy - piy);
    return b;
}

// ---- spacing rewards: CattleAviary.py:572-679 -------------------------------------------------
// (both spacing terms branch-free: each candidate is evaluated and one selected, the same operations as the
// reference's if-chain -- the drone lanes of a wave take different branches, so a branchy form ran every branch
// anyway, plus the exec-mask bookkeeping)
template <class R> __device__ __forceinline__ R simple_spacing(R r, const Level& L) {
    R desired = R(L.desired), tol = desired * R(L.tol);
    R lb = desired - tol, ub = desired + tol;
    const R below = R(-1) + (r / lb) * R(2);
    const R above = R(1) - ((r - ub) / (R(7.0) - ub)) * R(2);
    return (lb <= r && r <= ub) ? R(1.0) : (r < lb ? below : (r > ub ? above : R(-1.0)));
}
template <class R> __device__ __forceinline__ R complex_spacing(R r, const Level& L) {
    R ds = R(L.desired);
    R t = divc(r - ds, R(0.4 + 1e-9));
    R gauss = m_exp(R(-0.5) * (t * t));
    const R coll_v = R(-1.0) * (R(1.0) - divc(r, R(0.3 + 1e-9)));
    const R pull_v = divc(R(-0.3) * (r - R(1.5)), R(5.0 - 1.5));
    R coll = r < R(0.3) ? coll_v : R(0.0);
    R pull = r > R(1.5) ? pull_v : R(0.0);
    R rew = gauss + coll + pull;
    rew += R(0.1) * (R(1) - fabs(r - ds));
    return rew;
}
// cc = the continuation constant fr0 / exp(-lambda r0) of the r > r0 branch, evaluated once on the host
// (ch_api.cpp: cattle_spacing_cc) with the same expression the reference evaluates per call
template <class R> __device__ __forceinline__ R cattle_spacing(R r, R cc) {
    const double A = 1.2, B = 2.1, C = 3.3, K = 0.2, D = -1, R0 = 1.3, LAM = 0.8;
    if (r <= R(R0))
        return R(A) * m_exp(divc(-((r - R(D)) * (r - R(D))), R(2 * (C * C)))) - R(B) * m_exp(divc(-(r * r), R(2 * (K * K))));
    return cc * m_exp(R(-LAM) * r);
}

// ---- Philox4x32-10 (Random123) ------------------------------------------------------------------
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t lo0 = 0xD2511F53u * c[0], hi0 = __umulhi(0xD2511F53u, c[0]);
        uint32_t lo1 = 0xCD9E8D57u * c[2], hi1 = __umulhi(0xCD9E8D57u, c[2]);
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}
__device__ __forceinline__ double philox_uniform53(uint32_t k0, uint32_t k1, uint64_t episode, uint32_t j, uint32_t env) {
    uint32_t c[4] = {(uint32_t)episode, (uint32_t)(episode >> 32), j | (1u << 16), env};
    philox(c, k0, k1);
    return ((double)(c[0] >> 5) * 67108864.0 + (double)(c[1] >> 6)) * (1.0 / 9007199254740992.0);
}

}  // namespace ch
