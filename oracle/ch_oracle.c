/*
 * ch_oracle.c — scalar fp64 CPU restatement of the reference's env.step() hot path.
 *
 * TEST INFRASTRUCTURE ONLY (the checker and the CPU baseline).  The product path is the HIP code in
 * rl-cattle-herding_amd/csrc; it never links, loads or calls this file.
 *
 * Every function cites the reference lines it restates (paths relative to
 * /root/reference/gym_pybullet_drones).  Sums are taken sequentially in index order, as numpy does
 * for the axis-0 reductions and Python loops the reference uses; results match the golden vectors
 * to ~1e-12 relative (numpy's pairwise inner sums and scipy's Euler round trip differ in the last
 * bits only).
 */
#include "ch_oracle.h"

#include <math.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------------------------------------
 * Constants: assets/cf2x.urdf:5-12, BaseAviary.py:97-173, DSLPIDControl.py:37-53,
 * BaseRLAviary.py:101-102, CattleAviary.py:91-105, flockUtils.py:13-74, BaseAviary.py:51-55,579
 * ------------------------------------------------------------------------------------------- */
static const double G = 9.8, MASS = 0.027, KF = 3.16e-10, KM = 7.94e-12;
static const double JX = 1.4e-5, JY = 1.4e-5, JZ = 2.17e-5;
static const double PROP[4][2] = {{0.028, -0.028}, {-0.028, -0.028}, {-0.028, 0.028}, {0.028, 0.028}};
static const double TARGET_ALT = 0.45;
static const double P_FOR[3] = {.4, .4, 1.25}, I_FOR[3] = {.05, .05, .05}, D_FOR[3] = {.2, .2, .5};
static const double P_TOR[3] = {70000., 70000., 60000.}, I_TOR[3] = {.0, .0, 500.}, D_TOR[3] = {20000., 20000., 12000.};
static const double PWM2RPM_SCALE = 0.2685, PWM2RPM_CONST = 4070.3, MIN_PWM = 20000, MAX_PWM = 65535;
static const double MIXER[4][3] = {{-.5, -.5, -1}, {-.5, .5, 1}, {.5, .5, -1}, {.5, -.5, 1}};
static const double MAX_SPEED_KMH = 30.0;
static const double MISSION_BOUNDARY = 15, MAX_FORMATION_DISTANCE = 8, COLLISION_THRESHOLD = 0.2;
static const double SP_A = 1.2, SP_B = 2.1, SP_C = 3.3, SP_K = 0.2, SP_D = -1, SP_R0 = 1.3, SP_LAM = 0.8;
static const double MAX_VEL_CATTLE = 0.2;

/* curriculum_learning.py:10-194 — per level */
typedef struct {
    double desired, tol, hold, approach_min, min_eff, cattle_desired, cattle_tol;
    int min_drones, max_drones; double episode_len;
    double w_simple, w_complex, w_survival, w_approach, w_eff, w_cattle;
    int required_tally;
} level_t;
static const level_t LEVELS[8] = {
    {0.8, 0.3, 10, 0.0, 0, 0.0, 0.0, 3, 3, 40, 1, 0, 0, 0, 0, 0.0, 100},
    {0.8, 0.2, 25, 0.0, 0, 0.0, 0.0, 4, 4, 40, 0, 1, -0.5, 0, 0, 0.0, 300},
    {0.8, 0.2, 15, 0.6, 0, 0.0, 0.0, 4, 4, 40, 0, 0.8, 0, 1, 0, 0.0, 100},
    {0.8, 0.2, 15, 0.3, 0, 0.0, 0.0, 4, 4, 40, 0, 0.8, -0.5, 1, 0, 0.0, 400},
    {0.8, 0.2, 15, 0.3, 20, 0.0, 0.0, 4, 4, 80, 0, 0.7, -0.0, 0.8, 1, 0.0, 600},
    {0.8, 0.2, 15, 0.3, 50, 0.8, 0.1, 4, 4, 40, 0, 0.7, -0.5, 0.6, 1, 0.8, 600},
    {0.8, 0.3, 15, 0.2, 50, 0.0, 0.0, 4, 12, 80, 0.7, 0.0, -0.0, 0.8, 1, 0.0, 600},
    {0.8, 0.3, 15, 0.2, 50, 0.0, 0.0, 4, 12, 80, 0.0, 0.0, -0.0, 1, 1, 0.0, 600},
};

static double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* ---------------------------------------------------------------------------------------------
 * pybullet.c quaternion conventions (x, y, z, w) — used at BaseAviary.py:618,714,
 * DSLPIDControl.py:144,187,240-241 (third-party; restated, parity unpinned)
 * ------------------------------------------------------------------------------------------- */
void och_euler_from_quat(const double* q, double* rpy) {
    double x = q[0], y = q[1], z = q[2], w = q[3];
    double sqx = x * x, sqy = y * y, sqz = z * z, squ = w * w;
    double sarg = -2.0 * (x * z - w * y);
    if (sarg <= -0.99999) { rpy[0] = 0; rpy[1] = -0.5 * M_PI; rpy[2] = 2 * atan2(x, -y); }
    else if (sarg >= 0.99999) { rpy[0] = 0; rpy[1] = 0.5 * M_PI; rpy[2] = 2 * atan2(-x, y); }
    else {
        rpy[0] = atan2(2 * (y * z + w * x), squ - sqx - sqy + sqz);
        rpy[1] = asin(sarg);
        rpy[2] = atan2(2 * (x * y + w * z), squ + sqx - sqy - sqz);
    }
}

void och_matrix_from_quat(const double* q, double* R) {
    double x = q[0], y = q[1], z = q[2], w = q[3];
    double d = x * x + y * y + z * z + w * w, s = 2.0 / d;
    double xs = x * s, ys = y * s, zs = z * s;
    double wx = w * xs, wy = w * ys, wz = w * zs, xx = x * xs, xy = x * ys, xz = x * zs;
    double yy = y * ys, yz = y * zs, zz = z * zs;
    R[0] = 1.0 - (yy + zz); R[1] = xy - wz; R[2] = xz + wy;
    R[3] = xy + wz; R[4] = 1.0 - (xx + zz); R[5] = yz - wx;
    R[6] = xz - wy; R[7] = yz + wx; R[8] = 1.0 - (xx + yy);
}

static double norm2(double x, double y) { return sqrt(x * x + y * y); }
static double norm3(const double* v) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
static void cross3(const double* a, const double* b, double* c) {
    c[0] = a[1] * b[2] - a[2] * b[1]; c[1] = a[2] * b[0] - a[0] * b[2]; c[2] = a[0] * b[1] - a[1] * b[0];
}

/* ---------------------------------------------------------------------------------------------
 * DSLPIDControl.computeControl (DSLPIDControl.py:82-145) with _dslPIDPositionControl (149-208) and
 * _dslPIDAttitudeControl (212-259).  The scipy from_matrix→as_euler('XYZ')→from_euler→as_matrix
 * round trip (205, 242-244) is the identity on the orthonormal target frame and is elided.
 * ------------------------------------------------------------------------------------------- */
void och_pid_vel(const double* pos, const double* quat, const double* vel, const double* target_pos,
                 const double* target_rpy, const double* target_vel, double dt,
                 double* last_rpy, double* int_pos, double* int_rpy, double* rpm) {
    const double gravity = G * MASS;  /* BaseControl.py:35 */
    double R[9]; och_matrix_from_quat(quat, R);
    double pos_e[3], vel_e[3], T[3];
    for (int i = 0; i < 3; ++i) {
        pos_e[i] = target_pos[i] - pos[i];
        vel_e[i] = target_vel[i] - vel[i];
        int_pos[i] = clipd(int_pos[i] + pos_e[i] * dt, -2., 2.);
    }
    int_pos[2] = clipd(int_pos[2], -0.15, .15);
    for (int i = 0; i < 3; ++i) T[i] = P_FOR[i] * pos_e[i] + I_FOR[i] * int_pos[i] + D_FOR[i] * vel_e[i];
    T[2] += gravity;
    double scalar = T[0] * R[2] + T[1] * R[5] + T[2] * R[8];
    if (!(scalar > 0.)) scalar = 0.;  /* Python max(0., x): 0. for x <= 0 and for NaN */
    double thrust = (sqrt(scalar / (4 * KF)) - PWM2RPM_CONST) / PWM2RPM_SCALE;
    double tn = norm3(T), zax[3] = {T[0] / tn, T[1] / tn, T[2] / tn};
    double xc[3] = {cos(target_rpy[2]), sin(target_rpy[2]), 0};
    double yt[3]; cross3(zax, xc, yt);
    double yn = norm3(yt), yax[3] = {yt[0] / yn, yt[1] / yn, yt[2] / yn};
    double xax[3]; cross3(yax, zax, xax);
    /* target rotation columns = x, y, z axes */
    double Rt[9] = {xax[0], yax[0], zax[0], xax[1], yax[1], zax[1], xax[2], yax[2], zax[2]};
    double rpy[3]; och_euler_from_quat(quat, rpy);
    /* rot_matrix_e = Rt^T R - R^T Rt */
    double E[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double a = 0, b = 0;
            for (int k = 0; k < 3; ++k) { a += Rt[k * 3 + i] * R[k * 3 + j]; b += R[k * 3 + i] * Rt[k * 3 + j]; }
            E[i * 3 + j] = a - b;
        }
    double rot_e[3] = {E[7], E[2], E[3]};
    double rates_e[3], tt[3];
    for (int i = 0; i < 3; ++i) {
        rates_e[i] = 0.0 - (rpy[i] - last_rpy[i]) / dt;
        last_rpy[i] = rpy[i];
        int_rpy[i] = clipd(int_rpy[i] - rot_e[i] * dt, -1500., 1500.);
    }
    int_rpy[0] = clipd(int_rpy[0], -1., 1.);
    int_rpy[1] = clipd(int_rpy[1], -1., 1.);
    for (int i = 0; i < 3; ++i)
        tt[i] = clipd(-P_TOR[i] * rot_e[i] + D_TOR[i] * rates_e[i] + I_TOR[i] * int_rpy[i], -3200, 3200);
    for (int k = 0; k < 4; ++k) {
        double pwm = thrust + (MIXER[k][0] * tt[0] + MIXER[k][1] * tt[1] + MIXER[k][2] * tt[2]);
        pwm = clipd(pwm, MIN_PWM, MAX_PWM);
        rpm[k] = PWM2RPM_SCALE * pwm + PWM2RPM_CONST;
    }
}

/* ---------------------------------------------------------------------------------------------
 * Physics substep: _physics (BaseAviary.py:907-939) + p.stepSimulation (448).  Model of btMultiBody
 * (parity unpinned): link forces at prop offsets, z torque on link 4, gravity, default damping
 * -m v (k + k|v|) and -I w (k + k|w|), gyroscopic term, semi-implicit Euler, exponential-map
 * quaternion update.  Cattle: constant-velocity xy (pinned by evaluation_data.pkl).
 * ------------------------------------------------------------------------------------------- */
static void quat_mul(const double* a, const double* b, double* o) {
    o[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    o[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    o[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    o[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
}

/* ---------------------------------------------------------------------------------------------
 * Physics variants (BaseAviary.py:420-450): extra link forces applied after _physics, in the
 * reference's call order (ground effect, drag, downwash), each rotated from LINK_FRAME to world on
 * its own like p.applyExternalForce does; DYN replaces _physics + stepSimulation by the explicit
 * model _dynamics (1043-1102) + _integrateQ (1104-1118).  cf2x.urdf:5 coefficients.
 * ------------------------------------------------------------------------------------------- */
static const double GND_EFF_COEFF = 11.36859, PROP_RADIUS = 2.31348e-2, ARM = 0.0397;
static const double DRAG_XY = 9.1785e-7, DRAG_Z = 10.311e-7;
static const double DW_C1 = 2267.18, DW_C2 = .16, DW_C3 = -.11;
static const double THRUST2WEIGHT = 2.25;

enum { PH_PYB = 0, PH_DYN = 1, PH_GND = 2, PH_DRAG = 3, PH_DW = 4, PH_ALL = 5, PH_DYN_RK4 = 6 };
static int ph_gnd(int ph) { return ph == PH_GND || ph == PH_ALL; }
static int ph_drag(int ph) { return ph == PH_DRAG || ph == PH_ALL; }
static int ph_dw(int ph) { return ph == PH_DW || ph == PH_ALL; }

/* GND_EFF_H_CLIP (BaseAviary.py:163-173): 0.25 r_prop sqrt(15 MAX_RPM^2 KF c_gnd / MAX_THRUST) */
double och_gnd_eff_h_clip(void) {
    const double gravity = G * MASS;
    const double max_rpm = sqrt((THRUST2WEIGHT * gravity) / (4 * KF));
    const double max_thrust = (4 * KF * (max_rpm * max_rpm));
    return 0.25 * PROP_RADIUS * sqrt((15 * (max_rpm * max_rpm) * KF * GND_EFF_COEFF) / max_thrust);
}

typedef struct phys_ctx {
    int physics;
    const double* last_rpm;        /* [4] last_clipped_action of this drone */
    const double (*pos)[3];        /* all drones' positions at the start of the substep */
    int n, self;
    double h_clip;
} phys_ctx;

/* R: the current attitude (lever arms, heights, the drag's body frame); Rl: the cached link frame that turns the
 * link-frame forces into world forces (== R without link_lag).  _groundEffect reads p.getLinkStates with
 * computeForwardKinematics=1 (943-980), which refreshes the cached link transforms: its forces, and the drag and
 * downwash applied after it (PYB_GND_DRAG_DW), rotate by the current attitude; alone, drag and downwash use Rl. */
static void physics_forces(const phys_ctx* x, const double* p, const double* q, const double* v, const double* R,
                           const double* Rl, const double* rpm, double* F, double* Tw) {
    if (ph_gnd(x->physics)) {   /* _groundEffect (943-980) */
        double rpy[3]; och_euler_from_quat(q, rpy);
        double g[4];
        for (int i = 0; i < 4; ++i) {
            double h = p[2] + (R[6] * PROP[i][0] + R[7] * PROP[i][1] + R[8] * 0.0);   /* prop link COM z */
            if (h < x->h_clip) h = x->h_clip;
            double r = PROP_RADIUS / (4 * h);
            g[i] = rpm[i] * rpm[i] * KF * GND_EFF_COEFF * (r * r);
        }
        if (fabs(rpy[0]) < M_PI / 2 && fabs(rpy[1]) < M_PI / 2) {
            for (int i = 0; i < 4; ++i) {
                double fw[3] = {R[2] * g[i], R[5] * g[i], R[8] * g[i]};
                double rw[3] = {R[0] * PROP[i][0] + R[1] * PROP[i][1], R[3] * PROP[i][0] + R[4] * PROP[i][1],
                                R[6] * PROP[i][0] + R[7] * PROP[i][1]};
                double t[3]; cross3(rw, fw, t);
                for (int k = 0; k < 3; ++k) { F[k] += fw[k]; Tw[k] += t[k]; }
            }
        }
    }
    if (ph_drag(x->physics)) {  /* _drag (982-1011) on last_clipped_action, applied at link 4 (the COM) */
        const double* lr = x->last_rpm;
        double sum = 0;
        for (int i = 0; i < 4; ++i) sum += (2 * M_PI * lr[i]) / 60;
        const double dv[3] = {(-DRAG_XY * sum) * v[0], (-DRAG_XY * sum) * v[1], (-DRAG_Z * sum) * v[2]};
        double b[3];   /* base_rot.T @ (drag_factors * vel): body frame */
        for (int k = 0; k < 3; ++k) b[k] = R[0 + k] * dv[0] + R[3 + k] * dv[1] + R[6 + k] * dv[2];
        const double* Rv = ph_gnd(x->physics) ? R : Rl;
        for (int k = 0; k < 3; ++k) F[k] += Rv[3 * k + 0] * b[0] + Rv[3 * k + 1] * b[1] + Rv[3 * k + 2] * b[2];
    }
    if (ph_dw(x->physics)) {    /* _downwash (1013-1041): one link-4 force per drone above within 10 m */
        const double* me = x->pos[x->self];
        for (int i = 0; i < x->n; ++i) {
            const double dz = x->pos[i][2] - me[2];
            const double ex = x->pos[i][0] - me[0], ey = x->pos[i][1] - me[1];
            const double dxy = sqrt(ex * ex + ey * ey);
            if (dz > 0 && dxy < 10) {
                const double r = PROP_RADIUS / (4 * dz);
                const double alpha = DW_C1 * (r * r);
                const double beta = DW_C2 * dz + DW_C3;
                const double u = dxy / beta;
                const double fz = -alpha * exp(-.5 * (u * u));
                const double* Rv = ph_gnd(x->physics) ? R : Rl;
                F[0] += Rv[2] * fz; F[1] += Rv[5] * fz; F[2] += Rv[8] * fz;
            }
        }
    }
}

/* _dynamics (BaseAviary.py:1043-1102) + _integrateQ (1104-1118): explicit Euler on the body rates
 * rr; the returned world angular velocity is rotation(old quat) @ rr, what resetBaseVelocity stores. */
static void dyn_substep(double* p, double* q, double* v, double* w, double* rr, const double* rpm, double dt) {
    double R[9]; och_matrix_from_quat(q, R);
    double f[4], z[4];
    for (int i = 0; i < 4; ++i) { f[i] = rpm[i] * rpm[i] * KF; z[i] = rpm[i] * rpm[i] * KM; }
    const double T = f[0] + f[1] + f[2] + f[3];
    const double fw[3] = {R[2] * T, R[5] * T, R[8] * T - G * MASS};
    const double zt = -z[0] + z[1] - z[2] + z[3];
    const double ls = ARM / sqrt(2.0);
    const double xt = (f[0] + f[1] - f[2] - f[3]) * ls, yt = (-f[0] + f[1] + f[2] - f[3]) * ls;
    const double Jr[3] = {JX * rr[0], JY * rr[1], JZ * rr[2]};
    double c[3]; cross3(rr, Jr, c);
    const double tq[3] = {xt - c[0], yt - c[1], zt - c[2]};
    const double jinv[3] = {1.0 / JX, 1.0 / JY, 1.0 / JZ};   /* np.linalg.inv(diag J), pinned by the fixture */
    for (int i = 0; i < 3; ++i) {
        v[i] = v[i] + dt * (fw[i] / MASS);
        rr[i] = rr[i] + dt * (jinv[i] * tq[i]);
    }
    for (int i = 0; i < 3; ++i) p[i] = p[i] + dt * v[i];
    const double on = sqrt(rr[0] * rr[0] + rr[1] * rr[1] + rr[2] * rr[2]);
    if (!(fabs(on) <= 1e-8)) {   /* np.isclose(omega_norm, 0): atol 1e-8 */
        const double th = on * dt / 2, co = cos(th), si = sin(th), k = 2 / on;
        const double P = rr[0], Q = rr[1], Rz = rr[2];
        const double L[4][4] = {{0, Rz, -Q, P}, {-Rz, 0, P, Q}, {Q, -P, 0, Rz}, {-P, -Q, -Rz, 0}};
        double o[4];
        for (int i = 0; i < 4; ++i) {
            double m[4];
            for (int j = 0; j < 4; ++j) m[j] = (i == j ? co : 0.0) + (k * (L[i][j] * .5)) * si;
            o[i] = m[0] * q[0] + m[1] * q[1] + m[2] * q[2] + m[3] * q[3];
        }
        for (int i = 0; i < 4; ++i) q[i] = o[i];
    }
    for (int i = 0; i < 3; ++i) w[i] = R[3 * i + 0] * rr[0] + R[3 * i + 1] * rr[1] + R[3 * i + 2] * rr[2];
}
/* RK4 option (north_star; not a reference path): the equations of motion of _dynamics
 * (BaseAviary.py:1043-1102) as an ODE in y = (p, v, q, w_b) -- p' = v, v' = (R(q) T e_z - m g e_z) / m,
 * w_b' = J^-1 (tau - w_b x J w_b), q' = 1/2 L(w_b) q with _integrateQ's L (1104-1118) -- integrated by the
 * classic four-stage Runge-Kutta over one substep at constant rpm; q renormalised after the step and the
 * world angular velocity reported as R(q_new) w_b (DYN reports R(q_old) w_b). */
static void dyn_deriv(const double* q, const double* v, const double* rr, const double* rpm, double* dp, double* dv,
                      double* dq, double* drr) {
    double R[9]; och_matrix_from_quat(q, R);
    double f[4], z[4];
    for (int i = 0; i < 4; ++i) { f[i] = rpm[i] * rpm[i] * KF; z[i] = rpm[i] * rpm[i] * KM; }
    const double T = f[0] + f[1] + f[2] + f[3];
    const double fw[3] = {R[2] * T, R[5] * T, R[8] * T - G * MASS};
    const double zt = -z[0] + z[1] - z[2] + z[3];
    const double ls = ARM / sqrt(2.0);
    const double xt = (f[0] + f[1] - f[2] - f[3]) * ls, yt = (-f[0] + f[1] + f[2] - f[3]) * ls;
    const double Jr[3] = {JX * rr[0], JY * rr[1], JZ * rr[2]};
    double c[3]; cross3(rr, Jr, c);
    const double tq[3] = {xt - c[0], yt - c[1], zt - c[2]};
    const double jinv[3] = {1.0 / JX, 1.0 / JY, 1.0 / JZ};
    for (int i = 0; i < 3; ++i) { dp[i] = v[i]; dv[i] = fw[i] / MASS; drr[i] = jinv[i] * tq[i]; }
    const double P = rr[0], Q = rr[1], Rz = rr[2];
    const double L[4][4] = {{0, Rz, -Q, P}, {-Rz, 0, P, Q}, {Q, -P, 0, Rz}, {-P, -Q, -Rz, 0}};
    for (int i = 0; i < 4; ++i) dq[i] = 0.5 * (L[i][0] * q[0] + L[i][1] * q[1] + L[i][2] * q[2] + L[i][3] * q[3]);
}
static void rk4_substep(double* p, double* q, double* v, double* w, double* rr, const double* rpm, double dt) {
    double kp[4][3], kv[4][3], kq[4][4], kr[4][3];
    double yp[3], yv[3], yq[4], yr[3];
    const double a[4] = {0.0, 0.5 * dt, 0.5 * dt, dt};
    for (int s = 0; s < 4; ++s) {
        for (int i = 0; i < 3; ++i) {
            yp[i] = s ? p[i] + a[s] * kp[s - 1][i] : p[i];
            yv[i] = s ? v[i] + a[s] * kv[s - 1][i] : v[i];
            yr[i] = s ? rr[i] + a[s] * kr[s - 1][i] : rr[i];
        }
        for (int i = 0; i < 4; ++i) yq[i] = s ? q[i] + a[s] * kq[s - 1][i] : q[i];
        (void)yp;
        dyn_deriv(yq, yv, yr, rpm, kp[s], kv[s], kq[s], kr[s]);
    }
    const double h6 = dt / 6.0;
    for (int i = 0; i < 3; ++i) {
        p[i] = p[i] + h6 * (((kp[0][i] + 2.0 * kp[1][i]) + 2.0 * kp[2][i]) + kp[3][i]);
        v[i] = v[i] + h6 * (((kv[0][i] + 2.0 * kv[1][i]) + 2.0 * kv[2][i]) + kv[3][i]);
        rr[i] = rr[i] + h6 * (((kr[0][i] + 2.0 * kr[1][i]) + 2.0 * kr[2][i]) + kr[3][i]);
    }
    for (int i = 0; i < 4; ++i) q[i] = q[i] + h6 * (((kq[0][i] + 2.0 * kq[1][i]) + 2.0 * kq[2][i]) + kq[3][i]);
    const double qn = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int i = 0; i < 4; ++i) q[i] = q[i] / qn;
    double R[9]; och_matrix_from_quat(q, R);
    for (int i = 0; i < 3; ++i) w[i] = R[3 * i + 0] * rr[0] + R[3 * i + 1] * rr[1] + R[3 * i + 2] * rr[2];
}

/* One drone, `steps` substeps of DYN (rk4 = 0, explicit Euler as the reference) or the RK4 option at
 * constant rpm: the order-of-convergence probe (tests/test_oracle_golden.py). y = p[3] v[3] q[4] rr[3] w[3]. */
void och_dyn_integrate(double* y, const double* rpm, double dt, int64_t steps, int rk4) {
    for (int64_t s = 0; s < steps; ++s) {
        if (rk4) rk4_substep(y, y + 6, y + 3, y + 13, y + 10, rpm, dt);
        else dyn_substep(y, y + 6, y + 3, y + 13, y + 10, rpm, dt);
    }
}

/* torque_world applies with link_lag = 0 (rounds 1-4: the z torque in the world frame, PyBullet's LINK_FRAME torque
 * quirk on a base).  Under the cached link frame the z torque turns with that frame like the prop forces: the torque
 * is applied to link 4, and PyBullet rotates a link's LINK_FRAME torque by the link's cached transform; the trace
 * rejects the world-frame alternative (torque_world = 2 here, a test-only value: 2e-5 m/s vs 2e-13 by step 4,
 * DESIGN.md §3).
 * ql != NULL (config link_lag): Bullet's cached link frame.  PyBullet's applyExternalForce / applyExternalTorque
 * with LINK_FRAME on a multibody link rotate the link-frame vector by that link's cached world transform, which a
 * link without a collision shape (the cf2x prop links and center_of_mass_link, cf2x.urdf:34-98) only gets from the
 * forward-kinematics pass at the start of the previous stepSimulation: the base attitude one substep old (ql).  The
 * force then acts at the link's current centre of mass, so the lever arms rotate with the current attitude R.  In
 * the body frame, with u = R^T ql_z: torque = sum_i f_i (r_i x u) + u tz, force = ql_z sum f.  Pinned by the
 * recorded real-PyBullet trace (tests/golden/trace_inverse.npz): the first evaluation episode's
 * drone xy velocities and positions to ~1e-12 relative over its first steps, where the current-attitude model
 * (ql = NULL) misses the first step's velocity by a factor 2.5. */
/* Test hook (tests/golden/make_trace_inverse.py): alternative rigid-body models the real-PyBullet trace is checked
 * against.  Bit 0: the base's linear acceleration with a velocity-product term -m (w x v) (what integrating Bullet's
 * body-frame spatial acceleration as a world-frame one would add).  Its trace residual is 7e-9 m/s on the first step
 * against 2e-16 without it, so 0 (the default) is the model. */
static int g_model_flags = 0;
void och__set_model_flags(int f) { g_model_flags = f; }
static void drone_substep(const och_config* c, double* p, double* q, double* v, double* w, const double* rpm, double dt,
                          const phys_ctx* x, double* ql) {
    double R[9]; och_matrix_from_quat(q, R);
    double F[3] = {0, 0, 0}, Tw[3] = {0, 0, 0}, tb[3];
    double t0 = rpm[0] * rpm[0] * KM, t1 = rpm[1] * rpm[1] * KM, t2 = rpm[2] * rpm[2] * KM, t3 = rpm[3] * rpm[3] * KM;
    double tz = (-t0 + t1 - t2 + t3);
    const int body = !x && (ql || c->torque_world);
    double Rl[9];   /* the cached link frame: directions of every LINK_FRAME force / torque on the links */
    if (ql) och_matrix_from_quat(ql, Rl);
    else memcpy(Rl, R, sizeof(Rl));
    if (body && ql) {
        double f[4];
        for (int i = 0; i < 4; ++i) f[i] = rpm[i] * rpm[i] * KF;
        const double T = ((f[0] + f[1]) + f[2]) + f[3];
        F[0] = Rl[2] * T; F[1] = Rl[5] * T; F[2] = Rl[8] * T;
        double u[3];
        for (int i = 0; i < 3; ++i) u[i] = (R[0 + i] * Rl[2] + R[3 + i] * Rl[5]) + R[6 + i] * Rl[8];
        const double sy = 0.028 * (((-f[0] - f[1]) + f[2]) + f[3]);   /* sum_i f_i r_iy */
        const double sx = 0.028 * (((-f[0] + f[1]) + f[2]) - f[3]);   /* -sum_i f_i r_ix */
        if (c->torque_world == 2) {   /* alternative model (trace inversion only): world-frame z torque, rejected */
            tb[0] = sy * u[2] + R[6] * tz;
            tb[1] = sx * u[2] + R[7] * tz;
            tb[2] = (-sx * u[1] - sy * u[0]) + R[8] * tz;
        } else {
            tb[0] = sy * u[2] + u[0] * tz;
            tb[1] = sx * u[2] + u[1] * tz;
            tb[2] = (-sx * u[1] - sy * u[0]) + u[2] * tz;
        }
    } else if (body) {
        /* PYB with the world-frame motor torque (the default): the four +z prop forces (LINK_FRAME at
         * (px, py, 0), cf2x.urdf:42-78) reduced to the body frame in closed form.  Their world torque
         * sum(R P_i x R e_z f_i) = R sum(P_i x e_z f_i) comes back to the body as (sum py f, -sum px f, 0);
         * the world-frame yaw torque tz e_z is R^T e_z tz = tz (R[6], R[7], R[8]). */
        double f[4];
        for (int i = 0; i < 4; ++i) f[i] = rpm[i] * rpm[i] * KF;
        const double T = ((f[0] + f[1]) + f[2]) + f[3];
        F[0] = R[2] * T; F[1] = R[5] * T; F[2] = R[8] * T;
        tb[0] = 0.028 * (((-f[0] - f[1]) + f[2]) + f[3]) + R[6] * tz;
        tb[1] = 0.028 * (((-f[0] + f[1]) + f[2]) - f[3]) + R[7] * tz;
        tb[2] = R[8] * tz;
    } else {
        for (int i = 0; i < 4; ++i) {
            double f = rpm[i] * rpm[i] * KF;
            double fw[3] = {Rl[2] * f, Rl[5] * f, Rl[8] * f};
            double rb[3] = {PROP[i][0], PROP[i][1], 0.0};
            double rw[3] = {R[0] * rb[0] + R[1] * rb[1], R[3] * rb[0] + R[4] * rb[1], R[6] * rb[0] + R[7] * rb[1]};
            double t[3]; cross3(rw, fw, t);
            for (int k = 0; k < 3; ++k) { F[k] += fw[k]; Tw[k] += t[k]; }
        }
        if (c->torque_world && (!ql || c->torque_world == 2)) Tw[2] += tz;
        else { Tw[0] += Rl[2] * tz; Tw[1] += Rl[5] * tz; Tw[2] += Rl[8] * tz; }
        if (x) physics_forces(x, p, q, v, R, Rl, rpm, F, Tw);
    }
    if (ql) memcpy(ql, q, 4 * sizeof(double));   /* the next substep's cached link frame: this substep's start */
    F[2] += -MASS * G;
    double k = c->damping;
    if (k != 0.0) {
        double sp = norm3(v);
        for (int i = 0; i < 3; ++i) F[i] -= MASS * v[i] * (k + k * sp);
    }
    double wb[3];
    for (int i = 0; i < 3; ++i) {
        wb[i] = R[0 + i] * w[0] + R[3 + i] * w[1] + R[6 + i] * w[2];
        if (!body) tb[i] = R[0 + i] * Tw[0] + R[3 + i] * Tw[1] + R[6 + i] * Tw[2];
    }
    const double J[3] = {JX, JY, JZ};
    if (k != 0.0) {
        double sw = norm3(wb);
        for (int i = 0; i < 3; ++i) tb[i] -= J[i] * wb[i] * (k + k * sw);
    }
    if (c->gyro) {
        double Jw[3] = {J[0] * wb[0], J[1] * wb[1], J[2] * wb[2]}, g[3];
        cross3(wb, Jw, g);
        for (int i = 0; i < 3; ++i) tb[i] -= g[i];
    }
    double ab[3] = {tb[0] / J[0], tb[1] / J[1], tb[2] / J[2]};
    if (g_model_flags & 1) {   /* alternative model (trace inversion only): a velocity-product term m w x v, rejected */
        double wxv[3]; cross3(w, v, wxv);
        for (int i = 0; i < 3; ++i) F[i] -= MASS * wxv[i];
    }
    for (int i = 0; i < 3; ++i) {
        double aw = R[i * 3 + 0] * ab[0] + R[i * 3 + 1] * ab[1] + R[i * 3 + 2] * ab[2];
        v[i] = v[i] + (F[i] / MASS) * dt;
        w[i] = w[i] + aw * dt;
    }
    for (int i = 0; i < 3; ++i) p[i] = p[i] + v[i] * dt;
    double fang = norm3(w);
    if (fang * dt > 0.5 * (0.5 * M_PI)) fang = 0.5 * (0.5 * M_PI) / dt;
    double axis[3];
    if (fang < 0.001) {
        double s = 0.5 * dt - (dt * dt * dt) * 0.020833333333 * fang * fang;
        for (int i = 0; i < 3; ++i) axis[i] = w[i] * s;
    } else {
        double s = sin(0.5 * fang * dt) / fang;
        for (int i = 0; i < 3; ++i) axis[i] = w[i] * s;
    }
    double dq[4] = {axis[0], axis[1], axis[2], cos(fang * dt * 0.5)}, qn[4];
    quat_mul(dq, q, qn);
    double n = sqrt(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
    for (int i = 0; i < 4; ++i) q[i] = qn[i] / n;
}

/* ---------------------------------------------------------------------------------------------
 * Flocking: BaseAviary._flockingStep (BaseAviary.py:1352-1400) → MathematicalFlock._flocking
 * (flockUtils.py:116-137), _global_clustering (150-160); _local_clustering (164-216) and the
 * boundary term (218-234) enter with weight 0 and are zero for one connected herd.
 * ------------------------------------------------------------------------------------------- */
static const double EPS = 0.1, H = 0.2;

static double sigma_norm_n(double n) { return (sqrt(1 + EPS * (n * n)) - 1) / EPS; }          /* 26-27 */
static double bump(double z) {                                                                   /* 34-39 */
    if (z < 0) return 0.0;
    if (z < H) return 1.0;
    if (z <= 1) return (1 + cos(M_PI * (z - H) / (1 - H))) / 2;
    return 0.0;
}
static double sigma_1(double z) { return z / sqrt(1 + z * z); }                                  /* 22-23 */
static double phi_alpha(double z, double r, double d) {                                          /* 41-49 */
    double ra = sigma_norm_n(fabs(r)), da = sigma_norm_n(fabs(d));
    double zz = z - da;
    return bump(z / ra) * (((5.0 + 5.0) * sigma_1(zz + 0.0) + (5.0 - 5.0)) / 2);
}

/* gradient + consensus of one neighbour set; flockUtils.py:327-337 */
static void pair_terms(double qix, double qiy, double pix, double piy, double qjx, double qjy, double pjx,
                       double pjy, double r, double d, double* gx, double* gy, double* cx, double* cy) {
    double zx = qjx - qix, zy = qjy - qiy;
    double n = norm2(zx, zy);
    double sn = sigma_norm_n(n);
    double den = sqrt(1 + EPS * (n * n));
    double ph = phi_alpha(sn, r, d);
    *gx += ph * (zx / den);
    *gy += ph * (zy / den);
    double a = bump(sn / sigma_norm_n(fabs(r)));
    *cx += a * (pjx - pix);
    *cy += a * (pjy - piy);
}

void och_flock_update(const double* cp, const double* cv, int m, const double* dxy, int n, double* new_cv) {
    const double C2A = 2 * sqrt(3.0), C2B = 2 * sqrt(20.0), C1G = 5, C2G = 0.2 * sqrt(5.0);
    const double sensing = 999, danger = 1.1, dt_sqr = 0.05 * 0.05;
    for (int i = 0; i < m; ++i) {
        double qix = cp[2 * i], qiy = cp[2 * i + 1], pix = cv[2 * i], piy = cv[2 * i + 1];
        /* alpha term: flockUtils.py:237-258 */
        double ux = 0, uy = 0;
        double gx = 0, gy = 0, cx = 0, cy = 0; int nb = 0;
        for (int j = 0; j < m; ++j) {
            if (j == i) continue;
            if (!(norm2(qix - cp[2 * j], qiy - cp[2 * j + 1]) <= sensing)) continue;
            ++nb;
            pair_terms(qix, qiy, pix, piy, cp[2 * j], cp[2 * j + 1], cv[2 * j], cv[2 * j + 1], 1.2, 1.2, &gx, &gy, &cx, &cy);
        }
        if (nb > 0) { ux = C2A * gx + C2A * cx; uy = C2A * gy + C2A * cy; }
        /* delta (shepherd) term: flockUtils.py:271-317 */
        double dx = 0, dy = 0;
        gx = gy = cx = cy = 0; nb = 0;
        for (int k = 0; k < n; ++k) {
            double yx = dxy[2 * k], yy = dxy[2 * k + 1];
            if (!(norm2(yx - qix, yy - qiy) <= sensing + 2)) continue;
            ++nb;
            double difx = qix - yx, dify = qiy - yy;
            double d = norm2(difx, dify) + 1e-6;
            double mu = d / 1.0 < 1.0 ? d / 1.0 : 1.0;
            double akx = difx / d, aky = dify / d;
            double P00 = 1 - akx * akx, P01 = 0 - akx * aky, P10 = 0 - aky * akx, P11 = 1 - aky * aky;
            double qkx = mu * qix + (1 - mu) * yx, qky = mu * qiy + (1 - mu) * yy;
            double pkx = mu * (P00 * pix + P01 * piy), pky = mu * (P10 * pix + P11 * piy);
            pair_terms(qix, qiy, pix, piy, qkx, qky, pkx, pky, 1.0, 1.0, &gx, &gy, &cx, &cy);
        }
        if (nb > 0) { dx = C2B * gx + C2B * cx; dy = C2B * gy + C2B * cy; }
        /* predator avoidance: flockUtils.py:343-348 */
        double sx = 0, sy = 0;
        for (int k = 0; k < n; ++k) {
            double ex = dxy[2 * k] - qix, ey = dxy[2 * k + 1] - qiy;
            double dn = norm2(ex, ey);
            if (dn <= danger) {
                double d3 = pow(dn, 3.0);   /* numpy float64 ** 3 */
                sx += -650000.0 * ex / d3;
                sy += -650000.0 * ey / d3;
            }
        }
        dx += sx; dy += sy;
        /* gamma: flockUtils.py:150-160, 340-341 (consensus target 1 → (1,1)) */
        double gmx = -C1G * sigma_1(qix - 1) - C2G * pix, gmy = -C1G * sigma_1(qiy - 1) - C2G * piy;
        double qx = (ux + dx) + gmx, qy = (uy + dy) + gmy;
        double vx = pix + qx * dt_sqr, vy = piy + qy * dt_sqr;
        double sp = norm2(vx, vy);
        if (sp > MAX_VEL_CATTLE) { double f = MAX_VEL_CATTLE / sp; vx *= f; vy *= f; }
        new_cv[2 * i] = vx; new_cv[2 * i + 1] = vy;
    }
}

/* ---------------------------------------------------------------------------------------------
 * evaluate_herding_effectiveness (evaluation.py:100-138), is_left (271-273)
 * ------------------------------------------------------------------------------------------- */
double och_effectiveness(const double* cxy, int m, const double* dxy, int n) {
    if (m <= 0) return 0;
    int herded = 0;
    for (int c = 0; c < m; ++c) {
        double px = cxy[2 * c], py = cxy[2 * c + 1];
        int wn = 0;
        for (int i = 0; i < n; ++i) {
            double x1 = dxy[2 * i], y1 = dxy[2 * i + 1];
            double x2 = dxy[2 * ((i + 1) % n)], y2 = dxy[2 * ((i + 1) % n) + 1];
            double il = (x2 - x1) * (py - y1) - (px - x1) * (y2 - y1);
            if (y1 <= py) { if (y2 > py && il > 0) wn += 1; }
            else { if (y2 <= py && il < 0) wn -= 1; }
        }
        if (wn) herded += 1;
    }
    return (double)herded / m * 100;
}

/* ---------------------------------------------------------------------------------------------
 * Spacing rewards: CattleAviary.py:572-679 (= MARLCattleAviary.py:402-509)
 * ------------------------------------------------------------------------------------------- */
double och_simple_spacing(double r, int level) {
    double desired = LEVELS[level].desired, tol = desired * LEVELS[level].tol;
    double lb = desired - tol, ub = desired + tol;
    if (lb <= r && r <= ub) return 1.0;
    if (r < lb) return -1 + (r / lb) * 2;
    if (r > ub) return 1 - ((r - ub) / (7.0 - ub)) * 2;
    return -1.0;
}
double och_complex_spacing(double r, int level) {
    double ds = LEVELS[level].desired;
    double t = (r - ds) / (0.4 + 1e-9);
    double gauss = exp(-0.5 * (t * t));
    double coll = r < 0.3 ? -1.0 * (1.0 - (r / (0.3 + 1e-9))) : 0.0;
    double pull = r > 1.5 ? -0.3 * (r - 1.5) / (5.0 - 1.5) : 0.0;
    double rew = gauss + coll + pull;
    rew += 0.1 * (1 - fabs(r - ds));
    return rew;
}
double och_cattle_spacing(double r) {
    if (r <= SP_R0) return SP_A * exp(-((r - SP_D) * (r - SP_D)) / (2 * (SP_C * SP_C))) - SP_B * exp(-(r * r) / (2 * (SP_K * SP_K)));
    double fr0 = SP_A * exp(-((SP_R0 - SP_D) * (SP_R0 - SP_D)) / (2 * (SP_C * SP_C))) - SP_B * exp(-(SP_R0 * SP_R0) / (2 * (SP_K * SP_K)));
    double C = fr0 / exp(-SP_LAM * SP_R0);
    return C * exp(-SP_LAM * r);
}

/* ---------------------------------------------------------------------------------------------
 * Task helpers (shared geometry of CattleAviary / MARLCattleAviary)
 * ------------------------------------------------------------------------------------------- */
typedef struct { double cent, eff, min_spacing; double mean_cx, mean_cy; } geo_t;

static void geometry(const och_config* c, const och_state* s, geo_t* g) {
    int n = s->n, m = c->m;
    double cx = 0, cy = 0, dx = 0, dy = 0;
    for (int j = 0; j < m; ++j) { cx += s->cp[j][0]; cy += s->cp[j][1]; }
    for (int i = 0; i < n; ++i) { dx += s->dp[i][0]; dy += s->dp[i][1]; }
    cx /= m; cy /= m; dx /= n; dy /= n;   /* HerdCentroid / DroneCentroid, BaseRLAviary.py:348-392 */
    double ex = dx - cx, ey = dy - cy, ez = (TARGET_ALT + 0.5) - (TARGET_ALT + 0.5);
    g->cent = sqrt(ex * ex + ey * ey + ez * ez);
    g->mean_cx = cx; g->mean_cy = cy;
    double dxy[2 * OCH_NMAX], cxy[2 * OCH_MMAX];
    for (int i = 0; i < n; ++i) { dxy[2 * i] = s->dp[i][0]; dxy[2 * i + 1] = s->dp[i][1]; }
    for (int j = 0; j < m; ++j) { cxy[2 * j] = s->cp[j][0]; cxy[2 * j + 1] = s->cp[j][1]; }
    g->eff = och_effectiveness(cxy, m, dxy, n);
    double ms = INFINITY;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j)
            if (i != j) {
                double d = norm2(s->dp[i][0] - s->dp[j][0], s->dp[i][1] - s->dp[j][1]);
                if (d < ms || d != d) ms = (d != d) ? d : (d < ms ? d : ms);
            }
    g->min_spacing = ms;
}

/* np.partition(other_dists, 1)[:2] with other_dists[i] = inf */
static void nearest_two(const och_state* s, int i, double* a, double* b) {
    double m1 = INFINITY, m2 = INFINITY;
    for (int j = 0; j < s->n; ++j) {
        double d = (j == i) ? INFINITY : norm2(s->dp[j][0] - s->dp[i][0], s->dp[j][1] - s->dp[i][1]);
        if (d < m1) { m2 = m1; m1 = d; } else if (d < m2) m2 = d;
    }
    *a = m1; *b = m2;
}

static double closest_cow(const och_config* c, const och_state* s, int i) {
    double best = INFINITY;
    for (int j = 0; j < c->m; ++j) {
        double d = norm2(s->cp[j][0] - s->dp[i][0], s->cp[j][1] - s->dp[i][1]);
        if (d < best) best = d;
    }
    return best;
}

/* curriculum_learning.py:200-219 */
static void curriculum_success(och_state* s) {
    s->tally += 1;
    if (s->tally >= LEVELS[s->level].required_tally) {
        s->tally = 0;
        s->level += 1;
        if (s->level >= 8) s->level = 7;
    }
}

static double episode_len(const och_config* c) { return LEVELS[c->start_level].episode_len; }

/* CattleAviary._computeTerminated (CattleAviary.py:422-492) / MARLCattleAviary (246-321) */
static int term_call(const och_config* c, och_state* s, const geo_t* g) {
    const level_t* L = &LEVELS[s->level];
    int lvl = s->level;
    if (lvl == 0 || lvl == 1) {
        double up = L->desired + L->desired * L->tol, lo = L->desired - L->desired * L->tol;
        if (g->min_spacing < up && g->min_spacing > lo) {
            s->clock += (c->mode == 0) ? 1.0 / 240 : 1.0 / c->ctrl_freq;
            if (s->clock >= L->hold) return 1;
        } else s->clock = 0;
    } else if (lvl == 2 || lvl == 3) {
        if (g->cent < L->approach_min) return 1;
    } else if (lvl == 4 || lvl == 6) {
        if (g->eff > L->min_eff) return 1;
    } else if (lvl == 5) {
        if (g->eff > L->min_eff) {
            double up = L->cattle_desired + L->cattle_desired * L->cattle_tol;
            double lo = L->cattle_desired - L->cattle_desired * L->cattle_tol;
            if (g->min_spacing < up && g->min_spacing > lo) return 1;
        }
    }
    return 0;
}

static int trunc_drone(const och_config* c, const och_state* s, const geo_t* g, int i, int pairs_from) {
    (void)g;
    if (fabs(s->dp[i][2] - TARGET_ALT) > TARGET_ALT * 0.6) return 1;
    for (int j = pairs_from; j < s->n; ++j) {
        if (j == i) continue;
        if (norm2(s->dp[i][0] - s->dp[j][0], s->dp[i][1] - s->dp[j][1]) < COLLISION_THRESHOLD) return 1;
    }
    (void)c;
    return 0;
}

static int isolated(const och_state* s, int i) {
    for (int j = 0; j < s->n; ++j) {
        if (j == i) continue;
        double d = norm2(s->dp[j][0] - s->dp[i][0], s->dp[j][1] - s->dp[i][1]);
        if (!(d > MAX_FORMATION_DISTANCE)) return 0;
    }
    return 1;
}

/* CattleAviary._computeTruncated (CattleAviary.py:497-552) */
static int trunc_ctde(const och_config* c, const och_state* s, const geo_t* g) {
    for (int i = 0; i < s->n; ++i)
        if (fabs(s->dp[i][2] - TARGET_ALT) > TARGET_ALT * 0.6) return 1;
    for (int i = 0; i < s->n; ++i)
        for (int j = i + 1; j < s->n; ++j)
            if (norm2(s->dp[i][0] - s->dp[j][0], s->dp[i][1] - s->dp[j][1]) < COLLISION_THRESHOLD) return 1;
    for (int i = 0; i < s->n; ++i)
        if (isolated(s, i)) return 1;
    if (g->cent > MISSION_BOUNDARY) return 1;
    if ((double)s->step_counter / c->ctrl_freq > episode_len(c)) return 1;
    return 0;
}

/* MARLCattleAviary._computeTruncated (MARLCattleAviary.py:326-383) */
static int trunc_marl(const och_config* c, const och_state* s, const geo_t* g, int i) {
    if (trunc_drone(c, s, g, i, 0)) return 1;
    if (isolated(s, i)) return 1;
    if (g->cent > MISSION_BOUNDARY) return 1;
    if ((double)s->step_counter / c->ctrl_freq > episode_len(c)) return 1;
    return 0;
}

static double speed_limit(void) { return 0.3 * MAX_SPEED_KMH * (1000.0 / 3600.0); }

/* CattleAviary._computeReward (CattleAviary.py:213-332) incl. the nested term/trunc calls */
static double reward_ctde(const och_config* c, och_state* s, const geo_t* g) {
    int n = s->n;
    const level_t* L = &LEVELS[s->level];
    double sp_simple = 0, sp_complex = 0, per_sp[OCH_NMAX], per_cat[OCH_NMAX];
    for (int i = 0; i < n; ++i) {
        double a, b; nearest_two(s, i, &a, &b);
        if (!c->compat) { if (isinf(b)) b = NAN; if (isinf(a)) a = NAN; }
        per_sp[i] = 0;
        double ds[2] = {a, b};
        for (int k = 0; k < 2; ++k) {
            if (!c->compat && ds[k] != ds[k]) continue;
            double rc = och_complex_spacing(ds[k], s->level), rs = och_simple_spacing(ds[k], s->level);
            sp_complex += rc; sp_simple += rs; per_sp[i] += (rc + rs) / 2.0;
        }
    }
    sp_complex /= (n * 2.0); sp_simple /= (n * 2.0);
    double approach = 0;
    double max_step = speed_limit() / c->ctrl_freq;
    if (s->has_prev) approach = clipd(((s->prev_cent - g->cent) / (max_step + 1e-6)) * 5, -1.0, 1.0);
    s->prev_cent = g->cent; s->has_prev = 1;
    double herd = g->eff / 100;
    double cat = 0;
    for (int i = 0; i < n; ++i) { per_cat[i] = och_cattle_spacing(closest_cow(c, s, i)); cat += per_cat[i]; }
    cat /= n;
    double rg = sp_simple * L->w_simple + sp_complex * L->w_complex + 0.1 * L->w_survival + approach * L->w_approach +
                herd * L->w_eff + cat * L->w_cattle;
    double msp = 0, mcat = 0;
    for (int i = 0; i < n; ++i) { msp += per_sp[i]; mcat += per_cat[i]; }
    msp /= n; mcat /= n;
    double tot = 0;
    for (int i = 0; i < n; ++i) tot += rg + 0.5 * ((per_sp[i] - msp) + (per_cat[i] - mcat));
    double result = tot / n;
    int te = term_call(c, s, g);
    (void)trunc_ctde(c, s, g);
    if (te) curriculum_success(s);
    return result;
}

/* MARLCattleAviary._endOfEpisodeReward (183-241) */
static double eor_marl(const och_config* c, och_state* s, const geo_t* g, int i) {
    const level_t* L = &LEVELS[s->level];
    int lvl = s->level;
    double r = 0.0;
    if (lvl == 0 || lvl == 1) {
        double up = L->desired + L->desired * L->tol, lo = L->desired - L->desired * L->tol, a, b;
        nearest_two(s, i, &a, &b);
        if (a >= lo && a <= up && b >= lo && b <= up) r += 50.0 / s->n;
    } else if (lvl == 2 || lvl == 3) {
        if (g->cent < L->approach_min) r += 50.0;
    } else if (lvl == 4 || lvl == 6) {
        double dd = norm2(g->mean_cx - s->dp[i][0], g->mean_cy - s->dp[i][1]);
        double wgt = clipd(1.0 - dd / 10.0, 0, 1);
        r += g->eff * 2 * wgt;
    } else if (lvl == 5) {
        if (g->eff > L->min_eff) {
            double up = L->cattle_desired + L->cattle_desired * L->cattle_tol;
            double lo = L->cattle_desired - L->cattle_desired * L->cattle_tol, a, b;
            nearest_two(s, i, &a, &b);
            if (a >= lo && a <= up && b >= lo && b <= up) r += 50.0 / s->n;
        }
    }
    (void)c;
    return r;
}

/* MARLCattleAviary._computeReward (110-178) */
static double reward_marl(const och_config* c, och_state* s, const geo_t* g, int i) {
    const level_t* L = &LEVELS[s->level];
    double r = 0.0, a, b;
    nearest_two(s, i, &a, &b);
    if (!c->compat) { if (isinf(b)) b = a; if (isinf(a)) a = b = NAN; }
    double simple = (och_simple_spacing(a, s->level) + och_simple_spacing(b, s->level)) / 2;
    double cplx = (och_complex_spacing(a, s->level) + och_complex_spacing(b, s->level)) / 2;
    if (!c->compat && a != a) { simple = 0; cplx = 0; }
    r += simple * L->w_simple;
    r += cplx * L->w_complex;
    r += 0.1 * L->w_survival;
    double change = s->has_prev ? s->prev_cent - g->cent : 0.0;
    s->prev_cent = g->cent; s->has_prev = 1;
    double max_step = speed_limit() / c->ctrl_freq;
    r += clipd((change / (max_step + 1e-6)) * 5, -1.0, 1.0) * L->w_approach;
    r += (g->eff / 100) * L->w_eff;
    r += och_cattle_spacing(closest_cow(c, s, i)) * L->w_cattle;
    if (term_call(c, s, g)) {
        r += eor_marl(c, s, g, i);
        curriculum_success(s);
    } else if (trunc_marl(c, s, g, i)) {
        r -= 50;
    }
    return r;
}

void och_task(const och_config* c, och_state* s, double* reward, uint8_t* terminated, uint8_t* truncated) {
    geo_t g; geometry(c, s, &g);
    if (c->mode == 0) {
        /* BaseAviary.step: reward → terminated → truncated (sb3_envs/BaseAviary.py:458-460) */
        reward[0] = reward_ctde(c, s, &g);
        terminated[0] = (uint8_t)term_call(c, s, &g);
        truncated[0] = (uint8_t)trunc_ctde(c, s, &g);
    } else {
        int n = s->n;
        /* env.step's own dicts (rllib_envs/BaseAviary.py:425-431) */
        double r1[OCH_NMAX];
        uint8_t d1[OCH_NMAX];
        for (int i = 0; i < n; ++i) r1[i] = reward_marl(c, s, &g, i);
        for (int i = 0; i < n; ++i) d1[i] = (uint8_t)term_call(c, s, &g);
        for (int i = 0; i < c->n_ctor; ++i) { reward[i] = NAN; terminated[i] = 0; truncated[i] = 0; }
        if (!c->marl_wrapper) {
            for (int i = 0; i < n; ++i) {
                reward[i] = r1[i]; terminated[i] = d1[i]; truncated[i] = (uint8_t)trunc_marl(c, s, &g, i);
            }
            s->step_counter += 1;   /* rllib_envs/BaseAviary.py:436, after the dicts */
            return;
        }
        /* env.step counts its step before returning (rllib_envs/BaseAviary.py:436); the wrapper's
         * recomputation for active agents (marl_wrapper.py:104-113) sees the incremented counter */
        s->step_counter += 1;
        for (int i = 0; i < n; ++i) {
            if (!s->active[i]) continue;
            reward[i] = reward_marl(c, s, &g, i);
            terminated[i] = (uint8_t)term_call(c, s, &g);
            truncated[i] = (uint8_t)trunc_marl(c, s, &g, i);
        }
        for (int i = 0; i < n; ++i)
            if (s->active[i] && terminated[i]) s->active[i] = 0;
    }
}

/* ---------------------------------------------------------------------------------------------
 * Observations: BaseRLAviary._computeObs (BaseRLAviary.py:272-342), BaseMARLAviary._computeObs
 * (BaseMARLAviary.py:253-303).  The action-buffer block is always zero.
 * ------------------------------------------------------------------------------------------- */
int och_obs_rows(const och_config* c) { return c->mode == 0 ? 12 : c->n_ctor; }

static void obs_row(const och_config* c, const och_state* s, int i, float* row) {
    int nb_off = 10, cat_off = (c->mode == 0) ? 34 : 18;
    for (int k = 0; k < 86; ++k) row[k] = 0.0f;
    double rpy[3]; och_euler_from_quat(s->dq[i], rpy);
    double own[10] = {s->dp[i][2], rpy[0], rpy[1], rpy[2], s->dv[i][0], s->dv[i][1], s->dv[i][2],
                      s->dw[i][0], s->dw[i][1], s->dw[i][2]};
    for (int k = 0; k < 10; ++k) row[k] = (float)own[k];
    /* stable sort of (vec, dist) by dist; first two */
    int used = 0, idx[2] = {-1, -1};
    for (int pick = 0; pick < 2; ++pick) {
        double best = INFINITY; int bj = -1;
        for (int j = 0; j < s->n; ++j) {
            if (j == i || j == idx[0]) continue;
            double d = norm2(s->dp[j][0] - s->dp[i][0], s->dp[j][1] - s->dp[i][1]);
            if (bj < 0 || d < best) { best = d; bj = j; }
        }
        if (bj < 0) break;
        idx[pick] = bj; ++used;
    }
    for (int k = 0; k < used; ++k) {
        row[nb_off + 2 * k] = (float)(s->dp[idx[k]][0] - s->dp[i][0]);
        row[nb_off + 2 * k + 1] = (float)(s->dp[idx[k]][1] - s->dp[i][1]);
    }
    int mc = c->m < 16 ? c->m : 16;
    for (int j = 0; j < mc; ++j) {
        row[cat_off + 2 * j] = (float)(s->cp[j][0] - s->dp[i][0]);
        row[cat_off + 2 * j + 1] = (float)(s->cp[j][1] - s->dp[i][1]);
    }
}

void och_obs(const och_config* c, const och_state* s, float* obs) {
    int rows = och_obs_rows(c);
    for (int r = 0; r < rows; ++r) {
        if (r < s->n) obs_row(c, s, r, obs + 86 * r);
        else for (int k = 0; k < 86; ++k) obs[86 * r + k] = 0.0f;
    }
}

/* ---------------------------------------------------------------------------------------------
 * Philox4x32-10 (Random123) — synthetic actions and reset draws; identical on the GPU.
 * ------------------------------------------------------------------------------------------- */
static void philox(uint32_t ctr[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0], p1 = (uint64_t)0xCD9E8D57u * ctr[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ ctr[1] ^ k0, n2 = hi0 ^ ctr[3] ^ k1;
        ctr[0] = n0; ctr[1] = lo1; ctr[2] = n2; ctr[3] = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

void och_random_actions(const och_config* c, int64_t env_id, int64_t step, float* actions) {
    for (int k = 0; k < c->n_ctor; ++k) {
        uint32_t ctr[4] = {(uint32_t)step, (uint32_t)((uint64_t)step >> 32), (uint32_t)k, (uint32_t)env_id};
        philox(ctr, (uint32_t)c->seed, (uint32_t)(c->seed >> 32));
        for (int q = 0; q < 4; ++q) actions[4 * k + q] = (float)(ctr[q] >> 8) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
    }
}

static double reset_uniform(const och_config* c, const och_state* s, int j) {
    uint32_t ctr[4] = {(uint32_t)s->episode, (uint32_t)((uint64_t)s->episode >> 32), (uint32_t)j | (1u << 16),
                       (uint32_t)s->env_id};
    philox(ctr, (uint32_t)c->seed, (uint32_t)(c->seed >> 32));
    return ((double)(ctr[0] >> 5) * 67108864.0 + (double)(ctr[1] >> 6)) * (1.0 / 9007199254740992.0);
}

/* ---------------------------------------------------------------------------------------------
 * Reset: BaseAviary.reset (BaseAviary.py:280-331), initialize_drone_positions (251-277),
 * _housekeeping cattle spawn (600-637).  PID state, prev_cent_dists, drone_spacing_clock and the
 * curriculum persist across episodes in compat mode (they are never reset by the reference).
 * ------------------------------------------------------------------------------------------- */
void och_reset(const och_config* c, och_state* s) {
    int span = c->max_drones - c->min_drones + 1;
    int n = c->min_drones + (span > 1 ? (int)(reset_uniform(c, s, 0) * span) : 0);
    if (n > c->min_drones + span - 1) n = c->min_drones + span - 1;
    s->n = n;
    s->step_counter_A = 0;
    s->step_counter = 0;
    for (int i = 0; i < OCH_NMAX; ++i) {
        double x = 0, y = 0;
        if (i < n) {
            if (n <= 4) { x = i * 1.75; y = 0; }
            else { int r1 = n / 2; if (i < r1) { x = i * 1.75; y = 0; } else { x = (i - r1) * 1.75; y = 1.75; } }
        }
        s->dp[i][0] = x; s->dp[i][1] = y; s->dp[i][2] = i < n ? TARGET_ALT : 0;
        s->dq[i][0] = s->dq[i][1] = s->dq[i][2] = 0; s->dq[i][3] = 1;
        memcpy(s->qlag[i], s->dq[i], sizeof(s->qlag[i]));   /* loadURDF: the links' transforms at the spawn pose */
        for (int k = 0; k < 3; ++k) { s->dv[i][k] = 0; s->dw[i][k] = 0; }
        s->active[i] = (uint8_t)(i < n);
        for (int k = 0; k < 4; ++k) s->last_rpm[i][k] = 0;   /* _housekeeping (565, 581-582) */
        s->eval_dist[i] = 0;   /* episode_drone_distances = self.pos rows, zeroed by _housekeeping (567, 683-688) */
        for (int k = 0; k < 3; ++k) s->rpy_rates[i][k] = 0;
        if (!c->compat) for (int k = 0; k < 3; ++k) { s->pid_last_rpy[i][k] = 0; s->pid_int_pos[i][k] = 0; s->pid_int_rpy[i][k] = 0; }
    }
    s->spawn_index += 1;
    if (s->spawn_index >= c->spawn_scenarios) s->spawn_index = 0;
    for (int j = 0; j < c->m; ++j) {
        const double* p = c->spawn_table + ((size_t)s->spawn_index * c->spawn_cows + j) * 2;
        s->cp[j][0] = p[0]; s->cp[j][1] = p[1];
        double ang = M_PI * (2 * reset_uniform(c, s, 1 + j) - 1);
        s->cv[j][0] = MAX_VEL_CATTLE * cos(ang); s->cv[j][1] = MAX_VEL_CATTLE * sin(ang);
    }
    if (!c->compat) { s->has_prev = 0; s->prev_cent = 0; s->clock = 0; }
    s->episode += 1;
}

void och_init(const och_config* c, och_state* s, int64_t env_id) {
    memset(s, 0, sizeof(*s));
    s->env_id = env_id;
    s->level = c->start_level;
    s->spawn_index = (int32_t)((1 + env_id) % c->spawn_scenarios);  /* ctor's _housekeeping consumed one */
    s->prev_cent = 0; s->has_prev = 0;
    for (int i = 0; i < OCH_NMAX; ++i) { s->dq[i][3] = 1; s->qlag[i][3] = 1; }
}

/* ---------------------------------------------------------------------------------------------
 * step: BaseAviary.step (sb3_envs/BaseAviary.py:335-465; rllib_envs/BaseAviary.py:320-438)
 * ------------------------------------------------------------------------------------------- */
/* Test hook (tests/golden/make_trace_inverse.py): when set, the PID's target velocity of drone k is tv[3k..3k+2] in
 * float64 instead of the one _preprocessAction derives from the float32 action row -- a pure physics-model test that
 * the action's float32 rounding does not limit.  NULL (the default) restores the reference path. */
static const double* g_tv_override = NULL;
void och__set_target_vel(const double* tv) { g_tv_override = tv; }

int och_step(const och_config* c, och_state* s, const float* actions, float* obs, double* reward,
             uint8_t* terminated, uint8_t* truncated, float* terminal_obs, int autoreset) {
    int n = s->n;
    const double dt_ctrl = 1.0 / c->ctrl_freq, dt = 1.0 / c->pyb_freq;
    const int substeps = c->pyb_freq / c->ctrl_freq;
    s->step_counter_A += 1;
    double rpm[OCH_NMAX][4], p0[OCH_NMAX][2];
    for (int k = 0; k < n; ++k) { p0[k][0] = s->dp[k][0]; p0[k][1] = s->dp[k][1]; }
    const double sl = speed_limit();
    for (int k = 0; k < n; ++k) {
        /* _preprocessAction VEL branch: BaseRLAviary.py:185-222 */
        float a[4];
        for (int q = 0; q < 4; ++q) a[q] = (c->mode == 1 && !s->active[k]) ? 0.0f : actions[4 * k + q];
        /* the action row is float32: the norm and unit vector stay float32; SPEED_LIMIT * abs(a[3])
         * is float32 too under NumPy >= 2 (NEP 50 weak Python scalars; NumPy 1.x kept it fp64) */
        float hx = a[0], hy = a[1];
        float hn = sqrtf(hx * hx + hy * hy);
        float ux = 0.0f, uy = 0.0f;
        if (hn != 0.0f) { ux = hx / hn; uy = hy / hn; }
        float sc = (float)sl * fabsf(a[3]);
        double tv[3] = {(double)ux * (double)sc, (double)uy * (double)sc, 0.0 * (double)sc};
        if (g_tv_override) { tv[0] = g_tv_override[3 * k]; tv[1] = g_tv_override[3 * k + 1]; tv[2] = g_tv_override[3 * k + 2]; }
        double rpy[3]; och_euler_from_quat(s->dq[k], rpy);
        double tp[3] = {s->dp[k][0], s->dp[k][1], TARGET_ALT};
        double tr[3] = {0.0, 0.0, rpy[2]};
        och_pid_vel(s->dp[k], s->dq[k], s->dv[k], tp, tr, tv, dt_ctrl, s->pid_last_rpy[k], s->pid_int_pos[k],
                    s->pid_int_rpy[k], rpm[k]);
    }
    const int ph = c->physics;
    const double h_clip = och_gnd_eff_h_clip();
    for (int sub = 0; sub < substeps; ++sub) {
        double pos0[OCH_NMAX][3];   /* self.pos as of this substep's start (downwash) */
        memcpy(pos0, s->dp, sizeof(pos0));
        for (int k = 0; k < n; ++k) {
            if (ph == PH_DYN) {
                dyn_substep(s->dp[k], s->dq[k], s->dv[k], s->dw[k], s->rpy_rates[k], rpm[k], dt);
            } else if (ph == PH_DYN_RK4) {
                rk4_substep(s->dp[k], s->dq[k], s->dv[k], s->dw[k], s->rpy_rates[k], rpm[k], dt);
            } else {
                phys_ctx x = {ph, s->last_rpm[k], (const double (*)[3])pos0, n, k, h_clip};
                drone_substep(c, s->dp[k], s->dq[k], s->dv[k], s->dw[k], rpm[k], dt, ph == PH_PYB ? NULL : &x,
                              c->link_lag ? s->qlag[k] : NULL);
            }
        }
        if (ph != PH_DYN && ph != PH_DYN_RK4)   /* no p.stepSimulation under DYN: the cattle bodies do not move (447-448) */
            for (int j = 0; j < c->m; ++j) { s->cp[j][0] += s->cv[j][0] * dt; s->cp[j][1] += s->cv[j][1] * dt; }
        for (int k = 0; k < n; ++k) memcpy(s->last_rpm[k], rpm[k], sizeof(rpm[k]));   /* 450 */
    }
    /* update_evaluation_metrics (BaseAviary.py:1415-1426): |last_drones_pos - pos| * 1.7, last = the
     * previous read-back, (0, 0) on an episode's first step (reset() zeroes it, BaseAviary.py:317) */
    for (int k = 0; k < n; ++k) {
        const double lx = s->step_counter == 0 ? 0.0 : p0[k][0], ly = s->step_counter == 0 ? 0.0 : p0[k][1];
        const double ex = lx - s->dp[k][0], ey = ly - s->dp[k][1];
        s->eval_dist[k] += sqrt(ex * ex + ey * ey) * 1.7;
    }
    if (s->step_counter_A % 2 == 0) {
        double cp[2 * OCH_MMAX], cv[2 * OCH_MMAX], nv[2 * OCH_MMAX], dxy[2 * OCH_NMAX];
        for (int j = 0; j < c->m; ++j) { cp[2 * j] = s->cp[j][0]; cp[2 * j + 1] = s->cp[j][1]; cv[2 * j] = s->cv[j][0]; cv[2 * j + 1] = s->cv[j][1]; }
        for (int k = 0; k < n; ++k) { dxy[2 * k] = s->dp[k][0]; dxy[2 * k + 1] = s->dp[k][1]; }
        och_flock_update(cp, cv, c->m, dxy, n, nv);
        for (int j = 0; j < c->m; ++j) { s->cv[j][0] = nv[2 * j]; s->cv[j][1] = nv[2 * j + 1]; }
    }
    och_task(c, s, reward, terminated, truncated);   /* MARL: counts the step itself (436) */
    if (c->mode == 0) s->step_counter += substeps;   /* sb3_envs/BaseAviary.py:464 */
    int done;
    if (c->mode == 0) done = terminated[0] || truncated[0];
    else if (c->marl_wrapper) { done = 1; for (int i = 0; i < n; ++i) if (s->active[i]) done = 0; }
    else { done = 1; for (int i = 0; i < n; ++i) done &= terminated[i]; }
    if (done && autoreset) {
        if (terminal_obs) och_obs(c, s, terminal_obs);
        och_reset(c, s);
    }
    if (obs) och_obs(c, s, obs);
    return done;
}

/* ---------------------------------------------------------------------------------------------
 * CPU baseline: random-action rollout over E envs, one env per OpenMP thread iteration.
 * ------------------------------------------------------------------------------------------- */
double och_batch_rollout(const och_config* c, och_state* states, int64_t E, int64_t T, int threads) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
#endif
    {
        float act[OCH_NMAX * 4], obs[12 * 86];
        double rew[OCH_NMAX]; uint8_t te[OCH_NMAX], tr[OCH_NMAX];
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t e = 0; e < E; ++e)
            for (int64_t t = 0; t < T; ++t) {
                och_random_actions(c, states[e].env_id, t, act);
                och_step(c, &states[e], act, obs, rew, te, tr, NULL, 1);
            }
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
