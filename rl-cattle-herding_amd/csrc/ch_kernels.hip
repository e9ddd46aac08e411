// ch_kernels.hip — the fused env-step kernel for gfx950 (MI355X).
//
// One launch advances every environment by one control step (reference: BaseAviary.step,
// sb3_envs/BaseAviary.py:335-465).  Mapping: a workgroup is ONE wave (64 lanes) holding
// 64/TEAM environments; each environment gets a team of TEAM lanes (TEAM >= max(drones, cattle)).
// Inside a team, lane k owns drone k (PID + motor model + physics substeps, state in registers) and
// lane j owns cow j (integration + flocking over the herd staged in LDS).  Per-drone reward terms
// are evaluated in parallel; the reference's order-dependent bookkeeping (approach delta, hold clock,
// curriculum tally) runs on the team's lane 0 from LDS.  Observations are written with coalesced
// 16-byte stores.  State lives in HBM as structure-of-arrays, env-major within each component.
#include <hip/hip_runtime.h>

#include "ch_device.h"
#include "ch_internal.h"
#include "ch_common.h"

namespace ch {

template <class R, int TEAM>
struct Slot {
    R cx[TEAM], cy[TEAM], cvx[TEAM], cvy[TEAM];
    R dx[kNMax], dy[kNMax];
    // f32 mode: f64 positions for the centroids (StepParams::pos64); unused in f64 mode
    double cxd[sizeof(R) == 4 ? TEAM : 1], cyd[sizeof(R) == 4 ? TEAM : 1];
    double dxd[sizeof(R) == 4 ? kNMax : 1], dyd[sizeof(R) == 4 ? kNMax : 1];
    R pa[kNMax], pb[kNMax], pcat[kNMax];
    R sa[kNMax], sb[kNMax], ca[kNMax], cb[kNMax], scat[kNMax];
    float own[kNMax][10];
    float nbr[kNMax][4];
    uint8_t dflags[kNMax];  // bit0 altitude, bit1 collision, bit2 isolated, bit3 NaN distance
    uint8_t herded[TEAM];
    int done, n, reset, spawn, episode;
};

enum { F_ALT = 1, F_COLL = 2, F_ISO = 4, F_NAN = 8 };

template <class R>
__device__ __forceinline__ R ld(const R* base, int comp, long long stride, long long idx) { return base[comp * stride + idx]; }

// observation element f of an env block (BaseRLAviary.py:272-342 / BaseMARLAviary.py:253-303)
// observation element (row, col) of an env block (BaseRLAviary.py:272-342 / BaseMARLAviary.py:253-303)
template <class R, int TEAM>
__device__ __forceinline__ float obs_val(const Slot<R, TEAM>& S, int row, int col, int n, int m_obs, int cat_off) {
    if (row >= n) return 0.0f;
    if (col < 10) return S.own[row][col];
    if (col < 14) return S.nbr[row][col - 10];
    if (col < cat_off) return 0.0f;
    int k = (col - cat_off) >> 1;
    if (k >= m_obs) return 0.0f;
    if constexpr (sizeof(R) == 4)   // f32 mode: offsets from the f64 positions
        return (col & 1) ? (float)(S.cyd[k] - S.dyd[row]) : (float)(S.cxd[k] - S.dxd[row]);
    else
        return (col & 1) ? (float)(S.cy[k] - S.dy[row]) : (float)(S.cx[k] - S.dx[row]);
}

// the env's [rows][86] block with 16-byte (or 8-byte) coalesced stores; (row, col) advance
// incrementally so no division sits in the loop
template <int W, class R, int TEAM>
__device__ __forceinline__ void write_obs_w(float* out, int rows, const Slot<R, TEAM>& S, int t, int m_obs, int cat_off) {
    const int n = S.n, F = rows * 86;
    int f0 = t * W, row = f0 / 86, col = f0 - row * 86;
    for (int q = t; q < F / W; q += TEAM) {
        float v[W];
        int r = row, c = col;
#pragma unroll
        for (int u = 0; u < W; ++u) {
            v[u] = obs_val(S, r, c, n, m_obs, cat_off);
            if (++c == 86) { c = 0; ++r; }
        }
        if constexpr (W == 4) reinterpret_cast<float4*>(out)[q] = make_float4(v[0], v[1], v[2], v[3]);
        else reinterpret_cast<float2*>(out)[q] = make_float2(v[0], v[1]);
        col += W * TEAM;
        while (col >= 86) { col -= 86; ++row; }
    }
}

template <class R, int TEAM>
__device__ __forceinline__ void write_obs(float* out, int rows, const Slot<R, TEAM>& S, int t, int m_obs, int cat_off) {
    if (((rows * 86) & 3) == 0) write_obs_w<4>(out, rows, S, t, m_obs, cat_off);
    else write_obs_w<2>(out, rows, S, t, m_obs, cat_off);
}

// own-state block and nearest-two neighbour block of drone i (needs S.dx/S.dy of all drones)
template <class R, int TEAM>
__device__ __forceinline__ void drone_obs_prep(Slot<R, TEAM>& S, int i, int n, R z, const R rpy[3], const R v[3], const R w[3]) {
    S.own[i][0] = (float)z;
    S.own[i][1] = (float)rpy[0]; S.own[i][2] = (float)rpy[1]; S.own[i][3] = (float)rpy[2];
    S.own[i][4] = (float)v[0]; S.own[i][5] = (float)v[1]; S.own[i][6] = (float)v[2];
    S.own[i][7] = (float)w[0]; S.own[i][8] = (float)w[1]; S.own[i][9] = (float)w[2];
    (void)n;
}

template <class R, int TEAM>
__device__ __forceinline__ void neighbour_obs(Slot<R, TEAM>& S, int i, int n) {
    // stable sort of (vec, dist) by distance, first two (BaseRLAviary.py:303-317)
    int i1 = -1, i2 = -1;
    R b1 = 0, b2 = 0;
    for (int j = 0; j < n; ++j) {
        if (j == i) continue;
        R d = norm2(S.dx[j] - S.dx[i], S.dy[j] - S.dy[i]);
        if (i1 < 0 || d < b1) { i2 = i1; b2 = b1; i1 = j; b1 = d; }
        else if (i2 < 0 || d < b2) { i2 = j; b2 = d; }
    }
    if constexpr (sizeof(R) == 4) {   // f32 mode: offsets from the f64 positions
        S.nbr[i][0] = i1 >= 0 ? (float)(S.dxd[i1] - S.dxd[i]) : 0.0f;
        S.nbr[i][1] = i1 >= 0 ? (float)(S.dyd[i1] - S.dyd[i]) : 0.0f;
        S.nbr[i][2] = i2 >= 0 ? (float)(S.dxd[i2] - S.dxd[i]) : 0.0f;
        S.nbr[i][3] = i2 >= 0 ? (float)(S.dyd[i2] - S.dyd[i]) : 0.0f;
    } else {
        S.nbr[i][0] = i1 >= 0 ? (float)(S.dx[i1] - S.dx[i]) : 0.0f;
        S.nbr[i][1] = i1 >= 0 ? (float)(S.dy[i1] - S.dy[i]) : 0.0f;
        S.nbr[i][2] = i2 >= 0 ? (float)(S.dx[i2] - S.dx[i]) : 0.0f;
        S.nbr[i][3] = i2 >= 0 ? (float)(S.dy[i2] - S.dy[i]) : 0.0f;
    }
}

template <class R, int TEAM>
__device__ __forceinline__ void reset_env(const StepParams<R>& p, Slot<R, TEAM>& S, int e, int t, int n_new, int spawn,
                                          uint32_t episode, R* own_z) {
    const long long env_id = p.env_off + e;
    if (t < p.NC) {
        R x, y, z;
        reset_drone(p, (long long)e * p.NC + t, t, n_new, x, y, z);
        if (p.physics != CH_PHYS_PYB) {   // last_clipped_action, rpy_rates = 0 (_housekeeping, BaseAviary.py:565, 581-582)
            const long long DS = (long long)p.E * p.NC;
#pragma unroll
            for (int c = 0; c < kPhysComps; ++c) p.phys[c * DS + (long long)e * p.NC + t] = R(0);
        }
        S.dx[t] = x; S.dy[t] = y;
        if constexpr (sizeof(R) == 4) { S.dxd[t] = x; S.dyd[t] = y; }   // exact: multiples of 1.75
        *own_z = z;
    }
    if (t < p.M) {
        R x, y, vx, vy;
        reset_cow(p, (long long)e * p.M + t, env_id, t, spawn, episode, x, y, vx, vy);
        S.cx[t] = x; S.cy[t] = y; S.cvx[t] = vx; S.cvy[t] = vy;
        if constexpr (sizeof(R) == 4) {   // the spawn position in f64
            const double* tab = p.spawn + ((long long)spawn * p.n_cows + t) * 2;
            S.cxd[t] = tab[0]; S.cyd[t] = tab[1];
        }
    }
}

template <class R, int TEAM, bool RESET_ONLY, int MODE, bool PHYS = false>
__global__ __launch_bounds__(64) void k_env(StepParams<R> p) {
    constexpr int EPB = 64 / TEAM;
    __shared__ Slot<R, TEAM> slots[EPB];
    const int slot = threadIdx.x / TEAM, t = threadIdx.x % TEAM;
    const int e = blockIdx.x * EPB + slot;
    const bool valid = e < p.E;
    Slot<R, TEAM>& S = slots[slot];
    const long long E = p.E;
    const long long DS = E * p.NC, CS = E * p.M;
    constexpr bool marl = MODE == 1;   // CTDE and MARL are separate instantiations (smaller code)
    constexpr bool MIX = sizeof(R) == 4;   // f32 mode: positions, centroids and prev_cent in f64 (StepParams::pos64)
    const int m_obs = p.M < 16 ? p.M : 16;
    const int cat_off = marl ? 18 : 34;

    // ---- env scalars (broadcast loads) -------------------------------------------------------
    int n = 0, sc = 0, scA = 0, has_prev = 0, level = 0, tally = 0, spawn = 0, active = 0, episode = 0, stepi = 0;
    double prev = 0;   // prev_cent_dists: f64 in both modes (f32 mode: StepParams::prev64)
    R clock = 0;
    if (valid) {
        n = p.envi[0 * E + e]; sc = p.envi[1 * E + e]; scA = p.envi[2 * E + e]; has_prev = p.envi[3 * E + e];
        level = p.envi[4 * E + e]; tally = p.envi[5 * E + e]; spawn = p.envi[6 * E + e]; active = p.envi[7 * E + e];
        episode = p.envi[8 * E + e]; stepi = p.envi[9 * E + e];
        prev = MIX ? p.prev64[e] : (double)p.envr[0 * E + e]; clock = p.envr[1 * E + e];
    }
    if (t == 0) { S.done = 0; S.reset = 0; S.n = n; }
    // metric accumulators are fetched now so their latency hides behind the physics
    double mt[kMetricRows];
    if (!RESET_ONLY && valid && t == 0) {
#pragma unroll
        for (int r = 0; r < kMetricRows; ++r) mt[r] = p.metrics[r * E + e];
    }

    R own_z = 0;
    R rpy[3] = {0, 0, 0}, dv[3] = {0, 0, 0}, dw[3] = {0, 0, 0};
    bool do_reset = false;

    if (!RESET_ONLY) {
        scA += 1;
        // ---- phase 1: drones (lane k) and cattle (lane j) ----------------------------------------
        if (valid && t < n) {
            const long long di = (long long)e * p.NC + t;
            R pos[3] = {ld(p.drone, 0, DS, di), ld(p.drone, 1, DS, di), ld(p.drone, 2, DS, di)};
            double pd[3] = {0, 0, 0};
            if constexpr (MIX) {
#pragma unroll
                for (int c = 0; c < 3; ++c) { pd[c] = p.pos64[c * DS + di]; pos[c] = R(pd[c]); }
            }
            const R px0 = pos[0], py0 = pos[1];
            R q[4] = {ld(p.drone, 3, DS, di), ld(p.drone, 4, DS, di), ld(p.drone, 5, DS, di), ld(p.drone, 6, DS, di)};
            R v[3] = {ld(p.drone, 7, DS, di), ld(p.drone, 8, DS, di), ld(p.drone, 9, DS, di)};
            R w[3] = {ld(p.drone, 10, DS, di), ld(p.drone, 11, DS, di), ld(p.drone, 12, DS, di)};
            R pid[9], ql[4];
#pragma unroll
            for (int c = 0; c < 9; ++c) pid[c] = ld(p.drone, 13 + c, DS, di);
#pragma unroll
            for (int c = 0; c < 4; ++c) ql[c] = ld(p.drone, 22 + c, DS, di);   // Bullet's cached link frame
            float a[4];
            if (p.flags & CH_STEP_RANDOM_ACTIONS) {
                uint32_t c4[4] = {(uint32_t)stepi, 0u, (uint32_t)t, (uint32_t)(p.env_off + e)};
                philox(c4, p.k0, p.k1);
#pragma unroll
                for (int k = 0; k < 4; ++k) a[k] = (float)(c4[k] >> 8) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
                if (p.actions_out)
                    reinterpret_cast<float4*>(p.actions_out)[di] = make_float4(a[0], a[1], a[2], a[3]);
            } else {
                float4 a4 = reinterpret_cast<const float4*>(p.actions)[di];
                a[0] = a4.x; a[1] = a4.y; a[2] = a4.z; a[3] = a4.w;
            }
            if (marl && !((active >> t) & 1)) { a[0] = a[1] = a[2] = a[3] = 0.0f; }  // marl_wrapper.py:80-84
            R Rm[9];
            quat_to_mat(q, Rm);
            quat_to_euler(q, rpy);
            double rpm[4];
            if (!(p.phase_mask & 1)) {
                pid_vel(pos, q, v, Rm, rpy, a, R(p.dt_ctrl), pid, rpm, p.debug ? p.debug + di * 16 : nullptr);
                R zl[3] = {0, 0, 0};   // the cached link frame's z axis (link_lag)
                if (p.link_lag) quat_to_zcol(ql, zl);
                if constexpr (PHYS) {
                    const long long PS = (long long)p.E * p.NC;
                    R lr[4], rr[3];
#pragma unroll
                    for (int c = 0; c < 4; ++c) lr[c] = p.phys[c * PS + di];
#pragma unroll
                    for (int c = 0; c < 3; ++c) rr[c] = p.phys[(4 + c) * PS + di];
                    variant_substeps(p, slot * TEAM, p.NC, n, pos, q, v, w, rpm, lr, rr, MIX ? pd : nullptr, ql, zl, p.link_lag != 0);
#pragma unroll
                    for (int c = 0; c < 4; ++c) p.phys[c * PS + di] = lr[c];
#pragma unroll
                    for (int c = 0; c < 3; ++c) p.phys[(4 + c) * PS + di] = rr[c];
                } else {
                    for (int s = 0; s < p.substeps; ++s)
                        drone_substep(pos, q, v, w, rpm, R(p.dt), R(p.damping), p.torque_world != 0, p.gyro != 0,
                                      NoExtraForces(), MIX ? pd : nullptr, ql, zl, p.link_lag != 0);
                }
            }
            R* D = p.drone;
#pragma unroll
            for (int c = 0; c < 4; ++c) D[(22 + c) * DS + di] = ql[c];
            if (p.evald) p.evald[di] = eval_distance_step(p.evald[di], sc == 0, px0, py0, pos[0], pos[1]);
            D[0 * DS + di] = pos[0]; D[1 * DS + di] = pos[1]; D[2 * DS + di] = pos[2];
            if constexpr (MIX) {
#pragma unroll
                for (int c = 0; c < 3; ++c) p.pos64[c * DS + di] = pd[c];
                S.dxd[t] = pd[0]; S.dyd[t] = pd[1];
            }
            D[3 * DS + di] = q[0]; D[4 * DS + di] = q[1]; D[5 * DS + di] = q[2]; D[6 * DS + di] = q[3];
            D[7 * DS + di] = v[0]; D[8 * DS + di] = v[1]; D[9 * DS + di] = v[2];
            D[10 * DS + di] = w[0]; D[11 * DS + di] = w[1]; D[12 * DS + di] = w[2];
#pragma unroll
            for (int c = 0; c < 9; ++c) D[(13 + c) * DS + di] = pid[c];
            quat_to_euler(q, rpy);
            S.dx[t] = pos[0]; S.dy[t] = pos[1];
            own_z = pos[2];
#pragma unroll
            for (int k = 0; k < 3; ++k) { dv[k] = v[k]; dw[k] = w[k]; }
            drone_obs_prep(S, t, n, own_z, rpy, dv, dw);
        }
        R cvx = 0, cvy = 0;
        if (valid && t < p.M) {
            const long long ci = (long long)e * p.M + t;
            R x = ld(p.cattle, 0, CS, ci), y = ld(p.cattle, 1, CS, ci);
            cvx = ld(p.cattle, 2, CS, ci); cvy = ld(p.cattle, 3, CS, ci);
            const R dt = R(p.dt);
            double xd = 0, yd = 0;
            if constexpr (MIX) { xd = p.cpos64[ci]; yd = p.cpos64[CS + ci]; }
            // no p.stepSimulation under Physics.DYN: the cattle bodies keep their positions (BaseAviary.py:447-448)
            if (!PHYS || (p.physics != CH_PHYS_DYN && p.physics != CH_PHYS_DYN_RK4))
                for (int s = 0; s < p.substeps; ++s) {
                    if constexpr (MIX) { xd += (double)(cvx * dt); yd += (double)(cvy * dt); }
                    else { x += cvx * dt; y += cvy * dt; }
                }
            if constexpr (MIX) {
                x = R(xd); y = R(yd);
                p.cpos64[ci] = xd; p.cpos64[CS + ci] = yd;
                S.cxd[t] = xd; S.cyd[t] = yd;
            }
            p.cattle[0 * CS + ci] = x; p.cattle[1 * CS + ci] = y;
            S.cx[t] = x; S.cy[t] = y; S.cvx[t] = cvx; S.cvy[t] = cvy;
        }
        __syncthreads();

        // ---- phase 2: flocking every second step (BaseAviary.py:454-455, 1352-1400) -------------
        const bool flock = (scA % 2) == 0 && !(p.phase_mask & 2);
        if (valid && flock && t < p.M) {
            const R C2A = R(2 * 1.7320508075688772), C2B = R(2 * 4.47213595499958), C1G = R(5),
                    C2G = R(0.2 * 2.23606797749979);
            const R ra_a = sigma_norm_n(R(1.2)), da_a = ra_a, ra_b = sigma_norm_n(R(1.0)), da_b = ra_b;
            const R qix = S.cx[t], qiy = S.cy[t], pix = cvx, piy = cvy;
            R ux = 0, uy = 0, gx = 0, gy = 0, cxx = 0, cyy = 0;
            int nb = 0;
            // alpha term over the herd (flockUtils.py:237-258); |qj - qi| of the adjacency test is the
            // same number the gradient term needs, so it is computed once
            for (int j = 0; j < p.M; ++j) {
                if (j == t) continue;
                const R zx = S.cx[j] - qix, zy = S.cy[j] - qiy;
                const R nrm = sqrt(zx * zx + zy * zy);
                if (!(nrm <= R(999))) continue;
                ++nb;
                pair_terms_n(nrm, zx, zy, pix, piy, S.cvx[j], S.cvy[j], ra_a, da_a, gx, gy, cxx, cyy);
            }
            if (nb > 0) { ux = C2A * gx + C2A * cxx; uy = C2A * gy + C2A * cyy; }
            // delta (shepherd) term (271-317) and predator avoidance (343-348) share |y_k - q_i|
            R ddx = 0, ddy = 0, sx = 0, sy = 0;
            gx = gy = cxx = cyy = 0;
            nb = 0;
            for (int k = 0; k < n; ++k) {
                const R yx = S.dx[k], yy = S.dy[k];
                const R ex = yx - qix, ey = yy - qiy;
                const R dn = sqrt(ex * ex + ey * ey);
                if (dn <= R(999 + 2)) {
                    ++nb;
                    R difx = qix - yx, dify = qiy - yy;
                    R d = dn + R(1e-6);
                    R mu = d / R(1.0) < R(1.0) ? d / R(1.0) : R(1.0);
                    R akx = difx / d, aky = dify / d;
                    R P00 = R(1) - akx * akx, P01 = R(0) - akx * aky, P10 = R(0) - aky * akx, P11 = R(1) - aky * aky;
                    R qkx = mu * qix + (R(1) - mu) * yx, qky = mu * qiy + (R(1) - mu) * yy;
                    R pkx = mu * (P00 * pix + P01 * piy), pky = mu * (P10 * pix + P11 * piy);
                    pair_terms(qix, qiy, pix, piy, qkx, qky, pkx, pky, ra_b, da_b, gx, gy, cxx, cyy);
                }
                if (dn <= R(1.1)) {
                    R d3 = cube(dn);
                    sx += R(-650000.0) * ex / d3;
                    sy += R(-650000.0) * ey / d3;
                }
            }
            if (nb > 0) { ddx = C2B * gx + C2B * cxx; ddy = C2B * gy + C2B * cyy; }
            ddx += sx; ddy += sy;
            R gmx = -C1G * sigma_1(qix - R(1)) - C2G * pix, gmy = -C1G * sigma_1(qiy - R(1)) - C2G * piy;
            R qx = (ux + ddx) + gmx, qy = (uy + ddy) + gmy;
            const R dt_sqr = R(0.05 * 0.05);
            R vx = pix + qx * dt_sqr, vy = piy + qy * dt_sqr;
            R sp = norm2(vx, vy);
            if (sp > R(kMaxVelCattle)) { R f = R(kMaxVelCattle) / sp; vx *= f; vy *= f; }
            cvx = vx; cvy = vy;
            const long long ci = (long long)e * p.M + t;
            p.cattle[2 * CS + ci] = vx; p.cattle[3 * CS + ci] = vy;
        }
        __syncthreads();
        if (valid && flock && t < p.M) { S.cvx[t] = cvx; S.cvy[t] = cvy; }

        // ---- phase 3: per-drone reward terms (lane i) and per-cow herded flags (lane j) -----------
        const bool task = !(p.phase_mask & 4);
        if (valid && task && t < n) {
            const int i = t;
            R m1 = R(INFINITY), m2 = R(INFINITY);
            uint8_t fl = 0;
            bool iso = true;
#pragma unroll 4
            for (int j = 0; j < n; ++j) {
                if (j == i) continue;
                R d = norm2(S.dx[j] - S.dx[i], S.dy[j] - S.dy[i]);
                if (d != d) fl |= F_NAN;
                if (d < m1) { m2 = m1; m1 = d; } else if (d < m2) m2 = d;
                if (d < R(kCollision)) fl |= F_COLL;
                if (!(d > R(kMaxFormation))) iso = false;
            }
            if (iso) fl |= F_ISO;
            if (fabs(own_z - R(kTargetAlt)) > R(kTargetAlt * 0.6)) fl |= F_ALT;
            R best = R(INFINITY);
#pragma unroll 4
            for (int j = 0; j < p.M; ++j) {
                R d = norm2(S.cx[j] - S.dx[i], S.cy[j] - S.dy[i]);
                if (d < best) best = d;
            }
            S.pa[i] = m1; S.pb[i] = m2; S.pcat[i] = best; S.dflags[i] = fl;
            const Level& L = kLevels[level];
            S.sa[i] = simple_spacing(m1, L); S.sb[i] = simple_spacing(m2, L);
            S.ca[i] = complex_spacing(m1, L); S.cb[i] = complex_spacing(m2, L);
            S.scat[i] = cattle_spacing(best, R(p.cs_cc));
            neighbour_obs(S, i, n);
        }
        if (valid && task && t < p.M) {
            // evaluate_herding_effectiveness (evaluation.py:100-138)
            R px = S.cx[t], py = S.cy[t];
            int wn = 0;
            for (int i = 0; i < n; ++i) {
                int i2 = (i + 1 == n) ? 0 : i + 1;
                R x1 = S.dx[i], y1 = S.dy[i], x2 = S.dx[i2], y2 = S.dy[i2];
                R il = (x2 - x1) * (py - y1) - (px - x1) * (y2 - y1);
                if (y1 <= py) { if (y2 > py && il > R(0)) wn += 1; }
                else { if (y2 <= py && il < R(0)) wn -= 1; }
            }
            S.herded[t] = wn != 0;
        }
        __syncthreads();

        // ---- phase 4: order-dependent task bookkeeping on lane 0 ----------------------------------
        if (valid && task && t == 0) {
            // centroids and their distance in f64 (f32 mode: from the f64 positions)
            double scxd = 0, scyd = 0, sdx = 0, sdy = 0;
            int herded = 0;
#pragma unroll 8
            for (int j = 0; j < p.M; ++j) {
                scxd += MIX ? S.cxd[j] : (double)S.cx[j]; scyd += MIX ? S.cyd[j] : (double)S.cy[j];
                herded += S.herded[j];
            }
#pragma unroll 4
            for (int i = 0; i < n; ++i) { sdx += MIX ? S.dxd[i] : (double)S.dx[i]; sdy += MIX ? S.dyd[i] : (double)S.dy[i]; }
            scxd /= double(p.M); scyd /= double(p.M); sdx /= double(n); sdy /= double(n);
            const double ex = sdx - scxd, ey = sdy - scyd;
            const double cent = sqrt(ex * ex + ey * ey + 0.0 * 0.0);
            const R centR = R(cent), scx = R(scxd), scy = R(scyd);
            const R eff = R((double)herded / p.M * 100);
            R ms = R(INFINITY);
            bool anynan = false;
            uint8_t any_alt = 0, any_coll = 0, any_iso = 0;
            for (int i = 0; i < n; ++i) {
                if (S.pa[i] < ms) ms = S.pa[i];
                anynan |= (S.dflags[i] & F_NAN) != 0;
                any_alt |= S.dflags[i] & F_ALT; any_coll |= S.dflags[i] & F_COLL; any_iso |= S.dflags[i] & F_ISO;
            }
            if (anynan) ms = R(NAN);
            const double max_step = (0.3 * kMaxSpeedKmh * (1000.0 / 3600.0)) / double(p.ctrl_freq);
            const bool time_up = (double)sc / p.ctrl_freq > p.episode_len;
            int done = 0;
            double ret = 0;
            int n_term = 0, n_trunc = 0, n_nan = 0;
            if constexpr (!marl) {
                // CattleAviary._computeReward (CattleAviary.py:213-332)
                const Level& L = kLevels[level];
                R sp_simple = 0, sp_complex = 0, per_sp[kNMax], msp = 0, mcat = 0, cat = 0;
                for (int i = 0; i < n; ++i) {
                    per_sp[i] = 0;
                    R dd[2] = {S.pa[i], S.pb[i]}, rs[2] = {S.sa[i], S.sb[i]}, rc[2] = {S.ca[i], S.cb[i]};
                    for (int k = 0; k < 2; ++k) {
                        if (!p.compat && !(dd[k] < R(INFINITY))) continue;
                        sp_complex += rc[k]; sp_simple += rs[k]; per_sp[i] += (rc[k] + rs[k]) / R(2.0);
                    }
                }
                sp_complex /= R(n * 2.0); sp_simple /= R(n * 2.0);
                R approach = 0;
                if (has_prev) approach = R(clip(((prev - cent) / (max_step + 1e-6)) * 5.0, -1.0, 1.0));
                prev = cent; has_prev = 1;
                for (int i = 0; i < n; ++i) cat += S.scat[i];
                cat /= R(n);
                R rg = sp_simple * R(L.w_simple) + sp_complex * R(L.w_complex) + R(0.1) * R(L.w_survival) +
                       approach * R(L.w_approach) + (eff / R(100)) * R(L.w_eff) + cat * R(L.w_cattle);
                for (int i = 0; i < n; ++i) { msp += per_sp[i]; mcat += S.scat[i]; }
                msp /= R(n); mcat /= R(n);
                R tot = 0;
                for (int i = 0; i < n; ++i) tot += rg + R(0.5) * ((per_sp[i] - msp) + (S.scat[i] - mcat));
                R rew = tot / R(n);
                const R inc = R(1.0 / 240);
                bool te = term_call(kLevels, level, clock, inc, ms, centR, eff);
                if (te) curriculum_success(kLevels, level, tally);
                bool te2 = term_call(kLevels, level, clock, inc, ms, centR, eff);
                bool tr = any_alt || any_coll || any_iso || cent > kMissionBoundary || time_up;
                p.reward[e] = (float)rew;
                p.term[e] = te2; p.trunc[e] = tr;
                done = te2 || tr;
                ret = (double)rew;
                n_term = te2; n_trunc = tr; n_nan = rew != rew;
            } else {
                // MARLCattleAviary._computeReward / _computeTerminated / _computeTruncated in the order
                // env.step (rllib_envs/BaseAviary.py:425-431) and the wrapper (marl_wrapper.py:104-113) call them
                const R inc = R(1.0) / R(p.ctrl_freq);
                const int lvl0 = level;
                R rout[kNMax];
                uint8_t tout[kNMax], trout[kNMax];
                // the wrapper sees step_counter after env.step's += 1 (rllib_envs/BaseAviary.py:436)
                const bool time_up_w = (double)(sc + 1) / p.ctrl_freq > p.episode_len;
                auto trunc_i = [&](int i, bool tu) -> bool {
                    return (S.dflags[i] & (F_ALT | F_COLL | F_ISO)) || cent > kMissionBoundary || tu;
                };
                auto reward_i = [&](int i, bool tu) -> R {
                    const Level& L = kLevels[level];
                    R a = S.pa[i], b = S.pb[i];
                    R sa, sb, ca, cb;
                    if (level == lvl0) { sa = S.sa[i]; sb = S.sb[i]; ca = S.ca[i]; cb = S.cb[i]; }
                    else { sa = simple_spacing(a, L); sb = simple_spacing(b, L); ca = complex_spacing(a, L); cb = complex_spacing(b, L); }
                    R simple = (sa + sb) / R(2), cplx = (ca + cb) / R(2);
                    if (!p.compat) {
                        if (!(b < R(INFINITY))) { simple = sa; cplx = ca; }
                        if (!(a < R(INFINITY))) { simple = 0; cplx = 0; }
                    }
                    R r = 0;
                    r += simple * R(L.w_simple);
                    r += cplx * R(L.w_complex);
                    r += R(0.1) * R(L.w_survival);
                    double change = has_prev ? prev - cent : 0.0;
                    prev = cent; has_prev = 1;
                    r += R(clip((change / (max_step + 1e-6)) * 5.0, -1.0, 1.0)) * R(L.w_approach);
                    r += (eff / R(100)) * R(L.w_eff);
                    r += S.scat[i] * R(L.w_cattle);
                    if (term_call(kLevels, level, clock, inc, ms, centR, eff)) {
                        // _endOfEpisodeReward (MARLCattleAviary.py:183-241)
                        R eor = marl_end_of_episode(kLevels, level, a, b, centR, eff, norm2(scx - S.dx[i], scy - S.dy[i]), n);
                        r += eor;
                        curriculum_success(kLevels, level, tally);
                    } else if (trunc_i(i, tu)) {
                        r -= R(50);
                    }
                    return r;
                };
                R r1[kNMax];
                uint8_t d1[kNMax];
                for (int i = 0; i < n; ++i) r1[i] = reward_i(i, time_up);
                for (int i = 0; i < n; ++i) d1[i] = term_call(kLevels, level, clock, inc, ms, centR, eff);
                for (int i = 0; i < p.NC; ++i) { rout[i] = R(NAN); tout[i] = 0; trout[i] = 0; }
                if (p.marl_wrapper) {
                    for (int i = 0; i < n; ++i) {
                        if (!((active >> i) & 1)) continue;
                        rout[i] = reward_i(i, time_up_w);
                        tout[i] = term_call(kLevels, level, clock, inc, ms, centR, eff);
                        trout[i] = trunc_i(i, time_up_w);
                    }
                    int live = 0;
                    for (int i = 0; i < n; ++i)
                        if (((active >> i) & 1) && tout[i]) active &= ~(1 << i);
                    for (int i = 0; i < n; ++i) live += (active >> i) & 1;
                    done = live == 0;
                } else {
                    // bare env.step dicts; done = done["__all__"] = all(done.values())
                    done = 1;
                    for (int i = 0; i < n; ++i) {
                        rout[i] = r1[i]; tout[i] = d1[i]; trout[i] = trunc_i(i, time_up);
                        done &= tout[i];
                    }
                }
                for (int i = 0; i < p.NC; ++i) {
                    p.reward[(long long)e * p.NC + i] = (float)rout[i];
                    p.term[(long long)e * p.NC + i] = tout[i];
                    p.trunc[(long long)e * p.NC + i] = trout[i];
                    if (i < n && rout[i] == rout[i]) ret += (double)rout[i];
                    n_term += tout[i]; n_trunc += trout[i];
                    if (i < n && ((active >> i) & 1 || tout[i]) && rout[i] != rout[i]) n_nan += 1;
                }
            }
            sc += marl ? 1 : p.substeps;
            // metrics (rank-local accumulators; bench.py all-reduces them)
            mt[CH_METRIC_STEPS] += 1;
            mt[CH_METRIC_TERMINATED] += n_term;
            mt[CH_METRIC_TRUNCATED] += n_trunc;
            mt[CH_METRIC_NAN_REWARDS] += n_nan;
            mt[CH_METRIC_EFFECTIVENESS_SUM] += (double)eff;
            mt[kMetricCurReturn] += ret;
            mt[kMetricCurLen] += 1;
            if (done) {
                if (p.episode_stats) { p.episode_stats[2 * e] = mt[kMetricCurReturn]; p.episode_stats[2 * e + 1] = mt[kMetricCurLen]; }
                mt[CH_METRIC_EPISODES] += 1;
                mt[CH_METRIC_RETURN_SUM] += mt[kMetricCurReturn];
                mt[CH_METRIC_LENGTH_SUM] += mt[kMetricCurLen];
                mt[kMetricCurReturn] = 0;
                mt[kMetricCurLen] = 0;
            }
#pragma unroll
            for (int r = 0; r < kMetricRows; ++r) p.metrics[r * E + e] = mt[r];
            S.done = done;
            S.reset = done && (p.flags & CH_STEP_AUTORESET);
        }
        __syncthreads();
        do_reset = valid && S.reset;
        if (valid && t == 0) {
            if (p.agent_active && !S.reset) {
                for (int i = 0; i < p.NC; ++i) p.agent_active[(long long)e * p.NC + i] = (active >> i) & 1;
            }
        }
        // terminal observation of envs about to auto-reset (SB3 info["terminal_observation"])
        if (do_reset && p.terminal_obs)
            write_obs(p.terminal_obs + (long long)e * p.rows * 86, p.rows, S, t, m_obs, cat_off);
        __syncthreads();
    } else {
        do_reset = valid && (p.reset_mask == nullptr || p.reset_mask[e] != 0);
    }

    // ---- auto-reset / reset ------------------------------------------------------------------
    if (do_reset && t == 0) {
        reset_scalars(p, e, n, sc, scA, spawn, episode, active, has_prev, prev, clock);
        S.n = n; S.spawn = spawn; S.episode = episode;
    }
    __syncthreads();
    if (do_reset) {
        n = S.n; spawn = S.spawn; episode = S.episode;   // lane 0 drew them; every lane needs them
        reset_env(p, S, e, t, n, spawn, (uint32_t)(episode - 1), &own_z);
        if (t < n) {
            const R qid[4] = {0, 0, 0, 1};
            R rpy0[3], zero3[3] = {0, 0, 0};
            quat_to_euler(qid, rpy0);  // identity quaternion (getQuaternionFromEuler([0,0,0]))
            drone_obs_prep(S, t, n, own_z, rpy0, zero3, zero3);
        }
        if (t == 0) {
            if (p.reset_happened) p.reset_happened[e] = 1;
            if (p.agent_active)
                for (int i = 0; i < p.NC; ++i) p.agent_active[(long long)e * p.NC + i] = (active >> i) & 1;
        }
    } else if (valid && t == 0 && p.reset_happened) {
        p.reset_happened[e] = 0;
    }
    __syncthreads();
    if (do_reset && t < n) neighbour_obs(S, t, n);
    __syncthreads();

    // ---- observation + scalars back to HBM --------------------------------------------------
    const bool write = valid && (!RESET_ONLY || do_reset);
    if (write && !(p.phase_mask & 8)) write_obs(p.obs + (long long)e * p.rows * 86, p.rows, S, t, m_obs, cat_off);
    if (write && t == 0) {
        if (p.stale) p.stale[e] = 1;   // this kernel does not keep the v2 step's Euler-angle cache
        // every block this kernel writes is written in full
        if (p.obs_tag) p.obs_tag[e] = (p.phase_mask & 8) ? 0ull : (unsigned long long)(uintptr_t)p.obs;
        p.envi[0 * E + e] = n; p.envi[1 * E + e] = sc; p.envi[2 * E + e] = scA; p.envi[3 * E + e] = has_prev;
        p.envi[4 * E + e] = level; p.envi[5 * E + e] = tally; p.envi[6 * E + e] = spawn; p.envi[7 * E + e] = active;
        p.envi[8 * E + e] = episode;
        if (!RESET_ONLY) p.envi[9 * E + e] = stepi + 1;   // ch_step calls on this env (Philox action counter)
        p.envr[0 * E + e] = R(prev); p.envr[1 * E + e] = clock;
        if constexpr (MIX) p.prev64[e] = prev;
    }
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
template <class R, bool RESET_ONLY, int MODE>
static void launch_mode(const StepParams<R>& p, int team, hipStream_t st) {
    int epb = 64 / team;
    dim3 grid((p.E + epb - 1) / epb), block(64);
    if constexpr (!RESET_ONLY) {
        if (p.physics != CH_PHYS_PYB) {   // variant instantiations (BaseAviary.py:420-450)
            switch (team) {
                case 16: hipLaunchKernelGGL((k_env<R, 16, false, MODE, true>), grid, block, 0, st, p); break;
                case 32: hipLaunchKernelGGL((k_env<R, 32, false, MODE, true>), grid, block, 0, st, p); break;
                default: hipLaunchKernelGGL((k_env<R, 64, false, MODE, true>), grid, block, 0, st, p); break;
            }
            return;
        }
    }
    switch (team) {
        case 16: hipLaunchKernelGGL((k_env<R, 16, RESET_ONLY, MODE>), grid, block, 0, st, p); break;
        case 32: hipLaunchKernelGGL((k_env<R, 32, RESET_ONLY, MODE>), grid, block, 0, st, p); break;
        default: hipLaunchKernelGGL((k_env<R, 64, RESET_ONLY, MODE>), grid, block, 0, st, p); break;
    }
}

template <class R, bool RESET_ONLY>
static hipError_t launch_team(const StepParams<R>& p, int team, hipStream_t st) {
    if (p.mode == 1) launch_mode<R, RESET_ONLY, 1>(p, team, st);
    else launch_mode<R, RESET_ONLY, 0>(p, team, st);
    return hipGetLastError();
}

template <class R>
hipError_t launch_step(const StepParams<R>& p, int team, hipStream_t st) { return launch_team<R, false>(p, team, st); }
template <class R>
hipError_t launch_reset(const StepParams<R>& p, int team, hipStream_t st) { return launch_team<R, true>(p, team, st); }

template hipError_t launch_step<double>(const StepParams<double>&, int, hipStream_t);
template hipError_t launch_step<float>(const StepParams<float>&, int, hipStream_t);
template hipError_t launch_reset<double>(const StepParams<double>&, int, hipStream_t);
template hipError_t launch_reset<float>(const StepParams<float>&, int, hipStream_t);

}  // namespace ch
