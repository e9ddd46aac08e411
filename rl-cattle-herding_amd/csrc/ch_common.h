// ch_common.h — per-env task bookkeeping and reset pieces shared by the step kernels.
//
// Restates the order-dependent parts of the reference's env.step(): curriculum tally
// (curriculum_learning.py:200-219), _computeTerminated (CattleAviary.py:422-492,
// MARLCattleAviary.py:246-321) and the reset bookkeeping of BaseAviary.reset / _housekeeping
// (BaseAviary.py:280-331, 547-700).  Paths relative to gym_pybullet_drones/.
#pragma once
#include "ch_device.h"
#include "ch_internal.h"

namespace ch {

// curriculum_learning.py:200-219
__device__ __forceinline__ void curriculum_success(const Level* LT, int& level, int& tally) {
    tally += 1;
    const bool up = tally >= LT[level].required_tally;   // (selects: the env lanes of a wave differ)
    tally = up ? 0 : tally;
    level = up ? min(level + 1, 7) : level;
}

// _computeTerminated (CattleAviary.py:422-492; MARLCattleAviary.py:246-321)
// Branch-free: every level's test is evaluated and the level selects (the same operations; the env lanes of a
// wave sit at different levels, so the if-chain ran most of its arms anyway, plus the exec-mask bookkeeping).
template <class R>
__device__ __forceinline__ bool term_call_L(const Level& L, int level, R& clock, R clock_inc, R min_spacing, R cent,
                                            R eff) {
    const R up = R(L.desired) + R(L.desired) * R(L.tol), lo = R(L.desired) - R(L.desired) * R(L.tol);
    const bool l01 = level == 0 || level == 1;
    const bool in01 = min_spacing < up && min_spacing > lo;
    const R held = clock + clock_inc;
    const bool t01 = l01 && in01 && held >= R(L.hold);
    clock = l01 ? (in01 ? held : R(0)) : clock;
    const bool t23 = (level == 2 || level == 3) && cent < R(L.approach_min);
    const bool t46 = (level == 4 || level == 6) && eff > R(L.min_eff);
    const R cup = R(L.cattle_desired) + R(L.cattle_desired) * R(L.cattle_tol);
    const R clo = R(L.cattle_desired) - R(L.cattle_desired) * R(L.cattle_tol);
    const bool t5 = level == 5 && eff > R(L.min_eff) && min_spacing < cup && min_spacing > clo;
    return t01 || t23 || t46 || t5;
}
template <class R>
__device__ __forceinline__ bool term_call(const Level* LT, int level, R& clock, R clock_inc, R min_spacing, R cent, R eff) {
    return term_call_L(LT[level], level, clock, clock_inc, min_spacing, cent, eff);
}

// NUM_DRONES of the episode that starts after `episode` resets (BaseAviary.py:307: random.randint over
// the curriculum's [min, max]); U from Philox keyed (seed, env id, episode, 0)
template <class R>
__device__ __forceinline__ int reset_draw_n(const StepParams<R>& p, int episode, long long env_id) {
    int span = p.max_drones - p.min_drones + 1;
    int nn = p.min_drones;
    if (span > 1) {
        double u = philox_uniform53(p.k0, p.k1, (uint32_t)episode, 0, (uint32_t)env_id);
        nn = p.min_drones + (int)(u * span);
        if (nn > p.max_drones) nn = p.max_drones;
    }
    return nn;
}

// env-scalar part of a reset: NUM_DRONES draw (BaseAviary.py:307), counters (306, 557), spawn index
// advanced before use (600-606); prev_cent_dists / spacing clock persist in compat mode (CattleAviary.py:89)
template <class R, class PR>
__device__ __forceinline__ void reset_scalars(const StepParams<R>& p, int e, int& n, int& sc, int& scA, int& spawn,
                                              int& episode, int& active, int& has_prev, PR& prev, R& clock,
                                              int drawn = -1) {
    // drawn >= 0: the caller's draw for this episode (v2 takes it ahead of the reset decision)
    const int nn = drawn >= 0 ? drawn : p.reset_n ? p.reset_n[e] : reset_draw_n(p, episode, p.env_off + e);
    n = nn;
    sc = 0; scA = 0;
    spawn += 1;
    if (spawn >= p.n_scen) spawn = 0;
    active = (1 << nn) - 1;
    if (!p.compat) { has_prev = 0; prev = 0; clock = 0; }
    episode += 1;
}

// initial position of constructor drone k of an episode with n_new drones (initialize_drone_positions,
// BaseAviary.py:251-277); R = double also in f32 mode (the f64 position state)
template <class R>
__device__ __forceinline__ void reset_drone_xyz(int k, int n_new, R& x, R& y, R& z) {
    x = 0; y = 0; z = 0;
    if (k < n_new) {
        if (n_new <= 4) { x = R(k * 1.75); y = 0; }
        else {
            int r1 = n_new / 2;
            if (k < r1) { x = R(k * 1.75); y = 0; } else { x = R((k - r1) * 1.75); y = R(1.75); }
        }
        z = R(kTargetAlt);
    }
}

// the reset drone's state in the SoA arrays: position, identity attitude, zero velocities; the PID state
// persists across resets in compat mode (the reference's DSLPIDControl objects are created once,
// BaseRLAviary.py:80)
template <class R>
__device__ __forceinline__ void reset_drone_store(const StepParams<R>& p, long long di, double x, double y, double z) {
    const long long DS = (long long)p.E * p.NC;
    R* D = p.drone;
    if (p.evald) p.evald[di] = 0;   // episode_drone_distances: (0, 0) -- _housekeeping zeroes self.pos (BaseAviary.py:567, 683-688)
    D[0 * DS + di] = R(x); D[1 * DS + di] = R(y); D[2 * DS + di] = R(z);
    if (p.pos64) { p.pos64[0 * DS + di] = x; p.pos64[1 * DS + di] = y; p.pos64[2 * DS + di] = z; }
    D[3 * DS + di] = 0; D[4 * DS + di] = 0; D[5 * DS + di] = 0; D[6 * DS + di] = 1;
    // loadURDF: the links' cached transforms at the spawn attitude
    D[22 * DS + di] = 0; D[23 * DS + di] = 0; D[24 * DS + di] = 0; D[25 * DS + di] = 1;
#pragma unroll
    for (int c = 7; c < 13; ++c) D[c * DS + di] = 0;
    if (!p.compat) {
#pragma unroll
        for (int c = 13; c < 22; ++c) D[c * DS + di] = 0;
    }
}

// initial pose of constructor drone k, written to the SoA state; returns x, y, z
template <class R>
__device__ __forceinline__ void reset_drone(const StepParams<R>& p, long long di, int k, int n_new, R& x, R& y, R& z) {
    double xd, yd, zd;
    reset_drone_xyz(k, n_new, xd, yd, zd);
    reset_drone_store(p, di, xd, yd, zd);
    x = R(xd); y = R(yd); z = R(zd);
}

// velocity of cow j of a reset env: angle pi(2U-1) (BaseAviary.py:631-632), U from Philox keyed
// (seed, env id, episode, 1 + j), or the host's replay of the reference's own draws (ch_reset_with,
// cattleherd/seeded.py)
template <class R>
__device__ __forceinline__ void reset_cow_vel(const StepParams<R>& p, long long ci, long long env_id, int j,
                                              uint32_t episode, R& vx, R& vy) {
    if (p.reset_vel) {
        vx = R(p.reset_vel[2 * ci]); vy = R(p.reset_vel[2 * ci + 1]);
    } else {
        double u = philox_uniform53(p.k0, p.k1, episode, 1 + j, (uint32_t)env_id);
        double ang = kPi * (2 * u - 1);
        double sa, ca;
        sincos_pi(ang, &sa, &ca);   // |ang| <= pi
        vx = R(kMaxVelCattle * ca); vy = R(kMaxVelCattle * sa);
    }
}
template <class R>
__device__ __forceinline__ void reset_cow_store(const StepParams<R>& p, long long ci, double x, double y, R vx, R vy) {
    const long long CS = (long long)p.E * p.M;
    p.cattle[0 * CS + ci] = R(x); p.cattle[1 * CS + ci] = R(y); p.cattle[2 * CS + ci] = vx; p.cattle[3 * CS + ci] = vy;
    if (p.cpos64) { p.cpos64[0 * CS + ci] = x; p.cpos64[1 * CS + ci] = y; }
}

// cow j of a reset env at spawn position (x0, y0) (already looked up in the scenario table)
template <class R>
__device__ __forceinline__ void reset_cow_at(const StepParams<R>& p, long long ci, long long env_id, int j, double x0,
                                             double y0, uint32_t episode, R& x, R& y, R& vx, R& vy) {
    x = R(x0); y = R(y0);
    reset_cow_vel(p, ci, env_id, j, episode, vx, vy);
    reset_cow_store(p, ci, x0, y0, vx, vy);
}

// cow j of a reset env: YAML scenario position, yaw/velocity angle pi(2U-1) (BaseAviary.py:600-637),
// U from Philox keyed (seed, env id, episode, 1 + j)
template <class R>
__device__ __forceinline__ void reset_cow(const StepParams<R>& p, long long ci, long long env_id, int j, int spawn,
                                          uint32_t episode, R& x, R& y, R& vx, R& vy) {
    const double* tab = p.spawn + ((long long)spawn * p.n_cows + j) * 2;
    reset_cow_at(p, ci, env_id, j, tab[0], tab[1], episode, x, y, vx, vy);
}


// update_evaluation_metrics' per-drone distance (BaseAviary.py:1415-1426; rllib twin): |last - current| * 1.7
// added to the episode's accumulator, last = the previous step's read-back position, or (0, 0) on an
// episode's first step (reset() zeroes last_drones_pos, BaseAviary.py:317).  Both components of the
// reference's 2-vector accumulator start at 0 and receive the same additions, so one number is kept.
template <class R>
__device__ __forceinline__ double eval_distance_step(double acc, bool first, R x0, R y0, R x1, R y1) {
    const R lx = first ? R(0) : x0, ly = first ? R(0) : y0;
    const R ex = lx - x1, ey = ly - y1;
    return acc + (double)(sqrt(ex * ex + ey * ey) * R(1.7));
}

// end-of-episode bonus of MARLCattleAviary._endOfEpisodeReward (MARLCattleAviary.py:183-241)
template <class R>
__device__ __forceinline__ R marl_end_of_episode_L(const Level& L2, int level, R a, R b, R cent, R eff, R dist_to_herd,
                                                  int n) {
    R eor = 0;
    if (level == 0 || level == 1) {
        R up = R(L2.desired) + R(L2.desired) * R(L2.tol), lo = R(L2.desired) - R(L2.desired) * R(L2.tol);
        if (a >= lo && a <= up && b >= lo && b <= up) eor += R(50.0) / R(n);
    } else if (level == 2 || level == 3) {
        if (cent < R(L2.approach_min)) eor += R(50.0);
    } else if (level == 4 || level == 6) {
        R wgt = clip(R(1.0) - dist_to_herd / R(10.0), R(0), R(1));
        eor += eff * R(2) * wgt;
    } else if (level == 5) {
        if (eff > R(L2.min_eff)) {
            R up = R(L2.cattle_desired) + R(L2.cattle_desired) * R(L2.cattle_tol);
            R lo = R(L2.cattle_desired) - R(L2.cattle_desired) * R(L2.cattle_tol);
            if (a >= lo && a <= up && b >= lo && b <= up) eor += R(50.0) / R(n);
        }
    }
    return eor;
}
template <class R>
__device__ __forceinline__ R marl_end_of_episode(const Level* LT, int level, R a, R b, R cent, R eff, R dist_to_herd,
                                                int n) {
    return marl_end_of_episode_L(LT[level], level, a, b, cent, eff, dist_to_herd, n);
}

}  // namespace ch
