// ch_internal.h — shared between the C-ABI implementation (ch_api.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cattleherd.h"

namespace ch {

constexpr int kNMax = 12;          // GLOBAL_MAX_NUM_DRONES (BaseAviary.py:112)
constexpr int kMMax = 64;          // cattle per env supported by the team mapping (TEAM <= 64)
constexpr int kDroneComps = 26;    // px py pz qx qy qz qw vx vy vz wx wy wz pid[9] qlag[4] (cached link frame)
constexpr int kCattleComps = 4;    // x y vx vy
constexpr int kPhysComps = 7;      // last_clipped_action[4] (drag input), DYN rpy_rates[3]
constexpr int kEnvReal = 2;        // prev_cent, clock
constexpr int kEnvInt = 10;        // n sc scA has_prev level tally spawn active episode step_index
constexpr int kMetricCurReturn = CH_METRIC_COUNT;      // running episode return
constexpr int kMetricCurLen = CH_METRIC_COUNT + 1;     // running episode length
constexpr int kMetricRows = CH_METRIC_COUNT + 2;

template <class R>
struct StepParams {
    int E, NC, M, mode, rows;
    int min_drones, max_drones, ctrl_freq, substeps, compat, torque_world, gyro, marl_wrapper;
    int link_lag;   // ch_config.link_lag: LINK_FRAME forces rotate by Bullet's cached link frame (drone comps 22-25)
    double episode_len, damping, dt_ctrl, dt;
    uint32_t k0, k1;
    long long env_off;
    double cs_cc;   // CattleSpacingRewardFunction continuation constant (host-evaluated)
    R* drone;       // [26][E][NC]
    R* rpy;         // v2: [3][E][NC] Euler angles of the stored quaternion (valid unless stale[e])
    // per-env device flags, read by the v2 step with its env's state (so a captured HIP graph sees state changes
    // made after capture) and cleared at its write-back: row 0 the Euler cache is stale, row 1 the obs block's
    // constant bytes are unknown; set by every other writer (v1, ch_reset, ch_set_state, invalidate)
    uint8_t* stale; // [2][E]
    // [E] the address of the obs buffer whose block of env e holds the env's constant-zero bytes (0: none): set
    // by every full-block writer (v1 step / reset, v2 step) to the buffer it wrote.  A v2 step into any other
    // buffer -- e.g. a graph captured on buffer A replayed after steps into B -- writes the env's block in full.
    unsigned long long* obs_tag;
    R* cattle;      // [4][E][M]
    R* envr;        // [2][E]
    int* envi;      // [10][E]
    double* metrics;  // [kMetricRows][E]
    const double* spawn;
    int n_scen, n_cows;
    const float* actions;
    float* actions_out;
    float* obs;
    float* reward;
    uint8_t* term;
    uint8_t* trunc;
    float* terminal_obs;
    uint8_t* agent_active;
    uint8_t* reset_happened;
    double* episode_stats;    // optional [E][2]: return and length of the episode that ended in this step
    const uint8_t* reset_mask;
    uint32_t flags;
    double* debug;  // optional [E][NC][16] per-drone intermediates (diagnostics only)
    int obs_full;   // v2: also store the constant-zero bytes of every obs block (ch_api.cpp: obs_zero_ptr)
    int phase_mask; // diagnostics only: skip phases (1 drones, 2 flock, 4 task, 8 obs) for time attribution
    int G, P;                 // v2: envs per workgroup, cow pairs per env
    const uint16_t* pairs;    // v2: [P] unordered cow pairs (i | j << 8) in tri() order
    long long* tstamp;        // diagnostics only: [grid][16] per-workgroup phase timestamps (ch__set_tstamp)
    int physics;              // CH_PHYS_* (v1 kernel only; ch_api.cpp selects v1 for the variants)
    double gnd_h_clip;        // GND_EFF_H_CLIP (BaseAviary.py:173)
    R* phys;                  // [kPhysComps][E][NC]
    int* err;                 // device error word of the handle (CH_DEVERR_* bits), read by ch_sync & co.
    int pw;                   // v2: per-wave env tables (V2Layout W = block / 64 - 1)
    int sep;                  // v2 shared tables: separate shepherd-term region (V2Layout sep)
    double* evald;            // optional [E][NC]: update_evaluation_metrics' per-drone episode distance
    const int* reset_n;       // optional (ch_reset_with): NUM_DRONES of each reset env instead of the Philox draw
    const double* reset_vel;  // optional (ch_reset_with): [E][M][2] cattle spawn velocities instead of Philox
    // f32 mode (CH_PREC_F32): the positions and the centroid distance carried in f64 (every other state component is
    // f32): drone xyz [3][E][NC], cattle xy [2][E][M], prev_cent [E].  The kernels integrate positions into them
    // (f32 increments, f64 sums) and form centroids and the approach delta from them; the f32 arrays keep the rounded
    // copies the f32 arithmetic reads.  NULL in f64 mode (the R arrays are the f64 state).
    double* pos64;
    double* cpos64;
    double* prev64;
};

// device error word bits (ch_api.cpp reports them as CH_ERR_DEVICE)
constexpr int CH_DEVERR_HANDOFF = 1;       // a v2 LDS hand-off wait ran out of spins (ch_step.hip lds_wait)
// diagnostics phase_mask bits beyond 1/2/4/8 (skip drones / flock / task / obs)
constexpr int CH_PHASE_FORCE_TIMEOUT = 64; // test only: the drone wave waits for a hand-off that never comes

// one curriculum level (curriculum_learning.py:10-194); the table kLevels lives in ch_device.h
struct Level {
    double desired, tol, hold, approach_min, min_eff, cattle_desired, cattle_tol;
    int min_drones, max_drones;
    double episode_len;
    double w_simple, w_complex, w_survival, w_approach, w_eff, w_cattle;
    int required_tally;
};

// LDS carve of one v2 step workgroup (ch_step.hip); identical on host (size) and device (offsets).
#ifndef CH_V2_MAX_BLOCK
#define CH_V2_MAX_BLOCK 768   // v2 workgroup size bound: 12 waves, 3 per SIMD (shared-table kernels)
#endif
#ifndef CH_V2_MAX_BLOCK_PW
#define CH_V2_MAX_BLOCK_PW 512   // per-wave-table and physics-variant kernels: 8 waves (their register use allows 2 per SIMD)
#endif
constexpr int kV2EnvInts = 14;
constexpr int kV2Flags = 32;         // LDS hand-off counters between the drone wave and the cow waves + work counters
// W = 0: one alpha pair table for the whole workgroup (4 reals per pair, G*P pairs), reused for the
// shepherd terms.  W > 0 ("per-wave env tables", large herds): each of the W cow waves owns a slot for
// ONE env at a time -- 3 reals per pair (gradient x, y and the bump; the consensus term is recomputed
// from the velocities when the rows are summed), reused for that env's shepherd terms -- so the LDS
// no longer grows with G*P and a whole CU's envs fit in one workgroup.
struct V2Layout {
    enum { CX = 0, DRONE, DCOW, ENVR, PAIRS, TD, MET, IMG, EI, LEVELS, PAIRL, XD, BYTES, NOFF };
    int G, N, M, P, rows, W;
    bool sep;      // shared tables: the shepherd terms in a region of their own (not reusing the pair table)
    size_t slot;   // W > 0: reals per wave slot
    size_t off[NOFF + 1];
    static __host__ __device__ size_t al(size_t x) { return (x + 15) & ~size_t(15); }
    __host__ __device__ V2Layout(int G_, int N_, int M_, int P_, int mode, int rb, int W_ = 0, bool sep_ = false)
        : G(G_), N(N_), M(M_), P(P_), W(W_), sep(W_ == 0 && sep_) {
        rows = mode == CH_MODE_CTDE ? 12 : N;
        slot = 3 * (size_t)P > 6 * (size_t)M * N ? 3 * (size_t)P : 6 * (size_t)M * N;
        const size_t shared = (sep || 4 * (size_t)G * P > 6 * (size_t)G * M * N) ? 4 * (size_t)G * P : 6 * (size_t)G * M * N;
        size_t o = 0;
        off[CX] = o;     o = al(o + 8 * (size_t)G * M * rb);         // cx cy cvx cvy aux auy spx spy
        off[DRONE] = o;  o = al(o + 21 * (size_t)G * N * rb);        // dx dy dz pa pb sa sb ca cb scat psp mrew mq meor q[4] rd[3]
        off[DCOW] = o;   o = al(o + (size_t)G * N * M * rb);         // cow-drone distances
        off[ENVR] = o;   o = al(o + 4 * (size_t)G * rb);             // prev clock, herd centroid x y
        off[PAIRS] = o;  o = al(o + (W ? (size_t)W * slot : shared) * rb);   // alpha pair table(s), then shepherd terms
        off[TD] = o;     o = al(o + (sep ? 4 * (size_t)G * M * rb + 4 * (size_t)G * M : 0));   // sep: shepherd sums, new velocities, per-cow counts
        off[MET] = o;    o = al(o + (size_t)kMetricRows * G * 8);
        off[IMG] = o;                                                // (observations go straight to HBM)
        off[EI] = o;     o = al(o + ((size_t)kV2EnvInts * G + 2 * G + 2 + kV2Flags) * 4);   // + flock/reset lists
        off[LEVELS] = o; o = al(o + 8 * sizeof(Level));              // curriculum table
        off[PAIRL] = o;  o = al(o + 2 * (size_t)P);                  // unordered cow pairs (i | j << 8)
        // f32 mode: f64 copies of the positions and centroid inputs (drone x y, cattle x y, herd centroid x y, prev)
        off[XD] = o;     o = al(o + (rb == 4 ? (2 * (size_t)G * N + 2 * (size_t)G * M + 3 * (size_t)G) * 8 : 0));
        const size_t tabs = W ? (size_t)W : (size_t)G;               // pair flags and term flags: per slot / per env
        // per-cow neighbour masks (u64) and "has a neighbour in sensing range" bytes, then the queue of pairs
        // inside the bump's support (u16; one per slot for W > 0, one for the workgroup otherwise)
        off[BYTES] = o;  o = al(o + 8 * (size_t)G * M + al((size_t)G * M) + 2 * (size_t)tabs * P + 3 * (size_t)G * N +
                                (size_t)G * M + tabs * M * N);
        off[NOFF] = o;
    }
    __host__ __device__ size_t bytes() const { return off[NOFF]; }
};

// on-device policy (ch_policy.hip)
struct MlpArgs {
    int layers;
    int dims[5];
    const float* w[4];
    const float* b[4];
    int hidden_act, clip;
    float lo, hi;
    const float* x;
    long long rows;
    float* y;
    const int* env_n;          // optional: NUM_DRONES per env (handle envi row 0) -> live input width
    const uint8_t* row_mask;   // optional: only rows with a non-zero byte are computed and written
    long long rows_per_env;    // 1: CTDE (live width n * k_unit); N: MARL (agent j live iff j < n)
    int k_unit;
    int kcap;                  // widest live input row any tile can have (<= dims[0]): sizes k_mlp2's input tile
    int vec_w;                 // bit i: layer i's weights are 16-B aligned rows (float4 loads); bit 7: so is x
    long long* tstamp;         // diagnostics (ch__set_mlp_tstamp): k_mlp2 phase clocks [grid][16], or NULL
    const float* packed;       // ch_mlp_pack layout of every layer (NULL: the raw nn.Linear weights)
    long long pk_off[4];       // layer li's offset in `packed` (floats)
    int pk_pairs[4];           // layer li's padded K pair count in `packed`
    int split_out[4], split_in[4];   // block-diagonal layers (ch_mlp; 0: dense)
    const int* rows_dev;       // optional device row count (<= rows): workgroups past it leave at once
};
extern long long* g_mlp_tstamp;
// floats of the packed layout of an MLP (per-layer offsets / pair counts out, optional)
long long mlp_packed_floats(int layers, const int* dims, long long* off, int* pairs);
hipError_t launch_mlp_pack(const MlpArgs& a, float* dst, hipStream_t st);
size_t mlp_lds_bytes();
hipError_t launch_mlp(const MlpArgs& a, hipStream_t st);

// ch_aux.hip: metric rows [kMetricRows][E] -> out[CH_METRIC_COUNT] (sums over envs, fixed order);
// `err_word` (optional) is copied to err_out as a double; reset zeroes the summed rows
hipError_t launch_metrics_reduce(double* metrics, long long E, double* out, const int* err_word, double* err_out,
                                 int reset, hipStream_t st);

// ch_aux.hip: the on-device PPO rollout buffer (ch_rollout_*)
struct RolloutArgs {
    int T, t, obs_dim, act_dim, env_act_dim;
    int mean_ld, value_ld, tv_ld;   // row strides of mean / value / terminal_value (a fused actor-critic's output
                                    // holds both heads in one [rows][act_dim + 1] buffer)
    int post_prev;                  // store (t) / gae: first run step t - 1's (T - 1's) post (ch_rollout_collect)
    int copy_obs;                   // store: copy obs_now into obs[t] (0: the step already wrote obs[t] there)
    // deferred truncation bootstrap (ch_rollout_collect): the post of a step whose env was truncated and not
    // terminated queues the env's terminal observation (term_obs) at slot atomicAdd(tv_count) of tv_obs with its
    // rewards row in tv_row; every few steps one forward over the queue gives the values and k_rollout_apply adds
    // gamma V to those rows (the same f32 fma the immediate path does)
    int defer;
    int post_only;                  // store: only the previous step's post (the last step's, before GAE)
    int v_col;                      // kRoleTvApply: the value's column in the value net's output
    const float* term_obs;
    float* tv_obs;
    int* tv_count;
    long long* tv_row;
    long long rows;
    unsigned long long seed;
    float gamma, gamma_lambda;
    const float *obs_now, *mean, *value, *log_std, *terminal_value, *reward;
    const uint8_t *terminated, *truncated;
    float *env_actions, *obs, *actions, *rewards, *episode_starts, *values, *log_probs, *advantages, *returns,
        *last_episode_starts;
};
hipError_t launch_rollout(const RolloutArgs& a, int which, hipStream_t st);
// ch_aux.hip: the DTDE (RLlib) per-agent rollout (ch_marl_rollout_collect); rows = E * N agents
struct MarlArgs {
    int T, t, A, N;
    long long E, rows;
    const int* env_n;          // handle envi row 0 (NUM_DRONES) and row 7 (the live-agent mask) at the step's start
    const int* env_active;
    const float* pol;          // [rows][2A] policy output: mean, log_std
    const float* val;          // [rows] value output
    const float* obs_now;      // t == 0: the batch's observations, copied into obs[0]
    unsigned long long seed;
    int post_prev, post_only;
    const float* reward;       // the last step's outputs [rows]
    const uint8_t *term, *trunc;
    float gamma, gamma_lambda;
    float *obs, *actions, *log_probs, *values, *rewards, *advantages, *returns, *last_values, *env_actions;
    uint8_t *mask, *terminated, *truncated;
};
hipError_t launch_marl_rollout(const MarlArgs& a, int which, hipStream_t st);   // 0 store (+ post of t - 1), 1 gae

// ch_aux.hip: ch_outputs_to_host's compaction of the envs that auto-reset (ascending env order)
hipError_t launch_stage_ended(long long E, const uint8_t* reset, const float* term_obs, const double* stats,
                              int blk_floats, long long* count, long long* env_out, double* stats_out, float* obs_out,
                              hipStream_t st);   // 0 store, 1 post, 2 gae, 3 apply (cap slots)

// up to three independent forwards in one launch (ch_policy.hip k_mlp2).  A segment's role folds the rollout
// store into its last layer's epilogue (ch_rollout_collect): kRoleSample -- the actor's mean becomes the
// Gaussian sample, its log-probability and the env actions (k_rollout_store's action half); kRoleValue -- the
// critic's value goes into the buffer together with the previous step's post and the episode start (its
// other half).  `ro` holds the rollout buffer for both.
// kRoleTvApply -- the deferred truncation bootstrap's flush: the value of queued terminal observation q is added,
// times gamma, to its rewards row tv_row[q] (k_rollout_apply's fma) straight from the epilogue.
enum { kRoleNone = 0, kRoleSample = 1, kRoleValue = 2, kRoleTvApply = 3 };
struct MlpMulti {
    MlpArgs seg[3];
    int nseg;
    int start[4];              // first workgroup of each segment (start[nseg] = grid)
    int lda, ldh;
    int role[3];
    RolloutArgs ro;
};
hipError_t launch_mlp_multi(const MlpArgs* segs, int nseg, hipStream_t st, const int* roles = nullptr,
                            const RolloutArgs* ro = nullptr);
bool mlp_multi_fits(const MlpArgs* segs, int nseg);   // k_mlp2 takes these nets (the rollout epilogues need it)

template <class R> hipError_t launch_step(const StepParams<R>& p, int team, hipStream_t st);
template <class R> hipError_t launch_reset(const StepParams<R>& p, int team, hipStream_t st);
// launch = false only performs the once-per-device function-attribute opt-in (at ch_create, so that a
// step captured into a HIP graph needs no host-side setup)
template <class R> hipError_t launch_step_v2(const StepParams<R>& p, int block, size_t lds, hipStream_t st,
                                             bool launch = true);
// ch_step_n: n consecutive steps of the same io in one launch (k_step2_multi), for the BASELINE geometries under PYB
// without terminal observations; hipErrorNotSupported (nothing launched) elsewhere.  launch = false: the attribute
// opt-in only.
// `pd`: a device copy of p (the kernel reads its parameters from it).
template <class R> hipError_t launch_step_v2_multi(const StepParams<R>& p, const StepParams<R>* pd, int block, size_t lds,
                                                   hipStream_t st, int n_steps, bool launch = true);
// ch_rollout_collect's fused step (k_step2_actor): the step of the CTDE 16-env x 4-drone x 16-cattle geometry (f64,
// CH_V2_MAX_BLOCK threads) followed in each workgroup by the actor forward with the sampling epilogue on the 16
// observation rows it wrote.  hipErrorNotSupported (nothing launched) when the handle's geometry or the net does not
// fit it; launch = false checks only.
template <class R> hipError_t launch_step_v2_actor(const StepParams<R>& p, int block, size_t lds, hipStream_t st,
                                                   const MlpArgs& a, const RolloutArgs& ro, bool launch = true);
// k_mlp2's one-tile shape for a fused forward (ch_policy.hip): LDS strides and dynamic bytes; false when the net does
// not fit a 12-wave, one-column-tile-per-wave tile (layers <= 192 wide, first-layer live width <= 1152)
bool mlp2_fused_tile(const MlpArgs& a, int& lda, int& ldh, size_t& bytes);
// the v2 kernel runs with per-wave env tables (V2Layout W > 0) for herds above this size
constexpr int kPwMinCattle = 17;

}  // namespace ch
