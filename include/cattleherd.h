/*
 * cattleherd.h — C ABI of the MI355X-native batched cattle-herding environment (libcattleherd.so).
 *
 * The reference (BenCooper305/RL-Cattle-Herding, gym_pybullet_drones/) has no native FFI: its
 * hot path is a Python gym.Env whose step() drives PyBullet.  This ABI replaces that env object
 * for a whole batch of environments at once; each entry point names the reference interface it
 * stands in for (paths relative to gym_pybullet_drones/).  INTEGRATION.md shows the ctypes
 * binding and the Gymnasium / SB3 / RLlib adapters layered on top.
 *
 * Conventions
 *   - Every call returns an int status: CH_OK (0) or a negative CH_ERR_*; ch_last_error() gives the
 *     message.  No exception crosses the ABI.  NaN/Inf in the simulation propagate exactly like the
 *     reference (e.g. the CTDE reward is NaN for 2 drones — see DESIGN.md "Quirks").
 *   - Buffers passed to ch_reset/ch_step are DEVICE pointers owned by the caller (e.g. torch
 *     tensors' data_ptr()); state is owned by the handle and lives in HBM.
 *   - One handle <-> one device.  Work is enqueued on the given hipStream_t (NULL = default stream)
 *     and is asynchronous until the caller synchronises.  One host thread per handle.
 *   - Layouts (E = n_envs, N = num_drones from the config, R = obs rows, K = reward columns):
 *       actions       float32 [E][N][4]          (VEL action, BaseRLAviary.py:185-222)
 *       obs           float32 [E][R][86]         R = 12 (CTDE, BaseRLAviary.py:272-342) or N (MARL,
 *                                                BaseMARLAviary.py:253-303)
 *       reward        float32 [E][K]             K = 1 (CTDE) or N (MARL, per agent)
 *       terminated    uint8   [E][K]
 *       truncated     uint8   [E][K]
 *       agent_active  uint8   [E][N]             MARL wrapper's live agents (marl_wrapper.py:112-113)
 */
#ifndef CATTLEHERD_H
#define CATTLEHERD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CH_ABI_VERSION 6

enum {
    CH_OK = 0,
    CH_ERR_INVALID = -1,     /* bad argument / configuration (reference: print+exit / ValueError) */
    CH_ERR_DEVICE = -2,      /* HIP runtime error */
    CH_ERR_NOMEM = -3,
    CH_ERR_UNSUPPORTED = -4  /* configuration the reference itself cannot run (e.g. 1 drone) */
};

enum { CH_MODE_CTDE = 0, CH_MODE_MARL = 1 };
enum { CH_PREC_F64 = 0, CH_PREC_F32 = 1 };
/* Physics enum, in the reference's order (utils/enums.py:13-21; dispatch BaseAviary.py:420-450) */
enum {
    CH_PHYS_PYB = 0,          /* _physics + p.stepSimulation (default) */
    CH_PHYS_DYN = 1,          /* explicit _dynamics + _integrateQ (BaseAviary.py:1043-1118); cattle stay put */
    CH_PHYS_PYB_GND = 2,      /* + _groundEffect (943-980) */
    CH_PHYS_PYB_DRAG = 3,     /* + _drag (982-1011) */
    CH_PHYS_PYB_DW = 4,       /* + _downwash (1013-1041) */
    CH_PHYS_PYB_GND_DRAG_DW = 5,
    CH_PHYS_DYN_RK4 = 6       /* option, not in the reference: DYN's equations of motion integrated by classic
                                 RK4 per substep (q renormalised); cattle stay put as under DYN */
};

/* Flags for ch_step_io.flags */
#define CH_STEP_AUTORESET      0x1u  /* reset finished envs in the same launch (SB3 VecEnv semantics) */
#define CH_STEP_RANDOM_ACTIONS 0x2u  /* draw U[-1,1) actions on device (Philox4x32-10, key = seed,
                                        counter = (step, drone, env)); written to actions_out if set */

/* Environment configuration.  Mirrors the constructor of CattleAviary (sb3_envs/CattleAviary.py:14-28)
 * / MARLCattleAviary (rllib_envs/MARLCattleAviary.py:14-28) plus the knobs the reference hard-codes. */
typedef struct ch_config {
    int32_t abi_version;      /* = CH_ABI_VERSION */
    int32_t mode;             /* CH_MODE_CTDE (sb3_envs) or CH_MODE_MARL (rllib_envs) */
    int32_t num_drones;       /* constructor num_drones: action rows (BaseRLAviary.py:80), <= 12 */
    int32_t num_cattle;       /* num_cattle, <= 64 (reference spawns at most 16, BaseAviary.py:611) */
    int32_t min_drones;       /* NUM_DRONES drawn per reset in [min, max] (BaseAviary.py:307);      */
    int32_t max_drones;       /*   -1 = num_drones (pinned)                                          */
    int32_t curriculum_level; /* starting level; -1 = reference default (CTDE 7, MARL 0)             */
    int32_t ctrl_freq;        /* 60 (CattleAviary.py:23) */
    int32_t pyb_freq;         /* 240 (CattleAviary.py:22) */
    int32_t compat;           /* 1 = reproduce reference quirks bit-for-bit (DESIGN.md "Quirks") */
    int32_t precision;        /* CH_PREC_F64 (reference arithmetic) or CH_PREC_F32 */
    int32_t torque_world;     /* link_lag = 0 only: 1 = applyExternalTorque(LINK_FRAME) acts in world frame.  With
                                 link_lag = 1 the z torque turns with the cached link frame whatever this says: the
                                 recorded real-PyBullet trace rejects a world-frame z torque there (2e-5 vs 2e-13
                                 m/s by step 4) */
    int32_t gyro;             /* 1 = gyroscopic term (btMultiBody default) */
    int32_t marl_wrapper;     /* MARL only: 1 = RLlibMultiAgentWrapper.step semantics (marl_wrapper.py:77-119:
                                 per-agent recomputation, finished agents drop out, episode ends when all
                                 agents terminated); 0 = bare MARLCattleAviary.step dicts
                                 (rllib_envs/BaseAviary.py:425-431) */
    double damping;           /* btMultiBody default linear/angular damping 0.04 */
    uint64_t seed;            /* Philox key for resets and random actions */
    int64_t env_id_offset;    /* global index of env 0 (multi-GPU sharding) */
    const double* spawn_table;/* host [spawn_scenarios][spawn_cows][2]; NULL = built-in table
                                 (config/cattle_positions.yaml, 100 x 16; extended for > 16 cows) */
    int32_t spawn_scenarios;
    int32_t spawn_cows;
    int32_t physics;          /* CH_PHYS_* (CattleAviary ctor `physics`, CattleAviary.py:21) */
    int32_t eval_metrics;     /* 1 (default) = keep update_evaluation_metrics' per-drone episode distance on
                                 the device every step (BaseAviary.py:1406-1435), read with ch_get_eval */
    int32_t link_lag;         /* 1 (default) = _physics' applyExternalForce/Torque(LINK_FRAME) (BaseAviary.py:907-939)
                                 rotate by the link transform Bullet cached at the previous substep (the
                                 attitude one substep old, state components qlag): what the recorded real-PyBullet
                                 trace shows; 0 = the current attitude (rounds 1-4 model) */
} ch_config;

typedef struct ch_handle ch_handle;

/* Fill *cfg with the reference defaults for `mode` (CattleAviary / MARLCattleAviary constructors). */
int ch_default_config(ch_config* cfg, int32_t mode, int32_t num_drones, int32_t num_cattle);

/* Replaces: CattleAviary.__init__ (sb3_envs/CattleAviary.py:14-105) — one env — with n_envs envs on
 * `device`.  Allocates the SoA state in HBM and uploads the spawn table. */
int ch_create(const ch_config* cfg, int64_t n_envs, int32_t device, ch_handle** out);

/* Replaces: BaseAviary.close (sb3_envs/BaseAviary.py:498-503). */
int ch_destroy(ch_handle* h);

/* Message of the last failing call on `h` (or of the last failing ch_create when h == NULL). */
const char* ch_last_error(const ch_handle* h);

/* Shapes: obs rows R and reward columns K. */
int ch_shape(const ch_handle* h, int64_t* n_envs, int32_t* obs_rows, int32_t* obs_cols, int32_t* reward_cols);

/* Replaces: BaseAviary.reset (sb3_envs/BaseAviary.py:280-331; rllib_envs/BaseAviary.py:280-318).
 * Resets the envs whose mask byte is non-zero (mask = NULL: all) and writes their initial
 * observation into obs (device, [E][R][86]); other envs' obs rows are left untouched.
 * A full reset (mask = NULL) first reads and clears the handle's sticky device error word: it synchronises `stream`
 * (so it blocks the host and cannot be captured into a HIP graph), and a device error an earlier step recorded and no
 * ch_sync / ch_metrics / ch_get_state has reported yet is returned as CH_ERR_DEVICE after the reset has been done
 * (the state is then the fresh reset's). */
int ch_reset(ch_handle* h, const uint8_t* mask_dev, float* obs_dev, void* stream);

/* ch_reset with the reset's random draws supplied by the caller instead of the device's Philox stream:
 * num_drones host int32[E] (NUM_DRONES of each reset env, BaseAviary.py:307) and/or cow_vel host
 * double[E][M][2] (the cattle spawn velocities 0.2 (cos a, sin a), BaseAviary.py:631-632); either may be
 * NULL.  With cattleherd/seeded.py replaying the reference's own seeded `random` / NumPy draws this
 * reproduces the reference's reset state bit for bit.  Synchronises `stream`. */
int ch_reset_with(ch_handle* h, const uint8_t* mask_dev, const int32_t* num_drones, const double* cow_vel,
                  float* obs_dev, void* stream);

typedef struct ch_step_io {
    const float* actions;      /* device [E][N][4]; ignored with CH_STEP_RANDOM_ACTIONS */
    float* actions_out;        /* optional: where device-drawn random actions are stored */
    float* obs;                /* device [E][R][86] (required) */
    float* reward;             /* device [E][K] (required) */
    uint8_t* terminated;       /* device [E][K] (required) */
    uint8_t* truncated;        /* device [E][K] (required) */
    float* terminal_obs;       /* optional device [E][R][86]: pre-reset obs of envs that auto-reset; leave NULL
                                  when not needed: the 16-env x 4-drone geometry then rebuilds reset envs
                                  without a workgroup sync (same outputs) */
    uint8_t* agent_active;     /* optional device [E][N]: MARL live-agent mask after this step */
    uint8_t* reset_happened;   /* optional device [E]: 1 where the env auto-reset in this call */
    uint32_t flags;            /* CH_STEP_* */
    uint32_t _pad;
    double* episode_stats;     /* optional device [E][2]: where an episode ends in this call, its return (the sum of
                                  the float64 rewards the reference returns) and length in steps -- SB3 Monitor's
                                  info["episode"] "r" and "l" (CTDECattleHerder.py:91-99); other rows untouched */
} ch_step_io;

/* Replaces: BaseAviary.step (sb3_envs/BaseAviary.py:335-465) for every env at once — VEL action →
 * DSLPIDControl → motor model → pyb_freq/ctrl_freq physics substeps → flocking every 2nd step →
 * observation → reward / terminated / truncated; with CH_STEP_AUTORESET, SB3 VecEnv auto-reset.
 * MARL mode additionally applies RLlibMultiAgentWrapper.step's per-agent recomputation
 * (rllib_envs/marl_wrapper.py:77-119). */
int ch_step(ch_handle* h, const ch_step_io* io, void* stream);

/* n_steps consecutive ch_step calls with the same io, in as few launches as the geometry allows: the steps run in one
 * launch in which every workgroup steps its envs back to back (k_step2_multi) -- the BASELINE
 * geometries under PYB without terminal observations; elsewhere one launch per step.  A buffer whose constant
 * observation bytes are not known to be in place (first use, after ch_set_state / invalidation) gets one plain
 * ch_step first.  The kernel reads its parameters from a device copy that is re-uploaded (stream-ordered) when they
 * change (from host memory, staged by the runtime at the call): use one stream per handle.  Under stream capture
 * (a HIP graph) the call records n_steps plain ch_step launches instead.  The outputs in io are those of the last step; state, auto-resets, metrics and the device-drawn
 * random actions (CH_STEP_RANDOM_ACTIONS: each step draws its own) equal n_steps ch_step calls bit for bit.  For
 * random-action rollouts and data generation; a policy that reads each step's observation calls ch_step.
 * Replaces: n_steps iterations of the reference's env.step loop (BaseAviary.step, sb3_envs/BaseAviary.py:335-465). */
int ch_step_n(ch_handle* h, const ch_step_io* io, int32_t n_steps, void* stream);

/* Host delivery of one step's outputs (the batched SB3 VecEnv and RLlib dict surfaces).
 * Replaces: what SubprocVecEnv.step_wait gathers from its worker processes -- obs (E, R, 86), rewards,
 * dones, and for the envs that ended info["terminal_observation"] and Monitor's info["episode"]
 * (CTDECattleHerder.py:91-99) -- and the arrays RLlibMultiAgentWrapper.step builds its per-agent dicts from
 * (marl_wrapper.py:97-119).  After ch_step on `stream`: copies the step's outputs from io's device buffers
 * into caller-owned host buffers (pinned host memory for full speed), then synchronises `stream`.
 *   - The observation copy moves only the first num_drones rows of every block: a CTDE (12, 86) block's rows
 *     >= num_drones are always zero, so the caller zero-fills `obs` once and they stay zero.
 *   - The envs that auto-reset in the step (io->reset_happened) are compacted on the device, in ascending env
 *     order: their count, indices, terminal observations (io->terminal_obs, whole blocks) and episode statistics
 *     (io->episode_stats: return, length).  Before the count is known the call copies a first part sized from the
 *     recent counts (twice the larger of the last count and its running mean, plus 8): one synchronisation when at
 *     most that many envs ended, two otherwise. */
typedef struct ch_host_out {
    float* obs;                /* host [E][R][86] (required) */
    float* reward;             /* host [E][K] (required) */
    uint8_t* terminated;       /* host [E][K] (required) */
    uint8_t* truncated;        /* host [E][K] (required) */
    uint8_t* reset_happened;   /* optional host [E] (needs io->reset_happened) */
    uint8_t* agent_active;     /* optional host [E][N] (needs io->agent_active) */
    int64_t ended_count;       /* out: envs that auto-reset in the step (needs io->reset_happened) */
    int64_t* ended_env;        /* optional host [E]: their indices, ascending */
    float* ended_obs;          /* optional host [E][R][86]: their terminal observations (needs io->terminal_obs) */
    double* ended_stats;       /* optional host [E][2]: their episode return and length (needs io->episode_stats) */
} ch_host_out;
int ch_outputs_to_host(ch_handle* h, const ch_step_io* io, ch_host_out* out, void* stream);

/* Full SoA state, for checkpoint/resume and parity state-injection.  Layout of the two host
 * buffers (counts from ch_state_size):
 *   doubles: drone[26][E][N] (px py pz qx qy qz qw vx vy vz wx wy wz pid_last_rpy[3]
 *            pid_int_pos[3] pid_int_rpy[3] qlag[4] = the cached link frame, link_lag), cattle[4][E][M] (x y vx vy),
 *            env[2][E] (prev_cent clock),
 *            phys[7][E][N] (last_clipped_action[4] = drag input, DYN body rates rpy_rates[3])
 *   int32:   env[10][E] (n, step_counter, step_counter_A, has_prev, level, tally, spawn_index,
 *            active_mask, episode, step_index = ch_step calls so far = the Philox action counter) */
int ch_state_size(const ch_handle* h, int64_t* n_doubles, int64_t* n_ints);
int ch_get_state(ch_handle* h, double* host_doubles, int32_t* host_ints, void* stream);
int ch_set_state(ch_handle* h, const double* host_doubles, const int32_t* host_ints, void* stream);

/* End-of-rollout metrics (host double[CH_METRIC_COUNT]) accumulated on device since the last call
 * with reset_after != 0: see CH_METRIC_* below.  Rank-local; bench.py all-reduces them over RCCL. */
enum {
    CH_METRIC_STEPS = 0, CH_METRIC_EPISODES, CH_METRIC_RETURN_SUM, CH_METRIC_LENGTH_SUM,
    CH_METRIC_TERMINATED, CH_METRIC_TRUNCATED, CH_METRIC_NAN_REWARDS, CH_METRIC_EFFECTIVENESS_SUM,
    CH_METRIC_COUNT
};
int ch_metrics(ch_handle* h, double* host_out, int32_t reset_after, void* stream);

/* The same sums written to a DEVICE buffer double[CH_METRIC_COUNT] on `stream`, without a host sync:
 * the input of the end-of-rollout RCCL all-reduce (bench.py).  Replaces the same reference code. */
int ch_metrics_device(ch_handle* h, double* dev_out, int32_t reset_after, void* stream);

/* Wait for `stream` and report the handle's sticky device error word: CH_ERR_DEVICE if a step kernel
 * recorded a failure (e.g. an LDS hand-off that timed out), CH_OK otherwise.  ch_metrics and
 * ch_get_state report it too.  (The reference's analogue: an exception out of env.step,
 * marl_wrapper.py:87-95.) */
int ch_sync(ch_handle* h, void* stream);

/* update_evaluation_metrics' per-drone episode distance (sb3_envs/BaseAviary.py:1415-1426, the
 * `episode_drone_distances` the evaluator logs; both components of the reference's 2-vector are equal):
 * host double[E][N], zero for drones beyond NUM_DRONES; reset with the episode.  Needs
 * cfg->eval_metrics (CH_ERR_UNSUPPORTED otherwise).  Synchronises `stream`. */
int ch_get_eval(ch_handle* h, double* host_out, void* stream);

/* Number of built-in spawn scenarios / cows, and a copy of the table (host double[S][C][2]):
 * config/cattle_positions.yaml, 100 scenarios x 16 cows (BaseAviary.py:88-94). */
int ch_builtin_spawn_table(double* out, int32_t* scenarios, int32_t* cows);

/* The table ch_create uses when cfg->spawn_table is NULL: the built-in 16 cows per scenario, extended
 * deterministically for cows > 16 (out: host double[100][max(cows,16)][2]; out may be NULL to query). */
int ch_spawn_table(int32_t cows, double* out, int32_t* scenarios, int32_t* out_cows);

/* ---- On-device policy ---------------------------------------------------------
 * A dense MLP evaluated on the matrix cores in f32 (exact f32 products, f32 sums), weights in
 * device memory in torch nn.Linear layout.  The SB3 actor of the reference's CTDE driver is
 * dims {1032, 128, 128, 48}, tanh hidden, output clipped to [-1, 1]; its critic {1032, 128, 128, 1};
 * the RLlib per-agent model {86, 256, 256, 8}. */
#define CH_ACT_NONE 0
#define CH_ACT_TANH 1
#define CH_ACT_RELU 2
typedef struct ch_mlp {
    int32_t n_layers;          /* 1..4 */
    int32_t dims[5];           /* dims[0] inputs; dims[i + 1] outputs of layer i (<= 256) */
    const float* weight[4];    /* device [dims[i+1]][dims[i]] row-major (nn.Linear.weight) */
    const float* bias[4];      /* device [dims[i+1]] or NULL */
    int32_t hidden_act;        /* CH_ACT_* applied after every layer but the last */
    int32_t clip;              /* non-zero: clip the output to [lo, hi] */
    float lo, hi;
    const float* packed;       /* NULL, or the same weights in the MFMA operand layout written by ch_mlp_pack
                                  (read instead of `weight`; re-pack after every weight update) */
    int32_t split_out[4];      /* block-diagonal layer i (i >= 1; 0 = dense): outputs [0, split_out) read only */
    int32_t split_in[4];       /* inputs [0, split_in), outputs [split_out, N) only [split_in, K) -- the weights
                                  outside the two blocks are zero and are not multiplied (e.g. SB3's actor and
                                  critic packed as one net).  Used when split_in % 128 == 0 and split_out % 32 == 0,
                                  else the layer runs dense (same result). */
} ch_mlp;

/* The operand layout of the forward kernel: per layer [16-column tile][32-wide K pair][half][lane][4], so that
 * each wave's weight load is one contiguous 1 KB block.  ch_mlp_packed_size: floats of device memory the
 * layout of `net` takes; ch_mlp_pack: writes it (from net->weight) into dst on `stream`.  No reference
 * counterpart: the reference's torch forward reads nn.Linear weights (CTDECattleHerder.py:203). */
int64_t ch_mlp_packed_size(const ch_mlp* net);
int ch_mlp_pack(const ch_mlp* net, float* dst, void* stream);

/* Replaces: stable_baselines3 ActorCriticPolicy.predict(obs, deterministic=True) for a Box action
 * space (mlp_extractor.policy_net -> action_net -> np.clip to the space, CTDECattleHerder.py:203,
 * 106-127) and predict_values (value_net), and the RLlib model forward of DTDECattleHerder.py.
 * y[rows][dims[L]] = MLP(x[rows][dims[0]]); x and y are device buffers. */
int ch_mlp_forward(const ch_mlp* net, const float* x, int64_t rows, float* y, void* stream);

/* ch_mlp_forward for the rows whose byte in row_mask (device uint8 [rows]) is non-zero; the other rows of y
 * are left untouched, and 16-row tiles with no selected row cost next to nothing.  Replaces the SB3 rollout's
 * predict_values(terminal_observation) for the envs that just reset (OnPolicyAlgorithm.collect_rollouts'
 * TimeLimit.truncated bootstrap, CTDECattleHerder.py:107-150), evaluated only where it is used. */
int ch_mlp_forward_masked(const ch_mlp* net, const float* x, int64_t rows, const uint8_t* row_mask, float* y,
                          void* stream);

/* ch_mlp_forward on a handle's observation buffer: one row per env for CTDE (x = obs [E][R][86]
 * flattened, dims[0] = R*86) or per agent for MARL (x = obs [E][N][86], dims[0] = 86, E*N rows).
 * Input features past an env's NUM_DRONES rows (CTDE) or of agents past NUM_DRONES (MARL) are zero
 * in the observation and are not multiplied. */
int ch_policy_forward(ch_handle* h, const ch_mlp* net, const float* obs, float* y, void* stream);

/* ---- On-device PPO rollout buffer ---------------------------------------------
 * Replaces: stable_baselines3 OnPolicyAlgorithm.collect_rollouts' RolloutBuffer and
 * RolloutBuffer.compute_returns_and_advantage for the CTDE driver's PPO (CTDECattleHerder.py:107-150:
 * n_steps, gamma 0.99, gae_lambda 0.95, DiagGaussian actions with log_std).  CTDE handles only (one row
 * per env).  All buffers are caller-owned device float32 arrays, rows = n_envs:
 *   obs [T][rows][12*86], actions [T][rows][act_dim] (unclipped samples), rewards, episode_starts, values,
 *   log_probs, advantages, returns [T][rows]; last_episode_starts [rows] (SB3's _last_episode_starts,
 *   1 after a reset). */
typedef struct ch_rollout {
    int32_t n_steps;           /* T */
    int32_t act_dim;           /* policy action width (the reference's 12 x 4 = 48) */
    float* obs;
    float* actions;
    float* rewards;
    float* episode_starts;
    float* values;
    float* log_probs;
    float* advantages;
    float* returns;
    float* last_episode_starts;
} ch_rollout;

/* Step t, before env.step: copy obs [rows][12*86] into the buffer, sample actions = mean + exp(log_std) eps
 * (eps ~ N(0,1) from Philox keyed by seed, counter (t, action, env)), store them with their summed Normal
 * log-probability, value [rows] and the episode starts; write the actions clipped to [-1, 1] into
 * env_actions [rows][num_drones][4] (the first num_drones*4 of act_dim, as the env reads a (12, 4) action). */
int ch_rollout_store(ch_handle* h, const ch_rollout* rb, int32_t t, const float* obs, const float* mean,
                     const float* value, const float* log_std, uint64_t seed, float* env_actions, void* stream);

/* Step t, after env.step: rewards[t] = reward, plus gamma * terminal_value where the env was truncated and
 * not terminated (SB3's TimeLimit.truncated bootstrap; terminal_value may be NULL); the next step's
 * episode starts = terminated | truncated. */
int ch_rollout_post(ch_handle* h, const ch_rollout* rb, int32_t t, const float* reward, const uint8_t* terminated,
                    const uint8_t* truncated, const float* terminal_value, float gamma, void* stream);

/* compute_returns_and_advantage: GAE(gamma, gae_lambda) backwards over the T steps in float32 with
 * last_value [rows] = V(obs after the last step). */
int ch_rollout_gae(ch_handle* h, const ch_rollout* rb, const float* last_value, float gamma, float gae_lambda,
                   void* stream);

/* The whole collection in one call (the native loop behind cattleherd.rollout.DeviceRolloutBuffer.collect):
 * for t < n_steps, on `stream`: actor and critic forwards on step->obs (ch_policy_forward), ch_rollout_store,
 * ch_step with auto-reset and terminal observations, the critic on the terminal observations of the envs that
 * reset (ch_mlp_forward_masked; skipped with bootstrap_truncated = 0), ch_rollout_post; then the critic on the
 * last observations and ch_rollout_gae.
 * critic == NULL: `actor` is a fused actor-critic whose output is act_dim + 1 wide (the action mean, then the
 * value; e.g. SB3's two MLPs packed as one: layer 1 stacked, layers 2-3 block-diagonal, which leaves every output
 * bit-identical to the separate nets): one forward per step reads the observation once.  `mean` and
 * `terminal_value` are then [rows][act_dim + 1] (both heads); `value` is not used.
 * Device scratch (caller-owned): */
typedef struct ch_rollout_io {
    const ch_step_io* step;    /* the env's step buffers; obs, reward, terminated, truncated, terminal_obs and
                                  reset_happened are required (actions are env_actions below) */
    float* mean;               /* [rows][act_dim] ([rows][act_dim + 1] with a fused actor-critic) */
    float* value;              /* [rows] */
    float* terminal_value;     /* [rows] ([rows][act_dim + 1] with a fused actor-critic) */
    float* env_actions;        /* [rows][num_drones][4] */
} ch_rollout_io;
int ch_rollout_collect(ch_handle* h, const ch_rollout* rb, const ch_rollout_io* io, const ch_mlp* actor,
                       const ch_mlp* critic, const float* log_std, uint64_t seed, float gamma, float gae_lambda,
                       int32_t bootstrap_truncated, void* stream);

/* ---- On-device rollout collection for the DTDE (RLlib) driver ----------------------------------------------
 * Replaces: RLlib PPO's sampling of RLlibMultiAgentWrapper envs with one shared policy over every agent
 * (DTDECattleHerder.py:62-97: policies = {"shared_policy"}, gamma 0.99, train_batch_size 4096; the wrapper's
 * agent drop-out and "__all__", marl_wrapper.py:77-119) and its GAE postprocessing.  MARL handles only.  Rows are
 * agents: rows = n_envs * num_drones, row e * num_drones + i = agent_i of env e.  Per step t < n_steps:
 *   the policy (output [rows][2 * act_dim]: RLlib's DiagGaussian inputs, the mean then log_std) and the value net
 *   on the agents' observations (obs[t] = [rows][86]); for every agent live at the step's start (the wrapper's
 *   self.agents: agent i < NUM_DRONES, not dropped out) a Gaussian sample a = mean + exp(log_std) eps (Philox keyed
 *   by seed, counter (t, action, row), Box-Muller), stored unclipped with its summed Normal log-probability, the
 *   value and agent_mask = 1; the env gets the samples clipped to [-1, 1] (RLlib's unsquash for Box(-1, 1)) and 0
 *   for the other agents (ignored by the env); ch_step with auto-reset; the step's reward / terminated / truncated
 *   per agent (0 where agent_mask is 0).
 * Then last_values = V(obs after the last step) and GAE(gamma, gae_lambda) per agent backwards in float32: an
 * agent's trajectory ends where it terminates (bootstrap 0; the env resets only once every agent has terminated, so
 * a live agent that did not terminate is live at the next step of the same episode); rows with agent_mask 0 get
 * advantage and return 0; truncation does not end a trajectory (the wrapper keeps truncated agents acting).
 * Divergence note: RLlib's per-agent episodes treat terminated OR truncated as done and bootstrap V(obs) at a
 * truncation; this restatement follows the wrapper's "__all__" rule instead and bootstraps straight through the
 * time limit (marl_wrapper.py:104-117).  Parity unpinned either way: RLlib is not installed here.
 * RLlib is not installed here: these semantics are restated from its PPO defaults ("parity unpinned" to its
 * source).  All arrays are caller-owned device memory. */
typedef struct ch_marl_rollout {
    int32_t n_steps;           /* T */
    int32_t act_dim;           /* 4 (the VEL action of one agent) */
    float* obs;                /* [T][rows][86] */
    float* actions;            /* [T][rows][act_dim] unclipped samples (0 where not live) */
    float* log_probs;          /* [T][rows] */
    float* values;             /* [T][rows] */
    float* rewards;            /* [T][rows] */
    uint8_t* agent_mask;       /* [T][rows]: the agent was live at the start of step t */
    uint8_t* terminated;       /* [T][rows] */
    uint8_t* truncated;        /* [T][rows] */
    float* advantages;         /* [T][rows] */
    float* returns;            /* [T][rows] (advantages + values) */
    float* last_values;        /* [rows] */
} ch_marl_rollout;
typedef struct ch_marl_rollout_io {
    const ch_step_io* step;    /* the env's step buffers: obs, reward, terminated, truncated (actions are env_actions) */
    float* policy_out;         /* scratch [rows][2 * act_dim] */
    float* value_out;          /* scratch [rows] */
    float* env_actions;        /* scratch [n_envs][num_drones][4] */
} ch_marl_rollout_io;
int ch_marl_rollout_collect(ch_handle* h, const ch_marl_rollout* rb, const ch_marl_rollout_io* io, const ch_mlp* policy,
                            const ch_mlp* value, uint64_t seed, float gamma, float gae_lambda, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CATTLEHERD_H */
