/*
 * ch_oracle.h — CPU restatement (fp64, scalar C) of the reference env step.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker / CPU baseline — never as the product path.
 *
 * Parity: pinned against the golden vectors in tests/golden/ (generated from the reference's own
 * Python, see tests/golden/make_golden.py) and against the recorded PyBullet trace
 * tests/golden/trace_eval.npz.  The drone rigid-body model (what p.stepSimulation does) is
 * "parity unpinned" beyond the trace's symplectic-Euler fit — see DESIGN.md.
 */
#ifndef CH_ORACLE_H
#define CH_ORACLE_H
#include <stdint.h>

#define OCH_NMAX 12
#define OCH_MMAX 64

typedef struct och_config {
    int32_t mode;             /* 0 = CTDE (sb3_envs), 1 = MARL (rllib_envs + marl_wrapper) */
    int32_t n_ctor;           /* constructor num_drones: action rows / controller count */
    int32_t m;                /* num_cattle */
    int32_t min_drones, max_drones;
    int32_t start_level;      /* CTDE reference: 7, MARL reference: 0 */
    int32_t ctrl_freq, pyb_freq;
    int32_t compat;           /* 1 = reproduce reference quirks (default) */
    double damping;           /* btMultiBody default 0.04 */
    int32_t torque_world;     /* applyExternalTorque(LINK_FRAME) as world frame */
    int32_t gyro;
    uint64_t seed;
    const double* spawn_table;   /* [n_scen][n_cows][2] */
    int32_t spawn_scenarios, spawn_cows;
    int32_t marl_wrapper;     /* MARL: 1 = RLlibMultiAgentWrapper.step semantics, 0 = bare env.step */
    int32_t physics;          /* Physics enum order (utils/enums.py:13-21): 0 PYB, 1 DYN, 2 PYB_GND,
                                 3 PYB_DRAG, 4 PYB_DW, 5 PYB_GND_DRAG_DW */
    int32_t link_lag;         /* 1 = applyExternalForce/Torque(LINK_FRAME) on the drone's links rotate by the
                                 link transform Bullet cached at the previous substep (qlag); pinned by the
                                 real-PyBullet trace.  0 = the current attitude (rounds 1-4) */
} och_config;

typedef struct och_state {
    int32_t n;                          /* NUM_DRONES this episode */
    double dp[OCH_NMAX][3], dq[OCH_NMAX][4], dv[OCH_NMAX][3], dw[OCH_NMAX][3];
    double pid_last_rpy[OCH_NMAX][3], pid_int_pos[OCH_NMAX][3], pid_int_rpy[OCH_NMAX][3];
    double cp[OCH_MMAX][2], cv[OCH_MMAX][2];
    int64_t step_counter, step_counter_A;
    double prev_cent; int32_t has_prev;
    double clock; int32_t level, tally, spawn_index;
    uint8_t active[OCH_NMAX];
    int64_t episode;                    /* resets so far (Philox counter for reset draws) */
    int64_t env_id;                     /* global env index (Philox key part) */
    double last_rpm[OCH_NMAX][4];       /* last_clipped_action (BaseAviary.py:450, 565): drag input */
    double rpy_rates[OCH_NMAX][3];      /* DYN body rates (BaseAviary.py:581-582, 1075) */
    double eval_dist[OCH_NMAX];         /* update_evaluation_metrics' episode distance (BaseAviary.py:1415-1426) */
    double qlag[OCH_NMAX][4];           /* attitude at the start of the previous substep: the frame of the prop and
                                           centre-of-mass links' cached world transforms (link_lag) */
} och_state;

#ifdef __cplusplus
extern "C" {
#endif
/* pieces (unit-tested against individual golden vectors) */
void och_flock_update(const double* cp, const double* cv, int m, const double* dxy, int n, double* new_cv);
double och_effectiveness(const double* cxy, int m, const double* dxy, int n);
void och_euler_from_quat(const double* q, double* rpy);
void och_matrix_from_quat(const double* q, double* R);
void och_pid_vel(const double* pos, const double* quat, const double* vel, const double* target_pos,
                 const double* target_rpy, const double* target_vel, double dt,
                 double* last_rpy, double* int_pos, double* int_rpy, double* rpm);
double och_simple_spacing(double r, int level);
double och_complex_spacing(double r, int level);
double och_cattle_spacing(double r);
double och_gnd_eff_h_clip(void);   /* BaseAviary.py:173 */
void och_dyn_integrate(double* y, const double* rpm, double dt, int64_t steps, int rk4);   /* DYN / RK4 probe */

/* whole env */
int  och_obs_rows(const och_config* c);
void och_obs(const och_config* c, const och_state* s, float* obs);
void och_reset(const och_config* c, och_state* s);
void och_init(const och_config* c, och_state* s, int64_t env_id);
/* reward/terminated/truncated sized K = 1 (CTDE) or n_ctor (MARL); returns 1 if the env auto-resets */
int  och_step(const och_config* c, och_state* s, const float* actions, float* obs, double* reward,
              uint8_t* terminated, uint8_t* truncated, float* terminal_obs, int autoreset);
void och_task(const och_config* c, och_state* s, double* reward, uint8_t* terminated, uint8_t* truncated);
void och__set_target_vel(const double* tv);   /* test hook: float64 PID target velocities, NULL = off */
void och__set_model_flags(int f);            /* test hook: alternative rigid-body models (trace inversion) */
void och_random_actions(const och_config* c, int64_t env_id, int64_t step, float* actions);
/* CPU baseline: E envs x T steps of random-action rollout, OpenMP over envs; returns seconds */
double och_batch_rollout(const och_config* c, och_state* states, int64_t E, int64_t T, int threads);
#ifdef __cplusplus
}
#endif
#endif
