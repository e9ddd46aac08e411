// ch_internal.h — shared between the C-ABI implementation (ch_api.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cattleherd.h"

namespace ch {

constexpr int kNMax = 12;          // GLOBAL_MAX_NUM_DRONES (BaseAviary.py:112)
constexpr int kMMax = 64;          // cattle per env supported by the team mapping (TEAM <= 64)
constexpr int kDroneComps = 22;    // px py pz qx qy qz qw vx vy vz wx wy wz pid[9]
constexpr int kCattleComps = 4;    // x y vx vy
constexpr int kEnvReal = 2;        // prev_cent, clock
constexpr int kEnvInt = 10;        // n sc scA has_prev level tally spawn active episode reserved
constexpr int kMetricCurReturn = CH_METRIC_COUNT;      // running episode return
constexpr int kMetricCurLen = CH_METRIC_COUNT + 1;     // running episode length
constexpr int kMetricRows = CH_METRIC_COUNT + 2;

template <class R>
struct StepParams {
    int E, NC, M, mode, rows;
    int min_drones, max_drones, ctrl_freq, substeps, compat, torque_world, gyro, marl_wrapper;
    double episode_len, damping, dt_ctrl, dt;
    uint32_t k0, k1;
    long long env_off, step_index;
    R* drone;       // [22][E][NC]
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
    const uint8_t* reset_mask;
    uint32_t flags;
    double* debug;  // optional [E][NC][16] per-drone intermediates (diagnostics only)
    int phase_mask; // diagnostics only: skip phases (1 drones, 2 flock, 4 task, 8 obs) for time attribution
};

template <class R> hipError_t launch_step(const StepParams<R>& p, int team, hipStream_t st);
template <class R> hipError_t launch_reset(const StepParams<R>& p, int team, hipStream_t st);

}  // namespace ch
