// ch_api.cpp — C ABI of libcattleherd.so (see include/cattleherd.h).
//
// Host side: validates the configuration the way the reference's constructors do, owns the SoA
// state in HBM, and launches the kernels in ch_kernels.hip.  No host<->device traffic on the
// ch_step path: actions, observations, rewards and flags stay in caller-owned device buffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "ch_internal.h"
#include "ch_spawn_table.inc"

using namespace ch;

struct ch_handle {
    ch_config cfg{};
    int64_t E = 0;
    int device = 0;
    int NC = 0, M = 0, rows = 0, K = 0, team = 0;
    int start_level = 0;
    double episode_len = 0;
    size_t rsize = 8;
    void* drone = nullptr;
    // Euler angles of each drone's stored quaternion, written by the v2 step at the end of every
    // step (it needs them for the observation anyway) and read by the next one instead of
    // recomputing atan2/asin/atan2; any other writer of the state clears rpy_valid.
    void* rpy = nullptr;
    uint8_t* stale = nullptr;   // device [2][E]: StepParams::stale (Euler cache stale, obs bytes unknown, per env)
    unsigned long long* obs_tag = nullptr;   // device [E]: StepParams::obs_tag (the buffer holding env e's constant obs bytes)
    void* cattle = nullptr;
    void* phys = nullptr;   // [kPhysComps][E][NC]: last_clipped_action, DYN rpy_rates
    void* envr = nullptr;
    // f32 mode only: the f64 copies of the positions and prev_cent_dists the step integrates and measures
    // centroids on (StepParams::pos64 / cpos64 / prev64); the f32 arrays above keep their rounded values
    double* pos64 = nullptr;    // [3][E][NC]
    double* cpos64 = nullptr;   // [2][E][M]
    double* prev64 = nullptr;   // [E]
    int* envi = nullptr;
    double* metrics = nullptr;
    double* spawn = nullptr;
    int n_scen = 0, n_cows = 0;
    double* debug = nullptr;
    int phase_mask = 0;
    // The obs buffer whose constant-zero bytes (rows >= NUM_DRONES, the action-buffer block, padding)
    // are known to hold zeros: the last one a full-block writer (v1 step, full ch_reset, v2 step with
    // obs_full) wrote.  The v2 step then stores only the entries that change.
    const float* obs_zero_ptr = nullptr;
    // v2 step kernel (ch_step.hip): envs per workgroup, block size, dynamic LDS, cow-pair list
    int kernel = 2;
    long long* tstamp = nullptr;
    int G = 1, block = 64, P = 0;
    bool pw = false;   // v2 with per-wave env tables (herds of kPwMinCattle cows and more)
    bool sep = false;  // v2 shared tables with the shepherd terms in their own LDS region
    size_t lds = 0;
    uint16_t* pairs = nullptr;
    int* errw = nullptr;        // device error word (CH_DEVERR_* bits), sticky
    double* evald = nullptr;    // [E][NC] evaluation distances (cfg.eval_metrics)
    int* rdn = nullptr;         // ch_reset_with: device copies of the injected draws
    double* rdv = nullptr;
    double* mdev = nullptr;     // device [CH_METRIC_COUNT + 1]: reduced metrics + error word
    double* mhost = nullptr;    // pinned host copy of mdev
    // ch_rollout_collect's deferred-bootstrap queue (allocated on first use): terminal observations, their rewards
    // rows, the count, the values
    float* tv_obs = nullptr;
    long long* tv_row = nullptr;
    int* tv_count = nullptr;
    float* tv_val = nullptr;
    size_t tv_obs_n = 0, tv_val_n = 0;
    // ch_rollout_collect's path (diagnostics / tests, ch__set_rollout_path): bit 0 copy every step's observation into
    // the buffer instead of stepping into its slots, bit 1 the stand-alone store kernel instead of the forward epilogues,
    // bit 2 the actor forward fused into the step kernel (k_step2_actor, where the geometry takes it), bit 3 never fused
    int rollout_path = 0;
    long long fused_steps = 0;   // fused steps launched by ch_rollout_collect (ch__rollout_fused_steps)
    long long multi_steps = 0;   // steps ch_step_n ran inside k_step2_multi (ch__multi_steps)
    void* d_params = nullptr;    // k_step2_multi's parameters (device copy, ch_step_n)
    std::vector<unsigned char> params_host;   // what d_params holds (uploaded again only when the parameters change)
    // ch_outputs_to_host's device staging of the envs that auto-reset (allocated on first use): count, indices,
    // episode statistics, terminal observation blocks; and the pinned host copy of the count
    long long* st_count = nullptr;
    long long* st_env = nullptr;
    double* st_stats = nullptr;
    float* st_obs = nullptr;
    long long* st_count_host = nullptr;
    // how many ended envs ch_outputs_to_host copies before it knows the count: twice the larger of the last count and
    // its running mean, plus 8 (a step where more end costs one more copy and stream sync)
    double ended_mean = 8.0;
    int64_t ended_last = 8;
    // the device error word was reported to the caller (device_status) since it was last cleared
    bool err_seen = false;
    std::string err;
};

static thread_local std::string g_create_err;

static int fail(ch_handle* h, int code, const std::string& msg) {
    if (h) h->err = msg; else g_create_err = msg;
    return code;
}

#define HIP_TRY(h, expr)                                                                           \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess)                                                                      \
            return fail((h), CH_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));   \
    } while (0)

// episode_length per curriculum level (curriculum_learning.py:24-182)
static const double kEpisodeLen[8] = {40, 40, 40, 40, 80, 40, 80, 80};
static const int kLevelMin[8] = {3, 4, 4, 4, 4, 4, 4, 4};
static const int kLevelMax[8] = {3, 4, 4, 4, 4, 4, 12, 12};

// --------------------------------------------------------------------------------------------
// Spawn table.  Cows 0..15 of every scenario come from config/cattle_positions.yaml (the
// reference's only table, BaseAviary.py:88-94, 600-637).  For num_cattle > 16 (beyond what the
// reference can run, BaseAviary.py:611,719) extra cows are drawn around the scenario's herd
// centroid with the generator's rules (utils/cattle_spawn.py:5-12: min spacing 0.8, uniform
// offsets), the offset box widened by 1.25 sqrt(cows/16), rounded to 3 decimals, from a fixed-seed
// splitmix64 stream — deterministic and identical for every caller.
// --------------------------------------------------------------------------------------------
static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static std::vector<double> make_spawn_table(int cows) {
    const int S = CH_SPAWN_SCENARIOS, C0 = CH_SPAWN_COWS;
    const int C = std::max(cows, C0);
    std::vector<double> t((size_t)S * C * 2);
    for (int s = 0; s < S; ++s) {
        double cx = 0, cy = 0;
        for (int j = 0; j < C0; ++j) {
            t[((size_t)s * C + j) * 2] = CH_SPAWN_TABLE[(s * C0 + j) * 2];
            t[((size_t)s * C + j) * 2 + 1] = CH_SPAWN_TABLE[(s * C0 + j) * 2 + 1];
            cx += CH_SPAWN_TABLE[(s * C0 + j) * 2];
            cy += CH_SPAWN_TABLE[(s * C0 + j) * 2 + 1];
        }
        cx /= C0; cy /= C0;
        uint64_t st = 0xC0FFEEull * (s + 1);
        double half = 2.5 * std::sqrt((double)C / C0), mind = 0.8;
        for (int j = C0; j < C; ++j) {
            for (int attempt = 0;; ++attempt) {
                if (attempt > 0 && attempt % 2000 == 0) mind *= 0.95;
                double ox = ((splitmix(st) >> 11) * (1.0 / 9007199254740992.0) * 2 - 1) * half;
                double oy = ((splitmix(st) >> 11) * (1.0 / 9007199254740992.0) * 2 - 1) * half;
                double x = std::round((cx + ox) * 1000.0) / 1000.0, y = std::round((cy + oy) * 1000.0) / 1000.0;
                bool ok = true;
                for (int k = 0; k < j && ok; ++k) {
                    double dx = x - t[((size_t)s * C + k) * 2], dy = y - t[((size_t)s * C + k) * 2 + 1];
                    ok = std::sqrt(dx * dx + dy * dy) >= mind;
                }
                if (ok) { t[((size_t)s * C + j) * 2] = x; t[((size_t)s * C + j) * 2 + 1] = y; break; }
            }
        }
    }
    return t;
}

// CattleSpacingRewardFunction (CattleAviary.py:572-592), r > r0 branch: C = f(r0) / exp(-lambda r0) is the
// same number on every call; evaluated once here with the reference's expression.
static double cattle_spacing_cc() {
    const double A = 1.2, B = 2.1, C = 3.3, K = 0.2, D = -1, R0 = 1.3, LAM = 0.8;
    volatile double r0 = R0;   // evaluate at run time with the host libm, as the reference (and the oracle) do
    double fr0 = A * std::exp(-((r0 - D) * (r0 - D)) / (2 * (C * C))) - B * std::exp(-(r0 * r0) / (2 * (K * K)));
    return fr0 / std::exp(-LAM * r0);
}

// GND_EFF_H_CLIP (BaseAviary.py:163-173): 0.25 r_prop sqrt(15 MAX_RPM^2 KF c_gnd / MAX_THRUST), cf2x.urdf:5
static double gnd_eff_h_clip() {
    const double G = 9.8, MASS = 0.027, KF = 3.16e-10, T2W = 2.25, C = 11.36859, PR = 2.31348e-2;
    const double max_rpm = std::sqrt((T2W * (G * MASS)) / (4 * KF));
    const double max_thrust = 4 * KF * (max_rpm * max_rpm);
    return 0.25 * PR * std::sqrt((15 * (max_rpm * max_rpm) * KF * C) / max_thrust);
}

template <class R>
static StepParams<R> params(ch_handle* h) {
    StepParams<R> p{};
    const ch_config& c = h->cfg;
    p.E = (int)h->E; p.NC = h->NC; p.M = h->M; p.mode = c.mode; p.rows = h->rows;
    p.min_drones = c.min_drones; p.max_drones = c.max_drones; p.ctrl_freq = c.ctrl_freq;
    p.substeps = c.pyb_freq / c.ctrl_freq; p.compat = c.compat; p.torque_world = c.torque_world; p.gyro = c.gyro;
    p.link_lag = c.link_lag;
    p.marl_wrapper = c.marl_wrapper;
    p.episode_len = h->episode_len; p.damping = c.damping;
    p.dt_ctrl = 1.0 / c.ctrl_freq; p.dt = 1.0 / c.pyb_freq;
    p.k0 = (uint32_t)c.seed; p.k1 = (uint32_t)(c.seed >> 32);
    p.env_off = c.env_id_offset;
    p.cs_cc = cattle_spacing_cc();
    p.drone = (R*)h->drone; p.rpy = (R*)h->rpy; p.stale = h->stale; p.obs_tag = h->obs_tag; p.cattle = (R*)h->cattle; p.envr = (R*)h->envr; p.envi = h->envi;
    p.pos64 = h->pos64; p.cpos64 = h->cpos64; p.prev64 = h->prev64;
    p.metrics = h->metrics; p.spawn = h->spawn; p.n_scen = h->n_scen; p.n_cows = h->n_cows;
    p.debug = h->debug;
    p.phase_mask = h->phase_mask;
    p.G = h->G; p.P = h->P; p.pairs = h->pairs; p.pw = h->pw; p.sep = h->sep;
    p.tstamp = h->tstamp;
    p.physics = c.physics; p.gnd_h_clip = gnd_eff_h_clip(); p.phys = (R*)h->phys;
    p.err = h->errw;
    p.evald = h->evald;
    return p;
}

// the v2 step's once-per-device function attribute, set outside any stream capture
static hipError_t prepare_step(ch_handle* h) {
    if (h->kernel != 2) return hipSuccess;
    if (h->rsize == sizeof(double)) return launch_step_v2(params<double>(h), h->block, h->lds, nullptr, false);
    return launch_step_v2(params<float>(h), h->block, h->lds, nullptr, false);
}

extern "C" {

int ch_builtin_spawn_table(double* out, int32_t* scenarios, int32_t* cows) {
    if (scenarios) *scenarios = CH_SPAWN_SCENARIOS;
    if (cows) *cows = CH_SPAWN_COWS;
    if (out) std::memcpy(out, CH_SPAWN_TABLE, sizeof(CH_SPAWN_TABLE));
    return CH_OK;
}

int ch_spawn_table(int32_t cows, double* out, int32_t* scenarios, int32_t* out_cows) {
    std::vector<double> t = make_spawn_table(cows);
    int C = std::max(cows, (int)CH_SPAWN_COWS);
    if (scenarios) *scenarios = CH_SPAWN_SCENARIOS;
    if (out_cows) *out_cows = C;
    if (out) std::memcpy(out, t.data(), t.size() * sizeof(double));
    return CH_OK;
}

int ch_default_config(ch_config* c, int32_t mode, int32_t num_drones, int32_t num_cattle) {
    if (!c) return fail(nullptr, CH_ERR_INVALID, "ch_default_config: cfg is NULL");
    std::memset(c, 0, sizeof(*c));
    c->abi_version = CH_ABI_VERSION;
    c->mode = mode;
    c->num_drones = num_drones;
    c->num_cattle = num_cattle;
    c->min_drones = -1;
    c->max_drones = -1;
    c->curriculum_level = -1;
    c->ctrl_freq = 60;
    c->pyb_freq = 240;
    c->compat = 1;
    c->precision = CH_PREC_F64;
    c->torque_world = 1;
    c->gyro = 1;
    c->marl_wrapper = 1;
    c->damping = 0.04;
    c->seed = 0x5EEDull;
    c->env_id_offset = 0;
    c->spawn_table = nullptr;
    c->physics = CH_PHYS_PYB;
    c->eval_metrics = 1;
    c->link_lag = 1;
    return CH_OK;
}

const char* ch_last_error(const ch_handle* h) { return h ? h->err.c_str() : g_create_err.c_str(); }

constexpr size_t kParamsBytes = 1024;   // ch_step_n's device copy of StepParams

static void free_all(ch_handle* h) {
    void* ptrs[] = {h->drone, h->rpy, h->cattle, h->phys, h->envr, h->envi, h->metrics, h->spawn, h->pairs,
                    h->errw, h->mdev, h->stale, h->obs_tag, h->evald, h->rdn, h->rdv, h->pos64, h->cpos64, h->prev64,
                    h->d_params};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (void* p : {(void*)h->tv_obs, (void*)h->tv_row, (void*)h->tv_count, (void*)h->tv_val, (void*)h->st_count,
                    (void*)h->st_env, (void*)h->st_stats, (void*)h->st_obs})
        if (p) (void)hipFree(p);
    if (h->mhost) (void)hipHostFree(h->mhost);
    if (h->st_count_host) (void)hipHostFree(h->st_count_host);
}

// the sticky device error word as a status (call after the stream has drained)
static int device_status(ch_handle* h, int word) {
    if (!word) return CH_OK;
    h->err_seen = true;
    return fail(h, CH_ERR_DEVICE,
                "device error word " + std::to_string(word) +
                    ((word & CH_DEVERR_HANDOFF) ? ": a step kernel's LDS hand-off timed out (ch_step.hip lds_wait); "
                                                  "the results of that step are wrong"
                                                : ""));
}

int ch_create(const ch_config* c, int64_t n_envs, int32_t device, ch_handle** out) {
    if (!c || !out) return fail(nullptr, CH_ERR_INVALID, "ch_create: NULL argument");
    *out = nullptr;
    if (c->abi_version != CH_ABI_VERSION) return fail(nullptr, CH_ERR_INVALID, "ch_create: abi_version mismatch");
    if (c->mode != CH_MODE_CTDE && c->mode != CH_MODE_MARL) return fail(nullptr, CH_ERR_INVALID, "ch_create: bad mode");
    if (c->physics < CH_PHYS_PYB || c->physics > CH_PHYS_DYN_RK4)
        return fail(nullptr, CH_ERR_INVALID, "ch_create: physics must be one of CH_PHYS_* (utils/enums.py:13-21)");
    if (n_envs <= 0 || n_envs > (1ll << 28)) return fail(nullptr, CH_ERR_INVALID, "ch_create: n_envs out of range");
    if (c->num_drones < 1 || c->num_drones > kNMax)
        return fail(nullptr, CH_ERR_INVALID, "ch_create: num_drones must be in [1, 12] (GLOBAL_MAX_NUM_DRONES)");
    if (c->num_cattle < 1 || c->num_cattle > kMMax)
        return fail(nullptr, CH_ERR_INVALID, "ch_create: num_cattle must be in [1, 64]");
    if (c->ctrl_freq <= 0 || c->pyb_freq <= 0 || c->pyb_freq % c->ctrl_freq != 0)
        return fail(nullptr, CH_ERR_INVALID, "[ERROR] in BaseAviary.__init__(), pyb_freq is not divisible by env_freq.");
    if (c->precision != CH_PREC_F64 && c->precision != CH_PREC_F32)
        return fail(nullptr, CH_ERR_INVALID, "ch_create: bad precision");
    int level = c->curriculum_level < 0 ? (c->mode == CH_MODE_CTDE ? 7 : 0) : c->curriculum_level;
    if (level > 7) return fail(nullptr, CH_ERR_INVALID, "ch_create: curriculum_level must be in [0, 7]");
    int mn = c->min_drones < 0 ? c->num_drones : c->min_drones;
    int mx = c->max_drones < 0 ? c->num_drones : c->max_drones;
    if (mn < 1 || mx < mn || mx > c->num_drones)
        return fail(nullptr, CH_ERR_INVALID,
                    "ch_create: need 1 <= min_drones <= max_drones <= num_drones (the reference indexes "
                    "self.ctrl[k] sized by num_drones, BaseRLAviary.py:80)");
    if (c->compat && mn < 2)
        return fail(nullptr, CH_ERR_UNSUPPORTED,
                    "compat mode: the reference raises ValueError for a single drone (np.partition kth=1, "
                    "CattleAviary.py:234); use compat=0");
    if (c->spawn_table && (c->spawn_scenarios < 1 || c->spawn_cows < c->num_cattle))
        return fail(nullptr, CH_ERR_INVALID, "ch_create: spawn table smaller than num_cattle");
    int dev_count = 0;
    hipError_t ge = hipGetDeviceCount(&dev_count);
    if (ge != hipSuccess || dev_count == 0)
        return fail(nullptr, CH_ERR_DEVICE, std::string("ch_create: no HIP device: ") + hipGetErrorString(ge));
    if (device < 0 || device >= dev_count) return fail(nullptr, CH_ERR_INVALID, "ch_create: bad device index");

    ch_handle* h = new (std::nothrow) ch_handle();
    if (!h) return fail(nullptr, CH_ERR_NOMEM, "ch_create: out of host memory");
    h->cfg = *c;
    h->cfg.curriculum_level = level;
    h->cfg.min_drones = mn;
    h->cfg.max_drones = mx;
    h->E = n_envs;
    h->device = device;
    h->NC = c->num_drones;
    h->M = c->num_cattle;
    h->rows = c->mode == CH_MODE_CTDE ? 12 : c->num_drones;
    h->K = c->mode == CH_MODE_CTDE ? 1 : c->num_drones;
    int need = std::max(h->NC, h->M);
    h->team = need <= 16 ? 16 : (need <= 32 ? 32 : 64);
    h->start_level = level;
    h->episode_len = kEpisodeLen[level];
    h->rsize = c->precision == CH_PREC_F64 ? sizeof(double) : sizeof(float);
    h->P = h->M * (h->M - 1) / 2;
    (void)kLevelMin; (void)kLevelMax;
    {   // ch_rollout_collect's path: the environment's choice, ch__set_rollout_path overrides it per handle
        const char* v = getenv("CH_ROLLOUT_COPY");
        const char* k = getenv("CH_ROLLOUT_STORE_KERNEL");
        const char* f = getenv("CH_FUSED_ACTOR");
        h->rollout_path = ((v && v[0] == '1') ? 1 : 0) | ((k && k[0] == '1') ? 2 : 0) | ((f && f[0] == '1') ? 4 : 0);
    }

    auto cleanup = [&](int code) { free_all(h); std::string m = h->err; delete h; g_create_err = m; return code; };
#define CTRY(expr)                                                                                  \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess) {                                                                     \
            h->err = std::string(#expr) + ": " + hipGetErrorString(_e);                             \
            return cleanup(_e == hipErrorOutOfMemory ? CH_ERR_NOMEM : CH_ERR_DEVICE);               \
        }                                                                                           \
    } while (0)
    CTRY(hipSetDevice(device));
    const int64_t E = h->E;
    CTRY(hipMalloc(&h->drone, h->rsize * kDroneComps * E * h->NC));
    CTRY(hipMalloc(&h->rpy, h->rsize * 3 * E * h->NC));
    CTRY(hipMalloc(&h->cattle, h->rsize * kCattleComps * E * h->M));
    CTRY(hipMalloc(&h->phys, h->rsize * kPhysComps * E * h->NC));
    CTRY(hipMemset(h->phys, 0, h->rsize * kPhysComps * E * h->NC));
    CTRY(hipMalloc(&h->envr, h->rsize * kEnvReal * E));
    if (h->rsize == sizeof(float)) {
        CTRY(hipMalloc(&h->pos64, sizeof(double) * 3 * E * h->NC));
        CTRY(hipMalloc(&h->cpos64, sizeof(double) * 2 * E * h->M));
        CTRY(hipMalloc(&h->prev64, sizeof(double) * E));
    }
    CTRY(hipMalloc(&h->envi, sizeof(int) * kEnvInt * E));
    CTRY(hipMalloc(&h->metrics, sizeof(double) * kMetricRows * E));
    {
        CTRY(hipMalloc(&h->stale, 2 * (size_t)E));
        CTRY(hipMemset(h->stale, 1, 2 * (size_t)E));   // no Euler cache yet; obs bytes unknown
        CTRY(hipMalloc(&h->obs_tag, sizeof(unsigned long long) * (size_t)E));
        CTRY(hipMemset(h->obs_tag, 0, sizeof(unsigned long long) * (size_t)E));   // no buffer holds them
    }
    if (c->eval_metrics) {
        CTRY(hipMalloc(&h->evald, sizeof(double) * E * h->NC));
        CTRY(hipMemset(h->evald, 0, sizeof(double) * E * h->NC));
    }
    CTRY(hipMalloc(&h->errw, sizeof(int)));
    CTRY(hipMemset(h->errw, 0, sizeof(int)));
    CTRY(hipMalloc(&h->mdev, sizeof(double) * (CH_METRIC_COUNT + 1)));
    CTRY(hipHostMalloc(&h->mhost, sizeof(double) * (CH_METRIC_COUNT + 1), hipHostMallocDefault));

    std::vector<double> table;
    if (c->spawn_table) {
        table.assign(c->spawn_table, c->spawn_table + (size_t)c->spawn_scenarios * c->spawn_cows * 2);
        h->n_scen = c->spawn_scenarios;
        h->n_cows = c->spawn_cows;
    } else {
        table = make_spawn_table(h->M);
        h->n_scen = CH_SPAWN_SCENARIOS;
        h->n_cows = std::max(h->M, (int)CH_SPAWN_COWS);
    }
    CTRY(hipMalloc(&h->spawn, table.size() * sizeof(double)));
    {
        // v2 geometry: G envs per workgroup with all G*N drone chains in wave 0, the LDS
        // carve within the per-CU budget, and at least one workgroup per CU when E allows it.
        int cus = 256, lds_max = 64 * 1024;
        CTRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        if (hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device) != hipSuccess)
            lds_max = 64 * 1024;
        const size_t budget = std::min<size_t>((size_t)lds_max, 160 * 1024);
        // a drone wave (G*N <= 64 drone chains) plus three cow waves (G*M cows, one per lane when it fits)
        int G = std::max(1, std::min(64 / h->NC, 192 / h->M));
        G = (int)std::min<int64_t>(G, std::max<int64_t>(1, E / std::max(cus, 1)));
        while (G & (G - 1)) G &= G - 1;   // power of two: whole workgroups per CU at E = 2^k
        while (G > 1 && V2Layout(G, h->NC, h->M, h->P, c->mode, (int)h->rsize).bytes() > budget) --G;
        h->G = G;
        h->lds = V2Layout(G, h->NC, h->M, h->P, c->mode, (int)h->rsize).bytes();
        h->block = 256;
        // measured (tools/geom_sweep.py, profiles/r02/geom_*.log): at 4 drones x 16 cattle one workgroup
        // of 16 envs per CU (a full 64-drone wave + cow waves sharing the work counters) beats two of 8
        // envs, and 11 cow waves (768 threads, 3 waves per SIMD) edge out 7 (24.1 vs 24.8 us at 4096 envs);
        // the physics variants keep 512 (their register use allows 2 waves per SIMD)
        if (c->mode == CH_MODE_CTDE && h->NC == 4 && h->M == 16 && E >= 16 * (int64_t)cus &&
            V2Layout(16, 4, 16, h->P, c->mode, (int)h->rsize).bytes() <= budget) {
            h->G = 16;
            h->lds = V2Layout(16, 4, 16, h->P, c->mode, (int)h->rsize).bytes();
            // f32: 512 threads (tools/f32_geom_probe.py: 419 vs 273 M env-steps/s at 262144 envs, 1.5 % slower
            // at 4096; f64 keeps 768, 230 vs 225 M at 262144 and 1 % faster at 4096)
            h->block = (c->physics == CH_PHYS_PYB && h->rsize == 8) ? CH_V2_MAX_BLOCK : CH_V2_MAX_BLOCK_PW;
        }
        // 2 drones x 8 cattle (configs[1]/[2]), f64: 16 envs / 512 threads per workgroup from 1024 envs up, also when
        // that leaves CUs idle (configs[1]: 64 workgroups) -- tools/multi_geom.py, profiles/r06/ab/r6y_*: at 1024 envs
        // 78.1 vs 76.4 M env-steps/s (ch_step_n) and 61.8 vs 58.5 M (ch_step) against 4 envs / 256 threads; at 4096
        // envs 311.9 vs 311.0 M and 238.3 vs 229.4 M against 16 envs / 256 threads
        if (c->mode == CH_MODE_CTDE && h->NC == 2 && h->M == 8 && h->rsize == 8 && c->physics == CH_PHYS_PYB &&
            E >= 1024 && V2Layout(16, 2, 8, h->P, c->mode, (int)h->rsize).bytes() <= budget) {
            h->G = 16;
            h->lds = V2Layout(16, 2, 8, h->P, c->mode, (int)h->rsize).bytes();
            h->block = CH_V2_MAX_BLOCK_PW;
        }
        // measured (tools/ab/marl.py, MI355X, 4096 envs): the dataflow kernel wins for every CTDE size
        // (2x8 19.4 vs 41.1 us, 8x16 39.7 vs 55.8, 12x16 59.9 vs 67.1) and for MARL with up to 16
        // cattle (3x8 25.8 vs 43.2).  Above 16 cows one shared pair table per workgroup (15.9 KB per
        // env at 32 cows) leaves room for 4 envs per CU; the per-wave env tables (V2Layout W) keep a
        // CU's 16 envs in one workgroup instead.
        if (h->M >= kPwMinCattle) {
            h->kernel = 1;   // unless a per-wave geometry fits (physics variants stay on v1)
            if (c->physics == CH_PHYS_PYB) {
                const int cand[][2] = {{16, 512}, {8, 512}, {8, 256}, {4, 256}, {2, 128}, {1, 128}};
                for (const auto& gb : cand) {
                    const int g = gb[0], blk = gb[1];
                    if (g * h->NC > 64 || g * h->M > 3 * (blk - 64)) continue;
                    if (g > 1 && E < (int64_t)g * cus) continue;
                    const size_t l = V2Layout(g, h->NC, h->M, h->P, c->mode, (int)h->rsize, blk / 64 - 1).bytes();
                    if (l > budget) continue;
                    h->G = g; h->block = blk; h->lds = l; h->pw = true; h->kernel = 2;
                    break;
                }
            }
        }
        // shared tables: the shepherd terms in their own region when it fits, so they need not wait for every
        // alpha row to have read the pair table
        if (!h->pw) {
            const size_t l = V2Layout(h->G, h->NC, h->M, h->P, c->mode, (int)h->rsize, 0, true).bytes();
            if (l <= budget) { h->sep = true; h->lds = l; }
        }
        if (h->lds > budget) h->kernel = 1;   // one env's pair table alone exceeds the budget
        std::vector<uint16_t> pl((size_t)std::max(h->P, 1));
        for (int i = 0, r = 0; i < h->M; ++i)
            for (int j = i + 1; j < h->M; ++j) pl[r++] = (uint16_t)(i | (j << 8));
        CTRY(hipMalloc(&h->pairs, pl.size() * sizeof(uint16_t)));
        CTRY(hipMemcpy(h->pairs, pl.data(), pl.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    }
    CTRY(hipMemcpy(h->spawn, table.data(), table.size() * sizeof(double), hipMemcpyHostToDevice));

    // initial state = what the constructors leave behind before the first reset():
    // identity quaternions, zero PID state, spawn index advanced once by __init__'s _housekeeping.
    std::vector<double> dz((size_t)kDroneComps * E * h->NC, 0.0);
    for (int64_t i = 0; i < E * h->NC; ++i) {
        dz[(size_t)6 * E * h->NC + i] = 1.0;
        dz[(size_t)25 * E * h->NC + i] = 1.0;   // cached link frame: identity too
    }
    std::vector<int> ei((size_t)kEnvInt * E, 0);
    for (int64_t e = 0; e < E; ++e) {
        ei[4 * E + e] = level;
        ei[6 * E + e] = (int)((1 + c->env_id_offset + e) % h->n_scen);
    }
    int rc = 0;
    {
        std::vector<double> cz((size_t)kCattleComps * E * h->M, 0.0), rz((size_t)kEnvReal * E, 0.0);
        if (h->rsize == sizeof(double)) {
            CTRY(hipMemcpy(h->drone, dz.data(), dz.size() * 8, hipMemcpyHostToDevice));
            CTRY(hipMemcpy(h->cattle, cz.data(), cz.size() * 8, hipMemcpyHostToDevice));
            CTRY(hipMemcpy(h->envr, rz.data(), rz.size() * 8, hipMemcpyHostToDevice));
        } else {
            std::vector<float> f(dz.begin(), dz.end()), fc(cz.begin(), cz.end()), fr(rz.begin(), rz.end());
            CTRY(hipMemcpy(h->drone, f.data(), f.size() * 4, hipMemcpyHostToDevice));
            CTRY(hipMemcpy(h->cattle, fc.data(), fc.size() * 4, hipMemcpyHostToDevice));
            CTRY(hipMemcpy(h->envr, fr.data(), fr.size() * 4, hipMemcpyHostToDevice));
            CTRY(hipMemcpy(h->pos64, dz.data(), sizeof(double) * 3 * E * h->NC, hipMemcpyHostToDevice));
            CTRY(hipMemcpy(h->cpos64, cz.data(), sizeof(double) * 2 * E * h->M, hipMemcpyHostToDevice));
            CTRY(hipMemcpy(h->prev64, rz.data(), sizeof(double) * E, hipMemcpyHostToDevice));
        }
        CTRY(hipMemcpy(h->envi, ei.data(), ei.size() * sizeof(int), hipMemcpyHostToDevice));
        CTRY(hipMemset(h->metrics, 0, sizeof(double) * kMetricRows * E));
    }
    (void)rc;
    CTRY(prepare_step(h));
#undef CTRY
    *out = h;
    return CH_OK;
}

int ch_destroy(ch_handle* h) {
    if (!h) return CH_OK;
    (void)hipSetDevice(h->device);
    free_all(h);
    delete h;
    return CH_OK;
}

int ch_shape(const ch_handle* h, int64_t* n_envs, int32_t* obs_rows, int32_t* obs_cols, int32_t* reward_cols) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_shape: NULL handle");
    if (n_envs) *n_envs = h->E;
    if (obs_rows) *obs_rows = h->rows;
    if (obs_cols) *obs_cols = 86;
    if (reward_cols) *reward_cols = h->K;
    return CH_OK;
}

// A full reset rebuilds every env, so the results a failed hand-off spoiled are gone and the sticky device error word
// is cleared.  The word is read first (a stream sync: full resets are rare): if it was set and no ch_sync /
// ch_metrics / ch_get_state has reported it yet, the reset still happens but returns CH_ERR_DEVICE, so that the
// failure of the steps before it is never lost silently.
static int clear_error_word(ch_handle* h, hipStream_t st, const char* who) {
    int word = 0;
    HIP_TRY(h, hipStreamSynchronize(st));
    HIP_TRY(h, hipMemcpy(&word, h->errw, sizeof(int), hipMemcpyDeviceToHost));
    HIP_TRY(h, hipMemsetAsync(h->errw, 0, sizeof(int), st));
    const bool unseen = word && !h->err_seen;
    h->err_seen = false;
    if (unseen)
        return fail(h, CH_ERR_DEVICE, std::string(who) + ": the envs were reset, but the steps before it had set device "
                                          "error word " + std::to_string(word) + " (never reported: the results of "
                                          "those steps are wrong); the word is now cleared");
    return CH_OK;
}

int ch_reset(ch_handle* h, const uint8_t* mask_dev, float* obs_dev, void* stream) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_reset: NULL handle");
    if (!obs_dev) return fail(h, CH_ERR_INVALID, "ch_reset: obs is NULL");
    HIP_TRY(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    if (h->rsize == sizeof(double)) {
        StepParams<double> p = params<double>(h);
        p.reset_mask = mask_dev; p.obs = obs_dev;
        e = launch_reset(p, h->team, st);
    } else {
        StepParams<float> p = params<float>(h);
        p.reset_mask = mask_dev; p.obs = obs_dev;
        e = launch_reset(p, h->team, st);
    }
    if (e != hipSuccess) return fail(h, CH_ERR_DEVICE, std::string("ch_reset launch: ") + hipGetErrorString(e));
    if (!mask_dev) h->obs_zero_ptr = obs_dev;                    // every block written in full
    else if (h->obs_zero_ptr != obs_dev) h->obs_zero_ptr = nullptr;   // some blocks of obs_dev unknown
    return mask_dev ? CH_OK : clear_error_word(h, st, "ch_reset");
}

int ch_reset_with(ch_handle* h, const uint8_t* mask_dev, const int32_t* num_drones, const double* cow_vel,
                  float* obs_dev, void* stream) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_reset_with: NULL handle");
    if (!obs_dev) return fail(h, CH_ERR_INVALID, "ch_reset_with: obs is NULL");
    if (num_drones)
        for (int64_t e = 0; e < h->E; ++e)
            if (num_drones[e] < 1 || num_drones[e] > h->NC)
                return fail(h, CH_ERR_INVALID,
                            "ch_reset_with: NUM_DRONES " + std::to_string(num_drones[e]) + " outside [1, num_drones] "
                            "(the reference indexes controllers sized by num_drones, BaseRLAviary.py:80)");
    HIP_TRY(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    if (num_drones) {
        if (!h->rdn) HIP_TRY(h, hipMalloc(&h->rdn, sizeof(int) * h->E));
        HIP_TRY(h, hipMemcpyAsync(h->rdn, num_drones, sizeof(int) * h->E, hipMemcpyHostToDevice, st));
    }
    if (cow_vel) {
        if (!h->rdv) HIP_TRY(h, hipMalloc(&h->rdv, sizeof(double) * h->E * h->M * 2));
        HIP_TRY(h, hipMemcpyAsync(h->rdv, cow_vel, sizeof(double) * h->E * h->M * 2, hipMemcpyHostToDevice, st));
    }
    hipError_t e;
    if (h->rsize == sizeof(double)) {
        StepParams<double> p = params<double>(h);
        p.reset_mask = mask_dev; p.obs = obs_dev;
        p.reset_n = num_drones ? h->rdn : nullptr; p.reset_vel = cow_vel ? h->rdv : nullptr;
        e = launch_reset(p, h->team, st);
    } else {
        StepParams<float> p = params<float>(h);
        p.reset_mask = mask_dev; p.obs = obs_dev;
        p.reset_n = num_drones ? h->rdn : nullptr; p.reset_vel = cow_vel ? h->rdv : nullptr;
        e = launch_reset(p, h->team, st);
    }
    if (e != hipSuccess) return fail(h, CH_ERR_DEVICE, std::string("ch_reset_with launch: ") + hipGetErrorString(e));
    HIP_TRY(h, hipStreamSynchronize(st));   // the host arrays may be reused as soon as this returns
    if (!mask_dev) h->obs_zero_ptr = obs_dev;
    else if (h->obs_zero_ptr != obs_dev) h->obs_zero_ptr = nullptr;
    return mask_dev ? CH_OK : clear_error_word(h, st, "ch_reset_with");   // as ch_reset
}

extern "C++" template <class P>
static void fill_step(const ch_handle* h, const ch_step_io* io, P& p) {
    p.actions = io->actions; p.actions_out = io->actions_out; p.obs = io->obs; p.reward = io->reward;
    p.term = io->terminated; p.trunc = io->truncated; p.terminal_obs = io->terminal_obs;
    p.agent_active = io->agent_active; p.reset_happened = io->reset_happened; p.flags = io->flags;
    p.episode_stats = io->episode_stats;
    p.obs_full = io->obs != h->obs_zero_ptr;
}

// ch_rollout_collect's fused step (launch_step_v2_actor): the step of `io` with the actor forward `fa` on the
// observations it writes (fa.x == io->obs) and the sampling epilogue `ro`.  launch = false: hipSuccess iff the handle
// and the net fit the fused kernel (nothing launched).
static hipError_t step_actor(ch_handle* h, const ch_step_io* io, hipStream_t st, const MlpArgs& fa, const RolloutArgs& ro,
                             bool launch) {
    if (h->kernel != 2 || h->rsize != sizeof(double) || h->phase_mask) return hipErrorNotSupported;
    StepParams<double> p = params<double>(h);
    fill_step(h, io, p);
    const hipError_t e = launch_step_v2_actor(p, h->block, h->lds, st, fa, ro, launch);
    if (e == hipSuccess && launch) { h->obs_zero_ptr = io->obs; ++h->fused_steps; }
    return e;
}

int ch_step(ch_handle* h, const ch_step_io* io, void* stream) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_step: NULL handle");
    if (!io) return fail(h, CH_ERR_INVALID, "ch_step: io is NULL");
    if (!io->obs || !io->reward || !io->terminated || !io->truncated)
        return fail(h, CH_ERR_INVALID, "ch_step: obs, reward, terminated and truncated are required");
    if (!(io->flags & CH_STEP_RANDOM_ACTIONS) && !io->actions)
        return fail(h, CH_ERR_INVALID, "ch_step: actions is NULL (and CH_STEP_RANDOM_ACTIONS not set)");
    if (io->actions && (reinterpret_cast<uintptr_t>(io->actions) & 15))
        return fail(h, CH_ERR_INVALID, "ch_step: actions must be 16-byte aligned");
    if ((reinterpret_cast<uintptr_t>(io->obs) & 15) ||
        (io->terminal_obs && (reinterpret_cast<uintptr_t>(io->terminal_obs) & 15)))
        return fail(h, CH_ERR_INVALID, "ch_step: obs buffers must be 16-byte aligned");
    HIP_TRY(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    hipError_t e;
    auto fill = [&](auto& p) { fill_step(h, io, p); };
    if (h->rsize == sizeof(double)) {
        StepParams<double> p = params<double>(h);
        fill(p);
        e = h->kernel == 2 ? launch_step_v2(p, h->block, h->lds, st) : launch_step(p, h->team, st);
    } else {
        StepParams<float> p = params<float>(h);
        fill(p);
        e = h->kernel == 2 ? launch_step_v2(p, h->block, h->lds, st) : launch_step(p, h->team, st);
    }
    if (e != hipSuccess) return fail(h, CH_ERR_DEVICE, std::string("ch_step launch: ") + hipGetErrorString(e));
    h->obs_zero_ptr = (h->phase_mask & 8) ? nullptr : io->obs;
    // Which buffer holds each env's constant-zero obs bytes is also tracked on the device, per env: the step kernels
    // record the address they wrote (StepParams::obs_tag) and write an env's block in full when the buffer they are
    // given is not that one (k_step2 and k_env compare p.obs_tag[e] with p.obs), so a HIP graph captured on one
    // buffer and replayed after steps into another stays exact.  A new tensor at a recycled address is the caller's
    // to flag (HerdBatch.step(obs_out=...) calls invalidate_obs when the tensor changes).
    return CH_OK;
}

int ch_step_n(ch_handle* h, const ch_step_io* io, int32_t n_steps, void* stream) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_step_n: NULL handle");
    if (n_steps < 1) return fail(h, CH_ERR_INVALID, "ch_step_n: n_steps must be >= 1");
    if (!io) return fail(h, CH_ERR_INVALID, "ch_step_n: io is NULL");
    // the same validation as ch_step
    if (!io->obs || !io->reward || !io->terminated || !io->truncated)
        return fail(h, CH_ERR_INVALID, "ch_step_n: obs, reward, terminated and truncated are required");
    if (!(io->flags & CH_STEP_RANDOM_ACTIONS) && !io->actions)
        return fail(h, CH_ERR_INVALID, "ch_step_n: actions is NULL (and CH_STEP_RANDOM_ACTIONS not set)");
    if ((io->actions && (reinterpret_cast<uintptr_t>(io->actions) & 15)) || (reinterpret_cast<uintptr_t>(io->obs) & 15) ||
        (io->terminal_obs && (reinterpret_cast<uintptr_t>(io->terminal_obs) & 15)))
        return fail(h, CH_ERR_INVALID, "ch_step_n: actions and obs buffers must be 16-byte aligned");
    HIP_TRY(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    int done = 0, rc = CH_OK;
    // under stream capture: n_steps plain launches (a captured multi-step launch would read the handle's parameter copy
    // as a later call left it, and the upload's host source would not outlive the call)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cap) != hipSuccess) { (void)hipGetLastError(); cap = hipStreamCaptureStatusNone; }
    if (cap != hipStreamCaptureStatusNone) {
        for (int k = 0; k < n_steps; ++k)
            if ((rc = ch_step(h, io, stream)) != CH_OK) return rc;
        return CH_OK;
    }
    // a buffer whose constant observation bytes are not known to be in place gets one plain step first (it writes
    // them); every step of the multi-step kernel then finds them there
    if (io->obs != h->obs_zero_ptr || h->kernel != 2 || h->phase_mask) {
        if ((rc = ch_step(h, io, stream)) != CH_OK) return rc;
        done = 1;
    }
    if (done == n_steps) return CH_OK;
    const int rest = n_steps - done;
    hipError_t e = hipErrorNotSupported;
    if (h->kernel == 2 && !h->phase_mask) {
        // the multi-step kernel reads its parameters from a device copy (k_step2_multi), uploaded when they differ
        // from the last upload (stream-ordered; a pageable source is staged by the runtime before the call returns)
        if (!h->d_params) HIP_TRY(h, hipMalloc(&h->d_params, kParamsBytes));
        auto go = [&](auto p) -> hipError_t {
            fill_step(h, io, p);
            using P = decltype(p);
            static_assert(sizeof(P) <= kParamsBytes, "StepParams fits the device copy");
            const P* pd = static_cast<const P*>(h->d_params);
            if (launch_step_v2_multi(p, pd, h->block, h->lds, st, rest, false) != hipSuccess) return hipErrorNotSupported;
            if (h->params_host.size() != sizeof(P) || std::memcmp(h->params_host.data(), &p, sizeof(P)) != 0) {
                const hipError_t ce = hipMemcpyAsync(h->d_params, &p, sizeof(P), hipMemcpyHostToDevice, st);
                if (ce != hipSuccess) return ce;
                h->params_host.assign(reinterpret_cast<const unsigned char*>(&p),
                                      reinterpret_cast<const unsigned char*>(&p) + sizeof(P));
            }
            return launch_step_v2_multi(p, pd, h->block, h->lds, st, rest);
        };
        e = h->rsize == sizeof(double) ? go(params<double>(h)) : go(params<float>(h));
    }
    if (e == hipSuccess) {
        h->multi_steps += rest;
        h->obs_zero_ptr = io->obs;
        return CH_OK;
    }
    if (e != hipErrorNotSupported) return fail(h, CH_ERR_DEVICE, std::string("ch_step_n launch: ") + hipGetErrorString(e));
    (void)hipGetLastError();
    for (int k = 0; k < rest; ++k)   // other geometries: one launch per step
        if ((rc = ch_step(h, io, stream)) != CH_OK) return rc;
    return CH_OK;
}

/* Internal (tests): steps ch_step_n has run inside its multi-step kernel on this handle. */
int64_t ch__multi_steps(const ch_handle* h) { return h ? (int64_t)h->multi_steps : -1; }

int ch_state_size(const ch_handle* h, int64_t* n_doubles, int64_t* n_ints) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_state_size: NULL handle");
    if (n_doubles)
        *n_doubles = (int64_t)kDroneComps * h->E * h->NC + (int64_t)kCattleComps * h->E * h->M + kEnvReal * h->E +
                     (int64_t)kPhysComps * h->E * h->NC;
    if (n_ints) *n_ints = (int64_t)kEnvInt * h->E;
    return CH_OK;
}

int ch_get_state(ch_handle* h, double* hd, int32_t* hi, void* stream) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_get_state: NULL handle");
    HIP_TRY(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(h, hipStreamSynchronize(st));
    const size_t nd = (size_t)kDroneComps * h->E * h->NC, nc = (size_t)kCattleComps * h->E * h->M,
                 nr = (size_t)kEnvReal * h->E, np_ = (size_t)kPhysComps * h->E * h->NC;
    if (hd) {
        if (h->rsize == sizeof(double)) {
            HIP_TRY(h, hipMemcpy(hd, h->drone, nd * 8, hipMemcpyDeviceToHost));
            HIP_TRY(h, hipMemcpy(hd + nd, h->cattle, nc * 8, hipMemcpyDeviceToHost));
            HIP_TRY(h, hipMemcpy(hd + nd + nc, h->envr, nr * 8, hipMemcpyDeviceToHost));
            HIP_TRY(h, hipMemcpy(hd + nd + nc + nr, h->phys, np_ * 8, hipMemcpyDeviceToHost));
        } else {
            std::vector<float> f(nd + nc + nr + np_);
            HIP_TRY(h, hipMemcpy(f.data(), h->drone, nd * 4, hipMemcpyDeviceToHost));
            HIP_TRY(h, hipMemcpy(f.data() + nd, h->cattle, nc * 4, hipMemcpyDeviceToHost));
            HIP_TRY(h, hipMemcpy(f.data() + nd + nc, h->envr, nr * 4, hipMemcpyDeviceToHost));
            HIP_TRY(h, hipMemcpy(f.data() + nd + nc + nr, h->phys, np_ * 4, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < f.size(); ++i) hd[i] = f[i];
            // the positions and prev_cent_dists as the step holds them (f64)
            HIP_TRY(h, hipMemcpy(hd, h->pos64, sizeof(double) * 3 * h->E * h->NC, hipMemcpyDeviceToHost));
            HIP_TRY(h, hipMemcpy(hd + nd, h->cpos64, sizeof(double) * 2 * h->E * h->M, hipMemcpyDeviceToHost));
            HIP_TRY(h, hipMemcpy(hd + nd + nc, h->prev64, sizeof(double) * h->E, hipMemcpyDeviceToHost));
        }
    }
    if (hi) HIP_TRY(h, hipMemcpy(hi, h->envi, sizeof(int) * kEnvInt * h->E, hipMemcpyDeviceToHost));
    int word = 0;
    HIP_TRY(h, hipMemcpy(&word, h->errw, sizeof(int), hipMemcpyDeviceToHost));
    return device_status(h, word);
}

int ch_set_state(ch_handle* h, const double* hd, const int32_t* hi, void* stream) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_set_state: NULL handle");
    HIP_TRY(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(h, hipStreamSynchronize(st));
    h->obs_zero_ptr = nullptr;   // NUM_DRONES may change: the next step writes every obs block in full
    // the same on the device, for steps replayed from a graph captured earlier
    HIP_TRY(h, hipMemset(h->stale, 1, 2 * (size_t)h->E));
    const size_t nd = (size_t)kDroneComps * h->E * h->NC, nc = (size_t)kCattleComps * h->E * h->M,
                 nr = (size_t)kEnvReal * h->E, np_ = (size_t)kPhysComps * h->E * h->NC;
    if (hd) {
        if (h->rsize == sizeof(double)) {
            HIP_TRY(h, hipMemcpy(h->drone, hd, nd * 8, hipMemcpyHostToDevice));
            HIP_TRY(h, hipMemcpy(h->cattle, hd + nd, nc * 8, hipMemcpyHostToDevice));
            HIP_TRY(h, hipMemcpy(h->envr, hd + nd + nc, nr * 8, hipMemcpyHostToDevice));
            HIP_TRY(h, hipMemcpy(h->phys, hd + nd + nc + nr, np_ * 8, hipMemcpyHostToDevice));
        } else {
            std::vector<float> f(hd, hd + nd + nc + nr + np_);
            HIP_TRY(h, hipMemcpy(h->drone, f.data(), nd * 4, hipMemcpyHostToDevice));
            HIP_TRY(h, hipMemcpy(h->cattle, f.data() + nd, nc * 4, hipMemcpyHostToDevice));
            HIP_TRY(h, hipMemcpy(h->envr, f.data() + nd + nc, nr * 4, hipMemcpyHostToDevice));
            HIP_TRY(h, hipMemcpy(h->phys, f.data() + nd + nc + nr, np_ * 4, hipMemcpyHostToDevice));
            HIP_TRY(h, hipMemcpy(h->pos64, hd, sizeof(double) * 3 * h->E * h->NC, hipMemcpyHostToDevice));
            HIP_TRY(h, hipMemcpy(h->cpos64, hd + nd, sizeof(double) * 2 * h->E * h->M, hipMemcpyHostToDevice));
            HIP_TRY(h, hipMemcpy(h->prev64, hd + nd + nc, sizeof(double) * h->E, hipMemcpyHostToDevice));
        }
    }
    if (hi) HIP_TRY(h, hipMemcpy(h->envi, hi, sizeof(int) * kEnvInt * h->E, hipMemcpyHostToDevice));
    return CH_OK;
}

/* Internal, not part of the public ABI: device buffer [E][N][16] receiving per-drone PID intermediates. */
int ch__set_debug(ch_handle* h, double* dev) {
    if (!h) return CH_ERR_INVALID;
    h->debug = dev;
    return CH_OK;
}

/* Internal diagnostics: step kernel version (1 = team-per-env ch_kernels.hip, 2 = role-split ch_step.hip). */
int ch__set_kernel(ch_handle* h, int32_t version) {
    if (!h || (version != 1 && version != 2)) return CH_ERR_INVALID;
    if (version == 2 && h->lds > 160 * 1024) return CH_ERR_UNSUPPORTED;
    h->kernel = version;
    HIP_TRY(h, prepare_step(h));
    return CH_OK;
}

/* Internal diagnostics: device buffer [grid][16] of per-workgroup timestamps written by the v2 kernel. */
int ch__set_tstamp(ch_handle* h, long long* dev) {
    if (!h) return CH_ERR_INVALID;
    h->tstamp = dev;
    return CH_OK;
}

/* Internal diagnostics: override the v2 geometry (envs per workgroup, block size) for sweeps. */
int ch__set_geometry(ch_handle* h, int32_t G, int32_t block) {
    if (!h || G < 1 || G > 64 || G * h->NC > 64 || block < 128 || block % 64 ||
        block > ((h->pw || h->cfg.physics != CH_PHYS_PYB) ? CH_V2_MAX_BLOCK_PW : CH_V2_MAX_BLOCK))
        return CH_ERR_INVALID;
    if (G * h->M > 3 * (block - 64)) return CH_ERR_UNSUPPORTED;   // the cow waves prefetch <= 3 spawn slots per lane
    size_t lds = V2Layout(G, h->NC, h->M, h->P, h->cfg.mode, (int)h->rsize, h->pw ? block / 64 - 1 : 0).bytes();
    if (lds > 160 * 1024) return CH_ERR_UNSUPPORTED;
    bool sep = false;
    if (!h->pw) {
        const size_t l = V2Layout(G, h->NC, h->M, h->P, h->cfg.mode, (int)h->rsize, 0, true).bytes();
        if (l <= 160 * 1024) { sep = true; lds = l; }
    }
    h->G = G; h->block = block; h->lds = lds; h->sep = sep;
    HIP_TRY(h, prepare_step(h));
    return CH_OK;
}

/* Internal diagnostics: v2 geometry (envs per workgroup, block size, dynamic LDS bytes). */
int ch__geometry(const ch_handle* h, int32_t* G, int32_t* block, int64_t* lds, int32_t* kernel) {
    if (!h) return CH_ERR_INVALID;
    if (G) *G = h->G;
    if (block) *block = h->block;
    if (lds) *lds = (int64_t)h->lds;
    if (kernel) *kernel = h->kernel;
    return CH_OK;
}

/* Internal diagnostics: skip kernel phases (1 drones, 2 flock, 4 task, 8 obs) to attribute time; 128 / 256: cow waves
 * on the drone wave's SIMD take no chunks after / before the drone hand-off (v2 scheduling experiments). */
/* Internal: forget which obs buffer holds valid constant-zero bytes (the caller wrote into it); the
 * next ch_step writes every obs block in full. */
int ch__obs_invalidate(ch_handle* h, void* stream) {
    if (!h) return CH_ERR_INVALID;
    h->obs_zero_ptr = nullptr;
    // and on the device (stale row 1), for steps replayed from a graph captured before this call
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipMemsetAsync(h->stale + h->E, 1, (size_t)h->E, (hipStream_t)stream));
    return CH_OK;
}

// diagnostics: k_mlp2 writes wave 0's phase clocks of every workgroup to dev[blockIdx][16] (NULL: off); the fused
// step + actor kernel (k_step2_actor) writes its forward's clocks and wall-clock slots 13-15 to rows [grid, 2 grid),
// so a buffer for a collection on the fused path holds 2 x 16 x (E / 16) entries (tools/fused_probe.py trace)
extern "C" int ch__set_mlp_tstamp(long long* dev) {
    g_mlp_tstamp = dev;
    return CH_OK;
}

/* Internal (tests / diagnostics): ch_rollout_collect's path, bit 0 copy each step's observation into the buffer
 * (CH_ROLLOUT_COPY=1), bit 1 the stand-alone store kernel instead of the forward epilogues (CH_ROLLOUT_STORE_KERNEL=1),
 * bit 2 the actor forward fused into the step (CH_FUSED_ACTOR=1), bit 3 never fused. */
int ch__set_rollout_path(ch_handle* h, int32_t bits) {
    if (!h || bits < 0 || bits > 15) return CH_ERR_INVALID;
    h->rollout_path = bits;
    return CH_OK;
}

/* Internal: the handle's current rollout path bits (ch__set_rollout_path), or -1 for a null handle. */
int ch__get_rollout_path(const ch_handle* h) { return h ? h->rollout_path : -1; }

/* Internal (tests): steps ch_rollout_collect has launched as the fused step + actor kernel on this handle. */
int64_t ch__rollout_fused_steps(const ch_handle* h) { return h ? (int64_t)h->fused_steps : -1; }

int ch__set_phase_mask(ch_handle* h, int32_t mask) {
    if (!h) return CH_ERR_INVALID;
    h->phase_mask = mask;
    return CH_OK;
}

static int mlp_args(const ch_mlp* net, const float* x, int64_t rows, float* y, MlpArgs& a, std::string& err) {
    if (!net || !x || !y) { err = "NULL argument"; return CH_ERR_INVALID; }
    if (net->n_layers < 1 || net->n_layers > 4) { err = "n_layers must be 1..4"; return CH_ERR_INVALID; }
    if (rows < 0) { err = "rows < 0"; return CH_ERR_INVALID; }
    std::memset(&a, 0, sizeof(a));
    a.layers = net->n_layers;
    for (int i = 0; i <= net->n_layers; ++i) {
        a.dims[i] = net->dims[i];
        if (net->dims[i] < 1 || (i > 0 && net->dims[i] > 256)) { err = "layer widths must be 1..256"; return CH_ERR_UNSUPPORTED; }
    }
    for (int i = 0; i < net->n_layers; ++i) {
        if (!net->weight[i]) { err = "NULL weight"; return CH_ERR_INVALID; }
        a.w[i] = net->weight[i]; a.b[i] = net->bias[i];
    }
    if (net->hidden_act < CH_ACT_NONE || net->hidden_act > CH_ACT_RELU) { err = "unknown activation"; return CH_ERR_INVALID; }
    a.hidden_act = net->hidden_act; a.clip = net->clip != 0; a.lo = net->lo; a.hi = net->hi;
    a.x = x; a.rows = rows; a.y = y; a.rows_per_env = 1;
    a.kcap = net->dims[0];
    // float4 weight loads need 16-B aligned rows of a multiple of 8 floats (k_mlp2 reads 8 per lane), inputs 4
    for (int i = 0; i < net->n_layers; ++i)
        if (net->dims[i] % 8 == 0 && (reinterpret_cast<uintptr_t>(net->weight[i]) & 15) == 0) a.vec_w |= 1 << i;
    if (net->dims[0] % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) a.vec_w |= 1 << 7;
    // block-diagonal layers the kernel can skip by whole K-pair groups (ch_mlp.split_*); others run dense
    for (int i = 1; i < net->n_layers; ++i) {
        const int so = net->split_out[i], si = net->split_in[i];
        if (so > 0 && so < net->dims[i + 1] && so % 32 == 0 && si > 0 && si < net->dims[i] && si % 128 == 0) {
            a.split_out[i] = so; a.split_in[i] = si;
        }
    }
    if (net->packed) {
        if (reinterpret_cast<uintptr_t>(net->packed) & 15) { err = "packed weights must be 16-byte aligned"; return CH_ERR_INVALID; }
        a.packed = net->packed;
        mlp_packed_floats(a.layers, a.dims, a.pk_off, a.pk_pairs);
    }
    return CH_OK;
}

int64_t ch_mlp_packed_size(const ch_mlp* net) {
    if (!net || net->n_layers < 1 || net->n_layers > 4) return -1;
    for (int i = 0; i <= net->n_layers; ++i)
        if (net->dims[i] < 1 || (i > 0 && net->dims[i] > 256)) return -1;
    return mlp_packed_floats(net->n_layers, net->dims, nullptr, nullptr);
}

int ch_mlp_pack(const ch_mlp* net, float* dst, void* stream) {
    MlpArgs a;
    std::string err;
    float one = 0.0f;
    const int rc = mlp_args(net, &one, 0, &one, a, err);
    if (rc) return fail(nullptr, rc, "ch_mlp_pack: " + err);
    if (!dst || (reinterpret_cast<uintptr_t>(dst) & 15)) return fail(nullptr, CH_ERR_INVALID, "ch_mlp_pack: dst NULL or not 16-byte aligned");
    const hipError_t e = launch_mlp_pack(a, dst, (hipStream_t)stream);
    if (e != hipSuccess) return fail(nullptr, CH_ERR_DEVICE, std::string("ch_mlp_pack launch: ") + hipGetErrorString(e));
    return CH_OK;
}

int ch_mlp_forward(const ch_mlp* net, const float* x, int64_t rows, float* y, void* stream) {
    MlpArgs a;
    std::string err;
    const int rc = mlp_args(net, x, rows, y, a, err);
    if (rc) return fail(nullptr, rc, "ch_mlp_forward: " + err);
    const hipError_t e = launch_mlp(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(nullptr, CH_ERR_DEVICE, std::string("ch_mlp_forward launch: ") + hipGetErrorString(e));
    return CH_OK;
}

int ch_mlp_forward_masked(const ch_mlp* net, const float* x, int64_t rows, const uint8_t* row_mask, float* y,
                          void* stream) {
    MlpArgs a;
    std::string err;
    const int rc = mlp_args(net, x, rows, y, a, err);
    if (rc) return fail(nullptr, rc, "ch_mlp_forward_masked: " + err);
    if (!row_mask) return fail(nullptr, CH_ERR_INVALID, "ch_mlp_forward_masked: NULL row mask");
    a.row_mask = row_mask;
    const hipError_t e = launch_mlp(a, (hipStream_t)stream);
    if (e != hipSuccess)
        return fail(nullptr, CH_ERR_DEVICE, std::string("ch_mlp_forward_masked launch: ") + hipGetErrorString(e));
    return CH_OK;
}

// the forward of `net` on a handle's observation buffer: one row per env (CTDE) or agent (MARL), live widths from
// NUM_DRONES (envi row 0)
static int policy_args(ch_handle* h, const ch_mlp* net, const float* obs, float* y, MlpArgs& a, const char* who) {
    const bool marl = h->cfg.mode == CH_MODE_MARL;
    const int64_t rows = marl ? h->E * h->NC : h->E;
    const int want = marl ? 86 : h->rows * 86;
    if (net && net->dims[0] != want)
        return fail(h, CH_ERR_INVALID, std::string(who) + ": dims[0] must be " + std::to_string(want) + " for this handle");
    std::string err;
    const int rc = mlp_args(net, obs, rows, y, a, err);
    if (rc) return fail(h, rc, std::string(who) + ": " + err);
    a.env_n = h->envi;   // envi row 0: NUM_DRONES of the episode each env is in
    a.rows_per_env = marl ? h->NC : 1;
    a.k_unit = 86;
    a.kcap = std::min(a.dims[0], marl ? 86 : h->NC * 86);   // NUM_DRONES <= the constructor's drones
    return CH_OK;
}

int ch_policy_forward(ch_handle* h, const ch_mlp* net, const float* obs, float* y, void* stream) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_policy_forward: NULL handle");
    MlpArgs a;
    const int rc = policy_args(h, net, obs, y, a, "ch_policy_forward");
    if (rc) return rc;
    HIP_TRY(h, hipSetDevice(h->device));
    const hipError_t e = launch_mlp(a, (hipStream_t)stream);
    if (e != hipSuccess) return fail(h, CH_ERR_DEVICE, std::string("ch_policy_forward launch: ") + hipGetErrorString(e));
    return CH_OK;
}

static int rollout_args(ch_handle* h, const ch_rollout* rb, RolloutArgs& a, const char* who) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, std::string(who) + ": NULL handle");
    if (!rb) return fail(h, CH_ERR_INVALID, std::string(who) + ": NULL rollout buffer");
    if (h->cfg.mode != CH_MODE_CTDE)
        return fail(h, CH_ERR_UNSUPPORTED, std::string(who) + ": the SB3 rollout buffer is for CTDE handles");
    // the env reads a (num_drones, 4) action per env (ch_step: float4 [e * num_drones + k]), so the policy must
    // produce at least num_drones * 4 outputs (SB3: Box((NUM_DRONES, 4)) or the reference's (12, 4))
    if (rb->n_steps < 1 || rb->act_dim < h->NC * 4 || rb->act_dim > 256)
        return fail(h, CH_ERR_INVALID, std::string(who) + ": n_steps >= 1 and num_drones * 4 = " +
                                           std::to_string(h->NC * 4) + " <= act_dim <= 256 required");
    std::memset(&a, 0, sizeof(a));
    a.T = rb->n_steps; a.rows = h->E; a.obs_dim = h->rows * 86; a.act_dim = rb->act_dim;
    a.env_act_dim = h->NC * 4;
    a.mean_ld = rb->act_dim; a.value_ld = 1; a.tv_ld = 1; a.post_prev = 0;
    a.obs = rb->obs; a.actions = rb->actions; a.rewards = rb->rewards; a.episode_starts = rb->episode_starts;
    a.values = rb->values; a.log_probs = rb->log_probs; a.advantages = rb->advantages; a.returns = rb->returns;
    a.last_episode_starts = rb->last_episode_starts;
    return CH_OK;
}

int ch_rollout_store(ch_handle* h, const ch_rollout* rb, int32_t t, const float* obs, const float* mean,
                     const float* value, const float* log_std, uint64_t seed, float* env_actions, void* stream) {
    RolloutArgs a;
    int rc = rollout_args(h, rb, a, "ch_rollout_store");
    if (rc) return rc;
    if (t < 0 || t >= rb->n_steps) return fail(h, CH_ERR_INVALID, "ch_rollout_store: t outside [0, n_steps)");
    if (!obs || !mean || !value || !log_std || !env_actions || !rb->obs || !rb->actions || !rb->values ||
        !rb->log_probs || !rb->episode_starts || !rb->last_episode_starts)
        return fail(h, CH_ERR_INVALID, "ch_rollout_store: NULL buffer");
    if ((reinterpret_cast<uintptr_t>(obs) | reinterpret_cast<uintptr_t>(rb->obs)) & 15)
        return fail(h, CH_ERR_INVALID, "ch_rollout_store: obs buffers must be 16-byte aligned");
    a.t = t; a.obs_now = obs; a.mean = mean; a.value = value; a.log_std = log_std; a.seed = seed;
    a.env_actions = env_actions; a.copy_obs = 1;
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, launch_rollout(a, 0, (hipStream_t)stream));
    return CH_OK;
}

int ch_rollout_post(ch_handle* h, const ch_rollout* rb, int32_t t, const float* reward, const uint8_t* terminated,
                    const uint8_t* truncated, const float* terminal_value, float gamma, void* stream) {
    RolloutArgs a;
    int rc = rollout_args(h, rb, a, "ch_rollout_post");
    if (rc) return rc;
    if (t < 0 || t >= rb->n_steps) return fail(h, CH_ERR_INVALID, "ch_rollout_post: t outside [0, n_steps)");
    if (!reward || !terminated || !truncated || !rb->rewards || !rb->last_episode_starts)
        return fail(h, CH_ERR_INVALID, "ch_rollout_post: NULL buffer");
    a.t = t; a.reward = reward; a.terminated = terminated; a.truncated = truncated; a.terminal_value = terminal_value;
    a.gamma = gamma;
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, launch_rollout(a, 1, (hipStream_t)stream));
    return CH_OK;
}

int ch_rollout_gae(ch_handle* h, const ch_rollout* rb, const float* last_value, float gamma, float gae_lambda,
                   void* stream) {
    RolloutArgs a;
    int rc = rollout_args(h, rb, a, "ch_rollout_gae");
    if (rc) return rc;
    if (!last_value || !rb->rewards || !rb->values || !rb->episode_starts || !rb->advantages || !rb->returns)
        return fail(h, CH_ERR_INVALID, "ch_rollout_gae: NULL buffer");
    a.value = last_value; a.gamma = gamma;
    a.gamma_lambda = (float)((double)gamma * (double)gae_lambda);   // SB3: float32(self.gamma * self.gae_lambda)
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, launch_rollout(a, 2, (hipStream_t)stream));
    return CH_OK;
}

int ch_rollout_collect(ch_handle* h, const ch_rollout* rb, const ch_rollout_io* io, const ch_mlp* actor,
                       const ch_mlp* critic, const float* log_std, uint64_t seed, float gamma, float gae_lambda,
                       int32_t bootstrap_truncated, void* stream) {
    RolloutArgs ra;
    int rc = rollout_args(h, rb, ra, "ch_rollout_collect");
    if (rc) return rc;
    if (!io || !io->step || !io->mean || !io->env_actions || !log_std || !actor || (critic && !io->value))
        return fail(h, CH_ERR_INVALID, "ch_rollout_collect: NULL argument");
    const ch_step_io* sio = io->step;
    if (!sio->obs || !sio->reward || !sio->terminated || !sio->truncated || !sio->terminal_obs || !sio->reset_happened ||
        (bootstrap_truncated && !io->terminal_value))
        return fail(h, CH_ERR_INVALID, "ch_rollout_collect: the step buffers (obs, reward, terminated, truncated, "
                                       "terminal_obs, reset_happened) and terminal_value are required");
    if (!rb->obs || !rb->actions || !rb->rewards || !rb->episode_starts || !rb->values || !rb->log_probs ||
        !rb->advantages || !rb->returns || !rb->last_episode_starts)
        return fail(h, CH_ERR_INVALID, "ch_rollout_collect: NULL rollout buffer array");
    if ((reinterpret_cast<uintptr_t>(sio->obs) | reinterpret_cast<uintptr_t>(rb->obs)) & 15)
        return fail(h, CH_ERR_INVALID, "ch_rollout_collect: obs buffers must be 16-byte aligned");
    // critic == NULL: `actor` is a fused actor-critic (both heads in one net, output act_dim + 1 wide: the action
    // mean, then the value); one forward per step reads the observation once.  io->mean is then its
    // [rows][act_dim + 1] output and io->terminal_value a [rows][act_dim + 1] one for the terminal observations.
    const bool fused = critic == nullptr;
    const int out_w = fused ? rb->act_dim + 1 : rb->act_dim;
    if (actor->dims[actor->n_layers] != out_w || (!fused && critic->dims[critic->n_layers] != 1))
        return fail(h, CH_ERR_INVALID, fused ? "ch_rollout_collect: a fused actor-critic's output must be act_dim + 1 wide"
                                             : "ch_rollout_collect: actor output must be act_dim wide, critic output 1");
    hipStream_t st = (hipStream_t)stream;
    ch_step_io s = *sio;
    s.actions = io->env_actions; s.actions_out = nullptr;
    s.flags = (s.flags & ~CH_STEP_RANDOM_ACTIONS) | CH_STEP_AUTORESET;
    const ch_mlp* vnet = fused ? actor : critic;
    float* value = fused ? io->mean + rb->act_dim : io->value;
    float* tv_out = io->terminal_value;
    const float* tval = fused ? io->terminal_value + rb->act_dim : io->terminal_value;
    RolloutArgs a = ra;
    a.mean_ld = out_w; a.value_ld = fused ? out_w : 1; a.tv_ld = fused ? out_w : 1;
    // each step's post (reward + gamma V(terminal obs), next episode start) runs in the next step's store, the
    // last one in the GAE kernel: the step outputs and terminal values it reads are still that step's then
    a.post_prev = 1;
    a.reward = sio->reward; a.terminated = sio->terminated; a.truncated = sio->truncated;
    a.terminal_value = bootstrap_truncated ? tval : nullptr; a.gamma = gamma;
    a.obs_now = sio->obs; a.mean = io->mean; a.value = value; a.log_std = log_std; a.seed = seed;
    a.env_actions = io->env_actions;
    // The step writes its observations straight into the buffer's next slot (obs[t + 1]; the last step into the
    // env's own obs buffer): the obs of step t > 0 is already in place when it is stored, and only obs[0] is copied
    // (a v2 step into a buffer other than the one it wrote last writes every block in full, ch_step's obs_zero_ptr).
    // The actor and critic on obs[t + 1] go out as one launch (launch_mlp_multi; their workgroups share the CUs,
    // so each forward's latencies hide behind the other's matrix work).  The truncation bootstrap is deferred: the
    // post of step t queues the terminal observations of the envs that were truncated and not terminated, and
    // every kTvEvery steps one forward over the queue gives their values, added to those rewards rows (the queue
    // holds at most kTvEvery * E rows).  Per step that leaves two launches with separate nets (forwards with the
    // store in their epilogues, step) and three with a fused net or CH_ROLLOUT_STORE_KERNEL=1 (forward, store, step).
    // (the period: 16 steps, fewer when the queue would pass 1 GiB -- one flush is a whole forward's latency, ~20 us
    // at configs[2]'s size, whatever the queue holds)
    const int kTvEvery = (int)std::min<long long>(16, std::max<long long>(1, (1LL << 30) / ((long long)h->E * ra.obs_dim * 4)));
    const bool copy_each = (h->rollout_path & 1) != 0;
    const size_t slot = (size_t)h->E * (size_t)ra.obs_dim;
    auto obs_at = [&](int32_t t) { return (t == 0 || t == rb->n_steps || copy_each) ? sio->obs : rb->obs + (size_t)t * slot; };
    MlpArgs fa, fc, ftv;
    if ((rc = policy_args(h, actor, sio->obs, io->mean, fa, "ch_rollout_collect (actor)"))) return rc;
    if (!fused && (rc = policy_args(h, critic, sio->obs, io->value, fc, "ch_rollout_collect (critic)"))) return rc;
    HIP_TRY(h, hipSetDevice(h->device));
    const long long cap = (long long)h->E * kTvEvery;
    RolloutArgs ap = a;   // k_rollout_apply over the queue
    if (bootstrap_truncated) {
        const size_t nobs = (size_t)cap * ra.obs_dim, nval = (size_t)cap * out_w;
        if (h->tv_obs_n < nobs) {
            if (h->tv_obs) HIP_TRY(h, hipFree(h->tv_obs));
            h->tv_obs = nullptr;
            HIP_TRY(h, hipMalloc(&h->tv_obs, sizeof(float) * nobs));
            if (h->tv_row) HIP_TRY(h, hipFree(h->tv_row));
            h->tv_row = nullptr;
            HIP_TRY(h, hipMalloc(&h->tv_row, sizeof(long long) * (size_t)cap));
            h->tv_obs_n = nobs;
        }
        if (h->tv_val_n < nval) {
            if (h->tv_val) HIP_TRY(h, hipFree(h->tv_val));
            h->tv_val = nullptr;
            HIP_TRY(h, hipMalloc(&h->tv_val, sizeof(float) * nval));
            h->tv_val_n = nval;
        }
        if (!h->tv_count) HIP_TRY(h, hipMalloc(&h->tv_count, sizeof(int)));
        HIP_TRY(h, hipMemsetAsync(h->tv_count, 0, sizeof(int), st));
        // V(terminal obs) over the queue: whole (12, 86) blocks, zero past the constructor's drones
        std::string err;
        if ((rc = mlp_args(vnet, h->tv_obs, cap, h->tv_val, ftv, err))) return fail(h, rc, "ch_rollout_collect: " + err);
        ftv.rows_dev = h->tv_count;
        ftv.kcap = std::min(ftv.dims[0], h->NC * 86);
        a.defer = 1; a.term_obs = sio->terminal_obs; a.tv_obs = h->tv_obs; a.tv_count = h->tv_count; a.tv_row = h->tv_row;
        a.terminal_value = nullptr;
        ap = a;
        ap.rows = cap;
        ap.terminal_value = h->tv_val + (fused ? rb->act_dim : 0);
        ap.tv_ld = fused ? out_w : 1;   // the value net's output width
        ap.v_col = fused ? rb->act_dim : 0;
    }
    // the flush: V over the queue with the reward update in the forward's epilogue (kRoleTvApply), or (a net k_mlp2
    // does not take) the forward into tv_val and k_rollout_apply; then the queue is emptied
    const bool tv_epi = bootstrap_truncated && mlp_multi_fits(&ftv, 1) && !(h->rollout_path & 2);
    auto flush = [&]() -> hipError_t {
        hipError_t e;
        if (tv_epi) {
            const int role = kRoleTvApply;
            e = launch_mlp_multi(&ftv, 1, st, &role, &ap);
        } else {
            e = launch_mlp_multi(&ftv, 1, st);
            if (e == hipSuccess) e = launch_rollout(ap, 3, st);
        }
        if (e == hipSuccess) e = hipMemsetAsync(h->tv_count, 0, sizeof(int), st);
        return e;
    };
    MlpArgs segs[2];
    segs[0] = fa; segs[1] = fc;
    const bool no_epi = (h->rollout_path & 2) != 0;
    if (!fused && !no_epi && mlp_multi_fits(segs, 2)) {
        // Two launches per step: the actor and critic forwards with the store folded into their epilogues (the
        // actor's samples its actions, log-probabilities and env actions; the critic's writes the values, the
        // previous step's post and the episode starts, and at t = 0 copies obs[0]), then the step.
        // With the fused step (rollout_path bit 2: CH_FUSED_ACTOR=1 or ch__set_rollout_path; bit 3 forbids it) the
        // actor forward of step t + 1 runs in the step kernel of step t, in the workgroup that wrote those
        // observations (k_step2_actor), and the critic goes out alone: the same work in the same stream order.
        const int roles[2] = {kRoleSample, kRoleValue};
        const bool fuse = (h->rollout_path & 4) && !(h->rollout_path & 8) &&
                          step_actor(h, &s, st, segs[0], a, false) == hipSuccess;
        RolloutArgs ro = a;
        for (int32_t t = 0; t < rb->n_steps; ++t) {
            segs[0].x = segs[1].x = obs_at(t);
            ro.t = t;
            ro.copy_obs = t == 0 || copy_each;
            if (fuse && t > 0) HIP_TRY(h, launch_mlp_multi(&segs[1], 1, st, &roles[1], &ro));   // the critic
            else HIP_TRY(h, launch_mlp_multi(segs, 2, st, roles, &ro));
            if (bootstrap_truncated && t > 0 && t % kTvEvery == 0) HIP_TRY(h, flush());
            s.obs = (t + 1 < rb->n_steps && !copy_each) ? rb->obs + (size_t)(t + 1) * slot : sio->obs;
            if (fuse && t + 1 < rb->n_steps) {
                MlpArgs fa = segs[0];
                fa.x = obs_at(t + 1);   // = s.obs
                RolloutArgs rn = ro;
                rn.t = t + 1;
                const hipError_t e = step_actor(h, &s, st, fa, rn, true);
                if (e != hipSuccess) return fail(h, CH_ERR_DEVICE, std::string("ch_rollout_collect fused step: ") + hipGetErrorString(e));
            } else if ((rc = ch_step(h, &s, stream))) {
                return rc;
            }
        }
        // the last step's post (and queue) and flush, V(obs after the last step), GAE without a post of its own
        RolloutArgs pa = a;
        pa.t = rb->n_steps;
        pa.post_only = 1;
        HIP_TRY(h, launch_rollout(pa, 0, st));
        if (bootstrap_truncated) HIP_TRY(h, flush());
        MlpArgs fv = fc;
        fv.x = obs_at(rb->n_steps);
        HIP_TRY(h, launch_mlp_multi(&fv, 1, st));
        a.post_prev = 0;
        a.gamma_lambda = (float)((double)gamma * (double)gae_lambda);   // SB3: float32(self.gamma * self.gae_lambda)
        HIP_TRY(h, launch_rollout(a, 2, st));
        return CH_OK;
    }
    HIP_TRY(h, launch_mlp_multi(segs, fused ? 1 : 2, st));
    for (int32_t t = 0; t < rb->n_steps; ++t) {
        // SB3 collect_rollouts, one step of every env: policy(obs) -> sample, log-prob, value -> env.step ->
        // bootstrap truncated rewards with V(terminal obs) -> buffer (OnPolicyAlgorithm.collect_rollouts)
        a.t = t;
        a.copy_obs = t == 0 || copy_each;
        HIP_TRY(h, launch_rollout(a, 0, st));   // (with the post of step t - 1)
        if (bootstrap_truncated && t > 0 && t % kTvEvery == 0) HIP_TRY(h, flush());
        s.obs = (t + 1 < rb->n_steps && !copy_each) ? rb->obs + (size_t)(t + 1) * slot : sio->obs;
        if ((rc = ch_step(h, &s, stream))) return rc;
        int n = 0;
        if (t + 1 < rb->n_steps) {
            fa.x = fc.x = obs_at(t + 1);
            segs[n++] = fa;
            if (!fused) segs[n++] = fc;
        } else {   // the last observations' values: GAE's last_value
            MlpArgs fv = fused ? fa : fc;
            fv.x = obs_at(t + 1);
            segs[n++] = fv;
        }
        HIP_TRY(h, launch_mlp_multi(segs, n, st));
    }
    if (bootstrap_truncated) {
        // the last step's post (and queue), the last flush; GAE then runs without a post of its own
        RolloutArgs pa = a;
        pa.t = rb->n_steps;
        pa.post_only = 1;
        HIP_TRY(h, launch_rollout(pa, 0, st));
        HIP_TRY(h, flush());
        a.post_prev = 0;
    }
    a.gamma_lambda = (float)((double)gamma * (double)gae_lambda);   // SB3: float32(self.gamma * self.gae_lambda)
    HIP_TRY(h, launch_rollout(a, 2, st));
    return CH_OK;
}

int ch_marl_rollout_collect(ch_handle* h, const ch_marl_rollout* rb, const ch_marl_rollout_io* io, const ch_mlp* policy,
                            const ch_mlp* value, uint64_t seed, float gamma, float gae_lambda, void* stream) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_marl_rollout_collect: NULL handle");
    if (h->cfg.mode != CH_MODE_MARL)
        return fail(h, CH_ERR_UNSUPPORTED, "ch_marl_rollout_collect: the per-agent rollout is for MARL handles");
    if (!rb || !io || !io->step || !policy || !value || !io->policy_out || !io->value_out || !io->env_actions)
        return fail(h, CH_ERR_INVALID, "ch_marl_rollout_collect: NULL argument");
    if (rb->n_steps < 1 || rb->act_dim != 4)
        return fail(h, CH_ERR_INVALID, "ch_marl_rollout_collect: n_steps >= 1 and act_dim = 4 (one VEL action per agent)");
    if (!rb->obs || !rb->actions || !rb->log_probs || !rb->values || !rb->rewards || !rb->agent_mask || !rb->terminated ||
        !rb->truncated || !rb->advantages || !rb->returns || !rb->last_values)
        return fail(h, CH_ERR_INVALID, "ch_marl_rollout_collect: NULL rollout buffer array");
    const ch_step_io* sio = io->step;
    if (!sio->obs || !sio->reward || !sio->terminated || !sio->truncated)
        return fail(h, CH_ERR_INVALID, "ch_marl_rollout_collect: the step buffers obs, reward, terminated, truncated are required");
    if ((reinterpret_cast<uintptr_t>(sio->obs) | reinterpret_cast<uintptr_t>(rb->obs)) & 15)
        return fail(h, CH_ERR_INVALID, "ch_marl_rollout_collect: obs buffers must be 16-byte aligned");
    if (policy->dims[policy->n_layers] != 2 * rb->act_dim || value->dims[value->n_layers] != 1)
        return fail(h, CH_ERR_INVALID, "ch_marl_rollout_collect: the policy must output 2 * act_dim (mean, log_std), the value net 1");
    int rc;
    MlpArgs fp, fv;
    if ((rc = policy_args(h, policy, sio->obs, io->policy_out, fp, "ch_marl_rollout_collect (policy)"))) return rc;
    if ((rc = policy_args(h, value, sio->obs, io->value_out, fv, "ch_marl_rollout_collect (value)"))) return rc;
    HIP_TRY(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    MarlArgs a;
    std::memset(&a, 0, sizeof(a));
    a.T = rb->n_steps; a.A = rb->act_dim; a.N = h->NC; a.E = h->E; a.rows = h->E * h->NC;
    a.env_n = h->envi; a.env_active = h->envi + 7 * h->E;
    a.pol = io->policy_out; a.val = io->value_out; a.seed = seed; a.post_prev = 1;
    a.reward = sio->reward; a.term = sio->terminated; a.trunc = sio->truncated;
    a.gamma = gamma; a.gamma_lambda = (float)((double)gamma * (double)gae_lambda);
    a.obs = rb->obs; a.actions = rb->actions; a.log_probs = rb->log_probs; a.values = rb->values; a.rewards = rb->rewards;
    a.advantages = rb->advantages; a.returns = rb->returns; a.last_values = rb->last_values; a.env_actions = io->env_actions;
    a.mask = rb->agent_mask; a.terminated = rb->terminated; a.truncated = rb->truncated;
    // the step writes its observations straight into the buffer's next slot (a step into a buffer other than the one
    // it wrote last writes every block in full); the last step into the env's own buffer.  No terminal observations:
    // an agent's trajectory ends only where it terminates (no bootstrap), so the reset path needs no copy.
    ch_step_io s = *sio;
    s.actions = io->env_actions; s.actions_out = nullptr; s.terminal_obs = nullptr;
    s.flags = (s.flags & ~CH_STEP_RANDOM_ACTIONS) | CH_STEP_AUTORESET;
    const size_t slot = (size_t)a.rows * 86;
    MlpArgs segs[2];
    for (int32_t t = 0; t < rb->n_steps; ++t) {
        const float* x = t == 0 ? sio->obs : rb->obs + (size_t)t * slot;
        segs[0] = fp; segs[1] = fv;
        segs[0].x = segs[1].x = x;
        HIP_TRY(h, launch_mlp_multi(segs, 2, st));
        a.t = t;
        a.obs_now = t == 0 ? sio->obs : nullptr;
        HIP_TRY(h, launch_marl_rollout(a, 0, st));
        s.obs = t + 1 < rb->n_steps ? rb->obs + (size_t)(t + 1) * slot : sio->obs;
        if ((rc = ch_step(h, &s, stream))) return rc;
    }
    // V(obs after the last step) -> last_values, the last step's post, GAE
    fv.x = sio->obs;
    HIP_TRY(h, launch_mlp_multi(&fv, 1, st));
    HIP_TRY(h, launch_marl_rollout(a, 1, st));
    return CH_OK;
}

int ch_metrics(ch_handle* h, double* out, int32_t reset_after, void* stream) {
    if (!h || !out) return fail(h, CH_ERR_INVALID, "ch_metrics: NULL argument");
    HIP_TRY(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    // device reduction on the caller's stream, then one 72-byte copy into pinned memory
    HIP_TRY(h, launch_metrics_reduce(h->metrics, h->E, h->mdev, h->errw, h->mdev + CH_METRIC_COUNT, reset_after, st));
    HIP_TRY(h, hipMemcpyAsync(h->mhost, h->mdev, sizeof(double) * (CH_METRIC_COUNT + 1), hipMemcpyDeviceToHost, st));
    HIP_TRY(h, hipStreamSynchronize(st));
    std::memcpy(out, h->mhost, sizeof(double) * CH_METRIC_COUNT);
    return device_status(h, (int)h->mhost[CH_METRIC_COUNT]);
}

int ch_metrics_device(ch_handle* h, double* dev_out, int32_t reset_after, void* stream) {
    if (!h || !dev_out) return fail(h, CH_ERR_INVALID, "ch_metrics_device: NULL argument");
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, launch_metrics_reduce(h->metrics, h->E, dev_out, nullptr, nullptr, reset_after, (hipStream_t)stream));
    return CH_OK;
}

int ch_get_eval(ch_handle* h, double* host_out, void* stream) {
    if (!h || !host_out) return fail(h, CH_ERR_INVALID, "ch_get_eval: NULL argument");
    if (!h->evald) return fail(h, CH_ERR_UNSUPPORTED, "ch_get_eval: the handle was created with eval_metrics = 0");
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(h, hipMemcpy(host_out, h->evald, sizeof(double) * h->E * h->NC, hipMemcpyDeviceToHost));
    return CH_OK;
}

int ch_outputs_to_host(ch_handle* h, const ch_step_io* io, ch_host_out* out, void* stream) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_outputs_to_host: NULL handle");
    if (!io || !out || !io->obs || !io->reward || !io->terminated || !io->truncated || !out->obs || !out->reward ||
        !out->terminated || !out->truncated)
        return fail(h, CH_ERR_INVALID, "ch_outputs_to_host: obs, reward, terminated and truncated are required on both sides");
    if ((out->reset_happened || out->ended_env || out->ended_obs || out->ended_stats) && !io->reset_happened)
        return fail(h, CH_ERR_INVALID, "ch_outputs_to_host: the reset list needs io->reset_happened");
    if ((out->ended_obs && !io->terminal_obs) || (out->ended_stats && !io->episode_stats))
        return fail(h, CH_ERR_INVALID, "ch_outputs_to_host: ended_obs needs io->terminal_obs, ended_stats io->episode_stats");
    if (out->agent_active && !io->agent_active)
        return fail(h, CH_ERR_INVALID, "ch_outputs_to_host: agent_active needs io->agent_active");
    HIP_TRY(h, hipSetDevice(h->device));
    hipStream_t st = (hipStream_t)stream;
    const int64_t E = h->E;
    const size_t blk = (size_t)h->rows * 86, live = (size_t)h->NC * 86;   // floats per block / in its first NC rows
    if (io->reset_happened) {
        if (!h->st_count) {
            HIP_TRY(h, hipMalloc(&h->st_count, sizeof(long long)));
            HIP_TRY(h, hipMalloc(&h->st_env, sizeof(long long) * E));
            HIP_TRY(h, hipMalloc(&h->st_stats, sizeof(double) * 2 * E));
            HIP_TRY(h, hipMalloc(&h->st_obs, sizeof(float) * blk * E));
            HIP_TRY(h, hipHostMalloc(&h->st_count_host, sizeof(long long), hipHostMallocDefault));
        }
        HIP_TRY(h, launch_stage_ended(E, io->reset_happened, out->ended_obs ? io->terminal_obs : nullptr,
                                      out->ended_stats ? io->episode_stats : nullptr, (int)blk, h->st_count, h->st_env,
                                      h->st_stats, h->st_obs, st));
        HIP_TRY(h, hipMemcpyAsync(h->st_count_host, h->st_count, sizeof(long long), hipMemcpyDeviceToHost, st));
    }
    // the first NC rows of every block (CTDE: rows >= NC are always zero; MARL: R = NC, one contiguous copy)
    if (live == blk)
        HIP_TRY(h, hipMemcpyAsync(out->obs, io->obs, sizeof(float) * blk * E, hipMemcpyDeviceToHost, st));
    else
        HIP_TRY(h, hipMemcpy2DAsync(out->obs, sizeof(float) * blk, io->obs, sizeof(float) * blk, sizeof(float) * live, E,
                                    hipMemcpyDeviceToHost, st));
    const size_t K = (size_t)h->K;
    HIP_TRY(h, hipMemcpyAsync(out->reward, io->reward, sizeof(float) * K * E, hipMemcpyDeviceToHost, st));
    HIP_TRY(h, hipMemcpyAsync(out->terminated, io->terminated, K * E, hipMemcpyDeviceToHost, st));
    HIP_TRY(h, hipMemcpyAsync(out->truncated, io->truncated, K * E, hipMemcpyDeviceToHost, st));
    if (out->reset_happened) HIP_TRY(h, hipMemcpyAsync(out->reset_happened, io->reset_happened, E, hipMemcpyDeviceToHost, st));
    if (out->agent_active)
        HIP_TRY(h, hipMemcpyAsync(out->agent_active, io->agent_active, (size_t)h->NC * E, hipMemcpyDeviceToHost, st));
    // the ended envs' lists: a speculative first part sized from the recent counts (the usual case: a few envs end per
    // step -- at C4 under random actions ~20, in a training rollout ~3), the rest after the count
    const int64_t cap = std::min<int64_t>(E, 2 * std::max<int64_t>(h->ended_last, (int64_t)h->ended_mean) + 8);
    auto copy_ended = [&](int64_t lo, int64_t hi) -> int {
        if (hi <= lo) return CH_OK;
        if (out->ended_env)
            HIP_TRY(h, hipMemcpyAsync(out->ended_env + lo, h->st_env + lo, sizeof(long long) * (hi - lo), hipMemcpyDeviceToHost, st));
        if (out->ended_stats)
            HIP_TRY(h, hipMemcpyAsync(out->ended_stats + 2 * lo, h->st_stats + 2 * lo, sizeof(double) * 2 * (hi - lo),
                                      hipMemcpyDeviceToHost, st));
        if (out->ended_obs)
            HIP_TRY(h, hipMemcpyAsync(out->ended_obs + blk * lo, h->st_obs + blk * lo, sizeof(float) * blk * (hi - lo),
                                      hipMemcpyDeviceToHost, st));
        return CH_OK;
    };
    int rc = CH_OK;
    if (io->reset_happened && (rc = copy_ended(0, cap))) return rc;
    HIP_TRY(h, hipStreamSynchronize(st));
    out->ended_count = io->reset_happened ? *h->st_count_host : 0;
    if (io->reset_happened) {
        h->ended_last = out->ended_count;
        h->ended_mean = 0.9 * h->ended_mean + 0.1 * (double)out->ended_count;
    }
    if (out->ended_count > cap) {
        if ((rc = copy_ended(cap, out->ended_count))) return rc;
        HIP_TRY(h, hipStreamSynchronize(st));
    }
    return CH_OK;
}

int ch_sync(ch_handle* h, void* stream) {
    if (!h) return fail(nullptr, CH_ERR_INVALID, "ch_sync: NULL handle");
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipStreamSynchronize((hipStream_t)stream));
    int word = 0;
    HIP_TRY(h, hipMemcpy(&word, h->errw, sizeof(int), hipMemcpyDeviceToHost));
    return device_status(h, word);
}

}  // extern "C"
