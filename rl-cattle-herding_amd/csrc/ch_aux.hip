// ch_aux.hip — small device-side helpers around the step: the end-of-rollout metric reduction.
//
// Reference: BaseAviary.update_evaluation_metrics (sb3_envs/BaseAviary.py:1406-1435) appends per-step
// values to host lists; here every env accumulates its rows in HBM during the step kernel and one
// launch sums them over the envs at the end of a rollout, on the caller's stream, so the RCCL
// all-reduce (bench.py, cattleherd/distributed.py) reads a device buffer and nothing syncs the host.
#include <hip/hip_runtime.h>

#include "ch_internal.h"
#include "ch_rollout_dev.h"

namespace ch {

constexpr int kReduceThreads = 256;

// one workgroup per metric row; thread t sums envs t, t + 256, ... in order, then a fixed LDS tree:
// the result is the same for every call on the same data (sharding-invariance tests compare it)
__global__ __launch_bounds__(kReduceThreads) void k_metrics_reduce(double* metrics, long long E, double* out,
                                                                 const int* err_word, double* err_out, int reset) {
    __shared__ double part[kReduceThreads];
    const int r = blockIdx.x, t = threadIdx.x;
    double* row = metrics + (long long)r * E;
    double s = 0;
    for (long long e = t; e < E; e += kReduceThreads) {
        s += row[e];
        if (reset) row[e] = 0;
    }
    part[t] = s;
    __syncthreads();
    for (int w = kReduceThreads / 2; w > 0; w >>= 1) {
        if (t < w) part[t] += part[t + w];
        __syncthreads();
    }
    if (t == 0) {
        out[r] = part[0];
        if (r == 0 && err_out) *err_out = err_word ? (double)*err_word : 0.0;
    }
}

hipError_t launch_metrics_reduce(double* metrics, long long E, double* out, const int* err_word, double* err_out,
                                 int reset, hipStream_t st) {
    hipLaunchKernelGGL(k_metrics_reduce, dim3(CH_METRIC_COUNT), dim3(kReduceThreads), 0, st, metrics, E, out,
                       err_word, err_out, reset);
    return hipGetLastError();
}


// ---- on-device PPO rollout buffer (the SB3 loop of CTDECattleHerder.py:107-150) -------------
// stable_baselines3 2.7 OnPolicyAlgorithm.collect_rollouts / RolloutBuffer.compute_returns_and_advantage
// (SB3 is not in this image: restated from its published algorithm, "parity unpinned" to its source):
//   actions ~ N(mean, exp(log_std)) stored unclipped, the env gets them clipped to the Box [-1, 1];
//   log_prob = sum_i Normal(mean_i, std_i).log_prob(a_i); episode_start = the previous step's done;
//   a done that is a truncation (TimeLimit.truncated = truncated and not terminated) bootstraps the
//   reward with gamma V(terminal_observation); GAE(gamma, lambda) backwards over the buffer in float32.
namespace {
constexpr int kRollThreads = 256;
}  // namespace

// one wave per env (kRollThreads / 64 envs per workgroup): the observation row into the buffer (copy_obs), the
// Gaussian sample of every action (lane k: action k, k + 64, ...), the summed log-probability (a wave tree
// sum), the clipped env action, value and episode start; with post_prev, the previous step's post first (one
// launch per step less in ch_rollout_collect)
__global__ __launch_bounds__(kRollThreads) void k_rollout_store(RolloutArgs a) {
    const int lane = threadIdx.x & 63;
    const long long e = (long long)blockIdx.x * (kRollThreads / 64) + (threadIdx.x >> 6);
    if (e >= a.rows) return;
    const long long row = (long long)a.t * a.rows + e;
    float les = 0.0f;
    bool queue = false;
    if (lane == 0) les = a.post_prev && a.t > 0 ? rollout_post_env(a, a.t - 1, e, &queue) : a.last_episode_starts[e];
    if (__ballot(queue)) {
        // deferred bootstrap: the terminal observation of step t - 1 into the queue (the wave copies it)
        int slot = 0;
        if (lane == 0) { slot = atomicAdd(a.tv_count, 1); a.tv_row[slot] = (long long)(a.t - 1) * a.rows + e; }
        slot = __shfl(slot, 0);
        const float4* src = reinterpret_cast<const float4*>(a.term_obs + e * a.obs_dim);
        float4* dst = reinterpret_cast<float4*>(a.tv_obs + (long long)slot * a.obs_dim);
        for (int k = lane; k < a.obs_dim / 4; k += 64) dst[k] = src[k];
    }
    if (a.post_only) return;
    if (a.copy_obs) {
        const float4* src = reinterpret_cast<const float4*>(a.obs_now + e * a.obs_dim);
        float4* dst = reinterpret_cast<float4*>(a.obs + row * a.obs_dim);
        for (int k = lane; k < a.obs_dim / 4; k += 64) dst[k] = src[k];
    }
    // the log-probability: every dimension's term into LDS, then summed in action order by one lane (the order
    // the policy forward's sampling epilogue uses too)
    __shared__ float lpt[kRollThreads / 64][256];
    float* lp = lpt[threadIdx.x >> 6];
    for (int k = lane; k < a.act_dim; k += 64) lp[k] = rollout_sample(a, a.t, k, e, a.mean[e * a.mean_ld + k]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    if (lane == 0) {
        float lps = 0.0f;
        for (int k = 0; k < a.act_dim; ++k) lps += lp[k];
        a.log_probs[row] = lps;
        a.values[row] = a.value[e * a.value_ld];
        a.episode_starts[row] = les;
    }
}

// after the env step: reward (+ gamma V(terminal obs) for truncations), next episode start
__global__ void k_rollout_post(RolloutArgs a) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.rows) return;
    rollout_post_env(a, a.t, e);
}

// the deferred bootstraps: rewards[row of slot] += gamma V(terminal obs of slot), for the queued slots
__global__ void k_rollout_apply(RolloutArgs a, const float* tv_val) {
    const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= *a.tv_count) return;
    const long long row = a.tv_row[q];
    a.rewards[row] = fmaf(a.gamma, tv_val[q * a.tv_ld], a.rewards[row]);
}

// RolloutBuffer.compute_returns_and_advantage, one env per thread, backwards over the buffer in float32.  The
// recursion is serial in the step; its inputs are not: each chunk of kGaeChunk steps is loaded at once (one memory
// round trip per chunk instead of per step), then folded backwards.
constexpr int kGaeChunk = 16;
__global__ void k_rollout_gae(RolloutArgs a) {
    const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.rows) return;
    const float les = a.post_prev ? rollout_post_env(a, a.T - 1, e) : a.last_episode_starts[e];   // the last step's post
    const float g = a.gamma, gl = a.gamma_lambda;
    float last = 0.0f;
    float nnt = 1.0f - les, nv = a.value[e * a.value_ld];   // the step after s: (1 - its episode start), its value
    for (int s1 = a.T; s1 > 0; s1 -= kGaeChunk) {
        const int s0 = s1 > kGaeChunk ? s1 - kGaeChunk : 0;
        float rw[kGaeChunk], vl[kGaeChunk], es[kGaeChunk];
#pragma unroll
        for (int i = 0; i < kGaeChunk; ++i) {
            const long long row = (long long)min(s0 + i, s1 - 1) * a.rows + e;
            rw[i] = a.rewards[row]; vl[i] = a.values[row]; es[i] = a.episode_starts[row];
        }
#pragma unroll
        for (int i = kGaeChunk - 1; i >= 0; --i) {
            if (s0 + i >= s1) continue;
            const long long row = (long long)(s0 + i) * a.rows + e;
            const float delta = (rw[i] + (g * nv) * nnt) - vl[i];
            last = delta + (gl * nnt) * last;
            a.advantages[row] = last;
            a.returns[row] = last + vl[i];
            nnt = 1.0f - es[i]; nv = vl[i];
        }
    }
}

// ---- the DTDE (RLlib) per-agent rollout (ch_marl_rollout_collect; DTDECattleHerder.py:62-97, marl_wrapper.py:77-119)
// RLlib PPO with one shared policy over every agent row (RLlib is not in this image: its defaults restated, "parity
// unpinned"): the policy output is DiagGaussian's (mean, log_std), actions a = mean + exp(log_std) eps stored
// unclipped, the env gets them clipped to Box(-1, 1); the log-probability is summed in action order.  The log_std
// half is clamped to [-20, 20] first, as RLlib's MLP head does for a DiagGaussian (clip_log_std with
// log_std_clip_param 20: the trained weights simulator/policy_weights.pkl carry pi.log_std_clip_param_const = 20).
constexpr float kRllibLogStdClip = 20.0f;

// after the env step t - 1: the agent's reward / terminated / truncated into the buffer (0 where it was not live)
__device__ __forceinline__ void marl_post(const MarlArgs& a, int t, long long r) {
    const long long row = (long long)t * a.rows + r;
    const bool m = a.mask[row] != 0;
    a.rewards[row] = m ? a.reward[r] : 0.0f;
    a.terminated[row] = m ? a.term[r] : 0;
    a.truncated[row] = m ? a.trunc[r] : 0;
}

// one thread per agent row: the previous step's post, then step t's mask (the wrapper's self.agents: agent i <
// NUM_DRONES and not dropped out, read from the env state the step starts from), the samples, log-probability,
// value and clipped env action; at t == 0 the batch's observation row into obs[0]
__global__ __launch_bounds__(256) void k_marl_store(MarlArgs a) {
    const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.rows) return;
    if (a.post_prev && a.t > 0) marl_post(a, a.t - 1, r);
    if (a.post_only) return;
    const long long e = r / a.N;
    const int i = (int)(r - e * a.N);
    const bool live = i < a.env_n[e] && ((a.env_active[e] >> i) & 1);
    const long long row = (long long)a.t * a.rows + r;
    if (a.obs_now) {
        const float2* src = reinterpret_cast<const float2*>(a.obs_now + r * 86);
        float2* dst = reinterpret_cast<float2*>(a.obs + row * 86);
#pragma unroll 1
        for (int k = 0; k < 43; ++k) dst[k] = src[k];
    }
    a.mask[row] = live;
    float lps = 0.0f;
    for (int k = 0; k < a.A; ++k) {
        float act = 0.0f;
        if (live) {
            uint32_t c[4] = {(uint32_t)a.t, (uint32_t)k, (uint32_t)r, (uint32_t)(r >> 32)};
            philox_k(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
            const float u1 = ((float)(c[0] >> 8) + 1.0f) * (1.0f / 16777216.0f);   // (0, 1]
            const float u2 = (float)(c[1] >> 8) * (1.0f / 16777216.0f);
            const float eps = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853071795865f * u2);
            const float mu = a.pol[r * 2 * a.A + k];
            const float ls = fminf(fmaxf(a.pol[r * 2 * a.A + a.A + k], -kRllibLogStdClip), kRllibLogStdClip);
            const float sd = expf(ls);
            act = mu + sd * eps;
            const float d = act - mu, var = sd * sd;
            lps += -(d * d) / (2.0f * var) - ls - 0.91893853320467274f;
        }
        a.actions[row * a.A + k] = act;
        a.env_actions[r * 4 + k] = live ? fminf(fmaxf(act, -1.0f), 1.0f) : 0.0f;
    }
    a.log_probs[row] = lps;
    a.values[row] = live ? a.val[r] : 0.0f;
}

// the last step's post, then GAE per agent row backwards in float32: a trajectory ends where the agent terminates;
// rows the agent was not live in get 0 (include/cattleherd.h ch_marl_rollout)
constexpr int kMarlGaeChunk = 16;
__global__ __launch_bounds__(256) void k_marl_gae(MarlArgs a) {
    const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.rows) return;
    if (a.post_prev) marl_post(a, a.T - 1, r);
    const float g = a.gamma, gl = a.gamma_lambda;
    const float lv = a.val[r];
    a.last_values[r] = lv;
    float last = 0.0f, nv = lv;
    for (int s1 = a.T; s1 > 0; s1 -= kMarlGaeChunk) {
        const int s0 = s1 > kMarlGaeChunk ? s1 - kMarlGaeChunk : 0;
        float rw[kMarlGaeChunk], vl[kMarlGaeChunk];
        uint8_t mk[kMarlGaeChunk], te[kMarlGaeChunk];
#pragma unroll
        for (int i = 0; i < kMarlGaeChunk; ++i) {
            const long long row = (long long)min(s0 + i, s1 - 1) * a.rows + r;
            rw[i] = a.rewards[row]; vl[i] = a.values[row]; mk[i] = a.mask[row]; te[i] = a.terminated[row];
        }
#pragma unroll
        for (int i = kMarlGaeChunk - 1; i >= 0; --i) {
            if (s0 + i >= s1) continue;
            const long long row = (long long)(s0 + i) * a.rows + r;
            if (!mk[i]) {
                a.advantages[row] = 0.0f; a.returns[row] = 0.0f;
                last = 0.0f; nv = 0.0f;
                continue;
            }
            const float nnt = te[i] ? 0.0f : 1.0f;
            const float delta = (rw[i] + (g * nv) * nnt) - vl[i];
            last = delta + (gl * nnt) * last;
            a.advantages[row] = last;
            a.returns[row] = last + vl[i];
            nv = vl[i];
        }
    }
}

hipError_t launch_marl_rollout(const MarlArgs& a, int which, hipStream_t st) {
    const unsigned g = (unsigned)((a.rows + 255) / 256);
    if (which == 0) hipLaunchKernelGGL(k_marl_store, dim3(g), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_marl_gae, dim3(g), dim3(256), 0, st, a);
    return hipGetLastError();
}

// ---- host delivery (ch_outputs_to_host): the envs that auto-reset in a step, compacted in ascending env order ------
// One workgroup: each chunk of 1024 envs is ranked by wave ballots (lane prefix) and a scan of the 16 wave totals, so
// the slots follow the env order; then the terminal observation blocks of the listed envs are copied into the
// staging buffer (float4, whole blocks) by the whole workgroup.
constexpr int kStageThreads = 1024;
__global__ __launch_bounds__(kStageThreads) void k_stage_ended(long long E, const uint8_t* reset, const float* term_obs,
                                                               const double* stats, int blk_floats, long long* count,
                                                               long long* env_out, double* stats_out, float* obs_out) {
    __shared__ long long wsum[kStageThreads / 64 + 1];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    long long base = 0;
    for (long long c0 = 0; c0 < E; c0 += kStageThreads) {
        const long long e = c0 + t;
        const bool f = e < E && reset[e] != 0;
        const unsigned long long m = __ballot(f);
        if (lane == 0) wsum[w] = __popcll(m);
        __syncthreads();
        if (t == 0) {
            long long s = 0;
            for (int k = 0; k < kStageThreads / 64; ++k) { const long long v = wsum[k]; wsum[k] = s; s += v; }
            wsum[kStageThreads / 64] = s;
        }
        __syncthreads();
        if (f) {
            const long long slot = base + wsum[w] + __popcll(m & ((1ull << lane) - 1ull));
            env_out[slot] = e;
            if (stats) { stats_out[2 * slot] = stats[2 * e]; stats_out[2 * slot + 1] = stats[2 * e + 1]; }
        }
        base += wsum[kStageThreads / 64];
        __syncthreads();
    }
    if (t == 0) *count = base;
    if (!term_obs) return;
    __threadfence_block();
    __syncthreads();
    const int q = blk_floats / 2;   // float2 per block (R * 86 is even, so every block starts 8-byte aligned)
    for (long long i = t; i < base * q; i += kStageThreads) {
        const long long s = i / q, k = i - s * q;
        reinterpret_cast<float2*>(obs_out + s * blk_floats)[k] =
            reinterpret_cast<const float2*>(term_obs + env_out[s] * blk_floats)[k];
    }
}

hipError_t launch_stage_ended(long long E, const uint8_t* reset, const float* term_obs, const double* stats,
                              int blk_floats, long long* count, long long* env_out, double* stats_out, float* obs_out,
                              hipStream_t st) {
    hipLaunchKernelGGL(k_stage_ended, dim3(1), dim3(kStageThreads), 0, st, E, reset, term_obs, stats, blk_floats, count,
                       env_out, stats_out, obs_out);
    return hipGetLastError();
}

hipError_t launch_rollout(const RolloutArgs& a, int which, hipStream_t st) {
    if (which == 0)
        hipLaunchKernelGGL(k_rollout_store, dim3((unsigned)((a.rows + kRollThreads / 64 - 1) / (kRollThreads / 64))),
                           dim3(kRollThreads), 0, st, a);
    else if (which == 1) hipLaunchKernelGGL(k_rollout_post, dim3((unsigned)((a.rows + 255) / 256)), dim3(256), 0, st, a);
    else if (which == 3) hipLaunchKernelGGL(k_rollout_apply, dim3((unsigned)((a.rows + 255) / 256)), dim3(256), 0, st, a,
                                            a.terminal_value);
    else hipLaunchKernelGGL(k_rollout_gae, dim3((unsigned)((a.rows + 63) / 64)), dim3(64), 0, st, a);
    return hipGetLastError();
}

}  // namespace ch
