// ch_rollout_dev.h -- the device-side arithmetic of the SB3 rollout store, shared by k_rollout_store
// (ch_aux.hip) and the sampling / value epilogues of the policy forward (ch_policy.hip k_mlp2), so both
// produce the same bits.  stable_baselines3 2.7 OnPolicyAlgorithm.collect_rollouts / DiagGaussianDistribution
// (restated; SB3 is not in this image: "parity unpinned" to its source).
#pragma once
#include "ch_internal.h"

namespace ch {

__device__ __forceinline__ void philox_k(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t lo0 = 0xD2511F53u * c[0], hi0 = __umulhi(0xD2511F53u, c[0]);
        uint32_t lo1 = 0xCD9E8D57u * c[2], hi1 = __umulhi(0xCD9E8D57u, c[2]);
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

// action k of env e at step t: a = mu + exp(log_std) eps, eps ~ N(0, 1) from Philox4x32-10 (seed, t, k, e) by
// Box-Muller; stored unclipped, the env gets it clipped to the Box [-1, 1]; returns this dimension's
// torch.distributions.Normal.log_prob term -((a - mu)^2) / (2 var) - log(std) - log(sqrt(2 pi))
__device__ __forceinline__ float rollout_sample(const RolloutArgs& a, int t, int k, long long e, float mu) {
    uint32_t c[4] = {(uint32_t)t, (uint32_t)k, (uint32_t)e, (uint32_t)(e >> 32)};
    philox_k(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
    const float u1 = ((float)(c[0] >> 8) + 1.0f) * (1.0f / 16777216.0f);   // (0, 1]
    const float u2 = (float)(c[1] >> 8) * (1.0f / 16777216.0f);
    const float eps = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853071795865f * u2);
    const float ls = a.log_std[k], sd = expf(ls);
    const float act = mu + sd * eps;
    const long long row = (long long)t * a.rows + e;
    a.actions[row * a.act_dim + k] = act;
    if (k < a.env_act_dim) a.env_actions[e * a.env_act_dim + k] = fminf(fmaxf(act, -1.0f), 1.0f);
    const float d = act - mu, var = sd * sd;
    return -(d * d) / (2.0f * var) - ls - 0.91893853320467274f;
}

// after the env step t: reward (+ gamma V(terminal obs) for truncations) into the buffer, next episode start
// (returned too, so that the caller need not read back what it just stored); *queue: the bootstrap is deferred
// (a.defer) and this env's terminal observation must be queued
__device__ __forceinline__ float rollout_post_env(const RolloutArgs& a, int t, long long e, bool* queue = nullptr) {
    const long long row = (long long)t * a.rows + e;
    const bool te = a.terminated[e] != 0, tr = a.truncated[e] != 0;
    float r = a.reward[e];
    const bool boot = tr && !te && (a.terminal_value || a.defer);
    if (boot && !a.defer) r = fmaf(a.gamma, a.terminal_value[e * a.tv_ld], r);   // rewards[idx] += gamma * terminal_value
    a.rewards[row] = r;
    if (queue) *queue = boot && a.defer;
    const float les = (te || tr) ? 1.0f : 0.0f;
    a.last_episode_starts[e] = les;
    return les;
}

}  // namespace ch
