// ch_policy.hip — on-device policy forward: the SB3 MlpPolicy actor/critic
// (CTDECattleHerder.py:106-127: PPO("MlpPolicy", net_arch pi=[128,128] vf=[128,128], tanh) on the
// flattened (12, 86) observation) and the RLlib per-agent MLP, evaluated for every env of a handle in
// one launch, f32 in / f32 out on the matrix cores.
//
// Layout: a workgroup owns 16 input rows (envs or agents) and carries them through every layer.
// The 4 waves split each layer's output columns into 16x16 tiles (v_mfma_f32_16x16x4_f32: exact f32,
// a k-ordered fma chain per output element).  The K dimension streams in chunks of 32 through LDS:
// the next chunk of the input rows and of the weight rows is loaded into registers while the current
// one is multiplied.  Hidden activations stay in LDS between layers.  The grid is rows/16
// workgroups: 4096 envs fill 256 CUs with one workgroup each.
//
// Zero input columns.  An observation row has NUM_DRONES live rows of 86 features and zeros after
// them (BaseRLAviary.py:272-342).  With per-row live widths the tile multiplies only the chunks below
// its widest live row: the skipped products are 0 * w, which add +-0 to the sums.
#include <hip/hip_runtime.h>

#include "ch_internal.h"

namespace ch {

namespace {

constexpr int kTM = 16;            // rows per workgroup
constexpr int kKC = 64;            // K chunk
constexpr int kKS = kKC + 4;       // LDS row stride of a chunk (conflict-free operand reads)
constexpr int kWMax = 256;         // widest layer

using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ float act_fn(float v, int act) {
    if (act == CH_ACT_TANH) return tanhf(v);
    if (act == CH_ACT_RELU) return v > 0.0f ? v : 0.0f;
    return v;
}

// One layer: out[16][N] = act(A[16][K] W^T + b).  A comes from global memory (layer 0, rows of x)
// or from LDS (hidden activations).  Only k < kloop is multiplied (kloop <= K, see "Zero input
// columns").  The last layer writes y (clipped) instead of LDS.
// TW = 16-column tiles per wave (the layer's tiles rounded up to 4 TW): every wave runs the same
// straight-line MFMA sequence; tiles past the layer width multiply zero weight rows (a branch per
// tile would make the compiler shuffle the accumulators around every MFMA).
template <bool AG, int TW>
__device__ __forceinline__ void mlp_layer(const MlpArgs& a, int li, const float* __restrict__ Ag, long long lda,
                                          const float* Al, int ldl, int K, int kloop, float* xs, float* ws, float* out,
                                          int ldo, bool last) {
    const int N = a.dims[li + 1];
    const float* __restrict__ W = a.w[li];
    const float* __restrict__ bias = a.b[li];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: tile branches stay scalar
    const int nt = (N + 15) >> 4;                    // 16-column tiles
    const long long row0 = (long long)blockIdx.x * kTM;
    f32x4 acc[TW];
#pragma unroll
    for (int j = 0; j < TW; ++j) acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    // register prefetch of one chunk: 4 input floats and 4 TW float4 of weights per thread.  Thread
    // t covers weight row n = t / 16 + 16 i, columns 4 (t % 16) .. +3 of the chunk (a 256-B row
    // segment per 16 lanes); rows past the layer width are zero.  Loads are branch-free: clamped
    // (always valid) addresses and a select, so a chunk's loads are all in flight together.
    constexpr int kWP = 4 * TW;                     // float4 per thread: 64 TW rows x kKC / 4 / 256
    const bool vec = (K & 3) == 0;   // weight rows 16-B aligned: float4 loads
    float xr[4];
    float4 wr[kWP];
    const int wn0 = tid >> 4, wc = (tid & 15) * 4;
    auto fetch = [&](int kc) {
        if constexpr (AG) {
            const int r = tid >> 4, c = (tid & 15) * 4;
            const bool rv = row0 + r < a.rows;
            const float* src = Ag + min(row0 + r, a.rows - 1) * lda;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float v = src[min(kc + c + q, K - 1)];
                xr[q] = rv && kc + c + q < K ? v : 0.0f;
            }
        }
        if (vec) {
#pragma unroll
            for (int i = 0; i < kWP; ++i) {
                const int n = wn0 + 16 * i, k = kc + wc;
                const float4 v = *reinterpret_cast<const float4*>(W + min(n, N - 1) * K + min(k, K - 4));
                wr[i] = n < N && k < K ? v : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
        } else {
#pragma unroll
            for (int i = 0; i < kWP; ++i) {
                const int n = wn0 + 16 * i, k = kc + wc;
                const bool nv = n < N;
                const float* src = W + min(n, N - 1) * K;
                const float v0 = src[min(k, K - 1)], v1 = src[min(k + 1, K - 1)], v2 = src[min(k + 2, K - 1)],
                            v3 = src[min(k + 3, K - 1)];
                wr[i] = make_float4(nv && k < K ? v0 : 0.0f, nv && k + 1 < K ? v1 : 0.0f, nv && k + 2 < K ? v2 : 0.0f,
                                    nv && k + 3 < K ? v3 : 0.0f);
            }
        }
    };
    if (kloop > 0) fetch(0);
    for (int kc = 0; kc < kloop; kc += kKC) {
        if constexpr (AG) {
            const int r = tid >> 4, c = (tid & 15) * 4;
            *reinterpret_cast<float4*>(xs + r * kKS + c) = make_float4(xr[0], xr[1], xr[2], xr[3]);
        }
#pragma unroll
        for (int i = 0; i < kWP; ++i) *reinterpret_cast<float4*>(ws + (wn0 + 16 * i) * kKS + wc) = wr[i];
        __syncthreads();
        if (kc + kKC < kloop) fetch(kc + kKC);   // in flight during the multiplies below
        // A[row l&15][k = 4 ks + (l >> 4)], B[k][col l&15] (16x16x4 f32 operand map).  All operands of
        // the chunk are read first (one LDS latency), then the MFMAs issue back to back.  Hidden-layer A
        // columns past K read zeros or finite stale values, which meet zero weight rows.
        float av[kKC / 4], bv[TW][kKC / 4];
#pragma unroll
        for (int ks = 0; ks < kKC / 4; ++ks) {
            const int kk = ks * 4 + (lane >> 4);
            if constexpr (AG) av[ks] = xs[(lane & 15) * kKS + kk];
            else av[ks] = Al[(lane & 15) * ldl + kc + kk];
#pragma unroll
            for (int j = 0; j < TW; ++j) bv[j][ks] = ws[((wave + 4 * j) * 16 + (lane & 15)) * kKS + kk];
        }
#pragma unroll
        for (int ks = 0; ks < kKC / 4; ++ks) {
#pragma unroll
            for (int j = 0; j < TW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ks], bv[j][ks], acc[j], 0, 0, 0);
        }
        __syncthreads();
    }
    // epilogue: C/D map col = lane & 15, row = 4 (lane >> 4) + r
#pragma unroll
    for (int j = 0; j < TW; ++j) {
        const int t = wave + 4 * j;
        if (t >= nt) continue;
        const int col = t * 16 + (lane & 15);
        const float bv = col < N && bias ? bias[col] : 0.0f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = (lane >> 4) * 4 + r;
            float v = acc[j][r] + bv;
            if (!last) {
                out[row * ldo + col] = col < N ? act_fn(v, a.hidden_act) : 0.0f;
            } else if (col < N && row0 + row < a.rows) {
                if (a.clip) v = fminf(fmaxf(v, a.lo), a.hi);
                a.y[(row0 + row) * (long long)N + col] = v;
            }
        }
    }
    if (!last) {   // columns past this layer's tiles: zero for the next layer's chunk reads
        for (int idx = tid; idx < kTM * (kWMax - 16 * nt); idx += 256) {
            const int r = idx / (kWMax - 16 * nt), c = 16 * nt + idx - r * (kWMax - 16 * nt);
            out[r * ldo + c] = 0.0f;
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_mlp(MlpArgs a) {
    extern __shared__ __align__(16) float sm[];
    float* xs = sm;                                  // [16][kKS]
    float* ws = xs + kTM * kKS;                      // [kWMax][kKS]
    float* h0 = ws + kWMax * kKS;                    // [16][kWMax + 4]
    float* h1 = h0 + kTM * (kWMax + 4);
    const int ldh = kWMax + 4;
    __shared__ int kmax;
    const long long row0 = (long long)blockIdx.x * kTM;
    // widest live input row of this tile
    if (threadIdx.x == 0) kmax = 0;
    __syncthreads();
    if (threadIdx.x < kTM && row0 + threadIdx.x < a.rows) {
        int k = a.dims[0];
        if (a.env_n) {
            const long long r = row0 + threadIdx.x, e = r / a.rows_per_env;
            const int j = (int)(r - e * a.rows_per_env), n = a.env_n[e];
            k = a.rows_per_env == 1 ? n * a.k_unit : (j < n ? a.k_unit : 0);
            k = min(k, a.dims[0]);
        }
        atomicMax(&kmax, k);
    }
    __syncthreads();
    const int kloop0 = kmax;
    float* cur = h0;
    float* nxt = h1;
    for (int li = 0; li < a.layers; ++li) {
        const bool last = li == a.layers - 1;
        const int nt = (a.dims[li + 1] + 15) >> 4;
        if (li == 0) {
            if (nt <= 4) mlp_layer<true, 1>(a, 0, a.x, a.dims[0], nullptr, 0, a.dims[0], kloop0, xs, ws, cur, ldh, last);
            else if (nt <= 8) mlp_layer<true, 2>(a, 0, a.x, a.dims[0], nullptr, 0, a.dims[0], kloop0, xs, ws, cur, ldh, last);
            else mlp_layer<true, 4>(a, 0, a.x, a.dims[0], nullptr, 0, a.dims[0], kloop0, xs, ws, cur, ldh, last);
        } else {
            const int K = a.dims[li];
            if (nt <= 4) mlp_layer<false, 1>(a, li, nullptr, 0, cur, ldh, K, K, xs, ws, nxt, ldh, last);
            else if (nt <= 8) mlp_layer<false, 2>(a, li, nullptr, 0, cur, ldh, K, K, xs, ws, nxt, ldh, last);
            else mlp_layer<false, 4>(a, li, nullptr, 0, cur, ldh, K, K, xs, ws, nxt, ldh, last);
            float* t = cur; cur = nxt; nxt = t;
        }
    }
}

}  // namespace

size_t mlp_lds_bytes() { return sizeof(float) * (kTM * kKS + kWMax * kKS + 2 * kTM * (kWMax + 4)); }

hipError_t launch_mlp(const MlpArgs& a, hipStream_t st) {
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mlp),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlp_lds_bytes());
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const long long grid = (a.rows + kTM - 1) / kTM;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mlp, dim3((unsigned)grid), dim3(256), mlp_lds_bytes(), st, a);
    return hipGetLastError();
}

}  // namespace ch
