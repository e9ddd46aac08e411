// ch_policy.hip — on-device policy forward: the SB3 MlpPolicy actor/critic
// (CTDECattleHerder.py:106-127: PPO("MlpPolicy", net_arch pi=[128,128] vf=[128,128], tanh) on the
// flattened (12, 86) observation) and the RLlib per-agent MLP, evaluated for every env of a handle in
// one launch, f32 in / f32 out on the matrix cores.
//
// Layout: a workgroup owns 16 input rows (envs or agents) and carries them through every layer.
// The 4 waves split each layer's output columns into 16x16 tiles (v_mfma_f32_16x16x4_f32: exact f32,
// a k-ordered fma chain per output element).  The K dimension streams in chunks of 64 through LDS, from
// a register ring that keeps the next 3 chunks of input and weight rows in flight (1 for 256-wide
// layers) while the current one is multiplied.  Hidden activations stay in LDS between layers.  The grid is rows/16
// workgroups: 4096 envs fill 256 CUs with one workgroup each.
//
// Zero input columns.  An observation row has NUM_DRONES live rows of 86 features and zeros after
// them (BaseRLAviary.py:272-342).  With per-row live widths the tile multiplies only the chunks below
// its widest live row: the skipped products are 0 * w, which add +-0 to the sums.
#include <hip/hip_runtime.h>

#include <atomic>

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
template <bool AG, int TW, int DEPTH, int NW>
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

    // Register ring of DEPTH chunks: 4 input floats and 4 TW float4 of weights per thread and chunk.  Thread
    // t covers weight row n = t / 16 + 16 i, columns 4 (t % 16) .. +3 of the chunk (a 256-B row segment
    // per 16 lanes); rows past the layer width are zero.  Loads are branch-free: clamped (always valid)
    // addresses and a select.  DEPTH chunks are in flight while one is multiplied: a chunk's multiplies
    // take a few hundred cycles, its loads (L2/MALL) thousands.
    constexpr int kWP = 4 * TW;                     // float4 per thread: 64 TW rows x kKC / 4 / 256
    const bool vec = (K & 3) == 0;   // weight rows 16-B aligned: float4 loads
    float xr[DEPTH][4];
    float4 wr[DEPTH][kWP];
    const int wn0 = tid >> 4, wc = (tid & 15) * 4;
    // fetch chunk kc into ring slot S (a literal: the ring stays in registers)
#define CH_MLP_FETCH(S, kc_)                                                                                        \
    do {                                                                                                            \
        const int kcf = (kc_);                                                                                      \
        if (AG && tid < 256) {                                                                                      \
            const int r = tid >> 4, c = (tid & 15) * 4;                                                             \
            const float* src = Ag + min(row0 + r, a.rows - 1) * lda;                                                \
            _Pragma("unroll") for (int q = 0; q < 4; ++q) xr[S][q] = src[min(kcf + c + q, K - 1)];                  \
        }                                                                                                           \
        if (vec) {                                                                                                  \
            _Pragma("unroll") for (int i = 0; i < kWP; ++i) {                                                       \
                const int n = wn0 + 4 * NW * i, k = kcf + wc;                                                           \
                wr[S][i] = *reinterpret_cast<const float4*>(W + min(n, N - 1) * K + min(k, K - 4));                 \
            }                                                                                                       \
        } else {                                                                                                    \
            _Pragma("unroll") for (int i = 0; i < kWP; ++i) {                                                       \
                const int n = wn0 + 4 * NW * i, k = kcf + wc;                                                           \
                const float* src = W + min(n, N - 1) * K;                                                           \
                wr[S][i] = make_float4(src[min(k, K - 1)], src[min(k + 1, K - 1)], src[min(k + 2, K - 1)],         \
                                       src[min(k + 3, K - 1)]);                                                     \
            }                                                                                                       \
        }                                                                                                           \
    } while (0)
    // chunk c from ring slot S into LDS -- out-of-range rows and columns masked to zero here, not at the load,
    // so that no instruction waits for a load before its store -- then the fetch of chunk c + DEPTH into the
    // freed slot (DEPTH chunks in flight during the multiplies), then the multiplies
#define CH_MLP_STEP(S)                                                                                              \
    if constexpr (S < DEPTH) {                                                                                      \
        const int c = c0 + S, kc = c * kKC;                                                                         \
        if (c < nch) {                                                                                              \
            if (AG && tid < 256) {                                                                                  \
                const int r = tid >> 4, cc = (tid & 15) * 4;                                                        \
                const bool rv = row0 + r < a.rows;                                                                  \
                float xq[4];                                                                                        \
                _Pragma("unroll") for (int q = 0; q < 4; ++q) xq[q] = rv && kc + cc + q < K ? xr[S][q] : 0.0f;      \
                *reinterpret_cast<float4*>(xs + r * kKS + cc) = make_float4(xq[0], xq[1], xq[2], xq[3]);            \
            }                                                                                                       \
            _Pragma("unroll") for (int i = 0; i < kWP; ++i) {                                                       \
                const int n = wn0 + 4 * NW * i, k = kc + wc;                                                            \
                const bool nv = n < N;                                                                              \
                const float4 v = wr[S][i];                                                                          \
                *reinterpret_cast<float4*>(ws + n * kKS + wc) =                                                     \
                    make_float4(nv && k < K ? v.x : 0.0f, nv && k + 1 < K ? v.y : 0.0f, nv && k + 2 < K ? v.z : 0.0f, \
                                nv && k + 3 < K ? v.w : 0.0f);                                                      \
            }                                                                                                       \
            __syncthreads();                                                                                        \
            if (c + DEPTH < nch) CH_MLP_FETCH(S, kc + DEPTH * kKC);                                                 \
            float av[kKC / 4], bv[TW][kKC / 4];                                                                     \
            _Pragma("unroll") for (int ks = 0; ks < kKC / 4; ++ks) {                                                \
                const int kk = ks * 4 + (lane >> 4);                                                                \
                if constexpr (AG) av[ks] = xs[(lane & 15) * kKS + kk];                                              \
                else av[ks] = Al[(lane & 15) * ldl + kc + kk];                                                      \
                _Pragma("unroll") for (int j = 0; j < TW; ++j)                                                      \
                    bv[j][ks] = ws[((wave + NW * j) * 16 + (lane & 15)) * kKS + kk];                                 \
            }                                                                                                       \
            _Pragma("unroll") for (int ks = 0; ks < kKC / 4; ++ks) {                                                \
                _Pragma("unroll") for (int j = 0; j < TW; ++j)                                                      \
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ks], bv[j][ks], acc[j], 0, 0, 0);              \
            }                                                                                                       \
            __syncthreads();                                                                                        \
        }                                                                                                           \
    }
    const int nch = (kloop + kKC - 1) / kKC;
    const int c0 = 0;   // (the prologue's chunk indices)
    (void)c0;
    if (0 < nch) CH_MLP_FETCH(0, 0);
    if constexpr (DEPTH > 1) { if (1 < nch) CH_MLP_FETCH(1, kKC); }
    if constexpr (DEPTH > 2) { if (2 < nch) CH_MLP_FETCH(2, 2 * kKC); }
    if constexpr (DEPTH > 3) { if (3 < nch) CH_MLP_FETCH(3, 3 * kKC); }
    // A[row l&15][k = 4 ks + (l >> 4)], B[k][col l&15] (16x16x4 f32 operand map).  All operands of a chunk
    // are read first (one LDS latency), then the MFMAs issue back to back.  Hidden-layer A columns past K
    // read zeros or finite stale values, which meet zero weight rows.
    for (int c0 = 0; c0 < nch; c0 += DEPTH) {
        CH_MLP_STEP(0)
        CH_MLP_STEP(1)
        CH_MLP_STEP(2)
        CH_MLP_STEP(3)
    }
#undef CH_MLP_STEP
#undef CH_MLP_FETCH
    // epilogue: C/D map col = lane & 15, row = 4 (lane >> 4) + r
#pragma unroll
    for (int j = 0; j < TW; ++j) {
        const int t = wave + NW * j;
        if (t >= nt) continue;
        const int col = t * 16 + (lane & 15);
        const float bv = col < N && bias ? bias[col] : 0.0f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = (lane >> 4) * 4 + r;
            float v = acc[j][r] + bv;
            if (!last) {
                out[row * ldo + col] = col < N ? act_fn(v, a.hidden_act) : 0.0f;
            } else if (col < N && row0 + row < a.rows && (!a.row_mask || a.row_mask[row0 + row])) {
                if (a.clip) v = fminf(fmaxf(v, a.lo), a.hi);
                a.y[(row0 + row) * (long long)N + col] = v;
            }
        }
    }
    if (!last) {   // columns past this layer's tiles: zero for the next layer's chunk reads
        for (int idx = tid; idx < kTM * (kWMax - 16 * nt); idx += 64 * NW) {
            const int r = idx / (kWMax - 16 * nt), c = 16 * nt + idx - r * (kWMax - 16 * nt);
            out[r * ldo + c] = 0.0f;
        }
    }
    __syncthreads();
}


// WIDE: some layer is wider than 128 (the RLlib 256-wide model): 16-column tiles up to 4 per wave, one
// chunk in flight; otherwise (the SB3 actor / critic, 128 wide) up to 2 tiles per wave and two chunks in
// flight.  Separate kernels keep the narrow one's register ring from spilling.  (Tried and reverted: a
// split-K layer with each wave loading its K chunks straight from global memory into the MFMA operand
// layout, no LDS staging: 85 us for one 16-row tile of the 1032-wide forward vs 35 us, the 16-row x
// 64-byte operand loads being far slower than the coalesced staging loads.)
template <bool WIDE>
__global__ __launch_bounds__(WIDE ? 256 : 512) void k_mlp(MlpArgs a) {
    constexpr int NW = WIDE ? 4 : 8;   // waves: the narrow kernel gives every wave one 16-column tile
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
    // masked forward: a tile with no selected row has nothing to do (the usual case for the terminal-value
    // forward of a rollout, where only the envs that just reset are selected)
    const bool any = __syncthreads_or(a.row_mask && threadIdx.x < kTM && row0 + threadIdx.x < a.rows &&
                                      a.row_mask[row0 + threadIdx.x] != 0);
    if (a.row_mask && !any) return;
    const int kloop0 = kmax;
    float* cur = h0;
    float* nxt = h1;
    for (int li = 0; li < a.layers; ++li) {
        const bool last = li == a.layers - 1;
        const int nt = (a.dims[li + 1] + 15) >> 4;
        if constexpr (WIDE) {
            if (li == 0) {
                if (nt <= 4) mlp_layer<true, 1, 1, NW>(a, 0, a.x, a.dims[0], nullptr, 0, a.dims[0], kloop0, xs, ws, cur, ldh, last);
                else if (nt > 8) mlp_layer<true, 4, 1, NW>(a, 0, a.x, a.dims[0], nullptr, 0, a.dims[0], kloop0, xs, ws, cur, ldh, last);
                else mlp_layer<true, 2, 1, NW>(a, 0, a.x, a.dims[0], nullptr, 0, a.dims[0], kloop0, xs, ws, cur, ldh, last);
            } else {
                const int K = a.dims[li];
                if (nt <= 4) mlp_layer<false, 1, 1, NW>(a, li, nullptr, 0, cur, ldh, K, K, xs, ws, nxt, ldh, last);
                else if (nt > 8) mlp_layer<false, 4, 1, NW>(a, li, nullptr, 0, cur, ldh, K, K, xs, ws, nxt, ldh, last);
                else mlp_layer<false, 2, 1, NW>(a, li, nullptr, 0, cur, ldh, K, K, xs, ws, nxt, ldh, last);
                float* t = cur; cur = nxt; nxt = t;
            }
        } else {   // 8 waves, one tile each; two chunks in flight (3 measured no faster)
            if (li == 0) {
                mlp_layer<true, 1, 2, NW>(a, 0, a.x, a.dims[0], nullptr, 0, a.dims[0], kloop0, xs, ws, cur, ldh, last);
            } else {
                const int K = a.dims[li];
                mlp_layer<false, 1, 2, NW>(a, li, nullptr, 0, cur, ldh, K, K, xs, ws, nxt, ldh, last);
                float* t = cur; cur = nxt; nxt = t;
            }
        }
    }
}

}  // namespace

size_t mlp_lds_bytes() { return sizeof(float) * (kTM * kKS + kWMax * kKS + 2 * kTM * (kWMax + 4)); }

hipError_t launch_mlp(const MlpArgs& a, hipStream_t st) {
    // the dynamic-LDS opt-in, once per device (the attribute is per device context)
    static std::atomic<unsigned long long> attr_set{0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (!(attr_set.load(std::memory_order_relaxed) & bit)) {
        for (const void* f : {reinterpret_cast<const void*>(&k_mlp<false>), reinterpret_cast<const void*>(&k_mlp<true>)}) {
            e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlp_lds_bytes());
            if (e != hipSuccess) return e;
        }
        attr_set.fetch_or(bit, std::memory_order_relaxed);
    }
    const long long grid = (a.rows + kTM - 1) / kTM;
    if (grid == 0) return hipSuccess;
    bool wide = false;
    for (int i = 1; i <= a.layers; ++i) wide |= a.dims[i] > 128;
    if (wide) hipLaunchKernelGGL(k_mlp<true>, dim3((unsigned)grid), dim3(256), mlp_lds_bytes(), st, a);
    else hipLaunchKernelGGL(k_mlp<false>, dim3((unsigned)grid), dim3(512), mlp_lds_bytes(), st, a);
    return hipGetLastError();
}

}  // namespace ch
