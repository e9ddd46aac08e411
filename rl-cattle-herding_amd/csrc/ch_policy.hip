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
#include <cstdlib>

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


// NW waves per workgroup, up to TWMAX 16-column tiles per wave, DEPTH K-chunks in flight:
//   <8, 1, 2> the SB3 actor / critic (128 wide): every wave one tile, two chunks in flight;
//   <8, 2, 2> layers up to 256 wide (the fused actor-critic, the RLlib model): two tiles per wave, still eight
//             waves and two chunks in flight;
//   <4, 4, 1> the previous 256-wide kernel (four waves of up to four tiles, one chunk in flight), kept for
//             A/B (CH_MLP_WIDE4=1): at 4096 rows it ran the fused 1032-256-256-49 forward in 41.9 us, twice the
//             128-wide forward's 20.3 us (profiles/r03/c/policy_kernel_stats.csv).
// Separate instantiations keep the narrow one's register ring from spilling.  (Tried and reverted: a split-K
// layer with each wave loading its K chunks straight from global memory into the MFMA operand layout, no LDS
// staging: 85 us for one 16-row tile of the 1032-wide forward vs 35 us, the 16-row x 64-byte operand loads
// being far slower than the coalesced staging loads.)
template <int NW, int TWMAX, int DEPTH>
__global__ __launch_bounds__(64 * NW) void k_mlp(MlpArgs a) {
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
        const int tw = nt <= NW ? 1 : (nt <= 2 * NW ? 2 : 4);   // tiles per wave this layer needs
        const bool ag = li == 0;
        const int K = ag ? a.dims[0] : a.dims[li];
        const int kl = ag ? kloop0 : K;
        float* out = ag ? cur : nxt;
#define CH_MLP_LAYER(TW)                                                                                            \
        if (ag) mlp_layer<true, TW, DEPTH, NW>(a, 0, a.x, a.dims[0], nullptr, 0, K, kl, xs, ws, out, ldh, last);     \
        else mlp_layer<false, TW, DEPTH, NW>(a, li, nullptr, 0, cur, ldh, K, kl, xs, ws, out, ldh, last)
        if constexpr (TWMAX >= 4) {
            if (tw >= 4) { CH_MLP_LAYER(4); } else if (tw == 2) { CH_MLP_LAYER(2); } else { CH_MLP_LAYER(1); }
        } else if constexpr (TWMAX >= 2) {
            if (tw >= 2) { CH_MLP_LAYER(2); } else { CH_MLP_LAYER(1); }
        } else {
            CH_MLP_LAYER(1);
        }
#undef CH_MLP_LAYER
        if (!ag) { float* t = cur; cur = nxt; nxt = t; }
    }
}

}  // namespace

size_t mlp_lds_bytes() { return sizeof(float) * (kTM * kKS + kWMax * kKS + 2 * kTM * (kWMax + 4)); }

hipError_t launch_mlp(const MlpArgs& a, hipStream_t st) {
    // the dynamic-LDS opt-in, once per device (the attribute is per device context)
    static std::atomic<unsigned long long> attr_set{0};
    static const bool wide4 = [] { const char* v = getenv("CH_MLP_WIDE4"); return v && v[0] == '1'; }();
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (!(attr_set.load(std::memory_order_relaxed) & bit)) {
        for (const void* f : {reinterpret_cast<const void*>(&k_mlp<8, 1, 2>), reinterpret_cast<const void*>(&k_mlp<8, 2, 2>),
                              reinterpret_cast<const void*>(&k_mlp<4, 4, 1>)}) {
            e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mlp_lds_bytes());
            if (e != hipSuccess) return e;
        }
        attr_set.fetch_or(bit, std::memory_order_relaxed);
    }
    const long long grid = (a.rows + kTM - 1) / kTM;
    if (grid == 0) return hipSuccess;
    int maxw = 0;
    for (int i = 1; i <= a.layers; ++i) maxw = a.dims[i] > maxw ? a.dims[i] : maxw;
    if (maxw <= 128) hipLaunchKernelGGL((k_mlp<8, 1, 2>), dim3((unsigned)grid), dim3(512), mlp_lds_bytes(), st, a);
    else if (wide4) hipLaunchKernelGGL((k_mlp<4, 4, 1>), dim3((unsigned)grid), dim3(256), mlp_lds_bytes(), st, a);
    else hipLaunchKernelGGL((k_mlp<8, 2, 2>), dim3((unsigned)grid), dim3(512), mlp_lds_bytes(), st, a);
    return hipGetLastError();
}

}  // namespace ch
