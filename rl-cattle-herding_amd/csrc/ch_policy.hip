// ch_policy.hip — on-device policy forward: the SB3 MlpPolicy actor/critic
// (CTDECattleHerder.py:106-127: PPO("MlpPolicy", net_arch pi=[128,128] vf=[128,128], tanh) on the
// flattened (12, 86) observation) and the RLlib per-agent MLP, evaluated for every env of a handle in
// one launch, f32 in / f32 out on the matrix cores.
//
// Layout: a workgroup owns 16 input rows (envs or agents) and carries them through every layer.
// The 8 waves split each layer's output columns into 16x16 tiles (v_mfma_f32_16x16x4_f32: exact f32,
// a k-ordered fma chain per output element).  Hidden activations stay in LDS between layers.  The grid is
// rows/16 workgroups: 4096 envs fill 256 CUs with one workgroup each.  Two kernels: k_mlp2 (the default,
// further down) stages the input rows in LDS once and streams each wave's weight rows from global memory
// straight into registers; k_mlp (the round-2 kernel, kept for first-layer widths past 1152 and for A/B with
// CH_MLP_V1=1) streams K chunks of 64 of inputs and weights through LDS.
//
// Zero input columns.  An observation row has NUM_DRONES live rows of 86 features and zeros after
// them (BaseRLAviary.py:272-342).  With per-row live widths the tile multiplies only the chunks below
// its widest live row: the skipped products are 0 * w, which add +-0 to the sums.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>

#include "ch_internal.h"
#include "ch_rollout_dev.h"
#include "ch_mlp2_dev.h"   // kTM, act_fn, mlp2_body (in this file's anonymous namespace)

namespace ch {

long long* g_mlp_tstamp = nullptr;

namespace {


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
    if (a.rows_dev && row0 >= *a.rows_dev) return;
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


// up to three independent forwards in one launch (MlpMulti): workgroups [start[s], start[s + 1]) run segment s.
// Their workgroups share the CUs (two <4, 2> workgroups fit one CU), so one forward's load latencies overlap the
// other's matrix work -- the rollout's actor, critic and terminal-value critic in one launch.
// SHARE: registers capped at 128 per lane (4 waves per SIMD) so that two 8-wave workgroups fit a CU -- the
// multi-segment launches; a single forward runs without the cap (fewer, faster waves: 17-18 vs 19.7 us alone)
// RT: row tiles of 16 per workgroup (launch_mlp_multi picks 2 or 4 for row counts that fill the chip anyway: each
// weight pair then feeds RT x more MFMAs, the 256-wide RLlib nets' forward is otherwise bound by the weight stream).
// <4, 4, *, 2> is held to 256 registers so that two workgroups share a CU (one's epilogue beside the other's MFMAs)
template <int NW, int TW, bool SHARE = false, int RT = 1>
__global__ __launch_bounds__(64 * NW, SHARE ? 4 : ((NW == 4 && RT == 2) ? 2 : 1)) void k_mlp2(MlpMulti m) {
    int sg = 0;
    if (m.nseg > 1 && (int)blockIdx.x >= m.start[1]) sg = 1;
    if (m.nseg > 2 && (int)blockIdx.x >= m.start[2]) sg = 2;
    mlp2_body<NW, TW, RT>(m.seg[sg], (long long)blockIdx.x - m.start[sg], m.lda, m.ldh, m.role[sg], m.ro);
}

// ch_mlp_pack: layer li's weights into the [tile][pair][half][lane][4] layout (zero past N and K)
__global__ void k_mlp_pack(const float* __restrict__ W, int N, int K, int P, float* __restrict__ out, long long total) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        const int q = (int)(i & 3), l = (int)((i >> 2) & 63), h = (int)((i >> 8) & 1);
        const long long tp = i >> 9;
        const int p = (int)(tp % P), t = (int)(tp / P);
        const int n = 16 * t + (l & 15), k = 32 * p + 8 * (l >> 4) + 4 * h + q;
        out[i] = n < N && k < K ? W[(long long)n * K + k] : 0.0f;
    }
}

}  // namespace

size_t mlp_lds_bytes() { return sizeof(float) * (kTM * kKS + kWMax * kKS + 2 * kTM * (kWMax + 4)); }

long long mlp_packed_floats(int layers, const int* dims, long long* off, int* pairs) {
    long long total = 0;
    for (int li = 0; li < layers; ++li) {
        const int P = pad_pairs(dims[li]), nt = (dims[li + 1] + 15) / 16;
        if (off) off[li] = total;
        if (pairs) pairs[li] = P;
        total += (long long)nt * P * 512;
    }
    return total;
}

hipError_t launch_mlp_pack(const MlpArgs& a, float* dst, hipStream_t st) {
    long long off[4];
    int pairs[4];
    mlp_packed_floats(a.layers, a.dims, off, pairs);
    for (int li = 0; li < a.layers; ++li) {
        const long long n = (long long)((a.dims[li + 1] + 15) / 16) * pairs[li] * 512;
        const int blocks = (int)std::min<long long>((n + 255) / 256, 4096);
        hipLaunchKernelGGL(k_mlp_pack, dim3(blocks), dim3(256), 0, st, a.w[li], a.dims[li + 1], a.dims[li], pairs[li],
                           dst + off[li], n);
    }
    return hipGetLastError();
}

static hipError_t mlp_attrs() {
    // the dynamic-LDS opt-in, once per device (the attribute is per device context)
    static std::atomic<unsigned long long> attr_set{0};
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
        for (const void* f : {reinterpret_cast<const void*>(&k_mlp2<4, 2>), reinterpret_cast<const void*>(&k_mlp2<8, 2>),
                              reinterpret_cast<const void*>(&k_mlp2<8, 1>), reinterpret_cast<const void*>(&k_mlp2<8, 1, true>),
                              reinterpret_cast<const void*>(&k_mlp2<4, 4, false, 2>),
                              reinterpret_cast<const void*>(&k_mlp2<4, 4, false, 4>),
                              reinterpret_cast<const void*>(&k_mlp2<8, 1, false, 2>)}) {
            e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsMax2);
            if (e != hipSuccess) return e;
        }
        attr_set.fetch_or(bit, std::memory_order_relaxed);
    }
    return hipSuccess;
}

// k_mlp2's shape for one net: widest layer, LDS strides (the live input width rounded to whole K pairs, rows
// padded to 4 mod 64 floats); false when the net does not fit it (then k_mlp)
// LDS floats of k_mlp2's tile: RT == 1 input rows and two hidden buffers; RT > 1 the odd layers' hidden buffer in the
// input rows' region (dead after layer 0)
static size_t mlp2_lds_floats(int rt, int lda, int ldh) {
    return rt == 1 ? (size_t)kTM * (lda + 2 * ldh) : (size_t)kTM * rt * ((lda > ldh ? lda : ldh) + ldh);
}

static bool mlp2_shape(const MlpArgs& a, int& maxw, int& lda, int& ldh) {
    int maxhid = 32;
    maxw = 0;
    for (int i = 1; i <= a.layers; ++i) {
        maxw = a.dims[i] > maxw ? a.dims[i] : maxw;
        maxhid = a.dims[i] > maxhid ? a.dims[i] : maxhid;   // (the output too: the sampling epilogue stages there)
    }
    const int np0 = pad_pairs(std::max(a.kcap, 1));
    lda = (32 * np0 + 63) / 64 * 64 + 4;
    ldh = (std::max(maxhid, 32 * kD2) + 32 * kD2 - 1) / (32 * kD2) * (32 * kD2) + 4;
    return np0 <= kMaxPair0 && sizeof(float) * mlp2_lds_floats(1, lda, ldh) <= (size_t)kLdsMax2;
}

bool mlp2_fused_tile(const MlpArgs& a, int& lda, int& ldh, size_t& bytes) {
    int maxw = 0;
    if (!mlp2_shape(a, maxw, lda, ldh) || maxw > 16 * (CH_V2_MAX_BLOCK / 64)) return false;
    if (a.rows_dev || a.row_mask || a.rows_per_env != 1) return false;
    bytes = sizeof(float) * mlp2_lds_floats(1, lda, ldh);
    return true;
}

bool mlp_multi_fits(const MlpArgs* segs, int nseg) {
    static const bool v1 = [] { const char* v = getenv("CH_MLP_V1"); return v && v[0] == '1'; }();
    if (v1) return false;
    for (int s = 0; s < nseg; ++s) {
        int w, la, lh;
        if (!mlp2_shape(segs[s], w, la, lh)) return false;
    }
    return true;
}

hipError_t launch_mlp_multi(const MlpArgs* segs, int nseg, hipStream_t st, const int* roles, const RolloutArgs* ro) {
    static const bool v1 = [] { const char* v = getenv("CH_MLP_V1"); return v && v[0] == '1'; }();
    static const bool nw4 = [] { const char* v = getenv("CH_MLP2_NW4"); return v && v[0] == '1'; }();   // A/B
    static const bool wide4 = [] { const char* v = getenv("CH_MLP_WIDE4"); return v && v[0] == '1'; }();
    if (nseg < 1 || nseg > 3) return hipErrorInvalidValue;
    hipError_t e = mlp_attrs();
    if (e != hipSuccess) return e;
    // row tiles per workgroup: the most (1, 2 or 4 tiles of 16 rows) that still leave a workgroup for every CU across
    // the launch's segments -- each weight pair a workgroup streams then feeds RT times the MFMAs, and the forward of
    // a chip-filling batch waits on that stream, not on the matrix cores; CH_MLP_RT overrides
    static const int rt_env = [] { const char* v = getenv("CH_MLP_RT"); return v ? atoi(v) : 0; }();
    int maxw0 = 0, cus = 256;
    long long rows_all = 0;
    for (int s = 0; s < nseg; ++s) {
        for (int i = 1; i <= segs[s].layers; ++i) maxw0 = std::max(maxw0, segs[s].dims[i]);
        rows_all += segs[s].rows;
    }
    {
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    }
    int rt = 1;
    if (rt_env == 1 || rt_env == 2 || rt_env == 4) rt = rt_env;
    else
        for (int r : {4, 2})
            if (rows_all >= (long long)kTM * r * cus) { rt = r; break; }
    rt = std::min(rt, maxw0 > 128 ? 4 : (nw4 ? 1 : 2));   // the instantiations below
    for (int s = 0; s < nseg; ++s)
        if (maxw0 > 128 && !segs[s].packed) rt = 1;          // the wide row-tiled kernels read packed weights only
    MlpMulti m;
    int maxw = 0, fits = 0, grid = 0, n = 0;
    for (;;) {   // the largest rt <= the chosen one whose tile fits the LDS
        std::memset(&m, 0, sizeof(m));
        maxw = 0; fits = !v1; grid = 0; n = 0;
        for (int s = 0; s < nseg; ++s) {
            const long long g = (segs[s].rows + kTM * rt - 1) / (kTM * rt);
            if (g == 0) continue;
            int w, la, lh;
            fits &= mlp2_shape(segs[s], w, la, lh);
            maxw = std::max(maxw, w); m.lda = std::max(m.lda, la); m.ldh = std::max(m.ldh, lh);
            m.seg[n] = segs[s];
            m.seg[n].tstamp = g_mlp_tstamp;
            m.role[n] = roles ? roles[s] : kRoleNone;
            m.start[n] = grid;
            grid += (int)g;
            ++n;
        }
        if (rt == 1 || sizeof(float) * mlp2_lds_floats(rt, m.lda, m.ldh) <= (size_t)kLdsMax2) break;
        rt >>= 1;
    }
    if (n == 0) return hipSuccess;
    if (ro) m.ro = *ro;
    m.nseg = n;
    m.start[n] = grid;
    const size_t lds2 = sizeof(float) * mlp2_lds_floats(rt, m.lda, m.ldh);
    if (fits && lds2 <= (size_t)kLdsMax2) {
        if (maxw > 128) {
            // RT > 1: four waves of 64 columns each, one per SIMD (the 512-register budget of a lone wave holds the
            // 4 x 4 accumulators and the 4 x 4 weight ring)
            if (rt == 4) hipLaunchKernelGGL((k_mlp2<4, 4, false, 4>), dim3((unsigned)grid), dim3(256), lds2, st, m);
            else if (rt == 2) hipLaunchKernelGGL((k_mlp2<4, 4, false, 2>), dim3((unsigned)grid), dim3(256), lds2, st, m);
            else hipLaunchKernelGGL((k_mlp2<8, 2>), dim3((unsigned)grid), dim3(512), lds2, st, m);
        } else if (nw4) hipLaunchKernelGGL((k_mlp2<4, 2>), dim3((unsigned)grid), dim3(256), lds2, st, m);
        else if (n > 1 && rt == 1) {   // two workgroups per CU (128 registers)
            hipLaunchKernelGGL((k_mlp2<8, 1, true>), dim3((unsigned)grid), dim3(512), lds2, st, m);
        } else {
            if (rt >= 2) hipLaunchKernelGGL((k_mlp2<8, 1, false, 2>), dim3((unsigned)grid), dim3(512), lds2, st, m);
            else hipLaunchKernelGGL((k_mlp2<8, 1>), dim3((unsigned)grid), dim3(512), lds2, st, m);
        }
        return hipGetLastError();
    }
    // the round-2 kernel, one launch per net (no rollout epilogues: callers check mlp_multi_fits first)
    for (int s = 0; s < n; ++s) {
        if (m.role[s] != kRoleNone) return hipErrorInvalidValue;
        const MlpArgs& a = m.seg[s];
        const unsigned g = (unsigned)((a.rows + kTM - 1) / kTM);
        int w = 0;
        for (int i = 1; i <= a.layers; ++i) w = std::max(w, a.dims[i]);
        if (w <= 128) hipLaunchKernelGGL((k_mlp<8, 1, 2>), dim3(g), dim3(512), mlp_lds_bytes(), st, a);
        else if (wide4) hipLaunchKernelGGL((k_mlp<4, 4, 1>), dim3(g), dim3(256), mlp_lds_bytes(), st, a);
        else hipLaunchKernelGGL((k_mlp<8, 2, 2>), dim3(g), dim3(512), mlp_lds_bytes(), st, a);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_mlp(const MlpArgs& a, hipStream_t st) { return launch_mlp_multi(&a, 1, st); }

}  // namespace ch
