// ch_mlp2_dev.h -- the device side of the on-device policy forward: constants, the tanh epilogue and k_mlp2's
// workgroup body (mlp2_body), shared by the forward kernels (ch_policy.hip) and the step kernel that runs the
// actor forward of a PPO collection step in the workgroup that wrote the observations (ch_step.hip k_step2_actor).
#pragma once
#include <hip/hip_runtime.h>

#include "ch_internal.h"
#include "ch_rollout_dev.h"

namespace ch {
namespace {

constexpr int kTM = 16;            // rows per workgroup
constexpr int kKC = 64;            // K chunk
constexpr int kKS = kKC + 4;       // LDS row stride of a chunk (conflict-free operand reads)
constexpr int kWMax = 256;         // widest layer

using f32x4 = __attribute__((ext_vector_type(4))) float;

// tanh(v) = 1 - 2 / (exp(2v) + 1) on the hardware exp2 and reciprocal: an absolute error of a few 1e-8 (the relative
// error of a small |v| is larger -- the tests hold the forward's outputs, i.e. absolute errors of the hidden units
// summed through the next layer, to 1e-5 and 2e-5), about 8 instructions instead of ocml's tanhf.  A 64-row tile
// applies it to 64 values per lane and layer, which made the epilogues as long as the matrix loops.
// CH_OCML_TANH: ocml's tanhf.
constexpr float kTanhScale = 2.8853900817779268f;   // 2 log2(e): 2^(kTanhScale v) = e^(2v)
// tanh from s = kTanhScale v (the hidden epilogue folds its bias into the fma that forms s): 5 instructions, two of
// them transcendental, with the bias add
__device__ __forceinline__ float tanh_fast_scaled(float s) {
    return fmaf(-2.0f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(s) + 1.0f), 1.0f);
}
__device__ __forceinline__ float tanh_fast(float v) {
#ifdef CH_OCML_TANH
    return tanhf(v);
#else
    return tanh_fast_scaled(v * kTanhScale);
#endif
}

__device__ __forceinline__ float act_fn(float v, int act) {
    if (act == CH_ACT_TANH) return tanh_fast(v);
    if (act == CH_ACT_RELU) return v > 0.0f ? v : 0.0f;
    return v;
}

// ---- k_mlp2: weights streamed from global memory straight into the MFMA operand layout (the default) --------------
//
// k_mlp (above) staged every 64-wide K chunk of the weights through LDS between two barriers, with two chunks in
// flight: 20 us for the 4096-row SB3 actor forward, 17 % of the f32 MFMA peak, the waves mostly waiting.  k_mlp2
// keeps the 16-row tile and the 8 waves (each wave 16 or 32 of a layer's output columns), but
//   * the input rows of the tile are staged in LDS once, whole (the live width only), with one barrier;
//   * each wave loads its own weight columns straight from global memory (L2-resident: every workgroup reads the
//     same matrix) into registers, and keeps D = 4 K-pairs of 32 in flight with no barrier inside a layer;
//   * the next layer's first pairs are requested before this layer's epilogue, and the barriers order LDS only
//     (a __syncthreads would wait for those loads).
// K order.  Pair p of 32 columns is 8 MFMAs; in MFMA e lane group g = lane >> 4 supplies k = 32 p + 8 g + e
// (A[row][k] from LDS, B[k][col] = W[col][k]).  Each output is the f32 fma chain over k in the order (p, e, g);
// zero columns (dead observation rows, block-diagonal zeros) add +0 exactly, so the live-width skip and the fused
// actor-critic stay bit-identical to the full-width and separate forwards.
// Packed weights (ch_mlp.packed, ch_mlp_pack): layer li as [tile t][pair p][half h][lane l][4], element
// W[16 t + (l & 15)][32 p + 8 (l >> 4) + 4 h + q] (zero past N and K): a wave's load of one half-pair is 1 KB
// contiguous.  Raw nn.Linear weights: each lane reads two float4 of its own row, 16 rows per instruction.
// Static load counts.  Every fetch issues the same loads whatever its pair index (raw: addresses clamped into
// the row; the A side is zero past the live width, the layer width and the padded pair count, so a clamped weight
// meets a zero), and the pair count is padded to a multiple of D: no load is conditional, so the compiler's vmcnt
// waits count exactly the D - 1 younger pairs instead of draining every load in flight.

constexpr int kD2 = 4;         // K pairs in flight per wave
constexpr int kMaxPair0 = 36;  // first-layer live width <= 1152 (else k_mlp)
constexpr int kLdsMax2 = 160 * 1024 - 1024;   // k_mlp2 dynamic LDS cap (the static kmax word included)

// D pairs in flight (kD2; 2 when a pair's MFMAs already take ~1 k cycles: TW x RT >= 8 tiles per wave)
template <int TW, int D = kD2>
struct Ring2 {
    float4 v[D][TW][2];
};
template <int TW, int RT> constexpr int ring_depth() { return TW * RT >= 8 ? 2 : kD2; }

__device__ __host__ __forceinline__ int pad_pairs(int k) { return ((k + 31) / 32 + kD2 - 1) / kD2 * kD2; }

// the wave's weight source for one layer: per tile, the packed tile's lane base, or the raw row
template <int TW>
struct WSrc {
    const float* w[TW];
    int K;
};

// request pair p into ring slot S (S a literal: the ring stays in registers).  MODE 0: packed; 1: raw rows,
// K % 8 == 0 and 16-B aligned (two float4 at min(k, K - 8)); 2: raw rows, element loads at min(k + q, K - 1)
template <int S, int TW, int MODE, int D>
__device__ __forceinline__ void mlp2_fetch(Ring2<TW, D>& r, const WSrc<TW>& ws, int p, int g) {
#pragma unroll
    for (int j = 0; j < TW; ++j) {
        if constexpr (MODE == 0) {
            r.v[S][j][0] = *reinterpret_cast<const float4*>(ws.w[j] + p * 512);
            r.v[S][j][1] = *reinterpret_cast<const float4*>(ws.w[j] + p * 512 + 256);
        } else if constexpr (MODE == 1) {
            const float* src = ws.w[j] + min(32 * p + 8 * g, ws.K - 8);
            r.v[S][j][0] = *reinterpret_cast<const float4*>(src);
            r.v[S][j][1] = *reinterpret_cast<const float4*>(src + 4);
        } else {
            const float* src = ws.w[j];
            const int k = 32 * p + 8 * g, K = ws.K;
            r.v[S][j][0] = make_float4(src[min(k, K - 1)], src[min(k + 1, K - 1)], src[min(k + 2, K - 1)], src[min(k + 3, K - 1)]);
            r.v[S][j][1] = make_float4(src[min(k + 4, K - 1)], src[min(k + 5, K - 1)], src[min(k + 6, K - 1)], src[min(k + 7, K - 1)]);
        }
    }
}

__device__ __forceinline__ float f4_at(const float4& v, int i) {
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// pair p from ring slot S: the lane's 8 A values of each of the RT row tiles from LDS, 8 MFMAs per (row tile, column
// tile); then (FETCH) refill the slot with pair p + D.  One weight pair feeds RT row tiles: a workgroup of 16 RT rows
// streams each weight once for all of them.
template <int S, int NT, int TW, int MODE, bool FETCH, int RT, int D>
__device__ __forceinline__ void mlp2_pair(f32x4 (&acc)[RT][TW], Ring2<TW, D>& r, const WSrc<TW>& ws, const float* A, int lda,
                                          int p, int lane) {
    const int g = lane >> 4;
    float4 a0[RT], a1[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        const float* ap = A + (16 * t + (lane & 15)) * lda + 32 * p + 8 * g;
        a0[t] = *reinterpret_cast<const float4*>(ap);
        a1[t] = *reinterpret_cast<const float4*>(ap + 4);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            const float av = f4_at(e < 4 ? a0[t] : a1[t], e & 3);
#pragma unroll
            for (int j = 0; j < NT; ++j)
                acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, f4_at(r.v[S][j][e >> 2], e & 3), acc[t][j], 0, 0, 0);
        }
    }
    if constexpr (FETCH) mlp2_fetch<S, TW, MODE>(r, ws, p + D, g);
    // keep the refill here: left alone, the scheduler sinks all four refills below the group's last MFMAs, and
    // the next group then waits for loads issued a moment earlier
    __builtin_amdgcn_sched_barrier(0);
}

// npad >= 1 pairs: the steady state refills every slot it drains, the last (up to D) pairs only drain.  The loads
// are those of the padded count (a multiple of D, in bounds: packed layers hold their padded pairs, raw fetches
// clamp); a count that is not a multiple of D -- the first layer's live pairs -- skips the drain's all-zero tail
// (+0 products: the outputs are bit-identical)
template <int NT, int TW, int MODE, int RT, int D>
__device__ __forceinline__ void mlp2_loop(f32x4 (&acc)[RT][TW], Ring2<TW, D>& r, const WSrc<TW>& ws, const float* A, int lda,
                                          int npad, int lane) {
    static_assert(D == 2 || D == 4, "ring depth");
    int p0 = 0;
    for (; p0 < npad - D; p0 += D) {
        mlp2_pair<0, NT, TW, MODE, true, RT>(acc, r, ws, A, lda, p0 + 0, lane);
        mlp2_pair<1, NT, TW, MODE, true, RT>(acc, r, ws, A, lda, p0 + 1, lane);
        if constexpr (D == 4) {
            mlp2_pair<2, NT, TW, MODE, true, RT>(acc, r, ws, A, lda, p0 + 2, lane);
            mlp2_pair<3, NT, TW, MODE, true, RT>(acc, r, ws, A, lda, p0 + 3, lane);
        }
    }
    mlp2_pair<0, NT, TW, MODE, false, RT>(acc, r, ws, A, lda, p0 + 0, lane);
    if (p0 + 1 < npad) mlp2_pair<1, NT, TW, MODE, false, RT>(acc, r, ws, A, lda, p0 + 1, lane);
    if constexpr (D == 4) {
        if (p0 + 2 < npad) mlp2_pair<2, NT, TW, MODE, false, RT>(acc, r, ws, A, lda, p0 + 2, lane);
        if (p0 + 3 < npad) mlp2_pair<3, NT, TW, MODE, false, RT>(acc, r, ws, A, lda, p0 + 3, lane);
    }
}

template <int TW>
__device__ __forceinline__ int layer_mode(const MlpArgs& a, int li) {
    return a.packed ? 0 : (((a.vec_w >> li) & 1) ? 1 : 2);
}

// one wave's share of layer li: its tiles -- strided (t = wave + NW j) or, in a block-diagonal layer (ch_mlp
// split_out / split_in), contiguous (t = TW wave + j, all in one block) -- their count, and the K pairs it
// multiplies, [pb, pb + npad): a block-diagonal layer's wave skips the other block's zero weights (each output's
// fma chain loses only +0 terms, so the result is bit-identical)
struct Plan2 {
    int ntw, pb, npad;
    bool contig;
    int rs, tile0;   // row-split output layer (mlp2_plan_out): the wave's row tile (-1: not split) and its column tile
};

template <int NW, int TW>
__device__ __forceinline__ Plan2 mlp2_plan(const MlpArgs& a, int li, int wave, int np0) {
    const int N = a.dims[li + 1], K = a.dims[li], nt = (N + 15) >> 4;
    Plan2 pl;
    pl.contig = li > 0 && a.split_out[li] > 0;   // (validated on the host)
    if (pl.contig) {
        const int t0 = TW * wave;
        pl.ntw = max(0, min(TW, nt - t0));
        const bool hi = 16 * t0 >= a.split_out[li];
        pl.pb = hi ? a.split_in[li] / 32 : 0;
        pl.npad = pad_pairs(hi ? K - a.split_in[li] : a.split_in[li]);
    } else {
        pl.ntw = wave < nt ? min(TW, (nt - wave + NW - 1) / NW) : 0;   // tiles wave, wave + NW, ... below nt
        pl.pb = 0;
        pl.npad = li == 0 ? np0 : pad_pairs(K);
    }
    pl.rs = -1;
    pl.tile0 = 0;
    return pl;
}

// the output layer li > 0 of a row-tiled workgroup (RT > 1) whose column tiles x row tiles fit the waves (and not
// block-diagonal): wave w computes column tile w % nt of row tile w / nt alone, instead of the first nt waves each
// running all RT row tiles while the rest wait -- each output's fma chain is the same (bit-identical)
template <int NW, int TW, int RT>
__device__ __forceinline__ Plan2 mlp2_plan_out(const MlpArgs& a, int li, int wave) {
    Plan2 pl = mlp2_plan<NW, TW>(a, li, wave, 0);
    const int nt = (a.dims[li + 1] + 15) >> 4;
    // (not <4, 4, *, 2>, held to 256 registers for two workgroups per CU: the split's accumulators spill there)
    if (RT > 1 && !(NW == 4 && RT == 2) && !pl.contig && nt * RT <= NW) {
        const bool has = wave < nt * RT;
        pl.ntw = has ? 1 : 0;
        pl.rs = has ? wave / nt : 0;
        pl.tile0 = has ? wave - (wave / nt) * nt : 0;
    }
    return pl;
}

template <int NW, int TW>
__device__ __forceinline__ int mlp2_tile(const Plan2& pl, int wave, int j) {
    return pl.rs >= 0 ? pl.tile0 : (pl.contig ? TW * wave + j : wave + NW * j);
}

// the wave's weight source for layer li (tiles past the layer width clamped to its last tile / row: computed,
// never stored), starting at pair pl.pb, and the loads of its first D pairs
// PKO: packed weights only (the host launches such a kernel only with ch_mlp.packed set): the raw-row fetch paths
// and their address registers are not compiled in
// (the layer's scalars given: the tile's start reads layer 0's with its own, in one scalar round trip)
template <int NW, int TW, int D, bool PKO = false>
__device__ __forceinline__ void mlp2_prologue_s(int N, int K, int pkp, int vw, const float* pk, const float* wl,
                                                long long pko, int li, const Plan2& pl, Ring2<TW, D>& r, WSrc<TW>& ws,
                                                int wave, int lane) {
    const int nt = (N + 15) >> 4;
    const int mode = (PKO || pk) ? 0 : (((vw >> li) & 1) ? 1 : 2);
    ws.K = K - 32 * pl.pb;
#pragma unroll
    for (int j = 0; j < TW; ++j) {
        const int t = min(mlp2_tile<NW, TW>(pl, wave, j), nt - 1);
        ws.w[j] = mode == 0 ? pk + pko + ((long long)t * pkp + pl.pb) * 512 + lane * 4
                            : wl + (long long)min(t * 16 + (lane & 15), N - 1) * K + 32 * pl.pb;
    }
    const int g = lane >> 4;
#define CH_MLP2_PRO(M)                                                                                              \
    mlp2_fetch<0, TW, M>(r, ws, 0, g); mlp2_fetch<1, TW, M>(r, ws, 1, g);                                            \
    if constexpr (D == 4) { mlp2_fetch<2, TW, M>(r, ws, 2, g); mlp2_fetch<3, TW, M>(r, ws, 3, g); }
    if (PKO || mode == 0) { CH_MLP2_PRO(0); } else if (mode == 1) { CH_MLP2_PRO(1); } else { CH_MLP2_PRO(2); }
#undef CH_MLP2_PRO
}

template <int NW, int TW, int D, bool PKO = false>
__device__ __forceinline__ void mlp2_prologue(const MlpArgs& a, int li, const Plan2& pl, Ring2<TW, D>& r, WSrc<TW>& ws,
                                              int wave, int lane) {
    // the layer's scalars read together and pinned in scalar registers here: read where each is first used
    // (inside a branch, after another field's use) they would cost a chain of dependent scalar-cache round
    // trips (~0.5 k cycles each at kernel start) before the first weight load
    int N = a.dims[li + 1], K = a.dims[li], pkp = a.pk_pairs[li], vw = a.vec_w;
    const float* pk = a.packed;
    const float* wl = a.w[li];
    long long pko = a.pk_off[li];
    asm volatile("" : "+s"(N), "+s"(K), "+s"(pkp), "+s"(vw), "+s"(pk), "+s"(wl), "+s"(pko));
    mlp2_prologue_s<NW, TW, D, PKO>(N, K, pkp, vw, pk, wl, pko, li, pl, r, ws, wave, lane);
}

// a hidden layer's epilogue: bias + activation of the wave's NT tiles into the LDS activations, straight-line.
// Written per element with the activation switch and the bounds inside (act_fn, col < N), the 64-row tile's
// epilogue compiled to ~1000 scalar branches and took as long as the layer's matrix loop (17.6 k cycles,
// tools/mlp_marl_probe.py).  Columns past the layer width land in [N, 32 npn), which the caller zeroes next.
template <int ACT, int NT, int NW, int TW, int RT>
__device__ __forceinline__ void mlp2_epi_hidden(const f32x4 (&acc)[RT][TW], const float (&bcol)[TW], float* out, int ldh,
                                                const Plan2& pl, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int col = mlp2_tile<NW, TW>(pl, wave, j) * 16 + (lane & 15);
        const float bs = bcol[j] * kTanhScale;   // tanh: the bias folded into the exponent's fma
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v;
#ifdef CH_OCML_TANH
                if constexpr (ACT == CH_ACT_TANH) v = tanhf(acc[t][j][r] + bcol[j]);
#else
                if constexpr (ACT == CH_ACT_TANH) v = tanh_fast_scaled(fmaf(acc[t][j][r], kTanhScale, bs));
#endif
                else if constexpr (ACT == CH_ACT_RELU) { v = acc[t][j][r] + bcol[j]; v = v > 0.0f ? v : 0.0f; }
                else v = acc[t][j][r] + bcol[j];
                out[(16 * t + (lane >> 4) * 4 + r) * ldh + col] = v;
            }
    }
}

// the output layer's epilogue: bias, optional clip, into y (or, STAGE, the LDS buffer the rollout epilogue reads);
// each lane's row bound and row mask are read once per row, not per element
template <bool STAGE, int NT, int NW, int TW, int RT>
__device__ __forceinline__ void mlp2_epi_out(const MlpArgs& a, const f32x4 (&acc)[RT][TW], const float (&bcol)[TW],
                                             float* out, int ldh, const Plan2& pl, int wave, int lane, long long row0,
                                             int N) {
    const bool clip = a.clip != 0;
    const float lo = a.lo, hi = a.hi;
    const long long rows = a.rows;
    const uint8_t* mask = a.row_mask;
    float* y = a.y;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 16 * t + (lane >> 4) * 4 + r;
            const bool ok = row0 + row < rows && (!mask || mask[row0 + row]);
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int col = mlp2_tile<NW, TW>(pl, wave, j) * 16 + (lane & 15);
                float v = acc[t][j][r] + bcol[j];
                if (clip) v = fminf(fmaxf(v, lo), hi);
                if (ok && col < N) {
                    if constexpr (STAGE) out[row * ldh + col] = v;
                    else y[(row0 + row) * (long long)N + col] = v;
                }
            }
        }
}

// a workgroup barrier ordering LDS only: the weight loads in flight stay in flight (__syncthreads' release fence
// would wait for every outstanding global load)
__device__ __forceinline__ void mlp2_lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// NW waves of TW 16-column tiles each (<4, 2>: layers <= 128 wide, one wave per SIMD with two independent
// accumulator chains; <8, 2>: <= 256 wide).  lda / ldh: LDS row strides (floats) of the staged input rows and of
// the hidden activations, both = 4 mod 64 (conflict-free 16-B operand reads), wide enough for the padded pair
// counts.
// RT row tiles of 16 per workgroup (RT > 1: the hidden buffer of odd layers reuses the input rows' region, which is
// dead after layer 0 -- see mlp2_lds_floats).
template <int NW, int TW, int RT>
__device__ __forceinline__ void mlp2_body(const MlpArgs& a, long long blk, int lda, int ldh, int role,
                                          const RolloutArgs& ro) {
    extern __shared__ __align__(16) float sm[];
    constexpr int TMR = kTM * RT;      // rows of the workgroup
    static_assert(TMR <= 64, "the live-width scan reduces the rows in wave 0");
    float* xa = sm;                    // [TMR][lda]
    float* hb0 = RT == 1 ? xa + kTM * lda : xa + TMR * (lda > ldh ? lda : ldh);   // [TMR][ldh]
    float* hb1 = RT == 1 ? hb0 + kTM * ldh : xa;
    __shared__ int kmax, kany;
    __shared__ int qslot[TMR];         // kRoleValue: each row's slot in the deferred-bootstrap queue (-1: none)
    constexpr int kT = 64 * NW;        // threads
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const long long row0 = blk * TMR;
    constexpr bool PKO = NW == 4 && RT > 1;   // packed weights only (launch_mlp_multi)
    // the arguments the tile's start needs -- the live-width scan's and the first layer's (plan, weight fetch, input
    // rows) -- read together and pinned (see mlp2_prologue): one scalar round trip before the first loads (read where
    // each is used, the start of a tile was ~5 k cycles of dependent scalar reads, tools/mlp_marl_probe.py --ctde)
    const int* rows_dev = a.rows_dev;
    const int* env_n = a.env_n;
    const uint8_t* row_mask = a.row_mask;
    long long rows = a.rows, rpe = a.rows_per_env;
    int d0 = a.dims[0], ku = a.k_unit;
    int d1 = a.dims[1], pkp0 = a.pk_pairs[0], vw = a.vec_w, kcap = a.kcap;
    const float* pk = a.packed;
    const float* w0 = a.w[0];
    const float* x = a.x;
    long long pko0 = a.pk_off[0];
    asm volatile("" : "+s"(rows_dev), "+s"(env_n), "+s"(row_mask), "+s"(rows), "+s"(rpe), "+s"(d0), "+s"(ku), "+s"(d1),
                 "+s"(pkp0), "+s"(vw), "+s"(kcap), "+s"(pk), "+s"(w0), "+s"(x), "+s"(pko0));
    if (rows_dev && row0 >= *rows_dev) return;   // (uniform: every thread reads the same count)
    long long* ts = a.tstamp && tid == 0 ? a.tstamp + blk * 16 : nullptr;
    if (ts) ts[0] = clock64();
    // the tile's live input width (the drones of each row's env) and row mask: the rows are all in wave 0 (TMR <= 64);
    // requested first, reduced after the loads below are in flight
    // (only the loads here: the width is formed after the weight and row loads below are issued, so that waiting for
    // these does not hold them back; 32-bit row arithmetic, rows < 2^31)
    const bool rl = tid < TMR && row0 + tid < rows;
    int n_env = 0, jr = 0, mr = 0;
    if (rl) {
        if (env_n) {
            const int ri = (int)(row0 + tid), rp = (int)rpe;
            const int e = rp == 1 ? ri : ri / rp;
            jr = ri - e * rp;
            n_env = env_n[e];
        }
        if (row_mask) mr = row_mask[row0 + tid];
    }

    // the first layer's first weight pairs (L2 hits), then the first pass of the tile's input rows (from HBM) at the
    // host's cap width kcap (zeroed past the live width when stored): thread t owns row t / (4 NW) and float4 columns
    // t % (4 NW) + 4 NW i, i < nld, of the padded width 32 np0.  Both are in flight while wave 0 reduces the live width.
    Ring2<TW, ring_depth<TW, RT>()> ring;
    WSrc<TW> ws;
    Plan2 pl;   // layer 0 (mlp2_plan; its pair count follows the scan)
    {
        const int nt = (d1 + 15) >> 4;
        pl.contig = false;
        pl.ntw = wave < nt ? min(TW, (nt - wave + NW - 1) / NW) : 0;
        pl.pb = 0;
        pl.npad = 1;
        pl.rs = -1;
        pl.tile0 = 0;
    }
    mlp2_prologue_s<NW, TW, ring_depth<TW, RT>(), PKO>(d1, d0, pkp0, vw, pk, w0, pko0, 0, pl, ring, ws, wave, lane);
    if (ts) ts[1] = clock64();
    const int np0 = min(pad_pairs(max(kcap, 1)), kMaxPair0);
    // rows srow + 16 rt; as many row tiles per pass as the kQ registers hold (RT nld <= kQ for the reference's nets)
    constexpr int kTPR = 4 * NW, kQ = RT > 1 && NW < 8 ? 8 : 8 * kMaxPair0 / kTPR;   // (RT > 1: more passes, fewer registers)
    const int K0 = d0, srow = tid / kTPR, sc = 4 * (tid % kTPR), nld = (8 * np0 + kTPR - 1) / kTPR;
    const int rper = max(1, min(RT, kQ / nld));
    const bool vec_x = (vw >> 7) & 1, vec2_x = !vec_x && (K0 & 1) == 0 && K0 >= 2 && (reinterpret_cast<uintptr_t>(x) & 7) == 0;
    float4 xr[kQ];
    // (the vector / element choice outside the unrolled loop: inside it, every iteration's two paths wrote the same
    // registers and the compiler drained the loads in flight at each join -- one memory round trip per float4)
    auto load_pass = [&](int rb) {
        const long long rr0 = row0 + 16 * rb + srow;
        if (vec_x) {
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const int t = q / nld, i = q - t * nld, c = sc + 4 * kTPR * i;
                if (t < rper && rb + t < RT)
                    xr[q] = *reinterpret_cast<const float4*>(x + min(rr0 + 16 * t, rows - 1) * K0 + min(c, K0 - 4));
            }
        } else if (vec2_x) {   // even rows (the RLlib agents' 86 floats): two float2 (past the row: clamped, zeroed below)
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const int t = q / nld, i = q - t * nld, c = sc + 4 * kTPR * i;
                if (t < rper && rb + t < RT) {
                    const float* xs = x + min(rr0 + 16 * t, rows - 1) * K0;
                    const float2 lo = *reinterpret_cast<const float2*>(xs + min(c, K0 - 2));
                    const float2 hi = *reinterpret_cast<const float2*>(xs + min(c + 2, K0 - 2));
                    xr[q] = make_float4(lo.x, lo.y, hi.x, hi.y);
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < kQ; ++q) {
                const int t = q / nld, i = q - t * nld, c = sc + 4 * kTPR * i;
                if (t < rper && rb + t < RT) {
                    const float* xs = x + min(rr0 + 16 * t, rows - 1) * K0;
                    xr[q] = make_float4(xs[min(c, K0 - 1)], xs[min(c + 1, K0 - 1)], xs[min(c + 2, K0 - 1)], xs[min(c + 3, K0 - 1)]);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);   // every load above issued before the first wait
    };
    load_pass(0);
    asm volatile("" : "+v"(mr), "+v"(n_env));   // (the row mask and width used from here: their wait lands here)
    if (ts) ts[2] = clock64();
    if (wave == 0) {
        int km = 0;
        if (rl) km = env_n ? min(rpe == 1 ? n_env * ku : (jr < n_env ? ku : 0), d0) : d0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) km = max(km, __shfl_xor(km, o));
        const bool anyr = __ballot(mr != 0) != 0;
        if (lane == 0) { kmax = km; kany = anyr ? 1 : 0; }
    }
    mlp2_lds_barrier();   // (LDS only: the loads stay in flight)
    if (row_mask && !kany) return;
    const int kloop = min(kmax, kcap);   // (the host sized the tile for kcap)
    pl.npad = min((max(kloop, 1) + 31) / 32, np0);   // the first layer multiplies its live pairs only
    for (int rb = 0; rb < RT; rb += rper) {
        if (rb > 0) load_pass(rb);
        const long long rr0 = row0 + 16 * rb + srow;
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int t = q / nld, i = q - t * nld, c = sc + 4 * kTPR * i;
            if (t < rper && rb + t < RT && c < 32 * np0) {
                const bool srv = rr0 + 16 * t < rows;
                float4 v = xr[q];
                v.x = srv && c < kloop ? v.x : 0.0f;
                v.y = srv && c + 1 < kloop ? v.y : 0.0f;
                v.z = srv && c + 2 < kloop ? v.z : 0.0f;
                v.w = srv && c + 3 < kloop ? v.w : 0.0f;
                *reinterpret_cast<float4*>(xa + (16 * (rb + t) + srow) * lda + c) = v;
            }
        }
    }
    if (ts) ts[3] = clock64();
    mlp2_lds_barrier();
    if (ts) ts[4] = clock64();

    const float* cur = xa;
    int ldc = lda;
    for (int li = 0; li < a.layers; ++li) {
        const bool last = li == a.layers - 1;
        const int N = a.dims[li + 1];
        const int mode = PKO ? 0 : layer_mode<TW>(a, li);
        const int ntw = pl.ntw;
        const float* A = cur + 32 * pl.pb;
        float bcol[TW];
#pragma unroll
        for (int j = 0; j < TW; ++j) {
            const int col = mlp2_tile<NW, TW>(pl, wave, j) * 16 + (lane & 15);
            bcol[j] = a.b[li] && col < N ? a.b[li][col] : 0.0f;
        }
        if (RT > 1 && !(NW == 4 && RT == 2) && pl.rs >= 0) {
            // the row-split output layer (mlp2_plan_out): one row tile of one column tile per wave
            f32x4 acc1[1][TW];
#pragma unroll
            for (int j = 0; j < TW; ++j) acc1[0][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            const float* A1 = A + 16 * pl.rs * ldc;
            if (ntw > 0) {
                if (PKO || mode == 0) mlp2_loop<1, TW, 0, 1>(acc1, ring, ws, A1, ldc, pl.npad, lane);
                else if constexpr (!PKO) {
                    if (mode == 1) mlp2_loop<1, TW, 1, 1>(acc1, ring, ws, A1, ldc, pl.npad, lane);
                    else mlp2_loop<1, TW, 2, 1>(acc1, ring, ws, A1, ldc, pl.npad, lane);
                }
            }
            if (ts && li < 3) ts[5 + 2 * li] = clock64();
            float* out = (li & 1 ? hb1 : hb0) + 16 * pl.rs * ldh;
            if (ntw > 0) {
                if (role != kRoleNone) mlp2_epi_out<true, 1, NW>(a, acc1, bcol, out, ldh, pl, wave, lane, row0 + 16 * pl.rs, N);
                else mlp2_epi_out<false, 1, NW>(a, acc1, bcol, out, ldh, pl, wave, lane, row0 + 16 * pl.rs, N);
            }
            break;
        }
        f32x4 acc[RT][TW];
#pragma unroll
        for (int t = 0; t < RT; ++t)
#pragma unroll
            for (int j = 0; j < TW; ++j) acc[t][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#define CH_MLP2_LOOP(NT_)                                                                                           \
        if (PKO || mode == 0) mlp2_loop<NT_, TW, 0, RT>(acc, ring, ws, A, ldc, pl.npad, lane);                       \
        else if constexpr (!PKO) {                                                                                   \
            if (mode == 1) mlp2_loop<NT_, TW, 1, RT>(acc, ring, ws, A, ldc, pl.npad, lane);                          \
            else mlp2_loop<NT_, TW, 2, RT>(acc, ring, ws, A, ldc, pl.npad, lane);                                    \
        }
        if (ntw == TW) { CH_MLP2_LOOP(TW); }
        else if constexpr (TW >= 4) { if (ntw == 3) { CH_MLP2_LOOP(3); } else if (ntw == 2) { CH_MLP2_LOOP(2); } else if (ntw == 1) { CH_MLP2_LOOP(1); } }
        else if (ntw > 0) { CH_MLP2_LOOP(1); }
#undef CH_MLP2_LOOP
        if (ts && li < 3) ts[5 + 2 * li] = clock64();
        // the next layer's first pairs, in flight during this epilogue and barrier
        const Plan2 cpl = pl;
        const int npn = last ? 0 : pad_pairs(N);
        if (!last) {
            pl = li + 2 == a.layers ? mlp2_plan_out<NW, TW, RT>(a, li + 1, wave) : mlp2_plan<NW, TW>(a, li + 1, wave, 0);
            mlp2_prologue<NW, TW, ring_depth<TW, RT>(), PKO>(a, li + 1, pl, ring, ws, wave, lane);
        }
        float* out = li & 1 ? hb1 : hb0;
        // epilogue: C/D map col = lane & 15, row = 16 t + 4 (lane >> 4) + r
        if (!last) {
            const int act = a.hidden_act;
#define CH_MLP2_EPI(NT_)                                                                                            \
            if (act == CH_ACT_TANH) mlp2_epi_hidden<CH_ACT_TANH, NT_, NW>(acc, bcol, out, ldh, cpl, wave, lane);       \
            else if (act == CH_ACT_RELU) mlp2_epi_hidden<CH_ACT_RELU, NT_, NW>(acc, bcol, out, ldh, cpl, wave, lane);  \
            else mlp2_epi_hidden<CH_ACT_NONE, NT_, NW>(acc, bcol, out, ldh, cpl, wave, lane);
            if (ntw == TW) { CH_MLP2_EPI(TW); }
            else if constexpr (TW >= 4) { if (ntw == 3) { CH_MLP2_EPI(3); } else if (ntw == 2) { CH_MLP2_EPI(2); } else if (ntw == 1) { CH_MLP2_EPI(1); } }
            else if (ntw > 0) { CH_MLP2_EPI(1); }
#undef CH_MLP2_EPI
        } else if (ntw > 0) {
            // the output layer (narrow: one or a few tiles); a rollout role stages it in LDS for the epilogue below
#define CH_MLP2_OUT(NT_)                                                                                            \
            if (role != kRoleNone) mlp2_epi_out<true, NT_, NW>(a, acc, bcol, out, ldh, cpl, wave, lane, row0, N);    \
            else mlp2_epi_out<false, NT_, NW>(a, acc, bcol, out, ldh, cpl, wave, lane, row0, N);
            if (ntw == TW) { CH_MLP2_OUT(TW); }
            else if constexpr (TW >= 4) { if (ntw == 3) { CH_MLP2_OUT(3); } else if (ntw == 2) { CH_MLP2_OUT(2); } else { CH_MLP2_OUT(1); } }
            else { CH_MLP2_OUT(1); }
#undef CH_MLP2_OUT
        }
        if (ts && li < 2) ts[11 + li] = clock64();
        if (last) break;
        // columns [N, 32 npn) of the activations: zero for the next layer's padded pairs
        const int zc = 32 * npn - N;
        for (int idx = tid; idx < TMR * zc; idx += kT) {
            const int r = idx / zc;
            out[r * ldh + N + idx - r * zc] = 0.0f;
        }
        mlp2_lds_barrier();
        if (ts && li < 2) ts[6 + 2 * li] = clock64();
        cur = out;
        ldc = ldh;
    }
    if (ts) ts[10] = clock64();
    if (role == kRoleSample) {
        // the actor's means (staged in the last layer's would-be output buffer) become the samples, their env
        // actions and per-dimension log-probability terms -- spread over the whole workgroup -- then each row's
        // terms are summed in action order by one lane (k_rollout_store's order)
        float* lp = a.layers & 1 ? hb0 : hb1;
        const int NA = a.dims[a.layers];
        const int nrow = (int)min((long long)TMR, a.rows - row0);
        mlp2_lds_barrier();
        for (int idx = tid; idx < nrow * NA; idx += kT) {
            const int r = idx / NA, k = idx - r * NA;
            lp[r * ldh + k] = rollout_sample(ro, ro.t, k, row0 + r, lp[r * ldh + k]);
        }
        mlp2_lds_barrier();
        if (tid < nrow) {
            float s = 0.0f;
            for (int k = 0; k < NA; ++k) s += lp[tid * ldh + k];
            ro.log_probs[(long long)ro.t * ro.rows + row0 + tid] = s;
        }
    } else if (role == kRoleValue) {
        // the critic's values (staged like the actor's means), the previous step's post (reward, next episode
        // start, deferred-bootstrap queue) and this step's episode starts for the tile's rows; at t = 0 the
        // observation rows into obs[0]
        const float* vl = a.layers & 1 ? hb0 : hb1;
        mlp2_lds_barrier();
        if (tid < TMR) {
            const long long e = row0 + tid;
            int slot = -1;
            if (e < a.rows) {
                ro.values[(long long)ro.t * ro.rows + e] = vl[tid * ldh];
                bool q = false;
                const float les = ro.t > 0 ? rollout_post_env(ro, ro.t - 1, e, &q) : ro.last_episode_starts[e];
                ro.episode_starts[(long long)ro.t * ro.rows + e] = les;
                if (q) {
                    slot = atomicAdd(ro.tv_count, 1);
                    ro.tv_row[slot] = (long long)(ro.t - 1) * ro.rows + e;
                }
            }
            qslot[tid] = slot;
        }
        mlp2_lds_barrier();
        const int nq4 = ro.obs_dim / 4;
        for (int r = 0; r < TMR; ++r) {
            const int slot = qslot[r];
            if (slot < 0) continue;
            const float4* src = reinterpret_cast<const float4*>(ro.term_obs + (row0 + r) * ro.obs_dim);
            float4* dst = reinterpret_cast<float4*>(ro.tv_obs + (long long)slot * ro.obs_dim);
            for (int k = tid; k < nq4; k += kT) dst[k] = src[k];
        }
        if (ro.copy_obs) {
            const int nr = (int)min((long long)TMR, a.rows - row0);
            for (int k = tid; k < nr * nq4; k += kT) {
                const int r = k / nq4, c = k - r * nq4;
                reinterpret_cast<float4*>(ro.obs + ((long long)ro.t * ro.rows + row0 + r) * ro.obs_dim)[c] =
                    reinterpret_cast<const float4*>(a.x + (row0 + r) * (long long)ro.obs_dim)[c];
            }
        }
    } else if (role == kRoleTvApply) {
        // ch_rollout_collect's flush of the deferred truncation bootstrap: rewards[tv_row[q]] += gamma V(terminal obs
        // q) for the tile's queue rows, k_rollout_apply's fma without its launch
        const float* vl = a.layers & 1 ? hb0 : hb1;
        mlp2_lds_barrier();
        if (tid < TMR) {
            const long long q = row0 + tid;
            if (q < (a.rows_dev ? (long long)*a.rows_dev : a.rows)) {
                const long long row = ro.tv_row[q];
                ro.rewards[row] = fmaf(ro.gamma, vl[tid * ldh + ro.v_col], ro.rewards[row]);
            }
        }
    }
}

}  // namespace
}  // namespace ch
