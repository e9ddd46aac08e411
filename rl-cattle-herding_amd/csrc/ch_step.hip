// ch_step.hip — the fused env-step kernel, v2: a drone wave and cow waves in dataflow (gfx950 / MI355X).
//
// One launch advances every environment by one control step (reference: BaseAviary.step,
// sb3_envs/BaseAviary.py:335-465; rllib_envs/BaseAviary.py:320-438 + marl_wrapper.py:77-119).
//
// Every piece of this step is a long dependent fp64 chain (PID, rigid-body substeps, libm sequences),
// so the kernel is organised around latency rather than lanes.  A workgroup holds G environments
// (G*N <= 64) in 2..4 waves:
//   wave 0 ("drone wave"), the critical path:
//       Philox action -> PID -> 4 physics substeps -> state, LDS positions      [signal D]
//       per-drone reward terms + nearest-neighbour observation entries         [signal T]
//       (wait H) closest cow from the cow waves' distance table -> cattle term
//       per-env reward / terminated / truncated / curriculum / metrics bookkeeping
//   waves 1.. ("cow waves"), concurrently on the other SIMDs:
//       flock alpha term as a table of the M(M-1)/2 unordered cow pairs      [A: all cow waves]
//       per-cow alpha row sums in the reference's neighbour order (each pair quantity is symmetric and
//       the two directed contributions are exact negations: bit-identical to the ordered loop)
//       (wait D) cow-drone distances, herded winding number, cattle observation entries   [signal H]
//       shepherd / predator / gamma terms and the velocity update (flockUtils.py:271-348)
//       (wait T, all H) copy of the workgroup's observation image to HBM (16-byte stores)
// The hand-offs are LDS counters (release/acquire at workgroup scope, LDS only); the two workgroup
// barriers are LDS-only too, so no wave ever waits for its own global stores to drain.  Auto-resets
// (rare) run after the second barrier.  The SoA state layout is shared with ch_kernels.hip.
#include <hip/hip_runtime.h>

#include <atomic>

#include "ch_common.h"
#include "ch_device.h"
#include "ch_internal.h"
#include "ch_mlp2_dev.h"   // mlp2_body (k_step2_actor)

namespace ch {

// per-env integer scalars kept in LDS (index I * G + g)
enum { I_N = 0, I_SC, I_SCA, I_HASPREV, I_LEVEL, I_TALLY, I_SPAWN, I_ACTIVE, I_EPISODE, I_FLOCK, I_RESET, I_NEWN,
       I_HERD, I_OBSD, I_COUNT };
static_assert(I_COUNT == kV2EnvInts, "LDS env-int rows");
enum { F_D = 0, F_T, F_H, F_A, F_E, F_R, F_X0, F_X1, F_X2,     // hand-off counters (F_H counts finished items)
       C_PAIRS, C_ROWS, C_COWS, C_FLOCK, C_DELTA, F_W, F_Q,      // work counters (grab), cow-wave syncs
       Q_LEN, C_QUEUE, F_C,                                       // shared alpha queue: length, grab, cheap pass done
       C_EULER,                                                   // Euler angles of the new attitudes (cow waves)
       V_DSIMD,                                                   // 1 + the SIMD the drone wave runs on
       F_S, C_SPC, C_SCAT,                                        // split: drone reward terms done on the cow waves
       F_HC,                                                      // herd centroids done (first cow wave)
       FLAG_COUNT };
static_assert(FLAG_COUNT <= kV2Flags, "LDS flag words");
// after the per-env rows: flocking-env list [G], reset-env list [G], their counts, then the counters
#define FL_LIST (I_COUNT * G)
#define RS_LIST (I_COUNT * G + G)
#define NF_AT (I_COUNT * G + 2 * G)
#define NR_AT (I_COUNT * G + 2 * G + 1)

// full unroll when the trip count is a compile-time constant (the geometry-specialised kernels): every
// LDS load of a small per-env loop is then issued up front instead of one round trip per iteration
#define CH_UNROLL _Pragma("unroll")

// index of unordered pair (i, j), i < j, in row-major upper-triangle order
__device__ __forceinline__ int tri(int i, int j, int M) { return i * M - ((i * (i + 1)) >> 1) + (j - i - 1); }

// q / d for 0 <= q < 2^22 without an integer divide
__device__ __forceinline__ int qdiv(int q, int d, float rd) {
    int r = (int)((float)q * rd);
    int rem = q - r * d;
    if (rem < 0) --r;
    else if (rem >= d) ++r;
    return r;
}

// workgroup barrier that orders LDS only (no wait for outstanding global stores)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// LDS writes of this wave visible to its other lanes
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
// Quad broadcast: lane K of every group of four lanes, to all four (DPP quad_perm: a VALU move, no LDS traffic).
// Called convergently by the whole wave.  With four drones per env the drones of an env are one quad of the drone wave.
template <int K> __device__ __forceinline__ int qb(int x) {
    return __builtin_amdgcn_update_dpp(0, x, K | (K << 2) | (K << 4) | (K << 6), 0xf, 0xf, false);
}
template <int K> __device__ __forceinline__ float qb(float x) { return __builtin_bit_cast(float, qb<K>(__builtin_bit_cast(int, x))); }
template <int K> __device__ __forceinline__ double qb(double x) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
    const int lo = qb<K>((int)(unsigned)u), hi = qb<K>((int)(unsigned)(u >> 32));
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// the four drones' values of this lane's env, in drone order
template <class T> __device__ __forceinline__ void qall(T x, T out[4]) {
    out[0] = qb<0>(x); out[1] = qb<1>(x); out[2] = qb<2>(x); out[3] = qb<3>(x);
}

// called convergently by a whole wave: its LDS writes are published, then the counter is bumped once
__device__ __forceinline__ void lds_signal(int* f) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int lds_peek(int* f) {
    return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// a hand-off that never completed: the kernel goes on (never a hang) and the handle's device error
// word records it; ch_metrics / ch_get_state / ch_sync return CH_ERR_DEVICE from then on
__device__ __forceinline__ void handoff_failed(int* err) {
    if (err && (threadIdx.x & 63) == 0) atomicOr(err, CH_DEVERR_HANDOFF);
}
// diagnostics (-DCH_COUNT_SPINS builds only, tools/spin_split.py): sleep iterations of the hand-off waits, per wave
// kind (drone wave, cow waves), and the number of waits, summed over every k_step2 launch since the last read
#ifdef CH_COUNT_SPINS
static __device__ unsigned long long g_ch_spins[4];
__device__ __forceinline__ void spin_note(int n) {
    if ((threadIdx.x & 63) == 0) {
        const int w = threadIdx.x < 64 ? 0 : 1;
        atomicAdd(&g_ch_spins[w], (unsigned long long)n);
        atomicAdd(&g_ch_spins[2 + w], 1ull);
    }
}
#else
__device__ __forceinline__ void spin_note(int) {}
#endif
// spin until *f >= target (bounded, about 0.1 s)
__device__ __forceinline__ void lds_wait(int* f, int target, int* err) {
    int spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target && ++spins < (1 << 22))
        __builtin_amdgcn_s_sleep(1);
    if (spins >= (1 << 22)) handoff_failed(err);
    spin_note(spins);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Dynamic share-out of a cow-wave loop: each call hands the calling wave the next n items of the
// counter.  The cow waves do not run at equal speed (one of them shares its SIMD with the other
// resident workgroup's prioritised drone wave), so a static lane -> item split leaves the slowest
// wave with as many items as the fastest.
__device__ __forceinline__ int grab(int* ctr, int n, bool skip = false) {
    if (skip) return 1 << 28;   // (wave-uniform) this wave takes no more items of the loop
    int b = 0;
    if ((threadIdx.x & 63) == 0) b = atomicAdd(ctr, n);
    return __builtin_amdgcn_readfirstlane(b);
}

// barrier among the cow waves only (the drone wave keeps running); `global` also publishes their
// global stores (needed before other cow lanes rewrite the same state)
__device__ __forceinline__ void cow_sync(int* f, int waves, bool global, int* err) {
    if (global) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    lds_signal(f);
    lds_wait(f, waves, err);
    if (global) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// diagnostics: per-workgroup timestamps (slots: 0/1 wall clock at start/end, 2 shader clock at start,
// 3 after the first barrier, 4 drone chain done, 5 reward terms done, 6 herded flags received,
// 7 bookkeeping done, 8 cow waves: alpha rows done, 9 drone positions received, 10 velocity update
// done, 11 obs copy done, 12 CU id, 13 second barrier, 14 end)
#define TS(slot, val) do { if (p.tstamp) p.tstamp[(long long)blockIdx.x * 128 + (slot)] = (val); } while (0)
// diagnostics: per cow wave 1..6, chunks taken and cycles spent in each dynamic loop (slots 64 + 10 (w - 1) + 2 loop)
#define CHUNK_T0 const long long ck0_ = p.tstamp ? (long long)clock64() : 0
// diagnostics: the latest of the cow waves at a point (per-workgroup max of the shader clock in slot `slot`)
#define TS_MAX(slot) do { if (p.tstamp && (threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned long long*>(p.tstamp + (long long)blockIdx.x * 128 + (slot)), (unsigned long long)clock64()); } while (0)
#define CHUNK_T1(loop) do { if (p.tstamp && (threadIdx.x & 63) == 0 && (threadIdx.x >> 6) <= 6) { long long* q_ = p.tstamp + (long long)blockIdx.x * 128 + 64 + 10 * ((threadIdx.x >> 6) - 1) + 2 * (loop); q_[0] += 1; q_[1] += (long long)clock64() - ck0_; } } while (0)

template <class R>
struct V2Smem {
    R *cx, *cy, *cvx, *cvy, *aux, *auy;              // [G*M] positions after integration, pre-flock velocities, alpha
    R *spx, *spy;                                    // [G*M] spawn positions of the next episode (prefetched)
    R *dx, *dy, *dz;                                 // [G*N] drone position after physics
    R *pa, *pb, *sa, *sb, *ca, *cb, *scat, *psp;     // [G*N] per-drone reward terms
    R* mrew;                                         // [G*N] MARL per-agent reward scratch
    R *mq, *meor;                                    // [G*N] MARL: reward without the approach term, end-of-episode bonus
    R* dq;                                           // [4][G*N] drone attitude after physics (for the Euler angles)
    R *rdx, *rdy, *rdz;                              // [G*N] auto-reset: the new episode's drone positions
    R* dcow;                                         // [G*N*M] squared cow-drone distances, (g*N + k)*M + j
    R *prev, *clock, *hcx, *hcy;                     // [G] env reals; herd centroid (cow waves)
    // f64 positions and centroid inputs (the same arrays as dx, dy, cx, cy, hcx, hcy, prev in f64 mode; f32 mode keeps
    // f64 copies beside its f32 ones: StepParams::pos64)
    double *dxd, *dyd, *cxd, *cyd, *hcxd, *hcyd, *prevd;
    R *tgx, *tgy, *tcx, *tcy;                        // [G*P] alpha pair table
    R* td;                                           // sep: [4][G*M] shepherd sums, new velocities; else [6][G*M*N] shepherd/predator terms (the pair table's space)
    int* cnt;                                        // sep: [G*M] per-cow arrivals (alpha row, shepherd sum)
    double* met;                                     // [kMetricRows*G]
    int* ei;                                         // [I_COUNT*G] + list [G] + 2 + flags
    int* flags;
    Level* LT;                                       // curriculum table (curriculum_learning.py:10-194)
    const uint16_t* pl;                              // [P] unordered cow pairs, copied from p.pairs
    uint8_t *dflags, *herded, *md1, *md2;            // [G*N], [G*M], [G*N], [G*N]
    uint8_t* tdf;                                    // [G*M*N] shepherd term in range | predator in range << 1
    uint8_t* hasnb;                                  // PW: [G] int flags, flock-list env f's alpha rows are written
    unsigned long long* nbm;                         // PW: [G*M] neighbours k whose pair is inside the bump support
    uint16_t* queue;                                 // PW: [W][P] pairs of the slot's env inside the bump support

    __device__ V2Smem(unsigned char* base, const V2Layout& L) {
        const int GM = L.G * L.M, GN = L.G * L.N, GP = (L.W ? L.W : L.G) * L.P;
        cx = (R*)(base + L.off[V2Layout::CX]); cy = cx + GM; cvx = cy + GM; cvy = cvx + GM; aux = cvy + GM; auy = aux + GM;
        spx = auy + GM; spy = spx + GM;
        dx = (R*)(base + L.off[V2Layout::DRONE]); dy = dx + GN; dz = dy + GN;
        pa = dz + GN; pb = pa + GN; sa = pb + GN; sb = sa + GN; ca = sb + GN; cb = ca + GN; scat = cb + GN;
        psp = scat + GN; mrew = psp + GN; mq = mrew + GN; meor = mq + GN; dq = meor + GN;
        rdx = dq + 4 * GN; rdy = rdx + GN; rdz = rdy + GN;
        dcow = (R*)(base + L.off[V2Layout::DCOW]);
        prev = (R*)(base + L.off[V2Layout::ENVR]); clock = prev + L.G; hcx = clock + L.G; hcy = hcx + L.G;
        if constexpr (sizeof(R) == 8) {
            dxd = (double*)dx; dyd = (double*)dy; cxd = (double*)cx; cyd = (double*)cy;
            hcxd = (double*)hcx; hcyd = (double*)hcy; prevd = (double*)prev;
        } else {
            dxd = (double*)(base + L.off[V2Layout::XD]); dyd = dxd + GN; cxd = dyd + GN; cyd = cxd + GM;
            hcxd = cyd + GM; hcyd = hcxd + L.G; prevd = hcyd + L.G;
        }
        pl = (const uint16_t*)(base + L.off[V2Layout::PAIRL]);
        tgx = (R*)(base + L.off[V2Layout::PAIRS]); tgy = tgx + GP; tcx = tgy + GP; tcy = tcx + GP;
        td = L.sep ? (R*)(base + L.off[V2Layout::TD]) : tgx;
        cnt = (int*)(base + L.off[V2Layout::TD] + 4 * (size_t)L.G * L.M * sizeof(R));
        met = (double*)(base + L.off[V2Layout::MET]);
        ei = (int*)(base + L.off[V2Layout::EI]);
        flags = ei + I_COUNT * L.G + 2 * L.G + 2;
        LT = (Level*)(base + L.off[V2Layout::LEVELS]);
        unsigned char* bytes = base + L.off[V2Layout::BYTES];
        nbm = reinterpret_cast<unsigned long long*>(bytes);   // BYTES is 16-byte aligned
        hasnb = bytes + 8 * GM;
        const int GMa = (GM + 15) & ~15;
        queue = reinterpret_cast<uint16_t*>(hasnb + GMa);
        dflags = hasnb + GMa + 2 * GP;
        herded = dflags + GN; md1 = herded + GM;
        md2 = md1 + GN; tdf = md2 + GN;
    }
};

// Observation blocks are written straight to HBM by the lanes that produce each entry (BaseRLAviary.py:
// 272-342 / BaseMARLAviary.py:253-303): own state (drone wave, after the chain), two nearest drones
// (drone wave, after the reward terms), cattle offsets (cow waves, after the distance table), and the
// always-zero bytes (cow waves, during the alpha phase).  `eb` is the env's block (row 0, col 0); 86 is
// even, so every float2 below is 8-byte aligned.
#if !defined(CH_NT_STORES) && !defined(CH_NO_NT_STORES)
// Write-through stores (an agent-scope relaxed atomic store is a global_store ... sc1): the lines leave the
// XCD's L2 while the kernel runs instead of in the kernel-end write-back, which the next launch waits for.
// Measured at C4 (tools/gpu_ab_store.sh): inter-kernel gap 2.6 -> 1.75 us, 164 -> 171 M env-steps/s;
// non-temporal (nt, CH_NT_STORES) and plain stores both leave the lines dirty in L2.  Used for the outputs
// (observations, rewards); the state uses CH_STS below.
template <class T> __device__ __forceinline__ void ch_st_wt(T* ptr, T v) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "4- or 8-byte stores");
    if constexpr (sizeof(T) == 8)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(ptr), __builtin_bit_cast(unsigned long long, v),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        __hip_atomic_store(reinterpret_cast<unsigned*>(ptr), __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
#define CH_ST(ptr, val) ch_st_wt((ptr), static_cast<std::remove_pointer_t<decltype(ptr)>>(val))
#elif defined(CH_NT_STORES)
#define CH_ST(ptr, val) __builtin_nontemporal_store((val), (ptr))
#else
#define CH_ST(ptr, val) (*(ptr) = (val))
#endif
// State the next step reads back (drones, cattle, env scalars, metrics, Euler cache) stays in the XCD's L2
// (nt): the next launch's first loads then hit L2 instead of MALL.  Same box, same build otherwise
// (tools/gpu_ab_store.sh, profiles/r02/ab/): state nt + outputs write-through 161.7 M/s (span 23.5 us, gap
// 2.3 us) vs everything write-through 158.8 M/s (24.2, 1.7).  CH_STATE_WT / CH_STATE_PLAIN for the A/B.
#if defined(CH_STATE_WT)
#define CH_STS(ptr, val) CH_ST(ptr, val)
#elif defined(CH_STATE_PLAIN)
#define CH_STS(ptr, val) (*(ptr) = (val))
#else
#define CH_STS(ptr, val) __builtin_nontemporal_store(static_cast<std::remove_pointer_t<decltype(ptr)>>(val), (ptr))
#endif
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st2(float* eb, int off, float a, float b) {
    f2v v = {a, b};
    CH_ST(reinterpret_cast<f2v*>(eb + off), v);
}

// own-state entries of row `row` (BaseRLAviary.py:289-295)
template <class R>
__device__ __forceinline__ void obs_own(float* eb, int row, R z, const R rpy[3], const R v[3], const R w[3]) {
    const int o = row * 86;
    st2(eb, o + 0, (float)z, (float)rpy[0]);
    st2(eb, o + 2, (float)rpy[1], (float)rpy[2]);
    st2(eb, o + 4, (float)v[0], (float)v[1]);
    st2(eb, o + 6, (float)v[2], (float)w[0]);
    st2(eb, o + 8, (float)w[1], (float)w[2]);
}

// the own-state row but its Euler angles (drone wave), and the Euler angles (cow waves, from the published
// attitude): the same entries obs_own writes
template <class R>
__device__ __forceinline__ void obs_own_nrpy(float* eb, int row, R z, const R v[3], const R w[3]) {
    const int o = row * 86;
    CH_ST(eb + o, (float)z);
    st2(eb, o + 4, (float)v[0], (float)v[1]);
    st2(eb, o + 6, (float)v[2], (float)w[0]);
    st2(eb, o + 8, (float)w[1], (float)w[2]);
}
template <class R>
__device__ __forceinline__ void obs_rpy(float* eb, int row, const R rpy[3]) {
    const int o = row * 86;
    CH_ST(eb + o + 1, (float)rpy[0]);
    st2(eb, o + 2, (float)rpy[1], (float)rpy[2]);
}

// nearest-neighbour entries (columns 10..13) of drone i from its two nearest drones i1, i2
template <class R>
__device__ __forceinline__ void obs_nbr(float* eb, const R* dx, const R* dy, int b0, int i, int i1, int i2) {
    const R xi = dx[b0 + i], yi = dy[b0 + i];
    const int o = i * 86 + 10;
    if (i1 >= 0) st2(eb, o, (float)(dx[b0 + i1] - xi), (float)(dy[b0 + i1] - yi)); else st2(eb, o, 0.0f, 0.0f);
    if (i2 >= 0) st2(eb, o + 2, (float)(dx[b0 + i2] - xi), (float)(dy[b0 + i2] - yi)); else st2(eb, o + 2, 0.0f, 0.0f);
}

// cattle-relative entries of cow j for every live drone row (BaseRLAviary.py:319-331)
template <class A, class Q>
__device__ __forceinline__ void obs_cattle(float* eb, const A* dx, const A* dy, int b0, int j, int n, int cat_off, Q qx,
                                           Q qy) {
    for (int r = 0; r < n; ++r) st2(eb, r * 86 + cat_off + 2 * j, (float)(qx - dx[b0 + r]), (float)(qy - dy[b0 + r]));
}

// The bytes of an env block no producer writes this step: rows n..rows-1 in full, and in the live rows
// columns 14..cat_off-1 and cat_off+2*m_obs..85 (the always-zero action-buffer block and padding).
// Lane t of the team covers float2 t, t + stride, ... of the block (consecutive lanes, consecutive
// addresses); float2 u sits at row u / 43, column 2 * (u % 43).
__device__ __forceinline__ void obs_zero_env(float* eb, int n, int rows, int cat_off, int m_obs, int t0, int stride) {
    for (int u = t0; u < rows * 43; u += stride) {
        const int r = u / 43, c = 2 * (u - 43 * r);
        if (r >= n || (c >= 14 && c < cat_off) || c >= cat_off + 2 * m_obs) st2(eb, 2 * u, 0.0f, 0.0f);
    }
}

// two nearest drones of drone i in the reference's stable order (BaseRLAviary.py:303-317), packed as
// (i1 + 1) | (i2 + 1) << 8 (0 = none); returned by value so nothing lands in scratch
template <class R>
__device__ __forceinline__ int nearest_two(const R* dx, const R* dy, int b0, int i, int n) {
    const R xi = dx[b0 + i], yi = dy[b0 + i];
    R b1 = 0, b2 = 0;
    int i1 = -1, i2 = -1;
    for (int j = 0; j < n; ++j) {
        if (j == i) continue;
        const R d = norm2(dx[b0 + j] - xi, dy[b0 + j] - yi);
        if (i1 < 0 || d < b1) { i2 = i1; b2 = b1; i1 = j; b1 = d; }
        else if (i2 < 0 || d < b2) { i2 = j; b2 = d; }
    }
    return (i1 + 1) | ((i2 + 1) << 8);
}

// spacing reward terms of drone slot u from its two nearest-neighbour distances (CattleAviary.py:230-246,
// 572-679): simple and complex spacing of both, and the drone's spacing reward
template <class R>
__device__ __forceinline__ void spacing_terms_r(const Level& Lv, bool compat, R m1, R m2, R& sa, R& sb, R& ca, R& cb,
                                                R& ps) {
    sa = simple_spacing(m1, Lv); sb = simple_spacing(m2, Lv);
    ca = complex_spacing(m1, Lv); cb = complex_spacing(m2, Lv);
    ps = 0;   // per-drone spacing reward (CattleAviary.py:238-246)
    if (compat || m1 < R(INFINITY)) ps += (ca + sa) / R(2.0);
    if (compat || m2 < R(INFINITY)) ps += (cb + sb) / R(2.0);
}
template <class R>
__device__ __forceinline__ void spacing_terms(V2Smem<R>& S, const Level& Lv, bool compat, int u, R m1, R m2) {
    R sa, sb, ca, cb, ps;
    spacing_terms_r(Lv, compat, m1, m2, sa, sb, ca, cb, ps);
    S.sa[u] = sa; S.sb[u] = sb; S.ca[u] = ca; S.cb[u] = cb; S.psp[u] = ps;
}

// closest cow of drone slot u (CattleAviary.py:248-252) from the cow waves' distance table -> cattle term:
// min over cows of |y - q|^2, then one square root (sqrt is correctly rounded and monotonic, so this is
// the minimum of the distances; a NaN entry is skipped either way)
template <class R>
__device__ __forceinline__ R cattle_term(const V2Smem<R>& S, int u, int M, R cc) {
    const R* dc = S.dcow + u * M;
    R best = R(INFINITY);
    for (int j = 0; j < M; ++j) {
        const R d = dc[j];
        if (d < best) best = d;
    }
    return cattle_spacing(sqrt(best), cc);
}

// flock alpha term, pair form, for every flocking env (flockUtils.py:237-258, 327-337; MathUtils 11-58):
// one table of the workgroup's unordered cow pairs, evaluated in the bump's support only.  The bump is
// exactly 0 for sigma_norm(|z|) / r_alpha > 1 (beyond the lattice range d_alpha = 1.2 m); such a pair adds
// +-0 to both rows, which leaves a row sum that starts at +0 unchanged.  A cheap pass over every pair (no
// square root) marks the pairs with |z|^2 <= 1.44 (1 + 1e-9) -- a superset of the support, see
// kAlphaSupport2 -- in both cows' neighbour masks and appends them to a queue; the full evaluation runs on
// full waves of queued pairs; the rows visit the masked neighbours in ascending order like the dense loop.
constexpr double kAlphaSupport2 = 1.44 * (1.0 + 1e-9);

// |z| <= 999 (the sensing range) from |z|^2 without the square root away from the boundary: sqrt is
// correctly rounded and monotonic, and sqrt(998001) = 999 exactly
template <class R> __device__ __forceinline__ bool in_sensing(R n2) {
    bool s = n2 <= R(998001.0);
    if (!s && n2 < R(998010.0)) s = sqrt(n2) <= R(999);
    return s;
}

// Cow j of env g has another cow of its env within sensing range (flockUtils.py:237-258: the alpha sums run over the
// neighbours inside r = 999 m; with none, its alpha term is 0).  One partner decides it almost always -- the next cow --
// and only a cow out of that one's range scans the rest, with the pair's difference taken in the pair list's order
// (the same n2 as the cheap pass).  Evaluated by the row instead of marked by the cheap pass: those byte stores (many
// lanes of a pass chunk on the same cow) took ~40 % of the pass (tools/wg_trace.py, profiles/r04/zc).
template <class R>
__device__ __forceinline__ bool has_sensing_neighbour(const V2Smem<R>& S, int M, int g, int j) {
    auto ins = [&](int k) {
        const int lo = g * M + min(j, k), hi = g * M + max(j, k);
        const R zx = S.cx[hi] - S.cx[lo], zy = S.cy[hi] - S.cy[lo];
        return in_sensing(zx * zx + zy * zy);
    };
    bool has = M > 1 && ins(j + 1 < M ? j + 1 : 0);
    if (!has)
        for (int k = 0; k < M; ++k)
            if (k != j && ins(k)) { has = true; break; }
    return has;
}

template <class R>
__device__ __forceinline__ void alpha_cheap(V2Smem<R>& S, int* fl, int M, int P, int nf, const int* flist, bool skip) {
    const float rP = 1.0f / (float)P;
    const int lane = threadIdx.x & 63;
    for (;;) {
        const int b = grab(fl + C_PAIRS, 64, skip);
        if (b >= nf * P) break;
        const int q = b + lane;
        bool cand = false;
        int gi = 0;
        if (q < nf * P) {
            const int f = qdiv(q, P, rP), r = q - f * P, g = flist[f];
            const uint32_t pr = S.pl[r];
            const int li = pr & 0xff, hi = pr >> 8;
            const int bi = g * M + li, bj = g * M + hi;
            const R zx = S.cx[bj] - S.cx[bi], zy = S.cy[bj] - S.cy[bi];
            const R n2 = zx * zx + zy * zy;
            cand = n2 <= R(kAlphaSupport2);
            if (cand) {
                atomicOr(&S.nbm[bi], 1ull << hi);
                atomicOr(&S.nbm[bj], 1ull << li);
            }
            gi = g * P + r;
        }
        const unsigned long long m = __ballot(cand);
        int base = 0;
        if (lane == 0 && m) base = atomicAdd(fl + Q_LEN, (int)__popcll(m));
        base = __builtin_amdgcn_readfirstlane(base);
        if (cand) S.queue[base + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)gi;
    }
}

// The full evaluation of the queued pairs.  Streamed (default; CH_NO_STREAM_FULL for the barrier form): a wave
// that runs out of cheap-pass chunks starts on the queue at once instead of waiting at a pass-wide barrier for
// the other waves' last cheap chunks.  Every queue slot starts as kQEmpty (phase 0); a chunk of 64 slots is taken
// when all of them are reserved (Q_LEN) or the cheap pass is complete (F_C counts the waves done with it, so
// Q_LEN is then final), and each lane waits for its own slot's pair index to be written -- a per-slot ready mark.
constexpr uint16_t kQEmpty = 0xFFFF;
template <class R>
__device__ __forceinline__ void alpha_full(V2Smem<R>& S, int* fl, int M, int P, bool skip, int W1, int* err) {
    const R ra = sigma_norm_n(R(1.2)), da = ra;
    const float rP = 1.0f / (float)P;
    const int lane = threadIdx.x & 63;
#ifdef CH_NO_STREAM_FULL
    (void)W1; (void)err;
    const int qn = lds_peek(fl + Q_LEN);   // final: every cow wave's cheap pass is done (F_C)
#endif
    for (;;) {
        const int b = grab(fl + C_QUEUE, 64, skip);
#ifndef CH_NO_STREAM_FULL
        if (b >= (1 << 28)) break;   // (skip)
        int qn = 0;
        bool done = false;
        int spins = 0;
        for (;; ++spins) {
            done = lds_peek(fl + F_C) >= W1;      // F_C before Q_LEN: once every wave is done, Q_LEN is final
            qn = lds_peek(fl + Q_LEN);
            if (done || qn >= b + 64) break;
            if (spins >= (1 << 22)) { handoff_failed(err); done = true; break; }
            __builtin_amdgcn_s_sleep(1);
        }
        spin_note(spins);
        if (b >= qn) break;   // done: no slot of this chunk was ever reserved
#else
        if (b >= qn) break;
#endif
        if (b + lane < qn) {
#ifndef CH_NO_STREAM_FULL
            int gi = kQEmpty;
            for (int spins = 0; spins < (1 << 22); ++spins) {
                gi = *reinterpret_cast<volatile const uint16_t*>(&S.queue[b + lane]);
                if (gi != kQEmpty) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (gi == kQEmpty) { handoff_failed(err); gi = 0; }
#else
            const int gi = S.queue[b + lane];
#endif
            const int g = qdiv(gi, P, rP), r = gi - g * P;
            const uint32_t pr = S.pl[r];
            const int bi = g * M + (pr & 0xff), bj = g * M + (pr >> 8);
            const R zx = S.cx[bj] - S.cx[bi], zy = S.cy[bj] - S.cy[bi];
            const R nrm = sqrt(zx * zx + zy * zy);
            R gx = 0, gy = 0, cx = 0, cy = 0;
            pair_terms_n(nrm, zx, zy, S.cvx[bi], S.cvy[bi], S.cvx[bj], S.cvy[bj], ra, da, gx, gy, cx, cy);
            S.tgx[gi] = gx; S.tgy[gi] = gy; S.tcx[gi] = cx; S.tcy[gi] = cy;
        }
    }
}

// alpha row of cow u = g*M + j in neighbour order over its masked neighbours, scaled by c2_alpha
// (flockUtils.py:237-258); the two directed contributions of a pair are exact negations
template <class R>
__device__ __forceinline__ void alpha_row(V2Smem<R>& S, int M, int P, int u, int g, int j) {
    const R C2A = R(2 * 1.7320508075688772);
    R gx = 0, gy = 0, cxx = 0, cyy = 0, ux = 0, uy = 0;
    const int pb = g * P;
    // Four neighbours per round, branch-free: the table loads of a round are issued together (an empty slot
    // reads the env's first pair), then summed in neighbour order.  An empty slot adds +0, which leaves the
    // sum unchanged: it starts at +0 and a round-to-nearest sum is -0 only if both addends are.
    for (unsigned long long m = S.nbm[u]; m;) {
        R t[4][4];
        bool v[4], fwd[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            v[r] = m != 0;
            const int k = __ffsll((long long)m) - 1;
            m &= m - 1;
            fwd[r] = j < k;
            const int idx = v[r] ? pb + tri(min(j, k), max(j, k), M) : pb;
            t[r][0] = S.tgx[idx]; t[r][1] = S.tgy[idx]; t[r][2] = S.tcx[idx]; t[r][3] = S.tcy[idx];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            gx += v[r] ? (fwd[r] ? t[r][0] : -t[r][0]) : R(0); gy += v[r] ? (fwd[r] ? t[r][1] : -t[r][1]) : R(0);
            cxx += v[r] ? (fwd[r] ? t[r][2] : -t[r][2]) : R(0); cyy += v[r] ? (fwd[r] ? t[r][3] : -t[r][3]) : R(0);
        }
    }
    if (has_sensing_neighbour(S, M, g, j)) { ux = C2A * gx + C2A * cxx; uy = C2A * gy + C2A * cyy; }
    S.aux[u] = ux; S.auy[u] = uy;
}

// ---- per-wave env tables (V2Layout W > 0, large herds) ---------------------------------------------
// Env g's alpha pair table in the calling wave's slot: gradient x, y and the bump b per pair
// (flockUtils.py:237-258, 327-337).  The consensus term b (p_hi - p_lo) is not stored: alpha_row_pw
// recomputes it from the velocities with the same rounding.
//
// Sparse in the bump's support.  The bump is exactly 0 for sigma_norm(|z|) / r_alpha > 1, i.e. beyond
// the lattice range d_alpha = 1.2 m, and such a pair adds +-0 to both rows, which leaves a row sum that
// starts at +0 unchanged.  A cheap pass over all pairs (no square root) queues the pairs with
// |z|^2 <= 1.44 (1 + 1e-9) -- a superset of the support: any pair beyond it has z > 1 + 5e-10 exactly and
// z > 1 as computed -- and marks them in both cows' neighbour masks; the full evaluation (square roots,
// the bump's cos, sigma_1, divisions) runs on full waves of queued pairs only, and the rows visit only
// masked neighbours, in ascending neighbour order like the dense loop.
template <class R>
__device__ __forceinline__ void alpha_cheap_pw(V2Smem<R>& S, int M, int P, int g, uint16_t* qu, int& qn) {
    const int lane = threadIdx.x & 63;
    for (int r0 = 0; r0 < P; r0 += 64) {
        const int r = r0 + lane;
        bool cand = false;
        if (r < P) {
            const uint32_t pr = S.pl[r];
            const int li = pr & 0xff, hi = pr >> 8;
            const int bi = g * M + li, bj = g * M + hi;
            const R zx = S.cx[bj] - S.cx[bi], zy = S.cy[bj] - S.cy[bi];
            const R n2 = zx * zx + zy * zy;
            cand = n2 <= R(kAlphaSupport2);
            if (cand) {
                atomicOr(&S.nbm[bi], 1ull << hi);
                atomicOr(&S.nbm[bj], 1ull << li);
            }
        }
        const unsigned long long m = __ballot(cand);
        if (cand) qu[qn + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)r;
        qn += __popcll(m);
    }
}

// The same pass for a geometry-specialised herd (NC = the pass's 64-pair chunks, a compile-time count): the lane's
// pair words come from registers (prw, read from LDS once per kernel) and every chunk's position loads are issued
// before any chunk's test, so the pass costs about one LDS round trip instead of one per chunk.  The queue and
// masks are filled in the same (chunk, lane) order as alpha_cheap_pw.
template <class R, int NC>
__device__ __forceinline__ void alpha_cheap_pw_b(V2Smem<R>& S, int M, int P, int g, uint16_t* qu, int& qn,
                                                 const uint32_t (&prw)[NC]) {
    const int lane = threadIdx.x & 63;
    R n2[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t pr = prw[c];
        const int bi = g * M + (pr & 0xff), bj = g * M + (pr >> 8);
        const R zx = S.cx[bj] - S.cx[bi], zy = S.cy[bj] - S.cy[bi];
        n2[c] = zx * zx + zy * zy;
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int r = 64 * c + lane;
        bool cand = false;
        if (r < P) {
            const uint32_t pr = prw[c];
            const int li = pr & 0xff, hi = pr >> 8;
            const int bi = g * M + li, bj = g * M + hi;
            cand = n2[c] <= R(kAlphaSupport2);
            if (cand) {
                atomicOr(&S.nbm[bi], 1ull << hi);
                atomicOr(&S.nbm[bj], 1ull << li);
            }
        }
        const unsigned long long m = __ballot(cand);
        if (cand) qu[qn + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)r;
        qn += __popcll(m);
    }
}

template <class R>
__device__ __forceinline__ void alpha_full_pw(V2Smem<R>& S, int M, int P, int g, int q0, int qn, R* tb,
                                              const uint16_t* qu) {
    const R ra = sigma_norm_n(R(1.2)), da = ra;
    const int q = q0 + (threadIdx.x & 63);
    if (q >= qn) return;
    const int r = qu[q];
    const uint32_t pr = S.pl[r];
    const int bi = g * M + (pr & 0xff), bj = g * M + (pr >> 8);
    const R zx = S.cx[bj] - S.cx[bi], zy = S.cy[bj] - S.cy[bi];
    const R nrm = sqrt(zx * zx + zy * zy);
    R gx = 0, gy = 0, cx = 0, cy = 0;
    const R b = pair_terms_n(nrm, zx, zy, R(0), R(0), R(0), R(0), ra, da, gx, gy, cx, cy);
    tb[r] = gx; tb[P + r] = gy; tb[2 * P + r] = b;
}

// alpha row of cow j of env g from the wave's slot, in neighbour order (as alpha_row), visiting the
// masked neighbours only.  The pair's consensus term is b * (p_hi - p_lo), hi/lo the pair's cows,
// exactly as the shared table holds it.
template <class R>
__device__ __forceinline__ void alpha_row_pw(V2Smem<R>& S, int M, int P, int g, int j, const R* tb) {
    const R C2A = R(2 * 1.7320508075688772);
    const int u = g * M + j;
    R gx = 0, gy = 0, cxx = 0, cyy = 0, ux = 0, uy = 0;
    const R pjx = S.cvx[u], pjy = S.cvy[u];
    // four neighbours per round, branch-free as in alpha_row (an empty slot reads pair 0 / cow j, adds +0)
    for (unsigned long long m = S.nbm[u]; m;) {
        R t[4][5];
        bool v[4], fwd[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            v[r] = m != 0;
            const int k = v[r] ? __ffsll((long long)m) - 1 : j;
            m &= m - 1;
            fwd[r] = j < k;
            const int idx = v[r] ? tri(min(j, k), max(j, k), M) : 0;
            t[r][0] = tb[idx]; t[r][1] = tb[P + idx]; t[r][2] = tb[2 * P + idx];
            t[r][3] = S.cvx[g * M + k]; t[r][4] = S.cvy[g * M + k];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const R b = t[r][2], pkx = t[r][3], pky = t[r][4];
            const R dvx = fwd[r] ? pkx - pjx : pjx - pkx, dvy = fwd[r] ? pky - pjy : pjy - pky;
            const R tcx = b * dvx, tcy = b * dvy;
            gx += v[r] ? (fwd[r] ? t[r][0] : -t[r][0]) : R(0); gy += v[r] ? (fwd[r] ? t[r][1] : -t[r][1]) : R(0);
            cxx += v[r] ? (fwd[r] ? tcx : -tcx) : R(0); cyy += v[r] ? (fwd[r] ? tcy : -tcy) : R(0);
        }
    }
    if (has_sensing_neighbour(S, M, g, j)) { ux = C2A * gx + C2A * cxx; uy = C2A * gy + C2A * cyy; }
    S.aux[u] = ux; S.auy[u] = uy;
}

// the shepherd term of a drone closer than 1 m (mu < 1: the projected agent q_ik lies between cow and drone),
// the general pair_terms evaluation.  Rare, so it is kept out of line: inlined at each of the unrolled drone
// slots of shepherd_sum it would add ~1.2k instructions to the kernel's instruction-cache footprint.
template <class R> struct Terms4 { R gx, gy, cx, cy; };
template <class R>
__device__ __noinline__ Terms4<R> near_drone_terms(R qix, R qiy, R pix, R piy, R yx, R yy, R mu, R pkx, R pky) {
    const R ra_b = sigma_norm_n(R(1.0)), da_b = ra_b;
    R qkx = mu * qix + (R(1) - mu) * yx, qky = mu * qiy + (R(1) - mu) * yy;
    Terms4<R> t = {0, 0, 0, 0};
    pair_terms(qix, qiy, pix, piy, qkx, qky, pkx, pky, ra_b, da_b, t.gx, t.gy, t.cx, t.cy);
    return t;
}

// shepherd (delta, flockUtils.py:271-317) and predator (343-348) terms of drone k on cow u = g*M + j:
// t[0..3] the delta gradient and consensus parts, t[4..5] the predator push; returns in-range | predator << 1
template <class R>
__device__ __forceinline__ int delta_vals(const V2Smem<R>& S, int N, int u, int g, int k, R t[6]) {
    const R qix = S.cx[u], qiy = S.cy[u], pix = S.cvx[u], piy = S.cvy[u];
    const R yx = S.dx[g * N + k], yy = S.dy[g * N + k];
    const R ex = yx - qix, ey = yy - qiy;
    const R dn = sqrt(ex * ex + ey * ey);   // = the distance table entry
    const bool in = dn <= R(999 + 2), pr = dn <= R(1.1);
#pragma unroll
    for (int c = 0; c < 6; ++c) t[c] = 0;
    if (in) {
        R difx = qix - yx, dify = qiy - yy;
        R d = dn + R(1e-6);
        R mu = d / R(1.0) < R(1.0) ? d / R(1.0) : R(1.0);
        R akx = difx / d, aky = dify / d;
        R P00 = R(1) - akx * akx, P01 = R(0) - akx * aky, P10 = R(0) - aky * akx, P11 = R(1) - aky * aky;
        R pkx = mu * (P00 * pix + P01 * piy), pky = mu * (P10 * pix + P11 * piy);
        if (mu == R(1) && isfinite(yx) && isfinite(yy) && isfinite(qix) && isfinite(qiy)) {
            // a drone 1 m away or more: q_ik = 1 q_i + 0 y_k = q_i exactly, so pair_terms sees z = +0:
            // |z| = 0, den = 1, sigma_norm = 0, bump(0) = 1, gradient ph * (0 / 1) = +-0 (+0 in the table),
            // consensus 1 * (p_ik - p_i) -- the same values without the square roots and divisions
            t[2] = pkx - pix;
            t[3] = pky - piy;
        } else {
            const Terms4<R> n4 = near_drone_terms(qix, qiy, pix, piy, yx, yy, mu, pkx, pky);
            t[0] = n4.gx; t[1] = n4.gy; t[2] = n4.cx; t[3] = n4.cy;
        }
    }
    if (pr) {
        R d3 = cube(dn);
        t[4] = R(-650000.0) * ex / d3;
        t[5] = R(-650000.0) * ey / d3;
    }
    return (int)in | ((int)pr << 1);
}

// the same terms, one (cow, drone) item per lane, stored in the term table for flock_combine
template <class R>
__device__ __forceinline__ void delta_term(V2Smem<R>& S, int N, int u, int g, int k, R* td, uint8_t* tdf, int i,
                                           int T) {
    R t[6];
    const int f = delta_vals(S, N, u, g, k, t);
#pragma unroll
    for (int c = 0; c < 6; ++c) td[c * T + i] = t[c];
    tdf[i] = (uint8_t)f;
}

// the shepherd/predator sum of cow u over its env's n live drones in drone order (flockUtils.py:271-348),
// one cow per lane with the drone terms in registers: delta = c2_beta (sum grad + sum consensus) over the
// drones in range, plus the predator pushes.  A term out of range is +0, which leaves a sum that starts at
// +0 unchanged (the same sums flock_combine forms from the term table).
template <class R, int NT>
__device__ __forceinline__ void shepherd_sum(const V2Smem<R>& S, int N, int u, int g, int n, R& ddx, R& ddy) {
    const R C2B = R(2 * 4.47213595499958);
    R gx = 0, gy = 0, cxx = 0, cyy = 0, sx = 0, sy = 0;
    int nb = 0;
    constexpr int NK = NT ? NT : 64;
    CH_UNROLL for (int k = 0; k < NK; ++k) {
        if (k >= N || k >= n) break;
        R t[6];
        const int f = delta_vals(S, N, u, g, k, t);
        if (f & 1) { ++nb; gx += t[0]; gy += t[1]; cxx += t[2]; cyy += t[3]; }
        if (f & 2) { sx += t[4]; sy += t[5]; }
    }
    ddx = 0; ddy = 0;
    if (nb > 0) { ddx = C2B * gx + C2B * cxx; ddy = C2B * gy + C2B * cyy; }
    ddx += sx; ddy += sy;
}

// gamma term (flockUtils.py:150-160, 340-341) and the velocity update with the speed clip
// (BaseAviary.py:1384-1400) of cow u from its alpha row (aux, auy) and shepherd sum (ddx, ddy)
// nv != nullptr: the new velocity goes to LDS (nv[u], nv[GM + u]) instead of HBM
template <class R>
__device__ __forceinline__ void velocity_update(const StepParams<R>& p, const V2Smem<R>& S, int M, int e0, int u, R ddx,
                                                R ddy, R* nv = nullptr, int GM = 0) {
    const long long CS = (long long)p.E * M;
    const R C1G = R(5), C2G = R(0.2 * 2.23606797749979);
    const R qix = S.cx[u], qiy = S.cy[u], pix = S.cvx[u], piy = S.cvy[u];
    R gmx = -C1G * sigma_1(qix - R(1)) - C2G * pix, gmy = -C1G * sigma_1(qiy - R(1)) - C2G * piy;
    R qx = (S.aux[u] + ddx) + gmx, qy = (S.auy[u] + ddy) + gmy;
    const R dt_sqr = R(0.05 * 0.05);
    R vx = pix + qx * dt_sqr, vy = piy + qy * dt_sqr;
    R sp = norm2(vx, vy);
    if (sp > R(kMaxVelCattle)) { R f = R(kMaxVelCattle) / sp; vx *= f; vy *= f; }
    if (nv) { nv[u] = vx; nv[GM + u] = vy; return; }
    const long long ci = (long long)e0 * M + u;
    CH_STS(&p.cattle[2 * CS + ci], vx); CH_STS(&p.cattle[3 * CS + ci], vy);
}

// the drone terms of cow u from the term table summed in drone order, then the velocity update.  A term
// out of range is +0 in the table, and adding +0 to a sum that starts at +0 leaves it unchanged, so only
// the count needs the flag.
template <class R>
__device__ __forceinline__ void flock_combine(const StepParams<R>& p, V2Smem<R>& S, int N, int M, int e0, int u, int n,
                                              const R* td, const uint8_t* tdf, int ib, int T) {
    const R C2B = R(2 * 4.47213595499958);
    R ddx = 0, ddy = 0, sx = 0, sy = 0, gx = 0, gy = 0, cxx = 0, cyy = 0;
    int nb = 0;
    CH_UNROLL for (int k = 0; k < N; ++k) {
        if (k >= n) break;
        const int i = ib + k;
        const int f = tdf[i];
        if (f & 1) { ++nb; gx += td[i]; gy += td[T + i]; cxx += td[2 * T + i]; cyy += td[3 * T + i]; }
        if (f & 2) { sx += td[4 * T + i]; sy += td[5 * T + i]; }
    }
    if (nb > 0) { ddx = C2B * gx + C2B * cxx; ddy = C2B * gy + C2B * cyy; }
    ddx += sx; ddy += sy;
    velocity_update(p, S, M, e0, u, ddx, ddy);
}

// GT/NT/MT > 0 specialise the kernel for one geometry (envs per workgroup, drones, cattle): the LDS
// carve and all index arithmetic then fold to immediates, which keeps the kernel within the SGPR file.
// TOBS: the instantiation that writes terminal observations from their producers in the fast path (configs[3]'s
// geometry, launched when the step asks for them); without it the same geometry takes the drained-copy path for them
// The f32 geometry-specialised kernels keep 4 waves per SIMD (<= 128 VGPRs): their f64 torque path (ch_device.h
// drone_substep) would otherwise take them to 135 and 3 waves, one resident workgroup fewer per CU at large E.
// salt: 0.  k_step2_multi passes an opaque 0 per step (an empty asm's output), so that the values derived from the
// thread / workgroup indices and the LDS carve are computed inside each step instead of being hoisted out of its step
// loop and held across it (which overflowed the registers); k_step2's constant 0 folds away.
template <class R, int MODE, int GT, int NT, int MT, bool PHYS, bool PW, bool TOBS>
__device__ __forceinline__ void step2_body(const StepParams<R>& p, int salt = 0) {
    extern __shared__ __align__(16) unsigned char smem_[];
    unsigned char* const smem = smem_ + salt;
    constexpr bool marl = MODE == 1;
    // f32 mode: positions, centroids and the approach delta in f64 (StepParams::pos64); PT = their type
    constexpr bool MIX = sizeof(R) == 4;
    using PT = double;
    // SPLIT (opt-in, CH_SPLIT; the CTDE 16-env x 4-drone geometry): the drones' spacing and cattle reward terms
    // run on the cow waves, next to the drone wave's bookkeeping instead of before it; the reward waits for
    // them (F_S).  The drone wave then ends ~3k cycles earlier, but the cow waves, already the busier side after
    // the drone hand-off, end later: C4 168.3 vs 178.5 M env-steps/s without it (tools/gpu_ab.sh, ab4).
#ifdef CH_SPLIT
    constexpr bool SPLIT = !marl && GT == 16 && NT == 4;
#else
    constexpr bool SPLIT = false;
#endif
    // QUAD (the CTDE 16-env x 4-drone geometry): the per-env bookkeeping -- centroids, _computeTerminated /
    // _computeTruncated, the reset decision, the reward's per-drone sums, metrics and the env write-back -- runs on the
    // drone wave's quads (env g = lanes 4g..4g+3, the env's drones) with the per-drone terms in registers and
    // gathered by DPP quad broadcasts in drone order, instead of on 16 env lanes reading them back from LDS.
    // CH_NO_QUAD for the env-lane form.
    // PW_READY (per-wave tables): per-env ready flags between the alpha rows and the shepherd / velocity pass instead of
    // a cow-wave barrier (CH_NO_PW_READY for the barrier)
#ifdef CH_NO_PW_READY
    constexpr bool PW_READY = false;
#else
    constexpr bool PW_READY = PW;
#endif
#ifdef CH_NO_QUAD
    constexpr bool QUAD = false;
#else
    constexpr bool QUAD = !marl && GT == 16 && NT == 4 && !SPLIT;
#endif
    const int G = GT ? GT : p.G, N = NT ? NT : p.NC, M = MT ? MT : p.M, P = MT ? MT * (MT - 1) / 2 : p.P;
    const int rows = marl ? N : 12;
    const V2Layout L(G, N, M, P, MODE, (int)sizeof(R), PW ? (int)(blockDim.x >> 6) - 1 : 0, !PW && p.sep);
    const bool sep = L.sep;
    V2Smem<R> S(smem, L);
    const int BS = blockDim.x + salt, tid = threadIdx.x + salt;
    const int e0 = (blockIdx.x + salt) * G;
    const int Gv = min(G, p.E - e0);
    const long long E = p.E, DS = E * N, CS = E * M;
    const int m_obs = M < 16 ? M : 16, cat_off = marl ? 18 : 34, RW = rows * 86;
    const bool task = !(p.phase_mask & 4);
    const int W1 = (BS >> 6) - 1;   // cow waves (host guarantees BS >= 128)
    const int ct = tid - 64, CW = BS - 64;
    int* ei = S.ei;
    int* fl = S.flags;
    const Level* LT = S.LT;
    if (tid == 0) { TS(0, (long long)wall_clock64()); TS(2, (long long)clock64()); TS(12, (long long)__smid()); }
    if ((tid & 63) == 0 && tid < 256) TS(22 + (tid >> 6), (long long)__builtin_amdgcn_s_getreg((31 << 11) | 4));   // HW_ID

    // ---- phase 0: env scalars, drone prefetch (wave 0); cattle integration, image zero-fill (cow waves).
    // Every wave issues its global loads before the first barrier, so their latency overlaps the launch of
    // the workgroup's other waves; LDS is written only after it.
    const int nd = Gv * N;
    const bool dlane = tid < nd;
    const int dg = dlane ? tid / N : 0, dk = tid - dg * N;
    const long long di = (long long)e0 * N + tid;
    R pos[3], q[4], v[3], w[3], pid[9], ql[4], rpy_in[3] = {0, 0, 0};
    R ph_lr[4] = {0, 0, 0, 0}, ph_rr[3] = {0, 0, 0};   // PHYS: last_clipped_action, DYN rpy_rates
    int stepi = 0, n0 = 0, act0 = 0, stepi_env = 0;
    double ev_acc = 0;   // update_evaluation_metrics' distance of this drone (optional)
    R spx_r[3] = {0, 0, 0}, spy_r[3] = {0, 0, 0};   // cow waves: prefetched spawn positions
    bool co_simd = false;   // a cow wave on the drone wave's SIMD (starved while the drone wave issues)
    // Phase 0 issues loads only: the values are combined after the barrier (the Euler cache flag, the obs block flag),
    // and the cow waves' registers are not zeroed for the lanes that load nothing (those lanes never read them) -- a
    // compare right after a load, or a zero written to a register whose load is in flight on other lanes, made the
    // wave wait for its loads before the barrier, one round trip each, and the barrier held the drone wave's chain
    // (CH_PHASE0_ZERO: the zeroed, combined-before-the-barrier form).
    uint8_t stale_d = 1;   // drone lanes: this env's Euler cache flag (0: valid)
#ifdef CH_PHASE0_ZERO
    R c0[4] = {0, 0, 0, 0};
    double c0d[2] = {0, 0}, prev0d = 0;
    int ei0[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    R er0[2] = {0, 0};
    double met0[kMetricRows];
#pragma unroll
    for (int r = 0; r < kMetricRows; ++r) met0[r] = 0;
#else
    R c0[4];
    double c0d[2], prev0d;
    int ei0[10];
    R er0[2];
    double met0[kMetricRows];
#endif
    double pd[3] = {0, 0, 0};   // MIX: f64 drone position
    uint8_t stale_o = 0;        // cow waves' env lanes: the obs block flag and the buffer tag, combined after the barrier
    unsigned long long tag_o = 0;
    if (tid >= 64) {
        if (ct < Gv * M) {
            const long long ci = (long long)e0 * M + ct;
#pragma unroll
            for (int c = 0; c < 4; ++c) c0[c] = p.cattle[c * CS + ci];
            if constexpr (MIX) { c0d[0] = p.cpos64[ci]; c0d[1] = p.cpos64[CS + ci]; }
        }
        if (ct < Gv) {
            const int e = e0 + ct;
#pragma unroll
            for (int r = 0; r < 9; ++r) ei0[r] = p.envi[r * E + e];
            // constant obs bytes unknown: flagged, or this buffer is not the one that holds them
#ifdef CH_PHASE0_ZERO
            ei0[9] = p.stale[E + e] | (p.obs_tag[e] != (unsigned long long)(uintptr_t)p.obs ? 1 : 0);
#else
            stale_o = p.stale[E + e];
            tag_o = p.obs_tag[e];
#endif
            er0[0] = p.envr[e]; er0[1] = p.envr[E + e];
            if constexpr (MIX) prev0d = p.prev64[e];
#pragma unroll
            for (int r = 0; r < kMetricRows; ++r) met0[r] = p.metrics[r * E + e];
        }
    } else if (dlane) {
        // the drone wave loads only what its chain reads, so the chain starts after one round trip; the
        // cow waves stage the env scalars, the curriculum table and the pair list meanwhile
        n0 = p.envi[0 * E + e0 + dg];
#ifdef CH_PHASE0_ZERO
        stale_d = p.stale[e0 + dg] == 0 ? 0 : 1;   // (compared before the barrier)
#else
        stale_d = p.stale[e0 + dg];   // this env's Euler cache (written by the last v2 step)
#endif
        if (marl) act0 = p.envi[7 * E + e0 + dg];
        pos[0] = p.drone[0 * DS + di]; pos[1] = p.drone[1 * DS + di]; pos[2] = p.drone[2 * DS + di];
        if constexpr (MIX) {
#pragma unroll
            for (int c = 0; c < 3; ++c) { pd[c] = p.pos64[c * DS + di]; pos[c] = R(pd[c]); }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) q[c] = p.drone[(3 + c) * DS + di];
#pragma unroll
        for (int c = 0; c < 3; ++c) { v[c] = p.drone[(7 + c) * DS + di]; w[c] = p.drone[(10 + c) * DS + di]; }
#pragma unroll
        for (int c = 0; c < 9; ++c) pid[c] = p.drone[(13 + c) * DS + di];
#pragma unroll
        for (int c = 0; c < 4; ++c) ql[c] = p.drone[(22 + c) * DS + di];   // Bullet's cached link frame (link_lag)
        // Euler angles of this quaternion, stored by the previous step (used iff the cache is
        // valid; loaded regardless so the loads issue with the state's, not after the stale flag returns)
#pragma unroll
        for (int c = 0; c < 3; ++c) rpy_in[c] = p.rpy[c * DS + di];
        stepi = p.envi[9 * E + e0 + dg];   // ch_step calls on this env so far: the Philox action counter
        if (p.evald) ev_acc = p.evald[di];
        if constexpr (PHYS) {
#pragma unroll
            for (int c = 0; c < 4; ++c) ph_lr[c] = p.phys[c * DS + di];
#pragma unroll
            for (int c = 0; c < 3; ++c) ph_rr[c] = p.phys[(4 + c) * DS + di];
        }
    }
    if (tid < Gv) stepi_env = p.envi[9 * E + e0 + tid];   // env lanes: the counter the write-back advances
    if (tid < kV2Flags) fl[tid] = 0;
    if constexpr (PW) { if (tid < G) reinterpret_cast<int*>(S.hasnb)[tid] = 0; }   // per-env alpha-row ready flags
    lds_barrier();   // hand-off counters cleared before anyone signals

    if (tid < 64) {
        __builtin_amdgcn_s_setprio(3);   // the drone wave is the critical path: it wins issue on a shared SIMD
        if (tid == 0)
            __hip_atomic_store(fl + V_DSIMD, 1 + (int)((__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
        const float rM0 = 1.0f / (float)M;
        for (int u = ct; u < Gv * M; u += CW) {
            const long long ci = (long long)e0 * M + u;   // the workgroup's cows are contiguous per component
            const bool first = u == ct;                  // loaded before the barrier
            R x = first ? c0[0] : p.cattle[0 * CS + ci], y = first ? c0[1] : p.cattle[1 * CS + ci];
            const R vx = first ? c0[2] : p.cattle[2 * CS + ci], vy = first ? c0[3] : p.cattle[3 * CS + ci];
            const R dt = R(p.dt);
            double xd = 0, yd = 0;
            if constexpr (MIX) { xd = first ? c0d[0] : p.cpos64[ci]; yd = first ? c0d[1] : p.cpos64[CS + ci]; }
            // frictionless cube (trace-pinned); no p.stepSimulation under Physics.DYN (BaseAviary.py:447-448)
            if (!PHYS || (p.physics != CH_PHYS_DYN && p.physics != CH_PHYS_DYN_RK4))
                for (int s = 0; s < p.substeps; ++s) {
                    if constexpr (MIX) { xd += (double)(vx * dt); yd += (double)(vy * dt); }
                    else { x += vx * dt; y += vy * dt; }
                }
            if constexpr (MIX) {
                x = R(xd); y = R(yd);
                CH_STS(&p.cpos64[ci], xd); CH_STS(&p.cpos64[CS + ci], yd);
                S.cxd[u] = xd; S.cyd[u] = yd;
            }
            CH_STS(&p.cattle[0 * CS + ci], x); CH_STS(&p.cattle[1 * CS + ci], y);
            S.cx[u] = x; S.cy[u] = y; S.cvx[u] = vx; S.cvy[u] = vy;
        }
        for (int k = ct; k < (int)(sizeof(kLevels) / 4); k += CW)
            reinterpret_cast<uint32_t*>(S.LT)[k] = reinterpret_cast<const uint32_t*>(kLevels)[k];
        for (int k = ct; k < P; k += CW) const_cast<uint16_t*>(S.pl)[k] = p.pairs[k];
        for (int k = ct; k < G * M; k += CW) {
            S.nbm[k] = 0;
            if (sep) S.cnt[k] = 0;
        }
#ifndef CH_NO_STREAM_FULL
        if constexpr (!PW)   // the shared queue's per-slot ready marks (alpha_full)
            for (int k = ct; k < G * P; k += CW) S.queue[k] = kQEmpty;
#endif
        if (ct < 64) {   // the first cow wave: env scalars, one env per lane
        const int g = ct;
        bool flk = false;
        if (g < Gv) {
            const int scA = ei0[2] + 1;   // the env scalars were loaded before the barrier
            flk = (scA % 2) == 0 && !(p.phase_mask & 2);
            ei[I_N * G + g] = ei0[0]; ei[I_SC * G + g] = ei0[1]; ei[I_SCA * G + g] = scA;
            ei[I_HASPREV * G + g] = ei0[3]; ei[I_LEVEL * G + g] = ei0[4];
            ei[I_TALLY * G + g] = ei0[5]; ei[I_SPAWN * G + g] = ei0[6];
            ei[I_ACTIVE * G + g] = ei0[7]; ei[I_EPISODE * G + g] = ei0[8];
            ei[I_FLOCK * G + g] = flk; ei[I_RESET * G + g] = 0; ei[I_HERD * G + g] = 0;
#ifndef CH_PHASE0_ZERO
            ei0[9] = stale_o | (tag_o != (unsigned long long)(uintptr_t)p.obs ? 1 : 0);
#endif
            ei[I_OBSD * G + g] = ei0[9];   // the obs block's constant bytes are unknown
            S.prev[g] = er0[0]; S.clock[g] = er0[1];
            if constexpr (MIX) S.prevd[g] = prev0d;
#pragma unroll
            for (int r = 0; r < kMetricRows; ++r) S.met[r * G + g] = met0[r];
        }
        // compact list of flocking envs (BaseAviary.py:454: every second step_counter_A)
        const unsigned long long bal = __ballot(flk);
        if (flk) ei[FL_LIST + __popcll(bal & ((1ull << ct) - 1ull))] = g;
        if (ct == 0) { ei[NF_AT] = __popcll(bal); ei[NR_AT] = 0; }
        }
        cow_sync(fl + F_E, W1, false, p.err);   // env scalars, flocking list, tables: seen by every cow wave
        {
            int ds = lds_peek(fl + V_DSIMD);
            int spins = 0;
            for (; ds == 0 && spins < (1 << 22); ++spins) {   // stored by the drone wave at its start
                __builtin_amdgcn_s_sleep(1);
                ds = lds_peek(fl + V_DSIMD);
            }
            spin_note(spins);
            co_simd = (int)((__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3) + 1 == ds;
        }
        if (ct == 0) TS(11, (long long)clock64());
        if (ct < 64) {
            // herd centroid (CattleAviary.py: HerdCentroid, np.mean over the cattle): needs only the integrated
            // cows, so it is done before the drone hand-off (signal HC)
            const int g = ct;
            if (g < Gv) {
                PT sx = 0, sy = 0;
                CH_UNROLL for (int j = 0; j < M; ++j) { sx += S.cxd[g * M + j]; sy += S.cyd[g * M + j]; }
                S.hcxd[g] = sx / PT(M); S.hcyd[g] = sy / PT(M);
                if constexpr (MIX) { S.hcx[g] = R(S.hcxd[g]); S.hcy[g] = R(S.hcyd[g]); }
            }
            lds_signal(fl + F_HC);
        }
        // spawn positions of the episode an auto-reset would start: scenario index + 1 (BaseAviary.py:600-606).
        // Loaded into registers here and parked in LDS after the pair loop, so the load latency hides
        // behind it and a reset needs no global load.  (Host geometry: G*M <= 3 * cow lanes.)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int u = ct + k * CW;
            if (u < Gv * M) {
                const int g = qdiv(u, M, rM0), j = u - g * M;
                int sp = ei[I_SPAWN * G + g] + 1;
                if (sp >= p.n_scen) sp = 0;
                const double* tab = p.spawn + ((long long)sp * p.n_cows + j) * 2;
                spx_r[k] = R(tab[0]); spy_r[k] = R(tab[1]);
            }
        }
    }
    if (tid == 0) TS(3, (long long)clock64());

    const bool wobs = !(p.phase_mask & 8);
    // late (shared tables with their own shepherd region): the cattle observation entries and the Euler angles
    // are written after the reset list is known, and each cow's final velocity by the last of three arrivals
    // (alpha row, shepherd sum, final pass).  fast (late, no terminal observation requested): the reset envs'
    // new bodies and observation rows are then written by the lanes that wrote their old values (drones: the
    // drone wave; cattle state: the phase-0 lane; obs: the single late writer), with no drain or sync.
    // Only the 16-env x 4-drone geometry: at 2 drones x 8 cattle (C2/C3, 3 cow waves) the final pass after the
    // reset list costs more than the reset sync it saves (C2 16.2 -> 17.2 us, C3 17.1 -> 17.8 us).
    // tobs (fast): the terminal observation of a reset env is written by the same producers, into p.terminal_obs,
    // each from the values it holds (drone rows: the drone wave; Euler angles, cattle entries, constant bytes: the cow
    // waves), instead of a drained copy of the finished block behind two cow-wave syncs
    const bool late = sep && GT == 16 && NT == 4, fast = late && (TOBS || !p.terminal_obs);
    const bool tobs = TOBS && p.terminal_obs != nullptr;
    float* obs_wg = p.obs + (long long)e0 * RW;
    // final per-env scalars, held by the drone wave's env lanes until the write-back
    int f_n = 0, f_sc = 0, f_scA = 0, f_hp = 0, f_level = 0, f_tally = 0, f_spawn = 0, f_active = 0, f_episode = 0;
    PT f_prev = 0;   // prev_cent_dists (f64 also in f32 mode: the approach delta is a difference of two ~10 m distances)
    R f_clock = 0;

    if (tid < 64) {
        // ============ drone wave: the critical path ============================================
        const int n = dlane ? n0 : 0;
        const bool live = dlane && dk < n;
        R px0 = 0, py0 = 0;
        if (live) {
            px0 = pos[0]; py0 = pos[1];
            const int e = e0 + dg;
            float a[4];
            if (p.flags & CH_STEP_RANDOM_ACTIONS) {
                uint32_t c4[4] = {(uint32_t)stepi, 0u, (uint32_t)dk, (uint32_t)(p.env_off + e)};
                philox(c4, p.k0, p.k1);
#pragma unroll
                for (int k = 0; k < 4; ++k) a[k] = (float)(c4[k] >> 8) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
                if (p.actions_out) reinterpret_cast<float4*>(p.actions_out)[di] = make_float4(a[0], a[1], a[2], a[3]);
            } else {
                float4 a4 = reinterpret_cast<const float4*>(p.actions)[di];
                a[0] = a4.x; a[1] = a4.y; a[2] = a4.z; a[3] = a4.w;
            }
            if (marl && !((act0 >> dk) & 1)) { a[0] = a[1] = a[2] = a[3] = 0.0f; }  // marl_wrapper.py:80-84
            R Rm[9], rpy[3];
            quat_to_mat(q, Rm);
            if (stale_d == 0) { rpy[0] = rpy_in[0]; rpy[1] = rpy_in[1]; rpy[2] = rpy_in[2]; }
            else quat_to_euler(q, rpy);
            if (!(p.phase_mask & 1)) {
                double rpm[4];
                pid_vel(pos, q, v, Rm, rpy, a, R(p.dt_ctrl), pid, rpm, p.debug ? p.debug + di * 16 : nullptr);
                R zl[3] = {0, 0, 0};   // the cached link frame's z axis (link_lag)
                if (p.link_lag) quat_to_zcol(ql, zl);
                if constexpr (PHYS) {
                    variant_substeps(p, dg * N, N, n, pos, q, v, w, rpm, ph_lr, ph_rr, MIX ? pd : nullptr, ql,
                                     zl, p.link_lag != 0);
#pragma unroll
                    for (int c = 0; c < 4; ++c) CH_STS(&p.phys[c * DS + di], ph_lr[c]);
#pragma unroll
                    for (int c = 0; c < 3; ++c) CH_STS(&p.phys[(4 + c) * DS + di], ph_rr[c]);
                } else {
#ifdef CH_SUBSTEP_UNROLL
                    // (ch_step_multi.hip: its translation unit runs without machine LICM; the default 4 substeps
                    // straight-line keep the loop-invariant parts of the substep out of a loop there)
                    if (p.substeps == 4) {
                        CH_UNROLL for (int s = 0; s < 4; ++s)
                            drone_substep(pos, q, v, w, rpm, R(p.dt), R(p.damping), p.torque_world != 0, p.gyro != 0,
                                          NoExtraForces(), MIX ? pd : nullptr, ql, zl, p.link_lag != 0);
                    } else
#endif
                    for (int s = 0; s < p.substeps; ++s)
                        drone_substep(pos, q, v, w, rpm, R(p.dt), R(p.damping), p.torque_world != 0, p.gyro != 0,
                                      NoExtraForces(), MIX ? pd : nullptr, ql, zl, p.link_lag != 0);
                }
            }
            R* D = p.drone;
            if constexpr (MIX) {
#pragma unroll
                for (int c = 0; c < 3; ++c) CH_STS(&p.pos64[c * DS + di], pd[c]);
                S.dxd[tid] = pd[0]; S.dyd[tid] = pd[1];
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) CH_STS(&D[c * DS + di], pos[c]);
#pragma unroll
            for (int c = 0; c < 4; ++c) CH_STS(&D[(3 + c) * DS + di], q[c]);
#pragma unroll
            for (int c = 0; c < 3; ++c) { CH_STS(&D[(7 + c) * DS + di], v[c]); CH_STS(&D[(10 + c) * DS + di], w[c]); }
#pragma unroll
            for (int c = 0; c < 9; ++c) CH_STS(&D[(13 + c) * DS + di], pid[c]);
            if (p.link_lag) {
#pragma unroll
                for (int c = 0; c < 4; ++c) CH_STS(&D[(22 + c) * DS + di], ql[c]);
            }
            S.dx[tid] = pos[0]; S.dy[tid] = pos[1]; S.dz[tid] = pos[2];
#pragma unroll
            for (int c = 0; c < 4; ++c) S.dq[c * (G * N) + tid] = q[c];
        }
        wave_sync();
        lds_signal(fl + F_D);   // positions published: the cow waves' distance work starts now
        // the own-state row but its Euler angles, which a cow wave computes from S.dq (obs_euler)
        if (live && wobs) obs_own_nrpy(obs_wg + dg * RW, dk, pos[2], v, w);
        if (tid == 0) TS(4, (long long)clock64());
        lds_wait(fl + F_E, W1, p.err);   // env scalars and the curriculum table (staged by the cow waves)
        if (p.evald && live) CH_STS(&p.evald[di], eval_distance_step(ev_acc, ei[I_SC * G + dg] == 0, px0, py0, pos[0], pos[1]));

        // per-drone reward terms (CattleAviary.py:230-246, 572-679) and neighbour obs (BaseRLAviary.py:303-317)
        int nb1 = -1, nb2 = -1;   // the two nearest drones (kept for a fast reset's terminal observation)
        // QUAD: this drone's terms in registers (nearest distances, flags, spacing terms; the cattle term after H)
        R q_pa = 0, q_pb = 0, q_sa = 0, q_sb = 0, q_ca = 0, q_cb = 0, q_ps = 0, q_sc = 0;
        int q_df = 0;
        if (live && task) {
            const int i = dk, b0 = dg * N;
            const R xi = pos[0], yi = pos[1];
            R m1 = R(INFINITY), m2 = R(INFINITY), b1 = 0, b2 = 0;
            int i1 = -1, i2 = -1;
            uint8_t f = 0;
            bool iso = true;
            // (branch-free: every other drone slot is evaluated and the updates selected -- the lanes' j == i
            // differ, so the branchy loop ran every body anyway)
            CH_UNROLL for (int j = 0; j < N; ++j) {
                const bool v = j < n && j != i;
                const R d = norm2(S.dx[b0 + j] - xi, S.dy[b0 + j] - yi);
                f |= (v && d != d) ? 8 : 0;
                const bool lt1 = v && d < m1, lt2 = v && !(d < m1) && d < m2;
                m2 = lt1 ? m1 : (lt2 ? d : m2);
                m1 = lt1 ? d : m1;
                f |= (v && d < R(kCollision)) ? 2 : 0;
                iso = iso && !(v && !(d > R(kMaxFormation)));
                const bool n1 = v && (i1 < 0 || d < b1), n2 = v && !n1 && (i2 < 0 || d < b2);
                i2 = n1 ? i1 : (n2 ? j : i2);
                b2 = n1 ? b1 : (n2 ? d : b2);
                i1 = n1 ? j : i1;
                b1 = n1 ? d : b1;
            }
            if (iso) f |= 4;
            if (fabs(pos[2] - R(kTargetAlt)) > R(kTargetAlt * 0.6)) f |= 1;
            if constexpr (QUAD) {
                q_pa = m1; q_pb = m2; q_df = f;
                spacing_terms_r(LT[ei[I_LEVEL * G + dg]], p.compat != 0, m1, m2, q_sa, q_sb, q_ca, q_cb, q_ps);
            } else {
                S.pa[tid] = m1; S.pb[tid] = m2; S.dflags[tid] = f;
                if constexpr (!SPLIT) spacing_terms(S, LT[ei[I_LEVEL * G + dg]], p.compat != 0, tid, m1, m2);
            }
            // offsets from the f64 positions in f32 mode (S.dxd; the same array as S.dx in f64 mode)
            if (wobs) obs_nbr(obs_wg + dg * RW, S.dxd, S.dyd, b0, i, i1, i2);
            nb1 = i1; nb2 = i2;
        }
        lds_signal(fl + F_T);
        if (tid == 0) TS(5, (long long)clock64());
        const int force = (p.phase_mask & CH_PHASE_FORCE_TIMEOUT) ? 1 : 0;
        lds_wait(fl + F_HC, 1, p.err);   // herd centroids
        // EARLY (CTDE, opt-in CH_EARLY_RESET): the auto-reset decision comes before the cow items (hand-off H:
        // cow-drone distances, winding numbers).  CattleAviary's _computeTerminated reads the herding effectiveness
        // only at curriculum levels 4-6 (CattleAviary.py:465-474; a success at level 3 can move its second call to
        // level 4) and _computeTruncated never does (497-552): a workgroup without such an env publishes its reset
        // list from the drone terms and the centroids alone, and waits for H only for the reward.  Measured (same box,
        // profiles/r03/b/ab.log): no gain -- H completes at ~27.0k cycles, before the drone wave would wait for it,
        // and the reset decision itself takes ~3k cycles after the drone terms; the reset list moved from 31.4k to
        // 30.5k cycles but the drone wave's end moved from 37.0k to 38.4k (the cow waves' final pass now competes
        // with its reward), 197.4 vs 196.8 M env-steps/s.
#ifdef CH_EARLY_RESET
        constexpr bool EARLY = !marl && !SPLIT && !QUAD;
#else
        constexpr bool EARLY = false;
#endif
        // the env this lane keeps the books of: lane g (env lanes), or the lane's quad (QUAD; lane k = 0 stores)
        const int g = QUAD ? dg : tid;
        const bool envl = QUAD ? dlane : g < Gv;
        const bool envw = envl && (!QUAD || dk == 0);
        bool h_done = !EARLY;
        if constexpr (EARLY) {
            const int lv0 = envl ? ei[I_LEVEL * G + g] : 0;
            h_done = __ballot(envl && task && lv0 >= 3 && lv0 <= 6) != 0;
        }
        if (h_done) lds_wait(fl + F_H, Gv * M + force, p.err);   // every cow item
        if (tid == 0) TS(6, (long long)clock64());
        if (live && task && !SPLIT && h_done) {
            if constexpr (QUAD) q_sc = cattle_term(S, tid, M, R(p.cs_cc));
            else S.scat[tid] = cattle_term(S, tid, M, R(p.cs_cc));
            if constexpr (marl) {
                // MARLCattleAviary._computeReward's per-agent part at the step's starting level
                // (MARLCattleAviary.py:110-178), on every drone lane at once: the prefix
                // P = simple w_s + complex w_c + 0.1 w_surv (psp), Q = P + eff/100 w_eff + cattle w_cat --
                // the whole reward when the approach term is +-0, i.e. for every call but the first of a step
                // (mq) -- and the end-of-episode bonus (meor, 183-241).  The env lane then only chains the
                // calls' side effects (bookkeeping below); cent and eff are computed as the env lane does.
                const int g = dg, n = n0, b0 = dg * N;
                const int lv = ei[I_LEVEL * G + g];
                const Level& Lv = LT[lv];
                const R a = S.pa[tid], b = S.pb[tid], sa = S.sa[tid], sb = S.sb[tid], ca = S.ca[tid], cb = S.cb[tid];
                R simple = (sa + sb) / R(2), cplx = (ca + cb) / R(2);
                if (!p.compat) {
                    if (!(b < R(INFINITY))) { simple = sa; cplx = ca; }
                    if (!(a < R(INFINITY))) { simple = 0; cplx = 0; }
                }
                R P = 0;
                P += simple * R(Lv.w_simple);
                P += cplx * R(Lv.w_complex);
                P += R(0.1) * R(Lv.w_survival);
                PT sdx = 0, sdy = 0;
                CH_UNROLL for (int i = 0; i < N; ++i) {
                    const bool li = i < n;
                    sdx += li ? S.dxd[b0 + i] : PT(0); sdy += li ? S.dyd[b0 + i] : PT(0);
                }
                sdx = divc(sdx, PT(n)); sdy = divc(sdy, PT(n));
                const R scx = S.hcx[g], scy = S.hcy[g];
                const PT ex = sdx - S.hcxd[g], ey = sdy - S.hcyd[g];
                const R cent = R(sqrt(ex * ex + ey * ey + PT(0) * PT(0)));
                const R eff = R((double)ei[I_HERD * G + g] / M * 100);
                R Q = P;
                Q += divc(eff, R(100)) * R(Lv.w_eff);
                Q += S.scat[tid] * R(Lv.w_cattle);
                S.psp[tid] = P;
                S.mq[tid] = Q;
                S.meor[tid] = marl_end_of_episode_L(Lv, lv, a, b, cent, eff, norm2(scx - pos[0], scy - pos[1]), n);
            }
        }
        wave_sync();
        if (tid == 0) TS(26, (long long)clock64());

        // per-env bookkeeping, one env per lane, in the reference's call order; the final scalars stay in
        // this lane's registers and go to HBM after the last barrier
        const int e = e0 + g, b0 = g * N;
        if (envl) {
            f_n = ei[I_N * G + g]; f_sc = ei[I_SC * G + g]; f_scA = ei[I_SCA * G + g]; f_hp = ei[I_HASPREV * G + g];
            f_level = ei[I_LEVEL * G + g]; f_tally = ei[I_TALLY * G + g]; f_spawn = ei[I_SPAWN * G + g];
            f_active = ei[I_ACTIVE * G + g]; f_episode = ei[I_EPISODE * G + g];
            f_prev = S.prevd[g]; f_clock = S.clock[g];
        }
        int done = 0, rs = 0, n_term = 0, n_trunc = 0, n_nan = 0, level_r = f_level;
        double ret = 0;
        bool te2 = false, tr = false;
        PT cent = 0;   // HerdCentroid/DroneCentroid distance (f64 also in f32 mode; R(cent) where the f32 math reads it)
        R eff = 0, ms = R(INFINITY), scx = 0, scy = 0;
        const PT max_step_p = PT(0.3 * kMaxSpeedKmh * (1000.0 / 3600.0)) / PT(p.ctrl_freq);
        // QUAD: the env's four drones' positions and terms on every lane of its quad (convergent DPP moves)
        constexpr int NQ = QUAD ? 4 : 1;
        PT qx[NQ], qy[NQ];
        R qpa[NQ], qpb[NQ], qsa[NQ], qsb[NQ], qca[NQ], qcb[NQ], qps[NQ], qsc[NQ];
        int qdf[NQ];
        if constexpr (QUAD) {
            PT x0 = 0, y0 = 0;
            if (live) {
                if constexpr (MIX) { x0 = pd[0]; y0 = pd[1]; } else { x0 = PT(pos[0]); y0 = PT(pos[1]); }
            }
            qall(x0, qx); qall(y0, qy); qall(q_pa, qpa); qall(q_pb, qpb); qall(q_df, qdf);
            qall(q_sa, qsa); qall(q_sb, qsb); qall(q_ca, qca); qall(q_cb, qcb); qall(q_ps, qps); qall(q_sc, qsc);
        }
        if (envl && task) {
            const int n = f_n;
            PT sdx = 0, sdy = 0;
            const int herded = h_done ? ei[I_HERD * G + g] : 0;   // counted by the cow waves (winding number)
            scx = S.hcx[g]; scy = S.hcy[g];          // herd centroid, summed by the cow waves
            // per-drone sums without per-lane branches: a drone beyond NUM_DRONES adds +0, which leaves a sum
            // that starts at +0 unchanged (x + +0 = x unless x = -0, and such a sum is never -0)
            CH_UNROLL for (int i = 0; i < N; ++i) {
                const bool li = i < n;
                const PT xi = QUAD ? qx[i % NQ] : S.dxd[b0 + i], yi = QUAD ? qy[i % NQ] : S.dyd[b0 + i];
                sdx += li ? xi : PT(0); sdy += li ? yi : PT(0);
            }
            sdx = divc(sdx, PT(n)); sdy = divc(sdy, PT(n));
            PT ex = sdx - S.hcxd[g], ey = sdy - S.hcyd[g];
            cent = sqrt(ex * ex + ey * ey + PT(0) * PT(0));   // HerdCentroid/DroneCentroid, z = 0.95 both
            eff = h_done ? R((double)herded / M * 100) : R(0);   // (not read by this step's terminated calls)
            bool anynan = false;
            uint8_t any = 0;
            CH_UNROLL for (int i = 0; i < N; ++i) {
                const bool li = i < n;
                const R pa = QUAD ? qpa[i % NQ] : S.pa[b0 + i];
                const uint8_t df = li ? (QUAD ? (uint8_t)qdf[i % NQ] : S.dflags[b0 + i]) : 0;
                if (li && pa < ms) ms = pa;
                anynan |= (df & 8) != 0;
                any |= df;
            }
            if (anynan) ms = R(NAN);
            const bool time_up = (double)f_sc / p.ctrl_freq > p.episode_len;
            if (g == 0) TS(32, (long long)clock64());
            if constexpr (!marl) {
                // CattleAviary: _computeReward (CattleAviary.py:213-332), then _computeTerminated twice and
                // _computeTruncated.  The terminated calls read nothing the reward writes (the reward uses the
                // level it started with), so they run first and the reset decision is published early.
                const R inc = R(1.0 / 240);
                bool te = term_call(LT, f_level, f_clock, inc, ms, R(cent), eff);
                if (te) curriculum_success(LT, f_level, f_tally);
                te2 = term_call(LT, f_level, f_clock, inc, ms, R(cent), eff);
                tr = (any & 7) || cent > PT(kMissionBoundary) || time_up;
                done = te2 || tr;
            } else {
                // MARLCattleAviary reward / terminated / truncated in the order env.step
                // (rllib_envs/BaseAviary.py:425-431) and the wrapper (marl_wrapper.py:104-113) call them.
                // Up to 2N rewards and 3N terminated calls run in sequence (their side effects chain), so the
                // per-agent inputs and the current curriculum level live in registers (geometry-specialised
                // kernels: NT > 0, every agent loop unrolled) instead of being re-read from LDS per call.
                int& level = f_level;
                int& tally = f_tally;
                int& has_prev = f_hp;
                int& active = f_active;
                PT& prev = f_prev;
                R& clock = f_clock;
                const R inc = R(1.0) / R(p.ctrl_freq);
                const int lvl0 = level;
                // env.step counts its step (step_counter += 1, rllib_envs/BaseAviary.py:436) between its
                // own dicts and the wrapper's recomputation, so the wrapper sees the time limit one step
                // earlier (MARLCattleAviary.py:376)
                const bool time_up_w = (double)(f_sc + 1) / p.ctrl_freq > p.episode_len;
                constexpr int NR = NT ? NT : 1;
                R r_pa[NR], r_pb[NR], r_sc[NR], r_dh[NR], r_rw[NR];
                R r_pp[NR], r_qq[NR], r_eo[NR];
                uint8_t r_df[NR], r_d1[NR];
                if constexpr (NT > 0) {
                    CH_UNROLL for (int i = 0; i < NT; ++i) {
                        r_pa[i] = S.pa[b0 + i]; r_pb[i] = S.pb[b0 + i]; r_sc[i] = S.scat[b0 + i];
                        r_dh[i] = norm2(scx - S.dx[b0 + i], scy - S.dy[b0 + i]);   // drone to herd centroid (level 4/6 bonus)
                        r_df[i] = S.dflags[b0 + i];
                        r_pp[i] = S.psp[b0 + i]; r_qq[i] = S.mq[b0 + i]; r_eo[i] = S.meor[b0 + i];
                    }
                }
#define AG(arr, lds) [&](int i_) { if constexpr (NT > 0) return arr[i_]; else return lds; }
                auto PA = AG(r_pa, S.pa[b0 + i_]);
                auto PB = AG(r_pb, S.pb[b0 + i_]);
                auto SC = AG(r_sc, S.scat[b0 + i_]);
                auto DH = AG(r_dh, norm2(scx - S.dx[b0 + i_], scy - S.dy[b0 + i_]));
                auto DF = AG(r_df, S.dflags[b0 + i_]);
                auto PP = AG(r_pp, S.psp[b0 + i_]);
                auto QQ = AG(r_qq, S.mq[b0 + i_]);
                auto EO = AG(r_eo, S.meor[b0 + i_]);
#undef AG
                Level Lc = LT[level];   // the current level's constants (re-read when the level changes)
                const PT approach_div = max_step_p + PT(1e-6);
                const R eff100 = divc(eff, R(100));   // eff / 100, the same for every call of this step
                auto succeed = [&]() {   // curriculum_success (curriculum_learning.py:200-219)
                    tally += 1;
                    if (tally >= Lc.required_tally) {
                        tally = 0;
                        level += 1;
                        if (level >= 8) level = 7;
                        Lc = LT[level];
                    }
                };
                auto trunc_i = [&](int i, bool tu) -> bool {
                    return (DF(i) & 7) || cent > PT(kMissionBoundary) || tu;
                };
                const R centR = R(cent);
                auto reward_i = [&](int i, bool tu) -> R {
                    const R a = PA(i), b = PB(i);
                    const bool same = level == lvl0;   // the drone lanes' prefixes hold for this level
                    PT change = has_prev ? prev - cent : PT(0.0);
                    prev = cent; has_prev = 1;
                    R r;
                    if (same && change == PT(0)) {
                        // the approach term is +-0 and leaves P unchanged: the reward is Q
                        r = QQ(i);
                    } else {
                        if (same) {
                            r = PP(i);
                        } else {
                            const R sa = simple_spacing(a, Lc), sb = simple_spacing(b, Lc);
                            const R ca = complex_spacing(a, Lc), cb = complex_spacing(b, Lc);
                            R simple = (sa + sb) / R(2), cplx = (ca + cb) / R(2);
                            if (!p.compat) {
                                if (!(b < R(INFINITY))) { simple = sa; cplx = ca; }
                                if (!(a < R(INFINITY))) { simple = 0; cplx = 0; }
                            }
                            r = 0;
                            r += simple * R(Lc.w_simple);
                            r += cplx * R(Lc.w_complex);
                            r += R(0.1) * R(Lc.w_survival);
                        }
                        r += R(clip(divc(change, approach_div) * PT(5), PT(-1.0), PT(1.0))) * R(Lc.w_approach);
                        r += eff100 * R(Lc.w_eff);
                        r += SC(i) * R(Lc.w_cattle);
                    }
                    if (term_call_L(Lc, level, clock, inc, ms, centR, eff)) {
                        r += same ? EO(i) : marl_end_of_episode_L(Lc, level, a, b, centR, eff, DH(i), n);
                        succeed();
                    } else if (trunc_i(i, tu)) {
                        r -= R(50);
                    }
                    return r;
                };
                // Fast path (wrapper semantics, the common step): every terminated call of the step -- n in
                // env.step's rewards, n for its dict, then a reward and a terminated call per live agent in
                // the wrapper -- sees the same inputs, so whether any returns True follows from the level and,
                // at levels 0/1, the clock recurrence alone.  If none does, there is no end-of-episode bonus,
                // no curriculum step and no agent drop-out; every wrapper reward is Q (its approach term is +-0
                // after env.step's first call) minus the truncation penalty.  Otherwise the calls run in order.
                const int act0 = active;
                bool fast = p.marl_wrapper != 0;
                if (fast) {
                    int nact = 0;
                    CH_UNROLL for (int i = 0; i < N; ++i) nact += (i < n && ((act0 >> i) & 1)) ? 1 : 0;
                    const int K = 2 * n + 2 * nact;
                    R ck = clock;
                    if (level == 0 || level == 1) {
                        const R up = R(Lc.desired) + R(Lc.desired) * R(Lc.tol), lo = R(Lc.desired) - R(Lc.desired) * R(Lc.tol);
                        if (ms < up && ms > lo) {
                            for (int k = 0; k < K && fast; ++k) {
                                ck += inc;
                                if (ck >= R(Lc.hold)) fast = false;
                            }
                        } else if (K > 0) {
                            ck = 0;
                        }
                    } else if (K > 0) {
                        fast = !term_call_L(Lc, level, ck, inc, ms, centR, eff);
                    }
                    if (fast) {
                        clock = ck;
                        if (n > 0) { prev = cent; has_prev = 1; }
                        done = 1;
                        CH_UNROLL for (int i = 0; i < N; ++i) {
                            R rr = R(NAN);
                            uint8_t trr = 0;
                            if (i < n && ((act0 >> i) & 1)) {
                                rr = QQ(i);
                                trr = trunc_i(i, time_up_w);
                                if (trr) rr -= R(50);
                                done = 0;
                            }
                            CH_ST(&p.reward[(long long)e * N + i], (float)rr);
                            p.term[(long long)e * N + i] = 0;
                            p.trunc[(long long)e * N + i] = trr;
                            if (i < n && rr == rr) ret += (double)rr;
                            n_trunc += trr;
                            if (i < n && ((act0 >> i) & 1) && rr != rr) n_nan += 1;
                        }
                    }
                }
                if (!fast) {
                    if (g == 0) TS(33, (long long)clock64());
                    // env.step's own dicts (rllib_envs/BaseAviary.py:425-431)
                    CH_UNROLL for (int i = 0; i < N; ++i) {
                        if (i >= n) break;
                        const R rr = reward_i(i, time_up);
                        if constexpr (NT > 0) r_rw[i] = rr; else S.mrew[b0 + i] = rr;
                    }
                    CH_UNROLL for (int i = 0; i < N; ++i) {
                        if (i >= n) break;
                        const uint8_t d = term_call_L(Lc, level, clock, inc, ms, centR, eff);
                        if constexpr (NT > 0) r_d1[i] = d; else S.md1[b0 + i] = d;
                    }
                    if (g == 0) TS(34, (long long)clock64());
                    if (p.marl_wrapper) {
                        // the wrapper recomputes everything per live agent (marl_wrapper.py:104-110)
                        done = 1;
                        CH_UNROLL for (int i = 0; i < N; ++i) {
                            R rr = R(NAN);
                            uint8_t tt = 0, trr = 0;
                            if (i < n && ((act0 >> i) & 1)) {
                                rr = reward_i(i, time_up_w);
                                tt = term_call_L(Lc, level, clock, inc, ms, centR, eff);
                                trr = trunc_i(i, time_up_w);
                            }
                            CH_ST(&p.reward[(long long)e * N + i], (float)rr);
                            p.term[(long long)e * N + i] = tt;
                            p.trunc[(long long)e * N + i] = trr;
                            if (i < n && rr == rr) ret += (double)rr;
                            n_term += tt; n_trunc += trr;
                            if (i < n && (((act0 >> i) & 1) || tt) && rr != rr) n_nan += 1;
                            if (i < n && ((act0 >> i) & 1) && tt) active &= ~(1 << i);   // finished agents drop out
                        }
                        CH_UNROLL for (int i = 0; i < N; ++i)
                            if (i < n && ((active >> i) & 1)) done = 0;   // __all__: every agent terminated (marl_wrapper.py:113-117)
                    } else {
                        done = 1;   // bare env.step dicts: __all__ = all(done.values())
                        CH_UNROLL for (int i = 0; i < N; ++i) {
                            R rr = R(NAN);
                            uint8_t tt = 0, trr = 0;
                            if (i < n) {
                                if constexpr (NT > 0) { rr = r_rw[i]; tt = r_d1[i]; } else { rr = S.mrew[b0 + i]; tt = S.md1[b0 + i]; }
                                trr = trunc_i(i, time_up);
                                done &= tt;
                            }
                            CH_ST(&p.reward[(long long)e * N + i], (float)rr);
                            p.term[(long long)e * N + i] = tt;
                            p.trunc[(long long)e * N + i] = trr;
                            if (i < n && rr == rr) ret += (double)rr;
                            n_term += tt; n_trunc += trr;
                            if (i < n && (((act0 >> i) & 1) || tt) && rr != rr) n_nan += 1;
                        }
                    }
                }
            }
            rs = done && (p.flags & CH_STEP_AUTORESET);
        }
        // publish the reset list: the cow waves rebuild those envs while this wave finishes the reward.
        // This wave's drone-state stores are complete first (the cow waves overwrite reset drones).
        if (envw) ei[I_RESET * G + g] = rs;
        // the next episode's NUM_DRONES draw (BaseAviary.py:307), once: reset_scalars takes it from here.  (Drawn on
        // every env lane ahead of the cow items' hand-off instead, measured: no gain, profiles/r03/n/ab_draw.log.)
        int n_next = 0;
        if (envl && rs) n_next = p.reset_n ? p.reset_n[e] : reset_draw_n(p, f_episode, p.env_off + e);
        if (envw && rs) ei[I_NEWN * G + g] = n_next;
        const unsigned long long rbal = __ballot(envw && rs != 0);
        if (envw && rs) ei[RS_LIST + __popcll(rbal & ((1ull << tid) - 1ull))] = g;   // (writers in env order)
        if (tid == 0) ei[NR_AT] = __popcll(rbal);
        if (tid == 0) TS(27, (long long)clock64());
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        lds_signal(fl + F_R);
        if (tid == 0) TS(15, (long long)clock64());
        if (fast && ei[NR_AT]) {
            // SB3 auto-reset, drone side (BaseAviary.reset, BaseAviary.py:280-331): each drone lane of a reset env
            // writes its new body, Euler cache and observation row itself (it wrote the old ones)
            wave_sync();   // the reset flags and NUM_DRONES draws of the env lanes
            const bool rd = dlane && ei[I_RESET * G + dg];
            const int n_new = rd ? ei[I_NEWN * G + dg] : 0;
            if (tobs && wobs && rd && live) {
                // the terminal observation's own and neighbour entries, from this lane's end-of-episode state (its
                // Euler angles, cattle entries and constant bytes come from the cow waves)
                float* tb = p.terminal_obs + (long long)(e0 + dg) * RW;
                obs_own_nrpy(tb, dk, pos[2], v, w);
                if (task) obs_nbr(tb, S.dxd, S.dyd, dg * N, dk, nb1, nb2);
            }
            double xd = 0, yd = 0, zd = 0;
            if (rd) {
                reset_drone_xyz(dk, n_new, xd, yd, zd);
                S.rdx[tid] = R(xd); S.rdy[tid] = R(yd); S.rdz[tid] = R(zd);
            }
            const R z = R(zd);
            wave_sync();   // the env's new drone positions (nearest neighbours)
            if (rd) {
                reset_drone_store(p, di, xd, yd, zd);
                if constexpr (PHYS) {   // last_clipped_action, rpy_rates = 0 (_housekeeping, BaseAviary.py:565, 581-582)
#pragma unroll
                    for (int c = 0; c < kPhysComps; ++c) CH_STS(&p.phys[c * DS + di], R(0));
                }
                // identity attitude: Euler angles (+0, -0, +0) for the next step's cache
                CH_STS(&p.rpy[di], R(0)); CH_STS(&p.rpy[DS + di], -R(0)); CH_STS(&p.rpy[2 * DS + di], R(0));
                if (wobs) {
                    float* eb = obs_wg + dg * RW;
                    if (dk < n_new) {
                        // identity quaternion: getEulerFromQuaternion gives (+0, -0, +0) (quat_to_euler); zero velocities
                        const R zero3[3] = {0, 0, 0}, rpy0[3] = {R(0), -R(0), R(0)};
                        obs_own(eb, dk, z, rpy0, zero3, zero3);
                        const int nb = nearest_two(S.rdx, S.rdy, dg * N, dk, n_new);
                        obs_nbr(eb, S.rdx, S.rdy, dg * N, dk, (nb & 0xff) - 1, (nb >> 8) - 1);
                    } else if (dk < ei[I_N * G + dg]) {
                        // a row the old episode used and the new one does not: own and neighbour entries (the late
                        // cattle pass zeroes its cattle entries; the rest of the row is constant zero)
                        for (int c = 0; c < 14; c += 2) st2(eb, dk * 86 + c, 0.0f, 0.0f);
                    }
                }
            }
        }
        if constexpr (EARLY) {
            if (!h_done) {   // the reward's inputs from the cow items: closest cows, the effectiveness
                lds_wait(fl + F_H, Gv * M + force, p.err);
                if (tid == 0) TS(6, (long long)clock64());
                if (live && task) S.scat[tid] = cattle_term(S, tid, M, R(p.cs_cc));
                wave_sync();
                if (envl && task) eff = R((double)ei[I_HERD * G + g] / M * 100);
            }
        }
        if constexpr (SPLIT) lds_wait(fl + F_S, 2 * Gv * N, p.err);   // spacing and cattle terms (cow waves)
        if (envl && task) {
            const int n = f_n;
            if constexpr (!marl) {
                const Level& Lv = LT[level_r];
                // branch-free per-drone sums (a skipped term adds +0, see the centroid above)
                R sp_simple = 0, sp_complex = 0, msp = 0, mcat = 0, cat = 0;
                R psp_i[NT ? NT : 12], scat_i[NT ? NT : 12];
                CH_UNROLL for (int i = 0; i < N; ++i) {
                    const bool li = i < n;
                    const int iq = i % NQ;
                    const R pa = QUAD ? qpa[iq] : S.pa[b0 + i], pb = QUAD ? qpb[iq] : S.pb[b0 + i];
                    const bool ua = li && (p.compat || pa < R(INFINITY)), ub = li && (p.compat || pb < R(INFINITY));
                    sp_complex += ua ? (QUAD ? qca[iq] : S.ca[b0 + i]) : R(0);
                    sp_simple += ua ? (QUAD ? qsa[iq] : S.sa[b0 + i]) : R(0);
                    sp_complex += ub ? (QUAD ? qcb[iq] : S.cb[b0 + i]) : R(0);
                    sp_simple += ub ? (QUAD ? qsb[iq] : S.sb[b0 + i]) : R(0);
                    psp_i[i] = QUAD ? qps[iq] : S.psp[b0 + i]; scat_i[i] = QUAD ? qsc[iq] : S.scat[b0 + i];
                }
                const R n2 = R(n * 2.0), nn = R(n);
                sp_complex = divc(sp_complex, n2); sp_simple = divc(sp_simple, n2);
                R approach = 0;
                if (f_hp) approach = R(clip(divc(f_prev - cent, max_step_p + PT(1e-6)) * PT(5), PT(-1.0), PT(1.0)));
                f_prev = cent; f_hp = 1;
                CH_UNROLL for (int i = 0; i < N; ++i) cat += i < n ? scat_i[i] : R(0);
                cat = divc(cat, nn);
                R rg = sp_simple * R(Lv.w_simple) + sp_complex * R(Lv.w_complex) + R(0.1) * R(Lv.w_survival) +
                       approach * R(Lv.w_approach) + divc(eff, R(100)) * R(Lv.w_eff) + cat * R(Lv.w_cattle);
                CH_UNROLL for (int i = 0; i < N; ++i) { msp += i < n ? psp_i[i] : R(0); mcat += i < n ? scat_i[i] : R(0); }
                msp = divc(msp, nn); mcat = divc(mcat, nn);
                R tot = 0;
                CH_UNROLL for (int i = 0; i < N; ++i) tot += i < n ? rg + R(0.5) * ((psp_i[i] - msp) + (scat_i[i] - mcat)) : R(0);
                R rew = divc(tot, nn);
                if (envw) {
                    CH_ST(&p.reward[e], (float)rew);
                    p.term[e] = te2; p.trunc[e] = tr;
                }
                ret = (double)rew;
                n_term = te2; n_trunc = tr; n_nan = rew != rew;
            }
            if (g == 0) TS(19, (long long)clock64());
            f_sc += marl ? 1 : p.substeps;
            // metric accumulators (rank-local; bench.py all-reduces them)
            const double* mt = S.met;
            double o[kMetricRows];
#pragma unroll
            for (int r = 0; r < kMetricRows; ++r) o[r] = mt[r * G + g];
            o[CH_METRIC_STEPS] += 1;
            o[CH_METRIC_TERMINATED] += n_term;
            o[CH_METRIC_TRUNCATED] += n_trunc;
            o[CH_METRIC_NAN_REWARDS] += n_nan;
            o[CH_METRIC_EFFECTIVENESS_SUM] += (double)eff;
            o[kMetricCurReturn] += ret;
            o[kMetricCurLen] += 1;
            if (done) {
                // SB3 Monitor's episode record (its reward sum and length) for the env that ends here
                if (p.episode_stats && envw) {
                    CH_ST(&p.episode_stats[2 * (long long)e], o[kMetricCurReturn]);
                    CH_ST(&p.episode_stats[2 * (long long)e + 1], o[kMetricCurLen]);
                }
                o[CH_METRIC_EPISODES] += 1;
                o[CH_METRIC_RETURN_SUM] += o[kMetricCurReturn];
                o[CH_METRIC_LENGTH_SUM] += o[kMetricCurLen];
                o[kMetricCurReturn] = 0;
                o[kMetricCurLen] = 0;
            }
#pragma unroll
            for (int r = 0; r < kMetricRows; ++r)
                if (envw) CH_STS(&p.metrics[r * E + e], o[r]);
            if (g == 0) TS(28, (long long)clock64());
            if (p.reset_happened && envw) p.reset_happened[e] = rs;
            // SB3 auto-reset: the new episode's scalars (the cow waves rebuild its bodies and observation)
            if (rs) reset_scalars(p, e, f_n, f_sc, f_scA, f_spawn, f_episode, f_active, f_hp, f_prev, f_clock, n_next);
            if (p.agent_active && envw)
                for (int i = 0; i < N; ++i) p.agent_active[(long long)e * N + i] = (f_active >> i) & 1;
        } else if (envw && p.reset_happened) {
            p.reset_happened[e] = 0;
        }
        if (tid == 0) TS(7, (long long)clock64());
        // ---- env scalars back to HBM from the env lanes' registers (nothing after this step reads them)
        if (QUAD ? envw : tid < Gv) {
            const int e = e0 + (QUAD ? dg : tid);
            CH_STS(&p.envi[0 * E + e], f_n); CH_STS(&p.envi[1 * E + e], f_sc); CH_STS(&p.envi[2 * E + e], f_scA);
            CH_STS(&p.envi[3 * E + e], f_hp); CH_STS(&p.envi[4 * E + e], f_level); CH_STS(&p.envi[5 * E + e], f_tally);
            CH_STS(&p.envi[6 * E + e], f_spawn); CH_STS(&p.envi[7 * E + e], f_active); CH_STS(&p.envi[8 * E + e], f_episode);
            CH_STS(&p.envi[9 * E + e], (QUAD ? stepi : stepi_env) + 1);   // ch_step calls on this env
            CH_STS(&p.envr[0 * E + e], R(f_prev)); CH_STS(&p.envr[1 * E + e], f_clock);
            if constexpr (MIX) CH_STS(&p.prev64[e], f_prev);
            // this step wrote the env's Euler cache and, unless obs were masked off, its whole obs block
            p.stale[e] = 0;
            if (wobs) p.stale[E + e] = 0;
            p.obs_tag[e] = wobs ? (unsigned long long)(uintptr_t)p.obs : 0ull;
        }
    } else {
        // ============ cow waves ================================================================
        const float rM = 1.0f / (float)M;
        const int nf = ei[NF_AT];
        const int* flist = ei + FL_LIST;
        const int lane = tid & 63;
        // a cow wave on the drone wave's SIMD takes no chunks before the drone hand-off (phase-mask bit 256: it
        // does) and, with bit 128, none after it either: a chunk it holds finishes late, as the prioritised drone
        // wave wins the SIMD's issue.  Before the hand-off that was the last cheap-pass chunk the F_C barrier
        // waited for (workgroup max 45.7-46.8 k -> 43.2-43.9 k cycles, profiles/r03/q)
        const bool co = co_simd && W1 >= 4;   // the other cow waves (>= 2 of them) take the work
#ifdef CH_CO_PRE_TAKE
        const bool skip_pre = co && (p.phase_mask & 256);
#else
        // (the per-wave-table path keeps the co-SIMD wave on its pre-hand-off work: C5 measured 140.8 -> 134.3 M
        // env-steps/s without it, profiles/r03/q)
        const bool skip_pre = co && (PW ? (p.phase_mask & 256) != 0 : !(p.phase_mask & 256));
#endif
        const bool skip_post = co && (p.phase_mask & 128);
        bool skip_now = skip_pre;
        // PW: this wave's env slot and queue, the env (flock-list index) it holds, the next cheap-pass
        // chunk, and the queue length / position of the expensive pass
        R* tb = nullptr;
        uint8_t* tf = nullptr;
        uint16_t* qu = nullptr;
        int f_cur = -1, ch = 0, qn = 0, qd = 0;
        const int NCH = (P + 63) >> 6;
        // PW with a compile-time herd: this lane's pair words (i | j << 8) of every 64-pair chunk, read from the
        // staged pair list once (pairs past P repeat pair 0, whose test is masked out by r < P)
        constexpr int NCHC = MT > 0 ? (MT * (MT - 1) / 2 + 63) / 64 : 1;
        uint32_t prw[NCHC];
#pragma unroll
        for (int c = 0; c < NCHC; ++c) {
            const int r = 64 * c + (tid & 63);
            prw[c] = (PW && MT > 0) ? S.pl[r < P ? r : 0] : 0u;
        }
        // one unit of PW alpha work (a cheap-pass chunk or an expensive-pass wave of queued pairs, plus the
        // env's rows after its last unit); false when no flocking env is left.  The state is wave-uniform
        // (grab is readfirstlane'd, the queue length a ballot count).
        // sep: one of a cow's two inputs to its velocity update is complete -- its alpha row (aux, auy) or its
        // shepherd sum (td[u], td[GM + u]); the second arrival runs the update
        // late: the second input computes the new velocity into LDS (nv) and marks it ready (+8); the final pass
        // after the reset list arrives with +4; whichever of the two comes last stores the velocity -- the new
        // episode's draw for a fast-reset env
        R* const nv = S.td + 2 * G * M;
        // spawn position component c of cow j in env g's next episode (scenario index + 1, BaseAviary.py:600-606), f64
        auto spawn_d = [&](int g, int j, int c) -> double {
            int sp = ei[I_SPAWN * G + g] + 1;
            if (sp >= p.n_scen) sp = 0;
            return p.spawn[((long long)sp * p.n_cows + j) * 2 + c];
        };
        auto store_final = [&](int u) {
            const int g = qdiv(u, M, 1.0f / (float)M);
            const long long ci = (long long)e0 * M + u;
            R vx = nv[u], vy = nv[G * M + u];
            if (fast && ei[I_RESET * G + g])
                reset_cow_vel(p, ci, p.env_off + e0 + g, u - g * M, (uint32_t)ei[I_EPISODE * G + g], vx, vy);
            CH_STS(&p.cattle[2 * CS + ci], vx); CH_STS(&p.cattle[3 * CS + ci], vy);
        };
        auto arrive = [&](int u) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            const int old = __hip_atomic_fetch_add(&S.cnt[u], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if ((old & 3) == 1) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                if (!late) {
                    velocity_update(p, S, M, e0, u, S.td[u], S.td[G * M + u]);
                } else {
                    velocity_update(p, S, M, e0, u, S.td[u], S.td[G * M + u], nv, G * M);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                    const int o2 = __hip_atomic_fetch_add(&S.cnt[u], 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (o2 & 4) store_final(u);
                }
            }
        };
        auto arrive_final = [&](int u) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            const int old = __hip_atomic_fetch_add(&S.cnt[u], 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old & 8) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                store_final(u);
            }
        };
        auto alpha_step = [&]() -> bool {
            if (f_cur < 0) {
                f_cur = grab(fl + C_PAIRS, 1, skip_now);
                ch = 0; qn = 0; qd = 0;
            }
            if (f_cur >= nf) return false;
            CHUNK_T0;
            const int g = flist[f_cur];
            if (ch < NCH) {
#ifndef CH_NO_BATCHED_CHEAP
                if constexpr (PW && MT > 0) alpha_cheap_pw_b<R, NCHC>(S, M, P, g, qu, qn, prw);
                else alpha_cheap_pw(S, M, P, g, qu, qn);
#else
                alpha_cheap_pw(S, M, P, g, qu, qn);
#endif
                ch = NCH;
                wave_sync();   // the queue
            } else if (qd < qn) {
                alpha_full_pw(S, M, P, g, qd, qn, tb, qu);
                qd += 64;
            }
            if (ch == NCH && qd >= qn) {
                wave_sync();   // every table entry of the env
                for (int j = lane; j < M; j += 64) alpha_row_pw(S, M, P, g, j, tb);
                wave_sync();   // the slot is free again
                if constexpr (PW_READY) lds_signal(reinterpret_cast<int*>(S.hasnb) + f_cur);   // the env's rows are in
                f_cur = -1;
            }
            CHUNK_T1(0);
            return true;
        };
        if constexpr (PW) {
            tb = S.tgx + (size_t)(tid / 64 - 1) * L.slot;
            tf = S.tdf + (size_t)(tid / 64 - 1) * M * N;
            qu = S.queue + (size_t)(tid / 64 - 1) * P;
        } else {
            alpha_cheap(S, fl, M, P, nf, flist, skip_pre);
            if (ct == 0) TS(38, (long long)clock64());
            lds_signal(fl + F_C);
#ifdef CH_NO_STREAM_FULL
            lds_wait(fl + F_C, W1, p.err);   // the queue is complete
#endif
            if (ct == 0) { TS(39, (long long)clock64()); TS(29, (long long)lds_peek(fl + Q_LEN)); }
            alpha_full(S, fl, M, P, skip_pre, W1, p.err);
        }
        if (ct == 0) TS(18, (long long)clock64());
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int u = ct + k * CW;
            if (u < Gv * M) { S.spx[u] = spx_r[k]; S.spy[u] = spy_r[k]; }
        }
        // the constant-zero bytes of the observation blocks, when the host cannot vouch that this buffer
        // already holds them (first step into a buffer, after ch_set_state, ...; ch_api.cpp obs_zero_ptr)
        if (wobs)
            for (int g = 0; g < Gv; ++g)
                if (p.obs_full || ei[I_OBSD * G + g]) obs_zero_env(obs_wg + g * RW, ei[I_N * G + g], rows, cat_off, m_obs, ct, CW);
        if constexpr (PW) {
            // whole envs' alpha tables and rows, one env per wave at a time, until the drone positions arrive
            while (lds_peek(fl + F_D) < 1 && alpha_step()) {
            }
        } else {
            lds_signal(fl + F_A);
            // alpha rows while the drone wave still integrates: once every pair is in the table, row chunks
            // are taken until the drone positions arrive; the rest follows the drone hand-off below
            int sleeps = 0;
            for (int spins = 0; spins < (1 << 22); ++spins) {
                if (lds_peek(fl + F_D) >= 1) break;
                if (lds_peek(fl + F_A) < W1) { __builtin_amdgcn_s_sleep(1); ++sleeps; continue; }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");   // the pair table
                const int b = grab(fl + C_ROWS, 64, skip_pre), u = b + lane;
                if (b >= nf * M) break;
                CHUNK_T0;
                if (u < nf * M) {
                    const int f = qdiv(u, M, rM), g = flist[f], j = u - f * M;
                    alpha_row(S, M, P, g * M + j, g, j);
                    if (sep) arrive(g * M + j);
                }
                CHUNK_T1(2);
            }
            spin_note(sleeps);
        }
        if (ct == 0) TS(8, (long long)clock64());
        lds_wait(fl + F_D, 1, p.err);
        if (ct == 0) TS(9, (long long)clock64());
        skip_now = skip_post;
        for (;;) {   // per cow: distances, winding number, observation entries (the herd centroid is done)
            const int b = grab(fl + C_COWS, 64, skip_post), u = b + lane;
            if (b >= Gv * M) break;
            CHUNK_T0;
            if (u < Gv * M) {
            const int g = qdiv(u, M, rM), j = u - g * M;
            const int n = ei[I_N * G + g], b0 = g * N;
            const R qix = S.cx[u], qiy = S.cy[u];
            CH_UNROLL for (int k = 0; k < N; ++k) {
                if (k >= n) break;   // |y_k - q_j| for the shepherd term and the closest-cow search
                const R ex = S.dx[b0 + k] - qix, ey = S.dy[b0 + k] - qiy;
                S.dcow[(b0 + k) * M + j] = ex * ex + ey * ey;
            }
            if (task) {
                // evaluate_herding_effectiveness winding number (evaluation.py:100-138)
                int wn = 0;
                CH_UNROLL for (int i = 0; i < N; ++i) {
                    if (i >= n) break;
                    int i2 = (i + 1 == n) ? 0 : i + 1;
                    R x1 = S.dx[b0 + i], y1 = S.dy[b0 + i], x2 = S.dx[b0 + i2], y2 = S.dy[b0 + i2];
                    R il = (x2 - x1) * (qiy - y1) - (qix - x1) * (y2 - y1);
                    if (y1 <= qiy) { if (y2 > qiy && il > R(0)) wn += 1; }
                    else { if (y2 <= qiy && il < R(0)) wn -= 1; }
                }
                if (wn != 0) atomicAdd(&ei[I_HERD * G + g], 1);
            }
            if (j < m_obs && wobs && !late) obs_cattle(obs_wg + g * RW, S.dxd, S.dyd, b0, j, n, cat_off, S.cxd[u], S.cyd[u]);
            }
            // H counts finished items, so a wave still busy with an alpha chunk does not hold the drone wave up
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            if (lane == 0) __hip_atomic_fetch_add(fl + F_H, min(64, Gv * M - b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            CHUNK_T1(1);
        }
        const float rN = 1.0f / (float)N;
        if constexpr (SPLIT) {
            // the drones' spacing terms (from the drone wave's nearest-neighbour distances, signal T) and cattle
            // terms (from the distance table, complete at H); each finished item counts towards F_S
            for (int pass = 0; pass < 2; ++pass) {
                for (;;) {
                    const int b = grab(fl + (pass ? C_SCAT : C_SPC), 64, skip_post), u = b + lane;
                    if (b >= Gv * N) break;
                    if (pass) lds_wait(fl + F_H, Gv * M, p.err);
                    else lds_wait(fl + F_T, 1, p.err);
                    if (u < Gv * N && task) {
                        const int g = qdiv(u, N, rN), k = u - g * N;
                        if (k < ei[I_N * G + g]) {
                            if (pass) S.scat[u] = cattle_term(S, u, M, R(p.cs_cc));
                            else spacing_terms(S, LT[ei[I_LEVEL * G + g]], p.compat != 0, u, S.pa[u], S.pb[u]);
                        }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                    if (lane == 0) __hip_atomic_fetch_add(fl + F_S, min(64, Gv * N - b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        }
        // getEulerFromQuaternion of the new attitudes (BaseAviary.py:704-766): the own row's roll, pitch, yaw and
        // the next step's PID input (the Euler cache); late: after the reset list, skipping fast-reset envs
        auto euler_pass = [&]() {
          // one item per (angle, drone): 3 G N items, so three waves share a workgroup's transcendentals
          for (;;) {
            const int b = grab(fl + C_EULER, 64, skip_post), t = b + lane;
            if (b >= 3 * Gv * N) break;
            if (t < 3 * Gv * N) {
                const int c = t >= Gv * N ? (t >= 2 * Gv * N ? 2 : 1) : 0, u = t - c * Gv * N;
                const int g = qdiv(u, N, rN), k = u - g * N;
                const bool rsf = fast && ei[I_RESET * G + g];   // (its cache and observation: the new episode's)
                if (k < ei[I_N * G + g] && (!rsf || (tobs && wobs))) {
                    const int GN = G * N;
                    const R qq[4] = {S.dq[u], S.dq[GN + u], S.dq[2 * GN + u], S.dq[3 * GN + u]};
                    const R r = quat_to_euler_c(qq, c);
                    const long long dd = (long long)e0 * N + u;
                    if (!rsf) {
                        CH_STS(&p.rpy[c * DS + dd], r);
                        if (wobs) CH_ST(obs_wg + g * RW + k * 86 + 1 + c, (float)r);
                    } else {
                        CH_ST(p.terminal_obs + (long long)(e0 + g) * RW + k * 86 + 1 + c, (float)r);   // the terminal observation's
                    }
                }
            }
          }
        };
        if (!late) euler_pass();
        if constexpr (PW) {
            while (alpha_step()) {   // the rest of the alpha work (the current env first)
            }
            // PW_READY: no cow-wave barrier here -- each env's shepherd sums and velocity update wait only for that env's
            // alpha rows (its ready flag), so the waves that run out of alpha work take the envs that are done while the
            // last envs' alpha work finishes (the velocity update reads the env's own positions, velocities and rows only)
            if constexpr (!PW_READY) cow_sync(fl + F_W, W1, false, p.err);   // every alpha row (aux, auy) is written
            if (ct == 0) TS(21, (long long)clock64());
            // shepherd / predator sums and the velocity update, one cow per lane with its drones' terms in
            // registers (shepherd_sum, drone order), 64 / M flocking envs per wave at a time
            const int per = M <= 64 ? 64 / M : 1;
            for (;;) {
                const int f0 = grab(fl + C_DELTA, per, skip_post);
                if (f0 >= nf) break;
                if constexpr (PW_READY) {
                    for (int fi = 0; fi < per && f0 + fi < nf; ++fi) lds_wait(reinterpret_cast<int*>(S.hasnb) + f0 + fi, 1, p.err);
                }
                CHUNK_T0;
                for (int q = lane; q < per * M; q += 64) {
                    const int fi = per > 1 ? qdiv(q, M, rM) : 0, j = q - fi * M, f = f0 + fi;
                    if (f < nf) {
                        const int g = flist[f], u = g * M + j;
                        R ddx, ddy;
                        shepherd_sum<R, NT>(S, N, u, g, ei[I_N * G + g], ddx, ddy);
                        velocity_update(p, S, M, e0, u, ddx, ddy);
                    }
                }
                CHUNK_T1(3);
            }
            if (ct == 0) TS(16, (long long)clock64());
        } else {
        if (sep) {
            // The alpha rows that remain first (the longest chunks: started last they would end last), then the
            // shepherd/predator (cow, drone) items; each cow's velocity update runs as soon as its row and its N
            // terms are in, whichever arrives last
            lds_wait(fl + F_A, W1, p.err);   // every pair of the table
            if (ct == 0) TS(20, (long long)clock64());
            for (;;) {
                const int b = grab(fl + C_ROWS, 64, skip_post), u = b + lane;
                if (b >= nf * M) break;
                CHUNK_T0;
                if (u < nf * M) {
                    const int f = qdiv(u, M, rM), g = flist[f], j = u - f * M;
                    alpha_row(S, M, P, g * M + j, g, j);
                    arrive(g * M + j);
                }
                CHUNK_T1(2);
            }
            if (ct == 0) TS(21, (long long)clock64());
            // shepherd/predator sums, one cow of a flocking env per lane with its drones' terms in registers
            for (;;) {
                const int b = grab(fl + C_DELTA, 64, skip_post), u = b + lane;
                if (b >= nf * M) break;
                CHUNK_T0;
                if (u < nf * M) {
                    const int f = qdiv(u, M, rM), g = flist[f], j = u - f * M, uc = g * M + j;
                    R ddx, ddy;
                    shepherd_sum<R, NT>(S, N, uc, g, ei[I_N * G + g], ddx, ddy);
                    S.td[uc] = ddx; S.td[G * M + uc] = ddy;
                    arrive(uc);
                }
                CHUNK_T1(3);
            }
            if (ct == 0) TS(16, (long long)clock64());
        } else {
        // the alpha rows only feed the velocity update: they wait until the drone wave has its hand-off
            lds_wait(fl + F_A, W1, p.err);   // every pair of the table
            if (ct == 0) TS(20, (long long)clock64());
            for (;;) {   // alpha rows of the cows of flocking envs
                const int b = grab(fl + C_ROWS, 64, skip_post), u = b + lane;
                if (b >= nf * M) break;
                CHUNK_T0;
                if (u < nf * M) {
                    const int f = qdiv(u, M, rM), g = flist[f], j = u - f * M;
                    alpha_row(S, M, P, g * M + j, g, j);
                }
                CHUNK_T1(2);
            }
            cow_sync(fl + F_W, W1, false, p.err);   // every alpha row read the pair table: its space now takes the drone terms
            if (ct == 0) TS(21, (long long)clock64());
            const int T = G * M * N, MN = M * N;
            const float rMN = 1.0f / (float)MN;
            // (cow, drone) items of flocking envs: shepherd and predator terms.  A chunk of 64 items holds
            // whole cows when N divides 64 (the cow's N items are consecutive): the wave that computed a cow's
            // terms then finishes that cow's velocity update itself (lane k = 0), with no workgroup sync.
            const bool fuse = (64 % N) == 0;
            for (;;) {
                const int b = grab(fl + C_DELTA, 64, skip_post), q = b + lane;
                if (b >= nf * MN) break;
                CHUNK_T0;
                int f = 0, j = 0, k = 0, g = 0, n = 0;
                const bool valid = q < nf * MN;
                if (valid) {
                    f = qdiv(q, MN, rMN);
                    const int rem = q - f * MN;
                    j = qdiv(rem, N, rN); k = rem - j * N;
                    g = flist[f]; n = ei[I_N * G + g];
                    if (k < n) delta_term(S, N, g * M + j, g, k, S.td, S.tdf, (g * M + j) * N + k, T);
                }
                if (fuse) {
                    wave_sync();   // the cow's terms, written by other lanes of this wave
                    if (valid && k == 0) flock_combine(p, S, N, M, e0, g * M + j, n, S.td, S.tdf, (g * M + j) * N, T);
                }
                CHUNK_T1(3);
            }
            if (ct == 0) TS(16, (long long)clock64());
            if (!fuse) {
                cow_sync(fl + F_Q, W1, false, p.err);   // every drone term of every cow
                if (ct == 0) TS(17, (long long)clock64());
                for (;;) {   // cows of flocking envs only
                    const int b = grab(fl + C_FLOCK, 64, skip_post), u = b + lane;
                    if (b >= nf * M) break;
                    CHUNK_T0;
                    if (u < nf * M) {
                        const int f = qdiv(u, M, rM), g = flist[f], j = u - f * M;
                        flock_combine(p, S, N, M, e0, g * M + j, ei[I_N * G + g], S.td, S.tdf, (g * M + j) * N, T);
                    }
                    CHUNK_T1(4);
                }
            }
            }
        }
        if (lane == 0) TS(40 + (tid >> 6), (long long)clock64());   // this cow wave's flock work done
        TS_MAX(57);
        if (ct == 0) TS(31, (long long)nf);
        lds_wait(fl + F_R, 1, p.err);    // the reset list
        if (tid == 64) TS(37, (long long)clock64());
        const int nr = ei[NR_AT];
        if (ct == 0) TS(30, (long long)nr);
        if (nr && ct == 0) TS(52, (long long)clock64());
        TS_MAX(56);
        if (late) {
            // the Euler items (one chunk) go to the first wave that holds no cow of the final pass, so that their
            // stream overlaps the final pass; a wave with final-pass cows takes them only after its own cows (when
            // every other wave is still busy with flock work)
#ifdef CH_EULER_ANYWAVE
            const bool ew = true;
#else
            const bool ew = Gv * M > CW - 64 || ct - lane >= Gv * M;
#endif
            if (ew) euler_pass();
            TS_MAX(58);
            // final pass, each cow on its phase-0 lane: cattle observation entries (of the new episode for a
            // fast-reset env, whose new positions and velocities this lane writes too), then the flocking envs'
            // third arrival
            for (int u = ct; u < Gv * M; u += CW) {
                const int g = qdiv(u, M, rM), j = u - g * M;
                const bool rs_ = fast && ei[I_RESET * G + g];
                const int n_old = ei[I_N * G + g];
                const long long ci = (long long)e0 * M + u;
                if (rs_) {
                    if (tobs && wobs && j < m_obs)   // the terminal observation's entries, from this step's positions
                        obs_cattle(p.terminal_obs + (long long)(e0 + g) * RW, S.dxd, S.dyd, g * N, j, n_old, cat_off,
                                   S.cxd[u], S.cyd[u]);
                    // the new episode's spawn position (prefetched in LDS; in f32 mode re-read in f64 from the table)
                    const double x = MIX ? spawn_d(g, j, 0) : (double)S.spx[u], y = MIX ? spawn_d(g, j, 1) : (double)S.spy[u];
                    p.cattle[0 * CS + ci] = R(x); p.cattle[1 * CS + ci] = R(y);
                    if constexpr (MIX) { p.cpos64[ci] = x; p.cpos64[CS + ci] = y; }
                    if (!ei[I_FLOCK * G + g]) {   // no flock update: the velocity is written here
                        R vx, vy;
                        reset_cow_vel(p, ci, p.env_off + e0 + g, j, (uint32_t)ei[I_EPISODE * G + g], vx, vy);
                        p.cattle[2 * CS + ci] = vx; p.cattle[3 * CS + ci] = vy;
                    }
                    if (wobs && j < m_obs) {
                        const int n_new = ei[I_NEWN * G + g];
                        float* eb = obs_wg + g * RW;
                        for (int r = 0; r < N; ++r) {
                            if (r >= n_new && r >= n_old) break;
                            if (r < n_new) {
                                double dx, dy, dz;
                                reset_drone_xyz(r, n_new, dx, dy, dz);
                                st2(eb, r * 86 + cat_off + 2 * j, (float)(x - dx), (float)(y - dy));
                            } else {
                                st2(eb, r * 86 + cat_off + 2 * j, 0.0f, 0.0f);
                            }
                        }
                    }
                } else if (wobs && j < m_obs) {
                    obs_cattle(obs_wg + g * RW, S.dxd, S.dyd, g * N, j, n_old, cat_off, S.cxd[u], S.cyd[u]);
                }
                if (ei[I_FLOCK * G + g]) arrive_final(u);
            }
            if (!ew) euler_pass();
            if (tobs && wobs)   // the terminal observations' constant bytes (no producer writes them)
                for (int k = 0; k < nr; ++k) {
                    const int g = ei[RS_LIST + k];
                    obs_zero_env(p.terminal_obs + (long long)(e0 + g) * RW, ei[I_N * G + g], rows, cat_off, m_obs, ct, CW);
                }
            TS_MAX(60);
        }
        if (nr && !fast) {   // uniform across the cow waves
            // ---- SB3 auto-reset of the listed envs (BaseAviary.reset, BaseAviary.py:280-331), rebuilt from
            // the pre-step scalars (NUM_DRONES draw, spawn index + 1, episode) while the drone wave still
            // computes rewards: the terminal observation (on request), then the bodies and observation rows.
            const int* rl = ei + RS_LIST;
            if (nr && p.terminal_obs) {   // info["terminal_observation"]: the pre-reset observation, from HBM
                cow_sync(fl + F_X0, W1, true, p.err);   // every cow wave's observation stores of this step are visible
                for (int q = ct; q < nr * (RW >> 1); q += CW) {
                    const int k = q / (RW >> 1), o = rl[k] * (RW >> 1) + (q - k * (RW >> 1));
                    reinterpret_cast<float2*>(p.terminal_obs + (long long)e0 * RW)[o] = reinterpret_cast<const float2*>(obs_wg)[o];
                }
            }
            // The new episode's bodies are computed before the sync (into registers, the new drone positions also
            // into LDS rd*), so the sync's wait for the slowest cow wave hides that latency; after it only the stores
            // remain.  The reset envs' drones go to the first cow wave, their cattle to the others (concurrently).
            const int dl = W1 >= 2 ? 64 : CW, c0l = W1 >= 2 ? 64 : 0, cl = CW - c0l;
            // drones: one per lane of the first cow wave (nr * N <= G * N <= 64 <= dl)
            const bool dit = ct < dl && ct < nr * N;
            double rx = 0, ry = 0, rz = 0;
            if (dit) {
                const int k0 = qdiv(ct, N, rN), g = rl[k0], k = ct - k0 * N, ud = g * N + k;
                const int n = reset_draw_n(p, ei[I_EPISODE * G + g], p.env_off + e0 + g);
                if (k == 0) ei[I_NEWN * G + g] = n;
                reset_drone_xyz(k, n, rx, ry, rz);
                S.rdx[ud] = R(rx); S.rdy[ud] = R(ry); S.rdz[ud] = R(rz);
            }
            // cattle: the first two per lane in registers (the rest, beyond 2 cl, after the sync)
            constexpr int RI = 2;
            R cvx_r[RI], cvy_r[RI];
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                const int u = ct - c0l + i * cl;
                cvx_r[i] = cvy_r[i] = 0;
                if (ct >= c0l && u < nr * M) {
                    const int k0 = qdiv(u, M, rM), g = rl[k0], j = u - k0 * M, uc = g * M + j;
                    reset_cow_vel(p, (long long)e0 * M + uc, p.env_off + e0 + g, j, (uint32_t)ei[I_EPISODE * G + g],
                                  cvx_r[i], cvy_r[i]);
                }
            }
            if (ct == 0) TS(55, (long long)clock64());
            cow_sync(fl + F_X1, W1, true, p.err);   // terminal observation read; this step's stores done; rd* and NEWN seen
            if (ct == 0) TS(53, (long long)clock64());
            if (dit) {
                const int k0 = qdiv(ct, N, rN), g = rl[k0], k = ct - k0 * N, ud = g * N + k;
                const int n = ei[I_NEWN * G + g];
                const long long dd = (long long)e0 * N + ud;
                reset_drone_store(p, dd, rx, ry, rz);
                if constexpr (PHYS) {   // last_clipped_action, rpy_rates = 0 (_housekeeping, BaseAviary.py:565, 581-582)
#pragma unroll
                    for (int c = 0; c < kPhysComps; ++c) CH_STS(&p.phys[c * DS + dd], R(0));
                }
                // identity attitude: Euler angles (+0, -0, +0) for the next step's cache
                CH_STS(&p.rpy[dd], R(0)); CH_STS(&p.rpy[DS + dd], -R(0)); CH_STS(&p.rpy[2 * DS + dd], R(0));
                if (wobs) {
                    float* eb = obs_wg + g * RW;
                    if (k < n) {
                        // identity quaternion: getEulerFromQuaternion gives atan2(+0, 1), asin(-2 * (+0)), atan2(+0, 1)
                        // = (+0, -0, +0) (quat_to_euler); zero velocities
                        const R zero3[3] = {0, 0, 0}, rpy0[3] = {R(0), -R(0), R(0)};
                        obs_own(eb, k, R(rz), rpy0, zero3, zero3);
                        const int nb = nearest_two(S.rdx, S.rdy, g * N, k, n);
                        obs_nbr(eb, S.rdx, S.rdy, g * N, k, (nb & 0xff) - 1, (nb >> 8) - 1);
                    } else if (k < ei[I_N * G + g]) {
                        // a row the old episode used and the new one does not (rows >= the old NUM_DRONES are zero)
                        for (int c = 0; c < 86; c += 2) st2(eb, k * 86 + c, 0.0f, 0.0f);
                    }
                }
            }
            if (ct >= c0l)
                for (int u = ct - c0l, i = 0; u < nr * M; u += cl, ++i) {
                    const int k0 = qdiv(u, M, rM), g = rl[k0], j = u - k0 * M, uc = g * M + j;
                    R vx = i == 0 ? cvx_r[0] : cvx_r[1], vy = i == 0 ? cvy_r[0] : cvy_r[1];
                    if (i >= RI)
                        reset_cow_vel(p, (long long)e0 * M + uc, p.env_off + e0 + g, j, (uint32_t)ei[I_EPISODE * G + g], vx, vy);
                    const double x = MIX ? spawn_d(g, j, 0) : (double)S.spx[uc], y = MIX ? spawn_d(g, j, 1) : (double)S.spy[uc];
                    reset_cow_store(p, (long long)e0 * M + uc, x, y, vx, vy);
                    if (wobs && j < m_obs) obs_cattle(obs_wg + g * RW, S.rdx, S.rdy, g * N, j, ei[I_NEWN * G + g], cat_off, x, y);
                }
            if (ct == 0) TS(54, (long long)clock64());
        }
    }
    if (tid == 0) TS(35, (long long)clock64());
    if (tid == 64) TS(36, (long long)clock64());
    if (tid >= 64) TS_MAX(63);   // diagnostics: the last cow wave's end
    // No closing barrier: every wave leaves when its own work is done (the LDS lives until the last one
    // has).  With timestamps on, one barrier marks the workgroup's end for the trace.
    if (p.tstamp) {
        lds_barrier();
        if (tid == 0) { TS(13, (long long)clock64()); TS(14, (long long)clock64()); TS(1, (long long)wall_clock64()); }
    }
}

#ifndef CH_STEP_BODY_ONLY   // (ch_step_multi.hip includes this file for step2_body alone)
template <class R, int MODE, int GT, int NT, int MT, bool PHYS = false, bool PW = false, bool TOBS = false>
__global__ __launch_bounds__((PW || PHYS) ? CH_V2_MAX_BLOCK_PW : CH_V2_MAX_BLOCK)
__attribute__((amdgpu_waves_per_eu((sizeof(R) == 4 && GT > 0 && !PW && !PHYS) ? 4 : 1)))
void k_step2(StepParams<R> p) {
    step2_body<R, MODE, GT, NT, MT, PHYS, PW, TOBS>(p);
}

// The PPO collection step with the actor forward of the next step fused in (ch_rollout_collect, CH_FUSED_ACTOR /
// ch__set_rollout_path bit 2): the workgroup steps its 16 envs, then -- once every wave has written its observation
// stores -- runs the SB3 actor (k_mlp2's body, one 16-row tile, 12 waves of which 8 carry the 128-wide layers' column
// tiles) on the 16 observation rows it has just written, with the sampling epilogue (kRoleSample: actions,
// log-probabilities, the next step's env actions).  The rows are read back through the CU's caches (the stores of
// this workgroup; a workgroup-scope release before the barrier, a workgroup-scope acquire after it),
// the weights stream from L2 as in the separate launch; the LDS of the step is dead by then and the forward's tile
// reuses it.  The critic and its value epilogue stay a separate launch.  Same arithmetic as the separate forward
// (the K order of each output does not depend on the wave count): bit-identical rollouts.
constexpr int kFusedLdsMax = 160 * 1024 - 256;   // k_step2_actor's dynamic LDS cap
struct FusedActor {
    MlpArgs a;
    RolloutArgs ro;
    int lda, ldh;
};
template <class R, int MODE, int GT, int NT, int MT, bool TOBS>
__global__ __launch_bounds__(CH_V2_MAX_BLOCK)
void k_step2_actor(StepParams<R> p, FusedActor f) {
    // diagnostics (ch__set_mlp_tstamp): wall clocks of the workgroup's start, barrier and end in slots 13-15
    long long* ts = f.a.tstamp && threadIdx.x == 0 ? f.a.tstamp + (long long)blockIdx.x * 16 : nullptr;
    if (ts) ts[13] = (long long)wall_clock64();
    step2_body<R, MODE, GT, NT, MT, false, false, TOBS>(p);
    // workgroup scope both ways: the waves of a workgroup share the CU's vector L1, so the release's store-counter
    // wait makes every observation store visible to the forward's loads after the barrier (an agent-scope acquire
    // would also invalidate this XCD's L2 -- measured: the forward's first weight loads then waited ~17 us)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    __builtin_amdgcn_s_setprio(0);   // (the drone wave's raised priority)
    if (ts) ts[14] = (long long)wall_clock64();
    mlp2_body<CH_V2_MAX_BLOCK / 64, 1, 1>(f.a, (long long)blockIdx.x, f.lda, f.ldh, kRoleSample, f.ro);
    if (ts) ts[15] = (long long)wall_clock64();
}

template <class R, int MODE, int GT, int NT, int MT, bool PHYS = false, bool PW = false, bool TOBS = false>
static hipError_t launch_v2_kernel(const StepParams<R>& p, int block, size_t lds, hipStream_t st, bool launch) {
    // opt-in to > 64 KiB of dynamic LDS, once per device (the attribute is per device context)
    static std::atomic<unsigned long long> attr_set{0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (!(attr_set.load(std::memory_order_relaxed) & bit)) {
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_step2<R, MODE, GT, NT, MT, PHYS, PW, TOBS>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set.fetch_or(bit, std::memory_order_relaxed);
    }
    if (!launch) return hipSuccess;
    dim3 grid((p.E + p.G - 1) / p.G);
    hipLaunchKernelGGL((k_step2<R, MODE, GT, NT, MT, PHYS, PW, TOBS>), grid, dim3(block), lds, st, p);
    return hipGetLastError();
}

// geometry specialisations: the BASELINE configs at their default geometry (ch_api.cpp)
template <class R>
hipError_t launch_step_v2(const StepParams<R>& p, int block, size_t lds, hipStream_t st, bool launch) {
    const int G = p.G, N = p.NC, M = p.M;
    if (p.physics != CH_PHYS_PYB) {   // physics variants (BaseAviary.py:420-450): runtime-geometry instantiation
        if (p.mode == 1) return launch_v2_kernel<R, 1, 0, 0, 0, true>(p, block, lds, st, launch);
        if (G == 16 && N == 4 && M == 16) return launch_v2_kernel<R, 0, 16, 4, 16, true>(p, block, lds, st, launch);   // configs[3]
        return launch_v2_kernel<R, 0, 0, 0, 0, true>(p, block, lds, st, launch);
    }
    if (p.pw) {   // per-wave env tables (herds > 16 cows)
        if (p.mode == 1 && G == 16 && N == 4 && M == 32)
            return launch_v2_kernel<R, 1, 16, 4, 32, false, true>(p, block, lds, st, launch);   // configs[4]
        if (p.mode == 1) return launch_v2_kernel<R, 1, 0, 0, 0, false, true>(p, block, lds, st, launch);
        return launch_v2_kernel<R, 0, 0, 0, 0, false, true>(p, block, lds, st, launch);
    }
    if (p.mode == 1) return launch_v2_kernel<R, 1, 0, 0, 0>(p, block, lds, st, launch);
    if (G == 8 && N == 4 && M == 16) return launch_v2_kernel<R, 0, 8, 4, 16>(p, block, lds, st, launch);          // configs[3]
    if (G == 16 && N == 4 && M == 16) {   // configs[3]: terminal observations from their producers (TOBS) when asked for
        if (!launch) {   // (both instantiations' attribute opt-in at ch_create)
            const hipError_t e = launch_v2_kernel<R, 0, 16, 4, 16, false, false, true>(p, block, lds, st, false);
            if (e != hipSuccess) return e;
        }
        if (p.terminal_obs) return launch_v2_kernel<R, 0, 16, 4, 16, false, false, true>(p, block, lds, st, launch);
        return launch_v2_kernel<R, 0, 16, 4, 16>(p, block, lds, st, launch);
    }
    if (G == 16 && N == 2 && M == 8) return launch_v2_kernel<R, 0, 16, 2, 8>(p, block, lds, st, launch);          // configs[2]
    if (G == 4 && N == 2 && M == 8) return launch_v2_kernel<R, 0, 4, 2, 8>(p, block, lds, st, launch);            // configs[1]
    return launch_v2_kernel<R, 0, 0, 0, 0>(p, block, lds, st, launch);
}

template <class R, bool TOBS>
static hipError_t launch_actor_kernel(const StepParams<R>& p, int block, size_t lds, hipStream_t st, const FusedActor& f,
                                      bool launch) {
    static std::atomic<unsigned long long> attr_set{0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (!(attr_set.load(std::memory_order_relaxed) & bit)) {
        // (the forward's static words -- kmax, kany, the row slots -- sit beside the dynamic LDS)
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_step2_actor<R, 0, 16, 4, 16, TOBS>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, kFusedLdsMax);
        if (e != hipSuccess) { (void)hipGetLastError(); return e; }
        attr_set.fetch_or(bit, std::memory_order_relaxed);
    }
    if (!launch) return hipSuccess;
    hipLaunchKernelGGL((k_step2_actor<R, 0, 16, 4, 16, TOBS>), dim3((p.E + 15) / 16), dim3(block), lds, st, p, f);
    return hipGetLastError();
}

template <class R>
hipError_t launch_step_v2_actor(const StepParams<R>& p, int block, size_t lds, hipStream_t st, const MlpArgs& a,
                                const RolloutArgs& ro, bool launch) {
    if constexpr (sizeof(R) != sizeof(double)) {
        return hipErrorNotSupported;
    } else {
        if (p.physics != CH_PHYS_PYB || p.pw || p.mode != 0 || p.G != 16 || p.NC != 4 || p.M != 16 ||
            block != CH_V2_MAX_BLOCK || a.rows != p.E)
            return hipErrorNotSupported;
        FusedActor f;
        size_t mb = 0;
        if (!mlp2_fused_tile(a, f.lda, f.ldh, mb)) return hipErrorNotSupported;
        f.a = a;
        // (diagnostics, ch__set_mlp_tstamp: the forward's phase clocks in the buffer's second half, rows [grid, 2 grid),
        // so that the separate launches of the same collection, which use the first, do not overwrite them)
        f.a.tstamp = g_mlp_tstamp ? g_mlp_tstamp + 16LL * ((p.E + 15) / 16) : nullptr;
        f.ro = ro;
        const size_t l = lds > mb ? lds : mb;
        if (l > (size_t)kFusedLdsMax) return hipErrorNotSupported;
        return p.terminal_obs ? launch_actor_kernel<R, true>(p, block, l, st, f, launch)
                              : launch_actor_kernel<R, false>(p, block, l, st, f, launch);
    }
}

#ifdef CH_COUNT_SPINS
// (diagnostic builds) read and clear the k_step2 spin counters: out[0..3] = drone-wave sleeps, cow-wave sleeps,
// drone-wave waits, cow-wave waits
extern "C" int ch__spin_counts(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ch_spins), sizeof(g_ch_spins)) != hipSuccess) return -1;
    const unsigned long long z[4] = {0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_ch_spins), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

template hipError_t launch_step_v2<double>(const StepParams<double>&, int, size_t, hipStream_t, bool);
template hipError_t launch_step_v2_actor<double>(const StepParams<double>&, int, size_t, hipStream_t, const MlpArgs&,
                                                 const RolloutArgs&, bool);
template hipError_t launch_step_v2_actor<float>(const StepParams<float>&, int, size_t, hipStream_t, const MlpArgs&,
                                                const RolloutArgs&, bool);
template hipError_t launch_step_v2<float>(const StepParams<float>&, int, size_t, hipStream_t, bool);

#endif   // CH_STEP_BODY_ONLY

}  // namespace ch
