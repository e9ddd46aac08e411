// ch_step_multi.hip — ch_step_n's kernel: n consecutive steps of a handle in one launch (k_step2_multi).
//
// The step is ch_step.hip's step2_body (included here for it alone).  This translation unit is compiled with machine
// LICM off (cattleherd/_build.py): with it, the step loop hoisted the body's loop-invariant values (LDS addresses,
// constants) to the loop preheader and held them across the whole step, and configs[3]'s instantiation spilled 80-145
// VGPRs; without it the body keeps k_step2's register allocation (173 VGPRs, no scratch).
#define CH_STEP_BODY_ONLY
#include "ch_step.hip"

namespace ch {

// n consecutive steps of the same io in one launch (ch_step_n): each workgroup steps its G envs n times back to back.
// The env groups are independent, so no workgroup waits for another between steps: the launch gap, the wait of every
// step on the grid's slowest workgroup, and the state loads' first-touch latency at workgroup start are paid once per
// launch instead of once per step.  Between two steps a workgroup-scope release (the step's global stores complete),
// s_barrier (every wave is done with the step's LDS) and a workgroup-scope acquire: the waves of a workgroup share the
// CU's vector L1, so the next step's loads see this step's stores (as k_step2_actor's forward does).  Every step is the
// full step2_body: the outputs, the auto-resets and the state are those of n ch_step calls (test_gpu_runtime.py).
// One step.  The parameters come from a device copy (ch_step_n uploads them before the launch): the pointer is made
// uniform (readfirstlane) and read through the constant address space, so every parameter read is a scalar load where
// the step uses it, as from k_step2's kernel arguments (the address of a by-value kernel argument would be a private
// copy).
template <class R, int MODE, int GT, int NT, int MT, bool PHYS, bool PW>
__device__ __forceinline__ void step2_once(const StepParams<R>* p, int salt) {
    const unsigned long long a = (unsigned long long)(uintptr_t)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    using KP = const __attribute__((address_space(4))) StepParams<R>*;
    const KP kp = (KP)(((unsigned long long)hi << 32) | lo);
    step2_body<R, MODE, GT, NT, MT, PHYS, PW, false>(*(const StepParams<R>*)kp, salt);
}
// n consecutive steps in one launch (ch_step_n); `pd`: the step's parameters in device memory
// WPE: the waves per SIMD the registers are allocated for (4: two workgroups per CU, for grids of more workgroups than
// CUs -- the f32 mode at 262 144 envs: 395.5 vs 294.4 M env-steps/s; at 4096 envs, one workgroup per CU, the register
// cap only spills: 261.9 vs 297.2 M, profiles/r06/ab/r6n_*)
#ifndef CH_MULTI_MAX_BLOCK
#define CH_MULTI_MAX_BLOCK CH_V2_MAX_BLOCK_PW   // 512 threads: 2 waves per SIMD (A/B)
#endif
template <class R, int MODE, int GT, int NT, int MT, bool PHYS = false, bool PW = false, int WPE = 1>
__global__ __launch_bounds__(PW ? CH_V2_MAX_BLOCK_PW : CH_MULTI_MAX_BLOCK)
__attribute__((amdgpu_waves_per_eu(WPE)))
void k_step2_multi(const StepParams<R>* __restrict__ pd, int n_steps) {
    for (int k = 0; k < n_steps; ++k) {
        int salt = 0;
        const StepParams<R>* q = pd;
        asm volatile("" : "+s"(salt), "+s"(q));   // an opaque 0 (step2_body's salt) and parameter pointer, per step
        step2_once<R, MODE, GT, NT, MT, PHYS, PW>(q, salt);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        __builtin_amdgcn_s_setprio(0);   // (the drone wave's raised priority)
    }
}

template <class R, int MODE, int GT, int NT, int MT, bool PHYS = false, bool PW = false, int WPE = 1>
static hipError_t launch_v2_multi_kernel(const StepParams<R>& p, const StepParams<R>* pd, int block, size_t lds,
                                         hipStream_t st, int n_steps, bool launch) {
    static std::atomic<unsigned long long> attr_set{0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const unsigned long long bit = 1ull << (dev & 63);
    if (!(attr_set.load(std::memory_order_relaxed) & bit)) {
        e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_step2_multi<R, MODE, GT, NT, MT, PHYS, PW, WPE>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_set.fetch_or(bit, std::memory_order_relaxed);
    }
    if (!launch) return hipSuccess;
    dim3 grid((p.E + p.G - 1) / p.G);
    // at most 8 waves: the step loop needs the registers of 2 waves per SIMD (at 3 per SIMD, 768 threads, the loop's
    // longer live ranges spilled); the cow waves share their work out dynamically, so the outputs do not depend on it
    hipLaunchKernelGGL((k_step2_multi<R, MODE, GT, NT, MT, PHYS, PW, WPE>), grid, dim3(block < (PW ? CH_V2_MAX_BLOCK_PW : CH_MULTI_MAX_BLOCK) ? block : (PW ? CH_V2_MAX_BLOCK_PW : CH_MULTI_MAX_BLOCK)),
                       lds, st, pd, n_steps);
    return hipGetLastError();
}

// ch_step_n's kernel for the BASELINE geometries (PYB, no terminal observations); hipErrorNotSupported elsewhere (the
// caller then launches ch_step n times)
template <class R>
hipError_t launch_step_v2_multi(const StepParams<R>& p, const StepParams<R>* pd, int block, size_t lds, hipStream_t st,
                                int n_steps, bool launch) {
    const int G = p.G, N = p.NC, M = p.M;
    if (p.physics != CH_PHYS_PYB || p.terminal_obs) return hipErrorNotSupported;
    if constexpr (sizeof(R) == sizeof(double)) {
        if (p.pw) {
            if (p.mode == 1 && G == 16 && N == 4 && M == 32)
                return launch_v2_multi_kernel<R, 1, 16, 4, 32, false, true>(p, pd, block, lds, st, n_steps, launch);   // configs[4]
            return hipErrorNotSupported;
        }
        if (p.mode != 0) return hipErrorNotSupported;
        if (G == 16 && N == 4 && M == 16) return launch_v2_multi_kernel<R, 0, 16, 4, 16>(p, pd, block, lds, st, n_steps, launch);   // configs[3]
        if (G == 8 && N == 4 && M == 16) return launch_v2_multi_kernel<R, 0, 8, 4, 16>(p, pd, block, lds, st, n_steps, launch);     // configs[3], 2 per CU
        if (G == 16 && N == 2 && M == 8) return launch_v2_multi_kernel<R, 0, 16, 2, 8>(p, pd, block, lds, st, n_steps, launch);     // configs[2]
        if (G == 4 && N == 2 && M == 8) return launch_v2_multi_kernel<R, 0, 4, 2, 8>(p, pd, block, lds, st, n_steps, launch);       // configs[1]
        return hipErrorNotSupported;
    } else {
        if (!p.pw && p.mode == 0 && G == 16 && N == 4 && M == 16) {
            // two workgroups per CU once the grid has them (more than 256 workgroups); attribute opt-in for both at
            // ch_create (launch == false)
            if (!launch) {
                const hipError_t e = launch_v2_multi_kernel<R, 0, 16, 4, 16, false, false, 4>(p, pd, block, lds, st, n_steps, false);
                if (e != hipSuccess) return e;
            }
            if ((p.E + G - 1) / G > 256)
                return launch_v2_multi_kernel<R, 0, 16, 4, 16, false, false, 4>(p, pd, block, lds, st, n_steps, launch);
            return launch_v2_multi_kernel<R, 0, 16, 4, 16>(p, pd, block, lds, st, n_steps, launch);
        }
        return hipErrorNotSupported;
    }
}


template hipError_t launch_step_v2_multi<double>(const StepParams<double>&, const StepParams<double>*, int, size_t,
                                                 hipStream_t, int, bool);
template hipError_t launch_step_v2_multi<float>(const StepParams<float>&, const StepParams<float>*, int, size_t,
                                                hipStream_t, int, bool);

}  // namespace ch
