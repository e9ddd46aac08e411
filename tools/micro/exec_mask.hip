// Microbenchmark: does a wave64 VALU instruction cost less when only the low 16/32 lanes are active?
// One workgroup of 64 threads per CU (one wave per SIMD at most), a long dependent chain per lane.
#include <hip/hip_runtime.h>
#include <cstdio>

template <class T>
__global__ void chain(T* out, int iters, int active, int dep) {
    T a = (T)threadIdx.x * (T)1e-3 + (T)1, b = (T)0.999999, c = (T)1e-7;
    T x0 = a, x1 = a + 1, x2 = a + 2, x3 = a + 3;
    if ((int)threadIdx.x < active) {
        if (dep) {
            for (int i = 0; i < iters; ++i) { x0 = x0 * b + c; x0 = x0 * b + c; x0 = x0 * b + c; x0 = x0 * b + c; }
        } else {
            for (int i = 0; i < iters; ++i) { x0 = x0 * b + c; x1 = x1 * b + c; x2 = x2 * b + c; x3 = x3 * b + c; }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}

template <class T>
__global__ void sincos_chain(T* out, int iters, int active) {
    T x = (T)threadIdx.x * (T)1e-3 + (T)0.1;
    if ((int)threadIdx.x < active)
        for (int i = 0; i < iters; ++i) x = sin(x) + cos(x) * (T)0.5;
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// 8 independent dependency chains, unrolled: the single-wave issue interval of the FMA
template <class T>
__global__ void ilp8(T* out, int iters) {
    T x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = (T)threadIdx.x * (T)1e-3 + (T)k;
    const T b = (T)0.999999, c = (T)1e-7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = __builtin_fma(x[k], b, c);
    }
    T s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <class T>
__global__ void dep1(T* out, int iters) {
    T x = (T)threadIdx.x * (T)1e-3;
    const T b = (T)0.999999, c = (T)1e-7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 64; ++r) x = __builtin_fma(x, b, c);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
    double* d;
    hipMalloc(&d, 1 << 24);
    hipEvent_t s, e;
    hipEventCreate(&s); hipEventCreate(&e);
    const int blocks = 1024, iters = 20000;   // 1024 waves of 64 = one per SIMD on 256 CUs
    for (int prec = 0; prec < 2; ++prec)
        for (int dep = 1; dep >= 0; --dep)
            for (int act : {1, 16, 32, 33, 64}) {
                for (int rep = 0; rep < 2; ++rep) {
                    hipEventRecord(s);
                    if (prec == 0) hipLaunchKernelGGL(chain<double>, dim3(blocks), dim3(64), 0, 0, d, iters, act, dep);
                    else hipLaunchKernelGGL(chain<float>, dim3(blocks), dim3(64), 0, 0, (float*)d, iters, act, dep);
                    hipEventRecord(e);
                    hipEventSynchronize(e);
                    float ms; hipEventElapsedTime(&ms, s, e);
                    if (rep) printf("%s %s active=%2d: %.3f ms  -> %.2f ns per FMA-instr\n", prec ? "f32" : "f64",
                                    dep ? "dependent  " : "independent", act, ms, ms * 1e6 / (iters * 4.0));
                }
            }
    for (int prec = 0; prec < 2; ++prec)
        for (int act : {16, 32, 64}) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(s);
                if (prec == 0) hipLaunchKernelGGL(sincos_chain<double>, dim3(blocks), dim3(64), 0, 0, d, 2000, act);
                else hipLaunchKernelGGL(sincos_chain<float>, dim3(blocks), dim3(64), 0, 0, (float*)d, 2000, act);
                hipEventRecord(e);
                hipEventSynchronize(e);
                float ms; hipEventElapsedTime(&ms, s, e);
                if (rep) printf("%s sin+cos chain active=%2d: %.3f ms -> %.1f ns per iteration\n", prec ? "f32" : "f64", act, ms,
                                ms * 1e6 / 2000);
            }
        }
    for (int waves : {1024, 2048, 4096})
        for (int prec = 0; prec < 2; ++prec) {
            for (int kind = 0; kind < 2; ++kind) {
                float best = 1e9;
                for (int rep = 0; rep < 3; ++rep) {
                    hipEventRecord(s);
                    if (kind == 0) {
                        if (prec == 0) hipLaunchKernelGGL(ilp8<double>, dim3(waves), dim3(64), 0, 0, d, 2000);
                        else hipLaunchKernelGGL(ilp8<float>, dim3(waves), dim3(64), 0, 0, (float*)d, 2000);
                    } else {
                        if (prec == 0) hipLaunchKernelGGL(dep1<double>, dim3(waves), dim3(64), 0, 0, d, 2000);
                        else hipLaunchKernelGGL(dep1<float>, dim3(waves), dim3(64), 0, 0, (float*)d, 2000);
                    }
                    hipEventRecord(e);
                    hipEventSynchronize(e);
                    float ms; hipEventElapsedTime(&ms, s, e);
                    if (ms < best) best = ms;
                }
                printf("%s %s waves=%d (%d/SIMD): %.3f ms -> %.2f ns per wave-FMA (per wave)\n", prec ? "f32" : "f64",
                       kind == 0 ? "8 independent" : "1 dependent  ", waves, waves / 1024, best,
                       best * 1e6 / (2000.0 * 64));
            }
        }
    // two waves per SIMD: 2048 blocks
    for (int act : {16, 32, 64}) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(s);
            hipLaunchKernelGGL(chain<double>, dim3(2048), dim3(64), 0, 0, d, iters, act, 1);
            hipEventRecord(e);
            hipEventSynchronize(e);
            float ms; hipEventElapsedTime(&ms, s, e);
            if (rep) printf("f64 dependent, 2 waves/SIMD, active=%2d: %.3f ms\n", act, ms);
        }
    }
    return 0;
}
