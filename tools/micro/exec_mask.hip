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
