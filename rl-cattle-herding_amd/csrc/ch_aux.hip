// ch_aux.hip — small device-side helpers around the step: the end-of-rollout metric reduction.
//
// Reference: BaseAviary.update_evaluation_metrics (sb3_envs/BaseAviary.py:1406-1435) appends per-step
// values to host lists; here every env accumulates its rows in HBM during the step kernel and one
// launch sums them over the envs at the end of a rollout, on the caller's stream, so the RCCL
// all-reduce (bench.py, cattleherd/distributed.py) reads a device buffer and nothing syncs the host.
#include <hip/hip_runtime.h>

#include "ch_internal.h"

namespace ch {

constexpr int kReduceThreads = 256;

// one workgroup per metric row; thread t sums envs t, t + 256, ... in order, then a fixed LDS tree:
// the result is the same for every call on the same data (sharding-invariance tests compare it)
__global__ __launch_bounds__(kReduceThreads) void k_metrics_reduce(double* metrics, long long E, double* out,
                                                                 const int* err_word, double* err_out, int reset) {
    __shared__ double part[kReduceThreads];
    const int r = blockIdx.x, t = threadIdx.x;
    double* row = metrics + (long long)r * E;
    double s = 0;
    for (long long e = t; e < E; e += kReduceThreads) {
        s += row[e];
        if (reset) row[e] = 0;
    }
    part[t] = s;
    __syncthreads();
    for (int w = kReduceThreads / 2; w > 0; w >>= 1) {
        if (t < w) part[t] += part[t + w];
        __syncthreads();
    }
    if (t == 0) {
        out[r] = part[0];
        if (r == 0 && err_out) *err_out = err_word ? (double)*err_word : 0.0;
    }
}

hipError_t launch_metrics_reduce(double* metrics, long long E, double* out, const int* err_word, double* err_out,
                                 int reset, hipStream_t st) {
    hipLaunchKernelGGL(k_metrics_reduce, dim3(CH_METRIC_COUNT), dim3(kReduceThreads), 0, st, metrics, E, out,
                       err_word, err_out, reset);
    return hipGetLastError();
}

}  // namespace ch
