// Probe: throughput of LDS float atomics vs plain LDS RMW on gfx950 (tools/, not product).
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int MODE>
__global__ __launch_bounds__(1024) void k(float* out, int iters, int stride) {
    __shared__ float acc[16384];
    for (int i = threadIdx.x; i < 16384; i += 1024) acc[i] = 0.f;
    __syncthreads();
    const int t = threadIdx.x;
    float v = 1.0f + t * 1e-7f;
    int a = (t * stride) & 16383;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) atomicAdd(&acc[a], v);
        else if (MODE == 1) { acc[a] += v; }
        else if (MODE == 2) { __hip_atomic_fetch_add(&acc[a], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
        a = (a + 1024) & 16383;
    }
    __syncthreads();
    out[blockIdx.x * 1024 + t] = acc[t];
}
int main() {
    float* out; hipMalloc(&out, 1024 * 1024 * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int iters = 4096, blocks = 512;
    for (int stride : {1, 2, 33}) {
        for (int mode = 0; mode < 3; ++mode) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(1024), 0, 0, out, iters, stride);
                if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(1024), 0, 0, out, iters, stride);
                if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(1024), 0, 0, out, iters, stride);
                hipEventRecord(e1); hipEventSynchronize(e1);
                float ms; hipEventElapsedTime(&ms, e0, e1);
                double ops = (double)blocks * 1024 * iters;
                if (rep) printf("stride %2d mode %d (%s): %.3f ms  %.1f lane-ops/clk/CU\n", stride, mode,
                       mode == 0 ? "atomicAdd" : mode == 1 ? "plain RMW" : "hip_atomic relaxed", ms,
                       ops / (ms * 1e-3) / 256 / 2.4e9);
            }
        }
    }
    return 0;
}
