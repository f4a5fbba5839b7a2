// Probe: LDS integer atomics (u32 / u64) vs float on gfx950 (tools/, not product).
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int MODE>
__global__ __launch_bounds__(1024) void k(unsigned long long* out, int iters) {
    __shared__ unsigned long long acc64[8192];
    unsigned int* acc32 = (unsigned int*)acc64;
    for (int i = threadIdx.x; i < 8192; i += 1024) acc64[i] = 0;
    __syncthreads();
    const int t = threadIdx.x;
    int a = t & 8191;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) atomicAdd(&acc32[a], (unsigned)t);
        else atomicAdd(&acc64[a & 8191], (unsigned long long)t);
        a = (a + 1024) & 8191;
    }
    __syncthreads();
    out[blockIdx.x * 1024 + t] = acc64[t];
}
int main() {
    unsigned long long* out; (void)hipMalloc(&out, 1024 * 1024 * 8);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int iters = 4096, blocks = 512;
    for (int mode = 0; mode < 2; ++mode)
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(1024), 0, 0, out, iters);
            else hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(1024), 0, 0, out, iters);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            double ops = (double)blocks * 1024 * iters;
            if (rep) printf("mode %s: %.3f ms  %.1f lane-ops/clk/CU\n", mode == 0 ? "ds_add_u32" : "ds_add_u64", ms,
                            ops / (ms * 1e-3) / 256 / 2.4e9);
        }
    return 0;
}
