// Probe (tools/, not product): ds_add_u64 throughput per CU against waves resident per CU, in
// the dTab scatter's pattern (64 lanes = two 32-lane halves, each half 32 consecutive u64 of its
// own 256-B block, 16 atomics then s_waitcnt lgkmcnt(15)).  Dynamic LDS pads each workgroup so
// exactly WG_PER_CU 1024-thread workgroups fit a CU: 16 or 32 waves per CU.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/probe3 tools/lds_atomic_probe3.hip && /tmp/probe3
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(1024) void k(unsigned long long* out, int iters, unsigned seed) {
    extern __shared__ unsigned long long acc[];        // 256 blocks x 32 u64 = 64 KiB used
    for (int i = threadIdx.x; i < 8192; i += 1024) acc[i] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31;
    const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)acc;
    unsigned q = (seed + threadIdx.x / 64 * 977u + h * 131u) * 2654435761u;
    const unsigned long long v = threadIdx.x;
    for (int i = 0; i < iters; ++i) {
        unsigned ad[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            q = q * 1664525u + 1013904223u;
            ad[j] = base + ((q >> 24) & 255u) * 256u + (unsigned)l * 8u;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) asm volatile("ds_add_u64 %0, %1" ::"v"(ad[j]), "v"(v) : "memory");
        asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    out[blockIdx.x * 1024 + threadIdx.x] = acc[threadIdx.x];
}

int main() {
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    unsigned long long* out;
    (void)hipMalloc(&out, (size_t)8 * ncu * 1024 * 8);   // the largest grid: 2 x 4 x ncu blocks
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 2048;
    for (int wpc = 1; wpc <= 2; ++wpc) {
        const size_t lds = wpc == 1 ? 100 * 1024 : 72 * 1024;   // 1 or 2 workgroups per CU
        const int blocks = ncu * wpc * 4;                        // 4 rounds of resident workgroups
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(blocks), dim3(1024), lds, 0, out, iters, 12345u + rep);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double ops = (double)blocks * 1024 * iters * 16;
            if (rep)
                printf("%d waves/CU: %.3f ms  %.2f G lane-ops/s/CU  (%.1f per clock at 2.4 GHz)\n",
                       16 * wpc, ms, ops / (ms * 1e-3) / ncu / 1e9, ops / (ms * 1e-3) / ncu / 2.4e9);
        }
    }
    return 0;
}
