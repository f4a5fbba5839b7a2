// Probe (tools/, not product): does the dTab scatter's vector-memory pattern slow its LDS
// atomics?  Same ds_add_u64 pattern as lds_atomic_probe3 (16 waves/CU, 16 atomics then
// lgkmcnt(15)); mode 1 adds, per 16 atomics, the scatter's da load: each lane reads 4 B of a
// different 2-KiB row (16 rows x 2 adjacent lanes per half-wave: 32 cache lines per
// instruction, 8 B used of each), issued four batches ahead, its value feeding the atomics;
// mode 2 the same loads from a column-blocked layout (the 16 rows' 8-B pairs contiguous: one
// whole line per half-wave).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe4.bin tools/lds_atomic_probe4.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int NROWS = 65536;       // 65536 rows x 2 KiB = 128 MiB source
constexpr int ROWU = 512;          // u32 per row

template <int MODE>
__global__ __launch_bounds__(1024) void k(const unsigned* __restrict__ src,
                                          unsigned long long* out, int iters, unsigned seed) {
    extern __shared__ unsigned long long acc[];
    for (int i = threadIdx.x; i < 8192; i += 1024) acc[i] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31, li = lane & 15;
    const int p = (lane >> 4) & 1, wave = threadIdx.x >> 6;
    const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)acc;
    unsigned q = (seed + wave * 977u + h * 131u) * 2654435761u;
    const int col = (int)(blockIdx.x % 256u) * 2 + p;                 // < 512: inside a row
    const int row0 = (int)((blockIdx.x * 16 + wave) * 2 + h) * 4096;
    auto ld = [&](int i) -> unsigned {
        const int row = (row0 + i * 16 + li) & (NROWS - 1);
        if (MODE == 2) return src[(size_t)row * 2 + p];           // < 2 * NROWS: in bounds
        return src[(size_t)row * ROWU + col];
    };
    unsigned r0 = 0, r1 = 0, r2 = 0, r3 = 0;
    if (MODE) { r0 = ld(0); r1 = ld(1); r2 = ld(2); r3 = ld(3); }
    unsigned long long v = threadIdx.x;
    for (int i = 0; i < iters; ++i) {
        if (MODE) {
            v = (unsigned long long)r0 + threadIdx.x;
            r0 = r1; r1 = r2; r2 = r3; r3 = ld(i + 4);
        }
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
    out[(size_t)blockIdx.x * 1024 + threadIdx.x] = acc[threadIdx.x] + r0 + r1 + r2 + r3;
}

int main() {
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipFuncSetAttribute((const void*)k<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)k<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)k<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const int blocks = ncu * 4;                   // 4 rounds of one 1024-thread workgroup per CU
    unsigned long long* out;
    unsigned* src;
    (void)hipMalloc(&out, (size_t)blocks * 1024 * 8);
    (void)hipMalloc(&src, (size_t)NROWS * ROWU * 4);
    (void)hipMemset(src, 1, (size_t)NROWS * ROWU * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 2048;
    for (int mode = 0; mode < 3; ++mode)
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(e0);
            if (mode == 0)
                hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(1024), 100 * 1024, 0, src, out, iters, 7u + rep);
            else if (mode == 1)
                hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(1024), 100 * 1024, 0, src, out, iters, 7u + rep);
            else
                hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(1024), 100 * 1024, 0, src, out, iters, 7u + rep);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double ops = (double)blocks * 1024 * iters * 16;
            if (rep)
                printf("mode %d (%s): %.3f ms  %.1f lane-ops per clock per CU at 2.4 GHz\n", mode,
                       mode == 2 ? "atomics + whole-line loads" : mode ? "atomics + da-pattern loads"
                                                                   : "atomics only", ms,
                       ops / (ms * 1e-3) / ncu / 2.4e9);
        }
    return 0;
}
