// Probe: what a cooperative launch buys the persistent sweeps on MI355X (ROCm 7).
//   A  plain launch of a 256-workgroup grid-barrier kernel (1 workgroup per CU) while a
//      holder kernel occupies 64 CUs for ~150 ms on another stream
//   B  the same through hipLaunchCooperativeKernel
//   C  hipLaunchCooperativeKernel under stream capture (thread-local) + graph replay
//   D  launch cost: 200 back-to-back launches of the grid kernel, plain vs cooperative
// Every wait is bounded by s_memrealtime (100 MHz); a timeout is reported, never a hang.
// Build: hipcc -O2 --offload-arch=gfx950 tools/coop_probe.hip -o /tmp/coop_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <unistd.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("%s -> %s\n", #x, hipGetErrorString(e_)); } } while (0)

__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

// every workgroup arrives, then waits (<= limit ticks) for the whole grid
__global__ void grid_kernel(int* arrive, int* fail, unsigned long long limit, int expect) {
    extern __shared__ int lds[];
    if (threadIdx.x == 0) {
        lds[0] = 0;
        __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t0 = rt();
        while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < expect) {
            __builtin_amdgcn_s_sleep(2);
            if (rt() - t0 > limit) {
                __hip_atomic_fetch_add(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
}

__global__ void holder_kernel(unsigned long long ticks) {
    extern __shared__ int lds[];
    if (threadIdx.x == 0) lds[0] = 1;
    const unsigned long long t0 = rt();
    while (rt() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    __syncthreads();
}

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
    int dev = 0, cus = 0, coop = 0, occ = 0;
    CK(hipSetDevice(dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
    const size_t lds = 160 * 1024;
    CK(hipFuncSetAttribute((const void*)grid_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CK(hipFuncSetAttribute((const void*)holder_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)grid_kernel, 256, lds));
    printf("E cus=%d cooperative=%d occupancy_per_cu=%d\n", cus, coop, occ);
    const int G = cus;
    int *arrive, *fail;
    CK(hipMalloc(&arrive, 64));
    CK(hipMalloc(&fail, 64));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const unsigned long long limit = 500000000ull;   // 5 s
    const unsigned long long hold = 15000000ull;     // 150 ms
    int zero[16] = {};
    for (int mode = 0; mode < 2; ++mode) {
        CK(hipMemcpy(arrive, zero, 64, hipMemcpyHostToDevice));
        CK(hipMemcpy(fail, zero, 64, hipMemcpyHostToDevice));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(holder_kernel, dim3(64), dim3(256), lds, s2, hold);
        usleep(2000);
        auto t = std::chrono::steady_clock::now();
        int expect = G;
        if (mode == 0) {
            hipLaunchKernelGGL(grid_kernel, dim3(G), dim3(256), lds, s1, arrive, fail, limit, expect);
        } else {
            void* args[] = {&arrive, &fail, (void*)&limit, &expect};
            CK(hipLaunchCooperativeKernel((const void*)grid_kernel, dim3(G), dim3(256), args,
                                          (unsigned)lds, s1));
        }
        CK(hipStreamSynchronize(s1));
        const double el = ms_since(t);
        CK(hipDeviceSynchronize());
        int f = 0;
        CK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
        printf("%s %s launch beside a 150 ms 64-CU holder: grid done in %.1f ms, timeouts %d\n",
               mode ? "B" : "A", mode ? "cooperative" : "plain", el, f);
    }
    // C: capture
    {
        CK(hipMemcpy(arrive, zero, 64, hipMemcpyHostToDevice));
        CK(hipDeviceSynchronize());
        hipGraph_t g = nullptr;
        hipGraphExec_t ge = nullptr;
        int expect = G;
        CK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
        void* args[] = {&arrive, &fail, (void*)&limit, &expect};
        hipError_t e = hipLaunchCooperativeKernel((const void*)grid_kernel, dim3(G), dim3(256),
                                                  args, (unsigned)lds, s1);
        printf("C capture: cooperative launch inside capture -> %s\n", hipGetErrorString(e));
        hipError_t e2 = hipStreamEndCapture(s1, &g);
        printf("C capture: end capture -> %s\n", hipGetErrorString(e2));
        if (e == hipSuccess && e2 == hipSuccess) {
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            for (int r = 0; r < 3; ++r) {
                CK(hipMemcpyAsync(arrive, zero, 64, hipMemcpyHostToDevice, s1));
                CK(hipGraphLaunch(ge, s1));
            }
            CK(hipStreamSynchronize(s1));
            int f = 0;
            CK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
            printf("C replay x3 ok, timeouts %d\n", f);
            // replay beside the holder
            CK(hipMemcpy(arrive, zero, 64, hipMemcpyHostToDevice));
            CK(hipDeviceSynchronize());
            hipLaunchKernelGGL(holder_kernel, dim3(64), dim3(256), lds, s2, hold);
            usleep(2000);
            auto t = std::chrono::steady_clock::now();
            CK(hipGraphLaunch(ge, s1));
            CK(hipStreamSynchronize(s1));
            printf("C replay beside holder: %.1f ms\n", ms_since(t));
            CK(hipDeviceSynchronize());
        }
        hipGetLastError();
    }
    // D: launch cost (expect = 0 so the kernel does not wait)
    for (int mode = 0; mode < 2; ++mode) {
        int expect = 0;
        CK(hipDeviceSynchronize());
        auto t = std::chrono::steady_clock::now();
        for (int i = 0; i < 200; ++i) {
            if (mode == 0) {
                hipLaunchKernelGGL(grid_kernel, dim3(G), dim3(256), lds, s1, arrive, fail, limit, expect);
            } else {
                void* args[] = {&arrive, &fail, (void*)&limit, &expect};
                CK(hipLaunchCooperativeKernel((const void*)grid_kernel, dim3(G), dim3(256), args,
                                              (unsigned)lds, s1));
            }
        }
        CK(hipStreamSynchronize(s1));
        printf("D %s: %.2f us per launch (200 back to back)\n", mode ? "cooperative" : "plain",
               ms_since(t) * 1000.0 / 200);
    }
    return 0;
}
