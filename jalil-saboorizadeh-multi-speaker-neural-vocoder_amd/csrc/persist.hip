// Sticky failure flag of the persistent sweeps (gru_xcd.hip, gru_seq.hip).
//
// A persistent sweep that gives up a hand-off (bounded spin) produces invalid hidden states
// and gradients.  Its per-call error word lives in a work buffer the next call re-zeroes, so
// every failing workgroup also raises ONE per-device flag in device memory here.  Three
// readers, all stream-ordered or at the caller's own sync point:
//   * the fused clip + Adam kernel (misc.hip) reads it on the device and skips the update,
//     so a failed step never reaches the weights or the Adam moments;
//   * under data parallelism the flag rides in the last gradient bucket (f32 0 / 1,
//     srnn_persistent_flag_to_f32 / _or_f32) so the SUM all-reduce gives every rank the same
//     verdict: all ranks skip the update together and raise together;
//   * srnn_persistent_error_take (host, synchronises) reports and clears it.
#include "samplernn_hip_internal.hpp"

namespace {
constexpr int MAXDEV = 64;
int* g_flag[MAXDEV] = {nullptr};
}  // namespace

int* srnn_sticky_flag() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAXDEV) return nullptr;
    if (!g_flag[dev]) {
        int* p = nullptr;
        if (hipMalloc(&p, 64) != hipSuccess) return nullptr;
        if (hipMemset(p, 0, 64) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            (void)hipFree(p);
            return nullptr;
        }
        g_flag[dev] = p;
    }
    return g_flag[dev];
}

// ---- co-residency of the persistent grids (handoff.hpp).  `share`: processes that run
// persistent kernels on this device at once (1 normally; distributed.init sets the number
// of ranks sharing one GPU in a rehearsal).  A persistent launch of `blocks` workgroups is
// only taken when every process's grid fits the device at once:
//   occupancy(kernel, threads, lds) x CUs >= blocks x share
// so each workgroup is guaranteed to start, at the latest once the non-persistent kernels
// that held CUs at launch time have ended -- and the in-kernel arrival gate waits for that.
namespace {
int g_share = 1;
int g_cus = 0;
}  // namespace

extern "C" int srnn_set_device_share(int n) {
    g_share = n < 1 ? 1 : n;
    return 0;
}

extern "C" int srnn_device_share(void) { return g_share; }

int srnn_device_cus() {
    if (!g_cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            g_cus = 0;
    }
    return g_cus;
}

// the support predicates' form: one workgroup per CU assumed (the persistent kernels take
// 100-160 KiB of LDS or 256 VGPRs each)
int srnn_persist_fits_cus(int64_t blocks) {
    const int ncu = srnn_device_cus();
    return ncu > 0 && blocks * g_share <= ncu;
}

// the launch-time check with the kernel's real occupancy; 0 = fits, else an error (reported)
int srnn_persist_check(const void* kernel, int threads, size_t lds, int64_t blocks,
                       const char* what) {
    // (the occupancy query is cached per (kernel, threads, lds): the eager step asks per sweep)
    static struct { const void* k; int t; size_t l; int occ; } cache[32];
    static int ncache = 0;
    int occ = 0;
    for (int i = 0; i < ncache; ++i)
        if (cache[i].k == kernel && cache[i].t == threads && cache[i].l == lds) occ = cache[i].occ;
    if (!occ) {
        SRNN_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, threads, lds));
        if (ncache < 32) cache[ncache++] = {kernel, threads, lds, occ};
    }
    const int ncu = srnn_device_cus();
    SRNN_REQUIRE(occ > 0 && ncu > 0 && (int64_t)occ * ncu >= blocks * g_share,
                 "%s: %lld persistent workgroups x %d processes sharing the device cannot all "
                 "be resident (%d per CU x %d CUs): refused", what, (long long)blocks, g_share,
                 occ, ncu);
    return 0;
}

// Diagnostics / tests: occupy `blocks` CUs (a full 160 KiB of LDS each, so one workgroup
// per CU) for `usec` microseconds of wall time -- the "other work holding CUs when a
// persistent grid starts" of the co-residency tests (tests/test_gpu_coresidency.py).
__global__ void hold_cus_kernel(unsigned long long ticks, int* done) {
    extern __shared__ int lds_hold[];
    if (threadIdx.x == 0) lds_hold[0] = 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    __syncthreads();
    if (threadIdx.x == 0 && done)
        __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

extern "C" int srnn_hold_cus(int blocks, int usec, int* done, void* stream) {
    SRNN_REQUIRE(blocks > 0 && usec >= 0 && usec <= 10000000, "hold_cus: bad arguments");
    static bool attr = false;
    if (!attr) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)hold_cus_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           160 * 1024));
        attr = true;
    }
    hipLaunchKernelGGL(hold_cus_kernel, dim3(blocks), dim3(64), 160 * 1024, (hipStream_t)stream,
                       (unsigned long long)usec * 100ull, done);
    SRNN_LAUNCH_CHECK();
    return 0;
}

int srnn_persist_spin_limit(int dflt) {
    // SRNN_PERSIST_FORCE_FAIL=1 (tests only): one workgroup withholds its hand-offs and the
    // spin limit is short, so the real give-up path runs end to end in milliseconds
    return env_flag("SRNN_PERSIST_FORCE_FAIL", 0) ? 256 : dflt;
}

__global__ void flag_to_f32_kernel(const int* flag, float* dst) {
    if (threadIdx.x == 0) *dst = *flag ? 1.f : 0.f;
}
__global__ void flag_or_f32_kernel(int* flag, const float* src) {
    if (threadIdx.x == 0 && *src > 0.f) *flag = 1;
}

extern "C" int srnn_persistent_flag_to_f32(float* dst, void* stream) {
    int* f = srnn_sticky_flag();
    SRNN_REQUIRE(f && dst, "persistent_flag_to_f32: no flag / null destination");
    hipLaunchKernelGGL(flag_to_f32_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, f, dst);
    SRNN_LAUNCH_CHECK();
    return 0;
}

extern "C" int srnn_persistent_flag_or_f32(const float* src, void* stream) {
    int* f = srnn_sticky_flag();
    SRNN_REQUIRE(f && src, "persistent_flag_or_f32: no flag / null source");
    hipLaunchKernelGGL(flag_or_f32_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, f, src);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// nonzero if any persistent sweep since the last call gave up a hand-off (its results are
// invalid); clears the flag.  Synchronises the device; -1 on a HIP error.
extern "C" int srnn_persistent_error_take(void) {
    int* f = srnn_sticky_flag();
    int v = 0;
    if (!f || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(&v, f, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    if (v && (hipMemset(f, 0, sizeof(int)) != hipSuccess || hipDeviceSynchronize() != hipSuccess))
        return -1;
    return v;          // 0, 1 (a hand-off gave up) or 2 (workgroups never all resident)
}

// Stream-ordered snapshot of the flag into `dst` (pinned host memory, 4 bytes): the host
// reads it one step later, after that copy's event, with no device synchronisation
// (samplernn_hip.PersistentErrorWatch: the Trainer's lagged per-iteration check).
extern "C" int srnn_persistent_flag_snapshot(int* dst, void* stream) {
    int* f = srnn_sticky_flag();
    SRNN_REQUIRE(f && dst, "persistent_flag_snapshot: no flag / null destination");
    SRNN_CHECK_HIP(hipMemcpyAsync(dst, f, sizeof(int), hipMemcpyDeviceToHost,
                                  (hipStream_t)stream));
    return 0;
}

// dtype forms of srnn_persistent_flag_to_f32 / _or_f32 for gradient buckets in bf16
__global__ void flag_to_bf16_kernel(const int* flag, bf16* dst) {
    if (threadIdx.x == 0) *dst = __float2bfloat16(*flag ? 1.f : 0.f);
}
__global__ void flag_or_bf16_kernel(int* flag, const bf16* src) {
    if (threadIdx.x == 0 && __bfloat162float(*src) > 0.f) *flag = 1;
}

extern "C" int srnn_persistent_flag_to(void* dst, int dtype, void* stream) {
    if (dtype == SRNN_F32) return srnn_persistent_flag_to_f32((float*)dst, stream);
    int* f = srnn_sticky_flag();
    SRNN_REQUIRE(f && dst && dtype == SRNN_BF16, "persistent_flag_to: bad arguments");
    hipLaunchKernelGGL(flag_to_bf16_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, f,
                       (bf16*)dst);
    SRNN_LAUNCH_CHECK();
    return 0;
}

extern "C" int srnn_persistent_flag_or(const void* src, int dtype, void* stream) {
    if (dtype == SRNN_F32) return srnn_persistent_flag_or_f32((const float*)src, stream);
    int* f = srnn_sticky_flag();
    SRNN_REQUIRE(f && src && dtype == SRNN_BF16, "persistent_flag_or: bad arguments");
    hipLaunchKernelGGL(flag_or_bf16_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, f,
                       (const bf16*)src);
    SRNN_LAUNCH_CHECK();
    return 0;
}
