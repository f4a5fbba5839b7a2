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
    return v ? 1 : 0;
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
