// Shared helpers for the SampleRNN HIP/CDNA4 (gfx950) library.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef __hip_bfloat16 bf16;

enum SrnnDtype { SRNN_F32 = 0, SRNN_BF16 = 1 };

// ---- error reporting (C-ABI returns int status; text via srnn_last_error) --------
void srnn_set_error(const char* fmt, ...);

#define SRNN_CHECK_HIP(expr)                                                        \
    do {                                                                            \
        hipError_t _e = (expr);                                                     \
        if (_e != hipSuccess) {                                                     \
            srnn_set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr,             \
                           hipGetErrorString(_e));                                  \
            return 2;                                                               \
        }                                                                           \
    } while (0)

#define SRNN_REQUIRE(cond, ...)                                                     \
    do {                                                                            \
        if (!(cond)) {                                                              \
            srnn_set_error(__VA_ARGS__);                                            \
            return 1;                                                               \
        }                                                                           \
    } while (0)

#define SRNN_LAUNCH_CHECK()                                                         \
    do {                                                                            \
        hipError_t _e = hipGetLastError();                                          \
        if (_e != hipSuccess) {                                                     \
            srnn_set_error("%s:%d launch -> %s", __FILE__, __LINE__,                \
                           hipGetErrorString(_e));                                  \
            return 2;                                                               \
        }                                                                           \
    } while (0)

// ---- scalar conversions --------------------------------------------------------------
__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return __bfloat162float(x); }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return __float2bfloat16(x); }

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// exact-ish transcendental forms used where parity with torch CPU matters
__device__ __forceinline__ float sigmoid_acc(float x) { return 1.0f / (1.0f + expf(-x)); }

// ---- cross-lane moves without LDS ------------------------------------------------------
// (__shfl* is a ds_bpermute: an LDS round trip of ~100+ cycles; these are VALU ops)
template <int CTRL> __device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, true);
}
// value of lane + 1 within the lane's 16-lane row (DPP row_shl:1; 0 at a row's last lane)
__device__ __forceinline__ uint32_t lane_next16(uint32_t v) { return dpp_u32<0x101>(v); }
// pair exchange across lanes i, i ^ 16 (v_permlane16_swap) and i, i ^ 32 (v_permlane32_swap):
// lo = the value of the pair's lower lane, hi = its upper lane's, in both lanes
__device__ __forceinline__ void xpair16(uint32_t v, uint32_t& lo, uint32_t& hi) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    lo = r[0];
    hi = r[1];
}
__device__ __forceinline__ void xpair32(uint32_t v, uint32_t& lo, uint32_t& hi) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    lo = r[0];
    hi = r[1];
}

// ---- MFMA wrappers -------------------------------------------------------------------
// One "k-unit" = 64 bytes of k per row: 16 fp32 (4 x v_mfma_f32_16x16x4_f32) or
// 32 bf16 (1 x v_mfma_f32_16x16x32_bf16).  Each lane supplies the 16 bytes at offset
// (lane>>4)*16 of its row's unit for both A (row = lane&15) and B (col = lane&15).
// For fp32 the four MFMAs of a unit use element kk of the lane's float4, i.e. the
// k-order inside a unit is permuted identically for A and B (exact same product set).
template <typename T> struct Mma;

template <> struct Mma<float> {
    typedef floatx4 frag;
    __device__ __forceinline__ static void run(floatx4& acc, const floatx4& a, const floatx4& b) {
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], acc, 0, 0, 0);
    }
};

template <> struct Mma<bf16> {
    typedef bf16x8 frag;
    __device__ __forceinline__ static void run(floatx4& acc, const bf16x8& a, const bf16x8& b) {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
};

static inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
