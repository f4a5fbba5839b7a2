// Shared pieces of the 256 x 256 bf16 GEMM kernels (gemm3.hip, gemm3e.hip): the argument
// block, the LDS image layouts (ring mode: 32-deep stages; pair mode: 64-deep stages of 128-B
// rows) and their per-lane DMA sources / fragment reads, the XCD-aware tile order.
#pragma once
#include "samplernn_hip_internal.hpp"

typedef short short4_ __attribute__((ext_vector_type(4)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
#define G3_LDS(p) ((__attribute__((address_space(3))) void*)(p))
#define G3_GLB(p) ((const __attribute__((address_space(1))) void*)(p))

struct Gemm3Args {
    const void* A;
    const void* B;
    void* C;
    const float* Cin;
    const float* bias;
    const void* mask;
    int64_t lda, ldb, ldc, ldcin, ldmask;
    int M, N, K, ksplit;
    float alpha, beta;
    int bias_mode, relu;
    int diag;   // timing experiments (SRNN_G3DIAG): 1 no MFMA, 2 no DMA wait, 4 no DMA, 8 no epilogue
    float* part;  // split-K: [ksplit][M][N] fp32 partial tiles (summed in k order by
                  // g3_splitk_sum_kernel: deterministic); null -> fp32 atomics into C
    // ReLU masks as bits (bit c % 16 of u16 [row][c / 16] = value(row, c) > 0): mbi zeroes
    // the outputs whose bit is clear (in place of the bf16 mask); mbo receives the bits of
    // this GEMM's bf16 output (the forward of a ReLU layer, for its backward)
    const unsigned short* mbi;
    int64_t ldmbi;
    unsigned short* mbo;
    int64_t ldmbo;
    // optional: max |C| over the stored bf16 values, as float bits, atomicMax-ed here (the
    // packed dTab scatter's scale, dtab.hip); the word must be zero before the GEMM
    unsigned* amax;
    // optional (with amax): a column-blocked copy of the bf16 output, [N / 4][M][4] -- the
    // dTab scatter's operand (dtab.hip: one load instruction then reads whole lines)
    bf16* blk;
    // optional (srnn_gemm_csum_next): column sums of the stored bf16 output per 128-row
    // block, csp[M / 128][N] fp32 (each entry written once; the caller sums the blocks) --
    // the bias gradient of the layer whose output gradient this GEMM produces
    float* csp;
    // optional (srnn_gemm_logsoftmax_next; fp32 out, N = 256 = one tile column): the epilogue
    // writes log_softmax of every output row (the SampleLevelMLP's logits, model.py:324-325)
    // instead of the row itself
    int lsm;
};

namespace g3 {
constexpr int BM = 256, BN = 256, BK = 32, NS = 5, NT = 512;
constexpr int OPB = 256 * BK * 2;       // 16 KiB per operand image
constexpr int SLOT = 2 * OPB;           // A + B
constexpr int LDS = NS * SLOT;          // 160 KiB
constexpr int GLW = 2;                  // glds per wave per operand per stage
}  // namespace g3

template <int N>
__device__ __forceinline__ void g3_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// wait until at most min(ahead, I) stages (PER glds each) of this wave remain in flight
template <int PER, int I>
__device__ __forceinline__ void g3_wait_sel(int ahead) {
    if constexpr (I == 0) {
        g3_wait_vm<0>();
    } else {
        if (ahead >= I) g3_wait_vm<I * PER>();
        else g3_wait_sel<PER, I - 1>(ahead);
    }
}

// 16-B slot swizzle of a 64-B k-contiguous row: row block (r >> 2) -> 0, 2, 3, 1.  The
// ds_read_b128 lane groups are {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32): with this
// permutation each group's 16 lanes hit 16 distinct 4-bank chunks (the plain
// (r >> 2) & 3 puts two lanes on each chunk -- 8 LDS cycles per read instead of 4).
__device__ __forceinline__ int g3_kcswz(int r) { return (0x78 >> (2 * ((r >> 2) & 3))) & 3; }

// per-lane source of DMA piece c (1 KiB of the stage image) at k = k0
template <bool KC>
__device__ __forceinline__ const bf16* g3_src(const bf16* __restrict__ base, int64_t ld, int r0,
                                              int k0, int c, int lane) {
    if constexpr (KC) {
        const int row = c * 16 + (lane >> 2);
        const int slot = (lane & 3) ^ g3_kcswz(row);
        return base + (int64_t)(r0 + row) * ld + k0 + slot * 8;
    } else {
        const int kr = c * 2 + (lane >> 5);
        const int slot = (lane & 31) ^ (2 * (kr & 3) + 8 * ((kr >> 3) & 1));
        return base + (int64_t)(k0 + kr) * ld + r0 + slot * 8;
    }
}

// fragment of image rows (or columns) f0..f0+15, the stage's 32 k
template <bool KC>
__device__ __forceinline__ bf16x8 g3_frag(const char* img, int f0, int lane) {
    if constexpr (KC) {
        const int r = f0 + (lane & 15);
        const int slot = (lane >> 4) ^ g3_kcswz(r);
        return *reinterpret_cast<const bf16x8*>(img + r * 64 + slot * 16);
    } else {
        const int h = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
        const int j = (f0 >> 2) + p;                   // 8-B column chunk
        short4_ lo, hi;
        {
            const int kr = 8 * h + q;
            const int s = (j >> 1) ^ (2 * (kr & 3) + 8 * ((kr >> 3) & 1));
            lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) short4_*)(img + kr * 512 + s * 16 + (j & 1) * 8));
        }
        {
            const int kr = 8 * h + 4 + q;
            const int s = (j >> 1) ^ (2 * (kr & 3) + 8 * ((kr >> 3) & 1));
            hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) short4_*)(img + kr * 512 + s * 16 + (j & 1) * 8));
        }
        u16x8 v;
        v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
        v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
        return __builtin_bit_cast(bf16x8, v);
    }
}

__device__ __forceinline__ int g3_xcd_remap(int wgid, int nwg) {
    const int q = nwg / 8, r = nwg % 8;
    const int xcd = wgid % 8, local = wgid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// Pair mode: 64-deep stages, 2 slots x 64 KiB.  A k-contiguous operand keeps 128-B rows
// (a whole cache line per row per stage: every DMA piece is 8 rows x 128 B, half the L1
// tag lookups / L2 requests of 64-B half lines), two slots of 64 KiB
// with one stage of look-ahead (stage s+1 streams in while stage s computes), the
// structure of the 256 x 256 templates in the CDNA4 guide.
namespace g3p {
constexpr int BK = 64;
constexpr int OPB = 256 * BK * 2;       // 32 KiB per operand image
constexpr int SLOT = 2 * OPB;
constexpr int LDS = 2 * SLOT;           // 128 KiB
constexpr int GLW = 4;                  // glds per wave per operand per stage
}  // namespace g3p

// per-lane source of DMA piece c at k = k0
template <bool KC>
__device__ __forceinline__ const bf16* g3p_src(const bf16* __restrict__ base, int64_t ld, int r0,
                                               int k0, int c, int lane) {
    if constexpr (KC) {
        const int row = c * 8 + (lane >> 3);
        const int slot = (lane & 7) ^ ((row >> 1) & 7);
        return base + (int64_t)(r0 + row) * ld + k0 + slot * 8;
    } else {
        const int kr = c * 2 + (lane >> 5);
        const int slot = (lane & 31) ^ (2 * (kr & 3) + 8 * ((kr >> 3) & 1));
        return base + (int64_t)(k0 + kr) * ld + r0 + slot * 8;
    }
}

// fragment rows f0..f0+15, k-unit u (0..1: 32 k each) of the stage
template <bool KC>
__device__ __forceinline__ bf16x8 g3p_frag(const char* img, int f0, int u, int lane) {
    if constexpr (KC) {
        const int r = f0 + (lane & 15);
        const int slot = (u * 4 + (lane >> 4)) ^ ((r >> 1) & 7);
        return *reinterpret_cast<const bf16x8*>(img + r * 128 + slot * 16);
    } else {
        return g3_frag<false>(img + u * 32 * 512, f0, lane);
    }
}


// gemm3e.hip: the 8-phase ping-pong NT kernel; returns -1 if the call is not eligible
int srnn_gemm3e_launch(const Gemm3Args& g, bool out_f32, int ncu, hipStream_t s);
