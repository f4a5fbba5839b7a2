// Large bf16 GEMM path, 256 x 256 tiles (M, N multiples of 256, K a multiple of 32): the
// projections of the TBPTT step -- MLP hidden/output layers, the tier-to-MLP upsampling
// (8192 x 16384 x 1024), GRU input projections -- forward, dgrad and wgrad.
//
// One 512-thread workgroup (8 waves, 2 along M x 4 along N, 128 x 64 outputs per wave =
// 8 x 4 fragments of v_mfma_f32_16x16x32_bf16) per CU.  The whole 160 KiB of LDS is a
// 5-slot ring of 32-deep k-stages (16 KiB per operand per stage) filled directly by
// global_load_lds_dwordx4; three stages stay in flight across the raw s_barrier that
// opens each stage (counted s_waitcnt vmcnt, never a __syncthreads that would drain the
// DMA queue).  LDS images (the global source addresses carry the swizzle, the DMA writes
// lane-linear):
//   k-contiguous operand   [256 rows][64 B]    16-B slot ^ ((row >> 2) & 3): the 16 lanes
//                          of each ds_read_b128 pass hit 16 distinct bank quads;
//   row-contiguous operand [32 k-rows][512 B]  16-B slot ^ (2*(k&3) + 8*((k>>3)&1)):
//                          ds_read_b64_tr_b16 transposed reads, 32 distinct 8-B bank
//                          slots per 32-lane pass.
// The MFMA runs with the operands swapped (B fragment as the "A" input), so each lane
// ends up with 4 CONSECUTIVE COLUMNS of one output row: the epilogue loads Cin / bias /
// the ReLU mask and stores C as 8- or 16-byte vectors instead of 2-4 byte scalars.
// Split-K (gridDim.z) accumulates fp32 partial tiles with atomics into a zeroed C for the
// weight-gradient shapes whose 256 x 256 tile grid cannot fill 256 CUs.
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

template <bool KC>
__device__ __forceinline__ void g3_issue(const bf16* __restrict__ base, int64_t ld, int r0, int k0,
                                         char* img, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < g3::GLW; ++i) {
        const int c = wave * g3::GLW + i;              // 1-KiB chunk of the image
        const bf16* src;
        if constexpr (KC) {
            const int row = c * 16 + (lane >> 2);
            const int slot = (lane & 3) ^ ((row >> 2) & 3);
            src = base + (int64_t)(r0 + row) * ld + k0 + slot * 8;
        } else {
            const int kr = c * 2 + (lane >> 5);
            const int slot = (lane & 31) ^ (2 * (kr & 3) + 8 * ((kr >> 3) & 1));
            src = base + (int64_t)(k0 + kr) * ld + r0 + slot * 8;
        }
        __builtin_amdgcn_global_load_lds(G3_GLB(src), G3_LDS(img + c * 1024), 16, 0, 0);
    }
}

// fragment of image rows (or columns) f0..f0+15, the stage's 32 k
template <bool KC>
__device__ __forceinline__ bf16x8 g3_frag(const char* img, int f0, int lane) {
    if constexpr (KC) {
        const int r = f0 + (lane & 15);
        const int slot = (lane >> 4) ^ ((r >> 2) & 3);
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

__device__ __forceinline__ void g3_load4(const float* p, float (&v)[4]) {
    const floatx4 x = *reinterpret_cast<const floatx4*>(p);
    v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
}
__device__ __forceinline__ void g3_load4(const bf16* p, float (&v)[4]) {
    const u16x4 x = *reinterpret_cast<const u16x4*>(p);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = __uint_as_float((unsigned)x[e] << 16);
}
__device__ __forceinline__ void g3_store4(float* p, const float (&v)[4]) {
    *reinterpret_cast<floatx4*>(p) = floatx4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ void g3_store4(bf16* p, const float (&v)[4]) {
    u16x4 x;
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = __bfloat16_as_ushort(__float2bfloat16(v[e]));
    *reinterpret_cast<u16x4*>(p) = x;
}

// SW: operands swapped in the MFMA (vector epilogue); !SW: the plain split-K partial
// path, where a lane's 4 values are 4 rows of one column and each atomic instruction
// covers 16 consecutive columns (64 B) of 4 rows instead of 16 rows x 4 B.
template <typename TO, bool KCA, bool KCB, bool SW>
__global__ __launch_bounds__(512, 1) void gemm3_kernel(Gemm3Args g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave & 1, wn = wave >> 1;
    const int ntm = g.M / g3::BM, ntn = g.N / g3::BN;
    const int t = g3_xcd_remap(blockIdx.x, ntm * ntn);
    const int tm = t / ntn, tn = t % ntn;
    const int m0 = tm * g3::BM, n0 = tn * g3::BN;
    const int kslice = g.K / g.ksplit;
    const int kbeg = blockIdx.z * kslice;
    const int nk = kslice / g3::BK;
    const bf16* A = reinterpret_cast<const bf16*>(g.A);
    const bf16* B = reinterpret_cast<const bf16*>(g.B);

    floatx4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    auto issue = [&](int kt, int slot) {
        char* img = smem + slot * g3::SLOT;
        const int k0 = kbeg + kt * g3::BK;
        g3_issue<KCA>(A, g.lda, m0, k0, img, wave, lane);
        g3_issue<KCB>(B, g.ldb, n0, k0, img + g3::OPB, wave, lane);
    };
#pragma unroll
    for (int s = 0; s < g3::NS - 1; ++s)
        if (s < nk) issue(s, s);

    int rs = 0, ws = g3::NS - 1;
    for (int kt = 0; kt < nk; ++kt) {
        g3_wait_sel<2 * g3::GLW, g3::NS - 2>(nk - 1 - kt);
        __builtin_amdgcn_s_barrier();
        if (kt + g3::NS - 1 < nk) issue(kt + g3::NS - 1, ws);
        ws = ws == g3::NS - 1 ? 0 : ws + 1;
        const char* ia = smem + rs * g3::SLOT;
        const char* ib = ia + g3::OPB;
        rs = rs == g3::NS - 1 ? 0 : rs + 1;
        bf16x8 a[8], b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = g3_frag<KCB>(ib, wn * 64 + j * 16, lane);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = g3_frag<KCA>(ia, wm * 128 + i * 16, lane);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0)
                               : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    }

    if constexpr (!SW) {
        float* Cf = reinterpret_cast<float*>(g.C);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = n0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = m0 + wm * 128 + i * 16 + (lane >> 4) * 4 + e;
                    float* dst = Cf + (int64_t)row * g.ldc + col;
                    if (g.ksplit > 1) atomicAdd(dst, g.alpha * acc[i][j][e]);
                    else *dst = g.alpha * acc[i][j][e];
                }
            }
        return;
    }

    // epilogue: lane holds C[row][col .. col+3] of each fragment
    TO* Cp = reinterpret_cast<TO*>(g.C);
    const bf16* mask = reinterpret_cast<const bf16*>(g.mask);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int row = m0 + wm * 128 + i * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = n0 + wn * 64 + j * 16 + (lane >> 4) * 4;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = g.alpha * acc[i][j][e];
            if (g.beta != 0.f) {
                float c[4];
                g3_load4(g.Cin + (int64_t)row * g.ldcin + col, c);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += g.beta * c[e];
            }
            if (g.bias_mode == 1) {
                float bb[4];
                g3_load4(g.bias + col, bb);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += bb[e];
            } else if (g.bias_mode == 2) {
                const float bb = g.bias[row];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += bb;
            }
            if (g.relu) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
            }
            if (mask) {
                float mk[4];
                g3_load4(mask + (int64_t)row * g.ldmask + col, mk);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = mk[e] > 0.f ? v[e] : 0.f;
            }
            g3_store4(Cp + (int64_t)row * g.ldc + col, v);
        }
    }
}

template <typename TO, bool KCA, bool KCB, bool SW>
static int launch3(const Gemm3Args& g, hipStream_t s) {
    auto k = gemm3_kernel<TO, KCA, KCB, SW>;
    static bool attr = false;
    if (!attr) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)k,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, g3::LDS));
        attr = true;
    }
    dim3 grid((g.M / g3::BM) * (g.N / g3::BN), 1, g.ksplit);
    hipLaunchKernelGGL(k, grid, dim3(g3::NT), g3::LDS, s, g);
    SRNN_LAUNCH_CHECK();
    return 0;
}

template <typename TO, bool SW>
static int launch3_layout(const Gemm3Args& g, bool kca, bool kcb, hipStream_t s) {
    if (kca && kcb) return launch3<TO, true, true, SW>(g, s);
    if (kca && !kcb) return launch3<TO, true, false, SW>(g, s);
    if (!kca && kcb) return launch3<TO, false, true, SW>(g, s);
    return launch3<TO, false, false, SW>(g, s);
}

// Split-K factor for a plain fp32-out product: the power of two that minimises
// (rounds of 256 workgroups) x (k-stages per workgroup + epilogue allowance).
static int g3_pick_split(int tiles, int K) {
    int best = 1;
    double best_cost = 1e30;
    for (int ks = 1; ks <= 64; ks *= 2) {
        if (K % (ks * g3::BK) || K / ks < 8 * g3::BK) break;
        const int rounds = (tiles * ks + 255) / 256;
        const double cost = rounds * (K / ks / (double)g3::BK + (ks > 1 ? 24.0 : 8.0));
        if (cost < best_cost * 0.97) {
            best_cost = cost;
            best = ks;
        }
    }
    return best;
}

// Returns -1 if the shape/layout is not eligible (caller falls back), else the status.
// force: take the path whenever eligible (tile == 5), else only when the 256-tile grid
// (with split-K) occupies the chip at least as well as the 128-tile kernel would.
int srnn_gemm3_try(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                   float alpha, const void* A, int64_t lda, const void* B, int64_t ldb,
                   float beta, const float* Cin, int64_t ldcin, void* C, int64_t ldc,
                   const float* bias, int bias_mode, int relu, const void* mask, int64_t ldmask,
                   int force, hipStream_t s) {
    if (dtype != SRNN_BF16) return -1;
    if (M % g3::BM || N % g3::BN || K % g3::BK || K == 0) return -1;
    auto al = [](const void* p, int64_t ld, int es) {
        return ((uintptr_t)p % 16 == 0) && ((ld * es) % 16 == 0);
    };
    if (!al(A, lda, 2) || !al(B, ldb, 2)) return -1;
    if ((uintptr_t)C % (out_dtype == SRNN_F32 ? 16 : 8) || ldc % 4) return -1;
    if (beta != 0.f && (!Cin || (uintptr_t)Cin % 16 || ldcin % 4)) return -1;
    if (mask && ((uintptr_t)mask % 8 || ldmask % 4)) return -1;
    if (bias && bias_mode == 1 && (uintptr_t)bias % 16) return -1;
    Gemm3Args g;
    g.A = A; g.B = B; g.C = C; g.Cin = Cin; g.bias = bias; g.mask = mask;
    g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldcin = ldcin; g.ldmask = ldmask;
    g.M = M; g.N = N; g.K = K; g.alpha = alpha; g.beta = beta;
    g.bias_mode = bias ? bias_mode : 0; g.relu = relu;
    const int tiles = (M / g3::BM) * (N / g3::BN);
    const bool plain = beta == 0.f && !bias && !relu && !mask && out_dtype == SRNN_F32;
    const int ks = plain ? g3_pick_split(tiles, K) : 1;
    if (!force) {
        const int64_t wg3 = (int64_t)tiles * ks;
        const int64_t wg2 = (int64_t)(M / 128) * (N / 128);
        if (wg3 < 192 && wg2 > wg3) return -1;
    }
    g.ksplit = ks;
    if (ks > 1) {
        if (ldc == N) {
            SRNN_CHECK_HIP(hipMemsetAsync(C, 0, (size_t)M * N * 4, s));
        } else {
            SRNN_CHECK_HIP(hipMemset2DAsync(C, ldc * 4, 0, (size_t)N * 4, M, s));
        }
    }
    const bool kca = !transA, kcb = transB;
    if (ks > 1) return launch3_layout<float, false>(g, kca, kcb, s);
    if (out_dtype == SRNN_F32) return launch3_layout<float, true>(g, kca, kcb, s);
    return launch3_layout<bf16, true>(g, kca, kcb, s);
}
