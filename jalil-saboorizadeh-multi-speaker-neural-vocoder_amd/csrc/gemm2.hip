// Large-GEMM path (M, N multiples of 128, K a multiple of the k-stage): the projections of
// the TBPTT step (MLP hidden/output, upsampling, GRU input projections) forward, dgrad
// and wgrad.
//
// 128x128 tile per 256-thread workgroup (4 waves, 2x2, 64x64 per wave = 4x4 16x16 MFMA
// fragments).  A 4-slot LDS ring (32 KiB per slot) is filled directly by
// global_load_lds_dwordx4 (no register staging, no ds_write), three k-stages in flight,
// counted `s_waitcnt vmcnt` + a raw s_barrier per stage (a __syncthreads would drain the
// DMA queue).  Images:
//   k-contiguous operand  [128 rows][128 B], 16-B slot XOR (row & 7)      -> ds_read_b128
//   row-contiguous operand [KB k-rows][128 elems], bf16: 16-B slot XOR
//       2*(k&3) + 8*((k>>3)&1) so the ds_read_b64_tr_b16 transposed reads of the
//       16x16x32 operand hit 32 distinct 8-B bank slots per 32-lane half; fp32: b32 reads.
// The source addresses carry the inverse swizzle (glds writes lane-linear).  Split-K
// (gridDim.z slices) accumulates with fp32 atomics into a zeroed C for wgrad shapes
// whose M x N has too few tiles to fill 256 CUs.  Workgroup ids are remapped so the
// N-tiles of one M-row land on one XCD (A rows stream through one L2).
#include "samplernn_hip_internal.hpp"

typedef short short4_ __attribute__((ext_vector_type(4)));
#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))
#define GLB_PTR(p) ((const __attribute__((address_space(1))) void*)(p))

struct Gemm2Args {
    const void* A;
    const void* B;
    void* C;
    const float* Cin;
    const float* bias;
    const void* mask;
    int64_t lda, ldb, ldc, ldcin, ldmask;
    int M, N, K, ksplit;
    float* part;          // split-K partial tiles [ksplit][M][N] (deterministic ordered sum),
                          // or null: fp32 atomics into C
    float alpha, beta;
    int bias_mode, relu;
};

template <int N>
__device__ __forceinline__ void wait_vm() {
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
}

template <typename T>
struct G2 {
    static constexpr int E = 16 / (int)sizeof(T);       // elements per 16-B chunk
    static constexpr int KB = 128 / (int)sizeof(T);     // k per stage (2 units of 64 B)
    static constexpr int OPB = 128 * 128;               // bytes per operand image
    static constexpr int SLOT = 2 * OPB;                // A + B
    static constexpr int NS = 4;
};

// ---------------------------------------------------------------- glds issue
// Each operand image is 16 KiB = 16 wave-instructions of 1 KiB; wave w issues 4.
template <typename T, bool KC>
__device__ __forceinline__ void issue_operand(const T* __restrict__ base, int64_t ld, int r0,
                                              int k0, char* img, int wave, int lane) {
    typedef G2<T> C;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = wave * 4 + i;
        const T* src;
        if constexpr (KC) {
            const int row = c * 8 + (lane >> 3);
            const int slot = (lane & 7) ^ (row & 7);
            src = base + (int64_t)(r0 + row) * ld + k0 + slot * C::E;
        } else if constexpr (sizeof(T) == 2) {
            const int kr = c * 4 + (lane >> 4);
            const int slot = (lane & 15) ^ (2 * (kr & 3) + 8 * ((kr >> 3) & 1));
            src = base + (int64_t)(k0 + kr) * ld + r0 + slot * C::E;
        } else {
            const int kr = c * 2 + (lane >> 5);
            const int slot = lane & 31;
            src = base + (int64_t)(k0 + kr) * ld + r0 + slot * C::E;
        }
        __builtin_amdgcn_global_load_lds(GLB_PTR(src), LDS_PTR(img + c * 1024), 16, 0, 0);
    }
}

// ---------------------------------------------------------------- fragment reads
// fragment rows f0..f0+15 of the operand, k-unit u (0..1) of the stage
template <typename T, bool KC>
__device__ __forceinline__ typename Mma<T>::frag read_frag(const char* img, int f0, int u,
                                                           int lane, int kk_unused = 0) {
    typedef typename Mma<T>::frag F;
    if constexpr (KC) {
        const int r = f0 + (lane & 15);
        const int slot = (u * 4 + (lane >> 4)) ^ (r & 7);
        return *reinterpret_cast<const F*>(img + r * 128 + slot * 16);
    } else if constexpr (sizeof(T) == 2) {
        const int h = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
        const int j = (f0 >> 2) + p;                      // 8-B column chunk
        short4_ lo, hi;
        {
            const int kr = u * 32 + 8 * h + q;
            const int s = (j >> 1) ^ (2 * (kr & 3) + 8 * ((kr >> 3) & 1));
            lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) short4_*)(img + kr * 256 + s * 16 + (j & 1) * 8));
        }
        {
            const int kr = u * 32 + 8 * h + 4 + q;
            const int s = (j >> 1) ^ (2 * (kr & 3) + 8 * ((kr >> 3) & 1));
            hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) short4_*)(img + kr * 256 + s * 16 + (j & 1) * 8));
        }
        u16x8 v;
        v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
        v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
        return __builtin_bit_cast(F, v);
    } else {
        // fp32 row-contiguous: MFMA kk of unit u uses k = 16u + 4*(lane>>4) + kk
        const int col = f0 + (lane & 15);
        const int kq = lane >> 4;
        F v;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
            v[kk] = *reinterpret_cast<const float*>(img + (u * 16 + 4 * kq + kk) * 512 + col * 4);
        return v;
    }
}

__device__ __forceinline__ int xcd_remap(int wgid, int nwg) {
    const int q = nwg / 8, r = nwg % 8;
    const int xcd = wgid % 8, local = wgid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

template <typename T, typename TO, bool KCA, bool KCB>
__global__ __launch_bounds__(256, 1) void gemm2_kernel(Gemm2Args g) {
    typedef G2<T> C;
    typedef typename Mma<T>::frag F;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave & 1, wn = wave >> 1;
    const int ntm = g.M / 128, ntn = g.N / 128;
    const int nwg = ntm * ntn;
    const int t = xcd_remap(blockIdx.x, nwg);
    const int tm = t / ntn, tn = t % ntn;
    const int m0 = tm * 128, n0 = tn * 128;
    const int kslice = g.K / g.ksplit;
    const int kbeg = blockIdx.z * kslice;
    const int nk = kslice / C::KB;
    const T* A = reinterpret_cast<const T*>(g.A);
    const T* B = reinterpret_cast<const T*>(g.B);

    floatx4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    auto issue = [&](int kt) {
        char* slot = smem + (kt % C::NS) * C::SLOT;
        const int k0 = kbeg + kt * C::KB;
        issue_operand<T, KCA>(A, g.lda, m0, k0, slot, wave, lane);
        issue_operand<T, KCB>(B, g.ldb, n0, k0, slot + C::OPB, wave, lane);
    };
#pragma unroll
    for (int s = 0; s < C::NS - 1; ++s)
        if (s < nk) issue(s);

    for (int kt = 0; kt < nk; ++kt) {
        const int ahead = nk - 1 - kt;          // stages issued after kt (<= NS-2)
        if (ahead >= 2) wait_vm<16>();
        else if (ahead == 1) wait_vm<8>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        if (kt + C::NS - 1 < nk) issue(kt + C::NS - 1);
        const char* slot = smem + (kt % C::NS) * C::SLOT;
        const char* ia = slot;
        const char* ib = slot + C::OPB;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            F a[4], b[4];
#pragma unroll
            for (int f = 0; f < 4; ++f) a[f] = read_frag<T, KCA>(ia, wm * 64 + f * 16, u, lane);
#pragma unroll
            for (int f = 0; f < 4; ++f) b[f] = read_frag<T, KCB>(ib, wn * 64 + f * 16, u, lane);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) Mma<T>::run(acc[i][j], a[i], b[j]);
        }
    }

    // epilogue
    TO* Cp = reinterpret_cast<TO*>(g.C);
    const T* mask = reinterpret_cast<const T*>(g.mask);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = n0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + e;
                float v = g.alpha * acc[i][j][e];
                if (g.ksplit > 1) {
                    if (g.part)
                        g.part[((int64_t)blockIdx.z * g.M + row) * g.N + col] = v;
                    else
                        atomicAdd(reinterpret_cast<float*>(Cp) + (int64_t)row * g.ldc + col, v);
                    continue;
                }
                if (g.beta != 0.f) v += g.beta * g.Cin[(int64_t)row * g.ldcin + col];
                if (g.bias_mode == 1) v += g.bias[col];
                else if (g.bias_mode == 2) v += g.bias[row];
                if (g.relu) v = fmaxf(v, 0.f);
                if (mask && !(to_f(mask[(int64_t)row * g.ldmask + col]) > 0.f)) v = 0.f;
                Cp[(int64_t)row * g.ldc + col] = from_f<TO>(v);
            }
        }
}

template <typename T, typename TO, bool KCA, bool KCB>
static int launch2(const Gemm2Args& g, hipStream_t s) {
    typedef G2<T> C;
    auto k = gemm2_kernel<T, TO, KCA, KCB>;
    static bool attr = false;
    if (!attr) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)k,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           C::NS * C::SLOT));
        attr = true;
    }
    dim3 grid((g.M / 128) * (g.N / 128), 1, g.ksplit);
    hipLaunchKernelGGL(k, grid, dim3(256), C::NS * C::SLOT, s, g);
    SRNN_LAUNCH_CHECK();
    return 0;
}

template <typename T, typename TO>
static int launch2_layout(const Gemm2Args& g, bool kca, bool kcb, hipStream_t s) {
    if (kca && kcb) return launch2<T, TO, true, true>(g, s);
    if (kca && !kcb) return launch2<T, TO, true, false>(g, s);
    if (!kca && kcb) return launch2<T, TO, false, true>(g, s);
    return launch2<T, TO, false, false>(g, s);
}

// Returns -1 if the shape/layout is not eligible (caller falls back to the general
// kernel), else the launch status.
int srnn_gemm2_try(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                   float alpha, const void* A, int64_t lda, const void* B, int64_t ldb,
                   float beta, const float* Cin, int64_t ldcin, void* C, int64_t ldc,
                   const float* bias, int bias_mode, int relu, const void* mask, int64_t ldmask,
                   hipStream_t s) {
    const int es = dtype == SRNN_F32 ? 4 : 2;
    const int KB = 128 / es;
    if (M % 128 || N % 128 || K % KB || K == 0) return -1;
    auto al = [&](const void* p, int64_t ld) {
        return ((uintptr_t)p % 16 == 0) && ((ld * es) % 16 == 0);
    };
    if (!al(A, lda) || !al(B, ldb)) return -1;
    Gemm2Args g;
    g.A = A; g.B = B; g.C = C; g.Cin = Cin; g.bias = bias; g.mask = mask;
    g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldcin = ldcin; g.ldmask = ldmask;
    g.M = M; g.N = N; g.K = K; g.alpha = alpha; g.beta = beta;
    g.bias_mode = bias ? bias_mode : 0; g.relu = relu;
    // split K when the tile grid cannot fill the chip (wgrad shapes: K = B*T rows)
    const int tiles = (M / 128) * (N / 128);
    int ks = 1;
    const bool plain = beta == 0.f && !bias && !relu && !mask && out_dtype == SRNN_F32;
    if (plain) {
        while (tiles * ks < 512 && (K / (ks * 2)) % KB == 0 && K / (ks * 2) >= 8 * KB) ks *= 2;
    }
    g.ksplit = ks;
    g.part = nullptr;
    // split K deterministically (partials + ordered sum, as gemm3) where C allows the float4
    // sum; fp32 atomics otherwise (SRNN_G3_SPLITK_PART=0 forces them)
    const bool det = ks > 1 && env_flag("SRNN_G3_SPLITK_PART", 1) && ldc % 4 == 0 &&
                     (uintptr_t)C % 16 == 0;
    if (det) {
        g.part = srnn_splitk_scratch((size_t)ks * M * N * sizeof(float));
        SRNN_REQUIRE(g.part, "gemm2: split-K scratch allocation failed");
        const int rc = dtype == SRNN_F32 ? launch2_layout<float, float>(g, !transA, transB, s)
                                         : launch2_layout<bf16, float>(g, !transA, transB, s);
        if (rc) return rc;
        return srnn_splitk_sum(g.part, (float*)C, ldc, M, N, ks, s);
    }
    if (ks > 1) {
        if (ldc == N) {
            SRNN_CHECK_HIP(hipMemsetAsync(C, 0, (size_t)M * N * 4, s));
        } else {
            SRNN_CHECK_HIP(hipMemset2DAsync(C, ldc * 4, 0, (size_t)N * 4, M, s));
        }
    }
    const bool kca = !transA, kcb = transB;
    if (dtype == SRNN_F32) {
        if (out_dtype == SRNN_F32) return launch2_layout<float, float>(g, kca, kcb, s);
        return launch2_layout<float, bf16>(g, kca, kcb, s);
    }
    if (out_dtype == SRNN_F32) return launch2_layout<bf16, float>(g, kca, kcb, s);
    return launch2_layout<bf16, bf16>(g, kca, kcb, s);
}
