// General MFMA GEMM with fused epilogue:  C = act(alpha * op(A) op(B) + beta * Cin + bias)
// Used for every dense projection of the SampleRNN hot path (tier input_expand /
// cond_expand / spk_expand conv-k1, GRU input projection, LearnedUpsampling1d, the
// MLP hidden/output conv-k1 layers) and their backward dgrad/wgrad products.
#include "gemm_core.hpp"
#include "ring_core.hpp"
#include "samplernn_hip_internal.hpp"

struct GemmArgs {
    const void* A;
    const void* B;
    void* C;
    const float* Cin;
    const float* bias;
    int64_t lda, ldb, ldc, ldcin;
    int64_t sA, sB, sC, sCin;
    int M, N, K;
    float alpha, beta;
    int bias_mode;  // 0 none, 1 per column, 2 per row
    int relu;
    int vecA, vecB;
    const void* mask;  // optional relu-backward mask (input dtype): out = 0 where mask <= 0
    int64_t ldmask;
    unsigned long long* diag;   // skinny path timing diagnostics (workgroup 0, wave 0), or null
    int vecC;          // skinny path: C (and Cin / bias / mask) allow 4-column vector access
};

template <typename T, typename TO, int BM, int BN, int KS, int WM, int WN, int WK, bool KCA,
          bool KCB>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
    typedef GemmCfg<T, BM, BN, KS, WM, WN, WK> C;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int bz = blockIdx.z;
    const T* A = reinterpret_cast<const T*>(g.A) + (int64_t)bz * g.sA;
    const T* B = reinterpret_cast<const T*>(g.B) + (int64_t)bz * g.sB;
    TO* Cp = reinterpret_cast<TO*>(g.C) + (int64_t)bz * g.sC;
    const float* Cin = g.Cin ? g.Cin + (int64_t)bz * g.sCin : nullptr;
    const T* mask = g.mask ? reinterpret_cast<const T*>(g.mask) + (int64_t)bz * g.sC : nullptr;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    floatx4 acc[C::FM][C::FN];
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    gemm_core<T, BM, BN, KS, WM, WN, WK, KCA, KCB>(
        A, g.lda, RowIdentity{m0, g.M}, m0, g.M, g.vecA != 0, B, g.ldb, RowIdentity{n0, g.N}, n0,
        g.N, g.vecB != 0, g.K, smem, acc);
    wk_reduce<T, BM, BN, KS, WM, WN, WK>(smem, acc);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = wave % WM, wn = (wave / WM) % WN, wk = wave / (WM * WN);
    if (wk != 0) return;
#pragma unroll
    for (int fm = 0; fm < C::FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < C::FN; ++fn) {
            const int col = n0 + wn * C::FN * 16 + fn * 16 + (lane & 15);
            if (col >= g.N) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = m0 + wm * C::FM * 16 + fm * 16 + (lane >> 4) * 4 + i;
                if (row >= g.M) continue;
                float v = g.alpha * acc[fm][fn][i];
                if (g.beta != 0.f) v += g.beta * Cin[(int64_t)row * g.ldcin + col];
                if (g.bias_mode == 1) v += g.bias[col];
                else if (g.bias_mode == 2) v += g.bias[row];
                if (g.relu) v = fmaxf(v, 0.f);
                if (mask && !(to_f(mask[(int64_t)row * g.ldmask + col]) > 0.f))
                    v = 0.f;
                Cp[(int64_t)row * g.ldc + col] = from_f<TO>(v);
            }
        }
}

// Skinny NT path (M = batch rows, e.g. the generation loop's y = x W^T with M = 128):
// small tiles so >= 256 workgroups exist, and the deep glds ring of ring_core.hpp so a
// workgroup's K chain is not one exposed memory latency per stage.
template <typename T, typename TO, int BM, int BN, int WM, int WN, int WK, int NS = 4,
          int AUXB = 0>
__global__ __launch_bounds__(256) void skinny_kernel(GemmArgs g) {
    typedef Ring<T, BM, BN, WM, WN, WK, NS> R;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    floatx4 acc[R::FM][R::FN];
#pragma unroll
    for (int i = 0; i < R::FM; ++i)
#pragma unroll
        for (int j = 0; j < R::FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    unsigned long long* st = (g.diag && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
                                 ? g.diag : nullptr;
    if (st) st[0] = __builtin_amdgcn_s_memrealtime();
    ring_core<T, BM, BN, WM, WN, WK, NS, RowClamp, RowClamp, AUXB>(
        (const T*)g.A, g.lda, RowClamp{m0, g.M}, (const T*)g.B, g.ldb, RowClamp{n0, g.N}, g.K,
        smem, acc, st);
    ring_reduce<T, BM, BN, WM, WN, WK, NS>(smem, acc);
    if (st) st[31] = __builtin_amdgcn_s_memrealtime();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = wave % WM, wn = (wave / WM) % WN, wk = wave / (WM * WN);
    TO* Cp = reinterpret_cast<TO*>(g.C);
    const T* mask = reinterpret_cast<const T*>(g.mask);
    if (g.vecC) {
        // Staged epilogue: the tile goes through LDS (the ring is free) so the stores are
        // whole row segments, 4 columns per lane (16 B fp32 / 8 B bf16), instead of 4-byte
        // scalars scattered over 4 rows per instruction (5.8 of 14.8 us at 128 x 16384 x 1024)
        constexpr int P = BN + 4;                   // LDS pitch (floats): 4 rows apart -> +16 banks
        static_assert(BM * P * 4 <= R::LDS, "staged epilogue tile must fit the ring");
        float* Tl = reinterpret_cast<float*>(smem);
        if (wk == 0) {
#pragma unroll
            for (int fm = 0; fm < R::FM; ++fm)
#pragma unroll
                for (int fn = 0; fn < R::FN; ++fn)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        Tl[(wm * R::FM * 16 + fm * 16 + (lane >> 4) * 4 + i) * P + wn * R::FN * 16 +
                           fn * 16 + (lane & 15)] = g.alpha * acc[fm][fn][i];
        }
        __syncthreads();
        if (!mask) {
            // every load the epilogue needs (bias, Cin) is issued before the first store: vmcnt
            // is in order, so a load waited for between stores also waits for every older
            // store (10 serialised store round trips per tile at BN = 80: 3.8 of 13.4 us)
            constexpr int IT = (BM * BN / 4 + 255) / 256;
            // (raw operands: the arithmetic below is the same expression, in the same order,
            //  as the mask path's, so both round alike)
            floatx4 cin[IT], bq[IT];
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int e = threadIdx.x + it * 256;
                const int r = e / (BN / 4), c = (e % (BN / 4)) * 4;
                const int row = m0 + r, col = n0 + c;
                cin[it] = bq[it] = floatx4{0.f, 0.f, 0.f, 0.f};
                if (e < BM * BN / 4 && row < g.M && col < g.N) {
                    if (g.beta != 0.f)
                        cin[it] = *reinterpret_cast<const floatx4*>(g.Cin + (int64_t)row * g.ldcin + col);
                    if (g.bias_mode == 1) bq[it] = *reinterpret_cast<const floatx4*>(g.bias + col);
                    else if (g.bias_mode == 2) bq[it] = floatx4{1.f, 1.f, 1.f, 1.f} * g.bias[row];
                }
            }
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int e = threadIdx.x + it * 256;
                const int r = e / (BN / 4), c = (e % (BN / 4)) * 4;
                const int row = m0 + r, col = n0 + c;
                if (e >= BM * BN / 4 || row >= g.M || col >= g.N) continue;
                floatx4 v = *reinterpret_cast<const floatx4*>(Tl + r * P + c);
                if (g.beta != 0.f) v += g.beta * cin[it];
                if (g.bias_mode == 1) v += bq[it];
                else if (g.bias_mode == 2) v += bq[it][0];
                if (g.relu) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
                }
                TO* cp = Cp + (int64_t)row * g.ldc + col;
                if constexpr (sizeof(TO) == 4) {
                    *reinterpret_cast<floatx4*>(cp) = v;
                } else {
                    const uint32_t lo = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[0])) |
                                        ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[1])) << 16);
                    const uint32_t hi = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[2])) |
                                        ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[3])) << 16);
                    *reinterpret_cast<uint2*>(cp) = make_uint2(lo, hi);
                }
            }
            if (st) st[32] = __builtin_amdgcn_s_memrealtime();
            return;
        }
        for (int e = threadIdx.x; e < BM * BN / 4; e += 256) {
            const int r = e / (BN / 4), c = (e % (BN / 4)) * 4;
            const int row = m0 + r, col = n0 + c;
            if (row >= g.M || col >= g.N) continue;     // N % 4 == 0: a quad is in or out
            floatx4 v = *reinterpret_cast<const floatx4*>(Tl + r * P + c);
            if (g.beta != 0.f) {
                const floatx4 ci = *reinterpret_cast<const floatx4*>(g.Cin + (int64_t)row * g.ldcin + col);
                v += g.beta * ci;
            }
            if (g.bias_mode == 1) v += *reinterpret_cast<const floatx4*>(g.bias + col);
            else if (g.bias_mode == 2) v += g.bias[row];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (g.relu) v[j] = fmaxf(v[j], 0.f);
                if (mask && !(to_f(mask[(int64_t)row * g.ldmask + col + j]) > 0.f)) v[j] = 0.f;
            }
            TO* cp = Cp + (int64_t)row * g.ldc + col;
            if constexpr (sizeof(TO) == 4) {
                *reinterpret_cast<floatx4*>(cp) = v;
            } else {
                const uint32_t lo = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[0])) |
                                    ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[1])) << 16);
                const uint32_t hi = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[2])) |
                                    ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[3])) << 16);
                *reinterpret_cast<uint2*>(cp) = make_uint2(lo, hi);
            }
        }
        if (st) st[32] = __builtin_amdgcn_s_memrealtime();
        return;
    }
    if (wk != 0) return;
#pragma unroll
    for (int fm = 0; fm < R::FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < R::FN; ++fn) {
            const int col = n0 + wn * R::FN * 16 + fn * 16 + (lane & 15);
            if (col >= g.N) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = m0 + wm * R::FM * 16 + fm * 16 + (lane >> 4) * 4 + i;
                if (row >= g.M) continue;
                float v = g.alpha * acc[fm][fn][i];
                if (g.beta != 0.f) v += g.beta * g.Cin[(int64_t)row * g.ldcin + col];
                if (g.bias_mode == 1) v += g.bias[col];
                else if (g.bias_mode == 2) v += g.bias[row];
                if (g.relu) v = fmaxf(v, 0.f);
                if (mask && !(to_f(mask[(int64_t)row * g.ldmask + col]) > 0.f)) v = 0.f;
                Cp[(int64_t)row * g.ldc + col] = from_f<TO>(v);
            }
        }
    if (st) st[32] = __builtin_amdgcn_s_memrealtime();
}

// SRNN_SKINNY_DIAG=1: stage timestamps of workgroup 0 of every skinny launch into a device
// buffer (the last launch wins) that srnn_skinny_diag_dump prints (timing diagnostics only)
static unsigned long long* skinny_diag() {
    static unsigned long long* d = nullptr;
    static int armed = -1;
    if (armed < 0) {
        armed = env_flag("SRNN_SKINNY_DIAG", 0);
        if (armed && hipMalloc(&d, 64 * 8) != hipSuccess) d = nullptr;
        if (d) (void)hipMemset(d, 0, 64 * 8);
    }
    return d;
}

extern "C" int srnn_skinny_diag_dump(void) {
    unsigned long long h[64];
    unsigned long long* d = skinny_diag();
    if (!d || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
        return 1;
    fprintf(stderr, "skinny diag (us from workgroup 0 start):");
    for (int k = 1; k <= 32; ++k)
        if (h[k]) fprintf(stderr, " %d:%.2f", k, (double)(h[k] - h[0]) / 100.0);
    fprintf(stderr, "\n");
    return 0;
}

// all M (<= 128) rows in one tile, so every weight row streams through the chip ONCE (the
// generation loop's upsampling, 128 x 16384 x 1024): 128 x 64 tiles with a 3-stage ring
// (144 KiB) when that still gives >= 256 tiles, else 128 x 32 with 4 stages (160 KiB)
template <typename T, typename TO, int BN, int WM, int WN, int NS>
static int launch_skinny_rows(const GemmArgs& g, hipStream_t s) {
    typedef Ring<T, 128, BN, WM, WN, 1, NS> R;
    // SRNN_SKINNY_NT=1: every weight row is read by exactly one workgroup, once, so the
    // weights may take non-temporal loads (MI355X guide 'nt-weights'); measured in the
    // generation loop's replayed ticks it is slower (16.2 -> 17.1 us for 128 x 19456 x 1024)
    // and leaves the persistent loop's prologue unchanged, so the default policy stays
    static const bool nt = env_flag("SRNN_SKINNY_NT", 0) != 0;
    auto k = nt ? skinny_kernel<T, TO, 128, BN, WM, WN, 1, NS, 2>
                : skinny_kernel<T, TO, 128, BN, WM, WN, 1, NS>;
    static bool attr[2] = {false, false};
    if (!attr[nt]) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)k,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, R::LDS));
        attr[nt] = true;
    }
    hipLaunchKernelGGL(k, dim3(cdiv(g.N, BN), 1), dim3(256), R::LDS, s, g);
    SRNN_LAUNCH_CHECK();
    return 0;
}

template <typename T, typename TO>
static int launch_skinny(const GemmArgs& g, hipStream_t s) {
    if (g.M > 64 && g.M <= 128 && g.N >= 64 * 64 && env_flag("SRNN_SKINNY_ROWS", 1)) {
        // the narrowest tile that keeps it to one round of <= 256 workgroups (the generation
        // ticks: N = 4 D top upsampling, 12 D folded upper tick, 16 D / 19 D bottom tick)
        if (cdiv(g.N, 32) <= 256) return launch_skinny_rows<T, TO, 32, 4, 1, 4>(g, s);
        if (cdiv(g.N, 48) <= 256) return launch_skinny_rows<T, TO, 48, 4, 1, 3>(g, s);
        if (cdiv(g.N, 64) <= 256 || cdiv(g.N, 80) > 256)
            return launch_skinny_rows<T, TO, 64, 2, 2, 3>(g, s);
        return launch_skinny_rows<T, TO, 80, 4, 1, 3>(g, s);
    }
    // 32 x 16 tiles (waves: 2 along M, 2 along K) unless 32 x 32 already gives 512 tiles
    const int64_t t32 = (int64_t)cdiv(g.M, 32) * cdiv(g.N, 32);
    if (t32 >= 512) {
        typedef Ring<T, 32, 32, 2, 2, 1, 4> R;
        dim3 grid(cdiv(g.N, 32), cdiv(g.M, 32));
        hipLaunchKernelGGL((skinny_kernel<T, TO, 32, 32, 2, 2, 1>), grid, dim3(256), R::LDS, s, g);
    } else {
        typedef Ring<T, 32, 16, 2, 1, 2, 4> R;
        dim3 grid(cdiv(g.N, 16), cdiv(g.M, 32));
        hipLaunchKernelGGL((skinny_kernel<T, TO, 32, 16, 2, 1, 2>), grid, dim3(256), R::LDS, s, g);
    }
    SRNN_LAUNCH_CHECK();
    return 0;
}

template <typename T, typename TO, int BM, int BN, int KS, int WM, int WN, int WK, bool KCA,
          bool KCB>
static int launch_t(const GemmArgs& g, int batch, hipStream_t s) {
    typedef GemmCfg<T, BM, BN, KS, WM, WN, WK> C;
    dim3 grid(cdiv(g.N, BN), cdiv(g.M, BM), batch);
    auto k = gemm_kernel<T, TO, BM, BN, KS, WM, WN, WK, KCA, KCB>;
    static bool attr_set = false;
    if (!attr_set && C::LDS > 65536) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)k,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS));
    }
    attr_set = true;
    hipLaunchKernelGGL(k, grid, dim3(256), C::LDS, s, g);
    SRNN_LAUNCH_CHECK();
    return 0;
}

template <typename T, typename TO, bool KCA, bool KCB>
static int launch_layout(const GemmArgs& g, int batch, int tile, hipStream_t s) {
    switch (tile) {
    case 0:  return launch_t<T, TO, 128, 128, 2, 2, 2, 1, KCA, KCB>(g, batch, s);
    case 1:  return launch_t<T, TO, 64, 64, 4, 2, 2, 1, KCA, KCB>(g, batch, s);
    default: return launch_t<T, TO, 32, 32, 4, 1, 1, 4, KCA, KCB>(g, batch, s);
    }
}

template <typename T, typename TO>
static int launch_types(const GemmArgs& g, int transA, int transB, int batch, int tile,
                        hipStream_t s) {
    const bool kca = !transA, kcb = transB;
    if (kca && kcb) return launch_layout<T, TO, true, true>(g, batch, tile, s);
    if (kca && !kcb) return launch_layout<T, TO, true, false>(g, batch, tile, s);
    if (!kca && kcb) return launch_layout<T, TO, false, true>(g, batch, tile, s);
    return launch_layout<T, TO, false, false>(g, batch, tile, s);
}

int srnn_gemm2_try(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                   float alpha, const void* A, int64_t lda, const void* B, int64_t ldb,
                   float beta, const float* Cin, int64_t ldcin, void* C, int64_t ldc,
                   const float* bias, int bias_mode, int relu, const void* mask, int64_t ldmask,
                   hipStream_t s);

int srnn_gemm3_try(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                   float alpha, const void* A, int64_t lda, const void* B, int64_t ldb,
                   float beta, const float* Cin, int64_t ldcin, void* C, int64_t ldc,
                   const float* bias, int bias_mode, int relu, const void* mask, int64_t ldmask,
                   int force, hipStream_t s, const unsigned short* mbi = nullptr,
                   int64_t ldmbi = 0, unsigned short* mbo = nullptr, int64_t ldmbo = 0);

int srnn_gemm_small_try(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                        float alpha, const void* A, int64_t lda, const void* B, int64_t ldb,
                        float beta, const float* Cin, int64_t ldcin, void* C, int64_t ldc,
                        const float* bias, int bias_mode, int relu, const void* mask,
                        hipStream_t s);

static bool env_on(const char* name) {
    const char* e = getenv(name);
    return !(e && e[0] == '0');
}

static bool g_use_gemm2() {
    static int v = -1;
    if (v < 0) v = env_on("SRNN_GEMM2") ? 1 : 0;
    return v == 1;
}

static bool g_use_gemm3() {
    static int v = -1;
    if (v < 0) v = env_on("SRNN_GEMM3") ? 1 : 0;
    return v == 1;
}

static int pick_tile(int M, int N, int batch) {
    const int64_t t128 = (int64_t)cdiv(M, 128) * cdiv(N, 128) * batch;
    if (t128 >= 256) return 0;
    const int64_t t64 = (int64_t)cdiv(M, 64) * cdiv(N, 64) * batch;
    if (t64 >= 192) return 1;
    return 2;
}

static int gemm_core(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                     float alpha, const void* A, int64_t lda, int64_t strideA, const void* B,
                     int64_t ldb, int64_t strideB, float beta, const float* Cin, int64_t ldcin,
                     int64_t strideCin, void* C, int64_t ldc, int64_t strideC,
                     const float* bias, int bias_mode, int relu, int batch, int tile,
                     hipStream_t s, const void* mask, int64_t ldmask);

// ---- ReLU masks as bits: bit c % 16 of the u16 of (row, column group c / 16) = (value(row,
// c) > 0).  Two layouts (srnn_bits_index): row-major, u16 [row][c / 16] with row stride ldb;
// or, ldb = 0, grouped: column-group-major u16 [c / 16][row] (N % 64 == 0) -- the L1 kernel's
// 16-column workgroups write consecutive rows as one contiguous run, and a GEMM tile's rows
// of a column group are contiguous for its LDS-DMA staging (gemm3.hip)
// (one thread per 16-column group; a column group past N contributes zero bits; grouped:
//  consecutive threads take consecutive rows)
template <typename T>
__global__ void relu_bits_kernel(const T* __restrict__ a, int64_t lda, int M, int N,
                                 unsigned short* __restrict__ bits, int64_t ldb) {
    const int ng = (N + 15) / 16;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)M * ng) return;
    const int r = ldb ? (int)(e / ng) : (int)(e % M);
    const int c0 = (ldb ? (int)(e % ng) : (int)(e / M)) * 16;
    unsigned w = 0u;
    for (int c = 0; c < 16 && c0 + c < N; ++c)
        w |= (to_f(a[(int64_t)r * lda + c0 + c]) > 0.f ? 1u : 0u) << c;
    bits[srnn_bits_index(r, c0 / 16, M, ldb)] = (unsigned short)w;
}

// the bits as a mask tensor of the GEMM input dtype (1 / 0), for the paths without bit input
template <typename T>
__global__ void bits_expand_kernel(const unsigned short* __restrict__ bits, int64_t ldb, int M,
                                   int N, T* __restrict__ m, int64_t ldm) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)M * N) return;
    const int r = (int)(e / N), c = (int)(e % N);
    m[(int64_t)r * ldm + c] =
        from_f<T>((float)((bits[srnn_bits_index(r, c / 16, M, ldb)] >> (c & 15)) & 1u));
}

int srnn_relu_bits_impl(int dtype, const void* a, int64_t lda, int M, int N, unsigned short* bits,
                        int64_t ldb, hipStream_t s) {
    SRNN_REQUIRE(M >= 0 && N >= 0 && bits && (ldb >= (N + 15) / 16 || (ldb == 0 && N % 64 == 0)),
                 "relu_bits: bad args (row stride >= N / 16, or 0 for the grouped layout with "
                 "N % 64 == 0)");
    const int64_t n = (int64_t)M * ((N + 15) / 16);
    if (n == 0) return 0;
    if (dtype == SRNN_F32)
        hipLaunchKernelGGL((relu_bits_kernel<float>), dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                           s, (const float*)a, lda, M, N, bits, ldb);
    else
        hipLaunchKernelGGL((relu_bits_kernel<bf16>), dim3((unsigned)cdiv(n, 256)), dim3(256), 0,
                           s, (const bf16*)a, lda, M, N, bits, ldb);
    SRNN_LAUNCH_CHECK();
    return 0;
}

extern "C" int srnn_relu_bits(int dtype, const void* a, int64_t lda, int M, int N,
                              unsigned short* bits, int64_t ldb, void* stream) {
    return srnn_relu_bits_impl(dtype, a, lda, M, N, bits, ldb, (hipStream_t)stream);
}

int srnn_gemm_impl(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                   float alpha, const void* A, int64_t lda, int64_t strideA, const void* B,
                   int64_t ldb, int64_t strideB, float beta, const float* Cin, int64_t ldcin,
                   int64_t strideCin, void* C, int64_t ldc, int64_t strideC, const float* bias,
                   int bias_mode, int relu, int batch, int tile, hipStream_t s,
                   const void* mask, int64_t ldmask, const unsigned short* mbi, int64_t ldmbi,
                   unsigned short* mbo, int64_t ldmbo) {
    if (!mbi && !mbo)
        return gemm_core(dtype, out_dtype, transA, transB, M, N, K, alpha, A, lda, strideA, B,
                         ldb, strideB, beta, Cin, ldcin, strideCin, C, ldc, strideC, bias,
                         bias_mode, relu, batch, tile, s, mask, ldmask);
    SRNN_REQUIRE(batch == 1 && !(mbi && mask), "gemm: bit masks need batch 1 and no bf16 mask");
    SRNN_REQUIRE(!(mbi && ldmbi == 0) || N % 64 == 0, "gemm: grouped mask bits need N % 64 == 0");
    SRNN_REQUIRE(!(mbo && ldmbo == 0) || N % 64 == 0, "gemm: grouped mask bits need N % 64 == 0");
    if (M == 0 || N == 0) return 0;
    // the 256-tile kernel reads / writes the bits in its epilogue
    if ((tile < 0 || tile == 5) && (tile == 5 || g_use_gemm3())) {
        const int rc = srnn_gemm3_try(dtype, out_dtype, transA, transB, M, N, K, alpha, A, lda, B,
                                      ldb, beta, Cin, ldcin, C, ldc, bias, bias_mode, relu, mask,
                                      ldmask, tile == 5, s, mbi, ldmbi, mbo, ldmbo);
        if (rc >= 0) return rc;
    }
    // other paths (and gemm3 without the bit epilogue, e.g. fp32 out): the bits as a mask
    // tensor in, the output's bits computed after
    const void* mk = mask;
    int64_t ldmk = ldmask;
    if (mbi) {
        const int es = dtype == SRNN_F32 ? 4 : 2;
        void* scratch = srnn_scratch(SRNN_SCRATCH_MASK, (size_t)M * N * es);
        SRNN_REQUIRE(scratch, "gemm: mask scratch allocation failed");
        const int64_t n = (int64_t)M * N;
        if (dtype == SRNN_F32)
            hipLaunchKernelGGL((bits_expand_kernel<float>), dim3((unsigned)cdiv(n, 256)), dim3(256),
                               0, s, mbi, ldmbi, M, N, (float*)scratch, (int64_t)N);
        else
            hipLaunchKernelGGL((bits_expand_kernel<bf16>), dim3((unsigned)cdiv(n, 256)), dim3(256),
                               0, s, mbi, ldmbi, M, N, (bf16*)scratch, (int64_t)N);
        SRNN_LAUNCH_CHECK();
        mk = scratch;
        ldmk = N;
    }
    int rc = gemm_core(dtype, out_dtype, transA, transB, M, N, K, alpha, A, lda, strideA, B, ldb,
                       strideB, beta, Cin, ldcin, strideCin, C, ldc, strideC, bias, bias_mode,
                       relu, batch, tile, s, mk, ldmk);
    if (rc || !mbo) return rc;
    return srnn_relu_bits_impl(out_dtype, C, ldc, M, N, mbo, ldmbo, s);
}

static int gemm_core(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                     float alpha, const void* A, int64_t lda, int64_t strideA, const void* B,
                     int64_t ldb, int64_t strideB, float beta, const float* Cin, int64_t ldcin,
                     int64_t strideCin, void* C, int64_t ldc, int64_t strideC,
                     const float* bias, int bias_mode, int relu, int batch, int tile,
                     hipStream_t s, const void* mask, int64_t ldmask) {
    SRNN_REQUIRE(M >= 0 && N >= 0 && K >= 0 && batch >= 1, "gemm: bad sizes");
    SRNN_REQUIRE(dtype == SRNN_F32 || dtype == SRNN_BF16, "gemm: bad dtype %d", dtype);
    SRNN_REQUIRE(out_dtype == SRNN_F32 || out_dtype == SRNN_BF16, "gemm: bad out dtype");
    SRNN_REQUIRE(!(beta != 0.f && Cin == nullptr), "gemm: beta != 0 needs Cin");
    if (M == 0 || N == 0) return 0;
    const int es = dtype == SRNN_F32 ? 4 : 2;
    const int E = 16 / es;
    GemmArgs g;
    g.A = A; g.B = B; g.C = C; g.Cin = Cin; g.bias = bias;
    g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldcin = ldcin;
    g.sA = strideA; g.sB = strideB; g.sC = strideC; g.sCin = strideCin;
    g.M = M; g.N = N; g.K = K; g.alpha = alpha; g.beta = beta;
    g.bias_mode = bias ? bias_mode : 0; g.relu = relu;
    g.mask = mask; g.ldmask = ldmask;
    g.diag = skinny_diag();
    {
        // 4-column vector epilogue (skinny path): every row of C (and Cin, mask) starts on a
        // 4-element boundary and N is whole quads
        const int eo = out_dtype == SRNN_F32 ? 4 : 2;
        auto al = [](const void* p, int64_t ld, int b) {
            return p == nullptr || (((uintptr_t)p % b == 0) && (ld % 4 == 0));
        };
        g.vecC = N % 4 == 0 && al(C, ldc, 4 * eo) && (beta == 0.f || al(Cin, ldcin, 16)) &&
                 (bias == nullptr || bias_mode != 1 || (uintptr_t)bias % 16 == 0) &&
                 al(mask, ldmask, 4 * es) && batch == 1 && env_flag("SRNN_SKINNY_VEC", 1);
    }
    auto aligned = [&](const void* p, int64_t ld, int64_t st) {
        return ((uintptr_t)p % 16 == 0) && (ld % E == 0) && (batch == 1 || st % E == 0);
    };
    g.vecA = aligned(A, lda, strideA);
    g.vecB = aligned(B, ldb, strideB);
    // thin problems (N <= 64 weight gradients, K <= 64 input projections); tile 6 forces
    if ((tile < 0 || tile == 6) && batch == 1) {
        int rc = srnn_gemm_small_try(dtype, out_dtype, transA, transB, M, N, K, alpha, A, lda, B,
                                     ldb, beta, Cin, ldcin, C, ldc, bias, bias_mode, relu, mask, s);
        if (rc >= 0) return rc;
        SRNN_REQUIRE(tile != 6, "gemm: shape not eligible for the thin path");
    }
    // skinny NT problems (M = batch rows): small-tile deep-ring kernel; tile 4 forces it.
    // Up to 512 rows: the reverse sweep's dh_0 = dgh_0 W_hh + dh_direct at 512 rows (512 x 1024
    // x 3072 with Cin) 55 -> 13.4 us against the 128-tile kernel it fell to above 256 rows
    // (tools/gemm_route_probe.py, profiles/r06_gemm_route_b512.txt)
    {
        const int KBr = 256 / es;
        const bool ok = batch == 1 && !transA && transB && K % KBr == 0 && K > 0 && g.vecA &&
                        g.vecB && ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0);
        if ((tile == 4 || (tile < 0 && M <= 512 && g_use_gemm2())) && ok) {
            if (dtype == SRNN_F32)
                return out_dtype == SRNN_F32 ? launch_skinny<float, float>(g, s)
                                             : launch_skinny<float, bf16>(g, s);
            return out_dtype == SRNN_F32 ? launch_skinny<bf16, float>(g, s)
                                         : launch_skinny<bf16, bf16>(g, s);
        }
        SRNN_REQUIRE(tile != 4, "gemm: shape not eligible for the skinny path");
    }
    // large plain bf16 problems: hipBLASLt (blaslt.cpp) unless a fused epilogue or a pending
    // max |C| / column-sum request needs gemm3; strided batches too (the folded
    // embedding . conv table, 16 x (256 x 1024 x 256) with the embedding shared: 33 us on the
    // 128-tile kernel per step at every batch size)
    if (tile < 0 && !mask && !srnn_gemm_amax_pending() && !srnn_gemm_csum_pending() &&
        !srnn_gemm_lsm_pending()) {
        int rc = srnn_blaslt_try(dtype, out_dtype, transA, transB, M, N, K, alpha, A, lda, B, ldb,
                                 beta, C, ldc, bias, bias_mode, relu, s, batch, strideA, strideB,
                                 strideC);
        if (rc >= 0) return rc;
    }
    // large aligned bf16 problems: the 256x256 8-wave kernel (gemm3.hip); tile 5 forces it
    if ((tile < 0 || tile == 5) && batch == 1 && (tile == 5 || g_use_gemm3())) {
        int rc = srnn_gemm3_try(dtype, out_dtype, transA, transB, M, N, K, alpha, A, lda, B, ldb,
                                beta, Cin, ldcin, C, ldc, bias, bias_mode, relu, mask, ldmask,
                                tile == 5, s);
        if (rc >= 0) return rc;
        SRNN_REQUIRE(tile != 5, "gemm: shape not eligible for the gemm3 path");
    }
    // large aligned problems: the glds-ring kernel (gemm2.hip); tile 3 forces it
    if ((tile < 0 || tile == 3) && batch == 1 && g_use_gemm2()) {
        int rc = srnn_gemm2_try(dtype, out_dtype, transA, transB, M, N, K, alpha, A, lda, B, ldb,
                                beta, Cin, ldcin, C, ldc, bias, bias_mode, relu, mask, ldmask, s);
        if (rc >= 0) return rc;
        SRNN_REQUIRE(tile != 3, "gemm: shape not eligible for the gemm2 path");
    }
    if (tile < 0 || tile == 3) tile = pick_tile(M, N, batch);
    if (dtype == SRNN_F32) {
        if (out_dtype == SRNN_F32) return launch_types<float, float>(g, transA, transB, batch, tile, s);
        return launch_types<float, bf16>(g, transA, transB, batch, tile, s);
    }
    if (out_dtype == SRNN_F32) return launch_types<bf16, float>(g, transA, transB, batch, tile, s);
    return launch_types<bf16, bf16>(g, transA, transB, batch, tile, s);
}

extern "C" int srnn_gemm_bits(int dtype, int out_dtype, int transA, int transB, int M, int N,
                              int K, float alpha, const void* A, int64_t lda, const void* B,
                              int64_t ldb, float beta, const float* Cin, int64_t ldcin, void* C,
                              int64_t ldc, const float* bias, int bias_mode, int relu, int tile,
                              const unsigned short* mask_bits, int64_t ldmb,
                              unsigned short* bits_out, int64_t ldbo, void* stream) {
    return srnn_gemm_impl(dtype, out_dtype, transA, transB, M, N, K, alpha, A, lda, 0, B, ldb, 0,
                          beta, Cin, ldcin, 0, C, ldc, 0, bias, bias_mode, relu, 1, tile,
                          (hipStream_t)stream, nullptr, 0, mask_bits, ldmb, bits_out, ldbo);
}

extern "C" int srnn_gemm(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                         float alpha, const void* A, int64_t lda, int64_t strideA, const void* B,
                         int64_t ldb, int64_t strideB, float beta, const float* Cin, int64_t ldcin,
                         int64_t strideCin, void* C, int64_t ldc, int64_t strideC,
                         const float* bias, int bias_mode, int relu, int batch, int tile,
                         const void* mask, int64_t ldmask, void* stream) {
    return srnn_gemm_impl(dtype, out_dtype, transA, transB, M, N, K, alpha, A, lda, strideA, B,
                          ldb, strideB, beta, Cin, ldcin, strideCin, C, ldc, strideC, bias,
                          bias_mode, relu, batch, tile, (hipStream_t)stream, mask, ldmask);
}
