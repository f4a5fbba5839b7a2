// Thin GEMMs of the TBPTT step that the MFMA tile kernels handle badly: one output
// dimension or the reduction dimension is tiny, so a 32..256-wide tile is mostly padding
// and its K loop is one long dependent chain.
//
//  * small N (N <= 64, B stored K x N): the weight gradients of the input / conditioning /
//    speaker projections (dW = dX^T . input, N = frame samples, cond_dim, spk_dim) with K =
//    all frames of the batch, and the speaker-embedding gradient.  A thread owns one output
//    row m and all N columns in registers; the workgroup's K chunk of B is staged in LDS
//    and read as broadcasts; K is split over workgroups, whose partial rows go to a scratch
//    and are summed in split order by a second kernel (deterministic: no atomics), so the
//    grid fills the chip whatever M is.
//  * small K (K <= 64, NT): the input projections of the tiers (frame samples -> dim,
//    cond_dim -> dim) with the upper-tier conditioning added (beta * Cin) and the bias:
//    a thread computes 4 adjacent columns of one row from LDS-staged rows of A and B, so
//    the Cin read and the C write are coalesced 16-B accesses -- the op is HBM-bound.
#include <algorithm>

#include "samplernn_hip_internal.hpp"

template <typename T>
__device__ __forceinline__ float ldf(const T* p) { return to_f(*p); }

// ---------------------------------------------------------------- small N
// C[m][n] (+)= alpha * sum_k opA[m][k] * B[k][n];  opA = A^T (A stored K x M) if TA
// grid: (M / 256, N / NMAX column groups, K splits).  Each 32-deep k block's A values are
// loaded back to back into registers before the FMAs, so a thread waits one memory
// latency per block, not one per k.
template <typename T, bool TA, int NMAX>
__global__ __launch_bounds__(256) void gemm_small_n_kernel(const T* __restrict__ A, int64_t lda,
                                                           const T* __restrict__ B, int64_t ldb,
                                                           float* __restrict__ C, int64_t ldc,
                                                           int M, int N, int K, int kchunk,
                                                           float alpha, float* __restrict__ P) {
    constexpr int KC = 32;
    __shared__ float bs[KC][NMAX];
    const int m = blockIdx.x * 256 + threadIdx.x;
    const int n0 = blockIdx.y * NMAX;
    const int k0 = blockIdx.z * kchunk;
    const int k1 = min(K, k0 + kchunk);
    const int mm = m < M ? m : M - 1;
    float acc[NMAX];
#pragma unroll
    for (int n = 0; n < NMAX; ++n) acc[n] = 0.f;
    for (int kb = k0; kb < k1; kb += KC) {
        const int kn = min(KC, k1 - kb);
        __syncthreads();
        for (int i = threadIdx.x; i < KC * NMAX; i += 256) {
            const int kk = i / NMAX, n = i % NMAX;
            bs[kk][n] = (kk < kn && n0 + n < N) ? ldf(B + (int64_t)(kb + kk) * ldb + n0 + n) : 0.f;
        }
        float a[KC];
#pragma unroll
        for (int kk = 0; kk < KC; ++kk) {
            const int k = kb + (kk < kn ? kk : 0);
            a[kk] = kk < kn ? (TA ? ldf(A + (int64_t)k * lda + mm) : ldf(A + (int64_t)mm * lda + k))
                            : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < KC; ++kk)
#pragma unroll
            for (int n = 0; n < NMAX; ++n) acc[n] += a[kk] * bs[kk][n];
    }
    if (m >= M) return;
    if (P) {            // split K: this split's partial row, P[z][n][m] (summed in z order)
        float* pp = P + (int64_t)blockIdx.z * N * M + m;
#pragma unroll
        for (int n = 0; n < NMAX; ++n)
            if (n0 + n < N) pp[(int64_t)(n0 + n) * M] = acc[n];
        return;
    }
    float* c = C + (int64_t)m * ldc + n0;
#pragma unroll
    for (int n = 0; n < NMAX; ++n)
        if (n0 + n < N) c[n] = alpha * acc[n];
}

__global__ __launch_bounds__(256) void gemm_small_nt_sum_kernel(const float* __restrict__ P,
                                                                float* __restrict__ C,
                                                                int64_t ldc, int M, int N,
                                                                int nks, float alpha);

template <typename T, bool TA>
static int launch_small_n(const void* A, int64_t lda, const void* B, int64_t ldb, float* C,
                          int64_t ldc, int M, int N, int K, float alpha, hipStream_t s) {
    const int mblk = cdiv(M, 256);
    const int NM = N <= 8 ? 8 : 16;                 // columns per workgroup
    const int ngrp = cdiv(N, NM);
    // split K so that ~1024 workgroups run, each with >= 64 k
    int nks = std::max(1, std::min(cdiv(K, 64), 1024 / (mblk * ngrp)));
    const int kchunk = ((cdiv(K, nks) + 31) / 32) * 32;
    nks = cdiv(K, kchunk);
    float* P = nullptr;
    if (nks > 1) {
        P = (float*)srnn_scratch(SRNN_SCRATCH_NT, (size_t)nks * N * M * sizeof(float));
        SRNN_REQUIRE(P, "gemm_small: split-K scratch allocation failed");
    }
    dim3 grid(mblk, ngrp, nks);
    if (NM == 8)
        hipLaunchKernelGGL((gemm_small_n_kernel<T, TA, 8>), grid, dim3(256), 0, s, (const T*)A,
                           lda, (const T*)B, ldb, C, ldc, M, N, K, kchunk, alpha, P);
    else
        hipLaunchKernelGGL((gemm_small_n_kernel<T, TA, 16>), grid, dim3(256), 0, s, (const T*)A,
                           lda, (const T*)B, ldb, C, ldc, M, N, K, kchunk, alpha, P);
    SRNN_LAUNCH_CHECK();
    if (P) {
        const int64_t tot = (int64_t)M * N;
        hipLaunchKernelGGL(gemm_small_nt_sum_kernel, dim3((unsigned)cdiv(tot, (int64_t)256)),
                           dim3(256), 0, s, P, C, ldc, M, N, nks, alpha);
        SRNN_LAUNCH_CHECK();
    }
    return 0;
}

// ---------------------------------------------------------------- small N, A^T
// The weight-gradient shape (A stored K x M, K = all frames): K is split into chunks, each
// workgroup writes its partial C chunk to a scratch P[z][n][m] with plain stores, and a
// second kernel sums the chunks in a fixed order -- no atomics (a device-scope fp32 atomic
// costs ~60 ns of aggregate throughput here, which made the atomic version ~100 us) and
// the result is deterministic.
// Workgroup: 4 waves x 64 lanes; a lane owns 4 adjacent m (one 8-B / 16-B load per k row)
// and NG = 16 columns; wave w sums k rows [k0 + w * kw, k0 + (w + 1) * kw) of the chunk.
namespace gsn {
constexpr int NG = 16, KR = 16;   // columns per workgroup, k rows per register batch
}

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float (&v)[4]);
template <>
__device__ __forceinline__ void ld4<float>(const float* p, float (&v)[4]) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
}
template <>
__device__ __forceinline__ void ld4<bf16>(const bf16* p, float (&v)[4]) {
    const uint2 x = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
    v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
}

template <typename T>
__global__ __launch_bounds__(256) void gemm_small_nt_part_kernel(
    const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
    float* __restrict__ P, int M, int N, int K, int kchunk) {
    using namespace gsn;
    __shared__ float bs[4][KR][NG];
    __shared__ float4 red[3][NG][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int m = blockIdx.x * 256 + lane * 4;
    const int n0 = blockIdx.y * NG;
    const int kw = kchunk / 4;
    const int kbeg = blockIdx.z * kchunk + wave * kw;
    const int kend = min(K, kbeg + kw);
    const int mm = m < M ? m : 0;
    float acc[4][NG];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int n = 0; n < NG; ++n) acc[j][n] = 0.f;
    for (int kb = kbeg; kb < kend; kb += KR) {
        // this wave's KR x NG slice of B (zero beyond K / N)
#pragma unroll
        for (int i = 0; i < KR * NG / 64; ++i) {
            const int e = i * 64 + lane, kk = e / NG, n = e % NG;
            bs[wave][kk][n] = (kb + kk < kend && n0 + n < N)
                                  ? to_f(B[(int64_t)(kb + kk) * ldb + n0 + n]) : 0.f;
        }
        float a[KR][4];
#pragma unroll
        for (int kk = 0; kk < KR; ++kk) {
            const int k = kb + kk < kend ? kb + kk : kb;
            ld4<T>(A + (int64_t)k * lda + mm, a[kk]);
        }
#pragma unroll
        for (int kk = 0; kk < KR; ++kk)      // rows past the wave's range contribute 0
            if (kb + kk >= kend) a[kk][0] = a[kk][1] = a[kk][2] = a[kk][3] = 0.f;
        __builtin_amdgcn_s_waitcnt(0);   // (one wave owns bs[wave]: no block barrier)
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int kk = 0; kk < KR; ++kk) {
            float b[NG];
#pragma unroll
            for (int n = 0; n < NG; n += 4) {
                const float4 v = *reinterpret_cast<const float4*>(&bs[wave][kk][n]);
                b[n] = v.x; b[n + 1] = v.y; b[n + 2] = v.z; b[n + 3] = v.w;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int n = 0; n < NG; ++n) acc[j][n] += a[kk][j] * b[n];
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (wave > 0) {
#pragma unroll
        for (int n = 0; n < NG; ++n)
            red[wave - 1][n][lane] = make_float4(acc[0][n], acc[1][n], acc[2][n], acc[3][n]);
    }
    __syncthreads();
    if (wave > 0 || m >= M) return;
    float* p = P + (int64_t)blockIdx.z * N * M;
#pragma unroll
    for (int n = 0; n < NG; ++n) {
        if (n0 + n >= N) break;
        float4 v = make_float4(acc[0][n], acc[1][n], acc[2][n], acc[3][n]);
#pragma unroll
        for (int w = 0; w < 3; ++w) {
            const float4 r = red[w][n][lane];
            v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
        }
        *reinterpret_cast<float4*>(p + (int64_t)(n0 + n) * M + m) = v;
    }
}

// C[m][n] = alpha * sum_z P[z][n][m]  (z in order)
__global__ __launch_bounds__(256) void gemm_small_nt_sum_kernel(const float* __restrict__ P,
                                                                float* __restrict__ C,
                                                                int64_t ldc, int M, int N,
                                                                int nks, float alpha) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)M * N) return;
    const int n = (int)(i / M), m = (int)(i % M);
    const int64_t zs = (int64_t)N * M;
    const float* p = P + (int64_t)n * M + m;
    float s = 0.f;
    int z = 0;
    for (; z + 8 <= nks; z += 8) {          // 8 loads in flight, summed in z order
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = p[(z + u) * zs];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; z < nks; ++z) s += p[z * zs];
    C[(int64_t)m * ldc + n] = alpha * s;
}

// Split-K partials of the thin NT path: one grow-only scratch buffer reused by every call
// (stream-ordered on the caller's stream; srnn_scratch).  A stream-ordered hipMallocAsync per
// call cost up to 4 ms of host time per TBPTT step (the 1024 x 64 x 2048 input-projection
// weight gradient), which stalled the launch queue; growth only happens on the first calls.

template <typename T>
static int launch_small_nt(const void* A, int64_t lda, const void* B, int64_t ldb, float* C,
                           int64_t ldc, int M, int N, int K, float alpha, hipStream_t s) {
    const int mblk = cdiv(M, 256), ngrp = cdiv(N, gsn::NG);
    // ~768 workgroups, each wave >= KR rows of k
    int nks = std::max(1, std::min(cdiv(K, 4 * gsn::KR), cdiv(768, mblk * ngrp)));
    const int kchunk = cdiv(cdiv(K, nks), 4 * gsn::KR) * 4 * gsn::KR;
    nks = cdiv(K, kchunk);
    const size_t need = (size_t)nks * N * M * sizeof(float);
    float* P = (float*)srnn_scratch(SRNN_SCRATCH_NT, need);
    SRNN_REQUIRE(P, "gemm_small: split-K scratch allocation failed");
    hipLaunchKernelGGL((gemm_small_nt_part_kernel<T>), dim3(mblk, ngrp, nks), dim3(256), 0, s,
                       (const T*)A, lda, (const T*)B, ldb, P, M, N, K, kchunk);
    SRNN_LAUNCH_CHECK();
    const int64_t tot = (int64_t)M * N;
    hipLaunchKernelGGL(gemm_small_nt_sum_kernel, dim3((unsigned)cdiv(tot, (int64_t)256)),
                       dim3(256), 0, s, P, C, ldc, M, N, nks, alpha);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// ---------------------------------------------------------------- small K (NT)
// C[m][n] = alpha * sum_k A[m][k] * B[n][k] + beta * Cin[m][n] + bias[n]
template <typename T, typename TO, int KMAX>
__global__ __launch_bounds__(256) void gemm_small_k_kernel(
    const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
    TO* __restrict__ C, int64_t ldc, const float* __restrict__ Cin, int64_t ldcin,
    const float* __restrict__ bias, int M, int N, int K, float alpha, float beta, int relu) {
    // block: 16 rows x 256 columns (64 lanes x 4 columns per row, 4 rows per pass)
    __shared__ float as[16][KMAX];
    __shared__ float bs[256][KMAX + 1];
    const int m0 = blockIdx.y * 16, n0 = blockIdx.x * 256;
    for (int i = threadIdx.x; i < 16 * KMAX; i += 256) {
        const int r = i / KMAX, k = i % KMAX;
        as[r][k] = (m0 + r < M && k < K) ? ldf(A + (int64_t)(m0 + r) * lda + k) : 0.f;
    }
    for (int i = threadIdx.x; i < 256 * KMAX; i += 256) {
        const int c = i / KMAX, k = i % KMAX;
        bs[c][k] = (n0 + c < N && k < K) ? ldf(B + (int64_t)(n0 + c) * ldb + k) : 0.f;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const int c = lane * 4;
    for (int r = rg; r < 16; r += 4) {
        const int m = m0 + r;
        if (m >= M) break;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < K; ++k) {
            const float a = as[r][k];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += a * bs[c + e][k];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int n = n0 + c + e;
            if (n >= N) continue;
            float o = alpha * v[e];
            if (beta != 0.f) o += beta * Cin[(int64_t)m * ldcin + n];
            if (bias) o += bias[n];
            if (relu) o = fmaxf(o, 0.f);
            C[(int64_t)m * ldc + n] = from_f<TO>(o);
        }
    }
}

// Tile: 32 rows x 256 columns per workgroup; lane owns 4 adjacent columns of 8 rows (its
// wave's), so the Cin read and the C write are 16-B / 8-B per lane and coalesced; B's 256
// x K slice sits in LDS k-major (one float4 per lane per k), A's 32 x K rows are read as
// broadcasts.  The Cin rows are requested before the staging so their latency overlaps it.
template <typename T>
__device__ __forceinline__ void st4(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <typename T>
__device__ __forceinline__ void st4(bf16* p, const float (&v)[4]) {
    uint2 x;
    x.x = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[0])) |
          ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[1])) << 16);
    x.y = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[2])) |
          ((uint32_t)__bfloat16_as_ushort(__float2bfloat16(v[3])) << 16);
    *reinterpret_cast<uint2*>(p) = x;
}

template <typename T, typename TO, int KMAX>
__global__ __launch_bounds__(256) void gemm_small_k2_kernel(
    const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
    TO* __restrict__ C, int64_t ldc, const float* __restrict__ Cin, int64_t ldcin,
    const float* __restrict__ bias, int M, int N, int K, float alpha, float beta, int relu) {
    __shared__ float4 bsT[KMAX][64];          // [k][column / 4]
    __shared__ float4 as[32][KMAX / 4];       // [row][k / 4]
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 256;
    const int c = n0 + lane * 4;
    const bool cv = c < N;                    // N % 4 == 0 (host-checked)
    float cin[8][4];
    if (beta != 0.f && cv) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int m = min(m0 + wave * 8 + r, M - 1);
            const float4 v = *reinterpret_cast<const float4*>(Cin + (int64_t)m * ldcin + c);
            cin[r][0] = v.x; cin[r][1] = v.y; cin[r][2] = v.z; cin[r][3] = v.w;
        }
    }
    {   // B: thread t loads column n0 + t, all k
        float* bt = reinterpret_cast<float*>(bsT);
        const int n = n0 + tid;
        // loads from clamped addresses, zeroed after the load: a "load or zero" select per
        // element would make the compiler wait for each load in turn (one L2 round trip each)
        const T* bp = B + (int64_t)min(n, N - 1) * ldb;
        const bool nok = n < N;
#pragma unroll 16
        for (int k = 0; k < KMAX; ++k) {
            const float v = to_f(bp[min(k, K - 1)]);
            bt[k * 256 + tid] = (k < K && nok) ? v : 0.f;
        }
        float* at = reinterpret_cast<float*>(as);
#pragma unroll
        for (int i0 = 0; i0 < 32 * KMAX; i0 += 256) {
            const int i = i0 + tid, r = i / KMAX, k = i % KMAX;
            const float v = to_f(A[(int64_t)min(m0 + r, M - 1) * lda + min(k, K - 1)]);
            at[i] = (k < K && m0 + r < M) ? v : 0.f;
        }
    }
    __syncthreads();
    float acc[8][4];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[r][e] = 0.f;
    const int kq = (K + 3) >> 2;
    for (int q = 0; q < kq; ++q) {
        float4 b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) b[i] = bsT[q * 4 + i][lane];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const float4 a = as[wave * 8 + r][q];
            const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                acc[r][0] += av[i] * b[i].x; acc[r][1] += av[i] * b[i].y;
                acc[r][2] += av[i] * b[i].z; acc[r][3] += av[i] * b[i].w;
            }
        }
    }
    if (!cv) return;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (bias) {
        const float4 v = *reinterpret_cast<const float4*>(bias + c);
        bv[0] = v.x; bv[1] = v.y; bv[2] = v.z; bv[3] = v.w;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int m = m0 + wave * 8 + r;
        if (m >= M) break;
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            o[e] = alpha * acc[r][e];
            if (beta != 0.f) o[e] += beta * cin[r][e];
            o[e] += bv[e];
            if (relu) o[e] = fmaxf(o[e], 0.f);
        }
        st4<TO>(C + (int64_t)m * ldc + c, o);
    }
}

template <typename T, typename TO>
static int launch_small_k(const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                          int64_t ldc, const float* Cin, int64_t ldcin, const float* bias, int M,
                          int N, int K, float alpha, float beta, int relu, hipStream_t s) {
    const int eo = sizeof(TO);
    if (N % 4 == 0 && ldc % 4 == 0 && (uintptr_t)C % (4 * eo) == 0 &&
        (!Cin || (ldcin % 4 == 0 && (uintptr_t)Cin % 16 == 0)) && (!bias || (uintptr_t)bias % 16 == 0) &&
        env_flag("SRNN_SMALL_K2", 1)) {
        dim3 g2(cdiv(N, 256), cdiv(M, 32));
        if (K <= 16)
            hipLaunchKernelGGL((gemm_small_k2_kernel<T, TO, 16>), g2, dim3(256), 0, s,
                               (const T*)A, lda, (const T*)B, ldb, (TO*)C, ldc, Cin, ldcin, bias,
                               M, N, K, alpha, Cin ? beta : 0.f, relu);
        else
            hipLaunchKernelGGL((gemm_small_k2_kernel<T, TO, 64>), g2, dim3(256), 0, s,
                               (const T*)A, lda, (const T*)B, ldb, (TO*)C, ldc, Cin, ldcin, bias,
                               M, N, K, alpha, Cin ? beta : 0.f, relu);
        SRNN_LAUNCH_CHECK();
        return 0;
    }
    dim3 grid(cdiv(N, 256), cdiv(M, 16));
    if (K <= 16)
        hipLaunchKernelGGL((gemm_small_k_kernel<T, TO, 16>), grid, dim3(256), 0, s, (const T*)A,
                           lda, (const T*)B, ldb, (TO*)C, ldc, Cin, ldcin, bias, M, N, K, alpha,
                           beta, relu);
    else
        hipLaunchKernelGGL((gemm_small_k_kernel<T, TO, 64>), grid, dim3(256), 0, s, (const T*)A,
                           lda, (const T*)B, ldb, (TO*)C, ldc, Cin, ldcin, bias, M, N, K, alpha,
                           beta, relu);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// Returns -1 when the problem is not one of the two thin shapes.
int srnn_gemm_small_try(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                        float alpha, const void* A, int64_t lda, const void* B, int64_t ldb,
                        float beta, const float* Cin, int64_t ldcin, void* C, int64_t ldc,
                        const float* bias, int bias_mode, int relu, const void* mask,
                        hipStream_t s) {
    if (mask) return -1;
    // small N: plain fp32 output, B (K x N)
    if (N <= 64 && !transB && beta == 0.f && !bias && !relu && out_dtype == SRNN_F32 &&
        K >= 128 && (int64_t)M * K >= (1 << 16)) {
        // vector path: 4 adjacent m per lane (aligned rows of A)
        const int es = dtype == SRNN_F32 ? 4 : 2;
        if (transA && M % 4 == 0 && lda % 4 == 0 && ((uintptr_t)A % (4 * es)) == 0 &&
            env_flag("SRNN_SMALL_NT", 1))
            return dtype == SRNN_F32
                       ? launch_small_nt<float>(A, lda, B, ldb, (float*)C, ldc, M, N, K, alpha, s)
                       : launch_small_nt<bf16>(A, lda, B, ldb, (float*)C, ldc, M, N, K, alpha, s);
        if (dtype == SRNN_F32)
            return transA ? launch_small_n<float, true>(A, lda, B, ldb, (float*)C, ldc, M, N, K, alpha, s)
                          : launch_small_n<float, false>(A, lda, B, ldb, (float*)C, ldc, M, N, K, alpha, s);
        return transA ? launch_small_n<bf16, true>(A, lda, B, ldb, (float*)C, ldc, M, N, K, alpha, s)
                      : launch_small_n<bf16, false>(A, lda, B, ldb, (float*)C, ldc, M, N, K, alpha, s);
    }
    // small K: NT with the full epilogue (column bias only).  K = 64 without Cin over enough
    // rows for gemm3's own occupancy rule (>= 96 tiles of 256 x 256) goes to gemm3 instead
    // (the top tier's 64-sample input projection at 512 rows, 8192 x 1024 x 64 with bias, fp32
    // out: 42 -> 15 us, profiles/r06_gemm_route_b512.txt); SRNN_SMALLK_G3=0 keeps it here
    const bool to_g3 = K == 64 && beta == 0.f && M % 256 == 0 && N % 256 == 0 &&
                       (int64_t)(M / 256) * (N / 256) >= 96 && dtype == SRNN_BF16 &&
                       env_flag("SRNN_SMALLK_G3", 1);
    if (K <= 64 && K > 0 && !transA && transB && (!bias || bias_mode == 1) && M >= 256 && !to_g3) {
        if (dtype == SRNN_F32)
            return out_dtype == SRNN_F32
                       ? launch_small_k<float, float>(A, lda, B, ldb, C, ldc, Cin, ldcin, bias, M, N, K, alpha, beta, relu, s)
                       : launch_small_k<float, bf16>(A, lda, B, ldb, C, ldc, Cin, ldcin, bias, M, N, K, alpha, beta, relu, s);
        return out_dtype == SRNN_F32
                   ? launch_small_k<bf16, float>(A, lda, B, ldb, C, ldc, Cin, ldcin, bias, M, N, K, alpha, beta, relu, s)
                   : launch_small_k<bf16, bf16>(A, lda, B, ldb, C, ldc, Cin, ldcin, bias, M, N, K, alpha, beta, relu, s);
    }
    return -1;
}
