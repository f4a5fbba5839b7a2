// Thin GEMMs of the TBPTT step that the MFMA tile kernels handle badly: one output
// dimension or the reduction dimension is tiny, so a 32..256-wide tile is mostly padding
// and its K loop is one long dependent chain.
//
//  * small N (N <= 64, B stored K x N): the weight gradients of the input / conditioning /
//    speaker projections (dW = dX^T . input, N = frame samples, cond_dim, spk_dim) with K =
//    all frames of the batch, and the speaker-embedding gradient.  A thread owns one output
//    row m and all N columns in registers; the workgroup's K chunk of B is staged in LDS
//    and read as broadcasts; K is split over workgroups and the partial rows meet with
//    fp32 atomics (C zeroed first), so the grid fills the chip whatever M is.
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
                                                           float alpha, int atomic) {
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
    float* c = C + (int64_t)m * ldc + n0;
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n0 + n < N) {
            if (atomic) atomicAdd(c + n, alpha * acc[n]);
            else c[n] = alpha * acc[n];
        }
    }
}

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
    if (nks > 1) {
        if (ldc == N) {
            SRNN_CHECK_HIP(hipMemsetAsync(C, 0, (size_t)M * N * 4, s));
        } else {
            SRNN_CHECK_HIP(hipMemset2DAsync(C, ldc * 4, 0, (size_t)N * 4, M, s));
        }
    }
    dim3 grid(mblk, ngrp, nks);
    if (NM == 8)
        hipLaunchKernelGGL((gemm_small_n_kernel<T, TA, 8>), grid, dim3(256), 0, s, (const T*)A,
                           lda, (const T*)B, ldb, C, ldc, M, N, K, kchunk, alpha, nks > 1 ? 1 : 0);
    else
        hipLaunchKernelGGL((gemm_small_n_kernel<T, TA, 16>), grid, dim3(256), 0, s, (const T*)A,
                           lda, (const T*)B, ldb, C, ldc, M, N, K, kchunk, alpha, nks > 1 ? 1 : 0);
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

template <typename T, typename TO>
static int launch_small_k(const void* A, int64_t lda, const void* B, int64_t ldb, void* C,
                          int64_t ldc, const float* Cin, int64_t ldcin, const float* bias, int M,
                          int N, int K, float alpha, float beta, int relu, hipStream_t s) {
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
        if (dtype == SRNN_F32)
            return transA ? launch_small_n<float, true>(A, lda, B, ldb, (float*)C, ldc, M, N, K, alpha, s)
                          : launch_small_n<float, false>(A, lda, B, ldb, (float*)C, ldc, M, N, K, alpha, s);
        return transA ? launch_small_n<bf16, true>(A, lda, B, ldb, (float*)C, ldc, M, N, K, alpha, s)
                      : launch_small_n<bf16, false>(A, lda, B, ldb, (float*)C, ldc, M, N, K, alpha, s);
    }
    // small K: NT with the full epilogue (column bias only)
    if (K <= 64 && K > 0 && !transA && transB && (!bias || bias_mode == 1) && M >= 256) {
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
