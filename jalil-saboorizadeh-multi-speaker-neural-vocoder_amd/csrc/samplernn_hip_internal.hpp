// Internal (C++) entry points shared between translation units of the library.
#pragma once
#include "common.hpp"

int srnn_gemm_impl(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                   float alpha, const void* A, int64_t lda, int64_t strideA, const void* B,
                   int64_t ldb, int64_t strideB, float beta, const float* Cin, int64_t ldcin,
                   int64_t strideCin, void* C, int64_t ldc, int64_t strideC, const float* bias,
                   int bias_mode, int relu, int batch, int tile, hipStream_t s,
                   const void* mask = nullptr, int64_t ldmask = 0,
                   const unsigned short* mbi = nullptr, int64_t ldmbi = 0,
                   unsigned short* mbo = nullptr, int64_t ldmbo = 0);
int srnn_relu_bits_impl(int dtype, const void* a, int64_t lda, int M, int N, unsigned short* bits,
                        int64_t ldb, hipStream_t s);

// u16 index of (row r, 16-column group g) in a ReLU bit mask (gemm.hip): row-major [r][g] with
// row stride ld, or ld == 0: column-group-major [g][M] (the grouped layout)
__host__ __device__ __forceinline__ int64_t srnn_bits_index(int64_t r, int g, int64_t M, int64_t ld) {
    return ld ? r * ld + g : (int64_t)g * M + r;
}

// y[M,N] = act(x[M,K] . W[N,K]^T + bias)   (nn.Linear / Conv1d(k=1) forward)
static inline int linear_fwd(int dt, int odt, int M, int N, int K, const void* x, int64_t ldx,
                             const void* W, int64_t ldw, const float* bias, void* y, int64_t ldy,
                             int relu, hipStream_t s, float beta = 0.f, const float* yin = nullptr,
                             int64_t ldyin = 0) {
    return srnn_gemm_impl(dt, odt, 0, 1, M, N, K, 1.f, x, ldx, 0, W, ldw, 0, beta, yin, ldyin, 0,
                          y, ldy, 0, bias, 1, relu, 1, -1, s);
}

// integer value of an environment switch (dflt when unset or empty)
static inline int env_flag(const char* name, int dflt) {
    const char* e = getenv(name);
    return (e && *e) ? atoi(e) : dflt;
}

// persist.hip: the per-device sticky failure flag of the persistent sweeps (device pointer,
// allocated zeroed on first use; null on a HIP error) and their spin limit (short when the
// SRNN_PERSIST_FORCE_FAIL test switch is set)
int* srnn_sticky_flag();
int srnn_persist_spin_limit(int dflt);
// persist.hip: co-residency of persistent grids (handoff.hpp) -- CUs of the current device,
// whether `blocks` one-per-CU workgroups fit it for every process sharing it, and the
// launch-time check with the kernel's occupancy (0 = fits, else reported error)
int srnn_device_cus();
extern "C" int srnn_device_share(void);
int srnn_persist_fits_cus(int64_t blocks);
int srnn_persist_check(const void* kernel, int threads, size_t lds, int64_t blocks,
                       const char* what);

// gemm3.hip: grow-only device scratch buffers, one per slot, never freed (a captured HIP graph
// keeps the pointer current at its capture); null on a HIP error.  Allocated on first use,
// i.e. by the eager warm-up step, outside graph captures.
enum { SRNN_SCRATCH_SPLITK = 0, SRNN_SCRATCH_MASK = 1, SRNN_SCRATCH_NT = 2, SRNN_SCRATCH_BLASLT = 3,
       SRNN_SCRATCH_SLOTS = 4 };
void* srnn_scratch(int slot, size_t bytes);

// Deterministic split-K support.  srnn_splitk_scratch = srnn_scratch(SRNN_SCRATCH_SPLITK);
// srnn_splitk_sum writes C[m][n] = sum_z part[z][m][n] in z order (float4 columns:
// N % 4 == 0, C 16-B aligned, ldc % 4 == 0).
float* srnn_splitk_scratch(size_t bytes);
int srnn_splitk_sum(const float* part, float* C, int64_t ldc, int M, int N, int ks, hipStream_t s);

// blaslt.cpp: plain large bf16 GEMMs (alpha, optional per-column bias, optional ReLU, beta 0)
// through hipBLASLt; 0 done, -1 not taken (run the library's own kernels), > 0 error
int srnn_blaslt_enabled();
// (batch > 1: strided batches, element strides sA / sB / sC; sA or sB may be 0 -- one
//  operand shared by every batch)
int srnn_blaslt_try(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                    float alpha, const void* A, int64_t lda, const void* B, int64_t ldb, float beta,
                    void* C, int64_t ldc, const float* bias, int bias_mode, int relu,
                    hipStream_t s, int batch = 1, int64_t sA = 0, int64_t sB = 0, int64_t sC = 0);
// gemm3.hip: a max |C| request (srnn_gemm_amax_next) waits for the next bf16 gemm3 launch
int srnn_gemm_amax_pending();
// gemm3.hip: a column-sum request (srnn_gemm_csum_next) waits for the next bf16 gemm3 launch
int srnn_gemm_csum_pending();
int srnn_gemm_lsm_pending();
