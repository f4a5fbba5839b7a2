// Backward of the folded embedding . conv of SampleLevelMLP (model.py:274-285,311-320):
//     dTab[x_{b, t+k}][k][:] += da[b, t, :]     for all rows (b, t) and taps k < FS0
// i.e. 2.1 G scattered adds per TBPTT step at config B (131072 rows x 16 taps x 1024).
//
// Measured on MI355X (tools/lds_atomic_probe*.hip): LDS fp32 atomics (ds_add_f32) retire
// only 0.3 lane-ops/clk/CU, integer LDS atomics 14.6 (u32) / 9.9 (u64).  So the scatter
// accumulates in 64-bit FIXED POINT (value * 2^40, rounded) with ds_add_u64: fast, and
// exact/order-independent, which makes dTab bit-deterministic across runs and workgroup
// schedules.  Resolution 2^-40 ~ 9e-13 absolute per term (terms clamped to +-2^11),
// range of a sum +-2^23.
//
// A workgroup (1024 threads) owns CW columns and a block of whole batch rows: it stages
// the block's sample indices in LDS as bytes, gives each thread a fixed (tap k, column c)
// (one wave = one row), and flushes its Q x FS0 x CW accumulator with global 64-bit
// integer atomics into a zeroed int64 buffer; a final pass converts to fp32/bf16 in the
// q-major layout [q][k][:] the dE / dW GEMMs consume.
#include <algorithm>

#include "samplernn_hip_internal.hpp"

#define DTAB_NT 1024
#define DTAB_SCALE 1099511627776.0          // 2^40

// round(g * 2^40) as int64 in four instructions: the f64 fma against 1.5 * 2^52 leaves
// the rounded (to nearest even) integer in the low mantissa bits, and subtracting the
// magic's bit pattern recovers it.  Exact for |g| < 2^11 (terms are clamped there; the
// per-sample gradients reaching the table are many orders of magnitude smaller).
__device__ __forceinline__ long long fx40(float g) {
    g = __builtin_amdgcn_fmed3f(g, -2047.0f, 2047.0f);
    const double d = __builtin_fma((double)g, DTAB_SCALE, 6755399441055744.0);
    return __double_as_longlong(d) - 0x4338000000000000ll;
}

// FSC: compile-time FS0 (0 = runtime).  When FS0 * CW == 64 one wave owns one row per
// pass, so the row walk (b, t) is wave-uniform and lives in scalar registers.
template <typename T, int CW, int FSC>
__global__ __launch_bounds__(DTAB_NT) void dtab_fx_kernel(
    const T* __restrict__ da, int64_t ldda, const int64_t* __restrict__ x, int64_t ldx, int xoff,
    int Tlen, int B, int nb, unsigned long long* __restrict__ fx, int D, int FS0, int Q) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int FS = FSC ? FSC : FS0;
    unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem);  // [Q][FS][CW]
    unsigned char* idx = reinterpret_cast<unsigned char*>(smem + (size_t)Q * FS * CW * 8);
    const int tid = threadIdx.x;
    const int c0 = blockIdx.x * CW;
    const int b0 = blockIdx.y * nb;
    const int nbb = min(nb, B - b0);
    const int W = Tlen + FS - 1;
    const int nacc = Q * FS * CW;
    for (int i = tid; i < nacc; i += DTAB_NT) acc[i] = 0ull;
    for (int i = tid; i < nbb * W; i += DTAB_NT) {
        const int b = i / W, p = i - b * W;
        idx[i] = (unsigned char)x[(int64_t)(b0 + b) * ldx + xoff + p];
    }
    __syncthreads();
    const int per_row = FS * CW;
    const int rpp = DTAB_NT / per_row;
    if (tid < rpp * per_row) {
        const int rem = tid % per_row;
        const int k = rem / CW, c = rem % CW;
        const int nrows = nbb * Tlen;
        // columns past D read column D - 1 and add into accumulators that are never flushed
        const T* dab = da + (int64_t)b0 * Tlen * ldda + min(c0 + c, D - 1);
        unsigned long long* ak = acc + k * CW + c;
        const unsigned char* ik = idx + k;
        constexpr int U = 8;
        int r0 = tid / per_row;
        if constexpr (FSC * CW == 64) r0 = __builtin_amdgcn_readfirstlane(r0);
        int b = r0 / Tlen, t = r0 - b * Tlen;
        // full blocks of U rows: no bounds checks, so the U loads and index reads issue
        // back to back before the first conversion needs them
        for (; r0 + (U - 1) * rpp < nrows; r0 += U * rpp) {
            float g[U];
            int q[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                g[u] = to_f(dab[(int64_t)(r0 + u * rpp) * ldda]);
                q[u] = ik[b * W + t];
                t += rpp;
                while (t >= Tlen) { t -= Tlen; ++b; }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                atomicAdd(ak + q[u] * (FS * CW), (unsigned long long)fx40(g[u]));
        }
        for (; r0 < nrows; r0 += rpp) {
            atomicAdd(ak + ik[b * W + t] * (FS * CW),
                      (unsigned long long)fx40(to_f(dab[(int64_t)r0 * ldda])));
            t += rpp;
            while (t >= Tlen) { t -= Tlen; ++b; }
        }
    }
    __syncthreads();
    for (int i = tid; i < nacc; i += DTAB_NT) {
        const unsigned long long v = acc[i];
        const int c = i % CW, qk = i / CW;         // qk = q * FS + k
        if (v != 0ull && c0 + c < D) atomicAdd(&fx[(int64_t)qk * D + c0 + c], v);
    }
}

template <typename TO>
__global__ void dtab_fx_convert_kernel(const unsigned long long* __restrict__ fx,
                                       TO* __restrict__ out, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = from_f<TO>((float)((double)(long long)fx[i] * (1.0 / DTAB_SCALE)));
}

template <typename T, int CW, int FSC>
static int launch_dtab(const void* da, int64_t ldda, const int64_t* x, int64_t ldx, int xoff,
                       int B, int Tlen, unsigned long long* fx, int D, int FS0, int Q,
                       hipStream_t s) {
    const int acc_bytes = Q * FS0 * CW * 8;
    const int W = Tlen + FS0 - 1;
    const int nb_cap = std::max(1, (160 * 1024 - acc_bytes) / W);
    const int nslices = cdiv(D, CW);
    const int nblk = std::max(1, 1024 / nslices);
    int nb = std::min(B, std::max(cdiv(B, nblk), 1));
    nb = std::min(nb, nb_cap);
    const int lds = acc_bytes + ((nb * W + 15) / 16) * 16;
    static bool attr = false;
    if (!attr) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)dtab_fx_kernel<T, CW, FSC>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
    }
    dim3 grid(nslices, cdiv(B, nb));
    hipLaunchKernelGGL((dtab_fx_kernel<T, CW, FSC>), grid, dim3(DTAB_NT), lds, s, (const T*)da, ldda, x,
                       ldx, xoff, Tlen, B, nb, fx, D, FS0, Q);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// dtab_out (Q, FS0, D) in out_dtype; work: >= Q*FS0*D*8 bytes of device scratch
extern "C" int srnn_mlp_dtab(int dtype, const void* da, int64_t ldda, const int64_t* x,
                             int64_t ldx, int xoff, int B, int Tlen, void* dtab_out,
                             int out_dtype, int D, int FS0, int Q, void* work, size_t work_bytes,
                             void* stream) {
    SRNN_REQUIRE(Q <= 256, "dtab: q_levels must be <= 256 (byte indices)");
    const int64_t n = (int64_t)Q * FS0 * D;
    SRNN_REQUIRE(work && work_bytes >= (size_t)n * 8, "dtab: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    unsigned long long* fx = (unsigned long long*)work;
    SRNN_CHECK_HIP(hipMemsetAsync(fx, 0, (size_t)n * 8, s));
    if ((int64_t)B * Tlen > 0) {
        const int W = Tlen + FS0 - 1;
        int cw = 4;
        while (cw > 1 && (Q * FS0 * cw * 8 + W > 160 * 1024 || FS0 * cw > DTAB_NT)) cw /= 2;
        SRNN_REQUIRE(Q * FS0 * cw * 8 + W <= 160 * 1024 && FS0 * cw <= DTAB_NT,
                     "dtab: FS0 too large");
        int rc;
#define DTAB_GO(TT, CWV, FSV) launch_dtab<TT, CWV, FSV>(da, ldda, x, ldx, xoff, B, Tlen, fx, D, FS0, Q, s)
        if (dtype == SRNN_F32)
            rc = (cw == 4 && FS0 == 16) ? DTAB_GO(float, 4, 16)
               : cw == 4 ? DTAB_GO(float, 4, 0) : cw == 2 ? DTAB_GO(float, 2, 0) : DTAB_GO(float, 1, 0);
        else
            rc = (cw == 4 && FS0 == 16) ? DTAB_GO(bf16, 4, 16)
               : cw == 4 ? DTAB_GO(bf16, 4, 0) : cw == 2 ? DTAB_GO(bf16, 2, 0) : DTAB_GO(bf16, 1, 0);
#undef DTAB_GO
        if (rc) return rc;
    }
    if (out_dtype == SRNN_F32)
        hipLaunchKernelGGL(dtab_fx_convert_kernel<float>, dim3(cdiv(n, 256)), dim3(256), 0, s, fx,
                           (float*)dtab_out, n);
    else
        hipLaunchKernelGGL(dtab_fx_convert_kernel<bf16>, dim3(cdiv(n, 256)), dim3(256), 0, s, fx,
                           (bf16*)dtab_out, n);
    SRNN_LAUNCH_CHECK();
    return 0;
}
