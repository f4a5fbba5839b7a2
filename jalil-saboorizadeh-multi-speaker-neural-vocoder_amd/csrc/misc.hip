#include <type_traits>
// Memory-bound support kernels of the hot path: mu-law quantize/dequantize (utils.py),
// weight-norm forward/backward (torch weight_norm, model.py:119-131,177-178,303-306),
// layout permutes for the folded weights, row gathers (nn.Embedding), column sums
// (bias grads), and the fused clip + Adam update (optim.py:4-21, train.py:238).
#include <algorithm>

#include "samplernn_hip_internal.hpp"
#include "ulaw_tables.h"

__constant__ uint32_t c_ulaw_f32_steps[256];
__constant__ uint64_t c_ulaw_f64_thresh[256];
__constant__ uint32_t c_ulaw_lut[256];

static int g_tables_ready = 0;
static int ensure_tables() {
    if (g_tables_ready) return 0;
    SRNN_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_ulaw_f32_steps), SRNN_ULAW_F32_STEPS_BITS,
                                     sizeof(SRNN_ULAW_F32_STEPS_BITS)));
    SRNN_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_ulaw_f64_thresh), SRNN_ULAW_F64_THRESH_BITS,
                                     sizeof(SRNN_ULAW_F64_THRESH_BITS)));
    SRNN_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_ulaw_lut), SRNN_ULAW_LUT_BITS,
                                     sizeof(SRNN_ULAW_LUT_BITS)));
    g_tables_ready = 1;
    return 0;
}
int srnn_init_tables() { return ensure_tables(); }

// ------------------------------------------------------------------ mu-law quantize
// Bit-exact to utils.uquantize on [-1, 1] by counting reference-derived bin edges
// (branch-free 8-step binary search); outside [-1, 1] (not audio) the formula in
// double is used.
__device__ __forceinline__ int64_t uq_formula(double x, int q) {
    double s = (x > 0) - (x < 0);
    double y = s * log(255.0 * fabs(x) + 1.0) / 5.5451774444795623;
    y = 0.5 * (y + 1.0) * ((double)q - 1e-6);
    return (int64_t)y;
}

__global__ void uquantize_f32_kernel(const float* __restrict__ x, int64_t* __restrict__ out,
                                     int64_t n, int q) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = x[i];
    if (q == 256 && v >= -1.0f && v <= 1.0f) {
        int lo = 0;  // count of steps <= v
#pragma unroll
        for (int s = 128; s > 0; s >>= 1)
            if (__uint_as_float(c_ulaw_f32_steps[lo + s - 1]) <= v) lo += s;
        // the loop counts over steps[0..254]; steps[255] (value 256 at x = 1) last
        if (lo == 255 && __uint_as_float(c_ulaw_f32_steps[255]) <= v) lo = 256;
        out[i] = lo;
    } else {
        // float32 formula path (utils.py:33-36, 48-51) for out-of-domain values
        float sgn = (float)((v > 0) - (v < 0));
        float y = sgn * logf(255.0f * fabsf(v) + 1.0f) / 5.5451774444795623f;
        y = 0.5f * (y + 1.0f);
        y *= (float)((double)q - 1e-6);
        out[i] = (int64_t)y;
    }
}

__global__ void uquantize_f64_kernel(const double* __restrict__ x, int64_t* __restrict__ out,
                                     int64_t n, int q) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = x[i];
    if (q == 256 && v >= -1.0 && v <= 1.0) {
        int lo = 0;
#pragma unroll
        for (int s = 128; s > 0; s >>= 1)
            if (__longlong_as_double((long long)c_ulaw_f64_thresh[lo + s - 1]) <= v) lo += s;
        out[i] = lo;
    } else {
        out[i] = uq_formula(v, q);
    }
}

// mode 0: mu-law (utils.py:62-63, LUT for q = 256), mode 1: linear (utils.py:18-19)
__device__ __forceinline__ float udeq_one(int64_t kk, int q, float scale, int mode) {
    float v;
    if (mode == 1) {
        v = (float)kk / (float)(q / 2) - 1.0f;
    } else if (q == 256 && kk >= 0 && kk < 256) {
        v = __uint_as_float(c_ulaw_lut[kk]);
    } else {
        float c = (float)kk * 2.0f / (float)q - 1.0f;
        float e = expf(fabsf(c) * 5.5451774444795623f) - 1.0f;
        v = (float)((c > 0) - (c < 0)) * e / 255.0f;
    }
    return scale * v;
}

__global__ void udequantize_kernel(const int64_t* __restrict__ k, float* __restrict__ out,
                                   int64_t n, int q, float scale, int mode) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = udeq_one(k[i], q, scale, mode);
}

// strided rows (a window of the index stream) -> contiguous rows x cols
__global__ void udequantize2d_kernel(const int64_t* __restrict__ k, int64_t ldk,
                                     float* __restrict__ out, int cols, int64_t n, int q,
                                     float scale, int mode) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = i / cols, c = i - r * cols;
    out[i] = udeq_one(k[r * ldk + c], q, scale, mode);
}

extern "C" int srnn_uquantize_f32(const float* x, int64_t* out, int64_t n, int q, void* stream) {
    if (int e = ensure_tables()) return e;
    if (n <= 0) return 0;
    hipLaunchKernelGGL(uquantize_f32_kernel, dim3(cdiv(n, 256)), dim3(256), 0,
                       (hipStream_t)stream, x, out, n, q);
    SRNN_LAUNCH_CHECK();
    return 0;
}
extern "C" int srnn_uquantize_f64(const double* x, int64_t* out, int64_t n, int q, void* stream) {
    if (int e = ensure_tables()) return e;
    if (n <= 0) return 0;
    hipLaunchKernelGGL(uquantize_f64_kernel, dim3(cdiv(n, 256)), dim3(256), 0,
                       (hipStream_t)stream, x, out, n, q);
    SRNN_LAUNCH_CHECK();
    return 0;
}
extern "C" int srnn_udequantize(const int64_t* k, float* out, int64_t n, int q, float scale,
                                int mode, void* stream) {
    if (int e = ensure_tables()) return e;
    if (n <= 0) return 0;
    hipLaunchKernelGGL(udequantize_kernel, dim3(cdiv(n, 256)), dim3(256), 0,
                       (hipStream_t)stream, k, out, n, q, scale, mode);
    SRNN_LAUNCH_CHECK();
    return 0;
}

extern "C" int srnn_udequantize2d(const int64_t* k, int64_t ldk, float* out, int rows, int cols,
                                  int q, float scale, int mode, void* stream) {
    if (int e = ensure_tables()) return e;
    const int64_t n = (int64_t)rows * cols;
    if (n <= 0) return 0;
    hipLaunchKernelGGL(udequantize2d_kernel, dim3(cdiv(n, 256)), dim3(256), 0,
                       (hipStream_t)stream, k, ldk, out, cols, n, q, scale, mode);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// host (CPU) forms with the same tables: the DataLoader-side quantiser (dataset.py:253-254)
static int64_t uq_host_f64(double v, int q) {
    if (q == 256 && v >= -1.0 && v <= 1.0) {
        int lo = 0;
        for (int s = 128; s > 0; s >>= 1) {
            double t;
            memcpy(&t, &SRNN_ULAW_F64_THRESH_BITS[lo + s - 1], 8);
            if (t <= v) lo += s;
        }
        return lo;
    }
    double s = (v > 0) - (v < 0);
    double y = s * log(255.0 * fabs(v) + 1.0) / 5.5451774444795623;
    y = 0.5 * (y + 1.0) * ((double)q - 1e-6);
    return (int64_t)y;
}
static int64_t uq_host_f32(float v, int q) {
    if (q == 256 && v >= -1.0f && v <= 1.0f) {
        int lo = 0;
        for (int s = 128; s > 0; s >>= 1) {
            float t;
            memcpy(&t, &SRNN_ULAW_F32_STEPS_BITS[lo + s - 1], 4);
            if (t <= v) lo += s;
        }
        float t255;
        memcpy(&t255, &SRNN_ULAW_F32_STEPS_BITS[255], 4);
        if (lo == 255 && t255 <= v) lo = 256;
        return lo;
    }
    float sg = (float)((v > 0) - (v < 0));
    float y = sg * logf(255.0f * fabsf(v) + 1.0f) / 5.5451774444795623f;
    y = 0.5f * (y + 1.0f);
    y *= (float)((double)q - 1e-6);
    return (int64_t)y;
}
extern "C" int srnn_uquantize_f64_host(const double* x, int64_t* out, int64_t n, int q) {
    for (int64_t i = 0; i < n; ++i) out[i] = uq_host_f64(x[i], q);
    return 0;
}
extern "C" int srnn_uquantize_f32_host(const float* x, int64_t* out, int64_t n, int q) {
    for (int64_t i = 0; i < n; ++i) out[i] = uq_host_f32(x[i], q);
    return 0;
}
extern "C" int srnn_udequantize_host(const int64_t* k, float* out, int64_t n, int q) {
    for (int64_t i = 0; i < n; ++i) {
        const int64_t kk = k[i];
        if (q == 256 && kk >= 0 && kk < 256) {
            memcpy(&out[i], &SRNN_ULAW_LUT_BITS[kk], 4);
        } else {
            float c = (float)kk * 2.0f / (float)q - 1.0f;
            float e = expf(fabsf(c) * 5.5451774444795623f) - 1.0f;
            out[i] = (float)((c > 0) - (c < 0)) * e / 255.0f;
        }
    }
    return 0;
}

// ------------------------------------------------------------------ weight norm
// w[o, r] = g[o] * v[o, r] / ||v[o, :]||   (norm over all dims but 0; one block per o)
__device__ __forceinline__ float block_sum(float v, float* sh) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) sh[w] = v;
    __syncthreads();
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
    return t;
}

// Every weight-norm kernel walks a row of R floats in the same per-thread order -- float4
// chunks c = tid, tid + 256, ... (elements 4c .. 4c + 3) when the row is 16-B aligned and
// R % 4 == 0, else single elements r = tid, tid + 256, ... -- four chunks loaded ahead, and
// reduces with block_sum: the fused conv_t kernels below reproduce wn_fwd / wn_bwd bit for bit.
__device__ __forceinline__ bool wn_vec(const float* row, int64_t R) {
    return R % 4 == 0 && (uintptr_t)row % 16 == 0;
}

// f(r, v[r]) for r of this thread, in the common order
template <typename F>
__device__ __forceinline__ void wn_walk(const float* __restrict__ row, int64_t R, bool vec, F f) {
    const int tid = threadIdx.x;
    if (vec) {
        const int64_t R4 = R / 4;
        const floatx4* r4 = reinterpret_cast<const floatx4*>(row);
        int64_t c = tid;
        for (; c + 768 < R4; c += 1024) {
            floatx4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) x[u] = r4[c + 256 * u];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int e = 0; e < 4; ++e) f(4 * (c + 256 * u) + e, x[u][e]);
        }
        for (; c < R4; c += 256) {
            const floatx4 x = r4[c];
#pragma unroll
            for (int e = 0; e < 4; ++e) f(4 * c + e, x[e]);
        }
    } else {
        for (int64_t r = tid; r < R; r += 256) f(r, row[r]);
    }
}

__global__ __launch_bounds__(256) void wn_fwd_kernel(const float* __restrict__ g,
                                                     const float* __restrict__ v,
                                                     float* __restrict__ w,
                                                     float* __restrict__ norm, int64_t R) {
    __shared__ float sh[16];
    const int64_t o = blockIdx.x;
    const float* vr = v + o * R;
    const bool vec = wn_vec(vr, R) && (uintptr_t)w % 16 == 0;
    float s = 0.f;
    wn_walk(vr, R, vec, [&](int64_t, float x) { s += x * x; });
    s = block_sum(s, sh);
    const float nrm = sqrtf(s);
    const float scale = g[o] / nrm;
    if (norm && threadIdx.x == 0) norm[o] = nrm;
    wn_walk(vr, R, vec, [&](int64_t r, float x) { w[o * R + r] = x * scale; });
}

// dg[o] = sum_r dw v / n ;  dv = (g/n) (dw - (dg/n) v)
__global__ __launch_bounds__(256) void wn_bwd_kernel(const float* __restrict__ g,
                                                     const float* __restrict__ v,
                                                     const float* __restrict__ dw,
                                                     float* __restrict__ dg,
                                                     float* __restrict__ dv, int64_t R,
                                                     int accumulate) {
    __shared__ float sh[16];
    const int64_t o = blockIdx.x;
    const float* vr = v + o * R;
    const float* dr = dw + o * R;
    const bool vec = wn_vec(vr, R);
    float s = 0.f, d = 0.f;
    wn_walk(vr, R, vec, [&](int64_t r, float x) {
        s += x * x;
        d += dr[r] * x;
    });
    s = block_sum(s, sh);
    d = block_sum(d, sh);
    const float n = sqrtf(s);
    const float dgo = d / n;
    const float gn = g[o] / n;
    if (threadIdx.x == 0) dg[o] = accumulate ? dg[o] + dgo : dgo;
    wn_walk(vr, R, vec, [&](int64_t r, float x) {
        const float val = gn * (dr[r] - dgo / n * x);
        dv[o * R + r] = accumulate ? dv[o * R + r] + val : val;
    });
}

extern "C" int srnn_weight_norm_fwd(const float* g, const float* v, float* w, float* norm, int O,
                                    int64_t R, void* stream) {
    if (O <= 0) return 0;
    hipLaunchKernelGGL(wn_fwd_kernel, dim3(O), dim3(256), 0, (hipStream_t)stream, g, v, w, norm, R);
    SRNN_LAUNCH_CHECK();
    return 0;
}
extern "C" int srnn_weight_norm_bwd(const float* g, const float* v, const float* dw, float* dg,
                                    float* dv, int O, int64_t R, int accumulate, void* stream) {
    if (O <= 0) return 0;
    hipLaunchKernelGGL(wn_bwd_kernel, dim3(O), dim3(256), 0, (hipStream_t)stream, g, v, dw, dg, dv,
                       R, accumulate);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------ weight norm of conv_t
// The always-on weight norm of LearnedUpsampling1d.conv_t (model.py:177-178, nn.py:33-43)
// feeds ONE consumer: the upsampling GEMM operand W_up[(j * Cout + o)][i] = w[i][o][j].
// Forward: s[i] = g[i] / ||v[i]|| (srnn_weight_norm_scale, reads v once, writes Cin floats),
// then srnn_convt_fold writes the scaled, permuted operand straight from v (no fp32 w).
// Backward: the GEMM produces dW^T[i][(j * Cout + o)] (rows per input channel), and one
// block per channel computes dg and dv in v's own layout (srnn_convt_wn_bwd): the same
// per-thread element order and block reduction as wn_bwd_kernel, so the results are the
// ones weight_norm_bwd would give for the permuted gradient.
__global__ __launch_bounds__(256) void wn_scale_kernel(const float* __restrict__ g,
                                                       const float* __restrict__ v,
                                                       float* __restrict__ scale, int64_t R) {
    __shared__ float sh[16];
    const int64_t o = blockIdx.x;
    const float* vr = v + o * R;
    float s = 0.f;
    wn_walk(vr, R, wn_vec(vr, R), [&](int64_t, float x) { s += x * x; });
    s = block_sum(s, sh);
    if (threadIdx.x == 0) scale[o] = g[o] / sqrtf(s);
}

extern "C" int srnn_weight_norm_scale(const float* g, const float* v, float* scale, int O,
                                      int64_t R, void* stream) {
    if (O <= 0) return 0;
    hipLaunchKernelGGL(wn_scale_kernel, dim3(O), dim3(256), 0, (hipStream_t)stream, g, v, scale, R);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// dst[(j * Cout + o) * Cin + i] = v[i][o][j] * scale[i]: 64 channels x 64 (o, j) per block
// (64 / k output channels), 256-B row reads, 128-B (bf16) / 256-B (fp32) row writes
template <typename TO>
__global__ __launch_bounds__(256) void convt_fold_kernel(const float* __restrict__ v,
                                                         const float* __restrict__ scale,
                                                         TO* __restrict__ dst, int Cin, int Cout,
                                                         int k) {
    __shared__ float tile[64][65];
    const int tid = threadIdx.x;
    const int i0 = blockIdx.x * 64;
    const int e0 = blockIdx.y * 64;                // flat (o, j) = o * k + j
    const int64_t R = (int64_t)Cout * k;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int row = p * 16 + (tid >> 4), c4 = (tid & 15) * 4;
        const floatx4 x = *reinterpret_cast<const floatx4*>(v + (int64_t)(i0 + row) * R + e0 + c4);
        const float sc = scale ? scale[i0 + row] : 1.f;
        tile[row][c4 + 0] = x[0] * sc;
        tile[row][c4 + 1] = x[1] * sc;
        tile[row][c4 + 2] = x[2] * sc;
        tile[row][c4 + 3] = x[3] * sc;
    }
    __syncthreads();
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int e = p * 16 + (tid >> 4), i4 = (tid & 15) * 4;
        const int ef = e0 + e, o = ef / k, j = ef - o * k;
        TO* q = dst + ((int64_t)j * Cout + o) * Cin + i0 + i4;
        float w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) w[u] = tile[i4 + u][e];
        if constexpr (sizeof(TO) == 4) {
            *reinterpret_cast<floatx4*>(q) = floatx4{w[0], w[1], w[2], w[3]};
        } else {
            unsigned short h[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) h[u] = __bfloat16_as_ushort(__float2bfloat16(w[u]));
            *reinterpret_cast<uint2*>(q) = make_uint2(h[0] | ((unsigned)h[1] << 16),
                                                      h[2] | ((unsigned)h[3] << 16));
        }
    }
}

extern "C" int srnn_convt_fold(const float* v, const float* scale, void* dst, int dst_dtype,
                               int Cin, int Cout, int k, void* stream) {
    if ((int64_t)Cin * Cout * k <= 0) return 0;
    SRNN_REQUIRE(Cin % 64 == 0 && ((int64_t)Cout * k) % 64 == 0 && 64 % k == 0,
                 "convt_fold: needs Cin %% 64 == 0, 64 %% k == 0 (Cin %d Cout %d k %d)", Cin, Cout, k);
    SRNN_REQUIRE((uintptr_t)v % 16 == 0, "convt_fold: v must be 16-B aligned");
    dim3 grid(Cin / 64, (unsigned)(((int64_t)Cout * k) / 64));
    hipStream_t s = (hipStream_t)stream;
    if (dst_dtype == SRNN_F32)
        hipLaunchKernelGGL(convt_fold_kernel<float>, grid, dim3(256), 0, s, v, scale, (float*)dst,
                           Cin, Cout, k);
    else
        hipLaunchKernelGGL(convt_fold_kernel<bf16>, grid, dim3(256), 0, s, v, scale, (bf16*)dst,
                           Cin, Cout, k);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// one block per input channel i: dW^T row [j][o] staged in LDS (row pitch Cout + 4 floats:
// the reads at flat (o, j) order hit distinct banks for k = 16), then wn_bwd_kernel's math
template <bool HAS_G>
__global__ __launch_bounds__(256) void convt_wn_bwd_kernel(const float* __restrict__ g,
                                                           const float* __restrict__ v,
                                                           const float* __restrict__ dwt,
                                                           float* __restrict__ dg,
                                                           float* __restrict__ dv, int Cout,
                                                           int k) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* dl = reinterpret_cast<float*>(smem);           // [k][Cout + 4]
    __shared__ float sh[16];
    const int64_t i = blockIdx.x;
    const int64_t R = (int64_t)Cout * k;
    const int pitch = Cout + 4;
    const float* drow = dwt + i * R;
    for (int64_t e = threadIdx.x * 4; e < R; e += 256 * 4) {
        const floatx4 x = *reinterpret_cast<const floatx4*>(drow + e);
        const int j = (int)(e / Cout), o = (int)(e - (int64_t)j * Cout);
        *reinterpret_cast<floatx4*>(dl + j * pitch + o) = x;
    }
    __syncthreads();
    const float* vr = v + i * R;
    const bool vec = wn_vec(vr, R);
    auto dw_at = [&](int64_t r) {
        const int o = (int)(r / k), j = (int)(r - (int64_t)o * k);
        return dl[j * pitch + o];
    };
    float s = 0.f, d = 0.f;
    wn_walk(vr, R, vec, [&](int64_t r, float x) {
        s += x * x;
        d += dw_at(r) * x;
    });
    s = block_sum(s, sh);
    d = block_sum(d, sh);
    const float n = sqrtf(s);
    const float dgo = d / n;
    const float gn = (HAS_G ? g[i] : 1.f) / n;
    if (threadIdx.x == 0) dg[i] = dgo;
    wn_walk(vr, R, vec, [&](int64_t r, float x) { dv[i * R + r] = gn * (dw_at(r) - dgo / n * x); });
}

extern "C" int srnn_convt_wn_bwd(const float* g, const float* v, const float* dwt, float* dg,
                                 float* dv, int Cin, int Cout, int k, void* stream) {
    if ((int64_t)Cin * Cout * k <= 0) return 0;
    SRNN_REQUIRE(Cout % 4 == 0 && (uintptr_t)dwt % 16 == 0, "convt_wn_bwd: Cout %% 4, 16-B dW^T");
    const size_t lds = (size_t)k * (Cout + 4) * sizeof(float);
    SRNN_REQUIRE(lds <= 150 * 1024, "convt_wn_bwd: k * Cout too large for LDS (%d x %d)", k, Cout);
    static bool attr = false;
    if (!attr) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)convt_wn_bwd_kernel<true>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
        attr = true;
    }
    hipLaunchKernelGGL(convt_wn_bwd_kernel<true>, dim3(Cin), dim3(256), lds, (hipStream_t)stream, g,
                       v, dwt, dg, dv, Cout, k);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------ layout permutes
// dst = src.permute(p0, p1, p2) made contiguous, src (d0, d1, d2) row-major fp32; dst
// fp32 (optionally accumulated) or bf16.  When the innermost axis changes (o = p2 != 2)
// the copy is a batch of 2-D transposes between src axis o and src axis 2, done through
// 32 x 32 LDS tiles so that both the reads and the writes are coalesced.
struct Perm3 {
    int64_t S[3];    // src stride of src axis a
    int64_t Dd[3];   // dst stride of src axis a
    int d[3];
    int o, b;        // src axis innermost in dst; remaining (batch) axis
};

template <typename TO, bool ACC>
__global__ __launch_bounds__(256) void permute3_tiled_kernel(const float* __restrict__ src,
                                                             TO* __restrict__ dst, Perm3 P) {
    __shared__ float tile[32][33];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    const int nt2 = (P.d[2] + 31) / 32;
    const int t2 = blockIdx.x % nt2;
    const int64_t bi = blockIdx.x / nt2;
    const int i0 = t2 * 32, o0 = blockIdx.y * 32;
    const float* sb = src + bi * P.S[P.b];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int oi = o0 + ty + 8 * k, ii = i0 + tx;
        if (oi < P.d[P.o] && ii < P.d[2]) tile[ty + 8 * k][tx] = sb[(int64_t)oi * P.S[P.o] + ii];
    }
    __syncthreads();
    TO* db = dst + bi * P.Dd[P.b];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int ii = i0 + ty + 8 * k, oi = o0 + tx;
        if (oi < P.d[P.o] && ii < P.d[2]) {
            TO* q = db + (int64_t)ii * P.Dd[2] + oi;
            const float v = tile[tx][ty + 8 * k];
            if (ACC) *q = from_f<TO>(to_f(*q) + v);
            else *q = from_f<TO>(v);
        }
    }
}

// innermost axis kept: walk src order (coalesced reads), dst rows of d2 stay contiguous
template <typename TO, bool ACC>
__global__ void permute3_copy_kernel(const float* __restrict__ src, TO* __restrict__ dst, Perm3 P) {
    const int64_t n = (int64_t)P.d[0] * P.d[1] * P.d[2];
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n) return;
    const int i2 = idx % P.d[2];
    const int64_t q = idx / P.d[2];
    const int i1 = q % P.d[1];
    const int i0 = q / P.d[1];
    TO* o = dst + i0 * P.Dd[0] + i1 * P.Dd[1] + i2;
    if (ACC) *o = from_f<TO>(to_f(*o) + src[idx]);
    else *o = from_f<TO>(src[idx]);
}

template <typename TO, bool ACC>
static int permute3_launch(const float* src, TO* dst, const Perm3& P, hipStream_t s) {
    if (P.o == 2) {
        const int64_t n = (int64_t)P.d[0] * P.d[1] * P.d[2];
        hipLaunchKernelGGL((permute3_copy_kernel<TO, ACC>), dim3(cdiv(n, 256)), dim3(256), 0, s,
                           src, dst, P);
    } else {
        const int64_t gx = (int64_t)cdiv(P.d[2], 32) * P.d[P.b];
        SRNN_REQUIRE(gx < (1ll << 31), "permute3: too large");
        hipLaunchKernelGGL((permute3_tiled_kernel<TO, ACC>), dim3((unsigned)gx, cdiv(P.d[P.o], 32)),
                           dim3(256), 0, s, src, dst, P);
    }
    SRNN_LAUNCH_CHECK();
    return 0;
}

extern "C" int srnn_permute3(const float* src, void* dst, int dst_dtype, int d0, int d1, int d2,
                             int p0, int p1, int p2, int accumulate, void* stream) {
    const int64_t n = (int64_t)d0 * d1 * d2;
    if (n <= 0) return 0;
    SRNN_REQUIRE(p0 + p1 + p2 == 3 && p0 != p1 && p1 != p2 && p0 != p2 && p0 >= 0 && p1 >= 0 &&
                 p2 >= 0, "permute3: bad perm");
    Perm3 P;
    P.d[0] = d0; P.d[1] = d1; P.d[2] = d2;
    P.S[0] = (int64_t)d1 * d2; P.S[1] = d2; P.S[2] = 1;
    const int pr[3] = {p0, p1, p2};
    const int64_t ds[3] = {(int64_t)P.d[p1] * P.d[p2], P.d[p2], 1};
    for (int j = 0; j < 3; ++j) P.Dd[pr[j]] = ds[j];
    P.o = p2;
    P.b = p2 == 2 ? 0 : 1 - p2;       // the axis that is neither 2 nor o
    hipStream_t s = (hipStream_t)stream;
    if (dst_dtype == SRNN_F32) {
        if (accumulate) return permute3_launch<float, true>(src, (float*)dst, P, s);
        return permute3_launch<float, false>(src, (float*)dst, P, s);
    }
    SRNN_REQUIRE(!accumulate, "permute3: accumulate needs fp32 dst");
    return permute3_launch<bf16, false>(src, (bf16*)dst, P, s);
}

// 2-D strided copy with dtype conversion (fp32 -> fp32/bf16, bf16 -> fp32)
template <typename TI, typename TO>
__global__ void copy2d_kernel(const TI* __restrict__ src, int64_t lds, TO* __restrict__ dst,
                              int64_t ldd, int rows, int cols) {
    int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)rows * cols) return;
    int r = idx / cols, c = idx % cols;
    dst[(int64_t)r * ldd + c] = from_f<TO>(to_f(src[(int64_t)r * lds + c]));
}

extern "C" int srnn_copy2d(int src_dtype, int dst_dtype, int rows, int cols, const void* src,
                           int64_t lds, void* dst, int64_t ldd, void* stream) {
    const int64_t n = (int64_t)rows * cols;
    if (n <= 0) return 0;
    dim3 grid(cdiv(n, 256));
    hipStream_t s = (hipStream_t)stream;
    if (src_dtype == SRNN_F32 && dst_dtype == SRNN_F32)
        hipLaunchKernelGGL((copy2d_kernel<float, float>), grid, dim3(256), 0, s, (const float*)src,
                           lds, (float*)dst, ldd, rows, cols);
    else if (src_dtype == SRNN_F32 && dst_dtype == SRNN_BF16)
        hipLaunchKernelGGL((copy2d_kernel<float, bf16>), grid, dim3(256), 0, s, (const float*)src,
                           lds, (bf16*)dst, ldd, rows, cols);
    else if (src_dtype == SRNN_BF16 && dst_dtype == SRNN_F32)
        hipLaunchKernelGGL((copy2d_kernel<bf16, float>), grid, dim3(256), 0, s, (const bf16*)src,
                           lds, (float*)dst, ldd, rows, cols);
    else
        hipLaunchKernelGGL((copy2d_kernel<bf16, bf16>), grid, dim3(256), 0, s, (const bf16*)src,
                           lds, (bf16*)dst, ldd, rows, cols);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------ gathers / adds
// out[r, :] = table[idx[r], :]   (nn.Embedding forward, model.py:103-106, 274-277)
template <typename T>
__global__ void gather_rows_kernel(const float* __restrict__ table, int64_t ldt,
                                   const int64_t* __restrict__ idx, int64_t n, int cols,
                                   T* __restrict__ out, int64_t ldo) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * cols) return;
    int64_t r = e / cols;
    int c = e % cols;
    out[r * ldo + c] = from_f<T>(table[idx[r] * ldt + c]);
}

extern "C" int srnn_gather_rows(const float* table, int64_t ldt, const int64_t* idx, int64_t n,
                                int cols, void* out, int out_dtype, int64_t ldo, void* stream) {
    if (n * cols <= 0) return 0;
    dim3 grid(cdiv(n * cols, 256));
    if (out_dtype == SRNN_F32)
        hipLaunchKernelGGL((gather_rows_kernel<float>), grid, dim3(256), 0, (hipStream_t)stream,
                           table, ldt, idx, n, cols, (float*)out, ldo);
    else
        hipLaunchKernelGGL((gather_rows_kernel<bf16>), grid, dim3(256), 0, (hipStream_t)stream,
                           table, ldt, idx, n, cols, (bf16*)out, ldo);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// table[idx[r], :] += src[r, :]  (embedding backward; fp32 atomics, few rows)
__global__ void scatter_add_rows_kernel(float* __restrict__ table, int64_t ldt,
                                        const int64_t* __restrict__ idx, int64_t n, int cols,
                                        const float* __restrict__ src, int64_t lds) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * cols) return;
    int64_t r = e / cols;
    int c = e % cols;
    atomicAdd(&table[idx[r] * ldt + c], src[r * lds + c]);
}

extern "C" int srnn_scatter_add_rows(float* table, int64_t ldt, const int64_t* idx, int64_t n,
                                     int cols, const float* src, int64_t lds, void* stream) {
    if (n * cols <= 0) return 0;
    hipLaunchKernelGGL(scatter_add_rows_kernel, dim3(cdiv(n * cols, 256)), dim3(256), 0,
                       (hipStream_t)stream, table, ldt, idx, n, cols, src, lds);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// table[q, :] += sum over r with idx[r] == q of src[r, :], in r order: the embedding backward
// (speaker rows, model.py:203-207) without atomics, so the gradient is the same bits on every
// run.  One workgroup per table entry: its threads stage the entry's column of src in LDS
// (rows of another entry as -0.0, the exact no-op of an fp32 add, so the left fold is the
// sequential one bit for bit), then one lane adds them in row order from LDS -- one thread
// per entry walking global memory row by row took ~90 us for 512 rows.
constexpr int IAR_NT = 256, IAR_CHUNK = 2048;
__global__ __launch_bounds__(IAR_NT) void index_add_rows_kernel(
    float* __restrict__ table, int64_t ldt, int trows, const int64_t* __restrict__ idx, int64_t n,
    int cols, const float* __restrict__ src, int64_t lds) {
    __shared__ float sv[IAR_CHUNK];
    const int e = blockIdx.x;
    const int q = e / cols, c = e % cols;
    float acc = 0.f;
    if (threadIdx.x == 0) acc = table[(int64_t)q * ldt + c];
    for (int64_t r0 = 0; r0 < n; r0 += IAR_CHUNK) {
        const int cnt = (int)min((int64_t)IAR_CHUNK, n - r0);
        for (int i = threadIdx.x; i < cnt; i += IAR_NT)
            sv[i] = idx[r0 + i] == q ? src[(r0 + i) * lds + c] : -0.f;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int i = 0; i < cnt; ++i) acc += sv[i];
        __syncthreads();
    }
    if (threadIdx.x == 0) table[(int64_t)q * ldt + c] = acc;
}

extern "C" int srnn_index_add_rows(float* table, int64_t ldt, int trows, const int64_t* idx,
                                   int64_t n, int cols, const float* src, int64_t lds,
                                   void* stream) {
    if ((int64_t)trows * cols <= 0 || n <= 0) return 0;
    SRNN_REQUIRE((int64_t)trows * cols < (1ll << 31), "index_add_rows: table too large");
    hipLaunchKernelGGL(index_add_rows_kernel, dim3((unsigned)((int64_t)trows * cols)), dim3(IAR_NT),
                       0, (hipStream_t)stream, table, ldt, trows, idx, n, cols, src, lds);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// out = alpha * a + beta * b  (fp32, elementwise; out may alias a or b)
__global__ void axpby_kernel(float* out, const float* a, const float* b, float alpha, float beta,
                             int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = alpha * a[i] + (b ? beta * b[i] : 0.f);
}

extern "C" int srnn_axpby(float* out, const float* a, const float* b, float alpha, float beta,
                          int64_t n, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(axpby_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, out, a,
                       b, alpha, beta, n);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// x[b, f, :] += v[b, :]  for x (B, F, D) with row stride ldx per (b, f)
__global__ void add_bcast_rows_kernel(float* __restrict__ x, const float* __restrict__ v, int B,
                                      int F, int D, int64_t ldv) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)B * F * D) return;
    int d = e % D;
    int64_t bf = e / D;
    int b = bf / F;
    x[e] += v[(int64_t)b * ldv + d];
}

extern "C" int srnn_add_bcast_rows(float* x, const float* v, int B, int F, int D, int64_t ldv,
                                   void* stream) {
    if ((int64_t)B * F * D <= 0) return 0;
    hipLaunchKernelGGL(add_bcast_rows_kernel, dim3(cdiv((int64_t)B * F * D, 256)), dim3(256), 0,
                       (hipStream_t)stream, x, v, B, F, D, ldv);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------ column sums
// partial[rb, c] = sum_{r in row block rb} src[r, c]  then out[c] (+)= alpha * sum_rb partial.
// A 256-thread block owns 64 columns (16 lanes x 4 adjacent columns, vector loads when
// aligned) and 16 row lanes that stride its row block; the 16 row sums meet in LDS.  The
// final pass is the same kernel over the partial matrix.  Fixed summation order: the
// result is deterministic.
typedef unsigned short cs_u16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void cs_ld4(const float* p, float (&v)[4]) {
    const floatx4 x = *reinterpret_cast<const floatx4*>(p);
    v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
}
__device__ __forceinline__ void cs_ld4(const bf16* p, float (&v)[4]) {
    const cs_u16x4 x = *reinterpret_cast<const cs_u16x4*>(p);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = __uint_as_float((unsigned)x[e] << 16);
}

template <typename T, bool VEC, bool FINAL>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ src, int64_t lds,
                                                     int64_t rows, int cols, int64_t rpb,
                                                     float* __restrict__ dst, float alpha,
                                                     int accumulate) {
    __shared__ float red[16][65];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int c = blockIdx.x * 64 + tx * 4;
    const int64_t r0 = (int64_t)blockIdx.y * rpb;
    const int64_t r1 = min(rows, r0 + rpb);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (VEC && c + 3 < cols) {
        // four rows' loads in flight before their adds (one 8-16 B load per thread and
        // round trip left the pass latency-bound at ~4.9 TB/s); same summation order
        int64_t r = r0 + ty;
        for (; r + 48 < r1; r += 64) {
            float v[4][4];
#pragma unroll
            for (int u = 0; u < 4; ++u) cs_ld4(src + (r + 16 * u) * lds + c, v[u]);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                s0 += v[u][0]; s1 += v[u][1]; s2 += v[u][2]; s3 += v[u][3];
            }
        }
        for (; r < r1; r += 16) {
            float v[4];
            cs_ld4(src + r * lds + c, v);
            s0 += v[0]; s1 += v[1]; s2 += v[2]; s3 += v[3];
        }
    } else {
        for (int64_t r = r0 + ty; r < r1; r += 16) {
            const T* p = src + r * lds;
            if (c < cols) s0 += to_f(p[c]);
            if (c + 1 < cols) s1 += to_f(p[c + 1]);
            if (c + 2 < cols) s2 += to_f(p[c + 2]);
            if (c + 3 < cols) s3 += to_f(p[c + 3]);
        }
    }
    red[ty][tx * 4 + 0] = s0; red[ty][tx * 4 + 1] = s1;
    red[ty][tx * 4 + 2] = s2; red[ty][tx * 4 + 3] = s3;
    __syncthreads();
    if (threadIdx.x < 64) {
        const int cc = blockIdx.x * 64 + threadIdx.x;
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) t += red[i][threadIdx.x];
        if (cc < cols) {
            if (FINAL) dst[cc] = accumulate ? dst[cc] + alpha * t : alpha * t;
            else dst[(int64_t)blockIdx.y * cols + cc] = t;
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void colsum_narrow_kernel(const T* __restrict__ src, int64_t lds,
                                                            int64_t rows, float* __restrict__ dst,
                                                            float alpha, int accumulate) {
    __shared__ float sh[16];
    const int c = blockIdx.x;
    float s = 0.f;
    for (int64_t r = threadIdx.x; r < rows; r += 256) s += to_f(src[r * lds + c]);
    s = block_sum(s, sh);
    if (threadIdx.x == 0) dst[c] = accumulate ? dst[c] + alpha * s : alpha * s;
}

template <typename T>
static void colsum_pass(const T* src, int64_t lds, int64_t rows, int cols, int64_t rpb, int nrb,
                        float* dst, float alpha, int accumulate, bool final_, hipStream_t s) {
    const bool vec = (lds % 4 == 0) && ((uintptr_t)src % (4 * sizeof(T)) == 0);
    dim3 grid(cdiv(cols, 64), nrb);
    if (final_ && cols < 16 && nrb == 1) {
        // few columns (the loss sum): every thread of a block strides the rows of one column
        hipLaunchKernelGGL((colsum_narrow_kernel<T>), dim3(cols), dim3(256), 0, s, src, lds, rows,
                           dst, alpha, accumulate);
        return;
    }
    if (final_) {
        if (vec) hipLaunchKernelGGL((colsum_kernel<T, true, true>), grid, dim3(256), 0, s, src, lds, rows, cols, rpb, dst, alpha, accumulate);
        else hipLaunchKernelGGL((colsum_kernel<T, false, true>), grid, dim3(256), 0, s, src, lds, rows, cols, rpb, dst, alpha, accumulate);
    } else {
        if (vec) hipLaunchKernelGGL((colsum_kernel<T, true, false>), grid, dim3(256), 0, s, src, lds, rows, cols, rpb, dst, alpha, accumulate);
        else hipLaunchKernelGGL((colsum_kernel<T, false, false>), grid, dim3(256), 0, s, src, lds, rows, cols, rpb, dst, alpha, accumulate);
    }
}

int srnn_colsum_impl(int dtype, const void* src, int64_t lds, int64_t rows, int cols, float* out,
                     float alpha, int accumulate, float* work, int64_t work_elems, hipStream_t s) {
    if (cols <= 0) return 0;
    const int cblk = cdiv(cols, 64);
    // ~2048 blocks in the first pass, at least 64 rows per block, partials within `work`
    int64_t nrb = std::max<int64_t>(1, std::min<int64_t>(2048 / cblk, rows / 64));
    nrb = std::min<int64_t>(nrb, work_elems / cols);
    // few rows (per-row bias sums of the GRU sweeps, speaker rows: B = 128): one pass -- a
    // second launch costs more than the rows it would parallelise
    if (rows <= 256 && cblk >= 16) nrb = 1;
    if (rows <= 0 || nrb <= 1) {
        if (dtype == SRNN_F32)
            colsum_pass<float>((const float*)src, lds, rows, cols, std::max<int64_t>(rows, 1), 1,
                               out, alpha, accumulate, true, s);
        else
            colsum_pass<bf16>((const bf16*)src, lds, rows, cols, std::max<int64_t>(rows, 1), 1,
                              out, alpha, accumulate, true, s);
        SRNN_LAUNCH_CHECK();
        return 0;
    }
    const int64_t rpb = (rows + nrb - 1) / nrb;
    nrb = (rows + rpb - 1) / rpb;
    SRNN_REQUIRE(nrb * cols <= work_elems, "colsum: workspace too small");
    if (dtype == SRNN_F32)
        colsum_pass<float>((const float*)src, lds, rows, cols, rpb, (int)nrb, work, 1.f, 0, false, s);
    else
        colsum_pass<bf16>((const bf16*)src, lds, rows, cols, rpb, (int)nrb, work, 1.f, 0, false, s);
    SRNN_LAUNCH_CHECK();
    colsum_pass<float>(work, cols, nrb, cols, nrb, 1, out, alpha, accumulate, true, s);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// out[b][c] = sum_{f < F} src[(b * F + f) * lds + c]   (per-sequence sum over frames)
__global__ void segsum_kernel(const float* __restrict__ src, int64_t lds, int B, int F, int D,
                              float* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (c >= D) return;
    const float* p = src + (int64_t)b * F * lds + c;
    float s = 0.f;
    for (int f = 0; f < F; ++f) s += p[(int64_t)f * lds];
    out[(int64_t)b * D + c] = s;
}

extern "C" int srnn_segsum(const float* src, int64_t lds, int B, int F, int D, float* out,
                           void* stream) {
    if ((int64_t)B * D <= 0) return 0;
    hipLaunchKernelGGL(segsum_kernel, dim3(cdiv(D, 256), B), dim3(256), 0, (hipStream_t)stream,
                       src, lds, B, F, D, out);
    SRNN_LAUNCH_CHECK();
    return 0;
}

extern "C" int srnn_colsum(int dtype, const void* src, int64_t lds, int64_t rows, int cols,
                           float* out, float alpha, int accumulate, float* work,
                           int64_t work_elems, void* stream) {
    return srnn_colsum_impl(dtype, src, lds, rows, cols, out, alpha, accumulate, work, work_elems,
                            (hipStream_t)stream);
}

// ------------------------------------------------------------------ clip + Adam
// optim.py:11-13 clamps every grad to [lo, hi]; then torch.optim.Adam (single-tensor
// form, torch 2.x order): m.lerp_(g, 1-b1); v = v*b2 + (1-b2)*g*g;
// p -= step_size * m / (sqrt(v)/sqrt(bc2) + eps).  Optionally refreshes a bf16 copy.
__global__ void adam_clip_kernel(float* __restrict__ p, float* __restrict__ g,
                                 float* __restrict__ m, float* __restrict__ v,
                                 bf16* __restrict__ p_lp, int64_t n, float lo, float hi, float w1,
                                 float b2, float omb2, float step_size, float bc2s, float eps) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float gi = fminf(fmaxf(g[i], lo), hi);
    g[i] = gi;   // hardtanh_ is in place in the reference (optim.py:13)
    float mi = m[i];
    mi = mi + w1 * (gi - mi);
    float vi = v[i] * b2;
    vi = vi + omb2 * gi * gi;
    float denom = sqrtf(vi) / bc2s + eps;
    float pi = p[i] + (-step_size) * mi / denom;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    if (p_lp) p_lp[i] = __float2bfloat16(pi);
}

// Multi-tensor form: every parameter of the optimizer in ONE launch (the per-tensor
// descriptors travel in the kernel argument block).  A workgroup takes a 2048-element
// chunk of the concatenated index space; the chunk's first tensor is found by a uniform
// scan of the offsets, and a thread steps to the next tensor at a boundary.
// GT: gradient element type (float, or bf16 for gradients reduced in bf16 buckets under data
// parallelism); gscale multiplies the gradient before the clamp (the DP mean's 1 / N, so the
// summed buckets need no separate scaling pass).  fp32 gradients are written back clamped
// (hardtanh_ is in place in the reference, optim.py:13); bf16 ones are only read.
#define ADAM_MT 64
struct AdamMulti {
    int nt;
    int64_t off[ADAM_MT + 1];     // element offsets
    int boff[ADAM_MT + 1];        // first workgroup of each tensor
    float* p[ADAM_MT];
    void* g[ADAM_MT];
    float* m[ADAM_MT];
    float* v[ADAM_MT];
    bf16* plp[ADAM_MT];
};

__device__ __forceinline__ floatx4 adam_ld4(const float* g) {
    return *reinterpret_cast<const floatx4*>(g);
}
__device__ __forceinline__ floatx4 adam_ld4(const bf16* g) {
    const uint2 u = *reinterpret_cast<const uint2*>(g);
    return floatx4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                   __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
}

template <typename GT>
__global__ __launch_bounds__(256) void adam_clip_multi_kernel(AdamMulti a, float lo, float hi,
                                                              float w1, float b2, float omb2,
                                                              float step_size, float bc2s,
                                                              float eps, float gscale,
                                                              const int* skip,
                                                              const int64_t* dstep, double lr,
                                                              double beta1, double beta2) {
    constexpr int CH = 2048;
    constexpr bool WB = std::is_same<GT, float>::value;      // write the clamped grad back
    // a persistent sweep of this step gave up a hand-off (persist.hip): its gradients are
    // invalid, so neither the weights nor the Adam moments move (the host raises after)
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(skip, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT)))
        return;
    // device-resident step count (graph-replayed steps, srnn_adam_clip_multi3): the bias
    // corrections follow from the count of completed steps, with the host formula
    if (dstep) {
        const double s = (double)(*dstep + 1);
        step_size = (float)(lr / (1.0 - pow(beta1, s)));
        bc2s = (float)sqrt(1.0 - pow(beta2, s));
    }
    // workgroups never straddle tensors, so the tensor index is uniform and its pointers
    // come from the argument block with scalar loads
    int t = 0;
    while (t + 1 < a.nt && a.boff[t + 1] <= (int)blockIdx.x) ++t;
    t = __builtin_amdgcn_readfirstlane(t);
    const int64_t n = a.off[t + 1] - a.off[t];
    float* __restrict__ P = a.p[t];
    GT* __restrict__ G = (GT*)a.g[t];
    float* __restrict__ Mm = a.m[t];
    float* __restrict__ V = a.v[t];
    bf16* __restrict__ PL = a.plp[t];
    const int64_t j0 = (int64_t)(blockIdx.x - a.boff[t]) * CH;
    // (a null gradient is an all-zero one: a parameter backward did not reach this
    //  step, e.g. the learned h0 on a carried chunk -- torch-0.4 zero_grad semantics)
    auto upd = [&](float g, float& p, float& m, float& v) {
        const float gi = fminf(fmaxf(g * gscale, lo), hi);
        m = m + w1 * (gi - m);
        v = v * b2;
        v = v + omb2 * gi * gi;
        const float denom = sqrtf(v) / bc2s + eps;
        p = p + (-step_size) * m / denom;
        return gi;
    };
    // two 4-element chunks per thread (16-B accesses; every tensor is its own allocation or a
    // 64-element-aligned view, so chunk starts are 16-B aligned); the ragged end element by
    // element
#pragma unroll
    for (int c = 0; c < CH / 1024; ++c) {
        const int64_t j = j0 + c * 1024 + 4 * threadIdx.x;
        if (j + 4 <= n) {
            floatx4 g4 = G ? adam_ld4(G + j) : floatx4{0.f, 0.f, 0.f, 0.f};
            floatx4 p4 = *reinterpret_cast<const floatx4*>(P + j);
            floatx4 m4 = *reinterpret_cast<const floatx4*>(Mm + j);
            floatx4 v4 = *reinterpret_cast<const floatx4*>(V + j);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float pe = p4[e], me = m4[e], ve = v4[e];
                g4[e] = upd(g4[e], pe, me, ve);
                p4[e] = pe; m4[e] = me; v4[e] = ve;
            }
            if (WB && G) *reinterpret_cast<floatx4*>((float*)G + j) = g4;
            *reinterpret_cast<floatx4*>(Mm + j) = m4;
            *reinterpret_cast<floatx4*>(V + j) = v4;
            *reinterpret_cast<floatx4*>(P + j) = p4;
            if (PL) {
                const unsigned lo2 = (unsigned)__bfloat16_as_ushort(__float2bfloat16(p4[0])) |
                                     ((unsigned)__bfloat16_as_ushort(__float2bfloat16(p4[1])) << 16);
                const unsigned hi2 = (unsigned)__bfloat16_as_ushort(__float2bfloat16(p4[2])) |
                                     ((unsigned)__bfloat16_as_ushort(__float2bfloat16(p4[3])) << 16);
                *reinterpret_cast<uint2*>(PL + j) = make_uint2(lo2, hi2);
            }
        } else {
            for (int64_t k = j; k < n && k < j + 4; ++k) {
                float pe = P[k], me = Mm[k], ve = V[k];
                const float gi = upd(G ? to_f(G[k]) : 0.f, pe, me, ve);
                if (WB && G) ((float*)G)[k] = gi;
                Mm[k] = me;
                V[k] = ve;
                P[k] = pe;
                if (PL) PL[k] = __float2bfloat16(pe);
            }
        }
    }
}

extern "C" int srnn_adam_clip_multi3(int ntensors, float* const* p, void* const* g, int gdtype,
                                     float gscale, float* const* m, float* const* v,
                                     void* const* p_bf16, const int64_t* n, float clip_lo,
                                     float clip_hi, double lr, double beta1, double beta2,
                                     double eps, int64_t step, const int64_t* dstep,
                                     void* stream) {
    SRNN_REQUIRE(ntensors >= 0, "adam_multi: bad tensor count");
    SRNN_REQUIRE(dstep || step >= 1, "adam: step must be >= 1");
    if (dstep) step = 1;   // placeholder: the kernel reads the count
    SRNN_REQUIRE(gdtype == SRNN_F32 || gdtype == SRNN_BF16, "adam_multi: gradient dtype");
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    const float step_size = (float)(lr / bc1);
    const float bc2s = (float)sqrt(bc2);
    const int* skip = srnn_sticky_flag();
    SRNN_REQUIRE(skip, "adam_multi: sticky flag allocation failed");
    // chunks of up to ADAM_MT non-empty tensors; the next chunk starts where this one's scan
    // stopped (empty tensors are skipped, so that is not t0 + ADAM_MT)
    for (int t0 = 0; t0 < ntensors;) {
        AdamMulti a;
        a.nt = 0;
        a.off[0] = 0;
        a.boff[0] = 0;
        int t = t0;
        for (; t < ntensors && a.nt < ADAM_MT; ++t) {
            if (n[t] <= 0) continue;
            const int k = a.nt++;
            a.p[k] = p[t]; a.g[k] = g[t]; a.m[k] = m[t]; a.v[k] = v[t];
            a.plp[k] = p_bf16 ? (bf16*)p_bf16[t] : nullptr;
            a.off[k + 1] = a.off[k] + n[t];
            a.boff[k + 1] = a.boff[k] + (int)((n[t] + 2047) / 2048);
        }
        t0 = t;
        if (a.nt == 0) continue;
        const int64_t nblk = a.boff[a.nt];
        if (gdtype == SRNN_F32)
            hipLaunchKernelGGL(adam_clip_multi_kernel<float>, dim3((unsigned)nblk), dim3(256), 0,
                               (hipStream_t)stream, a, clip_lo, clip_hi, (float)(1.0 - beta1),
                               (float)beta2, (float)(1.0 - beta2), step_size, bc2s, (float)eps,
                               gscale, skip, dstep, lr, beta1, beta2);
        else
            hipLaunchKernelGGL(adam_clip_multi_kernel<bf16>, dim3((unsigned)nblk), dim3(256), 0,
                               (hipStream_t)stream, a, clip_lo, clip_hi, (float)(1.0 - beta1),
                               (float)beta2, (float)(1.0 - beta2), step_size, bc2s, (float)eps,
                               gscale, skip, dstep, lr, beta1, beta2);
        SRNN_LAUNCH_CHECK();
    }
    return 0;
}

extern "C" int srnn_adam_clip_multi2(int ntensors, float* const* p, void* const* g, int gdtype,
                                     float gscale, float* const* m, float* const* v,
                                     void* const* p_bf16, const int64_t* n, float clip_lo,
                                     float clip_hi, double lr, double beta1, double beta2,
                                     double eps, int64_t step, void* stream) {
    return srnn_adam_clip_multi3(ntensors, p, g, gdtype, gscale, m, v, p_bf16, n, clip_lo,
                                 clip_hi, lr, beta1, beta2, eps, step, nullptr, stream);
}

// Completed-step counters of srnn_adam_clip_multi3: +1 each, unless the sticky failure flag
// is up (that step's update was skipped, so the bias correction must not advance either).
__global__ void step_advance_kernel(int64_t* dstep, int n, const int* skip) {
    if (__hip_atomic_load(skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    const int i = threadIdx.x;
    if (i < n) dstep[i] = dstep[i] + 1;
}

extern "C" int srnn_step_advance(int64_t* dstep, int n, void* stream) {
    SRNN_REQUIRE(dstep && n >= 0 && n <= 1024, "step_advance: bad arguments");
    if (n == 0) return 0;
    const int* skip = srnn_sticky_flag();
    SRNN_REQUIRE(skip, "step_advance: sticky flag allocation failed");
    hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64 * (unsigned)cdiv(n, 64)), 0,
                       (hipStream_t)stream, dstep, n, skip);
    SRNN_LAUNCH_CHECK();
    return 0;
}

extern "C" int srnn_adam_clip_multi(int ntensors, float* const* p, float* const* g,
                                    float* const* m, float* const* v, void* const* p_bf16,
                                    const int64_t* n, float clip_lo, float clip_hi, double lr,
                                    double beta1, double beta2, double eps, int64_t step,
                                    void* stream) {
    return srnn_adam_clip_multi2(ntensors, p, (void* const*)g, SRNN_F32, 1.0f, m, v, p_bf16, n,
                                 clip_lo, clip_hi, lr, beta1, beta2, eps, step, stream);
}

// ------------------------------------------------------------------ gradient buckets
// Data-parallel gradient packing (distributed.py GradAllReduce): n gradient tensors (fp32,
// or NULL = all zero) copied into one flat bucket at 64-element-aligned offsets, converted to
// the bucket's dtype, in ONE launch (the per-parameter copy_ launches it replaces cost a
// launch each); the reduced bucket is read in place by srnn_adam_clip_multi2.
#define PACK_MT 64
struct PackMulti {
    int nt;
    int boff[PACK_MT + 1];
    const float* src[PACK_MT];
    int64_t n[PACK_MT];
    int64_t dst_off[PACK_MT];
};

template <typename TD>
__global__ __launch_bounds__(256) void pack_grads_kernel(PackMulti a, TD* __restrict__ flat) {
    int t = 0;
    while (t + 1 < a.nt && a.boff[t + 1] <= (int)blockIdx.x) ++t;
    t = __builtin_amdgcn_readfirstlane(t);
    const float* __restrict__ src = a.src[t];
    const int64_t n = a.n[t];
    TD* __restrict__ dst = flat + a.dst_off[t];
    const int64_t j0 = (int64_t)(blockIdx.x - a.boff[t]) * 2048;
    for (int64_t j = j0 + threadIdx.x; j < n && j < j0 + 2048; j += 256)
        dst[j] = from_f<TD>(src ? src[j] : 0.f);
}

extern "C" int srnn_pack_grads(int ntensors, const float* const* src, const int64_t* n,
                               const int64_t* dst_off, void* flat, int dtype, void* stream) {
    SRNN_REQUIRE(ntensors >= 0 && flat, "pack_grads: bad arguments");
    SRNN_REQUIRE(dtype == SRNN_F32 || dtype == SRNN_BF16, "pack_grads: dtype");
    for (int t0 = 0; t0 < ntensors;) {
        PackMulti a;
        a.nt = 0;
        a.boff[0] = 0;
        int t = t0;
        for (; t < ntensors && a.nt < PACK_MT; ++t) {
            if (n[t] <= 0) continue;
            const int k = a.nt++;
            a.src[k] = src[t]; a.n[k] = n[t]; a.dst_off[k] = dst_off[t];
            a.boff[k + 1] = a.boff[k] + (int)((n[t] + 2047) / 2048);
        }
        t0 = t;
        if (a.nt == 0) continue;
        if (dtype == SRNN_F32)
            hipLaunchKernelGGL(pack_grads_kernel<float>, dim3((unsigned)a.boff[a.nt]), dim3(256),
                               0, (hipStream_t)stream, a, (float*)flat);
        else
            hipLaunchKernelGGL(pack_grads_kernel<bf16>, dim3((unsigned)a.boff[a.nt]), dim3(256),
                               0, (hipStream_t)stream, a, (bf16*)flat);
        SRNN_LAUNCH_CHECK();
    }
    return 0;
}

// bf16 copies of n fp32 tensors in ONE launch (ZeRO-1 data parallelism, distributed.py: after the
// parameter all-gather, the other ranks' shards of every parameter refresh its bf16 copy).
struct CastMulti {
    int nt;
    int boff[PACK_MT + 1];
    const float* src[PACK_MT];
    bf16* dst[PACK_MT];
    int64_t n[PACK_MT];
};

__global__ __launch_bounds__(256) void cast_multi_kernel(CastMulti a) {
    int t = 0;
    while (t + 1 < a.nt && a.boff[t + 1] <= (int)blockIdx.x) ++t;
    t = __builtin_amdgcn_readfirstlane(t);
    const float* __restrict__ src = a.src[t];
    bf16* __restrict__ dst = a.dst[t];
    const int64_t n = a.n[t];
    const int64_t j0 = (int64_t)(blockIdx.x - a.boff[t]) * 2048;
    for (int64_t j = j0 + threadIdx.x; j < n && j < j0 + 2048; j += 256) dst[j] = __float2bfloat16(src[j]);
}

extern "C" int srnn_cast_multi(int ntensors, const float* const* src, void* const* dst,
                               const int64_t* n, void* stream) {
    SRNN_REQUIRE(ntensors >= 0, "cast_multi: bad arguments");
    for (int t0 = 0; t0 < ntensors;) {
        CastMulti a;
        a.nt = 0;
        a.boff[0] = 0;
        int t = t0;
        for (; t < ntensors && a.nt < PACK_MT; ++t) {
            if (n[t] <= 0) continue;
            SRNN_REQUIRE(src[t] && dst[t], "cast_multi: null tensor");
            const int k = a.nt++;
            a.src[k] = src[t]; a.dst[k] = (bf16*)dst[t]; a.n[k] = n[t];
            a.boff[k + 1] = a.boff[k] + (int)((n[t] + 2047) / 2048);
        }
        t0 = t;
        if (a.nt == 0) continue;
        hipLaunchKernelGGL(cast_multi_kernel, dim3((unsigned)a.boff[a.nt]), dim3(256), 0,
                           (hipStream_t)stream, a);
        SRNN_LAUNCH_CHECK();
    }
    return 0;
}

extern "C" int srnn_adam_clip(float* p, float* g, float* m, float* v, void* p_bf16,
                              int64_t n, float clip_lo, float clip_hi, double lr, double beta1,
                              double beta2, double eps, int64_t step, void* stream) {
    if (n <= 0) return 0;
    SRNN_REQUIRE(step >= 1, "adam: step must be >= 1");
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    const float step_size = (float)(lr / bc1);
    const float bc2s = (float)sqrt(bc2);
    hipLaunchKernelGGL(adam_clip_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, p,
                       g, m, v, (bf16*)p_bf16, n, clip_lo, clip_hi, (float)(1.0 - beta1),
                       (float)beta2, (float)(1.0 - beta2), step_size, bc2s, (float)eps);
    SRNN_LAUNCH_CHECK();
    return 0;
}
