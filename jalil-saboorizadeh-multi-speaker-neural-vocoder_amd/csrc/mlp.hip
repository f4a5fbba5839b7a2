// SampleLevelMLP kernels (model.py:266-325) and the loss / sampler around it.
//
// The embedding (Q x Q) followed by the FS0-tap Conv1d (D x Q x FS0, no bias) is a
// linear map of one-hot inputs, so it is folded into a per-tap table
//     Tab[k][q][:] = W[:, :, k] . E[q, :]          (FS0 x Q x D, built by one batched GEMM)
// and the first MLP layer becomes a 16-row gather-sum:  a1 = relu(sum_k Tab[k][x_{t+k}] + u_t).
// That removes the Q*FS0*D = 4.2 M MAC/sample dense conv (59 % of the reference's MLP
// FLOPs) from both the training and the generation path.
//
// The log-softmax + NLL (nn.py:66-70) is one wave per row (Q = 256 -> 4 values / lane,
// wave shuffles for max / sum) and writes the loss row and dlogits in the same pass.
// The generation sampler draws  argmax(exp(logp) / q), q ~ Exp(1)  -- exactly how
// torch>=2 implements `multinomial(1)` on CPU (model.py:514-517) -- with q either
// supplied (bit-replay of the reference's RNG) or from a counter-based Philox4x32-10.
#include <algorithm>

#include "samplernn_hip_internal.hpp"
#include "sampler.hpp"

// ------------------------------------------------------------------ L1 gather
// rows r = b * Tlen + t;  idx_k = x[b * ldx + xoff(+base) + t + k]
template <typename T, typename TU, int VPT>
__global__ __launch_bounds__(256) void mlp_l1_kernel(const T* __restrict__ tab,
                                                     const int64_t* __restrict__ x, int64_t ldx,
                                                     int xoff, const int* __restrict__ base,
                                                     int Tlen, const TU* __restrict__ upper,
                                                     int64_t ldu, T* __restrict__ out, int64_t ldo,
                                                     int D, int FS0, int Q) {
    const int64_t r = blockIdx.y;
    const int b = r / Tlen, t = r % Tlen;
    const int off = xoff + (base ? *base : 0);
    const int64_t* xr = x + (int64_t)b * ldx + off + t;
    const int o0 = (blockIdx.x * 256 + threadIdx.x) * VPT;
    if (o0 >= D) return;
    float acc[VPT];
    const TU* ur = upper + r * ldu + o0;
#pragma unroll
    for (int j = 0; j < VPT; ++j) acc[j] = to_f(ur[j]);
    // all index loads first, then all table-row loads: one exposed latency, not FS0
    constexpr int KMAX = 32;
    int qs[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
        if (k < FS0) qs[k] = (int)xr[k];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        if (k < FS0) {
            const T* tr = tab + ((int64_t)k * Q + qs[k]) * D + o0;
#pragma unroll
            for (int j = 0; j < VPT; ++j) acc[j] += to_f(tr[j]);
        }
    }
    T* orow = out + r * ldo + o0;
#pragma unroll
    for (int j = 0; j < VPT; ++j) orow[j] = from_f<T>(fmaxf(acc[j], 0.f));
}

// XCD-sliced variant for the training shape (many rows, D a multiple of 128): workgroup
// b works on column slice b % (D / 128), so with D = 1024 every XCD only ever gathers its
// own 128-column slice of the table -- 1 MiB in bf16, resident in that XCD's 4 MiB L2 --
// instead of all XCDs streaming the whole 8 MiB table from the Infinity Cache.  A row is
// one 16-lane group (8 columns = one 16-B bf16 load per lane and table row); its FS0
// (<= 32) indices are fetched by the group's lanes and broadcast with shuffles; each
// group works on two rows at a time so that 2 x FS0 gathers are in flight.
typedef unsigned short l1_u16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void l1_add8(const float* p, float (&a)[8]) {
    const floatx4 x = *reinterpret_cast<const floatx4*>(p);
    const floatx4 y = *reinterpret_cast<const floatx4*>(p + 4);
    a[0] += x[0]; a[1] += x[1]; a[2] += x[2]; a[3] += x[3];
    a[4] += y[0]; a[5] += y[1]; a[6] += y[2]; a[7] += y[3];
}
__device__ __forceinline__ void l1_add8(const bf16* p, float (&a)[8]) {
    const l1_u16x8 x = *reinterpret_cast<const l1_u16x8*>(p);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] += __uint_as_float((unsigned)x[e] << 16);
}
__device__ __forceinline__ void l1_store8(float* p, const float (&a)[8]) {
    *reinterpret_cast<floatx4*>(p) = floatx4{fmaxf(a[0], 0.f), fmaxf(a[1], 0.f), fmaxf(a[2], 0.f), fmaxf(a[3], 0.f)};
    *reinterpret_cast<floatx4*>(p + 4) = floatx4{fmaxf(a[4], 0.f), fmaxf(a[5], 0.f), fmaxf(a[6], 0.f), fmaxf(a[7], 0.f)};
}
__device__ __forceinline__ void l1_store8(bf16* p, const float (&a)[8]) {
    l1_u16x8 x;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = __bfloat16_as_ushort(__float2bfloat16(fmaxf(a[e], 0.f)));
    *reinterpret_cast<l1_u16x8*>(p) = x;
}

template <typename T, typename TU>
__global__ __launch_bounds__(256) void mlp_l1_xcd_kernel(const T* __restrict__ tab,
                                                         const int64_t* __restrict__ x,
                                                         int64_t ldx, int xoff, int Tlen, int64_t nrows,
                                                         int rows_per_block, int nslices,
                                                         const TU* __restrict__ upper,
                                                         int64_t ldu, T* __restrict__ out,
                                                         int64_t ldo, int D, int FS0, int Q) {
    const int slice = blockIdx.x % nslices;
    const int64_t rb = blockIdx.x / nslices;
    const int lane = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int c0 = slice * 128 + lane * 8;
    const int64_t rbeg = rb * rows_per_block;
    const int64_t rend = min(nrows, rbeg + rows_per_block);
    for (int64_t r = rbeg + grp; r < rend; r += 32) {
        const int64_t r2 = r + 16;
        const bool two = r2 < rend;
        const int b = (int)(r / Tlen), t = (int)(r - (int64_t)b * Tlen);
        const int64_t* xr = x + (int64_t)b * ldx + xoff + t;
        const int64_t rr = two ? r2 : r;
        const int b2 = (int)(rr / Tlen), t2 = (int)(rr - (int64_t)b2 * Tlen);
        const int64_t* xr2 = x + (int64_t)b2 * ldx + xoff + t2;
        const int qa0 = lane < FS0 ? (int)xr[lane] : 0;
        const int qa1 = lane + 16 < FS0 ? (int)xr[lane + 16] : 0;
        const int qb0 = lane < FS0 ? (int)xr2[lane] : 0;
        const int qb1 = lane + 16 < FS0 ? (int)xr2[lane + 16] : 0;
        float a[8], c[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] = c[e] = 0.f;
        l1_add8(upper + r * ldu + c0, a);
        l1_add8(upper + rr * ldu + c0, c);
        for (int k = 0; k < FS0; ++k) {
            const int qa = k < 16 ? __shfl(qa0, k, 16) : __shfl(qa1, k - 16, 16);
            const int qb = k < 16 ? __shfl(qb0, k, 16) : __shfl(qb1, k - 16, 16);
            l1_add8(tab + ((int64_t)k * Q + qa) * D + c0, a);
            l1_add8(tab + ((int64_t)k * Q + qb) * D + c0, c);
        }
        l1_store8(out + r * ldo + c0, a);
        if (two) l1_store8(out + r2 * ldo + c0, c);
    }
}

// LDS-resident variant for the bf16 training shape (FS0 = 16, Q = 256): workgroup (cg, rc)
// keeps the table slice Tab[:, :, 16 cg .. 16 cg + 16) -- 16 x 256 x 16 bf16 = 128 KiB -- in
// LDS for its whole chunk of batch rows, so every gather is a ds_read_b128 instead of an L2
// round trip (the L2 gather of mlp_l1_xcd_kernel moves 16 x 2 B per output element through
// the L2 -> CU path).  A row is two lanes (8 columns each); its 16 byte indices come from a
// double-buffered LDS copy of the batch row's index stream (aligned dword reads + alignbyte).
// Accumulation: v_dot2c_f32_bf16 against (1, 0) / (0, 1) adds one bf16 to an fp32 sum
// with a single rounding -- the same result as convert + add, in one instruction instead
// of two.  The (1, 0) operand must live in a VGPR: hipcc (ROCm 7.2) folds the constant
// 0x00003f80 into the inline constant 1.0, which the instruction reads as (0, 1)
// (tools/dot2_probe).  The summation order (upper, then taps 0..15) is mlp_l1_xcd_kernel's,
// so both produce identical bits.
typedef __bf16 l1_bf16x2 __attribute__((ext_vector_type(2)));
constexpr int L1L_NT = 1024;

__device__ __forceinline__ void l1l_add8(const uint4 v, float (&a)[8], l1_bf16x2 lo1,
                                         l1_bf16x2 hi1) {
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const l1_bf16x2 p = __builtin_bit_cast(l1_bf16x2, w[i]);
        a[2 * i] = __builtin_amdgcn_fdot2_f32_bf16(p, lo1, a[2 * i], false);
        a[2 * i + 1] = __builtin_amdgcn_fdot2_f32_bf16(p, hi1, a[2 * i + 1], false);
    }
}

// RPT: rows per thread per batch row (Tlen <= RPT * L1L_NT / 2), compile-time so the prefetch
// registers of unused rows are not allocated: at 1024 threads a wave has 128 VGPRs, and the
// spills of RPT = 4 at Tlen = 1024 put scratch reloads -- each waiting, vmcnt being in order,
// for every store issued before it -- inside the row loop
template <int RPT>
__global__ __launch_bounds__(L1L_NT, 1) void mlp_l1_lds_kernel(
    const bf16* __restrict__ tab, const int64_t* __restrict__ x, int64_t ldx, int xoff, int B,
    int Tlen, int bpc, const bf16* __restrict__ upper, int64_t ldu, bf16* __restrict__ out,
    int64_t ldo, int D, unsigned short* __restrict__ bits, int64_t ldb) {
    constexpr int FS = 16, Q = 256;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* tl = smem;                                        // [FS * Q][16] bf16 = 128 KiB
    unsigned char* ib = reinterpret_cast<unsigned char*>(smem + FS * Q * 32);
    const int W = Tlen + FS - 1, WP = (W + 4 + 15) & ~15;   // + 4: the last dword read
    const int tid = threadIdx.x;
    // blocks of one XCD (blockIdx % 8 under round-robin dispatch) cover 8 adjacent column
    // groups, so the 32-B pieces of a 128-B line of `upper` / `out` meet in one L2
    const int ncg = D / 16, xcd = blockIdx.x % 8, loc = blockIdx.x / 8;
    int cg, rc;
    if (ncg % 8 == 0) {
        const int per = ncg / 8;
        cg = xcd * per + loc % per;
        rc = loc / per;
    } else {
        cg = blockIdx.x % ncg;
        rc = blockIdx.x / ncg;
    }
    const int b0 = rc * bpc, b1 = min(B, b0 + bpc);
    if (b0 >= b1) return;
    const int c0 = cg * 16;
    for (int i = tid; i < FS * Q * 2; i += L1L_NT) {       // the table slice, 16 B per thread
        const int row = i >> 1, h = i & 1;
        *reinterpret_cast<uint4*>(tl + i * 16) =
            *reinterpret_cast<const uint4*>(tab + (int64_t)row * D + c0 + h * 8);
    }
    // the next batch row's indices and `upper` rows are loaded into registers one batch
    // row ahead (loads in flight across the current row's gathers), written / used after
    const int nrt = (Tlen + L1L_NT / 2 - 1) / (L1L_NT / 2);
    const int h = tid & 1, t0 = tid >> 1;
    // (the low 32-bit word of each int64 index: indices are < Q)
    unsigned xn[2];
    auto load_x = [&](int b) {
        const unsigned* xr = reinterpret_cast<const unsigned*>(x + (int64_t)b * ldx + xoff);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int p = tid + j * L1L_NT;
            xn[j] = xr[2 * min(p, W - 1)];
        }
    };
    auto put_x = [&](unsigned char* dst) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int p = tid + j * L1L_NT;
            if (p < WP) dst[p] = p < W ? (unsigned char)xn[j] : 0;
        }
    };
    uint4 un[RPT];
    auto load_u = [&](int b) {
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            const int t = min(t0 + i * (L1L_NT / 2), Tlen - 1);
            if (i < nrt)
                un[i] = *reinterpret_cast<const uint4*>(upper + ((int64_t)b * Tlen + t) * ldu + c0 + h * 8);
        }
    };
    unsigned one_lo = 0x00003f80u, one_hi = 0x3f800000u;   // (1, 0), (0, 1) in VGPRs
    asm volatile("" : "+v"(one_lo), "+v"(one_hi));
    const l1_bf16x2 lo1 = __builtin_bit_cast(l1_bf16x2, one_lo);
    const l1_bf16x2 hi1 = __builtin_bit_cast(l1_bf16x2, one_hi);
    const char* const tlh = tl + h * 16;                    // this lane's 8 columns of an entry
    load_x(b0);
    load_u(b0);
    put_x(ib);
    __syncthreads();
    for (int b = b0; b < b1; ++b) {
        const unsigned char* cur = ib + ((b - b0) & 1) * WP;
        const bool more = b + 1 < b1;
        if (more) load_x(b + 1);
        uint4 uc[RPT];
#pragma unroll
        for (int i = 0; i < RPT; ++i) uc[i] = un[i];
        if (more) load_u(b + 1);
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            const int t = t0 + i * (L1L_NT / 2);
            if (i >= nrt || t >= Tlen) break;
            const int64_t r = (int64_t)b * Tlen + t;
            float a[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] = 0.f;
            l1l_add8(uc[i], a, lo1, hi1);
            const int tb = t & ~3, sh = t & 3;
            const unsigned* iw = reinterpret_cast<const unsigned*>(cur + tb);
            unsigned w5[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) w5[j] = iw[j];
            unsigned q4[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) q4[j] = __builtin_amdgcn_alignbyte(w5[j + 1], w5[j], sh);
            uint4 tv[FS];
#pragma unroll
            for (int k = 0; k < FS; ++k) {
                // (q << 5) + this half's base, the tap's k Q 32 an immediate offset: one
                // shift-add per read after the byte extract
                const unsigned q = (q4[k >> 2] >> (8 * (k & 3))) & 0xffu;
                tv[k] = *reinterpret_cast<const uint4*>(tlh + k * Q * 32 + (q << 5));
            }
#pragma unroll
            for (int k = 0; k < FS; ++k) l1l_add8(tv[k], a, lo1, hi1);
            l1_u16x8 xv;
#pragma unroll
            for (int e = 0; e < 8; ++e) xv[e] = __bfloat16_as_ushort(__float2bfloat16(fmaxf(a[e], 0.f)));
            *reinterpret_cast<l1_u16x8*>(out + r * ldo + c0 + h * 8) = xv;
            if (bits) {
                // ReLU mask bits of the 16 columns (stored bf16 > 0): this thread's 8, its
                // pair lane's 8 (DPP quad_perm 1,0,3,2).  A stored value is a bf16 in
                // [0, 0x7f80] (fmax took NaN to 0), so u != 0 is bit 15 of u + 0x7fff, for
                // both halves of a word in one add (no carry crosses: 0x7f80 + 0x7fff < 2^16)
                const uint4 w = __builtin_bit_cast(uint4, xv);
                const unsigned t0 = (w.x + 0x7fff7fffu) & 0x80008000u;
                const unsigned t1 = (w.y + 0x7fff7fffu) & 0x80008000u;
                const unsigned t2 = (w.z + 0x7fff7fffu) & 0x80008000u;
                const unsigned t3 = (w.w + 0x7fff7fffu) & 0x80008000u;
                const unsigned sb = (t0 >> 15) | (t1 >> 13) | (t2 >> 11) | (t3 >> 9);
                const unsigned nib = (sb | (sb >> 15)) & 0xffu;   // bit e = value e
                const unsigned pn = dpp_u32<0xB1>(nib);
                // (grouped layout, ldb = 0: [column group][row] -- the wave's 32 rows are one
                //  contiguous 64-B run)
                if (h == 0)
                    bits[srnn_bits_index(r, c0 >> 4, (int64_t)B * Tlen, ldb)] =
                        (unsigned short)(nib | (pn << 8));
            }
        }
        if (more) put_x(ib + ((b + 1 - b0) & 1) * WP);
        __syncthreads();                                    // next buffer staged, cur free
    }
}

template <typename T, typename TU>
static int mlp_l1_launch(const T* tab, const int64_t* x, int64_t ldx, int xoff, const int* base,
                         int B, int Tlen, const TU* upper, int64_t ldu, T* out, int64_t ldo,
                         int D, int FS0, int Q, hipStream_t s, unsigned short* bits = nullptr,
                         int64_t ldb = 0) {
    const int64_t nrows = (int64_t)B * Tlen;
    const int ue = (int)sizeof(TU);
    if constexpr (sizeof(T) == 2 && sizeof(TU) == 2) {
        const int W = Tlen + FS0 - 1, WP = (W + 4 + 15) & ~15;
        const int ncg = D / 16;
        const int lds = 16 * 256 * 32 + 2 * WP;
        if (!base && FS0 == 16 && Q == 256 && D % 16 == 0 && ncg <= 256 && lds <= 160 * 1024 &&
            Tlen <= 4 * (L1L_NT / 2) && WP <= 2 * L1L_NT &&
            nrows >= 4096 && ldu % 8 == 0 && (uintptr_t)upper % 16 == 0 && ldo % 8 == 0 &&
            (uintptr_t)out % 16 == 0 && (uintptr_t)tab % 16 == 0 && env_flag("SRNN_L1_LDS", 1)) {
            const int nrc = std::max(1, std::min(B, 256 / ncg));
            const int bpc = (B + nrc - 1) / nrc;
            const int nrc2 = (B + bpc - 1) / bpc;
            const int nrt = (Tlen + L1L_NT / 2 - 1) / (L1L_NT / 2);
            auto kern = nrt <= 2 ? mlp_l1_lds_kernel<2> : mlp_l1_lds_kernel<4>;
            static bool attr[2] = {false, false};
            if (!attr[nrt > 2]) {
                SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)kern,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   160 * 1024));
                attr[nrt > 2] = true;
            }
            hipLaunchKernelGGL(kern, dim3(ncg * nrc2), dim3(L1L_NT), lds, s,
                               (const bf16*)tab, x, ldx, xoff, B, Tlen, bpc, (const bf16*)upper,
                               ldu, (bf16*)out, ldo, D, bits, ldb);
            SRNN_LAUNCH_CHECK();
            return 0;
        }
    }
    if (!base && D % 128 == 0 && nrows >= 4096 && (ldu * ue) % 16 == 0 &&
        (uintptr_t)upper % 16 == 0 && (ldo * (int)sizeof(T)) % 16 == 0 &&
        (uintptr_t)out % 16 == 0 && (uintptr_t)tab % 16 == 0) {
        const int nslices = D / 128;
        const int rpb = 64;
        const int64_t nblk = (nrows + rpb - 1) / rpb * nslices;
        SRNN_REQUIRE(nblk < (1ll << 31), "mlp_l1: too many rows");
        hipLaunchKernelGGL((mlp_l1_xcd_kernel<T, TU>), dim3((unsigned)nblk), dim3(256), 0, s, tab,
                           x, ldx, xoff, Tlen, nrows, rpb, nslices, upper, ldu, out, ldo, D, FS0, Q);
    } else {
        dim3 grid(cdiv(D, 256 * 4), nrows);
        hipLaunchKernelGGL((mlp_l1_kernel<T, TU, 4>), grid, dim3(256), 0, s, tab, x, ldx, xoff,
                           base, Tlen, upper, ldu, out, ldo, D, FS0, Q);
    }
    SRNN_LAUNCH_CHECK();
    // (the other paths: the mask bits from the written rows)
    if (bits)
        return srnn_relu_bits_impl(sizeof(T) == 2 ? SRNN_BF16 : SRNN_F32, out, ldo, (int)nrows, D,
                                   bits, ldb, s);
    return 0;
}

int srnn_mlp_l1_impl(int dtype, const void* tab, const int64_t* x, int64_t ldx, int xoff,
                     const int* base, int B, int Tlen, int upper_dtype, const void* upper,
                     int64_t ldu, void* out, int64_t ldo, int D, int FS0, int Q, hipStream_t s) {
    SRNN_REQUIRE(D % 4 == 0, "mlp_l1: D must be a multiple of 4");
    SRNN_REQUIRE(FS0 <= 32, "mlp_l1: frame_sizes[0] must be <= 32");
    SRNN_REQUIRE(upper_dtype == SRNN_F32 || upper_dtype == SRNN_BF16, "mlp_l1: bad upper dtype");
    if ((int64_t)B * Tlen <= 0) return 0;
    if (dtype == SRNN_F32) {
        if (upper_dtype == SRNN_F32)
            return mlp_l1_launch<float, float>((const float*)tab, x, ldx, xoff, base, B, Tlen,
                                               (const float*)upper, ldu, (float*)out, ldo, D, FS0, Q, s);
        return mlp_l1_launch<float, bf16>((const float*)tab, x, ldx, xoff, base, B, Tlen,
                                          (const bf16*)upper, ldu, (float*)out, ldo, D, FS0, Q, s);
    }
    if (upper_dtype == SRNN_F32)
        return mlp_l1_launch<bf16, float>((const bf16*)tab, x, ldx, xoff, base, B, Tlen,
                                          (const float*)upper, ldu, (bf16*)out, ldo, D, FS0, Q, s);
    return mlp_l1_launch<bf16, bf16>((const bf16*)tab, x, ldx, xoff, base, B, Tlen,
                                     (const bf16*)upper, ldu, (bf16*)out, ldo, D, FS0, Q, s);
}

// the same with the ReLU mask of a1 as bits (u16 per 16 columns, row stride ldb) for the
// backward's masked GEMM (bf16 table and upper)
extern "C" int srnn_mlp_l1_bits(const void* tab, const int64_t* x, int64_t ldx, int xoff, int B,
                                int Tlen, const void* upper, int64_t ldu, void* out, int64_t ldo,
                                int D, int FS0, int Q, unsigned short* bits, int64_t ldb,
                                void* stream) {
    SRNN_REQUIRE(D % 16 == 0 && FS0 <= 32 && bits && (ldb >= D / 16 || (ldb == 0 && D % 64 == 0)),
                 "mlp_l1_bits: bad args (bit row stride >= D / 16, or 0 for the grouped layout)");
    if ((int64_t)B * Tlen <= 0) return 0;
    return mlp_l1_launch<bf16, bf16>((const bf16*)tab, x, ldx, xoff, nullptr, B, Tlen,
                                     (const bf16*)upper, ldu, (bf16*)out, ldo, D, FS0, Q,
                                     (hipStream_t)stream, bits, ldb);
}

extern "C" int srnn_mlp_l1(int dtype, const void* tab, const int64_t* x, int64_t ldx, int xoff,
                           int B, int Tlen, int upper_dtype, const void* upper, int64_t ldu,
                           void* out, int64_t ldo, int D, int FS0, int Q, void* stream) {
    return srnn_mlp_l1_impl(dtype, tab, x, ldx, xoff, nullptr, B, Tlen, upper_dtype, upper, ldu,
                            out, ldo, D, FS0, Q, (hipStream_t)stream);
}

// ------------------------------------------------------------------ log-softmax + NLL
// One wave per row (Q = 256: lane holds q = lane + 64 j).  Writes
//   loss_row[r] = lse - z[target]     (if loss_row)
//   logp[r, q]  = (z - max) - log(sum exp(z - max))   (if logp; torch CPU op order)
//   dz[r, q]    = (softmax - onehot) * gscale        (if dz; T dtype)
template <typename TG>
__global__ __launch_bounds__(256) void logsoftmax_nll_kernel(
    const float* __restrict__ z, int64_t ldz, const int64_t* __restrict__ target, int64_t ldt,
    int Tlen, int64_t rows, float* __restrict__ loss_row, float* __restrict__ logp, int64_t ldl,
    TG* __restrict__ dz, int64_t ldd, float gscale) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    const float* zr = z + r * ldz;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = zr[lane + 64 * j];
    float m = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) s += expf(v[j] - m);
    s = wave_sum(s);
    const float ls = logf(s);
    int64_t tgt = -1;
    if (target) {
        const int b = r / Tlen, t = r % Tlen;
        tgt = target[(int64_t)b * ldt + t];
    }
    if (logp) {
        float* lr = logp + r * ldl;
#pragma unroll
        for (int j = 0; j < 4; ++j) lr[lane + 64 * j] = (v[j] - m) - ls;
    }
    if (loss_row && lane == (int)(tgt & 63)) {
        const int j = (int)(tgt >> 6);
        float vt = v[0];
#pragma unroll
        for (int jj = 1; jj < 4; ++jj) if (jj == j) vt = v[jj];
        loss_row[r] = -((vt - m) - ls);
    }
    if (dz) {
        TG* dr = dz + r * ldd;
        const float inv = 1.0f / s;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int q = lane + 64 * j;
            float p = expf(v[j] - m) * inv;
            if (q == tgt) p -= 1.0f;
            dr[q] = from_f<TG>(p * gscale);
        }
    }
}

extern "C" int srnn_logsoftmax_nll(const float* z, int64_t ldz, const int64_t* target, int64_t ldt,
                                   int Tlen, int64_t rows, int Q, float* loss_row, float* logp,
                                   int64_t ldl, void* dz, int dz_dtype, int64_t ldd, float gscale,
                                   void* stream) {
    SRNN_REQUIRE(Q == 256, "logsoftmax_nll: q_levels must be 256");
    SRNN_REQUIRE(!(loss_row || dz) || target, "logsoftmax_nll: loss/grad needs target");
    if (rows <= 0) return 0;
    dim3 grid(cdiv(rows, 4));
    hipStream_t s = (hipStream_t)stream;
    if (dz_dtype == SRNN_BF16)
        hipLaunchKernelGGL((logsoftmax_nll_kernel<bf16>), grid, dim3(256), 0, s, z, ldz, target,
                           ldt, Tlen, rows, loss_row, logp, ldl, (bf16*)dz, ldd, gscale);
    else
        hipLaunchKernelGGL((logsoftmax_nll_kernel<float>), grid, dim3(256), 0, s, z, ldz, target,
                           ldt, Tlen, rows, loss_row, logp, ldl, (float*)dz, ldd, gscale);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// dz = dlogp - exp(logp) * sum(dlogp)   (one wave per row)
template <typename TG>
__global__ __launch_bounds__(256) void logsoftmax_bwd_kernel(const float* __restrict__ dl,
                                                             int64_t lddl,
                                                             const float* __restrict__ lp,
                                                             int64_t ldl, int64_t rows,
                                                             TG* __restrict__ dz, int64_t ldd) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    float g[4], p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        g[j] = dl[r * lddl + lane + 64 * j];
        p[j] = lp[r * ldl + lane + 64 * j];
    }
    float s = wave_sum(g[0] + g[1] + g[2] + g[3]);
#pragma unroll
    for (int j = 0; j < 4; ++j) dz[r * ldd + lane + 64 * j] = from_f<TG>(g[j] - expf(p[j]) * s);
}

extern "C" int srnn_logsoftmax_bwd(const float* dlogp, int64_t lddl, const float* logp,
                                   int64_t ldl, int64_t rows, int Q, void* dz, int dz_dtype,
                                   int64_t ldd, void* stream) {
    SRNN_REQUIRE(Q == 256, "logsoftmax_bwd: q_levels must be 256");
    if (rows <= 0) return 0;
    dim3 grid(cdiv(rows, 4));
    if (dz_dtype == SRNN_BF16)
        hipLaunchKernelGGL((logsoftmax_bwd_kernel<bf16>), grid, dim3(256), 0, (hipStream_t)stream,
                           dlogp, lddl, logp, ldl, rows, (bf16*)dz, ldd);
    else
        hipLaunchKernelGGL((logsoftmax_bwd_kernel<float>), grid, dim3(256), 0,
                           (hipStream_t)stream, dlogp, lddl, logp, ldl, rows, (float*)dz, ldd);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// Fused NLL-in-bits + log-softmax backward (nn.py:66-70 then model.py:324-325): the loss
// gradient w.r.t. the log-probs is -c onehot(target), c = g log2(e) / N, so the logits'
// gradient is dz = dlogp - exp(logp) sum(dlogp) = c (exp(logp) - onehot), written straight
// in the GEMM operand dtype -- the dense (rows, Q) fp32 dlogp of the two-kernel path is
// never materialised nor re-read.  The arithmetic is the two-kernel path's, value for value
// (g_q = -c or 0, s = -c exactly, dz = g_q - exp(logp) s), so the results are identical.
template <typename TG>
__global__ __launch_bounds__(256) void nll_logsoftmax_bwd_kernel(
    const int64_t* __restrict__ target, int64_t ldt, int Tlen, int64_t rows,
    const float* __restrict__ lp, int64_t ldl, float gscale, const float* __restrict__ gmul,
    TG* __restrict__ dz, int64_t ldd) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    if (gmul) gscale *= *gmul;
    const int64_t b = r / Tlen, t = r - b * Tlen;
    const int tq = (int)target[b * ldt + t];
    float g[4], p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        g[j] = (lane + 64 * j == tq) ? -gscale : 0.f;
        p[j] = lp[r * ldl + lane + 64 * j];
    }
    const float s = wave_sum(g[0] + g[1] + g[2] + g[3]);
#pragma unroll
    for (int j = 0; j < 4; ++j) dz[r * ldd + lane + 64 * j] = from_f<TG>(g[j] - expf(p[j]) * s);
}

extern "C" int srnn_nll_logsoftmax_bwd(const int64_t* target, int64_t ldt, int Tlen,
                                       int64_t rows, int Q, const float* logp, int64_t ldl,
                                       float gscale, const float* gmul, void* dz, int dz_dtype,
                                       int64_t ldd, void* stream) {
    SRNN_REQUIRE(Q == 256, "nll_logsoftmax_bwd: q_levels must be 256");
    if (rows <= 0) return 0;
    dim3 grid(cdiv(rows, 4));
    if (dz_dtype == SRNN_BF16)
        hipLaunchKernelGGL((nll_logsoftmax_bwd_kernel<bf16>), grid, dim3(256), 0,
                           (hipStream_t)stream, target, ldt, Tlen, rows, logp, ldl, gscale, gmul,
                           (bf16*)dz, ldd);
    else
        hipLaunchKernelGGL((nll_logsoftmax_bwd_kernel<float>), grid, dim3(256), 0,
                           (hipStream_t)stream, target, ldt, Tlen, rows, logp, ldl, gscale, gmul,
                           (float*)dz, ldd);
    SRNN_LAUNCH_CHECK();
    return 0;
}

__global__ void nll_fwd_kernel(const float* __restrict__ lp, int64_t ldl,
                               const int64_t* __restrict__ target, int64_t ldt, int Tlen,
                               int64_t rows, float* __restrict__ loss_row) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const int64_t b = r / Tlen, t = r % Tlen;
    loss_row[r] = -lp[r * ldl + target[b * ldt + t]];
}

__global__ void nll_bwd_kernel(const int64_t* __restrict__ target, int64_t ldt, int Tlen,
                               int64_t rows, int Q, float* __restrict__ dl, int64_t ldd,
                               float gscale, const float* __restrict__ gmul) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= rows * Q) return;
    if (gmul) gscale *= *gmul;
    const int64_t r = e / Q;
    const int q = e % Q;
    const int64_t b = r / Tlen, t = r % Tlen;
    dl[r * ldd + q] = (q == target[b * ldt + t]) ? -gscale : 0.f;
}

extern "C" int srnn_nll_fwd(const float* logp, int64_t ldl, const int64_t* target, int64_t ldt,
                            int Tlen, int64_t rows, float* loss_row, void* stream) {
    if (rows <= 0) return 0;
    hipLaunchKernelGGL(nll_fwd_kernel, dim3(cdiv(rows, 256)), dim3(256), 0, (hipStream_t)stream,
                       logp, ldl, target, ldt, Tlen, rows, loss_row);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// Q = 256: one wave per row, 16-B stores (the dense gradient is 4 B x Q per row)
__global__ __launch_bounds__(256) void nll_bwd_q256_kernel(const int64_t* __restrict__ target,
                                                           int64_t ldt, int Tlen, int64_t rows,
                                                           float* __restrict__ dl, int64_t ldd,
                                                           float gscale,
                                                           const float* __restrict__ gmul) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= rows) return;
    if (gmul) gscale *= *gmul;
    const int64_t b = r / Tlen, t = r - b * Tlen;
    const int tq = (int)target[b * ldt + t] - 4 * lane;
    floatx4 v = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (tq == e) v[e] = -gscale;
    *reinterpret_cast<floatx4*>(dl + r * ldd + 4 * lane) = v;
}

extern "C" int srnn_nll_bwd(const int64_t* target, int64_t ldt, int Tlen, int64_t rows, int Q,
                            float* dlogp, int64_t ldd, float gscale, const float* gmul,
                            void* stream) {
    if (rows <= 0) return 0;
    if (Q == 256 && ldd % 4 == 0 && (uintptr_t)dlogp % 16 == 0) {
        hipLaunchKernelGGL(nll_bwd_q256_kernel, dim3(cdiv(rows, 4)), dim3(256), 0,
                           (hipStream_t)stream, target, ldt, Tlen, rows, dlogp, ldd, gscale, gmul);
        SRNN_LAUNCH_CHECK();
        return 0;
    }
    hipLaunchKernelGGL(nll_bwd_kernel, dim3(cdiv(rows * Q, 256)), dim3(256), 0,
                       (hipStream_t)stream, target, ldt, Tlen, rows, Q, dlogp, ldd, gscale, gmul);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// ------------------------------------------------------------------ sampler
// One wave per row; lane holds q = 4 * lane + j (16-B loads of logits and noise).  The
// per-row math lives in sampler.hpp, shared with the persistent generation loop.
__global__ __launch_bounds__(256) void sample_kernel(
    const float* __restrict__ z, int64_t ldz, int B, const float* __restrict__ noise,
    uint64_t seed, int row0, const int* __restrict__ base, int off, int L,
    int64_t* __restrict__ seq, int64_t ldseq, float* __restrict__ logp_out) {
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (b >= B) return;
    const int i = *base + off;        // absolute sample index being generated
    const int step = i - L;
    const floatx4 v = *reinterpret_cast<const floatx4*>(z + (int64_t)b * ldz + 4 * lane);
    const floatx4 lq = log_noise(sample_noise(noise, seed, B, b, step, lane, row0));
    const int bi = sample_row(v, lq, logp_out ? logp_out + ((int64_t)step * B + b) * 256 : nullptr,
                              lane);
    if (lane == 0) seq[(int64_t)b * ldseq + i] = bi;
}

int srnn_sample_impl(const float* z, int64_t ldz, int B, const float* noise, uint64_t seed,
                     int row0, const int* base, int off, int L, int64_t* seq, int64_t ldseq,
                     float* logp_out, hipStream_t s) {
    hipLaunchKernelGGL(sample_kernel, dim3(cdiv(B, 4)), dim3(256), 0, s, z, ldz, B, noise, seed,
                       row0, base, off, L, seq, ldseq, logp_out);
    SRNN_LAUNCH_CHECK();
    return 0;
}

