// Autoregressive generation (Generator.__call__, model.py:445-520) on the device.
//
// The reference runs a Python loop per sample: ~10 small kernels + a host<->device
// round trip + a print per tier tick.  Here the whole loop stays on the GPU: the
// sample indices live in a device int64 buffer (never copied back until the end),
// every kernel that depends on the current sample position reads a device-side
// block base `*base` plus a compile-time-constant offset, so one block of 2 top-tier
// periods (2 * lookback samples, every tier ticking an even number of times so the
// GRU state ping-pong returns to buffer 0) is captured once as a hipGraph and
// replayed n_cond / 2 times.  Per sample: L1 gather -> hidden GEMM (relu) -> output
// GEMM -> softmax/sampler; per tier tick: input build -> input GEMM -> GRU cell(s) ->
// upsampling GEMM.
#include <vector>

#include "samplernn_hip_internal.hpp"
#include "ulaw_tables.h"
#include "../../include/samplernn_hip.h"
#include "gen_mlp.hpp"
#include "sampler.hpp"

int srnn_mlp_l1_impl(int dtype, const void* tab, const int64_t* x, int64_t ldx, int xoff,
                     const int* base, int B, int Tlen, int upper_dtype, const void* upper,
                     int64_t ldu, void* out, int64_t ldo, int D, int FS0, int Q, hipStream_t s);
int srnn_sample_impl(const float* z, int64_t ldz, int B, const float* noise, uint64_t seed,
                     int row0,
                     const int* base, int off, int L, int64_t* seq, int64_t ldseq,
                     float* logp_out, hipStream_t s);
int srnn_gru_cell_impl(int dtype, int B, int D, int Din, const void* x, int64_t ldx,
                       const void* wih, const float* bih, const float* gi, int64_t ldgi,
                       const void* h, int64_t ldh, const float* hf, int64_t ldhf, const void* whh,
                       const float* bhh, float* hout, int64_t ldho, void* hout_lp, int64_t ldhl,
                       float* gates, int64_t ldgt, hipStream_t s);
int srnn_gru_cell_x_impl(int dtype, int B, int D, int Din, const void* x, int64_t ldx,
                         const void* wih, const float* bih, const float* gadd, int64_t ldgadd,
                         const float* gh, int64_t ldgh, const float* hf, int64_t ldhf, float* hout,
                         int64_t ldho, void* hout_lp, int64_t ldhl, hipStream_t s);

// Fused tier input (build_input + input projection of one tier tick), one row per block:
//   a[s] = 2*deq(seq[b, i - nfs + s]) (s < nfs) | cond[b, i/L - 1, s - nfs]   (rounded to T,
//          as the GEMM path's T operand)
//   x[b, o] = sum_s a[s] W_in[o, s] + bias[o] + add[b][o]
// add = the top tier's per-row bias (speaker + cond/input biases) or the upper tier's
// upsampled conditioning row (model.py:196-220).  in_dim <= 16 + cond_dim is small, so a
// thread per output with the row's inputs in LDS beats a GEMM launch plus an input kernel.
template <typename T>
__global__ __launch_bounds__(256) void tier_input_kernel(
    const int64_t* __restrict__ seq, int64_t ldseq, const int* __restrict__ base, int off,
    int nfs, const float* __restrict__ lut2, const float* __restrict__ cond, int n_cond, int C,
    int L, const T* __restrict__ w_in, int in_dim, const float* __restrict__ bias,
    const float* __restrict__ add, int64_t ldadd, T* __restrict__ x, int D) {
    extern __shared__ float av[];
    const int b = blockIdx.x;
    const int i = *base + off;
    for (int s = threadIdx.x; s < in_dim; s += blockDim.x) {
        float v;
        if (s < nfs) v = lut2[seq[(int64_t)b * ldseq + i - nfs + s]];
        else v = cond[((int64_t)b * n_cond + (i / L - 1)) * C + (s - nfs)];
        av[s] = to_f(from_f<T>(v));
    }
    __syncthreads();
    for (int o = threadIdx.x; o < D; o += blockDim.x) {
        const T* w = w_in + (int64_t)o * in_dim;
        float acc = 0.f;
        for (int s = 0; s < in_dim; ++s) acc += av[s] * to_f(w[s]);
        if (bias) acc += bias[o];
        acc += add[(int64_t)b * ldadd + o];
        x[(int64_t)b * D + o] = from_f<T>(acc);
    }
}

// Same computation tiled over (TI_RB rows) x (TI_OB outputs): the block stages its W_in
// rows (contiguous, coalesced) and its rows' inputs in LDS as fp32 (odd row stride: the 64
// lanes of a wave read 64 distinct banks), so every thread's loads are in flight at once
// instead of one dependent weight load per multiply-add (the per-row kernel above is
// latency-bound: 6 us at in_dim 16, 23 us at 107).  Each (row, output) still accumulates
// over s in order from 0 with the same fused multiply-adds, then + bias + add: results are
// bit-identical to tier_input_kernel.
// The bottom tick's launch also draws the next persistent sample loop's noise (planes
// blockIdx.z >= 1: log q of steps *base + off + s - L, s < nsteps, one wave per (step, row)),
// which saves that loop a launch of its own.
struct NoiseJob {
    const float* noise;      // (T, B, Q) Exp(1) draws, or null -> Philox(seed)
    uint64_t seed;
    int row0;                // global index of row 0 (Philox counters)
    int nsteps;              // 0: no noise work
    float* lq;               // (nsteps, B, Q)
};

// noise plane z >= 1 of a 256-thread launch: one wave per (step, row)
__device__ __forceinline__ void noise_plane(const NoiseJob& nz, const int* base, int off, int L,
                                            int B) {
    const int idx = (((int)blockIdx.z - 1) * (int)(gridDim.x * gridDim.y) +
                     (int)(blockIdx.y * gridDim.x + blockIdx.x)) * 4 + (int)(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (idx >= nz.nsteps * B) return;
    const int st = idx / B, b = idx - st * B;
    const int i = *base + off + st;
    *reinterpret_cast<floatx4*>(nz.lq + ((int64_t)st * B + b) * 256 + 4 * lane) =
        log_noise(sample_noise(nz.noise, nz.seed, B, b, i - L, lane, nz.row0));
}

constexpr int TI_RB = 8, TI_OB = 64;
template <typename T>
__global__ __launch_bounds__(256) void tier_input_tiled_kernel(
    const int64_t* __restrict__ seq, int64_t ldseq, const int* __restrict__ base, int off,
    int nfs, const float* __restrict__ lut2, const float* __restrict__ cond, int n_cond, int C,
    int L, const T* __restrict__ w_in, int in_dim, const float* __restrict__ bias,
    const float* __restrict__ add, int64_t ldadd, T* __restrict__ x, int B, int D,
    NoiseJob nz) {
    if (blockIdx.z > 0) {
        noise_plane(nz, base, off, L, B);
        return;
    }
    extern __shared__ float tsh[];
    const int S1 = in_dim | 1;
    float* wsh = tsh;                       // [TI_OB][S1]
    float* ash = tsh + TI_OB * S1;          // [TI_RB][S1]
    const int o0 = blockIdx.x * TI_OB, b0 = blockIdx.y * TI_RB;
    const int i = *base + off;
    const int nw = min(TI_OB, D - o0) * in_dim;
    for (int e = threadIdx.x; e < nw; e += 256) {
        const int o = e / in_dim, s = e - o * in_dim;
        wsh[o * S1 + s] = to_f(w_in[(int64_t)o0 * in_dim + e]);
    }
    for (int e = threadIdx.x; e < TI_RB * in_dim; e += 256) {
        const int r = e / in_dim, s = e - r * in_dim;
        const int b = min(b0 + r, B - 1);
        float v;
        if (s < nfs) v = lut2[seq[(int64_t)b * ldseq + i - nfs + s]];
        else v = cond[((int64_t)b * n_cond + (i / L - 1)) * C + (s - nfs)];
        ash[r * S1 + s] = to_f(from_f<T>(v));
    }
    __syncthreads();
    const int o = threadIdx.x & 63, rg = threadIdx.x >> 6;
    if (o0 + o >= D) return;
    constexpr int RPT = TI_RB / 4;
    float acc[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) acc[j] = 0.f;
    const float* wr = wsh + o * S1;
    for (int s = 0; s < in_dim; ++s) {
        const float w = wr[s];
#pragma unroll
        for (int j = 0; j < RPT; ++j) acc[j] += ash[(rg + 4 * j) * S1 + s] * w;
    }
    const float bo = bias ? bias[o0 + o] : 0.f;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
        const int b = b0 + rg + 4 * j;
        if (b >= B) break;
        float v = acc[j];
        if (bias) v += bo;
        v += add[(int64_t)b * ldadd + o0 + o];
        x[(int64_t)b * D + o0 + o] = from_f<T>(v);
    }
}

// ---- folded bottom tick (bf16, one GRU layer) ----------------------------------------
// The bottom tier's tick is x = W_in a + b_in + up_upper[fi]; gi = W_ih x + b_ih; GRU;
// up = W_up h + b_up (model.py:196-244).  With x linear in its three terms it folds to
//     gi = Min a + G[fi],  Min = W_ih W_in (3D x nfs),
//     G[fi] = W_ih up_upper[fi] + W_ih b_in + b_ih = Wfold[fi] h_upper + bfold[fi],
//     Wfold[fi] = W_ih W_up_upper[fi] (3D x D),  bfold[fi] = W_ih (b_up_upper[fi] + b_in) + b_ih
// so the upper tier's tick produces G for all its FS_upper positions with ONE skinny GEMM
// over its h (weights (FS_upper 3D, D), folded once per call) in place of its upsampling
// GEMM, and Min a is 16 multiply-adds per gate.  gh = W_hh h + b_hh of the NEXT tick only
// needs this tick's h, so it rides in this tick's upsampling GEMM (weights [W_up; W_hh]:
// the h operand is streamed once for both).  What stays between the sample loop launches
// is a gate-update kernel and one GEMM, instead of input kernel + GRU-cell GEMM + GEMM.
// Rounding differs from the unfolded bf16 path (x and up_upper are never rounded to bf16;
// the folded weights are), at the same bf16 scale; fp32 models keep the unfolded tick.

// Min[g][s] (row-padded to 16) = sum_o W_ih[g, o] W_in[o, s], and the folded upper-tick bias
// bfold[j][g] = sum_o W_ih[g, o] (b_in[o] + b_up1[j D + o]) + b_ih[g], j < fs1: one wave per
// gate row, once per generate call
constexpr int FOLD_MAX_FS1 = 8;
template <typename T>
__global__ __launch_bounds__(256) void fold_input_kernel(const T* __restrict__ wih,
                                                         const T* __restrict__ win, int nfs,
                                                         const float* __restrict__ bin,
                                                         const float* __restrict__ bih,
                                                         const float* __restrict__ bup1, int fs1,
                                                         float* __restrict__ Min,
                                                         float* __restrict__ bfold, int G3, int D) {
    const int g = blockIdx.x * 4 + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (g >= G3) return;
    constexpr int NA = 17 + FOLD_MAX_FS1;
    float acc[NA];
#pragma unroll
    for (int s = 0; s < NA; ++s) acc[s] = 0.f;
    for (int o = lane; o < D; o += 64) {
        const float w = to_f(wih[(int64_t)g * D + o]);
#pragma unroll
        for (int s = 0; s < 16; ++s)
            if (s < nfs) acc[s] += w * to_f(win[(int64_t)o * nfs + s]);
        if (bin) acc[16] += w * bin[o];
#pragma unroll
        for (int j = 0; j < FOLD_MAX_FS1; ++j)
            if (j < fs1 && bup1) acc[17 + j] += w * bup1[(int64_t)j * D + o];
    }
#pragma unroll
    for (int s = 0; s < NA; ++s) acc[s] = wave_sum(acc[s]);
    if (lane == 0) {
#pragma unroll
        for (int s = 0; s < 16; ++s) Min[(int64_t)g * 16 + s] = acc[s];
        const float c0 = acc[16] + (bih ? bih[g] : 0.f);
#pragma unroll
        for (int j = 0; j < FOLD_MAX_FS1; ++j)
            if (j < fs1) bfold[(int64_t)j * G3 + g] = c0 + acc[17 + j];
    }
}

// gate update of the folded bottom tick: block = FG_RB rows x 256 units (+ noise planes)
constexpr int FG_RB = 2;
template <typename T>
__global__ __launch_bounds__(256) void fold_gru_kernel(
    const int64_t* __restrict__ seq, int64_t ldseq, const int* __restrict__ base, int off,
    int nfs, const float* __restrict__ lut2, int L, const float* __restrict__ Min,
    const float* __restrict__ G, int64_t ldg, const float* __restrict__ gh, int64_t ldgh,
    const float* __restrict__ hp, float* __restrict__ hn, T* __restrict__ hn_lp, int B, int D,
    NoiseJob nz) {
    if (blockIdx.z > 0) {
        noise_plane(nz, base, off, L, B);
        return;
    }
    __shared__ float ash[FG_RB][16];
    const int u = blockIdx.x * 256 + (int)threadIdx.x, b0 = blockIdx.y * FG_RB;
    // every operand that does not depend on the samples is loaded first, so its latency
    // overlaps the seq -> LUT chain below (clamped addresses, no branches)
    const int uc = min(u, D - 1);
    floatx4 mr[4], mz[4], mn[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        mr[j] = *reinterpret_cast<const floatx4*>(Min + (int64_t)uc * 16 + 4 * j);
        mz[j] = *reinterpret_cast<const floatx4*>(Min + (int64_t)(D + uc) * 16 + 4 * j);
        mn[j] = *reinterpret_cast<const floatx4*>(Min + (int64_t)(2 * D + uc) * 16 + 4 * j);
    }
    float gv[FG_RB][6], hv[FG_RB];
#pragma unroll
    for (int r = 0; r < FG_RB; ++r) {
        const int b = min(b0 + r, B - 1);
        const float* gr = G + (int64_t)b * ldg;
        const float* hr = gh + (int64_t)b * ldgh;
        gv[r][0] = gr[uc]; gv[r][1] = gr[D + uc]; gv[r][2] = gr[2 * D + uc];
        gv[r][3] = hr[uc]; gv[r][4] = hr[D + uc]; gv[r][5] = hr[2 * D + uc];
        hv[r] = hp[(int64_t)b * D + uc];
    }
    if (threadIdx.x < FG_RB * 16) {
        const int r = threadIdx.x >> 4, s = threadIdx.x & 15;
        const int b = min(b0 + r, B - 1);
        const int i = *base + off;
        // a[s] = 2 deq(seq[b, i - nfs + s]) rounded to T, as the unfolded input's operand
        ash[r][s] = s < nfs ? to_f(from_f<T>(lut2[seq[(int64_t)b * ldseq + i - nfs + s]])) : 0.f;
    }
    __syncthreads();
    if (u >= D) return;
#pragma unroll
    for (int r = 0; r < FG_RB; ++r) {
        const int b = b0 + r;
        if (b >= B) break;
        float gir = gv[r][0], giz = gv[r][1], gin = gv[r][2];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float a = ash[r][4 * j + e];
                gir += a * mr[j][e];
                giz += a * mz[j][e];
                gin += a * mn[j][e];
            }
        const float ghr = gv[r][3], ghz = gv[r][4], ghn = gv[r][5];
        const float rg = 1.0f / (1.0f + expf(-(ghr + gir)));
        const float zg = 1.0f / (1.0f + expf(-(ghz + giz)));
        const float ng = tanhf(gin + ghn * rg);
        const float v = (hv[r] - ng) * zg + ng;
        hn[(int64_t)b * D + u] = v;
        hn_lp[(int64_t)b * D + u] = from_f<T>(v);
    }
}

// Input row of the folded top tick: a[b][s] = 2 deq(seq[b, i - nfs + s]) (s < nfs) |
// cond[b, i/L - 1, s - nfs] (s < in_dim) | 0 (s < AP), rounded to T as the unfolded input's
// GEMM operand; gi = a . Min1^T + P1[b] then replaces x = W_in a + row_bias, gi = W_ih x + b_ih
// (Min1 = W_ih W_in, P1 = W_ih row_bias + b_ih, folded once per call).  Two rows per block;
// planes blockIdx.z >= 1 draw the noise of the persistent launches of the tick's period.
constexpr int TA_AP = 128;
template <typename T>
__global__ __launch_bounds__(256) void tier_a_kernel(
    const int64_t* __restrict__ seq, int64_t ldseq, const int* __restrict__ base, int off,
    int nfs, const float* __restrict__ lut2, const float* __restrict__ cond, int n_cond, int C,
    int L, int in_dim, T* __restrict__ a, int B, NoiseJob nz) {
    if (blockIdx.z > 0) {
        noise_plane(nz, base, off, L, B);
        return;
    }
    const int b = blockIdx.x * 2 + (int)(threadIdx.x >> 7), s = threadIdx.x & 127;
    if (b >= B) return;
    const int i = *base + off;
    float v = 0.f;
    if (s < nfs) v = lut2[seq[(int64_t)b * ldseq + i - nfs + s]];
    else if (s < in_dim) v = cond[((int64_t)b * n_cond + (i / L - 1)) * C + (s - nfs)];
    a[(int64_t)b * TA_AP + s] = from_f<T>(v);
}

template <typename T>
__global__ void init_state_kernel(const float* __restrict__ h0, float* __restrict__ h,
                                  T* __restrict__ hlp, int B, int D) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= B * D) return;
    const float v = h0[e % D];
    h[e] = v;
    if (hlp) hlp[e] = from_f<T>(v);
}

__global__ void advance_kernel(int* base, int by) { *base += by; }

template <typename T>
__global__ void copy_cast_kernel(const float* __restrict__ src, T* __restrict__ dst, int n) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n) dst[e] = from_f<T>(src[e]);
}

namespace {

constexpr size_t ALIGN = 256;
inline size_t al(size_t x) { return (x + ALIGN - 1) / ALIGN * ALIGN; }

struct Bufs {
    void* x[SRNN_MAX_TIERS];
    float* h[SRNN_MAX_TIERS][SRNN_MAX_RNN][2];
    void* hlp[SRNN_MAX_TIERS][SRNN_MAX_RNN][2];
    float* up[SRNN_MAX_TIERS];
    void* a1;
    void* a2;
    float* logits;
    float* lut2;
    int* base;
    // persistent sample loop (gen_mlp.hip): hand-off granules + error word, one zeroed block
    unsigned long long* xa1;
    unsigned long long* xa2;
    void* wfr_hid;                   // fragment-order weight images (gen_mlp_prep_weights)
    void* wfr_out;
    unsigned long long* xz;
    int* gerr;
    float* lq;               // (lq_steps, B, Q) log q of the persistent launches' draws
    int lq_steps;            // FS0, or the upper tier's period FS0 FS1 when that tick draws
    size_t gm_bytes;
    // folded bottom tick (fold_ok): up[0] rows are [up (FS0 D) | gh of the next tick (3D)]
    bool fold;
    int64_t ldup0;           // row stride of up[0]
    void* wcat;              // (FS0 D + 3D, D) [W_up; W_hh] of the bottom tier
    float* bcat;             // [b_up; b_hh]
    float* fmin;             // (3D, 16) W_ih W_in, rows zero-padded
    void* wfold;             // (FS1 3D + 3D, D) [W_ih0 W_up1[j], j < FS1; W_hh1]
    float* bfold;            // (FS1 3D + 3D) [bfold[j]; b_hh1]
    GenMlpArgs::Tick* ticks; // [fi][cur]: the persistent loop's gate-update operands
    // folded top tick (fold_top: two tiers, the upper one is the top)
    bool fold_top;
    void* min1;              // (3D, TA_AP) W_ih1 W_in1, zero columns past in_dim
    float* p1;               // (B, 3D) W_ih1 row_bias + b_ih1
    void* atop;              // (B, TA_AP) the top tick's input row
    float* fg;               // (B, ldg1): [G of the current upper frame | gh1 of the next
    int64_t ldg1;            //  upper tick], ldg1 = FS1 3D + 3D
};

// fp32 too (SRNN_GEN_FOLD_F32=0: unfolded fp32 ticks): the folds reassociate fp32 sums
// (W_ih (W_in a + b) -> (W_ih W_in) a + W_ih b), same precision, rounding in the last bits
bool fold_ok(const SrnnModel* m) {
    const SrnnTier& t = m->tier[0];
    return (m->dtype == SRNN_BF16 || (env_flag("SRNN_GEN_FOLD_F32", 1) && m->dim % 64 == 0)) &&
           m->n_tiers >= 2 &&
           m->n_rnn == 1 &&
           t.in_dim == t.n_frame_samples && t.n_frame_samples <= 16 && t.b_up &&
           m->tier[1].frame_size <= FOLD_MAX_FS1 &&
           env_flag("SRNN_GEN_FOLD", 1);
}

// carve (or size, if ws == nullptr) the workspace
size_t carve(const SrnnModel* m, int B, char* ws, Bufs* b, const GenMlpPlan* pl) {
    const int D = m->dim, Q = m->q_levels;
    const size_t es = m->dtype == SRNN_F32 ? 4 : 2;
    const bool lp = m->dtype != SRNN_F32;
    size_t off = 0;
    auto take = [&](size_t bytes) -> char* {
        char* p = ws ? ws + off : nullptr;
        off += al(bytes);
        return p;
    };
    for (int k = 0; k < m->n_tiers; ++k) {
        const SrnnTier& t = m->tier[k];
        b->x[k] = take((size_t)B * D * es);
        for (int l = 0; l < m->n_rnn; ++l)
            for (int p = 0; p < 2; ++p) {
                b->h[k][l][p] = (float*)take((size_t)B * D * 4);
                b->hlp[k][l][p] = lp ? (void*)take((size_t)B * D * es) : (void*)b->h[k][l][p];
            }
        b->up[k] = (float*)take((size_t)B * (t.frame_size + 3) * D * 4);
    }
    b->fold = fold_ok(m);
    b->ldup0 = (int64_t)m->tier[0].frame_size * D + (b->fold ? 3 * D : 0);
    b->wcat = nullptr;
    b->wfold = nullptr;
    b->ticks = nullptr;
    b->fold_top = false;
    b->min1 = b->atop = nullptr;
    b->p1 = nullptr;
    b->ldg1 = 0;
    b->bcat = b->fmin = b->bfold = b->fg = nullptr;
    if (b->fold) {
        const int N0 = m->tier[0].frame_size * D + 3 * D;
        b->wcat = take((size_t)N0 * D * es);
        b->bcat = (float*)take((size_t)N0 * 4);
        b->fmin = (float*)take((size_t)3 * D * 16 * 4);
        const int F1 = m->tier[1].frame_size;
        b->ldg1 = (int64_t)(F1 + 1) * 3 * D;
        b->wfold = take((size_t)b->ldg1 * D * es);
        b->bfold = (float*)take((size_t)b->ldg1 * 4);
        b->fg = (float*)take((size_t)B * b->ldg1 * 4);
        b->ticks = (GenMlpArgs::Tick*)take((size_t)2 * F1 * sizeof(GenMlpArgs::Tick));
        b->fold_top = m->n_tiers == 2 && m->tier[1].in_dim <= TA_AP &&
                      env_flag("SRNN_GEN_FOLD_TOP", 1);
        if (b->fold_top) {
            b->min1 = take((size_t)3 * D * TA_AP * es);
            b->p1 = (float*)take((size_t)B * 3 * D * 4);
            b->atop = take((size_t)B * TA_AP * es);
        }
    }
    b->a1 = take((size_t)B * D * es);
    b->a2 = take((size_t)B * D * es);
    b->logits = (float*)take((size_t)B * Q * 4);
    b->lut2 = (float*)take((size_t)Q * 4);
    b->base = (int*)take(64);
    b->xa1 = b->xa2 = b->xz = nullptr;
    b->wfr_hid = b->wfr_out = nullptr;
    b->gerr = nullptr;
    b->lq = nullptr;
    b->lq_steps = 0;
    b->gm_bytes = 0;
    if (pl && pl->ok) {
        const size_t start = off;
        b->gerr = (int*)take(8192);          // [0] error word, [64..) 2 keyed census arrays
        b->xa1 = (unsigned long long*)take(pl->xa_words * 8);
        b->xa2 = (unsigned long long*)take(pl->xa_words * 8);
        b->xz = (unsigned long long*)take(pl->xz_words * 8);
        b->wfr_hid = pl->wfr_hid_bytes ? take(pl->wfr_hid_bytes) : nullptr;
        b->wfr_out = pl->wfr_out_bytes ? take(pl->wfr_out_bytes) : nullptr;
        b->lq_steps = m->tier[0].frame_size * (b->fold ? m->tier[1].frame_size : 1);
        b->lq = (float*)take((size_t)b->lq_steps * B * Q * 4);
        b->gm_bytes = off - start;
    }
    return off;
}

struct Ctx {
    const SrnnModel* m;
    Bufs b;
    int B, n_cond, L;
    const float* cond;
    const float* row_bias;
    const float* noise;
    uint64_t seed;
    int row0 = 0;             // global index of row 0 (rank-sharded generation)
    int64_t* seq;
    int64_t ldseq;
    float* logp;
    hipStream_t s;
    const GenMlpPlan* pl;     // persistent sample loop, or null for per-sample kernels
    // lq holds the draws of block-relative steps [noise_beg, noise_end): drawn ahead by the
    // input launch of the bottom tick (FS0 steps) or, with the folded bottom tick, of the
    // upper tier's tick (its whole period)
    int noise_beg = 0, noise_end = -1;
    bool gate_done = false;   // the last persistent launch did the next bottom tick's gates
    // the folded bottom tick's GEMM runs inside the persistent launch that follows it
    // (GenMlpArgs::tg): set by tier_tick, consumed by that launch
    bool tick_gemm = false;
    GenMlpArgs::TickGemm pending{};
};

#define RET(x) do { int _r = (x); if (_r) return _r; } while (0)

// one tier tick at block-relative offset `off`; `par` = tick parity of this tier
int tier_tick(Ctx& c, int k, int off, int par) {
    const SrnnModel* m = c.m;
    const SrnnTier& t = m->tier[k];
    const int D = m->dim, B = c.B, dt = m->dtype;
    const bool top = (k == m->n_tiers - 1);
    const bool lp = dt != SRNN_F32;
    const int cur = par, nxt = par ^ 1;
    if (k == 0 && c.b.fold) {
        // folded bottom tick: gate update (gi = Min a + G[fi], gh from the last tick's GEMM),
        // then [up | gh'] = h [W_up; W_hh]^T + [b_up; b_hh]
        const SrnnTier& u = m->tier[1];
        const int fi = (off / t.n_frame_samples) % u.frame_size;
        const NoiseJob nz{c.noise, c.seed, c.row0, 0, nullptr};    // (the upper tick drew them)
        const dim3 g2(cdiv(D, 256), cdiv(B, FG_RB));
        const int planes = 1;
        const int64_t fs0d = (int64_t)t.frame_size * D;
        // [up | gh'] = h [W_up; W_hh]^T + [b_up; b_hh]: its own launch, or inside the
        // persistent launch that follows (c.tick_gemm)
        auto tick_gemm = [&]() -> int {
            if (c.tick_gemm) {
                SRNN_REQUIRE(c.pending.N == 0, "generate: tick GEMM left unconsumed");
                c.pending.A = c.b.hlp[0][0][nxt];
                c.pending.W = c.b.wcat;
                c.pending.bias = c.b.bcat;
                c.pending.C = c.b.up[0];
                c.pending.ldc = c.b.ldup0;
                c.pending.N = (int)(fs0d + 3 * D);
                c.pending.K = D;
                return 0;
            }
            return linear_fwd(dt, SRNN_F32, B, (int)(fs0d + 3 * D), D, c.b.hlp[0][0][nxt], D,
                              c.b.wcat, D, c.b.bcat, c.b.up[0], c.b.ldup0, 0, c.s);
        };
        if (c.gate_done) {
            // the gate update ran at the end of the last persistent launch (GenMlpArgs::tk)
            c.gate_done = false;
            return tick_gemm();
        }
        if (dt == SRNN_F32)
            hipLaunchKernelGGL((fold_gru_kernel<float>), dim3(g2.x, g2.y, planes), dim3(256), 0,
                               c.s, c.seq, c.ldseq, c.b.base, off, t.n_frame_samples, c.b.lut2,
                               c.L, c.b.fmin, c.b.fg + (size_t)fi * 3 * D, c.b.ldg1,
                               c.b.up[0] + fs0d, c.b.ldup0, c.b.h[0][0][cur], c.b.h[0][0][nxt],
                               (float*)c.b.hlp[0][0][nxt], B, D, nz);
        else
            hipLaunchKernelGGL((fold_gru_kernel<bf16>), dim3(g2.x, g2.y, planes), dim3(256), 0,
                               c.s, c.seq, c.ldseq, c.b.base, off, t.n_frame_samples, c.b.lut2,
                               c.L, c.b.fmin, c.b.fg + (size_t)fi * 3 * D, c.b.ldg1,
                               c.b.up[0] + fs0d, c.b.ldup0, c.b.h[0][0][cur], c.b.h[0][0][nxt],
                               (bf16*)c.b.hlp[0][0][nxt], B, D, nz);
        SRNN_LAUNCH_CHECK();
        return tick_gemm();
    }
    if (k == 1 && c.b.fold_top) {
        // folded top tick: a (+ the period's noise) -> gi = a Min1^T + P1, gh1 carried ->
        // [G | gh1'] = h [Wfold; W_hh1]^T + [bfold; b_hh1]
        NoiseJob nz{c.noise, c.seed, c.row0, 0, nullptr};
        const int gx = cdiv(B, 2);
        int planes = 1;
        if (c.pl && c.b.lq && env_flag("SRNN_GEN_NOISE_AHEAD", 1)) {
            nz.nsteps = c.b.lq_steps;
            nz.lq = c.b.lq;
            planes = 1 + cdiv(cdiv((int64_t)nz.nsteps * B, 4), gx);
            c.noise_beg = off;
            c.noise_end = off + nz.nsteps;
        }
        if (dt == SRNN_F32)
            hipLaunchKernelGGL((tier_a_kernel<float>), dim3(gx, 1, planes), dim3(256), 0, c.s,
                               c.seq, c.ldseq, c.b.base, off, t.n_frame_samples, c.b.lut2, c.cond,
                               c.n_cond, m->cond_dim, c.L, t.in_dim, (float*)c.b.atop, B, nz);
        else
            hipLaunchKernelGGL((tier_a_kernel<bf16>), dim3(gx, 1, planes), dim3(256), 0, c.s,
                               c.seq, c.ldseq, c.b.base, off, t.n_frame_samples, c.b.lut2, c.cond,
                               c.n_cond, m->cond_dim, c.L, t.in_dim, (bf16*)c.b.atop, B, nz);
        SRNN_LAUNCH_CHECK();
        const int64_t g0 = (int64_t)t.frame_size * 3 * D;
        RET(srnn_gru_cell_x_impl(dt, B, D, TA_AP, c.b.atop, TA_AP, c.b.min1, nullptr, c.b.p1,
                                 3 * D, c.b.fg + g0, c.b.ldg1, c.b.h[k][0][cur], D,
                                 c.b.h[k][0][nxt], D, c.b.hlp[k][0][nxt], D, c.s));
        return linear_fwd(dt, SRNN_F32, B, (int)c.b.ldg1, D, c.b.hlp[k][0][nxt], D, c.b.wfold,
                          D, c.b.bfold, c.b.fg, c.b.ldg1, 0, c.s);
    }
    // 1. x = A_in . W_in^T + (top: row_bias ; lower: b_in + upper-tier conditioning row)
    {
        const float* add;
        int64_t ldadd;
        const float* bias;
        if (top) {
            add = c.row_bias; ldadd = D; bias = nullptr;
        } else {
            const SrnnTier& u = m->tier[k + 1];
            // frame_index = (i // nfs_k) % FS_{k+1}  (model.py:491-492); base is a multiple of L
            const int fi = (off / t.n_frame_samples) % u.frame_size;
            add = c.b.up[k + 1] + (size_t)fi * D; ldadd = (int64_t)u.frame_size * D;
            bias = t.b_in;
        }
        const size_t tlds = (size_t)(TI_OB + TI_RB) * (t.in_dim | 1) * sizeof(float);
        if (tlds <= 160 * 1024) {
            // (attribute raised once, to the whole LDS, before the first launch that needs it)
            static bool attr[2] = {false, false};
            const int ai = dt == SRNN_F32 ? 0 : 1;
            if (tlds > 65536 && !attr[ai]) {
                SRNN_CHECK_HIP(hipFuncSetAttribute(
                    dt == SRNN_F32 ? (const void*)tier_input_tiled_kernel<float>
                                   : (const void*)tier_input_tiled_kernel<bf16>,
                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
                attr[ai] = true;
            }
            NoiseJob nz{c.noise, c.seed, c.row0, 0, nullptr};
            int planes = 1;
            if (k == (c.b.fold ? 1 : 0) && c.pl && c.b.lq && env_flag("SRNN_GEN_NOISE_AHEAD", 1)) {
                nz.nsteps = c.b.lq_steps;             // the persistent launches after this tick
                nz.lq = c.b.lq;
                const int per = cdiv(D, TI_OB) * cdiv(B, TI_RB);
                planes = 1 + cdiv(cdiv((int64_t)nz.nsteps * B, 4), per);
                c.noise_beg = off;
                c.noise_end = off + nz.nsteps;
            }
            const dim3 grid(cdiv(D, TI_OB), cdiv(B, TI_RB), planes);
            if (dt == SRNN_F32)
                hipLaunchKernelGGL((tier_input_tiled_kernel<float>), grid, dim3(256), tlds, c.s,
                                   c.seq, c.ldseq, c.b.base, off, t.n_frame_samples, c.b.lut2,
                                   c.cond, c.n_cond, m->cond_dim, c.L, (const float*)t.w_in,
                                   t.in_dim, bias, add, ldadd, (float*)c.b.x[k], B, D, nz);
            else
                hipLaunchKernelGGL((tier_input_tiled_kernel<bf16>), grid, dim3(256), tlds, c.s,
                                   c.seq, c.ldseq, c.b.base, off, t.n_frame_samples, c.b.lut2,
                                   c.cond, c.n_cond, m->cond_dim, c.L, (const bf16*)t.w_in,
                                   t.in_dim, bias, add, ldadd, (bf16*)c.b.x[k], B, D, nz);
        } else {
            const size_t lds = (size_t)t.in_dim * sizeof(float);
            if (dt == SRNN_F32)
                hipLaunchKernelGGL((tier_input_kernel<float>), dim3(B), dim3(256), lds, c.s,
                                   c.seq, c.ldseq, c.b.base, off, t.n_frame_samples, c.b.lut2,
                                   c.cond, c.n_cond, m->cond_dim, c.L, (const float*)t.w_in,
                                   t.in_dim, bias, add, ldadd, (float*)c.b.x[k], D);
            else
                hipLaunchKernelGGL((tier_input_kernel<bf16>), dim3(B), dim3(256), lds, c.s,
                                   c.seq, c.ldseq, c.b.base, off, t.n_frame_samples, c.b.lut2,
                                   c.cond, c.n_cond, m->cond_dim, c.L, (const bf16*)t.w_in,
                                   t.in_dim, bias, add, ldadd, (bf16*)c.b.x[k], D);
        }
        SRNN_LAUNCH_CHECK();
    }
    // 3. GRU layers
    if (k == 1 && c.b.fold) {
        // folded upper tick: gh carried by its last GEMM ([Wfold; W_hh1] . h)
        const int64_t g0 = (int64_t)t.frame_size * 3 * D;
        RET(srnn_gru_cell_x_impl(dt, B, D, D, c.b.x[k], D, t.w_ih[0], t.b_ih[0], nullptr, 0,
                                 c.b.fg + g0, c.b.ldg1, c.b.h[k][0][cur], D, c.b.h[k][0][nxt], D,
                                 c.b.hlp[k][0][nxt], D, c.s));
        // G = h . Wfold^T + bfold and the next tick's gh1, (B, ldg1) fp32
        return linear_fwd(dt, SRNN_F32, B, (int)c.b.ldg1, D, c.b.hlp[k][0][nxt], D, c.b.wfold,
                          D, c.b.bfold, c.b.fg, c.b.ldg1, 0, c.s);
    }
    for (int l = 0; l < m->n_rnn; ++l) {
        const void* xin = l == 0 ? c.b.x[k] : c.b.hlp[k][l - 1][nxt];
        RET(srnn_gru_cell_impl(dt, B, D, D, xin, D, t.w_ih[l], t.b_ih[l], nullptr, 0,
                               c.b.hlp[k][l][cur], D, c.b.h[k][l][cur], D, t.w_hh[l], t.b_hh[l],
                               c.b.h[k][l][nxt], D, lp ? c.b.hlp[k][l][nxt] : nullptr, D, nullptr,
                               0, c.s));
    }
    // 4. LearnedUpsampling1d: up = h . W_up^T + b_up   (B, fs*D) fp32
    RET(linear_fwd(dt, SRNN_F32, B, t.frame_size * D, D, c.b.hlp[k][m->n_rnn - 1][nxt], D, t.w_up,
                   D, t.b_up, c.b.up[k], (int64_t)t.frame_size * D, 0, c.s));
    return 0;
}

int mlp_step(Ctx& c, int off) {
    const SrnnModel* m = c.m;
    const int D = m->dim, Q = m->q_levels, B = c.B, dt = m->dtype;
    const int FS0 = m->tier[0].frame_size;
    RET(srnn_mlp_l1_impl(dt, m->tab, c.seq, c.ldseq, off - FS0, c.b.base, B, 1, SRNN_F32,
                         c.b.up[0] + (size_t)(off % FS0) * D, c.b.ldup0, c.b.a1, D, D, FS0,
                         Q, c.s));
    RET(linear_fwd(dt, dt, B, D, D, c.b.a1, D, m->w_hid, D, m->b_hid, c.b.a2, D, 1, c.s));
    RET(linear_fwd(dt, SRNN_F32, B, Q, D, c.b.a2, D, m->w_out, D, m->b_out, c.b.logits, Q, 0,
                   c.s));
    RET(srnn_sample_impl(c.b.logits, Q, B, c.noise, c.seed, c.row0, c.b.base, off, c.L, c.seq, c.ldseq,
                         c.logp, c.s));
    return 0;
}

// `periods` consecutive top-tier periods starting at sample *base; tick parity restarts
// at 0 (callers only chain blocks with an even tick count per tier)
int run_block(Ctx& c, int periods) {
    const SrnnModel* m = c.m;
    int ticks[SRNN_MAX_TIERS] = {0};
    c.noise_end = -1;
    c.gate_done = false;
    for (int off = 0; off < periods * c.L; ++off) {
        for (int k = m->n_tiers - 1; k >= 0; --k) {
            if (off % m->tier[k].n_frame_samples != 0) continue;
            RET(tier_tick(c, k, off, ticks[k] & 1));
            ticks[k]++;
        }
        if (!c.pl) {
            RET(mlp_step(c, off));
        } else if (off % m->tier[0].frame_size == 0) {
            // the FS0 samples up to the next bottom-tier tick in one persistent launch
            GenMlpArgs a;
            memset(&a, 0, sizeof(a));
            a.tab = m->tab; a.w_hid = m->w_hid; a.b_hid = m->b_hid;
            a.w_out = m->w_out; a.b_out = m->b_out;
            a.wfr_hid = c.b.wfr_hid; a.wfr_out = c.b.wfr_out;
            a.up0 = c.b.up[0]; a.ldup = c.b.ldup0;
            a.noise = c.noise; a.seed = c.seed; a.row0 = c.row0;
            a.seq = c.seq; a.ldseq = c.ldseq; a.logp = c.logp;
            a.base = c.b.base; a.off = off; a.nsteps = m->tier[0].frame_size; a.L = c.L;
            a.B = c.B; a.D = m->dim; a.FS0 = m->tier[0].frame_size;
            a.xa1 = c.b.xa1; a.xa2 = c.b.xa2; a.xz = c.b.xz; a.err = c.b.gerr;
            a.census = c.b.gerr + 64;
            if (c.b.lq && env_flag("SRNN_GEN_NOISE_AHEAD", 1)) {
                // drawn ahead by a tick's input launch, else by a launch here
                if (off < c.noise_beg || off + a.nsteps > c.noise_end) {
                    RET(gen_noise_launch(c.noise, c.seed, c.row0, c.b.base, off, a.nsteps, c.L, c.B,
                                         c.b.lq, c.s));
                    c.noise_beg = off;
                    c.noise_end = off + a.nsteps;
                }
                a.lq = c.b.lq + (size_t)(off - c.noise_beg) * c.B * m->q_levels;
            }
            // the next bottom tick's gate update rides at the end of this launch unless an
            // upper tick (new G) comes first
            const int nx = off + m->tier[0].frame_size;
            if (c.b.fold && nx < periods * c.L && nx % m->tier[1].n_frame_samples != 0 &&
                env_flag("SRNN_GEN_FUSE_GATES", 1)) {
                const int fi = (nx / m->tier[0].n_frame_samples) % m->tier[1].frame_size;
                a.tk = c.b.ticks + 2 * fi + (ticks[0] & 1);    // that tick's G row, cur / nxt
                c.gate_done = true;
            }
            if (c.pending.N) {        // this bottom tick's GEMM, in the launch
                a.tg = c.pending;
                c.pending = GenMlpArgs::TickGemm{};
            }
            RET(gen_mlp_launch(c.pl, a, c.s));
        }
    }
    hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(1), 0, c.s, c.b.base, periods * c.L);
    SRNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace

// persistent sample loop plan for this model/batch (ok = 0: per-sample kernels)
static void plan_for(const SrnnModel* m, int n_seqs, GenMlpPlan* pl) {
    if (!gen_mlp_plan(m->dtype, n_seqs, m->dim, m->tier[0].frame_size, m->q_levels, pl) ||
        !env_flag("SRNN_GEN_PERSIST", 1))
        pl->ok = 0;
}

extern "C" int srnn_gen_persistent_rows(int dtype, int n_seqs, int dim, int fs0, int q_levels) {
    GenMlpPlan pl;
    if (!gen_mlp_plan(dtype, n_seqs, dim, fs0, q_levels, &pl) || !env_flag("SRNN_GEN_PERSIST", 1))
        return 0;
    return pl.R;
}

extern "C" int srnn_gen_workspace_size(const SrnnModel* m, int n_seqs, size_t* bytes) {
    SRNN_REQUIRE(m && bytes && n_seqs > 0, "gen_workspace_size: bad args");
    Bufs b;
    GenMlpPlan pl;
    plan_for(m, n_seqs, &pl);
    *bytes = carve(m, n_seqs, nullptr, &b, &pl);
    return 0;
}

extern "C" int srnn_generate2(const SrnnModel* m, int n_seqs, int n_cond, const float* cond,
                              const float* row_bias, const float* noise, uint64_t seed,
                              int row0, int64_t* seq, float* logp, void* workspace,
                              size_t workspace_bytes, int flags, void* stream);

extern "C" int srnn_generate(const SrnnModel* m, int n_seqs, int n_cond, const float* cond,
                             const float* row_bias, const float* noise, uint64_t seed,
                             int64_t* seq, float* logp, void* workspace, size_t workspace_bytes,
                             int flags, void* stream) {
    return srnn_generate2(m, n_seqs, n_cond, cond, row_bias, noise, seed, 0, seq, logp,
                          workspace, workspace_bytes, flags, stream);
}

extern "C" int srnn_generate2(const SrnnModel* m, int n_seqs, int n_cond, const float* cond,
                              const float* row_bias, const float* noise, uint64_t seed,
                              int row0, int64_t* seq, float* logp, void* workspace,
                              size_t workspace_bytes, int flags, void* stream) {
    SRNN_REQUIRE(row0 >= 0, "generate: negative row offset");
    SRNN_REQUIRE(m && n_seqs > 0 && n_cond > 0 && seq && workspace, "generate: bad args");
    SRNN_REQUIRE(m->n_tiers >= 1 && m->n_tiers <= SRNN_MAX_TIERS, "generate: n_tiers");
    SRNN_REQUIRE(m->n_rnn >= 1 && m->n_rnn <= SRNN_MAX_RNN, "generate: n_rnn");
    SRNN_REQUIRE(m->q_levels == 256, "generate: q_levels must be 256");
    SRNN_REQUIRE(m->dim % 16 == 0, "generate: dim must be a multiple of 16");
    Ctx c;
    c.m = m;
    GenMlpPlan pl;
    plan_for(m, n_seqs, &pl);
    if (flags & 2) pl.ok = 0;          // caller asked for the per-sample kernel path
    size_t need = carve(m, n_seqs, (char*)workspace, &c.b, &pl);
    SRNN_REQUIRE(workspace_bytes >= need, "generate: workspace %zu < %zu", workspace_bytes, need);
    c.B = n_seqs;
    c.n_cond = n_cond;
    c.L = m->tier[m->n_tiers - 1].n_frame_samples;
    c.cond = cond;
    c.row_bias = row_bias;
    c.noise = noise;
    c.seed = seed;
    c.row0 = row0;
    c.seq = seq;
    c.ldseq = (int64_t)c.L * (n_cond + 1);
    c.logp = logp;
    c.pl = pl.ok ? &pl : nullptr;
    c.tick_gemm = c.pl && c.b.fold &&
                  gen_mlp_tick_gemm_ok(&pl, (m->tier[0].frame_size + 3) * m->dim, m->dim, n_seqs);
    hipStream_t user = (hipStream_t)stream;
    const int D = m->dim, B = n_seqs;
    // private stream so a hipGraph can be captured regardless of the caller's stream
    hipStream_t s;
    SRNN_CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    SRNN_CHECK_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    SRNN_CHECK_HIP(hipEventRecord(ev, user));
    SRNN_CHECK_HIP(hipStreamWaitEvent(s, ev, 0));
    c.s = s;
    int rc = 0;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    do {
        // 2 * udequantize LUT (bit-exact reference table for mu-law q = 256)
        {
            float lut2[256];
            for (int q = 0; q < 256; ++q) {
                float v;
                memcpy(&v, &SRNN_ULAW_LUT_BITS[q], 4);
                lut2[q] = 2.0f * v;
            }
            rc = hipMemcpyAsync(c.b.lut2, lut2, sizeof(lut2), hipMemcpyHostToDevice, s) ? 2 : 0;
            if (rc) { srnn_set_error("generate: lut upload"); break; }
            rc = hipMemsetAsync(c.b.base, 0, 64, s) ? 2 : 0;
            if (rc) break;
            if (c.pl) {
                rc = hipMemsetAsync(c.b.gerr, 0, c.b.gm_bytes, s) ? 2 : 0;
                if (rc) break;
                rc = gen_mlp_prep_weights(c.pl, m->w_hid, m->w_out, D, m->q_levels,
                                          c.b.wfr_hid, c.b.wfr_out, s);
                if (rc) break;
            }
            int L = c.L;
            rc = hipMemcpyAsync(c.b.base, &L, sizeof(int), hipMemcpyHostToDevice, s) ? 2 : 0;
            if (rc) break;
            rc = hipStreamSynchronize(s) ? 2 : 0;   // host staging arrays go out of scope
            if (rc) break;
        }
        // initial hidden states: h0 expanded over rows (model.py:224-228)
        for (int k = 0; k < m->n_tiers && !rc; ++k)
            for (int l = 0; l < m->n_rnn; ++l) {
                const float* h0 = m->tier[k].h0 + (size_t)l * D;
                if (m->dtype == SRNN_F32)
                    hipLaunchKernelGGL((init_state_kernel<float>), dim3(cdiv(B * D, 256)),
                                       dim3(256), 0, s, h0, c.b.h[k][l][0], (float*)nullptr, B, D);
                else
                    hipLaunchKernelGGL((init_state_kernel<bf16>), dim3(cdiv(B * D, 256)),
                                       dim3(256), 0, s, h0, c.b.h[k][l][0],
                                       (bf16*)c.b.hlp[k][l][0], B, D);
            }
        if (!rc && c.b.fold) {
            // folded bottom tick operands (see fold_gru_kernel), and gh of its first tick
            const SrnnTier& t0 = m->tier[0];
            const size_t upw = (size_t)t0.frame_size * D;
            const size_t es = m->dtype == SRNN_F32 ? 4 : 2;
            rc = (hipMemcpyAsync(c.b.wcat, t0.w_up, upw * D * es, hipMemcpyDeviceToDevice, s) ||
                  hipMemcpyAsync((char*)c.b.wcat + upw * D * es, t0.w_hh[0], (size_t)3 * D * D * es,
                                 hipMemcpyDeviceToDevice, s) ||
                  hipMemcpyAsync(c.b.bcat, t0.b_up, upw * 4, hipMemcpyDeviceToDevice, s))
                     ? 2 : 0;
            if (!rc)
                rc = (t0.b_hh[0] ? hipMemcpyAsync(c.b.bcat + upw, t0.b_hh[0], (size_t)3 * D * 4,
                                                  hipMemcpyDeviceToDevice, s)
                                 : hipMemsetAsync(c.b.bcat + upw, 0, (size_t)3 * D * 4, s))
                         ? 2 : 0;
            if (rc) { srnn_set_error("generate: fold weight copy"); break; }
            const SrnnTier& t1 = m->tier[1];
            if (m->dtype == SRNN_F32)
                hipLaunchKernelGGL((fold_input_kernel<float>), dim3(cdiv(3 * D, 4)), dim3(256), 0,
                                   s, (const float*)t0.w_ih[0], (const float*)t0.w_in,
                                   t0.n_frame_samples, t0.b_in, t0.b_ih[0], t1.b_up,
                                   t1.frame_size, c.b.fmin, c.b.bfold, 3 * D, D);
            else
                hipLaunchKernelGGL((fold_input_kernel<bf16>), dim3(cdiv(3 * D, 4)), dim3(256), 0,
                                   s, (const bf16*)t0.w_ih[0], (const bf16*)t0.w_in,
                                   t0.n_frame_samples, t0.b_in, t0.b_ih[0], t1.b_up,
                                   t1.frame_size, c.b.fmin, c.b.bfold, 3 * D, D);
            if (hipGetLastError() != hipSuccess) {
                srnn_set_error("generate: fold_input launch");
                rc = 2;
                break;
            }
            // Wfold[j] = W_ih0 (3D x D) . W_up1[j] (D x D, rows j D .. j D + D - 1), bf16 out
            rc = srnn_gemm_impl(m->dtype, m->dtype, 0, 0, 3 * D, D, D, 1.f, t0.w_ih[0], D, 0,
                                t1.w_up, D, (int64_t)D * D, 0.f, nullptr, 0, 0, c.b.wfold, D,
                                (int64_t)3 * D * D, nullptr, 0, 0, t1.frame_size, -1, s);
            if (rc) break;
            // [W_hh1; b_hh1] after the folded rows, and gh1 of the first upper tick
            const size_t g0 = (size_t)t1.frame_size * 3 * D;
            rc = (hipMemcpyAsync((char*)c.b.wfold + g0 * D * es, t1.w_hh[0], (size_t)3 * D * D * es,
                                 hipMemcpyDeviceToDevice, s) ||
                  (t1.b_hh[0] ? hipMemcpyAsync(c.b.bfold + g0, t1.b_hh[0], (size_t)3 * D * 4,
                                               hipMemcpyDeviceToDevice, s)
                              : hipMemsetAsync(c.b.bfold + g0, 0, (size_t)3 * D * 4, s)))
                     ? 2 : 0;
            if (rc) { srnn_set_error("generate: fold weight copy"); break; }
            rc = linear_fwd(m->dtype, SRNN_F32, B, 3 * D, D, c.b.hlp[1][0][0], D, t1.w_hh[0], D,
                            t1.b_hh[0], c.b.fg + g0, c.b.ldg1, 0, s);
            if (rc) break;
            // gate-update operand table of the persistent loop, [fi][cur]
            std::vector<GenMlpArgs::Tick> tt(2 * t1.frame_size);
            for (int fi = 0; fi < t1.frame_size; ++fi)
                for (int pc = 0; pc < 2; ++pc) {
                    GenMlpArgs::Tick& e = tt[2 * fi + pc];
                    e.fmin = c.b.fmin;
                    e.G = c.b.fg + (size_t)fi * 3 * D;
                    e.ldg = c.b.ldg1;
                    e.gh = c.b.up[0] + upw;
                    e.ldgh = c.b.ldup0;
                    e.hp = c.b.h[0][0][pc];
                    e.hn = c.b.h[0][0][pc ^ 1];
                    e.hn_lp = c.b.hlp[0][0][pc ^ 1];
                    e.lut2 = c.b.lut2;
                }
            rc = (hipMemcpyAsync(c.b.ticks, tt.data(), tt.size() * sizeof(tt[0]),
                                 hipMemcpyHostToDevice, s) || hipStreamSynchronize(s)) ? 2 : 0;
            if (rc) { srnn_set_error("generate: tick table upload"); break; }
            if (c.b.fold_top) {
                // Min1 = W_ih1 (3D x D) . W_in1 (D x in_dim), zero-padded to TA_AP columns;
                // P1 = bf16(row_bias) . W_ih1^T + b_ih1
                rc = hipMemsetAsync(c.b.min1, 0, (size_t)3 * D * TA_AP * es, s) ? 2 : 0;
                if (!rc)
                    rc = srnn_gemm_impl(m->dtype, m->dtype, 0, 0, 3 * D, t1.in_dim, D, 1.f,
                                        t1.w_ih[0], D, 0, t1.w_in, t1.in_dim, 0, 0.f, nullptr, 0,
                                        0, c.b.min1, TA_AP, 0, nullptr, 0, 0, 1, -1, s);
                if (!rc) {
                    if (m->dtype == SRNN_F32)
                        hipLaunchKernelGGL((copy_cast_kernel<float>), dim3(cdiv(B * D, 256)),
                                           dim3(256), 0, s, c.row_bias, (float*)c.b.x[1], B * D);
                    else
                        hipLaunchKernelGGL((copy_cast_kernel<bf16>), dim3(cdiv(B * D, 256)),
                                           dim3(256), 0, s, c.row_bias, (bf16*)c.b.x[1], B * D);
                    rc = linear_fwd(m->dtype, SRNN_F32, B, 3 * D, D, c.b.x[1], D, t1.w_ih[0], D,
                                    t1.b_ih[0], c.b.p1, 3 * D, 0, s);
                }
                if (rc) break;
            }
            rc = linear_fwd(m->dtype, SRNN_F32, B, 3 * D, D, c.b.hlp[0][0][0], D, t0.w_hh[0], D,
                            t0.b_hh[0], c.b.up[0] + upw, c.b.ldup0, 0, s);
        }
        if (rc) break;
        const bool use_graph = (flags & 1) != 0;
        int done = 0;
        const int nblocks = n_cond / 2;
        if (nblocks > 0) {
            // first block eagerly (also warms up per-kernel attributes)
            rc = run_block(c, 2);
            if (rc) break;
            done = 1;
            if (use_graph && nblocks > 1) {
                if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) {
                    srnn_set_error("generate: begin capture failed");
                    rc = 2;
                    break;
                }
                rc = run_block(c, 2);
                hipError_t ce = hipStreamEndCapture(s, &graph);
                if (rc) break;
                if (ce != hipSuccess || hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) !=
                                            hipSuccess) {
                    srnn_set_error("generate: graph capture/instantiate failed");
                    rc = 2;
                    break;
                }
                for (; done < nblocks; ++done) {
                    if (hipGraphLaunch(exec, s) != hipSuccess) {
                        srnn_set_error("generate: graph launch failed");
                        rc = 2;
                        break;
                    }
                }
                if (rc) break;
            } else {
                for (; done < nblocks && !rc; ++done) rc = run_block(c, 2);
                if (rc) break;
            }
        }
        if (n_cond % 2) rc = run_block(c, 1);
    } while (0);
    // the private stream is drained before its resources go (generation is one long call)
    if (hipStreamSynchronize(s) != hipSuccess && !rc) {
        srnn_set_error("generate: %s", hipGetErrorString(hipGetLastError()));
        rc = 2;
    }
    if (!rc && c.pl) {
        int e = 0;
        if (hipMemcpy(&e, c.b.gerr, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess || e) {
            srnn_set_error(e == 2 ? "generate: persistent sample loop's workgroups were not all "
                                    "resident within 30 s (another process holds the CUs?)"
                                  : "generate: persistent sample loop lost a hand-off (spin limit)");
            rc = 2;
        }
    }
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    (void)hipEventDestroy(ev);
    (void)hipStreamDestroy(s);
    return rc;
}
