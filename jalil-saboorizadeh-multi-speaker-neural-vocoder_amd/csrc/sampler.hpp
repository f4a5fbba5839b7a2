// Per-row mu-law sampler shared by the per-step sampler kernel (mlp.hip) and the persistent
// generation loop (gen_mlp.hip), so both paths draw bit-identical samples from identical
// logits.
//
// Reference: Generator.__call__ (model.py:514-517) samples
//     x_t = exp(log_softmax(z)).multinomial(1)
// which torch>=2 on CPU implements as argmax(p / q), q ~ Exp(1) (first index on ties);
// here argmax(z - log q), the same index up to fp rounding of near-ties.
// q comes either from a device buffer (bit-replay of the reference RNG stream) or from a
// counter-based Philox4x32-10 (counter = (lane, row, step, 0), key = seed).
#pragma once
#include "common.hpp"

// All-lane reductions over the wave without LDS: xor-1, xor-2 (DPP quad_perm), the
// 8-lane half mirror and the 16-lane mirror (DPP), then the lane pairs i, i ^ 16 and i, i ^ 32
// (permlane swaps).  Every step combines the same two operands in both lanes of a pair
// (a + b == b + a bitwise), so all 64 lanes end with the identical value.
template <typename Op>
__device__ __forceinline__ float wave_allreduce(float v, Op op) {
    v = op(v, __uint_as_float(dpp_u32<0xB1>(__float_as_uint(v))));    // quad_perm [1,0,3,2]
    v = op(v, __uint_as_float(dpp_u32<0x4E>(__float_as_uint(v))));    // quad_perm [2,3,0,1]
    v = op(v, __uint_as_float(dpp_u32<0x141>(__float_as_uint(v))));   // row_half_mirror
    v = op(v, __uint_as_float(dpp_u32<0x140>(__float_as_uint(v))));   // row_mirror
    uint32_t lo, hi;
    xpair16(__float_as_uint(v), lo, hi);
    v = op(__uint_as_float(lo), __uint_as_float(hi));
    xpair32(__float_as_uint(v), lo, hi);
    return op(__uint_as_float(lo), __uint_as_float(hi));
}
__device__ __forceinline__ float wave_max(float v) {
    return wave_allreduce(v, [](float a, float b) { return fmaxf(a, b); });
}
__device__ __forceinline__ float wave_sum(float v) {
    return wave_allreduce(v, [](float a, float b) { return a + b; });
}

// (best, index) argmax over the wave, first index on ties (torch argmax); same step
// sequence as wave_allreduce
__device__ __forceinline__ void amax_take(float& best, int& bi, float ob, int oi) {
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
}
template <int CTRL>
__device__ __forceinline__ void amax_dpp(float& best, int& bi) {
    const float ob = __uint_as_float(dpp_u32<CTRL>(__float_as_uint(best)));
    const int oi = (int)dpp_u32<CTRL>((uint32_t)bi);
    amax_take(best, bi, ob, oi);
}
__device__ __forceinline__ int wave_argmax(float best, int bi) {
    amax_dpp<0xB1>(best, bi);
    amax_dpp<0x4E>(best, bi);
    amax_dpp<0x141>(best, bi);
    amax_dpp<0x140>(best, bi);
    uint32_t lo, hi, ilo, ihi;
    xpair16(__float_as_uint(best), lo, hi);
    xpair16((uint32_t)bi, ilo, ihi);
    best = __uint_as_float(lo);
    bi = (int)ilo;
    amax_take(best, bi, __uint_as_float(hi), (int)ihi);
    xpair32(__float_as_uint(best), lo, hi);
    xpair32((uint32_t)bi, ilo, ihi);
    best = __uint_as_float(lo);
    bi = (int)ilo;
    amax_take(best, bi, __uint_as_float(hi), (int)ihi);
    return bi;
}

// Philox4x32-10 (Salmon et al. 2011)
__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t lo0 = c.x * 0xD2511F53u, hi0 = __umulhi(c.x, 0xD2511F53u);
        const uint32_t lo1 = c.z * 0xCD9E8D57u, hi1 = __umulhi(c.z, 0xCD9E8D57u);
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

// Exp(1) from a 32-bit draw: u in (0, 1], q = -log(u)
__device__ __forceinline__ float exp1_from_u32(uint32_t x) {
    const float u = ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
    return -logf(u);
}

// Exp(1) noise of lane `lane` (q = 4 lane .. 4 lane + 3) for (row b, generation step `step`).
// Philox counters use the GLOBAL row row0 + b: a rank generating rows [row0, row0 + B) of a
// larger batch (rank-sharded generation) draws exactly the single-process stream.
__device__ __forceinline__ floatx4 sample_noise(const float* noise, uint64_t seed, int B, int b,
                                                int step, int lane, int row0 = 0) {
    if (noise)
        return *reinterpret_cast<const floatx4*>(noise + ((int64_t)step * B + b) * 256 + 4 * lane);
    const uint4 rnd = philox4x32(make_uint4((uint32_t)lane, (uint32_t)(row0 + b), (uint32_t)step,
                                            0u),
                                 make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    return floatx4{exp1_from_u32(rnd.x), exp1_from_u32(rnd.y), exp1_from_u32(rnd.z),
                   exp1_from_u32(rnd.w)};
}

// log q of a lane's 4 noise values (computed ahead of the logits: off the critical path)
__device__ __forceinline__ floatx4 log_noise(const floatx4& q) {
    return floatx4{logf(q[0]), logf(q[1]), logf(q[2]), logf(q[3])};
}

// One wave, one row of Q = 256 logits (lane holds q = 4 lane + j), lq = log_noise(q).
// Returns the sampled index (wave-uniform); writes the row's log-probs to logp_row (if
// non-null).  The draw argmax_j softmax(z)_j / q_j (model.py:514) is taken in log space as
// argmax_j (z_j - log q_j): the softmax normaliser is common to all j, so the index needs no
// reduction but the argmax (first index on ties); log-probs, when asked for, come after.
__device__ __forceinline__ int sample_row(const floatx4& v, const floatx4& lq, float* logp_row,
                                          int lane) {
    float best = v[0] - lq[0];
    int bi = 4 * lane;
#pragma unroll
    for (int j = 1; j < 4; ++j) {
        const float t = v[j] - lq[j];
        if (t > best) { best = t; bi = 4 * lane + j; }
    }
    bi = __builtin_amdgcn_readfirstlane(wave_argmax(best, bi));
    if (logp_row) {
        float m = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
        m = wave_max(m);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) s += expf(v[j] - m);
        s = wave_sum(s);
        const float ls = logf(s);
#pragma unroll
        for (int j = 0; j < 4; ++j) logp_row[4 * lane + j] = (v[j] - m) - ls;
    }
    return bi;
}
