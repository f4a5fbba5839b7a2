// Per-row mu-law sampler shared by the per-step sampler kernel (mlp.hip) and the persistent
// generation loop (gen_mlp.hip), so both paths draw bit-identical samples from identical
// logits.
//
// Reference: Generator.__call__ (model.py:514-517) samples
//     x_t = exp(log_softmax(z)).multinomial(1)
// which torch>=2 on CPU implements as argmax(p / q), q ~ Exp(1) (first index on ties).
// q comes either from a device buffer (bit-replay of the reference RNG stream) or from a
// counter-based Philox4x32-10 (counter = (lane, row, step, 0), key = seed).
#pragma once
#include "common.hpp"

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
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

// Exp(1) noise of lane `lane` (q = 4 lane .. 4 lane + 3) for (row b, generation step `step`)
__device__ __forceinline__ floatx4 sample_noise(const float* noise, uint64_t seed, int B, int b,
                                                int step, int lane) {
    if (noise)
        return *reinterpret_cast<const floatx4*>(noise + ((int64_t)step * B + b) * 256 + 4 * lane);
    const uint4 rnd = philox4x32(make_uint4((uint32_t)lane, (uint32_t)b, (uint32_t)step, 0u),
                                 make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    return floatx4{exp1_from_u32(rnd.x), exp1_from_u32(rnd.y), exp1_from_u32(rnd.z),
                   exp1_from_u32(rnd.w)};
}

// One wave, one row of Q = 256 logits (lane holds q = 4 lane + j).  Returns the sampled index
// (wave-uniform); writes the row's log-probs to logp_row (if non-null).
__device__ __forceinline__ int sample_row(const floatx4& v, const floatx4& q, float* logp_row,
                                          int lane) {
    float m = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) s += expf(v[j] - m);
    s = wave_sum(s);
    const float ls = logf(s);
    float best = -1.0f;
    int bi = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float lp = (v[j] - m) - ls;
        if (logp_row) logp_row[4 * lane + j] = lp;
        const float r = expf(lp) / q[j];
        if (r > best) { best = r; bi = 4 * lane + j; }
    }
    // wave argmax, first index on ties (torch argmax)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o);
        const int oi = __shfl_xor(bi, o);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    return __builtin_amdgcn_readfirstlane(bi);
}
