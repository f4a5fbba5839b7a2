// Large bf16 GEMM path, 256 x 256 tiles (M, N multiples of 256, K a multiple of 32): the
// projections of the TBPTT step -- MLP hidden/output layers, the tier-to-MLP upsampling
// (8192 x 16384 x 1024), GRU input projections -- forward, dgrad and wgrad.
//
// One 512-thread workgroup (8 waves, 2 along M x 4 along N, 128 x 64 outputs per wave =
// 8 x 4 fragments of v_mfma_f32_16x16x32_bf16) per CU.  The whole 160 KiB of LDS is a
// 5-slot ring of 32-deep k-stages (16 KiB per operand per stage) filled directly by
// global_load_lds_dwordx4; three stages stay in flight across the raw s_barrier that
// opens each stage (counted s_waitcnt vmcnt, never a __syncthreads that would drain the
// DMA queue).  LDS images (the global source addresses carry the swizzle, the DMA writes
// lane-linear):
//   k-contiguous operand   [256 rows][64 B]    16-B slot ^ g3_kcswz(row): the 16 lanes
//                          of each ds_read_b128 lane group hit 16 distinct bank quads;
//   row-contiguous operand [32 k-rows][512 B]  16-B slot ^ (2*(k&3) + 8*((k>>3)&1)):
//                          ds_read_b64_tr_b16 transposed reads, 32 distinct 8-B bank
//                          slots per 32-lane pass.
// The MFMA runs with the operands swapped (B fragment as the "A" input), so each lane
// ends up with 4 CONSECUTIVE COLUMNS of one output row: the epilogue loads Cin / bias /
// the ReLU mask and stores C as 8- or 16-byte vectors instead of 2-4 byte scalars.
// Split-K (gridDim.z) accumulates fp32 partial tiles with atomics into a zeroed C for the
// weight-gradient shapes whose 256 x 256 tile grid cannot fill 256 CUs.
#include "gemm3_core.hpp"

__device__ __forceinline__ void g3_load4(const float* p, float (&v)[4]) {
    const floatx4 x = *reinterpret_cast<const floatx4*>(p);
    v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
}
__device__ __forceinline__ void g3_load4(const bf16* p, float (&v)[4]) {
    const u16x4 x = *reinterpret_cast<const u16x4*>(p);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = __uint_as_float((unsigned)x[e] << 16);
}
__device__ __forceinline__ void g3_store4(float* p, const float (&v)[4]) {
    *reinterpret_cast<floatx4*>(p) = floatx4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ void g3_store4(bf16* p, const float (&v)[4]) {
    u16x4 x;
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = __bfloat16_as_ushort(__float2bfloat16(v[e]));
    *reinterpret_cast<u16x4*>(p) = x;
}

// SW: operands swapped in the MFMA (vector epilogue); !SW: the plain split-K partial
// path, where a lane's 4 values are 4 rows of one column and each atomic instruction
// covers 16 consecutive columns (64 B) of 4 rows instead of 16 rows x 4 B.
// epilogue of one finished tile (registers -> C); zeroes the accumulators
// AMX: also reduce max |C| into g.amax (its own instantiation: tracking the max in the
// plain epilogue pushed the main loops past 256 VGPRs -- ~100 spilled)
// MB: ReLU mask bits -- 1: g.mbi / g.mbo row-major, read / written here; 2: g.mbi grouped
// (srnn_bits_index, ldmbi = 0), this wave's 128 rows x 4 column groups already staged in LDS at
// mbl ([group][row] u16) by the kernel's LDS-DMA ahead of the epilogue
// AMX: the lane's running max |C| bits (amx) over the launch's tiles: reduced and atomicMax-ed
// once per wave at the end of the kernel (g3_amax_flush), not per tile -- one atomic address
// taking 65536 per-tile atomics cost ~0.14 ms of a 1.2-ms GEMM
template <typename TO, bool SW, bool CIN, int MB = 0, bool AMX = false, int CS = 0>
__device__ __forceinline__ void g3_epilogue_t(const Gemm3Args& g, floatx4 (&acc)[8][4], int m0,
                                              int n0, int wm, int wn, int lane, int kb,
                                              const char* mbl = nullptr, unsigned* amx_run = nullptr) {
    if constexpr (!SW) {
        // plain fp32 partials: lane holds 4 rows x 1 column per fragment
        if (g.ksplit > 1 && g.part) {
            // this k-slice's partial tile, plain stores (rows of 16 consecutive columns)
            float* Pz = g.part + (size_t)(kb / (g.K / g.ksplit)) * g.M * g.N;
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int col = n0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int row = m0 + wm * 128 + i * 16 + (lane >> 4) * 4 + e;
                        Pz[(int64_t)row * g.N + col] = g.alpha * acc[i][j][e];
                    }
                    acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
                }
            return;
        }
        float* Cf = reinterpret_cast<float*>(g.C);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = n0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = m0 + wm * 128 + i * 16 + (lane >> 4) * 4 + e;
                    float* dst = Cf + (int64_t)row * g.ldc + col;
                    if (g.ksplit > 1) atomicAdd(dst, g.alpha * acc[i][j][e]);
                    else *dst = g.alpha * acc[i][j][e];
                }
                acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
        return;
    }
    // lane holds C[row][col .. col+3] of each fragment.  Every operand the epilogue needs
    // (bias, ReLU mask) is loaded up front with ONE wait: a load waited for between the
    // stores would also wait for every older store and in-flight DMA piece (vmcnt is in
    // order), serialising 32 round trips per tile.  Exactly 32 stores per wave follow.
    TO* Cp = reinterpret_cast<TO*>(g.C);
    // (MB == 2 kernels take no bf16 mask: srnn_gemm3_try admits grouped bits without one)
    const bf16* mask = MB == 2 ? nullptr : reinterpret_cast<const bf16*>(g.mask);
    const int rbase = m0 + wm * 128 + (lane & 15);
    const int cbase = n0 + wn * 64 + (lane >> 4) * 4;
    // MB == 2 (the da1 GEMM's kernels) is lean: no bias, ReLU or blocked copy (srnn_gemm3_try
    // routes such calls elsewhere), so none of their code or registers is in the epilogue; the
    // (the same for the column-sum kernels measured slower: da2 0.67 -> 0.70 ms, not kept)
    constexpr bool LEAN = MB == 2;
    constexpr bool NOB = LEAN;
    floatx4 bcol[4];
    float brow[8];
    if (!NOB && g.bias_mode == 1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bcol[j] = *reinterpret_cast<const floatx4*>(g.bias + cbase + j * 16);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) bcol[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    if (!NOB && g.bias_mode == 2) {
#pragma unroll
        for (int i = 0; i < 8; ++i) brow[i] = g.bias[rbase + i * 16];
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) brow[i] = 0.f;
    }
    // bit mask: the row's 64 bits of the wave's columns, one 8-B load per row (per half,
    // with the bf16 mask's loads); lane's bit for (fragment j, element e) at
    // (j & 1) * 16 + (lane >> 4) * 4 + e of word j >> 1
    const unsigned short* mbi = MB == 1 ? g.mbi : nullptr;
    unsigned short* mbo = MB == 1 ? g.mbo : nullptr;
    const bool mbits = MB == 2 || mbi;             // outputs zeroed where the mask bit is clear
    const int g4 = (lane >> 4) * 4;
    unsigned amx = AMX ? *amx_run : 0u;
    unsigned amx2 = 0u;                        // LEAN: two 15-bit maxima, packed
    float cs[CS ? 4 : 1][4];                   // CS: the lane's 16 columns summed over its rows
    if constexpr (CS) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) cs[j][e] = 0.f;
    }
    // the mask in two halves of 16 fragments (register budget): two waits per tile
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        u16x4 mk[4][4];                        // (bit mask: row ii's 64 bits in mk[ii][0])
        if (mask) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    mk[i][j] = *reinterpret_cast<const u16x4*>(
                        mask + (int64_t)(rbase + (4 * h + i) * 16) * g.ldmask + cbase + j * 16);
        } else if (mbi) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                mk[i][0] = *reinterpret_cast<const u16x4*>(
                    mbi + (int64_t)(rbase + (4 * h + i) * 16) * g.ldmbi + (n0 + wn * 64) / 16);
        } else if constexpr (MB == 2) {
            const unsigned short* mw = reinterpret_cast<const unsigned short*>(mbl);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = (lane & 15) + (4 * h + i) * 16;
#pragma unroll
                for (int c = 0; c < 4; ++c) mk[i][0][c] = mw[c * 128 + r];
            }
        }
        auto mbit = [&](int ii, int j, int e) -> bool {
            const unsigned w = (unsigned)mk[ii][0][(j >> 1) * 2] |
                               ((unsigned)mk[ii][0][(j >> 1) * 2 + 1] << 16);
            return (w >> (((j & 1) << 4) + g4 + e)) & 1u;
        };
        if constexpr (sizeof(TO) == 2 && !CIN) {
            // bf16 out: fragments j, j + 1 of a row combined by two v_permlane16_swap per
            // pair, so every lane stores 16 B (8 columns) -- half the store instructions of
            // the 8-B-per-fragment form (the epilogue tail is store-issue-bound).  amx: the
            // largest |value| stored (bf16 magnitude bits: their unsigned order is the
            // magnitude order)
            const int grp = lane >> 4;
            const int coff = 16 * (grp & 1) + 8 * (grp >> 1) - 4 * grp;   // lane's 16-B column
            unsigned wbits[4][2];                      // bits out: rows 4h + ii, words lo / hi
#pragma unroll
            for (int ii = 0; ii < 4; ++ii) {
                const int i = 4 * h + ii;
                const int row = rbase + i * 16;
                wbits[ii][0] = wbits[ii][1] = 0u;
#pragma unroll
                for (int jp = 0; jp < 2; ++jp) {
                    unsigned pk[2][2];
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const int j = 2 * jp + t;
                        if constexpr (LEAN) {
                            // two columns per instruction: one packed conversion, then the
                            // pair's two mask bits widened to a 32-bit AND mask (a zeroed
                            // value's bits are +0, as the select's)
                            const unsigned w = (unsigned)mk[ii][0][2 * jp] |
                                               ((unsigned)mk[ii][0][2 * jp + 1] << 16);
#pragma unroll
                            for (int e = 0; e < 2; ++e) {
                                typedef float g3f2 __attribute__((ext_vector_type(2)));
                                typedef __bf16 g3b2 __attribute__((ext_vector_type(2)));
                                const g3f2 pv = {g.alpha * acc[i][j][2 * e], g.alpha * acc[i][j][2 * e + 1]};
                                const unsigned c = __builtin_bit_cast(unsigned, __builtin_convertvector(pv, g3b2));
                                const unsigned x = __builtin_amdgcn_ubfe(w, (t << 4) + g4 + 2 * e, 2);
                                pk[t][e] = c & __umul24((x | (x << 15)) & 0x10001u, 0xffffu);
                            }
                            acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
                            continue;
                        }
                        float v[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            v[e] = NOB ? g.alpha * acc[i][j][e] : g.alpha * acc[i][j][e] + bcol[j][e] + brow[i];
                        acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
                        if (!NOB && g.relu) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                        }
                        if (mask) {
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                v[e] = __uint_as_float((unsigned)mk[ii][j][e] << 16) > 0.f ? v[e] : 0.f;
                        } else if (mbits) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) v[e] = mbit(ii, j, e) ? v[e] : 0.f;
                        }
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            pk[t][e] = (unsigned)__bfloat16_as_ushort(__float2bfloat16(v[2 * e])) |
                                       ((unsigned)__bfloat16_as_ushort(__float2bfloat16(v[2 * e + 1])) << 16);
                            if constexpr (CS) {        // the stored (bf16-rounded) values
                                cs[j][2 * e] += __uint_as_float(pk[t][e] << 16);
                                cs[j][2 * e + 1] += __uint_as_float(pk[t][e] & 0xffff0000u);
                            }
                        }
                        if (mbo) {
                            // value > 0 of the stored bf16: 0x0001 .. 0x7f80 (no -0, no NaN)
                            unsigned nib = 0u;
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const unsigned u = (pk[t][e >> 1] >> (16 * (e & 1))) & 0xffffu;
                                nib |= (u - 1u < 0x7f80u ? 1u : 0u) << e;
                            }
                            wbits[ii][j >> 1] |= nib << (((j & 1) << 4) + g4);
                        }
                    }
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const auto r = __builtin_amdgcn_permlane16_swap(pk[0][e], pk[1][e], false, false);
                        pk[0][e] = r[0];
                        pk[1][e] = r[1];
                    }
                    if constexpr (AMX) {
                        // (after the swap: the wave's maximum is the same over any lane
                        //  permutation, and no pre-swap copy stays live; LEAN: both halves at
                        //  once, v_pk_max_u16, folded once per epilogue)
#pragma unroll
                        for (int t = 0; t < 2; ++t)
#pragma unroll
                            for (int e = 0; e < 2; ++e) {
                                if constexpr (LEAN) {
                                    typedef unsigned short g3u2 __attribute__((ext_vector_type(2)));
                                    amx2 = __builtin_bit_cast(unsigned, __builtin_elementwise_max(
                                        __builtin_bit_cast(g3u2, amx2),
                                        __builtin_bit_cast(g3u2, pk[t][e] & 0x7fff7fffu)));
                                } else {
                                    amx = max(amx, max(pk[t][e] & 0x7fffu, (pk[t][e] >> 16) & 0x7fffu));
                                }
                            }
                    }
                    *reinterpret_cast<uint4*>(Cp + (int64_t)row * g.ldc + cbase + 32 * jp + coff) =
                        make_uint4(pk[0][0], pk[0][1], pk[1][0], pk[1][1]);
                    if constexpr (AMX && !LEAN) {
                        if (g.blk) {
                            // the same 8 columns as two 4-column blocks: 16 lanes (rows
                            // rbase .. + 15) of a block write one contiguous 128-B line
                            const int cb = (cbase + 32 * jp + coff) >> 2;
                            bf16* bp = g.blk + ((int64_t)cb * g.M + row) * 4;
                            *reinterpret_cast<uint2*>(bp) = make_uint2(pk[0][0], pk[0][1]);
                            *reinterpret_cast<uint2*>(bp + (int64_t)g.M * 4) =
                                make_uint2(pk[1][0], pk[1][1]);
                        }
                    }
                }
            }
            if (mbo) {
                // OR over the 4 lanes of a row (lane ^ 16, ^ 32), then lane group g stores
                // row 4h + g: one 8-B store per lane for the half's 4 rows
                unsigned sel[2] = {0u, 0u};
#pragma unroll
                for (int ii = 0; ii < 4; ++ii)
#pragma unroll
                    for (int w = 0; w < 2; ++w) {
                        unsigned a, b, x = wbits[ii][w];
                        xpair16(x, a, b);
                        x = a | b;
                        xpair32(x, a, b);
                        x = a | b;
                        if (ii == grp) sel[w] = x;
                    }
                *reinterpret_cast<uint2*>(mbo + (int64_t)(rbase + (4 * h + grp) * 16) * g.ldmbo +
                                          (n0 + wn * 64) / 16) = make_uint2(sel[0], sel[1]);
            }
            continue;
        }
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) {
            const int i = 4 * h + ii;
            const int row = rbase + i * 16;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = cbase + j * 16;
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = g.alpha * acc[i][j][e];
                acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
                if (CIN) {     // (no model GEMM on this path uses Cin)
                    float c[4];
                    g3_load4(g.Cin + (int64_t)row * g.ldcin + col, c);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] += g.beta * c[e];
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += bcol[j][e] + brow[i];
                if (g.relu) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                }
                if (mask) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        v[e] = __uint_as_float((unsigned)mk[ii][j][e] << 16) > 0.f ? v[e] : 0.f;
                } else if (mbits) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = mbit(ii, j, e) ? v[e] : 0.f;
                }
                g3_store4(Cp + (int64_t)row * g.ldc + col, v);
            }
        }
    }
    if constexpr (CS) {
        // sum over the 16 lanes of a DPP row (the wave's 16 rows of each i; every lane ends
        // with a total, in a fixed order), then lane q of the row stores column (q >> 2) * 16
        // + (q & 3) of its group: one 4-B store per lane, 64 columns per wave -- exactly one
        // store more per tile (g3_epilogue's count)
        float o = 0.f;
        const int q = lane & 15;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float x = cs[j][e];
                x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xf, 0xf, false));
                x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xf, 0xf, false));
                x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x122, 0xf, 0xf, false));
                x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x121, 0xf, 0xf, false));
                o = (q == j * 4 + e) ? x : o;
            }
        g.csp[(int64_t)((m0 + wm * 128) / 128) * g.N + n0 + wn * 64 + g4 + (q >> 2) * 16 + (q & 3)] = o;
    }
    if constexpr (AMX) *amx_run = LEAN ? max(amx, max(amx2 & 0xffffu, amx2 >> 16)) : amx;
}

// The Cin branch is resolved once per tile: a uniform branch inside the store loop makes
// the compiler join its wait states with an s_waitcnt vmcnt(0) per fragment, which waits
// for every store issued before it (32 serialised store round trips per tile).
// Returns the number of stores each wave issued (SW path): the main loops' counted DMA
// waits leave exactly that many younger stores in flight, so the count must be exact -- a
// larger allowance would let a stage's DMA pieces still be outstanding at the read.
template <typename TO, bool SW, int MB = 0, bool AMX = false, int CS = 0>
__device__ __forceinline__ int g3_epilogue(const Gemm3Args& g, floatx4 (&acc)[8][4], int m0,
                                           int n0, int wm, int wn, int lane, int kb,
                                           const char* mbl = nullptr, unsigned* amx_run = nullptr) {
    if constexpr (CS && sizeof(TO) == 2 && SW) {
        // the column-sum kernels (bf16 out, no Cin, no bit masks, no max |C|)
        g3_epilogue_t<TO, SW, false, 0, false, CS>(g, acc, m0, n0, wm, wn, lane, kb);
        return 17;
    }
    if constexpr (AMX) {
        // (with MB == 2 at most: max |C| is never combined with row-major bits or bits out)
        g3_epilogue_t<TO, SW, false, MB == 2 ? 2 : 0, true>(g, acc, m0, n0, wm, wn, lane, kb, mbl,
                                                            amx_run);
        return g.blk ? 48 : 16;                    // + the blocked copy's 2 stores per store
    }
    if constexpr (MB != 0) {
        // the bit-mask kernels (their own instantiation: the plain epilogue keeps its registers)
        g3_epilogue_t<TO, SW, false, MB>(g, acc, m0, n0, wm, wn, lane, kb, mbl);
        return sizeof(TO) == 2 ? 16 + (MB == 1 && g.mbo ? 2 : 0) : 32;
    }
    if (SW && g.beta != 0.f) {
        g3_epilogue_t<TO, SW, true>(g, acc, m0, n0, wm, wn, lane, kb);
        return 32;
    }
    g3_epilogue_t<TO, SW, false>(g, acc, m0, n0, wm, wn, lane, kb);
    return sizeof(TO) == 2 ? 16 : 32;
}

// C[m][n] = sum_z part[z][m][n], z in order (4 columns per thread)
__global__ __launch_bounds__(256) void g3_splitk_sum_kernel(const float* __restrict__ part,
                                                             float* __restrict__ C, int64_t ldc,
                                                             int M, int N, int ks) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;      // float4 index
    const int64_t MN = (int64_t)M * N;
    if (q * 4 >= MN) return;
    const int64_t e = q * 4;
    const int m = (int)(e / N), n = (int)(e % N);
    const floatx4* p = reinterpret_cast<const floatx4*>(part + e);
    const int64_t zs = MN / 4;
    floatx4 s = p[0];
    int z = 1;
    for (; z + 4 <= ks; z += 4) {            // 4 slices in flight, summed in z order
        floatx4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = p[(z + u) * zs];
#pragma unroll
        for (int u = 0; u < 4; ++u) s += v[u];
    }
    for (; z < ks; ++z) s += p[z * zs];
    *reinterpret_cast<floatx4*>(C + (int64_t)m * ldc + n) = s;
}

// Grow-only device scratch buffers, one per slot (samplernn_hip_internal.hpp).  A buffer
// that is outgrown is retired, never freed: a captured HIP graph (trainer graph mode) keeps
// the pointer that was current at capture, so every buffer must outlive later growth.  The
// retired ones total less than the live one (sizes grow geometrically from the first calls).
void* srnn_scratch(int slot, size_t bytes) {
    static void* buf[SRNN_SCRATCH_SLOTS] = {};
    static size_t have[SRNN_SCRATCH_SLOTS] = {};
    if (slot < 0 || slot >= SRNN_SCRATCH_SLOTS) return nullptr;
    if (bytes > have[slot]) {
        const size_t want = bytes > 2 * have[slot] ? bytes : 2 * have[slot];
        void* p = nullptr;
        if (hipMalloc(&p, want) != hipSuccess) return nullptr;
        buf[slot] = p;
        have[slot] = want;
    }
    return buf[slot];
}

float* srnn_splitk_scratch(size_t bytes) {
    return (float*)srnn_scratch(SRNN_SCRATCH_SPLITK, bytes);
}

int srnn_splitk_sum(const float* part, float* C, int64_t ldc, int M, int N, int ks, hipStream_t s) {
    const int64_t nq = (int64_t)M * N / 4;
    hipLaunchKernelGGL(g3_splitk_sum_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, s,
                       part, C, ldc, M, N, ks);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// Persistent: workgroup w owns work units w, w + G, ... (unit = output tile x k-slice);
// the k-stages of all its units form ONE stream through the ring, so the DMA of the next
// tile's first stages runs under the current tile's last MFMAs and epilogue.
template <typename TO, bool KCA, bool KCB, bool SW, bool MB = false>
__global__ __launch_bounds__(512, 1) void gemm3_kernel(Gemm3Args g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave & 1, wn = wave >> 1;
    const int ntm = g.M / g3::BM, ntn = g.N / g3::BN;
    const int ntiles = ntm * ntn;
    const int nunits = ntiles * g.ksplit;
    const int G = gridDim.x;
    const int nmine = (nunits - (int)blockIdx.x + G - 1) / G;
    const int kslice = g.K / g.ksplit;
    const int nk = kslice / g3::BK;
    const int S = nmine * nk;                  // stages of this workgroup
    const bf16* A = reinterpret_cast<const bf16*>(g.A);
    const bf16* B = reinterpret_cast<const bf16*>(g.B);

    // unit i of this workgroup -> (m0, n0, kbeg); units on one XCD walk adjacent tiles
    auto unit = [&](int i, int& m0, int& n0, int& kbeg) {
        const int v = (int)blockIdx.x + i * G;
        const int z = v / ntiles;
        const int t = g3_xcd_remap(v - z * ntiles, ntiles);
        m0 = (t / ntn) * g3::BM;
        n0 = (t % ntn) * g3::BN;
        kbeg = z * kslice;
    };

    floatx4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // issue cursor: unit iu, stage kti; per-lane sources of this wave's 4 DMA pieces
    int iu = 0, kti = 0;
    const bf16* srcA[g3::GLW];
    const bf16* srcB[g3::GLW];
    auto set_src = [&]() {
        int m0, n0, kb;
        unit(iu, m0, n0, kb);
#pragma unroll
        for (int i = 0; i < g3::GLW; ++i) {
            const int c = wave * g3::GLW + i;
            srcA[i] = g3_src<KCA>(A, g.lda, m0, kb, c, lane);
            srcB[i] = g3_src<KCB>(B, g.ldb, n0, kb, c, lane);
        }
    };
    set_src();
    auto glds = [&](const bf16* src, int64_t koff, char* img, int i) {
        __builtin_amdgcn_global_load_lds(G3_GLB(src + koff), G3_LDS(img + (wave * g3::GLW + i) * 1024),
                                         16, 0, 0);
    };
    auto koffA = [&](int kt) { return KCA ? (int64_t)kt * g3::BK : (int64_t)kt * g3::BK * g.lda; };
    auto koffB = [&](int kt) { return KCB ? (int64_t)kt * g3::BK : (int64_t)kt * g3::BK * g.ldb; };
    auto advance_issue = [&]() {
        if (++kti == nk) {
            kti = 0;
            ++iu;
            if (iu < nmine) set_src();
        }
    };
    int ws = 0;
    auto next_ws = [&]() { ws = ws == g3::NS - 1 ? 0 : ws + 1; };
#pragma unroll
    for (int s = 0; s < g3::NS - 1; ++s)
        if (s < S) {
            char* img = smem + ws * g3::SLOT;
            const int64_t oa = koffA(kti), ob = koffB(kti);
#pragma unroll
            for (int i = 0; i < g3::GLW; ++i) glds(srcA[i], oa, img, i);
#pragma unroll
            for (int i = 0; i < g3::GLW; ++i) glds(srcB[i], ob, img + g3::OPB, i);
            next_ws();
            advance_issue();
        }

    constexpr int PER = 2 * g3::GLW;
    int rs = 0;
    bf16x8 a[8], b[4];
    auto read_stage = [&]() {
        const char* ia = smem + rs * g3::SLOT;
        const char* ib = ia + g3::OPB;
        rs = rs == g3::NS - 1 ? 0 : rs + 1;
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = g3_frag<KCB>(ib, wn * 64 + j * 16, lane);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = g3_frag<KCA>(ia, wm * 128 + i * 16, lane);
    };
    auto mfma_row = [&](int i) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0)
                           : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    };
    // compute cursor: unit ic, stage ktc
    int ic = 0, ktc = 0;
    int epi = 0;                               // stores of the just-finished tile's epilogue
    auto finish_stage = [&]() {
        if (++ktc == nk) {
            int m0, n0, kb;
            unit(ic, m0, n0, kb);
            epi = g3_epilogue<TO, SW, MB>(g, acc, m0, n0, wm, wn, lane, kb);
            ktc = 0;
            ++ic;
        }
    };
    // Steady state: every stage issues the DMA pieces of stage s+NS-1 into the slot freed
    // by stage s-1, one piece after each of the first four 4-MFMA groups, so the issue
    // cost of the LDS-DMA hides behind the matrix pipe instead of stalling all waves
    // right after the barrier.
    int s = 0;
    for (; s + g3::NS - 1 < S; ++s) {
        // the 32 epilogue stores of a just-finished tile are younger than the pieces
        // waited for here: leave them in flight
        if (SW && epi == 16) g3_wait_vm<(g3::NS - 2) * PER + 16>();
        else if (SW && epi == 18) g3_wait_vm<(g3::NS - 2) * PER + 18>();   // + mask bits
        else if (SW && epi) g3_wait_vm<(g3::NS - 2) * PER + 32>();
        else g3_wait_vm<(g3::NS - 2) * PER>();
        epi = 0;
        __builtin_amdgcn_s_barrier();
        char* img = smem + ws * g3::SLOT;
        next_ws();
        const int64_t oa = koffA(kti), ob = koffB(kti);
        const bf16* a0 = srcA[0];
        const bf16* a1 = srcA[1];
        const bf16* b0 = srcB[0];
        const bf16* b1 = srcB[1];
        advance_issue();
        read_stage();
        __builtin_amdgcn_s_setprio(1);
        mfma_row(0);
        glds(a0, oa, img, 0);
        mfma_row(1);
        glds(a1, oa, img, 1);
        mfma_row(2);
        glds(b0, ob, img + g3::OPB, 0);
        mfma_row(3);
        glds(b1, ob, img + g3::OPB, 1);
#pragma unroll
        for (int i = 4; i < 8; ++i) mfma_row(i);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
        finish_stage();
    }
    // tail: nothing left to issue, the in-flight stages drain
    for (; s < S; ++s) {
        g3_wait_sel<PER, g3::NS - 2>(S - 1 - s);
        __builtin_amdgcn_s_barrier();
        read_stage();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 8; ++i) mfma_row(i);
        __builtin_amdgcn_s_setprio(0);
        finish_stage();
    }
}

// ---------------------------------------------------------------------------------
// Log-softmax epilogue (g.lsm; fp32 out, N = 256, so a tile holds whole rows): logp =
// (v - max) - log(sum exp(v - max)) per row with v = alpha acc + bias, the same arithmetic as
// logsoftmax_nll_kernel (mlp.hip), so the (B T, Q) logits never round-trip through HBM
// (model.py:324-325).  A row's 256 columns live in the 4 waves of equal wm (64 each): the
// per-wave row maxima, then the per-wave sums of exp, meet in LDS (red: [2][2 wm][4 wn][128]
// floats) across two raw barriers every wave of the workgroup takes.  Returns the stores (32).
__device__ __forceinline__ int g3_epilogue_lsm(const Gemm3Args& g, floatx4 (&acc)[8][4], int m0,
                                               int n0, int wm, int wn, int lane, float* red) {
    const int rl = lane & 15;
    const int rbase = m0 + wm * 128 + rl;
    const int cbase = n0 + wn * 64 + (lane >> 4) * 4;
    floatx4 bcol[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        bcol[j] = g.bias ? *reinterpret_cast<const floatx4*>(g.bias + cbase + j * 16)
                         : floatx4{0.f, 0.f, 0.f, 0.f};
    float mx[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        float m = -INFINITY;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            acc[i][j] = acc[i][j] * g.alpha + bcol[j];
#pragma unroll
            for (int e = 0; e < 4; ++e) m = fmaxf(m, acc[i][j][e]);
        }
        m = fmaxf(m, __shfl_xor(m, 16));
        m = fmaxf(m, __shfl_xor(m, 32));
        mx[i] = m;
    }
    float* rmax = red + (wm * 4) * 128;            // [wn][128] for this wm
    float* rsum = red + (8 + wm * 4) * 128;
    if (lane < 16) {
#pragma unroll
        for (int i = 0; i < 8; ++i) rmax[wn * 128 + i * 16 + rl] = mx[i];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    float sm[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int r = i * 16 + rl;
        const float m = fmaxf(fmaxf(rmax[r], rmax[128 + r]), fmaxf(rmax[256 + r], rmax[384 + r]));
        mx[i] = m;
        float sv = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) sv += expf(acc[i][j][e] - m);
        sv += __shfl_xor(sv, 16);
        sv += __shfl_xor(sv, 32);
        sm[i] = sv;
    }
    if (lane < 16) {
#pragma unroll
        for (int i = 0; i < 8; ++i) rsum[wn * 128 + i * 16 + rl] = sm[i];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    float* Cf = reinterpret_cast<float*>(g.C);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int r = i * 16 + rl;
        const float ls = logf(rsum[r] + rsum[128 + r] + rsum[256 + r] + rsum[384 + r]);
        const float m = mx[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            floatx4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (acc[i][j][e] - m) - ls;
            acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
            *reinterpret_cast<floatx4*>(Cf + (int64_t)(rbase + i * 16) * g.ldc + cbase + j * 16) = o;
        }
    }
    return 32;
}

// PF: the k-unit 1 fragments of a stage are read into a second register set while unit 0's
// MFMAs run (3 reads after each of its last four MFMA rows), so the unit-1 MFMAs do not wait
// for a burst of 12 LDS reads.
template <typename TO, bool KCA, bool KCB, bool SW, int MB = 0, bool PF = false,
          bool AMX = false, int CS = 0, int LS = 0>
__global__ __launch_bounds__(512, 1) void gemm3p_kernel(Gemm3Args g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave & 1, wn = wave >> 1;
    const int ntm = g.M / g3::BM, ntn = g.N / g3::BN;
    const int ntiles = ntm * ntn;
    const int nunits = ntiles * g.ksplit;
    const int G = gridDim.x;
    const int nmine = (nunits - (int)blockIdx.x + G - 1) / G;
    const int kslice = g.K / g.ksplit;
    const int nk = kslice / g3p::BK;
    const int S = nmine * nk;
    const bf16* A = reinterpret_cast<const bf16*>(g.A);
    const bf16* B = reinterpret_cast<const bf16*>(g.B);

    auto unit = [&](int i, int& m0, int& n0, int& kbeg) {
        const int v = (int)blockIdx.x + i * G;
        const int z = v / ntiles;
        const int t = g3_xcd_remap(v - z * ntiles, ntiles);
        m0 = (t / ntn) * g3::BM;
        n0 = (t % ntn) * g3::BN;
        kbeg = z * kslice;
    };

    floatx4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // pieces i and i+2 of a wave differ by a fixed row (k-row) offset, so two per-lane
    // pointers per operand cover all four
    const int64_t stepA = KCA ? (int64_t)16 * g.lda : (int64_t)4 * g.lda;
    const int64_t stepB = KCB ? (int64_t)16 * g.ldb : (int64_t)4 * g.ldb;
    int iu = 0, kti = 0;
    const bf16* srcA[2];
    const bf16* srcB[2];
    // MB == 2: tile iu's mask bits (grouped layout) for this wave's 128 rows x 4 column groups,
    // 1 KiB: lane l takes 8 rows of group l / 16 (16 B), issued with the tile's first DMA
    // pieces into LDS buffer iu & 1 (the epilogue of tile iu - 1 reads the other); the stage
    // waits retire it long before the epilogue reads it (this wave's own bytes: no barrier)
    auto set_src = [&]() {
        int m0, n0, kb;
        unit(iu, m0, n0, kb);
        if constexpr (MB == 2) {
            // (the wave's block offset is uniform: a scalar; < 2^31 u16 -- M N / 16)
            const int o = __builtin_amdgcn_readfirstlane(((n0 + wn * 64) >> 4) * g.M + m0 + wm * 128);
            __builtin_amdgcn_global_load_lds(
                G3_GLB(g.mbi + o + (int64_t)(lane >> 4) * g.M + (lane & 15) * 8),
                G3_LDS(smem + g3p::LDS + (iu & 1) * 8192 + wave * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = wave * g3p::GLW + i;
            srcA[i] = g3p_src<KCA>(A, g.lda, m0, kb, c, lane);
            srcB[i] = g3p_src<KCB>(B, g.ldb, n0, kb, c, lane);
        }
    };
    set_src();
    auto glds = [&](const bf16* src, char* img, int i) {
        __builtin_amdgcn_global_load_lds(G3_GLB(src), G3_LDS(img + (wave * g3p::GLW + i) * 1024),
                                         16, 0, 0);
    };
    auto koffA = [&](int kt) { return KCA ? (int64_t)kt * g3p::BK : (int64_t)kt * g3p::BK * g.lda; };
    auto koffB = [&](int kt) { return KCB ? (int64_t)kt * g3p::BK : (int64_t)kt * g3p::BK * g.ldb; };
    auto advance_issue = [&]() {
        if (++kti == nk) {
            kti = 0;
            ++iu;
            if (iu < nmine) set_src();
        }
    };
    auto issue_all = [&](char* img) {
        const int64_t oa = koffA(kti), ob = koffB(kti);
#pragma unroll
        for (int i = 0; i < g3p::GLW; ++i) glds(srcA[i & 1] + oa + (i >> 1) * stepA, img, i);
#pragma unroll
        for (int i = 0; i < g3p::GLW; ++i)
            glds(srcB[i & 1] + ob + (i >> 1) * stepB, img + g3p::OPB, i);
        advance_issue();
    };
    if (S > 0) issue_all(smem);

    bf16x8 a[8], b[4];
    bf16x8 a1[PF ? 8 : 1], b1[PF ? 4 : 1];
    int ic = 0, ktc = 0;
    int epi = 0;                               // stores of the just-finished tile's epilogue
    auto read_unit = [&](const char* img, int u) {
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = g3p_frag<KCB>(img + g3p::OPB, wn * 64 + j * 16, u, lane);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = g3p_frag<KCA>(img, wm * 128 + i * 16, u, lane);
    };
    auto mfma_row = [&](int i) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0)
                           : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    };
    auto mfma_row1 = [&](int i) {
        if constexpr (PF) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a1[i], acc[i][j], 0, 0, 0)
                               : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);
        }
    };
    // fragment f (0..11) of unit 1: B fragments first, then A
    auto read1 = [&](const char* img, int f) {
        if constexpr (PF) {
            if (f < 4) b1[f] = g3p_frag<KCB>(img + g3p::OPB, wn * 64 + f * 16, 1, lane);
            else a1[f - 4] = g3p_frag<KCA>(img, wm * 128 + (f - 4) * 16, 1, lane);
        }
    };
    unsigned amx_run = 0u;                     // AMX: this lane's max |C| bits so far
    auto finish_stage = [&]() {
        if (++ktc == nk) {
            int m0, n0, kb;
            unit(ic, m0, n0, kb);
            const char* mbl = smem + g3p::LDS + (ic & 1) * 8192 + wave * 1024;
            if constexpr (LS) {
                (void)mbl;
                epi = g3_epilogue_lsm(g, acc, m0, n0, wm, wn, lane,
                                      reinterpret_cast<float*>(smem + g3p::LDS));
            } else {
                epi = (g.diag & 8) ? 0
                                   : g3_epilogue<TO, SW, MB, AMX, CS>(g, acc, m0, n0, wm, wn, lane,
                                                                      kb, mbl, &amx_run);
            }
            ktc = 0;
            ++ic;
        }
    };
    // Stage s+1 is issued right after the barrier that opens stage s, into the slot
    // stage s-1 just vacated, two DMA pieces per MFMA group of the first k-unit.
    int s = 0;
    for (; s + 1 < S; ++s) {
        const char* img = smem + (s & 1) * g3p::SLOT;
        char* nimg = smem + ((s + 1) & 1) * g3p::SLOT;
        if (SW && epi == 16) g3_wait_vm<16>();
        else if (SW && epi == 17) g3_wait_vm<17>();                        // + column sums
        else if (SW && epi == 18) g3_wait_vm<18>();                        // + mask bits
        else if (SW && epi == 48) g3_wait_vm<48>();                        // + blocked copy
        else if (SW && epi) g3_wait_vm<32>();
        else g3_wait_vm<0>();
        epi = 0;
        __builtin_amdgcn_s_barrier();
        const int64_t oa = koffA(kti), ob = koffB(kti);
        const bf16* pa0 = srcA[0] + oa;
        const bf16* pa1 = srcA[1] + oa;
        const bf16* pb0 = srcB[0] + ob;
        const bf16* pb1 = srcB[1] + ob;
        advance_issue();
        read_unit(img, 0);
        __builtin_amdgcn_s_setprio(1);
        mfma_row(0); glds(pa0, nimg, 0); glds(pa1, nimg, 1);
        mfma_row(1); glds(pa0 + stepA, nimg, 2); glds(pa1 + stepA, nimg, 3);
        mfma_row(2); glds(pb0, nimg + g3p::OPB, 0); glds(pb1, nimg + g3p::OPB, 1);
        mfma_row(3); glds(pb0 + stepB, nimg + g3p::OPB, 2); glds(pb1 + stepB, nimg + g3p::OPB, 3);
        if constexpr (PF) {
#pragma unroll
            for (int i = 4; i < 8; ++i) {
                mfma_row(i);
#pragma unroll
                for (int f = 0; f < 3; ++f) read1(img, 3 * (i - 4) + f);
            }
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 8; ++i) mfma_row1(i);
            __builtin_amdgcn_s_setprio(0);
        } else {
#pragma unroll
            for (int i = 4; i < 8; ++i) mfma_row(i);
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
            __builtin_amdgcn_sched_barrier(0);
            read_unit(img, 1);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 8; ++i) mfma_row(i);
            __builtin_amdgcn_s_setprio(0);
        }
        finish_stage();
    }
    if (s < S) {
        const char* img = smem + (s & 1) * g3p::SLOT;
        g3_wait_vm<0>();
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            read_unit(img, u);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < 8; ++i) mfma_row(i);
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
        }
        finish_stage();
    }
    if constexpr (AMX) {
        if (g.amax) {
            unsigned m = amx_run;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
            if (lane == 0 && m) atomicMax(g.amax, m << 16);
        }
    }
}

// ---------------------------------------------------------------------------------
// 8-phase ping-pong kernel for NT products (both operands k-contiguous: the MLP layers'
// forward and input-gradient GEMMs, the upsampling and GRU input projections' forward).
// The pair-mode LDS layout (two 64 KiB slots of 64-deep k-tiles, 128-B rows, XOR-swizzled
// 16-B slots) with the two wave groups X = waves 0-3 (output rows 0-127 of the tile) and
// Y = waves 4-7 (rows 128-255) one segment apart: every k-tile is 8 segments per group,
//      R0 | M0 | R1 | M1 | R2 | M2 | R3 | M3       (Y one segment behind X)
// Rp: the LDS reads of phase p (R0: the m-fragments 0-3 and n-fragments 0-1 of both 32-k
//     units, 12 ds_read_b128; R1: m 4-7, n 2-3), completed (lgkmcnt(0)) inside the
//     segment; R2 / R3 issue the A / B pieces of k-tile t + 2 into the slot k-tile t was
//     just read from (4 global_load_lds per wave each); R3 also waits (counted vmcnt) for
//     k-tile t + 1, whose reads start two segments later in both groups;
// Mp: one quadrant of the wave's 128 x 64 outputs (4 m x 2 n fragments x both k units =
//     16 v_mfma_f32_16x16x32_bf16).
// Every segment ends with a raw s_barrier, so while one group's waves wait on LDS reads or
// issue DMA, the other group's wave on the same SIMD runs its MFMAs.  A k-tile's DMA has
// ten segments (five phases) between its issue and the wait that needs it; the epilogue of
// a finished tile runs in the next k-tile's R0, its stores counted in R3's vmcnt.
// ---------------------------------------------------------------------------------
// Ping-pong mode: the pair-mode LDS layout (64-deep stages, 2 x 64 KiB slots) with the
// two waves of each SIMD working in opposite phases.  Waves 0-3 (X) and 4-7 (Y) each
// alternate a LOAD segment (12 fragment reads of one 32-deep k-unit into registers) and
// a COMPUTE segment (its 32 MFMAs of that unit), Y one segment behind X, so while one
// wave of a SIMD keeps the matrix pipe busy its partner fetches its next operands:
//      X:  L0 | C0 | L1 | C1 | L2 | ...
//      Y:  -- | L0 | C0 | L1 | C1 | ...
// with one raw s_barrier between segments.  X alone streams HBM -> LDS: in its LOAD
// segment of a stage's first unit it issues all 16 DMA pieces (of 64) of the next stage
// into the slot Y finished reading one segment earlier, and waits for them at the end of
// its COMPUTE segment of the stage's second unit, three segments later.  A finished tile's
// epilogue runs in the wave's next LOAD segment.
template <typename TO, bool KCA, bool KCB, bool SW>
__global__ __launch_bounds__(512, 1) void gemm3pp_kernel(Gemm3Args g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave & 1, wn = wave >> 1;
    const int grp = wave >> 2, wx = wave & 3;
    const int ntm = g.M / g3::BM, ntn = g.N / g3::BN;
    const int ntiles = ntm * ntn;
    const int nunits = ntiles * g.ksplit;
    const int G = gridDim.x;
    const int nmine = (nunits - (int)blockIdx.x + G - 1) / G;
    const int kslice = g.K / g.ksplit;
    const int nk = kslice / g3p::BK;
    const int S = nmine * nk;
    const bf16* A = reinterpret_cast<const bf16*>(g.A);
    const bf16* B = reinterpret_cast<const bf16*>(g.B);

    auto unit = [&](int i, int& m0, int& n0, int& kbeg) {
        const int v = (int)blockIdx.x + i * G;
        const int z = v / ntiles;
        const int t = g3_xcd_remap(v - z * ntiles, ntiles);
        m0 = (t / ntn) * g3::BM;
        n0 = (t % ntn) * g3::BN;
        kbeg = z * kslice;
    };

    floatx4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // X wave wx streams pieces c = 4 i + wx (i = 0..7) of each operand: pieces i and
    // i + 2 share the source swizzle and sit 8 pieces (64 rows / 16 k-rows) apart
    const int64_t stepA = KCA ? (int64_t)64 * g.lda : (int64_t)16 * g.lda;
    const int64_t stepB = KCB ? (int64_t)64 * g.ldb : (int64_t)16 * g.ldb;
    int iu = 0, kti = 0;
    const bf16* srcA[2];
    const bf16* srcB[2];
    auto set_src = [&]() {
        int m0, n0, kb;
        unit(iu, m0, n0, kb);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = 4 * i + wx;
            srcA[i] = g3p_src<KCA>(A, g.lda, m0, kb, c, lane);
            srcB[i] = g3p_src<KCB>(B, g.ldb, n0, kb, c, lane);
        }
    };
    auto koffA = [&](int kt) { return KCA ? (int64_t)kt * g3p::BK : (int64_t)kt * g3p::BK * g.lda; };
    auto koffB = [&](int kt) { return KCB ? (int64_t)kt * g3p::BK : (int64_t)kt * g3p::BK * g.ldb; };
    auto issue_stage = [&](char* img) {      // X waves only: 8 + 8 pieces of the next stage
        const int64_t oa = koffA(kti), ob = koffB(kti);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_global_load_lds(G3_GLB(srcA[i & 1] + oa + (i >> 1) * stepA),
                                             G3_LDS(img + (4 * i + wx) * 1024), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            __builtin_amdgcn_global_load_lds(G3_GLB(srcB[i & 1] + ob + (i >> 1) * stepB),
                                             G3_LDS(img + g3p::OPB + (4 * i + wx) * 1024), 16,
                                             0, 0);
        if (++kti == nk) {
            kti = 0;
            ++iu;
            if (iu < nmine) set_src();
        }
    };
    if (grp == 0) set_src();

    bf16x8 a[8], b[4];
    auto bar = []() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // prologue: stage 0 resident before anyone reads
    if (S > 0 && grp == 0) {
        issue_stage(smem);
        g3_wait_vm<0>();
    }
    bar();
    if (grp == 1) bar();                     // Y runs one segment behind
    int ic = 0, ktc = 0;
    bool epi = false;
    const int U = 2 * S;
    for (int u = 0; u < U; ++u) {
        const int st = u >> 1, h = u & 1;
        const char* img = smem + (st & 1) * g3p::SLOT;
        // ---- LOAD segment
        if (epi) {
            int m0, n0, kb;
            unit(ic - 1, m0, n0, kb);
            if (!(g.diag & 8)) g3_epilogue<TO, SW>(g, acc, m0, n0, wm, wn, lane, kb);
            epi = false;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = g3p_frag<KCB>(img + g3p::OPB, wn * 64 + j * 16, h, lane);
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = g3p_frag<KCA>(img, wm * 128 + i * 16, h, lane);
        if (grp == 0 && h == 0 && st + 1 < S && !(g.diag & 4))
            issue_stage(smem + ((st + 1) & 1) * g3p::SLOT);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar();
        // ---- COMPUTE segment
        __builtin_amdgcn_s_setprio(1);
        if (!(g.diag & 1)) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0)
                                   : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j][0] += (float)a[i][0] * (float)b[j][0];
        }
        __builtin_amdgcn_s_setprio(0);
        if (h == 1) {
            if (++ktc == nk) {
                ktc = 0;
                ++ic;
                epi = true;
            }
            // X: the next stage's DMA (issued three segments ago) lands before Y and X read it
            if (grp == 0 && !(g.diag & 2)) g3_wait_vm<0>();
        }
        bar();
    }
    if (grp == 0) bar();
    if (epi) {
        int m0, n0, kb;
        unit(ic - 1, m0, n0, kb);
        g3_epilogue<TO, SW>(g, acc, m0, n0, wm, wn, lane, kb);
    }
}

// ---------------------------------------------------------------------------------
// Ping-pong over the 32-deep ring (mode 4): the LOAD / COMPUTE alternation of the
// ping-pong kernel on the 5-slot ring of 32-deep stages, so the DMA can be spread: every
// wave issues its 4 pieces of stage u + NS - 1 in its LOAD segment of unit u (into the
// slot Y finished reading one segment earlier), and waits, counted, for stage v at the end
// of the segment before X reads it (X: its COMPUTE of v - 1; Y: its LOAD of v - 1).
template <typename TO, bool KCA, bool KCB, bool SW>
__global__ __launch_bounds__(512, 1) void gemm3q_kernel(Gemm3Args g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave & 1, wn = wave >> 1;
    const int grp = wave >> 2;
    const int ntm = g.M / g3::BM, ntn = g.N / g3::BN;
    const int ntiles = ntm * ntn;
    const int nunits = ntiles * g.ksplit;
    const int G = gridDim.x;
    const int nmine = (nunits - (int)blockIdx.x + G - 1) / G;
    const int kslice = g.K / g.ksplit;
    const int nk = kslice / g3::BK;
    const int S = nmine * nk;
    const bf16* A = reinterpret_cast<const bf16*>(g.A);
    const bf16* B = reinterpret_cast<const bf16*>(g.B);
    (void)ntm;

    auto unit = [&](int i, int& m0, int& n0, int& kbeg) {
        const int v = (int)blockIdx.x + i * G;
        const int z = v / ntiles;
        const int t = g3_xcd_remap(v - z * ntiles, ntiles);
        m0 = (t / ntn) * g3::BM;
        n0 = (t % ntn) * g3::BN;
        kbeg = z * kslice;
    };

    floatx4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    int iu = 0, kti = 0, isl = 0;        // issue cursor: unit, stage in unit, ring slot
    const bf16* srcA[g3::GLW];
    const bf16* srcB[g3::GLW];
    auto set_src = [&]() {
        int m0, n0, kb;
        unit(iu, m0, n0, kb);
#pragma unroll
        for (int i = 0; i < g3::GLW; ++i) {
            const int c = wave * g3::GLW + i;
            srcA[i] = g3_src<KCA>(A, g.lda, m0, kb, c, lane);
            srcB[i] = g3_src<KCB>(B, g.ldb, n0, kb, c, lane);
        }
    };
    set_src();
    auto issue_stage = [&]() {
        char* img = smem + isl * g3::SLOT;
        const int64_t oa = KCA ? (int64_t)kti * g3::BK : (int64_t)kti * g3::BK * g.lda;
        const int64_t ob = KCB ? (int64_t)kti * g3::BK : (int64_t)kti * g3::BK * g.ldb;
#pragma unroll
        for (int i = 0; i < g3::GLW; ++i)
            __builtin_amdgcn_global_load_lds(G3_GLB(srcA[i] + oa),
                                             G3_LDS(img + (wave * g3::GLW + i) * 1024), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < g3::GLW; ++i)
            __builtin_amdgcn_global_load_lds(G3_GLB(srcB[i] + ob),
                                             G3_LDS(img + g3::OPB + (wave * g3::GLW + i) * 1024),
                                             16, 0, 0);
        isl = isl == g3::NS - 1 ? 0 : isl + 1;
        if (++kti == nk) {
            kti = 0;
            ++iu;
            if (iu < nmine) set_src();
        }
    };
    constexpr int PER = 2 * g3::GLW;
    int issued = 0;                      // stages issued so far
#pragma unroll
    for (int st = 0; st < g3::NS - 1; ++st)
        if (st < S) {
            issue_stage();
            ++issued;
        }
    // wait until stage v of this wave has landed (stages > v may stay in flight)
    auto wait_stage = [&](int v) {
        if (!(g.diag & 2)) g3_wait_sel<PER, g3::NS - 2>(issued - 1 - v);
    };

    bf16x8 a[8], b[4];
    auto bar = []() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    if (S > 0) wait_stage(0);
    bar();                                 // stage 0 resident
    if (grp == 1) bar();                   // Y runs one segment behind
    int ic = 0, ktc = 0, rsl = 0;
    bool epi = false;
    for (int u = 0; u < S; ++u) {
        // ---- LOAD segment of unit u
        if (epi) {
            int m0, n0, kb;
            unit(ic - 1, m0, n0, kb);
            if (!(g.diag & 8)) g3_epilogue<TO, SW>(g, acc, m0, n0, wm, wn, lane, kb);
            epi = false;
        }
        {
            const char* ia = smem + rsl * g3::SLOT;
            const char* ib = ia + g3::OPB;
            rsl = rsl == g3::NS - 1 ? 0 : rsl + 1;
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = g3_frag<KCB>(ib, wn * 64 + j * 16, lane);
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] = g3_frag<KCA>(ia, wm * 128 + i * 16, lane);
        }
        if (issued < S && !(g.diag & 4)) {   // stage u + NS - 1 into the slot of u - 1
            issue_stage();
            ++issued;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (grp == 1 && u + 1 < S) wait_stage(u + 1);  // Y: before X's LOAD of u + 1
        bar();
        // ---- COMPUTE segment of unit u
        __builtin_amdgcn_s_setprio(1);
        if (!(g.diag & 1)) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = SW ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0)
                                   : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j][0] += (float)a[i][0] * (float)b[j][0];
        }
        __builtin_amdgcn_s_setprio(0);
        if (++ktc == nk) {
            ktc = 0;
            ++ic;
            epi = true;
        }
        if (grp == 0 && u + 1 < S) wait_stage(u + 1);  // X: before its LOAD of u + 1
        bar();
    }
    if (grp == 0) bar();
    if (epi) {
        int m0, n0, kb;
        unit(ic - 1, m0, n0, kb);
        if (!(g.diag & 8)) g3_epilogue<TO, SW>(g, acc, m0, n0, wm, wn, lane, kb);
    }
}

static int g3_mode() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("SRNN_G3MODE");
        v = e ? atoi(e) : 2;
    }
    return v;
}

static int g3_ncu() {
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        SRNN_CHECK_HIP(hipGetDevice(&dev));
        SRNN_CHECK_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    }
    return ncu;
}

// The 8-phase ping-pong NT kernel (gemm3e.hip) for plain / bias / ReLU / bits-out epilogues
// of NT products with K a multiple of 64, K >= 128 (SRNN_G3E=0: the pair-mode kernel)
static bool g3e_on() { return env_flag("SRNN_G3E", 0) != 0; }

template <typename TO, bool KCA, bool KCB, bool SW>
static int launch3(const Gemm3Args& g, hipStream_t s) {
    if constexpr (KCA && KCB && SW) {
        if (g3e_on()) {
            const int rc = srnn_gemm3e_launch(g, sizeof(TO) == 4, g3_ncu(), s);
            if (rc >= 0) return rc;
        }
    }
    // mode 0: 32-deep 5-slot ring; 1: 64-deep pair mode; 2 (default): pair mode when an
    // operand is k-contiguous (full-line DMA pieces), the ring otherwise
    const int mode = g3_mode();
    const bool k64 = (g.K / g.ksplit) % g3p::BK == 0;
    const bool pp = mode == 3 && k64;
    // mode 2 also takes the ring ping-pong for the NN shapes with enough tiles for two rounds
    // (A k-contiguous, B n-contiguous, plain output): measured on the step's upsampling
    // dX (32768 x 1024 x 16384: 1090 -> 900 us) and GRU dX (32768 x 1024 x 3072: 247 -> 204 us);
    // at one round of tiles (8192 x 1024 x 3072 / 4096) the pair mode stays ahead
    // (profiles/r04_gemm_modes_b512.txt)
    const int units = (g.M / g3::BM) * (g.N / g3::BN) * g.ksplit;
    const bool q = !g.csp && (mode == 4 ||
                   (mode == 2 && KCA && !KCB && g.ksplit == 1 && !g.mbi && !g.mbo && !g.amax &&
                    !g.mask && units >= 2 * g3_ncu() && env_flag("SRNN_G3_NNQ", 1)));
    const bool pair = !pp && !q && (mode == 1 || (mode == 2 && (KCA || KCB))) && k64;
    // unit-1 fragment prefetch (gemm3p PF): measured 14 % faster on the bf16 NT shapes (MLP
    // hidden forward, upsampling forward, B = 512), 3 % on NN; slower on the fp32-output NT
    // logits GEMM (N = 256), which keeps the plain schedule.  SRNN_G3_PF=0/1 overrides.
    const int pfe = env_flag("SRNN_G3_PF", -1);
    const bool pf = pfe >= 0 ? pfe != 0 : !(sizeof(TO) == 4 && KCA && KCB);
    auto k = q ? gemm3q_kernel<TO, KCA, KCB, SW>
               : pp ? gemm3pp_kernel<TO, KCA, KCB, SW>
                    : pair ? (pf ? gemm3p_kernel<TO, KCA, KCB, SW, false, true>
                                 : gemm3p_kernel<TO, KCA, KCB, SW>)
                           : gemm3_kernel<TO, KCA, KCB, SW>;
    int ki = q ? 3 : pp ? 2 : pair ? (pf ? 8 : 1) : 0;
    const bool grouped = g.mbi && g.ldmbi == 0;
    SRNN_REQUIRE(!grouped || (sizeof(TO) == 2 && SW && pair && !g.mbo &&
                              g.K / g.ksplit >= 2 * g3p::BK),
                 "gemm3: grouped mask bits need the bf16 pair-mode kernel and >= 2 k-chunks");
    if constexpr (sizeof(TO) == 2 && SW) {
        if (grouped) {               // grouped bits staged by LDS-DMA (+ max |C| for the dTab)
            // with the unit-1 fragment prefetch (SRNN_G3_BITS_PF=0: without): da1 1.11 -> 1.09
            // ms at B = 512 on one box (profiles/r05_da1_grouped_bits.txt)
            const bool bpf = env_flag("SRNN_G3_BITS_PF", 1) != 0;
            k = g.amax ? (bpf ? gemm3p_kernel<TO, KCA, KCB, SW, 2, true, true>
                              : gemm3p_kernel<TO, KCA, KCB, SW, 2, false, true>)
                       : gemm3p_kernel<TO, KCA, KCB, SW, 2>;
            ki = g.amax ? (bpf ? 15 : 14) : 13;
        } else if (g.mbi || g.mbo) { // ReLU bit masks (srnn_gemm3_try admits modes 0-2 only)
            k = pair ? gemm3p_kernel<TO, KCA, KCB, SW, true> : gemm3_kernel<TO, KCA, KCB, SW, true>;
            ki += 4;
        } else if (g.csp && pair) {   // column sums wanted (srnn_gemm_csum_next)
            k = pf ? gemm3p_kernel<TO, KCA, KCB, SW, 0, true, false, 1>
                   : gemm3p_kernel<TO, KCA, KCB, SW, 0, false, false, 1>;
            ki = pf ? 12 : 11;
        } else if (g.amax && pair) {  // max |C| wanted (srnn_gemm_amax_next)
            // (SRNN_G3_AMX_PF: with the unit-1 fragment prefetch as well)
            const int amx_pf = env_flag("SRNN_G3_AMX_PF", 0);
            k = amx_pf ? gemm3p_kernel<TO, KCA, KCB, SW, false, true, true>
                       : gemm3p_kernel<TO, KCA, KCB, SW, false, false, true>;
            ki = amx_pf ? 10 : 9;
        }
    }
    if constexpr (sizeof(TO) == 4 && SW && KCA && KCB) {
        if (g.lsm) {                 // row log-softmax in the epilogue (srnn_gemm_logsoftmax_next)
            SRNN_REQUIRE(pair && g.N == g3::BN && g.ksplit == 1,
                         "gemm3: the log-softmax epilogue needs one pair-mode tile column");
            k = gemm3p_kernel<TO, KCA, KCB, SW, 0, false, false, 0, 1>;
            ki = 16;
        }
    }
    SRNN_REQUIRE(!g.csp || pair, "gemm3: column sums need the pair-mode kernel");
    const int lds = (pp || pair) ? g3p::LDS + (grouped ? 16 * 1024 : g.lsm ? 8 * 1024 : 0)
                                 : g3::LDS;
    static bool attr[24] = {};
    if (!attr[ki]) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)k,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        attr[ki] = true;
    }
    const int ncu = g3_ncu();
    dim3 grid(units < ncu ? units : ncu);
    hipLaunchKernelGGL(k, grid, dim3(g3::NT), lds, s, g);
    SRNN_LAUNCH_CHECK();
    return 0;
}

template <typename TO, bool SW>
static int launch3_layout(const Gemm3Args& g, bool kca, bool kcb, hipStream_t s) {
    if (kca && kcb) return launch3<TO, true, true, SW>(g, s);
    if (kca && !kcb) return launch3<TO, true, false, SW>(g, s);
    if (!kca && kcb) return launch3<TO, false, true, SW>(g, s);
    return launch3<TO, false, false, SW>(g, s);
}

// Split-K factor for a plain fp32-out product: the power of two that minimises
// (rounds of 256 workgroups) x (k-stages per workgroup + epilogue allowance).
static int g3_pick_split(int tiles, int K) {
    int best = 1;
    double best_cost = 1e30;
    for (int ks = 1; ks <= 64; ks *= 2) {
        if (K % (ks * (ks > 1 ? g3p::BK : g3::BK)) || K / ks < 8 * g3::BK) break;
        const int rounds = (tiles * ks + 255) / 256;
        const double cost = rounds * (K / ks / (double)g3::BK + (ks > 1 ? 24.0 : 8.0));
        if (cost < best_cost * 0.97) {
            best_cost = cost;
            best = ks;
        }
    }
    return best;
}

// Returns -1 if the shape/layout is not eligible (caller falls back), else the status.
// force: take the path whenever eligible (tile == 5), else only when the 256-tile grid
// (with split-K) occupies the chip at least as well as the 128-tile kernel would.
// max |C| request for the next bf16-output GEMM that takes the gemm3 path (srnn_gemm_amax_next)
static unsigned*& g3_amax_pending() {
    static unsigned* p = nullptr;
    return p;
}
static int& g3_amax_taken() {
    static int t = 0;
    return t;
}
static bf16*& g3_blk_pending() {
    static bf16* p = nullptr;
    return p;
}

int srnn_gemm_amax_pending() { return g3_amax_pending() != nullptr; }

extern "C" int srnn_gemm_amax_next(unsigned* amax) {
    g3_amax_pending() = amax;
    g3_blk_pending() = nullptr;
    g3_amax_taken() = 0;
    return 0;
}

extern "C" int srnn_gemm_amax_blk_next(unsigned* amax, void* blk) {
    g3_amax_pending() = amax;
    g3_blk_pending() = (bf16*)blk;
    g3_amax_taken() = 0;
    return 0;
}

// column-sum request for the next bf16-output GEMM that takes the gemm3 pair path
static float*& g3_csum_pending() {
    static float* p = nullptr;
    return p;
}
static int& g3_csum_taken() {
    static int t = 0;
    return t;
}

int srnn_gemm_csum_pending() { return g3_csum_pending() != nullptr; }

extern "C" int srnn_gemm_csum_next(float* part) {
    g3_csum_pending() = part;
    g3_csum_taken() = 0;
    return 0;
}

// log-softmax request for the next fp32-output NT GEMM with N = 256 that takes the gemm3
// pair path (the SampleLevelMLP's logits)
static int& g3_lsm_pending() {
    static int p = 0;
    return p;
}
static int& g3_lsm_taken() {
    static int t = 0;
    return t;
}

int srnn_gemm_lsm_pending() { return g3_lsm_pending(); }

extern "C" int srnn_gemm_logsoftmax_next(void) {
    g3_lsm_pending() = 1;
    g3_lsm_taken() = 0;
    return 0;
}

extern "C" int srnn_gemm_logsoftmax_taken(void) {
    const int t = g3_lsm_taken();
    g3_lsm_pending() = 0;
    g3_lsm_taken() = 0;
    return t;
}

extern "C" int srnn_gemm_csum_taken(void) {
    const int t = g3_csum_taken();
    g3_csum_pending() = nullptr;
    g3_csum_taken() = 0;
    return t;
}

extern "C" int srnn_gemm_amax_taken(void) {
    const int t = g3_amax_taken();
    g3_amax_pending() = nullptr;
    g3_blk_pending() = nullptr;
    g3_amax_taken() = 0;
    return t;
}

int srnn_gemm3_try(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                   float alpha, const void* A, int64_t lda, const void* B, int64_t ldb,
                   float beta, const float* Cin, int64_t ldcin, void* C, int64_t ldc,
                   const float* bias, int bias_mode, int relu, const void* mask, int64_t ldmask,
                   int force, hipStream_t s, const unsigned short* mbi, int64_t ldmbi,
                   unsigned short* mbo, int64_t ldmbo) {
    if (dtype != SRNN_BF16) return -1;
    if ((mbi || mbo) && (out_dtype != SRNN_BF16 || g3_mode() > 2)) return -1;
    if ((mbi && ((uintptr_t)mbi % 8 || ldmbi % 4 || mask)) ||
        (mbo && ((uintptr_t)mbo % 8 || ldmbo % 4 || ldmbo == 0 || beta != 0.f)))
        return -1;
    // grouped bits in (ldmbi = 0): the pair-mode kernels only (an operand k-contiguous, K a
    // multiple of 64, modes 1-2); the caller's fallback expands them otherwise.  K >= 128:
    // the kernel stages tile iu's bits into buffer iu & 1 while issuing the previous tile's
    // LAST k-chunk, and with one chunk per tile (K = 64) that is the stage whose epilogue
    // still reads tile iu - 2's bits from the same buffer
    if (mbi && ldmbi == 0 &&
        (!(g3_mode() == 1 || (g3_mode() == 2 && (!transA || transB))) || K % g3p::BK ||
         K < 2 * g3p::BK || mbo || (uintptr_t)mbi % 16 || bias || relu || beta != 0.f))
        return -1;
    if (M % g3::BM || N % g3::BN || K % g3::BK || K == 0) return -1;
    auto al = [](const void* p, int64_t ld, int es) {
        return ((uintptr_t)p % 16 == 0) && ((ld * es) % 16 == 0);
    };
    if (!al(A, lda, 2) || !al(B, ldb, 2)) return -1;
    if ((uintptr_t)C % (out_dtype == SRNN_F32 ? 16 : 8) || ldc % 4) return -1;
    if (beta != 0.f && (!Cin || (uintptr_t)Cin % 16 || ldcin % 4)) return -1;
    if (mask && ((uintptr_t)mask % 8 || ldmask % 4)) return -1;
    if (bias && bias_mode == 1 && (uintptr_t)bias % 16) return -1;
    Gemm3Args g;
    g.A = A; g.B = B; g.C = C; g.Cin = Cin; g.bias = bias; g.mask = mask;
    g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldcin = ldcin; g.ldmask = ldmask;
    g.M = M; g.N = N; g.K = K; g.alpha = alpha; g.beta = beta;
    g.bias_mode = bias ? bias_mode : 0; g.relu = relu;
    g.diag = env_flag("SRNN_G3DIAG", 0);
    g.mbi = mbi; g.ldmbi = ldmbi; g.mbo = mbo; g.ldmbo = ldmbo;
    g.amax = nullptr;
    g.blk = nullptr;
    g.csp = nullptr;
    g.lsm = 0;
    const int tiles = (M / g3::BM) * (N / g3::BN);
    const bool plain = beta == 0.f && !bias && !relu && !mask && !mbi && !mbo &&
                       out_dtype == SRNN_F32;
    const int ks = plain ? g3_pick_split(tiles, K) : 1;
    if (!force) {
        const int64_t wg3 = (int64_t)tiles * ks;
        const int64_t wg2 = (int64_t)(M / 128) * (N / 128);
        // (measured: 96-128 tiles of 256 beat 384-512 of the 128-tile kernel on the TBPTT's
        //  top-tier NT projections, 2048 x 3072/4096 x 1024; 32 tiles do not)
        if (wg3 < 96 && wg2 > wg3) return -1;
    }
    g.ksplit = ks;
    g.part = nullptr;
    const bool det = ks > 1 && env_flag("SRNN_G3_SPLITK_PART", 1) && g3_mode() <= 2 &&
                     ldc % 4 == 0 && (uintptr_t)C % 16 == 0;
    if (ks > 1 && det) {
        // partial tiles in a grow-only scratch, then one ordered sum (no memset, no atomics)
        g.part = srnn_splitk_scratch((size_t)ks * M * N * sizeof(float));
        SRNN_REQUIRE(g.part, "gemm3: split-K scratch allocation failed");
    } else if (ks > 1) {
        if (ldc == N) {
            SRNN_CHECK_HIP(hipMemsetAsync(C, 0, (size_t)M * N * 4, s));
        } else {
            SRNN_CHECK_HIP(hipMemset2DAsync(C, ldc * 4, 0, (size_t)N * 4, M, s));
        }
    }
    const bool kca = !transA, kcb = transB;
    if (ks > 1) {
        const int rc = launch3_layout<float, false>(g, kca, kcb, s);
        if (rc || !g.part) return rc;
        return srnn_splitk_sum((const float*)g.part, (float*)C, ldc, M, N, ks, s);
    }
    if (out_dtype == SRNN_F32) {
        if (g3_lsm_pending() && N == g3::BN && g.ksplit == 1 && beta == 0.f && !mask && !mbi && !mbo &&
            (!bias || bias_mode == 1) && kca && kcb && K % g3p::BK == 0 &&
            (g3_mode() == 1 || g3_mode() == 2)) {
            g.lsm = 1;
            g3_lsm_pending() = 0;
            g3_lsm_taken() = 1;
        }
        return launch3_layout<float, true>(g, kca, kcb, s);
    }
    // max |C| (srnn_gemm_amax_next): computed by the pair-mode kernels (an operand
    // k-contiguous, K a multiple of 64, no bit masks) -- the request is taken only then
    if (g3_amax_pending() && beta == 0.f && (!mbi || ldmbi == 0) && !mbo && (kca || kcb) &&
        K % g3p::BK == 0 && g3_mode() <= 2 && (g3_mode() != 0)) {
        g.amax = g3_amax_pending();
        // the blocked copy needs whole 4-column blocks (N % 256 == 0 holds here); the grouped-
        // bits kernels write none (the caller sees taken == 1 and reads the row-major da1)
        g.blk = (mbi && ldmbi == 0) ? nullptr : g3_blk_pending();
        g3_amax_pending() = nullptr;
        g3_blk_pending() = nullptr;
        g3_amax_taken() = g.blk ? 2 : 1;
    }
    // column sums (srnn_gemm_csum_next): the pair-mode kernels' plain bf16 epilogue only
    // (no Cin, bit masks or max |C|); M % 128 == 0 holds here
    if (g3_csum_pending() && !g.amax && beta == 0.f && !mbi && !mbo && (kca || kcb) &&
        K % g3p::BK == 0 && (g3_mode() == 1 || g3_mode() == 2)) {
        g.csp = g3_csum_pending();
        g3_csum_pending() = nullptr;
        g3_csum_taken() = 1;
    }
    return launch3_layout<bf16, true>(g, kca, kcb, s);
}
