// The 8-phase ping-pong NT GEMM kernel (gemm3e_kernel) and its lean epilogue; shares the
// pair-mode LDS layout and argument block with gemm3.hip (gemm3_core.hpp).
#include "gemm3_core.hpp"

// LDS reads as inline asm: hipcc's waitcnt pass puts an s_waitcnt vmcnt(0) (the whole DMA
// queue) in front of plain LDS reads it cannot prove disjoint from the in-flight
// global_load_lds, which would retire k-tile t + 1 two phases early.  The reads' completion
// is then ordered only by the lgkmcnt(0) that names every destination as "+v".
template <int OFF>
__device__ __forceinline__ bf16x8 g3e_ds(unsigned a) {
    bf16x8 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF) : "memory");
    return v;
}
template <int OFF>
__device__ __forceinline__ floatx4 g3e_dsf(unsigned a) {
    floatx4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF) : "memory");
    return v;
}

// counted wait with a run-time count (the values gemm3e_kernel produces; anything else
// drains the queue, which is always safe)
__device__ __forceinline__ void g3e_wait_vm(int n) {
    switch (n) {
    case 8: g3_wait_vm<8>(); break;
    case 9: g3_wait_vm<9>(); break;
    case 16: g3_wait_vm<16>(); break;
    case 18: g3_wait_vm<18>(); break;
    case 24: g3_wait_vm<24>(); break;
    case 25: g3_wait_vm<25>(); break;
    case 26: g3_wait_vm<26>(); break;
    case 27: g3_wait_vm<27>(); break;
    case 32: g3_wait_vm<32>(); break;
    case 40: g3_wait_vm<40>(); break;
    case 41: g3_wait_vm<41>(); break;
    default: g3_wait_vm<0>(); break;
    }
}

// gemm3e's epilogue: C = act(alpha acc + bias) in TO, optionally the ReLU bits of the stored
// bf16 values (mbo, row-major).  No global loads at all -- the bias slice was staged in LDS by
// the kernel's DMA (bsa: this wave's 64 columns, or ~0u for none) -- so nothing here makes
// the compiler wait on the DMA queue.  Lane holds C[row][col .. col + 3] of each fragment
// (operands swapped in the MFMA).  Returns the number of stores (the main loop's vmcnt).
template <typename TO, bool MBO>
__device__ __forceinline__ int g3e_epilogue(const Gemm3Args& g, floatx4 (&acc)[8][4], int m0,
                                            int n0, int wm, int wn, int lane, unsigned bsa) {
    const int rbase = m0 + wm * 128 + (lane & 15);
    const int cbase = n0 + wn * 64 + (lane >> 4) * 4;
    floatx4 bc[4];
    if (bsa != ~0u) {
        const unsigned ba = bsa + (unsigned)((lane >> 4) * 16);
        bc[0] = g3e_dsf<0>(ba);
        bc[1] = g3e_dsf<64>(ba);
        bc[2] = g3e_dsf<128>(ba);
        bc[3] = g3e_dsf<192>(ba);
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(bc[0]), "+v"(bc[1]), "+v"(bc[2]), "+v"(bc[3])
                     :: "memory");
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) bc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    // ReLU as max(v, lo) without a branch: lo = 0, or NaN (max(v, NaN) = v, NaN passes)
    const float lo = g.relu ? 0.f : __builtin_nanf("");
    const float alpha = g.alpha;
    if constexpr (sizeof(TO) == 4) {
        float* Cp = reinterpret_cast<float*>(g.C);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                floatx4 v = acc[i][j] * alpha + bc[j];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], lo);
                acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
                *reinterpret_cast<floatx4*>(Cp + (int64_t)(rbase + i * 16) * g.ldc + cbase + j * 16) = v;
            }
        return 32;
    } else {
        bf16* Cp = reinterpret_cast<bf16*>(g.C);
        const int grp = lane >> 4, g4 = grp * 4;
        const int coff = 16 * (grp & 1) + 8 * (grp >> 1) - 4 * grp;   // lane's 16-B column
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            unsigned wbits[4][2];
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
                        floatx4 v = acc[i][j] * alpha + bc[j];
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], lo);
                        acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            typedef float g3f2 __attribute__((ext_vector_type(2)));
                            typedef __bf16 g3b2 __attribute__((ext_vector_type(2)));
                            const g3f2 pv = {v[2 * e], v[2 * e + 1]};
                            pk[t][e] = __builtin_bit_cast(unsigned, __builtin_convertvector(pv, g3b2));
                        }
                        if constexpr (MBO) {
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
                    *reinterpret_cast<uint4*>(Cp + (int64_t)row * g.ldc + cbase + 32 * jp + coff) =
                        make_uint4(pk[0][0], pk[0][1], pk[1][0], pk[1][1]);
                }
            }
            if constexpr (MBO) {
                // OR over the 4 lanes of a row (lane ^ 16, ^ 32), then lane group grp stores
                // row 4h + grp: one 8-B store per lane for the half's 4 rows
                unsigned sel[2] = {0u, 0u};
#pragma unroll
                for (int ii = 0; ii < 4; ++ii)
#pragma unroll
                    for (int w = 0; w < 2; ++w) {
                        unsigned lo, hi, x = wbits[ii][w];
                        xpair16(x, lo, hi);
                        x = lo | hi;
                        xpair32(x, lo, hi);
                        x = lo | hi;
                        if (ii == grp) sel[w] = x;
                    }
                *reinterpret_cast<uint2*>(g.mbo + (int64_t)(rbase + (4 * h + grp) * 16) * g.ldmbo +
                                          (n0 + wn * 64) / 16) = make_uint2(sel[0], sel[1]);
            }
        }
        return MBO ? 18 : 16;
    }
}

// ---------------------------------------------------------------------------------
// 8-phase ping-pong kernel for NT products (both operands k-contiguous: the MLP layers'
// forward, the upsampling and GRU input projections' forward) with a plain / bias / ReLU /
// ReLU-bits-out epilogue.  The pair-mode LDS layout (two 64 KiB slots of 64-deep k-tiles,
// 128-B rows, XOR-swizzled 16-B slots) with the two wave groups X = waves 0-3 (output rows
// 0-127 of the tile) and Y = waves 4-7 (rows 128-255) one segment apart: every k-tile is 8
// segments per group,
//      R0 | M0 | R1 | M1 | R2 | M2 | R3 | M3       (Y one segment behind X)
// Rp: the LDS reads of phase p (R0: the m-fragments 0-3 and n-fragments 0-1 of both 32-k
//     units, 12 ds_read_b128; R1: m 4-7, n 2-3), completed (lgkmcnt(0)) inside the
//     segment; R2 / R3 issue the A / B pieces of k-tile t + 2 into the slot k-tile t was
//     just read from (4 global_load_lds per wave each; with a tile's first k-tile also the
//     tile's bias slice, one 4-B-per-lane DMA per wave); R3 also waits (counted vmcnt) for
//     k-tile t + 1, whose reads start two segments later in both groups;
// Mp: one quadrant of the wave's 128 x 64 outputs (4 m x 2 n fragments x both k units =
//     16 v_mfma_f32_16x16x32_bf16).
// Every segment ends with a raw s_barrier, so while one group's waves wait on LDS reads or
// issue DMA, the other group's wave on the same SIMD runs its MFMAs.  A k-tile's DMA has
// ten segments (five phases) between its issue and the wait that needs it; the epilogue of
// a finished tile runs in the next k-tile's R0, its stores counted in R3's vmcnt.
// Needs K / 64 >= 2 (the bias buffer of tile i is rewritten for tile i + 2 two k-tiles
// before that tile starts).
namespace g3e {
constexpr int LDS = g3p::LDS + 4096;    // + 2 x 8 waves x 256 B of bias slices
}

template <typename TO, bool MBO>
__global__ __launch_bounds__(512, 1) void gemm3e_kernel(Gemm3Args g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int grp = wave >> 2;
    const int wm = grp, wn = wave & 3;
    const int ntm = g.M / g3::BM, ntn = g.N / g3::BN;
    const int ntiles = ntm * ntn;
    const int G = gridDim.x;
    const int nmine = (ntiles - (int)blockIdx.x + G - 1) / G;
    const int nk = g.K / g3p::BK;
    const int S = nmine * nk;
    const bf16* A = reinterpret_cast<const bf16*>(g.A);
    const bf16* B = reinterpret_cast<const bf16*>(g.B);
    const bool hasb = g.bias != nullptr;

    auto unit = [&](int i, int& m0, int& n0) {
        const int t = g3_xcd_remap((int)blockIdx.x + i * G, ntiles);
        m0 = (t / ntn) * g3::BM;
        n0 = (t % ntn) * g3::BN;
    };

    floatx4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    // DMA cursor: the k-tile (unit iu, k-step kti) whose pieces are issued next.  This wave
    // issues pieces wave * 4 .. + 3 of each operand (rows 32 wave .. + 31 of the k-tile image)
    // as buffer loads to LDS: the per-lane byte offset (row within the tile, swizzled 16-B
    // slot) does not depend on the tile, the tile's row / k offset is a scalar soffset -- one
    // VGPR per piece pair instead of 64-bit pointers (register pressure here spilled, and a
    // spill reload's vmcnt(0) drains the DMA queue).  Pieces c and c + 2 are 16 rows apart,
    // which keeps the row swizzle ((row >> 1) & 7)
    int iu = 0, kti = 0;
    const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16*>(A), (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16*>(B), (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(g.bias), (short)0, 0x7fffffff, 0x00020000);
    unsigned voA[2], voB[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = (wave * 4 + i) * 8 + (lane >> 3);
        const int slot = (lane & 7) ^ ((row >> 1) & 7);
        voA[i] = (unsigned)(((int64_t)row * g.lda + slot * 8) * 2);
        voB[i] = (unsigned)(((int64_t)row * g.ldb + slot * 8) * 2);
    }
    const unsigned vob = (unsigned)((wn * 64 + lane) * 4);
    unsigned soA = 0, soB = 0, sob = 0;            // the current unit's scalar offsets
    auto set_src = [&]() {
        int m0, n0;
        unit(iu, m0, n0);
        soA = (unsigned)((int64_t)m0 * g.lda * 2);
        soB = (unsigned)((int64_t)n0 * g.ldb * 2);
        sob = (unsigned)(n0 * 4);
    };
    set_src();
    const unsigned stA = (unsigned)(16 * g.lda * 2), stB = (unsigned)(16 * g.ldb * 2);
    auto issue_op = [&](const __amdgpu_buffer_rsrc_t& rs, const unsigned (&vo)[2], unsigned so,
                        unsigned st, char* img) {
        const unsigned s0 = so + (unsigned)(kti * g3p::BK * 2);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, G3_LDS(img + (wave * 4 + i) * 1024), 16, vo[i & 1], s0 + (i >> 1) * st, 0, 0);
    };
    // one k-tile's pieces (+ with a tile's first k-tile its bias slice); returns the DMAs
    auto issue_kt = [&](char* slot) -> int {
        issue_op(rsA, voA, soA, stA, slot);
        issue_op(rsB, voB, soB, stB, slot + g3p::OPB);
        int n = 8;
        if (hasb && kti == 0) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rsb, G3_LDS(smem + g3p::LDS + (iu & 1) * 2048 + wave * 256), 4, vob, sob, 0, 0);
            n = 9;
        }
        if (++kti == nk) {
            kti = 0;
            if (++iu < nmine) set_src();
        }
        return n;
    };
    // prologue: k-tiles 0 and 1 in flight, k-tile 0 landed
    if (S > 0) (void)issue_kt(smem);
    if (S > 1) {
        const int n1 = issue_kt(smem + g3p::SLOT);
        g3e_wait_vm(n1);
    } else {
        g3_wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (grp) __builtin_amdgcn_s_barrier();         // Y runs one segment behind X

    bf16x8 a[8][2], b[4][2];
    // per-lane part of a fragment read's LDS address (g3p_frag<true>): row l & 15 of the
    // fragment, 16-B slot (4 u + (l >> 4)) ^ ((row >> 1) & 7) -- the swizzle depends only on
    // the lane, as every fragment starts at a multiple of 16 rows
    const unsigned sm0 = (unsigned)(uintptr_t)G3_LDS(smem);
    unsigned lb[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
        lb[u] = (unsigned)((lane & 15) * 128 + (((u * 4 + (lane >> 4)) ^ ((lane >> 1) & 7)) * 16));
    int ic = 0, ktc = 0;                           // the k-tile being computed
    auto seg_end = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto quad = [&](int i0, int j0) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = i0; i < i0 + 4; ++i)
#pragma unroll
            for (int j = j0; j < j0 + 2; ++j)
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][u], a[i][u],
                                                                         acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        seg_end();
    };
    auto bias_lds = [&](int i) -> unsigned {
        return hasb ? sm0 + (unsigned)(g3p::LDS + (i & 1) * 2048 + wave * 256) : ~0u;
    };
    // segment order per k-tile s (Y one segment behind X; the reads of a segment complete
    // during the barrier that closes it, their lgkmcnt wait opens the MFMA segment):
    //   R0: the finished tile's epilogue, reads m 0-3 / n 0-1 | M0
    //   R1: reads m 4-7 / n 2-3 | M1          R2: - | M2
    //   R3: the pieces of k-tile s + 2 into k-tile s's slot (its reads retired >= 2 segments
    //       ago); wait for k-tile s + 1 (younger: the epilogue's stores, k-tile s + 2) | M3
    for (int s = 0; s < S; ++s) {
        int epi = 0;
        // ---- R0
        if (ktc == 0 && s > 0) {
            int m0, n0;
            unit(ic - 1, m0, n0);
            epi = g3e_epilogue<TO, MBO>(g, acc, m0, n0, wm, wn, lane, bias_lds(ic - 1));
        }
        const unsigned sb = sm0 + (unsigned)((s & 1) * g3p::SLOT);
        const unsigned aA0 = sb + (unsigned)(wm * 128 * 128) + lb[0], aA1 = aA0 - lb[0] + lb[1];
        const unsigned aB0 = sb + (unsigned)(g3p::OPB + wn * 64 * 128) + lb[0], aB1 = aB0 - lb[0] + lb[1];
#define G3E_RD_B(J) b[J][0] = g3e_ds<(J) * 2048>(aB0); b[J][1] = g3e_ds<(J) * 2048>(aB1);
#define G3E_RD_A(I) a[I][0] = g3e_ds<(I) * 2048>(aA0); a[I][1] = g3e_ds<(I) * 2048>(aA1);
#define G3E_WAIT(I0, J0)                                                                      \
        asm volatile("s_waitcnt lgkmcnt(0)"                                                   \
                     : "+v"(a[I0][0]), "+v"(a[I0][1]), "+v"(a[I0 + 1][0]), "+v"(a[I0 + 1][1]), \
                       "+v"(a[I0 + 2][0]), "+v"(a[I0 + 2][1]), "+v"(a[I0 + 3][0]),             \
                       "+v"(a[I0 + 3][1]), "+v"(b[J0][0]), "+v"(b[J0][1]), "+v"(b[J0 + 1][0]), \
                       "+v"(b[J0 + 1][1])                                                     \
                     :                                                                        \
                     : "memory");
        G3E_RD_B(0) G3E_RD_B(1) G3E_RD_A(0) G3E_RD_A(1) G3E_RD_A(2) G3E_RD_A(3)
        seg_end();
        G3E_WAIT(0, 0)
        __builtin_amdgcn_sched_barrier(0);
        quad(0, 0);                                    // M0
        // ---- R1
        G3E_RD_B(2) G3E_RD_B(3) G3E_RD_A(4) G3E_RD_A(5) G3E_RD_A(6) G3E_RD_A(7)
        seg_end();
        G3E_WAIT(4, 2)
        __builtin_amdgcn_sched_barrier(0);
#undef G3E_RD_A
#undef G3E_RD_B
#undef G3E_WAIT
        quad(0, 2);                                    // M1
        // ---- R2
        seg_end();
        quad(4, 2);                                    // M2
        // ---- R3
        int nis = 0;
        if (s + 2 < S) nis = issue_kt(smem + (s & 1) * g3p::SLOT);
        if (s + 1 < S) g3e_wait_vm(epi + nis);
        seg_end();
        quad(4, 0);                                    // M3
        if (++ktc == nk) {
            ktc = 0;
            ++ic;
        }
    }
    if (S > 0) {
        int m0, n0;
        unit(ic - 1, m0, n0);
        g3e_epilogue<TO, MBO>(g, acc, m0, n0, wm, wn, lane, bias_lds(ic - 1));
    }
    if (!grp) __builtin_amdgcn_s_barrier();        // X's barrier count meets Y's
}


int srnn_gemm3e_launch(const Gemm3Args& g, bool out_f32, int ncu, hipStream_t s) {
    // (buffer-load DMA: every operand byte offset below 2^31)
    if ((int64_t)g.M * g.lda * 2 >= (1ll << 31) || (int64_t)g.N * g.ldb * 2 >= (1ll << 31))
        return -1;
    if (g.ksplit != 1 || g.amax || g.csp || g.mbi || g.mask || g.blk || g.beta != 0.f ||
        g.bias_mode == 2 || (g.mbo && out_f32) || g.K % g3p::BK || g.K < 2 * g3p::BK || g.diag)
        return -1;
    const bool mb = g.mbo != nullptr;
    const void* k = out_f32 ? (const void*)gemm3e_kernel<float, false>
                  : mb      ? (const void*)gemm3e_kernel<bf16, true>
                            : (const void*)gemm3e_kernel<bf16, false>;
    const int ki = out_f32 ? 0 : mb ? 1 : 2;
    static bool attr[3] = {};
    if (!attr[ki]) {
        SRNN_CHECK_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, g3e::LDS));
        attr[ki] = true;
    }
    const int tiles = (g.M / g3::BM) * (g.N / g3::BN);
    Gemm3Args a = g;
    void* args[] = {&a};
    SRNN_CHECK_HIP(hipLaunchKernel(k, dim3(tiles < ncu ? tiles : ncu), dim3(g3::NT), args,
                                   g3e::LDS, s));
    return 0;
}
