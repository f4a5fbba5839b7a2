// LDS-staged MFMA GEMM core for gfx950 (64-wide waves, 16x16 MFMA fragments).
//
// Tile BM x BN per 256-thread workgroup (4 waves laid out WM x WN x WK; WK > 1 splits
// each stage's k-units over waves and reduces through LDS at the end).  A stage holds
// KS "k-units" of 64 bytes per row (16 fp32 / 32 bf16), stored k-contiguous in LDS:
//      row stride RS = 64*KS + 16 bytes (16-byte pad breaks the 64-B row bank period),
// so fp32 (4 x v_mfma_f32_16x16x4_f32) and bf16 (v_mfma_f32_16x16x32_bf16) read their
// fragments with the same ds_read_b128 addressing.  Operands may be k-contiguous in
// global memory (row loads, 16-B vectors, optional row remap) or row-contiguous
// (vectors along rows, transposed into LDS on the write).  Out-of-range rows / k are
// zero-filled so edge tiles need no special MFMA path.  Global->register prefetch of
// stage t+1 overlaps the MFMAs of stage t (double-buffered LDS).
#pragma once
#include "common.hpp"

struct RowIdentity {
    int base, limit;
    __device__ __forceinline__ int operator()(int i) const {
        int r = base + i;
        return r < limit ? r : -1;
    }
};

// Rows of a GRU weight block: tile row n -> gate (n / U) * D + u0 + n % U.
struct RowGate {
    int u0, U, D;
    __device__ __forceinline__ int operator()(int i) const {
        int g = i / U, j = i - g * U;
        int u = u0 + j;
        return u < D ? g * D + u : -1;
    }
};

template <typename T, int ROWS, int KS, bool KC>
struct TileLoader {
    static constexpr int E = 16 / (int)sizeof(T);
    static constexpr int KB = KS * 64 / (int)sizeof(T);
    static constexpr int RS = 64 * KS + 16;
    static constexpr int NV = ROWS * KB / E;             // 16-B vectors per stage
    static constexpr int VT = (NV + 255) / 256;          // per thread
    uint4 v[VT];

    // KC: element (row, k) at p[grow(row) * ld + k]; !KC: at p[k * ld + r0 + row]
    template <class Map>
    __device__ __forceinline__ void load(const T* __restrict__ p, int64_t ld, int K, int k0,
                                         Map grow, int r0, int rlimit, bool vec_ok, int tid) {
#pragma unroll
        for (int j = 0; j < VT; ++j) {
            int vi = tid + 256 * j;
            uint4 val = make_uint4(0, 0, 0, 0);
            if (vi < NV) {
                if (KC) {
                    int row = vi / (KB / E), vk = vi % (KB / E);
                    int g = grow(row);
                    int k = k0 + vk * E;
                    if (g >= 0 && k < K) {
                        const T* src = p + (int64_t)g * ld + k;
                        if (vec_ok && k + E <= K) {
                            val = *reinterpret_cast<const uint4*>(src);
                        } else {
                            T tmp[E];
#pragma unroll
                            for (int e = 0; e < E; ++e) tmp[e] = (k + e < K) ? src[e] : from_f<T>(0.0f);
                            memcpy(&val, tmp, 16);
                        }
                    }
                } else {
                    int kk = vi / (ROWS / E), vr = vi % (ROWS / E);
                    int k = k0 + kk;
                    int r = r0 + vr * E;
                    if (k < K && r < rlimit) {
                        const T* src = p + (int64_t)k * ld + r;
                        if (vec_ok && r + E <= rlimit) {
                            val = *reinterpret_cast<const uint4*>(src);
                        } else {
                            T tmp[E];
#pragma unroll
                            for (int e = 0; e < E; ++e) tmp[e] = (r + e < rlimit) ? src[e] : from_f<T>(0.0f);
                            memcpy(&val, tmp, 16);
                        }
                    }
                }
            }
            v[j] = val;
        }
    }

    __device__ __forceinline__ void store(char* s, int tid) const {
#pragma unroll
        for (int j = 0; j < VT; ++j) {
            int vi = tid + 256 * j;
            if (vi < NV) {
                if (KC) {
                    int row = vi / (KB / E), vk = vi % (KB / E);
                    *reinterpret_cast<uint4*>(s + row * RS + vk * 16) = v[j];
                } else {
                    int kk = vi / (ROWS / E), vr = vi % (ROWS / E);
                    T tmp[E];
                    memcpy(tmp, &v[j], 16);
#pragma unroll
                    for (int e = 0; e < E; ++e)
                        *reinterpret_cast<T*>(s + (vr * E + e) * RS + kk * (int)sizeof(T)) = tmp[e];
                }
            }
        }
    }
};

template <typename T, int BM, int BN, int KS, int WM, int WN, int WK>
struct GemmCfg {
    static_assert(WM * WN * WK == 4, "4 waves");
    static_assert(KS % WK == 0, "k-units split evenly");
    static constexpr int RS = 64 * KS + 16;
    static constexpr int KB = KS * 64 / (int)sizeof(T);
    static constexpr int FM = BM / WM / 16;
    static constexpr int FN = BN / WN / 16;
    static constexpr int UPW = KS / WK;
    static constexpr int STAGE = (BM + BN) * RS;
    static constexpr int RED = (WK - 1) * WM * WN * FM * FN * 4 * 64 * 4;
    static constexpr int LDS = (2 * STAGE > RED) ? 2 * STAGE : RED;
};

template <typename T, int BM, int BN, int KS, int WM, int WN, int WK>
__device__ __forceinline__ void mma_stage(const char* sA, const char* sB,
                                          floatx4 (&acc)[GemmCfg<T, BM, BN, KS, WM, WN, WK>::FM]
                                                        [GemmCfg<T, BM, BN, KS, WM, WN, WK>::FN],
                                          int wm, int wn, int wk, int lane) {
    typedef GemmCfg<T, BM, BN, KS, WM, WN, WK> C;
    typedef typename Mma<T>::frag frag;
    const int lr = lane & 15, lq = (lane >> 4) * 16;
#pragma unroll
    for (int j = 0; j < C::UPW; ++j) {
        const int u = wk + WK * j;
        frag a[C::FM], b[C::FN];
#pragma unroll
        for (int fm = 0; fm < C::FM; ++fm)
            a[fm] = *reinterpret_cast<const frag*>(sA + (wm * C::FM * 16 + fm * 16 + lr) * C::RS +
                                                   u * 64 + lq);
#pragma unroll
        for (int fn = 0; fn < C::FN; ++fn)
            b[fn] = *reinterpret_cast<const frag*>(sB + (wn * C::FN * 16 + fn * 16 + lr) * C::RS +
                                                   u * 64 + lq);
#pragma unroll
        for (int fm = 0; fm < C::FM; ++fm)
#pragma unroll
            for (int fn = 0; fn < C::FN; ++fn) Mma<T>::run(acc[fm][fn], a[fm], b[fn]);
    }
}

// Accumulates op(A)[rows of tile] . op(B)[cols of tile]^T over k in [0, K) into acc.
// The caller zero-initialises acc.  smem must hold GemmCfg::LDS bytes (16-B aligned).
template <typename T, int BM, int BN, int KS, int WM, int WN, int WK, bool KCA, bool KCB,
          class MapA, class MapB>
__device__ __forceinline__ void gemm_core(const T* __restrict__ A, int64_t lda, MapA mapA, int am0,
                                          int alimit, bool vecA, const T* __restrict__ B,
                                          int64_t ldb, MapB mapB, int bn0, int blimit, bool vecB,
                                          int K, char* smem,
                                          floatx4 (&acc)[GemmCfg<T, BM, BN, KS, WM, WN, WK>::FM]
                                                        [GemmCfg<T, BM, BN, KS, WM, WN, WK>::FN]) {
    typedef GemmCfg<T, BM, BN, KS, WM, WN, WK> C;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wm = wave % WM, wn = (wave / WM) % WN, wk = wave / (WM * WN);
    TileLoader<T, BM, KS, KCA> la;
    TileLoader<T, BN, KS, KCB> lb;
    const int nt = (K + C::KB - 1) / C::KB;
    char* buf[2] = {smem, smem + C::STAGE};
    la.load(A, lda, K, 0, mapA, am0, alimit, vecA, tid);
    lb.load(B, ldb, K, 0, mapB, bn0, blimit, vecB, tid);
    la.store(buf[0], tid);
    lb.store(buf[0] + BM * C::RS, tid);
    __syncthreads();
    for (int kt = 0; kt < nt; ++kt) {
        const int cur = kt & 1;
        const bool more = kt + 1 < nt;
        if (more) {
            la.load(A, lda, K, (kt + 1) * C::KB, mapA, am0, alimit, vecA, tid);
            lb.load(B, ldb, K, (kt + 1) * C::KB, mapB, bn0, blimit, vecB, tid);
        }
        mma_stage<T, BM, BN, KS, WM, WN, WK>(buf[cur], buf[cur] + BM * C::RS, acc, wm, wn, wk,
                                             lane);
        if (more) {
            la.store(buf[cur ^ 1], tid);
            lb.store(buf[cur ^ 1] + BM * C::RS, tid);
        }
        __syncthreads();
    }
}

// Sum the WK partial accumulators into the wk == 0 wave (requires a prior barrier).
template <typename T, int BM, int BN, int KS, int WM, int WN, int WK>
__device__ __forceinline__ void wk_reduce(char* smem,
                                          floatx4 (&acc)[GemmCfg<T, BM, BN, KS, WM, WN, WK>::FM]
                                                        [GemmCfg<T, BM, BN, KS, WM, WN, WK>::FN]) {
    if (WK == 1) return;
    typedef GemmCfg<T, BM, BN, KS, WM, WN, WK> C;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int wmn = wave % (WM * WN), wk = wave / (WM * WN);
    floatx4* red = reinterpret_cast<floatx4*>(smem);
    if (wk > 0) {
#pragma unroll
        for (int fm = 0; fm < C::FM; ++fm)
#pragma unroll
            for (int fn = 0; fn < C::FN; ++fn)
                red[(((wk - 1) * WM * WN + wmn) * C::FM * C::FN + fm * C::FN + fn) * 64 + lane] =
                    acc[fm][fn];
    }
    __syncthreads();
    if (wk == 0) {
#pragma unroll
        for (int w = 1; w < WK; ++w)
#pragma unroll
            for (int fm = 0; fm < C::FM; ++fm)
#pragma unroll
                for (int fn = 0; fn < C::FN; ++fn)
                    acc[fm][fn] +=
                        red[(((w - 1) * WM * WN + wmn) * C::FM * C::FN + fm * C::FN + fn) * 64 + lane];
    }
}
