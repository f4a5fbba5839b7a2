// Small-tile MFMA core with a deep global_load_lds ring, for the latency-bound
// products of the hot path: the per-step GRU cell (B x 3D x D, forward and backward)
// and the M = batch projections of the generation loop.  These have K = 1024..3072 and
// only a few hundred output tiles, so the time of one workgroup is a chain of K stages;
// with the LDS ring NS-1 stages of both operands are in flight at once (one 256-B
// k-slab per row per stage, 16-B slots XOR-swizzled by row & 15 so the ds_read_b128
// fragment reads are bank-conflict free) instead of one register-prefetched stage.
// Both operands must be k-contiguous; rows are fetched through row maps (which must
// return an in-bounds row: out-of-range tile rows are clamped and their results
// discarded by the caller).  K must be a multiple of the stage (64 fp32 / 128 bf16).
#pragma once
#include "common.hpp"

#define RC_LDS(p) ((__attribute__((address_space(3))) void*)(p))
#define RC_GLB(p) ((const __attribute__((address_space(1))) void*)(p))

template <int N>
__device__ __forceinline__ void rc_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// wait until at most min(ahead, I) stages of PER loads each remain in flight
template <int PER, int I>
__device__ __forceinline__ void rc_wait_sel(int ahead) {
    if constexpr (I == 0) {
        rc_wait_vm<0>();
    } else {
        if (ahead >= I) rc_wait_vm<I * PER>();
        else rc_wait_sel<PER, I - 1>(ahead);
    }
}

struct RowClamp {
    int base, limit;
    __device__ __forceinline__ int operator()(int i) const {
        int r = base + i;
        return r < limit ? r : limit - 1;
    }
};

// GRU weight rows of tile row n: gate (n / U) * D + unit, units clamped to D - 1
struct RowGateClamp {
    int u0, U, D;
    __device__ __forceinline__ int operator()(int i) const {
        int g = i / U, j = i - g * U;
        int u = u0 + j;
        return g * D + (u < D ? u : D - 1);
    }
};

template <typename T, int BM, int BN, int WM, int WN, int WK, int NS>
struct Ring {
    static constexpr int KSB = 256;                        // bytes of k per row per stage
    static constexpr int KB = KSB / (int)sizeof(T);        // k per stage
    static constexpr int E = 16 / (int)sizeof(T);
    static constexpr int IA = BM * KSB / 1024 / 4;         // glds per wave per stage (A)
    static constexpr int IB = BN * KSB / 1024 / 4;
    static constexpr int SLOT = (BM + BN) * KSB;
    static constexpr int LDS = NS * SLOT;
    static constexpr int FM = BM / WM / 16;
    static constexpr int FN = BN / WN / 16;
    static constexpr int UPW = 4 / WK;                     // k-units per wave per stage
    static_assert(WM * WN * WK == 4, "4 waves");
    static_assert(IA * 4 * 1024 == BM * KSB && IB * 4 * 1024 == BN * KSB, "balanced issue");
    static_assert((NS - 2) * (IA + IB) <= 63, "vmcnt range");
    static constexpr int RED = (WK - 1) * WM * WN * FM * FN * 4 * 64 * 4;
};

template <typename T, int ROWS, int I, class Map, int AUX = 0>
__device__ __forceinline__ void rc_issue(const T* __restrict__ base, int64_t ld, Map map, int k0,
                                         char* img, int wave, int lane) {
    constexpr int E = 16 / (int)sizeof(T);
#pragma unroll
    for (int i = 0; i < I; ++i) {
        const int c = wave * I + i;
        const int row = c * 4 + (lane >> 4);
        const int slot = (lane & 15) ^ (row & 15);
        const T* src = base + (int64_t)map(row) * ld + k0 + slot * E;
        __builtin_amdgcn_global_load_lds(RC_GLB(src), RC_LDS(img + c * 1024), 16, 0, AUX);
    }
}

// acc += A[rows of tile] . B[rows of tile]^T over k in [0, K); ends with a barrier so
// the ring can be reused by a following call.  AUXB: cache policy of the B pieces (2 = nt,
// for weights that this workgroup alone reads, once).
template <typename T, int BM, int BN, int WM, int WN, int WK, int NS, class MapA, class MapB,
          int AUXB = 0>
__device__ __forceinline__ void ring_core(
    const T* __restrict__ A, int64_t lda, MapA mapA, const T* __restrict__ B, int64_t ldb,
    MapB mapB, int K, char* smem,
    floatx4 (&acc)[Ring<T, BM, BN, WM, WN, WK, NS>::FM][Ring<T, BM, BN, WM, WN, WK, NS>::FN],
    unsigned long long* stamp = nullptr) {
    typedef Ring<T, BM, BN, WM, WN, WK, NS> R;
    typedef typename Mma<T>::frag F;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave % WM, wn = (wave / WM) % WN, wk = wave / (WM * WN);
    const int nk = K / R::KB;
    auto issue = [&](int kt) {
        char* slot = smem + (kt % NS) * R::SLOT;
        rc_issue<T, BM, R::IA>(A, lda, mapA, kt * R::KB, slot, wave, lane);
        rc_issue<T, BN, R::IB, MapB, AUXB>(B, ldb, mapB, kt * R::KB, slot + BM * R::KSB, wave,
                                           lane);
    };
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nk) issue(s);
    const int lr = lane & 15, lh = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        rc_wait_sel<R::IA + R::IB, NS - 2>(nk - 1 - kt);
        if (stamp && kt < 30) stamp[1 + kt] = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_s_barrier();
        if (kt + NS - 1 < nk) issue(kt + NS - 1);
        const char* ia = smem + (kt % NS) * R::SLOT;
        const char* ib = ia + BM * R::KSB;
#pragma unroll
        for (int j = 0; j < R::UPW; ++j) {
            const int u = wk + WK * j;
            F a[R::FM], b[R::FN];
#pragma unroll
            for (int f = 0; f < R::FM; ++f) {
                const int r = wm * R::FM * 16 + f * 16 + lr;
                a[f] = *reinterpret_cast<const F*>(ia + r * R::KSB + (((u * 4 + lh) ^ (r & 15)) * 16));
            }
#pragma unroll
            for (int f = 0; f < R::FN; ++f) {
                const int r = wn * R::FN * 16 + f * 16 + lr;
                b[f] = *reinterpret_cast<const F*>(ib + r * R::KSB + (((u * 4 + lh) ^ (r & 15)) * 16));
            }
#pragma unroll
            for (int fm = 0; fm < R::FM; ++fm)
#pragma unroll
                for (int fn = 0; fn < R::FN; ++fn) Mma<T>::run(acc[fm][fn], a[fm], b[fn]);
        }
    }
    __syncthreads();
}

// Sum the WK partial accumulators into the wk == 0 waves (smem must hold R::RED bytes).
template <typename T, int BM, int BN, int WM, int WN, int WK, int NS>
__device__ __forceinline__ void ring_reduce(
    char* smem,
    floatx4 (&acc)[Ring<T, BM, BN, WM, WN, WK, NS>::FM][Ring<T, BM, BN, WM, WN, WK, NS>::FN]) {
    if constexpr (WK > 1) {
        typedef Ring<T, BM, BN, WM, WN, WK, NS> R;
        const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
        const int wmn = wave % (WM * WN), wk = wave / (WM * WN);
        floatx4* red = reinterpret_cast<floatx4*>(smem);
        if (wk > 0) {
#pragma unroll
            for (int fm = 0; fm < R::FM; ++fm)
#pragma unroll
                for (int fn = 0; fn < R::FN; ++fn)
                    red[(((wk - 1) * WM * WN + wmn) * R::FM * R::FN + fm * R::FN + fn) * 64 + lane] =
                        acc[fm][fn];
        }
        __syncthreads();
        if (wk == 0) {
#pragma unroll
            for (int w = 1; w < WK; ++w)
#pragma unroll
                for (int fm = 0; fm < R::FM; ++fm)
#pragma unroll
                    for (int fn = 0; fn < R::FN; ++fn)
                        acc[fm][fn] += red[(((w - 1) * WM * WN + wmn) * R::FM * R::FN + fm * R::FN +
                                            fn) * 64 + lane];
        }
        __syncthreads();
    }
}
