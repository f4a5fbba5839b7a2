// Persistent sample loop of autoregressive generation (Generator.__call__, model.py:496-518):
// the SampleLevelMLP chain of FS0 consecutive samples (everything between two bottom-tier
// ticks) in ONE launch.
//
// Per sample i and row b the chain is strictly sequential:
//   a1 = relu(sum_k Tab[k][x_{i-FS0+k}] + up0[b][i % FS0])        (folded embedding . conv)
//   a2 = relu(W_hid a1 + b_hid)                                   (D x D)
//   z  = W_out a2 + b_out                                         (Q x D)
//   x_i = argmax(exp(log_softmax(z)) / q),  q ~ Exp(1)             (multinomial, model.py:514)
// The per-step kernel path (generate.hip) pays four dependent launches per sample.  Here:
//
// * Rows are split into groups of R (8 or 16) rows; the P = D / CW workgroups of a group
//   (CW = 64 columns each, 16 groups x 16 workgroups = 256 at B = 128, D = 1024: one per CU)
//   cooperate on that group only.  Workgroup p owns columns [p*CW, (p+1)*CW) of a1 and a2 and
//   Q/P logits.  Groups are blocks b with equal b % G, i.e. one XCD under round-robin dealing
//   (speed only; correctness never depends on placement).
// * Weights never move during the loop: each wave keeps its K-slice of the W_hid and W_out
//   columns of its workgroup as MFMA B fragments in VGPRs (64 + 16 VGPRs in bf16 at D = 1024),
//   and the newest-tap table slice Tab[FS0-1][:, cols] sits in LDS, so the sample -> a1 step
//   is an LDS gather.  The FS0-1 older taps + up0 are summed off the critical path while the
//   previous step's exchanges are in flight.
// * The three hand-offs per sample (a1, a2, z: every workgroup of the group needs every
//   column) are data-tagged 8-byte granules {value, tag = sample index} written by single
//   sc1 (write-through) stores and polled by sc1 loads (MI355X guide, Guideline 16 R2): no
//   flags, fences or barriers; a consumer spins on the data itself.  A buffer is only
//   rewritten after every consumer of its previous contents has produced a later result,
//   so a single buffer per hand-off suffices (see the note at gen_mlp_kernel).
// * Every workgroup of a group samples all R rows itself (the same logits, the same code:
//   identical indices), so the sampled index needs no hand-off; workgroup 0 writes seq/logp.
// * Spins are bounded: a lost hand-off sets the error word and the loop runs out instead of
//   hanging.
#include <algorithm>
#include <type_traits>

#include "samplernn_hip_internal.hpp"
#include "sampler.hpp"
#include "gen_mlp.hpp"
#include "handoff.hpp"

namespace gm {
constexpr int NW = 8;                  // waves per workgroup (the K split of both GEMMs)
constexpr int NTHR = NW * 64;
constexpr int Q = 256;
constexpr int HIST = 32;               // sample history ring per row (FS0 <= 32)
}  // namespace gm


#define GM_DIAG_WAVE0 (512 + 3 * 1024)

template <typename T> struct GmT;
template <> struct GmT<bf16> {
    static constexpr int GV = 2;       // values per granule
    static constexpr int UK = 32;      // k elements per MFMA unit (64 bytes)
    typedef bf16x8 frag;
};
template <> struct GmT<float> {
    static constexpr int GV = 1;
    static constexpr int UK = 16;
    typedef floatx4 frag;
};

__device__ __forceinline__ u64 gm_get(const u64* p) {
    return __hip_atomic_load(const_cast<u64*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename F>
__device__ __forceinline__ F gm_frag(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const uint4 u = make_uint4(a, b, c, d);
    F f;
    __builtin_memcpy(&f, &u, 16);
    return f;
}

template <typename F>
__device__ __forceinline__ F gm_load16(const void* p) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    F f;
    __builtin_memcpy(&f, &u, 16);
    return f;
}

template <typename T> __device__ __forceinline__ float gm_ld(const T* p) { return to_f(*p); }

__device__ __forceinline__ uint32_t gm_bits(float v) { return __float_as_uint(v); }
__device__ __forceinline__ uint32_t gm_bf16_bits(float v) {
    return (uint32_t)__bfloat16_as_ushort(__float2bfloat16(v));
}

// Hand-off images in fragment order.  A group's a1 / a2 buffer holds, for every MFMA k-unit
// u, the 4 granules each lane of a wave reads (row r < 8 = lane & 15, columns
// u UK + (lane >> 4) EPL ..) as two 16-B halves: granule index
//     (((u * 2 + half) * 4 + chunk) * 8 + r) * 2 + sub,
// so one poll instruction reads 512 B of whole lines (lanes of rows >= R read row R - 1's
// slots: the same addresses) instead of one half line per row.  Images are NU * 128 granules
// per group (= R * D / GV at R = 8, D % UK == 0).
template <typename T>
__device__ __forceinline__ uint32_t gm_slot(int r, int k) {
    constexpr int GV = GmT<T>::GV, UK = GmT<T>::UK, EPL = UK / 4;
    const int u = k / UK, kk = k - u * UK, c = kk / EPL, gi = (kk - c * EPL) / GV;
    return (uint32_t)((((u * 2 + (gi >> 1)) * 4 + c) * 8 + r) * 2 + (gi & 1));
}

// A-operand fragments of one wave for one hand-off buffer (the image of its group, starting
// at granule `gbase`; `rr` = the lane's row, clamped below R): for unit j (global unit
// u = wave + NW*j) the lane's 16 data bytes are 4 granules = two 16-B loads.  Spins until
// every tag == tag.  `work` (independent of the hand-off) runs once between the first poll's
// issue and its check, so it fills the hand-off's latency (the first check is straight-line
// code after it: its vmcnt leaves work's own loads in flight).
template <typename T, int UPW, typename W>
__device__ __forceinline__ void gm_fetch_a(__amdgpu_buffer_rsrc_t src, uint32_t gbase, int rr,
                                           bool rv, int wave, int lane, int NU, int D,
                                           uint32_t tag, uint32_t (&w)[UPW][4], int* err,
                                           W&& work) {
    constexpr int UK = GmT<T>::UK, EPL = UK / 4;
    uint4 x[UPW][2];
    // every load unconditional (clamped unit), so all 2 x UPW are in flight at once; a branch
    // per unit would put a vmcnt(0) between them
    const uint32_t lo = (gbase + (uint32_t)(((lane >> 4) * 8 + rr) * 2)) * 8u;
    auto issue = [&]() {
#pragma unroll
        for (int j = 0; j < UPW; ++j) {
            const int u = min(wave + gm::NW * j, NU - 1);
            const uint32_t off = lo + (uint32_t)u * (2u * 4 * 8 * 2 * 8);
            x[j][0] = hx_get2(src, off);
            x[j][1] = hx_get2(src, off + 4 * 8 * 2 * 8);
        }
    };
    auto check = [&]() -> bool {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < UPW; ++j) {
            const int u = wave + gm::NW * j;
            const bool v = rv && u < NU && u * UK + (lane >> 4) * EPL < D;
            w[j][0] = v ? x[j][0].x : 0u; w[j][1] = v ? x[j][0].z : 0u;
            w[j][2] = v ? x[j][1].x : 0u; w[j][3] = v ? x[j][1].z : 0u;
            ok &= !v || ((x[j][0].y == tag) & (x[j][0].w == tag) & (x[j][1].y == tag) &
                         (x[j][1].w == tag));
        }
        return __all(ok);
    };
    issue();
    work();
    if (check()) return;
    int spins = 0;
    for (;;) {
        if (hx_spin_fail(spins, err, lane)) return;
        issue();
        if (check()) return;
    }
}

// Note on single buffering: a1(i+1) is written only after its writer sampled x_i, i.e. after
// it read every z(i) granule of its group; each of those was written after its producer had
// read all of a2(i), which in turn came after every producer had read all of a1(i).  So when
// any a1(i+1) granule lands, a1(i) has been consumed by everyone; the same chain covers a2
// and z.  A consumer therefore only ever sees tag i-1 (keep polling) or tag i (done).
//
// Thread tid owns a1/a2 element (r, c) = (tid / CW, tid % CW) of its workgroup (R*CW <= 512).
template <typename T> __device__ __forceinline__ T gm_tap_load(__amdgpu_buffer_rsrc_t r, uint32_t off);
template <> __device__ __forceinline__ bf16 gm_tap_load<bf16>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __ushort_as_bfloat16(__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0));
}
template <> __device__ __forceinline__ float gm_tap_load<float>(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

// ---- in-launch tick GEMM (TG kernels) --------------------------------------------------
// up0 = A W^T + bias for all B (<= 128) rows; workgroup w takes 16-column tiles
// [w ntl / nblk, (w + 1) ntl / nblk) (<= TMAX of them).  Both operands stream through a 4-slot
// LDS ring of 64-deep k chunks by global_load_lds (128-B rows, 16-B slots XOR-swizzled by
// (row >> 1) & 7: conflict-free fragment reads), three chunks in flight, only the weight rows
// of the workgroup's own tiles staged; wave w owns output rows [16 w, 16 w + 16).  The MFMA runs with the operands swapped, so a lane holds 4 consecutive
// columns of one row: the epilogue is one 16-B write-through (sc1) store per tile.  The
// fragment reads are inline asm and every wait is counted by hand: the resident-fragment
// loads of the prologue are issued between the chunks and must stay in flight across them.
namespace gmt {
constexpr int KC = 64;                  // k per chunk
constexpr int ROWB = KC * 2;            // 128 B per staged row (8 x 16-B slots)
constexpr int TMAX = 5;                 // 16-column tiles per workgroup at most
constexpr int AROWS = 128;              // A rows staged (B <= 128; clamped)
constexpr int WROWS = 16 * TMAX;        // weight rows staged (the workgroup's tiles only)
constexpr int ASLOT = AROWS * ROWB, WSLOT = WROWS * ROWB;   // 16 / 10 KiB
constexpr int SLOT = ASLOT + WSLOT;
constexpr int NSL = 4;                  // ring slots: chunks ch + 1 .. ch + 3 in flight
constexpr int LDS = NSL * SLOT;
constexpr int PA = ASLOT / 1024 / gm::NW;      // A DMA pieces per wave per chunk (2)
constexpr int WORDS = 1280;             // grid-barrier words start at gerr + WORDS
}  // namespace gmt

#define GMT_LDS(p) ((__attribute__((address_space(3))) void*)(p))
#define GMT_GLB(p) ((const __attribute__((address_space(1))) void*)(p))

template <int N>
__device__ __forceinline__ void gmt_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
// vmcnt(n) for a wave-uniform count (0 .. 31; anything else waits for everything)
__device__ __forceinline__ void gmt_wait_n(int n) {
#define GMT_W(k) case k: gmt_wait_vm<k>(); break;
    switch (n) {
        GMT_W(1) GMT_W(2) GMT_W(3) GMT_W(4) GMT_W(5) GMT_W(6) GMT_W(7) GMT_W(8) GMT_W(9)
        GMT_W(10) GMT_W(11) GMT_W(12) GMT_W(13) GMT_W(14) GMT_W(15) GMT_W(16) GMT_W(17)
        GMT_W(18) GMT_W(19) GMT_W(20) GMT_W(21) GMT_W(22) GMT_W(23) GMT_W(24) GMT_W(25)
        GMT_W(26) GMT_W(27) GMT_W(28) GMT_W(29) GMT_W(30) GMT_W(31)
        default: gmt_wait_vm<0>(); break;
    }
#undef GMT_W
}

// Grid barrier of the TG kernels (MI355X guide, valid form R1): every storing thread drains
// its write-through stores, the workgroup joins, one lane publishes `epoch` (monotonic within
// a generate call) in its word, and wave 0 polls every word with sc1 loads; the other waves
// wait at the closing workgroup barrier.  Bounded by the co-residency wall-time guard
// (handoff.hpp): on a timeout (or another workgroup's error) the error word is raised and the
// launch runs out through the hand-off spins' checks.
__device__ __forceinline__ void gmt_grid_barrier(int* bar, int nblk, int epoch, int* err) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(bar + blockIdx.x, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        int polls = 0;
        for (;;) {
            bool done = true;
            for (int q = lane; q < nblk; q += 64)
                done &= __hip_atomic_load(bar + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
            if (__all(done)) break;
            __builtin_amdgcn_s_sleep(2);
            if ((++polls & 63) == 0) {
                if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > hx::ARRIVAL_TICKS) {
                    if (lane == 0)
                        __hip_atomic_fetch_max(err, hx::ERR_RESIDENCY, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
    }
    __syncthreads();
}

// FS0C: FS0 as a compile-time constant (0: runtime a.FS0).  DC: the whole launch shape as
// constants -- D = DC, R = 8, CW = 64, NZ = Q / (D / 64) (0: runtime); the per-unit validity
// masks of the runtime shape would otherwise be scalar-register spills in the loop.
// TG: the bottom tick's GEMM runs in this launch before the sample loop (GenMlpArgs::tg;
// bf16 only), with the prologue's resident-fragment loads in flight beside it.
template <typename T, int UPW, int NT, int NZT, int MAXT, int FS0C, int DC, bool TG = false>
__global__ __launch_bounds__(gm::NTHR, 2) void gen_mlp_kernel(GenMlpArgs a) {
    using F = typename GmT<T>::frag;
    constexpr int GV = GmT<T>::GV, UK = GmT<T>::UK, EPL = UK / 4;
    constexpr int Q = gm::Q;
    constexpr int HU = UPW > 4 ? 4 : UPW;
    static_assert(UPW % HU == 0, "gen_mlp: UPW must be a multiple of the fetch chunk");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int D = DC ? DC : a.D, R = DC ? 8 : a.R, CW = DC ? 64 : a.CW;
    const int NZ = DC ? gm::Q / (DC / 64) : a.NZ, B = a.B;
    const int FS0 = FS0C ? FS0C : a.FS0;
    // ---- group / member of this workgroup: static map, group g = block % G, member
    // p = block / G (one XCD per group under round-robin dealing); the placement check
    // (a.census, handoff.hpp) confirms it, and then the hand-offs stay in that XCD's L2.
    // (the 16-B word block at the very end of the dynamic LDS; no static __shared__: it would
    //  shift the 16-B alignment of the dynamic base)
    int* gsh = (int*)(smem + ((((size_t)gm::Q * CW * sizeof(T) + 15) & ~(size_t)15) +
                              (size_t)min(gm::NW, (D + UK - 1) / UK) *
                                  max(CW / 16, NZ / 16) * 32 * sizeof(floatx4) +
                              (size_t)R * gm::HIST * 4));
    // WOL (fp32, D = 1024): the W_out slice lives in LDS after the word block, rows padded to
    // D + 8 floats (conflict-free ds_read_b128 B fragments), instead of in 32 VGPRs
    constexpr bool WOL = std::is_same<T, float>::value && UPW > 4;
    const T* wol = (const T*)((char*)gsh + 16);
    const int p = blockIdx.x / a.G;
    const int c0 = p * CW, z0 = p * NZ;
    const int NU = (D + UK - 1) / UK;
    const int KW = min(gm::NW, NU);
    const int nt = CW / 16, nzt = NZ / 16, ntm = max(nt, nzt);
    const int DG = D / GV;
    const int XW = max(R * DG, ((D + UK - 1) / UK) * 128);   // granules per group image
    const T* __restrict__ tab = (const T*)a.tab;
    // optional phase timestamps (workgroup 0, thread 0; s_memrealtime = 100 MHz)
    unsigned long long* dg = (a.diag && blockIdx.x == 0 && tid == 0) ? a.diag : nullptr;
    unsigned long long* dgb = (a.diag && tid == 0 && blockIdx.x < 1024)
                                  ? a.diag + 512 + 3 * blockIdx.x : nullptr;
    if (dgb) dgb[0] = __builtin_amdgcn_s_memrealtime();
    int nd = 0;
#define GM_STAMP() do { if (dg && nd < 511) dg[nd++] = __builtin_amdgcn_s_memrealtime(); } while (0)
    // per-wave stamps of blocks 0 and G (group 0), steps 2..4 (timing diagnostics only)
    unsigned long long* dgw = (a.diag && lane == 0 && (blockIdx.x == 0 || blockIdx.x == a.G))
                                  ? a.diag + GM_DIAG_WAVE0 + ((blockIdx.x ? 8 : 0) + wave) * 64
                                  : nullptr;
#define GM_W(k) do { if (dgw && s >= 2 && s < 5) dgw[(s - 2) * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
    GM_STAMP();
    // LDS: [tab15 Q x CW][red KW x ntm x 32 floatx4][hist R x HIST][words][W_out slice (WOL)]
    T* tab15 = (T*)smem;
    size_t lo = ((size_t)Q * CW * sizeof(T) + 15) & ~(size_t)15;
    floatx4* red = (floatx4*)(smem + lo);
    lo += (size_t)KW * ntm * 32 * sizeof(floatx4);   // rows 0..7 of each 16 x 16 tile (R <= 8)
    int* hist = (int*)(smem + lo);
    const __amdgpu_buffer_rsrc_t rx1 = hx_rsrc(a.xa1), rx2 = hx_rsrc(a.xa2), rxz = hx_rsrc(a.xz);

    // ---- resident weights: B fragments of this wave's K units
    F wh[UPW][NT], wo[WOL ? 1 : UPW][NZT];
    // (loads from clamped addresses with no branches, so all of them are in flight at once;
    //  fragments outside the shape are zeroed afterwards)
    const int g = blockIdx.x % a.G;
    bool local;
    {
        int* cen = nullptr;
        if (a.census) {
            const int n = (*a.base + a.off - a.L) / FS0;          // launch index in this call
            cen = a.census + (n & 1) * HX_KEYED_WORDS;
            if (tid == 0) hx_group_arrive(cen + g * a.P + p);
            else if (blockIdx.x == 0 && wave == 1) {
                // zero the next launch's array (last used two launches ago)
                int* nxt = a.census + ((n + 1) & 1) * HX_KEYED_WORDS;
                for (int j = lane; j < HX_KEYED_WORDS; j += 64)
                    __hip_atomic_store(nxt + j, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        uint4 lw[UPW][NT], lz[WOL ? 1 : UPW][NZT];
        // fragment-order images (gen_mlp_prep_weights): the wave's 16 B per lane of (unit,
        // tile) are one contiguous KiB -- whole lines, where the (D, D) layout read 16 rows x
        // 64 B per instruction
        const uint4* fh = reinterpret_cast<const uint4*>(a.wfr_hid);
        const uint4* fo = reinterpret_cast<const uint4*>(a.wfr_out);
        const int nzt1 = nzt > 0 ? nzt : 1;
        auto ld_w = [&](int j, int t) {
            const int u = wave + gm::NW * j;
            const int uc = min(u, NU - 1);
            const int ke = min(u * UK + (lane >> 4) * EPL, D - EPL);
            const int n = min(c0 + t * 16 + (lane & 15), D - 1);
            // (TG: the images are required -- a load without a branch around it, which would
            //  make the wait analysis drain every load in flight at the join)
            if (TG || fh)
                lw[j][t] = fh[(((size_t)p * NU + uc) * nt + min(t, nt - 1)) * 64 + lane];
            else
                lw[j][t] = *reinterpret_cast<const uint4*>((const T*)a.w_hid + (int64_t)n * D + ke);
        };
        auto ld_z = [&](int j, int t) {
            if constexpr (!WOL) {
                const int u = wave + gm::NW * j;
                const int uc = min(u, NU - 1);
                const int ke = min(u * UK + (lane >> 4) * EPL, D - EPL);
                const int n = min(z0 + t * 16 + (lane & 15), Q - 1);
                if (TG || fo)
                    lz[j][t] = fo[(((size_t)p * NU + uc) * nzt1 + min(t, nzt1 - 1)) * 64 + lane];
                else
                    lz[j][t] = *reinterpret_cast<const uint4*>((const T*)a.w_out + (int64_t)n * D + ke);
            }
        };
        constexpr int PER = 16 / sizeof(T);
        const int cpr = CW / PER;                       // pieces per table row
        const int npc = Q * cpr;
        constexpr int MAXIT = gm::Q * 64 * (int)sizeof(T) / 16 / gm::NTHR;   // CW = 64: 4 / 8
        uint4 buf[MAXIT];
        auto ld_tab = [&](int it) {
            const int e = min(tid + it * gm::NTHR, npc - 1);
            const int q = e / cpr, c = (e % cpr) * PER;
            const T* src = tab + ((int64_t)(FS0 - 1) * Q + q) * D + c0 + c;
            if constexpr (TG) {
                // straight into the LDS slice (piece e at e * 16 B: this wave's 64 pieces of
                // round it are one contiguous KiB; npc is a multiple of the 512 threads here)
                __builtin_amdgcn_global_load_lds(
                    GMT_GLB(src), GMT_LDS(reinterpret_cast<char*>(tab15) +
                                          (size_t)(it * gm::NTHR + wave * 64) * 16),
                    16, 0, 0);
            } else {
                buf[it] = *reinterpret_cast<const uint4*>(src);
            }
        };
        // every resident-fragment / table load, in issue order
        constexpr int NLW = UPW * NT, NLZ = WOL ? 0 : UPW * NZT, NLD = NLW + NLZ + MAXIT;
        auto ld = [&](int i) {
            if (i < NLW) ld_w(i / NT, i % NT);
            else if (i < NLW + NLZ) ld_z((i - NLW) / NZT, (i - NLW) % NZT);
            else ld_tab(i - NLW - NLZ);
        };
        if constexpr (TG) {
            // ---- the bottom tick's GEMM (GenMlpArgs::tg), the fragment loads interleaved:
            // group c (4 loads, chunks 0 .. 6) is issued after chunk c + 3's DMA, so it is
            // younger than the chunk waited for next and lands while the GEMM runs (vmcnt is
            // in order)
            using namespace gmt;
            static_assert(DC == 1024 && NLD == 28, "TG: 7 groups of 4 loads over 16 chunks");
            constexpr int NCH = DC / KC;
            const int nblk = a.G * a.P;
            const int ntl = a.tg.N / 16;
            const int tb0 = (int)((int64_t)blockIdx.x * ntl / nblk);
            const int tb1 = (int)((int64_t)(blockIdx.x + 1) * ntl / nblk);
            const int nt = tb1 - tb0;                   // 1 .. TMAX (gen_mlp_tick_gemm_ok)
            // the tiles' bias, loaded before the ring (older than every chunk: no wait of its own)
            floatx4 bq[TMAX];
#pragma unroll
            for (int t = 0; t < TMAX; ++t)
                bq[t] = *reinterpret_cast<const floatx4*>(
                    a.tg.bias + max(min(tb0 + t, tb1 - 1), 0) * 16 + (lane >> 4) * 4);
            char* stg = reinterpret_cast<char*>(gsh) + 16;
            const bf16* asrc[PA];
#pragma unroll
            for (int i = 0; i < PA; ++i) {
                const int r = 8 * (wave * PA + i) + (lane >> 3);           // A row 0..127
                const int sl = (lane & 7) ^ ((r >> 1) & 7);
                asrc[i] = reinterpret_cast<const bf16*>(a.tg.A) + (int64_t)min(r, a.B - 1) * DC +
                          sl * 8;
            }
            // weight rows 0 .. 16 nt - 1 in 1-KiB pieces of 8 rows: piece wave + 8 i (i = 0, 1)
            // when it is one of the 2 nt (a wave-uniform count dW of 0 .. 2 per chunk)
            const int npw = 2 * nt;
            const int dW = (wave < npw ? 1 : 0) + (wave + gm::NW < npw ? 1 : 0);
            const bf16* wsrc[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int r = 8 * (wave + gm::NW * i) + (lane >> 3);     // weight row 0..79
                const int tile = max(min(tb0 + r / 16, tb1 - 1), 0);
                const int sl = (lane & 7) ^ ((r >> 1) & 7);
                wsrc[i] = reinterpret_cast<const bf16*>(a.tg.W) +
                          (int64_t)(tile * 16 + (r & 15)) * DC + sl * 8;
            }
            auto dma = [&](int ch) {
                char* slot = stg + (ch % NSL) * SLOT;
#pragma unroll
                for (int i = 0; i < PA; ++i)
                    __builtin_amdgcn_global_load_lds(GMT_GLB(asrc[i] + ch * KC),
                                                     GMT_LDS(slot + (wave * PA + i) * 1024), 16, 0, 0);
                if (wave < npw)
                    __builtin_amdgcn_global_load_lds(GMT_GLB(wsrc[0] + ch * KC),
                                                     GMT_LDS(slot + ASLOT + wave * 1024), 16, 0, 0);
                if (wave + gm::NW < npw)
                    __builtin_amdgcn_global_load_lds(
                        GMT_GLB(wsrc[1] + ch * KC),
                        GMT_LDS(slot + ASLOT + (wave + gm::NW) * 1024), 16, 0, 0);
            };
            floatx4 acc[TMAX];
#pragma unroll
            for (int t = 0; t < TMAX; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
            const unsigned lbase = (unsigned)(uintptr_t)GMT_LDS(stg);
            // issue order: DMA(0 .. NSL - 2); iteration ch: DMA(ch + NSL - 1), fragment group
            // ch (4 loads, ch < 7); a DMA is PA + dW loads of this wave
            constexpr int AH = NSL - 1;                 // chunks in flight
#pragma unroll
            for (int c = 0; c < AH; ++c) dma(c);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) {
                if (ch + AH < NCH) dma(ch + AH);
                if (ch < 7) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) ld(ch * 4 + i);
                }
                __builtin_amdgcn_sched_barrier(0);
                // chunk ch landed: count the loads issued after its DMA (compile-time counts of
                // DMAs nd and fragment groups nf after it)
                int nd = 0, nf = 0;
                if (ch < AH) {
                    nd = AH - 1 - ch;                   // the prologue's later DMAs
                    for (int i = 0; i <= ch; ++i) {
                        nd += i + AH < NCH ? 1 : 0;
                        nf += i < 7 ? 1 : 0;
                    }
                } else {
                    nf = ch - AH < 7 ? 1 : 0;           // its own iteration's fragment group
                    for (int i = ch - AH + 1; i <= ch; ++i) {
                        nd += i + AH < NCH ? 1 : 0;
                        nf += i < 7 ? 1 : 0;
                    }
                }
                gmt_wait_n(nd * (PA + dW) + nf * 4);
                // (raw barrier: __syncthreads would also drain vmcnt -- the fragment loads)
                __builtin_amdgcn_s_barrier();
                const unsigned sa = lbase + (unsigned)((ch % NSL) * SLOT);
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int j = u * 4 + (lane >> 4);
                    bf16x8 af, bfr[TMAX];
                    {
                        const int r = 16 * wave + (lane & 15);
                        const unsigned ad = sa + (unsigned)(r * ROWB + ((j ^ ((r >> 1) & 7)) * 16));
                        asm volatile("ds_read_b128 %0, %1" : "=v"(af) : "v"(ad) : "memory");
                    }
#pragma unroll
                    for (int t = 0; t < TMAX; ++t) {
                        const int r = t * 16 + (lane & 15);
                        const unsigned ad =
                            sa + (unsigned)(ASLOT + r * ROWB + ((j ^ ((r >> 1) & 7)) * 16));
                        asm volatile("ds_read_b128 %0, %1" : "=v"(bfr[t]) : "v"(ad) : "memory");
                    }
                    // the wait names the fragments as operands: the MFMAs that read them cannot
                    // be scheduled above it (the compiler does not know an asm LDS read is
                    // asynchronous)
                    static_assert(TMAX == 5, "TG: the wait below lists TMAX fragments");
                    asm volatile("s_waitcnt lgkmcnt(0)"
                                 : "+v"(af), "+v"(bfr[0]), "+v"(bfr[1]), "+v"(bfr[2]), "+v"(bfr[3]),
                                   "+v"(bfr[4])
                                 :
                                 : "memory");
#pragma unroll
                    for (int t = 0; t < TMAX; ++t)
                        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[t], af, acc[t], 0, 0, 0);
                }
                __builtin_amdgcn_s_barrier();      // slot ch % NSL is chunk ch + NSL's
                __builtin_amdgcn_sched_barrier(0);
            }
            GM_STAMP();                            // GEMM main loop done
            // epilogue: lane holds C[m][n .. n + 3] of each tile; 16-B write-through stores
            const int m = 16 * wave + (lane & 15);
            const __amdgpu_buffer_rsrc_t rcw =
                __builtin_amdgcn_make_buffer_rsrc(a.tg.C, (short)0, 0x7fffffff, 0x00020000);
            typedef unsigned int u32x4_ __attribute__((ext_vector_type(4)));
#pragma unroll
            for (int t = 0; t < TMAX; ++t) {
                if (t < tb1 - tb0 && m < a.B) {
                    const int n = (tb0 + t) * 16 + (lane >> 4) * 4;
                    __builtin_amdgcn_raw_buffer_store_b128(
                        __builtin_bit_cast(u32x4_, acc[t] + bq[t]), rcw,
                        (int)(((int64_t)m * a.tg.ldc + n) * 4), 0, 16 /* sc1 */);
                }
            }
            // every workgroup's part of up0 is out before any sample loop reads it
            const int epoch = (*a.base + a.off - a.L) / FS0 + 1;
            GM_STAMP();                            // epilogue stores issued
            gmt_grid_barrier(a.tg.bar, nblk, epoch, a.err);
            GM_STAMP();                            // grid barrier passed
        } else {
            // (the pre-TG order and form: per unit its W_hid then its W_out fragments)
#pragma unroll
            for (int j = 0; j < UPW; ++j) {
                const int u = wave + gm::NW * j;
                const int uc = min(u, NU - 1);
                const int ke = min(u * UK + (lane >> 4) * EPL, D - EPL);
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const int n = min(c0 + t * 16 + (lane & 15), D - 1);
                    lw[j][t] = fh ? fh[(((size_t)p * NU + uc) * nt + min(t, nt - 1)) * 64 + lane]
                                  : *reinterpret_cast<const uint4*>((const T*)a.w_hid + (int64_t)n * D + ke);
                }
                if constexpr (!WOL) {
#pragma unroll
                    for (int t = 0; t < NZT; ++t) {
                        const int n = min(z0 + t * 16 + (lane & 15), Q - 1);
                        lz[j][t] = fo ? fo[(((size_t)p * NU + uc) * nzt1 + min(t, nzt1 - 1)) * 64 + lane]
                                      : *reinterpret_cast<const uint4*>((const T*)a.w_out + (int64_t)n * D + ke);
                    }
                }
            }
        }
        if constexpr (WOL) {
            // rows z0 .. z0 + 15 of W_out into LDS (16-B pieces; NZ = 16 at D = 1024)
            const int pr = D / 4;
            for (int e = tid; e < 16 * pr; e += gm::NTHR) {
                const int n = e / pr, k = (e - n * pr) * 4;
                *reinterpret_cast<uint4*>((T*)wol + (size_t)n * (D + 8) + k) =
                    *reinterpret_cast<const uint4*>((const T*)a.w_out +
                                                    (int64_t)min(z0 + n, Q - 1) * D + k);
            }
        }
        if constexpr (!TG) {
            // the table slice after the W_out copy (its registers are not live across that
            // loop), an inline loop as before the TG kernels
#pragma unroll
            for (int it = 0; it < MAXIT; ++it) {
                const int e = min(tid + it * gm::NTHR, npc - 1);
                const int q = e / cpr, c = (e % cpr) * PER;
                buf[it] = *reinterpret_cast<const uint4*>(
                    tab + ((int64_t)(FS0 - 1) * Q + q) * D + c0 + c);
            }
        }
        // placement check (wave 0, after its own loads are in flight)
        if (wave == 0) {
            const int loc = cen && hx_group_local(cen + g * a.P, a.P, a.err, !a.nolocal) ? 1 : 0;
            if (tid == 0) {
                gsh[2] = loc;
                GM_STAMP();
                if (dgb) dgb[1] = __builtin_amdgcn_s_memrealtime();
            }
        }
        __syncthreads();
        local = gsh[2] != 0;
        if (dg) dg[511] = local ? 1 : 2;
#pragma unroll
        for (int j = 0; j < UPW; ++j) {
            const int u = wave + gm::NW * j;
            const bool kv = u < NU && u * UK + (lane >> 4) * EPL < D;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const bool v = kv && t < nt;
                wh[j][t] = gm_frag<F>(v ? lw[j][t].x : 0u, v ? lw[j][t].y : 0u,
                                      v ? lw[j][t].z : 0u, v ? lw[j][t].w : 0u);
            }
            if constexpr (!WOL) {
#pragma unroll
                for (int t = 0; t < NZT; ++t) {
                    const bool v = kv && t < nzt;
                    wo[j][t] = gm_frag<F>(v ? lz[j][t].x : 0u, v ? lz[j][t].y : 0u,
                                          v ? lz[j][t].z : 0u, v ? lz[j][t].w : 0u);
                }
            }
        }
        // newest-tap table slice (Q x CW, loaded in 16-B pieces above, before the census wait)
        // (clamped pieces store the same bytes to the same slot: no branch)
        if constexpr (!TG) {     // (TG: loaded straight into LDS, landed at the grid barrier)
#pragma unroll
            for (int it = 0; it < MAXIT; ++it) {
                const int e = min(tid + it * gm::NTHR, npc - 1);
                *reinterpret_cast<uint4*>(tab15 + (size_t)e * PER) = buf[it];
            }
        }
        GM_STAMP();
    }
    // ---- the sample history of this group's rows
    const int i0 = *a.base + a.off;
    for (int e = tid; e < R * FS0; e += gm::NTHR) {
        const int r = e / FS0, k = e % FS0;
        const int b = min(g * R + r, B - 1);
        const int j = i0 - FS0 + k;
        hist[r * gm::HIST + (j & (gm::HIST - 1))] = (int)a.seq[(int64_t)b * a.ldseq + j];
    }
    // this thread's a1/a2 element
    const bool own = tid < R * CW;
    // every wave's elements lie in the row that wave samples (r = wave)
    const bool row_wave = CW == 64 && R <= gm::NW;
    const int er = own ? tid / CW : 0, ec = own ? tid % CW : 0;
    const int eb = min(g * R + er, B - 1);
    const float bh = own ? a.b_hid[c0 + ec] : 0.f;
    const float bo = tid < R * NZ ? a.b_out[z0 + tid % NZ] : 0.f;
    // the next tick's gate operands that do not depend on this launch's samples, loaded now
    // (7 registers across the loop) so the gate update after it waits only for the LUT
    const int tr = tid / CW, tb = g * R + tr, tu = c0 + (tid - tr * CW);
    float tg[7];
    // (WOL: loaded after the loop instead -- 7 registers the fp32 loop cannot spare)
    auto load_tick = [&]() {
        const float* gr = a.tk->G + (int64_t)tb * a.tk->ldg;
        const float* hr = a.tk->gh + (int64_t)tb * a.tk->ldgh;
        tg[0] = gr[tu]; tg[1] = gr[D + tu]; tg[2] = gr[2 * D + tu];
        tg[3] = hr[tu]; tg[4] = hr[D + tu]; tg[5] = hr[2 * D + tu];
        tg[6] = a.tk->hp[(int64_t)tb * D + tu];
    };
    if (!WOL && a.tk && tr < R && tb < B && tu < D) {
        const float* gr = a.tk->G + (int64_t)tb * a.tk->ldg;
        const float* hr = a.tk->gh + (int64_t)tb * a.tk->ldgh;
        tg[0] = gr[tu]; tg[1] = gr[D + tu]; tg[2] = gr[2 * D + tu];
        if constexpr (TG) {     // gh: this launch's GEMM output (global sc1 loads, as up0;
                                // the pointer comes from memory, so force the global form)
            typedef __attribute__((address_space(1))) float gf;
            gf* hw = (gf*)const_cast<float*>(hr);
            tg[3] = __hip_atomic_load(hw + tu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            tg[4] = __hip_atomic_load(hw + D + tu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            tg[5] = __hip_atomic_load(hw + 2 * D + tu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            tg[3] = hr[tu]; tg[4] = hr[D + tu]; tg[5] = hr[2 * D + tu];
        }
        tg[6] = a.tk->hp[(int64_t)tb * D + tu];
    }
    __syncthreads();

    // partial a1 sum of sample i: up0 + the FS0-1 older taps.  issue_part puts every load in
    // flight (indices first, then table rows); finish_part sums them -- callers place other
    // work (the next hand-off wait) in between so the gathers' latency hides behind it.
    // The loads are unconditional (clamped tap index; unused taps re-read tap 0 and are
    // dropped by a select), so the compiler keeps them all in flight in one basic block.
    // (32-bit buffer offsets computed in VGPRs from the index: no per-tap 64-bit base
    //  address to keep live in scalar registers)
    T tv[MAXT];
    float upv = 0.f, part = 0.f;
    const __amdgpu_buffer_rsrc_t rtab =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(tab), (short)0, 0x7fffffff, 0x00020000);
    const uint32_t colb = (uint32_t)(c0 + ec) * (uint32_t)sizeof(T);
    auto issue_part = [&](int i) {
        int xs[MAXT];
#pragma unroll
        for (int k = 0; k < MAXT; ++k)
            xs[k] = hist[er * gm::HIST + ((i - FS0 + (k < FS0 - 1 ? k : 0)) & (gm::HIST - 1))];
#pragma unroll
        for (int k = 0; k < MAXT; ++k) {
            const uint32_t row = (uint32_t)xs[k] + (uint32_t)((k < FS0 - 1 ? k : 0) * Q);
            tv[k] = gm_tap_load<T>(rtab, row * (uint32_t)D * (uint32_t)sizeof(T) + colb);
        }
        if constexpr (TG) {
            // (TG: up0 was written in this launch by other workgroups, write-through: every
            //  load of it an sc1 load -- MI355X guide, valid forms)
            const float* up = a.up0 + (int64_t)eb * a.ldup + (int64_t)(i % FS0) * D + c0 + ec;
            upv = __hip_atomic_load(const_cast<float*>(up), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
        } else {
            upv = a.up0[(int64_t)eb * a.ldup + (int64_t)(i % FS0) * D + c0 + ec];
        }
    };
    auto finish_part = [&]() {
        float v = upv;
#pragma unroll
        for (int k = 0; k < MAXT; ++k) v += k < FS0 - 1 ? to_f(tv[k]) : 0.f;
        part = own ? v : 0.f;
    };
    // publish a1(i) = relu(part + Tab[FS0-1][x_{i-1}]) as granules tagged i (x = x_{i-1} of
    // this thread's row)
    auto publish_a1 = [&](int i, int x) {
        u64* dst = a.xa1 + (size_t)g * XW;
        float v = 0.f;
        if (own) v = fmaxf(part + to_f(tab15[x * CW + ec]), 0.f);
        if (GV == 2) {
            const uint32_t mine = gm_bf16_bits(v);
            const uint32_t nb = lane_next16(mine);
            if (own && (ec & 1) == 0) hx_put(dst + gm_slot<T>(er, c0 + ec), i, mine | (nb << 16), local);
        } else if (own) {
            hx_put(dst + gm_slot<T>(er, c0 + ec), i, gm_bits(v), local);
        }
    };

    GM_STAMP();
    if (dgb) dgb[2] = __builtin_amdgcn_s_memrealtime();
    issue_part(i0);
    finish_part();
    publish_a1(i0, hist[er * gm::HIST + ((i0 - 1) & (gm::HIST - 1))]);

    const int row = lane & 15;
    const bool rv = row < R;
    const int rr = min(row, R - 1);                 // (rows >= R read row R - 1's slots)
    const uint32_t gb1 = (uint32_t)((size_t)g * XW);
    for (int s = 0; s < a.nsteps; ++s) {
        const int i = i0 + s;
        const uint32_t tag = (uint32_t)i;
        GM_W(0);
        // ---------------- a2 = relu(W_hid a1 + b_hid), this workgroup's CW columns
        {
            floatx4 acc[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
            // the next sample's table gathers go in flight under the a1 hand-off
            // (WOL: after the a2 products instead -- the gathers' 15 registers would be live
            //  across them)
            auto work = [&]() { if (!WOL && s + 1 < a.nsteps) issue_part(i + 1); };
            if (wave >= KW) work();
            if (wave < KW) {
                // (HU units per fetch: at UPW = 8 -- fp32, D = 1024 -- the hand-off is read in
                //  two halves, so its load buffers fit beside the resident weights)
#pragma unroll
                for (int h = 0; h < UPW / HU; ++h) {
                    uint32_t w[HU][4];
                    if (h == 0)
                        gm_fetch_a<T, HU>(rx1, gb1, rr, rv, wave, lane, NU, D, tag, w, a.err, work);
                    else
                        gm_fetch_a<T, HU>(rx1, gb1, rr, rv, wave + gm::NW * HU * h, lane, NU, D, tag,
                                          w, a.err, [] {});
                    if (h == 0) GM_W(1);
#pragma unroll
                    for (int j = 0; j < HU; ++j) {
                        const F af = gm_frag<F>(w[j][0], w[j][1], w[j][2], w[j][3]);
#pragma unroll
                        for (int t = 0; t < NT; ++t) Mma<T>::run(acc[t], af, wh[h * HU + j][t]);
                    }
                }
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    if (t < nt && lane < 32) red[(wave * ntm + t) * 32 + lane] = acc[t];
            }
            if (WOL && s + 1 < a.nsteps) issue_part(i + 1);
            GM_W(2);
            GM_W(3);
            __syncthreads();
            GM_W(4);
            u64* dst = a.xa2 + (size_t)g * XW;
            float v = 0.f;
            if (own) {
                const int t = ec >> 4, ln = (er >> 2) * 16 + (ec & 15), ii = er & 3;
                float pr[gm::NW];
                #pragma unroll
                for (int kw = 0; kw < gm::NW; ++kw)
                    pr[kw] = red[(min(kw, KW - 1) * ntm + t) * 32 + ln][ii];
                #pragma unroll
                for (int kw = 0; kw < gm::NW; ++kw) v += kw < KW ? pr[kw] : 0.f;
                v = fmaxf(v + bh, 0.f);
            }
            if (GV == 2) {
                const uint32_t mine = gm_bf16_bits(v);
                const uint32_t nb = lane_next16(mine);
                if (own && (ec & 1) == 0)
                    hx_put(dst + gm_slot<T>(er, c0 + ec), tag, mine | (nb << 16), local);
            } else if (own) {
                hx_put(dst + gm_slot<T>(er, c0 + ec), tag, gm_bits(v), local);
            }
            GM_W(5);
            __syncthreads();                   // red is reused by the next phase
        }
        GM_W(6);
        // ---------------- z = W_out a2 + b_out, this workgroup's NZ logits
        {
            floatx4 acc[NZT];
#pragma unroll
            for (int t = 0; t < NZT; ++t) acc[t] = floatx4{0.f, 0.f, 0.f, 0.f};
            // ... and are summed under the a2 hand-off
            auto work = [&]() { if (s + 1 < a.nsteps) finish_part(); };
            if (wave >= KW) work();
            if (wave < KW) {
#pragma unroll
                for (int h = 0; h < UPW / HU; ++h) {
                    uint32_t w[HU][4];
                    if (h == 0)
                        gm_fetch_a<T, HU>(rx2, gb1, rr, rv, wave, lane, NU, D, tag, w, a.err, work);
                    else
                        gm_fetch_a<T, HU>(rx2, gb1, rr, rv, wave + gm::NW * HU * h, lane, NU, D, tag,
                                          w, a.err, [] {});
                    if (h == 0) GM_W(7);
#pragma unroll
                    for (int j = 0; j < HU; ++j) {
                        const F af = gm_frag<F>(w[j][0], w[j][1], w[j][2], w[j][3]);
#pragma unroll
                        for (int t = 0; t < NZT; ++t) {
                            if (t >= nzt) continue;
                            if constexpr (WOL) {
                                const int u = wave + gm::NW * (h * HU + j);
                                const int ke = u * UK + (lane >> 4) * EPL;
                                Mma<T>::run(acc[t], af,
                                            gm_load16<F>(wol + (size_t)(t * 16 + (lane & 15)) *
                                                                   (D + 8) + ke));
                            } else {
                                Mma<T>::run(acc[t], af, wo[h * HU + j][t]);
                            }
                        }
                    }
                }
#pragma unroll
                for (int t = 0; t < NZT; ++t)
                    if (t < nzt && lane < 32) red[(wave * ntm + t) * 32 + lane] = acc[t];
            }
            GM_W(8);
            __syncthreads();
            GM_W(9);
            for (int e = tid; e < R * NZ; e += gm::NTHR) {
                const int r = e / NZ, c = e % NZ;
                const int t = c >> 4, ln = (r >> 2) * 16 + (c & 15), ii = r & 3;
                float v = 0.f;
                float pr[gm::NW];
                #pragma unroll
                for (int kw = 0; kw < gm::NW; ++kw)
                    pr[kw] = red[(min(kw, KW - 1) * ntm + t) * 32 + ln][ii];
                #pragma unroll
                for (int kw = 0; kw < gm::NW; ++kw) v += kw < KW ? pr[kw] : 0.f;
                // (a row's logits in the order the draw reads them: lane l's z[4l .. 4l+1] at
                //  granule 2l, z[4l+2 .. 4l+3] at 128 + 2l: each poll reads 1 KiB of lines)
                const int zc = z0 + c;
                hx_put(a.xz + ((size_t)g * R + r) * Q + ((((zc & 3) >> 1) * 64 + (zc >> 2)) * 2 +
                                                         (zc & 1)), tag,
                       gm_bits(v + (e < gm::NTHR ? bo : a.b_out[z0 + c])), local);
            }
            GM_W(10);
            __syncthreads();
        }
        GM_W(11);
        // ---------------- sample x_i for every row of the group (one wave per row)
        int xw = 0;
        for (int r = wave; r < R; r += gm::NW) {
            const int b = g * R + r;
            const bool valid = b < B;
            const uint32_t zoff = (uint32_t)((((size_t)g * R + r) * Q + 2 * lane) * 8);
            floatx4 v;
            uint4 x0, x1;
            auto zcheck = [&]() -> bool {
                v = floatx4{__uint_as_float(x0.x), __uint_as_float(x0.z), __uint_as_float(x1.x),
                            __uint_as_float(x1.z)};
                return __all((x0.y == tag) & (x0.w == tag) & (x1.y == tag) & (x1.w == tag));
            };
            x0 = hx_get2(rxz, zoff);
            x1 = hx_get2(rxz, zoff + 1024);
            // the row's noise: precomputed by gen_noise_kernel (loaded under the z hand-off)
            // or drawn here, under the first poll
            floatx4 lq = floatx4{0.f, 0.f, 0.f, 0.f};
            if (valid)
                lq = a.lq ? *reinterpret_cast<const floatx4*>(a.lq + ((int64_t)s * B + b) * Q + 4 * lane)
                          : log_noise(sample_noise(a.noise, a.seed, B, b, i - a.L, lane, a.row0));
            if (!zcheck()) {
                int spins = 0;
                for (;;) {
                    if (hx_spin_fail(spins, a.err, lane)) break;
                    x0 = hx_get2(rxz, zoff);
                    x1 = hx_get2(rxz, zoff + 1024);
                    if (zcheck()) break;
                }
            }
            if (r == wave) GM_W(12);
            float* lrow = (p == 0 && valid && a.logp)
                              ? a.logp + ((int64_t)(i - a.L) * B + b) * Q : nullptr;
            const int x = sample_row(v, lq, lrow, lane);
            if (lane == 0) {
                hist[r * gm::HIST + (i & (gm::HIST - 1))] = x;
                if (p == 0 && valid) a.seq[(int64_t)b * a.ldseq + i] = x;
            }
            if (r == wave) xw = x;
        }
        GM_W(13);
        // ---------------- next sample's a1; the one after's gathers go in flight
        // (row-per-wave layout: this wave sampled its own elements' row, so a1(i+1) leaves
        //  before the barrier; otherwise the row's index comes from the history after it)
        if (row_wave && s + 1 < a.nsteps) publish_a1(i + 1, xw);
        GM_W(14);
        __syncthreads();
        GM_W(15);
        if (!row_wave && s + 1 < a.nsteps)
            publish_a1(i + 1, hist[er * gm::HIST + (i & (gm::HIST - 1))]);
        GM_STAMP();
    }
    // ---- the next bottom tick's gate update for this group's rows x this workgroup's
    // columns (the history now holds the FS0 samples it takes; same arithmetic and order as
    // fold_gru_kernel: gi = G + sum_s a_s Min[., s], a_s = 2 deq rounded to T)
    if (a.tk) {
        const GenMlpArgs::Tick* tk = a.tk;
        asm volatile("" : "+s"(tk));            // fresh loads of the table after the loop
        if (tr < R && tb < B && tu < D) {
            if (WOL) load_tick();
            const int inx = i0 + a.nsteps;
            const float* mr = tk->fmin + (int64_t)tu * 16;
            const float* mz = tk->fmin + (int64_t)(D + tu) * 16;
            const float* mn = tk->fmin + (int64_t)(2 * D + tu) * 16;
            floatx4 wr[4], wz[4], wn[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                wr[j] = *reinterpret_cast<const floatx4*>(mr + 4 * j);
                wz[j] = *reinterpret_cast<const floatx4*>(mz + 4 * j);
                wn[j] = *reinterpret_cast<const floatx4*>(mn + 4 * j);
            }
            float av[16];
#pragma unroll
            for (int s = 0; s < 16; ++s)
                av[s] = s < FS0 ? to_f(from_f<T>(tk->lut2[hist[tr * gm::HIST +
                                  ((inx - FS0 + s) & (gm::HIST - 1))]])) : 0.f;
            float gir = tg[0], giz = tg[1], gin = tg[2];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    gir += av[4 * j + e] * wr[j][e];
                    giz += av[4 * j + e] * wz[j][e];
                    gin += av[4 * j + e] * wn[j][e];
                }
            const float rg = 1.0f / (1.0f + expf(-(tg[3] + gir)));
            const float zg = 1.0f / (1.0f + expf(-(tg[4] + giz)));
            const float ng = tanhf(gin + tg[5] * rg);
            const float v = (tg[6] - ng) * zg + ng;
            tk->hn[(int64_t)tb * D + tu] = v;
            ((T*)tk->hn_lp)[(int64_t)tb * D + tu] = from_f<T>(v);
        }
    }
#undef GM_STAMP
#undef GM_W
}

// log q of the draws of nsteps generation steps, one wave per (step, row)
__global__ __launch_bounds__(256) void gen_noise_kernel(const float* __restrict__ noise,
                                                        uint64_t seed, int row0,
                                                        const int* __restrict__ base,
                                                        int off, int nsteps, int L, int B,
                                                        float* __restrict__ lq) {
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (idx >= nsteps * B) return;
    const int s = idx / B, b = idx - s * B;
    const int i = *base + off + s;
    *reinterpret_cast<floatx4*>(lq + ((int64_t)s * B + b) * gm::Q + 4 * lane) =
        log_noise(sample_noise(noise, seed, B, b, i - L, lane, row0));
}

int gen_noise_launch(const float* noise, uint64_t seed, int row0, const int* base, int off,
                     int nsteps, int L, int B, float* lq, hipStream_t s) {
    if (nsteps <= 0 || B <= 0) return 0;
    hipLaunchKernelGGL(gen_noise_kernel, dim3(cdiv((int64_t)nsteps * B, 4)), dim3(256), 0, s,
                       noise, seed, row0, base, off, nsteps, L, B, lq);
    SRNN_LAUNCH_CHECK();
    return 0;
}

// Fragment-order weight images: piece (p, u, t, lane) = 16 B of row p CW + t 16 + (lane & 15)
// (W_hid) or p NZ + t 16 + (lane & 15) (W_out, clamped to Q - 1), columns u UK + (lane >> 4)
// EPL .. (clamped to D - EPL), at index ((p NU + u) NT + t) 64 + lane.
__global__ void gen_wfrag_kernel(const char* __restrict__ w, int64_t ld_bytes, int rows_max,
                                 int P, int NU, int NT, int RPW, int UKB, int EPLB, int DB,
                                 uint4* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)P * NU * NT * 64;
    if (i >= total) return;
    const int lane = (int)(i & 63);
    const int64_t q = i >> 6;
    const int t = (int)(q % NT), u = (int)((q / NT) % NU), p = (int)(q / ((int64_t)NT * NU));
    const int row = min(p * RPW + t * 16 + (lane & 15), rows_max - 1);
    const int colb = min(u * UKB + (lane >> 4) * EPLB, DB - EPLB);
    dst[i] = *reinterpret_cast<const uint4*>(w + (int64_t)row * ld_bytes + colb);
}

// ------------------------------------------------------------------ host side
namespace {
typedef void (*GmKernel)(GenMlpArgs);

template <typename T, int MAXT, int FS0C>
GmKernel pick_t(int upw, int nzt) {
    if (upw <= 1 && nzt <= 16) return gen_mlp_kernel<T, 1, 4, 16, MAXT, FS0C, 0>;
    if (upw <= 2 && nzt <= 4) return gen_mlp_kernel<T, 2, 4, 4, MAXT, FS0C, 0>;
    if (upw <= 4 && nzt <= 2) return gen_mlp_kernel<T, 4, 4, 2, MAXT, FS0C, 0>;
    return nullptr;     // other fp32 shapes at D > 512 would spill their resident weights
}
// MAXT = older taps gathered per sample (FS0 - 1 <= MAXT)
template <typename T>
GmKernel pick(int upw, int nzt, int fs0, int D, int R) {
    // (FS0 = 16, the bottom frame of every published config, gets its own build: a
    //  constant FS0 folds the tap bookkeeping that would otherwise live in scalar registers;
    //  dim 1024 in bf16 -- the published model -- has its whole launch shape compiled in)
    if (std::is_same<T, bf16>::value && fs0 == 16 && D == 1024 && R == 8)
        return gen_mlp_kernel<T, 4, 4, 2, 15, 16, 1024>;
    // fp32 at dim 1024 (the reference's precision): 8 K units per wave, one 16-logit tile
    // whose W_out rows sit in LDS (WOL)
    if (std::is_same<T, float>::value && fs0 == 16 && D == 1024 && R == 8)
        return gen_mlp_kernel<T, 8, 4, 1, 15, 16, 1024>;
    if (fs0 == 16) return pick_t<T, 15, 16>(upw, nzt);
    return fs0 - 1 <= 15 ? pick_t<T, 15, 0>(upw, nzt) : pick_t<T, 31, 0>(upw, nzt);
}

int device_cus() {
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            ncu = 0;
    }
    return ncu;
}
}  // namespace

int gen_mlp_plan(int dtype, int B, int D, int FS0, int Q, GenMlpPlan* pl) {
    memset(pl, 0, sizeof(*pl));
    if (Q != gm::Q || FS0 < 1 || FS0 > gm::HIST || D % 16 || D > 1024 || B < 1) return 0;
    const int CW = D < 64 ? D : 64;
    if (D % CW) return 0;
    const int P = D / CW;
    const int NZ = Q / P;
    if (NZ % 16) return 0;
    const int UK = dtype == SRNN_BF16 ? 32 : 16;
    const int NU = (D + UK - 1) / UK;
    const int upw = (NU + gm::NW - 1) / gm::NW;
    int R = 0;
    for (int r : {8})          // one a1 element per thread: R * CW <= 512
        // every workgroup co-resident, for each process sharing the device (persist.hip)
        if (srnn_persist_fits_cus((int64_t)cdiv(B, r) * P)) { R = r; break; }
    if (!R) return 0;
    const GmKernel k = dtype == SRNN_BF16 ? pick<bf16>(upw, NZ / 16, FS0, D, R)
                                          : pick<float>(upw, NZ / 16, FS0, D, R);
    if (!k) return 0;
    // the in-launch tick GEMM variant (bf16, the compiled D = 1024 / FS0 = 16 shape);
    // SRNN_GEN_TICK_GEMM=0 keeps the bottom tick's GEMM a launch of its own
    pl->kernel_tg = nullptr;
    pl->lds_tg = 0;
    if (dtype == SRNN_BF16 && FS0 == 16 && D == 1024 && R == 8 && Q == gm::Q &&
        env_flag("SRNN_GEN_TICK_GEMM", 1))
        pl->kernel_tg = (const void*)gen_mlp_kernel<bf16, 4, 4, 2, 15, 16, 1024, true>;
    const int es = dtype == SRNN_BF16 ? 2 : 4;
    const int KW = NU < gm::NW ? NU : gm::NW;
    const int ntm = (CW / 16) > (NZ / 16) ? CW / 16 : NZ / 16;
    size_t lds = ((size_t)gm::Q * CW * es + 15) & ~(size_t)15;
    lds += (size_t)KW * ntm * 32 * 16;                // rows 0..7 of the 16-row tiles (R = 8)
    lds += (size_t)R * gm::HIST * 4;
    lds += 16;                                        // group / member / mode words
    if (dtype == SRNN_F32 && upw > 4)                 // W_out slice in LDS (gen_mlp_kernel WOL)
        lds += (size_t)NZ * (D + 8) * 4;
    if (lds > 160 * 1024) return 0;
    if (pl->kernel_tg) {
        pl->lds_tg = lds + gmt::LDS;
        if (pl->lds_tg > 160 * 1024) pl->kernel_tg = nullptr;
    }
    pl->ok = 1;
    pl->local = env_flag("SRNN_GEN_LOCAL", 1);
    pl->dtype = dtype;
    pl->R = R;
    pl->G = cdiv(B, R);
    pl->P = P;
    pl->CW = CW;
    pl->NZ = NZ;
    pl->lds = lds;
    pl->kernel = (const void*)k;
    const int GV = dtype == SRNN_BF16 ? 2 : 1;
    // fragment-order images: max(R D / GV, NU * 128) granules per group (gm_slot)
    pl->xa_words = (size_t)pl->G * std::max(R * (D / GV), NU * 128);
    pl->xz_words = (size_t)pl->G * R * Q;
    // fragment-order weight images (16 B per lane per (p, unit, tile)); the fp32 WOL form
    // keeps W_out in LDS and reads it row-wise
    const int nt = CW / 16, nzt = NZ / 16 > 0 ? NZ / 16 : 1;
    pl->wfr_hid_bytes = (size_t)P * NU * nt * 64 * 16;
    pl->wfr_out_bytes = (dtype == SRNN_F32 && upw > 4) ? 0 : (size_t)P * NU * nzt * 64 * 16;
    if (!env_flag("SRNN_GEN_WFRAG", 1)) pl->wfr_hid_bytes = pl->wfr_out_bytes = 0;
    if (!pl->wfr_hid_bytes || !pl->wfr_out_bytes) pl->kernel_tg = nullptr;   // (TG reads them)
    return 1;
}

int gen_mlp_prep_weights(const GenMlpPlan* pl, const void* w_hid, const void* w_out, int D,
                         int Q, void* fr_hid, void* fr_out, hipStream_t s) {
    const int es = pl->dtype == SRNN_BF16 ? 2 : 4;
    const int UK = pl->dtype == SRNN_BF16 ? 32 : 16;
    const int NU = (D + UK - 1) / UK;
    const int EPLB = UK / 4 * es;
    if (pl->wfr_hid_bytes && fr_hid) {
        const int nt = pl->CW / 16;
        const int64_t n = (int64_t)pl->P * NU * nt * 64;
        hipLaunchKernelGGL(gen_wfrag_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s,
                           (const char*)w_hid, (int64_t)D * es, D, pl->P, NU, nt, pl->CW,
                           UK * es, EPLB, D * es, (uint4*)fr_hid);
        SRNN_LAUNCH_CHECK();
    }
    if (pl->wfr_out_bytes && fr_out) {
        const int nzt = pl->NZ / 16 > 0 ? pl->NZ / 16 : 1;
        const int64_t n = (int64_t)pl->P * NU * nzt * 64;
        hipLaunchKernelGGL(gen_wfrag_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, s,
                           (const char*)w_out, (int64_t)D * es, Q, pl->P, NU, nzt, pl->NZ,
                           UK * es, EPLB, D * es, (uint4*)fr_out);
        SRNN_LAUNCH_CHECK();
    }
    return 0;
}

#define GM_DIAG_BLOCKS 1024
#define GM_DIAG_WORDS (GM_DIAG_WAVE0 + 16 * 64)
unsigned long long*& gm_diag_buf() {
    static unsigned long long* p = nullptr;
    return p;
}

extern "C" int srnn_gen_diag_dump(void) {
    static unsigned long long h[GM_DIAG_WORDS];
    if (!gm_diag_buf() || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(h, gm_diag_buf(), sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
        return 1;
    fprintf(stderr, "gen_mlp diag mode: %s\n", h[511] == 1 ? "xcd-local" : "static map");
    for (int k = 1; k < 511 && h[k]; ++k)
        fprintf(stderr, "gen_mlp diag %3d: +%8.2f us\n", k, (double)(h[k] - h[k - 1]) / 100.0);
    // per-workgroup start / group known / prologue done, relative to the earliest start
    unsigned long long t0 = ~0ull, smax = 0, cmax = 0, pmax = 0;
    int nb = 0;
    for (int b = 0; b < GM_DIAG_BLOCKS && h[512 + 3 * b]; ++b, ++nb) t0 = std::min(t0, h[512 + 3 * b]);
    for (int b = 0; b < nb; ++b) {
        smax = std::max(smax, h[512 + 3 * b] - t0);
        cmax = std::max(cmax, h[513 + 3 * b] - t0);
        pmax = std::max(pmax, h[514 + 3 * b] - t0);
    }
    fprintf(stderr, "gen_mlp diag %d blocks: last start +%.2f us, last group +%.2f us, "
            "last prologue +%.2f us\n", nb, smax / 100.0, cmax / 100.0, pmax / 100.0);
    // per-wave stamps (blocks 0 and G, steps 2..4), us relative to wave 0 of block 0 at the
    // step's start
    for (int st = 0; st < 3; ++st) {
        const unsigned long long t0w = h[GM_DIAG_WAVE0 + st * 16];
        if (!t0w) break;
        fprintf(stderr, "gen_mlp wave stamps, step %d (block 0 waves 0-7 | block G waves 0-7):\n", st + 2);
        for (int k = 0; k < 16; ++k) {
            fprintf(stderr, "  k=%2d", k);
            for (int w = 0; w < 16; ++w) {
                const unsigned long long v = h[GM_DIAG_WAVE0 + w * 64 + st * 16 + k];
                if (w == 8) fprintf(stderr, " |");
                if (v) fprintf(stderr, " %5.2f", ((double)v - (double)t0w) / 100.0);
                else fprintf(stderr, "     -");
            }
            fprintf(stderr, "\n");
        }
    }
    return 0;
}

int gen_mlp_tick_gemm_ok(const GenMlpPlan* pl, int N, int K, int B) {
    const int nblk = pl->G * pl->P;
    return pl->ok && pl->kernel_tg && K == 1024 && N % 16 == 0 && N / 16 >= nblk &&
           cdiv(N / 16, nblk) <= gmt::TMAX && B <= 128 && nblk <= 2048 - gmt::WORDS;
}

int gen_mlp_launch(const GenMlpPlan* pl, GenMlpArgs a, hipStream_t s) {
    SRNN_REQUIRE(pl && pl->ok, "gen_mlp: no plan");
    a.R = pl->R;
    a.G = pl->G;
    a.P = pl->P;
    a.CW = pl->CW;
    a.NZ = pl->NZ;
    // the census is the arrival gate (handoff.hpp) as well as the placement check: always on;
    // SRNN_GEN_LOCAL=0 only forces the global-mode hand-offs
    SRNN_REQUIRE(a.census && pl->G * pl->P <= HX_KEYED_WORDS, "gen_mlp: no census array");
    a.nolocal = pl->local ? 0 : 1;
    {
        // SRNN_GEN_DIAG=1: phase timestamps of the first launch into a device buffer that
        // srnn_gen_diag_dump prints (timing diagnostics only)
        // (SRNN_GEN_DIAG=n: the n-th launch of the process, so n > 1 skips the cold one)
        static unsigned long long* diag = nullptr;
        static int armed = -1;
        if (armed < 0) armed = env_flag("SRNN_GEN_DIAG", 0);
        // (allocated at the first launch, which runs eagerly, not inside a graph capture)
        if (armed >= 1 && !diag && hipMalloc(&diag, GM_DIAG_WORDS * 8) == hipSuccess)
            (void)hipMemset(diag, 0, GM_DIAG_WORDS * 8);
        if (armed >= 1 && diag && --armed == 0) {
            a.diag = diag;
            gm_diag_buf() = diag;
        }
    }
    const bool tg = a.tg.N > 0;
    if (tg) {
        SRNN_REQUIRE(pl->kernel_tg && a.wfr_hid && a.wfr_out,
                     "gen_mlp: no in-launch tick GEMM for this shape");
        SRNN_REQUIRE(gen_mlp_tick_gemm_ok(pl, a.tg.N, a.tg.K, a.B) && a.tg.ldc % 4 == 0 &&
                         a.tg.A && a.tg.W && a.tg.bias && a.tg.C,
                     "gen_mlp: tick GEMM shape (N %d, K %d, B %d) not supported", a.tg.N, a.tg.K,
                     a.B);
        a.tg.bar = a.err + gmt::WORDS;
    }
    const GmKernel k = (GmKernel)(tg ? pl->kernel_tg : pl->kernel);
    const size_t lds = tg ? pl->lds_tg : pl->lds;
    // raise the dynamic-LDS limit once per kernel (not inside a graph capture's launches)
    static const void* done[16];
    static size_t done_lds[16];
    int slot = 0;
    while (slot < 16 && done[slot] && done[slot] != (const void*)k) ++slot;
    if (slot == 16 || !done[slot] || done_lds[slot] < lds) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)k,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        if (slot < 16) { done[slot] = (const void*)k; done_lds[slot] = 160 * 1024; }
    }
    if (srnn_persist_check((const void*)k, gm::NTHR, lds, (int64_t)pl->G * pl->P, "gen_mlp"))
        return 1;
    hipLaunchKernelGGL(k, dim3(pl->G * pl->P), dim3(gm::NTHR), lds, s, a);
    SRNN_LAUNCH_CHECK();
    return 0;
}
