// Whole-sequence GRU recurrence in ONE persistent launch (forward of a FrameLevelRNN
// layer over all Fr frames, model.py:148-165 / torch.nn.GRU, gate order [r | z | n]).
//
// The per-step kernel (gru.hip) pays, every step, a launch boundary plus a fresh fetch of
// its 96 KiB W_hh slice and 64 KiB of h rows.  Here each of the 256 workgroups (64 unit
// tiles x 4 row tiles at B = 128, D = 1024; one per CU) keeps its W_hh slice RESIDENT in
// LDS for the whole sequence and per step only streams the 64 KiB of h_{t-1} rows of its
// row tile.  A step of row tile m may start once all unit tiles of m finished the previous
// one: a monotonic per-row-tile arrival counter.  The handed-off h rows are stored
// write-through (sc1) and read back by device-scope DMA, so no L2 write-back / invalidate
// fence sits in the loop; the spin is bounded (a workgroup that waits too long raises an
// error word and exits instead of hanging).
// The arithmetic (fragment order, k split over waves, reduction, gate epilogue) is the
// per-step ring kernel's, so both paths give identical bits.
#include "ring_core.hpp"
#include "gru_point.hpp"
#include "samplernn_hip_internal.hpp"

namespace gseq {
constexpr int BM = 32, BN = 48, WM = 2, WN = 1, WK = 2;
typedef Ring<bf16, BM, BN, WM, WN, WK, 2> R;      // geometry helpers only (KSB, IA, IB)
constexpr int MAXK = 1024;                         // D (k) supported: 8 stages of 128 bf16
constexpr int NSTAGE = MAXK / R::KB;
constexpr int WIMG = BN * R::KSB * NSTAGE;         // 96 KiB resident W_hh slice
constexpr int HIMG = BM * R::KSB * NSTAGE;         // 64 KiB h rows of one step
constexpr int LDS = WIMG + HIMG;                   // 160 KiB
constexpr long long SPIN_LIMIT = 1ll << 24;        // ~ seconds of polling (fits an int)
}  // namespace gseq

struct GruSeqArgs {
    const float* gi; int64_t ldgi; int64_t sgi;      // gi[b][t] = gi + b*ldgi + t*sgi (3D)
    const float* h0; const bf16* h0_lp;              // (B, D) initial state, fp32 + bf16
    const bf16* whh; const float* bhh;
    float* out; bf16* out_lp; int64_t ldo; int64_t so;       // out[b][t] = out + b*ldo + t*so
    float* gates; int64_t ldg; int64_t sg;                   // (4D per row and step)
    int* cnt;                          // step flags [row tile][64 unit tiles], zeroed
    int* err;
    int* sticky;                       // persist.hip flag, raised by a workgroup that gives up
    long long spin_limit;
    int withhold;                      // test switch: workgroup (0, 0) never publishes
    int B, D, Fr;
    int diag;          // timing diagnostics only (SRNN_GSEQ_DIAG): 1 no wait, 2 no h load,
                       // 4 no epilogue
};

// Wait until the n (<= 64) step flags of a row tile all reached `target`: one 256-B
// device-scope load per poll (lane i reads flag i), a ballot decides.  Flags are plain
// write-through stores of the step count -- no atomics serialising on one address.
__device__ __forceinline__ bool gseq_wait_flags(const int* flags, int n, int target, int* err,
                                                int* sticky, long long limit, int lane) {
    long long spins = 0;
    for (;;) {
        const int v = lane < n ? __hip_atomic_load(flags + lane, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)
                               : target;
        if (__builtin_amdgcn_ballot_w64(v < target) == 0) return true;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > limit) {
            if (lane == 0) {
                __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(sticky, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return false;
        }
        if ((spins & 63) == 0 &&
            __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            if (lane == 0) __hip_atomic_store(sticky, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
    }
}

// h rows of a step, device-scope (sc1) DMA reads: they see the other workgroups'
// write-through stores without an L2-invalidating acquire fence
__device__ __forceinline__ void gseq_issue_h(const bf16* __restrict__ base, int64_t ld,
                                             RowClamp map, int k0, char* img, int wave,
                                             int lane) {
    constexpr int I = gseq::R::IA;
#pragma unroll
    for (int i = 0; i < I; ++i) {
        const int c = wave * I + i;
        const int row = c * 4 + (lane >> 4);
        const int slot = (lane & 15) ^ (row & 15);
        const bf16* src = base + (int64_t)map(row) * ld + k0 + slot * 8;
        __builtin_amdgcn_global_load_lds(RC_GLB(src), RC_LDS(img + c * 1024), 16, 0, 16 /*sc1*/);
    }
}

// write-through (sc1) bf16 store: visible at device scope once the store has completed
__device__ __forceinline__ void gseq_store_wt(bf16* p, bf16 v) {
    const unsigned short bits = __bfloat16_as_ushort(v);
    asm volatile("global_store_short %0, %1, off sc1" ::"v"(p), "v"((unsigned)bits) : "memory");
}

__global__ __launch_bounds__(256, 1) void gru_seq_fwd_kernel(GruSeqArgs a) {
    using namespace gseq;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* wimg = smem;
    char* himg = smem + WIMG;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave % WM, wk = wave / (WM * WN);
    const int u0 = blockIdx.x * 16, m0 = blockIdx.y * BM;
    const int D = a.D, nk = D / R::KB;
    const int nunits = gridDim.x;
    const RowGateClamp gmap{u0, 16, D};
    const RowClamp hmap{m0, a.B};

    // resident W_hh slice: stage s of the image = k-range [s*KB, (s+1)*KB)
    for (int s = 0; s < nk; ++s)
        rc_issue<bf16, BN, R::IB>(a.whh, D, gmap, s * R::KB, wimg + s * BN * R::KSB, wave, lane);

    const int lr = lane & 15, lh = lane >> 4;
    const int u = u0 + lr;
    const int uc = min(u, D - 1);
    const float bhr = a.bhh[uc], bhz = a.bhh[D + uc], bhn = a.bhh[2 * D + uc];
    // the epilogue lanes keep their h_{t-1} values in registers across steps
    const bool epi = wk == 0 && u < D;
    float hprev[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = min(m0 + wm * 16 + lh * 4 + i, a.B - 1);
        hprev[i] = epi ? a.h0[(int64_t)row * D + uc] : 0.f;
    }
    for (int t = 0; t < a.Fr; ++t) {
        // this step's input projections, loaded before the h rows so that waiting for the
        // h pieces (younger in the vmcnt queue) also covers them
        float gir[4], giz[4], gin[4];
        if (epi) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = min(m0 + wm * 16 + lh * 4 + i, a.B - 1);
                const float* g = a.gi + (int64_t)row * a.ldgi + (int64_t)t * a.sgi;
                gir[i] = g[u]; giz[i] = g[D + u]; gin[i] = g[2 * D + u];
            }
        }
        if (t > 0 && !(a.diag & 1)) {
            // every wave polls for itself (all 160 KiB of LDS hold operands, no room for a
            // broadcast word); the counter is monotonic, so all waves reach the same verdict
            if (!gseq_wait_flags(a.cnt + blockIdx.y * 64, nunits, t, a.err, a.sticky, a.spin_limit,
                                 lane))
                return;
        }
        // h_{t-1} rows of this row tile (bf16)
        const bf16* hsrc = t == 0 ? a.h0_lp : a.out_lp + (int64_t)(t - 1) * a.so;
        const int64_t ldh = t == 0 ? (int64_t)D : a.ldo;
        if (!(a.diag & 2) || t == 0)
            for (int s = 0; s < nk; ++s)
                gseq_issue_h(hsrc, ldh, hmap, s * R::KB, himg + s * BM * R::KSB, wave, lane);
        floatx4 acc[1][3];
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[0][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < nk; ++kt) {
            // the stage's h pieces (and everything issued before them)
            rc_wait_sel<R::IA, NSTAGE - 1>(nk - 1 - kt);
            __builtin_amdgcn_s_barrier();
            const char* ia = himg + kt * BM * R::KSB;
            const char* ib = wimg + kt * BN * R::KSB;
#pragma unroll
            for (int j = 0; j < R::UPW; ++j) {
                const int uu = wk + WK * j;
                const int ra = wm * 16 + lr;
                const bf16x8 av = *reinterpret_cast<const bf16x8*>(
                    ia + ra * R::KSB + (((uu * 4 + lh) ^ (ra & 15)) * 16));
#pragma unroll
                for (int f = 0; f < 3; ++f) {
                    const int rb = f * 16 + lr;
                    const bf16x8 bv = *reinterpret_cast<const bf16x8*>(
                        ib + rb * R::KSB + (((uu * 4 + lh) ^ (rb & 15)) * 16));
                    Mma<bf16>::run(acc[0][f], av, bv);
                }
            }
        }
        __syncthreads();                       // h image free: reused by the reduction
        ring_reduce<bf16, BM, BN, WM, WN, WK, 2>(himg, acc);
        float hn[4], rr[4], zz[4], nn[4], gn[4];
        if (epi && !(a.diag & 4)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float ghr = acc[0][0][i] + bhr;
                const float ghz = acc[0][1][i] + bhz;
                const float ghn = acc[0][2][i] + bhn;
                const float r = 1.0f / (1.0f + expf(-(ghr + gir[i])));
                const float z = 1.0f / (1.0f + expf(-(ghz + giz[i])));
                const float n = tanhf(gin[i] + ghn * r);
                hn[i] = (hprev[i] - n) * z + n;
                rr[i] = r; zz[i] = z; nn[i] = n; gn[i] = ghn;
                hprev[i] = hn[i];
                const int row = m0 + wm * 16 + lh * 4 + i;
                if (row < a.B)     // the row tile's next step reads these: write-through first
                    gseq_store_wt(a.out_lp + (int64_t)row * a.ldo + (int64_t)t * a.so + u,
                                  from_f<bf16>(hn[i]));
            }
        }
        // publish step t of this tile: the bf16 h stores completed, then one arrival (no L2
        // write-back fence: the handed-off bytes are already coherent)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0 && !(a.withhold && blockIdx.x == 0 && blockIdx.y == 0))
            __hip_atomic_store(a.cnt + blockIdx.y * 64 + blockIdx.x, t + 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        // outputs nobody inside this launch reads: fire and forget
        if (epi && !(a.diag & 4)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = m0 + wm * 16 + lh * 4 + i;
                if (row >= a.B) continue;
                a.out[(int64_t)row * a.ldo + (int64_t)t * a.so + u] = hn[i];
                float* gt = a.gates + (int64_t)row * a.ldg + (int64_t)t * a.sg;
                gt[u] = rr[i]; gt[D + u] = zz[i]; gt[2 * D + u] = nn[i]; gt[3 * D + u] = gn[i];
            }
        }
    }
}

// ------------------------------------------------------------------ backward
// Reverse sweep of one layer (gru.hip's backward step, t = Fr-1 .. 0):
//   dh_t = dy_t + ddir_{t+1} + dgh_{t+1} . W_hh,  then the gate backward.
// Workgroup (unit tile, row tile) keeps W_hh^T[u0:u0+16, :] (16 x 3D bf16 = 96 KiB)
// resident; per step the 32 rows x 3D of dgh_{t+1} of its row tile stream through an
// 8-slot ring (64 KiB).  dh_direct (= dh z) stays in registers between steps.  The
// hand-off is the forward's: write-through bf16 dgh, per-tile step flags.
namespace gseqb {
constexpr int BM = 32, BN = 16, WM = 2, WN = 1, WK = 2, NS = 8;
typedef Ring<bf16, BM, BN, WM, WN, WK, NS> R;
constexpr int MAXK = 3072;                         // 3D for D <= 1024
constexpr int NSTAGE = MAXK / R::KB;               // 24
constexpr int WIMG = BN * R::KSB * NSTAGE;         // 96 KiB
constexpr int LDS = WIMG + NS * BM * R::KSB;       // + 64 KiB ring
}  // namespace gseqb

struct GruSeqBwdArgs {
    const float* dy; int64_t lddy; int64_t sdy;          // dy[b][t] (D)
    const float* gates; int64_t ldg; int64_t sg;         // forward gates r|z|n|ghn
    const float* hout; int64_t ldo; int64_t so;          // forward h_t (fp32) for h_{t-1}
    const float* h0;                                     // (B, D) initial state
    const bf16* whh_t;                                   // (D, 3D)
    float* dgh; bf16* dgh_lp; float* dgi; int64_t ldd; int64_t sd;   // (3D per row/step)
    float* ddir0;                                        // (B, D): dh_direct of step 0
    int* flags; int* err;
    int* sticky;
    long long spin_limit;
    int withhold;
    int B, D, Fr;
};

__global__ __launch_bounds__(256, 1) void gru_seq_bwd_kernel(GruSeqBwdArgs a) {
    using namespace gseqb;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* wimg = smem;
    char* ring = smem + WIMG;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave % WM, wk = wave / (WM * WN);
    const int u0 = blockIdx.x * 16, m0 = blockIdx.y * BM;
    const int D = a.D, K3 = 3 * D, nk = K3 / R::KB;
    const int nunits = gridDim.x;
    const RowClamp wmap{u0, D};
    const RowClamp hmap{m0, a.B};
    for (int s = 0; s < nk; ++s)
        rc_issue<bf16, BN, R::IB>(a.whh_t, K3, wmap, s * R::KB, wimg + s * BN * R::KSB, wave,
                                  lane);
    const int lr = lane & 15, lh = lane >> 4;
    const int u = u0 + lr;
    const bool epi = wk == 0 && u < D;
    float ddir[4] = {0.f, 0.f, 0.f, 0.f};
    for (int t = a.Fr - 1; t >= 0; --t) {
        const bool has_next = t + 1 < a.Fr;
        // epilogue operands first (older than the ring pieces in the vmcnt queue)
        float dyv[4], gr[4], gz[4], gn[4], gg[4], hp[4];
        if (epi) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = min(m0 + wm * 16 + lh * 4 + i, a.B - 1);
                dyv[i] = a.dy[(int64_t)row * a.lddy + (int64_t)t * a.sdy + u];
                const float* g = a.gates + (int64_t)row * a.ldg + (int64_t)t * a.sg;
                gr[i] = g[u]; gz[i] = g[D + u]; gn[i] = g[2 * D + u]; gg[i] = g[3 * D + u];
                hp[i] = t > 0 ? a.hout[(int64_t)row * a.ldo + (int64_t)(t - 1) * a.so + u]
                              : a.h0[(int64_t)row * D + u];
            }
        }
        floatx4 acc[1][1];
        acc[0][0] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (has_next) {
            if (!gseq_wait_flags(a.flags + blockIdx.y * 64, nunits, a.Fr - 1 - t, a.err, a.sticky,
                                 a.spin_limit, lane))
                return;
            const bf16* src = a.dgh_lp + (int64_t)(t + 1) * a.sd;
            auto issue = [&](int kt) {
                char* slot = ring + (kt % NS) * BM * R::KSB;
                const int k0 = kt * R::KB;
#pragma unroll
                for (int i = 0; i < R::IA; ++i) {
                    const int c = wave * R::IA + i;
                    const int row = c * 4 + (lane >> 4);
                    const int sl = (lane & 15) ^ (row & 15);
                    const bf16* p = src + (int64_t)hmap(row) * a.ldd + k0 + sl * 8;
                    __builtin_amdgcn_global_load_lds(RC_GLB(p), RC_LDS(slot + c * 1024), 16, 0,
                                                     16 /*sc1*/);
                }
            };
#pragma unroll
            for (int st = 0; st < NS - 1; ++st)
                if (st < nk) issue(st);
            for (int kt = 0; kt < nk; ++kt) {
                rc_wait_sel<R::IA, NS - 2>(nk - 1 - kt);
                __builtin_amdgcn_s_barrier();
                if (kt + NS - 1 < nk) issue(kt + NS - 1);
                const char* ia = ring + (kt % NS) * BM * R::KSB;
                const char* ib = wimg + kt * BN * R::KSB;
#pragma unroll
                for (int j = 0; j < R::UPW; ++j) {
                    const int uu = wk + WK * j;
                    const int ra = wm * 16 + lr;
                    const bf16x8 av = *reinterpret_cast<const bf16x8*>(
                        ia + ra * R::KSB + (((uu * 4 + lh) ^ (ra & 15)) * 16));
                    const int rb = lr;
                    const bf16x8 bv = *reinterpret_cast<const bf16x8*>(
                        ib + rb * R::KSB + (((uu * 4 + lh) ^ (rb & 15)) * 16));
                    Mma<bf16>::run(acc[0][0], av, bv);
                }
            }
            __syncthreads();                   // ring free: reused by the reduction
            ring_reduce<bf16, BM, BN, WM, WN, WK, NS>(ring, acc);
        } else {
            // first backward step: nothing to wait for, but the resident W_hh^T pieces must
            // have landed before any later step reads them (the ring waits cover them then)
        }
        float o_dar[4], o_daz[4], o_dghn[4], o_dan[4];
        if (epi) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float dh = acc[0][0][i] + dyv[i];
                if (has_next) dh += ddir[i];
                const float r = gr[i], z = gz[i], n = gn[i], ghn = gg[i];
                const GruBwdPoint o = gru_bwd_point(dh, r, z, n, ghn, hp[i]);
                const float dar = o.dar, daz = o.daz, dghn = o.dghn, dan = o.dan;
                ddir[i] = o.ddir;
                o_dar[i] = dar; o_daz[i] = daz; o_dghn[i] = dghn; o_dan[i] = dan;
                const int row = m0 + wm * 16 + lh * 4 + i;
                if (row < a.B) {      // the row tile's previous step reads these first
                    bf16* dl = a.dgh_lp + (int64_t)row * a.ldd + (int64_t)t * a.sd;
                    gseq_store_wt(dl + u, from_f<bf16>(dar));
                    gseq_store_wt(dl + D + u, from_f<bf16>(daz));
                    gseq_store_wt(dl + 2 * D + u, from_f<bf16>(dghn));
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0 && !(a.withhold && blockIdx.x == 0 && blockIdx.y == 0))
            __hip_atomic_store(a.flags + blockIdx.y * 64 + blockIdx.x, a.Fr - t, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (epi) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = m0 + wm * 16 + lh * 4 + i;
                if (row >= a.B) continue;
                float* dg = a.dgh + (int64_t)row * a.ldd + (int64_t)t * a.sd;
                dg[u] = o_dar[i]; dg[D + u] = o_daz[i]; dg[2 * D + u] = o_dghn[i];
                float* di = a.dgi + (int64_t)row * a.ldd + (int64_t)t * a.sd;
                di[u] = o_dar[i]; di[D + u] = o_daz[i]; di[2 * D + u] = o_dan[i];
                if (t == 0) a.ddir0[(int64_t)row * D + u] = ddir[i];
            }
        }
    }
}


// 1 if the persistent path can run this shape on this device, else 0
extern "C" int srnn_gru_seq_supported(int dtype, int B, int D) {
    if (dtype != SRNN_BF16 || D % 128 != 0 || D > gseq::MAXK || B <= 0) return 0;
    // every workgroup must be co-resident (one per CU: 160 KiB LDS each, for every process
    // sharing the device, persist.hip); <= 64 unit tiles
    return D / 16 <= 64 && srnn_persist_fits_cus((int64_t)(D / 16) * cdiv(B, gseq::BM)) ? 1 : 0;
}

extern "C" int srnn_gru_seq_bwd(int dtype, int B, int D, int Fr, const float* dy, int64_t lddy,
                                int64_t sdy, const float* gates, int64_t ldg, int64_t sg,
                                const float* hout, int64_t ldo, int64_t so, const float* h0,
                                const void* whh_t, float* dgh, void* dgh_lp, float* dgi,
                                int64_t ldd, int64_t sd, float* ddir0, int* work,
                                size_t work_bytes, void* stream) {
    SRNN_REQUIRE(srnn_gru_seq_supported(dtype, B, D), "gru_seq: shape/device not supported");
    SRNN_REQUIRE(3 * D <= gseqb::MAXK && (3 * D) % gseqb::R::KB == 0, "gru_seq_bwd: D");
    const int nm = cdiv(B, gseqb::BM);
    const size_t words = (size_t)nm * 64 + 1;
    SRNN_REQUIRE(work && work_bytes >= words * sizeof(int), "gru_seq_bwd: workspace");
    if (Fr <= 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    SRNN_CHECK_HIP(hipMemsetAsync(work, 0, words * sizeof(int), s));
    static bool attr = false;
    if (!attr) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)gru_seq_bwd_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           gseqb::LDS));
        attr = true;
    }
    GruSeqBwdArgs a;
    a.dy = dy; a.lddy = lddy; a.sdy = sdy;
    a.gates = gates; a.ldg = ldg; a.sg = sg;
    a.hout = hout; a.ldo = ldo; a.so = so; a.h0 = h0;
    a.whh_t = (const bf16*)whh_t;
    a.dgh = dgh; a.dgh_lp = (bf16*)dgh_lp; a.dgi = dgi; a.ldd = ldd; a.sd = sd;
    a.ddir0 = ddir0;
    a.flags = work; a.err = work + (size_t)nm * 64;
    a.sticky = srnn_sticky_flag();
    SRNN_REQUIRE(a.sticky, "gru_seq: sticky flag allocation failed");
    a.spin_limit = srnn_persist_spin_limit((int)gseq::SPIN_LIMIT);
    a.withhold = env_flag("SRNN_PERSIST_FORCE_FAIL", 0);
    a.B = B; a.D = D; a.Fr = Fr;
    if (srnn_persist_check((const void*)gru_seq_bwd_kernel, 256, gseqb::LDS,
                           (int64_t)(D / 16) * nm, "gru_seq_bwd"))
        return 1;
    hipLaunchKernelGGL(gru_seq_bwd_kernel, dim3(D / 16, nm), dim3(256), gseqb::LDS, s, a);
    SRNN_LAUNCH_CHECK();
    return 0;
}

extern "C" int srnn_gru_seq_fwd(int dtype, int B, int D, int Fr, const float* gi, int64_t ldgi,
                                int64_t sgi, const float* h0, const void* h0_lp, const void* whh,
                                const float* bhh, float* out, void* out_lp, int64_t ldo,
                                int64_t so, float* gates, int64_t ldg, int64_t sg, int* work,
                                size_t work_bytes, void* stream) {
    SRNN_REQUIRE(srnn_gru_seq_supported(dtype, B, D), "gru_seq: shape/device not supported");
    const int nm = cdiv(B, gseq::BM);
    const size_t words = (size_t)nm * 64 + 1;
    SRNN_REQUIRE(work && work_bytes >= words * sizeof(int), "gru_seq: workspace");
    if (Fr <= 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    SRNN_CHECK_HIP(hipMemsetAsync(work, 0, words * sizeof(int), s));
    static bool attr = false;
    if (!attr) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)gru_seq_fwd_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           gseq::LDS));
        attr = true;
    }
    GruSeqArgs a;
    a.gi = gi; a.ldgi = ldgi; a.sgi = sgi;
    a.h0 = h0; a.h0_lp = (const bf16*)h0_lp;
    a.whh = (const bf16*)whh; a.bhh = bhh;
    a.out = out; a.out_lp = (bf16*)out_lp; a.ldo = ldo; a.so = so;
    a.gates = gates; a.ldg = ldg; a.sg = sg;
    a.cnt = work; a.err = work + (size_t)nm * 64;
    a.sticky = srnn_sticky_flag();
    SRNN_REQUIRE(a.sticky, "gru_seq: sticky flag allocation failed");
    a.spin_limit = srnn_persist_spin_limit((int)gseq::SPIN_LIMIT);
    a.withhold = env_flag("SRNN_PERSIST_FORCE_FAIL", 0);
    a.B = B; a.D = D; a.Fr = Fr;
    {
        const char* e = getenv("SRNN_GSEQ_DIAG");
        a.diag = e ? atoi(e) : 0;
    }
    if (srnn_persist_check((const void*)gru_seq_fwd_kernel, 256, gseq::LDS,
                           (int64_t)(D / 16) * nm, "gru_seq_fwd"))
        return 1;
    hipLaunchKernelGGL(gru_seq_fwd_kernel, dim3(D / 16, nm), dim3(256), gseq::LDS, s, a);
    SRNN_LAUNCH_CHECK();
    return 0;
}
