// Whole-sequence GRU forward of one FrameLevelRNN layer (model.py:148-165, torch.nn.GRU
// gate order [r | z | n]) as ONE persistent launch organised like the generation sample
// loop (gen_mlp.hip): row groups that live on one XCD, weights resident in VGPRs,
// data-tagged granule hand-offs through that XCD's L2.
//
// gru_seq.hip tiles 32 rows x 16 units per workgroup, so one row tile's 64 workgroups span
// every XCD and each step's h hand-off (64 KiB per workgroup behind 64 step flags) crosses
// the Infinity Fabric.  Here:
//   * a group = 16 rows (one MFMA M tile) x all D units, split over P = D / 32 workgroups of
//     32 units (B = 128, D = 1024: 8 groups x 32 = 256 workgroups, one group per XCD when the
//     per-launch placement check (handoff.hpp) confirms it);
//   * each of the 8 waves holds its K-slice of the workgroup's 96 W_hh rows (3 gates x 32
//     units) as MFMA B fragments in VGPRs for the whole sequence (96 VGPRs at D = 1024);
//   * per step every workgroup reads the group's h_{t-1} as 8-byte {2 x bf16, tag} granules
//     (16 rows x D: 64 KiB, each wave its own K-slice) with sc1 loads -- the data is the flag
//     -- and publishes its 16 x 32 slice of h_t the same way; h is double-buffered (a buffer
//     is rewritten only after every member read the previous step from it);
//   * gate math, outputs and saved gates are gru_seq's (fp32 state, bf16 MMA operands).
#include <algorithm>

#include "samplernn_hip_internal.hpp"
#include "handoff.hpp"
#include "gru_point.hpp"

namespace gx {
constexpr int NW = 8, NTHR = NW * 64;
constexpr int RG = 16;                 // rows per tile (one MFMA M tile)
constexpr int CU = 32;                 // units per workgroup
constexpr int NT = 6;                  // n tiles: 3 gates x 2 x 16 units
constexpr int UK = 32;                 // k per bf16 MFMA unit
constexpr int MAXMT = 4;               // row tiles per group (B up to 512 rows at D = 1024)
// cross-wave reduction buffer: component planes of PS floats, [buf][kw][tile][e][PS]; a
// reader half-wave takes component e of 16 lanes of two adjacent tiles, 4 PS = 16 (mod 32)
// banks apart: conflict-free ds_read_b32 (the lane-major floatx4 layout was 4-way)
constexpr int PS = 68;
// work header: [0] error word, ints [16, HDR / 4) the placement-check slots ([G][P])
constexpr int HDR = 2048;
}  // namespace gx

// Failure reporting: the per-call error word lives in a work buffer the next call re-zeroes,
// so every workgroup folds it into the per-device sticky flag (persist.hip) on exit; the
// fused Adam skips its update while that flag is up and the host reads it at its own sync
// points (srnn_persistent_error_take).
__device__ __forceinline__ void gx_note_failure(const int* err, int* sticky) {
    if (threadIdx.x == 0) {
        const int e = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (e) __hip_atomic_fetch_max(sticky, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Row layout of a sweep (host-chosen, gx_layout): G groups x MT tiles of RV <= 16 valid rows;
// tile m of group g holds batch rows [(g MT + m) RV, +RV).  MT > 1 (B > 16 G: several
// 128-row sets per launch) runs the tiles of one step back to back in every workgroup, so
// one tile's hand-off latency hides behind the others' work; RV < 16 (B < 128) keeps all
// eight XCDs busy with fewer rows each.  Hand-off slots are indexed per tile with a 16-row
// stride whatever RV is.
struct GruXArgs {
    const float* gi; int64_t ldgi; int64_t sgi;     // gi[b][t] (3D, includes b_ih)
    const float* h0;                                // (B, D) fp32
    const bf16* whh; const float* bhh;
    float* out; bf16* out_lp; int64_t ldo; int64_t so;
    bf16* hp_lp;                                    // optional: h_{t-1} (bf16), same layout as out
    float* gates; int64_t ldg; int64_t sg;          // r | z | n | gh_n per row and step
    u64* xh;                                        // 2 x G x MT x RG x D/2 granules
    int* census;                                    // [G][P] zeroed slots (arrival + placement)
    int nolocal;                                    // 1: global-mode hand-offs (SRNN_GEN_LOCAL=0)
    int* err;
    int* sticky;                                    // persist.hip flag
    int spin_limit;
    int withhold;                                   // test switch: workgroup 0 never publishes
    int B, D, Fr, G, P, RV;
    int poll_sleep;                                 // s_sleep 1 repeats between polls
    unsigned long long* diag;                       // optional phase timestamps (timing only)
    int exp;                                        // timing experiments (SRNN_GX_EXP, results
                                                    // invalid): 1 no output stores, 2 no gi loads
};

// DC: D at compile time (0: a.D) -- at D = 1024 the unit-validity selects and the hand-off
// offsets fold to constants (245 -> 186-226 VGPRs, no scalar spills at MT = 2 / 4)
template <int UPW, int MT, int DC = 0>
__global__ __launch_bounds__(gx::NTHR, 2) void gru_xcd_fwd_kernel(GruXArgs a) {
    using namespace gx;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int D = DC ? DC : a.D, B = a.B, RV = a.RV;
    const int NU = D / UK, KW = NW < NU ? NW : NU;
    // double-buffered by the (step, tile) parity: one barrier per (step, tile)
    float* red = (float*)smem;                                  // [2][KW][NT][4][PS]
    int* gsh = (int*)(smem + (size_t)2 * KW * NT * 4 * PS * sizeof(float));
    // static map (handoff.hpp): group g = block % G, member p = block / G; the placement
    // check runs while the weights load
    const int g = blockIdx.x % a.G, p = blockIdx.x / a.G;
    if (tid == 0) hx_group_arrive(a.census + g * a.P + p);
    const int u0 = p * CU;
    const int DG = D / 2;
    unsigned long long* dg = (a.diag && blockIdx.x == 0 && tid == 0) ? a.diag : nullptr;
    int nd = 0;
#define GX_STAMP() do { if (dg && nd < 255) dg[nd++] = __builtin_amdgcn_s_memrealtime(); } while (0)
    // ---- resident W_hh fragments: unit j of this wave = k-range [(wave + NW j) * 32, +32)
    bf16x8 wf[UPW][NT];
    {
        // The workgroup's 3 x 32 W_hh rows are staged through the front of the dynamic LDS one
        // gate at a time (32 x D bf16, whole-row 16-B loads; the reduction buffers there are
        // first used after this block), and each lane reads its 16-B fragments from there:
        // read from global memory, every fragment load touched 16 rows' lines (round 6, the
        // reverse sweep's form of this cut its launch intercept by ~18 us).  Row pitch
        // 2 D + 16 B.
        const int PW = 2 * D + 16;
        const int PPR = D / 8;                                  // 16-B pieces per row
        char* stg = smem;
        uint4 lw[UPW][NT];
#pragma unroll
        for (int gate = 0; gate < 3; ++gate) {
            if (gate) __syncthreads();                          // the previous gate's reads
            const bf16* src = a.whh + (int64_t)(gate * D + u0) * D;
            if constexpr (DC != 0) {
                constexpr int NPT = 32 * (DC / 8) / NTHR;
                uint4 v[NPT];
#pragma unroll
                for (int i = 0; i < NPT; ++i) {
                    const int e = tid + i * NTHR, rr = e / PPR, c = e - rr * PPR;
                    v[i] = *reinterpret_cast<const uint4*>(src + (int64_t)rr * D + c * 8);
                }
#pragma unroll
                for (int i = 0; i < NPT; ++i) {
                    const int e = tid + i * NTHR, rr = e / PPR, c = e - rr * PPR;
                    *reinterpret_cast<uint4*>(stg + rr * PW + c * 16) = v[i];
                }
            } else {
                for (int e = tid; e < 32 * PPR; e += NTHR) {
                    const int rr = e / PPR, c = e - rr * PPR;
                    *reinterpret_cast<uint4*>(stg + rr * PW + c * 16) =
                        *reinterpret_cast<const uint4*>(src + (int64_t)rr * D + c * 8);
                }
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < UPW; ++j) {
                const int u = wave + NW * j;
                const int ke = min(u * UK + (lane >> 4) * 8, D - 8);
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    lw[j][2 * gate + h] = *reinterpret_cast<const uint4*>(
                        stg + (h * 16 + (lane & 15)) * PW + ke * 2);
            }
        }
        __syncthreads();                                        // staging area free again
#pragma unroll
        for (int j = 0; j < UPW; ++j) {
            const bool kv = wave + NW * j < NU;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const uint4 v = kv ? lw[j][t] : make_uint4(0u, 0u, 0u, 0u);
                __builtin_memcpy(&wf[j][t], &v, 16);
            }
        }
    }
    if (wave == 0) {
        const int loc = hx_group_local(a.census + g * a.P, a.P, a.err, !a.nolocal) ? 1 : 0;
        if (tid == 0) gsh[2] = loc;
    }
    __syncthreads();
    const bool local = gsh[2] != 0;
    if (dg) dg[255] = local ? 1 : 2;
    // ---- this thread's state elements: row r of each tile, unit u0 + uu
    const int r = tid >> 5, uu = tid & 31;
    const bool rv = r < RV;
    const int unit = u0 + uu;
    // row_of's lane part is re-made opaque every trip of the step loop (rop below), so the
    // compiler recomputes the per-tile row addresses instead of keeping MT sets of 64-bit
    // pointers live across the loop (at MT = 4 they spilled)
    int rop = r;
    auto row_of = [&](int m) { return (g * MT + m) * RV + rop; };
    const float bhr = a.bhh[unit], bhz = a.bhh[D + unit], bhn = a.bhh[2 * D + unit];
    float hprev[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int row = row_of(m);
        const int b = min(row, B - 1);
        hprev[m] = a.h0[(int64_t)b * D + unit];
        // the previous-state sequence for the backward's W_hh gradient: [h0, h_0 .. h_{F-2}]
        if (a.hp_lp && rv && row < B)
            a.hp_lp[(int64_t)b * a.ldo + unit] = __float2bfloat16(hprev[m]);
    }
    const __amdgpu_buffer_rsrc_t rx = hx_rsrc(a.xh);
    const size_t bufw = (size_t)a.G * MT * RG * DG;             // granules per buffer
    auto publish = [&](int s, int m, float h) {   // h_s of tile m -> buffer (s + 1) & 1, tag s + 2
        const uint32_t mine = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(h));
        const uint32_t nb = lane_next16(mine);
        // fragment-order tile image (see the poll): the granule of units (U, U + 1) is 16-B
        // half (U % 8) / 4 of lane ((U % 32) / 8) * 16 + r in k-unit U / 32's 2 KiB
        if ((uu & 1) == 0 && !(a.withhold && blockIdx.x == 0))
            hx_put(a.xh + ((s + 1) & 1) * bufw + (size_t)(g * MT + m) * RG * DG +
                       ((size_t)(((unit >> 5) * 2 + ((unit & 7) >> 2)) * 64 +
                                 ((unit & 31) >> 3) * 16 + r) << 1) + ((unit & 3) >> 1),
                   (uint32_t)(s + 2), mine | (nb << 16), local);
    };
#pragma unroll
    for (int m = 0; m < MT; ++m) publish(-1, m, hprev[m]);
    const int lrow = lane & 15;
    // input projections: the next (step, tile)'s are issued as soon as this one's hand-off
    // has landed (vmcnt is in order: issued after the publish they made the next hand-off
    // check wait for their latency too), into the other of two register sets used
    // alternately (the (step, tile) sequence unrolled by two: a copy into the current set
    // would wait for the loads at once)
    struct Gi { float r, z, n; };
    Gi ga, gb{0.f, 0.f, 0.f};
    // The input projections are read once and the outputs / saved gates are not read again in
    // this launch: non-temporal (nt) loads and stores, so they do not compete in the L2 with
    // the hand-off lines every poll reads (the reverse sweep's operand loads: 11.8 -> 10.8 us
    // per step at 512 rows).  SRNN_GX_EXP bit 512: plain loads, bit 2048: plain stores (A/B)
    const bool ntl = !(a.exp & 512), nts = !(a.exp & 2048);
    auto ld = [ntl](const float* p) { return ntl ? __builtin_nontemporal_load(p) : *p; };
    {
        const float* gp0 = a.gi + (int64_t)min(row_of(0), B - 1) * a.ldgi;
        ga = Gi{ld(gp0 + unit), ld(gp0 + D + unit), ld(gp0 + 2 * D + unit)};
    }
    auto fetch_gi = [&](int t, int m, Gi& nx) {     // operands of the (step, tile) after (t, m)
        if (a.exp & 2) return;
        int tn = t, mn = m + 1;
        if (mn == MT) { mn = 0; tn = min(t + 1, a.Fr - 1); }
        const float* gp = a.gi + (int64_t)min(row_of(mn), B - 1) * a.ldgi + (int64_t)tn * a.sgi;
        nx.r = ld(gp + unit); nx.z = ld(gp + D + unit); nx.n = ld(gp + 2 * D + unit);
    };
    auto step = [&](int t, int m, const Gi& cu, Gi& nx) {
            floatx4 acc[NT];
    #pragma unroll
            for (int i = 0; i < NT; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
            // (UPW >= 2: NU > NW units, every wave polls -- known at compile time, so the
            //  wait analysis sees the poll's vmcnt(0) on every path and the step's operands
            //  from the previous step need no further wait)
            const bool polls = UPW >= 2 || wave < KW;
            if (!polls) fetch_gi(t, m, nx);
            if (polls) {
                const uint32_t tag = (uint32_t)(t + 1);
                // the tile's image in fragment order: k-unit u's 2 KiB hold lane l's first 16 B
                // (row l & 15, k = 32 u + 8 (l >> 4) + 0..3) at l * 16 and its second at
                // 1 KiB + l * 16, so each poll instruction reads 1 KiB of whole lines (the
                // row-major image took 16 half lines per instruction)
                // (RV < 16, B < 128: a lane of a padding row -- lrow >= RV, never stored --
                //  reads nothing: its offset is past the buffer's range, so the load returns
                //  zeros without a memory access, and the poll moves RV / 16 of the bytes)
                const uint32_t base = (uint32_t)(((size_t)(t & 1) * bufw +
                                                  (size_t)(g * MT + m) * RG * DG) * 8) +
                                      (lrow < RV ? lane * 16u : 0x80000000u);
                uint32_t w[UPW][4];
                int spins = 0;
                for (;;) {
                    // every load unconditional (clamped unit), so all 2 x UPW are in flight at
                    // once; a branch per unit would put a vmcnt(0) between them
                    uint4 x[UPW][2];
    #pragma unroll
                    for (int j = 0; j < UPW; ++j) {
                        const int u = min(wave + NW * j, NU - 1);
                        const uint32_t off = base + (uint32_t)u * 2048u;
                        x[j][0] = hx_get2(rx, off);
                        x[j][1] = hx_get2(rx, off + 1024);
                    }
                    bool ok = true;
    #pragma unroll
                    for (int j = 0; j < UPW; ++j) {
                        const bool v = wave + NW * j < NU;
                        w[j][0] = v ? x[j][0].x : 0u; w[j][1] = v ? x[j][0].z : 0u;
                        w[j][2] = v ? x[j][1].x : 0u; w[j][3] = v ? x[j][1].z : 0u;
                        ok &= !v || ((x[j][0].y == tag) & (x[j][0].w == tag) &
                                     (x[j][1].y == tag) & (x[j][1].w == tag));
                    }
                    ok |= lrow >= RV;
                    if (__all(ok)) break;
                    if (hx_spin_fail(spins, a.err, lane, a.poll_sleep, a.spin_limit)) break;
                }
                fetch_gi(t, m, nx);
                GX_STAMP();
    #pragma unroll
                for (int j = 0; j < UPW; ++j) {
                    const uint4 v = make_uint4(w[j][0], w[j][1], w[j][2], w[j][3]);
                    bf16x8 af;
                    __builtin_memcpy(&af, &v, 16);
    #pragma unroll
                    for (int i = 0; i < NT; ++i) Mma<bf16>::run(acc[i], af, wf[j][i]);
                }
                float* rb = red + (size_t)(((t * MT + m) & 1) * KW + wave) * NT * 4 * PS + lane;
    #pragma unroll
                for (int i = 0; i < NT; ++i)
    #pragma unroll
                    for (int e = 0; e < 4; ++e) rb[(i * 4 + e) * PS] = acc[i][e];
            }
            GX_STAMP();
            __syncthreads();
            GX_STAMP();
            float gh[3];
            {
                const int ln = (r >> 2) * 16 + (uu & 15), ii = r & 3;
                const float* rb = red + (size_t)((t * MT + m) & 1) * KW * NT * 4 * PS + ii * PS + ln;
    #pragma unroll
                for (int gt = 0; gt < 3; ++gt) {
                    const int tile = 2 * gt + (uu >> 4);
                    float v = 0.f;
                    float pr[NW];
                    #pragma unroll
                    for (int kw = 0; kw < NW; ++kw)
                        pr[kw] = rb[(min(kw, KW - 1) * NT + tile) * 4 * PS];
                    #pragma unroll
                    for (int kw = 0; kw < NW; ++kw) v += kw < KW ? pr[kw] : 0.f;
                    gh[gt] = v;
                }
            }
            const float ghr = gh[0] + bhr, ghz = gh[1] + bhz, ghn = gh[2] + bhn;
            const float rr = 1.0f / (1.0f + expf(-(ghr + cu.r)));
            const float zz = 1.0f / (1.0f + expf(-(ghz + cu.z)));
            const float nn = tanhf(cu.n + ghn * rr);
            const float hn = (hprev[m] - nn) * zz + nn;
            hprev[m] = hn;
            publish(t, m, hn);
            GX_STAMP();
            const int row = row_of(m);
            if (rv && row < B && !(a.exp & 1)) {
                const int64_t o = (int64_t)row * a.ldo + (int64_t)t * a.so + unit;
                float* gt = a.gates + (int64_t)row * a.ldg + (int64_t)t * a.sg;
                const unsigned short hb = __bfloat16_as_ushort(__float2bfloat16(hn));
                unsigned short* olp = reinterpret_cast<unsigned short*>(a.out_lp);
                unsigned short* hlp = reinterpret_cast<unsigned short*>(a.hp_lp);
                if (nts) {
                    __builtin_nontemporal_store(hn, a.out + o);
                    __builtin_nontemporal_store(hb, olp + o);
                    if (a.hp_lp && t + 1 < a.Fr) __builtin_nontemporal_store(hb, hlp + o + a.so);
                    __builtin_nontemporal_store(rr, gt + unit);
                    __builtin_nontemporal_store(zz, gt + D + unit);
                    __builtin_nontemporal_store(nn, gt + 2 * D + unit);
                    __builtin_nontemporal_store(ghn, gt + 3 * D + unit);
                } else {
                    a.out[o] = hn;
                    olp[o] = hb;
                    if (a.hp_lp && t + 1 < a.Fr) hlp[o + a.so] = hb;
                    gt[unit] = rr; gt[D + unit] = zz; gt[2 * D + unit] = nn; gt[3 * D + unit] = ghn;
                }
            }
            // (no barrier: the next (step, tile) writes the other red buffer, and this one is
            //  rewritten only after every wave passed the next (step, tile)'s barrier)
            GX_STAMP();
    };
    // (step, tile) sequence, unrolled by two for the alternating operand sets (MT = 1: two
    // steps per trip; MT even: the tiles of one step)
    constexpr int TU = MT == 1 ? 2 : 1;
    for (int t0 = 0; t0 < a.Fr; t0 += TU) {
        if (MT > 1) asm volatile("" : "+v"(rop));
#pragma unroll
        for (int q = 0; q < TU * MT; ++q) {
            const int t = t0 + q / MT, m = q % MT;
            if (t >= a.Fr) break;
            if (q & 1) step(t, m, gb, ga);
            else step(t, m, ga, gb);
        }
    }
#undef GX_STAMP
    gx_note_failure(a.err, a.sticky);
}

// ------------------------------------------------------------------ backward
// Reverse sweep of one layer (gru_seq.hip's backward, same pointwise code, gru_point.hpp):
//   dh_t = dy_t + ddir_{t+1} + dgh_{t+1} . W_hh,  then the gate backward.
// Same groups and tiles as the forward; each wave keeps its K-slice (3D / 8 = 384 k) of the
// workgroup's 32 W_hh^T rows as B fragments (96 VGPRs at D = 1024); per step and tile the
// tile's dgh_{t+1} (16 rows x 3D bf16) arrives as granules (double-buffered, tag = Fr - step).
struct GruXBwdArgs {
    const float* dy; int64_t lddy; int64_t sdy;
    const float* gates; int64_t ldg; int64_t sg;
    const float* hout; int64_t ldo; int64_t so;
    const float* h0;
    const bf16* whh_t;                              // (D, 3D)
    float* dgh; bf16* dgh_lp; float* dgi; int64_t ldd; int64_t sd;   // dgh / dgi optional
    bf16* dgi_lp;                                   // optional bf16 dgi (same layout)
    float* bsum;                                    // optional (B, 4D): per-row sums over t of
                                                    // [dar | daz | dghn | dan] (bias grads)
    float* ddir0;                                   // (B, D)
    u64* xg;                                        // 2 x G x MT x RG x 3D/2 granules
    int* census;
    int nolocal;
    int* err;
    int* sticky;
    int spin_limit;
    int withhold;
    int B, D, Fr, G, P, RV;
    int exp;                                        // timing experiments (as the forward)
};

template <int UPW, bool FULL, int MT>   // FULL: NU == UPW * NW (every unit of every wave in range)
__global__ __launch_bounds__(gx::NTHR, 2) void gru_xcd_bwd_kernel(GruXBwdArgs a) {
    using namespace gx;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int D = a.D, B = a.B, K3 = 3 * D, RV = a.RV;
    const int NU = K3 / UK, KW = NW < NU ? NW : NU;
    constexpr int NTB = 2;                                      // 32 units = 2 n tiles
    float* red = (float*)smem;                                  // [2][KW][NTB][4][PS]
    const size_t red_bytes = (size_t)2 * KW * NTB * 4 * PS * sizeof(float);
    int* gsh = (int*)(smem + red_bytes);
    // static map (handoff.hpp): group g = block % G, member p = block / G; the placement
    // check runs while the weights load
    const int g = blockIdx.x % a.G, p = blockIdx.x / a.G;
    if (tid == 0) hx_group_arrive(a.census + g * a.P + p);
    const int u0 = p * CU;
    const int KG = K3 / 2;                                      // granules per row
    bf16x8 wf[UPW][NTB];
    {
        uint4 lw[UPW][NTB];
#pragma unroll
        for (int j = 0; j < UPW; ++j) {
            const int u = wave + NW * j;
            const int ke = min(u * UK + (lane >> 4) * 8, K3 - 8);
#pragma unroll
            for (int t = 0; t < NTB; ++t) {
                const int row = u0 + t * 16 + (lane & 15);
                lw[j][t] = *reinterpret_cast<const uint4*>(a.whh_t + (int64_t)row * K3 + ke);
            }
        }
#pragma unroll
        for (int j = 0; j < UPW; ++j) {
            const bool kv = wave + NW * j < NU;
#pragma unroll
            for (int t = 0; t < NTB; ++t) {
                const uint4 v = kv ? lw[j][t] : make_uint4(0u, 0u, 0u, 0u);
                __builtin_memcpy(&wf[j][t], &v, 16);
            }
        }
    }
    if (wave == 0) {
        const int loc = hx_group_local(a.census + g * a.P, a.P, a.err, !a.nolocal) ? 1 : 0;
        if (tid == 0) gsh[2] = loc;
    }
    __syncthreads();
    const bool local = gsh[2] != 0;
    const int r = tid >> 5, uu = tid & 31;
    const bool rv = r < RV;
    const int unit = u0 + uu;
    int rop = r;                                    // (opaque per step: see the forward)
    auto row_of = [&](int m) { return (g * MT + m) * RV + rop; };
    const __amdgpu_buffer_rsrc_t rx = hx_rsrc(a.xg);
    const size_t bufw = (size_t)a.G * MT * RG * KG;
    const int lrow = lane & 15;
    // this (step, tile)'s operands, loaded one (step, tile) ahead (see the forward)
    auto fetch = [&](int t, int m, float& dyv, float& gr, float& gz, float& gn, float& gg,
                     float& hp) {
        const int b = min(row_of(m), B - 1);
        dyv = a.dy[(int64_t)b * a.lddy + (int64_t)t * a.sdy + unit];
        const float* gp = a.gates + (int64_t)b * a.ldg + (int64_t)t * a.sg;
        gr = gp[unit]; gz = gp[D + unit]; gn = gp[2 * D + unit]; gg = gp[3 * D + unit];
        hp = t > 0 ? a.hout[(int64_t)b * a.ldo + (int64_t)(t - 1) * a.so + unit]
                   : a.h0[(int64_t)b * D + unit];
    };
    float dyv, gr, gz, gn, gg, hp;
    // per-tile state (the carried dh_direct and the bias-gradient row sums over t): registers
    // at MT = 1, per-thread LDS slots above (the register file is full at D = 1024: W_hh^T
    // slice + poll buffer; the tile loop is not unrolled, so its index is not a constant)
    float ddir1 = 0.f, sar1 = 0.f, saz1 = 0.f, sghn1 = 0.f, san1 = 0.f;
    float* sl = (float*)(smem + red_bytes + 64);                 // [MT][5][NTHR]
    if (MT > 1)
        for (int k = 0; k < 5 * MT; ++k) sl[k * NTHR + tid] = 0.f;
    fetch(a.Fr - 1, 0, dyv, gr, gz, gn, gg, hp);
    for (int t = a.Fr - 1; t >= 0; --t) {
    asm volatile("" : "+v"(rop));
#pragma unroll 1
    for (int m = 0; m < MT; ++m) {
        const bool has_next = t + 1 < a.Fr;
        float* q = sl + (m * 5) * NTHR + tid;             // (MT > 1) this tile's state slots
        const float ddir_in = MT == 1 ? ddir1 : q[0];
        floatx4 acc[NTB];
#pragma unroll
        for (int i = 0; i < NTB; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (has_next) {
            if (UPW >= 2 || wave < KW) {                        // (as the forward)
                const uint32_t tag = (uint32_t)(a.Fr - 1 - t);     // dgh_{t+1}
                const uint32_t base = (uint32_t)((((size_t)((t + 1) & 1)) * bufw +
                                                  (size_t)((g * MT + m) * RG + lrow) * KG) * 8);
                uint4 x[UPW][2];
                int spins = 0;
                // unit j's granules sit at lane offset + j * NW units (every unit of the wave
                // in range: NU == UPW * NW, e.g. D = 1024); the lane offset is made opaque per
                // step so the compiler does not keep UPW hoisted offsets live (at UPW = 12 they
                // were spilled to scratch and reloaded serially every step)
                uint32_t lb = (uint32_t)((wave * UK + (lane >> 4) * 8) / 2) * 8u;
                asm volatile("" : "+v"(lb));
                for (;;) {
                    if (a.exp & 32) {                    // (timing: no hand-off reads at all)
#pragma unroll
                        for (int j = 0; j < UPW; ++j)
                            x[j][0] = x[j][1] = make_uint4(lane, tag, lane, tag);
                        asm volatile("" : "+v"(x[0][0].x));
                        break;
                    }
#pragma unroll
                    for (int j = 0; j < UPW; ++j) {
                        const int u = min(wave + NW * j, NU - 1);
                        const uint32_t off =
                            FULL ? base + lb + (uint32_t)(j * NW * UK / 2 * 8)
                                 : base + (uint32_t)((u * UK + (lane >> 4) * 8) / 2) * 8u;
                        x[j][0] = hx_get2(rx, off);
                        x[j][1] = hx_get2(rx, off + 16);
                    }
                    if (a.exp & 8) break;                // (timing: no tag check / wait)
                    bool ok = true;
#pragma unroll
                    for (int j = 0; j < UPW; ++j)
                        ok &= (wave + NW * j >= NU) ||
                              ((x[j][0].y == tag) & (x[j][0].w == tag) & (x[j][1].y == tag) &
                               (x[j][1].w == tag));
                    if (__all(ok)) break;
                    if (hx_spin_fail(spins, a.err, lane, 1, a.spin_limit)) break;
                }
#pragma unroll
                for (int j = 0; j < UPW; ++j) {
                    const bool kv = wave + NW * j < NU;      // (weights are zero there too)
                    const uint4 v = kv ? make_uint4(x[j][0].x, x[j][0].z, x[j][1].x, x[j][1].z)
                                       : make_uint4(0u, 0u, 0u, 0u);
                    bf16x8 af;
                    __builtin_memcpy(&af, &v, 16);
                    if (a.exp & 4) {                     // (timing: no MFMA)
                        asm volatile("" :: "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
                        continue;
                    }
#pragma unroll
                    for (int i = 0; i < NTB; ++i) Mma<bf16>::run(acc[i], af, wf[j][i]);
                }
                float* rb = red + (size_t)((((a.Fr - 1 - t) * MT + m) & 1) * KW + wave) * NTB * 4 * PS + lane;
#pragma unroll
                for (int i = 0; i < NTB; ++i)
#pragma unroll
                    for (int e = 0; e < 4; ++e) rb[(i * 4 + e) * PS] = acc[i][e];
            }
            if (!(a.exp & 16)) __syncthreads();          // (timing: no barrier)
        }
        float s = 0.f;
        if (has_next) {
            const int ln = (r >> 2) * 16 + (uu & 15), ii = r & 3, tile = uu >> 4;
            const float* rb = red + (size_t)(((a.Fr - 1 - t) * MT + m) & 1) * KW * NTB * 4 * PS +
                              ii * PS + ln;
            float pr[NW];
#pragma unroll
            for (int kw = 0; kw < NW; ++kw) pr[kw] = rb[(min(kw, KW - 1) * NTB + tile) * 4 * PS];
#pragma unroll
            for (int kw = 0; kw < NW; ++kw) s += kw < KW ? pr[kw] : 0.f;
        }
        float dh = s + dyv;
        if (has_next) dh += ddir_in;
        const GruBwdPoint o = gru_bwd_point(dh, gr, gz, gn, gg, hp);
        if (MT == 1) ddir1 = o.ddir;
        else q[0] = o.ddir;
        // publish dgh_t = [dar | daz | dghn] (bf16 granules, pairs of units), tag Fr - t
        {
            const float vals[3] = {o.dar, o.daz, o.dghn};
            u64* dst = a.xg + (size_t)(t & 1) * bufw + (size_t)((g * MT + m) * RG + r) * KG;
#pragma unroll
            for (int gt = 0; gt < 3; ++gt) {
                const uint32_t mine = (uint32_t)__bfloat16_as_ushort(__float2bfloat16(vals[gt]));
                const uint32_t nb = lane_next16(mine);
                if ((uu & 1) == 0 && !(a.withhold && blockIdx.x == 0))
                    hx_put(dst + (gt * D + unit) / 2, (uint32_t)(a.Fr - t), mine | (nb << 16), local);
            }
        }
        const float cdar = o.dar, cdaz = o.daz, cdghn = o.dghn, cdan = o.dan;
        if (!(a.exp & 2)) {
            if (m + 1 < MT) fetch(t, m + 1, dyv, gr, gz, gn, gg, hp);
            else if (t > 0) fetch(t - 1, 0, dyv, gr, gz, gn, gg, hp);
        }
        const int row = row_of(m);
        if (rv && row < B && !(a.exp & 1)) {
            const int64_t ob = (int64_t)row * a.ldd + (int64_t)t * a.sd;
            if (a.dgh) {
                float* dg = a.dgh + ob;
                dg[unit] = cdar; dg[D + unit] = cdaz; dg[2 * D + unit] = cdghn;
            }
            bf16* dl = a.dgh_lp + ob;
            const bf16 har = __float2bfloat16(cdar), haz = __float2bfloat16(cdaz);
            dl[unit] = har; dl[D + unit] = haz; dl[2 * D + unit] = __float2bfloat16(cdghn);
            if (a.dgi) {
                float* di = a.dgi + ob;
                di[unit] = cdar; di[D + unit] = cdaz; di[2 * D + unit] = cdan;
            }
            if (a.dgi_lp) {
                bf16* dj = a.dgi_lp + ob;
                dj[unit] = har; dj[D + unit] = haz; dj[2 * D + unit] = __float2bfloat16(cdan);
            }
            if (MT == 1) {
                sar1 += cdar; saz1 += cdaz; sghn1 += cdghn; san1 += cdan;
            } else {
                q[NTHR] += cdar; q[2 * NTHR] += cdaz; q[3 * NTHR] += cdghn; q[4 * NTHR] += cdan;
            }
            if (t == 0) a.ddir0[(int64_t)row * D + unit] = o.ddir;
        }
        // (no barrier: red is double-buffered by the (step, tile) parity, see the forward)
    }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int row = row_of(m);
        if (a.bsum && rv && row < B) {
            float* bs = a.bsum + (int64_t)row * 4 * D;
            if (MT == 1) {
                bs[unit] = sar1; bs[D + unit] = saz1; bs[2 * D + unit] = sghn1;
                bs[3 * D + unit] = san1;
            } else {
                const float* q = sl + (m * 5) * NTHR + tid;
                bs[unit] = q[NTHR]; bs[D + unit] = q[2 * NTHR]; bs[2 * D + unit] = q[3 * NTHR];
                bs[3 * D + unit] = q[4 * NTHR];
            }
        }
    }
    gx_note_failure(a.err, a.sticky);
}

// Packed hand-off form of the reverse sweep (the default at D % 64 == 0).  A thread's dgh_t
// for its unit is ONE 8-byte granule {dar, daz, dghn (bf16), tag (16 bits)} instead of 1.5
// {2 x bf16, 32-bit tag} granules per value pair: the consumers read 16 x D x 8 B per tile
// (128 KiB at D = 1024) instead of 16 x 3D/2 x 8 B (192 KiB) -- the hand-off reads are what
// the sweep's per-step time goes to (tools/gx_exp.py: without them 2.6 of 7.7 us at B = 128).
// The product dgh_{t+1} . W_hh then runs over K' = 4D with k' = 4 unit + slot: slots 0-2 are
// the gates (the granule's bytes ARE the MFMA A operand, unpacked nowhere) and slot 3, the
// tag, meets zero weights (tags are small positive integers: finite bf16 bit patterns, so
// tag x 0 = 0).  The W_hh^T fragments are gathered into that order once, in the prologue.
template <int UPW, int MT>
__global__ __launch_bounds__(gx::NTHR, 2) void gru_xcd_bwd_pk_kernel(GruXBwdArgs a) {
    using namespace gx;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    constexpr int D = UPW * 64;                                 // the host picks UPW = D / 64
    const int B = a.B, RV = a.RV;
    constexpr int KW = NW;                                      // NU' = D / 8 = UPW * NW
    constexpr int NTB = 2;
    float* red = (float*)smem;                                  // [2][KW][NTB][4][PS]
    const size_t red_bytes = (size_t)2 * KW * NTB * 4 * PS * sizeof(float);
    int* gsh = (int*)(smem + red_bytes);
    const int g = blockIdx.x % a.G, p = blockIdx.x / a.G;
    if (tid == 0) hx_group_arrive(a.census + g * a.P + p);
    const int u0 = p * CU;
    bf16x8 wf[UPW][NTB];
    {
        // lane's k' = [32 u + 8 (lane >> 4), +8): input units iu, iu + 1, slots 0..3 each.
        // The workgroup's 32 W_hh^T rows are staged through LDS one gate at a time (32 x D
        // bf16, whole-row 16-B loads), and each lane picks its 4-B pairs from there: read
        // straight from global memory, those 96 4-B loads per lane touched 16 rows' lines per
        // instruction and cost ~20 us per launch (round 6, tools/gru_fixed_probe.py: reverse
        // sweep intercept 22.7 -> 4.4 us at B = 64 without them).  Row pitch 2 D + 16 B: the
        // 16 rows x 4 lane groups of a b32 read hit 64 distinct banks.  The staging area is the
        // front of the dynamic LDS, free until the reduction buffers are first used below.
        constexpr int PW = 2 * D + 16;
        constexpr int PPR = D / 8;                              // 16-B pieces per row
        constexpr int NPT = 32 * PPR / NTHR;                    // pieces per thread per gate
        static_assert((32 * PPR) % NTHR == 0, "gru_xcd_bwd_pk: staging split");
        char* stg = smem;
        // one array per gate (constant indices only: a [3] dimension indexed by the gate loop
        // was placed in scratch)
        unsigned lr[UPW][NTB], lz[UPW][NTB], ln[UPW][NTB];
        auto stage = [&](int gt, unsigned (&lw)[UPW][NTB]) __attribute__((always_inline)) {
            if (gt) __syncthreads();                            // the previous gate's reads
            // (unrolled load / store pairs: global and LDS do not alias, so the loads issue
            //  back to back; an array of the NPT pieces was left in scratch at 243 VGPRs)
#pragma unroll
            for (int i = 0; i < NPT; ++i) {
                const int e = tid + i * NTHR, rr = e / PPR, c = e - rr * PPR;
                *reinterpret_cast<uint4*>(stg + rr * PW + c * 16) =
                    *reinterpret_cast<const uint4*>(a.whh_t + (int64_t)(u0 + rr) * 3 * D +
                                                    gt * D + c * 8);
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < UPW; ++j) {
                const int iu = (wave + NW * j) * 8 + (lane >> 4) * 2;
#pragma unroll
                for (int t = 0; t < NTB; ++t)
                    lw[j][t] = *reinterpret_cast<const unsigned*>(
                        stg + (t * 16 + (lane & 15)) * PW + iu * 2);
            }
        };
        stage(0, lr);
        stage(1, lz);
        stage(2, ln);
        __syncthreads();                                        // staging area free again
#pragma unroll
        for (int j = 0; j < UPW; ++j)
#pragma unroll
            for (int t = 0; t < NTB; ++t) {
                // [r0 z0 n0 0 | r1 z1 n1 0] (low / high halves of each gate word)
                const unsigned r2 = lr[j][t], z2 = lz[j][t], n2 = ln[j][t];
                const uint4 v = make_uint4((r2 & 0xffffu) | (z2 << 16), n2 & 0xffffu,
                                           (r2 >> 16) | (z2 & 0xffff0000u), n2 >> 16);
                __builtin_memcpy(&wf[j][t], &v, 16);
            }
    }
    if (wave == 0) {
        const int loc = hx_group_local(a.census + g * a.P, a.P, a.err, !a.nolocal) ? 1 : 0;
        if (tid == 0) gsh[2] = loc;
    }
    __syncthreads();
    const bool local = gsh[2] != 0;
    const int r = tid >> 5, uu = tid & 31;
    const bool rv = r < RV;
    const int unit = u0 + uu;
    int rop = r;
    auto row_of = [&](int m) { return (g * MT + m) * RV + rop; };
    const __amdgpu_buffer_rsrc_t rx = hx_rsrc(a.xg);
    const size_t bufw = (size_t)a.G * MT * RG * D;              // granules per buffer
    const int lrow = lane & 15;
    // The next (step, tile)'s operands -- dy, the saved gates, h_{t-1}: read once, ~1.5 MB per
    // XCD and step at 512 rows -- as non-temporal (nt) buffer loads, so they stream past the
    // L2 instead of competing there with the hand-off lines every poll reads: reverse sweep
    // 11.8 -> 10.8 us per step at 512 rows (round 6, tools/gru_fixed_probe.py; no change at 64
    // rows).  Issuing them earlier in the step (after the hand-off's MFMAs) measured no better
    // at 512 rows and slower at 64.  SRNN_GX_EXP bit 512: plain loads (A/B).  32-bit byte
    // offsets, resources in SGPRs.
    const __amdgpu_buffer_rsrc_t rdy = hx_rsrc(a.dy), rgt = hx_rsrc(a.gates),
                                 rho = hx_rsrc(a.hout), rh0 = hx_rsrc(a.h0);
    const bool plain = (a.exp & 512) != 0;
    auto ldf = [plain](__amdgpu_buffer_rsrc_t r, uint32_t off) {
        return __uint_as_float(plain ? __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0)
                                     : __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 2 /*nt*/));
    };
    // (the host sends launches with a byte offset past 2 GB -- very long sequences -- to the
    //  unpacked kernel, whose operand loads use 64-bit pointers)
    auto fetch = [&](int t, int m, float& dyv, float& gr, float& gz, float& gn, float& gg,
                     float& hp) {
        const uint32_t b = (uint32_t)min(row_of(m), B - 1);
        dyv = ldf(rdy, (uint32_t)(b * a.lddy + t * a.sdy + unit) * 4u);
        const uint32_t go = (uint32_t)(b * a.ldg + t * a.sg + unit) * 4u;
        gr = ldf(rgt, go); gz = ldf(rgt, go + 4u * D); gn = ldf(rgt, go + 8u * D);
        gg = ldf(rgt, go + 12u * D);
        hp = t > 0 ? ldf(rho, (uint32_t)(b * a.ldo + (t - 1) * a.so + unit) * 4u)
                   : ldf(rh0, (uint32_t)(b * D + unit) * 4u);
    };
    float dyv, gr, gz, gn, gg, hp;
    float ddir1 = 0.f, sar1 = 0.f, saz1 = 0.f, sghn1 = 0.f, san1 = 0.f;
    float* sl = (float*)(smem + red_bytes + 64);                 // [MT][5][NTHR]
    if (MT > 1)
        for (int k = 0; k < 5 * MT; ++k) sl[k * NTHR + tid] = 0.f;
    fetch(a.Fr - 1, 0, dyv, gr, gz, gn, gg, hp);
    for (int t = a.Fr - 1; t >= 0; --t) {
    asm volatile("" : "+v"(rop));
#pragma unroll 1
    for (int m = 0; m < MT; ++m) {
        const bool has_next = t + 1 < a.Fr;
        float* q = sl + (m * 5) * NTHR + tid;
        const float ddir_in = MT == 1 ? ddir1 : q[0];
        floatx4 acc[NTB];
#pragma unroll
        for (int i = 0; i < NTB; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (has_next) {
            const uint32_t tag = (uint32_t)(a.Fr - 1 - t);          // dgh_{t+1}
            // fragment-major tile image: k'-unit u's 1 KiB holds lane l's 16 B at l * 16 (row
            // l & 15, k' 32 u + 8 (l >> 4) ..): every poll instruction reads 1 KiB of whole
            // lines (the row-major image took 16 half lines per instruction)
            const uint32_t base = (uint32_t)((((size_t)((t + 1) & 1)) * bufw +
                                              (size_t)(g * MT + m) * RG * D) * 8);
            uint4 x[UPW];
            int spins = 0;
            // (made opaque per step, see the unpacked kernel)
            // (a padding-row lane, lrow >= RV: out-of-range offset, zeros without a memory
            //  access -- see the forward)
            uint32_t lb = lrow < RV ? (uint32_t)(wave * 64 + lane) * 16u : 0x80000000u;
            asm volatile("" : "+v"(lb));
            for (;;) {
#pragma unroll
                for (int j = 0; j < UPW; ++j)
                    x[j] = hx_get2(rx, base + lb + (uint32_t)(j * NW * 64 * 16));
                bool ok = true;
#pragma unroll
                for (int j = 0; j < UPW; ++j)
                    ok &= ((x[j].y >> 16) == tag) & ((x[j].w >> 16) == tag);
                ok |= lrow >= RV;
                if (__all(ok)) break;
                if (hx_spin_fail(spins, a.err, lane, 1, a.spin_limit)) break;
            }
#pragma unroll
            for (int j = 0; j < UPW; ++j) {
                bf16x8 af;
                __builtin_memcpy(&af, &x[j], 16);
#pragma unroll
                for (int i = 0; i < NTB; ++i) Mma<bf16>::run(acc[i], af, wf[j][i]);
            }
            float* rb = red + (size_t)((((a.Fr - 1 - t) * MT + m) & 1) * KW + wave) * NTB * 4 * PS + lane;
#pragma unroll
            for (int i = 0; i < NTB; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) rb[(i * 4 + e) * PS] = acc[i][e];
            __syncthreads();
        }
        float s = 0.f;
        if (has_next) {
            const int ln = (r >> 2) * 16 + (uu & 15), ii = r & 3, tile = uu >> 4;
            const float* rb = red + (size_t)(((a.Fr - 1 - t) * MT + m) & 1) * KW * NTB * 4 * PS +
                              ii * PS + ln;
            float pr[NW];
#pragma unroll
            for (int kw = 0; kw < NW; ++kw) pr[kw] = rb[(kw * NTB + tile) * 4 * PS];
#pragma unroll
            for (int kw = 0; kw < NW; ++kw) s += pr[kw];
        }
        float dh = s + dyv;
        if (has_next) dh += ddir_in;
        const GruBwdPoint o = gru_bwd_point(dh, gr, gz, gn, gg, hp);
        if (MT == 1) ddir1 = o.ddir;
        else q[0] = o.ddir;
        // publish dgh_t of this unit: one granule {dar, daz, dghn, tag = Fr - t}
        if (!(a.withhold && blockIdx.x == 0)) {
            // granule of (row r, unit U): k'-unit U / 8, lane ((U % 8) / 2) * 16 + r, half U % 2
            u64* dst = a.xg + (size_t)(t & 1) * bufw + (size_t)(g * MT + m) * RG * D +
                       ((size_t)((unit >> 3) * 64 + ((unit & 7) >> 1) * 16 + r) << 1) + (unit & 1);
            const u64 v = (u64)__bfloat16_as_ushort(__float2bfloat16(o.dar)) |
                          ((u64)__bfloat16_as_ushort(__float2bfloat16(o.daz)) << 16) |
                          ((u64)__bfloat16_as_ushort(__float2bfloat16(o.dghn)) << 32) |
                          ((u64)(uint32_t)(a.Fr - t) << 48);
            if (local) __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const float cdar = o.dar, cdaz = o.daz, cdghn = o.dghn, cdan = o.dan;
        if (!(a.exp & 64)) {                       // (timing: SRNN_GX_EXP 64 skips the fetch)
            if (m + 1 < MT) fetch(t, m + 1, dyv, gr, gz, gn, gg, hp);
            else if (t > 0) fetch(t - 1, 0, dyv, gr, gz, gn, gg, hp);
        }
        const int row = row_of(m);
        if (rv && row < B && !(a.exp & 1)) {     // (timing: SRNN_GX_EXP 1 skips the stores)
            const int64_t ob = (int64_t)row * a.ldd + (int64_t)t * a.sd;
            if (a.dgh) {
                float* dg = a.dgh + ob;
                dg[unit] = cdar; dg[D + unit] = cdaz; dg[2 * D + unit] = cdghn;
            }
            // (the bf16 GEMM operands are read by later launches only: nt stores, as the
            //  operand loads; SRNN_GX_EXP bit 2048: plain stores)
            unsigned short* dl = reinterpret_cast<unsigned short*>(a.dgh_lp + ob);
            const unsigned short har = __bfloat16_as_ushort(__float2bfloat16(cdar)),
                                 haz = __bfloat16_as_ushort(__float2bfloat16(cdaz)),
                                 hgn = __bfloat16_as_ushort(__float2bfloat16(cdghn)),
                                 han = __bfloat16_as_ushort(__float2bfloat16(cdan));
            const bool nts = !(a.exp & 2048);
            if (nts) {
                __builtin_nontemporal_store(har, dl + unit);
                __builtin_nontemporal_store(haz, dl + D + unit);
                __builtin_nontemporal_store(hgn, dl + 2 * D + unit);
            } else {
                dl[unit] = har; dl[D + unit] = haz; dl[2 * D + unit] = hgn;
            }
            if (a.dgi) {
                float* di = a.dgi + ob;
                di[unit] = cdar; di[D + unit] = cdaz; di[2 * D + unit] = cdan;
            }
            if (a.dgi_lp) {
                unsigned short* dj = reinterpret_cast<unsigned short*>(a.dgi_lp + ob);
                if (nts) {
                    __builtin_nontemporal_store(har, dj + unit);
                    __builtin_nontemporal_store(haz, dj + D + unit);
                    __builtin_nontemporal_store(han, dj + 2 * D + unit);
                } else {
                    dj[unit] = har; dj[D + unit] = haz; dj[2 * D + unit] = han;
                }
            }
            if (MT == 1) {
                sar1 += cdar; saz1 += cdaz; sghn1 += cdghn; san1 += cdan;
            } else {
                q[NTHR] += cdar; q[2 * NTHR] += cdaz; q[3 * NTHR] += cdghn; q[4 * NTHR] += cdan;
            }
            if (t == 0) a.ddir0[(int64_t)row * D + unit] = o.ddir;
        }
    }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int row = row_of(m);
        if (a.bsum && rv && row < B) {
            float* bs = a.bsum + (int64_t)row * 4 * D;
            if (MT == 1) {
                bs[unit] = sar1; bs[D + unit] = saz1; bs[2 * D + unit] = sghn1;
                bs[3 * D + unit] = san1;
            } else {
                const float* q = sl + (m * 5) * NTHR + tid;
                bs[unit] = q[NTHR]; bs[D + unit] = q[2 * NTHR]; bs[2 * D + unit] = q[3 * NTHR];
                bs[3 * D + unit] = q[4 * NTHR];
            }
        }
    }
    gx_note_failure(a.err, a.sticky);
}

// ------------------------------------------------------------------ host side

static unsigned long long*& gx_diag_buf() {
    static unsigned long long* p = nullptr;
    return p;
}

// timing diagnostics only (SRNN_GRU_DIAG=1): prints the first armed launch's stamps
extern "C" int srnn_gru_diag_dump(void) {
    unsigned long long h[256];
    if (!gx_diag_buf() || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(h, gx_diag_buf(), sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
        return 1;
    fprintf(stderr, "gru_xcd diag mode: %s\n", h[255] == 1 ? "xcd-local" : "static map");
    for (int k = 1; k < 255 && h[k]; ++k)
        fprintf(stderr, "gru_xcd diag %3d: +%8.2f us\n", k, (double)(h[k] - h[k - 1]) / 100.0);
    return 0;
}

// CUs one process's sweep may count on: the device's, divided among the processes that run
// persistent kernels on it at once (persist.hip, srnn_set_device_share) -- every launch's
// G x P workgroups then fit beside theirs (handoff.hpp co-residency)
static int gx_cus() {
    return srnn_device_cus() / srnn_device_share();
}

// Row layout of one launch for B rows at width D (GruXArgs): false if the device or shape
// is not supported.  B beyond what one launch holds (16 MAXMT rows per group) is run as
// several launches of gx_launch_rows(D) rows each (srnn_gru_xcd_fwd2 / bwd2).
struct GxLayout { int mt, G, rv, P; };

static int gx_launch_rows(int D) {
    const int ncu = gx_cus();
    if (ncu <= 0 || D % 256 != 0 || D > 1024) return 0;
    return (ncu / (D / gx::CU)) * gx::RG * gx::MAXMT;
}

static bool gx_layout(int B, int D, GxLayout& L) {
    const int ncu = gx_cus();
    if (ncu <= 0 || B <= 0 || D % 256 != 0 || D > 1024) return false;
    L.P = D / gx::CU;
    const int gmax = ncu / L.P;
    if (gmax < 1) return false;
    L.mt = 1;
    while (L.mt < gx::MAXMT && cdiv(B, gx::RG * L.mt) > gmax) L.mt *= 2;
    int G = cdiv(B, gx::RG * L.mt);
    if (G > gmax) return false;
    // whole groups of 8: with the round-robin dealing every group then sits on one XCD, and a
    // small batch spreads over all of them (fewer rows per group, e.g. 8 at B = 64)
    L.G = (G + 7) / 8 * 8 <= gmax ? (G + 7) / 8 * 8 : G;
    L.rv = cdiv(B, L.G * L.mt);
    return L.rv <= gx::RG;
}

// work-buffer bytes of srnn_gru_xcd_fwd for (B, D); 0 if the shape / device is not supported
extern "C" size_t srnn_gru_xcd_work_bytes(int dtype, int B, int D) {
    if (dtype != SRNN_BF16 || B <= 0) return 0;
    const int lr = gx_launch_rows(D);
    GxLayout L;
    if (lr <= 0 || !gx_layout(B < lr ? B : lr, D, L)) return 0;
    return gx::HDR + (size_t)2 * L.G * L.mt * gx::RG * (D / 2) * 8;
}

extern "C" int srnn_gru_xcd_fwd2(int dtype, int B, int D, int Fr, const float* gi, int64_t ldgi,
                                 int64_t sgi, const float* h0, const void* whh, const float* bhh,
                                 float* out, void* out_lp, int64_t ldo, int64_t so, float* gates,
                                 int64_t ldg, int64_t sg, void* hprev_lp, void* work,
                                 size_t work_bytes, void* stream) {
    const size_t need = srnn_gru_xcd_work_bytes(dtype, B, D);
    SRNN_REQUIRE(need > 0, "gru_xcd: shape/device not supported");
    SRNN_REQUIRE(work && work_bytes >= need, "gru_xcd: workspace %zu < %zu", work_bytes, need);
    if (Fr <= 0) return 0;
    const int lr = gx_launch_rows(D);
    if (B > lr) {     // rows are independent: consecutive launches over row chunks
        for (int c = 0; c < B; c += lr) {
            const int n = B - c < lr ? B - c : lr;
            const int rc = srnn_gru_xcd_fwd2(
                dtype, n, D, Fr, gi + (int64_t)c * ldgi, ldgi, sgi, h0 + (int64_t)c * D, whh,
                bhh, out + (int64_t)c * ldo, (bf16*)out_lp + (int64_t)c * ldo, ldo, so,
                gates + (int64_t)c * ldg, ldg, sg,
                hprev_lp ? (void*)((bf16*)hprev_lp + (int64_t)c * ldo) : nullptr, work,
                work_bytes, stream);
            if (rc) return rc;
        }
        return 0;
    }
    GxLayout L;
    SRNN_REQUIRE(gx_layout(B, D, L), "gru_xcd: no row layout for B=%d D=%d", B, D);
    hipStream_t s = (hipStream_t)stream;
    // granules, census and error word start zeroed every call (tags count from 1)
    SRNN_CHECK_HIP(hipMemsetAsync(work, 0, need, s));
    GruXArgs a;
    a.gi = gi; a.ldgi = ldgi; a.sgi = sgi;
    a.h0 = h0; a.whh = (const bf16*)whh; a.bhh = bhh;
    a.out = out; a.out_lp = (bf16*)out_lp; a.ldo = ldo; a.so = so;
    a.hp_lp = (bf16*)hprev_lp;
    a.gates = gates; a.ldg = ldg; a.sg = sg;
    a.err = (int*)work;
    a.sticky = srnn_sticky_flag();
    SRNN_REQUIRE(a.sticky, "gru_xcd: sticky flag allocation failed");
    a.spin_limit = srnn_persist_spin_limit(hx::SPIN_LIMIT);
    a.withhold = env_flag("SRNN_PERSIST_FORCE_FAIL", 0);
    a.census = (int*)work + 16;
    a.nolocal = !env_flag("SRNN_GEN_LOCAL", 1);
    a.xh = (u64*)((char*)work + gx::HDR);
    a.B = B; a.D = D; a.Fr = Fr;
    a.diag = nullptr;
    a.poll_sleep = env_flag("SRNN_POLL_SLEEP", 1);
    a.exp = env_flag("SRNN_GX_EXP", 0);
    {
        static unsigned long long* diag = nullptr;
        static int armed = -1;
        if (armed < 0) armed = env_flag("SRNN_GRU_DIAG", 0);
        if (armed == 1 && Fr >= 32 && hipMalloc(&diag, 256 * 8) == hipSuccess) {
            SRNN_CHECK_HIP(hipMemsetAsync(diag, 0, 256 * 8, s));
            a.diag = diag;
            armed = 2;
            gx_diag_buf() = diag;
        }
    }
    a.G = L.G;
    a.P = L.P;
    a.RV = L.rv;
    const int NU = D / gx::UK;
    const int KW = NU < gx::NW ? NU : gx::NW;
    const size_t lds = (size_t)2 * KW * gx::NT * 4 * gx::PS * 4 + 16;
    const int upw = cdiv(NU, gx::NW);
    const int ui = upw <= 1 ? 0 : upw <= 2 ? 1 : 2;
    const int mi = L.mt == 1 ? 0 : L.mt == 2 ? 1 : 2;
    typedef void (*FwdK)(GruXArgs);
    static const FwdK ks[3][3] = {
        {gru_xcd_fwd_kernel<1, 1>, gru_xcd_fwd_kernel<1, 2>, gru_xcd_fwd_kernel<1, 4>},
        {gru_xcd_fwd_kernel<2, 1>, gru_xcd_fwd_kernel<2, 2>, gru_xcd_fwd_kernel<2, 4>},
        {gru_xcd_fwd_kernel<4, 1>, gru_xcd_fwd_kernel<4, 2>, gru_xcd_fwd_kernel<4, 4>}};
    static const FwdK k1024[3] = {gru_xcd_fwd_kernel<4, 1, 1024>, gru_xcd_fwd_kernel<4, 2, 1024>,
                                  gru_xcd_fwd_kernel<4, 4, 1024>};
    const FwdK k = D == 1024 && env_flag("SRNN_GX_DC", 1) ? k1024[mi] : ks[ui][mi];
    static bool attr[4][3] = {};
    const int ai = k == ks[ui][mi] ? ui : 3;
    if (!attr[ai][mi]) {
        SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)k,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           160 * 1024));
        attr[ai][mi] = true;
    }
    if (srnn_persist_check((const void*)k, gx::NTHR, lds, (int64_t)a.G * a.P, "gru_xcd_fwd"))
        return 1;
    hipLaunchKernelGGL(k, dim3(a.G * a.P), dim3(gx::NTHR), lds, s, a);
    SRNN_LAUNCH_CHECK();
    return 0;
}

extern "C" int srnn_gru_xcd_fwd(int dtype, int B, int D, int Fr, const float* gi, int64_t ldgi,
                                int64_t sgi, const float* h0, const void* whh, const float* bhh,
                                float* out, void* out_lp, int64_t ldo, int64_t so, float* gates,
                                int64_t ldg, int64_t sg, void* work, size_t work_bytes,
                                void* stream) {
    return srnn_gru_xcd_fwd2(dtype, B, D, Fr, gi, ldgi, sgi, h0, whh, bhh, out, out_lp, ldo, so,
                             gates, ldg, sg, nullptr, work, work_bytes, stream);
}


// work-buffer bytes of srnn_gru_xcd_bwd for (B, D); 0 if not supported
extern "C" size_t srnn_gru_xcd_bwd_work_bytes(int dtype, int B, int D) {
    if (!srnn_gru_xcd_work_bytes(dtype, B, D)) return 0;
    const int lr = gx_launch_rows(D);
    GxLayout L;
    if (!gx_layout(B < lr ? B : lr, D, L)) return 0;
    return gx::HDR + (size_t)2 * L.G * L.mt * gx::RG * (3 * D / 2) * 8;
}

extern "C" int srnn_gru_xcd_bwd2(int dtype, int B, int D, int Fr, const float* dy, int64_t lddy,
                                 int64_t sdy, const float* gates, int64_t ldg, int64_t sg,
                                 const float* hout, int64_t ldo, int64_t so, const float* h0,
                                 const void* whh_t, float* dgh, void* dgh_lp, float* dgi,
                                 void* dgi_lp, float* bsum, int64_t ldd, int64_t sd, float* ddir0,
                                 void* work, size_t work_bytes, void* stream) {
    const size_t need = srnn_gru_xcd_bwd_work_bytes(dtype, B, D);
    SRNN_REQUIRE(need > 0, "gru_xcd_bwd: shape/device not supported");
    SRNN_REQUIRE(work && work_bytes >= need, "gru_xcd_bwd: workspace %zu < %zu", work_bytes, need);
    SRNN_REQUIRE(dgh_lp, "gru_xcd_bwd: dgh_lp is required");
    if (Fr <= 0) return 0;
    const int lr = gx_launch_rows(D);
    if (B > lr) {     // rows are independent: consecutive launches over row chunks
        for (int c = 0; c < B; c += lr) {
            const int n = B - c < lr ? B - c : lr;
            const int rc = srnn_gru_xcd_bwd2(
                dtype, n, D, Fr, dy + (int64_t)c * lddy, lddy, sdy, gates + (int64_t)c * ldg,
                ldg, sg, hout + (int64_t)c * ldo, ldo, so, h0 + (int64_t)c * D, whh_t,
                dgh ? dgh + (int64_t)c * ldd : nullptr, (bf16*)dgh_lp + (int64_t)c * ldd,
                dgi ? dgi + (int64_t)c * ldd : nullptr,
                dgi_lp ? (void*)((bf16*)dgi_lp + (int64_t)c * ldd) : nullptr,
                bsum ? bsum + (int64_t)c * 4 * D : nullptr, ldd, sd, ddir0 + (int64_t)c * D,
                work, work_bytes, stream);
            if (rc) return rc;
        }
        return 0;
    }
    GxLayout L;
    SRNN_REQUIRE(gx_layout(B, D, L), "gru_xcd_bwd: no row layout for B=%d D=%d", B, D);
    hipStream_t s = (hipStream_t)stream;
    // packed hand-off form (gru_xcd_bwd_pk_kernel): one {3 x bf16, tag} granule per unit;
    // tags (<= Fr) must stay finite bf16 patterns (< 0x7f80); SRNN_GX_PK=0 restores the form
    // with {2 x bf16, 32-bit tag} granules
    // (the packed kernel's operand fetch uses 32-bit buffer offsets: a launch with any byte
    //  offset past 2 GB -- very long sequences -- takes the unpacked kernel's 64-bit pointers)
    const int64_t omax = std::max({((int64_t)(B - 1) * lddy + (int64_t)(Fr - 1) * sdy + D) * 4,
                                   ((int64_t)(B - 1) * ldg + (int64_t)(Fr - 1) * sg + 4 * D) * 4,
                                   ((int64_t)(B - 1) * ldo + (int64_t)(Fr - 1) * so + D) * 4,
                                   (int64_t)B * D * 4});
    const bool pk = D % 64 == 0 && D / 64 <= 16 && (D / 64) % 4 == 0 && Fr < 0x7f80 &&
                    omax < 0x7fffffffll - 64 && env_flag("SRNN_GX_PK", 1);
    const size_t clear = pk ? gx::HDR + (size_t)2 * L.G * L.mt * gx::RG * D * 8 : need;
    SRNN_CHECK_HIP(hipMemsetAsync(work, 0, clear, s));
    GruXBwdArgs a;
    a.dy = dy; a.lddy = lddy; a.sdy = sdy;
    a.gates = gates; a.ldg = ldg; a.sg = sg;
    a.hout = hout; a.ldo = ldo; a.so = so; a.h0 = h0;
    a.whh_t = (const bf16*)whh_t;
    a.dgh = dgh; a.dgh_lp = (bf16*)dgh_lp; a.dgi = dgi; a.ldd = ldd; a.sd = sd;
    a.dgi_lp = (bf16*)dgi_lp; a.bsum = bsum;
    a.ddir0 = ddir0;
    a.err = (int*)work;
    a.sticky = srnn_sticky_flag();
    SRNN_REQUIRE(a.sticky, "gru_xcd_bwd: sticky flag allocation failed");
    a.spin_limit = srnn_persist_spin_limit(hx::SPIN_LIMIT);
    a.withhold = env_flag("SRNN_PERSIST_FORCE_FAIL", 0);
    a.census = (int*)work + 16;
    a.nolocal = !env_flag("SRNN_GEN_LOCAL", 1);
    a.xg = (u64*)((char*)work + gx::HDR);
    a.B = B; a.D = D; a.Fr = Fr;
    a.exp = env_flag("SRNN_GX_EXP", 0);
    a.G = L.G;
    a.P = L.P;
    a.RV = L.rv;
    const int NU = 3 * D / gx::UK;
    const int KW = pk ? gx::NW : NU < gx::NW ? NU : gx::NW;
    size_t lds = (size_t)2 * KW * 2 * 4 * gx::PS * 4 + 64 +
                 (L.mt > 1 ? (size_t)L.mt * 5 * gx::NTHR * 4 : 0);
    if (pk) {
        // (the prologue stages 32 W_hh^T rows of one gate in the same dynamic LDS)
        const size_t stage = (size_t)32 * (2 * D + 16);
        if (lds < stage) lds = stage;
        typedef void (*PkK)(GruXBwdArgs);
        static const PkK kp[4][3] = {
            {gru_xcd_bwd_pk_kernel<4, 1>, gru_xcd_bwd_pk_kernel<4, 2>, gru_xcd_bwd_pk_kernel<4, 4>},
            {gru_xcd_bwd_pk_kernel<8, 1>, gru_xcd_bwd_pk_kernel<8, 2>, gru_xcd_bwd_pk_kernel<8, 4>},
            {gru_xcd_bwd_pk_kernel<12, 1>, gru_xcd_bwd_pk_kernel<12, 2>,
             gru_xcd_bwd_pk_kernel<12, 4>},
            {gru_xcd_bwd_pk_kernel<16, 1>, gru_xcd_bwd_pk_kernel<16, 2>,
             gru_xcd_bwd_pk_kernel<16, 4>}};
        const int mi = L.mt == 1 ? 0 : L.mt == 2 ? 1 : 2;
        const PkK k = kp[D / 256 - 1][mi];
        static bool attr[4][3] = {};
        if (!attr[D / 256 - 1][mi]) {
            SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)k,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               160 * 1024));
            attr[D / 256 - 1][mi] = true;
        }
        if (srnn_persist_check((const void*)k, gx::NTHR, lds, (int64_t)a.G * a.P, "gru_xcd_bwd"))
            return 1;
        hipLaunchKernelGGL(k, dim3(a.G * a.P), dim3(gx::NTHR), lds, s, a);
        SRNN_LAUNCH_CHECK();
        return 0;
    }
    const int upw = cdiv(NU, gx::NW);
    const int ui = upw <= 3 ? 0 : upw <= 6 ? 1 : 2;
    const bool full = NU == (ui == 0 ? 3 : ui == 1 ? 6 : 12) * gx::NW;
    const int mi = L.mt == 1 ? 0 : L.mt == 2 ? 1 : 2;
    typedef void (*BwdK)(GruXBwdArgs);
    // FULL holds for D = 256 / 512 / 1024 (UPW = 3 / 6 / 12); D = 768 takes the UPW = 12 form
    static const BwdK ks[2][3][3] = {
        {{nullptr, nullptr, nullptr},
         {nullptr, nullptr, nullptr},
         {gru_xcd_bwd_kernel<12, false, 1>, gru_xcd_bwd_kernel<12, false, 2>,
          gru_xcd_bwd_kernel<12, false, 4>}},
        {{gru_xcd_bwd_kernel<3, true, 1>, gru_xcd_bwd_kernel<3, true, 2>,
          gru_xcd_bwd_kernel<3, true, 4>},
         {gru_xcd_bwd_kernel<6, true, 1>, gru_xcd_bwd_kernel<6, true, 2>,
          gru_xcd_bwd_kernel<6, true, 4>},
         {gru_xcd_bwd_kernel<12, true, 1>, gru_xcd_bwd_kernel<12, true, 2>,
          gru_xcd_bwd_kernel<12, true, 4>}}};
    const BwdK k = ks[full ? 1 : 0][ui][mi];
    SRNN_REQUIRE(k, "gru_xcd_bwd: no kernel for D=%d", D);
    if (srnn_persist_check((const void*)k, gx::NTHR, lds, (int64_t)a.G * a.P, "gru_xcd_bwd"))
        return 1;
    hipLaunchKernelGGL(k, dim3(a.G * a.P), dim3(gx::NTHR), lds, s, a);
    SRNN_LAUNCH_CHECK();
    return 0;
}

extern "C" int srnn_gru_xcd_bwd(int dtype, int B, int D, int Fr, const float* dy, int64_t lddy,
                                int64_t sdy, const float* gates, int64_t ldg, int64_t sg,
                                const float* hout, int64_t ldo, int64_t so, const float* h0,
                                const void* whh_t, float* dgh, void* dgh_lp, float* dgi,
                                int64_t ldd, int64_t sd, float* ddir0, void* work,
                                size_t work_bytes, void* stream) {
    return srnn_gru_xcd_bwd2(dtype, B, D, Fr, dy, lddy, sdy, gates, ldg, sg, hout, ldo, so, h0,
                             whh_t, dgh, dgh_lp, dgi, nullptr, nullptr, ldd, sd, ddir0, work,
                             work_bytes, stream);
}

// nonzero if the previous srnn_gru_xcd_fwd/bwd on `work` gave up a hand-off (synchronises)
extern "C" int srnn_gru_xcd_error(const void* work) {
    int e = 0;
    if (hipMemcpy(&e, work, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return e;
}
