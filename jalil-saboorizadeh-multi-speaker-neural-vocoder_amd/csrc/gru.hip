// GRU recurrence for the FrameLevelRNN tiers (torch.nn.GRU semantics, model.py:148-165,
// 244; gate order [r | z | n]):
//     r = sig(gi_r + gh_r)   z = sig(gi_z + gh_z)   n = tanh(gi_n + r * gh_n)
//     h' = (h - n) * z + n
// One launch per time step.  A workgroup owns BM batch rows x 16 hidden units and
// computes the 3 x 16 gate columns of h . W_hh^T (and optionally x . W_ih^T) on MFMA
// (RowGate remaps the tile's B rows to the r/z/n weight rows of its units), so each
// lane ends up holding r, z, n of the same (row, unit) and the whole gate update is a
// register epilogue -- no gate tensor round-trips HBM.  The backward step is the mirror
// image: dh_t = dy_t + dh_direct + dgh_{t+1} . W_hh (MFMA over K = 3D), then the gate
// backward in the epilogue.
#include "gemm_core.hpp"
#include "ring_core.hpp"
#include "gru_point.hpp"
#include "samplernn_hip_internal.hpp"

// ring depth of the per-step GRU kernels: 8 slots (7 k-stages in flight) fit the 160 KiB
// LDS and put nearly the whole W_hh slice + h rows of a step in flight at once
#define GRU_NS 8

struct GruCellArgs {
    const void* x;      // layer input (T), row stride ldx; null -> use gi
    int64_t ldx;
    const void* wih;    // (3D, Din) T
    const float* bih;   // (3D)
    const float* gi;    // precomputed x.W_ih^T + b_ih (fp32), row stride ldgi
    int64_t ldgi;
    const void* h;      // h_{t-1} (T) row stride ldh
    int64_t ldh;
    const float* hf;    // h_{t-1} fp32
    int64_t ldhf;
    const void* whh;    // (3D, D) T
    const float* bhh;
    float* hout;        // h_t fp32
    int64_t ldho;
    void* hout_lp;      // optional h_t (T) copy
    int64_t ldhl;
    float* gates;       // optional saved r|z|n|ghn, row stride ldgt (4D per row)
    int64_t ldgt;
    const float* ghp;   // optional precomputed h.W_hh^T + b_hh (fp32), row stride ldghp: the
    int64_t ldghp;      // h GEMM is skipped (ring kernel only)
    const float* gadd;  // optional per-row term added to x.W_ih^T (fp32), row stride ldgadd
    int64_t ldgadd;     // (ring kernel only)
    int B, D, Din;
    int vec_x, vec_h, vec_wih, vec_whh;
};

template <typename T, int BM>
__global__ __launch_bounds__(256) void gru_cell_kernel(GruCellArgs a) {
    constexpr int WM = BM / 16, WK = 4 / WM;
    typedef GemmCfg<T, BM, 48, 4, WM, 1, WK> C;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int u0 = blockIdx.x * 16, m0 = blockIdx.y * BM;
    floatx4 acc_h[C::FM][3], acc_i[C::FM][3];
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc_h[i][j] = acc_i[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const RowGate gmap{u0, 16, a.D};
    if (a.x) {
        gemm_core<T, BM, 48, 4, WM, 1, WK, true, true>(
            (const T*)a.x, a.ldx, RowIdentity{m0, a.B}, m0, a.B, a.vec_x != 0, (const T*)a.wih,
            a.Din, gmap, 0, 3 * a.D, a.vec_wih != 0, a.Din, smem, acc_i);
    }
    gemm_core<T, BM, 48, 4, WM, 1, WK, true, true>(
        (const T*)a.h, a.ldh, RowIdentity{m0, a.B}, m0, a.B, a.vec_h != 0, (const T*)a.whh, a.D,
        gmap, 0, 3 * a.D, a.vec_whh != 0, a.D, smem, acc_h);
    if (a.x) {
        wk_reduce<T, BM, 48, 4, WM, 1, WK>(smem, acc_i);
        __syncthreads();
    }
    wk_reduce<T, BM, 48, 4, WM, 1, WK>(smem, acc_h);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = wave % WM, wk = wave / WM;
    if (wk != 0) return;
    const int u = u0 + (lane & 15);
    if (u >= a.D) return;
    const int D = a.D;
    const float bhr = a.bhh[u], bhz = a.bhh[D + u], bhn = a.bhh[2 * D + u];
    float bir = 0.f, biz = 0.f, bin = 0.f;
    if (a.x) { bir = a.bih[u]; biz = a.bih[D + u]; bin = a.bih[2 * D + u]; }
#pragma unroll
    for (int fm = 0; fm < C::FM; ++fm)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = m0 + wm * C::FM * 16 + fm * 16 + (lane >> 4) * 4 + i;
            if (row >= a.B) continue;
            float gir, giz, gin;
            if (a.x) {
                gir = acc_i[fm][0][i] + bir;
                giz = acc_i[fm][1][i] + biz;
                gin = acc_i[fm][2][i] + bin;
            } else {
                const float* g = a.gi + (int64_t)row * a.ldgi;
                gir = g[u]; giz = g[D + u]; gin = g[2 * D + u];
            }
            const float ghr = acc_h[fm][0][i] + bhr;
            const float ghz = acc_h[fm][1][i] + bhz;
            const float ghn = acc_h[fm][2][i] + bhn;
            const float r = 1.0f / (1.0f + expf(-(ghr + gir)));
            const float z = 1.0f / (1.0f + expf(-(ghz + giz)));
            const float n = tanhf(gin + ghn * r);
            const float hp = a.hf[(int64_t)row * a.ldhf + u];
            const float hn = (hp - n) * z + n;
            a.hout[(int64_t)row * a.ldho + u] = hn;
            if (a.hout_lp) ((T*)a.hout_lp)[(int64_t)row * a.ldhl + u] = from_f<T>(hn);
            if (a.gates) {
                float* gt = a.gates + (int64_t)row * a.ldgt;
                gt[u] = r; gt[D + u] = z; gt[2 * D + u] = n; gt[3 * D + u] = ghn;
            }
        }
}

static inline bool al16(const void* p, int64_t ld, int es) {
    return ((uintptr_t)p % 16 == 0) && ((ld * es) % 16 == 0);
}

// Ring variant (ring_core.hpp): same tile (32 rows x 3 gates x 16 units), NS-1 k-stages
// of both operands in flight.  Needs D (and Din) multiples of the ring stage.
template <typename T>
__global__ __launch_bounds__(256) void gru_cell_ring_kernel(GruCellArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int u0 = blockIdx.x * 16, m0 = blockIdx.y * 32;
    floatx4 acc_h[1][3], acc_i[1][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) acc_h[0][j] = acc_i[0][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const RowGateClamp gmap{u0, 16, a.D};
    if (a.x)
        ring_core<T, 32, 48, 2, 1, 2, GRU_NS>((const T*)a.x, a.ldx, RowClamp{m0, a.B}, (const T*)a.wih,
                                         a.Din, gmap, a.Din, smem, acc_i);
    if (!a.ghp)
        ring_core<T, 32, 48, 2, 1, 2, GRU_NS>((const T*)a.h, a.ldh, RowClamp{m0, a.B},
                                             (const T*)a.whh, a.D, gmap, a.D, smem, acc_h);
    if (a.x) ring_reduce<T, 32, 48, 2, 1, 2, GRU_NS>(smem, acc_i);
    if (!a.ghp) ring_reduce<T, 32, 48, 2, 1, 2, GRU_NS>(smem, acc_h);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = wave % 2, wk = wave / 2;
    if (wk != 0) return;
    const int u = u0 + (lane & 15);
    if (u >= a.D) return;
    const int D = a.D;
    const float bhr = a.ghp ? 0.f : a.bhh[u], bhz = a.ghp ? 0.f : a.bhh[D + u];
    const float bhn = a.ghp ? 0.f : a.bhh[2 * D + u];
    float bir = 0.f, biz = 0.f, bin = 0.f;
    if (a.x && a.bih) { bir = a.bih[u]; biz = a.bih[D + u]; bin = a.bih[2 * D + u]; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = m0 + wm * 16 + (lane >> 4) * 4 + i;
        if (row >= a.B) continue;
        float gir, giz, gin;
        if (a.x) {
            gir = acc_i[0][0][i] + bir; giz = acc_i[0][1][i] + biz; gin = acc_i[0][2][i] + bin;
            if (a.gadd) {
                const float* ga = a.gadd + (int64_t)row * a.ldgadd;
                gir += ga[u]; giz += ga[D + u]; gin += ga[2 * D + u];
            }
        } else {
            const float* g = a.gi + (int64_t)row * a.ldgi;
            gir = g[u]; giz = g[D + u]; gin = g[2 * D + u];
        }
        float ghr, ghz, ghn;
        if (a.ghp) {
            const float* g = a.ghp + (int64_t)row * a.ldghp;
            ghr = g[u]; ghz = g[D + u]; ghn = g[2 * D + u];
        } else {
            ghr = acc_h[0][0][i] + bhr; ghz = acc_h[0][1][i] + bhz; ghn = acc_h[0][2][i] + bhn;
        }
        const float r = 1.0f / (1.0f + expf(-(ghr + gir)));
        const float z = 1.0f / (1.0f + expf(-(ghz + giz)));
        const float n = tanhf(gin + ghn * r);
        const float hp = a.hf[(int64_t)row * a.ldhf + u];
        const float hn = (hp - n) * z + n;
        a.hout[(int64_t)row * a.ldho + u] = hn;
        if (a.hout_lp) ((T*)a.hout_lp)[(int64_t)row * a.ldhl + u] = from_f<T>(hn);
        if (a.gates) {
            float* gt = a.gates + (int64_t)row * a.ldgt;
            gt[u] = r; gt[D + u] = z; gt[2 * D + u] = n; gt[3 * D + u] = ghn;
        }
    }
}

template <typename T, int BM>
static int launch_cell(GruCellArgs& a, hipStream_t s) {
    typedef Ring<T, 32, 48, 2, 1, 2, GRU_NS> R;
    const int es = (int)sizeof(T);
    const bool ring = a.D % R::KB == 0 && (!a.x || a.Din % R::KB == 0) && a.vec_h && a.vec_whh &&
                      (!a.x || (a.vec_x && a.vec_wih));
    SRNN_REQUIRE(ring || (!a.ghp && !a.gadd), "gru_cell: precomputed gh / gadd need the ring shape");
    if (ring) {
        static bool attr = false;
        if (!attr) {
            SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)gru_cell_ring_kernel<T>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, R::LDS));
            attr = true;
        }
        dim3 grid(cdiv(a.D, 16), cdiv(a.B, 32));
        hipLaunchKernelGGL((gru_cell_ring_kernel<T>), grid, dim3(256), R::LDS, s, a);
        SRNN_LAUNCH_CHECK();
        (void)es;
        return 0;
    }
    constexpr int WM = BM / 16, WK = 4 / WM;
    typedef GemmCfg<T, BM, 48, 4, WM, 1, WK> C;
    dim3 grid(cdiv(a.D, 16), cdiv(a.B, BM));
    hipLaunchKernelGGL((gru_cell_kernel<T, BM>), grid, dim3(256), C::LDS, s, a);
    SRNN_LAUNCH_CHECK();
    return 0;
}

int srnn_gru_cell_impl(int dtype, int B, int D, int Din, const void* x, int64_t ldx,
                       const void* wih, const float* bih, const float* gi, int64_t ldgi,
                       const void* h, int64_t ldh, const float* hf, int64_t ldhf, const void* whh,
                       const float* bhh, float* hout, int64_t ldho, void* hout_lp, int64_t ldhl,
                       float* gates, int64_t ldgt, hipStream_t s) {
    SRNN_REQUIRE(B > 0 && D > 0, "gru_cell: bad sizes");
    SRNN_REQUIRE(x || gi, "gru_cell: need x or gi");
    const int es = dtype == SRNN_F32 ? 4 : 2;
    GruCellArgs a;
    a.x = x; a.ldx = ldx; a.wih = wih; a.bih = bih; a.gi = gi; a.ldgi = ldgi;
    a.h = h; a.ldh = ldh; a.hf = hf; a.ldhf = ldhf; a.whh = whh; a.bhh = bhh;
    a.hout = hout; a.ldho = ldho; a.hout_lp = hout_lp; a.ldhl = ldhl;
    a.gates = gates; a.ldgt = ldgt; a.B = B; a.D = D; a.Din = Din;
    a.ghp = nullptr; a.ldghp = 0;
    a.gadd = nullptr; a.ldgadd = 0;
    a.vec_x = x ? al16(x, ldx, es) : 0;
    a.vec_h = al16(h, ldh, es);
    a.vec_wih = x ? al16(wih, Din, es) : 0;
    a.vec_whh = al16(whh, D, es);
    // 32-row tiles give >= 256 workgroups at B = 128, D = 1024
    if (dtype == SRNN_F32) return launch_cell<float, 32>(a, s);
    return launch_cell<bf16, 32>(a, s);
}

// GRU cell with h . W_hh^T + b_hh precomputed (the generation loop's folded upper tick carries
// it in the previous tick's upsampling GEMM): gi = x . W_ih^T (+ b_ih) (+ gadd[row]) on MFMA
// (x: B x Din), then the gate update
int srnn_gru_cell_x_impl(int dtype, int B, int D, int Din, const void* x, int64_t ldx,
                         const void* wih, const float* bih, const float* gadd, int64_t ldgadd,
                         const float* gh, int64_t ldgh, const float* hf, int64_t ldhf, float* hout,
                         int64_t ldho, void* hout_lp, int64_t ldhl, hipStream_t s) {
    SRNN_REQUIRE(B > 0 && D > 0 && x && gh, "gru_cell_x: bad args");
    const int es = dtype == SRNN_F32 ? 4 : 2;
    GruCellArgs a;
    memset(&a, 0, sizeof(a));
    a.x = x; a.ldx = ldx; a.wih = wih; a.bih = bih;
    a.hf = hf; a.ldhf = ldhf;
    a.hout = hout; a.ldho = ldho; a.hout_lp = hout_lp; a.ldhl = ldhl;
    a.ghp = gh; a.ldghp = ldgh;
    a.gadd = gadd; a.ldgadd = ldgadd;
    a.B = B; a.D = D; a.Din = Din;
    a.vec_x = al16(x, ldx, es);
    a.vec_h = 1;
    a.vec_wih = al16(wih, Din, es);
    a.vec_whh = 1;
    if (dtype == SRNN_F32) return launch_cell<float, 32>(a, s);
    return launch_cell<bf16, 32>(a, s);
}

// ------------------------------------------------------------------ backward step
// dh = dy + ddir_next + dgh_next . W_hh        (W_hh (3D, D) is the K x N operand)
// dn = dh (1-z); dz = dh (h_prev - n); ddir = dh z
// dan = dn (1 - n^2); dr = dan ghn; dar = dr r (1-r); daz = dz z (1-z)
// dgh = [dar | daz | dan r],  dgi = [dar | daz | dan]
struct GruBwdArgs {
    const float* dy; int64_t lddy;
    const void* dgh_next; int64_t lddgn;
    const float* ddir_next;        // (B, D) contiguous or null
    const void* whh;               // (3D, D) or null
    const void* whh_t;             // (D, 3D) = W_hh^T or null (ring path)
    const float* gates; int64_t ldgt;
    const float* hprev; int64_t ldhp;
    float* dgh; int64_t lddgh;
    void* dgh_lp; int64_t lddghl;
    float* dgi; int64_t lddgi;
    float* ddir;                   // (B, D) contiguous
    int B, D;
    int vec_dgn, vec_whh, vec_wt;
};

template <typename T>
__device__ __forceinline__ void gru_bwd_epilogue(const GruBwdArgs& a, int row, int u, float acc) {
    const int D = a.D;
    float dh = acc + a.dy[(int64_t)row * a.lddy + u];
    if (a.ddir_next) dh += a.ddir_next[(int64_t)row * D + u];
    const float* g = a.gates + (int64_t)row * a.ldgt;
    const float r = g[u], z = g[D + u], n = g[2 * D + u], ghn = g[3 * D + u];
    const float hp = a.hprev[(int64_t)row * a.ldhp + u];
    const GruBwdPoint o = gru_bwd_point(dh, r, z, n, ghn, hp);
    const float dar = o.dar, daz = o.daz, dghn = o.dghn, dan = o.dan;
    float* dgh = a.dgh + (int64_t)row * a.lddgh;
    dgh[u] = dar; dgh[D + u] = daz; dgh[2 * D + u] = dghn;
    if (a.dgh_lp) {
        T* dl = (T*)a.dgh_lp + (int64_t)row * a.lddghl;
        dl[u] = from_f<T>(dar); dl[D + u] = from_f<T>(daz); dl[2 * D + u] = from_f<T>(dghn);
    }
    float* dgi = a.dgi + (int64_t)row * a.lddgi;
    dgi[u] = dar; dgi[D + u] = daz; dgi[2 * D + u] = dan;
    a.ddir[(int64_t)row * D + u] = o.ddir;
}

template <typename T, int BM>
__global__ __launch_bounds__(256) void gru_bwd_kernel(GruBwdArgs a) {
    constexpr int WM = BM / 16, WK = 4 / WM;
    typedef GemmCfg<T, BM, 16, 4, WM, 1, WK> C;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int u0 = blockIdx.x * 16, m0 = blockIdx.y * BM;
    const int D = a.D;
    floatx4 acc[C::FM][1];
#pragma unroll
    for (int i = 0; i < C::FM; ++i) acc[i][0] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (a.dgh_next) {
        gemm_core<T, BM, 16, 4, WM, 1, WK, true, false>(
            (const T*)a.dgh_next, a.lddgn, RowIdentity{m0, a.B}, m0, a.B, a.vec_dgn != 0,
            (const T*)a.whh, D, RowIdentity{0, 0}, u0, D, a.vec_whh != 0, 3 * D, smem, acc);
        wk_reduce<T, BM, 16, 4, WM, 1, WK>(smem, acc);
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = wave % WM, wk = wave / WM;
    if (wk != 0) return;
    const int u = u0 + (lane & 15);
    if (u >= D) return;
#pragma unroll
    for (int fm = 0; fm < C::FM; ++fm)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = m0 + wm * C::FM * 16 + fm * 16 + (lane >> 4) * 4 + i;
            if (row < a.B) gru_bwd_epilogue<T>(a, row, u, acc[fm][0][i]);
        }
}

// ring variant: dgh_next (B, 3D) . W_hh^T^T with W_hh^T (D, 3D) k-contiguous
template <typename T>
__global__ __launch_bounds__(256) void gru_bwd_ring_kernel(GruBwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int u0 = blockIdx.x * 16, m0 = blockIdx.y * 32;
    const int D = a.D;
    floatx4 acc[1][1];
    acc[0][0] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (a.dgh_next) {
        ring_core<T, 32, 16, 2, 1, 2, GRU_NS>((const T*)a.dgh_next, a.lddgn, RowClamp{m0, a.B},
                                         (const T*)a.whh_t, 3 * D, RowClamp{u0, D}, 3 * D, smem,
                                         acc);
        ring_reduce<T, 32, 16, 2, 1, 2, GRU_NS>(smem, acc);
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = wave % 2, wk = wave / 2;
    if (wk != 0) return;
    const int u = u0 + (lane & 15);
    if (u >= D) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = m0 + wm * 16 + (lane >> 4) * 4 + i;
        if (row < a.B) gru_bwd_epilogue<T>(a, row, u, acc[0][0][i]);
    }
}

template <typename T, int BM>
static int launch_bwd(GruBwdArgs& a, hipStream_t s) {
    typedef Ring<T, 32, 16, 2, 1, 2, GRU_NS> R;
    if (a.whh_t && (3 * a.D) % R::KB == 0 && a.vec_wt && (!a.dgh_next || a.vec_dgn)) {
        static bool attr = false;
        if (!attr) {
            SRNN_CHECK_HIP(hipFuncSetAttribute((const void*)gru_bwd_ring_kernel<T>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, R::LDS));
            attr = true;
        }
        dim3 grid(cdiv(a.D, 16), cdiv(a.B, 32));
        hipLaunchKernelGGL((gru_bwd_ring_kernel<T>), grid, dim3(256), R::LDS, s, a);
        SRNN_LAUNCH_CHECK();
        return 0;
    }
    SRNN_REQUIRE(a.whh, "gru_cell_bwd: W_hh needed for this shape");
    constexpr int WM = BM / 16, WK = 4 / WM;
    typedef GemmCfg<T, BM, 16, 4, WM, 1, WK> C;
    dim3 grid(cdiv(a.D, 16), cdiv(a.B, BM));
    hipLaunchKernelGGL((gru_bwd_kernel<T, BM>), grid, dim3(256), C::LDS, s, a);
    SRNN_LAUNCH_CHECK();
    return 0;
}

extern "C" int srnn_gru_cell_bwd(int dtype, int B, int D, const float* dy, int64_t lddy,
                                 const void* dgh_next, int64_t lddgn, const float* ddir_next,
                                 const void* whh, const void* whh_t, const float* gates,
                                 int64_t ldgt, const float* hprev, int64_t ldhp, float* dgh,
                                 int64_t lddgh, void* dgh_lp, int64_t lddghl, float* dgi,
                                 int64_t lddgi, float* ddir, void* stream) {
    SRNN_REQUIRE(B > 0 && D > 0 && dy && gates && hprev && dgh && dgi && ddir,
                 "gru_cell_bwd: bad args");
    SRNN_REQUIRE(ddir != ddir_next, "gru_cell_bwd: ddir must not alias ddir_next");
    SRNN_REQUIRE(whh || whh_t, "gru_cell_bwd: need W_hh or W_hh^T");
    const int es = dtype == SRNN_F32 ? 4 : 2;
    GruBwdArgs a;
    a.dy = dy; a.lddy = lddy; a.dgh_next = dgh_next; a.lddgn = lddgn; a.ddir_next = ddir_next;
    a.whh = whh; a.whh_t = whh_t; a.gates = gates; a.ldgt = ldgt; a.hprev = hprev; a.ldhp = ldhp;
    a.dgh = dgh; a.lddgh = lddgh; a.dgh_lp = dgh_lp; a.lddghl = lddghl;
    a.dgi = dgi; a.lddgi = lddgi; a.ddir = ddir; a.B = B; a.D = D;
    a.vec_dgn = dgh_next ? al16(dgh_next, lddgn, es) : 0;
    a.vec_whh = whh ? al16(whh, D, es) : 0;
    a.vec_wt = whh_t ? al16(whh_t, 3 * (int64_t)D, es) : 0;
    if (dtype == SRNN_F32) return launch_bwd<float, 32>(a, (hipStream_t)stream);
    return launch_bwd<bf16, 32>(a, (hipStream_t)stream);
}

extern "C" int srnn_gru_cell(int dtype, int B, int D, int Din, const void* x, int64_t ldx,
                             const void* wih, const float* bih, const float* gi, int64_t ldgi,
                             const void* h, int64_t ldh, const float* hf, int64_t ldhf,
                             const void* whh, const float* bhh, float* hout, int64_t ldho,
                             void* hout_lp, int64_t ldhl, float* gates, int64_t ldgt,
                             void* stream) {
    return srnn_gru_cell_impl(dtype, B, D, Din, x, ldx, wih, bih, gi, ldgi, h, ldh, hf, ldhf, whh,
                              bhh, hout, ldho, hout_lp, ldhl, gates, ldgt, (hipStream_t)stream);
}
