// Plain large bf16 GEMMs through hipBLASLt (the ROCm library GEMM).  The TBPTT step's GEMMs
// whose epilogue is plain -- alpha, an optional per-column bias, optional ReLU, bf16 or fp32
// out -- (the upsampling forward / dX / dW, the GRU input projections and their gradients, the
// sample-level MLP's hidden forward) run 25-40 % faster in hipBLASLt's kernels than in
// gemm3 on MI355X (tools/blaslt_ab.py: 32768 x 16384 x 1024 NT 0.92 vs 1.32 ms); the fused
// epilogues hipBLASLt does not offer (ReLU-mask backward from the activations, max |C|, bit
// masks, Cin accumulation) and the very deep reductions gemm3 splits deterministically
// (D x D x B*T weight gradients) stay on gemm3.
//
// Row-major C (M x N) = op(A) (M x K) . op(B) (K x N) is column-major C^T = op(B)^T . op(A)^T:
// hipBLASLt's A is our B, its B our A, m = N, n = M; the bias vector (length m) is per output
// column of the row-major C.  One matmul descriptor, layouts and heuristic algorithm per shape,
// cached; the workspace is a grow-only scratch buffer (a captured HIP graph keeps its pointer).
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <tuple>
#include <vector>

#include "samplernn_hip_internal.hpp"

namespace {

constexpr size_t kWorkspace = 64ull << 20;

struct Plan {
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
    hipblasLtMatmulAlgo_t algo;
    size_t ws = 0;
    bool ok = false;
    std::vector<hipblasLtMatmulHeuristicResult_t> cand;   // the heuristic's candidates, best first
};

typedef std::tuple<int, int, int, int, int, int64_t, int64_t, int64_t, int, int, int, int, int,
                   int64_t, int64_t, int64_t>
    Key;

// Routing thresholds (srnn_blaslt_set_min; SRNN_BLASLT_MIN_MN / SRNN_BLASLT_MIN_MFLOP) and
// the per-shape algorithm choice (srnn_blaslt_set_tune; SRNN_BLASLT_TUNE): 0 takes the
// heuristic's first algorithm, n > 0 times its first n candidates once per shape on the call's
// own operands (never while the stream is capturing) and keeps the fastest
struct Routing {
    long long min_mn = 4ll << 20;
    double min_flop = 8589934592.0;
    int wide_k = 4096;
    int tune = 0;
    Routing() {
        min_mn = env_flag("SRNN_BLASLT_MIN_MN", (int)min_mn);
        const int mf = env_flag("SRNN_BLASLT_MIN_MFLOP", -1);
        if (mf >= 0) min_flop = mf * 1e6;
        wide_k = env_flag("SRNN_BLASLT_WIDE_K", wide_k);
        tune = env_flag("SRNN_BLASLT_TUNE", 0);
    }
};
Routing& routing() {
    static Routing r;
    return r;
}

hipblasLtHandle_t handle() {
    static hipblasLtHandle_t h = nullptr;
    static bool tried = false;
    if (!tried) {
        tried = true;
        if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) h = nullptr;
    }
    return h;
}

bool make_plan(Plan& p, int out_dtype, int transA, int transB, int M, int N, int K, int64_t lda,
               int64_t ldb, int64_t ldc, int epi, bool bias, int batch, int64_t sA, int64_t sB,
               int64_t sC) {
    hipblasLtHandle_t h = handle();
    if (!h) return false;
    const hipDataType tout = out_dtype == SRNN_F32 ? HIP_R_32F : HIP_R_16BF;
    if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS)
        return false;
    const hipblasOperation_t opa = transB ? HIPBLAS_OP_T : HIPBLAS_OP_N;   // lt A = our B
    const hipblasOperation_t opb = transA ? HIPBLAS_OP_T : HIPBLAS_OP_N;   // lt B = our A
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa));
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb));
    const hipblasLtEpilogue_t e = (hipblasLtEpilogue_t)epi;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
    if (bias) {
        const hipDataType bt = HIP_R_32F;
        hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    }
    // column-major shapes of the stored operands
    if (hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, transB ? K : N, transB ? N : K, ldb) !=
            HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, transA ? M : K, transA ? K : M, lda) !=
            HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&p.lc, tout, N, M, ldc) != HIPBLAS_STATUS_SUCCESS)
        return false;
    if (batch > 1) {
        // lt A = our B (stride sB), lt B = our A (sA), C (sC); a stride of 0 repeats the operand
        const int32_t bc = batch;
        const int64_t st[3] = {sB, sA, sC};
        hipblasLtMatrixLayout_t ls[3] = {p.la, p.lb, p.lc};
        for (int i = 0; i < 3; ++i)
            if (hipblasLtMatrixLayoutSetAttribute(ls[i], HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc,
                                                  sizeof(bc)) != HIPBLAS_STATUS_SUCCESS ||
                hipblasLtMatrixLayoutSetAttribute(ls[i],
                                                  HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET,
                                                  &st[i], sizeof(st[i])) != HIPBLAS_STATUS_SUCCESS)
                return false;
    }
    hipblasLtMatmulPreference_t pref;
    if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return false;
    const uint64_t wsmax = kWorkspace;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsmax,
                                          sizeof(wsmax));
    const int want = routing().tune > 1 ? routing().tune : 1;
    std::vector<hipblasLtMatmulHeuristicResult_t> res(want);
    int n = 0;
    const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.la, p.lb, p.lc, p.lc,
                                                               pref, want, res.data(), &n);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (st != HIPBLAS_STATUS_SUCCESS || n < 1) return false;
    res.resize(n);
    p.cand = res;
    p.algo = res[0].algo;
    p.ws = res[0].workspaceSize;
    return true;
}

}  // namespace

int srnn_blaslt_enabled() { return env_flag("SRNN_BLASLT", 1); }

static int g_blaslt_calls = 0;

// GEMMs launched through hipBLASLt so far in this process (tests: the path was taken)
extern "C" int srnn_blaslt_calls(void) { return g_blaslt_calls; }

// routing thresholds of srnn_blaslt_try: problems with fewer than min_outputs outputs or
// min_flop flop stay on the hand-written kernels (defaults 4 Mi, 2^33)
extern "C" int srnn_blaslt_set_min(long long min_outputs, double min_flop) {
    routing().min_mn = min_outputs;
    routing().min_flop = min_flop;
    routing().wide_k = min_outputs == 0 ? 1 << 30 : 4096;
    return 0;
}

// per-shape algorithm choice: 0 = the heuristic's first; n > 1 = the fastest of its first n
// candidates, timed once per shape outside graph capture
extern "C" int srnn_blaslt_set_tune(int n) {
    routing().tune = n < 0 ? 0 : n;
    return 0;
}

// 0 = done, -1 = not taken (the caller runs its own kernels), > 0 = HIP / library error
int srnn_blaslt_try(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                    float alpha, const void* A, int64_t lda, const void* B, int64_t ldb, float beta,
                    void* C, int64_t ldc, const float* bias, int bias_mode, int relu,
                    hipStream_t s, int batch, int64_t sA, int64_t sB, int64_t sC) {
    if (!srnn_blaslt_enabled() || dtype != SRNN_BF16 || beta != 0.f || batch < 1) return -1;
    if (batch > 1 && (bias || sA % 8 || sB % 8 || sC % 8 || sC == 0)) return -1;
    if (bias && bias_mode != 1) return -1;
    if (M <= 0 || N <= 0 || K <= 0) return -1;
    // large enough to pay for the library's launch and wide enough that gemm3's split-K deep
    // reductions are not the better choice (M N >= 4 Mi outputs, 2 M N K >= 2^33 flop) -- or,
    // below that, at least 1 Mi outputs over a shallow reduction (256 <= K <= wide_k = 4096):
    // the 64-row step's top-tier GRU / upsampling products and the bottom tier's K = 4096
    // weight gradients, where gemm3's 256-wide tiles fill only 16-48 CUs and its split-K pays
    // a partial-sum pass (tools/gemm_route_probe.py, profiles/r06_gemm_route_b64.txt:
    // 3072 x 1024 x 1024 TN 28.3 -> 17.4 us, 1024 x 1024 x 4096 NN 34.2 -> 23.2 us); the deep
    // weight gradients (K = 8192 .. 524288) stay on gemm3, which is faster there
    const int64_t outs = (int64_t)M * N * batch;
    const bool big = outs >= routing().min_mn && 2.0 * outs * K >= routing().min_flop;
    const bool wide = outs >= (1ll << 20) && K >= 256 && K <= routing().wide_k;
    if (!big && !wide) return -1;
    // (SRNN_BLASLT_F32_MINK: fp32-output problems only from this K on.  In isolation gemm3 writes
    //  fp32 faster at K of a few thousand -- GRU input projection 32768 x 3072 x 1024: 220 vs
    //  266 us -- but inside the step the library form measured 0.1-0.2 ms per step faster)
    if (out_dtype == SRNN_F32 && K < env_flag("SRNN_BLASLT_F32_MINK", 0)) return -1;
    if (M % 16 || N % 16 || K % 16 || lda % 8 || ldb % 8 || ldc % 8) return -1;
    const int epi = bias ? (relu ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS)
                         : (relu ? HIPBLASLT_EPILOGUE_RELU : HIPBLASLT_EPILOGUE_DEFAULT);
    static std::map<Key, Plan> plans;
    const Key key{out_dtype, transA, transB, M, N, lda, ldb, ldc, K, epi, bias ? 1 : 0,
                  routing().tune, batch, sA, sB, sC};
    auto it = plans.find(key);
    bool fresh = false;
    if (it == plans.end()) {
        Plan p;
        p.ok = make_plan(p, out_dtype, transA, transB, M, N, K, lda, ldb, ldc, epi, bias != nullptr,
                         batch, sA, sB, sC);
        it = plans.emplace(key, p).first;
        fresh = true;
    }
    Plan& p = it->second;
    if (!p.ok) return -1;
    void* ws = p.cand.size() > 1 || p.ws ? srnn_scratch(SRNN_SCRATCH_BLASLT, kWorkspace) : nullptr;
    if ((p.cand.size() > 1 || p.ws) && !ws) return -1;
    if (bias)
        hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias,
                                        sizeof(bias));
    const float zero = 0.f;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (fresh && p.cand.size() > 1 && hipStreamIsCapturing(s, &cap) == hipSuccess &&
        cap == hipStreamCaptureStatusNone) {
        // time every candidate on these operands (1 warm-up + 5 runs each) and keep the
        // fastest; the call below then writes C with it
        hipEvent_t e0, e1;
        SRNN_CHECK_HIP(hipEventCreate(&e0));
        SRNN_CHECK_HIP(hipEventCreate(&e1));
        float best = 1e30f;
        for (const auto& c : p.cand) {
            if (hipblasLtMatmul(handle(), p.desc, &alpha, B, p.la, A, p.lb, &zero, C, p.lc, C,
                                p.lc, &c.algo, ws, c.workspaceSize, s) != HIPBLAS_STATUS_SUCCESS)
                continue;
            SRNN_CHECK_HIP(hipEventRecord(e0, s));
            for (int r = 0; r < 5; ++r)
                hipblasLtMatmul(handle(), p.desc, &alpha, B, p.la, A, p.lb, &zero, C, p.lc, C,
                                p.lc, &c.algo, ws, c.workspaceSize, s);
            SRNN_CHECK_HIP(hipEventRecord(e1, s));
            SRNN_CHECK_HIP(hipEventSynchronize(e1));
            float ms = 0.f;
            SRNN_CHECK_HIP(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) {
                best = ms;
                p.algo = c.algo;
                p.ws = c.workspaceSize;
            }
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    const hipblasStatus_t st = hipblasLtMatmul(handle(), p.desc, &alpha, B, p.la, A, p.lb, &zero,
                                               C, p.lc, C, p.lc, &p.algo, ws, p.ws, s);
    if (st != HIPBLAS_STATUS_SUCCESS) {
        if (batch > 1) {          // (a batched form the library declines: own kernels from now)
            p.ok = false;
            return -1;
        }
        srnn_set_error("hipblasLtMatmul failed (%d) for %dx%dx%d", (int)st, M, N, K);
        return 2;
    }
    ++g_blaslt_calls;
    return 0;
}
