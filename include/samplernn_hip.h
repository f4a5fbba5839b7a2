/* samplernn_hip.h -- C ABI of the MI355X-native SampleRNN hot path (libsamplernn_hip.so).
 *
 * Plain pointers and sizes only: every buffer argument is a device pointer allocated
 * and owned by the caller; `stream` is the caller's hipStream_t (NULL = default).
 * Every entry point returns 0 on success, 1 on a bad argument and 2 on a HIP error;
 * srnn_last_error() returns the text (per host thread).  Dtype codes: 0 = fp32,
 * 1 = bf16.  GEMM operands follow BLAS conventions on row-major storage.
 *
 * The reference (mahdeslami11/jalil-saboorizadeh-Multi-speaker-Neural-Vocoder) is pure
 * Python with no FFI; each entry point below names the reference function/operator it
 * replaces.  The drop-in binding is the Python package beside this header
 * (model.py / nn.py / utils.py / optim.py / trainer), see INTEGRATION.md.
 */
#ifndef SAMPLERNN_HIP_H
#define SAMPLERNN_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRNN_MAX_TIERS 6
#define SRNN_MAX_RNN 4

const char* srnn_last_error(void);
int srnn_abi_version(void);
/* Content hash (16 hex digits, csrc/srchash.py) of the sources this library was compiled
 * from; the Python binding refuses a library whose hash differs from its tree's (a stale
 * build).  Replaces no reference interface.                                             */
const char* srnn_build_hash(void);

/* ---- mu-law / linear quantisation ------------------------------------------------
 * utils.uquantize (utils.py:58-59 = midrise(ulaw(x)), utils.py:33-36,48-51): bit-exact to
 * the reference for every float32 / float64 input in [-1, 1] (q_levels = 256).        */
int srnn_uquantize_f32(const float* x, int64_t* out, int64_t n, int q_levels, void* stream);
int srnn_uquantize_f64(const double* x, int64_t* out, int64_t n, int q_levels, void* stream);
/* out = scale * udequantize(k) (utils.py:62-63, mode 0) or linear_dequantize
 * (utils.py:18-19, mode 1); scale = 2 gives the model's `2 * dequantize` (model.py:385,471) */
int srnn_udequantize(const int64_t* k, float* out, int64_t n, int q_levels, float scale,
                     int mode, void* stream);
/* srnn_udequantize of a rows x cols window with row stride ldk (a slice of the index stream,
 * model.py:385 `input_sequences[:, a:b]`) into contiguous rows (no copy of the slice first) */
int srnn_udequantize2d(const int64_t* k, int64_t ldk, float* out, int rows, int cols,
                       int q_levels, float scale, int mode, void* stream);

/* ---- dense projections -------------------------------------------------------------
 * C = act(alpha * op(A) . op(B) + beta * Cin + bias)  (bias_mode 1: per column, 2: per row)
 * Replaces the Conv1d(k=1) / nn.Linear / GRU-input / ConvTranspose1d matmuls of
 * model.py:85-116,148-178,287-301 and nn.py:12-43 (forward, dgrad and wgrad).
 * tile = -1 picks the tile shape from the problem size.  mask (optional, input dtype,
 * row stride ldmask) zeroes outputs where mask <= 0 (the ReLU backward of model.py:320-321). */
int srnn_gemm(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
              float alpha, const void* A, int64_t lda, int64_t strideA, const void* B,
              int64_t ldb, int64_t strideB, float beta, const float* Cin, int64_t ldcin,
              int64_t strideCin, void* C, int64_t ldc, int64_t strideC, const float* bias,
              int bias_mode, int relu, int batch, int tile, const void* mask, int64_t ldmask,
              void* stream);

/* The same product (batch 1) with ReLU masks as bits -- bit c % 16 of the u16 at
 * [row * ld + c / 16] is (value(row, c) > 0): mask_bits (optional) zeroes the outputs whose
 * bit is clear (in place of srnn_gemm's bf16 mask, 16x fewer bytes for the ReLU backward of
 * model.py:320-321); bits_out (optional, bf16 out) receives the bits of C (the forward of
 * the ReLU layer, for that backward). */
int srnn_gemm_bits(int dtype, int out_dtype, int transA, int transB, int M, int N, int K,
                   float alpha, const void* A, int64_t lda, const void* B, int64_t ldb,
                   float beta, const float* Cin, int64_t ldcin, void* C, int64_t ldc,
                   const float* bias, int bias_mode, int relu, int tile,
                   const unsigned short* mask_bits, int64_t ldmb, unsigned short* bits_out,
                   int64_t ldbo, void* stream);
/* bits[row * ldb + c / 16] bit c % 16 = (a[row * lda + c] > 0), a in dtype (M x N).
 * ldb = 0: the grouped layout, u16 [c / 16][row] (N % 64 == 0) -- the same bits, rows
 * contiguous per 16-column group; srnn_gemm_bits takes it (ldmb = 0) and its bf16
 * pair-mode kernels stage it by LDS-DMA ahead of the epilogue.                         */
int srnn_relu_bits(int dtype, const void* a, int64_t lda, int M, int N, unsigned short* bits,
                   int64_t ldb, void* stream);

/* ---- GRU (torch.nn.GRU, model.py:148-165,244) -----------------------------------------
 * One time step for B rows: h_t from h_{t-1} and either x (gi computed in-kernel with
 * W_ih) or a precomputed gi = x W_ih^T + b_ih.  Optionally saves r|z|n|gh_n (4D/row).  */
int srnn_gru_cell(int dtype, int B, int D, int Din, const void* x, int64_t ldx, const void* wih,
                  const float* bih, const float* gi, int64_t ldgi, const void* h, int64_t ldh,
                  const float* hf, int64_t ldhf, const void* whh, const float* bhh, float* hout,
                  int64_t ldho, void* hout_lp, int64_t ldhl, float* gates, int64_t ldgt,
                  void* stream);
/* Backward of one step: dh_t = dy_t + dh_direct_{t+1} + dgh_{t+1} . W_hh, then the gate
 * backward.  Writes dgh_t (fp32 + optional T copy), dgi_t (fp32), dh_direct_t = z*dh_t.
 * Pass W_hh (3D, D) and/or its transpose (D, 3D); the transpose enables the deep-ring
 * kernel.                                                                                */
int srnn_gru_cell_bwd(int dtype, int B, int D, const float* dy, int64_t lddy,
                      const void* dgh_next, int64_t lddgn, const float* ddir_next,
                      const void* whh, const void* whh_t, const float* gates, int64_t ldgt,
                      const float* hprev, int64_t ldhp, float* dgh, int64_t lddgh, void* dgh_lp,
                      int64_t lddghl, float* dgi, int64_t lddgi, float* ddir, void* stream);

/* Whole-sequence forward of one GRU layer in a single persistent launch (bf16, D <= 1024,
 * D % 128 == 0, (D/16) * ceil(B/32) workgroups co-resident): out[b][t] / out_lp /
 * gates[b][t] exactly as Fr calls of srnn_gru_cell with gi[b][t] = gi + b*ldgi + t*sgi.
 * work: >= (64 * ceil(B/32) + 1) ints (zeroed by the call; the last word is an error flag
 * raised if a workgroup gave up waiting).  srnn_gru_seq_supported returns 1 / 0.       */
int srnn_gru_seq_supported(int dtype, int B, int D);
/* Whole-sequence GRU forward of one layer as ONE persistent launch with row groups placed per
 * XCD (gru_xcd.hip): W_hh resident in VGPRs, h hand-offs as data-tagged granules in the XCD's
 * L2.  Any B: up to 4 tiles of 16 rows per group (512 rows per launch at D = 1024; more rows run
 * as consecutive launches over row chunks, rows being independent).  Same operands and outputs as srnn_gru_seq_fwd (torch.nn.GRU recurrence,
 * model.py:148-165 / 244), gi includes b_ih; work = srnn_gru_xcd_work_bytes(dtype, B, D) bytes
 * (0 = shape or device not supported; zeroed by the call).  srnn_gru_xcd_error(work)
 * synchronises and returns nonzero if a hand-off was given up (bounded spin). */
size_t srnn_gru_xcd_work_bytes(int dtype, int B, int D);
int srnn_gru_xcd_fwd(int dtype, int B, int D, int Fr, const float* gi, int64_t ldgi, int64_t sgi,
                     const float* h0, const void* whh, const float* bhh, float* out,
                     void* out_lp, int64_t ldo, int64_t so, float* gates, int64_t ldg,
                     int64_t sg, void* work, size_t work_bytes, void* stream);
/* srnn_gru_xcd_fwd that also writes the previous-state sequence the W_hh gradient consumes,
 * hprev_lp[b][t] = bf16(t == 0 ? h0[b] : out[b][t - 1]) (same ldo / so layout as out_lp), so the
 * backward needs no shifted copy (model.py:222-244 carry; hprev_lp may be null). */
int srnn_gru_xcd_fwd2(int dtype, int B, int D, int Fr, const float* gi, int64_t ldgi, int64_t sgi,
                      const float* h0, const void* whh, const float* bhh, float* out,
                      void* out_lp, int64_t ldo, int64_t so, float* gates, int64_t ldg,
                      int64_t sg, void* hprev_lp, void* work, size_t work_bytes, void* stream);
/* Reverse sweep of one layer in the same organisation (W_hh^T K-slices in VGPRs, dgh
 * hand-offs as granules): same operands and outputs as srnn_gru_seq_bwd; work =
 * srnn_gru_xcd_bwd_work_bytes(dtype, B, D) bytes. */
size_t srnn_gru_xcd_bwd_work_bytes(int dtype, int B, int D);
int srnn_gru_xcd_bwd(int dtype, int B, int D, int Fr, const float* dy, int64_t lddy, int64_t sdy,
                     const float* gates, int64_t ldg, int64_t sg, const float* hout, int64_t ldo,
                     int64_t so, const float* h0, const void* whh_t, float* dgh, void* dgh_lp,
                     float* dgi, int64_t ldd, int64_t sd, float* ddir0, void* work,
                     size_t work_bytes, void* stream);
/* Same sweep with the bf16 TBPTT step's outputs: dgh / dgi (fp32) may be NULL; dgi_lp (bf16,
 * dgi's layout, the operand of the dW_ih / dX GEMMs) and bsum ((B, 4D) fp32: per batch row the
 * sums over t of [dar | daz | dghn | dan], from which b_hh / b_ih gradients are one column sum)
 * are optional.  Replaces the cast of dgi and the two bias column sums over B x Fr rows. */
int srnn_gru_xcd_bwd2(int dtype, int B, int D, int Fr, const float* dy, int64_t lddy, int64_t sdy,
                      const float* gates, int64_t ldg, int64_t sg, const float* hout, int64_t ldo,
                      int64_t so, const float* h0, const void* whh_t, float* dgh, void* dgh_lp,
                      float* dgi, void* dgi_lp, float* bsum, int64_t ldd, int64_t sd,
                      float* ddir0, void* work, size_t work_bytes, void* stream);
int srnn_gru_xcd_error(const void* work);
/* Sticky form for callers that do not keep the work buffer: nonzero if ANY persistent GRU
 * sweep (srnn_gru_xcd_fwd/bwd, srnn_gru_seq_fwd/bwd) since the previous call gave up a
 * hand-off, -1 on a HIP error; clears the flag and synchronises the device.  While the flag
 * is up srnn_adam_clip_multi skips its update (the failed step's gradients never reach the
 * weights).  The training path checks it once per Trainer iteration (the reference has no
 * equivalent: its cuDNN GRU cannot fail this way).                                        */
int srnn_persistent_error_take(void);
/* Co-residency of the persistent kernels (csrc/handoff.hpp, persist.hip): n processes run
   persistent grids on this device at once (a multi-rank rehearsal on one GPU; default 1).
   Support predicates (srnn_gru_xcd_work_bytes, srnn_gru_seq_supported, the generation plan)
   then only accept grids that fit the device n times over; every persistent launch checks
   occupancy x CUs >= workgroups x n and refuses (error) otherwise.  The reference has no
   counterpart (its GRU is torch.nn.GRU, model.py:148-165).                                 */
int srnn_set_device_share(int n);
int srnn_device_share(void);
/* Diagnostics: occupy `blocks` CUs (160 KiB LDS each) for `usec` us; *done += 1 per
   workgroup at the end (optional) -- the co-residency tests' stand-in for other work.      */
int srnn_hold_cus(int blocks, int usec, int* done, void* stream);
/* Stream-ordered access to that flag for data parallelism: dst = flag ? 1.f : 0.f, and
 * flag |= (src > 0).  The flag rides in a gradient bucket so every rank agrees.           */
int srnn_persistent_flag_to_f32(float* dst, void* stream);
int srnn_persistent_flag_or_f32(const float* src, void* stream);
/* Stream-ordered 4-byte copy of the flag into pinned host memory `dst`: the Trainer's lagged
 * per-iteration check reads step n's copy after enqueuing step n+1 (trainer/__init__.py:116-117
 * without a device synchronisation per iteration). */
int srnn_persistent_flag_snapshot(int* dst, void* stream);
/* dtype (fp32 / bf16) forms of srnn_persistent_flag_to_f32 / _or_f32 (bf16 gradient buckets) */
int srnn_persistent_flag_to(void* dst, int dtype, void* stream);
int srnn_persistent_flag_or(const void* src, int dtype, void* stream);
int srnn_gru_seq_fwd(int dtype, int B, int D, int Fr, const float* gi, int64_t ldgi,
                     int64_t sgi, const float* h0, const void* h0_lp, const void* whh,
                     const float* bhh, float* out, void* out_lp, int64_t ldo, int64_t so,
                     float* gates, int64_t ldg, int64_t sg, int* work, size_t work_bytes,
                     void* stream);
/* Whole-sequence backward of one GRU layer (t = Fr-1 .. 0) in one persistent launch:
 * the Fr calls of srnn_gru_cell_bwd, with dh_direct kept on chip; ddir0 receives the
 * dh_direct of step 0.  dgh / dgh_lp / dgi share the row stride ldd and step stride sd.  */
int srnn_gru_seq_bwd(int dtype, int B, int D, int Fr, const float* dy, int64_t lddy,
                     int64_t sdy, const float* gates, int64_t ldg, int64_t sg, const float* hout,
                     int64_t ldo, int64_t so, const float* h0, const void* whh_t, float* dgh,
                     void* dgh_lp, float* dgi, int64_t ldd, int64_t sd, float* ddir0, int* work,
                     size_t work_bytes, void* stream);

/* ---- SampleLevelMLP (model.py:308-325) ----------------------------------------------
 * a1[b*Tlen+t] = relu(sum_k tab[k][x[b*ldx + xoff + t + k]] + upper[b*Tlen+t])
 * tab / out in `dtype`; upper in `upper_dtype` (SRNN_F32 or SRNN_BF16)                  */
int srnn_mlp_l1(int dtype, const void* tab, const int64_t* x, int64_t ldx, int xoff, int B,
                int Tlen, int upper_dtype, const void* upper, int64_t ldu, void* out,
                int64_t ldo, int D, int FS0, int Q, void* stream);
/* The same (bf16 table, upper and a1) writing a1's ReLU mask as bits too (srnn_gemm_bits
 * layout, row stride ldb u16; ldb = 0: the grouped layout of srnn_relu_bits), for the
 * masked GEMM of the backward.                                                         */
int srnn_mlp_l1_bits(const void* tab, const int64_t* x, int64_t ldx, int xoff, int B, int Tlen,
                     const void* upper, int64_t ldu, void* out, int64_t ldo, int D, int FS0,
                     int Q, unsigned short* bits, int64_t ldb, void* stream);
/* dtab[x_{t+k}][k][:] += da_t  (Q, FS0, D) fp32 accumulate; backward of the folded     *
 * embedding+conv                                                                        */
int srnn_mlp_dtab(int dtype, const void* da, int64_t ldda, const int64_t* x, int64_t ldx,
                  int xoff, int B, int Tlen, void* dtab, int out_dtype, int D, int FS0, int Q,
                  void* work, size_t work_bytes, void* stream);
/* Same, and (colsum != NULL) the bottom tier's upsampling bias gradient from the same pass:
 * colsum[j * D + c] = sum over batch rows and t = j (mod FS0) of da[b, t, c] (fp32, FS0 x D);
 * *colsum_done (host int) = 1 when it was written (the direct position-major path), else 0
 * and the caller sums the columns itself.                                                   */
int srnn_mlp_dtab2(int dtype, const void* da, int64_t ldda, const int64_t* x, int64_t ldx,
                   int xoff, int B, int Tlen, void* dtab_out, int out_dtype, int D, int FS0, int Q,
                   void* work, size_t work_bytes, float* colsum, int* colsum_done, void* stream);
/* (deterministic: 2^-40 fixed-point int64 accumulation; work >= Q*FS0*D*8 bytes)        *
 * bf16 da and bf16 output at FS0 = 16, Q = 256, D % 8 == 0 take the packed form: two      *
 * columns per 64-bit LDS atomic in 32-bit fixed point at a power-of-2 scale from max |da| *
 * and the most frequent sample value (exact integer sums, deterministic).                 */
/* srnn_mlp_dtab2 with amax_in (device, may be NULL): max |da| as float bits, measured by  *
 * the GEMM that produced da (srnn_gemm_amax_next), so the packed form skips its own pass  *
 * over da.  Replaces nothing new in the reference: the same model.py:311-320 backward.    */
int srnn_mlp_dtab3(int dtype, const void* da, int64_t ldda, const int64_t* x, int64_t ldx,
                   int xoff, int B, int Tlen, void* dtab_out, int out_dtype, int D, int FS0, int Q,
                   void* work, size_t work_bytes, float* colsum, int* colsum_done,
                   const unsigned* amax_in, void* stream);
/* Ask the next bf16-output GEMM that runs on the 256 x 256 gemm3 path (model.py:311-320's
 * da1 = (da2 W_hid) * relu', the GEMM producing the dTab scatter's input) to also write
 * max |C| (float bits, atomicMax into *amax, which must be zero).  srnn_gemm_amax_taken()
 * returns 1 if a GEMM did since (host state; also clears a request no GEMM took).        */
int srnn_gemm_amax_next(unsigned* amax);
int srnn_gemm_amax_taken(void);
/* srnn_gemm_amax_next, and the same GEMM also writes a column-blocked copy of its bf16
 * output into blk[N / 4][M][4] (M x N bf16, caller-allocated); srnn_gemm_amax_taken()
 * then returns 2.  The dTab scatter's operand layout (srnn_mlp_dtab4).                   */
int srnn_gemm_amax_blk_next(unsigned* amax, void* blk);
/* Ask the next bf16-output GEMM that runs on the 256 x 256 gemm3 pair path (model.py:320's
 * da2 = (dz W_out) * relu', whose column sums are the hidden layer's bias gradient,
 * model.py:317's Conv1d bias) to also write the column sums of its stored bf16 output per
 * 128-row block into part[M / 128][N] (fp32, caller-allocated; every entry written once, no
 * zeroing needed); the caller sums the M / 128 rows.  srnn_gemm_csum_taken() returns 1 if a
 * GEMM did since (host state; also clears a request no GEMM took).                        */
int srnn_gemm_csum_next(float* part);
int srnn_gemm_csum_taken(void);
/* Ask the next fp32-output NT GEMM with N = 256 (one 256-column tile: whole rows) that runs
 * on the gemm3 pair path -- the SampleLevelMLP's logits, model.py:324 -- to write
 * log_softmax of every output row (model.py:325) instead of the row: logp = (v - max) -
 * log(sum exp(v - max)), v = alpha A B^T + bias, the logsoftmax_nll arithmetic.
 * srnn_gemm_logsoftmax_taken() returns 1 if a GEMM did since (host state; also clears a
 * request no GEMM took).                                                              */
int srnn_gemm_logsoftmax_next(void);
int srnn_gemm_logsoftmax_taken(void);
/* srnn_mlp_dtab3 with blk (device, may be NULL): the column-blocked copy of da
 * (blk[D / 4][B * Tlen][4], srnn_gemm_amax_blk_next) the packed form reads instead of da
 * (whole 128-B lines per load).  Same outputs bit for bit.  A sample histogram skewed past
 * the packed form's precision bound (one value at > 65,536 positions) makes the exact
 * 2^-40 form run instead; a non-finite da makes dTab and colsum NaN.  Replaces
 * model.py:311-320's backward like srnn_mlp_dtab.                                         */
int srnn_mlp_dtab4(int dtype, const void* da, int64_t ldda, const int64_t* x, int64_t ldx,
                   int xoff, int B, int Tlen, void* dtab_out, int out_dtype, int D, int FS0, int Q,
                   void* work, size_t work_bytes, float* colsum, int* colsum_done,
                   const unsigned* amax_in, const void* blk, void* stream);
/* 1 if the packed dTab kernels may run: they address their LDS bins without a base, valid
 * only while they have no static LDS (checked from the compiled kernels' attributes; 0 sends
 * srnn_mlp_dtab4 to the exact form).  Diagnostic; needs a device.                        */
int srnn_dtab_packed_ok(void);
/* Number of GEMMs srnn_gemm / srnn_gemm_bits handed to hipBLASLt so far in this process:
 * large plain bf16 problems (alpha, per-column bias, ReLU, beta 0, no mask; M N >= 4 Mi,
 * 2 M N K >= 2^33) run as the ROCm library GEMM (SRNN_BLASLT=0: the library's own gemm3
 * kernels).  Diagnostic; replaces no reference interface.                               */
int srnn_blaslt_calls(void);
/* Routing of srnn_blaslt_calls' path: plain bf16 problems with fewer than min_outputs
 * outputs (M N) or min_flop flop (2 M N K) stay on the hand-written kernels (defaults 4 Mi and
 * 2^33; env SRNN_BLASLT_MIN_MN / SRNN_BLASLT_MIN_MFLOP).  srnn_blaslt_set_tune(n): n > 1 times
 * the library heuristic's first n algorithms once per shape, outside graph capture, on the
 * call's own operands and keeps the fastest (0: the heuristic's first; env SRNN_BLASLT_TUNE).
 * Tuning knobs; replace no reference interface.                                           */
int srnn_blaslt_set_min(long long min_outputs, double min_flop);
int srnn_blaslt_set_tune(int n);
/* log_softmax (model.py:324-325) + NLL rows (nn.py:66-70) + dlogits (softmax-onehot)*g  */
/* dz = dlogp - exp(logp) * rowsum(dlogp)   (log_softmax backward, rows of Q)          */
int srnn_logsoftmax_bwd(const float* dlogp, int64_t lddl, const float* logp, int64_t ldl,
                        int64_t rows, int Q, void* dz, int dz_dtype, int64_t ldd, void* stream);
/* NLL over log-probs (nn.py:66-70): loss_row[r] = -logp[r, target]; and its gradient
 * dlogp[r, :] = 0 except dlogp[r, target] = -gscale                                      */
int srnn_nll_fwd(const float* logp, int64_t ldl, const int64_t* target, int64_t ldt, int Tlen,
                 int64_t rows, float* loss_row, void* stream);
int srnn_nll_bwd(const int64_t* target, int64_t ldt, int Tlen, int64_t rows, int Q,
                 float* dlogp, int64_t ldd, float gscale, const float* gmul, void* stream);
/* Fused backward of sequence_nll_loss_bits (nn.py:66-70) through the MLP's log_softmax
 * (model.py:324-325): dz = c (exp(logp) - onehot(target)), c = gscale * (*gmul), in dz_dtype
 * (fp32 / bf16) -- srnn_nll_bwd + srnn_logsoftmax_bwd in one pass, bit-identical to them,
 * without the dense fp32 dlogp. */
int srnn_nll_logsoftmax_bwd(const int64_t* target, int64_t ldt, int Tlen, int64_t rows, int Q,
                            const float* logp, int64_t ldl, float gscale, const float* gmul,
                            void* dz, int dz_dtype, int64_t ldd, void* stream);
/* (gmul: optional device scalar the scale is multiplied by -- the incoming loss gradient,
 *  read on the device so the backward never synchronises with the host)                 */
int srnn_logsoftmax_nll(const float* z, int64_t ldz, const int64_t* target, int64_t ldt,
                        int Tlen, int64_t rows, int Q, float* loss_row, float* logp,
                        int64_t ldl, void* dz, int dz_dtype, int64_t ldd, float gscale,
                        void* stream);

/* Host-side (no GPU) bit-exact quantisers with the same tables, for the CPU data path. */
int srnn_uquantize_f64_host(const double* x, int64_t* out, int64_t n, int q_levels);
int srnn_uquantize_f32_host(const float* x, int64_t* out, int64_t n, int q_levels);
int srnn_udequantize_host(const int64_t* k, float* out, int64_t n, int q_levels);

/* ---- weight norm (torch weight_norm dim=0, model.py:119-131,177-178,303-306) -------- */
int srnn_weight_norm_fwd(const float* g, const float* v, float* w, float* norm, int O,
                         int64_t R, void* stream);
int srnn_weight_norm_bwd(const float* g, const float* v, const float* dw, float* dg, float* dv,
                         int O, int64_t R, int accumulate, void* stream);
/* The always-on weight norm of LearnedUpsampling1d.conv_t (model.py:177-178) folded into its
 * GEMM operand: scale[i] = g[i] / ||v[i]||; dst[(j * Cout + o) * Cin + i] = v[i][o][j] * scale[i]
 * (dst fp32 or bf16; scale NULL = 1: a plain (2, 1, 0) permute); backward from the GEMM's
 * transposed weight gradient dwt[i][(j * Cout + o)] to dg[i] and dv (v's layout).          */
int srnn_weight_norm_scale(const float* g, const float* v, float* scale, int O, int64_t R,
                           void* stream);
int srnn_convt_fold(const float* v, const float* scale, void* dst, int dst_dtype, int Cin,
                    int Cout, int k, void* stream);
int srnn_convt_wn_bwd(const float* g, const float* v, const float* dwt, float* dg, float* dv,
                      int Cin, int Cout, int k, void* stream);

/* ---- layout / elementwise helpers ------------------------------------------------- */
int srnn_permute3(const float* src, void* dst, int dst_dtype, int d0, int d1, int d2, int p0,
                  int p1, int p2, int accumulate, void* stream);
int srnn_copy2d(int src_dtype, int dst_dtype, int rows, int cols, const void* src, int64_t lds,
                void* dst, int64_t ldd, void* stream);
int srnn_gather_rows(const float* table, int64_t ldt, const int64_t* idx, int64_t n, int cols,
                     void* out, int out_dtype, int64_t ldo, void* stream);
int srnn_scatter_add_rows(float* table, int64_t ldt, const int64_t* idx, int64_t n, int cols,
                          const float* src, int64_t lds, void* stream);
/* table[q,:] += sum_{r: idx[r]==q} src[r,:] in r order, q < trows -- the speaker-embedding
   backward (model.py:203-207, nn.Embedding's gradient) without atomics: deterministic     */
int srnn_index_add_rows(float* table, int64_t ldt, int trows, const int64_t* idx, int64_t n,
                        int cols, const float* src, int64_t lds, void* stream);
int srnn_axpby(float* out, const float* a, const float* b, float alpha, float beta, int64_t n,
               void* stream);
int srnn_add_bcast_rows(float* x, const float* v, int B, int F, int D, int64_t ldv, void* stream);
/* out[b][c] = sum_{f<F} src[(b*F + f)*lds + c]  (per-sequence frame sums, fp32)        */
int srnn_segsum(const float* src, int64_t lds, int B, int F, int D, float* out, void* stream);
int srnn_colsum(int dtype, const void* src, int64_t lds, int64_t rows, int cols, float* out,
                float alpha, int accumulate, float* work, int64_t work_elems, void* stream);

/* ---- optimizer: gradient_clipping(-1, 1) + Adam (optim.py:4-21, train.py:238) --------
 * Elementwise in-place clamp of g to [clip_lo, clip_hi] then torch.optim.Adam update.
 * p_bf16 (optional) receives the updated parameters rounded to bf16.                    */
int srnn_adam_clip(float* p, float* g, float* m, float* v, void* p_bf16, int64_t n,
                   float clip_lo, float clip_hi, double lr, double beta1, double beta2,
                   double eps, int64_t step, void* stream);
/* The same for `ntensors` parameters in one launch (per 64 tensors): host arrays of device
 * pointers and element counts; p_bf16 may be NULL (no copies) or hold NULL entries; a NULL
 * entry of g is an all-zero gradient (a parameter the step's backward did not reach).
 * Skipped entirely (on the device) while the persistent-sweep failure flag is up.        */
int srnn_adam_clip_multi(int ntensors, float* const* p, float* const* g, float* const* m,
                         float* const* v, void* const* p_bf16, const int64_t* n, float clip_lo,
                         float clip_hi, double lr, double beta1, double beta2, double eps,
                         int64_t step, void* stream);
/* srnn_adam_clip_multi over gradients of dtype gdtype (fp32, or bf16 from bf16 gradient
 * buckets) scaled by gscale before the clamp: under data parallelism the SUM-reduced buckets
 * are read in place with gscale = 1 / world (the mean before the clip, optim.py:11-13 applied
 * to the full-batch gradient).  fp32 gradients are written back clamped, bf16 ones only read. */
int srnn_adam_clip_multi2(int ntensors, float* const* p, void* const* g, int gdtype, float gscale,
                          float* const* m, float* const* v, void* const* p_bf16, const int64_t* n,
                          float clip_lo, float clip_hi, double lr, double beta1, double beta2,
                          double eps, int64_t step, void* stream);
/* srnn_adam_clip_multi2 with the step count on the device: dstep (NULL = use `step`) holds
 * the number of completed steps and the kernel takes step = *dstep + 1 for the bias
 * corrections (host formula, torch.optim.Adam).  With srnn_step_advance this makes the
 * optimizer step replayable from a captured HIP graph (trainer/__init__.py graph mode).   */
int srnn_adam_clip_multi3(int ntensors, float* const* p, void* const* g, int gdtype, float gscale,
                          float* const* m, float* const* v, void* const* p_bf16, const int64_t* n,
                          float clip_lo, float clip_hi, double lr, double beta1, double beta2,
                          double eps, int64_t step, const int64_t* dstep, void* stream);
/* dstep[0..n) += 1 unless the persistent-sweep failure flag is up (the step's update was
 * skipped, so its count must not advance either).  n <= 1024.                            */
int srnn_step_advance(int64_t* dstep, int n, void* stream);
/* Data-parallel gradient bucket packing: src[i] (fp32, n[i] elements, NULL = zeros) ->
 * flat + dst_off[i] in dtype (fp32 / bf16), all tensors in one launch.  The reference has no
 * distributed step; this feeds distributed.GradAllReduce's RCCL all-reduce.   */
int srnn_pack_grads(int ntensors, const float* const* src, const int64_t* n,
                    const int64_t* dst_off, void* flat, int dtype, void* stream);
/* bf16 copies of n fp32 tensors (dst[t][j] = bf16(src[t][j]), j < n[t]) in one launch per 64
 * tensors: ZeRO-1 data parallelism refreshes every parameter's bf16 copy after the parameter
 * all-gather (the reference's replicated Adam, optim.py:4-21, sharded over ranks).          */
int srnn_cast_multi(int ntensors, const float* const* src, void* const* dst, const int64_t* n,
                    void* stream);

/* ---- autoregressive generation (Generator.__call__, model.py:445-520) --------------- */
typedef struct SrnnTier {
    int frame_size;            /* upsampling ratio of this tier                           */
    int n_frame_samples;       /* nfs = cumprod(frame_sizes)                              */
    int in_dim;                /* columns of w_in: nfs (+ cond_dim for the top tier)      */
    const void* w_in;          /* (D, in_dim) [input_expand | cond_expand]               */
    const float* b_in;         /* (D) input_expand bias (lower tiers; top uses row_bias)  */
    const void* w_ih[SRNN_MAX_RNN];
    const float* b_ih[SRNN_MAX_RNN];
    const void* w_hh[SRNN_MAX_RNN];
    const float* b_hh[SRNN_MAX_RNN];
    const void* w_up;          /* (fs*D, D): row j*D+o = conv_t.weight[:, o, j]            */
    const float* b_up;         /* (fs*D):   [j*D+o] = upsampling.bias[o, j]               */
    const float* h0;           /* (n_rnn, D) learned / buffer initial state               */
} SrnnTier;

typedef struct SrnnModel {
    int n_tiers, n_rnn, dim, q_levels, cond_dim, dtype;
    SrnnTier tier[SRNN_MAX_TIERS]; /* index 0 = bottom tier (frame_sizes[0])             */
    const void* tab;           /* (FS0, Q, D) folded embedding . input conv               */
    const void* w_hid;         /* (D, D)  */
    const float* b_hid;
    const void* w_out;         /* (Q, D)  */
    const float* b_out;
} SrnnModel;

/* Rows per group R (8 or 16) of the persistent generation sample loop (gen_mlp.hip) for this
 * shape on this device, or 0 when srnn_generate will use per-sample kernels instead.
 * Replaces nothing in the reference: a capability query for the Generator wrapper. */
int srnn_gen_persistent_rows(int dtype, int n_seqs, int dim, int fs0, int q_levels);
/* Workspace bytes needed by srnn_generate for n_seqs rows. */
int srnn_gen_workspace_size(const SrnnModel* m, int n_seqs, size_t* bytes);
/* Generates n_cond * lookback samples for n_seqs rows.
 *   cond     (n_seqs, n_cond, cond_dim) fp32, per-row conditioning frames
 *   row_bias (n_seqs, D) fp32 = spk_expand(spk_embedding(spk)) + b_spk + b_cond + b_in (top)
 *   noise    (n_cond*L, n_seqs, Q) fp32 Exp(1) draws consumed as argmax(p/q), or NULL to
 *            draw q in-kernel from Philox4x32-10(seed)
 *   seq      (n_seqs, L + n_cond*L) int64, columns [0, L) pre-filled (q_zero); output
 *   logp     optional (n_cond*L, n_seqs, Q) fp32 per-step log-probs (debug / parity)
 *   flags    bit 0: replay the generation block as a hipGraph
 *            bit 1: per-sample kernels instead of the persistent sample loop (gen_mlp.hip,
 *                   used by default where the shape fits; env SRNN_GEN_PERSIST=0 also
 *                   disables it)                                                        */
int srnn_generate(const SrnnModel* m, int n_seqs, int n_cond, const float* cond,
                  const float* row_bias, const float* noise, uint64_t seed, int64_t* seq,
                  float* logp, void* workspace, size_t workspace_bytes, int flags, void* stream);
/* srnn_generate for rows [row0, row0 + n_seqs) of a larger batch (rank-sharded generation,
 * SURVEY §8e, generate.py:241-253 run per rank): the Philox noise of local row b is that of
 * global row row0 + b, so the shards together draw exactly the single-process stream.    */
int srnn_generate2(const SrnnModel* m, int n_seqs, int n_cond, const float* cond,
                   const float* row_bias, const float* noise, uint64_t seed, int row0,
                   int64_t* seq, float* logp, void* workspace, size_t workspace_bytes, int flags,
                   void* stream);

#ifdef __cplusplus
}
#endif
#endif
