/*
 * fs2_hip.h -- C ABI of the MI355X (gfx950) FastSpeech2-with-emotion-intensity train path.
 *
 * The reference (Orca0917/fine-grained-emotional-control-of-tts) has no native boundary:
 * its hot path is Python calling speechbrain/torch ops.  Each entry point below replaces
 * one op site of that path ("op-site inventory" K1..K17) and cites the
 * reference line(s) it stands in for.  Conventions (identical for every function):
 *
 *   - all tensor arguments are DEVICE pointers; sizes are explicit ints; row pitches are in
 *     ELEMENTS; nothing is allocated, freed or synchronised inside a call;
 *   - `dtype` selects the activation storage type: FS2_F32 (parity mode) or FS2_BF16;
 *     statistics, losses, gradients of parameters and optimiser state are always fp32;
 *   - `stream` is a hipStream_t passed as void*; all work is stream-ordered (graph-capturable);
 *   - return value: 0 on success, a hipError_t code (>0) on launch failure, or a negative
 *     FS2_E* code for an invalid argument (checked on the host before any launch).
 *
 * Row layout of every token tensor: row m = b*T + t (utterance-major, padded to T), channels
 * contiguous -- the (B, T_max, hidden) layout of the reference (model.py:335-431).
 */
#ifndef FS2_HIP_H
#define FS2_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FS2_F32 0
#define FS2_BF16 1

#define FS2_EINVAL (-1)  /* inconsistent sizes / pointers                                  */
#define FS2_EALIGN (-2)  /* pitch or pointer not 16-byte aligned where the kernel needs it */

/* ------------------------------------------------------------------------------------------
 * Generalised MFMA GEMM:  C[m][n] = epilogue( sum_k A(m,k) * B(k,n) )
 * Replaces: every nn.Linear / nn.Conv1d / bmm of the FFT blocks, variance predictors,
 * concat projection, mel linear and PostNet, forward and backward (K4, K6-K8, K12, K13, K16);
 * SB Conv1d "same"+reflect (App. A.1) is folded into the operand loader ("implicit conv").
 * ------------------------------------------------------------------------------------------ */
typedef struct fs2_gemm_desc {
  int M, N, K;          /* problem size; K is the iterated reduction length                  */
  int kvalid;           /* MN-major operands: k rows >= kvalid read as zero (<=0: = K)       */
  int mvalid, nvalid;   /* epilogue stores only m < mvalid, n < nvalid (<=0: M / N)          */
  int dtype;            /* FS2_F32 | FS2_BF16 : A, B and activation-typed outputs            */
  const void* A; int64_t lda; int a_kmajor;   /* 1: A(m,k)=A[m*lda+k]   0: A[k*lda+m]       */
  const void* B; int64_t ldb; int b_kmajor;   /* 1: B(k,n)=B[n*ldb+k]   0: B[k*ldb+n]       */
  /* implicit 1-D convolution over the token axis (SB Conv1d, reflect "same" padding):
   *   1: A fwd   A(m=(b,t), k=(j,c)) = X[b, reflect(t+j-P), c]                  (a_kmajor)
   *   2: A dgrad A(m=(b,s), k=(j,o)) = sum_{t: reflect(t+j-P)=s} dY[b, t, o]     (a_kmajor)
   *   3: B wgrad B(k=(b,t), n=(j,c)) = X[b, reflect(t+j-P), c]                  (!b_kmajor)
   *   4: A shift A(m=(b,p), k=(j,o)) = dY[b, p-j, o] (0 outside [0,T)), T+2P rows per
   *      utterance: the data gradient in the padded domain, finished by fs2_conv_fold
   *   5: A fwd   A(m=(b,t), k=(j,c)) = X[b, t+j-P, c], 0 outside [0,T): zero-padded "same"
   *      conv (torch nn.Conv1d(padding=k//2), IntensityExtractor FFN, rank_model/model.py:23-24)
   *   6: B wgrad, K-major over padded channel-major images (fs2_pad_transpose):
   *      B(k, n=(j,c)) = B[c*ldb + k + j - P] (b_kmajor; k runs over the padded token domain,
   *      T+2P columns per utterance; A = the zero-padded channel-major dY image, so products
   *      across utterances vanish).  B must have 64 readable elements before it and P after
   *      each row end; K % 64 == 0; fp32 output, split-K only as split_stride slices with
   *      K % (64 * split_k) == 0, no epilogue operations
   * P = (conv_kw-1)/2, conv_c = channels per tap, conv_t = tokens per utterance.          */
  int conv_mode, conv_t, conv_kw, conv_c;
  void* C; int64_t ldc; int c_fp32;           /* output; c_fp32: float output else dtype     */
  int c_conv_kw;        /* >0: output column n=(j,c) is stored at c*c_conv_kw + j            */
  const float* bias;    /* [N]       v += bias[n]                                             */
  int relu;             /* 1: v = max(v, 0); 2: v = GELU(v) = v/2 (1 + erf(v/sqrt 2));
                           3: leaky ReLU slope 0.1; 4: tanh                                    */
  const void* gate; int64_t ldg;              /* dtype [M][ldg]: v *= (gate > 0)             */
  const float* row_scale;                     /* [M]: v *= row_scale[m]                      */
  const void* residual; int64_t ldr;          /* dtype [M][ldr]: v += residual               */
  const float* row_scale_post;                /* [M]: v *= row_scale_post[m]                 */
  int accumulate;       /* fp32 output only: C += v (split_k > 1 implies atomic accumulate)   */
  int split_k;          /* >1: K split over blockIdx.z, fp32 atomics into C                  */
  int64_t split_stride; /* >0 (with split_k > 1, !accumulate): split z stores its fp32 partial
                         * to C + z*split_stride elements instead -- no atomics; slices a
                         * shortened split leaves unused are zeroed.  Consumers sum slices.    */
  /* batched: z in [0,batch): offset(z) = (z / batch_div)*s1 + (z % batch_div)*s2 (elements) */
  int batch, batch_div;
  int64_t sA1, sA2, sB1, sB2, sC1, sC2, sR1, sR2;
  int conv_dil;         /* dilation of conv modes 1 / 5 (tap j reads row t + (j-P)*dil); 0 = 1 */
  /* c_row_t > 0, c_row_pad > 0: output row m is stored at C row m + (m / c_row_t) * c_row_pad
   * -- a token-major result written into a padded token domain (c_row_pad zero rows between
   * utterances, which the caller keeps zero), e.g. the FFN conv2 data gradient straight into
   * the zero-padded dY image of the conv1 data gradient.  c_row_pad < 0: the inverse -- rows m
   * of a padded domain (L = c_row_t - c_row_pad rows per utterance) with m mod L < c_row_t are
   * stored at m - (m / L) * (-c_row_pad), the others dropped (a conv forward over the padded
   * domain, fs2_pad_rows).  bf16, both K-major, no split / batch / conv; runs on the 4-wave
   * or the persistent 256-row kernel (FS2_EINVAL where neither applies).                    */
  int c_row_t, c_row_pad;
  /* grid budget of the persistent GEMM kernels for this call (0 or >= 256: one block per CU):
   * a GEMM enqueued beside a latency-critical stream -- the weight gradients of the train step
   * (model.py:279-441 backward) beside the data-gradient chain -- leaves 256 - max_ctas CUs to
   * the other stream's kernels; 8..255, rounded down to 8.  Results do not depend on it.     */
  int max_ctas;
  /* a_kw > 0: tap-inner K order for a plain K-major A whose rows overlap (the conv1 data
   * gradient over the padded dY image, lda = the image's channel count Ci, K = a_kw * Ci,
   * Ci % 64 == 0): k = (chunk q, tap j, i) -> A(m, k) = A[(m + j)*lda + 64 q + i], i < 64 --
   * consecutive 64-deep K-stages read image rows one tap apart, so each row is fetched from HBM
   * about once instead of once per tap.  B must be in the same order (fs2_weight_prep w_okc
   * bit 2; the forward's Wf: bit 3).  bf16, no split / batch / conv; always the 4-wave
   * kernel.                                                                                 */
  int a_kw;
} fs2_gemm_desc;

int fs2_gemm(const fs2_gemm_desc* d, void* stream);

/* reflect-padding adjoint + dgrad epilogue (K16): Xpad fp32 [B][T+2P][C] from conv_mode 4
 * (nsplit split-K slices split_stride floats apart, summed here; nsplit <= 1: one slice),
 *   out[b,s] = ((Xpad[s+P] + Xpad[P-s]{1<=s<=P} + Xpad[2(T-1)-s+P]{T-1-P<=s<=T-2}) * rs
 *              + residual) * rs2                                                           */
int fs2_conv_fold(const float* Xpad, int nsplit, int64_t split_stride, int B, int T, int P,
                  int C, void* out, int64_t ldo, const void* residual, int64_t ldr,
                  const float* row_scale, const float* row_scale_post, int dtype, void* stream);

/* channel-major padded image for conv_mode 6 (backward of the SB Conv1d weights, App. A.1;
 * model.py:241-267 FFN conv1): out[c][b*(T+2P) + i] = X[b*T + reflect(i-P)][c] (reflect = 1)
 * or X[b*T + i-P][c] inside [0,T) and 0 outside (reflect = 0), i in [0, T+2P); columns
 * [B*(T+2P), ncols) are written as 0.  X bf16 [B*T][ldx]; out bf16 [C][ldo]; C, ldx, ldo,
 * ncols multiples of 8, ldo >= ncols >= B*(T+2P), both pointers 16-byte aligned.
 * colsum (optional, reflect = 0 only): colsum[c] += sum_t X[t][c] -- the conv bias gradient
 * (K13 bias), replacing an fs2_colsum pass; workspace >= ceil(ncols/64) * C floats.        */
int fs2_pad_transpose(const void* X, int64_t ldx, int B, int T, int C, int P, int reflect,
                      void* out, int64_t ldo, int ncols, float* colsum, float* workspace,
                      int dtype, void* stream);

/* out[i] (+)= sum_{s < nslices} ws[s*stride + i], i < n (fp32; n, stride multiples of 4,
 * 16-byte aligned): the sum of split-K weight-gradient slices written by fs2_gemm with
 * split_stride (no atomics; fixed summation order)                                         */
int fs2_sum_slices(const float* ws, int nslices, int64_t stride, int64_t n, float* out,
                   int accumulate, void* stream);

/* token-major padded image for a conv forward over the padded token domain (SB Conv1d
 * "same"+reflect, App. A.1; model.py:241-267 FFN conv1): out row b*(T+2P) + i = X row
 * b*T + reflect(i-P) (reflect = 1) or X row b*T + i-P inside [0,T) and zero outside
 * (reflect = 0), i in [0, T+2P); then `tail` zero rows (the guard the overlapping-row GEMM
 * reads past the last utterance).  With it the conv is a plain K-major GEMM over the padded
 * domain, A(m, k=(j,c)) = out[m*ldo + k] (lda = ldo = C), whose rows m with
 * m mod (T+2P) >= T are dropped by fs2_gemm's c_row (T, -2P).  bf16; C, ldx, ldo multiples
 * of 8, 16-byte aligned pointers. */
int fs2_pad_rows(const void* X, int64_t ldx, int B, int T, int C, int P, int reflect, int tail,
                 void* out, int64_t ldo, int dtype, void* stream);

/* column sums: out[n] (+)= sum_m X[m][n]   (bias gradients; SB Linear/Conv1d bias, K16) */
int fs2_colsum(const void* X, int64_t ldx, int M, int N, int dtype, float* out, int accumulate,
               float* workspace, void* stream);
int64_t fs2_colsum_workspace_floats(int M, int N);

/* ------------------------------------------------------------------------------------------
 * LayerNorm with fused residual / dropout / tanh / mask (K5, K8, K13)
 *   s = x + drop(r; p_r)          (r optional; SB TransformerEncoderLayer, App. A.2)
 *   y = LN(s)*gamma + beta         (eps per call: 1e-6 FFT, 1e-5 predictors/PostNet)
 *   y = tanh(y) (opt) ; y = drop(y; p_o) ; y *= row_mask (opt) ; y += post_add (opt)
 * ------------------------------------------------------------------------------------------ */
/* img (optional, bf16, M % img_t == 0, img_p < img_t): also y's reflect-padded token-major
 * image as fs2_pad_rows(y, ..., img_t, D, img_p, reflect 1, tail 0) writes it (row pitch D) --
 * the FFN conv1 forward's operand, written by the LayerNorm that produces its input
 * (SB Conv1d "same"+reflect, App. A.1) instead of a separate pass.                        */
int fs2_ln_fwd(const void* x, int64_t ldx, const void* r, int64_t ldr, float p_r, uint32_t salt_r,
               void* s_out, const float* gamma, const float* beta, float eps, int do_tanh,
               float p_o, uint32_t salt_o, const float* row_mask, const void* post_add,
               int64_t ldp, void* y, int64_t ldy, float* mean, float* rstd, int M, int D,
               int dtype, uint32_t seed, void* img, int img_t, int img_p, void* stream);

/* backward of fs2_ln_fwd; dgamma/dbeta (+)= column sums (fp32).  ds = dL/ds (optionally
 * gated by (s > 0) for a ReLU that produced s), dr = ds * dropmask_r / (1 - p_r).
 * dcol (optional) (+)= column sums of dr (or of ds when dr is NULL): the bias gradient of
 * the layer whose output fed r (resp. s), fused here instead of a separate fs2_colsum.    */
int fs2_ln_bwd(const void* dy, int64_t lddy, const void* s, int64_t lds, const float* mean,
               const float* rstd, const float* gamma, const float* beta, int do_tanh, float p_o,
               uint32_t salt_o, const float* row_mask, int relu_gate_in, void* ds, int64_t ldds,
               void* dr, float p_r, uint32_t salt_r, float* dgamma, float* dbeta, float* dcol,
               int M, int D,
               int dtype, uint32_t seed, float* workspace, void* stream);
int64_t fs2_ln_workspace_floats(int M, int D);

/* ------------------------------------------------------------------------------------------
 * Attention softmax over materialised scores, with the reference's key masking
 * (model.py:338-343 / 414-419 + key_padding_mask; head-major tiling quirk):
 *   mask_mode 1: batch z = b*H + h masks key k iff key_pad[b][k] || key_pad[(b*H+h) % B][k];
 *   mask_mode 0: plain key padding key_pad[b][k] (IntensityExtractor MHA,
 *                rank_model/model.py:35,101).
 * S: fp32 [z][Tq][ldt]; P, Pd: dtype [z][Tq][ldt] (softmax and dropped softmax, zero-padded
 * to ldt); scale applied to S before the softmax (torch MHA q-scaling).
 * ------------------------------------------------------------------------------------------ */
int fs2_softmax_fwd(const float* S, const uint8_t* key_pad, int mask_mode, int B, int H, int Tq,
                    int Tk, int ldt, float scale, float p_drop, uint32_t seed, uint32_t salt,
                    void* P, void* Pd, int dtype, void* stream);
/* dS = scale * P * (dP - rowsum(P*dP)) with dP = dPd * dropmask / (1-p). dPd fp32.        */
int fs2_softmax_bwd(const float* dPd, const void* P, int B, int H, int Tq, int Tk, int ldt,
                    float scale, float p_drop, uint32_t seed, uint32_t salt, void* dS, int dtype,
                    void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused attention (bf16; K4/K16): softmax(scale * Q K^T with the tiling mask) -> dropout -> PV
 * without materialising the (B*H, T, T) scores.  Q | K | V are column blocks of the packed
 * projection qkv [B*T][ldq] (head h at columns h*dh of each block); out [B*T][ldo] gets head h
 * at h*dh; lse [B*H][T] keeps the log2-domain log-sum-exp for the backward, which writes
 * dQ | dK | dV into dqkv with the same layout as qkv.  Same mask rule and dropout indices as
 * fs2_softmax_fwd/bwd.  Requires dtype bf16, dh in {64,128,192,256}, T <= 2048
 * (fs2_attn_supported); workspace: fs2_attn_workspace_floats.
 * ------------------------------------------------------------------------------------------ */
int fs2_attn_supported(int T, int dh, int dtype);
int fs2_attn_fwd(const void* qkv, int64_t ldq, const uint8_t* key_pad, int mask_mode, int B,
                 int H, int T, int dh, float scale, float p_drop, uint32_t seed, uint32_t salt,
                 void* out, int64_t ldo, float* lse, int dtype, void* stream);
int fs2_attn_bwd(const void* qkv, int64_t ldq, const uint8_t* key_pad, int mask_mode,
                 const void* out,
                 int64_t ldo, const void* dout, int64_t lddo, const float* lse, int B, int H,
                 int T, int dh, float scale, float p_drop, uint32_t seed, uint32_t salt,
                 void* dqkv, int64_t lddq, float* workspace, int dtype, void* stream);
int64_t fs2_attn_workspace_floats(int B, int H, int T);

/* ------------------------------------------------------------------------------------------
 * Token embedding + positional encoding + pad mask (K1, K2; model.py:331-337)
 *   X[m] = (E[tok[m]] + pe[t]) * (tok[m] != pad);  keep[m] = (tok[m] != pad)
 * ------------------------------------------------------------------------------------------ */
int fs2_embed_fwd(const int64_t* tokens, const float* table, const float* pe, int pad_idx,
                  int B, int T, int D, void* X, float* keep, int dtype, void* stream);
/* dTable[v] (+)= sum_{m: tok[m]==v} dX[m] * keep[m]   (deterministic: token-chunk partials in
 * per-wave LDS accumulators, summed in a fixed order); V <= 128;
 * workspace >= fs2_embed_bwd_workspace_floats(D, V) floats                                 */
int fs2_embed_bwd(const int64_t* tokens, const void* dX, const float* keep, int M, int D,
                  int V, float* dtable, float* workspace, int dtype, void* stream);
int64_t fs2_embed_bwd_workspace_floats(int D, int V);

/* key padding masks: from tokens (tok==pad) or from lengths (t >= len)                    */
int fs2_keypad_from_tokens(const int64_t* tokens, int pad_idx, int M, uint8_t* key_pad,
                           void* stream);
int fs2_keypad_from_lengths(const int64_t* lens, int B, int T, uint8_t* key_pad, float* keep,
                            void* stream);

/* concat [feats, spk_emb[spk[b]], intensity, 0-pad] (model.py:352-358) -> cat [M][ldc]    */
int fs2_concat_fwd(const void* feats, const float* spk_table, const int64_t* spk,
                   const float* intensity, int B, int T, int D, int E, void* cat, int ldc,
                   int dtype, void* stream);
/* dSpk[spk[b]] (+)= sum_t dcat[b,t,D:2D]                                                  */
int fs2_concat_bwd_spk(const void* dcat, int ldc, const int64_t* spk, int B, int T, int D,
                       int n_spk, float* dspk, int dtype, float* workspace /* B*D */,
                       void* stream);

/* rows: X[m][:] *= keep[m]   (in place)                                                   */
int fs2_mask_rows(void* X, int64_t ldx, const float* keep, int M, int D, int dtype, void* stream);
/* X = (X + Y + Z) * keep[row] over M x D (row pitch ld for all three), summed in fp32 and
 * rounded once: the join of the predictor input gradients when the duration / pitch predictor
 * backward runs on its own stream (model.py:365-403 variance adaptor backward).  Z may be null
 * (X = (X + Y) * keep[row]). */
int fs2_add3_mask_rows(void* X, const void* Y, const void* Z, int64_t ld, const float* keep,
                       int M, int D, int dtype, void* stream);

/* predictor head: y[m] = (dot(u[m], w) + b) * scale (SB DurationPredictor.linear, App. A.7) */
int fs2_rowdot_fwd(const void* u, int64_t ldu, const float* w, const float* b, float scale, int M,
                   int D, void* y, int dtype, void* stream);
/* du = dy*scale*w ; dw (+)= sum_m dy*scale*u ; db (+)= sum_m dy*scale                     */
int fs2_rowdot_bwd(const void* dy, const void* u, int64_t ldu, const float* w, float scale, int M,
                   int D, void* du, float* dw, float* db, int dtype, float* workspace,
                   void* stream);

/* average_over_durations (SB, App. A.10; model.py:383,397): mean of NON-ZERO frame values
 * per phoneme via double-accumulated prefix sums (replicates torch CPU cumsum).            */
int fs2_avg_over_durations(const float* values, int Tm_in, const int64_t* durs, int B, int Tp,
                           float* avg, float* workspace, void* stream);
int64_t fs2_avg_workspace_floats(int B, int Tm_in);

/* pitch/energy embedding conv (SB Conv1d(1->D, k, reflect), model.py:226-240,384-403) fused
 * with the residual add:  out[b,t,:] = base[b,t,:] + bias + sum_j W[:, 0, j] a[b, refl(t+j-P)] */
int fs2_embed1d_fwd(const void* base, const float* a, const float* W, const float* bias, int B,
                    int T, int D, int KW, void* out, int dtype, void* stream);
/* dW[o][j] (+)= sum dOut[b,t,o] a[b,refl(t+j-P)]; dbias (+)= sum dOut                     */
int fs2_embed1d_bwd(const void* dout, const float* a, int B, int T, int D, int KW, float* dW,
                    float* dbias, int dtype, float* workspace, void* stream);

/* ------------------------------------------------------------------------------------------
 * LengthRegulator (SB upsample, App. A.9; model.py:406-413), K11.
 *   n[b,p] = (int64)(pace * (float)d[b,p])  (float32 product, truncation == .long())
 *   mel_len[b] = sum_p n[b,p];  frame_src[b,t] = p with cum[p-1] <= t < cum[p], -1 past mel_len
 * The integer expansion is bit-exact to repeat_interleave.  d: int64 (teacher forcing) or
 * float (predicted, already clamp(expm1(.),0)) selected by d_is_float.
 * ------------------------------------------------------------------------------------------ */
int fs2_lr_index(const void* durs, int d_is_float, float pace, int B, int Tp, int Tm,
                 int64_t* mel_len, int32_t* cum, int32_t* frame_src, void* stream);
/* Y[b,t] = (X[b, frame_src[b,t]] + pe[t]) * keep[b,t]  (fused decoder PE add, model.py:422-423) */
int fs2_lr_gather(const void* X, const int32_t* frame_src, const float* pe, int B, int Tp,
                  int Tm, int D, void* Y, float* keep, int dtype, void* stream);
/* dX[b,p] = sum_{t in segment p} dY[b,t] * keep[b,t]                                      */
int fs2_lr_scatter(const void* dY, const int32_t* cum, const float* keep, int B, int Tp, int Tm,
                   int D, void* dX, int dtype, void* stream);

/* ------------------------------------------------------------------------------------------
 * Loss (loss.py:62-186), K14/K15.  loss_out[8] fp32 = {total, ssim, mel, postnet, dur, pitch,
 * energy, ssim_gradient_scale}; gradients are written for a unit upstream gradient.
 * ------------------------------------------------------------------------------------------ */
typedef struct fs2_loss_desc {
  int B, Tm, Tp, NM;           /* Tm: padded frames of predictions AND target               */
  int dtype;                   /* predictions' dtype                                         */
  const void* mel_out; const void* postnet_out;       /* [B][Tm][NM]                       */
  const void* log_dur; const void* pitch_pred; const void* energy_pred;  /* [B][Tp]         */
  const float* mel_tgt;                               /* [B][Tm][NM]                        */
  const int64_t* dur_tgt;                             /* [B][Tp]                            */
  const float* pitch_avg; const float* energy_avg;    /* [B][Tp] (average_over_durations)   */
  const int64_t* mel_len; const int64_t* phon_len;    /* [B]                                */
  float w_ssim, w_mel, w_post, w_dur, w_pitch, w_energy;
  float* loss_out;                                     /* [8]                                */
  void* d_mel_out; void* d_postnet_out;               /* dtype, [B][Tm][NM]                 */
  void* d_log_dur; void* d_pitch; void* d_energy;     /* dtype, [B][Tp]                     */
  float* workspace;                                    /* fs2_loss_workspace_floats()        */
} fs2_loss_desc;
int fs2_loss_fwd_bwd(const fs2_loss_desc* d, void* stream);
int64_t fs2_loss_workspace_floats(int B, int Tm, int NM);

/* ------------------------------------------------------------------------------------------
 * Optimiser + weight preparation (K17; train.py:232 torch.optim.AdamW defaults).
 * ------------------------------------------------------------------------------------------ */
/* torch AdamW (single-tensor algorithm, fp32), grads scaled by grad_scale (1/world_size).
 * c_* constants are computed on the host exactly as torch does (see fastspeech2/optim.py). */
int fs2_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
              float decay_mul, float one_minus_beta1, float beta2, float one_minus_beta2,
              float step_size, float bc2_sqrt, float eps, float grad_scale, void* stream);

/* master weight W (fp32) -> fwd copy Wf[O][KW][C] and dgrad copy Wb[C][KW][O] in dtype, each
 * with row pitch padded to ldf / ldb elements (zeros in the pad).  W is stored torch-style
 * [O][C][KW] (w_okc bit 0 clear) or [O][KW][C] (bit 0 set, the flat-buffer layout of conv
 * weights).  w_okc bit 1: Wb's taps reversed, Wb[C][KW-1-j][O] -- the order in which the conv
 * data gradient over a zero-padded token-major dY image is a plain K-major GEMM whose A rows
 * overlap (A(m, k) = image[m*O + k], lda = O).  w_okc bit 2 (O % 64 == 0): Wb's columns in
 * tap-inner 64-channel chunks, column (o/64)*KW*64 + j*64 + o%64 (fs2_gemm_desc.a_kw); bit 3
 * (C % 64 == 0, ldf == KW*C): Wf's columns the same way, (c/64)*KW*64 + j*64 + c%64. */
int fs2_weight_prep(const float* W, int O, int C, int KW, int w_okc, void* Wf, int ldf, void* Wb,
                    int ldb, int dtype, void* stream);

/* All of a model's weight images in ONE launch: descs (DEVICE memory) lists n weights, each
 * cut into 64 x 64 tiles of its [O][ldf] forward image; tile0 = first tile index of weight i
 * (prefix sum, ascending), tiles_k = ceil(ldf / 64).  Each tile is read once (coalesced),
 * written to Wf, and transposed through LDS into Wb (coalesced along o); Wb may be NULL.
 * total_tiles = tile0 + tiles of the last weight; n <= 256.                               */
typedef struct fs2_wprep_desc {
  const float* W; void* Wf; void* Wb;
  int O, C, KW, w_okc, ldf, ldb;
  int tile0, tiles_k;
} fs2_wprep_desc;
int fs2_weight_prep_batched(const fs2_wprep_desc* descs, int n, int total_tiles, int dtype,
                            void* stream);
/* AdamW fused with the weight images (replaces fs2_adamw + fs2_weight_prep_batched after an
 * optimiser step, K17 of SURVEY §2): the descriptor table's weights are updated tile by tile
 * and their Wf / Wb images written from the updated values; every other parameter lies in
 * `ranges` (int64 triples: flat start, length, first block; 1024 elements per block).  All
 * pointers index the same flat layout: descs[i].W - param is a weight's flat offset. */
int fs2_adamw_prep(const fs2_wprep_desc* descs, int n, int total_tiles, const int64_t* ranges,
                   int n_ranges, int range_blocks, float* param, const float* grad,
                   float* exp_avg, float* exp_avg_sq, float decay_mul, float one_minus_beta1,
                   float beta2, float one_minus_beta2, float step_size, float bc2_sqrt, float eps,
                   float grad_scale, int dtype, void* stream);

/* ------------------------------------------------------------------------------------------
 * Frozen IntensityExtractor forward pieces + phoneme averaging (SURVEY §8f-1;
 * rank_model/model.py:96-109, fastspeech2/train.py:16-51).  The extractor's GEMMs use
 * fs2_gemm (conv_mode 5 zero-padded k=9 convs, relu=2 GELU), fs2_attn_fwd / fs2_softmax_fwd
 * with mask_mode 0, and fs2_ln_fwd (eps 1e-5).
 * ------------------------------------------------------------------------------------------ */
/* rank_X fp32 (B,T,C) (layout_bct=0) or the collate's (B,C,T) (layout_bct=1, the explicit fix of
 * SURVEY App. B-2) -> GEMM rows X[B*T][ldx] in dtype, columns >= C zero.                    */
int fs2_intensity_input(const float* x, int layout_bct, int B, int T, int C, void* X, int ldx,
                        int dtype, void* stream);
/* I[b,t,e] = (t < lengths[b]) ? (H[b,t] + emo_table[emotions[b]]) . Wc[e] + bc[e] : bc[e]
 * (model.py:103-107: emotion embedding add, masked_fill, classifier); I fp32 (B,T,E), E <= 8 */
int fs2_intensity_head(const void* H, int64_t ldh, const float* emo_table,
                       const int64_t* emotions, const int64_t* lengths, const float* Wc,
                       const float* bc, int B, int T, int D, int E, float* I, int dtype,
                       void* stream);
/* out[b,p,:] = sum of I[b, t, :] over phoneme p's frames [sum d[:p], sum d[:p+1]) (clipped to
 * T) / max(d[b,p], 1) for p < phon_len[b]; 0 otherwise (train.py:33-49). Tp <= 1024.        */
int fs2_phoneme_average(const float* I, int T, int E, const int64_t* durations,
                        const int64_t* phon_len, int B, int Tp, float* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * GPU collate: TextMelCollateWithAlignment (fastspeech2/dataset.py:62-133) over
 * one packed upload.  Item u's phonemes / durations are [offsets[u], offsets[u+1]) of the
 * packed int64 arrays; its mel is (n_mels, T_u) channel-major at frame_offsets[u] * n_mels,
 * pitch / energy at frame_offsets[u].  order[i] = item placed at batch row i (the collate's
 * descending torch.sort of phoneme lengths).  Outputs are zero padded: phoneme / duration
 * (B, Tp) int64, mel (B, Tm, n_mels) (the collate's permute(0,2,1), contiguous), pitch /
 * energy (B, Tm), rank_x (B, n_mels+2, Tm) = cat(mel, pitch, energy), lengths (B,) int64.
 * ------------------------------------------------------------------------------------------ */
int fs2_collate_phonemes(const int32_t* order, const int64_t* offsets, const int64_t* phonemes,
                         const int64_t* durations, int B, int Tp, int64_t* phoneme_padded,
                         int64_t* duration_padded, int64_t* input_lengths, void* stream);
int fs2_collate_frames(const int32_t* order, const int64_t* frame_offsets, const float* mel,
                       const float* pitch, const float* energy, int B, int Tm, int n_mels,
                       float* mel_padded, float* pitch_padded, float* energy_padded,
                       float* rank_x, int64_t* output_lengths, void* stream);

/* ------------------------------------------------------------------------------------------
 * HiFi-GAN generator forward (speechbrain HIFIGAN.decode_batch,
 * fastspeech2/inference.py:60-63,85).  Convs on fs2_gemm (conv_mode 1 + conv_dil, transposed
 * convs as 3-tap polyphase conv_mode 5, act 3 / 4 epilogues, residual epilogue).
 * ------------------------------------------------------------------------------------------ */
/* mel (B, n_mels, T) fp32 -> X[B*(T+2 pad)][ldx] (dtype), pad replicated frames each side   */
int fs2_vocoder_input(const float* mel, int B, int n_mels, int T, int pad, void* X, int ldx,
                      int dtype, void* stream);
/* y = leaky_relu(x, slope); n % (16 / sizeof(dtype)) == 0, 16-byte aligned                  */
int fs2_leaky_relu(const void* x, void* y, int64_t n, float slope, int dtype, void* stream);
/* y = leaky_relu(((a + b) + c) / 3, slope)                                                  */
int fs2_mean3_leaky_relu(const void* a, const void* b, const void* c, void* y, int64_t n,
                         float slope, int dtype, void* stream);

/* utilities */
int fs2_fill(void* X, int64_t n, float value, int dtype, void* stream);
/* X[i] += alpha * Y[i] over n elements of dtype                                           */
int fs2_add(void* X, const void* Y, int64_t n, float alpha, int dtype, void* stream);
int fs2_cast(const void* src, int src_dtype, void* dst, int dst_dtype, int64_t n, void* stream);
/* Dropout seed base (device-resident, added to every launch's seed argument): HIP-graph
 * replays of a step captured with seed 0 set it to the step's seed first; eager steps leave
 * it 0.  Stream-ordered. */
int fs2_set_dropout_seed(uint32_t seed_base, void* stream);
const char* fs2_version(void);
/* first 16 hex digits of the SHA-256 of the sources the library was built from (csrc/*.hip
 * in name order, csrc/fs2_common.h, this header): fastspeech2/_native.py refuses a library
 * whose hash differs from the tree's sources (a stale build)                                */
const char* fs2_source_hash(void);

#ifdef __cplusplus
}
#endif
#endif /* FS2_HIP_H */
