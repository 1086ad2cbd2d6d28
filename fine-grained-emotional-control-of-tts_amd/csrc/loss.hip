// FastSpeech2 loss (loss.py:62-186) forward + gradient in one stream-ordered pass.
//
//  * mel / postnet MSE over [:mel_len] per utterance, duration MSE on log1p targets over
//    [:phon_len], pitch / energy MSE over [:min(mel_len, Tp)] of the PHONEME axis (the
//    reference slices the phoneme-level tensors by the mel length);
//    each term is a per-utterance mean, summed over utterances, divided by B (App. B-7).
//  * SSIM (SB SSIMLoss, App. A.12) on the pre-PostNet mel: per-sample masked min-max
//    normalisation (max taken over the zero-filled padded tensor), 11x11 Gaussian (sigma
//    1.5) "valid" filtering, 1 - mean(SSIM), clamped to [0, 1] (clamped -> zero gradient).
//    The backward routes the min/max gradients to every element equal to the extremum,
//    divided by the tie count (torch amax/amin semantics).
// All reductions are fp32 and deterministic (fixed-order block sums, no float atomics
// except the two per-utterance SSIM normalisation sums).
#include "fs2_common.h"

namespace {

constexpr int WIN = 11;
constexpr int LOSS_CHUNK = 8192;  // mel elements per MSE block
constexpr float C1 = 0.01f * 0.01f, C2 = 0.03f * 0.03f;

struct LossP {
  int B, Tm, Tp, NM;
  const void* mel_out; const void* post_out; const void* log_dur; const void* pitch_pred;
  const void* energy_pred; const float* mel_tgt; const int64_t* dur_tgt; const float* pitch_avg;
  const float* energy_avg; const int64_t* mel_len; const int64_t* phon_len;
  float w_ssim, w_mel, w_post, w_dur, w_pitch, w_energy;
  float* loss_out; void* d_mel; void* d_post; void* d_dur; void* d_pitch; void* d_energy;
  // workspace carve
  float* per_b;      // [5][B]
  float* part_mel;   // [2][B][nch] chunk sums of squared mel / postnet errors
  int nch;
  float* stats;      // [8][B] ymax, ymin, hmax, hmin, cnt_hmax, cnt_hmin, S1, S2
  float* mm_part;    // [B][MMCH][4] chunk max / min of target and prediction
  float* cnt_part;   // [B][MMCH][2] chunk tie counts of the prediction's max / min
  float* ssim_part;  // [B][nblk_pix]
  float* dmap;       // [3][B][npix]
  float* dnmap;      // [B][Tm][NM]
  float* scal;       // [4]
  int npix, nblk_pix;
  int vec;           // every mel operand 16-byte aligned (vectorised MSE pass)
};

__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += sh[i];
  return s;
}
__device__ __forceinline__ float block_max(float v, float* sh) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float s = -INFINITY;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s = fmaxf(s, sh[i]);
  return s;
}
__device__ __forceinline__ float block_min(float v, float* sh) {
  v = wave_min(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float s = INFINITY;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s = fminf(s, sh[i]);
  return s;
}

__device__ __forceinline__ float gauss1(int i) {
  // normalised 1-D Gaussian tap; the 2-D window of gaussian_filter() is its outer product
  float s = 0.f;
  for (int k = 0; k < WIN; ++k) { const float c = k - 5.f; s += expf(-(c * c) / 4.5f); }
  const float c = i - 5.f;
  return expf(-(c * c) / 4.5f) / s;
}

// ---- 1: MSE terms + their gradients -------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) mse_kernel(LossP p) {
  __shared__ float sh[8];
  const int b = blockIdx.x, B = p.B, Tm = p.Tm, Tp = p.Tp, NM = p.NM;
  const int L = (int)min((int64_t)Tm, p.mel_len[b]);
  const int Pl = (int)min((int64_t)Tp, p.phon_len[b]);
  const int Ln = min(L, Tp);  // pitch/energy slice [:mel_len] of the Tp axis
  const T* mo = (const T*)p.mel_out + (long)b * Tm * NM;
  const T* po = (const T*)p.post_out + (long)b * Tm * NM;
  const float* mt = p.mel_tgt + (long)b * Tm * NM;
  T* dmo = (T*)p.d_mel + (long)b * Tm * NM;
  T* dpo = (T*)p.d_post + (long)b * Tm * NM;
  const float cm = 2.f * p.w_mel / ((float)L * NM * B), cp = 2.f * p.w_post / ((float)L * NM * B);
  float s_mel = 0.f, s_post = 0.f;
  const int i0 = blockIdx.y * LOSS_CHUNK, i1 = min(Tm * NM, i0 + LOSS_CHUNK);
  constexpr int V = Vec<T>::N;   // 16-byte accesses: 8 bf16 / 4 fp32 elements per lane
  if (p.vec && NM % V == 0) {    // a lane's V elements share one mel frame (one validity test)
    for (int i = i0 + threadIdx.x * V; i < i1; i += blockDim.x * V) {
      const bool valid = (i / NM) < L;
      float y[V], a[V], c[V], g1[V], g2[V];
#pragma unroll
      for (int e = 0; e < V; e += 4) vload<float>(y + e, mt + i + e);
      vload<T>(a, mo + i);
      vload<T>(c, po + i);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float d1 = a[e] - y[e], d2 = c[e] - y[e];
        if (valid) { s_mel += d1 * d1; s_post += d2 * d2; }
        g1[e] = valid ? cm * d1 : 0.f;
        g2[e] = valid ? cp * d2 : 0.f;
      }
      vstore<T>(dmo + i, g1);
      vstore<T>(dpo + i, g2);
    }
  } else {
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
      const bool valid = (i / NM) < L;
      const float y = mt[i];
      const float d1 = to_f(mo[i]) - y, d2 = to_f(po[i]) - y;
      if (valid) { s_mel += d1 * d1; s_post += d2 * d2; }
      dmo[i] = from_f<T>(valid ? cm * d1 : 0.f);
      dpo[i] = from_f<T>(valid ? cp * d2 : 0.f);
    }
  }
  s_mel = block_sum(s_mel, sh);
  s_post = block_sum(s_post, sh);
  if (threadIdx.x == 0) {
    p.part_mel[(long)b * p.nch + blockIdx.y] = s_mel;
    p.part_mel[(long)(B + b) * p.nch + blockIdx.y] = s_post;
  }
  if (blockIdx.y != 0) return;
  const T* ld = (const T*)p.log_dur + (long)b * Tp;
  const T* pp = (const T*)p.pitch_pred + (long)b * Tp;
  const T* ep = (const T*)p.energy_pred + (long)b * Tp;
  const int64_t* dt = p.dur_tgt + (long)b * Tp;
  const float* pa = p.pitch_avg + (long)b * Tp;
  const float* ea = p.energy_avg + (long)b * Tp;
  T* dd = (T*)p.d_dur + (long)b * Tp;
  T* dpi = (T*)p.d_pitch + (long)b * Tp;
  T* den = (T*)p.d_energy + (long)b * Tp;
  const float cd = 2.f * p.w_dur / ((float)Pl * B);
  const float cpi = 2.f * p.w_pitch / ((float)Ln * B), ce = 2.f * p.w_energy / ((float)Ln * B);
  float s_dur = 0.f, s_pi = 0.f, s_en = 0.f;
  for (int i = threadIdx.x; i < Tp; i += blockDim.x) {
    const float e1 = to_f(ld[i]) - log1pf((float)dt[i]);
    const float e2 = to_f(pp[i]) - pa[i];
    const float e3 = to_f(ep[i]) - ea[i];
    const bool vd = i < Pl, vn = i < Ln;
    if (vd) s_dur += e1 * e1;
    if (vn) { s_pi += e2 * e2; s_en += e3 * e3; }
    dd[i] = from_f<T>(vd ? cd * e1 : 0.f);
    dpi[i] = from_f<T>(vn ? cpi * e2 : 0.f);
    den[i] = from_f<T>(vn ? ce * e3 : 0.f);
  }
  s_dur = block_sum(s_dur, sh);
  s_pi = block_sum(s_pi, sh);
  s_en = block_sum(s_en, sh);
  if (threadIdx.x == 0) {
    p.per_b[2 * B + b] = s_dur / (float)Pl;
    p.per_b[3 * B + b] = s_pi / (float)Ln;
    p.per_b[4 * B + b] = s_en / (float)Ln;
  }
}

// ---- 2: masked min / max of target and prediction -----------------------------------------
// Two passes over MMCH chunks per utterance (grid MMCH x B; one block per utterance left 224 of
// the 256 CUs idle: 83 us): chunk extrema, then every chunk block combines the MMCH partials
// in a fixed order and counts its ties to the prediction's extrema; finalize_kernel sums the
// tie counts.  Same values as one pass over the utterance (max / min are order-free).
constexpr int MMCH = 16;
template <typename T>
__global__ void __launch_bounds__(256) minmax_part_kernel(LossP p) {
  __shared__ float sh[8];
  const int c = blockIdx.x, b = blockIdx.y, Tm = p.Tm, NM = p.NM;
  const int L = (int)min((int64_t)Tm, p.mel_len[b]);
  const int n = L * NM, per = (n + MMCH - 1) / MMCH;
  const int i0 = c * per, i1 = min(n, i0 + per);
  const T* h = (const T*)p.mel_out + (long)b * Tm * NM;
  const float* y = p.mel_tgt + (long)b * Tm * NM;
  float ymx = -INFINITY, ymn = INFINITY, hmx = -INFINITY, hmn = INFINITY;
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const float yv = y[i], hv = to_f(h[i]);
    ymx = fmaxf(ymx, yv); ymn = fminf(ymn, yv); hmx = fmaxf(hmx, hv); hmn = fminf(hmn, hv);
  }
  ymx = block_max(ymx, sh); ymn = block_min(ymn, sh);
  hmx = block_max(hmx, sh); hmn = block_min(hmn, sh);
  if (threadIdx.x == 0) {
    float* o = p.mm_part + ((long)b * MMCH + c) * 4;
    o[0] = ymx; o[1] = ymn; o[2] = hmx; o[3] = hmn;
  }
}
template <typename T>
__global__ void __launch_bounds__(256) minmax_count_kernel(LossP p) {
  __shared__ float sh[8];
  const int c = blockIdx.x, b = blockIdx.y, Tm = p.Tm, NM = p.NM, B = p.B;
  const int L = (int)min((int64_t)Tm, p.mel_len[b]);
  const float* q = p.mm_part + (long)b * MMCH * 4;
  float ymx = -INFINITY, ymn = INFINITY, hmx = -INFINITY, hmn = INFINITY;
  for (int k = 0; k < MMCH; ++k) {
    ymx = fmaxf(ymx, q[4 * k]); ymn = fminf(ymn, q[4 * k + 1]);
    hmx = fmaxf(hmx, q[4 * k + 2]); hmn = fminf(hmn, q[4 * k + 3]);
  }
  const bool has_pad = L < Tm;  // masked_fill(~mask, 0) contributes zeros to the max
  if (has_pad) { ymx = fmaxf(ymx, 0.f); hmx = fmaxf(hmx, 0.f); }
  const int n = L * NM, per = (n + MMCH - 1) / MMCH;
  const int i0 = c * per, i1 = min(n, i0 + per);
  const T* h = (const T*)p.mel_out + (long)b * Tm * NM;
  float cmx = 0.f, cmn = 0.f;
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const float hv = to_f(h[i]);
    cmx += (hv == hmx) ? 1.f : 0.f;
    cmn += (hv == hmn) ? 1.f : 0.f;
  }
  cmx = block_sum(cmx, sh);
  cmn = block_sum(cmn, sh);
  if (threadIdx.x == 0) {
    float* o = p.cnt_part + ((long)b * MMCH + c) * 2;
    o[0] = cmx; o[1] = cmn;
    if (c == 0) {
      float* st = p.stats;
      st[0 * B + b] = ymx; st[1 * B + b] = ymn; st[2 * B + b] = hmx; st[3 * B + b] = hmn;
      st[6 * B + b] = 0.f; st[7 * B + b] = 0.f;
    }
  }
}

// per-utterance min-max normalisation constants, read once per block
struct NormC {
  int L;
  float ymn, yden, hmn, hden;
  __device__ NormC(const LossP& p, int b) {
    L = (int)min((int64_t)p.Tm, p.mel_len[b]);
    const float* st = p.stats;
    const int B = p.B;
    ymn = st[1 * B + b]; yden = st[0 * B + b] - ymn + 1e-8f;
    hmn = st[3 * B + b]; hden = st[2 * B + b] - hmn + 1e-8f;
  }
};
template <typename T>
__device__ __forceinline__ void norm_xy(const LossP& p, const NormC& nc, int b, int t, int f,
                                        float& X, float& Y) {
  if (t >= nc.L) { X = 0.f; Y = 0.f; return; }
  const long i = ((long)b * p.Tm + t) * p.NM + f;
  X = (p.mel_tgt[i] - nc.ymn) / nc.yden;
  Y = (to_f(((const T*)p.mel_out)[i]) - nc.hmn) / nc.hden;
}

// (row, column) walk of a rows x W index space by 256 threads without a division per element
struct Walk {
  int r, c, dr, dc, W;
  __device__ Walk(int W_) : W(W_) {
    r = (int)threadIdx.x / W; c = (int)threadIdx.x - r * W;
    dr = 256 / W; dc = 256 - dr * W;
  }
  __device__ __forceinline__ void next() {
    c += dc; r += dr;
    if (c >= W) { c -= W; ++r; }
  }
};

// ---- 3: SSIM map and its partial derivatives wrt the prediction's local statistics --------
// Separable Gaussian: a block takes SSIM_TI output rows of one utterance, stages the
// normalised X / Y of the SSIM_TI + 10 input rows in LDS, filters along the mel axis (5 moment
// planes), then along time -- 2 x 11 taps per moment instead of 121.
constexpr int SSIM_TI = 16;
constexpr int SSIM_MAXW = 96;                  // n_mels <= 96
constexpr int SSIM_R = SSIM_TI + WIN - 1;
template <typename T>
__global__ void __launch_bounds__(256) ssim_map_kernel(LossP p) {
  __shared__ float sh[8];
  __shared__ float w1[WIN];
  __shared__ float xs[SSIM_R][SSIM_MAXW], ys[SSIM_R][SSIM_MAXW];
  __shared__ float hs[5][SSIM_R][SSIM_MAXW - WIN + 1];
  if (threadIdx.x < WIN) w1[threadIdx.x] = gauss1(threadIdx.x);
  const int b = blockIdx.y, i0 = blockIdx.x * SSIM_TI;
  const int NM = p.NM, OW = NM - (WIN - 1), OH = p.Tm - (WIN - 1);
  const NormC nc(p, b);
  for (Walk w(NM); w.r < SSIM_R; w.next()) {
    const int r = w.r, f = w.c, t = i0 + r;
    float X = 0.f, Y = 0.f;
    if (t < p.Tm) norm_xy<T>(p, nc, b, t, f, X, Y);
    xs[r][f] = X;
    ys[r][f] = Y;
  }
  __syncthreads();
  for (Walk wk(OW); wk.r < SSIM_R; wk.next()) {
    const int r = wk.r, j = wk.c;
    float mx = 0.f, my = 0.f, exx = 0.f, eyy = 0.f, exy = 0.f;
#pragma unroll
    for (int dj = 0; dj < WIN; ++dj) {
      const float w = w1[dj], X = xs[r][j + dj], Y = ys[r][j + dj];
      mx += w * X; my += w * Y; exx += w * X * X; eyy += w * Y * Y; exy += w * X * Y;
    }
    hs[0][r][j] = mx; hs[1][r][j] = my; hs[2][r][j] = exx; hs[3][r][j] = eyy; hs[4][r][j] = exy;
  }
  __syncthreads();
  float ss = 0.f;
  const long plane = (long)p.B * p.npix;
  for (Walk wk(OW); wk.r < SSIM_TI; wk.next()) {
    const int ti = wk.r, j = wk.c, i = i0 + ti;
    if (i >= OH) continue;
    float a = 0.f, bb = 0.f, exx = 0.f, eyy = 0.f, exy = 0.f;
#pragma unroll
    for (int di = 0; di < WIN; ++di) {
      const float w = w1[di];
      a += w * hs[0][ti + di][j]; bb += w * hs[1][ti + di][j]; exx += w * hs[2][ti + di][j];
      eyy += w * hs[3][ti + di][j]; exy += w * hs[4][ti + di][j];
    }
    const float sxx = exx - a * a, syy = eyy - bb * bb, sxy = exy - a * bb;
    const float L1 = 2.f * a * bb + C1, D1 = a * a + bb * bb + C1;
    const float N2 = 2.f * sxy + C2, D2 = sxx + syy + C2;
    const float cs = N2 / D2;
    ss += (L1 / D1) * cs;
    const float dl_db = (2.f * a * D1 - L1 * 2.f * bb) / (D1 * D1);
    const float dn_db = (-2.f * a * D2 + 2.f * bb * N2) / (D2 * D2);
    const float Db = cs * dl_db + (L1 / D1) * dn_db;
    const float Deyy = (L1 / D1) * (-N2 / (D2 * D2));
    const float Dexy = (L1 / D1) * (2.f / D2);
    const long o = (long)b * p.npix + (long)i * OW + j;
    p.dmap[o] = Db; p.dmap[plane + o] = Deyy; p.dmap[2 * plane + o] = Dexy;
  }
  ss = block_sum(ss, sh);
  if (threadIdx.x == 0) p.ssim_part[(long)b * p.nblk_pix + blockIdx.x] = ss;
}

// ---- 4: finalise all loss values ----------------------------------------------------------
__global__ void __launch_bounds__(256) finalize_kernel(LossP p) {
  __shared__ double dsh[256];
  const int B = p.B;
  // deterministic: per-thread strided double sums, then a fixed-shape LDS tree
  double part = 0.0;
  for (int i = threadIdx.x; i < B * p.nblk_pix; i += 256) part += p.ssim_part[i];
  dsh[threadIdx.x] = part;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) dsh[threadIdx.x] += dsh[threadIdx.x + w];
    __syncthreads();
  }
  const double tot = dsh[0];
  // per-utterance mel / postnet means from the chunk partials
  for (int b = threadIdx.x; b < B; b += 256) {
    const int L = (int)min((int64_t)p.Tm, p.mel_len[b]);
    float sm = 0.f, sp = 0.f;
    for (int c = 0; c < p.nch; ++c) {
      sm += p.part_mel[(long)b * p.nch + c];
      sp += p.part_mel[(long)(B + b) * p.nch + c];
    }
    p.per_b[0 * B + b] = sm / ((float)L * p.NM);
    p.per_b[1 * B + b] = sp / ((float)L * p.NM);
    float cmx = 0.f, cmn = 0.f;   // tie counts of the prediction's extrema, fixed order
    for (int c = 0; c < MMCH; ++c) {
      cmx += p.cnt_part[((long)b * MMCH + c) * 2];
      cmn += p.cnt_part[((long)b * MMCH + c) * 2 + 1];
    }
    if (L < p.Tm && p.stats[2 * B + b] == 0.f) cmx += (float)(p.Tm - L) * p.NM;   // zero pads
    p.stats[4 * B + b] = cmx;
    p.stats[5 * B + b] = cmn;
  }
  __syncthreads();
  // utterance means of the five terms: fixed-order block sums (each thread's utterances
  // b = tid, tid + 256, ... in order) instead of a serial thread-0 loop of 5 B dependent loads
  __shared__ float fsh[8];
  float t[5];
  for (int k = 0; k < 5; ++k) {
    float v = 0.f;
    for (int b = threadIdx.x; b < B; b += 256) v += p.per_b[k * B + b];
    t[k] = block_sum(v, fsh) / (float)B;
  }
  if (threadIdx.x != 0) return;
  const float ssim_val = (float)(tot / ((double)B * p.npix));
  float l_ssim = 1.f - ssim_val;
  float gate = 1.f;
  if (l_ssim > 1.f) { l_ssim = 1.f; gate = 0.f; }
  if (l_ssim < 0.f) { l_ssim = 0.f; gate = 0.f; }
  const float ssim_w = l_ssim * p.w_ssim, mel_w = t[0] * p.w_mel, post_w = t[1] * p.w_post;
  const float dur_w = t[2] * p.w_dur, pi_w = t[3] * p.w_pitch, en_w = t[4] * p.w_energy;
  p.loss_out[0] = ssim_w + mel_w + post_w + dur_w + pi_w + en_w;
  p.loss_out[1] = ssim_w; p.loss_out[2] = mel_w; p.loss_out[3] = post_w;
  p.loss_out[4] = dur_w; p.loss_out[5] = pi_w; p.loss_out[6] = en_w;
  const float g = -p.w_ssim * gate / ((float)B * p.npix);
  p.loss_out[7] = g;
  p.scal[0] = g;
}

// ---- 5: gradient wrt the normalised prediction (transposed filtering) ---------------------
template <typename T>
__global__ void __launch_bounds__(256) ssim_grad_kernel(LossP p) {
  // dL/dY at input rows t0 .. t0 + SSIM_TI - 1: the transposed (correlation) Gaussian of the
  // three dmap planes over output rows t0 - 10 .. t0 + SSIM_TI - 1, separable as in the map
  __shared__ float sh[8];
  __shared__ float w1[WIN];
  __shared__ float dsm[3][SSIM_R][SSIM_MAXW - WIN + 1];
  __shared__ float hsm[3][SSIM_R][SSIM_MAXW];
  if (threadIdx.x < WIN) w1[threadIdx.x] = gauss1(threadIdx.x);
  const int b = blockIdx.y, t0 = blockIdx.x * SSIM_TI;
  const int Tm = p.Tm, NM = p.NM, B = p.B;
  const int OH = Tm - (WIN - 1), OW = NM - (WIN - 1);
  const long plane = (long)B * p.npix;
  const float* Db = p.dmap + (long)b * p.npix;
  for (Walk wk(OW); wk.r < SSIM_R; wk.next()) {
    const int r = wk.r, j = wk.c, i = t0 - (WIN - 1) + r;
    const bool ok = i >= 0 && i < OH;
    const long o = (long)i * OW + j;
    dsm[0][r][j] = ok ? Db[o] : 0.f;
    dsm[1][r][j] = ok ? Db[plane + o] : 0.f;
    dsm[2][r][j] = ok ? Db[2 * plane + o] : 0.f;
  }
  __syncthreads();
  for (Walk wk(NM); wk.r < SSIM_R; wk.next()) {
    const int r = wk.r, f = wk.c;
    float u = 0.f, v = 0.f, w = 0.f;
#pragma unroll
    for (int dj = 0; dj < WIN; ++dj) {
      const int j = f - dj;
      if (j < 0 || j >= OW) continue;
      const float g = w1[dj];
      u += g * dsm[0][r][j]; v += g * dsm[1][r][j]; w += g * dsm[2][r][j];
    }
    hsm[0][r][f] = u; hsm[1][r][f] = v; hsm[2][r][f] = w;
  }
  __syncthreads();
  const float g = p.scal[0];
  const NormC nc(p, b);
  const int L = nc.L;
  float s1 = 0.f, s2 = 0.f;
  for (Walk wk(NM); wk.r < SSIM_TI; wk.next()) {
    const int tt = wk.r, f = wk.c, t = t0 + tt;
    if (t >= Tm) continue;
    float U = 0.f, V = 0.f, W = 0.f;
#pragma unroll
    for (int di = 0; di < WIN; ++di) {
      const int r = tt + (WIN - 1) - di;
      const float w = w1[di];
      U += w * hsm[0][r][f]; V += w * hsm[1][r][f]; W += w * hsm[2][r][f];
    }
    float X, Y;
    norm_xy<T>(p, nc, b, t, f, X, Y);
    float dn = 0.f;
    if (t < L) dn = g * (U + 2.f * Y * V + X * W);
    const long q = (long)t * NM + f;
    p.dnmap[(long)b * Tm * NM + q] = dn;
    if (t < L) {
      const float hv = to_f(((const T*)p.mel_out)[(long)b * Tm * NM + q]);
      s1 += dn;
      s2 += dn * (hv - nc.hmn);
    }
  }
  s1 = block_sum(s1, sh);
  s2 = block_sum(s2, sh);
  if (threadIdx.x == 0) {
    atomicAdd(&p.stats[6 * B + b], s1);
    atomicAdd(&p.stats[7 * B + b], s2);
  }
}

// ---- 6: chain through the min-max normalisation into d_mel_out ----------------------------
template <typename T>
__global__ void ssim_apply_kernel(LossP p) {
  const int b = blockIdx.y;
  const int Tm = p.Tm, NM = p.NM, B = p.B;
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (long)Tm * NM) return;
  const int t = (int)(q / NM);
  const int L = (int)min((int64_t)Tm, p.mel_len[b]);
  if (t >= L) return;
  const float* st = p.stats;
  const float hmx = st[2 * B + b], hmn = st[3 * B + b];
  const float den = hmx - hmn + 1e-8f;
  const float r = 1.f / den;
  const float S1 = st[6 * B + b], S2 = st[7 * B + b];
  const float dmn = -r * S1 + r * r * S2;
  const float dmx = -r * r * S2;
  const long i = (long)b * Tm * NM + q;
  const float hv = to_f(((const T*)p.mel_out)[i]);
  float g = p.dnmap[i] * r;
  if (hv == hmx) g += dmx / st[4 * B + b];
  if (hv == hmn) g += dmn / st[5 * B + b];
  T* d = (T*)p.d_mel + i;
  *d = from_f<T>(to_f(*d) + g);
}

template <typename T>
int run_loss(LossP& p, hipStream_t s) {
  hipLaunchKernelGGL(mse_kernel<T>, dim3(p.B, p.nch), dim3(256), 0, s, p);
  hipLaunchKernelGGL(minmax_part_kernel<T>, dim3(MMCH, p.B), dim3(256), 0, s, p);
  hipLaunchKernelGGL(minmax_count_kernel<T>, dim3(MMCH, p.B), dim3(256), 0, s, p);
  hipLaunchKernelGGL(ssim_map_kernel<T>, dim3(p.nblk_pix, p.B), dim3(256), 0, s, p);
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, s, p);
  const unsigned nq = (unsigned)(((long)p.Tm * p.NM + 255) / 256);
  hipLaunchKernelGGL(ssim_grad_kernel<T>, dim3((p.Tm + SSIM_TI - 1) / SSIM_TI, p.B), dim3(256),
                     0, s, p);
  hipLaunchKernelGGL(ssim_apply_kernel<T>, dim3(nq, p.B), dim3(256), 0, s, p);
  FS2_CHECK_LAUNCH();
  return 0;
}

void carve(LossP& p, float* ws) {
  const int B = p.B;
  p.npix = (p.Tm - (WIN - 1)) * (p.NM - (WIN - 1));
  p.nblk_pix = (p.Tm - (WIN - 1) + SSIM_TI - 1) / SSIM_TI;   // ssim_map blocks per utterance
  p.nch = (p.Tm * p.NM + LOSS_CHUNK - 1) / LOSS_CHUNK;
  float* w = ws;
  p.per_b = w; w += 5L * B;
  p.part_mel = w; w += 2L * B * p.nch;
  p.stats = w; w += 8L * B;
  p.mm_part = w; w += 4L * B * MMCH;
  p.cnt_part = w; w += 2L * B * MMCH;
  p.scal = w; w += 4;
  p.ssim_part = w; w += (long)B * p.nblk_pix;
  w = (float*)(((uintptr_t)w + 15) & ~(uintptr_t)15);
  p.dmap = w; w += 3L * B * p.npix;
  p.dnmap = w;
}

}  // namespace

extern "C" int64_t fs2_loss_workspace_floats(int B, int Tm, int NM) {
  const long npix = (long)(Tm - (WIN - 1)) * (NM - (WIN - 1));
  const long nblk = (Tm - (WIN - 1) + SSIM_TI - 1) / SSIM_TI;
  const long nch = ((long)Tm * NM + LOSS_CHUNK - 1) / LOSS_CHUNK;
  return 5L * B + 2L * B * nch + 8L * B + 6L * B * MMCH + 4 + B * nblk + 4 + 3L * B * npix +
         (long)B * Tm * NM;
}

extern "C" int fs2_loss_fwd_bwd(const fs2_loss_desc* d, void* stream) {
  if (!d) return FS2_EINVAL;
  if (d->B <= 0) return 0;
  if (d->Tm < WIN || d->NM < WIN) return FS2_EINVAL;  // SSIM: kernel larger than input
  if (d->NM > SSIM_MAXW) return FS2_EINVAL;           // SSIM LDS tiles
  if (!d->mel_out || !d->postnet_out || !d->log_dur || !d->pitch_pred || !d->energy_pred ||
      !d->mel_tgt || !d->dur_tgt || !d->pitch_avg || !d->energy_avg || !d->mel_len ||
      !d->phon_len || !d->loss_out || !d->d_mel_out || !d->d_postnet_out || !d->d_log_dur ||
      !d->d_pitch || !d->d_energy || !d->workspace)
    return FS2_EINVAL;
  LossP p{};
  p.B = d->B; p.Tm = d->Tm; p.Tp = d->Tp; p.NM = d->NM;
  p.mel_out = d->mel_out; p.post_out = d->postnet_out; p.log_dur = d->log_dur;
  p.pitch_pred = d->pitch_pred; p.energy_pred = d->energy_pred; p.mel_tgt = d->mel_tgt;
  p.dur_tgt = d->dur_tgt; p.pitch_avg = d->pitch_avg; p.energy_avg = d->energy_avg;
  p.mel_len = d->mel_len; p.phon_len = d->phon_len;
  p.w_ssim = d->w_ssim; p.w_mel = d->w_mel; p.w_post = d->w_post; p.w_dur = d->w_dur;
  p.w_pitch = d->w_pitch; p.w_energy = d->w_energy;
  p.loss_out = d->loss_out; p.d_mel = d->d_mel_out; p.d_post = d->d_postnet_out;
  p.d_dur = d->d_log_dur; p.d_pitch = d->d_pitch; p.d_energy = d->d_energy;
  carve(p, d->workspace);
  {
    const auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    p.vec = al(p.mel_out) && al(p.post_out) && al(p.mel_tgt) && al(p.d_mel) && al(p.d_post);
  }
  hipStream_t s = (hipStream_t)stream;
  if (d->dtype == FS2_BF16) return run_loss<bf16>(p, s);
  if (d->dtype == FS2_F32) return run_loss<float>(p, s);
  return FS2_EINVAL;
}
