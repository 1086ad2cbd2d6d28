#include <cstdlib>
#include <algorithm>
// LayerNorm forward/backward with fused residual-add, dropout, tanh, row-mask, post-add,
// plus column-sum reductions for bias / gamma / beta gradients.
//
// Replaces: SB LayerNorm (eps 1e-6) inside TransformerEncoderLayer "add & norm"
// (src = norm1(src + dropout1(att))), the encoder/decoder final norm
// (App. A.3), DurationPredictor ln1/ln2 (eps 1e-5, App. A.7) and PostNet ln1..ln3 with
// tanh/dropout (App. A.8); K5/K8/K13 of SURVEY.md section 2.
//
// One 64-lane wave per row; statistics in fp32 with a two-pass (mean, then centred
// variance) over the row held in registers, matching torch's LayerNorm numerics.
#include "fs2_common.h"

namespace {

constexpr int MAXJ = 16;  // D <= 1024

template <bool DPP>
__device__ __forceinline__ float wsum(float v) {
  if constexpr (DPP) return wave_sum_dpp(v);
  else return wave_sum(v);
}

struct LnFwdP {
  const char* x; long ldx; const char* r; long ldr; float p_r; uint32_t salt_r;
  char* s_out; const float* gamma; const float* beta; float eps; int do_tanh;
  float p_o; uint32_t salt_o; const float* row_mask; const char* post_add; long ldp;
  char* y; long ldy; float* mean; float* rstd; int M, D; uint32_t seed;
  // optional reflect-padded token-major copy of y (the bf16 rows kernels; fs2_pad_rows layout,
  // row pitch D): token (b, t) at image row b*(T+2P) + P + t, and mirrored into the pad rows
  char* img; int img_t, img_p;
};

template <typename T>
__global__ void __launch_bounds__(256) ln_fwd_kernel(LnFwdP p) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.M) return;
  const T* x = (const T*)p.x + (long)row * p.ldx;
  const T* r = p.r ? (const T*)p.r + (long)row * p.ldr : nullptr;
  const float inv_r = p.p_r > 0.f ? 1.f / (1.f - p.p_r) : 1.f;
  float v[MAXJ];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int d = lane + 64 * j;
    float a = 0.f;
    if (d < p.D) {
      a = to_f(x[d]);
      if (r) {
        float rv = to_f(r[d]);
        if (p.p_r > 0.f)
          rv = fs2_keep(p.seed, p.salt_r, (uint64_t)row * p.D + d, p.p_r) ? rv * inv_r : 0.f;
        a += rv;
      }
      if (p.s_out) ((T*)p.s_out)[(long)row * p.D + d] = from_f<T>(a);
      if (r && p.s_out) a = to_f(((T*)p.s_out)[(long)row * p.D + d]);  // stats of the stored s
      sum += a;
    }
    v[j] = a;
  }
  const float mean = wave_sum(sum) / (float)p.D;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int d = lane + 64 * j;
    if (d < p.D) { const float c = v[j] - mean; sq += c * c; }
  }
  const float var = wave_sum(sq) / (float)p.D;
  const float rstd = 1.f / sqrtf(var + p.eps);
  if (lane == 0) { p.mean[row] = mean; p.rstd[row] = rstd; }
  const float inv_o = p.p_o > 0.f ? 1.f / (1.f - p.p_o) : 1.f;
  const float rm = p.row_mask ? p.row_mask[row] : 1.f;
  T* y = (T*)p.y + (long)row * p.ldy;
  const T* pa = p.post_add ? (const T*)p.post_add + (long)row * p.ldp : nullptr;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int d = lane + 64 * j;
    if (d < p.D) {
      float o = (v[j] - mean) * rstd * p.gamma[d] + p.beta[d];
      if (p.do_tanh) o = tanhf(o);
      if (p.p_o > 0.f)
        o = fs2_keep(p.seed, p.salt_o, (uint64_t)row * p.D + d, p.p_o) ? o * inv_o : 0.f;
      o *= rm;
      if (pa) o += to_f(pa[d]);
      y[d] = from_f<T>(o);
    }
  }
}

// bf16, D <= 512 (one 16-byte chunk per lane): R rows per wave (rows w, w + 4, ... of the
// block's 4R), every row's x / r / post-add loaded before the first row is reduced.  One row
// per wave kept ~1.5 KB in flight per wave -- 48 KB per CU at full occupancy -- and ran the
// decoder LayerNorm (96 MB) at 3.6 TB/s.  Per-row arithmetic, dropout indices and rounding
// points are those of ln_fwd_vec_kernel<bf16, 1> (outputs bit-identical).
template <int R, bool DPP>
__global__ void __launch_bounds__(256) ln_fwd_rows_kernel(LnFwdP p) {
  constexpr int V = 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int d0 = lane * V;
  const bool act = d0 < p.D;
  const int dd = act ? d0 : 0;
  const float inv_r = p.p_r > 0.f ? 1.f / (1.f - p.p_r) : 1.f;
  const float inv_o = p.p_o > 0.f ? 1.f / (1.f - p.p_o) : 1.f;
  float g[V], b[V];
  vload<float>(g, p.gamma + dd);
  vload<float>(g + 4, p.gamma + dd + 4);
  vload<float>(b, p.beta + dd);
  vload<float>(b + 4, p.beta + dd + 4);
  float v[R][V], rv[R][V], a[R][V], rm[R];
  int rows[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    rows[j] = blockIdx.x * (4 * R) + 4 * j + wave;
    const int rr = min(rows[j], p.M - 1);
    vload<bf16>(v[j], (const bf16*)p.x + (long)rr * p.ldx + dd);
    if (p.r) vload<bf16>(rv[j], (const bf16*)p.r + (long)rr * p.ldr + dd);
    if (p.post_add) vload<bf16>(a[j], (const bf16*)p.post_add + (long)rr * p.ldp + dd);
    rm[j] = p.row_mask ? p.row_mask[rr] : 1.f;
  }
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int row = rows[j];
    if (row >= p.M) break;
    float sum = 0.f;
    if (act) {
      if (p.r) {
        bool kr[V];
        if (p.p_r > 0.f) fs2_keep_run<V>(p.seed, p.salt_r, (uint64_t)row * p.D + d0, p.p_r, kr);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          float q = rv[j][e];
          if (p.p_r > 0.f) q = kr[e] ? q * inv_r : 0.f;
          v[j][e] += q;
        }
      }
      if (p.s_out) {
        vstore<bf16>((bf16*)p.s_out + (long)row * p.D + d0, v[j]);
        if (p.r) {  // statistics of the stored (rounded) s, as the backward re-reads it
#pragma unroll
          for (int e = 0; e < V; ++e) v[j][e] = to_f(from_f<bf16>(v[j][e]));
        }
      }
#pragma unroll
      for (int e = 0; e < V; ++e) sum += v[j][e];
    }
    const float mean = wsum<DPP>(sum) / (float)p.D;
    float sq = 0.f;
    if (act) {
#pragma unroll
      for (int e = 0; e < V; ++e) { const float c = v[j][e] - mean; sq += c * c; }
    }
    const float var = wsum<DPP>(sq) / (float)p.D;
    const float rstd = 1.f / sqrtf(var + p.eps);
    if (lane == 0) { p.mean[row] = mean; p.rstd[row] = rstd; }
    if (act) {
      float o[V];
      bool ko[V];
      if (p.p_o > 0.f) fs2_keep_run<V>(p.seed, p.salt_o, (uint64_t)row * p.D + d0, p.p_o, ko);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        float q = (v[j][e] - mean) * rstd * g[e] + b[e];
        if (p.do_tanh) q = tanhf(q);
        if (p.p_o > 0.f) q = ko[e] ? q * inv_o : 0.f;
        q *= rm[j];
        if (p.post_add) q += a[j][e];
        o[e] = q;
      }
      vstore<bf16>((bf16*)p.y + (long)row * p.ldy + d0, o);
      if (p.img) {   // padded index i holds token reflect(i - P): i = P + t, P - t, P + 2(T-1) - t
        const int T = p.img_t, P = p.img_p, b = row / T, t = row - b * T;
        bf16* ib = (bf16*)p.img + (long)b * (T + 2 * P) * p.D + d0;
        vstore<bf16>(ib + (long)(P + t) * p.D, o);
        if (t >= 1 && t <= P) vstore<bf16>(ib + (long)(P - t) * p.D, o);
        if (t >= T - 1 - P && t <= T - 2) vstore<bf16>(ib + (long)(P + 2 * (T - 1) - t) * p.D, o);
      }
    }
  }
}

// the bf16 rows kernels' row sums through DPP (wave_sum_dpp; FS2_LN_DPP=0: __shfl_xor)
int ln_dpp() {
  static const int r = fs2_exp_int("FS2_LN_DPP", 1);
  return r;
}
// rows per wave of the bf16 LayerNorm forward (FS2_LN_FWD_ROWS: 1 = ln_fwd_vec_kernel)
int ln_fwd_rows() {
  static const int r = fs2_exp_int("FS2_LN_FWD_ROWS", 2);
  return r;
}

// tanh for the bf16 backward's (1 - t^2) gate: exp-based, absolute error ~1e-7 (the gate's
// error is 2|t| times that, far below the bf16 gradient it scales); tanhf's branchy
// polynomial costs ~3x the instructions.  The forward keeps tanhf (its result is the layer's
// output), and so do the fp32 kernels.  do_tanh == 2 (FS2_LN_TANH_EXACT, experiments build)
// keeps tanhf in the bf16 backward too.
__device__ __forceinline__ float tanh_gate(float x) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * x) + 1.f);
}

struct LnBwdP {
  const char* dy; long lddy; const char* s; long lds; const float* mean; const float* rstd;
  const float* gamma; const float* beta; int do_tanh; float p_o; uint32_t salt_o;
  const float* row_mask; int relu_gate_in; char* ds; long ldds; char* dr; float p_r;
  uint32_t salt_r; float* part_g; float* part_b; int M, D; uint32_t seed; int rows_per_block;
  float* part_c; long pstride;  // partial rows are pstride floats apart (scalar kernel)
};

template <typename T>
__global__ void __launch_bounds__(256) ln_bwd_kernel(LnBwdP p) {
  __shared__ float red[2][4][1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pg[MAXJ], pb[MAXJ], pc[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) { pg[j] = 0.f; pb[j] = 0.f; pc[j] = 0.f; }
  const float inv_o = p.p_o > 0.f ? 1.f / (1.f - p.p_o) : 1.f;
  const float inv_r = p.p_r > 0.f ? 1.f / (1.f - p.p_r) : 1.f;
  const int rbeg = blockIdx.x * p.rows_per_block;
  const int rend = min(p.M, rbeg + p.rows_per_block);
  for (int row = rbeg + wave; row < rend; row += 4) {
    const T* dy = (const T*)p.dy + (long)row * p.lddy;
    const T* s = (const T*)p.s + (long)row * p.lds;
    const float mean = p.mean[row], rstd = p.rstd[row];
    const float rm = p.row_mask ? p.row_mask[row] : 1.f;
    float g[MAXJ], xh[MAXJ], sv[MAXJ];
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int d = lane + 64 * j;
      g[j] = 0.f; xh[j] = 0.f; sv[j] = 0.f;
      if (d < p.D) {
        sv[j] = to_f(s[d]);
        xh[j] = (sv[j] - mean) * rstd;
        float gg = to_f(dy[d]) * rm;
        if (p.p_o > 0.f)
          gg = fs2_keep(p.seed, p.salt_o, (uint64_t)row * p.D + d, p.p_o) ? gg * inv_o : 0.f;
        if (p.do_tanh) {
          const float t = tanhf(xh[j] * p.gamma[d] + p.beta[d]);
          gg *= (1.f - t * t);
        }
        pg[j] += gg * xh[j];
        pb[j] += gg;
        g[j] = gg * p.gamma[d];
        a1 += g[j];
        a2 += g[j] * xh[j];
      }
    }
    a1 = wave_sum(a1) / (float)p.D;
    a2 = wave_sum(a2) / (float)p.D;
    T* ds = (T*)p.ds + (long)row * p.ldds;
    T* dr = p.dr ? (T*)p.dr + (long)row * p.D : nullptr;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int d = lane + 64 * j;
      if (d < p.D) {
        float v = rstd * (g[j] - a1 - xh[j] * a2);
        if (p.relu_gate_in && !(sv[j] > 0.f)) v = 0.f;
        ds[d] = from_f<T>(v);
        if (dr) {
          float w = v;
          if (p.p_r > 0.f)
            w = fs2_keep(p.seed, p.salt_r, (uint64_t)row * p.D + d, p.p_r) ? w * inv_r : 0.f;
          dr[d] = from_f<T>(w);
          pc[j] += w;
        } else {
          pc[j] += v;
        }
      }
    }
  }
  if (p.part_g) {
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int d = lane + 64 * j;
      if (d < p.D) { red[0][wave][d] = pg[j]; red[1][wave][d] = pb[j]; }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < p.D; d += 256) {
      p.part_g[(long)blockIdx.x * p.pstride + d] = (red[0][0][d] + red[0][1][d]) + (red[0][2][d] + red[0][3][d]);
      p.part_b[(long)blockIdx.x * p.pstride + d] = (red[1][0][d] + red[1][1][d]) + (red[1][2][d] + red[1][3][d]);
    }
  }
  if (p.part_c) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int d = lane + 64 * j;
      if (d < p.D) red[0][wave][d] = pc[j];
    }
    __syncthreads();
    for (int d = threadIdx.x; d < p.D; d += 256)
      p.part_c[(long)blockIdx.x * p.pstride + d] = (red[0][0][d] + red[0][1][d]) + (red[0][2][d] + red[0][3][d]);
  }
}

template <typename T>
__global__ void colsum_partial_kernel(const T* X, long ldx, int M, int N, int rows_per_block,
                                      float* part) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int rbeg = blockIdx.y * rows_per_block;
  const int rend = min(M, rbeg + rows_per_block);
  float s = 0.f;
  for (int m = rbeg; m < rend; ++m) s += to_f(X[(long)m * ldx + n]);
  part[(long)blockIdx.y * N + n] = s;
}


// ---- 16-byte vectorised variants (D % VEC == 0, 16-B aligned rows): lane owns NCH chunks of
// VEC consecutive features, so a D=384 bf16 row is one 768-B wave access instead of six
// 128-B ones.  Same arithmetic, dropout indices and rounding points as the scalar kernels.
template <typename T, int NCH>
__global__ void __launch_bounds__(256) ln_fwd_vec_kernel(LnFwdP p) {
  constexpr int V = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.M) return;
  const T* x = (const T*)p.x + (long)row * p.ldx;
  const T* r = p.r ? (const T*)p.r + (long)row * p.ldr : nullptr;
  const float inv_r = p.p_r > 0.f ? 1.f / (1.f - p.p_r) : 1.f;
  float v[NCH][V];
  float sum = 0.f;
  // the epilogue operands are loaded up front, so their latency overlaps the two row sums
  float g[NCH][V], b[NCH][V], a[NCH][V];
  const T* pa = p.post_add ? (const T*)p.post_add + (long)row * p.ldp : nullptr;
  const float rm = p.row_mask ? p.row_mask[row] : 1.f;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int d0 = (lane + 64 * ch) * V;
    if (d0 < p.D) {
      vload<float>(g[ch], p.gamma + d0);
      vload<float>(b[ch], p.beta + d0);
      if constexpr (V == 8) { vload<float>(g[ch] + 4, p.gamma + d0 + 4); vload<float>(b[ch] + 4, p.beta + d0 + 4); }
      if (pa) vload<T>(a[ch], pa + d0);
    }
  }
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int d0 = (lane + 64 * ch) * V;
    if (d0 < p.D) {
      vload<T>(v[ch], x + d0);
      if (r) {
        float rv[V];
        vload<T>(rv, r + d0);
        bool kr[V];
        if (p.p_r > 0.f) fs2_keep_run<V>(p.seed, p.salt_r, (uint64_t)row * p.D + d0, p.p_r, kr);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          float q = rv[e];
          if (p.p_r > 0.f) q = kr[e] ? q * inv_r : 0.f;
          v[ch][e] += q;
        }
      }
      if (p.s_out) {
        vstore<T>((T*)p.s_out + (long)row * p.D + d0, v[ch]);
        if (r) {  // statistics of the stored (rounded) s, as the backward re-reads it
#pragma unroll
          for (int e = 0; e < V; ++e) v[ch][e] = to_f(from_f<T>(v[ch][e]));
        }
      }
#pragma unroll
      for (int e = 0; e < V; ++e) sum += v[ch][e];
    }
  }
  const float mean = wave_sum(sum) / (float)p.D;
  float sq = 0.f;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int d0 = (lane + 64 * ch) * V;
    if (d0 < p.D) {
#pragma unroll
      for (int e = 0; e < V; ++e) { const float c = v[ch][e] - mean; sq += c * c; }
    }
  }
  const float var = wave_sum(sq) / (float)p.D;
  const float rstd = 1.f / sqrtf(var + p.eps);
  if (lane == 0) { p.mean[row] = mean; p.rstd[row] = rstd; }
  const float inv_o = p.p_o > 0.f ? 1.f / (1.f - p.p_o) : 1.f;
  T* y = (T*)p.y + (long)row * p.ldy;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int d0 = (lane + 64 * ch) * V;
    if (d0 < p.D) {
      float o[V];
      bool ko[V];
      if (p.p_o > 0.f) fs2_keep_run<V>(p.seed, p.salt_o, (uint64_t)row * p.D + d0, p.p_o, ko);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        float q = (v[ch][e] - mean) * rstd * g[ch][e] + b[ch][e];
        if (p.do_tanh) q = tanhf(q);
        if (p.p_o > 0.f) q = ko[e] ? q * inv_o : 0.f;
        q *= rm;
        if (pa) q += a[ch][e];
        o[e] = q;
      }
      vstore<T>(y + d0, o);
    }
  }
}

// part layout: [gridDim.x][npart * D] (gamma, beta, then optionally the column sum of the
// emitted gradient -- the bias gradient of the layer that produced the residual branch)
template <typename T, int NCH>
__global__ void __launch_bounds__(256) ln_bwd_vec_kernel(LnBwdP p, float* part, int npart,
                                                         int kind0) {
  constexpr int V = Vec<T>::N;
  __shared__ float red[4][1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pg[NCH][V], pb[NCH][V], pc[NCH][V];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
    for (int e = 0; e < V; ++e) { pg[ch][e] = 0.f; pb[ch][e] = 0.f; pc[ch][e] = 0.f; }
  const float inv_o = p.p_o > 0.f ? 1.f / (1.f - p.p_o) : 1.f;
  const float inv_r = p.p_r > 0.f ? 1.f / (1.f - p.p_r) : 1.f;
  const int rbeg = blockIdx.x * p.rows_per_block;
  const int rend = min(p.M, rbeg + p.rows_per_block);
  for (int row = rbeg + wave; row < rend; row += 4) {
    const T* dy = (const T*)p.dy + (long)row * p.lddy;
    const T* s = (const T*)p.s + (long)row * p.lds;
    const float mean = p.mean[row], rstd = p.rstd[row];
    const float rm = p.row_mask ? p.row_mask[row] : 1.f;
    float g[NCH][V], xh[NCH][V], sv[NCH][V];
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int d0 = (lane + 64 * ch) * V;
      if (d0 < p.D) {
        float dv[V], gm[V], bt[V];
        vload<T>(sv[ch], s + d0);
        vload<T>(dv, dy + d0);
        vload<float>(gm, p.gamma + d0);
        if constexpr (V == 8) vload<float>(gm + 4, p.gamma + d0 + 4);
        if (p.do_tanh) {
          vload<float>(bt, p.beta + d0);
          if constexpr (V == 8) vload<float>(bt + 4, p.beta + d0 + 4);
        }
        bool ko[V];
        if (p.p_o > 0.f) fs2_keep_run<V>(p.seed, p.salt_o, (uint64_t)row * p.D + d0, p.p_o, ko);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          xh[ch][e] = (sv[ch][e] - mean) * rstd;
          float gg = dv[e] * rm;
          if (p.p_o > 0.f) gg = ko[e] ? gg * inv_o : 0.f;
          if (p.do_tanh) {
            const float z = xh[ch][e] * gm[e] + bt[e];
            const float t = (sizeof(T) == 2 && p.do_tanh == 1) ? tanh_gate(z) : tanhf(z);
            gg *= (1.f - t * t);
          }
          pg[ch][e] += gg * xh[ch][e];
          pb[ch][e] += gg;
          g[ch][e] = gg * gm[e];
          a1 += g[ch][e];
          a2 += g[ch][e] * xh[ch][e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e) { g[ch][e] = 0.f; xh[ch][e] = 0.f; sv[ch][e] = 0.f; }
      }
    }
    a1 = wave_sum(a1) / (float)p.D;
    a2 = wave_sum(a2) / (float)p.D;
    T* ds = (T*)p.ds + (long)row * p.ldds;
    T* dr = p.dr ? (T*)p.dr + (long)row * p.D : nullptr;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int d0 = (lane + 64 * ch) * V;
      if (d0 < p.D) {
        float o[V], w[V];
        bool kr[V];
        if (dr && p.p_r > 0.f) fs2_keep_run<V>(p.seed, p.salt_r, (uint64_t)row * p.D + d0, p.p_r, kr);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          float q = rstd * (g[ch][e] - a1 - xh[ch][e] * a2);
          if (p.relu_gate_in && !(sv[ch][e] > 0.f)) q = 0.f;
          o[e] = q;
          if (dr) {
            float t = q;
            if (p.p_r > 0.f) t = kr[e] ? t * inv_r : 0.f;
            w[e] = t;
          }
        }
        vstore<T>(ds + d0, o);
        if (dr) vstore<T>(dr + d0, w);
#pragma unroll
        for (int e = 0; e < V; ++e) pc[ch][e] += dr ? w[e] : o[e];
      }
    }
  }
  if (!part) return;
  // fixed-order combine of the 4 waves' partials, one pass per partial kind
  for (int k = 0; k < npart; ++k) {
    const int kind = kind0 + k;  // 0 gamma, 1 beta, 2 column sum
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int d0 = (lane + 64 * ch) * V;
      if (d0 < p.D) {
#pragma unroll
        for (int e = 0; e < V; ++e)
          red[wave][d0 + e] = kind == 0 ? pg[ch][e] : (kind == 1 ? pb[ch][e] : pc[ch][e]);
      }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < p.D; d += 256)
      part[((long)blockIdx.x * npart + k) * p.D + d] =
          (red[0][d] + red[1][d]) + (red[2][d] + red[3][d]);
    __syncthreads();
  }
}

// bf16, D <= 512 (one 16-byte chunk per lane): the same per-row arithmetic and the same
// per-wave accumulation order as ln_bwd_vec_kernel<bf16, 1> (so identical results), but each
// wave loads R rows (r, r+4, ..., r+4(R-1)) before computing any of them.  The one-row loop
// keeps ~1.5 KB per wave in flight and ran at 1-2 TB/s (latency bound: 15 waves per CU).  The
// tanh-gated case (PostNet) uses R = 2 (ln_tanh_rows).
template <int R, bool TANH, bool DPP>
__global__ void __launch_bounds__(256) ln_bwd_rows_kernel(LnBwdP p, float* part, int npart,
                                                          int kind0) {
  constexpr int V = 8;
  __shared__ float red[3][4][512];   // [kind][wave][column]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int d0 = lane * V;
  const bool act = d0 < p.D;
  float pg[V], pb[V], pc[V], gm[V], bt[V];
#pragma unroll
  for (int e = 0; e < V; ++e) { pg[e] = 0.f; pb[e] = 0.f; pc[e] = 0.f; gm[e] = 0.f; bt[e] = 0.f; }
  if (act) {
    vload<float>(gm, p.gamma + d0);
    vload<float>(gm + 4, p.gamma + d0 + 4);
    if constexpr (TANH) { vload<float>(bt, p.beta + d0); vload<float>(bt + 4, p.beta + d0 + 4); }
    
  }
  const float inv_o = p.p_o > 0.f ? 1.f / (1.f - p.p_o) : 1.f;
  const float inv_r = p.p_r > 0.f ? 1.f / (1.f - p.p_r) : 1.f;
  const uint32_t key_o = fs2_drop_key(p.seed, p.salt_o), key_r = fs2_drop_key(p.seed, p.salt_r);
  const uint32_t thr_o = fs2_thr16(p.p_o), thr_r = fs2_thr16(p.p_r);
  const int rbeg = blockIdx.x * p.rows_per_block;
  const int rend = min(p.M, rbeg + p.rows_per_block);
  for (int row0 = rbeg + wave; row0 < rend; row0 += 4 * R) {
    u32x4 us[R], ud[R];
    float mean[R], rstd[R], rm[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int row = row0 + 4 * j;
      const bool ok = row < rend;
      const int rr = ok ? row : row0;
      us[j] = act ? *(const u32x4*)((const bf16*)p.s + (long)rr * p.lds + d0) : u32x4{0, 0, 0, 0};
      ud[j] = act ? *(const u32x4*)((const bf16*)p.dy + (long)rr * p.lddy + d0) : u32x4{0, 0, 0, 0};
      mean[j] = p.mean[rr];
      rstd[j] = p.rstd[rr];
      rm[j] = p.row_mask ? p.row_mask[rr] : 1.f;
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int row = row0 + 4 * j;
      if (row >= rend) break;
      float sv[V], g[V], xh[V];
      float a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        sv[2 * w] = __builtin_bit_cast(float, us[j][w] << 16);
        sv[2 * w + 1] = __builtin_bit_cast(float, us[j][w] & 0xffff0000u);
      }
      // element (row, d0 + e): pairs (e, e + 1) share one hash (row * D + d0 is even)
      const uint64_t ib = (uint64_t)row * p.D + d0;
      uint32_t ho[V / 2], hr[V / 2];
#pragma unroll
      for (int e = 0; e < V / 2; ++e) {
        ho[e] = p.p_o > 0.f ? fs2_hash_pair(key_o, (ib >> 1) + e) : 0u;
        hr[e] = (p.dr && p.p_r > 0.f) ? fs2_hash_pair(key_r, (ib >> 1) + e) : 0u;
      }
      if (act) {
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const float dv = __builtin_bit_cast(float, (e & 1) ? (ud[j][e >> 1] & 0xffff0000u)
                                                             : (ud[j][e >> 1] << 16));
          xh[e] = (sv[e] - mean[j]) * rstd[j];
          float gg = dv * rm[j];
          if (p.p_o > 0.f) gg = fs2_keep_pair_bit(ho[e >> 1], ib + e, thr_o) ? gg * inv_o : 0.f;
          if constexpr (TANH) {
            const float z = xh[e] * gm[e] + bt[e];
            const float t = p.do_tanh == 1 ? tanh_gate(z) : tanhf(z);
            gg *= (1.f - t * t);
          }
          pg[e] += gg * xh[e];
          pb[e] += gg;
          g[e] = gg * gm[e];
          a1 += g[e];
          a2 += g[e] * xh[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < V; ++e) { g[e] = 0.f; xh[e] = 0.f; }
      }
      a1 = wsum<DPP>(a1) / (float)p.D;
      a2 = wsum<DPP>(a2) / (float)p.D;
      if (act) {
        float o[V], w[V];
#pragma unroll
        for (int e = 0; e < V; ++e) {
          float q = rstd[j] * (g[e] - a1 - xh[e] * a2);
          if (p.relu_gate_in && !(sv[e] > 0.f)) q = 0.f;
          o[e] = q;
          w[e] = q;
          if (p.dr && p.p_r > 0.f) w[e] = fs2_keep_pair_bit(hr[e >> 1], ib + e, thr_r) ? q * inv_r : 0.f;
        }
        vstore<bf16>((bf16*)p.ds + (long)row * p.ldds + d0, o);
        if (p.dr) vstore<bf16>((bf16*)p.dr + (long)row * p.D + d0, w);
#pragma unroll
        for (int e = 0; e < V; ++e) pc[e] += p.dr ? w[e] : o[e];
      }
    }
  }
  if (!part) return;
  // every kind's wave partials into LDS, ONE barrier, then the block's npart partial rows in
  // one contiguous pass (the same fixed-order sums as one barrier pair per kind)
  if (act) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k < npart) {
        const int kind = kind0 + k;  // 0 gamma, 1 beta, 2 column sum
#pragma unroll
        for (int e = 0; e < V; ++e)
          red[k][wave][d0 + e] = kind == 0 ? pg[e] : (kind == 1 ? pb[e] : pc[e]);
      }
    }
  }
  __syncthreads();
  float* prow = part + (long)blockIdx.x * npart * p.D;
  for (int i = threadIdx.x; i < npart * p.D; i += 256) {
    const int k = i / p.D, d = i - k * p.D;
    prow[i] = (red[k][0][d] + red[k][1][d]) + (red[k][2][d] + red[k][3][d]);
  }
}

// out_k[d] (+)= sum_b part[b][k*D + d] for k < npart: 16 columns x SL row-slices per block
// (16 SL threads), fixed-order combine through LDS (deterministic).  With 16 row-slices each
// thread walked ~61 partial rows of a decoder LayerNorm backward in sequence: 7.6 us per call,
// 62 calls per step.
template <int SL>
__global__ void __launch_bounds__(SL * 16) reduce_parts_kernel(const float* part, int nb, int D,
                                                              int npart, float* o0, float* o1,
                                                              float* o2, int accumulate) {
  __shared__ float red[SL][17];
  const int c = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int ncols = npart * D;
  const int n = blockIdx.x * 16 + c;
  float s = 0.f;
  if (n < ncols) {
#pragma unroll 4
    for (int b = sl; b < nb; b += SL) s += part[(long)b * ncols + n];
  }
  red[sl][c] = s;
  __syncthreads();
  for (int w = SL / 2; w >= 1; w >>= 1) {   // pairwise tree, fixed order
    if (sl < w) red[sl][c] += red[sl + w][c];
    __syncthreads();
  }
  if (sl == 0 && n < ncols) {
    const float t = red[0][c];
    const int k = n / D, d = n - k * D;
    float* o = k == 0 ? o0 : (k == 1 ? o1 : o2);
    o[d] = accumulate ? o[d] + t : t;
  }
}

// 16 row-slices (256 threads): a block that fits beside the side stream's GEMM blocks on a
// busy CU, each thread walking 4x the rows of the 1024-thread form, whose blocks waited for a
// whole free CU (21-27 us per call in the step against 4 standalone).  Step 17.25 -> 17.14 ms
// (3 x 3 interleaved; 64 threads: 17.36).  FS2_RP_SL=64 (experiments build): the 1024-thread form.
void launch_reduce_parts(hipStream_t st, const float* part, int nb, int D, int npart, float* o0,
                         float* o1, float* o2, int accumulate) {
  static const int sl = fs2_exp_int("FS2_RP_SL", 16);
  const dim3 g((npart * D + 15) / 16);
  if (sl == 16)
    hipLaunchKernelGGL(reduce_parts_kernel<16>, g, dim3(256), 0, st, part, nb, D, npart, o0, o1,
                       o2, accumulate);
  else
    hipLaunchKernelGGL(reduce_parts_kernel<64>, g, dim3(1024), 0, st, part, nb, D, npart, o0, o1,
                       o2, accumulate);
}

// column sums, 16-B loads: thread = (row sub-lane, column chunk of VEC)
template <typename T>
__global__ void __launch_bounds__(256) colsum_vec_kernel(const T* X, long ldx, int M, int N,
                                                        int rows_per_block, float* part) {
  constexpr int V = Vec<T>::N;
  __shared__ float red[256 * V];
  const int ncc = N / V, nsub = 256 / ncc;
  const int t = threadIdx.x, rsub = t / ncc, cc = t - rsub * ncc;
  const int rbeg = blockIdx.x * rows_per_block;
  const int rend = min(M, rbeg + rows_per_block);
  float acc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = 0.f;
  if (rsub < nsub) {
    int m = rbeg + rsub;
    for (; m + 3 * nsub < rend; m += 4 * nsub) {
      float a[4][V];
#pragma unroll
      for (int u = 0; u < 4; ++u) vload<T>(a[u], X + (long)(m + u * nsub) * ldx + cc * V);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += a[u][e];
    }
    for (; m < rend; m += nsub) {
      float a[V];
      vload<T>(a, X + (long)m * ldx + cc * V);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] += a[e];
    }
#pragma unroll
    for (int e = 0; e < V; ++e) red[rsub * N + cc * V + e] = acc[e];
  }
  __syncthreads();
  for (int n = t; n < N; n += 256) {
    float s = 0.f;
    for (int i = 0; i < nsub; ++i) s += red[i * N + n];
    part[(long)blockIdx.x * N + n] = s;
  }
}

// column sums for wide rows (N / VEC >= 32 chunks): block (row range, 64-chunk column slab),
// wave w walks rows w, w + 4, ... with U 16-byte loads in flight; colsum_vec_kernel gave a
// 1152-wide bf16 row (the QKV bias gradient) one sub-row per block, 144 of 256 threads each
// walking all 64 rows 4 loads at a time (111 us for 72 MB in the step)
template <typename T, int U>
__global__ void __launch_bounds__(256) colsum_slab_kernel(const T* X, long ldx, int M, int N,
                                                         int rows_per_block, float* part) {
  constexpr int V = Vec<T>::N;
  __shared__ float red[4][64 * V];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cc = blockIdx.y * 64 + lane;
  const bool act = cc * V < N;
  const int rbeg = blockIdx.x * rows_per_block;
  const int rend = min(M, rbeg + rows_per_block);
  float acc[V];
#pragma unroll
  for (int e = 0; e < V; ++e) acc[e] = 0.f;
  if (act) {
    const T* x = X + (long)cc * V;
    int m = rbeg + w;
    for (; m + 4 * (U - 1) < rend; m += 4 * U) {
      float a[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) vload<T>(a[u], x + (long)(m + 4 * u) * ldx);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += a[u][e];
    }
    for (; m < rend; m += 4) {
      float a[V];
      vload<T>(a, x + (long)m * ldx);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] += a[e];
    }
  }
#pragma unroll
  for (int e = 0; e < V; ++e) red[w][lane * V + e] = acc[e];
  __syncthreads();
  const int n0 = blockIdx.y * 64 * V;
  for (int i = threadIdx.x; i < 64 * V; i += 256) {
    const int n = n0 + i;
    if (n < N) part[(long)blockIdx.x * N + n] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

// Adjoint of SB Conv1d's reflect "same" padding for the data gradient (K16):
//   dX[b,s] = Xp[b,s+P] + [1<=s<=P] Xp[b,P-s] + [T-1-P<=s<=T-2] Xp[b,2(T-1)-s+P]
// where Xp (fp32, T+2P rows per utterance) is the zero-padded shift-conv GEMM output
// (fs2_gemm conv_mode 4), fused with the dgrad epilogue: out = (dX*rs + residual)*rs2.
//
// bf16 form: one lane per 8 channels of a row, every access 16 bytes wide (two fp32 x4 per
// slice and source row, one bf16 x8 residual load and one bf16 x8 store).  The 4-channel form
// below moved the residual and the output as 2-byte scalars: 87 us for the decoder's
// 31264 x 384 fold, ~1.1 TB/s.  Same per-element arithmetic and summation order.
__global__ void __launch_bounds__(256) conv_fold8_kernel(const float* Xp, int nsplit, long sstride,
                                                         int T_, int P, int C8, bf16* out, long ldo,
                                                         const bf16* res, long ldr, const float* rs,
                                                         const float* rs2, unsigned n8) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const unsigned m = i / (unsigned)C8;
  const int c = (int)(i - m * (unsigned)C8) * 8;
  const int C = C8 * 8;
  const int b = (int)(m / (unsigned)T_), s = (int)(m - (unsigned)b * (unsigned)T_);
  const long rb = (long)b * (T_ + 2 * P);
  const bool lo = s >= 1 && s <= P, hi = s >= T_ - 1 - P && s <= T_ - 2;
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
  for (int z = 0; z < nsplit; ++z) {
    const float* X = Xp + z * sstride;
    const float* x0 = X + (rb + s + P) * C + c;
    a0 += *(const f32x4*)x0;
    a1 += *(const f32x4*)(x0 + 4);
    if (lo) {
      const float* x1 = X + (rb + P - s) * C + c;
      a0 += *(const f32x4*)x1;
      a1 += *(const f32x4*)(x1 + 4);
    }
    if (hi) {
      const float* x2 = X + (rb + 2 * (T_ - 1) - s + P) * C + c;
      a0 += *(const f32x4*)x2;
      a1 += *(const f32x4*)(x2 + 4);
    }
  }
  const float r1 = rs ? rs[m] : 1.f, r2 = rs2 ? rs2[m] : 1.f;
  float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (res) {
    const u32x4 u = *(const u32x4*)(res + (long)m * ldr + c);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      rv[2 * w] = __builtin_bit_cast(float, u[w] << 16);
      rv[2 * w + 1] = __builtin_bit_cast(float, u[w] & 0xffff0000u);
    }
  }
  u32x4 o;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const int e = 2 * w;
    const float v0 = w < 2 ? a0[e] : a1[e - 4], v1 = w < 2 ? a0[e + 1] : a1[e - 3];
    float x0 = v0 * r1, x1 = v1 * r1;
    if (res) { x0 += rv[e]; x1 += rv[e + 1]; }
    const bf16 h0 = (bf16)(x0 * r2), h1 = (bf16)(x1 * r2);
    o[w] = (unsigned)__builtin_bit_cast(unsigned short, h0) |
           ((unsigned)__builtin_bit_cast(unsigned short, h1) << 16);
  }
  *(u32x4*)(out + (long)m * ldo + c) = o;
}

template <typename T>
__global__ void conv_fold_kernel(const float* Xp, int nsplit, long sstride, int T_, int P, int C,
                                 T* out, long ldo, const T* res, long ldr, const float* rs,
                                 const float* rs2, long n) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  const long m = i / C;
  const int c = (int)(i - m * C);
  const int b = (int)(m / T_), s = (int)(m - (long)b * T_);
  const long rb = (long)b * (T_ + 2 * P);
  const bool lo = s >= 1 && s <= P, hi = s >= T_ - 1 - P && s <= T_ - 2;
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  for (int z = 0; z < nsplit; ++z) {
    const float* X = Xp + z * sstride;
    a += *(const f32x4*)(X + (rb + s + P) * C + c);
    if (lo) a += *(const f32x4*)(X + (rb + P - s) * C + c);
    if (hi) a += *(const f32x4*)(X + (rb + 2 * (T_ - 1) - s + P) * C + c);
  }
  const float r1 = rs ? rs[m] : 1.f, r2 = rs2 ? rs2[m] : 1.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float x = a[e] * r1;
    if (res) x += to_f(res[m * ldr + c + e]);
    out[m * ldo + c + e] = from_f<T>(x * r2);
  }
}

// out[i] (+)= sum_s ws[s * stride + i]: split-K weight-gradient slices (fixed order)
__global__ void __launch_bounds__(256) sum_slices_kernel(const float* ws, int ns, long stride,
                                                         long n4, float* out, int accumulate) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  f32x4 a = accumulate ? ((const f32x4*)out)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < ns; ++s) a += *(const f32x4*)(ws + s * stride + i * 4);
  ((f32x4*)out)[i] = a;
}

// rows per LayerNorm-backward block (4 waves at 3 waves per SIMD): enough that the grid's
// waves fit one round of the chip's 3 x 1024 wave slots (the decoder's M = 31264: 41 rows, 763
// blocks -- 32 rows left a second round of 836 waves: 41.6 -> 38.8 us standalone, step 17.20 ->
// 17.13 ms, tools/r06_probe.sh), at least 16 (M = 6400: 16.9 us; 20.0 with 8)
// FS2_LN_RPB forces
int ln_rpb(int M) {
  static const int r = fs2_exp_int("FS2_LN_RPB", 0);
  if (r) return std::max(4, r);
  return std::max(16, (4 * M + 3071) / 3072);
}
int ln_blocks(int M) { return min(8192, max(1, (M + ln_rpb(M) - 1) / ln_rpb(M))); }
// rows in flight per wave in the bf16 LayerNorm backward (FS2_LN_ROWS=1 selects the one-row
// kernel for A/B runs)
// the tanh-gated bf16 LayerNorm backward (PostNet, D = 512) through the R = 2 rows kernel:
// 43.2 us vs 48.7 for the one-row kernel with the same exp-based gate, 57.1 with tanhf
// (tools/r06_ln_tanh.sh, M = 31264); FS2_LN_TANH_ROWS=0 selects the one-row kernel
int ln_tanh_rows() {
  static const int r = fs2_exp_int("FS2_LN_TANH_ROWS", 1);
  return r;
}
int ln_rows_r() {
  static const int r = fs2_exp_int("FS2_LN_ROWS", 4);
  return r;
}
// ---- token-major -> channel-major padded images for the K-major weight gradient (conv_mode 6)
//
// The FFN conv1 weight gradient dW[o][j][c] = sum_{b,t} dH[b,t,o] * X[b, reflect(t+j-P), c]
// (SB Conv1d k=9 "same"+reflect; backward of model.py:241-267) reduces over the
// token axis, which is the ROW axis of both token-major operands.  Read in that layout both
// fragments go through ds_read_b64_tr_b16 (two LDS instructions per MFMA operand instead of
// one ds_read_b128: the 442 us vs 350 us of DESIGN 6.3).  This pass writes the channel-major
// images once per layer so the GEMM reads both operands K-major:
//   out[c][b*(T+2P) + i] = X[b*T + reflect(i-P)][c]          (reflect = 1: the conv input)
//                        = X[b*T + i-P][c] or 0 outside [0,T) (reflect = 0: dH, zero pads)
// for i in [0, T+2P); columns [B*(T+2P), ncols) are zero.  In that padded token domain the tap
// shift of the conv is a constant column offset j - P per GEMM row (conv_mode 6), and the zero
// pad columns of dH cancel every product that would cross an utterance.
constexpr int TJ = 64, TC = 64;     // tile: 64 output columns (tokens) x 64 channels
constexpr int PITCH = 144;          // LDS row pitch in bytes: 64 channels (128 B) + 16

// grid (ceil(ncols / 64), ceil(C / 64)), 256 threads.  Load: thread -> (token row jr, 8-channel
// chunk ch), two passes of 32 rows, one 16-byte load each.  Store: thread -> (channel row cr,
// 8-token chunk jc), two passes of 32 rows, one 16-byte store each.
// part (optional): the block's column sums of X over its 64 tokens (pads contribute zero /
// their reflected copies: only the reflect = 0 image is summed), part[blockIdx.x][c]
__global__ void __launch_bounds__(256) pad_transpose_kernel(const bf16* X, long ldx, int B, int T,
                                                            int C, int P, int reflect, bf16* out,
                                                            long ldo, int ncols, float* part) {
  __shared__ __attribute__((aligned(16))) char tile[TJ * PITCH];
  const int tid = threadIdx.x;
  const int j0 = blockIdx.x * TJ, c0 = blockIdx.y * TC;
  const int Tp = T + 2 * P;
  const long jend = (long)B * Tp;
  {
    const int jr = tid >> 3, ch = tid & 7;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int jl = jr + 32 * pass, j = j0 + jl;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (j < jend && c0 + ch * 8 < C) {
        const int b = j / Tp;
        int t = j - b * Tp - P;
        bool ok = true;
        if (reflect) t = reflect_idx(t, T);
        else ok = t >= 0 && t < T;
        if (ok) v = *(const u32x4*)(X + ((long)b * T + t) * ldx + c0 + ch * 8);
      }
      *(u32x4*)(tile + jl * PITCH + ch * 16) = v;
    }
  }
  __syncthreads();
  {
    const int cr = tid >> 3, jc = tid & 7;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int cl = cr + 32 * pass, c = c0 + cl;
      const int j = j0 + jc * 8;
      const unsigned short* col = (const unsigned short*)(tile + jc * 8 * PITCH) + cl;
      u32x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = (unsigned)col[(2 * e) * (PITCH / 2)] | ((unsigned)col[(2 * e + 1) * (PITCH / 2)] << 16);
      if (part) {   // 8 tokens per lane, then the 8 lanes of the row (fixed order)
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          s += bf16_bits_to_f((unsigned short)(w[e] & 0xffffu)) + bf16_bits_to_f((unsigned short)(w[e] >> 16));
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        if (jc == 0 && c < C) part[(long)blockIdx.x * C + c] = s;
      }
      if (c >= C || j >= ncols) continue;
      *(u32x4*)(out + (long)c * ldo + j) = w;
    }
  }
}

// token-major padded image (conv forward over the padded domain, fs2_pad_rows):
// out row b*(T+2P) + i = X row b*T + reflect(i-P) (reflect) or zero outside [0,T); rows past
// B*(T+2P) zero.  One thread per 16-byte chunk, 32-bit indices (host-checked).
__global__ void __launch_bounds__(256) pad_rows_kernel(const bf16* X, long ldx, int B, int T,
                                                       int C8, int P, int reflect, bf16* out,
                                                       long ldo, unsigned n8) {
  const unsigned idx = blockIdx.x * 256u + threadIdx.x;
  if (idx >= n8) return;
  const unsigned r = idx / (unsigned)C8;
  const int c = (int)(idx - r * (unsigned)C8) * 8;
  const unsigned L = (unsigned)(T + 2 * P);
  const unsigned b = r / L;
  const int i = (int)(r - b * L) - P;
  u32x4 v = {0u, 0u, 0u, 0u};
  if ((int)b < B) {
    const int t = reflect ? reflect_idx(i, T) : i;
    if (t >= 0 && t < T) v = *(const u32x4*)(X + ((long)b * T + t) * ldx + c);
  }
  *(u32x4*)(out + (long)r * ldo + c) = v;
}

int colsum_blocks(int M) { return min(512, max(1, (M + 63) / 64)); }
bool a16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int64_t fs2_ln_workspace_floats(int M, int D) { return 3L * ln_blocks(M) * D; }
extern "C" int64_t fs2_colsum_workspace_floats(int M, int N) { return (int64_t)colsum_blocks(M) * N; }

extern "C" int fs2_ln_fwd(const void* x, int64_t ldx, const void* r, int64_t ldr, float p_r,
                          uint32_t salt_r, void* s_out, const float* gamma, const float* beta,
                          float eps, int do_tanh, float p_o, uint32_t salt_o,
                          const float* row_mask, const void* post_add, int64_t ldp, void* y,
                          int64_t ldy, float* mean, float* rstd, int M, int D, int dtype,
                          uint32_t seed, void* img, int img_t, int img_p, void* stream) {
  if (M <= 0) return 0;
  if (D <= 0 || D > 64 * MAXJ || !x || !y || !gamma || !beta || !mean || !rstd) return FS2_EINVAL;
  if (img && (dtype != FS2_BF16 || img_t <= 0 || M % img_t || img_p < 0 || img_p >= img_t ||
              (D % 8) || !a16(img)))
    return FS2_EINVAL;
  LnFwdP p{(const char*)x, ldx, (const char*)r, ldr, p_r, salt_r, (char*)s_out, gamma, beta,
           eps, do_tanh, p_o, salt_o, row_mask, (const char*)post_add, ldp, (char*)y, ldy, mean,
           rstd, M, D, seed, nullptr, img_t, img_p};
  bool img_done = false;
  dim3 grid((M + 3) / 4);
  hipStream_t s = (hipStream_t)stream;
  const int V = dtype == FS2_BF16 ? 8 : 4;
  const int nch = (D / V + 63) / 64;
  const bool vec = (D % V) == 0 && nch <= 4 && a16(x) && (ldx % V) == 0 && a16(y) &&
                   (ldy % V) == 0 && a16(gamma) && a16(beta) && (!r || (a16(r) && ldr % V == 0)) &&
                   (!s_out || a16(s_out)) && (!post_add || (a16(post_add) && ldp % V == 0));
  if (dtype == FS2_BF16) {
    if (!vec) hipLaunchKernelGGL(ln_fwd_kernel<bf16>, grid, dim3(256), 0, s, p);
    else if (nch == 1 && ln_fwd_rows() == 2 && a16(gamma) && a16(beta)) {
      p.img = (char*)img;
      img_done = true;
      hipLaunchKernelGGL((ln_dpp() ? ln_fwd_rows_kernel<2, true> : ln_fwd_rows_kernel<2, false>), dim3((M + 7) / 8), dim3(256), 0, s, p);
    } else if (nch == 1 && ln_fwd_rows() == 4 && a16(gamma) && a16(beta)) {
      p.img = (char*)img;
      img_done = true;
      hipLaunchKernelGGL((ln_dpp() ? ln_fwd_rows_kernel<4, true> : ln_fwd_rows_kernel<4, false>), dim3((M + 15) / 16), dim3(256), 0, s, p);
    }
    else if (nch == 1) hipLaunchKernelGGL((ln_fwd_vec_kernel<bf16, 1>), grid, dim3(256), 0, s, p);
    else if (nch == 2) hipLaunchKernelGGL((ln_fwd_vec_kernel<bf16, 2>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((ln_fwd_vec_kernel<bf16, 4>), grid, dim3(256), 0, s, p);
  } else if (dtype == FS2_F32) {
    if (!vec) hipLaunchKernelGGL(ln_fwd_kernel<float>, grid, dim3(256), 0, s, p);
    else if (nch == 1) hipLaunchKernelGGL((ln_fwd_vec_kernel<float, 1>), grid, dim3(256), 0, s, p);
    else if (nch == 2) hipLaunchKernelGGL((ln_fwd_vec_kernel<float, 2>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((ln_fwd_vec_kernel<float, 4>), grid, dim3(256), 0, s, p);
  } else {
    return FS2_EINVAL;
  }
  FS2_CHECK_LAUNCH();
  if (img && !img_done)   // the other kernels: the image from y in a second pass
    return fs2_pad_rows(y, ldy, M / img_t, img_t, D, img_p, 1, 0, img, D, dtype, stream);
  return 0;
}

extern "C" int fs2_ln_bwd(const void* dy, int64_t lddy, const void* s, int64_t lds,
                          const float* mean, const float* rstd, const float* gamma,
                          const float* beta, int do_tanh, float p_o, uint32_t salt_o,
                          const float* row_mask, int relu_gate_in, void* ds, int64_t ldds,
                          void* dr, float p_r, uint32_t salt_r, float* dgamma, float* dbeta,
                          float* dcol, int M, int D, int dtype, uint32_t seed, float* workspace,
                          void* stream) {
  if (M <= 0) return 0;
  if (D <= 0 || D > 64 * MAXJ || !dy || !s || !ds || !gamma || !beta) return FS2_EINVAL;
  if ((dgamma || dbeta) && (!dgamma || !dbeta)) return FS2_EINVAL;
  if ((dgamma || dcol) && !workspace) return FS2_EINVAL;
  const int nb = ln_blocks(M);
  const int rpb = (M + nb - 1) / nb;
  // partial rows [nb][npart*D]: (gamma, beta)?, col?
  const int npart = (dgamma ? 2 : 0) + (dcol ? 1 : 0);
  float* pg = dgamma ? workspace : nullptr;
  float* pb = dgamma ? workspace + D : nullptr;
  float* pcl = dcol ? workspace + (dgamma ? 2 * D : 0) : nullptr;
  LnBwdP p{(const char*)dy, lddy, (const char*)s, lds, mean, rstd, gamma, beta, do_tanh, p_o,
           salt_o, row_mask, relu_gate_in, (char*)ds, ldds, (char*)dr, p_r, salt_r, pg, pb, M,
           D, seed, rpb, pcl, (long)npart * D};
  hipStream_t st = (hipStream_t)stream;
  static const int tanh_exact = fs2_exp_int("FS2_LN_TANH_EXACT", 0);
  if (tanh_exact && do_tanh) p.do_tanh = 2;
  const int V = dtype == FS2_BF16 ? 8 : 4;
  const int nch = (D / V + 63) / 64;
  const bool vec = (D % V) == 0 && nch <= 4 && a16(dy) && (lddy % V) == 0 && a16(s) &&
                   (lds % V) == 0 && a16(ds) && (ldds % V) == 0 && (!dr || a16(dr)) &&
                   a16(gamma) && a16(beta);
  float* part = npart ? workspace : nullptr;
  const int kind0 = dgamma ? 0 : 2;
  if (dtype == FS2_BF16) {
    if (!vec) hipLaunchKernelGGL(ln_bwd_kernel<bf16>, dim3(nb), dim3(256), 0, st, p);
    else if (nch == 1 && do_tanh && ln_tanh_rows()) hipLaunchKernelGGL((ln_dpp() ? ln_bwd_rows_kernel<2, true, true> : ln_bwd_rows_kernel<2, true, false>), dim3(nb), dim3(256), 0, st, p, part, npart, kind0);
    else if (nch == 1 && ln_rows_r() == 4 && !do_tanh) hipLaunchKernelGGL((ln_dpp() ? ln_bwd_rows_kernel<4, false, true> : ln_bwd_rows_kernel<4, false, false>), dim3(nb), dim3(256), 0, st, p, part, npart, kind0);
    else if (nch == 1 && ln_rows_r() == 2 && !do_tanh) hipLaunchKernelGGL((ln_dpp() ? ln_bwd_rows_kernel<2, false, true> : ln_bwd_rows_kernel<2, false, false>), dim3(nb), dim3(256), 0, st, p, part, npart, kind0);
    else if (nch == 1) hipLaunchKernelGGL((ln_bwd_vec_kernel<bf16, 1>), dim3(nb), dim3(256), 0, st, p, part, npart, kind0);
    else if (nch == 2) hipLaunchKernelGGL((ln_bwd_vec_kernel<bf16, 2>), dim3(nb), dim3(256), 0, st, p, part, npart, kind0);
    else hipLaunchKernelGGL((ln_bwd_vec_kernel<bf16, 4>), dim3(nb), dim3(256), 0, st, p, part, npart, kind0);
  } else if (dtype == FS2_F32) {
    if (!vec) hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3(nb), dim3(256), 0, st, p);
    else if (nch == 1) hipLaunchKernelGGL((ln_bwd_vec_kernel<float, 1>), dim3(nb), dim3(256), 0, st, p, part, npart, kind0);
    else if (nch == 2) hipLaunchKernelGGL((ln_bwd_vec_kernel<float, 2>), dim3(nb), dim3(256), 0, st, p, part, npart, kind0);
    else hipLaunchKernelGGL((ln_bwd_vec_kernel<float, 4>), dim3(nb), dim3(256), 0, st, p, part, npart, kind0);
  } else {
    return FS2_EINVAL;
  }
  FS2_CHECK_LAUNCH();
  // FS2_LN_NORED=1 (experiments build, timing probe only -- the parameter gradients are then
  // left unreduced): what the reduce_parts launches cost the step
  static const int nored = fs2_exp_int("FS2_LN_NORED", 0);
  if (npart && !nored) {
    float* o0 = dgamma ? dgamma : dcol;
    float* o1 = dgamma ? dbeta : nullptr;
    float* o2 = dgamma ? dcol : nullptr;
    launch_reduce_parts(st, workspace, nb, D, npart, o0, o1, o2, 1);
    FS2_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int fs2_colsum(const void* X, int64_t ldx, int M, int N, int dtype, float* out,
                          int accumulate, float* workspace, void* stream) {
  if (N <= 0) return 0;
  if (!X || !out || !workspace || M < 0) return FS2_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int nb = colsum_blocks(M);
  const int rpb = (M + nb - 1) / nb;
  const int V = dtype == FS2_BF16 ? 8 : 4;
  const bool vec = (N % V) == 0 && N / V <= 256 && a16(X) && (ldx % V) == 0;
  static const int slab = fs2_exp_int("FS2_COLSUM_SLAB", 1);
  if (vec && slab && N / V >= 32) {
    const dim3 g(nb, (N / V + 63) / 64);
    if (dtype == FS2_BF16)
      hipLaunchKernelGGL((colsum_slab_kernel<bf16, 8>), g, dim3(256), 0, st, (const bf16*)X, (long)ldx, M, N, rpb, workspace);
    else if (dtype == FS2_F32)
      hipLaunchKernelGGL((colsum_slab_kernel<float, 8>), g, dim3(256), 0, st, (const float*)X, (long)ldx, M, N, rpb, workspace);
    else
      return FS2_EINVAL;
  } else if (dtype == FS2_BF16) {
    if (vec)
      hipLaunchKernelGGL(colsum_vec_kernel<bf16>, dim3(nb), dim3(256), 0, st, (const bf16*)X, (long)ldx, M, N, rpb, workspace);
    else
      hipLaunchKernelGGL(colsum_partial_kernel<bf16>, dim3((N + 255) / 256, nb), dim3(256), 0, st, (const bf16*)X, ldx, M, N, rpb, workspace);
  } else if (dtype == FS2_F32) {
    if (vec)
      hipLaunchKernelGGL(colsum_vec_kernel<float>, dim3(nb), dim3(256), 0, st, (const float*)X, (long)ldx, M, N, rpb, workspace);
    else
      hipLaunchKernelGGL(colsum_partial_kernel<float>, dim3((N + 255) / 256, nb), dim3(256), 0, st, (const float*)X, ldx, M, N, rpb, workspace);
  } else {
    return FS2_EINVAL;
  }
  launch_reduce_parts(st, workspace, nb, N, 1, out, nullptr, nullptr, accumulate);
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_sum_slices(const float* ws, int nslices, int64_t stride, int64_t n,
                              float* out, int accumulate, void* stream) {
  if (n == 0) return 0;
  if (!ws || !out || nslices < 1 || (n % 4) || (stride % 4) || !a16(ws) || !a16(out))
    return FS2_EINVAL;
  const long n4 = n / 4;
  hipLaunchKernelGGL(sum_slices_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, ws, nslices, (long)stride, n4, out, accumulate);
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_conv_fold(const float* Xpad, int nsplit, int64_t split_stride, int B, int T,
                             int P, int C, void* out, int64_t ldo, const void* residual,
                             int64_t ldr, const float* row_scale, const float* row_scale_post,
                             int dtype, void* stream) {
  const long n = (long)B * T * C;
  if (n == 0) return 0;
  if (nsplit < 1) nsplit = 1;
  if (!Xpad || !out || (C % 4) || P < 0 || (P > 0 && P >= T)) return FS2_EINVAL;
  if (nsplit > 1 && (split_stride < (long)B * (T + 2 * P) * C || (split_stride % 4)))
    return FS2_EINVAL;
  const dim3 g((unsigned)((n / 4 + 255) / 256)), b(256);
  hipStream_t s = (hipStream_t)stream;
  static const bool no8 = fs2_exp_int("FS2_FOLD8", 1) == 0;
  const bool v8 = !no8 && dtype == FS2_BF16 && C % 8 == 0 && a16(out) && ldo % 8 == 0 &&
                  (!residual || (a16(residual) && ldr % 8 == 0)) && a16(Xpad) &&
                  (nsplit == 1 || split_stride % 4 == 0) && n / 8 < (1L << 31);
  if (v8) {
    const unsigned n8 = (unsigned)(n / 8);
    hipLaunchKernelGGL(conv_fold8_kernel, dim3((n8 + 255) / 256), b, 0, s, Xpad, nsplit,
                       (long)split_stride, T, P, C / 8, (bf16*)out, (long)ldo,
                       (const bf16*)residual, (long)ldr, row_scale, row_scale_post, n8);
  } else if (dtype == FS2_BF16)
    hipLaunchKernelGGL(conv_fold_kernel<bf16>, g, b, 0, s, Xpad, nsplit, (long)split_stride, T,
                       P, C, (bf16*)out, (long)ldo, (const bf16*)residual, (long)ldr, row_scale,
                       row_scale_post, n);
  else if (dtype == FS2_F32)
    hipLaunchKernelGGL(conv_fold_kernel<float>, g, b, 0, s, Xpad, nsplit, (long)split_stride, T,
                       P, C, (float*)out, (long)ldo, (const float*)residual, (long)ldr, row_scale,
                       row_scale_post, n);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}

// this translation unit's dropout seed base (fs2_common.h)
FS2_SEED_SETTER(fs2_seed_base_norm)

extern "C" int fs2_pad_transpose(const void* X, int64_t ldx, int B, int T, int C, int P,
                                 int reflect, void* out, int64_t ldo, int ncols, float* colsum,
                                 float* workspace, int dtype, void* stream) {
  if (B <= 0 || T <= 0 || C <= 0) return 0;
  if (dtype != FS2_BF16 || !X || !out || P < 0 || (reflect && P >= T)) return FS2_EINVAL;
  if ((C % 8) || (ldx % 8) || (ldo % 8) || (ncols % 8) || ncols < (long)B * (T + 2 * P) ||
      ldo < ncols || !a16(X) || !a16(out))
    return FS2_EALIGN;
  if (colsum && (reflect || !workspace)) return FS2_EINVAL;
  dim3 grid((ncols + TJ - 1) / TJ, (C + TC - 1) / TC);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(pad_transpose_kernel, grid, dim3(256), 0, s, (const bf16*)X, (long)ldx, B, T,
                     C, P, reflect, (bf16*)out, (long)ldo, ncols, colsum ? workspace : nullptr);
  FS2_CHECK_LAUNCH();
  if (colsum) {   // colsum[c] += sum over the token blocks' partials (fixed order)
    launch_reduce_parts(s, workspace, (int)grid.x, C, 1, colsum, nullptr, nullptr, 1);
    FS2_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int fs2_pad_rows(const void* X, int64_t ldx, int B, int T, int C, int P, int reflect,
                            int tail, void* out, int64_t ldo, int dtype, void* stream) {
  if (B <= 0 || T <= 0 || C <= 0) return 0;
  if (dtype != FS2_BF16 || !X || !out || P < 0 || tail < 0 || (reflect && P >= T))
    return FS2_EINVAL;
  if ((C % 8) || (ldx % 8) || (ldo % 8) || ldo < C || ldx < C || !a16(X) || !a16(out))
    return FS2_EALIGN;
  const long rows = (long)B * (T + 2 * P) + tail;
  const long n8 = rows * (C / 8);
  if (n8 >= 0x7fffffffL || rows * ldo >= 0x7fffffffL) return FS2_EINVAL;
  hipLaunchKernelGGL(pad_rows_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const bf16*)X, (long)ldx, B, T, C / 8, P, reflect,
                     (bf16*)out, (long)ldo, (unsigned)n8);
  FS2_CHECK_LAUNCH();
  return 0;
}
