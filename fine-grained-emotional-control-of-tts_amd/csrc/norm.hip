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

struct LnFwdP {
  const char* x; long ldx; const char* r; long ldr; float p_r; uint32_t salt_r;
  char* s_out; const float* gamma; const float* beta; float eps; int do_tanh;
  float p_o; uint32_t salt_o; const float* row_mask; const char* post_add; long ldp;
  char* y; long ldy; float* mean; float* rstd; int M, D; uint32_t seed;
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

struct LnBwdP {
  const char* dy; long lddy; const char* s; long lds; const float* mean; const float* rstd;
  const float* gamma; const float* beta; int do_tanh; float p_o; uint32_t salt_o;
  const float* row_mask; int relu_gate_in; char* ds; long ldds; char* dr; float p_r;
  uint32_t salt_r; float* part_g; float* part_b; int M, D; uint32_t seed; int rows_per_block;
};

template <typename T>
__global__ void __launch_bounds__(256) ln_bwd_kernel(LnBwdP p) {
  __shared__ float red[2][4][1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float pg[MAXJ], pb[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) { pg[j] = 0.f; pb[j] = 0.f; }
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
      p.part_g[(long)blockIdx.x * p.D + d] = red[0][0][d] + red[0][1][d] + red[0][2][d] + red[0][3][d];
      p.part_b[(long)blockIdx.x * p.D + d] = red[1][0][d] + red[1][1][d] + red[1][2][d] + red[1][3][d];
    }
  }
}

// out[n] (+)= sum_b part[b][n]: 64 columns x 4 row-slices per block, fixed-order LDS combine
__global__ void __launch_bounds__(256) reduce_partials_kernel(const float* part, int nb, int N,
                                                             float* out, int accumulate) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c;
  float s = 0.f;
  if (n < N) {
#pragma unroll 8
    for (int b = sl; b < nb; b += 4) s += part[(long)b * N + n];
  }
  red[sl][c] = s;
  __syncthreads();
  if (sl == 0 && n < N) {
    const float t = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    out[n] = accumulate ? out[n] + t : t;
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


// Adjoint of SB Conv1d's reflect "same" padding for the data gradient (K16):
//   dX[b,s] = Xp[b,s+P] + [1<=s<=P] Xp[b,P-s] + [T-1-P<=s<=T-2] Xp[b,2(T-1)-s+P]
// where Xp (fp32, T+2P rows per utterance) is the zero-padded shift-conv GEMM output
// (fs2_gemm conv_mode 4), fused with the dgrad epilogue: out = (dX*rs + residual)*rs2.
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

int ln_blocks(int M) { return min(512, max(1, (M + 15) / 16)); }
int colsum_blocks(int M) { return min(256, max(1, (M + 63) / 64)); }

}  // namespace

extern "C" int64_t fs2_ln_workspace_floats(int M, int D) { return 2L * ln_blocks(M) * D; }
extern "C" int64_t fs2_colsum_workspace_floats(int M, int N) { return (int64_t)colsum_blocks(M) * N; }

extern "C" int fs2_ln_fwd(const void* x, int64_t ldx, const void* r, int64_t ldr, float p_r,
                          uint32_t salt_r, void* s_out, const float* gamma, const float* beta,
                          float eps, int do_tanh, float p_o, uint32_t salt_o,
                          const float* row_mask, const void* post_add, int64_t ldp, void* y,
                          int64_t ldy, float* mean, float* rstd, int M, int D, int dtype,
                          uint32_t seed, void* stream) {
  if (M <= 0) return 0;
  if (D <= 0 || D > 64 * MAXJ || !x || !y || !gamma || !beta || !mean || !rstd) return FS2_EINVAL;
  LnFwdP p{(const char*)x, ldx, (const char*)r, ldr, p_r, salt_r, (char*)s_out, gamma, beta,
           eps, do_tanh, p_o, salt_o, row_mask, (const char*)post_add, ldp, (char*)y, ldy, mean,
           rstd, M, D, seed};
  dim3 grid((M + 3) / 4);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FS2_BF16) hipLaunchKernelGGL(ln_fwd_kernel<bf16>, grid, dim3(256), 0, s, p);
  else if (dtype == FS2_F32) hipLaunchKernelGGL(ln_fwd_kernel<float>, grid, dim3(256), 0, s, p);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_ln_bwd(const void* dy, int64_t lddy, const void* s, int64_t lds,
                          const float* mean, const float* rstd, const float* gamma,
                          const float* beta, int do_tanh, float p_o, uint32_t salt_o,
                          const float* row_mask, int relu_gate_in, void* ds, int64_t ldds,
                          void* dr, float p_r, uint32_t salt_r, float* dgamma, float* dbeta,
                          int M, int D, int dtype, uint32_t seed, float* workspace,
                          void* stream) {
  if (M <= 0) return 0;
  if (D <= 0 || D > 64 * MAXJ || !dy || !s || !ds || !gamma || !beta) return FS2_EINVAL;
  if ((dgamma || dbeta) && (!dgamma || !dbeta || !workspace)) return FS2_EINVAL;
  const int nb = ln_blocks(M);
  const int rpb = (M + nb - 1) / nb;
  float* pg = dgamma ? workspace : nullptr;
  float* pb = dgamma ? workspace + (long)nb * D : nullptr;
  LnBwdP p{(const char*)dy, lddy, (const char*)s, lds, mean, rstd, gamma, beta, do_tanh, p_o,
           salt_o, row_mask, relu_gate_in, (char*)ds, ldds, (char*)dr, p_r, salt_r, pg, pb, M,
           D, seed, rpb};
  hipStream_t st = (hipStream_t)stream;
  if (dtype == FS2_BF16) hipLaunchKernelGGL(ln_bwd_kernel<bf16>, dim3(nb), dim3(256), 0, st, p);
  else if (dtype == FS2_F32) hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3(nb), dim3(256), 0, st, p);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  if (dgamma) {
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((D + 63) / 64), dim3(256), 0, st, pg, nb, D,
                       dgamma, 1);
    hipLaunchKernelGGL(reduce_partials_kernel, dim3((D + 63) / 64), dim3(256), 0, st, pb, nb, D,
                       dbeta, 1);
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
  dim3 grid((N + 255) / 256, nb);
  if (dtype == FS2_BF16)
    hipLaunchKernelGGL(colsum_partial_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)X, ldx, M, N, rpb, workspace);
  else if (dtype == FS2_F32)
    hipLaunchKernelGGL(colsum_partial_kernel<float>, grid, dim3(256), 0, st, (const float*)X, ldx, M, N, rpb, workspace);
  else return FS2_EINVAL;
  hipLaunchKernelGGL(reduce_partials_kernel, dim3((N + 63) / 64), dim3(256), 0, st, workspace, nb,
                     N, out, accumulate);
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
  if (dtype == FS2_BF16)
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
