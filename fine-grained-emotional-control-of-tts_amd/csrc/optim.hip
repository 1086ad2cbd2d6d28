// AdamW over the flat fp32 parameter buffer and per-step weight preparation.
//
// AdamW replaces torch.optim.AdamW(model.parameters(), lr=1e-4) of the reference train step
// (fastspeech2/train.py:232; defaults betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2),
// following torch's single-tensor algorithm op for op:
//   p *= 1 - lr*wd ; m = lerp(m, g, 1-b1) ; v = v*b2 + (1-b2) g^2
//   p += -(lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// One pass over 85.3 M params: 7 x 4 B read/written per param -> HBM bound (K17).
//
// weight_prep turns each torch-layout master weight W[O][C][KW] (fp32) into the two GEMM
// operand images the MFMA kernels read K-major: Wf[O][KW*C] (forward) and Wb[C][KW*O]
// (data gradient), cast to the activation dtype.
#include "fs2_common.h"

namespace {

// 4 elements per lane through 16-byte loads / stores (same per-element arithmetic as
// adamw_kernel, so identical results): the scalar kernel ran at ~5.3 TB/s
__device__ __forceinline__ void adamw_elem(float& pi, float& mi, float& vi, float gi,
                                           float decay_mul, float w1, float beta2, float omb2,
                                           float step_size, float bc2_sqrt, float eps,
                                           float gscale) {
  // no FMA contraction: every kernel that inlines this (vector, tile-fused, ranges) must round
  // identically, whatever the surrounding code lets the compiler fuse
#pragma clang fp contract(off)
  const float gr = gi * gscale;
  pi = pi * decay_mul;
  mi = (w1 < 0.5f) ? mi + w1 * (gr - mi) : gr - (gr - mi) * (1.f - w1);
  vi = vi * beta2 + omb2 * gr * gr;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  pi = pi + (-step_size) * (mi / denom);
}

__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                             float* __restrict__ m, float* __restrict__ v, long n, float decay_mul,
                             float w1, float beta2, float omb2, float step_size, float bc2_sqrt,
                             float eps, float gscale) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // torch lerp: weight < 0.5 -> self + w * (end - self)  (adamw_elem)
  float pi = p[i], mi = m[i], vi = v[i];
  adamw_elem(pi, mi, vi, g[i], decay_mul, w1, beta2, omb2, step_size, bc2_sqrt, eps, gscale);
  p[i] = pi; m[i] = mi; v[i] = vi;
}

__global__ void __launch_bounds__(256) adamw_vec_kernel(float* __restrict__ p,
                                                        const float* __restrict__ g,
                                                        float* __restrict__ m,
                                                        float* __restrict__ v, long n4,
                                                        float decay_mul, float w1, float beta2,
                                                        float omb2, float step_size,
                                                        float bc2_sqrt, float eps, float gscale) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  f32x4 pp = ((const f32x4*)p)[i], gg = ((const f32x4*)g)[i];
  f32x4 mm = ((const f32x4*)m)[i], vv = ((const f32x4*)v)[i];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float pi = pp[e], mi = mm[e], vi = vv[e];
    adamw_elem(pi, mi, vi, gg[e], decay_mul, w1, beta2, omb2, step_size, bc2_sqrt, eps, gscale);
    pp[e] = pi; mm[e] = mi; vv[e] = vi;
  }
  ((f32x4*)p)[i] = pp;
  ((f32x4*)m)[i] = mm;
  ((f32x4*)v)[i] = vv;
}

template <typename T>
__global__ void weight_prep_kernel(const float* W, int O, int C, int KW, int okc, T* Wf, int ldf,
                                   T* Wb, int ldb) {
  // one thread per (row of Wf / Wb, padded column): write-coalesced on Wf
  const long n = (long)O * ldf;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int o = (int)(i / ldf), col = (int)(i - (long)o * ldf);
    float v = 0.f;
    if (col < KW * C) {
      int j, c;
      if (okc & 8) {   // tap-inner 64-channel chunks (wf_col)
        const int ch = col / (KW * 64), r = col - ch * (KW * 64);
        j = r >> 6;
        c = ch * 64 + (r & 63);
      } else {
        j = col / C;
        c = col - j * C;
      }
      v = (okc & 1) ? W[((long)o * KW + j) * C + c] : W[((long)o * C + c) * KW + j];
    }
    Wf[i] = from_f<T>(v);
  }
  if (Wb) {
    const long nb = (long)C * ldb;
    if (i < nb) {
      const int c = (int)(i / ldb), col = (int)(i - (long)c * ldb);
      float v = 0.f;
      if (col < KW * O) {
        int jb, o;
        if (okc & 4) {   // tap-inner 64-channel chunks (wb_col)
          const int ch = col / (KW * 64), r = col - ch * (KW * 64);
          jb = r >> 6;
          o = ch * 64 + (r & 63);
        } else {
          jb = col / O;
          o = col - jb * O;
        }
        const int j = (okc & 2) ? KW - 1 - jb : jb;   // bit 1: Wb's taps reversed
        v = (okc & 1) ? W[((long)o * KW + j) * C + c] : W[((long)o * C + c) * KW + j];
      }
      Wb[i] = from_f<T>(v);
    }
  }
}

// tap index of Wb (w_okc bit 1: taps reversed)
__device__ __forceinline__ int wb_tap(const fs2_wprep_desc& d, int j) {
  return (d.w_okc & 2) ? d.KW - 1 - j : j;
}
// Wb column of (tap j, output channel o): j*O + o, or with w_okc bit 2 (O % 64 == 0) the
// tap-inner order of 64-channel chunks, (o / 64)*(KW*64) + j*64 + o % 64 -- the K order in which
// the padded-dY data gradient reads its image rows one tap apart in consecutive 64-deep stages
// (fs2_gemm_desc.a_kw)
__device__ __forceinline__ long wb_col(int okc, int KW, int O, int j, int o) {
  return (okc & 4) ? (long)(o >> 6) * (KW * 64) + j * 64 + (o & 63) : (long)j * O + o;
}
// Wf column of (tap j, input channel c): k = j*C + c, or with w_okc bit 3 (C % 64 == 0) the same
// tap-inner chunk order (the padded-image conv forward, fs2_gemm_desc.a_kw)
__device__ __forceinline__ int wf_col(int okc, int KW, int k, int j, int c) {
  return (okc & 8) ? (c >> 6) * (KW * 64) + j * 64 + (c & 63) : k;
}

// one block per 64x64 tile (o, k = j*C + c) of one weight's forward image; the weight is found
// by binary search over the descriptor prefix sums (staged in LDS)
template <typename T>
__global__ void __launch_bounds__(256) weight_prep_batched_kernel(const fs2_wprep_desc* descs,
                                                                  int n) {
  __shared__ int t0s[256];
  __shared__ float tile[64][65];
  for (int i = threadIdx.x; i < n; i += blockDim.x) t0s[i] = descs[i].tile0;
  __syncthreads();
  const int blk = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {               // last descriptor with tile0 <= blk
    const int mid = (lo + hi + 1) >> 1;
    if (t0s[mid] <= blk) lo = mid; else hi = mid - 1;
  }
  const fs2_wprep_desc d = descs[lo];
  const int t = blk - d.tile0;
  const int to = t / d.tiles_k, tk = t - to * d.tiles_k;
  const int o0 = to * 64, k0 = tk * 64;
  const int KC = d.KW * d.C;
  T* Wf = (T*)d.Wf;
  // (tap j, channel c) of the tile's 64 k columns, one division each instead of one per element
  __shared__ int jcs[64];
  if (threadIdx.x < 64) {
    const int k = k0 + threadIdx.x;
    const int j = k / d.C;
    jcs[threadIdx.x] = (j << 16) | (k - j * d.C);
  }
  __syncthreads();
  // read (coalesced along k for the [O][KW][C] layout) -> Wf, and stage for the transpose
  for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) {
    const int ol = i >> 6, kl = i & 63, o = o0 + ol, k = k0 + kl;
    if (o >= d.O || k >= d.ldf) continue;
    float v = 0.f;
    if (k < KC) {
      const int j = jcs[kl] >> 16, c = jcs[kl] & 0xffff;
      v = (d.w_okc & 1) ? d.W[(long)o * KC + k] : d.W[((long)o * d.C + c) * d.KW + j];
    }
    const int kf = k < KC ? wf_col(d.w_okc, d.KW, k, jcs[kl] >> 16, jcs[kl] & 0xffff) : k;
    Wf[(long)o * d.ldf + kf] = from_f<T>(v);
    tile[ol][kl] = v;
  }
  if (!d.Wb) return;
  __syncthreads();
  // Wb[c][j*O + o]: consecutive threads take consecutive o
  T* Wb = (T*)d.Wb;
  for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) {
    const int kl = i >> 6, ol = i & 63, o = o0 + ol, k = k0 + kl;
    if (o >= d.O || k >= KC) continue;
    const int j = wb_tap(d, jcs[kl] >> 16), c = jcs[kl] & 0xffff;
    Wb[(long)c * d.ldb + wb_col(d.w_okc, d.KW, d.O, j, o)] = from_f<T>(tile[ol][kl]);
  }
}

// ---- AdamW fused with the weight-image preparation ----------------------------------------
// The optimiser pass is the last reader and writer of every master weight in a step, and the
// next forward's GEMMs need the bf16 images Wf (forward, [O][ldf]) and Wb (data gradient,
// [C][KW*O]) of exactly the updated values.  One block per 64x64 tile (o, k = j*C + c) of each
// GEMM weight runs the AdamW update of the tile (same per-element arithmetic as adamw_elem, so
// identical parameters and moments) and writes the tile's Wf rows and, through an LDS
// transpose, its Wb rows: the separate fs2_weight_prep_batched pass re-read all 85 M fp32
// masters (0.33 GB) after AdamW had just written them.  Every other parameter (biases, norms,
// embeddings) goes through the element-wise ranges kernel.
struct AdamScal {
  float decay_mul, w1, beta2, omb2, step_size, bc2_sqrt, eps, gscale;
};

template <typename T>
__global__ void __launch_bounds__(256) adamw_prep_tiles_kernel(const fs2_wprep_desc* descs, int n,
                                                               float* __restrict__ pb,
                                                               const float* __restrict__ gb,
                                                               float* __restrict__ mb,
                                                               float* __restrict__ vb, AdamScal a) {
  __shared__ int t0s[256];
  __shared__ float tile[64][65];
  __shared__ int jcs[64];
  for (int i = threadIdx.x; i < n; i += blockDim.x) t0s[i] = descs[i].tile0;
  __syncthreads();
  const int blk = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (t0s[mid] <= blk) lo = mid; else hi = mid - 1;
  }
  const fs2_wprep_desc d = descs[lo];
  const int t = blk - d.tile0;
  const int to = t / d.tiles_k, tk = t - to * d.tiles_k;
  const int o0 = to * 64, k0 = tk * 64;
  const int KC = d.KW * d.C;
  const long base = d.W - pb;          // the weight's offset in the flat buffers ([O][KW][C])
  if (threadIdx.x < 64) {
    const int k = k0 + threadIdx.x;
    const int j = k / d.C;
    jcs[threadIdx.x] = (j << 16) | (k - j * d.C);
  }
  __syncthreads();
  T* Wf = (T*)d.Wf;
  T* Wb = (T*)d.Wb;
  // 16-byte form: 4 consecutive k per lane for the fp32 streams (p, g, m, v: 80 % of the
  // bytes) and 4 consecutive o per lane for the transposed image -- when the weight's flat
  // offset and row pitches keep every quad aligned (all the model's weights); the scalar form
  // below otherwise.  Same adamw_elem per element either way.
  const bool vec = sizeof(T) == 2 && (base & 3) == 0 && (KC & 3) == 0 && (d.ldf & 3) == 0 &&
                   (!d.Wb || ((d.ldb & 3) == 0 && (d.O & 3) == 0));
  if (vec) {
    // all 4 quads' loads in flight before the first update (blockDim.x == 256)
#pragma unroll
    for (int i = threadIdx.x; i < 64 * 16; i += 256) {
      const int ol = i >> 4, kl = (i & 15) * 4, o = o0 + ol, k = k0 + kl;
      if (o >= d.O || k >= d.ldf) continue;
      f32x4 w = {0.f, 0.f, 0.f, 0.f};
      if (k < KC) {   // KC % 4 == 0: the quad is all in or all out
        const long e = base + (long)o * KC + k;
        f32x4 pi = *(const f32x4*)(pb + e), mi = *(const f32x4*)(mb + e);
        f32x4 vi = *(const f32x4*)(vb + e);
        const f32x4 gi = *(const f32x4*)(gb + e);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float pq = pi[q], mq = mi[q], vq = vi[q];
          adamw_elem(pq, mq, vq, gi[q], a.decay_mul, a.w1, a.beta2, a.omb2, a.step_size,
                     a.bc2_sqrt, a.eps, a.gscale);
          pi[q] = pq; mi[q] = mq; vi[q] = vq;
        }
        *(f32x4*)(pb + e) = pi;
        *(f32x4*)(mb + e) = mi;
        *(f32x4*)(vb + e) = vi;
        w = pi;
      }
      uint2 h;
      h.x = (unsigned)__builtin_bit_cast(unsigned short, (bf16)w[0]) |
            ((unsigned)__builtin_bit_cast(unsigned short, (bf16)w[1]) << 16);
      h.y = (unsigned)__builtin_bit_cast(unsigned short, (bf16)w[2]) |
            ((unsigned)__builtin_bit_cast(unsigned short, (bf16)w[3]) << 16);
      const int kf = k < KC ? wf_col(d.w_okc, d.KW, k, jcs[kl] >> 16, jcs[kl] & 0xffff) : k;
      *(uint2*)(Wf + (long)o * d.ldf + kf) = h;
#pragma unroll
      for (int q = 0; q < 4; ++q) tile[ol][kl + q] = w[q];
    }
    if (!d.Wb) return;
    __syncthreads();
#pragma unroll
    for (int i = threadIdx.x; i < 64 * 16; i += 256) {
      const int kl = i >> 4, ol = (i & 15) * 4, o = o0 + ol, k = k0 + kl;
      if (o >= d.O || k >= KC) continue;   // O % 4 == 0: the quad is all in or all out
      const int j = wb_tap(d, jcs[kl] >> 16), c = jcs[kl] & 0xffff;
      uint2 h;
      h.x = (unsigned)__builtin_bit_cast(unsigned short, (bf16)tile[ol][kl]) |
            ((unsigned)__builtin_bit_cast(unsigned short, (bf16)tile[ol + 1][kl]) << 16);
      h.y = (unsigned)__builtin_bit_cast(unsigned short, (bf16)tile[ol + 2][kl]) |
            ((unsigned)__builtin_bit_cast(unsigned short, (bf16)tile[ol + 3][kl]) << 16);
      *(uint2*)(Wb + (long)c * d.ldb + wb_col(d.w_okc, d.KW, d.O, j, o)) = h;
    }
    return;
  }
  for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) {
    const int ol = i >> 6, kl = i & 63, o = o0 + ol, k = k0 + kl;
    if (o >= d.O || k >= d.ldf) continue;
    float v = 0.f;
    if (k < KC) {
      const long e = base + (long)o * KC + k;
      float pi = pb[e], mi = mb[e], vi = vb[e];
      adamw_elem(pi, mi, vi, gb[e], a.decay_mul, a.w1, a.beta2, a.omb2, a.step_size, a.bc2_sqrt,
                 a.eps, a.gscale);
      pb[e] = pi; mb[e] = mi; vb[e] = vi;
      v = pi;
    }
    const int kf = k < KC ? wf_col(d.w_okc, d.KW, k, jcs[kl] >> 16, jcs[kl] & 0xffff) : k;
    Wf[(long)o * d.ldf + kf] = from_f<T>(v);
    tile[ol][kl] = v;
  }
  if (!d.Wb) return;
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) {
    const int kl = i >> 6, ol = i & 63, o = o0 + ol, k = k0 + kl;
    if (o >= d.O || k >= KC) continue;
    const int j = wb_tap(d, jcs[kl] >> 16), c = jcs[kl] & 0xffff;
    Wb[(long)c * d.ldb + wb_col(d.w_okc, d.KW, d.O, j, o)] = from_f<T>(tile[ol][kl]);
  }
}

// ranges: int64 triples (flat start, length, first block); 1024 elements per block
__global__ void __launch_bounds__(256) adamw_ranges_kernel(const int64_t* ranges, int n,
                                                           float* __restrict__ pb,
                                                           const float* __restrict__ gb,
                                                           float* __restrict__ mb,
                                                           float* __restrict__ vb, AdamScal a) {
  const int blk = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ranges[3 * mid + 2] <= blk) lo = mid; else hi = mid - 1;
  }
  const long start = ranges[3 * lo], len = ranges[3 * lo + 1];
  const long i0 = (long)(blk - ranges[3 * lo + 2]) * 1024 + threadIdx.x * 4;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long i = i0 + e;
    if (i >= len) break;
    const long x = start + i;
    float pi = pb[x], mi = mb[x], vi = vb[x];
    adamw_elem(pi, mi, vi, gb[x], a.decay_mul, a.w1, a.beta2, a.omb2, a.step_size, a.bc2_sqrt,
               a.eps, a.gscale);
    pb[x] = pi; mb[x] = mi; vb[x] = vi;
  }
}

}  // namespace

extern "C" int fs2_adamw_prep(const fs2_wprep_desc* descs, int n, int total_tiles,
                              const int64_t* ranges, int n_ranges, int range_blocks,
                              float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                              float decay_mul, float one_minus_beta1, float beta2,
                              float one_minus_beta2, float step_size, float bc2_sqrt, float eps,
                              float grad_scale, int dtype, void* stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq) return FS2_EINVAL;
  if (n < 0 || n > 256 || (n > 0 && !descs) || (n_ranges > 0 && !ranges)) return FS2_EINVAL;
  if (dtype != FS2_BF16 && dtype != FS2_F32) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const AdamScal a{decay_mul, one_minus_beta1, beta2, one_minus_beta2, step_size, bc2_sqrt, eps,
                   grad_scale};
  if (n > 0 && total_tiles > 0) {
    if (dtype == FS2_BF16)
      hipLaunchKernelGGL(adamw_prep_tiles_kernel<bf16>, dim3(total_tiles), dim3(256), 0, s, descs,
                         n, param, grad, exp_avg, exp_avg_sq, a);
    else
      hipLaunchKernelGGL(adamw_prep_tiles_kernel<float>, dim3(total_tiles), dim3(256), 0, s,
                         descs, n, param, grad, exp_avg, exp_avg_sq, a);
    FS2_CHECK_LAUNCH();
  }
  if (n_ranges > 0 && range_blocks > 0) {
    hipLaunchKernelGGL(adamw_ranges_kernel, dim3(range_blocks), dim3(256), 0, s, ranges, n_ranges,
                       param, grad, exp_avg, exp_avg_sq, a);
    FS2_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int fs2_weight_prep_batched(const fs2_wprep_desc* descs, int n, int total_tiles,
                                       int dtype, void* stream) {
  if (n == 0 || total_tiles == 0) return 0;
  if (!descs || n < 0 || n > 256 || total_tiles < 0) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FS2_BF16)
    hipLaunchKernelGGL(weight_prep_batched_kernel<bf16>, dim3(total_tiles), dim3(256), 0, s,
                       descs, n);
  else if (dtype == FS2_F32)
    hipLaunchKernelGGL(weight_prep_batched_kernel<float>, dim3(total_tiles), dim3(256), 0, s,
                       descs, n);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                         int64_t n, float decay_mul, float one_minus_beta1, float beta2,
                         float one_minus_beta2, float step_size, float bc2_sqrt, float eps,
                         float grad_scale, void* stream) {
  if (n == 0) return 0;
  if (!param || !grad || !exp_avg || !exp_avg_sq) return FS2_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const bool al = (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg |
                    (uintptr_t)exp_avg_sq) & 15) == 0;
  long done = 0;
  if (al && n >= 4) {
    const long n4 = n / 4;
    hipLaunchKernelGGL(adamw_vec_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st,
                       param, grad, exp_avg, exp_avg_sq, n4, decay_mul, one_minus_beta1, beta2,
                       one_minus_beta2, step_size, bc2_sqrt, eps, grad_scale);
    FS2_CHECK_LAUNCH();
    done = n4 * 4;
  }
  if (done < n) {
    const long r = n - done;
    hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)((r + 255) / 256)), dim3(256), 0, st,
                       param + done, grad + done, exp_avg + done, exp_avg_sq + done, r,
                       decay_mul, one_minus_beta1, beta2, one_minus_beta2, step_size, bc2_sqrt,
                       eps, grad_scale);
    FS2_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int fs2_weight_prep(const float* W, int O, int C, int KW, int w_okc, void* Wf, int ldf,
                               void* Wb, int ldb, int dtype, void* stream) {
  if (!W || !Wf || ldf < KW * C || (Wb && ldb < KW * O)) return FS2_EINVAL;
  const long n = max((long)O * ldf, Wb ? (long)C * ldb : 0L);
  const dim3 g((unsigned)((n + 255) / 256)), b(256);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FS2_BF16)
    hipLaunchKernelGGL(weight_prep_kernel<bf16>, g, b, 0, s, W, O, C, KW, w_okc, (bf16*)Wf, ldf,
                       (bf16*)Wb, ldb);
  else if (dtype == FS2_F32)
    hipLaunchKernelGGL(weight_prep_kernel<float>, g, b, 0, s, W, O, C, KW, w_okc, (float*)Wf, ldf,
                       (float*)Wb, ldb);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}
