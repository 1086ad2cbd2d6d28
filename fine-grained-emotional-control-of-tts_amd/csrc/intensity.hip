// Frozen IntensityExtractor forward: input staging, emotion head, and the phoneme averaging of
// the FastSpeech2 train step.
//
//   rank_model/model.py:96-109   IntensityExtractor.forward (eval, no grad)
//   fastspeech2/train.py:16-51   get_intensity_representation
//
// The GEMM-shaped work of the extractor (input projection, QKV / out projections, the two
// k=9 zero-padded convs with GELU) runs on fs2_gemm (conv mode 5, act 2) and fs2_attn_fwd
// (mask_mode 0); the LayerNorms on fs2_ln_fwd.  This file holds the three HBM-bound pieces
// around them:
//   intensity_input_kernel  rank_X fp32 (B,T,C) or (B,C,T) -> GEMM rows [B*T][ldx] in the
//                           activation dtype, zero-padded columns (K multiple of 16 bytes)
//   intensity_head_kernel   I[m][e] = (keep[m] * (H[m] + emo_emb[emo[b]])) . Wc[e] + bc[e]
//                           (model.py:103-107: embedding add, masked_fill, classifier), fp32
//   phon_avg_kernel         out[b][p] = sum_{t in seg(b,p)} I[b][t] / max(d[b][p], 1) for
//                           p < phon_len[b], 0 elsewhere (train.py:33-49: repeat_interleave +
//                           index_add_ + clamp(min=1)); one block per utterance
#include "fs2_common.h"

namespace {

template <typename TO>
__global__ void intensity_input_kernel(const float* x, int bct, int T, int C, TO* X, int ldx,
                                       long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long m = i / ldx;
  const int c = (int)(i - m * ldx);
  const int b = (int)(m / T), t = (int)(m - (long)b * T);
  float v = 0.f;
  if (c < C) v = bct ? x[((long)b * C + c) * T + t] : x[m * C + c];
  X[i] = from_f<TO>(v);
}

// one wave per frame row; E <= 8 classifier outputs
template <typename T>
__global__ void __launch_bounds__(256) intensity_head_kernel(const T* H, long ldh,
                                                             const float* emo_tab,
                                                             const int64_t* emo,
                                                             const int64_t* lens, const float* Wc,
                                                             const float* bc, int B, int Tt, int D,
                                                             int E, float* I) {
  const int lane = threadIdx.x & 63;
  const long m = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= (long)B * Tt) return;
  const int b = (int)(m / Tt), t = (int)(m - (long)b * Tt);
  const bool keep = t < lens[b];
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  if (keep) {
    const float* em = emo_tab + emo[b] * D;
    const T* h = H + m * ldh;
    for (int d = lane; d < D; d += 64) {
      const float v = to_f(h[d]) + em[d];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e < E) acc[e] += v * Wc[(long)e * D + d];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e)
    if (e < E) {
      const float s = wave_sum(acc[e]);
      if (lane == 0) I[m * E + e] = s + bc[e];
    }
}

__global__ void __launch_bounds__(256) phon_avg_kernel(const float* I, int Tt, int E,
                                                       const int64_t* durs, const int64_t* phon_len,
                                                       int Tp, float* out) {
  __shared__ int cs[1025];
  const int b = blockIdx.x;
  const int np = (int)min<int64_t>(max<int64_t>(phon_len[b], 0), Tp);
  if (threadIdx.x == 0) {  // exclusive prefix sum of the first np durations (serial: Tp <= 1024)
    long c = 0;
    cs[0] = 0;
    for (int p = 0; p < np; ++p) {
      c += durs[(long)b * Tp + p];
      cs[p + 1] = (int)c;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < Tp * E; i += blockDim.x) {
    const int p = i / E, e = i - p * E;
    float v = 0.f;
    if (p < np) {
      const int t0 = cs[p], t1 = min(cs[p + 1], Tt);
      float s = 0.f;
      for (int t = t0; t < t1; ++t) s += I[((long)b * Tt + t) * E + e];
      v = s / fmaxf((float)(cs[p + 1] - cs[p]), 1.f);
    }
    out[((long)b * Tp + p) * E + e] = v;
  }
}

inline unsigned nblk(long n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

extern "C" int fs2_intensity_input(const float* x, int layout_bct, int B, int T, int C, void* X,
                                   int ldx, int dtype, void* stream) {
  const long n = (long)B * T * ldx;
  if (n == 0) return 0;
  if (!x || !X || ldx < C) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FS2_BF16)
    hipLaunchKernelGGL(intensity_input_kernel<bf16>, dim3(nblk(n)), dim3(256), 0, s, x,
                       layout_bct, T, C, (bf16*)X, ldx, n);
  else if (dtype == FS2_F32)
    hipLaunchKernelGGL(intensity_input_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, x,
                       layout_bct, T, C, (float*)X, ldx, n);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_intensity_head(const void* H, int64_t ldh, const float* emo_table,
                                  const int64_t* emotions, const int64_t* lengths, const float* Wc,
                                  const float* bc, int B, int T, int D, int E, float* I,
                                  int dtype, void* stream) {
  const long M = (long)B * T;
  if (M == 0) return 0;
  if (!H || !emo_table || !emotions || !lengths || !Wc || !bc || !I || E < 1 || E > 8)
    return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(nblk(M, 4));
  if (dtype == FS2_BF16)
    hipLaunchKernelGGL(intensity_head_kernel<bf16>, g, dim3(256), 0, s, (const bf16*)H, ldh,
                       emo_table, emotions, lengths, Wc, bc, B, T, D, E, I);
  else if (dtype == FS2_F32)
    hipLaunchKernelGGL(intensity_head_kernel<float>, g, dim3(256), 0, s, (const float*)H, ldh,
                       emo_table, emotions, lengths, Wc, bc, B, T, D, E, I);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_phoneme_average(const float* I, int T, int E, const int64_t* durations,
                                   const int64_t* phon_len, int B, int Tp, float* out,
                                   void* stream) {
  if ((long)B * Tp * E == 0) return 0;
  if (!I || !durations || !phon_len || !out || Tp > 1024) return FS2_EINVAL;
  hipLaunchKernelGGL(phon_avg_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, I, T, E,
                     durations, phon_len, Tp, out);
  FS2_CHECK_LAUNCH();
  return 0;
}
