// Masked softmax (+ attention-probability dropout) over materialised attention scores,
// and its backward.
//
// Replaces the softmax/dropout inside torch nn.MultiheadAttention as SB calls it
//  with the reference's masks (model.py:331-343, 411-419):
//   attn_mask = srcmask.unsqueeze(-1).repeat(nhead, 1, T).permute(0, 2, 1)   (head-major)
//   key_padding_mask = srcmask
// torch reads the (B*nhead) attn_mask batch-major, so for batch z = b*H + h the key k is
// masked iff key_pad[b][k] OR key_pad[(b*H + h) % B][k]  (verified with
// torch in this container) -- mask_mode 1.  mask_mode 0 is plain key padding (key_pad[b][k]),
// the IntensityExtractor's src_key_padding_mask (rank_model/model.py:35,101).  A fully masked row yields NaN, as torch's softmax does.
//
// One wave per (z, query) row; scores fp32, probabilities stored in the activation dtype.
// Dropout: fs2_attn_keep(dkey, row, k) (fs2_common.h; the same draw as flash.hip).
#include "fs2_common.h"

namespace {

template <typename T>
__global__ void __launch_bounds__(256) softmax_fwd_kernel(const float* S, const uint8_t* kp,
                                                          int tiled, int B, int H, int Tq, int Tk, int ldt,
                                                          float scale, float p_drop,
                                                          uint32_t seed, uint32_t salt, T* P,
                                                          T* Pd, long nrows) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const int z = (int)(row / Tq);
  const int b = z / H, h = z - b * H;
  const int b2 = tiled ? (b * H + h) % B : b;
  const uint8_t* k1 = kp + (long)b * Tk;
  const uint8_t* k2 = kp + (long)b2 * Tk;
  const float* s = S + row * ldt;
  float m = -INFINITY;
  for (int k = lane; k < Tk; k += 64)
    if (!(k1[k] | k2[k])) m = fmaxf(m, s[k] * scale);
  m = wave_max(m);
  float l = 0.f;
  for (int k = lane; k < Tk; k += 64)
    if (!(k1[k] | k2[k])) l += expf(s[k] * scale - m);
  l = wave_sum(l);
  const float inv = 1.f / l;  // l == 0 (all keys masked) -> inf * 0 = NaN below, like torch
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const uint32_t dkey = fs2_drop_key(seed, salt), thr = fs2_thr16(p_drop);
  T* prow = P + row * ldt;
  T* pdrow = Pd ? Pd + row * ldt : nullptr;
  for (int k = lane; k < ldt; k += 64) {
    float pv = 0.f;
    if (k < Tk) pv = (k1[k] | k2[k]) ? 0.f * inv : expf(s[k] * scale - m) * inv;
    prow[k] = from_f<T>(pv);
    if (pdrow) {
      float q = pv;
      if (p_drop > 0.f && k < Tk)
        q = fs2_attn_keep(dkey, (uint32_t)row, (uint32_t)k, thr) ? pv * inv_keep : 0.f;
      pdrow[k] = from_f<T>(q);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) softmax_bwd_kernel(const float* dPd, const T* P, int Tk,
                                                          int ldt, float scale, float p_drop,
                                                          uint32_t seed, uint32_t salt, T* dS,
                                                          long nrows) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const float* g = dPd + row * ldt;
  const T* prow = P + row * ldt;
  const float inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const uint32_t dkey = fs2_drop_key(seed, salt), thr = fs2_thr16(p_drop);
  float dot = 0.f;
  for (int k = lane; k < Tk; k += 64) {
    float gv = g[k];
    if (p_drop > 0.f) gv = fs2_attn_keep(dkey, (uint32_t)row, (uint32_t)k, thr) ? gv * inv_keep : 0.f;
    dot += gv * to_f(prow[k]);
  }
  dot = wave_sum(dot);
  T* drow = dS + row * ldt;
  for (int k = lane; k < ldt; k += 64) {
    float v = 0.f;
    if (k < Tk) {
      float gv = g[k];
      if (p_drop > 0.f) gv = fs2_attn_keep(dkey, (uint32_t)row, (uint32_t)k, thr) ? gv * inv_keep : 0.f;
      v = scale * to_f(prow[k]) * (gv - dot);
    }
    drow[k] = from_f<T>(v);
  }
}

}  // namespace

extern "C" int fs2_softmax_fwd(const float* S, const uint8_t* key_pad, int mask_mode, int B,
                               int H, int Tq,
                               int Tk, int ldt, float scale, float p_drop, uint32_t seed,
                               uint32_t salt, void* P, void* Pd, int dtype, void* stream) {
  if (B <= 0 || Tq <= 0) return 0;
  if (!S || !key_pad || !P || H <= 0 || Tk <= 0 || ldt < Tk) return FS2_EINVAL;
  const long nrows = (long)B * H * Tq;
  dim3 grid((unsigned)((nrows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FS2_BF16)
    hipLaunchKernelGGL(softmax_fwd_kernel<bf16>, grid, dim3(256), 0, s, S, key_pad, mask_mode != 0, B, H, Tq, Tk,
                       ldt, scale, p_drop, seed, salt, (bf16*)P, (bf16*)Pd, nrows);
  else if (dtype == FS2_F32)
    hipLaunchKernelGGL(softmax_fwd_kernel<float>, grid, dim3(256), 0, s, S, key_pad, mask_mode != 0, B, H, Tq, Tk,
                       ldt, scale, p_drop, seed, salt, (float*)P, (float*)Pd, nrows);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_softmax_bwd(const float* dPd, const void* P, int B, int H, int Tq, int Tk,
                               int ldt, float scale, float p_drop, uint32_t seed, uint32_t salt,
                               void* dS, int dtype, void* stream) {
  if (B <= 0 || Tq <= 0) return 0;
  if (!dPd || !P || !dS || ldt < Tk) return FS2_EINVAL;
  const long nrows = (long)B * H * Tq;
  dim3 grid((unsigned)((nrows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FS2_BF16)
    hipLaunchKernelGGL(softmax_bwd_kernel<bf16>, grid, dim3(256), 0, s, dPd, (const bf16*)P, Tk, ldt,
                       scale, p_drop, seed, salt, (bf16*)dS, nrows);
  else if (dtype == FS2_F32)
    hipLaunchKernelGGL(softmax_bwd_kernel<float>, grid, dim3(256), 0, s, dPd, (const float*)P, Tk,
                       ldt, scale, p_drop, seed, salt, (float*)dS, nrows);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}

// this translation unit's dropout seed base (fs2_common.h)
FS2_SEED_SETTER(fs2_seed_base_attention)
