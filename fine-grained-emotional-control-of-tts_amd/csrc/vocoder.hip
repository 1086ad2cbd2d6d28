// HiFi-GAN generator forward (the reference's speechbrain HIFIGAN.decode_batch,
// fastspeech2/inference.py:60-63,85): the HBM-bound pieces around the GEMMs.
//
// The convolutions run on fs2_gemm: "same" reflect convs with dilation (conv_mode 1 +
// conv_dil), the stride-u transposed convs as 3-tap zero-padded polyphase convs (conv_mode 5,
// the u output phases stacked along N so the GEMM output [B*L][u*C] IS the upsampled
// [B*L*u][C] sequence), leaky-ReLU / tanh epilogues (act 3 / 4) and the resblock residual add.
// This file holds:
//   vocoder_input_kernel   mel (B, n_mels, T) fp32 -> rows X[B*(T+2 pad)][ldx] in the
//                          activation dtype with `pad` replicated frames each side
//                          (HifiganGenerator.inference: F.pad(c, (pad, pad), "replicate"))
//   lrelu_kernel           y = leaky_relu(x, slope) (ResBlock1: xt = F.leaky_relu(x, 0.1))
//   mean3_lrelu_kernel     y = leaky_relu(((a + b) + c) / 3, slope) (the generator's
//                          z_sum / num_kernels followed by the next stage's leaky ReLU)
#include "fs2_common.h"

namespace {

template <typename T>
__global__ void vocoder_input_kernel(const float* mel, int NM, int Tin, int pad, T* X, int ldx,
                                     long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int Tp = Tin + 2 * pad;
  const long row = i / ldx;
  const int c = (int)(i - row * ldx);
  const int b = (int)(row / Tp), t = (int)(row - (long)b * Tp);
  const int ts = min(max(t - pad, 0), Tin - 1);
  X[i] = from_f<T>(c < NM ? mel[((long)b * NM + c) * Tin + ts] : 0.f);
}

template <typename T>
__global__ void lrelu_kernel(const T* x, T* y, long n, float slope) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * Vec<T>::N;
  if (i >= n) return;
  float v[Vec<T>::N];
  vload<T>(v, x + i);
#pragma unroll
  for (int e = 0; e < Vec<T>::N; ++e) v[e] = v[e] >= 0.f ? v[e] : v[e] * slope;
  vstore<T>(y + i, v);
}

template <typename T>
__global__ void mean3_lrelu_kernel(const T* a, const T* b, const T* c, T* y, long n,
                                   float slope) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * Vec<T>::N;
  if (i >= n) return;
  float va[Vec<T>::N], vb[Vec<T>::N], vc[Vec<T>::N];
  vload<T>(va, a + i);
  vload<T>(vb, b + i);
  vload<T>(vc, c + i);
#pragma unroll
  for (int e = 0; e < Vec<T>::N; ++e) {
    const float m = ((va[e] + vb[e]) + vc[e]) / 3.f;
    va[e] = m >= 0.f ? m : m * slope;
  }
  vstore<T>(y + i, va);
}

inline unsigned nblk(long n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

extern "C" int fs2_vocoder_input(const float* mel, int B, int n_mels, int T, int pad, void* X,
                                 int ldx, int dtype, void* stream) {
  const long n = (long)B * (T + 2 * pad) * ldx;
  if (n == 0) return 0;
  if (!mel || !X || ldx < n_mels || T < 1 || pad < 0) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FS2_BF16)
    hipLaunchKernelGGL(vocoder_input_kernel<bf16>, dim3(nblk(n)), dim3(256), 0, s, mel, n_mels, T,
                       pad, (bf16*)X, ldx, n);
  else if (dtype == FS2_F32)
    hipLaunchKernelGGL(vocoder_input_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, mel, n_mels,
                       T, pad, (float*)X, ldx, n);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_leaky_relu(const void* x, void* y, int64_t n, float slope, int dtype,
                              void* stream) {
  if (n == 0) return 0;
  const int V = dtype == FS2_BF16 ? 8 : 4;
  if (!x || !y || (n % V) || ((uintptr_t)x & 15) || ((uintptr_t)y & 15)) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(nblk(n / V));
  if (dtype == FS2_BF16)
    hipLaunchKernelGGL(lrelu_kernel<bf16>, g, dim3(256), 0, s, (const bf16*)x, (bf16*)y, (long)n,
                       slope);
  else if (dtype == FS2_F32)
    hipLaunchKernelGGL(lrelu_kernel<float>, g, dim3(256), 0, s, (const float*)x, (float*)y,
                       (long)n, slope);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_mean3_leaky_relu(const void* a, const void* b, const void* c, void* y,
                                    int64_t n, float slope, int dtype, void* stream) {
  if (n == 0) return 0;
  const int V = dtype == FS2_BF16 ? 8 : 4;
  if (!a || !b || !c || !y || (n % V) || (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c |
                                            (uintptr_t)y) & 15))
    return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(nblk(n / V));
  if (dtype == FS2_BF16)
    hipLaunchKernelGGL(mean3_lrelu_kernel<bf16>, g, dim3(256), 0, s, (const bf16*)a,
                       (const bf16*)b, (const bf16*)c, (bf16*)y, (long)n, slope);
  else if (dtype == FS2_F32)
    hipLaunchKernelGGL(mean3_lrelu_kernel<float>, g, dim3(256), 0, s, (const float*)a,
                       (const float*)b, (const float*)c, (float*)y, (long)n, slope);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}
