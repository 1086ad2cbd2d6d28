// Batch collate on the GPU: TextMelCollateWithAlignment
// (fastspeech2/dataset.py:62-133) as two scatter kernels over one packed upload.
//
// The host concatenates the B utterances of a batch (the dataset's per-item arrays, in the
// order they arrive) into packed buffers and uploads them once; `order[i]` is the item placed
// at batch row i (descending phoneme length, the collate's torch.sort), so the kernels write
// the padded, sorted tensors directly:
//   collate_phon_kernel   phoneme_padded, duration_padded (B, Tp) int64, zero padded
//   collate_frames_kernel per 64-frame tile of one row: the packed mel (80, T_u) channel-major
//                         tile goes through LDS so that both outputs are written coalesced:
//                         mel_padded (B, Tm, n_mels) (the collate's permute(0, 2, 1), here
//                         contiguous), pitch / energy (B, Tm), and
//                         rank_X (B, n_mels + 2, Tm) = cat(mel, pitch, energy) (:94,116-117)
// HBM-bound byte movement: 4 B x (2 n_mels + 4) per valid frame + the zero padding.
#include "fs2_common.h"

namespace {

__global__ void collate_phon_kernel(const int32_t* order, const int64_t* off,
                                    const int64_t* phon, const int64_t* dur, int B, int Tp,
                                    int64_t* phon_out, int64_t* dur_out, int64_t* in_len) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * Tp) return;
  const int b = (int)(i / Tp), p = (int)(i - (long)b * Tp);
  const int u = order[b];
  const long o0 = off[u], n = off[u + 1] - o0;
  const bool in = p < n;
  phon_out[i] = in ? phon[o0 + p] : 0;
  dur_out[i] = in ? dur[o0 + p] : 0;
  if (p == 0) in_len[b] = n;
}

constexpr int CT = 64;   // frames per tile

__global__ void __launch_bounds__(256) collate_frames_kernel(
    const int32_t* order, const int64_t* foff, const float* mel, const float* pitch,
    const float* energy, int B, int Tm, int NM, float* mel_out, float* pitch_out,
    float* energy_out, float* rank_out, int64_t* out_len) {
  __shared__ float tile[CT][129];   // [frame][channel], NM <= 128
  const int b = blockIdx.y, t0 = blockIdx.x * CT;
  const int u = order[b];
  const long f0 = foff[u];
  const int T = (int)(foff[u + 1] - f0);
  const float* mu = mel + f0 * NM;   // utterance u: (NM, T) channel-major
  const int NC = NM + 2;
  // rank_X rows: channel c, frames t0..t0+63 (coalesced along t); mel rows staged in LDS
  for (int i = threadIdx.x; i < NC * CT; i += blockDim.x) {
    const int c = i / CT, tl = i - c * CT, t = t0 + tl;
    if (t >= Tm) continue;
    float v = 0.f;
    if (t < T) v = c < NM ? mu[(long)c * T + t] : (c == NM ? pitch[f0 + t] : energy[f0 + t]);
    rank_out[((long)b * NC + c) * Tm + t] = v;
    if (c < NM) tile[tl][c] = v;
    else if (c == NM) pitch_out[(long)b * Tm + t] = v;
    else energy_out[(long)b * Tm + t] = v;
  }
  __syncthreads();
  // mel_padded rows: frame t, channels 0..NM-1 (coalesced along c)
  for (int i = threadIdx.x; i < CT * NM; i += blockDim.x) {
    const int tl = i / NM, c = i - tl * NM, t = t0 + tl;
    if (t < Tm) mel_out[((long)b * Tm + t) * NM + c] = tile[tl][c];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) out_len[b] = T;
}

inline unsigned nblk(long n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

extern "C" int fs2_collate_phonemes(const int32_t* order, const int64_t* offsets,
                                    const int64_t* phonemes, const int64_t* durations, int B,
                                    int Tp, int64_t* phoneme_padded, int64_t* duration_padded,
                                    int64_t* input_lengths, void* stream) {
  if ((long)B * Tp == 0) return 0;
  if (!order || !offsets || !phonemes || !durations || !phoneme_padded || !duration_padded ||
      !input_lengths)
    return FS2_EINVAL;
  hipLaunchKernelGGL(collate_phon_kernel, dim3(nblk((long)B * Tp)), dim3(256), 0,
                     (hipStream_t)stream, order, offsets, phonemes, durations, B, Tp,
                     phoneme_padded, duration_padded, input_lengths);
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_collate_frames(const int32_t* order, const int64_t* frame_offsets,
                                  const float* mel, const float* pitch, const float* energy,
                                  int B, int Tm, int n_mels, float* mel_padded,
                                  float* pitch_padded, float* energy_padded, float* rank_x,
                                  int64_t* output_lengths, void* stream) {
  if ((long)B * Tm == 0) return 0;
  if (!order || !frame_offsets || !mel || !pitch || !energy || !mel_padded || !pitch_padded ||
      !energy_padded || !rank_x || !output_lengths || n_mels < 1 || n_mels > 128)
    return FS2_EINVAL;
  hipLaunchKernelGGL(collate_frames_kernel, dim3((Tm + CT - 1) / CT, B), dim3(256), 0,
                     (hipStream_t)stream, order, frame_offsets, mel, pitch, energy, B, Tm,
                     n_mels, mel_padded, pitch_padded, energy_padded, rank_x, output_lengths);
  FS2_CHECK_LAUNCH();
  return 0;
}
