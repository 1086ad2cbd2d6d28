// Token-major -> channel-major images for the K-major weight-gradient GEMM (conv_mode 6).
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
#include "fs2_common.h"

namespace {

constexpr int TJ = 64, TC = 64;     // tile: 64 output columns (tokens) x 64 channels
constexpr int PITCH = 144;          // LDS row pitch in bytes: 64 channels (128 B) + 16

// grid (ceil(ncols / 64), ceil(C / 64)), 256 threads.  Load: thread -> (token row jr, 8-channel
// chunk ch), two passes of 32 rows, one 16-byte load each.  Store: thread -> (channel row cr,
// 8-token chunk jc), two passes of 32 rows, one 16-byte store each.
__global__ void __launch_bounds__(256) pad_transpose_kernel(const bf16* X, long ldx, int B, int T,
                                                            int C, int P, int reflect, bf16* out,
                                                            long ldo, int ncols) {
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
      if (c >= C || j >= ncols) continue;
      const unsigned short* col = (const unsigned short*)(tile + jc * 8 * PITCH) + cl;
      u32x4 w;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = (unsigned)col[(2 * e) * (PITCH / 2)] | ((unsigned)col[(2 * e + 1) * (PITCH / 2)] << 16);
      *(u32x4*)(out + (long)c * ldo + j) = w;
    }
  }
}

}  // namespace

extern "C" int fs2_pad_transpose(const void* X, int64_t ldx, int B, int T, int C, int P,
                                 int reflect, void* out, int64_t ldo, int ncols, int dtype,
                                 void* stream) {
  if (B <= 0 || T <= 0 || C <= 0) return 0;
  if (dtype != FS2_BF16 || !X || !out || P < 0 || (reflect && P >= T)) return FS2_EINVAL;
  if ((C % 8) || (ldx % 8) || (ldo % 8) || (ncols % 8) || ncols < (long)B * (T + 2 * P) ||
      ldo < ncols || ((uintptr_t)X & 15) || ((uintptr_t)out & 15))
    return FS2_EALIGN;
  dim3 grid((ncols + TJ - 1) / TJ, (C + TC - 1) / TC);
  hipLaunchKernelGGL(pad_transpose_kernel, grid, dim3(256), 0, (hipStream_t)stream,
                     (const bf16*)X, (long)ldx, B, T, C, P, reflect, (bf16*)out, (long)ldo, ncols);
  FS2_CHECK_LAUNCH();
  return 0;
}
