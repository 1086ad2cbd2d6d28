/*
 * CPU oracle (TEST INFRASTRUCTURE ONLY) for the integer / prefix-sum parts of the path:
 *
 *  - fs2o_lr_index: SB upsample's index expansion (model.py:406-410):
 *      n[b,p] = (int64)((float)pace * (float)d[b,p])    (torch: (pace*durs).long())
 *      repeat_interleave(arange(Tp), n) -> frame_src, padded with -1; mel_len = sum n
 *  - fs2o_avg_over_durations: SB average_over_durations (App. A.10; model.py:383,397) with
 *      torch-CPU cumsum semantics (double accumulation, float storage), non-zero counting.
 *
 * Plain C restatement; the product kernels in csrc/regulator.hip must match it bit-exactly.
 */
#include <stdint.h>

int fs2o_lr_index(const int64_t* durs, const float* durs_f, float pace, int B, int Tp, int Tm,
                  int64_t* mel_len, int32_t* frame_src) {
  for (int b = 0; b < B; ++b) {
    int64_t t = 0;
    for (int p = 0; p < Tp; ++p) {
      const float d = durs ? (float)durs[(int64_t)b * Tp + p] : durs_f[(int64_t)b * Tp + p];
      const int64_t n = (int64_t)(pace * d);
      for (int64_t k = 0; k < n; ++k, ++t)
        if (t < Tm) frame_src[(int64_t)b * Tm + t] = p;
    }
    mel_len[b] = t;
    for (int64_t k = t; k < Tm; ++k) frame_src[(int64_t)b * Tm + k] = -1;
  }
  return 0;
}

int fs2o_avg_over_durations(const float* values, int Tm, const int64_t* durs, int B, int Tp,
                            float* avg) {
  for (int b = 0; b < B; ++b) {
    /* prefix sums over frames: vc[t] = float(sum_{<t} v) (double accumulated), nc[t] = count */
    double acc = 0.0;
    int64_t cnt = 0;
    int64_t s0 = 0;
    float vc_prev = 0.f;
    int64_t nc_prev = 0;
    int64_t tpos = 0;
    /* walk phonemes in order; gather cumsums at segment ends */
    for (int p = 0; p < Tp; ++p) {
      const int64_t s1 = s0 + durs[(int64_t)b * Tp + p];
      int64_t e = s1 > Tm ? Tm : s1;
      while (tpos < e) {
        const float v = values[(int64_t)b * Tm + tpos];
        acc += (double)v;
        cnt += (v != 0.f);
        ++tpos;
      }
      const float vc_e = (float)acc;
      const int64_t nc_e = cnt;
      const float sums = vc_e - vc_prev;
      const float nel = (float)(nc_e - nc_prev);
      avg[(int64_t)b * Tp + p] = (nel == 0.f) ? nel : sums / nel;
      vc_prev = vc_e;
      nc_prev = nc_e;
      s0 = s1;
    }
  }
  return 0;
}
