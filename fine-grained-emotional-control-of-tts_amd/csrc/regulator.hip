// Token-axis data movement of the FastSpeech2 path: embedding + positional encoding,
// key-padding masks, speaker/intensity concat, LengthRegulator, average_over_durations,
// the pitch/energy embedding conv, predictor heads and small utilities.
//
// These are HBM-bound integer / gather / segment-reduction kernels (SURVEY K1-K3, K7,
// K9-K11): coalesced row copies, no MFMA.
#include "fs2_common.h"

namespace {

// N (a multiple of 4) fp32 values from a 16-byte aligned address
template <int N>
__device__ __forceinline__ void vload_f32(float* o, const float* src) {
#pragma unroll
  for (int q = 0; q < N / 4; ++q) vload(o + 4 * q, src + 4 * q);
}

// ---------------------------------------------------------------- embedding (K1, K2)
template <typename T>
__global__ void embed_fwd_kernel(const int64_t* tok, const float* table, const float* pe, int pad,
                                 int T_, int D, T* X, float* keep, long n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // n < 2^31 (host)
  if (i >= n) return;
  const int m = i / D;
  const int d = i - m * D;
  const int t = m % T_;
  const int64_t v = tok[m];
  const float k = (v != pad) ? 1.f : 0.f;
  X[i] = from_f<T>((table[v * D + d] + pe[(long)t * D + d]) * k);
  if (d == 0) keep[m] = k;
}

// Token-embedding backward, dtable[v] += sum_{m: tok[m] = v} dX[m] * keep[m], deterministic:
// grid (D/64 column chunks, EMB_CH token chunks), 4 waves; a wave walks its tokens in order and
// adds each row chunk (lane = column) to its own LDS accumulator row of the token's id; the 4
// wave accumulators are combined in a fixed order into part[chunk][v][64-column chunk], which
// embed_bwd_reduce_kernel sums over the chunks in order.  (One block per vocabulary id that
// rescanned every token took 68 us at M = 6400, V = 95.)  Vocabularies larger than the LDS
// accumulator take several id windows of EMB_VMAX, one per grid.z (ids v0 .. v0 + EMB_VMAX - 1).
constexpr int EMB_CH = 16, EMB_VMAX = 128;
template <typename T>
__global__ void __launch_bounds__(256) embed_bwd_kernel(const int64_t* tok, const T* dX,
                                                        const float* keep, int M, int D, int V,
                                                        float* part) {
  __shared__ float acc[4][EMB_VMAX][64];   // 128 KiB
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int d = blockIdx.x * 64 + lane;
  const int v0 = blockIdx.z * EMB_VMAX, vn = min(EMB_VMAX, V - v0);
  for (int i = threadIdx.x; i < 4 * EMB_VMAX * 64; i += 256) (&acc[0][0][0])[i] = 0.f;
  __syncthreads();
  const int per = (M + EMB_CH - 1) / EMB_CH;
  const int c0 = blockIdx.y * per, c1 = min(M, c0 + per);
  const int wper = (c1 - c0 + 3) / 4;
  const int m0 = c0 + w * wper, m1 = min(c1, m0 + wper);
  for (int m = m0; m < m1; ++m) {
    const int v = (int)tok[m] - v0;
    if (d < D && v >= 0 && v < vn) acc[w][v][lane] += to_f(dX[(long)m * D + d]) * keep[m];
  }
  __syncthreads();
  for (int v = w; v < vn; v += 4)
    if (d < D)
      part[((long)blockIdx.y * V + v0 + v) * D + d] =
          (acc[0][v][lane] + acc[1][v][lane]) + (acc[2][v][lane] + acc[3][v][lane]);
}
__global__ void embed_bwd_reduce_kernel(const float* part, int nch, long n, float* dtable) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int c = 0; c < nch; ++c) s += part[c * n + i];
  dtable[i] += s;
}

__global__ void keypad_tokens_kernel(const int64_t* tok, int pad, int M, uint8_t* kp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < M) kp[i] = tok[i] == pad;
}

__global__ void keypad_lengths_kernel(const int64_t* lens, int B, int T_, uint8_t* kp,
                                      float* keep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * T_) return;
  const int b = i / T_, t = i - b * T_;
  const bool valid = t < lens[b];
  kp[i] = !valid;
  if (keep) keep[i] = valid ? 1.f : 0.f;
}

// ---------------------------------------------------------------- concat (K7)
template <typename T>
__global__ void concat_fwd_kernel(const T* feats, const float* spk_table, const int64_t* spk,
                                  const float* inten, int T_, int D, int E, T* cat, int ldc,
                                  long n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // n < 2^31 (host)
  if (i >= n) return;
  const int m = i / ldc;
  const int c = i - m * ldc;
  const int b = m / T_;
  float v = 0.f;
  if (c < D) v = to_f(feats[m * D + c]);
  else if (c < 2 * D) v = spk_table[spk[b] * D + (c - D)];
  else if (c < 2 * D + E) v = inten ? inten[m * E + (c - 2 * D)] : 0.f;
  cat[i] = from_f<T>(v);
}

// stage 1: U[b][d] = sum_t dcat[b,t,D+d]   grid (B, D/64), 4 waves split t
template <typename T>
__global__ void __launch_bounds__(256) concat_bwd_utt_kernel(const T* dcat, int ldc, int T_, int D,
                                                             float* U) {
  __shared__ float red[4][64];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int d = blockIdx.y * 64 + lane;
  float s = 0.f;
  if (d < D)
    for (int t = w; t < T_; t += 4) s += to_f(dcat[((long)b * T_ + t) * ldc + D + d]);
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && d < D) U[(long)b * D + d] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}
// row-vector variant (wave per row, 16 B per lane; the element-wise kernel divides per element)
template <typename T>
__global__ void __launch_bounds__(256) concat_fwd_vec_kernel(const T* feats, const float* spk_table,
                                                             const int64_t* spk,
                                                             const float* inten, int T_, int D,
                                                             int E, T* cat, int ldc, int M) {
  constexpr int VN = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (m >= M) return;
  const float* srow = spk_table + spk[m / T_] * D;
  for (int c = lane * VN; c < ldc; c += 64 * VN) {
    float v[VN];
    if (c + VN <= D) {
      vload(v, feats + (long)m * D + c);
    } else if (c >= D && c + VN <= 2 * D) {
      vload_f32<VN>(v, srow + (c - D));
    } else {
#pragma unroll
      for (int k = 0; k < VN; ++k) {
        const int cc = c + k;
        float x = 0.f;
        if (cc < D) x = to_f(feats[(long)m * D + cc]);
        else if (cc < 2 * D) x = srow[cc - D];
        else if (cc < 2 * D + E) x = inten ? inten[(long)m * E + (cc - 2 * D)] : 0.f;
        v[k] = x;
      }
    }
    vstore(cat + (long)m * ldc + c, v);
  }
}

// The vectorised row reductions below (concat, predictor head, pitch/energy embedding
// backward) share one geometry: lane l of a wave owns the VN = 16 B / sizeof(T) adjacent
// columns c0 = (blockIdx.y * 64 + l) * VN, so one load instruction of a wave reads a
// 64 * VN-column row slab (1 KiB), blockIdx.y walks the slabs of a wider row and the waves of
// a block take rows round-robin; the waves' partial sums are combined through LDS in a fixed
// order.  The row index is wave-uniform (readfirstlane), so per-row scalars (dy, the tap
// values a[...]) are plain uniform loads.  The earlier one-column-per-lane versions (2 B
// loads, 32-64 dependent loads per lane) took 47-116 us in-step at M = 6400 (r06f trace).
template <typename T>
__device__ __forceinline__ void slab_combine_store(float (&red)[8][64 * Vec<T>::N], int nw,
                                                   float* dst, int D, int stride, int off) {
  // dst[col * stride + off] = fixed-order sum over the nw wave rows of red (nw = 4 or 8)
  constexpr int SC = 64 * Vec<T>::N;
  for (int i = threadIdx.x; i < SC; i += blockDim.x) {
    float s = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
    if (nw == 8) s += (red[4][i] + red[5][i]) + (red[6][i] + red[7][i]);
    const int c = (blockIdx.y * 64 + (i & 63)) * Vec<T>::N + (i >> 6);
    if (c < D) dst[(long)c * stride + off] = s;
  }
}

// stage 1 (vector): U[b][d] = sum_t dcat[b,t,D+d]; grid (B, slabs), 8 waves over t
template <typename T>
__global__ void __launch_bounds__(512) concat_bwd_utt_vec_kernel(const T* dcat, int ldc, int T_,
                                                                 int D, float* U) {
  constexpr int VN = Vec<T>::N;
  __shared__ float red[8][64 * VN];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c0 = (blockIdx.y * 64 + lane) * VN;
  float acc[VN];
#pragma unroll
  for (int k = 0; k < VN; ++k) acc[k] = 0.f;
  if (c0 < D) {
    const T* base = dcat + (long)blockIdx.x * T_ * ldc + D + c0;
#pragma unroll 4
    for (int t = wv; t < T_; t += 8) {
      float x[VN];
      vload(x, base + (long)t * ldc);
#pragma unroll
      for (int k = 0; k < VN; ++k) acc[k] += x[k];
    }
  }
#pragma unroll
  for (int k = 0; k < VN; ++k) red[wv][k * 64 + lane] = acc[k];
  __syncthreads();
  slab_combine_store<T>(red, 8, U + (long)blockIdx.x * D, D, 1, 0);
}

// stage 2: dspk[s][d] += sum_{b: spk[b]==s} U[b][d]  (utterance order)
__global__ void concat_bwd_spk_kernel(const float* U, const int64_t* spk, int B, int D, int n_spk,
                                      float* dspk) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_spk * D) return;
  const int s = i / D, d = i - s * D;
  float acc = 0.f;
  for (int b = 0; b < B; ++b)
    if (spk[b] == s) acc += U[(long)b * D + d];
  dspk[i] += acc;
}

template <typename T>
__global__ void mask_rows_kernel(T* X, long ldx, const float* keep, int M, int D) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // M * D < 2^31 (host)
  if (i >= M * D) return;
  const int m = i / D;
  const int d = i - m * D;
  T* p = X + (long)m * ldx + d;
  *p = from_f<T>(to_f(*p) * keep[m]);
}

// X = (X + Y + Z) * keep[row], summed in fp32 and rounded once (the aux-stream join of the
// three predictor input gradients)
template <typename T>
__global__ void add3_mask_rows_kernel(T* X, const T* Y, const T* Z, long ld, const float* keep,
                                      int M, int D) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // M * D < 2^31 (host)
  if (i >= M * D) return;
  const int m = i / D;
  const long o = (long)m * ld + (i - m * D);
  X[o] = from_f<T>(((to_f(X[o]) + to_f(Y[o])) + (Z ? to_f(Z[o]) : 0.f)) * keep[m]);
}

// ---------------------------------------------------------------- predictor head
template <typename T>
__global__ void __launch_bounds__(256) rowdot_fwd_kernel(const T* u, long ldu, const float* w,
                                                         const float* b, float scale, int M,
                                                         int D, T* y) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) s += to_f(u[(long)row * ldu + d]) * w[d];
  s = wave_sum(s);
  if (lane == 0) y[row] = from_f<T>((s + b[0]) * scale);
}

template <typename T>
__global__ void __launch_bounds__(256) rowdot_bwd_kernel(const T* dy, const T* u, long ldu,
                                                         const float* w, float scale, int M,
                                                         int D, T* du, float* part,
                                                         int rows_per_block) {
  // part: [nb][D+1] partial sums of dy*scale*u and dy*scale
  const int rbeg = blockIdx.x * rows_per_block, rend = min(M, rbeg + rows_per_block);
  for (int d = threadIdx.x; d <= D; d += blockDim.x) {
    float s = 0.f;
#pragma unroll 8
    for (int m = rbeg; m < rend; ++m) {
      const float g = to_f(dy[m]) * scale;
      s += (d < D) ? g * to_f(u[(long)m * ldu + d]) : g;
    }
    part[(long)blockIdx.x * (D + 1) + d] = s;
  }
  for (int m = rbeg; m < rend; ++m) {   // row-wise: no 64-bit division per element
    const float g = to_f(dy[m]) * scale;
    for (int d = threadIdx.x; d < D; d += blockDim.x) du[(long)m * D + d] = from_f<T>(g * w[d]);
  }
}

// vector variant: grid (row blocks, slabs), 4 waves; part as rowdot_bwd_kernel
template <typename T>
__global__ void __launch_bounds__(256) rowdot_bwd_vec_kernel(const T* dy, const T* u, long ldu,
                                                             const float* w, float scale, int M,
                                                             int D, T* du, float* part,
                                                             int rows_per_block) {
  constexpr int VN = Vec<T>::N, SC = 64 * VN;
  __shared__ float red[8][SC];
  __shared__ float gred[4];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c0 = (blockIdx.y * 64 + lane) * VN;
  const bool live = c0 < D;   // D % VN == 0 (host)
  const int rbeg = blockIdx.x * rows_per_block, rend = min(M, rbeg + rows_per_block);
  float wr[VN], acc[VN];
#pragma unroll
  for (int k = 0; k < VN; ++k) {
    wr[k] = live ? w[c0 + k] : 0.f;
    acc[k] = 0.f;
  }
  float gs = 0.f;
#pragma unroll 4
  for (int m = rbeg + wv; m < rend; m += 4) {
    const float g = to_f(dy[m]) * scale;
    gs += g;
    if (live) {
      float x[VN], o[VN];
      vload(x, u + (long)m * ldu + c0);
#pragma unroll
      for (int k = 0; k < VN; ++k) {
        acc[k] += g * x[k];
        o[k] = g * wr[k];
      }
      vstore(du + (long)m * D + c0, o);
    }
  }
#pragma unroll
  for (int k = 0; k < VN; ++k) red[wv][k * 64 + lane] = acc[k];
  if (lane == 0) gred[wv] = gs;
  __syncthreads();
  float* pp = part + (long)blockIdx.x * (D + 1);
  slab_combine_store<T>(red, 4, pp, D, 1, 0);
  if (blockIdx.y == 0 && threadIdx.x == 0) pp[D] = (gred[0] + gred[1]) + (gred[2] + gred[3]);
}

__global__ void __launch_bounds__(256) reduce_cols_kernel(const float* part, int nb, int N,
                                                          float* out, float* out2, int split) {
  // out[n] += sum_b part[b][n] for n < split; out2[n - split] += ... for n >= split.
  // 16 columns x 16 row-slices per block, fixed-order LDS combine (deterministic)
  __shared__ float red[16][17];
  const int c = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int n = blockIdx.x * 16 + c;
  float s = 0.f;
  if (n < N) {
#pragma unroll 4
    for (int b = sl; b < nb; b += 16) s += part[(long)b * N + n];
  }
  red[sl][c] = s;
  __syncthreads();
  if (sl == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][c];
    if (n < split) out[n] += t;
    else out2[n - split] += t;
  }
}

// ---------------------------------------------------------------- average_over_durations (K9)
// Replicates torch CPU semantics of SB average_over_durations (App. A.10): cumsum of the
// values accumulated in double and stored as float, cumsum of (values != 0) as int64,
// differences gathered at the duration cumsum ends/starts, float division.
//
// The double cumsum is order-sensitive only when an addition rounds.  Every partial sum of
// the row (in any grouping) is an integer multiple of 2^L, L = the lowest ulp exponent over
// the row's non-zero values, and at most S = sum |v| in magnitude; when S < 2^(L + 52) every
// such sum is exact in double (53-bit significand, one bit of margin for S's own rounding),
// so a parallel scan gives the sequential result bit for bit.  Rows that fail the test (a
// dynamic range beyond ~2^52 within one utterance, or a non-finite value) take the
// sequential scan by one thread, as torch does.  (The sequential scan alone took 35 us per
// call at B = 32, T_mel = 1000, r06f trace.)
__global__ void __launch_bounds__(256) avg_over_dur_kernel(const float* vals, int Tm,
                                                           const int64_t* durs, int Tp,
                                                           float* avg, float* vcum, int* nzcum) {
  __shared__ double sd[256];
  __shared__ int si[256];
  __shared__ int slo[256];
  __shared__ long long cs[1024 + 1];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* v = vals + (long)b * Tm;
  float* vc = vcum + (long)b * (Tm + 1);
  int* nc = nzcum + (long)b * (Tm + 1);
  // thread tid owns frames [i0, i1): row totals, |v| mass, lowest ulp exponent, non-finite flag
  const int R = (Tm + 255) / 256;
  const int i0 = min(Tm, tid * R), i1 = min(Tm, i0 + R);
  double s = 0.0, sabs = 0.0;
  int cnt = 0, lo = 1 << 20;
  for (int i = i0; i < i1; ++i) {
    const float x = v[i];
    const int e = (int)((__builtin_bit_cast(uint32_t, x) >> 23) & 0xffu);
    if (e == 255) lo = -(1 << 20);                        // inf / nan: force the fallback
    else if (x != 0.f) lo = min(lo, e ? e - 150 : -149);
    cnt += (x != 0.f);
    s += (double)x;
    sabs += fabs((double)x);
  }
  sd[tid] = sabs;
  slo[tid] = lo;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) { sd[tid] += sd[tid + o]; slo[tid] = min(slo[tid], slo[tid + o]); }
    __syncthreads();
  }
  const double S = sd[0];
  const int L = slo[0];
  const bool exact = L > -(1 << 19) && (L >= 1 << 19 || S < ldexp(1.0, min(L + 52, 1000)));
  __syncthreads();
  if (tid == 0) { vc[0] = 0.f; nc[0] = 0; }
  if (exact) {
    // inclusive Hillis-Steele scan of the per-thread totals (every partial sum exact)
    sd[tid] = s;
    si[tid] = cnt;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      const double ds = tid >= o ? sd[tid - o] : 0.0;
      const int di = tid >= o ? si[tid - o] : 0;
      __syncthreads();
      sd[tid] += ds;
      si[tid] += di;
      __syncthreads();
    }
    double acc = tid ? sd[tid - 1] : 0.0;
    int c = tid ? si[tid - 1] : 0;
    for (int i = i0; i < i1; ++i) {
      const float x = v[i];
      acc += (double)x;
      c += (x != 0.f);
      vc[i + 1] = (float)acc;
      nc[i + 1] = c;
    }
  } else if (tid == 0) {   // sequential: exact torch-CPU (double-accumulated) cumsum order
    double acc = 0.0;
    int c = 0;
    for (int i = 0; i < Tm; ++i) {
      const float x = v[i];
      acc += (double)x;
      c += (x != 0.f);
      vc[i + 1] = (float)acc;
      nc[i + 1] = c;
    }
  }
  // int64 duration cumsum (exact in any order): block scan, 256 threads x up to 4 phonemes
  __shared__ long long dpart[256];
  {
    const int Rp = (Tp + 255) / 256;
    const int q0 = min(Tp, tid * Rp), q1 = min(Tp, q0 + Rp);
    long long loc = 0;
    for (int p = q0; p < q1; ++p) loc += durs[(long)b * Tp + p];
    dpart[tid] = loc;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
      const long long add = tid >= o ? dpart[tid - o] : 0;
      __syncthreads();
      dpart[tid] += add;
      __syncthreads();
    }
    long long c = tid ? dpart[tid - 1] : 0;
    if (tid == 0) cs[0] = 0;
    for (int p = q0; p < q1; ++p) { c += durs[(long)b * Tp + p]; cs[p + 1] = c; }
  }
  __syncthreads();
  for (int p = tid; p < Tp; p += blockDim.x) {
    long long s0 = cs[p], s1 = cs[p + 1];
    s0 = s0 < 0 ? 0 : (s0 > Tm ? Tm : s0);
    s1 = s1 < 0 ? 0 : (s1 > Tm ? Tm : s1);
    const float sums = vc[s1] - vc[s0];
    const float nel = (float)(nc[s1] - nc[s0]);
    avg[(long)b * Tp + p] = (nel == 0.f) ? nel : sums / nel;
  }
}

// ---------------------------------------------------------------- pitch/energy embed (K10)
template <typename T>
__global__ void embed1d_fwd_kernel(const T* base, const float* a, const float* W, const float* bias,
                                   int T_, int D, int KW, T* out, long n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;   // n < 2^31 (host)
  if (i >= n) return;
  const int m = i / D;
  const int o = i - m * D;
  const int b = m / T_, t = m - b * T_;
  const int P = (KW - 1) / 2;
  float s = bias[o];
  for (int j = 0; j < KW; ++j) s += W[o * KW + j] * a[(long)b * T_ + reflect_idx(t + j - P, T_)];
  out[i] = from_f<T>(to_f(base[i]) + s);
}

// row-vector variant: a wave walks EMB1_ROWS consecutive rows with its lanes' weight / bias
// columns held in registers (one 16 B column vector per lane per sweep); the KW tap values
// of a row are wave-uniform loads.  (One row per wave re-read the D x KW weights per row:
// 24 us, slower than the element-wise kernel's 15.)
constexpr int EMB1_ROWS = 8;
template <typename T>
__global__ void __launch_bounds__(256) embed1d_fwd_vec_kernel(const T* base, const float* a,
                                                              const float* W, const float* bias,
                                                              int T_, int D, int KW, T* out,
                                                              int M) {
  constexpr int VN = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int m0 = (blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * EMB1_ROWS;
  if (m0 >= M) return;
  const int m1 = min(M, m0 + EMB1_ROWS);
  const int P = (KW - 1) / 2;
  for (int c = lane * VN; c < D; c += 64 * VN) {
    float w[8][VN], bs[VN];
#pragma unroll
    for (int k = 0; k < VN; ++k) {
      bs[k] = bias[c + k];
#pragma unroll
      for (int j = 0; j < 8; ++j) w[j][k] = j < KW ? W[(c + k) * KW + j] : 0.f;
    }
    for (int m = m0; m < m1; ++m) {
      const int b = m / T_, t = m - b * T_;
      float av[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) av[j] = j < KW ? a[(long)b * T_ + reflect_idx(t + j - P, T_)] : 0.f;
      float x[VN];
      vload(x, base + (long)m * D + c);
#pragma unroll
      for (int k = 0; k < VN; ++k) {
        float s = bs[k];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < KW) s += w[j][k] * av[j];
        x[k] = x[k] + s;
      }
      vstore(out + (long)m * D + c, x);
    }
  }
}

template <typename T>
__global__ void embed1d_bwd_kernel(const T* dout, const float* a, int M, int T_, int D, int KW,
                                   int rows_per_block, float* part) {
  // part: [nb][KW+1][D]
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= D) return;
  const int P = (KW - 1) / 2;
  const int rbeg = blockIdx.y * rows_per_block, rend = min(M, rbeg + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float ab = 0.f;
  for (int m = rbeg; m < rend; ++m) {
    const int b = m / T_, t = m - b * T_;
    const float g = to_f(dout[(long)m * D + o]);
    ab += g;
    for (int j = 0; j < KW && j < 8; ++j) acc[j] += g * a[(long)b * T_ + reflect_idx(t + j - P, T_)];
  }
  float* pp = part + (long)blockIdx.y * (KW + 1) * D;
  for (int j = 0; j < KW && j < 8; ++j) pp[(long)j * D + o] = acc[j];
  pp[(long)KW * D + o] = ab;
}

// vector variant: grid (row blocks, slabs), 8 waves; part [nb][KW*D + D] holds the dW partial
// at o*KW + j (dW's own layout) and the dbias partial at KW*D + o, so reduce_cols_kernel adds
// both in one pass
template <typename T>
__global__ void __launch_bounds__(512) embed1d_bwd_vec_kernel(const T* dout, const float* a, int M,
                                                              int T_, int D, int KW,
                                                              int rows_per_block, float* part) {
  constexpr int VN = Vec<T>::N;
  __shared__ float red[8][64 * VN];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c0 = (blockIdx.y * 64 + lane) * VN;
  const bool live = c0 < D;
  const int P = (KW - 1) / 2;
  const int rbeg = blockIdx.x * rows_per_block, rend = min(M, rbeg + rows_per_block);
  float acc[8][VN], ab[VN];
#pragma unroll
  for (int k = 0; k < VN; ++k) {
    ab[k] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j][k] = 0.f;
  }
#pragma unroll 2
  for (int m = rbeg + wv; m < rend; m += 8) {
    const int b = m / T_, t = m - b * T_;
    float x[VN];
    if (live) vload(x, dout + (long)m * D + c0);
    else {
#pragma unroll
      for (int k = 0; k < VN; ++k) x[k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < VN; ++k) ab[k] += x[k];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j < KW) {
        const float av = a[(long)b * T_ + reflect_idx(t + j - P, T_)];
#pragma unroll
        for (int k = 0; k < VN; ++k) acc[j][k] += x[k] * av;
      }
    }
  }
  float* pp = part + (long)blockIdx.x * (KW + 1) * D;
#pragma unroll
  for (int j = 0; j <= 8; ++j) {
    if (j <= KW) {   // block-uniform
      if (j) __syncthreads();   // the previous round's readers are done with red
#pragma unroll
      for (int k = 0; k < VN; ++k)
        red[wv][k * 64 + lane] = (j == KW) ? ab[k] : acc[j < 8 ? j : 7][k];
      __syncthreads();
      if (j == KW) slab_combine_store<T>(red, 8, pp + (long)KW * D, D, 1, 0);
      else slab_combine_store<T>(red, 8, pp, D, KW, j);
    }
  }
}

__global__ void embed1d_reduce_kernel(const float* part, int nb, int D, int KW, float* dW,
                                      float* dbias) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // i over (KW+1)*D
  if (i >= (KW + 1) * D) return;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) s += part[(long)b * (KW + 1) * D + i];
  const int j = i / D, o = i - j * D;
  if (j < KW) dW[o * KW + j] += s;
  else dbias[o] += s;
}

// ---------------------------------------------------------------- LengthRegulator (K11)
// durations -> frame counts -> int64 cumsum: an integer scan, exact in any order, so a block
// scan over 256 threads x up to 4 phonemes (T_p <= 1024) replaces the one-thread loop (18 us)
template <typename DT>
__global__ void __launch_bounds__(256) lr_index_kernel(const DT* durs, float pace, int Tp, int Tm,
                                                       int64_t* mel_len, int32_t* cum,
                                                       int32_t* frame_src) {
  const int b = blockIdx.x, tid = threadIdx.x;
  __shared__ int32_t cs[1024];
  __shared__ long long part[256];
  const int R = (Tp + 255) / 256;   // <= 4 (host: Tp <= 1024)
  const int p0 = min(Tp, tid * R), p1 = min(Tp, p0 + R);
  long long loc[4], sum = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    long long d = 0;
    if (p0 + k < p1) {
      // torch: (pace * durs).long() -- float32 product, truncation toward zero
      const float prod = pace * (float)durs[(long)b * Tp + p0 + k];
      d = (long long)prod;
    }
    loc[k] = d;
    sum += d;
  }
  part[tid] = sum;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const long long add = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += add;
    __syncthreads();
  }
  long long c = tid ? part[tid - 1] : 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (p0 + k < p1) {
      c += loc[k];
      cs[p0 + k] = (int32_t)c;
      cum[(long)b * Tp + p0 + k] = (int32_t)c;
    }
  }
  if (tid == 255) mel_len[b] = part[255];
  __syncthreads();
  if (!frame_src) return;  // lengths-only pass (host learns T_mel before sizing buffers)
  const int total = Tp > 0 ? cs[Tp - 1] : 0;
  for (int t = threadIdx.x; t < Tm; t += blockDim.x) {
    int src = -1;
    if (t < total) {  // first p with cs[p] > t (binary search)
      int lo = 0, hi = Tp - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cs[mid] > t) hi = mid; else lo = mid + 1;
      }
      src = lo;
    }
    frame_src[(long)b * Tm + t] = src;
  }
}

template <typename T>
__global__ void lr_gather_kernel(const T* X, const int32_t* fsrc, const float* pe, int Tp, int Tm,
                                 int D, T* Y, float* keep, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long m = i / D;
  const int d = (int)(i - m * D);
  const int b = (int)(m / Tm), t = (int)(m - (long)b * Tm);
  const int src = fsrc[m];
  float v = 0.f;
  if (src >= 0) v = to_f(X[((long)b * Tp + src) * D + d]) + pe[(long)t * D + d];
  Y[i] = from_f<T>(v);
  if (d == 0 && keep) keep[m] = src >= 0 ? 1.f : 0.f;
}

template <typename T>
__global__ void lr_scatter_kernel(const T* dY, const int32_t* cum, const float* keep, int Tp,
                                  int Tm, int D, T* dX) {
  const int bp = blockIdx.x;  // b*Tp + p
  const int b = bp / Tp, p = bp - b * Tp;
  int t0 = p > 0 ? cum[bp - 1] : 0, t1 = cum[bp];
  t0 = min(t0, Tm); t1 = min(t1, Tm);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int t = t0; t < t1; ++t) {
      const long m = (long)b * Tm + t;
      s += to_f(dY[m * D + d]) * keep[m];
    }
    dX[(long)bp * D + d] = from_f<T>(s);
  }
}

// Row-vector variants: one wave per frame row (gather) / phoneme row (scatter), 16 B per lane
// along the features, so the row index and its divisions are wave-uniform; same per-element
// arithmetic (and summation order) as the element-wise kernels above.  The element-wise gather
// spent most of its 28 us on two 64-bit divisions per element.
template <typename T>
__global__ void __launch_bounds__(256) lr_gather_vec_kernel(const T* X, const int32_t* fsrc,
                                                            const float* pe, int Tp, int Tm,
                                                            int D, T* Y, float* keep, int Mm) {
  constexpr int VN = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (m >= Mm) return;
  const int b = m / Tm, t = m - b * Tm;
  const int src = fsrc[m];
  const T* xr = X + ((long)b * Tp + (src >= 0 ? src : 0)) * D;
  const float* pr = pe + (long)t * D;
  T* yr = Y + (long)m * D;
  for (int c = lane * VN; c < D; c += 64 * VN) {
    float v[VN];
    if (src >= 0) {
      float p[VN];
      vload(v, xr + c);
      vload_f32<VN>(p, pr + c);
#pragma unroll
      for (int k = 0; k < VN; ++k) v[k] += p[k];
    } else {
#pragma unroll
      for (int k = 0; k < VN; ++k) v[k] = 0.f;
    }
    vstore(yr + c, v);
  }
  if (lane == 0 && keep) keep[m] = src >= 0 ? 1.f : 0.f;
}

template <typename T>
__global__ void __launch_bounds__(256) lr_scatter_vec_kernel(const T* dY, const int32_t* cum,
                                                             const float* keep, int Tp, int Tm,
                                                             int D, T* dX, int Mp) {
  constexpr int VN = Vec<T>::N;
  const int lane = threadIdx.x & 63;
  const int bp = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (bp >= Mp) return;
  const int b = bp / Tp, p = bp - b * Tp;
  int t0 = p > 0 ? cum[bp - 1] : 0, t1 = cum[bp];
  t0 = min(t0, Tm);
  t1 = min(t1, Tm);
  for (int c = lane * VN; c < D; c += 64 * VN) {
    float s[VN];
#pragma unroll
    for (int k = 0; k < VN; ++k) s[k] = 0.f;
    for (int t = t0; t < t1; ++t) {
      const long m = (long)b * Tm + t;
      const float kk = keep[m];
      float x[VN];
      vload(x, dY + m * D + c);
#pragma unroll
      for (int k = 0; k < VN; ++k) s[k] += x[k] * kk;
    }
    vstore(dX + (long)bp * D + c, s);
  }
}

// ---------------------------------------------------------------- utilities
template <typename T>
__global__ void fill_kernel(T* X, long n, float v) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) X[i] = from_f<T>(v);
}
template <typename T>
__global__ void add_kernel(T* X, const T* Y, long n, float alpha) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) X[i] = from_f<T>(to_f(X[i]) + alpha * to_f(Y[i]));
}
template <typename S, typename D>
__global__ void cast_kernel(const S* src, D* dst, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = from_f<D>(to_f(src[i]));
}

inline unsigned nblk(long n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

// every entry point dispatching through DISPATCH_T reports its own launch status (the macro
// ends in FS2_CHECK_LAUNCH), as do the entry points that launch directly
#define DISPATCH_T(dtype, KERNEL_CALL_BF16, KERNEL_CALL_F32) \
  do {                                                     \
    if ((dtype) == FS2_BF16) { KERNEL_CALL_BF16; }          \
    else if ((dtype) == FS2_F32) { KERNEL_CALL_F32; }       \
    else return FS2_EINVAL;                                 \
    FS2_CHECK_LAUNCH();                                     \
  } while (0)

// the vectorised row kernels: rows of D columns at a 16-byte aligned base and a
// row pitch of whole 16-byte vectors
static bool vec_rows_ok(int dtype, int D, long ld, const void* p0, const void* p1) {
  const int vn = dtype == FS2_BF16 ? 8 : 4;
  return D % vn == 0 && ld % vn == 0 && ((uintptr_t)p0 & 15) == 0 && ((uintptr_t)p1 & 15) == 0;
}
static int slabs(int dtype, int D) { const int sc = 64 * (dtype == FS2_BF16 ? 8 : 4); return (D + sc - 1) / sc; }


extern "C" int fs2_embed_fwd(const int64_t* tokens, const float* table, const float* pe,
                             int pad_idx, int B, int T, int D, void* X, float* keep, int dtype,
                             void* stream) {
  const long n = (long)B * T * D;
  if (n == 0) return 0;
  if (n >= 0x7fffffffL) return FS2_EINVAL;   // 32-bit element index
  if (!tokens || !table || !pe || !X || !keep) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(embed_fwd_kernel<bf16>, dim3(nblk(n)), dim3(256), 0, s, tokens, table, pe, pad_idx, T, D, (bf16*)X, keep, n),
    hipLaunchKernelGGL(embed_fwd_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, tokens, table, pe, pad_idx, T, D, (float*)X, keep, n));
  return 0;
}

extern "C" int64_t fs2_embed_bwd_workspace_floats(int D, int V) {
  return (int64_t)EMB_CH * V * D;
}

extern "C" int fs2_embed_bwd(const int64_t* tokens, const void* dX, const float* keep, int M,
                             int D, int V, float* dtable, float* workspace, int dtype,
                             void* stream) {
  if (M == 0 || V == 0) return 0;
  if (!tokens || !dX || !keep || !dtable || !workspace || V < 0) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((D + 63) / 64, EMB_CH, (V + EMB_VMAX - 1) / EMB_VMAX);
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(embed_bwd_kernel<bf16>, grid, dim3(256), 0, s, tokens, (const bf16*)dX, keep, M, D, V, workspace),
    hipLaunchKernelGGL(embed_bwd_kernel<float>, grid, dim3(256), 0, s, tokens, (const float*)dX, keep, M, D, V, workspace));
  const long n = (long)V * D;
  hipLaunchKernelGGL(embed_bwd_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     workspace, EMB_CH, n, dtable);
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_keypad_from_tokens(const int64_t* tokens, int pad_idx, int M, uint8_t* key_pad,
                                      void* stream) {
  if (M == 0) return 0;
  if (!tokens || !key_pad) return FS2_EINVAL;
  hipLaunchKernelGGL(keypad_tokens_kernel, dim3(nblk(M)), dim3(256), 0, (hipStream_t)stream,
                     tokens, pad_idx, M, key_pad);
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_keypad_from_lengths(const int64_t* lens, int B, int T, uint8_t* key_pad,
                                       float* keep, void* stream) {
  if (B * T == 0) return 0;
  if (!lens || !key_pad) return FS2_EINVAL;
  hipLaunchKernelGGL(keypad_lengths_kernel, dim3(nblk((long)B * T)), dim3(256), 0,
                     (hipStream_t)stream, lens, B, T, key_pad, keep);
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_concat_fwd(const void* feats, const float* spk_table, const int64_t* spk,
                              const float* intensity, int B, int T, int D, int E, void* cat,
                              int ldc, int dtype, void* stream) {
  const long n = (long)B * T * ldc;
  if (n == 0) return 0;
  if (n >= 0x7fffffffL) return FS2_EINVAL;   // 32-bit element index
  if (!feats || !spk_table || !spk || !cat || ldc < 2 * D + E) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (vec_rows_ok(dtype, D, ldc, feats, cat) && ((uintptr_t)spk_table & 15) == 0) {
    const int M = B * T;
    DISPATCH_T(dtype,
      hipLaunchKernelGGL(concat_fwd_vec_kernel<bf16>, dim3((M + 3) / 4), dim3(256), 0, s, (const bf16*)feats, spk_table, spk, intensity, T, D, E, (bf16*)cat, ldc, M),
      hipLaunchKernelGGL(concat_fwd_vec_kernel<float>, dim3((M + 3) / 4), dim3(256), 0, s, (const float*)feats, spk_table, spk, intensity, T, D, E, (float*)cat, ldc, M));
    return 0;
  }
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(concat_fwd_kernel<bf16>, dim3(nblk(n)), dim3(256), 0, s, (const bf16*)feats, spk_table, spk, intensity, T, D, E, (bf16*)cat, ldc, n),
    hipLaunchKernelGGL(concat_fwd_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, (const float*)feats, spk_table, spk, intensity, T, D, E, (float*)cat, ldc, n));
  return 0;
}

extern "C" int fs2_concat_bwd_spk(const void* dcat, int ldc, const int64_t* spk, int B, int T,
                                  int D, int n_spk, float* dspk, int dtype, float* workspace,
                                  void* stream) {
  if (n_spk == 0 || D == 0 || B == 0) return 0;
  if (!dcat || !spk || !dspk || !workspace) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (vec_rows_ok(dtype, D, ldc, dcat, (const char*)dcat + (long)D * (dtype == FS2_BF16 ? 2 : 4))) {
    dim3 grid(B, slabs(dtype, D));
    DISPATCH_T(dtype,
      hipLaunchKernelGGL(concat_bwd_utt_vec_kernel<bf16>, grid, dim3(512), 0, s, (const bf16*)dcat, ldc, T, D, workspace),
      hipLaunchKernelGGL(concat_bwd_utt_vec_kernel<float>, grid, dim3(512), 0, s, (const float*)dcat, ldc, T, D, workspace));
    hipLaunchKernelGGL(concat_bwd_spk_kernel, dim3(nblk((long)n_spk * D)), dim3(256), 0, s,
                       workspace, spk, B, D, n_spk, dspk);
    FS2_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid(B, (D + 63) / 64);
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(concat_bwd_utt_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)dcat, ldc, T, D, workspace),
    hipLaunchKernelGGL(concat_bwd_utt_kernel<float>, grid, dim3(256), 0, s, (const float*)dcat, ldc, T, D, workspace));
  hipLaunchKernelGGL(concat_bwd_spk_kernel, dim3(nblk((long)n_spk * D)), dim3(256), 0, s, workspace,
                     spk, B, D, n_spk, dspk);
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_mask_rows(void* X, int64_t ldx, const float* keep, int M, int D, int dtype,
                             void* stream) {
  const long n = (long)M * D;
  if (n == 0) return 0;
  if (n >= 0x7fffffffL) return FS2_EINVAL;   // 32-bit element index
  if (!X || !keep) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(mask_rows_kernel<bf16>, dim3(nblk(n)), dim3(256), 0, s, (bf16*)X, ldx, keep, M, D),
    hipLaunchKernelGGL(mask_rows_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, (float*)X, ldx, keep, M, D));
  return 0;
}

extern "C" int fs2_add3_mask_rows(void* X, const void* Y, const void* Z, int64_t ld,
                                  const float* keep, int M, int D, int dtype, void* stream) {
  const long n = (long)M * D;
  if (n == 0) return 0;
  if (n >= 0x7fffffffL) return FS2_EINVAL;   // 32-bit element index
  if (!X || !Y || !keep) return FS2_EINVAL;   // Z may be null (a two-term sum)
  hipStream_t s = (hipStream_t)stream;
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(add3_mask_rows_kernel<bf16>, dim3(nblk(n)), dim3(256), 0, s, (bf16*)X, (const bf16*)Y, (const bf16*)Z, ld, keep, M, D),
    hipLaunchKernelGGL(add3_mask_rows_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, (float*)X, (const float*)Y, (const float*)Z, ld, keep, M, D));
  return 0;
}

extern "C" int fs2_rowdot_fwd(const void* u, int64_t ldu, const float* w, const float* b,
                              float scale, int M, int D, void* y, int dtype, void* stream) {
  if (M == 0) return 0;
  if (!u || !w || !b || !y) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((M + 3) / 4);
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(rowdot_fwd_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)u, ldu, w, b, scale, M, D, (bf16*)y),
    hipLaunchKernelGGL(rowdot_fwd_kernel<float>, grid, dim3(256), 0, s, (const float*)u, ldu, w, b, scale, M, D, (float*)y));
  return 0;
}

extern "C" int fs2_rowdot_bwd(const void* dy, const void* u, int64_t ldu, const float* w,
                              float scale, int M, int D, void* du, float* dw, float* db,
                              int dtype, float* workspace, void* stream) {
  if (M == 0) return 0;
  if (!dy || !u || !w || !du || !dw || !db || !workspace) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int nb = min(256, max(1, (M + 31) / 32));
  const int rpb = (M + nb - 1) / nb;
  if (vec_rows_ok(dtype, D, ldu, u, du)) {
    dim3 grid(nb, slabs(dtype, D));
    DISPATCH_T(dtype,
      hipLaunchKernelGGL(rowdot_bwd_vec_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)dy, (const bf16*)u, ldu, w, scale, M, D, (bf16*)du, workspace, rpb),
      hipLaunchKernelGGL(rowdot_bwd_vec_kernel<float>, grid, dim3(256), 0, s, (const float*)dy, (const float*)u, ldu, w, scale, M, D, (float*)du, workspace, rpb));
  } else {
    DISPATCH_T(dtype,
    hipLaunchKernelGGL(rowdot_bwd_kernel<bf16>, dim3(nb), dim3(256), 0, s, (const bf16*)dy, (const bf16*)u, ldu, w, scale, M, D, (bf16*)du, workspace, rpb),
    hipLaunchKernelGGL(rowdot_bwd_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)dy, (const float*)u, ldu, w, scale, M, D, (float*)du, workspace, rpb));
  }
  hipLaunchKernelGGL(reduce_cols_kernel, dim3((D + 1 + 15) / 16), dim3(256), 0, s, workspace, nb,
                     D + 1, dw, db, D);
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t fs2_avg_workspace_floats(int B, int Tm_in) { return 2L * B * (Tm_in + 1); }

extern "C" int fs2_avg_over_durations(const float* values, int Tm_in, const int64_t* durs, int B,
                                      int Tp, float* avg, float* workspace, void* stream) {
  if (B == 0 || Tp == 0) return 0;
  if (!values || !durs || !avg || !workspace || Tp > 1024) return FS2_EINVAL;
  float* vcum = workspace;
  int* nzc = (int*)(workspace + (long)B * (Tm_in + 1));
  hipLaunchKernelGGL(avg_over_dur_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream, values,
                     Tm_in, durs, Tp, avg, vcum, nzc);
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_embed1d_fwd(const void* base, const float* a, const float* W,
                               const float* bias, int B, int T, int D, int KW, void* out,
                               int dtype, void* stream) {
  const long n = (long)B * T * D;
  if (n == 0) return 0;
  if (n >= 0x7fffffffL) return FS2_EINVAL;   // 32-bit element index
  if (!base || !a || !W || !bias || !out || KW > 8 || (KW - 1) / 2 >= T) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (vec_rows_ok(dtype, D, D, base, out)) {
    const int M = B * T;
    DISPATCH_T(dtype,
      hipLaunchKernelGGL(embed1d_fwd_vec_kernel<bf16>, dim3((M + 4 * EMB1_ROWS - 1) / (4 * EMB1_ROWS)), dim3(256), 0, s, (const bf16*)base, a, W, bias, T, D, KW, (bf16*)out, M),
      hipLaunchKernelGGL(embed1d_fwd_vec_kernel<float>, dim3((M + 4 * EMB1_ROWS - 1) / (4 * EMB1_ROWS)), dim3(256), 0, s, (const float*)base, a, W, bias, T, D, KW, (float*)out, M));
    return 0;
  }
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(embed1d_fwd_kernel<bf16>, dim3(nblk(n)), dim3(256), 0, s, (const bf16*)base, a, W, bias, T, D, KW, (bf16*)out, n),
    hipLaunchKernelGGL(embed1d_fwd_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, (const float*)base, a, W, bias, T, D, KW, (float*)out, n));
  return 0;
}

extern "C" int fs2_embed1d_bwd(const void* dout, const float* a, int B, int T, int D, int KW,
                               float* dW, float* dbias, int dtype, float* workspace,
                               void* stream) {
  const int M = B * T;
  if (M == 0) return 0;
  if (!dout || !a || !dW || !dbias || !workspace || KW > 8) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int nb = min(128, max(1, (M + 63) / 64));
  const int rpb = (M + nb - 1) / nb;
  if (vec_rows_ok(dtype, D, D, dout, dout)) {
    DISPATCH_T(dtype,
      hipLaunchKernelGGL(embed1d_bwd_vec_kernel<bf16>, dim3(nb, slabs(dtype, D)), dim3(512), 0, s, (const bf16*)dout, a, M, T, D, KW, rpb, workspace),
      hipLaunchKernelGGL(embed1d_bwd_vec_kernel<float>, dim3(nb, slabs(dtype, D)), dim3(512), 0, s, (const float*)dout, a, M, T, D, KW, rpb, workspace));
    hipLaunchKernelGGL(reduce_cols_kernel, dim3(((KW + 1) * D + 15) / 16), dim3(256), 0, s,
                       workspace, nb, (KW + 1) * D, dW, dbias, KW * D);
    FS2_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid((D + 255) / 256, nb);
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(embed1d_bwd_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)dout, a, M, T, D, KW, rpb, workspace),
    hipLaunchKernelGGL(embed1d_bwd_kernel<float>, grid, dim3(256), 0, s, (const float*)dout, a, M, T, D, KW, rpb, workspace));
  hipLaunchKernelGGL(embed1d_reduce_kernel, dim3(nblk((long)(KW + 1) * D)), dim3(256), 0, s,
                     workspace, nb, D, KW, dW, dbias);
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_lr_index(const void* durs, int d_is_float, float pace, int B, int Tp, int Tm,
                            int64_t* mel_len, int32_t* cum, int32_t* frame_src, void* stream) {
  if (B == 0) return 0;
  if (!durs || !mel_len || !cum || Tp > 1024 || Tp <= 0) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (d_is_float)
    hipLaunchKernelGGL(lr_index_kernel<float>, dim3(B), dim3(256), 0, s, (const float*)durs, pace,
                       Tp, Tm, mel_len, cum, frame_src);
  else
    hipLaunchKernelGGL(lr_index_kernel<int64_t>, dim3(B), dim3(256), 0, s, (const int64_t*)durs,
                       pace, Tp, Tm, mel_len, cum, frame_src);
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_lr_gather(const void* X, const int32_t* frame_src, const float* pe, int B,
                             int Tp, int Tm, int D, void* Y, float* keep, int dtype,
                             void* stream) {
  const long n = (long)B * Tm * D;
  if (n == 0) return 0;
  if (!X || !frame_src || !pe || !Y) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const long Mm = (long)B * Tm;
  if (Mm < 0x7fffffffL && vec_rows_ok(dtype, D, D, X, Y) && ((uintptr_t)pe & 15) == 0) {
    DISPATCH_T(dtype,
      hipLaunchKernelGGL(lr_gather_vec_kernel<bf16>, dim3((Mm + 3) / 4), dim3(256), 0, s, (const bf16*)X, frame_src, pe, Tp, Tm, D, (bf16*)Y, keep, (int)Mm),
      hipLaunchKernelGGL(lr_gather_vec_kernel<float>, dim3((Mm + 3) / 4), dim3(256), 0, s, (const float*)X, frame_src, pe, Tp, Tm, D, (float*)Y, keep, (int)Mm));
    return 0;
  }
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(lr_gather_kernel<bf16>, dim3(nblk(n)), dim3(256), 0, s, (const bf16*)X, frame_src, pe, Tp, Tm, D, (bf16*)Y, keep, n),
    hipLaunchKernelGGL(lr_gather_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, (const float*)X, frame_src, pe, Tp, Tm, D, (float*)Y, keep, n));
  return 0;
}

extern "C" int fs2_lr_scatter(const void* dY, const int32_t* cum, const float* keep, int B,
                              int Tp, int Tm, int D, void* dX, int dtype, void* stream) {
  if ((long)B * Tp == 0) return 0;
  if (!dY || !cum || !keep || !dX) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  if (vec_rows_ok(dtype, D, D, dY, dX)) {
    const int Mp = B * Tp;
    DISPATCH_T(dtype,
      hipLaunchKernelGGL(lr_scatter_vec_kernel<bf16>, dim3((Mp + 3) / 4), dim3(256), 0, s, (const bf16*)dY, cum, keep, Tp, Tm, D, (bf16*)dX, Mp),
      hipLaunchKernelGGL(lr_scatter_vec_kernel<float>, dim3((Mp + 3) / 4), dim3(256), 0, s, (const float*)dY, cum, keep, Tp, Tm, D, (float*)dX, Mp));
    return 0;
  }
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(lr_scatter_kernel<bf16>, dim3(B * Tp), dim3(128), 0, s, (const bf16*)dY, cum, keep, Tp, Tm, D, (bf16*)dX),
    hipLaunchKernelGGL(lr_scatter_kernel<float>, dim3(B * Tp), dim3(128), 0, s, (const float*)dY, cum, keep, Tp, Tm, D, (float*)dX));
  return 0;
}

extern "C" int fs2_fill(void* X, int64_t n, float value, int dtype, void* stream) {
  if (n == 0) return 0;
  if (!X) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(fill_kernel<bf16>, dim3(nblk(n)), dim3(256), 0, s, (bf16*)X, (long)n, value),
    hipLaunchKernelGGL(fill_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, (float*)X, (long)n, value));
  return 0;
}

extern "C" int fs2_add(void* X, const void* Y, int64_t n, float alpha, int dtype, void* stream) {
  if (n == 0) return 0;
  if (!X || !Y) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  DISPATCH_T(dtype,
    hipLaunchKernelGGL(add_kernel<bf16>, dim3(nblk(n)), dim3(256), 0, s, (bf16*)X, (const bf16*)Y, (long)n, alpha),
    hipLaunchKernelGGL(add_kernel<float>, dim3(nblk(n)), dim3(256), 0, s, (float*)X, (const float*)Y, (long)n, alpha));
  return 0;
}

extern "C" int fs2_cast(const void* src, int src_dtype, void* dst, int dst_dtype, int64_t n,
                        void* stream) {
  if (n == 0) return 0;
  if (!src || !dst) return FS2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(nblk(n)), b(256);
  if (src_dtype == FS2_F32 && dst_dtype == FS2_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16>), g, b, 0, s, (const float*)src, (bf16*)dst, (long)n);
  else if (src_dtype == FS2_BF16 && dst_dtype == FS2_F32)
    hipLaunchKernelGGL((cast_kernel<bf16, float>), g, b, 0, s, (const bf16*)src, (float*)dst, (long)n);
  else if (src_dtype == FS2_F32 && dst_dtype == FS2_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), g, b, 0, s, (const float*)src, (float*)dst, (long)n);
  else if (src_dtype == FS2_BF16 && dst_dtype == FS2_BF16)
    hipLaunchKernelGGL((cast_kernel<bf16, bf16>), g, b, 0, s, (const bf16*)src, (bf16*)dst, (long)n);
  else return FS2_EINVAL;
  FS2_CHECK_LAUNCH();
  return 0;
}

int fs2_seed_base_norm(uint32_t v, void* stream);
int fs2_seed_base_attention(uint32_t v, void* stream);
int fs2_seed_base_flash(uint32_t v, void* stream);

extern "C" int fs2_set_dropout_seed(uint32_t seed_base, void* stream) {
  if (int rc = fs2_seed_base_norm(seed_base, stream)) return rc;
  if (int rc = fs2_seed_base_attention(seed_base, stream)) return rc;
  return fs2_seed_base_flash(seed_base, stream);
}

extern "C" const char* fs2_version(void) { return "fs2_hip 0.1 gfx950"; }
