// Generalised MFMA GEMM for gfx950 with implicit reflect-padded 1-D convolution.
//
// One kernel family serves every dense contraction of the FastSpeech2 train step
// (SURVEY.md op sites K4, K6-K8, K12, K13 and their backward K16):
//   fwd   Y = X W^T (+bias, ReLU, mask)        A = tokens (K-major, optional conv mode 1)
//   dgrad dX = dY W (+ReLU gate, +residual)     A = tokens (K-major, optional conv mode 2)
//   wgrad dW = dY^T X                           A, B token-major ("MN-major"), conv mode 3
//   attention bmm's (S = Q K^T, O = P V, dP, dQ, dK, dV) through the batch strides.
//
// Tile 128x128 per 256-thread workgroup (4 waves as 2x2, 64x64 per wave = 4x4 MFMA
// 16x16 tiles).  K-major operands are staged as [128 rows][128 bytes] with a 16-byte-chunk
// XOR swizzle (chunk ^= row & 7): conflict-free ds_read_b128 fragments.  MN-major operands
// (token-major activations in the weight-gradient GEMMs and the attention bmm's) are staged
// untransposed as [BK k-rows][128] and read through ds_read_b64_tr_b16, the gfx950 LDS
// transpose read, so no lane ever shuffles data.  bf16 uses v_mfma_f32_16x16x32_bf16, fp32 (parity
// mode) the exact-f32 v_mfma_f32_16x16x4_f32; both share the 16x16 C/D layout
// (col = lane&15, row = 4*(lane>>4) + r), so the epilogue is common.
// Register-staged double buffering: the next K-tile's global loads are in flight while
// the current tile's MFMAs run; one barrier per K-tile.
#include "fs2_common.h"

namespace {

constexpr int BM = 128, BN = 128, NT = 256;
constexpr int TILE_BYTES = 128 * 128;  // one operand, one stage

struct GemmP {
  int M, N, K, kvalid, mvalid, nvalid;
  const char* A; long lda; const char* B; long ldb;
  int conv_mode, conv_t, conv_kw, conv_c, conv_p;
  char* C; long ldc; int c_fp32; int c_conv_kw;
  const float* bias; int relu;
  const char* gate; long ldg;
  const float* row_scale;
  const char* residual; long ldr;
  const float* row_scale_post;
  int accumulate; int split_k; int k_per_split;
  int batch_div;
  long sA1, sA2, sB1, sB2, sC1, sC2, sR1, sR2;
  int tiles_m, tiles_n;
};

__device__ __forceinline__ u32x4 add_bf16x8(u32x4 a, u32x4 b) {
  u32x4 r;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    float a0 = __builtin_bit_cast(float, a[w] << 16), a1 = __builtin_bit_cast(float, a[w] & 0xffff0000u);
    float b0 = __builtin_bit_cast(float, b[w] << 16), b1 = __builtin_bit_cast(float, b[w] & 0xffff0000u);
    bf16 r0 = (bf16)(a0 + b0), r1 = (bf16)(a1 + b1);
    r[w] = (unsigned)__builtin_bit_cast(unsigned short, r0) |
           ((unsigned)__builtin_bit_cast(unsigned short, r1) << 16);
  }
  return r;
}
__device__ __forceinline__ u32x4 add_f32x4(u32x4 a, u32x4 b) {
  const f32x4 fa = __builtin_bit_cast(f32x4, a), fb = __builtin_bit_cast(f32x4, b);
  return __builtin_bit_cast(u32x4, fa + fb);
}

template <typename T>
struct Cfg {
  static constexpr int ES = sizeof(T);
  static constexpr int EPC = 16 / ES;   // elements per 16-byte chunk
  static constexpr int BK = 8 * EPC;    // 64 (bf16) / 32 (fp32): 128-byte LDS rows
};

__device__ __forceinline__ u32x4 ld16(const char* p) { return *(const u32x4*)p; }

// ---- K-major tile loader: rows [row0, row0+128), k in [k0, k0+BK) --------------------------
// thread handles chunks id = tid + 256 i : row = id >> 3, kc = id & 7
template <typename T>
__device__ __forceinline__ void load_kmajor(u32x4 (&st)[4], const char* base, long ld, int row0,
                                            int nrows, int k0, int kend, const GemmP& p,
                                            int cmode, const int (&rb)[4], const int (&rt)[4]) {
  constexpr int ES = Cfg<T>::ES, EPC = Cfg<T>::EPC;
  const int tid = threadIdx.x;
  const int kc = tid & 7;
  const int k = k0 + kc * EPC;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (tid >> 3) + 32 * i;
    const int row = row0 + r;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (row < nrows && k < kend) {
      if (cmode == 0) {
        v = ld16(base + ((long)row * ld + k) * ES);
      } else {
        const int C = p.conv_c, T_ = p.conv_t, P = p.conv_p;
        const int j = k / C, c = k - j * C;
        const int b = rb[i], t = rt[i];
        if (cmode == 1) {
          const int ts = reflect_idx(t + j - P, T_);
          v = ld16(base + ((long)(b * T_ + ts) * ld + c) * ES);
        } else {  // cmode == 2: transposed conv with reflect fold
          const int t1 = t - j + P;
          if (t1 >= 0 && t1 < T_) v = ld16(base + ((long)(b * T_ + t1) * ld + c) * ES);
          const int t2 = P - j - t;  // t2 + j - P = -t  (t >= 1)
          if (t >= 1 && t2 >= 0 && t2 < T_) {
            u32x4 w = ld16(base + ((long)(b * T_ + t2) * ld + c) * ES);
            v = (ES == 2) ? add_bf16x8(v, w) : add_f32x4(v, w);
          }
          const int t3 = 2 * (T_ - 1) - t - j + P;  // t3 + j - P = 2(T-1) - t  (t <= T-2)
          if (t <= T_ - 2 && t3 >= 0 && t3 < T_ && t3 + j - P >= T_) {
            u32x4 w = ld16(base + ((long)(b * T_ + t3) * ld + c) * ES);
            v = (ES == 2) ? add_bf16x8(v, w) : add_f32x4(v, w);
          }
        }
      }
    }
    st[i] = v;
  }
}

template <typename T>
__device__ __forceinline__ void store_kmajor(char* lds, const u32x4 (&st)[4]) {
  const int tid = threadIdx.x;
  const int kc = tid & 7;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (tid >> 3) + 32 * i;
    *(u32x4*)(lds + r * 128 + ((kc ^ (r & 7)) << 4)) = st[i];
  }
}

// ---- MN-major tile: LDS image [BK k-rows][128 mn] (row = 256 B bf16 / 512 B fp32) -------------
// Stored untransposed (16-byte chunks copied as loaded); bf16 fragments come out through the
// gfx950 hardware-transpose read ds_read_b64_tr_b16.  Chunk swizzle per k-row:
//   bf16: phys = c ^ (2*(k&3) + 8*((k>>3)&1))  -> the 8 rows one 32-lane half of a tr-read
//         touches land on 16 distinct 16-byte slots (conflict-free)
//   fp32: phys = c ^ (4*(k&1))                  -> ds_read_b32 rows k, k+1 on disjoint banks
template <typename T>
__device__ __forceinline__ int mn_swz(int k) {
  if constexpr (sizeof(T) == 2) return 2 * (k & 3) + 8 * ((k >> 3) & 1);
  else return 4 * (k & 1);
}

template <typename T>
__device__ __forceinline__ void load_mnmajor(u32x4 (&st)[4], const char* base, long ld, int mn0,
                                             int nmn, int k0, int kend, const GemmP& p,
                                             bool conv3) {
  constexpr int ES = Cfg<T>::ES, EPC = Cfg<T>::EPC;
  constexpr int CPR = 128 / EPC;  // chunks per k-row: 16 (bf16) / 32 (fp32)
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = tid + 256 * i;
    const int kr = id / CPR, c = id - kr * CPR;
    const int k = k0 + kr;
    const int mn = mn0 + c * EPC;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (k < kend && mn < nmn) {
      long srow = k;
      int col = mn;
      if (conv3) {
        const int j = mn / p.conv_c;
        col = mn - j * p.conv_c;
        const int b = k / p.conv_t, t = k - b * p.conv_t;
        srow = (long)b * p.conv_t + reflect_idx(t + j - p.conv_p, p.conv_t);
      }
      v = ld16(base + (srow * ld + col) * ES);
    }
    st[i] = v;
  }
}

template <typename T>
__device__ __forceinline__ void store_mnmajor(char* lds, const u32x4 (&st)[4]) {
  constexpr int EPC = Cfg<T>::EPC;
  constexpr int CPR = 128 / EPC, RB = 128 * sizeof(T);
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = tid + 256 * i;
    const int kr = id / CPR, c = id - kr * CPR;
    *(u32x4*)(lds + kr * RB + ((c ^ mn_swz<T>(kr)) << 4)) = st[i];
  }
}

// ---- fragment readers -------------------------------------------------------------------
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// bf16 16x16x32 operand, lane l: rows (mn) r0 + (l&15), k = s*32 + 8*(l>>4) + j, j = 0..7
__device__ __forceinline__ bf16x8 frag_bf16_kmajor(const char* lds, int r0, int s, int lane) {
  const int r = r0 + (lane & 15);
  const int ch = s * 4 + (lane >> 4);
  return *(const bf16x8*)(lds + r * 128 + ((ch ^ (r & 7)) << 4));
}
__device__ __forceinline__ bf16x8 frag_bf16_mnmajor(const char* lds, int r0, int s, int lane) {
  const int li = lane & 15, g = lane >> 4, q = li >> 2, p = li & 3;
  const int m = r0 + 4 * p;             // this lane supplies columns m..m+3 of k-row (.., q)
  const int c = m >> 3, boff = (m & 7) * 2;
  const int k1 = s * 32 + 8 * g + q, k2 = k1 + 4;
  const char* a1 = lds + k1 * 256 + ((c ^ mn_swz<bf16>(k1)) << 4) + boff;
  const char* a2 = lds + k2 * 256 + ((c ^ mn_swz<bf16>(k2)) << 4) + boff;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a2);
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// fp32 16x16x4 operand, lane l: row (mn) r0 + (l&15), k = s*4 + (l>>4)
__device__ __forceinline__ float frag_f32_kmajor(const char* lds, int r0, int s, int lane) {
  const int r = r0 + (lane & 15);
  return *(const float*)(lds + r * 128 + ((s ^ (r & 7)) << 4) + (lane >> 4) * 4);
}
__device__ __forceinline__ float frag_f32_mnmajor(const char* lds, int r0, int s, int lane) {
  const int m = r0 + (lane & 15), k = s * 4 + (lane >> 4);
  return *(const float*)(lds + k * 512 + (((m >> 2) ^ mn_swz<float>(k)) << 4) + (m & 3) * 4);
}

template <typename T, bool AK, bool BKM>
__global__ void __launch_bounds__(NT) gemm_kernel(GemmP p) {
  constexpr int ES = Cfg<T>::ES, BK = Cfg<T>::BK;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // tile coordinates (row-major over tiles so neighbouring blocks share the A panel)
  const int bid = blockIdx.x;
  const int tm = bid / p.tiles_n, tn = bid - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // batch / split-K
  int z = 0, kbeg = 0, kend = p.K;
  if (p.split_k > 1) {
    kbeg = blockIdx.z * p.k_per_split;
    kend = min(p.K, kbeg + p.k_per_split);
  } else {
    z = blockIdx.z;
  }
  const long zb = z / p.batch_div, zh = z - zb * p.batch_div;
  const char* Ab = p.A + (zb * p.sA1 + zh * p.sA2) * ES;
  const char* Bb = p.B + (zb * p.sB1 + zh * p.sB2) * ES;
  const int kvalid = p.kvalid;  // MN-major operand k-row bound

  // conv row coordinates for the K-major A loader (rows fixed per block)
  int rb[4] = {0, 0, 0, 0}, rt[4] = {0, 0, 0, 0};
  const int amode = (p.conv_mode == 1 || p.conv_mode == 2) ? p.conv_mode : 0;
  if (AK && amode) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + (tid >> 3) + 32 * i;
      rb[i] = row / p.conv_t;
      rt[i] = row - rb[i] * p.conv_t;
    }
  }
  const bool bconv3 = (p.conv_mode == 3);
  const int zero4[4] = {0, 0, 0, 0};

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 stA[4], stB[4];
  auto load_tiles = [&](int k0) {
    if constexpr (AK) load_kmajor<T>(stA, Ab, p.lda, m0, p.M, k0, kend, p, amode, rb, rt);
    else load_mnmajor<T>(stA, Ab, p.lda, m0, p.M, k0, min(kend, kvalid), p, false);
    if constexpr (BKM) load_kmajor<T>(stB, Bb, p.ldb, n0, p.N, k0, kend, p, 0, zero4, zero4);
    else load_mnmajor<T>(stB, Bb, p.ldb, n0, p.N, k0, min(kend, kvalid), p, bconv3);
  };
  auto store_tiles = [&](int stage) {
    char* la = smem + stage * 2 * TILE_BYTES;
    char* lb = la + TILE_BYTES;
    if constexpr (AK) store_kmajor<T>(la, stA); else store_mnmajor<T>(la, stA);
    if constexpr (BKM) store_kmajor<T>(lb, stB); else store_mnmajor<T>(lb, stB);
  };

  const int nk = (kend > kbeg) ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    load_tiles(kbeg);
    store_tiles(0);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int stage = kt & 1;
    if (kt + 1 < nk) load_tiles(kbeg + (kt + 1) * BK);
    const char* la = smem + stage * 2 * TILE_BYTES;
    const char* lb = la + TILE_BYTES;
    if constexpr (ES == 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          af[i] = AK ? frag_bf16_kmajor(la, wm * 64 + i * 16, s, lane)
                     : frag_bf16_mnmajor(la, wm * 64 + i * 16, s, lane);
          bfr[i] = BKM ? frag_bf16_kmajor(lb, wn * 64 + i * 16, s, lane)
                       : frag_bf16_mnmajor(lb, wn * 64 + i * 16, s, lane);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        float af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          af[i] = AK ? frag_f32_kmajor(la, wm * 64 + i * 16, s, lane)
                     : frag_f32_mnmajor(la, wm * 64 + i * 16, s, lane);
          bfr[i] = BKM ? frag_f32_kmajor(lb, wn * 64 + i * 16, s, lane)
                       : frag_f32_mnmajor(lb, wn * 64 + i * 16, s, lane);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) store_tiles(stage ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
  const int OES = p.c_fp32 ? 4 : ES;
  char* Cb = p.C + (zb * p.sC1 + zh * p.sC2) * OES;
  const char* Rb = p.residual ? p.residual + (zb * p.sR1 + zh * p.sR2) * ES : nullptr;
  const bool atomic = p.split_k > 1;
  const int cc = p.c_conv_kw > 0 ? p.N / p.c_conv_kw : 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
      if (m >= p.mvalid) continue;
      const float rs = p.row_scale ? p.row_scale[m] : 1.f;
      const float rs2 = p.row_scale_post ? p.row_scale_post[m] : 1.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + (lane & 15);
        if (n >= p.nvalid) continue;
        float v = acc[i][j][r];
        if (p.bias) v += p.bias[n];
        if (p.relu) v = fmaxf(v, 0.f);
        if (p.gate) v = (to_f(((const T*)p.gate)[(long)m * p.ldg + n]) > 0.f) ? v : 0.f;
        v *= rs;
        if (Rb) v += to_f(((const T*)Rb)[(long)m * p.ldr + n]);
        v *= rs2;
        long col = n;
        if (cc > 0) { const int jj = n / cc; col = (long)(n - jj * cc) * p.c_conv_kw + jj; }
        const long off = (long)m * p.ldc + col;
        if (p.c_fp32) {
          float* Cf = (float*)Cb;
          if (atomic) atomicAdd(Cf + off, v);
          else if (p.accumulate) Cf[off] += v;
          else Cf[off] = v;
        } else {
          ((T*)Cb)[off] = from_f<T>(v);
        }
      }
    }
  }
}

template <typename T>
int launch_gemm(const GemmP& p, int gz, hipStream_t s, int ak, int bk) {
  dim3 grid(p.tiles_m * p.tiles_n, 1, gz);
  if (ak && bk) hipLaunchKernelGGL((gemm_kernel<T, true, true>), grid, dim3(NT), 0, s, p);
  else if (ak && !bk) hipLaunchKernelGGL((gemm_kernel<T, true, false>), grid, dim3(NT), 0, s, p);
  else if (!ak && bk) hipLaunchKernelGGL((gemm_kernel<T, false, true>), grid, dim3(NT), 0, s, p);
  else hipLaunchKernelGGL((gemm_kernel<T, false, false>), grid, dim3(NT), 0, s, p);
  FS2_CHECK_LAUNCH();
  return 0;
}

bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }

}  // namespace

extern "C" int fs2_gemm(const fs2_gemm_desc* d, void* stream) {
  if (!d || d->M < 0 || d->N < 0 || d->K < 0) return FS2_EINVAL;
  if (d->M == 0 || d->N == 0) return 0;
  const int es = d->dtype == FS2_BF16 ? 2 : 4;
  const int epc = 16 / es;
  const int bk = 8 * epc;
  GemmP p{};
  p.M = d->M; p.N = d->N; p.K = d->K;
  p.kvalid = d->kvalid > 0 ? d->kvalid : d->K;
  p.mvalid = d->mvalid > 0 ? min(d->mvalid, d->M) : d->M;
  p.nvalid = d->nvalid > 0 ? min(d->nvalid, d->N) : d->N;
  p.A = (const char*)d->A; p.lda = d->lda; p.B = (const char*)d->B; p.ldb = d->ldb;
  p.conv_mode = d->conv_mode; p.conv_t = d->conv_t; p.conv_kw = d->conv_kw; p.conv_c = d->conv_c;
  p.conv_p = d->conv_kw > 0 ? (d->conv_kw - 1) / 2 : 0;
  p.C = (char*)d->C; p.ldc = d->ldc; p.c_fp32 = d->c_fp32; p.c_conv_kw = d->c_conv_kw;
  p.bias = d->bias; p.relu = d->relu;
  p.gate = (const char*)d->gate; p.ldg = d->ldg;
  p.row_scale = d->row_scale;
  p.residual = (const char*)d->residual; p.ldr = d->ldr;
  p.row_scale_post = d->row_scale_post;
  p.accumulate = d->accumulate;
  p.split_k = d->split_k > 1 ? d->split_k : 1;
  p.batch_div = d->batch_div > 0 ? d->batch_div : 1;
  p.sA1 = d->sA1; p.sA2 = d->sA2; p.sB1 = d->sB1; p.sB2 = d->sB2;
  p.sC1 = d->sC1; p.sC2 = d->sC2; p.sR1 = d->sR1; p.sR2 = d->sR2;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.N + BN - 1) / BN;
  const int batch = d->batch > 1 ? d->batch : 1;

  // ---- argument checks (host) ----
  if (!p.A || !p.B || !p.C) return FS2_EINVAL;
  if (p.K % epc) return FS2_EINVAL;
  if (!aligned16(p.A) || !aligned16(p.B)) return FS2_EALIGN;
  if ((p.lda % epc) || (p.ldb % epc)) return FS2_EALIGN;
  if ((batch > 1) && ((p.sA1 | p.sA2 | p.sB1 | p.sB2) % epc)) return FS2_EALIGN;
  if (!d->a_kmajor && (p.M % epc)) return FS2_EINVAL;
  if (!d->b_kmajor && (p.N % epc)) return FS2_EINVAL;
  if (p.conv_mode) {
    if (p.conv_t <= 0 || p.conv_kw <= 0 || p.conv_c <= 0 || (p.conv_c % epc)) return FS2_EINVAL;
    if (p.conv_p >= p.conv_t) return FS2_EINVAL;  // torch reflect pad needs pad < T
    if ((p.conv_mode == 1 || p.conv_mode == 2) && (!d->a_kmajor || p.K != p.conv_kw * p.conv_c))
      return FS2_EINVAL;
    if ((p.conv_mode == 1 || p.conv_mode == 2) && (p.M % p.conv_t)) return FS2_EINVAL;
    if (p.conv_mode == 3 && (d->b_kmajor || p.N != p.conv_kw * p.conv_c)) return FS2_EINVAL;
  }
  if (p.c_conv_kw > 0 && (p.N % p.c_conv_kw)) return FS2_EINVAL;
  if (p.split_k > 1) {
    if (!p.c_fp32 || batch > 1) return FS2_EINVAL;
    p.k_per_split = ((p.K + p.split_k - 1) / p.split_k + bk - 1) / bk * bk;
    p.split_k = (p.K + p.k_per_split - 1) / p.k_per_split;
  }
  if (p.accumulate && !p.c_fp32) return FS2_EINVAL;
  const int gz = p.split_k > 1 ? p.split_k : batch;
  hipStream_t s = (hipStream_t)stream;
  if (d->dtype == FS2_BF16) return launch_gemm<bf16>(p, gz, s, d->a_kmajor, d->b_kmajor);
  if (d->dtype == FS2_F32) return launch_gemm<float>(p, gz, s, d->a_kmajor, d->b_kmajor);
  return FS2_EINVAL;
}
