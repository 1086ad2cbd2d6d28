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
#include <type_traits>

#include "fs2_common.h"

#include <cstdlib>
#include <cstring>

typedef __attribute__((ext_vector_type(4))) int i32x4;
__device__ void llvm_raw_buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) uint32_t* lds,
                                         int size, int voffset, int soffset, int offset,
                                         int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

namespace {

// Measurement switches (FS2_* environment variables and the g4_flags timing bits, some of
// which produce WRONG results on purpose) exist only in a build with -DFS2_EXPERIMENTS, the
// one tools/ A/B runs use; the product library compiles them to their defaults.
#ifdef FS2_EXPERIMENTS
bool getenv_flag(const char* name) {
  const char* v = std::getenv(name);
  return v && v[0] && std::strcmp(v, "0") != 0;
}
int getenv_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v ? std::atoi(v) : dflt;
}
#define XFLAGS(p) ((p).g4_flags)
#else
constexpr bool getenv_flag(const char*) { return false; }
constexpr int getenv_int(const char*, int dflt) { return dflt; }
#define XFLAGS(p) 0
#endif

constexpr int BM = 128, BN = 128, NT = 256;
constexpr int TILE_BYTES = 128 * 128;  // one operand, one stage

struct GemmP {
  int M, N, K, kvalid, mvalid, nvalid;
  const char* A; long lda; const char* B; long ldb;
  int conv_mode, conv_t, conv_kw, conv_c, conv_p;
  int conv_dil;       // dilation of the forward conv modes 1 and 5 (tap j at (j - P) * dil)
  char* C; long ldc; int c_fp32; int c_conv_kw;
  const float* bias; int relu;
  const char* gate; long ldg;
  const float* row_scale;
  const char* residual; long ldr;
  const float* row_scale_post;
  int accumulate; int split_k; int k_per_split;
  long split_stride;  // >0: split z stores its partial to C + z*split_stride (no atomics)
  int g4_flags;       // FS2_EXPERIMENTS builds only (XFLAGS): timing switches of the large kernels
  int batch_div;
  long sA1, sA2, sB1, sB2, sC1, sC2, sR1, sR2;
  int tiles_m, tiles_n;
  int vec_ok;
  int vec_align;  // vector epilogue possible if K were not split
  int c_row_t, c_row_pad;  // >0: output row m stored at m + (m / c_row_t) * c_row_pad (ps kernel)
  int max_ctas;            // grid budget of the persistent kernels (blocks), 8..256
  int a_bytes, b_bytes;    // gemm_w4b_kernel: readable byte extents of A and B (zeros past them)
  int a_kw;                // gemm_w4b_kernel: tap-inner K order of an overlapping-row A (desc a_kw)
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

// epilogue activation: 1 ReLU (SB pos_ffn, model.py:241-267), 2 GELU with erf
// (nn.GELU() of the IntensityExtractor FFN, rank_model/model.py:30,42), 3 leaky ReLU 0.1 and
// 4 tanh (HiFi-GAN generator: LRELU_SLOPE, output tanh)
// GELU / leaky ReLU / tanh (the intensity extractor and the vocoder): out of line, so the
// unrolled epilogues keep ONE compact body for the train step's none / ReLU.  Inlined, the
// five-way select put an erf and a tanh expansion behind a branch on every output element and
// grew the large-tile kernels to 40-80 KiB of code -- an epilogue fetched cold from the
// instruction cache once per tile.
__device__ __attribute__((noinline)) float epi_act_rare(float v, int act) {
  if (act == 2) return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
  if (act == 3) return v >= 0.f ? v : 0.1f * v;
  if (act == 4) return tanhf(v);
  return v;
}
__device__ __forceinline__ float epi_act(float v, int act) {
  if (act > 1) return epi_act_rare(v, act);
  return act ? fmaxf(v, 0.f) : v;   // a select: NaN passes through when there is no activation
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
          const int ts = reflect_idx(t + (j - P) * p.conv_dil, T_);
          v = ld16(base + ((long)(b * T_ + ts) * ld + c) * ES);
        } else if (cmode == 5) {  // zero-padded "same" conv (nn.Conv1d(padding=k//2))
          const int ts = t + (j - P) * p.conv_dil;
          if (ts >= 0 && ts < T_) v = ld16(base + ((long)(b * T_ + ts) * ld + c) * ES);
        } else if (cmode == 4) {  // shift conv over the padded domain, zero outside [0,T)
          const int ts = t - j;
          if (ts >= 0 && ts < T_) v = ld16(base + ((long)(b * T_ + ts) * ld + c) * ES);
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

// ---- LDS-DMA (global_load_lds_dwordx4) staging, bf16 -----------------------------------
// Each wave-instruction writes 1 KiB of LDS at a wave-uniform base (lane l -> bytes 16l..16l+15),
// so the XOR swizzles above are applied on the SOURCE address: lane l fetches the logical
// chunk that belongs at its physical slot.  Out-of-range chunks read a zero line.
__device__ __attribute__((aligned(64))) char g_fs2_zero[64];

typedef __attribute__((address_space(1))) void gptr_t;
typedef __attribute__((address_space(3))) void lptr_t;

__device__ __forceinline__ void glds16(const char* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const gptr_t*)src, (lptr_t*)lds_wave_base, 16, 0, 0);
}

// Buffer-resource form of the LDS-DMA (buffer_load_dwordx4 ... lds): a wave-uniform base in
// SGPRs, a 32-bit per-lane byte offset and a uniform SGPR offset.  Lanes with the offset
// BUF_OOB fall outside num_records and load zeros -- no per-lane pointer selects.
constexpr int BUF_OOB = (int)0x80000000u;
__device__ __forceinline__ i32x4 make_rsrc(const void* base) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane((int)(a >> 32));
  r[2] = 0x7fffffff;
  r[3] = 0x00020000;
  return r;
}
__device__ __forceinline__ void blds16(i32x4 rsrc, int voff, int soff, char* lds_wave_base) {
  llvm_raw_buffer_load_lds(rsrc, (__attribute__((address_space(3))) uint32_t*)lds_wave_base, 16,
                           voff, soff, 0, 0);
}

// K-major tile (128 rows x 128 B): 16 x 1 KiB pieces, wave w issues pieces 4w..4w+3 (8 rows each)
__device__ __forceinline__ void glds_kmajor(char* lds, const char* base, long ld, int row0,
                                            int nrows, int k0, int kend, const GemmP& p,
                                            int cmode, const int (&rb)[4], const int (&rt)[4],
                                            int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;
    const int r = piece * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ (r & 7);
    const int row = row0 + r;
    const int k = k0 + lc * 8;
    const char* src = g_fs2_zero;
    if (row < nrows && k < kend) {
      if (cmode == 0) {
        src = base + ((long)row * ld + k) * 2;
      } else {  // cmode 1: reflect-padded implicit conv / cmode 4: zero-padded shift
        const int C = p.conv_c, T_ = p.conv_t;
        const int j = k / C, c = k - j * C;
        if (cmode == 1) {
          const int ts = reflect_idx(rt[i] + (j - p.conv_p) * p.conv_dil, T_);
          src = base + ((long)(rb[i] * T_ + ts) * ld + c) * 2;
        } else {
          const int ts = cmode == 5 ? rt[i] + (j - p.conv_p) * p.conv_dil : rt[i] - j;
          if (ts >= 0 && ts < T_) src = base + ((long)(rb[i] * T_ + ts) * ld + c) * 2;
        }
      }
    }
    glds16(src, lds + piece * 1024);
  }
}

// MN-major tile (64 k-rows x 256 B): wave w issues pieces 4w..4w+3 (4 k-rows each)
__device__ __forceinline__ void glds_mnmajor(char* lds, const char* base, long ld, int mn0,
                                             int nmn, int k0, int kend, const GemmP& p,
                                             bool conv3, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = wave * 4 + i;
    const int kr = piece * 4 + (lane >> 4);
    const int lc = (lane & 15) ^ mn_swz<bf16>(kr);
    const int k = k0 + kr;
    const int mn = mn0 + lc * 8;
    const char* src = g_fs2_zero;
    if (k < kend && mn < nmn) {
      long srow = k;
      int col = mn;
      if (conv3) {
        const int j = mn / p.conv_c;
        col = mn - j * p.conv_c;
        const int b = k / p.conv_t, t = k - b * p.conv_t;
        srow = (long)b * p.conv_t + reflect_idx(t + j - p.conv_p, p.conv_t);
      }
      src = base + (srow * ld + col) * 2;
    }
    glds16(src, lds + piece * 1024);
  }
}

// ---- fp32 C staging in LDS (cs[row][col ^ cs_swz(row)], 128 floats per row) ----------------
// An accumulator fragment is written with lanes on 16 rows x 2 column quads per 32-lane half;
// rows are 512 B apart, so only the swizzle separates their banks.  XOR-ing the column by 4x
// (row & 15) spreads them over all 16 quads of banks (2-way, the minimum for 32 lanes whose
// column is fixed mod 4; the old (row >> 2 & 1) << 4 left 8-way: 22 % of the 256 x 128
// weight-gradient kernel's LDS cycles were conflicts, profiles/r03s2_gemm_lds_pmc.json), and
// keeps every aligned 4-float group contiguous for the 16-byte epilogue reads.
__device__ __forceinline__ int cs_swz(int row) { return (row & 15) << 2; }

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
// The same MN-major fragment through inline-asm transposed reads, for the LDS-DMA ring kernels
// (gemm_big_kernel, gemm256_kernel).  hipcc's waitcnt pass treats the ds_read_tr16_b64 builtin
// as a read that may alias any in-flight LDS-DMA and puts an s_waitcnt vmcnt(0) in front of it:
// in the MN-major instances (the weight gradients) that drained the whole prefetch ring at
// every K-tile.  The asm reads are invisible to that pass; mn_ready() after an explicit
// lgkmcnt wait hands the registers back to the compiler.
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
template <int ROWB>   // bytes per k-row of the image: 256 (128 mn) or 512 (256 mn)
__device__ __forceinline__ bf16x8 frag_bf16_mnmajor_asm(const char* lds, int r0, int s, int lane) {
  const int li = lane & 15, g = lane >> 4, q = li >> 2, p = li & 3;
  const int m = r0 + 4 * p;
  const int c = m >> 3, boff = (m & 7) * 2;
  const int k1 = s * 32 + 8 * g + q, k2 = k1 + 4;
  const char* a1 = lds + k1 * ROWB + ((c ^ mn_swz<bf16>(k1)) << 4) + boff;
  const char* a2 = lds + k2 * ROWB + ((c ^ mn_swz<bf16>(k2)) << 4) + boff;
  s16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(lds_off(a1)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(lds_off(a2)));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// after an asm "s_waitcnt lgkmcnt(..)" that retired the reads of f: order every consumer of f
// after that wait (an empty asm that "rewrites" the registers; volatile asm keeps its order)
__device__ __forceinline__ void mn_ready(bf16x8& f) { asm volatile("" : "+v"(f)); }

// fp32 16x16x4 operand, lane l: row (mn) r0 + (l&15), k = s*4 + (l>>4)
__device__ __forceinline__ float frag_f32_kmajor(const char* lds, int r0, int s, int lane) {
  const int r = r0 + (lane & 15);
  return *(const float*)(lds + r * 128 + ((s ^ (r & 7)) << 4) + (lane >> 4) * 4);
}
__device__ __forceinline__ float frag_f32_mnmajor(const char* lds, int r0, int s, int lane) {
  const int m = r0 + (lane & 15), k = s * 4 + (lane >> 4);
  return *(const float*)(lds + k * 512 + (((m >> 2) ^ mn_swz<float>(k)) << 4) + (m & 3) * 4);
}

// 8 consecutive elements <-> float[8] (16-byte bf16 / 2x16-byte fp32 when complete)
template <typename T>
__device__ __forceinline__ void load8(float (&o)[8], const T* src, int nn) {
  if (nn == 8) {
    if constexpr (sizeof(T) == 2) {
      const u32x4 u = *(const u32x4*)src;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        o[2 * w] = __builtin_bit_cast(float, u[w] << 16);
        o[2 * w + 1] = __builtin_bit_cast(float, u[w] & 0xffff0000u);
      }
    } else {
      const f32x4 a = *(const f32x4*)src, b = *(const f32x4*)(src + 4);
      o[0] = a[0]; o[1] = a[1]; o[2] = a[2]; o[3] = a[3];
      o[4] = b[0]; o[5] = b[1]; o[6] = b[2]; o[7] = b[3];
    }
  } else {
    for (int e = 0; e < 8; ++e) o[e] = e < nn ? to_f(src[e]) : 0.f;
  }
}
template <typename T>
__device__ __forceinline__ void store8(T* dst, const float (&v)[8], int nn) {
  if (nn == 8) {
    if constexpr (sizeof(T) == 2) {
      u32x4 u;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const bf16 a = (bf16)v[2 * w], b = (bf16)v[2 * w + 1];
        u[w] = (unsigned)__builtin_bit_cast(unsigned short, a) |
               ((unsigned)__builtin_bit_cast(unsigned short, b) << 16);
      }
      *(u32x4*)dst = u;
    } else {
      *(f32x4*)dst = f32x4{v[0], v[1], v[2], v[3]};
      *(f32x4*)(dst + 4) = f32x4{v[4], v[5], v[6], v[7]};
    }
  } else {
    for (int e = 0; e < nn; ++e) dst[e] = from_f<T>(v[e]);
  }
}

template <typename T, bool AK, bool BKM, bool GA, bool GB>
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
  const int amode = (p.conv_mode == 1 || p.conv_mode == 2 || p.conv_mode == 4 || p.conv_mode == 5) ? p.conv_mode : 0;
  if (AK && amode) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // register staging: row (tid>>3) + 32 i ; LDS-DMA: piece rows (4*wave + i)*8 + (lane>>3)
      const int row = m0 + (GA ? (wave * 4 + i) * 8 + (lane >> 3) : (tid >> 3) + 32 * i);
      const int rpu = amode == 4 ? p.conv_t + 2 * p.conv_p : p.conv_t;  // rows per utterance
      rb[i] = row / rpu;
      rt[i] = row - rb[i] * rpu;
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
  // issue the loads of one K-tile: LDS-DMA straight into the stage (GA/GB) or into registers
  auto load_tiles = [&](int k0, int stage) {
    char* la = smem + stage * 2 * TILE_BYTES;
    char* lb = la + TILE_BYTES;
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    if constexpr (GA) {
      if constexpr (AK) glds_kmajor(la, Ab, p.lda, m0, p.M, k0, kend, p, amode, rb, rt, wv, lane);
      else glds_mnmajor(la, Ab, p.lda, m0, p.M, k0, min(kend, kvalid), p, false, wv, lane);
    } else {
      if constexpr (AK) load_kmajor<T>(stA, Ab, p.lda, m0, p.M, k0, kend, p, amode, rb, rt);
      else load_mnmajor<T>(stA, Ab, p.lda, m0, p.M, k0, min(kend, kvalid), p, false);
    }
    if constexpr (GB) {
      if constexpr (BKM) glds_kmajor(lb, Bb, p.ldb, n0, p.N, k0, kend, p, 0, zero4, zero4, wv, lane);
      else glds_mnmajor(lb, Bb, p.ldb, n0, p.N, k0, min(kend, kvalid), p, bconv3, wv, lane);
    } else {
      if constexpr (BKM) load_kmajor<T>(stB, Bb, p.ldb, n0, p.N, k0, kend, p, 0, zero4, zero4);
      else load_mnmajor<T>(stB, Bb, p.ldb, n0, p.N, k0, min(kend, kvalid), p, bconv3);
    }
  };
  // write register-staged operands to LDS (no-op for LDS-DMA operands)
  auto store_tiles = [&](int stage) {
    char* la = smem + stage * 2 * TILE_BYTES;
    char* lb = la + TILE_BYTES;
    if constexpr (!GA) { if constexpr (AK) store_kmajor<T>(la, stA); else store_mnmajor<T>(la, stA); }
    if constexpr (!GB) { if constexpr (BKM) store_kmajor<T>(lb, stB); else store_mnmajor<T>(lb, stB); }
  };

  const int nk = (kend > kbeg) ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    load_tiles(kbeg, 0);
    store_tiles(0);
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int stage = kt & 1;
    if (kt + 1 < nk) load_tiles(kbeg + (kt + 1) * BK, stage ^ 1);
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
  if (p.split_stride > 0 && p.split_k > 1) Cb += (long)blockIdx.z * p.split_stride * OES;
  const char* Rb = p.residual ? p.residual + (zb * p.sR1 + zh * p.sR2) * ES : nullptr;
  const bool atomic = p.split_k > 1 && p.split_stride == 0;
  const int cc = p.c_conv_kw > 0 ? p.N / p.c_conv_kw : 0;
  if (!p.vec_ok) {  // scalar path: scattered (conv-remapped) or atomic fp32 gradient outputs
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
          v = epi_act(v, p.relu);
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
    return;
  }
  // vector path: accumulators -> LDS (fp32 128x128, column bit 4 flipped on rows with bit 2
  // set so the two 16-lane row groups of a ds_write_b32 half hit disjoint banks), then each
  // thread owns 8 consecutive columns of a row: 16-byte loads of bias / gate / residual and
  // 16-byte stores -- one 256-byte segment per 16 threads.
  float* cs = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        const int col = wn * 64 + j * 16 + (lane & 15);
        cs[row * 128 + (col ^ cs_swz(row))] = acc[i][j][r];
      }
  __syncthreads();
  const int c8 = (tid & 15) * 8;
  const int n = n0 + c8;
#pragma unroll 2
  for (int pass = 0; pass < 8; ++pass) {
    const int row = (tid >> 4) + 16 * pass;
    const int m = m0 + row;
    if (m >= p.mvalid || n >= p.nvalid) continue;
    const int sw = cs_swz(row);
    const f32x4 lo = *(const f32x4*)&cs[row * 128 + (c8 ^ sw)];
    const f32x4 hi = *(const f32x4*)&cs[row * 128 + ((c8 + 4) ^ sw)];
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    const int nn = min(8, p.nvalid - n);
    const float rs = p.row_scale ? p.row_scale[m] : 1.f;
    const float rs2 = p.row_scale_post ? p.row_scale_post[m] : 1.f;
    if (p.bias) {
      if (nn == 8) {
        const f32x4 b0 = *(const f32x4*)(p.bias + n), b1 = *(const f32x4*)(p.bias + n + 4);
        v[0] += b0[0]; v[1] += b0[1]; v[2] += b0[2]; v[3] += b0[3];
        v[4] += b1[0]; v[5] += b1[1]; v[6] += b1[2]; v[7] += b1[3];
      } else {
        for (int e = 0; e < nn; ++e) v[e] += p.bias[n + e];
      }
    }
    float g[8], rr[8];
    if (p.gate) load8<T>(g, (const T*)p.gate + (long)m * p.ldg + n, nn);
    if (Rb) load8<T>(rr, (const T*)Rb + (long)m * p.ldr + n, nn);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = v[e];
      x = epi_act(x, p.relu);
      if (p.gate) x = (g[e] > 0.f) ? x : 0.f;
      x *= rs;
      if (Rb) x += rr[e];
      v[e] = x * rs2;
    }
    const long off = (long)m * p.ldc + n;
    if (p.c_fp32) {
      float* Cf = (float*)Cb + off;
      if (nn == 8) {
        f32x4 o0 = {v[0], v[1], v[2], v[3]}, o1 = {v[4], v[5], v[6], v[7]};
        if (p.accumulate) { o0 += *(const f32x4*)Cf; o1 += *(const f32x4*)(Cf + 4); }
        *(f32x4*)Cf = o0;
        *(f32x4*)(Cf + 4) = o1;
      } else {
        for (int e = 0; e < nn; ++e) Cf[e] = p.accumulate ? Cf[e] + v[e] : v[e];
      }
    } else {
      store8<T>((T*)Cb + off, v, nn);
    }
  }
}

// ============================================================================================
// "Big" bf16 kernel: 256x128 tile, 8 waves (4 x 2, 64x64 per wave), BK = 64, three-stage
// LDS-DMA ring (48 KiB per stage, prefetch distance 2) paced by COUNTED vmcnt waits and raw
// s_barrier (a __syncthreads() would drain the in-flight prefetch), XCD-aware tile order.
// Used for every bf16 GEMM with enough tiles except the reflect-fold dgrad operand.
// ============================================================================================
constexpr int BBM = 256, BNT = 512;
constexpr int BIG_A = 256 * 128;          // A stage bytes (32 KiB)
constexpr int BIG_B = 128 * 128;          // B stage bytes (16 KiB)
constexpr int BIG_STAGE = BIG_A + BIG_B;  // 48 KiB
constexpr int BIG_LDS = 3 * BIG_STAGE;    // 144 KiB (the 256x128 fp32 epilogue tile fits)


// Direct epilogue of one wave's 4 x 4 grid of 16x16 result blocks.  The large-tile kernels
// compute every block TRANSPOSED (MFMA A operand = the B tile's fragment), so a lane holds
// row m = mb + 16 i + (lane & 15) and the 4 CONSECUTIVE columns n = nb + 16 j + 4 (lane >> 4)
// + 0..3 of block (i, j): the result leaves the registers as 8-byte (bf16) / 16-byte (fp32)
// stores with no LDS staging and no barrier.  Every global operand (bias, row scales, gate,
// residual) is loaded before the first store: vmcnt counts loads and stores in one in-order
// queue, so a load issued after a store would wait for that store as well (the LDS-staged pass
// loop this replaces ran its stores at ~1.7 TB/s for exactly that reason).
__device__ __forceinline__ void epilogue_direct(const GemmP& p, const f32x4* acc, int mb, int nb,
                                                char* Cb, const char* Rb, int lane) {
  const int li = lane & 15, g = lane >> 4;
  f32x4 bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = nb + 16 * j + 4 * g;
    bv[j] = (p.bias && n < p.nvalid) ? *(const f32x4*)(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float rs[4], rs2[4];
  u32x2 gv[4][4], rv[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mb + 16 * i + li;
    const bool in = m < p.mvalid;
    rs[i] = (p.row_scale && in) ? p.row_scale[m] : 1.f;
    rs2[i] = (p.row_scale_post && in) ? p.row_scale_post[m] : 1.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nb + 16 * j + 4 * g;
      const bool ok = in && n < p.nvalid;
      gv[i][j] = (p.gate && ok) ? *(const u32x2*)((const bf16*)p.gate + (long)m * p.ldg + n) : u32x2{0u, 0u};
      rv[i][j] = (Rb && ok) ? *(const u32x2*)((const bf16*)Rb + (long)m * p.ldr + n) : u32x2{0u, 0u};
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mb + 16 * i + li;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = nb + 16 * j + 4 * g;
      if (m >= p.mvalid || n >= p.nvalid) continue;
      const f32x4 a = acc[i * 4 + j];
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = epi_act(a[e] + bv[j][e], p.relu);
        if (p.gate) {
          const unsigned w = gv[i][j][e >> 1];
          const float gg = __builtin_bit_cast(float, (e & 1) ? (w & 0xffff0000u) : (w << 16));
          x = gg > 0.f ? x : 0.f;
        }
        x *= rs[i];
        if (Rb) {
          const unsigned w = rv[i][j][e >> 1];
          x += __builtin_bit_cast(float, (e & 1) ? (w & 0xffff0000u) : (w << 16));
        }
        v[e] = x * rs2[i];
      }
      const long off = (long)m * p.ldc + n;
      if (p.c_fp32) {
        f32x4 o = {v[0], v[1], v[2], v[3]};
        float* Cf = (float*)Cb + off;
        if (p.accumulate) o += *(const f32x4*)Cf;
        *(f32x4*)Cf = o;
      } else {
        u32x2 w;
        w[0] = (unsigned)__builtin_bit_cast(unsigned short, (bf16)v[0]) |
               ((unsigned)__builtin_bit_cast(unsigned short, (bf16)v[1]) << 16);
        w[1] = (unsigned)__builtin_bit_cast(unsigned short, (bf16)v[2]) |
               ((unsigned)__builtin_bit_cast(unsigned short, (bf16)v[3]) << 16);
        *(u32x2*)((bf16*)Cb + off) = w;
      }
    }
  }
}

// Epilogue of a 256-row x 128-column fp32 tile staged in LDS (cs[row][col ^ swz], 512 threads):
// vector pass (bias, ReLU, gate, row scales, residual, 16-byte stores), or the scalar pass for
// weight gradients (column remap, split-K atomics).
__device__ __forceinline__ void epilogue_256x128(const GemmP& p, const float* cs, int m0, int n0,
                                                 char* Cb, const char* Rb, int tid) {
  if (!p.vec_ok) {  // weight gradients: fp32, conv column remap n=(j,c) -> c*KW + j, atomics
    const int cc = p.c_conv_kw > 0 ? p.N / p.c_conv_kw : 0;
    const bool atomic = p.split_k > 1 && p.split_stride == 0;
    float* Cf = (float*)Cb;
    for (int idx = tid; idx < BBM * 128; idx += BNT) {
      const int row = idx >> 7, col = idx & 127;
      const int m = m0 + row, n = n0 + col;
      if (m >= p.mvalid || n >= p.nvalid) continue;
      float v = cs[row * 128 + (col ^ cs_swz(row))];
      long c2 = n;
      if (cc > 0) { const int jj = n / cc; c2 = (long)(n - jj * cc) * p.c_conv_kw + jj; }
      const long off = (long)m * p.ldc + c2;
      if (atomic) atomicAdd(Cf + off, v);
      else if (p.accumulate) Cf[off] += v;
      else Cf[off] = v;
    }
    return;
  }
  const int c8 = (tid & 15) * 8;
  const int n = n0 + c8;
  if (n >= p.nvalid) return;
  const int nn = min(8, p.nvalid - n);
  // this thread's 8 bias columns, loaded once per tile half (in the pass loop the compiler had
  // to reload them after every output store, which may alias the bias)
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (p.bias) {
    if (nn == 8) {
      const f32x4 b0 = *(const f32x4*)(p.bias + n), b1 = *(const f32x4*)(p.bias + n + 4);
      bv[0] = b0[0]; bv[1] = b0[1]; bv[2] = b0[2]; bv[3] = b0[3];
      bv[4] = b1[0]; bv[5] = b1[1]; bv[6] = b1[2]; bv[7] = b1[3];
    } else {
      for (int e = 0; e < nn; ++e) bv[e] = p.bias[n + e];
    }
  }
#pragma unroll 2
  for (int pass = 0; pass < 8; ++pass) {
    const int row = (tid >> 4) + 32 * pass;
    const int m = m0 + row;
    if (m >= p.mvalid) continue;
    const int sw = cs_swz(row);
    const f32x4 lo = *(const f32x4*)&cs[row * 128 + (c8 ^ sw)];
    const f32x4 hi = *(const f32x4*)&cs[row * 128 + ((c8 + 4) ^ sw)];
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    const float rs = p.row_scale ? p.row_scale[m] : 1.f;
    const float rs2 = p.row_scale_post ? p.row_scale_post[m] : 1.f;
    if (p.bias) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bv[e];
    }
    float g[8], rr[8];
    if (p.gate) load8<bf16>(g, (const bf16*)p.gate + (long)m * p.ldg + n, nn);
    if (Rb) load8<bf16>(rr, (const bf16*)Rb + (long)m * p.ldr + n, nn);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float x = v[e];
      x = epi_act(x, p.relu);
      if (p.gate) x = (g[e] > 0.f) ? x : 0.f;
      x *= rs;
      if (Rb) x += rr[e];
      v[e] = x * rs2;
    }
    const long off = (long)m * p.ldc + n;
    if (p.c_fp32) {
      float* Cf = (float*)Cb + off;
      if (nn == 8) {
        f32x4 o0 = {v[0], v[1], v[2], v[3]}, o1 = {v[4], v[5], v[6], v[7]};
        if (p.accumulate) { o0 += *(const f32x4*)Cf; o1 += *(const f32x4*)(Cf + 4); }
        *(f32x4*)Cf = o0;
        *(f32x4*)(Cf + 4) = o1;
      } else {
        for (int e = 0; e < nn; ++e) Cf[e] = p.accumulate ? Cf[e] + v[e] : v[e];
      }
    } else {
      store8<bf16>((bf16*)Cb + off, v, nn);
    }
  }
}

// CM: A-operand conv mode fixed at compile time (0 plain, 1 reflect conv, 4 shift conv, both
// with 64-aligned taps) or -1 = decided at run time; B3: B-operand conv3 (0/1) or -1 = run time.
template <bool AK, bool BKM, int CM, int B3>
__global__ void __launch_bounds__(BNT) gemm_big_kernel(GemmP p) {
  __shared__ __attribute__((aligned(16))) char smem[BIG_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware bijective remap: blocks b and b+8 share an XCD; give each XCD a contiguous run
  const int nwg = p.tiles_m * p.tiles_n;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r8 = nwg & 7;
  const int bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
  const int tm = bid / p.tiles_n, tn = bid - tm * p.tiles_n;
  const int m0 = tm * BBM, n0 = tn * 128;
  const int z = p.split_k > 1 ? 0 : blockIdx.z;
  const long zb = z / p.batch_div, zh = z - zb * p.batch_div;
  const char* Ab = p.A + (zb * p.sA1 + zh * p.sA2) * 2;
  const char* Bb = p.B + (zb * p.sB1 + zh * p.sB2) * 2;
  const int K = p.K;
  const int kva = min(K, p.kvalid);
  const int amode = CM >= 0 ? CM : ((p.conv_mode == 1 || p.conv_mode == 4 || p.conv_mode == 5) ? p.conv_mode : 0);
  // split-K: this block reduces k-tiles [kt0, kt1) and accumulates with fp32 atomics
  const int nk_all = (K + 63) / 64;
  int kt0 = 0, kt1 = nk_all;
  if (p.split_k > 1) {
    const int kps = (nk_all + p.split_k - 1) / p.split_k;
    kt0 = blockIdx.z * kps;
    kt1 = min(nk_all, kt0 + kps);
  }
  const bool bconv3 = B3 >= 0 ? B3 == 1 : p.conv_mode == 3;
  // a 64-wide k-tile sits in one tap
  const bool tap_uniform = CM > 0 ? true : (CM == 0 ? false : amode && (p.conv_c % 64) == 0);
  const int rpu = amode == 4 ? p.conv_t + 2 * p.conv_p : p.conv_t;  // rows per utterance

  // ---- per-lane, per-piece DMA source state (32-bit byte offsets from the operand base,
  // BUF_OOB = zero fill), advanced by wave-uniform offsets; implicit-conv rows re-pointed only
  // when the tap changes.
  // A K-major: pieces 4w+i (8 rows each), lane row r = piece*8 + (lane>>3), chunk alc
  const i32x4 rsA = make_rsrc(Ab), rsB = make_rsrc(Bb);
  int avo[4];
  int abt[4], at[4], alc[4];
  bool aval[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (AK) {
      const int r = (wave * 4 + i) * 8 + (lane >> 3);
      alc[i] = (lane & 7) ^ (r & 7);
      const int row = m0 + r;
      aval[i] = row < p.M;
      const int rr = aval[i] ? row : 0;
      const int b = amode ? rr / rpu : 0;
      abt[i] = b * p.conv_t;       // source row base (unpadded utterance)
      at[i] = rr - b * rpu;        // position inside the (padded) utterance
      avo[i] = aval[i] ? (int)(((long)rr * p.lda + alc[i] * 8) * 2) : BUF_OOB;
    } else {  // MN-major (512-byte k-rows): piece = 2 k-rows
      const int kr = (wave * 4 + i) * 2 + (lane >> 5);
      alc[i] = (lane & 31) ^ mn_swz<bf16>(kr);
      at[i] = kr;
      const int mn = m0 + alc[i] * 8;
      aval[i] = mn < p.M;
      avo[i] = aval[i] ? (int)(((long)mn + (long)kr * p.lda) * 2) : BUF_OOB;
      abt[i] = 0;
    }
  }
  int a_tap = -1;
  int bvo[2];
  int blc[2], bkr[2], bb[2], bt[2];
  bool bval[2];
  int b_k = kt0 * 64;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if constexpr (BKM) {
      const int r = (wave * 2 + i) * 8 + (lane >> 3);
      blc[i] = (lane & 7) ^ (r & 7);
      const int row = n0 + r;
      bval[i] = row < p.N;
      bvo[i] = bval[i] ? (int)(((long)row * p.ldb + blc[i] * 8) * 2) : BUF_OOB;
      bkr[i] = 0; bb[i] = 0; bt[i] = 0;
    } else {  // MN-major (256-byte k-rows): piece = 4 k-rows
      const int kr = (wave * 2 + i) * 4 + (lane >> 4);
      blc[i] = (lane & 15) ^ mn_swz<bf16>(kr);
      bkr[i] = kr;
      const int mn = n0 + blc[i] * 8;
      bval[i] = mn < p.N;
      int col = mn;
      if (bconv3 && bval[i]) { const int j = mn / p.conv_c; col = mn - j * p.conv_c; blc[i] = j; }
      else if (bconv3) blc[i] = 0;
      bvo[i] = bval[i] ? (int)(((long)col + (bconv3 ? 0L : (long)kr * p.ldb)) * 2) : BUF_OOB;
      const int k = b_k + kr;
      bb[i] = bconv3 ? k / p.conv_t : 0;
      bt[i] = bconv3 ? k - bb[i] * p.conv_t : 0;
    }
  }

  auto issue = [&](int kt, int stage) {   // 6 LDS-DMA pieces per wave
    const int k0 = kt * 64;
    char* la = smem + stage * BIG_STAGE;
    char* lb = la + BIG_A;
    if constexpr (AK) {
      if (amode && tap_uniform) {
        const int j = k0 / p.conv_c, c0 = k0 - j * p.conv_c;   // wave-uniform
        if (j != a_tap) {
          a_tap = j;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            int ts;
            bool ok = aval[i];
            if (amode == 1) {
              ts = reflect_idx(at[i] + (j - p.conv_p) * p.conv_dil, p.conv_t);
            } else {
              ts = amode == 5 ? at[i] + (j - p.conv_p) * p.conv_dil : at[i] - j;
              ok = ok && ts >= 0 && ts < p.conv_t;
            }
            avo[i] = ok ? (int)(((long)(abt[i] + ts) * p.lda + alc[i] * 8) * 2) : BUF_OOB;
          }
        }
        const bool kin = k0 + 64 <= K;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int vo = (kin || k0 + alc[i] * 8 < K) ? avo[i] : BUF_OOB;
          blds16(rsA, vo, c0 * 2, la + (wave * 4 + i) * 1024);
        }
      } else if (!amode) {
        const bool kin = k0 + 64 <= K;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int vo = (kin || k0 + alc[i] * 8 < K) ? avo[i] : BUF_OOB;
          blds16(rsA, vo, k0 * 2, la + (wave * 4 + i) * 1024);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = k0 + alc[i] * 8;
          bool ok = aval[i] && k < K;
          const int j = k / p.conv_c, c = k - j * p.conv_c;
          int ts;
          if (amode == 1) {
            ts = reflect_idx(at[i] + (j - p.conv_p) * p.conv_dil, p.conv_t);
          } else {
            ts = amode == 5 ? at[i] + (j - p.conv_p) * p.conv_dil : at[i] - j;
            ok = ok && ts >= 0 && ts < p.conv_t;
          }
          const int vo = ok ? (int)(((long)(abt[i] + ts) * p.lda + c) * 2) : BUF_OOB;
          blds16(rsA, vo, 0, la + (wave * 4 + i) * 1024);
        }
      }
    } else {
      const bool kin = k0 + 64 <= kva;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int vo = (kin || k0 + at[i] < kva) ? avo[i] : BUF_OOB;
        blds16(rsA, vo, (int)((long)k0 * p.lda * 2), la + (wave * 4 + i) * 1024);
      }
    }
    if constexpr (BKM) {
      const bool kin = k0 + 64 <= K;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int vo = (kin || k0 + blc[i] * 8 < K) ? bvo[i] : BUF_OOB;
        blds16(rsB, vo, k0 * 2, lb + (wave * 2 + i) * 1024);
      }
    } else if (!bconv3) {
      const bool kin = k0 + 64 <= kva;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int vo = (kin || k0 + bkr[i] < kva) ? bvo[i] : BUF_OOB;
        blds16(rsB, vo, (int)((long)k0 * p.ldb * 2), lb + (wave * 2 + i) * 1024);
      }
    } else {
      const int dk = k0 - b_k;
      b_k = k0;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        int t = bt[i] + dk, b = bb[i];
        while (t >= p.conv_t) { t -= p.conv_t; ++b; }
        bt[i] = t; bb[i] = b;
        int ts = t + blc[i] - p.conv_p;
        ts = ts < 0 ? -ts : (ts >= p.conv_t ? 2 * (p.conv_t - 1) - ts : ts);
        const bool ok = bval[i] && k0 + bkr[i] < kva;
        const int vo = ok ? bvo[i] + (int)(((long)b * p.conv_t + ts) * p.ldb * 2) : BUF_OOB;
        blds16(rsB, vo, 0, lb + (wave * 2 + i) * 1024);
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = kt1 - kt0;
  if (nk > 0) issue(kt0, 0);
  if (nk > 1) issue(kt0 + 1, 1);
  for (int it = 0; it < nk; ++it) {
    // tile it landed for this wave (leave tile it+1's 6 pieces in flight) ...
    if (it + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ... and for every wave; every wave is also done reading stage (it+2)%3 == (it-1)%3
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (it + 2 < nk) issue(kt0 + it + 2, (it + 2) % 3);
    const char* la = smem + (it % 3) * BIG_STAGE;
    const char* lb = la + BIG_A;
    // all fragments of both k-steps first (distinct registers), then 32 MFMAs
    bf16x8 af[2][4], bfr[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        af[s][i] = AK ? frag_bf16_kmajor(la, wm * 64 + i * 16, s, lane)
                      : frag_bf16_mnmajor_asm<512>(la, wm * 64 + i * 16, s, lane);
        bfr[s][i] = BKM ? frag_bf16_kmajor(lb, wn * 64 + i * 16, s, lane)
                        : frag_bf16_mnmajor_asm<256>(lb, wn * 64 + i * 16, s, lane);
      }
    if constexpr (!AK || !BKM) {   // asm reads: retire them before the MFMAs
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if constexpr (!AK) mn_ready(af[s][i]);
          if constexpr (!BKM) mn_ready(bfr[s][i]);
        }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[s][j], af[s][i], acc[i][j], 0, 0, 0);
    // pin the order: every fragment read of the tile is issued before the first MFMA, so the
    // step-1 reads land while step-0 MFMAs run (hipcc otherwise recycles 2 registers and
    // waits lgkmcnt(0) in front of every MFMA group)
    if constexpr (AK && BKM) {
      __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 32, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  // ---- epilogue (blocks computed transposed: lane = row, 4 consecutive columns) ----
  char* Cb = p.C + (zb * p.sC1 + zh * p.sC2) * (p.c_fp32 ? 4 : 2);
  if (p.split_stride > 0 && p.split_k > 1) Cb += (long)blockIdx.z * p.split_stride * 4;
  const char* Rb = p.residual ? p.residual + (zb * p.sR1 + zh * p.sR2) * 2 : nullptr;
  if (p.vec_ok && !(XFLAGS(p) & 64)) {
    epilogue_direct(p, &acc[0][0], m0 + wm * 64, n0 + wn * 64, Cb, Rb, lane);
    return;
  }
  __syncthreads();
  float* cs = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + (lane & 15);
        const int col = wn * 64 + j * 16 + (lane >> 4) * 4 + r;
        cs[row * 128 + (col ^ cs_swz(row))] = acc[i][j][r];
      }
  __syncthreads();
  epilogue_256x128(p, cs, m0, n0, Cb, Rb, tid);
}

// ---------------------------------------------------------------------------------------------
// 256x256 tile, BK = 64, 8 waves as 2 (M) x 4 (N), 128x64 outputs per wave (acc 8x4 fragments).
// Phased main loop after the CDNA4 256^2 template (cdna_hip_programming.md section 5): a K-tile
// is 4 phases; phase p = (k-half s = p>>1, m-half mq = p&1) runs one 64x64 quadrant x K=32
// = 16 MFMAs per wave.  LDS holds two K-tile slots of four 16 KiB regions
// [A k0 | B k0 | A k1 | B k1] (K-major: 256 rows x 64 B; MN-major: 32 k-rows x 512 B).
// Each phase: ds_read its fragments, issue ONE region of the next K-tile (2 LDS-DMA pieces per
// wave, region p), barrier, MFMAs at raised priority, barrier.  Region p of tile t+1 is written
// >= 3 phases after that slot region's last read of tile t-1 and waited for (counted vmcnt(4),
// never 0 in the loop) >= 3 phases after issue.  Waves 4-7 run half a phase behind (one extra
// barrier) so each SIMD pairs one wave's MFMA cluster with its partner's reads and DMA issue;
// they retire their DMA at the end of their memory section, the first group at the end of its
// MFMA section -- both before the barrier instance that precedes the first read of the data.
constexpr int G4_NT = 512;
constexpr int G4_REG = 16384;
constexpr int G4_SLOT = 4 * G4_REG;
constexpr int G4_LDS = 2 * G4_SLOT;   // 128 KiB; also holds the 256x128 fp32 epilogue half-tile

// 16-byte chunk swizzle of the 64-byte-row K-major region: conflict-free ds_read_b128 for
// 16 consecutive rows x chunk (lane >> 4)
__device__ __forceinline__ int g4_fsw(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

__device__ __forceinline__ bf16x8 g4_frag_k(const char* rg, int row, int g) {
  return *(const bf16x8*)(rg + row * 64 + ((g ^ g4_fsw(row)) << 4));
}

template <bool AK, bool BKM, int CM, int B3>   // CM, B3: as gemm_big_kernel (32-aligned taps)
__global__ void __launch_bounds__(G4_NT, 1) gemm256_kernel(GemmP p) {
  __shared__ __attribute__((aligned(16))) char smem[G4_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int nwg = p.tiles_m * p.tiles_n;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tm = bid / p.tiles_n, tn = bid - tm * p.tiles_n;
  const int m0 = tm * 256, n0 = tn * 256;
  const int z = p.split_k > 1 ? 0 : blockIdx.z;
  const long zb = z / p.batch_div, zh = z - zb * p.batch_div;
  const char* Ab = p.A + (zb * p.sA1 + zh * p.sA2) * 2;
  const char* Bb = p.B + (zb * p.sB1 + zh * p.sB2) * 2;
  const int K = p.K;
  const int kva = min(K, p.kvalid);
  const int amode = CM >= 0 ? CM : ((p.conv_mode == 1 || p.conv_mode == 4 || p.conv_mode == 5) ? p.conv_mode : 0);
  const int nk_all = (K + 63) / 64;
  int kt0 = 0, kt1 = nk_all;
  if (p.split_k > 1) {
    const int kps = (nk_all + p.split_k - 1) / p.split_k;
    kt0 = blockIdx.z * kps;
    kt1 = min(nk_all, kt0 + kps);
  }
  const bool bconv3 = B3 >= 0 ? B3 == 1 : p.conv_mode == 3;
  // a 32-wide region sits in one tap
  const bool tap_uniform = CM > 0 ? true : (CM == 0 ? false : amode && (p.conv_c % 32) == 0);
  const int rpu = amode == 4 ? p.conv_t + 2 * p.conv_p : p.conv_t;

  // ---- per-lane DMA source state of this wave's two pieces of an A region and of a B region:
  // 32-bit byte offsets from the operand base (BUF_OOB: zero fill), advanced by wave-uniform
  // offsets as regions are issued in increasing k; the implicit-conv rows are re-pointed only
  // when the tap changes.
  const i32x4 rsA = make_rsrc(Ab), rsB = make_rsrc(Bb);
  int avo[2];          // A: offset at k = 0 of the current tap (conv) or of the row/column
  int abt[2], at[2], ac[2];
  bool aval[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = wave * 2 + i;
    if constexpr (AK) {  // 16 rows x 64 B per piece
      const int r = piece * 16 + (lane >> 2);
      ac[i] = (lane & 3) ^ g4_fsw(r);
      const int row = m0 + r;
      aval[i] = row < p.M;
      const int rr = aval[i] ? row : 0;
      const int b = amode ? rr / rpu : 0;
      abt[i] = b * p.conv_t;
      at[i] = rr - b * rpu;
      avo[i] = aval[i] ? (int)(((long)rr * p.lda + ac[i] * 8) * 2) : BUF_OOB;
      if (XFLAGS(p) & 128) {  // timing experiment: 8 full 128-B rows per piece (wrong results)
        const int r2 = m0 + piece * 16 + (lane >> 3) + 8 * i;
        avo[i] = r2 < p.M ? (int)(((long)r2 * p.lda + (lane & 7) * 8) * 2) : BUF_OOB;
      }
    } else {             // 2 k-rows x 512 B per piece
      const int kr = piece * 2 + (lane >> 5);
      ac[i] = (lane & 31) ^ mn_swz<bf16>(kr);
      at[i] = kr;
      const int mn = m0 + ac[i] * 8;
      aval[i] = mn < p.M;
      avo[i] = aval[i] ? (int)(((long)mn + (long)kr * p.lda) * 2) : BUF_OOB;
      abt[i] = 0;
    }
  }
  int a_tap = -1;      // tap whose rows avo[] point at (implicit conv)
  int bvo[2];
  int bc[2], bkr[2], bb[2], bt[2];
  bool bval[2];
  int b_k = kt0 * 64;  // k of the last B region issued (conv3 incremental (b, t))
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = wave * 2 + i;
    if constexpr (BKM) {
      const int r = piece * 16 + (lane >> 2);
      bc[i] = (lane & 3) ^ g4_fsw(r);
      const int row = n0 + r;
      bval[i] = row < p.N;
      bvo[i] = bval[i] ? (int)(((long)row * p.ldb + bc[i] * 8) * 2) : BUF_OOB;
      if (XFLAGS(p) & 128) {
        const int r2 = n0 + piece * 16 + (lane >> 3) + 8 * i;
        bvo[i] = r2 < p.N ? (int)(((long)r2 * p.ldb + (lane & 7) * 8) * 2) : BUF_OOB;
      }
      bkr[i] = 0; bb[i] = 0; bt[i] = 0;
    } else {
      const int kr = piece * 2 + (lane >> 5);
      const int lc = (lane & 31) ^ mn_swz<bf16>(kr);
      bkr[i] = kr;
      const int mn = n0 + lc * 8;
      bval[i] = mn < p.N;
      int col = mn;
      bc[i] = 0;
      if (bconv3 && bval[i]) { const int j = mn / p.conv_c; col = mn - j * p.conv_c; bc[i] = j; }
      bvo[i] = bval[i] ? (int)(((long)col + (bconv3 ? 0L : (long)kr * p.ldb)) * 2) : BUF_OOB;
      const int k = b_k + kr;
      bb[i] = bconv3 ? k / p.conv_t : 0;
      bt[i] = bconv3 ? k - bb[i] * p.conv_t : 0;
    }
  }

  auto issueA = [&](char* dst, int k0) {
    if constexpr (AK) {
      if (amode && tap_uniform) {
        const int j = k0 / p.conv_c;            // wave-uniform
        const int c0 = k0 - j * p.conv_c;
        if (j != a_tap) {                       // new tap: re-point the rows
          a_tap = j;
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            int ts;
            bool ok = aval[i];
            if (amode == 1) {
              ts = reflect_idx(at[i] + (j - p.conv_p) * p.conv_dil, p.conv_t);
            } else {
              ts = amode == 5 ? at[i] + (j - p.conv_p) * p.conv_dil : at[i] - j;
              ok = ok && ts >= 0 && ts < p.conv_t;
            }
            avo[i] = ok ? (int)(((long)(abt[i] + ts) * p.lda + ac[i] * 8) * 2) : BUF_OOB;
          }
        }
        const bool kin = k0 + 32 <= K;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int vo = (kin || k0 + ac[i] * 8 < K) ? avo[i] : BUF_OOB;
          blds16(rsA, vo, c0 * 2, dst + (wave * 2 + i) * 1024);
        }
      } else if (!amode) {
        const bool kin = k0 + 32 <= K;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int vo = (kin || k0 + ac[i] * 8 < K) ? avo[i] : BUF_OOB;
          blds16(rsA, vo, ((XFLAGS(p) & 128) ? (k0 & ~63) : k0) * 2, dst + (wave * 2 + i) * 1024);
        }
      } else {                                  // taps not aligned to 32-wide regions
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int k = k0 + ac[i] * 8;
          bool ok = aval[i] && k < K;
          const int j = k / p.conv_c, c = k - j * p.conv_c;
          int ts;
          if (amode == 1) {
            ts = reflect_idx(at[i] + (j - p.conv_p) * p.conv_dil, p.conv_t);
          } else {
            ts = amode == 5 ? at[i] + (j - p.conv_p) * p.conv_dil : at[i] - j;
            ok = ok && ts >= 0 && ts < p.conv_t;
          }
          const int vo = ok ? (int)(((long)(abt[i] + ts) * p.lda + c) * 2) : BUF_OOB;
          blds16(rsA, vo, 0, dst + (wave * 2 + i) * 1024);
        }
      }
    } else {
      const bool kin = k0 + 32 <= kva;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int vo = (kin || k0 + at[i] < kva) ? avo[i] : BUF_OOB;
        blds16(rsA, vo, (int)((long)k0 * p.lda * 2), dst + (wave * 2 + i) * 1024);
      }
    }
  };
  auto issueB = [&](char* dst, int k0) {
    if constexpr (BKM) {
      const bool kin = k0 + 32 <= K;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int vo = (kin || k0 + bc[i] * 8 < K) ? bvo[i] : BUF_OOB;
        blds16(rsB, vo, ((XFLAGS(p) & 128) ? (k0 & ~63) : k0) * 2, dst + (wave * 2 + i) * 1024);
      }
    } else if (!bconv3) {
      const bool kin = k0 + 32 <= kva;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int vo = (kin || k0 + bkr[i] < kva) ? bvo[i] : BUF_OOB;
        blds16(rsB, vo, (int)((long)k0 * p.ldb * 2), dst + (wave * 2 + i) * 1024);
      }
    } else {
      // k-row k = k0 + bkr = b*T + t, advanced incrementally from the previous region
      const int dk = k0 - b_k;
      b_k = k0;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        int t = bt[i] + dk, b = bb[i];
        while (t >= p.conv_t) { t -= p.conv_t; ++b; }
        bt[i] = t; bb[i] = b;
        int ts = t + bc[i] - p.conv_p;
        ts = ts < 0 ? -ts : (ts >= p.conv_t ? 2 * (p.conv_t - 1) - ts : ts);
        const bool ok = bval[i] && k0 + bkr[i] < kva;
        const int vo = ok ? bvo[i] + (int)(((long)b * p.conv_t + ts) * p.ldb * 2) : BUF_OOB;
        blds16(rsB, vo, 0, dst + (wave * 2 + i) * 1024);
      }
    }
  };
  // region reg (0: A k0, 1: B k0, 2: A k1, 3: B k1) of relative K-tile it -> slot it & 1
  auto issue = [&](int it, int reg) {
    const int k0 = (kt0 + it) * 64 + (reg >> 1) * 32;
    char* dst = smem + (it & 1) * G4_SLOT + reg * G4_REG;
    if ((reg & 1) == 0) issueA(dst, k0);
    else issueB(dst, k0);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Region schedule (prefetch ~1.5 K-tiles ahead): phase p of tile t issues B k1, A k1 of tile
  // t+1 (p = 0, 1) and B k0, A k0 of tile t+2 (p = 2, 3) -- each into the slot region its
  // previous occupant (tile t-1 / t) left >= 2 phases earlier -- so a region has 4-5 phases to
  // land instead of 2-3 (the LDS-DMA latency under full load stalled the 1-tile-ahead ring:
  // with the DMA issue removed the same loop ran 1470 vs 800 TF/s at 8192^3).  The prologue
  // issues in the same order: B k0, A k0, B k1, A k1 of tile 0, then B k0, A k0 of tile 1.
  const int nk = kt1 - kt0;
  if (nk > 0) {
    issue(0, 1); issue(0, 0); issue(0, 3); issue(0, 2);
  }
  if (nk > 1) {
    issue(1, 1); issue(1, 0);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // k0 regions of the first tile
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  const bool stag = !(XFLAGS(p) & 1);
  const bool prio = !(XFLAGS(p) & 2);
  const bool nowait = XFLAGS(p) & 4;   // timing experiments only (wrong results)
  const bool noissue = XFLAGS(p) & 8;
  // stagger: waves 4-7 half a phase behind; without it both groups retire DMA like group 1
  const int grp = stag ? wr : 1;
  if (stag && wr == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  bf16x8 af[4], bfr[4];
  for (int it = 0; it < nk; ++it) {
    const bool more = it + 1 < nk;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int s = ph >> 1, mq = ph & 1;
      const char* rA = smem + (it & 1) * G4_SLOT + (2 * s) * G4_REG;
      const char* rB = rA + G4_REG;
      // ---- memory section: fragments of this phase, then one region of the next tile ----
      if (mq == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          bfr[j] = BKM ? g4_frag_k(rB, wc * 64 + j * 16 + (lane & 15), lane >> 4)
                       : frag_bf16_mnmajor_asm<512>(rB, wc * 64 + j * 16, 0, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = AK ? g4_frag_k(rA, wr * 128 + mq * 64 + i * 16 + (lane & 15), lane >> 4)
                   : frag_bf16_mnmajor_asm<512>(rA, wr * 128 + mq * 64 + i * 16, 0, lane);
      const bool iss = !noissue && (ph < 2 ? more : it + 2 < nk);
      if (iss) issue(ph < 2 ? it + 1 : it + 2, 3 - ph);
      // phase 1 retires this tile's k1 regions, phase 3 the next tile's k0 regions
      if (grp == 1 && (ph & 1) && !nowait && !noissue) {
        if (iss) {
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else if (ph == 3 && more) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (!AK) {
#pragma unroll
        for (int i = 0; i < 4; ++i) mn_ready(af[i]);
      }
      if constexpr (!BKM) {
#pragma unroll
        for (int j = 0; j < 4; ++j) mn_ready(bfr[j]);
      }
      // ---- matrix section: one 64x64 quadrant x K=32 ----
      if (prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[mq * 4 + i][j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[mq * 4 + i][j], 0, 0, 0);
      }
      if (prio) __builtin_amdgcn_s_setprio(0);
      if (grp == 0 && (ph & 1) && !nowait && !noissue) {
        if (ph == 1 ? more : it + 2 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (ph == 3 && more) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (stag && wr == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  __syncthreads();

  // ---- epilogue: two 256x128 column halves through LDS (16-byte row stores: the direct
  // 8-byte-store epilogue measured slower on this tile, 69 -> 95 us for a K = 64 M x 1536) ----
  char* Cb = p.C + (zb * p.sC1 + zh * p.sC2) * (p.c_fp32 ? 4 : 2);
  if (p.split_stride > 0 && p.split_k > 1) Cb += (long)blockIdx.z * p.split_stride * 4;
  const char* Rb = p.residual ? p.residual + (zb * p.sR1 + zh * p.sR2) * 2 : nullptr;
  float* cs = (float*)smem;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if ((wc >> 1) == h) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = wr * 128 + i * 16 + (lane >> 4) * 4 + r;
            const int col = (wc & 1) * 64 + j * 16 + (lane & 15);
            cs[row * 128 + (col ^ cs_swz(row))] = acc[i][j][r];
          }
    }
    __syncthreads();
    if (n0 + h * 128 < p.nvalid) epilogue_256x128(p, cs, m0, n0 + h * 128, Cb, Rb, tid);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// gemm256r_kernel: the 256x256 phased kernel for K-major A and B with FULL-ROW LDS regions.
//
// gemm256_kernel's regions are K-halves (256 rows x 64 B): every LDS-DMA piece fetches 16 rows
// of 64-byte half lines.  Here a region is 128 rows x one whole 64-wide K-tile (128 B per row,
// 8 rows x 128 B per DMA piece): A0 = tile rows {0-63, 128-191} (the wave rows of m-half 0),
// A1 = rows {64-127, 192-255}, B0 = columns 0-127, B1 = columns 128-255; chunk swizzle
// (row >> 1) & 7 (conflict-free ds_read_b128 for the 16-lane groups).  Phases run (m-half, k-half)
// = (p >> 1, p & 1): B fragments of both k-halves are read in phases 0-1 and kept in registers
// (bfr[2][4]), so B0 / B1 / A0 are free after phase 1 and A1 after phase 3.  Region schedule,
// one or two per phase: phase 0 of tile t issues A1 of t+1 (read from its phase 2: 6 phases to
// land), phase 2 issues A0 and B0 of t+2 and phase 3 B1 of t+2 (read from phase 0 of t+2: 6 / 5
// phases).  Counted waits, both 8 pieces in the steady state: phase 3 retires the next tile's
// A0 / B0 / B1, phase 1 this tile's A1 (group 1 before its memory-section barrier, group 0 after
// its MFMAs -- before the barrier that precedes the first read, as gemm256_kernel).  Each wave
// drains its own ds_reads (lgkmcnt(0)) before the barrier that ends its memory section, so a
// region is restaged one phase after its last read.  Taps: a 64-wide K-tile lies in one tap
// (conv_c % 64 == 0 for CM > 0; the dispatcher falls back to gemm256_kernel otherwise).
constexpr int G4R_REG = 16384;
__device__ __forceinline__ int g4r_sw(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ bf16x8 g4r_frag(const char* rg, int row, int chunk) {
  return *(const bf16x8*)(rg + row * 128 + ((chunk ^ g4r_sw(row)) << 4));
}

// TR: the MFMA operands swapped (B fragment as the A operand), so a lane's accumulator holds 4
// consecutive OUTPUT COLUMNS of one row; the epilogue then stores straight from registers: an
// exchange between lanes l and l ^ 16 over two row fragments gives each lane 8 consecutive
// columns, written as one 16-byte store (bf16 output, no gate / split; see the dispatcher), with
// no LDS staging and no block barrier.  The products and their order per output are unchanged.
// WN: output columns per wave (64: 256x256 tiles; 48: 256x192 tiles for N = 384 outputs, TR only
// -- the B regions hold 96 columns, and waves 6-7's B pieces fill region rows 96-127, never read).
template <int CM, bool TR = false, int WN = 64>   // CM: 0 plain, 1 / 4 / 5 implicit conv
__global__ void __launch_bounds__(G4_NT, 1) gemm256r_kernel(GemmP p) {
  static_assert(WN == 64 || (WN == 48 && TR), "the 192-wide tile has only the direct epilogue");
  constexpr int NJ = WN / 16, BR = 2 * WN;   // column fragments per wave, B rows per region
  __shared__ __attribute__((aligned(16))) char smem[G4_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int nwg = p.tiles_m * p.tiles_n;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tm = bid / p.tiles_n, tn = bid - tm * p.tiles_n;
  const int m0 = tm * 256, n0 = tn * (4 * WN);
  const int z = p.split_k > 1 ? 0 : blockIdx.z;
  const long zb = z / p.batch_div, zh = z - zb * p.batch_div;
  const char* Ab = p.A + (zb * p.sA1 + zh * p.sA2) * 2;
  const char* Bb = p.B + (zb * p.sB1 + zh * p.sB2) * 2;
  const int K = p.K;
  const int nk_all = (K + 63) / 64;
  int kt0 = 0, kt1 = nk_all;
  if (p.split_k > 1) {
    const int kps = (nk_all + p.split_k - 1) / p.split_k;
    kt0 = blockIdx.z * kps;
    kt1 = min(nk_all, kt0 + kps);
  }
  const int rpu = CM == 4 ? p.conv_t + 2 * p.conv_p : p.conv_t;

  // per-lane DMA state: piece i (0, 1) of region q (A0 / A1) or h (B0 / B1) covers region rows
  // (2 wave + i) * 8 + lane / 8; the lane fetches logical chunk lc[i] of that row
  const i32x4 rsA = make_rsrc(Ab), rsB = make_rsrc(Bb);
  int lc[2];
  int avo[4], at[4], abt[4];
  bool aval[4];
  int bvo[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rho = (2 * wave + i) * 8 + (lane >> 3);
    lc[i] = (lane & 7) ^ g4r_sw(rho);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int idx = q * 2 + i;
      const int row = m0 + (rho < 64 ? rho : rho + 64) + q * 64;
      aval[idx] = row < p.M;
      const int rr = aval[idx] ? row : 0;
      const int b = CM ? rr / rpu : 0;
      abt[idx] = b * p.conv_t;
      at[idx] = rr - b * rpu;
      avo[idx] = aval[idx] ? (int)(((long)rr * p.lda + lc[i] * 8) * 2) : BUF_OOB;
      const int col = n0 + rho + q * BR;
      bvo[idx] = (rho < BR && col < p.N) ? (int)(((long)col * p.ldb + lc[i] * 8) * 2) : BUF_OOB;
    }
  }
  int a_tap = -1;

  auto issueA = [&](int q, int rel) {
    const int k0 = (kt0 + rel) * 64;
    char* dst = smem + (rel & 1) * G4_SLOT + q * G4R_REG + wave * 2048;
    const bool kin = k0 + 64 <= K;
    if constexpr (CM > 0) {
      const int j = k0 / p.conv_c;            // wave-uniform: the K-tile lies in one tap
      const int c0 = k0 - j * p.conv_c;
      if (j != a_tap) {
        a_tap = j;
#pragma unroll
        for (int idx = 0; idx < 4; ++idx) {
          int ts;
          bool ok = aval[idx];
          if (CM == 1) {
            ts = reflect_idx(at[idx] + (j - p.conv_p) * p.conv_dil, p.conv_t);
          } else {
            ts = CM == 5 ? at[idx] + (j - p.conv_p) * p.conv_dil : at[idx] - j;
            ok = ok && ts >= 0 && ts < p.conv_t;
          }
          avo[idx] = ok ? (int)(((long)(abt[idx] + ts) * p.lda + lc[idx & 1] * 8) * 2) : BUF_OOB;
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int vo = (kin || k0 + lc[i] * 8 < K) ? avo[q * 2 + i] : BUF_OOB;
        blds16(rsA, vo, c0 * 2, dst + i * 1024);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int vo = (kin || k0 + lc[i] * 8 < K) ? avo[q * 2 + i] : BUF_OOB;
        blds16(rsA, vo, k0 * 2, dst + i * 1024);
      }
    }
  };
  auto issueB = [&](int h, int rel) {
    const int k0 = (kt0 + rel) * 64;
    char* dst = smem + (rel & 1) * G4_SLOT + (2 + h) * G4R_REG + wave * 2048;
    const bool kin = k0 + 64 <= K;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int vo = (kin || k0 + lc[i] * 8 < K) ? bvo[h * 2 + i] : BUF_OOB;
      blds16(rsB, vo, k0 * 2, dst + i * 1024);
    }
  };

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = kt1 - kt0;
  if (nk > 0) { issueA(0, 0); issueB(0, 0); issueB(1, 0); issueA(1, 0); }
  if (nk > 1) {
    issueA(0, 1); issueB(0, 1); issueB(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // tile 0's A0 / B0 / B1
  } else {
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();   // group 1 runs half a phase behind
  __builtin_amdgcn_sched_barrier(0);

  bf16x8 af[4], bfr[2][NJ];
  // timing switches (experiments build; wrong results): 8 no DMA issue in the loop, 16 no
  // fragment reads in the loop, 64 no setprio, 128 no counted waits in the loop, 512 no read
  // drain before the memory-section barrier, 1024 no barrier after the MFMA section, 2048 no
  // barrier before it, 4096 no epilogue
  const int xf = XFLAGS(p);
  if (xf & 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = g4r_frag(smem, i * 16 + (lane & 15), lane >> 4);
#pragma unroll
    for (int j = 0; j < NJ; ++j) { bfr[0][j] = af[j]; bfr[1][j] = af[j]; }
  }
  for (int it = 0; it < nk; ++it) {
    const char* slot = smem + (it & 1) * G4_SLOT;
    const bool more = it + 1 < nk, more2 = it + 2 < nk;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int mq = ph >> 1, s = ph & 1;
      // ---- memory section: this phase's fragments, the phase's regions of a later tile ----
      if (!(xf & 16)) {
        if (mq == 0) {
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            bfr[s][j] = g4r_frag(slot + (2 + (wc >> 1)) * G4R_REG,
                                 (wc & 1) * WN + j * 16 + (lane & 15), s * 4 + (lane >> 4));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = g4r_frag(slot + mq * G4R_REG, wr * 64 + i * 16 + (lane & 15), s * 4 + (lane >> 4));
      }
      // phase 0's A1 region is issued inside the MFMA section, after the first two fragment
      // rows (same box, 4 x 2 interleaved: step 18.24-18.26 -> 18.16-18.20 ms); phase 2's A0 /
      // B0 or phase 3's B1 moved there measured neutral or slower
      if (!(xf & 8)) {
        if (ph == 2 && more2) { issueA(0, it + 2); issueB(0, it + 2); }
        if (ph == 3 && more2) issueB(1, it + 2);
      }
      if (!(xf & 512)) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else if (xf & 16) asm volatile("" ::: "memory");
      if (wr == 1 && !(xf & 128)) {
        if (ph == 1) {
          if (more) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (ph == 3 && more) {
          if (more2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        }
      }
      if (!(xf & 2048)) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // ---- matrix section: rows mq of this wave x K = 32 ----
      if (!(xf & 64)) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i == 2 && ph == 0) {
          __builtin_amdgcn_sched_barrier(0);
          if (more && !(xf & 8)) issueA(1, it + 1);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[mq * 4 + i][j] =
              TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[s][j], af[i], acc[mq * 4 + i][j], 0, 0, 0)
                 : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[s][j], acc[mq * 4 + i][j], 0, 0, 0);
      }
      if (!(xf & 64)) __builtin_amdgcn_s_setprio(0);
      if (wr == 0 && !(xf & 128)) {
        if (ph == 1) {
          if (more) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (ph == 3 && more) {
          if (more2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        }
      }
      if (!(xf & 1024)) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  __syncthreads();

  // ---- epilogue: as gemm256_kernel (two 256x128 column halves through LDS) ----
  if (XFLAGS(p) & 4096) {   // timing: keep the accumulators live, store nothing
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) asm volatile("" :: "v"(acc[i][j]));
    return;
  }
  char* Cb = p.C + (zb * p.sC1 + zh * p.sC2) * (p.c_fp32 ? 4 : 2);
  if (p.split_stride > 0 && p.split_k > 1) Cb += (long)blockIdx.z * p.split_stride * 4;
  const char* Rb = p.residual ? p.residual + (zb * p.sR1 + zh * p.sR2) * 2 : nullptr;
  if constexpr (TR) {
    // lane row q = lane >> 4: after the swap, even q hold row fragment 2t, odd q fragment 2t+1,
    // columns j*16 + (q >> 1)*8 .. +7
    const int q = lane >> 4;
    const int ncol0 = n0 + wc * WN + (q >> 1) * 8;
    float bv[NJ][8];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = ncol0 + j * 16;
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[j][e] = 0.f;
      if (p.bias && n < p.nvalid) {
        const f32x4 b0 = *(const f32x4*)(p.bias + n), b1 = *(const f32x4*)(p.bias + n + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { bv[j][e] = b0[e]; bv[j][e + 4] = b1[e]; }
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int m = m0 + wr * 128 + (2 * t + (q & 1)) * 16 + (lane & 15);
      const bool mok = m < p.mvalid;
      const float rs = (p.row_scale && mok) ? p.row_scale[m] : 1.f;
      const float rs2 = (p.row_scale_post && mok) ? p.row_scale_post[m] : 1.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // even lane rows keep fragment 2t and take the partner's (lane ^ 16) columns 4..7 of
          // it; odd lane rows keep fragment 2t+1 and take the partner's columns 0..3
          const float own = (q & 1) ? acc[2 * t + 1][j][r] : acc[2 * t][j][r];
          const float give = (q & 1) ? acc[2 * t][j][r] : acc[2 * t + 1][j][r];
          const float got = __shfl_xor(give, 16, 64);
          v[r] = (q & 1) ? got : own;
          v[r + 4] = (q & 1) ? own : got;
        }
        const int n = ncol0 + j * 16;
        if (!mok || n >= p.nvalid) continue;
        float rr[8];
        if (Rb) load8<bf16>(rr, (const bf16*)Rb + (long)m * p.ldr + n, 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = epi_act(v[e] + bv[j][e], p.relu);
          x *= rs;
          if (Rb) x += rr[e];
          v[e] = x * rs2;
        }
        if (p.c_fp32) {
          float* Cf = (float*)Cb + (long)m * p.ldc + n;
          *(f32x4*)Cf = f32x4{v[0], v[1], v[2], v[3]};
          *(f32x4*)(Cf + 4) = f32x4{v[4], v[5], v[6], v[7]};
        } else {
          store8<bf16>((bf16*)Cb + (long)m * p.ldc + n, v, 8);
        }
      }
    }
    return;
  } else {
  float* cs = (float*)smem;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if ((wc >> 1) == h) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = wr * 128 + i * 16 + (lane >> 4) * 4 + r;
            const int col = (wc & 1) * 64 + j * 16 + (lane & 15);
            cs[row * 128 + (col ^ cs_swz(row))] = acc[i][j][r];
          }
    }
    __syncthreads();
    if (n0 + h * 128 < p.nvalid) epilogue_256x128(p, cs, m0, n0 + h * 128, Cb, Rb, tid);
    __syncthreads();
  }
  }
}

// ============================================================================================
// Persistent 256x128 kernel for the short-K GEMMs (K <= 1536, plain K-major A and B: the
// attention projections, the FFN conv2 and the data gradients of the 1x1 weights).
//
// Why: at K = 384 a 256x128 tile is 6 K-tiles of MFMA work, while the non-persistent kernels
// pay, per tile and in series, the first LDS-DMA round trip, the epilogue, and the drain of
// the tile's 64 KiB of stores before the CU takes its next block (one 144 KiB block per CU):
// a K-sweep at fixed M x N put ~45 of the 82 us of the decoder QKV projection in that fixed
// part, while the same stores alone stream at ~6 TB/s (tools/micro/store_bw.hip).
// How: one block per CU walks its tiles through ONE continuous K-tile sequence: the 3-stage
// LDS-DMA ring runs straight across tile boundaries (tile i+1's first K-tiles land while tile
// i finishes), and each tile's epilogue stores straight from the MFMA registers (blocks
// computed transposed: a lane holds 4 consecutive columns of one row) while the next tile's
// loads are in flight.  Epilogue operands (bias, row scales, gate OR residual) are loaded
// before the K-tile prefetch of the tile's last iteration, so waiting for them never waits for
// a younger DMA; epilogue stores and loads go through the buffer resource with out-of-range
// lanes at BUF_OOB, so every epilogue issues exactly 16 stores and the counted vmcnt waits of
// the ring stay exact.  Tiles are split into 8 contiguous chunks, one per XCD (blocks b and
// b + 8 share an XCD), walked row-major so consecutive tiles of a block share the A panel.
// ============================================================================================
typedef __attribute__((ext_vector_type(2))) int i32x2;
__device__ void llvm_raw_buffer_store_v2i32(i32x2 data, i32x4 rsrc, int voffset, int soffset,
                                            int aux) __asm("llvm.amdgcn.raw.buffer.store.v2i32");
__device__ void llvm_raw_buffer_store_v4i32(i32x4 data, i32x4 rsrc, int voffset, int soffset,
                                            int aux) __asm("llvm.amdgcn.raw.buffer.store.v4i32");
__device__ i32x2 llvm_raw_buffer_load_v2i32(i32x4 rsrc, int voffset, int soffset,
                                            int aux) __asm("llvm.amdgcn.raw.buffer.load.v2i32");

// epilogue store instructions per wave per tile (gemm_pk_kernel ST32 / ST16): fp32 one 16-byte
// store per 16x16 block; bf16 one 16-byte store per block PAIR (lanes l and l ^ 16 trade halves)

template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
template <int N>
__device__ __forceinline__ void lgkm_wait() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory"); }

// ------------------------------------------------------------------ gemm_w4b_kernel
// 256 x 32NF output tile on FOUR waves (2 x 2), each wave a 128 x 16NF register tile: 8 x NF
// fragments of v_mfma_f32_16x16x32_bf16 in 32NF accumulator registers, one wave per SIMD --
// NF = 8 is the geometry hipBLASLt runs on these shapes (MT256x256x64, 4 waves); NF = 6 the
// 256 x 192 tile for N = 384 / 768 and for short-M shapes (more tiles for the 256 CUs).  A
// wave reads 8 + NF fragments per 8 NF MFMAs (NF = 8: 0.25 per MFMA; the 8-wave kernels' 128 x
// 64 wave tile: 0.375).  The PMC comparison on the FFN conv1 shape
// (profiles/r05_gemm_vs_hipblaslt_pmc_*.json) put our 8-wave kernels at ~1 VALU and ~2 SALU
// instructions per MFMA, hipBLASLt at 0.19 VALU: here every LDS and source address is a lane
// constant plus an immediate or an SGPR offset, and the main loop holds no VALU besides the
// MFMAs.  Plain K-major operands (A(m,k) = A[m lda + k], B(n,k) = B[n ldb + k]; rows may
// overlap, as in the padded-domain convs), K % 128 == 0; epilogue bias / activation / c_row
// remap; bf16 or fp32 output.  Bytes past a_bytes / b_bytes of an operand read as zeros.
constexpr int W4_NT = 256;

// 256 accumulators live in the accumulator file only when pinned there: through the builtin,
// the allocator parks some in VGPRs and shuttles them (~600 v_accvgpr moves per 128 MFMAs).
// The statement is an MFMA accumulate chain (D = C, whole): no wait states between them; the
// readers after the loop wait behind mfma_drain().
__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_drain() { asm volatile("s_nop 15\n\ts_nop 3" ::: "memory"); }

// epilogue of the 4-wave kernels: lane holds columns n .. n+3 (n = n0 + wn 16NF + 16 j +
// 4 (l >> 4)) of row m = m0 + wm 128 + 16 i + (l & 15); bias, activation, c_row remap.  bf16
// output: fragments j, j+1 are paired by one v_permlane16_swap per dword -- lane row g even
// then holds columns 16 j + 4 g .. +7 and row g odd 16 (j+1) + 4 (g-1) .. +7 -- so every lane
// stores 16 bytes per fragment pair (half the store instructions of the 8-byte form; 16-byte
// aligned rows only, else the 8-byte stores)
template <bool C32, int NF>
__device__ __forceinline__ void w4_epilogue(const GemmP& p, f32x4 (&acc)[8][NF], int m0, int n0,
                                            int wm, int wn, int lane) {
  const int g = lane >> 4, g4 = g * 4;
  f32x4 bv[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int n = n0 + wn * 16 * NF + j * 16 + g4;
    bv[j] = (p.bias && n < p.nvalid) ? *(const f32x4*)(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bool pair16 = !C32 && (NF % 2) == 0 && (p.ldc % 8) == 0 && ((uintptr_t)p.C & 15) == 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + (lane & 15);
    bool ok = m < p.mvalid;
    int mo = m;
    if (p.c_row_t) {
      if (p.c_row_pad >= 0) {
        mo = m + (m / p.c_row_t) * p.c_row_pad;
      } else {   // drop the pad rows of a padded-domain result
        const int L = p.c_row_t - p.c_row_pad, u = m / L;
        ok = ok && m - u * L < p.c_row_t;
        mo = m + u * p.c_row_pad;
      }
    }
    if constexpr (!C32 && (NF % 2) == 0) {
      if (pair16) {   // every lane takes part in the swaps; stores are guarded
        const int odd = g & 1;
#pragma unroll
        for (int jj = 0; jj < NF; jj += 2) {
          u32x2 w[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            f32x4 v = acc[i][jj + h] + bv[jj + h];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = epi_act(v[e], p.relu);
            w[h][0] = (unsigned)__builtin_bit_cast(unsigned short, (bf16)v[0]) |
                      ((unsigned)__builtin_bit_cast(unsigned short, (bf16)v[1]) << 16);
            w[h][1] = (unsigned)__builtin_bit_cast(unsigned short, (bf16)v[2]) |
                      ((unsigned)__builtin_bit_cast(unsigned short, (bf16)v[3]) << 16);
          }
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const auto r = __builtin_amdgcn_permlane16_swap(w[0][d], w[1][d], false, false);
            w[0][d] = r[0];
            w[1][d] = r[1];
          }
          const int n = n0 + wn * 16 * NF + (jj + odd) * 16 + 4 * (g - odd);
          if (ok && n < p.nvalid) {
            bf16* dst = (bf16*)p.C + (long)mo * p.ldc + n;
            if (n + 8 <= p.nvalid) *(u32x4*)dst = u32x4{w[0][0], w[0][1], w[1][0], w[1][1]};
            else *(u32x2*)dst = w[0];
          }
        }
        continue;
      }
    }
    if (!ok) continue;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int n = n0 + wn * 16 * NF + j * 16 + g4;
      if (n >= p.nvalid) continue;
      f32x4 v = acc[i][j] + bv[j];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = epi_act(v[e], p.relu);
      if constexpr (C32) {
        *(f32x4*)((float*)p.C + (long)mo * p.ldc + n) = v;
      } else {
        u32x2 w;
        w[0] = (unsigned)__builtin_bit_cast(unsigned short, (bf16)v[0]) |
               ((unsigned)__builtin_bit_cast(unsigned short, (bf16)v[1]) << 16);
        w[1] = (unsigned)__builtin_bit_cast(unsigned short, (bf16)v[2]) |
               ((unsigned)__builtin_bit_cast(unsigned short, (bf16)v[3]) << 16);
        *(u32x2*)((bf16*)p.C + (long)mo * p.ldc + n) = w;
      }
    }
  }
}

// K in stages of 64 with 128-byte LDS rows, so every LDS-DMA instruction fetches 8 whole
// 128-byte lines (a 32-deep, 4-slot version fetching 16 half lines per instruction measured
// 1330 vs 978 us at 8192^3 and 375 vs 344 us on the FFN conv1 shape).  Two slots of (256 + 32NF)
// x 128 B (NF = 8: 128 KB); a stage is two 32-deep halves.  During half 0 of stage s the
// fragments of half 1 are read (B first); a barrier after row 3 (every wave's B reads of the
// slot retired by a counted lgkmcnt) releases the slot's B image, so the B pieces of stage s+2
// are issued over rows 4-7; then vmcnt (stage s+1 landed), lgkmcnt(0) and the second barrier
// release the A image, whose pieces of stage s+2 go out over half 1 while the fragments of
// (s+1, 0) are read.  On the FFN conv1 shape: 344-347 us; issuing all of a stage's DMA at the
// start of half 1 436 us, two pieces per row over half 1 only (one barrier per stage) 375 us,
// A and B swapped (the last pieces with 1.5 halves to land instead of 1) 357 us -- the vector
// memory path's throughput bounds it, not its latency.  Wave-cycles waiting (SQ_WAIT_ANY):
// 22 % against hipBLASLt's 7 % on the same instruction mix (SQ_ACTIVE_INST_LDS / _VMEM within
// 10 %), MFMA busy 50 vs 76 %.  Row r of an image holds logical chunk c at
// physical chunk c ^ (r & 7): conflict-free for the fragment reads' ds_read_b128 lane groups
// ({0-3, 12-15, 20-27}, ...), and lane-constant for a DMA piece (8 rows x 8 chunks).
// FS2_W4_FLAGS (experiments build; results wrong): 1 no barriers, 2 no DMA, 4 no fragment
// reads -- on the FFN conv1 shape 364 -> 361 / 306 / 331 us, both of the last two 272.
template <bool C32, int NF>
__global__ void __launch_bounds__(W4_NT, 1) gemm_w4b_kernel(GemmP p) {
  constexpr int BNW = 32 * NF;                 // block tile columns
  constexpr int STAGE = (256 + BNW) * 128;     // bytes of one 64-deep stage (A and B images)
  constexpr int NP = 8 + NF;                   // LDS-DMA pieces per wave per stage (A 8, B NF)
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = p.tiles_m * p.tiles_n;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, r8 = nwg & 7;
  const int bid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
  int tm = bid / p.tiles_n, tn = bid - tm * p.tiles_n;
  if (XFLAGS(p) & 8) {   // experiments: column-tile-major order (an XCD's blocks share B tiles)
    tn = bid / p.tiles_m;
    tm = bid - tn * p.tiles_m;
  }
  const int m0 = tm * 256, n0 = tn * BNW;
  const int nst = p.K / 64;

  // DMA piece i of an image = rows 8i .. 8i+7; lane L writes row 8i + (L >> 3) at physical
  // chunk L & 7 = logical chunk (L & 7) ^ (L >> 3)
  const int lc = (lane & 7) ^ (lane >> 3);
  const int voa = ((lane >> 3) * (int)p.lda + lc * 8) * 2;
  const int vob = ((lane >> 3) * (int)p.ldb + lc * 8) * 2;
  i32x4 rsA = make_rsrc(p.A), rsB = make_rsrc(p.B);
  rsA[2] = p.a_bytes;
  rsB[2] = p.b_bytes;
  const int lda8 = (int)p.lda * 16, ldb8 = (int)p.ldb * 16;   // bytes per 8 rows
  const int sa0 = m0 * (int)p.lda * 2, sb0 = n0 * (int)p.ldb * 2;
  // A's byte offset of K-stage st: st * 128, or in the tap-inner order (a_kw) the image row
  // (st % a_kw) further down, channel chunk st / a_kw
  auto aoff = [&](int st) {
    if (!p.a_kw) return st * 128;
    const int q64 = st / p.a_kw;
    return ((st - q64 * p.a_kw) * (int)p.lda + q64 * 64) * 2;
  };
  // DMA piece j (0 .. NP-1) of this wave for the stage at A / B byte offsets ka / kb, into slot
  // base dst.  The raw-buffer range check covers voffset only (the piece's row and K offsets ride
  // in soffset), so a lane whose row is past M (A) or N (B) -- the partial last tile -- gets
  // voffset BUF_OOB and loads zeros instead of reading past the operand
  auto dma = [&](int j, int ka, int kb, char* dst) {
    if (j < 8) {
      const int pi = wave * 8 + j;
      const int vo = (lane >> 3) < p.M - m0 - pi * 8 ? voa : BUF_OOB;
      blds16(rsA, vo, sa0 + pi * lda8 + ka, dst + pi * 1024);
    } else {
      const int pi = wave * NF + j - 8;
      const int vo = (lane >> 3) < p.N - n0 - pi * 8 ? vob : BUF_OOB;
      blds16(rsB, vo, sb0 + pi * ldb8 + kb, dst + 256 * 128 + pi * 1024);
    }
  };
  // fragment reads: lane l, row (l & 15) of a 16-row fragment, logical chunk 4h + (l >> 4)
  const int fr = (lane & 15) * 128;
  const int fl0 = fr + (((lane >> 4) ^ (lane & 7)) << 4);
  const int fl1 = fr + (((4 + (lane >> 4)) ^ (lane & 7)) << 4);
  const int fa = wm * 128 * 128, fb = 256 * 128 + wn * 16 * NF * 128;

  f32x4 acc[8][NF];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[2][8], bfr[2][NF];   // [0]: half 0 of a stage, [1]: half 1

  const int ka1 = aoff(1);
#pragma unroll
  for (int j = 0; j < NP; ++j) dma(j, 0, 0, smem);
#pragma unroll
  for (int j = 0; j < NP; ++j) dma(j, ka1, 128, smem + STAGE);
  vm_wait<NP>();   // stage 0 landed (this wave's pieces)
  __builtin_amdgcn_s_barrier();
  {
    const char* b0 = smem + fl0;
#pragma unroll
    for (int j = 0; j < NF; ++j) bfr[0][j] = *(const bf16x8*)(b0 + fb + j * 2048);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[0][i] = *(const bf16x8*)(b0 + fa + i * 2048);
  }
  const int xf = XFLAGS(p);   // experiments build: 1 no barrier, 2 no DMA, 4 no fragment reads

  // one stage; SL = its slot (compile-time).  Every stage has the same body: the last two
  // issue DMA for stages nst, nst+1 (K offsets past the row: bytes of the next row, or zeros
  // past the operand's extent) into slots no one reads again, and the last reads fragments it
  // never uses -- a branch-free loop, whose accumulators stay in place across the back edge
  auto stage = [&](int s, auto SLc) {
    constexpr int SL = decltype(SLc)::value;
    char* slot = smem + SL * STAGE;
    const char* nslot = smem + (SL ^ 1) * STAGE;
    // half 0: MFMAs on set 0; reads of this stage's half 1 into set 1, B first (three per
    // row: B in rows 0-2, A in rows 2-5); a barrier after row 3 (every wave's B reads of this
    // slot retired: 12 reads issued, NF of them B) releases the slot's B image, whose pieces of
    // stage s+2 go out over rows 4-7
    // the last two stages' DMA (into slots no one reads again) re-fetches stage 0: K offsets past
    // the operand would not be range-checked (soffset)
    const bool live = s + 2 < nst;
    const int kb = live ? (s + 2) * 128 : 0, ka = live ? aoff(s + 2) : 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i >= 4 && !(xf & 2)) {
#pragma unroll
        for (int t = 0; t < NF; ++t)
          if (t * 4 / NF == i - 4) dma(8 + t, ka, kb, slot);
      }
#pragma unroll
      for (int j = 0; j < NF; ++j) mfma_acc(acc[i][j], bfr[0][j], af[0][i]);
      if (!(xf & 4)) {
#pragma unroll
        for (int h = 0; h < 3; ++h) {
          const int r = 3 * i + h;
          if (r < NF) bfr[1][r] = *(const bf16x8*)(slot + fl1 + fb + r * 2048);
          else if (r < NF + 8) af[1][r - NF] = *(const bf16x8*)(slot + fl1 + fa + (r - NF) * 2048);
        }
      }
      if (i == 3) {
        lgkm_wait<12 - NF>();
        if (!(xf & 1)) __builtin_amdgcn_s_barrier();
      }
    }
    vm_wait<NF>();   // stage s+1 landed; the B pieces of s+2 may be in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this slot's reads done
    if (!(xf & 1)) __builtin_amdgcn_s_barrier();
    // half 1: MFMAs on set 1; the A pieces of stage s+2 into this slot, one per row; reads of
    // (s+1, half 0), B first
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (!(xf & 2)) dma(i, ka, kb, slot);
#pragma unroll
      for (int j = 0; j < NF; ++j) mfma_acc(acc[i][j], bfr[1][j], af[1][i]);
      if (!(xf & 4)) {
#pragma unroll
        for (int h = 0; h < 3; ++h) {
          const int r = 3 * i + h;
          if (r < NF) bfr[0][r] = *(const bf16x8*)(nslot + fl0 + fb + r * 2048);
          else if (r < NF + 8) af[0][r - NF] = *(const bf16x8*)(nslot + fl0 + fa + (r - NF) * 2048);
        }
      }
    }
  };
  // two stages per trip (slots 0, 1); K % 128 == 0, so nst is even.  Each trip ends in
  // mfma_drain(): should the compiler copy accumulators on the exit edge, its v_accvgpr reads
  // are spaced from the MFMA statements that wrote them (it does not see them as MFMAs).
  for (int s = 0; s < nst; s += 2) {
    stage(s, std::integral_constant<int, 0>{});
    stage(s + 1, std::integral_constant<int, 1>{});
    mfma_drain();
  }
  vm_wait<0>();   // the last stages' DMA (never read) has landed before the block ends
  w4_epilogue<C32, NF>(p, acc, m0, n0, wm, wn, lane);
}

// MI x NJ: the 16 x 16 blocks of a wave's sub-tile (waves as 4 rows x 2 columns), so one tile is
// (64 MI) x (32 NJ): 4 x 4 = 256 x 128 (the decoder's short-K shapes), 2 x 4 = 128 x 128 and
// 2 x 2 = 128 x 64 for the encoder / predictor shapes (M = 6400), where 256-row tiles left most
// CUs idle (75 tiles of 256 x 128 at N = 384); the 128 x 64 instance needs 72 KiB of LDS, so two
// blocks share a CU.
template <int MI, int NJ>
__global__ void __launch_bounds__(BNT) gemm_pk_kernel(GemmP p) {
  constexpr int TM = 64 * MI, TN = 32 * NJ;
  constexpr int SA = TM * 128, SSTAGE = (TM + TN) * 128;   // A bytes / stage bytes
  constexpr int NPC = MI + NJ / 2;                           // DMA pieces per wave per K-tile
  constexpr int ST32 = MI * NJ, ST16 = MI * NJ / 2;          // epilogue stores per wave
  static_assert(NJ % 2 == 0 && MI >= 1 && 3 * SSTAGE <= BIG_LDS, "pk tile");
  __shared__ __attribute__((aligned(16))) char smem[3 * SSTAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 15, lg = lane >> 4;
  // this block's tiles: chunk [c0, c1) of its XCD, every nbx-th from c0 + local
  const int ntile = p.tiles_m * p.tiles_n;
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, local = blockIdx.x >> 3;
  const int nbx = (G - xcd + 7) >> 3;
  const int c0 = (int)((long)ntile * xcd / 8), c1 = (int)((long)ntile * (xcd + 1) / 8);
  const int mine = local < c1 - c0 ? (c1 - c0 - local + nbx - 1) / nbx : 0;
  const int nk = (p.K + 63) / 64;
  const int total = mine * nk;
  const i32x4 rsA = make_rsrc(p.A), rsB = make_rsrc(p.B), rsC = make_rsrc(p.C);
  const i32x4 rsE = make_rsrc(p.gate ? p.gate : (p.residual ? p.residual : p.C));
  const long lde = p.gate ? p.ldg : p.ldr;
  const bool has_e = p.gate || p.residual;

  // per-lane parts of the DMA addressing (as gemm_big_kernel, plain operands)
  int ar[MI], alc[MI], br[NJ / 2], blc[NJ / 2];
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    ar[i] = (wave * MI + i) * 8 + (lane >> 3);
    alc[i] = (lane & 7) ^ (ar[i] & 7);
  }
#pragma unroll
  for (int i = 0; i < NJ / 2; ++i) {
    br[i] = (wave * (NJ / 2) + i) * 8 + (lane >> 3);
    blc[i] = (lane & 7) ^ (br[i] & 7);
  }
  auto issue = [&](int t, int kt, int stage) {
    const int tile = c0 + local + t * nbx;
    const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
    const int k0 = kt * 64;
    char* la = smem + stage * SSTAGE;
    char* lb = la + SA;
    const bool kin = k0 + 64 <= p.K;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = tm * TM + ar[i];
      const bool ok = row < p.M && (kin || k0 + alc[i] * 8 < p.K);
      blds16(rsA, ok ? ((row * (int)p.lda + alc[i] * 8) * 2) : BUF_OOB, k0 * 2,
             la + (wave * MI + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < NJ / 2; ++i) {
      const int row = tn * TN + br[i];
      const bool ok = row < p.N && (kin || k0 + blc[i] * 8 < p.K);
      blds16(rsB, ok ? ((row * (int)p.ldb + blc[i] * 8) * 2) : BUF_OOB, k0 * 2,
             lb + (wave * (NJ / 2) + i) * 1024);
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // epilogue operands of the current tile
  f32x4 bv[NJ] = {};
  float rs[MI], rs2[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) { rs[i] = 1.f; rs2[i] = 1.f; }
  i32x2 ev[MI][NJ] = {};

  // (t, kt) of iterations it (current), it + 2 (prefetch)
  int t = 0, kt = 0, t2 = 0, kt2 = 0;
  if (total > 0) issue(0, 0, 0);
  if (total > 1) { t2 = nk > 1 ? 0 : 1; kt2 = nk > 1 ? 1 : 0; issue(t2, kt2, 1); }
  if (++kt2 == nk) { kt2 = 0; ++t2; }     // (t2, kt2) = iteration 2
  bool prev_last = false;
  int it = 0;
  // One K-tile iteration.  The tile's second-to-final iteration (LOADS: epilogue operands)
  // and its final one (EPI: epilogue) are separate instantiations, peeled out of the K loop:
  // with the operand loads under a runtime test inside one loop body, the compiler saw them
  // pending across the back edge and put a vmcnt(0) before every re-load -- one full DMA drain
  // per tile (FS2_PK_FLAGS=64 timing runs: FFN conv2 data gradient 100 -> 78 us without it).
  auto step = [&](auto LD, auto EP) __attribute__((always_inline)) {
    constexpr bool LOADS = decltype(LD)::value, EPI = decltype(EP)::value;
    const bool more = it + 1 < total;
    // stage it landed: younger than its NPC pieces are those of it + 1 and, after a tile's
    // epilogue, that epilogue's stores
    if (more) {
      if (!prev_last) vm_wait<NPC>();
      else if (p.c_fp32) vm_wait<NPC + ST32>();
      else vm_wait<NPC + ST16>();
    } else {
      if (!prev_last) vm_wait<0>();
      else if (p.c_fp32) vm_wait<ST32>();
      else vm_wait<ST16>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const int tile = c0 + local + t * nbx;
    const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
    const int mb = tm * TM + wm * 16 * MI, nb = tn * TN + wn * 16 * NJ;
    // epilogue operands one iteration ahead of the epilogue (nk >= 2): issued before this
    // iteration's prefetch, they are retired by the NEXT iteration's stage wait, so the
    // epilogue itself never waits on a load (with nk == 1 they are issued in the same one)
    if constexpr (LOADS) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = nb + 16 * j + 4 * lg;
        bv[j] = (p.bias && n < p.nvalid) ? *(const f32x4*)(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = mb + 16 * i + li;
        const bool in = m < p.mvalid;
        rs[i] = (p.row_scale && in) ? p.row_scale[m] : 1.f;
        rs2[i] = (p.row_scale_post && in) ? p.row_scale_post[m] : 1.f;
        if (has_e) {
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int n = nb + 16 * j + 4 * lg;
            const bool ok = in && n < p.nvalid;
            ev[i][j] = llvm_raw_buffer_load_v2i32(rsE, ok ? ((m * (int)lde + n) * 2) : BUF_OOB, 0, 0);
          }
        }
      }
    }
    const bool pre = it + 2 < total;
    if (pre) {
      issue(t2, kt2, (it + 2) % 3);
      if (++kt2 == nk) { kt2 = 0; ++t2; }
    }
    const char* la = smem + (it % 3) * SSTAGE;
    const char* lb = la + SA;
    bf16x8 af[2][MI], bfr[2][NJ];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < MI; ++i) af[s][i] = frag_bf16_kmajor(la, wm * 16 * MI + i * 16, s, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[s][j] = frag_bf16_kmajor(lb, wn * 16 * NJ + j * 16, s, lane);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[s][j], af[s][i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * (MI + NJ), 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 2 * MI * NJ, 0);
    if constexpr (EPI) {
      if (nk == 1) {   // operands issued this iteration: retire them, keep the prefetch in flight
        if (pre) vm_wait<NPC>(); else vm_wait<0>();
      }
      const bool nost = XFLAGS(p) & 16;   // timing experiments only: no stores (wrong results)
      const bool odd = lg & 1;
      auto fin = [&](int i, int j) {         // epilogue values of block (i, j); acc cleared
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = epi_act(acc[i][j][e] + bv[j][e], p.relu);
          const unsigned w = (unsigned)ev[i][j][e >> 1];
          const float ef = __builtin_bit_cast(float, (e & 1) ? (w & 0xffff0000u) : (w << 16));
          if (p.gate) x = ef > 0.f ? x : 0.f;
          x *= rs[i];
          if (p.residual) x += ef;
          v[e] = x * rs2[i];
        }
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        return v;
      };
      auto pack = [](f32x4 v) {
        return u32x2{(unsigned)__builtin_bit_cast(unsigned short, (bf16)v[0]) |
                         ((unsigned)__builtin_bit_cast(unsigned short, (bf16)v[1]) << 16),
                     (unsigned)__builtin_bit_cast(unsigned short, (bf16)v[2]) |
                         ((unsigned)__builtin_bit_cast(unsigned short, (bf16)v[3]) << 16)};
      };
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = mb + 16 * i + li;
        const bool rowok = m < p.mvalid;
        if (p.c_fp32) {
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int n = nb + 16 * j + 4 * lg;
            const f32x4 v = fin(i, j);
            if (nost) continue;
            llvm_raw_buffer_store_v4i32(__builtin_bit_cast(i32x4, v), rsC,
                                        rowok && n < p.nvalid ? ((m * (int)p.ldc + n) * 4) : BUF_OOB, 0, 0);
          }
          continue;
        }
        // bf16: lanes l and l ^ 16 trade halves of a block pair -> 8 consecutive columns each,
        // one 16-byte store (the CU's store path, not HBM, bounds the 8-byte form)
#pragma unroll
        for (int j = 0; j < NJ; j += 2) {
          const u32x2 a = pack(fin(i, j)), b = pack(fin(i, j + 1));
          const unsigned r0 = (unsigned)__shfl_xor((int)(odd ? a[0] : b[0]), 16, 64);
          const unsigned r1 = (unsigned)__shfl_xor((int)(odd ? a[1] : b[1]), 16, 64);
          const u32x4 o = odd ? u32x4{r0, r1, b[0], b[1]} : u32x4{a[0], a[1], r0, r1};
          const int n0 = nb + 16 * (j + (odd ? 1 : 0)) + 4 * (lg - (odd ? 1 : 0));
          if (nost) continue;
          if (!rowok || n0 + 8 <= p.nvalid || n0 >= p.nvalid) {
            llvm_raw_buffer_store_v4i32(__builtin_bit_cast(i32x4, o), rsC,
                                        rowok && n0 < p.nvalid ? ((m * (int)p.ldc + n0) * 2) : BUF_OOB, 0, 0);
          } else {   // 4 valid columns at the right edge: still ONE store (the count is exact)
            llvm_raw_buffer_store_v2i32(i32x2{(int)o[0], (int)o[1]}, rsC,
                                        ((m * (int)p.ldc + n0) * 2), 0, 0);
          }
        }
      }
    }
    prev_last = EPI;
    if (++kt == nk) { kt = 0; ++t; }
    ++it;
  };
  using F_ = std::false_type;
  using T_ = std::true_type;
  for (int tt = 0; tt < mine; ++tt) {   // nk >= 2 (the dispatcher routes K <= 64 elsewhere)
    for (int k = 0; k < nk - 2; ++k) step(F_{}, F_{});
    step(T_{}, F_{});
    step(F_{}, T_{});
  }
}

// ============================================================================================
// Persistent 256 x BN kernel (BN = 4 * WN = 256 or 192) for the long-K GEMMs with K-major A and
// B: the FFN conv1 forward (implicit reflect conv, K = 9 x 384) and its data gradient over the
// padded domain (K = 9 x 1536, N = 384: 256 x 192 tiles put the decoder's 248 tiles in ONE round
// of the 256 CUs without a K split) -- and the decoder's short-K projections whose tiles fill
// a round (N = 384 / 1152, K = 384 / 1536 at M = 31264), where the continuous K-tile stream
// across tiles and the LDS-staged epilogue operands beat the per-tile kernels.
//
// Why not gemm256_kernel: a K-sweep at M = 31264, N = 1536 (tools/gemm256_ksweep.py) split its
// time into ~25 us per round of tiles (prologue DMA round trip, LDS-staged epilogue and store
// drain, all in series per tile) and a main loop at 1186 TF/s -- 1583 with the LDS-DMA issue
// removed, 1300 when each DMA piece covers whole 128-byte rows.  Its regions hold 32-wide K
// halves, so every global cache line is fetched twice, half at a time, phases apart.
// How:
//  * LDS images with 128-byte rows (one 64-wide K-tile): A 256 x 128 B, B BN x 128 B per slot,
//    2 slots; 16-byte chunk c of row r at c ^ ((r >> 1) & 7) (conflict-free ds_read_b128 of 16
//    rows x one chunk per lane group; the swizzle is applied to the DMA SOURCE address).
//  * DMA units of one K-tile: A0 = rows {0-63, 128-191}, A1 = rows {64-127, 192-255} (2 pieces
//    of 8 rows per wave each), B0 = B rows 0-127 (2 per wave), B1 = B rows 128.. (NB1 per wave).
//  * 4 phases per K-tile, each 16 MFMAs of one 64-row half of the wave's 128 x WN block x
//    K = 32 (ph = 2 * mq + kh); the wave's B fragments for both K halves are read in phase 0.
//    Last reads of a slot: A0 and B in phase 0/1, A1 in phase 3.  Iteration g issues A0(g+1),
//    A1(g+1), B0(g+2), B1(g+2) in phases 0..3 -- each >= 2 phases after the last read of its
//    slot region and 4-6 phases before its first read -- and retires them with counted waits
//    in phase 1 (A1 of g) and phase 3 (A0, B of g+1), never vmcnt(0) inside a tile.
//  * Waves 4-7 run half a phase behind (one extra barrier) so each SIMD pairs one wave's
//    MFMA section with its partner's LDS reads and DMA issue (as gemm256_kernel).
//  * One block per CU walks its tiles (8 contiguous XCD chunks, row-major so consecutive tiles
//    share the A panel) through ONE continuous K-tile stream: the next tile's first K-tiles
//    land while the current one finishes; each tile's epilogue stores straight from the MFMA
//    registers (blocks computed transposed: a lane holds 4 consecutive columns of one row),
//    exactly 8 x NJ buffer stores per wave (out-of-range lanes at BUF_OOB) so the counted waits
//    of the ring stay exact.
// ============================================================================================
__device__ __forceinline__ int ps_sw(int row) { return (row >> 1) & 7; }

// CM: 0 plain, 1 reflect "same" conv, 4 padded-domain conv (dgrad).  EO: 1 = a bf16 [M][N]
// epilogue operand (the ReLU gate OR the residual; plain A, 256 x 192 tiles), loaded into
// registers in the tile's last K-tile ahead of that iteration's DMA.
// BT: 1 = conv_mode 6, the K-major weight gradient over channel-major padded images
// (layout.hip): B row n = (tap j, channel c) reads image row c shifted by j - P columns, i.e.
// a per-lane constant source offset; the source is then only 2-byte aligned, which the
// LDS-DMA takes (tools/micro/dma_unaligned.hip).  The resource base sits BT_GUARD elements
// before B so the first row's negative shifts stay in range (the caller allocates that guard).
// Split-K (BT only): work unit u = (split s, tile), s = u / tiles; split s covers K-tiles
// [s * nk, (s + 1) * nk) of K = split_k * k_per_split and stores its fp32 partial to
// C + s * split_stride (caller sums the slices).  The launch gives every unit its own block
// (units <= grid), so a block's unit, K base and output slice are fixed at entry -- per-tile
// unit arithmetic in the loop spilled SGPRs into VGPR lanes and corrupted the accumulators.
constexpr int BT_GUARD = 64;
template <int CM, int WN, int EO = 0, int BT = 0>
__global__ void __launch_bounds__(BNT, 1) gemm_ps_kernel(GemmP p) {
  constexpr int BN = 4 * WN, NJ = WN / 16;
  constexpr int AIMG = 256 * 128;
  constexpr int SLOT = AIMG + BN * 128;
  constexpr int NB1 = (BN - 128) / 64;     // B1 pieces per wave
  constexpr int S32 = 8 * NJ;              // epilogue stores per wave per tile: fp32 output
  constexpr int S16 = 8 * ((NJ + 1) / 2);  // bf16 output (fragment pairs, one 16-B store each)
  // per-wave epilogue operands of the current tile, LDS-DMA'd at its first K-tile: bias of the
  // wave's WN columns (256 B), row_scale and row_scale_post of its 128 rows (512 B each)
  constexpr int EPW = 1280;
  static_assert(2 * SLOT + 8 * EPW <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[2 * SLOT + 8 * EPW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  char* const epl = smem + 2 * SLOT + wave * EPW;
  const int li = lane & 15, lg = lane >> 4;
  const int ntile = p.tiles_m * p.tiles_n;
  const int nsplit = BT && p.split_k > 1 ? p.split_k : 1;   // compile-time 1 unless BT
  const int nunit = ntile * nsplit;   // BT: <= gridDim.x, one unit per block
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7, local = blockIdx.x >> 3;
  const int nbx = (G - xcd + 7) >> 3;
  const int c0 = (int)((long)nunit * xcd / 8), c1 = (int)((long)nunit * (xcd + 1) / 8);
  const int mine = local < c1 - c0 ? (c1 - c0 - local + nbx - 1) / nbx : 0;
  const int nk = nsplit > 1 ? p.k_per_split / 64 : (p.K + 63) / 64;
  const int total = mine * nk;
  if (total == 0) return;
  // BT: this block's unit (split bt_sp, tile bt_tile), fixed for the whole launch
  const int bt_unit = c0 + local;
  const int bt_sp = BT && nsplit > 1 ? __builtin_amdgcn_readfirstlane(bt_unit / ntile) : 0;
  const int bt_tile = BT ? bt_unit - bt_sp * ntile : 0;
  const int bt_kb = BT ? bt_sp * nk * 64 : 0;
  const i32x4 rsA = make_rsrc(p.A), rsC = make_rsrc(p.C);
  const i32x4 rsB = make_rsrc(BT ? p.B - BT_GUARD * 2 : p.B);
  static_assert(EO == 0 || (CM == 0 && WN == 48), "epilogue operands: plain 256 x 192 only");
  constexpr int EL = EO ? 8 * (WN / 16) : 0;   // operand loads per wave in a tile's last K-tile
  const i32x4 rsE = make_rsrc(EO ? (p.gate ? (const void*)p.gate : (const void*)p.residual)
                                 : (const void*)p.C);
  const long lde = p.gate ? p.ldg : p.ldr;
  const int K = p.K;
  const int rpu = CM == 4 ? p.conv_t + 2 * p.conv_p : p.conv_t;
  const int cpt = CM ? p.conv_c / 64 : 1;   // K-tiles per tap

  // ---- per-lane DMA state.  A pieces q = 0..3 (unit q >> 1, piece q & 1), B pieces 0..3.
  const int prow = lane >> 3;
  // piece base rows (wave-uniform: the LDS-DMA destination goes through M0) and lane rows
  int abase[4], arow[4], alc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int u = wave * 2 + (q & 1);
    abase[q] = (u < 8 ? u * 8 : 128 + (u - 8) * 8) + (q >> 1) * 64;
    arow[q] = abase[q] + prow;
    alc[q] = (lane & 7) ^ ps_sw(arow[q]);
  }
  int bbase[2 + NB1], brow[2 + NB1], blc[2 + NB1];
#pragma unroll
  for (int q = 0; q < 2 + NB1; ++q) {
    bbase[q] = q < 2 ? (wave * 2 + q) * 8 : 128 + (NB1 == 2 ? wave * 2 + (q - 2) : wave) * 8;
    brow[q] = bbase[q] + prow;
    blc[q] = (lane & 7) ^ ps_sw(brow[q]);
  }
  // A stream (units of iteration g + 1): tile ordinal, k-tile, tap, row info, lane offsets
  int a_t = 0, a_kt = -1, a_tap = 0, a_c = 0, a_kb = 0;
  int abt[4], at_[4], aoff[4];
  bool aval[4];
  auto a_point = [&]() {   // lane offsets of the current tap (conv) / row (plain)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (CM == 0) {
        aoff[q] = aval[q] ? ((at_[q] * (int)p.lda + alc[q] * 8) * 2) : BUF_OOB;
      } else {
        int ts;
        bool ok = aval[q];
        if constexpr (CM == 1) {
          ts = reflect_idx(at_[q] + a_tap - p.conv_p, p.conv_t);
        } else {
          ts = at_[q] - a_tap;
          ok = ok && ts >= 0 && ts < p.conv_t;
        }
        aoff[q] = ok ? (((abt[q] + ts) * (int)p.lda + alc[q] * 8) * 2) : BUF_OOB;
      }
    }
  };
  auto a_advance = [&]() {  // to the next iteration of the A stream
    if (++a_kt == nk) { a_kt = 0; ++a_t; }
    if (a_kt == 0 && (!BT || a_t == 0)) {
      const int tile = BT ? bt_tile : c0 + local + a_t * nbx;
      a_kb = bt_kb;
      const int tm = tile / p.tiles_n;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = tm * 256 + arow[q];
        aval[q] = row < p.M;
        const int rr = aval[q] ? row : 0;
        if constexpr (CM == 0) {
          at_[q] = rr;
          abt[q] = 0;
        } else {
          const int b = rr / rpu;
          abt[q] = b * p.conv_t;
          at_[q] = rr - b * rpu;
        }
      }
      a_tap = 0; a_c = 0;
      a_point();
    } else if constexpr (CM != 0) {
      if (++a_c == cpt) { a_c = 0; ++a_tap; a_point(); }
    }
  };
  auto issue_a = [&](int unit, char* slot) {
    const int k0 = a_kb + a_kt * 64;
    const int soff = __builtin_amdgcn_readfirstlane((CM ? a_c * 64 : k0) * 2);   // uniform by construction
    const bool kin = k0 + 64 <= K;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = unit * 2 + j;
      const int vo = (kin || k0 + alc[q] * 8 < K) ? aoff[q] : BUF_OOB;
      blds16(rsA, vo, soff, slot + abase[q] * 128);
    }
  };
  // B stream (units of iteration g + 2)
  int b_t = 0, b_kt = -1, b_kb = 0;
  int boff[2 + NB1];
  auto b_advance = [&]() {
    if (++b_kt == nk) { b_kt = 0; ++b_t; }
    if (!BT && b_kt == 0) {   // BT: one tile per block, offsets set below
      const int tile = c0 + local + b_t * nbx;
      const int tn = tile - (tile / p.tiles_n) * p.tiles_n;
#pragma unroll
      for (int q = 0; q < 2 + NB1; ++q) {
        const int row = tn * BN + brow[q];
        boff[q] = row < p.N ? ((row * (int)p.ldb + blc[q] * 8) * 2) : BUF_OOB;
      }
    }
  };
  if constexpr (BT) {   // the block's one tile: row = (tap j, channel c) reads image row c
    b_kb = bt_kb;       // shifted j - P columns
    const int tn = bt_tile - (bt_tile / p.tiles_n) * p.tiles_n;
#pragma unroll
    for (int q = 0; q < 2 + NB1; ++q) {
      const int row = tn * BN + brow[q];
      const int j = row / p.conv_c, c = row - j * p.conv_c;
      boff[q] = row < p.N ? ((c * (int)p.ldb + blc[q] * 8 + j - p.conv_p + BT_GUARD) * 2)
                          : BUF_OOB;
    }
  }
  auto issue_b = [&](int unit, char* slot) {
    const int k0 = b_kb + b_kt * 64;
    const bool kin = k0 + 64 <= K;
#pragma unroll
    for (int q = unit * 2; q < (unit ? 2 + NB1 : 2); ++q) {
      const int vo = (kin || k0 + blc[q] * 8 < K) ? boff[q] : BUF_OOB;
      blds16(rsB, vo, __builtin_amdgcn_readfirstlane(k0 * 2), slot + AIMG + bbase[q] * 128);
    }
  };

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // epilogue operands of tile ordinal tt: 5 LDS-DMA instructions per wave, always (absent
  // operands at BUF_OOB read zeros), issued at the tile's first K-tile before A0 of the next
  // iteration, so the ring's counted waits retire them long before the epilogue reads them --
  // no vmcnt(0) drain of the ring per tile (global loads there cost ~5-10 us per tile)
  auto issue_epi = [&](int tt) {
    const int tile = BT ? bt_tile : c0 + local + tt * nbx;
    const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
    const int n = tn * BN + wc * WN + 4 * lane;
    const bool bok = p.bias && lane < WN / 4 && n < p.nvalid;
    blds16(make_rsrc(p.bias ? (const void*)p.bias : (const void*)p.C), bok ? n * 4 : BUF_OOB, 0,
           epl);
    const i32x4 r1 = make_rsrc(p.row_scale ? (const void*)p.row_scale : (const void*)p.C);
    const i32x4 r2 = make_rsrc(p.row_scale_post ? (const void*)p.row_scale_post : (const void*)p.C);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = tm * 256 + wr * 128 + 64 * h + lane;
      const bool in = m < p.mvalid;
      llvm_raw_buffer_load_lds(r1, (__attribute__((address_space(3))) uint32_t*)(epl + 256 + 256 * h),
                               4, (p.row_scale && in) ? m * 4 : BUF_OOB, 0, 0, 0);
      llvm_raw_buffer_load_lds(r2, (__attribute__((address_space(3))) uint32_t*)(epl + 768 + 256 * h),
                               4, (p.row_scale_post && in) ? m * 4 : BUF_OOB, 0, 0, 0);
    }
  };
  constexpr int EPI_OPS = 5;

  // prologue: tile 0's epilogue operands, B0, B1, A0, A1 of iteration 0, then B0, B1 of
  // iteration 1 (total >= nk >= 2)
  issue_epi(0);
  b_advance();
  issue_b(0, smem); issue_b(1, smem);
  a_advance();
  issue_a(0, smem); issue_a(1, smem);
  b_advance();
  issue_b(0, smem + SLOT); issue_b(1, smem + SLOT);
  vm_wait<4 + NB1>();      // A0, B of iteration 0
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();   // stagger: waves 4-7 half a phase behind
  __builtin_amdgcn_sched_barrier(0);

  int t = 0, kt = 0;          // tile ordinal / k-tile of iteration g
  bf16x8 af[4], bfr[2][NJ];
  i32x2 ev[EO ? 8 : 1][EO ? NJ : 1];   // EO: the tile's gate / residual values (4 bf16 each)
  for (int g = 0; g < total; ++g) {
    const bool more1 = g + 1 < total, more2 = g + 2 < total;
    const bool first = kt == 0 && g > 0;        // previous iteration ended a tile (stores)
    const bool last = kt == nk - 1;
    char* cur = smem + (g & 1) * SLOT;
    char* nxt = smem + ((g + 1) & 1) * SLOT;
    // the 4 phases as compile-time instances (a run-time phase index would put acc in scratch)
    auto phase = [&](auto PH) {
      constexpr int ph = decltype(PH)::value;
      constexpr int mq = ph >> 1, kh = ph & 1;
      // ---- memory section ----
      if (ph == 0) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const int r = wc * WN + j * 16 + li;
            bfr[h][j] = *(const bf16x8*)(cur + AIMG + r * 128 + (((h * 4 + lg) ^ ps_sw(r)) << 4));
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wr * 128 + mq * 64 + i * 16 + li;
        af[i] = *(const bf16x8*)(cur + r * 128 + (((kh * 4 + lg) ^ ps_sw(r)) << 4));
      }
      if (ph == 0 && first) issue_epi(t);
      if constexpr (EO && ph == 0) {
        if (last) {   // older than this iteration's DMA: the epilogue waits for them, not it
          const int tile = c0 + local + t * nbx;   // EO: no split, unit == tile
          const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
          const int mb = tm * 256 + wr * 128, nb = tn * BN + wc * WN;
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
              const int m = mb + 16 * i + li, n = nb + 16 * j + 4 * lg;
              // inline asm: hipcc's own wait for a builtin load's registers descended to
              // vmcnt(0) -- a drain of the whole DMA ring per tile; the asm
              // loads are retired by the ring's counted waits (phase 3 of this iteration
              // retires everything older than its A0 pieces) and handed back below
              const int vo = (m < p.mvalid && n < p.nvalid) ? ((m * (int)lde + n) * 2) : BUF_OOB;
              asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(ev[i][j]) : "v"(vo), "s"(rsE));
            }
        }
      }
      // phase 0's A0 region of the next K-tile is issued inside the MFMA section, after the
      // first two fragment rows (its counted wait is a phase later, so the counts hold): same
      // box, 3 x 2 interleaved, step 18.17-18.18 -> 17.88-17.92 ms, decoder conv1 data gradient
      // 403-412 -> 394-395 us.  Moving phase 2's B0, phase 1's A1 or phase 3's B1 the same way
      // measured slower
      if (ph == 1 && more1) issue_a(1, nxt);
      if (ph == 2 && more2) { b_advance(); issue_b(0, cur); }
      if (ph == 3 && more2) issue_b(1, cur);
      auto dwait = [&]() {   // wave group 1 before this phase's MFMA section, group 0 after it
        if constexpr (ph == 1) {
          // younger than A1 of this iteration: B of the next one, the previous tile's
          // epilogue stores and this tile's operands (first K-tile), A0 / A1 of the next one
          // (EO: + the operand loads of a tile's last K-tile; nk >= 2, so never also first)
          if (more1) {
            if (EO && last) vm_wait<6 + NB1 + EL>();
            else if (!first) vm_wait<6 + NB1>();
            else if (p.c_fp32) vm_wait<6 + NB1 + S32 + EPI_OPS>();
            else vm_wait<6 + NB1 + S16 + EPI_OPS>();
          } else {
            if (EO && last) vm_wait<EL>();
            else if (!first) vm_wait<0>();
            else if (p.c_fp32) vm_wait<S32 + EPI_OPS>();
            else vm_wait<S16 + EPI_OPS>();
          }
        } else {
          if (more2) vm_wait<4 + NB1>();
          else if (more1) vm_wait<2>();
          else vm_wait<0>();
        }
      };
      if constexpr ((ph & 1) != 0) { if (wr == 1) dwait(); }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // ---- matrix section ----
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i == 2 && ph == 0) {
          __builtin_amdgcn_sched_barrier(0);
          if (more1) { a_advance(); issue_a(0, nxt); }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[mq * 4 + i][j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[kh][j], af[i], acc[mq * 4 + i][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      if constexpr ((ph & 1) != 0) { if (wr == 0) dwait(); }
      if (ph == 3 && last && !(XFLAGS(p) & 32)) {   // flag 32: timing only, no epilogue
        // ---- tile epilogue, straight from the accumulators; operands from the wave's LDS
        // area (landed: retired by the counted waits since the tile's first K-tile) ----
        const int tile = BT ? bt_tile : c0 + local + t * nbx;
        const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
        const int mb = tm * 256 + wr * 128, nb = tn * BN + wc * WN;
        const int soc = BT ? (int)(bt_sp * p.split_stride * 4) : 0;
        if constexpr (EO) {   // the operand loads were retired by this phase's counted wait
#pragma unroll
          for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(ev[i][j]));
        }
        f32x4 bv[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bv[j] = *(const f32x4*)(epl + (16 * j + 4 * lg) * 4);
        float rs[8], rsp[8];   // EO: row_scale and row_scale_post apart (the operand between)
        const float* rs1l = (const float*)(epl + 256);
        const float* rs2l = (const float*)(epl + 768);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int r = 16 * i + li;
          rs[i] = p.row_scale ? rs1l[r] : 1.f;
          rsp[i] = p.row_scale_post ? rs2l[r] : 1.f;
          if constexpr (!EO) rs[i] *= rsp[i];
        }
        // compact, branch-free body (ReLU as a select): the epilogue runs once
        // per tile, so its code is fetched cold every time -- keep it small
        const bool relu = p.relu;
        const bool c32 = p.c_fp32, nost = XFLAGS(p) & 16;
        const bool odd = lg & 1;
        auto fin = [&](int i, int j) {   // epilogue values of fragment (i, j), acc cleared
          f32x4 v = acc[i][j] + bv[j];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (relu ? fmaxf(v[e], 0.f) : v[e]) * rs[i];
          if constexpr (EO) {   // as gemm_pk_kernel: gate select / residual add, then rs2
            const bool gate = p.gate;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const unsigned w = (unsigned)ev[i][j][e >> 1];
              const float ef = __builtin_bit_cast(float, (e & 1) ? (w & 0xffff0000u) : (w << 16));
              v[e] = (gate ? (ef > 0.f ? v[e] : 0.f) : v[e] + ef) * rsp[i];
            }
          }
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          return v;
        };
        auto pack = [](f32x4 v) {
          return u32x2{(unsigned)__builtin_bit_cast(unsigned short, (bf16)v[0]) |
                           ((unsigned)__builtin_bit_cast(unsigned short, (bf16)v[1]) << 16),
                       (unsigned)__builtin_bit_cast(unsigned short, (bf16)v[2]) |
                           ((unsigned)__builtin_bit_cast(unsigned short, (bf16)v[3]) << 16)};
        };
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int m0 = mb + 16 * i + li;
          bool rowok = m0 < p.mvalid;
          // padded-domain output rows (c_row_t): one division per fragment row
          int m = m0;
          if (p.c_row_t) {
            if (p.c_row_pad >= 0) {
              m = m0 + (m0 / p.c_row_t) * p.c_row_pad;
            } else {   // drop the pad rows of a padded-domain result
              const int L = p.c_row_t - p.c_row_pad, u = m0 / L;
              rowok = rowok && m0 - u * L < p.c_row_t;
              m = m0 + u * p.c_row_pad;
            }
          }
          if (c32) {   // a lane's 4 consecutive fp32 columns: one 16-byte store per fragment
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
              const f32x4 v = fin(i, j);
              const int n = nb + 16 * j + 4 * lg;
              const bool ok = rowok && n < p.nvalid && !nost;
              // the slice offset goes into voffset, soffset stays 0: with an SGPR soffset
              // LLVM assumes no VMEM-store-data hazard and inserts no wait before the next
              // write of the store's data VGPRs -- on gfx950 the store then read the NEXT
              // fragment's values in lanes 12-15 of each row group (tools/km_debug.py)
              llvm_raw_buffer_store_v4i32(__builtin_bit_cast(i32x4, v), rsC,
                                          ok ? ((m * (int)p.ldc + n) * 4) + soc : BUF_OOB, 0, 0);
            }
            continue;
          }
          // bf16: lanes l and l ^ 16 trade halves of a fragment pair so each holds 8
          // consecutive columns -> 16-byte stores (the store path, not HBM, bounds this part)
#pragma unroll
          for (int j = 0; j + 1 < NJ; j += 2) {
            const u32x2 a = pack(fin(i, j)), b = pack(fin(i, j + 1));
            const unsigned r0 = (unsigned)__shfl_xor((int)(odd ? a[0] : b[0]), 16, 64);
            const unsigned r1 = (unsigned)__shfl_xor((int)(odd ? a[1] : b[1]), 16, 64);
            const u32x4 o = odd ? u32x4{r0, r1, b[0], b[1]} : u32x4{a[0], a[1], r0, r1};
            const int n0 = nb + 16 * (j + (odd ? 1 : 0)) + 4 * (lg - (odd ? 1 : 0));
            if (nost) {
            } else if (!rowok || n0 + 8 <= p.nvalid || n0 >= p.nvalid) {
              const bool ok = rowok && n0 < p.nvalid;
              llvm_raw_buffer_store_v4i32(__builtin_bit_cast(i32x4, o), rsC,
                                          ok ? ((m * (int)p.ldc + n0) * 2) : BUF_OOB, 0, 0);
            } else {   // 4 valid columns at the right edge
              llvm_raw_buffer_store_v2i32(i32x2{(int)o[0], (int)o[1]}, rsC,
                                          ((m * (int)p.ldc + n0) * 2), 0, 0);
            }
          }
          if constexpr (NJ % 2 == 1) {
            const u32x2 a = pack(fin(i, NJ - 1));
            const int n = nb + 16 * (NJ - 1) + 4 * lg;
            const bool ok = rowok && n < p.nvalid && !nost;
            llvm_raw_buffer_store_v2i32(i32x2{(int)a[0], (int)a[1]}, rsC,
                                        ok ? ((m * (int)p.ldc + n) * 2) : BUF_OOB, 0, 0);
          }
        }
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    phase(std::integral_constant<int, 0>{});
    phase(std::integral_constant<int, 1>{});
    phase(std::integral_constant<int, 2>{});
    phase(std::integral_constant<int, 3>{});
    if (++kt == nk) { kt = 0; ++t; }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();   // balance the stagger
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// compile-time A-operand conv variant for the large-tile kernels: 0 plain, 1 / 4 conv with
// taps aligned to the k-granule, -1 anything else (run-time generic path)
int conv_variant(const GemmP& q, int granule) {
  if (q.conv_mode == 0 || q.conv_mode == 3) return 0;
  if ((q.conv_mode == 1 || q.conv_mode == 4 || q.conv_mode == 5) && q.conv_c % granule == 0)
    return q.conv_mode;
  return -1;
}

template <typename T, bool GA, bool GB>
void launch4(const GemmP& p, dim3 grid, hipStream_t s, int ak, int bk) {
  if (ak && bk) hipLaunchKernelGGL((gemm_kernel<T, true, true, GA, GB>), grid, dim3(NT), 0, s, p);
  else if (ak && !bk) hipLaunchKernelGGL((gemm_kernel<T, true, false, GA, GB>), grid, dim3(NT), 0, s, p);
  else if (!ak && bk) hipLaunchKernelGGL((gemm_kernel<T, false, true, GA, GB>), grid, dim3(NT), 0, s, p);
  else hipLaunchKernelGGL((gemm_kernel<T, false, false, GA, GB>), grid, dim3(NT), 0, s, p);
}

template <typename T>
int launch_gemm(const GemmP& p, int gz, hipStream_t s, int ak, int bk) {
  dim3 grid(p.tiles_m * p.tiles_n, 1, gz);
  if constexpr (sizeof(T) == 2) {
    // bf16: LDS-DMA for both operands, except the reflect-fold dgrad operand (register staged)
    static const bool no_big = getenv_flag("FS2_GEMM_NO_BIG");
    const int tiles_big = ((p.M + BBM - 1) / BBM) * p.tiles_n;
    const int batch = p.split_k > 1 ? 1 : gz;
    // weight-gradient GEMMs (fp32 accumulate, no epilogue ops): the big kernel picks its own
    // K split; split > 1 takes the LDS-staged atomic epilogue (row-contiguous atomics)
    const bool wgrad = p.split_stride == 0 && p.c_fp32 && (p.accumulate || p.split_k > 1) &&
                       batch == 1 && !p.gate &&
                       !p.residual && !p.bias && !p.row_scale && !p.row_scale_post && !p.relu &&
                       p.c_conv_kw == 0 && p.vec_align;
    int split_big = 1;
    if (wgrad) {
      const int nk = (p.K + 63) / 64;
      // ~one round of blocks: fewer K slices halve the fp32 atomics (decoder QKV weight
      // gradient 95 -> 75 us vs two rounds); FS2_WGRAD_BIG_TARGET overrides for A/B runs
      static const int tgt = getenv_int("FS2_WGRAD_BIG_TARGET", 240);
      split_big = max(1, min((tgt + tiles_big - 1) / tiles_big, nk / 8));
    }
    const bool slices = p.split_stride > 0 && p.split_k > 1;  // caller-chosen split, plain stores
    // persistent 256x128 kernel: short-K plain GEMMs (FS2_GEMM_NO_PK=1 restores the per-tile
    // kernels for A/B runs); 32-bit buffer offsets must cover A, B, C and the gate/residual
    static const bool no_pk = getenv_flag("FS2_GEMM_NO_PK");
    const long lim = 0x7fffffffL;
    const long crows = p.c_row_t && p.c_row_pad > 0
                           ? p.mvalid + ((long)p.mvalid / p.c_row_t + 1) * p.c_row_pad
                           : p.mvalid;
    const bool pk_fits = (long)p.M * p.lda * 2 < lim && (long)p.N * p.ldb * 2 < lim &&
                         crows * p.ldc * (p.c_fp32 ? 4 : 2) < lim &&
                         (long)p.mvalid * (p.gate ? p.ldg : p.ldr) * 2 < lim;
    // the large-tile kernels address their operands through 32-bit buffer offsets (per batch
    // entry); operands beyond 2 GiB take the pointer-based 128x128 kernel instead
    const long a_rows = ak ? (long)(p.conv_mode ? p.M + 2L * p.conv_p : p.M) : (long)min(p.K, p.kvalid);
    const long b_rows = bk ? (long)p.N : (long)min(p.K, p.kvalid);
    const bool big_fits = a_rows * p.lda * 2 < lim && b_rows * p.ldb * 2 < lim;
    // persistent 256 x 256 / 256 x 192 kernel: long-K K-major GEMMs without gate / residual
    // operands (FS2_GEMM_NO_PS=1 restores the per-tile kernels for A/B runs)
    static const bool no_ps = getenv_flag("FS2_GEMM_NO_PS");
    // the 4-wave 128 x 128-per-wave kernel: plain K-major GEMMs with wide outputs and long K
    // (FS2_GEMM_W4=0 in the experiments build: the 8-wave kernels, for A/B runs)
    static const bool w4_on = getenv_int("FS2_GEMM_W4", 1) != 0;
    // K >= 2048 and >= 160 tiles: the decoder conv2 forward (K = 1536) measured 52 vs 49 us on
    // the short-K persistent kernel, the encoder's (50 tiles of 256 x 192) 43 us
    static const int w4_min_k = getenv_int("FS2_W4_MIN_K", 2048);
    static const int w4_min_tiles = getenv_int("FS2_W4_MIN_TILES", 160);
    {
      const long a_ext = ak ? (long)(p.M - 1) * p.lda + p.K : 0;
      const long b_ext = bk ? (long)(p.N - 1) * p.ldb + p.K : 0;
      const bool w4 = w4_on && ak && bk && p.conv_mode == 0 && batch == 1 && p.split_k <= 1 &&
                      !p.accumulate && !p.gate && !p.residual && !p.row_scale && !p.row_scale_post &&
                      p.K % 128 == 0 && p.K >= (p.a_kw ? 256 : max(256, w4_min_k)) &&
                      (p.a_kw || (p.N >= 384 && p.M >= 2048)) &&
                      p.nvalid % 4 == 0 && p.ldc % 4 == 0 && p.vec_align &&
                      a_ext * 2 < 0x7fffffffL && b_ext * 2 < 0x7fffffffL &&
                      ((long)p.M + 257) * p.lda * 2 < 0x7fffffffL &&
                      ((long)p.N + 257) * p.ldb * 2 < 0x7fffffffL;
      // tile width by rounds x width over the 256 CUs (ties to the wider tile)
      const int tm4 = (p.M + 255) / 256;
      const int t256 = tm4 * ((p.N + 255) / 256), t192 = tm4 * ((p.N + 191) / 192);
      const bool w192 = (long)((t192 + 255) / 256) * 192 < (long)((t256 + 255) / 256) * 256;
      if (p.a_kw && !w4) return FS2_EINVAL;   // the tap-inner order exists on this kernel only
      if (w4 && ((w192 ? t192 : t256) >= w4_min_tiles || p.a_kw)) {
        GemmP q = p;
        q.tiles_m = tm4;
        q.tiles_n = w192 ? (p.N + 191) / 192 : (p.N + 255) / 256;
        q.a_bytes = (int)(a_ext * 2);
        q.b_bytes = (int)(b_ext * 2);
        q.g4_flags = getenv_int("FS2_W4_FLAGS", 0);
        const dim3 g(q.tiles_m * q.tiles_n);
        if (w192) {
          if (p.c_fp32) hipLaunchKernelGGL((gemm_w4b_kernel<true, 6>), g, dim3(W4_NT), 0, s, q);
          else hipLaunchKernelGGL((gemm_w4b_kernel<false, 6>), g, dim3(W4_NT), 0, s, q);
        } else {
          if (p.c_fp32) hipLaunchKernelGGL((gemm_w4b_kernel<true, 8>), g, dim3(W4_NT), 0, s, q);
          else hipLaunchKernelGGL((gemm_w4b_kernel<false, 8>), g, dim3(W4_NT), 0, s, q);
        }
        FS2_CHECK_LAUNCH();
        return 0;
      }
    }
    if (p.conv_mode == 6) {
      if (!p.vec_align) return FS2_EALIGN;
      GemmP q = p;
      q.g4_flags = getenv_int("FS2_PS_FLAGS", 0);
      q.tiles_m = (p.M + 255) / 256;
      q.tiles_n = (p.N + 255) / 256;
      const int nu = q.tiles_m * q.tiles_n * max(1, p.split_k);
      if (nu > 1024) return FS2_EINVAL;   // one unit per block (gemm_ps_kernel BT)
      const int g = (nu + 7) / 8 * 8;
      hipLaunchKernelGGL((gemm_ps_kernel<0, 64, 0, 1>), dim3(g), dim3(BNT), 0, s, q);
      FS2_CHECK_LAUNCH();
      return 0;
    }
    // FS2_PS_MODES: bit 0 plain, bit 1 reflect conv (fwd), bit 2 padded-domain conv (dgrad).
    // Default 5: in the bench step the unsplit decoder conv1 data gradient gains 0.15-0.2 ms,
    // while the conv1 forward measured 0-0.1 ms slower than gemm256_kernel (A/B runs).
    // Short K (256 <= K < 2048) when the tiles fill at least 200 of the 256 CUs: the decoder's
    // N = 384 / 1152 projections and FFN conv2 forward (M = 31264; tools/pk_bench.py: conv2 fwd
    // 63.8 -> 49.1 us, out_proj 29.1 -> 22.0, in_proj 65.6 -> 52.6); the encoder's 25-row-tile
    // shapes stay on the per-tile kernels (ps 30 -> 43 us).  FS2_PS_MIN_K / FS2_PS_SHORT_TILES
    // override for A/B runs.
    static const int ps_modes = getenv_int("FS2_PS_MODES", 5);
    static const int ps_min_k = getenv_int("FS2_PS_MIN_K", 256);
    static const int ps_short_tiles = getenv_int("FS2_PS_SHORT_TILES", 200);
    const int cm_ps = p.conv_mode == 0 ? 0
                      : ((p.conv_mode == 1 || p.conv_mode == 4) && p.conv_dil == 1 && p.conv_c % 64 == 0
                             ? p.conv_mode : -1);
    const bool ps_on = cm_ps >= 0 && (ps_modes >> (cm_ps == 0 ? 0 : (cm_ps == 1 ? 1 : 2))) & 1;
    // tile width by rounds x width over the 256 CUs (ties to the wider tile)
    const int ps_tm = (p.M + 255) / 256;
    const int ps_t256 = ps_tm * ((p.N + 255) / 256), ps_t192 = ps_tm * ((p.N + 191) / 192);
    // a gate / residual operand (plain A only) takes the 256 x 192 instance (its register budget)
    const bool ps_op = p.gate || p.residual;
    // a gate / residual operand takes the 256 x 192 instance (a 256 x 128 one, free of the
    // spills of this one, measured slower: decoder gated dgrad 105-110 -> 120-122 us, step
    // 18.05-18.11 -> 18.23-18.25 ms, tools/r04_eo.sh)
    const bool ps_w192 = ps_op ||
                         (long)((ps_t192 + 255) / 256) * 192 < (long)((ps_t256 + 255) / 256) * 256;
    const int ps_nt = ps_w192 ? ps_t192 : ps_t256;
    // a padded-domain output (c_row_t) exists only on this kernel: it takes every such GEMM
    const bool ps_k = p.K >= 2048 || (p.K >= max(ps_min_k, 128) && ps_nt >= ps_short_tiles) ||
                      (p.c_row_t && p.K >= 128);
    const bool ps_go = !no_ps && ak && bk && ps_on && batch == 1 && p.split_k <= 1 && p.vec_ok &&
        !p.accumulate && !(p.gate && p.residual) && (!ps_op || cm_ps == 0) && p.relu <= 1 && ps_k &&
        p.N >= 128 && pk_fits;
    if (p.c_row_t && !ps_go) return FS2_EINVAL;
    if (!ps_go && !big_fits && p.conv_mode != 6) {
      if (p.conv_mode == 2) launch4<T, false, true>(p, grid, s, ak, bk);
      else launch4<T, true, true>(p, grid, s, ak, bk);
      FS2_CHECK_LAUNCH();
      return 0;
    }
    if (ps_go) {
      GemmP q = p;
      q.g4_flags = getenv_int("FS2_PS_FLAGS", 0);
      q.tiles_m = ps_tm;
      const bool w192 = ps_w192;
      q.tiles_n = w192 ? (p.N + 191) / 192 : (p.N + 255) / 256;
      const int nt = q.tiles_m * q.tiles_n;
      const int cus = p.max_ctas;
      const int g = nt < cus ? (nt + 7) / 8 * 8 : cus;
      if (w192) {
        if (ps_op) hipLaunchKernelGGL((gemm_ps_kernel<0, 48, 1>), dim3(g), dim3(BNT), 0, s, q);
        else if (cm_ps == 0) hipLaunchKernelGGL((gemm_ps_kernel<0, 48>), dim3(g), dim3(BNT), 0, s, q);
        else if (cm_ps == 1) hipLaunchKernelGGL((gemm_ps_kernel<1, 48>), dim3(g), dim3(BNT), 0, s, q);
        else hipLaunchKernelGGL((gemm_ps_kernel<4, 48>), dim3(g), dim3(BNT), 0, s, q);
      } else {
        if (cm_ps == 0) hipLaunchKernelGGL((gemm_ps_kernel<0, 64>), dim3(g), dim3(BNT), 0, s, q);
        else if (cm_ps == 1) hipLaunchKernelGGL((gemm_ps_kernel<1, 64>), dim3(g), dim3(BNT), 0, s, q);
        else hipLaunchKernelGGL((gemm_ps_kernel<4, 64>), dim3(g), dim3(BNT), 0, s, q);
      }
      FS2_CHECK_LAUNCH();
      return 0;
    }
    // narrow outputs with K >= 1152 (FFN conv2 forward, QKV data gradient) measured faster
    // on the per-tile 256x128 kernel: decoder 70.5 -> 63.6 and 58.3 -> 55.6 us, encoder
    // 33.7 -> 29.5 and 32.7 -> 29.0 (tools/gemm_bench.py, FS2_GEMM_NO_PK A/B);
    // FS2_PK_NARROW=1 keeps them on the persistent kernel
    static const bool pk_narrow = getenv_flag("FS2_PK_NARROW");
    const bool pk_shape = p.K <= 768 || p.N > 512 || pk_narrow;
    const bool pk_ok = !no_pk && ak && bk && p.conv_mode == 0 && batch == 1 && p.split_k <= 1 &&
                       p.vec_ok && !p.accumulate && !(p.gate && p.residual) && p.K > 64 && pk_fits;
    // tile of the persistent short-K kernel: 256 x 128 where those tiles fill most of a round
    // (the decoder's shapes that gemm_ps_kernel does not take); below 160 such tiles (the
    // encoder / predictor shapes, M = 6400) 128 x 128 or 128 x 64 tiles, whichever finishes in
    // fewer per-CU tile-areas (two 128 x 64 blocks share a CU) -- K up to 4096 there, since the
    // per-tile 256 x 128 kernel that takes the narrow long-K shapes fills 75 of the 256 CUs.
    // FS2_PK_CFG = 44 / 24 / 22 forces one for A/B runs.
    int pk_cfg = 0;
    if (pk_ok) {
      const long t44 = (long)((p.M + 255) / 256) * ((p.N + 127) / 128);
      const long t24 = (long)((p.M + 127) / 128) * ((p.N + 127) / 128);
      const long t22 = (long)((p.M + 127) / 128) * ((p.N + 63) / 64);
      // per-CU work in 128 x 128 tile units over the rounds each needs (ties: larger tile)
      const long c44 = (t44 + 255) / 256 * 2, c24 = (t24 + 255) / 256, c22 = (t22 + 511) / 512;
      long best = 1L << 40;
      if (p.K <= 1536 && pk_shape) { pk_cfg = 44; best = c44; }
      if (t44 < 400 && p.K <= 4096) {
        if (c24 < best) { pk_cfg = 24; best = c24; }
        if (c22 < best) { pk_cfg = 22; best = c22; }
      }
      static const int force = getenv_int("FS2_PK_CFG", 0);
      if (force == 44 || force == 24 || force == 22) pk_cfg = force;
    }
    if (pk_cfg) {
      GemmP q = p;
      q.g4_flags = getenv_int("FS2_PK_FLAGS", 0);
      const int TM = pk_cfg == 44 ? 256 : 128, TN = pk_cfg == 22 ? 64 : 128;
      q.tiles_m = (p.M + TM - 1) / TM;
      q.tiles_n = (p.N + TN - 1) / TN;
      const int nt = q.tiles_m * q.tiles_n;
      const int slots = (pk_cfg == 22 ? 2 : 1) * p.max_ctas;   // blocks resident at once (LDS)
      // >= 8 blocks: every XCD chunk needs a block (blocks with no tile exit at once)
      const int g = nt < slots ? (nt + 7) / 8 * 8 : slots;
      if (pk_cfg == 44) hipLaunchKernelGGL((gemm_pk_kernel<4, 4>), dim3(g), dim3(BNT), 0, s, q);
      else if (pk_cfg == 24) hipLaunchKernelGGL((gemm_pk_kernel<2, 4>), dim3(g), dim3(BNT), 0, s, q);
      else hipLaunchKernelGGL((gemm_pk_kernel<2, 2>), dim3(g), dim3(BNT), 0, s, q);
      FS2_CHECK_LAUNCH();
      return 0;
    }
    // 256x256 phased kernel: wide outputs (< 10 % column padding; the QKV projection's
    // N = 1152 pads 11 % and measured 100 vs 85 us on the 256x128 kernel at M = 31264)
    static const bool no256 = getenv_flag("FS2_GEMM_NO256");
    const int tm256 = (p.M + 255) / 256, tn256 = (p.N + 255) / 256;
    const int tiles256 = tm256 * tn256;
    const bool wide = p.N >= 512 && tn256 * 256 * 100 <= p.N * 110;
    int split256 = 1;
    if (wgrad) {
      const int nk = (p.K + 63) / 64;
      split256 = max(1, min((240 + tiles256 - 1) / tiles256, nk / 8));
    }
    // from 150 tiles: the encoder FFN conv1 forward (M = 6400, N = 1536: 150 tiles of 256^2 in
    // one round vs 300 of 256x128 in 1.2 rounds) 122 -> 112 us; FS2_G4_MIN_TILES overrides
    static const int g4_min = getenv_int("FS2_G4_MIN_TILES", 150);
    const bool use256 = !no256 && wide && p.conv_mode != 2 &&
                        ((p.vec_ok && p.split_k <= 1 && tiles256 * batch >= g4_min) ||
                         (slices && p.vec_ok && tiles256 * p.split_k >= 160) ||
                         (wgrad && tiles256 * split256 >= 160));
    if (use256) {
      GemmP q = p;
      q.g4_flags = getenv_int("FS2_G4_FLAGS", 0);
      q.tiles_m = tm256;
      q.tiles_n = tn256;
      int gz2 = slices ? p.split_k : gz;
      if (wgrad) {
        q.k_per_split = ((p.K + split256 - 1) / split256 + 63) / 64 * 64;
        q.split_k = (p.K + q.k_per_split - 1) / q.k_per_split;
        q.vec_ok = q.split_k == 1;
        q.accumulate = 1;
        gz2 = q.split_k;
      }
      dim3 g2(tiles256, 1, gz2);
      const int cm = conv_variant(q, 32);
      // full-row regions (gemm256r_kernel) for K-major A and B with 64-aligned taps;
      // FS2_G4R=0 (experiments build) keeps gemm256_kernel
      static const bool g4r = getenv_int("FS2_G4R", 1) != 0;
      const int cm64 = conv_variant(q, 64);
      if (ak && bk && g4r && cm64 >= 0) {
        // register-direct epilogue (TR): bf16 output, no gate, one K split, 8-column granules
        static const bool g4tr = getenv_int("FS2_G4R_TR", 1) != 0;
        const bool tr = g4tr && q.vec_ok && !q.c_fp32 && !q.gate && q.split_k <= 1 &&
                        q.nvalid % 8 == 0 && q.ldc % 8 == 0 && (!q.residual || q.ldr % 8 == 0) &&
                        (q.relu <= 1) && !q.accumulate;
        if (cm64 == 0 && tr) hipLaunchKernelGGL((gemm256r_kernel<0, true>), g2, dim3(G4_NT), 0, s, q);
        else if (cm64 == 1 && tr) hipLaunchKernelGGL((gemm256r_kernel<1, true>), g2, dim3(G4_NT), 0, s, q);
        else if (cm64 == 0) hipLaunchKernelGGL((gemm256r_kernel<0>), g2, dim3(G4_NT), 0, s, q);
        else if (cm64 == 1) hipLaunchKernelGGL((gemm256r_kernel<1>), g2, dim3(G4_NT), 0, s, q);
        else if (cm64 == 4) hipLaunchKernelGGL((gemm256r_kernel<4>), g2, dim3(G4_NT), 0, s, q);
        else hipLaunchKernelGGL((gemm256r_kernel<5>), g2, dim3(G4_NT), 0, s, q);
      } else if (ak && bk) {
        if (cm == 0) hipLaunchKernelGGL((gemm256_kernel<true, true, 0, 0>), g2, dim3(G4_NT), 0, s, q);
        else if (cm == 1) hipLaunchKernelGGL((gemm256_kernel<true, true, 1, 0>), g2, dim3(G4_NT), 0, s, q);
        else if (cm == 4) hipLaunchKernelGGL((gemm256_kernel<true, true, 4, 0>), g2, dim3(G4_NT), 0, s, q);
        else if (cm == 5) hipLaunchKernelGGL((gemm256_kernel<true, true, 5, 0>), g2, dim3(G4_NT), 0, s, q);
        else hipLaunchKernelGGL((gemm256_kernel<true, true, -1, -1>), g2, dim3(G4_NT), 0, s, q);
      } else if (!ak && !bk) {
        if (q.conv_mode == 3) hipLaunchKernelGGL((gemm256_kernel<false, false, 0, 1>), g2, dim3(G4_NT), 0, s, q);
        else if (q.conv_mode == 0) hipLaunchKernelGGL((gemm256_kernel<false, false, 0, 0>), g2, dim3(G4_NT), 0, s, q);
        else hipLaunchKernelGGL((gemm256_kernel<false, false, -1, -1>), g2, dim3(G4_NT), 0, s, q);
      } else if (ak) {
        hipLaunchKernelGGL((gemm256_kernel<true, false, -1, -1>), g2, dim3(G4_NT), 0, s, q);
      } else {
        hipLaunchKernelGGL((gemm256_kernel<false, true, -1, -1>), g2, dim3(G4_NT), 0, s, q);
      }
      FS2_CHECK_LAUNCH();
      return 0;
    }
    // 256x128 tiles down to 60 of them (M = 6400 encoder / predictor GEMMs: 75 tiles beat the
    // 150 tiles of the 128x128 kernel, e.g. predictor conv fwd 45 -> 31 us); FS2_GEMM_BIG_MIN
    // overrides for A/B runs
    static const int big_min = getenv_int("FS2_GEMM_BIG_MIN", 60);
    const bool use_big = !no_big && p.conv_mode != 2 &&
                         ((p.vec_ok && p.split_k <= 1 && tiles_big * batch >= big_min) ||
                          (slices && p.vec_ok && tiles_big * p.split_k >= 160) ||
                          (wgrad && tiles_big * split_big >= 160));
    if (use_big) {
      GemmP q = p;
      q.g4_flags = getenv_int("FS2_BIG_FLAGS", 0);
      q.tiles_m = (p.M + BBM - 1) / BBM;
      if (wgrad) {
        q.split_k = split_big;
        q.k_per_split = ((p.K + split_big - 1) / split_big + 63) / 64 * 64;
        q.split_k = (p.K + q.k_per_split - 1) / q.k_per_split;
        split_big = q.split_k;
        q.vec_ok = split_big == 1;
        q.accumulate = 1;
      }
      dim3 g2(q.tiles_m * q.tiles_n, 1, wgrad ? split_big : (slices ? p.split_k : gz));
      const int cm = conv_variant(q, 64);
      if (ak && bk) {
        if (cm == 0) hipLaunchKernelGGL((gemm_big_kernel<true, true, 0, 0>), g2, dim3(BNT), 0, s, q);
        else if (cm == 1) hipLaunchKernelGGL((gemm_big_kernel<true, true, 1, 0>), g2, dim3(BNT), 0, s, q);
        else if (cm == 4) hipLaunchKernelGGL((gemm_big_kernel<true, true, 4, 0>), g2, dim3(BNT), 0, s, q);
        else if (cm == 5) hipLaunchKernelGGL((gemm_big_kernel<true, true, 5, 0>), g2, dim3(BNT), 0, s, q);
        else hipLaunchKernelGGL((gemm_big_kernel<true, true, -1, -1>), g2, dim3(BNT), 0, s, q);
      } else if (!ak && !bk) {
        if (q.conv_mode == 3) hipLaunchKernelGGL((gemm_big_kernel<false, false, 0, 1>), g2, dim3(BNT), 0, s, q);
        else if (q.conv_mode == 0) hipLaunchKernelGGL((gemm_big_kernel<false, false, 0, 0>), g2, dim3(BNT), 0, s, q);
        else hipLaunchKernelGGL((gemm_big_kernel<false, false, -1, -1>), g2, dim3(BNT), 0, s, q);
      } else if (ak) {
        hipLaunchKernelGGL((gemm_big_kernel<true, false, -1, -1>), g2, dim3(BNT), 0, s, q);
      } else {
        hipLaunchKernelGGL((gemm_big_kernel<false, true, -1, -1>), g2, dim3(BNT), 0, s, q);
      }
    } else {
      if (p.conv_mode == 2) launch4<T, false, true>(p, grid, s, ak, bk);
      else launch4<T, true, true>(p, grid, s, ak, bk);
    }
  } else {
    launch4<T, false, false>(p, grid, s, ak, bk);
  }
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
  p.conv_dil = d->conv_dil > 1 ? d->conv_dil : 1;
  p.C = (char*)d->C; p.ldc = d->ldc; p.c_fp32 = d->c_fp32; p.c_conv_kw = d->c_conv_kw;
  p.bias = d->bias; p.relu = d->relu;
  p.gate = (const char*)d->gate; p.ldg = d->ldg;
  p.row_scale = d->row_scale;
  p.residual = (const char*)d->residual; p.ldr = d->ldr;
  p.row_scale_post = d->row_scale_post;
  p.accumulate = d->accumulate;
  p.split_k = d->split_k > 1 ? d->split_k : 1;
  p.split_stride = d->split_stride > 0 ? d->split_stride : 0;
  p.batch_div = d->batch_div > 0 ? d->batch_div : 1;
  p.sA1 = d->sA1; p.sA2 = d->sA2; p.sB1 = d->sB1; p.sB2 = d->sB2;
  p.sC1 = d->sC1; p.sC2 = d->sC2; p.sR1 = d->sR1; p.sR2 = d->sR2;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.N + BN - 1) / BN;
  const int batch = d->batch > 1 ? d->batch : 1;
  p.c_row_t = d->c_row_t > 0 ? d->c_row_t : 0;
  p.c_row_pad = p.c_row_t ? d->c_row_pad : 0;
  p.max_ctas = d->max_ctas > 0 && d->max_ctas < 256 ? max(8, d->max_ctas / 8 * 8) : 256;
  p.a_kw = d->a_kw > 0 ? d->a_kw : 0;
  if (p.a_kw && (d->dtype != FS2_BF16 || !d->a_kmajor || !d->b_kmajor || d->conv_mode ||
                 batch > 1 || p.split_k > 1 || p.lda % 64 ||
                 (long)p.a_kw * p.lda != p.K))
    return FS2_EINVAL;
  if (p.c_row_t && (d->dtype != FS2_BF16 || !d->a_kmajor || !d->b_kmajor ||
                    p.conv_mode || batch > 1 || p.split_k > 1 || p.accumulate || p.c_conv_kw))
    return FS2_EINVAL;

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
    if (p.conv_dil > 1 && p.conv_mode != 1 && p.conv_mode != 5) return FS2_EINVAL;
    if ((p.conv_mode == 1 || p.conv_mode == 2 || p.conv_mode == 3) && p.conv_p * p.conv_dil >= p.conv_t)
      return FS2_EINVAL;  // reflect pad needs pad < T
    if ((p.conv_mode == 1 || p.conv_mode == 2 || p.conv_mode == 5) && (!d->a_kmajor || p.K != p.conv_kw * p.conv_c))
      return FS2_EINVAL;
    if ((p.conv_mode == 1 || p.conv_mode == 2 || p.conv_mode == 5) && (p.M % p.conv_t)) return FS2_EINVAL;
    if (p.conv_mode == 4 && (p.M % (p.conv_t + 2 * p.conv_p))) return FS2_EINVAL;
    if (p.conv_mode == 4 && !d->a_kmajor) return FS2_EINVAL;
    if (p.conv_mode == 4 && p.K != p.conv_kw * p.conv_c) return FS2_EINVAL;
    if (p.conv_mode == 3 && (d->b_kmajor || p.N != p.conv_kw * p.conv_c)) return FS2_EINVAL;
    if (p.conv_mode == 6) {   // K-major weight gradient over padded channel-major images
      if (d->dtype != FS2_BF16 || !d->a_kmajor || !d->b_kmajor || !p.c_fp32 ||
          p.N != p.conv_kw * p.conv_c || (p.K % 64) || p.bias || p.gate || p.residual ||
          p.row_scale || p.row_scale_post || p.relu || p.c_conv_kw || batch > 1 || p.accumulate)
        return FS2_EINVAL;
      if (p.split_k > 1 && (p.split_stride <= 0 || (p.K % (64 * p.split_k)))) return FS2_EINVAL;
      const long lim = 0x7fffffffL;
      if ((long)p.M * p.lda * 2 >= lim || ((long)p.conv_c * p.ldb + 2 * BT_GUARD) * 2 >= lim ||
          (long)p.split_k * (p.split_stride + (long)p.mvalid * p.ldc) * 4 >= lim)
        return FS2_EINVAL;
    }
  }
  if (p.c_conv_kw > 0 && (p.N % p.c_conv_kw)) return FS2_EINVAL;
  int split_req = p.split_k;
  if (p.split_k > 1) {
    if (!p.c_fp32 || batch > 1) return FS2_EINVAL;
    if (p.split_stride > 0 && (p.accumulate || p.split_stride < (long)(p.mvalid - 1) * p.ldc + p.nvalid))
      return FS2_EINVAL;
    // k-tiles per split (64-wide for bf16 in both kernels, 32 for fp32)
    const int nkt = (p.K + bk - 1) / bk;
    const int kps = (nkt + p.split_k - 1) / p.split_k;
    p.k_per_split = kps * bk;
    p.split_k = (nkt + kps - 1) / kps;
  }
  if (p.accumulate && !p.c_fp32) return FS2_EINVAL;
  {
    const int oes = p.c_fp32 ? 4 : es;
    const int ov = 16 / oes;  // output elements per 16 bytes
    bool v = p.c_conv_kw == 0 && aligned16(p.C) && (p.ldc % 8) == 0;
    if (batch > 1) v = v && ((p.sC1 | p.sC2) % ov) == 0 && ((p.sR1 | p.sR2) % epc) == 0;
    if (p.bias) v = v && aligned16(p.bias);
    if (p.gate) v = v && aligned16(p.gate) && (p.ldg % 8) == 0;
    if (p.residual) v = v && aligned16(p.residual) && (p.ldr % 8) == 0;
    v = v && (p.nvalid % 4) == 0;   // 4-column lane groups of the direct epilogue
    p.vec_align = v;
    p.vec_ok = v && (p.split_k <= 1 || p.split_stride > 0);
  }
  hipStream_t s0 = (hipStream_t)stream;
  if (p.split_stride > 0) {
    // slices the shortened split leaves unwritten read as zero
    const int oes = p.c_fp32 ? 4 : es;
    for (int z = max(p.split_k, 1); z < split_req; ++z)
      if (hipMemset2DAsync(p.C + (long)z * p.split_stride * oes, p.ldc * oes, 0,
                           (size_t)p.nvalid * oes, p.mvalid, s0) != hipSuccess)
        return FS2_EINVAL;
    if (p.split_k <= 1) p.split_stride = 0;
  }
  const int gz = p.split_k > 1 ? p.split_k : batch;
  hipStream_t s = (hipStream_t)stream;
  if (d->dtype == FS2_BF16) return launch_gemm<bf16>(p, gz, s, d->a_kmajor, d->b_kmajor);
  if (d->dtype == FS2_F32) return launch_gemm<float>(p, gz, s, d->a_kmajor, d->b_kmajor);
  return FS2_EINVAL;
}
