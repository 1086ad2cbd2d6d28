// Fused multi-head self-attention (bf16, MFMA) for the FFT blocks: forward and backward
// without materialising the (B*H, T, T) score / probability tensors.
//
// Replaces, for the bf16 train path, the QK^T GEMM + masked softmax + dropout + PV GEMM of
// torch nn.MultiheadAttention as SB calls it (model.py:338-346, 411-427),
// with the reference's head-major mask tiling: for z = b*H + h the key k is
// masked iff key_pad[b][k] | key_pad[(b*H + h) % B][k] (mask_mode 1), or with plain key padding
// key_pad[b][k] (mask_mode 0: the IntensityExtractor's MHA, rank_model/model.py:35).  Dropout on the probabilities uses
// the same pair hash (fs2_keep_fast) and element index ((z*T + q)*round_up(T, 2) + k) as the
// materialised path (attention.hip), so both paths draw identical masks.
//
// Layout: Q, K, V are column blocks of the packed projection QKV [B*T][ldq] (q | k | v, head
// h at columns h*dh of each block); the context O is [B*T][ldo] with head h at h*dh.
//
// MFMA orientation (v_mfma_f32_16x16x32_bf16; C lane layout col = lane&15, rows 4*(lane>>4)+r):
//   forward / dQ:  S^T = K Q^T  -> lanes own queries, so the row softmax statistics, the
//                  log-sum-exp and D = rowsum(dO*O) are per-lane scalars;
//                  O^T += V^T P^T, dQ^T += K^T dS^T take P^T / dS^T straight from registers:
//                  the 32-wide reduction runs over keys {4g..4g+3, 16+4g..16+4g+3} for lane
//                  group g, and the V^T / K^T fragments are read with ds_read_b64_tr_b16 over
//                  the same key rows (the order of a reduction's terms is free).
//   dK, dV:        S = Q K^T  -> lanes own keys; dV += P^T dO, dK += dS^T Q likewise.
// LDS tiles [rows][dh] bf16 with 16-byte chunk c stored at c ^ (row & 7): conflict-free for
// both the ds_read_b128 (row-major fragment) and the ds_read_b64_tr_b16 (transposed) reads.
#include <cstdlib>
#include <type_traits>

#include "fs2_common.h"

typedef __attribute__((ext_vector_type(4))) int i32x4;
__device__ void llvm_raw_buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) uint32_t* lds,
                                         int size, int voffset, int soffset, int offset,
                                         int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

namespace {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
constexpr float LOG2E = 1.4426950408889634f;
constexpr int TMAX = 2048;

struct AttnP {
  const bf16* qkv; long ldq;
  const uint8_t* kpad;
  int tiled;                     // mask_mode: 1 head-major tiling quirk, 0 plain padding
  const bf16* o; long ldo;       // forward: written; backward: read
  bf16* out; long ldout;         // forward: O
  const bf16* dout; long lddo;   // backward: dO
  bf16* dqkv; long lddq;         // backward: dQ | dK | dV
  float* lse;                    // [B*H][T], log2 domain of the scaled scores
  float* dsum;                   // [B*H][T], D = rowsum(dO * O)
  int B, H, T, D;
  float scale, scale_log2, p_drop, inv_keep;
  uint32_t seed, salt;
  uint32_t thr16;                // dropout threshold (fs2_thr16)
  int xflags;                    // FS2_ATTN_FLAGS (experiments build only: timing bits, WRONG results)
};

__device__ __forceinline__ bf16x8 ld_frag(const bf16* g) { return *(const bf16x8*)g; }

// 2^x as the bare v_exp_f32 (exp2f adds a denormal range fix-up and, under a select, a branch
// per element; softmax probabilities below 2^-126 are zero either way).  Every kernel of this
// file uses it, so forward and backward recompute identical probabilities.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// row-major fragment: 8 consecutive features (chunk) of one row
__device__ __forceinline__ bf16x8 lds_row_frag(const char* t, int rowbytes, int row, int chunk) {
  return *(const bf16x8*)(t + row * rowbytes + ((chunk ^ (row & 7)) << 4));
}

// transposed fragment for an A operand A[m = feature][k = row] over the 32 rows
// {4g..4g+3, 16+4g..16+4g+3} + rbase of lane group g, features m0..m0+15
__device__ __forceinline__ bf16x8 lds_tr_frag(const char* t, int rowbytes, int rbase, int m0,
                                              int lane) {
  const int li = lane & 15, g = lane >> 4, q = li >> 2, p = li & 3;
  const int m = m0 + 4 * p;
  const int c = m >> 3, boff = (m & 7) * 2;
  const int k1 = rbase + 4 * g + q, k2 = k1 + 16;
  const char* a1 = t + k1 * rowbytes + ((c ^ (k1 & 7)) << 4) + boff;
  const char* a2 = t + k2 * rowbytes + ((c ^ (k2 & 7)) << 4) + boff;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a2);
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// The same transposed fragment read through inline asm.  hipcc's waitcnt pass treats a
// ds_read_tr16_b64 builtin as a read that may alias ANY in-flight LDS-DMA and puts an
// s_waitcnt vmcnt(0) in front of it -- which drained the next tile's K/V (Q/dO) prefetch in the
// middle of every tile (profiles/r04_attention_pmc.json: SQ_WAIT_ANY 44-51 % of wave cycles).
// The asm read is invisible to that pass; its results are retired by lds_wait<N> below.
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
struct TrFrag { s16x4 lo, hi; };
__device__ __forceinline__ void lds_tr_frag_issue(TrFrag& f, const char* t, int rowbytes, int rbase,
                                                  int m0, int lane) {
  const int li = lane & 15, g = lane >> 4, q = li >> 2, p = li & 3;
  const int m = m0 + 4 * p;
  const int c = m >> 3, boff = (m & 7) * 2;
  const int k1 = rbase + 4 * g + q, k2 = k1 + 16;
  const char* a1 = t + k1 * rowbytes + ((c ^ (k1 & 7)) << 4) + boff;
  const char* a2 = t + k2 * rowbytes + ((c ^ (k2 & 7)) << 4) + boff;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f.lo) : "v"(lds_off(a1)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f.hi) : "v"(lds_off(a2)));
}
__device__ __forceinline__ bf16x8 tr_val(const TrFrag& f) {
  const s16x8 v = {f.lo[0], f.lo[1], f.lo[2], f.lo[3], f.hi[0], f.hi[1], f.hi[2], f.hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// retire all but the N youngest LDS reads; the fragments named are the ones being consumed
template <int N>
__device__ __forceinline__ void lds_wait(TrFrag& a, TrFrag& b) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a.lo), "+v"(a.hi), "+v"(b.lo), "+v"(b.hi) : "n"(N));
}

// rows [r0, r0 + NR) of a [rows][DH] column block starting at src (row pitch ld) -> LDS tile
template <int DH, int NR>
__device__ __forceinline__ void load_tile(char* t, const bf16* src, long ld, int r0, int nrows,
                                          int tid, int nthreads) {
  constexpr int CPR = DH / 8;
  for (int i = tid; i < NR * CPR; i += nthreads) {
    const int r = i / CPR, c = i - r * CPR;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (r0 + r < nrows) v = *(const u32x4*)(src + (long)(r0 + r) * ld + c * 8);
    *(u32x4*)(t + r * DH * 2 + ((c ^ (r & 7)) << 4)) = v;
  }
}

// Buffer-resource LDS-DMA (buffer_load_dwordx4 ... lds): wave-uniform base, 32-bit lane
// offset, lanes at BUF_OOB load zeros.
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

// 4-byte variant: 64 lanes x 4 B land contiguously (one float per lane, e.g. a row statistic)
__device__ __forceinline__ void blds4(i32x4 rsrc, int voff, int soff, char* lds_wave_base) {
  llvm_raw_buffer_load_lds(rsrc, (__attribute__((address_space(3))) uint32_t*)lds_wave_base, 4,
                           voff, soff, 0, 0);
}

// A 64-row x DH tile image (16-byte chunk c of row r stored at c ^ (r & 7)) filled by LDS-DMA:
// 1 KiB instruction i covers image bytes [1024 i, 1024 i + 1024) and each lane fetches the
// logical chunk that lands at its slot.  NW waves issue NI / NW instructions each.
template <int DH, int NW>
struct TileDma {
  static constexpr int NI = 64 * DH * 2 / 1024;
  static constexpr int PER = NI / NW;
  static_assert(NI % NW == 0, "tile instructions must split evenly over the waves");
  int lane16;   // lane * 16: the per-lane byte offset inside each 1 KiB instruction
  __device__ __forceinline__ void init(int, int lane, long) { lane16 = lane * 16; }
  // rows r0 .. r0+63 of the column block (rows >= nrows read zeros); slots are recomputed per
  // call (a few VALU per instruction) to keep the register budget for the MFMA work
  __device__ __forceinline__ void issue(char* tile, i32x4 rs, long ld, int r0, int nrows,
                                        int wave) const {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int o = (wave + j * NW) * 1024 + lane16;
      const int r = o / (DH * 2), cp = (o - r * DH * 2) >> 4;
      const int vo = (r * (int)ld + (cp ^ (r & 7)) * 8) * 2;
      blds16(rs, r0 + r < nrows ? vo : BUF_OOB, (int)((long)r0 * ld * 2),
             tile + (wave + j * NW) * 1024);
    }
  }
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

__device__ __forceinline__ bf16x8 pack8(const float* a, const float* b) {
  bf16x8 r;
  r[0] = (bf16)a[0]; r[1] = (bf16)a[1]; r[2] = (bf16)a[2]; r[3] = (bf16)a[3];
  r[4] = (bf16)b[0]; r[5] = (bf16)b[1]; r[6] = (bf16)b[2]; r[7] = (bf16)b[3];
  return r;
}

// Explicit LDS addressing for the swizzled [rows][DH] tiles (chunk c of row r at c ^ (r & 7)):
// one per-lane VGPR base per parity / residue class and the rest as the instruction's 16-bit
// immediate offset.  Left to itself the compiler hoisted one per-lane address per fragment out
// of the tile loop (24 row-fragment + 48 transposed-read addresses) and spilled.
//   row fragment (16 rows from row0, 32-dim step s): row0 * RB + s * 64 + rbase[s & 1]
//   (chunk (4s + g) ^ l7 = 4 (s ^ (l7 >> 2)) + (g ^ (l7 & 3)), l7 = lane & 7)
__device__ __forceinline__ void row_frag_bases(int lane, int rb, int (&base)[2]) {
  const int li = lane & 15, g = lane >> 4, l7 = lane & 7, hb = l7 >> 2;
  const int c = li * rb + ((g ^ (l7 & 3)) << 4);
  base[0] = c + hb * 64;    // even s: s ^ 1 = s + 1 where hb = 1
  base[1] = c - hb * 64;    // odd s:  s ^ 1 = s - 1
}
template <int OFF>
__device__ __forceinline__ bf16x8 lds_frag_at(const char* tile, int base) {
  return *(const bf16x8*)(tile + base + OFF);
}
//   transposed fragment (rows rbase .. rbase + 31 as lane groups, features 16 d ..): the
//   address is tbase[d & 3] + rbase * RB + (d & ~3) * 32 (lo) and + 16 RB (hi)
__device__ __forceinline__ void tr_frag_bases(int lane, int rb, int (&base)[4]) {
  const int li = lane & 15, g = lane >> 4, q = li >> 2, pp = li & 3;
  const int x = (4 * g + q) & 7, y = x >> 1;
  const int c = (4 * g + q) * rb + ((((pp >> 1) ^ (x & 1))) << 4) + ((pp & 1) * 4) * 2;
#pragma unroll
  for (int dd = 0; dd < 4; ++dd) base[dd] = c + ((dd ^ y) << 5);
}
// (the builtin: an asm read's result is a plain value to the compiler, which may copy it into
// the MFMA's operand quad before the counted wait that retires it -- it did, here)
template <int OFF, int RBYTES>
__device__ __forceinline__ bf16x8 lds_tr_frag_at(const char* tile, int base) {
  const char* a = tile + base + OFF;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a + 16 * RBYTES));
  const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// max / sum over the 4 lane groups (lanes l, l ^ 16, l ^ 32, l ^ 48) of a 16x16 C fragment: the
// gfx950 permlane swaps are VALU ops (the __shfl_xor they replace went through ds_bpermute)
__device__ __forceinline__ float xg_max(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v),
                                                  __builtin_bit_cast(unsigned, v), false, false);
  v = fmaxf(__builtin_bit_cast(float, (unsigned)a[0]), __builtin_bit_cast(float, (unsigned)a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v),
                                                  __builtin_bit_cast(unsigned, v), false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)b[0]), __builtin_bit_cast(float, (unsigned)b[1]));
}
__device__ __forceinline__ float xg_sum(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v),
                                                  __builtin_bit_cast(unsigned, v), false, false);
  v = __builtin_bit_cast(float, (unsigned)a[0]) + __builtin_bit_cast(float, (unsigned)a[1]);
  const auto b = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v),
                                                  __builtin_bit_cast(unsigned, v), false, false);
  return __builtin_bit_cast(float, (unsigned)b[0]) + __builtin_bit_cast(float, (unsigned)b[1]);
}

// Store one query row's ND 16-feature blocks (C layout: lane (l & 15) = query, features 16 d +
// 4 g .. +3 in acc[d][qg], g = l >> 4) as bf16, scaled: blocks d, d+1 are paired by one
// v_permlane16_swap per dword, so lane row g even holds features 16 d + 4 g .. +7 and row g odd
// 16 (d+1) + 4 (g-1) .. +7 -- one 16-byte store per block pair instead of two 8-byte ones (the
// 4-wave GEMM's epilogue measured 7 % faster this way).  Every lane takes part in the swaps.
template <int ND, int QG>
__device__ __forceinline__ void store_row_pairs(bf16* row, const f32x4 (&acc)[ND][QG], int qg,
                                                float sc, int g, bool ok) {
  static_assert(ND % 2 == 0, "feature blocks come in pairs");
  const int odd = g & 1;
#pragma unroll
  for (int d = 0; d < ND; d += 2) {
    u32x2 w[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const f32x4 a = acc[d + hh][qg] * sc;
      w[hh][0] = (unsigned)__builtin_bit_cast(unsigned short, (bf16)a[0]) |
                 ((unsigned)__builtin_bit_cast(unsigned short, (bf16)a[1]) << 16);
      w[hh][1] = (unsigned)__builtin_bit_cast(unsigned short, (bf16)a[2]) |
                 ((unsigned)__builtin_bit_cast(unsigned short, (bf16)a[3]) << 16);
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const auto r = __builtin_amdgcn_permlane16_swap(w[0][e], w[1][e], false, false);
      w[0][e] = r[0];
      w[1][e] = r[1];
    }
    if (ok) *(u32x4*)(row + 16 * (d + odd) + 4 * (g - odd)) = u32x4{w[0][0], w[0][1], w[1][0], w[1][1]};
  }
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N)
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// XCD-aware block coordinates: blocks are dispatched round-robin over the 8 XCDs in linear
// order (x fastest), which put the query (or key) blocks of one (b, h) on 8 DIFFERENT XCDs --
// each XCD's L2 then fetched every K/V (Q/dO) tile of every (b, h) from the Infinity Cache:
// ~390 MB per decoder forward against 48 MB of K/V.  Remapped (bijectively, as the GEMMs' T1
// swizzle) so that an XCD's blocks cover whole (b, h) groups, whose tiles its L2 then serves.
__device__ __forceinline__ void attn_block_coords(int& blk, int& z) {
  const int nb = gridDim.x, n = nb * gridDim.y;
  const int orig = blockIdx.x + nb * blockIdx.y;
  const int xcd = orig & 7, q = n >> 3, r = n & 7;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  z = id / nb;
  blk = id - z * nb;
}

// key-valid flags for (b, h); returns the end of the last valid key and sets *kfull to the
// first masked key (keys below it are all valid: the tiles entirely below it skip the per-key
// mask -- with the decoder's length masks that is every tile but the last)
__device__ __forceinline__ int build_kvalid(uint8_t* kval, int* kbuf, const AttnP& p, int b,
                                            int h, int* kfull) {
  const int b2 = p.tiled ? (b * p.H + h) % p.B : b;
  const uint8_t* k1 = p.kpad + (long)b * p.T;
  const uint8_t* k2 = p.kpad + (long)b2 * p.T;
  const int tpad = (p.T + 63) & ~63;   // bytes past T read as masked (word reads of 4 keys)
  if (threadIdx.x == 0) { kbuf[0] = 0; kbuf[1] = tpad; }
  __syncthreads();
  int last = 0, first = tpad;
  for (int j = threadIdx.x; j < tpad; j += blockDim.x) {
    const uint8_t v = j < p.T ? !(k1[j] | k2[j]) : 0;
    kval[j] = v;
    if (v) last = j + 1;
    else first = min(first, j);
  }
  // one LDS atomic per wave: 512 same-address atomics serialised into ~10 k cycles of every
  // block's prologue (tools/attn_stamps.py)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    last = max(last, __shfl_xor(last, o, 64));
    first = min(first, __shfl_xor(first, o, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&kbuf[0], last);
    atomicMin(&kbuf[1], first);
  }
  __syncthreads();
  *kfull = kbuf[1];
  return kbuf[0];
}

// per-lane dropout constants of a query-owning lane (forward, dQ): the fs2_attn_mix inputs of
// its row for the pairs (kt, e) of a tile at key 0 -- tile k0 adds (k0 / 2) * FS2_ATTN_KC
__device__ __forceinline__ void drop_lane_consts(uint32_t (&c)[4][2], uint32_t dkey, uint32_t row,
                                                 int g) {
  const uint32_t rh = fs2_attn_rowhash(dkey, row);
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int e = 0; e < 2; ++e) c[kt][e] = rh + (uint32_t)(kt * 8 + 2 * g + e) * FS2_ATTN_KC;
}

// ------------------------------------------------------------------------------ forward
// block: 16 * W8 queries = (W8 / QG) waves x QG 16-query groups; K/V tiles of 64 keys
// (W8 = 8: 128 queries; W8 = 4 for short sequences, so B*H*ceil(T/64) blocks fill the chip).
// Per-element VALU is what bounds this loop (one 16x16x32 MFMA leaves issue room for two VALU
// instructions): raw scores feed the row max, the scale folds into the exponent's FMA, full
// tiles skip the key mask, and dropout is one add + one 24-bit multiply round per key pair.
template <int DH, int QG, int W8 = 8>
__global__ void __launch_bounds__(W8 * 64 / QG, 1) attn_fwd_kernel(AttnP p) {
  constexpr int NT = W8 * 64 / QG;
  constexpr int NS = DH / 32, ND = DH / 16;
  constexpr int TB = 64 * DH * 2;
  // one LDS array (a second __shared__ object can make hipcc drain the DMA ring early):
  // [tile buffer 0: 2 tensors | tile buffer 1: 2 tensors | kval | kend, kfull]
  __shared__ __attribute__((aligned(16))) char smem[4 * TB + TMAX + 16];
  uint8_t* kval = (uint8_t*)(smem + 4 * TB);
  int* kbuf = (int*)(smem + 4 * TB + TMAX);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  int blk, z;
  attn_block_coords(blk, z);
  const int b = z / p.H, h = z - b * p.H;
  const uint32_t dkey = fs2_drop_key(p.seed, p.salt);
  const bool drop = p.p_drop > 0.f;
  const bf16* Qb = p.qkv + (long)b * p.T * p.ldq + h * DH;
  const bf16* Kb = Qb + p.D;
  const bf16* Vb = Qb + 2 * p.D;
  const float c = p.scale_log2;

  // prologue: the Q fragments, tile 0's K / V DMA and the key-pad bytes issued before anything
  // waits (one memory round trip instead of two in sequence)
  int qi[QG];
  bf16x8 qf[QG][NS];
  uint32_t dc[QG][4][2];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    qi[qg] = blk * (16 * W8) + wave * 16 * QG + qg * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (qi[qg] < p.T) qf[qg][s] = ld_frag(Qb + (long)qi[qg] * p.ldq + 32 * s + 8 * g);
      else qf[qg][s] = bf16x8{};
    }
    drop_lane_consts(dc[qg], dkey, (uint32_t)(z * p.T + qi[qg]), g);
  }
  f32x4 oacc[ND][QG];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int qg = 0; qg < QG; ++qg) oacc[d][qg] = f32x4{0, 0, 0, 0};
  float mrow[QG], lrow[QG];   // raw-score row max, row sum of exp2(c * (s - max))
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) { mrow[qg] = -INFINITY; lrow[qg] = 0.f; }

  // K/V tiles double-buffered through LDS-DMA: tile t+1 streams in while tile t computes
  TileDma<DH, NT / 64> dma;
  dma.init(wave, lane, p.ldq);
  const i32x4 rsK = make_rsrc(Kb), rsV = make_rsrc(Vb);
  dma.issue(smem, rsK, p.ldq, 0, p.T, wave);
  dma.issue(smem + TB, rsV, p.ldq, 0, p.T, wave);
  int kfull;
  const int kend = build_kvalid(kval, kbuf, p, b, h, &kfull);
  const int ntile = (kend + 63) / 64;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // Q fragments and tile 0 resident
  for (int t = 0; t < ntile; ++t) {
    const int k0 = t * 64;
#ifdef FS2_EXPERIMENTS
    const int tb = (p.xflags & 2) ? 0 : t;
#else
    const int tb = t;
#endif
    const char* Ks = smem + (tb & 1) * 2 * TB;
    const char* Vs = Ks + TB;
    if (t + 1 < ntile && tb == t) {
      char* nx = smem + ((t + 1) & 1) * 2 * TB;
      dma.issue(nx, rsK, p.ldq, k0 + 64, p.T, wave);
      dma.issue(nx + TB, rsV, p.ldq, k0 + 64, p.T, wave);
      wait_vmcnt<2 * TileDma<DH, NT / 64>::PER>();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    f32x4 sacc[4][QG];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qg = 0; qg < QG; ++qg) sacc[kt][qg] = f32x4{0, 0, 0, 0};
    // S^T = K Q^T with the K fragments two 32-dim steps ahead of their MFMAs (a 3-deep register
    // ring, order pinned by sched_group_barrier): the compiler's own schedule read each fragment
    // one or two MFMAs ahead, so every MFMA waited out most of an LDS read latency
    bf16x8 kb[3][4];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) kb[s][kt] = lds_row_frag(Ks, DH * 2, kt * 16 + (lane & 15), 4 * s + g);
    static_for<0, NS>([&](auto SI) {
      constexpr int s = decltype(SI)::value;
      if constexpr (s + 2 < NS) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
          kb[(s + 2) % 3][kt] = lds_row_frag(Ks, DH * 2, kt * 16 + (lane & 15), 4 * (s + 2) + g);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      }
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int qg = 0; qg < QG; ++qg)
          sacc[kt][qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kb[s % 3][kt], qf[qg][s], sacc[kt][qg], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4 * QG, 0);
    });
    const bool full = k0 + 64 <= kfull;
    const uint32_t tkc = (uint32_t)(k0 >> 1) * FS2_ATTN_KC;
    bf16x8 pf[QG][2];
#ifdef FS2_EXPERIMENTS
    if (p.xflags & 1) {
#pragma unroll
      for (int qg = 0; qg < QG; ++qg) {
        float pd[4][4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) pd[kt][r] = sacc[kt][qg][r];
        pf[qg][0] = pack8(pd[0], pd[1]);
        pf[qg][1] = pack8(pd[2], pd[3]);
      }
    } else
#endif
#pragma unroll
    for (int qg = 0; qg < QG; ++qg) {
      float v[4][4];
      float mt = -INFINITY;
      if (full) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[kt][r] = sacc[kt][qg][r];
            mt = fmaxf(mt, v[kt][r]);
          }
      } else {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          const uint32_t kw = *(const uint32_t*)(kval + k0 + kt * 16 + 4 * g);   // keys 4g..4g+3
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[kt][r] = (kw >> (8 * r)) & 1u ? sacc[kt][qg][r] : -INFINITY;
            mt = fmaxf(mt, v[kt][r]);
          }
        }
      }
      mt = xg_max(mt);
      const float mnew = fmaxf(mrow[qg], mt);
      const float alpha = mnew == -INFINITY ? 1.f : fexp2((mrow[qg] - mnew) * c);
      const float nmc = mnew == -INFINITY ? 0.f : -mnew * c;
      mrow[qg] = mnew;
      float ls = 0.f;
      float pd[4][4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = fexp2(fmaf(v[kt][r], c, nmc));   // masked: exp2(-inf) = 0
          ls += e;
          pd[kt][r] = e;
        }
      if (drop) {
        // key pair (k0 + 16 kt + 4g + 2e) / 2; the 1 / (1 - p) of the kept probabilities is
        // applied once, to O at the end
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const uint32_t hh = fs2_attn_mix(dc[qg][kt][e] + tkc);
            pd[kt][2 * e] = (hh & 0xffffu) >= p.thr16 ? pd[kt][2 * e] : 0.f;
            pd[kt][2 * e + 1] = (hh >> 16) >= p.thr16 ? pd[kt][2 * e + 1] : 0.f;
          }
      }
      lrow[qg] = lrow[qg] * alpha + ls;
      if (__any(alpha != 1.f)) {   // once the row maxima settle most tiles skip the rescale
#pragma unroll
        for (int d = 0; d < ND; ++d) oacc[d][qg] *= alpha;
      }
      pf[qg][0] = pack8(pd[0], pd[1]);
      pf[qg][1] = pack8(pd[2], pd[3]);
    }
    // O^T += V^T P^T, the V^T fragments (two transposed reads each, asm: see lds_tr_frag_issue)
    // two output blocks ahead of their MFMAs, retired by counted lgkmcnt waits
    TrFrag vb[3][2];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the softmax's LDS reads retired
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int j = 0; j < 2; ++j) lds_tr_frag_issue(vb[d][j], Vs, DH * 2, 32 * j, 16 * d, lane);
    static_for<0, ND>([&](auto DI) {
      constexpr int d = decltype(DI)::value;
      if constexpr (d + 2 < ND) {
#pragma unroll
        for (int j = 0; j < 2; ++j) lds_tr_frag_issue(vb[(d + 2) % 3][j], Vs, DH * 2, 32 * j, 16 * (d + 2), lane);
        lds_wait<8>(vb[d % 3][0], vb[d % 3][1]);
      } else if constexpr (d + 1 < ND) {
        lds_wait<4>(vb[d % 3][0], vb[d % 3][1]);
      } else {
        lds_wait<0>(vb[d % 3][0], vb[d % 3][1]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int qg = 0; qg < QG; ++qg)
          oacc[d][qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_val(vb[d % 3][j]), pf[qg][j], oacc[d][qg], 0, 0, 0);
    });
    __builtin_amdgcn_s_barrier();   // every wave is done with buffer t & 1 before t+2 lands
  }
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    const float l = xg_sum(lrow[qg]);
    const float inv = p.inv_keep / l;
    const bool qok = qi[qg] < p.T;
    if (qok && g == 0) p.lse[(long)z * p.T + qi[qg]] = mrow[qg] * c + log2f(l);
    bf16* orow = p.out + ((long)b * p.T + (qok ? qi[qg] : 0)) * p.ldout + h * DH;
    store_row_pairs<ND>(orow, oacc, qg, inv, g, qok);
  }
}

// ------------------------------------------------------------------------------ backward dQ
// block: 16 * W8 queries = (W8 / QG) waves x QG 16-query groups; also writes D = rowsum(dO * O)
// and the dropout row hash of every query row (workspace) for the dK/dV kernel
template <int DH, int QG, int W8 = 8>
__global__ void __launch_bounds__(W8 * 64 / QG, 1) attn_bwd_dq_kernel(AttnP p) {
  constexpr int NT = W8 * 64 / QG;
  constexpr int NS = DH / 32, ND = DH / 16;
  constexpr int TB = 64 * DH * 2;
  // one LDS array (a second __shared__ object can make hipcc drain the DMA ring early):
  // [tile buffer 0: 2 tensors | tile buffer 1: 2 tensors | kval | kend, kfull]
  __shared__ __attribute__((aligned(16))) char smem[4 * TB + TMAX + 16];
  uint8_t* kval = (uint8_t*)(smem + 4 * TB);
  int* kbuf = (int*)(smem + 4 * TB + TMAX);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  int blk, z;
  attn_block_coords(blk, z);
  const int b = z / p.H, h = z - b * p.H;
  const uint32_t dkey = fs2_drop_key(p.seed, p.salt);
  const bool drop = p.p_drop > 0.f;
  const bf16* Qb = p.qkv + (long)b * p.T * p.ldq + h * DH;
  const bf16* Kb = Qb + p.D;
  const bf16* Vb = Qb + 2 * p.D;
  const float c = p.scale_log2;

  // prologue: the Q / dO / O fragments, lse, tile 0's K / V DMA and the key-pad bytes are all
  // issued before anything waits (one memory round trip instead of three in sequence)
  int qi[QG];
  bf16x8 qf[QG][NS], dof[QG][NS], of[QG][NS];
  float nlse[QG], dsum[QG];
  uint32_t dc[QG][4][2];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    qi[qg] = blk * (16 * W8) + wave * 16 * QG + qg * 16 + (lane & 15);
    const bool in = qi[qg] < p.T;
    const long ro = (long)b * p.T + (in ? qi[qg] : 0);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      qf[qg][s] = in ? ld_frag(Qb + (long)qi[qg] * p.ldq + 32 * s + 8 * g) : bf16x8{};
      dof[qg][s] = in ? ld_frag(p.dout + ro * p.lddo + h * DH + 32 * s + 8 * g) : bf16x8{};
      of[qg][s] = in ? ld_frag(p.o + ro * p.ldo + h * DH + 32 * s + 8 * g) : bf16x8{};
    }
    nlse[qg] = in ? -p.lse[(long)z * p.T + qi[qg]] : 0.f;
  }
  // K/V tiles double-buffered through LDS-DMA: tile t+1 streams in while tile t computes
  TileDma<DH, NT / 64> dma;
  dma.init(wave, lane, p.ldq);
  const i32x4 rsK = make_rsrc(Kb), rsV = make_rsrc(Vb);
  dma.issue(smem, rsK, p.ldq, 0, p.T, wave);
  dma.issue(smem + TB, rsV, p.ldq, 0, p.T, wave);
  int kfull;
  const int kend = build_kvalid(kval, kbuf, p, b, h, &kfull);
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    const bool in = qi[qg] < p.T;
    float dot = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) dot += (float)dof[qg][s][e] * (float)of[qg][s][e];
    dsum[qg] = xg_sum(dot);
    const uint32_t row = (uint32_t)(z * p.T + qi[qg]);
    drop_lane_consts(dc[qg], dkey, row, g);
    if (in && g == 0) {
      p.dsum[(long)z * p.T + qi[qg]] = dsum[qg];
      ((uint32_t*)p.dsum)[(long)p.B * p.H * p.T + (long)z * p.T + qi[qg]] = fs2_attn_rowhash(dkey, row);
    }
  }
  f32x4 qacc[ND][QG];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int qg = 0; qg < QG; ++qg) qacc[d][qg] = f32x4{0, 0, 0, 0};
  const int ntile = (kend + 63) / 64;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // fragments and tile 0 resident
  for (int t = 0; t < ntile; ++t) {
    const int k0 = t * 64;
    const char* Ks = smem + (t & 1) * 2 * TB;
    const char* Vs = Ks + TB;
    if (t + 1 < ntile) {
      char* nx = smem + ((t + 1) & 1) * 2 * TB;
      dma.issue(nx, rsK, p.ldq, k0 + 64, p.T, wave);
      dma.issue(nx + TB, rsV, p.ldq, k0 + 64, p.T, wave);
      wait_vmcnt<2 * TileDma<DH, NT / 64>::PER>();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    f32x4 sacc[4][QG], pacc[4][QG];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qg = 0; qg < QG; ++qg) { sacc[kt][qg] = f32x4{0, 0, 0, 0}; pacc[kt][qg] = f32x4{0, 0, 0, 0}; }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const bf16x8 kf = lds_row_frag(Ks, DH * 2, kt * 16 + (lane & 15), 4 * s + g);
        const bf16x8 vf = lds_row_frag(Vs, DH * 2, kt * 16 + (lane & 15), 4 * s + g);
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) {
          sacc[kt][qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qg][s], sacc[kt][qg], 0, 0, 0);
          pacc[kt][qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, dof[qg][s], pacc[kt][qg], 0, 0, 0);
        }
      }
    const bool full = k0 + 64 <= kfull;
    const uint32_t tkc = (uint32_t)(k0 >> 1) * FS2_ATTN_KC;
    bf16x8 sf[QG][2];
#pragma unroll
    for (int qg = 0; qg < QG; ++qg) {
      float ds[4][4];
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const uint32_t kw = full ? 0x01010101u : *(const uint32_t*)(kval + k0 + kt * 16 + 4 * g);
#pragma unroll
        for (int e2 = 0; e2 < 2; ++e2) {
          const uint32_t hh = drop ? fs2_attn_mix(dc[qg][kt][e2] + tkc) : 0u;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int r = 2 * e2 + e;
            float pr = fexp2(fmaf(sacc[kt][qg][r], c, nlse[qg]));
            if (!full) pr = (kw >> (8 * r)) & 1u ? pr : 0.f;
            float dp = pacc[kt][qg][r];
            if (drop) dp = ((hh >> (16 * e)) & 0xffffu) >= p.thr16 ? dp * p.inv_keep : 0.f;
            ds[kt][r] = pr * (dp - dsum[qg]);
          }
        }
      }
      sf[qg][0] = pack8(ds[0], ds[1]);
      sf[qg][1] = pack8(ds[2], ds[3]);
    }
    // dQ^T += K^T dS^T: K^T fragments by asm transposed reads (no compiler DMA drain), two
    // output blocks ahead of their MFMAs
    TrFrag kb2[3][2];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int j = 0; j < 2; ++j) lds_tr_frag_issue(kb2[d][j], Ks, DH * 2, 32 * j, 16 * d, lane);
    static_for<0, ND>([&](auto DI) {
      constexpr int d = decltype(DI)::value;
      if constexpr (d + 2 < ND) {
#pragma unroll
        for (int j = 0; j < 2; ++j) lds_tr_frag_issue(kb2[(d + 2) % 3][j], Ks, DH * 2, 32 * j, 16 * (d + 2), lane);
        lds_wait<8>(kb2[d % 3][0], kb2[d % 3][1]);
      } else if constexpr (d + 1 < ND) {
        lds_wait<4>(kb2[d % 3][0], kb2[d % 3][1]);
      } else {
        lds_wait<0>(kb2[d % 3][0], kb2[d % 3][1]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int qg = 0; qg < QG; ++qg)
          qacc[d][qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr_val(kb2[d % 3][j]), sf[qg][j], qacc[d][qg], 0, 0, 0);
    });
    __builtin_amdgcn_s_barrier();   // every wave is done with buffer t & 1 before t+2 lands
  }
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    const bool qok = qi[qg] < p.T;
    bf16* row = p.dqkv + ((long)b * p.T + (qok ? qi[qg] : 0)) * p.lddq + h * DH;
    store_row_pairs<ND>(row, qacc, qg, p.scale, g, qok);
  }
}

// ------------------------------------------------------------------------------ backward dK dV
// block: W8 waves x 16 keys; query tiles of 64 (Q, dO, lse, D and the dropout row hashes staged
// in LDS).  Q / dO tiles are double-buffered through LDS-DMA (tile t+1 streams in while tile t
// computes); wave 0 streams tile t+1's lse / D / row-hash rows the same way.  A masked key's
// lane computes unmasked (finite) values and stores zeros; rows past T read zero Q / dO / lse /
// D, so their P = 1 multiplies zero dO and their dS is 0 -- no per-element mask.
template <int DH, int W8 = 8>
__global__ void __launch_bounds__(W8 * 64, 1) attn_bwd_dkv_kernel(AttnP p) {
  constexpr int NS = DH / 32, ND = DH / 16;
  constexpr int TB = 64 * DH * 2;
#ifdef FS2_EXPERIMENTS
  const uint64_t st_entry = __builtin_amdgcn_s_memtime();
#endif
  // one LDS array (a second __shared__ object can make hipcc drain the DMA ring early):
  // [Q 0 | dO 0 | Q 1 | dO 1 | (lse, D, rowhash) 0 | (lse, D, rowhash) 1 | kval | kend, kfull]
  __shared__ __attribute__((aligned(16))) char smem[4 * TB + 1536 + TMAX + 16];
  float* lsd = (float*)(smem + 4 * TB);
  uint8_t* kval = (uint8_t*)(smem + 4 * TB + 1536);
  int* kbuf = (int*)(smem + 4 * TB + 1536 + TMAX);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  int blk, z;
  attn_block_coords(blk, z);
  const int b = z / p.H, h = z - b * p.H;
  const bool drop = p.p_drop > 0.f;
  const bf16* Qb = p.qkv + (long)b * p.T * p.ldq + h * DH;
  const bf16* Kb = Qb + p.D;
  const bf16* Vb = Qb + 2 * p.D;
  const bf16* dOb = p.dout + (long)b * p.T * p.lddo + h * DH;
  const float c = p.scale_log2;

  const int key = blk * (16 * W8) + wave * 16 + (lane & 15);   // this lane's key (B col)
  const bool kin = key < p.T;
  const uint32_t kc = (uint32_t)(key >> 1) * FS2_ATTN_KC;
  // prologue: the K / V fragments, tile 0's Q / dO / stats DMA and the key-pad bytes are all
  // issued before anything waits (one memory round trip instead of three in sequence: the
  // serial prologue took ~22 k cycles of a ~110 k-cycle block, tools/attn_stamps.py)
  bf16x8 kf[NS], vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    kf[s] = kin ? ld_frag(Kb + (long)key * p.ldq + 32 * s + 8 * g) : bf16x8{};
    vf[s] = kin ? ld_frag(Vb + (long)key * p.ldq + 32 * s + 8 * g) : bf16x8{};
  }
  f32x4 dk[ND], dv[ND];
#pragma unroll
  for (int d = 0; d < ND; ++d) { dk[d] = f32x4{0, 0, 0, 0}; dv[d] = f32x4{0, 0, 0, 0}; }

  TileDma<DH, W8> dma;
  dma.init(wave, lane, 0);
  const i32x4 rsQ = make_rsrc(Qb), rsO = make_rsrc(dOb);
  const int ntile_all = (p.T + 63) / 64;
  // lse / D / row-hash rows of a tile: wave 0 streams them in by 4-byte LDS-DMA
  const long BHT = (long)p.B * p.H * p.T;
  const i32x4 rsL = make_rsrc(p.lse + (long)z * p.T), rsD = make_rsrc(p.dsum + (long)z * p.T);
  const i32x4 rsH = make_rsrc(p.dsum + BHT + (long)z * p.T);
  auto issue_stats = [&](int q0, int buf) {
    if (wave == 0) {
      const int vo = q0 + lane < p.T ? lane * 4 : BUF_OOB;
      blds4(rsL, vo, q0 * 4, (char*)(lsd + buf * 192));
      blds4(rsD, vo, q0 * 4, (char*)(lsd + buf * 192 + 64));
      blds4(rsH, vo, q0 * 4, (char*)(lsd + buf * 192 + 128));
    }
  };
  if (ntile_all > 0) {
    issue_stats(0, 0);
    dma.issue(smem, rsQ, p.ldq, 0, p.T, wave);
    dma.issue(smem + TB, rsO, p.lddo, 0, p.T, wave);
  }
  int kfull;
  build_kvalid(kval, kbuf, p, b, h, &kfull);
  const bool kok = kin && kval[key];
  // a block whose keys are all masked contributes nothing: skip the query loop
  const int anyk = __syncthreads_or(kok);
  const int ntile = anyk ? ntile_all : 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // K/V fragments and tile 0 resident
#ifdef FS2_EXPERIMENTS
  // xflags 64 (diagnostic, tools/attn_stamps.py): s_memtime cycles per loop segment, summed
  // over the tiles, written per wave after the workspace's 2*B*H*T floats
  const bool stamps = p.xflags & 64;
  uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0};
  uint64_t st_prev = __builtin_amdgcn_s_memtime();
  const uint64_t st_pro = st_prev - st_entry;
#define FS2_STAMP(i) do { if (stamps) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_prev; st_prev = t_; } } while (0)
#else
#define FS2_STAMP(i) do { } while (0)
#endif
  for (int t = 0; t < ntile; ++t) {
    const int q0 = t * 64;
    const char* Qs = smem + (t & 1) * 2 * TB;
    const char* Os = Qs + TB;
    const float* ls_s = lsd + (t & 1) * 192;
    const float* ds_s = ls_s + 64;
    const uint32_t* rh_s = (const uint32_t*)(ls_s + 128);
    // the next tile's pieces go out in one burst here (spread between the S / dP MFMAs below
    // they cost 2.5 k cycles per tile more, tools/attn_stamps.py)
    if (t + 1 < ntile) {
      issue_stats(q0 + 64, (t + 1) & 1);
      char* nx = smem + ((t + 1) & 1) * 2 * TB;
      dma.issue(nx, rsQ, p.ldq, q0 + 64, p.T, wave);
      dma.issue(nx + TB, rsO, p.lddo, q0 + 64, p.T, wave);
      // tile t's pieces landed (wave 0 also has its three stat-row loads behind them)
      if (wave == 0) wait_vmcnt<2 * TileDma<DH, W8>::PER + 3>();
      else wait_vmcnt<2 * TileDma<DH, W8>::PER>();
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    FS2_STAMP(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    FS2_STAMP(1);
    // S = Q K^T, dP = dO V^T for 64 queries x this wave's 16 keys (C: col key, rows queries)
    f32x4 sacc[4], pacc[4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) { sacc[qt] = f32x4{0, 0, 0, 0}; pacc[qt] = f32x4{0, 0, 0, 0}; }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
        const bf16x8 qa = lds_row_frag(Qs, DH * 2, qt * 16 + (lane & 15), 4 * s + g);
        const bf16x8 oa = lds_row_frag(Os, DH * 2, qt * 16 + (lane & 15), 4 * s + g);
        sacc[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf[s], sacc[qt], 0, 0, 0);
        pacc[qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(oa, vf[s], pacc[qt], 0, 0, 0);
      }
    FS2_STAMP(2);
    float pdv[4][4], dsv[4][4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      const f32x4 l4 = *(const f32x4*)(ls_s + qt * 16 + 4 * g);   // rows 4g..4g+3 of this qt
      const f32x4 d4 = *(const f32x4*)(ds_s + qt * 16 + 4 * g);
      // dropout: keys 2m and 2m+1 (lanes 2m, 2m+1) share one draw per query row; the even
      // lane draws rows r = 0, 1 and the odd lane rows 2, 3, then they swap (DPP quad_perm)
      uint32_t hx[4];
      if (drop) {
        const int odd = lane & 1;
        const u32x2 rh2 = *(const u32x2*)(rh_s + qt * 16 + 4 * g + 2 * odd);
        uint32_t mine[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) mine[e] = fs2_attn_mix(rh2[e] + kc);
        uint32_t other[2];
#pragma unroll
        for (int e = 0; e < 2; ++e)
          other[e] = (uint32_t)__builtin_amdgcn_mov_dpp((int)mine[e], 0xB1, 0xF, 0xF, false);
        hx[0] = odd ? other[0] : mine[0];
        hx[1] = odd ? other[1] : mine[1];
        hx[2] = odd ? mine[0] : other[0];
        hx[3] = odd ? mine[1] : other[1];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pr = fexp2(fmaf(sacc[qt][r], c, -l4[r]));
        float dp = pacc[qt][r];
        float pd = pr;
        if (drop) {
          const bool keep = ((hx[r] >> ((key & 1) * 16)) & 0xffffu) >= p.thr16;
          dp = keep ? dp * p.inv_keep : 0.f;
          pd = keep ? pr : 0.f;       // 1 / (1 - p) applied to dV once, at the store
        }
        pdv[qt][r] = pd;
        dsv[qt][r] = pr * (dp - d4[r]);
      }
    }
    // dV += Pd^T dO, dK += dS^T Q : A = (key x query) from registers, B = tile^T via tr reads
    // (asm transposed reads of dO^T / Q^T one (j, d) step ahead of their MFMAs: the kernel sits
    // at the 256-register budget, a deeper ring spills)
    bf16x8 pa, sa;
    TrFrag ob[2], qb[2];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    FS2_STAMP(3);
    lds_tr_frag_issue(ob[0], Os, DH * 2, 0, 0, lane);
    lds_tr_frag_issue(qb[0], Qs, DH * 2, 0, 0, lane);
    static_for<0, 2 * ND>([&](auto NI) {
      constexpr int n = decltype(NI)::value, j = n / ND, d = n % ND;
      if constexpr (n + 1 < 2 * ND) {
        constexpr int n1 = n + 1;
        lds_tr_frag_issue(ob[n1 & 1], Os, DH * 2, 32 * (n1 / ND), 16 * (n1 % ND), lane);
        lds_tr_frag_issue(qb[n1 & 1], Qs, DH * 2, 32 * (n1 / ND), 16 * (n1 % ND), lane);
        lds_wait<4>(ob[n & 1], qb[n & 1]);
      } else {
        lds_wait<0>(ob[n & 1], qb[n & 1]);
      }
      if constexpr (d == 0) {
        pa = pack8(pdv[2 * j], pdv[2 * j + 1]);
        sa = pack8(dsv[2 * j], dsv[2 * j + 1]);
      }
      dv[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, tr_val(ob[n & 1]), dv[d], 0, 0, 0);
      dk[d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, tr_val(qb[n & 1]), dk[d], 0, 0, 0);
    });
    FS2_STAMP(4);
    __builtin_amdgcn_s_barrier();   // every wave is done with buffer t & 1 before t+2 lands
    FS2_STAMP(5);
  }
#ifdef FS2_EXPERIMENTS
  const uint64_t st_loop_end = __builtin_amdgcn_s_memtime();
#endif
  // C layout: col = feature (lane & 15), rows = keys 4g + r of this wave's 16; a masked key's
  // gradients are zero (its lane computed with the key unmasked).  Staged through the (now
  // free) tile ring as [key][dK | dV] rows, then stored as 16-byte chunks of whole rows: the
  // 2-byte stores straight from the accumulators were store-issue bound (~6 k cycles/block)
  if (ntile > 0) {   // the loop's last barrier: every wave is done with the ring
    constexpr int RB = 4 * DH;   // bytes per staged key row (dK | dV)
    static_assert(16 * W8 * RB <= 4 * TB, "dK/dV staging must fit the tile ring");
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kl = wave * 16 + 4 * g + r;
      const bool ok = kval[min(blk * (16 * W8) + kl, p.T - 1)];
      bf16* row = (bf16*)(smem + kl * RB);
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        row[16 * d + (lane & 15)] = (bf16)(ok ? dk[d][r] * p.scale : 0.f);
        row[DH + 16 * d + (lane & 15)] = (bf16)(ok ? dv[d][r] * p.inv_keep : 0.f);
      }
    }
    __syncthreads();
    constexpr int CPR = RB / 16;   // 16-byte chunks per staged row
    for (int i = threadIdx.x; i < 16 * W8 * CPR; i += W8 * 64) {
      const int kl = i / CPR, cc = i - kl * CPR;
      const int kr = blk * (16 * W8) + kl;
      if (kr >= p.T) continue;
      const int half = cc >= CPR / 2;   // 0: dK, 1: dV
      bf16* dst = p.dqkv + ((long)b * p.T + kr) * p.lddq + (1 + half) * p.D + h * DH +
                  (cc - half * (CPR / 2)) * 8;
      *(u32x4*)dst = *(const u32x4*)(smem + kl * RB + cc * 16);
    }
  } else {
    // an all-masked key block stores zeros (no loop ran; the speculative tile-0 DMA retired above)
    for (int i = threadIdx.x; i < 16 * W8 * (DH / 8) * 2; i += W8 * 64) {
      const int kl = i / (DH / 4), cc = i - kl * (DH / 4);
      const int kr = blk * (16 * W8) + kl;
      if (kr >= p.T) continue;
      const int half = cc >= DH / 8;
      bf16* dst = p.dqkv + ((long)b * p.T + kr) * p.lddq + (1 + half) * p.D + h * DH +
                  (cc - half * (DH / 8)) * 8;
      *(u32x4*)dst = u32x4{0u, 0u, 0u, 0u};
    }
  }
#ifdef FS2_EXPERIMENTS
  if (stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t st_end = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
      uint64_t* o = (uint64_t*)(p.dsum + 2L * p.B * p.H * p.T) +
                    ((long)(blockIdx.x + gridDim.x * blockIdx.y) * W8 + wave) * 16;
      for (int i = 0; i < 6; ++i) o[i] = st_acc[i];
      o[6] = ntile;
      o[7] = st_pro;
      o[8] = st_end - st_loop_end;
      o[9] = st_entry;
      o[10] = st_end;
    }
  }
#endif
#undef FS2_STAMP
}

// ------------------------------------------------------------------------ backward dK dV, paired
// block: 8 waves = 4 pairs x 32 keys (128 keys); query tiles of 64 as attn_bwd_dkv_kernel.  The two
// waves of a pair own the same 32 keys and split the work by role instead of each computing all
// four products for 16 keys: role 0 (waves 0-3) keeps the K fragments, computes S = Q K^T, the
// probabilities P and dV += Pd^T dO; role 1 (waves 4-7) keeps the V fragments, computes
// dP = dO V^T and, with P handed over through LDS (fp32, one 16-byte slot per lane and 16-query
// block), dS = P (dP' - D) and dK += dS^T Q.  Every Q / dO fragment and every transposed
// dO^T / Q^T fragment read from LDS then feeds two MFMAs (one per 16-key group) instead of one,
// at the register budget of the 16-key kernel (K or V fragments 48, dK or dV accumulators 96,
// S or dP 32 per wave).  Same arithmetic and accumulation order as attn_bwd_dkv_kernel: the
// results are bit-identical.
template <int DH, bool DROP>
__global__ void __launch_bounds__(512, 1) attn_bwd_dkv2_kernel(AttnP p) {
  constexpr int NS = DH / 32, ND = DH / 16;
  constexpr int TB = 64 * DH * 2;
  constexpr int KB = 128;          // keys per block
  constexpr int XB = 4 * 2 * 4 * 64 * 16;   // hand-over: [pair][kg][qt][lane] x 16 B = 32 KiB
  // [Q 0 | dO 0 | Q 1 | dO 1 | P hand-over | (lse, D, rowhash) 0 | (lse, D, rowhash) 1 | kval | kend, kfull]
  __shared__ __attribute__((aligned(16))) char smem[4 * TB + XB + 1536 + TMAX + 16];
  char* xbuf = smem + 4 * TB;
  float* lsd = (float*)(smem + 4 * TB + XB);
  uint8_t* kval = (uint8_t*)(smem + 4 * TB + XB + 1536);
  int* kbuf = (int*)(smem + 4 * TB + XB + 1536 + TMAX);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int role = __builtin_amdgcn_readfirstlane(wave >> 2), kw = wave & 3;
  int blk, z;
  attn_block_coords(blk, z);
  const int b = z / p.H, h = z - b * p.H;
  constexpr bool drop = DROP;   // compile-time: a runtime flag branched per element
  const bf16* Qb = p.qkv + (long)b * p.T * p.ldq + h * DH;
  const bf16* Kb = Qb + p.D;
  const bf16* Vb = Qb + 2 * p.D;
  const bf16* dOb = p.dout + (long)b * p.T * p.lddo + h * DH;
  const float c = p.scale_log2;

  int key[2];
  uint32_t kc[2];
#pragma unroll
  for (int kg = 0; kg < 2; ++kg) {
    key[kg] = blk * KB + kw * 32 + kg * 16 + (lane & 15);
    kc[kg] = (uint32_t)(key[kg] >> 1) * FS2_ATTN_KC;
  }
  // role 0: K fragments (S = Q K^T); role 1: V fragments (dP = dO V^T)
  const bf16* Rb = role ? Vb : Kb;
  bf16x8 rf[2][NS];
#pragma unroll
  for (int kg = 0; kg < 2; ++kg)
#pragma unroll
    for (int s = 0; s < NS; ++s)
      rf[kg][s] = key[kg] < p.T ? ld_frag(Rb + (long)key[kg] * p.ldq + 32 * s + 8 * g) : bf16x8{};
  f32x4 acc[2][ND];   // role 0: dV, role 1: dK
#pragma unroll
  for (int kg = 0; kg < 2; ++kg)
#pragma unroll
    for (int d = 0; d < ND; ++d) acc[kg][d] = f32x4{0, 0, 0, 0};

  TileDma<DH, 8> dma;
  dma.init(wave, lane, 0);
  const i32x4 rsQ = make_rsrc(Qb), rsO = make_rsrc(dOb);
  const int ntile_all = (p.T + 63) / 64;
  const long BHT = (long)p.B * p.H * p.T;
  const i32x4 rsL = make_rsrc(p.lse + (long)z * p.T), rsD = make_rsrc(p.dsum + (long)z * p.T);
  const i32x4 rsH = make_rsrc(p.dsum + BHT + (long)z * p.T);
  auto issue_tile = [&](int q0, int buf) {
    if (wave == 0) {
      const int vo = q0 + lane < p.T ? lane * 4 : BUF_OOB;
      blds4(rsL, vo, q0 * 4, (char*)(lsd + buf * 192));
      blds4(rsD, vo, q0 * 4, (char*)(lsd + buf * 192 + 64));
      blds4(rsH, vo, q0 * 4, (char*)(lsd + buf * 192 + 128));
    }
    char* nx = smem + buf * 2 * TB;
    dma.issue(nx, rsQ, p.ldq, q0, p.T, wave);
    dma.issue(nx + TB, rsO, p.lddo, q0, p.T, wave);
  };
  if (ntile_all > 0) issue_tile(0, 0);
  int kfull;
  build_kvalid(kval, kbuf, p, b, h, &kfull);
  bool kok = false;
#pragma unroll
  for (int kg = 0; kg < 2; ++kg) kok = kok || (key[kg] < p.T && kval[key[kg]]);
  const int anyk = __syncthreads_or(kok);
  const int ntile = anyk ? ntile_all : 0;
  // per-lane hand-over slot: [kw][kg][qt] blocks of 64 lanes x 16 B
  char* xl = xbuf + kw * (2 * 4 * 1024) + lane * 16;
  int rb0[2], tb0[4];
  row_frag_bases(lane, DH * 2, rb0);
  tr_frag_bases(lane, DH * 2, tb0);
  for (int t = 0; t < ntile; ++t) {
    const int q0 = t * 64;
    const char* T1 = smem + (t & 1) * 2 * TB + role * TB;         // role 0: Q, role 1: dO
    const char* T2 = smem + (t & 1) * 2 * TB + (role ^ 1) * TB;   // role 0: dO, role 1: Q
    const float* ls_s = lsd + (t & 1) * 192;
    const float* ds_s = ls_s + 64;
    const uint32_t* rh_s = (const uint32_t*)(ls_s + 128);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile t (and the K/V fragments) landed
    __builtin_amdgcn_s_barrier();   // ... for every wave; every wave is done with tile t-1
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < ntile) issue_tile(q0 + 64, (t + 1) & 1);
    // phase 1: S (role 0) or dP (role 1) for 64 queries x 32 keys; 24 steps (s, qt) of one
    // fragment read and two MFMAs, each read two steps ahead of its MFMAs
    f32x4 s1[2][4];
#pragma unroll
    for (int kg = 0; kg < 2; ++kg)
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) s1[kg][qt] = f32x4{0, 0, 0, 0};
    {
      bf16x8 fa[3];
      const char* T1b0 = T1 + rb0[0];
      const char* T1b1 = T1 + rb0[1];
      auto rd = [&](auto STc) {
        constexpr int st = decltype(STc)::value, s = st >> 2, qt = st & 3;
        constexpr int off = qt * 16 * DH * 2 + s * 64;
        return lds_frag_at<off>(s & 1 ? T1b1 : T1b0, 0);
      };
      fa[0] = rd(std::integral_constant<int, 0>{});
      fa[1] = rd(std::integral_constant<int, 1>{});
      static_for<0, 4 * NS>([&](auto SI) {
        constexpr int st = decltype(SI)::value, s = st >> 2, qt = st & 3;
        if constexpr (st + 2 < 4 * NS) {
          fa[(st + 2) % 3] = rd(std::integral_constant<int, st + 2>{});
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
#pragma unroll
        for (int kg = 0; kg < 2; ++kg)
          s1[kg][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[st % 3], rf[kg][s], s1[kg][qt], 0, 0, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      });
    }
    // dropout draws of this lane's (query row, key) elements, identical in both roles: keys 2m
    // and 2m+1 (lanes 2m, 2m+1) share one draw per query row; the even lane draws rows r = 0, 1
    // and the odd lane rows 2, 3, then they swap (DPP quad_perm)
    auto keep_bits = [&](int kg, int qt, uint32_t (&hx)[4]) {
      const int odd = lane & 1;
      const u32x2 rh2 = *(const u32x2*)(rh_s + qt * 16 + 4 * g + 2 * odd);
      uint32_t mine[2], other[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) mine[e] = fs2_attn_mix(rh2[e] + kc[kg]);
#pragma unroll
      for (int e = 0; e < 2; ++e)
        other[e] = (uint32_t)__builtin_amdgcn_mov_dpp((int)mine[e], 0xB1, 0xF, 0xF, false);
      hx[0] = odd ? other[0] : mine[0];
      hx[1] = odd ? other[1] : mine[1];
      hx[2] = odd ? mine[0] : other[0];
      hx[3] = odd ? mine[1] : other[1];
    };
    bf16x8 pk[2][2];   // role 0: Pd, role 1: dS, per (kg, 32-query half j): the phase-2 A operands
    if (role == 0) {
#pragma unroll
      for (int kg = 0; kg < 2; ++kg)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float pdv[2][4];
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const int qt = 2 * j + h2;
            const f32x4 l4 = *(const f32x4*)(ls_s + qt * 16 + 4 * g);
            uint32_t hx[4];
            if constexpr (DROP) keep_bits(kg, qt, hx);
            f32x4 pr4;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float pr = fexp2(fmaf(s1[kg][qt][r], c, -l4[r]));
              pr4[r] = pr;
              pdv[h2][r] = (!drop || ((hx[r] >> ((lane & 1) * 16)) & 0xffffu) >= p.thr16) ? pr : 0.f;
            }
            *(f32x4*)(xl + (kg * 4 + qt) * 1024) = pr4;
          }
          pk[kg][j] = pack8(pdv[0], pdv[1]);
        }
    }
    // the P hand-over written: its LDS stores retired before the barrier (s_barrier alone does
    // not wait for them)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (role == 1) {
#pragma unroll
      for (int kg = 0; kg < 2; ++kg)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float dsv[2][4];
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const int qt = 2 * j + h2;
            const f32x4 d4 = *(const f32x4*)(ds_s + qt * 16 + 4 * g);
            const f32x4 pr4 = *(const f32x4*)(xl + (kg * 4 + qt) * 1024);
            uint32_t hx[4];
            if constexpr (DROP) keep_bits(kg, qt, hx);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float dp = s1[kg][qt][r];
              if constexpr (DROP) {
                const bool keep = ((hx[r] >> ((lane & 1) * 16)) & 0xffffu) >= p.thr16;
                dp = keep ? dp * p.inv_keep : 0.f;
              }
              dsv[h2][r] = pr4[r] * (dp - d4[r]);
            }
          }
          pk[kg][j] = pack8(dsv[0], dsv[1]);
        }
    }
    // phase 2: role 0 dV += Pd^T dO, role 1 dK += dS^T Q: the transposed tile fragments two
    // (j, d) steps ahead of their MFMAs
    bf16x8 tf[3];
    auto trd = [&](auto NC) {
      constexpr int n = decltype(NC)::value, j = n / ND, d = n % ND;
      return lds_tr_frag_at<32 * j * DH * 2 + (d & ~3) * 32, DH * 2>(T2, tb0[d & 3]);
    };
    tf[0] = trd(std::integral_constant<int, 0>{});
    tf[1] = trd(std::integral_constant<int, 1>{});
    static_for<0, 2 * ND>([&](auto NI) {
      constexpr int n = decltype(NI)::value, j = n / ND, d = n % ND;
      if constexpr (n + 2 < 2 * ND) {
        tf[(n + 2) % 3] = trd(std::integral_constant<int, n + 2>{});
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
#pragma unroll
      for (int kg = 0; kg < 2; ++kg)
        acc[kg][d] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pk[kg][j], tf[n % 3], acc[kg][d], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    });
  }
  // the speculative tile-0 DMA of a block whose keys are all masked (no loop ran) has landed,
  // and every wave is done with the tile ring, before the results are staged there
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // C layout: col = feature (lane & 15), rows = keys 4g + r of the 16-key group kg; staged as
  // [key][dK | dV] rows through the tile ring, then stored as 16-byte chunks of whole rows
  constexpr int RB = 4 * DH;
  static_assert(KB * RB <= 4 * TB, "dK/dV staging must fit the tile ring");
  const float osc = ntile > 0 ? (role ? p.scale : p.inv_keep) : 0.f;
#pragma unroll
  for (int kg = 0; kg < 2; ++kg)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int kl = kw * 32 + kg * 16 + 4 * g + r;
      const bool ok = kval[min(blk * KB + kl, p.T - 1)];
      bf16* row = (bf16*)(smem + kl * RB) + (role ? 0 : DH);
#pragma unroll
      for (int d = 0; d < ND; ++d) row[16 * d + (lane & 15)] = (bf16)(ok ? acc[kg][d][r] * osc : 0.f);
    }
  __syncthreads();
  constexpr int CPR = RB / 16;   // 16-byte chunks per staged row
  for (int i = threadIdx.x; i < KB * CPR; i += 512) {
    const int kl = i / CPR, cc = i - kl * CPR;
    const int kr = blk * KB + kl;
    if (kr >= p.T) continue;
    const int half = cc >= CPR / 2;   // 0: dK, 1: dV
    bf16* dst = p.dqkv + ((long)b * p.T + kr) * p.lddq + (1 + half) * p.D + h * DH +
                (cc - half * (CPR / 2)) * 8;
    *(u32x4*)dst = *(const u32x4*)(smem + kl * RB + cc * 16);
  }
}

int attn_qg_fwd(int dh) { return dh <= 128 ? 2 : 1; }

// half-size forward blocks (64 queries) when 128-row blocks would leave CUs idle (the
// encoder: T = 200, B*H = 64 -> 128 blocks of 128 rows for 256 CUs; 26.3 -> 24.2 us)
bool attn_small_blocks(const AttnP& p) {
  return (long)((p.T + 127) / 128) * p.B * p.H < 256;
}

template <int DH>
void launch_fwd(const AttnP& p, hipStream_t s) {
  if (attn_small_blocks(p)) {
    dim3 grid((p.T + 63) / 64, p.B * p.H);
    if (attn_qg_fwd(DH) == 2) hipLaunchKernelGGL((attn_fwd_kernel<DH, 2, 4>), grid, dim3(128), 0, s, p);
    else hipLaunchKernelGGL((attn_fwd_kernel<DH, 1, 4>), grid, dim3(256), 0, s, p);
    return;
  }
  // dh = 192 at decoder lengths: 8 waves x 32 queries (256-query blocks, one per CU at B = 32,
  // T = 977): every K fragment and V^T fragment feeds two MFMAs, halving the LDS reads per
  // MFMA that bound the 16-query form (tools/attn_bench.py: 86.2 -> 72.9 us; 4 waves x 32
  // queries at one wave per SIMD: 111 us)
  if (DH == 192 && !(p.xflags & 4)) {
    hipLaunchKernelGGL((attn_fwd_kernel<DH, 2, 16>), dim3((p.T + 255) / 256, p.B * p.H), dim3(512), 0, s, p);
    return;
  }
  dim3 grid((p.T + 127) / 128, p.B * p.H);
  if (attn_qg_fwd(DH) == 2) hipLaunchKernelGGL((attn_fwd_kernel<DH, 2>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((attn_fwd_kernel<DH, 1>), grid, dim3(512), 0, s, p);
}
template <int DH>
void launch_bwd(const AttnP& p, hipStream_t s) {
  // 64-key / 64-query blocks when 128-row blocks underfill the chip, as the forward (encoder
  // T = 200 with the LDS-DMA dK/dV kernel: 60.2 -> 56.7 us)
  if (attn_small_blocks(p)) {
    dim3 g1((p.T + 63) / 64, p.B * p.H);
    if (DH <= 64) hipLaunchKernelGGL((attn_bwd_dq_kernel<DH, 2, 4>), g1, dim3(128), 0, s, p);
    else hipLaunchKernelGGL((attn_bwd_dq_kernel<DH, 1, 4>), g1, dim3(256), 0, s, p);
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<DH, 4>), g1, dim3(256), 0, s, p);
    return;
  }
  dim3 g1((p.T + 127) / 128, p.B * p.H);
  if (DH <= 64) hipLaunchKernelGGL((attn_bwd_dq_kernel<DH, 2>), g1, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((attn_bwd_dq_kernel<DH, 1>), g1, dim3(512), 0, s, p);
  // FS2_ATTN_BWD=4 (experiments build): the paired dK / dV kernel -- bit-identical, 241 -> 235
  // us without dropout but 251 -> 263 us with it (tools/attn_ab_bwd.sh), so off
#ifdef FS2_EXPERIMENTS
  if constexpr (DH <= 192) {
    if (fs2_exp_int("FS2_ATTN_BWD", 0) & 4) {
      if (p.p_drop > 0.f) hipLaunchKernelGGL((attn_bwd_dkv2_kernel<DH, true>), g1, dim3(512), 0, s, p);
      else hipLaunchKernelGGL((attn_bwd_dkv2_kernel<DH, false>), g1, dim3(512), 0, s, p);
      return;
    }
  }
#endif
  hipLaunchKernelGGL(attn_bwd_dkv_kernel<DH>, g1, dim3(512), 0, s, p);
}

bool a16(const void* q) { return ((uintptr_t)q & 15) == 0; }

int check(int B, int H, int T, int dh, long ldq, const void* qkv, int dtype) {
  if (dtype != FS2_BF16) return FS2_EINVAL;
  if (B <= 0 || H <= 0 || T <= 0 || T > TMAX) return FS2_EINVAL;
  if (dh != 64 && dh != 128 && dh != 192 && dh != 256) return FS2_EINVAL;
  if (!qkv || !a16(qkv) || (ldq % 8) || ldq < 3L * H * dh) return FS2_EALIGN;
  return 0;
}

}  // namespace

extern "C" int fs2_attn_supported(int T, int dh, int dtype) {
  return dtype == FS2_BF16 && T > 0 && T <= TMAX &&
         (dh == 64 || dh == 128 || dh == 192 || dh == 256);
}

extern "C" int fs2_attn_fwd(const void* qkv, int64_t ldq, const uint8_t* key_pad, int mask_mode,
                            int B, int H, int T, int dh, float scale, float p_drop, uint32_t seed,
                            uint32_t salt, void* out, int64_t ldo, float* lse, int dtype,
                            void* stream) {
  if (int rc = check(B, H, T, dh, ldq, qkv, dtype)) return rc;
  if (!key_pad || !out || !lse || !a16(out) || (ldo % 8)) return FS2_EINVAL;
  AttnP p{};
  p.qkv = (const bf16*)qkv; p.ldq = ldq; p.kpad = key_pad; p.tiled = mask_mode != 0;
  p.out = (bf16*)out; p.ldout = ldo; p.lse = lse;
  p.B = B; p.H = H; p.T = T; p.D = H * dh;
  p.scale = scale; p.scale_log2 = scale * LOG2E; p.p_drop = p_drop;
  p.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  p.seed = seed; p.salt = salt;
  p.thr16 = (uint32_t)(p_drop * 65536.f + 0.5f);
  p.xflags = fs2_exp_int("FS2_ATTN_FLAGS", 0);
  hipStream_t s = (hipStream_t)stream;
  switch (dh) {
    case 64: launch_fwd<64>(p, s); break;
    case 128: launch_fwd<128>(p, s); break;
    case 192: launch_fwd<192>(p, s); break;
    default: launch_fwd<256>(p, s); break;
  }
  FS2_CHECK_LAUNCH();
  return 0;
}

extern "C" int fs2_attn_bwd(const void* qkv, int64_t ldq, const uint8_t* key_pad, int mask_mode,
                            const void* out, int64_t ldo, const void* dout, int64_t lddo,
                            const float* lse, int B, int H, int T, int dh, float scale,
                            float p_drop, uint32_t seed, uint32_t salt, void* dqkv,
                            int64_t lddq, float* workspace, int dtype, void* stream) {
  if (int rc = check(B, H, T, dh, ldq, qkv, dtype)) return rc;
  if (!key_pad || !out || !dout || !lse || !dqkv || !workspace) return FS2_EINVAL;
  if (!a16(out) || !a16(dout) || !a16(dqkv) || (ldo % 8) || (lddo % 8) || (lddq % 8))
    return FS2_EALIGN;
  AttnP p{};
  p.qkv = (const bf16*)qkv; p.ldq = ldq; p.kpad = key_pad; p.tiled = mask_mode != 0;
  p.o = (const bf16*)out; p.ldo = ldo;
  p.dout = (const bf16*)dout; p.lddo = lddo;
  p.dqkv = (bf16*)dqkv; p.lddq = lddq;
  p.lse = (float*)lse; p.dsum = workspace;
  p.B = B; p.H = H; p.T = T; p.D = H * dh;
  p.scale = scale; p.scale_log2 = scale * LOG2E; p.p_drop = p_drop;
  p.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  p.seed = seed; p.salt = salt;
  p.thr16 = (uint32_t)(p_drop * 65536.f + 0.5f);
  p.xflags = fs2_exp_int("FS2_ATTN_FLAGS", 0);
  hipStream_t s = (hipStream_t)stream;
  switch (dh) {
    case 64: launch_bwd<64>(p, s); break;
    case 128: launch_bwd<128>(p, s); break;
    case 192: launch_bwd<192>(p, s); break;
    default: launch_bwd<256>(p, s); break;
  }
  FS2_CHECK_LAUNCH();
  return 0;
}

// D = rowsum(dO * O) and the dropout row hashes of every query row (dQ kernel -> dK/dV kernel)
extern "C" int64_t fs2_attn_workspace_floats(int B, int H, int T) { return 2 * (int64_t)B * H * T; }

// this translation unit's dropout seed base (fs2_common.h)
FS2_SEED_SETTER(fs2_seed_base_flash)
