// Shared device helpers for the FastSpeech2 MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fs2_hip.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

#define FS2_WAVE 64

// FS2_* A/B switches: read from the environment only in the experiments build
// (make experiments, -DFS2_EXPERIMENTS, used by tools/); the product library compiles every
// switch to its default.
#ifdef FS2_EXPERIMENTS
#include <cstdlib>
inline int fs2_exp_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && v[0] ? std::atoi(v) : dflt;
}
#else
constexpr int fs2_exp_int(const char*, int dflt) { return dflt; }
#endif

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

__device__ __forceinline__ float bf16_bits_to_f(unsigned short u) {
  return __builtin_bit_cast(float, ((unsigned int)u) << 16);
}

// ---- 16-byte vector access: VEC<T> elements per lane (8 bf16 / 4 fp32), fp32 in registers ----
template <typename T> struct Vec { static constexpr int N = 16 / (int)sizeof(T); };
template <typename T>
__device__ __forceinline__ void vload(float* o, const T* src) {
  if constexpr (sizeof(T) == 2) {
    const u32x4 u = *(const u32x4*)src;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      o[2 * w] = __builtin_bit_cast(float, u[w] << 16);
      o[2 * w + 1] = __builtin_bit_cast(float, u[w] & 0xffff0000u);
    }
  } else {
    const f32x4 a = *(const f32x4*)src;
    o[0] = a[0]; o[1] = a[1]; o[2] = a[2]; o[3] = a[3];
  }
}
template <typename T>
__device__ __forceinline__ void vstore(T* dst, const float* v) {
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
  }
}
__device__ __forceinline__ bool aligned16_dev(const void* p) { return ((uintptr_t)p & 15) == 0; }

// ---- wave reductions (64 lanes) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// the same sum through DPP -- quad_perm xor 1 / xor 2, then row_ror 4 / 8 (every lane of a
// 16-lane row then holds the row's sum) -- and four readlanes added in a fixed order (a
// wave-uniform result): ~30 cycles against the six dependent LDS round trips (ds_bpermute) of
// __shfl_xor.  Every lane must be active.  Sums in a different order from wave_sum.
template <int C>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), C, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f32<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f32<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f32<0x124>(v);  // row_ror:4
  v += dpp_f32<0x128>(v);  // row_ror:8
  const int u = __float_as_int(v);
  return (__int_as_float(__builtin_amdgcn_readlane(u, 0)) +
          __int_as_float(__builtin_amdgcn_readlane(u, 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(u, 32)) +
          __int_as_float(__builtin_amdgcn_readlane(u, 48)));
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---- counter-based dropout RNG: keep(seed, salt, index) ----
// A stateless 32-bit mixer (murmur3 finaliser over a 64-bit counter); forward and
// backward regenerate the same mask from (seed, salt, element index), so no mask
// tensor is stored.
__device__ __forceinline__ uint32_t fs2_mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
//
// The step's seed is the launch's ``seed`` argument PLUS a device-resident base (one cell per
// translation unit, written by fs2_set_dropout_seed).  Eager steps pass their seed as the
// argument with base 0; a captured HIP graph replays launches with their captured arguments,
// so the graph is captured with seed 0 and each replay first sets the base to the step's seed.
// Both give identical masks for the same step seed.
namespace {
__device__ uint32_t g_fs2_seed_base = 0u;
__global__ void fs2_seed_base_kernel(uint32_t v) { g_fs2_seed_base = v; }
}  // namespace
#define FS2_SEED_SETTER(NAME)                                            \
  int NAME(uint32_t v, void* stream) {                                    \
    hipLaunchKernelGGL(fs2_seed_base_kernel, dim3(1), dim3(1), 0,          \
                       (hipStream_t)stream, v);                           \
    return (int)hipGetLastError();                                        \
  }


// Attention-probability dropout draws B*H*T^2 masks per layer, so it uses a cheaper form:
// one murmur-finaliser round per PAIR of elements (idx >> 1) keyed by a per-call key, 16 bits
// per element compared with thr16 = round(p * 65536).  Element indices are row-major over
// rows padded to an even length, so a lane's consecutive keys share one hash.
__device__ __forceinline__ uint32_t fs2_drop_key(uint32_t seed, uint32_t salt) {
  seed += g_fs2_seed_base;
  return fs2_mix32(seed ^ (salt * 0x9E3779B9u)) | 1u;
}
__device__ __forceinline__ uint32_t fs2_hash_pair(uint32_t key, uint64_t pair) {
  uint32_t h = ((uint32_t)pair * 0x9E3779B1u) ^ ((uint32_t)(pair >> 32) * 0x85EBCA77u) ^ key;
  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
  return h;
}
__device__ __forceinline__ bool fs2_keep_pair_bit(uint32_t h, uint64_t idx, uint32_t thr16) {
  return ((h >> ((uint32_t)(idx & 1) * 16)) & 0xffffu) >= thr16;
}
__device__ __forceinline__ bool fs2_keep_fast(uint32_t key, uint64_t idx, uint32_t thr16) {
  return fs2_keep_pair_bit(fs2_hash_pair(key, idx >> 1), idx, thr16);
}
__device__ __forceinline__ uint32_t fs2_thr16(float p) { return (uint32_t)(p * 65536.f + 0.5f); }

// Element dropout (LayerNorm residual / output dropout) uses the same pair hash: element idx of
// the (seed, salt) stream is kept iff its 16-bit half of hash_pair(key, idx >> 1) >= thr16(p).
// Kernels that own consecutive elements compute one hash per pair (fs2_keep_pair_bit);
// fs2_keep is the per-element form with identical results.  (One murmur-style round per two
// elements instead of two full murmur finalisers per element: the LayerNorm kernels spent
// more VALU on their masks than on the normalisation.)
__device__ __forceinline__ bool fs2_keep(uint32_t seed, uint32_t salt, uint64_t idx, float p) {
  if (p <= 0.f) return true;
  return fs2_keep_fast(fs2_drop_key(seed, salt), idx, fs2_thr16(p));
}
// keep bits of V consecutive elements from an EVEN index ib, one hash per pair (== fs2_keep)
template <int V>
__device__ __forceinline__ void fs2_keep_run(uint32_t seed, uint32_t salt, uint64_t ib, float p,
                                             bool (&k)[V]) {
  const uint32_t key = fs2_drop_key(seed, salt), thr = fs2_thr16(p);
#pragma unroll
  for (int e = 0; e < V; e += 2) {
    const uint32_t h = fs2_hash_pair(key, (ib + e) >> 1);
    k[e] = p <= 0.f || fs2_keep_pair_bit(h, ib + e, thr);
    k[e + 1] = p <= 0.f || fs2_keep_pair_bit(h, ib + e + 1, thr);
  }
}

// Attention-probability dropout (flash.hip's fused kernels, attention.hip's materialised path):
// element (row, key) of the (seed, salt) draw, row = (b*H + h)*T + query, is kept iff the 16-bit
// half (key & 1) of fs2_attn_bits(fs2_attn_rowhash(dkey, row), key >> 1) >= thr16.  The per-row
// part is a full lowbias32 round, computed once per query row; the per-element part is ONE add
// of the key pair's multiple of FS2_ATTN_KC (a lane constant plus a per-tile scalar in the
// kernels) and one xorshift-multiply-xorshift round on the full-rate 24-bit multiplier
// (v_mul_lo_u32 issues at a quarter of the VALU rate; the murmur-style pair hash of the
// LayerNorm masks costs four of them per pair).  Measured on 31 M draws: keep rate, 1024-bin
// chi^2 and lag correlations over keys / rows at the level of an ideal generator (|c| < 0.003).
constexpr uint32_t FS2_ATTN_KC = 0x27D4EB2Fu;
__device__ __forceinline__ uint32_t fs2_attn_rowhash(uint32_t dkey, uint32_t row) {
  uint32_t h = (row * 0x9E3779B1u) ^ dkey;
  h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t fs2_attn_mix(uint32_t u) {   // u = rowhash + kpair * KC
  u ^= u >> 15;
  u = __umul24(u, 0x5BD1E9u);
  return u ^ (u >> 13);
}
__device__ __forceinline__ bool fs2_attn_keep(uint32_t dkey, uint32_t row, uint32_t key,
                                              uint32_t thr16) {
  const uint32_t h = fs2_attn_mix(fs2_attn_rowhash(dkey, row) + (key >> 1) * FS2_ATTN_KC);
  return ((h >> ((key & 1u) * 16)) & 0xffffu) >= thr16;
}

// reflect index into [0, T) (torch F.pad(mode="reflect") semantics, single bounce)
__device__ __forceinline__ int reflect_idx(int i, int T) {
  if (i < 0) i = -i;
  if (i >= T) i = 2 * (T - 1) - i;
  return i;
}

#define FS2_CHECK_LAUNCH()                         \
  do {                                             \
    hipError_t e__ = hipGetLastError();            \
    if (e__ != hipSuccess) return (int)e__;        \
  } while (0)
