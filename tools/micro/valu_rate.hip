// VALU issue rates on gfx950: v_mul_lo_u32 vs v_add_u32 vs v_mul_u32_u24 vs the dropout pair
// hash (fs2_hash_pair), 64-bit-free chains, many independent chains per lane.
// hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
template <int OP>
__global__ void __launch_bounds__(256) chain(unsigned* out, int iters, unsigned k) {
  unsigned a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i + blockIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) a[i] = a[i] * k;
      else if (OP == 1) a[i] = a[i] + k;
      else if (OP == 2) a[i] = (a[i] & 0xffffffu) * (k & 0xffffffu);
      else {
        unsigned h = (a[i] * 0x9E3779B1u) ^ k;
        h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
        a[i] = h;
      }
    }
  }
  unsigned s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int OP>
float run(unsigned* out, int iters) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  chain<OP><<<2048, 256>>>(out, iters, 0x12345u);
  hipEventRecord(a);
  chain<OP><<<2048, 256>>>(out, iters, 0x12345u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms;
}
int main() {
  unsigned* out; hipMalloc(&out, 2048 * 256 * 4);
  const int iters = 4096;
  const double ops = 2048.0 * 256 * iters * 8;   // chain steps (lanes)
  const char* names[] = {"v_mul_lo_u32", "v_add_u32", "v_mul_u32_u24", "pair hash"};
  float t[4] = {run<0>(out, iters), run<1>(out, iters), run<2>(out, iters), run<3>(out, iters)};
  for (int i = 0; i < 4; ++i)
    printf("%-14s %8.3f ms  %7.1f G lane-ops/s\n", names[i], t[i], ops / (t[i] * 1e-3) / 1e9);
  return 0;
}
