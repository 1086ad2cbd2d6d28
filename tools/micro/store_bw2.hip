// Store patterns of the GEMM epilogues at the decoder QKV shape (M = 31264, N = 1152, 256x128
// tiles, 8 waves of 64x64), persistent (256 blocks) and one-block-per-tile grids.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

template <int PAT>
__device__ __forceinline__ void wave_tile(unsigned short* C, int M, int N, int mb, int nb, int lane) {
  if (PAT == 0) {           // direct MFMA-fragment pattern: 8 B per lane, 16 rows x 32 B per instr
    const int li = lane & 15, g = lane >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mb + 16 * i + li, n = nb + 16 * j + 4 * g;
        if (m < M) *(u32x2*)(C + (long)m * N + n) = u32x2{(unsigned)m, (unsigned)n};
      }
  } else {                  // row pattern: 16 B per lane, 8 rows x 128 B per instr
    const int c = (lane & 7) * 8, r = lane >> 3;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = mb + 8 * i + r;
      if (m < M) *(u32x4*)(C + (long)m * N + nb + c) = u32x4{(unsigned)m, 1u, 2u, 3u};
    }
  }
}

template <int PAT>
__global__ void __launch_bounds__(512) persist(unsigned short* C, int M, int N, int tiles_n, int ntile) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int t = blockIdx.x; t < ntile; t += gridDim.x) {
    const int tm = t / tiles_n, tn = t % tiles_n;
    wave_tile<PAT>(C, M, N, tm * 256 + (wave >> 1) * 64, tn * 128 + (wave & 1) * 64, lane);
  }
}

template <typename F>
float timeit(F f) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  (void)hipEventRecord(a);
  for (int i = 0; i < 20; ++i) f();
  (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  return ms / 20 * 1e3f;
}

int main() {
  const int M = 31264, N = 1152, tn = N / 128, nt = ((M + 255) / 256) * tn;
  unsigned short* C; (void)hipMalloc(&C, (size_t)M * N * 2);
  for (int g : {256, 512, nt}) {
    float a = timeit([&] { hipLaunchKernelGGL(persist<0>, dim3(g), dim3(512), 0, 0, C, M, N, tn, nt); });
    float b = timeit([&] { hipLaunchKernelGGL(persist<1>, dim3(g), dim3(512), 0, 0, C, M, N, tn, nt); });
    printf("grid %5d: 8B-fragment pattern %.1f us, 16B-row pattern %.1f us (72 MB)\n", g, a, b);
  }
  return 0;
}
