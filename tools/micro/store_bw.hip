// Store-bandwidth microbenchmark: the GEMM epilogue's tile write pattern vs contiguous writes.
// hipcc --offload-arch=gfx950 -O3 store_bw.hip -o store_bw
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// tile (BM x BN) per block, 512 threads, thread: 8 columns x (BM*BN/8/512) passes
template <int BM, int BN>
__global__ void __launch_bounds__(512) tile_store(unsigned short* C, int M, int N, int tiles_n) {
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int tid = threadIdx.x;
  constexpr int TPR = BN / 8;               // threads per row
  constexpr int RPP = 512 / TPR;            // rows per pass
  const int c8 = (tid % TPR) * 8;
  const u32x4 v = {1u, 2u, 3u, (unsigned)tid};
#pragma unroll
  for (int pass = 0; pass < BM / RPP; ++pass) {
    const int m = tm * BM + tid / TPR + RPP * pass;
    if (m < M) *(u32x4*)(C + (long)m * N + tn * BN + c8) = v;
  }
}
__global__ void lin_store(u32x4* C, long n16) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n16) C[i] = u32x4{1u, 2u, 3u, (unsigned)i};
}

template <typename F>
float timeit(F f) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(a);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 20 * 1e3f;
}

int main() {
  const int M = 31264;
  for (int N : {384, 1152, 1536}) {
    unsigned short* C; hipMalloc(&C, (size_t)M * N * 2);
    const double mb = (double)M * N * 2 / 1e6;
    float t1 = timeit([&] { int tn = N / 128; hipLaunchKernelGGL((tile_store<256, 128>), dim3(((M + 255) / 256) * tn), dim3(512), 0, 0, C, M, N, tn); });
    float t2 = N % 256 == 0 ? timeit([&] { int tn = N / 256; hipLaunchKernelGGL((tile_store<256, 256>), dim3(((M + 255) / 256) * tn), dim3(512), 0, 0, C, M, N, tn); }) : 0.f;
    float t3 = timeit([&] { long n16 = (long)M * N / 8; hipLaunchKernelGGL(lin_store, dim3((n16 + 255) / 256), dim3(256), 0, 0, (u32x4*)C, n16); });
    printf("N=%d  %.1f MB: tile256x128 %.1f us (%.2f TB/s)  tile256x256 %.1f us  linear %.1f us (%.2f TB/s)\n",
           N, mb, t1, mb / t1 / 1e6 * 1e6 / 1e6, t2, t3, mb / t3 / 1e6 * 1e6 / 1e6);
    hipFree(C);
  }
  return 0;
}
