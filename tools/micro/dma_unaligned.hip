// LDS-DMA (buffer_load_dwordx4 ... lds) from global addresses that are only 2-byte aligned:
// correctness (LDS image == the source shifted by `shift` bytes) and streaming rate against the
// 16-byte-aligned case.  Question it answers: can a K-major implicit-conv operand whose tap
// shift moves the K window by an odd number of bf16 elements be DMA'd straight into LDS?
// hipcc --offload-arch=gfx950 -O3 dma_unaligned.hip -o /tmp/dma_unaligned
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
__device__ void llvm_raw_buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) uint32_t* lds,
                                         int size, int voffset, int soffset, int offset,
                                         int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

__device__ __forceinline__ i32x4 make_rsrc(const void* base) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane((int)(a >> 32));
  r[2] = 0x7fffffff;
  r[3] = 0x00020000;
  return r;
}

// copy: block of 4 waves, wave w moves 1 KiB chunks src + shift -> LDS -> dst
__global__ void __launch_bounds__(256) dma_copy(const char* src, char* dst, long nchunks, int shift) {
  __shared__ __attribute__((aligned(16))) char lds[4 * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const i32x4 rs = make_rsrc(src);
  char* mine = lds + wave * 1024;
  for (long c = (long)blockIdx.x * 4 + wave; c < nchunks; c += (long)gridDim.x * 4) {
    llvm_raw_buffer_load_lds(rs, (__attribute__((address_space(3))) uint32_t*)mine, 16,
                             lane * 16 + shift, (int)(c * 1024), 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const u32x4 v = *(const u32x4*)(mine + lane * 16);
    *(u32x4*)(dst + c * 1024 + lane * 16) = v;
    asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");
  }
}

// stream: each wave keeps 8 DMA pieces in flight through an 8 KiB ring; no LDS reads
__global__ void __launch_bounds__(256) dma_stream(const char* src, long nchunks, int shift) {
  __shared__ __attribute__((aligned(16))) char lds[4 * 8 * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const i32x4 rs = make_rsrc(src);
  char* ring = lds + wave * 8 * 1024;
  int slot = 0;
  for (long c = (long)blockIdx.x * 4 + wave; c < nchunks; c += (long)gridDim.x * 4) {
    llvm_raw_buffer_load_lds(rs, (__attribute__((address_space(3))) uint32_t*)(ring + slot * 1024),
                             16, lane * 16 + shift, (int)(c * 1024), 0, 0);
    slot = (slot + 1) & 7;
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int main() {
  const long bytes = 512L << 20;
  const long nch = bytes / 1024 - 1;
  char *src, *dst;
  hipMalloc(&src, bytes + 64);
  hipMalloc(&dst, bytes);
  std::vector<unsigned short> h(bytes / 2 + 32);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned short)(i * 2654435761u >> 7);
  hipMemcpy(src, h.data(), bytes + 64, hipMemcpyHostToDevice);
  std::vector<unsigned short> o(bytes / 2);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int shift : {0, 2, 4, 6, 8, 14}) {
    hipMemset(dst, 0, bytes);
    hipLaunchKernelGGL(dma_copy, dim3(2048), dim3(256), 0, 0, src, dst, nch, shift);
    hipError_t e = hipDeviceSynchronize();
    hipMemcpy(o.data(), dst, nch * 1024, hipMemcpyDeviceToHost);
    long bad = 0;
    for (long i = 0; i < nch * 512; ++i)
      if (o[i] != h[i + shift / 2]) ++bad;
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(dma_stream, dim3(2048), dim3(256), 0, 0, src, nch, shift);
    hipEventRecord(a);
    for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(dma_stream, dim3(2048), dim3(256), 0, 0, src, nch, shift);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("shift %2d B: err=%s mismatches=%ld  stream %.1f us per 512 MiB = %.2f TB/s\n", shift,
           hipGetErrorString(e), bad, ms / 10 * 1e3, (double)nch * 1024 / (ms / 10 * 1e-3) / 1e12);
  }
  return 0;
}
