// Correctness probe: LDS-DMA (global_load_lds_dwordx4, M0 = the destination's LDS address) with two
// workgroups resident per CU (dynamic LDS just under 80 KiB each, the fp64 engine's ShapeW4
// geometry). Every workgroup copies workgroup-specific data into its LDS, waits for its own DMA
// (vmcnt(0)), barriers, and checks every word; mismatches are counted. If the DMA destination were
// not relative to the workgroup's own LDS allocation, the second workgroup on a CU would write into
// the first one's LDS. Build: hipcc --offload-arch=gfx950 -O3 ldsdma_2wg.hip -o ldsdma_2wg
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);       \
      return 1;                                                              \
    }                                                                        \
  } while (0)

constexpr int LDS_BYTES = 79360;

__device__ __forceinline__ void dma16(const double* src, double* lds_wave) {
  const unsigned l = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) void*)lds_wave);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off sc1" ::"v"(src), "{m0}"(l) : "memory");
}

__global__ __launch_bounds__(256, 2) void k_probe(const double* src, int iters, unsigned* bad, unsigned long long* where) {
  extern __shared__ __align__(16) double lds[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  constexpr int UNITS = 38912 / 1024;  // 1-KiB DMA units per buffer (38)
  for (int it = 0; it < iters; ++it) {
    const int buf = it & 1;
    const int srcblk = (blockIdx.x * 131 + it * 17) % 4096;  // a workgroup- and iteration-specific source
    const double* s = src + (size_t)srcblk * (UNITS * 128);
    double* d = lds + buf * (UNITS * 128);
    for (int u = w; u < UNITS; u += 4) dma16(s + u * 128 + 2 * lane, d + u * 128);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned nb = 0;
    for (int e = threadIdx.x; e < UNITS * 128; e += 256) {
      const double want = (double)((size_t)srcblk * (UNITS * 128) + e);
      if (d[e] != want) ++nb;
    }
    if (nb) {
      atomicAdd(bad, nb);
      atomicMax(where, (unsigned long long)blockIdx.x);
    }
    __syncthreads();
  }
}

__global__ void k_fill(double* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = (double)i;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const size_t n = (size_t)4096 * 38 * 128 + 1024;
  double* src;
  unsigned* bad;
  unsigned long long* where;
  CK(hipMalloc(&src, n * sizeof(double)));
  CK(hipMalloc(&bad, sizeof(unsigned)));
  CK(hipMalloc(&where, sizeof(unsigned long long)));
  hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, src, n);
  CK(hipFuncSetAttribute((const void*)k_probe, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
  for (int grid : {p.multiProcessorCount, 2 * p.multiProcessorCount}) {
    CK(hipMemset(bad, 0, sizeof(unsigned)));
    CK(hipMemset(where, 0, sizeof(unsigned long long)));
    hipLaunchKernelGGL(k_probe, dim3(grid), dim3(256), LDS_BYTES, 0, src, 2000, bad, where);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned hb = 0;
    unsigned long long hw = 0;
    CK(hipMemcpy(&hb, bad, sizeof hb, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hw, where, sizeof hw, hipMemcpyDeviceToHost));
    printf("grid %d (LDS %d B per workgroup): %u mismatched LDS words (last workgroup with one: %llu)\n", grid, LDS_BYTES, hb, hw);
  }
  return 0;
}
