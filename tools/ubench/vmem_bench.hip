// Microbenchmark: cost of the chain engine's vector-memory traffic per wave, 4 waves per CU, all
// CUs busy: (a) 32 x buffer_load_dwordx4 sc1 of a 16-column strip (the X strip), (b) 32 x
// buffer_store_dwordx4 sc1, (c) 20 x global_load_lds_dwordx4 (one group's V/T image share),
// (d) the same as (c) issued between MFMAs. Reports us per wave-pass (s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "tiles.hpp"
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
using namespace tqr;
typedef __attribute__((address_space(3))) void lds_t;
typedef __attribute__((address_space(1))) void glb_t;

template <int MODE>
__global__ __launch_bounds__(256, 1) void k_vmem(double* mat, const double* img, unsigned long long* out, int iters, long ldm) {
  extern __shared__ __align__(16) double lds[];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double X[64];
  for (int i = 0; i < 64; ++i) X[i] = i;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    // tile (it % 64, blockIdx) strip of 64 columns: wave w columns 16w..16w+15
    double* tile = mat + (size_t)(blockIdx.x % 64) * 256 * ldm + (size_t)((it + blockIdx.x) % 64) * 256;
    if (MODE == 0) {
      load_strip_pair<256, double>(X, tile, ldm, 16 * w);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (MODE == 1) {
      store_strip_pair<256, double>(X, tile, ldm, 16 * w);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (MODE == 2) {
      const double* src = img + (size_t)((it + blockIdx.x) % 512) * 9856;
      for (int m = 0; m < 20; ++m) {
        const int u = w + 4 * m;
        if (u < 77) __builtin_amdgcn_global_load_lds((glb_t*)(src + u * 128 + 2 * lane), (lds_t*)(lds + u * 128), 16, 0, 16);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      const double* src = img + (size_t)((it + blockIdx.x) % 512) * 9856;
      double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int m = 0; m < 20; ++m) {
        const int u = w + 4 * m;
        if (u < 77) __builtin_amdgcn_global_load_lds((glb_t*)(src + u * 128 + 2 * lane), (lds_t*)(lds + u * 128), 16, 0, 16);
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[r] = mfma4(X[r], X[8 + r], acc[r]);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int r = 0; r < 8; ++r) X[r] += acc[r] * 1e-30;
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
  for (int i = 0; i < 64; ++i) s += X[i];
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (s == 12345.678) out[0] = 0;
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int blocks = p.multiProcessorCount, iters = 200;
  const long ldm = 16384;
  double *mat, *img; unsigned long long* out;
  CK(hipMalloc(&mat, sizeof(double) * ldm * 16384)); CK(hipMemset(mat, 0, sizeof(double) * ldm * 16384));
  CK(hipMalloc(&img, sizeof(double) * 9856 * 512)); CK(hipMemset(img, 0, sizeof(double) * 9856 * 512));
  CK(hipMalloc(&out, sizeof(unsigned long long) * blocks));
  unsigned long long h[1024];
  const size_t lds = 9856 * 8;
  auto run = [&](auto kern, const char* name) -> int {
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (int r = 0; r < 2; ++r) {
      kern<<<blocks, 256, lds>>>(mat, img, out, iters, ldm);
      CK(hipDeviceSynchronize());
    }
    CK(hipMemcpy(h, out, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost));
    double s = 0; for (int b = 0; b < blocks; ++b) s += h[b];
    printf("%-44s %8.3f us per pass per wave\n", name, s / blocks / iters / 100.0);
    return 0;
  };
  run(k_vmem<0>, "32 x buffer_load_dwordx4 sc1 (strip)");
  run(k_vmem<1>, "32 x buffer_store_dwordx4 sc1 (strip)");
  run(k_vmem<2>, "20 x global_load_lds_dwordx4 sc1 (77 KB/CU)");
  run(k_vmem<3>, "20 x glds between 8-MFMA blocks");
  return 0;
}
