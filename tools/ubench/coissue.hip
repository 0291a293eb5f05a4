// Microbenchmark: can fp64 vector FMAs (v_fma_f64) run beside fp64 MFMAs (v_mfma_f64_4x4x4_4b)
// on the same SIMD? If the matrix core and the VALU's fp64 datapath are separate, the combined
// rate exceeds either alone; if they share it, the sum stays at one unit's peak.
// Variants (one workgroup per CU, all CUs):
//   mfma      4 or 8 waves, each 8 independent 4x4x4 accumulators
//   fma       4 or 8 waves, each 8 independent v_fma_f64 chains
//   split     8 waves: waves 0-3 MFMA, waves 4-7 FMA (two waves per SIMD, one of each)
//   mixed     4 waves, each interleaving R MFMAs with F FMAs per iteration
// Build: hipcc --offload-arch=gfx950 -O3 coissue.hip -o coissue
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ void mfma8(double (&acc)[8], double a, double b) {
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
}
template <int NF>
__device__ __forceinline__ void fmaN(double (&x)[16], double a, double b) {
#pragma unroll
  for (int i = 0; i < NF; ++i) x[i % 16] = __builtin_fma(x[i % 16], a, b);
}

// MODE 0: all waves MFMA; 1: all waves FMA; 2: waves < 4 MFMA, >= 4 FMA; 3: every wave mixes
// 8 MFMAs with NF FMAs per iteration
template <int MODE, int NF>
__global__ __launch_bounds__(512) void k_co(double* out, unsigned long long* clk, int iters, double seed) {
  double acc[8], x[16];
  for (int i = 0; i < 8; ++i) acc[i] = seed * i;
  for (int i = 0; i < 16; ++i) x[i] = seed + i + threadIdx.x * 1e-3;
  const double a = seed * (threadIdx.x + 1), b = seed * 0.5 - threadIdx.x * 1e-7;
  const double fa = 0.9999999, fb = 1e-9 * threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x == 0) clk[blockIdx.x * 2] = __builtin_amdgcn_s_memrealtime();
  const bool dom = MODE == 0 || MODE == 3 || (MODE == 2 && w < 4);
  const bool dof = MODE == 1 || MODE == 3 || (MODE == 2 && w >= 4);
  if (dom && dof) {
    for (int it = 0; it < iters; ++it) {
      mfma8(acc, a, b);
      fmaN<NF>(x, fa, fb);
    }
  } else if (dom) {
    for (int it = 0; it < iters; ++it) mfma8(acc, a, b);
  } else {
    for (int it = 0; it < iters; ++it) fmaN<NF>(x, fa, fb);
  }
  __syncthreads();
  if (threadIdx.x == 0) clk[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime();
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  for (int i = 0; i < 16; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int nb = p.multiProcessorCount;
  double* out;
  CK(hipMalloc(&out, nb * 512 * sizeof(double)));
  unsigned long long *clk, *h = new unsigned long long[nb * 2];
  CK(hipMalloc(&clk, nb * 2 * sizeof(unsigned long long)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20000;
  float ms;
  // MFMA: 8 x 512 flop per wave-iteration; FMA: NF x 64 lanes x 2 flop
#define RUN(NAME, MODE, NF, THREADS, MFLOP, FFLOP)                                                           \
  k_co<MODE, NF><<<nb, THREADS>>>(out, clk, iters, 1e-3);                                                   \
  CK(hipEventRecord(e0));                                                                                    \
  k_co<MODE, NF><<<nb, THREADS>>>(out, clk, iters, 1e-3);                                                   \
  CK(hipEventRecord(e1));                                                                                    \
  CK(hipEventSynchronize(e1));                                                                               \
  CK(hipEventElapsedTime(&ms, e0, e1));                                                                      \
  printf("%-44s %8.3f ms  mfma %6.2f  fma %6.2f  total %6.2f TFLOP/s\n", NAME, ms,                          \
         (double)nb * iters * (MFLOP) / ms / 1e9, (double)nb * iters * (FFLOP) / ms / 1e9,                   \
         (double)nb * iters * ((MFLOP) + (FFLOP)) / ms / 1e9);
  RUN("mfma only, 4 waves", 0, 8, 256, 4.0 * 8 * 512, 0.0);
  RUN("mfma only, 8 waves", 0, 8, 512, 8.0 * 8 * 512, 0.0);
  RUN("fma only (16 chains), 4 waves", 1, 16, 256, 0.0, 4.0 * 16 * 128);
  RUN("fma only (16 chains), 8 waves", 1, 16, 512, 0.0, 8.0 * 16 * 128);
  RUN("split: 4 mfma waves + 4 fma waves", 2, 16, 512, 4.0 * 8 * 512, 4.0 * 16 * 128);
  RUN("split: 4 mfma waves + 4 fma waves (8 fma)", 2, 8, 512, 4.0 * 8 * 512, 4.0 * 8 * 128);
  RUN("mixed: 8 mfma + 4 fma per wave, 4 waves", 3, 4, 256, 4.0 * 8 * 512, 4.0 * 4 * 128);
  RUN("mixed: 8 mfma + 8 fma per wave, 4 waves", 3, 8, 256, 4.0 * 8 * 512, 4.0 * 8 * 128);
  RUN("mixed: 8 mfma + 16 fma per wave, 4 waves", 3, 16, 256, 4.0 * 8 * 512, 4.0 * 16 * 128);
  RUN("mixed: 8 mfma + 8 fma per wave, 8 waves", 3, 8, 512, 8.0 * 8 * 512, 8.0 * 8 * 128);
  return 0;
}
