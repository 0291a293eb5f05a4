// Microbenchmark (round 6): does the ISSUE ORDER of the fp64 chain's phase-1 MFMAs matter?
// Phase 1 forms Z[r] += V[ks][r]^T X[ks] for 8 reflector blocks r over 64 k-steps: 512
// v_mfma_f64_4x4x4_4b_f64 per wave and group. The engine issues them k-step-major (8 independent
// accumulators interleaved); r-major orders interleave only 2 or 4 accumulators (each accumulator's
// sum keeps its k order, so the results are bit-identical). tools/ubench/mfma_f64.hip measured 69.0
// TF/s with 8 accumulators and 76.0 with 2 (two waves per SIMD). Operands from registers only: 64
// X values (B), 8 x 2 A values, rotated per k-step so that every MFMA reads a different A register.
// 512 threads per workgroup (two waves per SIMD), one workgroup per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 mfma_order.hip -o mfma_order
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);         \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// (a scheduling barrier after every MFMA: left free, the compiler re-interleaves any order into
// the k-step-major one)
__device__ __forceinline__ double mf(double a, double b, double c) {
  const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  return d;
}

// ORD: 8 = k-step-major (8 accumulators interleaved, the engine's order), 4 = r-major in quads,
// 2 = r-major in pairs, 1 = one accumulator at a time
template <int ORD>
__global__ __launch_bounds__(512, 1) void k_order(double* out, const double* xin, unsigned long long* clk, int iters) {
  const int t = threadIdx.x;
  double X[64], A[2][8], Z[8];
#pragma unroll
  for (int k = 0; k < 64; ++k) X[k] = xin[k * 512 + t];  // 64 distinct B registers
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    A[0][r] = 1e-3 * (r + 1);
    A[1][r] = -1e-3 * (r + 2);
    Z[r] = 0.0;
  }
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (ORD == 8) {
#pragma unroll
      for (int ks = 0; ks < 64; ++ks)
#pragma unroll
        for (int r = 0; r < 8; ++r) Z[r] = mf(A[ks & 1][r], X[ks], Z[r]);
    } else {
#pragma unroll
      for (int r0 = 0; r0 < 8; r0 += ORD)
#pragma unroll
        for (int ks = 0; ks < 64; ++ks)
#pragma unroll
          for (int r = r0; r < r0 + ORD; ++r) Z[r] = mf(A[ks & 1][r], X[ks], Z[r]);
    }
    asm volatile("" ::: "memory");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  double s = 0.0;
#pragma unroll
  for (int r = 0; r < 8; ++r) s += Z[r];
  out[blockIdx.x * 512 + t] = s;
  if (t == 0) clk[blockIdx.x] = t1 - t0;
}

template <int ORD>
static int run(double* out, const double* xin, unsigned long long* clk, int nwg, int iters) {
  hipLaunchKernelGGL(k_order<ORD>, dim3(nwg), dim3(512), 0, 0, out, xin, clk, iters);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_order<ORD>, dim3(nwg), dim3(512), 0, 0, out, xin, clk, iters);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double flop = (double)nwg * 8 * iters * 512.0 * 512.0;  // 8 waves x 512 MFMAs x 512 flop
  printf("order %d (%s) %3d WG: %8.3f ms  %6.2f TFLOP/s\n", ORD,
         ORD == 8 ? "k-step-major, 8 accumulators" : ORD == 4 ? "r-major, 4 accumulators" : ORD == 2 ? "r-major, 2 accumulators" : "r-major, 1 accumulator",
         nwg, ms, flop / (ms * 1e-3) / 1e12);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  double* out;
  unsigned long long* clk;
  CK(hipMalloc(&out, sizeof(double) * ncu * 512));
  CK(hipMalloc(&clk, sizeof(unsigned long long) * ncu));
  double* xin;
  CK(hipMalloc(&xin, sizeof(double) * 64 * 512));
  CK(hipMemset(xin, 0, sizeof(double) * 64 * 512));
  const int iters = 400;
  for (int rep = 0; rep < 2; ++rep) {
    if (run<8>(out, xin, clk, ncu, iters)) return 1;
    if (run<4>(out, xin, clk, ncu, iters)) return 1;
    if (run<2>(out, xin, clk, ncu, iters)) return 1;
    if (run<1>(out, xin, clk, ncu, iters)) return 1;
  }
  return 0;
}
