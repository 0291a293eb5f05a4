// Probe: operand/result lane maps of v_mfma_f64_4x4x4_4b_f64 (with and without CBSZ/ABID
// A-broadcast) and of v_mfma_f64_16x16x4_f64, by one-hot A operands with distinct B values.
// Plus the issue rate of the broadcast 4x4x4 form. Output is parsed by hand (DESIGN.md notes).
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void probe(double* out) {
  int l = threadIdx.x;
  for (int p = 0; p < 64; ++p) {
    double a = (l == p) ? 1.0 : 0.0;
    double b = (double)(l + 1);
    if (MODE == 0) { double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0); out[p * 64 + l] = d; }
    if (MODE == 1) { double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 2, 0, 0); out[p * 64 + l] = d; }
    if (MODE == 2) { double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 2, 1, 0); out[p * 64 + l] = d; }
    if (MODE == 3) { d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d4{0, 0, 0, 0}, 0, 0, 0);
                     for (int r = 0; r < 4; ++r) out[(p * 64 + l) * 4 + r] = d[r]; }
  }
}

template <int NACC>
__global__ __launch_bounds__(256) void rate_bcast(double* out, int iters, double seed) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = seed * i;
  double a = seed * (threadIdx.x + 1), b = seed * 0.5 - threadIdx.x * 1e-7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if ((i & 3) == 0) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 2, 0, 0);
      if ((i & 3) == 1) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 2, 1, 0);
      if ((i & 3) == 2) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 2, 2, 0);
      if ((i & 3) == 3) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 2, 3, 0);
    }
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double* d; CK(hipMalloc(&d, 64 * 64 * 4 * sizeof(double)));
  double* h = new double[64 * 64 * 4];
  const char* names[4] = {"4x4x4 plain", "4x4x4 cbsz2 abid0", "4x4x4 cbsz2 abid1", "16x16x4"};
  for (int mode = 0; mode < 4; ++mode) {
    if (mode == 0) probe<0><<<1, 64>>>(d);
    if (mode == 1) probe<1><<<1, 64>>>(d);
    if (mode == 2) probe<2><<<1, 64>>>(d);
    if (mode == 3) probe<3><<<1, 64>>>(d);
    CK(hipDeviceSynchronize());
    int R = mode == 3 ? 4 : 1;
    CK(hipMemcpy(h, d, 64 * 64 * R * sizeof(double), hipMemcpyDeviceToHost));
    printf("== %s: for A one-hot lane p: list of (outlane[.reg]=Blane) ==\n", names[mode]);
    for (int p = 0; p < 64; ++p) {
      printf("p%02d:", p);
      for (int l = 0; l < 64; ++l) for (int r = 0; r < R; ++r) {
        double v = h[(p * 64 + l) * R + r];
        if (v != 0) { if (R > 1) printf(" %d.%d=%d", l, r, (int)v - 1); else printf(" %d=%d", l, (int)v - 1); }
      }
      printf("\n");
    }
  }
  hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, 0));
  double* out; CK(hipMalloc(&out, pr.multiProcessorCount * 2 * 256 * sizeof(double)));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int bpc = 1; bpc <= 2; ++bpc) {
    int blocks = pr.multiProcessorCount * bpc; int iters = 20000; float ms;
    rate_bcast<8><<<blocks, 256>>>(out, 100, 1e-3);
    CK(hipEventRecord(e0)); rate_bcast<8><<<blocks, 256>>>(out, iters, 1e-3); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("4x4x4 bcast x8acc %d wave/SIMD: %.3f ms %.2f TFLOP/s (512 flop/instr)\n", bpc, ms, (double)blocks * 4 * iters * 8 * 512.0 / ms / 1e9);
  }
  return 0;
}
