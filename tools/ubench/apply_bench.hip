// Microbenchmark: throughput of the chain's inner block-reflector application (tiles.hpp
// apply_group<256, HEAD=true>) with V/T resident in LDS and the strip in registers — no global
// traffic, no synchronisation. One 256-thread workgroup per CU (as k_flow). Reports the
// algorithmic rate 4*b*IB*16 flop per wave per group against the 78.6 TF fp64 peak.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "tiles.hpp"
#include "gridscheduler.h"
namespace tqr { struct Item { int ts, l, m, k; }; }
#include "flow.hpp"
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
using namespace tqr;
constexpr int B = 256;
using G = Geo<B>;

__global__ __launch_bounds__(256, 1) void k_apply(double* out, int iters) {
  extern __shared__ __align__(16) double lds[];
  double* Vs = lds;
  double* Ts = Vs + G::VSZ;
  for (int i = threadIdx.x; i < G::VSZ + G::TSZ; i += 256) lds[i] = 1e-3 * ((i * 37) % 101 - 50) / 50.0;
  __syncthreads();
  double X[G::NKS], H[G::NRI];
  for (int k = 0; k < G::NKS; ++k) X[k] = 1.0 + 1e-3 * (threadIdx.x + k);
  for (int r = 0; r < G::NRI; ++r) H[r] = 0.5 + 1e-3 * r;
  for (int it = 0; it < iters; ++it) {
    asm volatile("" ::: "memory");
    apply_group<B, true>(Vs, Ts, X, H, 0);
  }
  double s = 0;
  for (int k = 0; k < G::NKS; ++k) s += X[k];
  for (int r = 0; r < G::NRI; ++r) s += H[r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}


// software-pipelined variant: the LDS reads of k-step ks+1 are issued before the MFMAs of ks
template <int B, bool HEAD>
__device__ __forceinline__ void apply_group_sp(const double* __restrict__ Vs, const double* __restrict__ Ts,
                                               double (&X)[Geo<B>::NKS], double (&H)[Geo<B>::NRI], int ks0) {
  using g = Geo<B>;
  constexpr int NRI = g::NRI, NKS = g::NKS, VP = g::VP, TP = g::TP;
  const int lane = threadIdx.x & 63, x = lane >> 4, y = lane & 3;
  double Z[NRI];
#pragma unroll
  for (int r = 0; r < NRI; ++r) Z[r] = HEAD ? H[r] : 0.0;
  auto ldz = [&](double (&a)[NRI], int ks) {
    const double2* vr = reinterpret_cast<const double2*>(Vs + (4 * ks + x) * VP + y * NRI);
#pragma unroll
    for (int h = 0; h < NRI / 2; ++h) { double2 t = vr[h]; a[2 * h] = t.x; a[2 * h + 1] = t.y; }
  };
  double ac[NRI], an[NRI];
  ldz(ac, 0);
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    asm volatile("" ::: "memory");
    if (ks + 1 < NKS) ldz(an, ks + 1);
#pragma unroll
    for (int r = 0; r < NRI; ++r) Z[r] = mfma4(ac[r], X[ks], Z[r]);
#pragma unroll
    for (int r = 0; r < NRI; ++r) ac[r] = an[r];
  }
  double W[NRI];
#pragma unroll
  for (int wi = 0; wi < NRI; ++wi) {
    double acc = 0.0;
#pragma unroll
    for (int k2 = 0; k2 <= wi; ++k2) acc = mfma4(Ts[(4 * k2 + x) * TP + 4 * wi + y], Z[k2], acc);
    W[wi] = -acc;
  }
  if (HEAD) {
#pragma unroll
    for (int r = 0; r < NRI; ++r) H[r] += W[r];
  }
  auto ldx = [&](double (&a)[NRI], int ks) {
    const double2* vr = reinterpret_cast<const double2*>(Vs + (4 * ks + y) * VP + x * NRI);
#pragma unroll
    for (int h = 0; h < NRI / 2; ++h) { double2 t = vr[h]; a[2 * h] = t.x; a[2 * h + 1] = t.y; }
  };
  double bc[2][NRI], bn[2][NRI];
  ldx(bc[0], 0); ldx(bc[1], 1);
#pragma unroll
  for (int kb = 0; kb < NKS; kb += 2) {
    asm volatile("" ::: "memory");
    if (kb + 2 < NKS) { ldx(bn[0], kb + 2); ldx(bn[1], kb + 3); }
#pragma unroll
    for (int wi = 0; wi < NRI; ++wi)
#pragma unroll
      for (int u = 0; u < 2; ++u) X[kb + u] = mfma4(bc[u][wi], W[wi], X[kb + u]);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < NRI; ++r) bc[u][r] = bn[u][r];
  }
}

__global__ __launch_bounds__(256, 1) void k_apply_sp(double* out, int iters) {
  extern __shared__ __align__(16) double lds[];
  double* Vs = lds;
  double* Ts = Vs + G::VSZ;
  for (int i = threadIdx.x; i < G::VSZ + G::TSZ; i += 256) lds[i] = 1e-3 * ((i * 37) % 101 - 50) / 50.0;
  __syncthreads();
  double X[G::NKS], H[G::NRI];
  for (int k = 0; k < G::NKS; ++k) X[k] = 1.0 + 1e-3 * (threadIdx.x + k);
  for (int r = 0; r < G::NRI; ++r) H[r] = 0.5 + 1e-3 * r;
  for (int it = 0; it < iters; ++it) {
    asm volatile("" ::: "memory");
    apply_group_sp<B, true>(Vs, Ts, X, H, 0);
  }
  double s = 0;
  for (int k = 0; k < G::NKS; ++k) s += X[k];
  for (int r = 0; r < G::NRI; ++r) s += H[r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}


// two 16-column strips per wave: every LDS operand read feeds two MFMAs
template <int B>
__device__ __forceinline__ void apply2(const double* __restrict__ Vs, const double* __restrict__ Ts,
                                       double (&X0)[Geo<B>::NKS], double (&X1)[Geo<B>::NKS],
                                       double (&H0)[Geo<B>::NRI], double (&H1)[Geo<B>::NRI]) {
  using g = Geo<B>;
  constexpr int NRI = g::NRI, NKS = g::NKS, VP = g::VP, TP = g::TP;
  const int lane = threadIdx.x & 63, x = lane >> 4, y = lane & 3;
  double Z0[NRI], Z1[NRI];
#pragma unroll
  for (int r = 0; r < NRI; ++r) { Z0[r] = H0[r]; Z1[r] = H1[r]; }
  auto ldz = [&](double (&a)[NRI], int ks) {
    const double2* vr = reinterpret_cast<const double2*>(Vs + (4 * ks + x) * VP + y * NRI);
#pragma unroll
    for (int h = 0; h < NRI / 2; ++h) { const double2 t = vr[h]; a[2 * h] = t.x; a[2 * h + 1] = t.y; }
  };
  {
    double ac[NRI], an[NRI];
    ldz(ac, 0);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      asm volatile("" ::: "memory");
      if (ks + 1 < NKS) ldz(an, ks + 1);
#pragma unroll
      for (int r = 0; r < NRI; ++r) { Z0[r] = mfma4(ac[r], X0[ks], Z0[r]); Z1[r] = mfma4(ac[r], X1[ks], Z1[r]); }
#pragma unroll
      for (int r = 0; r < NRI; ++r) ac[r] = an[r];
    }
  }
  double W0[NRI], W1[NRI];
#pragma unroll
  for (int wi = 0; wi < NRI; ++wi) {
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int k2 = 0; k2 <= wi; ++k2) {
      const double tv = Ts[(4 * k2 + x) * TP + 4 * wi + y];
      a0 = mfma4(tv, Z0[k2], a0);
      a1 = mfma4(tv, Z1[k2], a1);
    }
    W0[wi] = -a0; W1[wi] = -a1;
  }
#pragma unroll
  for (int r = 0; r < NRI; ++r) { H0[r] += W0[r]; H1[r] += W1[r]; }
  auto ldx = [&](double (&a)[NRI], int ks) {
    const double2* vr = reinterpret_cast<const double2*>(Vs + (4 * ks + y) * VP + x * NRI);
#pragma unroll
    for (int h = 0; h < NRI / 2; ++h) { const double2 t = vr[h]; a[2 * h] = t.x; a[2 * h + 1] = t.y; }
  };
  {
    double bc[NRI], bn[NRI];
    ldx(bc, 0);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      asm volatile("" ::: "memory");
      if (ks + 1 < NKS) ldx(bn, ks + 1);
#pragma unroll
      for (int wi = 0; wi < NRI; ++wi) {
        X0[ks] = mfma4(bc[wi], W0[wi], X0[ks]);
        X1[ks] = mfma4(bc[wi], W1[wi], X1[ks]);
      }
#pragma unroll
      for (int r = 0; r < NRI; ++r) bc[r] = bn[r];
    }
  }
}

__global__ __launch_bounds__(256, 1) void k_apply2(double* out, int iters) {
  extern __shared__ __align__(16) double lds[];
  double* Vs = lds;
  double* Ts = Vs + G::VSZ;
  for (int i = threadIdx.x; i < G::VSZ + G::TSZ; i += 256) lds[i] = 1e-3 * ((i * 37) % 101 - 50) / 50.0;
  __syncthreads();
  double X0[G::NKS], X1[G::NKS], H0[G::NRI], H1[G::NRI];
  for (int k = 0; k < G::NKS; ++k) { X0[k] = 1.0 + 1e-3 * (threadIdx.x + k); X1[k] = 1.0 - 1e-3 * (threadIdx.x + k); }
  for (int r = 0; r < G::NRI; ++r) { H0[r] = 0.5 + 1e-3 * r; H1[r] = 0.25 + 1e-3 * r; }
  for (int it = 0; it < iters; ++it) {
    asm volatile("" ::: "memory");
    apply2<B>(Vs, Ts, X0, X1, H0, H1);
  }
  double s = 0;
  for (int k = 0; k < G::NKS; ++k) s += X0[k] + X1[k];
  for (int r = 0; r < G::NRI; ++r) s += H0[r] + H1[r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}


// the chain's group step without global data dependencies: apply_zw with the next group's
// LDS-DMA in its hook (DMA on/off), apply_x, vmcnt(0) + barrier per group
template <bool DMA>
__global__ __launch_bounds__(256, 1) void k_apply_dma(double* out, const double* img, int iters) {
  extern __shared__ __align__(16) double lds[];
  constexpr int BUF = G::VIMG + G::TIMG;
  for (int i = threadIdx.x; i < 2 * BUF; i += 256) lds[i] = 1e-3 * ((i * 37) % 101 - 50) / 50.0;
  __syncthreads();
  double X[G::NKS], H[G::NRI], W[G::NRI];
  for (int k = 0; k < G::NKS; ++k) X[k] = 1.0 + 1e-3 * (threadIdx.x + k);
  for (int r = 0; r < G::NRI; ++r) H[r] = 0.5 + 1e-3 * r;
  int buf = 0;
  for (int it = 0; it < iters; ++it) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const double* Vs = lds + buf * BUF;
    const double* src = img + (size_t)((it + blockIdx.x) % 512) * BUF;
    if constexpr (DMA) {
      DmaJob<B> d{lds + (buf ^ 1) * BUF, src, src + G::VIMG};
      apply_zw<B, true>(Vs, Vs + G::VIMG, X, H, W, 0, d);
    } else {
      apply_zw<B, true>(Vs, Vs + G::VIMG, X, H, W, 0);
    }
    apply_x<B, true>(Vs, X, W, 0);
    buf ^= 1;
  }
  double s = 0;
  for (int k = 0; k < G::NKS; ++k) s += X[k];
  for (int r = 0; r < G::NRI; ++r) s += H[r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}


// 8 waves per workgroup (two per SIMD), reads not software-pipelined
__global__ __launch_bounds__(512, 1) void k_apply8(double* out, int iters) {
  extern __shared__ __align__(16) double lds[];
  double* Vs = lds;
  double* Ts = Vs + G::VSZ;
  for (int i = threadIdx.x; i < G::VSZ + G::TSZ; i += 512) lds[i] = 1e-3 * ((i * 37) % 101 - 50) / 50.0;
  __syncthreads();
  double X[G::NKS], H[G::NRI];
  for (int k = 0; k < G::NKS; ++k) X[k] = 1.0 + 1e-3 * (threadIdx.x + k);
  for (int r = 0; r < G::NRI; ++r) H[r] = 0.5 + 1e-3 * r;
  for (int it = 0; it < iters; ++it) {
    asm volatile("" ::: "memory");
    apply_group<B, true, false>(Vs, Ts, X, H, 0);
  }
  double s = 0;
  for (int k = 0; k < G::NKS; ++k) s += X[k];
  for (int r = 0; r < G::NRI; ++r) s += H[r];
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  const int blocks = p.multiProcessorCount, iters = 2000;
  double* out; CK(hipMalloc(&out, blocks * 512 * sizeof(double)));
  const size_t lds = (G::VSZ + G::TSZ) * sizeof(double);
  CK(hipFuncSetAttribute((const void*)k_apply, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)k_apply2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)k_apply_sp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  k_apply<<<blocks, 256, lds>>>(out, iters / 4);
  CK(hipDeviceSynchronize());
  CK(hipFuncSetAttribute((const void*)k_apply8, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
    CK(hipEventRecord(e0)); k_apply8<<<blocks, 512, lds>>>(out, iters); CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    const double fl = (double)blocks * 8 * iters * 4.0 * B * G::IB * 16;
    printf("8-wave WG, 2 waves/SIMD, no read pipelining: %.2f TFLOP/s (%.1f%% of 78.6), %.2f us per group (128 cols)\n", fl / ms / 1e9, fl / ms / 1e9 / 78.6 * 100, ms * 1e3 / iters);
  }
  {
    double* img; CK(hipMalloc(&img, sizeof(double) * 9856 * 520)); CK(hipMemset(img, 0, sizeof(double) * 9856 * 520));
    const size_t l2 = 2 * (G::VIMG + G::TIMG) * 8;
    CK(hipFuncSetAttribute((const void*)k_apply_dma<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l2));
    CK(hipFuncSetAttribute((const void*)k_apply_dma<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l2));
    for (int rep = 0; rep < 4; ++rep) {
      float ms;
      CK(hipEventRecord(e0));
      if (rep & 1) k_apply_dma<true><<<blocks, 256, l2>>>(out, img, iters); else k_apply_dma<false><<<blocks, 256, l2>>>(out, img, iters);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      printf("group step %s: %.2f us/group\n", (rep & 1) ? "with DMA   " : "without DMA", ms * 1e3 / iters);
    }
  }
  for (int rep = 0; rep < 3; ++rep) {
    float ms;
    CK(hipEventRecord(e0)); k_apply2<<<blocks, 256, lds>>>(out, iters / 2); CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    const double fl = (double)blocks * 4 * (iters / 2) * 2 * 4.0 * B * G::IB * 16;
    printf("2-strip    apply x%d, %d WG: %.3f ms  %.2f TFLOP/s  (%.1f%% of 78.6)\n", iters / 2, blocks, ms, fl / ms / 1e9, fl / ms / 1e9 / 78.6 * 100);
  }
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    CK(hipEventRecord(e0));
    if (rep % 2 == 1) k_apply_sp<<<blocks, 256, lds>>>(out, iters);
    else k_apply<<<blocks, 256, lds>>>(out, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    const double fl = (double)blocks * 4 * iters * 4.0 * B * G::IB * 16;
    printf("%s apply_group<256,TS> x%d, %d WG: %.3f ms  %.2f TFLOP/s  (%.1f%% of 78.6), %.2f us/group\n", rep % 2 == 1 ? "bench-copy" : "tiles.hpp ", iters, blocks, ms,
           fl / ms / 1e9, fl / ms / 1e9 / 78.6 * 100, ms * 1e3 / iters);
  }
  return 0;
}
