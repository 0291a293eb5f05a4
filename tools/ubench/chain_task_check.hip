// The engine's chain task functions themselves — flow_chain_asm (hand-scheduled) and flow_chain
// (compiler-scheduled) — called by one workgroup on synthetic inputs: a p x q tile matrix, the
// panel-k workspace filled with random V/T images, every panel counter already "published".
// Runs CHAIN(k=0, j=1, s, seg 0) over rows i = 0 (UNMQR) .. i1-1 for each strip s and compares the
// tile column j of both versions. Diagnostic for the asm chain's task-level glue (it found the stale-readfirstlane hazard, see
// chain_asm.hpp sreg). LDS is poisoned before every launch so stale images of an earlier launch cannot
// pass for fresh ones.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I../../gpu-tiled-qr-decomposition_amd/csrc chain_task_check.hip -o chain_task_check
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <vector>

#include "gridscheduler.h"
namespace tqr {
struct Item {
  int ts, l, m, k;
};
}  // namespace tqr
#include "flow.hpp"

using namespace tqr;
#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                 \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

template <int B, int ASM>
__global__ __launch_bounds__(512, 1) void k_task(FlowArgs a, int s, int i1) {
  extern __shared__ __align__(16) double lds[];
  int* s_task = reinterpret_cast<int*>(lds + flow_lds_doubles<B, double, ShapeW8>());
  int* sflag = s_task + 1;
  {  // LDS poisoned with a recognisable value (1.0e300): stale images from an earlier launch can't pass for fresh ones
    constexpr int ND = flow_lds_doubles<B, double, ShapeW8>();
    for (int e = threadIdx.x; e < ND; e += 512) lds[e] = 1.0e300;
    for (int e = threadIdx.x; e < 384; e += 512) s_task[e] = 0;
    __syncthreads();
  }
  if (ASM)
    flow_chain_asm<B, ShapeW8>(a, s, 1, i1, 1, 0, 0, lds, sflag);
  else
    flow_chain<B, double, ShapeW8>(a, s, 1, i1, 1, 0, 0, lds, sflag);
}

__global__ void k_fill(double* p, size_t n, double scale, unsigned long long seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned long long z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 31;
    p[i] = scale * (((double)(z % 2001) - 1000.0) / 1000.0);
  }
}

template <int B>
static int run(int p) {
  const int q = 2, m = p * B, n = q * B, ns = B / 128;
  using G = FGeo<B, ShapeW8>;
  const int NG = G::NG;
  const size_t wk_d = (size_t)p * NG * (FImg<B, double, ShapeW8>::V + FImg<B, double, ShapeW8>::T);
  double *A0, *A1, *A2, *wk, **dwk;
  int* ctr;
  CK(hipMalloc(&A0, (size_t)m * n * 8));
  CK(hipMalloc(&A1, (size_t)m * n * 8));
  CK(hipMalloc(&A2, (size_t)m * n * 8));
  CK(hipMalloc(&wk, wk_d * 8));
  CK(hipMalloc(&dwk, sizeof(double*)));
  CK(hipMemcpy(dwk, &wk, sizeof(double*), hipMemcpyHostToDevice));
  const int nctr = 4096;
  CK(hipMalloc(&ctr, nctr * 4));
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, A0, (size_t)m * n, 1.0, 1ull);
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, wk, wk_d, 0.05, 3ull);
  CK(hipMemcpy(A1, A0, (size_t)m * n * 8, hipMemcpyDeviceToDevice));
  CK(hipMemcpy(A2, A0, (size_t)m * n * 8, hipMemcpyDeviceToDevice));
  std::vector<int> hc(nctr, 0);
  for (int g = 0; g < NG; ++g) hc[4 + g] = 1 << 20;  // Rc[0][g]: every member of panel 0 published
  FlowArgs f{};
  f.Wk = dwk;
  f.ldm = m;
  f.m = m;
  f.p = p;
  f.q = q;
  f.kmax = 1;
  f.ns = ns;
  f.next = ctr;
  f.err = ctr + 1;
  f.exitc = ctr + 3;
  f.Rc = ctr + 4;
  f.Tc = f.Rc + 64;
  f.Ac = f.Tc + 1024;
  f.Rt = f.Ac + 1024;
  f.Rr = f.Rt + 64;
  f.cdiv = 1;
  f.seglen = 8;
  f.seglen_la = 8;
  const size_t lds = flow_lds_doubles<B, double, ShapeW8>() * 8 + 1536;
  CK(hipFuncSetAttribute((const void*)k_task<B, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)k_task<B, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int v = 0; v < 2; ++v) {
    CK(hipMemcpy(ctr, hc.data(), nctr * 4, hipMemcpyHostToDevice));
    f.A = v ? A1 : A2;
    for (int s = 0; s < ns; ++s) {
      if (v)
        hipLaunchKernelGGL((k_task<B, 1>), dim3(1), dim3(512), lds, 0, f, s, p);
      else
        hipLaunchKernelGGL((k_task<B, 0>), dim3(1), dim3(512), lds, 0, f, s, p);
      CK(hipDeviceSynchronize());
    }
    int err = 0;
    CK(hipMemcpy(&err, ctr + 1, 4, hipMemcpyDeviceToHost));
    if (err) printf("  variant %d: engine error word %d\n", v, err);
  }
  std::vector<double> a(m * (size_t)n), b(m * (size_t)n), o(m * (size_t)n);
  CK(hipMemcpy(a.data(), A1, (size_t)m * n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), A2, (size_t)m * n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o.data(), A0, (size_t)m * n * 8, hipMemcpyDeviceToHost));
  double d = 0, mx = 0, dch = 0;
  int nn = 0;
  for (int c = B; c < 2 * B; ++c)
    for (int r = 0; r < m; ++r) {
      const size_t e = (size_t)c * m + r;
      nn += !std::isfinite(a[e]);
      d = fmax(d, fabs(a[e] - b[e]));
      mx = fmax(mx, fabs(b[e]));
      dch = fmax(dch, fabs(b[e] - o[e]));
    }
  printf("B=%d p=%d: tile column 1 max|asm - C++| %.3e (max %.3e, changed by C++ %.3e), %d non-finite\n", B, p, d, mx,
         dch, nn);
  if (d > 1e-12 || nn) {
    // error by wave strip (16 columns) x 32-row block
    for (int w = 0; w < B / 16; ++w) {
      printf("   strip %2d:", w);
      for (int rb = 0; rb < m / 32; ++rb) {
        double e = 0;
        int bad = 0;
        for (int c = B + 16 * w; c < B + 16 * w + 16; ++c)
          for (int r = 32 * rb; r < 32 * rb + 32; ++r) {
            const size_t ix = (size_t)c * m + r;
            if (!std::isfinite(a[ix])) bad = 1;
            else e = fmax(e, fabs(a[ix] - b[ix]));
          }
        if (bad) printf("   NaN  ");
        else printf(" %7.1e", e);
      }
      printf("\n");
    }
  }
  return 0;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 1;
  for (int r = 0; r < reps; ++r)
    if (run<128>(1)) return 1;
  for (int p : {1, 2, 3})
    if (run<128>(p)) return 1;
  for (int p : {1, 2, 3})
    if (run<256>(p)) return 1;
  return 0;
}
