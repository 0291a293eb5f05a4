// Microbenchmark: latency of one reflector group of the TSQRT / GEQRT panel (tiles.hpp
// panel_factor, 32 reflectors on a 256-row block in LDS) at 256 and 512 threads per workgroup,
// one workgroup per CU, no global traffic. Prints us per group.
#include <hip/hip_runtime.h>
#include <cstdio>
#define TQR_BT_STAMPS
#include "tiles.hpp"
namespace tqr { __device__ unsigned long long g_bt[8]; }
#ifdef TQR_PS_STAMPS
namespace tqr { __device__ unsigned long long g_ps[8]; }
#endif
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
using namespace tqr;
constexpr int B = 256;
using G = Geo<B>;
constexpr int LDS_D = G::VSZ + 2 * G::TSZ + G::IB + 2 + 2 * 4 * 32 + 4 * 32 + 2 * 32 + G::TSZ;

template <bool TS, int NTH>
__global__ __launch_bounds__(NTH, 1) void k_panel(double* out, int iters) {
  extern __shared__ __align__(16) double lds[];
  double* Vs = lds;
  double* Hs = Vs + G::VSZ;
  double* tauv = Hs + G::TSZ;
  double* scratch = tauv + G::IB + 2;
  for (int i = threadIdx.x; i < LDS_D; i += NTH) lds[i] = 1e-2 * ((i * 37) % 101 - 50) + (i % 35 == 0 ? 1.0 : 0.0);
  __syncthreads();
  for (int it = 0; it < iters; ++it) panel_factor<B, TS, true>(Vs, Hs, tauv, scratch, TS ? 0 : 32 * (it & 3));
  __syncthreads();
  if (threadIdx.x < 64) out[blockIdx.x * 64 + threadIdx.x] = Vs[threadIdx.x] + tauv[threadIdx.x & 31];
}

template <int NTH>
__global__ __launch_bounds__(NTH, 1) void k_buildt(double* out, int iters) {
  extern __shared__ __align__(16) double lds[];
  double* Vs = lds;
  double* tauv = Vs + G::VSZ;
  double* Gs = tauv + G::IB + 2;
  double* Ts = Gs + G::TSZ;
  double* Gp = Ts + G::TSZ;
  for (int i = threadIdx.x; i < G::VSZ + G::IB + 2; i += NTH) lds[i] = 1e-2 * ((i * 37) % 101 - 50) + 1.0;
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    build_t<B>(Vs, tauv, Gs, Ts, Gp, 0);
    pack_t<B, NTH>(Ts, Gs);
    __syncthreads();
  }
  if (threadIdx.x < 64) out[blockIdx.x * 64 + threadIdx.x] = Gs[threadIdx.x];
}

template <int NTH>
static int run_bt(double* out, int blocks) {
  const size_t lds = (G::VSZ + G::IB + 2 + 6 * G::TSZ) * sizeof(double);
  CK(hipFuncSetAttribute((const void*)k_buildt<NTH>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 400;
  k_buildt<NTH><<<blocks, NTH, lds>>>(out, 4);
  CK(hipDeviceSynchronize());
  {
    unsigned long long z[8] = {0};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(tqr::g_bt), z, sizeof(z)));
  }
  float ms;
  CK(hipEventRecord(e0));
  k_buildt<NTH><<<blocks, NTH, lds>>>(out, iters);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("build_t+pack_t %3d threads: %7.2f us per group\n", NTH, ms * 1e3 / iters);
  unsigned long long bt[8];
  CK(hipMemcpyFromSymbol(bt, HIP_SYMBOL(tqr::g_bt), sizeof(bt)));
  const double tot = (double)(bt[3] - bt[0]);
  printf("   build_t phases (share of build_t, block 0): Gram %.0f%%, sum %.0f%%, back-subst %.0f%%\n",
         100.0 * (bt[1] - bt[0]) / tot, 100.0 * (bt[2] - bt[1]) / tot, 100.0 * (bt[3] - bt[2]) / tot);
  unsigned long long z[8] = {0};
  CK(hipMemcpyToSymbol(HIP_SYMBOL(tqr::g_bt), z, sizeof(z)));
  return 0;
}

template <bool TS, int NTH>
static int run(const char* name, double* out, int blocks) {
  const size_t lds = LDS_D * sizeof(double);
  CK(hipFuncSetAttribute((const void*)k_panel<TS, NTH>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 400;
  k_panel<TS, NTH><<<blocks, NTH, lds>>>(out, 4);
  CK(hipDeviceSynchronize());
  float ms;
#ifdef TQR_PS_STAMPS
  {
    unsigned long long z[8] = {0};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(tqr::g_ps), z, sizeof(z)));
  }
#endif
  CK(hipEventRecord(e0));
  k_panel<TS, NTH><<<blocks, NTH, lds>>>(out, iters);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-8s %3d threads: %7.2f us per group (%5.3f us per reflector)\n", name, NTH, ms * 1e3 / iters,
         ms * 1e3 / iters / G::IB);
#ifdef TQR_PS_STAMPS
  unsigned long long ps[8];
  CK(hipMemcpyFromSymbol(ps, HIP_SYMBOL(tqr::g_ps), sizeof(ps)));
  double tot = 0;
  for (int i = 0; i < 5; ++i) tot += (double)ps[i];
  const double per = tot / (iters * (double)G::IB);  // s_memtime ticks per reflector step (wave 0 of block 0)
  printf("   step phases (wave 0, %.0f ticks per step): products+reduce %.0f%%, barrier+sums %.0f%%, scalar %.0f%%, "
         "f broadcast %.0f%%, update+shift %.0f%%\n", per, 100 * ps[0] / tot, 100 * ps[1] / tot, 100 * ps[2] / tot,
         100 * ps[3] / tot, 100 * ps[4] / tot);
#endif
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  double* out;
  CK(hipMalloc(&out, p.multiProcessorCount * 64 * sizeof(double)));
  for (int blocks : {1, p.multiProcessorCount}) {
    printf("-- %d workgroup(s)\n", blocks);
    if (run<true, 256>("TSQRT", out, blocks) || run<true, 512>("TSQRT", out, blocks) ||
        run<false, 256>("GEQRT", out, blocks) || run<false, 512>("GEQRT", out, blocks) ||
        run_bt<256>(out, blocks) || run_bt<512>(out, blocks))
      return 1;
  }
  return 0;
}
