// Microbenchmark: the fp64 chain's element loop (TSMQR on one column strip of a 256-row tile,
// reflector group by group) in two workgroup shapes, without the engine's dependencies:
//   w8ib32  one 8-wave workgroup per CU, 128-column strips, 32-reflector groups (the round-3 engine:
//           every wave of the CU in one barrier-synchronised group loop, 152 KiB of LDS images)
//   w4ib16  TWO 4-wave workgroups per CU, 64-column strips each, 16-reflector groups (76 KiB of LDS
//           images per workgroup): the two are independent, so one's strip hand-over, barrier
//           waits and dependent-MFMA tails run beside the other's MFMA stream
//   w4ib32  one 4-wave workgroup per CU, 64-column strips, 32-reflector groups (reference point)
// Per element: strip loads (paired rows, 16-B sc1|nt), per group: barrier (waits for the group's
// LDS-DMA'd V/T images), phase 1 Z = H + V^T X, W = -T^T Z, H += W (the next group's images
// LDS-DMA'd inside it), head-row store + next head-row load, phase 2 X += V W; strip stores (sc1)
// at the end. Data: every workgroup streams its own tile rows from HBM (ldm 16384), images from a
// shared 64-tile pool (L2 / MALL), like the engine. TF/s counts the algorithmic TSMQR flops
// (4 b^2 per column). MODE bits: 1 = no strip I/O, 2 = no head I/O, 4 = the engine's hand-over (the
// finished strip stored and the next one loaded row pair by row pair inside the last group's
// phase 2, loads trailing stores by 2 pairs), 8 = plain (write-back) strip stores instead of sc1,
// 16 = stagger: the second half of the workgroups first runs half an element of groups without I/O
// (two-per-CU shapes: the two workgroups of a CU out of phase, as different tasks are in the engine),
// 32 = desync: every workgroup first runs (5 blockIdx) mod NG groups without I/O, so the element
// hand-overs of the CUs are spread over time as in the engine (without it every CU streams its
// strips at the same moment and the chip's HBM sees the sum as one burst).
// Build: hipcc --offload-arch=gfx950 -O3 -I../../gpu-tiled-qr-decomposition_amd/csrc chain2_bench.hip -o chain2_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "tiles.hpp"

using namespace tqr;
#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                   \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

constexpr int B = 256;
constexpr long LDM = 16384;
constexpr int NTILE = 64;  // tile rows streamed per workgroup (and image pool tiles)

template <int IB>
struct Im {
  using G = Geo<B, IB>;
  static constexpr int V = G::VIMG, T = G::TPIMG, BUF = V + T;
};

template <int NW, int IB>
struct Dma {
  static constexpr int NIV = Im<IB>::V / 128, NIT = Im<IB>::T / 128;
  static constexpr int PV = (NIV + NW - 1) / NW, PT = (NIT + NW - 1) / NW;
  static constexpr int STEPS = PV + PT;
  double* dst;
  const double* v;
  const double* t;
  __device__ __forceinline__ void mid() const {}
  __device__ __forceinline__ void step(int m) const {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (m < PV) {
      const int u = min(w + NW * m, NIV - 1);
      dma16(v + u * 128 + 2 * lane, dst + u * 128);
    } else if (m < STEPS) {
      const int u = min(w + NW * (m - PV), NIT - 1);
      dma16(t + u * 128 + 2 * lane, dst + Im<IB>::V + u * 128);
    }
  }
  static __device__ __forceinline__ void dma16(const double* src, double* lds_wave) {
    const unsigned l = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) void*)lds_wave);
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off sc1" ::"v"(src), "{m0}"(l) : "memory");
  }
};

template <int STAUX>
struct Handover {  // the engine's XPipe: at(h) after row pair h's MFMAs, fin() after the loop
  static constexpr int NP = B / 8, LAG = 2;
  __amdgpu_buffer_rsrc_t out, in;
  unsigned base;
  __device__ __forceinline__ void st(int h, double (&X)[B / 4]) const {
    const unsigned long long a = (unsigned long long)__double_as_longlong(X[2 * h]);
    const unsigned long long b = (unsigned long long)__double_as_longlong(X[2 * h + 1]);
    __attribute__((ext_vector_type(4))) unsigned v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(v, out, base + 64 * h, 0, STAUX);
  }
  __device__ __forceinline__ void ld(int h, double (&X)[B / 4]) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(in, base + 64 * h, 0, 18);
    X[2 * h] = __longlong_as_double((long long)(((unsigned long long)v[1] << 32) | v[0]));
    X[2 * h + 1] = __longlong_as_double((long long)(((unsigned long long)v[3] << 32) | v[2]));
  }
  __device__ __forceinline__ void at(int h, double (&X)[B / 4]) const {
    if (h >= 1) st(h - 1, X);
    if (h >= 1 + LAG) ld(h - 1 - LAG, X);
  }
  __device__ __forceinline__ void fin(double (&X)[B / 4]) const {
    st(NP - 1, X);
#pragma unroll
    for (int h = NP - 1 - LAG; h < NP; ++h) ld(h, X);
  }
};
template <int STAUX>
__device__ __forceinline__ void store_strip_aux(const double (&X)[B / 4], double* tile) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = lane & 15;
  const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(tile);
  const unsigned base = (unsigned)(((size_t)c * LDM + 2 * x) * sizeof(double));
#pragma unroll
  for (int h = 0; h < B / 8; ++h) {
    const unsigned long long a = (unsigned long long)__double_as_longlong(X[2 * h]);
    const unsigned long long b = (unsigned long long)__double_as_longlong(X[2 * h + 1]);
    __attribute__((ext_vector_type(4))) unsigned v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, base, 64 * h, STAUX);
  }
}

template <int N>
__device__ __forceinline__ void sync_cnt() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int NW, int IB, int MODE, int WPC>
__global__ __launch_bounds__(64 * NW, WPC) void k_chain(double* X0, double* H0, const double* img, int nelem,
                                                          unsigned long long* clk) {
  using G = Geo<B, IB>;
  constexpr int NG = G::NG, NRI = G::NRI, NKS = G::NKS, SW = 16 * NW, BUF = Im<IB>::BUF;
  extern __shared__ __align__(16) double lds[];
  const int t = threadIdx.x, w = t >> 6;
  const size_t colo = (size_t)(blockIdx.x * SW + 16 * w) * LDM;  // this wave's first column
  double* const Xs = X0 + colo;
  const __amdgpu_buffer_rsrc_t hrs = head_rsrc(H0 + colo, true);
  const unsigned hoff = head_off_pair<B>(LDM, 0);
  auto vimg = [&](int i, int g) { return img + ((size_t)i * NG + g) * BUF; };
  double X[NKS], H[NRI], W[NRI];
  if (t == 0) clk[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  int buf = 0;
  {
    Dma<NW, IB> d{lds, vimg(0, 0), vimg(0, 0) + Im<IB>::V};
    for (int m = 0; m < Dma<NW, IB>::STEPS; ++m) d.step(m);
  }
  constexpr int STAUX = (MODE & 8) ? 0 : 16;
  constexpr bool XP = (MODE & 4) && !(MODE & 1);
  if ((MODE & 1) || (MODE & 48)) load_strip_pair<B, double>(X, Xs, LDM, 0);
  const int pre = (MODE & 32) ? (5 * blockIdx.x) % NG : (MODE & 16) && blockIdx.x >= gridDim.x / 2 ? NG / 2 : 0;
  if (pre > 0) {  // stagger / desync: groups without I/O first
    for (int g = 0; g < pre; ++g) {
      sync_cnt<0>();
      const double* Vs = lds + buf * BUF;
      Dma<NW, IB> d{lds + (buf ^ 1) * BUF, vimg(0, (g + 1) % NG), vimg(0, (g + 1) % NG) + Im<IB>::V};
      apply_zw<B, true, Dma<NW, IB>, true, true, true, IB>(Vs, Vs + Im<IB>::V, X, H, W, 0, d);
      apply_x4<B, NoPost, IB>(Vs, X, W);
      buf ^= 1;
    }
    sync_cnt<0>();
    Dma<NW, IB> d{lds + buf * BUF, vimg(0, 0), vimg(0, 0) + Im<IB>::V};
    for (int m = 0; m < Dma<NW, IB>::STEPS; ++m) d.step(m);
  }
  bool xin = false;
  for (int e = 0; e < nelem; ++e) {
    const int ti = e % NTILE;
    double* Xt = Xs + (size_t)ti * B;
    if (!(MODE & 2)) load_head_pair<B, 16, IB>(H, hrs, hoff);
    if (!(MODE & 1) && !xin) load_strip_pair<B, double>(X, Xt, LDM, 0);
    for (int g = 0; g < NG; ++g) {
      // the group's DMA (issued in the previous group's phase 1) and everything older complete; the
      // youngest operations (this element's strip / head loads, the previous group's head stores and
      // this group's head loads) may still be in flight
      constexpr int NX = ((MODE & 1) ? 0 : NKS / 2) + ((MODE & 2) ? 0 : NRI / 2), NH = (MODE & 2) ? 0 : NRI;
      if (g == 0) sync_cnt<NX>();
      else if (XP && xin && g == 1) sync_cnt<0>();  // (the streamed hand-over's stores drained)
      else sync_cnt<NH>();
      const double* Vs = lds + buf * BUF;
      const double* Ts = Vs + Im<IB>::V;
      const int gn = g + 1 < NG ? g + 1 : 0, in = g + 1 < NG ? ti : (ti + 1) % NTILE;
      Dma<NW, IB> d{lds + (buf ^ 1) * BUF, vimg(in, gn), vimg(in, gn) + Im<IB>::V};
      apply_zw<B, true, Dma<NW, IB>, true, true, true, IB>(Vs, Ts, X, H, W, 0, d);
      if (!(MODE & 2)) {
        store_head_pair<B, 0, IB>(H, hrs, hoff + g * IB * 8);
        if (g + 1 < NG) load_head_pair<B, 18, IB>(H, hrs, hoff + (g + 1) * IB * 8);
      }
      if (XP && g + 1 == NG && e + 1 < nelem) {
        const Handover<STAUX> hp{uniform_rsrc(Xt), uniform_rsrc(Xs + (size_t)((e + 1) % NTILE) * B),
                                 (unsigned)((((size_t)(t & 15)) * LDM + 2 * ((t & 63) >> 4)) * sizeof(double))};
        apply_x4<B, Handover<STAUX>, IB>(Vs, X, W, hp);
      } else {
        apply_x4<B, NoPost, IB>(Vs, X, W);
      }
      buf ^= 1;
    }
    xin = XP && e + 1 < nelem;
    if (!(MODE & 1) && !xin) store_strip_aux<STAUX>(X, Xt);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  if (MODE & 1) store_strip_pair<B, double>(X, Xs, LDM, 0);
  if (MODE & 2) store_head_pair<B, 0, IB>(H, hrs, hoff);
}

template <int NW, int IB, int MODE, int WPC>
static int run(const char* name, double* X, double* H, double* img, int ncu, int nelem, unsigned long long* clk) {
  constexpr int SW = 16 * NW;
  const int nwg = ncu * WPC;
  const size_t lds = 2 * Im<IB>::BUF * sizeof(double);
  auto k = k_chain<NW, IB, MODE, WPC>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(nwg), dim3(64 * NW), lds, 0, X, H, img, nelem, clk);
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  const double flops = 4.0 * B * B * (double)SW * nelem * nwg;
  printf("%-8s mode %d: %d WG x %d waves (%d per CU), %d-col strips, IB %d, LDS %zu KiB: %.3f ms, %.2f TF/s, "
         "%.1f us per element per WG\n",
         name, MODE, nwg, NW, WPC, SW, IB, lds / 1024, best, flops / best / 1e9, best * 1e3 / nelem);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return 0;
}

__global__ void k_fill(double* p, size_t n, double scale, unsigned long long seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned long long z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 31;
    p[i] = scale * (((double)(z % 2001) - 1000.0) / 1000.0);
  }
}

int main(int argc, char** argv) {
  const int nelem = argc > 1 ? atoi(argv[1]) : 96;
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  const size_t cols = (size_t)ncu * 128;  // both shapes: 128 columns per CU
  double *X, *H, *img;
  const size_t nx = cols * LDM, nimg = (size_t)NTILE * 16 * Im<16>::BUF + (size_t)NTILE * 8 * Im<32>::BUF;
  CK(hipMalloc(&X, nx * sizeof(double)));
  CK(hipMalloc(&H, nx * sizeof(double)));
  CK(hipMalloc(&img, nimg * sizeof(double)));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, X, nx, 0.5, 1ull);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, H, nx, 0.5, 2ull);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, img, nimg, 1e-3, 3ull);
  unsigned long long* clk;
  CK(hipMalloc(&clk, sizeof(unsigned long long) * 2 * 2 * ncu));
  CK(hipDeviceSynchronize());
  printf("%d CUs, %d elements per workgroup (tile rows streamed from HBM, ldm %ld)\n", ncu, nelem, LDM);
  if (argc > 2 && atoi(argv[2]) == 1) {  // one wave per SIMD: what the I/O costs there
    if (run<4, 32, 0, 1>("w4ib32", X, H, img, ncu, nelem, clk)) return 1;
    if (run<4, 32, 1, 1>("w4ib32", X, H, img, ncu, nelem, clk)) return 1;
    if (run<4, 32, 2, 1>("w4ib32", X, H, img, ncu, nelem, clk)) return 1;
    if (run<4, 32, 3, 1>("w4ib32", X, H, img, ncu, nelem, clk)) return 1;
    if (run<4, 32, 35, 1>("w4ib32", X, H, img, ncu, nelem, clk)) return 1;
    if (run<8, 32, 2, 1>("w8ib32", X, H, img, ncu, nelem, clk)) return 1;
    return 0;
  }
  if (run<8, 32, 0, 1>("w8ib32", X, H, img, ncu, nelem, clk)) return 1;
  if (run<8, 32, 32, 1>("w8ib32", X, H, img, ncu, nelem, clk)) return 1;
  if (run<8, 32, 40, 1>("w8ib32", X, H, img, ncu, nelem, clk)) return 1;
  if (run<8, 32, 33, 1>("w8ib32", X, H, img, ncu, nelem, clk)) return 1;
  if (run<8, 32, 35, 1>("w8ib32", X, H, img, ncu, nelem, clk)) return 1;
  if (run<4, 16, 0, 2>("w4ib16", X, H, img, ncu, nelem, clk)) return 1;
  if (run<4, 16, 32, 2>("w4ib16", X, H, img, ncu, nelem, clk)) return 1;
  if (run<4, 16, 40, 2>("w4ib16", X, H, img, ncu, nelem, clk)) return 1;
  if (run<4, 16, 33, 2>("w4ib16", X, H, img, ncu, nelem, clk)) return 1;
  if (run<4, 16, 35, 2>("w4ib16", X, H, img, ncu, nelem, clk)) return 1;
  return 0;
}
