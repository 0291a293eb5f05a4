// Microbenchmark: the chain's element hand-over (flow.hpp XPipe) in isolation. One 512-thread
// workgroup per CU (8 waves, as k_flow); each iteration is one reflector group on a 256 x 16 strip
// per wave with V/T resident in LDS (phase 1 apply_zw, phase 2 apply_x4, one barrier), and every
// 8th group (staggered across CUs, as elements end at different times on the chip) streams the
// finished strip out and the next one in during phase 2, as the real last group of an element.
// Variants (MODE): 0 no hand-over; 1 XPipe (stores + loads interleaved); 2 stores only; 3 loads
// only; 4 stores interleaved, loads all after the last store; 5 as 1 with plain (non sc1)
// stores; 6 as 1 with sc1 loads (no nt); 7 as 1 without the phase priority flips.
// Reports the median duration of ordinary and of hand-over groups (workgroup 0..N, wave 0).
// Build: hipcc --offload-arch=gfx950 -O3 -I../../include -I../../gpu-tiled-qr-decomposition_amd/csrc handover_bench.hip -o handover_bench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
#include "tiles.hpp"
#include "gridscheduler.h"
namespace tqr { struct Item { int ts, l, m, k; }; }
#include "flow.hpp"
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
using namespace tqr;
constexpr int B = 256;
using G = Geo<B>;

template <int STAUX, int LDAUX>
struct XP {
  static constexpr int NP = G::NKS / 2;
  __amdgpu_buffer_rsrc_t out, in;
  unsigned base;
  bool do_st, do_ld, late;
  __device__ __forceinline__ void st(int h, double (&X)[G::NKS]) const {
    if (do_st) st_pair<double, STAUX>(out, base + 8 * h * sizeof(double), X[2 * h], X[2 * h + 1]);
  }
  __device__ __forceinline__ void ld(int h, double (&X)[G::NKS]) const {
    if (do_ld) ld_pair<double, LDAUX>(in, base + 8 * h * sizeof(double), X[2 * h], X[2 * h + 1]);
  }
  __device__ __forceinline__ void at(int h, double (&X)[G::NKS]) const {
    if (h >= 1) st(h - 1, X);
    if (!late && h >= 3) ld(h - 3, X);
  }
  __device__ __forceinline__ void fin(double (&X)[G::NKS]) const {
    st(NP - 1, X);
    if (late) {
#pragma unroll
      for (int h = 0; h < NP; ++h) ld(h, X);
    } else {
#pragma unroll
      for (int h = NP - 3; h < NP; ++h) ld(h, X);
    }
  }
};

template <int MODE>
__global__ __launch_bounds__(512, 1) void k_hand(double* mat, long ldm, unsigned long long* tim, int iters) {
  extern __shared__ __align__(16) double lds[];
  double* Vs = lds;
  double* Ts = Vs + G::VIMG;
  for (int i = threadIdx.x; i < G::VIMG + G::TPIMG; i += 512) lds[i] = 1e-3 * ((i * 37) % 101 - 50) / 50.0;
  __syncthreads();
  const int w = threadIdx.x >> 6, t = threadIdx.x;
  double X[G::NKS], H[G::NRI], W[G::NRI];
  for (int k = 0; k < G::NKS; ++k) X[k] = 1.0 + 1e-3 * (threadIdx.x + k);
  for (int r = 0; r < G::NRI; ++r) H[r] = 0.5 + 1e-3 * r;
  // this CU's strip: 128 columns (blockIdx % 128), tile rows advance by one per element
  const int cb = blockIdx.x % 128;
  constexpr int STAUX = MODE == 5 ? 0 : 16;
  constexpr int LDAUX = MODE == 6 ? 16 : 18;
  unsigned long long* mine = tim + (size_t)blockIdx.x * iters;
  int tile = blockIdx.x / 128;
  for (int it = 0; it < iters; ++it) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    asm volatile("" ::: "memory");
    if (MODE != 7) phase_prio(false);
    apply_zw<B, true, NoHook, true, true, true>(Vs, Ts, X, H, W, 0);
    if (MODE != 7) phase_prio(true);
    const bool hand = MODE != 0 && ((it + blockIdx.x) & 7) == 7;
    if (hand) {
      double* Xt = mat + (size_t)(cb * 128 + 16 * w) * ldm + (size_t)(tile % 64) * B;
      double* Xn = mat + (size_t)(cb * 128 + 16 * w) * ldm + (size_t)((tile + 1) % 64) * B;
      const XP<STAUX, LDAUX> xp{uniform_rsrc(Xt), uniform_rsrc(Xn),
                                (unsigned)((((size_t)(t & 15)) * ldm + 2 * ((t & 63) >> 4)) * sizeof(double)),
                                MODE != 3, MODE != 2, MODE == 4};
      apply_x4<B, XP<STAUX, LDAUX>>(Vs, X, W, xp);
      ++tile;
    } else {
      apply_x4<B>(Vs, X, W);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (threadIdx.x == 0) mine[it] = (__builtin_amdgcn_s_memrealtime() - t0) | ((unsigned long long)hand << 63);
  }
  double s = 0;
  for (int k = 0; k < G::NKS; ++k) s += X[k];
  if (s == 12345.678) mat[threadIdx.x] = s;
}

template <int MODE>
static int run(const char* name, double* mat, long ldm, unsigned long long* tim, int nb, int iters) {
  const size_t lds = (G::VIMG + G::TPIMG) * sizeof(double);
  CK(hipFuncSetAttribute((const void*)k_hand<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  k_hand<MODE><<<nb, 512, lds>>>(mat, ldm, tim, iters);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> h((size_t)nb * iters);
  CK(hipMemcpy(h.data(), tim, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> norm, hand;
  for (int b = 0; b < nb; ++b)
    for (int i = 8; i < iters; ++i) {
      const unsigned long long v = h[(size_t)b * iters + i];
      ((v >> 63) ? hand : norm).push_back((double)(v & ~(1ull << 63)) / 100.0);
    }
  auto med = [](std::vector<double>& v) { if (v.empty()) return 0.0; std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  double sn = 0, sh = 0;
  for (double x : norm) sn += x;
  for (double x : hand) sh += x;
  printf("%-44s ordinary group median %6.2f us (mean %6.2f), hand-over median %6.2f us (mean %6.2f)\n", name, med(norm),
         norm.empty() ? 0 : sn / norm.size(), med(hand), hand.empty() ? 0 : sh / hand.size());
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int nb = p.multiProcessorCount, iters = 400;
  const long ldm = 16384;
  double* mat;
  CK(hipMalloc(&mat, (size_t)ldm * 16384 * sizeof(double)));
  CK(hipMemset(mat, 0, (size_t)ldm * 16384 * sizeof(double)));
  unsigned long long* tim;
  CK(hipMalloc(&tim, (size_t)nb * iters * 8));
  run<0>("0 no hand-over", mat, ldm, tim, nb, iters);
  run<1>("1 XPipe (stores sc1 + loads sc1|nt)", mat, ldm, tim, nb, iters);
  run<2>("2 stores only", mat, ldm, tim, nb, iters);
  run<3>("3 loads only", mat, ldm, tim, nb, iters);
  run<4>("4 stores, then all loads after the last", mat, ldm, tim, nb, iters);
  run<5>("5 XPipe, plain stores", mat, ldm, tim, nb, iters);
  run<6>("6 XPipe, sc1 loads (no nt)", mat, ldm, tim, nb, iters);
  run<7>("7 XPipe, no priority flips", mat, ldm, tim, nb, iters);
  run<1>("1 XPipe (again)", mat, ldm, tim, nb, iters);
  return 0;
}
