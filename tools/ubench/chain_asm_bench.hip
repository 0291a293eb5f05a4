// Microbenchmark: the hand-scheduled fp64 chain (csrc/chain_asm.hpp, one asm statement per reflector
// group) in chain2_bench's setting: one 8-wave workgroup per CU, 128-column strips of 256-row tiles,
// 32-reflector groups, every workgroup streaming its own tile rows from HBM (ldm 16384) and the V/T
// images from a shared 64-tile pool, the element hand-over inside the last group. No engine
// dependencies (no polls, no counters). TF/s counts the algorithmic TSMQR flops (4 b^2 per column).
// MODE bits: 1 = strip I/O on empty resources (loads return 0, stores dropped: no HBM traffic for the
// strips), 2 = head rows on empty resources, 4 = one barrier-only group step per group (no body:
// the sync skeleton's own cost), 8 = per-group timestamps of every workgroup's wave 0 (after each
// group's barrier), printed as the average duration of each group position over elements 4..nelem-1,
// 16 = the hand-over's strip stores dropped (empty resource), 32 = its strip loads return 0 (empty
// resource), 64 = desync: every workgroup first runs (5 blockIdx) mod NG groups without strip I/O, so
// the hand-overs of the CUs are spread over the group positions as in the engine, 128 = the next strip
// loaded from a tile 33 rows of tiles away (not the row block right below the stored one), 256 = the
// hand-over loads only the next strip's first TQR_CHAIN_ASM_XLEAD_B* row pairs, the next element's
// first body the rest inside its phase 1 (TQR_CHAIN_ASM=2 in the engine).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I../../gpu-tiled-qr-decomposition_amd/csrc chain_asm_bench.hip -o chain_asm_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

#ifndef CAB_B
#define CAB_B 256
#endif
constexpr int B = CAB_B;  // tile size (build with -DCAB_B=128 for 128-row tiles)
static long LDM = 16384;  // leading dimension of the streamed matrix (argv[3])
constexpr int NTILE = 64;
using C = ShapeW8;
using G = FGeo<B, C>;
constexpr int BUF = G::VIMG + G::TPIMG;

template <int N>
__device__ __forceinline__ void bsync() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int MODE>
__global__ __launch_bounds__(512, 1) void k_asm(double* X0, double* H0, const double* img, int nelem,
                                                unsigned long long* clk, long ldm) {
  constexpr int NG = G::NG, NRI = G::NRI, VP = G::VP, IB = G::IB, NP = B / 8;
  extern __shared__ __align__(16) double lds[];
  const int t = threadIdx.x, lane = t & 63, x = lane >> 4, y = lane & 3;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const size_t colo = (size_t)(blockIdx.x * 128 + 16 * w) * ldm;
  double* const Xs = X0 + colo;
  const __amdgpu_buffer_rsrc_t hrs = (MODE & 2) ? null_rsrc(H0 + colo) : head_rsrc(H0 + colo, true);
  auto xr = [&](const double* p) { return (MODE & 1) ? null_rsrc(p) : uniform_rsrc(p); };
  auto vimg = [&](int i, int g) { return img + ((size_t)i * NG + g) * BUF; };
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) void*)lds);
  const unsigned oz = (unsigned)((x * VP + y * NRI) * 8), ox = (unsigned)((y * VP + x * NRI) * 8);
  const unsigned ot = (unsigned)(G::VIMG * 8 + (x * 4 + y) * NRI * 8);
  const unsigned loff = head_off_pair<B>(ldm, 0);
  const unsigned vl16 = 16u * lane;
  if (t == 0) clk[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  int buf = 0;
  ca_dma<B>(vimg(0, 0), vimg(0, 0) + G::VIMG, sreg(lds0), w, vl16);
  ca_load_strip_head<B>(xr(Xs), hrs, loff);
  if (MODE & 64) {  // desync: groups on the first element's images, no strip I/O
    const int pre = (5 * blockIdx.x) % NG;
    for (int g = 0; g < pre; ++g) {
      bsync<0>();
      const unsigned vb = lds0 + (unsigned)(buf * BUF * 8);
      CaGroup o;
      o.vz = vb + oz;
      o.vx = vb + ox;
      o.vt = vb + ot;
      o.vl16 = vl16;
      o.loff = loff;
      o.bpa = coal_bpa(lane);  // (used by GEN_COALESCE bodies only)
      o.loffc = coal_off(lane, ldm);
      o.hoff = __builtin_amdgcn_readfirstlane((int)(8 * ldm * 8));
      o.svsrc = vimg(0, 0);
      o.stsrc = vimg(0, 0) + G::VIMG;
      o.sdst = sreg(lds0 + (unsigned)((buf ^ 1) * BUF * 8));
      o.sw = w;
      o.hrs = hrs;
      o.hsc = (int)sreg(0u);
      o.goff = 0;
#ifdef TQR_CA_TS
      o.ts = nullptr;
#endif
      ca_group<B, 0>(o);
      buf = __builtin_amdgcn_readfirstlane(buf ^ 1);
    }
    bsync<0>();
  }
  bool xin = false;
  for (int e = 0; e < nelem; ++e) {
    const int ti = e % NTILE;
    const bool has_next = e + 1 < nelem;
    for (int g = 0; g < NG; ++g) {
      constexpr int NHO = 2 * NP + 8 < 63 ? 2 * NP + 8 : 63;
      constexpr int XL = B == 256 ? TQR_CHAIN_ASM_XLEAD_B256 : TQR_CHAIN_ASM_XLEAD_B128;
      constexpr int NHL = NP + XL + 8 < 63 ? NP + XL + 8 : 63;
      if (g == 0) {
        if (xin && (MODE & 256)) bsync<NHL>();
        else if (xin) bsync<NHO>();
        else bsync<NP + 4>();
      } else {
        bsync<4>();
      }
      if ((MODE & 8) && t == 0) clk[2 * gridDim.x + ((size_t)blockIdx.x * nelem + e) * NG + g] = __builtin_amdgcn_s_memrealtime();
      if (MODE & 4) {
        buf = __builtin_amdgcn_readfirstlane(buf ^ 1);
        continue;
      }
      const int gd = g + 1 < NG ? g + 1 : 0, id = g + 1 < NG ? ti : (ti + 1) % NTILE;
      const unsigned vb = lds0 + (unsigned)(buf * BUF * 8);
      CaGroup o;
      o.vz = vb + oz;
      o.vx = vb + ox;
      o.vt = vb + ot;
      o.vl16 = vl16;
      o.loff = loff;
      o.bpa = coal_bpa(lane);  // (used by GEN_COALESCE bodies only)
      o.loffc = coal_off(lane, ldm);
      o.hoff = __builtin_amdgcn_readfirstlane((int)(8 * ldm * 8));
      o.svsrc = vimg(id, gd);
      o.stsrc = vimg(id, gd) + G::VIMG;
      o.sdst = sreg(lds0 + (unsigned)((buf ^ 1) * BUF * 8));
      o.sw = w;
      o.hrs = hrs;
      o.hsc = (int)sreg(has_next ? 0u : 1u);
      o.goff = __builtin_amdgcn_readfirstlane(g * IB * 8);
#ifdef TQR_CA_TS
      o.ts = (MODE & 8) && t == 0 ? clk + 2 * gridDim.x + (size_t)gridDim.x * nelem * NG + ((size_t)blockIdx.x * nelem + e) * NG * 4 + g * 4 : nullptr;
#endif
      if (g + 1 < NG) {
        if ((MODE & 256) && g == 0 && xin) {
          o.xin = xr(Xs + (size_t)ti * B);
          ca_group<B, 3>(o);
        } else {
          ca_group<B, 0>(o);
        }
      } else {
        const double* xn = Xs + (size_t)((ti + ((MODE & 128) ? 33 : 1)) % NTILE) * B;
        o.xout = (MODE & 16) ? null_rsrc(Xs) : xr(Xs + (size_t)ti * B);
        o.xin = has_next && !(MODE & 32) ? xr(xn) : null_rsrc(xn);
        o.hnx = has_next ? hrs : null_rsrc(H0 + colo);
        if (MODE & 256) ca_group<B, 2>(o);
        else ca_group<B, 1>(o);
      }
      buf = __builtin_amdgcn_readfirstlane(buf ^ 1);
    }
    xin = has_next;
  }
  bsync<0>();
  if (t == 0) clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
}


// ---- one wave per SIMD prototype (TQR_CHAIN_ASM4_*: 4 waves, the strip in AGPRs) ----
__device__ __forceinline__ void ca4_group(const CaGroup& o, bool ho) {
  unsigned m0s, st;
#define TQR_CA4_INS                                                                                  \
  [vz] "v"(o.vz), [vx] "v"(o.vx), [vt] "v"(o.vt), [vl16] "v"(o.vl16), [loff] "v"(o.loff), [svsrc] "s"(o.svsrc), \
      [stsrc] "s"(o.stsrc), [sdst] "s"(o.sdst), [sw] "s"(o.sw), [hrs] "s"(o.hrs), [goff] "s"(o.goff),          \
      [hsc] "s"(o.hsc), [xout] "s"(o.xout), [xin] "s"(o.xin), [hnx] "s"(o.hnx)
  if (ho)
    asm volatile(TQR_CHAIN_ASM4_HANDOVER_B256 : [m0s] "=&s"(m0s), [st] "=&s"(st) : TQR_CA4_INS
                 : "memory", "scc", TQR_CHAIN_ASM4_CLOBBERS);
  else
    asm volatile(TQR_CHAIN_ASM4_PLAIN_B256 : [m0s] "=&s"(m0s), [st] "=&s"(st) : TQR_CA4_INS
                 : "memory", "scc", TQR_CHAIN_ASM4_CLOBBERS);
#undef TQR_CA4_INS
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void k_asm4(double* X0, double* H0, const double* img, int nelem,
                                                 unsigned long long* clk, long ldm) {
  static_assert(B == 256, "W4 prototype: 256-row tiles");
  constexpr int NG = G::NG, NRI = G::NRI, VP = G::VP, IB = G::IB, NP = B / 8;
  extern __shared__ __align__(16) double lds[];
  const int t = threadIdx.x, lane = t & 63, x = lane >> 4, y = lane & 3;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const size_t colo = (size_t)(blockIdx.x * 64 + 16 * w) * ldm;
  double* const Xs = X0 + colo;
  const __amdgpu_buffer_rsrc_t hrs = (MODE & 2) ? null_rsrc(H0 + colo) : head_rsrc(H0 + colo, true);
  auto xr = [&](const double* p) { return (MODE & 1) ? null_rsrc(p) : uniform_rsrc(p); };
  auto vimg = [&](int i, int g) { return img + ((size_t)i * NG + g) * BUF; };
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) void*)lds);
  const unsigned oz = (unsigned)((x * VP + y * NRI) * 8), ox = (unsigned)((y * VP + x * NRI) * 8);
  const unsigned ot = (unsigned)(G::VIMG * 8 + (x * 4 + y) * NRI * 8);
  const unsigned loff = head_off_pair<B>(ldm, 0);
  const unsigned vl16 = 16u * lane;
  if (t == 0) clk[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  int buf = 0;
  {
    unsigned m0s, st;
    asm volatile(TQR_CHAIN_ASM4_DMA_B256 : [m0s] "=&s"(m0s), [st] "=&s"(st)
                 : [svsrc] "s"(vimg(0, 0)), [stsrc] "s"(vimg(0, 0) + G::VIMG), [sdst] "s"(sreg(lds0)), [sw] "s"(w),
                   [vl16] "v"(vl16)
                 : "memory", "scc", TQR_CHAIN_ASM4_CLOBBERS);
    asm volatile("s_nop 4\n\t" TQR_CHAIN_ASM4_STRIP_LOAD_B256 "\n\t" TQR_CHAIN_ASM_HEAD_LOAD
                 :: [loff] "v"(loff), [xin] "s"(xr(Xs)), [hrs] "s"(hrs) : "memory", TQR_CHAIN_ASM4_CLOBBERS);
  }
  bool xin = false;
  for (int e = 0; e < nelem; ++e) {
    const int ti = e % NTILE;
    const bool has_next = e + 1 < nelem;
    for (int g = 0; g < NG; ++g) {
      constexpr int NHO = 2 * NP + 8 < 63 ? 2 * NP + 8 : 63;
      if (g == 0) {
        if (xin) bsync<NHO>();
        else bsync<NP + 4>();
      } else {
        bsync<4>();
      }
      if ((MODE & 8) && t == 0) clk[2 * gridDim.x + ((size_t)blockIdx.x * nelem + e) * NG + g] = __builtin_amdgcn_s_memrealtime();
      const int gd = g + 1 < NG ? g + 1 : 0, id = g + 1 < NG ? ti : (ti + 1) % NTILE;
      const unsigned vb = lds0 + (unsigned)(buf * BUF * 8);
      CaGroup o;
      o.vz = vb + oz;
      o.vx = vb + ox;
      o.vt = vb + ot;
      o.vl16 = vl16;
      o.loff = loff;
      o.bpa = coal_bpa(lane);  // (used by GEN_COALESCE bodies only)
      o.loffc = coal_off(lane, ldm);
      o.hoff = __builtin_amdgcn_readfirstlane((int)(8 * ldm * 8));
      o.svsrc = vimg(id, gd);
      o.stsrc = vimg(id, gd) + G::VIMG;
      o.sdst = sreg(lds0 + (unsigned)((buf ^ 1) * BUF * 8));
      o.sw = w;
      o.hrs = hrs;
      o.hsc = (int)sreg(has_next ? 0u : 1u);
      o.goff = __builtin_amdgcn_readfirstlane(g * IB * 8);
      const double* xn = Xs + (size_t)((ti + 1) % NTILE) * B;
      o.xout = xr(Xs + (size_t)ti * B);
      o.xin = has_next ? xr(xn) : null_rsrc(xn);
      o.hnx = has_next ? hrs : null_rsrc(H0 + colo);
      ca4_group(o, g + 1 == NG);
      buf = __builtin_amdgcn_readfirstlane(buf ^ 1);
    }
    xin = has_next;
  }
  bsync<0>();
  if (t == 0) clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
}

template <int MODE>
static int run4(double* X, double* H, double* img, int ncu, int nelem, unsigned long long* clk) {
  const size_t lds = flow_lds_doubles<B, double, C>() * 8 + 1536;
  auto k = k_asm4<MODE>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(ncu), dim3(256), lds, 0, X, H, img, nelem, clk, LDM);
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  const double flops = 4.0 * B * B * 64.0 * nelem * ncu;
  if (MODE & 8) {
    constexpr int NG = G::NG;
    const size_t n = (size_t)ncu * nelem * NG;
    unsigned long long* h = (unsigned long long*)malloc(n * 8);
    CK(hipMemcpy(h, clk + 2 * ncu, n * 8, hipMemcpyDeviceToHost));
    double sum[NG] = {0};
    int cnt = 0;
    for (int b = 0; b < ncu; ++b)
      for (int e = 4; e + 1 < nelem; ++e, ++cnt)
        for (int g = 0; g < NG; ++g) {
          const size_t i0 = ((size_t)b * nelem + e) * NG + g;
          sum[g] += (double)(h[i0 + 1] - h[i0]) * 10.0 / 1000.0;
        }
    printf("   per group position (us, barrier to barrier):");
    for (int g = 0; g < NG; ++g) printf(" %.2f", sum[g] / cnt);
    printf("\n");
    free(h);
  }
  printf("asm w4 (AGPR strip) mode %d: %d WG: %.3f ms, %.2f TF/s, %.2f us per element per WG\n", MODE, ncu, best,
         flops / best / 1e9, best * 1e3 / nelem);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return 0;
}

template <int MODE>
static int run(double* X, double* H, double* img, int ncu, int nelem, unsigned long long* clk) {
  const size_t lds = flow_lds_doubles<B, double, C>() * 8 + 1536;
  auto k = k_asm<MODE>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(ncu), dim3(512), lds, 0, X, H, img, nelem, clk, LDM);
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  const double flops = 4.0 * B * B * 128.0 * nelem * ncu;
  if (MODE & 8) {  // average duration of each group position (100 MHz realtime clock)
    constexpr int NG = G::NG;
    const size_t n = (size_t)ncu * nelem * NG;
    unsigned long long* h = (unsigned long long*)malloc(n * 8);
    CK(hipMemcpy(h, clk + 2 * ncu, n * 8, hipMemcpyDeviceToHost));
    double sum[NG] = {0};
    int cnt = 0;
    for (int b = 0; b < ncu; ++b)
      for (int e = 4; e + 1 < nelem; ++e, ++cnt)
        for (int g = 0; g < NG; ++g) {
          const size_t i0 = ((size_t)b * nelem + e) * NG + g;
          sum[g] += (double)(h[i0 + 1] - h[i0]) * 10.0 / 1000.0;  // us
        }
    printf("   per group position (us, barrier to barrier):");
    for (int g = 0; g < NG; ++g) printf(" %.2f", sum[g] / cnt);
    printf("\n");
#ifdef TQR_CA_TS
    {  // inside the statement: start -> P1 end -> P2 start -> P2 end -> next barrier
      unsigned long long* q = (unsigned long long*)malloc(n * 4 * 8);
      CK(hipMemcpy(q, clk + 2 * ncu + n, n * 4 * 8, hipMemcpyDeviceToHost));
      for (int g = 0; g < NG; ++g) {
        double ph[5] = {0};
        for (int b = 0; b < ncu; ++b)
          for (int e = 4; e + 1 < nelem; ++e) {
            const size_t i0 = ((size_t)b * nelem + e) * NG + g;
            const unsigned long long* z = q + i0 * 4;
            ph[0] += (double)(z[0] - h[i0]) * 0.01;
            ph[1] += (double)(z[1] - z[0]) * 0.01;
            ph[2] += (double)(z[2] - z[1]) * 0.01;
            ph[3] += (double)(z[3] - z[2]) * 0.01;
            ph[4] += (double)(h[i0 + 1] - z[3]) * 0.01;
          }
        printf("   group %d: sync->body %.2f  P1 %.2f  T %.2f  P2 %.2f  tail+sync %.2f us\n", g, ph[0] / cnt, ph[1] / cnt,
               ph[2] / cnt, ph[3] / cnt, ph[4] / cnt);
      }
      free(q);
    }
#endif
    free(h);
  }
  printf("asm w8ib32 mode %d: %d WG: %.3f ms, %.2f TF/s, %.2f us per element per WG\n", MODE, ncu, best,
         flops / best / 1e9, best * 1e3 / nelem);
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
  if (argc > 3) LDM = atol(argv[3]);
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  const size_t cols = (size_t)ncu * 128;
  double *X, *H, *img;
  const size_t nx = cols * LDM, nimg = (size_t)NTILE * G::NG * BUF;
  CK(hipMalloc(&X, nx * sizeof(double)));
  CK(hipMalloc(&H, nx * sizeof(double)));
  CK(hipMalloc(&img, nimg * sizeof(double)));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, X, nx, 0.5, 1ull);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, H, nx, 0.5, 2ull);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, img, nimg, 1e-3, 3ull);
  unsigned long long* clk;
  CK(hipMalloc(&clk, sizeof(unsigned long long) * (2 * ncu + (size_t)ncu * nelem * G::NG * 5)));
  CK(hipDeviceSynchronize());
  printf("%d CUs, %d elements per workgroup (tile rows streamed from HBM, ldm %ld)\n", ncu, nelem, LDM);
  const int sel = argc > 2 ? atoi(argv[2]) : 0;
  if (sel == 4) {  // the one-wave-per-SIMD prototype beside the 8-wave form
    if (run4<0>(X, H, img, ncu, nelem, clk)) return 1;
    if (run4<1>(X, H, img, ncu, nelem, clk)) return 1;
    if (run4<2>(X, H, img, ncu, nelem, clk)) return 1;
    if (run4<3>(X, H, img, ncu, nelem, clk)) return 1;
    if (run4<8>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<3>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<8>(X, H, img, ncu, nelem, clk)) return 1;
    return 0;
  }
  if (sel == 0) {
    if (run<0>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<1>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<2>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<3>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<4>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<8>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<10>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<24>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<40>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<64>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<72>(X, H, img, ncu, nelem, clk)) return 1;
  } else if (sel == 6) {  // round 6: the late-load hand-over decomposed (stores dropped / loads zero / no strip
                          // I/O), in lockstep and with the workgroups' hand-overs spread (desync)
    if (run<264>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<264 + 16>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<264 + 32>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<264 + 1>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<264 + 64>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<264 + 64 + 16>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<264 + 64 + 32>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<264 + 64 + 1>(X, H, img, ncu, nelem, clk)) return 1;
  } else if (sel == 2) {  // late strip loads vs the whole strip in the hand-over
    if (run<8>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<264>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<8>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<264>(X, H, img, ncu, nelem, clk)) return 1;
  } else {  // the hand-over variants only
    if (run<8>(X, H, img, ncu, nelem, clk)) return 1;
    if (run<136>(X, H, img, ncu, nelem, clk)) return 1;
  }
  return 0;
}
