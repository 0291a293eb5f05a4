// One reflector group of the fp64 chain, hand-scheduled (csrc/chain_asm.hpp, generated body) against
// the compiler-scheduled device functions (tiles.hpp apply_zw + apply_x4), on the same LDS images,
// strip and head rows (random data): max |difference| of the updated strip and head rows.
// Build: hipcc --offload-arch=gfx950 -O3 -I../../include -I../../gpu-tiled-qr-decomposition_amd/csrc chain_asm_check.hip -o chain_asm_check
#include <hip/hip_runtime.h>

#include <cmath>
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

constexpr long LDM = 1024;

template <int B>
struct Im {
  using G = Geo<B, 32>;
  static constexpr int V = G::VIMG, T = G::TPIMG, BUF = V + T;
};

// mode 0: asm body (plain), 1: C++ reference, 2: asm hand-over body (next strip from Xn, next head from H)
template <int B, int MODE>
__global__ __launch_bounds__(512, 1) void k_group(const double* img, double* X, double* H, double* Xn, double* Xo,
                                                 double* Ho) {
  extern __shared__ __align__(16) double lds[];
  constexpr int BUF = Im<B>::BUF;
  for (int i = threadIdx.x; i < BUF; i += 512) lds[i] = img[i];
  __syncthreads();
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, x = lane >> 4, y = lane & 3;
  const size_t colo = (size_t)(16 * w) * LDM;
  const unsigned loff = head_off_pair<B>(LDM, 0);
  using G = Geo<B, 32>;
  constexpr int NRI = G::NRI, VP = G::VP;
  if constexpr (MODE == 1) {
    double Xr[G::NKS], Hr[NRI], W[NRI];
    load_strip_pair<B, double>(Xr, X + colo, LDM, 0);
    load_head_pair<B, 16, 32>(Hr, head_rsrc(H + colo, true), loff);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    apply_zw<B, true, NoHook, true, true, true, 32>(lds, lds + G::VIMG, Xr, Hr, W, 0);
    apply_x4<B, NoPost, 32>(lds, Xr, W);
    store_strip_pair<B, double>(Xr, Xo + colo, LDM, 0);
    store_head_pair<B, 16, 32>(Hr, head_rsrc(Ho + colo, true), loff);
  } else {
    const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)lds;
    ca_load_strip_head<B>(uniform_rsrc(X + colo), head_rsrc(H + colo, true), loff);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    CaGroup o;
    o.vz = lds0 + (unsigned)((x * VP + y * NRI) * 8);
    o.vx = lds0 + (unsigned)((y * VP + x * NRI) * 8);
    o.vt = lds0 + (unsigned)(G::VIMG * 8 + (x * 4 + y) * NRI * 8);
    o.vl16 = 16u * lane;
    o.loff = loff;
    o.svsrc = uni(img);
    o.stsrc = uni(img + G::VIMG);
    o.sdst = sreg(lds0 + BUF * 8);
    o.sw = __builtin_amdgcn_readfirstlane(w);
    o.hrs = head_rsrc(Ho + colo, true);  // the group's head rows stored here (loads of the next group: unused)
    o.goff = 0;
    o.hsc = (int)sreg(1u);
    if constexpr (MODE == 0) {
      ca_group<B, 0>(o);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // the updated strip
      if constexpr (B == 256)
        asm volatile(TQR_CHAIN_ASM_STRIP_STORE_B256 ::[loff] "v"(loff), [xout] "s"(uniform_rsrc(Xo + colo)) : "memory");
      else
        asm volatile(TQR_CHAIN_ASM_STRIP_STORE_B128 ::[loff] "v"(loff), [xout] "s"(uniform_rsrc(Xo + colo)) : "memory");
    } else {
      o.xout = uniform_rsrc(Xo + colo);
      o.xin = uniform_rsrc(Xn + colo);
      o.hnx = head_rsrc(H + colo, true);
      ca_group<B, 1>(o);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // the next strip and head rows as loaded by the hand-over: stored behind the updated ones
      if constexpr (B == 256)
        asm volatile(TQR_CHAIN_ASM_STRIP_STORE_B256 ::[loff] "v"(loff), [xout] "s"(uniform_rsrc(Xo + colo + (size_t)B)) : "memory");
      else
        asm volatile(TQR_CHAIN_ASM_STRIP_STORE_B128 ::[loff] "v"(loff), [xout] "s"(uniform_rsrc(Xo + colo + (size_t)B)) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// A whole element (NG groups): images of group g at img + g * BUF, LDS-DMA'd group by group into
// alternating buffers (the engine's pattern); head rows group by group from H. MODE 3: asm, 4: C++.
template <int B, int MODE>
__global__ __launch_bounds__(512, 1) void k_elem(const double* img, double* X, double* H, double* Xo, int ngu, int var) {
  extern __shared__ __align__(16) double lds[];
  using G = Geo<B, 32>;
  constexpr int BUF = Im<B>::BUF, NG = G::NG, NRI = G::NRI, VP = G::VP;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, x = lane >> 4, y = lane & 3;
  const size_t colo = (size_t)(16 * w) * LDM;
  const unsigned loff = head_off_pair<B>(LDM, 0);
  if constexpr (MODE == 4) {
    double Xr[G::NKS], Hr[NRI], W[NRI];
    load_strip_pair<B, double>(Xr, X + colo, LDM, 0);
    for (int g = 0; g < ngu; ++g) {
      __syncthreads();
      for (int i = threadIdx.x; i < BUF; i += 512) lds[i] = img[(size_t)((var & 1) ? 0 : g) * BUF + i];
      __syncthreads();
      load_head_pair<B, 16, 32>(Hr, head_rsrc(H + colo, true), loff + g * 256);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      apply_zw<B, true, NoHook, true, true, true, 32>(lds, lds + G::VIMG, Xr, Hr, W, 0);
      apply_x4<B, NoPost, 32>(lds, Xr, W);
      store_head_pair<B, 16, 32>(Hr, head_rsrc(H + colo, true), loff + g * 256);
    }
    store_strip_pair<B, double>(Xr, Xo + colo, LDM, 0);
  } else {
    const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)lds;
    const unsigned vl16 = 16u * lane;
    const int ws = __builtin_amdgcn_readfirstlane(w);
    ca_dma<B>(uni(img), uni(img + G::VIMG), sreg(lds0), ws, vl16);
    ca_load_strip_head<B>(uniform_rsrc(X + colo), head_rsrc(H + colo, true), loff);
    int par = 0;
    int* sflag = (int*)(lds + 2 * BUF);
    for (int g = 0; g < ngu; ++g) {
      const int buf = g & 1;
      if (g == 0) ca_sync<B / 8 + 4>(true, w == 7, sflag, par);
      else ca_sync<4>(true, w == 7, sflag, par);
      const unsigned vb = lds0 + (unsigned)(buf * BUF * 8);
      const int gn = (var & 1) ? 0 : g + 1 < ngu ? g + 1 : g;
      CaGroup o;
      o.vz = vb + (unsigned)((x * VP + y * NRI) * 8);
      o.vx = vb + (unsigned)((y * VP + x * NRI) * 8);
      o.vt = vb + (unsigned)(G::VIMG * 8 + (x * 4 + y) * NRI * 8);
      o.vl16 = vl16;
      o.loff = loff;
      o.svsrc = uni(img + (size_t)gn * BUF);
      o.stsrc = uni(img + (size_t)gn * BUF + G::VIMG);
      o.sdst = sreg(lds0 + (unsigned)((buf ^ 1) * BUF * 8));
      o.sw = ws;
      o.hrs = head_rsrc(H + colo, true);
      o.goff = __builtin_amdgcn_readfirstlane(g * 256);
      o.hsc = (int)sreg(1u);
      if (g + 1 < ngu || (var & 2)) {
        ca_group<B, 0>(o);
        if (g + 1 == ngu) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if constexpr (B == 256)
            asm volatile(TQR_CHAIN_ASM_STRIP_STORE_B256 ::[loff] "v"(loff), [xout] "s"(uniform_rsrc(Xo + colo)) : "memory");
          else
            asm volatile(TQR_CHAIN_ASM_STRIP_STORE_B128 ::[loff] "v"(loff), [xout] "s"(uniform_rsrc(Xo + colo)) : "memory");
        }
      } else {
        o.xout = uniform_rsrc(Xo + colo);
        o.xin = null_rsrc(X);
        o.hnx = null_rsrc(X);
        ca_group<B, 1>(o);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// the LDS-DMA statement alone: group images into LDS buffer `buf`, copied back out
template <int B>
__global__ __launch_bounds__(512, 1) void k_dma(const double* img, double* out, int buf) {
  extern __shared__ __align__(16) double lds[];
  constexpr int BUF = Im<B>::BUF;
  for (int i = threadIdx.x; i < 2 * BUF; i += 512) lds[i] = -1.0;
  __syncthreads();
  const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)lds;
  const int ws = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  ca_dma<B>(uni(img), uni(img + Im<B>::V), sreg(lds0 + (unsigned)(buf * BUF * 8)), ws, 16u * (threadIdx.x & 63));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * BUF; i += 512) out[i] = lds[i];
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
static int check() {
  constexpr int BUF = Im<B>::BUF;
  const size_t nx = (size_t)128 * LDM;
  double *img, *X, *H, *Xn, *Xo0, *Ho0, *Xo1, *Ho1, *Xo2;
  CK(hipMalloc(&img, BUF * sizeof(double)));
  for (double** p : {&X, &H, &Xn, &Xo0, &Ho0, &Xo1, &Ho1, &Xo2}) CK(hipMalloc(p, nx * sizeof(double)));
  hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, img, (size_t)BUF, 0.05, 3ull);
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, X, nx, 1.0, 1ull);
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, H, nx, 1.0, 2ull);
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, Xn, nx, 1.0, 7ull);
  for (double* p : {Xo0, Ho0, Xo1, Ho1, Xo2}) CK(hipMemset(p, 0, nx * sizeof(double)));
  const size_t lds = 2 * BUF * sizeof(double);
  CK(hipFuncSetAttribute((const void*)k_group<B, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)k_group<B, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)k_group<B, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL((k_group<B, 0>), dim3(1), dim3(512), lds, 0, img, X, H, Xn, Xo0, Ho0);
  hipLaunchKernelGGL((k_group<B, 1>), dim3(1), dim3(512), lds, 0, img, X, H, Xn, Xo1, Ho1);
  hipLaunchKernelGGL((k_group<B, 2>), dim3(1), dim3(512), lds, 0, img, X, H, Xn, Xo2, Ho0);
  CK(hipDeviceSynchronize());
  std::vector<double> a(nx), b(nx), c(nx), ha(nx), hb(nx), xn(nx), hh(nx);
  CK(hipMemcpy(a.data(), Xo0, nx * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), Xo1, nx * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(c.data(), Xo2, nx * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ha.data(), Ho0, nx * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb.data(), Ho1, nx * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(xn.data(), Xn, nx * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hh.data(), H, nx * 8, hipMemcpyDeviceToHost));
  double dx = 0, dh = 0, dxh = 0, dnx = 0, mx = 0;
  int nnan = 0, first = -1;
  for (int col = 0; col < 128; ++col)
    for (int r = 0; r < B; ++r) {
      const size_t e = (size_t)col * LDM + r;
      if (!std::isfinite(a[e])) {
        ++nnan;
        if (first < 0) first = (int)e;
      }
      dx = fmax(dx, fabs(a[e] - b[e]));
      dxh = fmax(dxh, fabs(c[e] - b[e]));
      dnx = fmax(dnx, fabs(c[e + B] - xn[e]));
      mx = fmax(mx, fabs(b[e]));
    }
  for (int col = 0; col < 128; ++col)
    for (int r = 0; r < 32; ++r) {
      const size_t e = (size_t)col * LDM + r;
      dh = fmax(dh, fabs(ha[e] - hb[e]));
    }
  printf("B=%d: strip max|asm-C++| %.3e (max|X| %.3e, %d non-finite, first at col %d row %d), head %.3e; "
         "hand-over body: strip %.3e, next strip loaded %.3e\n",
         B, dx, mx, nnan, first < 0 ? -1 : first / (int)LDM, first < 0 ? -1 : first % (int)LDM, dh, dxh, dnx);
  if (first >= 0) {
    for (int r = 0; r < 8; ++r) printf("  row %d: asm %.6e c++ %.6e\n", r, a[r], b[r]);
  }
  return 0;
}

template <int B>
static int check_elem() {
  using G = Geo<B, 32>;
  constexpr int BUF = Im<B>::BUF, NG = G::NG;
  const size_t nx = (size_t)128 * LDM;
  double *img, *X, *H0, *H1, *Xo0, *Xo1;
  CK(hipMalloc(&img, (size_t)NG * BUF * sizeof(double)));
  for (double** p : {&X, &H0, &H1, &Xo0, &Xo1}) CK(hipMalloc(p, nx * sizeof(double)));
  hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, img, (size_t)NG * BUF, 0.05, 3ull);
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, X, nx, 1.0, 1ull);
  double* Hs;
  CK(hipMalloc(&Hs, nx * sizeof(double)));
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, Hs, nx, 1.0, 2ull);
  const size_t lds = 2 * BUF * sizeof(double) + 1024;
  CK(hipFuncSetAttribute((const void*)k_elem<B, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  CK(hipFuncSetAttribute((const void*)k_elem<B, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  for (int var = 0; var < 4; ++var)
  for (int ngu = 1; ngu <= 3; ++ngu) {
  CK(hipMemcpy(H0, Hs, nx * 8, hipMemcpyDeviceToDevice));
  CK(hipMemcpy(H1, Hs, nx * 8, hipMemcpyDeviceToDevice));
  CK(hipMemset(Xo0, 0, nx * 8));
  CK(hipMemset(Xo1, 0, nx * 8));
  hipLaunchKernelGGL((k_elem<B, 3>), dim3(1), dim3(512), lds, 0, img, X, H0, Xo0, ngu, var);
  hipLaunchKernelGGL((k_elem<B, 4>), dim3(1), dim3(512), lds, 0, img, X, H1, Xo1, ngu, var);
  CK(hipDeviceSynchronize());
  std::vector<double> a(nx), b(nx), ha(nx), hb(nx);
  {
  CK(hipMemcpy(a.data(), Xo0, nx * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), Xo1, nx * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ha.data(), H0, nx * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb.data(), H1, nx * 8, hipMemcpyDeviceToHost));
  double dx = 0, dh = 0;
  int nnan = 0;
  for (int col = 0; col < 128; ++col)
    for (int r = 0; r < B; ++r) {
      const size_t e = (size_t)col * LDM + r;
      nnan += !std::isfinite(a[e]);
      dx = fmax(dx, fabs(a[e] - b[e]));
      dh = fmax(dh, fabs(ha[e] - hb[e]));
    }
  printf("element B=%d var %d (%d of %d groups, LDS-DMA): strip max|asm-C++| %.3e (%d non-finite), head rows %.3e\n", B, var, ngu, NG, dx, nnan, dh);
  }
  }
  return 0;
}

template <int B>
static int check_dma() {
  constexpr int BUF = Im<B>::BUF;
  double *img, *out;
  CK(hipMalloc(&img, BUF * sizeof(double)));
  CK(hipMalloc(&out, 2 * BUF * sizeof(double)));
  hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, img, (size_t)BUF, 0.05, 3ull);
  const size_t lds = 2 * BUF * sizeof(double);
  CK(hipFuncSetAttribute((const void*)k_dma<B>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  std::vector<double> hi(BUF), ho(2 * BUF);
  CK(hipMemcpy(hi.data(), img, BUF * 8, hipMemcpyDeviceToHost));
  for (int buf = 0; buf < 2; ++buf) {
    hipLaunchKernelGGL(k_dma<B>, dim3(1), dim3(512), lds, 0, img, out, buf);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ho.data(), out, 2 * BUF * 8, hipMemcpyDeviceToHost));
    int bad = 0, first = -1, untouched = 0;
    for (int i = 0; i < BUF; ++i) {
      if (ho[buf * BUF + i] != hi[i]) {
        ++bad;
        if (first < 0) first = i;
      }
      untouched += ho[(buf ^ 1) * BUF + i] == -1.0;
    }
    printf("dma B=%d buf %d: %d of %d doubles wrong (first %d: %.4e vs %.4e), other buffer untouched %d\n", B, buf, bad, BUF,
           first, first >= 0 ? ho[buf * BUF + first] : 0.0, first >= 0 ? hi[first] : 0.0, untouched);
  }
  return 0;
}

int main() {

  if (check_elem<128>()) return 1;
  if (check_elem<256>()) return 1;
  return 0;
}
