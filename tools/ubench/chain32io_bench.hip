// Microbenchmark: the fp32 chain's element loop WITH its traffic (strips streamed from HBM, the next
// group's V/T images LDS-DMA'd inside phase 1, counted waits at every group's sync point, as the
// engine), in two designs (128 columns per CU, head strip resident, 256-row tiles, 32-reflector
// groups):
//   w8  the engine's: 8 waves × one 16-column tile; the finished strip stored and the next one
//       loaded tile by tile inside the last group's phase 2 (XPipe32) — every load of the next
//       element queues behind the finished strip's write-through stores on the in-order vmcnt
//   w4  one wave per SIMD × two 16-column tiles in one interleaved stream (apply32_2), and TWO
//       strips per wave: while element e runs on one, the other (element e-1's result) is stored
//       and element e+1's strip loaded into it, a quarter per group over the first four groups —
//       each group's sync point waits only for the DMA issued before that group's I/O
// MODE 1: no strip I/O (both designs' ceiling with the DMA and the waits). MODE 2: desync — every
// workgroup first runs (5 blockIdx) mod NG groups without I/O, so that the CUs' strip traffic is
// spread over time as in the engine (in lockstep all 256 CUs stream at once: an HBM burst).
// MODE 8 (w4): the second strip's I/O spread through phase 2 (one instruction per tile row).
// MODE 4 (w8): plain write-back strip stores instead of write-through (sc1) — not a valid hand-over
// by itself (another XCD would not see them without an L2 write-back), the cost of sc1 alone.
// TF/s counts the algorithmic TSMQR flops (4 b^2 per column and element).
// Build: hipcc --offload-arch=gfx950 -O3 -I../../gpu-tiled-qr-decomposition_amd/csrc -I../../include chain32io_bench.hip -o chain32io_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "gridscheduler.h"
#include "tiles.hpp"
namespace tqr {
struct Item {  // (as engine.hip: flow.hpp, which chain32.hpp needs, names it)
  int ts, l, m, k;
};
}  // namespace tqr
#include "flow.hpp"

using namespace tqr;
#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);         \
      return 1;                                                                \
    }                                                                          \
  } while (0)

constexpr int B = 256;
using G32 = Geo32<B>;
constexpr int NMT = G32::NMT, NMI = G32::NMI, NG = G32::NG;
constexpr long LDM = 16384;  // rows of the streamed matrix (64 tile rows)
constexpr int NTILE = 64;
constexpr int IMG = G32::VIMG + G32::TIMG;  // doubles per group image (V then T)
constexpr int NU = IMG / 128;               // 1-KiB DMA units

template <int NW>
struct Dma32 {  // the next group's images into the other LDS buffer, 16 B per lane per step
  static constexpr int STEPS = (NU + NW - 1) / NW;
  double* dst;
  const double* src;
  __device__ __forceinline__ void mid() const {}
  __device__ __forceinline__ void step(int m) const {
    if (m >= STEPS) return;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int u = min(w + NW * m, NU - 1);
    const unsigned l =
        __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) void*)(dst + u * 128));
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off sc1" ::"v"(src + u * 128 + 2 * lane), "{m0}"(l) : "memory");
  }
};

template <int N>
__device__ __forceinline__ void sync_cnt() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct NoPost2 {
  __device__ __forceinline__ void at(int) const {}
};
// apply32 for two 16-column tiles of one wave (same V and T), one interleaved stream; post.at(mt)
// after phase 2's MFMAs of tile row mt (strip I/O spread through the MFMA stream)
template <typename Hook, typename Post = NoPost2>
__device__ __forceinline__ void apply32_2(const float* VR, const float* TPi, f4v (&X0)[NMT], f4v (&X1)[NMT],
                                          f4v (&H0)[NMT], f4v (&H1)[NMT], const Hook& hook,
                                          const Post& post = Post()) {
  constexpr int IB = G32::IB;
  const int lane = threadIdx.x & 63, x = lane >> 4, y = lane & 15, q = y >> 2, e = y & 3;
  const int sx = (x & 1) | (((x >> 1) & 1) << 2);
  const int sy = (((y >> 1) ^ (y >> 2)) & 1) | (((y >> 3) & 1) << 2);
  const unsigned vb = lds_addr_f(VR);
  unsigned b1[NMI], b2[NMI];
#pragma unroll
  for (int m = 0; m < NMI; ++m) {
    b1[m] = vb + 4u * (4 * x * IB + (((NMI * q + m) ^ sx) << 2) + e);
    b2[m] = vb + 4u * (y * IB + (((NMI * x + m) ^ sy) << 2));
  }
  auto ld1 = [&](float (&a)[4 * NMI], int mt) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int mi = 0; mi < NMI; ++mi) a[r * NMI + mi] = lds_rdf(b1[mi ^ ((r >> 1) & 1)] + 4u * ((16 * mt + r) * IB));
  };
  auto ld2 = [&](float (&a)[4 * NMI], int mt) {
#pragma unroll
    for (int wi = 0; wi < NMI; ++wi) {
      const f4v t = lds_rdf4(b2[wi] + 4u * (16 * mt * IB));
#pragma unroll
      for (int r = 0; r < 4; ++r) a[4 * wi + r] = t[r];
    }
  };
  f4v Z0[NMI], Z1[NMI];
#pragma unroll
  for (int mi = 0; mi < NMI; ++mi) {
    Z0[mi] = H0[mi];
    Z1[mi] = H1[mi];
  }
  float ac[4 * NMI], an[4 * NMI];
  ld1(ac, 0);
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    hook.step(mt);
    if (mt + 1 < NMT) ld1(an, mt + 1);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int mi = 0; mi < NMI; ++mi) {
        Z0[mi] = mfma16(ac[r * NMI + mi], X0[mt][r], Z0[mi]);
        Z1[mi] = mfma16(ac[r * NMI + mi], X1[mt][r], Z1[mi]);
      }
#pragma unroll
    for (int k = 0; k < 4 * NMI; ++k) ac[k] = an[k];
  }
  f4v W0[NMI], W1[NMI];
  {
    float tp[4 * G32::NPR];
    ld_chunks<G32::NPR>(tp, TPi, 0, lane);
#pragma unroll
    for (int wi = 0, pr = 0; wi < NMI; ++wi) {
      W0[wi] = f4v{0.f, 0.f, 0.f, 0.f};
      W1[wi] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int mi = 0; mi <= wi; ++mi, ++pr)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          W0[wi] = mfma16(tp[4 * pr + r], Z0[mi][r], W0[wi]);
          W1[wi] = mfma16(tp[4 * pr + r], Z1[mi][r], W1[wi]);
        }
    }
  }
#pragma unroll
  for (int wi = 0; wi < NMI; ++wi) {
    H0[wi] += W0[wi];
    H1[wi] += W1[wi];
  }
  float c0[4 * NMI];
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    ld2(c0, mt);
#pragma unroll
    for (int wi = 0; wi < NMI; ++wi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        X0[mt] = mfma16(c0[4 * wi + r], W0[wi][r], X0[mt]);
        X1[mt] = mfma16(c0[4 * wi + r], W1[wi][r], X1[mt]);
      }
    post.at(mt);
  }
}

// MODE 8 (w4): chunk C of the second strip's I/O as ONE vector-memory instruction per phase-2 tile
// row (stores at mt < 8, loads at mt >= 8) instead of a burst after the group
template <int C>
struct IoPost {
  __amdgpu_buffer_rsrc_t rs;
  f4v (&B0)[NMT];
  f4v (&B1)[NMT];
  unsigned o0, o1, i0, i1;
  bool st, ld;
  __device__ __forceinline__ void at(int mt) const {
    const int k = 4 * C + ((mt & 7) >> 1);
    if (mt < 8) {
      if (st) st_f4(rs, ((mt & 1) ? o1 : o0) + 64u * k, (mt & 1) ? B1[k] : B0[k]);
    } else if (ld) {
      if (mt & 1) B1[k] = ld_f4(rs, i1 + 64u * k);
      else B0[k] = ld_f4(rs, i0 + 64u * k);
    }
  }
};

// strip tile I/O: tile mt of a 16-column tile at column c, rows 16mt + 4x .. + 3 (Strip32's layout)
__device__ __forceinline__ unsigned tile_off(int c, int ti) {
  const int lane = threadIdx.x & 63, x = lane >> 4, y = lane & 15;
  return (unsigned)((((size_t)(c + y)) * LDM + (size_t)ti * B + 4 * x) * sizeof(float));
}

template <int MODE>
__global__ __launch_bounds__(512, 1) void k_w8(float* S, const double* img, int nelem) {
  extern __shared__ __align__(16) double lds[];
  const int w = threadIdx.x >> 6;
  const int col = blockIdx.x * 128 + 16 * w;
  const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(S);
  f4v X[NMT], H[NMT];
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) H[mt] = f4v{1e-3f, 0.f, 0.f, 1e-3f};
  auto gimg = [&](int ti, int g) { return img + ((size_t)ti * NG + g) * IMG; };
  {
    Dma32<8> d{lds, gimg(0, 0)};
    for (int m = 0; m < Dma32<8>::STEPS; ++m) d.step(m);
  }
  int buf = 0;
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) X[mt] = ld_f4(rs, tile_off(col, 0) + 64u * mt);
  if (MODE & 2) {  // desync: (5 blockIdx) mod NG groups without I/O first
    const int pre = (5 * blockIdx.x) % NG;
    for (int g = 0; g < pre; ++g) {
      sync_cnt<0>();
      Dma32<8> d{lds + (buf ^ 1) * IMG, gimg(0, g + 1)};
      apply32<B, true, Dma32<8>>((const float*)(lds + buf * IMG), (const float*)(lds + buf * IMG + G32::VIMG), X, H, d);
      buf ^= 1;
    }
  }
  for (int e = 0; e < nelem; ++e) {
    const int ti = e % NTILE, tn = (e + 1) % NTILE;
    for (int g = 0; g < NG; ++g) {
      sync_cnt<0>();
      const float* VR = (const float*)(lds + buf * IMG);
      const float* TPi = (const float*)(lds + buf * IMG + G32::VIMG);
      const int gn = g + 1 < NG ? g + 1 : 0;
      Dma32<8> d{lds + (buf ^ 1) * IMG, gimg(g + 1 < NG ? ti : tn, gn)};
      if (!(MODE & 1) && g + 1 == NG) {
        // XPipe32 with the next element's strip at another offset of the same buffer
        constexpr int SC1 = (MODE & 4) ? 0 : 1;
        struct Pipe {
          __amdgpu_buffer_rsrc_t rs;
          unsigned out, in;
          __device__ __forceinline__ void at(int mt, f4v (&X)[NMT]) const {
            if (mt >= 2) {
              st_f4(rs, out + 64u * (mt - 2), X[mt - 2], SC1);
              st_f4(rs, out + 64u * (mt - 1), X[mt - 1], SC1);
            }
            if (mt >= 4) {
              X[mt - 4] = ld_f4(rs, in + 64u * (mt - 4));
              X[mt - 3] = ld_f4(rs, in + 64u * (mt - 3));
            }
          }
          __device__ __forceinline__ void fin(f4v (&X)[NMT]) const {
            st_f4(rs, out + 64u * (NMT - 2), X[NMT - 2], SC1);
            st_f4(rs, out + 64u * (NMT - 1), X[NMT - 1], SC1);
#pragma unroll
            for (int mt = NMT - 4; mt < NMT; ++mt) X[mt] = ld_f4(rs, in + 64u * mt);
          }
        } pp{rs, tile_off(col, ti), tile_off(col, tn)};
        apply32<B, true, Dma32<8>, Pipe>(VR, TPi, X, H, d, pp);
      } else {
        apply32<B, true, Dma32<8>>(VR, TPi, X, H, d);
      }
      buf ^= 1;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) st_f4(rs, tile_off(col, 0) + 64u * mt, X[mt] + H[mt & 1]);
}

// element e's strip I/O chunk C (of 4) on the second strip: store element e-1's result, load e+1's
template <int C>
__device__ __forceinline__ void io_chunk(__amdgpu_buffer_rsrc_t rs, f4v (&B0)[NMT], f4v (&B1)[NMT], unsigned o0,
                                         unsigned o1, unsigned i0, unsigned i1, bool st, bool ld) {
  constexpr int M0 = 4 * C;
  if (st) {
#pragma unroll
    for (int mt = M0; mt < M0 + 4; ++mt) {
      st_f4(rs, o0 + 64u * mt, B0[mt]);
      st_f4(rs, o1 + 64u * mt, B1[mt]);
    }
  }
  if (ld) {
#pragma unroll
    for (int mt = M0; mt < M0 + 4; ++mt) {
      B0[mt] = ld_f4(rs, i0 + 64u * mt);
      B1[mt] = ld_f4(rs, i1 + 64u * mt);
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void k_w4(float* S, const double* img, int nelem) {
  extern __shared__ __align__(16) double lds[];
  const int w = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 128 + 32 * w, c1 = c0 + 16;
  const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(S);
  f4v A0[NMT], A1[NMT], B0[NMT], B1[NMT], H0[NMT], H1[NMT];
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    H0[mt] = f4v{1e-3f, 0.f, 0.f, 1e-3f};
    H1[mt] = H0[mt];
    B0[mt] = B1[mt] = f4v{0.f, 0.f, 0.f, 0.f};
  }
  auto gimg = [&](int ti, int g) { return img + ((size_t)ti * NG + g) * IMG; };
  {
    Dma32<4> d{lds, gimg(0, 0)};
    for (int m = 0; m < Dma32<4>::STEPS; ++m) d.step(m);
  }
  int buf = 0;
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    A0[mt] = ld_f4(rs, tile_off(c0, 0) + 64u * mt);
    A1[mt] = ld_f4(rs, tile_off(c1, 0) + 64u * mt);
  }
  if (MODE & 2) {  // desync, as k_w8
    const int pre = (5 * blockIdx.x) % NG;
    for (int g = 0; g < pre; ++g) {
      sync_cnt<0>();
      Dma32<4> d{lds + (buf ^ 1) * IMG, gimg(0, g + 1)};
      apply32_2((const float*)(lds + buf * IMG), (const float*)(lds + buf * IMG + G32::VIMG), A0, A1, H0, H1, d);
      buf ^= 1;
    }
  }
  constexpr bool IO = !(MODE & 1);
  for (int e = 0; e < nelem; ++e) {
    const int ti = e % NTILE, tn = (e + 1) % NTILE, tp = (e + NTILE - 1) % NTILE;
    const bool st = IO && e > 0, ld = IO && e + 1 < nelem;
    const unsigned o0 = tile_off(c0, tp), o1 = tile_off(c1, tp), i0 = tile_off(c0, tn), i1 = tile_off(c1, tn);
    auto group = [&](int g, auto io) {
      if (g == 0 || !IO) sync_cnt<0>();
      else sync_cnt<16>();  // this group's DMA (issued before the previous group's 16 strip I/O ops)
      const float* VR = (const float*)(lds + buf * IMG);
      const float* TPi = (const float*)(lds + buf * IMG + G32::VIMG);
      const int gn = g + 1 < NG ? g + 1 : 0;
      Dma32<4> d{lds + (buf ^ 1) * IMG, gimg(g + 1 < NG ? ti : tn, gn)};
      io(VR, TPi, d);
      buf ^= 1;
    };
    auto plain = [&](const float* VR, const float* TPi, const Dma32<4>& d) { apply32_2(VR, TPi, A0, A1, H0, H1, d); };
    if constexpr (MODE & 8) {
      group(0, [&](const float* VR, const float* TPi, const Dma32<4>& d) {
        apply32_2(VR, TPi, A0, A1, H0, H1, d, IoPost<0>{rs, B0, B1, o0, o1, i0, i1, st, ld}); });
      group(1, [&](const float* VR, const float* TPi, const Dma32<4>& d) {
        apply32_2(VR, TPi, A0, A1, H0, H1, d, IoPost<1>{rs, B0, B1, o0, o1, i0, i1, st, ld}); });
      group(2, [&](const float* VR, const float* TPi, const Dma32<4>& d) {
        apply32_2(VR, TPi, A0, A1, H0, H1, d, IoPost<2>{rs, B0, B1, o0, o1, i0, i1, st, ld}); });
      group(3, [&](const float* VR, const float* TPi, const Dma32<4>& d) {
        apply32_2(VR, TPi, A0, A1, H0, H1, d, IoPost<3>{rs, B0, B1, o0, o1, i0, i1, st, ld}); });
    } else {
      group(0, [&](const float* VR, const float* TPi, const Dma32<4>& d) { plain(VR, TPi, d); io_chunk<0>(rs, B0, B1, o0, o1, i0, i1, st, ld); });
      group(1, [&](const float* VR, const float* TPi, const Dma32<4>& d) { plain(VR, TPi, d); io_chunk<1>(rs, B0, B1, o0, o1, i0, i1, st, ld); });
      group(2, [&](const float* VR, const float* TPi, const Dma32<4>& d) { plain(VR, TPi, d); io_chunk<2>(rs, B0, B1, o0, o1, i0, i1, st, ld); });
      group(3, [&](const float* VR, const float* TPi, const Dma32<4>& d) { plain(VR, TPi, d); io_chunk<3>(rs, B0, B1, o0, o1, i0, i1, st, ld); });
    }
#pragma clang loop unroll(disable)
    for (int g = 4; g < NG; ++g) group(g, plain);
    if (IO) {  // element e+1 runs on the strip just loaded; element e's result is stored during it
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt) {
        const f4v t0 = A0[mt], t1 = A1[mt];
        A0[mt] = B0[mt];
        A1[mt] = B1[mt];
        B0[mt] = t0;
        B1[mt] = t1;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    st_f4(rs, tile_off(c0, 0) + 64u * mt, A0[mt] + B0[mt] + H0[mt & 1]);
    st_f4(rs, tile_off(c1, 0) + 64u * mt, A1[mt] + B1[mt] + H1[mt & 1]);
  }
}

template <typename K>
static int run(const char* name, K kern, int nth, float* S, const double* img, int ncu, int nelem) {
  const size_t lds = 2 * IMG * sizeof(double);
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    CK(hipEventRecord(e0, 0));
    kern<<<ncu, nth, lds>>>(S, img, nelem);
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  const double flops = 4.0 * B * B * 128.0 * nelem * ncu;
  printf("%-34s %8.3f ms  %6.1f TF/s  %6.2f us per element\n", name, best, flops / best / 1e9, best * 1e3 / nelem);
  return 0;
}

__global__ void k_fill(float* p, size_t n, float scale, unsigned long long seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned long long z = (i + seed) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 31;
    p[i] = scale * (((float)(z % 2001) - 1000.0f) / 1000.0f);
  }
}

int main(int argc, char** argv) {
  const int nelem = argc > 1 ? atoi(argv[1]) : 96;
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  const size_t ns = (size_t)ncu * 128 * LDM, nimg = (size_t)NTILE * NG * IMG;
  float* S;
  double* img;
  CK(hipMalloc(&S, ns * sizeof(float)));
  CK(hipMalloc(&img, nimg * sizeof(double)));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, S, ns, 0.5f, 1ull);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (float*)img, 2 * nimg, 1e-3f, 3ull);
  CK(hipDeviceSynchronize());
  printf("fp32 chain element loop with traffic: %d CUs, %d elements per workgroup, 128 columns per CU\n", ncu, nelem);
  if (run("w8 (engine: XPipe32 hand-over)", k_w8<0>, 512, S, img, ncu, nelem)) return 1;
  if (run("w8 no strip I/O", k_w8<1>, 512, S, img, ncu, nelem)) return 1;
  if (run("w4 two strips (I/O over 4 groups)", k_w4<0>, 256, S, img, ncu, nelem)) return 1;
  if (run("w4 no strip I/O", k_w4<1>, 256, S, img, ncu, nelem)) return 1;
  if (run("w8 hand-over, desync", k_w8<2>, 512, S, img, ncu, nelem)) return 1;
  if (run("w8 no strip I/O, desync", k_w8<3>, 512, S, img, ncu, nelem)) return 1;
  if (run("w8 hand-over, desync, plain stores", k_w8<6>, 512, S, img, ncu, nelem)) return 1;
  if (run("w4 two strips, desync", k_w4<2>, 256, S, img, ncu, nelem)) return 1;
  if (run("w4 no strip I/O, desync", k_w4<3>, 256, S, img, ncu, nelem)) return 1;
  if (run("w4 two strips, I/O in the stream, desync", k_w4<10>, 256, S, img, ncu, nelem)) return 1;
  return 0;
}
