// Microbenchmark: the fp32 chain's group loop (chain32.hpp apply32, v_mfma_f32_16x16x4_f32) at
// two occupancies, MFMA stream only (images resident in LDS, no strip or head I/O, no DMA):
//   w8  one 8-wave workgroup per CU, one 16-column strip tile per wave (the engine's shape, 256 VGPRs)
//   w4  one 4-wave workgroup per CU (one wave per SIMD, up to 512 registers), two 16-column strip
//       tiles per wave; MODE 1: also two more strips held live across the loop — the register
//       budget of a chain that keeps the next element's strip resident (loaded a whole element
//       ahead) so that no load waits behind the finished strip's stores; MODE 2: the two tiles in
//       one interleaved stream (apply32_2) instead of two apply32 calls
// The question for the one-wave-per-SIMD fp32 chain (DESIGN.md §10, round-5 plan): does one wave
// per SIMD keep the f32 MFMA pipe as busy as two (issue 32 cycles, dependent latency 40), and do
// the extra strips fit without spills. TF/s counts the issued MFMAs (2048 flop each).
// Build: hipcc --offload-arch=gfx950 -O3 -I../../gpu-tiled-qr-decomposition_amd/csrc -I../../include chain32_bench.hip -o chain32_bench
#include <hip/hip_runtime.h>

#include <cstdio>

#include "gridscheduler.h"
#include "tiles.hpp"
namespace tqr {
struct Item {  // (as engine.hip: flow.hpp, which chain32.hpp needs, names it)
  int ts, l, m, k;
};
}  // namespace tqr
#include "flow.hpp"  // (includes chain32.hpp, which uses its helpers)

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
constexpr int NMT = G32::NMT, NMI = G32::NMI;
constexpr int LDS_F = G32::VR + G32::TP;  // floats
// MFMAs per apply32 call (one 16-column strip tile): phase 1, W, phase 2
constexpr int MFMA_PER_APPLY = NMT * 4 * NMI + 4 * G32::NPR + NMT * 4 * NMI;

__device__ __forceinline__ void init_lds(float* lds, int nth) {
  for (int i = threadIdx.x; i < LDS_F; i += nth) lds[i] = 1e-3f * (float)((i * 37) % 101 - 50);
  __syncthreads();
}

template <int NT>
__device__ __forceinline__ void load_tile(f4v (&X)[NMT], const float* in, int salt) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    const float* p = in + ((blockIdx.x * NT + threadIdx.x) * 4 + mt * 4 * NT * gridDim.x + salt) % (1 << 20);
    X[mt] = f4v{p[0], p[1], p[2], p[3]} * 1e-2f + (float)lane * 1e-4f;
  }
}

__global__ __launch_bounds__(512, 1) void k_w8(const float* in, float* out, int groups) {
  extern __shared__ __align__(16) float lds[];
  init_lds(lds, 512);
  f4v X[NMT], H[NMT];
  load_tile<512>(X, in, 0);
  load_tile<512>(H, in, 7);
  for (int g = 0; g < groups; ++g) {
    apply32<B, true, NoHook>(lds, lds + G32::VR, X, H, NoHook());
    __syncthreads();
  }
  f4v s = H[0] + H[1];
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) s += X[mt];
  out[blockIdx.x * 512 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// apply32 for TWO 16-column strip tiles of one wave (the same V and T): every V operand read
// feeds both tiles' MFMAs, and the two tiles' accumulation chains interleave (phase 1: 2 NMI
// chains, phase 2: 2 tiles) — the w4 form's own instruction stream, as a one-wave chain would have
__device__ __forceinline__ void apply32_2(const float* VR, const float* TPi, f4v (&X0)[NMT], f4v (&X1)[NMT],
                                          f4v (&H0)[NMT], f4v (&H1)[NMT]) {
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
    ld2(c0, mt);
#pragma unroll
    for (int wi = 0; wi < NMI; ++wi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        X0[mt] = mfma16(c0[4 * wi + r], W0[wi][r], X0[mt]);
        X1[mt] = mfma16(c0[4 * wi + r], W1[wi][r], X1[mt]);
      }
  }
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void k_w4(const float* in, float* out, int groups) {
  extern __shared__ __align__(16) float lds[];
  init_lds(lds, 256);
  f4v X0[NMT], X1[NMT], H0[NMT], H1[NMT];
  load_tile<256>(X0, in, 0);
  load_tile<256>(X1, in, 3);
  load_tile<256>(H0, in, 7);
  load_tile<256>(H1, in, 11);
  f4v N0[NMT], N1[NMT];  // MODE 1: the next element's strips, live across the loop
  if constexpr (MODE & 1) {
    load_tile<256>(N0, in, 13);
    load_tile<256>(N1, in, 17);
  }
  for (int g = 0; g < groups; ++g) {
    if constexpr (MODE & 2) {
      apply32_2(lds, lds + G32::VR, X0, X1, H0, H1);
    } else {
      apply32<B, true, NoHook>(lds, lds + G32::VR, X0, H0, NoHook());
      apply32<B, true, NoHook>(lds, lds + G32::VR, X1, H1, NoHook());
    }
    __syncthreads();
  }
  f4v s = H0[0] + H0[1] + H1[0] + H1[1];
#pragma unroll
  for (int mt = 0; mt < NMT; ++mt) {
    s += X0[mt] + X1[mt];
    if constexpr (MODE & 1) s += N0[mt] * N1[mt];
  }
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

template <typename K>
static int time_kernel(const char* name, K kern, int nth, int tiles_per_wave, const float* in, float* out, int cus) {
  const size_t lds = LDS_F * sizeof(float);
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int groups = 2000;
  kern<<<cus, nth, lds>>>(in, out, 50);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    kern<<<cus, nth, lds>>>(in, out, groups);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double flops = (double)cus * (nth / 64) * tiles_per_wave * groups * MFMA_PER_APPLY * 2048.0;
  printf("%-26s %7.3f ms  %6.1f TF/s issued  (%.2f us per group)\n", name, best, flops / (best * 1e-3) / 1e12,
         best * 1e3 / groups);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  float *in, *out;
  CK(hipMalloc(&in, (1 << 20) * sizeof(float) + 4096));
  CK(hipMalloc(&out, (size_t)cus * 512 * sizeof(float)));
  CK(hipMemset(in, 0, (1 << 20) * sizeof(float) + 4096));
  printf("fp32 chain group loop, %d CUs, %d MFMAs per strip tile and group\n", cus, MFMA_PER_APPLY);
  if (time_kernel("w8: 8 waves x 1 tile", k_w8, 512, 1, in, out, cus)) return 1;
  if (time_kernel("w4: 4 waves x 2 tiles", k_w4<0>, 256, 2, in, out, cus)) return 1;
  if (time_kernel("w4: + 2 strips held live", k_w4<1>, 256, 2, in, out, cus)) return 1;
  if (time_kernel("w4: 2 tiles interleaved", k_w4<2>, 256, 2, in, out, cus)) return 1;
  if (time_kernel("w4: interleaved + 2 live", k_w4<3>, 256, 2, in, out, cus)) return 1;
  return 0;
}
