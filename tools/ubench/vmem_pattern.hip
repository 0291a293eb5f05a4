// Microbenchmark: the fp64 chain's strip hand-over I/O on its own — per wave 32 row pairs of a
// 16-column strip (buffer_load/store_dwordx4, 4 lanes per column, 64 B per column per instruction,
// columns ldm*8 bytes apart), no MFMAs. Measures one workgroup alone and all CUs at once, stores
// only, loads only, and both interleaved as in the chain (store pair p, load pair p-2), so the
// hand-over's cost can be split into issue / per-CU throughput / chip-wide bandwidth.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 vmem_pattern.hip -o vmem_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                 \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

constexpr int NP = 32;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  const unsigned long long u = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, 0x7fffffff, 0x00020000);
}

// MODE 1 = stores, 2 = loads, 3 = both (store p, then load p - 2); REP elements back to back.
// +4: full-line layout (each instruction 8 columns x 128 B: lane (x, c) -> column c & 7 (+8 for odd
// instructions), rows 16 (p/2) + 2x + 8 (c >= 8)), +8: contiguous (1 KiB per instruction in one column)
// Round 6, the strip's own 16 x 256 geometry with fewer columns per instruction (the same bytes):
// +16: 1 column per instruction (1 KiB = 128 rows), +32: 4 columns x 256 B, +64: 8 columns x 128 B,
// +128: the strip's own 16 columns x 64 B per instruction, but the 4 lanes of a column consecutive;
// +256 / +512: the strip layout moved by ds_bpermute to +128's / to 8 columns x 128 B (stores only)
template <int MODE, int SAUX = 16>
__global__ __launch_bounds__(512, 1) void k_io(double* X, long ldm, int rep, unsigned long long* clk) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, x = lane >> 4, c = lane & 15;
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  v4u r[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) r[p] = v4u{(unsigned)p, (unsigned)t, 1u, 2u};
  unsigned off = (unsigned)(((size_t)c * ldm + 2 * x) * 8), off2 = off;
  if (MODE & 4) {
    off = (unsigned)(((size_t)(c & 7) * ldm + 2 * x + (c >= 8 ? 8 : 0)) * 8);
    off2 = off + (unsigned)(8 * ldm * 8);
  }
  if (MODE & 8) off = off2 = (unsigned)(lane * 16);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int e = 0; e < rep; ++e) {
    double* base = X + (size_t)(blockIdx.x * 128 + 16 * w) * ldm + (size_t)(e % 32) * 256;
    const __amdgpu_buffer_rsrc_t so = rsrc(base), si = rsrc(base + 256);
    auto o = [&](int p) {
      if (MODE & 128) return (unsigned)(((size_t)(lane >> 2) * ldm + 8 * p + 2 * (lane & 3)) * 8);
      if (MODE & 16) return (unsigned)((size_t)(p / 2) * ldm * 8 + (p % 2) * 1024 + lane * 16);
      if (MODE & 32) return (unsigned)(((size_t)(4 * (p % 4) + lane / 16) * ldm + 32 * (p / 4) + 2 * (lane % 16)) * 8);
      if (MODE & 64) return (unsigned)(((size_t)(8 * (p % 2) + lane / 8) * ldm + 16 * (p / 2) + 2 * (lane % 8)) * 8);
      if (MODE & 8) return (unsigned)(p * 1024 + ((p & 1) ? 0 : 0)) + off + (unsigned)(w * 0);
      if (MODE & 4) return ((p & 1) ? off2 : off) + 128u * (p >> 1);
      return off + 64u * p;
    };
    if constexpr ((MODE & 256) != 0) {  // strip layout -> 16 columns x 64 B, 4 consecutive lanes per column
      const int src = (((lane & 3) << 4) | (lane >> 2)) * 4;
      const unsigned oq = (unsigned)(((size_t)(lane >> 2) * ldm + 2 * (lane & 3)) * 8);
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        v4u v;
#pragma unroll
        for (int d = 0; d < 4; ++d) v[d] = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)r[p][d]);
        __builtin_amdgcn_raw_buffer_store_b128(v, so, oq + 64u * p, 0, SAUX);
      }
    } else if constexpr ((MODE & 512) != 0) {  // strip layout -> 8 columns x 128 B (two row pairs), 8 lanes per column
      const int c1 = lane >> 3, r1 = lane & 7;
#pragma unroll
      for (int q = 0; q < NP / 2; ++q)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int src = (((r1 & 3) << 4) | ((2 * h + (c1 >> 2)) << 2) | (c1 & 3)) * 4;
          v4u v;
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const unsigned a = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)r[2 * q][d]);
            const unsigned b = (unsigned)__builtin_amdgcn_ds_bpermute(src, (int)r[2 * q + 1][d]);
            v[d] = (r1 & 4) ? b : a;
          }
          __builtin_amdgcn_raw_buffer_store_b128(v, so, (unsigned)(((size_t)(8 * h + c1) * ldm + 16 * q + 2 * r1) * 8), 0, SAUX);
        }
    } else
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      if (MODE & 1) __builtin_amdgcn_raw_buffer_store_b128(r[p], so, o(p), 0, SAUX);
      if ((MODE & 2) && (!(MODE & 1) || p >= 2)) r[(MODE & 1) ? p - 2 : p] = __builtin_amdgcn_raw_buffer_load_b128(si, o((MODE & 1) ? p - 2 : p), 0, 18);
    }
    if ((MODE & 3) == 3) {
      r[NP - 2] = __builtin_amdgcn_raw_buffer_load_b128(si, o(NP - 2), 0, 18);
      r[NP - 1] = __builtin_amdgcn_raw_buffer_load_b128(si, o(NP - 1), 0, 18);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) clk[blockIdx.x] = t1 - t0;
  if (r[3][0] == 12345u && r[7][1] == 999u) X[0] = 1.0;  // keep the loads
}

template <int MODE, int SAUX = 16>
static int run(double* X, long ldm, int nwg, int rep, unsigned long long* clk) {
  hipLaunchKernelGGL((k_io<MODE, SAUX>), dim3(nwg), dim3(512), 0, 0, X, ldm, rep, clk);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL((k_io<MODE, SAUX>), dim3(nwg), dim3(512), 0, 0, X, ldm, rep, clk);
  CK(hipDeviceSynchronize());
  unsigned long long h[1024];
  CK(hipMemcpy(h, clk, sizeof(unsigned long long) * nwg, hipMemcpyDeviceToHost));
  double s = 0;
  for (int i = 0; i < nwg; ++i) s += (double)h[i];
  const double us = s / nwg / rep * 0.01;
  const double kib = ((MODE & 3) == 3 ? 2.0 : 1.0) * NP * 8;  // KiB per workgroup per element
  printf("aux %2d mode %2d (%s, %s) %3d WG: %.2f us per element per WG, %.1f GB/s per CU\n", SAUX, MODE,
         (MODE & 3) == 1 ? "stores" : (MODE & 3) == 2 ? "loads " : "both  ",
         (MODE & 256) ? "bperm->quad" : (MODE & 512) ? "bperm->line" : (MODE & 128) ? "16x64B quad" : (MODE & 16) ? "1 col/insn" : (MODE & 32) ? "4 col/insn" : (MODE & 64) ? "8 col/insn" : (MODE & 8) ? "contiguous"
         : (MODE & 4) ? "full lines" : "half lines", nwg, us, kib * 1024 / us / 1e3);
  return 0;
}

int main(int argc, char** argv) {
  const long ldm = argc > 1 ? atol(argv[1]) : 16384;
  const int rep = 32;
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  double* X;
  CK(hipMalloc(&X, (size_t)ncu * 128 * ldm * 8));
  CK(hipMemset(X, 0, (size_t)ncu * 128 * ldm * 8));
  unsigned long long* clk;
  CK(hipMalloc(&clk, sizeof(unsigned long long) * 1024));
  if (argc > 2 && atoi(argv[2]) == 2) {  // columns per instruction (round 6)
    for (int nwg : {1, ncu}) {
      if (run<1 + 128>(X, ldm, nwg, rep, clk)) return 1;
      if (run<1 + 256>(X, ldm, nwg, rep, clk)) return 1;
      if (run<1 + 512>(X, ldm, nwg, rep, clk)) return 1;
      if (run<3 + 128>(X, ldm, nwg, rep, clk)) return 1;
      if (run<1>(X, ldm, nwg, rep, clk)) return 1;
      if (run<1 + 64>(X, ldm, nwg, rep, clk)) return 1;
      if (run<1 + 32>(X, ldm, nwg, rep, clk)) return 1;
      if (run<1 + 16>(X, ldm, nwg, rep, clk)) return 1;
      if (run<3>(X, ldm, nwg, rep, clk)) return 1;
      if (run<3 + 64>(X, ldm, nwg, rep, clk)) return 1;
      if (run<3 + 32>(X, ldm, nwg, rep, clk)) return 1;
      if (run<3 + 16>(X, ldm, nwg, rep, clk)) return 1;
    }
    return 0;
  }
  if (argc > 2) {  // store cache-policy sweep
    for (int nwg : {1, ncu}) {
      if (run<1, 0>(X, ldm, nwg, rep, clk)) return 1;
      if (run<1, 1>(X, ldm, nwg, rep, clk)) return 1;
      if (run<1, 2>(X, ldm, nwg, rep, clk)) return 1;
      if (run<1, 16>(X, ldm, nwg, rep, clk)) return 1;
      if (run<1, 17>(X, ldm, nwg, rep, clk)) return 1;
      if (run<3, 0>(X, ldm, nwg, rep, clk)) return 1;
      if (run<3, 2>(X, ldm, nwg, rep, clk)) return 1;
      if (run<7, 0>(X, ldm, nwg, rep, clk)) return 1;
      if (run<7, 2>(X, ldm, nwg, rep, clk)) return 1;
    }
    return 0;
  }
  for (int nwg : {1, ncu}) {
    if (run<1>(X, ldm, nwg, rep, clk)) return 1;
    if (run<2>(X, ldm, nwg, rep, clk)) return 1;
    if (run<3>(X, ldm, nwg, rep, clk)) return 1;
    if (run<5>(X, ldm, nwg, rep, clk)) return 1;
    if (run<6>(X, ldm, nwg, rep, clk)) return 1;
    if (run<7>(X, ldm, nwg, rep, clk)) return 1;
    if (run<9>(X, ldm, nwg, rep, clk)) return 1;
    if (run<10>(X, ldm, nwg, rep, clk)) return 1;
    if (run<11>(X, ldm, nwg, rep, clk)) return 1;
  }
  return 0;
}
