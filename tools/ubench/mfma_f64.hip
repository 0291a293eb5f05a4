// Microbenchmark: fp64 MFMA (v_mfma_f64_16x16x4_f64, v_mfma_f64_4x4x4_4b_f64), fp32-input MFMA
// (v_mfma_f32_16x16x4_f32, v_mfma_f32_32x32x2_f32, v_mfma_f32_4x4x1_16b_f32) and fp64 vector FMA
// throughput on gfx950, with the in-kernel clock (s_memtime / s_memrealtime @100 MHz).
// Flops per wave-instruction: 16x16x4 f64 2*16*16*4 = 2048; 4x4x4_4b f64 4 blocks * 2*4*4*4 = 512;
// 16x16x4 f32 2048; 32x32x2 f32 2*32*32*2 = 4096; 4x4x1_16b f32 16 blocks * 2*4*4*1 = 512.
// Establishes the roofline denominators used in bench.py (DESIGN.md "Roofline").
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
typedef double d4 __attribute__((ext_vector_type(4)));

__device__ inline void stamp(unsigned long long* clk, int first) {
  if (threadIdx.x == 0) {
    unsigned long long t = __builtin_amdgcn_s_memtime();
    unsigned long long r = __builtin_amdgcn_s_memrealtime();
    clk[blockIdx.x * 4 + (first ? 0 : 2)] = t;
    clk[blockIdx.x * 4 + (first ? 1 : 3)] = r;
  }
}

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma(double* out, unsigned long long* clk, int iters, double seed) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{seed, -seed, seed, -seed};
  double a = seed * (threadIdx.x + 1), b = seed * 0.5 - threadIdx.x * 1e-7;
  stamp(clk, 1);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  stamp(clk, 0);
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma4(double* out, unsigned long long* clk, int iters, double seed) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = seed * i;
  double a = seed * (threadIdx.x + 1), b = seed * 0.5 - threadIdx.x * 1e-7;
  stamp(clk, 1);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  }
  stamp(clk, 0);
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
// SHAPE 0: 16x16x4 f32 (4 acc regs), 1: 32x32x2 f32 (16 acc regs), 2: 4x4x1_16b f32 (4 acc regs)
template <int SHAPE, int NACC>
__global__ __launch_bounds__(256) void k_mfma32(float* out, unsigned long long* clk, int iters, float seed) {
  float a = seed * (threadIdx.x + 1), b = seed * 0.5f - threadIdx.x * 1e-7f;
  stamp(clk, 1);
  float s = 0;
  if constexpr (SHAPE == 1) {
    f16v acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = f16v{} + seed * i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
    }
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
  } else {
    f4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = f4{seed, -seed, seed * i, -seed};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < NACC; ++i)
        acc[i] = SHAPE == 0 ? __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
    }
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][3];
  }
  stamp(clk, 0);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fma(double* out, unsigned long long* clk, int iters, double seed) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = seed + i + threadIdx.x * 1e-3;
  double a = 0.9999999, b = 1e-9 * threadIdx.x;
  stamp(clk, 1);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], a, b);
  }
  stamp(clk, 0);
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static void report(const char* name, float ms, double flops, unsigned long long* hclk, int blocks) {
  double fsum = 0; int n = 0;
  for (int b = 0; b < blocks; ++b) {
    double dt = (double)(hclk[b * 4 + 2] - hclk[b * 4 + 0]);
    double dr = (double)(hclk[b * 4 + 3] - hclk[b * 4 + 1]);
    if (dr > 0) { fsum += dt / dr * 100.0; ++n; }
  }
  printf("%-34s %8.3f ms %8.2f TFLOP/s  in-kernel clock %.0f MHz\n", name, ms, flops / ms / 1e9, n ? fsum / n : 0.0);
}

int main() {
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  printf("device gcn %s CUs %d clock %d kHz LDS/blk %zu L2 %d\n", p.gcnArchName, p.multiProcessorCount, p.clockRate, p.sharedMemPerBlock, p.l2CacheSize);
  int maxblocks = p.multiProcessorCount * 4;
  double* out; CK(hipMalloc(&out, maxblocks * 256 * sizeof(double)));
  unsigned long long *clk, *hclk = new unsigned long long[maxblocks * 4];
  CK(hipMalloc(&clk, maxblocks * 4 * sizeof(unsigned long long)));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int iters = 20000;
  // warm the clock up
  k_fma<<<maxblocks, 256>>>(out, clk, iters * 8, 1.0);
  CK(hipDeviceSynchronize());
  for (int bpc = 1; bpc <= 4; bpc *= 2) {
    int blocks = p.multiProcessorCount * bpc;
    char nm[64]; float ms;
#define RUN(NAME, LAUNCH, FLOPS)                                                        \
    CK(hipEventRecord(e0)); LAUNCH; CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); \
    CK(hipEventElapsedTime(&ms, e0, e1));                                               \
    CK(hipMemcpy(hclk, clk, blocks * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost)); \
    snprintf(nm, sizeof nm, NAME " %d wave/SIMD", bpc); report(nm, ms, FLOPS, hclk, blocks);
    RUN("mfma_f64_16x16x4 x4acc", (k_mfma<4><<<blocks, 256>>>(out, clk, iters, 1e-3)), (double)blocks * 4 * iters * 4 * 2048.0);
    RUN("mfma_f64_16x16x4 x8acc", (k_mfma<8><<<blocks, 256>>>(out, clk, iters / 2, 1e-3)), (double)blocks * 4 * (iters / 2) * 8 * 2048.0);
    RUN("mfma_f64_4x4x4_4b x8acc", (k_mfma4<8><<<blocks, 256>>>(out, clk, iters, 1e-3)), (double)blocks * 4 * iters * 8 * 512.0);
    // dependent-accumulator latency: fewer independent chains than the latency / issue ratio
    // leave the pipe idle (one wave per SIMD shows it directly)
    RUN("mfma_f64_4x4x4_4b x1acc", (k_mfma4<1><<<blocks, 256>>>(out, clk, iters, 1e-3)), (double)blocks * 4 * iters * 1 * 512.0);
    RUN("mfma_f64_4x4x4_4b x2acc", (k_mfma4<2><<<blocks, 256>>>(out, clk, iters, 1e-3)), (double)blocks * 4 * iters * 2 * 512.0);
    RUN("mfma_f64_4x4x4_4b x3acc", (k_mfma4<3><<<blocks, 256>>>(out, clk, iters, 1e-3)), (double)blocks * 4 * iters * 3 * 512.0);
    RUN("mfma_f64_4x4x4_4b x4acc", (k_mfma4<4><<<blocks, 256>>>(out, clk, iters, 1e-3)), (double)blocks * 4 * iters * 4 * 512.0);
    RUN("mfma_f32_16x16x4 x8acc", (k_mfma32<0, 8><<<blocks, 256>>>((float*)out, clk, iters / 2, 1e-3f)), (double)blocks * 4 * (iters / 2) * 8 * 2048.0);
    RUN("mfma_f32_32x32x2 x4acc", (k_mfma32<1, 4><<<blocks, 256>>>((float*)out, clk, iters / 2, 1e-3f)), (double)blocks * 4 * (iters / 2) * 4 * 4096.0);
    RUN("mfma_f32_4x4x1_16b x8acc", (k_mfma32<2, 8><<<blocks, 256>>>((float*)out, clk, iters, 1e-3f)), (double)blocks * 4 * iters * 8 * 512.0);
    RUN("v_fma_f64 x8", (k_fma<<<blocks, 256>>>(out, clk, iters * 4, 1.0)), (double)blocks * 256 * iters * 4 * 8 * 2.0);
  }
  return 0;
}
