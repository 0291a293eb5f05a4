// Does s_waitcnt vmcnt(N) cover an older operation of another class on gfx950?
// (The fp64 asm chain counts waits across LDS-DMA, buffer loads and buffer stores.)
//   A: LDS-DMA from cold memory, then K buffer loads from hot memory, vmcnt(K): has the DMA landed?
//   B: a buffer load from cold memory, then K LDS-DMAs from hot memory, vmcnt(K): has the load landed?
//   C: a buffer load from cold memory, then K buffer stores to hot memory, vmcnt(K): has the load landed?
//   D: an LDS-DMA from cold memory, then K buffer stores, vmcnt(K): has the DMA landed?
// Every workgroup (one wave) repeats each test over fresh cold addresses; failures are counted.
// Build: hipcc --offload-arch=gfx950 -O3 vmcnt_order.hip -o vmcnt_order
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int K = 8;
constexpr int REPS = 64;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  const unsigned long long u = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, 0x7fffffff, 0x00020000);
}
// MUBUF variants of A-D (the chain's form: buffer loads / stores beside global_load_lds), plus
// E: a buffer load (cold) then K buffer loads (hot, sc1 nt) — in order within the class?
__global__ __launch_bounds__(64) void k_order_buf(const float* cold, float* hot, int* fails, size_t stride_f) {
  __shared__ __align__(16) float lds[64 * 4 * (K + 2)];
  const int lane = threadIdx.x;
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) void*)lds;
  int fa = 0, fb = 0, fc = 0, fd = 0, fe = 0;
  const __amdgpu_buffer_rsrc_t hr = rsrc_of(hot);
  for (int rep = 0; rep < REPS; ++rep) {
    const float* c = cold + ((size_t)(blockIdx.x * REPS + rep) * stride_f);
    const __amdgpu_buffer_rsrc_t cr = rsrc_of(c);
    for (int i = lane; i < 64 * 4; i += 64) lds[i] = -1.0f;
    __syncthreads();
    {  // A: DMA(cold) then K buffer loads (hot)
      float v, hd;
      asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %[ca], off\n\t.rept 8\n\tbuffer_load_dword %[hd], %[ho], %[hr], 0 offen sc1 nt\n\t.endr\n\t"
                   "s_waitcnt vmcnt(8)\n\tds_read_b32 %[v], %[la]\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                   : [v] "=&v"(v), [hd] "=&v"(hd)
                   : [l] "{m0}"(__builtin_amdgcn_readfirstlane(lds0)), [ca] "v"(c + 4 * lane), [ho] "v"(4u * lane), [hr] "s"(hr),
                     [la] "v"(lds0 + 16 * lane)
                   : "memory");
      if (v != c[4 * lane]) ++fa;
    }
    __syncthreads();
    {  // B: buffer load (cold) then K DMAs (hot)
      float v, r;
      asm volatile("v_mov_b32 %[v], -1.0\n\tbuffer_load_dword %[v], %[co], %[cr], 0 offen offset:0 sc1 nt\n\ts_nop 0\n\t.rept 8\n\t"
                   "global_load_lds_dwordx4 %[ha], off\n\t.endr\n\ts_waitcnt vmcnt(8)\n\tv_mov_b32 %[r], %[v]\n\ts_waitcnt vmcnt(0)"
                   : [v] "=&v"(v), [r] "=&v"(r)
                   : [l] "{m0}"(__builtin_amdgcn_readfirstlane(lds0 + 1024)), [co] "v"(4u * (2048 + lane)), [cr] "s"(cr),
                     [ha] "v"(hot + 4 * lane)
                   : "memory");
      if (r != c[2048 + lane]) ++fb;
    }
    __syncthreads();
    {  // C: buffer load (cold) then K buffer stores (hot, sc1)
      float v, r;
      asm volatile("v_mov_b32 %[v], -1.0\n\tbuffer_load_dword %[v], %[co], %[cr], 0 offen sc1 nt\n\t.rept 8\n\t"
                   "buffer_store_dword %[s], %[ho], %[hr], 0 offen offset:2048 sc1\n\t.endr\n\ts_waitcnt vmcnt(8)\n\tv_mov_b32 %[r], %[v]\n\ts_waitcnt vmcnt(0)"
                   : [v] "=&v"(v), [r] "=&v"(r)
                   : [co] "v"(4u * (4096 + lane)), [cr] "s"(cr), [ho] "v"(4u * lane), [hr] "s"(hr), [s] "v"((float)lane)
                   : "memory");
      if (r != c[4096 + lane]) ++fc;
    }
    __syncthreads();
    for (int i = lane; i < 64 * 4; i += 64) lds[i] = -1.0f;
    __syncthreads();
    {  // D: DMA (cold) then K buffer stores (hot)
      float v;
      asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %[ca], off\n\t.rept 8\n\tbuffer_store_dword %[s], %[ho], %[hr], 0 offen offset:4096 sc1\n\t.endr\n\t"
                   "s_waitcnt vmcnt(8)\n\tds_read_b32 %[v], %[la]\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                   : [v] "=&v"(v)
                   : [l] "{m0}"(__builtin_amdgcn_readfirstlane(lds0)), [ca] "v"(c + 6144 + 4 * lane), [ho] "v"(4u * lane), [hr] "s"(hr),
                     [s] "v"((float)lane), [la] "v"(lds0 + 16 * lane)
                   : "memory");
      if (v != c[6144 + 4 * lane]) ++fd;
    }
    __syncthreads();
    for (int i = lane; i < 64 * 4; i += 64) lds[i] = -1.0f;
    __syncthreads();
    {  // F: DMA (cold) then K buffer loads through a null resource (num_records = 0)
      float v, hd;
      const __amdgpu_buffer_rsrc_t nr = __builtin_amdgcn_make_buffer_rsrc((void*)hot, 0, 0, 0x00020000);
      asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %[ca], off\n\t.rept 8\n\tbuffer_load_dword %[hd], %[ho], %[hr], 0 offen sc1 nt\n\t.endr\n\t"
                   "s_waitcnt vmcnt(8)\n\tds_read_b32 %[v], %[la]\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                   : [v] "=&v"(v), [hd] "=&v"(hd)
                   : [l] "{m0}"(__builtin_amdgcn_readfirstlane(lds0)), [ca] "v"(c + 5120 + 4 * lane), [ho] "v"(4u * lane), [hr] "s"(nr),
                     [la] "v"(lds0 + 16 * lane)
                   : "memory");
      if (v != c[5120 + 4 * lane]) atomicAdd(&fails[9], 1);
    }
    __syncthreads();
    for (int i = lane; i < 64 * 4; i += 64) lds[i] = -1.0f;
    __syncthreads();
    {  // G: DMA (cold) then K buffer stores through a null resource
      float v;
      const __amdgpu_buffer_rsrc_t nr = __builtin_amdgcn_make_buffer_rsrc((void*)hot, 0, 0, 0x00020000);
      asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %[ca], off\n\t.rept 8\n\tbuffer_store_dword %[s], %[ho], %[hr], 0 offen sc1\n\t.endr\n\t"
                   "s_waitcnt vmcnt(8)\n\tds_read_b32 %[v], %[la]\n\ts_waitcnt vmcnt(0) lgkmcnt(0)"
                   : [v] "=&v"(v)
                   : [l] "{m0}"(__builtin_amdgcn_readfirstlane(lds0)), [ca] "v"(c + 3072 + 4 * lane), [ho] "v"(4u * lane), [hr] "s"(nr),
                     [s] "v"((float)lane), [la] "v"(lds0 + 16 * lane)
                   : "memory");
      if (v != c[3072 + 4 * lane]) atomicAdd(&fails[10], 1);
    }
    __syncthreads();
    {  // E: buffer load (cold) then K buffer loads (hot)
      float v, r, hd;
      asm volatile("v_mov_b32 %[v], -1.0\n\tbuffer_load_dword %[v], %[co], %[cr], 0 offen sc1 nt\n\t.rept 8\n\t"
                   "buffer_load_dword %[hd], %[ho], %[hr], 0 offen sc1 nt\n\t.endr\n\ts_waitcnt vmcnt(8)\n\tv_mov_b32 %[r], %[v]\n\ts_waitcnt vmcnt(0)"
                   : [v] "=&v"(v), [r] "=&v"(r), [hd] "=&v"(hd)
                   : [co] "v"(4u * (7168 + lane)), [cr] "s"(cr), [ho] "v"(4u * lane), [hr] "s"(hr)
                   : "memory");
      if (r != c[7168 + lane]) ++fe;
    }
    __syncthreads();
  }
  atomicAdd(&fails[4], fa);
  atomicAdd(&fails[5], fb);
  atomicAdd(&fails[6], fc);
  atomicAdd(&fails[7], fd);
  atomicAdd(&fails[8], fe);
}

__global__ __launch_bounds__(64) void k_order(const float* cold, float* hot, int* fails, size_t stride_f) {
  __shared__ __align__(16) float lds[64 * 4 * (K + 2)];
  const int lane = threadIdx.x;
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) void*)lds;
  int fa = 0, fb = 0, fc = 0, fd = 0;
  for (int rep = 0; rep < REPS; ++rep) {
    const float* c = cold + ((size_t)(blockIdx.x * REPS + rep) * stride_f);  // fresh cold line per rep
    const float expect = c[0];                                               // (the host filled c[i] = i-derived)
    (void)expect;
    // ---- A: DMA (cold) then K loads (hot) ----
    for (int i = lane; i < 64 * 4; i += 64) lds[i] = -1.0f;
    __syncthreads();
    {
      float v, hdummy;
      asm volatile(
          "s_nop 0\n\t"
          "global_load_lds_dwordx4 %[ca], off\n\t"
          ".rept 8\n\t"
          "global_load_dword %[hd], %[ha], off\n\t"
          ".endr\n\t"
          "s_waitcnt vmcnt(8)\n\t"
          "ds_read_b32 %[v], %[la]\n\t"
          "s_waitcnt vmcnt(0) lgkmcnt(0)"
          : [v] "=&v"(v), [hd] "=&v"(hdummy)
          : [l] "{m0}"(__builtin_amdgcn_readfirstlane(lds0)), [ca] "v"(c + 4 * lane), [ha] "v"(hot + lane),
            [la] "v"(lds0 + 16 * lane)
          : "memory");
      if (v != c[4 * lane]) ++fa;
    }
    __syncthreads();
    // ---- B: load (cold) then K DMAs (hot) ----
    {
      float v, r;
      asm volatile(
          "v_mov_b32 %[v], -1.0\n\t"
          "global_load_dword %[v], %[ca], off\n\t"
          "s_nop 0\n\t"
          ".rept 8\n\t"
          "global_load_lds_dwordx4 %[ha], off\n\t"
          ".endr\n\t"
          "s_waitcnt vmcnt(8)\n\t"
          "v_mov_b32 %[r], %[v]\n\t"
          "s_waitcnt vmcnt(0)"
          : [v] "=&v"(v), [r] "=&v"(r)
          : [l] "{m0}"(__builtin_amdgcn_readfirstlane(lds0 + 1024)), [ca] "v"(c + 2048 + lane), [ha] "v"(hot + 4 * lane)
          : "memory");
      if (r != c[2048 + lane]) ++fb;
    }
    __syncthreads();
    // ---- C: load (cold) then K stores (hot) ----
    {
      float v, r;
      asm volatile(
          "v_mov_b32 %[v], -1.0\n\t"
          "global_load_dword %[v], %[ca], off\n\t"
          ".rept 8\n\t"
          "global_store_dword %[ha], %[s], off sc1\n\t"
          ".endr\n\t"
          "s_waitcnt vmcnt(8)\n\t"
          "v_mov_b32 %[r], %[v]\n\t"
          "s_waitcnt vmcnt(0)"
          : [v] "=&v"(v), [r] "=&v"(r)
          : [ca] "v"(c + 4096 + lane), [ha] "v"(hot + 4096 + lane), [s] "v"((float)lane)
          : "memory");
      if (r != c[4096 + lane]) ++fc;
    }
    __syncthreads();
    // ---- D: DMA (cold) then K stores (hot) ----
    for (int i = lane; i < 64 * 4; i += 64) lds[i] = -1.0f;
    __syncthreads();
    {
      float v;
      asm volatile(
          "s_nop 0\n\t"
          "global_load_lds_dwordx4 %[ca], off\n\t"
          ".rept 8\n\t"
          "global_store_dword %[ha], %[s], off sc1\n\t"
          ".endr\n\t"
          "s_waitcnt vmcnt(8)\n\t"
          "ds_read_b32 %[v], %[la]\n\t"
          "s_waitcnt vmcnt(0) lgkmcnt(0)"
          : [v] "=&v"(v)
          : [l] "{m0}"(__builtin_amdgcn_readfirstlane(lds0)), [ca] "v"(c + 6144 + 4 * lane), [ha] "v"(hot + 8192 + lane),
            [s] "v"((float)lane), [la] "v"(lds0 + 16 * lane)
          : "memory");
      if (v != c[6144 + 4 * lane]) ++fd;
    }
    __syncthreads();
  }
  atomicAdd(&fails[0], fa);
  atomicAdd(&fails[1], fb);
  atomicAdd(&fails[2], fc);
  atomicAdd(&fails[3], fd);
}

__global__ void k_fill(float* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (float)(i % 100003) + 0.5f;
}

int main() {
  const int nwg = 1024;
  const size_t stride_f = 8192;  // 32 KiB between reps: every test reads lines nothing has touched
  const size_t n = (size_t)nwg * REPS * stride_f + 4096;
  float *cold, *hot;
  int* fails;
  if (hipMalloc(&cold, n * 4) != hipSuccess || hipMalloc(&hot, 65536 * 4) != hipSuccess || hipMalloc(&fails, 64) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, cold, n);
  hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, 0, hot, (size_t)65536);
  (void)hipMemset(fails, 0, 64);
  (void)hipDeviceSynchronize();
  // flush caches from the fill: a large unrelated pass
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, cold + n / 2, n / 2 - 4096);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(k_order, dim3(nwg), dim3(64), 0, 0, cold, hot, fails, stride_f);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, cold + n / 2, n / 2 - 4096);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(k_order_buf, dim3(nwg), dim3(64), 0, 0, cold, hot, fails, stride_f);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 1;
  }
  int f[16];
  (void)hipMemcpy(f, fails, 64, hipMemcpyDeviceToHost);
  const long tot = (long)nwg * REPS * 64;
  printf("lane-tests per case %ld (vmcnt(%d) with %d younger ops of another class):\n", tot, K, K);
  printf("  A  DMA(cold)  then loads(hot):  DMA not landed   %d\n", f[0]);
  printf("  B  load(cold) then DMAs(hot):   load not landed  %d\n", f[1]);
  printf("  C  load(cold) then stores(hot): load not landed  %d\n", f[2]);
  printf("  D  DMA(cold)  then stores(hot): DMA not landed   %d\n", f[3]);
  printf("buffer (MUBUF) loads / stores beside global_load_lds:\n");
  printf("  A  DMA(cold)  then buffer loads(hot):   DMA not landed   %d\n", f[4]);
  printf("  B  buffer load(cold) then DMAs(hot):    load not landed  %d\n", f[5]);
  printf("  C  buffer load(cold) then buffer stores: load not landed %d\n", f[6]);
  printf("  D  DMA(cold)  then buffer stores(hot):  DMA not landed   %d\n", f[7]);
  printf("  E  buffer load(cold) then buffer loads:  load not landed %d\n", f[8]);
  printf("  F  DMA(cold) then null-resource buffer loads:  DMA not landed %d\n", f[9]);
  printf("  G  DMA(cold) then null-resource buffer stores: DMA not landed %d\n", f[10]);
  return 0;
}
