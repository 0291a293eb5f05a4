// MI355X tiled-QR engine: wave-batched kernels over the static DAG plan, plans, C ABI.
//
// Execution model (DESIGN.md "Engine"): the host scheduler (sched.c) turns the reference DAG
// (src/gridscheduler.c) into BFS waves; every wave is two launches on two HIP streams —
//   * panel kernel:  one 256-thread workgroup per GEQRT / TSQRT task (critical path),
//   * update kernel: one 256-thread workgroup per 64-column strip of every UNMQR / TSMQR
//     task of the wave (the bulk of the flops),
// joined by events before the next wave. Tasks inside a wave are independent by
// construction, so no intra-launch synchronisation is needed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <thread>
#include <mutex>
#include <string>
#include <new>
#include <tuple>
#include <vector>

#include "gridscheduler.h"
#include "tiles.hpp"
#include "tqr.h"

namespace tqr {

// item = {type | strip << 8, l, m, k}  (reference Task fields, gridscheduler.h:13-17)
struct Item {
  int ts, l, m, k;
};

struct Args {
  void* A;        // matrix (S*)
  void* tau;      // compact tau (S*), m x kmax
  double* Tw;     // T factors: [(k*p + i)*NG + g][IB*IB]
  const Item* items;
  long ldm;
  int m, p, kmax;
};

#ifdef TQR_STAMPS
// Diagnostic build only (make stamps): per-phase cycle sums of the panel kernel's TSQRT tasks.
__device__ unsigned long long g_stamps[8];
__device__ unsigned long long g_pstamps[8];
#define STAMP_INIT unsigned long long st_last = __builtin_amdgcn_s_memrealtime();
#define STAMP(i)                                                          \
  do {                                                                    \
    if (threadIdx.x == 0) {                                               \
      unsigned long long now_ = __builtin_amdgcn_s_memrealtime();             \
      atomicAdd(&g_stamps[i], now_ - st_last);                            \
      st_last = now_;                                                     \
    }                                                                     \
  } while (0)
#else
#define STAMP_INIT
#define STAMP(i) do {} while (0)
#endif

#ifdef TQR_FLOW_STAMPS
__device__ unsigned long long g_fst[4096 * 24];  // >= FST_N categories per workgroup
__device__ unsigned long long g_ttl[3 << 18];     // task timeline (first 2^18 tasks)
__device__ unsigned long long g_wst[4096 * 64];   // per-wave activity sums (flow.hpp WSL slots x 8 waves)
__device__ unsigned long long g_gtr[4096 * 8 * 8];  // group trace of workgroup 0 (flow.hpp GTR)
__device__ unsigned long long g_xtr[4096 * 8 * 8];  // its hand-over phase-2 marks (flow.hpp XPipe)
#endif
}  // namespace tqr
#include "flow.hpp"
namespace tqr {
static_assert(FST_N <= 24, "g_fst holds 24 categories per workgroup");
static_assert(Geo<256>::TPIMG == 1024 && Geo<16>::TPIMG == 256 && Geo<256, 16>::TPIMG == 256 &&
                  Geo<256, 16>::VIMG == 4608 && Geo<64, 16>::VIMG == 1152,
              "host tpimg_doubles / vimg_doubles mirror Geo::TPIMG / VIMG");
static_assert(Img<256, float>::V == 4096 && Img<256, float>::T == 384 && Img<16, float>::V == 128 && Img<16, float>::T == 128 &&
                  Img<64, float>::V == 1024 && Img<64, float>::T == 384,
              "host wk_bytes mirrors Img<B, float>");
static_assert(Geo<256>::TPK <= Geo<256>::TSZ && Geo<16>::TPK <= Geo<16>::TSZ, "packed T fits the Gram buffer");

template <int B>
__device__ __forceinline__ double* tw_ptr(const Args& a, int i, int k, int g) {
  using G = Geo<B>;
  return a.Tw + (((size_t)k * a.p + i) * G::NG + g) * G::TIMG;
}

// ---------------------------------------------------------------------------------------
// Panel kernel: GEQRT (QRS) and TSQRT (QRD) tasks, one workgroup each.
// ---------------------------------------------------------------------------------------
template <int B, typename S>
__global__ __launch_bounds__(NT, 1) void k_panel(Args a) {
  using G = Geo<B>;
  constexpr int IB = G::IB, VP = G::VP, TP = G::TP, NG = G::NG;
  extern __shared__ __align__(16) double lds[];
  double* Vs = lds;
  double* Hs = Vs + G::VSZ;
  double* Ts = Hs + G::TSZ;
  double* Gs = Ts + G::TSZ;
  double* tauv = Gs + G::TSZ;
  double* scratch = tauv + IB + 2;
  double* Gp = scratch + 2 * 4 * 32 + 4 * 32 + 2 * 32 + G::TSZ;  // 4 partial Grams

  const Item it = a.items[blockIdx.x];
  const int type = it.ts & 0xff, l = it.l, k = it.k;
  S* A = (S*)a.A;
  S* tau = (S*)a.tau;
  const size_t ldm = a.ldm;
  const int t = threadIdx.x, w = t >> 6;
  S* Rt = A + (size_t)k * B * ldm + (size_t)k * B;  // tile (k,k)
  double X[G::NKS];
  double H[G::NRI];

  if (type == QRS) {
    for (int g = 0; g < NG; ++g) {
      const int c0 = g * IB, ks0 = c0 / 4;
#pragma unroll 8
      for (int idx = t; idx < B * IB; idx += NT) {
        int r = idx % B, c = idx / B;
        Vs[r * VP + G::pc(c)] = r >= c0 ? ld(Rt + (size_t)(c0 + c) * ldm + r) : 0.0;
      }
      __syncthreads();
      panel_factor<B, false>(Vs, Hs, tauv, scratch, c0);
      // write back R / V of the panel, taus; then make V explicit (0 above, 1 on the diagonal)
      for (int idx = t; idx < B * IB; idx += NT) {
        int r = idx % B, c = idx / B, d = c0 + c;
        double v = Vs[r * VP + G::pc(c)];
        if (r >= c0) st(Rt + (size_t)d * ldm + r, v);
      }
      if (t < IB) st(tau + (size_t)k * a.m + (size_t)k * B + c0 + t, tauv[t]);
      __syncthreads();
      for (int idx = t; idx < B * IB; idx += NT) {
        int r = idx % B, c = idx / B, d = c0 + c;
        if (r <= d) Vs[r * VP + G::pc(c)] = r == d ? 1.0 : 0.0;
      }
      __syncthreads();
      build_t<B>(Vs, tauv, Gs, Ts, Gp, ks0);
      double* tg = tw_ptr<B>(a, k, k, g);
      for (int idx = t; idx < G::TSZ; idx += NT) tg[idx] = Ts[idx];
      // trailing columns of the tile
      const int nstr = (B - c0 - IB) / 16;
      for (int s = w; s < nstr; s += NT / 64) {
        asm volatile("" ::: "memory");  // keep the V-image reads inside the loop (no LICM of ~1k LDS loads)
        const int col = c0 + IB + 16 * s;
        load_strip<B>(X, Rt, ldm, col, ks0);
        apply_group<B, false>(Vs, Ts, X, H, ks0);
        store_strip<B>(X, Rt, ldm, col, ks0);
      }
      __syncthreads();
    }
  } else {  // QRD: TSQRT of [R_kk ; tile (l,k)]
    S* Bt = A + (size_t)k * B * ldm + (size_t)l * B;
    STAMP_INIT
    for (int g = 0; g < NG; ++g) {
      const int c0 = g * IB;
#pragma unroll 8
      for (int idx = t; idx < B * IB; idx += NT) {
        int r = idx % B, c = idx / B;
        Vs[r * VP + G::pc(c)] = ld(Bt + (size_t)(c0 + c) * ldm + r);
      }
      for (int idx = t; idx < IB * IB; idx += NT) {
        int r = idx % IB, c = idx / IB;
        if (r <= c) Hs[r * TP + c] = ld(Rt + (size_t)(c0 + c) * ldm + c0 + r);
      }
      __syncthreads();
      STAMP(0);
      panel_factor<B, true>(Vs, Hs, tauv, scratch, c0);
      STAMP(1);
      for (int idx = t; idx < B * IB; idx += NT) {
        int r = idx % B, c = idx / B;
        st(Bt + (size_t)(c0 + c) * ldm + r, Vs[r * VP + G::pc(c)]);
      }
      for (int idx = t; idx < IB * IB; idx += NT) {
        int r = idx % IB, c = idx / IB;
        if (r <= c) st(Rt + (size_t)(c0 + c) * ldm + c0 + r, Hs[r * TP + c]);
      }
      if (t < IB) st(tau + (size_t)k * a.m + (size_t)l * B + c0 + t, tauv[t]);
      __syncthreads();
      STAMP(2);
      build_t<B>(Vs, tauv, Gs, Ts, Gp, 0);
      STAMP(3);
      double* tg = tw_ptr<B>(a, l, k, g);
      for (int idx = t; idx < G::TSZ; idx += NT) tg[idx] = Ts[idx];
      const int nstr = (B - c0 - IB) / 16;
      for (int s = w; s < nstr; s += NT / 64) {
        asm volatile("" ::: "memory");  // keep the V-image reads inside the loop (no LICM of ~1k LDS loads)
        const int col = c0 + IB + 16 * s;
        load_strip<B>(X, Bt, ldm, col, 0);
        load_head<B>(H, Rt, ldm, c0, col);
        apply_group<B, true>(Vs, Ts, X, H, 0);
        store_strip<B>(X, Bt, ldm, col, 0);
        store_head<B>(H, Rt, ldm, c0, col);
      }
      __syncthreads();
      STAMP(4);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Update kernel: UNMQR (SAPP) and TSMQR (DAPP) on one 64-column strip, one workgroup each;
// wave w owns columns strip*64 + 16w .. +15 of the target tile(s).
// ---------------------------------------------------------------------------------------
template <int B, typename S>
__global__ __launch_bounds__(NT, 2) void k_update(Args a) {
  using G = Geo<B>;
  constexpr int IB = G::IB, NG = G::NG;
  extern __shared__ __align__(16) double lds[];
  double* Vs = lds;
  double* Ts = Vs + G::VSZ;

  const Item it = a.items[blockIdx.x];
  const int type = it.ts & 0xff, strip = it.ts >> 8, l = it.l, j = it.m, k = it.k;
  S* A = (S*)a.A;
  const size_t ldm = a.ldm;
  const int w = threadIdx.x >> 6;
  const int col = strip * 64 + 16 * w;  // strip column inside the tile
  const bool active = col < B;
  double X[G::NKS];
  double H[G::NRI];

  if (type == DAPP) {
    const S* Vt = A + (size_t)k * B * ldm + (size_t)l * B;  // tile (l,k): V_B
    S* At = A + (size_t)j * B * ldm + (size_t)k * B;        // tile (k,j): head rows
    S* Bt = A + (size_t)j * B * ldm + (size_t)l * B;        // tile (l,j)
    if (active) load_strip<B>(X, Bt, ldm, col, 0);
    for (int g = 0; g < NG; ++g) {
      __syncthreads();
      stage_v_ts<B>(Vs, Vt, ldm, g * IB);
      stage_t<B>(Ts, tw_ptr<B>(a, l, k, g));
      __syncthreads();
      if (active) {
        load_head<B>(H, At, ldm, g * IB, col);
        apply_group<B, true>(Vs, Ts, X, H, 0);
        store_head<B>(H, At, ldm, g * IB, col);
      }
    }
    if (active) store_strip<B>(X, Bt, ldm, col, 0);
  } else {  // SAPP
    const S* Vt = A + (size_t)k * B * ldm + (size_t)k * B;  // tile (k,k)
    S* Ct = A + (size_t)j * B * ldm + (size_t)k * B;        // tile (k,j)
    if (active) load_strip<B>(X, Ct, ldm, col, 0);
    for (int g = 0; g < NG; ++g) {
      __syncthreads();
      stage_v_ge<B>(Vs, Vt, ldm, g * IB);
      stage_t<B>(Ts, tw_ptr<B>(a, k, k, g));
      __syncthreads();
      if (active) apply_group<B, false>(Vs, Ts, X, H, g * IB / 4);
    }
    if (active) store_strip<B>(X, Ct, ldm, col, 0);
  }
}

// T factors from a stored V and tau (for the single-tile API, where the caller hands over V
// and tau as the reference's SLARFT/SSSRFT take them). One workgroup per (item, group).
template <int B, typename S>
__global__ __launch_bounds__(NT, 1) void k_build_t(Args a) {
  using G = Geo<B>;
  constexpr int IB = G::IB, NG = G::NG;
  extern __shared__ __align__(16) double lds[];
  double* Vs = lds;
  double* Ts = Vs + G::VSZ;
  double* Gs = Ts + G::TSZ;
  double* tauv = Gs + G::TSZ;
  double* Gp = tauv + IB + 2;
  const Item it = a.items[blockIdx.x / NG];
  const int g = blockIdx.x % NG, c0 = g * IB, type = it.ts & 0xff, l = it.l, k = it.k;
  const S* A = (const S*)a.A;
  const S* tau = (const S*)a.tau;
  const size_t ldm = a.ldm;
  const int row0 = type == QRS ? k * B : l * B;
  if (type == QRS) stage_v_ge<B>(Vs, A + (size_t)k * B * ldm + (size_t)k * B, ldm, c0);
  else stage_v_ts<B>(Vs, A + (size_t)k * B * ldm + (size_t)l * B, ldm, c0);
  if (threadIdx.x < IB) tauv[threadIdx.x] = ld(tau + (size_t)k * a.m + row0 + c0 + threadIdx.x);
  __syncthreads();
  build_t<B>(Vs, tauv, Gs, Ts, Gp, type == QRS ? c0 / 4 : 0);
  double* tg = tw_ptr<B>(a, type == QRS ? k : l, k, g);
  for (int idx = threadIdx.x; idx < G::TSZ; idx += NT) tg[idx] = Ts[idx];
}

// RANDZO-distributed synthetic input: ((h mod 201) - 100) / 100 from a splitmix64 hash.
// col0: the first column's index in the global matrix (the value of element (i, j) depends only on
// the seed and its global position, so a rank can fill just its own columns)
template <typename S>
__global__ void k_randzo(S* A, int m, int n, long ldm, unsigned long long seed, long col0) {
  long total = (long)m * n;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long jj = e / m, ii = e % m;
    const unsigned long long eg = (unsigned long long)(e + col0 * m);  // global element index
    unsigned long long z = seed * 0x9E3779B97F4A7C15ull + eg + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    A[jj * ldm + ii] = (S)(((double)(long)(z % 201ull) - 100.0) / 100.0);
  }
}

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------
static size_t lds_panel(int b) {
  int ib = b < 32 ? b : 32;
  size_t d = (size_t)b * (ib + 2) + 8 * (size_t)ib * (ib + 1) + (ib + 2) + 2 * 4 * 32 + 4 * 32 + 2 * 32;
  return d * sizeof(double);
}
static size_t lds_update(int b) {
  int ib = b < 32 ? b : 32;
  return ((size_t)b * (ib + 2) + (size_t)ib * (ib + 1)) * sizeof(double);
}

typedef void (*kfn)(Args);
template <int B, typename S>
static void get_kernels(kfn* p, kfn* u, kfn* t) {
  *p = k_panel<B, S>;
  *u = k_update<B, S>;
  *t = k_build_t<B, S>;
}
typedef void (*ffn)(FlowArgs);
// Engine shape of the persistent kernel (flow.hpp FlowShape): 8 = ShapeW8 (one 8-wave workgroup per
// CU, 128-column strips, 32-reflector groups; the default), 4 = ShapeW4 (two 4-wave workgroups per
// CU, 64-column strips, 16-reflector groups; fp64 with TQR_FLOW_SHAPE=w4)
struct ShapeInfo {
  int nw, nt, sw, ib, wpc;
};
static ShapeInfo shape_info(int shape) {
  return shape == 4   ? ShapeInfo{ShapeW4::NW, ShapeW4::NT, ShapeW4::SW, ShapeW4::IB, ShapeW4::WPC}
         : shape == 5 ? ShapeInfo{ShapeR::NW, ShapeR::NT, ShapeR::SW, ShapeR::IB, ShapeR::WPC}
                      : ShapeInfo{ShapeW8::NW, ShapeW8::NT, ShapeW8::SW, ShapeW8::IB, ShapeW8::WPC};
}
// fp64 default: ShapeW8 — ShapeW4 measured 138.6-139.0 vs 126.7-126.9 ms at 16384^2 (two alternating
// A/B rounds on one box, profiles/r04/shape_ab); TQR_FLOW_SHAPE=w4 selects it
// 5 = ShapeR (chain_res.hpp: one 4-wave workgroup per CU, one wave per SIMD with the whole register
// file, 64-column strips double-buffered in AGPRs, the head strip resident; fp64, b = 256;
// TQR_FLOW_SHAPE=r)
static int flow_shape(int dtype, int b) {
  if (dtype != TQR_F64) return 8;
  const char* e = getenv("TQR_FLOW_SHAPE");
  if (e && strcmp(e, "w4") == 0) return 4;
  if (e && strcmp(e, "r") == 0 && b == 256) return 5;
  return 8;
}
static int shape_ib(int shape, int b) { return std::min(b, shape_info(shape).ib); }
static int shape_ns(int shape, int b) { const int sw = shape_info(shape).sw; return (b + sw - 1) / sw; }
template <int B, typename S, class C>
static ffn get_flow() { return k_flow<B, S, C>; }
template <int B>
static ffn get_flow_res() {
  if constexpr (B == 256) return k_flow<256, double, ShapeR>;
  else return nullptr;
}
template <int B>
static int lds_res() {
  if constexpr (B == 256) return flow_lds_doubles<256, double, ShapeR>();
  else return 0;
}
static size_t lds_flow(int b, int dtype, int shape) {
  int d = 0;
#define TQR_L(BB)                                                                                  \
  case BB:                                                                                         \
    d = dtype != TQR_F64 ? flow_lds_doubles<BB, float, ShapeW8>()                                  \
        : shape == 4     ? flow_lds_doubles<BB, double, ShapeW4>()                                 \
        : shape == 5     ? lds_res<BB>()                                                           \
                         : flow_lds_doubles<BB, double, ShapeW8>();                                \
    break;
  switch (b) { TQR_L(16) TQR_L(32) TQR_L(64) TQR_L(128) TQR_L(256) }
#undef TQR_L
  return (size_t)d * sizeof(double) + 1536;  // + task index, sync-point verdicts, Rc view, FST sums, wave sums
}
static ffn resolve_flow(int b, int dtype, int shape) {
  ffn f = nullptr;
#define TQR_F(BB)                                                                                  \
  case BB:                                                                                         \
    f = dtype != TQR_F64 ? get_flow<BB, float, ShapeW8>()                                          \
        : shape == 4     ? get_flow<BB, double, ShapeW4>()                                         \
        : shape == 5     ? get_flow_res<BB>()                                                      \
                         : get_flow<BB, double, ShapeW8>();                                        \
    break;
  switch (b) { TQR_F(16) TQR_F(32) TQR_F(64) TQR_F(128) TQR_F(256) }
#undef TQR_F
  if (f && hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_flow(b, dtype, shape)) !=
               hipSuccess)
    return nullptr;
  return f;
}

// ---------------------------------------------------------------------------------------
// Flow task list: panel tasks P(i,k) (i == k: GEQRT) and chain segments C(k,j,s,e), ordered
// by an as-soon-as-possible start-time estimate of the pipelined DAG (unit = one chain
// element), then checked to be topological (else the always-valid step-major order is used).
// ---------------------------------------------------------------------------------------
struct FlowPlan {
  std::vector<Item> items;
  bool est_order = false;
};

// Is a flow task list topological for the engine's in-task waits? Every task must come after
// every task it waits on (in-order dequeue then guarantees progress, flow.hpp header):
//   panel (i,k):        panel (i-1,k); the chain segments of step k-1, column k, holding row i;
//   chain (k,j,s,e):    segment e-1 (head rows) or, for e = 0, GEQRT(k) and the step-(k-1)
//                       segment holding row k; for each of its rows i: panel (i,k) and the
//                       step-(k-1) segment holding row i.
// Segment boundaries are read from the list itself (any segment lengths).
// Host-pointer API lists (xfer.hpp) also hold UP(j, c) / DOWN(j, c): every step-0 task of tile
// column j (GEQRT(0) / TSQRT(i, 0) for j = 0, the chains of step 0 on j) must come after all
// UP(j, *); DOWN(j, c) after every chain of a step k < j on column j and every panel task of step j.
static bool flow_list_topological(const std::vector<Item>& L, int p, int q, int ns) {
  std::map<std::pair<int, int>, int> ppos;                       // (i, k) -> position
  std::map<std::tuple<int, int, int, int>, int> cpos;            // (k, j, s, e) -> position
  std::map<std::tuple<int, int, int, int>, int> rowpos;          // (k, j, s, row) -> position
  std::map<std::pair<int, int>, int> upos, dpos;                 // (j, c) -> position
  std::vector<int> uplast(q, -1);                                // last UP(j, *) of column j
  std::vector<int> collast(q, -1);                               // last task DOWN(j, *) waits for
  for (int x = 0; x < (int)L.size(); ++x) {
    const Item& it = L[x];
    const int ty = it.ts & 0xff;
    if (ty == T_CHAIN) {
      const int s = (it.ts >> 8) & 0xff, k = it.k & 0xffff, e = it.k >> 16, j = it.m, i0 = it.l & 0xffff, i1 = it.l >> 16;
      if (j < 0 || j >= q) return false;
      if (!cpos.emplace(std::make_tuple(k, j, s, e), x).second) return false;
      if (e == 0) rowpos[std::make_tuple(k, j, s, k)] = x;
      for (int i = i0; i < i1; ++i) rowpos[std::make_tuple(k, j, s, i)] = x;
      if (k < j) collast[j] = std::max(collast[j], x);
    } else if (ty == QRS || ty == QRD) {
      if (it.k < 0 || it.k >= q) return false;
      if (!ppos.emplace(std::make_pair(it.l, it.k), x).second) return false;
      collast[it.k] = std::max(collast[it.k], x);
    } else if (ty == T_UP || ty == T_DOWN) {
      if (it.m < 0 || it.m >= q) return false;
      auto& mp = ty == T_UP ? upos : dpos;
      if (!mp.emplace(std::make_pair(it.m, (it.ts >> 8) & 0xff), x).second) return false;
      if (ty == T_UP) uplast[it.m] = std::max(uplast[it.m], x);
    } else {
      return false;
    }
  }
  auto before = [&](auto& mp, const auto& key, int x) {
    auto f = mp.find(key);
    return f != mp.end() && f->second < x;
  };
  const bool xfer = !upos.empty();
  if (xfer) {  // every column uploaded and downloaded by the same number of chunks
    const int nxc = (int)upos.size() / q;
    if ((int)upos.size() != nxc * q || dpos.size() != upos.size()) return false;
    for (int j = 0; j < q; ++j)
      for (int c = 0; c < nxc; ++c)
        if (!upos.count(std::make_pair(j, c)) || !dpos.count(std::make_pair(j, c))) return false;
  } else if (!dpos.empty()) {
    return false;
  }
  for (int x = 0; x < (int)L.size(); ++x) {
    const Item& it = L[x];
    const int ty = it.ts & 0xff;
    if (ty == T_CHAIN) {
      const int s = (it.ts >> 8) & 0xff, k = it.k & 0xffff, e = it.k >> 16, j = it.m, i0 = it.l & 0xffff, i1 = it.l >> 16;
      if (e > 0 && !before(cpos, std::make_tuple(k, j, s, e - 1), x)) return false;
      if (e == 0 && !before(ppos, std::make_pair(k, k), x)) return false;
      if (e == 0 && k > 0 && !before(rowpos, std::make_tuple(k - 1, j, s, k), x)) return false;
      if (xfer && k == 0 && !(uplast[j] < x)) return false;
      for (int i = i0; i < i1; ++i) {
        if (!before(ppos, std::make_pair(i, k), x)) return false;
        if (k > 0 && !before(rowpos, std::make_tuple(k - 1, j, s, i), x)) return false;
      }
    } else if (ty == T_DOWN) {
      if (!(collast[it.m] < x)) return false;
    } else if (ty == QRS || ty == QRD) {
      const int i = it.l, k = it.k;
      if (i > k && !before(ppos, std::make_pair(i - 1, k), x)) return false;
      if (xfer && k == 0 && !(uplast[0] < x)) return false;
      if (k > 0)
        for (int s = 0; s < ns; ++s)
          if (!before(rowpos, std::make_tuple(k - 1, k, s, i), x)) return false;
    }
  }
  (void)p;
  return true;
}

// Host-pointer API: the persistent launch also carries the transfers (xfer.hpp). nxc chunks per
// tile column; tcol = one column's upload time in the estimator's unit (a chain element).
struct XferPlan {
  int nxc = 0;
  double tcol = 0.0;
};

// Order knobs of the flow task list, read from the environment ONCE per plan (plan_create) and
// kept with it: the host-API task list (plan_xfer_list, built at the first host call) and the
// device's column-final counts (xfer.hpp, from FlowArgs) must see the same segment lengths as the
// plan's own list, whatever the environment says later.
//   seglen     chain segment length (TQR_SEGLEN, default 8)
//   seglen_la  the lookahead column's (j = k+1, the DAG's critical path: its chain elements feed
//              the next panel's members; TQR_SEGLEN_LA, default seglen)
//   la_tail    the last la_tail steps (TQR_LA_TAIL): their lookahead column runs one element per
//              segment, so the element that finishes the next diagonal tile runs beside the UNMQR
//              element instead of behind it
//   tail       the last `tail` steps (TQR_TAIL; default: default_tail): every chain tail_sl elements
//              per segment (TQR_TAIL_SEGLEN, default 1)
//   ualone     the last ualone steps (TQR_UNMQR_ALONE; default: tail): the lookahead column's UNMQR
//              element alone in segment 0 (flow.hpp unmqr_alone)
//   Tg         the estimator's panel group-step cost in chain elements (TQR_TG, default 1.4)
//   lazy       TQR_LAZY (default 1), la / lac: TQR_LA (default: default_la) / TQR_LAC (see
//              build_flow_plan)
struct FlowKnobs {
  int seglen = 8, seglen_la = 8, la_tail = 0, tail = 0, tail_sl = 1, ualone = 0;
  double Tg = 1.4, lazy = 1.0, la = 0.0, lac = 0.0;
};
// Default tail (fp64 storage): the steps whose columns have at most kTailRows rows below the
// diagonal, i.e. whose chains are short and on the critical path. One element per segment lets a
// column's elements run on different workgroups, pipelined group by group through the head rows
// (Ac), instead of one after the other in one workgroup. Measured at 16384^2 (64 steps): tail 32
// 122.7-122.8 ms against 124.7-124.9 (24: 124.0, 40: 122.9-123.3, 48: 124.2-124.3; profiles/r04/
// tail/). fp32 storage keeps its head strip in registers across a segment, so one-element segments
// add a head load and store per element there: no gain at 16-32 steps of 128, slower beyond
// (48: +2.3 ms) — off for fp32. Tall matrices (65536 x 16384) never reach the tail rows.
constexpr int kTailRows = 31;
static int default_tail(int p, int q, int dtype) {
  const int kmax = std::min(p, q);
  if (dtype != TQR_F64) return 0;
  return std::max(0, std::min(kmax, kmax - (p - 1 - kTailRows)));
}
// Default panel lookahead (TQR_LA, chain elements): 2 for fp32 storage, whose run is paced by the
// panel groups (c5 465.8-466.4 vs 467.2-467.3 ms, two alternating rounds; 4: 466.2-466.5, 6:
// 467.7; round 4's earlier 4 vs 0: 469.0-469.1 vs 470.4-470.7), 0 for fp64 (2: +0.1-0.2 ms;
// profiles/r04/la_f32/).
static double default_la(int dtype) { return dtype == TQR_F32 ? 2.0 : 0.0; }
// Multi-rank defaults (4+ ranks, each launch covering its whole device — the plans of the 8-GPU
// run): besides 2-element segments (env_seglen), one-element segments in the last 7/16 of the steps
// (28 of 64 at 65536x16384) and the lookahead column's chains keyed 4 elements earlier. The model
// with round-5 chain costs (tools/sched_sim.py dist5): S(8) 6.41 against 6.16 with
// 2-element segments alone (tail 24 / 32: 6.35 / 6.39 with the keying, 6.38 at 32 without).
// Round 6 calibrated the model against the one-GPU rehearsals (tools/sched_sim.py calib,
// profiles/r06/model): measured / model 1.032-1.053 for 2 and 4 ranks; with that error the 8-GPU
// time is 92.0-93.9 ms with these defaults against 95.6-97.6 ms with 2-element segments alone
// (S(8) 6.19-6.32 vs 5.96-6.08), and the 4-rank rehearsal with these lists forced was predicted
// slower (602.8 vs 572.0 ms model) and measured slower (621.8 vs 602.1 ms) — the model carries the
// direction of the one-GPU cost; its 8-GPU gain (3.8 %) is a scale-free comparison of two lists
// under the same error. The lone UNMQR segments do not follow the tail on these plans (the model:
// no difference at 8 ranks, 89.2 ms either way): one-GPU plans only. TQR_DIST_DEFAULTS=r4 keeps the
// round-4 list (2-element segments only) for an A/B on an 8-GPU node.
struct MultiRankDefaults {
  int tail;
  double lac;   // < 0: the panel keying (TQR_LA's default)
  int ualone;   // < 0: follow the tail
};
static MultiRankDefaults multi_rank_defaults(int p, int q, int dtype, int world, bool full) {
  const int kmax = std::min(p, q);
  const char* e = getenv("TQR_DIST_DEFAULTS");
  const bool r4 = e && std::string(e) == "r4";
  if (world >= 4 && full && !r4) return {std::max(default_tail(p, q, dtype), 7 * kmax / 16), 4.0, 0};
  if (world > 1) return {default_tail(p, q, dtype), -1.0, 0};
  return {default_tail(p, q, dtype), -1.0, -1};
}
static FlowKnobs knobs_from_env(int seglen, int tail_default = 0, double la_default = 0.0, double lac_default = -1.0,
                                int ualone_default = -1) {
  FlowKnobs kn;
  kn.seglen = std::max(1, seglen);
  kn.tail = tail_default;
  kn.la = la_default;
  const char* esl = getenv("TQR_SEGLEN_LA");
  kn.seglen_la = esl ? std::max(1, atoi(esl)) : kn.seglen;
  const char* e = getenv("TQR_LA_TAIL");
  kn.la_tail = e ? std::max(0, atoi(e)) : 0;
  if (const char* et = getenv("TQR_TAIL")) kn.tail = std::max(0, atoi(et));
  if (const char* ets = getenv("TQR_TAIL_SEGLEN")) kn.tail_sl = std::max(1, atoi(ets));
  kn.ualone = ualone_default >= 0 ? ualone_default : kn.tail;
  if (const char* eua = getenv("TQR_UNMQR_ALONE")) kn.ualone = std::max(0, atoi(eua));
  if (const char* eg = getenv("TQR_TG")) kn.Tg = atof(eg);
  if (const char* el = getenv("TQR_LAZY")) kn.lazy = atof(el);
  if (const char* ela = getenv("TQR_LA")) kn.la = atof(ela);
  kn.lac = lac_default >= 0.0 ? lac_default : kn.la;
  if (const char* elac = getenv("TQR_LAC")) kn.lac = atof(elac);  // lookahead column's chains (default: TQR_LA)
  return kn;
}
// Chain segment length (elements per chain task; TQR_SEGLEN overrides). 8, except for 4 and more
// ranks with a whole device each (1024+ workgroups in all): 2 — more, shorter chain tasks give
// each rank work it can start while its columns' wavefronts (the head rows going down a column)
// wait on other ranks' panels. The model of the 8-GPU run (tools/sched_sim_seglen.py, per-segment
// cost calibrated on one MI355X) gives S(8) 6.17 at length 2 against 5.44 at 8; one GPU pays
// 4.6 % for length 2 (65536x16384: 635.3 vs 607.6 ms), and so do the one-GPU rehearsals (4 ranks
// x 64 CUs: 645.8 vs 628.8 ms; model 600.5 vs 575.1), whose ranks have work to spare.
// full: the rank's launch covers its whole device (every rank must decide alike — tqr_dist_import
// checks the ranks' task-list signatures).
static int env_seglen(int world = 1, bool full = true) {
  const char* sl = getenv("TQR_SEGLEN");
  return sl ? std::max(1, atoi(sl)) : (world >= 4 && full ? 2 : 8);
}

// ns: chain strips per tile column, ng: reflector groups per tile (the engine shape's, shape_ns /
// b / shape_ib)
static void build_flow_plan(int p, int q, int ns, int ng, const FlowKnobs& kn, FlowPlan& fp, const XferPlan* xp = nullptr) {
  const int kmax = std::min(p, q);
  // segment length per chain: shorter segments for the lookahead column pipeline consecutive
  // elements on different workgroups at reflector-group granularity
  auto seglen_of = [&](int k, int j) { return seglen_of_chain(k, j, kmax, kn.seglen, kn.seglen_la, kn.la_tail, kn.tail, kn.tail_sl); };
  // host-pointer API: tile column j arrives (uploaded) at arrive(j); step-0 tasks start after it
  const bool xfer = xp && xp->nxc > 0;
  auto arrive = [&](int j) { return xfer ? (j + 1) * xp->tcol : 0.0; };
  // cost model (unit: one chain element): Tg = one panel group-step; tunable for experiments
  const double Tg = kn.Tg, Te = 1.0;
  const double lazy = kn.lazy;
  // lookahead (TQR_LA / TQR_LAC, unit: chain elements): panel tasks / the lookahead column's
  // chains are keyed this much earlier than their estimate (the critical path first)
  const double la = kn.la;
  const double lac = kn.lac;
  // fin_elem[k][i][j] (strips move together in the estimate): finish of chain element (i,j,k)
  auto id3 = [&](int k, int i, int j) { return ((size_t)k * p + i) * q + j; };
  std::vector<double> fin((size_t)kmax * p * q, 0.0), pstart((size_t)kmax * p, 0.0);
  auto fin_prev = [&](int k, int i, int j) { return k > 0 ? fin[id3(k - 1, i, j)] : 0.0; };
  struct T { double est; int ord; Item it; };
  std::vector<T> tl;
  if (xfer)  // uploads, in column order (one column's chunks together: they share the link)
    for (int j = 0; j < q; ++j)
      for (int c = 0; c < xp->nxc; ++c) tl.push_back({arrive(j) - xp->tcol, -1, Item{T_UP | (c << 8), 0, j, 0}});
  for (int k = 0; k < kmax; ++k) {
    // panel
    double ps = std::max(fin_prev(k, k, k), k == 0 ? arrive(0) : 0.0);
    pstart[(size_t)k * p + k] = ps;
    tl.push_back({ps - la, 0, Item{QRS, k, k, k}});
    for (int i = k + 1; i < p; ++i) {
      double st = std::max(fin_prev(k, i, k), pstart[(size_t)k * p + i - 1] + Tg);
      pstart[(size_t)k * p + i] = st;
      tl.push_back({st - la, 0, Item{QRD, i, k, k}});
    }
    // chains
    for (int j = k + 1; j < q; ++j) {
      double t0 = std::max({fin_prev(k, k, j), pstart[(size_t)k * p + k] + Tg, k == 0 ? arrive(j) : 0.0});
      double prev = t0 + 0.5 * Te;  // UNMQR
      fin[id3(k, k, j)] = prev;
      std::vector<double> seg_start;
      seg_start.push_back(t0);
      const int seglen = seglen_of(k, j);
      const bool ua = unmqr_alone(k, j, kmax, kn.ualone) && p - k - 1 > 0;  // segment 0: the UNMQR alone
      for (int i = k + 1; i < p; ++i) {
        double st = std::max({prev, fin_prev(k, i, j), pstart[(size_t)k * p + i] + Tg});
        if ((i - k - 1) % seglen == 0 && i > k + 1) seg_start.push_back(st);
        double f = std::max(st + Te, pstart[(size_t)k * p + i] + ng * Tg + Te / ng);
        fin[id3(k, i, j)] = f;
        prev = f;
      }
      const int nseg = nseg_of_chain(k, j, p, kmax, seglen, kn.ualone);
      if (ua) seg_start.insert(seg_start.begin(), t0);
      for (int e = 0; e < nseg; ++e) {
        const int er = ua ? e - 1 : e;  // the segment's run of rows
        int i0 = k + 1 + er * seglen, i1 = std::min(p, i0 + seglen);
        if (p - k - 1 == 0) { i0 = p; i1 = p; }
        if (er < 0) i0 = i1 = k + 1;  // (the UNMQR-only segment: no rows)
        // lazy keys (TQR_LAZY, default 1): a segment of a non-lookahead column is keyed by the
        // estimated completion of its first panel member, so a workgroup does not dequeue it
        // long before its V/T images exist (it would wait group by group); the lookahead
        // column k+1 feeds the next panel and stays eager
        double key = seg_start[std::min<size_t>(e, seg_start.size() - 1)];
        if (lazy > 0 && j != k + 1 && i0 < p) key = std::max(key, pstart[(size_t)k * p + i0] + lazy * ng * Tg);
        if (j == k + 1) key -= lac;
        for (int s = 0; s < ns; ++s)
          tl.push_back({key, 1,
                        Item{T_CHAIN | (s << 8), i0 | (i1 << 16), j, k | (e << 16)}});
      }
    }
  }
  if (xfer) {  // downloads: when tile column j is final (its last chain element, its panel)
    for (int j = 0; j < q; ++j) {
      double cf = 0.0;
      for (int k = 0; k < std::min(j, kmax); ++k) cf = std::max(cf, fin[id3(k, p - 1 > k ? p - 1 : k, j)]);
      if (j < kmax) cf = std::max(cf, pstart[(size_t)j * p + p - 1] + ng * Tg);
      for (int c = 0; c < xp->nxc; ++c) tl.push_back({cf, 2, Item{T_DOWN | (c << 8), 0, j, 0}});
    }
  }
  // bump every task's key past its dependencies' keys (tl is topological), so the
  // estimated-time order is topological by construction
  {
    std::map<std::tuple<int, int, int, int, int>, int> idx;
    for (int x = 0; x < (int)tl.size(); ++x) {
      const Item& it = tl[x].it;
      int ty = it.ts & 0xff;
      if (ty == T_CHAIN) idx[std::make_tuple(T_CHAIN, it.k & 0xffff, it.m, (it.ts >> 8) & 0xff, it.k >> 16)] = x;
      else if (ty == T_UP || ty == T_DOWN) idx[std::make_tuple(ty, it.m, (it.ts >> 8) & 0xff, 0, 0)] = x;
      else idx[std::make_tuple(0, it.l, it.k, 0, 0)] = x;
    }
    auto seg_of = [&](int k, int j, int i) { return seg_of_row(k, j, i, kmax, seglen_of(k, j), kn.ualone); };
    auto nseg_of = [&](int k, int j) { return nseg_of_chain(k, j, p, kmax, seglen_of(k, j), kn.ualone); };
    for (int x = 0; x < (int)tl.size(); ++x) {
      const Item& it = tl[x].it;
      int ty = it.ts & 0xff;
      double key = tl[x].est;
      auto bump = [&](int d) { key = std::max(key, tl[d].est + 1e-6); };
      auto bump_up = [&](int j) {
        if (xfer)
          for (int c = 0; c < xp->nxc; ++c) bump(idx[std::make_tuple(T_UP, j, c, 0, 0)]);
      };
      if (ty == T_CHAIN) {
        int s = (it.ts >> 8) & 0xff, k = it.k & 0xffff, e = it.k >> 16, j = it.m, i0 = it.l & 0xffff, i1 = it.l >> 16;
        if (e > 0) bump(idx[std::make_tuple(T_CHAIN, k, j, s, e - 1)]);
        else bump(idx[std::make_tuple(0, k, k, 0, 0)]);
        if (e == 0 && k > 0) bump(idx[std::make_tuple(T_CHAIN, k - 1, j, s, seg_of(k - 1, j, k))]);
        if (k == 0) bump_up(j);
        for (int i = i0; i < i1; ++i) {
          bump(idx[std::make_tuple(0, i, k, 0, 0)]);
          if (k > 0) bump(idx[std::make_tuple(T_CHAIN, k - 1, j, s, seg_of(k - 1, j, i))]);
        }
      } else if (ty == T_UP) {
      } else if (ty == T_DOWN) {
        const int j = it.m;
        for (int k = 0; k < std::min(j, kmax); ++k)
          for (int s = 0; s < ns; ++s)
            for (int e = 0; e < nseg_of(k, j); ++e) bump(idx[std::make_tuple(T_CHAIN, k, j, s, e)]);
        if (j < kmax)
          for (int i = j; i < p; ++i) bump(idx[std::make_tuple(0, i, j, 0, 0)]);
      } else {
        int i = it.l, k = it.k;
        if (i > k) bump(idx[std::make_tuple(0, i - 1, k, 0, 0)]);
        if (k == 0) bump_up(0);
        if (k > 0)
          for (int s = 0; s < ns; ++s) bump(idx[std::make_tuple(T_CHAIN, k - 1, k, s, seg_of(k - 1, k, i))]);
      }
      tl[x].est = key;
    }
  }
  std::vector<T> sorted = tl;
  std::stable_sort(sorted.begin(), sorted.end(), [](const T& x, const T& y) {
    if (x.est != y.est) return x.est < y.est;
    return x.ord < y.ord;
  });
  fp.items.clear();
  for (auto& t : sorted) fp.items.push_back(t.it);
  fp.est_order = flow_list_topological(fp.items, p, q, ns);
  if (!fp.est_order) {  // step-major: always topological
    fp.items.clear();
    for (auto& t : tl) fp.items.push_back(t.it);
  }
}
// Multi-GPU: keep this rank's share of the global (topological) order — panel tasks of the tile
// columns it owns (column k on rank tile_owner(k, world); each forwards its images to the peers itself) and
// the chain tasks of its own tile columns. Every rank's list is the global order restricted, so
// the earliest unfinished task of the whole job can always progress: the multi-rank engine is
// deadlock-free like the single-GPU one.
// TQR_DIST_PART=cyclic: the round-2 partition j % world (A/B diagnostics; default snake)
static int dist_cyclic() {
  const char* e = getenv("TQR_DIST_PART");
  return e && strcmp(e, "cyclic") == 0;
}
static void partition_flow_plan(FlowPlan& fp, int rank, int world) {
  const int cyc = dist_cyclic();
  std::vector<Item> mine;
  for (const Item& it : fp.items) {
    const int ty = it.ts & 0xff;
    if (ty == T_CHAIN) {
      if (tile_owner(it.m, world, cyc) == rank) mine.push_back(it);
    } else if (tile_owner(it.k, world, cyc) == rank) {  // QRS(k,k) / QRD(l,k): tile column k
      mine.push_back(it);
    }
  }
  fp.items.swap(mine);
}
static size_t lds_build_t(int b) {
  int ib = b < 32 ? b : 32;
  return ((size_t)b * (ib + 2) + 6 * (size_t)ib * (ib + 1) + ib + 2) * sizeof(double);
}
// Resolve the kernels of one (b, dtype) and raise their dynamic-LDS limits.
static int resolve(int b, int dtype, kfn* kp, kfn* ku, kfn* kt) {
#define TQR_K(BB)                                                   \
  case BB:                                                          \
    if (dtype == TQR_F64) get_kernels<BB, double>(kp, ku, kt);      \
    else get_kernels<BB, float>(kp, ku, kt);                        \
    break;
  switch (b) { TQR_K(16) TQR_K(32) TQR_K(64) TQR_K(128) TQR_K(256) default: return TQR_EINVAL; }
#undef TQR_K
  if (hipFuncSetAttribute((const void*)*kp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_panel(b)) != hipSuccess ||
      hipFuncSetAttribute((const void*)*ku, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_update(b)) != hipSuccess ||
      hipFuncSetAttribute((const void*)*kt, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_build_t(b)) != hipSuccess)
    return TQR_EHIP;
  return TQR_OK;
}

static bool valid_b(int b) { return b == 16 || b == 32 || b == 64 || b == 128 || b == 256; }
// The engine's buffer resources are based at a strip's or reflector group's first column and
// address at most 32 columns with 32-bit byte offsets (tiles.hpp load_strip_pair, flow.hpp):
// 32 * ldm * es must stay below 2^31 (ldm <= 8,388,607 rows fp64, 16,777,215 fp32).
static bool valid_ld(long ld, size_t es) { return ld > 0 && (size_t)32 * (size_t)ld * es <= 0x7fffffffull; }
// workspace slot sizes (doubles) of Geo<b, ib>::TIMG / VIMG / TPIMG (ib: reflectors per group)
static size_t timg_doubles(int b, int ib = 32) {
  ib = std::min(b, ib);
  return ((size_t)ib * (ib + 1) + 127) / 128 * 128;
}
static size_t vimg_doubles(int b, int ib = 32) {
  ib = std::min(b, ib);
  return ((size_t)b * (ib + 2) + 127) / 128 * 128;
}
static size_t tpimg_doubles(int b, int ib = 32) {  // packed T image (Geo<b, ib>::TPIMG)
  const size_t nri = std::min(b, ib) / 4;
  return (16 * nri * nri + 127) / 128 * 128;
}
// fp32 chain image slots (doubles; tiles.hpp Geo32 / Img<B, float>)
static size_t vimg32_doubles(int b) { return (size_t)b * (b < 32 ? b : 32) / 2; }  // VR floats / 2
static size_t timg32_doubles(int b) {
  const size_t nmi = (b < 32 ? b : 32) / 16, npr = nmi * (nmi + 1) / 2;
  return (npr * 256 / 2 + 127) / 128 * 128;
}
// flow engine workspace of one step with `rows` tile rows (flow.hpp flow_vw_off / flow_tw_off);
// ib: the engine shape's group size (fp32: 32)
static size_t wk_bytes(int b, int rows, int dtype, int ib) {
  ib = std::min(b, ib);
  const size_t ng = b / ib;
  const size_t slot = dtype == TQR_F64 ? vimg_doubles(b, ib) + tpimg_doubles(b, ib) : vimg32_doubles(b) + timg32_doubles(b);
  return (size_t)rows * ng * slot * sizeof(double);
}

}  // namespace tqr

using namespace tqr;

struct tqr_plan {
  int m, n, b, p, q, kmax, dtype, nlevels;
  size_t es;
  std::vector<long> off_p, off_u;  // per wave offsets into the item arrays
  Item* d_items_p = nullptr;
  Item* d_items_u = nullptr;
  double* d_T = nullptr;   // T factors of the wave-batched engine
  std::vector<double*> wk;  // flow engine: per-step panel workspaces (V and T images)
  double** d_wk = nullptr;  // device table of wk
  hipStream_t sP = nullptr, sU = nullptr;
  hipEvent_t evP = nullptr, evU = nullptr, evStart = nullptr;
  kfn kp = nullptr, ku = nullptr;
  size_t ldsP = 0, ldsU = 0;
  int profile = 0;
  int chain_asm = 2;  // fp64 chains on the hand-scheduled MFMA stream (TQR_CHAIN_ASM: 0 compiler-scheduled, 1 whole strip loaded in the hand-over, 2 late strip loads)
  // flow engine
  int engine = 1;          // 1 = persistent dataflow (default), 0 = wave-batched launches
  Item* d_flow = nullptr;
  int nflow = 0;
  int nflow_global = 0;  // tasks of the global list (before a multi-GPU partition)
  unsigned list_hash = 0;  // FNV-1a of the global list's items in order (plan_signature)
  int* d_sync = nullptr;   // next, err, Rc, Tc, Ac, Rt, Rr
  size_t sync_ints = 0;
  int ns = 1, ng = 1, grid = 256, est_order = 0;
  int shape = 8, nt = 512;  // flow engine shape (flow_shape) and its workgroup size
  ffn kflow = nullptr;
  size_t ldsF = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<hipEvent_t> prof_ev;  // pairs per launch when profiling
  std::vector<int> prof_kind;
  int nl_u = 0, nl_p = 0;
  double ms_u = 0, ms_p = 0;
  // multi-GPU (tile-column snake partition; cyclic = TQR_DIST_PART=cyclic): rank / world, uncached
  // panel counters, forward counters, peer workspaces opened by IPC
  int rank = 0, world = 1, cyclic = 0;
  int* d_rf = nullptr;     // multi-GPU member flags (uncached), kmax x p x ng, then Done[world]
  int epoch = 0;           // multi-GPU: launches so far (the member flags' and Done's values)
  PeerBufs* d_peers = nullptr;
  double** d_peer_wk = nullptr;  // world x kmax opened peer workspace pointers
  std::vector<void*> opened;     // IPC-opened peer pointers
  bool imported = false;         // tqr_dist_import succeeded (world > 1 may execute)
  // executions of one plan share its counters and workspaces: they are serialised — a host
  // mutex around each enqueue sequence, and every execute's stream waits for the previous one
  std::mutex mu;
  hipEvent_t evDone = nullptr;
  FlowKnobs knobs;  // task-list order knobs, read once at creation (segment lengths: flow.hpp seglen_of_chain)
  // host-pointer path (geqrt_host): device matrix and compact tau, kept with the (cached) plan
  // (tqr_cache_clear releases them); hmu serialises whole host-API calls on one plan. The flow
  // engine's transfers run inside its launch (xfer.hpp): a second task list with UP / DOWN
  // tasks (d_flow_x), nxc chunks of xrows rows per tile column. The wave engine stages through
  // two pinned buffers (pin, pev, sC) before / after its launches.
  std::mutex hmu;
  std::atomic<int> users{0};  // one-shot helpers using this cached plan right now (PlanRef)
  void* hA = nullptr;
  void* hT = nullptr;
  Item* d_flow_x = nullptr;
  int nflow_x = 0, nxc = 0, xrows = 0;
  void* pin[2] = {nullptr, nullptr};
  size_t pin_bytes = 0;
  hipStream_t sC = nullptr;
  hipEvent_t pev[2] = {nullptr, nullptr};
};

// transfer arguments of one host-pointer execute of the flow engine (xfer.hpp)
struct XferArgs {
  const void* hsrc;
  void* hdst;
  long hld;
  int* hup;  // device view of the host flags (or null)
  int* hdn;
  int gen;
};

#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "tqr: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return TQR_EHIP;                                                                    \
    }                                                                                     \
  } while (0)

extern "C" {

const char* tqr_strerror(int s) {
  switch (s) {
    case TQR_OK: return "ok";
    case TQR_EINVAL: return "invalid argument";
    case TQR_ENOMEM: return "out of memory";
    case TQR_EHIP: return "HIP runtime error";
    case TQR_ENODEV: return "no usable gfx950 device";
    case TQR_ERCCL: return "RCCL error";
  }
  return "unknown";
}

const char* tqr_version(void) { return "tqr 0.1 (gfx950, flat-tree tiled Householder QR)"; }

long tqr_total_tasks(int m, int n, int b) {
  if (b <= 0 || m % b || n % b) return -1;
  return tqr_sched_total_tasks(m / b, n / b);
}

static int check_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return TQR_ENODEV;
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, dev) != hipSuccess) return TQR_ENODEV;
  if (strncmp(pr.gcnArchName, "gfx950", 6) != 0) {
    fprintf(stderr, "tqr: device %d is %s, this build targets gfx950 only\n", dev, pr.gcnArchName);
    return TQR_ENODEV;
  }
  return TQR_OK;
}

static void close_opened(tqr_plan* pl);
void tqr_plan_destroy(tqr_plan* pl) {
  if (!pl) return;
  if (pl->d_items_p) (void)hipFree(pl->d_items_p);
  if (pl->d_items_u) (void)hipFree(pl->d_items_u);
  if (pl->d_T) (void)hipFree(pl->d_T);
  for (double* w : pl->wk) (void)hipFree(w);
  if (pl->d_wk) (void)hipFree(pl->d_wk);
  if (pl->sP) (void)hipStreamDestroy(pl->sP);
  if (pl->sU) (void)hipStreamDestroy(pl->sU);
  if (pl->evP) (void)hipEventDestroy(pl->evP);
  if (pl->evU) (void)hipEventDestroy(pl->evU);
  if (pl->evStart) (void)hipEventDestroy(pl->evStart);
  if (pl->d_flow) (void)hipFree(pl->d_flow);
  if (pl->d_sync) (void)hipFree(pl->d_sync);
  if (pl->ev0) (void)hipEventDestroy(pl->ev0);
  if (pl->ev1) (void)hipEventDestroy(pl->ev1);
  if (pl->evDone) (void)hipEventDestroy(pl->evDone);
  if (pl->hA) (void)hipFree(pl->hA);
  if (pl->hT) (void)hipFree(pl->hT);
  if (pl->d_flow_x) (void)hipFree(pl->d_flow_x);
  for (int x = 0; x < 2; ++x) {
    if (pl->pin[x]) (void)hipHostFree(pl->pin[x]);
    if (pl->pev[x]) (void)hipEventDestroy(pl->pev[x]);
  }
  if (pl->sC) (void)hipStreamDestroy(pl->sC);
  for (auto e : pl->prof_ev) (void)hipEventDestroy(e);
  close_opened(pl);
  if (pl->d_peers) (void)hipFree(pl->d_peers);
  if (pl->d_peer_wk) (void)hipFree(pl->d_peer_wk);
  if (pl->d_rf) (void)hipFree(pl->d_rf);
  delete pl;
}

static int plan_create(tqr_plan** out, int m, int n, int b, int dtype, int rank, int world, int engine);
int tqr_plan_create(tqr_plan** out, int m, int n, int b, int dtype) {
  return plan_create(out, m, n, b, dtype, 0, 1, TQR_ENGINE_DEFAULT);
}
int tqr_plan_create_engine(tqr_plan** out, int m, int n, int b, int dtype, int engine) {
  if (engine != TQR_ENGINE_DEFAULT && engine != TQR_ENGINE_WAVES && engine != TQR_ENGINE_FLOW) return TQR_EINVAL;
  return plan_create(out, m, n, b, dtype, 0, 1, engine);
}
// The engine's wait limit (flow.hpp g_flow_wait_limit, read only after a wait's first 5 s): 5 s for
// one-GPU plans, TQR_PEER_TIMEOUT_S (default 60, at least 5) for multi-GPU plans, whose peers'
// launches may start seconds apart. It is a per-device symbol, so every launch sets its plan's
// value on its own stream when the device holds another one (a per-device cache skips the copy
// otherwise): a one-GPU launch after a multi-GPU plan reports a real stall after 5 s again, and a
// multi-GPU plan on any device gets its limit there. (Round 5 raised it once per process, on the
// current device only.) Launches of plans with different limits running at once on one device
// share whichever value was set last — only how long a real stall takes to be reported differs.
static unsigned long long plan_wait_limit(int world) {
  if (world <= 1) return FLOW_TIMEOUT;
  double sec = 60.0;
  if (const char* e = getenv("TQR_PEER_TIMEOUT_S")) sec = std::max(5.0, atof(e));
  return (unsigned long long)(sec * 1e8);  // s_memrealtime: 100 MHz
}
static int set_wait_limit(unsigned long long ticks, hipStream_t cs) {
  constexpr int kDev = 64;
  static std::mutex mu;
  static unsigned long long cur[kDev] = {};  // per device: the value last set (0: unknown); also the
                                             // copy's source, alive after the async copy returns
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  if (dev < 0 || dev >= kDev) {
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_flow_wait_limit), &ticks, sizeof(ticks)));
    return TQR_OK;
  }
  std::lock_guard<std::mutex> lk(mu);
  if (cur[dev] == ticks) return TQR_OK;
  cur[dev] = ticks;
  if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_flow_wait_limit), &cur[dev], sizeof(ticks), 0, hipMemcpyHostToDevice, cs) !=
      hipSuccess) {
    cur[dev] = 0;
    return TQR_EHIP;
  }
  return TQR_OK;
}
int tqr_dist_plan_create(tqr_plan** out, int m, int n, int b, int dtype, int rank, int world) {
  if (world < 1 || rank < 0 || rank >= world) return TQR_EINVAL;
  return plan_create(out, m, n, b, dtype, rank, world, TQR_ENGINE_FLOW);
}
static int plan_create(tqr_plan** out, int m, int n, int b, int dtype, int rank, int world, int engine) {
  if (!out) return TQR_EINVAL;
  *out = nullptr;
  if (!valid_b(b) || m <= 0 || n <= 0 || m % b || n % b || (dtype != TQR_F32 && dtype != TQR_F64) ||
      !valid_ld(m, dtype == TQR_F64 ? 8 : 4))
    return TQR_EINVAL;
  int st = check_device();
  if (st) return st;
  tqr_plan* pl = new (std::nothrow) tqr_plan();
  if (!pl) return TQR_ENOMEM;
  pl->m = m; pl->n = n; pl->b = b; pl->p = m / b; pl->q = n / b;
  pl->rank = rank; pl->world = world; pl->cyclic = world > 1 && dist_cyclic();
  pl->kmax = std::min(pl->p, pl->q);
  pl->dtype = dtype;
  pl->es = dtype == TQR_F64 ? 8 : 4;

  tqr_plan_t sp;
  if (tqr_sched_plan(pl->p, pl->q, &sp) != 0) { delete pl; return TQR_ENOMEM; }
  pl->nlevels = sp.nlevels;
  const int nstrips = (b + 63) / 64;
  std::vector<Item> ip, iu;
  ip.reserve(sp.ntasks);
  iu.reserve(sp.ntasks * nstrips);
  for (int L = 0; L < sp.nlevels; ++L) {
    pl->off_p.push_back((long)ip.size());
    pl->off_u.push_back((long)iu.size());
    for (long x = sp.level_off[L]; x < sp.level_off[L + 1]; ++x) {
      const int* tk = sp.tasks + 4 * x;
      if (tk[0] == QRS || tk[0] == QRD) {
        ip.push_back(Item{tk[0], tk[1], tk[2], tk[3]});
      } else {
        for (int s = 0; s < nstrips; ++s) iu.push_back(Item{tk[0] | (s << 8), tk[1], tk[2], tk[3]});
      }
    }
  }
  pl->off_p.push_back((long)ip.size());
  pl->off_u.push_back((long)iu.size());
  tqr_sched_plan_free(&sp);

  int ib = b < 32 ? b : 32;
  if (engine == TQR_ENGINE_DEFAULT) {
    const char* eng = getenv("TQR_ENGINE");
    engine = (eng && strcmp(eng, "waves") == 0) ? TQR_ENGINE_WAVES : TQR_ENGINE_FLOW;
  }
  pl->engine = world > 1 ? TQR_ENGINE_FLOW : engine;  // the multi-GPU protocol lives in the flow engine
  size_t tw = pl->engine == 0 ? (size_t)pl->p * pl->kmax * (b / ib) * timg_doubles(b) * sizeof(double) : 8;
  if (hipMalloc(&pl->d_items_p, std::max<size_t>(1, ip.size()) * sizeof(Item)) != hipSuccess ||
      hipMalloc(&pl->d_items_u, std::max<size_t>(1, iu.size()) * sizeof(Item)) != hipSuccess ||
      hipMalloc(&pl->d_T, tw) != hipSuccess) {
    tqr_plan_destroy(pl);
    return TQR_ENOMEM;
  }
  if (!ip.empty() && hipMemcpy(pl->d_items_p, ip.data(), ip.size() * sizeof(Item), hipMemcpyHostToDevice) != hipSuccess) {
    tqr_plan_destroy(pl); return TQR_EHIP;
  }
  if (!iu.empty() && hipMemcpy(pl->d_items_u, iu.data(), iu.size() * sizeof(Item), hipMemcpyHostToDevice) != hipSuccess) {
    tqr_plan_destroy(pl); return TQR_EHIP;
  }
  if (hipStreamCreateWithFlags(&pl->sP, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&pl->sU, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&pl->evP, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&pl->evU, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&pl->evStart, hipEventDisableTiming) != hipSuccess) {
    tqr_plan_destroy(pl); return TQR_EHIP;
  }
  kfn kt;
  if (resolve(b, dtype, &pl->kp, &pl->ku, &kt) != TQR_OK) { tqr_plan_destroy(pl); return TQR_EHIP; }
  pl->ldsP = lds_panel(b);
  pl->ldsU = lds_update(b);
  if (hipEventCreate(&pl->ev0) != hipSuccess || hipEventCreate(&pl->ev1) != hipSuccess ||
      hipEventCreateWithFlags(&pl->evDone, hipEventDisableTiming) != hipSuccess) {
    tqr_plan_destroy(pl); return TQR_EHIP;
  }
  // persistent dataflow engine: task list, progress counters, panel workspaces, kernel
  pl->shape = flow_shape(dtype, b);
  pl->nt = shape_info(pl->shape).nt;
  pl->ns = shape_ns(pl->shape, b);  // chain strips per tile
  pl->ng = b / shape_ib(pl->shape, b);  // reflector groups per tile
  if (pl->engine == TQR_ENGINE_FLOW) {
    int dev = 0;
    hipDeviceProp_t pr;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&pr, dev) != hipSuccess) {
      tqr_plan_destroy(pl); return TQR_EHIP;
    }
    const int full_grid = pr.multiProcessorCount * shape_info(pl->shape).wpc;  // (ShapeW4: two workgroups per CU)
    pl->grid = full_grid;
    if (const char* gs = getenv("TQR_FLOW_GRID")) pl->grid = std::max(1, atoi(gs));
    FlowPlan fp;
    const MultiRankDefaults mrd = multi_rank_defaults(pl->p, pl->q, dtype, world, pl->grid >= full_grid);
    pl->knobs = knobs_from_env(env_seglen(world, pl->grid >= full_grid), mrd.tail, default_la(dtype), mrd.lac, mrd.ualone);
    if (const char* eca = getenv("TQR_CHAIN_ASM")) pl->chain_asm = atoi(eca) & 3;  // 0 off, 1 on, 2 late strip loads
    // (bit 2: UNMQR elements on the full TSMQR bodies instead of the zero-row-skipping ones; A/B only)
    if (const char* eu = getenv("TQR_UNMQR_SKIP"); eu && atoi(eu) == 0 && pl->chain_asm) pl->chain_asm |= 4;
    // (bit 3: fp32 storage on the compiler-scheduled flow_chain32; A/B only)
    if (const char* e32 = getenv("TQR_CHAIN32_ASM"); e32 && atoi(e32) == 0) pl->chain_asm |= 8;
    build_flow_plan(pl->p, pl->q, pl->ns, pl->ng, pl->knobs, fp);
    pl->nflow_global = (int)fp.items.size();
    {  // FNV-1a of the global list in order: every knob that shapes it (segments, lookahead keys,
       // TQR_LA / LAC / TG / LAZY) must agree across the ranks (tqr_dist_import)
      unsigned h = 2166136261u;
      for (const Item& it : fp.items)
        for (int v : {it.ts, it.l, it.m, it.k})
          for (int byte = 0; byte < 4; ++byte) h = (h ^ ((unsigned)v >> (8 * byte) & 0xffu)) * 16777619u;
      pl->list_hash = h;
    }
    if (world > 1) partition_flow_plan(fp, rank, world);
    pl->nflow = (int)fp.items.size();
    pl->est_order = fp.est_order;
    // next, err, host-transfer progress (flow.hpp timed_out), exit count, Rc, Tc, Ac, Rt, Rr, then Uc (upload chunks per tile column, host-pointer API)
    pl->sync_ints = 4 + 3 * (size_t)pl->kmax * pl->ng + (size_t)pl->p * pl->q * pl->ns +
                    (size_t)pl->kmax * pl->q * pl->ns * pl->ng + (size_t)pl->q;
    if (pl->nflow <= 0 || hipMalloc(&pl->d_flow, sizeof(Item) * pl->nflow) != hipSuccess ||
        hipMalloc(&pl->d_sync, sizeof(int) * pl->sync_ints) != hipSuccess ||
        hipMalloc(&pl->d_wk, sizeof(double*) * pl->kmax) != hipSuccess) {
      tqr_plan_destroy(pl); return TQR_ENOMEM;
    }
    // one workspace per step k: V then T images of tiles (k..p-1, k), every group.
    // Multi-GPU: peers' panel tasks write images of their panels into these slots over xGMI,
    // and such writes do not pass through this device's L2 — a line of a slot left in L2 by the
    // previous execute's reads would be served stale to this execute's chains. The slots are
    // therefore uncached (like the member flags); TQR_DIST_WK_CACHED=1 keeps them cached (the
    // one-GPU rehearsal's A/B of that cost only).
    const bool wk_uc = world > 1 && !(getenv("TQR_DIST_WK_CACHED") && atoi(getenv("TQR_DIST_WK_CACHED")) == 1);
    for (int k = 0; k < pl->kmax; ++k) {
      double* w = nullptr;
      const size_t wb = wk_bytes(b, pl->p - k, dtype, shape_ib(pl->shape, b));
      if ((wk_uc ? hipExtMallocWithFlags((void**)&w, wb, hipDeviceMallocUncached) : hipMalloc(&w, wb)) != hipSuccess) {
        tqr_plan_destroy(pl); return TQR_ENOMEM;
      }
      pl->wk.push_back(w);
    }
    if (hipMemcpy(pl->d_wk, pl->wk.data(), sizeof(double*) * pl->kmax, hipMemcpyHostToDevice) != hipSuccess) {
      tqr_plan_destroy(pl); return TQR_EHIP;
    }
    if (hipMemcpy(pl->d_flow, fp.items.data(), sizeof(Item) * pl->nflow, hipMemcpyHostToDevice) != hipSuccess) {
      tqr_plan_destroy(pl); return TQR_EHIP;
    }
    if (world > 1) {
      // member flags (+ Done[world] + Probe[world]) in uncached memory (peers' panels set them over
      // xGMI); zeroed once: their values are launch epochs (flow.hpp FlowArgs), Probe[r] rank r's
      // setup token (tqr_dist_probe)
      const size_t nrf = sizeof(int) * ((size_t)pl->kmax * pl->p * pl->ng + 2 * (size_t)world);
      if (hipExtMallocWithFlags((void**)&pl->d_rf, nrf, hipDeviceMallocUncached) != hipSuccess || hipMemset(pl->d_rf, 0, nrf) != hipSuccess ||
          hipMalloc(&pl->d_peers, sizeof(PeerBufs) * world) != hipSuccess ||
          hipMalloc(&pl->d_peer_wk, sizeof(double*) * (size_t)world * pl->kmax) != hipSuccess) {
        tqr_plan_destroy(pl); return TQR_ENOMEM;
      }
    }
    pl->kflow = resolve_flow(b, dtype, pl->shape);
    pl->ldsF = lds_flow(b, dtype, pl->shape);
    if (!pl->kflow) { tqr_plan_destroy(pl); return TQR_EHIP; }
  }
  *out = pl;
  return TQR_OK;
}

int tqr_plan_status(tqr_plan* pl, void* stream) {
  if (!pl) return TQR_EINVAL;
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  if (pl->engine != TQR_ENGINE_FLOW) return TQR_OK;  // wave engine: no in-kernel waits to time out
  int err = 0;
  HIPCHK(hipMemcpy(&err, pl->d_sync + 1, sizeof(int), hipMemcpyDeviceToHost));
  if (err) {
    fprintf(stderr, "tqr: dataflow engine aborted (error word %d: a dependency wait timed out)\n", err);
    return TQR_EHIP;
  }
  return TQR_OK;
}

// ---- multi-GPU ------------------------------------------------------------------------------
// handle block: the PCI bus id of the exporting device (64 bytes), then the IPC handles of its
// member flags and of its per-step panel workspaces
static constexpr size_t kBusIdBytes = 64;
// a rank's handle: PCI bus id, the task-list signature (every rank must partition the same global
// list: segment lengths, lookahead tail, list length), the IPC handles of Rf and the workspaces
constexpr size_t kSigInts = 7;
static void plan_signature(const tqr_plan* pl, int* sig) {
  sig[0] = pl->knobs.seglen; sig[1] = pl->knobs.seglen_la; sig[2] = pl->knobs.la_tail; sig[3] = pl->nflow_global;
  sig[4] = pl->knobs.tail; sig[5] = pl->knobs.tail_sl; sig[6] = (int)pl->list_hash;
}
size_t tqr_dist_handle_bytes(const tqr_plan* pl) {
  return pl ? kBusIdBytes + sizeof(int) * kSigInts + sizeof(hipIpcMemHandle_t) * (1 + (size_t)pl->kmax) : 0;
}

int tqr_dist_export(tqr_plan* pl, void* buf, size_t len) {
  if (!pl || pl->world < 2 || !buf || len < tqr_dist_handle_bytes(pl)) return TQR_EINVAL;
  char bus[kBusIdBytes] = {0};
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  HIPCHK(hipDeviceGetPCIBusId(bus, (int)kBusIdBytes - 1, dev));
  std::vector<hipIpcMemHandle_t> h(1 + pl->kmax);
  HIPCHK(hipIpcGetMemHandle(&h[0], pl->d_rf));
  for (int k = 0; k < pl->kmax; ++k) HIPCHK(hipIpcGetMemHandle(&h[1 + k], pl->wk[k]));
  int sig[kSigInts];
  plan_signature(pl, sig);
  memcpy(buf, bus, kBusIdBytes);
  memcpy((char*)buf + kBusIdBytes, sig, sizeof(sig));
  memcpy((char*)buf + kBusIdBytes + sizeof(sig), h.data(), sizeof(hipIpcMemHandle_t) * h.size());
  return TQR_OK;
}

static void close_opened(tqr_plan* pl) {
  for (void* p : pl->opened) (void)hipIpcCloseMemHandle(p);
  pl->opened.clear();
}

// Peer reachability of the device that exported `bus`: the same device (ranks sharing a GPU)
// needs nothing; another device must be peer-accessible from this one (xGMI), and peer access
// is enabled explicitly before any handle is opened — a missing link fails here, loudly,
// instead of as a fault or a hang inside the persistent launch.
static int enable_peer(int rank, int r, const char* bus) {
  int me = 0, peer = -1;
  HIPCHK(hipGetDevice(&me));
  if (hipDeviceGetByPCIBusId(&peer, bus) != hipSuccess) {
    (void)hipGetLastError();
    // not visible in this process (e.g. HIP_VISIBLE_DEVICES): the IPC open decides
    fprintf(stderr, "tqr: rank %d: rank %d's device %s is not visible here; relying on IPC peer mapping\n", rank, r, bus);
    return TQR_OK;
  }
  if (peer == me) return TQR_OK;
  int can = 0;
  HIPCHK(hipDeviceCanAccessPeer(&can, me, peer));
  if (!can) {
    fprintf(stderr, "tqr: rank %d: device %d cannot access rank %d's device %d (%s): no peer path\n", rank, me, r, peer, bus);
    return TQR_EHIP;
  }
  hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
  } else if (e != hipSuccess) {
    fprintf(stderr, "tqr: rank %d: enabling peer access to device %d failed: %s\n", rank, peer, hipGetErrorString(e));
    return TQR_EHIP;
  }
  return TQR_OK;
}

int tqr_dist_import(tqr_plan* pl, const void* all, size_t len) {
  const size_t hb = tqr_dist_handle_bytes(pl);
  if (!pl || pl->world < 2 || !all || len < (size_t)pl->world * hb || pl->imported) return TQR_EINVAL;
  close_opened(pl);  // a previous failed import
  std::vector<PeerBufs> pb(pl->world);
  std::vector<double*> pwk((size_t)pl->world * pl->kmax, nullptr);
  for (int r = 0; r < pl->world; ++r) {
    double** tab = pl->d_peer_wk + (size_t)r * pl->kmax;
    if (r == pl->rank) {
      for (int k = 0; k < pl->kmax; ++k) pwk[(size_t)r * pl->kmax + k] = pl->wk[k];
      pb[r] = PeerBufs{tab, pl->d_rf};
      continue;
    }
    const char* blk = (const char*)all + (size_t)r * hb;
    int sig[kSigInts], mine[kSigInts];
    memcpy(sig, blk + kBusIdBytes, sizeof(sig));
    plan_signature(pl, mine);
    if (memcmp(sig, mine, sizeof(sig)) != 0) {  // a launch over different lists would deadlock
      fprintf(stderr, "tqr: rank %d and rank %d built different task lists (segment lengths %d/%d vs %d/%d, "
              "lookahead tail %d vs %d, tail %d/%d vs %d/%d, %d vs %d tasks, list hash %08x vs %08x): set "
              "TQR_SEGLEN / TQR_TAIL / TQR_LA / TQR_LAC / TQR_TG / TQR_LAZY / TQR_FLOW_GRID alike on every rank\n",
              pl->rank, r, mine[0], mine[1], sig[0], sig[1], mine[2], sig[2], mine[4], mine[5], sig[4], sig[5],
              mine[3], sig[3], (unsigned)mine[6], (unsigned)sig[6]);
      close_opened(pl);
      return TQR_EINVAL;
    }
    char bus[kBusIdBytes];
    memcpy(bus, blk, kBusIdBytes);
    bus[kBusIdBytes - 1] = 0;
    int st = enable_peer(pl->rank, r, bus);
    if (st) { close_opened(pl); return st; }
    std::vector<hipIpcMemHandle_t> h(1 + pl->kmax);
    memcpy(h.data(), blk + kBusIdBytes + sizeof(sig), hb - kBusIdBytes - sizeof(sig));
    for (int x = 0; x <= pl->kmax; ++x) {
      void* p = nullptr;
      if (hipIpcOpenMemHandle(&p, h[x], hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
        fprintf(stderr, "tqr: rank %d cannot open rank %d's workspace (IPC handle %d)\n", pl->rank, r, x);
        close_opened(pl);
        return TQR_EHIP;
      }
      pl->opened.push_back(p);
      if (x == 0) pb[r].Rf = (int*)p;
      else pwk[(size_t)r * pl->kmax + x - 1] = (double*)p;
    }
    pb[r].Wk = tab;
  }
  if (hipMemcpy(pl->d_peer_wk, pwk.data(), sizeof(double*) * pwk.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(pl->d_peers, pb.data(), sizeof(PeerBufs) * pl->world, hipMemcpyHostToDevice) != hipSuccess) {
    close_opened(pl);
    return TQR_EHIP;
  }
  pl->imported = true;
  return TQR_OK;
}

// ---- peer-path probe (setup): the flag path of the persistent launch, exercised once ----------
// A panel's owner sets the member flags in its peers' Rf with system-scope stores through the
// IPC-mapped peer pointers, and the chains poll their own Rf with system-scope loads (flow.hpp).
// A broken path would otherwise show up only as a 60 s wait timeout inside the first factorisation
// (or never, as a hang, if the stores are silently lost), so the setup runs the same two operations
// on a probe word per rank: put (every rank stores its token into each peer's Probe[rank]), a host
// barrier, then check (every rank loads its own Probe[r] of every peer r).
static int probe_token(int rank) { return 0x7e510000 | (rank + 1); }
__global__ void k_probe_put(const PeerBufs* peers, long off, int rank, int world, int token) {
  const int r = threadIdx.x;
  if (r < world && r != rank)
    __hip_atomic_store((__attribute__((address_space(1))) int*)(peers[r].Rf + off + rank), token, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_probe_get(int* rf, long off, int world, int* out) {
  const int r = threadIdx.x;
  if (r < world) out[r] = ld_sys(rf + off + r);
}
int tqr_dist_probe(tqr_plan* pl, int phase, unsigned long long* seen) {
  if (!pl || pl->world < 2 || !pl->imported || pl->world > 64 || (phase != 0 && phase != 1)) return TQR_EINVAL;
  const long off = (long)pl->kmax * pl->p * pl->ng + pl->world;  // Probe[] after Done[]
  if (phase == 0) {
    hipLaunchKernelGGL(k_probe_put, dim3(1), dim3(64), 0, 0, (const PeerBufs*)pl->d_peers, off, pl->rank, pl->world,
                       probe_token(pl->rank));
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    return TQR_OK;
  }
  int* d_out = nullptr;
  HIPCHK(hipMalloc(&d_out, sizeof(int) * 64));
  hipLaunchKernelGGL(k_probe_get, dim3(1), dim3(64), 0, 0, pl->d_rf, off, pl->world, d_out);
  int h[64] = {0};
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpy(h, d_out, sizeof(int) * pl->world, hipMemcpyDeviceToHost);
  (void)hipFree(d_out);
  if (e != hipSuccess) {
    fprintf(stderr, "tqr: rank %d: peer probe failed: %s\n", pl->rank, hipGetErrorString(e));
    return TQR_EHIP;
  }
  unsigned long long got = 0;
  for (int r = 0; r < pl->world; ++r)
    if (r != pl->rank && h[r] == probe_token(r)) got |= 1ull << r;
  if (seen) *seen = got;
  int st = TQR_OK;
  for (int r = 0; r < pl->world; ++r)
    if (r != pl->rank && !((got >> r) & 1)) {
      fprintf(stderr, "tqr: rank %d does not see rank %d's flag stores (probe word 0x%08x, expected 0x%08x): no working "
              "peer path for the panel flags\n", pl->rank, r, (unsigned)h[r], (unsigned)probe_token(r));
      st = TQR_EHIP;
    }
  return st;
}

// Kept for the API: since round 4 every execute resets its own (local) counters, and the
// cross-rank flags carry launch epochs, so consecutive multi-GPU executes need no reset, host
// synchronisation or barrier (flow.hpp FlowArgs Done[]).
int tqr_dist_reset(tqr_plan* pl, void* stream) {
  (void)stream;
  if (!pl || pl->world < 2) return TQR_EINVAL;
  return TQR_OK;
}

int tqr_dist_local_cols(const tqr_plan* pl) {
  if (!pl) return TQR_EINVAL;
  int c = 0;
  for (int j = 0; j < pl->q; ++j) c += tile_owner(j, pl->world, pl->cyclic) == pl->rank;
  return c;
}

long long tqr_plan_fwd_bytes(const tqr_plan* pl) {
  if (!pl) return TQR_EINVAL;
  if (pl->world < 2) return 0;
  long long members = 0;  // panel members of the tile columns this rank owns
  for (int k = 0; k < pl->kmax; ++k)
    if (tile_owner(k, pl->world, pl->cyclic) == pl->rank) members += pl->p - k;
  const long long slot = (long long)(wk_bytes(pl->b, 1, pl->dtype, shape_ib(pl->shape, pl->b)));  // one member's images, all groups
  return members * slot * (pl->world - 1);
}

int tqr_dist_owner(const tqr_plan* pl, int tile_col) {
  if (!pl || tile_col < 0 || tile_col >= pl->q) return TQR_EINVAL;
  return tile_owner(tile_col, pl->world, pl->cyclic);
}

// Host-only task-list helpers below describe the fp64 engine's list (flow_shape(TQR_F64)); world:
// the ranks of a multi-GPU plan, each launch covering its whole device (the multi-rank defaults
// apply as in tqr_dist_plan_create; the segment length is the caller's). M, N: tiles.
static void host_flow_plan(int M, int N, int b, int seglen, FlowPlan& fp, const XferPlan* xp = nullptr, int world = 1) {
  const int sh = flow_shape(TQR_F64, b);
  const MultiRankDefaults mrd = multi_rank_defaults(M, N, TQR_F64, world, true);
  build_flow_plan(M, N, shape_ns(sh, b), b / shape_ib(sh, b),
                  knobs_from_env(seglen, mrd.tail, default_la(TQR_F64), mrd.lac, mrd.ualone), fp, xp);
}
int tqr_dist_plan_check(int M, int N, int b, int seglen, int rank, int world, int* ntasks, int* nfwd) {
  if (M <= 0 || N <= 0 || !valid_b(b) || seglen < 1 || world < 1 || rank < 0 || rank >= world) return TQR_EINVAL;
  FlowPlan fp;
  host_flow_plan(M, N, b, seglen, fp, nullptr, world);
  if (world > 1) partition_flow_plan(fp, rank, world);
  if (ntasks) *ntasks = (int)fp.items.size();
  if (nfwd) {  // panel members that forward their images (the panel tasks, when world > 1)
    int c = 0;
    if (world > 1)
      for (auto& it : fp.items) c += (it.ts & 0xff) != T_CHAIN;
    *nfwd = c;
  }
  return TQR_OK;
}

int tqr_flow_strip_width(void) { return shape_info(flow_shape(TQR_F64, 256)).sw; }

int tqr_flow_order_check(int M, int N, int b, const int* items, int n) {
  if (M <= 0 || N <= 0 || !valid_b(b) || !items || n <= 0) return TQR_EINVAL;
  std::vector<Item> L(n);
  for (int x = 0; x < n; ++x) L[x] = Item{items[4 * x], items[4 * x + 1], items[4 * x + 2], items[4 * x + 3]};
  return flow_list_topological(L, M, N, shape_ns(flow_shape(TQR_F64, b), b)) ? 1 : 0;
}

int tqr_plan_set_tasks(tqr_plan* pl, const int* items, int n) {
  if (!pl || !items || pl->engine != TQR_ENGINE_FLOW || pl->world != 1 || n != pl->nflow) return TQR_EINVAL;
  std::vector<Item> L(n), cur(n);
  for (int x = 0; x < n; ++x) L[x] = Item{items[4 * x], items[4 * x + 1], items[4 * x + 2], items[4 * x + 3]};
  std::lock_guard<std::mutex> lk(pl->mu);
  HIPCHK(hipEventSynchronize(pl->evDone));  // no execute may be using the current list
  HIPCHK(hipMemcpy(cur.data(), pl->d_flow, sizeof(Item) * n, hipMemcpyDeviceToHost));
  auto key = [](const Item& a) { return std::make_tuple(a.ts, a.l, a.m, a.k); };
  std::vector<std::tuple<int, int, int, int>> ka, kb;
  for (auto& it : L) ka.push_back(key(it));
  for (auto& it : cur) kb.push_back(key(it));
  std::sort(ka.begin(), ka.end());
  std::sort(kb.begin(), kb.end());
  if (ka != kb || !flow_list_topological(L, pl->p, pl->q, pl->ns)) return TQR_EINVAL;
  HIPCHK(hipMemcpy(pl->d_flow, L.data(), sizeof(Item) * n, hipMemcpyHostToDevice));
  return TQR_OK;
}

int tqr_plan_debug_workspace(const tqr_plan* pl, int k, void* host, size_t bytes) {
  if (!pl || pl->engine != TQR_ENGINE_FLOW || k < 0 || k >= pl->kmax || !host) return TQR_EINVAL;
  const size_t have = wk_bytes(pl->b, pl->p - k, pl->dtype, shape_ib(pl->shape, pl->b));
  HIPCHK(hipMemcpy(host, pl->wk[k], std::min(bytes, have), hipMemcpyDeviceToHost));
  return (int)std::min<size_t>(have, 0x7fffffff);
}

int tqr_flow_plan_export(int M, int N, int b, int seglen, int* items, int cap) {
  if (M <= 0 || N <= 0 || !valid_b(b) || seglen < 1) return TQR_EINVAL;
  FlowPlan fp;
  host_flow_plan(M, N, b, seglen, fp);
  const int n = (int)fp.items.size();
  if (items)
    for (int x = 0; x < n && x < cap; ++x) {
      items[4 * x] = fp.items[x].ts; items[4 * x + 1] = fp.items[x].l;
      items[4 * x + 2] = fp.items[x].m; items[4 * x + 3] = fp.items[x].k;
    }
  return n;
}

int tqr_flow_plan_check(int M, int N, int b, int seglen, int* ntasks, int* est_order) {
  if (M <= 0 || N <= 0 || !valid_b(b) || seglen < 1) return TQR_EINVAL;
  FlowPlan fp;
  host_flow_plan(M, N, b, seglen, fp);
  if (ntasks) *ntasks = (int)fp.items.size();
  if (est_order) *est_order = fp.est_order;
  return TQR_OK;
}

int tqr_flow_xfer_plan_check(int M, int N, int b, int seglen, int nxc, double tcol, int* ntasks, int* est_order) {
  if (M <= 0 || N <= 0 || !valid_b(b) || seglen < 1 || nxc < 1 || nxc > 255 || !(tcol >= 0.0)) return TQR_EINVAL;
  FlowPlan fp;
  XferPlan xp;
  xp.nxc = nxc;
  xp.tcol = tcol;
  host_flow_plan(M, N, b, seglen, fp, &xp);
  if (ntasks) *ntasks = (int)fp.items.size();
  if (est_order) *est_order = fp.est_order;
  return TQR_OK;
}

int tqr_plan_info(const tqr_plan* pl, int* engine, int* ntasks, int* est_order, int* grid) {
  if (!pl) return TQR_EINVAL;
  if (engine) *engine = pl->engine;
  if (ntasks) *ntasks = pl->engine == 1 ? pl->nflow : (int)pl->off_u.back();
  if (est_order) *est_order = pl->est_order;
  if (grid) *grid = pl->grid;
  return TQR_OK;
}

int tqr_plan_set_profile(tqr_plan* pl, int on) {
  if (!pl) return TQR_EINVAL;
  pl->profile = on;
  return TQR_OK;
}

int tqr_plan_stats(const tqr_plan* pl, int* nu, double* msu, int* np, double* msp) {
  if (!pl) return TQR_EINVAL;
  if (nu) *nu = pl->nl_u;
  if (msu) *msu = pl->ms_u;
  if (np) *np = pl->nl_p;
  if (msp) *msp = pl->ms_p;
  return TQR_OK;
}

static int plan_execute(tqr_plan* pl, void* dA, int ldda, void* dtau, hipStream_t cs, const XferArgs* xa = nullptr);
// Serialised enqueue of one execute (see tqr.h): the stream first waits for the plan's previous
// execute; evDone marks this one. If enqueuing fails part-way, evDone is still recorded behind
// whatever was enqueued (the wave engine's side streams are joined first), so the next execute
// stays ordered after it.
static int plan_execute_serial(tqr_plan* pl, void* dA, int ldda, void* dtau, hipStream_t cs, const XferArgs* xa) {
  std::lock_guard<std::mutex> lk(pl->mu);
  HIPCHK(hipStreamWaitEvent(cs, pl->evDone, 0));  // the previous execute of this plan (any stream)
  int st = plan_execute(pl, dA, ldda, dtau, cs, xa);
  if (st != TQR_OK && pl->engine != TQR_ENGINE_FLOW) {
    (void)hipStreamWaitEvent(cs, pl->evP, 0);
    (void)hipStreamWaitEvent(cs, pl->evU, 0);
  }
  const hipError_t e = hipEventRecord(pl->evDone, cs);
  if (st == TQR_OK && e != hipSuccess) HIPCHK(e);
  return st;
}
int tqr_plan_execute(tqr_plan* pl, void* dA, int ldda, void* dtau, void* stream) {
  if (!pl || !dA || !dtau || ldda < pl->m || !valid_ld(ldda, pl->es)) return TQR_EINVAL;
  // a multi-GPU plan whose peers were never imported would dereference unset peer pointers
  if (pl->world > 1 && !pl->imported) return TQR_EINVAL;
  return plan_execute_serial(pl, dA, ldda, dtau, (hipStream_t)stream, nullptr);
}
static int plan_execute(tqr_plan* pl, void* dA, int ldda, void* dtau, hipStream_t cs, const XferArgs* xa) {
  if (pl->engine == 1) {
    if (!pl->kflow || !pl->d_flow || !pl->d_sync || (xa && !pl->d_flow_x)) return TQR_EINVAL;
    FlowArgs f;
    f.A = dA; f.tau = dtau; f.Wk = pl->d_wk; f.ldm = ldda;
    f.tasks = xa ? pl->d_flow_x : pl->d_flow;
    f.ntasks = xa ? pl->nflow_x : pl->nflow;
    f.m = pl->m; f.p = pl->p; f.q = pl->q; f.kmax = pl->kmax; f.ns = pl->ns;
    f.next = pl->d_sync; f.err = pl->d_sync + 1; f.exitc = pl->d_sync + 3; f.Rc = pl->d_sync + 4;
    f.Tc = f.Rc + (size_t)pl->kmax * pl->ng;
    f.Ac = f.Tc + (size_t)pl->p * pl->q * pl->ns;
    f.Rt = f.Ac + (size_t)pl->kmax * pl->q * pl->ns * pl->ng;
    f.Rr = f.Rt + (size_t)pl->kmax * pl->ng;
    f.dist = pl->world > 1; f.rank = pl->rank; f.world = pl->world; f.cyclic = pl->cyclic; f.peers = pl->d_peers; f.Rf = pl->d_rf;
    f.cdiv = pl->world;  // multi-GPU: the rank's own tile columns only, packed (FlowArgs::cdiv)
    f.rf_done = (long)pl->kmax * pl->p * pl->ng;
    // the launch's epoch: committed to the plan only once the launch is enqueued (a failed
    // enqueue must not leave this rank one epoch ahead of its peers for good)
    f.epoch = pl->world > 1 ? pl->epoch + 1 : 0;
    f.chain_asm = pl->chain_asm;
    f.seglen = pl->knobs.seglen; f.seglen_la = pl->knobs.seglen_la; f.la_tail = pl->knobs.la_tail;
    f.tail = pl->knobs.tail; f.tail_sl = pl->knobs.tail_sl; f.ualone = pl->knobs.ualone;
    if (xa) {
      f.hsrc = xa->hsrc; f.hdst = xa->hdst; f.hld = xa->hld; f.hup = xa->hup; f.hdn = xa->hdn; f.gen = xa->gen;
      f.Uc = f.Rr + (size_t)pl->kmax * pl->ng;
      f.nxc = pl->nxc; f.xrows = pl->xrows;
    } else {
      f.hsrc = nullptr; f.hdst = nullptr; f.hld = 0; f.hup = nullptr; f.hdn = nullptr; f.gen = 0;
      f.Uc = nullptr; f.nxc = 0; f.xrows = 0;
    }
    // local progress counters (multi-GPU: the member flags are epoch-valued and never reset)
    HIPCHK(hipMemsetAsync(pl->d_sync, 0, sizeof(int) * pl->sync_ints, cs));
    if (const int st = set_wait_limit(plan_wait_limit(pl->world), cs)) return st;
    if (pl->profile) HIPCHK(hipEventRecord(pl->ev0, cs));
    hipLaunchKernelGGL(pl->kflow, dim3(pl->grid), dim3(pl->nt), pl->ldsF, cs, f);
    HIPCHK(hipGetLastError());
    if (pl->world > 1) pl->epoch = f.epoch;
    if (pl->profile) {
      HIPCHK(hipEventRecord(pl->ev1, cs));
      HIPCHK(hipEventSynchronize(pl->ev1));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, pl->ev0, pl->ev1));
      pl->nl_u = 1; pl->ms_u = ms; pl->nl_p = 0; pl->ms_p = 0;
    }
    return TQR_OK;
  }
  Args a;
  a.A = dA; a.tau = dtau; a.Tw = pl->d_T; a.ldm = ldda; a.m = pl->m; a.p = pl->p; a.kmax = pl->kmax;
  // both work streams start after everything already queued on the caller's stream
  HIPCHK(hipEventRecord(pl->evStart, cs));
  HIPCHK(hipStreamWaitEvent(pl->sP, pl->evStart, 0));
  HIPCHK(hipStreamWaitEvent(pl->sU, pl->evStart, 0));
  HIPCHK(hipEventRecord(pl->evP, pl->sP));
  HIPCHK(hipEventRecord(pl->evU, pl->sU));
  size_t nev = 0;
  if (pl->profile) {
    size_t need = 2 * (size_t)pl->nlevels * 2;
    while (pl->prof_ev.size() < need) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      pl->prof_ev.push_back(e);
    }
    pl->prof_kind.assign(need / 2, -1);
  }
  for (int L = 0; L < pl->nlevels; ++L) {
    long np = pl->off_p[L + 1] - pl->off_p[L];
    long nu = pl->off_u[L + 1] - pl->off_u[L];
    // each stream waits for the other stream's previous wave (events hold wave L-1)
    HIPCHK(hipStreamWaitEvent(pl->sP, pl->evU, 0));
    HIPCHK(hipStreamWaitEvent(pl->sU, pl->evP, 0));
    if (np) {
      a.items = pl->d_items_p + pl->off_p[L];
      if (pl->profile) { pl->prof_kind[nev / 2] = 1; HIPCHK(hipEventRecord(pl->prof_ev[nev++], pl->sP)); }
      hipLaunchKernelGGL(pl->kp, dim3((unsigned)np), dim3(NT), pl->ldsP, pl->sP, a);
      HIPCHK(hipGetLastError());
      if (pl->profile) HIPCHK(hipEventRecord(pl->prof_ev[nev++], pl->sP));
    }
    if (nu) {
      a.items = pl->d_items_u + pl->off_u[L];
      if (pl->profile) { pl->prof_kind[nev / 2] = 0; HIPCHK(hipEventRecord(pl->prof_ev[nev++], pl->sU)); }
      hipLaunchKernelGGL(pl->ku, dim3((unsigned)nu), dim3(NT), pl->ldsU, pl->sU, a);
      HIPCHK(hipGetLastError());
      if (pl->profile) HIPCHK(hipEventRecord(pl->prof_ev[nev++], pl->sU));
    }
    HIPCHK(hipEventRecord(pl->evP, pl->sP));
    HIPCHK(hipEventRecord(pl->evU, pl->sU));
  }
  HIPCHK(hipStreamWaitEvent(cs, pl->evP, 0));
  HIPCHK(hipStreamWaitEvent(cs, pl->evU, 0));
  if (pl->profile) {
    HIPCHK(hipStreamSynchronize(cs));
    pl->nl_u = pl->nl_p = 0;
    pl->ms_u = pl->ms_p = 0;
    for (size_t x = 0; x + 1 < nev; x += 2) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, pl->prof_ev[x], pl->prof_ev[x + 1]));
      if (pl->prof_kind[x / 2] == 1) { pl->nl_p++; pl->ms_p += ms; }
      else { pl->nl_u++; pl->ms_u += ms; }
    }
  }
  return TQR_OK;
}

// ---- plan cache for the one-shot helpers -------------------------------------------------
static std::mutex g_cache_mu;
static std::map<std::tuple<int, int, int, int, int, int>, tqr_plan*> g_cache;

// A cached plan in use by a one-shot helper: counted in plan->users from the lookup (under
// g_cache_mu) until the call returns, so tqr_cache_clear never frees a plan another thread is
// still using (it unlinks the plans first, then waits for each one's users to drain).
struct PlanRef {
  tqr_plan* pl = nullptr;
  PlanRef() = default;
  PlanRef(const PlanRef&) = delete;
  PlanRef& operator=(const PlanRef&) = delete;
  ~PlanRef() {
    if (pl) pl->users.fetch_sub(1);
  }
};
static int cached_plan(int m, int n, int b, int dtype, PlanRef& ref, int engine = TQR_ENGINE_DEFAULT) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return TQR_ENODEV;
  std::lock_guard<std::mutex> lk(g_cache_mu);
  auto key = std::make_tuple(dev, m, n, b, dtype, engine);
  auto itc = g_cache.find(key);
  tqr_plan* pl = nullptr;
  if (itc != g_cache.end()) {
    pl = itc->second;
  } else {
    int st = tqr_plan_create_engine(&pl, m, n, b, dtype, engine);
    if (st) return st;
    g_cache[key] = pl;
  }
  pl->users.fetch_add(1);
  ref.pl = pl;
  return TQR_OK;
}

int tqr_dgeqrt_tiled(int m, int n, int b, double* dA, int ldda, double* dtau, void* stream) {
  PlanRef r;
  int st = cached_plan(m, n, b, TQR_F64, r);
  return st ? st : tqr_plan_execute(r.pl, dA, ldda, dtau, stream);
}
int tqr_sgeqrt_tiled(int m, int n, int b, float* dA, int ldda, float* dtau, void* stream) {
  PlanRef r;
  int st = cached_plan(m, n, b, TQR_F32, r);
  return st ? st : tqr_plan_execute(r.pl, dA, ldda, dtau, stream);
}

// Host-pointer factorisation (the reference's calling convention: cudaQRTask copies a host matrix
// in and out, gpucalc.cu:1614-1619, 1665-1670 — one cudaMemcpy per column, before and after the
// kernel). The flow engine moves the matrix INSIDE its persistent launch (xfer.hpp): UP tasks
// read tile columns from host memory ahead of the step-0 tasks that need them, DOWN tasks write
// each tile column back as soon as it is final, so PCIe traffic overlaps the factorisation.
// Host memory, one of:
//   * staging (default): a pinned, fine-grained buffer shared by all host-API calls of the device;
//     host threads copy the caller's columns into it tile column by tile column (flag hup[j] per
//     column, polled by the UP tasks) and copy finished chunks back out as the DOWN tasks flag them
//     (hdn[j][c]) — while the kernel runs;
//   * registered (TQR_HOST_XFER=register): the caller's array itself is page-locked for the call
//     (hipHostRegister) and read / written by the launch directly; no host copies.
// The wave engine (cudaQRFull) keeps pre/post copies through two pinned buffers of the plan.
// The device matrix and compact tau stay with the cached plan; tqr_cache_clear releases them.

// host threads for host-side copies (the GPU box exports OMP_NUM_THREADS = this job's CPU share;
// hardware_concurrency() there is the whole machine)
static int host_threads() {
  const char* e = getenv("OMP_NUM_THREADS");
  int n = e ? atoi(e) : 0;
  if (n <= 0) n = (int)std::max(1u, std::thread::hardware_concurrency());
  return std::min(n, 32);
}

// Run jobs on their own threads; a job whose thread cannot be created runs on the caller, after
// the others were started (jobs are ordered so that no job waits for a later one).
static void run_jobs(std::vector<std::function<void()>>& jobs) {
  std::vector<std::thread> th;
  size_t created = 0;
  try {
    for (; created + 1 < jobs.size(); ++created) th.emplace_back(jobs[created]);
  } catch (...) {
  }
  for (size_t x = created; x < jobs.size(); ++x) jobs[x]();
  for (auto& t : th) t.join();
}

// wave engine: device buffers + two pinned staging buffers. Everything is allocated into locals and
// committed to the plan only when all of it succeeded (a failed call leaves the plan untouched).
static constexpr size_t kPinBytes = 64ull << 20;
static int plan_host_buffers(tqr_plan* pl, size_t es) {
  if (pl->hA) return TQR_OK;
  const size_t abytes = es * (size_t)pl->m * pl->n, tbytes = es * (size_t)pl->m * pl->kmax;
  void *hA = nullptr, *hT = nullptr;
  if (hipMalloc(&hA, abytes) != hipSuccess || hipMalloc(&hT, tbytes) != hipSuccess) {
    if (hA) (void)hipFree(hA);
    return TQR_ENOMEM;
  }
  pl->hA = hA;
  pl->hT = hT;
  return TQR_OK;
}
static int plan_pinned_staging(tqr_plan* pl, size_t es) {
  if (pl->pin[0]) return TQR_OK;
  const size_t bytes = std::min(kPinBytes, std::max(es * (size_t)pl->m * pl->n, es * (size_t)pl->m * pl->kmax));
  void* pin[2] = {nullptr, nullptr};
  hipEvent_t pev[2] = {nullptr, nullptr};
  hipStream_t sC = nullptr;
  int st = TQR_OK;
  for (int x = 0; x < 2 && st == TQR_OK; ++x) {
    if (hipHostMalloc(&pin[x], bytes, hipHostMallocDefault) != hipSuccess) st = TQR_ENOMEM;
    else if (hipEventCreateWithFlags(&pev[x], hipEventDisableTiming) != hipSuccess) st = TQR_EHIP;
  }
  if (st == TQR_OK && hipStreamCreateWithFlags(&sC, hipStreamNonBlocking) != hipSuccess) st = TQR_EHIP;
  if (st != TQR_OK) {
    for (int x = 0; x < 2; ++x) {
      if (pin[x]) (void)hipHostFree(pin[x]);
      if (pev[x]) (void)hipEventDestroy(pev[x]);
    }
    return st;
  }
  for (int x = 0; x < 2; ++x) {
    pl->pin[x] = pin[x];
    pl->pev[x] = pev[x];
  }
  pl->pin_bytes = bytes;
  pl->sC = sC;
  return TQR_OK;
}

// copy `ncols` columns of `rows` elements between strided host memory (ld) and packed device memory
// through the plan's pinned buffers, double-buffered (wave engine)
static int staged_copy(tqr_plan* pl, char* host, size_t ld, char* dev, size_t rows, size_t ncols, size_t es, bool h2d) {
  const size_t col = es * rows, per = std::max<size_t>(1, pl->pin_bytes / col);
  const size_t nchunk = (ncols + per - 1) / per;
  const int nthr = std::min(8, host_threads());
  auto chunk = [&](size_t c, size_t& c0, size_t& nc) { c0 = c * per; nc = std::min(per, ncols - c0); };
  auto par_columns = [&](size_t nc, const std::function<void(size_t)>& f) {
    const size_t nt = std::min<size_t>(nc, (size_t)nthr);
    std::vector<std::function<void()>> jobs;
    for (size_t t = 0; t < nt; ++t)
      jobs.push_back([&, t] {
        for (size_t j = t; j < nc; j += nt) f(j);
      });
    run_jobs(jobs);
  };
  if (h2d) {
    for (size_t c = 0; c < nchunk; ++c) {
      size_t c0, nc;
      chunk(c, c0, nc);
      char* pb = (char*)pl->pin[c & 1];
      HIPCHK(hipEventSynchronize(pl->pev[c & 1]));  // the DMA from this buffer two chunks ago is done
      par_columns(nc, [&](size_t j) { memcpy(pb + j * col, host + (c0 + j) * ld * es, col); });
      HIPCHK(hipMemcpyAsync(dev + c0 * col, pb, nc * col, hipMemcpyHostToDevice, pl->sC));
      HIPCHK(hipEventRecord(pl->pev[c & 1], pl->sC));
    }
    return TQR_OK;
  }
  auto issue = [&](size_t c) -> int {
    size_t c0, nc;
    chunk(c, c0, nc);
    HIPCHK(hipMemcpyAsync(pl->pin[c & 1], dev + c0 * col, nc * col, hipMemcpyDeviceToHost, pl->sC));
    HIPCHK(hipEventRecord(pl->pev[c & 1], pl->sC));
    return TQR_OK;
  };
  for (size_t c = 0; c < std::min<size_t>(2, nchunk); ++c)
    if (int st = issue(c)) return st;
  for (size_t c = 0; c < nchunk; ++c) {
    size_t c0, nc;
    chunk(c, c0, nc);
    HIPCHK(hipEventSynchronize(pl->pev[c & 1]));
    const char* pb = (const char*)pl->pin[c & 1];
    par_columns(nc, [&](size_t j) { memcpy(host + (c0 + j) * ld * es, pb + j * col, col); });
    if (c + 2 < nchunk)
      if (int st = issue(c + 2)) return st;
  }
  return TQR_OK;
}

// The pinned, fine-grained staging buffer and flag words of the flow engine's host path, one per
// device, shared by all plans (grown on demand; tqr_cache_clear frees it). `mu` serialises the
// host-API calls that use it.
struct HostStage {
  std::mutex mu;
  char* buf = nullptr;
  size_t bytes = 0;
  int* flags = nullptr;  // host view: hup[q] then hdn[q * nxc]
  int* dflags = nullptr;  // device view
  size_t nflags = 0;
  int gen = 0;
  void release() {
    if (buf) (void)hipHostFree(buf);
    if (flags) (void)hipHostFree(flags);
    buf = nullptr; flags = nullptr; dflags = nullptr; bytes = 0; nflags = 0;
  }
  int ensure(size_t need, size_t nf) {
    if (bytes < need) {
      if (buf) (void)hipHostFree(buf);
      buf = nullptr; bytes = 0;
      void* p = nullptr;
      if (hipHostMalloc(&p, need, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return TQR_ENOMEM;
      buf = (char*)p;
      bytes = need;
    }
    if (nflags < nf) {
      if (flags) (void)hipHostFree(flags);
      flags = nullptr; dflags = nullptr; nflags = 0;
      void* p = nullptr;
      if (hipHostMalloc(&p, nf * sizeof(int), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return TQR_ENOMEM;
      memset(p, 0, nf * sizeof(int));
      flags = (int*)p;
      nflags = nf;
      gen = 0;
      void* d = nullptr;
      if (hipHostGetDevicePointer(&d, flags, 0) != hipSuccess) { release(); return TQR_EHIP; }
      dflags = (int*)d;
    }
    return TQR_OK;
  }
};
static std::map<int, HostStage*> g_stage;  // guarded by g_cache_mu

static int plan_xfer_list(tqr_plan* pl) {
  if (pl->d_flow_x) return TQR_OK;
  // chunk rows: one UP / DOWN task moves ~8 MiB (16-B vectors, 4 columns x 4 vectors per lane in
  // flight), a multiple of 4 rows so 16-B vectors stay whole (fp32), and
  // at most 255 chunks per column (the task word's chunk field)
  int xrows = std::max(4, (int)((8u << 20) / (pl->es * (size_t)pl->b)) & ~3);
  xrows = std::min(pl->m, std::max(xrows, ((pl->m + 254) / 255 + 3) & ~3));
  XferPlan xp;
  xp.nxc = (pl->m + xrows - 1) / xrows;
  // estimator unit = one chain element (4 b^2 SW flop at ~1/256 of the chip, SW the shape's strip
  // width); a tile column over PCIe at TQR_XFER_GBS (default 45 GB/s)
  const char* eg = getenv("TQR_XFER_GBS");
  const double gbs = eg ? std::max(1.0, atof(eg)) : 45.0;
  const double elem_s = 4.0 * pl->b * pl->b * shape_info(pl->shape).sw / (pl->dtype == TQR_F64 ? 0.175e12 : 0.38e12);
  xp.tcol = ((double)pl->m * pl->b * pl->es / (gbs * 1e9)) / elem_s;
  FlowPlan fp;
  build_flow_plan(pl->p, pl->q, pl->ns, pl->ng, pl->knobs, fp, &xp);  // the plan's own knobs (not the environment now)
  Item* d = nullptr;
  if (hipMalloc(&d, sizeof(Item) * fp.items.size()) != hipSuccess) return TQR_ENOMEM;
  if (hipMemcpy(d, fp.items.data(), sizeof(Item) * fp.items.size(), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    return TQR_EHIP;
  }
  pl->d_flow_x = d;
  pl->nflow_x = (int)fp.items.size();
  pl->nxc = xp.nxc;
  pl->xrows = xrows;
  return TQR_OK;
}

// tau: compact device array -> the reference's m x n matrix (column k*b of tau = compact column k,
// rows k*b .. m-1; other entries untouched)
static int tau_out(tqr_plan* pl, void* tau, int ldm, size_t es, hipStream_t s) {
  const int m = pl->m, b = pl->b, kmax = pl->kmax;
  std::vector<char> ct(es * (size_t)m * kmax);
  HIPCHK(hipMemcpyAsync(ct.data(), pl->hT, ct.size(), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (int k = 0; k < kmax; ++k)
    memcpy((char*)tau + es * ((size_t)k * b * ldm + (size_t)k * b), ct.data() + es * ((size_t)k * m + (size_t)k * b),
           es * (size_t)(m - k * b));
  return TQR_OK;
}

static int geqrt_host_flow(tqr_plan* pl, void* A, void* tau, int ldm, size_t es) {
  const int m = pl->m, n = pl->n, q = pl->q, b = pl->b;
  int st;
  if ((st = plan_host_buffers(pl, es)) || (st = plan_xfer_list(pl))) return st;
  if (!pl->sC && hipStreamCreateWithFlags(&pl->sC, hipStreamNonBlocking) != hipSuccess) return TQR_EHIP;
  hipStream_t s = pl->sC;
  HIPCHK(hipMemsetAsync(pl->hT, 0, es * (size_t)m * pl->kmax, s));
  const char* mode = getenv("TQR_HOST_XFER");
  if (mode && strcmp(mode, "register") == 0) {
    const size_t span = es * ((size_t)(n - 1) * ldm + m);
    if (hipHostRegister(A, span, hipHostRegisterMapped) == hipSuccess) {
      void* dv = nullptr;
      if (hipHostGetDevicePointer(&dv, A, 0) != hipSuccess) {
        (void)hipHostUnregister(A);
        return TQR_EHIP;
      }
      XferArgs xa{dv, dv, ldm, nullptr, nullptr, 0};
      st = plan_execute_serial(pl, pl->hA, m, pl->hT, s, &xa);
      if (st == TQR_OK) st = tqr_plan_status(pl, s);
      else (void)hipStreamSynchronize(s);
      (void)hipHostUnregister(A);
      if (st == TQR_OK && tau) st = tau_out(pl, tau, ldm, es, s);
      return st;
    }
    (void)hipGetLastError();  // not registrable: stage instead
  }
  HostStage* hs;
  {
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_cache_mu);
    auto& e = g_stage[dev];
    if (!e) e = new (std::nothrow) HostStage();
    if (!e) return TQR_ENOMEM;
    hs = e;
  }
  std::lock_guard<std::mutex> lk(hs->mu);
  const int nxc = pl->nxc;
  if ((st = hs->ensure(es * (size_t)m * n, (size_t)q * (1 + nxc)))) return st;
  void* dbuf = nullptr;
  HIPCHK(hipHostGetDevicePointer(&dbuf, hs->buf, 0));
  const int gen = ++hs->gen;
  int* hup = hs->flags;
  int* hdn = hs->flags + q;
  XferArgs xa{dbuf, dbuf, m, hs->dflags, hs->dflags + q, gen};
  // TQR_HOST_XFER_VERBOSE=1: where the time goes (launch, staging done, kernel, drain done)
  const bool verbose = getenv("TQR_HOST_XFER_VERBOSE") && atoi(getenv("TQR_HOST_XFER_VERBOSE")) == 1;
  auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t0 = now();
  std::atomic<long long> t_up{0}, t_dn{0};
  // host side, beside the launch: nu threads stage tile columns in order (the last one to finish a
  // column flags it), nd threads move finished chunks back to the caller's array. They start
  // BEFORE the launch call: the launched kernel waits for the staging flags, so the staging must
  // not depend on this thread returning from HIP calls (another thread's hipFree — e.g. a
  // concurrent tqr_cache_clear — waits for the device to be idle, i.e. for this kernel; a staging
  // started behind a HIP call stalled by it would leave the kernel waiting until its timeout)
  std::atomic<int> launched{0};
  const int nthr = host_threads();
  const int nu = std::max(1, nthr / 2), nd = std::max(1, nthr - nu);
  const size_t col = es * (size_t)m;
  char* user = (char*)A;
  std::vector<std::atomic<int>> staged(q);
  for (auto& x : staged) x.store(0);
  std::atomic<int> failed{0};
  std::vector<std::function<void()>> jobs;
  // TQR_HOST_STAGE_DELAY_MS (tests only): a slow host, each tile column staged that much later
  const char* edl = getenv("TQR_HOST_STAGE_DELAY_MS");
  const int stage_delay_ms = edl ? std::max(0, atoi(edl)) : 0;
  for (int t = 0; t < nu; ++t)
    jobs.push_back([&, t] {
      for (int j = 0; j < q; ++j) {
        if (stage_delay_ms) std::this_thread::sleep_for(std::chrono::milliseconds(stage_delay_ms));
        for (int c = j * b + t; c < (j + 1) * b; c += nu) memcpy(hs->buf + c * col, user + (size_t)c * ldm * es, col);
        if (staged[j].fetch_add(1) + 1 == nu) __atomic_store_n(&hup[j], gen, __ATOMIC_RELEASE);
      }
      if (verbose) t_up.store(std::max<long long>(t_up.load(), (long long)((now() - t0) * 1e3)));
    });
  for (int t = 0; t < nd; ++t)
    jobs.push_back([&, t] {
      for (int j = 0; j < q; ++j) {
        for (int c = 0; c < nxc; ++c) {
          // the chunk's flag, or the launch ended without setting it (an engine error)
          for (long spins = 0; __atomic_load_n(&hdn[(size_t)j * nxc + c], __ATOMIC_ACQUIRE) < gen; ++spins) {
            if (failed.load(std::memory_order_relaxed)) return;
            if ((spins & 255) == 255) {
              if (launched.load(std::memory_order_acquire) && hipStreamQuery(s) != hipErrorNotReady &&
                  __atomic_load_n(&hdn[(size_t)j * nxc + c], __ATOMIC_ACQUIRE) < gen) {
                failed.store(1);
                return;
              }
              std::this_thread::yield();
            } else {
              __builtin_ia32_pause();
            }
          }
        }
        for (int c = j * b + t; c < (j + 1) * b; c += nd) memcpy(user + (size_t)c * ldm * es, hs->buf + c * col, col);
      }
      if (verbose) t_dn.store(std::max<long long>(t_dn.load(), (long long)((now() - t0) * 1e3)));
    });
  std::vector<std::thread> th;
  std::vector<size_t> inline_jobs;  // jobs whose thread could not be created: run after the launch
  for (size_t x = 0; x < jobs.size(); ++x) {
    try {
      th.emplace_back(jobs[x]);
    } catch (...) {
      inline_jobs.push_back(x);
    }
  }
  if (verbose) (void)hipEventRecord(pl->ev0, s);
  st = plan_execute_serial(pl, pl->hA, m, pl->hT, s, &xa);
  if (st == TQR_OK) {
    if (verbose) (void)hipEventRecord(pl->ev1, s);
    launched.store(1, std::memory_order_release);
  } else {
    failed.store(1);  // (the copy-out threads stop waiting)
  }
  for (size_t x : inline_jobs) jobs[x]();
  for (auto& t : th) t.join();
  if (st != TQR_OK) {
    (void)hipStreamSynchronize(s);
    return st;
  }
  st = tqr_plan_status(pl, s);
  if (st == TQR_OK && failed.load()) st = TQR_EHIP;
  if (verbose && st == TQR_OK) {
    float kms = 0;
    HIPCHK(hipEventElapsedTime(&kms, pl->ev0, pl->ev1));
    fprintf(stderr, "tqr host xfer: %d host threads (%d in, %d out); staged all columns at %.2f ms, kernel %.2f ms, "
            "last chunk copied out at %.2f ms, done %.2f ms after the launch call\n", nthr, nu, nd, t_up.load() * 1e-3, kms,
            t_dn.load() * 1e-3, now() - t0);
  }
  if (st == TQR_OK && tau) st = tau_out(pl, tau, ldm, es, s);
  return st;
}

static int geqrt_host(void* A, void* tau, int m, int n, int ldm, int b, int dtype, int engine = TQR_ENGINE_DEFAULT) {
  if (!A || ldm < m || !valid_b(b) || m <= 0 || n <= 0 || m % b || n % b) return TQR_EINVAL;
  PlanRef ref;
  int st = cached_plan(m, n, b, dtype, ref, engine);
  if (st) return st;
  tqr_plan* pl = ref.pl;
  std::lock_guard<std::mutex> lk(pl->hmu);
  const size_t es = dtype == TQR_F64 ? 8 : 4;
  if (pl->engine == TQR_ENGINE_FLOW) return geqrt_host_flow(pl, A, tau, ldm, es);
  if ((st = plan_host_buffers(pl, es)) || (st = plan_pinned_staging(pl, es))) return st;
  char* dA = (char*)pl->hA;
  if ((st = staged_copy(pl, (char*)A, ldm, dA, m, n, es, true))) return st;
  HIPCHK(hipMemsetAsync(pl->hT, 0, es * (size_t)m * pl->kmax, pl->sC));
  if ((st = plan_execute_serial(pl, dA, m, pl->hT, pl->sC, nullptr))) return st;
  if ((st = tqr_plan_status(pl, pl->sC))) return st;
  if ((st = staged_copy(pl, (char*)A, ldm, dA, m, n, es, false))) return st;
  return tau ? tau_out(pl, tau, ldm, es, pl->sC) : TQR_OK;
}

int tqr_dgeqrt_host(double* A, double* tau, int m, int n, int ldm, int b) { return geqrt_host(A, tau, m, n, ldm, b, TQR_F64); }
int tqr_sgeqrt_host(float* A, float* tau, int m, int n, int ldm, int b) { return geqrt_host(A, tau, m, n, ldm, b, TQR_F32); }
int tqr_geqrt_host_engine(int dtype, void* A, void* tau, int m, int n, int ldm, int b, int engine) {
  if (dtype != TQR_F32 && dtype != TQR_F64) return TQR_EINVAL;
  if (engine != TQR_ENGINE_DEFAULT && engine != TQR_ENGINE_WAVES && engine != TQR_ENGINE_FLOW) return TQR_EINVAL;
  return geqrt_host(A, tau, m, n, ldm, b, dtype, engine);
}

// Release every cached plan (the one-shot helpers' and the host API's device matrices, compact
// tau, pinned buffers) and the host-API staging buffers. Safe against concurrent tqr calls: the
// plans are unlinked from the cache under its lock (later calls build new ones), then each is
// destroyed once no call still uses it (PlanRef count) and its last execute has finished (its
// evDone event, whatever device or stream it ran on). A staging buffer is released under its own
// mutex, which a host-API call holds from before its launch until its last copy out; the
// HostStage objects themselves are kept (a call may hold a pointer to one), so a later call just
// allocates again.
int tqr_cache_clear(void) {
  std::vector<tqr_plan*> plans;
  std::vector<HostStage*> stages;
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    for (auto& kv : g_cache) plans.push_back(kv.second);
    g_cache.clear();
    for (auto& kv : g_stage) stages.push_back(kv.second);
  }
  int st = TQR_OK;
  for (tqr_plan* pl : plans) {
    while (pl->users.load() > 0) std::this_thread::yield();
    {
      std::lock_guard<std::mutex> l1(pl->hmu);
      std::lock_guard<std::mutex> l2(pl->mu);
      if (pl->evDone && hipEventSynchronize(pl->evDone) != hipSuccess) st = TQR_EHIP;
    }
    tqr_plan_destroy(pl);
  }
  for (HostStage* hs : stages) {
    std::lock_guard<std::mutex> l2(hs->mu);
    hs->release();
  }
  return st;
}

int tqr_fill_randzo_cols(int dtype, void* dA, int m, int ncols, int ldda, unsigned long long seed, long col0, void* stream) {
  if (!dA || ldda < m || m <= 0 || ncols <= 0 || col0 < 0) return TQR_EINVAL;
  long total = (long)m * ncols;
  int blocks = (int)std::min<long>(65536, (total + 255) / 256);
  if (dtype == TQR_F64)
    hipLaunchKernelGGL(k_randzo<double>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (double*)dA, m, ncols, (long)ldda, seed, col0);
  else
    hipLaunchKernelGGL(k_randzo<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (float*)dA, m, ncols, (long)ldda, seed, col0);
  HIPCHK(hipGetLastError());
  return TQR_OK;
}
int tqr_fill_randzo(int dtype, void* dA, int m, int n, int ldda, unsigned long long seed, void* stream) {
  return tqr_fill_randzo_cols(dtype, dA, m, n, ldda, seed, 0, stream);
}

}  // extern "C"

// ---- single-tile API ----------------------------------------------------------------------
// The tile(s) are copied into a small device matrix laid out as the corresponding corner of
// a tiled matrix, the task runs as a one-item wave, and the result is copied back.
namespace {
struct TileRun {
  int b, dtype, mr, nc;  // device matrix mr x nc (ld = mr)
  size_t es;
  void* dA = nullptr;
  void* dtau = nullptr;
  double* dT = nullptr;
  Item* dit = nullptr;
  kfn kp, ku, kt;
  int init(int b_, int dtype_, int p, int q) {
    b = b_; dtype = dtype_; mr = p * b; nc = q * b; es = dtype == TQR_F64 ? 8 : 4;
    if (!valid_b(b) || (dtype != TQR_F64 && dtype != TQR_F32)) return TQR_EINVAL;
    int st = check_device();
    if (st) return st;
    if ((st = resolve(b, dtype, &kp, &ku, &kt))) return st;
    int ib = b < 32 ? b : 32;
    if (hipMalloc(&dA, es * mr * nc) != hipSuccess || hipMalloc(&dtau, es * mr) != hipSuccess ||
        hipMalloc(&dT, sizeof(double) * (size_t)p * (b / ib) * timg_doubles(b)) != hipSuccess || hipMalloc(&dit, sizeof(Item) * 4) != hipSuccess)
      return TQR_ENOMEM;
    if (hipMemset(dA, 0, es * mr * nc) != hipSuccess || hipMemset(dtau, 0, es * mr) != hipSuccess) return TQR_EHIP;
    return TQR_OK;
  }
  ~TileRun() {
    if (dA) (void)hipFree(dA);
    if (dtau) (void)hipFree(dtau);
    if (dT) (void)hipFree(dT);
    if (dit) (void)hipFree(dit);
  }
  int put(const void* h, int ldm, int r, int c) {  // host tile -> device tile (r,c)
    return hipMemcpy2D((char*)dA + es * ((size_t)c * b * mr + (size_t)r * b), es * mr, h, es * ldm, es * b, b,
                       hipMemcpyHostToDevice) == hipSuccess ? TQR_OK : TQR_EHIP;
  }
  int get(void* h, int ldm, int r, int c) {
    return hipMemcpy2D(h, es * ldm, (char*)dA + es * ((size_t)c * b * mr + (size_t)r * b), es * mr, es * b, b,
                       hipMemcpyDeviceToHost) == hipSuccess ? TQR_OK : TQR_EHIP;
  }
  int put_tau(const void* h, int row0) {
    return hipMemcpy((char*)dtau + es * row0, h, es * b, hipMemcpyHostToDevice) == hipSuccess ? TQR_OK : TQR_EHIP;
  }
  int get_tau(void* h, int row0) {
    return hipMemcpy(h, (char*)dtau + es * row0, es * b, hipMemcpyDeviceToHost) == hipSuccess ? TQR_OK : TQR_EHIP;
  }
  int run(kfn k, Item item, int grid, size_t lds) {
    if (hipMemcpy(dit, &item, sizeof item, hipMemcpyHostToDevice) != hipSuccess) return TQR_EHIP;
    Args a;
    a.A = dA; a.tau = dtau; a.Tw = dT; a.items = dit; a.ldm = mr; a.m = mr; a.p = mr / b; a.kmax = 1;
    hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, 0, a);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return TQR_EHIP;
    return TQR_OK;
  }
  int ng() const { return b / (b < 32 ? b : 32); }
  int nstrips() const { return (b + 63) / 64; }
  int run_update(Item item) {
    for (int s = 0; s < nstrips(); ++s) {
      Item it2 = item;
      it2.ts |= s << 8;
      int st = run(ku, it2, 1, lds_update(b));
      if (st) return st;
    }
    return TQR_OK;
  }
};
}  // namespace

extern "C" {

int tqr_tile_geqrt(int dtype, void* blk, void* tau, int b, int ldm) {
  if (!blk || !tau || ldm < b) return TQR_EINVAL;
  TileRun tr;
  int st = tr.init(b, dtype, 1, 1);
  if (!st) st = tr.put(blk, ldm, 0, 0);
  if (!st) st = tr.run(tr.kp, Item{QRS, 0, 0, 0}, 1, lds_panel(b));
  if (!st) st = tr.get(blk, ldm, 0, 0);
  if (!st) st = tr.get_tau(tau, 0);
  return st;
}

int tqr_tile_unmqr(int dtype, void* C, const void* V, const void* tau, int b, int ldm) {
  if (!C || !V || !tau || ldm < b) return TQR_EINVAL;
  TileRun tr;
  int st = tr.init(b, dtype, 1, 2);
  if (!st) st = tr.put(V, ldm, 0, 0);
  if (!st) st = tr.put(C, ldm, 0, 1);
  if (!st) st = tr.put_tau(tau, 0);
  if (!st) st = tr.run(tr.kt, Item{QRS, 0, 0, 0}, tr.ng(), lds_build_t(b));
  if (!st) st = tr.run_update(Item{SAPP, 0, 1, 0});
  if (!st) st = tr.get(C, ldm, 0, 1);
  return st;
}

int tqr_tile_tsqrt(int dtype, void* A, void* Bm, void* tau, int b, int ldm) {
  if (!A || !Bm || !tau || ldm < b) return TQR_EINVAL;
  TileRun tr;
  int st = tr.init(b, dtype, 2, 1);
  if (!st) st = tr.put(A, ldm, 0, 0);
  if (!st) st = tr.put(Bm, ldm, 1, 0);
  if (!st) st = tr.run(tr.kp, Item{QRD, 1, 0, 0}, 1, lds_panel(b));
  if (!st) st = tr.get(A, ldm, 0, 0);
  if (!st) st = tr.get(Bm, ldm, 1, 0);
  if (!st) st = tr.get_tau(tau, b);
  return st;
}

int tqr_tile_tsmqr(int dtype, const void* V, void* A, void* Bm, const void* tau, int b, int ldm) {
  if (!V || !A || !Bm || !tau || ldm < b) return TQR_EINVAL;
  TileRun tr;
  int st = tr.init(b, dtype, 2, 2);
  if (!st) st = tr.put(V, ldm, 1, 0);
  if (!st) st = tr.put(A, ldm, 0, 1);
  if (!st) st = tr.put(Bm, ldm, 1, 1);
  if (!st) st = tr.put_tau(tau, b);
  if (!st) st = tr.run(tr.kt, Item{QRD, 1, 0, 0}, tr.ng(), lds_build_t(b));
  if (!st) st = tr.run_update(Item{DAPP, 1, 1, 0});
  if (!st) st = tr.get(A, ldm, 0, 1);
  if (!st) st = tr.get(Bm, ldm, 1, 1);
  return st;
}

// Batched independent tile updates (the reference's testDAPP microbenchmark, gpucalc.cu:1687-1774,
// generalised): nblocks copies of one tile (pair) updated by ONE launch of the update kernel.
int tqr_tile_batch(int dtype, int type, int b, int nblocks, const void* V, int ldv, const void* tau,
                   const void* blk, int ldb, void* out, int ldo, float* ms) {
  if ((type != SAPP && type != DAPP) || nblocks <= 0 || !V || !tau || !blk || !valid_b(b) ||
      (dtype != TQR_F32 && dtype != TQR_F64))
    return TQR_EINVAL;
  const int rows = type == DAPP ? 2 * b : b;  // rows of one block: [A; B] or C
  if (ldv < b || ldb < rows || (out && ldo < rows)) return TQR_EINVAL;
  // the batch lives in one 2b-row device matrix addressed by 32-bit buffer offsets
  if ((size_t)(dtype == TQR_F64 ? 8 : 4) * 2 * b * ((size_t)(1 + nblocks) * b) > 0x7fffffffull) return TQR_EINVAL;
  int st = check_device();
  if (st) return st;
  kfn kp, ku, kt;
  if ((st = resolve(b, dtype, &kp, &ku, &kt))) return st;
  const size_t es = dtype == TQR_F64 ? 8 : 4;
  const int mr = 2 * b, ng = b / (b < 32 ? b : 32), nstrips = (b + 63) / 64;
  const size_t nc = (size_t)(1 + nblocks) * b;
  void *dA = nullptr, *dtau = nullptr;
  double* dT = nullptr;
  Item* dit = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  std::vector<Item> items;
  items.push_back(type == DAPP ? Item{QRD, 1, 0, 0} : Item{QRS, 0, 0, 0});  // T factors of V
  for (int j = 1; j <= nblocks; ++j)
    for (int s = 0; s < nstrips; ++s) items.push_back(Item{type | (s << 8), type == DAPP ? 1 : 0, j, 0});
  auto fin = [&](int code) {
    if (dA) (void)hipFree(dA);
    if (dtau) (void)hipFree(dtau);
    if (dT) (void)hipFree(dT);
    if (dit) (void)hipFree(dit);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return code;
  };
  if (hipMalloc(&dA, es * mr * nc) != hipSuccess || hipMalloc(&dtau, es * mr) != hipSuccess ||
      hipMalloc(&dT, sizeof(double) * 2 * ng * timg_doubles(b)) != hipSuccess ||
      hipMalloc(&dit, sizeof(Item) * items.size()) != hipSuccess)
    return fin(TQR_ENOMEM);
  if (hipMemset(dA, 0, es * mr * nc) != hipSuccess || hipMemset(dtau, 0, es * mr) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
    return fin(TQR_EHIP);
  const int vrow = type == DAPP ? b : 0;  // V: tile (1,0) (TSQRT V_B) or tile (0,0) (GEQRT V)
  if (hipMemcpy2D((char*)dA + es * vrow, es * mr, V, es * ldv, es * b, b, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy((char*)dtau + es * vrow, tau, es * b, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dit, items.data(), sizeof(Item) * items.size(), hipMemcpyHostToDevice) != hipSuccess)
    return fin(TQR_EHIP);
  for (int j = 1; j <= nblocks; ++j)
    if (hipMemcpy2D((char*)dA + es * (size_t)j * b * mr, es * mr, blk, es * ldb, es * rows, b, hipMemcpyHostToDevice) != hipSuccess)
      return fin(TQR_EHIP);
  Args a;
  a.A = dA; a.tau = dtau; a.Tw = dT; a.items = dit; a.ldm = mr; a.m = mr; a.p = 2; a.kmax = 1;
  hipLaunchKernelGGL(kt, dim3(ng), dim3(NT), lds_build_t(b), 0, a);
  if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return fin(TQR_EHIP);
  a.items = dit + 1;
  if (hipEventRecord(e0, 0) != hipSuccess) return fin(TQR_EHIP);
  hipLaunchKernelGGL(ku, dim3((unsigned)(items.size() - 1)), dim3(NT), lds_update(b), 0, a);
  if (hipGetLastError() != hipSuccess || hipEventRecord(e1, 0) != hipSuccess || hipEventSynchronize(e1) != hipSuccess)
    return fin(TQR_EHIP);
  float t = 0;
  if (hipEventElapsedTime(&t, e0, e1) != hipSuccess) return fin(TQR_EHIP);
  if (ms) *ms = t;
  if (out)
    for (int j = 1; j <= nblocks; ++j)
      if (hipMemcpy2D((char*)out + es * (size_t)(j - 1) * b * ldo, es * ldo, (char*)dA + es * (size_t)j * b * mr, es * mr,
                      es * rows, b, hipMemcpyDeviceToHost) != hipSuccess)
        return fin(TQR_EHIP);
  return fin(TQR_OK);
}

}  // extern "C"

#ifdef TQR_STAMPS
extern "C" int tqr_debug_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 8) != hipSuccess) return TQR_EHIP;
  if (hipMemcpyFromSymbol(out + 8, HIP_SYMBOL(g_pstamps), sizeof(unsigned long long) * 8) != hipSuccess) return TQR_EHIP;
  if (reset) {
    unsigned long long z[8] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof z) != hipSuccess) return TQR_EHIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_pstamps), z, sizeof z) != hipSuccess) return TQR_EHIP;
  }
  return TQR_OK;
}
#endif

#ifdef TQR_FLOW_STAMPS
extern "C" int tqr_debug_flow_stamp_count(void) { return FST_N; }
// per-workgroup activity sums of the last k_flow launch (FST_N categories, flow.hpp FST)
extern "C" int tqr_debug_flow_stamps(unsigned long long* out, int nblocks) {
  if (nblocks > 4096) return TQR_EINVAL;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fst), sizeof(unsigned long long) * FST_N * nblocks) != hipSuccess) return TQR_EHIP;
  return TQR_OK;
}
// per-wave activity sums of the last k_flow launch: [workgroup][wave][WSL slots, flow.hpp]
extern "C" int tqr_debug_flow_wave_stamps(unsigned long long* out, int nblocks) {
  if (nblocks > 4096) return TQR_EINVAL;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wst), sizeof(unsigned long long) * 8 * WSL * nblocks) != hipSuccess) return TQR_EHIP;
  return TQR_OK;
}
// group trace of workgroup 0 in the last k_flow launch: [group][wave][mark] s_memrealtime (flow.hpp GTR),
// then the hand-over phase-2 marks [group][wave][8] (XPipe); `out` holds 2 x 64 x ngroups values
extern "C" int tqr_debug_group_trace(unsigned long long* out, int ngroups) {
  if (ngroups > GTR_GROUPS) return TQR_EINVAL;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gtr), sizeof(unsigned long long) * 64 * ngroups) != hipSuccess) return TQR_EHIP;
  if (hipMemcpyFromSymbol(out + 64 * (size_t)ngroups, HIP_SYMBOL(g_xtr), sizeof(unsigned long long) * 64 * ngroups) != hipSuccess)
    return TQR_EHIP;
  return TQR_OK;
}
// task timeline of the last k_flow launch: (start, end, workgroup) per task index, and the task list
extern "C" int tqr_debug_task_timeline(const tqr_plan* plan, unsigned long long* out, int ntasks, int* items) {
  if (ntasks > (1 << 18)) return TQR_EINVAL;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ttl), sizeof(unsigned long long) * 3 * ntasks) != hipSuccess) return TQR_EHIP;
  if (items && plan->d_flow && hipMemcpy(items, plan->d_flow, sizeof(Item) * ntasks, hipMemcpyDeviceToHost) != hipSuccess)
    return TQR_EHIP;
  return TQR_OK;
}
#endif
