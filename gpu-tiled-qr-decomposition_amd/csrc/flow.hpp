// Persistent dataflow engine ("flow"): one 256-thread workgroup per CU pulls tasks from a
// statically ordered list (atomic dequeue) and synchronises with other workgroups only through
// monotone progress counters in global memory (agent-scope release / acquire, CDNA4 recipe of
// MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility").
//
// Tasks (the reference DAG of src/gridscheduler.c, regrouped):
//   QRS(k)          GEQRT of tile (k,k), reflector group by group;
//   QRD(i,k)        TSQRT of [R_kk; tile (i,k)], group by group;
//   CHAIN(k,j,s,e)  one 64-column strip s of tile column j at step k: segment e of the chain
//                   UNMQR(k,j) (segment 0 only), TSMQR(i,j,k) for i in [i0,i1). The strip of
//                   tile (k,j) (the TSMQR head rows) stays owned by the chain across elements.
// Progress counters (zeroed per factorisation):
//   Rc[k][g]   members of panel k (GEQRT(k), TSQRT(k+1,k), ...) that finished group g — a
//              TSQRT's group g may start once its predecessor finished group g, so the flat
//              TS chain is pipelined at group (32-reflector) granularity, not tile granularity;
//   Tc[i][j][s] steps completed on strip s of tile (i,j);
//   Ac[k][j][s] segments completed of chain (k,j,s).
// Deadlock freedom: every wait is on a task earlier in the list (host checks it), and tasks are
// dequeued in list order, so the earliest unfinished dequeued task can always progress. Every
// spin is bounded (FLOW_TIMEOUT); on timeout an error word is set and all workgroups drain.
#pragma once
#include "tiles.hpp"

namespace tqr {

constexpr int T_CHAIN = 4;
constexpr int FLOW_NT = 256;
constexpr unsigned long long FLOW_TIMEOUT = 500000000ull;  // 5 s of s_memrealtime (100 MHz)

struct FlowArgs {
  void* A;
  void* tau;
  double* Tw;
  const Item* tasks;
  int ntasks;
  long ldm;
  int m, p, q, kmax, ns;
  int* next;
  int* err;
  int* Rc;
  int* Tc;
  int* Ac;
};

// ---- synchronisation ---------------------------------------------------------------------
__device__ __forceinline__ int ld_relaxed(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// thread 0 only: spin until *p >= target; false on error / timeout
__device__ __noinline__ bool spin_ge(int* p, int target, int* err) {
  if (ld_relaxed(p) >= target) return true;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (ld_relaxed(p) < target) {
    if (ld_relaxed(err)) return false;
    __builtin_amdgcn_s_sleep(8);
    if (__builtin_amdgcn_s_memrealtime() - t0 > FLOW_TIMEOUT) {
      __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}

// all threads: thread 0's verdict, made visible after an agent-scope acquire
__device__ __forceinline__ bool wg_acquire(bool ok0, int* sflag) {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *sflag = ok0 ? 1 : 0;
  }
  __syncthreads();
  const bool ok = *sflag != 0;
  __syncthreads();
  return ok;
}

// all threads: every wave's stores drained, then thread 0 releases and bumps the counter
__device__ __forceinline__ void wg_publish(int* p, int delta) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(p, delta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int B>
__device__ __forceinline__ double* flow_tw(const FlowArgs& a, int i, int k, int g) {
  using G = Geo<B>;
  return a.Tw + (((size_t)k * a.p + i) * G::NG + g) * (G::IB * G::IB);
}

// ---- register-staged prefetch of one reflector group (V block + T) -------------------------
template <int B>
struct GroupRegs {
  static constexpr int NV = B * Geo<B>::IB / FLOW_NT;  // V values per thread
  static constexpr int NTT = (Geo<B>::IB * Geo<B>::IB + FLOW_NT - 1) / FLOW_NT;
  double v[NV > 0 ? NV : 1];
  double t[NTT];
};

// TS-type (V_B dense) or GE-type (explicit unit lower) group g of tile `vt`
template <int B, bool GE, typename S>
__device__ __forceinline__ void group_load(GroupRegs<B>& R, const S* __restrict__ vt, size_t ldm, int c0,
                                           const double* __restrict__ tg) {
  using G = Geo<B>;
  // thread t reads rows r = (t + 256u) % B of columns c0 + (t + 256u) / B: a running pointer,
  // made opaque per step so the compiler does not keep 32 precomputed 64-bit offsets alive
  constexpr int CPS = FLOW_NT / B > 0 ? FLOW_NT / B : 1;  // columns per step (B <= 256)
  const int r = threadIdx.x % B;
  const S* pv = vt + (size_t)(c0 + threadIdx.x / B) * ldm + r;
#pragma unroll
  for (int u = 0; u < GroupRegs<B>::NV; ++u) {
    const int d = c0 + (threadIdx.x + FLOW_NT * u) / B;
    if (GE) R.v[u] = r <= d ? 0.0 : ld(pv);
    else R.v[u] = ld(pv);
    pv += (size_t)CPS * ldm;
    asm volatile("" : "+v"(pv));
  }
#pragma unroll
  for (int u = 0; u < GroupRegs<B>::NTT; ++u) {
    const int idx = threadIdx.x + FLOW_NT * u;
    R.t[u] = idx < G::IB * G::IB ? tg[idx] : 0.0;
  }
}
template <int B, bool GE>
__device__ __forceinline__ void group_commit(const GroupRegs<B>& R, double* Vs, double* Ts, int c0) {
  using G = Geo<B>;
#pragma unroll
  for (int u = 0; u < GroupRegs<B>::NV; ++u) {
    const int idx = threadIdx.x + FLOW_NT * u, r = idx % B, c = idx / B;
    Vs[r * G::VP + G::pc(c)] = (GE && r == c0 + c) ? 1.0 : R.v[u];
  }
#pragma unroll
  for (int u = 0; u < GroupRegs<B>::NTT; ++u) {
    const int idx = threadIdx.x + FLOW_NT * u;
    if (idx < G::IB * G::IB) Ts[(idx / G::IB) * G::TP + idx % G::IB] = R.t[u];
  }
}

// ---- panel tasks ---------------------------------------------------------------------------
template <int B, typename S>
__device__ void flow_panel(const FlowArgs& a, int type, int l, int k, double* lds, int* sflag) {
  using G = Geo<B>;
  constexpr int IB = G::IB, VP = G::VP, TP = G::TP, NG = G::NG;
  double* Vs = lds;
  double* Hs = Vs + G::VSZ;
  double* Ts = Hs + G::TSZ;
  double* Gs = Ts + G::TSZ;
  double* tauv = Gs + G::TSZ;
  double* scratch = tauv + IB + 2;
  double* Gp = scratch + 2 * 4 * 32 + 4 * 32 + 2 * 32 + G::TSZ;
  S* A = (S*)a.A;
  S* tau = (S*)a.tau;
  const size_t ldm = a.ldm;
  const int t = threadIdx.x, w = t >> 6;
  S* Rt = A + (size_t)k * B * ldm + (size_t)k * B;
  const bool qrs = type == QRS;
  S* Bt = qrs ? Rt : A + (size_t)k * B * ldm + (size_t)l * B;
  const int pos = qrs ? 0 : l - k;  // position in the panel chain
  // the tile(s) must have received step k-1 on every strip
  {
    bool ok = true;
    if (t == 0 && k > 0)
      for (int s = 0; s < a.ns && ok; ++s) ok = spin_ge(&a.Tc[((size_t)(qrs ? k : l) * a.q + k) * a.ns + s], k, a.err);
    if (!wg_acquire(ok, sflag)) return;
  }
  double X[G::NKS];
  double H[G::NRI];
  for (int g = 0; g < NG; ++g) {
    const int c0 = g * IB, ks0 = c0 / 4;
    if (!qrs) {  // R_kk rows of group g as left by the previous chain member
      const bool ok = t == 0 ? spin_ge(&a.Rc[(size_t)k * NG + g], pos, a.err) : true;
      if (!wg_acquire(ok, sflag)) return;
    }
    if (qrs) {
#pragma unroll 8
      for (int idx = t; idx < B * IB; idx += FLOW_NT) {
        const int r = idx % B, c = idx / B;
        Vs[r * VP + G::pc(c)] = r >= c0 ? ld(Rt + (size_t)(c0 + c) * ldm + r) : 0.0;
      }
    } else {
#pragma unroll 8
      for (int idx = t; idx < B * IB; idx += FLOW_NT) {
        const int r = idx % B, c = idx / B;
        Vs[r * VP + G::pc(c)] = ld(Bt + (size_t)(c0 + c) * ldm + r);
      }
      for (int idx = t; idx < IB * IB; idx += FLOW_NT) {
        const int r = idx % IB, c = idx / IB;
        if (r <= c) Hs[r * TP + c] = ld(Rt + (size_t)(c0 + c) * ldm + c0 + r);
      }
    }
    __syncthreads();
    if (qrs) panel_factor<B, false>(Vs, Hs, tauv, scratch, c0);
    else panel_factor<B, true>(Vs, Hs, tauv, scratch, c0);
    if (qrs) {
      for (int idx = t; idx < B * IB; idx += FLOW_NT) {
        const int r = idx % B, c = idx / B;
        if (r >= c0) st(Rt + (size_t)(c0 + c) * ldm + r, Vs[r * VP + G::pc(c)]);
      }
    } else {
      for (int idx = t; idx < B * IB; idx += FLOW_NT) {
        const int r = idx % B, c = idx / B;
        st(Bt + (size_t)(c0 + c) * ldm + r, Vs[r * VP + G::pc(c)]);
      }
      for (int idx = t; idx < IB * IB; idx += FLOW_NT) {
        const int r = idx % IB, c = idx / IB;
        if (r <= c) st(Rt + (size_t)(c0 + c) * ldm + c0 + r, Hs[r * TP + c]);
      }
    }
    if (t < IB) st(tau + (size_t)k * a.m + (size_t)(qrs ? k : l) * B + c0 + t, tauv[t]);
    __syncthreads();
    if (qrs) {
      for (int idx = t; idx < B * IB; idx += FLOW_NT) {
        const int r = idx % B, c = idx / B, d = c0 + c;
        if (r <= d) Vs[r * VP + G::pc(c)] = r == d ? 1.0 : 0.0;
      }
      __syncthreads();
    }
    build_t<B>(Vs, tauv, Gs, Ts, Gp, qrs ? ks0 : 0);
    double* tg = flow_tw<B>(a, qrs ? k : l, k, g);
    for (int idx = t; idx < IB * IB; idx += FLOW_NT) st(tg + idx, Ts[(idx / IB) * TP + idx % IB]);
    const int nstr = (B - c0 - IB) / 16;
    for (int s = w; s < nstr; s += FLOW_NT / 64) {
      asm volatile("" ::: "memory");
      const int col = c0 + IB + 16 * s;
      if (qrs) {
        load_strip<B>(X, Rt, ldm, col, ks0);
        apply_group<B, false>(Vs, Ts, X, H, ks0);
        store_strip<B>(X, Rt, ldm, col, ks0);
      } else {
        load_strip<B>(X, Bt, ldm, col, 0);
        load_head<B>(H, Rt, ldm, c0, col);
        apply_group<B, true>(Vs, Ts, X, H, 0);
        store_strip<B>(X, Bt, ldm, col, 0);
        store_head<B>(H, Rt, ldm, c0, col);
      }
    }
    wg_publish(&a.Rc[(size_t)k * NG + g], 1);
  }
}

// ---- chain tasks ---------------------------------------------------------------------------
template <int B, typename S>
__device__ void flow_chain(const FlowArgs& a, int s, int i0, int i1, int j, int k, int seg, double* lds,
                           int* sflag) {
  using G = Geo<B>;
  constexpr int IB = G::IB, NG = G::NG;
  // double-buffered V/T images: buffer b at lds + b * (VSZ + TSZ)
  auto Vb = [&](int b) { return lds + b * (G::VSZ + G::TSZ); };
  auto Tb = [&](int b) { return lds + b * (G::VSZ + G::TSZ) + G::VSZ; };
  S* A = (S*)a.A;
  const size_t ldm = a.ldm;
  const int t = threadIdx.x, w = t >> 6;
  const int col = s * 64 + 16 * w;  // this wave's 16 columns inside the tile
  const bool active = col < B;
  S* At = A + (size_t)j * B * ldm + (size_t)k * B;  // tile (k,j): the chain's head rows
  const S* Vk = A + (size_t)k * B * ldm + (size_t)k * B;
  double X[G::NKS];
  double H[G::NRI];
  GroupRegs<B> R;
  int* const tc_kj = &a.Tc[((size_t)k * a.q + j) * a.ns + s];
  int* const ac = &a.Ac[((size_t)k * a.q + j) * a.ns + s];
  int buf = 0;

  if (seg == 0) {
    // UNMQR of tile (k,j) with GEQRT(k): the strip of tile (k,j) is in X
    bool ok = t == 0 ? (k == 0 || spin_ge(tc_kj, k, a.err)) : true;
    ok = ok && (t != 0 || spin_ge(&a.Rc[(size_t)k * NG + 0], 1, a.err));
    if (!wg_acquire(ok, sflag)) return;
    if (active) load_strip<B>(X, At, ldm, col, 0);
    group_load<B, true>(R, Vk, ldm, 0, flow_tw<B>(a, k, k, 0));
    for (int g = 0; g < NG; ++g) {
      group_commit<B, true>(R, Vb(buf), Tb(buf), g * IB);
      __syncthreads();
      if (g + 1 < NG) {
        const bool okg = t == 0 ? spin_ge(&a.Rc[(size_t)k * NG + g + 1], 1, a.err) : true;
        if (!wg_acquire(okg, sflag)) return;
        group_load<B, true>(R, Vk, ldm, (g + 1) * IB, flow_tw<B>(a, k, k, g + 1));
      }
      if (active) apply_group<B, false>(Vb(buf), Tb(buf), X, H, g * IB / 4);
      buf ^= 1;
    }
    if (active) store_strip<B>(X, At, ldm, col, 0);
    __syncthreads();
  } else {
    const bool ok = t == 0 ? spin_ge(ac, seg, a.err) : true;
    if (!wg_acquire(ok, sflag)) return;
  }
  for (int i = i0; i < i1; ++i) {
    // tile (i,j) strip at step k-1, and TSQRT(i,k) group 0
    const int need = i - k + 1;
    int* tc_ij = &a.Tc[((size_t)i * a.q + j) * a.ns + s];
    bool ok = true;
    if (t == 0) {
      if (k > 0) ok = spin_ge(tc_ij, k, a.err);
      ok = ok && spin_ge(&a.Rc[(size_t)k * NG + 0], need, a.err);
    }
    if (!wg_acquire(ok, sflag)) return;
    S* Bt = A + (size_t)j * B * ldm + (size_t)i * B;
    const S* Vt = A + (size_t)k * B * ldm + (size_t)i * B;
    if (active) load_strip<B>(X, Bt, ldm, col, 0);
    group_load<B, false>(R, Vt, ldm, 0, flow_tw<B>(a, i, k, 0));
    for (int g = 0; g < NG; ++g) {
      group_commit<B, false>(R, Vb(buf), Tb(buf), g * IB);
      __syncthreads();
      if (g + 1 < NG) {
        const bool okg = t == 0 ? spin_ge(&a.Rc[(size_t)k * NG + g + 1], need, a.err) : true;
        if (!wg_acquire(okg, sflag)) return;
        group_load<B, false>(R, Vt, ldm, (g + 1) * IB, flow_tw<B>(a, i, k, g + 1));
      }
      if (active) {
        load_head<B>(H, At, ldm, g * IB, col);
        apply_group<B, true>(Vb(buf), Tb(buf), X, H, 0);
        store_head<B>(H, At, ldm, g * IB, col);
      }
      buf ^= 1;
    }
    if (active) store_strip<B>(X, Bt, ldm, col, 0);
    wg_publish(tc_ij, 1);
  }
  wg_publish(ac, 1);
}

// dynamic LDS (doubles) of the two task paths; two ints follow (task index, wait verdict)
template <int B>
constexpr int flow_lds_doubles() {
  using G = Geo<B>;
  constexpr int panel = G::VSZ + 8 * G::TSZ + G::IB + 2 + 2 * 4 * 32 + 4 * 32 + 2 * 32;
  constexpr int chain = 2 * (G::VSZ + G::TSZ);
  return panel > chain ? panel : chain;
}

template <int B, typename S>
__global__ __launch_bounds__(FLOW_NT, 1) void k_flow(FlowArgs a) {
  extern __shared__ __align__(16) double lds[];
  int* s_task = reinterpret_cast<int*>(lds + flow_lds_doubles<B>());
  int* s_flag = s_task + 1;
  for (;;) {
    if (threadIdx.x == 0) {
      int idx = __hip_atomic_fetch_add(a.next, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ld_relaxed(a.err)) idx = a.ntasks;
      *s_task = idx;
    }
    __syncthreads();
    const int idx = *s_task;
    __syncthreads();
    if (idx >= a.ntasks) break;
    const Item it = a.tasks[idx];
    const int type = it.ts & 0xff;
    if (type == T_CHAIN) {
      flow_chain<B, S>(a, (it.ts >> 8) & 0xff, it.l & 0xffff, it.l >> 16, it.m, it.k & 0xffff, it.k >> 16, lds,
                       s_flag);
    } else {
      flow_panel<B, S>(a, type, it.l, it.k, lds, s_flag);
    }
    __syncthreads();
  }
}

}  // namespace tqr
