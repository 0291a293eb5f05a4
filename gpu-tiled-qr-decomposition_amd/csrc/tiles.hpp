// Tile operations of the flat-tree tiled QR for gfx950 (CDNA4), fp64 arithmetic.
//
// The four reference tile kernels (qrdecomp.c:532 GEQRT "QRS", :559 UNMQR "SAPP",
// :689 TSQRT "QRD", :723 TSMQR "DAPP"; device versions gpucalc.cu:1013-1359) are
// re-designed around compact-WY block reflectors with inner blocking IB = 32:
//
//   * a reflector group g (IB consecutive reflectors of a tile) is applied to a column strip
//     X as   Z = [head] + V_g^T X ;  W = T_g^T Z ;  [head] -= W ;  X -= V_g W
//     with the three products on v_mfma_f64_4x4x4_4b_f64 (measured ~1.5x the issue rate of
//     v_mfma_f64_16x16x4_f64 on gfx950, profiles/r01/ubench_mfma_f64.txt);
//   * the IB-column panel of GEQRT/TSQRT is factorised in LDS, reflector by reflector, with
//     the reference's conventions (qrdecomp.c:1201-1272): sign(0) = +1, v scaled to v0 = 1
//     by the reciprocal of x0 + sign*|x|, no scaling for a zero column, tau = 2/(v'v);
//   * T_g (IB x IB upper triangular, LAPACK dlarft "forward, columnwise") is formed from the
//     Gram matrix V_g^T V_g, itself one MFMA product.
//
// Mathematically every tile op applies exactly the reflectors the reference applies, in the
// same order; only the rounding differs (parity tolerances in tests/).
//
// Register layout of a 4x4x4_4b operand (probed, profiles/r01/ubench_mfma_probe.txt):
// lane = 16*x + 4*blk + y holds A[blk][i=y][k=x], B[blk][k=x][j=y], D[blk][i=x][j=y].
// A wave owns a strip of 16 matrix columns (blk = column quad, y = column in quad); register
// X[ks] holds rows 4ks..4ks+3 of the strip (row 4ks+x at lane x), which is at the same time
// the B-operand layout (k = row) and the accumulator layout (i = row) — so the strip is both
// summed over (Z = V^T X) and updated (X -= V W) without any data movement.
#pragma once
#include <hip/hip_runtime.h>

// cache policy of the strip traffic (tile strips streamed once per step): aux bits of the buffer
// loads / stores (16 = sc1 write-through / L1 bypass, | 2 = nt streaming)
// fp64 strips: sc1 | nt loads (16384^2: 127.7 vs 128.9-129.0 ms, two A/B rounds); fp32 strips
// (the fp32 panels' trailing update) keep sc1 (nt: 481.5 vs 474.1-475.1 ms at 32768^2)
#ifndef TQR_STRIP_LD_AUX
#define TQR_STRIP_LD_AUX 18
#endif
#ifndef TQR_STRIP_LD_AUX32
#define TQR_STRIP_LD_AUX32 16
#endif
#ifndef TQR_STRIP_ST_AUX
#define TQR_STRIP_ST_AUX 16  // (nt stores: 131.1, slower)
#endif
namespace tqr {

#ifdef TQR_STAMPS
extern __device__ unsigned long long g_pstamps[8];
#define PSTAMP(i)                                                  \
  do {                                                             \
    if (threadIdx.x == 0) {                                        \
      unsigned long long n_ = __builtin_amdgcn_s_memtime();        \
      atomicAdd(&g_pstamps[i], n_ - ps_last);                      \
      ps_last = n_;                                                \
    }                                                              \
  } while (0)
#define PSTAMP_INIT unsigned long long ps_last = __builtin_amdgcn_s_memtime();
#else
#define PSTAMP(i) do {} while (0)
#define PSTAMP_INIT
#endif
// build_t phase stamps (tools/ubench/panel_bench.hip only)
#ifdef TQR_BT_STAMPS
extern __device__ unsigned long long g_bt[8];
#define BT_STAMP(i)                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(&g_bt[i], (unsigned long long)__builtin_amdgcn_s_memtime()); \
  } while (0)
#else
#define BT_STAMP(i) do {} while (0)
#endif
// reflector-step phase stamps (tools/ubench/panel_bench.hip built with -DTQR_PS_STAMPS only):
// per step, s_memtime deltas summed in registers, added to g_ps at the end of the group
#ifdef TQR_PS_STAMPS
extern __device__ unsigned long long g_ps[8];
#define PS_DECL unsigned long long ps_acc_[6] = {0, 0, 0, 0, 0, 0}, ps_t_ = 0;
#define PS_MARK(i)                                                   \
  do {                                                               \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime();      \
    if ((i) > 0) ps_acc_[(i) - 1] += n_ - ps_t_;                     \
    ps_t_ = n_;                                                      \
  } while (0)
#define PS_ARGS , ps_acc_, ps_t_
#define PS_PARAMS , unsigned long long (&ps_acc_)[6], unsigned long long& ps_t_
#define PS_FLUSH()                                                                   \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.x == 0)                                         \
      for (int i_ = 0; i_ < 6; ++i_) atomicAdd(&g_ps[i_], ps_acc_[i_]);              \
  } while (0)
#else
#define PS_DECL
#define PS_MARK(i) do {} while (0)
#define PS_ARGS
#define PS_PARAMS
#define PS_FLUSH() do {} while (0)
#endif

constexpr int NT = 256;  // threads per workgroup (4 waves)

__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

template <int B, int IB_ = (B < 32 ? B : 32)>
struct Geo {
  static constexpr int IB = IB_;              // reflectors per group (default: 32, or B if smaller)
  static constexpr int NG = B / IB;           // groups per tile
  static constexpr int NKS = B / 4;           // 4-row k-steps over a tile
  static constexpr int NRI = IB / 4;          // 4-row blocks of a group
  static constexpr int VP = IB + 2;           // LDS pitch (doubles) of the V image, 16-B rows
  static constexpr int TP = IB + 1;           // LDS pitch of T / Gram / head images
  static constexpr int VSZ = B * VP;          // V image (doubles)
  static constexpr int TSZ = IB * TP;         // T image (doubles)
  // workspace slots / LDS-DMA images, rounded up to whole KiB (128 doubles)
  static constexpr int VIMG = (VSZ + 127) / 128 * 128;
  static constexpr int TIMG = (TSZ + 127) / 128 * 128;
  // packed T image (pack_t): lane-major blocks of -T, what apply_zw<..., TPACK=true> reads
  static constexpr int TPK = 16 * NRI * NRI;
  static constexpr int TPIMG = (TPK + 127) / 128 * 128;
  // V image column permutation: the NRI values a lane needs per row are contiguous.
  __device__ static constexpr int pc(int c) { return (c & 3) * NRI + (c >> 2); }
};

// fp32 chain geometry (chain32.hpp): v_mfma_f32_16x16x4_f32 tiles of 16 strip rows (NMT per tile)
// and 16 reflectors (NMI per group). LDS / workspace images (floats):
//   VR [row R < B][IB]  V, one layout read by both phases: reflector c = 16wi + 4x + r at
//                       position 4NMI x + 4wi + r of its row (the 4 values a phase-2 lane needs
//                       are one 16-B slot), 16-B slots XOR-swizzled by sw(R) (vr_sw) so that
//                       phase 1's ds_read_b32 and phase 2's ds_read_b128 are conflict-free
//   TP [pair (mi <= wi)][lane][4]  W = -T^T Z operands -T[16mi + 4x + r][16wi + y]
// (lane = 16x + y); slots in doubles, whole KiB. (Round 2 had VA and VB, one layout per phase:
// twice the LDS-DMA bytes.)
template <int B>
struct Geo32 {
  static constexpr int IB = Geo<B>::IB, NG = Geo<B>::NG;
  static constexpr int NMT = B / 16, NMI = IB / 16, NPR = NMI * (NMI + 1) / 2;
  static constexpr int VR = B * IB, TP = NPR * 256;  // floats
  static constexpr int VIMG = VR / 2;                // doubles (multiple of 128)
  static constexpr int TIMG = (TP / 2 + 127) / 128 * 128;
  // slot swizzle of row R (IB = 32: found by exhaustive search over XOR maps of R's bits,
  // conflict-free for both phases' lane groups; IB = 16: none)
  __device__ static constexpr int vr_sw(int R) {
    return IB == 32 ? ((((R >> 1) ^ (R >> 2)) & 1) | (((R >> 3) & 1) << 2)) : 0;
  }
  // float offset of V(R, c) in the image
  __device__ static constexpr int vr_at(int R, int c) {
    const int wi = c >> 4, x = (c >> 2) & 3, r = c & 3, p = 4 * NMI * x + 4 * wi + r;
    return R * IB + (((p >> 2) ^ vr_sw(R)) << 2) + (p & 3);
  }
};
// workspace slot sizes (doubles) of one reflector group's images, by storage type: fp64 storage
// = the fp64 chain's V image + packed T; fp32 storage = the fp32 chain's VA/VB/TP images
template <int B, typename S>
struct Img {
  static constexpr int V = sizeof(S) == 8 ? Geo<B>::VIMG : Geo32<B>::VIMG;
  static constexpr int T = sizeof(S) == 8 ? Geo<B>::TPIMG : Geo32<B>::TIMG;
};

template <typename S>
__device__ __forceinline__ double ld(const S* p) { return (double)*p; }
// L1-bypassing (sc1) load: data handed over by another workgroup inside a launch, read without an
// agent-scope acquire (MI355X_MICROARCH.md, visibility "Valid forms", first table row: every
// byte stored sc1 and drained before one lane's counter add; every load of it sc1).
template <typename S>
__device__ __forceinline__ double ldc(const S* p) {
  return (double)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Global stores are write-through (sc1): results are handed to workgroups on other XCDs, and a
// release fence then has no dirty L2 lines of ours to write back (MI355X_MICROARCH.md,
// "publish-large").
template <typename S>
__device__ __forceinline__ void st(S* p, double v) {
  __hip_atomic_store(p, (S)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Sum over the workgroup; every thread gets the result. red >= 4 doubles.
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

// ---------------------------------------------------------------------------------------
// Apply reflector group g (V image Vs, T image Ts) to one wave's 16-column strip X (tile
// rows 0..B-1, registers) — (I - V T V^T)^T X.  HEAD: TS-type (V = [I; V_B], the identity
// part acting on the IB head rows H of the strip); else GE-type (V = unit-lower trapezoid
// stored explicitly, rows < 4*ks0 are zero and skipped).
// ---------------------------------------------------------------------------------------
// Phase 1: Z = [H] + V^T X, W = -T^T Z, H += W (TS). Phase 2: X += V W.
// hook.step(m) is called once per two k-steps of phase 1 (m = 0, 1, ...) inside the MFMA
// stream, then for the remaining m < Hook::STEPS after the loop: the chain engine issues the
// next group's LDS-DMA there (flow.hpp), so its issue cost hides under the MFMAs.
// LDS operand addressing: the byte address of p as an opaque 32-bit value (the optimizer cannot
// re-derive it per use), and a 16-B read at such an address
typedef double d2v_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const d2v_t lds_cd2_t;
__device__ __forceinline__ unsigned lds_base(const double* p) {
  unsigned a = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
  asm volatile("" : "+v"(a));
  return a;
}
__device__ __forceinline__ d2v_t lds_rd2(unsigned a) { return *(lds_cd2_t*)(size_t)a; }

struct NoHook {
  __device__ __forceinline__ void step(int) const {}
  __device__ __forceinline__ void mid() const {}  // between Z and W (activity stamps)
  static constexpr int STEPS = 0;
};
// PF: software-pipelined LDS operand reads (needed at one wave per SIMD; at two waves per SIMD
// the other wave hides the latency and the registers are better spent elsewhere)
// TPACK: Ts is the packed image of pack_t (W = -T^T Z as NRI batches of independent MFMAs with
// 16-B operand reads one batch ahead) instead of the row-major T (one 8-B read per MFMA).
// Paired reflector order of the fp64 chain's images (PAIRH): MFMA block r = 2h + e, lane row x
// <-> reflector 8h + 2x + e of the group, so a lane's head registers H[2h], H[2h+1] are two
// consecutive head rows (one 16-B access, as the strips). The relabelling is a permutation of the
// group's reflectors: T becomes block-upper-triangular at 8-reflector granularity, so W = -T^T Z
// needs the k-blocks kb >= (wi & ~1) instead of kb >= wi (40 instead of 36 MFMAs per group).
__device__ __forceinline__ constexpr int sigp(int r, int x) { return 8 * (r >> 1) + 2 * x + (r & 1); }
template <int B, bool HEAD, typename Hook = NoHook, bool PF = true, bool TPACK = false, bool PAIRH = false,
          int IBX = Geo<B>::IB>
__device__ __forceinline__ void apply_zw(const double* __restrict__ Vs, const double* __restrict__ Ts,
                                         const double (&X)[Geo<B>::NKS], double (&H)[Geo<B, IBX>::NRI],
                                         double (&W)[Geo<B, IBX>::NRI], int ks0, const Hook& hook = Hook()) {
  using g = Geo<B, IBX>;
  constexpr int NRI = g::NRI, NKS = g::NKS, VP = g::VP, TP = g::TP;
  const int lane = threadIdx.x & 63, x = lane >> 4, y = lane & 3;
  double Z[NRI];
#pragma unroll
  for (int r = 0; r < NRI; ++r) Z[r] = HEAD ? H[r] : 0.0;
  // Z += V^T X   (A operand: V[4ks+x][4ri+y]); software-pipelined: the LDS reads of k-step
  // ks+1 are issued ahead of the MFMAs of ks (one wave per SIMD cannot hide LDS latency
  // otherwise; tools/ubench/apply_bench.hip: 73 % -> 83 % of peak)
  // one opaque lane base + a per-k-step constant (immediate offsets): left to the optimizer the
  // row index was re-formed per k-step as (4ks | x), some of those products were kept in VGPRs,
  // spilled, and their reloads inside the MFMA stream waited (vmcnt(0)) for the LDS-DMA
  const unsigned vz = lds_base(Vs + x * VP + y * NRI);
  auto ldz = [&](double (&a)[NRI], int ks) {
#pragma unroll
    for (int h = 0; h < NRI / 2; ++h) {
      const d2v_t t = lds_rd2(vz + (unsigned)((4 * ks * VP + 2 * h) * sizeof(double)));
      a[2 * h] = t.x;
      a[2 * h + 1] = t.y;
    }
  };
  double ac[NRI], an[NRI];
  if (PF) ldz(ac, HEAD ? 0 : ks0);
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    // one k-step per scheduling region: the memory clobber bounds the LDS reads, the
    // sched_barrier the MFMAs (left free, the scheduler pulls the next k-step's MFMAs up against
    // their just-issued operand reads and every wait becomes lgkmcnt(0))
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    if ((ks & 1) == 0) hook.step(ks / 2);
    if (!HEAD && ks < ks0) continue;
    if (!PF) ldz(ac, ks);
    else if (ks + 1 < NKS) ldz(an, ks + 1);
#pragma unroll
    for (int r = 0; r < NRI; ++r) Z[r] = mfma4(ac[r], X[ks], Z[r]);
    if (PF) {
#pragma unroll
      for (int r = 0; r < NRI; ++r) ac[r] = an[r];
    }
  }
  for (int m = NKS / 2; m < Hook::STEPS; ++m) hook.step(m);
  hook.mid();
  if constexpr (TPACK) {
    // W = -T^T Z, k-block by k-block: batch kb is the NRI - kb independent MFMAs W[wi] +=
    // (-T)[kb-block][wi-block]^T Z[kb], wi >= kb; its operands (the lane's NRI values of
    // block row kb, contiguous in the packed image) are read while batch kb-1 runs.
    auto ldt = [&](double (&a)[NRI], int kb) {
      const double2* tr = reinterpret_cast<const double2*>(Ts + ((kb * 4 + x) * 4 + y) * NRI);
#pragma unroll
      for (int h = 0; h < NRI / 2; ++h) {
        const double2 v = tr[h];
        a[2 * h] = v.x;
        a[2 * h + 1] = v.y;
      }
    };
    double tc[NRI], tn[NRI];
    ldt(tc, 0);
#pragma unroll
    for (int kb = 0; kb < NRI; ++kb) {
      __builtin_amdgcn_sched_barrier(0);
      if (kb + 1 < NRI) ldt(tn, kb + 1);
#pragma unroll
      for (int wi = PAIRH ? (kb & ~1) : kb; wi < NRI; ++wi) W[wi] = mfma4(tc[wi], Z[kb], kb == 0 ? 0.0 : W[wi]);
#pragma unroll
      for (int r = 0; r < NRI; ++r) tc[r] = tn[r];
    }
  } else {
    // W = -T^T Z   (A operand: T[4k2+x][4wi+y]); T upper triangular -> k2 <= wi.
#pragma unroll
    for (int wi = 0; wi < NRI; ++wi) {
      double acc = 0.0;
#pragma unroll
      for (int k2 = 0; k2 <= wi; ++k2) acc = mfma4(Ts[(4 * k2 + x) * TP + 4 * wi + y], Z[k2], acc);
      W[wi] = -acc;
    }
  }
  if (HEAD) {
#pragma unroll
    for (int r = 0; r < NRI; ++r) H[r] += W[r];
  }
}

// Post hook of apply_x: at(h, X) runs after the MFMAs of row pair h (X[2h], X[2h+1] final once
// they retire), fin(X) after the loop — the chain streams its strip out / the next one in there.
struct NoPost {
  template <typename XA>
  __device__ __forceinline__ void at(int, XA&) const {}
  template <typename XA>
  __device__ __forceinline__ void fin(XA&) const {}
};
template <int B, bool HEAD, bool PF = true, typename Hook = NoHook, typename Post = NoPost, int IBX = Geo<B>::IB>
__device__ __forceinline__ void apply_x(const double* __restrict__ Vs, double (&X)[Geo<B>::NKS],
                                        const double (&W)[Geo<B, IBX>::NRI], int ks0, const Hook& hook = Hook(),
                                        const Post& post = Post()) {
  using g = Geo<B, IBX>;
  constexpr int NRI = g::NRI, NKS = g::NKS, VP = g::VP;
  const int lane = threadIdx.x & 63, x = lane >> 4, y = lane & 3;
  // X += V W   (A operand: V[4ks+y][4wi+x]); two k-steps per region, next pair's reads ahead.
  const unsigned vx = lds_base(Vs + y * VP + x * NRI);  // (see apply_zw)
  auto ldx = [&](double (&a)[NRI], int ks) {
#pragma unroll
    for (int h = 0; h < NRI / 2; ++h) {
      const d2v_t t = lds_rd2(vx + (unsigned)((4 * ks * VP + 2 * h) * sizeof(double)));
      a[2 * h] = t.x;
      a[2 * h + 1] = t.y;
    }
  };
  double bc[2][NRI], bn[2][NRI];
  const int kx = HEAD ? 0 : (ks0 & ~1);
  if (PF) {
    ldx(bc[0], kx);
    ldx(bc[1], kx + 1);
  }
#pragma unroll
  for (int kb = 0; kb < NKS; kb += 2) {
    __builtin_amdgcn_sched_barrier(0);  // (see apply_zw)
    asm volatile("" ::: "memory");
    hook.step(kb / 2);
    if (!HEAD && kb + 1 < ks0) continue;
    if (!PF) {
      ldx(bc[0], kb);
      ldx(bc[1], kb + 1);
    } else if (kb + 2 < NKS) {
      ldx(bn[0], kb + 2);
      ldx(bn[1], kb + 3);
    }
#pragma unroll
    for (int wi = 0; wi < NRI; ++wi)
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (HEAD || kb + u >= ks0) X[kb + u] = mfma4(bc[u][wi], W[wi], X[kb + u]);
    if (PF) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < NRI; ++r) bc[u][r] = bn[u][r];
    }
    post.at(kb / 2, X);
  }
  post.fin(X);
  for (int m = NKS / 2; m < Hook::STEPS; ++m) hook.step(m);
}

// Chain form of phase 2 (TS-type, all k-steps): X += V W over blocks of 4 k-steps, the group's
// reflectors in two halves, so 4 independent accumulation chains are interleaved (the 4x4x4 f64
// form's dependent latency is ~40 cycles, 2.5 instructions: with apply_x's 2 chains a wave alone
// on its SIMD issues at 64 %, with 3-4 at 93-96 %, profiles/r02/ubench_mfma_f64_latency.txt —
// the end of every group, when one wave of a pair has finished, runs on one wave). Operand
// registers as apply_x: 4 k-steps x NRI/2 values, the next half read ahead.
template <int B, typename Post = NoPost, int IBX = Geo<B>::IB>
__device__ __forceinline__ void apply_x4(const double* __restrict__ Vs, double (&X)[Geo<B>::NKS],
                                         const double (&W)[Geo<B, IBX>::NRI], const Post& post = Post()) {
  using g = Geo<B, IBX>;
  constexpr int NRI = g::NRI, NKS = g::NKS, VP = g::VP, NH = NRI / 2;
  static_assert(NKS % 4 == 0 && NH % 2 == 0, "apply_x4 blocks");
  const int lane = threadIdx.x & 63, x = lane >> 4, y = lane & 3;
  const unsigned vx = lds_base(Vs + y * VP + x * NRI);  // (see apply_zw)
  auto ldh = [&](double (&a)[4][NH], int kb, int half) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < NH / 2; ++q) {
        const d2v_t t = lds_rd2(vx + (unsigned)((4 * (kb + u) * VP + half * NH + 2 * q) * sizeof(double)));
        a[u][2 * q] = t.x;
        a[u][2 * q + 1] = t.y;
      }
  };
  double oc[4][NH], on[4][NH];
  ldh(oc, 0, 0);
#pragma unroll
  for (int kb = 0; kb < NKS; kb += 4) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      __builtin_amdgcn_sched_barrier(0);  // (see apply_zw)
      asm volatile("" ::: "memory");
      if (half == 0) ldh(on, kb, 1);
      else if (kb + 4 < NKS) ldh(on, kb + 4, 0);
#pragma unroll
      for (int q = 0; q < NH; ++q)
#pragma unroll
        for (int u = 0; u < 4; ++u) X[kb + u] = mfma4(oc[u][q], W[half * NH + q], X[kb + u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < NH; ++q) oc[u][q] = on[u][q];
    }
    post.at(kb / 2, X);
    post.at(kb / 2 + 1, X);
  }
  post.fin(X);
}

template <int B, bool HEAD, bool PF = true, bool TPACK = false, int IBX = Geo<B>::IB>
__device__ __forceinline__ void apply_group(const double* __restrict__ Vs, const double* __restrict__ Ts,
                                            double (&X)[Geo<B>::NKS], double (&H)[Geo<B, IBX>::NRI], int ks0) {
  double W[Geo<B, IBX>::NRI];
  apply_zw<B, HEAD, NoHook, PF, TPACK, false, IBX>(Vs, Ts, X, H, W, ks0);
  apply_x<B, HEAD, PF, NoHook, NoPost, IBX>(Vs, X, W, ks0);
}

// Strip loads/stores: X[ks] <- tile(rows 4ks+x, column col0 + 4blk + y).
// SC1: L1-bypassing loads (data another workgroup of the same launch stored, see ldc)
template <int B, typename S, bool SC1 = false>
__device__ __forceinline__ void load_strip(double (&X)[Geo<B>::NKS], const S* __restrict__ tile, size_t ldm,
                                           int col0, int ks0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = col0 + (lane & 15);
  const S* p = tile + (size_t)c * ldm + x;
#pragma unroll
  for (int ks = 0; ks < Geo<B>::NKS; ++ks) X[ks] = ks >= ks0 ? (SC1 ? ldc(p + 4 * ks) : ld(p + 4 * ks)) : 0.0;
}
template <int B, typename S>
__device__ __forceinline__ void store_strip(const double (&X)[Geo<B>::NKS], S* __restrict__ tile, size_t ldm,
                                            int col0, int ks0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = col0 + (lane & 15);
  S* p = tile + (size_t)c * ldm + x;
#pragma unroll
  for (int ks = 0; ks < Geo<B>::NKS; ++ks)
    if (ks >= ks0) st(p + 4 * ks, X[ks]);
}
// Head rows of group g: H[ri] <- tile(row r0 + 4ri + x, column col0 + 4blk + y).
template <int B, typename S, bool SC1 = false>
__device__ __forceinline__ void load_head(double (&H)[Geo<B>::NRI], const S* __restrict__ tile, size_t ldm,
                                          int r0, int col0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = col0 + (lane & 15);
  const S* p = tile + (size_t)c * ldm + r0 + x;
#pragma unroll
  for (int r = 0; r < Geo<B>::NRI; ++r) H[r] = SC1 ? ldc(p + 4 * r) : ld(p + 4 * r);
}

// Chain strips in the paired row map: X[2h + e] at lane x <-> tile row 8h + 2x + e, so a lane
// moves two consecutive rows of its column per (16-B for fp64) access. The chain's V images are
// stored with their rows permuted to match (vimg_row). Loads and stores are sc1 buffer accesses
// (L1-bypassing / write-through: inter-workgroup hand-off without acquire/release fences).
// buffer descriptor over a wave-uniform base: readfirstlane makes the uniformity provable, else
// hipcc wraps every buffer access in a waterfall loop (cdna_hip_programming.md T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p) {
  const unsigned long long u = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ int vimg_row(int q) { return 8 * (q >> 3) + 2 * (q & 3) + ((q >> 2) & 1); }
// inverse: tile row r -> image row
__device__ __forceinline__ int vimg_inv(int r) { return 8 * (r >> 3) + 4 * (r & 1) + ((r >> 1) & 3); }
// h0: 8-row blocks above it are neither loaded (zero) nor stored (the GEQRT panel's finished
// R rows, which other members' trailing updates may be writing meanwhile)
// The resource is based at the strip's first column (wave-uniform), so the 32-bit offsets span
// 16 columns only: ldm * sizeof(S) * 16 < 2^31 (checked by tqr_plan_create / execute).
template <int B, typename S>
__device__ __forceinline__ void load_strip_pair(double (&X)[Geo<B>::NKS], S* tile, size_t ldm, int col0, int h0 = 0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = lane & 15;
  __amdgpu_buffer_rsrc_t rs = uniform_rsrc(tile + (size_t)col0 * ldm);
  const unsigned base = (unsigned)(((size_t)c * ldm + 2 * x) * sizeof(S));
  // per-access displacement in the scalar offset (one VGPR offset for the whole strip: an
  // unsigned voffset + constant cannot be folded into the immediate field without a no-wrap proof)
#pragma unroll
  for (int h = 0; h < Geo<B>::NKS / 2; ++h) {
    if (h < h0) {
      X[2 * h] = X[2 * h + 1] = 0.0;
      continue;
    }
    const int so = 8 * h * sizeof(S);
    if constexpr (sizeof(S) == 8) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, base, so, TQR_STRIP_LD_AUX);
      X[2 * h] = __longlong_as_double(((long long)v[1] << 32) | v[0]);
      X[2 * h + 1] = __longlong_as_double(((long long)v[3] << 32) | v[2]);
    } else {
      auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, base, so, TQR_STRIP_LD_AUX32);
      X[2 * h] = (double)__uint_as_float(v[0]);
      X[2 * h + 1] = (double)__uint_as_float(v[1]);
    }
  }
}
template <int B, typename S>
__device__ __forceinline__ void store_strip_pair(const double (&X)[Geo<B>::NKS], S* tile, size_t ldm, int col0,
                                                 int h0 = 0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = lane & 15;
  __amdgpu_buffer_rsrc_t rs = uniform_rsrc(tile + (size_t)col0 * ldm);
  const unsigned base = (unsigned)(((size_t)c * ldm + 2 * x) * sizeof(S));
#pragma unroll
  for (int h = 0; h < Geo<B>::NKS / 2; ++h) {
    if (h < h0) continue;
    const int so = 8 * h * sizeof(S);
    if constexpr (sizeof(S) == 8) {
      const unsigned long long a = (unsigned long long)__double_as_longlong(X[2 * h]);
      const unsigned long long b = (unsigned long long)__double_as_longlong(X[2 * h + 1]);
      __attribute__((ext_vector_type(4))) unsigned v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, base, so, TQR_STRIP_ST_AUX);
    } else {
      __attribute__((ext_vector_type(2))) unsigned v = {__float_as_uint((float)X[2 * h]), __float_as_uint((float)X[2 * h + 1])};
      __builtin_amdgcn_raw_buffer_store_b64(v, rs, base, so, TQR_STRIP_ST_AUX);
    }
  }
}
// The same fp64 strip stored as full 128-B lines by 8 consecutive lanes (round 6): the MFMA layout
// above puts a column's four lanes 16 apart, and the CU's store path does not merge lanes that are
// not adjacent — 256 KiB per CU of strip stores take 7.1 us that way and 3.0 us with the row pairs
// first moved across lanes by ds_bpermute (tools/ubench/vmem_pattern.hip, profiles/r06/vmem/).
// Store q, half h: lane L = 8 c + r writes column 8 h + c, rows 16 q + 2 r, + 1 — row pair 2 q + (r >> 2)
// of lane ((r & 3) << 4) | (8 h + c). Loads need no such move (they merge at any lane order).
template <int B>
__device__ __forceinline__ void store_strip_coal(const double (&X)[Geo<B>::NKS], double* tile, size_t ldm, int col0,
                                                 int h0 = 0) {
  const int lane = threadIdx.x & 63, c = lane >> 3, r = lane & 7;
  __amdgpu_buffer_rsrc_t rs = uniform_rsrc(tile + (size_t)col0 * ldm);
  const unsigned base = (unsigned)(((size_t)c * ldm + 2 * r) * sizeof(double));
  const int hoff = __builtin_amdgcn_readfirstlane((int)(8 * ldm * sizeof(double)));
  const int src = 4 * (((r & 3) << 4) | c);
  const bool hi = (r & 4) != 0;
  typedef __attribute__((ext_vector_type(4))) unsigned v4u;
#pragma unroll
  for (int q = 0; q < Geo<B>::NKS / 4; ++q) {
    if (2 * q < h0) continue;  // (h0 even: the GEQRT panel's 8-row blocks above its group)
    unsigned w0[4], w1[4];
    const unsigned long long a0 = (unsigned long long)__double_as_longlong(X[4 * q]);
    const unsigned long long a1 = (unsigned long long)__double_as_longlong(X[4 * q + 1]);
    const unsigned long long b0 = (unsigned long long)__double_as_longlong(X[4 * q + 2]);
    const unsigned long long b1 = (unsigned long long)__double_as_longlong(X[4 * q + 3]);
    w0[0] = (unsigned)a0; w0[1] = (unsigned)(a0 >> 32); w0[2] = (unsigned)a1; w0[3] = (unsigned)(a1 >> 32);
    w1[0] = (unsigned)b0; w1[1] = (unsigned)(b0 >> 32); w1[2] = (unsigned)b1; w1[3] = (unsigned)(b1 >> 32);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      v4u v;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const unsigned x0 = (unsigned)__builtin_amdgcn_ds_bpermute(src + 32 * h, (int)w0[d]);
        const unsigned x1 = (unsigned)__builtin_amdgcn_ds_bpermute(src + 32 * h, (int)w1[d]);
        v[d] = hi ? x1 : x0;
      }
      __builtin_amdgcn_raw_buffer_store_b128(v, rs, base, h * hoff + 128 * q, TQR_STRIP_ST_AUX);
    }
  }
}
// Head rows through a buffer resource (chain engine): base = byte offset of (row r0 + x,
// column col0 + 4blk + y); soffset carries 4 rows per access. A resource with num_records = 0
// makes every load return 0 and drops every store — the branch-free "no head" of the UNMQR
// element (flow_chain).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t head_rsrc(const void* p, bool on) {
  const unsigned long long u = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  const int n = __builtin_amdgcn_readfirstlane(on ? 0x7fffffff : 0);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, n, 0x00020000);
}
// byte offset of (row r0 + x, column 4blk + y) relative to a resource based at the strip's
// first column (head_rsrc(tile + col0 * ldm, ...))
template <int B, typename S>
__device__ __forceinline__ unsigned head_off(size_t ldm, int r0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = lane & 15;
  return (unsigned)(((size_t)c * ldm + r0 + x) * sizeof(S));
}
template <int B, typename S, int AUX, int IBX = Geo<B>::IB, int NRI_ = Geo<B, IBX>::NRI>
__device__ __forceinline__ void load_head_buf(double (&H)[NRI_], __amdgpu_buffer_rsrc_t rs, unsigned base) {
#pragma unroll
  for (int r = 0; r < NRI_; ++r) {
    if constexpr (sizeof(S) == 8) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, base, 4 * r * 8, AUX);
      H[r] = __longlong_as_double((long long)(((unsigned long long)v[1] << 32) | v[0]));
    } else {
      H[r] = (double)__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, base, 4 * r * 4, AUX));
    }
  }
}
template <int B, typename S, int AUX, int IBX = Geo<B>::IB, int NRI_ = Geo<B, IBX>::NRI>
__device__ __forceinline__ void store_head_buf(const double (&H)[NRI_], __amdgpu_buffer_rsrc_t rs, unsigned base) {
#pragma unroll
  for (int r = 0; r < NRI_; ++r) {
    if constexpr (sizeof(S) == 8) {
      const unsigned long long u = (unsigned long long)__double_as_longlong(H[r]);
      __attribute__((ext_vector_type(2))) unsigned v = {(unsigned)u, (unsigned)(u >> 32)};
      __builtin_amdgcn_raw_buffer_store_b64(v, rs, base, 4 * r * 8, AUX);
    } else {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)H[r]), rs, base, 4 * r * 4, AUX);
    }
  }
}
// Head rows of one group in the paired order (fp64 chain, PAIRH): H[2h + e] at lane x <-> row
// r0 + 8h + 2x + e, column 4blk + y; base = head_off_pair (16-B aligned), 8 rows per access.
template <int B>
__device__ __forceinline__ unsigned head_off_pair(size_t ldm, int r0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = lane & 15;
  return (unsigned)(((size_t)c * ldm + r0 + 2 * x) * sizeof(double));
}
template <int B, int AUX, int IBX = Geo<B>::IB, int NRI_ = Geo<B, IBX>::NRI>
__device__ __forceinline__ void load_head_pair(double (&H)[NRI_], __amdgpu_buffer_rsrc_t rs, unsigned base) {
#pragma unroll
  for (int h = 0; h < Geo<B, IBX>::NRI / 2; ++h) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, base, 8 * h * 8, AUX);
    H[2 * h] = __longlong_as_double((long long)(((unsigned long long)v[1] << 32) | v[0]));
    H[2 * h + 1] = __longlong_as_double((long long)(((unsigned long long)v[3] << 32) | v[2]));
  }
}
template <int B, int AUX, int IBX = Geo<B>::IB, int NRI_ = Geo<B, IBX>::NRI>
__device__ __forceinline__ void store_head_pair(const double (&H)[NRI_], __amdgpu_buffer_rsrc_t rs, unsigned base) {
#pragma unroll
  for (int h = 0; h < Geo<B, IBX>::NRI / 2; ++h) {
    const unsigned long long a = (unsigned long long)__double_as_longlong(H[2 * h]);
    const unsigned long long b = (unsigned long long)__double_as_longlong(H[2 * h + 1]);
    __attribute__((ext_vector_type(4))) unsigned v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, base, 8 * h * 8, AUX);
  }
}
// Natural-order strip through a buffer resource (the panel's in-tile trailing update):
// X[ks] <- tile(row 4ks + x, column col0 + 4blk + y), rows < 4*ks0 zero (not loaded / stored).
// Buffer (not FLAT) accesses keep the LDS counter free for the MFMA operand waits.
template <int B, typename S, int AUX>
__device__ __forceinline__ void load_strip_buf(double (&X)[Geo<B>::NKS], __amdgpu_buffer_rsrc_t rs, unsigned base,
                                               int ks0) {
#pragma unroll
  for (int ks = 0; ks < Geo<B>::NKS; ++ks) {
    if (ks < ks0) {
      X[ks] = 0.0;
    } else if constexpr (sizeof(S) == 8) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, base, 4 * ks * 8, AUX);
      X[ks] = __longlong_as_double((long long)(((unsigned long long)v[1] << 32) | v[0]));
    } else {
      X[ks] = (double)__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, base, 4 * ks * 4, AUX));
    }
  }
}
template <int B, typename S, int AUX>
__device__ __forceinline__ void store_strip_buf(const double (&X)[Geo<B>::NKS], __amdgpu_buffer_rsrc_t rs, unsigned base,
                                                int ks0) {
#pragma unroll
  for (int ks = 0; ks < Geo<B>::NKS; ++ks) {
    if (ks < ks0) continue;
    if constexpr (sizeof(S) == 8) {
      const unsigned long long u = (unsigned long long)__double_as_longlong(X[ks]);
      __attribute__((ext_vector_type(2))) unsigned v = {(unsigned)u, (unsigned)(u >> 32)};
      __builtin_amdgcn_raw_buffer_store_b64(v, rs, base, 4 * ks * 8, AUX);
    } else {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)X[ks]), rs, base, 4 * ks * 4, AUX);
    }
  }
}
template <int B, typename S>
__device__ __forceinline__ void store_head(const double (&H)[Geo<B>::NRI], S* __restrict__ tile, size_t ldm,
                                           int r0, int col0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = col0 + (lane & 15);
  S* p = tile + (size_t)c * ldm + r0 + x;
#pragma unroll
  for (int r = 0; r < Geo<B>::NRI; ++r) st(p + 4 * r, H[r]);
}
template <int B, typename S>
__device__ __forceinline__ void store_head_plain(const double (&H)[Geo<B>::NRI], S* __restrict__ tile, size_t ldm,
                                                 int r0, int col0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = col0 + (lane & 15);
  S* p = tile + (size_t)c * ldm + r0 + x;
#pragma unroll
  for (int r = 0; r < Geo<B>::NRI; ++r) p[4 * r] = (S)H[r];
}

// ---------------------------------------------------------------------------------------
// LDS staging of a reflector group.
// ---------------------------------------------------------------------------------------
// TS-type: Vs[r][c] = V_B[r][c0+c] of a TSQRT tile (dense B x IB block).
template <int B, typename S>
__device__ __forceinline__ void stage_v_ts(double* Vs, const S* __restrict__ vt, size_t ldm, int c0) {
  using g = Geo<B>;
#pragma unroll 8
  for (int idx = threadIdx.x; idx < B * g::IB; idx += NT) {
    int r = idx % B, c = idx / B;
    Vs[r * g::VP + g::pc(c)] = ld(vt + (size_t)(c0 + c) * ldm + r);
  }
}
// GE-type: explicit unit-lower trapezoid of a GEQRT tile: 0 above row c0+c, 1 on it.
template <int B, typename S>
__device__ __forceinline__ void stage_v_ge(double* Vs, const S* __restrict__ vt, size_t ldm, int c0) {
  using g = Geo<B>;
#pragma unroll 8
  for (int idx = threadIdx.x; idx < B * g::IB; idx += NT) {
    int r = idx % B, c = idx / B, d = c0 + c;
    Vs[r * g::VP + g::pc(c)] = r < d ? 0.0 : (r == d ? 1.0 : ld(vt + (size_t)d * ldm + r));
  }
}
// T workspace slot (Tw): the T image itself, T[r][c] at r * TP + c, padded to whole KiB so the
// chain engine copies it verbatim by LDS-DMA.
template <int B>
__device__ __forceinline__ void stage_t(double* Ts, const double* __restrict__ tg) {
  using g = Geo<B>;
  for (int idx = threadIdx.x; idx < g::IB * g::TP; idx += NT) Ts[idx] = tg[idx];
}

// Packed T image: Tp[((kb * 4 + x) * 4 + y) * NRI + wi] = -T[4kb + x][4wi + y] (0 for wi < kb),
// i.e. the A operands of W = -T^T Z for lane (x, y) and k-block kb, contiguous over wi.
template <int B, int NTH, int IBX = Geo<B>::IB>
__device__ __forceinline__ void pack_t(const double* Ts, double* Tp) {
  using g = Geo<B, IBX>;
  constexpr int NRI = g::NRI;
  for (int idx = threadIdx.x; idx < g::TPIMG; idx += NTH) {
    const int wi = idx % NRI, y = (idx / NRI) & 3, x = (idx / (4 * NRI)) & 3, kb = idx / (16 * NRI);
    Tp[idx] = idx < g::TPK && kb <= wi ? -Ts[(4 * kb + x) * g::TP + 4 * wi + y] : 0.0;
  }
}

// ---------------------------------------------------------------------------------------
// Wave-level reduce-scatter of N (power of two, <= 32) per-lane values: on return lane l holds
// the sum over the 64 lanes of value index  (l >> (6 - log2 N)) & (N - 1)... see rs_col().
// Cost: N - 1 + (6 - log2 N) shuffles instead of 6N for N independent butterflies.
// ---------------------------------------------------------------------------------------
// Cross-lane exchange primitives (VALU, no LDS): v_permlane32_swap / v_permlane16_swap and
// DPP row_mirror / row_half_mirror / quad_perm.
__device__ __forceinline__ double dbl_of(unsigned lo, unsigned hi) {
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// a[32..63] <-> b[0..31]  (per 32-bit half)
__device__ __forceinline__ void swap32(double& a, double& b) {
  const unsigned long long ua = (unsigned long long)__double_as_longlong(a);
  const unsigned long long ub = (unsigned long long)__double_as_longlong(b);
  auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
  auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
  a = dbl_of(lo[0], hi[0]);
  b = dbl_of(lo[1], hi[1]);
}
// odd 16-lane rows of a <-> even rows of b
__device__ __forceinline__ void swap16(double& a, double& b) {
  const unsigned long long ua = (unsigned long long)__double_as_longlong(a);
  const unsigned long long ub = (unsigned long long)__double_as_longlong(b);
  auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ua, (unsigned)ub, false, false);
  auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
  a = dbl_of(lo[0], hi[0]);
  b = dbl_of(lo[1], hi[1]);
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  return __builtin_amdgcn_update_dpp(0.0, v, CTRL, 0xf, 0xf, false);
}
constexpr int DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141, DPP_QUAD_3210 = 0x1B, DPP_QUAD_1032 = 0xB1;

// One halving stage on lane-pairs given by a DPP mirror: lanes with `up` keep the upper half.
template <int CTRL, int H>
__device__ __forceinline__ void dpp_halve(const double* v, double* out, bool up) {
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const double send = up ? v[i] : v[i + H];
    const double keep = up ? v[i + H] : v[i];
    out[i] = keep + dpp<CTRL>(send);
  }
}

// Reduce-scatter of N = 32 or 16 per-lane doubles over the wave: on return lane l holds the
// wave sum of value index rs_col<N>(l). Stages pair lanes l^32 and l^16 with permlane swaps
// (no selects), then mirror partners inside 16-, 8- and 4-lane groups by DPP.
template <int N>
struct RS {
  __device__ static __forceinline__ double run(double (&v)[N], int lane) {
    static_assert(N == 32 || N == 16 || N == 8, "window of 8, 16 or 32 columns");
    constexpr int H1 = N / 2, H2 = N / 4, H3 = N / 8;
#pragma unroll
    for (int i = 0; i < H1; ++i) {
      double a = v[i], b = v[i + H1];
      swap32(a, b);
      v[i] = a + b;  // lanes < 32: index i, lanes >= 32: index i + H1
    }
#pragma unroll
    for (int i = 0; i < H2; ++i) {
      double a = v[i], b = v[i + H2];
      swap16(a, b);
      v[i] = a + b;
    }
    double c[H3 > 0 ? H3 : 1];
    dpp_halve<DPP_ROW_MIRROR, H3>(v, c, lane & 8);
    double e;
    if constexpr (N == 32) {
      double d2[2];
      dpp_halve<DPP_ROW_HALF_MIRROR, 2>(c, d2, lane & 4);
      double d1[1];
      dpp_halve<DPP_QUAD_3210, 1>(d2, d1, lane & 2);
      e = d1[0];
    } else if constexpr (N == 8) {
      e = c[0];
      e += dpp<DPP_ROW_HALF_MIRROR>(e);
      e += dpp<DPP_QUAD_3210>(e);
    } else {
      double d1[1];
      dpp_halve<DPP_ROW_HALF_MIRROR, 1>(c, d1, lane & 4);
      e = d1[0];
      e += dpp<DPP_QUAD_3210>(e);
    }
    e += dpp<DPP_QUAD_1032>(e);
    return e;
  }
};
template <int N>
__device__ __forceinline__ int rs_col(int lane) {
  // bit for xor 32 is the top index bit, then xor 16, ...
  int c = 0;
#pragma unroll
  for (int k = 0, X = 32; (1 << k) < N; ++k, X >>= 1) c = (c << 1) | ((lane & X) ? 1 : 0);
  return c;
}

// ---------------------------------------------------------------------------------------
// Panel factorisation of reflector group g (all NT threads; row-per-thread registers).
// On entry Vs holds the panel's B tile rows (perm layout; GE: rows >= c0 used), and for TS
// Hs holds the IB x IB head block R[c0.., c0..] (upper part used). Thread t owns panel row t.
// Per reflector c ONE workgroup reduction gives the raw dots D_j = x_c . x_j (tail rows,
// j >= c); D_c is the squared tail norm, so
//   norm = sqrt(x0^2 + D_c), v = x_c / (x0 + sign(x0) norm)  [no scaling if norm == 0],
//   tau = 2 / (1 + |v|^2),  d_j = head_j + v . x_j,  x_j -= tau d_j v,  head_j -= tau d_j
// — the reference's reflector (qrdecomp.c:1201-1272, 647-687) with its sums regrouped.
// On exit: Vs rows hold R (GE head rows) / V (tails) in place, Hs (TS) the updated head block,
// tauv[c] = tau_c. scratch >= 2*4*32 + 4*32 + 2*32 + IB*TP doubles.
// ---------------------------------------------------------------------------------------
// 1/a to full double precision: v_rcp_f64 + two Newton steps (a != 0, finite).
__device__ __forceinline__ double rcp_nr(double a) {
  double r = __builtin_amdgcn_rcp(a);
  r = fma(fma(-a, r, 1.0), r, r);
  r = fma(fma(-a, r, 1.0), r, r);
  return r;
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
  return dbl_of(lo, hi);
}

// One reflector step, as a loop body over a shifting window (the code stays a few KiB: a fully
// unrolled 32-step panel was 60 KiB of straight-line code per variant, streamed through the
// instruction cache on every call — 70 us per group in the persistent engine instead of ~35).
// Thread t holds row t of the live columns in x[0..NW): x[jr] = column C + jr; finished columns
// are written to the V image and shifted out, zeros shift in.
//   1. every tail row forms x_C * x_j (j in the window) and the wave reduce-scatters them;
//   2. one barrier; each lane sums the 4 wave partials of "its" column j and reads head_j;
//   3. the pivot's D_C and head_C are read from the owning lane (s_readlane, uniform);
//   4. lane of column j forms f_j = tau (head_j + scale D_j) and publishes it wave-privately;
//   5. rows update x_j -= f_j v (tails) / head_j -= f_j (GE head row, TS head in `hout`).
template <int B, bool TS, int NW, int IBX = Geo<B>::IB>
__device__ __forceinline__ void panel_step(double (&x)[IBX], double* Vs, double* Hs, double* tauv, double* red,
                                           double* wb, double* hrow, double* hout, int c0, int C, bool own, int rt PS_PARAMS) {
  using g = Geo<B, IBX>;
  constexpr int IB = g::IB, TP = g::TP, VP = g::VP;
  constexpr int SPAN = 64 / NW;  // lanes holding the same column after reduce-scatter
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int rc = c0 + C;  // GE: tile row of the reflector head
  const bool tail = own && (TS || rt > rc);  // rt: the tile row this thread holds
  PS_MARK(0);
  double pv[NW];
  const double xm = tail ? x[0] : 0.0;  // one select, not one per product (GE: 64 v_cndmask)
#pragma unroll
  for (int j = 0; j < NW; ++j) pv[j] = xm * x[j];
  const double ws = RS<NW>::run(pv, lane);
  const int cr = rs_col<NW>(lane);  // relative column of this lane's sum
  const int cw = C + cr;            // absolute column (>= IB: outside the panel, ignored)
  const bool wr = (lane & (SPAN - 1)) == 0;
  double* rb = red + (C & 1) * 128;
  if (wr && w < 4) rb[w * 32 + cr] = ws;  // rows live in waves 0-3
  PS_MARK(1);
  // (GE: the head row reached hrow at the end of the previous step, off this barrier's path)
  __syncthreads();
  const double Dm = (rb[cr] + rb[32 + cr]) + (rb[64 + cr] + rb[96 + cr]);
  const double Hm = TS ? (cw < IB ? Hs[C * TP + cw] : 0.0) : hrow[(C & 1) * 32 + cr];
  const double dc = readlane_d(Dm, 0);
  const double x0 = readlane_d(Hm, 0);
  PS_MARK(2);
  // norm, 1/norm from one reciprocal square root (two Newton steps), and tau = hd / (s norm) —
  // LAPACK's form of 2 / |v|^2 (|v|^2 = 1 + dc / hd^2 = 2 s norm / hd): two independent
  // reciprocals after the norm instead of a square root followed by two dependent reciprocals,
  // ~10 fewer dependent fp64 operations per reflector step. norm == 0 keeps scale 1, tau 2.
  const double n2 = fma(x0, x0, dc);
  const bool z = n2 == 0.0;
  const double h2 = 0.5 * n2;
  double rn = __builtin_amdgcn_rsq(n2);
  rn = rn * fma(-h2 * rn, rn, 1.5);
  rn = rn * fma(-h2 * rn, rn, 1.5);
  const double norm = z ? 0.0 : n2 * rn;
  const double sg = x0 >= 0.0 ? 1.0 : -1.0;
  const double hd = fma(sg, norm, x0);
  const double scale = z ? 1.0 : rcp_nr(hd);
  // (tau lies in [1, 2]; the product form can round an ulp outside)
  const double tau = z ? 2.0 : fmin(fmax(hd * (sg * rn), 1.0), 2.0);
  const double fm = cw < IB ? tau * fma(scale, Dm, Hm) : 0.0;  // f_j for j = cw
  PS_MARK(3);
  double* fb = wb + (w & 3) * 32;
  if (wr && w < 4) fb[cr] = fm;
  if (TS && w == 0 && wr && cw < IB) hout[C * TP + cw] = Hm - fm;  // cw == C: R_CC = x0 - f_C
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  double f[NW];
#pragma unroll
  for (int h = 0; h < NW / 2; ++h) {
    const double2 v2 = reinterpret_cast<const double2*>(fb)[h];
    f[2 * h] = v2.x;
    f[2 * h + 1] = v2.y;
  }
  PS_MARK(4);
  // branch-free update (a divergent tail/head-row branch made the wave holding the GE head row
  // run both streams): tails x_j -= f_j (scale x_C), the GE head row x_j -= f_j (coefficient 1,
  // the same rounding as a subtraction), all other rows coefficient 0 (x_j unchanged)
  const bool hr = !TS && rt == rc;
  const double xc = x[0] * scale;
  const double cf = tail ? xc : (hr ? 1.0 : 0.0);
#pragma unroll
  for (int j = 1; j < NW; ++j) x[j] = fma(-f[j], cf, x[j]);
  x[0] = tail ? xc : (hr ? x0 - f[0] : x[0]);
  if (t == 0) tauv[C] = tau;
  // column C is final (V entry / R entry): out to the image, shift the window
  if (own) Vs[t * VP + g::pc(C)] = x[0];
#pragma unroll
  for (int j = 0; j + 1 < NW; ++j) x[j] = x[j + 1];
  x[NW - 1] = 0.0;
  // GE: the next step's head row (updated just now as a tail) goes to the other hrow buffer
  // (every wave read this one's twin before passing this step's barrier)
  if (!TS && C + 1 < IBX && rt == rc + 1) {
    double2* hb = reinterpret_cast<double2*>(hrow + ((C + 1) & 1) * 32);
#pragma unroll
    for (int h = 0; h < NW / 2; ++h) hb[h] = make_double2(x[2 * h], x[2 * h + 1]);
  }
  PS_MARK(5);
}

// Work for the waves without panel rows (multi-GPU: forwarding the previous reflector group's
// images to the peers, flow.hpp panel_idle): step(C) before each reflector step's barrier, fin()
// after the last one. Defined in flow.hpp.
struct FwdJob;
__device__ void panel_idle(const FwdJob* fj, int IB, bool TS);

// PERM: LDS row q of Vs holds tile row vimg_row(q) (the chain engine's paired row order), else
// tile row q. idle: optional work of waves 4-7 (8-wave engine), see FwdJob.
template <int B, bool TS, bool PERM = false, int IBX = Geo<B>::IB>
__device__ __noinline__ void panel_factor(double* Vs, double* Hs, double* tauv, double* scratch, int c0,
                                          const FwdJob* idle = nullptr) {
  using g = Geo<B, IBX>;
  constexpr int IB = g::IB, VP = g::VP, TP = g::TP;
  double* red = scratch;             // 2 x [4 waves][32] cross-wave partials (double-buffered)
  double* wb = red + 2 * 4 * 32;     // [4 waves][32] per-wave totals
  double* hrow = wb + 4 * 32;        // 2 x [32] GE head row broadcast (double-buffered)
  double* hout = hrow + 2 * 32;      // [IB][TP] TS updated head rows
  const int t = threadIdx.x;
  if (t >= 256) {
    // waves beyond the 4 row waves (8-wave engine): no rows, but they would still run the whole
    // VALU reduction stream on zeros and compete with the row waves on their SIMDs — only
    // match the row waves' barriers (one per reflector step, then the exit ones), doing the
    // idle job between them if there is one
    if (idle) {
      panel_idle(idle, IB, TS);
      return;
    }
    for (int C = 0; C < IB; ++C) __syncthreads();
    __syncthreads();
    if (TS) __syncthreads();
    return;
  }
  const int rt = PERM ? vimg_row(t) : t;
  const bool own = t < B && (TS || rt >= c0);
  double x[IB];
#pragma unroll
  for (int j = 0; j < IB; ++j) x[j] = own ? Vs[t * VP + g::pc(j)] : 0.0;
  if (!TS && rt == c0) {  // head row of step 0 (later ones: end of the previous step)
#pragma unroll
    for (int j = 0; j < IB; ++j) hrow[j] = x[j];
  }
  // reduce the live window only: all IB columns while more than IB/2 are live, then the half,
  // then (IB = 32) the quarter for the last 8 reflectors
  constexpr int HALF = IB == 32 ? 16 : IB, Q3 = IB == 32 ? 24 : IB;
  PS_DECL
#pragma clang loop unroll(disable)
  for (int C = 0; C < HALF; ++C) panel_step<B, TS, IB, IBX>(x, Vs, Hs, tauv, red, wb, hrow, hout, c0, C, own, rt PS_ARGS);
  if constexpr (HALF < IB) {
#pragma clang loop unroll(disable)
    for (int C = HALF; C < Q3; ++C) panel_step<B, TS, IB / 2, IBX>(x, Vs, Hs, tauv, red, wb, hrow, hout, c0, C, own, rt PS_ARGS);
  }
  if constexpr (Q3 < IB) {
#pragma clang loop unroll(disable)
    for (int C = Q3; C < IB; ++C) panel_step<B, TS, IB / 4, IBX>(x, Vs, Hs, tauv, red, wb, hrow, hout, c0, C, own, rt PS_ARGS);
  }
  PS_FLUSH();
#ifdef TQR_DIAG_PFSLOW  // what-if: the factorisation N x ~3.4 us slower per group (marginal sensitivity)
  for (int i = 0; i < TQR_DIAG_PFSLOW; ++i) __builtin_amdgcn_s_sleep(127);
#endif
  __syncthreads();
  if (TS) {
    for (int idx = t; idx < IB * IB; idx += 256) {
      const int r = idx / IB, c = idx % IB;
      if (r <= c) Hs[r * TP + c] = hout[r * TP + c];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// T_g from the explicit V image and tauv.
//  1. Gram G = V^T V on MFMA, the B tile rows split over the 4 waves (64 rows each), partial
//     Grams summed in a fixed order (Gp: 4 x IB x TP scratch).
//  2. T = U^{-1} with U = diag(1/tau) + strict_upper(G) (the compact-WY identity
//     T^{-1} + T^{-T} = V^T V; this is LAPACK dlarft's forward columnwise T): 32 columns
//     solved in parallel by back substitution, 8 lanes per column, DPP-reduced dot products.
// Gs, Ts: IB x TP images. ks0: first non-zero 4-row block of V (GE), 0 for TS.
// ---------------------------------------------------------------------------------------
template <int B, int IBX = Geo<B>::IB>
__device__ __noinline__ void build_t(const double* Vs, const double* tauv, double* Gs, double* Ts, double* Gp, int ks0) {
  using g = Geo<B, IBX>;
  constexpr int IB = g::IB, VP = g::VP, TP = g::TP, NKS = g::NKS, NRI = g::NRI;
  constexpr int KPW = (NKS + 3) / 4;  // k-steps per wave
  constexpr int NCH = IB / 16;        // 16-column halves of the Gram
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, x = lane >> 4, y = lane & 3, blk = (lane >> 2) & 3;
  BT_STAMP(0);
  if (blockDim.x >= 512 && NCH == 2) {
    // 8 waves: wave w sums rows of k-step block (w & 3) into Gram column half (w >> 2)
    const int h = w >> 2;
    double Z[NRI];
#pragma unroll
    for (int r = 0; r < NRI; ++r) Z[r] = 0.0;
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      const int ks = (w & 3) * KPW + kk;
      if (ks >= NKS || ks < ks0) continue;
      const double2* vr = reinterpret_cast<const double2*>(Vs + (4 * ks + x) * VP + y * NRI);
      double a[NRI];
#pragma unroll
      for (int q = 0; q < NRI / 2; ++q) {
        double2 tt = vr[q];
        a[2 * q] = tt.x;
        a[2 * q + 1] = tt.y;
      }
      const double xb = Vs[(4 * ks + x) * VP + g::pc(16 * h + 4 * blk + y)];
#pragma unroll
      for (int r = 0; r < NRI; ++r) Z[r] = mfma4(a[r], xb, Z[r]);
    }
    double* gp = Gp + (w & 3) * IB * TP;
#pragma unroll
    for (int r = 0; r < NRI; ++r) gp[(4 * r + x) * TP + 16 * h + 4 * blk + y] = Z[r];
  } else {
    double Z[NCH][NRI];
#pragma unroll
    for (int h = 0; h < NCH; ++h)
#pragma unroll
      for (int r = 0; r < NRI; ++r) Z[h][r] = 0.0;
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      const int ks = w * KPW + kk;
      if (ks >= NKS || ks < ks0) continue;
      const double2* vr = reinterpret_cast<const double2*>(Vs + (4 * ks + x) * VP + y * NRI);
      double a[NRI];
#pragma unroll
      for (int q = 0; q < NRI / 2; ++q) {
        double2 tt = vr[q];
        a[2 * q] = tt.x;
        a[2 * q + 1] = tt.y;
      }
#pragma unroll
      for (int h = 0; h < NCH; ++h) {
        const double xb = Vs[(4 * ks + x) * VP + g::pc(16 * h + 4 * blk + y)];
#pragma unroll
        for (int r = 0; r < NRI; ++r) Z[h][r] = mfma4(a[r], xb, Z[h][r]);
      }
    }
    double* gp = Gp + (w & 3) * IB * TP;
    if (w < 4)
#pragma unroll
    for (int h = 0; h < NCH; ++h)
#pragma unroll
      for (int r = 0; r < NRI; ++r) gp[(4 * r + x) * TP + 16 * h + 4 * blk + y] = Z[h][r];
  }
  __syncthreads();
  BT_STAMP(1);
  for (int idx = t; idx < IB * IB; idx += blockDim.x) {
    const int r = idx / IB, c = idx % IB, o = r * TP + c;
    Gs[o] = (Gp[o] + Gp[IB * TP + o]) + (Gp[2 * IB * TP + o] + Gp[3 * IB * TP + o]);
  }
  __syncthreads();
  BT_STAMP(2);
  // back substitution: column j = t >> 3 (t < 8*IB), lane e = t & 7 holds x_k, k = e + 8q
  constexpr int NQ = IB / 8;
  const int j = t >> 3, e = t & 7;
  if (j < IB) {
    double xr[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) xr[q] = (e + 8 * q == j) ? tauv[j] : 0.0;
#pragma unroll
    for (int i = IB - 2; i >= 0; --i) {
      double part = 0.0;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        // the Gram entry is read unconditionally (always in range) and masked by a select: a
        // conditional read became a divergent branch with its own LDS wait per (i, q)
        const int k = e + 8 * q;
        double gv = Gs[i * TP + k];
        asm("" : "+v"(gv));  // keeps the read unconditional (else it is sunk into a branch)
        part += ((k > i && k <= j) ? gv : 0.0) * xr[q];
      }
      part += dpp<DPP_ROW_HALF_MIRROR>(part);
      part += dpp<DPP_QUAD_3210>(part);
      part += dpp<DPP_QUAD_1032>(part);
      double ti = tauv[i];
      asm("" : "+v"(ti));
      if (i < j && e == (i & 7)) xr[i >> 3] = -ti * part;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int k = e + 8 * q;
      Ts[k * TP + j] = k <= j ? xr[q] : 0.0;
    }
  }
  __syncthreads();
  BT_STAMP(3);
}

}  // namespace tqr
