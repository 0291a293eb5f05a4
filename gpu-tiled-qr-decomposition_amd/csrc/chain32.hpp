// fp32 chain of the persistent engine: fp32 storage, fp32 arithmetic on v_mfma_f32_16x16x4_f32
// (BASELINE configs[4], 32768^2 fp32). Included by flow.hpp (uses its sync / DMA / counter helpers).
//
// The same chain task as flow_chain (UNMQR(k,j) then TSMQR(i,j,k) for the rows of a segment, on a
// 128-column strip, 8 waves x 16 columns), with the fp32 MFMA at 64 flop/clk/SIMD — twice the fp64
// 4x4x4 form's rate (profiles/r02/ubench_mfma.txt: 152-155 vs 67-69 TF/s).
//
// Register layout (per wave, 16 columns, lane = 16x + y, x = lane >> 4, y = lane & 15): the f32
// 16x16x4 MFMA takes A[i][k] from lane 16k + i, B[k][j] from lane 16k + j and holds D[4x + r][y]
// in register r of lane 16x + y (probed: tools/ubench/mfma_probe32.hip, profiles/r02/
// ubench_mfma_probe32.txt — NOT the f64 16x16x4 form's D[4r + x][y]). A strip tile mt (16 rows)
// therefore sits with row 16mt + 4x + r in register r of lane x — four consecutive rows per lane,
// so the strip moves as 16-B accesses — and the same register is the B operand of k-step (mt, r)
// of Z = V^T X (k = x <-> row 16mt + 4x + r). Z, W and the head rows share the layout: reflector
// (row) 16mi + 4x + r in register r.
//   * X: the strip of tile (i,j), NMT float4 registers (64 VGPRs at b = 256);
//   * Hd: the strip of the chain's head tile (k,j) stays in registers for the whole segment (64
//     VGPRs): no head-row traffic inside a segment; the first element of a later segment loads it
//     group by group behind the previous segment (Ac), the last one stores it group by group;
//     Hd is rotated by NMI tiles per group, so the current group's rows are always Hd[0..NMI);
//   * per group: Z = Hd[0..NMI) + V^T X (NMT x 4 x NMI MFMAs), W = -T^T Z (4 NPR), Hd += W,
//     X += V W (NMT x 4 x NMI); the UNMQR element runs Z = V^T Hd, Hd += V W (explicit GE V).
// The images (VR, TP; tiles.hpp Geo32) are written by the panel task from its fp64 LDS block
// (the panel itself factorises in fp64 and stores fp32 V, R, tau) and LDS-DMA'd like the fp64 ones.
#pragma once

namespace tqr {

typedef float f4v __attribute__((ext_vector_type(4)));

// the MFMA row index i of A / D <-> the tile-local row or reflector: identity for this form
__device__ __forceinline__ int sig16(int y) { return y; }
__device__ __forceinline__ f4v mfma16(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void st_f4(__amdgpu_buffer_rsrc_t rs, unsigned off, f4v v, int aux_sc1 = 1) {
  __attribute__((ext_vector_type(4))) unsigned u = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                                     __float_as_uint(v[3])};
  if (aux_sc1) __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 16);
  else __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 0);
}
__device__ __forceinline__ f4v ld_f4(__amdgpu_buffer_rsrc_t rs, unsigned off) {
  const auto u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
  return f4v{__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3])};
}

// Panel side: the fp32 chain's images of one reflector group from the panel's fp64 LDS block (rows
// in the paired order of flow_panel: tile row R at LDS row vimg_inv(R), columns permuted by pc) and
// its T (row-major, pitch TP). All panel threads; 16-B write-through stores.
// lvr / ltp (LDS, optional): the same chunks, for the panel's own trailing update (flow_panel)
typedef __attribute__((address_space(3))) f4v lds_f4_t;
template <int B>
__device__ __noinline__ void write_images32(const double* Vs, const double* Ts, __amdgpu_buffer_rsrc_t rv,
                                            __amdgpu_buffer_rsrc_t rt, float* lvr, float* ltp) {
  lds_f4_t* const lv = lvr ? (lds_f4_t*)(const __attribute__((address_space(3))) void*)lvr : nullptr;
  lds_f4_t* const lt = ltp ? (lds_f4_t*)(const __attribute__((address_space(3))) void*)ltp : nullptr;
  using G = Geo<B>;
  using G32 = Geo32<B>;
  constexpr int NMI = G32::NMI, VP = G::VP, TP = G::TP;
  auto V = [&](int R, int c) { return (float)Vs[vimg_inv(R) * VP + G::pc(c)]; };
  for (int idx = threadIdx.x; idx < G32::VR / 4; idx += blockDim.x) {  // VR 16-B chunks
    const int R = idx / (G32::IB / 4), slot = (idx % (G32::IB / 4)) ^ G32::vr_sw(R);
    f4v v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int p = 4 * slot + e, x = p / (4 * NMI), wi = (p >> 2) % NMI, r = p & 3;
      v[e] = V(R, 16 * wi + 4 * x + r);
    }
    st_f4(rv, 16u * idx, v);
    if (lv) lv[idx] = v;
  }
  for (int idx = threadIdx.x; idx < G32::TIMG * 2 / 4; idx += blockDim.x) {  // TP chunks (+ zero pad)
    const int lane = idx & 63, pr = idx >> 6, x = lane >> 4, y = lane & 15;
    int mi = 0, wi = 0;
    for (int c = 0, q = 0; q < NMI * NMI; ++q) {  // pair pr -> (mi <= wi), wi-major
      const int w_ = q / NMI, m_ = q % NMI;
      if (m_ > w_) continue;
      if (c++ == pr) { mi = m_; wi = w_; }
    }
    f4v v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = pr < G32::NPR ? (float)(-Ts[(16 * mi + 4 * x + r) * TP + 16 * wi + sig16(y)]) : 0.0f;
    st_f4(rt, 16u * idx, v);
    if (lt) lt[idx] = v;
  }
}

// V image reads (Geo32 VR): opaque 32-bit LDS byte address (per-lane bases, immediate offsets)
typedef __attribute__((address_space(3))) const float lds_cf_t;
typedef __attribute__((address_space(3))) const f4v lds_cf4_t;
__device__ __forceinline__ unsigned lds_addr_f(const float* p) {
  unsigned a = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
  asm volatile("" : "+v"(a));
  return a;
}
__device__ __forceinline__ float lds_rdf(unsigned a) { return *(lds_cf_t*)(size_t)a; }
__device__ __forceinline__ f4v lds_rdf4(unsigned a) { return *(lds_cf4_t*)(size_t)a; }

// LDS operand reads: NMI float4 chunks of tile mt for this lane
template <int N>
__device__ __forceinline__ void ld_chunks(float (&a)[4 * N], const float* img, int mt, int lane) {
  const f4v* p = reinterpret_cast<const f4v*>(img) + (mt * N) * 64 + lane;
#pragma unroll
  for (int c = 0; c < N; ++c) {
    const f4v v = p[c * 64];
#pragma unroll
    for (int e = 0; e < 4; ++e) a[4 * c + e] = v[e];
  }
}

// Phase-2 hook: nothing after the strip tiles are final (every group but an element's last)
struct NoPost32 {
  template <int N>
  __device__ __forceinline__ void at(int, f4v (&)[N]) const {}
  template <int N>
  __device__ __forceinline__ void fin(f4v (&)[N]) const {}
};
// Element hand-over inside the last group's phase 2: once tile pair p of the strip is final (its
// MFMAs issued one pair earlier), it is stored (write-through) and the same registers start
// loading pair p of the next element's strip — the element boundary no longer waits for 128 KiB
// of strip out and in per workgroup (what-if without strip I/O: -71 ms at 32768^2 fp32).
// The loads trail the stores by one tile pair: reloading a tile's registers right behind its own
// store makes the load wait for that store to have read its data (see XPipe in flow.hpp).
template <int B>
struct XPipe32 {
  static constexpr int NMT = Geo32<B>::NMT;
  __amdgpu_buffer_rsrc_t out, in;  // this element's strip / the next element's (same columns)
  unsigned base;
  __device__ __forceinline__ void st(int mt, f4v (&X)[NMT]) const { st_f4(out, base + 64u * mt, X[mt]); }
  __device__ __forceinline__ void ld(int mt, f4v (&X)[NMT]) const { X[mt] = ld_f4(in, base + 64u * mt); }
  __device__ __forceinline__ void at(int mt, f4v (&X)[NMT]) const {
    if (mt >= 2) {
      st(mt - 2, X);
      st(mt - 1, X);
    }
    if (mt >= 4) {
      ld(mt - 4, X);
      ld(mt - 3, X);
    }
  }
  __device__ __forceinline__ void fin(f4v (&X)[NMT]) const {
    if constexpr (NMT >= 2) st(NMT - 2, X);
    st(NMT - 1, X);
#pragma unroll
    for (int mt = NMT - 4; mt < NMT; ++mt)
      if (mt >= 0) ld(mt, X);
  }
};

// One reflector group applied to a strip (X) with head accumulator Hg (TS) or none (GE, UNMQR:
// the strip is the head tile itself). Phase 1 carries the hook (next group's LDS-DMA), phase 2
// the post hook (element hand-over). K0 (GE group g: g NMI): V is zero in tiles mt < K0 (the GE
// group's unit-lower V, explicit zeros above its rows), so both phases start at tile K0.
template <int B, bool TS, typename Hook, typename Post = NoPost32, int K0 = 0>
__device__ __forceinline__ void apply32(const float* VR, const float* TPi, f4v (&X)[Geo32<B>::NMT],
                                        f4v (&Hg)[Geo32<B>::NMT], const Hook& hook, const Post& post = Post()) {
  using G32 = Geo32<B>;
  constexpr int NMT = G32::NMT, NMI = G32::NMI;
  constexpr int IB = G32::IB;
  constexpr bool SW = IB == 32;
  const int lane = threadIdx.x & 63, x = lane >> 4, y = lane & 15, q = y >> 2, e = y & 3;
  // per-lane byte bases of the two phases' reads (Geo32::vr_at, unrolled by hand): phase 1 reads
  // V(16mt + 4x + r, 16mi + y) — slot NMI q + mi of row R, swizzled by vr_sw(R), whose bits
  // from r only flip mi (r >= 2); phase 2 reads the 16-B slot NMI x + wi of row 16mt + y
  const int sx = SW ? ((x & 1) | (((x >> 1) & 1) << 2)) : 0;
  const int sy = SW ? ((((y >> 1) ^ (y >> 2)) & 1) | (((y >> 3) & 1) << 2)) : 0;
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
      for (int mi = 0; mi < NMI; ++mi)
        a[r * NMI + mi] = lds_rdf(b1[SW ? (mi ^ ((r >> 1) & 1)) : mi] + 4u * ((16 * mt + r) * IB));
  };
  auto ld2 = [&](float (&a)[4 * NMI], int mt) {
#pragma unroll
    for (int wi = 0; wi < NMI; ++wi) {
      const f4v t = lds_rdf4(b2[wi] + 4u * (16 * mt * IB));
#pragma unroll
      for (int r = 0; r < 4; ++r) a[4 * wi + r] = t[r];
    }
  };
  f4v Z[NMI];
#pragma unroll
  for (int mi = 0; mi < NMI; ++mi) Z[mi] = TS ? Hg[mi] : f4v{0.f, 0.f, 0.f, 0.f};
  // phase 1: Z += V^T X, operands of tile mt+1 read under the MFMAs of tile mt
  static_assert(K0 % 2 == 0 && K0 < NMT && (TS ? K0 == 0 : true), "K0: even, GE only");
  float ac[4 * NMI], an[4 * NMI];
  ld1(ac, K0);
#pragma unroll
  for (int mt = K0; mt < NMT; ++mt) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    hook.step(mt - K0);
    if (mt + 1 < NMT) ld1(an, mt + 1);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int mi = 0; mi < NMI; ++mi) Z[mi] = mfma16(ac[r * NMI + mi], X[mt][r], Z[mi]);
#pragma unroll
    for (int e = 0; e < 4 * NMI; ++e) ac[e] = an[e];
  }
  for (int m = NMT - K0; m < Hook::STEPS; ++m) hook.step(m);
  hook.mid();
  // W = -T^T Z (upper-triangular T: tile pairs mi <= wi, wi-major in the image)
  f4v W[NMI];
  {
    float tp[4 * G32::NPR];
    ld_chunks<G32::NPR>(tp, TPi, 0, lane);
#pragma unroll
    for (int wi = 0, pr = 0; wi < NMI; ++wi) {
      W[wi] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int mi = 0; mi <= wi; ++mi, ++pr)
#pragma unroll
        for (int r = 0; r < 4; ++r) W[wi] = mfma16(tp[4 * pr + r], Z[mi][r], W[wi]);
    }
  }
  if (TS) {
#pragma unroll
    for (int wi = 0; wi < NMI; ++wi) Hg[wi] += W[wi];
  }
  // phase 2: X += V W, two tiles interleaved (dependent-accumulator latency 40 > issue 32 cycles)
  float c0[4 * NMI], c1[4 * NMI];
#pragma unroll
  for (int mt = K0; mt < NMT; mt += 2) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    ld2(c0, mt);
    if (mt + 1 < NMT) ld2(c1, mt + 1);
#pragma unroll
    for (int wi = 0; wi < NMI; ++wi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        X[mt] = mfma16(c0[4 * wi + r], W[wi][r], X[mt]);
        if (mt + 1 < NMT) X[mt + 1] = mfma16(c1[4 * wi + r], W[wi][r], X[mt + 1]);
      }
    post.at(mt, X);  // the previous pair, behind this pair's MFMAs
  }
  post.fin(X);
}

// The UNMQR element's group g: tiles below g NMI skipped (g wave-uniform; one body per group)
template <int B, typename Hook>
__device__ __forceinline__ void apply32_ge(int g, const float* VR, const float* TPi, f4v (&Hd)[Geo32<B>::NMT], const Hook& h) {
  static_assert(Geo<B>::NG <= 8, "apply32_ge: up to 8 groups");
#ifdef TQR_NO_GE_SKIP32  // (A/B builds: the full GE V, zero tiles included)
  g = 0;
#endif
  switch (g) {
    case 0: apply32<B, false, Hook, NoPost32, 0>(VR, TPi, Hd, Hd, h); break;
    case 1: if constexpr (Geo<B>::NG > 1) apply32<B, false, Hook, NoPost32, 1 * Geo32<B>::NMI>(VR, TPi, Hd, Hd, h); break;
    case 2: if constexpr (Geo<B>::NG > 2) apply32<B, false, Hook, NoPost32, 2 * Geo32<B>::NMI>(VR, TPi, Hd, Hd, h); break;
    case 3: if constexpr (Geo<B>::NG > 3) apply32<B, false, Hook, NoPost32, 3 * Geo32<B>::NMI>(VR, TPi, Hd, Hd, h); break;
    case 4: if constexpr (Geo<B>::NG > 4) apply32<B, false, Hook, NoPost32, 4 * Geo32<B>::NMI>(VR, TPi, Hd, Hd, h); break;
    case 5: if constexpr (Geo<B>::NG > 5) apply32<B, false, Hook, NoPost32, 5 * Geo32<B>::NMI>(VR, TPi, Hd, Hd, h); break;
    case 6: if constexpr (Geo<B>::NG > 6) apply32<B, false, Hook, NoPost32, 6 * Geo32<B>::NMI>(VR, TPi, Hd, Hd, h); break;
    default: if constexpr (Geo<B>::NG > 7) apply32<B, false, Hook, NoPost32, 7 * Geo32<B>::NMI>(VR, TPi, Hd, Hd, h); break;
  }
}

// Strip / head tile I/O: tile mt of the strip at column col0 + y, rows 16mt + 4x .. + 3.
template <int B>
struct Strip32 {
  __amdgpu_buffer_rsrc_t rs;
  unsigned base;
  __device__ __forceinline__ Strip32(float* tile, size_t ldm, int col0) {
    const int lane = threadIdx.x & 63;
    rs = uniform_rsrc(tile + (size_t)col0 * ldm);
    base = (unsigned)(((size_t)(lane & 15) * ldm + 4 * (lane >> 4)) * sizeof(float));
  }
  __device__ __forceinline__ unsigned off(int mt) const { return base + 64u * mt; }
};

// fp32 storage: the panel group's in-tile trailing update in fp32 on v_mfma_f32_16x16x4_f32 (the
// chains' arithmetic and the reference's own precision, qrdecomp.c:559-763 in float), twice the
// fp64 4x4x4 form's rate, from the group's fp32 images that write_images32 also left in LDS (VRl,
// then the packed -T). Until round 5 the panel applied its fp64 V / T on the fp64 MFMA (what-if
// without the trailing update: -17.6 ms at 32768^2, profiles/r06/whatif_f32.txt). Wave w takes the
// 16-column strips w, w + nw, ... right of the group. GEQRT (qrs): the tiles above the group are
// neither loaded nor stored (finished R rows, which the next member's trailing may be updating) and
// the GE V's zero tiles are skipped (apply32_ge); TSQRT: R_kk's rows of the group are the head.
template <int B>
__device__ __noinline__ void panel_trail32(float* Bt, float* Rt, size_t ldm, bool qrs, int g, int c0, int nstr,
                                           const float* VRl, int nw) {
  using G32 = Geo32<B>;
  constexpr int NMT = G32::NMT, NMI = G32::NMI;
  const float* TPl = VRl + G32::VR;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mt0 = qrs ? c0 / 16 : 0;
  for (int s = w; s < nstr; s += nw) {
    const int col = c0 + G32::IB + 16 * s;
    const Strip32<B> xs(Bt, ldm, col);
    f4v X[NMT], Hg[NMT];
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt) X[mt] = mt >= mt0 ? ld_f4(xs.rs, xs.off(mt)) : f4v{0.f, 0.f, 0.f, 0.f};
    if (qrs) {
      apply32_ge<B>(g, VRl, TPl, X, NoHook());
    } else {
      const Strip32<B> hs(Rt, ldm, col);
#pragma unroll
      for (int mi = 0; mi < NMI; ++mi) Hg[mi] = ld_f4(hs.rs, hs.off(c0 / 16 + mi));
      apply32<B, true, NoHook>(VRl, TPl, X, Hg, NoHook());
#pragma unroll
      for (int mi = 0; mi < NMI; ++mi) st_f4(hs.rs, hs.off(c0 / 16 + mi), Hg[mi]);
    }
#pragma unroll
    for (int mt = 0; mt < NMT; ++mt)
      if (mt >= mt0) st_f4(xs.rs, xs.off(mt), X[mt]);
  }
}

template <int B>
__device__ __noinline__ void flow_chain32(const FlowArgs& a, int s_, int i0_, int i1_, int j_, int k_, int seg_,
                                          double* lds, int* sflag) {
  const int s = uni(s_), i0 = uni(i0_), i1 = uni(i1_), j = uni(j_), k = uni(k_), seg = uni(seg_);
  using G = Geo<B>;
  using G32 = Geo32<B>;
  constexpr int NG = G::NG, NMT = G32::NMT, NMI = G32::NMI, BUF = Img<B, float>::V + Img<B, float>::T;
  float* A = uni((float*)a.A);
  const size_t ldm = uni64(a.ldm);
  const int t = threadIdx.x, w = t >> 6;
  const int col = s * FLOW_SW + 16 * w;
  const bool active = B % FLOW_SW == 0 || col < B;
  float* const Aj = uni(A + (size_t)(j / uni(a.cdiv)) * B * ldm);  // tile column j (FlowArgs::cdiv)
  float* At = Aj + (size_t)k * B;
  double* const wk = uni(a.Wk[k]);
  const int P = uni(a.p), Q = uni(a.q), NS = uni(a.ns);
  int* const err = uni(a.err);
  int* const Tc = uni(a.Tc);
  auto vimg = [&](int i_, int g_) { return wk + flow_vw_off<B, float, ShapeW8>(P, i_, k, g_); };
  auto timg = [&](int i_, int g_) { return wk + flow_tw_off<B, float, ShapeW8>(P, i_, k, g_); };
  int* const rc = uni(&a.Rc[(size_t)k * NG]);
  int* const acg = uni(&a.Ac[(((size_t)k * Q + j) * NS + s) * NG]);
  auto tc = [&](int i) { return &Tc[((size_t)i * Q + j) * NS + s]; };
  f4v X[NMT], Hd[NMT];
  int buf = 0, par = 0;
  int* pending = nullptr;
  bool dma_next = false;
  // thread 0's early loads as LDS-DMAs into LDS slots (flow.hpp lds_prefetch; every sync point
  // here drains fully, so each has landed by the next one): the Rc counter (sflag[57]), the Tc of
  // the next element's tile (sflag[58], -1: none), a remote panel's member flag (sflag[59])
  PanelView<NG> pv;
  pv.init(sflag + 48, sflag + 57);
  int* const tcs = sflag + 58;
  int* const fls = sflag + 59;
  if (t == FLOW_PT) {
    *lds_int(tcs) = -1;
    *lds_int(fls) = -1;
  }
  bool xin = false;  // this element's strip was loaded during the previous element's last phase 2
  const bool remote = a.dist && tile_owner(k, a.world, a.cyclic) != a.rank;
  int* const rf = uni(a.Rf + (size_t)k * P * NG);
  const int ep = uni(a.epoch);
  int fl_pf = -1;  // index (i * NG + g) of the flag the early load in fls is of
  auto ready = [&](int i_, int g_) -> bool {
    if (!remote) return pv.ensure(rc, g_, i_ - k + 1, err, false);
    const int fi = i_ * NG + g_;
    if (fi == fl_pf && lds_ld_volatile(fls) >= ep) return true;
    return spin_ge_i(rf + fi, ep, err, true);
  };
  const Strip32<B> hs(At, ldm, col);  // the head tile's strip
  FST(6);
  if (k == 0 && a.Uc) {  // host-pointer API: tile column j uploaded (xfer.hpp)
    const bool ok = t == FLOW_PT ? spin_ge(&a.Uc[j], a.nxc, err) : true;
    if (!wg_verdict(ok, sflag)) return;
  }
  const int ifirst = seg == 0 ? k : i0;
  for (int i = ifirst; i < i1 || i == k; i = (i == k ? i0 : i + 1)) {
    const bool ts = i != k;
    const bool head_in = ts && i == ifirst;  // first element of a later segment: head arrives per group
    {
      bool ok = true;
      if (t == FLOW_PT) {
        if (head_in) ok = spin_ge(&acg[0], seg, err);
        FST(9);
        if (ok && k > 0 && lds_ld_volatile(tcs) < k) ok = spin_ge(tc(i), k, err);
        *lds_int(tcs) = -1;
        FST(8);
        if (ok && !dma_next) ok = ready(i, 0);
      }
      FST(j == k + 1 ? 18 : 19);
      if (!sync_point<false, true>(ok, sflag, par)) return;
    }
    FST(7);
    float* Xt = ts ? Aj + (size_t)i * B : At;
    if (!dma_next) {
      DmaJob<B, float, ShapeW8> d{lds + buf * BUF, vimg(i, 0), timg(i, 0), sflag};
      for (int m = 0; m < DmaJob<B, float, ShapeW8>::STEPS; ++m) d.step(m);
    }
    dma_next = false;
    const Strip32<B> xs(Xt, ldm, col);
    if (active) {
      if (ts) {
#ifndef TQR_DIAG_NOSTRIP
        if (!xin)
#pragma unroll
          for (int mt = 0; mt < NMT; ++mt) X[mt] = ld_f4(xs.rs, xs.off(mt));
#endif
        if (head_in)
#pragma unroll
          for (int mi = 0; mi < NMI; ++mi) Hd[mi] = ld_f4(hs.rs, hs.off(mi));
      } else {  // UNMQR: the head tile's strip is the operand, and stays as the segment's head
#pragma unroll
        for (int mt = 0; mt < NMT; ++mt) Hd[mt] = ld_f4(hs.rs, hs.off(mt));
      }
    }
    FST(4);
    const int inext = (i == k) ? i0 : i + 1;
    const bool has_next = inext < i1;
    auto groups = [&]() -> bool {
#ifdef TQR_FLOW_STAMPS
      // (group trace, tools/group_trace.py) this wave's running group count in the LDS tail
      __attribute__((address_space(3))) int* gtr_c = (__attribute__((address_space(3))) int*)(sflag + 113) + (threadIdx.x >> 6);
      int gtr_n = *gtr_c;
#endif
      for (int g = 0; g < NG; ++g) {
#ifdef TQR_FLOW_STAMPS
        if ((threadIdx.x & 63) == 0) *gtr_c = gtr_n + 1;
        GTR(0, __builtin_amdgcn_s_memrealtime());
        GTR(7, (unsigned long long)(g | (i << 8) | ((unsigned long long)j << 24) | ((unsigned long long)k << 40)));
#endif
        {
          bool ok = true;
          if (t == FLOW_PT && g + 1 == NG) {
            // last group: may the next element's strip stream in during this phase 2? (its tile
            // must have received step k-1: Tc, loaded two groups ahead)
#ifdef TQR_DIAG_NOSTRIP
            sflag[44] = 0;
#else
            sflag[44] = (NG > 1 && ts && has_next && (k == 0 || lds_ld_volatile(tcs) >= k)) ? 1 : 0;
#endif
          }
          if (t == FLOW_PT) {
            if (head_in && g + 1 < NG) ok = spin_ge_i(&acg[g + 1], seg, err);  // head rows of g+1 final
            if (ok) {
              if (g + 1 < NG) ok = ready(i, g + 1);
              else if (has_next) ok = ready(inext, 0);
            }
          }
          FST(j == k + 1 ? 20 : 0);
#ifdef TQR_FLOW_STAMPS
          GTR(1, __builtin_amdgcn_s_memrealtime());
#endif
          if (!sync_point<true, true>(ok, sflag, par)) return false;
#ifdef TQR_FLOW_STAMPS
          GTR(2, __builtin_amdgcn_s_memrealtime());
#endif
        }
        if (g == 0 && pending) {
          publish_after_drain(pending, 1);
          pending = nullptr;
        }
        if (!has_next && ts && g > 0) publish_after_drain(&acg[g - 1], 1);  // (a lone UNMQR: at the end)
        if (t == FLOW_PT) {  // early load of the counter the next sync point will test
          const int tg = next_test_group<NG>(g);
          const bool here = g + 2 < NG;
          if (here || has_next) {
            if (!remote) {
              pv.prefetch(rc, tg, false);
            } else {
              fl_pf = (here ? i : inext) * NG + tg;
              lds_prefetch<FLOW_PT>(rf + fl_pf, fls, true);
            }
          }
          if (g + 2 == NG && has_next && k > 0) lds_prefetch<FLOW_PT>(tc(inext), tcs, false);
        }
        FST(7);
        const float* img = reinterpret_cast<const float*>(lds + buf * BUF);
        const float* VRp = img;
        const float* TPi = img + 2 * Img<B, float>::V;
        const int gd = g + 1 < NG ? g + 1 : has_next ? 0 : g, id = g + 1 < NG ? i : has_next ? inext : i;
        DmaJob<B, float, ShapeW8> d{lds + (buf ^ 1) * BUF, vimg(id, gd), timg(id, gd), sflag};
        dma_next = g + 1 == NG && has_next;
#if defined(TQR_DIAG_DMA_FIXED)  // what-if: every DMA reads one L2-hot image (results wrong)
        d.v = vimg(k, 0);
        d.t = timg(k, 0);
#endif
#ifdef TQR_DIAG_NODMA  // what-if: no staging at all (results wrong)
        const NoHook dh{};
#else
        const DmaJob<B, float, ShapeW8>& dh = d;
#endif
        // (written before the sync; wave-uniform: a scalar branch around the hooked phase 2 — as a
        // per-lane value the two apply32 bodies became exec-masked twins, and at NG == 1 that
        // broke the non-hooked one)
        const bool pipe = NG > 1 && g + 1 == NG && uni(lds_ld_volatile(sflag + 44)) != 0;
#ifdef TQR_FLOW_STAMPS
        GTR(3, __builtin_amdgcn_s_memrealtime());
#endif
        if (active) {
          if (ts) {
            // next group's head rows (first element of a later segment) ride this group
            if (head_in && g + 1 < NG)
#pragma unroll
              for (int mi = 0; mi < NMI; ++mi) Hd[NMI + mi] = ld_f4(hs.rs, hs.off((g + 1) * NMI + mi));
            if (pipe) {
              float* Xn = Aj + (size_t)inext * B;
              const XPipe32<B> xp{xs.rs, uniform_rsrc(Xn + (size_t)col * ldm), xs.base};
              apply32<B, true>(VRp, TPi, X, Hd, dh, xp);
            } else {
              apply32<B, true>(VRp, TPi, X, Hd, dh);
            }
            FST(13);
#ifdef TQR_FLOW_STAMPS
            GTR(4, __builtin_amdgcn_s_memrealtime());
            GTR(5, __builtin_amdgcn_s_memrealtime());
#endif
            if (!has_next)  // segment's last element: the group's head rows leave (write-through)
#pragma unroll
              for (int mi = 0; mi < NMI; ++mi) st_f4(hs.rs, hs.off(g * NMI + mi), Hd[mi]);
            // rotate the head: the next group's rows to Hd[0..NMI)
            f4v tmp[NMI];
#pragma unroll
            for (int mi = 0; mi < NMI; ++mi) tmp[mi] = Hd[mi];
#pragma unroll
            for (int mt = 0; mt + NMI < NMT; ++mt) Hd[mt] = Hd[mt + NMI];
#pragma unroll
            for (int mi = 0; mi < NMI; ++mi) Hd[NMT - NMI + mi] = tmp[mi];
            FST(2);
          } else {
            apply32_ge<B>(g, VRp, TPi, Hd, dh);
            FST(13);
          }
        } else {
          for (int m = 0; m < DmaJob<B, float, ShapeW8>::STEPS; ++m) d.step(m);
        }
        if (g + 1 == NG) xin = pipe;
        buf ^= 1;
#ifdef TQR_FLOW_STAMPS
        GTR(6, __builtin_amdgcn_s_memrealtime());
        ++gtr_n;
#endif
      }
      return true;
    };
    if (!groups()) return;
    if (active) {
      if (ts) {
#ifndef TQR_DIAG_NOSTRIP
        if (!xin)
#pragma unroll
          for (int mt = 0; mt < NMT; ++mt) st_f4(xs.rs, xs.off(mt), X[mt]);
#endif
      } else if (!has_next) {  // a lone UNMQR (last step): its head tile strip is the result
#pragma unroll
        for (int mt = 0; mt < NMT; ++mt) st_f4(hs.rs, hs.off(mt), Hd[mt]);
      }
    }
    pending = tc(i);
    FST(4);
  }
  sync_point<true, true>(true, sflag, par);
  if (pending) publish_after_drain(pending, 1);
  if (seg == 0 && i0 >= i1)  // a segment of the UNMQR element alone: its head strip stored whole above
    for (int g = 0; g + 1 < NG; ++g) publish_after_drain(&acg[g], 1);
  publish_after_drain(&acg[NG - 1], 1);
  FST(4);
}

}  // namespace tqr
