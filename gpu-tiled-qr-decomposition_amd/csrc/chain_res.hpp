// fp64 chain task, "resident" form: one wave per SIMD (4 waves, 64-column strips, 256-row tiles),
// each wave owning the whole 512-register file — the engine's CHAIN(k, j, s, e) task of flow.hpp
// (UNMQR(k,j) then TSMQR(i,j,k) over the segment's rows, the reference's SLARFT / SSSRFT,
// /root/reference/qrdecomp.c:559-645,723-763, src/gpucalc.cu:1174-1359) on the generated group
// bodies of gen/gen_chain_asm.py (TQR_CHAIN_RES_*).
//
// What the register file buys:
//   * the element strip is double-buffered in AGPRs (a[0:127] / a[128:255]): while element e runs on
//     one bank, the other bank's strip (element e-1's result) is stored after groups 0 and 1, and
//     element e+1's strip loaded into it after groups 2..7 — spread over the element instead of
//     inside one group's phase 2, where the 8-wave form's hand-over doubled that group's time;
//   * the head strip (tile (k,j)'s 256 rows of this wave's 16 columns) stays in v[128:255] for the
//     whole segment (group g's rows VGPR-indexed by 16 g), so there is no head-row traffic inside a
//     segment at all: it is loaded group by group at the start of a later segment (or is the UNMQR
//     element's result) and stored group by group during the segment's last element.
// The I/O between two bodies is its own small asm statement (per group and bank); the sync point of
// the next group leaves exactly those operations in flight (vmcnt(n), n = their count), and a
// group's sync two groups later finds them complete (they are older than the LDS-DMA it waits for),
// which is when their counters are published (no drain).
// Registers: as chain_asm.hpp, with v[32:255] and a[0:255] owned by the statements (the build
// audit, tools/check_chain_asm.py, covers flow_chain_res too).
#pragma once

namespace tqr {

using ShapeR = FlowShape<4, 32, 1>;  // one 4-wave workgroup per CU, 64-column strips, 32-reflector groups

template <int N>
__device__ __forceinline__ bool res_sync_n(bool ok0, bool poller, int* sflag, int& par) {
  return ca_sync<N>(ok0, poller, sflag, par);
}
// the sync point with the previous I/O statement's n operations left in flight (n from the small set
// the I/O schedule produces; any other count waits for everything)
__device__ __forceinline__ bool res_sync(int n, bool ok0, bool poller, int* sflag, int& par) {
  switch (n) {
    case 0: return res_sync_n<0>(ok0, poller, sflag, par);
    case 4: return res_sync_n<4>(ok0, poller, sflag, par);
    case 5: return res_sync_n<5>(ok0, poller, sflag, par);
    case 6: return res_sync_n<6>(ok0, poller, sflag, par);
    case 8: return res_sync_n<8>(ok0, poller, sflag, par);
    case 9: return res_sync_n<9>(ok0, poller, sflag, par);
    case 10: return res_sync_n<10>(ok0, poller, sflag, par);
    case 16: return res_sync_n<16>(ok0, poller, sflag, par);
    case 20: return res_sync_n<20>(ok0, poller, sflag, par);
    default: return res_sync_n<0>(ok0, poller, sflag, par);
  }
}

struct ResGroup {
  unsigned vz, vx, vt, vl16;
  const double* svsrc;
  const double* stsrc;
  unsigned sdst;
  int sw, gidx;
};

template <int BANK, bool SW>
__device__ __forceinline__ void res_body(const ResGroup& o) {
  unsigned m0s, st;
#define TQR_RES_INS                                                                                          \
  [vz] "v"(o.vz), [vx] "v"(o.vx), [vt] "v"(o.vt), [vl16] "v"(o.vl16), [svsrc] "s"(o.svsrc), [stsrc] "s"(o.stsrc), \
      [sdst] "s"(o.sdst), [sw] "s"(o.sw), [gidx] "s"(o.gidx)
  if constexpr (BANK == 0 && !SW)
    asm volatile(TQR_CHAIN_RES_B256_X0 : [m0s] "=&s"(m0s), [st] "=&s"(st) : TQR_RES_INS
                 : "memory", "scc", TQR_CHAIN_RES_CLOBBERS);
  else if constexpr (BANK == 0)
    asm volatile(TQR_CHAIN_RES_B256_X0_SW : [m0s] "=&s"(m0s), [st] "=&s"(st) : TQR_RES_INS
                 : "memory", "scc", TQR_CHAIN_RES_CLOBBERS);
  else if constexpr (!SW)
    asm volatile(TQR_CHAIN_RES_B256_X1 : [m0s] "=&s"(m0s), [st] "=&s"(st) : TQR_RES_INS
                 : "memory", "scc", TQR_CHAIN_RES_CLOBBERS);
  else
    asm volatile(TQR_CHAIN_RES_B256_X1_SW : [m0s] "=&s"(m0s), [st] "=&s"(st) : TQR_RES_INS
                 : "memory", "scc", TQR_CHAIN_RES_CLOBBERS);
#undef TQR_RES_INS
}

#define TQR_RES_IO(TEXT, ...) asm volatile(TEXT ::__VA_ARGS__ : "memory", TQR_CHAIN_RES_CLOBBERS)

// stores of the other bank's pairs after group g (0, 1): 16 operations
template <int OB>
__device__ __forceinline__ void res_xst(int g, unsigned loff, __amdgpu_buffer_rsrc_t xout) {
  if (g == 0) {
    if constexpr (OB == 0) TQR_RES_IO(TQR_CHAIN_RES_XST0_X0, [loff] "v"(loff), [xout] "s"(xout));
    else TQR_RES_IO(TQR_CHAIN_RES_XST0_X1, [loff] "v"(loff), [xout] "s"(xout));
  } else {
    if constexpr (OB == 0) TQR_RES_IO(TQR_CHAIN_RES_XST1_X0, [loff] "v"(loff), [xout] "s"(xout));
    else TQR_RES_IO(TQR_CHAIN_RES_XST1_X1, [loff] "v"(loff), [xout] "s"(xout));
  }
}
// loads of the next element's pairs into the other bank after group g (2..7): TQR_CHAIN_RES_NLD(g)
template <int OB>
__device__ __forceinline__ void res_xld(int g, unsigned loff, __amdgpu_buffer_rsrc_t xin) {
#define TQR_RES_XLD_CASE(G)                                                                  \
  case G:                                                                                    \
    if constexpr (OB == 0) TQR_RES_IO(TQR_CHAIN_RES_XLD##G##_X0, [loff] "v"(loff), [xin] "s"(xin)); \
    else TQR_RES_IO(TQR_CHAIN_RES_XLD##G##_X1, [loff] "v"(loff), [xin] "s"(xin));            \
    break;
  switch (g) { TQR_RES_XLD_CASE(2) TQR_RES_XLD_CASE(3) TQR_RES_XLD_CASE(4) TQR_RES_XLD_CASE(5) TQR_RES_XLD_CASE(6) TQR_RES_XLD_CASE(7) }
#undef TQR_RES_XLD_CASE
}
// the head strip's group g loaded / stored (4 operations)
__device__ __forceinline__ void res_head(int g, bool store, unsigned loff, __amdgpu_buffer_rsrc_t hrs) {
#define TQR_RES_H_CASE(G)                                                          \
  case G:                                                                          \
    if (store) TQR_RES_IO(TQR_CHAIN_RES_HST##G, [loff] "v"(loff), [hrs] "s"(hrs)); \
    else TQR_RES_IO(TQR_CHAIN_RES_HLD##G, [loff] "v"(loff), [hrs] "s"(hrs));       \
    break;
  switch (g) {
    TQR_RES_H_CASE(0) TQR_RES_H_CASE(1) TQR_RES_H_CASE(2) TQR_RES_H_CASE(3)
    TQR_RES_H_CASE(4) TQR_RES_H_CASE(5) TQR_RES_H_CASE(6) TQR_RES_H_CASE(7)
  }
#undef TQR_RES_H_CASE
}

template <class C>
__device__ __noinline__ void flow_chain_res(const FlowArgs& a, int s_, int i0_, int i1_, int j_, int k_, int seg_,
                                            double* lds, int* sflag) {
  constexpr int B = 256;
  static_assert(C::NW == 4 && C::IB == 32 && C::WPC == 1, "resident chain: ShapeR");
  using S = double;
  using G = FGeo<B, C>;
  constexpr int NG = G::NG, BUF = G::VIMG + G::TPIMG, NRI = G::NRI, VP = G::VP;
  constexpr int SW = C::SW;
  static_assert(NG == 8, "resident chain: 8 groups of 32 reflectors");
  const int s = uni(s_), i0 = uni(i0_), i1 = uni(i1_), j = uni(j_), k = uni(k_), seg = uni(seg_);
  S* A = uni((S*)a.A);
  const size_t ldm = uni64(a.ldm);
  const int t = threadIdx.x, lane = t & 63, x = lane >> 4, y = lane & 3;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool pw = w == (chain_pt<C>() >> 6);  // the poll wave (uniform)
  const size_t colo = uni64((size_t)(s * SW + 16 * w) * ldm);
  S* const Aj = uni(A + (size_t)(j / uni(a.cdiv)) * B * ldm);
  S* const At = Aj + (size_t)k * B;
  double* const wk = uni(a.Wk[k]);
  const int P = uni(a.p), Q = uni(a.q), NS = uni(a.ns);
  int* const err = uni(a.err);
  int* const Tc = uni(a.Tc);
  auto vimg = [&](int i_, int g_) { return uni(wk + flow_vw_off<B, S, C>(P, i_, k, g_)); };
  auto timg = [&](int i_, int g_) { return uni(wk + flow_tw_off<B, S, C>(P, i_, k, g_)); };
  int* const rc = uni(&a.Rc[(size_t)k * NG]);
  int* const acg = uni(&a.Ac[(((size_t)k * Q + j) * NS + s) * NG]);
  auto tc = [&](int i) { return uni(&Tc[((size_t)i * Q + j) * NS + s]); };
  int par = 0;
  PanelViewU<NG> pv;
  pv.init(sflag + 260, sflag + 57);
  int* const tcs = sflag + 58;
  int* const fls = sflag + 59;
  int* const acs = sflag + 60;
  if (pw) {
    pv.reset();
    *lds_int(tcs) = -1;
    *lds_int(fls) = -1;
    *lds_int(acs) = -1;
  }
  const bool remote = a.dist && tile_owner(k, a.world, a.cyclic) != a.rank;
  int* const rf = uni(a.Rf + (size_t)k * P * NG);
  const int ep = uni(a.epoch);
  int fl_pf = -1;
  auto ready = [&](int i_, int g_) -> bool {
    if (!remote) return pv.ensure(rc, g_, i_ - k + 1, err);
    const int fi = i_ * NG + g_;
    if (fi == fl_pf && lds_u(fls) >= ep) return true;
    return spin_ge_u(rf + fi, ep, err, true);
  };
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) void*)lds);
  const unsigned oz = (unsigned)((x * VP + y * NRI) * 8), ox = (unsigned)((y * VP + x * NRI) * 8);
  const unsigned ot = (unsigned)(G::VIMG * 8 + (x * 4 + y) * NRI * 8);
  const unsigned loff = head_off_pair<B>(ldm, 0);
  const unsigned vl16 = 16u * lane;
  const __amdgpu_buffer_rsrc_t hrs = uniform_rsrc(At + colo);
  if (k == 0 && a.Uc) {  // host-pointer API: tile column j uploaded (xfer.hpp)
    const bool ok = pw ? spin_ge_u(&a.Uc[j], a.nxc, err) : true;
    if (!ca_sync<0>(ok, pw, sflag, par)) return;
  }
  const int ifirst = seg == 0 ? k : i0;
  FST(6);
  // ---- task start: dependencies, group 0's images, the first strip (bank 0), the head strip ----
  {
    bool ok = true;
    if (pw) {
      if (seg > 0) ok = spin_ge_u(&acg[0], seg, err);
      FST(9);
      if (ok && k > 0) ok = spin_ge_u(tc(ifirst), k, err);
      FST(8);
      if (ok) ok = ready(ifirst, 0);
    }
    FST(j == k + 1 ? 18 : 19);
    if (!ca_sync<0>(ok, pw, sflag, par)) return;
    FST(7);
  }
  {
    unsigned m0s, st;
    asm volatile(TQR_CHAIN_ASM4_DMA_B256 : [m0s] "=&s"(m0s), [st] "=&s"(st)
                 : [svsrc] "s"(vimg(ifirst, 0)), [stsrc] "s"(timg(ifirst, 0)), [sdst] "s"(sreg(lds0)), [sw] "s"(w),
                   [vl16] "v"(vl16)
                 : "memory", "scc", TQR_CHAIN_RES_CLOBBERS);
    S* const X0t = ifirst == k ? At : Aj + (size_t)ifirst * B;
    TQR_RES_IO("s_nop 4\n\t" TQR_CHAIN_RES_STRIP_LOAD_X0, [loff] "v"(loff), [xin] "s"(uniform_rsrc(X0t + colo)));
    if (seg == 0) TQR_RES_IO(TQR_CHAIN_RES_PARK_ZERO, "v"(0));  // the first element is the UNMQR: no head
    else res_head(0, false, loff, hrs);
    FST(4);
  }
  int nio = 0;            // operations of the last I/O statement (left in flight at the next sync)
  int buf = 0, bank = 0;  // LDS image buffer; AGPR bank of the current element
  bool has_prev = false, prev_unmqr = false;
  S* Xprev = nullptr;
  int iprev = 0;
  bool first = true;
  for (int i = ifirst; i < i1 || i == k; i = (i == k ? i0 : i + 1)) {
    const bool ts = i != k;
    S* const Xt = ts ? Aj + (size_t)i * B : At;
    const int inext = uni((i == k) ? i0 : i + 1);
    const bool has_next = uni(inext < i1 ? 1 : 0) != 0;
    S* const Xn = Aj + (size_t)(has_next ? inext : i) * B;
    const bool last = !has_next;
    const bool store_prev = has_prev && !prev_unmqr;
    const bool head_out = last && ts;  // the segment's last element stores the head strip group by group
    for (int g = 0; g < NG; ++g) {
      bool ok = true;
      if (pw) {
        // the next element's strip is loaded after groups 2..7: its tile must have received step k-1
        if (g == 2 && has_next && k > 0 && lds_u(tcs) < k) ok = spin_ge_u(tc(inext), k, err);
        // a later segment's head rows of group g + 1, loaded after this group (first element)
        if (ok && first && seg > 0 && g + 1 < NG && !(lds_u(acs) >= seg)) ok = spin_ge_u(&acg[g + 1], seg, err);
        if (ok) {
          if (g + 1 < NG) ok = ready(i, g + 1);
          else if (has_next) ok = ready(inext, 0);
        }
      }
      FST(j == k + 1 ? 20 : 0);
      // the first group of the task waits for everything (strip, head group 0, images)
      const bool v = (first && g == 0) ? ca_sync<0>(ok, pw, sflag, par) : res_sync(nio, ok, pw, sflag, par);
      if (!v) return;
      FST(7);
      // publishes of operations complete at this sync (older than the LDS-DMA it waited for)
      if (g == 3 && store_prev) publish_after_drain(tc(iprev), 1);
      if (head_out && g >= 2) publish_after_drain(&acg[g - 2], 1);
      if (pw) {
        const int tg = next_test_group<NG>(g);
        const bool here = g + 2 < NG;
        if (here || has_next) {
          if (!remote) {
            pv.prefetch(rc, tg);
          } else {
            fl_pf = (here ? i : inext) * NG + tg;
            lds_prefetch_u(rf + fl_pf, fls, true);
          }
        }
        if (g == 0 && has_next && k > 0) lds_prefetch_u(tc(inext), tcs, false);
        if (first && seg > 0 && g + 2 < NG) lds_prefetch_u(&acg[g + 2], acs, false);
      }
      const int gd = g + 1 < NG ? g + 1 : has_next ? 0 : g, id = g + 1 < NG ? i : has_next ? inext : i;
      const unsigned vb = lds0 + (unsigned)(buf * BUF * 8);
      ResGroup o;
      o.vz = vb + oz;
      o.vx = vb + ox;
      o.vt = vb + ot;
      o.vl16 = vl16;
      o.svsrc = vimg(id, gd);
      o.stsrc = timg(id, gd);
      o.sdst = sreg(lds0 + (unsigned)((buf ^ 1) * BUF * 8));
      o.sw = w;
      o.gidx = (int)sreg((unsigned)(16 * g));
      const bool sw = has_prev && g == 0;
      if (bank == 0) {
        if (sw) res_body<0, true>(o);
        else res_body<0, false>(o);
      } else {
        if (sw) res_body<1, true>(o);
        else res_body<1, false>(o);
      }
      FST(3);
      // ---- I/O after the body ----
      nio = 0;
      if (g < 2 && store_prev) {
        const __amdgpu_buffer_rsrc_t xo = uniform_rsrc(Xprev + colo);
        if (bank == 0) res_xst<1>(g, loff, xo);
        else res_xst<0>(g, loff, xo);
        nio += TQR_CHAIN_RES_NST;
      }
      if (g >= 2 && has_next) {
        const __amdgpu_buffer_rsrc_t xi = uniform_rsrc(Xn + colo);
        if (bank == 0) res_xld<1>(g, loff, xi);
        else res_xld<0>(g, loff, xi);
        nio += TQR_CHAIN_RES_NLD(g);
      }
      if (first && seg > 0 && g + 1 < NG) {
        res_head(g + 1, false, loff, hrs);
        nio += 4;
      }
      if (head_out) {
        res_head(g, true, loff, hrs);
        nio += 4;
      }
      FST(4);
      buf = uni(buf ^ 1);
    }
    if (!ts) {  // the UNMQR element's result is the head strip of the TSMQR elements that follow
      if (bank == 0) TQR_RES_IO(TQR_CHAIN_RES_PARK_FROM_X0, "v"(0));
      else TQR_RES_IO(TQR_CHAIN_RES_PARK_FROM_X1, "v"(0));
    }
    has_prev = true;
    prev_unmqr = !ts;
    Xprev = Xt;
    iprev = i;
    bank ^= 1;
    first = false;
  }
  // ---- task end: the last element's strip (an UNMQR's: the head tile, stored whole), drained ----
  {
    const int lb = bank ^ 1;  // the last element's bank
    if (!prev_unmqr) {
      const __amdgpu_buffer_rsrc_t xo = uniform_rsrc(Xprev + colo);
      if (lb == 0) TQR_RES_IO("s_nop 4\n\t" TQR_CHAIN_RES_STRIP_STORE_X0, [loff] "v"(loff), [xout] "s"(xo));
      else TQR_RES_IO("s_nop 4\n\t" TQR_CHAIN_RES_STRIP_STORE_X1, [loff] "v"(loff), [xout] "s"(xo));
    } else {
      for (int g = 0; g < NG; ++g) res_head(g, true, loff, hrs);
    }
  }
  ca_sync<0>(true, pw, sflag, par);
  FST(4);
  publish_after_drain(tc(iprev), 1);
  if (prev_unmqr) {
    for (int g = 0; g < NG; ++g) publish_after_drain(&acg[g], 1);
  } else {
    publish_after_drain(&acg[NG - 2], 1);
    publish_after_drain(&acg[NG - 1], 1);
  }
}

}  // namespace tqr
