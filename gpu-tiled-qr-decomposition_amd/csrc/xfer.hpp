// Host <-> HBM transfers inside the persistent launch (the host-pointer API, tqr_*geqrt_host /
// cudaQRTask / taskQRP_threads; reference gpucalc.cu:1614-1619 / 1665-1670 copy one column per
// cudaMemcpy before / after the kernel).
//
// The launch streams its own input in and its result out over PCIe, so the transfers overlap the
// factorisation instead of bracketing it:
//   UP(j, c)    copies rows chunk c of tile column j from host memory (the caller's registered
//               array, or the pinned staging buffer the host fills column by column while the
//               kernel runs — then it first polls the host's flag hup[j]) into the device matrix,
//               with write-through (sc1) 16-B stores, then bumps Uc[j]. Step 0 is the only step
//               that reads a column before its upload: GEQRT(0)/TSQRT(i,0) wait for Uc[0], the
//               chains of step 0 on column j for Uc[j].
//   DOWN(j, c)  waits until tile column j is final — every chain of the steps k < j on column j
//               has published its last segment's head rows (Ac), panel j's last member its last
//               group (Rt) — and copies rows chunk c to host memory with system-scope stores;
//               with a staging buffer it then sets the host flag hdn[j][c] (release, system scope)
//               so the host can move that chunk on while the kernel keeps running.
// Host memory is fine-grained (pinned coherent staging) or registered: every GPU access to it is
// system scope (sc0 sc1). The device-side hand-offs follow flow.hpp's protocol (sc1 stores,
// drained before one lane's counter add, sc1 loads after the poll).
#pragma once

namespace tqr {

constexpr int T_UP = 5, T_DOWN = 6;
constexpr int XFER_AUX_HOST = 17;  // sc0 | sc1: system scope

// thread FLOW_PT: is tile column j final? (see the header; the counts mirror build_flow_plan)
__device__ __noinline__ bool column_final(const FlowArgs& a, int j, int NG) {
  const int kend = min(j, a.kmax);
  for (int i = 0; i < kend; ++i) {
    const int sl = seglen_of_chain(i, j, a.kmax, a.seglen, a.seglen_la, a.la_tail, a.tail, a.tail_sl);
    const int nseg = nseg_of_chain(i, j, a.p, a.kmax, sl, a.ualone);
    for (int s = 0; s < a.ns; ++s)
      if (!spin_ge(&a.Ac[(((size_t)i * a.q + j) * a.ns + s) * NG + NG - 1], nseg, a.err)) return false;
  }
  if (j < a.kmax && !spin_ge(&a.Rt[(size_t)j * NG + NG - 1], a.p - j, a.err)) return false;
  return true;
}

// One chunk of one tile column between host memory and the device matrix: B columns of `nr`
// elements each, 16-B accesses when both sides allow them (else element by element). UNR columns
// at a time, KV 16-B vectors per lane and column in flight (a host read is a PCIe round trip).
template <typename S, bool UP, int NT>
__device__ __forceinline__ void xfer_columns(const FlowArgs& a, int B, int j, int r0, int nr) {
  const int t = threadIdx.x;
  S* dA = (S*)a.A;
  char* host = UP ? (char*)a.hsrc : (char*)a.hdst;
  const size_t hld = a.hld, dld = a.ldm;
  const size_t cb = (size_t)nr * sizeof(S);  // bytes per column of the chunk
  const bool v16 = (((size_t)host | (hld * sizeof(S)) | ((size_t)r0 * sizeof(S)) | cb) & 15) == 0;
  const int col0 = j * B;
  if (v16) {
    constexpr int UNR = 4, KV = 4;
    const int nv = (int)(cb / 16);
    for (int c0 = 0; c0 < B; c0 += UNR) {
      __attribute__((ext_vector_type(4))) unsigned v[UNR][KV];
      __amdgpu_buffer_rsrc_t hr[UNR], dr[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int col = col0 + min(c0 + u, B - 1);
        hr[u] = uniform_rsrc(host + ((size_t)col * hld + r0) * sizeof(S));
        dr[u] = uniform_rsrc(dA + (size_t)col * dld + r0);
      }
      for (int v0 = 0; v0 < nv; v0 += KV * NT) {
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
          for (int k = 0; k < KV; ++k) {
            const int x = v0 + k * NT + t;
            if (x < nv && c0 + u < B)
              v[u][k] = UP ? __builtin_amdgcn_raw_buffer_load_b128(hr[u], 16 * x, 0, XFER_AUX_HOST)
                           : __builtin_amdgcn_raw_buffer_load_b128(dr[u], 16 * x, 0, 16);
          }
#pragma unroll
        for (int u = 0; u < UNR; ++u)
#pragma unroll
          for (int k = 0; k < KV; ++k) {
            const int x = v0 + k * NT + t;
            if (x < nv && c0 + u < B) {
              if (UP) __builtin_amdgcn_raw_buffer_store_b128(v[u][k], dr[u], 16 * x, 0, 16);
              else __builtin_amdgcn_raw_buffer_store_b128(v[u][k], hr[u], 16 * x, 0, XFER_AUX_HOST);
            }
          }
      }
    }
  } else {  // unaligned host columns (odd leading dimension, unaligned array): element accesses
    for (int c = 0; c < B; ++c) {
      const int col = col0 + c;
      const __amdgpu_buffer_rsrc_t hr = uniform_rsrc(host + ((size_t)col * hld + r0) * sizeof(S));
      const __amdgpu_buffer_rsrc_t dr = uniform_rsrc(dA + (size_t)col * dld + r0);
      for (int r = t; r < nr; r += NT) {
        if constexpr (sizeof(S) == 8) {
          const auto v = UP ? __builtin_amdgcn_raw_buffer_load_b64(hr, 8 * r, 0, XFER_AUX_HOST)
                            : __builtin_amdgcn_raw_buffer_load_b64(dr, 8 * r, 0, 16);
          if (UP) __builtin_amdgcn_raw_buffer_store_b64(v, dr, 8 * r, 0, 16);
          else __builtin_amdgcn_raw_buffer_store_b64(v, hr, 8 * r, 0, XFER_AUX_HOST);
        } else {
          const auto v = UP ? __builtin_amdgcn_raw_buffer_load_b32(hr, 4 * r, 0, XFER_AUX_HOST)
                            : __builtin_amdgcn_raw_buffer_load_b32(dr, 4 * r, 0, 16);
          if (UP) __builtin_amdgcn_raw_buffer_store_b32(v, dr, 4 * r, 0, 16);
          else __builtin_amdgcn_raw_buffer_store_b32(v, hr, 4 * r, 0, XFER_AUX_HOST);
        }
      }
    }
  }
}

template <int B, typename S, class C>
__device__ __noinline__ void flow_xfer(const FlowArgs& a, bool up, int j, int c, int* sflag) {
  constexpr int NG = FGeo<B, C>::NG;
  const int r0 = c * a.xrows, nr = min(a.m - r0, a.xrows);
  FST(6);
  bool ok = true;
  if (threadIdx.x == FLOW_PT) {
    if (up) ok = !a.hup || spin_ge(a.hup + j, a.gen, a.err, true);  // the host staged column j
    else ok = column_final(a, j, NG);
  }
  if (!wg_verdict(ok, sflag)) return;
  if (up) {
    xfer_columns<S, true, C::NT>(a, B, j, r0, nr);
    wg_publish(&a.Uc[j], 1);  // sc1 stores drained, then one add
    // host-transfer progress: waits that expire while it moves keep waiting (flow.hpp timed_out)
    if (threadIdx.x == 0) __hip_atomic_fetch_add(gptr(a.err + 1), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    xfer_columns<S, false, C::NT>(a, B, j, r0, nr);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && a.hdn) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(a.hdn + (size_t)j * a.nxc + c, a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  FST(4);
}

}  // namespace tqr
