// Tile operations of the flat-tree tiled QR for gfx950 (CDNA4), fp64 arithmetic.
//
// The four reference tile kernels (qrdecomp.c:532 GEQRT "QRS", :559 UNMQR "SAPP",
// :689 TSQRT "QRD", :723 TSMQR "DAPP"; device versions gpucalc.cu:1013-1359) are
// re-designed around compact-WY block reflectors with inner blocking IB = 32:
//
//   * a reflector group g (IB consecutive reflectors of a tile) is applied to a column strip
//     X as   Z = [head] + V_g^T X ;  W = T_g^T Z ;  [head] -= W ;  X -= V_g W
//     with the three products on v_mfma_f64_4x4x4_4b_f64 (measured ~1.5x the issue rate of
//     v_mfma_f64_16x16x4_f64 on gfx950, profiles/r01_ubench_mfma.txt);
//   * the IB-column panel of GEQRT/TSQRT is factorised in LDS, reflector by reflector, with
//     the reference's conventions (qrdecomp.c:1201-1272): sign(0) = +1, v scaled to v0 = 1
//     by the reciprocal of x0 + sign*|x|, no scaling for a zero column, tau = 2/(v'v);
//   * T_g (IB x IB upper triangular, LAPACK dlarft "forward, columnwise") is formed from the
//     Gram matrix V_g^T V_g, itself one MFMA product.
//
// Mathematically every tile op applies exactly the reflectors the reference applies, in the
// same order; only the rounding differs (parity tolerances in tests/).
//
// Register layout of a 4x4x4_4b operand (probed, profiles/r01_ubench_mfma_probe.txt):
// lane = 16*x + 4*blk + y holds A[blk][i=y][k=x], B[blk][k=x][j=y], D[blk][i=x][j=y].
// A wave owns a strip of 16 matrix columns (blk = column quad, y = column in quad); register
// X[ks] holds rows 4ks..4ks+3 of the strip (row 4ks+x at lane x), which is at the same time
// the B-operand layout (k = row) and the accumulator layout (i = row) — so the strip is both
// summed over (Z = V^T X) and updated (X -= V W) without any data movement.
#pragma once
#include <hip/hip_runtime.h>

namespace tqr {

constexpr int NT = 256;  // threads per workgroup (4 waves)

__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

template <int B>
struct Geo {
  static constexpr int IB = B < 32 ? B : 32;  // reflectors per group
  static constexpr int NG = B / IB;           // groups per tile
  static constexpr int NKS = B / 4;           // 4-row k-steps over a tile
  static constexpr int NRI = IB / 4;          // 4-row blocks of a group
  static constexpr int VP = IB + 2;           // LDS pitch (doubles) of the V image, 16-B rows
  static constexpr int TP = IB + 1;           // LDS pitch of T / Gram / head images
  static constexpr int VSZ = B * VP;          // V image (doubles)
  static constexpr int TSZ = IB * TP;         // T image (doubles)
  // V image column permutation: the NRI values a lane needs per row are contiguous.
  __device__ static constexpr int pc(int c) { return (c & 3) * NRI + (c >> 2); }
};

template <typename S>
__device__ __forceinline__ double ld(const S* p) { return (double)*p; }
template <typename S>
__device__ __forceinline__ void st(S* p, double v) { *p = (S)v; }

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
template <int B, bool HEAD>
__device__ __forceinline__ void apply_group(const double* __restrict__ Vs, const double* __restrict__ Ts,
                                            double (&X)[Geo<B>::NKS], double (&H)[Geo<B>::NRI], int ks0) {
  using g = Geo<B>;
  constexpr int NRI = g::NRI, NKS = g::NKS, VP = g::VP, TP = g::TP;
  const int lane = threadIdx.x & 63, x = lane >> 4, y = lane & 3;
  double Z[NRI];
#pragma unroll
  for (int r = 0; r < NRI; ++r) Z[r] = HEAD ? H[r] : 0.0;
  // Z += V^T X   (A operand: V[4ks+x][4ri+y])
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (!HEAD && ks < ks0) continue;
    const double2* vr = reinterpret_cast<const double2*>(Vs + (4 * ks + x) * VP + y * NRI);
    double a[NRI];
#pragma unroll
    for (int h = 0; h < NRI / 2; ++h) {
      double2 t = vr[h];
      a[2 * h] = t.x;
      a[2 * h + 1] = t.y;
    }
#pragma unroll
    for (int r = 0; r < NRI; ++r) Z[r] = mfma4(a[r], X[ks], Z[r]);
  }
  // W = T^T Z   (A operand: T[4k2+x][4wi+y]); T upper triangular -> k2 <= wi.
  double W[NRI];
#pragma unroll
  for (int wi = 0; wi < NRI; ++wi) {
    double acc = 0.0;
#pragma unroll
    for (int k2 = 0; k2 <= wi; ++k2) acc = mfma4(Ts[(4 * k2 + x) * TP + 4 * wi + y], Z[k2], acc);
    W[wi] = -acc;
  }
  if (HEAD) {
#pragma unroll
    for (int r = 0; r < NRI; ++r) H[r] += W[r];
  }
  // X -= V W   (A operand: V[4ks+y][4wi+x]); 4 row blocks interleaved to hide MFMA latency.
#pragma unroll
  for (int kb = 0; kb < NKS; kb += 4) {
    if (!HEAD && kb + 3 < ks0) continue;
    double a[4][NRI];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double2* vr = reinterpret_cast<const double2*>(Vs + (4 * (kb + u) + y) * VP + x * NRI);
#pragma unroll
      for (int h = 0; h < NRI / 2; ++h) {
        double2 t = vr[h];
        a[u][2 * h] = t.x;
        a[u][2 * h + 1] = t.y;
      }
    }
#pragma unroll
    for (int wi = 0; wi < NRI; ++wi)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (HEAD || kb + u >= ks0) X[kb + u] = mfma4(a[u][wi], W[wi], X[kb + u]);
  }
}

// Strip loads/stores: X[ks] <- tile(rows 4ks+x, column col0 + 4blk + y).
template <int B, typename S>
__device__ __forceinline__ void load_strip(double (&X)[Geo<B>::NKS], const S* __restrict__ tile, size_t ldm,
                                           int col0, int ks0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = col0 + (lane & 15);
  const S* p = tile + (size_t)c * ldm + x;
#pragma unroll
  for (int ks = 0; ks < Geo<B>::NKS; ++ks) X[ks] = ks >= ks0 ? ld(p + 4 * ks) : 0.0;
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
template <int B, typename S>
__device__ __forceinline__ void load_head(double (&H)[Geo<B>::NRI], const S* __restrict__ tile, size_t ldm,
                                          int r0, int col0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = col0 + (lane & 15);
  const S* p = tile + (size_t)c * ldm + r0 + x;
#pragma unroll
  for (int r = 0; r < Geo<B>::NRI; ++r) H[r] = ld(p + 4 * r);
}
template <int B, typename S>
__device__ __forceinline__ void store_head(const double (&H)[Geo<B>::NRI], S* __restrict__ tile, size_t ldm,
                                           int r0, int col0) {
  const int lane = threadIdx.x & 63, x = lane >> 4, c = col0 + (lane & 15);
  S* p = tile + (size_t)c * ldm + r0 + x;
#pragma unroll
  for (int r = 0; r < Geo<B>::NRI; ++r) st(p + 4 * r, H[r]);
}

// ---------------------------------------------------------------------------------------
// LDS staging of a reflector group.
// ---------------------------------------------------------------------------------------
// TS-type: Vs[r][c] = V_B[r][c0+c] of a TSQRT tile (dense B x IB block).
template <int B, typename S>
__device__ __forceinline__ void stage_v_ts(double* Vs, const S* __restrict__ vt, size_t ldm, int c0) {
  using g = Geo<B>;
  for (int idx = threadIdx.x; idx < B * g::IB; idx += NT) {
    int r = idx % B, c = idx / B;
    Vs[r * g::VP + g::pc(c)] = ld(vt + (size_t)(c0 + c) * ldm + r);
  }
}
// GE-type: explicit unit-lower trapezoid of a GEQRT tile: 0 above row c0+c, 1 on it.
template <int B, typename S>
__device__ __forceinline__ void stage_v_ge(double* Vs, const S* __restrict__ vt, size_t ldm, int c0) {
  using g = Geo<B>;
  for (int idx = threadIdx.x; idx < B * g::IB; idx += NT) {
    int r = idx % B, c = idx / B, d = c0 + c;
    Vs[r * g::VP + g::pc(c)] = r < d ? 0.0 : (r == d ? 1.0 : ld(vt + (size_t)d * ldm + r));
  }
}
template <int B>
__device__ __forceinline__ void stage_t(double* Ts, const double* __restrict__ tg) {
  using g = Geo<B>;
  for (int idx = threadIdx.x; idx < g::IB * g::IB; idx += NT) {
    int r = idx / g::IB, c = idx % g::IB;
    Ts[r * g::TP + c] = tg[idx];
  }
}

// ---------------------------------------------------------------------------------------
// Panel factorisation of reflector group g in LDS (all NT threads).
// GE (GEQRT): Vs holds tile rows 0..B-1 of the IB panel columns (rows < c0 unused).
// TS (TSQRT): Hs holds the IB x IB head block R[c0.., c0..] (upper part used), Vs the B x IB
// block of the tile below. On exit: R entries in place, V (unit diag implied) in place,
// tauv[c] = tau of reflector c. scratch: >= 8*33 + 2*(IB+1) + 4 doubles.
// ---------------------------------------------------------------------------------------
template <int B, bool TS>
__device__ void panel_factor(double* Vs, double* Hs, double* tauv, double* scratch, int c0) {
  using g = Geo<B>;
  constexpr int IB = g::IB, VP = g::VP, TP = g::TP;
  double* red2 = scratch;             // 8 x 33 partial dots
  double* dsum = scratch + 8 * 33;    // IB + 1: full dots d_j, dsum[IB] = tail dot of the pivot
  double* red = dsum + 2 * (IB + 1);  // 4
  const int t = threadIdx.x, jj = t & 31, ch = t >> 5;
  for (int c = 0; c < IB; ++c) {
    const int rc = TS ? -1 : c0 + c;  // GE: tile row of the reflector head; tail rows > rc
    const int pcc = g::pc(c);
    const double x0 = TS ? Hs[c * TP + c] : Vs[rc * VP + pcc];
    double xr = (t > rc && t < B) ? Vs[t * VP + pcc] : 0.0;
    const double s = block_sum(xr * xr, red);
    const double norm = sqrt(x0 * x0 + s);
    const double hd = x0 + (x0 >= 0.0 ? norm : -norm);
    const double scale = norm != 0.0 ? 1.0 / hd : 1.0;
    // partial dots of the tail rows with the (scaled) reflector, columns c..IB-1
    double part = 0.0;
    if (jj >= c && jj < IB) {
      const int pj = g::pc(jj);
      for (int r = rc + 1 + ch; r < B; r += 8) part += Vs[r * VP + pj] * (Vs[r * VP + pcc] * scale);
    }
    red2[ch * 33 + jj] = part;
    __syncthreads();
    if (t >= c && t < IB) {
      double d = 0.0;
#pragma unroll
      for (int q = 0; q < 8; ++q) d += red2[q * 33 + t];
      const double head = TS ? Hs[c * TP + t] : Vs[rc * VP + g::pc(t)];
      dsum[t] = head + d;
      if (t == c) dsum[IB] = d;
    }
    __syncthreads();
    const double tau = 2.0 / (1.0 + scale * dsum[IB]);
    if (jj > c && jj < IB) {
      const int pj = g::pc(jj);
      const double f = tau * dsum[jj];
      for (int r = rc + 1 + ch; r < B; r += 8) Vs[r * VP + pj] -= f * (Vs[r * VP + pcc] * scale);
      if (ch == 0) {
        if (TS) Hs[c * TP + jj] -= f;
        else Vs[rc * VP + pj] -= f;
      }
    }
    __syncthreads();
    if (t > rc && t < B) Vs[t * VP + pcc] *= scale;
    if (t == 0) {
      const double rcc = x0 - tau * dsum[c];
      if (TS) Hs[c * TP + c] = rcc;
      else Vs[rc * VP + pcc] = rcc;
      tauv[c] = tau;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// T_g from the explicit V image and tauv: Gram G = V^T V on MFMA (waves 0..IB/16-1), then
// T[c][c] = tau_c, T[0:c,c] = -tau_c T[0:c,0:c] G[0:c,c] column by column.
// Gs, Ts: IB x TP images. ks0: first non-zero 4-row block of V (GE), 0 for TS.
// ---------------------------------------------------------------------------------------
template <int B>
__device__ void build_t(const double* Vs, const double* tauv, double* Gs, double* Ts, int ks0) {
  using g = Geo<B>;
  constexpr int IB = g::IB, VP = g::VP, TP = g::TP, NKS = g::NKS, NRI = g::NRI;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, x = lane >> 4, y = lane & 3, blk = (lane >> 2) & 3;
  if (w < (IB + 15) / 16) {
    const int cb = 16 * w + 4 * blk + y;  // Gram column of this lane's B operand
    double Z[NRI];
#pragma unroll
    for (int r = 0; r < NRI; ++r) Z[r] = 0.0;
    if (cb < IB) {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        if (ks < ks0) continue;
        const double xb = Vs[(4 * ks + x) * VP + g::pc(cb)];
        const double2* vr = reinterpret_cast<const double2*>(Vs + (4 * ks + x) * VP + y * NRI);
        double a[NRI];
#pragma unroll
        for (int h = 0; h < NRI / 2; ++h) {
          double2 tt = vr[h];
          a[2 * h] = tt.x;
          a[2 * h + 1] = tt.y;
        }
#pragma unroll
        for (int r = 0; r < NRI; ++r) Z[r] = mfma4(a[r], xb, Z[r]);
      }
    } else {
      // IB = 16 with 16 Gram columns per wave: no idle lanes; kept for generality.
    }
    if (cb < IB) {
#pragma unroll
      for (int r = 0; r < NRI; ++r) Gs[(4 * r + x) * TP + cb] = Z[r];
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  for (int c = 0; c < IB; ++c) {
    if (t < c) {
      double acc = 0.0;
      for (int s = t; s < c; ++s) acc += Ts[t * TP + s] * Gs[s * TP + c];
      Ts[t * TP + c] = -tauv[c] * acc;
    } else if (t < IB) {
      Ts[t * TP + c] = t == c ? tauv[c] : 0.0;
    }
    __syncthreads();
  }
}

}  // namespace tqr
