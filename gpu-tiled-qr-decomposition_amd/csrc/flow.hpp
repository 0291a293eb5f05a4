// Persistent dataflow engine ("flow"): one 512-thread workgroup per CU (engine shape ShapeW8;
// ShapeW4: two 256-thread workgroups) pulls tasks from a statically ordered list (atomic dequeue)
// and synchronises with other workgroups only through monotone progress counters in global memory
// (write-through stores drained before one lane's counter add, L1-bypassing loads after the poll:
// MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility", first table row).
//
// Tasks (the reference DAG of src/gridscheduler.c, regrouped):
//   QRS(k)          GEQRT of tile (k,k), reflector group by group;
//   QRD(i,k)        TSQRT of [R_kk; tile (i,k)], group by group;
//   CHAIN(k,j,s,e)  one 128-column strip s of tile column j at step k (ShapeW4: 64 columns):
//                   segment e of the chain
//                   UNMQR(k,j) (segment 0 only), TSMQR(i,j,k) for i in [i0,i1). The strip of
//                   tile (k,j) (the TSMQR head rows) stays owned by the chain across elements.
// Progress counters (zeroed per factorisation):
//   Rr[k][g]   members of panel k whose group-g factorisation (R diagonal block, V, tau) is in
//              memory — all the next member's factorisation of group g needs; build_t, the
//              images and the trailing update come after it, off the member-to-member path;
//   Rt[k][g]   members of panel k that finished the in-tile trailing update of group g (the R_kk
//              head rows of the group's columns right of it): the next member's trailing update
//              waits for it, its factorisation of group g does not (it needs only the 32 x 32
//              diagonal block, final at Rc) — so members are spaced by max(factor, trailing)
//              instead of their sum;
//   Rc[k][g]   members of panel k (GEQRT(k), TSQRT(k+1,k), ...) that finished group g — a
//              TSQRT's group g may start once its predecessor finished group g, so the flat
//              TS chain is pipelined at group (32-reflector) granularity, not tile granularity;
//   Tc[i][j][s] steps completed on strip s of tile (i,j);
//   Ac[k][j][s][g] segments of chain (k,j,s) whose head rows of group g are final (the next
//                 segment starts group g of its first element on it).
// Deadlock freedom: every wait is on a task earlier in the list (host checks it), and tasks are
// dequeued in list order, so the earliest unfinished dequeued task can always progress. Every
// spin is bounded (FLOW_TIMEOUT without progress of the host transfers: timed_out); on timeout an
// error word is set and all workgroups drain.
#pragma once
#include "tiles.hpp"

namespace tqr {

constexpr int T_CHAIN = 4;

// Diagnostic build only (make flowstamps): per-workgroup s_memrealtime sums by activity.
// Every FST(c) charges the time since the previous stamp to category c (LDS-resident sums,
// thread 0 only, written to g_fst[blockIdx.x][*] at exit). Categories: 0 chain waits,
// 1 panel waits, 2 chain head-row I/O, 3 chain apply (with the LDS-DMA issue), 4 chain strip
// I/O + publish, 5 panel compute, 6 dequeue/dispatch + kernel exit, 7 chain drain + barrier,
// 8 chain Tc waits (tile's previous step), 9 chain Ac waits (previous segment), 10 panel I/O +
// writeback + images, 11 panel build_t, 12 panel in-tile trailing update (+ its Rt publish),
// 13 chain phase 2 (X += V W; 3 is then phase 1 Z alone), 14 chain next-head load, 15 chain
// W = -T^T Z + head update, 16 panel trailing: strip/head loads, 17 panel trailing: stores
// (12 is then the trailing's MFMA part + Rt publish), 18 / 19 chain Rc waits at an element's
// start (lookahead column j = k+1 / other columns), 20 chain Rc waits inside a lookahead-column
// element (0 is then the same for other columns), 21 / 22 chain drain of the wave's own memory
// operations before the group's polls, groups > 0 / group 0 (stamps build only; at group 0 this
// includes the element's strip loads, which the real kernel overlaps with phase 1), 23 panel
// forwarding (multi-GPU: issuing the group's image copies to the peers, setting their flags).
constexpr int FST_N = 24;
constexpr int WSL = 8;  // per-wave stamp slots
#ifdef TQR_FLOW_STAMPS
extern __device__ unsigned long long g_fst[];
extern __device__ unsigned long long g_ttl[];  // per task: start, end (s_memrealtime), workgroup
#define FST(c)                                                                            \
  do {                                                                                    \
    if (threadIdx.x == 0) {                                                               \
      unsigned long long* l_ = reinterpret_cast<unsigned long long*>(sflag + 63);         \
      const unsigned long long n_ = __builtin_amdgcn_s_memrealtime();                     \
      l_[1 + (c)] += n_ - l_[0];                                                          \
      l_[0] = n_;                                                                         \
    }                                                                                     \
  } while (0)
// per-wave accounting (all 8 waves, lane 0; LDS tail ints 128.., written to g_wst at exit), WSL
// slots per wave: 0 own-memory drain and 1 barrier wait at the chain sync points; the fp64 chain's
// group loop (WMARK): 2 before the sync (polls), 3 after it (publish, setup), 4 phase 1 (Z, W, H),
// 5 head I/O, 6 phase 2, 7 after phase 2 (next-head hand-over, loop)
extern __device__ unsigned long long g_wst[];
#define WST_T0() const unsigned long long wst0_ = __builtin_amdgcn_s_memrealtime()
#define WST_ACC(slot, tref)                                                                        \
  do {                                                                                             \
    const unsigned long long n_ = __builtin_amdgcn_s_memrealtime();                                \
    if ((threadIdx.x & 63) == 0) {                                                                 \
      __attribute__((address_space(3))) unsigned long long* w_ =                                   \
          (__attribute__((address_space(3))) unsigned long long*)(sflag + 127) + WSL * (threadIdx.x >> 6); \
      w_[slot] += n_ - (tref);                                                                     \
    }                                                                                              \
  } while (0)
#define WST_MID() const unsigned long long wst1_ = __builtin_amdgcn_s_memrealtime(); WST_ACC(0, wst0_)
#define WST_END() WST_ACC(1, wst1_)
#define WST_ENDS(slot) WST_ACC(slot, wst1_)
// group trace of workgroup 0 (stamps build): per group and wave, the s_memrealtime of marks
// 0 loop top, 1 before the sync point, 2 after it, 3 phase 1 start, 4 phase 1 end, 5 head I/O end,
// 6 phase 2 end (tools/group_trace.py)
constexpr int GTR_GROUPS = 4096;
extern __device__ unsigned long long g_gtr[];
extern __device__ unsigned long long g_xtr[];  // [group][wave][8]: XPipe phase-2 progress marks
#define GTR(mark, tval)                                                                              \
  do {                                                                                               \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && gtr_n < GTR_GROUPS)                            \
      g_gtr[((size_t)gtr_n * 8 + (threadIdx.x >> 6)) * 8 + (mark)] = (tval);                         \
  } while (0)
#define WMARK_INIT() unsigned long long wt_ = __builtin_amdgcn_s_memrealtime()
#define WMARK(slot)                     \
  do {                                  \
    WST_ACC(slot, wt_);                 \
    wt_ = __builtin_amdgcn_s_memrealtime(); \
    GTR(wmark_gtr(slot), wt_);          \
  } while (0)
__device__ constexpr int wmark_gtr(int slot) { return slot == 7 ? 0 : slot == 2 ? 1 : slot == 3 ? 3 : slot == 4 ? 4 : slot == 5 ? 5 : 6; }
#else
#define FST(c) do {} while (0)
#define WST_T0() do {} while (0)
#define WMARK_INIT() do {} while (0)
#define WMARK(slot) do {} while (0)
#define GTR(mark, tval) do {} while (0)
#define WST_MID() do {} while (0)
#define WST_END() do {} while (0)
#define WST_ENDS(slot) do {} while (0)
#endif
// 512 threads = 8 waves = two waves per SIMD: a chain task updates a 128-column strip, so each
// LDS-DMA'd V/T image serves twice the flops of the 4-wave / 64-column form, and each SIMD's
// second wave issues MFMAs while the first waits on LDS, the memory pipeline or a barrier.
// The register budget is then 256 per wave (X strip 128, operands unpipelined — FLOW_PF off);
// it fits without inner-loop spills once the counter polls are global (not FLAT) loads and the
// UNMQR element shares the TSMQR code (see flow_chain). 4 waves (FLOW_NT = 256, pipelined operand
// reads) measured 159 ms at 16384^2 against 148.5 ms for this form.
constexpr int FLOW_NT = 512;
constexpr int FLOW_NW = FLOW_NT / 64;      // waves
constexpr int FLOW_SW = 16 * FLOW_NW;      // strip width (columns) of a chain task
constexpr bool FLOW_PF = true;

// Engine shapes. ShapeW8 is the form above (one 8-wave workgroup per CU, 128-column chain strips,
// 32-reflector groups): the default. ShapeW4 (round 4, fp64 under TQR_FLOW_SHAPE=w4): TWO
// independent 4-wave workgroups per CU, 64-column chain strips, 16-reflector groups — half the LDS
// images (76 KiB per workgroup, so two fit in the CU's 160 KiB), the two workgroups running
// different tasks, so that one's strip hand-over, barrier skew and dependent-MFMA tails could run
// beside the other's MFMA stream. Measured: no gain — the chain loop alone is 3-4 % slower
// (tools/ubench/chain2_bench.hip: the hand-over's cost is not hidden by the co-resident workgroup,
// with or without the two out of phase) and the factorisation 9 % (138.6 vs 126.7 ms at 16384^2).
template <int NW_, int IB_, int WPC_>
struct FlowShape {
  static constexpr int NW = NW_, NT = 64 * NW_, SW = 16 * NW_, IB = IB_, WPC = WPC_;
};
using ShapeW8 = FlowShape<8, 32, 1>;
using ShapeW4 = FlowShape<4, 16, 2>;
// the tile geometry a shape runs at (groups of min(B, IB) reflectors)
template <int B, class C>
using FGeo = Geo<B, (B < C::IB ? B : C::IB)>;
// cache policy of the chain's in-segment head-row traffic (buffer aux bits; 16 = sc1, 2 = nt)
#ifndef TQR_HEAD_ST_AUX
#define TQR_HEAD_ST_AUX 0
#endif
#ifndef TQR_HEAD_LD0_AUX  // (an element's first group)
#define TQR_HEAD_LD0_AUX 16
#endif
#ifndef TQR_HEAD_LD_AUX
#define TQR_HEAD_LD_AUX 18  // sc1 | nt: 129.86 vs 130.03-130.14 ms (2 A/B rounds; nt stores: 130.2, slower)
#endif  // software-pipelined operand reads (also at 2 waves/SIMD)
// The thread that polls a task's dependency counters, keeps the Rc view and writes the sync-point
// verdicts (publishes stay with thread 0).
#ifndef TQR_POLL_T
#define TQR_POLL_T 0
#endif
constexpr int FLOW_PT = TQR_POLL_T;
// The fp64 chain polls from wave 7: thread 0's wave also carries the publishes, and the waves'
// stamps showed it the last to reach most group barriers (its partner and waves 1-3 waiting on
// it); the upper waves, favoured in phase 1 (phase_prio), have slack. 130.6-130.9 ms against
// 132.6-133.0 at 16384^2 (waves 4-7 alike; moving the publishes as well measured no better).
#ifndef TQR_CHAIN_PT
#define TQR_CHAIN_PT 448
#endif
constexpr int FLOW_CHAIN_PT = TQR_CHAIN_PT;  // the fp64 chain's poll thread (ShapeW8)
// ShapeW4: the last wave's first lane (as wave 7 of the 8-wave form)
template <class C>
__device__ constexpr int chain_pt() { return C::NW == 8 ? FLOW_CHAIN_PT : C::NT - 64; }
constexpr unsigned long long FLOW_TIMEOUT = 500000000ull;  // 5 s of s_memrealtime (100 MHz)
// A wait gives up once FLOW_TIMEOUT has passed with no progress of the launch's host transfers:
// the word after the error word (err[1]) counts the upload chunks done (xfer.hpp UP tasks; it
// stays 0 on device-resident launches). With the host-pointer API every wait may depend on the
// host staging the input column by column, as slowly as the host goes (a 32 GiB matrix on one host
// thread takes several seconds); each expiry that finds the count moved restarts the wait.
// last: the count seen at the previous expiry (0 before the first: device-resident launches keep
// the 5 s limit). Multi-GPU launches: every wait of a rank may depend, directly or through a local
// counter, on a peer whose launch started later (process start-up, first touch, a slow host), so
// once a multi-GPU plan exists the limit is g_flow_wait_limit (tqr_dist_plan_create: 60 s,
// TQR_PEER_TIMEOUT_S) — read only after the first 5 s. Cold path only.
__device__ unsigned long long g_flow_wait_limit = FLOW_TIMEOUT;
__device__ __forceinline__ bool timed_out(unsigned long long& t0, int& last, int* err) {
  const unsigned long long now = __builtin_amdgcn_s_memrealtime();
  if (now - t0 <= FLOW_TIMEOUT) return false;
  if (now - t0 <= __hip_atomic_load(&g_flow_wait_limit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
  const int pr = __hip_atomic_load((__attribute__((address_space(1))) int*)(err + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (pr != last) {
    last = pr;
    t0 = now;
    return false;
  }
  return true;
}

// Multi-GPU (tile-column cyclic partition, one process per GPU): peer buffers opened by IPC.
struct PeerBufs {
  double* const* Wk;  // the peer's panel workspaces (IPC-opened into this process), one per k
  int* Rf;            // the peer's member flags
};

struct FlowArgs {
  void* A;
  void* tau;
  // panel workspaces, one allocation per step k (each under the 2 GiB a single IPC export
  // handles): V images of (i, k, g) for i = k..p-1 (Geo<B>::VIMG slots), then T images (TIMG)
  double* const* Wk;
  const Item* tasks;
  int ntasks;
  long ldm;
  int m, p, q, kmax, ns;
  int* next;
  int* err;
  int* Rc;
  int* Tc;
  int* Ac;
  int* Rt;
  int* Rr;
  // multi-GPU: dist = world > 1. Rf[k][i][g] (uncached memory) = the epoch of the launch whose
  // owner of panel k forwarded the V/T images of member i, group g into this rank's workspace
  // (set by the peer over xGMI, polled at system scope; never reset: a launch waits for its own
  // epoch). Panel counters Rc/Rr/Rt stay local to the owner. Rf + rf_done: Done[r] = the last
  // epoch rank r's launch completed (every rank writes its own entry into every peer's array at
  // the end of its launch); a panel task forwards into peer r's workspace only once Done[r] has
  // reached epoch - 1 (peer r no longer reads the previous launch's images) — so consecutive
  // launches need no host synchronisation or barrier between the ranks.
  int dist, rank, world, cyclic;  // cyclic: TQR_DIST_PART=cyclic diagnostic partition (j % world)
  const PeerBufs* peers;
  int* Rf;
  int epoch;
  long rf_done;  // offset of Done[] in Rf
  int* exitc;    // workgroups that left the task loop (local, zeroed per launch)
  // host-pointer API (xfer.hpp; all null / 0 on the device API): the launch uploads its input
  // from hsrc and downloads its result to hdst (host memory, leading dimension hld) in chunks of
  // xrows rows, nxc per tile column. hup[j] >= gen: the host staged column j (null: hsrc was
  // ready at launch); hdn[j * nxc + c] = gen: chunk c of column j is in hdst (null: not needed).
  // Uc[j]: upload chunks of column j done. seglen / seglen_la: the plan's chain segment lengths
  // (the download's column-final counts).
  const void* hsrc;
  void* hdst;
  long hld;
  int* hup;
  int* hdn;
  int* Uc;
  int gen, nxc, xrows, seglen, seglen_la, la_tail, tail, tail_sl, ualone;
  // storage of the tile columns: global tile column j is local column j / cdiv of A (and tau
  // column k of panel k local column k / cdiv). Single GPU: cdiv = 1. Multi-GPU: cdiv = world —
  // a rank stores only the tile columns it owns (one per block of `world` consecutive columns,
  // in the snake and the cyclic partition alike), packed in column order.
  int cdiv;
  // fp64 chains of 128- and 256-tiles on the hand-scheduled MFMA stream (chain_asm.hpp); 0: the
  // compiler-scheduled flow_chain (TQR_CHAIN_ASM=0, A/B runs); bits 0-1 the mode (1 whole next strip
  // loaded in the hand-over, 2 late loads), bit 2 UNMQR elements without the zero-row skip, bit 3
  // fp32 storage on flow_chain32 (else flow_chain32_asm)
  int chain_asm;
};

// Multi-GPU owner of tile column j (its panel and all its updates): "snake" order over the ranks
// (0..W-1, W-1..0, 0..W-1, ...), so that every rank's columns sum to the same index total — the
// chain work of a column grows with its index, and the plain cyclic j % W left the last rank 11 %
// more work at 65536x16384 on 8 ranks (tools/sched_sim.py dist: S(8) 5.39 vs 5.20).
// cyclic = 1 (TQR_DIST_PART=cyclic, A/B diagnostics only) restores j % W.
__host__ __device__ inline int tile_owner(int j, int world, int cyclic = 0) {
  const int blk = j / world, r = j - blk * world;
  if (cyclic) return r;
  return (blk & 1) ? world - 1 - r : r;
}

// Segment length of chain (k, j): the last `tail` steps' chains tail_sl elements per segment (their
// elements then pipeline group by group over workgroups instead of running one after the other in
// one: the factorisation's tail is a few short columns per step on the critical path); else the
// lookahead column (j = k+1) may use its own (seglen_la), and the last la_tail steps' lookahead
// column one element per segment (engine.hip FlowKnobs).
__host__ __device__ inline int seglen_of_chain(int k, int j, int kmax, int seglen, int seglen_la, int la_tail,
                                               int tail = 0, int tail_sl = 1) {
  if (k >= kmax - tail) return tail_sl;
  if (j != k + 1) return seglen;
  return k >= kmax - la_tail ? 1 : seglen_la;
}
// The last `ualone` steps' lookahead column (j = k+1) runs its UNMQR element alone in segment 0:
// the element that finishes the next diagonal tile, TSMQR(k+1, k+1, k), then starts segment 1,
// pipelined group by group behind the UNMQR (Ac) instead of running after it in the same task.
__host__ __device__ inline bool unmqr_alone(int k, int j, int kmax, int ualone) { return j == k + 1 && k >= kmax - ualone; }
// segments of chain (k, j) with segment length sl: rows k+1 .. p-1 in runs of sl, after the
// UNMQR-only segment when unmqr_alone; the segment holding row i > k
__host__ __device__ inline int nseg_of_chain(int k, int j, int p, int kmax, int sl, int ualone) {
  const int rows = p - k - 1;
  if (rows <= 0) return 1;
  return (rows + sl - 1) / sl + (unmqr_alone(k, j, kmax, ualone) ? 1 : 0);
}
__host__ __device__ inline int seg_of_row(int k, int j, int i, int kmax, int sl, int ualone) {
  return (i - k - 1) / sl + (unmqr_alone(k, j, kmax, ualone) ? 1 : 0);
}

// ---- synchronisation ---------------------------------------------------------------------
// Counter accesses go through global (address-space 1) pointers: a generic pointer makes them
// FLAT instructions, which also count on the LDS counter (lgkmcnt) and return out of order with
// LDS reads — one such poll in flight turned every operand wait of the MFMA stream that
// followed into lgkmcnt(0).
typedef __attribute__((address_space(1))) int gint;
__device__ __forceinline__ gint* gptr(int* p) { return (gint*)p; }
__device__ __forceinline__ int ld_relaxed(int* p) {
  return __hip_atomic_load(gptr(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int ld_sys(int* p) { return __hip_atomic_load(gptr(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }
__device__ __forceinline__ int ld_cnt(int* p, bool sys) { return sys ? ld_sys(p) : ld_relaxed(p); }

// Wave-uniform copies (SGPRs): arguments of a device function arrive in VGPRs, and without a
// readfirstlane the compiler keeps every value derived from them per lane.
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ size_t uni64(size_t v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return ((size_t)hi << 32) | lo;
}
template <typename T>
__device__ __forceinline__ T* uni(T* p) {
  const unsigned long long u = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return (T*)(((unsigned long long)hi << 32) | lo);
}

// thread 0 only: spin until *p >= target; false on error / timeout. sys: the counter is written
// by other devices (system-scope polls). spin_ge_i: the same inlined — the chains' group loops
// use it, because a call there made the register allocator keep the poll thread's pointers and
// prefetched counters in scratch (each reload behind an s_waitcnt vmcnt(0), i.e. a full drain of
// the poll wave's memory operations twice per group).
__device__ __forceinline__ bool spin_ge_i(int* p, int target, int* err, bool sys = false) {
  if (ld_cnt(p, sys) >= target) return true;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int last = 0;
  while (ld_cnt(p, sys) < target) {
    if (ld_relaxed(err)) return false;
    __builtin_amdgcn_s_sleep(8);
    if (timed_out(t0, last, err)) {
      __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}
__device__ __noinline__ bool spin_ge(int* p, int target, int* err, bool sys = false) {
  if (ld_cnt(p, sys) >= target) return true;
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int last = 0;
  while (ld_cnt(p, sys) < target) {
    if (ld_relaxed(err)) return false;
    __builtin_amdgcn_s_sleep(8);
    if (timed_out(t0, last, err)) {
      __hip_atomic_store(err, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}

// Hand-off protocol inside the launch (MI355X_MICROARCH.md, visibility "Valid forms", first
// table row): every handed-off byte is stored sc1 (write-through) and each storing wave drains
// (vmcnt(0)) before a workgroup barrier, after which ONE lane bumps the counter (agent atomic);
// a consumer's thread 0 polls the counter relaxed, a barrier follows, and the other waves read the
// bytes with sc1 loads — no release / acquire fences (each ~1.7 us at one workgroup per CU).
// The chain's LDS-DMA of V/T images reads write-once data (see PanelView) and needs neither.

// The LDS tail words (task word, verdicts, flags, Rc view) reach the task functions as generic
// pointers; accessed through them (volatile ones are never rewritten to LDS) they become flat
// operations, which count in vmcnt as well: the wait for a flat verdict read after a sync point
// was an s_waitcnt vmcnt(0) — a full drain of the wave's memory operations behind every partial
// drain. Every access to those words goes through an LDS-typed pointer (ds_read/ds_write).
typedef __attribute__((address_space(3))) int lds_int_t;
__device__ __forceinline__ lds_int_t* lds_int(int* p) { return (lds_int_t*)p; }
__device__ __forceinline__ int lds_ld_volatile(int* p) { return *(volatile lds_int_t*)lds_int(p); }

// all threads: thread 0's verdict (after its polls)
__device__ __forceinline__ bool wg_verdict(bool ok0, int* sflag) {
  if (threadIdx.x == FLOW_PT) *lds_int(sflag) = ok0 ? 1 : 0;
  __syncthreads();
  const bool ok = lds_ld_volatile(sflag) != 0;
  __syncthreads();
  return ok;
}

// all threads: every wave's (sc1) stores drained, then thread 0 bumps the counter (system
// scope when the counter is also polled by peers' ... / lives in uncached memory)
__device__ __forceinline__ void wg_publish(int* p, int delta, bool sys = false) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (sys) __hip_atomic_fetch_add(gptr(p), delta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else __hip_atomic_fetch_add(gptr(p), delta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// workspace slot sizes (doubles) of one reflector group's images in a shape: fp64 storage = the
// fp64 chain's V image + packed T at the shape's group size; fp32 storage = the fp32 chain's
// images (tiles.hpp Img, 32-reflector groups)
template <int B, typename S, class C>
struct FImg {
  static constexpr int V = sizeof(S) == 8 ? FGeo<B, C>::VIMG : Img<B, S>::V;
  static constexpr int T = sizeof(S) == 8 ? FGeo<B, C>::TPIMG : Img<B, S>::T;
};
// The same for a counter whose adds must stay in member order: thread 0 first waits until the
// `before` earlier members have added (no-op for the first), then adds. Rc (images of a panel
// member out) needs it: the next member's images need only this member's factorisation (Rr), so
// on a CU shared with another workgroup (ShapeW4) a member can finish its images before its
// predecessor — and a chain waiting for Rc >= i-k+1 would then read member i's images unwritten.
__device__ __forceinline__ void wg_publish_ordered(int* p, int before, int* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && (before == 0 || spin_ge(p, before, err)))
    __hip_atomic_fetch_add(gptr(p), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int B, typename S, class C>
__device__ __forceinline__ size_t flow_vw_off(int p, int i, int k, int g) {
  return ((size_t)(i - k) * FGeo<B, C>::NG + g) * FImg<B, S, C>::V;
}
template <int B, typename S, class C>
__device__ __forceinline__ size_t flow_tw_off(int p, int i, int k, int g) {
  constexpr int NG = FGeo<B, C>::NG;
  return (size_t)(p - k) * NG * FImg<B, S, C>::V + ((size_t)(i - k) * NG + g) * FImg<B, S, C>::T;
}
template <int B, typename S, class C>
__device__ __forceinline__ double* flow_tw(const FlowArgs& a, int i, int k, int g) {
  return a.Wk[k] + flow_tw_off<B, S, C>(a.p, i, k, g);
}
template <int B, typename S, class C>
__device__ __forceinline__ double* flow_vw(const FlowArgs& a, int i, int k, int g) {
  return a.Wk[k] + flow_vw_off<B, S, C>(a.p, i, k, g);
}

// ---- LDS-DMA staging of one reflector group ------------------------------------------------
// The producer (flow_panel) stores every group's V image (row-major, permuted columns, pitch VP,
// GE part made explicit) and T image into the workspaces; a consumer copies both verbatim with
// global_load_lds_dwordx4 (1 KiB per wave-instruction, lane-linear), so the staging costs no
// VGPRs, no ds_write pass and runs under the MFMA phase that follows (CDNA4 LDS-DMA,
// cdna_hip_programming.md §5).
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;
// DMA job of one group for apply_zw's hook: step m issues this wave's m-th LDS-DMA instruction
// (V image instructions first, then T), so the issue cost hides under the MFMA stream.
template <int B, typename S = double, class C = ShapeW8>
struct DmaJob {
  static constexpr int NW = C::NW;
  static constexpr int VIMG = FImg<B, S, C>::V;
  static constexpr int NIV = FImg<B, S, C>::V / 128, NIT = FImg<B, S, C>::T / 128;
  static constexpr int PV = (NIV + NW - 1) / NW, PT = (NIT + NW - 1) / NW;
  static constexpr int STEPS = PV + PT;
  double* dst;
  const double* v;
  const double* t;
  int* sflag;  // activity stamps only
  __device__ __forceinline__ void mid() const { FST(3); }
  // Branch-free: every wave issues exactly STEPS instructions (a wave past the end of an image
  // re-copies its last KiB — identical bytes to the same LDS words), and a job with nothing to
  // fetch is pointed by the caller at an image it may legally re-read into the idle buffer.
  // Control flow inside the MFMA stream made the compiler drop its partial lgkmcnt waits.
  __device__ __forceinline__ void step(int m) const {
    // wave id made provably uniform: addresses = scalar base + one per-lane offset register
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (m < PV) {
      const int u = min(w + NW * m, NIV - 1);
      dma16(v + u * 128 + 2 * lane, dst + u * 128);
    } else if (m < STEPS) {
      const int u = min(w + NW * (m - PV), NIT - 1);
      dma16(t + u * 128 + 2 * lane, dst + VIMG + u * 128);
    }
  }
  // One wave-wide 16-B-per-lane LDS-DMA (1 KiB, lane-linear at lds_wave). Issued as inline asm:
  // for the builtin the compiler cannot tell the DMA's LDS destination (the idle buffer) from the
  // operand reads of the buffer in use, and drains every outstanding ds_read (lgkmcnt(0)) before
  // each DMA, which unpipelines the MFMA stream. Completion is tracked by hand: every consumer
  // sits behind sync_point<true>'s explicit vmcnt(0); the compiler's own vmcnt accounting only
  // over-waits when it does not see these (in-order counter), never under-waits.
  static __device__ __forceinline__ void dma16(const double* src, double* lds_wave) {
    const unsigned l = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_void_t*)lds_wave);
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off sc1" ::"v"(src), "{m0}"(l) : "memory");
  }
};

// All threads: thread 0 has polled its dependencies (verdict ok0, and acquired if it needed
// to). Optionally drain this wave's vector-memory operations (its LDS-DMA landed, loads and
// stores complete), one raw barrier (no implicit vmcnt(0)), then every wave reads the verdict
// from a parity-alternating LDS slot (a slot is rewritten only after the next barrier).
// FLAT: the verdict read as a generic (flat) load — its wait is vmcnt(0), i.e. a full drain, which
// only the fp32 chain still uses (its register allocation spills in the phase loops otherwise;
// every sync point there drains fully anyway).
template <bool DRAIN, bool FLAT = false, int PT = FLOW_PT>
__device__ __forceinline__ bool sync_point(bool ok0, int* sflag, int& par) {
  int* slot = sflag + 40 + par;  // LDS tail (ints from the task word): [task][flag][..][verdicts 41,42][..][Rc view 49.. (fp32) / 261.. (fp64)][..][FST sums 64..]
  par ^= 1;
  if (threadIdx.x == PT) *lds_int(slot) = ok0 ? 1 : 0;
  WST_T0();
  if (DRAIN) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  WST_MID();
  __builtin_amdgcn_s_barrier();
  WST_END();
  asm volatile("" ::: "memory");
  if constexpr (FLAT) return *(volatile int*)slot != 0;
  return lds_ld_volatile(slot) != 0;
}
// A group's sync point inside a segment: only the LDS-DMA of this group (issued in the previous
// group's phase 1) and everything older must have landed; the N youngest operations — the
// previous group's head-row stores and this group's head-row loads, issued after that DMA — may
// still be in flight (the stores are read back by this workgroup only, the loads are waited for
// at their first use).
template <int N, int PT = FLOW_PT>
__device__ __forceinline__ bool sync_point_cnt(bool ok0, int* sflag, int& par) {
  int* slot = sflag + 40 + par;
  par ^= 1;
  if (threadIdx.x == PT) *lds_int(slot) = ok0 ? 1 : 0;
  static_assert(N >= 0 && N < 64, "vmcnt range");
  WST_T0();
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
  WST_MID();
  __builtin_amdgcn_s_barrier();
  WST_END();
  asm volatile("" ::: "memory");
  return lds_ld_volatile(slot) != 0;
}
// The first group's sync point of an element: everything older than the element's own strip and
// head loads (the previous element's stores, this group's LDS-DMA) must be complete, the NX
// loads issued after them need not be — phase 1 waits for each strip row as it reaches it (the
// compiler's vmcnt per use; the LDS-DMA of the next group, issued in between, only makes those
// waits conservative). A wave without loads (strip past the tile) drains fully.
template <int NX, int PT = FLOW_PT>
__device__ __forceinline__ bool sync_point_first(bool ok0, int* sflag, int& par, bool loaded) {
  int* slot = sflag + 40 + par;
  par ^= 1;
  if (threadIdx.x == PT) *lds_int(slot) = ok0 ? 1 : 0;
  static_assert(NX >= 0 && NX < 64, "vmcnt range");
  WST_T0();
  if (loaded) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NX) : "memory");
  else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  WST_MID();
  __builtin_amdgcn_s_barrier();
  WST_END();
  asm volatile("" ::: "memory");
  return lds_ld_volatile(slot) != 0;
}
// thread 0, after a draining sync point (every wave's sc1 stores complete): bump a counter
__device__ __forceinline__ void publish_after_drain(int* p, int delta) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(gptr(p), delta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The poll thread's view of one panel's group counters Rc[k][0..NG): rv[g] (LDS) holds an
// observed value, so the V/T images of any member < rv[g] of group g may be LDS-DMA'd.
// ensure(g, need) re-reads counter g (one round trip) only when rv[g] < need. No acquire fence:
// the images are write-once inside a launch (one producer, stored sc1 and drained before its
// counter add), no workgroup reads a slot before observing its counter, and the DMA itself is
// an sc1 (L1-bypassing) load — so no CU can hold a stale copy of an image line.
// prefetch(g) (the poll thread, right after a sync point) issues the load of the one counter the
// next sync point tests, so that ensure() normally finds a fresh value without an exposed round
// trip. (Round 2 prefetched the whole row into NG registers; in the 256-register budget of the
// fp64 chain the compiler kept them in scratch, and every reload waited behind the poll wave's
// outstanding memory operations. Staging the row into LDS by LDS-DMA: 132.5 ms against
// 130.6-130.9 at 16384^2.)
//
// Round 3: the early load is an LDS-DMA of the one counter word into an LDS slot (lds_prefetch):
// no VGPR holds it and nothing waits for it. In the VGPR form the value was spilled right after
// its load (the store to scratch waited for the load — a full round trip on the poll wave after
// every sync point) and reloaded behind an s_waitcnt vmcnt(0) before the next one.
typedef __attribute__((address_space(3))) void lds_void_t;
// Poll thread only (one active lane): start an asynchronous load of *p into the LDS word slot,
// which reads -1 until it lands. Every chain sync point drains the older memory operations of
// each wave, so a prefetch issued after one sync point has landed by the next one: the slot is
// reset (and re-targeted) only after that, and a late write can never land on a newer prefetch.
template <int PT>
__device__ __forceinline__ void lds_prefetch(int* p, int* slot, bool sys) {
  *lds_int(slot) = -1;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the reset is in LDS before the DMA can write
  // LDS-DMA writes lane-linear (M0 + 4 * lane): aim lane (PT & 63)'s word at the slot
  const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_void_t*)slot - 4u * (PT & 63));
  if (sys) asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, off sc0 sc1" ::"v"(p), "{m0}"(m0) : "memory");
  else asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, off sc1" ::"v"(p), "{m0}"(m0) : "memory");
}
template <int NG, int PT = FLOW_PT>
struct PanelView {
  lds_int_t* rv;
  int* pfs;  // LDS slot of the early load (lds_prefetch)
  int pfg;   // the group whose counter the slot was aimed at (-1: none)
  __device__ __forceinline__ void init(int* lds_words, int* slot) {
    rv = lds_int(lds_words);
    pfs = slot;
    pfg = -1;
    if (threadIdx.x == PT)
      for (int g = 0; g < NG; ++g) rv[g] = 0;
  }
  __device__ __forceinline__ void prefetch(int* rc, int g, bool sys) {
    lds_prefetch<PT>(rc + g, pfs, sys);
    pfg = g;
  }
  __device__ __forceinline__ bool ensure(int* rc, int g, int need, int* err, bool sys) {
    if (rv[g] >= need) return true;
    if (pfg == g) {
      rv[g] = max((int)rv[g], lds_ld_volatile(pfs));  // (-1 while the load is in flight)
      pfg = -1;
      if (rv[g] >= need) return true;
    }
    const int v = ld_cnt(rc + g, sys);
    rv[g] = v;
    if (v < need) {
      if (!spin_ge_i(rc + g, need, err, sys)) return false;
      rv[g] = ld_cnt(rc + g, sys);
    }
    return true;
  }
};
// The group whose counter a chain's next sync point tests, seen from group g's post-sync: group
// g+2 of this element, or of the next element (group 0 at g = NG-2, group 1 at g = NG-1: the next
// element's first sync point tests its group 1, its group 0 having been checked before its DMA).
template <int NG>
__device__ __forceinline__ int next_test_group(int g) {
  return g + 2 < NG ? g + 2 : (g + 2 == NG || NG == 1 ? 0 : 1);
}

// Two consecutive elements (a row pair of a column) as one sc1 buffer access: 16 B for fp64,
// 8 B for fp32 storage.
template <typename S, int AUX = 16>
__device__ __forceinline__ void ld_pair(__amdgpu_buffer_rsrc_t rs, unsigned off, double& a, double& b) {
  if constexpr (sizeof(S) == 8) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX);
    a = __longlong_as_double((long long)(((unsigned long long)v[1] << 32) | v[0]));
    b = __longlong_as_double((long long)(((unsigned long long)v[3] << 32) | v[2]));
  } else {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, AUX);
    a = (double)__uint_as_float(v[0]);
    b = (double)__uint_as_float(v[1]);
  }
}
template <typename S, int AUX = 16>
__device__ __forceinline__ void st_pair(__amdgpu_buffer_rsrc_t rs, unsigned off, double a, double b) {
  if constexpr (sizeof(S) == 8) {
    const unsigned long long ua = (unsigned long long)__double_as_longlong(a);
    const unsigned long long ub = (unsigned long long)__double_as_longlong(b);
    __attribute__((ext_vector_type(4))) unsigned v = {(unsigned)ua, (unsigned)(ua >> 32), (unsigned)ub, (unsigned)(ub >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, AUX);
  } else {
    __attribute__((ext_vector_type(2))) unsigned v = {__float_as_uint((float)a), __float_as_uint((float)b)};
    __builtin_amdgcn_raw_buffer_store_b64(v, rs, off, 0, AUX);
  }
}

// the fp32 chain's operand images of one group (chain32.hpp), optionally also into LDS
template <int B>
__device__ __noinline__ void write_images32(const double* Vs, const double* Ts, __amdgpu_buffer_rsrc_t rv,
                                            __amdgpu_buffer_rsrc_t rt, float* lvr = nullptr, float* ltp = nullptr);
// fp32 storage: a panel group's in-tile trailing update on the fp32 MFMA (chain32.hpp)
template <int B>
__device__ __noinline__ void panel_trail32(float* Bt, float* Rt, size_t ldm, bool qrs, int g, int c0, int nstr,
                                           const float* VRl, int nw);

// Multi-GPU: the panel task itself copies each group's V and T images from its workspace slot
// into every peer's (16-B system-scope stores over xGMI), right after the group's Rc publish;
// its next publish (Rt, after the in-tile trailing update) drains them, then thread 0 releases at
// system scope and sets the peers' member flags Rf[k][i][g]. (Round 2 had a separate forward
// task per member, dequeued right behind it: it held a workgroup while waiting for the member's
// groups — 5.4 % of workgroup time in the 2-rank rehearsal, 682 vs 667 ms for this form.)
template <int B, typename S, class C>
__device__ __forceinline__ void fwd_images(const FlowArgs& a, int k, size_t vo, size_t to) {
  const __amdgpu_buffer_rsrc_t vsrc = uniform_rsrc(a.Wk[k] + vo), tsrc = uniform_rsrc(a.Wk[k] + to);
  for (int r = 0; r < a.world; ++r) {
    if (r == a.rank) continue;
    double* pw = a.peers[r].Wk[k];
    const __amdgpu_buffer_rsrc_t vdst = uniform_rsrc(pw + vo), tdst = uniform_rsrc(pw + to);
#pragma unroll 4
    for (int c = threadIdx.x; c < FImg<B, S, C>::V / 2; c += blockDim.x)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_amdgcn_raw_buffer_load_b128(vsrc, 16 * c, 0, 16), vdst, 16 * c, 0, 17);
    for (int c = threadIdx.x; c < FImg<B, S, C>::T / 2; c += blockDim.x)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_amdgcn_raw_buffer_load_b128(tsrc, 16 * c, 0, 16), tdst, 16 * c, 0, 17);
  }
}

// Multi-GPU, off the member-to-member path: reflector group g-1's images are forwarded by the
// four waves that hold no panel rows (waves 4-7) while waves 0-3 factorise group g (panel_factor),
// one slice per reflector step — each lane loads its 16-B unit of the next slice while it stores
// the current one to every peer — and the last of those waves to drain its stores sets the peers'
// member flags of group g-1 (release, system scope). Before (round 2) all 512 threads copied the
// images between group g's Rc publish and its in-tile trailing update, on the path the next member's
// trailing waits for. The last group is still forwarded that way (no next factorisation).
struct FwdJob {
  const FlowArgs* a;
  int k;
  size_t vo, to;  // the group's V / T image offsets in workspace k (doubles)
  size_t fo;      // its member flag index in Rf: (k * p + i) * NG + g
  int nv, nt;     // 16-B units of the V and T images
  int* cnt;       // LDS arrival counter of the forwarding waves (0 between uses)
};

__device__ __noinline__ void panel_idle(const FwdJob* fjp, int IB, bool TS) {
  const FwdJob fj = *fjp;
  const FlowArgs& a = *fj.a;
  const int tid = threadIdx.x - 256, lane = threadIdx.x & 63;
  const int nu = fj.nv + fj.nt, per = (nu + IB - 1) / IB;  // units per reflector step
  // lane r holds peer r's workspace k and flag array (read once; v_readlane per use)
  unsigned long long pw = 0, pf = 0;
  if (lane < a.world) {
    pw = (unsigned long long)a.peers[lane].Wk[fj.k];
    pf = (unsigned long long)a.peers[lane].Rf;
  }
  // one resource per workspace (its base is wave-uniform), per-lane byte offsets: a wave's units
  // may straddle the V / T boundary (a workspace is < 2 GiB, the IPC export bound)
  const __amdgpu_buffer_rsrc_t sw = uniform_rsrc(a.Wk[fj.k]);
  auto unit_off = [&](int u) -> unsigned {
    return u < fj.nv ? (unsigned)(fj.vo * 8 + 16 * (size_t)u) : (unsigned)(fj.to * 8 + 16 * (size_t)(u - fj.nv));
  };
  typedef __attribute__((ext_vector_type(4))) unsigned v4u;
  auto unit_ld = [&](int u) -> v4u { return __builtin_amdgcn_raw_buffer_load_b128(sw, unit_off(u), 0, 16); };
  auto peer = [&](unsigned long long v, int r) {
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)v, r), hi = __builtin_amdgcn_readlane((unsigned)(v >> 32), r);
    return (char*)(((unsigned long long)hi << 32) | lo);
  };
  v4u cur = {0, 0, 0, 0}, nxt = {0, 0, 0, 0};
  if (tid < per && tid < nu) cur = unit_ld(tid);
  for (int C = 0; C < IB; ++C) {
    const int un = (C + 1) * per + tid, uc = C * per + tid;
    if (C + 1 < IB && tid < per && un < nu) nxt = unit_ld(un);
    if (tid < per && uc < nu) {
      const unsigned off = unit_off(uc);
      for (int r = 0; r < a.world; ++r)
        if (r != a.rank) __builtin_amdgcn_raw_buffer_store_b128(cur, uniform_rsrc(peer(pw, r)), off, 0, 17);
    }
    __syncthreads();
    cur = nxt;
  }
  __syncthreads();
  if (TS) __syncthreads();
  // every forwarding wave drains its own stores, then counts itself in; the last one signals
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(lds_int(fj.cnt), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  old = __shfl(old, 0);
  if (old == 3 && lane == 0) {
    *lds_int(fj.cnt) = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int r = 0; r < a.world; ++r)
      if (r != a.rank)
        __hip_atomic_store((int*)peer(pf, r) + fj.fo, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- panel tasks ---------------------------------------------------------------------------
// LDS of a panel task (doubles): V block Vs, head / T / Gram images Hs Ts Gs, tau, then the
// factorisation's scratch and build_t's partial Grams Gp (flow_panel). fp32 storage keeps the
// group's fp32 chain images (Geo32 VR floats, then the packed -T chunks) for its in-tile trailing
// update in that scratch + Gp region, dead by then (flow_panel_img32_at)
template <int B, class C>
constexpr int flow_panel_doubles() {
  using G = FGeo<B, C>;
  return G::VSZ + 8 * G::TSZ + G::IB + 2 + 2 * 4 * 32 + 4 * 32 + 2 * 32;
}
template <int B, class C>
constexpr int flow_panel_img32_at() {
  using G = FGeo<B, C>;
  constexpr int at = G::VSZ + 3 * G::TSZ + G::IB + 2;  // = scratch
  static_assert(at + Geo32<B>::VR / 2 + Geo32<B>::TIMG <= flow_panel_doubles<B, C>(), "fp32 images in the panel's LDS");
  return at;
}
template <int B, typename S, class C>
__device__ __noinline__ void flow_panel(const FlowArgs& a, int type, int l, int k, double* lds, int* sflag) {
  using G = FGeo<B, C>;
  constexpr int NT = C::NT;
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
  // tile column k and tau column k in this rank's storage (FlowArgs::cdiv)
  const int kl = k / a.cdiv;
  S* Rt = A + (size_t)kl * B * ldm + (size_t)k * B;
  const bool qrs = type == QRS;
  S* Bt = qrs ? Rt : A + (size_t)kl * B * ldm + (size_t)l * B;
  const int pos = qrs ? 0 : l - k;  // position in the panel chain
  FST(6);
  // the tile(s) must have received step k-1 on every strip (step 0, host-pointer API: tile
  // column 0 uploaded, xfer.hpp)
  {
    bool ok = true;
    if (t == FLOW_PT && k == 0 && a.Uc) ok = spin_ge(&a.Uc[0], a.nxc, a.err);
    if (t == FLOW_PT && k > 0)
      for (int s = 0; s < a.ns && ok; ++s) ok = spin_ge(&a.Tc[((size_t)(qrs ? k : l) * a.q + k) * a.ns + s], k, a.err);
    if (!wg_verdict(ok, sflag)) return;
  }
  FST(1);
  double X[G::NKS];
  double H[G::NRI];
  const int me = qrs ? k : l;
  if (a.dist && t == 0) *lds_int(sflag + 36) = 0;  // the forwarding waves' arrival counter
  if (a.dist) {  // every peer has finished the previous launch (it reads no more of its images)
    bool ok = true;
    if (t == FLOW_PT)
      for (int r = 0; r < a.world && ok; ++r)
        if (r != a.rank) ok = spin_ge(a.Rf + a.rf_done + r, a.epoch - 1, a.err, true);
    if (!wg_verdict(ok, sflag)) return;
  }
  for (int g = 0; g < NG; ++g) {
    const int c0 = g * IB;
#ifdef TQR_PANEL_LOAD_LATE  // (A/B: the block loaded after the previous member's Rr)
    if (!qrs) {  // R_kk rows of group g as left by the previous chain member
      FST(10);
      const bool ok = t == FLOW_PT ? spin_ge(&a.Rr[(size_t)k * NG + g], pos, a.err) : true;
      if (!wg_verdict(ok, sflag)) return;
      FST(1);
    }
#endif
    // the member's own block first: its columns depend on this member's own trailing update only,
    // so its load overlaps the wait for the previous member's R rows of the group (Rr, below)
    {  // the group's B x IB block, row pairs as 16-B sc1 buffer loads (GEQRT: rows above c0 zero)
      const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(Bt + (size_t)c0 * ldm);  // offsets span IB columns
      const int rlo = qrs ? c0 : 0;
#pragma unroll 4
      for (int idx = t; idx < B * IB / 2; idx += NT) {
        const int r = 2 * (idx % (B / 2)), c = idx / (B / 2);
        double v0 = 0.0, v1 = 0.0;
        if (r >= rlo) ld_pair<S>(rs, (unsigned)(((size_t)c * ldm + r) * sizeof(S)), v0, v1);
        Vs[vimg_inv(r) * VP + G::pc(c)] = v0;
        Vs[vimg_inv(r + 1) * VP + G::pc(c)] = v1;
      }
    }
#ifndef TQR_PANEL_LOAD_LATE
    if (!qrs) {  // R_kk rows of group g as left by the previous chain member
      FST(10);
      const bool ok = t == FLOW_PT ? spin_ge(&a.Rr[(size_t)k * NG + g], pos, a.err) : true;
      if (!wg_verdict(ok, sflag)) return;
      FST(1);
    }
#endif
    if (!qrs) {
      for (int idx = t; idx < IB * IB; idx += NT) {
        const int r = idx % IB, c = idx / IB;
        if (r <= c) Hs[r * TP + c] = ldc(Rt + (size_t)(c0 + c) * ldm + c0 + r);
      }
    }
    __syncthreads();
    FST(10);
    // Vs holds the panel rows in the chains' paired order (LDS row q = tile row vimg_row(q)): the
    // V image is then a verbatim copy and the trailing update moves 16-B row pairs
    // multi-GPU: waves 4-7 forward group g-1's images meanwhile (FwdJob)
    // (ShapeW4 has no idle waves: every group is forwarded inline, below)
    const FwdJob fj{&a, k, flow_vw_off<B, S, C>(a.p, me, k, g - 1), flow_tw_off<B, S, C>(a.p, me, k, g - 1),
                    ((size_t)k * a.p + me) * NG + g - 1, FImg<B, S, C>::V / 2, FImg<B, S, C>::T / 2, sflag + 36};
    const FwdJob* fjp = a.dist && g > 0 && NT > 256 ? &fj : nullptr;
#ifndef TQR_DIAG_NOPFACT  // what-if: no panel factorisation (results wrong)
    if (qrs) panel_factor<B, false, true, IB>(Vs, Hs, tauv, scratch, c0, fjp);
    else panel_factor<B, true, true, IB>(Vs, Hs, tauv, scratch, c0, fjp);
#endif
    FST(5);
    {  // write-back of the factored block (R / V), row pairs as 16-B write-through stores
      const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(Bt + (size_t)c0 * ldm);
      const int rlo = qrs ? c0 : 0;
#pragma unroll 4
      for (int idx = t; idx < B * IB / 2; idx += NT) {
        const int r = 2 * (idx % (B / 2)), c = idx / (B / 2);
        if (r >= rlo)
          st_pair<S>(rs, (unsigned)(((size_t)c * ldm + r) * sizeof(S)), Vs[vimg_inv(r) * VP + G::pc(c)],
                     Vs[vimg_inv(r + 1) * VP + G::pc(c)]);
      }
    }
    if (!qrs) {
      for (int idx = t; idx < IB * IB; idx += NT) {
        const int r = idx % IB, c = idx / IB;
        if (r <= c) st(Rt + (size_t)(c0 + c) * ldm + c0 + r, Hs[r * TP + c]);
      }
    }
    if (t < IB) st(tau + (size_t)kl * a.m + (size_t)(qrs ? k : l) * B + c0 + t, tauv[t]);
    wg_publish(&a.Rr[(size_t)k * NG + g], 1);  // includes the drain and the barrier
    if (qrs) {
      for (int idx = t; idx < B * IB; idx += NT) {
        const int r = idx % B, c = idx / B, d = c0 + c;
        if (r <= d) Vs[vimg_inv(r) * VP + G::pc(c)] = r == d ? 1.0 : 0.0;
      }
      __syncthreads();
    }
    FST(10);
#ifndef TQR_DIAG_NOBT  // what-if: no T formation (results wrong)
#ifdef TQR_DIAG_GEFAST  // what-if: GEQRT without T formation and in-tile trailing update (results wrong)
    if (!qrs)
#endif
    build_t<B, IB>(Vs, tauv, Gs, Ts, Gp, 0);  // (permuted rows: the GE zero rows are not a prefix)
#endif
    // packed T (the Gram buffer is free now): the trailing update's and the chains' T operand
    double* Tp = Gs;
    pack_t<B, NT, IB>(Ts, Tp);
    __syncthreads();
    FST(11);
    {  // V image (explicit) and packed T image of this group for the chains (LDS-DMA sources)
      double* tg = flow_tw<B, S, C>(a, qrs ? k : l, k, g);
      double* vg = flow_vw<B, S, C>(a, qrs ? k : l, k, g);
      const __amdgpu_buffer_rsrc_t rv = uniform_rsrc(vg), rt = uniform_rsrc(tg);
      if constexpr (sizeof(S) == 8) {
        // the chain's images in the paired reflector order (tiles.hpp sigp): V image position
        // x * NRI + r of a row holds reflector sigp(r, x); packed -T over k-blocks kb >= (wi & ~1)
        constexpr int NRI = G::NRI;
        auto tpk = [&](int e) -> double {
          const int wi = e % NRI, y = (e / NRI) & 3, x = (e / (4 * NRI)) & 3, kb = e / (16 * NRI);
          return e < G::TPK && (kb & ~1) <= wi ? -Ts[sigp(kb, x) * TP + sigp(wi, y)] : 0.0;
        };
        auto vim = [&](int e) -> double {
          const int row = e / VP, pos = e % VP;
          return pos < IB ? Vs[row * VP + G::pc(sigp(pos % NRI, pos / NRI))] : 0.0;
        };
        for (int idx = t; idx < G::TPIMG / 2; idx += NT) st_pair<double>(rt, 16 * idx, tpk(2 * idx), tpk(2 * idx + 1));
        for (int idx = t; idx < G::VSZ / 2; idx += NT) st_pair<double>(rv, 16 * idx, vim(2 * idx), vim(2 * idx + 1));
      } else {
        // the fp32 chain's operand images (chain32.hpp), kept in LDS for this group's trailing update
        write_images32<B>(Vs, Ts, rv, rt, (float*)(lds + flow_panel_img32_at<B, C>()),
                          (float*)(lds + flow_panel_img32_at<B, C>() + Geo32<B>::VR / 2));
      }
    }
    // group factorised: R diagonal block, V, tau, images out -> next member and the chains go
    // (in member order: a chain reads member i's images once Rc counts i - k + 1 members)
    wg_publish_ordered(&a.Rc[(size_t)k * NG + g], pos, a.err);
    FST(10);
    // multi-GPU, last group (every group in ShapeW4): the images to every peer now (drained by the
    // Rt publish below, flags after it); earlier groups go during the next group's factorisation
    // (FwdJob, waves 4-7 of ShapeW8)
    const bool fwd_inline = a.dist && (g + 1 == NG || NT <= 256);
    if (fwd_inline) fwd_images<B, S, C>(a, k, flow_vw_off<B, S, C>(a.p, me, k, g), flow_tw_off<B, S, C>(a.p, me, k, g));
    FST(23);
    if (!qrs) {  // R_kk head rows right of the group as left by the previous member's trailing
      const bool ok = t == FLOW_PT ? spin_ge(&a.Rt[(size_t)k * NG + g], pos, a.err) : true;
      if (!wg_verdict(ok, sflag)) return;
      FST(1);
    }
    const int nstr = (B - c0 - IB) / 16;
    // One code path for both panel types (16-B paired-row sc1 strip accesses; head rows through
    // a buffer resource): GEQRT's explicit V (zeros above the unit diagonal) under the TSQRT
    // stream with a zero head is exactly the GE update; its 8-row blocks above the group are
    // neither loaded nor stored (finished R rows, which the next member's trailing may be
    // updating meanwhile); the head resource is empty for GEQRT (loads 0, stores dropped) —
    // see flow_chain's UNMQR element.
    const int h0 = qrs ? c0 / 8 : 0;
#ifndef TQR_PANEL_TRAIL64_F32  // (A/B: fp32 storage's trailing update in fp64 on the 4x4x4 MFMA, as until round 5)
    constexpr bool trail32 = sizeof(S) == 4 && C::NW == 8;
#else
    constexpr bool trail32 = false;
#endif
    if constexpr (trail32) {
      // fp32 storage: the in-tile trailing update in fp32 on the fp32 MFMA (chain32.hpp panel_trail32)
      __syncthreads();  // (every wave's LDS image writes)
      panel_trail32<B>((float*)Bt, (float*)Rt, ldm, qrs, g, c0, nstr,
                       (const float*)(lds + flow_panel_img32_at<B, C>()), C::NW);
    }
#ifdef TQR_DIAG_NOPTRAIL  // what-if: no in-tile trailing update (results wrong)
    for (int s = nstr; s < nstr; s += C::NW) {
#elif defined(TQR_DIAG_GEFAST)
    for (int s = qrs ? nstr : w; s < nstr; s += C::NW) {
#else
    for (int s = trail32 ? nstr : w; s < nstr; s += C::NW) {
#endif
      asm volatile("" ::: "memory");
      const int col = c0 + IB + 16 * s;
      const __amdgpu_buffer_rsrc_t rsH = head_rsrc(Rt + (size_t)col * ldm, !qrs);
      const unsigned so = head_off<B, S>(ldm, c0);  // head row c0 + x, column col + lane's
      load_strip_pair<B, S>(X, Bt, ldm, col, h0);
      load_head_buf<B, S, 16, IB>(H, rsH, so);
#ifdef TQR_FLOW_STAMPS
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
      FST(16);
      // (a GE form over the k-steps from c0 / 4 only, fp64 storage, measured 119.8-120.2 vs
      // 119.2-119.7 ms: not kept, profiles/r05/gepanel)
      apply_group<B, true, FLOW_PF, true, IB>(Vs, Tp, X, H, 0);
      FST(12);
#ifndef TQR_PANEL_STRIP_PLAIN  // (A/B: the MFMA-layout stores)
      if constexpr (sizeof(S) == 8) store_strip_coal<B>(X, (double*)Bt, ldm, col, h0);
      else
#endif
        store_strip_pair<B, S>(X, Bt, ldm, col, h0);
      store_head_buf<B, S, 16, IB>(H, rsH, so);
      FST(17);
    }
    wg_publish(&a.Rt[(size_t)k * NG + g], 1);
    FST(12);
    if (fwd_inline && t == 0) {  // every wave's peer stores drained (the Rt publish): release, flags
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const size_t fo = ((size_t)k * a.p + me) * NG + g;
      for (int r = 0; r < a.world; ++r)
        if (r != a.rank) __hip_atomic_store(&a.peers[r].Rf[fo], a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    FST(23);
  }
}

// ---- chain tasks ---------------------------------------------------------------------------
// MFMA-issue fairness between the two waves of a SIMD (waves w and w + 4): the issue arbiter
// favours the older wave, which then finished its group's MFMAs early and sat at the group's
// barrier while its partner ran alone, every dependency and LDS bubble of a single wave exposed
// (stamps: waves 1-3 waited 44 ms per workgroup at the barriers, waves 5-7 11 ms). Phase 1
// favours the upper waves, phase 2 the lower ones, so the pair ends its group together.
template <class C>
__device__ __forceinline__ void phase_prio(bool phase2) {
  if constexpr (C::NW < 8) return;  // ShapeW4: the SIMD's other wave belongs to another workgroup
#ifndef TQR_NO_PRIO
  const bool upper = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 4;
  if (upper != phase2) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
#endif
}

// Element hand-over inside the last group's phase 2 (apply_x post hook): once row pair h-1 of the
// strip is final, it is stored (write-through), and the registers of pair h-3 — stored two pairs
// earlier — start loading pair h-3 of the next element's strip: the strip's 512 B per lane out and
// in ride the MFMA stream instead of sitting between two elements (what-if without strip I/O:
// -19 ms at 16384^2). Reloading a pair's registers right behind its own store (round 2) made
// every load wait for that store to have read its data: the group carrying the hand-over took
// 40.5 instead of 17.7 us, against 24.2 / 22.4 with the stores / the loads alone (what-if builds,
// tools/group_trace.py).
template <int B, typename S>
struct XPipe {
#ifndef TQR_XP_LAG
#define TQR_XP_LAG 2
#endif
  static constexpr int NP = Geo<B>::NKS / 2;  // row pairs
  static constexpr int LAG = TQR_XP_LAG < NP ? TQR_XP_LAG : NP - 1;  // loads trail stores by LAG pairs
  __amdgpu_buffer_rsrc_t out, in;  // this element's strip / the next element's (same columns)
  unsigned base;
#ifdef TQR_FLOW_STAMPS
  unsigned long long* tr;  // (stamps build) progress marks of this phase 2: pairs 0, 8, 16, 24, end
  __device__ __forceinline__ void mark(int q) const {
    if (tr && (threadIdx.x & 63) == 0) tr[q] = __builtin_amdgcn_s_memrealtime();
  }
#else
  __device__ __forceinline__ void mark(int) const {}
#endif
  __device__ __forceinline__ void st(int h, double (&X)[Geo<B>::NKS]) const {
#ifndef TQR_DIAG_XP_NOSTORE  // what-if builds (results wrong): the hand-over without its stores / loads
    st_pair<S, TQR_STRIP_ST_AUX>(out, base + 8 * h * sizeof(S), X[2 * h], X[2 * h + 1]);
#endif
  }
  __device__ __forceinline__ void ld(int h, double (&X)[Geo<B>::NKS]) const {
#ifndef TQR_DIAG_XP_NOLOAD
    ld_pair<S, TQR_STRIP_LD_AUX>(in, base + 8 * h * sizeof(S), X[2 * h], X[2 * h + 1]);
#endif
  }
  __device__ __forceinline__ void at(int h, double (&X)[Geo<B>::NKS]) const {
    if (h % 8 == 0) mark(h / 8);
    if (h >= 1) st(h - 1, X);  // pair h-1 retired one k-step pair ago
    if (h >= 1 + LAG) ld(h - 1 - LAG, X);
  }
  __device__ __forceinline__ void fin(double (&X)[Geo<B>::NKS]) const {
    mark(4);
    st(NP - 1, X);
#pragma unroll
    for (int h = NP - 1 - LAG; h < NP; ++h)
      if (h >= 0) ld(h, X);
  }
};

// Elements: UNMQR(k,j) (segment 0 only, GE-type, the strip of tile (k,j) is X) and TSMQR(i,j,k)
// for i in [i0,i1) (TS-type: X = strip of tile (i,j), head rows = strip of tile (k,j), group by
// group, prefetched one group ahead into registers). Per reflector group g, in every wave:
//   sync point (drain: DMA(g) landed, loads/stores done; thread 0 made sure the images of the
//   next DMA are published and covered by an acquire)
//   phase 1: Z, W, H (apply_zw); store H(g), load H(g+1)
//   phase 2: X += V W (apply_x), with DMA(g+1) (or group 0 of the next element) issued inside
//   its MFMA stream into the other LDS buffer.
// The tile-strip counter Tc of an element is published after the next element's first drain
// (its stores are complete by then), so no wave waits for its own stores to land.
template <int B, typename S, class C>
__device__ __noinline__ void flow_chain(const FlowArgs& a, int s_, int i0_, int i1_, int j_, int k_, int seg_,
                                        double* lds, int* sflag) {
  const int s = uni(s_), i0 = uni(i0_), i1 = uni(i1_), j = uni(j_), k = uni(k_), seg = uni(seg_);
  using G = FGeo<B, C>;
  constexpr int IB = G::IB, NG = G::NG, BUF = G::VIMG + G::TPIMG;
  constexpr int SW = C::SW;
  using Dma = DmaJob<B, S, C>;
  // (uniform: per-lane copies were spilled, and their reload at every element start waited for
  // vmcnt(0) — behind the previous element's whole strip hand-over)
  S* A = uni((S*)a.A);
  const size_t ldm = uni64(a.ldm);
  const int t = threadIdx.x, w = t >> 6;
  constexpr int PT = chain_pt<C>();
  constexpr int HPACK = 2;  // head rows per lane and access (16-B paired head rows, tiles.hpp sigp)
  const int col = s * SW + 16 * w;  // this wave's 16 columns inside the tile
  // byte-free element offset of the wave's first column, made uniform: as a per-lane product the
  // strip / head base pointers derived from it were VGPR pairs, spilled, and reloaded at every
  // element start behind an s_waitcnt vmcnt(0) (a full drain of the previous hand-over)
  const size_t colo = uni64((size_t)col * ldm);
  const bool active = B % SW == 0 || col < B;  // (compile-time true unless B < SW)
  // tile column j in this rank's storage (FlowArgs::cdiv)
  S* const Aj = uni(A + (size_t)(j / uni(a.cdiv)) * B * ldm);
  S* At = Aj + (size_t)k * B;  // tile (k,j): the chain's head rows
  // everything the group loop needs from FlowArgs, read once per task: the asm memory clobbers
  // of the sync points would otherwise force a reload per group — for Wk[k] a global load whose
  // latency sat in front of the group's first LDS-DMA
  double* const wk = uni(a.Wk[k]);
  const int P = uni(a.p), Q = uni(a.q), NS = uni(a.ns);
  int* const err = uni(a.err);
  int* const Tc = uni(a.Tc);
  auto vimg = [&](int i_, int g_) { return wk + flow_vw_off<B, S, C>(P, i_, k, g_); };
  auto timg = [&](int i_, int g_) { return wk + flow_tw_off<B, S, C>(P, i_, k, g_); };
  int* const rc = uni(&a.Rc[(size_t)k * NG]);
  int* const acg = uni(&a.Ac[(((size_t)k * Q + j) * NS + s) * NG]);  // per head-row group
  auto tc = [&](int i) { return &Tc[((size_t)i * Q + j) * NS + s]; };
  double X[G::NKS];
  double H[G::NRI], W[G::NRI];
  int buf = 0, par = 0;
  int* pending = nullptr;
  bool dma_next = false;  // group 0 of the next element already in flight
  // poll thread's early loads, LDS-DMA'd into LDS slots (lds_prefetch): the Rc counter the next
  // sync point tests (sflag[57]), the Tc of the next element's tile, loaded two groups ahead
  // (sflag[58]; -1: none), the member flag of a remote panel (sflag[59])
  PanelView<NG, PT> pv;
  // (the Rc view holds NG words: up to 16 at 16-reflector groups, past the stamps' LDS words)
  static_assert(NG <= 16, "LDS tail: Rc view of at most 16 groups");
  pv.init(sflag + 260, sflag + 57);
  int* const tcs = sflag + 58;
  int* const fls = sflag + 59;
  int* const acs = sflag + 60;  // Ac[g+1] of a later segment's first element, loaded a group ahead
  if (t == PT) {
    *lds_int(tcs) = -1;
    *lds_int(fls) = -1;
  }
  bool xin = false;  // this element's strip was loaded during the previous element's last phase 2
  // multi-GPU, panel owned by another rank: per-member flags forwarded by the owner
  const bool remote = a.dist && tile_owner(k, a.world, a.cyclic) != a.rank;
  int* const rf = uni(a.Rf + (size_t)k * P * NG);
  const int ep = uni(a.epoch);
  int fl_pf = -1;  // poll thread: index (i * NG + g) of the flag the early load in fls is of
  auto ready = [&](int i_, int g_) -> bool {
    if (!remote) return pv.ensure(rc, g_, i_ - k + 1, err, false);
    const int fi = i_ * NG + g_;
    if (fi == fl_pf && lds_ld_volatile(fls) >= ep) return true;
    return spin_ge_i(rf + fi, ep, err, true);
  };
  FST(6);
  if (k == 0 && a.Uc) {  // host-pointer API: tile column j uploaded (xfer.hpp)
    const bool ok = t == FLOW_PT ? spin_ge(&a.Uc[j], a.nxc, err) : true;
    if (!wg_verdict(ok, sflag)) return;
  }
  const int ifirst = seg == 0 ? k : i0;
  for (int i = ifirst; i < i1 || i == k; i = (i == k ? i0 : i + 1)) {
    const bool ts = i != k;
    {
      bool ok = true;
      if (t == PT) {
        if (i == ifirst && seg > 0) ok = spin_ge(&acg[0], seg, err);
        FST(9);
        // (the early load of Tc has landed: a sync point lies between its issue and here)
        if (ok && k > 0 && lds_ld_volatile(tcs) < k) ok = spin_ge(tc(i), k, err);
        *lds_int(tcs) = -1;
        FST(8);
        if (ok && !dma_next) ok = ready(i, 0);
      }
      FST(j == k + 1 ? 18 : 19);  // Rc wait at element start (lookahead column / other)
      if (!sync_point<false, false, PT>(ok, sflag, par)) return;
    }
    FST(7);
    S* Xt = ts ? Aj + (size_t)i * B : At;
    if (!dma_next) {  // (first: the strip and head loads must be the youngest, see sync_point_first)
      Dma d{lds + buf * BUF, vimg(i, 0), timg(i, 0), sflag};
      for (int m = 0; m < Dma::STEPS; ++m) d.step(m);
    }
    dma_next = false;
    // head rows: written by another workgroup before this segment or by this one (sc1 loads
    // for both). The UNMQR element (i == k, GE-type V) runs the very same TSMQR code with a zero
    // head: its V image is explicit (zeros above the unit diagonal), so Z = 0 + V^T X and X += V W
    // are exactly the GE update (the zero rows add exact zeros) — one MFMA stream for both
    // element types keeps the register allocation of the hot TSMQR path clean (a separate GE
    // variant with ks0-skipping cost the TSMQR phase 2 its operand prefetch), for ~1 % extra flops.
    // The head rows go first: the compiler moves them into the group loop's registers before the
    // loop, and that copy waits for them — issued after the strip it waited for the whole strip.
    const __amdgpu_buffer_rsrc_t hrs = head_rsrc(At + colo, ts);  // UNMQR: empty resource, head = 0
    const unsigned hoff = head_off_pair<B>(ldm, 0);
    if (FLOW_PF && active) load_head_pair<B, TQR_HEAD_LD0_AUX, IB>(H, hrs, hoff);
#ifndef TQR_DIAG_NOSTRIP
    if (active && !xin) load_strip_pair<B, S>(X, Xt + colo, ldm, 0);
#endif
    FST(4);
    const int inext = (i == k) ? i0 : i + 1;
    const bool has_next = inext < i1;
    // the group loop as a lambda with a single exit (an early return out of the loop itself made
    // the register allocator spill ~1 KiB around the poll calls)
    auto groups = [&]() -> bool {
    WMARK_INIT();
#ifdef TQR_FLOW_STAMPS
    // (group trace) this wave's running group count, kept in the LDS tail across tasks
    __attribute__((address_space(3))) int* gtr_c = (__attribute__((address_space(3))) int*)(sflag + 113) + (threadIdx.x >> 6);
    int gtr_n = *gtr_c;
#endif
    for (int g = 0; g < NG; ++g) {
#ifdef TQR_FLOW_STAMPS
      if ((threadIdx.x & 63) == 0) *gtr_c = gtr_n + 1;
#endif
      WMARK(7);
      GTR(7, (unsigned long long)(g | (i << 8) | ((unsigned long long)j << 24) | ((unsigned long long)k << 40)));
      {
        bool ok = true;
#ifdef TQR_FLOW_STAMPS
        // (diagnostic) separate this wave's own memory drain from the dependency polls below
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        FST(g == 0 ? 22 : 21);
#endif
        if (t == PT && g + 1 == NG) {
          // last group: may the next element's strip stream in during this phase 2? (its tile
          // must have received step k-1: Tc, loaded two groups ahead)
#ifdef TQR_DIAG_NOSTRIP
          sflag[44] = 0;
#else
          sflag[44] = (NG > 1 && has_next && (k == 0 || lds_ld_volatile(tcs) >= k)) ? 1 : 0;
#endif
        }
        if (t == PT) {
          // first element of a later segment: head rows of group g+1 (prefetched below) final?
          // (from group 1 on, its early load sits in acs)
          if (i == ifirst && seg > 0 && g + 1 < NG && !(g > 0 && lds_ld_volatile(acs) >= seg))
            ok = spin_ge_i(&acg[g + 1], seg, err);
          if (ok) {
            if (g + 1 < NG) ok = ready(i, g + 1);
            else if (has_next) ok = ready(inext, 0);
          }
        }
        FST(j == k + 1 ? 20 : 0);  // Rc wait inside an element (lookahead column / other)
        // group 0: the strip / head loads of this element may still be in flight
        constexpr int NX = G::NKS / 2 + (FLOW_PF ? G::NRI / HPACK : 0);
        // full drain where a publish follows: the segment's last element (head rows, Ac) and the
        // first group after a streamed hand-over (the previous element's strip stores, Tc); and in
        // a wave without a strip (B < FLOW_SW): its youngest operations are LDS-DMA instructions of
        // this group's images, which the counted wait would leave in flight
        const bool full = !has_next || (xin && g == 1) || !active;
        WMARK(2);
        constexpr int NH = (FLOW_PF ? 2 * G::NRI : G::NRI) / HPACK;  // head stores + next head loads
        if (!(g == 0 ? sync_point_first<NX, PT>(ok, sflag, par, active)
                     : full ? sync_point<true, false, PT>(ok, sflag, par) : sync_point_cnt<NH, PT>(ok, sflag, par)))
          return false;
#ifdef TQR_FLOW_STAMPS
        wt_ = __builtin_amdgcn_s_memrealtime();  // (the sync point's own time is in slots 0, 1)
        GTR(2, wt_);
#endif
      }
      // (an LDS-typed read: as a flat read its wait was vmcnt(0))
      bool pipe = false;
      if (g + 1 == NG) pipe = *(volatile int*)(sflag + 44) != 0;  // (written before this sync point)
      // the previous element's strip stores are drained: at group 0 (stored before this
      // element's loads) or, after a streamed hand-over (stores interleaved with the loads), at 1
      if (g == (xin ? 1 : 0) && pending) {
        publish_after_drain(pending, 1);
        pending = nullptr;
      }
      // segment's last element: its head rows of group g-1 (stored write-through) are drained
      if (!has_next && ts && g > 0) publish_after_drain(&acg[g - 1], 1);  // (a lone UNMQR: at the end)
      if (t == PT) {  // early load of the counter the next sync point will test
        const int tg = next_test_group<NG>(g);
        const bool here = g + 2 < NG;  // this element's counter, else the next element's
        if (here || has_next) {
          if (!remote) {
            pv.prefetch(rc, tg, false);
          } else {
            fl_pf = (here ? i : inext) * NG + tg;
            lds_prefetch<PT>(rf + fl_pf, fls, true);
          }
        }
        if (g + 2 == NG && has_next && k > 0) lds_prefetch<PT>(tc(inext), tcs, false);
        if (i == ifirst && seg > 0 && g + 2 < NG) lds_prefetch<PT>(&acg[g + 2], acs, false);
      }
      FST(7);
      if (!FLOW_PF && active) load_head_pair<B, 16, IB>(H, hrs, hoff + g * IB * sizeof(S));
      const double* Vs = lds + buf * BUF;
      const double* Ts = Vs + G::VIMG;
      // the other buffer is free (every wave passed this sync point): next DMA rides phase 1
      // (nothing next: re-read this group's own images into the idle buffer, keeping the
      // DMA stream branch-free)
      const int gd = g + 1 < NG ? g + 1 : has_next ? 0 : g, id = g + 1 < NG ? i : has_next ? inext : i;
      Dma d{lds + (buf ^ 1) * BUF, vimg(id, gd), timg(id, gd), sflag};
      dma_next = g + 1 == NG && has_next;
#if defined(TQR_DIAG_DMA_FIXED)  // what-if: every DMA reads one L2-hot image
      d.v = vimg(k, 0);
      d.t = timg(k, 0);
#endif
#ifdef TQR_DIAG_NODMA  // what-if: no staging at all
      if (active) apply_zw<B, true, NoHook, FLOW_PF, true, HPACK == 2, IB>(Vs, Ts, X, H, W, 0);
#else
      phase_prio<C>(false);
      WMARK(3);
      if (active) apply_zw<B, true, Dma, FLOW_PF, true, HPACK == 2, IB>(Vs, Ts, X, H, W, 0, d);
      else
        for (int m = 0; m < Dma::STEPS; ++m) d.step(m);
#endif
      FST(15);
      WMARK(4);
#ifndef TQR_DIAG_NOHEAD
      if (active) {
        // head rows stay with this workgroup inside the segment (plain write-back stores); the
        // segment's last element hands them to the next segment group by group: write-through
        // stores, drained, then Ac[k][j][s][g]++ (one group later, after the next drain)
        if (has_next) store_head_pair<B, TQR_HEAD_ST_AUX, IB>(H, hrs, hoff + g * IB * sizeof(S));
        else store_head_pair<B, 16, IB>(H, hrs, hoff + g * IB * sizeof(S));
        FST(2);
        // the next group's head rows straight into H (its stores above have read it): a separate
        // prefetch register set was copied into H after phase 2, and that copy waited vmcnt(0) —
        // in the hand-over group for the whole streamed strip
        if (FLOW_PF && g + 1 < NG) load_head_pair<B, TQR_HEAD_LD_AUX, IB>(H, hrs, hoff + (g + 1) * IB * sizeof(S));
      }
#endif
      FST(14);
      WMARK(5);
      phase_prio<C>(true);
      if (active) {
        if (pipe) {
          S* Xn = Aj + (size_t)inext * B;
          const XPipe<B, S> xp{uniform_rsrc(Xt + colo), uniform_rsrc(Xn + colo),
                               (unsigned)((((size_t)(t & 15)) * ldm + 2 * ((t & 63) >> 4)) * sizeof(S))
#ifdef TQR_FLOW_STAMPS
                               , blockIdx.x == 0 && gtr_n < GTR_GROUPS ? g_xtr + ((size_t)gtr_n * 8 + (t >> 6)) * 8 : nullptr
#endif
          };
          apply_x4<B, XPipe<B, S>, IB>(Vs, X, W, xp);
        } else {
          apply_x4<B, NoPost, IB>(Vs, X, W);
        }
      }
      if (g + 1 == NG) xin = pipe;
      FST(13);
      WMARK(6);
#ifdef TQR_FLOW_STAMPS
      ++gtr_n;
#endif
      buf ^= 1;
    }
    return true;
    };
    if (!groups()) return;
#ifndef TQR_DIAG_NOSTRIP
    if (active && !xin) store_strip_pair<B, S>(X, Xt + colo, ldm, 0);
#endif
    pending = tc(i);
    FST(4);
  }
  // last element's strip and its last head-row group: drain, then publish both (a segment of the
  // UNMQR element alone: its strip is the head tile, stored whole at its end — every group)
  sync_point<true, false, PT>(true, sflag, par);
  if (pending) publish_after_drain(pending, 1);
  if (seg == 0 && i0 >= i1)
    for (int g = 0; g + 1 < NG; ++g) publish_after_drain(&acg[g], 1);
  publish_after_drain(&acg[NG - 1], 1);
  FST(4);
}


}  // namespace tqr
#include "chain32.hpp"
#include "chain_asm.hpp"
#include "chain32_asm.hpp"
#include "chain_res.hpp"
#include "xfer.hpp"
namespace tqr {

// dynamic LDS (doubles) of the task paths; the LDS tail (task word, verdicts, ...) follows
template <int B, typename S, class C>
constexpr int flow_lds_doubles() {
  constexpr int panel = flow_panel_doubles<B, C>();
  constexpr int chain = 2 * (FImg<B, S, C>::V + FImg<B, S, C>::T);
  return panel > chain ? panel : chain;
}

template <int B, typename S, class C>
__global__ __launch_bounds__(C::NT, C::WPC) void k_flow(FlowArgs a) {
  static_assert(sizeof(S) == 8 || C::NW == 8, "the fp32 chain runs the 8-wave shape");
  static_assert(C::WPC == 1 || (flow_lds_doubles<B, S, C>() * 8 + 1536) * C::WPC <= 163840, "LDS per CU");
  extern __shared__ __align__(16) double lds[];
  int* s_task = reinterpret_cast<int*>(lds + flow_lds_doubles<B, S, C>());
  int* s_flag = s_task + 1;
#ifdef TQR_FLOW_STAMPS
  if (threadIdx.x == 0) {
    unsigned long long* l_ = reinterpret_cast<unsigned long long*>(s_task + 64);
    l_[0] = __builtin_amdgcn_s_memrealtime();
    for (int c = 0; c < FST_N; ++c) l_[1 + c] = 0;
    unsigned long long* w_ = reinterpret_cast<unsigned long long*>(s_task + 128);
    for (int c = 0; c < 8 * WSL; ++c) w_[c] = 0;
    for (int c = 0; c < 8; ++c) s_task[114 + c] = 0;  // group-trace counters (flow_chain)
  }
  int* sflag = s_flag;
#endif
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
#ifdef TQR_FLOW_STAMPS
    if (threadIdx.x == 0 && idx < (1 << 18)) {
      g_ttl[3 * idx] = __builtin_amdgcn_s_memrealtime();
      g_ttl[3 * idx + 2] = blockIdx.x;
    }
#endif
    if (type == T_CHAIN) {
      if constexpr (sizeof(S) == 8 && C::NW == 4 && C::WPC == 1 && C::IB == 32 && B == 256) {
        flow_chain_res<C>(a, (it.ts >> 8) & 0xff, it.l & 0xffff, it.l >> 16, it.m, it.k & 0xffff, it.k >> 16, lds, s_flag);
      } else if constexpr (sizeof(S) == 8 && C::NW == 8 && (B == 128 || B == 256)) {
        if (a.chain_asm & 3)
          flow_chain_asm<B, C>(a, (it.ts >> 8) & 0xff, it.l & 0xffff, it.l >> 16, it.m, it.k & 0xffff, it.k >> 16, lds,
                               s_flag);
        else
          flow_chain<B, S, C>(a, (it.ts >> 8) & 0xff, it.l & 0xffff, it.l >> 16, it.m, it.k & 0xffff, it.k >> 16, lds,
                              s_flag);
      } else if constexpr (sizeof(S) == 8)
        flow_chain<B, S, C>(a, (it.ts >> 8) & 0xff, it.l & 0xffff, it.l >> 16, it.m, it.k & 0xffff, it.k >> 16, lds,
                         s_flag);
      else if constexpr (C::NW == 8 && (B == 128 || B == 256)) {
        if ((a.chain_asm & 3) && !(a.chain_asm & 8))
          flow_chain32_asm<B, C>(a, (it.ts >> 8) & 0xff, it.l & 0xffff, it.l >> 16, it.m, it.k & 0xffff, it.k >> 16,
                                 lds, s_flag);
        else
          flow_chain32<B>(a, (it.ts >> 8) & 0xff, it.l & 0xffff, it.l >> 16, it.m, it.k & 0xffff, it.k >> 16, lds,
                          s_flag);
      } else
        flow_chain32<B>(a, (it.ts >> 8) & 0xff, it.l & 0xffff, it.l >> 16, it.m, it.k & 0xffff, it.k >> 16, lds,
                        s_flag);
    } else if (type == T_UP || type == T_DOWN) {
      flow_xfer<B, S, C>(a, type == T_UP, it.m, (it.ts >> 8) & 0xff, s_flag);
    } else {
      flow_panel<B, S, C>(a, type, it.l, it.k, lds, s_flag);
    }
    __syncthreads();
#ifdef TQR_FLOW_STAMPS
    if (threadIdx.x == 0 && idx < (1 << 18)) g_ttl[3 * idx + 1] = __builtin_amdgcn_s_memrealtime();
#endif
  }
  // multi-GPU: the last workgroup out tells every rank (itself included) that this launch is done
  // (flow.hpp FlowArgs Done[]): every workgroup's memory operations are complete before it counts
  // itself out, so no read of the workspaces is outstanding when the peers may write them again
  if (a.dist) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(gptr(a.exitc), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int r = 0; r < a.world; ++r)
        __hip_atomic_store(a.peers[r].Rf + a.rf_done + a.rank, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
#ifdef TQR_FLOW_STAMPS
  FST(6);
  if (threadIdx.x == 0) {
    unsigned long long* l_ = reinterpret_cast<unsigned long long*>(s_task + 64);
    for (int c = 0; c < FST_N; ++c) g_fst[blockIdx.x * FST_N + c] = l_[1 + c];
    const unsigned long long* w_ = reinterpret_cast<const unsigned long long*>(s_task + 128);
    for (int c = 0; c < 8 * WSL; ++c) g_wst[blockIdx.x * 8 * WSL + c] = w_[c];
  }
#endif
}

}  // namespace tqr
