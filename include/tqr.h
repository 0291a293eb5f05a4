/*
 * tqr — MI355X-native flat-tree tiled Householder QR (libtqr.so), the native API.
 *
 * Same algorithm and output layout as the reference (s10m/GPU-Tiled-QR-Decomposition):
 *   * A is column-major m x n with leading dimension ldm, factorised in place: the global
 *     upper triangle is R, the strict lower part of each diagonal tile (k,k) holds the
 *     unit-lower GEQRT V, and every tile (i,k), i>k, holds the dense TSQRT V_B
 *     (reference qrdecomp.c:522-523, 683-684);
 *   * Householder conventions of qrdecomp.c:1201-1272 (sign(0)=+1, v0=1, tau=2/v'v, tau=2
 *     for length-1 and zero columns).
 * The tile size b must divide m and n; b in {16, 32, 64, 128, 256}. The leading dimension is
 * bounded by the engine's 32-bit buffer offsets: 32 * ldm * sizeof(element) < 2^31, i.e.
 * ldm <= 8,388,607 (fp64) / 16,777,215 (fp32); larger values return TQR_EINVAL.
 *
 * tau, device API: "compact" m x kmax column-major array (kmax = min(m,n)/b), column k holds
 * the b*(p-k) taus of panel k in rows k*b .. m-1 — exactly column k*b of the reference's
 * m x n tau matrix (qrdecomp.c:392,420,435). The host API returns the reference's m x n
 * tau matrix (other entries untouched).
 *
 * Status codes: 0 = ok, negative = error (see tqr_strerror).
 */
#ifndef TQR_H
#define TQR_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

enum tqr_status {
    TQR_OK = 0,
    TQR_EINVAL = -1,   /* bad sizes / tile size / pointers */
    TQR_ENOMEM = -2,   /* device or host allocation failed */
    TQR_EHIP = -3,     /* a HIP runtime call failed */
    TQR_ENODEV = -4,   /* no usable gfx950 device */
    TQR_ERCCL = -5     /* an RCCL call failed */
};
enum tqr_dtype { TQR_F32 = 0, TQR_F64 = 1 };

const char* tqr_strerror(int status);
const char* tqr_version(void);

/* ---- plans: allocate once, execute many times (no allocation inside execute) ---------- */
typedef struct tqr_plan tqr_plan;

/* Plan a factorisation of an m x n matrix of `dtype` with tile size b on the current HIP
 * device. */
int tqr_plan_create(tqr_plan** plan, int m, int n, int b, int dtype);
/* Execution engines (both compute the same factorisation, bit for bit per tile operation):
 *   TQR_ENGINE_FLOW  — one persistent dataflow launch: workgroups pull GEQRT/TSQRT panel tasks
 *                      and fused UNMQR/TSMQR column chains from a static topological list and
 *                      synchronise through progress counters (default);
 *   TQR_ENGINE_WAVES — the host scheduler's BFS waves of the reference DAG, two batched launches
 *                      per wave (panel tasks, update strips) on two HIP streams joined by events:
 *                      the level-synchronous multi-stream form of the reference's cudaQRFull
 *                      sketch (src/gpucalc.cu:1801-1877).
 * TQR_ENGINE_DEFAULT = FLOW unless the environment sets TQR_ENGINE=waves. */
enum tqr_engine { TQR_ENGINE_DEFAULT = -1, TQR_ENGINE_WAVES = 0, TQR_ENGINE_FLOW = 1 };
int tqr_plan_create_engine(tqr_plan** plan, int m, int n, int b, int dtype, int engine);
void tqr_plan_destroy(tqr_plan* plan);

/* Factorise device matrix dA (ldda >= m) in place; dtau_compact is device memory of
 * m * kmax elements of the same dtype. `stream` is a hipStream_t (NULL = default stream).
 * Stream-ordered: returns once all work is enqueued.
 * A plan owns one set of progress counters and panel workspaces, so its executions are
 * serialised: calls from several host threads are mutually excluded while they enqueue, and
 * each execute's stream first waits for the plan's previous execute (whatever its stream). Two
 * executes of one plan never overlap on the GPU; use one plan per concurrent factorisation. */
int tqr_plan_execute(tqr_plan* plan, void* dA, int ldda, void* dtau_compact, void* stream);

/* Synchronise `stream` and report whether the last execute completed (the persistent engine
 * bounds every dependency wait and reports a timeout here instead of hanging). */
int tqr_plan_status(tqr_plan* plan, void* stream);
/* engine: 1 = persistent dataflow (default; TQR_ENGINE=waves selects 0 = wave-batched
 * launches), ntasks: task-list length, est_order: 1 if the start-time-estimate order was
 * used (else step-major), grid: workgroups of the persistent launch. */
int tqr_plan_info(const tqr_plan* plan, int* engine, int* ntasks, int* est_order, int* grid);

/* Host-only check of the persistent engine's task list for an M x N tile grid (no GPU):
 * number of tasks and whether the estimated-start-time order is topological. */
int tqr_flow_plan_check(int M, int N, int b, int seglen, int* ntasks, int* est_order);
/* Columns of one chain strip of the persistent engine (a tile column is split into
 * ceil(b / width) strips; one workgroup updates one strip). */
int tqr_flow_strip_width(void);
/* Host-only: the persistent engine's task list for an M x N tile grid, 4 ints per task
 * {type | strip << 8, l, m, k} (chains: type 4, l = i0 | i1 << 16, k = step | segment << 16);
 * returns the number of tasks (writes at most `cap`). */
int tqr_flow_plan_export(int M, int N, int b, int seglen, int* items, int cap);
/* Replace the persistent engine's task order (the same tasks as the plan's list, 4 ints each as
 * tqr_flow_plan_export gives them, e.g. from an offline list scheduler): rejected with
 * TQR_EINVAL unless it is a permutation of the plan's tasks that is topological for every
 * in-task wait (the engine's deadlock-freedom condition). Single-GPU flow plans only. */
int tqr_plan_set_tasks(tqr_plan* plan, const int* items, int n);
/* Host-only: 1 if `items` is topological for the engine's waits on an M x N tile grid, else 0. */
int tqr_flow_order_check(int M, int N, int b, const int* items, int n);
/* Diagnostics: copy the persistent engine's panel workspace of step k (the reflector groups'
 * operand images, DESIGN.md "Data layout") to host memory; returns its size in bytes. */
int tqr_plan_debug_workspace(const tqr_plan* plan, int k, void* host, size_t bytes);

/* Per-launch statistics of the last execute (filled when the plan was created with
 * tqr_plan_set_profile(plan, 1)): number of kernel launches and the summed device time of
 * the trailing-update (TSMQR/UNMQR) and panel (GEQRT/TSQRT) kernels in ms. */
int tqr_plan_set_profile(tqr_plan* plan, int on);
int tqr_plan_stats(const tqr_plan* plan, int* nlaunch_update, double* ms_update, int* nlaunch_panel,
                   double* ms_panel);

/* Number of flat-tree tasks (reference calcTotalTasks, src/gpucalc.cu:1546, for all m,n). */
long tqr_total_tasks(int m, int n, int b);

/* ---- multi-GPU: tile-column partition, one process per GPU ---------------------------------
 * Rank r owns the tile columns j with tqr_dist_owner(j) == r — snake order over the ranks
 * (0..W-1, W-1..0, 0..W-1, ...: every rank's columns sum to the same index total, balancing the
 * chain work that grows with j); the owner of column j factors it entirely (its panel when j <
 * kmax, and all its updates).
 * Storage (round 4): a rank holds ONLY its own tile columns, packed in column order — global tile
 * column j is local tile column j / W of the rank's dA (b * tqr_dist_local_cols(plan) columns,
 * leading dimension ldda >= m), and the taus of panel k are column k / W of its compact tau (m x
 * tqr_dist_local_cols(plan)). A 65536 x 16384 fp64 matrix on 8 ranks is 1 GiB per rank.
 * The owner of panel k forwards each finished reflector group's V/T images to every peer over
 * xGMI inside the persistent launch (peer workspaces opened by IPC), so panels of successive
 * steps overlap across GPUs exactly as on one GPU. Every rank calls tqr_plan_execute the same
 * number of times; consecutive executes need no host synchronisation or barrier between the
 * ranks (the cross-rank flags carry launch epochs, and a rank forwards into a peer only once that
 * peer's previous launch has finished, all on the device).
 * Chain tasks are shorter on 4+ ranks that each launch over a whole device (2 elements instead of
 * 8; TQR_SEGLEN overrides): more parallel slack per rank. Every rank must build the
 * same global task list — tqr_dist_import compares the ranks' list signatures (segment lengths,
 * lookahead tail, tail segments, list length and a hash of the whole list in order, so every
 * ordering knob is covered) and fails with TQR_EINVAL if they differ.
 * Setup once: tqr_dist_export -> exchange all ranks' handle blocks (e.g. an all-gather over
 * torch.distributed / MPI) -> tqr_dist_import(plan, blocks of rank 0..world-1). */
int tqr_dist_plan_create(tqr_plan** plan, int m, int n, int b, int dtype, int rank, int world);
/* bytes of one rank's handle block (its device's PCI bus id, its task-list signature, the IPC
 * handles of its panel counters and per-step panel workspaces — one allocation per step keeps
 * every export under 2 GiB) */
size_t tqr_dist_handle_bytes(const tqr_plan* plan);
int tqr_dist_export(tqr_plan* plan, void* handles, size_t len);
int tqr_dist_import(tqr_plan* plan, const void* all_handles, size_t len);
/* Peer-path probe, once after tqr_dist_import (fails fast instead of a wait timeout or a hang in the
 * first factorisation): phase 0 stores this rank's token into every peer's probe word (system-scope
 * stores through the IPC-mapped peer flags, the path panel flags take); then a host barrier over all
 * ranks; phase 1 loads this rank's probe words (system-scope loads, the path the chains poll) and
 * returns TQR_OK if every peer's token arrived, else TQR_EHIP with each missing rank printed.
 * *seen (may be NULL; phase 1) receives the bit mask of the peers whose token arrived. */
int tqr_dist_probe(tqr_plan* plan, int phase, unsigned long long* seen);
/* no-op since round 4 (executes reset their own counters); kept for source compatibility */
int tqr_dist_reset(tqr_plan* plan, void* stream);
int tqr_dist_owner(const tqr_plan* plan, int tile_col);
/* number of tile columns this rank stores (and of its compact tau columns) */
int tqr_dist_local_cols(const tqr_plan* plan);
/* bytes this rank forwards to its peers per factorisation (every owned panel member's V/T images,
 * all reflector groups, to each of the world - 1 peers); 0 for a single-GPU plan */
long long tqr_plan_fwd_bytes(const tqr_plan* plan);
/* host-only: this rank's task-list length and the number of its panel members that forward
 * their V/T images to the peers (its panel tasks when world > 1, else 0); the list is the one a
 * plan of `world` ranks with a whole device each builds (the multi-rank task-list defaults of
 * tqr_dist_plan_create apply; the segment length is `seglen`) */
int tqr_dist_plan_check(int M, int N, int b, int seglen, int rank, int world, int* ntasks, int* nfwd);

/* ---- one-shot helpers ------------------------------------------------------------------ */
/* Device pointers, stream-ordered; plan cached per (device,m,n,b,dtype) and shared by all
 * callers — concurrent calls with the same shape are serialised on the GPU (see execute). */
int tqr_dgeqrt_tiled(int m, int n, int b, double* dA, int ldda, double* dtau_compact, void* stream);
int tqr_sgeqrt_tiled(int m, int n, int b, float* dA, int ldda, float* dtau_compact, void* stream);

/* Host pointers, blocking: A in place; tau = the reference's m x n tau matrix (ldm), or NULL
 * (the reference's cudaQRTask discards tau). Any ldm >= m.
 * With the default (flow) engine the persistent launch moves the matrix itself, overlapping PCIe
 * with the factorisation: it reads each tile column from host memory just before step 0 needs it
 * and writes each tile column back as soon as it is final. Host memory is either a pinned staging
 * buffer that host threads fill and drain while the kernel runs (default), or — environment
 * TQR_HOST_XFER=register — the caller's array itself, page-locked for the call.
 * Retention: the plan of each (device, m, n, b, dtype) keeps an m x n device matrix and an
 * m x kmax tau array, and each device keeps one pinned staging buffer of the largest matrix seen,
 * until tqr_cache_clear(). Calls on one shape are serialised. */
int tqr_dgeqrt_host(double* A, double* tau, int m, int n, int ldm, int b);
int tqr_sgeqrt_host(float* A, float* tau, int m, int n, int ldm, int b);
/* the same with an explicit engine (tqr_engine) and dtype */
int tqr_geqrt_host_engine(int dtype, void* A, void* tau, int m, int n, int ldm, int b, int engine);
/* Release every cached plan of the one-shot helpers (device buffers, pinned buffers) and the
 * host-API staging buffers; synchronises the device first. Plans created by the caller are not
 * affected. */
int tqr_cache_clear(void);
/* Host-only check of the host-API task list (the flow list plus nxc upload / download tasks per
 * tile column, a column's upload estimated at tcol chain elements): number of tasks and whether
 * the estimated-start-time order is topological. */
int tqr_flow_xfer_plan_check(int M, int N, int b, int seglen, int nxc, double tcol, int* ntasks, int* est_order);

/* Host pointers, single tile tasks on the GPU (the reference's per-tile kernels; used by
 * qrdecomp.h's SGEQRF/SLARFT/STSQRF/SSSRFT and by the per-tile parity tests). Tile pointers
 * are tile origins inside one ldm-strided matrix; tau pointers point at the tile's b
 * consecutive taus, as in the reference. */
int tqr_tile_geqrt(int dtype, void* blk, void* tau, int b, int ldm);
int tqr_tile_unmqr(int dtype, void* C, const void* V, const void* tau, int b, int ldm);
int tqr_tile_tsqrt(int dtype, void* A, void* B, void* tau, int b, int ldm);
int tqr_tile_tsmqr(int dtype, const void* V, void* A, void* B, const void* tau, int b, int ldm);

/* Batched independent tile updates in ONE launch of the update kernel (the reference's testDAPP
 * microbenchmark, src/gpucalc.cu:1687-1774, generalised to UNMQR and any b): `nblocks` copies of
 * the host block `blk` are each updated with the same reflectors.
 *   type DAPP (TSMQR): V = b x b dense TSQRT V_B (ldv), tau = its b taus, blk = 2b x b [A; B] (ldb);
 *   type SAPP (UNMQR): V = b x b GEQRT tile (unit-lower V below the diagonal), blk = b x b C.
 * *ms = device time of the update launch (HIP events); out (optional) receives the nblocks
 * results, block j at out + j*b*ldo. The batch is one 2b-row device matrix of (1 + nblocks) b
 * columns addressed with 32-bit offsets: more than 2^31 - 1 bytes returns TQR_EINVAL. */
int tqr_tile_batch(int dtype, int type, int b, int nblocks, const void* V, int ldv, const void* tau,
                   const void* blk, int ldb, void* out, int ldo, float* ms);

/* Device-side synthetic input with the reference's RANDZO distribution
 * ((r mod 201) - 100)/100 (qrdecomp.c:1383), from a counter-based hash of (seed, i, j). */
int tqr_fill_randzo(int dtype, void* dA, int m, int n, int ldda, unsigned long long seed, void* stream);
/* columns col0 .. col0 + ncols - 1 of that matrix only (a multi-GPU rank's own tile columns) */
int tqr_fill_randzo_cols(int dtype, void* dA, int m, int ncols, int ldda, unsigned long long seed, long col0, void* stream);

#ifdef __cplusplus
}
#endif
#endif
