/*
 * GPU entry points of the tiled QR — source-compatible with the reference's
 * include/gpucalc.h:1-8 (s10m/GPU-Tiled-QR-Decomposition), implemented natively on MI355X
 * (HIP/gfx950) by libtqr.so. The names are the reference's; nothing here is a CUDA runtime
 * alias (there is no cudaMalloc/cudaDeviceReset etc. in this library).
 *
 * Behaviour vs the reference (src/gpucalc.cu:1579-1686):
 *   * cudaQRTask: same contract — host column-major `mat` (leading dim ldm), tile size 32,
 *     factorised in place (R + V, tau discarded, gpucalc.cu:1665-1675), blocking, prints
 *     "GPU: x ms". Differences: any m, n that are multiples of 32 (the reference's task count
 *     is wrong for m < n, gpucalc.cu:1546-1559); `maxblocks` is accepted and ignored (the
 *     HIP engine sizes its own launches); no device reset. Errors are printed to stderr and
 *     abort the process (no silent CPU fallback).
 *   * cudaQRFull: declared but never defined in the reference (gpucalc.cu:1801-1877 is a
 *     commented-out sketch of a host-scheduled, level-synchronous, multi-stream factorisation);
 *     here it is exactly that, natively: the wave engine (tqr.h TQR_ENGINE_WAVES) — the host
 *     scheduler's BFS waves of the DAG, two batched launches per wave on two HIP streams. b = 32,
 *     ldm = m, in place, tau discarded, prints "GPU: x ms".
 *   * testDAPP (gpucalc.cu:1706): the reference's TSMQR benchmark — per repetition, srand(5), one
 *     64 x 32 block and 32 taus of ((rand() % 101) - 50) / 50, `nblocks` independent b = 32 DAPPs
 *     on copies of it in one launch, timings[t] = ms x nblocks (tqr.h tqr_tile_batch).
 *   * doCUDADAPP (gpucalc.cu:1776): one DAPP on a 64 x 64 matrix, taus = its first 32 entries.
 */
#ifndef GPUCOMP_H
#define GPUCOMP_H
#ifdef __cplusplus
extern "C" {
#endif
void cudaQRTask(float* mat, int m, int n, int ldm, int maxblocks);      /* gpucalc.cu:1579 */
void cudaQRFull(float* mat, int m, int n);                              /* gpucalc.h:4 */
void testDAPP(float* timings, int n, int nblocks);                      /* gpucalc.cu:1706 */
void doCUDADAPP(float* mat);                                            /* gpucalc.cu:1776 */
/* fp64 sibling (the reference's -Dfloat=double build) */
void cudaQRTask_d(double* mat, int m, int n, int ldm, int maxblocks);
#ifdef __cplusplus
}
#endif
#endif
