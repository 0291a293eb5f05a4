/*
 * Host-side entry points of the tiled QR — source-compatible with the reference's
 * qrdecomp.h:1-57 for the live (useWY = 1) path, executed on the MI355X by libtqr.so.
 * Unlike the reference header this one is self-contained (it includes <pthread.h> and
 * gridscheduler.h itself, which the reference needed included first, qrdecomp.c:9,13,16).
 *
 *   taskQRP_threads (qrdecomp.c:145): copies matData into matResult and factorises it in
 *     place with tile size b; tau receives the m x n tau matrix (ldm), other entries left
 *     untouched as in the reference. Runs on the GPU; it prints the reference's "CPU: x ms" line
 *     (same prefix, for scripts that parse it) with "(taskQRP_threads on the GPU, host pointers,
 *     end to end)" appended, timing the whole call. useWY is accepted; both
 *     values compute the same factorisation (the reference's non-WY kernels are dead code,
 *     SURVEY §2 #7).
 *   SGEQRF / SLARFT / STSQRF / SSSRFT (qrdecomp.c:532, 559, 689, 723): one tile task on the
 *     GPU, host pointers, same arguments; m = n = b required (the only way the reference calls
 *     them, qrdecomp.c:395-441); b in {16,32,64,128,256}. Work arrays are ignored.
 *   doATask (qrdecomp.c:377): one DAG task with the reference's tile-pointer contract.
 *   pthr_doTasks / doPthrBcast (qrdecomp.c:306-367): the reference's worker loop for callers that
 *     run their own threads over one task grid.
 * D* / *_d: fp64 siblings. Errors print to stderr and abort (no CPU fallback exists).
 * The reference's non-WY kernels (qRSingleBlock ... insSingleHHVector, qrdecomp.c:777-1186)
 * are dead code there (useWY hard-coded to 1, qrdecomp.c:96) and are not provided.
 */
#ifndef QRDECOMP_H
#define QRDECOMP_H
#include <pthread.h>

#include "gridscheduler.h"
#ifdef __cplusplus
extern "C" {
#endif

/* The reference's worker-thread loop and its broadcast (qrdecomp.h:3-4, qrdecomp.c:306-367): run
 * pthr_doTasks(&info) on each of your own pthreads, all sharing one ThreadInfo (task grid from
 * initScheduler, one mutex, one condition variable); every task it takes runs on the GPU through
 * doATask. Returns NULL when the grid is done. */
void* pthr_doTasks(void* threadInfo);
void doPthrBcast(pthread_cond_t* cond, int* condMet);

struct ThreadInfo { /* qrdecomp.h:6-17 (pthr_doTasks' argument) */
    float *mat, *wspace[2], *tau;
    int ldm, b;
    Task* taskGrid;
    int taskM, taskN;
    pthread_mutex_t *getTaskMutex, *getSigMutex;
    pthread_cond_t* newTasksCond;
    int *condMet, useWY;
};

void taskQRP_threads(float* matData, float* matResult, float* tau, int m, int n, int b, int ldm, int useWY);
void doATask(Task t, float* mat, float* tau, int b, int ldm, float** colVect, int useWY);
void SGEQRF(float* block, float* tauBlock, int m, int n, int ldm, float* workVector);
void SLARFT(float* block, float* blockV, float* tauBlock, int m, int n, int ldm, float** w);
void STSQRF(float* blockA, float* blockB, float* blockTau, int ma, int mb, int n, int ldm, float* hhVector);
void SSSRFT(float* blockV, float* blockA, float* blockB, float* blockTau, int b, int n, int ldm);

void taskQRP_threads_d(double* matData, double* matResult, double* tau, int m, int n, int b, int ldm, int useWY);
void doATask_d(Task t, double* mat, double* tau, int b, int ldm, double** colVect, int useWY);
void DGEQRF(double* block, double* tauBlock, int m, int n, int ldm, double* workVector);
void DLARFT(double* block, double* blockV, double* tauBlock, int m, int n, int ldm, double** w);
void DTSQRF(double* blockA, double* blockB, double* blockTau, int ma, int mb, int n, int ldm, double* hhVector);
void DSSRFT(double* blockV, double* blockA, double* blockB, double* blockTau, int b, int n, int ldm);

/* Host utilities of the reference (qrdecomp.c:1313-1400), same behaviour. */
float* newMatrix(int m, int n);
void deleteMatrix(float* mat);
void initMatrix(float* mat, int m, int n, int ldm, int mode); /* 0 ZERO, 1 RAND, 2 RANDZO, 3 EYE */
void printMatrix(float* mat, int m, int n, int ldm);
void copyMatrix(float* mat, int m, int n, int ldm, float* copymat);
int checkEqual(float* matA, float* matB, int m, int n, int ldm); /* |diff| <= 1e-3, qrdecomp.c:23 */

#ifdef __cplusplus
}
#endif
#endif
