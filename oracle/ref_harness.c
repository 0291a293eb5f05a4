/*
 * TEST INFRASTRUCTURE ONLY — driver for the reference's own host code (oracle/_ref/).
 * Compiled together with the reference's qrdecomp.c tile kernels / worker loop and its
 * src/gridscheduler.c by oracle/build_ref.sh; `float` here is the reference's element type
 * (build_ref.sh passes -Dfloat=double for the fp64 library, exactly as SURVEY.md §8c builds
 * the fp64 reference). Everything below only calls reference functions; it replaces the
 * parts of qrdecomp.c that cannot be compiled here (main/tiledQR/taskQRP_threads need the
 * absent include/cycle.h for their rdtsc timers, qrdecomp.c:15,150,196,218).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "include/gridscheduler.h"
#include "qrdecomp.h"

/* Same thread setup as taskQRP_threads (qrdecomp.c:145-230), minus its rdtsc timer. */
double ref_factor(const float* A, float* R, float* tau, int m, int n, int b, int ldm, int nthreads) {
    pthread_t threads[256];
    struct ThreadInfo info[256];
    pthread_cond_t cond = PTHREAD_COND_INITIALIZER;
    pthread_mutex_t mutex = PTHREAD_MUTEX_INITIALIZER;
    int condMet = 0, p = m / b, q = n / b;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    copyMatrix((float*)A, m, n, ldm, R);
    Task* grid = initScheduler(p, q);
    for (int i = 0; i < nthreads; i++) {
        info[i].wspace[0] = newMatrix(2 * b, 1);
        info[i].wspace[1] = newMatrix(2 * b, 1);
        info[i].mat = R;
        info[i].useWY = 1;
        info[i].tau = tau;
        info[i].ldm = ldm;
        info[i].b = b;
        info[i].getTaskMutex = &mutex;
        info[i].newTasksCond = &cond;
        info[i].condMet = &condMet;
        info[i].taskGrid = grid;
        info[i].taskM = p;
        info[i].taskN = q;
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < nthreads; t++) pthread_create(&threads[t], NULL, pthr_doTasks, &info[t]);
    condMet = 1;
    for (int t = 0; t < nthreads; t++) pthread_join(threads[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    for (int i = 0; i < nthreads; i++) {
        deleteMatrix(info[i].wspace[0]);
        deleteMatrix(info[i].wspace[1]);
    }
    free(grid);
    return (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}

/* Single reference tile kernels (qrdecomp.c:532, 559, 689, 723). */
void ref_geqrt(float* blk, float* tau, int b, int ldm) {
    float* w = newMatrix(2 * b, 1);
    SGEQRF(blk, tau, b, b, ldm, w);
    deleteMatrix(w);
}
void ref_unmqr(float* C, float* V, float* tau, int b, int ldm) {
    float* w[2] = {newMatrix(2 * b, 1), newMatrix(2 * b, 1)};
    SLARFT(C, V, tau, b, b, ldm, w);
    deleteMatrix(w[0]);
    deleteMatrix(w[1]);
}
void ref_tsqrt(float* A, float* B, float* tau, int b, int ldm) {
    float* w = newMatrix(2 * b, 1);
    STSQRF(A, B, tau, b, b, b, ldm, w);
    deleteMatrix(w);
}
void ref_tsmqr(float* V, float* A, float* B, float* tau, int b, int ldm) { SSSRFT(V, A, B, tau, b, b, ldm); }

/* RANDZO init exactly as tiledQR does it (qrdecomp.c:81, 89): srand(seed) then initMatrix. */
void ref_randzo(float* A, int m, int n, int ldm, unsigned seed) {
    srand(seed);
    initMatrix(A, m, n, ldm, 2 /* RANDZO, qrdecomp.c:25 */);
}

/* Serial scheduler trace: getNextTask / doneATask until TASK_DONE (src/gridscheduler.c).
 * out[4*i..] = (type, l, m, k). Returns the number of tasks (or -1 past cap). */
int ref_sched_trace(int M, int N, int* out, int cap) {
    Task* grid = initScheduler(M, N);
    Task t;
    int n = 0;
    while (getNextTask(&t, grid, M, N) == TASK_AVAIL) {
        if (n >= cap) { free(grid); return -1; }
        out[4 * n + 0] = t.taskType; out[4 * n + 1] = t.l; out[4 * n + 2] = t.m; out[4 * n + 3] = t.k;
        n++;
        doneATask(grid, M, N, t);
    }
    free(grid);
    return n;
}

/* BFS levels ("waves") of the reference scheduler: take every READY task, complete them all
 * in scan order, repeat. level_sizes[L] = tasks in wave L; returns waves. */
int ref_sched_levels(int M, int N, int* level_sizes, int cap) {
    Task* grid = initScheduler(M, N);
    Task* batch = (Task*)malloc(sizeof(Task) * (size_t)M * N);
    int L = 0;
    for (;;) {
        int nb = 0;
        Task t;
        while (getNextTask(&t, grid, M, N) == TASK_AVAIL) batch[nb++] = t;
        if (nb == 0) break;
        if (L < cap) level_sizes[L] = nb;
        L++;
        for (int i = 0; i < nb; i++) doneATask(grid, M, N, batch[i]);
    }
    free(batch);
    free(grid);
    return L;
}
