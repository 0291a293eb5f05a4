/* The reference's own threading pattern (qrdecomp.c:145-230: copy, initScheduler, a pool of
 * pthreads each running pthr_doTasks over one shared ThreadInfo, join) written against this
 * repository's include/ and linked with libtqr.so: every task the threads take runs on the GPU
 * (doATask). Writes the input, the factorised matrix and tau (float32, column-major) to argv[3]
 * for the test to compare with the oracle. Usage: pthr_driver tiles threads out.bin */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gridscheduler.h"
#include "qrdecomp.h"

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    int t = atoi(argv[1]), nth = atoi(argv[2]), b = 32, m = t * b, n = t * b;
    float *A = newMatrix(m, n), *R = newMatrix(m, n), *tau = newMatrix(m, n);
    srand(5);
    initMatrix(A, m, n, m, 2); /* RANDZO */
    initMatrix(tau, m, n, m, 0);
    copyMatrix(A, m, n, m, R);
    Task* grid = initScheduler(m / b, n / b);
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER, sig = PTHREAD_MUTEX_INITIALIZER;
    pthread_cond_t cond = PTHREAD_COND_INITIALIZER;
    int condMet = 0;
    struct ThreadInfo ti;
    memset(&ti, 0, sizeof ti);
    ti.mat = R; ti.tau = tau; ti.ldm = m; ti.b = b;
    ti.taskGrid = grid; ti.taskM = m / b; ti.taskN = n / b;
    ti.getTaskMutex = &mu; ti.getSigMutex = &sig; ti.newTasksCond = &cond; ti.condMet = &condMet; ti.useWY = 1;
    pthread_t th[64];
    if (nth < 1 || nth > 64) return 2;
    for (int i = 0; i < nth; ++i) pthread_create(&th[i], NULL, pthr_doTasks, &ti);
    for (int i = 0; i < nth; ++i) pthread_join(th[i], NULL);
    free(grid);
    FILE* f = fopen(argv[3], "wb");
    if (!f) return 3;
    fwrite(A, sizeof(float), (size_t)m * n, f);
    fwrite(R, sizeof(float), (size_t)m * n, f);
    fwrite(tau, sizeof(float), (size_t)m * n, f);
    fclose(f);
    printf("done %d x %d on %d threads\n", m, n, nth);
    deleteMatrix(A); deleteMatrix(R); deleteMatrix(tau);
    return 0;
}
