/* A reference-style driver (the flow of qrdecomp.c:64-130 tiledQR) compiled against this
 * repository's include/ and linked with libtqr.so — no reference source is used. It is what
 * INTEGRATION.md shows a reference user writing: the host entry point (taskQRP_threads) and the
 * GPU entry points (cudaQRTask, cudaQRFull) produce the same in-place factorisation, checked with
 * the reference's own checkEqual (|diff| <= 1e-3). With a second argument it also writes the input,
 * taskQRP_threads' matrix and tau and cudaQRTask's matrix (float32, column-major) to that file, for
 * the test to compare with the oracle. Usage: tiledqr_driver [tiles per side] [out.bin] */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>

#include "gridscheduler.h"
#include "qrdecomp.h"
#include "gpucalc.h"

int main(int argc, char** argv) {
    int t = argc > 1 ? atoi(argv[1]) : 4, b = 32, m = t * b, n = t * b;
    float *A = newMatrix(m, n), *R = newMatrix(m, n), *tau = newMatrix(m, n);
    float *G = newMatrix(m, n), *H = newMatrix(m, n);
    srand(5);
    initMatrix(A, m, n, m, 2); /* RANDZO */
    initMatrix(tau, m, n, m, 0);
    taskQRP_threads(A, R, tau, m, n, b, m, 1);
    copyMatrix(A, m, n, m, G);
    cudaQRTask(G, m, n, m, 128);
    copyMatrix(A, m, n, m, H);
    cudaQRFull(H, m, n);
    int ok = checkEqual(G, R, m, n, m) && checkEqual(H, R, m, n, m);
    if (argc > 2) {
        FILE* f = fopen(argv[2], "wb");
        if (!f) return 3;
        fwrite(A, sizeof(float), (size_t)m * n, f);
        fwrite(R, sizeof(float), (size_t)m * n, f);
        fwrite(tau, sizeof(float), (size_t)m * n, f);
        fwrite(G, sizeof(float), (size_t)m * n, f);
        fclose(f);
    }
    printf(ok ? "Correct.\n" : "Failure.\n");
    deleteMatrix(A); deleteMatrix(R); deleteMatrix(tau); deleteMatrix(G); deleteMatrix(H);
    return ok ? 0 : 1;
}
