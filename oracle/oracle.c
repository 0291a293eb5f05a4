/*
 * TEST INFRASTRUCTURE ONLY — clean-room CPU restatement of the reference host path
 * (s10m/GPU-Tiled-QR-Decomposition: qrdecomp.c + src/gridscheduler.c) used as the parity
 * oracle and as the "port" CPU baseline. Never linked into, loaded by, or called from the
 * product library (gpu-tiled-qr-decomposition_amd/); only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load liboracle.so.
 *
 * Pinning: bit-identical to the reference's own host code built from its sources by
 * oracle/build_ref.sh (oracle/_ref/), checked by tests/test_oracle.py against the committed
 * fixtures in tests/golden/ (made by tests/golden/make_golden.py from oracle/_ref).
 *
 * Build: gcc -O2 -ffp-contract=off -fPIC -shared (oracle/Makefile).
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define REAL float
#define SFX _s
#include "oracle_kernels.inc"
#undef REAL
#undef SFX

#define REAL double
#define SFX _d
#include "oracle_kernels.inc"
#undef REAL
#undef SFX

/* ---------------------------------------------------------------------------------------
 * Multi-threaded executor of the same DAG (the reference runs 8 pthreads, qrdecomp.c:21,
 * 145-230). Successor rules restate doneATask (src/gridscheduler.c:176-256); readiness is a
 * dependency count per task instead of the reference's grid scan, which changes only the
 * order of independent tasks and therefore not a single output bit.
 * ------------------------------------------------------------------------------------- */
typedef struct {
    int p, q, kmax;
    int* deps; /* remaining dependency count per task id */
    int* ready; /* LIFO of ready task ids */
    int nready, ntasks, ndone;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    void* mat;
    void* tau;
    int b, ldm, dbl;
} ox_t;

static int ox_id(const ox_t* s, int i, int j, int k) { return (k * s->q + j) * s->p + i; }

static int ox_type(int i, int j, int k) {
    if (i == k) return j == k ? ORACLE_QRS : ORACLE_SAPP;
    return j == k ? ORACLE_QRD : ORACLE_DAPP;
}

static int ox_exists(const ox_t* s, int i, int j, int k) {
    return k >= 0 && k < s->kmax && i >= k && j >= k && i < s->p && j < s->q;
}

/* successors of (i,j,k); returns count */
static int ox_succ(const ox_t* s, int i, int j, int k, int* out) {
    int n = 0, t = ox_type(i, j, k);
    switch (t) {
    case ORACLE_QRS:
        for (int jj = k + 1; jj < s->q; jj++) out[n++] = ox_id(s, k, jj, k);
        if (ox_exists(s, k + 1, k, k)) out[n++] = ox_id(s, k + 1, k, k);
        break;
    case ORACLE_SAPP:
        if (ox_exists(s, k + 1, j, k)) out[n++] = ox_id(s, k + 1, j, k);
        break;
    case ORACLE_QRD:
        for (int jj = k + 1; jj < s->q; jj++) out[n++] = ox_id(s, i, jj, k);
        if (ox_exists(s, i + 1, k, k)) out[n++] = ox_id(s, i + 1, k, k);
        break;
    case ORACLE_DAPP:
        if (ox_exists(s, i, j, k + 1)) out[n++] = ox_id(s, i, j, k + 1);
        if (ox_exists(s, i + 1, j, k)) out[n++] = ox_id(s, i + 1, j, k);
        break;
    }
    return n;
}

static void* ox_worker(void* arg) {
    ox_t* s = (ox_t*)arg;
    int* succ = (int*)malloc(sizeof(int) * (s->q + s->p + 4));
    void* w = malloc((s->dbl ? sizeof(double) : sizeof(float)) * 2 * s->b);
    pthread_mutex_lock(&s->mu);
    for (;;) {
        while (s->nready == 0 && s->ndone < s->ntasks) pthread_cond_wait(&s->cv, &s->mu);
        if (s->ndone >= s->ntasks) break;
        int id = s->ready[--s->nready];
        pthread_mutex_unlock(&s->mu);
        int i = id % s->p, j = (id / s->p) % s->q, k = id / (s->p * s->q);
        int t = ox_type(i, j, k);
        if (s->dbl)
            oracle_do_task_d(t, i, j, k, (double*)s->mat, (double*)s->tau, s->b, s->ldm, (double*)w);
        else
            oracle_do_task_s(t, i, j, k, (float*)s->mat, (float*)s->tau, s->b, s->ldm, (float*)w);
        int ns = ox_succ(s, i, j, k, succ);
        pthread_mutex_lock(&s->mu);
        s->ndone++;
        for (int x = 0; x < ns; x++)
            if (--s->deps[succ[x]] == 0) s->ready[s->nready++] = succ[x];
        pthread_cond_broadcast(&s->cv);
    }
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
    free(succ);
    free(w);
    return NULL;
}

static void ox_run(void* A, void* R, void* tau, int m, int n, int b, int ldm, int nthreads, int dbl) {
    size_t es = dbl ? sizeof(double) : sizeof(float);
    for (int j = 0; j < n; j++) memcpy((char*)R + es * (size_t)j * ldm, (char*)A + es * (size_t)j * ldm, es * m);
    ox_t s;
    memset(&s, 0, sizeof s);
    s.p = m / b; s.q = n / b; s.kmax = s.p < s.q ? s.p : s.q;
    size_t cap = (size_t)s.p * s.q * s.kmax;
    s.deps = (int*)calloc(cap, sizeof(int));
    s.ready = (int*)malloc(sizeof(int) * cap);
    s.mat = R; s.tau = tau; s.b = b; s.ldm = ldm; s.dbl = dbl;
    int* succ = (int*)malloc(sizeof(int) * (s.p + s.q + 4));
    for (int k = 0; k < s.kmax; k++)
        for (int j = k; j < s.q; j++)
            for (int i = k; i < s.p; i++) {
                s.ntasks++;
                int ns = ox_succ(&s, i, j, k, succ);
                for (int x = 0; x < ns; x++) s.deps[succ[x]]++;
            }
    free(succ);
    s.ready[s.nready++] = ox_id(&s, 0, 0, 0);
    pthread_mutex_init(&s.mu, NULL);
    pthread_cond_init(&s.cv, NULL);
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, ox_worker, &s);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&s.mu);
    pthread_cond_destroy(&s.cv);
    free(s.deps);
    free(s.ready);
}

void oracle_factor_threads_s(const float* A, float* R, float* tau, int m, int n, int b, int ldm, int nthreads) {
    ox_run((void*)A, R, tau, m, n, b, ldm, nthreads, 0);
}
void oracle_factor_threads_d(const double* A, double* R, double* tau, int m, int n, int b, int ldm, int nthreads) {
    ox_run((void*)A, R, tau, m, n, b, ldm, nthreads, 1);
}

/* ---------------------------------------------------------------------------------------
 * Residual checker (fp64 accumulation) for the in-place layout: rebuilds Q^T A by applying
 * the stored reflectors tile task by tile task to a copy of A, in the same topological order,
 * and returns ||Q^T A - R||_F / ||A||_F with R = global upper triangle of F.
 * F and tau are the factorised matrix and the m x n tau matrix (any precision, passed as
 * double). This is an independent check that needs neither numpy nor the GPU.
 * ------------------------------------------------------------------------------------- */
double oracle_residual_d(const double* A, const double* F, const double* tau, int m, int n, int b, int ldm) {
    int p = m / b, q = n / b, kmax = p < q ? p : q;
    double* X = (double*)malloc(sizeof(double) * (size_t)ldm * n);
    memcpy(X, A, sizeof(double) * (size_t)ldm * n);
    double* v = (double*)malloc(sizeof(double) * 2 * b);
    for (int k = 0; k < kmax; k++) {
        size_t kb = (size_t)k * b;
        /* GEQRT reflectors of tile (k,k): v = [1; F[kb+r+1 .. kb+b-1, kb+r]] on rows kb+r.. */
        for (int r = 0; r < b; r++) {
            double t = tau[kb * ldm + kb + r];
            int len = b - r;
            v[0] = 1.0;
            for (int x = 1; x < len; x++) v[x] = F[(kb + r) * ldm + kb + r + x];
            for (int j = (int)kb; j < n; j++) {
                double* xj = X + (size_t)j * ldm + kb + r;
                double d = 0;
                for (int x = 0; x < len; x++) d += v[x] * xj[x];
                d *= t;
                for (int x = 0; x < len; x++) xj[x] -= d * v[x];
            }
        }
        /* TSQRT reflectors of tiles (i,k): v = e_(kb+r) + F[ib.., kb+r] on rows ib..ib+b-1 */
        for (int i = k + 1; i < p; i++) {
            size_t ib = (size_t)i * b;
            for (int r = 0; r < b; r++) {
                double t = tau[(kb)*ldm + ib + r];
                const double* vb = F + (kb + r) * ldm + ib;
                for (int j = (int)kb; j < n; j++) {
                    double* xj = X + (size_t)j * ldm;
                    double d = xj[kb + r];
                    for (int x = 0; x < b; x++) d += vb[x] * xj[ib + x];
                    d *= t;
                    xj[kb + r] -= d;
                    for (int x = 0; x < b; x++) xj[ib + x] -= d * vb[x];
                }
            }
        }
    }
    double num = 0, den = 0;
    for (int j = 0; j < n; j++)
        for (int i = 0; i < m; i++) {
            double a = A[(size_t)j * ldm + i];
            double r = i <= j ? F[(size_t)j * ldm + i] : 0.0;
            double d = X[(size_t)j * ldm + i] - r;
            num += d * d;
            den += a * a;
        }
    free(X);
    free(v);
    return den > 0 ? sqrt(num / den) : sqrt(num);
}
