/*
 * Tile-DAG scheduler (host C). Re-implements the reference scheduler's rules
 * (src/gridscheduler.c:13-256) behind its exact API (include/gridscheduler.h), and adds the
 * static wave plan the GPU engine launches from.
 *
 * The tiled QR DAG on an M x N tile grid: step k has QRS(k,k) (GEQRT), SAPP(k,j) j>k (UNMQR),
 * QRD(i,k) i>k (TSQRT) and DAPP(i,j,k) i,j>k (TSMQR). Dependencies:
 *   QRS(k)      <- DAPP(k,k,k-1)
 *   SAPP(k,j)   <- QRS(k), DAPP(k,j,k-1)
 *   QRD(i,k)    <- tile (i-1,k) finished at step k (QRS or QRD), DAPP(i,k,k-1)
 *   DAPP(i,j,k) <- QRD(i,k), tile (i-1,j) finished at step k (SAPP or DAPP), DAPP(i,j,k-1)
 */
#include <stdlib.h>
#include <string.h>

#include "gridscheduler.h"

/* ---------------------------------------------------------------------------------------
 * Reference-compatible grid state machine. One Task per tile carries the step k it is at,
 * the task type for that step and its status; a tile advances one step at a time.
 * ------------------------------------------------------------------------------------- */

static enum Type type_at(int row, int col, int k) {
    if (row == k) return col == k ? QRS : SAPP;
    return col == k ? QRD : DAPP;
}

static int in_grid(int M, int N, int x, int y) { return x >= 0 && y >= 0 && x < M && y < N; }

/* tile (x,y) has finished step k (or is already past it) — src/gridscheduler.c:51-64 */
static int finished(const Task* g, int M, int N, int x, int y, int k) {
    if (!in_grid(M, N, x, y)) return 0;
    const Task* t = &g[y * M + x];
    return (t->k == k && t->taskStatus == DONE) || t->k > k;
}

static int finished_as(const Task* g, int M, int N, int x, int y, int k, enum Type ty) {
    return finished(g, M, N, x, y, k) && g[y * M + x].taskType == ty;
}

/* DAPP at (x,y) step k done; off-grid counts as done (src/gridscheduler.c:81-95) */
static int dapp_done(const Task* g, int M, int N, int x, int y, int k) {
    if (!in_grid(M, N, x, y)) return 1;
    return finished_as(g, M, N, x, y, k, DAPP);
}

static int can_sapp(const Task* g, int M, int N, int x, int y, int k) {
    if (!in_grid(M, N, x - 1, y)) return 1; /* row 0: only QRS(0) needed, src/gridscheduler.c:122 */
    return finished_as(g, M, N, k, k, k, QRS) && dapp_done(g, M, N, x, y, k - 1);
}

static int can_qrd(const Task* g, int M, int N, int x, int y, int k) {
    if (!in_grid(M, N, x, y)) return 0;
    if (!finished(g, M, N, x - 1, y, k)) return 0;
    return k == 0 || dapp_done(g, M, N, x, y, k - 1);
}

/* The reference reads tile (0,k+1) through column-major aliasing when x == M
 * (src/gridscheduler.c:160 via :203/:251); bounds are checked explicitly here instead. */
static int can_dapp(const Task* g, int M, int N, int x, int y, int k) {
    if (!in_grid(M, N, x, y)) return 0;
    if (!finished_as(g, M, N, x, k, k, QRD)) return 0;
    if (!finished(g, M, N, x - 1, y, k)) return 0;
    return k == 0 || dapp_done(g, M, N, x, y, k - 1);
}

static void set_task(Task* g, int M, int x, int y, enum Type ty, enum Status st, int k) {
    Task* t = &g[y * M + x];
    t->taskType = ty;
    t->taskStatus = st;
    t->k = k;
}

Task* initScheduler(int M, int N) {
    Task* g = (Task*)malloc(sizeof(Task) * (size_t)M * N);
    if (!g) return NULL;
    for (int y = 0; y < N; y++)
        for (int x = 0; x < M; x++) {
            Task* t = &g[y * M + x];
            t->l = x;
            t->m = y;
            t->k = 0;
            t->taskType = type_at(x, y, 0);
            t->taskStatus = NONE;
        }
    set_task(g, M, 0, 0, QRS, READY, 0);
    return g;
}

void doneATask(Task* g, int M, int N, Task t) {
    int p = t.l, q = t.m;
    if (!in_grid(M, N, p, q)) return;
    int k = g[q * M + p].k;
    g[q * M + p].taskStatus = DONE;
    switch (type_at(p, q, k)) {
    case QRS: /* src/gridscheduler.c:189-200 */
        for (int j = k + 1; j < N; j++)
            if (can_sapp(g, M, N, p, j, k)) set_task(g, M, p, j, SAPP, READY, k);
        if (can_qrd(g, M, N, p + 1, q, k)) set_task(g, M, p + 1, q, QRD, READY, k);
        break;
    case SAPP: /* :201-206 */
        if (can_dapp(g, M, N, p + 1, q, k)) set_task(g, M, p + 1, q, DAPP, READY, k);
        break;
    case QRD: /* :207-218 */
        for (int j = k + 1; j < N; j++)
            if (can_dapp(g, M, N, p, j, k)) set_task(g, M, p, j, DAPP, READY, k);
        if (can_qrd(g, M, N, p + 1, q, k)) set_task(g, M, p + 1, q, QRD, READY, k);
        break;
    case DAPP: { /* :219-254 */
        int ok = 0;
        enum Type nt = type_at(p, q, k + 1);
        switch (nt) {
        case QRS: ok = in_grid(M, N, p, q); break;
        case SAPP: ok = can_sapp(g, M, N, p, q, k + 1); break;
        case QRD: ok = can_qrd(g, M, N, p, q, k + 1); break;
        case DAPP: ok = can_dapp(g, M, N, p, q, k + 1); break;
        }
        if (ok) set_task(g, M, p, q, nt, READY, k + 1);
        if (can_dapp(g, M, N, p + 1, q, k)) set_task(g, M, p + 1, q, DAPP, READY, k);
        break;
    }
    }
}

int getNextTask(Task* out, Task* g, int M, int N) {
    int r = TASK_DONE;
    Task none;
    memset(&none, 0, sizeof none);
    none.taskStatus = NONE;
    for (int i = M - 1; i >= 0; i--)
        for (int j = N - 1; j >= 0; j--) {
            Task* t = &g[j * M + i];
            if (t->taskStatus == READY) {
                t->taskStatus = DOING;
                *out = *t;
                return TASK_AVAIL;
            }
            if (t->taskStatus == DOING) r = TASK_NONE;
        }
    *out = none;
    return r;
}

/* ---------------------------------------------------------------------------------------
 * Static wave plan. wave(task) = 1 + max(wave(deps)), which equals the BFS wave the
 * reference scheduler produces when every READY task of a wave is completed before the next
 * wave is taken (tests/test_sched.py checks it against tests/golden/sched.npz).
 * ------------------------------------------------------------------------------------- */

long tqr_sched_total_tasks(int M, int N) {
    long n = 0;
    int kmax = M < N ? M : N;
    for (int k = 0; k < kmax; k++) n += (long)(M - k) * (N - k);
    return n;
}

int tqr_sched_plan(int M, int N, tqr_plan_t* plan) {
    memset(plan, 0, sizeof *plan);
    if (M <= 0 || N <= 0) return -1;
    int kmax = M < N ? M : N;
    plan->M = M;
    plan->N = N;
    plan->ntasks = tqr_sched_total_tasks(M, N);
    /* wave of the current step of every tile: lv[k-parity][y*M+x] */
    int* cur = (int*)malloc(sizeof(int) * (size_t)M * N);
    int* prev = (int*)malloc(sizeof(int) * (size_t)M * N);
    int* wave = (int*)malloc(sizeof(int) * (size_t)plan->ntasks);
    int* tk = (int*)malloc(sizeof(int) * 4 * (size_t)plan->ntasks);
    if (!cur || !prev || !wave || !tk) {
        free(cur); free(prev); free(wave); free(tk);
        return -2;
    }
    long n = 0;
    int maxw = 0;
    for (int k = 0; k < kmax; k++) {
        for (int x = k; x < M; x++)
            for (int y = k; y < N; y++) {
                int w = 0;
                enum Type ty = type_at(x, y, k);
                int dk = k > 0 ? prev[y * M + x] + 1 : 0; /* DAPP(x,y,k-1) */
                if (dk > w) w = dk;
                if (ty == SAPP) {
                    int d = cur[k * M + k] + 1; /* QRS(k) */
                    if (d > w) w = d;
                } else if (ty == QRD) {
                    int d = cur[y * M + x - 1] + 1; /* tile (x-1,k) at step k */
                    if (d > w) w = d;
                } else if (ty == DAPP) {
                    int d1 = cur[k * M + x] + 1;     /* QRD(x,k) */
                    int d2 = cur[y * M + x - 1] + 1; /* tile (x-1,y) at step k */
                    if (d1 > w) w = d1;
                    if (d2 > w) w = d2;
                }
                cur[y * M + x] = w;
                wave[n] = w;
                tk[4 * n + 0] = ty;
                tk[4 * n + 1] = x;
                tk[4 * n + 2] = y;
                tk[4 * n + 3] = k;
                if (w > maxw) maxw = w;
                n++;
            }
        int* t = prev; prev = cur; cur = t;
        memcpy(cur, prev, sizeof(int) * (size_t)M * N);
    }
    plan->nlevels = maxw + 1;
    plan->level_off = (long*)calloc((size_t)plan->nlevels + 1, sizeof(long));
    plan->tasks = (int*)malloc(sizeof(int) * 4 * (size_t)plan->ntasks);
    /* counting sort by (wave, class) with class 0 = QRS/QRD, 1 = SAPP, 2 = DAPP */
    long* cnt = (long*)calloc((size_t)plan->nlevels * 3 + 1, sizeof(long));
    for (long i = 0; i < n; i++) {
        int ty = tk[4 * i], cls = (ty == QRS || ty == QRD) ? 0 : (ty == SAPP ? 1 : 2);
        cnt[wave[i] * 3 + cls + 1]++;
    }
    for (long c = 0; c < (long)plan->nlevels * 3; c++) cnt[c + 1] += cnt[c];
    for (int L = 0; L <= plan->nlevels; L++) plan->level_off[L] = cnt[L * 3];
    for (long i = 0; i < n; i++) {
        int ty = tk[4 * i], cls = (ty == QRS || ty == QRD) ? 0 : (ty == SAPP ? 1 : 2);
        long pos = cnt[wave[i] * 3 + cls]++;
        memcpy(plan->tasks + 4 * pos, tk + 4 * i, sizeof(int) * 4);
    }
    free(cnt);
    free(cur);
    free(prev);
    free(wave);
    free(tk);
    return 0;
}

void tqr_sched_plan_free(tqr_plan_t* plan) {
    free(plan->tasks);
    free(plan->level_off);
    memset(plan, 0, sizeof *plan);
}
