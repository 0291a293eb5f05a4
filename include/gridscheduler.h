/*
 * Tile-DAG scheduler of the MI355X tiled QR — source-compatible with the reference's
 * include/gridscheduler.h (s10m/GPU-Tiled-QR-Decomposition, include/gridscheduler.h:1-23):
 * the same Task struct, enums, TASK_* codes and the three entry points, with the same
 * readiness rules (src/gridscheduler.c:13-256) and the same bottom-right-first selection
 * order of getNextTask (src/gridscheduler.c:259-300), so a serial getNextTask/doneATask loop
 * yields the reference's task sequence task for task. Implemented in
 * gpu-tiled-qr-decomposition_amd/csrc/sched.c; not thread-safe (as the reference: callers
 * serialise, qrdecomp.c:253,290).
 *
 * Extensions (tqr_sched_*): the task count for any grid shape and the static BFS wave plan the
 * GPU engines are built from. getNextTask keeps the reference's O(M*N) scan (its selection
 * order is part of the contract).
 */
#ifndef GRIDSCHEDULER_H
#define GRIDSCHEDULER_H

#ifdef __cplusplus
extern "C" {
#endif

#define tgrid(x, y) taskGrid[(((y) * M) + (x))]

#define TASK_AVAIL 0
#define TASK_NONE 1
#define TASK_DONE 2

enum Type { QRS, SAPP, QRD, DAPP };
enum Status { READY, DOING, DONE, NONE, NOTASKS };

typedef struct {
    enum Type taskType;
    int l, m, k;
    enum Status taskStatus;
} Task;

/* reference include/gridscheduler.h:19 — mark t done, make newly enabled tiles READY */
void doneATask(Task* taskGrid, int M, int N, Task t);
/* reference include/gridscheduler.h:20 — first READY tile scanning from (M-1,N-1);
 * returns TASK_AVAIL / TASK_NONE (only DOING left) / TASK_DONE */
int getNextTask(Task* t, Task* taskGrid, int M, int N);
/* reference include/gridscheduler.h:21 — malloc'd M x N grid, QRS(0,0) READY; caller frees */
Task* initScheduler(int M, int N);

/* ---- extensions ------------------------------------------------------------------------ */

/* Number of tasks of the flat-tree tiled QR on an M x N tile grid (any aspect ratio; the
 * reference's calcTotalTasks, src/gpucalc.cu:1546-1559, is only right for M >= N). */
long tqr_sched_total_tasks(int M, int N);

/* A static wave ("level") plan: every task of BFS wave L depends only on tasks of waves < L.
 * tasks[4*i .. 4*i+3] = (type, l, m, k); level_off[L] .. level_off[L+1] index wave L, and
 * inside a wave panel tasks (QRS, QRD) come first, then SAPP, then DAPP. */
typedef struct {
    int M, N, nlevels;
    long ntasks;
    int* tasks;
    long* level_off;
} tqr_plan_t;

int tqr_sched_plan(int M, int N, tqr_plan_t* plan); /* 0 on success */
void tqr_sched_plan_free(tqr_plan_t* plan);

#ifdef __cplusplus
}
#endif
#endif
