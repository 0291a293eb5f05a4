/*
 * TEST INFRASTRUCTURE ONLY — the parity oracle's C interface (liboracle.so).
 * A clean-room restatement of the reference host path; see oracle.c for the pinning story.
 * Suffix _s = float (the reference as shipped), _d = double (the reference built with
 * -Dfloat=double). Tile task types follow enum Type {QRS, SAPP, QRD, DAPP}
 * (reference include/gridscheduler.h:10).
 */
#ifndef TQR_ORACLE_H
#define TQR_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_QRS = 0, ORACLE_SAPP = 1, ORACLE_QRD = 2, ORACLE_DAPP = 3 };

void oracle_geqrt_s(float* blk, float* tau, int m, int n, int ldm, float* w);
void oracle_unmqr_s(float* C, const float* V, const float* tau, int m, int n, int ldm);
void oracle_tsqrt_s(float* A, float* B, float* tau, int ma, int mb, int n, int ldm, float* hh);
void oracle_tsmqr_s(const float* V, float* A, float* B, const float* tau, int b, int n, int ldm);
void oracle_do_task_s(int type, int l, int m, int k, float* mat, float* tau, int b, int ldm, float* w);
void oracle_factor_serial_s(const float* A, float* R, float* tau, int m, int n, int b, int ldm);
void oracle_factor_threads_s(const float* A, float* R, float* tau, int m, int n, int b, int ldm, int nthreads);
void oracle_randzo_s(float* A, int m, int n, int ldm, unsigned seed);

void oracle_geqrt_d(double* blk, double* tau, int m, int n, int ldm, double* w);
void oracle_unmqr_d(double* C, const double* V, const double* tau, int m, int n, int ldm);
void oracle_tsqrt_d(double* A, double* B, double* tau, int ma, int mb, int n, int ldm, double* hh);
void oracle_tsmqr_d(const double* V, double* A, double* B, const double* tau, int b, int n, int ldm);
void oracle_do_task_d(int type, int l, int m, int k, double* mat, double* tau, int b, int ldm, double* w);
void oracle_factor_serial_d(const double* A, double* R, double* tau, int m, int n, int b, int ldm);
void oracle_factor_threads_d(const double* A, double* R, double* tau, int m, int n, int b, int ldm, int nthreads);
void oracle_randzo_d(double* A, int m, int n, int ldm, unsigned seed);

double oracle_residual_d(const double* A, const double* F, const double* tau, int m, int n, int b, int ldm);

#ifdef __cplusplus
}
#endif
#endif
