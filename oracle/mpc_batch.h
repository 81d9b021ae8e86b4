/*
 * oracle/mpc_batch.h — TEST INFRASTRUCTURE ONLY (CPU checker / CPU baseline, never shipped).
 * Per-plant condense + setup + one controllerStep (ModelPredictiveControlAPI.cpp:3-65,81-108).
 */
#ifndef ORACLE_MPC_BATCH_H
#define ORACLE_MPC_BATCH_H
#include "mpc_condense.h"
#include "osqp_dense.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Plants p = 0..n_plants-1 with their own Ad (nx*nx), Bd (nx); shared Cd, K, Q, R, RD.
 * X n_plants*nx, U n_plants -> U_out (U + x[0] when solved), status, iters.  Returns failures. */
int ora_plants_step(int n_plants, int nx, int N, int s_rows, const double *Ad, const double *Bd,
                    const double *Cd, const double *K, double Q, double R, double RD, const double *X,
                    const double *U, double xref, const ora_settings *s, double *U_out, int *status,
                    int *iters, int nthreads, double *x_out, double *margin);

/* The receding-horizon stream (BASELINE config 5) on the CPU: `batch` copies of one plant (Ad, Bd, Cd, K,
 * Q, R, RD), each with its own warm-started solver, `steps` control steps of [controllerStep; plant
 * update X <- Ad X + Bd U + w] (the device's noise stream).  X (batch*nx), U (batch) evolve in place;
 * per plant the iterations summed over the steps and the steps that did not end SOLVED.
 * Returns -1 when setup fails. */
int ora_stream_run(int batch, int nx, int N, int s_rows, const double *Ad, const double *Bd, const double *Cd,
                   const double *K, double Q, double R, double RD, double *X, double *U, double xref,
                   const ora_settings *s, int steps, unsigned long long seed, long long first_qp,
                   long long first_step, double noise_std, int *it_total, int *unsolved, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
