/*
 * oracle/mpc_mimo.h — TEST INFRASTRUCTURE ONLY (CPU checker / CPU baseline, never shipped).
 *
 * Multi-input multi-output generalisation of the reference's condensed-QP construction
 * (src/ModelPredictiveControlAPI.cpp:111-375), for BASELINE config 4 (quad-rotor, n_x 12, n_u 4,
 * N 30).  The reference is SISO only (K(0) scalar :335,364; .diagonal() :305; Sbar with 4 columns,
 * ModelPredictiveControlAPI.h:160), so this formulation has no reference counterpart: every scalar
 * of the SISO code becomes a block, in the same expression order, and the SISO specialisation
 * (n_u = n_y = 1, K0 = K(0), w0 = 255) reproduces ora_condense (tests/test_oracle.py).  Its parity
 * is against this restatement (SURVEY.md §7 "MIMO quad-rotor").
 *
 * Decision variable: du, N blocks of n_u (n = N n_u).  Outputs y_k = Cd x_k (n_y each).
 *   CAB[k]   = Cd Ad^k Bd                                   (n_y x n_u)
 *   Su(i, j) = sum_{k <= i-j} CAB[k] for j <= i, else 0      (block lower-triangular, :195-204)
 *   Sx(i)    = Cd Ad^(i+1)                                  (:189)
 *   LL       = L (x) I_nu,  Qbar = I_N (x) Q, Rbar = I_N (x) R, RDbar = I_N (x) RD
 *   P        = sym(2 (LL' Rbar LL + RDbar + Su' Qbar Su))     (:250-251)
 *   Fu       = 2 (diagblocks(LL' Rbar') + (Su1' Qbar Su)')   (n x n_u; Su1 = first block column;
 *                                                              the .diagonal() quirk of :305 as blocks)
 *   Fr       = -2 (Qbar Su)'                                (n x N n_y, :306)
 *   Fx       = 2 (Sx' Qbar Su)'                             (n x n_x, :307)
 *   A        = [L (x) K0; -(L (x) K0)]                      (m = 2 n rows, :332-347)
 *   Sbar     = [S; -S], S block rows k < s_rows = K         (m x n_x, :185,208)
 *   Ku       = [-(1 (x) K0); 1 (x) K0]                       (m x n_u, :364-366)
 *   W0       = 1_2N (x) w0                                   (:368)
 *   q = Fx X + Fu U + Fr (1_N (x) yref),  u = W0 + Sbar X + Ku U,  l = -DBL_MAX.
 * All matrices row-major fp64.
 */
#ifndef ORACLE_MPC_MIMO_H
#define ORACLE_MPC_MIMO_H

#include "osqp_dense.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int nx, nu, ny, N, s_rows;
    const double *Ad, *Bd, *Cd;  /* nx*nx, nx*nu, ny*nx */
    const double *Q, *R, *RD;    /* ny*ny, nu*nu, nu*nu */
    const double *K, *K0;        /* nu*nx, nu*nu */
    const double *w0;            /* nu */
} ora_mimo_plant;

/* Caller-allocated outputs (n = N nu, m = 2n): P n*n, A m*n, Fx n*nx, Fu n*nu, Fr n*(N ny),
 * Sbar m*nx, Ku m*nu, W0 m, Su (N ny)*n. */
typedef struct {
    double *P, *A, *Fx, *Fu, *Fr, *Sbar, *Ku, *W0, *Su;
} ora_mimo_ops;

int ora_condense_mimo(const ora_mimo_plant *pl, ora_mimo_ops *o);
void ora_mimo_gradient(const ora_mimo_plant *pl, const ora_mimo_ops *o, const double *X, const double *U,
                       const double *yref, double *q);
void ora_mimo_upper_bound(const ora_mimo_plant *pl, const ora_mimo_ops *o, const double *X, const double *U,
                          double *u);

/* Per-plant batch (BASELINE config 4): plant p has its own Ad[p], Bd[p]; Cd, Q, R, RD, K, K0, w0 are
 * shared.  For each plant: condense, osqp setup with the ctor's data (q0 = 0, l = -DBL_MAX, u0 = W0),
 * one controllerStep from (X[p], U[p]) (U[p] += x[0:nu] when solved).  OpenMP over plants.
 * margin (nullable): each plant's decision margin (ora_info.margin).
 * Returns the number of plants whose setup failed. */
int ora_mimo_plants_step(int n_plants, int nx, int nu, int ny, int N, int s_rows, const double *Ad,
                         const double *Bd, const double *Cd, const double *Q, const double *R,
                         const double *RD, const double *K, const double *K0, const double *w0,
                         const double *X, const double *U, const double *yref, const ora_settings *s,
                         double *U_out, double *x_out, int *status, int *iters, int nthreads,
                         double *margin);

#ifdef __cplusplus
}
#endif
#endif
