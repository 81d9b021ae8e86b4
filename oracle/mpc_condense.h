/*
 * oracle/mpc_condense.h — TEST INFRASTRUCTURE ONLY (CPU checker, never shipped).
 *
 * Plain-C restatement of the condensed QP construction in LukeSchmitt96/solveMPC
 * (src/ModelPredictiveControlAPI.cpp:111-375, include/ModelPredictiveControlAPI.h:26-32,148-200).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 *
 * Parity status: pinned against the known-answer values recorded in SURVEY.md Appendix B
 * (produced by a survey-time probe build of the reference); the reference itself is
 * unbuildable in this image (needs OsqpEigen and Eigen's unsupported/MatrixFunctions,
 * both absent) — see DESIGN.md §Oracle.
 *
 * All matrices are row-major fp64.
 */
#ifndef ORACLE_MPC_CONDENSE_H
#define ORACLE_MPC_CONDENSE_H

#ifdef __cplusplus
extern "C" {
#endif

/* Plant + weights as read from config/MPC_API.json (SISO, n_x = 4 in the reference). */
typedef struct {
    int nx;            /* number of states (reference: N_S = 4, ModelPredictiveControlAPI.h:28) */
    int N;             /* horizon (reference: mpcWindow = 15, ModelPredictiveControlAPI.h:26) */
    int s_rows;        /* rows of S filled with K (reference hard-codes 10, :185) */
    const double *Ad;  /* nx*nx */
    const double *Bd;  /* nx */
    const double *Cd;  /* nx */
    const double *K;   /* nx  (row gain, :16) */
    double Q, R, RD;   /* 1x1 weights (:138-140) */
} ora_plant;

/* Outputs of the condensing (caller allocates):
 *   P   N*N     Hessian (setH :247-263, symmetrised)
 *   A   2N*N    Gbar (setLinearConstraints :326-347)
 *   Fx  N*nx    (setFVars :307)
 *   Fu  N       (setFVars :305, incl. the .diagonal() quirk)
 *   Fr  N*N     (setFVars :306)
 *   Sbar 2N*nx  (setTransformations :185,208; rows >= s_rows of S are zero)
 *   Ku  2N      (setUpperBound :364-366)
 *   W0  2N      (setUpperBound :368)
 *   Su  N*N     (setTransformations :197-204; strict upper triangle zero)
 *   Sx  N*nx    (setTransformations :189)
 */
typedef struct {
    double *P, *A, *Fx, *Fu, *Fr, *Sbar, *Ku, *W0, *Su, *Sx;
} ora_qp_ops;

/* Build all operators. Returns 0 on success. */
int ora_condense(const ora_plant *pl, ora_qp_ops *out);

/* q = Fx*X + Fu*U + Fr*ref' (setF :372-375); ref = xref * ones (updateRef :378-380). */
void ora_gradient(const ora_plant *pl, const ora_qp_ops *ops, const double *X, double U,
                  double xref, double *q);

/* u = W0 + Sbar*X + Ku*U (:43, :99). l = -DBL_MAX (:42). */
void ora_upper_bound(const ora_plant *pl, const ora_qp_ops *ops, const double *X, double U,
                     double *u);

/* Integer matrix power by binary powering (Eigen MatrixPower::computeIntPower order). */
void ora_matpow(int nx, const double *A, int p, double *out);

#ifdef __cplusplus
}
#endif
#endif
