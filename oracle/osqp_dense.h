/*
 * oracle/osqp_dense.h — TEST INFRASTRUCTURE ONLY (CPU checker / cpu_baseline, never shipped).
 *
 * Dense fp64 restatement of the OSQP v0.6 ADMM solver (oxfordcontrol/osqp, C, unpinned
 * `master` cloned by /root/reference/README.md:17-38; dated Oct 2020 => v0.6.x API) as driven
 * through osqp-eigen by LukeSchmitt96/solveMPC src/ModelPredictiveControlAPI.cpp:51-64
 * (setup) and :96-105 (per step).  Neither library is in /root/reference nor installed in
 * this image, so the restatement follows OSQP's published algorithm (Stellato et al.,
 * "OSQP: an operator splitting solver for quadratic programs", Math. Prog. Comp. 2020) and
 * the v0.6 source structure (osqp.c / auxil.c / scaling.c / lin_sys qdldl) as recalled.
 *
 * PARITY UNPINNED at this boundary: the reference has no tests or fixtures that pin OSQP's
 * output.  The restatement is instead certified by KKT optimality conditions at tight
 * tolerance (tests/test_oracle.py) — see DESIGN.md §Oracle.
 *
 * Differences from OSQP that change only rounding, never the iteration semantics:
 *   - dense storage; the quasi-definite KKT [P+sI A'; A -1/rho] is factored LDL' in natural
 *     order (QDLDL uses an AMD permutation);
 *   - adaptive_rho_interval == 0 resolves to 4*check_termination (OSQP's non-PROFILING rule;
 *     the PROFILING build times setup, which is not reproducible).
 */
#ifndef ORACLE_OSQP_DENSE_H
#define ORACLE_OSQP_DENSE_H

#ifdef __cplusplus
extern "C" {
#endif

/* OSQP status values (osqp constants.h) */
#define ORA_SOLVED 1
#define ORA_SOLVED_INACCURATE 2
#define ORA_MAX_ITER_REACHED (-2)
#define ORA_PRIMAL_INFEASIBLE (-3)
#define ORA_PRIMAL_INFEASIBLE_INACCURATE 3
#define ORA_DUAL_INFEASIBLE (-4)
#define ORA_DUAL_INFEASIBLE_INACCURATE 4
#define ORA_NON_CVX (-7)
#define ORA_UNSOLVED (-10)

typedef struct {
    double rho, sigma, alpha;
    double eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
    double adaptive_rho_tolerance, adaptive_rho_fraction;
    int max_iter, check_termination, scaling, adaptive_rho, adaptive_rho_interval;
    int warm_start, scaled_termination;
} ora_settings;

typedef struct {
    int iter, status, rho_updates;
    double pri_res, dua_res, rho_estimate, rho;
    /* smallest |ln(value / threshold)| over this solve's decisions (termination tests and
     * adaptive-rho tests): how far the iteration schedule is from flipping (test diagnostics) */
    double margin;
} ora_info;

typedef struct ora_work ora_work;

void ora_default_settings(ora_settings *s);

/* osqp_setup: P is n*n row-major; only its upper triangle is read (osqp-eigen passes
 * triangularView<Upper>).  A is m*n row-major.  Returns NULL on invalid data. */
ora_work *ora_setup(int n, int m, const double *P, const double *q, const double *A,
                    const double *l, const double *u, const ora_settings *s);
ora_work *ora_clone(const ora_work *w);
void ora_cleanup(ora_work *w);

int ora_update_lin_cost(ora_work *w, const double *q);        /* osqp_update_lin_cost */
int ora_update_upper_bound(ora_work *w, const double *u);     /* osqp_update_upper_bound */
int ora_update_lower_bound(ora_work *w, const double *l);     /* osqp_update_lower_bound */
int ora_update_bounds(ora_work *w, const double *l, const double *u);
int ora_warm_start(ora_work *w, const double *x, const double *y);
void ora_cold_start(ora_work *w);
int ora_solve(ora_work *w);                                    /* osqp_solve */

const double *ora_solution_x(const ora_work *w);               /* unscaled x (D x) */
const double *ora_solution_y(const ora_work *w);               /* unscaled y (E y / c) */
void ora_get_info(const ora_work *w, ora_info *info);
/* Scaling used by setup: D (n), E (m), c. */
void ora_get_scaling(const ora_work *w, double *D, double *E, double *c);
/* Scaled iterates (x n, z m, y m) — for trajectory-parity tests. */
void ora_get_iterates(const ora_work *w, double *x, double *z, double *y);

/* Batch driver used by tests and bench.py's cpu_baseline: one shared (P, A, l, setup q0/u0)
 * template; for every QP b: fresh copy of the template, update_lin_cost(q[b]),
 * update_upper_bound(u[b]), solve.  Writes x (batch*n), status, iter, final rho, decision margin
 * (each output may be NULL except x).
 * nthreads <= 0 => OpenMP default.  Returns the number of QPs whose update failed. */
int ora_batch_solve(int n, int m, const double *P, const double *A, const double *q0,
                    const double *l, const double *u0, const ora_settings *s, int batch,
                    const double *q, const double *u, double *x, int *status, int *iters,
                    double *rho_out, int nthreads, double *margin_out);

#ifdef __cplusplus
}
#endif
#endif
