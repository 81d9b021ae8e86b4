/*
 * oracle/mpc_batch.c — TEST INFRASTRUCTURE ONLY (CPU checker / CPU baseline, never shipped).
 *
 * Per-plant batches (BASELINE config 3) on the CPU: for every plant, the reference constructor
 * (condensing, ModelPredictiveControlAPI.cpp:3-65, with X = U = 0 setup data) followed by one
 * controllerStep (:81-108): q, u from (X, U), solve, U += x[0] when solved.  OpenMP over plants.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 */
#include <float.h>
#include <stdlib.h>

#include "mpc_batch.h"

#ifdef _OPENMP
#include <omp.h>
#endif

int ora_plants_step(int n_plants, int nx, int N, int s_rows, const double *Ad, const double *Bd,
                    const double *Cd, const double *K, double Q, double R, double RD, const double *X,
                    const double *U, double xref, const ora_settings *s, double *U_out, int *status,
                    int *iters, int nthreads, double *x_out, double *margin)
{
    int failed = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(+ : failed)
#endif
    {
        const int n = N, m = 2 * N;
        double *buf = (double *)malloc(sizeof(double) * (size_t)(5 * N * N + 2 * N * nx + 2 * N * nx + 16 * N + 8 * m));
        double *P = buf, *A = P + N * N, *Fx = A + 2 * N * N, *Fu = Fx + N * nx, *Fr = Fu + N;
        double *Sbar = Fr + N * N, *Ku = Sbar + 2 * N * nx, *W0 = Ku + 2 * N, *Su = W0 + 2 * N;
        double *Sx = Su + N * N, *q = Sx + N * nx, *u = q + n, *l = u + m, *q0 = l + m;
        ora_qp_ops ops = {P, A, Fx, Fu, Fr, Sbar, Ku, W0, Su, Sx};
        for (int j = 0; j < m; j++) l[j] = -DBL_MAX;
        for (int j = 0; j < n; j++) q0[j] = 0.0;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
        for (int p = 0; p < n_plants; p++) {
            ora_plant pl = {nx, N, s_rows, Ad + (size_t)p * nx * nx, Bd + (size_t)p * nx, Cd, K, Q, R, RD};
            ora_work *w = NULL;
            if (ora_condense(&pl, &ops) == 0) w = ora_setup(n, m, P, q0, A, l, W0, s);
            U_out[p] = U[p];
            if (!w) {
                failed++;
                status[p] = ORA_UNSOLVED;
                iters[p] = 0;
                continue;
            }
            ora_gradient(&pl, &ops, X + (size_t)p * nx, U[p], xref, q);
            ora_upper_bound(&pl, &ops, X + (size_t)p * nx, U[p], u);
            ora_update_lin_cost(w, q);
            ora_update_upper_bound(w, u);
            ora_solve(w);
            ora_info info;
            ora_get_info(w, &info);
            status[p] = info.status;
            iters[p] = info.iter;
            if (margin) margin[p] = info.margin;
            if (x_out)
                for (int j = 0; j < n; j++) x_out[(size_t)p * n + j] = ora_solution_x(w)[j];
            if (info.status == ORA_SOLVED) U_out[p] = U[p] + ora_solution_x(w)[0];
            ora_cleanup(w);
        }
        free(buf);
    }
    (void)nthreads;
    return failed;
}
