/*
 * oracle/mpc_batch.c — TEST INFRASTRUCTURE ONLY (CPU checker / CPU baseline, never shipped).
 *
 * Per-plant batches (BASELINE config 3) on the CPU: for every plant, the reference constructor
 * (condensing, ModelPredictiveControlAPI.cpp:3-65, with X = U = 0 setup data) followed by one
 * controllerStep (:81-108): q, u from (X, U), solve, U += x[0] when solved.  OpenMP over plants.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 */
#include <float.h>
#include <math.h>
#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif
#include <stdint.h>
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

/* The simulated plant's noise (mpcq_plant_sim.h, workload.plant_noise): SplitMix64 of (seed, global QP
 * index, draw), Box-Muller pairs from draws step*64 + 2p, 2p + 1. */
static uint64_t sm64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double uni01(uint64_t key, uint64_t idx, uint64_t d)
{
    const uint64_t x = sm64(key ^ (idx * 0x100000001B3ull + d * 0xD6E8FEB86659FD93ull));
    return ((double)(x >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}

int ora_stream_run(int batch, int nx, int N, int s_rows, const double *Ad, const double *Bd, const double *Cd,
                   const double *K, double Q, double R, double RD, double *X, double *U, double xref,
                   const ora_settings *s, int steps, unsigned long long seed, long long first_qp,
                   long long first_step, double noise_std, int *it_total, int *unsolved, int nthreads)
{
    const int n = N, m = 2 * N;
    if (N < 1 || N > 64 || nx < 1 || nx > 8) return -2; /* the per-thread q[64], u[128], xn[8] below */
    double *buf = (double *)malloc(sizeof(double) * (size_t)(5 * N * N + 4 * N * nx + 16 * N + 8 * m));
    double *P = buf, *A = P + N * N, *Fx = A + 2 * N * N, *Fu = Fx + N * nx, *Fr = Fu + N;
    double *Sbar = Fr + N * N, *Ku = Sbar + 2 * N * nx, *W0 = Ku + 2 * N, *Su = W0 + 2 * N;
    double *Sx = Su + N * N, *l = Sx + N * nx, *q0 = l + m;
    ora_qp_ops ops = {P, A, Fx, Fu, Fr, Sbar, Ku, W0, Su, Sx};
    for (int j = 0; j < m; j++) l[j] = -DBL_MAX;
    for (int j = 0; j < n; j++) q0[j] = 0.0;
    const ora_plant pl = {nx, N, s_rows, Ad, Bd, Cd, K, Q, R, RD};
    ora_work *tmpl = NULL;
    if (ora_condense(&pl, &ops) == 0) tmpl = ora_setup(n, m, P, q0, A, l, W0, s);
    if (!tmpl) {
        free(buf);
        return -1;
    }
    const uint64_t key = sm64((uint64_t)seed * 0x632BE59BD9B4E019ull + 1ull);
    const int np = (nx + 1) / 2;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
    {
        double q[64], u[128], xn[8];
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int b = 0; b < batch; b++) {
            ora_work *w = ora_clone(tmpl);  /* one warm-started solver per plant, as the reference keeps */
            double *x = X + (size_t)b * nx;
            int its = 0, uns = 0;
            for (int k = 0; k < steps; k++) {
                ora_gradient(&pl, &ops, x, U[b], xref, q);
                ora_upper_bound(&pl, &ops, x, U[b], u);
                ora_update_lin_cost(w, q);
                ora_update_upper_bound(w, u);
                ora_solve(w);
                ora_info info;
                ora_get_info(w, &info);
                its += info.iter;
                if (info.status == ORA_SOLVED) U[b] += ora_solution_x(w)[0];
                else uns++;
                const unsigned long long step = (unsigned long long)(first_step + k);
                for (int i = 0; i < nx; i++) {
                    double a = 0.0;
                    for (int t = 0; t < nx; t++) a += Ad[i * nx + t] * x[t];
                    a += Bd[i] * U[b];
                    if (noise_std != 0.0) {
                        const int pp = i < np ? i : i - np;
                        const uint64_t d0 = step * 64ull + 2ull * (uint64_t)pp, idx = (uint64_t)(first_qp + b);
                        const double r = sqrt(-2.0 * log(uni01(key, idx, d0)));
                        const double th = 2.0 * M_PI * uni01(key, idx, d0 + 1);
                        a += noise_std * (i < np ? r * cos(th) : r * sin(th));
                    }
                    xn[i] = a;
                }
                for (int i = 0; i < nx; i++) x[i] = xn[i];
            }
            if (it_total) it_total[b] = its;
            if (unsolved) unsolved[b] = uns;
            ora_cleanup(w);
        }
    }
    (void)nthreads;
    ora_cleanup(tmpl);
    free(buf);
    return 0;
}
