/*
 * oracle/mpc_mimo.c — TEST INFRASTRUCTURE ONLY (CPU checker / CPU baseline, never shipped).
 *
 * MIMO condensing (see mpc_mimo.h for the formulation): the SISO code of mpc_condense.c with
 * every scalar a block, computed in the same expression order (mm() sums in k order), so the
 * n_u = n_y = 1 case is ora_condense's arithmetic (ModelPredictiveControlAPI.cpp:180-369).
 */
#include "mpc_mimo.h"

#include <float.h>
#include <stdlib.h>
#include <string.h>

#include "mpc_condense.h"

#ifdef _OPENMP
#include <omp.h>
#endif

static void mm(int r, int k, int c, const double *A, const double *B, double *C)
{
    for (int i = 0; i < r; i++)
        for (int j = 0; j < c; j++) {
            double s = 0.0;
            for (int t = 0; t < k; t++) s += A[(size_t)i * k + t] * B[(size_t)t * c + j];
            C[(size_t)i * c + j] = s;
        }
}

static void transpose(int r, int c, const double *A, double *At)
{
    for (int i = 0; i < r; i++)
        for (int j = 0; j < c; j++) At[(size_t)j * r + i] = A[(size_t)i * c + j];
}

int ora_condense_mimo(const ora_mimo_plant *pl, ora_mimo_ops *o)
{
    const int N = pl->N, nx = pl->nx, nu = pl->nu, ny = pl->ny;
    if (N <= 0 || nx <= 0 || nu <= 0 || ny <= 0) return -1;
    const int n = N * nu, m = 2 * n, Ny = N * ny;
    double *Apow = malloc(sizeof(double) * nx * nx);
    double *CA = malloc(sizeof(double) * ny * nx);
    double *CAB = malloc(sizeof(double) * (size_t)N * ny * nu);
    double *Sx = malloc(sizeof(double) * (size_t)Ny * nx);
    double *LL = calloc((size_t)n * n, sizeof(double)), *LLT = malloc(sizeof(double) * (size_t)n * n);
    double *Rb = calloc((size_t)n * n, sizeof(double)), *RbT = calloc((size_t)n * n, sizeof(double));
    double *Qb = calloc((size_t)Ny * Ny, sizeof(double));
    double *T1 = malloc(sizeof(double) * (size_t)n * n), *T2 = malloc(sizeof(double) * (size_t)n * n);
    double *T1t = malloc(sizeof(double) * (size_t)n * n);
    double *SuT = malloc(sizeof(double) * (size_t)n * Ny), *T3 = malloc(sizeof(double) * (size_t)n * Ny);
    double *T4 = malloc(sizeof(double) * (size_t)n * n), *H1 = malloc(sizeof(double) * (size_t)n * n);
    double *QS = malloc(sizeof(double) * (size_t)Ny * n);
    double *SxT = malloc(sizeof(double) * (size_t)nx * Ny), *T5 = malloc(sizeof(double) * (size_t)nx * Ny);
    double *T6 = malloc(sizeof(double) * (size_t)nx * n);

    /* setTransformations :187-194 — Sx(i) = Cd Ad^(i+1); CAB[i] = (Cd Ad^i) Bd */
    for (int i = 0; i < N; i++) {
        ora_matpow(nx, pl->Ad, i + 1, Apow);
        mm(ny, nx, nx, pl->Cd, Apow, Sx + (size_t)i * ny * nx);
        ora_matpow(nx, pl->Ad, i, Apow);
        mm(ny, nx, nx, pl->Cd, Apow, CA);
        mm(ny, nx, nu, CA, pl->Bd, CAB + (size_t)i * ny * nu);
    }
    /* :197-204 — Su(i, j) = sum_{k <= i-j} CAB[k] (element-wise, k order); zero above */
    memset(o->Su, 0, sizeof(double) * (size_t)Ny * n);
    for (int i = 0; i < N; i++)
        for (int j = 0; j <= i; j++)
            for (int r = 0; r < ny; r++)
                for (int c = 0; c < nu; c++) {
                    double s = 0.0;
                    for (int k = 0; k <= i - j; k++) s += CAB[((size_t)k * ny + r) * nu + c];
                    o->Su[((size_t)i * ny + r) * n + (size_t)j * nu + c] = s;
                }
    /* :185,208 — S block rows k < s_rows = K, the rest 0; Sbar = [S; -S] */
    memset(o->Sbar, 0, sizeof(double) * (size_t)m * nx);
    const int srows = pl->s_rows < N ? pl->s_rows : N;
    for (int k = 0; k < srows; k++)
        for (int r = 0; r < nu; r++)
            for (int c = 0; c < nx; c++) {
                o->Sbar[((size_t)k * nu + r) * nx + c] = pl->K[r * nx + c];
                o->Sbar[((size_t)n + k * nu + r) * nx + c] = -pl->K[r * nx + c];
            }
    /* setLL :292 — L (x) I_nu;  setLiftedCosts :160-162 — block-diagonal Qbar, Rbar */
    for (int i = 0; i < N; i++)
        for (int j = 0; j <= i; j++)
            for (int c = 0; c < nu; c++) LL[((size_t)i * nu + c) * n + (size_t)j * nu + c] = 1.0;
    for (int b = 0; b < N; b++) {
        for (int r = 0; r < nu; r++)
            for (int c = 0; c < nu; c++) {
                Rb[((size_t)b * nu + r) * n + (size_t)b * nu + c] = pl->R[r * nu + c];
                RbT[((size_t)b * nu + r) * n + (size_t)b * nu + c] = pl->R[c * nu + r];
            }
        for (int r = 0; r < ny; r++)
            for (int c = 0; c < ny; c++) Qb[((size_t)b * ny + r) * Ny + (size_t)b * ny + c] = pl->Q[r * ny + c];
    }

    /* setH :250-251 — H1 = 2 (LL' Rbar LL + RDbar + Su' Qbar Su); P = (H1 + H1') / 2 */
    transpose(n, n, LL, LLT);
    transpose(Ny, n, o->Su, SuT);
    mm(n, n, n, LLT, Rb, T1);    /* LL' Rbar */
    mm(n, n, n, T1, LL, T2);     /* (LL' Rbar) LL */
    mm(n, Ny, Ny, SuT, Qb, T3);  /* Su' Qbar */
    mm(n, Ny, n, T3, o->Su, T4); /* (Su' Qbar) Su */
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            const int bi = i / nu, bj = j / nu;
            const double rd = bi == bj ? pl->RD[(i % nu) * nu + (j % nu)] : 0.0;
            H1[(size_t)i * n + j] = 2.0 * (T2[(size_t)i * n + j] + rd + T4[(size_t)i * n + j]);
        }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++)
            o->P[(size_t)i * n + j] = (H1[(size_t)i * n + j] + H1[(size_t)j * n + i]) / 2.0;

    /* setFVars :305 — Fu = 2 (diagblocks(LL' Rbar') + (Su1' Qbar Su)');  Su1 = Su(:, 0:nu) */
    mm(n, n, n, LLT, RbT, T1t);  /* LL' Rbar' */
    for (int i = 0; i < n; i++)
        for (int c = 0; c < nu; c++) {
            double s = 0.0;  /* (Su1' Qbar Su)(c, i) = sum_k (Su' Qbar)(c, k) Su(k, i) */
            for (int k = 0; k < Ny; k++) s += T3[(size_t)c * Ny + k] * o->Su[(size_t)k * n + i];
            const double d = T1t[(size_t)i * n + (size_t)(i / nu) * nu + c];
            o->Fu[(size_t)i * nu + c] = 2.0 * (d + s);
        }
    /* :306 — Fr = -2 (Qbar Su)' */
    mm(Ny, Ny, n, Qb, o->Su, QS);
    for (int i = 0; i < n; i++)
        for (int t = 0; t < Ny; t++) o->Fr[(size_t)i * Ny + t] = -2.0 * QS[(size_t)t * n + i];
    /* :307 — Fx = 2 (Sx' Qbar Su)' */
    transpose(Ny, nx, Sx, SxT);
    mm(nx, Ny, Ny, SxT, Qb, T5);
    mm(nx, Ny, n, T5, o->Su, T6);
    for (int i = 0; i < n; i++)
        for (int c = 0; c < nx; c++) o->Fx[(size_t)i * nx + c] = 2.0 * T6[(size_t)c * n + i];

    /* setLinearConstraints :332-335 — Gbar = [L (x) K0; L (x) (-K0)] */
    for (int k = 0; k < N; k++)
        for (int r = 0; r < nu; r++)
            for (int j = 0; j < N; j++)
                for (int c = 0; c < nu; c++) {
                    const double v = (j <= k) ? 1.0 : 0.0;
                    const double k0 = pl->K0[r * nu + c];
                    o->A[((size_t)k * nu + r) * n + (size_t)j * nu + c] = v * k0;
                    o->A[((size_t)n + k * nu + r) * n + (size_t)j * nu + c] = v * -k0;
                }
    /* setUpperBound :364-368 — Ku = [-(1 (x) K0); 1 (x) K0], W0 = 1 (x) w0 */
    for (int k = 0; k < N; k++)
        for (int r = 0; r < nu; r++)
            for (int c = 0; c < nu; c++) {
                o->Ku[((size_t)k * nu + r) * nu + c] = -pl->K0[r * nu + c];
                o->Ku[((size_t)n + k * nu + r) * nu + c] = pl->K0[r * nu + c];
            }
    for (int k = 0; k < 2 * N; k++)
        for (int r = 0; r < nu; r++) o->W0[(size_t)k * nu + r] = pl->w0[r];

    free(Apow); free(CA); free(CAB); free(Sx); free(LL); free(LLT); free(Rb); free(RbT); free(Qb);
    free(T1); free(T2); free(T1t); free(SuT); free(T3); free(T4); free(H1); free(QS); free(SxT);
    free(T5); free(T6);
    return 0;
}

void ora_mimo_gradient(const ora_mimo_plant *pl, const ora_mimo_ops *o, const double *X, const double *U,
                       const double *yref, double *q)
{
    const int N = pl->N, nx = pl->nx, nu = pl->nu, ny = pl->ny, n = N * nu, Ny = N * ny;
    for (int i = 0; i < n; i++) {
        double a = 0.0, b = 0.0, c = 0.0;
        for (int t = 0; t < nx; t++) a += o->Fx[(size_t)i * nx + t] * X[t];
        for (int t = 0; t < nu; t++) b += o->Fu[(size_t)i * nu + t] * U[t];
        for (int t = 0; t < Ny; t++) c += o->Fr[(size_t)i * Ny + t] * yref[t % ny];
        q[i] = a + b + c;
    }
}

void ora_mimo_upper_bound(const ora_mimo_plant *pl, const ora_mimo_ops *o, const double *X, const double *U,
                          double *u)
{
    const int nx = pl->nx, nu = pl->nu, m = 2 * pl->N * nu;
    for (int i = 0; i < m; i++) {
        double s = 0.0, k = 0.0;
        for (int t = 0; t < nx; t++) s += o->Sbar[(size_t)i * nx + t] * X[t];
        for (int t = 0; t < nu; t++) k += o->Ku[(size_t)i * nu + t] * U[t];
        u[i] = o->W0[i] + s + k;
    }
}

int ora_mimo_plants_step(int n_plants, int nx, int nu, int ny, int N, int s_rows, const double *Ad,
                         const double *Bd, const double *Cd, const double *Q, const double *R,
                         const double *RD, const double *K, const double *K0, const double *w0,
                         const double *X, const double *U, const double *yref, const ora_settings *s,
                         double *U_out, double *x_out, int *status, int *iters, int nthreads,
                         double *margin)
{
    int failed = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(+ : failed)
#endif
    {
        const int n = N * nu, m = 2 * n, Ny = N * ny;
        const size_t tot = (size_t)n * n + (size_t)m * n + (size_t)n * nx + (size_t)n * nu + (size_t)n * Ny +
                           (size_t)m * nx + (size_t)m * nu + m + (size_t)Ny * n + 2 * (size_t)n + 2 * (size_t)m;
        double *buf = (double *)malloc(sizeof(double) * tot);
        ora_mimo_ops o;
        double *p = buf;
        o.P = p; p += (size_t)n * n;
        o.A = p; p += (size_t)m * n;
        o.Fx = p; p += (size_t)n * nx;
        o.Fu = p; p += (size_t)n * nu;
        o.Fr = p; p += (size_t)n * Ny;
        o.Sbar = p; p += (size_t)m * nx;
        o.Ku = p; p += (size_t)m * nu;
        o.W0 = p; p += m;
        o.Su = p; p += (size_t)Ny * n;
        double *q = p, *q0 = q + n, *u = q0 + n, *l = u + m;
        for (int j = 0; j < m; j++) l[j] = -DBL_MAX;
        for (int j = 0; j < n; j++) q0[j] = 0.0;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int pp = 0; pp < n_plants; pp++) {
            ora_mimo_plant pl = {nx, nu, ny, N, s_rows, Ad + (size_t)pp * nx * nx, Bd + (size_t)pp * nx * nu,
                                 Cd, Q, R, RD, K, K0, w0};
            ora_work *w = NULL;
            if (ora_condense_mimo(&pl, &o) == 0) w = ora_setup(n, m, o.P, q0, o.A, l, o.W0, s);
            for (int c = 0; c < nu; c++) U_out[(size_t)pp * nu + c] = U[(size_t)pp * nu + c];
            if (!w) {
                failed++;
                status[pp] = ORA_UNSOLVED;
                iters[pp] = 0;
                continue;
            }
            ora_mimo_gradient(&pl, &o, X + (size_t)pp * nx, U + (size_t)pp * nu, yref, q);
            ora_mimo_upper_bound(&pl, &o, X + (size_t)pp * nx, U + (size_t)pp * nu, u);
            ora_update_lin_cost(w, q);
            ora_update_upper_bound(w, u);
            ora_solve(w);
            ora_info info;
            ora_get_info(w, &info);
            status[pp] = info.status;
            iters[pp] = info.iter;
            if (margin) margin[pp] = info.margin;
            const double *x = ora_solution_x(w);
            if (x_out)
                for (int i = 0; i < n; i++) x_out[(size_t)pp * n + i] = x[i];
            if (info.status == ORA_SOLVED)
                for (int c = 0; c < nu; c++) U_out[(size_t)pp * nu + c] = U[(size_t)pp * nu + c] + x[c];
            ora_cleanup(w);
        }
        free(buf);
    }
    (void)nthreads;
    return failed;
}
