/*
 * oracle/osqp_dense.c — TEST INFRASTRUCTURE ONLY (CPU checker / cpu_baseline, never shipped).
 *
 * Dense fp64 restatement of OSQP v0.6's ADMM as used by LukeSchmitt96/solveMPC
 * (src/ModelPredictiveControlAPI.cpp:51-64 setup, :96-105 per step).  Function names
 * follow OSQP's (osqp.c / auxil.c / scaling.c / qdldl_interface.c) so that each block can
 * be read against the published algorithm.  PARITY UNPINNED (no OSQP here, no reference
 * tests): certified by KKT conditions in tests/test_oracle.py.  See osqp_dense.h.
 */
#include "osqp_dense.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* osqp constants.h (v0.6) */
#define OSQP_INFTY 1e30
#define MIN_SCALING 1e-4
#define MAX_SCALING 1e4
#define RHO_MIN 1e-6
#define RHO_MAX 1e6
#define RHO_TOL 1e-4
#define RHO_EQ_OVER_RHO_INEQ 1e3
#define OSQP_DIVISION_TOL (1.0 / OSQP_INFTY)
#define ADAPTIVE_RHO_MULTIPLE_TERMINATION 4
#define ADAPTIVE_RHO_FIXED 100

struct ora_work {
    int n, m, K; /* K = n + m */
    ora_settings set;
    ora_info info;
    size_t nbuf;
    double *buf; /* every double array lives in buf (makes ora_clone a memcpy) */
    int *constr_type;
    /* views into buf */
    double *P, *A, *q, *l, *u;
    double *D, *Dinv, *E, *Einv, *sc; /* sc[0] = c, sc[1] = cinv */
    double *rho_vec, *rho_inv_vec;
    double *x, *y, *z, *xz_tilde, *x_prev, *z_prev;
    double *Ax, *Px, *Aty, *delta_y, *Atdelta_y, *delta_x, *Pdelta_x, *Adelta_x;
    double *D_temp, *D_temp_A, *E_temp;
    double *L, *Ld, *sol; /* dense LDL' of the KKT matrix */
    double *sol_x, *sol_y;
};

static void bind_views(ora_work *w)
{
    const int n = w->n, m = w->m, K = w->K;
    double *p = w->buf;
#define TAKE(f, cnt) do { w->f = p; p += (cnt); } while (0)
    TAKE(P, n * n); TAKE(A, m * n); TAKE(q, n); TAKE(l, m); TAKE(u, m);
    TAKE(D, n); TAKE(Dinv, n); TAKE(E, m); TAKE(Einv, m); TAKE(sc, 2);
    TAKE(rho_vec, m); TAKE(rho_inv_vec, m);
    TAKE(x, n); TAKE(y, m); TAKE(z, m); TAKE(xz_tilde, K); TAKE(x_prev, n); TAKE(z_prev, m);
    TAKE(Ax, m); TAKE(Px, n); TAKE(Aty, n); TAKE(delta_y, m); TAKE(Atdelta_y, n);
    TAKE(delta_x, n); TAKE(Pdelta_x, n); TAKE(Adelta_x, m);
    TAKE(D_temp, n); TAKE(D_temp_A, n); TAKE(E_temp, m);
    TAKE(L, K * K); TAKE(Ld, K); TAKE(sol, K);
    TAKE(sol_x, n); TAKE(sol_y, m);
#undef TAKE
    w->nbuf = (size_t)(p - w->buf);
}

static size_t buf_len(int n, int m)
{
    int K = n + m;
    return (size_t)n * n + (size_t)m * n + n + 2 * m + 2 * n + 2 * m + 2 + 2 * m + n + 2 * m +
           K + n + m + m + n + n + m + n + n + n + m + n + n + m + (size_t)K * K + K + K + n + m;
}

void ora_default_settings(ora_settings *s)
{
    /* osqp constants.h defaults; osqp-eigen setWarmStart(true) at :52 */
    s->rho = 0.1;
    s->sigma = 1e-6;
    s->alpha = 1.6;
    s->eps_abs = 1e-3;
    s->eps_rel = 1e-3;
    s->eps_prim_inf = 1e-4;
    s->eps_dual_inf = 1e-4;
    s->adaptive_rho_tolerance = 5.0;
    s->adaptive_rho_fraction = 0.4;
    s->max_iter = 4000;
    s->check_termination = 25;
    s->scaling = 10;
    s->adaptive_rho = 1;
    s->adaptive_rho_interval = 0;
    s->warm_start = 1;
    s->scaled_termination = 0;
}

/* ---------------------------------------------------------------- lin_alg helpers */
static double norm_inf(const double *v, int n)
{
    double r = 0.0;
    for (int i = 0; i < n; i++) r = fmax(r, fabs(v[i]));
    return r;
}
static double scaled_norm_inf(const double *s, const double *v, int n)
{
    double r = 0.0;
    for (int i = 0; i < n; i++) r = fmax(r, fabs(s[i] * v[i]));
    return r;
}
static void mat_vec(const double *M, int r, int c, const double *x, double *y)
{
    for (int i = 0; i < r; i++) {
        double s = 0.0;
        for (int j = 0; j < c; j++) s += M[i * c + j] * x[j];
        y[i] = s;
    }
}
static void mat_tpose_vec(const double *M, int r, int c, const double *x, double *y)
{
    for (int j = 0; j < c; j++) y[j] = 0.0;
    for (int i = 0; i < r; i++)
        for (int j = 0; j < c; j++) y[j] += M[i * c + j] * x[i];
}
static void limit_scaling(double *d, int n)
{
    for (int i = 0; i < n; i++) {
        d[i] = d[i] < MIN_SCALING ? 1.0 : d[i];
        d[i] = d[i] > MAX_SCALING ? MAX_SCALING : d[i];
    }
}

/* ---------------------------------------------------------------- scaling.c */
static void scale_data(ora_work *w)
{
    const int n = w->n, m = w->m;
    w->sc[0] = 1.0;
    for (int i = 0; i < n; i++) w->D[i] = w->Dinv[i] = 1.0;
    for (int i = 0; i < m; i++) w->E[i] = w->Einv[i] = 1.0;
    for (int it = 0; it < w->set.scaling; it++) {
        /* compute_inf_norm_cols_KKT: [P; A] columns and A' columns (= rows of A) */
        for (int j = 0; j < n; j++) {
            double a = 0.0, b = 0.0;
            for (int i = 0; i < n; i++) a = fmax(a, fabs(w->P[i * n + j]));
            for (int i = 0; i < m; i++) b = fmax(b, fabs(w->A[i * n + j]));
            w->D_temp[j] = fmax(a, b);
        }
        for (int i = 0; i < m; i++) {
            double b = 0.0;
            for (int j = 0; j < n; j++) b = fmax(b, fabs(w->A[i * n + j]));
            w->E_temp[i] = b;
        }
        limit_scaling(w->D_temp, n);
        limit_scaling(w->E_temp, m);
        for (int j = 0; j < n; j++) w->D_temp[j] = 1.0 / sqrt(w->D_temp[j]);
        for (int i = 0; i < m; i++) w->E_temp[i] = 1.0 / sqrt(w->E_temp[i]);
        /* P <- D P D ; A <- E A D ; q <- D q */
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) w->P[i * n + j] *= w->D_temp[i] * w->D_temp[j];
        for (int i = 0; i < m; i++)
            for (int j = 0; j < n; j++) w->A[i * n + j] *= w->E_temp[i] * w->D_temp[j];
        for (int j = 0; j < n; j++) w->q[j] *= w->D_temp[j];
        for (int j = 0; j < n; j++) w->D[j] *= w->D_temp[j];
        for (int i = 0; i < m; i++) w->E[i] *= w->E_temp[i];
        /* cost normalisation: c_temp = 1 / max(mean col-norm(P), max(|q|) or 1 if ~0) */
        double mean = 0.0;
        for (int j = 0; j < n; j++) {
            double a = 0.0;
            for (int i = 0; i < n; i++) a = fmax(a, fabs(w->P[i * n + j]));
            mean += a;
        }
        mean /= n;
        double inf_norm_q = norm_inf(w->q, n);
        limit_scaling(&inf_norm_q, 1);
        double c_temp = fmax(mean, inf_norm_q);
        limit_scaling(&c_temp, 1);
        c_temp = 1.0 / c_temp;
        for (int i = 0; i < n * n; i++) w->P[i] *= c_temp;
        for (int j = 0; j < n; j++) w->q[j] *= c_temp;
        w->sc[0] *= c_temp;
    }
    w->sc[1] = 1.0 / w->sc[0];
    for (int j = 0; j < n; j++) w->Dinv[j] = 1.0 / w->D[j];
    for (int i = 0; i < m; i++) w->Einv[i] = 1.0 / w->E[i];
    for (int i = 0; i < m; i++) {
        w->l[i] *= w->E[i];
        w->u[i] *= w->E[i];
    }
}

/* ---------------------------------------------------------------- lin_sys (dense LDL') */
static void kkt_factor(ora_work *w)
{
    const int n = w->n, m = w->m, K = w->K;
    double *L = w->L, *Ld = w->Ld;
    /* assemble lower triangle of KKT = [P + sigma I, A'; A, -diag(1/rho)] into L */
    memset(L, 0, sizeof(double) * K * K);
    for (int i = 0; i < n; i++)
        for (int j = 0; j <= i; j++) L[i * K + j] = w->P[i * n + j] + (i == j ? w->set.sigma : 0.0);
    for (int i = 0; i < m; i++) {
        for (int j = 0; j < n; j++) L[(n + i) * K + j] = w->A[i * n + j];
        L[(n + i) * K + n + i] = -w->rho_inv_vec[i];
    }
    /* right-looking LDL' without pivoting (quasi-definite => exists for any order) */
    for (int j = 0; j < K; j++) {
        double d = L[j * K + j];
        for (int k = 0; k < j; k++) d -= L[j * K + k] * L[j * K + k] * Ld[k];
        Ld[j] = d;
        for (int i = j + 1; i < K; i++) {
            double s = L[i * K + j];
            for (int k = 0; k < j; k++) s -= L[i * K + k] * L[j * K + k] * Ld[k];
            L[i * K + j] = s / d;
        }
        L[j * K + j] = 1.0;
    }
}

/* solve_linsys_qdldl (non-polish): sol = KKT^{-1} b; b[0:n] = sol[0:n];
 * b[n+j] += rho_inv[j] * sol[n+j]. */
static void kkt_solve(ora_work *w, double *b)
{
    const int n = w->n, m = w->m, K = w->K;
    double *s = w->sol, *L = w->L;
    memcpy(s, b, sizeof(double) * K);
    for (int i = 0; i < K; i++) {
        double t = s[i];
        for (int k = 0; k < i; k++) t -= L[i * K + k] * s[k];
        s[i] = t;
    }
    for (int i = 0; i < K; i++) s[i] /= w->Ld[i];
    for (int i = K - 1; i >= 0; i--) {
        double t = s[i];
        for (int k = i + 1; k < K; k++) t -= L[k * K + i] * s[k];
        s[i] = t;
    }
    for (int j = 0; j < n; j++) b[j] = s[j];
    for (int j = 0; j < m; j++) b[n + j] += w->rho_inv_vec[j] * s[n + j];
}

/* ---------------------------------------------------------------- auxil.c */
static void set_rho_vec(ora_work *w)
{
    w->set.rho = fmin(fmax(w->set.rho, RHO_MIN), RHO_MAX);
    for (int i = 0; i < w->m; i++) {
        if (w->l[i] < -OSQP_INFTY * MIN_SCALING && w->u[i] > OSQP_INFTY * MIN_SCALING) {
            w->constr_type[i] = -1;
            w->rho_vec[i] = RHO_MIN;
        } else if (w->u[i] - w->l[i] < RHO_TOL) {
            w->constr_type[i] = 1;
            w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->set.rho;
        } else {
            w->constr_type[i] = 0;
            w->rho_vec[i] = w->set.rho;
        }
        w->rho_inv_vec[i] = 1.0 / w->rho_vec[i];
    }
}

static int update_rho_vec(ora_work *w)
{
    int changed = 0;
    for (int i = 0; i < w->m; i++) {
        if (w->l[i] < -OSQP_INFTY * MIN_SCALING && w->u[i] > OSQP_INFTY * MIN_SCALING) {
            if (w->constr_type[i] != -1) {
                w->constr_type[i] = -1;
                w->rho_vec[i] = RHO_MIN;
                w->rho_inv_vec[i] = 1.0 / RHO_MIN;
                changed = 1;
            }
        } else if (w->u[i] - w->l[i] < RHO_TOL) {
            if (w->constr_type[i] != 1) {
                w->constr_type[i] = 1;
                w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->set.rho;
                w->rho_inv_vec[i] = 1.0 / w->rho_vec[i];
                changed = 1;
            }
        } else {
            if (w->constr_type[i] != 0) {
                w->constr_type[i] = 0;
                w->rho_vec[i] = w->set.rho;
                w->rho_inv_vec[i] = 1.0 / w->set.rho;
                changed = 1;
            }
        }
    }
    if (changed) kkt_factor(w);
    return 0;
}

static void update_xz_tilde(ora_work *w)
{
    const int n = w->n, m = w->m;
    for (int i = 0; i < n; i++) w->xz_tilde[i] = w->set.sigma * w->x_prev[i] - w->q[i];
    for (int i = 0; i < m; i++) w->xz_tilde[n + i] = w->z_prev[i] - w->rho_inv_vec[i] * w->y[i];
    kkt_solve(w, w->xz_tilde);
}

static void update_x(ora_work *w)
{
    const double a = w->set.alpha;
    for (int i = 0; i < w->n; i++) w->x[i] = a * w->xz_tilde[i] + (1.0 - a) * w->x_prev[i];
    for (int i = 0; i < w->n; i++) w->delta_x[i] = w->x[i] - w->x_prev[i];
}

static void update_z(ora_work *w)
{
    const double a = w->set.alpha;
    const int n = w->n;
    for (int i = 0; i < w->m; i++) {
        double v = a * w->xz_tilde[n + i] + (1.0 - a) * w->z_prev[i] + w->rho_inv_vec[i] * w->y[i];
        /* project(): z = min(max(z, l), u) */
        w->z[i] = fmin(fmax(v, w->l[i]), w->u[i]);
    }
}

static void update_y(ora_work *w)
{
    const double a = w->set.alpha;
    const int n = w->n;
    for (int i = 0; i < w->m; i++) {
        w->delta_y[i] = w->rho_vec[i] *
                        (a * w->xz_tilde[n + i] + (1.0 - a) * w->z_prev[i] - w->z[i]);
        w->y[i] += w->delta_y[i];
    }
}

/* compute_pri_res: z_prev <- Ax - z (working vector), returns ||Einv (Ax - z)|| */
static double compute_pri_res(ora_work *w)
{
    mat_vec(w->A, w->m, w->n, w->x, w->Ax);
    for (int i = 0; i < w->m; i++) w->z_prev[i] = w->Ax[i] - w->z[i];
    if (w->set.scaling && !w->set.scaled_termination)
        return scaled_norm_inf(w->Einv, w->z_prev, w->m);
    return norm_inf(w->z_prev, w->m);
}

static double compute_pri_tol(ora_work *w, double eps_abs, double eps_rel)
{
    double mx;
    if (w->set.scaling && !w->set.scaled_termination)
        mx = fmax(scaled_norm_inf(w->Einv, w->z, w->m), scaled_norm_inf(w->Einv, w->Ax, w->m));
    else
        mx = fmax(norm_inf(w->z, w->m), norm_inf(w->Ax, w->m));
    return eps_abs + eps_rel * mx;
}

/* compute_dua_res: x_prev <- q + P x + A' y (working vector) */
static double compute_dua_res(ora_work *w)
{
    const int n = w->n;
    mat_vec(w->P, n, n, w->x, w->Px);
    for (int i = 0; i < n; i++) w->x_prev[i] = w->q[i] + w->Px[i];
    if (w->m > 0) {
        mat_tpose_vec(w->A, w->m, n, w->y, w->Aty);
        for (int i = 0; i < n; i++) w->x_prev[i] += w->Aty[i];
    }
    if (w->set.scaling && !w->set.scaled_termination)
        return w->sc[1] * scaled_norm_inf(w->Dinv, w->x_prev, n);
    return norm_inf(w->x_prev, n);
}

static double compute_dua_tol(ora_work *w, double eps_abs, double eps_rel)
{
    double mx;
    if (w->set.scaling && !w->set.scaled_termination) {
        mx = scaled_norm_inf(w->Dinv, w->q, w->n);
        mx = fmax(mx, scaled_norm_inf(w->Dinv, w->Aty, w->n));
        mx = fmax(mx, scaled_norm_inf(w->Dinv, w->Px, w->n));
        mx *= w->sc[1];
    } else {
        mx = fmax(fmax(norm_inf(w->q, w->n), norm_inf(w->Aty, w->n)), norm_inf(w->Px, w->n));
    }
    return eps_abs + eps_rel * mx;
}

static void update_info(ora_work *w, int iter)
{
    w->info.iter = iter;
    w->info.pri_res = w->m ? compute_pri_res(w) : 0.0;
    w->info.dua_res = compute_dua_res(w);
}

static int is_primal_infeasible(ora_work *w, double eps)
{
    const int m = w->m;
    for (int i = 0; i < m; i++) {
        if (w->u[i] > OSQP_INFTY * MIN_SCALING) {
            if (w->l[i] < -OSQP_INFTY * MIN_SCALING) w->delta_y[i] = 0.0;
            else w->delta_y[i] = fmin(w->delta_y[i], 0.0);
        } else if (w->l[i] < -OSQP_INFTY * MIN_SCALING) {
            w->delta_y[i] = fmax(w->delta_y[i], 0.0);
        }
    }
    double ndy;
    if (w->set.scaling && !w->set.scaled_termination) {
        for (int i = 0; i < m; i++) w->Adelta_x[i] = w->E[i] * w->delta_y[i];
        ndy = norm_inf(w->Adelta_x, m);
    } else {
        ndy = norm_inf(w->delta_y, m);
    }
    if (ndy > OSQP_DIVISION_TOL) {
        double lhs = 0.0;
        for (int i = 0; i < m; i++)
            lhs += w->u[i] * fmax(w->delta_y[i], 0.0) + w->l[i] * fmin(w->delta_y[i], 0.0);
        if (lhs < eps * ndy) {
            mat_tpose_vec(w->A, m, w->n, w->delta_y, w->Atdelta_y);
            if (w->set.scaling && !w->set.scaled_termination)
                for (int j = 0; j < w->n; j++) w->Atdelta_y[j] *= w->Dinv[j];
            return norm_inf(w->Atdelta_y, w->n) < eps * ndy;
        }
    }
    return 0;
}

static int is_dual_infeasible(ora_work *w, double eps)
{
    const int n = w->n, m = w->m;
    double ndx, cs;
    if (w->set.scaling && !w->set.scaled_termination) {
        ndx = scaled_norm_inf(w->D, w->delta_x, n);
        cs = w->sc[0];
    } else {
        ndx = norm_inf(w->delta_x, n);
        cs = 1.0;
    }
    if (ndx > OSQP_DIVISION_TOL) {
        double qdx = 0.0;
        for (int j = 0; j < n; j++) qdx += w->q[j] * w->delta_x[j];
        if (qdx < -cs * eps * ndx) {
            mat_vec(w->P, n, n, w->delta_x, w->Pdelta_x);
            if (w->set.scaling && !w->set.scaled_termination)
                for (int j = 0; j < n; j++) w->Pdelta_x[j] *= w->Dinv[j];
            if (norm_inf(w->Pdelta_x, n) < cs * eps * ndx) {
                mat_vec(w->A, m, n, w->delta_x, w->Adelta_x);
                if (w->set.scaling && !w->set.scaled_termination)
                    for (int i = 0; i < m; i++) w->Adelta_x[i] *= w->Einv[i];
                for (int i = 0; i < m; i++) {
                    if ((w->u[i] < OSQP_INFTY * MIN_SCALING && w->Adelta_x[i] > eps * ndx) ||
                        (w->l[i] > -OSQP_INFTY * MIN_SCALING && w->Adelta_x[i] < -eps * ndx))
                        return 0;
                }
                return 1;
            }
        }
    }
    return 0;
}

/* decision margin (diagnostics only): |ln(value / threshold)| of one comparison */
static double log_margin(double v, double thr)
{
    return (v > 0 && thr > 0) ? fabs(log(v / thr)) : INFINITY;
}
static void note_margin(ora_work *w, double r)
{
    if (r < w->info.margin) w->info.margin = r;
}

static int check_termination(ora_work *w, int approximate)
{
    double eps_abs = w->set.eps_abs, eps_rel = w->set.eps_rel;
    double eps_pinf = w->set.eps_prim_inf, eps_dinf = w->set.eps_dual_inf;
    int prim_ok = 0, dual_ok = 0, prim_inf = 0, dual_inf = 0;
    double mp = INFINITY;
    if (w->info.pri_res > OSQP_INFTY || w->info.dua_res > OSQP_INFTY) {
        w->info.status = ORA_NON_CVX;
        return 1;
    }
    if (approximate) {
        eps_abs *= 10; eps_rel *= 10; eps_pinf *= 10; eps_dinf *= 10;
    }
    if (w->m == 0) {
        prim_ok = 1;
    } else {
        double ep = compute_pri_tol(w, eps_abs, eps_rel);
        mp = log_margin(w->info.pri_res, ep);
        if (w->info.pri_res < ep) prim_ok = 1;
        else prim_inf = is_primal_infeasible(w, eps_pinf);
    }
    double ed = compute_dua_tol(w, eps_abs, eps_rel);
    if (w->info.dua_res < ed) dual_ok = 1;
    else dual_inf = is_dual_infeasible(w, eps_dinf);
    if (!approximate) {  /* the solved test flips only when every failing comparison flips */
        const double md = log_margin(w->info.dua_res, ed);
        if (prim_ok && dual_ok) note_margin(w, fmin(mp, md));
        else note_margin(w, fmax(prim_ok ? 0.0 : mp, dual_ok ? 0.0 : md));
    }

    if (prim_ok && dual_ok) {
        w->info.status = approximate ? ORA_SOLVED_INACCURATE : ORA_SOLVED;
        return 1;
    }
    if (prim_inf) {
        w->info.status = approximate ? ORA_PRIMAL_INFEASIBLE_INACCURATE : ORA_PRIMAL_INFEASIBLE;
        if (w->set.scaling && !w->set.scaled_termination)
            for (int i = 0; i < w->m; i++) w->delta_y[i] *= w->E[i];
        return 1;
    }
    if (dual_inf) {
        w->info.status = approximate ? ORA_DUAL_INFEASIBLE_INACCURATE : ORA_DUAL_INFEASIBLE;
        if (w->set.scaling && !w->set.scaled_termination) {
            for (int j = 0; j < w->n; j++) w->delta_x[j] *= w->D[j];
        }
        return 1;
    }
    return 0;
}

static double compute_rho_estimate(ora_work *w)
{
    const int n = w->n, m = w->m;
    double pri = norm_inf(w->z_prev, m);
    double dua = norm_inf(w->x_prev, n);
    double pn = fmax(norm_inf(w->z, m), norm_inf(w->Ax, m));
    pri /= (pn + OSQP_DIVISION_TOL);
    double dn = fmax(norm_inf(w->q, n), norm_inf(w->Aty, n));
    dn = fmax(dn, norm_inf(w->Px, n));
    dua /= (dn + OSQP_DIVISION_TOL);
    double r = w->set.rho * sqrt(pri / (dua + OSQP_DIVISION_TOL));
    return fmin(fmax(r, RHO_MIN), RHO_MAX);
}

static int osqp_update_rho(ora_work *w, double rho_new)
{
    if (rho_new <= 0) return 1;
    w->set.rho = fmin(fmax(rho_new, RHO_MIN), RHO_MAX);
    for (int i = 0; i < w->m; i++) {
        if (w->constr_type[i] == 0) {
            w->rho_vec[i] = w->set.rho;
            w->rho_inv_vec[i] = 1.0 / w->set.rho;
        } else if (w->constr_type[i] == 1) {
            w->rho_vec[i] = RHO_EQ_OVER_RHO_INEQ * w->set.rho;
            w->rho_inv_vec[i] = 1.0 / w->rho_vec[i];
        }
    }
    kkt_factor(w);
    return 0;
}

static int adapt_rho(ora_work *w)
{
    double rho_new = compute_rho_estimate(w);
    w->info.rho_estimate = rho_new;
    note_margin(w, fmin(log_margin(rho_new, w->set.rho * w->set.adaptive_rho_tolerance),
                        log_margin(rho_new, w->set.rho / w->set.adaptive_rho_tolerance)));
    if (rho_new > w->set.rho * w->set.adaptive_rho_tolerance ||
        rho_new < w->set.rho / w->set.adaptive_rho_tolerance) {
        int e = osqp_update_rho(w, rho_new);
        w->info.rho_updates += 1;
        return e;
    }
    return 0;
}

static int has_solution(int st)
{
    return st != ORA_PRIMAL_INFEASIBLE && st != ORA_PRIMAL_INFEASIBLE_INACCURATE &&
           st != ORA_DUAL_INFEASIBLE && st != ORA_DUAL_INFEASIBLE_INACCURATE && st != ORA_NON_CVX;
}

void ora_cold_start(ora_work *w)
{
    memset(w->x, 0, sizeof(double) * w->n);
    memset(w->z, 0, sizeof(double) * w->m);
    memset(w->y, 0, sizeof(double) * w->m);
}

static void store_solution(ora_work *w)
{
    if (has_solution(w->info.status)) {
        for (int j = 0; j < w->n; j++) w->sol_x[j] = w->x[j];
        for (int i = 0; i < w->m; i++) w->sol_y[i] = w->y[i];
        if (w->set.scaling) {
            for (int j = 0; j < w->n; j++) w->sol_x[j] *= w->D[j];
            for (int i = 0; i < w->m; i++) w->sol_y[i] *= w->E[i] * w->sc[1];
        }
    } else {
        for (int j = 0; j < w->n; j++) w->sol_x[j] = NAN;
        for (int i = 0; i < w->m; i++) w->sol_y[i] = NAN;
        ora_cold_start(w);
    }
}

static void swap(double **a, double **b)
{
    double *t = *a;
    *a = *b;
    *b = t;
}

int ora_solve(ora_work *w)
{
    int iter, can_check = 0;
    w->info.margin = INFINITY;
    if (!w->set.warm_start) ora_cold_start(w);
    for (iter = 1; iter <= w->set.max_iter; iter++) {
        swap(&w->x, &w->x_prev);
        swap(&w->z, &w->z_prev);
        update_xz_tilde(w);
        update_x(w);
        update_z(w);
        update_y(w);
        can_check = w->set.check_termination && (iter % w->set.check_termination == 0);
        if (can_check) {
            update_info(w, iter);
            if (check_termination(w, 0)) break;
        }
        if (w->set.adaptive_rho && !w->set.adaptive_rho_interval) {
            w->set.adaptive_rho_interval = w->set.check_termination
                                               ? ADAPTIVE_RHO_MULTIPLE_TERMINATION * w->set.check_termination
                                               : ADAPTIVE_RHO_FIXED;
        }
        if (w->set.adaptive_rho && w->set.adaptive_rho_interval &&
            iter % w->set.adaptive_rho_interval == 0) {
            update_info(w, iter);
            if (adapt_rho(w)) return 1;
        }
    }
    if (!can_check) {
        update_info(w, iter - 1);
        check_termination(w, 0);
    }
    if (w->info.status == ORA_UNSOLVED) {
        if (!check_termination(w, 1)) w->info.status = ORA_MAX_ITER_REACHED;
    }
    w->info.rho_estimate = compute_rho_estimate(w);
    store_solution(w);
    return 0;
}

/* ---------------------------------------------------------------- setup / updates */
ora_work *ora_setup(int n, int m, const double *P, const double *q, const double *A,
                    const double *l, const double *u, const ora_settings *s)
{
    if (n <= 0 || m < 0 || !P || !q || (m && (!A || !l || !u)) || !s) return NULL;
    for (int i = 0; i < m; i++)
        if (l[i] > u[i]) return NULL; /* validate_data */
    if (s->rho <= 0 || s->sigma <= 0 || s->alpha <= 0 || s->alpha >= 2 || s->max_iter <= 0 ||
        s->eps_abs < 0 || s->eps_rel < 0 || (s->eps_abs == 0 && s->eps_rel == 0) ||
        s->scaling < 0 || s->check_termination < 0 || s->adaptive_rho_tolerance < 1)
        return NULL; /* validate_settings */
    ora_work *w = calloc(1, sizeof(ora_work));
    w->n = n;
    w->m = m;
    w->K = n + m;
    w->set = *s;
    w->buf = calloc(buf_len(n, m), sizeof(double));
    w->constr_type = calloc(m ? m : 1, sizeof(int));
    bind_views(w);
    /* osqp-eigen keeps only triangularView<Upper>() of the Hessian; mirror it */
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) w->P[i * n + j] = w->P[j * n + i] = P[i * n + j];
    memcpy(w->q, q, sizeof(double) * n);
    if (m) {
        memcpy(w->A, A, sizeof(double) * m * n);
        memcpy(w->l, l, sizeof(double) * m);
        memcpy(w->u, u, sizeof(double) * m);
    }
    if (w->set.scaling) {
        scale_data(w);
    } else {
        w->sc[0] = w->sc[1] = 1.0;
        for (int j = 0; j < n; j++) w->D[j] = w->Dinv[j] = 1.0;
        for (int i = 0; i < m; i++) w->E[i] = w->Einv[i] = 1.0;
    }
    set_rho_vec(w);
    kkt_factor(w);
    w->info.status = ORA_UNSOLVED;
    w->info.iter = 0;
    w->info.rho_updates = 0;
    return w;
}

/* ora_solve swaps x/x_prev and z/z_prev pointers; keep the same slots in a copy */
static void rebase_swapped(ora_work *w, const ora_work *src)
{
    w->x = w->buf + (src->x - src->buf);
    w->x_prev = w->buf + (src->x_prev - src->buf);
    w->z = w->buf + (src->z - src->buf);
    w->z_prev = w->buf + (src->z_prev - src->buf);
}

ora_work *ora_clone(const ora_work *src)
{
    ora_work *w = malloc(sizeof(ora_work));
    *w = *src;
    w->buf = malloc(sizeof(double) * src->nbuf);
    memcpy(w->buf, src->buf, sizeof(double) * src->nbuf);
    w->constr_type = malloc(sizeof(int) * (src->m ? src->m : 1));
    memcpy(w->constr_type, src->constr_type, sizeof(int) * (src->m ? src->m : 1));
    bind_views(w);
    rebase_swapped(w, src);
    return w;
}

static void restore_from(ora_work *w, const ora_work *src)
{
    /* keep w's own buffers, copy all state (x/x_prev swaps are undone by re-binding) */
    double *b = w->buf;
    int *ct = w->constr_type;
    *w = *src;
    w->buf = b;
    w->constr_type = ct;
    memcpy(w->buf, src->buf, sizeof(double) * src->nbuf);
    memcpy(w->constr_type, src->constr_type, sizeof(int) * (src->m ? src->m : 1));
    bind_views(w);
    rebase_swapped(w, src);
}

void ora_cleanup(ora_work *w)
{
    if (!w) return;
    free(w->buf);
    free(w->constr_type);
    free(w);
}

int ora_update_lin_cost(ora_work *w, const double *q)
{
    for (int j = 0; j < w->n; j++) w->q[j] = q[j];
    if (w->set.scaling)
        for (int j = 0; j < w->n; j++) w->q[j] *= w->D[j] * w->sc[0];
    w->info.status = ORA_UNSOLVED;
    w->info.rho_updates = 0;
    return 0;
}

int ora_update_upper_bound(ora_work *w, const double *u)
{
    for (int i = 0; i < w->m; i++) w->u[i] = u[i];
    if (w->set.scaling)
        for (int i = 0; i < w->m; i++) w->u[i] *= w->E[i];
    for (int i = 0; i < w->m; i++)
        if (w->u[i] < w->l[i]) return 1;
    w->info.status = ORA_UNSOLVED;
    w->info.rho_updates = 0;
    return update_rho_vec(w);
}

int ora_update_lower_bound(ora_work *w, const double *l)
{
    for (int i = 0; i < w->m; i++) w->l[i] = l[i];
    if (w->set.scaling)
        for (int i = 0; i < w->m; i++) w->l[i] *= w->E[i];
    for (int i = 0; i < w->m; i++)
        if (w->l[i] > w->u[i]) return 1;
    w->info.status = ORA_UNSOLVED;
    w->info.rho_updates = 0;
    return update_rho_vec(w);
}

int ora_update_bounds(ora_work *w, const double *l, const double *u)
{
    for (int i = 0; i < w->m; i++)
        if (l[i] > u[i]) return 1;
    for (int i = 0; i < w->m; i++) {
        w->l[i] = l[i];
        w->u[i] = u[i];
    }
    if (w->set.scaling)
        for (int i = 0; i < w->m; i++) {
            w->l[i] *= w->E[i];
            w->u[i] *= w->E[i];
        }
    w->info.status = ORA_UNSOLVED;
    w->info.rho_updates = 0;
    return update_rho_vec(w);
}

int ora_warm_start(ora_work *w, const double *x, const double *y)
{
    for (int j = 0; j < w->n; j++) w->x[j] = x[j] * (w->set.scaling ? w->Dinv[j] : 1.0);
    for (int i = 0; i < w->m; i++)
        w->y[i] = y[i] * (w->set.scaling ? w->Einv[i] * w->sc[0] : 1.0);
    mat_vec(w->A, w->m, w->n, w->x, w->z);
    return 0;
}

const double *ora_solution_x(const ora_work *w) { return w->sol_x; }
const double *ora_solution_y(const ora_work *w) { return w->sol_y; }

void ora_get_info(const ora_work *w, ora_info *info)
{
    *info = w->info;
    info->rho = w->set.rho;
}

void ora_get_scaling(const ora_work *w, double *D, double *E, double *c)
{
    if (D) memcpy(D, w->D, sizeof(double) * w->n);
    if (E) memcpy(E, w->E, sizeof(double) * w->m);
    if (c) *c = w->sc[0];
}

void ora_get_iterates(const ora_work *w, double *x, double *z, double *y)
{
    if (x) memcpy(x, w->x, sizeof(double) * w->n);
    if (z) memcpy(z, w->z, sizeof(double) * w->m);
    if (y) memcpy(y, w->y, sizeof(double) * w->m);
}

int ora_batch_solve(int n, int m, const double *P, const double *A, const double *q0,
                    const double *l, const double *u0, const ora_settings *s, int batch,
                    const double *q, const double *u, double *x, int *status, int *iters,
                    double *rho_out, int nthreads, double *margin_out)
{
    ora_work *tmpl = ora_setup(n, m, P, q0, A, l, u0, s);
    if (!tmpl) return -1;
    int failed = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(+ : failed)
#endif
    {
        ora_work *w = ora_clone(tmpl);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
        for (int b = 0; b < batch; b++) {
            restore_from(w, tmpl);
            int e = ora_update_lin_cost(w, q + (size_t)b * n);
            e |= ora_update_upper_bound(w, u + (size_t)b * m);
            if (e) {
                failed++;
                for (int j = 0; j < n; j++) x[(size_t)b * n + j] = NAN;
                if (status) status[b] = ORA_UNSOLVED;
                if (iters) iters[b] = 0;
                continue;
            }
            ora_solve(w);
            memcpy(x + (size_t)b * n, w->sol_x, sizeof(double) * n);
            if (status) status[b] = w->info.status;
            if (iters) iters[b] = w->info.iter;
            if (rho_out) rho_out[b] = w->set.rho;
            if (margin_out) margin_out[b] = w->info.margin;
        }
        ora_cleanup(w);
    }
    (void)nthreads;
    ora_cleanup(tmpl);
    return failed;
}
