// solvempc_amd/csrc/mpcq_admm.h — the per-plant path: batched OSQP-v0.6 ADMM on gfx950.
//
// Replaces osqp_solve behind OsqpEigen::Solver::solve (ModelPredictiveControlAPI.cpp:102), plus the
// per-step updates around it (updateGradient :96 -> osqp_update_lin_cost, updateUpperBound :99 ->
// osqp_update_upper_bound, getSolution :105) and, in the MPC front end, setF (:372-375),
// setUpperBound (:360-369) and the receding-horizon U += x0 (:105).
//
// Mapping (MI355X-first): ONE QP PER LANE.  A 64-lane wave carries 64 independent QPs of one plant;
// the plant operators (W, sigma W'W, B = A^W, ...; see mpcq_internal.h) are identical for every
// lane, so with a shared plant they are wave-uniform scalar-memory operands (s_load into SGPRs,
// one v_fma per matrix entry per lane) and the per-QP iterate x' (n), z (m), y (m) lives in VGPRs.
// No cross-lane traffic, no LDS broadcast, no barriers.  Per-QP constants that are read every
// iteration (scaled upper/lower bounds) sit in LDS in a [row][lane] layout (conflict-free).
//
// Iteration (OSQP osqp.c / auxil.c, in the W-basis x^ = W x'):
//   w      = rho_j z_j - y_j                                   (rhs_z of compute_rhs, times rho)
//   xi     = -W'q^ + sigma W'W x' + B' w                       (W' * KKT rhs)
//   eta    = xi / (1 + rho lambda)                             (M(rho)^-1 in the W-basis)
//   x'     = alpha eta + (1-alpha) x'                          (update_x)
//   zt_j   = b_j . eta                                         (z~ = A^ x~)
//   z_j    = Pi_[l,u](alpha zt_j + (1-alpha) z_j + y_j/rho_j)  (update_z)
//   y_j   += rho_j (alpha zt_j + (1-alpha) z_j_prev - z_j)     (update_y)
// every check_termination iterations: OSQP update_info / check_termination / adapt_rho.
#pragma once
#include "mpcq_internal.h"

#include <math.h>

namespace mpcq {


template <typename T> __device__ __forceinline__ T tfma(T a, T b, T c);
template <> __device__ __forceinline__ float tfma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
template <> __device__ __forceinline__ double tfma(double a, double b, double c) { return __builtin_fma(a, b, c); }
template <typename T> __device__ __forceinline__ T tabs(T a) { return a < T(0) ? -a : a; }
template <typename T> __device__ __forceinline__ T tmax(T a, T b) { return a > b ? a : b; }
template <typename T> __device__ __forceinline__ T tmin(T a, T b) { return a < b ? a : b; }

// ---------------------------------------------------------------------------------------------
// Cold-path certificates (OSQP is_primal_infeasible / is_dual_infeasible).  They run only when a
// residual test fails, so they read everything from global scratch (current iterate written by
// the caller, snapshot taken before the iteration) with rolled loops: no register arrays.
template <typename T, int NC, int MC>
__device__ bool primal_infeasible(const AdmmArgs<T> &a, const PlantOps<T> &op, const T *uh,
                                  const T *lh, int b, T eps, bool scaled)
{
    // lh == nullptr: every lower bound is -inf (LFREE kernel variant)
    auto dyj = [&](int j) -> T {  // delta_y projected onto the polar of the recession cone of [l,u]
        T d = a.ys[b * MC + j] - a.snap_y[b * MC + j];
        const T up = uh[j * 64], lo = lh ? lh[j * 64] : T(-kInfty);
        const bool uinf = up > T(kInfty * kMinScaling), linf = lo < T(-kInfty * kMinScaling);
        if (uinf) d = linf ? T(0) : tmin(d, T(0));
        else if (linf) d = tmax(d, T(0));
        return d;
    };
    T ndy = 0, lhs = 0;
#pragma unroll 1
    for (int j = 0; j < MC; j++) {
        const T d = dyj(j);
        ndy = tmax(ndy, tabs(scaled ? d : op.E[j] * d));
        const T up = uh[j * 64], lo = lh ? lh[j * 64] : T(-kInfty);
        if (up < T(kInfty * kMinScaling)) lhs += up * tmax(d, T(0));
        if (lo > T(-kInfty * kMinScaling)) lhs += lo * tmin(d, T(0));
    }
    if (!(ndy > T(kDivisionTol))) return false;
    if (!(lhs < eps * ndy)) return false;
    T nat = 0;
#pragma unroll 1
    for (int k = 0; k < NC; k++) {
        T s = 0;
#pragma unroll 1
        for (int j = 0; j < MC; j++) s = tfma(op.Ah[j * NC + k], dyj(j), s);
        nat = tmax(nat, tabs(scaled ? s : op.Dinv[k] * s));
    }
    return nat < eps * ndy;
}

template <typename T, int NC, int MC>
__device__ bool dual_infeasible(const AdmmArgs<T> &a, const PlantOps<T> &op, const T *g,
                                const T *uh, const T *lh, int b, T eps, bool scaled)
{
    auto dxp = [&](int k) -> T { return a.xs[b * NC + k] - a.snap_x[b * NC + k]; };
    T qdx = 0;  // q^' dx^ = (W' q^)' dx'
#pragma unroll 1
    for (int k = 0; k < NC; k++) qdx = tfma(g[k * 64], dxp(k), qdx);
    if (!(qdx < T(0))) return false;  // necessary: ||D dx^|| >= 0
    T ndx = 0;
#pragma unroll 1
    for (int i = 0; i < NC; i++) {
        T s = 0;
#pragma unroll 1
        for (int k = 0; k < NC; k++) s = tfma(op.W[i * NC + k], dxp(k), s);
        ndx = tmax(ndx, tabs(scaled ? s : op.D[i] * s));
    }
    const T cs = scaled ? T(1) : op.cs[0];
    if (!(ndx > T(kDivisionTol))) return false;
    if (!(qdx < -cs * eps * ndx)) return false;
    T npdx = 0;
#pragma unroll 1
    for (int i = 0; i < NC; i++) {
        T s = 0;
#pragma unroll 1
        for (int k = 0; k < NC; k++) s = tfma(op.PW[i * NC + k], dxp(k), s);
        npdx = tmax(npdx, tabs(scaled ? s : op.Dinv[i] * s));
    }
    if (!(npdx < cs * eps * ndx)) return false;
#pragma unroll 1
    for (int j = 0; j < MC; j++) {
        T s = 0;
#pragma unroll 1
        for (int k = 0; k < NC; k++) s = tfma(op.WtA[j * NC + k], dxp(k), s);
        if (!scaled) s *= op.Einv[j];
        const T up = uh[j * 64], lo = lh ? lh[j * 64] : T(-kInfty);
        if ((up < T(kInfty * kMinScaling) && s > eps * ndx) || (lo > T(-kInfty * kMinScaling) && s < -eps * ndx))
            return false;
    }
    return true;
}

// ---------------------------------------------------------------------------------------------
// Keep the plant operators out of registers: LLVM would otherwise hoist (LICM) or CSE the ~1.2k
// loop-invariant operator loads of an iteration into VGPRs and spill.  Re-laundering the base
// pointer before every phase makes each phase re-read its operators.  The returned pointer is in
// the constant address space (the operators are read-only for the whole launch), which lets the
// backend serve wave-uniform addresses (shared plant) from the scalar cache with s_load.
template <typename T> using cptr = const __attribute__((address_space(4))) T *;

template <bool SHARED, typename T>
__device__ __forceinline__ cptr<T> launder(const T *p)
{
    int zero;
    if (SHARED) asm volatile("s_mov_b32 %0, 0" : "=s"(zero));
    else asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
    return (cptr<T>)(p + zero);
}

// LDS per 64-lane block, [row][lane] (lane-contiguous => conflict-free):
//   g = W'q^ (NC), dk = 1/(1+rho lambda) (NC), u^ (MC), l^ (MC, only when !LFREE)
template <typename T, int NC, int MC, bool LFREE>
struct LdsLayout {
    static constexpr int g = 0, dk = NC * 64, uh = 2 * NC * 64, lh = (2 * NC + MC) * 64;
    static constexpr int total = (2 * NC + MC + (LFREE ? 0 : MC)) * 64;
};

// Register budget: the per-lane iterate is (NC + 2 MC) values (+ NC temporaries); ask for the
// occupancy that budget allows (fp32: 3 waves/SIMD <= 168 VGPRs, fp64: 2 waves/SIMD <= 256),
// otherwise the scheduler spends registers on ILP up to the 512 a 64-lane block permits.
template <typename T> constexpr int kWavesPerSimd = sizeof(T) == 4 ? 3 : 2;

template <typename T, int NC, int MC, bool SHARED, bool ALL_INEQ, bool LFREE>
__global__ __launch_bounds__(64) 
void admm_lane_kernel(AdmmArgs<T> a)
{
    constexpr OpsLayout L = OpsLayout::make(NC, MC);
    using LL = LdsLayout<T, NC, MC, LFREE>;
    __shared__ T lds[LL::total];
    const int lane = threadIdx.x;
    const int b = blockIdx.x * 64 + lane;
    if (b >= a.batch) return;  // lanes never exchange data: no barrier below
    const int n = a.n, m = a.m;
    const T *base0 = a.ops.lam + (SHARED ? 0 : (size_t)b * a.ops_stride);  // lam starts the block
    PlantOps<T> op;  // plain pointer view for the cold paths
    op.lam = base0 + L.lam; op.W = base0 + L.W; op.sWtW = base0 + L.sWtW; op.WtA = base0 + L.WtA;
    op.PW = base0 + L.PW; op.Winv = base0 + L.Winv; op.Ah = base0 + L.Ah; op.D = base0 + L.D;
    op.E = base0 + L.E; op.Dinv = base0 + L.Dinv; op.Einv = base0 + L.Einv; op.cs = base0 + L.cs;
    op.rscale = base0 + L.rscale;
    const int *ctype = a.ctype + (SHARED ? 0 : (size_t)b * MC);
    const SolverSettings &st = a.st;
    const bool scaled_term = st.scaled_termination != 0;
    T *g = lds + LL::g + lane, *dk = lds + LL::dk + lane, *uh = lds + LL::uh + lane;
    T *lh = LFREE ? uh : lds + LL::lh + lane;  // (unused when LFREE)
    const double c64 = (double)op.cs[0];

    // ---- MPC front end: q = Fx X + Fu U + Fr ref, u = W0 + Sbar X + Ku U (fp64, as the reference)
    double Xv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double Uv = 0.0;
    if (a.mpc) {
#pragma unroll
        for (int t = 0; t < 8; t++)
            if (t < a.nx) Xv[t] = a.X[(size_t)b * a.nx + t];
        Uv = a.U[b];
    }

    // ---- per-QP data: q^ = c D q (osqp_update_lin_cost), u^ = E u, l^ = E l (update_bounds)
    int status = kUnsolved;
    bool lfree_ok = true;
    {
        T qh[NC];
#pragma unroll
        for (int k = 0; k < NC; k++) {
            double qk = 0.0;
            if (k < n) {
                if (a.mpc) {
                    const double *fx = a.Fx + (SHARED ? 0 : (size_t)b * n * a.nx) + (size_t)k * a.nx;
                    const double *fr = a.Fr + (SHARED ? 0 : (size_t)b * n * n) + (size_t)k * n;
                    double s0 = 0.0, s2 = 0.0;
#pragma unroll
                    for (int t = 0; t < 8; t++)
                        if (t < a.nx) s0 += fx[t] * Xv[t];
                    const double s1 = a.Fu[(SHARED ? 0 : (size_t)b * n) + k] * Uv;
                    for (int t = 0; t < n; t++) s2 += fr[t] * a.xref;
                    qk = s0 + s1 + s2;
                    a.q_out[(size_t)b * n + k] = qk;
                } else {
                    qk = a.q[(size_t)b * n + k];
                }
            }
            qh[k] = (T)((qk * (double)op.D[k]) * c64);
        }
#pragma unroll
        for (int k = 0; k < NC; k++) {  // g = W' q^
            T s = 0;
#pragma unroll
            for (int i = 0; i < NC; i++) s = tfma(op.W[i * NC + k], qh[i], s);
            g[k * 64] = s;
        }
    }
#pragma unroll 1
    for (int j = 0; j < MC; j++) {
        double up = kInfty, lo = -kInfty;
        if (j < m) {
            if (a.mpc) {
                const double *sb = a.Sbar + (SHARED ? 0 : (size_t)b * m * a.nx) + (size_t)j * a.nx;
                double s = 0.0;
#pragma unroll
                for (int t = 0; t < 8; t++)
                    if (t < a.nx) s += sb[t] * Xv[t];
                up = a.W0[(SHARED ? 0 : (size_t)b * m) + j] + s + a.Ku[(SHARED ? 0 : (size_t)b * m) + j] * Uv;
                a.u_out[(size_t)b * m + j] = up;
            } else {
                up = a.u[(size_t)b * m + j];
            }
            lo = a.l[(a.l_shared ? 0 : (size_t)b * m) + j];
            const double e = (double)op.E[j];
            up *= e;
            lo *= e;
            if (up < lo) status = kInvalidBounds;
            const int ty = (lo < -kInfty * kMinScaling && up > kInfty * kMinScaling) ? -1 : (up - lo < kRhoTol ? 1 : 0);
            if (ty != ctype[j] && status == kUnsolved) status = kTypeChanged;
        }
        uh[j * 64] = (T)up;
        if (!LFREE) lh[j * 64] = (T)lo;
        else if (!((T)lo < T(-kInfty * kMinScaling))) lfree_ok = false;
    }
    if (LFREE && !lfree_ok && status == kUnsolved) status = kTypeChanged;  // host picked the wrong variant

    // ---- state (warm start keeps x', z, y on the device; rho always persists, as in OSQP)
    T xs[NC], z[MC], y[MC];
    T rho = a.fresh ? (T)fmin(fmax(st.rho, kRhoMin), kRhoMax) : a.rhos[b];
    if (a.warm && !a.fresh) {
#pragma unroll
        for (int k = 0; k < NC; k++) xs[k] = a.xs[b * NC + k];
#pragma unroll
        for (int j = 0; j < MC; j++) { z[j] = a.zs[b * MC + j]; y[j] = a.ys[b * MC + j]; }
    } else {
#pragma unroll
        for (int k = 0; k < NC; k++) xs[k] = 0;
#pragma unroll
        for (int j = 0; j < MC; j++) { z[j] = 0; y[j] = 0; }
    }
    T rinv = T(1) / rho;
#pragma unroll 1
    for (int k = 0; k < NC; k++) dk[k * 64] = T(1) / (T(1) + rho * op.lam[k]);

    const T alpha = (T)st.alpha, oma = T(1) - (T)st.alpha;
    const T eps_abs = (T)st.eps_abs, eps_rel = (T)st.eps_rel;
    int it = 0;
    if (status == kUnsolved) {
        for (it = 1; it <= st.max_iter; it++) {
            const bool at_check = st.check_termination && (it % st.check_termination == 0);
            const bool at_adapt = st.adaptive_rho && a.adaptive_interval && (it % a.adaptive_interval == 0);
            const bool last = it == st.max_iter;
            const bool info = at_check || at_adapt || last;
            if (info) {  // snapshot x', y: the certificates use this iteration's delta_x, delta_y
#pragma unroll
                for (int k = 0; k < NC; k++) a.snap_x[b * NC + k] = xs[k];
#pragma unroll
                for (int j = 0; j < MC; j++) a.snap_y[b * MC + j] = y[j];
            }
            // ---- xi = -g + sigma W'W x' + B' w,   w_j = rho_j z_j - y_j
            T xi[NC];
            {
                const cptr<T> base = launder<SHARED>(base0);
                const cptr<T> sWtW = base + L.sWtW, WtA = base + L.WtA;
#pragma unroll
                for (int k = 0; k < NC; k++) xi[k] = -g[k * 64];
#pragma unroll
                for (int i = 0; i < NC; i++) {
                    const T xv = xs[i];
#pragma unroll
                    for (int k = 0; k < NC; k++) xi[k] = tfma(sWtW[k * NC + i], xv, xi[k]);
                }
#pragma unroll
                for (int j = 0; j < MC; j++) {
                    T rj = rho;
                    if (!ALL_INEQ) rj = ctype[j] == -1 ? T(kRhoMin) : rho * base[L.rscale + j];
                    const T w = tfma(rj, z[j], -y[j]);
#pragma unroll
                    for (int k = 0; k < NC; k++) xi[k] = tfma(WtA[j * NC + k], w, xi[k]);
                }
            }
            // ---- eta = xi / (1 + rho lambda) ; x' = alpha eta + (1-alpha) x'
#pragma unroll
            for (int k = 0; k < NC; k++) {
                xi[k] = xi[k] * dk[k * 64];
                xs[k] = tfma(alpha, xi[k], oma * xs[k]);
            }
            // ---- rows: z~ = B eta ; relaxation ; projection ; dual update
            {
                const cptr<T> base = launder<SHARED>(base0);
                const cptr<T> WtA = base + L.WtA;
#pragma unroll
                for (int j = 0; j < MC; j++) {
                    T zt = 0;
#pragma unroll
                    for (int k = 0; k < NC; k++) zt = tfma(WtA[j * NC + k], xi[k], zt);
                    T rj = rho, rij = rinv;
                    if (!ALL_INEQ) {
                        rj = ctype[j] == -1 ? T(kRhoMin) : rho * base[L.rscale + j];
                        rij = T(1) / rj;
                    }
                    const T v = tfma(alpha, zt, oma * z[j]);
                    T zn = tfma(rij, y[j], v);
                    if (!LFREE) zn = tmax(zn, lh[j * 64]);
                    zn = tmin(zn, uh[j * 64]);
                    y[j] = tfma(rj, v - zn, y[j]);
                    z[j] = zn;
                }
            }
            if (!info) continue;

            // ---- update_info: residuals in the scaled space, reported unscaled
            const cptr<T> base = launder<SHARED>(base0);
            T ax_z = 0, ax_zs = 0, zn_s = 0, zn_r = 0, axn_s = 0, axn_r = 0;
#pragma unroll
            for (int j = 0; j < MC; j++) {
                T s = 0;
#pragma unroll
                for (int k = 0; k < NC; k++) s = tfma(base[L.WtA + j * NC + k], xs[k], s);
                const T r = s - z[j];
                const T ei = base[L.Einv + j];
                ax_z = tmax(ax_z, tabs(r));
                ax_zs = tmax(ax_zs, tabs(ei * r));
                zn_r = tmax(zn_r, tabs(z[j]));
                zn_s = tmax(zn_s, tabs(ei * z[j]));
                axn_r = tmax(axn_r, tabs(s));
                axn_s = tmax(axn_s, tabs(ei * s));
            }
            T dr_r = 0, dr_s = 0, qn_r = 0, qn_s = 0, atyn_r = 0, atyn_s = 0, pxn_r = 0, pxn_s = 0;
#pragma unroll
            for (int k = 0; k < NC; k++) {
                T px = 0, aty = 0;
#pragma unroll
                for (int i = 0; i < NC; i++) px = tfma(base[L.PW + k * NC + i], xs[i], px);
#pragma unroll
                for (int j = 0; j < MC; j++) aty = tfma(base[L.Ah + j * NC + k], y[j], aty);
                double qk = 0.0;
                if (k < n) qk = a.mpc ? a.q_out[(size_t)b * n + k] : a.q[(size_t)b * n + k];
                const T qh = (T)((qk * (double)base[L.D + k]) * c64);
                const T r = (qh + px) + aty;
                const T di = base[L.Dinv + k];
                dr_r = tmax(dr_r, tabs(r));
                dr_s = tmax(dr_s, tabs(di * r));
                qn_r = tmax(qn_r, tabs(qh));
                qn_s = tmax(qn_s, tabs(di * qh));
                atyn_r = tmax(atyn_r, tabs(aty));
                atyn_s = tmax(atyn_s, tabs(di * aty));
                pxn_r = tmax(pxn_r, tabs(px));
                pxn_s = tmax(pxn_s, tabs(di * px));
            }
            const T cinv = base[L.cs + 1];
            const T pri_res = scaled_term ? ax_z : ax_zs;
            const T dua_res = scaled_term ? dr_r : cinv * dr_s;

            // check_termination(approximate) — OSQP auxil.c
            auto check_termination = [&](int approx) -> bool {
                const T mul = approx ? T(10) : T(1);
                if (pri_res > T(kInfty) || dua_res > T(kInfty)) { status = kNonCvx; return true; }
                const T ea = eps_abs * mul, er = eps_rel * mul;
                bool prim_ok = (m == 0), dual_ok = false, prim_inf = false, dual_inf = false;
                if (m > 0) {
                    const T ep = ea + er * (scaled_term ? tmax(zn_r, axn_r) : tmax(zn_s, axn_s));
                    if (pri_res < ep) {
                        prim_ok = true;
                    } else {
#pragma unroll
                        for (int j = 0; j < MC; j++) a.ys[b * MC + j] = y[j];
                        prim_inf = primal_infeasible<T, NC, MC>(a, op, uh, LFREE ? nullptr : lh, b,
                                                                (T)st.eps_prim_inf * mul, scaled_term);
                    }
                }
                const T ed = ea + er * (scaled_term ? tmax(tmax(qn_r, atyn_r), pxn_r)
                                                    : cinv * tmax(tmax(qn_s, atyn_s), pxn_s));
                if (dua_res < ed) {
                    dual_ok = true;
                } else {
#pragma unroll
                    for (int k = 0; k < NC; k++) a.xs[b * NC + k] = xs[k];
                    dual_inf = dual_infeasible<T, NC, MC>(a, op, g, uh, LFREE ? nullptr : lh, b,
                                                          (T)st.eps_dual_inf * mul, scaled_term);
                }
                if (prim_ok && dual_ok) { status = approx ? kSolvedInaccurate : kSolved; return true; }
                if (prim_inf) { status = approx ? kPrimalInfeasibleInaccurate : kPrimalInfeasible; return true; }
                if (dual_inf) { status = approx ? kDualInfeasibleInaccurate : kDualInfeasible; return true; }
                return false;
            };

            bool term = false;
            if (at_check) term = check_termination(0);
            if (!term && at_adapt) {  // adapt_rho / compute_rho_estimate (scaled-space norms)
                const T pr = ax_z / (tmax(zn_r, axn_r) + T(kDivisionTol));
                const T dn = tmax(tmax(qn_r, atyn_r), pxn_r);
                const T du = dr_r / (dn + T(kDivisionTol));
                T rn = rho * (T)sqrt((double)(pr / (du + T(kDivisionTol))));
                rn = tmin(tmax(rn, T(kRhoMin)), T(kRhoMax));
                if (rn > rho * (T)st.adaptive_rho_tolerance || rn < rho / (T)st.adaptive_rho_tolerance) {
                    rho = tmin(tmax(rn, T(kRhoMin)), T(kRhoMax));
                    rinv = T(1) / rho;
#pragma unroll 1
                    for (int k = 0; k < NC; k++) dk[k * 64] = T(1) / (T(1) + rho * op.lam[k]);
                }
            }
            if (!term && last) {  // after the ADMM loop (osqp_solve)
                if (!at_check) term = check_termination(0);
                if (!term && !check_termination(1)) status = kMaxIterReached;
                term = true;
            }
            if (term) break;
        }
        if (it > st.max_iter) it = st.max_iter;
    }

    // ---- store_solution: x = D W x', y = E y / c   (NaN + cold start if no solution)
    const bool has_sol = status == kSolved || status == kSolvedInaccurate || status == kMaxIterReached;
    const double cinv64 = (double)op.cs[1];
#pragma unroll 1
    for (int i = 0; i < n; i++) {
        double v;
        if (has_sol) {
            T s = 0;
#pragma unroll
            for (int k = 0; k < NC; k++) s = tfma(op.W[i * NC + k], xs[k], s);
            v = (double)s * (double)op.D[i];
        } else {
            v = __builtin_nan("");
        }
        if (a.x) a.x[(size_t)b * n + i] = v;
        if (i == 0 && a.mpc_u && status == kSolved) a.U[b] = Uv + v;  // U += x(0)  (:105)
    }
    if (a.y) {
#pragma unroll
        for (int j = 0; j < MC; j++)
            if (j < m) a.y[(size_t)b * m + j] = has_sol ? ((double)y[j] * (double)op.E[j]) * cinv64 : __builtin_nan("");
    }
    const bool keep = has_sol || status == kInvalidBounds || status == kTypeChanged;
#pragma unroll
    for (int k = 0; k < NC; k++) a.xs[b * NC + k] = keep ? xs[k] : T(0);
#pragma unroll
    for (int j = 0; j < MC; j++) {
        a.zs[b * MC + j] = keep ? z[j] : T(0);
        a.ys[b * MC + j] = keep ? y[j] : T(0);
    }
    a.rhos[b] = rho;
    a.status[b] = status;
    a.iter[b] = it;
    a.rho_out[b] = (double)rho;
    if (a.it_acc) {
        a.it_acc[b] += it;
        a.uns_acc[b] += status != kSolved;
    }
}

// osqp_warm_start: x^ = Dinv x, x' = W^-1 x^, z = A^ x^, y^ = c Einv y  (all QPs).  Cold path with
// runtime capacities (nc, mc): serves the lane kernel's and the tile kernel's state layout alike.
template <typename T>
__global__ __launch_bounds__(64) void warm_start_kernel(AdmmArgs<T> a, int nc, int mc, const double *x, const double *y)
{
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= a.batch) return;
    const int n = a.n, m = a.m;
    const size_t po = a.shared ? 0 : (size_t)b * a.ops_stride;
    const PlantOps<T> op = a.ops;
    auto xh = [&](int i) -> T { return i < n ? (T)(x[(size_t)b * n + i] * (double)op.Dinv[po + i]) : T(0); };
    for (int k = 0; k < nc; k++) {
        T s = 0;
        for (int i = 0; i < nc; i++) s = tfma(op.Winv[po + (size_t)k * nc + i], xh(i), s);
        a.xs[(size_t)b * nc + k] = s;
    }
    for (int j = 0; j < mc; j++) {
        T s = 0;
        for (int k = 0; k < nc; k++) s = tfma(op.Ah[po + (size_t)j * nc + k], xh(k), s);
        a.zs[(size_t)b * mc + j] = s;
        a.ys[(size_t)b * mc + j] =
            j < m ? (T)((y[(size_t)b * m + j] * (double)op.Einv[po + j]) * (double)op.cs[po]) : T(0);
    }
}

// ---------------------------------------------------------------------------------------------
template <typename T, int NC, int MC>
static int launch_cap(const AdmmArgs<T> &a, hipStream_t s)
{
    const dim3 grid((a.batch + 63) / 64), block(64);
    // Specialisations: shared plant (scalar operands) x all-inequality rows x lower bounds all -inf.
    if (a.shared && a.all_ineq && a.lower_free)
        hipLaunchKernelGGL((admm_lane_kernel<T, NC, MC, true, true, true>), grid, block, 0, s, a);
    else if (a.shared)
        hipLaunchKernelGGL((admm_lane_kernel<T, NC, MC, true, false, false>), grid, block, 0, s, a);
    else
        hipLaunchKernelGGL((admm_lane_kernel<T, NC, MC, false, false, false>), grid, block, 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Kernel capacities (n <= NC, m <= MC); the host picks the smallest that fits.
#define MPCQ_CAPS(X) X(8, 16) X(16, 32) X(20, 40) X(32, 64)

template <typename T>
static int launch_any(const AdmmArgs<T> &a, int nc, int mc, hipStream_t s)
{
#define MPCQ_TRY(NC_, MC_) if (nc == NC_ && mc == MC_) return launch_cap<T, NC_, MC_>(a, s);
    MPCQ_CAPS(MPCQ_TRY)
#undef MPCQ_TRY
    return -1;
}

template <typename T>
static int warm_any(const AdmmArgs<T> &a, int nc, int mc, const double *x, const double *y, hipStream_t s)
{
    hipLaunchKernelGGL((warm_start_kernel<T>), dim3((a.batch + 63) / 64), dim3(64), 0, s, a, nc, mc, x, y);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace mpcq

