// solvempc_amd/csrc/mpcq_wave.h — one QP per wavefront: the latency path of the batched OSQP-v0.6
// ADMM (osqp_solve behind OsqpEigen::Solver::solve, ModelPredictiveControlAPI.cpp:102).
//
// Used (1) for per-plant batches (n_plants == batch: every QP has its own operators, so there is no
// shared GEMM for the tile kernel), and (2) for the tail phases of a shared-plant solve, when a few
// slow QPs remain: a wave then finishes an iteration in a few hundred cycles instead of the ~45
// dependent MFMAs of a tile wave.
//
// Mapping: lane k holds variable k (k < n) and lane j holds constraint row j (j < m); the operator
// rows a lane needs live in its VGPRs for the whole solve (row k of sigma W'W and column k of
// B = A^ W for the x-side product, row j of B for the z-side product).  The two broadcasts of an
// iteration (x' and w, then eta) go through LDS (one write per lane, 16-B broadcast reads).  Lane
// reductions (residual norms, certificates) are DPP + permlane swaps.  A QP can move from a tile
// launch to a wave launch at a phase boundary: both run OSQP's iteration on the same state (x', z, y,
// rho), with the products summed in different orders (last-bit differences, like any two OSQP builds).
#pragma once
#include "mpcq_plant_sim.h"
#include "mpcq_tile.h"

namespace mpcq {

// Ordering of the LDS broadcast buffers.  The workgroup is ONE wave, and the LDS executes one wave's
// DS instructions in issue order, so a lane's read after another lane's write of the same word (or a
// write after a read) needs no s_barrier and no lgkmcnt wait: only the compiler must keep program
// order (the memory clobber).  (With __syncthreads a broadcast cost a write -> wait -> barrier ->
// read round trip: ~450 cycles of an ~1,800-cycle tail iteration.)
__device__ __forceinline__ void wave_sync() { asm volatile("" ::: "memory"); }

// full lane permutations only (quad_perm, row mirrors: every lane has a source), so no "old" operand:
// the move needs no copy of v into its destination first.  bound_ctrl = true: a lane whose source lane is
// inactive reads 0, so these moves (and wave_reduce / the scans built on them, here and in mpcq_mimo.hip /
// mpcq_plant.hip) are only correct under a full EXEC mask.  Every caller runs them in wave-uniform control
// flow (all 64 lanes active, dead lanes masked by value, not by EXEC).
template <int CTRL> __device__ __forceinline__ unsigned dpp_u(unsigned v)
{
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
template <int CTRL> __device__ __forceinline__ float dpp_t(float v) { return __uint_as_float(dpp_u<CTRL>(__float_as_uint(v))); }
template <int CTRL> __device__ __forceinline__ double dpp_t(double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = dpp_u<CTRL>((unsigned)u), hi = dpp_u<CTRL>((unsigned)(u >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Whole-wave reduction with a symmetric op: quad swaps, half-row and row mirrors (DPP), then the
// 16/32-lane swaps of col_reduce.  Every lane ends with the same bits.
template <typename T, typename F> __device__ __forceinline__ T wave_reduce(T v, F op)
{
    v = op(v, dpp_t<0xB1>(v));   // quad_perm [1,0,3,2]
    v = op(v, dpp_t<0x4E>(v));   // quad_perm [2,3,0,1]
    v = op(v, dpp_t<0x141>(v));  // row_half_mirror
    v = op(v, dpp_t<0x140>(v));  // row_mirror
    return col_reduce(v, op);
}
template <typename T> __device__ __forceinline__ T wmax(T v)
{
    return wave_reduce(v, [](T a, T b) { return tt_fmax(a, b); });
}
template <typename T> __device__ __forceinline__ T wsum(T v)
{
    return wave_reduce(v, [](T a, T b) { return a + b; });
}
__device__ __forceinline__ int wor(int v) { return wave_any(v != 0) ? 1 : 0; }

// acc + sum_i row[i] * bc[i] over the whole capacity: rows are zero beyond n / m and so are the
// broadcast buffers, so the padding terms are exact no-ops (fixed trip count, no branches).  Four
// interleaved partial sums (i mod 4) keep the dependent-FMA chain at CAP / 4: this product is the
// latency of a lone QP's iteration (the tail of a shared-plant solve).
template <typename T, int CAP>
__device__ __forceinline__ T row_dot(const T (&row)[CAP], const T *bc, T acc)
{
    constexpr int VEC = 16 / sizeof(T);
    typedef T vec __attribute__((ext_vector_type(VEC)));
    bc += opaque(0);  // a divergent address: keep the broadcast values in VGPRs (not SGPR copies)
    T p[4] = {acc, T(0), T(0), T(0)};
#pragma unroll
    for (int i0 = 0; i0 < CAP; i0 += VEC) {
        const vec v = *(const vec *)(bc + i0);
#pragma unroll
        for (int e = 0; e < VEC; e++)
            if (i0 + e < CAP) p[(i0 + e) & 3] = tt_fma(row[i0 + e], v[e], p[(i0 + e) & 3]);
    }
    return (p[0] + p[1]) + (p[2] + p[3]);
}

// acc + sum_i M[i * stride] * bc[i] for i < CAP, M a zero-padded global operator column/row (cold
// paths).
template <typename T, int CAP>
__device__ __forceinline__ T mem_dot(const T *M, size_t stride, const T *bc, T acc)
{
    bc += opaque(0);
#pragma unroll 4
    for (int i = 0; i < CAP; i++) acc = tt_fma(M[(size_t)i * stride], bc[i], acc);
    return acc;
}

// Direct-inverse operators (mpcq_internal.h) for a rho other than the one they were built for:
// M = P^ + sigma I + sum_j rho_j a_j a_j' (fp64 in LDS, stride NCAP + 1) and its Gauss-Jordan inverse
// in place (SPD: no pivoting).  OSQP refactors its KKT matrix at the same points.  (Out of line and
// free of the caller's register arrays: the operator rows are reloaded from `mi` by the caller.)
template <typename T, int NCAP>
__device__ __noinline__ void build_minv(const T *ops, const int *ctype, const OpsLayout &L, int n, int m, int nc,
                                        double sigma, double rho, double *mi)
{
    constexpr int LD = NCAP + 1, PER = (NCAP * NCAP + 63) / 64;
    const int lane = threadIdx.x;
    __syncthreads();
    for (int e = lane; e < n * n; e += 64) {
        const int i = e / n, k = e % n;
        double v = (double)ops[L.PW + (size_t)i * nc + k] + (i == k ? sigma : 0.0);
        for (int r = 0; r < m; r++) {
            const double rj = ctype[r] == -1 ? kRhoMin : rho * (double)ops[L.rscale + r];
            v += rj * ((double)ops[L.WtA + (size_t)r * nc + i] * (double)ops[L.WtA + (size_t)r * nc + k]);
        }
        mi[i * LD + k] = v;
    }
    __syncthreads();
    for (int k = 0; k < n; k++) {
        const double ip = 1.0 / mi[k * LD + k];
        double nv[PER];
#pragma unroll
        for (int c = 0; c < PER; c++) {
            const int e = lane + 64 * c;
            if (e < n * n) {
                const int i = e / n, j = e % n;
                double v;
                if (i == k && j == k) v = ip;
                else if (i == k) v = mi[k * LD + j] * ip;
                else if (j == k) v = -mi[i * LD + k] * ip;
                else v = mi[i * LD + j] - mi[i * LD + k] * (mi[k * LD + j] * ip);
                nv[c] = v;
            }
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < PER; c++) {
            const int e = lane + 64 * c;
            if (e < n * n) mi[(e / n) * LD + e % n] = nv[c];
        }
        __syncthreads();
    }
}

template <typename T, int NCAP, int MCAP, bool ALL_INEQ, bool LFREE>
__device__ __forceinline__ void wave_solve_one(const AdmmArgs<T> &a, int nc, int mc, int b, T *bcx, T *bcw, double *mi,
                                               bool fresh_ok = true)
{
    constexpr int VEC = 16 / sizeof(T);
    constexpr int BN = (NCAP + VEC - 1) / VEC * VEC, BM = (MCAP + VEC - 1) / VEC * VEC;
    const int lane = threadIdx.x;
    wave_sync();  // the previous QP of this block is done with the broadcast buffers
    const int n = a.n, m = a.m;
    const bool ln = lane < n, lm = lane < m;
    const size_t po = a.shared ? 0 : (size_t)b * a.ops_stride;
    const OpsLayout L = OpsLayout::make(nc, mc);
    const T *ops = a.ops.lam + po;  // the plant's operator block (lam starts it)
    const int *ctype = a.ctype + (a.shared ? 0 : (size_t)b * mc);
    const SolverSettings &st = a.st;
    const bool scaled_term = st.scaled_termination != 0;
    const double c64 = (double)ops[L.cs];
    const int kl = ln ? lane : 0, jl = lm ? lane : 0;  // clamped row indices for loads

    // ---- operator rows (VGPRs for the whole solve)
    // (the operator block is zero beyond n, m and NCAP <= nc, MCAP <= mc: no per-element guards;
    // lanes beyond n / m read row 0 and their results are never published)
    T Srow[NCAP], Btrow[MCAP], Brow[NCAP];
#pragma unroll
    for (int i = 0; i < NCAP; i++) Srow[i] = ops[L.sWtW + (size_t)kl * nc + i];
#pragma unroll
    for (int j = 0; j < MCAP; j++) Btrow[j] = ops[L.Bt + (size_t)j * nc + kl];
#pragma unroll
    for (int k = 0; k < NCAP; k++) Brow[k] = ops[L.WtA + (size_t)jl * nc + k];
    for (int i = lane; i < BN; i += 64) bcx[i] = T(0);
    for (int i = lane; i < BM; i += 64) bcw[i] = T(0);

    // ---- per-QP data (setF / setUpperBound in the MPC front end, else the updated q, u, l)
    double Xv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double Uv = 0.0;
    if (a.mpc) {
#pragma unroll
        for (int t = 0; t < 8; t++)
            if (t < a.nx) Xv[t] = a.X[(size_t)b * a.nx + t];
    }
    if (a.mpc_u) Uv = a.U[b];
    T qh = T(0);
    if (ln) {
        double qk;
        if (a.mpc) {
            const size_t pp = a.shared ? 0 : (size_t)b;
            const double *fx = a.Fx + (pp * n + lane) * a.nx;
            const double *fr = a.Fr + (pp * n + lane) * n;
            double s0 = 0.0, s2 = 0.0;
#pragma unroll
            for (int t = 0; t < 8; t++)
                if (t < a.nx) s0 += fx[t] * Xv[t];
            const double s1 = a.Fu[pp * n + lane] * Uv;
            for (int t = 0; t < n; t++) s2 += fr[t] * a.xref;
            qk = s0 + s1 + s2;
            a.q_out[(size_t)b * n + lane] = qk;
        } else {
            qk = a.q[(size_t)b * n + lane];
        }
        qh = (T)((qk * (double)ops[L.D + lane]) * c64);
    }
    int bad = 0, tchg = 0;
    T uh = T(kInfty), lh = T(-kInfty), rs = T(1);
    if (lm) {
        double up, lo;
        if (a.mpc) {
            const size_t pp = a.shared ? 0 : (size_t)b;
            const double *sb = a.Sbar + (pp * m + lane) * a.nx;
            double sx = 0.0;
#pragma unroll
            for (int t = 0; t < 8; t++)
                if (t < a.nx) sx += sb[t] * Xv[t];
            up = a.W0[pp * m + lane] + sx + a.Ku[pp * m + lane] * Uv;
            a.u_out[(size_t)b * m + lane] = up;
        } else {
            up = a.u[(size_t)b * m + lane];
        }
        lo = a.l[(a.l_shared ? 0 : (size_t)b * m) + lane];
        const double e = (double)ops[L.E + lane];
        up *= e;
        lo *= e;
        if (up < lo) bad = 1;
        const int ty = (lo < -kInfty * kMinScaling && up > kInfty * kMinScaling) ? -1 : (up - lo < kRhoTol ? 1 : 0);
        if (ty != ctype[lane]) tchg = 1;
        if (LFREE && !((T)lo < T(-kInfty * kMinScaling))) tchg = 1;
        uh = (T)up;
        lh = (T)lo;
        rs = ctype[lane] == -1 ? T(-1) : ops[L.rscale + lane];
    }
    int status = wor(bad) ? kInvalidBounds : (wor(tchg) ? kTypeChanged : kUnsolved);

    // g = G' q^ (lane k: column k of G = W, or of M^-1 for direct-inverse operators)
    if (ln) bcx[lane] = qh;
    wave_sync();
    T gk = T(0);
    {
        gk = mem_dot<T, NCAP>(ops + L.G + kl, nc, bcx, gk);
    }
    gk = ln ? -gk : T(0);
    const T rho0 = ops[L.rho0];  // direct-inverse operators: the rho they hold (eigen basis: -1)
    const bool inv = rho0 > T(0);

    // ---- state
    T xs = T(0), z = T(0), y = T(0), rho;
    int it = 0;
    const int ncs = nc, mcs = mc;
    const bool fresh = a.fresh && fresh_ok;  // (the stream kernel: a reset applies to its first step only)
    const bool load_state = a.resume || (a.warm && !fresh);
    if (a.resume) {
        rho = a.rhos[b];
        it = a.it_state[b];
    } else {
        rho = fresh ? (T)fmin(fmax(st.rho, kRhoMin), kRhoMax) : a.rhos[b];
    }
    if (load_state) {
        if (ln) xs = a.xs[(size_t)b * ncs + lane];
        if (lm) {
            z = a.zs[(size_t)b * mcs + lane];
            y = a.ys[(size_t)b * mcs + lane];
        }
    }
    it = __builtin_amdgcn_readfirstlane(it);
    // direct-inverse operators for the QP's rho: sigma M^-1 (row k), (A^ M^-1)' (row k), g = -M^-1 q^
    // (q^ in bcx), from M(rho)^-1 rebuilt in `mi`
    auto reload_rows = [&]() {
        constexpr int LD = NCAP + 1;
#pragma unroll
        for (int i = 0; i < NCAP; i++) Srow[i] = (i < n) ? (T)(st.sigma * mi[kl * LD + i]) : T(0);
#pragma unroll
        for (int j = 0; j < MCAP; j++) {
            double v = 0.0;
            if (j < m)
                for (int r = 0; r < n; r++) v += (double)ops[L.WtA + (size_t)j * nc + r] * mi[r * LD + kl];
            Btrow[j] = (T)v;
        }
        double g = 0.0;
        for (int i = 0; i < n; i++) g += mi[i * LD + kl] * (double)bcx[i];
        gk = ln ? (T)(-g) : T(0);
        __syncthreads();
    };
    bool refactor = inv && rho != rho0;  // done at the top of the next iteration (one code site)
    T rinv = T(1) / rho;
    const T lamk = ln ? ops[L.lam + lane] : T(0);
    T dk = T(1) / (T(1) + rho * lamk);
    const T alpha = (T)st.alpha, oma = T(1) - (T)st.alpha;
    const T eps_abs = (T)st.eps_abs, eps_rel = (T)st.eps_rel;

    auto finalize = [&]() {
        // x = D W x' (lane i: row i of W)
        wave_sync();
        if (ln) bcx[lane] = xs;
        wave_sync();
        const T xh = mem_dot<T, NCAP>(ops + L.W + (size_t)kl * nc, 1, bcx, T(0));
        const bool has_sol = status == kSolved || status == kSolvedInaccurate || status == kMaxIterReached;
        if (ln) {
            const double xv = has_sol ? (double)xh * (double)ops[L.D + lane] : __builtin_nan("");
            if (a.x) a.x[(size_t)b * n + lane] = xv;
            if (lane == 0 && a.mpc_u && status == kSolved) a.U[b] = Uv + xv;  // U += x(0)  (:105)
        }
        if (lm && a.y) a.y[(size_t)b * m + lane] = has_sol ? ((double)y * (double)ops[L.E + lane]) * (double)ops[L.cs + 1]
                                                          : __builtin_nan("");
        const bool keep = has_sol || status == kInvalidBounds || status == kTypeChanged;
        if (ln) a.xs[(size_t)b * ncs + lane] = keep ? xs : T(0);
        if (lm) {
            a.zs[(size_t)b * mcs + lane] = keep ? z : T(0);
            a.ys[(size_t)b * mcs + lane] = keep ? y : T(0);
        }
        if (lane == 0) {
            a.rhos[b] = rho;
            a.status[b] = status;
            a.iter[b] = it;
            a.rho_out[b] = (double)rho;
            if (a.it_acc) {
                a.it_acc[b] += it;
                a.uns_acc[b] += status != kSolved;
            }
        }
    };
    if (status != kUnsolved) {
        finalize();
        return;
    }

    const int ct = st.check_termination;
    const int ai = (st.adaptive_rho && a.adaptive_interval) ? a.adaptive_interval : 0;
    const int stop = a.stop_iter;
    int next_check = ct ? (it / ct + 1) * ct : -1;
    int next_adapt = ai ? (it / ai + 1) * ai : -1;
    const T *Einv_p = ops + L.Einv;
    const T *Dinv_p = ops + L.Dinv;
#ifdef MPCQ_WAVE_STAMPS
#define MPCQ_WSTAMP(k)                                                                                  \
    do {                                                                                                \
        if (a.stamps && blockIdx.x < 2048 && (it == 140 || it == 141)) a.stamps[(size_t)blockIdx.x * 16 + (it - 140) * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#else
#define MPCQ_WSTAMP(k) do { } while (0)
#endif
    for (;;) {
        if (refactor) {  // (cold) OSQP's KKT refactorisation after a rho change
            wave_sync();
            if (ln) bcx[lane] = qh;
            wave_sync();
            build_minv<T, NCAP>(ops, ctype, L, n, m, nc, st.sigma, (double)rho, mi);
            reload_rows();
            refactor = false;
        }
        it++;
        MPCQ_WSTAMP(0);
        const bool at_check = it == next_check;
        const bool at_adapt = it == next_adapt;
        if (at_check) next_check += ct;
        if (at_adapt) next_adapt += ai;
        const bool last = it == st.max_iter;
        const bool info = at_check || at_adapt || last || it == stop;

        // ---- xi = -g + sigma W'W x' + B' w  (broadcast x' and w)
        T rj = rho, rij = rinv;
        if (!ALL_INEQ) {
            rj = rs < T(0) ? T(kRhoMin) : rho * rs;
            rij = T(1) / rj;
        }
        const T w = lm ? tt_fma(rj, z, -y) : T(0);
        wave_sync();  // previous readers of bcx / bcw are done
        if (ln) bcx[lane] = xs;
        if (lm) bcw[lane] = w;
        wave_sync();
        MPCQ_WSTAMP(1);
        T xi = row_dot(Srow, bcx, gk) + row_dot(Btrow, bcw, T(0));  // two independent chains
        const T eta = xi * dk;
        const T xn = ln ? tt_fma(alpha, eta, oma * xs) : T(0);
        const T dx = xn - xs;
        xs = xn;
        // ---- z~ = B eta ; relaxation ; projection ; dual update
        wave_sync();
        MPCQ_WSTAMP(2);
        if (ln) bcx[lane] = eta;
        wave_sync();
        MPCQ_WSTAMP(3);
        const T zt = row_dot(Brow, bcx, T(0));
        T dy = T(0);
        if (lm) {
            const T v = tt_fma(alpha, zt, oma * z);
            T zn = tt_fma(rij, y, v);
            if (!LFREE) zn = tt_fmax(zn, lh);
            zn = tt_fmin(zn, uh);
            dy = rj * (v - zn);
            y = tt_fma(rj, v - zn, y);
            z = zn;
        }
        MPCQ_WSTAMP(4);
        if (!info) continue;

        // ---- update_info: residual norms (whole-wave reductions)
        wave_sync();
        if (ln) bcx[lane] = xs;
        if (lm) bcw[lane] = y;
        wave_sync();
        T ax_z = 0, ax_zs = 0, zn_s = 0, zn_r = 0, axn_s = 0, axn_r = 0;
        if (lm) {
            const T ax = row_dot(Brow, bcx, T(0));
            const T r = ax - z, ei = Einv_p[lane];
            ax_z = tt_fabs(r);
            ax_zs = tt_fabs(ei * r);
            zn_r = tt_fabs(z);
            zn_s = tt_fabs(ei * z);
            axn_r = tt_fabs(ax);
            axn_s = tt_fabs(ei * ax);
        }
        T dr_r = 0, dr_s = 0, qn_r = 0, qn_s = 0, atyn_r = 0, atyn_s = 0, pxn_r = 0, pxn_s = 0;
        if (ln) {
            T px = T(0), aty = T(0);
            px = mem_dot<T, NCAP>(ops + L.PW + (size_t)lane * nc, 1, bcx, px);
            aty = mem_dot<T, MCAP>(ops + L.Ah + lane, nc, bcw, aty);
            const T r = (qh + px) + aty, di = Dinv_p[lane];
            dr_r = tt_fabs(r);
            dr_s = tt_fabs(di * r);
            qn_r = tt_fabs(qh);
            qn_s = tt_fabs(di * qh);
            atyn_r = tt_fabs(aty);
            atyn_s = tt_fabs(di * aty);
            pxn_r = tt_fabs(px);
            pxn_s = tt_fabs(di * px);
        }
        ax_z = wmax(ax_z); ax_zs = wmax(ax_zs); zn_s = wmax(zn_s); zn_r = wmax(zn_r);
        axn_s = wmax(axn_s); axn_r = wmax(axn_r);
        dr_r = wmax(dr_r); dr_s = wmax(dr_s); qn_r = wmax(qn_r); qn_s = wmax(qn_s);
        atyn_r = wmax(atyn_r); atyn_s = wmax(atyn_s); pxn_r = wmax(pxn_r); pxn_s = wmax(pxn_s);
        const T cinv = ops[L.cs + 1];
        const T pri_res = scaled_term ? ax_z : ax_zs;
        const T dua_res = scaled_term ? dr_r : cinv * dr_s;

        auto primal_infeasible = [&](T eps) -> bool {
            T d = T(0), ndy = 0, lhs = 0;
            if (lm) {
                d = dy;
                const T up = uh, lo = LFREE ? T(-kInfty) : lh;
                const bool uinf = up > T(kInfty * kMinScaling), linf = lo < T(-kInfty * kMinScaling);
                if (uinf) d = linf ? T(0) : tt_min(d, T(0));
                else if (linf) d = tt_max(d, T(0));
                ndy = tt_fabs(scaled_term ? d : ops[L.E + lane] * d);
                if (up < T(kInfty * kMinScaling)) lhs += up * tt_max(d, T(0));
                if (lo > T(-kInfty * kMinScaling)) lhs += lo * tt_min(d, T(0));
            }
            ndy = wmax(ndy);
            lhs = wsum(lhs);
            if (!(ndy > T(kDivisionTol) && lhs < eps * ndy)) return false;
            wave_sync();
            if (lm) bcw[lane] = d;
            wave_sync();
            T atd = T(0);
            if (ln) atd = mem_dot<T, MCAP>(ops + L.Ah + lane, nc, bcw, atd);
            const T nat = wmax(ln ? tt_fabs(scaled_term ? atd : Dinv_p[lane] * atd) : T(0));
            return nat < eps * ndy;
        };
        auto dual_infeasible = [&](T eps) -> bool {
            if (a.dinf_kappa > 2.0 * (scaled_term ? 1.0 : (double)ops[L.cs]) * (double)eps) return false;  // (AdmmArgs)
            const T qdx = wsum(ln ? -gk * dx : T(0));  // q^' dx^ = (W' q^)' dx'
            if (!(qdx < T(0))) return false;
            wave_sync();
            if (ln) bcx[lane] = dx;
            wave_sync();
            T t1 = T(0), t2 = T(0), t3 = T(0);
            if (ln) {
                t1 = mem_dot<T, NCAP>(ops + L.W + (size_t)lane * nc, 1, bcx, t1);
                t2 = mem_dot<T, NCAP>(ops + L.PW + (size_t)lane * nc, 1, bcx, t2);
            }
            if (lm) t3 = row_dot(Brow, bcx, T(0));
            const T ndx = wmax(ln ? tt_fabs(scaled_term ? t1 : ops[L.D + lane] * t1) : T(0));
            const T cs = scaled_term ? T(1) : ops[L.cs];
            if (!(ndx > T(kDivisionTol) && qdx < -cs * eps * ndx)) return false;
            const T npdx = wmax(ln ? tt_fabs(scaled_term ? t2 : Dinv_p[lane] * t2) : T(0));
            if (!(npdx < cs * eps * ndx)) return false;
            int viol = 0;
            if (lm) {
                const T sv = scaled_term ? t3 : Einv_p[lane] * t3;
                const T lo = LFREE ? T(-kInfty) : lh;
                if ((uh < T(kInfty * kMinScaling) && sv > eps * ndx) || (lo > T(-kInfty * kMinScaling) && sv < -eps * ndx))
                    viol = 1;
            }
            return !wor(viol);
        };
        auto check_termination = [&](bool approx) -> int {
            const T mul = approx ? T(10) : T(1);
            if (pri_res > T(kInfty) || dua_res > T(kInfty)) return kNonCvx;
            const T ea = eps_abs * mul, er = eps_rel * mul;
            bool prim_ok = (m == 0), dual_ok = false, prim_inf = false, dual_inf = false;
            if (m > 0) {
                const T ep = ea + er * (scaled_term ? tt_max(zn_r, axn_r) : tt_max(zn_s, axn_s));
                if (pri_res < ep) prim_ok = true;
                else prim_inf = primal_infeasible((T)st.eps_prim_inf * mul);
            }
            const T ed = ea + er * (scaled_term ? tt_max(tt_max(qn_r, atyn_r), pxn_r)
                                                : cinv * tt_max(tt_max(qn_s, atyn_s), pxn_s));
            if (dua_res < ed) dual_ok = true;
            else dual_inf = dual_infeasible((T)st.eps_dual_inf * mul);
            if (prim_ok && dual_ok) return approx ? kSolvedInaccurate : kSolved;
            if (prim_inf) return approx ? kPrimalInfeasibleInaccurate : kPrimalInfeasible;
            if (dual_inf) return approx ? kDualInfeasibleInaccurate : kDualInfeasible;
            return kUnsolved;
        };

        bool term = false;  // everything below is wave-uniform: one QP per wave
        if (at_check) {
            const int s0 = check_termination(false);
            if (s0 != kUnsolved) { status = s0; term = true; }
        }
        if (!term && at_adapt) {
            const T pr = ax_z / (tt_max(zn_r, axn_r) + T(kDivisionTol));
            const T dn = tt_max(tt_max(qn_r, atyn_r), pxn_r);
            const T du = dr_r / (dn + T(kDivisionTol));
            T rn = rho * (T)sqrt((double)(pr / (du + T(kDivisionTol))));
            rn = tt_min(tt_max(rn, T(kRhoMin)), T(kRhoMax));
            if (rn > rho * (T)st.adaptive_rho_tolerance || rn < rho / (T)st.adaptive_rho_tolerance) {
                rho = tt_min(tt_max(rn, T(kRhoMin)), T(kRhoMax));
                rinv = T(1) / rho;
                dk = T(1) / (T(1) + rho * lamk);
                refactor = inv;  // direct inverse: M(rho)^-1 and the operator rows built on it
            }
        }
        if (!term && last) {
            if (!at_check) {
                const int s1 = check_termination(false);
                if (s1 != kUnsolved) { status = s1; term = true; }
            }
            if (!term) {
                const int s2 = check_termination(true);
                status = s2 != kUnsolved ? s2 : kMaxIterReached;
                term = true;
            }
        }
        if (term) {
            finalize();
            return;
        }
        if (it == stop) {  // phase boundary (shared-plant tail): save and re-queue
            if (ln) a.xs[(size_t)b * ncs + lane] = xs;
            if (lm) {
                a.zs[(size_t)b * mcs + lane] = z;
                a.ys[(size_t)b * mcs + lane] = y;
            }
            if (lane == 0) {
                a.rhos[b] = rho;
                a.it_state[b] = it;
                const int sg = blockIdx.x % ListSeg::kShards;
                a.list_out[sg * a.list_seg + atomicAdd(a.count_out + sg * ListSeg::kStride, 1)] = b;
            }
            return;
        }
    }
}

template <typename T, int NCAP, int MCAP, bool ALL_INEQ, bool LFREE>
__global__ __launch_bounds__(64, 2) void admm_wave_kernel(AdmmArgs<T> a, int nc, int mc)
{
    static_assert(NCAP <= 64 && MCAP <= 64, "one row per lane");  // one wave per workgroup (wave_sync)
    constexpr int VEC = 16 / sizeof(T);
    constexpr int BN = (NCAP + VEC - 1) / VEC * VEC, BM = (MCAP + VEC - 1) / VEC * VEC;
    __shared__ __attribute__((aligned(16))) T bcx[BN];  // x'-side broadcast (x', eta, q^, dx)
    __shared__ __attribute__((aligned(16))) T bcw[BM];  // row-side broadcast (w, y, d)
    __shared__ double mi[NCAP * (NCAP + 1)];            // direct-inverse refactorisation (cold path)
    if (blockIdx.x == 0 && threadIdx.x < ListSeg::kShards) {  // counters no launch of this chain is using
        if (a.zero_cnt) a.zero_cnt[threadIdx.x * ListSeg::kStride] = 0;
        if (a.zero_cnt0) a.zero_cnt0[threadIdx.x * ListSeg::kStride] = 0;
    }
    if (a.list_in) {  // a resumed phase's ListSeg list: block b serves segment b % kShards (grid % kShards == 0)
        const int sg = blockIdx.x % ListSeg::kShards, per = gridDim.x / ListSeg::kShards;
        const int count = a.count_in[sg * ListSeg::kStride];
        for (int slot = blockIdx.x / ListSeg::kShards; slot < count; slot += per)  // uniform: one wave per block
            wave_solve_one<T, NCAP, MCAP, ALL_INEQ, LFREE>(a, nc, mc, a.list_in[sg * a.list_seg + slot], bcx, bcw, mi);
        return;
    }
    for (int slot = blockIdx.x; slot < a.batch; slot += gridDim.x)  // uniform: one wave per block
        wave_solve_one<T, NCAP, MCAP, ALL_INEQ, LFREE>(a, nc, mc, a.qp0 + slot, bcx, bcw, mi);
}


// The receding-horizon stream (BASELINE config 5; the reference's loop solver.cpp:43-74 around
// controllerStep :81-108) in ONE launch.  QPs of different plants never interact, so a wave owns its
// QP for all sa.steps control steps: controllerStep (front end, warm-started solve, U += x0), then the
// simulated plant X <- Ad X + Bd U + w (lane i: row i, mpcq_plant_sim.h), then the next step.  It
// replaces a hipGraph of three launches per step, whose step lasted as long as the batch's slowest QP;
// here a wave's run lasts its own QP's iterations summed over the steps.  Every operation is the
// per-step path's (wave_solve_one, sim_row), so the trajectory is bit-identical to it.  The state
// (x', z, y, rho, X, U) goes through HBM between steps as it does between launches; one wave writes
// and reads it, ordered by workgroup-scope fences (the workgroup is this one wave).
template <typename T, int NCAP, int MCAP, bool ALL_INEQ, bool LFREE>
#ifndef MPCQ_STREAM_WPE
#define MPCQ_STREAM_WPE 2
#endif
__global__ __launch_bounds__(64, MPCQ_STREAM_WPE) void stream_wave_kernel(AdmmArgs<T> a, int nc, int mc, StreamArgs sa)
{
    static_assert(NCAP <= 64 && MCAP <= 64, "one row per lane");
    constexpr int VEC = 16 / sizeof(T);
    constexpr int BN = (NCAP + VEC - 1) / VEC * VEC, BM = (MCAP + VEC - 1) / VEC * VEC;
    __shared__ __attribute__((aligned(16))) T bcx[BN];
    __shared__ __attribute__((aligned(16))) T bcw[BM];
    __shared__ double mi[NCAP * (NCAP + 1)];
    const int lane = threadIdx.x, nx = sa.nx;
    const unsigned long long key = sim_key(sa.seed);
    for (int slot = blockIdx.x; slot < a.batch; slot += gridDim.x) {  // uniform: one wave per block
        const int b = a.qp0 + slot;
        const double *Ad = sa.Ad + (sa.shared ? 0 : (size_t)b * nx * nx);
        const double *Bd = sa.Bd + (sa.shared ? 0 : (size_t)b * nx);
        for (int k = 0; k < sa.steps; k++) {
            wave_solve_one<T, NCAP, MCAP, ALL_INEQ, LFREE>(a, nc, mc, b, bcx, bcw, mi, k == 0);
            __threadfence_block();  // this step's U (lane 0) and state before the plant update reads them
            double x[8];
#pragma unroll
            for (int t = 0; t < 8; t++) x[t] = t < nx ? a.X[(size_t)b * nx + t] : 0.0;
            const double u = a.U[b];
            const double xn = lane < nx ? sim_row(lane, nx, Ad, Bd, x, u, key, (unsigned long long)(sa.first_qp + b),
                                                  sa.first_step + k, sa.noise_std)
                                        : 0.0;
            if (lane < nx) const_cast<double *>(a.X)[(size_t)b * nx + lane] = xn;
            __threadfence_block();  // the next step's front end reads X
        }
    }
}

template <typename T, int NCAP, int MCAP>
int stream_launch(const AdmmArgs<T> &a, int nc, int mc, const StreamArgs &sa, hipStream_t s)
{
    if (a.all_ineq && a.lower_free)
        hipLaunchKernelGGL((stream_wave_kernel<T, NCAP, MCAP, true, true>), dim3(a.batch), dim3(64), 0, s, a, nc, mc, sa);
    else
        hipLaunchKernelGGL((stream_wave_kernel<T, NCAP, MCAP, false, false>), dim3(a.batch), dim3(64), 0, s, a, nc, mc, sa);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <typename T, int NCAP, int MCAP>
int wave_launch(const AdmmArgs<T> &a, int nc, int mc, int grid, hipStream_t s)
{
    if (a.all_ineq && a.lower_free)
        hipLaunchKernelGGL((admm_wave_kernel<T, NCAP, MCAP, true, true>), dim3(grid), dim3(64), 0, s, a, nc, mc);
    else
        hipLaunchKernelGGL((admm_wave_kernel<T, NCAP, MCAP, false, false>), dim3(grid), dim3(64), 0, s, a, nc, mc);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Compiled row capacities (n <= NCAP <= 64, m <= MCAP <= 64); the host picks the smallest that fits.
#define MPCQ_WAVE_CAPS(X) X(8, 16) X(16, 32) X(20, 40) X(32, 64)

template <typename T>
int wave_launch_any(const AdmmArgs<T> &a, int nc, int mc, int grid, hipStream_t s)
{
    int best = -1, bn = 0, bm = 0;
#define MPCQ_PICK(NC_, MC_)                                                  \
    if (a.n <= NC_ && a.m <= MC_ && (best < 0 || NC_ * (NC_ + MC_) < best)) { \
        best = NC_ * (NC_ + MC_); bn = NC_; bm = MC_;                         \
    }
    MPCQ_WAVE_CAPS(MPCQ_PICK)
#undef MPCQ_PICK
#define MPCQ_TRY(NC_, MC_) if (bn == NC_ && bm == MC_) return wave_launch<T, NC_, MC_>(a, nc, mc, grid, s);
    MPCQ_WAVE_CAPS(MPCQ_TRY)
#undef MPCQ_TRY
    return -1;
}

template <typename T>
int stream_launch_any(const AdmmArgs<T> &a, int nc, int mc, const StreamArgs &sa, hipStream_t s)
{
    int best = -1, bn = 0, bm = 0;
#define MPCQ_PICK(NC_, MC_)                                                  \
    if (a.n <= NC_ && a.m <= MC_ && (best < 0 || NC_ * (NC_ + MC_) < best)) { \
        best = NC_ * (NC_ + MC_); bn = NC_; bm = MC_;                         \
    }
    MPCQ_WAVE_CAPS(MPCQ_PICK)
#undef MPCQ_PICK
#define MPCQ_TRY(NC_, MC_) if (bn == NC_ && bm == MC_) return stream_launch<T, NC_, MC_>(a, nc, mc, sa, s);
    MPCQ_WAVE_CAPS(MPCQ_TRY)
#undef MPCQ_TRY
    return -1;
}

}  // namespace mpcq
