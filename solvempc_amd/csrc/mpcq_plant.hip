// solvempc_amd/csrc/mpcq_plant.hip — one pass per batch of distinct SISO plants: the reference's
// constructor (condensing, ModelPredictiveControlAPI.cpp:3-65,111-369, and initSolver -> osqp_setup,
// :64) followed by its first controllerStep (:81-108), every stage of one plant kept on chip.
// BASELINE config 3 (randomised plants, each condensed, set up and solved once).
//
// Mapping (MI355X-first): two plants per wavefront, one per 32-lane half; lane r of a half owns
// horizon step r: decision variable r, and constraint rows r and N + r of
// Gbar = [K0 L; -K0 L] (:332-347; row N + r is the negation of row r, so the pair shares its Ruiz
// scale and every A-product runs over the N distinct rows).  Per plant, in LDS (fp64): the Hessian,
// the top half of A and the KKT inverse.  Stages:
//   1. condensing (:187-207, :250-251, :305-307): CAB = Cd Ad^k Bd and Sx = Cd Ad^(k+1) by a lane-
//      parallel recurrence, the Toeplitz Su from prefix sums of CAB, then per row (one lane each)
//      P = 2 (R (N - max(i,j)) + RD delta_ij + Q sum_k Su_ki Su_kj), Fu, Fx and Fr 1 xref;
//   2. OSQP scale_data (Ruiz, cost scaling) and set_rho_vec on (P, A), the same arithmetic as
//      setup_inv_kernel (mpcq_setup_wave.hip) on the half of A it needs;
//   3. M(rho) = P^ + sigma I + sum_j rho_j a_j a_j' and its Gauss-Jordan inverse; this lane's rows of
//      sigma M^-1, (A^ M^-1)' and A^ in VGPRs;
//   4. the front end (q = Fx X + Fu U + Fr ref, u = W0 + Sbar X + Ku U; :372-375, :360-369) and the
//      ADMM of OSQP v0.6 (mpcq_wave.h's iteration, paired rows), adaptive rho refactoring M in
//      place; U += x0 when solved (:105).
// The two halves share the iteration counter (checks and adapt_rho fall on the same iterations);
// a finished half idles until its partner finishes.
#include "mpcq_wave.h"

namespace mpcq {


// 32-lane (half-wave) reductions with every lane of the half ending on the same bits: DPP within the
// 16-lane rows, then v_permlane16_swap (rows 0 <-> 1 and 2 <-> 3: never across the halves).
template <typename F> __device__ __forceinline__ float swap16(float v, F op)
{
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return op(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
template <typename F> __device__ __forceinline__ double swap16(double v, F op)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
    auto r = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    auto mk = [](unsigned l, unsigned hh) { return __longlong_as_double((long long)(((unsigned long long)hh << 32) | l)); };
    return op(mk(r[0], h[0]), mk(r[1], h[1]));
}
template <typename T, typename F> __device__ __forceinline__ T half_reduce(T v, F op)
{
    v = op(v, dpp_t<0xB1>(v));   // quad_perm [1,0,3,2]
    v = op(v, dpp_t<0x4E>(v));   // quad_perm [2,3,0,1]
    v = op(v, dpp_t<0x141>(v));  // row_half_mirror
    v = op(v, dpp_t<0x140>(v));  // row_mirror
    return swap16(v, op);
}
template <typename T> __device__ __forceinline__ T hmax(T v)
{
    return half_reduce(v, [](T a, T b) { return __builtin_fmax(a, b); });
}
template <typename T> __device__ __forceinline__ T hsum(T v)
{
    return half_reduce(v, [](T a, T b) { return a + b; });
}
__device__ __forceinline__ bool hany(bool p)  // any lane of this lane's half
{
    const unsigned long long b = __ballot(p);
    return ((threadIdx.x & 32) ? (b >> 32) : (b & 0xffffffffull)) != 0ull;
}

__device__ inline double limit_scaling_p(double d)
{
    d = d < kMinScaling ? 1.0 : d;
    return d > kMaxScaling ? kMaxScaling : d;
}

template <int NC> struct PlantLds {
    static constexpr int LD = NC + 1;  // odd row stride: column walks by lane are conflict-free
    double Ph[NC * LD], Ah[NC * LD], Mi[NC * LD];
    double CAB[NC], CS[NC], Dv[NC], Ev[NC], Dt[NC], Et[NC], qh[NC], sh[4];
};

// Gauss-Jordan inverse of this half's SPD matrix (n x n, stride LD) in place, lane r of the half
// updating row r (its own row and the pivot row in registers; no pivoting: SPD).
template <int NC>
__device__ __forceinline__ bool gj_half(double *M, int n, int r)
{
    constexpr int LD = NC + 1;
    bool ok = true;
    for (int k = 0; k < n; k++) {
        const double ip = 1.0 / M[k * LD + k];
        if (!(M[k * LD + k] > 0.0)) ok = false;
        double row[NC];
        const double f = (r < n) ? M[r * LD + k] : 0.0;
#pragma unroll
        for (int j = 0; j < NC; j++) {
            if (j >= n || r >= n) continue;
            const double mk = M[k * LD + j];
            double v;
            if (r == k && j == k) v = ip;
            else if (r == k) v = mk * ip;
            else if (j == k) v = -f * ip;
            else v = M[r * LD + j] - f * (mk * ip);
            row[j] = v;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < NC; j++)
            if (j < n && r < n) M[r * LD + j] = row[j];
        __syncthreads();
    }
    return ok;
}

template <typename T, int NC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 2))) void plant_step_kernel(PlantStepArgs a)
{
    constexpr int LD = NC + 1;
    __shared__ PlantLds<NC> lds[2];
    __shared__ __attribute__((aligned(16))) T bx[2][NC], bw[2][NC];  // per-half broadcasts
    const int lane = threadIdx.x, h = lane >> 5, r = lane & 31;
    const int plant = blockIdx.x * 2 + h;
    const bool live = plant < a.n_plants;
    const int p = live ? plant : 0;  // a dead half runs plant 0's data and publishes nothing
    const int N = a.N, n = N, nx = a.nx;
    const bool lr = r < N;
    const int rr = lr ? r : 0;
    PlantLds<NC> &S = lds[h];
    const SolverSettings &st = a.st;
    if (r < NC) {  // broadcast slots beyond N stay zero (row_dot reads the whole capacity)
        bx[h][r] = T(0);
        bw[h][r] = T(0);
    }

    // ---------------------------------------------------------------- 1. condensing
    // CAB[k] = Cd Ad^k Bd and c_k = Cd Ad^k (Sx row k-1) by the recurrences v_{k+1} = Ad v_k,
    // c_{k+1} = c_k Ad: lane t < nx of the half owns component t (scratch in Mi).
    double *V = S.Mi, *Cr = S.Mi + (NC + 1) * 8;  // V[k][8], Cr[k][8] for k <= N
    {
        const double *Ad = a.Ad + (size_t)p * nx * nx, *Bd = a.Bd + (size_t)p * nx, *Cd = a.Cd + (size_t)p * nx;
        double adr[8], adc[8];  // row t and column t of Ad
#pragma unroll
        for (int s = 0; s < 8; s++) {
            adr[s] = (r < nx && s < nx) ? Ad[r * nx + s] : 0.0;
            adc[s] = (r < nx && s < nx) ? Ad[s * nx + r] : 0.0;
        }
        if (r < 8) {
            V[r] = r < nx ? Bd[r] : 0.0;
            Cr[r] = r < nx ? Cd[r] : 0.0;
        }
        __syncthreads();
        for (int k = 0; k < N; k++) {
            double v = 0.0, c = 0.0;
#pragma unroll
            for (int s = 0; s < 8; s++) {
                v += adr[s] * V[k * 8 + s];
                c += Cr[k * 8 + s] * adc[s];
            }
            __syncthreads();
            if (r < 8) {
                V[(k + 1) * 8 + r] = v;
                Cr[(k + 1) * 8 + r] = c;
            }
            __syncthreads();
        }
        if (lr) {
            double v = 0.0;
#pragma unroll
            for (int s = 0; s < 8; s++) v += Cd[s < nx ? s : 0] * (s < nx ? V[r * 8 + s] : 0.0);
            S.CAB[r] = v;  // Cd Ad^r Bd
        }
        __syncthreads();
        if (r == 0) {
            double v = 0.0;
            for (int k = 0; k < N; k++) { v += S.CAB[k]; S.CS[k] = v; }  // Su(i, j) = CS[i - j]
        }
        __syncthreads();
    }
    const double Q = a.Q[p], R = a.R[p], RD = a.RD[p];
    const double *K = a.K + (size_t)p * nx;
    const double K0 = K[0];
    // row r of P (setH :250-251: H1 = 2 (LL' Rbar LL + RbarD + Su' Qbar Su), symmetric as computed, so
    // (H1 + H1') / 2 = H1), Fu[r] (:305, incl. the diagonal() quirk: R 1), Fr 1 xref (:306, :374),
    // Fx row r (:307)
    double Fu = 0.0, frr = 0.0, Fx[8];
    if (lr) {
        for (int j = 0; j < N; j++) {
            const int mx = r > j ? r : j;
            double t4 = 0.0;
            for (int k = mx; k < N; k++) t4 += (S.CS[k - r] * Q) * S.CS[k - j];
            S.Ph[r * LD + j] = 2.0 * ((R * (double)(N - mx) + (r == j ? RD : 0.0)) + t4);
        }
        double s1 = 0.0, sf = 0.0;
        for (int k = r; k < N; k++) {
            s1 += (S.CS[k] * Q) * S.CS[k - r];
            sf += -2.0 * (Q * S.CS[k - r]) * a.xref;
        }
        Fu = 2.0 * (R + s1);
        frr = sf;
#pragma unroll
        for (int c = 0; c < 8; c++) {
            double v = 0.0;
            if (c < nx)
                for (int k = r; k < N; k++) v += (Cr[(k + 1) * 8 + c] * Q) * S.CS[k - r];
            Fx[c] = 2.0 * v;
        }
        for (int j = 0; j < N; j++) S.Ah[r * LD + j] = (j <= r) ? K0 : 0.0;  // top half of Gbar
        S.Dv[r] = 1.0;
        S.Ev[r] = 1.0;
        S.qh[r] = 0.0;  // the ctor's setup gradient (X = U = 0, xref = 0 in the reference config)
    }
    if (r == 0) S.sh[0] = 1.0;
    __syncthreads();

    // ---------------------------------------------------------------- 2. scale_data (Ruiz)
    // setup_inv_kernel's arithmetic; the bottom rows of A are the negated top rows, so their column
    // and row norms are the top ones and E is the same for rows r and N + r.
    double cp = 1.0;
    for (int it = 0; it < st.scaling; it++) {
        if (lr) {
            double vp = 0.0, va = 0.0, ve = 0.0;
            for (int i = 0; i < n; i++) vp = fmax(vp, fabs(S.Ph[i * LD + r]));
            for (int i = 0; i < n; i++) va = fmax(va, fabs(S.Ah[i * LD + r]));
            for (int j = 0; j < n; j++) ve = fmax(ve, fabs(S.Ah[r * LD + j]));
            S.Dt[r] = 1.0 / sqrt(limit_scaling_p(fmax(cp * vp, va)));
            S.Et[r] = 1.0 / sqrt(limit_scaling_p(ve));
        }
        __syncthreads();
        if (lr) {
            const double dr = S.Dt[r], er = S.Et[r];
            for (int k = 0; k < n; k++) {
                S.Ph[r * LD + k] = (dr * (S.Ph[r * LD + k] * cp)) * S.Dt[k];
                S.Ah[r * LD + k] = (er * S.Ah[r * LD + k]) * S.Dt[k];
            }
            S.qh[r] *= dr;
            S.Dv[r] *= dr;
            S.Ev[r] *= er;
        }
        __syncthreads();
        if (lr) {
            double v = 0.0;
            for (int i = 0; i < n; i++) v = fmax(v, fabs(S.Ph[i * LD + r]));
            S.Dt[r] = v;
        }
        __syncthreads();
        if (r == 0) {
            double mean = 0.0, qn = 0.0;
            for (int j = 0; j < n; j++) mean += S.Dt[j];
            mean /= n;
            for (int j = 0; j < n; j++) qn = fmax(qn, fabs(S.qh[j]));
            qn = limit_scaling_p(qn);
            const double ct = 1.0 / limit_scaling_p(fmax(mean, qn));
            S.sh[1] = ct;
            S.sh[0] *= ct;
        }
        __syncthreads();
        cp = S.sh[1];
        if (lr) S.qh[r] *= cp;
    }
    if (st.scaling > 0) {
        if (lr)
            for (int k = 0; k < n; k++) S.Ph[r * LD + k] *= cp;
        __syncthreads();
    }
    const double cost = S.sh[0], cinv = 1.0 / cost;
    // set_rho_vec: l = -DBL_MAX (:42) and u0 = W0 = 255 (:43, X = U = 0): every row an inequality
    // (the rows' type is checked again below against this step's bounds)
    const double Er = lr ? S.Ev[r] : 1.0, Dr = lr ? S.Dv[r] : 1.0;

    // ---------------------------------------------------------------- 3. M(rho)^-1, operator rows
    T Srow[NC], Btc[NC], Brow[NC];  // sigma M^-1 row r; (A^ M^-1) column r (top rows); A^ row r
    auto build_inverse = [&](double rho) -> bool {
        __syncthreads();
        if (lr)
            for (int k = 0; k < n; k++) {
                double v = S.Ph[r * LD + k] + (r == k ? st.sigma : 0.0);
                for (int pass = 0; pass < 2; pass++)  // rows j (top) then N + j (bottom: (-a)(-a)' = a a')
                    for (int j = 0; j < n; j++) v += rho * (S.Ah[j * LD + r] * S.Ah[j * LD + k]);
                S.Mi[r * LD + k] = v;
            }
        __syncthreads();
        const bool ok = gj_half<NC>(S.Mi, n, r);
#pragma unroll
        for (int i = 0; i < NC; i++) {
            Srow[i] = (lr && i < n) ? (T)(st.sigma * S.Mi[rr * LD + i]) : T(0);
            Brow[i] = (lr && i < n) ? (T)S.Ah[rr * LD + i] : T(0);
            double bt = 0.0;
            if (lr && i < n)
                for (int k = 0; k < n; k++) bt += S.Ah[i * LD + k] * S.Mi[k * LD + rr];
            Btc[i] = (T)bt;
        }
        return ok;
    };
    const double rho0 = fmin(fmax(st.rho, kRhoMin), kRhoMax);
    const bool setup_ok = build_inverse(rho0);

    // ---------------------------------------------------------------- 4. controllerStep
    double Xv[8];
    const double *Xp = a.X + (size_t)p * nx;
#pragma unroll
    for (int c = 0; c < 8; c++) Xv[c] = c < nx ? Xp[c] : 0.0;
    const double Uv = a.U[p];
    double kx = 0.0;  // K X (Sbar rows < s_rows, :185,208)
#pragma unroll
    for (int c = 0; c < 8; c++)
        if (c < nx) kx += K[c] * Xv[c];
    T qh = T(0), ut = T(kInfty), ub = T(kInfty);
    double qs = 0.0;
    if (lr) {
        double s0 = 0.0;
#pragma unroll
        for (int c = 0; c < 8; c++)
            if (c < nx) s0 += Fx[c] * Xv[c];
        const double qk = s0 + Fu * Uv + frr;                 // setF (:374)
        const double sx = r < a.s_rows ? kx : 0.0;
        const double up_t = 255.0 + sx + (-K0) * Uv;          // W0 + Sbar X + Ku U (:43, :99)
        const double up_b = 255.0 + (-sx) + K0 * Uv;
        qs = (qk * Dr) * cost;                                // q^ = c D q (osqp_update_lin_cost)
        qh = (T)qs;
        ut = (T)(up_t * Er);                                  // u^ = E u (osqp_update_upper_bound)
        ub = (T)(up_b * Er);
    }
    // the update's checks (l^ = -DBL_MAX E stays free of -OSQP_INFTY MIN_SCALING): u < l cannot occur;
    // a row whose u^ reaches OSQP_INFTY MIN_SCALING would change type (TYPE_CHANGED)
    int status = hany(lr && ((double)ut > kInfty * kMinScaling || (double)ub > kInfty * kMinScaling)) ? kTypeChanged
                                                                                                     : kUnsolved;
    if (!setup_ok) status = kNonCvx;
    if (!live) status = kSolved;  // (never published)
    // g = -M^-1 q^ (column r of the symmetric M^-1)
    auto make_g = [&]() -> T {
        double g = 0.0;
        if (lr)
            for (int i = 0; i < n; i++) g += S.Mi[i * LD + r] * (double)(T)S.qh[i];
        return lr ? (T)(-g) : T(0);
    };
    __syncthreads();
    if (lr) S.qh[r] = qs;  // (the setup copy of q^ is dead: reuse its slot for this step's q^)
    __syncthreads();
    T gk = make_g();

    T xs = T(0), zt = T(0), zb = T(0), yt = T(0), yb = T(0);
    T rho = (T)rho0, rinv = T(1) / rho;
    const T alpha = (T)st.alpha, oma = T(1) - (T)st.alpha;
    const T eps_abs = (T)st.eps_abs, eps_rel = (T)st.eps_rel;
    const T EiT = (T)(1.0 / Er), DiT = (T)(1.0 / Dr), ErT = (T)Er, cinvT = (T)cinv;
    const bool scaled_term = st.scaled_termination != 0;
    const int ct = st.check_termination;
    const int ai = (st.adaptive_rho && a.adaptive_interval) ? a.adaptive_interval : 0;
    int next_check = ct ? ct : -1, next_adapt = ai ? ai : -1;
    int it = 0;
    bool done = status != kUnsolved;
    bool refactor = false;
    T *bxh = bx[h], *bwh = bw[h];

    auto finalize = [&]() {
        const bool has_sol = status == kSolved || status == kSolvedInaccurate || status == kMaxIterReached;
        if (!live) return;
        if (lr) {
            const double xv = has_sol ? (double)xs * Dr : __builtin_nan("");
            a.x[(size_t)plant * n + r] = xv;
            if (r == 0) {
                if (status == kSolved) a.U[plant] = Uv + xv;  // U += x0 (:105)
                a.status[plant] = status;
                a.iter[plant] = it;
                a.rho_out[plant] = (double)rho;
            }
            a.y[(size_t)plant * 2 * n + r] = has_sol ? ((double)yt * Er) * cinv : __builtin_nan("");
            a.y[(size_t)plant * 2 * n + n + r] = has_sol ? ((double)yb * Er) * cinv : __builtin_nan("");
        }
    };
    if (done) finalize();

    while (!wave_all(done)) {
        if (refactor) {  // OSQP's KKT refactorisation after a rho change (each half at its own rho; a
                         // half whose rho did not move rebuilds the same bits)
            build_inverse((double)rho);
            gk = make_g();
            refactor = false;
        }
        it++;
        const bool at_check = it == next_check, at_adapt = it == next_adapt;
        if (at_check) next_check += ct;
        if (at_adapt) next_adapt += ai;
        const bool last = it == st.max_iter;
        const bool info = at_check || at_adapt || last;

        // xi = g + sigma M^-1 x + (A^ M^-1)' (w_top - w_bot),  w = rho z - y
        const T wt = tt_fma(rho, zt, -yt) - tt_fma(rho, zb, -yb);
        __syncthreads();
        if (lr) { bxh[r] = xs; bwh[r] = wt; }
        __syncthreads();
        const T xi = row_dot(Srow, bxh, gk) + row_dot(Btc, bwh, T(0));
        const T xn = lr ? tt_fma(alpha, xi, oma * xs) : T(0);
        const T dx = xn - xs;
        if (!done) xs = xn;
        // z~ = A^ x~ (top rows; bottom = -top), relaxation, projection onto [l, u], dual update
        __syncthreads();
        if (lr) bxh[r] = xi;
        __syncthreads();
        const T zz = row_dot(Brow, bxh, T(0));
        T dyt = T(0), dyb = T(0);
        if (lr && !done) {
            T v = tt_fma(alpha, zz, oma * zt);
            T zn = __builtin_fmin(tt_fma(rinv, yt, v), ut);
            dyt = rho * (v - zn);
            yt = tt_fma(rho, v - zn, yt);
            zt = zn;
            v = tt_fma(alpha, -zz, oma * zb);
            zn = __builtin_fmin(tt_fma(rinv, yb, v), ub);
            dyb = rho * (v - zn);
            yb = tt_fma(rho, v - zn, yb);
            zb = zn;
        }
        if (!info) continue;

        // ---- update_info: residuals (half-wave reductions)
        __syncthreads();
        if (lr) { bxh[r] = xs; bwh[r] = yt - yb; }
        __syncthreads();
        T ax_z = 0, ax_zs = 0, zn_s = 0, zn_r = 0, axn_s = 0, axn_r = 0;
        T dr_r = 0, dr_s = 0, qn_r = 0, qn_s = 0, atyn_r = 0, atyn_s = 0, pxn_r = 0, pxn_s = 0;
        if (lr) {
            const T ax = row_dot(Brow, bxh, T(0));
            const T r1 = ax - zt, r2 = -ax - zb;
            ax_z = __builtin_fmax(__builtin_fabs(r1), __builtin_fabs(r2));
            ax_zs = __builtin_fmax(__builtin_fabs(EiT * r1), __builtin_fabs(EiT * r2));
            zn_r = __builtin_fmax(__builtin_fabs(zt), __builtin_fabs(zb));
            zn_s = __builtin_fmax(__builtin_fabs(EiT * zt), __builtin_fabs(EiT * zb));
            axn_r = __builtin_fabs(ax);
            axn_s = __builtin_fabs(EiT * ax);
            T px = T(0), aty = T(0);
            for (int i = 0; i < n; i++) {
                px = tt_fma((T)S.Ph[r * LD + i], bxh[i], px);
                aty = tt_fma((T)S.Ah[i * LD + r], bwh[i], aty);
            }
            const T rd = (qh + px) + aty;
            dr_r = __builtin_fabs(rd);
            dr_s = __builtin_fabs(DiT * rd);
            qn_r = __builtin_fabs(qh);
            qn_s = __builtin_fabs(DiT * qh);
            atyn_r = __builtin_fabs(aty);
            atyn_s = __builtin_fabs(DiT * aty);
            pxn_r = __builtin_fabs(px);
            pxn_s = __builtin_fabs(DiT * px);
        }
        ax_z = hmax(ax_z); ax_zs = hmax(ax_zs); zn_s = hmax(zn_s); zn_r = hmax(zn_r);
        axn_s = hmax(axn_s); axn_r = hmax(axn_r);
        dr_r = hmax(dr_r); dr_s = hmax(dr_s); qn_r = hmax(qn_r); qn_s = hmax(qn_s);
        atyn_r = hmax(atyn_r); atyn_s = hmax(atyn_s); pxn_r = hmax(pxn_r); pxn_s = hmax(pxn_s);
        const T pri_res = scaled_term ? ax_z : ax_zs;
        const T dua_res = scaled_term ? dr_r : cinvT * dr_s;

        // OSQP is_primal_infeasible on delta_y (l = -inf: d = max(dy, 0) on every row)
        auto primal_infeasible = [&](T eps) -> bool {
            const T d1 = tt_max(dyt, T(0)), d2 = tt_max(dyb, T(0));
            T ndy = lr ? __builtin_fmax(__builtin_fabs(scaled_term ? d1 : ErT * d1), __builtin_fabs(scaled_term ? d2 : ErT * d2)) : T(0);
            T lhs = lr ? ut * d1 + ub * d2 : T(0);
            ndy = hmax(ndy);
            lhs = hsum(lhs);
            const bool cand = ndy > T(kDivisionTol) && lhs < eps * ndy;
            __syncthreads();
            if (lr) bwh[r] = d1 - d2;
            __syncthreads();
            T atd = T(0);
            if (lr)
                for (int i = 0; i < n; i++) atd = tt_fma((T)S.Ah[i * LD + r], bwh[i], atd);
            const T nat = hmax(lr ? __builtin_fabs(scaled_term ? atd : DiT * atd) : T(0));
            return cand && nat < eps * ndy;
        };
        // OSQP is_dual_infeasible on delta_x
        auto dual_infeasible = [&](T eps) -> bool {
            const T qdx = hsum(lr ? qh * dx : T(0));
            __syncthreads();
            if (lr) bxh[r] = dx;
            __syncthreads();
            T t2 = T(0);
            if (lr)
                for (int i = 0; i < n; i++) t2 = tt_fma((T)S.Ph[r * LD + i], bxh[i], t2);
            const T t3 = row_dot(Brow, bxh, T(0));
            const T ndx = hmax(lr ? __builtin_fabs(scaled_term ? dx : (T)Dr * dx) : T(0));
            const T cs = scaled_term ? T(1) : (T)cost;
            const T npdx = hmax(lr ? __builtin_fabs(scaled_term ? t2 : DiT * t2) : T(0));
            const T sv = scaled_term ? t3 : EiT * t3;
            const bool viol = hany(lr && (sv > eps * ndx || -sv > eps * ndx));  // rows r (u finite), N + r (-A x)
            return ndx > T(kDivisionTol) && qdx < -cs * eps * ndx && npdx < cs * eps * ndx && !viol;
        };
        auto check_termination = [&](bool approx) -> int {
            const T mul = approx ? T(10) : T(1);
            if (pri_res > T(kInfty) || dua_res > T(kInfty)) return kNonCvx;
            const T ea = eps_abs * mul, er = eps_rel * mul;
            bool prim_ok = false, dual_ok = false, prim_inf = false, dual_inf = false;
            const T ep = ea + er * (scaled_term ? tt_max(zn_r, axn_r) : tt_max(zn_s, axn_s));
            if (pri_res < ep) prim_ok = true;
            const bool pi = primal_infeasible((T)st.eps_prim_inf * mul);  // (uniform: evaluated for both halves)
            if (!prim_ok) prim_inf = pi;
            const T ed = ea + er * (scaled_term ? tt_max(tt_max(qn_r, atyn_r), pxn_r)
                                                : cinvT * tt_max(tt_max(qn_s, atyn_s), pxn_s));
            if (dua_res < ed) dual_ok = true;
            const bool di = dual_infeasible((T)st.eps_dual_inf * mul);
            if (!dual_ok) dual_inf = di;
            if (prim_ok && dual_ok) return approx ? kSolvedInaccurate : kSolved;
            if (prim_inf) return approx ? kPrimalInfeasibleInaccurate : kPrimalInfeasible;
            if (dual_inf) return approx ? kDualInfeasibleInaccurate : kDualInfeasible;
            return kUnsolved;
        };

        bool term = false;
        if (at_check) {
            const int s0 = check_termination(false);
            if (!done && s0 != kUnsolved) { status = s0; term = true; }
        }
        if (!term && at_adapt) {
            const T pr = ax_z / (tt_max(zn_r, axn_r) + T(kDivisionTol));
            const T dn = tt_max(tt_max(qn_r, atyn_r), pxn_r);
            const T du = dr_r / (dn + T(kDivisionTol));
            T rn = rho * (T)sqrt((double)(pr / (du + T(kDivisionTol))));
            rn = tt_min(tt_max(rn, T(kRhoMin)), T(kRhoMax));
            if (!done && (rn > rho * (T)st.adaptive_rho_tolerance || rn < rho / (T)st.adaptive_rho_tolerance)) {
                rho = tt_min(tt_max(rn, T(kRhoMin)), T(kRhoMax));
                rinv = T(1) / rho;
                refactor = true;
            }
        }
        if (last) {
            if (!at_check) {
                const int s1 = check_termination(false);
                if (!done && !term && s1 != kUnsolved) { status = s1; term = true; }
            }
            const int s2 = check_termination(true);
            if (!done && !term) { status = s2 != kUnsolved ? s2 : kMaxIterReached; term = true; }
        }
        refactor = wave_any(refactor);  // uniform (the other half rebuilds its own M at its own rho)
        if (term) {
            finalize();
            done = true;
        }
    }
    if (threadIdx.x == 0 && !wave_all(setup_ok || !live)) atomicOr(a.flags, 1);
}

template <typename T, int NC>
int plant_step_launch_t(const PlantStepArgs &a, hipStream_t s)
{
    hipLaunchKernelGGL((plant_step_kernel<T, NC>), dim3((a.n_plants + 1) / 2), dim3(64), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace mpcq

extern "C" int mpcq_internal_plant_step_launch(const mpcq::PlantStepArgs *a, int is_f32, hipStream_t s)
{
    if (a->N < 1 || a->N > 32 || a->nx < 1 || a->nx > 8) return -1;
    if (a->N <= 16) return is_f32 ? mpcq::plant_step_launch_t<float, 16>(*a, s) : mpcq::plant_step_launch_t<double, 16>(*a, s);
    if (a->N <= 20) return is_f32 ? mpcq::plant_step_launch_t<float, 20>(*a, s) : mpcq::plant_step_launch_t<double, 20>(*a, s);
    return is_f32 ? mpcq::plant_step_launch_t<float, 32>(*a, s) : mpcq::plant_step_launch_t<double, 32>(*a, s);
}
