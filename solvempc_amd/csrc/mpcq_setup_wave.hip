// solvempc_amd/csrc/mpcq_setup_wave.hip — per-plant QP setup, one wavefront per plant, LDS-resident.
//
// Same computation and output block as setup_kernel (mpcq_setup.hip; osqp_setup behind
// OsqpEigen::Solver::initSolver, ModelPredictiveControlAPI.cpp:64), restructured for batches of
// distinct plants (BASELINE config 3): every matrix of the plant lives in LDS (fp64, row stride
// ld = odd, so column walks by lane are conflict-free), and the O(n^3) stages run wave-parallel:
//   * Ruiz passes: lane-per-column / lane-per-row maxima, element-parallel rescale; the cost
//     scaling sums run serially on lane 0 in the order of setup_kernel (same c bit for bit);
//   * Cholesky of P~ and the triangular solves for C = L^-1 G L^-T: right-looking, one column (or
//     row) step at a time, the trailing update spread over the 64 lanes;
//   * Jacobi on C with the round-robin ("circle") ordering: ne/2 disjoint rotations per round, each
//     2x2 block of C owned by one lane, so a round is two LDS passes and no serial rotation chain;
//   * W = L^-T V, W^-1 = V' L', and the operator products element-parallel into the global block.
// A single-wave workgroup makes every __syncthreads a wave-level ordering point (no s_barrier cost).
// Shapes n <= 32, m <= 64 (the wave kernel's capacities); larger plants use setup_kernel.
#include "mpcq_internal.h"

namespace mpcq {

// Debug hook (MPCQ_SETUP_PROF): per-plant shader-clock stamps at the stage boundaries.
#define MPCQ_STAMP(k) \
    do { if (a.prof && t == 0) a.prof[(size_t)pl * 16 + (k)] = (long long)clock64(); } while (0)

struct SetupWaveShape {
    int n, m, ne, ld;
    size_t Ph, Ah, L, T, C, V, Dv, Ev, Dt, Et, qh, rot, total;  // offsets in doubles
    __host__ __device__ static SetupWaveShape make(int n, int m)
    {
        SetupWaveShape s{};
        s.n = n; s.m = m;
        s.ne = n + (n & 1);      // Jacobi pads to an even order (the pad row/column stays decoupled)
        s.ld = s.ne + 1;         // odd stride
        size_t o = 0;
        s.Ph = o; o += (size_t)n * s.ld;
        s.Ah = o; o += (size_t)m * s.ld;
        s.L = o;  o += (size_t)n * s.ld;
        s.T = o;  o += (size_t)s.ne * s.ld;
        s.C = o;  o += (size_t)s.ne * s.ld;
        s.V = s.T;  // V reuses T's space: T (L^-1 G) is dead once C = T' is formed
        s.Dv = o; o += n;
        s.Ev = o; o += m;
        s.Dt = o; o += n;
        s.Et = o; o += m;
        s.qh = o; o += n;
        s.rot = o; o += 5 * 16;  // per pair: c, s, new app, new aqq, (p | q << 8)
        s.total = o + 8;         // + cost-scaling slots
        return s;
    }
};

__device__ inline double limit_scaling_w(double d)
{
    d = d < kMinScaling ? 1.0 : d;
    return d > kMaxScaling ? kMaxScaling : d;
}

// Whole-wave sum with every lane ending on the same bits (symmetric pairwise adds): DPP quad swaps and
// row mirrors, then the 16/32-lane swaps (VALU only; a __shfl_xor ladder is 12 LDS-path permutes).
template <int CTRL> __device__ inline double dpp_f64(double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)u, (int)(unsigned)u, CTRL, 0xF, 0xF, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)(u >> 32), (int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ inline double swap_sum_f64(double v, bool w32)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
    auto r = w32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false) : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto h = w32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false) : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    auto mk = [](unsigned l, unsigned hh) { return __longlong_as_double((long long)(((unsigned long long)hh << 32) | l)); };
    return mk(r[0], h[0]) + mk(r[1], h[1]);
}
__device__ inline double wave_sum(double v)
{
    v = v + dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
    v = v + dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
    v = v + dpp_f64<0x141>(v);  // row_half_mirror
    v = v + dpp_f64<0x140>(v);  // row_mirror
    v = swap_sum_f64(v, false);
    return swap_sum_f64(v, true);
}

// Pair u of round r of the circle ordering on ne (even) indices.
__device__ inline void circle_pair(int r, int u, int ne, int &p, int &q)
{
    const int k = ne - 1;
    if (u == 0) { p = r; q = k; }
    else { p = (r + u) % k; q = (r - u + k) % k; }
}

// OSQP scale_data (Ruiz equilibration + cost normalisation) and set_rho_vec's constraint typing, on
// the LDS-resident plant (one wave).  On exit Ph, Ah hold P^, A^; Dv, Ev the scalings; Et the rho
// scale of each row (0 free, 1 inequality, RHO_EQ_OVER_RHO_INEQ equality); returns c.
__device__ double ruiz_and_types(const SetupArgs &a, int pl, int t, int n, int m, int mc, int ld, double *Ph,
                                 double *Ah, double *Dv, double *Ev, double *Dt, double *Et, double *qh, double *sh,
                                 int *ctype)
{
    const double *l0 = a.l0 + (size_t)pl * m;
    const double *u0 = a.u0 + (size_t)pl * m;
    // ---- Ruiz equilibration + cost normalisation (OSQP scale_data).  A pass's cost factor ct is not
    // swept over P^ on its own: it stays pending (cp) and is applied inside the next pass's column
    // norms (max |cp P| = cp max |P|: rounding is monotone) and D-scaling, or by one sweep after the
    // last pass, so every P^ element is rounded exactly as in the eager order.
    double cp = 1.0;
    for (int it = 0; it < a.scaling; it++) {
        if (t < n) {
            double vp = 0.0, va = 0.0;
            for (int i = 0; i < n; i++) vp = fmax(vp, fabs(Ph[i * ld + t]));
            for (int i = 0; i < m; i++) va = fmax(va, fabs(Ah[i * ld + t]));
            Dt[t] = 1.0 / sqrt(limit_scaling_w(fmax(cp * vp, va)));
        }
        for (int i = t; i < m; i += 64) {
            double v = 0.0;
            for (int j = 0; j < n; j++) v = fmax(v, fabs(Ah[i * ld + j]));
            Et[i] = 1.0 / sqrt(limit_scaling_w(v));
        }
        __syncthreads();
        for (int e = t; e < n * n; e += 64) {
            const int i = e / n, k = e % n;
            Ph[i * ld + k] = (Dt[i] * (Ph[i * ld + k] * cp)) * Dt[k];
        }
        for (int e = t; e < m * n; e += 64) {
            const int i = e / n, k = e % n;
            Ah[i * ld + k] = (Et[i] * Ah[i * ld + k]) * Dt[k];
        }
        if (t < n) { qh[t] *= Dt[t]; Dv[t] *= Dt[t]; }
        for (int i = t; i < m; i += 64) Ev[i] *= Et[i];
        __syncthreads();
        if (t < n) {
            double v = 0.0;
            for (int i = 0; i < n; i++) v = fmax(v, fabs(Ph[i * ld + t]));
            Dt[t] = v;
        }
        __syncthreads();
        if (t == 0) {
            double mean = 0.0, qn = 0.0;
            for (int j = 0; j < n; j++) mean += Dt[j];
            mean /= n;
            for (int j = 0; j < n; j++) qn = fmax(qn, fabs(qh[j]));
            qn = limit_scaling_w(qn);
            const double ct = 1.0 / limit_scaling_w(fmax(mean, qn));
            sh[1] = ct;
            sh[0] *= ct;
        }
        __syncthreads();
        cp = sh[1];  // (sh[1] is next written three barriers on)
        if (t < n) qh[t] *= cp;
    }
    if (a.scaling > 0) {
        for (int e = t; e < n * n; e += 64) Ph[(e / n) * ld + e % n] *= cp;
        __syncthreads();
    }
    const double cost = sh[0];

    // ---- constraint types from the scaled setup bounds (OSQP set_rho_vec); Et <- rscale
    for (int i = t; i < m; i += 64) {
        const double lo = l0[i] * Ev[i], up = u0[i] * Ev[i];
        int ty;
        double rs;
        if (lo < -kInfty * kMinScaling && up > kInfty * kMinScaling) { ty = -1; rs = 0.0; }
        else if (up - lo < kRhoTol) { ty = 1; rs = kRhoEqOverIneq; }
        else { ty = 0; rs = 1.0; }
        ctype[i] = ty;
        Et[i] = rs;
        if (ty != 0) atomicOr(a.flags, 2);
    }
    for (int i = m + t; i < mc; i += 64) ctype[i] = 0;
    __syncthreads();

    return cost;
}

__global__ __launch_bounds__(64) void setup_wave_kernel(SetupArgs a)
{
    extern __shared__ double sm[];
    const int pl = blockIdx.x;
    if (pl >= a.n_plants) return;
    const int t = threadIdx.x;
    const int n = a.n, m = a.m, nc = a.nc, mc = a.mc;
    const SetupWaveShape S = SetupWaveShape::make(n, m);
    const int ld = S.ld, ne = S.ne;
    double *Ph = sm + S.Ph, *Ah = sm + S.Ah, *L = sm + S.L, *Tm = sm + S.T, *C = sm + S.C, *V = sm + S.V;
    double *Dv = sm + S.Dv, *Ev = sm + S.Ev, *Dt = sm + S.Dt, *Et = sm + S.Et, *qh = sm + S.qh;
    double *rot = sm + S.rot, *sh = sm + S.total - 8;

    const double *P = a.P + (size_t)pl * n * n;
    const double *q0 = a.q0 + (size_t)pl * n;
    const double *A = a.A + (size_t)pl * m * n;
    const OpsLayout Lo = OpsLayout::make(nc, mc);
    double *out = a.ops + (size_t)pl * Lo.total;
    int *ctype = a.ctype + (size_t)pl * mc;

    MPCQ_STAMP(0);
    // ---- data (osqp-eigen keeps the upper triangle of the Hessian)
    for (int e = t; e < n * n; e += 64) {
        const int i = e / n, j = e % n;
        Ph[i * ld + j] = (i <= j) ? P[i * n + j] : P[j * n + i];
    }
    for (int e = t; e < m * n; e += 64) Ah[(e / n) * ld + e % n] = A[e];
    for (int j = t; j < n; j += 64) { qh[j] = q0[j]; Dv[j] = 1.0; }
    for (int i = t; i < m; i += 64) Ev[i] = 1.0;
    if (t == 0) sh[0] = 1.0;
    __syncthreads();

    MPCQ_STAMP(1);
    const double cost = ruiz_and_types(a, pl, t, n, m, mc, ld, Ph, Ah, Dv, Ev, Dt, Et, qh, sh, ctype);
    MPCQ_STAMP(3);
    // ---- P~ = P^ + sigma I + RHO_MIN sum_free a a' (into L), G = sum rscale a a' (into Tm)
    for (int e = t; e < n * n; e += 64) {
        const int i = e / n, k = e % n;
        double pt = Ph[i * ld + k] + (i == k ? a.sigma : 0.0), g = 0.0;
        for (int r = 0; r < m; r++) {
            const double aa = Ah[r * ld + i] * Ah[r * ld + k];
            const double rs = Et[r];
            if (rs == 0.0) pt += kRhoMin * aa;
            else g += rs * aa;
        }
        L[i * ld + k] = pt;
        Tm[i * ld + k] = g;
    }
    __syncthreads();

    MPCQ_STAMP(4);
    // ---- Cholesky P~ = L L' in place (right-looking; upper triangle zeroed at the end)
    int fail = 0;
    for (int j = 0; j < n; j++) {
        double d = L[j * ld + j];
        if (!(d > 0.0)) { fail = 1; d = 1.0; }
        d = sqrt(d);
        __syncthreads();
        if (t == 0) L[j * ld + j] = d;
        for (int i = j + 1 + t; i < n; i += 64) L[i * ld + j] /= d;
        __syncthreads();
        const int w = n - j - 1;  // trailing lower triangle rows/cols j+1..n-1
        for (int e = t; e < w * w; e += 64) {
            const int i = j + 1 + e / w, k = j + 1 + e % w;
            if (k <= i) L[i * ld + k] -= L[i * ld + j] * L[k * ld + j];
        }
        __syncthreads();
    }
    for (int e = t; e < n * n; e += 64) {
        const int i = e / n, k = e % n;
        if (k > i) L[i * ld + k] = 0.0;
    }
    __syncthreads();

    MPCQ_STAMP(5);
    // ---- C = L^-1 G L^-T: Tm <- L^-1 G (row steps), C <- Tm', C <- L^-1 C, symmetrise
    for (int i = 0; i < n; i++) {
        const double li = L[i * ld + i];
        if (t < n) Tm[i * ld + t] /= li;
        __syncthreads();
        for (int e = t; e < (n - i - 1) * n; e += 64) {
            const int r = i + 1 + e / n, c = e % n;
            Tm[r * ld + c] -= L[r * ld + i] * Tm[i * ld + c];
        }
        __syncthreads();
    }
    for (int e = t; e < ne * ne; e += 64) {
        const int i = e / ne, k = e % ne;
        C[i * ld + k] = (i < n && k < n) ? Tm[k * ld + i] : 0.0;
    }
    __syncthreads();
    for (int e = t; e < ne * ne; e += 64) {  // (V aliases Tm)
        const int i = e / ne, k = e % ne;
        V[i * ld + k] = (i == k) ? 1.0 : 0.0;
    }
    __syncthreads();
    for (int i = 0; i < n; i++) {
        const double li = L[i * ld + i];
        if (t < n) C[i * ld + t] /= li;
        __syncthreads();
        for (int e = t; e < (n - i - 1) * n; e += 64) {
            const int r = i + 1 + e / n, c = e % n;
            C[r * ld + c] -= L[r * ld + i] * C[i * ld + c];
        }
        __syncthreads();
    }
    for (int e = t; e < n * n; e += 64) {
        const int i = e / n, k = e % n;
        if (i < k) {
            const double v = 0.5 * (C[i * ld + k] + C[k * ld + i]);
            C[i * ld + k] = v;
            C[k * ld + i] = v;
        }
    }
    __syncthreads();

    MPCQ_STAMP(6);
    // ---- parallel-ordering Jacobi: C = V diag(lambda) V'
    const int np = ne / 2, nblk = np * (np + 1) / 2;
    // Block b = t of the upper-triangular pair grid, decoded once (the grid is the same every round).
    const int dq64 = np > 0 ? 64 / np : 0, dr64 = np > 0 ? 64 % np : 0;  // (row, u) step of the V-update walk (e += 64)
    int bu0 = 0, bv0 = 0;
    {
        int bb = t;
        while (bu0 < np && bb >= np - bu0) { bb -= np - bu0; bu0++; }
        bv0 = bu0 + bb;
    }
    bool converged = ne <= 1;
    for (int sweep = 0; sweep < 60 && ne > 1; sweep++) {
        double off = 0.0, dia = 0.0;
        for (int e = t; e < n * n; e += 64) {
            const int i = e / n, k = e % n;
            const double v = C[i * ld + k] * C[i * ld + k];
            if (i == k) dia += v; else off += v;
        }
        off = wave_sum(off);
        dia = wave_sum(dia);
        if (a.prof && t == 0) a.prof[(size_t)pl * 16 + 15] = sweep;
        if (off <= a.jacobi_tol * dia || off < 1e-300) { converged = true; break; }
        for (int r = 0; r < ne - 1; r++) {
            if (t < np) {
                int pp, qq;
                circle_pair(r, t, ne, pp, qq);
                const double apq = C[pp * ld + qq], app = C[pp * ld + pp], aqq = C[qq * ld + qq];
                double cs = 1.0, sn = 0.0, tt = 0.0;
                if (apq != 0.0) {
                    const double theta = (aqq - app) / (2.0 * apq);
                    tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                    cs = 1.0 / sqrt(tt * tt + 1.0);
                    sn = tt * cs;
                }
                rot[5 * t + 0] = cs;
                rot[5 * t + 1] = sn;
                rot[5 * t + 2] = app - tt * apq;
                rot[5 * t + 3] = aqq + tt * apq;
                rot[5 * t + 4] = (double)(pp | (qq << 8));
            }
            __syncthreads();
            for (int b = t; b < nblk; b += 64) {
                int u = bu0, v = bv0;
                if (b != t) {
                    int bb = b;
                    u = 0;
                    while (bb >= np - u) { bb -= np - u; u++; }
                    v = u + bb;
                }
                const int pu = (int)rot[5 * u + 4] & 255, qu = (int)rot[5 * u + 4] >> 8;
                if (u == v) {
                    C[pu * ld + pu] = rot[5 * u + 2];
                    C[qu * ld + qu] = rot[5 * u + 3];
                    C[pu * ld + qu] = 0.0;
                    C[qu * ld + pu] = 0.0;
                } else {
                    const int pv = (int)rot[5 * v + 4] & 255, qv = (int)rot[5 * v + 4] >> 8;
                    const double cu = rot[5 * u], su = rot[5 * u + 1], cv = rot[5 * v], sv = rot[5 * v + 1];
                    const double x00 = C[pu * ld + pv], x01 = C[pu * ld + qv];
                    const double x10 = C[qu * ld + pv], x11 = C[qu * ld + qv];
                    const double y00 = cv * x00 - sv * x01, y01 = sv * x00 + cv * x01;
                    const double y10 = cv * x10 - sv * x11, y11 = sv * x10 + cv * x11;
                    const double z00 = cu * y00 - su * y10, z10 = su * y00 + cu * y10;
                    const double z01 = cu * y01 - su * y11, z11 = su * y01 + cu * y11;
                    C[pu * ld + pv] = z00; C[pv * ld + pu] = z00;
                    C[pu * ld + qv] = z01; C[qv * ld + pu] = z01;
                    C[qu * ld + pv] = z10; C[pv * ld + qu] = z10;
                    C[qu * ld + qv] = z11; C[qv * ld + qu] = z11;
                }
            }
            for (int e = t, row = t / np, u = t % np; e < n * np; e += 64) {
                const int pu = (int)rot[5 * u + 4] & 255, qu = (int)rot[5 * u + 4] >> 8;
                const double cu = rot[5 * u], su = rot[5 * u + 1];
                const double vp = V[row * ld + pu], vq = V[row * ld + qu];
                V[row * ld + pu] = cu * vp - su * vq;
                V[row * ld + qu] = su * vp + cu * vq;
                row += dq64; u += dr64;
                if (u >= np) { u -= np; row++; }
            }
            __syncthreads();
        }
    }

    MPCQ_STAMP(7);
    // ---- W^-1 = V' L' (needs V before it is overwritten), then W = L^-T V in place on V
    double *o_lam = out + Lo.lam, *o_W = out + Lo.W, *o_sWtW = out + Lo.sWtW, *o_WtA = out + Lo.WtA;
    double *o_PW = out + Lo.PW, *o_Winv = out + Lo.Winv, *o_Ah = out + Lo.Ah, *o_D = out + Lo.D, *o_E = out + Lo.E;
    double *o_Dinv = out + Lo.Dinv, *o_Einv = out + Lo.Einv, *o_cs = out + Lo.cs, *o_rs = out + Lo.rscale;
    for (int e = t; e < nc * nc; e += 64) {
        const int i = e / nc, k = e % nc;
        double wi = 0.0;
        if (i < n && k < n)
            for (int r = 0; r <= k; r++) wi += V[r * ld + i] * L[k * ld + r];
        o_Winv[e] = wi;
    }
    for (int k = t; k < nc; k += 64) {
        o_lam[k] = k < n ? fmax(C[k * ld + k], 0.0) : 0.0;
        o_D[k] = k < n ? Dv[k] : 1.0;
        o_Dinv[k] = k < n ? 1.0 / Dv[k] : 1.0;
    }
    for (int i = t; i < mc; i += 64) {
        o_E[i] = i < m ? Ev[i] : 1.0;
        o_Einv[i] = i < m ? 1.0 / Ev[i] : 1.0;
        o_rs[i] = i < m ? Et[i] : 1.0;
    }
    if (t == 0) { o_cs[0] = cost; o_cs[1] = 1.0 / cost; }
    __syncthreads();
    for (int i = n - 1; i >= 0; i--) {  // (L')[r][i] = L[i][r]
        const double li = L[i * ld + i];
        if (t < n) V[i * ld + t] /= li;
        __syncthreads();
        for (int e = t; e < i * n; e += 64) {
            const int r = e / n, c = e % n;
            V[r * ld + c] -= L[i * ld + r] * V[i * ld + c];
        }
        __syncthreads();
    }
    const double *W = V;
    for (int e = t; e < nc * nc; e += 64) {
        const int i = e / nc, k = e % nc;
        double w = 0.0, wtw = 0.0, pw = 0.0;
        if (i < n && k < n) {
            w = W[i * ld + k];
            for (int r = 0; r < n; r++) {
                wtw += W[r * ld + i] * W[r * ld + k];
                pw += Ph[i * ld + r] * W[r * ld + k];
            }
            wtw *= a.sigma;
        }
        o_W[e] = w;
        o_sWtW[e] = wtw;
        o_PW[e] = pw;
    }
    for (int e = t; e < mc * nc; e += 64) {
        const int j = e / nc, k = e % nc;
        double b = 0.0, ah = 0.0;
        if (j < m && k < n) {
            ah = Ah[j * ld + k];
            for (int r = 0; r < n; r++) b += Ah[j * ld + r] * W[r * ld + k];
        }
        o_WtA[e] = b;
        o_Ah[e] = ah;
        out[Lo.Bt + e] = b;  // eigen-basis: Bt = A^ W, G = W
    }
    for (int e = t; e < nc * nc; e += 64) out[Lo.G + e] = o_W[e];
    if (t == 0) out[Lo.rho0] = -1.0;
    MPCQ_STAMP(8);
    if (t == 0) {
        a.status[pl] = fail ? kNonCvx : 0;
        if (fail) atomicOr(a.flags, 1);
        if (!converged) atomicOr(a.flags, 4);  // sweep cap hit: (lambda, W) would be inaccurate
    }
}

// In-place Gauss-Jordan inverse of an SPD matrix in LDS (n <= 32, row stride ld), 64 threads; no
// pivoting (SPD: every pivot is positive).  Returns false when a pivot is not positive (P^ + sigma I
// + rho A^'A^ not positive definite: OSQP's setup would fail to factor it).
__device__ bool gj_invert_spd(double *M, int n, int ld, int t)
{
    bool ok = true;
    for (int k = 0; k < n; k++) {
        const double piv = M[k * ld + k];
        if (!(piv > 0.0)) ok = false;
        const double ip = 1.0 / piv;
        double nv[16];  // this thread's elements t + 64 c (n*n <= 1024): static indices, registers
#pragma unroll
        for (int c = 0; c < 16; c++) {
            const int e = t + 64 * c;
            if (e < n * n) {
                const int i = e / n, j = e % n;
                double v;
                if (i == k && j == k) v = ip;
                else if (i == k) v = M[k * ld + j] * ip;
                else if (j == k) v = -M[i * ld + k] * ip;
                else v = M[i * ld + j] - M[i * ld + k] * (M[k * ld + j] * ip);
                nv[c] = v;
            }
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 16; c++) {
            const int e = t + 64 * c;
            if (e < n * n) M[(e / n) * ld + e % n] = nv[c];
        }
        __syncthreads();
    }
    return ok;
}

// Per-plant setup with the direct inverse (batches of distinct plants, BASELINE config 3): OSQP's
// scale_data and set_rho_vec as setup_wave_kernel, then M(rho0) = P^ + sigma I + sum_j rho_j a_j a_j'
// (rho_j = rho0 * rscale_j, RHO_MIN on free rows) and its inverse by Gauss-Jordan: O(n^3) in place
// of the eigen-basis's Cholesky + Jacobi sweeps.  Writes the operator block in the direct-inverse
// reading of OpsLayout (mpcq_internal.h): W = W^-1 = I, lambda = 0, sigma W'W = sigma M^-1,
// G = M^-1, Bt = A^ M^-1, PW = P^, WtA = Ah = A^, rho0.
__global__ __launch_bounds__(64) void setup_inv_kernel(SetupArgs a)
{
    extern __shared__ double sm[];
    const int pl = blockIdx.x;
    if (pl >= a.n_plants) return;
    const int t = threadIdx.x;
    const int n = a.n, m = a.m, nc = a.nc, mc = a.mc;
    const SetupWaveShape S = SetupWaveShape::make(n, m);
    const int ld = S.ld;
    double *Ph = sm + S.Ph, *Ah = sm + S.Ah, *Mi = sm + S.L;
    double *Dv = sm + S.Dv, *Ev = sm + S.Ev, *Dt = sm + S.Dt, *Et = sm + S.Et, *qh = sm + S.qh;
    double *sh = sm + S.total - 8;
    const double *P = a.P + (size_t)pl * n * n;
    const double *q0 = a.q0 + (size_t)pl * n;
    const double *A = a.A + (size_t)pl * m * n;
    const OpsLayout Lo = OpsLayout::make(nc, mc);
    double *out = a.ops + (size_t)pl * Lo.total;
    int *ctype = a.ctype + (size_t)pl * mc;

    MPCQ_STAMP(0);
    for (int e = t; e < n * n; e += 64) {  // (osqp-eigen keeps the upper triangle of the Hessian)
        const int i = e / n, j = e % n;
        Ph[i * ld + j] = (i <= j) ? P[i * n + j] : P[j * n + i];
    }
    for (int e = t; e < m * n; e += 64) Ah[(e / n) * ld + e % n] = A[e];
    for (int j = t; j < n; j += 64) { qh[j] = q0[j]; Dv[j] = 1.0; }
    for (int i = t; i < m; i += 64) Ev[i] = 1.0;
    if (t == 0) sh[0] = 1.0;
    __syncthreads();
    MPCQ_STAMP(1);
    const double cost = ruiz_and_types(a, pl, t, n, m, mc, ld, Ph, Ah, Dv, Ev, Dt, Et, qh, sh, ctype);
    MPCQ_STAMP(3);

    // ---- M(rho0) and its inverse
    const double rho = fmin(fmax(a.rho, kRhoMin), kRhoMax);
    for (int e = t; e < n * n; e += 64) {
        const int i = e / n, k = e % n;
        double v = Ph[i * ld + k] + (i == k ? a.sigma : 0.0);
        for (int r = 0; r < m; r++) {
            const double rr = Et[r] == 0.0 ? kRhoMin : rho * Et[r];
            v += rr * (Ah[r * ld + i] * Ah[r * ld + k]);
        }
        Mi[i * ld + k] = v;
    }
    __syncthreads();
    const bool ok = gj_invert_spd(Mi, n, ld, t);
    MPCQ_STAMP(6);

    // ---- operator block (zero padded to nc x mc)
    for (int e = t; e < nc * nc; e += 64) {
        const int i = e / nc, k = e % nc;
        const bool in = i < n && k < n;
        const double mi = in ? Mi[i * ld + k] : 0.0, id = (i == k && i < n) ? 1.0 : 0.0;
        out[Lo.W + e] = id;
        out[Lo.Winv + e] = id;
        out[Lo.sWtW + e] = a.sigma * mi;
        out[Lo.G + e] = mi;
        out[Lo.PW + e] = in ? Ph[i * ld + k] : 0.0;
    }
    for (int e = t; e < mc * nc; e += 64) {
        const int j = e / nc, k = e % nc;
        double ah = 0.0, bt = 0.0;
        if (j < m && k < n) {
            ah = Ah[j * ld + k];
            for (int r = 0; r < n; r++) bt += Ah[j * ld + r] * Mi[r * ld + k];
        }
        out[Lo.WtA + e] = ah;
        out[Lo.Ah + e] = ah;
        out[Lo.Bt + e] = bt;
    }
    for (int k = t; k < nc; k += 64) {
        out[Lo.lam + k] = 0.0;
        out[Lo.D + k] = k < n ? Dv[k] : 1.0;
        out[Lo.Dinv + k] = k < n ? 1.0 / Dv[k] : 1.0;
    }
    for (int i = t; i < mc; i += 64) {
        out[Lo.E + i] = i < m ? Ev[i] : 1.0;
        out[Lo.Einv + i] = i < m ? 1.0 / Ev[i] : 1.0;
        out[Lo.rscale + i] = i < m ? Et[i] : 1.0;
    }
    if (t == 0) {
        out[Lo.cs] = cost;
        out[Lo.cs + 1] = 1.0 / cost;
        out[Lo.rho0] = rho;
        a.status[pl] = ok ? 0 : kNonCvx;
        if (!ok) atomicOr(a.flags, 1);
    }
    MPCQ_STAMP(8);
}

}  // namespace mpcq

extern "C" int mpcq_internal_setup_inv_launch(const mpcq::SetupArgs *args, hipStream_t stream)
{
    if (args->n < 1 || args->n > 32 || args->m > 64) return -1;
    const size_t lds = 8 * mpcq::SetupWaveShape::make(args->n, args->m).total;
    hipLaunchKernelGGL(mpcq::setup_inv_kernel, dim3(args->n_plants), dim3(64), lds, stream, *args);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" size_t mpcq_internal_setup_wave_lds(int n, int m)
{
    if (n < 1 || n > 32 || m > 64) return 0;
    return 8 * mpcq::SetupWaveShape::make(n, m).total;
}

extern "C" int mpcq_internal_setup_wave_launch(const mpcq::SetupArgs *args, hipStream_t stream)
{
    const size_t lds = mpcq_internal_setup_wave_lds(args->n, args->m);
    if (!lds || lds > 65536) return -1;
    hipLaunchKernelGGL(mpcq::setup_wave_kernel, dim3(args->n_plants), dim3(64), lds, stream, *args);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
