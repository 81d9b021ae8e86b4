// solvempc_amd/csrc/mpcq_mimo.hip — BASELINE config 4: per-plant MIMO condensed MPC (quad-rotor
// hover linearisations, n_x 12, n_u 4, N 30 => n = 120 variables, m = 240 rows), fp64.
//
// The reference builds the condensed QP of one SISO plant on the CPU (ModelPredictiveControlAPI.cpp
// :180-369) and hands it to OSQP (:51-64) every control step (:81-108).  Config 4 asks for that
// pipeline for 262,144 distinct MIMO plants per GPU; its formulation is oracle/mpc_mimo.h (every SISO
// scalar a block).  Two kernels:
//
//  * mimo_setup_kernel — one 256-thread workgroup per plant, everything in LDS.  The horizon-stacked
//    contraction H = Su' Qbar Su is never formed densely: Su is block-Toeplitz (Su(i, j) = CS_{i-j},
//    CS_d = sum_{k<=d} Cd Ad^k Bd), so H(j1, j1+delta) is a prefix sum over the horizon,
//    G(delta, T) = sum_{t<=T} CS_{t+delta}' Q CS_t, and all of P costs N^2 nu^2 n_y multiply-adds
//    (0.18 MFLOP at config 4) instead of the dense 2 (N nu)^2 N n_y (10.4 MFLOP).  Then OSQP's Ruiz
//    equilibration (scale_data) on P (dense, LDS) and on A = [L (x) K0; -(L (x) K0)] (structured: its
//    row / column norms are prefix / suffix maxima over the horizon).  Writes P^ = c D P D and the
//    operator block of MimoLayout.
//
//  * mimo_solve_kernel — one 256-thread workgroup per QP, two per CU.  The reduced KKT matrix
//    M(rho) = P^ + sigma I + rho A^'A^ (A^'A^ from the suffix sums SW of the setup) lives in VGPRs as
//    4 x 16 blocks (thread (rg, cg): rows 4 rg.., columns 16 cg..) and is inverted in place by
//    Gauss-Jordan (SPD: no pivoting; one LDS row/column broadcast and one barrier per step).  An ADMM
//    iteration is then one GEMV with M^-1 (all 4 waves) plus O(n) vector work on wave 0 (lane k =
//    horizon block k), where A^ x and A^' w are lane prefix / suffix scans (DPP) and K0 products.  OSQP's adaptive rho
//    (adapt_rho at multiples of the interval) re-inverts M(rho_new) in place from P^ (global); the
//    dual residual's P^ x is carried through the KKT identity P^ x~ = rhs - sigma x~ - rho A^'A^ x~
//    (exact algebra; no P^ product per check).  Checks, certificates and statuses are OSQP v0.6's
//    (auxil.c), as in the tile kernel.
#include "mpcq_internal.h"
#include "mpcq_wave.h"

namespace mpcq {

__device__ inline double mimo_limit_scaling(double d)
{
    d = d < kMinScaling ? 1.0 : d;
    return d > kMaxScaling ? kMaxScaling : d;
}

// ----------------------------------------------------------------------------------------------
// setup: LDS carve (doubles)
struct MimoSetupShape {
    int N, nx, nu, ny, n, ldp;
    size_t P, Ad, Bd, Cd, Q, R, RD, K0, AB, AB2, CA, CA2, QCA, CS, QCS, Dv, Ev, Dt, Et, cn, sh, total;
    __host__ __device__ static MimoSetupShape make(int N, int nx, int nu, int ny)
    {
        MimoSetupShape s{};
        s.N = N; s.nx = nx; s.nu = nu; s.ny = ny; s.n = N * nu;
        s.ldp = s.n + 1;  // odd stride: column walks by consecutive lanes hit distinct banks
        size_t o = 0;
        s.P = o; o += (size_t)s.n * s.ldp;
        s.Ad = o; o += (size_t)nx * nx;
        s.Bd = o; o += (size_t)nx * nu;
        s.Cd = o; o += (size_t)ny * nx;
        s.Q = o; o += (size_t)ny * ny;
        s.R = o; o += (size_t)nu * nu;
        s.RD = o; o += (size_t)nu * nu;
        s.K0 = o; o += (size_t)nu * nu;
        s.AB = o; o += (size_t)nx * nu;
        s.AB2 = o; o += (size_t)nx * nu;
        s.CA = o; o += (size_t)ny * nx;
        s.CA2 = o; o += (size_t)ny * nx;
        s.QCA = o; o += (size_t)ny * nx;
        s.CS = o; o += (size_t)N * ny * nu;
        s.QCS = o; o += (size_t)N * ny * nu;
        s.Dv = o; o += s.n;
        s.Ev = o; o += s.n;
        s.Dt = o; o += s.n;
        s.Et = o; o += s.n;
        s.cn = o; o += s.n;
        s.sh = o; o += 8;
        s.total = o;
        return s;
    }
};

constexpr int kMimoSetupThreads = 256;
constexpr int kMimoFxPer = 8;  // Fx accumulators per thread: n nx <= 8 * 256

__global__ __launch_bounds__(kMimoSetupThreads) void mimo_setup_kernel(MimoSetupArgs a)
{
    extern __shared__ double sm[];
    const int pl = blockIdx.x;
    if (pl >= a.n_plants) return;
    const int t = threadIdx.x;
    constexpr int T = kMimoSetupThreads;
    const int N = a.N, nx = a.nx, nu = a.nu, ny = a.ny;
    const MimoSetupShape S = MimoSetupShape::make(N, nx, nu, ny);
    const int n = S.n, ldp = S.ldp;
    double *P = sm + S.P, *Ad = sm + S.Ad, *Bd = sm + S.Bd, *Cd = sm + S.Cd, *Q = sm + S.Q, *R = sm + S.R;
    double *RD = sm + S.RD, *K0 = sm + S.K0, *AB = sm + S.AB, *AB2 = sm + S.AB2, *CA = sm + S.CA, *CA2 = sm + S.CA2;
    double *QCA = sm + S.QCA, *CS = sm + S.CS, *QCS = sm + S.QCS, *Dv = sm + S.Dv, *Ev = sm + S.Ev, *Dt = sm + S.Dt;
    double *Et = sm + S.Et, *cn = sm + S.cn, *sh = sm + S.sh;
    const MimoLayout L = MimoLayout::make(N, nx, nu, ny);
    double *out = a.ops + (size_t)pl * L.total;

    // ---- plant data -> LDS
    for (int e = t; e < nx * nx; e += T) Ad[e] = a.Ad[(size_t)pl * nx * nx + e];
    for (int e = t; e < nx * nu; e += T) Bd[e] = a.Bd[(size_t)pl * nx * nu + e];
    for (int e = t; e < ny * nx; e += T) Cd[e] = a.Cd[(size_t)pl * ny * nx + e];
    for (int e = t; e < ny * ny; e += T) Q[e] = a.Q[(size_t)pl * ny * ny + e];
    for (int e = t; e < nu * nu; e += T) {
        R[e] = a.R[(size_t)pl * nu * nu + e];
        RD[e] = a.RD[(size_t)pl * nu * nu + e];
        K0[e] = a.K0[(size_t)pl * nu * nu + e];
        out[L.K0 + e] = K0[e];
    }
    for (int e = t; e < nu * nx; e += T) out[L.K + e] = a.K[(size_t)pl * nu * nx + e];
    for (int e = t; e < nu; e += T) out[L.w0 + e] = a.w0[(size_t)pl * nu + e];
    __syncthreads();

    // ---- setTransformations (:187-204): CS_d = sum_{k<=d} Cd Ad^k Bd (the distinct blocks of Su),
    // and Fx = 2 (Sx' Qbar Su)' (:307) accumulated as Fx_j += CS_{d-j}' Q Cd Ad^(d+1) for j <= d.
    for (int e = t; e < nx * nu; e += T) AB[e] = Bd[e];
    for (int e = t; e < ny * nx; e += T) {
        const int i = e / nx, c = e % nx;
        double s = 0.0;
        for (int k = 0; k < nx; k++) s += Cd[i * nx + k] * Ad[k * nx + c];
        CA[e] = s;  // Sx_0 = Cd Ad
    }
    double fx[kMimoFxPer];
#pragma unroll
    for (int s = 0; s < kMimoFxPer; s++) fx[s] = 0.0;
    __syncthreads();
    for (int d = 0; d < N; d++) {
        for (int e = t; e < ny * nu; e += T) {
            const int i = e / nu, c = e % nu;
            double cab = 0.0;
            for (int k = 0; k < nx; k++) cab += Cd[i * nx + k] * AB[k * nu + c];
            CS[(size_t)d * ny * nu + e] = (d ? CS[(size_t)(d - 1) * ny * nu + e] : 0.0) + cab;
        }
        for (int e = t; e < ny * nx; e += T) {
            const int i = e / nx, c = e % nx;
            double s = 0.0, s2 = 0.0;
            for (int k = 0; k < ny; k++) s += Q[i * ny + k] * CA[k * nx + c];
            for (int k = 0; k < nx; k++) s2 += CA[i * nx + k] * Ad[k * nx + c];
            QCA[e] = s;
            CA2[e] = s2;
        }
        for (int e = t; e < nx * nu; e += T) {
            const int i = e / nu, c = e % nu;
            double s = 0.0;
            for (int k = 0; k < nx; k++) s += Ad[i * nx + k] * AB[k * nu + c];
            AB2[e] = s;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < kMimoFxPer; s++) {
            const int it = t + T * s;  // (j, r, c) of Fx
            if (it < n * nx) {
                const int j = it / (nu * nx), r = (it / nx) % nu, c = it % nx;
                if (j <= d) {
                    const double *cs = CS + (size_t)(d - j) * ny * nu;
                    double acc = 0.0;
                    for (int k = 0; k < ny; k++) acc += cs[k * nu + r] * QCA[k * nx + c];
                    fx[s] += acc;
                }
            }
        }
        __syncthreads();
        for (int e = t; e < nx * nu; e += T) AB[e] = AB2[e];
        for (int e = t; e < ny * nx; e += T) CA[e] = CA2[e];
        __syncthreads();
    }
#pragma unroll
    for (int s = 0; s < kMimoFxPer; s++) {
        const int it = t + T * s;
        if (it < n * nx) out[L.Fx + it] = 2.0 * fx[s];
    }
    // QCS_d = Q CS_d
    for (int e = t; e < N * ny * nu; e += T) {
        const int d = e / (ny * nu), i = (e / nu) % ny, c = e % nu;
        double s = 0.0;
        for (int k = 0; k < ny; k++) s += Q[i * ny + k] * CS[(size_t)d * ny * nu + k * nu + c];
        QCS[e] = s;
    }
    __syncthreads();

    // ---- setH (:250-251): H(j1, j1+delta) = G(delta, N-1-j1-delta), G(delta, T) = sum_{t<=T}
    // CS_{t+delta}' Q CS_t; H1 = 2 ((N - max(j1, j2)) R + RD delta_{j1 j2} + H) (LL' Rbar LL has block
    // (j1, j2) = sum_{k >= max} R); P = (H1 + H1') / 2.
    for (int it = t; it < N * nu * nu; it += T) {
        const int dl = it / (nu * nu), r = (it / nu) % nu, c = it % nu;
        double acc = 0.0;
        for (int tt = 0; tt + dl < N; tt++) {
            const double *c1 = CS + (size_t)(tt + dl) * ny * nu, *c2 = QCS + (size_t)tt * ny * nu;
            double s = 0.0;
            for (int k = 0; k < ny; k++) s += c1[k * nu + r] * c2[k * nu + c];
            acc += s;
            const int j2 = N - 1 - tt, j1 = j2 - dl;
            const double rr = (double)(N - j2);  // N - max(j1, j2)
            P[(size_t)(j1 * nu + r) * ldp + j2 * nu + c] = 2.0 * (rr * R[r * nu + c] + (dl == 0 ? RD[r * nu + c] : 0.0) + acc);
            if (dl > 0)  // H(j2, j1) = H(j1, j2)'
                P[(size_t)(j2 * nu + c) * ldp + j1 * nu + r] = 2.0 * (rr * R[c * nu + r] + acc);
        }
    }
    // Fu = 2 (R' + H(j, 0)) per block (:305, the .diagonal() quirk as blocks; Q symmetric),
    // Frs = -2 sum_{d <= N-1-j} QCS_d' (Fr = -2 (Qbar Su)', :306, summed over the horizon blocks)
    for (int it = t; it < n * nu; it += T) {
        const int j = it / (nu * nu), r = (it / nu) % nu, c = it % nu;
        double acc = 0.0;
        for (int i = j; i < N; i++) {
            const double *c1 = CS + (size_t)(i - j) * ny * nu, *c2 = QCS + (size_t)i * ny * nu;
            double s = 0.0;
            for (int k = 0; k < ny; k++) s += c1[k * nu + r] * c2[k * nu + c];
            acc += s;
        }
        out[L.Fu + it] = 2.0 * (R[c * nu + r] + acc);
    }
    for (int it = t; it < n * ny; it += T) {
        const int j = it / (nu * ny), r = (it / ny) % nu, i = it % ny;
        double acc = 0.0;
        for (int d = 0; d <= N - 1 - j; d++) acc += QCS[(size_t)d * ny * nu + i * nu + r];
        out[L.Frs + it] = -2.0 * acc;
    }
    __syncthreads();
    for (int e = t; e < n * n; e += T) {
        const int i = e / n, j = e % n;
        if (i < j) {
            const double v = (P[(size_t)i * ldp + j] + P[(size_t)j * ldp + i]) / 2.0;
            P[(size_t)i * ldp + j] = v;
            P[(size_t)j * ldp + i] = v;
        }
    }
    for (int j = t; j < n; j += T) { Dv[j] = 1.0; Ev[j] = 1.0; }
    if (t == 0) sh[0] = 1.0;
    __syncthreads();

    // ---- Ruiz equilibration + cost scaling (OSQP scale_data, q0 = 0 at setup, :22-23,38-39).
    // A = [L (x) K0; -(L (x) K0)]: |A^((k, r), (j, c))| = E(k,r) |K0(r, c)| D(j, c) for j <= k, and the
    // bottom rows mirror the top ones (same norms, so the same E).
    for (int pass = 0; pass < a.scaling; pass++) {
        for (int j = t; j < n; j += T) {
            double v = 0.0;
            for (int i = 0; i < n; i++) v = fmax(v, fabs(P[(size_t)i * ldp + j]));
            const int bj = j / nu, cj = j % nu;
            double va = 0.0;
            for (int k = bj; k < N; k++)
                for (int r = 0; r < nu; r++) va = fmax(va, Ev[k * nu + r] * fabs(K0[r * nu + cj]));
            v = fmax(v, va * Dv[j]);
            Dt[j] = 1.0 / sqrt(mimo_limit_scaling(v));
        }
        for (int i = t; i < n; i += T) {
            const int bi = i / nu, ri = i % nu;
            double v = 0.0;
            for (int k = 0; k <= bi; k++)
                for (int c = 0; c < nu; c++) v = fmax(v, fabs(K0[ri * nu + c]) * Dv[k * nu + c]);
            Et[i] = 1.0 / sqrt(mimo_limit_scaling(Ev[i] * v));
        }
        __syncthreads();
        for (int e = t; e < n * n; e += T) {
            const int i = e / n, j = e % n;
            P[(size_t)i * ldp + j] = (Dt[i] * P[(size_t)i * ldp + j]) * Dt[j];
        }
        __syncthreads();
        for (int j = t; j < n; j += T) {
            Dv[j] *= Dt[j];
            Ev[j] *= Et[j];
            double v = 0.0;
            for (int i = 0; i < n; i++) v = fmax(v, fabs(P[(size_t)i * ldp + j]));
            cn[j] = v;
        }
        __syncthreads();
        if (t == 0) {
            double mean = 0.0;
            for (int j = 0; j < n; j++) mean += cn[j];
            mean /= n;
            const double qn = mimo_limit_scaling(0.0);  // |q^| = 0 at setup
            const double ct = 1.0 / mimo_limit_scaling(fmax(mean, qn));
            sh[1] = ct;
            sh[0] *= ct;
        }
        __syncthreads();
        const double ct = sh[1];
        for (int e = t; e < n * n; e += T) P[(size_t)(e / n) * ldp + e % n] *= ct;
        __syncthreads();
    }

    // ---- outputs: P^, D, E, c, SW (suffix sums of K0' diag(2 E_k^2) K0), row-type check
    for (int e = t; e < n * L.ldp; e += T) {
        const int i = e / L.ldp, j = e % L.ldp;
        out[L.Ph + e] = j < n ? P[(size_t)i * ldp + j] : 0.0;
    }
    for (int j = t; j < n; j += T) {
        out[L.D + j] = Dv[j];
        out[L.E + j] = Ev[j];
        // u0 = W0 (X = U = 0): a row with E w0 beyond OSQP_INFTY * MIN_SCALING would be free
        if (!(fabs(a.w0[(size_t)pl * nu + j % nu] * Ev[j]) < kInfty * kMinScaling)) atomicOr(a.flags, 2);
    }
    if (t == 0) {
        out[L.cs] = sh[0];
        out[L.cs + 1] = 1.0 / sh[0];
    }
    for (int it = t; it < N * nu * nu; it += T) {
        const int j = it / (nu * nu), c1 = (it / nu) % nu, c2 = it % nu;
        double acc = 0.0;
        for (int k = N - 1; k >= j; k--) {
            double s = 0.0;
            for (int r = 0; r < nu; r++) s += K0[r * nu + c1] * K0[r * nu + c2] * (2.0 * Ev[k * nu + r] * Ev[k * nu + r]);
            acc += s;
        }
        out[L.SW + it] = acc;
    }
}

// ----------------------------------------------------------------------------------------------
// solve: one 320-thread workgroup per QP (waves 0-3: the matrix; wave 4: the vector work), two QPs
// per CU (<= 168 VGPRs: three waves per SIMD).
//
// M(rho) = P^ + sigma I + rho A^'A^ lives in the matrix waves' VGPRs, padded to 128 x 128 with the
// identity: thread (rg, cg) = (t >> 3, t & 7) holds rows 4 rg .. 4 rg + 3, columns 16 cg .. 16 cg + 15
// (64 doubles).  Gauss-Jordan inverts it in place (SPD: no pivoting), one LDS row / column broadcast
// and one barrier per step; the step loop is unrolled by 16 so the owners of row / column k address
// their registers with compile-time indices.  An ADMM iteration is one GEMV with M^-1 (the 8-lane
// partial sums of a row group reduced by DPP) and O(n) work on the vector wave, where lane k holds
// horizon block k (its NU components): A^ x and A^' w are lane prefix / suffix scans (DPP row shifts
// plus one cross-row readlane) and per-lane K0 products.  The two roles run separate loops with the
// same barrier sequence, so the matrix registers are never live in the vector wave's code.
constexpr int kMimoThreads = 320;
constexpr int kMimoMat = 256;
constexpr int kMimoN = 128;       // n capacity
constexpr int kMimoBlk = 64 * 4;  // block-major vector slots: lane k, component c at 4 k + c

struct B4 {
    double v[4];
};

__device__ __forceinline__ B4 ldb(const double *arr, int lane)
{
    const double2 *p = (const double2 *)(arr + 4 * lane);
    const double2 u = p[0], w = p[1];
    return {{u.x, u.y, w.x, w.y}};
}
__device__ __forceinline__ void stb(double *arr, int lane, const B4 &x)
{
    double2 *p = (double2 *)(arr + 4 * lane);
    p[0] = make_double2(x.v[0], x.v[1]);
    p[1] = make_double2(x.v[2], x.v[3]);
}
// DPP move whose lanes without a source read 0 (row shifts)
template <int CTRL> __device__ __forceinline__ double dpp0(double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xF, 0xF, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double readlane_d(double v, int l)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// inclusive prefix over lanes 0..31 (horizon blocks; N <= 32): row_shr 1, 2, 4, 8, then row 1 adds
// lane 15's total
__device__ __forceinline__ double lane_prefix(double v, int lane)
{
    v += dpp0<0x111>(v);
    v += dpp0<0x112>(v);
    v += dpp0<0x114>(v);
    v += dpp0<0x118>(v);
    const double s = readlane_d(v, 15);
    return (lane >= 16) ? v + s : v;
}
// inclusive suffix over lanes 0..31 (lanes N..31 must hold 0): row_shl 1, 2, 4, 8, then row 0 adds
// lane 16's total
__device__ __forceinline__ double lane_suffix(double v, int lane)
{
    v += dpp0<0x101>(v);
    v += dpp0<0x102>(v);
    v += dpp0<0x104>(v);
    v += dpp0<0x108>(v);
    const double s = readlane_d(v, 16);
    return (lane < 16) ? v + s : v;
}

#define MPCQ_MSTAMP(k, v)                                                                  \
    do {                                                                                   \
        if (a.stamps && t == 0) a.stamps[(size_t)blockIdx.x * 8 + (k)] = (long long)(v);  \
    } while (0)

template <int NU>
__global__ __launch_bounds__(kMimoThreads, 3) void mimo_solve_kernel(MimoArgs a)
{
    const int b = blockIdx.x;
    if (b >= a.batch) return;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int N = a.N, nx = a.nx, ny = a.ny, n = N * NU, m = 2 * n;
    const MimoLayout L = MimoLayout::make(N, nx, NU, ny);
    const double *ops = a.ops + (size_t)b * a.ops_stride;
    const SolverSettings &st = a.st;
    MPCQ_MSTAMP(0, __builtin_amdgcn_s_memtime());

    __shared__ __attribute__((aligned(16))) double s_vec[kMimoN];  // GEMV input (natural order)
    __shared__ __attribute__((aligned(16))) double s_out[kMimoN];  // GEMV output
    __shared__ __attribute__((aligned(16))) double s_nat[kMimoN];  // warm start: x (natural), then P^ x
    __shared__ __attribute__((aligned(16))) double s_row[2][kMimoN], s_col[2][kMimoN];
    __shared__ __attribute__((aligned(16))) double s_D[kMimoBlk], s_E[kMimoBlk], s_K0[16], s_SW[32 * 16];
    __shared__ __attribute__((aligned(16))) double s_x[kMimoBlk], s_zt[kMimoBlk], s_zb[kMimoBlk], s_yt[kMimoBlk];
    __shared__ __attribute__((aligned(16))) double s_yb[kMimoBlk], s_px[kMimoBlk], s_qh[kMimoBlk], s_ut[kMimoBlk];
    __shared__ __attribute__((aligned(16))) double s_ub[kMimoBlk], s_rhs[kMimoBlk];
    __shared__ __attribute__((aligned(16))) double s_dx[kMimoBlk], s_dpx[kMimoBlk], s_dyt[kMimoBlk], s_dyb[kMimoBlk];
    __shared__ int s_ctrl[2];
    __shared__ double s_rho;
    for (int i = t; i < kMimoBlk; i += kMimoThreads) {
        const int k = i >> 2, c = i & 3;
        const bool ok = k < N && c < NU;
        s_D[i] = ok ? ops[L.D + k * NU + c] : 1.0;
        s_E[i] = ok ? ops[L.E + k * NU + c] : 1.0;
    }
    for (int i = t; i < 16; i += kMimoThreads) {
        const int r = i >> 2, c = i & 3;
        s_K0[i] = (r < NU && c < NU) ? ops[L.K0 + r * NU + c] : 0.0;
    }
    for (int i = t; i < 32 * 16; i += kMimoThreads) {
        const int k = i >> 4, ci = (i >> 2) & 3, cj = i & 3;
        s_SW[i] = (k < N && ci < NU && cj < NU) ? ops[L.SW + (k * NU + ci) * NU + cj] : 0.0;
    }
    for (int i = t; i < kMimoN; i += kMimoThreads) s_vec[i] = 0.0;
    __syncthreads();

    const double c64 = ops[L.cs], cinv = ops[L.cs + 1];
    const double sigma = st.sigma, alpha = st.alpha, oma = 1.0 - st.alpha;
    int fail = 0;

    if (wv < 4) {
        // ======== waves 0-3: M(rho) and M^-1 in VGPRs
        const int rg = t >> 3, cg = t & 7;
        double Mb[4][16];
        // rows 4 rg + i, columns 16 cg + j (P^ rows are padded to L.ldp: aligned, in-bounds loads);
        // the padding beyond n is the identity
        auto load_P = [&]() {
            const int seg = 16 * cg < L.ldp - 16 ? 16 * cg : L.ldp - 16;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int gi = 4 * rg + i;
                const double2 *row = (const double2 *)(ops + L.Ph + (size_t)(gi < n ? gi : n - 1) * L.ldp + seg);
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const double2 v = row[j];
                    const int gj = 16 * cg + 2 * j;
                    Mb[i][2 * j] = (gi < n && gj < n) ? v.x : (gi == gj ? 1.0 : 0.0);
                    Mb[i][2 * j + 1] = (gi < n && gj + 1 < n) ? v.y : (gi == gj + 1 ? 1.0 : 0.0);
                }
            }
        };
        // + sigma I + r D SW[max(bi, bj)] D on the n x n part (block of row gi: (4 rg + i) / NU)
        auto add_kkt = [&](double r) {
            double di[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int bi = (4 * rg) / NU + i / NU;
                di[i] = s_D[4 * (bi < 63 ? bi : 63) + i % NU];
            }
#pragma unroll
            for (int jc = 0; jc < 4; jc++) {
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    const int j = 4 * jc + jj, gj = 16 * cg + j;
                    const int bj = (16 * cg) / NU + j / NU, cj = j % NU;
                    const double dj = s_D[4 * (bj < 63 ? bj : 63) + cj];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int gi = 4 * rg + i, bi = (4 * rg) / NU + i / NU, ci = i % NU;
                        const int bm = bi > bj ? bi : bj;
                        const double g = (di[i] * dj) * s_SW[(bm < 31 ? bm : 31) * 16 + ci * 4 + cj];
                        const double v = Mb[i][j] + (gi == gj ? sigma : 0.0) + r * g;
                        if (gi < n && gj < n) Mb[i][j] = v;
                    }
                }
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int jj = 0; jj < 4; jj++) asm volatile("" : "+v"(Mb[i][4 * jc + jj]));  // (as in invert)
            }
        };
        // outv[4 rg + i] = row (4 rg + i) of M . in (the 8 lanes of a row group combine by DPP)
        auto gemv = [&](const double *in, double *outv) {
            double s0[4], s1[4];
#pragma unroll
            for (int i = 0; i < 4; i++) s0[i] = s1[i] = 0.0;
            const double2 *v2 = (const double2 *)(in + 16 * cg);
#pragma unroll
            for (int h = 0; h < 4; h++) {  // 4-column chunks (register budget)
                const double2 p0 = v2[2 * h], p1 = v2[2 * h + 1];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    s0[i] = __builtin_fma(Mb[i][4 * h], p0.x, s0[i]);
                    s1[i] = __builtin_fma(Mb[i][4 * h + 1], p0.y, s1[i]);
                    s0[i] = __builtin_fma(Mb[i][4 * h + 2], p1.x, s0[i]);
                    s1[i] = __builtin_fma(Mb[i][4 * h + 3], p1.y, s1[i]);
                }
#pragma unroll
                for (int i = 0; i < 4; i++) asm volatile("" : "+v"(s0[i]), "+v"(s1[i]));  // one chunk live at a time
            }
            double part[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                part[i] = s0[i] + s1[i];
                part[i] += dpp_t<0xB1>(part[i]);   // quad_perm [1,0,3,2]
                part[i] += dpp_t<0x4E>(part[i]);   // quad_perm [2,3,0,1]
                part[i] += dpp_t<0x141>(part[i]);  // row_half_mirror: the other quad of the 8
            }
            if (cg == 0) {
                double2 *o2 = (double2 *)(outv + 4 * rg);
                o2[0] = make_double2(part[0], part[1]);
                o2[1] = make_double2(part[2], part[3]);
            }
        };
        // Gauss-Jordan: a_ij -= (a_ik / a_kk) a_kj everywhere, then row k <- a_kj / a_kk, column k <-
        // -a_ik / a_kk, a_kk <- 1 / a_kk.  k = 16 kb + kk with kk unrolled: the owner of column k is
        // cg == kb (register column kk), of row k rg == k >> 2 (register row kk & 3).
        auto invert = [&]() {
            const int nkb = (n + 15) >> 4;
            for (int kb = 0; kb < nkb; kb++) {
#pragma unroll
                for (int kk = 0; kk < 16; kk++) {
                    const int k = 16 * kb + kk;
                    if (k >= n) continue;  // (not break: the loop must fully unroll, or Mb leaves the VGPRs)
                    const int p = k & 1;
                    const bool rown = rg == (k >> 2), coln = cg == kb;
                    if (rown) {
                        double2 *r2 = (double2 *)&s_row[p][16 * cg];
#pragma unroll
                        for (int j = 0; j < 8; j++) r2[j] = make_double2(Mb[kk & 3][2 * j], Mb[kk & 3][2 * j + 1]);
                    }
                    if (coln) {
                        double2 *c2 = (double2 *)&s_col[p][4 * rg];
                        c2[0] = make_double2(Mb[0][kk], Mb[1][kk]);
                        c2[1] = make_double2(Mb[2][kk], Mb[3][kk]);
                    }
                    __syncthreads();
                    const double piv = s_row[p][k];
                    if (!(piv > 0.0)) fail = 1;
                    const double inv = 1.0 / piv;
                    double nci[4];  // -a_ik / a_kk
                    {
                        const double2 *c2 = (const double2 *)&s_col[p][4 * rg];
                        const double2 u0 = c2[0], u1 = c2[1];
                        nci[0] = -u0.x * inv;
                        nci[1] = -u0.y * inv;
                        nci[2] = -u1.x * inv;
                        nci[3] = -u1.y * inv;
                    }
                    const double2 *r2 = (const double2 *)&s_row[p][16 * cg];
#pragma unroll
                    for (int h = 0; h < 4; h++) {  // 4-column chunks (register budget)
                        const double2 q0 = r2[2 * h], q1 = r2[2 * h + 1];
                        const double rj[4] = {q0.x, q0.y, q1.x, q1.y};
#pragma unroll
                        for (int i = 0; i < 4; i++)
#pragma unroll
                            for (int j = 0; j < 4; j++) Mb[i][4 * h + j] = __builtin_fma(nci[i], rj[j], Mb[i][4 * h + j]);
                        // pin the updates here: sunk below the fix-up branches they would keep every
                        // chunk of the row live (register budget)
#pragma unroll
                        for (int i = 0; i < 4; i++)
#pragma unroll
                            for (int j = 0; j < 4; j++) asm volatile("" : "+v"(Mb[i][4 * h + j]));
                    }
                    asm volatile("" ::: "memory");  // the row owners re-read the row below
                    if (rown) {  // row k <- a_kj / a_kk (re-read: the row owners are one wave's 8 lanes)
#pragma unroll
                        for (int h = 0; h < 8; h++) {
                            const double2 q = r2[h];
                            Mb[kk & 3][2 * h] = q.x * inv;
                            Mb[kk & 3][2 * h + 1] = q.y * inv;
                        }
                    }
                    if (coln) {
#pragma unroll
                        for (int i = 0; i < 4; i++) Mb[i][kk] = nci[i];
                        if (rown) Mb[kk & 3][kk] = inv;
                    }
                }
            }
        };

        load_P();  // overlaps the vector wave's front end
        __syncthreads();  // front end + first rhs done
        MPCQ_MSTAMP(1, __builtin_amdgcn_s_memtime());
        bool loaded = true;
        for (;;) {
            const int ctrl = s_ctrl[0];
            if (ctrl == 2) break;
            if (ctrl == 1) {  // (re-)invert M(s_rho); the first factorisation also forms P^ x of a warm start
                if (!loaded) load_P();
                loaded = false;
                if (s_ctrl[1]) {
                    __syncthreads();  // everyone has read s_ctrl[1]
                    gemv(s_nat, s_out);
                    __syncthreads();
                    for (int i = t; i < kMimoN; i += kMimoMat) s_nat[i] = s_out[i];
                    if (t == 0) s_ctrl[1] = 0;
                }
                add_kkt(s_rho);
                invert();  // its first barrier orders the writes above before the GEMV below
                MPCQ_MSTAMP(2, __builtin_amdgcn_s_memtime());
                if (fail) break;  // P^ + sigma I + rho A^'A^ not positive definite
            }
            gemv(s_vec, s_out);
            __syncthreads();  // x~ ready
            __syncthreads();  // the vector wave's phase done (next rhs, control word)
        }
        return;
    }

    // ======== wave 4 (lane k = horizon block k): the MPC front end and the ADMM vector work
    double rho = 0.0;
    int status = kUnsolved;
    const bool load = a.warm && !a.fresh;
    {
        double Xv[12], Uv[4], yr[12];
#pragma unroll
        for (int i = 0; i < 12; i++) {
            Xv[i] = i < nx ? a.X[(size_t)b * nx + (i < nx ? i : 0)] : 0.0;
            yr[i] = (i < ny && a.yref) ? a.yref[i < ny ? i : 0] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < NU; i++) Uv[i] = a.U[(size_t)b * NU + i];
        int tchg = 0;
        B4 qh, uth, ubh, x, zt, zb, yt, yb;
        const int k = lane;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            qh.v[c] = uth.v[c] = ubh.v[c] = x.v[c] = zt.v[c] = zb.v[c] = yt.v[c] = yb.v[c] = 0.0;
            if (c < NU && k < N) {
                const int e = k * NU + c;
                const double De = s_D[4 * k + c], Ee = s_E[4 * k + c];
                // setF (:372-375): q = Fx X + Fu U + Fr ref, ref = 1_N (x) yref (updateRef :378-380)
                double s0 = 0.0, s1 = 0.0, s2 = 0.0;
                for (int i = 0; i < nx; i++) s0 += ops[L.Fx + (size_t)e * nx + i] * Xv[i];
#pragma unroll
                for (int i = 0; i < NU; i++) s1 += ops[L.Fu + (size_t)e * NU + i] * Uv[i];
                for (int i = 0; i < ny; i++) s2 += ops[L.Frs + (size_t)e * ny + i] * yr[i];
                const double q = s0 + s1 + s2;
                if (a.q_out) a.q_out[(size_t)b * n + e] = q;
                qh.v[c] = (q * De) * c64;
                // (:93-99): u = W0 + Sbar X + Ku U; Sbar block rows k < s_rows = [K; -K]; Ku = [-K0; K0]
                double kx = 0.0, k0u = 0.0;
                if (k < a.s_rows)
                    for (int i = 0; i < nx; i++) kx += ops[L.K + c * nx + i] * Xv[i];
#pragma unroll
                for (int i = 0; i < NU; i++) k0u += ops[L.K0 + c * NU + i] * Uv[i];
                const double w0 = ops[L.w0 + c];
                const double utop = w0 + kx + -k0u, ubot = w0 + -kx + k0u;
                if (a.u_out) {
                    a.u_out[(size_t)b * m + e] = utop;
                    a.u_out[(size_t)b * m + n + e] = ubot;
                }
                uth.v[c] = utop * Ee;
                ubh.v[c] = ubot * Ee;
                // l = -DBL_MAX (:42): every row stays an inequality while u^ is finite
                if (!(uth.v[c] < kInfty * kMinScaling) || !(ubh.v[c] < kInfty * kMinScaling)) tchg = 1;
                if (load) {
                    x.v[c] = a.xs[(size_t)b * n + e];
                    zt.v[c] = a.zs[(size_t)b * m + e];
                    zb.v[c] = a.zs[(size_t)b * m + n + e];
                    yt.v[c] = a.ys[(size_t)b * m + e];
                    yb.v[c] = a.ys[(size_t)b * m + n + e];
                }
                s_nat[e] = x.v[c];
            }
        }
        stb(s_qh, lane, qh); stb(s_ut, lane, uth); stb(s_ub, lane, ubh);
        stb(s_x, lane, x); stb(s_zt, lane, zt); stb(s_zb, lane, zb); stb(s_yt, lane, yt); stb(s_yb, lane, yb);
        stb(s_px, lane, B4{{0.0, 0.0, 0.0, 0.0}});
        if (wave_any(tchg != 0)) status = kTypeChanged;
        rho = a.fresh ? fmin(fmax(st.rho, kRhoMin), kRhoMax) : a.rhos[b];
    }

    auto lmask = [&](B4 v) {
        if (lane >= N)
#pragma unroll
            for (int c = 0; c < 4; c++) v.v[c] = 0.0;
        return v;
    };
    auto k0_plain = [&](const B4 &x) {  // out[r] = sum_c K0[r][c] x[c]
        B4 o;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            double acc = 0.0;
#pragma unroll
            for (int c = 0; c < NU; c++) acc = __builtin_fma(s_K0[r * 4 + c], x.v[c], acc);
            o.v[r] = r < NU ? acc : 0.0;
        }
        return o;
    };
    auto k0_trans = [&](const B4 &x) {  // out[c] = sum_r K0[r][c] x[r]
        B4 o;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            double acc = 0.0;
#pragma unroll
            for (int r = 0; r < NU; r++) acc = __builtin_fma(s_K0[r * 4 + c], x.v[r], acc);
            o.v[c] = c < NU ? acc : 0.0;
        }
        return o;
    };
    auto A_of = [&](const B4 &xv) {  // (A^ x)_top = E (L (x) K0) D x; the bottom half is its negation
        const B4 D = ldb(s_D, lane), E = ldb(s_E, lane);
        B4 v;
#pragma unroll
        for (int c = 0; c < 4; c++) v.v[c] = c < NU ? lane_prefix(D.v[c] * xv.v[c], lane) : 0.0;
        v = k0_plain(v);
#pragma unroll
        for (int c = 0; c < 4; c++) v.v[c] *= E.v[c];
        return lmask(v);
    };
    // A^' [w_top; w_bot] = D (L (x) K0)' E d, d = w_top - w_bot; two right-hand sides in one pass
    auto At_of2 = [&](const B4 &d1, const B4 &d2, B4 &o1, B4 &o2) {
        const B4 D = ldb(s_D, lane), E = ldb(s_E, lane);
        const B4 v1 = lmask(d1), v2 = lmask(d2);
        B4 s1, s2;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            s1.v[c] = c < NU ? lane_suffix(E.v[c] * v1.v[c], lane) : 0.0;
            s2.v[c] = c < NU ? lane_suffix(E.v[c] * v2.v[c], lane) : 0.0;
        }
        s1 = k0_trans(s1);
        s2 = k0_trans(s2);
#pragma unroll
        for (int c = 0; c < 4; c++) {
            s1.v[c] *= D.v[c];
            s2.v[c] *= D.v[c];
        }
        o1 = lmask(s1);
        o2 = lmask(s2);
    };
    auto At_of = [&](const B4 &d) {
        const B4 D = ldb(s_D, lane), E = ldb(s_E, lane);
        B4 v = lmask(d);
#pragma unroll
        for (int c = 0; c < 4; c++) v.v[c] = c < NU ? lane_suffix(E.v[c] * v.v[c], lane) : 0.0;
        v = k0_trans(v);
#pragma unroll
        for (int c = 0; c < 4; c++) v.v[c] *= D.v[c];
        return lmask(v);
    };
    auto ld_nat = [&](const double *arr) {  // natural-order vector -> this lane's block
        B4 v;
        const int kk = lane < N ? lane : 0;
#pragma unroll
        for (int c = 0; c < 4; c++) v.v[c] = (c < NU && lane < N) ? arr[kk * NU + (c < NU ? c : 0)] : 0.0;
        return v;
    };
    auto st_rhs = [&](const B4 &r) {  // rhs to s_vec (natural, GEMV input) and s_rhs (block-major)
        stb(s_rhs, lane, r);
        if (lane < N)
#pragma unroll
            for (int c = 0; c < NU; c++) s_vec[lane * NU + c] = r.v[c];
    };
    auto make_rhs = [&]() {  // rhs = sigma x - q^ + A^'(rho z - y)
        const B4 zt = ldb(s_zt, lane), zb = ldb(s_zb, lane), yt = ldb(s_yt, lane), yb = ldb(s_yb, lane);
        B4 d;
#pragma unroll
        for (int c = 0; c < 4; c++) d.v[c] = (rho * zt.v[c] - yt.v[c]) - (rho * zb.v[c] - yb.v[c]);
        const B4 atw = At_of(d);
        const B4 x = ldb(s_x, lane), qh = ldb(s_qh, lane);
        B4 r;
#pragma unroll
        for (int c = 0; c < 4; c++) r.v[c] = (sigma * x.v[c] - qh.v[c]) + atw.v[c];
        st_rhs(lmask(r));
    };

    const int ct = st.check_termination;
    const int ai = (st.adaptive_rho && a.adaptive_interval) ? a.adaptive_interval : 0;
    int it = 0, nfact = 0;
    int next_check = ct ? ct : -1, next_adapt = ai ? ai : -1;
    bool px_pending = load;  // warm start: the first phase takes P^ x from s_nat

    auto finalize = [&]() {  // OSQP store_solution + the MPC front end's U += x[0:nu] (:105)
        const bool has_sol = status == kSolved || status == kSolvedInaccurate || status == kMaxIterReached;
        const bool keep = has_sol || status == kInvalidBounds || status == kTypeChanged;
        const B4 x = ldb(s_x, lane), zt = ldb(s_zt, lane), zb = ldb(s_zb, lane), yt = ldb(s_yt, lane);
        const B4 yb = ldb(s_yb, lane), D = ldb(s_D, lane), E = ldb(s_E, lane);
        if (lane < N) {
#pragma unroll
            for (int c = 0; c < NU; c++) {
                const int e = lane * NU + c;
                const double xv = has_sol ? x.v[c] * D.v[c] : __builtin_nan("");
                if (a.x) a.x[(size_t)b * n + e] = xv;
                if (a.y) {
                    a.y[(size_t)b * m + e] = has_sol ? (yt.v[c] * E.v[c]) * cinv : __builtin_nan("");
                    a.y[(size_t)b * m + n + e] = has_sol ? (yb.v[c] * E.v[c]) * cinv : __builtin_nan("");
                }
                if (lane == 0 && status == kSolved) a.U[(size_t)b * NU + c] = a.U[(size_t)b * NU + c] + xv;
                a.xs[(size_t)b * n + e] = keep ? x.v[c] : 0.0;
                a.zs[(size_t)b * m + e] = keep ? zt.v[c] : 0.0;
                a.zs[(size_t)b * m + n + e] = keep ? zb.v[c] : 0.0;
                a.ys[(size_t)b * m + e] = keep ? yt.v[c] : 0.0;
                a.ys[(size_t)b * m + n + e] = keep ? yb.v[c] : 0.0;
            }
        }
        if (lane == 0) {
            a.rhos[b] = rho;
            a.status[b] = status;
            a.iter[b] = it;
            a.rho_out[b] = rho;
        }
    };

    // control word (s_ctrl[0]): 0 continue, 1 (re-)invert M(s_rho) then continue, 2 done
    if (status != kUnsolved) {
        finalize();
    } else {
        make_rhs();
    }
    if (lane == 0) {
        s_rho = rho;
        s_ctrl[0] = status != kUnsolved ? 2 : 1;
        s_ctrl[1] = load ? 1 : 0;
    }
    __syncthreads();
    for (;;) {
        const int ctrl = s_ctrl[0];
        if (ctrl == 2) break;
        if (ctrl == 1) {
            if (s_ctrl[1]) {
                __syncthreads();
                __syncthreads();
            }
            for (int k = 0; k < n; k++) {  // the matrix waves' Gauss-Jordan steps
                __syncthreads();
                if (!(s_row[k & 1][k] > 0.0)) fail = 1;
            }
            nfact++;
            if (fail) {  // P^ + sigma I + rho A^'A^ not positive definite
                status = kNonCvx;
                finalize();
                break;
            }
        }
        __syncthreads();  // x~ ready
        it++;
        const bool at_check = it == next_check, at_adapt = it == next_adapt;
        if (at_check) next_check += ct;
        if (at_adapt) next_adapt += ai;
        const bool last = it == st.max_iter;
        const bool info = at_check || at_adapt || last;
        const double rinv = 1.0 / rho;
        // ---- x~ = M^-1 rhs ; z~ = A^ x~ ; P^ x~ = rhs - sigma x~ - rho A^'z~ ; relax ; project ; dual
        const B4 xt = ld_nat(s_out);
        const B4 ztl = A_of(xt);
        B4 d2, dr;
        {  // x: relaxation
            const B4 x = ldb(s_x, lane);
            B4 xn, dx;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                xn.v[c] = __builtin_fma(alpha, xt.v[c], oma * x.v[c]);
                dx.v[c] = xn.v[c] - x.v[c];
            }
            stb(s_x, lane, lmask(xn));
            stb(s_dx, lane, lmask(dx));
        }
        {  // z, y: top row e and bottom row n + e (z~_bot = -z~_top)
            B4 zt = ldb(s_zt, lane), zb = ldb(s_zb, lane), yt = ldb(s_yt, lane), yb = ldb(s_yb, lane);
            const B4 ut = ldb(s_ut, lane), ub = ldb(s_ub, lane);
            B4 dyt, dyb;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const double vt = __builtin_fma(alpha, ztl.v[c], oma * zt.v[c]);
                const double zn_t = fmin(__builtin_fma(rinv, yt.v[c], vt), ut.v[c]);
                dyt.v[c] = rho * (vt - zn_t);
                yt.v[c] = __builtin_fma(rho, vt - zn_t, yt.v[c]);
                zt.v[c] = zn_t;
                const double vb = __builtin_fma(alpha, -ztl.v[c], oma * zb.v[c]);
                const double zn_b = fmin(__builtin_fma(rinv, yb.v[c], vb), ub.v[c]);
                dyb.v[c] = rho * (vb - zn_b);
                yb.v[c] = __builtin_fma(rho, vb - zn_b, yb.v[c]);
                zb.v[c] = zn_b;
                d2.v[c] = 2.0 * ztl.v[c];
                dr.v[c] = (rho * zt.v[c] - yt.v[c]) - (rho * zb.v[c] - yb.v[c]);  // next rhs (rho unchanged)
            }
            stb(s_zt, lane, lmask(zt)); stb(s_zb, lane, lmask(zb)); stb(s_yt, lane, lmask(yt)); stb(s_yb, lane, lmask(yb));
            stb(s_dyt, lane, lmask(dyt)); stb(s_dyb, lane, lmask(dyb));
        }
        B4 gz, atw;
        if (info)
            gz = At_of(d2);
        else
            At_of2(d2, dr, gz, atw);
        {  // carried P^ x (KKT identity)
            const B4 rhs = ldb(s_rhs, lane);
            B4 px = px_pending ? ld_nat(s_nat) : ldb(s_px, lane);
            px_pending = false;
            B4 dpx;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const double ptx = (rhs.v[c] - sigma * xt.v[c]) - rho * gz.v[c];
                const double pxn = __builtin_fma(alpha, ptx, oma * px.v[c]);
                dpx.v[c] = pxn - px.v[c];
                px.v[c] = pxn;
            }
            stb(s_px, lane, lmask(px));
            stb(s_dpx, lane, lmask(dpx));
        }
        asm volatile("" ::: "memory");  // the stages below re-read the state (short register live ranges)
        int ctl = 0;
        if (info) {
            // ---- update_info: residuals (scaled norms _r, unscaled _s as OSQP reports them)
            double ax_z = 0, ax_zs = 0, zn_r = 0, zn_s = 0, axn_r = 0, axn_s = 0;
            double dr_r = 0, dr_s = 0, qn_r = 0, qn_s = 0, atyn_r = 0, atyn_s = 0, pxn_r = 0, pxn_s = 0;
            {
                const B4 ax = A_of(ldb(s_x, lane));
                const B4 zt = ldb(s_zt, lane), zb = ldb(s_zb, lane), E = ldb(s_E, lane);
                if (lane < N) {
#pragma unroll
                    for (int c = 0; c < NU; c++) {
                        const double ei = 1.0 / E.v[c];
                        const double rt = ax.v[c] - zt.v[c], rbm = -ax.v[c] - zb.v[c];
                        ax_z = fmax(ax_z, fmax(fabs(rt), fabs(rbm)));
                        ax_zs = fmax(ax_zs, fmax(fabs(ei * rt), fabs(ei * rbm)));
                        zn_r = fmax(zn_r, fmax(fabs(zt.v[c]), fabs(zb.v[c])));
                        zn_s = fmax(zn_s, fmax(fabs(ei * zt.v[c]), fabs(ei * zb.v[c])));
                        axn_r = fmax(axn_r, fabs(ax.v[c]));
                        axn_s = fmax(axn_s, fabs(ei * ax.v[c]));
                    }
                }
            }
            {
                const B4 yt = ldb(s_yt, lane), yb = ldb(s_yb, lane);
                B4 dy;
#pragma unroll
                for (int c = 0; c < 4; c++) dy.v[c] = yt.v[c] - yb.v[c];
                const B4 aty = At_of(dy);
                const B4 qh = ldb(s_qh, lane), px = ldb(s_px, lane), D = ldb(s_D, lane);
                if (lane < N) {
#pragma unroll
                    for (int c = 0; c < NU; c++) {
                        const double di = 1.0 / D.v[c];
                        const double r = (qh.v[c] + px.v[c]) + aty.v[c];
                        dr_r = fmax(dr_r, fabs(r));
                        dr_s = fmax(dr_s, fabs(di * r));
                        qn_r = fmax(qn_r, fabs(qh.v[c]));
                        qn_s = fmax(qn_s, fabs(di * qh.v[c]));
                        atyn_r = fmax(atyn_r, fabs(aty.v[c]));
                        atyn_s = fmax(atyn_s, fabs(di * aty.v[c]));
                        pxn_r = fmax(pxn_r, fabs(px.v[c]));
                        pxn_s = fmax(pxn_s, fabs(di * px.v[c]));
                    }
                }
            }
            ax_z = wmax(ax_z); ax_zs = wmax(ax_zs); zn_r = wmax(zn_r); zn_s = wmax(zn_s);
            axn_r = wmax(axn_r); axn_s = wmax(axn_s); dr_r = wmax(dr_r); dr_s = wmax(dr_s);
            qn_r = wmax(qn_r); qn_s = wmax(qn_s); atyn_r = wmax(atyn_r); atyn_s = wmax(atyn_s);
            pxn_r = wmax(pxn_r); pxn_s = wmax(pxn_s);
            const bool scaled_term = st.scaled_termination != 0;
            const double pri_res = scaled_term ? ax_z : ax_zs;
            const double dua_res = scaled_term ? dr_r : cinv * dr_s;

            // OSQP is_primal_infeasible on delta_y (u finite, l = -inf on every row: d = max(d, 0))
            auto primal_inf = [&](double eps) -> bool {
                const B4 dyt = ldb(s_dyt, lane), dyb = ldb(s_dyb, lane), ut = ldb(s_ut, lane), ub = ldb(s_ub, lane);
                const B4 E = ldb(s_E, lane), D = ldb(s_D, lane);
                double ndy = 0.0, lhs = 0.0;
                B4 dd;
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const double dt_ = fmax(dyt.v[c], 0.0), db_ = fmax(dyb.v[c], 0.0);
                    dd.v[c] = dt_ - db_;
                    if (lane < N && c < NU) {
                        ndy = fmax(ndy, fmax(fabs(scaled_term ? dt_ : E.v[c] * dt_), fabs(scaled_term ? db_ : E.v[c] * db_)));
                        lhs += ut.v[c] * dt_;
                        lhs += ub.v[c] * db_;
                    }
                }
                ndy = wmax(ndy);
                lhs = wsum(lhs);
                if (!(ndy > kDivisionTol && lhs < eps * ndy)) return false;
                const B4 atd = At_of(dd);
                double nat = 0.0;
#pragma unroll
                for (int c = 0; c < NU; c++)
                    if (lane < N) nat = fmax(nat, fabs(scaled_term ? atd.v[c] : atd.v[c] / D.v[c]));
                nat = wmax(nat);
                return nat < eps * ndy;
            };
            // OSQP is_dual_infeasible on delta_x (P^ delta_x = delta of the carried P^ x)
            auto dual_inf = [&](double eps) -> bool {
                const B4 dx = ldb(s_dx, lane), qh = ldb(s_qh, lane), D = ldb(s_D, lane);
                double qdx = 0.0, ndx = 0.0;
#pragma unroll
                for (int c = 0; c < NU; c++)
                    if (lane < N) {
                        qdx = __builtin_fma(qh.v[c], dx.v[c], qdx);
                        ndx = fmax(ndx, fabs(scaled_term ? dx.v[c] : D.v[c] * dx.v[c]));
                    }
                qdx = wsum(qdx);
                ndx = wmax(ndx);
                const double cs = scaled_term ? 1.0 : c64;
                if (!(qdx < 0.0 && ndx > kDivisionTol && qdx < -cs * eps * ndx)) return false;
                double npdx = 0.0;
                const B4 dpx = ldb(s_dpx, lane);
#pragma unroll
                for (int c = 0; c < NU; c++)
                    if (lane < N) npdx = fmax(npdx, fabs(scaled_term ? dpx.v[c] : dpx.v[c] / D.v[c]));
                npdx = wmax(npdx);
                if (!(npdx < cs * eps * ndx)) return false;
                const B4 adx = A_of(dx);
                const B4 ut = ldb(s_ut, lane), ub = ldb(s_ub, lane), E = ldb(s_E, lane);
                int viol = 0;
#pragma unroll
                for (int c = 0; c < NU; c++)
                    if (lane < N) {
                        const double sv = scaled_term ? adx.v[c] : adx.v[c] / E.v[c];
                        if (ut.v[c] < kInfty * kMinScaling && sv > eps * ndx) viol = 1;   // top row
                        if (ub.v[c] < kInfty * kMinScaling && -sv > eps * ndx) viol = 1;  // bottom row
                    }
                return !wave_any(viol != 0);
            };
            auto check = [&](bool approx) -> int {
                const double mul = approx ? 10.0 : 1.0;
                const double ea = st.eps_abs * mul, er = st.eps_rel * mul;
                if (pri_res > kInfty || dua_res > kInfty) return kNonCvx;
                const double ep = ea + er * (scaled_term ? fmax(zn_r, axn_r) : fmax(zn_s, axn_s));
                const double ed = ea + er * (scaled_term ? fmax(fmax(qn_r, atyn_r), pxn_r)
                                                         : cinv * fmax(fmax(qn_s, atyn_s), pxn_s));
                const bool pok = pri_res < ep, dok = dua_res < ed;
                if (pok && dok) return approx ? kSolvedInaccurate : kSolved;
                if (!pok && primal_inf(st.eps_prim_inf * mul))
                    return approx ? kPrimalInfeasibleInaccurate : kPrimalInfeasible;
                if (!dok && dual_inf(st.eps_dual_inf * mul))
                    return approx ? kDualInfeasibleInaccurate : kDualInfeasible;
                return kUnsolved;
            };
            // OSQP order: check at check iterations, adapt_rho at adapt iterations, and after the last
            // iteration an exact then an approximate check (osqp_solve); one call site for check()
            for (int pass = 0; pass < 2; pass++) {
                if (status != kUnsolved) break;
                if (pass == 0) {
                    if (at_check || last) status = check(false);
                    if (status == kUnsolved && at_adapt && !last) {  // adapt_rho (scaled norms)
                        const double pr = ax_z / (fmax(zn_r, axn_r) + kDivisionTol);
                        const double dn = fmax(fmax(qn_r, atyn_r), pxn_r);
                        const double du = dr_r / (dn + kDivisionTol);
                        double rn = rho * sqrt(pr / (du + kDivisionTol));
                        rn = fmin(fmax(rn, kRhoMin), kRhoMax);
                        if (rn > rho * st.adaptive_rho_tolerance || rn < rho / st.adaptive_rho_tolerance) {
                            rho = fmin(fmax(rn, kRhoMin), kRhoMax);
                            ctl = 1;
                        }
                    }
                } else if (last) {
                    const int s2 = check(true);
                    status = s2 != kUnsolved ? s2 : kMaxIterReached;
                }
            }
        }
        if (status != kUnsolved) {
            finalize();
            ctl = 2;
        } else if (info) {
            make_rhs();  // rho may have changed
        } else {
            const B4 qh = ldb(s_qh, lane), x = ldb(s_x, lane);
            B4 r;
#pragma unroll
            for (int c = 0; c < 4; c++) r.v[c] = (sigma * x.v[c] - qh.v[c]) + atw.v[c];
            st_rhs(lmask(r));
        }
        if (lane == 0) {
            s_ctrl[0] = ctl;
            s_rho = rho;
        }
        __syncthreads();
    }
    if (a.stamps && lane == 0) {
        a.stamps[(size_t)blockIdx.x * 8 + 3] = (long long)__builtin_amdgcn_s_memtime();
        a.stamps[(size_t)blockIdx.x * 8 + 4] = it;
        a.stamps[(size_t)blockIdx.x * 8 + 5] = nfact;
    }
}

}  // namespace mpcq

extern "C" int mpcq_internal_mimo_setup_launch(const mpcq::MimoSetupArgs *a, hipStream_t s)
{
    const mpcq::MimoSetupShape S = mpcq::MimoSetupShape::make(a->N, a->nx, a->nu, a->ny);
    const size_t lds = 8 * S.total;
    if (a->nx > 12 || a->nu > 4 || a->ny > 12 || a->N * a->nu > mpcq::kMimoN || a->N > 32 || lds > 160 * 1024 ||
        (size_t)a->N * a->nu * a->nx > (size_t)mpcq::kMimoFxPer * mpcq::kMimoSetupThreads)
        return -1;
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute((const void *)mpcq::mimo_setup_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
            hipSuccess)
        return -2;
    hipLaunchKernelGGL(mpcq::mimo_setup_kernel, dim3(a->n_plants), dim3(mpcq::kMimoSetupThreads), lds, s, *a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int mpcq_internal_mimo_solve_launch(const mpcq::MimoArgs *a, hipStream_t s)
{
    if (a->nx > 12 || a->ny > 12 || a->N * a->nu > mpcq::kMimoN || a->N > 32) return -1;
    const dim3 grid(a->batch), block(mpcq::kMimoThreads);
    switch (a->nu) {
    case 1: hipLaunchKernelGGL(mpcq::mimo_solve_kernel<1>, grid, block, 0, s, *a); break;
    case 2: hipLaunchKernelGGL(mpcq::mimo_solve_kernel<2>, grid, block, 0, s, *a); break;
    case 4: hipLaunchKernelGGL(mpcq::mimo_solve_kernel<4>, grid, block, 0, s, *a); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
