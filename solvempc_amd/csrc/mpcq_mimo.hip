// solvempc_amd/csrc/mpcq_mimo.hip — BASELINE config 4: per-plant MIMO condensed MPC (quad-rotor
// hover linearisations, n_x 12, n_u 4, N 30 => n = 120 variables, m = 240 rows), fp64.
//
// The reference builds the condensed QP of one SISO plant on the CPU (ModelPredictiveControlAPI.cpp
// :180-369) and hands it to OSQP (:51-64) every control step (:81-108).  Config 4 asks for that
// pipeline for 262,144 distinct MIMO plants per GPU; its formulation is oracle/mpc_mimo.h (every SISO
// scalar a block).  Two kernels:
//
//  * mimo_setup_kernel — one 1024-thread workgroup (16 waves) per plant, two per CU, everything in LDS
//    (under 80 KiB per plant at config 4: P as its packed upper triangle, regions shared by lifetime,
//    MimoSetupShape).  The horizon-stacked
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
#include <cstdlib>

#include "mpcq_internal.h"
#include "mpcq_wave.h"

namespace mpcq {

__device__ inline double mimo_limit_scaling(double d)
{
    d = d < kMinScaling ? 1.0 : d;
    return d > kMaxScaling ? kMaxScaling : d;
}

// inclusive max scans over lanes 0..31 of non-negative values (DPP row shifts read 0 outside the row,
// then one cross-row readlane); lanes >= 32 are ignored by the callers
template <int CTRL> __device__ __forceinline__ double dpp_zero(double v)
{  // (bound_ctrl: a lane without a source reads 0, with no zeroed destination to copy first)
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xF, 0xF, true);
    const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double readlane_f64(double v, int l)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double lane_prefix_max(double v, int lane)
{
    v = fmax(v, dpp_zero<0x111>(v));
    v = fmax(v, dpp_zero<0x112>(v));
    v = fmax(v, dpp_zero<0x114>(v));
    v = fmax(v, dpp_zero<0x118>(v));
    const double s = readlane_f64(v, 15);
    return (lane >= 16) ? fmax(v, s) : v;
}
__device__ __forceinline__ double lane_suffix_max(double v, int lane)
{
    v = fmax(v, dpp_zero<0x101>(v));
    v = fmax(v, dpp_zero<0x102>(v));
    v = fmax(v, dpp_zero<0x104>(v));
    v = fmax(v, dpp_zero<0x108>(v));
    const double s = readlane_f64(v, 16);
    return (lane < 16) ? fmax(v, s) : v;
}

// ----------------------------------------------------------------------------------------------
// setup: one 1024-thread workgroup (16 waves) per plant, two plants per CU; LDS carve (doubles), under
// 80 KiB per plant for config 4 (n 120).  P is symmetric and kept as its packed upper triangle (row i holds
// columns i .. n-1 at i n - i (i - 1) / 2), the diagonal nu x nu blocks of its construction in full (Dblk).
// Regions are shared by lifetime: X holds the recurrences' histories (QCA_d = Q Cd Ad^(d+1), Ad^d Bd, the
// powers Ad^1..Ad^4, then the Fx partial tiles) until P is built there, and after the last scan the Ruiz
// scalings D~, E~ take Dblk's place; Y holds CS until P is complete, then the Ruiz column partials.
struct MimoSetupShape {
    int N, nx, nu, ny, n, np;
    size_t P, Dblk, QCAh, ABh, Pw4, part, Dt, Et, CS, cm, wk;
    size_t Ad, Bd, Cd, Q, R, RD, K0, CA, Dv, Ev, red, sh, total;
    __host__ __device__ static size_t mx(size_t a, size_t b) { return a > b ? a : b; }
    __host__ __device__ static MimoSetupShape make(int N, int nx, int nu, int ny)
    {
        MimoSetupShape s{};
        s.N = N; s.nx = nx; s.nu = nu; s.ny = ny; s.n = N * nu;
        s.np = s.n * (s.n + 1) / 2;
        // region X
        s.QCAh = 0;
        s.ABh = s.QCAh + (size_t)N * ny * nx;
        s.Pw4 = s.ABh + (size_t)N * nx * nu;
        s.part = s.ABh;  // (Fx partial tiles: after the recurrences, over AB_d and the powers)
        const size_t xa = s.ABh + mx((size_t)N * nx * nu + (size_t)4 * nx * nx, (size_t)((s.n + 15) / 16) * 256);
        s.P = 0;
        s.Dblk = s.np;
        s.Dt = s.np;      // (after the scans: D~, E~ of the Ruiz passes where Dblk was)
        s.Et = s.np + s.n;
        const size_t xb = s.np + mx((size_t)N * nu * nu, (size_t)2 * s.n);
        size_t o = mx(xa, xb);
        // region Y
        s.CS = o;
        s.cm = o;         // (column-max partials, 8 row slices, once CS is dead)
        s.wk = o + 8 * 128;  // (A-norm block maxima, columns and rows)
        o += mx((size_t)N * ny * nu, (size_t)8 * 128 + 2 * 32 * 4);
        s.Ad = o; o += (size_t)nx * nx;
        s.Bd = o; o += (size_t)nx * nu;
        s.Cd = o; o += (size_t)ny * nx;
        s.Q = o; o += (size_t)ny * ny;
        s.R = o; o += (size_t)nu * nu;
        s.RD = o; o += (size_t)nu * nu;
        s.K0 = o; o += (size_t)nu * nu;
        s.CA = o; o += (size_t)ny * nx;
        s.Dv = o; o += s.n;
        s.Ev = o; o += s.n;
        s.red = o; o += 16;
        s.sh = o; o += 8;
        s.total = o;
        return s;
    }
};
// packed upper-triangle index of P(i, j), i <= j
__device__ __forceinline__ int pk_up(int i, int j, int n) { return i * n - (i * (i - 1)) / 2 + (j - i); }
__device__ __forceinline__ int pk(int i, int j, int n) { return i <= j ? pk_up(i, j, n) : pk_up(j, i, n); }

constexpr int kMimoSetupThreads = 1024;

// y = sum_k a[k * sa] b[k * sb] over k < len <= 12 (unrolled: the 12 loads are in flight together)
__device__ __forceinline__ double dot12(const double *a, int sa, const double *b, int sb, int len)
{
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = 0; k < 12; k += 2) {
        if (k < len) s0 = __builtin_fma(a[k * sa], b[k * sb], s0);
        if (k + 1 < len) s1 = __builtin_fma(a[(k + 1) * sa], b[(k + 1) * sb], s1);
    }
    return s0 + s1;
}

// One 16 x 16 tile (ti, tj) of C = A B with K <= 12 on v_mfma_f64_16x16x4f64, the operands read from LDS
// through index functors (entries outside M x K, K x N read as 0) and the valid outputs handed to `put`.
// The whole wave runs it.  Operand layouts as in the Fx product below: lane (g = lane >> 4, c = lane & 15)
// holds A(16 ti + c, 4 ks + g) and B(4 ks + g, 16 tj + c); accumulator v is C(16 ti + g + 4 v, 16 tj + c).
template <typename FA, typename FB, typename FC>
__device__ __forceinline__ void lds_mma_tile(int lane, int ti, int tj, int M, int N, int K, FA a_at, FB b_at, FC put)
{
    typedef double v4d __attribute__((ext_vector_type(4)));
    v4d acc = {0.0, 0.0, 0.0, 0.0};
    const int c = lane & 15, g = lane >> 4, m = 16 * ti + c, nn = 16 * tj + c;
#pragma unroll
    for (int ks = 0; ks < 3; ks++) {
        const int k = 4 * ks + g;
        const double av = (m < M && k < K) ? a_at(m, k) : 0.0;
        const double bv = (nn < N && k < K) ? b_at(k, nn) : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    }
#pragma unroll
    for (int v = 0; v < 4; v++) {
        const int mm = 16 * ti + g + 4 * v;
        if (mm < M && nn < N) put(mm, nn, acc[v]);
    }
}

__global__ __launch_bounds__(kMimoSetupThreads, 8) void mimo_setup_kernel(MimoSetupArgs a)
{
    extern __shared__ double sm[];
    const int pl = blockIdx.x;
    if (pl >= a.n_plants) return;
    const int t = threadIdx.x;
    constexpr int T = kMimoSetupThreads;
    const int N = a.N, nx = a.nx, nu = a.nu, ny = a.ny;
    const MimoSetupShape S = MimoSetupShape::make(N, nx, nu, ny);
    const int n = S.n;
    double *P = sm + S.P, *Dblk = sm + S.Dblk, *Ad = sm + S.Ad, *Bd = sm + S.Bd, *Cd = sm + S.Cd, *Q = sm + S.Q;
    double *R = sm + S.R, *RD = sm + S.RD, *K0 = sm + S.K0, *CA = sm + S.CA, *CS = sm + S.CS;
    double *Dv = sm + S.Dv, *Ev = sm + S.Ev, *Dt = sm + S.Dt, *Et = sm + S.Et, *cm = sm + S.cm, *wk = sm + S.wk;
    double *red = sm + S.red;
    const MimoLayout L = MimoLayout::make(N, nx, nu, ny);
    double *out = a.ops + (size_t)pl * L.total;
#define MPCQ_SSTAMP(k)                                                                              \
    do {                                                                                            \
        if (a.stamps && t == 0) a.stamps[(size_t)pl * 16 + (k)] = (long long)__builtin_amdgcn_s_memtime(); \
    } while (0)
    MPCQ_SSTAMP(0);
    if (a.stamps && t == 0) {  // (debug: where and when the workgroup ran, for co-residency)
        a.stamps[(size_t)pl * 16 + 12] = (long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
        a.stamps[(size_t)pl * 16 + 13] = (long long)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
        a.stamps[(size_t)pl * 16 + 14] = (long long)__builtin_amdgcn_s_memrealtime();
    }

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
    MPCQ_SSTAMP(1);

    // ---- setTransformations (:187-204): CS_d = sum_{k<=d} Cd Ad^k Bd (the distinct blocks of Su) and
    // QCA_d = Q Cd Ad^(d+1) (for Fx = 2 (Sx' Qbar Su)', :307).  By doubling: with Ad^2, Ad^4, Ad^8, Ad^16 at
    // hand, AB_(d + 2^k) = Ad^(2^k) AB_d and QCA_(d + 2^k) = QCA_d Ad^(2^k) give 2^k new steps per round, so
    // the N <= 32 steps take 5 rounds (one barrier each) instead of a step-by-step recurrence.
    double *QCAh = sm + S.QCAh;                         // QCA_d, [d][ny][nx]
    double *ABh = sm + S.ABh;                           // Ad^d Bd, [d][nx][nu]
    double *Pw = sm + S.Pw4;                            // Ad^(2^(s+1)) at Pw + s nx^2, s = 0..3
    double *QC = CA;                                    // Q Cd (ny x nx)
    const int ann = nx * nx, anu = nx * nu, ayx = ny * nx;
    // round r (r = 0..4) forms, each item a dot12 over LDS: Ad^(2^(r+1)) = (Ad^(2^r))^2 (r < 4), the AB steps
    // [2^r, 2^(r+1)) from [0, 2^r) (Ad^(2^r) times them; r = 0: AB_1 = Ad Bd) and the QCA steps ... likewise
    // one round behind (QCA_0 = QC Ad, QCA_1 = QC Ad^2 need QC: round 1)
    for (int e = t; e < ayx; e += T) QC[e] = dot12(Q + (e / nx) * ny, 1, Cd + e % nx, nx, ny);
    for (int e = t; e < anu; e += T) ABh[e] = Bd[e];
    // each round's products as 16 x 16 MFMA tiles, one wave per tile (Ad^(2h): one tile; the AB steps: the
    // columns of [AB_0 .. AB_(nab-1)] in tiles of 16; the QCA steps: the rows of [QCA_0; ..] in tiles of 16)
    const int lane = t & 63, wv = t >> 6;
    constexpr int NW = T / 64;
    for (int r = 0; r <= 5; r++) {
        __syncthreads();
        const int h = 1 << r;                          // AB: steps [h, 2h) from [0, h)
        const double *Ph = r == 0 ? Ad : Pw + (r - 1) * ann;  // Ad^h
        const int nab = N > h ? (N - h < h ? N - h : h) : 0;
        // QCA: round 1 forms steps 0, 1 from QC; round r >= 2 steps [2^(r-1), 2^r) from [0, 2^(r-1))
        const int hq = r >= 2 ? 1 << (r - 1) : 0;
        const int nqa = r == 1 ? (N < 2 ? N : 2) : (r >= 2 && N > hq ? (N - hq < hq ? N - hq : hq) : 0);
        const int ta = (r < 4 && ((2 << r) < N || r == 0)) ? 1 : 0;  // Ad^(2h): needed while 2h < N (Ad^2: QCA_1)
        const int tb = (nab * nu + 15) / 16;
        const int tc = r == 1 ? nqa : (nqa * ny + 15) / 16;
        for (int tile = wv; tile < ta + tb + tc; tile += NW) {  // (wave-uniform)
            if (tile < ta) {
                lds_mma_tile(lane, 0, 0, nx, nx, nx, [&](int i, int k) { return Ph[i * nx + k]; },
                             [&](int k, int c) { return Ph[k * nx + c]; },
                             [&](int i, int c, double v) { Pw[r * ann + i * nx + c] = v; });
            } else if (tile < ta + tb) {  // AB_(h + s) = Ad^h AB_s, column (s, c) of the stacked AB
                lds_mma_tile(lane, 0, tile - ta, nx, nab * nu, nx, [&](int i, int k) { return Ph[i * nx + k]; },
                             [&](int k, int col) { return ABh[(size_t)(col / nu) * anu + k * nu + col % nu]; },
                             [&](int i, int col, double v) { ABh[(size_t)(h + col / nu) * anu + i * nu + col % nu] = v; });
            } else if (r == 1) {          // QCA_0 = QC Ad, QCA_1 = QC Ad^2
                const int sdx = tile - ta - tb;
                const double *B = sdx ? Pw : Ad;
                lds_mma_tile(lane, 0, 0, ny, nx, nx, [&](int i, int k) { return QC[i * nx + k]; },
                             [&](int k, int c) { return B[k * nx + c]; },
                             [&](int i, int c, double v) { QCAh[(size_t)sdx * ayx + i * nx + c] = v; });
            } else {                      // QCA_(hq + s) = QCA_s Ad^hq (Ad^hq = Pw slot r - 2), row (s, i)
                const double *B = Pw + (r - 2) * ann;
                lds_mma_tile(lane, tile - ta - tb, 0, nqa * ny, nx, nx,
                             [&](int row, int k) { return QCAh[(size_t)(row / ny) * ayx + (row % ny) * nx + k]; },
                             [&](int k, int c) { return B[k * nx + c]; },
                             [&](int row, int c, double v) { QCAh[(size_t)(hq + row / ny) * ayx + (row % ny) * nx + c] = v; });
            }
        }
    }
    __syncthreads();
    for (int tile = wv; tile < (N * nu + 15) / 16; tile += NW)  // CS_d = Cd Ad^d Bd: Cd [AB_0 .. AB_(N-1)]
        lds_mma_tile(lane, 0, tile, ny, N * nu, nx, [&](int i, int k) { return Cd[i * nx + k]; },
                     [&](int k, int col) { return ABh[(size_t)(col / nu) * anu + k * nu + col % nu]; },
                     [&](int i, int col, double v) { CS[(size_t)(col / nu) * ny * nu + i * nu + col % nu] = v; });
    __syncthreads();
    for (int e = t; e < ny * nu; e += T) {  // prefix over the horizon
        double acc = 0.0;
        for (int d = 0; d < N; d++) {
            acc += CS[(size_t)d * ny * nu + e];
            CS[(size_t)d * ny * nu + e] = acc;
        }
    }
    __syncthreads();
    MPCQ_SSTAMP(2);
    // Fx_j = 2 sum_{d >= j} CS_{d-j}' QCA_d (block row j, nu x nx) on the matrix cores: Fx = sum_d A_d B_d
    // with A_d((j,r), kk) = CS_{d-j}(kk, r) (j <= d) and B_d = QCA_d, every horizon step accumulated in
    // the same 16 x 16 output tile (rows (j, r), columns c < nx <= 16); two waves per row tile split the
    // steps by parity and add through LDS.  (Q CS_d is formed where it is read, below: no LDS copy.)
    {
        typedef double v4d __attribute__((ext_vector_type(4)));
        const int lane = t & 63, wv = t >> 6, nt = (n + 15) >> 4, nks = (ny + 3) >> 2;
        double *part = sm + S.part;  // [tile][64 lanes][4], past the live histories
        const int ti = wv % 8, half = wv / 8;
        v4d acc = {0.0, 0.0, 0.0, 0.0};
        if (ti < nt) {
            const int g = ti * 16 + (lane & 15), j = g / nu, r = g % nu, cc = lane & 15;
            for (int d = half; d < N; d += 2) {
                for (int ks = 0; ks < nks; ks++) {
                    const int kk = ks * 4 + (lane >> 4);
                    const double av = (g < n && kk < ny && j <= d) ? CS[((size_t)(d - j) * ny + kk) * nu + r] : 0.0;
                    const double bv = (cc < nx && kk < ny) ? QCAh[((size_t)d * ny + kk) * nx + cc] : 0.0;
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
                }
            }
            if (half == 1)
#pragma unroll
                for (int v = 0; v < 4; v++) part[((size_t)ti * 64 + lane) * 4 + v] = acc[v];
        }
        __syncthreads();
        if (ti < nt && half == 0) {
#pragma unroll
            for (int v = 0; v < 4; v++) {  // D(row = (lane >> 4) + 4 v, col = lane & 15)
                const int g = ti * 16 + (lane >> 4) + 4 * v, c = lane & 15;
                const double f = acc[v] + part[((size_t)ti * 64 + lane) * 4 + v];
                if (g < n && c < nx) out[L.Fx + (size_t)g * nx + c] = 2.0 * f;
            }
        }
    }
    __syncthreads();  // (the QCA history is dead: P is written below)
    MPCQ_SSTAMP(3);

    // ---- setH (:250-251): H(j1, j1+delta) = G(delta, N-1-j1-delta), G(delta, T) = sum_{t<=T}
    // CS_{t+delta}' Q CS_t; H1 = 2 ((N - max(j1, j2)) R + RD delta_{j1 j2} + H) (LL' Rbar LL has block
    // (j1, j2) = sum_{k >= max} R); P = (H1 + H1') / 2.  The block products are one GEMM on the matrix
    // cores, Z = CS' (Q CS) with CS = [CS_0 .. CS_{N-1}] (n_y x n): Z((i,r),(k,c)) = (CS_i' Q CS_k)(r,c),
    // needed for i >= k (delta = i - k, T = k) -- v_mfma_f64_16x16x4_f64 over the lower 16 x 16 tiles,
    // each product stored to its P slot (row block N-1-i, column block N-1-k); then one prefix scan over
    // T per (delta, r, c).
    {
        typedef double v4d __attribute__((ext_vector_type(4)));
        const int lane = t & 63, wv = t >> 6, nt = (n + 15) >> 4, nks = (ny + 3) >> 2;
        const int ntiles = nt * (nt + 1) / 2;
        for (int tile = wv; tile < ntiles; tile += T / 64) {  // wave-uniform: (ti >= tk) pairs
            int ti = 0, rem = tile;
            while (rem > ti) { rem -= ti + 1; ti++; }
            const int tk = rem;
            const int ga = ti * 16 + (lane & 15), gb = tk * 16 + (lane & 15);  // A row / B column of this lane
            const int ia = ga / nu, ra = ga % nu, kb = gb / nu, cb = gb % nu;
            v4d acc = {0.0, 0.0, 0.0, 0.0};
            for (int ks = 0; ks < nks; ks++) {
                const int kk = ks * 4 + (lane >> 4);
                const double av = (ga < n && kk < ny) ? CS[((size_t)ia * ny + kk) * nu + ra] : 0.0;
                const double bv = (gb < n && kk < ny) ? dot12(Q + kk * ny, 1, CS + (size_t)kb * ny * nu + cb, nu, ny) : 0.0;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
            }
#pragma unroll
            for (int v = 0; v < 4; v++) {  // D(row = (lane >> 4) + 4 v, col = lane & 15)
                const int gi = ti * 16 + (lane >> 4) + 4 * v, gk = gb;
                const int i = gi / nu, r = gi % nu, k = kb, c = cb;
                if (gi < n && gk < n && i >= k) {  // block (N-1-i, N-1-k): strictly upper, or a diagonal block
                    if (i > k) P[pk_up((N - 1 - i) * nu + r, (N - 1 - k) * nu + c, n)] = acc[v];
                    else Dblk[((N - 1 - i) * nu + r) * nu + c] = acc[v];
                }
            }
        }
    }
    __syncthreads();
    // Fu = 2 (R' + H(j, 0)) per block (:305, the .diagonal() quirk as blocks; Q symmetric): block j of
    // sum_u CS_u' Q CS_(u+j) is G(j, N-1-j)', the last value of the scan over delta = j below
    // P = (H1 + H1') / 2: an off-diagonal block's entry and its mirror come from the same scan, so the
    // thread stores their mean; a diagonal block's (r, c) and (c, r) come from two scans (Dblk, merged below)
    for (int it = t; it < N * nu * nu; it += T) {
        const int dl = it / (nu * nu), r = (it / nu) % nu, c = it % nu;
        double acc = 0.0;
        for (int tt = 0; tt + dl < N; tt++) {
            const int j2 = N - 1 - tt, j1 = j2 - dl;
            double *pe = dl ? P + pk_up(j1 * nu + r, j2 * nu + c, n) : Dblk + (j1 * nu + r) * nu + c;
            acc += *pe;
            const double rr = (double)(N - j2);  // N - max(j1, j2)
            const double up = 2.0 * (rr * R[r * nu + c] + (dl == 0 ? RD[r * nu + c] : 0.0) + acc);
            if (dl > 0) *pe = (up + 2.0 * (rr * R[c * nu + r] + acc)) / 2.0;  // H(j2, j1) = H(j1, j2)'
            else *pe = up;
        }
        out[L.Fu + (dl * nu + c) * nu + r] = 2.0 * (R[r * nu + c] + acc);
    }
    // Frs = -2 sum_{d <= N-1-j} (Q CS_d)' = -2 (Q PCS_(N-1-j))' with PCS_k = sum_{d<=k} CS_d (Fr = -2 (Qbar Su)',
    // :306, summed over the horizon blocks): CS becomes its prefix in place (setH has read it), then one
    // Q product per block
    for (int e = t; e < ny * nu; e += T) {
        double acc = 0.0;
        for (int d = 0; d < N; d++) {
            acc += CS[(size_t)d * ny * nu + e];
            CS[(size_t)d * ny * nu + e] = acc;
        }
    }
    __syncthreads();
    for (int it = t; it < n * ny; it += T) {
        const int j = it / (nu * ny), r = (it / ny) % nu, i = it % ny;
        out[L.Frs + it] = -2.0 * dot12(Q + i * ny, 1, CS + (size_t)(N - 1 - j) * ny * nu + r, nu, ny);
    }
    __syncthreads();
    MPCQ_SSTAMP(4);
    for (int e = t; e < N * nu * nu; e += T) {  // the diagonal blocks into the packed triangle
        const int j = e / (nu * nu), r = (e / nu) % nu, c = e % nu;
        if (r <= c) {
            const double v = Dblk[(j * nu + r) * nu + c];
            P[pk_up(j * nu + r, j * nu + c, n)] = r == c ? v : (v + Dblk[(j * nu + c) * nu + r]) / 2.0;
        }
    }
    for (int j = t; j < n; j += T) { Dv[j] = 1.0; Ev[j] = 1.0; }
    __syncthreads();
    MPCQ_SSTAMP(5);

    // ---- Ruiz equilibration + cost scaling (OSQP scale_data, q0 = 0 at setup, :22-23,38-39), with P
    // kept unscaled: the scaled matrix is c D P D, so its column norms are c D_j max_i D_i |P_ij| (two
    // read-only sweeps per pass instead of rescaling P).  A = [L (x) K0; -(L (x) K0)]:
    // |A^((k, r), (j, c))| = E(k,r) |K0(r, c)| D(j, c) for j <= k, and the bottom rows mirror the top
    // ones (same norms, so the same E): column norms are suffix maxima over k, row norms prefix maxima.
    const int sc = t >> 7, cj = t & 127;  // column sweeps: column cj, row slice sc (8 x 16 rows)
    auto colpart = [&](const double *Dv) {  // cm[sc][j] = max over the slice's rows of D_i |P_ij|
        if (cj < n) {
            double m0 = 0.0, m1 = 0.0;
            const int i0 = sc * 16;
            // packed index of (i, cj) walked down the column: +(n - i - 1) above the diagonal, +1 below
            int idx = pk(i0, cj, n);
#pragma unroll
            for (int ii = 0; ii < 16; ii += 2) {
                const int i = i0 + ii;
                const int idx1 = idx + (i < cj ? n - i - 1 : 1);
                if (i < n) m0 = fmax(m0, Dv[i] * fabs(P[idx]));
                if (i + 1 < n) m1 = fmax(m1, Dv[i + 1] * fabs(P[idx1]));
                idx = idx1 + (i + 1 < cj ? n - i - 2 : 1);
            }
            cm[sc * 128 + cj] = fmax(m0, m1);
        }
    };
    auto colfull = [&](int j) {
        double m = cm[j];
#pragma unroll
        for (int q = 1; q < 8; q++) m = fmax(m, cm[q * 128 + j]);
        return m;
    };
    // One column sweep per pass: pass p's Dt uses the norms of c_p D_p P D_p, and pass p-1's cost
    // scaling uses the norms of c_(p-1) D_p P D_p -- the same sweep.  Per pass: sweep | column norms,
    // A-norm block maxima, mean partials | cost scaling of the previous pass, Dt, Et, D, E | ...
    double cst = 1.0;
    double *Dc = Dv, *Dn = Dt, *Ec = Ev, *En = Et;  // current / next scaling (double-buffered)
    colpart(Dc);
    for (int pass = 0; pass <= a.scaling; pass++) {
        if (pass == 1) MPCQ_SSTAMP(8);
        __syncthreads();  // the sweep's partials; the previous pass's D, E
        if (pass == 1) MPCQ_SSTAMP(9);
        double cmt = 0.0;
        if (t < n) cmt = colfull(t);
        if ((t >> 6) >= 2 && (t >> 6) < 6) {  // waves 2..5 (no column of their own), wave 2 + c for component c,
                                                // lane k = block k: A-norm block maxima, suffix / prefix maxima
            const int k = t & 63, c = (t >> 6) - 2;  // (components >= nu are zero)
            double w0 = 0.0, w1 = 0.0;  // max_r E(k,r) |K0(r,c)|, max_q |K0(c,q)| D(k,q)
            if (k < N && c < nu)
                for (int q = 0; q < nu; q++) {
                    w0 = fmax(w0, Ec[k * nu + q] * fabs(K0[q * nu + c]));
                    w1 = fmax(w1, fabs(K0[c * nu + q]) * Dc[k * nu + q]);
                }
            w0 = lane_suffix_max(w0, k);
            w1 = lane_prefix_max(w1, k);
            if (k < 32) {
                wk[k * 4 + c] = w0;
                wk[128 + k * 4 + c] = w1;
            }
        }
        if (pass > 0 && t < 128) {  // mean column norm of c D P D (previous pass's cost scaling)
            const double sv = wsum(t < n ? cst * Dc[t] * cmt : 0.0);
            if ((t & 63) == 0) red[t >> 6] = sv;
        }
        __syncthreads();
        if (pass > 0) {
            const double mean = (red[0] + red[1]) / n;
            const double qn = mimo_limit_scaling(0.0);  // |q^| = 0 at setup
            cst *= 1.0 / mimo_limit_scaling(fmax(mean, qn));
        }
        if (pass == a.scaling) break;
        if (pass == 1) MPCQ_SSTAMP(10);
        if (t < n) {
            const int bj = t / nu, c = t % nu;
            const double va = wk[bj * 4 + c], vr = wk[128 + bj * 4 + c];  // suffix / prefix maxima (wave 0)
            const double v = fmax(cst * Dc[t] * cmt, va * Dc[t]);
            Dn[t] = Dc[t] / sqrt(mimo_limit_scaling(v));
            En[t] = Ec[t] / sqrt(mimo_limit_scaling(Ec[t] * vr));
        }
        __syncthreads();
        if (pass == 1) MPCQ_SSTAMP(11);
        double *tp = Dc; Dc = Dn; Dn = tp;
        tp = Ec; Ec = En; En = tp;
        colpart(Dc);  // norms of the rescaled P
    }
    if (Dc != Dv) {  // the final scaling back in Dv, Ev
        if (t < n) {
            Dv[t] = Dc[t];
            Ev[t] = Ec[t];
        }
        __syncthreads();
    }
    MPCQ_SSTAMP(6);

    // ---- outputs: P^ = c D P D, D, E, c, SW (suffix sums of K0' diag(2 E_k^2) K0), row-type check
    for (int e = t; e < n * L.ldp; e += T) {
        const int i = e / L.ldp, j = e % L.ldp;
        const double v = j < n ? ((cst * Dv[i]) * P[pk(i, j, n)]) * Dv[j] : 0.0;
        out[L.Ph + e] = v;
        // osqp_setup fails on a non-convex P (the reference's ctor: solverFlag false); a diagonal of
        // P^ + sigma I that is not positive proves it.  (Necessary only: a P with positive diagonal
        // that is still indefinite surfaces as the QP's NON_CVX status at the solve's factorisation.)
        if (i == j && !(v + a.sigma > 0.0)) atomicOr(a.flags, 1);
    }
    for (int j = t; j < n; j += T) {
        out[L.D + j] = Dv[j];
        out[L.E + j] = Ev[j];
        // u0 = W0 (X = U = 0): a row with E w0 beyond OSQP_INFTY * MIN_SCALING would be free
        if (!(fabs(a.w0[(size_t)pl * nu + j % nu] * Ev[j]) < kInfty * kMinScaling)) atomicOr(a.flags, 2);
    }
    if (t < nu * nu && t / nu != t % nu && K0[t] != 0.0) atomicOr(a.flags, 4);  // off-diagonal K0
    if (t == 0) {
        out[L.cs] = cst;
        out[L.cs + 1] = 1.0 / cst;
    }
    // SW: the terms s_k (c1, c2) = sum_r K0(r, c1) K0(r, c2) 2 E(k, r)^2 of every k at once (into the Ruiz
    // partials' space, dead by now), then one suffix sum over k per (c1, c2), k descending as before
    for (int it = t; it < N * nu * nu; it += T) {
        const int k = it / (nu * nu), c1 = (it / nu) % nu, c2 = it % nu;
        double sk = 0.0;
        for (int r = 0; r < nu; r++) sk += K0[r * nu + c1] * K0[r * nu + c2] * (2.0 * Ev[k * nu + r] * Ev[k * nu + r]);
        cm[it] = sk;
    }
    __syncthreads();
    for (int it = t; it < nu * nu; it += T) {
        double acc = 0.0;
        for (int k = N - 1; k >= 0; k--) {
            acc += cm[k * nu * nu + it];
            out[L.SW + k * nu * nu + it] = acc;
        }
    }
    MPCQ_SSTAMP(7);
    if (a.stamps && t == 0) a.stamps[(size_t)pl * 16 + 15] = (long long)__builtin_amdgcn_s_memrealtime();
#undef MPCQ_SSTAMP
}

// ----------------------------------------------------------------------------------------------
// solve: one 256-thread workgroup (4 waves, one per SIMD) per QP, three QPs per CU (<= 168 VGPRs).
//
// M(rho) = P^ + sigma I + rho A^'A^ lives in VGPRs, padded to 128 x 128 with the identity: thread
// (rg, cg) = (t >> 3, t & 7) holds rows 4 rg .. 4 rg + 3, columns 16 cg .. 16 cg + 15 (64 doubles).
// Gauss-Jordan inverts it in place (SPD: no pivoting), one LDS row / column broadcast and one barrier
// per step; the step loop is unrolled by 16 so the owners of row / column k address their registers
// with compile-time indices.  An ADMM iteration is one GEMV with M^-1 (the 8-lane partial sums of a
// row group reduced by DPP) and O(n) vector work spread over the same four waves: wave c holds
// component c of every horizon block (lane k = block k), so A^ x and A^' w are lane prefix / suffix
// scans (DPP row shifts plus one cross-row readlane) followed by one LDS exchange for the K0 mix
// (one barrier per product).  Per-element state lives in LDS (component-major), so only the matrix
// holds registers across the loop.
constexpr int kMimoThreads = 256;
constexpr int kSegLd = 18;                  // padded stride of a 16-element segment (LDS banks)
constexpr int kSegN = 8 * kSegLd;
__device__ __forceinline__ int seg_of(int i) { return i + 2 * (i >> 4); }
constexpr int kMimoN = 128;       // n capacity

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
{  // (bound_ctrl: a lane without a source reads 0, with no zeroed destination to copy first)
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xF, 0xF, true);
    const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, true);
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

#ifndef MPCQ_MIMO_WAVES_PER_EU
#define MPCQ_MIMO_WAVES_PER_EU 2  // two QPs per CU (256 VGPRs); 3 spills the matrix path
#endif
template <int NU, bool DK>
__global__ __launch_bounds__(kMimoThreads, MPCQ_MIMO_WAVES_PER_EU) void mimo_solve_kernel(MimoArgs a)
{
    const int b = blockIdx.x;
    if (b >= a.batch) return;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int rg = t >> 3, cg = t & 7;
    const int N = a.N, nx = a.nx, ny = a.ny, n = N * NU, m = 2 * n;
    const MimoLayout L = MimoLayout::make(N, nx, NU, ny);
    const double *ops = a.ops + (size_t)b * a.ops_stride;
    const SolverSettings &st = a.st;
    // vector role: wave c = component, lane k = horizon block
    const int c = wv, k = lane;
    const bool valid = c < NU && k < N;
    const int e = valid ? k * NU + c : 0;  // natural index (masked when !valid)
    const int vi = c * 32 + (k & 31);      // component-major slot
    // ONE (n_u = 4, diagonal K0): the matrix rows are permuted so that wave c holds the rows of
    // component c, row group rg = 8 c + j register i = (block 4 j + i, component c): the GEMV output a
    // lane consumes is produced inside its own wave (a lane permute, no LDS round trip, no barrier),
    // and an iteration has one barrier (the rhs, double-buffered).  Otherwise row group rg holds the
    // natural rows 4 rg .. 4 rg + 3.
    constexpr bool ONE = NU == 4 && DK;
    // (r = rg laundered through an empty asm at the use: hoisted out of the solve loop, these
    // indices would hold registers the matrix needs)
    auto row_nat = [](int r, int i) { return ONE ? 16 * (r & 7) + 4 * i + (r >> 3) : 4 * r + i; };
    auto row_blk = [](int r, int i) { return ONE ? 4 * (r & 7) + i : (4 * r) / NU + i / NU; };
    auto row_cmp = [](int r, int i) { return ONE ? r >> 3 : i % NU; };
    auto rg_here = [&]() {
        int r = rg;
        if (ONE) asm volatile("" : "+v"(r));
        return r;
    };
    MPCQ_MSTAMP(0, __builtin_amdgcn_s_memtime());

    // GEMV inputs and the Gauss-Jordan row broadcast: natural order in 16-element segments padded to
    // 18 (kSegLd), so the 8 column groups' 16-B reads fall in distinct LDS banks; the GEMV output is
    // component-major (the vector role reads it lane-consecutively)
    __shared__ __attribute__((aligned(16))) double s_vec[2][kSegN];  // rhs (GEMV input; alternating in ONE)
    __shared__ __attribute__((aligned(16))) double s_nat[kSegN];   // warm start: x
    __shared__ __attribute__((aligned(16))) double s_out[kMimoN];  // GEMV output, component-major
    __shared__ __attribute__((aligned(16))) double s_row[2][2][kSegN];  // pivot rows k, k + 1 (alternating)
    __shared__ double s_D[kMimoN], s_E[kMimoN], s_K0[16], s_SW[32 * 16];  // D, E component-major
    __shared__ double s_xb[4][kMimoN];  // scan exchange buffers (rotated: a buffer is rewritten 4 barriers later)
    __shared__ double s_red[2][4][16];  // cross-wave reductions (alternating)
    // the checks' settings and the cost scaling, read from LDS where they are used: held in SGPRs
    // across the solve loop they spill into VGPR lanes that every iteration reloads
    // (read back through readfirstlane: the branches on them, some holding barriers, stay uniform)
    __shared__ double s_cfg[8];
    auto cfg = [&](int i) {
        const unsigned long long u = (unsigned long long)__double_as_longlong(s_cfg[i]);
        const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u);
        const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
        return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
    };
    for (int i = t; i < kMimoN; i += kMimoThreads) {
        const int cc = i >> 5, kk = i & 31;
        const bool ok = cc < NU && kk < N;
        s_D[i] = ok ? ops[L.D + kk * NU + cc] : 1.0;
        s_E[i] = ok ? ops[L.E + kk * NU + cc] : 1.0;
    }
    for (int i = t; i < kSegN; i += kMimoThreads) s_vec[0][i] = s_vec[1][i] = s_nat[i] = 0.0;
    for (int i = t; i < 16; i += kMimoThreads) {
        const int r = i >> 2, cc = i & 3;
        s_K0[i] = (r < NU && cc < NU) ? ops[L.K0 + r * NU + cc] : 0.0;
    }
    for (int i = t; i < 32 * 16; i += kMimoThreads) {
        const int kk = i >> 4, ci = (i >> 2) & 3, cj = i & 3;
        s_SW[i] = (kk < N && ci < NU && cj < NU) ? ops[L.SW + (kk * NU + ci) * NU + cj] : 0.0;
    }

    const double c64 = ops[L.cs];
    if (t == 0) {
        s_cfg[0] = st.eps_abs; s_cfg[1] = st.eps_rel; s_cfg[2] = st.eps_prim_inf; s_cfg[3] = st.eps_dual_inf;
        s_cfg[4] = st.adaptive_rho_tolerance; s_cfg[5] = st.scaled_termination ? 1.0 : 0.0;
        s_cfg[6] = c64; s_cfg[7] = ops[L.cs + 1];
    }
    const double sigma = st.sigma, alpha = st.alpha, oma = 1.0 - st.alpha;
    const bool load = a.warm && !a.fresh;

    // this lane's element of the ADMM state (registers; the products exchange through s_xb)
    double vx = 0.0, vzt = 0.0, vzb = 0.0, vyt = 0.0, vyb = 0.0, vpx = 0.0, vqh = 0.0, vut = 0.0, vub = 0.0;
    double vrhs = 0.0, vdx = 0.0, vdpx = 0.0, vdyt = 0.0, vdyb = 0.0;
    const double vD = valid ? ops[L.D + e] : 1.0, vE = valid ? ops[L.E + e] : 1.0;
    // ---- the MPC front end: this lane's element of q and u, and the state
    int tchg = 0;
    {
        double q = 0.0, uth = 0.0, ubh = 0.0, x = 0.0, zt = 0.0, zb = 0.0, yt = 0.0, yb = 0.0;
        if (valid) {
            const double De = vD, Ee = vE;
            // setF (:372-375): q = Fx X + Fu U + Fr ref, ref = 1_N (x) yref (updateRef :378-380)
            double s0 = 0.0, s1 = 0.0, s2 = 0.0, kx = 0.0, k0u = 0.0;
            const double *fx = ops + L.Fx + (size_t)e * nx, *fr = ops + L.Frs + (size_t)e * ny;
            const double *Kc = ops + L.K + c * nx;
#pragma unroll
            for (int i = 0; i < 12; i++)
                if (i < nx) {
                    const double xv = a.X[(size_t)b * nx + i];
                    s0 = __builtin_fma(fx[i], xv, s0);
                    kx = __builtin_fma(Kc[i], xv, kx);
                }
#pragma unroll
            for (int i = 0; i < 12; i++)
                if (i < ny && a.yref) s2 = __builtin_fma(fr[i], a.yref[i], s2);
#pragma unroll
            for (int i = 0; i < NU; i++) {
                const double uv = a.U[(size_t)b * NU + i];
                s1 = __builtin_fma(ops[L.Fu + (size_t)e * NU + i], uv, s1);
                k0u = __builtin_fma(ops[L.K0 + c * NU + i], uv, k0u);
            }
            q = s0 + s1 + s2;
            if (a.q_out) a.q_out[(size_t)b * n + e] = q;
            q = (q * De) * c64;
            // (:93-99): u = W0 + Sbar X + Ku U; Sbar block rows k < s_rows = [K; -K]; Ku = [-K0; K0]
            if (!(k < a.s_rows)) kx = 0.0;
            const double w0 = ops[L.w0 + c];
            const double utop = w0 + kx + -k0u, ubot = w0 + -kx + k0u;
            if (a.u_out) {
                a.u_out[(size_t)b * m + e] = utop;
                a.u_out[(size_t)b * m + n + e] = ubot;
            }
            uth = utop * Ee;
            ubh = ubot * Ee;
            // l = -DBL_MAX (:42): every row stays an inequality while u^ is finite
            if (!(uth < kInfty * kMinScaling) || !(ubh < kInfty * kMinScaling)) tchg = 1;
            if (load) {
                x = a.xs[(size_t)b * n + e];
                zt = a.zs[(size_t)b * m + e];
                zb = a.zs[(size_t)b * m + n + e];
                yt = a.ys[(size_t)b * m + e];
                yb = a.ys[(size_t)b * m + n + e];
            }
            s_nat[seg_of(e)] = x;
        }
        vqh = q; vut = uth; vub = ubh;
        vx = x; vzt = zt; vzb = zb; vyt = yt; vyb = yb;
    }
    int status = __syncthreads_or(tchg) ? kTypeChanged : kUnsolved;
    double rho = a.fresh ? fmin(fmax(st.rho, kRhoMin), kRhoMax) : a.rhos[b];
    MPCQ_MSTAMP(1, __builtin_amdgcn_s_memtime());

    // ---- vector products (every thread calls them: each holds one barrier)
    int xb = 0;
    auto scan_x = [&](double v, bool suffix) -> const double * {
        double *buf = s_xb[xb];
        xb = (xb + 1) & 3;
        const double p = suffix ? lane_suffix(v, lane) : lane_prefix(v, lane);
        if (k < 32) buf[vi] = p;
        return buf;
    };
    auto mix_plain = [&](const double *buf) {  // sum_c' K0[c][c'] buf[c'][k]
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < NU; j++) acc = __builtin_fma(s_K0[(c & 3) * 4 + j], buf[j * 32 + (k & 31)], acc);
        return acc;
    };
    auto mix_trans = [&](const double *buf) {  // sum_r K0[r][c] buf[r][k]
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < NU; j++) acc = __builtin_fma(s_K0[j * 4 + (c & 3)], buf[j * 32 + (k & 31)], acc);
        return acc;
    };
    // (A^ x)_top = E (L (x) K0) D x (the bottom half is its negation); x = this lane's element.  With
    // every K0 diagonal (DK) the products are lane-local scans: no exchange, no barrier.
    const double k0cc = s_K0[(c & 3) * 5];
    auto A_of = [&](double xv) {
        if constexpr (DK) {
            const double p = lane_prefix(valid ? vD * xv : 0.0, lane);
            return valid ? vE * (k0cc * p) : 0.0;
        } else {
            const double *bf = scan_x(valid ? vD * xv : 0.0, false);
            __syncthreads();
            return valid ? vE * mix_plain(bf) : 0.0;
        }
    };
    // A^' [w_top; w_bot] = D (L (x) K0)' E d, d = w_top - w_bot
    auto At_of = [&](double d) {
        if constexpr (DK) {
            const double p = lane_suffix(valid ? vE * d : 0.0, lane);
            return valid ? vD * (k0cc * p) : 0.0;
        } else {
            const double *bf = scan_x(valid ? vE * d : 0.0, true);
            __syncthreads();
            return valid ? vD * mix_trans(bf) : 0.0;
        }
    };
    auto At_of2 = [&](double d1, double d2, double &o1, double &o2) {
        const double E = valid ? vE : 0.0;
        if constexpr (DK) {
            const double p1 = lane_suffix(E * d1, lane), p2 = lane_suffix(E * d2, lane);
            o1 = valid ? vD * (k0cc * p1) : 0.0;
            o2 = valid ? vD * (k0cc * p2) : 0.0;
        } else {
            const double *b1 = scan_x(E * d1, true);
            const double *b2 = scan_x(E * d2, true);
            __syncthreads();
            o1 = valid ? vD * mix_trans(b1) : 0.0;
            o2 = valid ? vD * mix_trans(b2) : 0.0;
        }
    };
    // cross-wave max / sum of R per-lane values (uniform result in every thread)
    int rb = 0;
    auto block_reduce = [&](auto &v, unsigned sum_mask) {
        constexpr int R = sizeof(v) / sizeof(double);
#pragma unroll
        for (int i = 0; i < R; i++) v[i] = ((sum_mask >> i) & 1) ? wsum(v[i]) : wmax(v[i]);
        if (lane == 0)
#pragma unroll
            for (int i = 0; i < R; i++) s_red[rb][wv][i] = v[i];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < R; i++) {
            const double *r = &s_red[rb][0][i];
            v[i] = ((sum_mask >> i) & 1) ? ((r[0] + r[16]) + (r[32] + r[48]))
                                         : fmax(fmax(r[0], r[16]), fmax(r[32], r[48]));
        }
        rb ^= 1;
    };
    int svr = 0, svw = 0;  // the rhs buffer the next GEMV reads / the next rhs goes to
    auto st_rhs = [&](double r) {
        vrhs = r;
        if (valid) s_vec[svw][seg_of(e)] = r;
        svr = svw;
        if (ONE) svw ^= 1;
    };
    auto make_rhs = [&]() {  // rhs = sigma x - q^ + A^'(rho z - y)
        const double d = (rho * vzt - vyt) - (rho * vzb - vyb);
        const double atw = At_of(valid ? d : 0.0);
        st_rhs(valid ? (sigma * vx - vqh) + atw : 0.0);
    };

    const int ct = st.check_termination;
    const int ai = (st.adaptive_rho && a.adaptive_interval) ? a.adaptive_interval : 0;
    int it = 0, nfact = 0;
    int next_check = ct ? ct : -1, next_adapt = ai ? ai : -1;

    auto finalize = [&]() {  // OSQP store_solution + the MPC front end's U += x[0:nu] (:105)
        const bool has_sol = status == kSolved || status == kSolvedInaccurate || status == kMaxIterReached;
        const bool keep = has_sol || status == kInvalidBounds || status == kTypeChanged;
        if (valid) {
            const double x = vx, zt = vzt, zb = vzb, yt = vyt, yb = vyb;
            const double D = vD, E = vE;
            const double xv = has_sol ? x * D : __builtin_nan("");
            // (the element index laundered here: hoisted out of the solve loop, the eight store addresses
            // were held across it and spilled to scratch, ~40 KB of writes per QP)
            const int eo = opaque(e);
            const size_t on = (size_t)b * n + eo, om = (size_t)b * m + eo;
            if (a.x) a.x[on] = xv;
            if (a.y) {
                const double cinv = cfg(7);
                a.y[om] = has_sol ? (yt * E) * cinv : __builtin_nan("");
                a.y[om + n] = has_sol ? (yb * E) * cinv : __builtin_nan("");
            }
            if (k == 0 && status == kSolved) a.U[(size_t)b * NU + c] = a.U[(size_t)b * NU + c] + xv;
            a.xs[on] = keep ? x : 0.0;
            a.zs[om] = keep ? zt : 0.0;
            a.zs[om + n] = keep ? zb : 0.0;
            a.ys[om] = keep ? yt : 0.0;
            a.ys[om + n] = keep ? yb : 0.0;
        }
        if (t == 0) {
            a.rhos[b] = rho;
            a.status[b] = status;
            a.iter[b] = it;
            a.rho_out[b] = rho;
        }
    };

    if (status != kUnsolved) {
        finalize();
        return;
    }
    make_rhs();  // (its barrier also orders the front end's LDS writes before every read below)

    int fail = 0;
    double Mb[4][16];
    // rows row_nat(i), columns 16 cg + j (P^ rows are padded to L.ldp: aligned, in-bounds loads);
    // the padding beyond n is the identity
    auto load_P = [&]() {
        const int seg = 16 * cg < L.ldp - 16 ? 16 * cg : L.ldp - 16;
        const int r = rg_here();
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int gi = row_nat(r, i);
            const double2 *row = (const double2 *)(ops + L.Ph + (size_t)(gi < n ? gi : n - 1) * L.ldp + seg);
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const double2 v = row[j];
                const int gj = 16 * cg + 2 * j;
                Mb[i][2 * j] = (gi < n && gj < n) ? v.x : (gi == gj ? 1.0 : 0.0);
                Mb[i][2 * j + 1] = (gi < n && gj + 1 < n) ? v.y : (gi == gj + 1 ? 1.0 : 0.0);
            }
#pragma unroll
            for (int j = 0; j < 16; j++) asm volatile("" : "+v"(Mb[i][j]));  // one row of loads in flight
        }
    };
    // + sigma I + r D SW[max(bi, bj)] D on the n x n part (block of row gi: row_blk(i))
    auto add_kkt = [&](double r) {
        double di[4];
        const int rl = rg_here();
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int bi = row_blk(rl, i);
            di[i] = s_D[row_cmp(rl, i) * 32 + (bi < 31 ? bi : 31)];
        }
#pragma unroll
        for (int jc = 0; jc < 4; jc++) {
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const int j = 4 * jc + jj, gj = 16 * cg + j;
                const int bj = (16 * cg) / NU + j / NU, cj = j % NU;
                const double dj = s_D[cj * 32 + (bj < 31 ? bj : 31)];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int gi = row_nat(rl, i), bi = row_blk(rl, i), ci = row_cmp(rl, i);
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
    // part[i] = row row_nat(i) of M . in, in all 8 lanes of the row group (combined by DPP)
    auto gemv_rows = [&](const double *in, double (&part)[4]) {
        double s0[4], s1[4];
#pragma unroll
        for (int i = 0; i < 4; i++) s0[i] = s1[i] = 0.0;
        const double2 *v2 = (const double2 *)(in + kSegLd * cg);
        double2 q0 = v2[0], q1 = v2[1];
#pragma unroll
        for (int h = 0; h < 4; h++) {  // 4-column chunks (register budget), the next one in flight
            const double2 p0 = q0, p1 = q1;
            if (h < 3) {
                q0 = v2[2 * h + 2];
                q1 = v2[2 * h + 3];
            }
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
#pragma unroll
        for (int i = 0; i < 4; i++) {
            part[i] = s0[i] + s1[i];
            part[i] += dpp_t<0xB1>(part[i]);   // quad_perm [1,0,3,2]
            part[i] += dpp_t<0x4E>(part[i]);   // quad_perm [2,3,0,1]
            part[i] += dpp_t<0x141>(part[i]);  // row_half_mirror: the other quad of the 8
        }
    };
    // outv[component-major slot of row_nat(i)] = row row_nat(i) of M . in
    auto gemv = [&](const double *in, double *outv) {
        double part[4];
        gemv_rows(in, part);
        if (cg == 0)
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (row_nat(rg, i) < n) outv[row_cmp(rg, i) * 32 + row_blk(rg, i)] = part[i];
    };
    // ONE: this lane's element (block k, component c) of M . in, from lane 8 (k >> 2) + (k & 3) of the
    // same wave, whose register row (its cg & 3) is block k
    auto gemv_own = [&](const double *in) {
        double part[4];
        gemv_rows(in, part);
        const int ci = cg & 3;
        const double sel = ci == 0 ? part[0] : ci == 1 ? part[1] : ci == 2 ? part[2] : part[3];
        return __shfl(sel, 8 * ((k >> 2) & 7) + (k & 3), 64);
    };
    // Gauss-Jordan on pivot pairs K = {k, k + 1} (SPD: no pivoting; n odd pairs the last pivot with
    // the identity padding, which the update leaves as it is): A <- A - A(:,K) A_KK^-1 A(K,:) off K,
    // then rows K <- A_KK^-1 A(K,:), columns K <- -A(:,K) A_KK^-1, A_KK <- A_KK^-1.  One LDS broadcast of
    // the two rows and one barrier per pair; column K is read off the rows (the trailing block stays
    // symmetric, a_ik = a_ki, and the pivoted rows are its negation, a_ik = -a_ki: [A11^-1,
    // A11^-1 A12; -A21 A11^-1, S]).  k = 16 kb + kk with kk unrolled: the owner of column k is cg == kb
    // (register column kk), of row k rg == k >> 2 (register row kk & 3; ONE: rg == 8 (kk & 3) + kb,
    // register row kk >> 2).  Every thread forms A_KK^-1 from the broadcast (one division); the row
    // owners' rows restart from 0 and take the same FMA update with multipliers A_KK^-1.
    auto invert = [&]() {
        const int nkb = (n + 15) >> 4;
        for (int kb = 0; kb < nkb; kb++) {
#pragma unroll
            for (int kk = 0; kk < 16; kk += 2) {
                const int kp = 16 * kb + kk;
                if (kp >= n) continue;  // (not break: the loop must fully unroll, or Mb leaves the VGPRs)
                const int p = (kk >> 1) & 1;
                const int rk = ONE ? kk >> 2 : kk & 3, rl = ONE ? kk >> 2 : (kk & 3) + 1;
                const bool ownk = ONE ? rg == 8 * (kk & 3) + kb : rg == (kp >> 2);
                const bool ownl = ONE ? rg == 8 * (kk & 3) + 8 + kb : rg == (kp >> 2);
                const bool coln = cg == kb;
                if (ownk) {
                    double2 *r2 = (double2 *)&s_row[p][0][kSegLd * cg];
#pragma unroll
                    for (int j = 0; j < 8; j++) r2[j] = make_double2(Mb[rk][2 * j], Mb[rk][2 * j + 1]);
                }
                if (ownl) {
                    double2 *r2 = (double2 *)&s_row[p][1][kSegLd * cg];
#pragma unroll
                    for (int j = 0; j < 8; j++) r2[j] = make_double2(Mb[rl][2 * j], Mb[rl][2 * j + 1]);
                }
                __syncthreads();
                const double *R0 = s_row[p][0], *R1 = s_row[p][1];
                const double2 *k2 = (const double2 *)&R0[kSegLd * cg], *l2 = (const double2 *)&R1[kSegLd * cg];
                double2 qk = k2[0], ql = l2[0];  // row chunk 0, in flight with the pivot block
                const double2 pk = *(const double2 *)&R0[kSegLd * kb + kk];  // a_kk, a_kl
                const double all = R1[kSegLd * kb + kk + 1];
                const double det = __builtin_fma(pk.x, all, -(pk.y * pk.y));
                if (!(pk.x > 0.0) || !(det > 0.0)) fail = 1;
                const double idet = 1.0 / det;
                const double ikk = all * idet, ikl = -pk.y * idet, ill = pk.x * idet;
                double ck[4], cl[4];  // a_ik, a_il of this thread's rows, read off rows k, l
                if constexpr (ONE) {  // columns 16 (rg & 7) + 4 i + (rg >> 3)
                    const int r = rg_here();
                    const int o = kSegLd * (r & 7) + (r >> 3);
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        ck[i] = R0[o + 4 * i];
                        cl[i] = R1[o + 4 * i];
                    }
                } else {
                    const int o = kSegLd * (rg >> 2) + 4 * (rg & 3);
                    const double2 u0 = *(const double2 *)&R0[o], u1 = *(const double2 *)&R0[o + 2];
                    const double2 w0 = *(const double2 *)&R1[o], w1 = *(const double2 *)&R1[o + 2];
                    ck[0] = u0.x; ck[1] = u0.y; ck[2] = u1.x; ck[3] = u1.y;
                    cl[0] = w0.x; cl[1] = w0.y; cl[2] = w1.x; cl[3] = w1.y;
                }
                double fk[4], fl[4];  // -A(i,K) A_KK^-1 (rows K: A_KK^-1)
                {
                    const int r = rg_here();
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const bool piv = row_nat(r, i) < kp;
                        const double a0 = piv ? -ck[i] : ck[i], a1 = piv ? -cl[i] : cl[i];
                        fk[i] = -__builtin_fma(a0, ikk, a1 * ikl);
                        fl[i] = -__builtin_fma(a0, ikl, a1 * ill);
                    }
                }
                if (ownk) {  // row k <- ikk a_k. + ikl a_l. (the row restarts from 0)
                    fk[rk] = ikk;
                    fl[rk] = ikl;
#pragma unroll
                    for (int j = 0; j < 16; j++) Mb[rk][j] = 0.0;
                }
                if (ownl) {  // row l <- ikl a_k. + ill a_l.
                    fk[rl] = ikl;
                    fl[rl] = ill;
#pragma unroll
                    for (int j = 0; j < 16; j++) Mb[rl][j] = 0.0;
                }
#pragma unroll
                for (int h = 0; h < 8; h++) {  // 2-column chunks of both rows, the next one in flight
                    double2 nk = qk, nl = ql;
                    if (h < 7) {
                        nk = k2[h + 1];
                        nl = l2[h + 1];
                    }
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        Mb[i][2 * h] = __builtin_fma(fk[i], qk.x, __builtin_fma(fl[i], ql.x, Mb[i][2 * h]));
                        Mb[i][2 * h + 1] = __builtin_fma(fk[i], qk.y, __builtin_fma(fl[i], ql.y, Mb[i][2 * h + 1]));
                    }
                    qk = nk;
                    ql = nl;
                    // pin the updates here: sunk below the fix-up branches they would keep every
                    // chunk of the rows live (register budget)
#pragma unroll
                    for (int i = 0; i < 4; i++) asm volatile("" : "+v"(Mb[i][2 * h]), "+v"(Mb[i][2 * h + 1]));
                }
                if (coln) {  // columns K: -A(i,K) A_KK^-1, rows K: A_KK^-1
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        Mb[i][kk] = fk[i];
                        Mb[i][kk + 1] = fl[i];
                    }
                    if (ownk) {
                        Mb[rk][kk] = ikk;
                        Mb[rk][kk + 1] = ikl;
                    }
                    if (ownl) {
                        Mb[rl][kk] = ikl;
                        Mb[rl][kk + 1] = ill;
                    }
                }
            }
        }
    };

    load_P();
    bool refactor = true, loaded = true, px_pending = load;
    for (;;) {
        if (refactor) {  // (re-)invert M(rho); the first factorisation also forms P^ x of a warm start
            if (!loaded) load_P();
            loaded = false;
            if (px_pending) {
                gemv(s_nat, s_out);
                __syncthreads();
                if (valid) vpx = s_out[vi];
                __syncthreads();  // s_out is the GEMV output below
                px_pending = false;
            }
            add_kkt(rho);
            invert();  // its first barrier orders the rhs writes before the GEMV below
            nfact++;
#ifndef MPCQ_GJ_STAMPS
            MPCQ_MSTAMP(2, __builtin_amdgcn_s_memtime());
#endif
            if (fail) {  // P^ + sigma I + rho A^'A^ not positive definite
                status = kNonCvx;
                finalize();
                break;
            }
            refactor = false;
        }
        double xt;
        if constexpr (ONE) {
            xt = gemv_own(s_vec[svr]);
        } else {
            gemv(s_vec[svr], s_out);
            __syncthreads();  // x~ ready
            xt = s_out[vi];
        }
        xt = valid ? xt : 0.0;
        it++;
        const bool at_check = it == next_check, at_adapt = it == next_adapt;
        if (at_check) next_check += ct;
        if (at_adapt) next_adapt += ai;
        const bool last = it == st.max_iter;
        const bool info = at_check || at_adapt || last;
        const double rinv = 1.0 / rho;
        // ---- x~ = M^-1 rhs ; z~ = A^ x~ ; P^ x~ = rhs - sigma x~ - rho A^'z~ ; relax ; project ; dual
        const double ztl = A_of(xt);
        double d2, dr, xn;
        {
            const double x = vx;
            xn = __builtin_fma(alpha, xt, oma * x);
            double zt = vzt, zb = vzb, yt = vyt, yb = vyb;
            const double ut = vut, ub = vub;
            // top row e and bottom row n + e (z~_bot = -z~_top)
            const double vt = __builtin_fma(alpha, ztl, oma * zt);
            const double zn_t = fmin(__builtin_fma(rinv, yt, vt), ut);
            const double dyt = rho * (vt - zn_t);
            yt = __builtin_fma(rho, vt - zn_t, yt);
            zt = zn_t;
            const double vb = __builtin_fma(alpha, -ztl, oma * zb);
            const double zn_b = fmin(__builtin_fma(rinv, yb, vb), ub);
            const double dyb = rho * (vb - zn_b);
            yb = __builtin_fma(rho, vb - zn_b, yb);
            zb = zn_b;
            d2 = 2.0 * ztl;
            dr = (rho * zt - yt) - (rho * zb - yb);  // next rhs (rho unchanged)
            {
                vx = valid ? xn : 0.0;
                vdx = valid ? xn - x : 0.0;
                vzt = valid ? zt : 0.0; vzb = valid ? zb : 0.0;
                vyt = valid ? yt : 0.0; vyb = valid ? yb : 0.0;
                vdyt = valid ? dyt : 0.0; vdyb = valid ? dyb : 0.0;
            }
        }
        double gz, atw = 0.0;
        if (info)
            gz = At_of(valid ? d2 : 0.0);
        else
            At_of2(valid ? d2 : 0.0, valid ? dr : 0.0, gz, atw);
        {  // carried P^ x (KKT identity)
            const double px = vpx;
            const double ptx = (vrhs - sigma * xt) - rho * gz;
            const double pxn = __builtin_fma(alpha, ptx, oma * px);
            {
                vpx = valid ? pxn : 0.0;
                vdpx = valid ? pxn - px : 0.0;
            }
        }
        int ctl = 0;  // 0 continue, 1 refactor, 2 done
        if (info) {
            // ---- update_info: residuals (scaled norms _r, unscaled _s as OSQP reports them)
            // OSQP's tests read ||z||, ||A x|| only as max(||z||, ||A x||) and ||q||, ||A' y||, ||P x|| only as
            // their maximum: one reduction of the lanes' maxima each (max is exact in any order), eight
            // values per check instead of fourteen
            double v[8];
            {
                const double ax = A_of(valid ? vx : 0.0);
                const double zt = vzt, zb = vzb, ei = 1.0 / vE;
                const double rt = ax - zt, rbm = -ax - zb;
                v[0] = fmax(fabs(rt), fabs(rbm));                                  // ax_z
                v[1] = fmax(fabs(ei * rt), fabs(ei * rbm));                        // ax_zs
                v[2] = fmax(fmax(fabs(zt), fabs(zb)), fabs(ax));                   // max(zn_r, axn_r)
                v[3] = fmax(fmax(fabs(ei * zt), fabs(ei * zb)), fabs(ei * ax));    // max(zn_s, axn_s)
            }
            {
                const double aty = At_of(valid ? vyt - vyb : 0.0);
                const double qh = vqh, px = vpx, di = 1.0 / vD;
                const double r = (qh + px) + aty;
                v[4] = fabs(r);                                                    // dr_r
                v[5] = fabs(di * r);                                               // dr_s
                v[6] = fmax(fmax(fabs(qh), fabs(aty)), fabs(px));                  // max(qn_r, atyn_r, pxn_r)
                v[7] = fmax(fmax(fabs(di * qh), fabs(di * aty)), fabs(di * px));   // max(qn_s, atyn_s, pxn_s)
            }
            if (!valid)
#pragma unroll
                for (int i = 0; i < 8; i++) v[i] = 0.0;
            block_reduce(v, 0u);
            const double ax_z = v[0], ax_zs = v[1], zax_r = v[2], zax_s = v[3];
            const double dr_r = v[4], dr_s = v[5], qap_r = v[6], qap_s = v[7];
            const double cinv = cfg(7);
            const bool scaled_term = cfg(5) != 0.0;
            const double pri_res = scaled_term ? ax_z : ax_zs;
            const double dua_res = scaled_term ? dr_r : cinv * dr_s;

            // OSQP is_primal_infeasible on delta_y (u finite, l = -inf on every row: d = max(d, 0))
            auto primal_inf = [&](double eps) -> bool {
                const double dt_ = valid ? fmax(vdyt, 0.0) : 0.0, db_ = valid ? fmax(vdyb, 0.0) : 0.0;
                const double E = vE;
                double w[2];
                w[0] = fmax(fabs(scaled_term ? dt_ : E * dt_), fabs(scaled_term ? db_ : E * db_));  // ndy
                w[1] = valid ? vut * dt_ + vub * db_ : 0.0;                            // lhs
                block_reduce(w, 2u);
                const double ndy = w[0], lhs = w[1];
                if (!(ndy > kDivisionTol && lhs < eps * ndy)) return false;
                const double atd = At_of(dt_ - db_);
                double u[1] = {valid ? fabs(scaled_term ? atd : atd / vD) : 0.0};
                block_reduce(u, 0u);
                return u[0] < eps * ndy;
            };
            // OSQP is_dual_infeasible on delta_x (P^ delta_x = delta of the carried P^ x)
            auto dual_inf = [&](double eps) -> bool {
                const double dx = valid ? vdx : 0.0, D = vD;
                double w[3];
                w[0] = valid ? vqh * dx : 0.0;                                          // qdx
                w[1] = fabs(scaled_term ? dx : D * dx);                                      // ndx
                w[2] = valid ? fabs(scaled_term ? vdpx : vdpx / D) : 0.0;          // |P^ dx|
                block_reduce(w, 1u);
                const double qdx = w[0], ndx = w[1], npdx = w[2];
                const double cs = scaled_term ? 1.0 : cfg(6);
                if (!(qdx < 0.0 && ndx > kDivisionTol && qdx < -cs * eps * ndx)) return false;
                if (!(npdx < cs * eps * ndx)) return false;
                const double adx = A_of(dx);
                double u[1] = {0.0};
                if (valid) {
                    const double sv = scaled_term ? adx : adx / vE;
                    if (vut < kInfty * kMinScaling && sv > eps * ndx) u[0] = 1.0;   // top row
                    if (vub < kInfty * kMinScaling && -sv > eps * ndx) u[0] = 1.0;  // bottom row
                }
                block_reduce(u, 0u);
                return u[0] == 0.0;
            };
            auto check = [&](bool approx) -> int {
                const double mul = approx ? 10.0 : 1.0;
                const double ea = cfg(0) * mul, er = cfg(1) * mul;
                if (pri_res > kInfty || dua_res > kInfty) return kNonCvx;
                const double ep = ea + er * (scaled_term ? zax_r : zax_s);
                const double ed = ea + er * (scaled_term ? qap_r : cinv * qap_s);
                const bool pok = pri_res < ep, dok = dua_res < ed;
                if (pok && dok) return approx ? kSolvedInaccurate : kSolved;
                if (!pok && primal_inf(cfg(2) * mul))
                    return approx ? kPrimalInfeasibleInaccurate : kPrimalInfeasible;
                if (!dok && dual_inf(cfg(3) * mul))
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
                        const double pr = ax_z / (zax_r + kDivisionTol);
                        const double dn = qap_r;
                        const double du = dr_r / (dn + kDivisionTol);
                        double rn = rho * sqrt(pr / (du + kDivisionTol));
                        rn = fmin(fmax(rn, kRhoMin), kRhoMax);
                        if (rn > rho * cfg(4) || rn < rho / cfg(4)) {
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
            __syncthreads();  // every lane's state is final
            finalize();
            break;
        }
        if (info)
            make_rhs();  // rho may have changed
        else
            st_rhs(valid ? (sigma * xn - vqh) + atw : 0.0);
        refactor = ctl == 1;
        __syncthreads();  // next rhs ready
    }
#ifndef MPCQ_GJ_STAMPS
    if (a.stamps && t == 0) {
        a.stamps[(size_t)blockIdx.x * 8 + 3] = (long long)__builtin_amdgcn_s_memtime();
        a.stamps[(size_t)blockIdx.x * 8 + 4] = it;
        a.stamps[(size_t)blockIdx.x * 8 + 5] = nfact;
    }
#endif
}

}  // namespace mpcq

extern "C" int mpcq_internal_mimo_setup_launch(const mpcq::MimoSetupArgs *a, hipStream_t s)
{
    const mpcq::MimoSetupShape S = mpcq::MimoSetupShape::make(a->N, a->nx, a->nu, a->ny);
    const size_t lds = 8 * S.total;
    if (a->nx > 12 || a->nu > 4 || a->ny > 12 || a->N * a->nu > mpcq::kMimoN || a->N > 32 || lds > 160 * 1024)
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
#define MPCQ_MIMO_LAUNCH(U)                                                                  \
    do {                                                                                     \
        if (a->diag_k0)                                                                      \
            hipLaunchKernelGGL((mpcq::mimo_solve_kernel<U, true>), grid, block, 0, s, *a);   \
        else                                                                                 \
            hipLaunchKernelGGL((mpcq::mimo_solve_kernel<U, false>), grid, block, 0, s, *a);  \
    } while (0)
    switch (a->nu) {
    case 1: MPCQ_MIMO_LAUNCH(1); break;
    case 2: MPCQ_MIMO_LAUNCH(2); break;
    case 4: MPCQ_MIMO_LAUNCH(4); break;
    default: return -1;
    }
#undef MPCQ_MIMO_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
