// solvempc_amd/csrc/mpcq_internal.h — device data layout shared by the setup and ADMM kernels.
//
// Factorisations used on the device (replace OSQP's QDLDL LDL' of the KKT matrix): for a plant
// with scaled data (P^, A^) and constraint-type pattern s (rho_j = rho*s_j, or RHO_MIN for free
// rows), the reduced KKT matrix is a one-parameter family
//        M(rho) = P~ + rho G,   P~ = P^ + sigma I + RHO_MIN sum_free a_j a_j',  G = sum s_j a_j a_j'.
// * Eigen-basis (shared plants; per-plant shapes beyond one wave): setup computes W' P~ W = I,
//   W' G W = diag(lambda), so that M(rho)^-1 = W diag(1/(1 + rho lambda)) W' for EVERY rho: an
//   adaptive-rho update (OSQP adapt_rho) only rescales a diagonal, and all QPs of a plant share W
//   whatever rho each one has reached.  The iterate keeps x in that basis (x^ = W x').
// * Direct inverse (per-plant batches, n <= 32, m <= 64; setup_inv_kernel): M(rho0)^-1 itself, the
//   iterate in the scaled basis (x' = x^).  The same operator slots then hold W = W^-1 = I,
//   lambda = 0, sigma W'W = sigma M^-1, G = M^-1, Bt = A^ M^-1 (so one iteration is the same code
//   for both), and rho0 = the rho they were built for; a QP whose rho moves away from rho0 rebuilds
//   M^-1 in its kernel (OSQP's refactorisation, mpcq_wave.h).
#pragma once
#include <hip/hip_runtime.h>

namespace mpcq {

// OSQP v0.6 constants (constants.h)
constexpr double kInfty = 1e30;
constexpr double kMinScaling = 1e-4;
constexpr double kMaxScaling = 1e4;
constexpr double kRhoMin = 1e-6;
constexpr double kRhoMax = 1e6;
constexpr double kRhoTol = 1e-4;
constexpr double kRhoEqOverIneq = 1e3;
constexpr double kDivisionTol = 1.0 / kInfty;

// Per-plant operators, padded to the kernel capacity (NC variables, MC rows).  Row-major.
// Every array is [n_plants][...]; padding entries are zero (padded rows: free, E = 1).
template <typename T>
struct PlantOps {
    const T *lam;    // NC          generalised eigenvalues
    const T *W;      // NC x NC     x^ = W x'
    const T *sWtW;   // NC x NC     sigma * W'W   (the sigma x term of the KKT rhs, in W-basis)
    const T *WtA;    // MC x NC     B = A^ W   (row j: b_j)
    const T *PW;     // NC x NC     P^ W       (P x^ for the dual residual)
    const T *Winv;   // NC x NC     W^-1 = V' L'  (osqp_warm_start: x' = W^-1 x^)
    const T *Ah;     // MC x NC     A^         (A' y for the dual residual)
    const T *D;      // NC          Ruiz D     (Dinv = 1/D)
    const T *E;      // MC          Ruiz E
    const T *Dinv;   // NC
    const T *Einv;   // MC
    const T *cs;     // 2           c, 1/c
    const T *rscale; // MC          rho_j = rho * rscale_j  (0 => free row => RHO_MIN)
    const int *ctype;// MC          OSQP constr_type: -1 free, 0 inequality, 1 equality
};
// (G: NC x NC, g = -G' q^; Bt: MC x NC, the x-side product's operator rows; rho0: 1.  Eigen-basis:
// G = W, Bt = A^ W, rho0 = -1.  Direct inverse: G = M^-1, Bt = A^ M^-1, rho0 = the built-for rho.)

// Shapes of one plant's operator block, in elements, for capacities (nc, mc).
struct OpsLayout {
    int nc, mc;
    size_t lam, W, sWtW, WtA, PW, Winv, Ah, D, E, Dinv, Einv, cs, rscale, G, Bt, rho0, total;
    __host__ __device__ static constexpr OpsLayout make(int nc, int mc)
    {
        OpsLayout L{};
        L.nc = nc;
        L.mc = mc;
        size_t o = 0;
        L.lam = o; o += nc;
        L.W = o; o += (size_t)nc * nc;
        L.sWtW = o; o += (size_t)nc * nc;
        L.WtA = o; o += (size_t)mc * nc;
        L.PW = o; o += (size_t)nc * nc;
        L.Winv = o; o += (size_t)nc * nc;
        L.Ah = o; o += (size_t)mc * nc;
        L.D = o; o += nc;
        L.E = o; o += mc;
        L.Dinv = o; o += nc;
        L.Einv = o; o += mc;
        L.cs = o; o += 2;
        L.rscale = o; o += mc;
        L.G = o; o += (size_t)nc * nc;
        L.Bt = o; o += (size_t)mc * nc;
        L.rho0 = o; o += 2;
        L.total = o;
        return L;
    }
};

struct SolverSettings {
    double rho, sigma, alpha;
    double eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
    double adaptive_rho_tolerance;
    int max_iter, check_termination, adaptive_rho, adaptive_rho_interval;
    int warm_start, scaled_termination, scaling;
};

// Status values (mirror include/mpcq.h)
enum : int {
    kSolved = 1,
    kSolvedInaccurate = 2,
    kPrimalInfeasibleInaccurate = 3,
    kDualInfeasibleInaccurate = 4,
    kMaxIterReached = -2,
    kPrimalInfeasible = -3,
    kDualInfeasible = -4,
    kNonCvx = -7,
    kUnsolved = -10,
    kInvalidBounds = -20,
    kTypeChanged = -21,
};

// Arguments of the setup kernel (one 64-lane workgroup per plant).
struct SetupArgs {
    int n, m, nc, mc, n_plants;
    int scaling;       // Ruiz passes
    double sigma, rho;
    double jacobi_tol;  // Jacobi stops at off(C)^2 <= jacobi_tol * diag(C)^2 (fp64 solves 1e-32, fp32 1e-20)
    const double *P, *q0, *A, *l0, *u0;  // [plant] n*n, n, m*n, m, m
    double *ops;       // [plant] OpsLayout(nc, mc).total
    int *ctype;        // [plant] mc
    double *scratch;   // [plant] scratch_len(n, m)
    int *status;       // [plant] 0 ok, else error
    long long *prof;   // debug (MPCQ_SETUP_PROF): [plant][16] stage clock stamps, or null
    int *flags;        // OR over plants: 1 setup failed (non-convex), 2 a row is not an inequality,
                       // 4 the Jacobi eigen-solve hit its sweep cap (inaccurate basis)
};

// Phase lists of the tile path: the QPs a phase hands on are appended to one of kShards segments
// (the appending workgroup's blockIdx % kShards), each with its own counter on its own 128-B line, so
// the ~3,000 waves reaching a phase boundary together do not serialise on one device-scope counter
// (~11 ns per atomic).  Segment s holds entries [s cap, s cap + count[s * kStride]).  The next phase's
// workgroup b serves segment b % kShards (its 64 G slots at (b / kShards) 64 G): the workgroups of a
// segment are exactly those that can have filled it, so every entry is covered.
struct ListSeg {
    static constexpr int kShards = 32;
    static constexpr int kStride = 32;  // ints per counter line
    static constexpr int kCounters = kShards * kStride;
    __host__ __device__ static constexpr int cap(int batch) { return (batch + kShards - 1) / kShards + 256; }
};

// Hardest-first order of a shared-plant MPC step (mpcq_order.hip): the key v = max_j (A x_u - u)_j of a
// QP (its unconstrained optimum's largest bound violation) falls in bin floor(16 log2|v|) + 256 (16 bins
// per octave, 2^-16 .. 2^16, clamped), |v| = 0 in bin 0, a non-finite |v| in the last; phase 0 runs bin
// 0's QPs first.  The host's map (m rows of kStride doubles): v_j = r[0..nx) . X + r[8] U + r[9] +
// r[10] xref.  A QP's rank inside its bin takes the low kRankBits of its key word.
struct OrderBins {
    static constexpr int kBins = 512;
    static constexpr int kPerOctave = 16;
    static constexpr int kRankBits = 22;  // batches below 4,194,304 QPs
    static constexpr int kStride = 12;
    static constexpr int kMaxRows = 64;
    __host__ __device__ static int bin(double v)
    {
        const double a = v < 0.0 ? -v : v;
        if (!(a < __builtin_inf())) return kBins - 1;  // inf, NaN
        if (a == 0.0) return 0;
        int e = 0;
        const double f = __builtin_frexp(a, &e);  // a = f 2^e, f in [0.5, 1): log2 a = e - 1 + log2(2 f)
        // the fraction's 16 sub-octave steps from its top mantissa bits (a monotone map of a within the
        // octave: ordering only needs monotone bins, not exact logarithms)
        const int sub = (int)((f - 0.5) * 32.0);  // 0 .. 15
        const int i = (e - 1) * kPerOctave + sub + kBins / 2;
        return i < 0 ? 0 : (i > kBins - 2 ? kBins - 2 : i);
    }
};

// Arguments of the ADMM kernel (one QP per lane).
// Persistent receding-horizon stream (config 5): control steps first_step .. first_step + steps - 1 of
// the simulated plant X <- Ad X + Bd U + w (mpcq_plant_sim.h) between the solves.
struct StreamArgs {
    int steps, nx, shared;        // shared: every QP's plant is plant 0
    int cpw;                      // tile stream: plants (columns) per wave
    const double *Ad, *Bd;        // [plant] nx*nx, nx
    unsigned long long seed;
    long long first_qp, first_step;
    double noise_std;
    int occ;                      // tile stream: waves per SIMD the kernel is compiled for (1: at most one
                                  // wave per SIMD, the whole register file, no spills; 2 otherwise)
};

template <typename T>
struct AdmmArgs {
    int batch, n, m;
    int shared;                 // 1: every QP uses plant 0
    size_t ops_stride;          // elements per plant block (OpsLayout::total)
    PlantOps<T> ops;
    const int *ctype;           // [plant][mc]
    SolverSettings st;
    int adaptive_interval;      // resolved (0 -> 4*check_termination)
    int all_ineq;               // every row of every plant is an inequality (constr_type 0)
    int paired;                 // shared plant with m = 2n, n % 4 == 0, A rows n + j == -rows j (tile kernel)
    int lower_free;             // every l^ of every QP is below -OSQP_INFTY*MIN_SCALING
    // per-QP inputs (fp64, QP-major as in the C ABI)
    const double *q, *u, *l;    // batch*n, batch*m, batch*m (l may be a single shared m-vector)
    int l_shared;
    // state (QP-major [batch][row], T) for warm start
    T *xs, *zs, *ys, *rhos;
    int warm;                   // read xs/zs/ys at entry (settings.warm_start)
    int fresh;                  // ignore stored state: x = z = y = 0, rho = settings.rho (mpcq_reset)
    // snapshots for the infeasibility certificates (QP-major)
    T *snap_x, *snap_y;
    // outputs
    double *x, *y, *rho_out;
    int *status, *iter;
    // receding-horizon stream counters (mpcq_mpc_run_device; null otherwise): per QP, the iterations of
    // every solve and the solves that did not end SOLVED, accumulated at finalize
    int *it_acc, *uns_acc;
    // MPC front end (n = N, m = 2N); null when unused
    int mpc, nx;
    const double *X, *Fx, *Fu, *Fr, *Sbar, *Ku, *W0;
    double *U, *q_out, *u_out;
    double *X_save, *U_save;    // tile path: phase 0 saves X [batch][nx], U [batch] (q, u computed on demand)
    double xref;
    int mpc_u;                  // U += x[0] at termination (the front end may have run in an earlier phase)
    // tile kernel (shared plant): MFMA operand images and the phase machinery (mpcq_tile.h)
    const T *img;               // TileLayout images of the plant
    const int *list_in;         // active QP indices of this phase (null: identity 0..batch-1), ListSeg layout
    const int *count_in;        // ListSeg counters of list_in (null: batch)
    int *list_out, *count_out;  // QPs still running at stop_iter (appended, ListSeg layout)
    // ListSeg counter blocks this launch zeroes on entry (workgroup 0; null: none): the next phase's
    // output counters, and in a chain's last launch the first phase's (for the next solve)
    int *zero_cnt, *zero_cnt0;
    int list_seg;               // ListSeg segment capacity
    int *it_state;              // [batch] iterations done so far in this solve
    int qp0;                    // QP index of identity-list slot 0 (sub-batch parts of a tile solve)
    // phase 0 of a tile solve in hardest-first order (mpcq_order.hip; null: index order): slot i runs QP
    // ord_list[i]; workgroup 0 zeroes the OrderBins::kBins counters ord_zero for the next solve
    const int *ord_list;
    int *ord_zero;
    int stop_iter;              // phase boundary (multiple of check_termination, or max_iter)
    int resume;                 // 1: phase >= 2 (state, rho and iteration count come from the buffers)
    long long *stamps;          // debug build (MPCQ_DEBUG_HOOKS): [wave][8] s_memtime stamps, or null
    StreamArgs sim;             // the tile kernel's stream mode (tile_stream_launch): plants and noise
    // OSQP is_dual_infeasible needs ||P^ dx|| < c eps ||dx|| (norms as the termination mode reads them);
    // with lambda_min(P^) >= mu > 0 the left side is >= kappa ||dx|| (kappa from mu, D and n: host,
    // setup_on_device), so for kappa > 2 c eps the certificate cannot hold and its products are skipped
    // (0: always evaluated)
    double dinf_kappa;
    // mixed precision (MPCQ_F64_MIXED contexts, the tile kernel's paired loop): the last mix_r iterations
    // before every info iteration run in fp64, the earlier plain ones in fp32 (0: all fp64)
    int mix_r;
    // waves per SIMD of the f32 paired tile kernel (0: the default, 3; 2: the OCC-2 variant)
    int tile_occ;
    // (T) eps_abs, eps_rel, eps_prim_inf, eps_dual_inf times T(10), formed on the host in T: the tile
    // kernel's approximate check_termination (OSQP auxil.c, the 10x tolerances after max_iter)
    T eps10[4];
    // a hardest-first solve in one launch: the finalize stores (status, iter) of list slot i at
    // info_slot[2 i], [2 i + 1], one 8-B store per QP into the wave's own 128-B line, instead of two
    // scattered 4-B stores at the QP's index (mpcq_api.cpp materialize_info permutes them when read); null:
    // at the QP's index in status, iter
    int *info_slot;
};

// MFMA operand images of one shared plant for the tile kernel (mpcq_tile.h).  A vector of length
// 4*KS is held in "D-layout": lane l = 16 g + c (column c = QP, group g) keeps element 4 s + g of
// its QP in register s.  Image (tile t, k-step s, lane l) = M[16 t + arow(l & 15)][4 s + (l >> 4)],
// stored [t][s / VEC][lane][s % VEC] so one lane reads VEC consecutive k-steps with one 16-B load.
// paired (the tile kernel's paired loop, m = 2n, rows n + j of A = -rows j): only the top halves are
// kept, B~ = B's first n rows and B~' = its transpose, A~' = the first n columns of A^' (KBT = KNP
// k-steps, NT tiles), plus for f64 (VEC 2) BS = [B~; S] stacked (B~ rows 0 .. 4 KN - 1, then S): the
// plain iteration's z~ = B~ eta' and S eta' in one product (ceil(8 KN / 16) tiles instead of 2 NT).
// The buffer holds the generic set (make(.., false)) followed by the paired one (make(.., true)).
struct TileLayout {
    int KN, KM, NT, MT, VEC, KNP, KMP, KBT, NBS;
    bool paired;
    size_t S, Bt, B, PW, AhT, W, Wt, BS, total;
    __host__ __device__ static constexpr TileLayout make(int KN, int KM, int VEC, bool paired = false)
    {
        TileLayout L{};
        L.KN = KN; L.KM = KM; L.VEC = VEC; L.paired = paired;
        L.NT = (KN + 3) / 4; L.MT = (KM + 3) / 4;
        L.KNP = (KN + VEC - 1) / VEC * VEC; L.KMP = (KM + VEC - 1) / VEC * VEC;
        L.KBT = paired ? L.KNP : L.KMP;
        L.NBS = (paired && VEC == 2) ? (8 * KN + 15) / 16 : 0;
        const int BT = paired ? L.NT : L.MT;  // tiles of B
        size_t o = 0;
        L.S = o;   o += (size_t)L.NT * L.KNP * 64;   // sigma W'W       (n x n)
        L.Bt = o;  o += (size_t)L.NT * L.KBT * 64;   // B' = (A^ W)'    (n x m; paired n x n)
        L.B = o;   o += (size_t)BT * L.KNP * 64;     // B = A^ W        (m x n; paired n x n)
        L.PW = o;  o += (size_t)L.NT * L.KNP * 64;   // P^ W            (n x n)
        L.AhT = o; o += (size_t)L.NT * L.KBT * 64;   // A^'             (n x m; paired n x n)
        L.W = o;   o += (size_t)L.NT * L.KNP * 64;   // W               (n x n)
        L.Wt = o;  o += (size_t)L.NT * L.KNP * 64;   // W'              (n x n)
        L.BS = o;  o += (size_t)L.NBS * L.KNP * 64;  // [B~; S]         (8 KN x n; paired f64 only)
        L.total = o;
        return L;
    }
    // elements of the device buffer: both sets
    __host__ __device__ static constexpr size_t buffer(int KN, int KM, int VEC)
    {
        return make(KN, KM, VEC, false).total + make(KN, KM, VEC, true).total;
    }
    __host__ __device__ static constexpr size_t at(int KSP, int VEC, int t, int s, int lane)
    {
        return ((size_t)(t * (KSP / VEC) + s / VEC) * 64 + lane) * VEC + (s % VEC);
    }
};
// A-operand row i of an output tile holds logical row arow(i): the f32 16x16x4 accumulator keeps
// rows 4g + r of a tile in lane group g, register r; the f64 one keeps rows g + 4r.
__host__ __device__ constexpr int tile_arow(int is_f32, int i) { return is_f32 ? 4 * (i & 3) + (i >> 2) : i; }

}  // namespace mpcq

namespace mpcq {
struct CondenseArgs {
    int n_plants, nx, N, s_rows;
    const double *Ad, *Bd, *Cd, *K, *Q, *R, *RD;  // [plant] nx*nx, nx, nx, nx, 1, 1, 1
    double *P, *A, *Fx, *Fu, *Fr, *Sbar, *Ku, *W0;  // [plant] N*N, 2N*N, N*nx, N, N*N, 2N*nx, 2N, 2N
    double *scratch;                                 // [plant] condense_scratch_len (N > 32 only)
    double *q0, *l0, *u0;                            // optional: the ctor's setup data (0, -DBL_MAX, W0)
    int force_ref;                                   // test hook: the workgroup kernel at any N
};
}  // namespace mpcq

namespace mpcq {
// ---- MIMO condensed MPC (BASELINE config 4; mpcq_mimo.hip) -------------------------------------
// Per-plant operator block (fp64, offsets in doubles) written by mimo_setup_kernel: the scaled Hessian
// P^ = c D P D (row-major n x n), the Ruiz scaling (D: n; E: n, the same for row j and row n + j of
// A = [L (x) K0; -(L (x) K0)]), c and 1/c, the unscaled front-end operators Fx (n x nx), Fu (n x nu),
// Frs = Fr (1_N (x) I_ny) (n x ny), the bound data K (nu x nx), K0 (nu x nu), w0 (nu), and
// SW (N blocks of nu x nu): suffix sums over k >= j of K0' diag(2 E_k^2) K0, so that the constraint
// Gram matrix A^'A^ has block (j1, j2) = D SW[max(j1, j2)] D.
struct MimoLayout {
    int N, nx, nu, ny, n, ldp;
    int Ph, D, E, cs, Fx, Fu, Frs, K, K0, w0, SW, total;  // < 2^31 for n <= 128
    __host__ __device__ static MimoLayout make(int N, int nx, int nu, int ny)
    {
        MimoLayout L{};
        L.N = N; L.nx = nx; L.nu = nu; L.ny = ny; L.n = N * nu;
        const int n = L.n;
        L.ldp = (n + 15) & ~15;  // P^ rows padded (zeros) to 16 columns: aligned, in-bounds 16-column loads
        int o = 0;
        L.Ph = o; o += n * L.ldp;
        L.D = o; o += n;
        L.E = o; o += n;
        L.cs = o; o += 2;
        L.Fx = o; o += n * nx;
        L.Fu = o; o += n * nu;
        L.Frs = o; o += n * ny;
        L.K = o; o += nu * nx;
        L.K0 = o; o += nu * nu;
        L.w0 = o; o += nu;
        L.SW = o; o += N * nu * nu;
        L.total = (o + 1) & ~1;  // 16-B aligned blocks
        return L;
    }
};

struct MimoSetupArgs {
    int n_plants, N, nx, nu, ny, s_rows, scaling;
    double sigma;
    const double *Ad, *Bd, *Cd, *Q, *R, *RD, *K, *K0, *w0;  // [plant] nx*nx, nx*nu, ny*nx, ny*ny, nu*nu x2, nu*nx, nu*nu, nu
    double *ops;                                            // [plant] MimoLayout::total
    int *flags;                                             // OR: 1 a diagonal of P^ + sigma I is not positive
                                                            //     (non-convex), 2 a row is not an inequality,
                                                            //     4 some K0 is not diagonal
    long long *stamps;                                      // debug (MPCQ_MIMO_SETUP_STAMPS): 16 per plant, or null
};

struct MimoArgs {
    int batch, N, nx, nu, ny, s_rows;
    size_t ops_stride;
    const double *ops;          // [plant] MimoLayout
    SolverSettings st;
    int adaptive_interval;
    const double *X, *yref;     // batch*nx (device), ny (device)
    double *U;                  // batch*nu (device): U += x[0:nu] when solved (:105)
    double *q_out, *u_out;      // batch*n, batch*2n: this step's q, u (unscaled)
    double *xs, *zs, *ys, *rhos;// scaled state (warm start): batch*n, batch*2n, batch*2n, batch
    int warm, fresh;
    int diag_k0;                // every plant's K0 is diagonal: the A^ products need no cross-component mix
    double *x, *y;              // unscaled solution: batch*n, batch*2n
    int *status, *iter;
    double *rho_out;
    long long *stamps;          // debug (MPCQ_MIMO_STAMPS) or null
};
}  // namespace mpcq

namespace mpcq {
// Arguments of plant_step_kernel (mpcq_plant.hip): condensing + setup + one controllerStep per SISO plant.
struct PlantStepArgs {
    int n_plants, nx, N, s_rows;
    const double *Ad, *Bd, *Cd, *K, *Q, *R, *RD;  // [plant] nx*nx, nx, nx, nx, 1, 1, 1
    const double *X;                               // [plant] nx (device)
    double *U;                                     // [plant]    (device): U += x0 when solved
    double xref;
    SolverSettings st;
    int adaptive_interval;
    double *x, *y, *rho_out;                       // [plant] n, 2n unscaled solution; final rho
    int *status, *iter;
    int *flags;                                    // OR: 1 a plant's KKT matrix is not positive definite
    int wpe;                                       // waves per SIMD of the kernel variant (2; 3: A/B hook)
    int layout;                                    // plants per wave (0: the default, 3 for 17 <= N <= 20;
                                                   // 2: one per 32-lane half, test hook MPCQ_PLANT_LAYOUT)
    // hardest-first (mpcq_order.hip): slot i of the grid runs plant order[i] (null: plant i); workgroup 0
    // zeroes the OrderBins::kBins counters ord_zero for the next sort
    const int *order;
    int *ord_zero;
    long long *stamps;  // debug builds (-DMPCQ_PLANT_STAMPS): 16 per wave, stage clock stamps
};
}  // namespace mpcq

// Launchers (extern "C" so the host library links them without templates).
extern "C" {
int mpcq_internal_setup_launch(const mpcq::SetupArgs *args, hipStream_t stream);
int mpcq_internal_setup_wave_launch(const mpcq::SetupArgs *args, hipStream_t stream);
// Per-plant setup with the direct inverse M(rho)^-1 (mpcq_setup_wave.hip; n <= 32, m <= 64).
int mpcq_internal_setup_inv_launch(const mpcq::SetupArgs *args, hipStream_t stream);
size_t mpcq_internal_setup_wave_lds(int n, int m);
int mpcq_internal_f64_to_f32(const double *in, float *out, size_t count, hipStream_t s);
int mpcq_internal_broadcast(const double *src, double *dst, int len, int batch, int per_qp_src, hipStream_t s);
int mpcq_internal_fill(void *p, int is_f32, double v, size_t count, hipStream_t s);
int mpcq_internal_caps(int n, int m, int *nc, int *mc);
int mpcq_internal_condense_launch(const mpcq::CondenseArgs *a, hipStream_t s);
size_t mpcq_internal_condense_scratch(int nx, int N);
int mpcq_internal_admm_launch_f64(const mpcq::AdmmArgs<double> *a, int nc, int mc, hipStream_t s);
int mpcq_internal_admm_launch_f32(const mpcq::AdmmArgs<float> *a, int nc, int mc, hipStream_t s);
int mpcq_internal_warm_f64(const mpcq::AdmmArgs<double> *a, int nc, int mc, const double *x, const double *y,
                           hipStream_t s);
int mpcq_internal_warm_f32(const mpcq::AdmmArgs<float> *a, int nc, int mc, const double *x, const double *y,
                           hipStream_t s);
// Tile (MFMA) path for a shared plant: 0 = launched, -1 = (KN, KM) not compiled, -2 = HIP error.
int mpcq_internal_tile_supported(int KN, int KM);
int mpcq_internal_tile_launch_f64(const mpcq::AdmmArgs<double> *a, int KN, int KM, hipStream_t s);
int mpcq_internal_tile_launch_f32(const mpcq::AdmmArgs<float> *a, int KN, int KM, hipStream_t s);
// The lazily published x, y of the last tile solve from its stored warm state (mpcq_tile.h tile_publish_kernel).
int mpcq_internal_tile_publish_f64(const mpcq::AdmmArgs<double> *a, int KN, int KM, int paired, hipStream_t s);
int mpcq_internal_tile_publish_f32(const mpcq::AdmmArgs<float> *a, int KN, int KM, int paired, hipStream_t s);
// The receding-horizon stream in one tile launch (AdmmArgs::sim; every column one plant through all its
// control steps).  0 launched, -1 not the paired condensed-MPC shape.
int mpcq_internal_tile_stream_launch_f64(const mpcq::AdmmArgs<double> *a, int KN, int KM, hipStream_t s);
int mpcq_internal_tile_stream_launch_f32(const mpcq::AdmmArgs<float> *a, int KN, int KM, hipStream_t s);
// One-QP-per-wave path (mpcq_wave.h): grid blocks of 64 threads stride over the (listed) QPs;
// -1 = n > 32 or m > 64 (not compiled).
int mpcq_internal_wave_launch_f64(const mpcq::AdmmArgs<double> *a, int nc, int mc, int grid, hipStream_t s);
int mpcq_internal_wave_launch_f32(const mpcq::AdmmArgs<float> *a, int nc, int mc, int grid, hipStream_t s);
// The receding-horizon stream in one launch (mpcq_wave.h stream_wave_kernel): every wave owns one QP
// for all `steps` control steps (solve, U += x0, plant update).  0 launched, -1 no compiled capacity.
int mpcq_internal_stream_launch_f32(const mpcq::AdmmArgs<float> *a, int nc, int mc, const mpcq::StreamArgs *sa,
                                    hipStream_t s);
int mpcq_internal_stream_launch_f64(const mpcq::AdmmArgs<double> *a, int nc, int mc, const mpcq::StreamArgs *sa,
                                    hipStream_t s);
// Plant update of the receding-horizon stream (mpcq_stream.hip); step from *step_p when non-null.
int mpcq_internal_simulate(int batch, int nx, int shared, const double *Ad, const double *Bd, double *X,
                           const double *U, unsigned long long seed, long long first_qp, const long long *step_p,
                           long long step_v, double noise_std, hipStream_t s);
int mpcq_internal_tick(long long *step, hipStream_t s);
int mpcq_internal_front_end(int batch, int nx, int n, int m, const double *Xs, const double *Us, double xref,
                            const double *Fx, const double *Fu, const double *Fr, const double *Sbar,
                            const double *Ku, const double *W0, double *q, double *u, hipStream_t s);
int mpcq_internal_set_step(long long *step, long long v, hipStream_t s);
// Hardest-first order of a shared-plant MPC step (mpcq_order.hip): per-QP bound-violation key from the
// host's OrderBins map, counting-sorted into list (cnt: OrderBins::kBins counters, zero on entry); Xs, Us
// (or null): copies of X, U for the step's q, u on demand.
int mpcq_internal_order(int batch, int nx, int m, const double *X, const double *U, const double *kmap, double xref,
                        int *cnt, int *key, int *list, double *Xs, double *Us, hipStream_t s);
// status[list[i]], iter[list[i]] = slot[2 i], slot[2 i + 1] (an ordered launch's AdmmArgs::info_slot)
int mpcq_internal_order_info(int batch, const int *list, const int *slot, int *status, int *iter, hipStream_t s);
// MIMO condensed MPC (mpcq_mimo.hip): per-plant condensing + Ruiz + P^, then the per-QP solve
// (one 512-thread workgroup per QP: KKT inverse by Gauss-Jordan in VGPRs, structured A).
int mpcq_internal_mimo_setup_launch(const mpcq::MimoSetupArgs *a, hipStream_t s);
int mpcq_internal_mimo_solve_launch(const mpcq::MimoArgs *a, hipStream_t s);
// One pass per batch of distinct SISO plants (mpcq_plant.hip): condensing + setup + one
// controllerStep per plant, two plants per wave.  0 launched, -1 unsupported shape, -2 HIP error.
int mpcq_internal_plant_step_launch(const mpcq::PlantStepArgs *a, int is_f32, hipStream_t s);
// Build the TileLayout images (type T = f32 if is_f32) of plant 0 from its fp64 operator block.
int mpcq_internal_tile_images(const double *ops, int nc, int mc, int KN, int KM, int is_f32, void *img,
                              hipStream_t s);
}
