/*
 * include/mpcq.h — C ABI of the MI355X (gfx950) batched condensed-MPC QP solver.
 *
 * This is the drop-in boundary for the one hot path of LukeSchmitt96/solveMPC: the QP solve that
 * ModelPredictiveControlAPI performs through osqp-eigen (OsqpEigen::Solver, a member at
 * include/ModelPredictiveControlAPI.h:144).  Every entry point names the reference call it
 * replaces.  Conventions:
 *   - plain pointers and sizes; every function returns an int status, 0 == MPCQ_OK;
 *   - host buffers are caller-owned and only read/written during the call; device buffers are
 *     owned by the context;
 *   - matrices are dense, row-major, fp64 (the reference's c_float == double), QP-major across a
 *     batch: element (b, i, j) of a batch of r x c matrices sits at b*r*c + i*c + j;
 *   - one context per host thread; calls on one context are not re-entrant;
 *   - `stream` is a hipStream_t passed as void* (NULL = the default stream).
 *
 * A context holds `batch` independent QPs of identical shape (n variables, m constraints).
 * They either share one plant (n_plants == 1: one P and A, e.g. 65,536 copies of the reference's
 * controller fed different states) or carry one plant each (n_plants == batch).
 */
#ifndef MPCQ_H
#define MPCQ_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes -------------------------------------------------------------------------- */
#define MPCQ_OK 0
#define MPCQ_ERR_ARG (-1)      /* bad argument / unsupported size                              */
#define MPCQ_ERR_HIP (-2)      /* HIP runtime error or no usable gfx950 device                 */
#define MPCQ_ERR_SETUP (-3)    /* setup rejected the data (P not PSD / KKT not quasi-definite) */
#define MPCQ_ERR_ORDER (-4)    /* call order (e.g. solve before setup)                         */
#define MPCQ_ERR_BOUNDS (-5)   /* some u < l (osqp_update_*_bound failure)                     */

/* ---- per-QP status (OSQP v0.6 values; osqp-eigen's solve() is true only for SOLVED) ------- */
#define MPCQ_SOLVED 1
#define MPCQ_SOLVED_INACCURATE 2
#define MPCQ_PRIMAL_INFEASIBLE_INACCURATE 3
#define MPCQ_DUAL_INFEASIBLE_INACCURATE 4
#define MPCQ_MAX_ITER_REACHED (-2)
#define MPCQ_PRIMAL_INFEASIBLE (-3)
#define MPCQ_DUAL_INFEASIBLE (-4)
#define MPCQ_NON_CVX (-7)
#define MPCQ_UNSOLVED (-10)
#define MPCQ_INVALID_BOUNDS (-20) /* this QP's u < l: update rejected, not solved              */
#define MPCQ_TYPE_CHANGED (-21)   /* this QP's bounds changed a row's OSQP constraint type
                                     (equality/inequality/free) away from its plant's setup;
                                     re-run mpcq_setup with these bounds                     */

/* ---- precision of the device iterate ------------------------------------------------------- */
#define MPCQ_F64 0 /* fp64 throughout (the reference's precision)                            */
#define MPCQ_F32 1 /* fp32 ADMM iterate, fp64 setup.  Bound: where OSQP certifies primal
                      infeasibility an fp32 iterate may not (the dual iterate of an infeasible QP
                      grows without bound and its fp32 rounding moves the certificate's
                      ||A' dy|| / ||dy|| past eps_prim_inf), and the QP then runs to max_iter:
                      MPCQ_MAX_ITER_REACHED, or MPCQ_SOLVED_INACCURATE where OSQP's approximate
                      check passes there, instead of MPCQ_PRIMAL_INFEASIBLE (never MPCQ_SOLVED;
                      osqp-eigen's solve() is false either way).  MPCQ_F64 and MPCQ_F64_MIXED
                      return OSQP's status (tests/test_gpu.py test_infeasible_statuses_match_oracle) */
#define MPCQ_F64_MIXED 2 /* fp64 state, checks and solution; on the shared-plant tile path the plain
                            iterations before the last MPCQ_MIX_R of every check interval run in fp32
                            (MFMA f32 products), which the fp64 ones damp; every
                            other path is MPCQ_F64                                               */
#define MPCQ_MIX_R 5

/* OSQP v0.6 settings (osqp constants.h defaults via mpcq_default_settings).  Replaces
 * OsqpEigen::Settings as used at ModelPredictiveControlAPI.cpp:51-52 (setVerbosity,
 * setWarmStart(true)); polish is not supported (the reference leaves it off). */
typedef struct mpcq_settings {
    double rho, sigma, alpha;
    double eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
    double adaptive_rho_tolerance, adaptive_rho_fraction;
    int max_iter, check_termination, scaling, adaptive_rho, adaptive_rho_interval;
    int warm_start, scaled_termination, verbose;
} mpcq_settings;

typedef struct mpcq_dims {
    int n;        /* decision variables  (setNumberOfVariables, :54)   */
    int m;        /* constraint rows     (setNumberOfConstraints, :55) */
    int batch;    /* QPs in this context (reference: 1)                */
    int n_plants; /* 1 (shared P, A) or batch (one plant per QP)       */
    int dtype;    /* MPCQ_F64, MPCQ_F32 or MPCQ_F64_MIXED              */
    int device;   /* HIP device ordinal                                */
} mpcq_dims;

typedef struct mpcq_ctx mpcq_ctx;

/* Device-resident views of a context's buffers (fp64, QP-major), for zero-copy callers.
 * The pointers never change, but the OUTPUTS (x, y, status, iter, rho) are published lazily on the
 * shared-plant tile path: a solve leaves them in its warm state and they are formed
 * from it when something reads them.  mpcq_device_view_get is such a read: the output arrays hold the
 * last solve's values only after mpcq_device_view_get has been called AFTER that solve (call it again
 * after every mpcq_solve / mpcq_mpc_step_device / graph replay), and they are written by kernels
 * enqueued on the context's last stream (the stream of its last solve), so a reader on another stream
 * must order itself after that stream (an event) or synchronise it.  A view fetched once and re-read
 * after later solves shows an older solve's outputs.  The inputs (q, u, l) follow the same rule. */
typedef struct mpcq_device_view {
    double *q;     /* batch*n   gradient (input of the next solve)      */
    double *u;     /* batch*m   upper bounds                            */
    double *l;     /* batch*m   lower bounds                            */
    double *x;     /* batch*n   unscaled primal solution (output)       */
    double *y;     /* batch*m   unscaled dual solution (output)         */
    int *status;   /* batch     MPCQ_* status (output)                  */
    int *iter;     /* batch     ADMM iterations (output)                */
    double *rho;   /* batch     rho after the solve (output)            */
} mpcq_device_view;

void mpcq_default_settings(mpcq_settings *s);

/* Allocate a context on dims->device.  Fails with MPCQ_ERR_HIP when no gfx950 device exists. */
int mpcq_create(const mpcq_dims *dims, const mpcq_settings *settings, mpcq_ctx **out);
int mpcq_destroy(mpcq_ctx *ctx);

/* Setup: replaces setHessianMatrix / setGradient / setLinearConstraintsMatrix / setLowerBound /
 * setUpperBound + initSolver (ModelPredictiveControlAPI.cpp:57-64 -> osqp_setup).  Arrays are per
 * plant (n_plants copies): P n*n (upper triangle read, as osqp-eigen does), q0 n, A m*n, l0/u0 m.
 * Ruiz equilibration, cost scaling and the KKT factorisation run on the device.  q0/l0/u0 also
 * become the current q/l/u of every QP of the plant. */
int mpcq_setup(mpcq_ctx *ctx, const double *P, const double *q0, const double *A,
               const double *l0, const double *u0);

/* Per-QP data updates from host memory (batch*n or batch*m).
 * Replace OsqpEigen::Solver::updateGradient (:96 -> osqp_update_lin_cost) and
 * updateUpperBound (:99 -> osqp_update_upper_bound); lower/both-bound forms for completeness.
 * Bounds are validated per QP when the solve runs (status MPCQ_INVALID_BOUNDS). */
int mpcq_update_lin_cost(mpcq_ctx *ctx, const double *q);
int mpcq_update_upper_bound(mpcq_ctx *ctx, const double *u);
int mpcq_update_lower_bound(mpcq_ctx *ctx, const double *l);
int mpcq_update_bounds(mpcq_ctx *ctx, const double *l, const double *u);

/* osqp_warm_start / cold_start for every QP (x batch*n, y batch*m, unscaled). */
int mpcq_warm_start(mpcq_ctx *ctx, const double *x, const double *y);
int mpcq_cold_start(mpcq_ctx *ctx);

/* Return every QP to the state right after setup (x = z = y = 0, rho = settings.rho), as
 * re-running initSolver (:64) would; applied by the next solve at no cost. */
int mpcq_reset(mpcq_ctx *ctx);

/* Solve every QP (replaces OsqpEigen::Solver::solve, :102 -> osqp_solve).  Asynchronous on
 * `stream`; iterates stay on the device (warm start, :52). */
int mpcq_solve(mpcq_ctx *ctx, void *stream);

/* Results (synchronise the context's last stream).  Replace getSolution() (:105). */
int mpcq_get_solution(mpcq_ctx *ctx, double *x);            /* batch*n */
int mpcq_get_dual(mpcq_ctx *ctx, double *y);                /* batch*m */
int mpcq_get_info(mpcq_ctx *ctx, int *status, int *iter, double *rho); /* each batch, may be NULL */
int mpcq_get_scaling(mpcq_ctx *ctx, double *D, double *E, double *c); /* plant 0: n, m, 1 */

/* Device path the next solve takes (no OSQP counterpart; for benchmarks and tests):
 * *kind = MPCQ_PATH_TILE (shared plant, MFMA tile kernel's phase chain), MPCQ_PATH_WAVE
 * (one QP per wave: per-plant contexts, and shared-plant batches under 8,192 QPs) or MPCQ_PATH_LANE
 * (one QP per lane); *paired = 1 when the tile kernel runs its paired loop (rows n + j of A are the
 * negated rows j: the condensed-MPC constraint matrix). */
#define MPCQ_PATH_TILE 0
#define MPCQ_PATH_WAVE 1
#define MPCQ_PATH_LANE 2
int mpcq_get_path(mpcq_ctx *ctx, int *kind, int *paired);

/* Fill *view and publish the last solve's pending outputs into it (see mpcq_device_view above). */
int mpcq_device_view_get(mpcq_ctx *ctx, mpcq_device_view *view);

/* ---- condensed-MPC front end: ModelPredictiveControlAPI::controllerStep, batched ------------
 * Per-plant operators of the condensed problem (n == N, m == 2N; ModelPredictiveControlAPI.cpp
 * setFVars :303-307, setUpperBound :360-369, setTransformations :185,208): Fx N*nx, Fu N,
 * Fr N*N, Sbar m*nx, Ku m, W0 m (n_plants copies each). */
int mpcq_mpc_set_operators(mpcq_ctx *ctx, int nx, const double *Fx, const double *Fu,
                           const double *Fr, const double *Sbar, const double *Ku,
                           const double *W0);
/* One receding-horizon step for every QP, on device-resident X (batch*nx) and U (batch):
 *   q = Fx X + Fu U + Fr (xref 1)          (setF :372-375, updateRef :378-380)
 *   u = W0 + Sbar X + Ku U                 (:93-99)
 *   solve                                  (:102, warm-started)
 *   U += x[0] where status == SOLVED       (:105)
 * X_dev/U_dev are device pointers (fp64). */
int mpcq_mpc_step_device(mpcq_ctx *ctx, const double *X_dev, double *U_dev, double xref,
                         void *stream);

/* Host-memory convenience form of mpcq_mpc_step_device (copies in/out, synchronises). */
int mpcq_mpc_step(mpcq_ctx *ctx, const double *X, double *U, double xref);

/* ---- receding-horizon stream (BASELINE config 5; the solver.cpp loop, solver.cpp:43-74, with the
 * serial plant replaced by a simulated one) ----------------------------------------------------
 * Plant of every QP: X <- Ad X + Bd U + w,  w ~ N(0, noise_std^2 I) drawn from a counter-based
 * generator keyed by (seed, global QP index first_qp + b, step, component) — the same stream on any
 * sharding of the batch (solvempc_amd/workload.py restates it).  Ad nx*nx, Bd nx per plant. */
int mpcq_mpc_set_plant(mpcq_ctx *ctx, int nx, const double *Ad, const double *Bd);
/* One plant update on device-resident X (batch*nx) / U (batch); `step` selects the noise draw. */
int mpcq_mpc_simulate_device(mpcq_ctx *ctx, double *X_dev, const double *U_dev, unsigned long long seed,
                             long long first_qp, long long step, double noise_std, void *stream);
/* `steps` warm-started control steps  [controllerStep (:81-108) ; plant update]  for every QP
 * (steps first_step .. first_step+steps-1); X_dev/U_dev evolve in place.  One launch runs every
 * step: the tile kernel's stream mode for a shared plant of the condensed-MPC shape (each MFMA
 * column one plant), else one QP per wave; other shapes replay a hipGraph of per-step launches.
 * `stream` must not be the NULL stream (graph capture). */
int mpcq_mpc_run_device(mpcq_ctx *ctx, double *X_dev, double *U_dev, double xref, int steps,
                        unsigned long long seed, long long first_qp, long long first_step,
                        double noise_std, void *stream);
/* How the last mpcq_mpc_run_device call ran (benchmarks and tests): MPCQ_STREAM_TILE (one tile-kernel
 * launch), MPCQ_STREAM_WAVE (one one-QP-per-wave launch) or MPCQ_STREAM_GRAPH (per-step launches). */
#define MPCQ_STREAM_GRAPH 0
#define MPCQ_STREAM_WAVE 1
#define MPCQ_STREAM_TILE 2
int mpcq_get_stream_path(mpcq_ctx *ctx, int *kind);
/* Hardest-first order of the last solve (benchmarks and tests): *ordered = 1 when it
 * was a tile-path MPC step or a one-pass distinct-plants step (mpcq_mpc_plants_step_device; the key from the
 * batch's first plant) run in ascending |max_j (A x_u - u)_j| (x_u = -P^-1 q, the QP's unconstrained
 * optimum; binned 16 per octave), else 0; order (batch ints, or NULL) receives that step's QPs in the
 * order it ran them (synchronises).  The order changes no result. */
int mpcq_get_order(mpcq_ctx *ctx, int *ordered, int *order);
/* Per-QP counters of the last mpcq_mpc_run_device call (host arrays of `batch` ints, synchronises):
 * the ADMM iterations of all its control steps, and the steps whose solve did not end SOLVED
 * (controllerStep returning false, :102, where the reference's loop would exit, solver.cpp:50). */
int mpcq_mpc_stream_counters(mpcq_ctx *ctx, int *iters, int *unsolved);

/* Condensed-QP construction on device `device` for n_plants SISO plants (ModelPredictiveControlAPI
 * setTransformations / setLL / setLiftedCosts / setH / setFVars / setLinearConstraints /
 * setUpperBound, src/ModelPredictiveControlAPI.cpp:158-369).  Inputs per plant: Ad nx*nx, Bd nx,
 * Cd nx, K nx, Q, R, RD (scalars); N = horizon; s_rows = rows of S filled with K (reference: 10,
 * :185).  Outputs per plant (host memory, caller-allocated): P N*N, A 2N*N, Fx N*nx, Fu N, Fr N*N,
 * Sbar 2N*nx, Ku 2N, W0 2N.  nx <= 8. */
int mpcq_condense(int device, int n_plants, int nx, int N, int s_rows, const double *Ad,
                  const double *Bd, const double *Cd, const double *K, const double *Q,
                  const double *R, const double *RD, double *P, double *A, double *Fx, double *Fu,
                  double *Fr, double *Sbar, double *Ku, double *W0);

/* Per-plant condensing + setup on the device (BASELINE config 3): every plant of the context
 * (n_plants copies, device pointers, plant-major: Ad nx*nx, Bd nx, Cd nx, K nx, Q, R, RD) is
 * condensed as mpcq_condense does, its front-end operators installed (as mpcq_mpc_set_operators)
 * and the solver set up on the ctor's data (as mpcq_setup with q0 = 0, l0 = -DBL_MAX, u0 = W0:
 * ModelPredictiveControlAPI.cpp:22-23,38-43,51-64), all on `stream`; the only host transfer is
 * the setup's status word.  Needs n == N, m == 2N. */
int mpcq_mpc_setup_plants_device(mpcq_ctx *ctx, int nx, int s_rows, const double *Ad,
                                 const double *Bd, const double *Cd, const double *K,
                                 const double *Q, const double *R, const double *RD, void *stream);

/* Per-plant batch in one pass (BASELINE config 3): for every plant the reference's constructor
 * (condensing + osqp_setup on the ctor's data, X = U = 0: :3-65) and one controllerStep (:81-108) from
 * device-resident X (batch*nx) and U (batch; U += x[0] when SOLVED) — the work of
 * mpcq_mpc_setup_plants_device followed by mpcq_mpc_step_device, with each plant's operators kept on
 * chip instead of written to the context.  Plant arrays as in mpcq_mpc_setup_plants_device.
 * Afterwards the context holds this step's solution, dual, status, iterations and rho; it holds no
 * operators, so further solves need mpcq_mpc_setup_plants_device / mpcq_setup first (MPCQ_ERR_ORDER
 * otherwise).  Asynchronous on `stream`; a plant whose KKT matrix is not positive definite ends
 * MPCQ_NON_CVX.  Needs n == N <= 32, m == 2N, n_plants == batch, nx <= 8. */
int mpcq_mpc_plants_step_device(mpcq_ctx *ctx, int nx, int s_rows, const double *Ad, const double *Bd,
                                const double *Cd, const double *K, const double *Q, const double *R,
                                const double *RD, const double *X, double *U, double xref, void *stream);

/* ---- MIMO condensed MPC (BASELINE config 4: quad-rotor hover linearisations, n_x 12, n_u 4, N 30) --
 * The reference's condensing (ModelPredictiveControlAPI.cpp:158-369) with every SISO scalar a block
 * (oracle/mpc_mimo.h): decision du in R^(N n_u), A = [L (x) K0; -(L (x) K0)], u = W0 + Sbar X + Ku U,
 * l = -DBL_MAX.  The context must have n_plants == batch, n = N n_u (<= 128), m = 2n, dtype MPCQ_F64;
 * n_u in {1, 2, 4}, n_x, n_y <= 12, N <= 32.
 * Setup (replaces the ctor :3-65 + initSolver :64 per plant) from device-resident plant data,
 * plant-major fp64: Ad nx*nx, Bd nx*nu, Cd ny*nx, Q ny*ny (symmetric), R nu*nu, RD nu*nu, K nu*nx,
 * K0 nu*nu, w0 nu; S = K on block rows k < s_rows.  Condensing, Ruiz scaling and P^ on the device;
 * the solver state is reset (x = z = y = 0, rho = settings.rho). */
int mpcq_mimo_setup_plants_device(mpcq_ctx *ctx, int nx, int nu, int ny, int s_rows, const double *Ad,
                                  const double *Bd, const double *Cd, const double *Q, const double *R,
                                  const double *RD, const double *K, const double *K0, const double *w0,
                                  void *stream);
/* One controllerStep (:81-108) for every QP on device-resident X (batch*nx) and U (batch*nu):
 * q = Fx X + Fu U + Fr (1_N (x) yref), u = W0 + Sbar X + Ku U, solve (warm-started after the first
 * step), U += x[0:n_u] where SOLVED.  yref: device pointer to n_y values, or NULL for 0. */
int mpcq_mimo_step_device(mpcq_ctx *ctx, const double *X_dev, double *U_dev, const double *yref_dev,
                          void *stream);

/* Last HIP error string of this thread (static storage). */
const char *mpcq_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* MPCQ_H */
