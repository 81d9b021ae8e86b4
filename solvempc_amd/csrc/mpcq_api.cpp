// solvempc_amd/csrc/mpcq_api.cpp — host side of the C ABI declared in include/mpcq.h.
//
// Orchestration only: argument checks, device buffers, kernel launches.  All arithmetic on the
// QPs (setup, ADMM, MPC front end) runs in the HIP kernels of mpcq_setup.hip / mpcq_admm.hip.
// There is no CPU solve path: without a gfx950 device mpcq_create fails with MPCQ_ERR_HIP.
#include "../../include/mpcq.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "mpcq_internal.h"


namespace {
thread_local std::string g_err;

int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                  \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess) return fail(MPCQ_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

constexpr int kMaxPhases = 16;

// Test hooks: the library reads exactly these environment variables, here and nowhere else.  Each
// selects among production code paths so that the tests can cover every path on one device:
//   MPCQ_KERNEL=lane|wave|tile  the ADMM kernel family (mpcq_get_path reports the choice)
//   MPCQ_PHASES=0|k1,k2,..      the tile path's phase stops, in check_termination multiples
//   MPCQ_SETUP=ref              per-plant setup on the workgroup kernel (mpcq_setup.hip)
//   MPCQ_CONDENSE=ref           condensing on the workgroup kernel (mpcq_condense.hip)
//   MPCQ_MIMO_GENERAL_K0=1      the MIMO solve's general-K0 exchange path on a diagonal K0
//   MPCQ_STREAM=graph|wave      mpcq_mpc_run_device's per-step graph or one-QP-per-wave launch
//                               (mpcq_get_stream_path reports the choice)
//   MPCQ_STREAM_CPW=k           plants per wave of the tile stream mode
//   MPCQ_STREAM_OCC=1           the tile stream mode's one-wave-per-SIMD variant (when the waves fit)
//   MPCQ_TAIL=wave|tile         the tile chain's last launch on the one-QP-per-wave / tile kernel
//   MPCQ_MIX_R=r                MPCQ_F64_MIXED: fp64 iterations per check interval (default MPCQ_MIX_R)
//   MPCQ_TILE_OCC=2|3           waves per SIMD of the f32 paired tile kernel (default 3)
//   MPCQ_PLANT_WPE=2|3|4        waves per SIMD of the one-pass per-plant kernel (default f64 3, f32 2)
//   MPCQ_PLANT_LAYOUT=2         the one-pass per-plant kernel with two plants per wave at N 17 .. 20 (default 3)
//   MPCQ_ORDER=0                a shared-plant MPC step's tile solve in index order (default: hardest first)
//   MPCQ_LAZY_XY=0              the tile solve stores x, y at finalize (default: published on demand)
//   MPCQ_LAZY_INFO=0            an ordered one-launch solve stores status, iter at the QPs' indices
//                               (default: in list-slot order, permuted on demand)
// Debug builds (-DMPCQ_DEBUG_HOOKS) add the stamp / profiling dumps (MPCQ_TILE_STAMPS,
// MPCQ_SETUP_PROF, MPCQ_MIMO_SETUP_STAMPS, MPCQ_MIMO_STAMPS) and MPCQ_DEBUG_SYNC.
const char *test_hook(const char *name)
{
    const char *v = std::getenv(name);
    return v ? v : "";
}
const char *debug_hook(const char *name)
{
#ifdef MPCQ_DEBUG_HOOKS
    const char *v = std::getenv(name);
    return v ? v : "";
#else
    (void)name;
    return "";
#endif
}

size_t setup_scratch_len(int n, int m)
{
    return 7 * (size_t)n * n + (size_t)m * n + 3 * (size_t)n + 2 * (size_t)m + 64;
}
}  // namespace

struct mpcq_ctx {
    mpcq_dims dims{};
    mpcq_settings set{};
    int nc = 0, mc = 0;
    size_t ops_stride = 0;
    // The formulation the context was last set up for: the generic / condensed-MPC operators
    // (mpcq_setup, mpcq_mpc_setup_plants_device) or the MIMO operator blocks
    // (mpcq_mimo_setup_plants_device).  Each entry point checks for the one it runs on.
    // OneShot: mpcq_mpc_plants_step_device left this step's results but no operators behind.
    enum class Mode { None, Generic, Mimo, OneShot } mode = Mode::None;
    bool all_ineq = true, mpc_ready = false, lower_free = false, fresh = false;
    double dinf_ks = 0.0, dinf_ku = 0.0;  // dual-infeasibility bounds (AdmmArgs::dinf_kappa), 0: none
    int cus = 256;                        // compute units of the device (phase lists)
    // A tile-path controllerStep leaves q, u (the solver's data after updateGradient / updateUpperBound)
    // as the step's saved X, U: d_q, d_u are filled from them by materialize_qu before anything reads
    // them (a generic solve, the device view, an update, new operators).
    double *d_Xs = nullptr, *d_Us = nullptr;
    bool qu_lazy = false;
    double lazy_xref = 0.0;
    bool paired = false;  // shared plant of the condensed-MPC shape (tile kernel's paired loop)
    bool inv_ops = false; // per-plant operators in the direct-inverse reading (setup_inv_kernel): wave kernel only
    // tile (MFMA) path: shared plant with a compiled (KN, KM) shape
    bool tile = false;
    int KN = 0, KM = 0;
    void *d_img = nullptr;
    int *d_list = nullptr, *d_counts = nullptr, *d_itstate = nullptr;
    bool count0_clean = false;    // phase 0's ListSeg counters are zero (the last phase chain's final launch zeroed them)
    long long *d_stamps = nullptr;  // debug (MPCQ_TILE_STAMPS)
    hipStream_t last = nullptr;
    int nx = 0;
    // setup
    double *d_P = nullptr, *d_q0 = nullptr, *d_A = nullptr, *d_l0 = nullptr, *d_u0 = nullptr;
    double *d_ops = nullptr, *d_scratch = nullptr;
    int *d_flags = nullptr;
    float *d_ops32 = nullptr;
    int *d_ctype = nullptr, *d_setup_status = nullptr;
    // per QP
    double *d_q = nullptr, *d_u = nullptr, *d_l = nullptr, *d_x = nullptr, *d_y = nullptr, *d_rho = nullptr;
    int *d_status = nullptr, *d_iter = nullptr;
    void *d_xs = nullptr, *d_zs = nullptr, *d_ys = nullptr, *d_rhos = nullptr, *d_snx = nullptr, *d_sny = nullptr;
    // MPC front end
    double *d_Fx = nullptr, *d_Fu = nullptr, *d_Fr = nullptr, *d_Sbar = nullptr, *d_Ku = nullptr, *d_W0 = nullptr;
    double *d_X = nullptr, *d_U = nullptr;
    // receding-horizon stream: plant, step counter, captured graph of one control step
    double *d_Ad = nullptr, *d_Bd = nullptr;
    long long *d_step = nullptr;
    int plant_nx = 0;
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    // gen: bumped whenever buffers baked into the captured graph are reallocated or the kernel
    // variant flags (all_ineq, lower_free) may change; a replay needs the generation it captured
    unsigned long long gen = 1;
    struct { double *X, *U; double xref, noise; unsigned long long seed; long long first_qp; hipStream_t s;
             unsigned long long gen; } gkey{};
    // what the captured step leaves lazy (x, y; rho; status, iter; q, u) and its order flag: every replay
    // leaves the same, whatever a reader materialised in between
    struct { bool xy, rho, info, qu, ord; double xref; } glazy{};
    // MIMO condensed MPC (mpcq_mimo.hip): per-plant operator block, dims
    double *d_mimo = nullptr;
    int mimo_N = 0, mimo_nx = 0, mimo_nu = 0, mimo_ny = 0, mimo_srows = 0, mimo_diag_k0 = 0;
    bool mimo_only = false;  // n > 32 or m > 64 per plant: only the MIMO entry points serve it
    // receding-horizon stream counters (mpcq_mpc_run_device): per-QP iterations and unsolved steps
    int *d_it_acc = nullptr, *d_uns_acc = nullptr;
    bool stream_acc = false;  // launches made inside mpcq_mpc_run_device accumulate into them
    int stream_path = MPCQ_STREAM_GRAPH;  // how the last mpcq_mpc_run_device call ran
    // hardest-first order of a tile-path MPC step (mpcq_order.hip, build_order_map): the m x kStride
    // violation map of plant 0, the bin counters and lists; ord_ok when the map matches the current setup
    // and operators
    double *d_ordmap = nullptr;
    // OrderBins::kBins counters, then `batch` keys, the list of `batch` QPs, and `batch` (status, iter) pairs in
    // list-slot order (AdmmArgs::info_slot)
    int *d_ord = nullptr;
    bool ord_ok = false;
    // the same order for a batch of distinct plants (mpcq_mpc_plants_step_device): the map of the batch's first
    // plant, kept while the plant arrays are the same (pord_key); pord_ok when d_ordmap holds it
    bool pord_ok = false;
    struct { const double *Ad, *Bd, *Cd, *K, *Q, *R, *RD; int nx, s_rows; } pord_key{};
    bool ord_last = false;  // the last solve ran in that order (mpcq_get_order)
    bool ord_clean = false;  // its bin counters are zero (an ordered phase-0 launch clears them)
    // a tile solve whose finalize stored only the warm state (x', z, y) and U: d_x, d_y are formed from it by
    // materialize_xy before anything reads them (get_solution / get_dual, the device view, verbose, or a
    // call that overwrites the warm state)
    bool xy_lazy = false;
    // the same solve's rho (fp64 contexts): its warm-state rho d_rhos is the reported one; d_rho is copied
    // from it by materialize_rho before anything reads d_rho (get_info, the device view, verbose) or a
    // reset overwrites d_rhos
    bool rho_lazy = false;
    // an ordered single-launch solve left status, iter in list-slot order: materialize_info permutes them
    // into d_status, d_iter before anything reads those (get_info, the device view, verbose, the publish
    // kernel of materialize_xy)
    bool info_lazy = false;
    // host copies of plant-0 scaling
    std::vector<double> hD, hE;
    double hc = 1.0;
};

static int materialize_xy(mpcq_ctx *c);  // (below: the lazy x, y of a tile solve)
static int materialize_rho(mpcq_ctx *c);  // (and its rho)
static int materialize_info(mpcq_ctx *c);  // (and its status, iter)

namespace {

template <typename T>
void fill_ops(mpcq::PlantOps<T> &op, const T *base, const mpcq::OpsLayout &L, const int *ctype)
{
    op.lam = base + L.lam;
    op.W = base + L.W;
    op.sWtW = base + L.sWtW;
    op.WtA = base + L.WtA;
    op.PW = base + L.PW;
    op.Winv = base + L.Winv;
    op.Ah = base + L.Ah;
    op.D = base + L.D;
    op.E = base + L.E;
    op.Dinv = base + L.Dinv;
    op.Einv = base + L.Einv;
    op.cs = base + L.cs;
    op.rscale = base + L.rscale;
    op.ctype = ctype;
}

mpcq::SolverSettings to_solver(const mpcq_settings &s)
{
    mpcq::SolverSettings o{};
    o.rho = s.rho;
    o.sigma = s.sigma;
    o.alpha = s.alpha;
    o.eps_abs = s.eps_abs;
    o.eps_rel = s.eps_rel;
    o.eps_prim_inf = s.eps_prim_inf;
    o.eps_dual_inf = s.eps_dual_inf;
    o.adaptive_rho_tolerance = s.adaptive_rho_tolerance;
    o.max_iter = s.max_iter;
    o.check_termination = s.check_termination;
    o.adaptive_rho = s.adaptive_rho;
    o.adaptive_rho_interval = s.adaptive_rho_interval;
    o.warm_start = s.warm_start;
    o.scaled_termination = s.scaled_termination;
    o.scaling = s.scaling;
    return o;
}

template <typename T>
mpcq::AdmmArgs<T> make_args(mpcq_ctx *c)
{
    mpcq::AdmmArgs<T> a{};
    const mpcq::OpsLayout L = mpcq::OpsLayout::make(c->nc, c->mc);
    const T *base = std::is_same<T, double>::value ? (const T *)c->d_ops : (const T *)c->d_ops32;
    fill_ops(a.ops, base, L, c->d_ctype);
    a.batch = c->dims.batch;
    a.n = c->dims.n;
    a.m = c->dims.m;
    a.shared = c->dims.n_plants == 1;
    a.ops_stride = c->ops_stride;
    a.ctype = c->d_ctype;
    a.st = to_solver(c->set);
    a.eps10[0] = (T)a.st.eps_abs * T(10);
    a.eps10[1] = (T)a.st.eps_rel * T(10);
    a.eps10[2] = (T)a.st.eps_prim_inf * T(10);
    a.eps10[3] = (T)a.st.eps_dual_inf * T(10);
    const int ct = c->set.check_termination;
    a.adaptive_interval = c->set.adaptive_rho_interval ? c->set.adaptive_rho_interval : (ct ? 4 * ct : 100);
    a.all_ineq = c->all_ineq;
    a.dinf_kappa = c->set.scaled_termination ? c->dinf_ks : c->dinf_ku;
    a.lower_free = c->lower_free;
    a.q = c->d_q;
    a.u = c->d_u;
    a.l = c->d_l;
    a.l_shared = 0;
    a.xs = (T *)c->d_xs;
    a.zs = (T *)c->d_zs;
    a.ys = (T *)c->d_ys;
    a.rhos = (T *)c->d_rhos;
    a.warm = c->set.warm_start;
    a.fresh = c->fresh;
    a.snap_x = (T *)c->d_snx;
    a.snap_y = (T *)c->d_sny;
    a.x = c->d_x;
    a.y = c->d_y;
    a.rho_out = c->d_rho;
    a.status = c->d_status;
    a.iter = c->d_iter;
    a.it_acc = c->stream_acc ? c->d_it_acc : nullptr;
    a.uns_acc = c->stream_acc ? c->d_uns_acc : nullptr;
    {
        const char *o = test_hook("MPCQ_TILE_OCC");  // f32 paired tile kernel: 2 or 3 waves/SIMD (A/B)
        a.tile_occ = *o ? std::atoi(o) : 0;
    }
    if (c->dims.dtype == MPCQ_F64_MIXED) {  // (test hook MPCQ_MIX_R: another fp64 share for A/B)
        const char *r = test_hook("MPCQ_MIX_R");
        a.mix_r = *r ? std::max(1, std::atoi(r)) : MPCQ_MIX_R;
    }
    return a;
}

int reset_state(mpcq_ctx *c, bool reset_rho)
{
    if (int rc = materialize_xy(c)) return rc;  // (the warm state it zeroes is the last solve's x, y)
    if (int rc = materialize_rho(c)) return rc;
    const size_t B = c->dims.batch, es = c->dims.dtype == MPCQ_F32 ? 4 : 8;
    HIPCHK(hipMemsetAsync(c->d_xs, 0, es * c->nc * B, c->last));
    HIPCHK(hipMemsetAsync(c->d_zs, 0, es * c->mc * B, c->last));
    HIPCHK(hipMemsetAsync(c->d_ys, 0, es * c->mc * B, c->last));
    if (reset_rho) {
        const double r = std::min(std::max(c->set.rho, mpcq::kRhoMin), mpcq::kRhoMax);
        if (mpcq_internal_fill(c->d_rhos, c->dims.dtype == MPCQ_F32, r, B, c->last) != 0)
            return fail(MPCQ_ERR_HIP, "fill kernel failed");
    }
    return MPCQ_OK;
}

// True when every scaled lower bound is below -OSQP_INFTY*MIN_SCALING (the reference's
// l = -DBL_MAX, :42), which selects the kernel variant without the lower clamp.  Exact for a
// shared plant (its E is on the host); conservative (|l| >= 1e300) for per-plant contexts.
bool lower_all_free(const mpcq_ctx *c, const double *l)
{
    const size_t B = (l == nullptr) ? 0 : (size_t)c->dims.m;
    const size_t rows = c->dims.n_plants == 1 ? B : 0;
    if (c->dims.n_plants == 1) {
        for (size_t j = 0; j < rows; j++)
            if (!(l[j] * c->hE[j] < -mpcq::kInfty * mpcq::kMinScaling)) return false;
        return true;
    }
    return false;
}

bool lower_all_free_batch(const mpcq_ctx *c, const double *l)
{
    const size_t total = (size_t)c->dims.batch * c->dims.m;
    for (size_t i = 0; i < total; i++) {
        const double e = c->dims.n_plants == 1 ? c->hE[i % c->dims.m] : 1e-250;
        if (!(l[i] * e < -mpcq::kInfty * mpcq::kMinScaling) && !(l[i] <= -1e300)) return false;
    }
    return true;
}

enum Need { kNone, kGeneric, kAnySetup };

// kGeneric: the generic / condensed-MPC operators (the generic kernels run on them); kAnySetup:
// either formulation (result readers).  A MIMO-only context never passes kGeneric.
int check_ctx(mpcq_ctx *c, Need need)
{
    if (!c) return fail(MPCQ_ERR_ARG, "null context");
    if (need == kGeneric && c->mimo_only)
        return fail(MPCQ_ERR_ARG, "n > 32 or m > 64 per plant: this context is served by mpcq_mimo_* only");
    if (need == kGeneric && c->mode != mpcq_ctx::Mode::Generic)
        return fail(MPCQ_ERR_ORDER, c->mode == mpcq_ctx::Mode::Mimo
                                        ? "the context was last set up by mpcq_mimo_setup_plants_device (MIMO)"
                                    : c->mode == mpcq_ctx::Mode::OneShot
                                        ? "mpcq_mpc_plants_step_device keeps no operators: set the plants up again"
                                        : "mpcq_setup has not succeeded");
    if (need == kAnySetup && c->mode == mpcq_ctx::Mode::None) return fail(MPCQ_ERR_ORDER, "no setup has succeeded");
    HIPCHK(hipSetDevice(c->dims.device));
    return MPCQ_OK;
}

// The plants' setup data and operator blocks (generic setups; mimo-only contexts keep one unused block)
int ensure_plant_buffers(mpcq_ctx *c)
{
    // (no early return on one pointer: after a failed allocation the next call allocates whatever is still
    // missing, so a call that returns MPCQ_OK always leaves every non-empty buffer allocated)
    const size_t Pg = c->mimo_only ? 1 : c->dims.n_plants, n = c->dims.n, m = c->dims.m;
    const mpcq::OpsLayout L = mpcq::OpsLayout::make(c->nc, c->mc);
    void **ptrs[] = {(void **)&c->d_P, (void **)&c->d_q0, (void **)&c->d_A, (void **)&c->d_l0, (void **)&c->d_u0,
                     (void **)&c->d_ops, (void **)&c->d_ops32, (void **)&c->d_ctype};
    const size_t bytes[] = {8 * Pg * n * n, 8 * Pg * n, 8 * Pg * m * n, 8 * Pg * m, 8 * Pg * m, 8 * Pg * L.total,
                            c->dims.dtype == MPCQ_F32 ? 4 * Pg * L.total : 0, 4 * Pg * c->mc};
    for (int i = 0; i < 8; i++) {
        if (!bytes[i] || *ptrs[i]) continue;
        if (hipMalloc(ptrs[i], std::max<size_t>(bytes[i], 8)) != hipSuccess) {
            *ptrs[i] = nullptr;
            return fail(MPCQ_ERR_HIP, "hipMalloc failed (plant setup buffers)");
        }
    }
    return MPCQ_OK;
}

// Generic entry points that only need the device and the generic buffers (no setup yet)
int check_generic_dims(mpcq_ctx *c)
{
    int rc = check_ctx(c, kNone);
    if (rc) return rc;
    if (c->mimo_only) return fail(MPCQ_ERR_ARG, "n > 32 or m > 64 per plant: this context is served by mpcq_mimo_* only");
    return MPCQ_OK;
}

int h2d(void *dst, const void *src, size_t bytes, hipStream_t s)
{
    if (!bytes) return MPCQ_OK;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    return MPCQ_OK;
}

}  // namespace

static void verbose_header(const mpcq_ctx *c, const char *what);  // (settings.verbose: below)

extern "C" {

void mpcq_default_settings(mpcq_settings *s)
{
    if (!s) return;
    // osqp constants.h (v0.6) + osqp-eigen setWarmStart(true) (ModelPredictiveControlAPI.cpp:52)
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
    s->verbose = 0;
}

const char *mpcq_last_error(void) { return g_err.c_str(); }

int mpcq_create(const mpcq_dims *d, const mpcq_settings *s, mpcq_ctx **out)
{
    if (!d || !out) return fail(MPCQ_ERR_ARG, "null argument");
    *out = nullptr;
    if (d->n <= 0 || d->m < 0 || d->batch <= 0) return fail(MPCQ_ERR_ARG, "n > 0, m >= 0, batch > 0 required");
    if (d->n_plants != 1 && d->n_plants != d->batch) return fail(MPCQ_ERR_ARG, "n_plants must be 1 or batch");
    if (d->dtype != MPCQ_F64 && d->dtype != MPCQ_F32 && d->dtype != MPCQ_F64_MIXED) return fail(MPCQ_ERR_ARG, "dtype");
    mpcq_settings st;
    mpcq_default_settings(&st);
    if (s) st = *s;
    if (st.rho <= 0 || st.sigma <= 0 || st.alpha <= 0 || st.alpha >= 2 || st.max_iter <= 0 ||
        st.eps_abs < 0 || st.eps_rel < 0 || (st.eps_abs == 0 && st.eps_rel == 0) || st.scaling < 0 ||
        st.check_termination < 0 || st.adaptive_rho_tolerance < 1 || st.adaptive_rho_interval < 0)
        return fail(MPCQ_ERR_ARG, "invalid settings (osqp validate_settings)");
    int nc = 0, mc = 0;
    const int KN = (d->n + 3) / 4, KM = (std::max(d->m, 1) + 3) / 4;
    const bool tile = d->n_plants == 1 && mpcq_internal_tile_supported(KN, KM) &&
                      std::strcmp(test_hook("MPCQ_KERNEL"), "lane") != 0;
    if (tile) {
        nc = 16 * ((KN + 3) / 4);
        mc = 16 * ((KM + 3) / 4);
    } else if (mpcq_internal_caps(d->n, std::max(d->m, 1), &nc, &mc) != 0) {
        // larger per-plant QPs: only the MIMO condensed-MPC path (mpcq_mimo_*) serves them
        if (!(d->n_plants == d->batch && d->n <= 128 && d->m == 2 * d->n && d->dtype != MPCQ_F32))
            return fail(MPCQ_ERR_ARG, "n/m exceed the compiled kernel capacities (n <= 32, m <= 64; the MIMO "
                                      "MPC path takes per-plant n <= 128, m = 2n, fp64)");
        nc = d->n;
        mc = d->m;
    }

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= d->device || d->device < 0)
        return fail(MPCQ_ERR_HIP, "no HIP device with this ordinal");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, d->device) != hipSuccess)
        return fail(MPCQ_ERR_HIP, "hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(MPCQ_ERR_HIP, std::string("device is ") + prop.gcnArchName + ", gfx950 required");
    HIPCHK(hipSetDevice(d->device));

    mpcq_ctx *c = new mpcq_ctx();
    c->dims = *d;
    c->set = st;
    c->nc = nc;
    c->mc = mc;
    c->cus = prop.multiProcessorCount;
    c->tile = tile;
    c->mimo_only = !tile && (d->n > 32 || d->m > 64);
    c->KN = KN;
    c->KM = KM;
    const mpcq::OpsLayout L = mpcq::OpsLayout::make(nc, mc);
    c->ops_stride = L.total;
    const size_t P = d->n_plants, B = d->batch, n = d->n, m = d->m;
    const size_t es = d->dtype == MPCQ_F32 ? 4 : 8;
    bool ok = true;
    auto A = [&](void **p, size_t bytes) {
        if (!ok) return;
        if (hipMalloc(p, std::max<size_t>(bytes, 8)) != hipSuccess) ok = false;
    };
    // a shared plant's setup arrays now; per-plant ones at the first setup (ensure_plant_buffers): a
    // one-pass context (mpcq_mpc_plants_step_device, ~1M plants on one GPU) never allocates them
    if (P == 1 && !(ok = ensure_plant_buffers(c) == MPCQ_OK)) {
        mpcq_destroy(c);
        return fail(MPCQ_ERR_HIP, "hipMalloc failed");
    }
    A((void **)&c->d_setup_status, 4 * P);
    A((void **)&c->d_flags, 4);
    A((void **)&c->d_q, 8 * B * n);
    A((void **)&c->d_u, 8 * B * m);
    A((void **)&c->d_l, 8 * B * m);
    A((void **)&c->d_x, 8 * B * n);
    A((void **)&c->d_y, 8 * B * m);
    A((void **)&c->d_rho, 8 * B);
    A((void **)&c->d_status, 4 * B);
    A((void **)&c->d_iter, 4 * B);
    A(&c->d_xs, es * B * nc);
    A(&c->d_zs, es * B * mc);
    A(&c->d_ys, es * B * mc);
    A(&c->d_rhos, es * B);
    if (tile) {
        A(&c->d_img, es * mpcq::TileLayout::buffer(KN, KM, (int)(16 / es)));
        const size_t lcap = (size_t)mpcq::ListSeg::kShards * mpcq::ListSeg::cap(B);  // entries per phase list
        A((void **)&c->d_list, 4 * 2 * lcap);
        A((void **)&c->d_counts, 4 * kMaxPhases * mpcq::ListSeg::kCounters);
        A((void **)&c->d_itstate, 4 * B);
    } else if (!c->mimo_only) {
        A(&c->d_snx, es * B * nc);
        A(&c->d_sny, es * B * mc);
    }
    if (!ok) {
        mpcq_destroy(c);
        return fail(MPCQ_ERR_HIP, "hipMalloc failed");
    }
    c->hD.assign(n, 1.0);
    c->hE.assign(m, 1.0);
    *out = c;
    return MPCQ_OK;
}

int mpcq_destroy(mpcq_ctx *c)
{
    if (!c) return MPCQ_OK;
    (void)hipSetDevice(c->dims.device);
    void *ptrs[] = {c->d_P, c->d_q0, c->d_A, c->d_l0, c->d_u0, c->d_ops, c->d_ops32, c->d_scratch, c->d_ctype,
                    c->d_setup_status, c->d_q, c->d_u, c->d_l, c->d_x, c->d_y, c->d_rho, c->d_status, c->d_iter,
                    c->d_xs, c->d_zs, c->d_ys, c->d_rhos, c->d_snx, c->d_sny, c->d_Fx, c->d_Fu, c->d_Fr,
                    c->d_Sbar, c->d_Ku, c->d_W0, c->d_X, c->d_U, c->d_img, c->d_list, c->d_counts,
                    c->d_itstate, c->d_Ad, c->d_Bd, c->d_step, c->d_flags, c->d_stamps, c->d_mimo,
                    c->d_it_acc, c->d_uns_acc, c->d_Xs, c->d_Us, c->d_ordmap, c->d_ord};
    if (c->gexec) (void)hipGraphExecDestroy(c->gexec);
    if (c->graph) (void)hipGraphDestroy(c->graph);
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    delete c;
    return MPCQ_OK;
}

// Lower bounds kappa on ||P^ dx|| / ||dx|| in the two norms OSQP's is_dual_infeasible compares
// (AdmmArgs::dinf_kappa), for a shared plant in the eigen-basis with every row an inequality: then
// P~ = P^ + sigma I and W' P~ W = I, so lambda_min(P~) = 1 / ||W||_2^2 >= 1 / ||W||_F^2 and
// mu = 1 / ||W||_F^2 - sigma <= lambda_min(P^).  With v = dx (scaled space):
//   ||P^ v||_inf >= mu ||v||_2 / sqrt(n) >= (mu / sqrt(n)) ||v||_inf                     (scaled_termination)
//   ||D^-1 P^ v||_inf >= (min_i D_i^-1) (mu / sqrt(n)) ||v||_inf
//                     >= (min_i D_i^-1) mu / (sqrt(n) max_i D_i) ||D v||_inf              (unscaled)
static void dinf_bounds(mpcq_ctx *c, const double *blk, const mpcq::OpsLayout &L)
{
    c->dinf_ks = c->dinf_ku = 0.0;
    const size_t n = c->dims.n;
    if (c->dims.n_plants != 1 || c->inv_ops || !c->all_ineq || n == 0) return;
    double fro = 0.0, dmax = 0.0, dinv_min = HUGE_VAL;
    for (size_t i = 0; i < (size_t)c->nc * c->nc; i++) fro += blk[L.W + i] * blk[L.W + i];
    for (size_t i = 0; i < n; i++) {
        dmax = std::max(dmax, blk[L.D + i]);
        dinv_min = std::min(dinv_min, 1.0 / blk[L.D + i]);
    }
    const double mu = 1.0 / fro - c->set.sigma;
    if (!(fro > 0.0) || !(mu > 0.0) || !(dmax > 0.0)) return;
    c->dinf_ks = mu / std::sqrt((double)n);
    c->dinf_ku = dinv_min * mu / (std::sqrt((double)n) * dmax);
}

// Setup kernels on the device-resident setup data (d_P, d_q0, d_A, d_l0, d_u0), operator
// conversion / tile images, per-QP broadcast of q0/u0/l0, state reset and the plant-0 scaling
// readback.  One 4-byte flag word (non-convex plant, non-inequality row) comes back to the host.
int setup_on_device(mpcq_ctx *c, hipStream_t s)
{
    if (int rc = materialize_xy(c)) return rc;  // (with the images of the solve that left it)
    c->qu_lazy = false;  // (q, u are re-broadcast from the setup data below)
    c->gen++;
    const size_t Pn = c->dims.n_plants, n = c->dims.n, m = c->dims.m, B = c->dims.batch;
    HIPCHK(hipMemsetAsync(c->d_ops, 0, 8 * Pn * c->ops_stride, s));
    HIPCHK(hipMemsetAsync(c->d_flags, 0, 4, s));
    mpcq::SetupArgs a{};
    a.n = (int)n;
    a.m = (int)m;
    a.nc = c->nc;
    a.mc = c->mc;
    a.n_plants = (int)Pn;
    a.scaling = c->set.scaling;
    a.sigma = c->set.sigma;
    a.rho = c->set.rho;
    // an fp32 solve reads W to ~1e-7: a basis orthogonal to ~1e-10 saves the last Jacobi sweep
    a.jacobi_tol = c->dims.dtype == MPCQ_F32 ? 1e-20 : 1e-32;
    a.P = c->d_P;
    a.q0 = c->d_q0;
    a.A = c->d_A;
    a.l0 = c->d_l0;
    a.u0 = c->d_u0;
    a.ops = c->d_ops;
    a.ctype = c->d_ctype;
    a.status = c->d_setup_status;
    a.flags = c->d_flags;
    // One wavefront per plant, LDS-resident (mpcq_setup_wave.hip), where the plant fits: per-plant
    // batches take the direct inverse of M(rho) (no eigen-solve: their QPs are solved once or a few
    // times each), a shared plant the eigen-basis (every QP of the batch reuses it, whatever rho it
    // reaches; the tile kernel's images).  The global-scratch workgroup kernel (eigen-basis) serves
    // larger plants.  Test hook MPCQ_SETUP: "ref" forces the workgroup kernel, "eigen" the wave
    // kernel's eigen-basis for per-plant batches.
    const char *hook = test_hook("MPCQ_SETUP");
    const bool fits = mpcq_internal_setup_wave_lds((int)n, (int)m) != 0;
    const bool ref_setup = !std::strcmp(hook, "ref") || !fits;
    c->inv_ops = !ref_setup && Pn > 1 && std::strcmp(hook, "eigen") != 0;
    if (c->inv_ops) {
        if (mpcq_internal_setup_inv_launch(&a, s) != 0) return fail(MPCQ_ERR_HIP, "setup kernel launch failed");
    } else if (ref_setup) {
        if (!c->d_scratch && hipMalloc((void **)&c->d_scratch, 8 * Pn * setup_scratch_len((int)n, (int)m)) != hipSuccess)
            return fail(MPCQ_ERR_HIP, "hipMalloc failed (setup scratch)");
        a.scratch = c->d_scratch;
        if (mpcq_internal_setup_launch(&a, s) != 0) return fail(MPCQ_ERR_HIP, "setup kernel launch failed");
    } else {
        const char *pe = debug_hook("MPCQ_SETUP_PROF");  // per-stage clock stamps to a file
        long long *prof = nullptr;
        if (*pe && hipMalloc((void **)&prof, 8 * 16 * Pn) == hipSuccess) {
            (void)hipMemsetAsync(prof, 0, 8 * 16 * Pn, s);
            a.prof = prof;
        }
        if (mpcq_internal_setup_wave_launch(&a, s) != 0) return fail(MPCQ_ERR_HIP, "setup kernel launch failed");
        if (prof) {
            std::vector<long long> h(16 * Pn);
            HIPCHK(hipMemcpyAsync(h.data(), prof, 8 * 16 * Pn, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            (void)hipFree(prof);
            if (FILE *f = std::fopen(pe, "wb")) {
                std::fwrite(h.data(), 8, h.size(), f);
                std::fclose(f);
            } else {
                std::fprintf(stderr, "[mpcq] MPCQ_SETUP_PROF: cannot open %s for writing\n", pe);
            }
        }
    }
    // plant-0 scaling (mpcq_get_scaling, host-side bound checks) and the flag word: one sync
    const mpcq::OpsLayout L = mpcq::OpsLayout::make(c->nc, c->mc);
    std::vector<double> blk(c->ops_stride);
    int flags = 0;
    HIPCHK(hipMemcpyAsync(&flags, c->d_flags, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(blk.data(), c->d_ops, 8 * c->ops_stride, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (flags & 1) return fail(MPCQ_ERR_SETUP, "setup: P + sigma I (+ rho A'A) not positive definite (non-convex QP)");
    if (flags & 4) return fail(MPCQ_ERR_SETUP, "setup: Jacobi eigen-solve of the KKT family did not converge in 60 sweeps");
    c->all_ineq = !(flags & 2);
    for (size_t i = 0; i < n; i++) c->hD[i] = blk[L.D + i];
    for (size_t j = 0; j < m; j++) c->hE[j] = blk[L.E + j];
    c->hc = blk[L.cs];
    dinf_bounds(c, blk.data(), L);
    if (c->dims.dtype == MPCQ_F32 &&
        mpcq_internal_f64_to_f32(c->d_ops, c->d_ops32, Pn * c->ops_stride, s) != 0)
        return fail(MPCQ_ERR_HIP, "operator conversion failed");
    if (c->tile && mpcq_internal_tile_images(c->d_ops, c->nc, c->mc, c->KN, c->KM, c->dims.dtype == MPCQ_F32,
                                             c->d_img, s) != 0)
        return fail(MPCQ_ERR_HIP, "tile image kernel failed");
    const int per = Pn > 1;
    if (mpcq_internal_broadcast(c->d_q0, c->d_q, (int)n, (int)B, per, s) ||
        mpcq_internal_broadcast(c->d_u0, c->d_u, (int)m, (int)B, per, s) ||
        mpcq_internal_broadcast(c->d_l0, c->d_l, (int)m, (int)B, per, s))
        return fail(MPCQ_ERR_HIP, "broadcast failed");
    return reset_state(c, true);
}

static int build_order_map(mpcq_ctx *c);  // (below: the hardest-first order of a tile-path MPC step)

int mpcq_setup(mpcq_ctx *c, const double *P, const double *q0, const double *A, const double *l0,
               const double *u0)
{
    int rc = check_generic_dims(c);
    if (rc) return rc;
    const size_t Pn = c->dims.n_plants, n = c->dims.n, m = c->dims.m;
    if (!P || !q0 || (m && (!A || !l0 || !u0))) return fail(MPCQ_ERR_ARG, "null setup array");
    for (size_t i = 0; i < Pn * m; i++)
        if (l0[i] > u0[i]) return fail(MPCQ_ERR_BOUNDS, "lower bound above upper bound (osqp validate_data)");
    if ((rc = ensure_plant_buffers(c))) return rc;
    c->mode = mpcq_ctx::Mode::None;
    // rows n + j of A are the negated rows j (the reference's Gbar = [K0 L; -K0 L],
    // ModelPredictiveControlAPI.cpp:332-347), checked bit for bit: the tile kernel's paired loop
    c->paired = Pn == 1 && m == 2 * n && n % 4 == 0;
    for (size_t i = 0; c->paired && i < n * n; i++)
        if (!(A[n * n + i] == -A[i])) c->paired = false;
    hipStream_t s = c->last;
    if ((rc = h2d(c->d_P, P, 8 * Pn * n * n, s)) || (rc = h2d(c->d_q0, q0, 8 * Pn * n, s)) ||
        (rc = h2d(c->d_A, A, 8 * Pn * m * n, s)) || (rc = h2d(c->d_l0, l0, 8 * Pn * m, s)) ||
        (rc = h2d(c->d_u0, u0, 8 * Pn * m, s)))
        return rc;
    if ((rc = setup_on_device(c, s))) return rc;
    c->lower_free = lower_all_free(c, l0);
    c->gen++;
    c->mode = mpcq_ctx::Mode::Generic;
    if ((rc = build_order_map(c))) return rc;  // (new P, A: the MPC step's order map, if operators are set)
    verbose_header(c, "mpcq_setup (osqp_setup: Ruiz scaling, constraint types, KKT basis)");
    return MPCQ_OK;
}

static int materialize_qu(mpcq_ctx *c);  // (below: the lazy q, u of a tile-path controllerStep)

int mpcq_update_lin_cost(mpcq_ctx *c, const double *q)
{
    int rc = check_ctx(c, kGeneric);
    if (rc) return rc;
    if ((rc = materialize_qu(c))) return rc;  // (the other vector of the pending step)
    if (!q) return fail(MPCQ_ERR_ARG, "null q");
    return h2d(c->d_q, q, 8 * (size_t)c->dims.batch * c->dims.n, c->last);
}

int mpcq_update_upper_bound(mpcq_ctx *c, const double *u)
{
    int rc = check_ctx(c, kGeneric);
    if (rc) return rc;
    if ((rc = materialize_qu(c))) return rc;  // (the other vector of the pending step)
    if (!u) return fail(MPCQ_ERR_ARG, "null u");
    return h2d(c->d_u, u, 8 * (size_t)c->dims.batch * c->dims.m, c->last);
}

int mpcq_update_lower_bound(mpcq_ctx *c, const double *l)
{
    int rc = check_ctx(c, kGeneric);
    if (rc) return rc;
    if ((rc = materialize_qu(c))) return rc;  // (the other vector of the pending step)
    if (!l) return fail(MPCQ_ERR_ARG, "null l");
    const bool lf = lower_all_free_batch(c, l);
    if (lf != c->lower_free) c->gen++;
    c->lower_free = lf;
    return h2d(c->d_l, l, 8 * (size_t)c->dims.batch * c->dims.m, c->last);
}

int mpcq_update_bounds(mpcq_ctx *c, const double *l, const double *u)
{
    int rc = mpcq_update_lower_bound(c, l);
    return rc ? rc : mpcq_update_upper_bound(c, u);
}

int mpcq_cold_start(mpcq_ctx *c)
{
    int rc = check_ctx(c, kGeneric);
    if (rc) return rc;
    if ((rc = reset_state(c, false))) return rc;
    HIPCHK(hipStreamSynchronize(c->last));
    return MPCQ_OK;
}

int mpcq_warm_start(mpcq_ctx *c, const double *x, const double *y)
{
    int rc = check_ctx(c, kGeneric);
    if (rc) return rc;
    if (!x || (c->dims.m && !y)) return fail(MPCQ_ERR_ARG, "null x/y");
    c->xy_lazy = false;  // (x, y are staged in the output buffers below; a rejected call keeps a pending x, y)
    // stage in the output buffers (overwritten by the next solve)
    if ((rc = h2d(c->d_x, x, 8 * (size_t)c->dims.batch * c->dims.n, c->last))) return rc;
    if ((rc = h2d(c->d_y, y, 8 * (size_t)c->dims.batch * c->dims.m, c->last))) return rc;
    if (c->dims.dtype == MPCQ_F32) {
        auto a = make_args<float>(c);
        rc = mpcq_internal_warm_f32(&a, c->nc, c->mc, c->d_x, c->d_y, c->last);
    } else {
        auto a = make_args<double>(c);
        rc = mpcq_internal_warm_f64(&a, c->nc, c->mc, c->d_x, c->d_y, c->last);
    }
    if (rc) return fail(MPCQ_ERR_HIP, "warm start kernel failed");
    HIPCHK(hipStreamSynchronize(c->last));
    return MPCQ_OK;
}

}  // extern "C"

// Phase boundaries of the tile path (multiples of check_termination, then max_iter): QPs still
// running at a boundary are re-packed densely into the waves of the next launch.  Default: stops at
// 4 and 5 check_termination (100 and 125 iterations at the defaults), then the QPs that need more
// (the ~tens of the long tail) finish on the one-QP-per-wave kernel: each runs on its own SIMD at
// ~0.7 us per iteration, where a tile wave holding them runs at its slowest column's pace, ~0.9 us
// per lone-wave iteration (config 2: 347-350 us per solve against 368-371 us for [100, max_iter] on
// tile waves).  When the batch is more than ~1.5 rounds of the chip's tile-wave slots the
// chain is 3, 4 check_termination and max_iter on tile waves, where the re-pack at 75 pays; a tile
// chain forced onto a batch under 8,192 QPs (MPCQ_KERNEL=tile; the default there is the wave kernel)
// stops at 4 check_termination and runs the rest on tile waves.
// *wave_tail: the last launch runs on the wave kernel (test hooks MPCQ_PHASES, MPCQ_TAIL=wave|tile).
constexpr bool kWaveTail = false;  // [100, 125] + wave tail: slower in round 4 (tile tail f32 +2.4 %, mixed +8 %)
// ordered (phase 0 in hardest-first order, mpcq_order.hip): one launch per solve.  Its waves hold QPs of
// like difficulty, so a re-pack saves little, and the slow QPs start first instead of waiting for a
// later phase (config 2 mixed, one box: 0.335 ms against 0.406-0.416 ms for the same order with stops at
// 100 or 125 and 0.446-0.474 ms in index order, profiles/r05a_order_mixed.log).
static int phase_stops(const mpcq_settings &st, int batch, int cus, int *stops, bool *wave_tail, bool ordered = false)
{
    const int ct = st.check_termination;
    int np = 0;
    const char *e = test_hook("MPCQ_PHASES");  // "0" = one launch per solve, or check multiples "3,4,5"
    const char *t = test_hook("MPCQ_TAIL");
    const bool many = (long)batch / 16 > (long)cus * 4 * 3 * 3 / 2;  // waves vs 3 waves/SIMD, 4 SIMD/CU
    int mult[kMaxPhases] = {3, 4};
    int nm = 2;
    *wave_tail = false;
    if (ordered) {
        nm = 0;
    } else if (!many && batch < 8192) {  // (a tile chain forced onto a small batch: one stop, tile waves)
        mult[0] = 4;
        nm = 1;
    } else if (!many) {
        mult[0] = 4;
        mult[1] = 5;
        *wave_tail = kWaveTail;
        if (!kWaveTail) nm = 1;
    }
    const int cap = kMaxPhases;
    if (e[0] == '0') nm = 0;
    else if (*e) {
        nm = 0;
        *wave_tail = false;
        for (const char *p = e; *p && nm < cap - 1;) {
            mult[nm++] = std::atoi(p);
            while (*p && *p != ',') p++;
            if (*p == ',') p++;
        }
    }
    if (t[0] == 'w') {  // test hook: [100, 125] (or the MPCQ_PHASES list) + wave tail
        if (!*e && !many && batch >= 8192) {
            mult[1] = 5;
            nm = 2;
        }
        *wave_tail = true;
    }
    if (t[0] == 't') *wave_tail = false;
    if (ct > 0) {
        for (int i = 0; i < nm; i++) {
            const long it = (long)mult[i] * ct;
            if (it >= st.max_iter || np >= cap - 1) break;
            if (np && it <= stops[np - 1]) continue;
            stops[np++] = (int)it;
        }
    }
    stops[np++] = st.max_iter;
    if (np < 2) *wave_tail = false;  // (phase 0 stays on tile waves)
    return np;
}

static const char *env_kernel() { return test_hook("MPCQ_KERNEL"); }

template <typename T>
static int wave_launch(mpcq_ctx *c, const mpcq::AdmmArgs<T> &a, int grid, hipStream_t s)
{
    return std::is_same<T, float>::value
               ? mpcq_internal_wave_launch_f32((const mpcq::AdmmArgs<float> *)&a, c->nc, c->mc, grid, s)
               : mpcq_internal_wave_launch_f64((const mpcq::AdmmArgs<double> *)&a, c->nc, c->mc, grid, s);
}

// The phase chain of a tile solve on stream s: phase p's QPs still running at its stop are appended to
// the ListSeg list of phase p + 1 (two alternating lists; each phase its own block of counters).
template <typename T>
static int launch_phases(mpcq_ctx *c, mpcq::AdmmArgs<T> &a, hipStream_t s, bool wave_only)
{
    const int B = c->dims.batch;
    int stops[kMaxPhases];
    bool wave_tail = false;
    // an MPC step on the tile waves runs its batch hardest-first (mpcq_order.hip; test hook MPCQ_ORDER=0:
    // index order)
    const bool ordered = a.mpc && a.X && a.U && c->ord_ok && !wave_only && test_hook("MPCQ_ORDER")[0] != '0';
    const int np = phase_stops(c->set, B, c->cus, stops, &wave_tail, ordered);
    c->ord_last = ordered;
    int *const ord_cnt = c->d_ord, *const ord_key = c->d_ord + mpcq::OrderBins::kBins, *const ord_list = ord_key + B;
    if (ordered) {
        // the counters are zero unless the last ordered sort's tile launch did not run (it clears them)
        if (!c->ord_clean && hipMemsetAsync(ord_cnt, 0, 4 * (size_t)mpcq::OrderBins::kBins, s) != hipSuccess) return -2;
        c->ord_clean = false;
        if (mpcq_internal_order(B, c->nx, c->dims.m, a.X, a.U, c->d_ordmap, a.xref, ord_cnt, ord_key, ord_list,
                                a.X_save, a.U_save, s) != 0)
            return -2;
    }
    // (an ordered step's X, U copies are the order kernel's: its phase-0 tile launch skips them)
    double *const X_save = a.X_save, *const U_save = a.U_save;
    const int seg = mpcq::ListSeg::cap(B);
    const size_t lcap = (size_t)mpcq::ListSeg::kShards * seg;
    // Counter blocks: launch p zeroes block p + 1 (its successor's output) and a chain's final launch,
    // when it is at least the third, zeroes block 0 for the next solve; only a chain that could not
    // leave block 0 clean costs a memset here.
    if (!c->count0_clean && hipMemsetAsync(c->d_counts, 0, 4 * (size_t)mpcq::ListSeg::kCounters, s) != hipSuccess)
        return -2;
    c->count0_clean = false;
    const int mpc = a.mpc;
    // one QP per wave: from phase 0 for small batches, else the chain's last launch (phase_stops)
    const int tail_from = wave_only ? 0 : wave_tail ? np - 1 : kMaxPhases;
    int np_run = 0;
    a.list_seg = seg;
    // a chain entirely on tile waves publishes x, y lazily (materialize_xy; test hook MPCQ_LAZY_XY=0: eager)
    const bool lazy_xy = tail_from >= np && test_hook("MPCQ_LAZY_XY")[0] != '0';
    if (lazy_xy) {
        a.x = nullptr;
        a.y = nullptr;
        // fp64 state: the finalize stores rho once, as warm state (materialize_rho reports it)
        if (std::is_same<T, double>::value) a.rho_out = nullptr;
    }
    // ... and one ordered launch its status, iter in list-slot order (materialize_info; test hook
    // MPCQ_LAZY_INFO=0: at the QPs' indices)
    const bool lazy_info = lazy_xy && ordered && np == 1 && test_hook("MPCQ_LAZY_INFO")[0] != '0';
    a.info_slot = lazy_info ? ord_list + B : nullptr;

    // debug build: per-wave stage stamps of every phase launch, written to $MPCQ_TILE_STAMPS after the solve
    const char *stp = debug_hook("MPCQ_TILE_STAMPS");
    const size_t waves = (size_t)(B + 15) / 16 + 4 * mpcq::ListSeg::kShards;
    if (stp && *stp && !c->d_stamps && hipMalloc((void **)&c->d_stamps, 8 * 8 * waves * kMaxPhases) != hipSuccess)
        return -2;
    if (stp && *stp && hipMemsetAsync(c->d_stamps, 0, 8 * 8 * waves * kMaxPhases, s) != hipSuccess) return -2;
    for (int p = 0; p < np; p++) {
        a.stamps = (stp && *stp) ? c->d_stamps + (size_t)p * 8 * waves : nullptr;
        a.img = (const T *)c->d_img;
        a.list_in = p ? c->d_list + (size_t)(p % 2) * lcap : nullptr;
        a.count_in = p ? c->d_counts + (size_t)(p - 1) * mpcq::ListSeg::kCounters : nullptr;
        a.list_out = c->d_list + (size_t)((p + 1) % 2) * lcap;
        a.count_out = c->d_counts + (size_t)p * mpcq::ListSeg::kCounters;
        a.it_state = c->d_itstate;
        a.ord_list = (ordered && p == 0) ? ord_list : nullptr;
        a.X_save = (ordered && p == 0) ? nullptr : X_save;
        a.U_save = (ordered && p == 0) ? nullptr : U_save;
        a.ord_zero = (ordered && p == 0) ? ord_cnt : nullptr;
        a.stop_iter = stops[p];
        a.resume = p > 0;
        a.mpc = p == 0 ? mpc : 0;  // later phases read q, u from the buffers phase 0 filled
        const bool final_launch = p + 1 == np || (p >= tail_from && c->dims.n <= 32 && c->dims.m <= 64);
        a.zero_cnt = final_launch ? nullptr : c->d_counts + (size_t)(p + 1) * mpcq::ListSeg::kCounters;
        a.zero_cnt0 = (final_launch && p >= 2) ? c->d_counts : nullptr;
        int rc;
        if (p >= tail_from && c->dims.n <= 32 && c->dims.m <= 64) {
            // one QP per wave carries no idle columns: the rest of the solve is one launch (a resumed
            // list: a multiple of ListSeg::kShards blocks)
            a.stop_iter = c->set.max_iter;
            if (p > 0 && mpc && a.X_save) {
                // the wave kernel reads q, u from the buffers, which a lazy phase 0 did not fill: its
                // front end rebuilds them from X, U (the tile prologue's fp64 order) for the QPs it runs
                a.mpc = 1;
                a.q_out = c->d_q;
                a.u_out = c->d_u;
            }
            rc = wave_launch<T>(c, a, p == 0 ? B : 2048, s);
            if (rc) return rc;
            c->count0_clean = a.zero_cnt0 != nullptr;
            np_run = p + (stp && *stp ? 1 : 0);  // (the stamps dump includes the wave launch)
            break;
        }
        // every phase launches the phase-0 grid: list segment s is served by the blocks b % kShards == s
        rc = std::is_same<T, float>::value
                 ? mpcq_internal_tile_launch_f32((const mpcq::AdmmArgs<float> *)&a, c->KN, c->KM, s)
                 : mpcq_internal_tile_launch_f64((const mpcq::AdmmArgs<double> *)&a, c->KN, c->KM, s);
        if (rc) return rc;
        c->count0_clean = a.zero_cnt0 != nullptr;
        if (a.ord_zero) c->ord_clean = true;
        np_run = p + 1;
    }
    c->xy_lazy = lazy_xy;
    c->rho_lazy = lazy_xy && std::is_same<T, double>::value;
    c->info_lazy = lazy_info;
    if (stp && *stp) {
        std::vector<long long> h(8 * waves * kMaxPhases);
        if (hipMemcpyAsync(h.data(), c->d_stamps, 8 * h.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -2;
        if (FILE *f = std::fopen(stp, "wb")) {
            const long long hdr[2] = {(long long)np_run, (long long)waves};
            std::fwrite(hdr, 8, 2, f);
            std::fwrite(h.data(), 8, 8 * waves * np_run, f);
            std::fclose(f);
        }
    }
    return 0;
}

// The device path of this context's next solve, decided in one place for launch_args and
// mpcq_get_path: per-plant contexts run one QP per wave (n <= 32, m <= 64) or one QP per lane;
// shared-plant contexts run the MFMA tile kernel's phase chain (its tail one QP per wave), except
// that small batches (under 512 tile waves: latency-bound) run one QP per wave throughout.
struct PathChoice {
    int kind;    // MPCQ_PATH_*
    bool paired; // the tile kernel's paired loop
};
static PathChoice choose_path(const mpcq_ctx *c)
{
    const char *k = env_kernel();
    const bool fits_wave = c->dims.n <= 32 && c->dims.m <= 64;
    PathChoice p{MPCQ_PATH_LANE, false};
    if (c->inv_ops) return {MPCQ_PATH_WAVE, false};  // direct-inverse operators: the wave kernel's refactorisation
    if (std::strcmp(k, "lane") == 0 || !fits_wave) return p;
    if (!c->tile) return {MPCQ_PATH_WAVE, false};
    const bool small = c->dims.batch < 8192 && std::strcmp(k, "tile") != 0;
    if (small || std::strcmp(k, "wave") == 0) return {MPCQ_PATH_WAVE, false};
    return {MPCQ_PATH_TILE, c->paired && c->all_ineq && c->lower_free};
}

template <typename T>
static int launch_args(mpcq_ctx *c, mpcq::AdmmArgs<T> &a, hipStream_t s)
{
    const PathChoice p = choose_path(c);
    a.paired = p.paired;
    if (p.kind == MPCQ_PATH_LANE)
        return std::is_same<T, float>::value
                   ? mpcq_internal_admm_launch_f32((const mpcq::AdmmArgs<float> *)&a, c->nc, c->mc, s)
                   : mpcq_internal_admm_launch_f64((const mpcq::AdmmArgs<double> *)&a, c->nc, c->mc, s);
    if (!c->tile) {  // per-plant batches: one QP per wave (operators in VGPRs)
        a.stop_iter = c->set.max_iter;
        return wave_launch<T>(c, a, c->dims.batch, s);
    }
    return launch_phases<T>(c, a, s, p.kind == MPCQ_PATH_WAVE);
}

template <typename T>
static int launch_typed(mpcq_ctx *c, hipStream_t s, bool mpc, const double *X, double *U, double xref)
{
    auto a = make_args<T>(c);
    if (mpc) {
        a.mpc = 1; a.mpc_u = 1; a.nx = c->nx; a.X = X; a.U = U; a.xref = xref;
        a.Fx = c->d_Fx; a.Fu = c->d_Fu; a.Fr = c->d_Fr; a.Sbar = c->d_Sbar; a.Ku = c->d_Ku; a.W0 = c->d_W0;
        const bool lazy = c->tile && choose_path(c).kind == MPCQ_PATH_TILE && c->d_Xs && c->d_Us;
        if (lazy) {  // phase 0 saves X, U (40 B/QP) instead of writing q, u (480 B/QP): materialize_qu
            a.X_save = c->d_Xs; a.U_save = c->d_Us;
        } else {
            a.q_out = c->d_q; a.u_out = c->d_u;
        }
        c->qu_lazy = lazy;
        c->lazy_xref = xref;
    }
    return launch_args<T>(c, a, s);
}

// ---- settings.verbose (osqp-eigen setVerbosity, ModelPredictiveControlAPI.cpp:51, solver.cpp:21-25):
// OSQP v0.6's setup header, its iteration summary line and its status footer, for QP 0 of the context
// (the reference's one QP), plus the batch's status counts.  The device keeps no per-iteration record,
// so the summary is the final iterate's line: objective, primal and dual residual of the returned
// (x, y) in the unscaled problem, the final rho, the host-timed solve.  Printed on stdout as OSQP does;
// a verbose solve synchronises its stream.
static const char *status_name(int st)
{
    switch (st) {
    case MPCQ_SOLVED: return "solved";
    case MPCQ_SOLVED_INACCURATE: return "solved inaccurate";
    case MPCQ_MAX_ITER_REACHED: return "maximum iterations reached";
    case MPCQ_PRIMAL_INFEASIBLE: return "primal infeasible";
    case MPCQ_DUAL_INFEASIBLE: return "dual infeasible";
    case MPCQ_NON_CVX: return "problem non convex";
    case MPCQ_INVALID_BOUNDS: return "invalid bounds (u < l)";
    case MPCQ_TYPE_CHANGED: return "constraint type changed (re-run setup)";
    case MPCQ_UNSOLVED: return "unsolved";
    default: return st == 3 ? "primal infeasible inaccurate" : st == 4 ? "dual infeasible inaccurate" : "unknown";
    }
}

static void verbose_header(const mpcq_ctx *c, const char *what)
{
    if (!c->set.verbose) return;
    const mpcq_settings &s = c->set;
    const char *dt = c->dims.dtype == MPCQ_F32 ? "fp32 iterate, fp64 setup"
                     : c->dims.dtype == MPCQ_F64_MIXED ? "fp64 (fp32 plain iterations on the tile path)" : "fp64";
    std::printf("-----------------------------------------------------------------\n"
                "   libmpcq: batched OSQP-v0.6 ADMM on gfx950 (solvempc_amd)\n"
                "-----------------------------------------------------------------\n");
    std::printf("problem:  variables n = %d, constraints m = %d\n", c->dims.n, c->dims.m);
    std::printf("          batch = %d QPs, %s, %s\n", c->dims.batch,
                c->dims.n_plants == 1 ? "one shared (P, A)" : "one (P, A) per QP", dt);
    std::printf("          setup: %s\n", what);
    std::printf("settings: linear system solver = reduced KKT on the device (%s),\n",
                c->tile ? "eigenbasis, MFMA tile kernel" : c->inv_ops ? "direct inverse" : "eigenbasis");
    std::printf("          eps_abs = %.1e, eps_rel = %.1e,\n", s.eps_abs, s.eps_rel);
    std::printf("          eps_prim_inf = %.1e, eps_dual_inf = %.1e,\n", s.eps_prim_inf, s.eps_dual_inf);
    std::printf("          rho = %.2e %s,\n", s.rho, s.adaptive_rho ? "(adaptive)" : "");
    std::printf("          sigma = %.2e, alpha = %.2f, max_iter = %d\n", s.sigma, s.alpha, s.max_iter);
    if (s.check_termination) std::printf("          check_termination: on (interval %d),\n", s.check_termination);
    else std::printf("          check_termination: off,\n");
    std::printf("          scaling: %s, scaled_termination: %s\n", s.scaling ? "on" : "off",
                s.scaled_termination ? "on" : "off");
    std::printf("          warm start: %s, polish: off, time_limit: off\n\n", s.warm_start ? "on" : "off");
    std::fflush(stdout);
}

static void verbose_solve(mpcq_ctx *c, double seconds)
{
    const size_t B = c->dims.batch, n = c->dims.n, m = c->dims.m;
    std::vector<int> st(B), it(B);
    std::vector<double> rho(B), x(n), y(m), q(n), u(m), l(m), P(n * n), A(m * n);
    if (materialize_xy(c) != MPCQ_OK || materialize_rho(c) != MPCQ_OK || materialize_info(c) != MPCQ_OK ||
        hipStreamSynchronize(c->last) != hipSuccess ||
        hipMemcpy(st.data(), c->d_status, 4 * B, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(it.data(), c->d_iter, 4 * B, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(rho.data(), c->d_rho, 8 * B, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(x.data(), c->d_x, 8 * n, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(y.data(), c->d_y, 8 * m, hipMemcpyDeviceToHost) != hipSuccess)
        return;
    // QP 0's data in the unscaled problem (generic contexts: plant 0's P, A and this solve's q, l, u)
    bool have = c->mode == mpcq_ctx::Mode::Generic && materialize_qu(c) == MPCQ_OK &&
                hipMemcpy(q.data(), c->d_q, 8 * n, hipMemcpyDeviceToHost) == hipSuccess &&
                hipMemcpy(u.data(), c->d_u, 8 * m, hipMemcpyDeviceToHost) == hipSuccess &&
                hipMemcpy(l.data(), c->d_l, 8 * m, hipMemcpyDeviceToHost) == hipSuccess &&
                hipMemcpy(P.data(), c->d_P, 8 * n * n, hipMemcpyDeviceToHost) == hipSuccess &&
                hipMemcpy(A.data(), c->d_A, 8 * m * n, hipMemcpyDeviceToHost) == hipSuccess;
    const bool sol = st[0] == MPCQ_SOLVED || st[0] == MPCQ_SOLVED_INACCURATE || st[0] == MPCQ_MAX_ITER_REACHED;
    double obj = 0.0, pri = 0.0, dua = 0.0;
    if (have && sol) {
        std::vector<double> Px(n, 0.0), Aty(n, 0.0);
        for (size_t i = 0; i < n; i++)
            for (size_t k = 0; k < n; k++) Px[i] += P[std::min(i, k) * n + std::max(i, k)] * x[k];  // upper triangle
        for (size_t j = 0; j < m; j++) {
            double ax = 0.0;
            for (size_t k = 0; k < n; k++) {
                ax += A[j * n + k] * x[k];
                Aty[k] += A[j * n + k] * y[j];
            }
            pri = std::max(pri, std::max(ax - u[j], l[j] - ax));
        }
        for (size_t i = 0; i < n; i++) {
            obj += 0.5 * x[i] * Px[i] + q[i] * x[i];
            dua = std::max(dua, std::fabs(Px[i] + q[i] + Aty[i]));
        }
    }
    std::printf("iter   objective    pri res    dua res    rho        time\n");
    if (have && sol) std::printf("%4d  %12.4e  %9.2e  %9.2e  %9.2e  %9.2es\n\n", it[0], obj, pri, dua, rho[0], seconds);
    else std::printf("%4d  %12s  %9s  %9s  %9.2e  %9.2es\n\n", it[0], "-", "-", "-", rho[0], seconds);
    std::printf("status:               %s\n", status_name(st[0]));
    std::printf("number of iterations: %d\n", it[0]);
    if (have && sol) std::printf("optimal objective:    %.4f\n", obj);
    std::printf("run time:             %.2es\n", seconds);
    std::printf("final rho:            %.2e\n", rho[0]);
    if (B > 1) {
        size_t solved = 0;
        long long tot = 0;
        int mn = it[0], mx = it[0];
        for (size_t b = 0; b < B; b++) {
            solved += st[b] == MPCQ_SOLVED;
            tot += it[b];
            mn = std::min(mn, it[b]);
            mx = std::max(mx, it[b]);
        }
        std::printf("batch:                %zu QPs, %zu solved, iterations %d / %.1f / %d (min / mean / max)\n", B,
                    solved, mn, (double)tot / B, mx);
    }
    std::printf("\n");
    std::fflush(stdout);
}

extern "C" {

static int launch_solve(mpcq_ctx *c, hipStream_t s, bool mpc, const double *X, double *U, double xref)
{
    const auto t0 = std::chrono::steady_clock::now();
    c->ord_last = false;  // (launch_phases sets it for a hardest-first tile solve)
    c->xy_lazy = false;   // (and this, for a chain that publishes x, y lazily)
    c->rho_lazy = false;  // (the solve below writes d_rho, or leaves it lazy again)
    c->info_lazy = false;  // (and d_status, d_iter: every solve writes every QP's)
    const int rc = c->dims.dtype == MPCQ_F32 ? launch_typed<float>(c, s, mpc, X, U, xref)
                                             : launch_typed<double>(c, s, mpc, X, U, xref);
    if (rc) return fail(MPCQ_ERR_HIP, std::string("ADMM kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
    c->last = s;
    c->fresh = false;
    // settings.verbose: the summary needs the results on the host, so it synchronises the stream, which a
    // stream under capture (mpcq_mpc_run_device's per-step graph) must not do: there the replay loop prints
    // after each replayed step instead
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (c->set.verbose && hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone) {
        (void)hipStreamSynchronize(s);
        verbose_solve(c, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    return MPCQ_OK;
}

int mpcq_reset(mpcq_ctx *c)
{
    int rc = check_ctx(c, kAnySetup);
    if (rc) return rc;
    c->fresh = true;
    return MPCQ_OK;
}

int mpcq_solve(mpcq_ctx *c, void *stream)
{
    int rc = check_ctx(c, kGeneric);
    if (rc) return rc;
    if ((rc = materialize_qu(c))) return rc;
    return launch_solve(c, (hipStream_t)stream, false, nullptr, nullptr, 0.0);
}

static int d2h(mpcq_ctx *c, void *dst, const void *src, size_t bytes)
{
    if (!dst || !bytes) return MPCQ_OK;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->last));
    HIPCHK(hipStreamSynchronize(c->last));
    return MPCQ_OK;
}

int mpcq_get_solution(mpcq_ctx *c, double *x)
{
    int rc = check_ctx(c, kAnySetup);
    if (rc) return rc;
    if (!x) return fail(MPCQ_ERR_ARG, "null x");
    if ((rc = materialize_xy(c))) return rc;
    return d2h(c, x, c->d_x, 8 * (size_t)c->dims.batch * c->dims.n);
}

int mpcq_get_dual(mpcq_ctx *c, double *y)
{
    int rc = check_ctx(c, kAnySetup);
    if (rc) return rc;
    if (!y && c->dims.m) return fail(MPCQ_ERR_ARG, "null y");
    if ((rc = materialize_xy(c))) return rc;
    return d2h(c, y, c->d_y, 8 * (size_t)c->dims.batch * c->dims.m);
}

int mpcq_get_info(mpcq_ctx *c, int *status, int *iter, double *rho)
{
    int rc = check_ctx(c, kAnySetup);
    if (rc) return rc;
    const size_t B = c->dims.batch;
    if (rho && (rc = materialize_rho(c))) return rc;
    if ((status || iter) && (rc = materialize_info(c))) return rc;
    if ((rc = d2h(c, status, c->d_status, 4 * B))) return rc;
    if ((rc = d2h(c, iter, c->d_iter, 4 * B))) return rc;
    return d2h(c, rho, c->d_rho, 8 * B);
}

int mpcq_get_scaling(mpcq_ctx *c, double *D, double *E, double *cc)
{
    int rc = check_ctx(c, kGeneric);
    if (rc) return rc;
    if (D) std::copy(c->hD.begin(), c->hD.end(), D);
    if (E) std::copy(c->hE.begin(), c->hE.end(), E);
    if (cc) *cc = c->hc;
    return MPCQ_OK;
}

int mpcq_get_stream_path(mpcq_ctx *c, int *kind)
{
    if (!c || !kind) return fail(MPCQ_ERR_ARG, "null argument");
    *kind = c->stream_path;
    return MPCQ_OK;
}

int mpcq_get_order(mpcq_ctx *c, int *ordered, int *order)
{
    if (!c || !ordered) return fail(MPCQ_ERR_ARG, "null argument");
    *ordered = c->ord_last ? 1 : 0;
    if (order) {
        const size_t B = c->dims.batch;
        if (!c->ord_last) {
            for (size_t i = 0; i < B; i++) order[i] = (int)i;
        } else {
            HIPCHK(hipMemcpyAsync(order, c->d_ord + mpcq::OrderBins::kBins + B, 4 * B, hipMemcpyDeviceToHost, c->last));
            HIPCHK(hipStreamSynchronize(c->last));
        }
    }
    return MPCQ_OK;
}

int mpcq_get_path(mpcq_ctx *c, int *kind, int *paired)
{
    if (!c) return fail(MPCQ_ERR_ARG, "null context");
    const PathChoice p = choose_path(c);
    if (kind) *kind = p.kind;
    if (paired) *paired = p.paired;
    return MPCQ_OK;
}

int mpcq_device_view_get(mpcq_ctx *c, mpcq_device_view *v)
{
    if (!c || !v) return fail(MPCQ_ERR_ARG, "null argument");
    int rc = materialize_qu(c);  // (enqueued on the context's last stream)
    if (rc || (rc = materialize_xy(c)) || (rc = materialize_rho(c)) || (rc = materialize_info(c))) return rc;
    v->q = c->d_q;
    v->u = c->d_u;
    v->l = c->d_l;
    v->x = c->d_x;
    v->y = c->d_y;
    v->status = c->d_status;
    v->iter = c->d_iter;
    v->rho = c->d_rho;
    return MPCQ_OK;
}

// Device buffers of the MPC front-end operators for nx states (per plant) and X/U staging.
bool alloc_mpc_ops(mpcq_ctx *c, int nx)
{
    const size_t Pn = c->dims.n_plants, n = c->dims.n, m = c->dims.m;
    if (c->nx != nx) {
        c->gen++;
        for (double **p : {&c->d_Fx, &c->d_Sbar})
            if (*p) { (void)hipFree(*p); *p = nullptr; }
        if (c->d_X) { (void)hipFree(c->d_X); c->d_X = nullptr; }
        if (c->d_Xs) { (void)hipFree(c->d_Xs); c->d_Xs = nullptr; }
    }
    auto A = [&](double **p, size_t cnt) -> bool {
        return *p || hipMalloc((void **)p, 8 * std::max<size_t>(cnt, 1)) == hipSuccess;
    };
    return A(&c->d_Fx, Pn * n * nx) && A(&c->d_Fu, Pn * n) && A(&c->d_Fr, Pn * n * n) &&
           A(&c->d_Sbar, Pn * m * nx) && A(&c->d_Ku, Pn * m) && A(&c->d_W0, Pn * m) &&
           A(&c->d_X, (size_t)c->dims.batch * nx) && A(&c->d_U, (size_t)c->dims.batch) &&
           A(&c->d_Xs, (size_t)c->dims.batch * nx) && A(&c->d_Us, (size_t)c->dims.batch);
}

// d_q, d_u from the last tile-path controllerStep's saved X, U (mpcq_internal_front_end), once.
static int materialize_qu(mpcq_ctx *c)
{
    if (!c->qu_lazy) return MPCQ_OK;
    c->qu_lazy = false;
    if (mpcq_internal_front_end((int)c->dims.batch, c->nx, (int)c->dims.n, (int)c->dims.m, c->d_Xs, c->d_Us,
                                c->lazy_xref, c->d_Fx, c->d_Fu, c->d_Fr, c->d_Sbar, c->d_Ku, c->d_W0, c->d_q,
                                c->d_u, c->last) != 0)
        return fail(MPCQ_ERR_HIP, "front-end kernel launch failed");
    return MPCQ_OK;
}

// d_x, d_y of the last tile solve from its stored warm state (mpcq_tile.h tile_publish_kernel), once.
static int materialize_xy(mpcq_ctx *c)
{
    if (!c->xy_lazy) return MPCQ_OK;
    c->xy_lazy = false;
    int rc = materialize_info(c);  // (the publish kernel reads each QP's status)
    if (rc) return rc;
    if (c->dims.dtype == MPCQ_F32) {
        auto a = make_args<float>(c);
        a.img = (const float *)c->d_img;
        rc = mpcq_internal_tile_publish_f32(&a, c->KN, c->KM, a.paired = c->paired && c->all_ineq && c->lower_free, c->last);
    } else {
        auto a = make_args<double>(c);
        a.img = (const double *)c->d_img;
        rc = mpcq_internal_tile_publish_f64(&a, c->KN, c->KM, a.paired = c->paired && c->all_ineq && c->lower_free, c->last);
    }
    return rc ? fail(MPCQ_ERR_HIP, "solution publish kernel failed") : MPCQ_OK;
}

// d_rho of the last tile solve from its warm-state rho (fp64: the same value), once.
static int materialize_rho(mpcq_ctx *c)
{
    if (!c->rho_lazy) return MPCQ_OK;
    c->rho_lazy = false;
    HIPCHK(hipMemcpyAsync(c->d_rho, c->d_rhos, 8 * (size_t)c->dims.batch, hipMemcpyDeviceToDevice, c->last));
    return MPCQ_OK;
}

// d_status, d_iter of the last ordered single-launch solve from its list-slot pairs, once.
static int materialize_info(mpcq_ctx *c)
{
    if (!c->info_lazy) return MPCQ_OK;
    c->info_lazy = false;
    const int B = c->dims.batch;
    const int *list = c->d_ord + mpcq::OrderBins::kBins + B;
    if (mpcq_internal_order_info(B, list, list + B, c->d_status, c->d_iter, c->last) != 0)
        return fail(MPCQ_ERR_HIP, "status publish kernel failed");
    return MPCQ_OK;
}

// The bound-violation map of the hardest-first order (mpcq_order.hip) for a shared plant with MPC
// operators: x_u = -P^-1 q is the QP's unconstrained optimum and v = A x_u - u, with q = Fx X + Fu U +
// (Fr 1) xref and u = W0 + Sbar X + Ku U (setF :372-375, setUpperBound :360-369), so
//   v = (-A P^-1 Fx - Sbar) X + (-A P^-1 Fu - Ku) U + (-A P^-1 Fr 1) xref - W0   (OrderBins row layout).
// Host fp64 (Cholesky of plant 0's P, upper triangle as OSQP reads it), once per setup / operator set;
// the map only orders the batch (no result depends on it), so a P that is not positive definite or a
// shape the kernel does not take just leaves the order off.
// The order map's rows from one plant's condensed operators (host fp64): false when P is not positive
// definite or a row is not finite (no order then).
static bool order_map_rows(int n, int m, int nx, const std::vector<double> &P, const std::vector<double> &A,
                           const std::vector<double> &Fx, const std::vector<double> &Fu, const std::vector<double> &Fr,
                           const std::vector<double> &Sb, const std::vector<double> &Ku, const std::vector<double> &W0,
                           std::vector<double> &map)
{
    // Cholesky P = L L' (lower L in place, from P's upper triangle)
    std::vector<double> L((size_t)n * n, 0.0);
    for (int j = 0; j < n; j++) {
        for (int i = j; i < n; i++) {
            double v = P[(size_t)j * n + i];  // P(j, i), j <= i: upper triangle
            for (int k = 0; k < j; k++) v -= L[(size_t)i * n + k] * L[(size_t)j * n + k];
            if (i == j) {
                if (!(v > 0.0)) return false;  // not positive definite: no order
                L[(size_t)j * n + j] = std::sqrt(v);
            } else {
                L[(size_t)i * n + j] = v / L[(size_t)j * n + j];
            }
        }
    }
    // Z = P^-1 [Fx Fu Fr1] (n x (nx + 2)), then the map rows
    const int nr = nx + 2;
    std::vector<double> Z((size_t)n * nr);
    for (int i = 0; i < n; i++) {
        for (int t = 0; t < nx; t++) Z[(size_t)i * nr + t] = Fx[(size_t)i * nx + t];
        Z[(size_t)i * nr + nx] = Fu[i];
        double fr = 0.0;
        for (int t = 0; t < n; t++) fr += Fr[(size_t)i * n + t];
        Z[(size_t)i * nr + nx + 1] = fr;
    }
    for (int r = 0; r < nr; r++) {
        for (int i = 0; i < n; i++) {  // L y = b
            double v = Z[(size_t)i * nr + r];
            for (int k = 0; k < i; k++) v -= L[(size_t)i * n + k] * Z[(size_t)k * nr + r];
            Z[(size_t)i * nr + r] = v / L[(size_t)i * n + i];
        }
        for (int i = n - 1; i >= 0; i--) {  // L' z = y
            double v = Z[(size_t)i * nr + r];
            for (int k = i + 1; k < n; k++) v -= L[(size_t)k * n + i] * Z[(size_t)k * nr + r];
            Z[(size_t)i * nr + r] = v / L[(size_t)i * n + i];
        }
    }
    constexpr int KS = mpcq::OrderBins::kStride;
    map.assign((size_t)m * KS, 0.0);
    for (int j = 0; j < m; j++) {
        double az[10] = {0};
        for (int r = 0; r < nr; r++)
            for (int i = 0; i < n; i++) az[r] += A[(size_t)j * n + i] * Z[(size_t)i * nr + r];
        double *row = map.data() + (size_t)j * KS;
        for (int t = 0; t < nx; t++) row[t] = -az[t] - Sb[(size_t)j * nx + t];
        row[8] = -az[nx] - Ku[j];
        row[9] = -W0[j];
        row[10] = -az[nx + 1];
        for (int k = 0; k < KS; k++)
            if (!std::isfinite(row[k])) return false;
    }
    return true;
}

// The map to the device, with the order's counters and lists (allocated once per context).
static int upload_order_map(mpcq_ctx *c, const std::vector<double> &map, hipStream_t s)
{
    constexpr int KS = mpcq::OrderBins::kStride;
    const size_t ord_ints = (size_t)mpcq::OrderBins::kBins + 4 * (size_t)c->dims.batch;  // counters, keys, list, info
    if (!c->d_ordmap && hipMalloc((void **)&c->d_ordmap, 8 * (size_t)mpcq::OrderBins::kMaxRows * KS) != hipSuccess)
        return fail(MPCQ_ERR_HIP, "hipMalloc failed (order map)");
    if (!c->d_ord) {
        if (hipMalloc((void **)&c->d_ord, 4 * ord_ints) != hipSuccess) return fail(MPCQ_ERR_HIP, "hipMalloc failed (order lists)");
        HIPCHK(hipMemsetAsync(c->d_ord, 0, 4 * ord_ints, s));  // (list entries are batch indices, from the start)
        c->ord_clean = true;
        c->gen++;
    }
    if (int rc2 = h2d(c->d_ordmap, map.data(), 8 * map.size(), s)) return rc2;
    return MPCQ_OK;
}

static int build_order_map(mpcq_ctx *c)
{
    c->ord_ok = false;
    const int n = c->dims.n, m = c->dims.m, nx = c->nx;
    if (!c->tile || !c->mpc_ready || c->dims.n_plants != 1 || c->mode != mpcq_ctx::Mode::Generic || nx <= 0 ||
        nx > 8 || m > mpcq::OrderBins::kMaxRows)
        return MPCQ_OK;
    std::vector<double> P((size_t)n * n), A((size_t)m * n), Fx((size_t)n * nx), Fu(n), Fr((size_t)n * n),
        Sb((size_t)m * nx), Ku(m), W0(m);
    hipStream_t s = c->last;
    HIPCHK(hipMemcpyAsync(P.data(), c->d_P, 8 * P.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(A.data(), c->d_A, 8 * A.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(Fx.data(), c->d_Fx, 8 * Fx.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(Fu.data(), c->d_Fu, 8 * Fu.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(Fr.data(), c->d_Fr, 8 * Fr.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(Sb.data(), c->d_Sbar, 8 * Sb.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(Ku.data(), c->d_Ku, 8 * Ku.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(W0.data(), c->d_W0, 8 * W0.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    std::vector<double> map;
    if (!order_map_rows(n, m, nx, P, A, Fx, Fu, Fr, Sb, Ku, W0, map)) return MPCQ_OK;
    if (int rc = upload_order_map(c, map, s)) return rc;
    c->ord_ok = true;
    c->pord_ok = false;  // (the map is now this plant's)
    return MPCQ_OK;
}

int mpcq_mpc_set_operators(mpcq_ctx *c, int nx, const double *Fx, const double *Fu, const double *Fr,
                           const double *Sbar, const double *Ku, const double *W0)
{
    int rc = check_generic_dims(c);
    if (rc) return rc;
    const size_t Pn = c->dims.n_plants, n = c->dims.n, m = c->dims.m;
    if (nx <= 0 || nx > 8) return fail(MPCQ_ERR_ARG, "nx must be in 1..8");
    if (m != 2 * n) return fail(MPCQ_ERR_ARG, "MPC front end needs m == 2n (ModelPredictiveControlAPI.cpp:47-48)");
    if (!Fx || !Fu || !Fr || !Sbar || !Ku || !W0) return fail(MPCQ_ERR_ARG, "null operator");
    if ((rc = materialize_qu(c))) return rc;  // (with the operators the pending step used)
    if (!alloc_mpc_ops(c, nx)) return fail(MPCQ_ERR_HIP, "hipMalloc failed");
    c->nx = nx;
    hipStream_t s = c->last;
    if ((rc = h2d(c->d_Fx, Fx, 8 * Pn * n * nx, s)) || (rc = h2d(c->d_Fu, Fu, 8 * Pn * n, s)) ||
        (rc = h2d(c->d_Fr, Fr, 8 * Pn * n * n, s)) || (rc = h2d(c->d_Sbar, Sbar, 8 * Pn * m * nx, s)) ||
        (rc = h2d(c->d_Ku, Ku, 8 * Pn * m, s)) || (rc = h2d(c->d_W0, W0, 8 * Pn * m, s)))
        return rc;
    c->mpc_ready = true;
    return build_order_map(c);
}

int mpcq_mpc_step_device(mpcq_ctx *c, const double *X, double *U, double xref, void *stream)
{
    int rc = check_ctx(c, kGeneric);
    if (rc) return rc;
    if (!c->mpc_ready) return fail(MPCQ_ERR_ORDER, "mpcq_mpc_set_operators has not been called");
    if (!X || !U) return fail(MPCQ_ERR_ARG, "null X/U");
    return launch_solve(c, (hipStream_t)stream, true, X, U, xref);
}

int mpcq_mpc_step(mpcq_ctx *c, const double *X, double *U, double xref)
{
    int rc = check_ctx(c, kGeneric);
    if (rc) return rc;
    if (!c->mpc_ready) return fail(MPCQ_ERR_ORDER, "mpcq_mpc_set_operators has not been called");
    const size_t B = c->dims.batch;
    if ((rc = h2d(c->d_X, X, 8 * B * c->nx, c->last)) || (rc = h2d(c->d_U, U, 8 * B, c->last))) return rc;
    if ((rc = launch_solve(c, c->last, true, c->d_X, c->d_U, xref))) return rc;
    return d2h(c, U, c->d_U, 8 * B);
}

int mpcq_mpc_set_plant(mpcq_ctx *c, int nx, const double *Ad, const double *Bd)
{
    int rc = check_generic_dims(c);
    if (rc) return rc;
    if (nx <= 0 || nx > 8 || !Ad || !Bd) return fail(MPCQ_ERR_ARG, "set_plant: 1 <= nx <= 8 and Ad, Bd required");
    const size_t Pn = c->dims.n_plants;
    if (c->plant_nx != nx) {
        c->gen++;
        for (double **p : {&c->d_Ad, &c->d_Bd})
            if (*p) { (void)hipFree(*p); *p = nullptr; }
    }
    if (!c->d_it_acc) c->gen++;  // (the counters are baked into captured graphs)
    if ((!c->d_Ad && hipMalloc((void **)&c->d_Ad, 8 * Pn * nx * nx) != hipSuccess) ||
        (!c->d_Bd && hipMalloc((void **)&c->d_Bd, 8 * Pn * nx) != hipSuccess) ||
        (!c->d_step && hipMalloc((void **)&c->d_step, 8) != hipSuccess) ||
        (!c->d_it_acc && hipMalloc((void **)&c->d_it_acc, 4 * (size_t)c->dims.batch) != hipSuccess) ||
        (!c->d_uns_acc && hipMalloc((void **)&c->d_uns_acc, 4 * (size_t)c->dims.batch) != hipSuccess))
        return fail(MPCQ_ERR_HIP, "hipMalloc failed");
    c->plant_nx = nx;
    if ((rc = h2d(c->d_Ad, Ad, 8 * Pn * nx * nx, c->last)) || (rc = h2d(c->d_Bd, Bd, 8 * Pn * nx, c->last))) return rc;
    return MPCQ_OK;
}

int mpcq_mpc_stream_counters(mpcq_ctx *c, int *iters, int *unsolved)
{
    int rc = check_ctx(c, kGeneric);
    if (rc) return rc;
    if (!c->d_it_acc) return fail(MPCQ_ERR_ORDER, "mpcq_mpc_set_plant has not been called");
    const size_t B = c->dims.batch;
    if ((rc = d2h(c, iters, c->d_it_acc, 4 * B))) return rc;
    return d2h(c, unsolved, c->d_uns_acc, 4 * B);
}

int mpcq_mpc_simulate_device(mpcq_ctx *c, double *X, const double *U, unsigned long long seed, long long first_qp,
                             long long step, double noise_std, void *stream)
{
    int rc = check_generic_dims(c);
    if (rc) return rc;
    if (!c->plant_nx) return fail(MPCQ_ERR_ORDER, "mpcq_mpc_set_plant has not been called");
    if (!X || !U) return fail(MPCQ_ERR_ARG, "null X/U");
    if (mpcq_internal_simulate(c->dims.batch, c->plant_nx, c->dims.n_plants == 1, c->d_Ad, c->d_Bd, X, U, seed,
                               first_qp, nullptr, step, noise_std, (hipStream_t)stream))
        return fail(MPCQ_ERR_HIP, "simulate kernel launch failed");
    c->last = (hipStream_t)stream;
    return MPCQ_OK;
}

// The stream in one launch (stream_wave_kernel, mpcq_wave.h): the one-QP-per-wave path's control
// steps with the plant update between them, no per-step launches or graph.
}  // extern "C"
template <typename T>
static int launch_stream(mpcq_ctx *c, hipStream_t s, double *X, double *U, double xref, const mpcq::StreamArgs &sa)
{
    c->xy_lazy = false;  // (the stream writes every QP's x, y at its last step)
    c->rho_lazy = false;  // (and rho)
    c->info_lazy = false;  // (and status, iter)
    auto a = make_args<T>(c);
    a.mpc = 1; a.mpc_u = 1; a.nx = c->nx; a.X = X; a.U = U; a.xref = xref;
    a.Fx = c->d_Fx; a.Fu = c->d_Fu; a.Fr = c->d_Fr; a.Sbar = c->d_Sbar; a.Ku = c->d_Ku; a.W0 = c->d_W0;
    a.q_out = c->d_q; a.u_out = c->d_u;
    a.stop_iter = c->set.max_iter;
    c->qu_lazy = false;
    return std::is_same<T, float>::value
               ? mpcq_internal_stream_launch_f32((const mpcq::AdmmArgs<float> *)&a, c->nc, c->mc, &sa, s)
               : mpcq_internal_stream_launch_f64((const mpcq::AdmmArgs<double> *)&a, c->nc, c->mc, &sa, s);
}
extern "C" {

// The stream in one tile launch (admm_tile_kernel STREAM mode): every MFMA column is one plant that runs
// all its control steps, a wave holding `cpw` plants.  A control step of a column never waits for the
// others', so a wave lives as long as its slowest plant's iterations summed over the steps (not the
// per-step maximum over the batch); with a few thousand plants the chip is latency-bound, so cpw is
// chosen to spread the plants over every SIMD (MPCQ_STREAM_CPW: A/B).  Needs adapt_rho and max_iter
// on check iterations (multiples of check_termination, as OSQP's defaults are).
}  // extern "C"
template <typename T>
static int launch_tile_stream(mpcq_ctx *c, hipStream_t s, double *X, double *U, double xref, mpcq::StreamArgs sa)
{
    c->xy_lazy = false;  // (the stream writes every QP's x, y at its last step)
    c->rho_lazy = false;  // (and rho)
    c->info_lazy = false;  // (and status, iter)
    const mpcq_settings &st = c->set;
    const int ct = st.check_termination;
    auto a = make_args<T>(c);
    if (ct <= 0 || st.max_iter % ct || (st.adaptive_rho && a.adaptive_interval % ct)) return -1;
    const char *e = test_hook("MPCQ_STREAM_CPW");
    const long simds = (long)c->cus * 4;
    // plants per wave: one wave per SIMD (f32, 4 at 4,096 plants), twice that for fp64 / mixed, whose waves
    // measured faster at half the SIMDs (config 5: cpw 4 103.7 M QP/s, 6-16 105.5-106.3 M, r04w_*)
    const long per = ((long)c->dims.batch + simds - 1) / simds * (c->dims.dtype == MPCQ_F32 ? 1 : 2);
    sa.cpw = *e ? std::max(1, std::min(16, std::atoi(e))) : (int)std::max<long>(1, std::min<long>(16, per));
    // the kernel compiled for two waves per SIMD (its plant and check code spill outside the hot loop); the
    // variant compiled for one (no spills, MFMA accumulators in AGPRs) measured 2 % slower at config 5
    // (103.7 against 106.0 M QP/s, profiles/r05h_cfg5_occ_ab.jsonl): test hook MPCQ_STREAM_OCC=1 for A/B,
    // taken only when the waves fit one per SIMD
    const long waves = ((long)c->dims.batch + sa.cpw - 1) / sa.cpw;
    sa.occ = (waves <= simds && test_hook("MPCQ_STREAM_OCC")[0] == '1') ? 1 : 2;
    a.mpc = 1; a.mpc_u = 1; a.nx = c->nx; a.X = X; a.U = U; a.xref = xref;
    a.Fx = c->d_Fx; a.Fu = c->d_Fu; a.Fr = c->d_Fr; a.Sbar = c->d_Sbar; a.Ku = c->d_Ku; a.W0 = c->d_W0;
    a.X_save = c->d_Xs; a.U_save = c->d_Us;  // the last step's X, U: its q, u on demand (materialize_qu)
    a.paired = 1;
    a.img = (const T *)c->d_img;
    a.stop_iter = INT_MAX;
    a.sim = sa;
    // debug build: per-wave stage stamps of the launch (tools/stamps.py format, one phase), written to
    // $MPCQ_TILE_STAMPS after it
    const char *stp = debug_hook("MPCQ_TILE_STAMPS");
    const size_t swaves = (size_t)waves + 8;  // (+ a workgroup's idle waves)
    if (stp && *stp) {
        if (c->d_stamps) (void)hipFree(c->d_stamps);
        c->d_stamps = nullptr;
        if (hipMalloc((void **)&c->d_stamps, 8 * 8 * swaves) != hipSuccess ||
            hipMemsetAsync(c->d_stamps, 0, 8 * 8 * swaves, s) != hipSuccess)
            return -2;
        a.stamps = c->d_stamps;
    }
    const int rc = std::is_same<T, float>::value
                       ? mpcq_internal_tile_stream_launch_f32((const mpcq::AdmmArgs<float> *)&a, c->KN, c->KM, s)
                       : mpcq_internal_tile_stream_launch_f64((const mpcq::AdmmArgs<double> *)&a, c->KN, c->KM, s);
    if (rc == 0 && stp && *stp) {
        std::vector<long long> h(8 * swaves);
        if (hipMemcpyAsync(h.data(), c->d_stamps, 8 * h.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -2;
        if (FILE *f = std::fopen(stp, "wb")) {
            const long long hdr[2] = {1, (long long)swaves};
            std::fwrite(hdr, 8, 2, f);
            std::fwrite(h.data(), 8, h.size(), f);
            std::fclose(f);
        }
        (void)hipFree(c->d_stamps);
        c->d_stamps = nullptr;
    }
    if (rc == 0) {
        c->qu_lazy = true;
        c->lazy_xref = xref;
    }
    return rc;
}
extern "C" {

int mpcq_mpc_run_device(mpcq_ctx *c, double *X, double *U, double xref, int steps, unsigned long long seed,
                        long long first_qp, long long first_step, double noise_std, void *stream)
{
    int rc = check_ctx(c, kGeneric);
    if (rc) return rc;
    if (!c->mpc_ready || !c->plant_nx) return fail(MPCQ_ERR_ORDER, "mpc operators / plant not set");
    if (c->plant_nx != c->nx) return fail(MPCQ_ERR_ARG, "plant nx differs from the operators' nx");
    if (!X || !U || steps < 0) return fail(MPCQ_ERR_ARG, "null X/U or steps < 0");
    if (!stream) return fail(MPCQ_ERR_ARG, "graph capture needs a non-NULL stream");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemsetAsync(c->d_it_acc, 0, 4 * (size_t)c->dims.batch, s));
    HIPCHK(hipMemsetAsync(c->d_uns_acc, 0, 4 * (size_t)c->dims.batch, s));
    if (steps == 0) return MPCQ_OK;
    struct Acc {  // this call's launches (eager and captured) accumulate the stream counters
        mpcq_ctx *c;
        explicit Acc(mpcq_ctx *cc) : c(cc) { c->stream_acc = true; }
        ~Acc() { c->stream_acc = false; }
    } acc(c);
    if (mpcq_internal_set_step(c->d_step, first_step, s)) return fail(MPCQ_ERR_HIP, "set_step launch failed");
    const bool sync_each = debug_hook("MPCQ_DEBUG_SYNC")[0] == '1';  // synchronise every stage
    auto stage = [&](const char *what) -> int {
        if (!sync_each) return MPCQ_OK;
        const hipError_t e = hipStreamSynchronize(s);
        return e == hipSuccess ? MPCQ_OK : fail(MPCQ_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    };
    if ((rc = stage("set_step"))) return rc;
    // one launch for the whole stream: the tile kernel's stream mode for a shared plant of the paired
    // condensed-MPC shape, else one QP per wave (per-plant batches); MPCQ_STREAM=graph: the per-step
    // hipGraph below, MPCQ_STREAM=wave: the one-QP-per-wave launch (A/B and test cross-checks)
    const char *smode = test_hook("MPCQ_STREAM");
    const bool tile_ok = c->tile && c->paired && c->all_ineq && c->lower_free && c->d_Xs && c->d_Us &&
                         std::strcmp(smode, "graph") != 0 && std::strcmp(smode, "wave") != 0 &&
                         std::strcmp(test_hook("MPCQ_KERNEL"), "wave") != 0 && std::strcmp(test_hook("MPCQ_KERNEL"), "lane") != 0;
    if (tile_ok) {
        const mpcq::StreamArgs sa{steps, c->nx, c->dims.n_plants == 1, 0, c->d_Ad, c->d_Bd, seed, first_qp, first_step,
                                  noise_std};
        const int lrc = c->dims.dtype == MPCQ_F32 ? launch_tile_stream<float>(c, s, X, U, xref, sa)
                                                  : launch_tile_stream<double>(c, s, X, U, xref, sa);
        if (lrc == -2) return fail(MPCQ_ERR_HIP, std::string("tile stream launch failed: ") + hipGetErrorString(hipGetLastError()));
        if (lrc == 0) {
            if (mpcq_internal_set_step(c->d_step, first_step + steps, s)) return fail(MPCQ_ERR_HIP, "set_step launch failed");
            c->fresh = false;
            c->last = s;
            c->stream_path = MPCQ_STREAM_TILE;
            return stage("tile stream kernel");
        }
    }
    if (choose_path(c).kind == MPCQ_PATH_WAVE && c->dims.n <= 32 && c->dims.m <= 64 &&
        std::strcmp(smode, "graph") != 0) {
        const mpcq::StreamArgs sa{steps, c->nx, c->dims.n_plants == 1, 1, c->d_Ad, c->d_Bd, seed, first_qp, first_step,
                                  noise_std};
        const int lrc = c->dims.dtype == MPCQ_F32 ? launch_stream<float>(c, s, X, U, xref, sa)
                                                  : launch_stream<double>(c, s, X, U, xref, sa);
        if (lrc) return fail(MPCQ_ERR_HIP, std::string("stream kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
        if (mpcq_internal_set_step(c->d_step, first_step + steps, s)) return fail(MPCQ_ERR_HIP, "set_step launch failed");
        c->fresh = false;
        c->last = s;
        c->stream_path = MPCQ_STREAM_WAVE;
        return stage("stream kernel");
    }
    int done = 0;
    c->stream_path = MPCQ_STREAM_GRAPH;
    if (c->fresh) {  // a reset is a one-off (x = z = y = 0): run that step eagerly, capture the rest
        if ((rc = launch_solve(c, s, true, X, U, xref))) return rc;
        if (mpcq_internal_simulate(c->dims.batch, c->nx, c->dims.n_plants == 1, c->d_Ad, c->d_Bd, X, U, seed,
                                   first_qp, c->d_step, 0, noise_std, s) ||
            mpcq_internal_tick(c->d_step, s))
            return fail(MPCQ_ERR_HIP, "simulate kernel launch failed");
        done = 1;
        if ((rc = stage("eager first step"))) return rc;
    }
    const bool same = c->gexec && c->gkey.X == X && c->gkey.U == U && c->gkey.xref == xref &&
                      c->gkey.noise == noise_std && c->gkey.seed == seed && c->gkey.first_qp == first_qp &&
                      c->gkey.s == s && c->gkey.gen == c->gen;
    if (!same && done < steps) {
        if (c->gexec) { (void)hipGraphExecDestroy(c->gexec); c->gexec = nullptr; }
        if (c->graph) { (void)hipGraphDestroy(c->graph); c->graph = nullptr; }
        HIPCHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        int lrc = launch_solve(c, s, true, X, U, xref);
        if (!lrc && (mpcq_internal_simulate(c->dims.batch, c->nx, c->dims.n_plants == 1, c->d_Ad, c->d_Bd, X, U,
                                            seed, first_qp, c->d_step, 0, noise_std, s) ||
                     mpcq_internal_tick(c->d_step, s)))
            lrc = fail(MPCQ_ERR_HIP, "simulate kernel launch failed");
        hipGraph_t g = nullptr;
        const hipError_t ec = hipStreamEndCapture(s, &g);
        // a discarded capture ran none of its launches: the phase-list counters are not known clean
        if (lrc || ec != hipSuccess) c->count0_clean = false;
        if (lrc) { if (g) (void)hipGraphDestroy(g); return lrc; }
        if (ec != hipSuccess) return fail(MPCQ_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ec));
        c->graph = g;
        const hipError_t ei = hipGraphInstantiate(&c->gexec, c->graph, nullptr, nullptr, 0);
        if (ei != hipSuccess) {
            c->count0_clean = false;
            c->gexec = nullptr;
            return fail(MPCQ_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
        }
        c->gkey = {X, U, xref, noise_std, seed, first_qp, s, c->gen};
        c->glazy = {c->xy_lazy, c->rho_lazy, c->info_lazy, c->qu_lazy, c->ord_last, c->lazy_xref};
    }
    for (int k = done; k < steps; k++) {
        const auto t0 = std::chrono::steady_clock::now();
        HIPCHK(hipGraphLaunch(c->gexec, s));
        c->xy_lazy = c->glazy.xy;
        c->rho_lazy = c->glazy.rho;
        c->info_lazy = c->glazy.info;
        c->qu_lazy = c->glazy.qu;
        c->ord_last = c->glazy.ord;
        c->lazy_xref = c->glazy.xref;
        if (sync_each && (rc = stage(("graph replay " + std::to_string(k)).c_str()))) return rc;
        if (c->set.verbose) {  // (the captured solve printed nothing: launch_solve)
            HIPCHK(hipStreamSynchronize(s));
            c->last = s;
            verbose_solve(c, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
    }
    c->last = s;
    return MPCQ_OK;
}

int mpcq_condense(int device, int n_plants, int nx, int N, int s_rows, const double *Ad, const double *Bd,
                  const double *Cd, const double *K, const double *Q, const double *R, const double *RD, double *P,
                  double *A, double *Fx, double *Fu, double *Fr, double *Sbar, double *Ku, double *W0)
{
    if (n_plants <= 0 || nx <= 0 || nx > 8 || N <= 0 || s_rows < 0)
        return fail(MPCQ_ERR_ARG, "condense: n_plants > 0, 1 <= nx <= 8, N > 0, s_rows >= 0");
    const double *in[] = {Ad, Bd, Cd, K, Q, R, RD};
    double *outp[] = {P, A, Fx, Fu, Fr, Sbar, Ku, W0};
    for (auto p : in)
        if (!p) return fail(MPCQ_ERR_ARG, "condense: null input");
    for (auto p : outp)
        if (!p) return fail(MPCQ_ERR_ARG, "condense: null output");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(MPCQ_ERR_HIP, "no HIP device with this ordinal");
    HIPCHK(hipSetDevice(device));
    const size_t Pn = n_plants, X = nx, n = N;
    const size_t in_cnt[] = {Pn * X * X, Pn * X, Pn * X, Pn * X, Pn, Pn, Pn};
    const size_t out_cnt[] = {Pn * n * n, Pn * 2 * n * n, Pn * n * X, Pn * n, Pn * n * n, Pn * 2 * n * X, Pn * 2 * n, Pn * 2 * n};
    const bool force_ref = !std::strcmp(test_hook("MPCQ_CONDENSE"), "ref");  // the workgroup kernel
    const size_t scr = (N > 32 || force_ref) ? Pn * mpcq_internal_condense_scratch(nx, N) : 0;
    size_t total = scr;
    for (size_t c : in_cnt) total += c;
    for (size_t c : out_cnt) total += c;
    double *buf = nullptr;
    HIPCHK(hipMalloc((void **)&buf, 8 * total));
    mpcq::CondenseArgs a{};
    double *p = buf;
    const double **din[] = {&a.Ad, &a.Bd, &a.Cd, &a.K, &a.Q, &a.R, &a.RD};
    double **dout[] = {&a.P, &a.A, &a.Fx, &a.Fu, &a.Fr, &a.Sbar, &a.Ku, &a.W0};
    int rc = MPCQ_OK;
    for (int i = 0; i < 7 && !rc; i++) {
        *din[i] = p;
        if (hipMemcpy(p, in[i], 8 * in_cnt[i], hipMemcpyHostToDevice) != hipSuccess) rc = fail(MPCQ_ERR_HIP, "h2d");
        p += in_cnt[i];
    }
    for (int i = 0; i < 8; i++) {
        *dout[i] = p;
        p += out_cnt[i];
    }
    a.scratch = scr ? p : nullptr;
    a.force_ref = force_ref;
    a.n_plants = n_plants;
    a.nx = nx;
    a.N = N;
    a.s_rows = s_rows;
    if (!rc && mpcq_internal_condense_launch(&a, nullptr) != 0) rc = fail(MPCQ_ERR_HIP, "condense launch failed");
    if (!rc && hipDeviceSynchronize() != hipSuccess) rc = fail(MPCQ_ERR_HIP, "condense kernel failed");
    for (int i = 0; i < 8 && !rc; i++)
        if (hipMemcpy(outp[i], *dout[i], 8 * out_cnt[i], hipMemcpyDeviceToHost) != hipSuccess)
            rc = fail(MPCQ_ERR_HIP, "d2h");
    (void)hipFree(buf);
    return rc;
}


int mpcq_mpc_setup_plants_device(mpcq_ctx *c, int nx, int s_rows, const double *Ad, const double *Bd,
                                 const double *Cd, const double *K, const double *Q, const double *R,
                                 const double *RD, void *stream)
{
    int rc = check_generic_dims(c);
    if (rc) return rc;
    const size_t Pn = c->dims.n_plants, n = c->dims.n, m = c->dims.m;
    if (nx <= 0 || nx > 8 || s_rows < 0) return fail(MPCQ_ERR_ARG, "setup_plants: 1 <= nx <= 8, s_rows >= 0");
    if (m != 2 * n) return fail(MPCQ_ERR_ARG, "MPC front end needs m == 2n (ModelPredictiveControlAPI.cpp:47-48)");
    if (!Ad || !Bd || !Cd || !K || !Q || !R || !RD) return fail(MPCQ_ERR_ARG, "setup_plants: null plant array");
    if ((rc = ensure_plant_buffers(c))) return rc;
    if ((rc = materialize_qu(c))) return rc;  // (with the operators the pending step used)
    if (!alloc_mpc_ops(c, nx)) return fail(MPCQ_ERR_HIP, "hipMalloc failed");
    c->nx = nx;
    c->mode = mpcq_ctx::Mode::None;
    hipStream_t s = (hipStream_t)stream;
    c->last = s;
    mpcq::CondenseArgs a{};
    a.n_plants = (int)Pn;
    a.nx = nx;
    a.N = (int)n;
    a.s_rows = s_rows;
    a.Ad = Ad; a.Bd = Bd; a.Cd = Cd; a.K = K; a.Q = Q; a.R = R; a.RD = RD;
    a.P = c->d_P; a.A = c->d_A;
    a.Fx = c->d_Fx; a.Fu = c->d_Fu; a.Fr = c->d_Fr; a.Sbar = c->d_Sbar; a.Ku = c->d_Ku; a.W0 = c->d_W0;
    a.q0 = c->d_q0; a.l0 = c->d_l0; a.u0 = c->d_u0;
    double *scr = nullptr;
    if (n > 32 && hipMalloc((void **)&scr, 8 * Pn * mpcq_internal_condense_scratch(nx, (int)n)) != hipSuccess)
        return fail(MPCQ_ERR_HIP, "hipMalloc failed (condense scratch)");
    a.scratch = scr;
    rc = mpcq_internal_condense_launch(&a, s) != 0 ? fail(MPCQ_ERR_HIP, "condense launch failed") : MPCQ_OK;
    if (!rc) rc = setup_on_device(c, s);
    if (scr) (void)hipFree(scr);
    if (rc) return rc;
    c->last = s;
    c->lower_free = true;  // l0 = -DBL_MAX on every row (:42)
    c->gen++;
    c->mpc_ready = true;
    c->mode = mpcq_ctx::Mode::Generic;
    if ((rc = build_order_map(c))) return rc;  // (a shared plant's tile path: the step's order map)
    verbose_header(c, "mpcq_mpc_setup_plants_device (condensing + osqp_setup per plant)");
    return MPCQ_OK;
}


// The hardest-first map of a batch of distinct plants: the first plant's condensed operators (mpcq_condense,
// synchronous: once per set of plant arrays), folded as build_order_map folds a shared plant's.  The plants of
// config 3 are perturbations of one nominal plant (Ad, Bd +-2 %), so one plant's map ranks every QP's
// unconstrained-optimum violation closely enough to group QPs of like iteration counts in a wave and to run
// the slow ones first; the map only orders the batch, no result depends on it (a stale map, after the
// arrays' contents change under the same pointers, costs time only).
static int plants_order_map(mpcq_ctx *c, int nx, int s_rows, const double *Ad, const double *Bd, const double *Cd,
                            const double *K, const double *Q, const double *R, const double *RD, hipStream_t s)
{
    const int n = c->dims.n, m = c->dims.m;
    if (c->pord_ok && c->pord_key.Ad == Ad && c->pord_key.Bd == Bd && c->pord_key.Cd == Cd && c->pord_key.K == K &&
        c->pord_key.Q == Q && c->pord_key.R == R && c->pord_key.RD == RD && c->pord_key.nx == nx &&
        c->pord_key.s_rows == s_rows)
        return MPCQ_OK;
    c->pord_ok = false;
    c->ord_ok = false;  // (d_ordmap is about to hold the plants' map)
    if (m > mpcq::OrderBins::kMaxRows || nx > 8) return MPCQ_OK;
    std::vector<double> in((size_t)nx * nx + 3 * nx + 3);
    double *hAd = in.data(), *hBd = hAd + nx * nx, *hCd = hBd + nx, *hK = hCd + nx, *hQ = hK + nx;
    HIPCHK(hipMemcpyAsync(hAd, Ad, 8 * (size_t)nx * nx, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hBd, Bd, 8 * (size_t)nx, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hCd, Cd, 8 * (size_t)nx, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hK, K, 8 * (size_t)nx, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hQ, Q, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hQ + 1, R, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hQ + 2, RD, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    std::vector<double> P((size_t)n * n), A((size_t)m * n), Fx((size_t)n * nx), Fu(n), Fr((size_t)n * n),
        Sb((size_t)m * nx), Ku(m), W0(m);
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    if (mpcq_condense(dev, 1, nx, n, s_rows, hAd, hBd, hCd, hK, hQ, hQ + 1, hQ + 2, P.data(), A.data(), Fx.data(),
                      Fu.data(), Fr.data(), Sb.data(), Ku.data(), W0.data()) != MPCQ_OK)
        return MPCQ_OK;  // (no order: the step itself reports any error with these arrays)
    std::vector<double> map;
    if (!order_map_rows(n, m, nx, P, A, Fx, Fu, Fr, Sb, Ku, W0, map)) return MPCQ_OK;
    if (int rc = upload_order_map(c, map, s)) return rc;
    c->pord_ok = true;
    c->pord_key = {Ad, Bd, Cd, K, Q, R, RD, nx, s_rows};
    return MPCQ_OK;
}

int mpcq_mpc_plants_step_device(mpcq_ctx *c, int nx, int s_rows, const double *Ad, const double *Bd,
                                const double *Cd, const double *K, const double *Q, const double *R,
                                const double *RD, const double *X, double *U, double xref, void *stream)
{
    int rc = check_generic_dims(c);
    if (rc) return rc;
    const int n = c->dims.n, m = c->dims.m;
    if (nx <= 0 || nx > 8 || s_rows < 0) return fail(MPCQ_ERR_ARG, "plants_step: 1 <= nx <= 8, s_rows >= 0");
    if (m != 2 * n || n > 32) return fail(MPCQ_ERR_ARG, "plants_step: n = N <= 32, m = 2N (ModelPredictiveControlAPI.cpp:47-48)");
    if (c->dims.n_plants != c->dims.batch) return fail(MPCQ_ERR_ARG, "plants_step: one plant per QP (n_plants == batch)");
    if (!Ad || !Bd || !Cd || !K || !Q || !R || !RD || !X || !U) return fail(MPCQ_ERR_ARG, "plants_step: null array");
    hipStream_t s = (hipStream_t)stream;
    // the kernel below rewrites x, y, rho, status and iter of every QP on `s`: a pending lazy publication of an
    // earlier solve is dropped, not formed (it would be wasted work, and on another stream unordered with s)
    c->xy_lazy = c->rho_lazy = c->info_lazy = false;
    if (c->last && c->last != s) {  // (the earlier solve's work on its stream before this one's writes)
        hipEvent_t ev;
        HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        const hipError_t e1 = hipEventRecord(ev, c->last), e2 = e1 == hipSuccess ? hipStreamWaitEvent(s, ev, 0) : e1;
        (void)hipEventDestroy(ev);
        if (e2 != hipSuccess) return fail(MPCQ_ERR_HIP, "plants_step: stream ordering failed");
    }
    HIPCHK(hipMemsetAsync(c->d_flags, 0, 4, s));
    mpcq::PlantStepArgs a{};
    a.n_plants = c->dims.batch;
    a.nx = nx; a.N = n; a.s_rows = s_rows;
    a.Ad = Ad; a.Bd = Bd; a.Cd = Cd; a.K = K; a.Q = Q; a.R = R; a.RD = RD;
    a.X = X; a.U = U; a.xref = xref;
    a.st = to_solver(c->set);
    const int ct = c->set.check_termination;
    a.adaptive_interval = c->set.adaptive_rho_interval ? c->set.adaptive_rho_interval : (ct ? 4 * ct : 100);
    a.x = c->d_x; a.y = c->d_y; a.rho_out = c->d_rho; a.status = c->d_status; a.iter = c->d_iter;
    a.flags = c->d_flags;
    {
        // fp64 at 3 waves/SIMD (189 -> 168 VGPRs, a few spills in the check code: 39.4-40.0 M QP/s against
        // 35.5-35.9 M at 2), fp32 at 2 (3 spills into its loop: slower); MPCQ_PLANT_WPE=2|3 for A/B
        const char *w = test_hook("MPCQ_PLANT_WPE");
        a.wpe = *w ? std::atoi(w) : (c->dims.dtype == MPCQ_F32 ? 2 : 3);
        const char *l = test_hook("MPCQ_PLANT_LAYOUT");  // 2: two plants per wave at N 17 .. 20 (A/B, parity)
        a.layout = *l ? std::atoi(l) : 0;
    }
    // hardest-first (the first plant's map, mpcq_order.hip; test hook MPCQ_PLANT_ORDER=0: index order): slot i
    // of the grid runs plant list[i], and the kernel's workgroup 0 clears the bin counters for the next sort
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    const bool want = test_hook("MPCQ_PLANT_ORDER")[0] != '0' && c->dims.batch < (1 << mpcq::OrderBins::kRankBits) &&
                      hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone;
    if (want && (rc = plants_order_map(c, nx, s_rows, Ad, Bd, Cd, K, Q, R, RD, s))) return rc;
    const bool ordered = want && c->pord_ok;
    if (ordered) {
        const int B = c->dims.batch;
        int *const cnt = c->d_ord, *const key = cnt + mpcq::OrderBins::kBins, *const list = key + B;
        if (!c->ord_clean) HIPCHK(hipMemsetAsync(cnt, 0, 4 * (size_t)mpcq::OrderBins::kBins, s));
        c->ord_clean = false;
        if (mpcq_internal_order(B, nx, m, X, U, c->d_ordmap, xref, cnt, key, list, nullptr, nullptr, s) != 0)
            return fail(MPCQ_ERR_HIP, "plants_step order launch failed");
        a.order = list;
        a.ord_zero = cnt;
    }
    const char *pst = debug_hook("MPCQ_PLANT_STAMPS");  // per-wave stage stamps (a -DMPCQ_PLANT_STAMPS build)
    const size_t nwaves = (size_t)c->dims.batch;  // (an upper bound on the grid)
    if (pst && *pst) {
        if (c->d_stamps) (void)hipFree(c->d_stamps);
        c->d_stamps = nullptr;
        if (hipMalloc((void **)&c->d_stamps, 8 * 16 * nwaves) != hipSuccess) return fail(MPCQ_ERR_HIP, "hipMalloc failed (stamps)");
        HIPCHK(hipMemsetAsync(c->d_stamps, 0, 8 * 16 * nwaves, s));
        a.stamps = c->d_stamps;
    }
    const int lr = mpcq_internal_plant_step_launch(&a, c->dims.dtype == MPCQ_F32, s);
    if (lr) return fail(lr == -1 ? MPCQ_ERR_ARG : MPCQ_ERR_HIP, "plants_step kernel launch failed");
    if (pst && *pst) {
        std::vector<long long> h(16 * nwaves);
        HIPCHK(hipMemcpyAsync(h.data(), c->d_stamps, 8 * h.size(), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (FILE *f = std::fopen(pst, "wb")) {
            std::fwrite(h.data(), 8, h.size(), f);
            std::fclose(f);
        }
    }
    if (ordered) c->ord_clean = true;
    c->ord_last = ordered;
    c->mode = mpcq_ctx::Mode::OneShot;  // results only: no operator blocks were written
    c->mpc_ready = false;
    c->last = s;
    return MPCQ_OK;
}

int mpcq_mimo_setup_plants_device(mpcq_ctx *c, int nx, int nu, int ny, int s_rows, const double *Ad, const double *Bd,
                                  const double *Cd, const double *Q, const double *R, const double *RD, const double *K,
                                  const double *K0, const double *w0, void *stream)
{
    int rc = check_ctx(c, kNone);
    if (rc) return rc;
    if ((rc = materialize_xy(c))) return rc;  // (the operator blocks below replace the tile images' role)
    const int n = c->dims.n, m = c->dims.m;
    if (nu != 1 && nu != 2 && nu != 4) return fail(MPCQ_ERR_ARG, "mimo: n_u must be 1, 2 or 4");
    if (nx <= 0 || nx > 12 || ny <= 0 || ny > 12 || s_rows < 0) return fail(MPCQ_ERR_ARG, "mimo: 1 <= n_x, n_y <= 12");
    if (n % nu || n / nu > 32 || n > 128 || m != 2 * n) return fail(MPCQ_ERR_ARG, "mimo: n = N n_u <= 128 (N <= 32), m = 2n");
    if (c->dims.n_plants != c->dims.batch || c->dims.dtype == MPCQ_F32)
        return fail(MPCQ_ERR_ARG, "mimo: one plant per QP (n_plants == batch), dtype MPCQ_F64 or MPCQ_F64_MIXED");
    if (!Ad || !Bd || !Cd || !Q || !R || !RD || !K || !K0 || !w0) return fail(MPCQ_ERR_ARG, "mimo: null plant array");
    const int N = n / nu;
    const mpcq::MimoLayout L = mpcq::MimoLayout::make(N, nx, nu, ny);
    if (c->d_mimo && (c->mimo_N != N || c->mimo_nx != nx || c->mimo_nu != nu || c->mimo_ny != ny)) {
        (void)hipFree(c->d_mimo);
        c->d_mimo = nullptr;
    }
    if (!c->d_mimo && hipMalloc((void **)&c->d_mimo, 8 * (size_t)L.total * c->dims.n_plants) != hipSuccess)
        return fail(MPCQ_ERR_HIP, "hipMalloc failed (mimo operator blocks)");
    c->mimo_N = N; c->mimo_nx = nx; c->mimo_nu = nu; c->mimo_ny = ny; c->mimo_srows = s_rows;
    c->mode = mpcq_ctx::Mode::None;
    c->gen++;
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemsetAsync(c->d_flags, 0, 4, s));
    mpcq::MimoSetupArgs a{};
    a.n_plants = c->dims.n_plants;
    a.N = N; a.nx = nx; a.nu = nu; a.ny = ny; a.s_rows = s_rows;
    a.scaling = c->set.scaling;
    a.sigma = c->set.sigma;
    a.Ad = Ad; a.Bd = Bd; a.Cd = Cd; a.Q = Q; a.R = R; a.RD = RD; a.K = K; a.K0 = K0; a.w0 = w0;
    a.ops = c->d_mimo;
    a.flags = c->d_flags;
    const char *sst = debug_hook("MPCQ_MIMO_SETUP_STAMPS");  // per-plant phase stamps
    if (sst && *sst) {
        if (c->d_stamps) (void)hipFree(c->d_stamps);
        if (hipMalloc((void **)&c->d_stamps, 8 * 16 * (size_t)a.n_plants) != hipSuccess)
            return fail(MPCQ_ERR_HIP, "hipMalloc failed (stamps)");
        a.stamps = c->d_stamps;
    }
    const int lr = mpcq_internal_mimo_setup_launch(&a, s);
    if (lr == -1) return fail(MPCQ_ERR_ARG, "mimo: shape beyond the setup kernel's LDS capacity");
    if (lr) return fail(MPCQ_ERR_HIP, std::string("mimo setup launch failed: ") + hipGetErrorString(hipGetLastError()));
    int flags = 0;
    HIPCHK(hipMemcpyAsync(&flags, c->d_flags, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (sst && *sst) {
        std::vector<long long> h(16 * (size_t)a.n_plants);
        HIPCHK(hipMemcpy(h.data(), c->d_stamps, 8 * h.size(), hipMemcpyDeviceToHost));
        (void)hipFree(c->d_stamps);
        c->d_stamps = nullptr;
        if (FILE *f = std::fopen(sst, "wb")) {
            std::fwrite(h.data(), 8, h.size(), f);
            std::fclose(f);
        }
    }
    if (flags & 1) return fail(MPCQ_ERR_SETUP, "mimo: P + sigma I is not positive definite (non-convex QP)");
    if (flags & 2) return fail(MPCQ_ERR_SETUP, "mimo: a constraint row is not an inequality (|w0| beyond OSQP_INFTY)");
    c->mimo_diag_k0 = (flags & 4) ? 0 : 1;
    c->last = s;
    c->fresh = true;  // the first step starts from x = z = y = 0, rho = settings.rho (initSolver, :64)
    c->mpc_ready = false;  // the generic front-end operators no longer describe this context
    c->mode = mpcq_ctx::Mode::Mimo;
    return MPCQ_OK;
}

int mpcq_mimo_step_device(mpcq_ctx *c, const double *X, double *U, const double *yref, void *stream)
{
    int rc = check_ctx(c, kNone);
    if (rc) return rc;
    if ((rc = materialize_xy(c))) return rc;  // (a pending lazy x, y first: the kernel below rewrites the state)
    if (c->mode != mpcq_ctx::Mode::Mimo) return fail(MPCQ_ERR_ORDER, "mpcq_mimo_setup_plants_device has not succeeded");
    if (!X || !U) return fail(MPCQ_ERR_ARG, "null X/U");
    mpcq::MimoArgs a{};
    a.batch = c->dims.batch;
    a.N = c->mimo_N; a.nx = c->mimo_nx; a.nu = c->mimo_nu; a.ny = c->mimo_ny; a.s_rows = c->mimo_srows;
    a.diag_k0 = c->mimo_diag_k0 && !*test_hook("MPCQ_MIMO_GENERAL_K0");
    a.ops_stride = (size_t)mpcq::MimoLayout::make(a.N, a.nx, a.nu, a.ny).total;
    a.ops = c->d_mimo;
    a.st = to_solver(c->set);
    const int ct = c->set.check_termination;
    a.adaptive_interval = c->set.adaptive_rho_interval ? c->set.adaptive_rho_interval : (ct ? 4 * ct : 100);
    a.X = X; a.U = U; a.yref = yref;
    a.q_out = c->d_q; a.u_out = c->d_u;
    a.xs = (double *)c->d_xs; a.zs = (double *)c->d_zs; a.ys = (double *)c->d_ys; a.rhos = (double *)c->d_rhos;
    a.warm = c->set.warm_start;
    a.fresh = c->fresh;
    a.x = c->d_x; a.y = c->d_y; a.status = c->d_status; a.iter = c->d_iter; a.rho_out = c->d_rho;
    const char *stp = debug_hook("MPCQ_MIMO_STAMPS");  // per-QP stage stamps
    if (stp && *stp) {
        if (!c->d_stamps && hipMalloc((void **)&c->d_stamps, 8 * 8 * (size_t)a.batch) != hipSuccess)
            return fail(MPCQ_ERR_HIP, "hipMalloc failed (stamps)");
        a.stamps = c->d_stamps;
    }
    hipStream_t s = (hipStream_t)stream;
    const int lr = mpcq_internal_mimo_solve_launch(&a, s);
    if (lr) return fail(lr == -1 ? MPCQ_ERR_ARG : MPCQ_ERR_HIP, "mimo solve launch failed");
    if (stp && *stp) {
        std::vector<long long> h(8 * (size_t)a.batch);
        HIPCHK(hipMemcpyAsync(h.data(), c->d_stamps, 8 * h.size(), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (FILE *f = std::fopen(stp, "wb")) {
            std::fwrite(h.data(), 8, h.size(), f);
            std::fclose(f);
        }
    }
    c->last = s;
    c->fresh = false;
    return MPCQ_OK;
}

}  // extern "C"
