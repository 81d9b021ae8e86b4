// solvempc_amd/csrc/mpcq_tile.h — the hot path for a shared plant: batched OSQP-v0.6 ADMM with the
// per-iteration matrix products on the gfx950 matrix cores.
//
// Replaces osqp_solve behind OsqpEigen::Solver::solve (ModelPredictiveControlAPI.cpp:102) with the
// per-step updates around it (updateGradient :96, updateUpperBound :99, getSolution :105; in the MPC
// front end setF :372-375, setUpperBound :360-369 and U += x0 :105), exactly as mpcq_admm.hip's
// lane kernel does, for contexts whose QPs share one (P, A) (the reference controller replicated
// over many states, BASELINE config 2).
//
// Mapping (MI355X-first): 16 QPs per wave.  With a shared plant the ADMM products of a wave are
// GEMMs: xi = sigma W'W X' + B' Wz over the 16 columns X' (n x 16), Wz (m x 16), and zt = B Eta.
// They run as v_mfma_{f32,f64}_16x16x4 with the plant images in LDS (one copy per 256-thread
// workgroup, read with 16-B ds_reads) as the A operand and the iterates as the B operand.  The
// accumulator layout of one MFMA is the B-operand layout of the next (mpcq_internal.h TileLayout):
// iterates never leave VGPRs and never cross lanes except in the residual reductions every
// check_termination iterations (4-lane groups, __shfl_xor 16/32).  The element-wise part (x/z
// relaxation, projection onto [l,u], dual update) runs on the VALU beside the matrix pipe.
//
// Phases: a launch runs its QPs until they terminate or reach a.stop_iter (a multiple of
// check_termination); QPs still running are saved (x', z, y, rho, iteration) and appended to
// a.list_out, and the next launch packs them densely into waves, so a wave never carries finished
// columns for long.  A QP's arithmetic does not depend on which wave or phase runs it.
#pragma once
#include "mpcq_internal.h"

#include <cstdlib>
#include <type_traits>

namespace mpcq {

template <typename T> struct Mf;
template <> struct Mf<float> {
    typedef float acc __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc mma(float a, float b, acc c)
    {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
};
template <> struct Mf<double> {
    typedef double acc __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc mma(double a, double b, acc c)
    {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
};

template <typename T> __device__ __forceinline__ T tt_fma(T a, T b, T c);
template <> __device__ __forceinline__ float tt_fma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
template <> __device__ __forceinline__ double tt_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
template <typename T> __device__ __forceinline__ T tt_abs(T a) { return a < T(0) ? -a : a; }
template <typename T> __device__ __forceinline__ T tt_max(T a, T b) { return a > b ? a : b; }
template <typename T> __device__ __forceinline__ T tt_min(T a, T b) { return a < b ? a : b; }
// max(m, |x|) for the infinity norms (one v_max with an |.| source modifier; equals OSQP's
// c_max(m, c_absval(x)) for every non-NaN x).
template <typename T> __device__ __forceinline__ T nrm(T m, T x) { return __builtin_fmax(m, __builtin_fabs(x)); }

// Reductions over the 4 lanes (groups) of one QP column (lanes c, c+16, c+32, c+48) with the gfx950
// lane-swap instructions (v_permlane16_swap / v_permlane32_swap: VALU, no LDS round trip).  After a
// swap of v with itself, {r[0], r[1]} = {own value, partner's value} in some order, so a symmetric
// op of the pair gives the same, bit-identical result on all lanes of the column.
template <typename F>
__device__ __forceinline__ unsigned swap_combine(unsigned v, F op)
{
    auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = op(r[0], r[1]);
    auto t = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return op(t[0], t[1]);
}
template <typename T, typename F> __device__ __forceinline__ T col_reduce(T v, F op);
template <typename F> __device__ __forceinline__ float col_reduce(float v, F op)
{
    return __uint_as_float(swap_combine(__float_as_uint(v), [&](unsigned a, unsigned b) {
        return __float_as_uint(op(__uint_as_float(a), __uint_as_float(b)));
    }));
}
template <typename F> __device__ __forceinline__ double col_reduce(double v, F op)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
    auto r = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    auto mk = [](unsigned l, unsigned hh) { return __longlong_as_double((long long)(((unsigned long long)hh << 32) | l)); };
    double w = op(mk(r[0], h[0]), mk(r[1], h[1]));
    const unsigned long long u2 = (unsigned long long)__double_as_longlong(w);
    lo = (unsigned)u2;
    hi = (unsigned)(u2 >> 32);
    auto r2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return op(mk(r2[0], h2[0]), mk(r2[1], h2[1]));
}
template <typename T> __device__ __forceinline__ T col_max(T v)
{
    return col_reduce(v, [](T a, T b) { return __builtin_fmax(a, b); });
}
template <typename T> __device__ __forceinline__ T col_sum(T v)
{
    return col_reduce(v, [](T a, T b) { return a + b; });
}
__device__ __forceinline__ int col_or(int v)
{
    return (int)swap_combine((unsigned)v, [](unsigned a, unsigned b) { return a | b; });
}
__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0ull; }
__device__ __forceinline__ bool wave_all(bool p) { return __ballot(!p) == 0ull; }

// Hide a pointer's provenance from LICM: the images are re-read from LDS in every phase of every
// iteration instead of being hoisted into (and spilling) registers.
// An opaque copy of a per-lane index: addresses derived from it are recomputed where they are used
// (cold paths) instead of being kept live, as 64-bit VGPR pairs, across the hot loop.
__device__ __forceinline__ int opaque(int v)
{
    asm volatile("" : "+v"(v));
    return v;
}

template <typename P> __device__ __forceinline__ P fresh_ptr(P p)
{
    int zero;
    asm volatile("s_mov_b32 %0, 0" : "=s"(zero));
    return p + zero;
}

// y[0 .. 4 NTO) = init + M x over KS k-steps, M an LDS image with KSP padded k-steps.  All the
// operands of the product are read first (16-B ds_reads, one counted wait), then the NTO independent
// accumulator chains are interleaved k-step by k-step so that no MFMA waits on its predecessor's
// result (16x16x4: 32-cycle issue, 40-cycle dependent latency).
template <typename T, int NTO, int KS, int KSP, int XN>
__device__ __forceinline__ void tile_mv(const T *__restrict__ im, const T (&x)[XN], T (&y)[4 * NTO], int lane,
                                        const T *init)
{
    using A = typename Mf<T>::acc;
    constexpr int VEC = 16 / sizeof(T);
    constexpr int NG = (KS + VEC - 1) / VEC;
    typedef T vec __attribute__((ext_vector_type(VEC)));
    im = fresh_ptr(im);
    vec opnd[NTO][NG];
#pragma unroll
    for (int t = 0; t < NTO; t++)
#pragma unroll
        for (int q = 0; q < NG; q++) opnd[t][q] = *(const vec *)(im + TileLayout::at(KSP, VEC, t, q * VEC, lane));
    A acc[NTO];
#pragma unroll
    for (int t = 0; t < NTO; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) acc[t][r] = init ? init[4 * t + r] : T(0);
#pragma unroll
    for (int s = 0; s < KS; s++)
#pragma unroll
        for (int t = 0; t < NTO; t++) acc[t] = Mf<T>::mma(opnd[t][s / VEC][s % VEC], x[s], acc[t]);
#pragma unroll
    for (int t = 0; t < NTO; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) y[4 * t + r] = acc[t][r];
}

// OCC: waves per SIMD the register allocation is held to (256-thread workgroups).
template <typename T, int KN, int KM, bool ALL_INEQ, bool LFREE, int OCC>
__global__ __launch_bounds__(256, OCC) void admm_tile_kernel(AdmmArgs<T> a)
{
    constexpr int VEC = 16 / sizeof(T);
    constexpr TileLayout L = TileLayout::make(KN, KM, VEC);
    constexpr int NT = L.NT, MT = L.MT, KNP = L.KNP, KMP = L.KMP;
    constexpr int NS = 4 * NT, MS = 4 * MT;  // registers per n- / m-vector
    constexpr int is32 = sizeof(T) == 4;
    (void)is32;
    constexpr int NCP = 16 * NT, MCP = 16 * MT;  // padded row counts (== ctx nc, mc)
    __shared__ __attribute__((aligned(16))) T img[L.total];
    __shared__ T rowv[3 * NCP + 2 * MCP];        // lam, D, Dinv | E, Einv of the plant
    T *const s_lam = rowv, *const s_D = rowv + NCP, *const s_Dinv = rowv + 2 * NCP;
    T *const s_E = rowv + 3 * NCP, *const s_Einv = rowv + 3 * NCP + MCP;
    const int count = a.count_in ? *a.count_in : a.batch;
    if (blockIdx.x * 64 >= count) return;  // whole workgroup idle in this phase (uniform)
    for (int i = threadIdx.x; i < NCP; i += 256) {
        s_lam[i] = a.ops.lam[i];
        s_D[i] = a.ops.D[i];
        s_Dinv[i] = a.ops.Dinv[i];
    }
    for (int i = threadIdx.x; i < MCP; i += 256) {
        s_E[i] = a.ops.E[i];
        s_Einv[i] = a.ops.Einv[i];
    }

    // ---- plant images -> LDS (16 B per thread per step)
    {
        typedef T vec __attribute__((ext_vector_type(VEC)));
        const vec *src = (const vec *)a.img;
        vec *dst = (vec *)img;
        for (int i = threadIdx.x; i < (int)(L.total / VEC); i += 256) dst[i] = src[i];
    }
    __syncthreads();  // the only barrier: waves are independent from here on

    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int wave_slot = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
    if (wave_slot >= count) return;
    const bool valid = wave_slot + c < count;
    const int b_ = valid ? (a.list_in ? a.list_in[wave_slot + c] : wave_slot + c) : 0;
    int b = b_;
    const int n = a.n, m = a.m;
    const int ncs = 4 * NT * 4, mcs = 4 * MT * 4;  // state row strides (ctx nc = 16 NT, mc = 16 MT)
    const PlantOps<T> op = a.ops;                  // shared plant: block 0
    const int *ctype = a.ctype;
    const SolverSettings &st = a.st;
    const bool scaled_term = st.scaled_termination != 0;
    const double c64 = (double)op.cs[0];

    // ---- per-QP data (element v = 4 s + g of this lane's QP column)
    double Xv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double Uv = 0.0;
    if (a.mpc) {
#pragma unroll
        for (int t = 0; t < 8; t++)
            if (t < a.nx) Xv[t] = a.X[(size_t)b * a.nx + t];
    }
    if (a.mpc_u) Uv = a.U[b];
    T qh[NS];  // q^ = c D q (osqp_update_lin_cost), kept for the dual residual
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const int v = 4 * s + g;
        double qk = 0.0;
        if (s < KN && v < n) {
            if (a.mpc) {  // setF (:372-375): q = Fx X + Fu U + Fr ref
                const double *fx = a.Fx + (size_t)v * a.nx;
                const double *fr = a.Fr + (size_t)v * n;
                double s0 = 0.0, s2 = 0.0;
#pragma unroll
                for (int t = 0; t < 8; t++)
                    if (t < a.nx) s0 += fx[t] * Xv[t];
                const double s1 = a.Fu[v] * Uv;
                for (int t = 0; t < n; t++) s2 += fr[t] * a.xref;
                qk = s0 + s1 + s2;
                if (valid) a.q_out[(size_t)b * n + v] = qk;
            } else {
                qk = a.q[(size_t)b * n + v];
            }
        }
        qh[s] = s < KN ? (T)((qk * (double)op.D[s < KN ? v : 0]) * c64) : T(0);  // osqp_update_lin_cost
    }
    int bad = 0, tchg = 0;
    T uh[MS], lh[LFREE ? 1 : MS], rs[ALL_INEQ ? 1 : MS];
#pragma unroll
    for (int s = 0; s < MS; s++) {
        const int v = 4 * s + g;
        double up = kInfty, lo = -kInfty;
        if (s < KM && v < m) {
            if (a.mpc) {  // setUpperBound (:360-369) + :99: u = W0 + Sbar X + Ku U
                const double *sb = a.Sbar + (size_t)v * a.nx;
                double sx = 0.0;
#pragma unroll
                for (int t = 0; t < 8; t++)
                    if (t < a.nx) sx += sb[t] * Xv[t];
                up = a.W0[v] + sx + a.Ku[v] * Uv;
                if (valid) a.u_out[(size_t)b * m + v] = up;
            } else {
                up = a.u[(size_t)b * m + v];
            }
            lo = a.l[(a.l_shared ? 0 : (size_t)b * m) + v];
            const double e = (double)op.E[v];  // osqp_update_bounds: u^ = E u, l^ = E l
            up *= e;
            lo *= e;
            if (up < lo) bad = 1;
            const int ty = (lo < -kInfty * kMinScaling && up > kInfty * kMinScaling) ? -1 : (up - lo < kRhoTol ? 1 : 0);
            if (ty != ctype[v]) tchg = 1;
            if (LFREE && !((T)lo < T(-kInfty * kMinScaling))) tchg = 1;
        }
        uh[s] = (T)up;
        if (!LFREE) lh[s] = (T)lo;
        if (!ALL_INEQ) rs[s] = (s < KM && v < m) ? (ctype[v] == -1 ? T(-1) : op.rscale[v]) : T(1);
    }
    bad = col_or(bad);
    tchg = col_or(tchg);
    int status = bad ? kInvalidBounds : (tchg ? kTypeChanged : kUnsolved);

    // g = W' q^ (the q-part of the KKT right-hand side in the W-basis)
    T gv[NS];
    tile_mv<T, NT, KN, KNP>(img + L.Wt, qh, gv, lane, (const T *)nullptr);
#pragma unroll
    for (int s = 0; s < NS; s++) gv[s] = s < KN ? -gv[s] : T(0);  // xi starts from -g (padding rows 0)

    // ---- state: x' (W-basis), z, y; rho persists across solves (OSQP)
    T xs[NS], z[MS], y[MS];
    T rho;
    int it = 0;
    const bool load_state = a.resume || (a.warm && !a.fresh);
    if (a.resume) {
        rho = a.rhos[b];
        it = a.it_state[b];
    } else {
        rho = a.fresh ? (T)fmin(fmax(st.rho, kRhoMin), kRhoMax) : a.rhos[b];
    }
#pragma unroll
    for (int s = 0; s < NS; s++) xs[s] = (load_state && s < KN) ? a.xs[(size_t)b * ncs + 4 * s + g] : T(0);
#pragma unroll
    for (int s = 0; s < MS; s++) {
        z[s] = (load_state && s < KM) ? a.zs[(size_t)b * mcs + 4 * s + g] : T(0);
        y[s] = (load_state && s < KM) ? a.ys[(size_t)b * mcs + 4 * s + g] : T(0);
    }
    it = __builtin_amdgcn_readfirstlane(it);  // lane 0 is always a live column; a phase shares `it`
    T rinv = T(1) / rho;
    T dk[NS];
    auto set_dk = [&]() {
        const T *lam = fresh_ptr((const T *)s_lam);
#pragma unroll
        for (int s = 0; s < NS; s++) dk[s] = T(1) / (T(1) + rho * lam[4 * s + g]);  // lam padded with 0
    };
    set_dk();

    const T alpha = (T)st.alpha, oma = T(1) - (T)st.alpha;
    const T eps_abs = (T)st.eps_abs, eps_rel = (T)st.eps_rel;
    bool done = !valid;

    // ---- write one QP's results (OSQP store_solution / update_info; warm-start state)
    auto finalize = [&](bool mine) {
        const int b = opaque(b_);
        // x = D W x'  (all lanes run the MFMA; `mine` lanes store)
        T xh[NS];
        tile_mv<T, NT, KN, KNP>(img + L.W, xs, xh, lane, (const T *)nullptr);
        if (!mine) return;
        const bool has_sol = status == kSolved || status == kSolvedInaccurate || status == kMaxIterReached;
        const double cinv64 = (double)op.cs[1];
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int v = 4 * s + g;
            if (s < KN && v < n) {
                const double xv = has_sol ? (double)xh[s] * (double)s_D[v] : __builtin_nan("");
                if (a.x) a.x[(size_t)b * n + v] = xv;
                if (v == 0 && a.mpc_u && status == kSolved) a.U[b] = a.U[b] + xv;  // U += x(0)  (:105)
            }
        }
#pragma unroll
        for (int s = 0; s < MS; s++) {
            const int v = 4 * s + g;
            if (s < KM && v < m && a.y)
                a.y[(size_t)b * m + v] = has_sol ? ((double)y[s] * (double)s_E[v]) * cinv64 : __builtin_nan("");
        }
        const bool keep = has_sol || status == kInvalidBounds || status == kTypeChanged;
#pragma unroll
        for (int s = 0; s < NS; s++)
            if (s < KN) a.xs[(size_t)b * ncs + 4 * s + g] = keep ? xs[s] : T(0);
#pragma unroll
        for (int s = 0; s < MS; s++)
            if (s < KM) {
                a.zs[(size_t)b * mcs + 4 * s + g] = keep ? z[s] : T(0);
                a.ys[(size_t)b * mcs + 4 * s + g] = keep ? y[s] : T(0);
            }
        if (g == 0) {
            a.rhos[b] = rho;
            a.status[b] = status;
            a.iter[b] = it;
            a.rho_out[b] = (double)rho;
        }
    };

    if (wave_any(valid && status != kUnsolved)) {
        const bool mine = valid && status != kUnsolved;
        finalize(mine);
        done = done || mine;
    }

    const int ct = st.check_termination;
    const int ai = (st.adaptive_rho && a.adaptive_interval) ? a.adaptive_interval : 0;
    const int stop = a.stop_iter;
    int next_check = ct ? (it / ct + 1) * ct : -1;  // uniform; no integer division in the loop
    int next_adapt = ai ? (it / ai + 1) * ai : -1;
    while (!wave_all(done)) {
        it++;
        const bool at_check = it == next_check;
        const bool at_adapt = it == next_adapt;
        if (at_check) next_check += ct;
        if (at_adapt) next_adapt += ai;
        const bool last = it == st.max_iter;
        const bool info = at_check || at_adapt || last || it == stop;

        // ---- one ADMM iteration; the check iterations also keep delta_x', delta_y (OSQP's
        // delta_x / delta_y, for the infeasibility certificates)
        T dx[NS], dy[MS];
        auto iterate = [&](auto with_delta) {
            constexpr bool DELTA = decltype(with_delta)::value;
            // xi = -g + sigma W'W x' + B' w,   w_j = rho_j z_j - y_j   (w reuses the zt registers)
            T wz[MS];
#pragma unroll
            for (int s = 0; s < MS; s++) {
                T rj = rho;
                if (!ALL_INEQ) rj = rs[s] < T(0) ? T(kRhoMin) : rho * rs[s];
                wz[s] = s < KM ? tt_fma(rj, z[s], -y[s]) : T(0);
            }
            T xi[NS];
            tile_mv<T, NT, KN, KNP>(img + L.S, xs, xi, lane, gv);   // xi = -g + S x'
            tile_mv<T, NT, KM, KMP>(img + L.Bt, wz, xi, lane, xi);  //    + B' w
            // eta = xi / (1 + rho lambda) ; x' = alpha eta + (1 - alpha) x'
#pragma unroll
            for (int s = 0; s < KN; s++) {  // registers s >= KN are padding rows: x' stays 0 there
                xi[s] = xi[s] * dk[s];
                const T xn = tt_fma(alpha, xi[s], oma * xs[s]);
                if (DELTA) dx[s] = xn - xs[s];
                xs[s] = xn;
            }
            // z~ = B eta ; relaxation ; projection ; dual update
            tile_mv<T, MT, KN, KNP>(img + L.B, xi, wz, lane, (const T *)nullptr);
#pragma unroll
            for (int s = 0; s < KM; s++) {
                T rj = rho, rij = rinv;
                if (!ALL_INEQ) {
                    rj = rs[s] < T(0) ? T(kRhoMin) : rho * rs[s];
                    rij = T(1) / rj;
                }
                const T v = tt_fma(alpha, wz[s], oma * z[s]);
                T zn = tt_fma(rij, y[s], v);
                if (!LFREE) zn = __builtin_fmax(zn, lh[s]);  // == OSQP's c_max/c_min, NaN included
                zn = __builtin_fmin(zn, uh[s]);
                if (DELTA) dy[s] = rj * (v - zn);  // OSQP delta_y (certificates only)
                y[s] = tt_fma(rj, v - zn, y[s]);
                z[s] = zn;
            }
        };
        if (!info) {
            iterate(std::false_type{});
            continue;
        }
        iterate(std::true_type{});
#pragma unroll
        for (int s = KM; s < MS; s++) dy[s] = T(0);

        // ---- update_info: residuals in the scaled space (reported unscaled), 4-lane reductions
        T ax_z = 0, ax_zs = 0, zn_s = 0, zn_r = 0, axn_s = 0, axn_r = 0;
        {
            T ax[MS];
            tile_mv<T, MT, KN, KNP>(img + L.B, xs, ax, lane, (const T *)nullptr);
            const T *Einv = fresh_ptr((const T *)s_Einv);
#pragma unroll
            for (int s = 0; s < KM; s++) {
                const T r = ax[s] - z[s];
                const T ei = Einv[4 * s + g];
                ax_z = nrm(ax_z, r);
                ax_zs = nrm(ax_zs, ei * r);
                zn_r = nrm(zn_r, z[s]);
                zn_s = nrm(zn_s, ei * z[s]);
                axn_r = nrm(axn_r, ax[s]);
                axn_s = nrm(axn_s, ei * ax[s]);
            }
        }
        T dr_r = 0, dr_s = 0, qn_r = 0, qn_s = 0, atyn_r = 0, atyn_s = 0, pxn_r = 0, pxn_s = 0;
        {
            T px[NS], aty[NS];
            tile_mv<T, NT, KN, KNP>(img + L.PW, xs, px, lane, (const T *)nullptr);
            tile_mv<T, NT, KM, KMP>(img + L.AhT, y, aty, lane, (const T *)nullptr);
            const T *Dinv = fresh_ptr((const T *)s_Dinv);
#pragma unroll
            for (int s = 0; s < KN; s++) {
                const T qhs = qh[s];
                const T r = (qhs + px[s]) + aty[s];
                const T di = Dinv[4 * s + g];
                dr_r = nrm(dr_r, r);
                dr_s = nrm(dr_s, di * r);
                qn_r = nrm(qn_r, qhs);
                qn_s = nrm(qn_s, di * qhs);
                atyn_r = nrm(atyn_r, aty[s]);
                atyn_s = nrm(atyn_s, di * aty[s]);
                pxn_r = nrm(pxn_r, px[s]);
                pxn_s = nrm(pxn_s, di * px[s]);
            }
        }
        ax_z = col_max(ax_z); ax_zs = col_max(ax_zs); zn_s = col_max(zn_s); zn_r = col_max(zn_r);
        axn_s = col_max(axn_s); axn_r = col_max(axn_r);
        dr_r = col_max(dr_r); dr_s = col_max(dr_s); qn_r = col_max(qn_r); qn_s = col_max(qn_s);
        atyn_r = col_max(atyn_r); atyn_s = col_max(atyn_s); pxn_r = col_max(pxn_r); pxn_s = col_max(pxn_s);
        const T cinv = op.cs[1];
        const T pri_res = scaled_term ? ax_z : ax_zs;
        const T dua_res = scaled_term ? dr_r : cinv * dr_s;

        // OSQP is_primal_infeasible on delta_y = dy (this iteration's dual step).
        auto primal_infeasible = [&](T eps, bool need) -> bool {
            T d[MS];
            T ndy = 0, lhs = 0;
            const T *E = fresh_ptr((const T *)s_E);
#pragma unroll
            for (int s = 0; s < MS; s++) {
                if (s >= KM) { d[s] = T(0); continue; }
                T dd = dy[s];
                const T up = uh[s], lo = LFREE ? T(-kInfty) : lh[s];
                const bool uinf = up > T(kInfty * kMinScaling), linf = lo < T(-kInfty * kMinScaling);
                if (uinf) dd = linf ? T(0) : tt_min(dd, T(0));
                else if (linf) dd = tt_max(dd, T(0));
                d[s] = dd;
                ndy = nrm(ndy, scaled_term ? dd : E[4 * s + g] * dd);
                if (up < T(kInfty * kMinScaling)) lhs += up * tt_max(dd, T(0));
                if (lo > T(-kInfty * kMinScaling)) lhs += lo * tt_min(dd, T(0));
            }
            ndy = col_max(ndy);
            lhs = col_sum(lhs);
            const bool cand = need && ndy > T(kDivisionTol) && lhs < eps * ndy;
            if (!wave_any(cand)) return false;
            T atd[NS];
            tile_mv<T, NT, KM, KMP>(img + L.AhT, d, atd, lane, (const T *)nullptr);
            const T *Dinv = fresh_ptr((const T *)s_Dinv);
            T nat = 0;
#pragma unroll
            for (int s = 0; s < KN; s++) nat = nrm(nat, scaled_term ? atd[s] : Dinv[4 * s + g] * atd[s]);
            nat = col_max(nat);
            return cand && nat < eps * ndy;
        };
        // OSQP is_dual_infeasible on delta_x^ = W dx.
        auto dual_infeasible = [&](T eps, bool need) -> bool {
            T qdx = 0;  // q^' dx^ = (W' q^)' dx' = -gv' dx'
#pragma unroll
            for (int s = 0; s < KN; s++) qdx = tt_fma(-gv[s], dx[s], qdx);
            qdx = col_sum(qdx);
            bool cand = need && qdx < T(0);
            if (!wave_any(cand)) return false;
            T t1[NS];
            tile_mv<T, NT, KN, KNP>(img + L.W, dx, t1, lane, (const T *)nullptr);
            const T *D = fresh_ptr((const T *)s_D);
            T ndx = 0;
#pragma unroll
            for (int s = 0; s < KN; s++) ndx = nrm(ndx, scaled_term ? t1[s] : D[4 * s + g] * t1[s]);
            ndx = col_max(ndx);
            const T cs = scaled_term ? T(1) : op.cs[0];
            cand = cand && ndx > T(kDivisionTol) && qdx < -cs * eps * ndx;
            if (!wave_any(cand)) return false;
            tile_mv<T, NT, KN, KNP>(img + L.PW, dx, t1, lane, (const T *)nullptr);
            const T *Dinv = fresh_ptr((const T *)s_Dinv);
            T npdx = 0;
#pragma unroll
            for (int s = 0; s < KN; s++) npdx = nrm(npdx, scaled_term ? t1[s] : Dinv[4 * s + g] * t1[s]);
            npdx = col_max(npdx);
            cand = cand && npdx < cs * eps * ndx;
            if (!wave_any(cand)) return false;
            T adx[MS];
            tile_mv<T, MT, KN, KNP>(img + L.B, dx, adx, lane, (const T *)nullptr);
            const T *Einv = fresh_ptr((const T *)s_Einv);
            int viol = 0;
#pragma unroll
            for (int s = 0; s < KM; s++) {
                const T sv = scaled_term ? adx[s] : Einv[4 * s + g] * adx[s];
                const T up = uh[s], lo = LFREE ? T(-kInfty) : lh[s];
                if ((up < T(kInfty * kMinScaling) && sv > eps * ndx) || (lo > T(-kInfty * kMinScaling) && sv < -eps * ndx))
                    viol = 1;
            }
            viol = col_or(viol);
            return cand && !viol;
        };
        // check_termination(approximate) — OSQP auxil.c; returns the new status (kUnsolved: go on)
        auto check_termination = [&](bool approx, bool need) -> int {
            const T mul = approx ? T(10) : T(1);
            const bool noncvx = pri_res > T(kInfty) || dua_res > T(kInfty);
            need = need && !noncvx;  // every lane runs the (uniform) certificate code below
            const T ea = eps_abs * mul, er = eps_rel * mul;
            bool prim_ok = (m == 0), dual_ok = false;
            bool need_p = false;
            if (m > 0) {
                const T ep = ea + er * (scaled_term ? tt_max(zn_r, axn_r) : tt_max(zn_s, axn_s));
                prim_ok = pri_res < ep;
                need_p = !prim_ok;
            }
            const bool prim_inf = primal_infeasible((T)st.eps_prim_inf * mul, need && need_p);
            const T ed = ea + er * (scaled_term ? tt_max(tt_max(qn_r, atyn_r), pxn_r)
                                                : cinv * tt_max(tt_max(qn_s, atyn_s), pxn_s));
            dual_ok = dua_res < ed;
            const bool dual_inf = dual_infeasible((T)st.eps_dual_inf * mul, need && !dual_ok);
            if (noncvx) return kNonCvx;
            if (prim_ok && dual_ok) return approx ? kSolvedInaccurate : kSolved;
            if (prim_inf) return approx ? kPrimalInfeasibleInaccurate : kPrimalInfeasible;
            if (dual_inf) return approx ? kDualInfeasibleInaccurate : kDualInfeasible;
            return kUnsolved;
        };

        bool term = done;  // finished (or dead) columns ignore everything below
        if (at_check) {
            const int s0 = check_termination(false, !term);
            if (!term && s0 != kUnsolved) { status = s0; term = true; }
        }
        if (at_adapt && !term) {  // adapt_rho / compute_rho_estimate (scaled-space norms)
            const T pr = ax_z / (tt_max(zn_r, axn_r) + T(kDivisionTol));
            const T dn = tt_max(tt_max(qn_r, atyn_r), pxn_r);
            const T du = dr_r / (dn + T(kDivisionTol));
            T rn = rho * (T)sqrt((double)(pr / (du + T(kDivisionTol))));
            rn = tt_min(tt_max(rn, T(kRhoMin)), T(kRhoMax));
            if (rn > rho * (T)st.adaptive_rho_tolerance || rn < rho / (T)st.adaptive_rho_tolerance) {
                rho = tt_min(tt_max(rn, T(kRhoMin)), T(kRhoMax));
                rinv = T(1) / rho;
            }
        }
        if (at_adapt) set_dk();  // uniform; unchanged rho gives the same dk bit for bit
        if (last) {  // after the ADMM loop (osqp_solve)
            const int s1 = at_check ? kUnsolved : check_termination(false, !term);
            if (!term && s1 != kUnsolved) { status = s1; term = true; }
            const int s2 = check_termination(true, !term);
            if (!term) { status = s2 != kUnsolved ? s2 : kMaxIterReached; term = true; }
        }
        const bool newly = term && !done;
        if (wave_any(newly)) finalize(newly);
        done = term;
        if (it == stop && !wave_all(done)) {
            // phase boundary: save the running QPs and queue them for the next launch
            const bool run = !done;
            const int b = opaque(b_);
            if (run) {
#pragma unroll
                for (int s = 0; s < NS; s++)
                    if (s < KN) a.xs[(size_t)b * ncs + 4 * s + g] = xs[s];
#pragma unroll
                for (int s = 0; s < MS; s++)
                    if (s < KM) {
                        a.zs[(size_t)b * mcs + 4 * s + g] = z[s];
                        a.ys[(size_t)b * mcs + 4 * s + g] = y[s];
                    }
                if (g == 0) {
                    a.rhos[b] = rho;
                    a.it_state[b] = it;
                }
            }
            const unsigned long long mask = __ballot(run && g == 0);
            int base = 0;
            if (lane == 0) base = atomicAdd(a.count_out, __popcll(mask));
            base = __shfl(base, 0);
            if (run && g == 0) a.list_out[base + __popcll(mask & ((1ull << lane) - 1ull))] = b;
            break;
        }
    }
}

// occ: 0 = default for the shape/type, else a requested register budget (3 or 4 waves/SIMD) for
// the f32 fast variant (benchmark A/B hook).
template <typename T, int KN, int KM>
int tile_launch(const AdmmArgs<T> &a, int occ, hipStream_t s)
{
    const dim3 grid((a.batch + 63) / 64), block(256);
    if (a.all_ineq && a.lower_free) {
        if constexpr (sizeof(T) == 8)
            hipLaunchKernelGGL((admm_tile_kernel<T, KN, KM, true, true, 2>), grid, block, 0, s, a);
        else if (occ == 4)
            hipLaunchKernelGGL((admm_tile_kernel<T, KN, KM, true, true, 4>), grid, block, 0, s, a);
        else  // default: 3 waves/SIMD — the whole iteration fits in registers (no spills)
            hipLaunchKernelGGL((admm_tile_kernel<T, KN, KM, true, true, 3>), grid, block, 0, s, a);
    } else {
        hipLaunchKernelGGL((admm_tile_kernel<T, KN, KM, false, false, 2>), grid, block, 0, s, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Compiled (KN, KM) = (ceil(n/4), ceil(m/4)): the reference horizons N = 15 (n 15, m 30) and N = 20
// (n 20, m 40), plus two small shapes for the generic-QP tests.
#define MPCQ_TILE_SHAPES(X) X(1, 1) X(2, 3) X(4, 8) X(5, 10)

template <typename T>
int tile_launch_any(const AdmmArgs<T> &a, int KN, int KM, hipStream_t s)
{
    const char *e = getenv("MPCQ_TILE_OCC");
    const int occ = e ? atoi(e) : 0;
#define MPCQ_TRY(KN_, KM_) if (KN == KN_ && KM == KM_) return tile_launch<T, KN_, KM_>(a, occ, s);
    MPCQ_TILE_SHAPES(MPCQ_TRY)
#undef MPCQ_TRY
    return -1;
}

}  // namespace mpcq
