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
#include "mpcq_plant_sim.h"

#include <cstdlib>
#include <type_traits>

#ifndef MPCQ_REM4
#define MPCQ_REM4 1  // build switch for A/B: 0 runs the remainder tile as a full 16x16x4 tile
#endif
#ifndef MPCQ_PK
#define MPCQ_PK 1  // build switch for A/B: 0 runs the f32 plain iterations on scalar VALU ops
#endif

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
// IEEE minNum / maxNum / |x| at the operand's own width (__builtin_fmin & co. are the double builtins:
// on float operands they widen, compare in fp64 and narrow back)
__device__ __forceinline__ float tt_fmin(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ double tt_fmin(double a, double b) { return __builtin_fmin(a, b); }
__device__ __forceinline__ float tt_fmax(float a, float b) { return __builtin_fmaxf(a, b); }
__device__ __forceinline__ double tt_fmax(double a, double b) { return __builtin_fmax(a, b); }
__device__ __forceinline__ float tt_fabs(float a) { return __builtin_fabsf(a); }
__device__ __forceinline__ double tt_fabs(double a) { return __builtin_fabs(a); }
// max(m, |x|) for the infinity norms (one v_max with an |.| source modifier; equals OSQP's
// c_max(m, c_absval(x)) for every non-NaN x).
// min for the projection onto u without LLVM's NaN canonicalisation of the operands (a v_max x, x
// per element per iteration): the hardware v_min returns the non-NaN operand, as fmin does.
__device__ __forceinline__ float vmin(float a, float b)
{
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmin(double a, double b)
{
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
template <typename T> __device__ __forceinline__ T nrm(T m, T x) { return tt_fmax(m, tt_fabs(x)); }

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
    return col_reduce(v, [](T a, T b) { return tt_fmax(a, b); });
}
template <typename T> __device__ __forceinline__ T col_sum(T v)
{
    return col_reduce(v, [](T a, T b) { return a + b; });
}
// The values of the other lanes of this lane's column: v of lane group g ^ 1 (v_permlane16_swap pairs
// rows 0-1 and 2-3) and g ^ 2 (v_permlane32_swap pairs rows 0-2 and 1-3); a swap of v with itself
// leaves {own, partner} in even rows / halves and {partner, own} in odd ones.
__device__ __forceinline__ double col_x16(double v, int g)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
    auto r = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const int k = (g & 1) ? 0 : 1;
    return __longlong_as_double((long long)(((unsigned long long)h[k] << 32) | r[k]));
}
__device__ __forceinline__ double col_x32(double v, int g)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
    auto r = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const int k = (g & 2) ? 0 : 1;
    return __longlong_as_double((long long)(((unsigned long long)h[k] << 32) | r[k]));
}
// v of lane group `src` of this column, on every lane of the column (moves only: bit-exact)
__device__ __forceinline__ double col_from(double v, int src, int g)
{
    const double v1 = col_x16(v, g), v2 = col_x32(v, g), v3 = col_x32(v1, g);
    return src == g ? v : (src == (g ^ 1) ? v1 : (src == (g ^ 2) ? v2 : v3));
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

// The 4 x 4 x 1 MFMA's partial sums of the last, 4-row tile (rem_* below) to the tile layout: lane
// (g, c) holds p_i = sum over k = g (mod 4) of row i of the tile, for QP c; row i belongs to lane
// group g = i.  Two lane-swap stages (v_permlane32_swap: lanes 32-63 of the first operand with lanes
// 0-31 of the second; v_permlane16_swap: odd 16-lane rows of the first with even rows of the second)
// sum the four partials of each row into the lanes that keep it.
__device__ __forceinline__ float rem_reduce(const Mf<float>::acc &p)
{
    auto r02 = __builtin_amdgcn_permlane32_swap(__float_as_uint(p[0]), __float_as_uint(p[2]), false, false);
    auto r13 = __builtin_amdgcn_permlane32_swap(__float_as_uint(p[1]), __float_as_uint(p[3]), false, false);
    const float q0 = __uint_as_float(r02[0]) + __uint_as_float(r02[1]);  // rows 0 | 2 (lanes 0-31 | 32-63)
    const float q1 = __uint_as_float(r13[0]) + __uint_as_float(r13[1]);  // rows 1 | 3
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(q0), __float_as_uint(q1), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);                // row g
}

// Optional accumulator init of the products below: a [G][4 NTO] array, or nullptr (a compile-time choice:
// a runtime null test on a private array's address cannot fold -- private address 0 is valid -- and would
// keep the array in scratch memory)
template <typename IT> constexpr bool kHasInit = !std::is_same<IT, std::nullptr_t>::value;
template <typename T, typename IT> __device__ __forceinline__ T init_el(IT p, int gi, int k)
{
    if constexpr (kHasInit<IT>) return p[gi][k];
    else return T(0);
}

// The same product for G independent 16-QP groups of one wave: every A operand read from LDS feeds
// G MFMAs, and the G accumulator chains interleave (more independent work per wave).
// REM (f32, the last tile holds 4 real rows): that tile on v_mfma_f32_4x4x1_16b, its A fragment read
// from the 16x16x4 image's lane (g, 4 (c & 3)) (see reg_mv), then rem_reduce; init added after it.
template <typename T, int G, int NTO, int KS, int KSP, int XN, bool REM = false, typename IT = std::nullptr_t>
__device__ __forceinline__ void tile_mv_g(const T *__restrict__ im, const T (&x)[G][XN], T (&y)[G][4 * NTO],
                                          int lane, IT init)
{
    using A = typename Mf<T>::acc;
    constexpr int VEC = 16 / sizeof(T);
    constexpr int NG = (KS + VEC - 1) / VEC;
    constexpr int NF = REM ? NTO - 1 : NTO;
    static_assert(!REM || std::is_same<T, float>::value, "4x4x1 remainder tile: f32 only");
    typedef T vec __attribute__((ext_vector_type(VEC)));
    im = fresh_ptr(im);
    vec opnd[NTO][NG];
#pragma unroll
    for (int t = 0; t < NTO; t++) {
        const int ln = (REM && t == NF) ? ((lane & 48) | ((lane & 3) << 2)) : lane;
#pragma unroll
        for (int q = 0; q < NG; q++) opnd[t][q] = *(const vec *)(im + TileLayout::at(KSP, VEC, t, q * VEC, ln));
    }
    A acc[G][NTO];
#pragma unroll
    for (int gi = 0; gi < G; gi++)
#pragma unroll
        for (int t = 0; t < NTO; t++)
#pragma unroll
            for (int r = 0; r < 4; r++) acc[gi][t][r] = (kHasInit<IT> && t < NF) ? init_el<T>(init, gi, 4 * t + r) : T(0);
#pragma unroll
    for (int s = 0; s < KS; s++)
#pragma unroll
        for (int t = 0; t < NTO; t++)
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                if constexpr (REM) {
                    if (t == NF) {
                        acc[gi][t] = __builtin_amdgcn_mfma_f32_4x4x1f32(opnd[t][s / VEC][s % VEC], x[gi][s], acc[gi][t], 0, 0, 0);
                        continue;
                    }
                }
                acc[gi][t] = Mf<T>::mma(opnd[t][s / VEC][s % VEC], x[gi][s], acc[gi][t]);
            }
#pragma unroll
    for (int gi = 0; gi < G; gi++)
#pragma unroll
        for (int t = 0; t < NTO; t++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if constexpr (REM) {
                    if (t == NF) {
                        if (r == 0) {
                            const T v = rem_reduce(acc[gi][t]);
                            y[gi][4 * t] = kHasInit<IT> ? v + init_el<T>(init, gi, 4 * t) : v;
                        } else {
                            y[gi][4 * t + r] = T(0);
                        }
                        continue;
                    }
                }
                y[gi][4 * t + r] = acc[gi][t][r];
            }
}

// Products with the A operand held in VGPRs (one f32/f64 register per lane per tile and k-step: the
// 16x16x4 A fragment, lane l = A[16 t + arow(l & 15)][4 s + (l >> 4)]), for the paired hot loop:
// y = init + M1 x1 (+ M2 x2), the NTO x G accumulator chains interleaved k-step by k-step.
// REM (f32, n = 16 (NTO - 1) + 4, e.g. N = 20): the last tile holds 4 real rows, so it runs as
// v_mfma_f32_4x4x1_16b (16 blocks of 4 rows x 4 QPs, one k each: a quarter of a 16x16x4's issue
// cycles) with the A fragment lane (g, c) = A[16 (NTO - 1) + (c & 3)][4 s + g] and the iterate
// register as B operand, then rem_reduce; its init is added after the reduction.
// RMODE (REM only) defers the remainder tile's lane reduction across two products: 1 = leave its
// 4x4x1 partial sums unreduced in rem[] and put init's remainder element (not the product's) into y;
// 2 = start the remainder chain from rem[] (the partials of a mode-1 product), reduce, add init.
template <typename T, int G, int NTO, int KS, int XN, bool TWO, int XN2, bool REM = false, int RMODE = 0,
          typename IT = std::nullptr_t>
__device__ __forceinline__ void reg_mv(const T (&m1)[NTO][KS], const T (&x1)[G][XN], const T (&m2)[NTO][KS],
                                       const T (&x2)[G][XN2], T (&y)[G][4 * NTO], IT init,
                                       typename Mf<T>::acc *rem = nullptr)
{
    using A = typename Mf<T>::acc;
    constexpr int NF = REM ? NTO - 1 : NTO;  // full 16-row tiles
    static_assert(!REM || std::is_same<T, float>::value, "4x4x1 remainder tile: f32 only");
    static_assert(RMODE == 0 || REM, "deferred remainder reduction: remainder tile only");
    A acc[G][NTO];
#pragma unroll
    for (int gi = 0; gi < G; gi++)
#pragma unroll
        for (int t = 0; t < NTO; t++)
#pragma unroll
            for (int r = 0; r < 4; r++)
                acc[gi][t][r] = (kHasInit<IT> && t < NF) ? init_el<T>(init, gi, 4 * t + r)
                                                         : ((RMODE == 2 && t == NF) ? rem[gi][r] : T(0));
    auto step = [&](const T (&m)[NTO][KS], auto &x, int s) {
#pragma unroll
        for (int t = 0; t < NTO; t++)
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                if constexpr (REM) {
                    if (t == NF) {
                        acc[gi][t] = __builtin_amdgcn_mfma_f32_4x4x1f32(m[t][s], x[gi][s], acc[gi][t], 0, 0, 0);
                        continue;
                    }
                }
                acc[gi][t] = Mf<T>::mma(m[t][s], x[gi][s], acc[gi][t]);
            }
    };
#pragma unroll
    for (int s = 0; s < KS; s++) step(m1, x1, s);
    if constexpr (TWO) {
#pragma unroll
        for (int s = 0; s < KS; s++) step(m2, x2, s);
    }
#pragma unroll
    for (int gi = 0; gi < G; gi++)
#pragma unroll
        for (int t = 0; t < NTO; t++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                if constexpr (REM && RMODE == 1) {
                    if (t == NF) {
                        if (r == 0) rem[gi] = acc[gi][t];
                        y[gi][4 * t + r] = (kHasInit<IT> && r == 0) ? init_el<T>(init, gi, 4 * t) : T(0);
                        continue;
                    }
                }
                if constexpr (REM) {
                    if (t == NF) {
                        if (r == 0) {
                            const T v = rem_reduce(acc[gi][t]);
                            y[gi][4 * t] = kHasInit<IT> ? v + init_el<T>(init, gi, 4 * t) : v;
                        } else {
                            y[gi][4 * t + r] = T(0);
                        }
                        continue;
                    }
                }
                y[gi][4 * t + r] = acc[gi][t][r];
            }
}

// G: 16-QP groups per wave; OCC: waves per SIMD the register allocation is held to (256-thread
// workgroups, so one workgroup carries 64 G QPs).
// PAIRED (the condensed-MPC shape, m = 2n, n % 4 == 0, rows n + j = -rows j of A, all inequality
// rows, l = -inf; ModelPredictiveControlAPI.cpp:326-347 builds A = [K0 L; -K0 L]): Ruiz gives rows
// j and n + j the same E, so B = A^ W has B_{n+j} = -B_j exactly.  The hot loop then computes
// z~ for the top half only (z~_{n+j} = -z~_j) and B' w as B~' (w_top - w_bot), and keeps its three
// operators S, B~', B~ (3 NT KN registers) in VGPRs: no LDS traffic between check iterations.
// Element 4 s + g of a half-m vector pairs register s with register s + KN (same lane).
// Debug build hook (MPCQ_DEBUG_HOOKS + MPCQ_TILE_STAMPS): per-wave shader-clock stamps at the stage boundaries of a launch:
// 0 entry, 1 images in LDS, 2 loop entry, 3 phase-boundary save, 4 exit, 5 iteration at exit,
// 6 / 7 s_memrealtime (100 MHz) at entry / exit.
#ifdef MPCQ_DEBUG_HOOKS
#define MPCQ_TSTAMP(k, v)                                                                                  \
    do {                                                                                                   \
        if (a.stamps && (threadIdx.x & 63) == 0) a.stamps[(size_t)(blockIdx.x * WPB + (threadIdx.x >> 6)) * 8 + (k)] = (v); \
    } while (0)
#else
#define MPCQ_TSTAMP(k, v) do { } while (0)
#endif
// WPB: waves per workgroup (4, or 8 so that an image set serves 8 waves and 4 waves/SIMD fit the LDS).
// MIX (T = double, paired loop only): the fp64 kernel with each check interval's first plain iterations in
// fp32 (the fp32 kernel's packed-pair loop on rounded copies of the fp64 state, operators rounded from the
// fp64 images); the last a.mix_r iterations before every info iteration (check, adapt, stop) run in fp64,
// which damps the fp32 stretch's rounding below the north-star tolerance before the termination test,
// adapt_rho and the solution read the state (tools/precision_sim.py).
template <typename T, int KN, int KM, bool ALL_INEQ, bool LFREE, int G, int OCC, bool PAIRED = false, int WPB = 4,
          bool STREAM = false, bool MIX = false>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void admm_tile_kernel(AdmmArgs<T> a)
{
    MPCQ_TSTAMP(0, (long long)__builtin_amdgcn_s_memtime());
    MPCQ_TSTAMP(6, (long long)__builtin_amdgcn_s_memrealtime());
    static_assert(!PAIRED || (KM == 2 * KN && ALL_INEQ && LFREE), "paired loop: m = 2n, inequality rows, l free");
    static_assert(!MIX || (PAIRED && std::is_same<T, double>::value), "mixed: the fp64 paired loop");
    constexpr int VEC = 16 / sizeof(T);
    constexpr TileLayout L = TileLayout::make(KN, KM, VEC, PAIRED);
    // the paired loop reads the paired image set, stored after the generic one (TileLayout)
    constexpr size_t IMG0 = PAIRED ? TileLayout::make(KN, KM, VEC, false).total : 0;
    constexpr int KBT = L.KBT, NBS = L.NBS;  // k-steps of the Bt / AhT images; tiles of [B~; S]
    constexpr int NT = L.NT, MT = L.MT, KNP = L.KNP, KMP = L.KMP;
    constexpr int NS = 4 * NT, MS = 4 * MT;  // registers per n- / m-vector
    constexpr int NCP = 16 * NT, MCP = 16 * MT;  // padded row counts (== ctx nc, mc)
    constexpr int NTH = 64 * WPB;                // threads per workgroup
    constexpr int QPW = 16 * G * WPB;            // QPs per workgroup
    __shared__ __attribute__((aligned(16))) T img[L.total];
    __shared__ T rowv[3 * NCP + 2 * MCP];        // lam, D, Dinv | E, Einv of the plant
    // q^ of each wave's QPs (lane layout): the dual residual of every check iteration reads it here
    // instead of re-reading q (fp64, HBM) under the latency of a loaded memory system
    __shared__ T s_qh[WPB][G * KN][64];
    // stream (STREAM): every column's plant state X (8), U, in LDS rather than in VGPRs held across the
    // solve (the check and refill code of the stream instantiation spilled); all four lanes of a column
    // read and write the same values (one wave: its DS instructions execute in order)
    __shared__ double s_plant[STREAM ? WPB * 16 * 9 : 1];
    T *const s_lam = rowv, *const s_D = rowv + NCP, *const s_Dinv = rowv + 2 * NCP;
    T *const s_E = rowv + 3 * NCP, *const s_Einv = rowv + 3 * NCP + MCP;
    // resumed phase: this workgroup serves list segment `seg` (ListSeg), as its workgroup `blk`
    const bool seglist = a.list_in != nullptr;
    // receding-horizon stream (STREAM, AdmmArgs::sim): every column is one plant that runs all its
    // control steps in this launch; a wave holds a.sim.cpw columns (the rest idle), QPs cpw w ..
    constexpr bool refill = STREAM && G == 1;
    const int seg = blockIdx.x % ListSeg::kShards;
    const int count = seglist ? a.count_in[seg * ListSeg::kStride] : a.batch;  // slots of the list it serves
    const int blk = seglist ? (int)blockIdx.x / ListSeg::kShards : (int)blockIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < ListSeg::kShards) {  // counters no launch of this chain is using
        if (a.zero_cnt) a.zero_cnt[threadIdx.x * ListSeg::kStride] = 0;
        if (a.zero_cnt0) a.zero_cnt0[threadIdx.x * ListSeg::kStride] = 0;
    }
    if (blockIdx.x == 0 && a.ord_zero)  // the order's bin counters, read by its finished sort: the next solve's
        for (int i = threadIdx.x; i < OrderBins::kBins; i += NTH) a.ord_zero[i] = 0;
    if (blk * (refill ? WPB * a.sim.cpw : QPW) >= count) return;  // whole workgroup idle in this phase (uniform)
    const bool ordered = a.ord_list != nullptr && !seglist && !refill;  // phase 0 hardest-first (mpcq_order.hip)
    for (int i = threadIdx.x; i < NCP; i += NTH) {
        s_lam[i] = a.ops.lam[i];
        s_D[i] = a.ops.D[i];
        s_Dinv[i] = a.ops.Dinv[i];
    }
    for (int i = threadIdx.x; i < MCP; i += NTH) {
        s_E[i] = a.ops.E[i];
        s_Einv[i] = a.ops.Einv[i];
    }

    // ---- plant images -> LDS (16 B per thread per step; every load issued before the stores)
    {
        typedef T vec __attribute__((ext_vector_type(VEC)));
        const vec *src = (const vec *)(a.img + IMG0);
        vec *dst = (vec *)img;
        constexpr int NV = (int)(L.total / VEC), PER = (NV + NTH - 1) / NTH;
        vec buf[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int i = threadIdx.x + NTH * k;
            buf[k] = src[i < NV ? i : 0];
        }
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int i = threadIdx.x + NTH * k;
            if (i < NV) dst[i] = buf[k];
        }
    }
    // ---- MPC front-end operators of the plant (setF :372-375, setUpperBound :360-369) -> LDS, fp64:
    // Fx, Sbar rows padded to 8 columns; frr = Fr (xref 1) summed per row in the reference's order.
    constexpr int FE_FX = 0, FE_FU = 8 * NCP, FE_FR = 9 * NCP, FE_SB = 10 * NCP, FE_KU = 10 * NCP + 8 * MCP,
                  FE_W0 = 10 * NCP + 9 * MCP, FE_E = 10 * NCP + 10 * MCP, FE_D = 10 * NCP + 11 * MCP,
                  FE_TOT = 11 * NCP + 11 * MCP;
    __shared__ double fe[FE_TOT];
    // (an MPC step: every phase builds q, u from X, U; phase 0 also publishes them or saves X, U)
    const bool fe_on = a.X != nullptr;
    {
        const int n = a.n, m = a.m, nx = fe_on ? a.nx : 0;
        for (int i = threadIdx.x; i < MCP; i += NTH) fe[FE_E + i] = i < m ? (double)a.ops.E[i] : 0.0;
        for (int i = threadIdx.x; i < NCP; i += NTH) fe[FE_D + i] = i < n ? (double)a.ops.D[i] : 0.0;
        if (fe_on) {
            for (int i = threadIdx.x; i < 8 * NCP; i += NTH) {
                const int v = i >> 3, t = i & 7;
                fe[FE_FX + i] = (v < n && t < nx) ? a.Fx[(size_t)v * nx + t] : 0.0;
            }
            for (int i = threadIdx.x; i < 8 * MCP; i += NTH) {
                const int v = i >> 3, t = i & 7;
                fe[FE_SB + i] = (v < m && t < nx) ? a.Sbar[(size_t)v * nx + t] : 0.0;
            }
            for (int i = threadIdx.x; i < NCP; i += NTH) fe[FE_FU + i] = i < n ? a.Fu[i] : 0.0;
            for (int i = threadIdx.x; i < MCP; i += NTH) {
                fe[FE_KU + i] = i < m ? a.Ku[i] : 0.0;
                fe[FE_W0 + i] = i < m ? a.W0[i] : 0.0;
            }
            if (threadIdx.x < n) {  // Fr ref, ref = xref 1 (updateRef :378-380): row sums in order t = 0..n-1
                const int v = threadIdx.x;
                double fr[NCP];
#pragma unroll
                for (int t = 0; t < NCP; t++) fr[t] = a.Fr[(size_t)v * n + (t < n ? t : 0)];
                double s2 = 0.0;
#pragma unroll
                for (int t = 0; t < NCP; t++)
                    if (t < n) s2 += fr[t] * a.xref;
                fe[FE_FR + v] = s2;
            }
        }
    }
    __syncthreads();  // the only barrier: waves are independent from here on
    MPCQ_TSTAMP(1, (long long)__builtin_amdgcn_s_memtime());
    // debug build MPCQ_PRO_PART=p: stamp 5 holds the cycles between prologue marks p-1 and p
#ifdef MPCQ_PRO_PART
    long long t_pro = (long long)__builtin_amdgcn_s_memtime();
#define MPCQ_PRO_MARK(k)                                                                            \
    do {                                                                                            \
        if ((k) == MPCQ_PRO_PART - 1) t_pro = (long long)__builtin_amdgcn_s_memtime();              \
        if ((k) == MPCQ_PRO_PART) MPCQ_TSTAMP(5, (long long)__builtin_amdgcn_s_memtime() - t_pro); \
    } while (0)
#else
#define MPCQ_PRO_MARK(k) do { } while (0)
#endif

    const int lane = threadIdx.x & 63, c = lane & 15;
    constexpr int KNR = PAIRED ? KN : 1, NTR = PAIRED ? NT : 1;
    // f32 paired loop with n = 16 (NT - 1) + 4 (N = 20): the last tile's 4 rows on the 4x4x1 MFMA
    constexpr bool REM4F = PAIRED && KN % 4 == 1 && NT > 1 && MPCQ_REM4;  // (the fp32 loop's remainder tile)
    constexpr bool REM4 = REM4F && std::is_same<T, float>::value;
    const int n = a.n, m = a.m;
    const int ncs = NCP, mcs = MCP;                // state row strides (ctx nc, mc)
    const PlantOps<T> op = a.ops;                  // shared plant: block 0
    const int *ctype = a.ctype;
    const SolverSettings &st = a.st;
    const bool scaled_term = st.scaled_termination != 0;
    const double c64 = (double)op.cs[0];

    // One group of 16 G QPs (column c of group gi: QP b_[gi], live if valid[gi]) through this
    // launch's phase.
    auto run_group = [&](const int (&b0_)[G], const bool (&valid0)[G]) {
    // lane indices re-derived opaquely, so that no lane-dependent address of the body is hoisted
    // and held live (in VGPRs) across the hot loop
    const int lane = opaque((int)threadIdx.x & 63), c = lane & 15, g = lane >> 4;
    int b_[G];        // this lane's QP column (the refill schedule replaces finished ones)
    bool valid[G];
#pragma unroll
    for (int gi = 0; gi < G; gi++) {
        b_[gi] = b0_[gi];
        valid[gi] = valid0[gi];
    }
    const bool resume = a.resume != 0;
    const bool mpc_fe = a.mpc != 0;  // front end: the QP's first phase

    MPCQ_PRO_MARK(10);
    T uh[G][MS], lh[G][LFREE ? 1 : MS];
    T rs[ALL_INEQ ? 1 : MS];
    int status[G];
    T gv[G][NS];                         // W' q^
    T xs[G][NS], z[G][MS], y[G][MS];     // state: x' (W-basis), z, y
    T rho[G], rinv[G];
    int it = 0;
    int cst[G];  // the wave iteration the column's QP started at (its own iteration: it - cst)
    // stream (STREAM): per column, the control steps finished and whether its plant has run them all
    int kst[G];    // the column's control steps finished
    bool over[G];  // the column's plant has run all its steps (or the column is idle)
#pragma unroll
    for (int gi = 0; gi < G; gi++) {
        kst[gi] = 0;
        over[gi] = !valid[gi];
    }
    double *const pst = s_plant + (STREAM ? ((threadIdx.x >> 6) * 16 + c) * 9 : 0);  // stream: X[0..8), U
    // ---- per-QP data of the columns in `fill` (element v = 4 s + g of this lane's QP column), per
    // group: every column at entry, the refilled ones at a check (the others keep their registers and
    // reproduce their W' q^ bit for bit).  Every global load of a group is issued (index clamped into
    // the row, not branched) before any of it is used.
    auto load_cols = [&](const bool (&fill)[G], const bool entry) {
    T qh[G][NS];  // q^ = c D q (osqp_update_lin_cost); kept per wave in LDS (s_qh) for the checks
#pragma unroll
    for (int gi = 0; gi < G; gi++) {
        const int b = b_[gi];
        // this column's QP is (re)loaded: publish its outputs (a stream column: at its last step)
        const bool pub = valid[gi] && fill[gi] && (!refill || kst[gi] + 1 >= a.sim.steps);
        double qk[KN], up[KM], lo[LFREE ? 1 : KM];
        if (fe_on) {  // setF (:372-375) q = Fx X + Fu U + Fr ref;  (:93-99) u = W0 + Sbar X + Ku U
            // (a resumed phase recomputes them: X is read-only and U changes only at a QP's finalize)
            double Xv[8];
            const int nx = a.nx;
            double Uv;
            if (refill && !entry) {  // a stream column's later step: its plant state is in LDS
#pragma unroll
                for (int t = 0; t < 8; t++) Xv[t] = pst[t];
                Uv = pst[8];
            } else {
#pragma unroll
                for (int t = 0; t < 8; t++) Xv[t] = a.X[(size_t)b * nx + (t < nx ? t : 0)];
                Uv = a.U[b];
#pragma unroll
                for (int t = 0; t < 8; t++)
                    if (t >= nx) Xv[t] = 0.0;
                if (refill) {
#pragma unroll
                    for (int t = 0; t < 8; t++) pst[t] = Xv[t];
                    pst[8] = Uv;
                }
            }
#pragma unroll
            for (int s = 0; s < KN; s++) {
                const int v = 4 * s + g;  // < NCP: padded rows of fe are zero
                double s0 = 0.0;
#pragma unroll
                for (int t = 0; t < 8; t++)
                    if (t < nx) s0 += fe[FE_FX + 8 * v + t] * Xv[t];
                const double s1 = fe[FE_FU + v] * Uv;
                qk[s] = s0 + s1 + fe[FE_FR + v];
                if (mpc_fe && a.q_out && pub && v < n) a.q_out[(size_t)b * n + v] = qk[s];
            }
            if (mpc_fe && a.X_save && pub) {  // the step's X, U: q, u on demand (materialize_qu)
                if (refill) {  // (selects: no register index by lane)
                    double x0 = 0.0, x1 = 0.0;
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        x0 = t == g ? Xv[t] : x0;
                        x1 = t == g ? Xv[t + 4] : x1;
                    }
                    if (g < nx) a.X_save[(size_t)b * nx + g] = x0;
                    if (g + 4 < nx) a.X_save[(size_t)b * nx + g + 4] = x1;
                } else {
                    if (g < nx) a.X_save[(size_t)b * nx + g] = a.X[(size_t)b * nx + g];  // (cache-hot reloads:
                    if (g + 4 < nx) a.X_save[(size_t)b * nx + g + 4] = a.X[(size_t)b * nx + g + 4];  // no register index by lane)
                }
                if (g == 0) a.U_save[b] = Uv;
            }
            MPCQ_PRO_MARK(11);
#pragma unroll
            for (int s = 0; s < KM; s++) {
                const int v = 4 * s + g;
                double sx = 0.0;
#pragma unroll
                for (int t = 0; t < 8; t++)
                    if (t < nx) sx += fe[FE_SB + 8 * v + t] * Xv[t];
                up[s] = fe[FE_W0 + v] + sx + fe[FE_KU + v] * Uv;
                if (mpc_fe && a.u_out && pub && v < m) a.u_out[(size_t)b * m + v] = up[s];
            }
            MPCQ_PRO_MARK(12);
        } else {
#pragma unroll
            for (int s = 0; s < KN; s++) {
                const int v = 4 * s + g;
                qk[s] = a.q[(size_t)b * n + (v < n ? v : 0)];
            }
#pragma unroll
            for (int s = 0; s < KM; s++) {
                const int v = 4 * s + g;
                up[s] = a.u[(size_t)b * m + (v < m ? v : 0)];
            }
        }
        if constexpr (!LFREE) {
#pragma unroll
            for (int s = 0; s < KM; s++) {
                const int v = 4 * s + g;
                lo[s] = a.l[(a.l_shared ? 0 : (size_t)b * m) + (v < m ? v : 0)];
            }
        }
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int v = 4 * s + g;
            const int sk = s < KN ? s : 0;
            const T qn = (s < KN && v < n) ? (T)((qk[sk] * fe[FE_D + v]) * c64) : T(0);
            if (fill[gi]) {
                qh[gi][s] = qn;
                if (s < KN) s_qh[threadIdx.x >> 6][gi * KN + sk][lane] = qn;
            } else {
                qh[gi][s] = s < KN ? s_qh[threadIdx.x >> 6][gi * KN + sk][lane] : T(0);
            }
        }
        MPCQ_PRO_MARK(13);
        int bad = 0, tchg = 0;
#pragma unroll
        for (int s = 0; s < MS; s++) {
            const int v = 4 * s + g;
            double uu = kInfty, ll = -kInfty;
            if (s < KM && v < m) {
                const double e = fe[FE_E + v];  // osqp_update_bounds: u^ = E u, l^ = E l
                uu = up[s] * e;
                if constexpr (!LFREE) ll = lo[s] * e;
                if (!resume) {  // a resumed phase's QPs passed these checks in phase 0
                    if (uu < ll) bad = 1;
                    if constexpr (ALL_INEQ && LFREE) {
                        if (uu > kInfty * kMinScaling) tchg = 1;  // a free row: not the setup's type
                    } else {
                        const int ty = (ll < -kInfty * kMinScaling && uu > kInfty * kMinScaling) ? -1
                                                                                             : (uu - ll < kRhoTol ? 1 : 0);
                        if (ty != ctype[v]) tchg = 1;
                    }
                }
            }
            if (fill[gi]) {
                uh[gi][s] = (T)uu;
                if (!LFREE) lh[gi][s] = (T)ll;
            }
            if (!ALL_INEQ && gi == 0 && entry) rs[s] = (s < KM && v < m) ? (ctype[v] == -1 ? T(-1) : op.rscale[v]) : T(1);
        }
        bad = col_or(bad);
        tchg = col_or(tchg);
        if (fill[gi]) status[gi] = bad ? kInvalidBounds : (tchg ? kTypeChanged : kUnsolved);
    }
    MPCQ_PRO_MARK(1);
    MPCQ_PRO_MARK(14);

    // g = W' q^ (the q-part of the KKT right-hand side in the W-basis)
    tile_mv_g<T, G, NT, KN, KNP>(img + L.Wt, qh, gv, lane, nullptr);
#pragma unroll
    for (int gi = 0; gi < G; gi++)
#pragma unroll
        for (int s = 0; s < NS; s++) gv[gi][s] = s < KN ? -gv[gi][s] : T(0);  // xi starts from -g
    MPCQ_PRO_MARK(2);

    // ---- state: x' (W-basis), z, y; rho persists across solves (OSQP)
    const bool fresh = a.fresh && entry;  // (a stream's reset applies to its first step only)
    const bool load_state = resume || (a.warm && !fresh);
#pragma unroll
    for (int gi = 0; gi < G; gi++) {
        if (!fill[gi]) continue;
        if (refill && !entry) {  // a stream column's next step: x', z, y, rho are in its registers
            cst[gi] = it;
            continue;
        }
        const int b = b_[gi];
        if (resume) {
            rho[gi] = a.rhos[b];
            if (gi == 0) it = a.it_state[b];
        } else {
            rho[gi] = fresh ? (T)fmin(fmax(st.rho, kRhoMin), kRhoMax) : a.rhos[b];
        }
#pragma unroll
        for (int s = 0; s < NS; s++) xs[gi][s] = (load_state && s < KN) ? a.xs[(size_t)b * ncs + 4 * s + g] : T(0);
#pragma unroll
        for (int s = 0; s < MS; s++) {
            z[gi][s] = (load_state && s < KM) ? a.zs[(size_t)b * mcs + 4 * s + g] : T(0);
            y[gi][s] = (load_state && s < KM) ? a.ys[(size_t)b * mcs + 4 * s + g] : T(0);
        }
        rinv[gi] = T(1) / rho[gi];
        cst[gi] = it;
    }
    };
    {
        bool all[G];
#pragma unroll
        for (int gi = 0; gi < G; gi++) all[gi] = true;
        load_cols(all, true);
    }
    it = __builtin_amdgcn_readfirstlane(it);  // lane 0 is always a live column; a phase shares `it`
#pragma unroll
    for (int gi = 0; gi < G; gi++) cst[gi] = 0;  // (a resumed phase counts from its QPs' saved `it`)
    MPCQ_PRO_MARK(3);
    T dk[G][NS];
    auto set_dk = [&]() {
        const T *lam = fresh_ptr((const T *)s_lam);
#pragma unroll
        for (int gi = 0; gi < G; gi++)
#pragma unroll
            for (int s = 0; s < NS; s++) dk[gi][s] = T(1) / (T(1) + rho[gi] * lam[4 * s + g]);  // lam padded 0
    };
    set_dk();
    MPCQ_PRO_MARK(4);

    const T alpha = (T)st.alpha, oma = T(1) - (T)st.alpha;
    const T eps_abs = (T)st.eps_abs, eps_rel = (T)st.eps_rel;
    bool done[G];
#pragma unroll
    for (int gi = 0; gi < G; gi++) done[gi] = !valid[gi];

    // ---- write the results of the `mine` QPs (OSQP store_solution / update_info; warm-start state)
    // Uold: U of each column read ahead of time (the info iteration prefetches it, so that U += x(0)
    // does not wait on a global load after the termination test), or null: read it here.
    auto finalize = [&](const bool (&mine)[G], const double *Uold) {
        // x = D W x'  (all lanes run the MFMA; `mine` lanes store)
        T xh[G][NS];
        tile_mv_g<T, G, NT, KN, KNP>(img + L.W, xs, xh, lane, nullptr);
        const double cinv64 = (double)op.cs[1];
#pragma unroll
        for (int gi = 0; gi < G; gi++) {
            if (!mine[gi]) continue;
            const int b = opaque(b_[gi]);
            // (the lane's row offset and the output pointers re-derived here: per-pointer lane addresses are
            // not hoisted out of the finalize and held, as 64-bit VGPR pairs, across the hot loop)
            const int g = opaque((int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u))) >> 4;
            T *const o_xs = fresh_ptr(a.xs), *const o_zs = fresh_ptr(a.zs), *const o_ys = fresh_ptr(a.ys);
            T *const o_rhos = fresh_ptr(a.rhos);
            int *const o_status = fresh_ptr(a.status), *const o_iter = fresh_ptr(a.iter);
            double *const o_rho = fresh_ptr(a.rho_out), *const o_U = fresh_ptr(a.U);
            const int sta = status[gi];
            const bool has_sol = sta == kSolved || sta == kSolvedInaccurate || sta == kMaxIterReached;
            // a stream column between two of its control steps keeps the solver state in registers
            // (exactly what the next step would reload) and publishes only U; its last step writes all
            const bool full = !refill || kst[gi] + 1 >= a.sim.steps;
#pragma unroll
            for (int s = 0; s < NS; s++) {
                const int v = 4 * s + g;
                if (s < KN && v < n) {
                    const double xv = has_sol ? (double)xh[gi][s] * (double)s_D[v] : __builtin_nan("");
                    if (a.x && full) a.x[(size_t)b * n + v] = xv;
                    if (!refill && v == 0 && a.mpc_u && sta == kSolved) o_U[b] = (Uold ? Uold[gi] : o_U[b]) + xv;  // U += x(0)  (:105)
                }
            }
            if (refill) {  // stream: U += x(0) on every lane of the column (x(0): lane group 0, register 0)
                const double x0 = col_from(has_sol ? (double)xh[gi][0] * (double)s_D[0] : 0.0, 0, g);
                const double u1 = (a.mpc_u && sta == kSolved) ? pst[8] + x0 : pst[8];
                pst[8] = u1;
                if (full && g == 0) o_U[b] = u1;
            }
            const bool keep = has_sol || sta == kInvalidBounds || sta == kTypeChanged;
            if (!full) {
                if (!keep) {
#pragma unroll
                    for (int s = 0; s < NS; s++) xs[gi][s] = T(0);
#pragma unroll
                    for (int s = 0; s < MS; s++) z[gi][s] = y[gi][s] = T(0);
                }
                if (g == 0 && a.it_acc) {
                    a.it_acc[b] += it - cst[gi];
                    a.uns_acc[b] += sta != kSolved;
                }
                continue;
            }
#pragma unroll
            for (int s = 0; s < MS; s++) {
                const int v = 4 * s + g;
                if (s < KM && v < m && a.y)
                    a.y[(size_t)b * m + v] = has_sol ? ((double)y[gi][s] * (double)s_E[v]) * cinv64 : __builtin_nan("");
            }
#pragma unroll
            for (int s = 0; s < NS; s++)
                if (s < KN) o_xs[(size_t)b * ncs + 4 * s + g] = keep ? xs[gi][s] : T(0);
#pragma unroll
            for (int s = 0; s < MS; s++)
                if (s < KM) {
                    o_zs[(size_t)b * mcs + 4 * s + g] = keep ? z[gi][s] : T(0);
                    o_ys[(size_t)b * mcs + 4 * s + g] = keep ? y[gi][s] : T(0);
                }
            if (g == 0) {
                o_rhos[b] = rho[gi];
                if (!STREAM && a.info_slot) {  // (ordered single launch: slot = the list entry this column runs)
                    const int col = opaque((int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u))) & 15;
                    const int slot = (blk * WPB + ((int)threadIdx.x >> 6)) * 16 * G + 16 * gi + col;
                    *(int2 *)(fresh_ptr(a.info_slot) + 2 * (size_t)slot) = make_int2(sta, it - cst[gi]);
                } else {
                    o_status[b] = sta;
                    o_iter[b] = it - cst[gi];
                }
                if (a.rho_out) o_rho[b] = (double)rho[gi];  // (null: the fp64 rhos above is reported, mpcq_api.cpp
                                                            // materialize_rho)
                if (a.it_acc) {
                    a.it_acc[b] += it - cst[gi];
                    a.uns_acc[b] += sta != kSolved;
                }
            }
        }
    };
    auto all_done = [&]() {
        bool d = true;
#pragma unroll
        for (int gi = 0; gi < G; gi++) d = d && done[gi];
        return wave_all(d);
    };
    // stream (STREAM), at a check iteration after the finalize: a column whose control step just
    // finished advances its plant, X <- Ad X + Bd U + w (mpcq_plant_sim.h; lane g: components g, g + 4),
    // and, while steps remain, starts the next step's QP in place (front end from the new X and U,
    // warm state from the finalize's stores: the per-step path's arithmetic, bit for bit).  A column
    // never waits for the others of its wave: each runs its own plant's steps.
    auto stream_next = [&]() {
        if constexpr (refill) {
            const int nx = a.nx;
            for (;;) {
                const bool fin = done[0] && !over[0];
                if (!wave_any(fin)) return;
                const int b = b_[0];
                const double *Ad = a.sim.Ad + (a.sim.shared ? 0 : (size_t)b * nx * nx);
                const double *Bd = a.sim.Bd + (a.sim.shared ? 0 : (size_t)b * nx);
                const unsigned long long key = sim_key(a.sim.seed), idx = (unsigned long long)(a.sim.first_qp + b);
                const long long step = a.sim.first_step + kst[0];
                double x0 = 0.0, x1 = 0.0, sX[8];
#pragma unroll
                for (int t = 0; t < 8; t++) sX[t] = pst[t];
                const double sU = pst[8];
                if (fin && g < nx) x0 = sim_row(g, nx, Ad, Bd, sX, sU, key, idx, step, a.sim.noise_std);
                if (fin && g + 4 < nx) x1 = sim_row(g + 4, nx, Ad, Bd, sX, sU, key, idx, step, a.sim.noise_std);
                // the new X on every lane of the column (component t from lane group t & 3)
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    const double v = col_from(t < 4 ? x0 : x1, t & 3, g);
                    if (fin) pst[t] = t < nx ? v : 0.0;
                }
                bool fill[G];
                fill[0] = fin && kst[0] + 1 < a.sim.steps;
                if (fin) {
                    kst[0] += 1;
                    if (!fill[0]) over[0] = true;
                }
                if (fin && !fill[0]) {  // the plant's last step: its final X (U: the finalize)
                    double *Xw = const_cast<double *>(a.X);
                    if (g < nx) Xw[(size_t)b * nx + g] = x0;
                    if (g + 4 < nx) Xw[(size_t)b * nx + g + 4] = x1;
                }
                if (!wave_any(fill[0])) return;
                load_cols(fill, false);
                set_dk();
                bool bad[G];
                bad[0] = fill[0] && status[0] != kUnsolved;
                if (wave_any(bad[0])) finalize(bad, nullptr);
                done[0] = fill[0] ? bad[0] : done[0];
                if (!wave_any(bad[0])) return;  // (a step whose bounds were invalid: its plant advances again)
            }
        }
    };

    {
        bool mine[G], any = false;
#pragma unroll
        for (int gi = 0; gi < G; gi++) {
            mine[gi] = valid[gi] && status[gi] != kUnsolved;
            any = any || mine[gi];
        }
        if (wave_any(any)) {
            finalize(mine, nullptr);
#pragma unroll
            for (int gi = 0; gi < G; gi++) done[gi] = done[gi] || mine[gi];
            // a stream column whose first step failed at once advances now (a wave whose columns all
            // failed would otherwise never reach a check)
            if constexpr (refill) stream_next();
        }
    }

    MPCQ_PRO_MARK(5);
    [[maybe_unused]] long long info_cycles = 0;  // (debug build: cycles in info iterations)
    const int ct = st.check_termination;
    const int ai = (st.adaptive_rho && a.adaptive_interval) ? a.adaptive_interval : 0;
    const int stop = a.stop_iter;
    int next_check = ct ? (it / ct + 1) * ct : -1;  // uniform; no integer division in the loop
    // refill schedule: adapt_rho and max_iter fall on check iterations (host: multiples of ct) and are
    // decided per column (its own iteration count); the wave schedules only the checks
    const int ai_w = refill ? 0 : ai;
    int next_adapt = ai_w ? (it / ai_w + 1) * ai_w : -1;
    T dx[G][NS], dy[G][MS];
    // paired loop: operators S, B~', B~ from the LDS images into VGPRs (A-fragment per tile, k-step)
    auto load_regs = [&](T (&rS)[NTR][KNR], T (&rBt)[NTR][KNR], T (&rB)[NTR][KNR]) {
        const T *im = fresh_ptr((const T *)img);
#pragma unroll
        for (int t = 0; t < NTR; t++) {
            // REM4: the 4x4x1 tile's fragment lane (g, c) is the 16x16x4 image's lane (g, 4 (c & 3))
            // (image row i holds logical row arow(i) = 4 (i & 3) + (i >> 2))
            const int ln = (REM4 && t == NTR - 1) ? ((lane & 48) | ((lane & 3) << 2)) : lane;
#pragma unroll
            for (int k = 0; k < KNR; k++) {
                rS[t][k] = im[L.S + TileLayout::at(KNP, VEC, t, k, ln)];
                rBt[t][k] = im[L.Bt + TileLayout::at(KBT, VEC, t, k, ln)];
                rB[t][k] = im[L.B + TileLayout::at(KNP, VEC, t, k, ln)];
            }
        }
    };
    // one paired ADMM iteration (see the PAIRED note above the kernel)
    auto piter = [&](auto with_delta, const T (&rS)[NTR][KNR], const T (&rBt)[NTR][KNR], const T (&rB)[NTR][KNR]) {
        constexpr bool DELTA = decltype(with_delta)::value;
        if constexpr (PAIRED) {
            // xi = -g + S x' + B~' (w_top - w_bot),  w = rho z - y
            T wt[G][KNR];
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int s = 0; s < KN; s++)
                    wt[gi][s] = tt_fma(rho[gi], z[gi][s], -y[gi][s]) - tt_fma(rho[gi], z[gi][s + KN], -y[gi][s + KN]);
            T xi[G][NS];
            reg_mv<T, G, NT, KN, NS, true, KNR, REM4>(rS, xs, rBt, wt, xi, gv);
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int s = 0; s < KN; s++) {
                    xi[gi][s] = xi[gi][s] * dk[gi][s];
                    const T xn = tt_fma(alpha, xi[gi][s], oma * xs[gi][s]);
                    if (DELTA) dx[gi][s] = xn - xs[gi][s];
                    xs[gi][s] = xn;
                }
            // z~_top = B~ eta (z~_bot = -z~_top) ; relaxation ; projection ; dual update
            T zt[G][NS];
            reg_mv<T, G, NT, KN, NS, false, KNR, REM4>(rB, xi, rB, wt, zt, nullptr);
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int s = 0; s < KM; s++) {
                    const T rj = rho[gi], rij = rinv[gi];
                    const T zts = s < KN ? zt[gi][s] : -zt[gi][s - KN];
                    const T v = tt_fma(alpha, zts, oma * z[gi][s]);
                    T zn = tt_fma(rij, y[gi][s], v);
                    zn = tt_fmin(zn, uh[gi][s]);
                    if (DELTA) dy[gi][s] = rj * (v - zn);
                    y[gi][s] = tt_fma(rj, v - zn, y[gi][s]);
                    z[gi][s] = zn;
                }
        }
    };
    // The plain (non-info) paired iteration.  It runs on the scaled dual yt = y / rho (the y registers
    // hold yt between info iterations) and folds alpha into the KKT step, which takes the VALU work
    // per element from 3 (x) / 7 (z, y) to 2 / 4 (the f32 matrix and vector pipes share the SIMD, so
    // vector instructions cost MFMA time):
    //   w~  = rho ((z - yt)_top - (z - yt)_bot)
    //   xi  = (-g + S x') + B~' w~ ;  eta' = alpha dk xi ;  x' = eta' + (1 - alpha) x'
    //   zt' = B~ eta' (= alpha z~_top, z~_bot = -z~_top)
    //   t = (1 - alpha) z + zt' + yt ;  z = min(t, u) ;  yt = t - z
    // (OSQP: z = min(alpha z~ + (1 - alpha) z + y / rho, u), y += rho (alpha z~ + (1 - alpha) z - z_new)).
    // sx = -g + S x' of the NEXT iteration is issued right after x' so that its MFMAs run beside the
    // z/y update.
    auto piter_fast = [&](const T (&rS)[NTR][KNR], const T (&rBt)[NTR][KNR], const T (&rB)[NTR][KNR],
                          T (&sx)[G][NS], const T (&adk)[G][KNR]) {
        if constexpr (PAIRED) {
            T wt[G][KNR];
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int s = 0; s < KN; s++)
                    wt[gi][s] = rho[gi] * ((z[gi][s] - y[gi][s]) - (z[gi][s + KN] - y[gi][s + KN]));
            T xi[G][NS];
            reg_mv<T, G, NT, KN, KNR, false, KNR, REM4>(rBt, wt, rBt, wt, xi, sx);  // xi = (-g + S x') + B~' w~
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int s = 0; s < KN; s++) {
                    xi[gi][s] = adk[gi][s] * xi[gi][s];           // eta' = alpha eta
                    xs[gi][s] = tt_fma(oma, xs[gi][s], xi[gi][s]);  // x' = alpha eta + (1 - alpha) x'
                }
            T zt[G][NS];
            reg_mv<T, G, NT, KN, NS, false, KNR, REM4>(rB, xi, rB, wt, zt, nullptr);  // alpha z~_top = B~ eta'
            reg_mv<T, G, NT, KN, NS, false, KNR, REM4>(rS, xs, rS, wt, sx, gv);       // next: -g + S x'
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int s = 0; s < KM; s++) {
                    const T v = s < KN ? tt_fma(oma, z[gi][s], zt[gi][s]) : tt_fma(oma, z[gi][s], -zt[gi][s - KN]);
                    const T t = v + y[gi][s];
                    const T zn = vmin(t, uh[gi][s]);
                    y[gi][s] = t - zn;
                    z[gi][s] = zn;
                }
        }
    };
    // f64 paired loop (NBS > 0): piter_fast with z~ and the next S x' from ONE stacked product [B~; S] eta'
    // (ceil(8 KN / 16) tiles instead of 2 NT: 15 f64 MFMAs instead of 20 at N = 20; a 16x16x4 f64 MFMA
    // holds the matrix pipe 64 cycles, and the second tile of each separate product carries 4 rows).
    // x' = eta' + (1 - alpha) x'_old, so the next -g + S x' = (1 - alpha)(-g + S x'_old) + alpha (-g) + S eta':
    // the product's S rows start from that (a contraction by |1 - alpha| < 1: rounding does not build up).
    constexpr int NBR = NBS > 0 ? NBS : 1;
    auto load_regs_stk = [&](T (&rBt)[NTR][KNR], T (&rBS)[NBR][KNR]) {
        const T *im = fresh_ptr((const T *)img);
#pragma unroll
        for (int t = 0; t < NTR; t++)
#pragma unroll
            for (int k = 0; k < KNR; k++) rBt[t][k] = im[L.Bt + TileLayout::at(KBT, VEC, t, k, lane)];
#pragma unroll
        for (int t = 0; t < NBR; t++)
#pragma unroll
            for (int k = 0; k < KNR; k++) rBS[t][k] = im[L.BS + TileLayout::at(KNP, VEC, t, k, lane)];
    };
    auto piter_stk = [&](const T (&rBt)[NTR][KNR], const T (&rBS)[NBR][KNR], T (&sx)[G][NS], const T (&adk)[G][KNR],
                         const T (&agv)[G][KNR]) {
        if constexpr (NBS > 0) {
            T wt[G][KNR];
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int s = 0; s < KN; s++)
                    wt[gi][s] = rho[gi] * ((z[gi][s] - y[gi][s]) - (z[gi][s + KN] - y[gi][s + KN]));
            T xi[G][NS];
            reg_mv<T, G, NT, KN, KNR, false, KNR>(rBt, wt, rBt, wt, xi, sx);  // xi = (-g + S x') + B~' w~
            T ini[G][4 * NBR];  // z~ rows from 0, S rows from (1 - alpha)(-g + S x'_old) + alpha (-g)
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int f = 0; f < 4 * NBR; f++)
                    ini[gi][f] = (f >= KN && f < 2 * KN) ? tt_fma(oma, sx[gi][f - KN], agv[gi][f - KN]) : T(0);
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int s = 0; s < KN; s++) {
                    xi[gi][s] = adk[gi][s] * xi[gi][s];           // eta' = alpha eta
                    xs[gi][s] = tt_fma(oma, xs[gi][s], xi[gi][s]);  // x' = alpha eta + (1 - alpha) x'
                }
            T out[G][4 * NBR];
            reg_mv<T, G, NBR, KN, NS, false, KNR>(rBS, xi, rBS, wt, out, ini);  // [alpha z~_top; next -g + S x']
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
#pragma unroll
                for (int s = 0; s < KN; s++) sx[gi][s] = out[gi][KN + s];
#pragma unroll
                for (int s = 0; s < KM; s++) {
                    const T v = s < KN ? tt_fma(oma, z[gi][s], out[gi][s]) : tt_fma(oma, z[gi][s], -out[gi][s - KN]);
                    const T t = v + y[gi][s];
                    const T zn = vmin(t, uh[gi][s]);
                    y[gi][s] = t - zn;
                    z[gi][s] = zn;
                }
            }
        }
    };
    // piter_fast's f32 arithmetic on packed pairs (v_pk_fma/add/mul_f32: two elements per VALU issue,
    // the f32 vector and matrix work share the SIMD's issue time): element pairs (2k, 2k + 1) of each
    // half-vector (top rows s < KN, bottom rows KN + s) with an odd last element on its own.  The state
    // is held in pairs for the plain iterations between two info iterations.  With the 4x4x1 remainder
    // tile (REM4) the partial sums of S x' rows 16.. are not reduced on their own but seed the next xi's
    // remainder chain (one lane reduction per iteration fewer; the sum is reassociated there), otherwise
    // every operation and its order are piter_fast's.
    // (MIX: the same loop on fp32 copies of the fp64 kernel's state: xs_, z_, y_ (yt), uh_, rho_, oma_ are
    // this loop's fp32 state and data, the fp32 kernel's own registers otherwise)
    constexpr bool PK = PAIRED && std::is_same<T, float>::value && MPCQ_PK;
    auto piter_pk_loop = [&](const float (&rS)[NTR][KNR], const float (&rBt)[NTR][KNR], const float (&rB)[NTR][KNR],
                             float (&sx)[G][NS], const float (&adk)[G][KNR], typename Mf<float>::acc (&srem)[G],
                             const int nxt, float (&xs_)[G][NS], float (&z_)[G][MS], float (&y_)[G][MS],
                             const float (&uh_)[G][MS], const float (&gv_)[G][NS], const float (&rho_)[G],
                             const float oma_) {
        if constexpr (PK || MIX) {
            constexpr bool REM4 = REM4F;
            typedef float f2 __attribute__((ext_vector_type(2)));
            constexpr int NPR = KN / 2;
            constexpr bool ODD = (KN & 1) != 0;
            auto pfma = [](f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); };
            f2 XP[G][NPR], ZT[G][NPR], ZB[G][NPR], YT[G][NPR], YB[G][NPR], AD[G][NPR], RH[G];
            float X1[G], ZT1[G], ZB1[G], YT1[G], YB1[G], AD1[G];
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                RH[gi] = f2{rho_[gi], rho_[gi]};
#pragma unroll
                for (int k = 0; k < NPR; k++) {
                    XP[gi][k] = f2{xs_[gi][2 * k], xs_[gi][2 * k + 1]};
                    ZT[gi][k] = f2{z_[gi][2 * k], z_[gi][2 * k + 1]};
                    ZB[gi][k] = f2{z_[gi][KN + 2 * k], z_[gi][KN + 2 * k + 1]};
                    YT[gi][k] = f2{y_[gi][2 * k], y_[gi][2 * k + 1]};
                    YB[gi][k] = f2{y_[gi][KN + 2 * k], y_[gi][KN + 2 * k + 1]};
                    AD[gi][k] = f2{adk[gi][2 * k], adk[gi][2 * k + 1]};
                }
                if constexpr (ODD) {
                    X1[gi] = xs_[gi][KN - 1];
                    ZT1[gi] = z_[gi][KN - 1];
                    ZB1[gi] = z_[gi][2 * KN - 1];
                    YT1[gi] = y_[gi][KN - 1];
                    YB1[gi] = y_[gi][2 * KN - 1];
                    AD1[gi] = adk[gi][KN - 1];
                }
            }
            const f2 OMA = f2{oma_, oma_};
            do {
                it++;
                float wt[G][KNR];  // w~ = rho ((z - yt)_top - (z - yt)_bot)
#pragma unroll
                for (int gi = 0; gi < G; gi++) {
#pragma unroll
                    for (int k = 0; k < NPR; k++) {
                        const f2 w = RH[gi] * ((ZT[gi][k] - YT[gi][k]) - (ZB[gi][k] - YB[gi][k]));
                        wt[gi][2 * k] = w.x;
                        wt[gi][2 * k + 1] = w.y;
                    }
                    if constexpr (ODD) wt[gi][KN - 1] = rho_[gi] * ((ZT1[gi] - YT1[gi]) - (ZB1[gi] - YB1[gi]));
                }
                float xi[G][NS];
                if constexpr (REM4) reg_mv<float, G, NT, KN, KNR, false, KNR, REM4, 2>(rBt, wt, rBt, wt, xi, sx, srem);
                else reg_mv<float, G, NT, KN, KNR, false, KNR, REM4>(rBt, wt, rBt, wt, xi, sx);  // xi = (-g + S x') + B~' w~
                float xv[G][NS];  // x' as the next S x' product's operand
#pragma unroll
                for (int gi = 0; gi < G; gi++) {
#pragma unroll
                    for (int k = 0; k < NPR; k++) {
                        const f2 e = AD[gi][k] * f2{xi[gi][2 * k], xi[gi][2 * k + 1]};  // eta' = alpha eta
                        xi[gi][2 * k] = e.x;
                        xi[gi][2 * k + 1] = e.y;
                        XP[gi][k] = pfma(OMA, XP[gi][k], e);                           // x' = eta' + (1 - alpha) x'
                        xv[gi][2 * k] = XP[gi][k].x;
                        xv[gi][2 * k + 1] = XP[gi][k].y;
                    }
                    if constexpr (ODD) {
                        xi[gi][KN - 1] = AD1[gi] * xi[gi][KN - 1];
                        X1[gi] = tt_fma(oma_, X1[gi], xi[gi][KN - 1]);
                        xv[gi][KN - 1] = X1[gi];
                    }
#pragma unroll
                    for (int s = KN; s < NS; s++) xv[gi][s] = 0.0f;
                }
                float zt[G][NS];
                reg_mv<float, G, NT, KN, NS, false, KNR, REM4>(rB, xi, rB, wt, zt, nullptr);  // alpha z~_top = B~ eta'
                if constexpr (REM4) reg_mv<float, G, NT, KN, NS, false, KNR, REM4, 1>(rS, xv, rS, wt, sx, gv_, srem);
                else reg_mv<float, G, NT, KN, NS, false, KNR, REM4>(rS, xv, rS, wt, sx, gv_);  // next: -g + S x'
#pragma unroll
                for (int gi = 0; gi < G; gi++) {
#pragma unroll
                    for (int k = 0; k < NPR; k++) {
                        const f2 zp = f2{zt[gi][2 * k], zt[gi][2 * k + 1]};
                        f2 t = pfma(OMA, ZT[gi][k], zp) + YT[gi][k];  // t = (1 - alpha) z + zt' + yt
                        f2 zn = f2{vmin(t.x, uh_[gi][2 * k]), vmin(t.y, uh_[gi][2 * k + 1])};
                        YT[gi][k] = t - zn;
                        ZT[gi][k] = zn;
                        t = pfma(OMA, ZB[gi][k], -zp) + YB[gi][k];
                        zn = f2{vmin(t.x, uh_[gi][KN + 2 * k]), vmin(t.y, uh_[gi][KN + 2 * k + 1])};
                        YB[gi][k] = t - zn;
                        ZB[gi][k] = zn;
                    }
                    if constexpr (ODD) {
                        float t = tt_fma(oma_, ZT1[gi], zt[gi][KN - 1]) + YT1[gi];
                        float zn = vmin(t, uh_[gi][KN - 1]);
                        YT1[gi] = t - zn;
                        ZT1[gi] = zn;
                        t = tt_fma(oma_, ZB1[gi], -zt[gi][KN - 1]) + YB1[gi];
                        zn = vmin(t, uh_[gi][2 * KN - 1]);
                        YB1[gi] = t - zn;
                        ZB1[gi] = zn;
                    }
                }
            } while (it + 1 < nxt);
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
#pragma unroll
                for (int k = 0; k < NPR; k++) {
                    xs_[gi][2 * k] = XP[gi][k].x;
                    xs_[gi][2 * k + 1] = XP[gi][k].y;
                    z_[gi][2 * k] = ZT[gi][k].x;
                    z_[gi][2 * k + 1] = ZT[gi][k].y;
                    z_[gi][KN + 2 * k] = ZB[gi][k].x;
                    z_[gi][KN + 2 * k + 1] = ZB[gi][k].y;
                    y_[gi][2 * k] = YT[gi][k].x;
                    y_[gi][2 * k + 1] = YT[gi][k].y;
                    y_[gi][KN + 2 * k] = YB[gi][k].x;
                    y_[gi][KN + 2 * k + 1] = YB[gi][k].y;
                }
                if constexpr (ODD) {
                    xs_[gi][KN - 1] = X1[gi];
                    z_[gi][KN - 1] = ZT1[gi];
                    z_[gi][2 * KN - 1] = ZB1[gi];
                    y_[gi][KN - 1] = YT1[gi];
                    y_[gi][2 * KN - 1] = YB1[gi];
                }
            }
        }
    };
    MPCQ_TSTAMP(2, (long long)__builtin_amdgcn_s_memtime());
    // MIX: the wave runs every remaining iteration in fp64 once one of its running columns looks primal
    // infeasible (OSQP's certificate candidate, u' dy < eps ||dy||, with ||A' dy|| within 1e4 eps ||dy|| but not
    // below eps ||dy||): an infeasible QP's dual iterate grows without bound, the fp32 stretches' rounding of it
    // keeps ||A' dy|| / ||dy|| near 1e-4 .. 1e-2 where fp64 reaches ~1e-12, and the certificate would then be
    // missed (the QP running to max_iter).  Feasible QPs' candidates sit at ratios >= ~40 (config 2), so the
    // switch does not fire on them.  Wave-uniform.
    bool mix64 = false;
    while (!all_done()) {
        if constexpr (PAIRED) {
            // plain iterations up to the next info iteration, with the operators held in VGPRs
            // (loaded here, dead across the check code below)
            int nxt = refill ? next_check : (st.max_iter < stop ? st.max_iter : stop);
            if (ct && next_check < nxt) nxt = next_check;
            if (ai_w && next_adapt < nxt) nxt = next_adapt;
            if constexpr (MIX) {
                // fp32 stretch: iterations it + 1 .. nxt - mix_r on fp32 copies of the state (yt = y / rho),
                // the operators rounded from the fp64 images; then the last mix_r - 1 plain iterations and
                // the info iteration in fp64 (below)
                const int n32 = mix64 ? it : nxt - a.mix_r;  // (mix64: no fp32 stretch)
#ifdef MPCQ_MIX_STAMPS  // debug build: cycles in the fp32 stretches -> phase stamp 5
                const long long t_mix = a.stamps ? (long long)__builtin_amdgcn_s_memtime() : 0;
#endif
                if (it < n32) {
                    float xs32[G][NS], z32[G][MS], y32[G][MS], uh32[G][MS], gv32[G][NS], rho32[G], adk32[G][KNR];
#pragma unroll
                    for (int gi = 0; gi < G; gi++) {
                        rho32[gi] = (float)rho[gi];
#pragma unroll
                        for (int s = 0; s < NS; s++) {
                            xs32[gi][s] = (float)xs[gi][s];
                            gv32[gi][s] = (float)gv[gi][s];
                            asm volatile("" : "+v"(gv32[gi][s]));  // (as uh32 below)
                        }
#pragma unroll
                        for (int s = 0; s < MS; s++) {
                            z32[gi][s] = (float)z[gi][s];
                            y32[gi][s] = s < KM ? (float)(y[gi][s] * rinv[gi]) : 0.0f;
                            uh32[gi][s] = (float)uh[gi][s];
                            // (the fp32 bounds are values of their own: not re-converted from uh inside the loop)
                            asm volatile("" : "+v"(uh32[gi][s]));
                        }
#pragma unroll
                        for (int s = 0; s < KN; s++) adk32[gi][s] = (float)(alpha * dk[gi][s]);
                    }
                    // fp32 A fragments from the fp64 images (f64 image row i is logical row i; the f32
                    // 16x16x4 fragment of lane (g, c) is row arow_f32(c), the 4x4x1 one's row c & 3)
                    float rS32[NTR][KNR], rBt32[NTR][KNR], rB32[NTR][KNR];
                    {
                        const double *im = fresh_ptr((const double *)img);
#pragma unroll
                        for (int t = 0; t < NTR; t++) {
                            const int ln = (REM4F && t == NTR - 1) ? ((lane & 48) | (lane & 3))
                                                                   : ((lane & 48) | tile_arow(1, lane & 15));
#pragma unroll
                            for (int k = 0; k < KNR; k++) {
                                rS32[t][k] = (float)im[L.S + TileLayout::at(KNP, VEC, t, k, ln)];
                                rBt32[t][k] = (float)im[L.Bt + TileLayout::at(KBT, VEC, t, k, ln)];
                                rB32[t][k] = (float)im[L.B + TileLayout::at(KNP, VEC, t, k, ln)];
                            }
                        }
                    }
                    float sx32[G][NS];
                    typename Mf<float>::acc srem32[G];
                    if constexpr (REM4F) reg_mv<float, G, NT, KN, NS, false, NS, REM4F, 1>(rS32, xs32, rS32, xs32, sx32, gv32, srem32);
                    else reg_mv<float, G, NT, KN, NS, false, NS, REM4F>(rS32, xs32, rS32, xs32, sx32, gv32);
                    piter_pk_loop(rS32, rBt32, rB32, sx32, adk32, srem32, n32 + 1, xs32, z32, y32, uh32, gv32, rho32,
                                  (float)oma);
#pragma unroll
                    for (int gi = 0; gi < G; gi++) {
#pragma unroll
                        for (int s = 0; s < KN; s++) xs[gi][s] = (double)xs32[gi][s];
#pragma unroll
                        for (int s = 0; s < KM; s++) {
                            z[gi][s] = (double)z32[gi][s];
                            y[gi][s] = (double)y32[gi][s] * rho[gi];
                        }
                    }
                }
#ifdef MPCQ_MIX_STAMPS
                if (a.stamps) info_cycles += (long long)__builtin_amdgcn_s_memtime() - t_mix;
#endif
            }
            if constexpr (NBS > 0) {
                if (it + 1 < nxt) {
                    T rBt[NTR][KNR], rBS[NBR][KNR];
                    load_regs_stk(rBt, rBS);
                    T sx[G][NS], adk[G][KNR], agv[G][KNR];
                    tile_mv_g<T, G, NT, KN, KNP>(img + L.S, xs, sx, lane, gv);  // -g + S x'
#pragma unroll
                    for (int gi = 0; gi < G; gi++) {
#pragma unroll
                        for (int s = 0; s < KN; s++) {
                            // (loop invariants of their own: not recomputed inside the loop)
                            adk[gi][s] = alpha * dk[gi][s];
                            agv[gi][s] = alpha * gv[gi][s];
                            asm volatile("" : "+v"(adk[gi][s]), "+v"(agv[gi][s]));
                        }
#pragma unroll
                        for (int s = 0; s < KM; s++) y[gi][s] = y[gi][s] * rinv[gi];  // y -> yt = y / rho
                    }
                    do {
                        it++;
                        piter_stk(rBt, rBS, sx, adk, agv);
                    } while (it + 1 < nxt);
#pragma unroll
                    for (int gi = 0; gi < G; gi++)
#pragma unroll
                        for (int s = 0; s < KM; s++) y[gi][s] = y[gi][s] * rho[gi];  // yt -> y
                }
            } else if (it + 1 < nxt) {
                T rS[NTR][KNR], rBt[NTR][KNR], rB[NTR][KNR];
                load_regs(rS, rBt, rB);
                T sx[G][NS], adk[G][KNR];
                typename Mf<T>::acc srem[G];  // PK: the remainder partials of S x' (reduced inside the next xi)
                if constexpr (PK && REM4) reg_mv<T, G, NT, KN, NS, false, NS, REM4, 1>(rS, xs, rS, xs, sx, gv, srem);
                else reg_mv<T, G, NT, KN, NS, false, NS, REM4>(rS, xs, rS, xs, sx, gv);
#pragma unroll
                for (int gi = 0; gi < G; gi++) {
#pragma unroll
                    for (int s = 0; s < KN; s++) adk[gi][s] = alpha * dk[gi][s];
#pragma unroll
                    for (int s = 0; s < KM; s++) y[gi][s] = y[gi][s] * rinv[gi];  // y -> yt = y / rho
                }
                if constexpr (PK) {
                    piter_pk_loop(rS, rBt, rB, sx, adk, srem, nxt, xs, z, y, uh, gv, rho, oma);
                } else {
                    do {
                        it++;
                        piter_fast(rS, rBt, rB, sx, adk);
                    } while (it + 1 < nxt);
                }
#pragma unroll
                for (int gi = 0; gi < G; gi++)
#pragma unroll
                    for (int s = 0; s < KM; s++) y[gi][s] = y[gi][s] * rho[gi];  // yt -> y
            }
        }
        it++;
#ifdef MPCQ_INFO_STAMPS  // debug build: cycles in info iterations -> phase stamp 5
        long long t_info = a.stamps ? (long long)__builtin_amdgcn_s_memtime() : 0;
#endif
        // MPCQ_INFO_PART=p (with MPCQ_INFO_STAMPS): stamp 5 counts only the part between marks p-1, p
#if defined(MPCQ_INFO_STAMPS) && defined(MPCQ_INFO_PART)
#define MPCQ_INFO_MARK(k)                                                                          \
    do {                                                                                           \
        if (a.stamps && (k) == MPCQ_INFO_PART - 1) t_info = (long long)__builtin_amdgcn_s_memtime(); \
        if (a.stamps && (k) == MPCQ_INFO_PART) info_cycles += (long long)__builtin_amdgcn_s_memtime() - t_info; \
    } while (0)
#else
#define MPCQ_INFO_MARK(k) do { } while (0)
#endif
        const bool at_check = it == next_check;
        const bool at_adapt_w = it == next_adapt;
        if (at_check) next_check += ct;
        if (at_adapt_w) next_adapt += ai_w;
        const bool last_w = !refill && it == st.max_iter;
        const bool info = at_check || at_adapt_w || last_w || it == stop;
        // per column: adapt_rho and the end of the ADMM loop at the column's own iteration count
        bool adapt_c[G], last_c[G];
#pragma unroll
        for (int gi = 0; gi < G; gi++) {
            adapt_c[gi] = refill ? (at_check && ai && (it - cst[gi]) % ai == 0) : at_adapt_w;
            last_c[gi] = refill ? (at_check && it - cst[gi] == st.max_iter) : last_w;
        }
        bool at_adapt = at_adapt_w, last = last_w;  // any column
        if (refill && at_check) {
            bool aa = false, ll = false;
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                aa = aa || (adapt_c[gi] && !done[gi]);
                ll = ll || (last_c[gi] && !done[gi]);
            }
            at_adapt = wave_any(aa);
            last = wave_any(ll);
        }

        // ---- one ADMM iteration; the check iterations also keep delta_x', delta_y (OSQP's
        // delta_x / delta_y, for the infeasibility certificates)
        auto iterate = [&](auto with_delta) {
            constexpr bool DELTA = decltype(with_delta)::value;
            if constexpr (PAIRED) {
                T rS[NTR][KNR], rBt[NTR][KNR], rB[NTR][KNR];
                load_regs(rS, rBt, rB);
                piter(with_delta, rS, rBt, rB);
            } else {
            // xi = -g + sigma W'W x' + B' w,   w_j = rho_j z_j - y_j   (w reuses the zt registers)
            T wz[G][MS];
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int s = 0; s < MS; s++) {
                    T rj = rho[gi];
                    if (!ALL_INEQ) rj = rs[s] < T(0) ? T(kRhoMin) : rho[gi] * rs[s];
                    wz[gi][s] = s < KM ? tt_fma(rj, z[gi][s], -y[gi][s]) : T(0);
                }
            T xi[G][NS];
            tile_mv_g<T, G, NT, KN, KNP>(img + L.S, xs, xi, lane, gv);   // xi = -g + S x'
            tile_mv_g<T, G, NT, KM, KMP>(img + L.Bt, wz, xi, lane, xi);  //    + B' w
            // eta = xi / (1 + rho lambda) ; x' = alpha eta + (1 - alpha) x'
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int s = 0; s < KN; s++) {  // registers s >= KN are padding rows: x' stays 0 there
                    xi[gi][s] = xi[gi][s] * dk[gi][s];
                    const T xn = tt_fma(alpha, xi[gi][s], oma * xs[gi][s]);
                    if (DELTA) dx[gi][s] = xn - xs[gi][s];
                    xs[gi][s] = xn;
                }
            // z~ = B eta ; relaxation ; projection ; dual update
            tile_mv_g<T, G, MT, KN, KNP>(img + L.B, xi, wz, lane, nullptr);
#pragma unroll
            for (int gi = 0; gi < G; gi++)
#pragma unroll
                for (int s = 0; s < KM; s++) {
                    T rj = rho[gi], rij = rinv[gi];
                    if (!ALL_INEQ) {
                        rj = rs[s] < T(0) ? T(kRhoMin) : rho[gi] * rs[s];
                        rij = T(1) / rj;
                    }
                    const T v = tt_fma(alpha, wz[gi][s], oma * z[gi][s]);
                    T zn = tt_fma(rij, y[gi][s], v);
                    if (!LFREE) zn = tt_fmax(zn, lh[gi][s]);  // == OSQP's c_max/c_min, NaN included
                    zn = tt_fmin(zn, uh[gi][s]);
                    if (DELTA) dy[gi][s] = rj * (v - zn);  // OSQP delta_y (certificates only)
                    y[gi][s] = tt_fma(rj, v - zn, y[gi][s]);
                    z[gi][s] = zn;
                }
            }
        };
        if (!info) {
            iterate(std::false_type{});
            continue;
        }
        iterate(std::true_type{});
        double Uold[G];  // U of the running columns, ahead of a finalize (latency hidden by the checks)
#pragma unroll
        for (int gi = 0; gi < G; gi++) Uold[gi] = (!refill && a.mpc_u && g == 0 && !done[gi]) ? a.U[opaque(b_[gi])] : 0.0;
        MPCQ_INFO_MARK(1);
#pragma unroll
        for (int gi = 0; gi < G; gi++)
#pragma unroll
            for (int s = KM; s < MS; s++) dy[gi][s] = T(0);

        // ---- update_info: residuals in the scaled space (reported unscaled), 4-lane reductions.  The
        // termination test reads the unscaled-space norms (_s: E^-1, D^-1 applied) unless
        // scaled_termination, adapt_rho the scaled-space ones (_r): each set only where it is read.
        const bool need_r = scaled_term || at_adapt, need_s = !scaled_term;
        T ax_z[G], ax_zs[G], zn_s[G], zn_r[G], axn_s[G], axn_r[G];
        {
            T ax[G][MS];
            if constexpr (PAIRED) {  // A x: the top rows B~ x' (B's first NT tiles), the bottom ones their negation
                T axt[G][NS];
                tile_mv_g<T, G, NT, KN, KNP, NS, REM4>(img + L.B, xs, axt, lane, nullptr);
#pragma unroll
                for (int gi = 0; gi < G; gi++)
#pragma unroll
                    for (int s = 0; s < MS; s++)
                        ax[gi][s] = s < KN ? axt[gi][s] : (s < KM ? -axt[gi][s < KM ? s - KN : 0] : T(0));
            } else {
                tile_mv_g<T, G, MT, KN, KNP>(img + L.B, xs, ax, lane, nullptr);
            }
            const T *Einv = fresh_ptr((const T *)s_Einv);
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                ax_z[gi] = ax_zs[gi] = zn_s[gi] = zn_r[gi] = axn_s[gi] = axn_r[gi] = T(0);
                if (need_r) {
#pragma unroll
                    for (int s = 0; s < KM; s++) {
                        const T r = ax[gi][s] - z[gi][s];
                        ax_z[gi] = nrm(ax_z[gi], r);
                        zn_r[gi] = nrm(zn_r[gi], z[gi][s]);
                        axn_r[gi] = nrm(axn_r[gi], ax[gi][s]);
                    }
                }
                if (need_s) {
#pragma unroll
                    for (int s = 0; s < KM; s++) {
                        const T r = ax[gi][s] - z[gi][s];
                        const T ei = Einv[4 * s + g];
                        ax_zs[gi] = nrm(ax_zs[gi], ei * r);
                        zn_s[gi] = nrm(zn_s[gi], ei * z[gi][s]);
                        axn_s[gi] = nrm(axn_s[gi], ei * ax[gi][s]);
                    }
                }
            }
        }
        T dr_r[G], dr_s[G], qn_r[G], qn_s[G], atyn_r[G], atyn_s[G], pxn_r[G], pxn_s[G];
        {
            T px[G][NS], aty[G][NS];
            tile_mv_g<T, G, NT, KN, KNP, NS, REM4>(img + L.PW, xs, px, lane, nullptr);
            if constexpr (PAIRED) {  // A' y = A~' (y_top - y_bot): the first KN k-steps of the A^' image
                T yd[G][KNR];
#pragma unroll
                for (int gi = 0; gi < G; gi++)
#pragma unroll
                    for (int s = 0; s < KN; s++) yd[gi][s] = y[gi][s] - y[gi][s + KN];
                tile_mv_g<T, G, NT, KN, KBT, KNR, REM4>(img + L.AhT, yd, aty, lane, nullptr);
            } else {
                tile_mv_g<T, G, NT, KM, KMP>(img + L.AhT, y, aty, lane, nullptr);
            }
            const T *Dinv = fresh_ptr((const T *)s_Dinv);
            const T(*const qhw)[64] = s_qh[opaque((int)threadIdx.x >> 6)];  // this wave's q^ (prologue)
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                T qh[NS];
#pragma unroll
                for (int s = 0; s < KN; s++) qh[s] = qhw[gi * KN + s][lane];
                dr_r[gi] = dr_s[gi] = qn_r[gi] = qn_s[gi] = atyn_r[gi] = atyn_s[gi] = pxn_r[gi] = pxn_s[gi] = T(0);
                if (need_r) {
#pragma unroll
                    for (int s = 0; s < KN; s++) {
                        const T r = (qh[s] + px[gi][s]) + aty[gi][s];
                        dr_r[gi] = nrm(dr_r[gi], r);
                        qn_r[gi] = nrm(qn_r[gi], qh[s]);
                        atyn_r[gi] = nrm(atyn_r[gi], aty[gi][s]);
                        pxn_r[gi] = nrm(pxn_r[gi], px[gi][s]);
                    }
                }
                if (need_s) {
#pragma unroll
                    for (int s = 0; s < KN; s++) {
                        const T r = (qh[s] + px[gi][s]) + aty[gi][s];
                        const T di = Dinv[4 * s + g];
                        dr_s[gi] = nrm(dr_s[gi], di * r);
                        qn_s[gi] = nrm(qn_s[gi], di * qh[s]);
                        atyn_s[gi] = nrm(atyn_s[gi], di * aty[gi][s]);
                        pxn_s[gi] = nrm(pxn_s[gi], di * px[gi][s]);
                    }
                }
            }
        }
        T pri_res[G], dua_res[G];
        const T cinv = op.cs[1];
#pragma unroll
        for (int gi = 0; gi < G; gi++) {
            if (need_r) {
                ax_z[gi] = col_max(ax_z[gi]); zn_r[gi] = col_max(zn_r[gi]); axn_r[gi] = col_max(axn_r[gi]);
                dr_r[gi] = col_max(dr_r[gi]); qn_r[gi] = col_max(qn_r[gi]); atyn_r[gi] = col_max(atyn_r[gi]);
                pxn_r[gi] = col_max(pxn_r[gi]);
            }
            if (need_s) {
                ax_zs[gi] = col_max(ax_zs[gi]); zn_s[gi] = col_max(zn_s[gi]); axn_s[gi] = col_max(axn_s[gi]);
                dr_s[gi] = col_max(dr_s[gi]); qn_s[gi] = col_max(qn_s[gi]); atyn_s[gi] = col_max(atyn_s[gi]);
                pxn_s[gi] = col_max(pxn_s[gi]);
            }
            pri_res[gi] = scaled_term ? ax_z[gi] : ax_zs[gi];
            dua_res[gi] = scaled_term ? dr_r[gi] : cinv * dr_s[gi];
        }
        MPCQ_INFO_MARK(2);

        // OSQP is_primal_infeasible on delta_y = dy (this iteration's dual step), per group.
        auto primal_infeasible = [&](T eps, const bool (&need)[G], bool (&res)[G], bool track) {
            {  // no column of the wave asks (every live one primal-feasible): nothing to screen
                bool anyn = false;
#pragma unroll
                for (int gi = 0; gi < G; gi++) {
                    res[gi] = false;
                    anyn = anyn || need[gi];
                }
                if (!wave_any(anyn)) return;
            }
            T d[G][MS];
            T ndy[G], lhs[G];
            const T *E = fresh_ptr((const T *)s_E);
            bool cand[G], anyc = false;
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                ndy[gi] = lhs[gi] = T(0);
#pragma unroll
                for (int s = 0; s < MS; s++) {
                    if (s >= KM) { d[gi][s] = T(0); continue; }
                    T dd = dy[gi][s];
                    const T up = uh[gi][s], lo = LFREE ? T(-kInfty) : lh[gi][s];
                    const bool uinf = up > T(kInfty * kMinScaling), linf = lo < T(-kInfty * kMinScaling);
                    if (uinf) dd = linf ? T(0) : tt_min(dd, T(0));
                    else if (linf) dd = tt_max(dd, T(0));
                    d[gi][s] = dd;
                    ndy[gi] = nrm(ndy[gi], scaled_term ? dd : E[4 * s + g] * dd);
                    if (up < T(kInfty * kMinScaling)) lhs[gi] += up * tt_max(dd, T(0));
                    if (lo > T(-kInfty * kMinScaling)) lhs[gi] += lo * tt_min(dd, T(0));
                }
                ndy[gi] = col_max(ndy[gi]);
                lhs[gi] = col_sum(lhs[gi]);
                cand[gi] = need[gi] && ndy[gi] > T(kDivisionTol) && lhs[gi] < eps * ndy[gi];
                res[gi] = false;
                anyc = anyc || cand[gi];
            }
            if (!wave_any(anyc)) return;
            T atd[G][NS];
            if constexpr (PAIRED) {  // A' d = A~' (d_top - d_bot)
                T dd[G][KNR];
#pragma unroll
                for (int gi = 0; gi < G; gi++)
#pragma unroll
                    for (int s = 0; s < KN; s++) dd[gi][s] = d[gi][s] - d[gi][s + KN];
                tile_mv_g<T, G, NT, KN, KBT, KNR, REM4>(img + L.AhT, dd, atd, lane, nullptr);
            } else {
                tile_mv_g<T, G, NT, KM, KMP>(img + L.AhT, d, atd, lane, nullptr);
            }
            const T *Dinv = fresh_ptr((const T *)s_Dinv);
            bool near = false;
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                T nat = 0;
#pragma unroll
                for (int s = 0; s < KN; s++) nat = nrm(nat, scaled_term ? atd[gi][s] : Dinv[4 * s + g] * atd[gi][s]);
                nat = col_max(nat);
                res[gi] = cand[gi] && nat < eps * ndy[gi];
                if constexpr (MIX) near = near || (cand[gi] && !res[gi] && nat < T(1e4) * eps * ndy[gi]);
            }
            if constexpr (MIX) {
                if (track && wave_any(near)) mix64 = true;
            }
        };
        // OSQP is_dual_infeasible on delta_x^ = W dx, per group.
        auto dual_infeasible = [&](T eps, const bool (&need)[G], bool (&res)[G]) {
            if (a.dinf_kappa > 2.0 * (scaled_term ? 1.0 : c64) * (double)eps) {  // cannot hold (AdmmArgs)
#pragma unroll
                for (int gi = 0; gi < G; gi++) res[gi] = false;
                return;
            }
            T qdx[G];
            bool cand[G], anyc = false;
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                qdx[gi] = T(0);  // q^' dx^ = (W' q^)' dx' = -gv' dx'
#pragma unroll
                for (int s = 0; s < KN; s++) qdx[gi] = tt_fma(-gv[gi][s], dx[gi][s], qdx[gi]);
                qdx[gi] = col_sum(qdx[gi]);
                cand[gi] = need[gi] && qdx[gi] < T(0);
                res[gi] = false;
                anyc = anyc || cand[gi];
            }
            if (!wave_any(anyc)) return;
            T t1[G][NS], ndx[G];
            tile_mv_g<T, G, NT, KN, KNP>(img + L.W, dx, t1, lane, nullptr);
            const T *D = fresh_ptr((const T *)s_D);
            const T cs = scaled_term ? T(1) : op.cs[0];
            anyc = false;
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                ndx[gi] = T(0);
#pragma unroll
                for (int s = 0; s < KN; s++) ndx[gi] = nrm(ndx[gi], scaled_term ? t1[gi][s] : D[4 * s + g] * t1[gi][s]);
                ndx[gi] = col_max(ndx[gi]);
                cand[gi] = cand[gi] && ndx[gi] > T(kDivisionTol) && qdx[gi] < -cs * eps * ndx[gi];
                anyc = anyc || cand[gi];
            }
            if (!wave_any(anyc)) return;
            tile_mv_g<T, G, NT, KN, KNP>(img + L.PW, dx, t1, lane, nullptr);
            const T *Dinv = fresh_ptr((const T *)s_Dinv);
            anyc = false;
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                T npdx = 0;
#pragma unroll
                for (int s = 0; s < KN; s++) npdx = nrm(npdx, scaled_term ? t1[gi][s] : Dinv[4 * s + g] * t1[gi][s]);
                npdx = col_max(npdx);
                cand[gi] = cand[gi] && npdx < cs * eps * ndx[gi];
                anyc = anyc || cand[gi];
            }
            if (!wave_any(anyc)) return;
            T adx[G][MS];
            if constexpr (PAIRED) {  // A dx: the top rows B~ dx', the bottom ones their negation
                T adt[G][NS];
                tile_mv_g<T, G, NT, KN, KNP, NS, REM4>(img + L.B, dx, adt, lane, nullptr);
#pragma unroll
                for (int gi = 0; gi < G; gi++)
#pragma unroll
                    for (int s = 0; s < MS; s++)
                        adx[gi][s] = s < KN ? adt[gi][s] : (s < KM ? -adt[gi][s < KM ? s - KN : 0] : T(0));
            } else {
                tile_mv_g<T, G, MT, KN, KNP>(img + L.B, dx, adx, lane, nullptr);
            }
            const T *Einv = fresh_ptr((const T *)s_Einv);
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                int viol = 0;
#pragma unroll
                for (int s = 0; s < KM; s++) {
                    const T sv = scaled_term ? adx[gi][s] : Einv[4 * s + g] * adx[gi][s];
                    const T up = uh[gi][s], lo = LFREE ? T(-kInfty) : lh[gi][s];
                    if ((up < T(kInfty * kMinScaling) && sv > eps * ndx[gi]) ||
                        (lo > T(-kInfty * kMinScaling) && sv < -eps * ndx[gi]))
                        viol = 1;
                }
                viol = col_or(viol);
                res[gi] = cand[gi] && !viol;
            }
        };
        // check_termination(approximate) — OSQP auxil.c; new status per group (kUnsolved: go on)
        auto check_termination = [&](bool approx, const bool (&need0)[G], int (&out)[G]) {
            // (the approximate check's 10 eps from the arguments, formed on the host in T: products hoisted
            // out of the loop would be held, and spilled, in VGPRs)
            const T ea = approx ? a.eps10[0] : eps_abs, er = approx ? a.eps10[1] : eps_rel;
            bool noncvx[G], prim_ok[G], dual_ok[G], need_p[G], need_d[G], prim_inf[G], dual_inf[G];
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                noncvx[gi] = pri_res[gi] > T(kInfty) || dua_res[gi] > T(kInfty);
                const bool need = need0[gi] && !noncvx[gi];  // every lane runs the (uniform) code below
                prim_ok[gi] = (m == 0);
                need_p[gi] = false;
                if (m > 0) {
                    const T ep = ea + er * (scaled_term ? tt_max(zn_r[gi], axn_r[gi]) : tt_max(zn_s[gi], axn_s[gi]));
                    prim_ok[gi] = pri_res[gi] < ep;
                    need_p[gi] = need && !prim_ok[gi];
                }
                const T ed = ea + er * (scaled_term ? tt_max(tt_max(qn_r[gi], atyn_r[gi]), pxn_r[gi])
                                                    : cinv * tt_max(tt_max(qn_s[gi], atyn_s[gi]), pxn_s[gi]));
                dual_ok[gi] = dua_res[gi] < ed;
                need_d[gi] = need && !dual_ok[gi];
            }
            primal_infeasible(approx ? a.eps10[2] : (T)st.eps_prim_inf, need_p, prim_inf, !approx);
            dual_infeasible(approx ? a.eps10[3] : (T)st.eps_dual_inf, need_d, dual_inf);
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                int o = kUnsolved;
                if (noncvx[gi]) o = kNonCvx;
                else if (prim_ok[gi] && dual_ok[gi]) o = approx ? kSolvedInaccurate : kSolved;
                else if (prim_inf[gi]) o = approx ? kPrimalInfeasibleInaccurate : kPrimalInfeasible;
                else if (dual_inf[gi]) o = approx ? kDualInfeasibleInaccurate : kDualInfeasible;
                out[gi] = o;
            }
        };

        bool term[G], need[G];
#pragma unroll
        for (int gi = 0; gi < G; gi++) {
            term[gi] = done[gi];  // finished (or dead) columns ignore everything below
            need[gi] = !term[gi];
        }
        if (at_check) {
            int s0[G];
            check_termination(false, need, s0);
#pragma unroll
            for (int gi = 0; gi < G; gi++)
                if (!term[gi] && s0[gi] != kUnsolved) { status[gi] = s0[gi]; term[gi] = true; }
        }
        MPCQ_INFO_MARK(3);
        if (at_adapt) {  // adapt_rho / compute_rho_estimate (scaled-space norms)
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                if (term[gi] || !adapt_c[gi]) continue;
                const T pr = ax_z[gi] / (tt_max(zn_r[gi], axn_r[gi]) + T(kDivisionTol));
                const T dn = tt_max(tt_max(qn_r[gi], atyn_r[gi]), pxn_r[gi]);
                const T du = dr_r[gi] / (dn + T(kDivisionTol));
                T rn = rho[gi] * (T)sqrt((double)(pr / (du + T(kDivisionTol))));
                rn = tt_min(tt_max(rn, T(kRhoMin)), T(kRhoMax));
                if (rn > rho[gi] * (T)st.adaptive_rho_tolerance || rn < rho[gi] / (T)st.adaptive_rho_tolerance) {
                    rho[gi] = tt_min(tt_max(rn, T(kRhoMin)), T(kRhoMax));
                    rinv[gi] = T(1) / rho[gi];
                }
            }
            set_dk();  // uniform; unchanged rho gives the same dk bit for bit
        }
        if (last) {  // after the ADMM loop (osqp_solve)
            int s1[G], s2[G];
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                need[gi] = !term[gi] && last_c[gi];
                s1[gi] = kUnsolved;
            }
            if (!at_check) check_termination(false, need, s1);
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                if (!term[gi] && s1[gi] != kUnsolved) { status[gi] = s1[gi]; term[gi] = true; }
                need[gi] = !term[gi] && last_c[gi];
            }
            check_termination(true, need, s2);
#pragma unroll
            for (int gi = 0; gi < G; gi++)
                if (!term[gi] && last_c[gi]) { status[gi] = s2[gi] != kUnsolved ? s2[gi] : kMaxIterReached; term[gi] = true; }
        }
        MPCQ_INFO_MARK(4);
        {
            bool newly[G], any = false;
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                newly[gi] = term[gi] && !done[gi];
                any = any || newly[gi];
            }
            if (wave_any(any)) finalize(newly, Uold);
#pragma unroll
            for (int gi = 0; gi < G; gi++) done[gi] = term[gi];
        }
        if (refill && at_check) stream_next();
        MPCQ_INFO_MARK(6);
        MPCQ_INFO_MARK(5);
#if defined(MPCQ_INFO_STAMPS) && !defined(MPCQ_INFO_PART)
        if (a.stamps) info_cycles += (long long)__builtin_amdgcn_s_memtime() - t_info;
#endif
        if (it == stop && !all_done()) {
            MPCQ_TSTAMP(3, (long long)__builtin_amdgcn_s_memtime());
            // phase boundary: save the running QPs and list them for the next launch (the kernel
            // boundary publishes the stores; the XCD's L2 merges a QP row's 16-32 B pieces)
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                const bool run = !done[gi];
                const int b = opaque(b_[gi]);
                // (lane offset and pointers re-derived here, as in the finalize: nothing of this cold path is
                // hoisted and held across the hot loop)
                const int g = opaque((int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u))) >> 4;
                T *const o_xs = fresh_ptr(a.xs), *const o_zs = fresh_ptr(a.zs), *const o_ys = fresh_ptr(a.ys);
                if (run) {
#pragma unroll
                    for (int s = 0; s < NS; s++)
                        if (s < KN) o_xs[(size_t)b * ncs + 4 * s + g] = xs[gi][s];
#pragma unroll
                    for (int s = 0; s < MS; s++)
                        if (s < KM) {
                            o_zs[(size_t)b * mcs + 4 * s + g] = z[gi][s];
                            o_ys[(size_t)b * mcs + 4 * s + g] = y[gi][s];
                        }
                    if (g == 0) {
                        fresh_ptr(a.rhos)[b] = rho[gi];
                        fresh_ptr(a.it_state)[b] = opaque(it);  // (it == stop here: no VGPR copy of stop held)
                    }
                }
            }
            unsigned long long mask[G];
            unsigned total = 0;
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                mask[gi] = __ballot(!done[gi] && g == 0);
                total += (unsigned)__popcll(mask[gi]);
            }
            int base = 0;
            if (lane == 0) base = atomicAdd(a.count_out + (blockIdx.x % ListSeg::kShards) * ListSeg::kStride, (int)total);
            base = __shfl(base, 0);
            int *const qout = a.list_out + (blockIdx.x % ListSeg::kShards) * a.list_seg;
#pragma unroll
            for (int gi = 0; gi < G; gi++) {
                // the column's g = 0 lane is lane c: the mask's bits below it by mbcnt (no lane mask held)
                int pos = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask[gi] >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((unsigned)mask[gi], 0u));
#pragma unroll
                for (int gj = 0; gj < gi; gj++) pos += __popcll(mask[gj]);
                if (!done[gi] && g == 0) qout[pos] = opaque(b_[gi]);
            }
            break;
        }
    }
#ifndef MPCQ_PRO_PART
    MPCQ_TSTAMP(5, info_cycles);  // cycles in info iterations (checks, adapt, stop)
#endif
    };  // run_group

    // this wave's 16 G QPs: slots wave_slot.. of the launch's list (or of the batch in phase 0); a
    // stream wave holds a.sim.cpw plants in its first columns
    const int cpw = refill ? a.sim.cpw : 16 * G;
    const int wave_slot = (blk * WPB + (threadIdx.x >> 6)) * cpw;
    if (wave_slot < count) {
        bool valid[G];
        int b_[G];
#pragma unroll
        for (int gi = 0; gi < G; gi++) {
            const int slot = wave_slot + 16 * gi + c;
            valid[gi] = slot < count && (!refill || c < cpw);
            const int i = slot + (seglist ? seg * a.list_seg : 0);  // list entry
            int qp = a.qp0 + i;
            if (seglist) {
                qp = a.list_in[i];
            } else if (ordered && valid[gi]) {
                qp = a.ord_list[i];
                qp = qp < 0 ? 0 : (qp >= a.batch ? a.batch - 1 : qp);  // (the list holds batch indices only)
            }
            b_[gi] = valid[gi] ? qp : 0;
        }
        run_group(b_, valid);
    }
    MPCQ_TSTAMP(4, (long long)__builtin_amdgcn_s_memtime());
    MPCQ_TSTAMP(7, (long long)__builtin_amdgcn_s_memrealtime());
}

// Launch one tile-kernel variant: one workgroup per 64 G QPs of the phase's grid.
// lds_pad: dynamic LDS bytes on top of the kernel's static allocation (0, or enough that fewer
// workgroups fit a CU: the occupancy A/B below)
template <typename T, int KN, int KM, bool AI, bool LF, int G, int OCC, bool PAIRED = false, int WPB = 4, bool MIX = false>
int tile_launch_variant(const AdmmArgs<T> &a, hipStream_t s, unsigned lds_pad = 0)
{
    constexpr int QPW = 16 * G * WPB;
    const int blocks = (a.batch + QPW - 1) / QPW;
    hipLaunchKernelGGL((admm_tile_kernel<T, KN, KM, AI, LF, G, OCC, PAIRED, WPB, false, MIX>), dim3(blocks), dim3(64 * WPB),
                       lds_pad, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// The receding-horizon stream in one launch (AdmmArgs::sim): the paired condensed-MPC shape only
// (-1 otherwise: the caller replays per-step launches).
template <typename T, int KN, int KM>
int tile_stream_launch(const AdmmArgs<T> &a, hipStream_t s)
{
    if constexpr (KM == 2 * KN) {
        if (a.paired && a.all_ineq && a.lower_free) {
            // (a stream is latency-bound: few waves.  Compiled for two waves per SIMD (its plant and check code
            // spill, outside the hot loop), or with StreamArgs::occ 1 for one: the whole register file, no
            // spills, but slower (mpcq_api.cpp launch_tile_stream))
            constexpr int WPB = 4;
            const int waves = (a.batch + a.sim.cpw - 1) / a.sim.cpw;
            const dim3 grid((waves + WPB - 1) / WPB), block(64 * WPB);
            if constexpr (std::is_same<T, double>::value) {
                if (a.mix_r > 0) {  // MPCQ_F64_MIXED: each step's plain iterations before the last mix_r in fp32
                    if (a.sim.occ == 1)
                        hipLaunchKernelGGL((admm_tile_kernel<T, KN, KM, true, true, 1, 1, true, WPB, true, true>), grid, block, 0, s, a);
                    else
                        hipLaunchKernelGGL((admm_tile_kernel<T, KN, KM, true, true, 1, 2, true, WPB, true, true>), grid, block, 0, s, a);
                    return hipGetLastError() == hipSuccess ? 0 : -2;
                }
            }
            if (a.sim.occ == 1)
                hipLaunchKernelGGL((admm_tile_kernel<T, KN, KM, true, true, 1, 1, true, WPB, true>), grid, block, 0, s, a);
            else
                hipLaunchKernelGGL((admm_tile_kernel<T, KN, KM, true, true, 1, 2, true, WPB, true>), grid, block, 0, s, a);
            return hipGetLastError() == hipSuccess ? 0 : -2;
        }
    }
    return -1;
}

// One variant per shape and type (measured A/B): f32 runs one 16-QP group per
// wave at 3 waves/SIMD, f64 at 2 (2 groups per wave, 4 waves/SIMD and 8-wave workgroups were slower).
template <typename T, int KN, int KM>
int tile_launch(const AdmmArgs<T> &a, hipStream_t s)
{
    constexpr int OCC = sizeof(T) == 8 ? 2 : 3;
    if constexpr (KM == 2 * KN) {
        if (a.paired && a.all_ineq && a.lower_free) {  // the condensed-MPC shape: paired, VGPR-resident loop
            if constexpr (std::is_same<T, double>::value) {
                if (a.mix_r > 0) return tile_launch_variant<T, KN, KM, true, true, 1, OCC, true, 4, true>(a, s);
            } else {
                // f32 at 2 waves/SIMD (AdmmArgs::tile_occ): a batch of 2 k rounds of 2,048 wave slots runs
                // without the lone-wave last round 3 waves/SIMD leave (4,096 waves on 3,072 slots); the
                // registers allow 3, so dynamic LDS holds a CU to 2 workgroups (> 160 KiB / 3 each)
                if (a.tile_occ == 2) return tile_launch_variant<T, KN, KM, true, true, 1, OCC, true>(a, s, 16 * 1024);
            }
            return tile_launch_variant<T, KN, KM, true, true, 1, OCC, true>(a, s);
        }
    }
    if (a.all_ineq && a.lower_free) return tile_launch_variant<T, KN, KM, true, true, 1, OCC>(a, s);
    return tile_launch_variant<T, KN, KM, false, false, 1, 2>(a, s);
}

// Lazily published solution of a tile solve (osqp store_solution, read by getSolution :105 only when a
// caller asks: mpcq_api.cpp materialize_xy).  The tile finalize stores the warm state x' (W-basis), z, y,
// rho, status and U += x(0); x = D W x' and y = E y / c are formed here, for every QP, with the finalize's
// own arithmetic (the same MFMA product of the same W image, the same roundings): bit for bit what an eager
// finalize would have written.  One 16-QP column group per wave, index order.
template <typename T, int KN, int KM, bool PAIRED>
__global__ __launch_bounds__(256) void tile_publish_kernel(AdmmArgs<T> a)
{
    constexpr int VEC = 16 / sizeof(T);
    constexpr TileLayout L = TileLayout::make(KN, KM, VEC, PAIRED);
    constexpr size_t IMG0 = PAIRED ? TileLayout::make(KN, KM, VEC, false).total : 0;
    constexpr int NT = L.NT, MT = L.MT, KNP = L.KNP;
    constexpr int NS = 4 * NT, MS = 4 * MT, NCP = 16 * NT, MCP = 16 * MT;
    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int w = (int)blockIdx.x * 4 + ((int)threadIdx.x >> 6);
    if (16 * w >= a.batch) return;  // (wave-uniform)
    const int b = 16 * w + c;
    const bool valid = b < a.batch;
    const int bb = valid ? b : a.batch - 1;
    const int n = a.n, m = a.m;
    T xs[1][NS], xh[1][NS];
#pragma unroll
    for (int s = 0; s < NS; s++) xs[0][s] = s < KN ? a.xs[(size_t)bb * NCP + 4 * s + g] : T(0);
    tile_mv_g<T, 1, NT, KN, KNP>(a.img + IMG0 + L.W, xs, xh, lane, nullptr);
    if (!valid) return;
    const int sta = a.status[b];
    const bool has_sol = sta == kSolved || sta == kSolvedInaccurate || sta == kMaxIterReached;
    const double cinv64 = (double)a.ops.cs[1];
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const int v = 4 * s + g;
        if (s < KN && v < n) a.x[(size_t)b * n + v] = has_sol ? (double)xh[0][s] * (double)a.ops.D[v] : __builtin_nan("");
    }
#pragma unroll
    for (int s = 0; s < MS; s++) {
        const int v = 4 * s + g;
        if (s < KM && v < m)
            a.y[(size_t)b * m + v] = has_sol ? ((double)a.ys[(size_t)b * MCP + 4 * s + g] * (double)a.ops.E[v]) * cinv64
                                             : __builtin_nan("");
    }
}

template <typename T, int KN, int KM>
int tile_publish(const AdmmArgs<T> &a, bool paired, hipStream_t s)
{
    const int waves = (a.batch + 15) / 16;
    if (paired && KM == 2 * KN)
        hipLaunchKernelGGL((tile_publish_kernel<T, KN, KM, KM == 2 * KN>), dim3((waves + 3) / 4), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((tile_publish_kernel<T, KN, KM, false>), dim3((waves + 3) / 4), dim3(256), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Compiled (KN, KM) = (ceil(n/4), ceil(m/4)): the reference horizons N = 15 (n 15, m 30) and N = 20
// (n 20, m 40), plus two small shapes for the generic-QP tests.
#define MPCQ_TILE_SHAPES(X) X(1, 1) X(2, 3) X(4, 8) X(5, 10)

template <typename T>
int tile_launch_any(const AdmmArgs<T> &a, int KN, int KM, hipStream_t s)
{
#define MPCQ_TRY(KN_, KM_) if (KN == KN_ && KM == KM_) return tile_launch<T, KN_, KM_>(a, s);
    MPCQ_TILE_SHAPES(MPCQ_TRY)
#undef MPCQ_TRY
    return -1;
}

template <typename T>
int tile_publish_any(const AdmmArgs<T> &a, int KN, int KM, bool paired, hipStream_t s)
{
#define MPCQ_TRY(KN_, KM_) if (KN == KN_ && KM == KM_) return tile_publish<T, KN_, KM_>(a, paired, s);
    MPCQ_TILE_SHAPES(MPCQ_TRY)
#undef MPCQ_TRY
    return -1;
}

template <typename T>
int tile_stream_launch_any(const AdmmArgs<T> &a, int KN, int KM, hipStream_t s)
{
#define MPCQ_TRY(KN_, KM_) if (KN == KN_ && KM == KM_) return tile_stream_launch<T, KN_, KM_>(a, s);
    MPCQ_TILE_SHAPES(MPCQ_TRY)
#undef MPCQ_TRY
    return -1;
}

}  // namespace mpcq
