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
// max / max of magnitudes as single v_max instructions (|.| as a source modifier).  LLVM's maxnum adds a
// canonicalising v_max x, x per operand here; on the finite, non-NaN values these norms and scalings see
// the results are the same (max is exact).
__device__ __forceinline__ double hwmax(double a, double b)
{
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float hwmax(float a, float b)
{
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double hwmax_abs(double m, double x)  // max(m, |x|)
{
    double r;
    asm("v_max_f64 %0, %1, |%2|" : "=v"(r) : "v"(m), "v"(x));
    return r;
}
__device__ __forceinline__ double hwmax_abs2(double x, double y)  // max(|x|, |y|)
{
    double r;
    asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
template <typename T> __device__ __forceinline__ T hmax(T v)
{
    return half_reduce(v, [](T a, T b) { return hwmax(a, b); });
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

// DPP move whose lanes without a source (row shifts) or outside the row mask RM read 0.  With every row
// enabled the zero comes from bound_ctrl (no old value: no zeroing move before each DPP move).
template <int CTRL, int RM> __device__ __forceinline__ unsigned dpp0_u(unsigned v)
{
    if constexpr (RM == 0xF) return (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
    else return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xF, false);
}
template <int CTRL, int RM = 0xF> __device__ __forceinline__ float dpp0(float v)
{
    return __uint_as_float(dpp0_u<CTRL, RM>(__float_as_uint(v)));
}
template <int CTRL, int RM = 0xF> __device__ __forceinline__ double dpp0(double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = dpp0_u<CTRL, RM>((unsigned)u), hi = dpp0_u<CTRL, RM>((unsigned)(u >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ float readlane_t(float v, int l)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double readlane_t(double v, int l)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// Inclusive scans over the 32 lanes of each half (lane r = horizon step r), op with identity 0 (sums,
// maxima of non-negative values).  Prefix: row_shr 1, 2, 4, 8 inside the 16-lane rows, then
// row_bcast:15 into rows 1 and 3.  Suffix: row_shl 1, 2, 4, 8, then rows 0 and 2 take lane 16's /
// lane 48's total.  Call with the whole wave active (DPP and readlane read other lanes).
template <typename T, typename F> __device__ __forceinline__ T half_prefix(T v, F op)
{
    v = op(v, dpp0<0x111>(v));
    v = op(v, dpp0<0x112>(v));
    v = op(v, dpp0<0x114>(v));
    v = op(v, dpp0<0x118>(v));
    return op(v, dpp0<0x142, 0xA>(v));
}
template <typename T, typename F> __device__ __forceinline__ T half_suffix(T v, F op, int lane)
{
    v = op(v, dpp0<0x101>(v));
    v = op(v, dpp0<0x102>(v));
    v = op(v, dpp0<0x104>(v));
    v = op(v, dpp0<0x108>(v));
    const T s0 = readlane_t(v, 16), s1 = readlane_t(v, 48);
    return (lane & 16) ? v : op(v, (lane & 32) ? s1 : s0);
}
template <typename T> __device__ __forceinline__ T psum(T v) { return half_prefix(v, [](T a, T b) { return a + b; }); }
template <typename T> __device__ __forceinline__ T ssum(T v, int lane)
{
    return half_suffix(v, [](T a, T b) { return a + b; }, lane);
}

// ---- plants per wave (LAY).  LAY 2: two plants, one per 32-lane half, lane r of a half = horizon step r
// (the functions above).  LAY 3 (N <= 20): three plants, plant h on row h (lanes 16 h .. 16 h + 15: steps
// 0 .. 15) and steps 16 .. 19 interleaved over row 3 (step 16 + k at lane 48 + 4 k + h; lanes 48 + 4 k + 3
// hold no plant), so 60 of 64 lanes carry a step.  The scans and reductions keep the association of the
// two-plant layout: the row part runs the same DPP steps (rows 0 .. 2 only where row 3 would mix plants),
// the interleaved steps 16 .. 19 combine with row shifts by 4 and 8 lanes (one step apart, two steps
// apart), and the carry between a plant's row and its tail crosses rows by ds_bpermute (the LDS crossbar:
// no VALU issue).  Lanes of no plant hold 0 in every scan input (their predicates are false), and lane 63
// is the zero every other lane's carry reads; they count in plant 2's slot and take plant 2's reductions,
// so their decisions (status, `done`) are plant 2's.  Lane 63 feeds every plant's carry, so the lanes of no
// plant must hold exact, finite zeros whatever plant 2's data: they read a broadcast slot of their own (never
// written: zero), their M^-1 rows are zeroed after the inverse and their K0 is 0, so x~, z~, y and w stay 0
// on them even when plant 2 is non-finite (a NaN there would otherwise reach plants 0 and 1 through 0 * NaN).
__device__ __forceinline__ bool lay3_noplant(int lane) { return (lane & 51) == 51; }
__device__ __forceinline__ int lay3_plant(int lane) { return lane < 48 ? lane >> 4 : ((lane & 3) == 3 ? 2 : lane & 3); }
__device__ __forceinline__ int lay3_row(int lane) { return lane < 48 ? lane & 15 : ((lane & 3) == 3 ? 32 : 16 + ((lane >> 2) & 3)); }
template <int LAY> __device__ __forceinline__ int lay_plant(int lane) { return LAY == 3 ? lay3_plant(lane) : lane >> 5; }
template <int LAY> __device__ __forceinline__ int lay_row(int lane) { return LAY == 3 ? lay3_row(lane) : lane & 31; }

// DPP move under row / bank masks: lanes of a disabled row or bank keep `old`; bound_ctrl: a lane whose
// source lies outside its row reads 0
template <int CTRL, int RM, int BM> __device__ __forceinline__ float dppm(float old, float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, RM, BM, true));
}
template <int CTRL, int RM, int BM> __device__ __forceinline__ double dppm(double old, double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v), o = (unsigned long long)__double_as_longlong(old);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)o, (int)(unsigned)u, CTRL, RM, BM, true);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)(o >> 32), (int)(unsigned)(u >> 32), CTRL, RM, BM, true);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// the value of v at lane src (src4 = 4 src): ds_bpermute
__device__ __forceinline__ float lane_fetch(float v, int src4)
{
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src4, __float_as_int(v)));
}
__device__ __forceinline__ double lane_fetch(double v, int src4)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(src4, (int)(unsigned)u);
    const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(src4, (int)(unsigned)(u >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// LAY 3 inclusive prefix / suffix over a plant's steps (op with identity 0, as half_prefix / half_suffix).
// The one- and two-step shifts run on rows 0 .. 2 only, and a disabled row keeps the DPP destination's old
// value, which must be 0 there: `z` is a register whose row-3 lanes hold 0 and stay 0 (every write to it is
// one of these row-masked moves), so the moves take it as their old operand in place instead of a freshly
// zeroed copy (two v_mov per step and half of a 64-bit value).  Callers in the solve loop keep one z across
// iterations.
template <typename T, typename F> __device__ __forceinline__ T lay3_prefix(T v, F op, int lane, T &z)
{
    z = dppm<0x111, 0x7, 0xF>(z, v);  // row_shr 1, 2: rows 0 .. 2 only (row 3 reads z's 0)
    v = op(v, z);
    z = dppm<0x112, 0x7, 0xF>(z, v);
    v = op(v, z);
    v = op(v, dppm<0x114, 0xF, 0xF>(T(0), v));  // row_shr 4, 8: rows 0 .. 2, and row 3's steps 16 + k - 1, - 2
    v = op(v, dppm<0x118, 0xF, 0xF>(T(0), v));
    // a tail lane adds its plant's row total (lane 16 h + 15); row lanes read lane 63's zero
    const int src = lane >= 48 ? 16 * (lane & 3) + 15 : 63;
    return op(v, lane_fetch(v, 4 * src));
}
template <typename T, typename F> __device__ __forceinline__ T lay3_suffix(T v, F op, int lane, T &z)
{
    z = dppm<0x101, 0x7, 0xF>(z, v);  // row_shl 1, 2: rows 0 .. 2 only
    v = op(v, z);
    z = dppm<0x102, 0x7, 0xF>(z, v);
    v = op(v, z);
    v = op(v, dppm<0x104, 0xF, 0xF>(T(0), v));  // row_shl 4, 8: and row 3's steps 16 + k + 1, + 2
    v = op(v, dppm<0x108, 0xF, 0xF>(T(0), v));
    // a row lane adds its plant's tail suffix (step 16: lane 48 + h); tail lanes read lane 63's zero
    const int src = lane < 48 ? 48 + (lane >> 4) : 63;
    return op(v, lane_fetch(v, 4 * src));
}
template <typename T, typename F> __device__ __forceinline__ T lay3_prefix(T v, F op, int lane)
{
    T z = T(0);
    return lay3_prefix(v, op, lane, z);
}
template <typename T, typename F> __device__ __forceinline__ T lay3_suffix(T v, F op, int lane)
{
    T z = T(0);
    return lay3_suffix(v, op, lane, z);
}
// LAY 3 reduction over a plant's steps, every lane of the plant ending on the same bits (as half_reduce:
// the row butterfly, the tail's pairs (16, 17), (18, 19) then their sum, then row total op tail total)
template <typename T, typename F> __device__ __forceinline__ T lay3_reduce(T v, F op, int lane)
{
    v = op(v, dppm<0xB1, 0x7, 0xF>(T(0), v));   // quad_perm [1,0,3,2]     (rows 0 .. 2)
    v = op(v, dppm<0x4E, 0x7, 0xF>(T(0), v));   // quad_perm [2,3,0,1]
    v = op(v, dppm<0x141, 0x7, 0xF>(T(0), v));  // row_half_mirror
    v = op(v, dppm<0x140, 0x7, 0xF>(T(0), v));  // row_mirror
    T t = dppm<0x12C, 0x8, 0x5>(T(0), v);       // row 3: steps 16, 18 (banks 0, 2) take 17, 19 (row_ror 12) ...
    t = dppm<0x124, 0x8, 0xA>(t, v);            // ... and 17, 19 (banks 1, 3) take 16, 18 (row_ror 4)
    v = op(v, t);
    v = op(v, dppm<0x128, 0x8, 0xF>(T(0), v));  // row 3: (16 + 17) with (18 + 19) (row_ror 8)
    const int src = lane < 48 ? 48 + (lane >> 4) : ((lane & 3) == 3 ? 63 : 16 * (lane & 3));
    v = op(v, lane_fetch(v, 4 * src));
    // a lane of no plant counts in plant 2's slot: it takes plant 2's result and so decides with plant 2
    // (its status and `done` must not hold the wave)
    return lane_fetch(v, 4 * ((lane & 51) == 51 ? 32 : lane));
}
template <int LAY, typename T> __device__ __forceinline__ T l_psum(T v, int lane)
{
    if constexpr (LAY == 3) return lay3_prefix(v, [](T a, T b) { return a + b; }, lane);
    else return psum(v);
}
template <int LAY, typename T> __device__ __forceinline__ T l_ssum(T v, int lane)
{
    if constexpr (LAY == 3) return lay3_suffix(v, [](T a, T b) { return a + b; }, lane);
    else return ssum(v, lane);
}
// (the solve loop's forms: z as in lay3_prefix, unused by the two-plant layout)
template <int LAY, typename T> __device__ __forceinline__ T l_psum(T v, int lane, T &z)
{
    if constexpr (LAY == 3) return lay3_prefix(v, [](T a, T b) { return a + b; }, lane, z);
    else return psum(v);
}
template <int LAY, typename T> __device__ __forceinline__ T l_ssum(T v, int lane, T &z)
{
    if constexpr (LAY == 3) return lay3_suffix(v, [](T a, T b) { return a + b; }, lane, z);
    else return ssum(v, lane);
}
template <int LAY, typename T> __device__ __forceinline__ T l_prefix_max(T v, int lane)
{
    if constexpr (LAY == 3) return lay3_prefix(v, [](T a, T b) { return hwmax(a, b); }, lane);
    else return half_prefix(v, [](T a, T b) { return hwmax(a, b); });
}
template <int LAY, typename T> __device__ __forceinline__ T l_suffix_max(T v, int lane)
{
    if constexpr (LAY == 3) return lay3_suffix(v, [](T a, T b) { return hwmax(a, b); }, lane);
    else return half_suffix(v, [](T a, T b) { return hwmax(a, b); }, lane);
}
// LAY 3 maximum over a plant's steps: max is exact in any order, so the tail folds into the row first (row
// lane r < 4 takes step 16 + r by ds_bpermute), the row butterfly needs no masks (row 3 is ignored), and
// the tail lanes read their row's result back
template <typename T> __device__ __forceinline__ T lay3_max(T v, int lane)
{
    const int src_in = (lane < 48 && (lane & 15) < 4) ? 48 + 4 * (lane & 15) + (lane >> 4) : lane;
    v = hwmax(v, lane_fetch(v, 4 * src_in));
    v = hwmax(v, dpp_t<0xB1>(v));   // quad_perm [1,0,3,2]
    v = hwmax(v, dpp_t<0x4E>(v));   // quad_perm [2,3,0,1]
    v = hwmax(v, dpp_t<0x141>(v));  // row_half_mirror
    v = hwmax(v, dpp_t<0x140>(v));  // row_mirror
    const int src_out = lane < 48 ? lane : 16 * lay3_plant(lane);  // (a lane of no plant: plant 2's)
    return lane_fetch(v, 4 * src_out);
}
template <int LAY, typename T> __device__ __forceinline__ T l_max(T v, int lane)
{
    if constexpr (LAY == 3) return lay3_max(v, lane);
    else return hmax(v);
}
template <int LAY, typename T> __device__ __forceinline__ T l_sum(T v, int lane)
{
    if constexpr (LAY == 3) return lay3_reduce(v, [](T a, T b) { return a + b; }, lane);
    else return hsum(v);
}
template <int LAY> __device__ __forceinline__ bool l_any(bool p, int lane)  // any lane of this lane's plant
{
    const unsigned long long b = __ballot(p);
    if constexpr (LAY == 3) {
        const int h = lay3_plant(lane);
        return (b & ((0xFFFFull << (16 * h)) | (0x1111ull << (48 + h)))) != 0ull;
    } else {
        return ((lane & 32) ? (b >> 32) : (b & 0xffffffffull)) != 0ull;
    }
}

// Batched reductions over a plant's steps through LDS (the checks' norms and sums): every lane of a step r
// writes its K values to the plant's rows red[j][r]; lane j of the plant's first 16-lane row reduces row j
// over the NC steps (dead steps hold 0) — a maximum from 0 with v_max (skipping NaN, as OSQP's
// vec_norm_inf), or, for bit j of SUM set, a sum in four interleaved partials, (s0 + s1) + (s2 + s3) — and
// writes it back to red[j][0], which every lane then reads.  One LDS round trip and ~20 VALU for up to
// four reductions, where a DPP / permute reduction costs ~15 VALU and two LDS permutes each.  The same
// order in both layouts (LAY 2 and 3 give the same bits).  Call with the whole wave active.
template <int LAY, int NC, int K, unsigned SUM>
__device__ __forceinline__ void lay_reduce_k(double *red, double (&v)[K], int r, int lane)
{
    static_assert(K >= 1 && K <= 4 && NC % 2 == 0, "four work rows of NC steps");
    if (r < NC) {
#pragma unroll
        for (int j = 0; j < K; j++) red[j * NC + r] = v[j];
    }
    wave_sync();
    const int jr = LAY == 3 ? (lane < 48 ? (lane & 15) : 16) : (lane & 31);
    if (jr < K) {
        const double *row = red + jr * NC;
        double a[4] = {0.0, 0.0, 0.0, 0.0};
        if ((SUM >> jr) & 1u) {
#pragma unroll
            for (int k = 0; k < NC; k += 2) {
                const double2 x = *(const double2 *)(row + k);
                a[k & 3] += x.x;
                a[(k + 1) & 3] += x.y;
            }
            a[0] = (a[0] + a[1]) + (a[2] + a[3]);
        } else {
#pragma unroll
            for (int k = 0; k < NC; k += 2) {
                const double2 x = *(const double2 *)(row + k);
                a[k & 3] = hwmax(a[k & 3], x.x);
                a[(k + 1) & 3] = hwmax(a[(k + 1) & 3], x.y);
            }
            a[0] = hwmax(hwmax(a[0], a[1]), hwmax(a[2], a[3]));
        }
        red[jr * NC] = a[0];
    }
    wave_sync();
#pragma unroll
    for (int j = 0; j < K; j++) v[j] = red[j * NC];
    wave_sync();
}

// Per plant in LDS (fp64).  P^ is kept as its packed upper triangle (row i holds columns i .. N-1 at
// i NC - i (i - 1) / 2): OSQP's own P, one copy of each entry.  Union region u: first the condensing
// recurrences' histories V, Cr, then the lag table G (packed like P: G(d, T) for d + T < N), then P^ and
// the vectors Dv .. Di, each written once what it overlaps is dead.  Work region w (4 NC): CS and tmp while
// the plant is condensed and scaled, the pivot row of a Gauss-Jordan step, and the batched reductions of
// the checks (lay_reduce_k) — never live at the same time.
template <int NC> struct PlantLds {
    static constexpr int NP = NC * (NC + 1) / 2;
    static constexpr int NV = NP + 8 * NC;
    static constexpr int NU = (NC + 1) * 16 > NV ? (NC + 1) * 16 : NV;
    static_assert(NP % 2 == 0 && NU % 2 == 0, "16-B aligned vectors");
    double u[NU];
    double w[4 * NC];
    double sh[6];  // cost, 1 / cost, U, K0, max |q^|, max |D^-1 q^| (the checks' constant norms)
    __device__ double *V() { return u; }
    __device__ double *Cr() { return u + (NC + 1) * 8; }
    __device__ double *G() { return u; }
    __device__ double *Ph() { return u; }
    __device__ double *Dv() { return u + NP; }
    __device__ double *Ev() { return u + NP + NC; }
    __device__ double *SE() { return u + NP + 2 * NC; }
    __device__ double *qh() { return u + NP + 3 * NC; }
    __device__ double *Ut() { return u + NP + 4 * NC; }
    __device__ double *Ub() { return u + NP + 5 * NC; }
    __device__ double *Ei() { return u + NP + 6 * NC; }  // 1 / E, 1 / D (OSQP's Einv, Dinv; 1 beyond N)
    __device__ double *Di() { return u + NP + 7 * NC; }
    __device__ double *piv() { return w; }
    __device__ double *red() { return w; }
    __device__ double *CS() { return w + NC; }
    __device__ double *tmp() { return w + 2 * NC; }
    __device__ const double *Ei() const { return u + NP + 6 * NC; }
    __device__ const double *Di() const { return u + NP + 7 * NC; }
    __device__ const double *Dv() const { return u + NP; }
    __device__ const double *Ev() const { return u + NP + NC; }
    __device__ const double *qh() const { return u + NP + 3 * NC; }
    __device__ const double *Ut() const { return u + NP + 4 * NC; }
    __device__ const double *Ub() const { return u + NP + 5 * NC; }
    // packed upper-triangle index of (i, j), i, j < NC
    __device__ static int pk(int i, int j)
    {
        const int a = i < j ? i : j, b = i < j ? j : i;
        return a * NC - (a * (a - 1)) / 2 + (b - a);
    }
    // the same for row r's element i with q = row_q(r): an unrolled walk over i then costs one select per
    // element (both forms are a register plus a constant)
    __device__ static int row_q(int r) { return r * NC - (r * (r - 1)) / 2 - r; }
    __device__ static int pk_row(int r, int i, int q) { return i < r ? i * NC - (i * (i - 1)) / 2 - i + r : q + i; }
};

// Gauss-Jordan inverse of this plant's SPD matrix (n x n; SPD: no pivoting) on pivot pairs K = {k, k + 1},
// lane r holding row r in registers.  The two owners publish rows p0 = row k, p1 = row k + 1 through LDS
// (one wave: the DS queue keeps the order, wave_sync only pins the compiler's); every lane forms
// A_KK^-1 = [d, -b; -b, a] / (a d - b^2) from them and updates its row without a branch:
//     row <- fma(-g0, p0, fma(-g1, p1, s row)),   row[k], row[k + 1] <- -g0, -g1,
// with s = 1, [g0 g1] = [row[k] row[k + 1]] A_KK^-1 on the other rows (A - A(:,K) A_KK^-1 A(K,:), columns K
// -A(:,K) A_KK^-1) and s = 0, [g0 g1] = -(row k or k + 1 of A_KK^-1) on the pivot rows (rows K <- A_KK^-1
// A(K,:), whose columns K are then A_KK^-1).  Half the serial LDS round trips of one pivot per step and
// three VALU per element per pair where single pivots take four.  An odd n ends on a single pivot.
template <int NC>
__device__ __forceinline__ bool gj_rows(double (&row)[NC], double *piv, int n, int r)
{
    bool ok = true;
#pragma unroll
    for (int k = 0; k < NC; k += 2) {
        if (k >= n) continue;  // (uniform; continue keeps the loop fully unrollable)
        const bool pair = k + 1 < n;
        if (r == k || (pair && r == k + 1)) {
            double *dst = piv + (r - k) * NC;
#pragma unroll
            for (int j = 0; j < NC; j += 2) *(double2 *)(dst + j) = make_double2(row[j], row[j + 1]);
        }
        wave_sync();
        const double *p0 = piv, *p1 = piv + NC;
        const double a = p0[k];
        double g0, g1, sc;
        if (pair) {
            const double b = p0[k + 1], d = p1[k + 1];
            const double det = fma(a, d, -(b * b));
            if (!(a > 0.0) || !(det > 0.0)) ok = false;
            // 1 / det by v_rcp_f64 and two Newton steps (within an ulp; the inverse is compared with the oracle's
            // LDL solve at tolerance, not bitwise)
            double id = __builtin_amdgcn_rcp(det);
            id = fma(id, fma(-det, id, 1.0), id);
            id = fma(id, fma(-det, id, 1.0), id);
            const double ikk = d * id, ikl = -b * id, ill = a * id;
            const double f0 = row[k], f1 = row[k + 1];
            const bool pk0 = r == k, pk1 = r == k + 1;
            sc = (pk0 || pk1) ? 0.0 : 1.0;
            g0 = pk0 ? -ikk : pk1 ? -ikl : fma(f0, ikk, f1 * ikl);
            g1 = pk0 ? -ikl : pk1 ? -ill : fma(f0, ikl, f1 * ill);
        } else {  // the last pivot of an odd n
            if (!(a > 0.0)) ok = false;
            double ip = __builtin_amdgcn_rcp(a);
            ip = fma(ip, fma(-a, ip, 1.0), ip);
            ip = fma(ip, fma(-a, ip, 1.0), ip);
            const bool pk0 = r == k;
            sc = pk0 ? 0.0 : 1.0;
            g0 = pk0 ? -ip : row[k] * ip;
            g1 = 0.0;
        }
#pragma unroll
        for (int j = 0; j < NC; j += 2) {
            const double2 m0 = *(const double2 *)(p0 + j);
            const double2 m1 = *(const double2 *)(p1 + j);
            const double q0[2] = {m0.x, m0.y}, q1[2] = {m1.x, m1.y};
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const int jj = j + e;
                if (jj == k) row[jj] = -g0;
                else if (jj == k + 1 && pair) row[jj] = -g1;
                else if (pair) row[jj] = fma(-g0, q0[e], fma(-g1, q1[e], row[jj] * sc));
                else row[jj] = fma(-g0, q0[e], row[jj] * sc);
            }
        }
        wave_sync();
    }
    return ok;
}

// Stage clock stamps of a debug build (-DMPCQ_PLANT_STAMPS, tools/plant_stamps.py): 16 per wave
#ifdef MPCQ_PLANT_STAMPS
#define MPCQ_PSTAMP(k, v)                                                              \
    do {                                                                               \
        if (a.stamps && threadIdx.x == 0) a.stamps[(size_t)blockIdx.x * 16 + (k)] = (v); \
    } while (0)
#else
#define MPCQ_PSTAMP(k, v) \
    do {                  \
    } while (0)
#endif
#define MPCQ_PTIME(k) MPCQ_PSTAMP(k, (long long)__builtin_amdgcn_s_memtime())

// WPE: waves per SIMD the register allocation is held to (2, or 3 for A/B: MPCQ_PLANT_WPE); LAY: plants per
// wave (2: one per 32-lane half; 3: N <= 20, rows plus interleaved tails, see lay3_*)
template <typename T, int NC, int WPE, int LAY, int NXC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NC <= 20 ? WPE : 2, NC <= 20 ? 8 : 4))) void plant_step_kernel(PlantStepArgs a)
{
    static_assert(NXC == 4 || NXC == 8, "states: nx <= 4 (the cart-pole of the reference) or <= 8");
    static_assert(NC % 4 == 0, "broadcast rows are read 16 B at a time");
    static_assert(LAY == 2 || (LAY == 3 && NC <= 20), "three plants per wave: N <= 20");
    using PL = PlantLds<NC>;
    __shared__ PL lds[LAY];
    // per-plant broadcasts; LAY 3: slot 3 belongs to the lanes of no plant and stays zero
    constexpr int NB = LAY == 3 ? LAY + 1 : LAY;
    __shared__ __attribute__((aligned(16))) T bx[NB][NC], bw[NB][NC];
    const int lane = threadIdx.x, h = lay_plant<LAY>(lane), r = lay_row<LAY>(lane);
    const bool noplant = LAY == 3 && lay3_noplant(lane);
    const int slot = blockIdx.x * LAY + h;
    const bool live = slot < a.n_plants;
    // (hardest-first: the slot's plant from the order list, clamped to the batch like the tile kernel's)
    const int plant = !live ? 0 : (a.order ? min(max(a.order[slot], 0), a.n_plants - 1) : slot);
    const int p = plant;  // a dead half runs plant 0's data and publishes nothing
    if (blockIdx.x == 0 && a.ord_zero)  // the order's bin counters, read by its finished sort: the next sort's
        for (int i = threadIdx.x; i < OrderBins::kBins; i += 64) a.ord_zero[i] = 0;
    MPCQ_PTIME(0);
    const int N = a.N, n = N, nx = a.nx;
    const bool lr = r < N;
    PL &S = lds[h];
    T *bxh = bx[noplant ? NB - 1 : h], *bwh = bw[noplant ? NB - 1 : h];
    const SolverSettings &st = a.st;
    // cold-path views: lane indices re-derived opaquely, so the loop does not keep the addresses of
    // the refactorisation, the checks and the finalize live in VGPRs across the hot iteration
    auto cold_lane = [&]() { return opaque(lane); };
    if (r < NC) {  // broadcast slots beyond N stay zero (row_dot reads the whole capacity)
        bxh[r] = T(0);
        bwh[r] = T(0);
    }
    if (LAY == 3 && lane < NC) {
        bx[NB - 1][lane] = T(0);
        bw[NB - 1][lane] = T(0);
    }

    // ---------------------------------------------------------------- 1. condensing
    // CAB[k] = Cd Ad^k Bd and c_k = Cd Ad^k (Sx row k-1) by the recurrences v_{k+1} = Ad v_k,
    // c_{k+1} = c_k Ad: lane t < nx of the half owns component t (scratch in the P^ slot).
    double *V = S.V(), *Cr = S.Cr();  // V[k][8], Cr[k][8] for k <= N (the union region)
    // every global read of the plant's data and inputs issued here, together (each phase reading its own
    // at its point of use waited a full memory latency, four times per wave)
    const double *Cd = a.Cd + (size_t)p * nx;
    double cdv[NXC], Kv[NXC], Xv[NXC];
    const double *K = a.K + (size_t)p * nx, *Xp = a.X + (size_t)p * nx;
#pragma unroll
    for (int c = 0; c < NXC; c++) {
        cdv[c] = c < nx ? Cd[c] : 0.0;
        Kv[c] = c < nx ? K[c] : 0.0;
        Xv[c] = c < nx ? Xp[c] : 0.0;
    }
    const double Q = a.Q[p], R = a.R[p], RD = a.RD[p], Uv = a.U[p];
    const double K0 = Kv[0];
    {
        const double *Ad = a.Ad + (size_t)p * nx * nx, *Bd = a.Bd + (size_t)p * nx;
        double adr[NXC], adc[NXC];  // row t and column t of Ad
#pragma unroll
        for (int s = 0; s < NXC; s++) {
            adr[s] = (r < nx && s < nx) ? Ad[r * nx + s] : 0.0;
            adc[s] = (r < nx && s < nx) ? Ad[s * nx + r] : 0.0;
        }
        if (r < 8) {
            V[r] = r < nx ? Bd[r] : 0.0;
            Cr[r] = r < nx ? Cd[r] : 0.0;
        }
        wave_sync();
        MPCQ_PTIME(12);
        for (int k = 0; k < N; k++) {
            // (two FMA chains per product: the step's latency is the LDS round trip plus four FMAs)
            double v0 = 0.0, v1 = 0.0, c0 = 0.0, c1 = 0.0;
#pragma unroll
            for (int s = 0; s < NXC; s += 2) {
                v0 = fma(adr[s], V[k * 8 + s], v0);
                v1 = fma(adr[s + 1], V[k * 8 + s + 1], v1);
                c0 = fma(Cr[k * 8 + s], adc[s], c0);
                c1 = fma(Cr[k * 8 + s + 1], adc[s + 1], c1);
            }
            const double v = v0 + v1, c = c0 + c1;
            wave_sync();
            if (r < 8) {
                V[(k + 1) * 8 + r] = v;
                Cr[(k + 1) * 8 + r] = c;
            }
            wave_sync();
        }
        MPCQ_PTIME(1);
        double cab = 0.0;  // Cd Ad^r Bd
        if (lr) {
#pragma unroll
            for (int s = 0; s < NXC; s++) cab += cdv[s] * (s < nx ? V[r * 8 + s] : 0.0);
        }
        const double cs = l_psum<LAY>(cab, lane);  // Su(i, j) = CS[i - j] = sum_{k <= i - j} CAB[k]
        if (r < NC) S.CS()[r] = lr ? cs : 0.0;
        wave_sync();
        MPCQ_PTIME(13);
    }
    // (this step's inputs, controllerStep's X and U, are Xv and Uv above)
    // the free response (Sx X)_k = Cd Ad^(k+1) X, lane k: with it q = Fx X + Fu U + Fr 1 xref (setF,
    // :374; Fx = 2 Su' Qbar Sx, :307) is 2 Q sum_{k >= r} CS[k - r] ((Sx X)_k - xref) + Fu U
    {
        double y = 0.0;
        if (lr) {
#pragma unroll
            for (int c = 0; c < NXC; c++)
                if (c < nx) y += Cr[(r + 1) * 8 + c] * Xv[c];
        }
        if (r < NC) S.tmp()[r] = y;
    }
    wave_sync();
    // P (setH :250-251: H1 = 2 (LL' Rbar LL + RbarD + Su' Qbar Su), symmetric as computed, so
    // (H1 + H1') / 2 = H1): H = Su'Su, H(r, j) = sum_{k >= max(r,j)} CS[k - r] CS[k - j], by the diagonal
    // recurrence H(r, j) = H(r + 1, j + 1) + CS[N-1-r] CS[N-1-j] (the k = N - 1 term; H(N, .) = 0): one row
    // per step from r = N - 1 up, lane j >= r forming H(r, j) from the row below (one LDS read, one FMA and
    // one write per lane and step), the upper triangle packed in G (the recurrences' scratch is dead by
    // now); lane r then gathers its row from LDS.  Row r stays in registers.
    // Two rows per step: row rr - 1 by the same recurrence from H(rr, j + 1), which the lane forms itself from
    // row rr + 1 with the operands lane j + 1 uses for it (the same bits as one row per step), so ten LDS round
    // trips instead of twenty.
    double *H = S.G();
    {
        const double cj = lr ? S.CS()[N - 1 - r] : 0.0;                      // CS[N-1-j], j = this lane's step
        const double cj1 = (lr && r + 1 < N) ? S.CS()[N - 2 - r] : 0.0;       // CS[N-1-(j+1)]
        for (int rr = N - 1; rr >= 0; rr -= 2) {
            const double crr = S.CS()[N - 1 - rr], crm = rr >= 1 ? S.CS()[N - rr] : 0.0;  // rows rr, rr - 1
            const bool on = lr && r >= rr, on1 = lr && rr >= 1 && r >= rr - 1;
            const double b1 = ((on || on1) && r + 1 < N && rr + 1 < N) ? H[PL::pk(rr + 1, r + 1)] : 0.0;  // H(rr+1, j+1)
            const double b2 = (on1 && r + 2 < N && rr + 1 < N) ? H[PL::pk(rr + 1, r + 2)] : 0.0;  // H(rr+1, j+2)
            if (on) H[PL::pk(rr, r)] = fma(crr, cj, b1);                  // H(rr, j)
            if (on1) {
                const double hr1 = r + 1 < N ? fma(crr, cj1, b2) : 0.0;    // H(rr, j+1), as lane j + 1 forms it
                H[PL::pk(rr - 1, r)] = fma(crm, cj, hr1);                  // H(rr-1, j)
            }
            wave_sync();
        }
    }
    MPCQ_PTIME(14);
    double pr[NC];
#pragma unroll
    for (int j = 0; j < NC; j++) {
        double v = 0.0;
        if (lr && j < N) {
            const int mx = r > j ? r : j;
            v = 2.0 * ((R * (double)(N - mx) + (r == j ? RD : 0.0)) + Q * H[PL::pk(r, j)]);
        }
        pr[j] = v;
    }
    double qk = 0.0;
    if (lr) {
        const double Fu = 2.0 * (R + Q * H[PL::pk(0, r)]);  // Fu[r] (:305, incl. the diagonal() quirk: R 1)
        double f = 0.0;
        const double xr = a.xref;
#pragma unroll
        for (int kk = 0; kk < NC; kk++)  // k = r + kk (fixed trip count: the LDS reads issue together)
            if (r + kk < N) f += S.CS()[kk] * (S.tmp()[r + kk < NC ? r + kk : NC - 1] - xr);
        qk = (2.0 * Q) * f + Fu * Uv;
    }
    double kx = 0.0;  // K X (Sbar rows < s_rows, :185,208)
#pragma unroll
    for (int c = 0; c < NXC; c++)
        if (c < nx) kx += Kv[c] * Xv[c];

    MPCQ_PTIME(2);
    // ---------------------------------------------------------------- 2. scale_data (Ruiz)
    // setup_inv_kernel's arithmetic with A structural: the top half of Gbar is K0 L (L lower-triangular
    // ones, :332-347) and the bottom half its negation, so A^ = E K0 L D entrywise, its column norms are
    // |K0| D_r max_{i >= r} E_i (suffix maxima) and its row norms |K0| E_r max_{k <= r} D_k (prefix
    // maxima); P is symmetric, so its column norm is lane r's row maximum.  The ctor's gradient is zero
    // (X = U = 0, xref = 0), so the cost scaling's |q| term is limit_scaling(0) = 1.
    const double aK0 = fabs(K0);
    double Dr = lr ? 1.0 : 0.0, Er = lr ? 1.0 : 0.0;  // (0 on dead lanes: neutral in every scan)
    double cost = 1.0, cp = 1.0;
    // the row maximum max_j |P_rj| of the current (cost-unscaled) rows: the first pass forms it, every later
    // pass takes the previous pass's cn, the maximum of the same values (max is exact in any order)
    double vp;
    {
        double vq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < NC; j++) vq[j & 3] = hwmax_abs(vq[j & 3], pr[j]);
        vp = hwmax(hwmax(vq[0], vq[1]), hwmax(vq[2], vq[3]));
    }
    for (int it = 0; it < st.scaling; it++) {
        const double emax = l_suffix_max<LAY>(Er, lane), dpre = l_prefix_max<LAY>(Dr, lane);
        const double va = (aK0 * Dr) * emax, ve = (aK0 * Er) * dpre;
        const double dt = 1.0 / sqrt(limit_scaling_p(fmax(cp * vp, va)));
        const double et = 1.0 / sqrt(limit_scaling_p(ve));
        if (r < NC) S.tmp()[r] = lr ? dt : 0.0;
        wave_sync();
        double cn = 0.0;
        // (a uniform branch on cp == 1 saved the 20 cost multiplies but its two paths' row registers met in
        // 20 moves: measured no gain, one path kept)
#pragma unroll
        for (int j = 0; j < NC; j += 2) {
            const double2 d2 = *(const double2 *)(S.tmp() + j);
            pr[j] = (dt * (pr[j] * cp)) * d2.x;
            pr[j + 1] = (dt * (pr[j + 1] * cp)) * d2.y;
            cn = hwmax(cn, hwmax_abs2(pr[j], pr[j + 1]));
        }
        wave_sync();
        vp = cn;
        if (lr) { Dr *= dt; Er *= et; }
        double cb[1] = {lr ? cn : 0.0};
        lay_reduce_k<LAY, NC, 1, 1u>(S.red(), cb, r, lane);
        const double mean = cb[0] / n;
        cp = 1.0 / limit_scaling_p(fmax(mean, 1.0));
        cost *= cp;
    }
    if (st.scaling > 0) {
#pragma unroll
        for (int j = 0; j < NC; j++) pr[j] *= cp;
    }
    const double cinv = 1.0 / cost;
    if (r < NC) {  // (the lag table under P^ is dead: the rows are in registers)
#pragma unroll
        for (int j = 0; j < NC; j++)
            if (j >= r) S.Ph()[PL::pk(r, j)] = pr[j];  // the upper triangle, row r by lane r (zero rows beyond N)
        S.Dv()[r] = Dr;
        S.Ev()[r] = Er;
        S.Ei()[r] = 1.0 / (lr ? Er : 1.0);
        S.Di()[r] = 1.0 / (lr ? Dr : 1.0);
    }
    {
        const double se = l_ssum<LAY>(Er * Er, lane);  // sum_{i >= r} E_i^2: A^'A^ = 2 K0^2 D_r D_k SE[max(r, k)]
        if (r < NC) S.SE()[r] = se;
    }

    MPCQ_PTIME(3);
    // ---------------------------------------------------------------- 3. controllerStep front end
    T qh = T(0), ut = T(kInfty), ub = T(kInfty);
    double qs = 0.0, up_t = 0.0, up_b = 0.0;
    if (lr) {
        const double sx = r < a.s_rows ? kx : 0.0;
        up_t = 255.0 + sx + (-K0) * Uv;                      // W0 + Sbar X + Ku U (:43, :99)
        up_b = 255.0 + (-sx) + K0 * Uv;
        qs = (qk * Dr) * cost;                                // q^ = c D q (osqp_update_lin_cost)
        qh = (T)qs;
        ut = (T)(up_t * Er);                                  // u^ = E u (osqp_update_upper_bound)
        ub = (T)(up_b * Er);
    }
    if (r < NC) {  // the values only the checks and the finalize read stay in LDS (read there, after
                   // the loop's wave_syncs: not hoisted into registers for the whole solve)
        S.qh()[r] = (double)qh;  // q^ as the iteration sees it
        S.Ut()[r] = up_t;
        S.Ub()[r] = up_b;
    }
    {
        // |q^| in both scalings: q does not change during the solve, so every check reads these (the check's
        // own arithmetic: DiD = 1 / D_r, the max over the plant's steps)
        const double qd = (double)qh, DiD = 1.0 / (lr ? Dr : 1.0);  // (== S.Di()[r])
        double qb[2] = {lr ? fabs(qd) : 0.0, lr ? fabs(DiD * qd) : 0.0};
        lay_reduce_k<LAY, NC, 2, 0u>(S.red(), qb, r, lane);
        const double qn_r = qb[0], qn_s = qb[1];
        if (r == 0) {
            S.sh[0] = cost;
            S.sh[1] = cinv;
            S.sh[2] = Uv;
            S.sh[3] = K0;
            S.sh[4] = qn_r;
            S.sh[5] = qn_s;
        }
    }
    // the update's checks (l^ = -DBL_MAX E stays free of -OSQP_INFTY MIN_SCALING): u < l cannot occur;
    // a row whose u^ reaches OSQP_INFTY MIN_SCALING would change type (TYPE_CHANGED)
    int status = l_any<LAY>(lr && ((double)ut > kInfty * kMinScaling || (double)ub > kInfty * kMinScaling), lane)
                     ? kTypeChanged
                     : kUnsolved;

    // ---------------------------------------------------------------- 4. ADMM
    // M(rho) = P^ + sigma I + rho A^'A^ (set_rho_vec: every row an inequality at rho) and its inverse
    // row r; in registers sigma M^-1 row r (Srow) and column r of (A^ M^-1)' (Btc: A^ M^-1 = E K0 L D M^-1,
    // so Btc[i] = E_i K0 sum_{k<=i} D_k M^-1_kr, a prefix over this lane's own row), g = -M^-1 q^.
    // An iteration: x~ = g + Srow x + Btc (w_top - w_bot) (one broadcast round: the (A^ M^-1) product
    // formed in fp64 keeps the fp32 iterate as accurate as the dense operators), z~ = A^ x~ (a prefix
    // scan).
    // fp64 (MERGED): one GEMV per iteration, x~ = g + M^-1 (sigma x + A^'(w_top - w_bot)) with A^' w a suffix
    // scan (A^ = E K0 L D): row r of M^-1 in Srow, no Btc (half the FMAs, one broadcast, 40 VGPRs fewer).
    // fp32 keeps the two products, (A^ M^-1)' formed in fp64.
    constexpr bool MERGED = std::is_same<T, double>::value;
    T Srow[NC], Btc[MERGED ? 1 : NC];
    T gk = T(0);
    const double Dd = lr ? Dr : 0.0;
    auto factor = [&](double rho) -> bool {
        const int cl = cold_lane(), r = lay_row<LAY>(cl);
        PL &S = lds[lay_plant<LAY>(cl)];
        double row[NC];
        const int q = PL::row_q(r);
        // (D_r, K0 read back from LDS here: the loop's registers for them were spilled for this cold path)
        const double K0c = S.sh[3], A2c = 2.0 * K0c * K0c, Ddc = lr ? S.Dv()[r] : 0.0;
#pragma unroll
        for (int j = 0; j < NC; j++) {
            double v = 0.0;
            if (lr && j < n) {
                const int mx = r > j ? r : j;
                v = S.Ph()[PL::pk_row(r, j, q)] + (r == j ? st.sigma : 0.0) + rho * (((A2c * Ddc) * S.Dv()[j]) * S.SE()[mx]);
            }
            row[j] = v;
        }
        const bool ok = gj_rows<NC>(row, S.piv(), n, r);
        if (!lr) {  // (a row of no step: exact zeros, not 0 - 0 * t with t from a possibly non-finite pivot row)
#pragma unroll
            for (int j = 0; j < NC; j++) row[j] = 0.0;
        }
        double g = 0.0, pre = 0.0;
#pragma unroll
        for (int j = 0; j < NC; j += 2) {
            const double2 q2 = *(const double2 *)(S.qh() + j);
            const double2 d2 = *(const double2 *)(S.Dv() + j);
            const double2 e2 = *(const double2 *)(S.Ev() + j);
            g = fma(row[j], q2.x, g);
            g = fma(row[j + 1], q2.y, g);
            if constexpr (MERGED) {
                Srow[j] = (T)row[j];
                Srow[j + 1] = (T)row[j + 1];
            } else {
                Srow[j] = (T)(st.sigma * row[j]);
                Srow[j + 1] = (T)(st.sigma * row[j + 1]);
                pre += d2.x * row[j];
                Btc[j] = (T)((e2.x * K0) * pre);
                pre += d2.y * row[j + 1];
                Btc[j + 1] = (T)((e2.y * K0) * pre);
            }
        }
        gk = lr ? (T)(-g) : T(0);
        if constexpr (!MERGED) {
            if (!lr) {  // (D, E of a non-finite plant would make 0 * NaN here)
#pragma unroll
                for (int j = 0; j < NC; j++) Btc[j] = T(0);
            }
        }
        return ok;
    };

    MPCQ_PTIME(4);
    const double rho0 = fmin(fmax(st.rho, kRhoMin), kRhoMax);
    T xs = T(0), zt = T(0), zb = T(0), yt = T(0), yb = T(0);
    T rho = (T)rho0, rinv = T(1) / rho;
    // the rho this half's M(rho)^-1 is built at: rho0 until adapt_rho moves it (an fp32 half keeps the
    // fp64 rho0, not (double)(float)rho0, so a rebuild its partner half triggers reproduces its bits)
    double rho_f = rho0;
    const T alpha = (T)st.alpha, oma = T(1) - (T)st.alpha;
    const T ET = (T)(lr ? Er : 0.0), DT = (T)Dd, K0T = (T)(noplant ? 0.0 : K0);
    // (A^ x)_r = E_r K0 sum_{k<=r} D_k x_k: E_r K0 is formed in the loop from ET, K0T (one multiply,
    // where a hoisted copy was the 3-waves/SIMD allocation's spill reloaded every iteration)
    const T sigT = (T)st.sigma;
    const bool scaled_term = st.scaled_termination != 0;
    const int ct = st.check_termination;
    const int ai = (st.adaptive_rho && a.adaptive_interval) ? a.adaptive_interval : 0;
    int next_check = ct ? ct : -1, next_adapt = ai ? ai : -1;
    int it = 0;
    bool done = false, setup_ok = true, first = true, refactor = true;
    T z3 = T(0);  // the loop's scans' DPP destination, 0 on row 3 (lay3_prefix)
    // the loop's broadcast rows, addressed from a lane index laundered here: a fresh live range after the
    // setup's register peak (formed at entry and held across the setup, the address was spilled and
    // reloaded from scratch every iteration)
    T *bxl, *bwl;
    {
        const int ln = opaque(lane);
        const int hl = (LAY == 3 && lay3_noplant(ln)) ? NB - 1 : lay_plant<LAY>(ln);
        bxl = bx[hl];
        bwl = bw[hl];
    }

    auto finalize = [&]() {
        const int cl = cold_lane(), r = lay_row<LAY>(cl);
        const PL &S = lds[lay_plant<LAY>(cl)];
        const int sl = blockIdx.x * LAY + lay_plant<LAY>(cl);
        const int plant = a.order ? min(max(a.order[sl], 0), a.n_plants - 1) : sl;  // (live: sl < n_plants)
        const bool has_sol = status == kSolved || status == kSolvedInaccurate || status == kMaxIterReached;
        if (!live) return;
        if (lr) {
            const double Er = S.Ev()[r], Dr = S.Dv()[r], cinv = S.sh[1], Uv = S.sh[2];
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
    // P^ v for this half (row r of P^ from LDS, v broadcast)
    auto p_times = [&](T v) -> double {
        const int cl = cold_lane(), r = lay_row<LAY>(cl);
        PL &S = lds[lay_plant<LAY>(cl)];
        T *bxh = bx[lay_plant<LAY>(cl)];
        if (r < NC) bxh[r] = lr ? v : T(0);
        wave_sync();
        double acc = 0.0;
        if (lr) {
            const int q = PL::row_q(r);
#pragma unroll
            for (int i = 0; i < NC; i++)
                if (i < n) acc = fma(S.Ph()[PL::pk_row(r, i, q)], (double)bxh[i], acc);
        }
        wave_sync();
        return acc;
    };

    for (;;) {
        if (refactor) {  // initSolver's factorisation, then OSQP's refactorisation after a rho change (each
                         // half at its own rho_f; a half whose rho did not move rebuilds the same bits)
            const bool ok = factor(rho_f);
            refactor = false;
            MPCQ_PSTAMP(first ? 5 : 10, first ? (long long)__builtin_amdgcn_s_memtime() : (long long)it);
            if (first) {
                first = false;
                setup_ok = ok;
                if (!ok) status = kNonCvx;
                if (!live) status = kSolved;  // (never published)
                done = status != kUnsolved;
                if (done) finalize();
            }
        }
        if (wave_all(done)) break;
        it++;
        const bool at_check = it == next_check, at_adapt = it == next_adapt;
        if (at_check) next_check += ct;
        if (at_adapt) next_adapt += ai;
        const bool last = it == st.max_iter;
        const bool info = at_check || at_adapt || last;

        // x~ = g + sigma M^-1 x + (A^ M^-1)' (w_top - w_bot),  w = rho z - y
        const T wt = tt_fma(rho, zt, -yt) - tt_fma(rho, zb, -yb);
        T xi;
        if constexpr (MERGED) {
            const T atw = (DT * K0T) * l_ssum<LAY>(ET * wt, lane, z3);  // A^'(w_top - w_bot)
            if (r < NC) bxl[r] = tt_fma(sigT, xs, atw);  // (0 on a row beyond N: x = 0, D = 0)
            wave_sync();
            xi = row_dot(Srow, bxl, gk);
            wave_sync();
        } else {
            if (r < NC) {
                bxl[r] = lr ? xs : T(0);
                bwl[r] = lr ? wt : T(0);
            }
            wave_sync();
            xi = row_dot(Srow, bxl, gk) + row_dot(Btc, bwl, T(0));
            wave_sync();
        }
        const T xn = tt_fma(alpha, xi, oma * xs);  // (0 on a row beyond N: zero M^-1 row, g = 0)
        const T dx = xn - xs;
        // (no freeze of a finished plant: its results are published, its further iterates stay in its own
        // lanes and feed nothing but its own ignored checks; a lane of no step keeps 0: zero M^-1 row,
        // E = D = 0, u^ = OSQP_INFTY)
        xs = xn;
        // z~ = A^ x~ (top rows; bottom = -top), relaxation, projection onto [l, u], dual update
        T ETl = ET;
        asm volatile("" : "+v"(ETl));
        const T zz = (ETl * K0T) * l_psum<LAY>(DT * xi, lane, z3);
        T dyt, dyb;
        {
            T v = tt_fma(alpha, zz, oma * zt);
            T zn = tt_fmin(tt_fma(rinv, yt, v), ut);
            dyt = rho * (v - zn);
            yt = tt_fma(rho, v - zn, yt);
            zt = zn;
            v = tt_fma(alpha, -zz, oma * zb);
            zn = tt_fmin(tt_fma(rinv, yb, v), ub);
            dyb = rho * (v - zn);
            yb = tt_fma(rho, v - zn, yb);
            zb = zn;
        }
        if (it == 1) MPCQ_PTIME(6);
        if (!info) continue;
        if (it == ct) MPCQ_PTIME(7);

        // ---- update_info: residuals, norms, certificates and the rho estimate in fp64 from the T
        // iterate (exact in fp64), so an fp32 kernel takes OSQP's decisions on the same numbers as an
        // fp64 one does on its own iterate (half-wave reductions)
        using TD = double;
        const int cl = cold_lane(), rc = lay_row<LAY>(cl);
        PL &C = lds[lay_plant<LAY>(cl)];
        const TD Erl = lr ? C.Ev()[rc] : 1.0, Drl = lr ? C.Dv()[rc] : 1.0, Ddl = lr ? Drl : 0.0, qsl = lr ? C.qh()[rc] : 0.0;
        const TD utl = lr ? C.Ut()[rc] : 0.0, ubl = lr ? C.Ub()[rc] : 0.0;
        const TD costl = C.sh[0], cinvl = C.sh[1], K0l = C.sh[3];
        const TD xd = (TD)xs, ztd = (TD)zt, zbd = (TD)zb, ytd = (TD)yt, ybd = (TD)yb, dxd = (TD)dx;
        const TD EKd = lr ? Erl * K0l : 0.0, DKd = Ddl * K0l, Ed = lr ? Erl : 0.0;
        const TD EiD = lr ? C.Ei()[rc] : 1.0, DiD = lr ? C.Di()[rc] : 1.0;  // (1 / E, 1 / D from the setup)
        const TD utd = lr ? utl * Erl : 0.0, ubd = lr ? ubl * Erl : 0.0;  // (== (T) bounds for fp64)
        const TD ax = EKd * l_psum<LAY>(Ddl * xd, lane);
        const TD aty = DKd * l_ssum<LAY>(Ed * (ytd - ybd), lane);
        const TD px = p_times(xs);
        // OSQP's tests read ||z|| and ||A x|| only as max(||z||, ||A x||), and ||A' y||, ||P x|| only as
        // max(||q||, ||A' y||, ||P x||): each pair is one reduction of the lanes' pair maxima (max is exact in
        // any order), four per norm set instead of six
        TD ax_z = 0, ax_zs = 0, zax_r = 0, zax_s = 0, dr_r = 0, dr_s = 0, atpx_r = 0, atpx_s = 0;
        const TD qn_r = C.sh[4], qn_s = C.sh[5];
        if (lr) {
            const TD r1 = ax - ztd, r2 = -ax - zbd;
            ax_z = hwmax_abs2(r1, r2);
            ax_zs = hwmax_abs2(EiD * r1, EiD * r2);
            zax_r = hwmax_abs(hwmax_abs2(ztd, zbd), ax);
            zax_s = hwmax_abs(hwmax_abs2(EiD * ztd, EiD * zbd), EiD * ax);
            const TD rd = (qsl + px) + aty;
            dr_r = fabs(rd);
            dr_s = fabs(DiD * rd);
            atpx_r = hwmax_abs2(aty, px);
            atpx_s = hwmax_abs2(DiD * aty, DiD * px);
        }
        // the norms in the scaling the termination test reads (scaled_termination: OSQP's scaled residuals,
        // else the unscaled ones), and the scaled ones adapt_rho reads: only the sets this iteration uses
        // (wave-uniform; with the default intervals three checks in four test termination only), four maxima
        // per batch (lay_reduce_k: from 0, skipping NaN, as OSQP's vec_norm_inf)
        double *red = C.red();
        if (scaled_term || at_adapt) {
            double b[4] = {ax_z, zax_r, dr_r, atpx_r};
            lay_reduce_k<LAY, NC, 4, 0u>(red, b, rc, lane);
            ax_z = b[0]; zax_r = b[1]; dr_r = b[2]; atpx_r = b[3];
        }
        if (!scaled_term && (at_check || last)) {
            double b[4] = {ax_zs, zax_s, dr_s, atpx_s};
            lay_reduce_k<LAY, NC, 4, 0u>(red, b, rc, lane);
            ax_zs = b[0]; zax_s = b[1]; dr_s = b[2]; atpx_s = b[3];
        }
        const TD pri_res = scaled_term ? ax_z : ax_zs;
        const TD dua_res = scaled_term ? dr_r : cinvl * dr_s;

        // OSQP's certificates (is_primal_infeasible on delta_y: l = -inf, so d = max(dy, 0) on every row;
        // is_dual_infeasible on delta_x), evaluated only where a running plant's residual test failed (need),
        // as OSQP does.  Their norms and sums do not depend on eps: one batch (||dy||, ||dx||, u'd, q'dx) and,
        // for candidates, one more (||A' d||, ||P dx||), shared by every check_termination call of the iteration.
        const TD d1 = fmax((TD)dyt, 0.0), d2 = fmax((TD)dyb, 0.0);
        TD ndy = 0, ndx = 0, lhs = 0, qdx = 0, nat = 0, npdx = 0, sv = 0;
        bool have1 = false, have_p = false, have_d = false;
        auto cert1 = [&]() {
            if (have1) return;
            have1 = true;
            double b[4] = {lr ? fmax(fabs(scaled_term ? d1 : Erl * d1), fabs(scaled_term ? d2 : Erl * d2)) : 0.0,
                           lr ? fabs(scaled_term ? dxd : Drl * dxd) : 0.0, lr ? utd * d1 + ubd * d2 : 0.0,
                           lr ? qsl * dxd : 0.0};
            lay_reduce_k<LAY, NC, 4, 0xCu>(red, b, rc, lane);
            ndy = b[0]; ndx = b[1]; lhs = b[2]; qdx = b[3];
        };
        auto cert2 = [&](bool want_p, bool want_d) {  // (uniform flags)
            double b[2] = {0.0, 0.0};
            if (want_p && !have_p) {
                const TD atd = DKd * l_ssum<LAY>(Ed * (d1 - d2), lane);
                b[0] = lr ? fabs(scaled_term ? atd : DiD * atd) : 0.0;
            }
            if (want_d && !have_d) {
                const TD t2 = p_times(dx);
                const TD t3 = EKd * l_psum<LAY>(Ddl * dxd, lane);
                b[1] = lr ? fabs(scaled_term ? t2 : DiD * t2) : 0.0;
                sv = scaled_term ? t3 : EiD * t3;
            }
            lay_reduce_k<LAY, NC, 2, 0u>(red, b, rc, lane);
            if (want_p && !have_p) nat = b[0];
            if (want_d && !have_d) npdx = b[1];
            have_p = have_p || want_p;
            have_d = have_d || want_d;
        };
        auto primal_infeasible = [&](TD eps, bool need) -> bool {
            if (!wave_any(need)) return false;
            cert1();
            const bool cand = need && ndy > kDivisionTol && lhs < eps * ndy;
            if (!wave_any(cand)) return false;
            if (!have_p) cert2(true, false);
            return cand && nat < eps * ndy;
        };
        auto dual_infeasible = [&](TD eps, bool need) -> bool {
            if (!wave_any(need)) return false;
            cert1();
            const TD cs = scaled_term ? 1.0 : costl;
            const bool cand = need && ndx > kDivisionTol && qdx < -cs * eps * ndx;
            if (!wave_any(cand)) return false;
            if (!have_d) cert2(false, true);
            const bool viol = l_any<LAY>(lr && (sv > eps * ndx || -sv > eps * ndx), lane);  // rows r (u finite), N + r (-A x)
            return cand && npdx < cs * eps * ndx && !viol;
        };
        auto check_termination = [&](bool approx) -> int {
            const TD mul = approx ? 10.0 : 1.0;
            if (pri_res > kInfty || dua_res > kInfty) return kNonCvx;
            const TD ea = st.eps_abs * mul, er = st.eps_rel * mul;
            bool prim_ok = false, dual_ok = false, prim_inf = false, dual_inf = false;
            const TD ep = ea + er * (scaled_term ? zax_r : zax_s);
            if (pri_res < ep) prim_ok = true;
            const bool pi = primal_infeasible(st.eps_prim_inf * mul, !done && !prim_ok);  // (called uniformly)
            if (!prim_ok) prim_inf = pi;
            const TD ed = ea + er * (scaled_term ? fmax(qn_r, atpx_r) : cinvl * fmax(qn_s, atpx_s));
            if (dua_res < ed) dual_ok = true;
            const bool di = dual_infeasible(st.eps_dual_inf * mul, !done && !dual_ok);
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
            const TD rhod = (TD)rho;
            const TD pr_ = ax_z / (zax_r + kDivisionTol);
            const TD dn = fmax(qn_r, atpx_r);
            const TD du = dr_r / (dn + kDivisionTol);
            TD rn = rhod * sqrt(pr_ / (du + kDivisionTol));
            rn = fmin(fmax(rn, kRhoMin), kRhoMax);
            if (!done && (rn > rhod * st.adaptive_rho_tolerance || rn < rhod / st.adaptive_rho_tolerance)) {
                rho = (T)rn;
                rinv = T(1) / rho;
                rho_f = (double)rho;
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
        if (it == ct) MPCQ_PTIME(8);
        refactor = wave_any(refactor);  // uniform (the other half rebuilds its own M at its own rho)
        if (term) {
            finalize();
            done = true;
        }
    }
    MPCQ_PTIME(9);
    MPCQ_PSTAMP(11, (long long)it);
    if (threadIdx.x == 0 && !wave_all(setup_ok || !live)) atomicOr(a.flags, 1);
}
#undef MPCQ_PTIME
#undef MPCQ_PSTAMP

template <typename T, int NC, int LAY, int NXC>
int plant_step_launch_x(const PlantStepArgs &a, hipStream_t s)
{
    const dim3 grid((a.n_plants + LAY - 1) / LAY), block(64);
    if (NC <= 20 && a.wpe == 3) hipLaunchKernelGGL((plant_step_kernel<T, NC, 3, LAY, NXC>), grid, block, 0, s, a);
    else if (NC <= 20 && a.wpe == 4) hipLaunchKernelGGL((plant_step_kernel<T, NC, 4, LAY, NXC>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((plant_step_kernel<T, NC, 2, LAY, NXC>), grid, block, 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
// nx <= 4 (the reference's cart-pole): the state loops at four components; else eight
template <typename T, int NC, int LAY>
int plant_step_launch_l(const PlantStepArgs &a, hipStream_t s)
{
    return a.nx <= 4 ? plant_step_launch_x<T, NC, LAY, 4>(a, s) : plant_step_launch_x<T, NC, LAY, 8>(a, s);
}
// N in 17 .. 20: three plants per wave unless PlantStepArgs::layout asks for two (test hook)
template <typename T, int NC>
int plant_step_launch_t(const PlantStepArgs &a, hipStream_t s)
{
    if constexpr (NC == 20) {
        if (a.layout != 2) return plant_step_launch_l<T, NC, 3>(a, s);
    }
    return plant_step_launch_l<T, NC, 2>(a, s);
}

}  // namespace mpcq

extern "C" int mpcq_internal_plant_step_launch(const mpcq::PlantStepArgs *a, int is_f32, hipStream_t s)
{
    if (a->N < 1 || a->N > 32 || a->nx < 1 || a->nx > 8) return -1;
    if (a->N <= 16) return is_f32 ? mpcq::plant_step_launch_t<float, 16>(*a, s) : mpcq::plant_step_launch_t<double, 16>(*a, s);
    if (a->N <= 20) return is_f32 ? mpcq::plant_step_launch_t<float, 20>(*a, s) : mpcq::plant_step_launch_t<double, 20>(*a, s);
    return is_f32 ? mpcq::plant_step_launch_t<float, 32>(*a, s) : mpcq::plant_step_launch_t<double, 32>(*a, s);
}
