// solvempc_amd/csrc/mpcq_order.hip — hardest-first order of a shared-plant controllerStep batch
// (BASELINE config 2: ModelPredictiveControlAPI::controllerStep, :81-108, over many states).
//
// A tile solve is a set of independent QPs whose ADMM iteration counts differ by up to 9x (config 2:
// 25 .. 225 iterations, SURVEY §8d's batch).  Run in index order, the few QPs that need the most
// iterations start wherever their index puts them and finish long after the rest of the batch: the
// solve's last ~25 % of time is a handful of lone waves.  Which QPs are slow is visible in their data:
// OSQP's ADMM converges slowly when the unconstrained optimum x_u = -P^-1 q lies close to the boundary
// of {A x <= u} (a near-degenerate active set), fast when it violates a bound by much, and at a middling
// rate when it is interior.  So every QP gets the key
//     v = max_j (A x_u - u)_j ,
// the largest violation of a bound by its unconstrained optimum, and the batch is run in ascending |v|:
// near-degenerate QPs first (they start at t = 0 and overlap the rest of the batch), then the others,
// the clearly-constrained fast ones last (they fill the chip's last slots).  A QP's arithmetic does not
// depend on its wave or position (mpcq_tile.h), so the order changes no result bit.
//
// For an MPC step q = Fx X + Fu U + Fr 1 xref and u = W0 + Sbar X + Ku U (setF :372-375, setUpperBound
// :360-369) are affine in (X, U, xref), and so is v_j: the host folds -A P^-1 [Fx Fu Fr1] - [Sbar Ku 0]
// into one m x (nx + 3) map once per operator set (mpcq_api.cpp build_order_map), and the key costs
// m (nx + 2) fp64 FMAs per QP here.
//
// A counting sort in two launches: order_key_kernel bins the keys (OrderBins::bin: 16 bins per octave of
// |v|) and takes each QP's rank inside its bin from a per-workgroup LDS histogram (256 QPs) and one
// global atomic per (workgroup, bin); order_scatter_kernel (one thread per QP) forms the prefix of the bin
// counts in every workgroup and writes list[prefix[bin] + rank] = QP.  The tile kernel's phase 0 reads its QPs
// from the list and its workgroup 0 clears the counts for the next solve (AdmmArgs::ord_list, ord_zero).
#include "mpcq_internal.h"

namespace mpcq {

// Four threads per QP (each a quarter of the m rows, fully unrolled so the map's LDS reads and the FMA chains
// of different rows overlap), 256 QPs per 1,024-thread workgroup: the key's latency is spread over 16 waves
// per workgroup, and a workgroup's global atomics (one per non-empty bin) cover 256 QPs.
constexpr int kOrderThreads = 1024, kOrderQPW = kOrderThreads / 4;
__global__ __launch_bounds__(kOrderThreads) void order_key_kernel(int batch, int nx, int m, const double *__restrict__ X,
                                                                  const double *__restrict__ U,
                                                                  const double *__restrict__ kmap, double xref,
                                                                  int *__restrict__ cnt, int *__restrict__ key,
                                                                  double *__restrict__ Xs, double *__restrict__ Us)
{
    constexpr int KB = OrderBins::kBins, KS = OrderBins::kStride, RPT = OrderBins::kMaxRows / 4;
    __shared__ double k[OrderBins::kMaxRows * KS];
    __shared__ int h[KB], base[KB];
    for (int i = threadIdx.x; i < m * KS; i += blockDim.x) k[i] = i % KS == 9 ? __builtin_fma(kmap[i + 1], xref, kmap[i]) : kmap[i];
    for (int i = threadIdx.x; i < KB; i += blockDim.x) h[i] = 0;
    const int part = threadIdx.x & 3;
    const int b = blockIdx.x * kOrderQPW + (threadIdx.x >> 2);
    const int bb = b < batch ? b : batch - 1;
    double x[8];
#pragma unroll
    for (int t = 0; t < 8; t++) x[t] = t < nx ? X[(size_t)bb * nx + t] : 0.0;
    const double u = U[bb];
    if (Xs && b < batch) {  // the step's X, U for its q, u on demand (coalesced here, not per QP in the tile kernel)
        double xa = x[0], xb = x[4];  // components part, part + 4 (selects: no register index by thread)
#pragma unroll
        for (int t = 1; t < 4; t++) {
            xa = part == t ? x[t] : xa;
            xb = part == t ? x[t + 4] : xb;
        }
        if (part < nx) Xs[(size_t)b * nx + part] = xa;
        if (part + 4 < nx) Xs[(size_t)b * nx + part + 4] = xb;
        if (part == 0) Us[b] = u;
    }
    __syncthreads();
    // rows part, part + 4, ... (interleaved: the four threads of a QP read different rows of one LDS line)
    double v = -__builtin_inf();
#pragma unroll
    for (int q = 0; q < RPT; q++) {
        const int j = 4 * q + part;
        if (j < m) {
            const double *r = k + KS * j;
            double s = r[9];  // (-A P^-1 Fr 1) xref - W0, formed above
#pragma unroll
            for (int t = 0; t < 8; t++)
                if (t < nx) s = __builtin_fma(r[t], x[t], s);
            s = __builtin_fma(r[8], u, s);
            v = __builtin_fmax(v, s);
        }
    }
    v = __builtin_fmax(v, __shfl_xor(v, 1));  // the QP's four quarters (lanes 4 i .. 4 i + 3)
    v = __builtin_fmax(v, __shfl_xor(v, 2));
    int bin = 0, loc = 0;
    if (part == 0 && b < batch) {
        bin = OrderBins::bin(v);
        loc = atomicAdd(&h[bin], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < KB; i += blockDim.x)
        if (h[i]) base[i] = atomicAdd(&cnt[i], h[i]);
    __syncthreads();
    if (part == 0 && b < batch) key[b] = (bin << OrderBins::kRankBits) | (base[bin] + loc);
}

__global__ __launch_bounds__(256) void order_scatter_kernel(int batch, const int *__restrict__ cnt,
                                                            const int *__restrict__ key, int *__restrict__ list)
{
    constexpr int KB = OrderBins::kBins, PER = KB / 256;
    static_assert(KB % 256 == 0, "bins per thread");
    __shared__ int pre[KB], wsum[4];
    // exclusive prefix of the bin counts: PER consecutive bins per thread, then a 256-thread scan
    int loc[PER], tot = 0;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        loc[i] = tot;
        tot += cnt[threadIdx.x * PER + i];
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int inc = tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(inc, d);
        if (lane >= d) inc += t;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int off = inc - tot;
    for (int i = 0; i < w; i++) off += wsum[i];
#pragma unroll
    for (int i = 0; i < PER; i++) pre[threadIdx.x * PER + i] = off + loc[i];
    __syncthreads();
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < batch) {
        const int kv = key[b];
        const int pos = pre[kv >> OrderBins::kRankBits] + (kv & ((1 << OrderBins::kRankBits) - 1));
        if (pos < batch) list[pos] = b;  // (always: the counts sum to batch)
    }
}

// (status, iter) of an ordered single-launch solve from list-slot order to the QPs' indices
// (AdmmArgs::info_slot): status[list[i]], iter[list[i]] = slot i's pair
__global__ __launch_bounds__(256) void order_info_kernel(int batch, const int *__restrict__ list,
                                                         const int2 *__restrict__ slot, int *__restrict__ status,
                                                         int *__restrict__ iter)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= batch) return;
    const int b = list[i];
    if (b < 0 || b >= batch) return;  // (never: the list is a permutation of the batch)
    const int2 v = slot[i];
    status[b] = v.x;
    iter[b] = v.y;
}

}  // namespace mpcq

extern "C" int mpcq_internal_order_info(int batch, const int *list, const int *slot, int *status, int *iter,
                                        hipStream_t s)
{
    if (batch <= 0) return 0;
    hipLaunchKernelGGL(mpcq::order_info_kernel, dim3((batch + 255) / 256), dim3(256), 0, s, batch, list,
                       (const int2 *)slot, status, iter);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// cnt: OrderBins::kBins counters, zero on entry (cleared by the previous ordered tile launch, or by the
// caller); key: batch ints of scratch; list: batch ints, the QPs hardest first; Xs, Us (or null): copies of
// X, U (the tile kernel's X_save, U_save, which the ordered launch then leaves to this kernel).
extern "C" int mpcq_internal_order(int batch, int nx, int m, const double *X, const double *U, const double *kmap,
                                   double xref, int *cnt, int *key, int *list, double *Xs, double *Us, hipStream_t s)
{
    if (batch <= 0 || batch >= (1 << mpcq::OrderBins::kRankBits) || nx <= 0 || nx > 8 || m <= 0 ||
        m > mpcq::OrderBins::kMaxRows)
        return -1;
    const int blocks = (batch + 255) / 256;
    hipLaunchKernelGGL(mpcq::order_key_kernel, dim3((batch + mpcq::kOrderQPW - 1) / mpcq::kOrderQPW),
                       dim3(mpcq::kOrderThreads), 0, s, batch, nx, m, X, U, kmap, xref, cnt, key, Xs, Us);
    if (hipGetLastError() != hipSuccess) return -2;
    hipLaunchKernelGGL(mpcq::order_scatter_kernel, dim3(blocks), dim3(256), 0, s, batch, (const int *)cnt,
                       (const int *)key, list);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
