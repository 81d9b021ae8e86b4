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
// One thread per QP.  Bins: two per octave of |v| (OrderBins::bin), a counting scatter into fixed-capacity
// per-bin lists (each bin can hold the whole batch: no global prefix, so one launch); the tile kernel's
// phase 0 reads the 64 bin counts, forms their prefix in its prologue and maps its wave slots through it.
#include "mpcq_internal.h"

namespace mpcq {

__global__ __launch_bounds__(256) void order_bin_kernel(int batch, int nx, int m, const double *__restrict__ X,
                                                        const double *__restrict__ U, const double *__restrict__ kmap,
                                                        double xref, int *__restrict__ cnt, int *__restrict__ bins,
                                                        int cap)
{
    constexpr int KB = OrderBins::kBins, KS = OrderBins::kStride;
    __shared__ double k[OrderBins::kMaxRows * KS];
    __shared__ int h[KB], base[KB];
    for (int i = threadIdx.x; i < m * KS; i += blockDim.x) k[i] = kmap[i];
    if (threadIdx.x < KB) h[threadIdx.x] = 0;
    __syncthreads();
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    int bin = 0, loc = 0;
    if (b < batch) {
        double x[8];
#pragma unroll
        for (int t = 0; t < 8; t++) x[t] = t < nx ? X[(size_t)b * nx + t] : 0.0;
        const double u = U[b];
        double v = -__builtin_inf();
        for (int j = 0; j < m; j++) {
            const double *r = k + KS * j;
            double s = __builtin_fma(r[10], xref, r[9]);  // (-A P^-1 Fr 1) xref - W0
#pragma unroll
            for (int t = 0; t < 8; t++)
                if (t < nx) s = __builtin_fma(r[t], x[t], s);
            s = __builtin_fma(r[8], u, s);
            v = __builtin_fmax(v, s);
        }
        bin = OrderBins::bin(v);
        loc = atomicAdd(&h[bin], 1);
    }
    __syncthreads();
    if (threadIdx.x < KB && h[threadIdx.x]) base[threadIdx.x] = atomicAdd(&cnt[threadIdx.x], h[threadIdx.x]);
    __syncthreads();
    if (b < batch) bins[(size_t)bin * cap + base[bin] + loc] = b;
}

}  // namespace mpcq

// cnt: OrderBins::kBins counters, zero on entry (the caller clears them on the stream first).
extern "C" int mpcq_internal_order_bins(int batch, int nx, int m, const double *X, const double *U, const double *kmap,
                                        double xref, int *cnt, int *bins, int cap, hipStream_t s)
{
    if (batch <= 0 || nx <= 0 || nx > 8 || m <= 0 || m > mpcq::OrderBins::kMaxRows || cap < batch) return -1;
    hipLaunchKernelGGL(mpcq::order_bin_kernel, dim3((batch + 255) / 256), dim3(256), 0, s, batch, nx, m, X, U, kmap,
                       xref, cnt, bins, cap);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
