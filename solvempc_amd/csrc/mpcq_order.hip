// solvempc_amd/csrc/mpcq_order.hip — difficulty order of a shared-plant batch for the tile path's
// first phase.  A tile wave runs until its slowest QP stops, so QPs that need similar
// iteration counts should share waves.  The predictor is the violation of the unconstrained optimum:
// key = max_j (A x_u - u)_j with x_u = -P^-1 q, i.e. max_j (H q - u)_j for H = -A P^-1 (the plant's,
// built on the host).  A QP whose unconstrained optimum violates a bound by much has few near-active
// constraints and converges early; one with key ~ 0 sits on the boundary and takes longest (on the
// config-2 batch the key's Spearman correlation with OSQP's iteration count is -0.89).
//
// One launch: each workgroup takes a window of kOrderWin consecutive QPs, bins them by the binary
// exponent of the key and lists them largest bin first in the window's slots of perm (a counting sort
// in LDS; the order inside a bin is whatever the LDS atomics give).  A window is 64 tile waves, so
// all but the few waves that straddle a bin boundary hold QPs of one bin.  Only the wave a QP runs
// in depends on the order: a QP's arithmetic, and so its result, is the same in any wave.
//
// Opt-in (test hook MPCQ_ORDER=1): on config 2 it is slower than index order.  A global
// two-launch counting sort cut phase 0 by 15 us but cost 27 us itself; this one-launch window sort
// measured 423 us per solve against 372 us.
#include "mpcq_internal.h"

namespace mpcq {

constexpr int kOrderBins = 64, kOrderWin = 1024;

// One thread per QP.  MPC step (X non-null): key rows K [m][nx + 3] = [(H Fx - Sbar) | H Fu - Ku |
// H Fr 1 | -W0] against (X, U, xref, 1); generic solve: H [m][n] against q, minus u.  The key is
// evaluated in fp32 (it only bins).
__global__ void __launch_bounds__(kOrderWin) order_kernel(int batch, int n, int m, int nx, const double *K,
                                                          const double *H, const double *X, const double *U,
                                                          double xref, const double *q, const double *u, int *perm)
{
    __shared__ float sM[64 * 32];
    __shared__ int cnt[kOrderBins], off[kOrderBins];
    const int w = X ? nx + 3 : n, rows = m;
    for (int i = threadIdx.x; i < rows * w; i += blockDim.x) sM[i] = (float)(X ? K[i] : H[i]);
    if (threadIdx.x < kOrderBins) cnt[threadIdx.x] = 0;
    __syncthreads();
    const int b = blockIdx.x * kOrderWin + threadIdx.x;
    int bin = 0;
    if (b < batch) {
        float key = -1.0f;
        if (X) {
            float z[8];
#pragma unroll
            for (int t = 0; t < 8; t++) z[t] = t < nx ? (float)X[(size_t)b * nx + t] : 0.0f;
            const float Uv = (float)U[b], xr = (float)xref;
            for (int j = 0; j < m; j++) {
                const float *k = sM + j * w;
                float v = k[nx] * Uv + k[nx + 1] * xr + k[nx + 2];
#pragma unroll
                for (int t = 0; t < 8; t++)
                    if (t < nx) v += k[t] * z[t];
                key = fmaxf(key, v);
            }
        } else {
            const double *qb = q + (size_t)b * n, *ub = u + (size_t)b * m;
            float qv[32];
#pragma unroll
            for (int t = 0; t < 32; t++) qv[t] = t < n ? (float)qb[t] : 0.0f;
            for (int j = 0; j < m; j++) {
                const float *hr = sM + j * n;
                float v = -(float)ub[j];
#pragma unroll
                for (int t = 0; t < 32; t++)
                    if (t < n) v += hr[t] * qv[t];
                key = fmaxf(key, v);
            }
        }
        // bin 0: key <= 0 (or NaN); else 1 + the exponent of key, shifted into 1..63
        if (key > 0.0f) bin = min(max(ilogbf(key) + 32, 1), kOrderBins - 1);
        atomicAdd(&cnt[bin], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0;  // window slots: bins kOrderBins-1 .. 0
        for (int k = kOrderBins - 1; k >= 0; k--) {
            off[k] = s;
            s += cnt[k];
        }
    }
    __syncthreads();
    if (b < batch) perm[blockIdx.x * kOrderWin + atomicAdd(&off[bin], 1)] = b;
}

}  // namespace mpcq

extern "C" int mpcq_internal_order(int batch, int n, int m, int nx, const double *K, const double *H,
                                   const double *X, const double *U, double xref, const double *q, const double *u,
                                   int *perm, hipStream_t s)
{
    if (batch <= 0) return 0;
    if (m > 64 || (X ? (nx < 1 || nx > 8 || !K) : (n > 32 || !H))) return -1;
    const unsigned g = (unsigned)((batch + mpcq::kOrderWin - 1) / mpcq::kOrderWin);
    hipLaunchKernelGGL(mpcq::order_kernel, dim3(g), dim3(mpcq::kOrderWin), 0, s, batch, n, m, nx, K, H, X, U, xref, q,
                       u, perm);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
