// solvempc_amd/csrc/mpcq_stream.hip — the simulated plant of the receding-horizon stream
// (BASELINE config 5): the reference's control loop (src/solver.cpp:43-74) reads the plant state
// from a serial port; here every QP's plant evolves on the device between control steps,
//     X <- Ad X + Bd U + w,   w ~ N(0, noise_std^2 I),
// with w from a counter-based generator (SplitMix64 of (seed, global QP index, draw), Box-Muller),
// restated in solvempc_amd/workload.py so tests can reproduce every draw on the host.
#include "mpcq_internal.h"

#include <math.h>

namespace mpcq {

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// uniform in (0, 1) for (seed, global index, draw) — workload.uniforms
__device__ __forceinline__ double uni(unsigned long long key, unsigned long long idx, unsigned long long d)
{
    const unsigned long long x = splitmix64(key ^ (idx * 0x100000001B3ull + d * 0xD6E8FEB86659FD93ull));
    return ((double)(x >> 11) + 0.5) * (1.0 / 9007199254740992.0);
}

// One thread per QP.  Plant arrays: Ad [plant][nx][nx], Bd [plant][nx] (plant 0 when shared).
__global__ void simulate_kernel(int batch, int nx, int shared, const double *Ad, const double *Bd, double *X,
                                const double *U, unsigned long long seed, long long first_qp, const long long *step_p,
                                long long step_v, double noise_std)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    const long long step = step_p ? *step_p : step_v;
    const double *A = Ad + (shared ? 0 : (size_t)b * nx * nx);
    const double *B = Bd + (shared ? 0 : (size_t)b * nx);
    double x[8], xn[8];
    for (int t = 0; t < 8; t++) x[t] = t < nx ? X[(size_t)b * nx + t] : 0.0;
    const double u = U[b];
    const unsigned long long key = splitmix64(seed * 0x632BE59BD9B4E019ull + 1ull);
    const unsigned long long idx = (unsigned long long)(first_qp + b);
    const int np = (nx + 1) / 2;  // Box-Muller pairs: w[t] = r_t cos th_t (t < np), r_{t-np} sin th_{t-np}
    for (int i = 0; i < nx; i++) {
        double s = 0.0;
        for (int t = 0; t < nx; t++) s += A[i * nx + t] * x[t];
        s += B[i] * u;
        double w = 0.0;
        if (noise_std != 0.0) {
            const int p = i < np ? i : i - np;
            const unsigned long long d0 = (unsigned long long)step * 64ull + 2ull * p;
            const double r = sqrt(-2.0 * log(uni(key, idx, d0)));
            const double th = 2.0 * M_PI * uni(key, idx, d0 + 1);
            w = noise_std * (i < np ? r * cos(th) : r * sin(th));
        }
        xn[i] = s + w;
    }
    for (int i = 0; i < nx; i++) X[(size_t)b * nx + i] = xn[i];
}

__global__ void tick_kernel(long long *step) { *step += 1; }
__global__ void set_step_kernel(long long *step, long long v) { *step = v; }

}  // namespace mpcq

extern "C" int mpcq_internal_simulate(int batch, int nx, int shared, const double *Ad, const double *Bd, double *X,
                                      const double *U, unsigned long long seed, long long first_qp,
                                      const long long *step_p, long long step_v, double noise_std, hipStream_t s)
{
    hipLaunchKernelGGL(mpcq::simulate_kernel, dim3((batch + 255) / 256), dim3(256), 0, s, batch, nx, shared, Ad, Bd,
                       X, U, seed, first_qp, step_p, step_v, noise_std);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int mpcq_internal_set_step(long long *step, long long v, hipStream_t s)
{
    hipLaunchKernelGGL(mpcq::set_step_kernel, dim3(1), dim3(1), 0, s, step, v);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int mpcq_internal_tick(long long *step, hipStream_t s)
{
    hipLaunchKernelGGL(mpcq::tick_kernel, dim3(1), dim3(1), 0, s, step);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// The QP data a controllerStep leaves in the solver (OSQP's q and u after updateGradient /
// updateUpperBound, :96-99), computed from the step's saved X and U when a caller first reads them
// (mpcq_api.cpp materialize_qu): the tile path's phase 0 saves X, U instead of writing the 480 B/QP
// fp64 q, u.  The arithmetic is the tile kernel prologue's, operation for operation (fp64, no
// contraction): q = Fx X + Fu U + (Fr 1 xref), u = W0 + Sbar X + Ku U.
namespace mpcq {
__global__ void front_end_kernel(int batch, int nx, int n, int m, const double *Xs, const double *Us, double xref,
                                 const double *Fx, const double *Fu, const double *Fr, const double *Sbar,
                                 const double *Ku, const double *W0, double *q, double *u)
{
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int rows = n + m;
    if (i >= (long long)batch * rows) return;
    const int b = (int)(i / rows), v = (int)(i % rows);
    double Xv[8];
#pragma unroll
    for (int t = 0; t < 8; t++) Xv[t] = t < nx ? Xs[(size_t)b * nx + t] : 0.0;
    const double Uv = Us[b];
    if (v < n) {
        double s2 = 0.0;  // Fr ref, ref = xref 1 (updateRef :378-380), row sum in order
        for (int t = 0; t < n; t++) s2 += Fr[(size_t)v * n + t] * xref;
        double s0 = 0.0;
#pragma unroll
        for (int t = 0; t < 8; t++)
            if (t < nx) s0 += Fx[(size_t)v * nx + t] * Xv[t];
        const double s1 = Fu[v] * Uv;
        q[(size_t)b * n + v] = s0 + s1 + s2;
    } else {
        const int r = v - n;
        double sx = 0.0;
#pragma unroll
        for (int t = 0; t < 8; t++)
            if (t < nx) sx += Sbar[(size_t)r * nx + t] * Xv[t];
        u[(size_t)b * m + r] = W0[r] + sx + Ku[r] * Uv;
    }
}
}  // namespace mpcq

extern "C" int mpcq_internal_front_end(int batch, int nx, int n, int m, const double *Xs, const double *Us, double xref,
                                       const double *Fx, const double *Fu, const double *Fr, const double *Sbar,
                                       const double *Ku, const double *W0, double *q, double *u, hipStream_t s)
{
    if (nx < 1 || nx > 8) return -1;
    const long long total = (long long)batch * (n + m);
    if (total == 0) return 0;
    hipLaunchKernelGGL(mpcq::front_end_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, batch, nx, n, m, Xs,
                       Us, xref, Fx, Fu, Fr, Sbar, Ku, W0, q, u);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
