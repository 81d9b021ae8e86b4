// solvempc_amd/csrc/mpcq_stream.hip — the simulated plant of the receding-horizon stream
// (BASELINE config 5), one launch per control step (the hipGraph path of mpcq_mpc_run_device and
// mpcq_mpc_simulate_device); the row arithmetic and the noise are mpcq_plant_sim.h's.
#include "mpcq_internal.h"
#include "mpcq_plant_sim.h"

namespace mpcq {

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
    const unsigned long long key = sim_key(seed);
    const unsigned long long idx = (unsigned long long)(first_qp + b);
    for (int i = 0; i < nx; i++) xn[i] = sim_row(i, nx, A, B, x, u, key, idx, step, noise_std);
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
