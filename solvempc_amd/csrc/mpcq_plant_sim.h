// solvempc_amd/csrc/mpcq_plant_sim.h — one row of the simulated plant of the receding-horizon stream
// (BASELINE config 5).  The reference's control loop (src/solver.cpp:43-74) reads the plant state from
// a serial port; here every QP's plant evolves on the device between control steps,
//     X <- Ad X + Bd U + w,   w ~ N(0, noise_std^2 I),
// with w from a counter-based generator (SplitMix64 of (seed, global QP index, draw), Box-Muller),
// restated in solvempc_amd/workload.py so tests can reproduce every draw on the host.  Shared by the
// per-step simulate_kernel (mpcq_stream.hip) and the persistent stream kernel (mpcq_wave.h), so both
// produce the same bits.
#pragma once
#include <hip/hip_runtime.h>
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

__device__ __forceinline__ unsigned long long sim_key(unsigned long long seed)
{
    return splitmix64(seed * 0x632BE59BD9B4E019ull + 1ull);
}

// Row i of X_next = A x + B u + w for the QP with global index idx at control step `step`
// (A row-major nx x nx, B nx; x[t] = 0 for t >= nx).
__device__ __forceinline__ double sim_row(int i, int nx, const double *A, const double *B, const double (&x)[8],
                                          double u, unsigned long long key, unsigned long long idx, long long step,
                                          double noise_std)
{
    const int np = (nx + 1) / 2;  // Box-Muller pairs: w[t] = r_t cos th_t (t < np), r_{t-np} sin th_{t-np}
    double s = 0.0;
#pragma unroll
    for (int t = 0; t < 8; t++)  // (unrolled over the capacity: x stays in registers, no dynamic index)
        if (t < nx) s += A[i * nx + t] * x[t];
    s += B[i] * u;
    double w = 0.0;
    if (noise_std != 0.0) {
        const int p = i < np ? i : i - np;
        const unsigned long long d0 = (unsigned long long)step * 64ull + 2ull * p;
        const double r = sqrt(-2.0 * log(uni(key, idx, d0)));
        const double th = 2.0 * M_PI * uni(key, idx, d0 + 1);
        w = noise_std * (i < np ? r * cos(th) : r * sin(th));
    }
    return s + w;
}

}  // namespace mpcq
