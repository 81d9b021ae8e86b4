// solvempc_amd/csrc/mpcq_condense.hip — condensed-QP construction on the device.
//
// Replaces the Eigen code of ModelPredictiveControlAPI (src/ModelPredictiveControlAPI.cpp):
//   setTransformations :180-208   Sx[i] = Cd Ad^(i+1), CAB[i] = Cd Ad^i Bd, Su(i,j) = sum CAB[0..i-j],
//                                 S rows < s_rows = K (the reference hard-codes 10, :185), Sbar = [S; -S]
//   setLL :292, setLiftedCosts :160-162 (Qbar = Q I, Rbar = R I, RbarD = RD I)
//   setH :250-251                 P = sym(2 (LL' Rbar LL + RbarD + Su' Qbar Su))
//   setFVars :305-307             Fu = 2 (diag(LL' Rbar')' + Su1' Qbar Su)', Fr = -2 (Qbar Su)',
//                                 Fx = 2 (Sx' Qbar Su)'
//   setLinearConstraints :332-335 A = [K0 L; -K0 L]
//   setUpperBound :364-368        Ku = [-K0 1; K0 1], W0 = 255 1
// Unwritten Eigen blocks (S rows >= 10, upper triangle of Su) are explicit zeros.
// condense_kernel: one 64-lane workgroup per plant, fp64, global scratch (any N);
// condense_wave_kernel: one wavefront per plant, LDS-resident (N <= 32), same arithmetic.
#include "mpcq_internal.h"

namespace mpcq {

__host__ __device__ inline size_t condense_scratch_len(int nx, int N)
{
    return (size_t)N * nx + (size_t)N + 2 * (size_t)N * N + 64;
}

// Eigen MatrixPower::computeIntPower: res = I; loop { if odd: res = tmp*res; halve; tmp *= tmp }.
__device__ void mat_pow(int nx, const double *A, int p, double *out, double *tmp, double *t2)
{
    for (int i = 0; i < nx * nx; i++) { tmp[i] = A[i]; out[i] = (i / nx == i % nx) ? 1.0 : 0.0; }
    unsigned pp = (unsigned)p;
    while (pp) {
        if (pp & 1u) {
            for (int r = 0; r < nx; r++)
                for (int c = 0; c < nx; c++) {
                    double s = 0.0;
                    for (int t = 0; t < nx; t++) s += tmp[r * nx + t] * out[t * nx + c];
                    t2[r * nx + c] = s;
                }
            for (int i = 0; i < nx * nx; i++) out[i] = t2[i];
        }
        pp >>= 1;
        if (!pp) break;
        for (int r = 0; r < nx; r++)
            for (int c = 0; c < nx; c++) {
                double s = 0.0;
                for (int t = 0; t < nx; t++) s += tmp[r * nx + t] * tmp[t * nx + c];
                t2[r * nx + c] = s;
            }
        for (int i = 0; i < nx * nx; i++) tmp[i] = t2[i];
    }
}

__global__ __launch_bounds__(64) void condense_kernel(CondenseArgs a)
{
    const int p = blockIdx.x;
    if (p >= a.n_plants) return;
    const int t = threadIdx.x, T = blockDim.x, nx = a.nx, N = a.N;
    const double *Ad = a.Ad + (size_t)p * nx * nx, *Bd = a.Bd + (size_t)p * nx;
    const double *Cd = a.Cd + (size_t)p * nx, *K = a.K + (size_t)p * nx;
    const double Q = a.Q[p], R = a.R[p], RD = a.RD[p];
    double *P = a.P + (size_t)p * N * N, *A = a.A + (size_t)p * 2 * N * N;
    double *Fx = a.Fx + (size_t)p * N * nx, *Fu = a.Fu + (size_t)p * N, *Fr = a.Fr + (size_t)p * N * N;
    double *Sbar = a.Sbar + (size_t)p * 2 * N * nx, *Ku = a.Ku + (size_t)p * 2 * N, *W0 = a.W0 + (size_t)p * 2 * N;
    double *s = a.scratch + (size_t)p * condense_scratch_len(nx, N);
    double *Sx = s;  s += (size_t)N * nx;
    double *CAB = s; s += N;
    double *Su = s;  s += (size_t)N * N;
    double *H1 = s;  s += (size_t)N * N;

    // setTransformations :187-194 (thread i: powers i and i+1)
    for (int i = t; i < N; i += T) {
        double pw[64], tmp[64], t2[64];  // nx <= 8
        mat_pow(nx, Ad, i + 1, pw, tmp, t2);
        for (int c = 0; c < nx; c++) {
            double v = 0.0;
            for (int r = 0; r < nx; r++) v += Cd[r] * pw[r * nx + c];
            Sx[i * nx + c] = v;
        }
        mat_pow(nx, Ad, i, pw, tmp, t2);
        double row[8];
        for (int c = 0; c < nx; c++) {
            double v = 0.0;
            for (int r = 0; r < nx; r++) v += Cd[r] * pw[r * nx + c];
            row[c] = v;
        }
        double v = 0.0;
        for (int r = 0; r < nx; r++) v += row[r] * Bd[r];
        CAB[i] = v;
    }
    __syncthreads();
    // :197-204 Su(i,j) = sum(CAB[0..i-j]) for j <= i, else 0
    for (int e = t; e < N * N; e += T) {
        const int i = e / N, j = e % N;
        double v = 0.0;
        if (j <= i)
            for (int k = 0; k <= i - j; k++) v += CAB[k];
        Su[e] = v;
    }
    __syncthreads();
    // setH :250 — H1 = 2 (LL' Rbar LL + RbarD + Su' Qbar Su)
    for (int e = t; e < N * N; e += T) {
        const int i = e / N, j = e % N;
        double t2 = 0.0, t4 = 0.0;
        for (int k = 0; k < N; k++) {
            // (LL' Rbar)(i,k) = LL(k,i) R ; times LL(k,j)
            const double llr = (k >= i) ? R : 0.0;
            t2 += llr * ((k >= j) ? 1.0 : 0.0);
            t4 += (Su[k * N + i] * Q) * Su[k * N + j];
        }
        H1[e] = 2.0 * (t2 + (i == j ? RD : 0.0) + t4);
    }
    __syncthreads();
    for (int e = t; e < N * N; e += T) {
        const int i = e / N, j = e % N;
        P[e] = (H1[i * N + j] + H1[j * N + i]) / 2.0;
        Fr[e] = -2.0 * (Q * Su[j * N + i]);  // -2 (Qbar Su)'
    }
    // setFVars :305,307
    for (int j = t; j < N; j += T) {
        double s1 = 0.0;
        for (int k = 0; k < N; k++) s1 += (Su[k * N + 0] * Q) * Su[k * N + j];
        Fu[j] = 2.0 * (R + s1);  // (LL' Rbar').diagonal() = R * LL(j,j) = R
        for (int c = 0; c < nx; c++) {
            double v = 0.0;
            for (int k = 0; k < N; k++) v += (Sx[k * nx + c] * Q) * Su[k * N + j];
            Fx[j * nx + c] = 2.0 * v;
        }
    }
    // setLinearConstraints :332-335, setTransformations :185,208, setUpperBound :364-368
    const double K0 = K[0];
    for (int e = t; e < N * N; e += T) {
        const int i = e / N, j = e % N;
        const double v = (j <= i) ? 1.0 : 0.0;
        A[i * N + j] = v * K0;
        A[(N + i) * N + j] = v * -K0;
    }
    for (int i = t; i < N; i += T) {
        const bool k_row = i < a.s_rows;
        for (int c = 0; c < nx; c++) {
            Sbar[i * nx + c] = k_row ? K[c] : 0.0;
            Sbar[(N + i) * nx + c] = k_row ? -K[c] : 0.0;
        }
        Ku[i] = -K0;
        Ku[N + i] = K0;
        W0[i] = 255.0;
        W0[N + i] = 255.0;
    }
    for (int i = t; i < 2 * N; i += T) {
        if (a.u0) a.u0[(size_t)p * 2 * N + i] = 255.0;
        if (a.l0) a.l0[(size_t)p * 2 * N + i] = -1.7976931348623157e308;
    }
    if (a.q0)
        for (int i = t; i < N; i += T) a.q0[(size_t)p * N + i] = 0.0;
}

// One wavefront per plant, LDS-resident (N <= 32): the same arithmetic, in the same order, as
// condense_kernel (bit-identical outputs), without the global scratch round trips.  Lane i computes
// the powers Ad^(i+1), Ad^i by the same binary powering with register arrays (NX is a template
// parameter so they stay in VGPRs); Su(i,j) = cum[i-j] with cum the running sum of CAB (the
// sequential sum of condense_kernel); the N^3 products spread over the 64 lanes.
template <int NX>
__device__ void mat_pow_reg(const double (&A)[NX * NX], int p, double (&out)[NX * NX])
{
    double tmp[NX * NX], t2[NX * NX];
#pragma unroll
    for (int i = 0; i < NX * NX; i++) { tmp[i] = A[i]; out[i] = (i / NX == i % NX) ? 1.0 : 0.0; }
    unsigned pp = (unsigned)p;
    while (pp) {
        if (pp & 1u) {
#pragma unroll
            for (int r = 0; r < NX; r++)
#pragma unroll
                for (int c = 0; c < NX; c++) {
                    double s = 0.0;
#pragma unroll
                    for (int t = 0; t < NX; t++) s += tmp[r * NX + t] * out[t * NX + c];
                    t2[r * NX + c] = s;
                }
#pragma unroll
            for (int i = 0; i < NX * NX; i++) out[i] = t2[i];
        }
        pp >>= 1;
        if (!pp) break;
#pragma unroll
        for (int r = 0; r < NX; r++)
#pragma unroll
            for (int c = 0; c < NX; c++) {
                double s = 0.0;
#pragma unroll
                for (int t = 0; t < NX; t++) s += tmp[r * NX + t] * tmp[t * NX + c];
                t2[r * NX + c] = s;
            }
#pragma unroll
        for (int i = 0; i < NX * NX; i++) tmp[i] = t2[i];
    }
}

template <int NX>
__global__ __launch_bounds__(64) void condense_wave_kernel(CondenseArgs a)
{
    constexpr int NMAX = 32, LD = NMAX + 1;
    __shared__ double Sx[NMAX * NX], CAB[NMAX], cum[NMAX], Su[NMAX * LD], H1[NMAX * LD];
    const int p = blockIdx.x;
    if (p >= a.n_plants) return;
    const int t = threadIdx.x, N = a.N;
    const double *Adp = a.Ad + (size_t)p * NX * NX, *Bd = a.Bd + (size_t)p * NX;
    const double *Cd = a.Cd + (size_t)p * NX, *K = a.K + (size_t)p * NX;
    const double Q = a.Q[p], R = a.R[p], RD = a.RD[p];
    double *P = a.P + (size_t)p * N * N, *A = a.A + (size_t)p * 2 * N * N;
    double *Fx = a.Fx + (size_t)p * N * NX, *Fu = a.Fu + (size_t)p * N, *Fr = a.Fr + (size_t)p * N * N;
    double *Sbar = a.Sbar + (size_t)p * 2 * N * NX, *Ku = a.Ku + (size_t)p * 2 * N, *W0 = a.W0 + (size_t)p * 2 * N;

    // setTransformations :187-194
    if (t < N) {
        double Ad[NX * NX], pw[NX * NX];
#pragma unroll
        for (int i = 0; i < NX * NX; i++) Ad[i] = Adp[i];
        mat_pow_reg<NX>(Ad, t + 1, pw);
#pragma unroll
        for (int c = 0; c < NX; c++) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < NX; r++) v += Cd[r] * pw[r * NX + c];
            Sx[t * NX + c] = v;
        }
        mat_pow_reg<NX>(Ad, t, pw);
        double row[NX];
#pragma unroll
        for (int c = 0; c < NX; c++) {
            double v = 0.0;
#pragma unroll
            for (int r = 0; r < NX; r++) v += Cd[r] * pw[r * NX + c];
            row[c] = v;
        }
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < NX; r++) v += row[r] * Bd[r];
        CAB[t] = v;
    }
    __syncthreads();
    if (t == 0) {
        double v = 0.0;
        for (int k = 0; k < N; k++) { v += CAB[k]; cum[k] = v; }
    }
    __syncthreads();
    // :197-204 Su(i,j) = sum(CAB[0..i-j]) for j <= i, else 0
    for (int e = t; e < N * N; e += 64) {
        const int i = e / N, j = e % N;
        Su[i * LD + j] = (j <= i) ? cum[i - j] : 0.0;
    }
    __syncthreads();
    // setH :250 — H1 = 2 (LL' Rbar LL + RbarD + Su' Qbar Su)
    for (int e = t; e < N * N; e += 64) {
        const int i = e / N, j = e % N;
        double t2 = 0.0, t4 = 0.0;
        for (int k = 0; k < N; k++) {
            const double llr = (k >= i) ? R : 0.0;
            t2 += llr * ((k >= j) ? 1.0 : 0.0);
            t4 += (Su[k * LD + i] * Q) * Su[k * LD + j];
        }
        H1[i * LD + j] = 2.0 * (t2 + (i == j ? RD : 0.0) + t4);
    }
    __syncthreads();
    for (int e = t; e < N * N; e += 64) {
        const int i = e / N, j = e % N;
        P[e] = (H1[i * LD + j] + H1[j * LD + i]) / 2.0;
        Fr[e] = -2.0 * (Q * Su[j * LD + i]);
    }
    // setFVars :305,307
    if (t < N) {
        const int j = t;
        double s1 = 0.0;
        for (int k = 0; k < N; k++) s1 += (Su[k * LD + 0] * Q) * Su[k * LD + j];
        Fu[j] = 2.0 * (R + s1);
    }
    for (int e = t; e < N * NX; e += 64) {
        const int j = e / NX, c = e % NX;
        double v = 0.0;
        for (int k = 0; k < N; k++) v += (Sx[k * NX + c] * Q) * Su[k * LD + j];
        Fx[j * NX + c] = 2.0 * v;
    }
    // setLinearConstraints :332-335, setTransformations :185,208, setUpperBound :364-368
    const double K0 = K[0];
    for (int e = t; e < N * N; e += 64) {
        const int i = e / N, j = e % N;
        const double v = (j <= i) ? 1.0 : 0.0;
        A[i * N + j] = v * K0;
        A[(N + i) * N + j] = v * -K0;
    }
    for (int e = t; e < 2 * N * NX; e += 64) {
        const int i = e / NX, c = e % NX;
        const bool k_row = (i < N ? i : i - N) < a.s_rows;
        Sbar[e] = k_row ? (i < N ? K[c] : -K[c]) : 0.0;
    }
    for (int i = t; i < 2 * N; i += 64) {
        Ku[i] = i < N ? -K0 : K0;
        W0[i] = 255.0;
        // the ctor's setup data (X = U = ref = 0, :22-23,38-43): q0 = 0, l0 = -DBL_MAX, u0 = W0
        if (a.u0) a.u0[(size_t)p * 2 * N + i] = 255.0;
        if (a.l0) a.l0[(size_t)p * 2 * N + i] = -1.7976931348623157e308;
    }
    if (a.q0)
        for (int i = t; i < N; i += 64) a.q0[(size_t)p * N + i] = 0.0;
}

}  // namespace mpcq

extern "C" int mpcq_internal_condense_launch(const mpcq::CondenseArgs *a, hipStream_t s)
{
    const dim3 g(a->n_plants), b(64);
    if (a->N <= 32 && !a->force_ref) {
        switch (a->nx) {
#define MPCQ_CW(X) case X: hipLaunchKernelGGL(mpcq::condense_wave_kernel<X>, g, b, 0, s, *a); break;
            MPCQ_CW(1) MPCQ_CW(2) MPCQ_CW(3) MPCQ_CW(4) MPCQ_CW(5) MPCQ_CW(6) MPCQ_CW(7) MPCQ_CW(8)
#undef MPCQ_CW
        default: return -1;
        }
    } else {
        if (!a->scratch) return -1;
        hipLaunchKernelGGL(mpcq::condense_kernel, g, b, 0, s, *a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" size_t mpcq_internal_condense_scratch(int nx, int N) { return mpcq::condense_scratch_len(nx, N); }

