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
// One 64-lane workgroup per plant, fp64, in global scratch: setup-time code for per-plant batches.
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
}

}  // namespace mpcq

extern "C" int mpcq_internal_condense_launch(const mpcq::CondenseArgs *a, hipStream_t s)
{
    hipLaunchKernelGGL(mpcq::condense_kernel, dim3(a->n_plants), dim3(64), 0, s, *a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" size_t mpcq_internal_condense_scratch(int nx, int N) { return mpcq::condense_scratch_len(nx, N); }

