// solvempc_amd/csrc/mpcq_setup.hip — on-device QP setup (replaces osqp_setup behind
// OsqpEigen::Solver::initSolver, ModelPredictiveControlAPI.cpp:64).
//
// One 64-lane workgroup per plant, fp64 throughout:
//   1. Ruiz equilibration of [P A'; A 0] + cost scaling  (OSQP scaling.c, `settings.scaling` passes)
//   2. constraint typing from the setup bounds             (OSQP set_rho_vec)
//   3. generalised eigen-basis of M(rho) = P~ + rho G      (Cholesky of P~, cyclic Jacobi on
//      L^-1 G L^-T, W = L^-T V)  — see mpcq_internal.h
//   4. operator block for the ADMM kernel (padded to the kernel capacity).
// Setup runs once per plant; it is cold-path code written for clarity, not speed.
#include "mpcq_internal.h"

namespace mpcq {


__host__ __device__ inline size_t setup_scratch_len_dev(int n, int m)
{
    return 7 * (size_t)n * n + (size_t)m * n + 3 * (size_t)n + 2 * (size_t)m + 64;
}

__device__ inline double limit_scaling(double d)
{
    d = d < kMinScaling ? 1.0 : d;
    return d > kMaxScaling ? kMaxScaling : d;
}

__global__ __launch_bounds__(64) void setup_kernel(SetupArgs a)
{
    const int p = blockIdx.x;
    if (p >= a.n_plants) return;
    const int t = threadIdx.x, T = blockDim.x;
    const int n = a.n, m = a.m, nc = a.nc, mc = a.mc;
    const double *P = a.P + (size_t)p * n * n;
    const double *q0 = a.q0 + (size_t)p * n;
    const double *A = a.A + (size_t)p * m * n;
    const double *l0 = a.l0 + (size_t)p * m;
    const double *u0 = a.u0 + (size_t)p * m;
    const OpsLayout Lo = OpsLayout::make(nc, mc);
    double *out = a.ops + (size_t)p * Lo.total;
    int *ctype = a.ctype + (size_t)p * mc;

    double *s = a.scratch + (size_t)p * setup_scratch_len_dev(n, m);
    double *Ph = s;           s += (size_t)n * n;
    double *Ah = s;           s += (size_t)m * n;
    double *Pt = s;           s += (size_t)n * n;
    double *G = s;            s += (size_t)n * n;
    double *L = s;            s += (size_t)n * n;
    double *Tm = s;           s += (size_t)n * n;
    double *C = s;            s += (size_t)n * n;
    double *V = s;            s += (size_t)n * n;
    double *Dt = s;           s += n;
    double *Et = s;           s += m;
    double *qh = s;           s += n;
    double *Dv = s;           s += n;  // accumulated D
    double *Ev = s;           s += m;  // accumulated E
    __shared__ double sh[8];
    __shared__ int fail;

    // ---- 1. data copy (osqp-eigen passes triangularView<Upper>() of the Hessian)
    for (int e = t; e < n * n; e += T) {
        int i = e / n, j = e % n;
        Ph[e] = (i <= j) ? P[i * n + j] : P[j * n + i];
    }
    for (int e = t; e < m * n; e += T) Ah[e] = A[e];
    for (int j = t; j < n; j += T) { qh[j] = q0[j]; Dv[j] = 1.0; }
    for (int i = t; i < m; i += T) Ev[i] = 1.0;
    if (t == 0) { sh[0] = 1.0; fail = 0; }
    __syncthreads();

    // ---- Ruiz equilibration + cost normalisation (scale_data)
    for (int it = 0; it < a.scaling; it++) {
        for (int j = t; j < n; j += T) {
            double v = 0.0;
            for (int i = 0; i < n; i++) v = fmax(v, fabs(Ph[i * n + j]));
            for (int i = 0; i < m; i++) v = fmax(v, fabs(Ah[i * n + j]));
            Dt[j] = 1.0 / sqrt(limit_scaling(v));
        }
        for (int i = t; i < m; i += T) {
            double v = 0.0;
            for (int j = 0; j < n; j++) v = fmax(v, fabs(Ah[i * n + j]));
            Et[i] = 1.0 / sqrt(limit_scaling(v));
        }
        __syncthreads();
        for (int e = t; e < n * n; e += T) Ph[e] = (Dt[e / n] * Ph[e]) * Dt[e % n];
        for (int e = t; e < m * n; e += T) Ah[e] = (Et[e / n] * Ah[e]) * Dt[e % n];
        for (int j = t; j < n; j += T) { qh[j] *= Dt[j]; Dv[j] *= Dt[j]; }
        for (int i = t; i < m; i += T) Ev[i] *= Et[i];
        __syncthreads();
        for (int j = t; j < n; j += T) {
            double v = 0.0;
            for (int i = 0; i < n; i++) v = fmax(v, fabs(Ph[i * n + j]));
            Dt[j] = v;
        }
        __syncthreads();
        if (t == 0) {
            double mean = 0.0, qn = 0.0;
            for (int j = 0; j < n; j++) mean += Dt[j];
            mean /= n;
            for (int j = 0; j < n; j++) qn = fmax(qn, fabs(qh[j]));
            qn = limit_scaling(qn);
            double ct = 1.0 / limit_scaling(fmax(mean, qn));
            sh[1] = ct;
            sh[0] *= ct;
        }
        __syncthreads();
        const double ct = sh[1];
        for (int e = t; e < n * n; e += T) Ph[e] *= ct;
        for (int j = t; j < n; j += T) qh[j] *= ct;
        __syncthreads();
    }
    const double c = sh[0];

    // ---- 2. constraint types from the scaled setup bounds (set_rho_vec)
    for (int i = t; i < m; i += T) {
        double lo = l0[i] * Ev[i], up = u0[i] * Ev[i];
        int ty;
        double rs;
        if (lo < -kInfty * kMinScaling && up > kInfty * kMinScaling) { ty = -1; rs = 0.0; }
        else if (up - lo < kRhoTol) { ty = 1; rs = kRhoEqOverIneq; }
        else { ty = 0; rs = 1.0; }
        ctype[i] = ty;
        Et[i] = rs;  // reuse Et as rscale
        if (ty != 0) atomicOr(a.flags, 2);
    }
    __syncthreads();

    // ---- 3a. P~ = P^ + sigma I + RHO_MIN sum_free a a',  G = sum rscale a a'
    for (int e = t; e < n * n; e += T) {
        int i = e / n, k = e % n;
        double pt = Ph[e] + (i == k ? a.sigma : 0.0), g = 0.0;
        for (int r = 0; r < m; r++) {
            double aa = Ah[r * n + i] * Ah[r * n + k];
            if (Et[r] == 0.0) pt += kRhoMin * aa;
            else g += Et[r] * aa;
        }
        Pt[e] = pt;
        G[e] = g;
    }
    __syncthreads();

    // ---- 3b. Cholesky P~ = L L'  (column-by-column, lower triangle of L)
    for (int e = t; e < n * n; e += T) L[e] = 0.0;
    __syncthreads();
    for (int j = 0; j < n; j++) {
        if (t == 0) {
            double d = Pt[j * n + j];
            for (int k = 0; k < j; k++) d -= L[j * n + k] * L[j * n + k];
            if (!(d > 0.0)) { fail = 1; d = 1.0; }
            L[j * n + j] = sqrt(d);
        }
        __syncthreads();
        for (int i = j + 1 + t; i < n; i += T) {
            double v = Pt[i * n + j];
            for (int k = 0; k < j; k++) v -= L[i * n + k] * L[j * n + k];
            L[i * n + j] = v / L[j * n + j];
        }
        __syncthreads();
    }

    // ---- 3c. C = L^-1 G L^-T : Tm = L^-1 G (column solves), C = L^-1 Tm'
    for (int col = t; col < n; col += T) {
        for (int i = 0; i < n; i++) {
            double v = G[i * n + col];
            for (int k = 0; k < i; k++) v -= L[i * n + k] * Tm[k * n + col];
            Tm[i * n + col] = v / L[i * n + i];
        }
    }
    __syncthreads();
    for (int col = t; col < n; col += T) {  // rhs column col of Tm' = row col of Tm
        for (int i = 0; i < n; i++) {
            double v = Tm[col * n + i];
            for (int k = 0; k < i; k++) v -= L[i * n + k] * C[k * n + col];
            C[i * n + col] = v / L[i * n + i];
        }
    }
    __syncthreads();
    for (int e = t; e < n * n; e += T) {
        int i = e / n, k = e % n;
        if (i < k) {
            double v = 0.5 * (C[i * n + k] + C[k * n + i]);
            C[i * n + k] = v;
            C[k * n + i] = v;
        }
        V[e] = (i == k) ? 1.0 : 0.0;
    }
    __syncthreads();

    // ---- 3d. cyclic Jacobi: C = V diag(lambda) V'
    bool converged = false;
    for (int sweep = 0; sweep < 60; sweep++) {
        if (t == 0) {
            double off = 0.0, dia = 0.0;
            for (int i = 0; i < n; i++)
                for (int k = 0; k < n; k++) {
                    double v = C[i * n + k] * C[i * n + k];
                    if (i == k) dia += v; else off += v;
                }
            sh[2] = (off <= a.jacobi_tol * dia || off < 1e-300) ? 1.0 : 0.0;
        }
        __syncthreads();
        if (sh[2] != 0.0) { converged = true; break; }
        for (int pp = 0; pp < n - 1; pp++)
            for (int qq = pp + 1; qq < n; qq++) {
                const double apq = C[pp * n + qq];
                if (apq == 0.0) continue;  // uniform across the block
                const double app = C[pp * n + pp], aqq = C[qq * n + qq];
                const double theta = (aqq - app) / (2.0 * apq);
                const double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double cs = 1.0 / sqrt(tt * tt + 1.0), sn = tt * cs;
                __syncthreads();
                for (int k = t; k < n; k += T) {
                    if (k != pp && k != qq) {
                        double ckp = C[k * n + pp], ckq = C[k * n + qq];
                        double np_ = cs * ckp - sn * ckq, nq = sn * ckp + cs * ckq;
                        C[k * n + pp] = np_; C[pp * n + k] = np_;
                        C[k * n + qq] = nq;  C[qq * n + k] = nq;
                    }
                    double vkp = V[k * n + pp], vkq = V[k * n + qq];
                    V[k * n + pp] = cs * vkp - sn * vkq;
                    V[k * n + qq] = sn * vkp + cs * vkq;
                }
                __syncthreads();
                if (t == 0) {
                    C[pp * n + pp] = app - tt * apq;
                    C[qq * n + qq] = aqq + tt * apq;
                    C[pp * n + qq] = 0.0;
                    C[qq * n + pp] = 0.0;
                }
                __syncthreads();
            }
    }

    // ---- 3e. W = L^-T V  (back substitution per column)
    for (int col = t; col < n; col += T) {
        for (int i = n - 1; i >= 0; i--) {
            double v = V[i * n + col];
            for (int k = i + 1; k < n; k++) v -= L[k * n + i] * Tm[k * n + col];
            Tm[i * n + col] = v / L[i * n + i];  // Tm now holds W
        }
    }
    __syncthreads();

    // ---- 4. operator block (zero padded to nc x mc)
    double *o_lam = out + Lo.lam, *o_W = out + Lo.W, *o_sWtW = out + Lo.sWtW, *o_WtA = out + Lo.WtA;
    double *o_PW = out + Lo.PW, *o_Winv = out + Lo.Winv, *o_Ah = out + Lo.Ah, *o_D = out + Lo.D, *o_E = out + Lo.E;
    double *o_Dinv = out + Lo.Dinv, *o_Einv = out + Lo.Einv, *o_cs = out + Lo.cs, *o_rs = out + Lo.rscale;
    for (int k = t; k < nc; k += T) {
        o_lam[k] = k < n ? fmax(C[k * n + k], 0.0) : 0.0;
        o_D[k] = k < n ? Dv[k] : 1.0;
        o_Dinv[k] = k < n ? 1.0 / Dv[k] : 1.0;
    }
    for (int i = t; i < mc; i += T) {
        o_E[i] = i < m ? Ev[i] : 1.0;
        o_Einv[i] = i < m ? 1.0 / Ev[i] : 1.0;
        o_rs[i] = i < m ? Et[i] : 1.0;
        if (i >= m) ctype[i] = 0;
    }
    if (t == 0) { o_cs[0] = c; o_cs[1] = 1.0 / c; }
    for (int e = t; e < nc * nc; e += T) {
        int i = e / nc, k = e % nc;
        double w = 0.0, wtw = 0.0, pw = 0.0, wi = 0.0;
        if (i < n && k < n) {
            w = Tm[i * n + k];
            for (int r = 0; r < n; r++) {
                wtw += Tm[r * n + i] * Tm[r * n + k];
                pw += Ph[i * n + r] * Tm[r * n + k];
            }
            for (int r = 0; r <= k; r++) wi += V[r * n + i] * L[k * n + r];  // (V' L')_{ik}
            wtw *= a.sigma;
        }
        o_W[e] = w;
        o_sWtW[e] = wtw;
        o_PW[e] = pw;
        o_Winv[e] = wi;
    }
    for (int e = t; e < mc * nc; e += T) {
        int j = e / nc, k = e % nc;
        double b = 0.0, ah = 0.0;
        if (j < m && k < n) {
            ah = Ah[j * n + k];
            for (int r = 0; r < n; r++) b += Ah[j * n + r] * Tm[r * n + k];
        }
        o_WtA[e] = b;
        o_Ah[e] = ah;
        out[Lo.Bt + e] = b;  // eigen-basis: Bt = A^ W
    }
    for (int e = t; e < nc * nc; e += T) out[Lo.G + e] = o_W[e];  // G = W (written above by this thread)
    if (t == 0) out[Lo.rho0] = -1.0;
    __syncthreads();
    if (t == 0) {
        a.status[p] = fail ? kNonCvx : 0;
        if (fail) atomicOr(a.flags, 1);
        if (!converged) atomicOr(a.flags, 4);  // sweep cap hit: (lambda, W) would be inaccurate
    }
}

__global__ void f64_to_f32_kernel(const double *in, float *out, size_t count)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x)
        out[i] = (float)in[i];
}

// Replicate one plant's m- or n-vector over the QPs of that plant (QP-major destination).
__global__ void broadcast_kernel(const double *src, double *dst, int len, int batch, int per_qp_src)
{
    const size_t total = (size_t)batch * len;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t b = i / len, j = i % len;
        dst[i] = src[(per_qp_src ? b * len : 0) + j];
    }
}

template <typename T>
__global__ void fill_kernel(T *p, T v, size_t count)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x)
        p[i] = v;
}

}  // namespace mpcq

extern "C" int mpcq_internal_fill(void *p, int is_f32, double v, size_t count, hipStream_t s)
{
    if (!count) return 0;
    if (is_f32)
        hipLaunchKernelGGL(mpcq::fill_kernel<float>, dim3(256), dim3(256), 0, s, (float *)p, (float)v, count);
    else
        hipLaunchKernelGGL(mpcq::fill_kernel<double>, dim3(256), dim3(256), 0, s, (double *)p, v, count);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int mpcq_internal_f64_to_f32(const double *in, float *out, size_t count, hipStream_t s)
{
    hipLaunchKernelGGL(mpcq::f64_to_f32_kernel, dim3(1024), dim3(256), 0, s, in, out, count);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int mpcq_internal_broadcast(const double *src, double *dst, int len, int batch, int per_qp_src,
                                       hipStream_t s)
{
    if ((size_t)batch * len == 0) return 0;
    hipLaunchKernelGGL(mpcq::broadcast_kernel, dim3(1024), dim3(256), 0, s, src, dst, len, batch, per_qp_src);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int mpcq_internal_setup_launch(const mpcq::SetupArgs *args, hipStream_t stream)
{
    hipLaunchKernelGGL(mpcq::setup_kernel, dim3(args->n_plants), dim3(64), 0, stream, *args);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
