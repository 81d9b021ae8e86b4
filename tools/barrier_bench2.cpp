// Gauss-Jordan step skeleton variants (dev tool): 256 threads, one workgroup per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k(double *out, long long *cyc, int steps)
{
    __shared__ __attribute__((aligned(16))) double row[2][144], col[2][128];
    __shared__ __attribute__((aligned(16))) double2 pv[2];
    const int t = threadIdx.x, rg = t >> 3, cg = t & 7;
    double acc = t * 1e-3 + 1.0, invn = 1.0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < steps; s++) {
        const int p = s & 1, kp = s % 120;
        const bool rown = rg == (kp >> 2), coln = cg == (kp >> 4);
        if (rown) {
            double2 *r2 = (double2 *)&row[p][18 * cg];
#pragma unroll
            for (int j = 0; j < 8; j++) r2[j] = make_double2(acc + j, acc - j);
            if (MODE >= 1 && coln) pv[p] = make_double2(acc, invn);
        }
        if (MODE >= 1 && coln) {
            double2 *c2 = (double2 *)&col[p][4 * rg];
            c2[0] = make_double2(acc, acc);
            c2[1] = make_double2(acc, acc);
        }
        __syncthreads();
        const double2 *r2 = (const double2 *)&row[p][18 * cg];
        double2 a = r2[0], b = r2[1];
        if (MODE >= 1) {
            const double2 v = pv[p];
            const double2 *c2 = (const double2 *)&col[p][4 * rg];
            const double2 c0 = c2[0], c1 = c2[1];
            acc += (c0.x + c1.y) * v.y * 1e-9;
        }
        if (MODE >= 2) invn = 1.0 / (acc * a.x + 1.0);  // the lookahead division
        if (MODE >= 3 && rown) acc *= invn;
        acc += a.x * b.y * 1e-12;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + t] = acc + invn;
    if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

int main()
{
    const int blocks = 256, steps = 4096;
    double *out; long long *cyc;
    hipMalloc(&out, 8 * blocks * 1024);
    hipMalloc(&cyc, 8 * blocks);
    long long h[256];
    for (int mode = 0; mode < 4; mode++) {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, cyc, steps);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, cyc, steps);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, cyc, steps);
        if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, cyc, steps);
        hipDeviceSynchronize();
        hipMemcpy(h, cyc, 8 * blocks, hipMemcpyDeviceToHost);
        long long sum = 0;
        for (int i = 0; i < blocks; i++) sum += h[i];
        printf("mode %d: %.1f cycles/step\n", mode, (double)sum / blocks / steps);
    }
    return 0;
}
