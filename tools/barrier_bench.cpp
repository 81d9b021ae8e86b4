// Barrier + LDS broadcast round-trip latency (dev tool): one workgroup per CU, NW waves, per step one
// lane group writes a row to LDS, barrier, every lane reads it back (the Gauss-Jordan step skeleton).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int MODE>
__global__ void k(double *out, long long *cyc, int steps)
{
    __shared__ __attribute__((aligned(16))) double row[2][144];
    const int t = threadIdx.x;
    double acc = t;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < steps; s++) {
        const int p = s & 1;
        if (MODE >= 1 && (t >> 3) == (s & 31)) {
            double2 *r2 = (double2 *)&row[p][18 * (t & 7)];
#pragma unroll
            for (int j = 0; j < 8; j++) r2[j] = make_double2(acc + j, acc - j);
        }
        if (MODE == 2) {
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_s_barrier();
        } else {
            __syncthreads();
        }
        const double2 *r2 = (const double2 *)&row[p][18 * (t & 7)];
        const double2 a = r2[0], b = r2[1];
        acc += a.x * b.y;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + t] = acc;
    if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

int main()
{
    const int blocks = 256, steps = 4096;
    double *out; long long *cyc;
    hipMalloc(&out, 8 * blocks * 1024);
    hipMalloc(&cyc, 8 * blocks);
    long long h[256];
    for (int threads : {64, 128, 256, 512}) {
        for (int mode = 0; mode < 3; mode++) {
            if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, out, cyc, steps);
            if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(threads), 0, 0, out, cyc, steps);
            if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(threads), 0, 0, out, cyc, steps);
            hipDeviceSynchronize();
            hipMemcpy(h, cyc, 8 * blocks, hipMemcpyDeviceToHost);
            long long s = 0;
            for (int i = 0; i < blocks; i++) s += h[i];
            printf("threads %4d mode %d (%s): %.1f cycles/step\n", threads, mode,
                   mode == 0 ? "barrier + read" : mode == 1 ? "write + barrier + read" : "write + raw s_barrier + read",
                   (double)s / blocks / steps);
        }
    }
    return 0;
}
