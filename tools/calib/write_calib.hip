// WRITE_SIZE calibration (dev tool, gfx950): store patterns of the tile kernel's finalize, each its own kernel
// so rocprofv3 --pmc WRITE_SIZE reports them separately.  One wave per 16 "QPs"; rows at random (permuted)
// indices, as the hardest-first order leaves them.  Bytes written per pattern are printed for comparison.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>

constexpr int B = 65536;
// P1: one lane per QP stores 8 B at row b (rhos / U / rho_out)
__global__ void p1_scalar8(double *out, const int *perm)
{
    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int b = perm[16 * w + c];
    if (g == 0) out[b] = 1.0 + b;
}
// P2: 4 lanes per QP store 8 B each at 4s + g of a 256-B row, s = 0..4 (xs: 160 B of the row)
__global__ void p2_rows32(double *out, const int *perm)
{
    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int b = perm[16 * w + c];
#pragma unroll
    for (int s = 0; s < 5; s++) out[(size_t)b * 32 + 4 * s + g] = 1.0 + s;
}
// P3: the same 160 B per QP, each lane two consecutive doubles (16 B) of the row: 10 lanes' worth per QP
__global__ void p3_rows16B(double *out, const int *perm)
{
    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int b = perm[16 * w + c];
    for (int s = 0; s < 3; s++) {
        const int e = 8 * s + 2 * g;  // 0..23, pairs
        if (e < 20) *(double2 *)(out + (size_t)b * 32 + e) = make_double2(1.0, 2.0);
    }
}
// P4: contiguous 512 B per instruction (index order)
__global__ void p4_contig(double *out)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (int s = 0; s < 5; s++) out[i + (size_t)s * B * 16 / 5] = 1.0;
}
// P5: one lane per QP stores 4 B (status / iter)
__global__ void p5_scalar4(int *out, const int *perm)
{
    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int b = perm[16 * w + c];
    if (g == 0) out[b] = b;
}
// P6: one lane per QP stores 16 B (a packed {rho, status, iter} record)
__global__ void p6_rec16(double2 *out, const int *perm)
{
    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int b = perm[16 * w + c];
    if (g == 0) out[b] = make_double2(1.0, 2.0);
}

int main()
{
    std::vector<int> h(B);
    for (int i = 0; i < B; i++) h[i] = i;
    std::shuffle(h.begin(), h.end(), std::mt19937(1));
    int *perm;
    double *buf;
    hipMalloc(&perm, 4 * B);
    hipMalloc(&buf, (size_t)B * 32 * 8);
    hipMemcpy(perm, h.data(), 4 * B, hipMemcpyHostToDevice);
    const dim3 grid(B / 64), blk(256);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(p1_scalar8, grid, blk, 0, 0, buf, perm);
        hipLaunchKernelGGL(p2_rows32, grid, blk, 0, 0, buf, perm);
        hipLaunchKernelGGL(p3_rows16B, grid, blk, 0, 0, buf, perm);
        hipLaunchKernelGGL(p4_contig, dim3(B * 16 / 5 / 256 + 1), blk, 0, 0, buf);
        hipLaunchKernelGGL(p5_scalar4, grid, blk, 0, 0, (int *)buf, perm);
        hipLaunchKernelGGL(p6_rec16, grid, blk, 0, 0, (double2 *)buf, perm);
    }
    hipDeviceSynchronize();
    printf("bytes: p1 %d p2 %d p3 %d p4 %d p5 %d p6 %d\n", B * 8, B * 160, B * 160, B * 16 * 8, B * 4, B * 16);
    return 0;
}
