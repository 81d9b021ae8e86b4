// tools/mfma_valu_bench.cpp — micro-benchmark of the gfx950 issue model that the tile kernel's hot
// loop lives in (dev tool, run on the GPU box): cycles per loop iteration (s_memtime, shader clock)
// of a wave that issues MF v_mfma_f32_16x16x4_f32 (4 independent accumulators) and NV vector ops
// (v_fma_f32, or v_pk_fma_f32 when PK), spread evenly between the MFMAs, at W waves per SIMD.
//   build: hipcc -O3 --offload-arch=gfx950 -o /tmp/mvb tools/mfma_valu_bench.cpp
//   run:   /tmp/mvb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <int MF, int NV, bool PK, int KIND = 0>
__global__ __launch_bounds__(64) void bench(long long *out, int iters, float seed)
{
    f4 acc[4] = {{seed, 0, 0, 0}, {0, seed, 0, 0}, {0, 0, seed, 0}, {0, 0, 0, seed}};
    typedef float f16v __attribute__((ext_vector_type(16)));
    f16v acc16[2] = {f16v{} + seed, f16v{} + 2 * seed};
    float v[8];
    f2 p[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        v[i] = seed * (i + 1);
        p[i] = f2{seed * i, seed + i};
    }
    const float a = seed * 0.5f, b = seed * 0.25f;
    const f2 a2 = {a, b};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int m = 0; m < (MF > 0 ? MF : 1); m++) {
            if (MF > 0 && KIND == 0) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc[m & 3]) : "v"(a), "v"(b));
            if (MF > 0 && KIND == 1) asm volatile("v_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(acc[m & 3]) : "v"(a), "v"(b));
            if (MF > 0 && KIND == 2) asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+v"(acc16[m & 1]) : "v"(a), "v"(b));
            constexpr int per = MF > 0 ? NV / MF : NV;
#pragma unroll
            for (int k = 0; k < per; k++) {
                if (PK)
                    asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[k & 7]) : "v"(a2), "v"(a2));
                else
                    asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[k & 7]) : "v"(a), "v"(b));
            }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    s += acc16[0][0] + acc16[1][5];
#pragma unroll
    for (int i = 0; i < 8; i++) s += v[i] + p[i][0] + p[i][1];
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = t1 - t0;
        out[2 * blockIdx.x + 1] = (long long)s;  // keep the arithmetic alive
    }
}

template <int MF, int NV, bool PK, int KIND = 0>
void run(int waves_per_simd)
{
    const int blocks = 1024 * waves_per_simd, iters = 2000;
    long long *d;
    hipMalloc(&d, 16 * blocks);
    hipLaunchKernelGGL((bench<MF, NV, PK, KIND>), dim3(blocks), dim3(64), 0, 0, d, 10, 1.0f);  // warm
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((bench<MF, NV, PK, KIND>), dim3(blocks), dim3(64), 0, 0, d, iters, 1.0f);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(2 * blocks);
    hipMemcpy(h.data(), d, 16 * blocks, hipMemcpyDeviceToHost);
    double sum = 0;
    for (int i = 0; i < blocks; i++) sum += h[2 * i];
    const double cyc = sum / blocks / iters;
    const double fl = KIND == 0 ? 2048.0 : (KIND == 1 ? 512.0 : 4096.0);
    const double mf_tflops = (double)blocks * iters * MF * fl / (ms * 1e-3) / 1e12;
    std::printf("{\"kind\": %d, \"mfma\": %d, \"valu\": %d, \"pk\": %d, \"waves_per_simd\": %d, \"cycles_per_iter_per_wave\": %.1f, "
                "\"simd_cycles_per_wave_iter\": %.1f, \"ms\": %.3f, \"mfma_tflops\": %.1f, \"clk_ghz\": %.3f}\n",
                KIND, MF, NV, (int)PK, waves_per_simd, cyc, cyc / waves_per_simd, ms, mf_tflops, cyc * iters / (ms * 1e-3) / 1e9);
    hipFree(d);
}

int main()
{
    for (int w : {1, 2, 4}) {
        run<32, 0, false, 0>(w);
        run<32, 0, false, 1>(w);
        run<32, 0, false, 2>(w);
        run<32, 64, false, 1>(w);
        run<32, 64, false, 2>(w);
    }
    return 0;
}
