// valu_peak.hip -- measures the chip's wave64 VALU issue rate (the "peak" of bench.py's VALU
// roofline): every CU runs W waves per SIMD of independent v_fma_f32 chains (8 per lane), or of
// v_exp_f32, and the rate is  instructions / 256 CUs / (kernel time x shader clock), with the clock
// measured in the same kernel (s_memtime cycles over s_memrealtime's 100 MHz ticks).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/valu_peak tools/valu_peak.hip && build/valu_peak
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int KIND>
__global__ void __launch_bounds__(256) k_valu(float* out, int iters, float a, float b, unsigned long long* clk)
{
    float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1.f, x2 = x0 + 2.f, x3 = x0 + 3.f;
    float x4 = x0 + 4.f, x5 = x0 + 5.f, x6 = x0 + 6.f, x7 = x0 + 7.f;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int i = 0; i < iters; i++) {
        if (KIND == 0) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                x0 = fmaf(x0, a, b); x1 = fmaf(x1, a, b); x2 = fmaf(x2, a, b); x3 = fmaf(x3, a, b);
                x4 = fmaf(x4, a, b); x5 = fmaf(x5, a, b); x6 = fmaf(x6, a, b); x7 = fmaf(x7, a, b);
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                x0 = __builtin_amdgcn_exp2f(x0); x1 = __builtin_amdgcn_exp2f(x1);
                x2 = __builtin_amdgcn_exp2f(x2); x3 = __builtin_amdgcn_exp2f(x3);
                x4 = __builtin_amdgcn_exp2f(x4); x5 = __builtin_amdgcn_exp2f(x5);
                x6 = __builtin_amdgcn_exp2f(x6); x7 = __builtin_amdgcn_exp2f(x7);
            }
        }
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

int main()
{
    const int cus = 256, threads = 256;
    float* out;
    unsigned long long* clk;
    hipMalloc(&out, sizeof(float) * cus * 8 * threads);
    hipMalloc(&clk, 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int kind = 0; kind < 2; kind++)
        for (int wps = 1; wps <= 8; wps *= 2) {  // waves per SIMD: 4 wps waves per CU = wps blocks per CU
            const int blocks = cus * wps, iters = kind ? 2000 : 20000;
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                if (kind == 0) k_valu<0><<<blocks, threads>>>(out, iters, 1.0000001f, 1e-7f, clk);
                else k_valu<1><<<blocks, threads>>>(out, iters, 1.0f, 0.0f, clk);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            unsigned long long c[2];
            hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
            const double ghz = c[1] ? (double)c[0] / ((double)c[1] * 10.0) : 0.0;  // memrealtime: 100 MHz
            const double insts = (double)blocks * (threads / 64) * iters * 32.0;
            const double per_cu_cycle = insts / cus / (ms * 1e-3 * ghz * 1e9);
            printf("%s waves/SIMD %d: %.3f ms, clock %.3f GHz, %.3f wave64 instr / CU / cycle\n",
                   kind ? "v_exp_f32" : "v_fma_f32", wps, ms, ghz, per_cu_cycle);
        }
    return 0;
}
