// lsr_optim.hip -- Adam step for the trainable Gaussian parameters.
//
// LangSplat optimises with torch.optim.Adam(lr=0.0, eps=1e-15) over per-attribute parameter
// groups (scene/gaussian_model.py:203-229) and steps once per iteration (train.py:134-137).
// One launch per parameter tensor: a single HBM pass that reads param, grad, exp_avg,
// exp_avg_sq (16 B/element) and writes param, exp_avg, exp_avg_sq (12 B/element), in the
// operation order of torch's single-tensor Adam:
//     exp_avg    = lerp(exp_avg, grad, 1 - beta1)                    (fma, as torch's kernel)
//     exp_avg_sq = fma((1 - beta2) * grad, grad, exp_avg_sq * beta2)
//     denom      = sqrt(exp_avg_sq) * (1 / sqrt(bias_correction2)) + eps
//     param      = param + (-lr / bias_correction1) * exp_avg / denom
// The step-dependent scalars are computed on the host in double, as torch does.
#include "lsr_internal.h"

namespace lsr {

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamScalars& a)
{
    // torch lerp: weight < 0.5 ? self + weight * (end - self) : end - (end - self) * (1 - weight),
    // and addcmul self + value * t1 * t2, as torch's (contracted) kernels evaluate them
    m = a.w1 < 0.5f ? __builtin_fmaf(a.w1, g - m, m) : __builtin_fmaf(-(g - m), 1.0f - a.w1, g);
    v = __builtin_fmaf(a.w2 * g, g, v * a.beta2);
    const float denom = sqrtf(v) * a.inv_bc2_sqrt + a.eps;
    p = p + a.neg_step_size * m / denom;
}

__global__ __launch_bounds__(256) void k_adam(int64_t n, float* __restrict__ param, const float* __restrict__ grad,
                                              float* __restrict__ exp_avg, float* __restrict__ exp_avg_sq,
                                              AdamScalars a, int vec)
{
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if (vec) {
        const int64_t n4 = n >> 2;
        float4* p4 = reinterpret_cast<float4*>(param);
        const float4* g4 = reinterpret_cast<const float4*>(grad);
        float4* m4 = reinterpret_cast<float4*>(exp_avg);
        float4* v4 = reinterpret_cast<float4*>(exp_avg_sq);
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
            float4 p = p4[i], m = m4[i], v = v4[i];
            const float4 g = g4[i];
            adam_one(p.x, g.x, m.x, v.x, a);
            adam_one(p.y, g.y, m.y, v.y, a);
            adam_one(p.z, g.z, m.z, v.z, a);
            adam_one(p.w, g.w, m.w, v.w, a);
            p4[i] = p;
            m4[i] = m;
            v4[i] = v;
        }
        for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
            adam_one(param[i], grad[i], exp_avg[i], exp_avg_sq[i], a);
        return;
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        adam_one(param[i], grad[i], exp_avg[i], exp_avg_sq[i], a);
}

hipError_t launch_adam(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                       const AdamScalars& a, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    const int vec = al(param) && al(grad) && al(exp_avg) && al(exp_avg_sq);
    const int64_t work = vec ? (n + 3) / 4 : n;
    int64_t blocks = (work + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, s, n, param, grad, exp_avg, exp_avg_sq, a, vec);
    return hipGetLastError();
}

}  // namespace lsr
