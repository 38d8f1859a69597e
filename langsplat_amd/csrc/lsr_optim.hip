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
#include <stdlib.h>

#include <algorithm>

#include "lsr_internal.h"

namespace lsr {

constexpr int64_t kAdamDevBlocks = 512;  // device-step launches: 2 per CU

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamScalars& a)
{
    // torch lerp: weight < 0.5 ? self + weight * (end - self) : end - (end - self) * (1 - weight),
    // and addcmul self + value * t1 * t2, as torch's (contracted) kernels evaluate them
    m = a.w1 < 0.5f ? __builtin_fmaf(a.w1, g - m, m) : __builtin_fmaf(-(g - m), 1.0f - a.w1, g);
    v = __builtin_fmaf(a.w2 * g, g, v * a.beta2);
    const float denom = sqrtf(v) * a.inv_bc2_sqrt + a.eps;
    p = p + a.neg_step_size * m / denom;
}

// A table of tensors stepped by ONE launch (lsr_adam_multi): RGB mode's six parameter groups
// (scene/gaussian_model.py:219-226) -- each with its own lr, step count and moments, i.e. torch's
// per-parameter state -- in one pass, their gradients typically the slices of one all-reduced bucket
// (langsplat_amd.distributed.GradBucket).  grad_scale multiplies every gradient first (the 1 / N of
// an averaging all-reduce done as a SUM; 1: none).
__device__ __forceinline__ void adam_segment(const AdamSegment& g, int64_t chunk, float grad_scale)
{
    const int64_t first = (chunk - g.block0) * 256 + threadIdx.x;
    const bool scale = grad_scale != 1.0f;
    if (g.vec) {
        const int64_t i = first;
        if (4 * i + 3 < g.n) {
            float4 p = reinterpret_cast<float4*>(g.param)[i], m = reinterpret_cast<float4*>(g.m)[i],
                   v = reinterpret_cast<float4*>(g.v)[i];
            float4 gr = reinterpret_cast<const float4*>(g.grad)[i];
            if (scale) gr = make_float4(gr.x * grad_scale, gr.y * grad_scale, gr.z * grad_scale, gr.w * grad_scale);
            adam_one(p.x, gr.x, m.x, v.x, g.a);
            adam_one(p.y, gr.y, m.y, v.y, g.a);
            adam_one(p.z, gr.z, m.z, v.z, g.a);
            adam_one(p.w, gr.w, m.w, v.w, g.a);
            reinterpret_cast<float4*>(g.param)[i] = p;
            reinterpret_cast<float4*>(g.m)[i] = m;
            reinterpret_cast<float4*>(g.v)[i] = v;
        } else {
            for (int64_t k = 4 * i; k < g.n; k++) {
                const float gr = scale ? g.grad[k] * grad_scale : g.grad[k];
                adam_one(g.param[k], gr, g.m[k], g.v[k], g.a);
            }
        }
        return;
    }
    if (first < g.n) {
        const float gr = scale ? g.grad[first] * grad_scale : g.grad[first];
        adam_one(g.param[first], gr, g.m[first], g.v[first], g.a);
    }
}

// Device step count (tab.step_dev, for a step replayed from a HIP graph): a one-wave kernel
// advances *step_dev first and forms every tensor's bias-corrected scalars of that step once (torch's
// formulas, in double); the update's workgroups read them.  (Round 3's first form had every
// workgroup evaluate the double pow()s itself: 18.5 us against 15.4 us eager in the graph's trace.)  Measured on the graph-replayed C3 step (tools/ab_env.sh): 5 us
// faster than the alternative kept behind LSR_ADAM_ADVANCE=0, where the workgroup that finishes
// last (the last ticket) stores step + 1 and resets the ticket (same-address atomics from a small
// grid, and a long tail).
__device__ __forceinline__ AdamScalars adam_scalars_dev(const AdamHyper& h, int64_t step)
{
    const double bc1 = 1.0 - pow(h.beta1, (double)step);
    const double bc2 = 1.0 - pow(h.beta2, (double)step);
    AdamScalars a;
    a.w1 = (float)(1.0 - h.beta1);
    a.beta2 = (float)h.beta2;
    a.w2 = (float)(1.0 - h.beta2);
    a.inv_bc2_sqrt = 1.0f / (float)sqrt(bc2);
    a.eps = (float)h.eps;
    a.neg_step_size = (float)(-(h.lr / bc1));
    return a;
}

// One wave: every lane reads the step count before lane 0 stores it advanced, and lane k < count
// forms tensor k's scalars of the new step (torch's formulas, in double) into the words after the
// count -- once per step instead of once per workgroup of the update.
__global__ void k_adam_advance(int64_t* step_dev, AdamTable tab)
{
    const int64_t step = *step_dev + 1;
    const int k = (int)threadIdx.x;
    if (k < tab.count) reinterpret_cast<AdamScalars*>(step_dev + 1)[k] = adam_scalars_dev(tab.hyper[k], step);
    if (k == 0) *step_dev = step;
}

// Workgroups take 256-thread chunks grid-stride (chunk -> tensor through block0); with the ticket
// the grid is small (kAdamDevBlocks), so few tickets meet on the one counter.
__global__ __launch_bounds__(256) void k_adam_multi(AdamTable tab, int64_t chunks, float grad_scale)
{
    // device step: k_adam_advance formed the scalars (ticket null), or every workgroup forms them
    // from the count (the ticket form)
    const int64_t dstep = tab.step_dev && tab.ticket ? *tab.step_dev + 1 : 0;
    const AdamScalars* dev_scalars = tab.step_dev && !tab.ticket
        ? reinterpret_cast<const AdamScalars*>(tab.step_dev + 1) : nullptr;
    for (int64_t c = blockIdx.x; c < chunks; c += gridDim.x) {
        int s = 0;
        while (s + 1 < tab.count && c >= tab.seg[s + 1].block0) s++;
        AdamSegment g = tab.seg[s];
        if (dev_scalars) g.a = dev_scalars[s];
        else if (tab.step_dev) g.a = adam_scalars_dev(tab.hyper[s], dstep);
        adam_segment(g, c, grad_scale);
    }
    if (!tab.step_dev || !tab.ticket) return;
    __syncthreads();  // every wave of the workgroup has consumed its read of *step_dev
    if (threadIdx.x == 0) {
        // no fence: the reads were consumed (they formed the scalars above) before the ticket; the
        // stores reach the next launch at the kernel boundary
        if (__hip_atomic_fetch_add(tab.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
            *tab.step_dev = dstep;
            *tab.ticket = 0u;
        }
    }
}

hipError_t launch_adam_multi(AdamTable& tab, float grad_scale, hipStream_t s)
{
    int64_t blocks = 0;
    auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    for (int k = 0; k < tab.count; k++) {
        AdamSegment& g = tab.seg[k];
        g.vec = al(g.param) && al(g.grad) && al(g.m) && al(g.v);
        g.block0 = blocks;
        const int64_t work = g.vec ? (g.n + 3) / 4 : g.n;
        blocks += (work + 255) / 256;
    }
    if (blocks == 0) return hipSuccess;
    static const int64_t dev_blocks = [] {  // LSR_ADAM_DEV_BLOCKS: measurement knob
        const char* e = getenv("LSR_ADAM_DEV_BLOCKS");
        return e ? (int64_t)atoll(e) : kAdamDevBlocks;
    }();
    static const bool advance = [] {  // LSR_ADAM_ADVANCE=0: the ticket form (measurement knob)
        const char* e = getenv("LSR_ADAM_ADVANCE");
        return !(e && e[0] == '0');
    }();
    if (tab.step_dev && advance) {
        tab.ticket = nullptr;
        hipLaunchKernelGGL(k_adam_advance, dim3(1), dim3(64), 0, s, tab.step_dev, tab);
        const int64_t grid = std::min<int64_t>(blocks, 1 << 20);
        hipLaunchKernelGGL(k_adam_multi, dim3((unsigned)grid), dim3(256), 0, s, tab, blocks, grad_scale);
        return hipGetLastError();
    }
    const int64_t grid = tab.step_dev ? std::min<int64_t>(blocks, dev_blocks) : std::min<int64_t>(blocks, 1 << 20);
    hipLaunchKernelGGL(k_adam_multi, dim3((unsigned)grid), dim3(256), 0, s, tab, blocks, grad_scale);
    return hipGetLastError();
}

// Densification statistics of one view (train.py:125-126: max_radii2D[vis] = max(max_radii2D[vis],
// radii[vis]) and add_densification_stats, scene/gaussian_model.py:480-482: xyz_gradient_accum[vis]
// += ||viewspace.grad[vis, :2]||, denom[vis] += 1), vis = radii > 0, in one pass.
__global__ __launch_bounds__(256) void k_densification_stats(int P, const int* __restrict__ radii,
                                                             const float* __restrict__ dmeans2D,
                                                             float* __restrict__ max_radii, float* __restrict__ accum,
                                                             float* __restrict__ denom)
{
    const int i = (int)(blockIdx.x * 256 + threadIdx.x);
    if (i >= P) return;
    const int r = radii[i];
    if (!(r > 0)) return;
    const float gx = dmeans2D[3 * (size_t)i], gy = dmeans2D[3 * (size_t)i + 1];
    if (max_radii) max_radii[i] = fmaxf(max_radii[i], (float)r);
    if (accum) accum[i] = accum[i] + sqrtf(__builtin_fmaf(gy, gy, gx * gx));
    if (denom) denom[i] = denom[i] + 1.0f;
}

hipError_t launch_densification_stats(int P, const int* radii, const float* dmeans2D, float* max_radii, float* accum,
                                      float* denom, hipStream_t s)
{
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_densification_stats, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P, radii, dmeans2D,
                       max_radii, accum, denom);
    return hipGetLastError();
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
