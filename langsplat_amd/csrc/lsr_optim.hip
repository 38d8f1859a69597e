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
// workgroup evaluate the double pow()s itself: 18.5 us against 15.4 us eager in the graph's trace;
// a form where the last workgroup stored the advanced count measured 5 us slower still.)
__device__ __forceinline__ AdamScalars adam_scalars_dev(const AdamHyper& h, double lr, int64_t step)
{
    const double bc1 = 1.0 - pow(h.beta1, (double)step);
    const double bc2 = 1.0 - pow(h.beta2, (double)step);
    AdamScalars a;
    a.w1 = (float)(1.0 - h.beta1);
    a.beta2 = (float)h.beta2;
    a.w2 = (float)(1.0 - h.beta2);
    a.inv_bc2_sqrt = 1.0f / (float)sqrt(bc2);
    a.eps = (float)h.eps;
    a.neg_step_size = (float)(-(lr / bc1));
    return a;
}

// One wave: every lane reads the step count before lane 0 stores it advanced, and lane k < count
// forms tensor k's scalars of the new step (torch's formulas, in double; the lr the caller keeps in
// step_dev) into the words after the count -- once per step instead of once per workgroup of the
// update.  A skipped step (*skip != 0: the view was not rasterized) advances nothing but the skipped
// count.
__global__ void k_adam_advance(int64_t* step_dev, AdamTable tab)
{
    const int k = (int)threadIdx.x;
    if (tab.skip && *tab.skip) {
        if (k == 0) step_dev[LSR_ADAM_WORD_SKIPPED] = step_dev[LSR_ADAM_WORD_SKIPPED] + 1;
        return;
    }
    const int64_t step = *step_dev + 1;
    if (k < tab.count) {
        const double lr = __longlong_as_double((long long)step_dev[LSR_ADAM_WORD_LR + k]);
        // torch's per-parameter counts may differ by a constant (a group whose tensor was replaced,
        // scene/gaussian_model.py:326-339, skips the step of that iteration): offset per tensor
        reinterpret_cast<AdamScalars*>(step_dev + 1)[k] = adam_scalars_dev(tab.hyper[k], lr, step + tab.hyper[k].step_offset);
    }
    if (k == 0) *step_dev = step;
}

// Workgroups take 256-thread chunks grid-stride (chunk -> tensor through block0).
__global__ __launch_bounds__(256) void k_adam_multi(AdamTable tab, int64_t chunks, float grad_scale)
{
    if (tab.skip && *tab.skip) return;  // uniform: the whole launch is a no-op
    // device step: k_adam_advance formed the scalars
    const AdamScalars* dev_scalars = tab.step_dev ? reinterpret_cast<const AdamScalars*>(tab.step_dev + 1) : nullptr;
    for (int64_t c = blockIdx.x; c < chunks; c += gridDim.x) {
        int s = 0;
        while (s + 1 < tab.count && c >= tab.seg[s + 1].block0) s++;
        AdamSegment g = tab.seg[s];
        if (dev_scalars) g.a = dev_scalars[s];
        adam_segment(g, c, grad_scale);
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
    if (tab.step_dev) {  // even with no work: the count advances (or the skip is counted)
        hipLaunchKernelGGL(k_adam_advance, dim3(1), dim3(64), 0, s, tab.step_dev, tab);
        if (blocks == 0) return hipGetLastError();
    }
    if (blocks == 0) return hipSuccess;
    const int64_t grid = std::min<int64_t>(blocks, 1 << 20);
    hipLaunchKernelGGL(k_adam_multi, dim3((unsigned)grid), dim3(256), 0, s, tab, blocks, grad_scale);
    return hipGetLastError();
}

// The language step's tail in one pass (lsr_backward_args.update, N = 1): what k_grad_epilogue writes
// (dmeans2D, dlang from the packed 20-B record {dx, dy, l0, l1, l2} and the raw feature), then the Adam
// step of the raw feature from dlang (adam_one, the scalars k_adam_advance formed: the same operations
// as lsr_adam_multi after the epilogue), then -- fill set -- the activated updated feature into the
// language slots of another forward's records.  Per Gaussian every load is issued before any use
// (record, radius, feature, moments: one memory round trip).  The records' 20-B stride keeps their
// loads dword-sized; the 12-B feature / moment rows are read as three dwords by consecutive lanes.
__global__ __launch_bounds__(256) void k_language_tail(int P, const int32_t* __restrict__ radii,
                                                       const float* __restrict__ grad, float* __restrict__ lang,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       float* __restrict__ dmeans2D, float* __restrict__ dlang,
                                                       const int64_t* __restrict__ step_dev,
                                                       const int32_t* __restrict__ skip, float4* __restrict__ fill,
                                                       int deferred)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const size_t i3 = 3 * (size_t)i;
    float r0, r1, r2, r3, r4;
    if (deferred) {  // planar: P x 3 language partials (all-reduced), the flag word, P x 2 screen-space partials
        const float* rl = grad + i3;
        const float* rxy = grad + 3 * (size_t)P + kDeferXyOffset + 2 * (size_t)i;
        r0 = rxy[0];
        r1 = rxy[1];
        r2 = rl[0];
        r3 = rl[1];
        r4 = rl[2];
    } else {
        const float* r = grad + (size_t)i * kGradStrideLang;
        r0 = r[0];
        r1 = r[1];
        r2 = r[2];
        r3 = r[3];
        r4 = r[4];
    }
    const int rad = radii[i];
    float l[3] = {lang[i3], lang[i3 + 1], lang[i3 + 2]};
    float mm[3] = {m[i3], m[i3 + 1], m[i3 + 2]};
    float vv[3] = {v[i3], v[i3 + 1], v[i3 + 2]};
    const bool skipped = skip && *skip;
    const bool live = rad > 0;
    if (dmeans2D) {
        dmeans2D[i3] = live ? r0 : 0.f;
        dmeans2D[i3 + 1] = live ? r1 : 0.f;
        dmeans2D[i3 + 2] = 0.f;
    }
    float3 d = make_float3(0.f, 0.f, 0.f);
    if (live || deferred) d = act_lang_backward(l[0], l[1], l[2], r2, r3, r4);
    dlang[i3] = d.x;
    dlang[i3 + 1] = d.y;
    dlang[i3 + 2] = d.z;
    if (!skipped) {
        const AdamScalars a = *reinterpret_cast<const AdamScalars*>(step_dev + 1);  // tensor 0
        adam_one(l[0], d.x, mm[0], vv[0], a);
        adam_one(l[1], d.y, mm[1], vv[1], a);
        adam_one(l[2], d.z, mm[2], vv[2], a);
        lang[i3] = l[0];
        lang[i3 + 1] = l[1];
        lang[i3 + 2] = l[2];
        m[i3] = mm[0];
        m[i3 + 1] = mm[1];
        m[i3 + 2] = mm[2];
        v[i3] = vv[0];
        v[i3 + 1] = vv[1];
        v[i3 + 2] = vv[2];
    }
    if (fill) {  // record[3 i + 2] = {b, f0, f1, f2}: the three language slots, b untouched
        const float3 f = act_lang(l[0], l[1], l[2]);
        float* slot = reinterpret_cast<float*>(fill + 3 * (size_t)i + 2);
        slot[1] = f.x;
        *reinterpret_cast<float2*>(slot + 2) = make_float2(f.y, f.z);
    }
}

hipError_t launch_language_tail(int P, const int32_t* radii, const float* grad, float* lang, float* exp_avg,
                                float* exp_avg_sq, float* dmeans2D, float* dlang, const AdamHyper& h, int64_t* step_dev,
                                const int32_t* skip, float4* fill, int deferred, hipStream_t s)
{
    AdamTable tab{};
    tab.count = 1;
    tab.hyper[0] = h;
    tab.step_dev = step_dev;
    tab.skip = skip;
#ifndef LSR_TAIL_NO_ADVANCE  // timing-only knob: 1 leaves the step scalars as they are (wrong results)
#define LSR_TAIL_NO_ADVANCE 0
#endif
    if (!LSR_TAIL_NO_ADVANCE) hipLaunchKernelGGL(k_adam_advance, dim3(1), dim3(64), 0, s, step_dev, tab);
    if (P == 0) return hipGetLastError();
    hipLaunchKernelGGL(k_language_tail, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P, radii, grad, lang,
                       exp_avg, exp_avg_sq, dmeans2D, dlang, (const int64_t*)step_dev, skip, fill, deferred);
    return hipGetLastError();
}

// The language step's update at N > 1 (lsr_adam_fill_language): after the gradient all-reduce, the
// Adam step of the raw feature from its averaged gradient (one tensor; the scalars k_adam_advance
// formed) and -- as k_language_tail does at N = 1 -- the activated updated feature into the language
// slots of another forward's records, so that forward's composite phase needs no fill kernel
// (LSR_PHASE_COMPOSITE_FILLED).  One Gaussian per thread, its three values as three dwords of
// consecutive lanes; a skipped step leaves feature and moments alone and still fills.
__global__ __launch_bounds__(256) void k_adam_fill(int P, const float* __restrict__ grad, float grad_scale,
                                                   float* __restrict__ lang, float* __restrict__ m,
                                                   float* __restrict__ v, const int64_t* __restrict__ step_dev,
                                                   const int32_t* __restrict__ skip, float4* __restrict__ fill, int raw)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const size_t i3 = 3 * (size_t)i;
    float g[3] = {grad[i3], grad[i3 + 1], grad[i3 + 2]};
    float l[3] = {lang[i3], lang[i3 + 1], lang[i3 + 2]};
    float mm[3] = {m[i3], m[i3 + 1], m[i3 + 2]};
    float vv[3] = {v[i3], v[i3 + 1], v[i3 + 2]};
    if (!(skip && *skip)) {
        const AdamScalars a = *reinterpret_cast<const AdamScalars*>(step_dev + 1);  // tensor 0
#pragma unroll
        for (int k = 0; k < 3; k++) {
            adam_one(l[k], grad_scale != 1.0f ? g[k] * grad_scale : g[k], mm[k], vv[k], a);
            lang[i3 + k] = l[k];
            m[i3 + k] = mm[k];
            v[i3 + k] = vv[k];
        }
    }
    float3 f = make_float3(l[0], l[1], l[2]);
    if (raw & LSR_RAW_LANGUAGE) f = act_lang(l[0], l[1], l[2]);
    float* slot = reinterpret_cast<float*>(fill + 3 * (size_t)i + 2);  // {b, f0, f1, f2}, b untouched
    slot[1] = f.x;
    *reinterpret_cast<float2*>(slot + 2) = make_float2(f.y, f.z);
}

hipError_t launch_adam_fill(int P, const float* grad, float grad_scale, float* lang, float* exp_avg, float* exp_avg_sq,
                            const AdamHyper& h, int64_t* step_dev, const int32_t* skip, float4* fill, int raw,
                            hipStream_t s)
{
    AdamTable tab{};
    tab.count = 1;
    tab.hyper[0] = h;
    tab.step_dev = step_dev;
    tab.skip = skip;
    hipLaunchKernelGGL(k_adam_advance, dim3(1), dim3(64), 0, s, step_dev, tab);
    if (P == 0) return hipGetLastError();
    hipLaunchKernelGGL(k_adam_fill, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P, grad, grad_scale, lang,
                       exp_avg, exp_avg_sq, (const int64_t*)step_dev, skip, fill, raw);
    return hipGetLastError();
}

// Zero fill by a kernel instead of hipMemsetAsync: inside a stream capture the runtime turns a
// memset into a graph memset node, and instantiating a graph that held a ~220 MB one (the full
// backward's gradient records at 3.4M Gaussians) crashed the host runtime (tests/test_gpu_densify.py,
// round 4); a kernel node is what every other launch of a step is.
__global__ __launch_bounds__(256) void k_zero(uint4* __restrict__ p16, int64_t n16, uint8_t* __restrict__ tail,
                                              int ntail)
{
    const int64_t stride = (int64_t)gridDim.x * 256;
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) p16[i] = z;
    if (blockIdx.x == 0 && (int)threadIdx.x < ntail) tail[threadIdx.x] = 0;
}

hipError_t zero_fill(void* p, size_t bytes, hipStream_t s)
{
    if (bytes == 0) return hipSuccess;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const size_t head = (16 - (a & 15)) & 15;  // bytes before the first 16-B boundary
    if (head != 0) {                           // unaligned start: a byte kernel over the first head bytes
        const size_t h = head < bytes ? head : bytes;
        hipLaunchKernelGGL(k_zero, dim3(1), dim3(256), 0, s, (uint4*)nullptr, (int64_t)0, static_cast<uint8_t*>(p),
                           (int)h);
        if (h == bytes) return hipGetLastError();
    }
    uint8_t* body = static_cast<uint8_t*>(p) + head;
    const size_t rest = bytes - head;
    const int64_t n16 = (int64_t)(rest / 16);
    const int ntail = (int)(rest % 16);
    const int64_t blocks = std::min<int64_t>(std::max<int64_t>((n16 + 255) / 256, 1), 4096);
    hipLaunchKernelGGL(k_zero, dim3((unsigned)blocks), dim3(256), 0, s, reinterpret_cast<uint4*>(body), n16,
                       body + 16 * n16, ntail);
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

// ---- measurement aid: the engine clock over a ~20 us window (lsr_debug_clock_probe) ----
__global__ void k_clock_probe(uint64_t* out)
{
    const uint64_t r0 = wall_clock64(), c0 = clock64();
    uint64_t r1 = r0, c1 = c0;
    while (r1 - r0 < 2000) {  // 2000 ticks of the 100 MHz counter
        __builtin_amdgcn_s_sleep(1);
        r1 = wall_clock64();
        c1 = clock64();
    }
    if (threadIdx.x == 0) {
        out[0] = r0;
        out[1] = c0;
        out[2] = r1;
        out[3] = c1;
    }
}

hipError_t launch_clock_probe(uint64_t* out, hipStream_t s)
{
    hipLaunchKernelGGL(k_clock_probe, dim3(1), dim3(64), 0, s, out);
    return hipGetLastError();
}

// ---- a one-wave delay of `ticks` of the 100 MHz counter on a stream (lsr_debug_delay) ----
__global__ void k_delay(uint32_t ticks)
{
    const uint64_t r0 = wall_clock64();
    while (wall_clock64() - r0 < ticks) __builtin_amdgcn_s_sleep(1);
}

hipError_t launch_delay(uint32_t ticks, hipStream_t s)
{
    hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, ticks);
    return hipGetLastError();
}

}  // namespace lsr
