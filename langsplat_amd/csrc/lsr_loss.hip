// lsr_loss.hip -- the language-feature loss around the rasterizer.
//
// LangSplat's include_feature step computes (train.py:97-98, utils/loss_utils.py:17-18)
//     Ll1 = torch.abs(pred * m - gt * m).mean()        pred, gt: C x H x W, m: 1 x H x W
// which torch runs as 5 forward + ~6 backward elementwise/reduction kernels over the 3 x H x W
// images.  Here it is one streaming pass each way (HBM-bound: the forward reads pred + gt +
// mask, the backward reads them again and writes grad_pred):
//   k_masked_l1_forward  per-thread partial sums over 4-pixel quads (one 512-thread block per CU),
//                        block sums in double, and
//                        the last block to finish adds the block sums in a fixed order
//                        (deterministic, no second launch, no fences);
//   k_masked_l1_backward g * (1/N) * sign(pred*m - gt*m) * m, the operation order of autograd's
//                        mean -> abs -> sub -> mul backward chain, hence bit-identical to it.
// k_decode_language_feature is Camera.get_language_feature's gather (scene/cameras.py:58-92).
#include "lsr_internal.h"

namespace lsr {

constexpr int kLossThreads = 256;
constexpr int kLossMaxBlocks = 1024;
// the forward's blocks each take a ticket on ONE word (which saturates near 90 adds per us), so it
// runs on one 512-thread block per CU
constexpr int kFwdThreads = 512;
constexpr int kFwdBlocks = 256;
static_assert(kFwdBlocks <= kFwdThreads, "the last block's threads take one block sum each");

// mask value of pixel p (bool bytes or fp32)
__device__ __forceinline__ float mask_at(const void* mask, int is_float, int64_t p)
{
    return is_float ? static_cast<const float*>(mask)[p] : (static_cast<const uint8_t*>(mask)[p] ? 1.0f : 0.0f);
}

// V pixels starting at p of one channel (V = 4: aligned float4 path, V = 1: scalar)
template <int V>
__device__ __forceinline__ void load_px(const float* __restrict__ a, int64_t p, float* out)
{
    if (V == 4) {
        const float4 q = *reinterpret_cast<const float4*>(a + p);
        out[0] = q.x;
        out[1] = q.y;
        out[2] = q.z;
        out[3] = q.w;
    } else {
        out[0] = a[p];
    }
}

template <int V>
__device__ __forceinline__ void load_mask(const void* mask, int is_float, int64_t p, float* m)
{
    if (V == 4) {
        if (is_float) {
            const float4 q = *reinterpret_cast<const float4*>(static_cast<const float*>(mask) + p);
            m[0] = q.x;
            m[1] = q.y;
            m[2] = q.z;
            m[3] = q.w;
        } else {
            const uint32_t b = *reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(mask) + p);
#pragma unroll
            for (int k = 0; k < 4; k++) m[k] = ((b >> (8 * k)) & 0xFFu) ? 1.0f : 0.0f;
        }
    } else {
        m[0] = mask_at(mask, is_float, p);
    }
}

template <int kThreads>
__device__ __forceinline__ double block_sum_double(double v, double* wsum)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) wsum[wave] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < kThreads / 64; w++) t += wsum[w];
    return t;  // valid in thread 0
}

// Thread t's partial sum of block `bid` of the forward's grid (grid-stride over V-pixel groups).
// kC: the channel count at compile time (LangSplat's 3: every load of a group in flight at once),
// 0 = runtime C.  One function for the block's own pass and the last block's stall fallback, so
// a recomputed block sum is bit-identical to the one the block would have published.
template <int V, int kC>
__device__ __forceinline__ float l1_thread_partial(int bid, int nblocks, int C_rt, int64_t HW,
                                                   const float* __restrict__ pred, const float* __restrict__ gt,
                                                   const void* mask, int mask_is_float)
{
    const int C = kC > 0 ? kC : C_rt;
    const int64_t groups = HW / V;
    float acc = 0.0f;
    const int64_t stride = (int64_t)nblocks * kFwdThreads;
    int64_t gi = (int64_t)bid * kFwdThreads + threadIdx.x;
    if (kC > 0) {  // two groups per iteration: all 2 (2 kC + 1) loads in flight before the first use
        for (; gi + stride < groups; gi += 2 * stride) {
            float m[2][V], a[2][kC > 0 ? kC : 1][V], b[2][kC > 0 ? kC : 1][V];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int64_t p = (gi + u * stride) * V;
                load_mask<V>(mask, mask_is_float, p, m[u]);
#pragma unroll
                for (int c = 0; c < kC; c++) {
                    load_px<V>(pred + (int64_t)c * HW, p, a[u][c]);
                    load_px<V>(gt + (int64_t)c * HW, p, b[u][c]);
                }
            }
#pragma unroll
            for (int u = 0; u < 2; u++)
#pragma unroll
                for (int c = 0; c < kC; c++)
#pragma unroll
                    for (int k = 0; k < V; k++) acc += fabsf(a[u][c][k] * m[u][k] - b[u][c][k] * m[u][k]);
        }
    }
    for (; gi < groups; gi += stride) {
        const int64_t p = gi * V;
        float m[V];
        load_mask<V>(mask, mask_is_float, p, m);
        for (int c = 0; c < C; c++) {
            float a[V], b[V];
            load_px<V>(pred + (int64_t)c * HW, p, a);
            load_px<V>(gt + (int64_t)c * HW, p, b);
#pragma unroll
            for (int k = 0; k < V; k++) acc += fabsf(a[k] * m[k] - b[k] * m[k]);
        }
    }
    return acc;
}

// First set bit of the kFwdBlocks-bit LDS mask at index > after, or -1.
__device__ __forceinline__ int next_flagged(const uint32_t* mask, int after)
{
    for (int w = (after + 1) >> 5; w < kFwdBlocks / 32; w++) {
        uint32_t m = mask[w];
        if (w == (after + 1) >> 5) m &= ~0u << ((after + 1) & 31);
        if (m) return 32 * w + __builtin_ctz(m);
    }
    return -1;
}

// Block sums are published as ONE 64-bit word {epoch, float bits} with an sc1 store; the last
// block (ticket) waits until every word carries this launch's epoch, then adds them in block
// order.  No __threadfence (on gfx950 each one is an L2 writeback) and no scratch reset between
// launches: the host passes a fresh nonzero epoch per launch.  A word still missing after
// spin_limit polls (stall_spin_limit(), lsr_internal.h) is recomputed by the last block from the
// inputs and the event is noted in *stall.  The recomputation runs the SAME loop body as the
// block's own pass (one inlined copy: the loop below iterates over block ids), so the value is
// bit-identical to the one the block would have published.
template <int V, int kC>
__global__ __launch_bounds__(kFwdThreads) void k_masked_l1_forward(int C_rt, int64_t HW, const float* __restrict__ pred,
                                                                    const float* __restrict__ gt, const void* mask,
                                                                    int mask_is_float, float* __restrict__ loss,
                                                                    uint32_t* __restrict__ ticket,
                                                                    uint64_t* __restrict__ partial, uint32_t epoch,
                                                                    uint32_t* stall, uint32_t spin_limit)
{
    __shared__ double wsum[kFwdThreads / 64];
    __shared__ bool s_last;
    __shared__ uint32_t s_missing[kFwdBlocks / 32];
    __shared__ float s_redo[kFwdBlocks];
    const int C = kC > 0 ? kC : C_rt;
    const int nb = (int)gridDim.x;
    const int i = (int)threadIdx.x;  // in the last block: thread i takes block i's sum (nb <= kFwdThreads)
    float mine = 0.0f;
    bool any = false;
    for (int bid = (int)blockIdx.x;;) {
        const float acc = l1_thread_partial<V, kC>(bid, nb, C_rt, HW, pred, gt, mask, mask_is_float);
        const double bs = block_sum_double<kFwdThreads>((double)acc, wsum);
        if (bid == (int)blockIdx.x && !any) {  // the block's own pass
            if (threadIdx.x == 0) {
                const uint64_t word = ((uint64_t)epoch << 32) | __float_as_uint((float)bs);
                __hip_atomic_store(&partial[blockIdx.x], word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
            }
            if (threadIdx.x < kFwdBlocks / 32) s_missing[threadIdx.x] = 0u;
            __syncthreads();
            if (!s_last) return;
            if (i < nb) {
                uint64_t w = __hip_atomic_load(&partial[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                uint32_t spins = 0;
                while ((uint32_t)(w >> 32) != epoch || spin_limit == 0u) {
                    if (++spins > spin_limit) {
                        atomicOr(&s_missing[i >> 5], 1u << (i & 31));
                        break;
                    }
                    w = __hip_atomic_load(&partial[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                mine = __uint_as_float((uint32_t)w);
            }
            __syncthreads();
            bid = -1;
        } else {  // stall fallback: a missing block's sum
            if (threadIdx.x == 0) s_redo[bid] = (float)bs;
            __syncthreads();
        }
        bid = next_flagged(s_missing, bid);
        if (bid < 0) break;
        any = true;
    }
    if (any) {
        if (i < nb && ((s_missing[i >> 5] >> (i & 31)) & 1u)) mine = s_redo[i];
        if (threadIdx.x == 0) note_stall(stall);
    }
    const double total = block_sum_double<kFwdThreads>((double)mine, wsum);
    if (threadIdx.x == 0) {
        *loss = (float)(total / (double)((int64_t)C * HW));
        *ticket = 0u;  // the next launch on this scratch is stream-ordered after this one
    }
}

template <int V, int kC>
__global__ __launch_bounds__(kLossThreads) void k_masked_l1_backward(int C_rt, int64_t HW, const float* __restrict__ pred,
                                                                     const float* __restrict__ gt, const void* mask,
                                                                     int mask_is_float,
                                                                     const float* __restrict__ grad_loss,
                                                                     float* __restrict__ grad_pred)
{
    // autograd: mean backward grad.div(N) (torch's GPU div by a scalar multiplies by its
    // reciprocal), abs backward * sign, mul backward * m
    const int C = kC > 0 ? kC : C_rt;
    const float gN = grad_loss[0] * (1.0f / (float)((int64_t)C * HW));
    const int64_t groups = HW / V;
    for (int64_t gi = (int64_t)blockIdx.x * kLossThreads + threadIdx.x; gi < groups;
         gi += (int64_t)gridDim.x * kLossThreads) {
        const int64_t p = gi * V;
        float m[V];
        load_mask<V>(mask, mask_is_float, p, m);
        for (int c = 0; c < C; c++) {
            float a[V], b[V], o[V];
            load_px<V>(pred + (int64_t)c * HW, p, a);
            load_px<V>(gt + (int64_t)c * HW, p, b);
#pragma unroll
            for (int k = 0; k < V; k++) {
                const float d = a[k] * m[k] - b[k] * m[k];
                const float sg = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
                o[k] = gN * sg * m[k];
            }
            if (V == 4)
                *reinterpret_cast<float4*>(grad_pred + (int64_t)c * HW + p) = make_float4(o[0], o[1], o[2], o[3]);
            else
                grad_pred[(int64_t)c * HW + p] = o[0];
        }
    }
}

// Segment ids outside [-N, N) -- an IndexError in the reference's feature_map[seg] -- write zeros
// and set *bad (pinned host memory; the API syncs and reports it).
__global__ __launch_bounds__(256) void k_decode_language_feature(int H, int W, const int64_t* __restrict__ seg_level,
                                                                 int N, int D, const float* __restrict__ feature_map,
                                                                 float* __restrict__ out, uint8_t* __restrict__ mask,
                                                                 uint32_t* bad)
{
    const int64_t HW = (int64_t)H * W;
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= HW) return;
    int64_t s = seg_level[p];
    mask[p] = s != -1 ? 1 : 0;
    if (s < 0) s += N;  // torch indexing: -1 is the last row
    const bool ok = s >= 0 && s < N;
    if (!ok) __hip_atomic_store(bad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int d = 0; d < D; d++) out[(int64_t)d * HW + p] = ok ? feature_map[s * D + d] : 0.0f;
}

static bool vec4_ok(int64_t HW, const void* a, const void* b, const void* c, const void* mask, int mask_is_float)
{
    auto al = [](const void* q, uintptr_t m) { return (reinterpret_cast<uintptr_t>(q) & m) == 0; };
    return (HW % 4) == 0 && al(a, 15) && al(b, 15) && (!c || al(c, 15)) && al(mask, mask_is_float ? 15 : 3);
}

static int loss_blocks(int64_t groups)
{
    const int64_t b = (groups + kLossThreads - 1) / kLossThreads;
    return (int)(b < 1 ? 1 : (b > kLossMaxBlocks ? kLossMaxBlocks : b));
}

size_t masked_l1_scratch_bytes() { return 256 + 8 * (size_t)kLossMaxBlocks; }

hipError_t launch_masked_l1_forward(int C, int64_t HW, const float* pred, const float* gt, const void* mask,
                                    int mask_is_float, float* loss, void* scratch, uint32_t epoch, uint32_t* stall,
                                    hipStream_t s)
{
    const uint32_t spin = stall_spin_limit();
    uint32_t* counter = static_cast<uint32_t*>(scratch);
    uint64_t* partial = reinterpret_cast<uint64_t*>(static_cast<char*>(scratch) + 256);
    auto blocks = [](int64_t groups) {
        const int64_t b = (groups + kFwdThreads - 1) / kFwdThreads;
        return (int)(b < 1 ? 1 : (b > kFwdBlocks ? kFwdBlocks : b));
    };
    if (vec4_ok(HW, pred, gt, nullptr, mask, mask_is_float)) {
        if (C == 3)
            hipLaunchKernelGGL((k_masked_l1_forward<4, 3>), dim3(blocks(HW / 4)), dim3(kFwdThreads), 0, s, C, HW, pred,
                               gt, mask, mask_is_float, loss, counter, partial, epoch, stall, spin);
        else
            hipLaunchKernelGGL((k_masked_l1_forward<4, 0>), dim3(blocks(HW / 4)), dim3(kFwdThreads), 0, s, C, HW, pred,
                               gt, mask, mask_is_float, loss, counter, partial, epoch, stall, spin);
    } else {
        hipLaunchKernelGGL((k_masked_l1_forward<1, 0>), dim3(blocks(HW)), dim3(kFwdThreads), 0, s, C, HW, pred, gt,
                           mask, mask_is_float, loss, counter, partial, epoch, stall, spin);
    }
    return hipGetLastError();
}

hipError_t launch_masked_l1_backward(int C, int64_t HW, const float* pred, const float* gt, const void* mask,
                                     int mask_is_float, const float* grad_loss, float* grad_pred, hipStream_t s)
{
    if (vec4_ok(HW, pred, gt, grad_pred, mask, mask_is_float)) {
        if (C == 3)
            hipLaunchKernelGGL((k_masked_l1_backward<4, 3>), dim3(loss_blocks(HW / 4)), dim3(kLossThreads), 0, s, C, HW,
                               pred, gt, mask, mask_is_float, grad_loss, grad_pred);
        else
            hipLaunchKernelGGL((k_masked_l1_backward<4, 0>), dim3(loss_blocks(HW / 4)), dim3(kLossThreads), 0, s, C, HW,
                               pred, gt, mask, mask_is_float, grad_loss, grad_pred);
    } else {
        hipLaunchKernelGGL((k_masked_l1_backward<1, 0>), dim3(loss_blocks(HW)), dim3(kLossThreads), 0, s, C, HW, pred,
                           gt, mask, mask_is_float, grad_loss, grad_pred);
    }
    return hipGetLastError();
}

hipError_t launch_decode_language_feature(int H, int W, const int64_t* seg_level, int N, int D,
                                          const float* feature_map, float* out, uint8_t* mask, uint32_t* bad,
                                          hipStream_t s)
{
    const int64_t HW = (int64_t)H * W;
    hipLaunchKernelGGL(k_decode_language_feature, dim3((unsigned)((HW + 255) / 256)), dim3(256), 0, s, H, W, seg_level,
                       N, D, feature_map, out, mask, bad);
    return hipGetLastError();
}

}  // namespace lsr
