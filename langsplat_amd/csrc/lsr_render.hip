// lsr_render.hip -- per-tile compositing (forward) and its back-to-front replay (backward).
//
// One 256-thread workgroup per 16x16 screen tile; wave w of its 4 owns the 8x8 pixel block
// (8 (w & 1), 8 (w >> 1)) and every lane one pixel.  Workgroups take tiles longest first
// (scheduled_tile).  The tile's depth-ordered list is streamed through LDS in batches of 256
// entries (one per thread: {x, y, -conic.x/2, -conic.z/2}{conic.y, opacity, power cutoff, f1}
// {r, g, b, f0}{f2}); the loading thread also computes a 4-bit mask of the wave blocks the entry
// can reach (entry_cover: reach box, refined by the exact ellipse-vs-block test), and a wave skips
// the entries that cannot reach its block:
//   forward:  each wave compacts the batch into a slot list (wave_compact) and walks it two
//             entries per step (their exps as one packed chain);
//   backward: each wave walks the set bits of a ballot over the masks (no list).
// Semantics: upstream FORWARD/BACKWARD::renderCUDA extended by the 3-channel language feature
// (SURVEY.md §8a a10-a11, App. A.4-A.5); arithmetic order is that of oracle/lsr_oracle.c
// render_pixel / backward_pixel (the forward bit-identically, the backward's gradient arithmetic
// regrouped).
//
// Backward gradient scatter: every lane of a wave visits the same list entry at the same
// iteration, so the per-Gaussian partials of a wave are reduced in registers by a reduce-scatter
// (permlane32/16 swaps + DPP mirrors: 27 operations for 12 values, 16 for the language step's 5),
// the 4 waves' results are summed in LDS (ds_add_f32), and after each batch ONE atomic row per
// (tile, Gaussian) adds the tile's total into a per-Gaussian record -- instead of the upstream 12
// scattered atomics per pixel per blend.  Entries no lane contributes to are skipped by a ballot.
// The backward is specialised (template) on the language feature, on a zero colour gradient and on
// whether the geometry gradients are needed (k_render_backward<kStats, kFeat, kColor, kGeo>).
#include <stdlib.h>

#include "lsr_internal.h"

namespace lsr {

// Exact early-out: for power < cutoff(o) = ln(1/(255 o)) - 0.01 the composited alpha
// min(0.99, o * exp(power)) is certainly < 1/255 (1% margin >> the exp restatement's 2 ulp), so
// the entry is skipped exactly as the full test would skip it -- without evaluating exp.
// o < 1/255 (or o <= 0) skips always, as alpha <= o then.
__device__ __forceinline__ float power_cutoff(float o)
{
    return o > (1.0f / 255.0f) ? __logf(1.0f / (255.0f * o)) - 0.01f : 3.0e38f;
}

// Screen box of the pixels an entry can reach: power >= cut is the ellipse d^T Q d <= -2 cut
// (Q = conic), whose half-extents are sqrt(-2 cut (Q^-1)_xx) and sqrt(-2 cut (Q^-1)_yy); widened by
// a conservative margin (0.1% + 0.05 px >> fp32 error of the power evaluation).  Returns
// (xmin, xmax, ymin, ymax); empty for entries that always skip, unbounded if Q is degenerate.
// Waves cull a batch against their own pixel rectangle with it: an entry whose box misses the
// rectangle fails the cutoff test in every lane, so skipping it is exact.
__device__ __forceinline__ float4 entry_box(float x, float y, float cx, float cy, float cz, float cut)
{
    const float k = -2.0f * cut;
    if (!(k > 0.0f)) return make_float4(3.0e38f, -3.0e38f, 3.0e38f, -3.0e38f);
    const float detq = cx * cz - cy * cy;
    if (!(detq > 0.0f)) return make_float4(-3.0e38f, 3.0e38f, -3.0e38f, 3.0e38f);
    // hardware reciprocal and square root (a few ulp): far inside the 0.1 % margin, and the
    // correctly rounded division / sqrt sequences cost ~35 VALU per entry in the load phases
    const float kd = k * __builtin_amdgcn_rcpf(detq);
    const float ex = __builtin_amdgcn_sqrtf(kd * cz) * 1.001f + 0.05f;
    const float ey = __builtin_amdgcn_sqrtf(kd * cx) * 1.001f + 0.05f;
    return make_float4(x - ex, x + ex, y - ey, y + ey);
}

// 4-bit mask of the tile's wave blocks an entry's reach box E meets: wave w owns the pixels
// [x0 + 8 (w & 1), +7] x [y0 + 8 (w >> 1), +7].  An entry whose box misses a block fails the
// cutoff test in every pixel of it, so skipping it there is exact.
__device__ __forceinline__ uint32_t wave_cover(const float4& E, float x0, float y0)
{
    const bool xa = E.y >= x0 && E.x <= x0 + 7.0f;
    const bool xb = E.y >= x0 + 8.0f && E.x <= x0 + 15.0f;
    const bool ya = E.w >= y0 && E.z <= y0 + 7.0f;
    const bool yb = E.w >= y0 + 8.0f && E.z <= y0 + 15.0f;
    return (xa && ya ? 1u : 0u) | (xb && ya ? 2u : 0u) | (xa && yb ? 4u : 0u) | (xb && yb ? 8u : 0u);
}

// Does the cutoff ellipse Q(p - mu) <= k (Q = [[a, b], [b, c]], the conic; k = -2 cutoff) meet the
// rectangle of pixel centres [x0, x0 + 7] x [y0, y0 + 7]?  Exact minimum of the convex quadratic over
// the rectangle: 0 if the centre is inside, else the smallest of its four edge minima (each the 1D
// minimiser clamped to the edge).  A "no" is only returned with a margin (0.1 % of k + 1e-4 of the
// largest term magnitude over the rectangle) far above the fp32 error of the kernels' power
// evaluation, so an entry is dropped only where every pixel fails the cutoff test: exact, like the
// box test.  Degenerate conics answer "yes".
__device__ __forceinline__ bool ellipse_meets_block(float x, float y, float a, float b, float c, float k, float x0,
                                                    float y0)
{
    const float u0 = x0 - x, u1 = x0 + 7.0f - x, w0 = y0 - y, w1 = y0 + 7.0f - y;
    if (u0 <= 0.0f && u1 >= 0.0f && w0 <= 0.0f && w1 >= 0.0f) return true;
    if (!(a > 0.0f && c > 0.0f && a * c - b * b > 0.0f)) return true;
    const float ia = __builtin_amdgcn_rcpf(a), ic = __builtin_amdgcn_rcpf(c);
    auto q = [&](float u, float w) { return fma_(a * u, u, fma_(2.0f * b * u, w, c * w * w)); };
    auto on_u = [&](float u) { return q(u, fminf(fmaxf(-b * u * ic, w0), w1)); };
    auto on_w = [&](float w) { return q(fminf(fmaxf(-b * w * ia, u0), u1), w); };
    const float m = fminf(fminf(on_u(u0), on_u(u1)), fminf(on_w(w0), on_w(w1)));
    const float U = fmaxf(fabsf(u0), fabsf(u1)), V = fmaxf(fabsf(w0), fabsf(w1));
    const float S = fma_(a * U, U, fma_(c * V, V, 2.0f * fabsf(b) * U * V));
    return m <= fma_(k, 1.001f, fma_(1e-4f, S, 1e-6f));
}

// 4-bit mask of the tile's wave blocks (wave_cover) an entry can reach: the box test, refined by the
// exact ellipse test for the blocks the box meets.  conic = (a, b, c), cut = power_cutoff.
__device__ __forceinline__ uint32_t entry_cover(float x, float y, float a, float b, float c, float cut, float x0,
                                                float y0)
{
    uint32_t m = wave_cover(entry_box(x, y, a, b, c, cut), x0, y0);
    const float k = -2.0f * cut;
    for (uint32_t w = 0; w < 4; w++)
        if (((m >> w) & 1u) && !ellipse_meets_block(x, y, a, b, c, k, x0 + 8.0f * (w & 1), y0 + 8.0f * (w >> 1)))
            m &= ~(1u << w);
    return m;
}

// Compacts the batch slots [0, cnt) whose cover mask meets `bits` (the wave's blocks) into
// list[0, n) as LDS byte offsets 16 e of their 16-B records; returns n.
// n_mid: how many of them lie in slots [0, kSplitChunk) (the walk's split-replay boundary inside the
// batch when kSplitChunk < 256).
__device__ __forceinline__ int wave_compact(const uint8_t* sM, int cnt, uint32_t bits, int lane, uint16_t* list,
                                            int& n_mid)
{
    int n = 0;
    n_mid = 0;
    for (int r = 0; r < cnt; r += 64) {
        const int e = r + lane;
        const bool ov = e < cnt && (sM[e] & bits) != 0u;
        const uint64_t m = __ballot(ov);
        if (ov) list[n + __popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)(16 * e);
        n += __popcll(m);
        if (r + 64 == kSplitChunk) n_mid = n;
    }
    if (cnt <= kSplitChunk) n_mid = n;
    return n;
}

// Pixel of lane t of the tile (wave w owns the 8 x 8 block (8 (w & 1), 8 (w >> 1)): a compact
// block meets fewer reach boxes than a 16 x 4 strip).
__device__ __forceinline__ void pixel_map(int tx, int ty, int t, int& px, int& py)
{
    const int lane = t & 63, wave = t >> 6;
    px = tx * kTile + 8 * (wave & 1) + (lane & 7);
    py = ty * kTile + 8 * (wave >> 1) + (lane >> 3);
}

// Longest-first (LPT) tile schedule.  Tile work is very uneven -- at C3 2.8k of the 8.2k tiles
// hold entries and their replay lengths run from 1 to ~700 -- and the hardware hands workgroups
// to CUs in launch order, so in tile order the longest tiles may start last and the kernel ends
// on a tail.  Whoever learns a tile's work appends the tile to the list of its work class
// (work_class: half-octaves; k_bin_emit for the forward's list lengths, the forward for the
// backward's replay lengths); workgroup b then takes the b-th tile in descending class order.
// The order changes no result.
//
// Tile of workgroup b (every wave computes it, wave-uniform), or -1 - (scheduled tiles) when b is
// past them.
__device__ __forceinline__ int scheduled_tile(int b, const uint32_t* counts, const uint32_t* lists, int T)
{
    const int lane = threadIdx.x & 63;
    const uint32_t n = counts[kWorkClasses - 1 - lane];  // lane 0: the heaviest class
    uint32_t x = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if (lane >= o) x += y;
    }
    const uint32_t total = (uint32_t)__shfl((int)x, 63, 64);
    if ((uint32_t)b >= total) return -1 - (int)total;
    const int l = (int)__builtin_ctzll(__ballot(x > (uint32_t)b));
    const uint32_t first = (uint32_t)__shfl((int)(x - n), l, 64);
    return (int)lists[(size_t)(kWorkClasses - 1 - l) * T + ((uint32_t)b - first)];
}

// Measurement hook (LSR_RENDER_STATS=1, lsr_debug_render_timeline): per workgroup of the two render
// kernels {start, end} (s_memrealtime, 100 MHz), the tile and the hardware slot (XCC_ID << 16 |
// HW_ID bits 8..15: cu, sh, se).  Off by default.
constexpr int kTimelineMax = 1 << 15;
// start, end, tile, slot, load, compact, walk (ticks), batches | first load << 16, and the first
// batch's six milestones (PhaseTicks::st) in ticks after the start, two 16-bit fields per word
constexpr int kTimelineWords = 11;
__device__ uint32_t g_render_timeline[2][kTimelineMax * kTimelineWords];

__device__ __forceinline__ uint32_t hw_slot()
{
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    return ((xcc & 0xFu) << 16) | ((hw >> 8) & 0xFFu);
}

// Per-batch phase ticks of a workgroup as thread 0 sees them: load (global gather -> LDS, up to the
// barrier), compact / cover (up to the next barrier), walk (up to the next batch's start, so it
// includes the wait for the workgroup's slowest wave).
struct PhaseTicks {
    uint64_t load = 0, compact = 0, walk = 0, mark = 0, first_load = 0;
    // the first batch's milestones (absolute ticks): begin, ranges loaded, first barrier passed, ids
    // loaded, records gathered, load phase done (the stats variant waits for each load explicitly)
    uint64_t st[6] = {0, 0, 0, 0, 0, 0};
    uint32_t batches = 0;
    bool stopped = false;  // left the batch loop at a batch start (its walk time already counted)
    __device__ void begin() { mark = wall_clock64(); }
    __device__ void lap(uint64_t& acc)
    {
        const uint64_t now = wall_clock64();
        acc += now - mark;
        mark = now;
    }
};

__device__ __forceinline__ void timeline_put(int kernel, uint64_t t0, int tile, const PhaseTicks& ph = PhaseTicks())
{
    const int b = (int)blockIdx.x;
    if (threadIdx.x != 0 || b >= kTimelineMax) return;
    uint32_t* o = g_render_timeline[kernel] + kTimelineWords * b;
    o[0] = (uint32_t)t0;
    o[1] = (uint32_t)wall_clock64();
    o[2] = (uint32_t)tile;
    o[3] = hw_slot();
    o[4] = (uint32_t)ph.load;
    o[5] = (uint32_t)ph.compact;
    o[6] = (uint32_t)ph.walk;
    o[7] = (ph.batches & 0xFFFFu) | ((uint32_t)min(ph.first_load, (uint64_t)0xFFFF) << 16);
    uint32_t rel[6];
    for (int k = 0; k < 6; k++) rel[k] = ph.st[k] > t0 ? (uint32_t)min(ph.st[k] - t0, (uint64_t)0xFFFF) : 0u;
    o[8] = rel[0] | (rel[1] << 16);
    o[9] = rel[2] | (rel[3] << 16);
    o[10] = rel[4] | (rel[5] << 16);
}

// Wave priority by launch position (LSR_PRIO=0: off).  A tile's compositing is one serial chain
// per pixel, so the kernel can end no earlier than its longest tile's chain, and the longest tiles
// (launched first) share their SIMDs with up to 7 other waves.  Raising the first-launched
// workgroups' priority was meant to let those chains run closer to their own latency; measured at
// C3 it changes neither their duration nor the kernel's (tools/render_timeline.py).  No result
// depends on it.
__device__ __forceinline__ void launch_priority(int b, int prio)
{
    if (!prio) return;
    if (b < 256) __builtin_amdgcn_s_setprio(3);
    else if (b < 768) __builtin_amdgcn_s_setprio(2);
    else if (b < 1536) __builtin_amdgcn_s_setprio(1);
}

// One pixel's front-to-back state (upstream FORWARD::renderCUDA locals).
// T > 0 while the pixel composites; once it is done (the next entry would take T below 1e-4, or the
// pixel is outside the image) T holds -T: one compare tests "active", and |T| is the final T.
struct FwdPixel {
    float T;
    lsr_f2 C01, C2F0, F12;  // {C0, C1}, {C2, F0}, {F1, F2}: the colour / feature sums as packed pairs
    uint32_t contributor;
    uint32_t last16;        // 16 x upstream's 1-based contributor counter (the walk's byte offsets)
};

// One front-to-back blend of the entry at LDS byte offset o (slot o / 16) with alpha al (upstream
// FORWARD::renderCUDA; the operation order of oracle render_pixel): ok = the entry passes the
// pixel's alpha tests; stop before the entry once T would fall below 1e-4 (then T -> -T: done).
// lo = the offset of the batch's last blended entry (the walk adds the batch's base once).  Cc / Ff: the entry's colour record {r, g, b, f0} and
// {f1, f2}, read by the caller (both entries of a pair at once, so their LDS latency is paid once
// per pair).
// Without branches: an entry that fails its tests blends with alpha 0 (T * (1 - 0) = T and the sums
// gain +-0 exactly: the records are finite), a lane that is done keeps T (< 0, so the stop test
// holds and -|T| = T), so every lane runs the same instructions: the same values as the branchy form,
// without its exec-mask branches (~24 scalar instructions per pair of the walk's ~110 issue slots).
template <bool kFeat>
__device__ __forceinline__ void fwd_pixel_blend(FwdPixel& q, float al, bool ok, uint32_t o, uint32_t& lo,
                                                const float4& Cc, const lsr_f2& Ff)
{
    const float a = ok ? al : 0.0f;
    const float test_T = q.T * (1.0f - a);
    const bool go = !(test_T < 0.0001f);
    const float w = go ? a * q.T : 0.0f;
    const lsr_f2 w2 = make_f2(w, w);
    q.C01 = __builtin_elementwise_fma(make_f2(Cc.x, Cc.y), w2, q.C01);
    if (kFeat) {
        q.C2F0 = __builtin_elementwise_fma(make_f2(Cc.z, Cc.w), w2, q.C2F0);
        q.F12 = __builtin_elementwise_fma(Ff, w2, q.F12);
    } else {
        q.C2F0.x = fma_(Cc.z, w, q.C2F0.x);
    }
    lo = go && ok ? o : lo;
    q.T = go ? test_T : -fabsf(q.T);
}

// ---- fused language-feature loss (train.py:96-99: Ll1 = l1_loss(lang * mask, gt * mask)) ----
// Per pixel: d_c = f_c m - gt_c m (the operations of torch's lang * mask - gt * mask), the pixel's
// share sum_c |d_c| of the L1 sum, and a code byte for the backward -- bits 2c..2c+1 the sign of d_c
// (1: +, 2: -, 0: zero), bit 6 the mask -- from which the backward forms autograd's gradient
// grad * (1 / (3 HW)) * sign(d_c) * m without reading the images again.
__device__ __forceinline__ uint32_t sign_code(float d) { return d > 0.0f ? 1u : (d < 0.0f ? 2u : 0u); }

template <bool kCode = true>
__device__ __forceinline__ float loss_pixel(const RenderParams& p, size_t pix, size_t HW, float f0, float f1, float f2)
{
    const float m = p.loss_mask[pix] ? 1.0f : 0.0f;
    const float d0 = f0 * m - p.loss_gt[pix] * m;
    const float d1 = f1 * m - p.loss_gt[HW + pix] * m;
    const float d2 = f2 * m - p.loss_gt[2 * HW + pix] * m;
    if (kCode)
        p.loss_code[pix] =
            (uint8_t)(sign_code(d0) | (sign_code(d1) << 2) | (sign_code(d2) << 4) | (m != 0.0f ? 64u : 0u));
    return fabsf(d0) + fabsf(d1) + fabsf(d2);
}

// The workgroup's L1 share (every thread calls it): per-thread floats summed in double in a fixed
// order; thread 0 gets it.
__device__ __forceinline__ double loss_block_sum(float part)
{
    __shared__ double s_lw[kTilePixels / 64];
    double v = (double)part;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) s_lw[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < kTilePixels / 64; w++) t += s_lw[w];
    return t;
}

// P == 0 path: the partial into loss_partial[blockIdx.x] (k_loss_finalize adds them).
__device__ __forceinline__ void loss_block_partial(const RenderParams& p, float part)
{
    const double t = loss_block_sum(part);
    if (threadIdx.x == 0) p.loss_partial[blockIdx.x] = t;
}

// The language feature of one pixel composited by a scalar front-to-back walk over the whole tile
// list, reading the records from global memory: the oracle's render_pixel with the main walk's
// cutoff test (power < cut rejects exactly what alpha < 1/255 would), so the same operations and the
// same values as the kernel's packed two-entry walk.
__device__ void composite_lang_pixel(const RenderParams& p, uint2 range, float pfx, float pfy, float& f0, float& f1,
                                     float& f2)
{
    float T = 1.0f;
    f0 = f1 = f2 = 0.0f;
    for (uint32_t k = range.x; k < range.y; k++) {
        const uint32_t g = p.point_list[k];
        const float4 a = p.record[3 * (size_t)g], b = p.record[3 * (size_t)g + 1], c = p.record[3 * (size_t)g + 2];
        const float dx = a.x - pfx, dy = a.y - pfy;
        const float hx = -0.5f * a.z, hz = -0.5f * b.x;
        const float pw = fma_(dx, fma_(-a.w, dy, hx * dx), (hz * dy) * dy);
        if (pw > 0.0f || pw < power_cutoff(b.y)) continue;
        const float al = fminf(0.99f, b.y * expf_exact_render(pw));
        if (al < 1.0f / 255.0f) continue;
        const float test_T = T * (1.0f - al);
        if (test_T < 0.0001f) break;
        const float w = al * T;
        f0 = fma_(c.y, w, f0);
        f1 = fma_(c.z, w, f1);
        f2 = fma_(c.w, w, f2);
        T = test_T;
    }
}

// This thread's part of the loss share forward workgroup b publishes (b uniform): the same pixels
// and per-pixel operations as b's own (its tile, or its strided run of empty tiles), computed from
// the inputs, not from b's outputs.
__device__ float loss_share_part(const RenderParams& p, int b)
{
    const int T = p.gx * p.gy;
    const size_t HW = (size_t)p.W * p.H;
    int tile = b;
    if (p.sched_counts) tile = scheduled_tile(b, p.sched_counts + kCntFwdClass, p.sched_lists, T);
    float part = 0.0f;
    if (tile < 0) {  // render_empty_tiles(p, b - listed, T - listed)
        const int listed = -1 - tile, j = b - listed, M = T - listed;
        for (int u = j; u < T; u += M) {
            const uint2 r = p.ranges[u];
            if (r.x != r.y) continue;
            int px, py;
            pixel_map(u % p.gx, u / p.gx, (int)threadIdx.x, px, py);
            if (px < p.W && py < p.H) part += loss_pixel<false>(p, (size_t)py * p.W + px, HW, 0.0f, 0.0f, 0.0f);
        }
        return part;
    }
    int px, py;
    pixel_map(tile % p.gx, tile / p.gx, (int)threadIdx.x, px, py);
    if (!(px < p.W && py < p.H)) return 0.0f;
    float f0, f1, f2;
    composite_lang_pixel(p, p.ranges[tile], (float)px, (float)py, f0, f1, f2);
    return loss_pixel<false>(p, (size_t)py * p.W + px, HW, f0, f1, f2);
}

__device__ __forceinline__ void loss_word_store(const RenderParams& p, int b, double t)
{
    __hip_atomic_store(&p.loss_words[b], (1ull << 32) | __float_as_uint((float)t), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Render forward: each workgroup publishes its share as ONE 64-bit word {1, float} (agent-scope
// store, coherent across the XCDs' L2s; no atomic, so no workgroup waits for a round trip before it
// retires).  The LAST workgroup of the grid -- dispatched after every other one, so all of them are
// resident or done and none depends on it -- waits for every word and adds them in workgroup order
// (deterministic) into Ll1: no second launch.  The words start at 0 (cleared by preprocess).
// Bounded wait: a word still absent after p.spin_limit polls is computed by this workgroup from the
// inputs (loss_share_part: the same value workgroup b publishes, stored the same way) and the stall
// is flagged (lsr_debug_scan_stalls); spin_limit 0 takes that path for every word not yet there.
__device__ __forceinline__ void loss_block_publish(const RenderParams& p, float part)
{
    __shared__ double s_fw[kTilePixels / 64];
    const double t = loss_block_sum(part);
    const int nb = (int)gridDim.x;
    if (threadIdx.x == 0) loss_word_store(p, (int)blockIdx.x, t);
    if ((int)blockIdx.x != nb - 1) return;
    // thread i adds the run [i per, (i + 1) per) in order (threads in order = workgroups in order)
    const int per = (nb + kTilePixels - 1) / kTilePixels;
    const int i0 = (int)threadIdx.x * per, e = min(nb, i0 + per);
    double v = 0.0;
    constexpr int kBatch = 16;  // loads in flight per round trip
    bool miss = false;
    for (int i = i0; i < e; i += kBatch) {
        uint64_t w[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++)
            w[k] = i + k < e ? __hip_atomic_load(&p.loss_words[i + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                             : (1ull << 32);
#pragma unroll
        for (int k = 0; k < kBatch; k++) {
            for (uint32_t spins = 0; (w[k] >> 32) == 0ull && spins < p.spin_limit; spins++) {
                __builtin_amdgcn_s_sleep(2);
                w[k] = __hip_atomic_load(&p.loss_words[i + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            miss = miss || (w[k] >> 32) == 0ull;
            v += (double)__uint_as_float((uint32_t)w[k]);  // padding words add +0
        }
    }
    if (__syncthreads_or(miss)) {
        // a word did not come within the bound: compute the missing words one at a time (the smallest
        // missing index over the workgroup, then the next), then sum every word again in order
        __shared__ int s_b;
        for (;;) {
            int mine = 0x7FFFFFFF;
            for (int i = i0; i < e && mine == 0x7FFFFFFF; i++)
                if ((__hip_atomic_load(&p.loss_words[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32) == 0ull)
                    mine = i;
            if (threadIdx.x == 0) s_b = 0x7FFFFFFF;
            __syncthreads();
            if (mine != 0x7FFFFFFF) atomicMin(&s_b, mine);
            __syncthreads();
            const int bm = s_b;  // uniform
            if (bm == 0x7FFFFFFF) break;
            const double tb = loss_block_sum(loss_share_part(p, bm));
            if (threadIdx.x == 0) loss_word_store(p, bm, tb);
            __syncthreads();  // the store before the next scan (one workgroup: program order)
        }
        v = 0.0;
        for (int i = i0; i < e; i++)
            v += (double)__uint_as_float(
                (uint32_t)__hip_atomic_load(&p.loss_words[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (threadIdx.x == 0) note_stall(p.stall);
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {  // in-order prefix within the wave: lane 63 holds lanes 0..63 in order
        const double y = __shfl_up(v, o, 64);
        if ((threadIdx.x & 63) >= o) v += y;
    }
    if ((threadIdx.x & 63) == 63) s_fw[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double tot = 0.0;
        for (int w = 0; w < kTilePixels / 64; w++) tot += s_fw[w];
        *p.out_loss = (float)(tot / (double)(3 * (int64_t)p.W * p.H));
    }
}

// Output of the tiles without entries among u = j, j + M, ... (background colour, T = 1, no
// contributors); tiles with entries are skipped (their own workgroups render them).  kLoss: returns
// the thread's loss share of those pixels (language image 0 there).
template <bool kLoss>
__device__ float render_empty_tiles(const RenderParams& p, int j, int M)
{
    float part = 0.0f;
    const int T = p.gx * p.gy;
    const size_t HW = (size_t)p.W * p.H;
    for (int u = j; u < T; u += M) {
        const uint2 r = p.ranges[u];
        if (r.x != r.y) continue;
        int px, py;
        pixel_map(u % p.gx, u / p.gx, (int)threadIdx.x, px, py);
        if (!(px < p.W && py < p.H)) continue;
        const size_t pix = (size_t)py * p.W + px;
        if (!p.no_bwd) {
            p.final_T[pix] = 1.0f;
            p.n_contrib[pix] = 0u;
        }
        p.out_color[pix] = fma_(1.0f, p.bg[0], 0.0f);
        p.out_color[HW + pix] = fma_(1.0f, p.bg[1], 0.0f);
        p.out_color[2 * HW + pix] = fma_(1.0f, p.bg[2], 0.0f);
        p.out_lang[pix] = 0.0f;
        p.out_lang[HW + pix] = 0.0f;
        p.out_lang[2 * HW + pix] = 0.0f;
        if (kLoss) part += loss_pixel(p, pix, HW, 0.0f, 0.0f, 0.0f);
    }
    return part;
}

// 7 waves per SIMD (<= 72 VGPRs): the fused-loss variant's rare bounded-wait fallback
// (loss_block_publish) would otherwise raise its register count to 83 (6 waves); with the bound the
// compiler spills three values, stored once per workgroup and reloaded on that path only.
#ifndef LSR_FWD_WAVES  // waves per SIMD the forward is compiled for (measurement knob)
#define LSR_FWD_WAVES 7
#endif
#ifndef LSR_FWD_QUAD  // 1: four list entries per walk step (two packed exp chains), 0: two
#define LSR_FWD_QUAD 0
#endif
#if LSR_FWD_QUAD && LSR_SPLIT_CHUNK != 256
#error "the four-entry walk records split-replay states at batch starts only: LSR_SPLIT_CHUNK=256"
#endif
#ifndef LSR_FWD_PREFETCH  // 1: the next batch's records are gathered during the walk
#define LSR_FWD_PREFETCH 0
#endif
#ifndef LSR_BWD_WORK_ORDER  // 1: the backward's items ordered by the forward's walk counts, 0: by entries
#define LSR_BWD_WORK_ORDER 1
#endif
#ifndef LSR_FWD_STATE_SKIP  // 1: split-replay states stored only for the pixels the backward starts from them
#define LSR_FWD_STATE_SKIP 1
#endif
template <bool kStats, bool kFeat, bool kLoss>
__global__ __launch_bounds__(kTilePixels, LSR_FWD_WAVES) void k_render_forward(RenderParams p)
{
    const uint64_t t_start = kStats ? wall_clock64() : 0;
    constexpr int kThreads = kTilePixels;
    __shared__ float4 sA[kThreads];  // x, y, -0.5 conic.x, -0.5 conic.z
    __shared__ float4 sB[kThreads];  // conic.y, opacity, power cutoff, -
    __shared__ float4 sC[kThreads];  // r, g, b, f0
    __shared__ float4 sF[kThreads];  // f1, f2, -, -  (16-B slots: every record of slot s at byte 16 s)
    __shared__ uint8_t sM[kThreads];  // entry_cover mask
    // per-wave culled slot lists, as byte offsets 16 s; slots n .. n + 3 hold offset 0, so the walk
    // reads the entries of a step past the list's end without testing (their results are discarded).
    // Rows of kThreads + 8 (8-B aligned): a step's offsets are one 32- or 64-bit read, and the walk
    // reads the next step's one step ahead (up to slot n + 7)
    __shared__ __attribute__((aligned(8))) uint16_t sL[kThreads / 64][kThreads + 8];
    __shared__ uint32_t s_last;
    // LSR_BWD_WORK_ORDER: per wave, the list slots its walk visited in batches 0, 1, 2 and from 3 on
    // (one batch = one split-replay chunk): what the backward's item of that chunk visits in this wave
    constexpr bool kWorkOrder = LSR_BWD_WORK_ORDER && kSplitChunk == kThreads;
    __shared__ uint32_t s_walk[kWorkOrder ? kThreads / 64 : 1][kSplitItems];
    uint32_t wk0 = 0, wk1 = 0, wk2 = 0, wk3 = 0;  // (wave-uniform)
    uint32_t bi = 0;                              // batch index

    const int T = p.gx * p.gy;
    if (p.zero_records) {  // the backward's gradient records: stores beside the VALU-bound walk
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x; k < p.zero_records_n4;
             k += (int64_t)gridDim.x * kThreads)
            p.zero_records[k] = z;
    }
    int tile = (int)blockIdx.x;
    if (p.sched_counts) {
        tile = scheduled_tile((int)blockIdx.x, p.sched_counts + kCntFwdClass, p.sched_lists, T);
        if (tile < 0) {  // past the tiles with entries: fill the empty ones, strided
            const int listed = -1 - tile;
            const float part = render_empty_tiles<kLoss>(p, (int)blockIdx.x - listed, T - listed);
            if (kLoss) loss_block_publish(p, part);
            if (kStats) timeline_put(0, t_start, -1);
            return;
        }
    }
    launch_priority((int)blockIdx.x, p.prio);
    const int tx = tile % p.gx, ty = tile / p.gx;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    int px, py;
    pixel_map(tx, ty, t, px, py);
    const float pfx = (float)px, pfy = (float)py;
    const lsr_f2 pxy = make_f2(pfx, pfy);
    const float tx0 = (float)(tx * kTile), ty0 = (float)(ty * kTile);
    PhaseTicks ph;
    if (kStats) {
        ph.begin();
        ph.st[0] = ph.mark;
    }
    const uint2 range = p.ranges[tile];
    if (kStats) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ph.st[1] = wall_clock64();
    }
    const uint32_t start = range.x, end = range.y;
    const bool inside = px < p.W && py < p.H;
    if (t == 0) s_last = 0;
    uint32_t nrec = 0;  // split replay: boundaries recorded (kSplitChunk, 2 kSplitChunk, ... up to kSplitMax; uniform)

    FwdPixel q{inside ? 1.0f : -1.0f, make_f2(0.f, 0.f), make_f2(0.f, 0.f), make_f2(0.f, 0.f), 0u, 0u};
    // Software pipeline over the batches: a batch's records are gathered during the previous batch's
    // walk (into registers the walk leaves free), and the point_list ids one batch earlier still, so
    // a batch's load phase waits for no memory round trip (the timeline showed ~9 us of load phase per
    // batch on the heaviest tiles, a quarter of their time, mostly the gather's latency)
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a, c = a;
#if LSR_FWD_PREFETCH
    if (start + t < end) {
        const uint32_t g = p.point_list[start + t];
        a = p.record[3 * (size_t)g];
        b = p.record[3 * (size_t)g + 1];
        c = p.record[3 * (size_t)g + 2];
    }
    uint32_t g_next = start + kThreads + t < end ? p.point_list[start + kThreads + t] : 0u;
#else
    uint32_t g_next = start + t < end ? p.point_list[start + t] : 0u;
#endif
    for (uint32_t base = start; base < end; base += kThreads) {
        const bool all_done = __syncthreads_count(q.T < 0.0f) == kThreads;
        if (kStats && base != start) ph.lap(ph.walk);
        if (all_done) {
            if (kStats) ph.stopped = true;
            break;
        }
        if (kStats) ph.batches++;
        const uint32_t idx = base + t;
        if (kStats && base == start) {
            ph.st[2] = wall_clock64();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ph.st[3] = wall_clock64();
        }
#if !LSR_FWD_PREFETCH
        a = b = c = make_float4(0.f, 0.f, 0.f, 0.f);
        if (idx < end) {
            const uint32_t g = g_next;
            a = p.record[3 * (size_t)g];
            b = p.record[3 * (size_t)g + 1];
            c = p.record[3 * (size_t)g + 2];
        }
#endif
        if (kStats && base == start) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            ph.st[4] = wall_clock64();
        }
        // split-replay state of each pixel at list entry e (e = base - start here, or the middle of the
        // batch, below): slot e / kSplitChunk - 1, two float4 per pixel
        auto record_state = [&](uint32_t slot) {
            float4* st = reinterpret_cast<float4*>(p.split_pool) + ((size_t)tile * kSplitSlots + slot) * (2 * kThreads);
            // A pixel already done (or outside the image: T < 0) has its last contributor before the
            // boundary, so the backward never starts it from here: no store (LSR_FWD_STATE_SKIP=0 stores)
            if (!LSR_FWD_STATE_SKIP || q.T > 0.0f) {
                st[2 * t] = make_float4(q.T, q.C2F0.y, q.F12.x, q.F12.y);
                if (p.split_color) st[2 * t + 1] = make_float4(q.C01.x, q.C01.y, q.C2F0.x, 0.0f);
            }
        };
        if (p.split_pool && base != start && base - start <= (uint32_t)(kSplitMax * kSplitChunk)) {
            // split replay: every pixel's state before list entry 256 j while some pixel composites,
            // two float4 per pixel in the tile's own slot j - 1 (a grid-wide slot counter cost ~40 us
            // of contended cross-XCD atomics); a pixel already done is never started from here
            // {T, feature sums}, then {colour sums} unless no colour gradient can follow (the language
            // step: half the state traffic)
            record_state(nrec);
            nrec++;
        }
        if (idx < end) {
            const float cut = power_cutoff(b.y);
            sA[t] = make_float4(a.x, a.y, -0.5f * a.z, -0.5f * b.x);
            sB[t] = make_float4(a.w, b.y, cut, 0.0f);
            sC[t] = make_float4(b.z, b.w, c.x, c.y);
            sF[t] = make_float4(c.z, c.w, 0.0f, 0.0f);
            const uint8_t m = (uint8_t)entry_cover(a.x, a.y, a.z, a.w, b.x, cut, tx0, ty0);
            sM[t] = m;
            if (!p.no_bwd) p.cover[idx] = m;  // for the backward (coalesced: one byte per thread)
        }
        __syncthreads();
        if (kStats) {
            ph.lap(ph.load);
            if (base == start) {
                ph.first_load = ph.load;
                ph.st[5] = ph.mark;
            }
        }
        const int cnt = (int)min((uint32_t)kThreads, end - base);
        int n_mid_raw;
        const int n = __builtin_amdgcn_readfirstlane(
            wave_compact(sM, cnt, 1u << wave, lane, sL[wave], n_mid_raw));
        const int n_mid = __builtin_amdgcn_readfirstlane(n_mid_raw);
        // the boundary in the middle of the batch (kSplitChunk < 256), recorded by each wave when its
        // walk reaches it: uniform over the workgroup
        const bool mid = kSplitChunk < kThreads && p.split_pool && cnt > kSplitChunk &&
                         base - start + kSplitChunk <= (uint32_t)(kSplitMax * kSplitChunk);
        if (lane < 4) sL[wave][n + lane] = 0;
        __syncthreads();  // list visible to the wave's other lanes
        if (kStats) ph.lap(ph.compact);
#if LSR_FWD_PREFETCH
        if (idx + kThreads < end) {  // the next batch's records, and the ids of the one after
            const uint32_t g = g_next;
            a = p.record[3 * (size_t)g];
            b = p.record[3 * (size_t)g + 1];
            c = p.record[3 * (size_t)g + 2];
        }
        if (idx + 2 * kThreads < end) g_next = p.point_list[idx + 2 * kThreads];
#else
        if (idx + kThreads < end) g_next = p.point_list[idx + kThreads];
#endif
        const uint32_t lb16 = 16u * (base - start + 1u);  // 16 x (list index of slot 0 + 1)
        const char* const cA = reinterpret_cast<const char*>(sA);
        const char* const cB = reinterpret_cast<const char*>(sB);
        const char* const cC = reinterpret_cast<const char*>(sC);
        const char* const cF = reinterpret_cast<const char*>(sF);
        // Per list entry: power, exp and alpha do not depend on the pixel state, only the transmittance
        // test and the blend are sequential.  Two entries' exps run as one packed chain
        // (expf_exact_render2: the same IEEE operations per element).  The list holds byte offsets,
        // so every record read addresses LDS with the list value itself.  A step's offsets come from
        // one read issued during the previous step, so its record reads do not wait behind them.
        uint32_t lo = 0xFFFFFFFFu;  // offset of the batch's last blended entry, per lane
        // the alpha of the entries at offsets oa, ob (ob: only if hb) and their alpha tests
        auto pair_alpha = [&](uint32_t oa, uint32_t ob, bool hb, float& ala, float& alb, bool& oka, bool& okb) {
            const float4 Aa = *reinterpret_cast<const float4*>(cA + oa), Ba = *reinterpret_cast<const float4*>(cB + oa);
            const float4 Ab = *reinterpret_cast<const float4*>(cA + ob), Bb = *reinterpret_cast<const float4*>(cB + ob);
            // per entry {dx, dy} and {A.z dx, A.w dy} as packed ops on the record's own register pairs
            const lsr_f2 da = make_f2(Aa.x, Aa.y) - pxy, db = make_f2(Ab.x, Ab.y) - pxy;
            const lsr_f2 ma = make_f2(Aa.z, Aa.w) * da, mb = make_f2(Ab.z, Ab.w) * db;
            // power = dx (A.z dx - conic.y dy) + (A.w dy) dy: 4 operations after {A.z dx, A.w dy}
            // (the oracle's render_pixel / backward_pixel and the backward walk use the same order)
            const float pwa = fma_(da.x, fma_(-Ba.x, da.y, ma.x), ma.y * da.y);
            const float pwb = fma_(db.x, fma_(-Bb.x, db.y, mb.x), mb.y * db.y);
            const lsr_f2 G2 = expf_exact_render2(make_f2(pwa, pwb));
            ala = fminf(0.99f, Ba.y * G2.x);
            alb = fminf(0.99f, Bb.y * G2.y);
            oka = !(pwa > 0.0f || pwa < Ba.z) && !(ala < 1.0f / 255.0f);
            okb = hb && !(pwb > 0.0f || pwb < Bb.z) && !(alb < 1.0f / 255.0f);
        };
        auto blend_at = [&](float al, bool ok, uint32_t o) {
            const float4 Cc = *reinterpret_cast<const float4*>(cC + o);
            const lsr_f2 Ff = kFeat ? *reinterpret_cast<const lsr_f2*>(cF + o) : make_f2(0.f, 0.f);
            fwd_pixel_blend<kFeat>(q, al, ok, o, lo, Cc, Ff);
        };
        // one basic block per step (the blends have no branches, the wave's "all done" test closes the
        // iteration), so the next step's offset read stays beside this step's record reads
        int i = 0;
#if LSR_FWD_QUAD
        // four entries per step: two independent packed exp chains, so a wave has twice the
        // instruction-level parallelism between its dependent operations
        const uint2* const sL4 = reinterpret_cast<const uint2*>(sL[wave]);
        uint2 oo = sL4[0];
        if (n > 0 && __ballot(q.T > 0.0f) != 0ull) do {
            const uint32_t o0 = oo.x & 0xFFFFu, o1 = oo.x >> 16, o2 = oo.y & 0xFFFFu, o3 = oo.y >> 16;
            oo = sL4[(i >> 2) + 1];  // slots i + 4 .. i + 7 (<= n + 7)
            float al0, al1, al2, al3;
            bool ok0, ok1, ok2, ok3;
            pair_alpha(o0, o1, i + 1 < n, al0, al1, ok0, ok1);
            pair_alpha(o2, o3, i + 3 < n, al2, al3, ok2, ok3);
            ok2 = ok2 && i + 2 < n;
            blend_at(al0, ok0, o0);
            blend_at(al1, ok1, o1);
            blend_at(al2, ok2, o2);
            blend_at(al3, ok3, o3);
            // the next offsets are this iteration's value: the compiler may not defer their read to
            // the next iteration's start (where the record reads would wait behind it)
            asm volatile("" : "+v"(oo.x), "+v"(oo.y));
            i += 4;
        } while (i < n && __ballot(q.T > 0.0f) != 0ull);
#else
        const uint32_t* const sL2 = reinterpret_cast<const uint32_t*>(sL[wave]);
        // the pairs of list slots [i, lim), i even (a last odd slot alone)
        auto walk = [&](int lim) {
            uint32_t oo = sL2[i >> 1];
            if (i < lim && __ballot(q.T > 0.0f) != 0ull) do {
                const uint32_t o0 = oo & 0xFFFFu, o1 = oo >> 16;
                oo = sL2[(i >> 1) + 1];  // slots i + 2, i + 3 (<= n + 1)
                float al0, al1;
                bool ok0, ok1;
                pair_alpha(o0, o1, i + 1 < lim, al0, al1, ok0, ok1);
                blend_at(al0, ok0, o0);
                blend_at(al1, ok1, o1);
                asm volatile("" : "+v"(oo));
                i += 2;
            } while (i < lim && __ballot(q.T > 0.0f) != 0ull);
        };
        if (!mid) {
            walk(n);
        } else {
            // the wave's entries before the batch's middle, its pixels' state there, the rest
            walk(n_mid);
            record_state(nrec);
            i = n_mid;
            if ((n_mid & 1) && n_mid < n && __ballot(q.T > 0.0f) != 0ull) {  // slot n_mid alone
                const uint32_t o0 = sL[wave][n_mid];
                float al0, al1;
                bool ok0, ok1;
                pair_alpha(o0, o0, false, al0, al1, ok0, ok1);
                blend_at(al0, ok0, o0);
            }
            i = (n_mid + 1) & ~1;
            walk(n);
        }
        if (mid) nrec++;
#endif
        if (kWorkOrder) {
            const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(min(i, n));
            if (bi == 0) wk0 = wv;
            else if (bi == 1) wk1 = wv;
            else if (bi == 2) wk2 = wv;
            else wk3 += wv;
            bi++;
        }
        if (lo != 0xFFFFFFFFu) q.last16 = lb16 + lo;
    }
    if (kWorkOrder && lane == 0) {
        static_assert(kSplitItems == 4, "four walk counters per wave");
        s_walk[wave][0] = wk0;
        s_walk[wave][1] = wk1;
        s_walk[wave][2] = wk2;
        s_walk[wave][3] = wk3;
    }
    const uint32_t qlast = q.last16 >> 4;
    // the tile's replay length, for the backward's launch order
    uint32_t wl = qlast;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wl = max(wl, (uint32_t)__shfl_xor((int)wl, o, 64));
    __syncthreads();
    if (lane == 0) atomicMax(&s_last, wl);
    __syncthreads();
    // the backward's work items: the tile's replay [0, s_last) cut at the recorded boundaries below
    // s_last (split replay), each appended to the class of its length
    const uint32_t maxl = s_last;
    const uint32_t nsplit = p.split_pool && maxl > 0 ? min(nrec, (maxl - 1u) / (uint32_t)kSplitChunk) : 0u;
    // the backward's items into the longest-first class lists: the tile's full 256-entry chunks with
    // ONE returning atomic on their class (+nsplit), its last chunk with another, in parallel (thread
    // 1): an atomic per chunk put every heavy tile's chunks on one hot counter across the XCDs
    if (kWorkOrder && p.sched_counts && maxl > 0 && !p.no_bwd) {
        // one item per thread t <= nsplit, classed by its work: the walk's visits in the chunk's batch
        // (the last item: its batches' visits summed) in the wave that visited most, plus a fixed share
        // for its record loads and flush.  The class lists stay longest first by what the backward
        // will do, not by entry counts (a chunk whose pixels are mostly done replays little).
        if (t == 0 && p.split_pool) p.split_desc[tile] = make_uint4(nsplit, maxl, 0u, 0u);
        if (t <= (int)nsplit) {
            uint32_t w = 0;
            for (int wv = 0; wv < kThreads / 64; wv++) {
                uint32_t v = 0;
                if (t < (int)nsplit) {
                    v = s_walk[wv][t];
                } else {
                    for (int k = t; k < kSplitItems; k++) v += s_walk[wv][k];
                }
                w = max(w, v);
            }
            schedule_tile(p.sched_counts + kCntBwdClass, p.sched_lists + (size_t)kWorkClasses * T,
                          kSplitItems * T, kSplitItems * tile + t, 32u + w);
        }
    } else if (t < 2 && p.sched_counts && maxl > 0 && !p.no_bwd) {
        uint32_t* counts = p.sched_counts + kCntBwdClass;
        uint32_t* lists = p.sched_lists + (size_t)kWorkClasses * T;
        const size_t stride = (size_t)kSplitItems * T;
        if (t == 0 && p.split_pool) p.split_desc[tile] = make_uint4(nsplit, maxl, 0u, 0u);
        if (t == 0 && nsplit > 0) {
            const int c = work_class((uint32_t)kSplitChunk);
            const uint32_t base = atomicAdd(&counts[c], nsplit);
            for (uint32_t k = 0; k < nsplit; k++) lists[(size_t)c * stride + base + k] = kSplitItems * tile + k;
        }
        if (t == (nsplit > 0 ? 1 : 0))
            schedule_tile(counts, lists, (int)stride, kSplitItems * tile + (int)nsplit, maxl - nsplit * kSplitChunk);
    }
    // the final sums, for the backward's running `acc` at each boundary, (C_final - C_front) / T_b: a
    // store here (the tile's extra slot), the arithmetic in the backward -- normalising the slots in
    // place needed a load round trip at the end of every long tile, i.e. on the kernel's critical path
    // (read only for pixels that composite past the first boundary: q.last > hi >= kSplitChunk)
    if (nsplit > 0 && (!LSR_FWD_STATE_SKIP || qlast > (uint32_t)kSplitChunk)) {
        float4* fin = reinterpret_cast<float4*>(p.split_pool) + ((size_t)tile * kSplitSlots + kSplitMax) * (2 * kThreads);
        fin[2 * t] = make_float4(q.C2F0.y, q.F12.x, q.F12.y, 0.0f);
        if (p.split_color) fin[2 * t + 1] = make_float4(q.C01.x, q.C01.y, q.C2F0.x, 0.0f);
    }
    if (kStats) {
        if (!ph.stopped && ph.batches) ph.lap(ph.walk);  // the last batch's walk
        timeline_put(0, t_start, tile, ph);
    }
    const size_t HW = (size_t)p.W * p.H;
    const size_t pix = (size_t)py * p.W + px;
    const float part = kLoss && inside ? loss_pixel(p, pix, HW, q.C2F0.y, q.F12.x, q.F12.y) : 0.0f;
    // the outputs before the loss share's publication: the pixel state is dead during it (the last
    // workgroup's word gather holds 32 registers)
    if (inside) {
        const float Tf = fabsf(q.T);
        if (!p.no_bwd) {  // the backward's state
            p.final_T[pix] = Tf;
            p.n_contrib[pix] = qlast;
        }
        p.out_color[pix] = fma_(Tf, p.bg[0], q.C01.x);
        p.out_color[HW + pix] = fma_(Tf, p.bg[1], q.C01.y);
        p.out_color[2 * HW + pix] = fma_(Tf, p.bg[2], q.C2F0.x);
        p.out_lang[pix] = q.C2F0.y;
        p.out_lang[HW + pix] = q.F12.x;
        p.out_lang[2 * HW + pix] = q.F12.y;
    }
    if (kLoss) loss_block_publish(p, part);
}

// P == 0: the language image is 0 everywhere; its loss terms, one workgroup per 256 pixels.
__global__ __launch_bounds__(kTilePixels) void k_loss_background(RenderParams p)
{
    const size_t HW = (size_t)p.W * p.H;
    const size_t pix = (size_t)blockIdx.x * kTilePixels + threadIdx.x;
    loss_block_partial(p, pix < HW ? loss_pixel(p, pix, HW, 0.0f, 0.0f, 0.0f) : 0.0f);
}

// Ll1 = (sum of the n workgroup partials, in workgroup order) / (3 HW): one workgroup.
constexpr int kFinalizeThreads = 1024;
__global__ __launch_bounds__(kFinalizeThreads) void k_loss_finalize(int n, const double* __restrict__ partial,
                                                                    int64_t HW, float* __restrict__ loss)
{
    __shared__ double s_w[kFinalizeThreads / 64];
    // thread t sums the contiguous run [t * per, (t + 1) * per): threads in order = partials in order;
    // kBatch loads in flight before the first add (one memory round trip for n <= 8k partials)
    constexpr int kBatch = 8;
    const int per = (n + kFinalizeThreads - 1) / kFinalizeThreads;
    const int i0 = threadIdx.x * per, e = min(n, (int)(threadIdx.x + 1) * per);
    double v = 0.0;
    for (int i = i0; i < e; i += kBatch) {
        double x[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; k++) x[k] = i + k < e ? partial[i + k] : 0.0;
#pragma unroll
        for (int k = 0; k < kBatch; k++) v += x[k];
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {  // inclusive scan order within the wave: lane 63 = lanes 0..63 in order
        const double y = __shfl_up(v, o, 64);
        if ((threadIdx.x & 63) >= o) v += y;
    }
    if ((threadIdx.x & 63) == 63) s_w[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < kFinalizeThreads / 64; w++) t += s_w[w];
        *loss = (float)(t / (double)(3 * HW));
    }
}

hipError_t launch_loss_background(const RenderParams& p, hipStream_t s)
{
    const int64_t HW = (int64_t)p.W * p.H;
    const int n = (int)((HW + kTilePixels - 1) / kTilePixels);
    hipLaunchKernelGGL(k_loss_background, dim3(n), dim3(kTilePixels), 0, s, p);
    hipLaunchKernelGGL(k_loss_finalize, dim3(1), dim3(kFinalizeThreads), 0, s, n, (const double*)p.loss_partial, HW,
                       p.out_loss);
    return hipGetLastError();
}

static bool render_stats_on()
{
    static bool v = [] {
        const char* e = getenv("LSR_RENDER_STATS");
        return e && e[0] == '1';
    }();
    return v;
}

// LSR_PRIO=0 turns the launch-position wave priority off (measurement aid)
static int prio_levels()
{
    static const int v = [] {
        const char* e = getenv("LSR_PRIO");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    return v;
}

// LSR_DEBUG_GRID=n launches only the first n workgroups of each render kernel (measurement aid for
// the timeline: a long tile's time alone vs among others; the outputs are then incomplete)
static int debug_grid(int tiles)
{
    static const int v = [] {
        const char* e = getenv("LSR_DEBUG_GRID");
        return e ? atoi(e) : 0;
    }();
    return v > 0 && v < tiles ? v : tiles;
}

// LSR_FWD_PAD=bytes adds dynamic LDS to every forward workgroup, i.e. caps its workgroups per CU
// (measurement aid: how the longest tiles' chains respond to sharing their CU)
static size_t forward_pad()
{
    static const size_t v = [] {
        const char* e = getenv("LSR_FWD_PAD");
        return e ? (size_t)atoi(e) : (size_t)0;
    }();
    return v;
}

// LSR_BWD_PAD=bytes: the same for the backward
static size_t backward_pad()
{
    static const size_t v = [] {
        const char* e = getenv("LSR_BWD_PAD");
        return e ? (size_t)atoi(e) : (size_t)0;
    }();
    return v;
}

// LSR_SPLIT=0: no split replay (the forward records no boundary state, the backward replays each
// tile as one work item; measurement aid)
static bool split_replay()
{
    static const bool v = [] {
        const char* e = getenv("LSR_SPLIT");
        return !(e && e[0] == '0');
    }();
    return v;
}

// LSR_ORDER=0 launches the tiles in tile order (measurement aid)
static bool scheduled()
{
    static const bool v = [] {
        const char* e = getenv("LSR_ORDER");
        return !(e && e[0] == '0');
    }();
    return v;
}

// LSR_SPLIT_COLOR=1 stores the colour half of the split-replay states even under
// LSR_FWD_NO_COLOR_GRAD (measurement aid: same-box A/B of the state traffic)
static bool split_color_forced()
{
    static const bool v = [] {
        const char* e = getenv("LSR_SPLIT_COLOR");
        return e && e[0] == '1';
    }();
    return v;
}

// Workgroups per CU of the render kernels while another stream's kernels run beside them (the
// pipelined step, §5b): the backward at 7 of 8 and the forward at 6 of 7, so the geometry stream
// finds wave slots and VGPRs free on every CU instead of waiting for a render kernel's tail.
// Measured at C3 (profiles/r05_occupancy_sweep.txt, r05_fwd_share.txt): the backward 8 -> 7
// 0.418 -> 0.400 ms per step; the forward 7 -> 6 0.400-0.47 (bimodal, by box) -> 0.404-0.405 ms.
constexpr int kSharedWgsBwd = 7;
constexpr int kSharedWgsFwd = 6;
constexpr size_t kCuLds = 160 * 1024;
// Dynamic LDS that leaves room for exactly `wgs` workgroups of kernel fn per CU (0 if its static
// LDS already allows no more), rounded to 1 KiB: the allocation granularity must not push the
// last workgroup out.
#ifndef LSR_PAD_MIN
#define LSR_PAD_MIN 0
#endif
static size_t occupancy_pad(const void* fn, int wgs, const char* what)
{
    hipFuncAttributes at{};
    size_t stat = 20 * 1024;
    if (hipFuncGetAttributes(&at, fn) == hipSuccess) stat = at.sharedSizeBytes;
    // wgs of them fit, one more does not: the largest such 1 KiB multiple, or (LSR_PAD_MIN=1) the
    // smallest, which leaves the most LDS to the other stream's workgroups
    const size_t per = LSR_PAD_MIN ? ((kCuLds / (wgs + 1) + 1024) & ~(size_t)1023) : (kCuLds / wgs) & ~(size_t)1023;
    const size_t pad = per > stat && per * (wgs + 1) > kCuLds ? per - stat : 0;
    if (getenv("LSR_SHARE_PRINT")) fprintf(stderr, "lsr: %s static LDS %zu pad %zu\n", what, stat, pad);
    return pad;
}
// The forward's LDS pad (variants: 0 feature + fused loss, 1 feature, 2 colour only): LSR_FWD_PAD
// when set, else in a composite phase (another stream beside it) the kSharedWgsFwd cap unless
// LSR_FWD_SHARE=0, else none.
static size_t forward_launch_pad(const RenderParams& p, int variant)
{
    static const bool explicit_pad = getenv("LSR_FWD_PAD") != nullptr;
    static const bool on = [] {
        const char* e = getenv("LSR_FWD_SHARE");
        return !(e && e[0] == '0');
    }();
    if (explicit_pad || !on || !p.shared_cu) return forward_pad();
    static const size_t pad[3] = {
        occupancy_pad((const void*)k_render_forward<false, true, true>, kSharedWgsFwd, "forward (loss)"),
        occupancy_pad((const void*)k_render_forward<false, true, false>, kSharedWgsFwd, "forward (feature)"),
        occupancy_pad((const void*)k_render_forward<false, false, false>, kSharedWgsFwd, "forward (colour)")};
    return pad[variant];
}

hipError_t launch_render_forward(const RenderParams& pin, int tiles, hipStream_t s)
{
    if (tiles == 0) return hipSuccess;
    RenderParams p = pin;
    if (split_color_forced()) p.split_color = 1;
    if (!scheduled()) p.sched_counts = p.sched_lists = nullptr;
    if (!p.sched_counts || !split_replay()) p.split_pool = nullptr;
    p.prio = p.sched_counts ? prio_levels() : 0;
    const bool feat = p.include_feature != 0;
    const bool loss = feat && p.loss_words != nullptr;  // one word per workgroup: the full grid
    if (render_stats_on() && !loss) {
        tiles = debug_grid(tiles);
        if (feat)
            hipLaunchKernelGGL((k_render_forward<true, true, false>), dim3(tiles), dim3(kTilePixels), forward_pad(), s,
                               p);
        else
            hipLaunchKernelGGL((k_render_forward<true, false, false>), dim3(tiles), dim3(kTilePixels), forward_pad(), s,
                               p);
    } else if (loss) {
        hipLaunchKernelGGL((k_render_forward<false, true, true>), dim3(tiles), dim3(kTilePixels),
                           forward_launch_pad(p, 0), s, p);
    } else if (feat) {
        hipLaunchKernelGGL((k_render_forward<false, true, false>), dim3(tiles), dim3(kTilePixels),
                           forward_launch_pad(p, 1), s, p);
    } else {
        hipLaunchKernelGGL((k_render_forward<false, false, false>), dim3(tiles), dim3(kTilePixels),
                           forward_launch_pad(p, 2), s, p);
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------

// Cross-lane helpers for the wave64 reduce-scatter (gfx950).
//   swap32/16: v_permlane{32,16}_swap exchanges half-waves / odd-even rows, so for a value pair
//   (lo, hi) the sum of the two results is lo+lo' on the lanes that keep `lo` and hi+hi' on the
//   lanes that keep `hi` -- one exchange and one add per pair, no selects;
//   mirror: DPP row_mirror / row_half_mirror pair the lower and upper 8 / 4 lanes of a row.
__device__ __forceinline__ float swap32_add(float lo, float hi)
{
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ float swap16_add(float lo, float hi)
{
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <int kCtrl>
__device__ __forceinline__ float dpp(float x)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), kCtrl, 0xF, 0xF, true));
}

template <int kCtrl>
__device__ __forceinline__ float mirror_add(float lo, float hi, bool upper)
{
    const float send = upper ? lo : hi;
    const float keep = upper ? hi : lo;
    return keep + dpp<kCtrl>(send);
}

// Reduce-scatter of 12 per-lane values over the wave, 6 pairs wide: lane bit 5 picks v[k] / v[k + 6]
// (permlane32 swap), bit 4 r[m] / r[m + 3] (permlane16 swap), bit 3 s0 / s1 (row_mirror; s2 is
// summed on both sides), bit 2 t0 / t1 (row_half_mirror), then bits 1, 0 (quad_perm).  Afterwards
// lane l holds the wave total of value scatter_index(l); quads with bits 3 and 2 both set duplicate
// the quads with bit 3 clear (scatter_writer).
__device__ __forceinline__ float wave_reduce_scatter12(const float (&v)[12], int lane)
{
    const float r0 = swap32_add(v[0], v[6]), r1 = swap32_add(v[1], v[7]), r2 = swap32_add(v[2], v[8]);
    const float r3 = swap32_add(v[3], v[9]), r4 = swap32_add(v[4], v[10]), r5 = swap32_add(v[5], v[11]);
    const float s0 = swap16_add(r0, r3), s1 = swap16_add(r1, r4), s2 = swap16_add(r2, r5);
    const bool u8 = (lane & 8) != 0, u4 = (lane & 4) != 0;
    const float t0 = mirror_add<0x140>(s0, s1, u8);  // row_mirror
    const float t1 = s2 + dpp<0x140>(s2);
    float w = mirror_add<0x141>(t0, t1, u4);         // row_half_mirror
    w += dpp<0x4E>(w);                               // quad_perm [2,3,0,1]
    w += dpp<0xB1>(w);                               // quad_perm [1,0,3,2]
    asm volatile("" : "+v"(w));                      // see wave_reduce_scatter5
    return w;
}

__device__ __forceinline__ int scatter_index(int lane)
{
    const int m = (lane & 4) ? 2 : ((lane >> 3) & 1);
    return m + 3 * ((lane >> 4) & 1) + 6 * ((lane >> 5) & 1);
}

// One lane per distinct reduced value (12 of 64).
__device__ __forceinline__ bool scatter_writer(int lane)
{
    return (lane & 3) == 0 && (lane & 12) != 12;
}

// One pixel's back-to-front state (upstream BACKWARD::renderCUDA locals).  acc* is the colour /
// feature composited behind the current entry; upstream updates it at the start of the NEXT blend
// from (last_alpha, last_color) -- updating it at the end of this blend with (alpha, color) is the
// same expression on the same operands, one blend earlier, and needs no last_* registers.
struct BwdPixel {
    float T, T_final, bg_term;
    float dp0, dp1, dp2, dq0, dq1, dq2;
    float acc0, acc1, acc2, accF0, accF1, accF2;
    uint32_t last;
};

template <bool kFeat, bool kColor>
__device__ __forceinline__ void bwd_pixel_init(BwdPixel& q, const RenderParams& p, bool inside, size_t pix, size_t HW)
{
    q.T_final = inside ? p.final_T[pix] : 0.0f;
    q.T = q.T_final;
    q.last = inside ? p.n_contrib[pix] : 0u;
    q.dp0 = q.dp1 = q.dp2 = q.dq0 = q.dq1 = q.dq2 = 0.f;
    if (inside) {
        if (kColor) {
            q.dp0 = p.dL_dcolor[pix];
            q.dp1 = p.dL_dcolor[HW + pix];
            q.dp2 = p.dL_dcolor[2 * HW + pix];
        }
        if (kFeat && p.dL_dlang) {
            q.dq0 = p.dL_dlang[pix];
            q.dq1 = p.dL_dlang[HW + pix];
            q.dq2 = p.dL_dlang[2 * HW + pix];
        }
        if (kFeat && p.dL_dloss) {  // the fused loss: autograd's mean -> abs -> sub -> mul backward
            const uint32_t code = p.loss_code[pix];
            const float gN = p.dL_dloss[0] * (1.0f / (float)(3 * (int64_t)HW));
            const float m = (code & 64u) ? 1.0f : 0.0f;
            auto sg = [](uint32_t c) { return c == 1u ? 1.0f : (c == 2u ? -1.0f : 0.0f); };
            const float t0 = gN * sg(code & 3u) * m, t1 = gN * sg((code >> 2) & 3u) * m;
            const float t2 = gN * sg((code >> 4) & 3u) * m;
            q.dq0 = p.dL_dlang ? q.dq0 + t0 : t0;
            q.dq1 = p.dL_dlang ? q.dq1 + t1 : t1;
            q.dq2 = p.dL_dlang ? q.dq2 + t2 : t2;
        }
    }
    q.bg_term = kColor ? -q.T_final * fma_(p.bg[2], q.dp2, fma_(p.bg[1], q.dp1, p.bg[0] * q.dp0)) : 0.0f;
    q.acc0 = q.acc1 = q.acc2 = q.accF0 = q.accF1 = q.accF2 = 0.f;
}

// One replayed blend of one pixel: updates the pixel state and WRITES its 12 gradient partials to v
// (alpha and the skip tests are bit-identical to the forward; the gradient arithmetic is that of
// oracle backward_pixel, regrouped to fewer operations -- gradients need 1e-4, not bit-exactness).
// Branch-free: a lane without this blend passes alpha = G = 0, which leaves T and acc* unchanged
// (1 / (1 - 0) = 1, acc + 0 * (c - acc) = acc) and makes every partial 0 (each carries a factor
// alpha or G) -- so the wave needs no exec-mask split and no zero-fill of v.
// Constant factors are applied once per (tile, Gaussian) at the flush instead of per pixel
// (flush_scale): v[0] = dL/dmean2D.x / (2 ddelx_dx), v[1] likewise, v[2..4] = -2 dL/dconic.
// A = {x, y, -conic.x / 2, -conic.z / 2}, B = {conic.y, opacity, .., ..}, hB = -conic.y / 2.
template <bool kFeat, bool kColor, bool kGeo>
__device__ __forceinline__ void bwd_pixel_blend(BwdPixel& q, float G, float og, float alpha, float dx, float dy,
                                                const float4& A, const float4& B, const float3& C, const float3& F,
                                                float hB, float (&v)[12])
{
    const float one_m = 1.0f - alpha;
    // one v_rcp_f32 replaces the two IEEE divisions T / (1 - alpha) and T_final / (1 - alpha)
    const float inv_one_m = __builtin_amdgcn_rcpf(one_m);
    q.T = q.T * inv_one_m;
    const float dcd = alpha * q.T;
    // per channel: dL/dalpha += (c - acc) dL/dpix; acc <- acc + alpha (c - acc) (= alpha c + (1 - alpha) acc)
    float dL_dalpha = 0.0f;
    float e;
    if (kColor) {
        e = C.x - q.acc0;
        dL_dalpha = e * q.dp0;
        q.acc0 = fma_(alpha, e, q.acc0);
        v[6] = dcd * q.dp0;
        e = C.y - q.acc1;
        dL_dalpha = fma_(e, q.dp1, dL_dalpha);
        q.acc1 = fma_(alpha, e, q.acc1);
        v[7] = dcd * q.dp1;
        e = C.z - q.acc2;
        dL_dalpha = fma_(e, q.dp2, dL_dalpha);
        q.acc2 = fma_(alpha, e, q.acc2);
        v[8] = dcd * q.dp2;
    } else {  // the colour image does not reach the loss: its terms are exactly zero
        v[6] = v[7] = v[8] = 0.0f;
    }
    if (kFeat) {
        e = F.x - q.accF0;
        dL_dalpha = kColor ? fma_(e, q.dq0, dL_dalpha) : e * q.dq0;
        q.accF0 = fma_(alpha, e, q.accF0);
        v[9] = dcd * q.dq0;
        e = F.y - q.accF1;
        dL_dalpha = fma_(e, q.dq1, dL_dalpha);
        q.accF1 = fma_(alpha, e, q.accF1);
        v[10] = dcd * q.dq1;
        e = F.z - q.accF2;
        dL_dalpha = fma_(e, q.dq2, dL_dalpha);
        q.accF2 = fma_(alpha, e, q.accF2);
        v[11] = dcd * q.dq2;
    } else {
        v[9] = v[10] = v[11] = 0.0f;
    }
    // dL/dalpha = T (sum) - T_final / (1 - alpha) (bg . dL/dpix); bg_term = -T_final (bg . dL/dpix)
    dL_dalpha = kColor ? fma_(q.bg_term, inv_one_m, dL_dalpha * q.T) : dL_dalpha * q.T;
    if (kGeo) {
        const float dL_dG = B.y * dL_dalpha;  // conic and opacity partials: only the geometry gradients use them
        const float ga = (G * dx) * dL_dG, gb = (G * dy) * dL_dG;
        // dG/ddelx dL/dG = -(ga conic.x + gb conic.y) = 2 (ga A.z - gb conic.y / 2), likewise y
        v[0] = fma_(-0.5f, gb * B.x, ga * A.z);
        v[1] = fma_(-0.5f, ga * B.x, gb * A.w);
        v[2] = ga * dx;
        v[3] = ga * dy;
        v[4] = gb * dy;
        v[5] = G * dL_dalpha;
    } else {
        // the same two values factored as G dL/dG (A.z dx - conic.y dy / 2) and likewise y:
        // A.z dx, A.w dy and conic.y dx are the power's own products (shared by CSE).
        // G dL/dG = G o dL/dalpha with og = o G, the product the alpha was clamped from: one
        // multiply instead of two (dL/dG itself is not needed here)
        const float sG = og * dL_dalpha;
        v[0] = sG * fma_(hB, dy, A.z * dx);  // hB = -conic.y / 2
        v[1] = sG * fma_(-0.5f, B.x * dx, A.w * dy);
        v[2] = v[3] = v[4] = v[5] = 0.0f;
    }
}

// The language step's five values (no geometry, no colour gradient): v[0], v[1] (screen-space) and
// v[9..11] (language).  Reduce-scatter: lane bit 5 picks v0 / f0, v1 / f1, f2 / - (permlane32),
// bit 4 r0 / r1 (permlane16; r2 summed on both sides), bit 3 s0 / s1 (row_mirror), then bits 2..0.
// Lane l then holds the wave total of value scatter_index5(l); scatter_writer5 picks one lane each.
#ifndef LSR_BWD_DPP_DROP  // measurement knob: the last n (0..2) quad DPP steps left to the LDS atomics
#define LSR_BWD_DPP_DROP 0  // (2^n writer lanes per value, each adding a partial sum): backward 141 ->
#endif                      // 145 (n = 1) and 224 us (n = 2), same-address ds_add_f32 serialise
__device__ __forceinline__ float wave_reduce_scatter5(const float (&v)[12], int lane)
{
    const float r0 = swap32_add(v[0], v[9]), r1 = swap32_add(v[1], v[10]), r2 = swap32_add(v[11], 0.0f);
    const float s0 = swap16_add(r0, r1), s1 = swap16_add(r2, r2);
    float w = mirror_add<0x140>(s0, s1, (lane & 8) != 0);  // row_mirror
    w += dpp<0x141>(w);                                   // row_half_mirror
    if (LSR_BWD_DPP_DROP < 2) w += dpp<0x4E>(w);          // quad_perm [2,3,0,1]
    if (LSR_BWD_DPP_DROP < 1) w += dpp<0xB1>(w);          // quad_perm [1,0,3,2]
    // keep the last add next to its DPP move (one v_add_f32_dpp) instead of letting it sink into
    // the writers' branch as a separate v_mov_dpp + v_add
    asm volatile("" : "+v"(w));
    return w;
}

__device__ __forceinline__ int scatter_index5(int lane)
{
    const bool b3 = lane & 8, b4 = lane & 16, b5 = lane & 32;
    return b3 ? 11 : (b4 ? (b5 ? 10 : 1) : (b5 ? 9 : 0));
}

__device__ __forceinline__ bool scatter_writer5(int lane)
{
    constexpr int kPart = (1 << LSR_BWD_DPP_DROP) - 1;  // lanes of a quad holding partial sums
    return (lane & 7 & ~kPart) == 0 && (!(lane & 8) || (lane & 48) == 0);
}

// LDS slot of gradient value c: without the colour gradient values 6..8 are not stored; in the
// five-value form (no geometry, no colour) only 0, 1, 9, 10, 11.
template <bool kColor, bool k5>
__device__ __forceinline__ int gslot(int c)
{
    return k5 ? (c < 2 ? c : c - 7) : (kColor || c < 6 ? c : c - 3);
}

// Is gradient value c produced by this backward variant?
template <bool kColor, bool kGeo>
__device__ __forceinline__ bool gvalue(int c)
{
    return c < 2 || c >= 9 || (kGeo && c < 6) || (kColor && c >= 6);
}

// Factor of gradient slot c applied at the flush (see bwd_pixel_blend).
__device__ __forceinline__ float flush_scale(int c, int W, int H)
{
    return c == 0 ? (float)W : c == 1 ? (float)H : (c >= 2 && c <= 4) ? -0.5f : 1.0f;
}

// Measurement hook (LSR_RENDER_STATS=1, lsr_debug_render_stats): per wave-iteration counters of
// the backward -- [0] compacted entries, [1] entries passing the power test in some lane, [2] with
// an alpha hit, [3] lanes hit, [8 + c] histogram of lanes hit (c = 0..64).  Off by default.
__device__ unsigned long long g_render_stats[8 + 65];

// One list entry's staged record as the backward walk reads it from LDS.
struct BwdEntry {
    float4 A, B;  // {x, y, -conic.x / 2, -conic.z / 2}, {conic.y, opacity, power cutoff, f1 (kColor)}
    float4 C;     // kColor: {r, g, b, f0}
    float4 F;     // kColor: {f2, -, -, -}; k5: {f0, f1, f2, -conic.y / 2}; otherwise {f0, f2, -, -}
};

template <bool kFeat, bool kColor, bool kGeo>
__device__ __forceinline__ BwdEntry load_entry(const float4* sA, const float4* sB, const float4* sC, const float* sF,
                                               int j)
{
    BwdEntry e;
    e.A = sA[j];
    e.B = sB[j];
    e.C = make_float4(0.f, 0.f, 0.f, 0.f);
    e.F = make_float4(0.f, 0.f, 0.f, 0.f);
    if (kColor) {
        e.C = sC[j];
        if (kFeat) e.F.x = sF[j];
    } else if (!kGeo) {
        e.F = *reinterpret_cast<const float4*>(&sF[4 * j]);
    } else if (kFeat) {
        const float2 f = *reinterpret_cast<const float2*>(&sF[2 * j]);
        e.F = make_float4(f.x, f.y, 0.f, 0.f);
    }
    return e;
}

#ifndef LSR_BWD_F_EARLY  // 1: the language step's feature record read beside A and B (measurement knob)
#define LSR_BWD_F_EARLY 1
#endif
// One entry of a wave's back-to-front walk: the exact skip tests of the forward, the blend and the
// wave reduce-scatter of its partials into the tile sums (sG = this lane's value slot of entry 0,
// entry j at + j kGS).  kk = the entry's list index.
template <bool kStats, bool kFeat, bool kColor, bool kGeo, bool k5>
__device__ __forceinline__ void bwd_walk_entry(BwdPixel& q, const BwdEntry& E, int j, int kk, float pfx, float pfy,
                                               int lane, int vidx, float* sG, uint32_t* s_stat)
{
    constexpr int kGS = k5 ? 5 : (kColor ? 12 : 9);
    const float4& A = E.A;
    const float4& B = E.B;
    const float dx = A.x - pfx, dy = A.y - pfy;
    const float pw = fma_(dx, fma_(-B.x, dy, A.z * dx), (A.w * dy) * dy);  // the forward's order
    // the language step's feature record is read with A and B, not after the skip test below (the
    // compiler sinks it into the blend's block, a second LDS round trip on the visit's chain): the
    // empty asm takes it as an operand here, after the power, by when it has landed with A and B
    float4 Fv = E.F;
    if (k5 && LSR_BWD_F_EARLY) asm volatile("" : "+v"(Fv.x), "+v"(Fv.y), "+v"(Fv.z), "+v"(Fv.w));
    bool h = kk < (int)q.last && pw <= 0.0f && pw >= B.z;
    if (__ballot(h) == 0ull) return;  // wave-uniform skip
    // hardware exp (a few ulp): gradients need 1e-4.  Only the 1/255 skip decision must equal the
    // forward's, so alphas within 1e-6 of it use the exact exp: two compares bracket that band
    // (alpha = min(0.99, og) equals og = o G there), and the band's lanes take the exact exp.
    float G = __expf(pw);
    float og = B.y * G;
    bool hit = og >= 1.0f / 255.0f + 1e-6f;
    // two ballots of plain compares (a ballot of their combination is materialised per lane); in
    // the rare band branch every lane short of `hit` takes the exact exp (below the band it only
    // confirms the miss)
    if ((__ballot(og > 1.0f / 255.0f - 1e-6f) & ~__ballot(hit)) != 0ull) {  // wave-uniform
        if (!hit) {
            G = expf_exact_render(pw);  // the forward's exp (pw >= cutoff > -6 here)
            og = B.y * G;
            hit = og >= 1.0f / 255.0f;
        }
    }
    h = h && hit;
    if (kStats) {
        const int nh = __popcll(__ballot(h));
        if (lane == 0) {
            atomicAdd(&s_stat[1], 1u);
            if (nh) {
                atomicAdd(&s_stat[2], 1u);
                atomicAdd(&s_stat[3], (uint32_t)nh);
            }
            atomicAdd(&s_stat[8 + nh], 1u);
        }
    }
    og = h ? og : 0.0f;
    if (kGeo) G = h ? G : 0.0f;
    const float al = __builtin_amdgcn_fmed3f(og, 0.0f, 0.99f);  // min(0.99, og) (og >= 0), no canonicalise
    float3 C = make_float3(0.f, 0.f, 0.f), F = make_float3(0.f, 0.f, 0.f);
    if (kColor) {
        C = make_float3(E.C.x, E.C.y, E.C.z);
        if (kFeat) F = make_float3(E.C.w, B.w, E.F.x);
    } else if (kFeat) {
        F = kGeo ? make_float3(Fv.x, B.w, Fv.y) : make_float3(Fv.x, Fv.y, Fv.z);
    }
    float v[12];
    bwd_pixel_blend<kFeat, kColor, kGeo>(q, G, og, al, dx, dy, A, B, C, F, (kColor || kGeo) ? -0.5f * B.x : Fv.w,
                                         v);
    if (k5) {
        const float tot = wave_reduce_scatter5(v, lane);
        if (scatter_writer5(lane)) atomicAdd(sG + (uint32_t)(j * kGS), tot);  // sG: this lane's slot
    } else {
        const float tot = wave_reduce_scatter12(v, lane);
        if (scatter_writer(lane) && gvalue<kColor, kGeo>(vidx)) atomicAdd(sG + (uint32_t)(j * kGS), tot);
    }
}

#ifndef LSR_BWD_NOFLUSH  // measurement only: 1 drops the flush atomics (wrong gradients)
#define LSR_BWD_NOFLUSH 0
#endif
template <bool kStats, bool kFeat, bool kColor, bool kGeo>
__global__ __launch_bounds__(kTilePixels) void k_render_backward(RenderParams p)
{
    constexpr int kThreads = kTilePixels;
    __shared__ uint32_t s_stat[kStats ? 8 + 65 : 1];
    __shared__ uint32_t s_bmax;  // kStats: the batch's largest per-wave entry count
    __shared__ float4 sA[kThreads];      // x, y, -0.5 conic.x, -0.5 conic.z
    __shared__ float4 sB[kThreads];      // conic.y, opacity, power cutoff, f1
    // kColor: sC = {r, g, b, f0}, sF = {f2}; otherwise (the colour gradient is zero) only the language
    // feature is staged, sF = {f0, f2} (f1 in sB.w), and the tile sums hold 9 slots per entry (no colour
    // slots); the language step (k5) stages sF = {f0, f1, f2, -conic.y / 2}: one 16-B read, f0 / f1
    // adjacent for the packed subtract, the half conic.y of the screen-space gradient precomputed
    constexpr bool k5 = !kGeo && !kColor;  // the language step: five values per entry
    constexpr int kGS = k5 ? 5 : (kColor ? 12 : 9);
    __shared__ float4 sC[kColor ? kThreads : 1];
    __shared__ float4 sF4[k5 ? kThreads : 1];
    __shared__ float sF1[k5 ? 1 : (kColor ? kThreads : 2 * kThreads)];
    float* sF = k5 ? reinterpret_cast<float*>(sF4) : sF1;
    __shared__ float sG[kThreads * kGS];  // per-entry gradient sums of the tile
    __shared__ uint8_t sM[kThreads];     // wave_cover mask (& the waves' contributor bounds)
    __shared__ uint32_t s_wmax[kThreads / 64];
    __shared__ uint32_t s_gid[k5 ? kThreads : 1];  // the language step's flush: the batch's Gaussian ids

    const uint64_t t_start = kStats ? wall_clock64() : 0;
    // the forward's cleared records are used by this backward only (include/lsr.h): one store, no
    // reader in this launch
    if (p.fwd_flags && blockIdx.x == 0 && threadIdx.x == 0) *p.fwd_flags &= ~kFwdZeroedRecords;
    if (p.flag_dst && blockIdx.x == 0 && threadIdx.x == 0) *p.flag_dst = p.flag_src ? *p.flag_src : 0;
    int tile = (int)blockIdx.x;
    uint32_t chunk = 0;  // split replay: this workgroup replays list entries [kSplitChunk chunk, ...) of the tile
    if (p.sched_counts) {  // tiles without contributors are not scheduled: nothing to do
        const int T = p.gx * p.gy;
        const int item = scheduled_tile((int)blockIdx.x, p.sched_counts + kCntBwdClass,
                                        p.sched_lists + (size_t)kWorkClasses * T, kSplitItems * T);
        if (item < 0) return;
        const int it = __builtin_amdgcn_readfirstlane(item);  // uniform: scalar registers
        tile = it / kSplitItems;
        chunk = (uint32_t)(it % kSplitItems);
    }
    launch_priority((int)blockIdx.x, p.prio);
    const int tx = tile % p.gx, ty = tile / p.gx;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    int px, py;
    pixel_map(tx, ty, t, px, py);
    const float pfx = (float)px, pfy = (float)py;
    const size_t HW = (size_t)p.W * p.H;
    const uint32_t start = p.ranges[tile].x;

    BwdPixel q;
    bwd_pixel_init<kFeat, kColor>(q, p, px < p.W && py < p.H, (size_t)py * p.W + px, HW);
    // split replay: a chunk that ends at a recorded boundary hi = kSplitChunk (chunk + 1) starts the pixels
    // that composite past hi from the forward's state there (T and the normalised sums behind it);
    // pixels whose last contributor lies inside the chunk start from T_final as usual, and pixels
    // that end before it have nothing here (every entry >= their count is skipped)
    const uint32_t lo = chunk * (uint32_t)kSplitChunk;
    if (p.split_pool && p.sched_counts) {
        const uint4 desc = p.split_desc[tile];
        const uint32_t hi = lo + (uint32_t)kSplitChunk;
        if (chunk < desc.x && q.last > hi) {
            // the boundary's {T, feature sums}, {colour sums} and the tile's final sums (extra slot);
            // the colour halves exist unless the forward was told no colour gradient follows (a
            // colour variant is then refused by the host: include/lsr.h LSR_FWD_NO_COLOR_GRAD)
            const float4* st = reinterpret_cast<const float4*>(p.split_pool) + (size_t)tile * kSplitSlots * (2 * kThreads);
            const float4 s0 = st[chunk * 2 * kThreads + 2 * t], f0 = st[kSplitMax * 2 * kThreads + 2 * t];
            const float inv = 1.0f / s0.x;
            q.T = s0.x;
            if (kColor) {
                const float4 s1 = st[chunk * 2 * kThreads + 2 * t + 1];
                const float4 f1 = st[kSplitMax * 2 * kThreads + 2 * t + 1];
                q.acc0 = (f1.x - s1.x) * inv;
                q.acc1 = (f1.y - s1.y) * inv;
                q.acc2 = (f1.z - s1.z) * inv;
            }
            if (kFeat) {
                q.accF0 = (f0.x - s0.y) * inv;
                q.accF1 = (f0.y - s0.z) * inv;
                q.accF2 = (f0.z - s0.w) * inv;
            }
            q.last = hi;
        }
    }
    uint32_t wmax = q.last;

    if (kStats) {
        for (int i = t; i < 8 + 65; i += kThreads) s_stat[i] = 0;
        if (t == 0) s_bmax = 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o, 64));
    if (lane == 0) s_wmax[wave] = wmax;  // entries at list index >= this touch no pixel of the wave
    __syncthreads();
    const uint32_t w0 = s_wmax[0], w1 = s_wmax[1], w2 = s_wmax[2], w3 = s_wmax[3];
    // entries at list index >= max over the tile of n_contrib can contribute to no pixel
    const int maxl = (int)max(max(w0, w1), max(w2, w3));
    const int vidx = k5 ? scatter_index5(lane) : scatter_index(lane);
    float* const sGl = sG + gslot<kColor, k5>(vidx);  // this lane's value slot in the tile sums

    for (int done_cnt = 0; done_cnt < maxl - (int)lo; done_cnt += kThreads) {
        __syncthreads();
        const int kload = maxl - 1 - (done_cnt + t);
        uint32_t cover = 0;
        if (kload >= (int)lo) {
            const uint32_t g = p.point_list[start + (uint32_t)kload];
            if (k5) s_gid[t] = g;
            const float4 a = p.record[3 * (size_t)g];
            const float4 b = p.record[3 * (size_t)g + 1];
            const float4 c = p.record[3 * (size_t)g + 2];
            const float cut = power_cutoff(b.y);
            sA[t] = make_float4(a.x, a.y, -0.5f * a.z, -0.5f * b.x);
            sB[t] = make_float4(a.w, b.y, cut, c.z);
            if (kColor) {
                sC[t] = make_float4(b.z, b.w, c.x, c.y);
                sF[t] = c.w;
            } else if (k5) {
                sF4[t] = make_float4(c.y, c.z, c.w, -0.5f * a.w);
            } else {
                sF[2 * t] = c.y;
                sF[2 * t + 1] = c.w;
            }
            const uint32_t k = (uint32_t)kload;
            const uint32_t live = (k < w0 ? 1u : 0u) | (k < w1 ? 2u : 0u) | (k < w2 ? 4u : 0u) | (k < w3 ? 8u : 0u);
            // the forward's mask of this instance (it loaded every instance below any pixel's
            // contributor count): the same function of the same inputs, not recomputed
            cover = (uint32_t)p.cover[start + k] & live;
        }
        sM[t] = (uint8_t)cover;
        for (int i = t; i < kThreads * kGS; i += kThreads) sG[i] = 0.f;
        __syncthreads();
        const int cnt = min(kThreads, maxl - (int)lo - done_cnt);
        // the wave walks the set bits of a ballot over the cover masks (no list, no barrier)
        uint32_t nw = 0;  // kStats
        for (int r = 0; r < cnt; r += 64) {
            const int e = r + lane;
            uint64_t m = __ballot(e < cnt && ((sM[e] >> wave) & 1u));
            if (kStats) nw += (uint32_t)__popcll(m);
            if (kStats && lane == 0) atomicAdd(&s_stat[0], (uint32_t)__popcll(m));
            // (a one-entry LDS prefetch of the next set bit was measured: +8 VGPRs, one wave less
            // per SIMD, backward 0.185 -> 0.199 ms)
            while (m != 0ull) {
                const int j = r + (int)__builtin_ctzll(m);
                m &= m - 1ull;
                const BwdEntry cur = load_entry<kFeat, kColor, kGeo>(sA, sB, sC, sF, j);
                bwd_walk_entry<kStats, kFeat, kColor, kGeo, k5>(q, cur, j, maxl - 1 - (done_cnt + j), pfx, pfy, lane,
                                                                vidx, sGl, s_stat);
            }
        }
        if (kStats && lane == 0) atomicMax(&s_bmax, nw);
        __syncthreads();
        if (kStats && t == 0) {
            s_stat[4] += 4u * s_bmax;  // wave-entry slots the batch's barrier holds (4 x the busiest wave)
            s_stat[6] += 1u;           // batches
            s_bmax = 0u;
        }
        // flush: the batch's kGS x cnt tile sums on consecutive threads (every lane busy) -> one
        // atomic row per (tile, Gaussian).  The language step keeps the batch's ids in LDS (no
        // dependent global load before each atomic); the other variants, whose LDS is at the
        // occupancy limit, read them again from point_list (an L2 hit).
        for (int slot = t; slot < cnt * kGS; slot += kThreads) {
            const int e = slot / kGS, cs = slot - kGS * e;
            const float v = sG[slot];
            if (v == 0.0f || LSR_BWD_NOFLUSH) continue;
            if (k5) {  // packed 20-B record: dxy in slots 0, 1, the language feature in 2..4
                const float val = v * (cs == 0 ? (float)p.W : cs == 1 ? (float)p.H : 1.0f);
                const size_t g = s_gid[e];
                // (LSR_BWD_DEFER_TAIL: planar records, the language partials one all-reducible block)
                float* dst = !p.grad_xy ? p.grad + g * kGradStrideLang + cs
                                        : (cs < 2 ? p.grad_xy + 2 * g + cs : p.grad + 3 * g + (cs - 2));
                atomicAdd(dst, val);
            } else {
                const int c = (kColor || cs < 6) ? cs : cs + 3;  // gslot's inverse
                if (!gvalue<kColor, kGeo>(c)) continue;          // a value this variant does not produce
                const uint32_t g = p.point_list[start + (uint32_t)(maxl - 1 - (done_cnt + e))];
                atomicAdd(&p.grad[(size_t)g * kGradStride + c], v * flush_scale(c, p.W, p.H));
            }
        }
    }
    if (kStats) {
        __syncthreads();
        for (int i = t; i < 8 + 65; i += kThreads)
            if (s_stat[i]) atomicAdd(&g_render_stats[i], (unsigned long long)s_stat[i]);
        timeline_put(1, t_start, tile);
    }
}

hipError_t render_stats_read(unsigned long long* out, int n)
{
    if (n > 8 + 65) n = 8 + 65;
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_render_stats), sizeof(unsigned long long) * n, 0,
                                       hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    static const unsigned long long zeros[8 + 65] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_render_stats), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
}

hipError_t render_timeline_read(uint32_t* out, int kernel, int n)
{
    if (kernel < 0 || kernel > 1) return hipErrorInvalidValue;
    if (n > kTimelineMax) n = kTimelineMax;
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_render_timeline), sizeof(uint32_t) * kTimelineWords * n,
                                       sizeof(uint32_t) * kTimelineWords * kTimelineMax * kernel,
                                       hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    return hipSuccess;
}

// LSR_BWD_SHARED_CU: the dynamic LDS that caps a backward workgroup's CU at kSharedWgs workgroups
// (kSharedWgs x (static + pad) fits the CU's 160 KiB, one more does not), so that the pipelined
// step's other stream finds wave slots beside it.  Measured at C3 for the language-step variant
// (18704 B static; tools/pg_host.py with LSR_BWD_PAD, profiles/r05_occupancy_sweep.txt): 8 workgroups
// per CU (no pad) 0.417-0.421 ms per step; 7 with 18.6 KB of LDS left over (pad 2048) 0.406; 7 with
// 4.2 KB left (pad 4096) 0.400-0.401; 6 (pad 5120) 0.478; 5 (pad 8192) 0.416.  So the pad is the
// largest that still fits 7.  LSR_BWD_SHARE=0 disables it (LSR_BWD_PAD then applies).
template <int V>
static size_t shared_pad_of()
{
    return occupancy_pad((const void*)k_render_backward<false, (V & 1) != 0, (V & 2) != 0, (V & 4) != 0>, kSharedWgsBwd,
                         "backward");
}

static size_t shared_cu_pad(int variant)
{
    static const bool on = [] {
        const char* e = getenv("LSR_BWD_SHARE");
        return !(e && e[0] == '0');
    }();
    if (!on) return backward_pad();
    // variant bits (launch_render_backward): 1 feature, 2 colour, 4 geometry
    static const size_t pad[8] = {shared_pad_of<0>(), shared_pad_of<1>(), shared_pad_of<2>(), shared_pad_of<3>(),
                                  shared_pad_of<4>(), shared_pad_of<5>(), shared_pad_of<6>(), shared_pad_of<7>()};
    return pad[variant & 7];
}

hipError_t launch_render_backward(const RenderParams& pin, int tiles, hipStream_t s)
{
    if (tiles == 0) return hipSuccess;
    RenderParams p = pin;
    if (!scheduled()) p.sched_counts = p.sched_lists = nullptr;
    p.prio = p.sched_counts ? prio_levels() : 0;
    const bool feat = p.include_feature != 0;
    const bool color = p.dL_dcolor != nullptr;  // null: the colour image does not reach the loss
    const int variant = (feat ? 1 : 0) | (color ? 2 : 0) | (p.geo ? 4 : 0);
    if (!p.sched_counts || !split_replay()) p.split_pool = nullptr;
    if (p.split_pool) tiles *= kSplitItems;  // the items: up to kSplitItems chunks per tile
    if (render_stats_on()) tiles = debug_grid(tiles);
    const size_t pad = p.shared_cu && !render_stats_on() ? shared_cu_pad(variant) : backward_pad();
#define LSR_BWD(S, V)                                                                                         \
    hipLaunchKernelGGL((k_render_backward<S, (V & 1) != 0, (V & 2) != 0, (V & 4) != 0>), dim3(tiles), \
                       dim3(kTilePixels), pad, s, p)
#define LSR_BWD_ALL(S)            \
    switch (variant) {            \
    case 0: LSR_BWD(S, 0); break; \
    case 1: LSR_BWD(S, 1); break; \
    case 2: LSR_BWD(S, 2); break; \
    case 3: LSR_BWD(S, 3); break; \
    case 4: LSR_BWD(S, 4); break; \
    case 5: LSR_BWD(S, 5); break; \
    case 6: LSR_BWD(S, 6); break; \
    default: LSR_BWD(S, 7); break; \
    }
    if (render_stats_on()) {
        LSR_BWD_ALL(true)
    } else {
        LSR_BWD_ALL(false)
    }
#undef LSR_BWD_ALL
#undef LSR_BWD
    return hipGetLastError();
}

}  // namespace lsr
