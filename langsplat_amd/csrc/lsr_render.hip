// lsr_render.hip -- per-tile compositing (forward) and its back-to-front replay (backward).
//
// Backward: one 128-thread workgroup per 16x16 screen tile = 2 wave64s; every lane owns TWO
// vertically adjacent pixels, so each list entry read from LDS feeds two independent dependency
// chains (ILP) and the per-entry fixed costs (LDS reads, loop control, the wave reduction) are
// paid once per two pixels.  Forward: templated on pixels per lane (1 = 256 threads).  The tile's depth-ordered list is streamed through LDS in batches of 128
// entries (48 B records split into broadcast-friendly {x, y, -conic.x/2, -conic.z/2}
// {conic.y, opacity, power cutoff}{r, g, b, f0}{f1, f2} arrays).  Semantics: upstream FORWARD/BACKWARD::renderCUDA extended by
// the 3-channel language feature; arithmetic order is
// that of oracle/lsr_oracle.c render_pixel / backward_pixel.
//
// Backward gradient scatter: every lane of a wave visits the same list entry at the same
// iteration, so the 12 per-Gaussian partials of a wave are reduced in registers by a
// reduce-scatter (permlane32/16 swaps + DPP mirrors, ~35 VALU ops), the 2 waves' results are summed
// in LDS (ds_add_f32), and after each batch ONE 12-lane atomic instruction per (tile, Gaussian)
// adds the tile's total into a 64-byte-aligned per-Gaussian record -- instead of the upstream 12
// scattered atomics per pixel per blend.  Entries no lane contributes to are skipped by a ballot.
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
    const float ex = sqrtf(k * cz / detq) * 1.001f + 0.05f;
    const float ey = sqrtf(k * cx / detq) * 1.001f + 0.05f;
    return make_float4(x - ex, x + ex, y - ey, y + ey);
}

__device__ __forceinline__ uint64_t lanemask_lt64(int lane)
{
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Compacts the batch slots [0, cnt) whose box overlaps the wave's pixel rectangle (and, for the
// backward, whose list index is below the wave's contributor bound) into list[0, n); returns n.
template <typename Keep>
__device__ __forceinline__ int wave_compact(const float4* sE, int cnt, float wx0, float wx1, float wy0, float wy1,
                                            int lane, uint16_t* list, Keep keep)
{
    int n = 0;
    for (int r = 0; r < cnt; r += 64) {
        const int e = r + lane;
        bool ov = false;
        if (e < cnt && keep(e)) {
            const float4 E = sE[e];
            ov = E.y >= wx0 && E.x <= wx1 && E.w >= wy0 && E.z <= wy1;
        }
        const uint64_t m = __ballot(ov);
        if (ov) list[n + __popcll(m & lanemask_lt64(lane))] = (uint16_t)e;
        n += __popcll(m);
    }
    return n;
}


// Pixel ownership.  kPix = 1: wave w of the tile's 4 owns the 8 x 8 pixel block
// (8 (w & 1), 8 (w >> 1)) -- a compact block meets fewer reach boxes than a 16 x 4 strip.
// kPix = 2: lane l owns the vertically adjacent pixels (l % 16, 2 (l / 16) + k) and a wave a
// 16 x 8 strip.  (wx0, wx1, wy0, wy1) is the wave's pixel rectangle, for culling.
template <int kPix>
__device__ __forceinline__ void pixel_map(int tx, int ty, int t, int& px, int& py_base, float& wx0, float& wx1,
                                          float& wy0, float& wy1)
{
    const int lane = t & 63, wave = t >> 6;
    if (kPix == 1) {
        const int bx = tx * kTile + 8 * (wave & 1), by = ty * kTile + 8 * (wave >> 1);
        px = bx + (lane & 7);
        py_base = by + (lane >> 3);
        wx0 = (float)bx;
        wx1 = wx0 + 7.0f;
        wy0 = (float)by;
        wy1 = wy0 + 7.0f;
    } else {
        px = tx * kTile + (t & (kTile - 1));
        py_base = ty * kTile + kPix * (t >> 4);
        wx0 = (float)(tx * kTile);
        wx1 = wx0 + (float)(kTile - 1);
        wy0 = (float)(ty * kTile + 4 * kPix * wave);
        wy1 = wy0 + (float)(4 * kPix - 1);
    }
}

// One pixel's front-to-back state (upstream FORWARD::renderCUDA locals).
struct FwdPixel {
    float T, C0, C1, C2, F0, F1, F2;
    uint32_t contributor, last;
    bool done;
};

// kPix pixels per lane (pixel_map).
template <int kPix>
__global__ __launch_bounds__(kTilePixels / kPix) void k_render_forward(RenderParams p)
{
    constexpr int kThreads = kTilePixels / kPix;
    constexpr int kWaves = kThreads / 64;
    __shared__ float4 sA[kThreads];  // x, y, -0.5 conic.x, -0.5 conic.z
    __shared__ float4 sB[kThreads];  // conic.y, opacity, power cutoff, -
    __shared__ float4 sC[kThreads];  // r, g, b, f0
    __shared__ float2 sD[kThreads];  // f1, f2
    __shared__ float4 sE[kThreads];  // reach box (entry_box)
    __shared__ uint16_t sL[kWaves][kThreads];  // per-wave culled slot lists

    const int tile = blockIdx.x;
    const int tx = tile % p.gx, ty = tile / p.gx;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    int px, py_base;
    float wx0, wx1, wy0, wy1;
    pixel_map<kPix>(tx, ty, t, px, py_base, wx0, wx1, wy0, wy1);
    const float pfx = (float)px;
    const uint2 range = p.ranges[tile];
    const uint32_t start = range.x, end = range.y;
    const bool feat = p.include_feature != 0;

    FwdPixel q[kPix];
#pragma unroll
    for (int k = 0; k < kPix; k++)
        q[k] = FwdPixel{1.0f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0u, 0u, !(px < p.W && py_base + k < p.H)};

    for (uint32_t base = start; base < end; base += kThreads) {
        bool all_done = true;
#pragma unroll
        for (int k = 0; k < kPix; k++) all_done = all_done && q[k].done;
        if (__syncthreads_count(all_done) == kThreads) break;
        const uint32_t idx = base + t;
        if (idx < end) {
            const uint32_t g = p.point_list[idx];
            const float4 a = p.record[3 * (size_t)g];
            const float4 b = p.record[3 * (size_t)g + 1];
            const float4 c = p.record[3 * (size_t)g + 2];
            const float cut = power_cutoff(b.y);
            sA[t] = make_float4(a.x, a.y, -0.5f * a.z, -0.5f * b.x);
            sB[t] = make_float4(a.w, b.y, cut, 0.0f);
            sC[t] = make_float4(b.z, b.w, c.x, c.y);
            sD[t] = make_float2(c.z, c.w);
            sE[t] = entry_box(a.x, a.y, a.z, a.w, b.x, cut);
        }
        __syncthreads();
        const int cnt = (int)min((uint32_t)kThreads, end - base);
        const int n = wave_compact(sE, cnt, wx0, wx1, wy0, wy1, lane, sL[wave], [](int) { return true; });
        __syncthreads();  // list visible to the wave's other lanes
        const uint32_t list_base = base - start;  // list index of slot 0
        for (int i = 0; i < n && !all_done; i++) {
            const int j = sL[wave][i];
            const float4 A = sA[j];
            const float4 B = sB[j];
            const uint32_t contributor = list_base + (uint32_t)j + 1u;  // upstream's 1-based counter
            const float dx = A.x - pfx;
            float pw[kPix], al[kPix];
            bool ok[kPix];
            bool any = false;
#pragma unroll
            for (int k = 0; k < kPix; k++) {
                const float dy = A.y - (float)(py_base + k);
                pw[k] = fma_(A.z * dx, dx, fma_(A.w * dy, dy, -((B.x * dx) * dy)));
                ok[k] = !q[k].done && !(pw[k] > 0.0f || pw[k] < B.z);
                any = any || ok[k];
            }
            if (!any) continue;
            any = false;
#pragma unroll
            for (int k = 0; k < kPix; k++) {
                al[k] = fminf(0.99f, B.y * expf_exact(pw[k]));
                ok[k] = ok[k] && !(al[k] < 1.0f / 255.0f);
                const float test_T = q[k].T * (1.0f - al[k]);
                if (ok[k] && test_T < 0.0001f) {
                    q[k].done = true;
                    ok[k] = false;
                }
                pw[k] = test_T;  // reuse: the candidate transmittance
                any = any || ok[k];
            }
            if (any) {
                const float4 Cc = sC[j];
                const float2 D = sD[j];
#pragma unroll
                for (int k = 0; k < kPix; k++) {
                    if (!ok[k]) continue;
                    const float w = al[k] * q[k].T;
                    q[k].C0 = fma_(Cc.x, w, q[k].C0);
                    q[k].C1 = fma_(Cc.y, w, q[k].C1);
                    q[k].C2 = fma_(Cc.z, w, q[k].C2);
                    if (feat) {
                        q[k].F0 = fma_(Cc.w, w, q[k].F0);
                        q[k].F1 = fma_(D.x, w, q[k].F1);
                        q[k].F2 = fma_(D.y, w, q[k].F2);
                    }
                    q[k].T = pw[k];
                    q[k].last = contributor;
                }
            }
            all_done = true;
#pragma unroll
            for (int k = 0; k < kPix; k++) all_done = all_done && q[k].done;
        }
    }
    const size_t HW = (size_t)p.W * p.H;
#pragma unroll
    for (int k = 0; k < kPix; k++) {
        const int py = py_base + k;
        if (!(px < p.W && py < p.H)) continue;
        const size_t pix = (size_t)py * p.W + px;
        p.final_T[pix] = q[k].T;
        p.n_contrib[pix] = q[k].last;
        p.out_color[pix] = fma_(q[k].T, p.bg[0], q[k].C0);
        p.out_color[HW + pix] = fma_(q[k].T, p.bg[1], q[k].C1);
        p.out_color[2 * HW + pix] = fma_(q[k].T, p.bg[2], q[k].C2);
        p.out_lang[pix] = q[k].F0;
        p.out_lang[HW + pix] = q[k].F1;
        p.out_lang[2 * HW + pix] = q[k].F2;
    }
}

// LSR_FWD_PIXELS=1|2 selects the forward variant (measurement aid; default 1)
static int fwd_pixels_per_lane()
{
    static int v = [] {
        const char* e = getenv("LSR_FWD_PIXELS");
        return (e && e[0] == '2') ? 2 : 1;
    }();
    return v;
}

hipError_t launch_render_forward(const RenderParams& p, int tiles, hipStream_t s)
{
    if (tiles == 0) return hipSuccess;
    const int pix = fwd_pixels_per_lane();
    if (pix == 2)
        hipLaunchKernelGGL(k_render_forward<2>, dim3(tiles), dim3(kTilePixels / 2), 0, s, p);
    else
        hipLaunchKernelGGL(k_render_forward<1>, dim3(tiles), dim3(kTilePixels), 0, s, p);
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

// Reduce-scatter of 12 per-lane values (slots 12..15 implicit zeros) over the wave: afterwards
// lane l holds the wave total of value index bitrev(l>>2) (4 consecutive lanes hold the same one).
__device__ __forceinline__ float wave_reduce_scatter12(const float (&v)[12], int lane)
{
    const float r0 = swap32_add(v[0], v[8]), r1 = swap32_add(v[1], v[9]);
    const float r2 = swap32_add(v[2], v[10]), r3 = swap32_add(v[3], v[11]);
    const float r4 = swap32_add(v[4], 0.0f), r5 = swap32_add(v[5], 0.0f);
    const float r6 = swap32_add(v[6], 0.0f), r7 = swap32_add(v[7], 0.0f);
    const float s0 = swap16_add(r0, r4), s1 = swap16_add(r1, r5);
    const float s2 = swap16_add(r2, r6), s3 = swap16_add(r3, r7);
    const bool u8 = (lane & 8) != 0, u4 = (lane & 4) != 0;
    const float t0 = mirror_add<0x140>(s0, s2, u8);  // row_mirror
    const float t1 = mirror_add<0x140>(s1, s3, u8);
    float w = mirror_add<0x141>(t0, t1, u4);         // row_half_mirror
    w += dpp<0x4E>(w);                               // quad_perm [2,3,0,1]
    w += dpp<0xB1>(w);                               // quad_perm [1,0,3,2]
    return w;
}

__device__ __forceinline__ int scatter_index(int lane)
{
    // bits 5,4,3,2 of the lane select value bits 3,2,1,0
    return (((lane >> 5) & 1) << 3) | (((lane >> 4) & 1) << 2) | (((lane >> 3) & 1) << 1) | ((lane >> 2) & 1);
}

// One pixel's back-to-front state (upstream BACKWARD::renderCUDA locals).
struct BwdPixel {
    float T, T_final, bg_dot;
    float dp0, dp1, dp2, dq0, dq1, dq2;
    float acc0, acc1, acc2, accF0, accF1, accF2;
    float lc0, lc1, lc2, lf0, lf1, lf2;
    float last_alpha;
    uint32_t last;
};

__device__ __forceinline__ void bwd_pixel_init(BwdPixel& q, const RenderParams& p, bool inside, size_t pix,
                                               size_t HW, bool feat)
{
    q.T_final = inside ? p.final_T[pix] : 0.0f;
    q.T = q.T_final;
    q.last = inside ? p.n_contrib[pix] : 0u;
    q.dp0 = q.dp1 = q.dp2 = q.dq0 = q.dq1 = q.dq2 = 0.f;
    if (inside) {
        if (p.dL_dcolor) {  // null: the colour image does not reach the loss (zero gradient)
            q.dp0 = p.dL_dcolor[pix];
            q.dp1 = p.dL_dcolor[HW + pix];
            q.dp2 = p.dL_dcolor[2 * HW + pix];
        }
        if (feat && p.dL_dlang) {
            q.dq0 = p.dL_dlang[pix];
            q.dq1 = p.dL_dlang[HW + pix];
            q.dq2 = p.dL_dlang[2 * HW + pix];
        }
    }
    q.bg_dot = fma_(p.bg[2], q.dp2, fma_(p.bg[1], q.dp1, p.bg[0] * q.dp0));
    q.acc0 = q.acc1 = q.acc2 = q.accF0 = q.accF1 = q.accF2 = 0.f;
    q.lc0 = q.lc1 = q.lc2 = q.lf0 = q.lf1 = q.lf2 = 0.f;
    q.last_alpha = 0.f;
}

// One replayed blend of one pixel: updates the pixel state and ADDS its 12 gradient partials to v
// (order of oracle backward_pixel; alpha and the skip tests are bit-identical to the forward).
__device__ __forceinline__ void bwd_pixel_blend(BwdPixel& q, float G, float alpha, float dx, float dy,
                                                const float4& B, float cx, float cz, const float4& Cc,
                                                const float2& D, bool feat, float ddelx_dx, float ddely_dy,
                                                float (&v)[12])
{
    const float one_m = 1.0f - alpha;
    // gradients need 1e-4, not bit-exactness: one v_rcp_f32 replaces the two IEEE divisions
    // T / (1 - alpha) and T_final / (1 - alpha) (the skip decisions use power/alpha only)
    const float inv_one_m = __builtin_amdgcn_rcpf(one_m);
    q.T = q.T * inv_one_m;
    const float dcd = alpha * q.T;
    const float oml = 1.0f - q.last_alpha;
    float dL_dalpha = 0.0f;
    q.acc0 = fma_(q.last_alpha, q.lc0, oml * q.acc0);
    q.lc0 = Cc.x;
    dL_dalpha = fma_(Cc.x - q.acc0, q.dp0, dL_dalpha);
    v[6] += dcd * q.dp0;
    q.acc1 = fma_(q.last_alpha, q.lc1, oml * q.acc1);
    q.lc1 = Cc.y;
    dL_dalpha = fma_(Cc.y - q.acc1, q.dp1, dL_dalpha);
    v[7] += dcd * q.dp1;
    q.acc2 = fma_(q.last_alpha, q.lc2, oml * q.acc2);
    q.lc2 = Cc.z;
    dL_dalpha = fma_(Cc.z - q.acc2, q.dp2, dL_dalpha);
    v[8] += dcd * q.dp2;
    if (feat) {
        q.accF0 = fma_(q.last_alpha, q.lf0, oml * q.accF0);
        q.lf0 = Cc.w;
        dL_dalpha = fma_(Cc.w - q.accF0, q.dq0, dL_dalpha);
        v[9] += dcd * q.dq0;
        q.accF1 = fma_(q.last_alpha, q.lf1, oml * q.accF1);
        q.lf1 = D.x;
        dL_dalpha = fma_(D.x - q.accF1, q.dq1, dL_dalpha);
        v[10] += dcd * q.dq1;
        q.accF2 = fma_(q.last_alpha, q.lf2, oml * q.accF2);
        q.lf2 = D.y;
        dL_dalpha = fma_(D.y - q.accF2, q.dq2, dL_dalpha);
        v[11] += dcd * q.dq2;
    }
    dL_dalpha = dL_dalpha * q.T;
    q.last_alpha = alpha;
    dL_dalpha = fma_(-q.T_final * inv_one_m, q.bg_dot, dL_dalpha);
    const float cy = B.x;
    const float dL_dG = B.y * dL_dalpha;
    const float gdx = G * dx, gdy = G * dy;
    const float dG_ddelx = -gdx * cx - gdy * cy;
    const float dG_ddely = -gdy * cz - gdx * cy;
    v[0] += dL_dG * dG_ddelx * ddelx_dx;
    v[1] += dL_dG * dG_ddely * ddely_dy;
    v[2] += -0.5f * gdx * dx * dL_dG;
    v[3] += -0.5f * gdx * dy * dL_dG;
    v[4] += -0.5f * gdy * dy * dL_dG;
    v[5] += G * dL_dalpha;
}

// Measurement hook (LSR_RENDER_STATS=1, lsr_debug_render_stats): per wave-iteration counters of
// the backward -- [0] compacted entries, [1] entries passing the power test in some lane, [2] with
// an alpha hit, [3] lanes hit, [8 + c] histogram of lanes hit (c = 0..64).  Off by default.
__device__ unsigned long long g_render_stats[8 + 65];

template <int kPix, bool kStats = false>
__global__ __launch_bounds__(kTilePixels / kPix) void k_render_backward(RenderParams p)
{
    constexpr int kThreads = kTilePixels / kPix;
    __shared__ uint32_t s_stat[kStats ? 8 + 65 : 1];
    __shared__ float4 sA[kThreads];  // x, y, -0.5 conic.x, -0.5 conic.z
    __shared__ float4 sB[kThreads];  // conic.y, opacity, power cutoff, -
    __shared__ float4 sC[kThreads];  // r, g, b, f0
    __shared__ float2 sD[kThreads];  // f1, f2
    __shared__ uint32_t sId[kThreads];
    __shared__ float sG[kThreads * 12];  // per-entry gradient sums of the tile (12 floats)
    __shared__ float4 sE[kThreads];      // reach box (entry_box)
    __shared__ uint16_t sL[kThreads / 64][kThreads];  // per-wave culled slot lists
    __shared__ uint32_t s_max;

    const int tile = blockIdx.x;
    const int tx = tile % p.gx, ty = tile / p.gx;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    int px, py_base;
    float wx0, wx1, wy0, wy1;
    pixel_map<kPix>(tx, ty, t, px, py_base, wx0, wx1, wy0, wy1);
    const float pfx = (float)px;
    const size_t HW = (size_t)p.W * p.H;
    const uint32_t start = p.ranges[tile].x;
    const bool feat = p.include_feature != 0;
    const float ddelx_dx = 0.5f * (float)p.W, ddely_dy = 0.5f * (float)p.H;

    BwdPixel q[kPix];
    uint32_t wmax = 0;
#pragma unroll
    for (int k = 0; k < kPix; k++) {
        const int py = py_base + k;
        bwd_pixel_init(q[k], p, px < p.W && py < p.H, (size_t)py * p.W + px, HW, feat);
        wmax = max(wmax, q[k].last);
    }

    if (kStats)
        for (int i = t; i < 8 + 65; i += kThreads) s_stat[i] = 0;
    // entries at list index >= max over the tile of n_contrib can contribute to no pixel
    if (t == 0) s_max = 0;
    __syncthreads();
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o, 64));
    if (lane == 0) atomicMax(&s_max, wmax);
    __syncthreads();
    const int maxl = (int)s_max;
    const int wave_max = (int)wmax;  // entries at index >= this touch no pixel of this wave
    const int vidx = scatter_index(lane);

    for (int done_cnt = 0; done_cnt < maxl; done_cnt += kThreads) {
        __syncthreads();
        const int kload = maxl - 1 - (done_cnt + t);
        if (kload >= 0) {
            const uint32_t g = p.point_list[start + (uint32_t)kload];
            const float4 a = p.record[3 * (size_t)g];
            const float4 b = p.record[3 * (size_t)g + 1];
            const float4 c = p.record[3 * (size_t)g + 2];
            const float cut = power_cutoff(b.y);
            sA[t] = make_float4(a.x, a.y, -0.5f * a.z, -0.5f * b.x);
            sB[t] = make_float4(a.w, b.y, cut, 0.0f);
            sC[t] = make_float4(b.z, b.w, c.x, c.y);
            sD[t] = make_float2(c.z, c.w);
            sE[t] = entry_box(a.x, a.y, a.z, a.w, b.x, cut);
            sId[t] = g;
        }
        for (int i = t; i < kThreads * 12; i += kThreads) sG[i] = 0.f;
        __syncthreads();
        const int cnt = min(kThreads, maxl - done_cnt);
        // entries at list index >= wave_max touch no pixel of this wave
        const int n = wave_compact(sE, cnt, wx0, wx1, wy0, wy1, lane, sL[wave],
                                   [&](int e) { return maxl - 1 - (done_cnt + e) < wave_max; });
        __syncthreads();  // list visible to the wave's other lanes
        if (kStats && lane == 0) atomicAdd(&s_stat[0], (uint32_t)n);
        for (int i = 0; i < n; i++) {
            const int j = sL[wave][i];
            const float4 A = sA[j];
            const float4 B = sB[j];
            const int kk = maxl - 1 - (done_cnt + j);  // list index of this entry
            const float dx = A.x - pfx;
            float pw[kPix];
            bool h[kPix];
            bool any = false;
#pragma unroll
            for (int k = 0; k < kPix; k++) {
                const float dy = A.y - (float)(py_base + k);
                pw[k] = fma_(A.z * dx, dx, fma_(A.w * dy, dy, -((B.x * dx) * dy)));
                h[k] = kk < (int)q[k].last && pw[k] <= 0.0f && pw[k] >= B.z;
                any = any || h[k];
            }
            if (__ballot(any) != 0ull) {  // wave-uniform skip otherwise
                float v[12];
#pragma unroll
                for (int c = 0; c < 12; c++) v[c] = 0.f;
                float G[kPix], al[kPix];
                bool hit = false;
#pragma unroll
                for (int k = 0; k < kPix; k++) {
                    // hardware exp (a few ulp): gradients need 1e-4.  Only the 1/255 skip decision
                    // must equal the forward's, so alphas within 1e-6 of it use the exact exp.
                    G[k] = __expf(pw[k]);
                    al[k] = fminf(0.99f, B.y * G[k]);
                    const bool near = fabsf(al[k] - 1.0f / 255.0f) < 1e-6f;
                    if (__ballot(near) != 0ull) {  // wave-uniform: keeps the exact exp off the hot path
                        if (near) {
                            G[k] = expf_exact(pw[k]);
                            al[k] = fminf(0.99f, B.y * G[k]);
                        }
                    }
                    h[k] = h[k] && al[k] >= 1.0f / 255.0f;
                    hit = hit || h[k];
                }
                if (kStats) {
                    const int nh = __popcll(__ballot(hit));
                    if (lane == 0) {
                        atomicAdd(&s_stat[1], 1u);
                        if (nh) {
                            atomicAdd(&s_stat[2], 1u);
                            atomicAdd(&s_stat[3], (uint32_t)nh);
                        }
                        atomicAdd(&s_stat[8 + nh], 1u);
                    }
                }
                if (hit) {
                    const float4 Cc = sC[j];
                    const float2 D = sD[j];
                    const float cx = -2.0f * A.z, cz = -2.0f * A.w;
#pragma unroll
                    for (int k = 0; k < kPix; k++)
                        if (h[k])
                            bwd_pixel_blend(q[k], G[k], al[k], dx, A.y - (float)(py_base + k), B, cx, cz, Cc, D,
                                            feat, ddelx_dx, ddely_dy, v);
                }
                const float tot = wave_reduce_scatter12(v, lane);
                if ((lane & 3) == 0 && vidx < 12) atomicAdd(&sG[j * 12 + vidx], tot);
            }
        }
        __syncthreads();
        // flush: 16 lanes per entry (12 active) -> one 48-byte atomic row per (tile, Gaussian)
        for (int slot = t; slot < cnt * 16; slot += kThreads) {
            const int e = slot >> 4, c = slot & 15;
            if (c < 12) {
                const float val = sG[e * 12 + c];
                if (val != 0.0f) atomicAdd(&p.grad[(size_t)sId[e] * kGradStride + c], val);
            }
        }
    }
    if (kStats) {
        __syncthreads();
        for (int i = t; i < 8 + 65; i += kThreads)
            if (s_stat[i]) atomicAdd(&g_render_stats[i], (unsigned long long)s_stat[i]);
    }
}

static bool render_stats_on()
{
    static bool v = [] {
        const char* e = getenv("LSR_RENDER_STATS");
        return e && e[0] == '1';
    }();
    return v;
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

// LSR_BWD_PIXELS=1|2 selects the backward variant (measurement aid; default 1: 0.52 vs 0.58 ms at
// C3 -- with ~2300 busy tiles the chip is short of waves, so more waves per tile beat more ILP)
static int bwd_pixels_per_lane()
{
    static int v = [] {
        const char* e = getenv("LSR_BWD_PIXELS");
        return (e && e[0] == '2') ? 2 : 1;
    }();
    return v;
}

hipError_t launch_render_backward(const RenderParams& p, int tiles, hipStream_t s)
{
    if (tiles == 0) return hipSuccess;
    if (render_stats_on())
        hipLaunchKernelGGL((k_render_backward<1, true>), dim3(tiles), dim3(kTilePixels), 0, s, p);
    else if (bwd_pixels_per_lane() == 1)
        hipLaunchKernelGGL(k_render_backward<1>, dim3(tiles), dim3(kTilePixels), 0, s, p);
    else
        hipLaunchKernelGGL(k_render_backward<2>, dim3(tiles), dim3(kTilePixels / 2), 0, s, p);
    return hipGetLastError();
}

}  // namespace lsr
