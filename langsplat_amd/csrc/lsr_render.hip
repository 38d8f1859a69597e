// lsr_render.hip -- per-tile compositing (forward) and its back-to-front replay (backward).
//
// One 256-thread workgroup per 16x16 screen tile = 4 wave64s, each wave owning 16x4 pixels.
// The tile's depth-ordered list is streamed through LDS in batches of 256 Gaussians (48 B
// records split into broadcast-friendly {x, y, -conic.x/2, -conic.z/2}{conic.y, opacity}
// {r, g, b, f0}{f1, f2} arrays).  Semantics: upstream FORWARD/BACKWARD::renderCUDA extended by
// the 3-channel language feature; arithmetic order is
// that of oracle/lsr_oracle.c render_pixel / backward_pixel.
//
// Backward gradient scatter: every lane of a wave visits the same list entry at the same
// iteration, so the 12 per-Gaussian partials of a wave are reduced in registers by a
// reduce-scatter (permlane32/16 swaps + DPP mirrors, ~35 VALU ops), the 4 waves' results are summed
// in LDS (ds_add_f32), and after each batch ONE 12-lane atomic instruction per (tile, Gaussian)
// adds the tile's total into a 64-byte-aligned per-Gaussian record -- instead of the upstream 12
// scattered atomics per pixel per blend.  Entries no lane contributes to are skipped by a ballot.
#include "lsr_internal.h"

namespace lsr {

__global__ __launch_bounds__(kTilePixels) void k_render_forward(RenderParams p)
{
    __shared__ float4 sA[kTilePixels];  // x, y, -0.5 conic.x, -0.5 conic.z
    __shared__ float2 sB[kTilePixels];  // conic.y, opacity
    __shared__ float4 sC[kTilePixels];  // r, g, b, f0
    __shared__ float2 sD[kTilePixels];  // f1, f2

    const int tile = blockIdx.x;
    const int tx = tile % p.gx, ty = tile / p.gx;
    const int t = threadIdx.x;
    const int px = tx * kTile + (t & (kTile - 1)), py = ty * kTile + (t >> 4);
    const bool inside = px < p.W && py < p.H;
    const float pfx = (float)px, pfy = (float)py;
    const uint2 range = p.ranges[tile];
    const uint32_t start = range.x, end = range.y;
    const bool feat = p.include_feature != 0;

    float T = 1.0f;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f, F0 = 0.f, F1 = 0.f, F2 = 0.f;
    uint32_t contributor = 0, last = 0;
    bool done = !inside;

    for (uint32_t base = start; base < end; base += kTilePixels) {
        if (__syncthreads_count(done) == kTilePixels) break;
        const uint32_t idx = base + t;
        if (idx < end) {
            const uint32_t g = p.point_list[idx];
            const float4 a = p.record[3 * (size_t)g];
            const float4 b = p.record[3 * (size_t)g + 1];
            const float4 c = p.record[3 * (size_t)g + 2];
            sA[t] = make_float4(a.x, a.y, -0.5f * a.z, -0.5f * b.x);
            sB[t] = make_float2(a.w, b.y);
            sC[t] = make_float4(b.z, b.w, c.x, c.y);
            sD[t] = make_float2(c.z, c.w);
        }
        __syncthreads();
        const int cnt = (int)min((uint32_t)kTilePixels, end - base);
        for (int j = 0; j < cnt && !done; j++) {
            contributor++;
            const float4 A = sA[j];
            const float2 B = sB[j];
            const float dx = A.x - pfx, dy = A.y - pfy;
            const float power = fma_(A.z * dx, dx, fma_(A.w * dy, dy, -((B.x * dx) * dy)));
            if (power > 0.0f) continue;
            const float alpha = fminf(0.99f, B.y * expf_exact(power));
            if (alpha < 1.0f / 255.0f) continue;
            const float test_T = T * (1.0f - alpha);
            if (test_T < 0.0001f) {
                done = true;
                continue;
            }
            const float w = alpha * T;
            const float4 Cc = sC[j];
            C0 = fma_(Cc.x, w, C0);
            C1 = fma_(Cc.y, w, C1);
            C2 = fma_(Cc.z, w, C2);
            if (feat) {
                const float2 D = sD[j];
                F0 = fma_(Cc.w, w, F0);
                F1 = fma_(D.x, w, F1);
                F2 = fma_(D.y, w, F2);
            }
            T = test_T;
            last = contributor;
        }
    }
    if (inside) {
        const size_t HW = (size_t)p.W * p.H;
        const size_t pix = (size_t)py * p.W + px;
        p.final_T[pix] = T;
        p.n_contrib[pix] = last;
        p.out_color[pix] = fma_(T, p.bg[0], C0);
        p.out_color[HW + pix] = fma_(T, p.bg[1], C1);
        p.out_color[2 * HW + pix] = fma_(T, p.bg[2], C2);
        p.out_lang[pix] = F0;
        p.out_lang[HW + pix] = F1;
        p.out_lang[2 * HW + pix] = F2;
    }
}

hipError_t launch_render_forward(const RenderParams& p, int tiles, hipStream_t s)
{
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(k_render_forward, dim3(tiles), dim3(kTilePixels), 0, s, p);
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

__global__ __launch_bounds__(kTilePixels) void k_render_backward(RenderParams p)
{
    __shared__ float4 sA[kTilePixels];  // x, y, -0.5 conic.x, -0.5 conic.z
    __shared__ float2 sB[kTilePixels];  // conic.y, opacity
    __shared__ float4 sC[kTilePixels];  // r, g, b, f0
    __shared__ float2 sD[kTilePixels];  // f1, f2
    __shared__ uint32_t sId[kTilePixels];
    __shared__ float sG[kTilePixels * 12];  // per-entry gradient sums of the tile (12 floats)
    __shared__ uint32_t s_max;

    const int tile = blockIdx.x;
    const int tx = tile % p.gx, ty = tile / p.gx;
    const int t = threadIdx.x, lane = t & 63;
    const int px = tx * kTile + (t & (kTile - 1)), py = ty * kTile + (t >> 4);
    const bool inside = px < p.W && py < p.H;
    const float pfx = (float)px, pfy = (float)py;
    const size_t HW = (size_t)p.W * p.H;
    const size_t pix = (size_t)py * p.W + px;
    const uint32_t start = p.ranges[tile].x;
    const bool feat = p.include_feature != 0;

    const float T_final = inside ? p.final_T[pix] : 0.0f;
    const uint32_t last = inside ? p.n_contrib[pix] : 0u;
    float dp0 = 0.f, dp1 = 0.f, dp2 = 0.f, dq0 = 0.f, dq1 = 0.f, dq2 = 0.f;
    if (inside) {
        dp0 = p.dL_dcolor[pix];
        dp1 = p.dL_dcolor[HW + pix];
        dp2 = p.dL_dcolor[2 * HW + pix];
        if (feat && p.dL_dlang) {
            dq0 = p.dL_dlang[pix];
            dq1 = p.dL_dlang[HW + pix];
            dq2 = p.dL_dlang[2 * HW + pix];
        }
    }
    const float bg_dot = fma_(p.bg[2], dp2, fma_(p.bg[1], dp1, p.bg[0] * dp0));
    const float ddelx_dx = 0.5f * (float)p.W, ddely_dy = 0.5f * (float)p.H;

    // entries at list index >= max over the tile of n_contrib can contribute to no pixel
    if (t == 0) s_max = 0;
    __syncthreads();
    uint32_t wmax = last;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o, 64));
    if (lane == 0) atomicMax(&s_max, wmax);
    __syncthreads();
    const int maxl = (int)s_max;

    float T = T_final;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, accF0 = 0.f, accF1 = 0.f, accF2 = 0.f;
    float lc0 = 0.f, lc1 = 0.f, lc2 = 0.f, lf0 = 0.f, lf1 = 0.f, lf2 = 0.f;
    float last_alpha = 0.0f;
    const int vidx = scatter_index(lane);

    for (int done_cnt = 0; done_cnt < maxl; done_cnt += kTilePixels) {
        __syncthreads();
        const int k = maxl - 1 - (done_cnt + t);
        if (k >= 0) {
            const uint32_t g = p.point_list[start + (uint32_t)k];
            const float4 a = p.record[3 * (size_t)g];
            const float4 b = p.record[3 * (size_t)g + 1];
            const float4 c = p.record[3 * (size_t)g + 2];
            sA[t] = make_float4(a.x, a.y, -0.5f * a.z, -0.5f * b.x);
            sB[t] = make_float2(a.w, b.y);
            sC[t] = make_float4(b.z, b.w, c.x, c.y);
            sD[t] = make_float2(c.z, c.w);
            sId[t] = g;
        }
#pragma unroll
        for (int q = 0; q < 12; q++) sG[q * kTilePixels + t] = 0.f;
        __syncthreads();
        const int cnt = min(kTilePixels, maxl - done_cnt);
        for (int j = 0; j < cnt; j++) {
            const int kk = maxl - 1 - (done_cnt + j);  // list index of this entry
            float v[12];
#pragma unroll
            for (int q = 0; q < 12; q++) v[q] = 0.f;
            bool hit = false;
            if (kk < (int)last) {
                const float4 A = sA[j];
                const float2 B = sB[j];
                const float dx = A.x - pfx, dy = A.y - pfy;
                const float power = fma_(A.z * dx, dx, fma_(A.w * dy, dy, -((B.x * dx) * dy)));
                if (power <= 0.0f) {
                    const float G = expf_exact(power);
                    const float alpha = fminf(0.99f, B.y * G);
                    if (alpha >= 1.0f / 255.0f) {
                        hit = true;
                        const float4 Cc = sC[j];
                        const float one_m = 1.0f - alpha;
                        T = T / one_m;
                        const float dchannel_dcolor = alpha * T;
                        const float oml = 1.0f - last_alpha;
                        float dL_dalpha = 0.0f;
                        acc0 = fma_(last_alpha, lc0, oml * acc0);
                        lc0 = Cc.x;
                        dL_dalpha = fma_(Cc.x - acc0, dp0, dL_dalpha);
                        v[6] = dchannel_dcolor * dp0;
                        acc1 = fma_(last_alpha, lc1, oml * acc1);
                        lc1 = Cc.y;
                        dL_dalpha = fma_(Cc.y - acc1, dp1, dL_dalpha);
                        v[7] = dchannel_dcolor * dp1;
                        acc2 = fma_(last_alpha, lc2, oml * acc2);
                        lc2 = Cc.z;
                        dL_dalpha = fma_(Cc.z - acc2, dp2, dL_dalpha);
                        v[8] = dchannel_dcolor * dp2;
                        if (feat) {
                            const float2 D = sD[j];
                            accF0 = fma_(last_alpha, lf0, oml * accF0);
                            lf0 = Cc.w;
                            dL_dalpha = fma_(Cc.w - accF0, dq0, dL_dalpha);
                            v[9] = dchannel_dcolor * dq0;
                            accF1 = fma_(last_alpha, lf1, oml * accF1);
                            lf1 = D.x;
                            dL_dalpha = fma_(D.x - accF1, dq1, dL_dalpha);
                            v[10] = dchannel_dcolor * dq1;
                            accF2 = fma_(last_alpha, lf2, oml * accF2);
                            lf2 = D.y;
                            dL_dalpha = fma_(D.y - accF2, dq2, dL_dalpha);
                            v[11] = dchannel_dcolor * dq2;
                        }
                        dL_dalpha = dL_dalpha * T;
                        last_alpha = alpha;
                        dL_dalpha = fma_(-T_final / one_m, bg_dot, dL_dalpha);
                        const float cx = -2.0f * A.z, cz = -2.0f * A.w, cy = B.x;
                        const float dL_dG = B.y * dL_dalpha;
                        const float gdx = G * dx, gdy = G * dy;
                        const float dG_ddelx = -gdx * cx - gdy * cy;
                        const float dG_ddely = -gdy * cz - gdx * cy;
                        v[0] = dL_dG * dG_ddelx * ddelx_dx;
                        v[1] = dL_dG * dG_ddely * ddely_dy;
                        v[2] = -0.5f * gdx * dx * dL_dG;
                        v[3] = -0.5f * gdx * dy * dL_dG;
                        v[4] = -0.5f * gdy * dy * dL_dG;
                        v[5] = G * dL_dalpha;
                    }
                }
            }
            if (__ballot(hit) == 0ull) continue;  // wave-uniform skip
            const float tot = wave_reduce_scatter12(v, lane);
            if ((lane & 3) == 0 && vidx < 12) atomicAdd(&sG[j * 12 + vidx], tot);
        }
        __syncthreads();
        // flush: 16 lanes per entry (12 active) -> one 48-byte atomic row per (tile, Gaussian)
        for (int slot = t; slot < cnt * 16; slot += kTilePixels) {
            const int e = slot >> 4, q = slot & 15;
            if (q < 12) {
                const float val = sG[e * 12 + q];
                if (val != 0.0f) atomicAdd(&p.grad[(size_t)sId[e] * kGradStride + q], val);
            }
        }
    }
}

hipError_t launch_render_backward(const RenderParams& p, int tiles, hipStream_t s)
{
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(k_render_backward, dim3(tiles), dim3(kTilePixels), 0, s, p);
    return hipGetLastError();
}

}  // namespace lsr
