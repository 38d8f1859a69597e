// lsr_preprocess.hip -- per-Gaussian kernels: projection/culling/SH (forward) and the chain rule
// back to means, SH, scales and rotations (backward).  One thread per Gaussian; HBM-streaming.
//
// Forward restates upstream FORWARD::preprocessCUDA; backward
// restates computeCov2DCUDA + BACKWARD::preprocessCUDA (a12, a13, App. A.6).  Operation order
// mirrors oracle/lsr_oracle.c (preprocess_one / preprocess_backward_one).
#include "lsr_internal.h"

namespace lsr {

// SH coefficients of the block's 256 Gaussians are moved between HBM and LDS with coalesced
// accesses (the AoS P x M x 3 layout gives each lane 12M contiguous bytes, i.e. 48 separate cache
// lines per wave load otherwise); LDS rows are padded to 3M+1 floats, which keeps the per-lane
// row reads bank-conflict free.  A row can come from one source (shs, P x M x 3) or from two
// (the fused path's _features_dc P x 1 x 3 into columns 0-2 and _features_rest P x (M-1) x 3
// into columns 3..), which removes the per-step torch.cat of scene/gaussian_model.py:146-150.

// rows of w floats of the block's Gaussians from src -> LDS rows (stride ws) starting at col0;
// kW > 0 fixes the row width at compile time (the divisions become multiplies)
template <int kW, int kMaxPer>
__device__ __forceinline__ void rows_in(const float* __restrict__ src, int ng, int w_rt, float* lds, int ws, int col0)
{
    const int w = kW > 0 ? kW : w_rt;
    const int n = ng * w;
    const int n4 = (reinterpret_cast<uintptr_t>(src) & 15) == 0 ? (n >> 2) : 0;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    // kMaxPer dwordx4 loads per thread are issued before the first LDS write
    for (int k0 = 0; k0 < n4; k0 += kMaxPer * (int)blockDim.x) {
        float4 r[kMaxPer];
#pragma unroll
        for (int u = 0; u < kMaxPer; u++) {
            const int k = k0 + u * (int)blockDim.x + (int)threadIdx.x;
            if (k < n4) r[u] = s4[k];
        }
#pragma unroll
        for (int u = 0; u < kMaxPer; u++) {
            const int k = k0 + u * (int)blockDim.x + (int)threadIdx.x;
            if (k >= n4) continue;
            const int e = 4 * k;
            int gi = e / w, col = e - gi * w;
            if ((w & 3) == 0) {  // a float4 never straddles two rows
                float* d = lds + gi * ws + col0 + col;
                d[0] = r[u].x;
                d[1] = r[u].y;
                d[2] = r[u].z;
                d[3] = r[u].w;
            } else {
                const float v[4] = {r[u].x, r[u].y, r[u].z, r[u].w};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    lds[gi * ws + col0 + col] = v[j];
                    if (++col == w) {
                        col = 0;
                        gi++;
                    }
                }
            }
        }
    }
    for (int e = 4 * n4 + (int)threadIdx.x; e < n; e += blockDim.x) {
        const int gi = e / w;
        lds[gi * ws + col0 + (e - gi * w)] = src[e];
    }
}

template <int kW>
__device__ __forceinline__ void rows_out(float* __restrict__ dst, int ng, int w_rt, const float* lds, int ws, int col0)
{
    const int w = kW > 0 ? kW : w_rt;
    const int n = ng * w;
    const int n4 = (reinterpret_cast<uintptr_t>(dst) & 15) == 0 ? (n >> 2) : 0;
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int k = threadIdx.x; k < n4; k += blockDim.x) {
        const int e = 4 * k;
        int gi = e / w, col = e - gi * w;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            v[j] = lds[gi * ws + col0 + col];
            if (++col == w) {
                col = 0;
                gi++;
            }
        }
        d4[k] = make_float4(v[0], v[1], v[2], v[3]);
    }
    for (int e = 4 * n4 + (int)threadIdx.x; e < n; e += blockDim.x) {
        const int gi = e / w;
        dst[e] = lds[gi * ws + col0 + (e - gi * w)];
    }
}

// SH rows of the block into LDS (one source, or dc + rest); kDepth dwordx4 loads in flight per
// thread (deep for the forward, whose waves have registers to spare; shallower for the
// backward, whose arithmetic already limits its occupancy)
template <int kDepth>
__device__ __forceinline__ void stage_sh_in(const float* shs, const float* shs_rest, int P, int M, float* lds)
{
    const int g0 = blockIdx.x * blockDim.x, ng = min((int)blockDim.x, P - g0), ws = 3 * M + 1;
    if (!shs_rest) {
        if (M == 16) rows_in<48, kDepth>(shs + (size_t)g0 * 48, ng, 48, lds, ws, 0);
        else rows_in<0, kDepth>(shs + (size_t)g0 * 3 * M, ng, 3 * M, lds, ws, 0);
    } else {
        rows_in<3, kDepth>(shs + (size_t)g0 * 3, ng, 3, lds, ws, 0);
        if (M == 16) rows_in<45, kDepth>(shs_rest + (size_t)g0 * 45, ng, 45, lds, ws, 3);
        else if (M > 1) rows_in<0, kDepth>(shs_rest + (size_t)g0 * 3 * (M - 1), ng, 3 * (M - 1), lds, ws, 3);
    }
}

__device__ __forceinline__ void stage_sh_out(float* dsh, float* dsh_rest, int P, int M, const float* lds)
{
    const int g0 = blockIdx.x * blockDim.x, ng = min((int)blockDim.x, P - g0), ws = 3 * M + 1;
    if (!dsh_rest) {
        if (M == 16) rows_out<48>(dsh + (size_t)g0 * 48, ng, 48, lds, ws, 0);
        else rows_out<0>(dsh + (size_t)g0 * 3 * M, ng, 3 * M, lds, ws, 0);
    } else {
        rows_out<3>(dsh + (size_t)g0 * 3, ng, 3, lds, ws, 0);
        if (M == 16) rows_out<45>(dsh_rest + (size_t)g0 * 45, ng, 45, lds, ws, 3);
        else if (M > 1) rows_out<0>(dsh_rest + (size_t)g0 * 3 * (M - 1), ng, 3 * (M - 1), lds, ws, 3);
    }
}

// Split SH rows (_features_dc + _features_rest) with a 16-B aligned rest tensor: the block's rest
// rows are one contiguous run of ng x 3(M-1) floats, copied into LDS as it lies in HBM by LDS-DMA
// (global_load_lds_dwordx4: no VGPR destination, no per-element addressing), all in flight at once.
// A lane then reads its row at stride 3(M-1) floats: odd for even M (45 at M = 16), so the 32-bank
// ds_read_b32 rows of a wave never conflict.  The dc coefficients are read per lane.
__host__ __device__ __forceinline__ bool sh_dma(const float* shs, const float* shs_rest, int M)
{
    return shs && shs_rest && M >= 2 && (reinterpret_cast<uintptr_t>(shs_rest) & 15) == 0;
}

typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef __attribute__((address_space(1))) void* global_void_ptr;

__device__ __forceinline__ void stage_rest_dma(const float* __restrict__ rest, int P, int M, float* lds)
{
    const int w = 3 * (M - 1);
    const int g0 = blockIdx.x * kPreThreads, ng = min(kPreThreads, P - g0);
    const int n = ng * w, n4 = n >> 2;  // g0 * w * 4 bytes is 16-B aligned: kPreThreads % 4 == 0
    const float* src = rest + (size_t)g0 * w;
    const int lane = threadIdx.x & 63;
    // each wave-instruction writes 1 KiB of LDS at a wave-uniform base (+16 B per lane)
    for (int k0 = (int)(threadIdx.x & ~63); k0 < n4; k0 += kPreThreads)
        if (k0 + lane < n4)
            __builtin_amdgcn_global_load_lds((global_void_ptr)(src + 4 * (k0 + lane)),
                                             (lds_void_ptr)(lds + 4 * k0), 16, 0, 0);
    for (int e = 4 * n4 + (int)threadIdx.x; e < n; e += kPreThreads) lds[e] = src[e];  // ragged last block
}

static size_t sh_lds_bytes(const float* shs, const float* shs_rest, int M)
{
    if (!shs) return 0;
    if (sh_dma(shs, shs_rest, M)) return kPreThreads * (size_t)(3 * (M - 1)) * 4;
    return kPreThreads * (size_t)(3 * M + 1) * 4;
}

// SH staging variants: kShLds = register-staged rows (any layout), kShDma = stage_rest_dma
// (sh_dma() holds), kShDirect = no LDS, each lane loads its own 180-B _features_rest row
// (M == 16; dword-aligned dwordx4 loads) -- separate instances so that one path's VGPRs do not
// count against another
enum ShMode { kShLds = 0, kShDma = 1, kShDirect = 2 };

#ifndef LSR_PRE_NT  // 1: the SH rows (192 of the ~250 B read per Gaussian) loaded non-temporally
#define LSR_PRE_NT 0
#endif
#ifndef LSR_PRE_DIRECT_WAVES  // measurement knob: occupancy target of the kShDirect instance (0: none)
#define LSR_PRE_DIRECT_WAVES 0
#endif
template <int kSh>
__global__ __launch_bounds__(kPreThreads) __attribute__((amdgpu_waves_per_eu(
    kSh == kShDirect && LSR_PRE_DIRECT_WAVES > 0 ? LSR_PRE_DIRECT_WAVES : 1))) void k_preprocess(PreprocessParams p)
{
    extern __shared__ float s_sh[];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    for (int w = i; w < p.zero_words; w += gridDim.x * blockDim.x) p.zero[w] = 0u;
    for (int w = i; w < p.zero2_words; w += gridDim.x * blockDim.x) p.zero2[w] = 0u;
    // Per-Gaussian inputs are loaded first, so their latency overlaps the SH staging below
    // (issued after the barrier they would add a second memory round trip to every block).
    const bool live = i < p.P;
    float px = 0.f, py = 0.f, pz = 0.f, sx = 0.f, sy = 0.f, sz = 0.f, opac = 0.f;
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    float cov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float f0 = 0.f, f1 = 0.f, f2 = 0.f;
    const bool feat = p.include_feature && p.lang;
    constexpr bool dma = kSh != kShLds;  // split rows, dc read per lane
    float dc[3] = {0.f, 0.f, 0.f};
    float rr[45];  // kShDirect: the lane's _features_rest row
    // camera (uniform): kShDirect reads it into registers before the per-Gaussian loads, so its
    // loads neither trail those nor wait behind them
    const float* view = p.view;
    const float* proj = p.proj;
    const float* campos = p.campos;
    float cam_view[16], cam_proj[16], cam_pos[3];
    if (kSh == kShDirect) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            cam_view[k] = p.view[k];
            cam_proj[k] = p.proj[k];
        }
#pragma unroll
        for (int k = 0; k < 3; k++) cam_pos[k] = p.campos[k];
        view = cam_view;
        proj = cam_proj;
        campos = cam_pos;
    }
    if (kSh == kShDirect) {
        // the language step's layout (the launcher checks it): scales + rotations, the language
        // feature, split SH rows.  Every load is unconditional (a dead lane of the last block reads
        // Gaussian P - 1), so no branch joins sit between the loads and their registers.
        const uint32_t ic = (uint32_t)min(i, p.P - 1), o3 = ic * 12u;
        auto at = [](const float* base, uint32_t off) { return reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + off); };
        px = at(p.means, o3)[0];
        py = at(p.means, o3)[1];
        pz = at(p.means, o3)[2];
        q = load_f4u(at(p.rots, ic * 16u));
        sx = at(p.scales, o3)[0];
        sy = at(p.scales, o3)[1];
        sz = at(p.scales, o3)[2];
        opac = at(p.opac, ic * 4u)[0];
        if (!p.lang_deferred) {  // kernel-uniform
            f0 = at(p.lang, o3)[0];
            f1 = at(p.lang, o3)[1];
            f2 = at(p.lang, o3)[2];
        }
        dc[0] = at(p.shs, o3)[0];
        dc[1] = at(p.shs, o3)[1];
        dc[2] = at(p.shs, o3)[2];
        const char* row = reinterpret_cast<const char*>(p.shs_rest) + ic * 180u;
#pragma unroll
        for (int k = 0; k < 11; k++) {
            const float4 v = LSR_PRE_NT ? load_f4u_nt(row + 16 * k) : load_f4u(row + 16 * k);
            rr[4 * k] = v.x;
            rr[4 * k + 1] = v.y;
            rr[4 * k + 2] = v.z;
            rr[4 * k + 3] = v.w;
        }
        rr[44] = *reinterpret_cast<const float*>(row + 176);
        // a compiler-only memory clobber: the loads stay here, all in flight together, instead of
        // being sunk into the culling branches that use them (which made three round trips: the
        // means, then the rotation / scales behind the near-plane test, then the rest)
        asm volatile("" ::: "memory");
    } else if (live) {
        // 32-bit byte offsets on uniform bases (one VGPR per row width instead of a 64-bit address
        // per array; the launcher keeps 16 P below 2^31)
        const uint32_t o3 = (uint32_t)i * 12u, o4 = (uint32_t)i * 16u;
        auto at = [](const float* base, uint32_t off) { return reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + off); };
        px = at(p.means, o3)[0];
        py = at(p.means, o3)[1];
        pz = at(p.means, o3)[2];
        if (p.cov_pre) {
#pragma unroll
            for (int k = 0; k < 6; k++) cov[k] = p.cov_pre[6 * (size_t)i + k];
        } else {
            q = load_f4u(at(p.rots, o4));
            sx = at(p.scales, o3)[0];
            sy = at(p.scales, o3)[1];
            sz = at(p.scales, o3)[2];
        }
        opac = at(p.opac, 4u * (uint32_t)i)[0];
        if (feat && !p.lang_deferred) {
            f0 = at(p.lang, o3)[0];
            f1 = at(p.lang, o3)[1];
            f2 = at(p.lang, o3)[2];
        }
        if (dma) {
            dc[0] = at(p.shs, o3)[0];
            dc[1] = at(p.shs, o3)[1];
            dc[2] = at(p.shs, o3)[2];
        }
    }
    if (p.shs && kSh != kShDirect) {
        if (blockIdx.x * blockDim.x >= p.P) return;  // block-uniform
        if (dma) {
            stage_rest_dma(p.shs_rest, p.P, p.M, s_sh);
            __builtin_amdgcn_s_waitcnt(0);  // the LDS-DMA writes have landed (vmcnt 0)
        } else {
            stage_sh_in<12>(p.shs, p.shs_rest, p.P, p.M, s_sh);
        }
        __syncthreads();
    }
    // SH -> RGB (+0.5, clamp at 0, clamp flags: gaussian_renderer/__init__.py:80 semantics)
    float rgb[3];
    uint32_t clamp_bits = 0;
    auto eval_rgb = [&]() {
        const float dox = px - campos[0], doy = py - campos[1], doz = pz - campos[2];
        const float len = sqrtf(dot3(dox, doy, doz, dox, doy, doz));
        const float x = dox / len, y = doy / len, z = doz / len;
        const float* sh = kSh == kShDirect ? rr
                        : dma ? s_sh + threadIdx.x * (3 * (p.M - 1)) : s_sh + threadIdx.x * (3 * p.M + 1) + 3;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
            const float c0 = dma ? dc[ch] : sh[ch - 3];
            const float v = sh_eval_channel(p.D, c0, sh + ch, x, y, z) + 0.5f;
            clamp_bits |= (v < 0.0f ? 1u : 0u) << ch;
            rgb[ch] = fmaxf(v, 0.0f);
        }
    };
#ifndef LSR_PRE_EARLY_SH  // measurement knob: kShDirect evaluates the SH before the projection
#define LSR_PRE_EARLY_SH 0
#endif
    // (its 45 registers free before the projection arithmetic; culled Gaussians evaluate it too)
    constexpr bool early = kSh == kShDirect && LSR_PRE_EARLY_SH;
    if (early && live) eval_rgb();
    // per-thread contributions to the block partials: tile instances, super-tile entries, depth key
    uint32_t my_tiles = 0, my_supers = 0, my_key = 0xFFFFFFFFu, my_err = 0;
    bool vis = false;  // reached the end of the block below (else culled: written after it)
    if (live) do {  // `break` = culled
    const float3 pv = xform4x3(view, px, py, pz);
    if (pv.z <= 0.2f) {
        if (p.prefiltered) my_err = 0x80000000u;
        break;
    }
    const float3 hom = xform4x3(proj, px, py, pz);
    const float hw = xform4w(proj, px, py, pz);
    const float p_w = 1.0f / (hw + 0.0000001f);
    const float proj_x = hom.x * p_w, proj_y = hom.y * p_w;

    if (!p.cov_pre) {
        if (p.raw & LSR_RAW_ROTATIONS) q = act_normalize4(q);
        if (p.raw & LSR_RAW_SCALES) {
            sx = act_expf(sx);
            sy = act_expf(sy);
            sz = act_expf(sz);
        }
        cov3d(sx, sy, sz, p.scale_modifier, q, cov);
    }
    const Cov2D cv = cov2d(px, py, pz, p.focal_x, p.focal_y, p.tanfovx, p.tanfovy, cov, view);
    const float a = cv.a, b = cv.b, c = cv.c;
    const float det = a * c - b * b;
    if (det == 0.0f) break;
    const float det_inv = 1.f / det;
    const float cx = c * det_inv, cy = -b * det_inv, cz = a * det_inv;
    const float mid = 0.5f * (a + c);
    const float disc = fmaxf(0.1f, mid * mid - det);
    const float sq = sqrtf(disc);
    const float l1 = mid + sq, l2 = mid - sq;
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    const float ix = ndc2pix(proj_x, p.W), iy = ndc2pix(proj_y, p.H);
    const int r = (int)my_radius;
    int r4[4];
    tile_rect(ix, iy, r, p.gx, p.gy, r4);
    const uint32_t area = (uint32_t)((r4[2] - r4[0]) * (r4[3] - r4[1]));
    if (area == 0) break;

    if (p.shs) {
        if (!early) eval_rgb();
    } else {
        rgb[0] = p.colors[3 * i];
        rgb[1] = p.colors[3 * i + 1];
        rgb[2] = p.colors[3 * i + 2];
    }
    if (feat && (p.raw & LSR_RAW_LANGUAGE) && !p.lang_deferred) {
        const float3 f = act_lang(f0, f1, f2);
        f0 = f.x;
        f1 = f.y;
        f2 = f.z;
    }
    const float opacity = (p.raw & LSR_RAW_OPACITY) ? act_sigmoid(opac) : opac;
    p.depth_key[i] = __float_as_uint(pv.z);
    p.radii[i] = r;
    if (p.visible) p.visible[i] = r > 0 ? 1 : 0;
    p.tiles[i] = area;
    *reinterpret_cast<uint2*>(p.rect + 2 * (size_t)i) =
        make_uint2((uint32_t)r4[0] | ((uint32_t)r4[1] << 16), (uint32_t)r4[2] | ((uint32_t)r4[3] << 16));
    p.clamped[i] = clamp_bits;
    float4* rec = p.record + 3 * (size_t)i;
    rec[0] = make_float4(ix, iy, cx, cy);
    rec[1] = make_float4(cz, opacity, rgb[0], rgb[1]);
    if (p.lang_deferred)  // the language slots belong to the fill (which may already have run:
        reinterpret_cast<float*>(rec + 2)[0] = rgb[2];  // LSR_PHASE_COMPOSITE_FILLED); b only
    else
        rec[2] = make_float4(rgb[2], f0, f1, f2);
    my_tiles = area;
    my_supers = (uint32_t)(((r4[2] + kSuper - 1) / kSuper - r4[0] / kSuper) *
                           ((r4[3] + kSuper - 1) / kSuper - r4[1] / kSuper));
    my_key = __float_as_uint(pv.z);
    vis = true;
    } while (0);
    if (live && !vis) {  // culled: one store per output (the visible ones are written above)
        p.radii[i] = 0;
        if (p.visible) p.visible[i] = 0;
        p.tiles[i] = 0;
        p.depth_key[i] = 0xFFFFFFFFu;
        *reinterpret_cast<uint2*>(p.rect + 2 * (size_t)i) = make_uint2(0u, 0u);  // empty: culled
    }
    // block partials {R, E, min visible depth key, max visible depth key | error}: the host learns R, E and
    // the depth-key range before the depth sort (k_pre_reduce; the sort then needs only the bits
    // the visible keys actually span)
    __shared__ uint32_t red[4][kPreThreads / 64];
    // bit 31 of the max key carries the prefiltered error (visible keys are positive floats)
    uint32_t kmin = my_key, kmax = (my_key == 0xFFFFFFFFu ? 0u : my_key) | my_err;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        my_tiles += __shfl_xor(my_tiles, o, 64);
        my_supers += __shfl_xor(my_supers, o, 64);
        kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o, 64));
        kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o, 64));
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][wave] = my_tiles;
        red[1][wave] = my_supers;
        red[2][wave] = kmin;
        red[3][wave] = kmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint4 v = make_uint4(0u, 0u, 0xFFFFFFFFu, 0u);
        for (int w = 0; w < kPreThreads / 64; w++) {
            v.x += red[0][w];
            v.y += red[1][w];
            v.z = min(v.z, red[2][w]);
            v.w = max(v.w, red[3][w]);
        }
        p.partial[blockIdx.x] = v;
    }
}


// Deferred language feature (lsr_forward_args.language_ready): the records' language slots of the
// visible Gaussians, {b, f0, f1, f2} = record[3 i + 2] with b kept, after the stream has waited for
// the feature's update.  Same values (and activation) as the preprocess writes otherwise.  Four
// Gaussians per thread: their 48 feature bytes and 16 radius bytes are whole dwordx4 loads (a wave
// reads 3 KB + 1 KB contiguous); each record gets its three slots only (a dword and a dwordx2 store,
// no read of the colour word b).  On the pipelined step's critical path.
__device__ __forceinline__ void fill_one(float4* record, size_t i, float f0, float f1, float f2, int raw)
{
    if (raw & LSR_RAW_LANGUAGE) {
        const float3 f = act_lang(f0, f1, f2);
        f0 = f.x;
        f1 = f.y;
        f2 = f.z;
    }
    float* r = reinterpret_cast<float*>(record + 3 * i + 2);
    r[1] = f0;
    *reinterpret_cast<float2*>(r + 2) = make_float2(f1, f2);
}

__global__ __launch_bounds__(256) void k_fill_language(int P, const float* __restrict__ lang, int raw,
                                                       const int32_t* __restrict__ radii, float4* __restrict__ record)
{
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;  // Gaussians 4 q .. 4 q + 3
    const int64_t i0 = 4 * q;
    if (i0 >= P) return;
    const bool vec = i0 + 3 < P && ((reinterpret_cast<uintptr_t>(lang) | reinterpret_cast<uintptr_t>(radii)) & 15) == 0;
    if (vec) {
        const int4 r = reinterpret_cast<const int4*>(radii)[q];
        const float4* l4 = reinterpret_cast<const float4*>(lang) + 3 * q;
        const float4 a = l4[0], b = l4[1], c = l4[2];  // {f0 f1 f2 | f0} {f1 f2 | f0 f1} {f2 | f0 f1 f2}
        if (r.x > 0) fill_one(record, (size_t)i0, a.x, a.y, a.z, raw);
        if (r.y > 0) fill_one(record, (size_t)i0 + 1, a.w, b.x, b.y, raw);
        if (r.z > 0) fill_one(record, (size_t)i0 + 2, b.z, b.w, c.x, raw);
        if (r.w > 0) fill_one(record, (size_t)i0 + 3, c.y, c.z, c.w, raw);
        return;
    }
    for (int64_t i = i0; i < P && i < i0 + 4; i++)
        if (radii[i] > 0) fill_one(record, (size_t)i, lang[3 * i], lang[3 * i + 1], lang[3 * i + 2], raw);
}

hipError_t launch_fill_language(int P, const float* lang, int raw, const int32_t* radii, float4* record,
                                hipStream_t s)
{
    if (P == 0) return hipSuccess;
    const int64_t threads = ((int64_t)P + 3) / 4;
    hipLaunchKernelGGL(k_fill_language, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, P, lang, raw, radii,
                       record);
    return hipGetLastError();
}

// dynamic LDS beyond the 64 KiB default (M > 20 stored SH coefficients) must be opted into
static hipError_t allow_lds(const void* fn, size_t bytes)
{
    if (bytes <= 65536) return hipSuccess;
    if (bytes > 160 * 1024) return hipErrorInvalidValue;
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

hipError_t launch_preprocess(const PreprocessParams& p, hipStream_t s)
{
    if (p.P == 0) return hipSuccess;
    if (p.P >= (1 << 27)) return hipErrorInvalidValue;  // k_preprocess's 32-bit row offsets
    size_t lds = sh_lds_bytes(p.shs, p.shs_rest, p.M);
    static const int direct = [] {  // measurement knob: LSR_PRE_SH=dma (LDS-DMA staging instead)
        const char* v = getenv("LSR_PRE_SH");
        return v && v[0] == 'd' && v[1] == 'm' ? 0 : 1;
    }();
    const int mode = !sh_dma(p.shs, p.shs_rest, p.M) ? kShLds : (direct && p.M == 16 && p.D <= 3 && (int64_t)p.P * 180 < (int64_t)1 << 31 && !p.cov_pre && p.include_feature && p.lang)
                   ? kShDirect : kShDma;
    const void* fn = mode == kShDirect ? (const void*)k_preprocess<kShDirect>
                   : mode == kShDma ? (const void*)k_preprocess<kShDma> : (const void*)k_preprocess<kShLds>;
    if (mode == kShDirect) lds = 0;
    hipError_t e = allow_lds(fn, lds);
    if (e != hipSuccess) return e;
    const int nb = (p.P + kPreThreads - 1) / kPreThreads;
    if (mode == kShDirect) hipLaunchKernelGGL(k_preprocess<kShDirect>, dim3(nb), dim3(kPreThreads), 0, s, p);
    else if (mode == kShDma) hipLaunchKernelGGL(k_preprocess<kShDma>, dim3(nb), dim3(kPreThreads), lds, s, p);
    else hipLaunchKernelGGL(k_preprocess<kShLds>, dim3(nb), dim3(kPreThreads), lds, s, p);
    return hipGetLastError();  // the block partials are reduced by launch_publish_counters
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------

__device__ __forceinline__ void dnormvdv(float vx, float vy, float vz, float dx, float dy, float dz,
                                         float* out)
{
    const float sum2 = dot3(vx, vy, vz, vx, vy, vz);
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    out[0] = ((sum2 - vx * vx) * dx - vy * vx * dy - vz * vx * dz) * invsum32;
    out[1] = (-vx * vy * dx + (sum2 - vy * vy) * dy - vz * vy * dz) * invsum32;
    out[2] = (-vx * vz * dx - vy * vz * dy + (sum2 - vz * vz) * dz) * invsum32;
}

// SH backward (lso_sh_backward): writes all M coefficients of dsh, returns dL/dmean via the
// view direction.  drgb already masked by the clamp flags.
__device__ void sh_backward(int deg, int M, const float* sh, float dox, float doy, float doz,
                            const float* drgb, float* dsh, float* dmean)
{
    const float len = sqrtf(dot3(dox, doy, doz, dox, doy, doz));
    const float x = dox / len, y = doy / len, z = doz / len;
    float basis[16];
    float dx[3] = {0.f, 0.f, 0.f}, dy[3] = {0.f, 0.f, 0.f}, dz[3] = {0.f, 0.f, 0.f};
    const int K = (deg + 1) * (deg + 1);
    basis[0] = SH_C0;
    if (deg > 0) {
        basis[1] = -SH_C1 * y;
        basis[2] = SH_C1 * z;
        basis[3] = -SH_C1 * x;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            dx[c] = -SH_C1 * sh[3 * 3 + c];
            dy[c] = -SH_C1 * sh[1 * 3 + c];
            dz[c] = SH_C1 * sh[2 * 3 + c];
        }
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            basis[4] = SH_C2_0 * xy;
            basis[5] = SH_C2_1 * yz;
            basis[6] = SH_C2_2 * (2.f * zz - xx - yy);
            basis[7] = SH_C2_3 * xz;
            basis[8] = SH_C2_4 * (xx - yy);
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const float* s = sh + c;
                dx[c] = dx[c] + (SH_C2_0 * y * s[4 * 3] + SH_C2_2 * 2.f * -x * s[6 * 3] +
                                 SH_C2_3 * z * s[7 * 3] + SH_C2_4 * 2.f * x * s[8 * 3]);
                dy[c] = dy[c] + (SH_C2_0 * x * s[4 * 3] + SH_C2_1 * z * s[5 * 3] +
                                 SH_C2_2 * 2.f * -y * s[6 * 3] + SH_C2_4 * 2.f * -y * s[8 * 3]);
                dz[c] = dz[c] + (SH_C2_1 * y * s[5 * 3] + SH_C2_2 * 2.f * 2.f * z * s[6 * 3] +
                                 SH_C2_3 * x * s[7 * 3]);
            }
            if (deg > 2) {
                basis[9] = SH_C3_0 * y * (3.f * xx - yy);
                basis[10] = SH_C3_1 * xy * z;
                basis[11] = SH_C3_2 * y * (4.f * zz - xx - yy);
                basis[12] = SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
                basis[13] = SH_C3_4 * x * (4.f * zz - xx - yy);
                basis[14] = SH_C3_5 * z * (xx - yy);
                basis[15] = SH_C3_6 * x * (xx - 3.f * yy);
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const float* s = sh + c;
                    dx[c] = dx[c] + (SH_C3_0 * s[9 * 3] * 3.f * 2.f * xy + SH_C3_1 * s[10 * 3] * yz +
                                     SH_C3_2 * s[11 * 3] * -2.f * xy +
                                     SH_C3_3 * s[12 * 3] * -3.f * 2.f * xz +
                                     SH_C3_4 * s[13 * 3] * (-3.f * xx + 4.f * zz - yy) +
                                     SH_C3_5 * s[14 * 3] * 2.f * xz +
                                     SH_C3_6 * s[15 * 3] * 3.f * (xx - yy));
                    dy[c] = dy[c] + (SH_C3_0 * s[9 * 3] * 3.f * (xx - yy) + SH_C3_1 * s[10 * 3] * xz +
                                     SH_C3_2 * s[11 * 3] * (-3.f * yy + 4.f * zz - xx) +
                                     SH_C3_3 * s[12 * 3] * -3.f * 2.f * yz +
                                     SH_C3_4 * s[13 * 3] * -2.f * xy +
                                     SH_C3_5 * s[14 * 3] * -2.f * yz +
                                     SH_C3_6 * s[15 * 3] * -3.f * 2.f * xy);
                    dz[c] = dz[c] + (SH_C3_1 * s[10 * 3] * xy + SH_C3_2 * s[11 * 3] * 4.f * 2.f * yz +
                                     SH_C3_3 * s[12 * 3] * 3.f * (2.f * zz - xx - yy) +
                                     SH_C3_4 * s[13 * 3] * 4.f * 2.f * xz +
                                     SH_C3_5 * s[14 * 3] * (xx - yy));
                }
            }
        }
    }
    for (int k = 0; k < M; k++) {
        const float bk = k < K ? basis[k] : 0.0f;
        const bool live = k < K;
#pragma unroll
        for (int c = 0; c < 3; c++) dsh[3 * k + c] = live ? bk * drgb[c] : 0.0f;
    }
    const float ddx = dot3(dx[0], dx[1], dx[2], drgb[0], drgb[1], drgb[2]);
    const float ddy = dot3(dy[0], dy[1], dy[2], drgb[0], drgb[1], drgb[2]);
    const float ddz = dot3(dz[0], dz[1], dz[2], drgb[0], drgb[1], drgb[2]);
    dnormvdv(dox, doy, doz, ddx, ddy, ddz, dmean);
}

__device__ void cov3d_backward(float sx, float sy, float sz, float mod, float4 q, const float* dcov,
                               float* dscale, float* drot)
{
    const Mat3 R = quat_to_rot(q.x, q.y, q.z, q.w);
    const float s[3] = {mod * sx, mod * sy, mod * sz};
    float M[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int k = 0; k < 3; k++) M[i][k] = R.m[i][k] * s[k];
    const float D[3][3] = {{dcov[0], 0.5f * dcov[1], 0.5f * dcov[2]},
                           {0.5f * dcov[1], dcov[3], 0.5f * dcov[4]},
                           {0.5f * dcov[2], 0.5f * dcov[4], dcov[5]}};
    float G[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int k = 0; k < 3; k++)
            G[i][k] = 2.0f * fma_(D[i][2], M[2][k], fma_(D[i][1], M[1][k], D[i][0] * M[0][k]));
#pragma unroll
    for (int k = 0; k < 3; k++)
        dscale[k] = fma_(G[2][k], R.m[2][k], fma_(G[1][k], R.m[1][k], G[0][k] * R.m[0][k]));
    float dR[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int k = 0; k < 3; k++) dR[i][k] = G[i][k] * s[k];
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    drot[0] = 2.f * z * (dR[1][0] - dR[0][1]) + 2.f * y * (dR[0][2] - dR[2][0]) +
              2.f * x * (dR[2][1] - dR[1][2]);
    drot[1] = 2.f * y * (dR[0][1] + dR[1][0]) + 2.f * z * (dR[0][2] + dR[2][0]) +
              2.f * r * (dR[2][1] - dR[1][2]) - 4.f * x * (dR[2][2] + dR[1][1]);
    drot[2] = 2.f * x * (dR[0][1] + dR[1][0]) + 2.f * r * (dR[0][2] - dR[2][0]) +
              2.f * z * (dR[2][1] + dR[1][2]) - 4.f * y * (dR[2][2] + dR[0][0]);
    drot[3] = 2.f * r * (dR[1][0] - dR[0][1]) + 2.f * x * (dR[0][2] + dR[2][0]) +
              2.f * y * (dR[2][1] + dR[1][2]) - 4.f * z * (dR[1][1] + dR[0][0]);
}

// The per-Gaussian inputs of the backward, loaded before the SH staging so that the two memory
// round trips overlap.
struct BwdIn {
    int radius;
    uint32_t clamp;
    float4 ga, gb, gc;  // the 12 accumulated gradients (render backward record)
    float px, py, pz, opac;
    float4 q;
    float sc[3], lang[3], cov[6];
};

__device__ __forceinline__ void load_bwd_in(const PreprocessBwdParams& p, int i, BwdIn& in)
{
    const size_t i3 = 3 * (size_t)i;
    in.radius = p.radii[i];
    const float4* g4 = reinterpret_cast<const float4*>(p.grad + (size_t)i * kGradStride);
    in.ga = g4[0];
    in.gb = g4[1];
    in.gc = g4[2];
    in.px = p.means[i3];
    in.py = p.means[i3 + 1];
    in.pz = p.means[i3 + 2];
    in.clamp = p.shs ? p.clamped[i] : 0u;
    in.opac = (p.raw & LSR_RAW_OPACITY) ? p.opac[i] : 0.f;
    in.q = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < 3; k++) in.sc[k] = 0.f;
    for (int k = 0; k < 6; k++) in.cov[k] = 0.f;
    if (p.cov_pre) {
#pragma unroll
        for (int k = 0; k < 6; k++) in.cov[k] = p.cov_pre[6 * (size_t)i + k];
    } else {
        in.q = load_f4u(p.rots + 4 * (size_t)i);
        in.sc[0] = p.scales[i3];
        in.sc[1] = p.scales[i3 + 1];
        in.sc[2] = p.scales[i3 + 2];
    }
    const bool lang = (p.raw & LSR_RAW_LANGUAGE) && p.lang;
    for (int k = 0; k < 3; k++) in.lang[k] = lang ? p.lang[i3 + k] : 0.f;
}

__device__ __forceinline__ void preprocess_backward_one(const PreprocessBwdParams& p, int i, const BwdIn& in,
                                                        float* sh_row);

__global__ __launch_bounds__(kPreThreads) void k_preprocess_backward(PreprocessBwdParams p)
{
    extern __shared__ float s_sh[];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x * blockDim.x >= p.P) return;  // block-uniform
    BwdIn in;
    if (i < p.P) load_bwd_in(p, i, in);
    if (p.shs) {
        stage_sh_in<6>(p.shs, p.shs_rest, p.P, p.M, s_sh);
        __syncthreads();
    }
    if (i < p.P) preprocess_backward_one(p, i, in, s_sh + threadIdx.x * (3 * p.M + 1));
    if (p.shs && p.dsh) {
        __syncthreads();
        stage_sh_out(p.dsh, p.shs_rest ? p.dsh_rest : nullptr, p.P, p.M, s_sh);
    }
}

// One Gaussian.  `sh_row` holds its SH coefficients on entry (LDS) and receives dL/dsh.
__device__ __forceinline__ void preprocess_backward_one(const PreprocessBwdParams& p, int i, const BwdIn& in,
                                                        float* sh_row)
{
    const size_t i3 = 3 * (size_t)i;
    if (!(in.radius > 0)) {
        // culled: every output row is zero (upstream torch::zeros + skipped threads)
        for (int k = 0; k < 3; k++) {
            p.dmeans2D[i3 + k] = 0.f;
            p.dcolors[i3 + k] = 0.f;
            p.dlang[i3 + k] = 0.f;
            p.dmeans3D[i3 + k] = 0.f;
            if (p.dscales) p.dscales[i3 + k] = 0.f;
        }
        p.dopac[i] = 0.f;
        if (p.drots) *reinterpret_cast<float4*>(p.drots + 4 * (size_t)i) = make_float4(0.f, 0.f, 0.f, 0.f);
        if (p.dcov)
            for (int k = 0; k < 6; k++) p.dcov[6 * (size_t)i + k] = 0.f;
        if (p.shs)
            for (int k = 0; k < 3 * p.M; k++) sh_row[k] = 0.f;
        return;
    }
    const float4 ga = in.ga, gb = in.gb, gc = in.gc;
    // record: [0] dx [1] dy [2] dconic.x [3] dconic.y [4] dconic.w [5] dopacity [6..8] drgb [9..11] dlang
    const float dxy0 = ga.x, dxy1 = ga.y;
    const float dcx = ga.z, dcy = ga.w, dcz = gb.x;
    const float drgb_in[3] = {gb.z, gb.w, gc.x};
    p.dmeans2D[i3] = dxy0;
    p.dmeans2D[i3 + 1] = dxy1;
    p.dmeans2D[i3 + 2] = 0.f;
    p.dcolors[i3] = drgb_in[0];
    p.dcolors[i3 + 1] = drgb_in[1];
    p.dcolors[i3 + 2] = drgb_in[2];
    if ((p.raw & LSR_RAW_LANGUAGE) && p.lang) {
        const float3 d = act_lang_backward(in.lang[0], in.lang[1], in.lang[2], gc.y, gc.z, gc.w);
        p.dlang[i3] = d.x;
        p.dlang[i3 + 1] = d.y;
        p.dlang[i3 + 2] = d.z;
    } else {
        p.dlang[i3] = gc.y;
        p.dlang[i3 + 1] = gc.z;
        p.dlang[i3 + 2] = gc.w;
    }
    if (p.raw & LSR_RAW_OPACITY) {
        const float sg = act_sigmoid(in.opac);
        p.dopac[i] = gb.y * (1.0f - sg) * sg;  // torch sigmoid_backward: grad * (1 - y) * y
    } else {
        p.dopac[i] = gb.y;
    }

    const float px = in.px, py = in.py, pz = in.pz;
    float cov[6];
    float4 q = in.q;
    float sc[3] = {in.sc[0], in.sc[1], in.sc[2]};
    if (p.cov_pre) {
#pragma unroll
        for (int k = 0; k < 6; k++) cov[k] = in.cov[k];
    } else {
        if (p.raw & LSR_RAW_ROTATIONS) q = act_normalize4(q);
        if (p.raw & LSR_RAW_SCALES)
            for (int k = 0; k < 3; k++) sc[k] = act_expf(sc[k]);
        cov3d(sc[0], sc[1], sc[2], p.scale_modifier, q, cov);
    }
    const Cov2D cv = cov2d(px, py, pz, p.focal_x, p.focal_y, p.tanfovx, p.tanfovy, cov, p.view);
    const float limx = 1.3f * p.tanfovx, limy = 1.3f * p.tanfovy;
    const float x_grad_mul = (cv.txtz < -limx || cv.txtz > limx) ? 0.0f : 1.0f;
    const float y_grad_mul = (cv.tytz < -limy || cv.tytz > limy) ? 0.0f : 1.0f;
    const float a = cv.a, b = cv.b, c = cv.c;
    const float denom = a * c - b * b;
    float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
    const float denom2inv = 1.0f / (denom * denom + 0.0000001f);
    float dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float(&A)[2][3] = cv.A;
    if (denom2inv != 0.0f) {
        dL_da = denom2inv * (-c * c * dcx + 2.f * b * c * dcy + (denom - a * c) * dcz);
        dL_dc = denom2inv * (-a * a * dcz + 2.f * a * b * dcy + (denom - a * c) * dcx);
        dL_db = denom2inv * 2.f * (b * c * dcx - (denom + 2.f * b * b) * dcy + a * b * dcz);
        dcov[0] = A[0][0] * A[0][0] * dL_da + A[0][0] * A[1][0] * dL_db + A[1][0] * A[1][0] * dL_dc;
        dcov[3] = A[0][1] * A[0][1] * dL_da + A[0][1] * A[1][1] * dL_db + A[1][1] * A[1][1] * dL_dc;
        dcov[5] = A[0][2] * A[0][2] * dL_da + A[0][2] * A[1][2] * dL_db + A[1][2] * A[1][2] * dL_dc;
        dcov[1] = 2.f * A[0][0] * A[0][1] * dL_da + (A[0][0] * A[1][1] + A[0][1] * A[1][0]) * dL_db +
                  2.f * A[1][0] * A[1][1] * dL_dc;
        dcov[2] = 2.f * A[0][0] * A[0][2] * dL_da + (A[0][0] * A[1][2] + A[0][2] * A[1][0]) * dL_db +
                  2.f * A[1][0] * A[1][2] * dL_dc;
        dcov[4] = 2.f * A[0][2] * A[0][1] * dL_da + (A[0][1] * A[1][2] + A[0][2] * A[1][1]) * dL_db +
                  2.f * A[1][1] * A[1][2] * dL_dc;
    }
    const float S[3][3] = {{cov[0], cov[1], cov[2]}, {cov[1], cov[3], cov[4]}, {cov[2], cov[4], cov[5]}};
    float SA0[3], SA1[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        SA0[k] = dot3(A[0][0], A[0][1], A[0][2], S[k][0], S[k][1], S[k][2]);
        SA1[k] = dot3(A[1][0], A[1][1], A[1][2], S[k][0], S[k][1], S[k][2]);
    }
    float dA0[3], dA1[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        dA0[k] = 2.f * SA0[k] * dL_da + SA1[k] * dL_db;
        dA1[k] = 2.f * SA1[k] * dL_dc + SA0[k] * dL_db;
    }
    const float* v = p.view;
    const float dJ00 = fma_(v[8], dA0[2], fma_(v[4], dA0[1], v[0] * dA0[0]));
    const float dJ02 = fma_(v[10], dA0[2], fma_(v[6], dA0[1], v[2] * dA0[0]));
    const float dJ11 = fma_(v[9], dA1[2], fma_(v[5], dA1[1], v[1] * dA1[0]));
    const float dJ12 = fma_(v[10], dA1[2], fma_(v[6], dA1[1], v[2] * dA1[0]));
    const float tz = 1.f / cv.t[2];
    const float tz2 = tz * tz;
    const float tz3 = tz2 * tz;
    const float fx = p.focal_x, fy = p.focal_y;
    const float dtx = x_grad_mul * -fx * tz2 * dJ02;
    const float dty = y_grad_mul * -fy * tz2 * dJ12;
    const float dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2.f * fx * cv.t[0]) * tz3 * dJ02 +
                      (2.f * fy * cv.t[1]) * tz3 * dJ12;
    float dmean[3];
    dmean[0] = fma_(v[2], dtz, fma_(v[1], dty, v[0] * dtx));
    dmean[1] = fma_(v[6], dtz, fma_(v[5], dty, v[4] * dtx));
    dmean[2] = fma_(v[10], dtz, fma_(v[9], dty, v[8] * dtx));

    const float* m = p.proj;
    const float3 hom = xform4x3(m, px, py, pz);
    const float hw = xform4w(m, px, py, pz);
    const float m_w = 1.0f / (hw + 0.0000001f);
    const float mul1 = hom.x * m_w * m_w;
    const float mul2 = hom.y * m_w * m_w;
    dmean[0] += (m[0] * m_w - m[3] * mul1) * dxy0 + (m[1] * m_w - m[3] * mul2) * dxy1;
    dmean[1] += (m[4] * m_w - m[7] * mul1) * dxy0 + (m[5] * m_w - m[7] * mul2) * dxy1;
    dmean[2] += (m[8] * m_w - m[11] * mul1) * dxy0 + (m[9] * m_w - m[11] * mul2) * dxy1;

    if (p.shs) {
        const uint32_t cb = in.clamp;
        float drgb[3];
#pragma unroll
        for (int ch = 0; ch < 3; ch++) drgb[ch] = ((cb >> ch) & 1u) ? 0.0f : drgb_in[ch];
        float dm_sh[3];
        sh_backward(p.D, p.M, sh_row, px - p.campos[0], py - p.campos[1], pz - p.campos[2], drgb, sh_row,
                    dm_sh);
        dmean[0] += dm_sh[0];
        dmean[1] += dm_sh[1];
        dmean[2] += dm_sh[2];
    } else if (p.dsh) {
        for (int k = 0; k < 3 * p.M; k++) p.dsh[(size_t)i * 3 * p.M + k] = 0.f;
    }
    p.dmeans3D[i3] = dmean[0];
    p.dmeans3D[i3 + 1] = dmean[1];
    p.dmeans3D[i3 + 2] = dmean[2];
    if (p.dcov)
        for (int k = 0; k < 6; k++) p.dcov[6 * (size_t)i + k] = dcov[k];
    if (!p.cov_pre) {
        float ds[3], dr[4];
        cov3d_backward(sc[0], sc[1], sc[2], p.scale_modifier, q, dcov, ds, dr);
        if (p.raw & LSR_RAW_SCALES)
            for (int k = 0; k < 3; k++) ds[k] = ds[k] * sc[k];  // torch exp backward: grad * result
        if (p.raw & LSR_RAW_ROTATIONS) {
            const float4 d = act_normalize4_backward(in.q, make_float4(dr[0], dr[1], dr[2], dr[3]));
            dr[0] = d.x;
            dr[1] = d.y;
            dr[2] = d.z;
            dr[3] = d.w;
        }
        if (p.dscales) {
            p.dscales[i3] = ds[0];
            p.dscales[i3 + 1] = ds[1];
            p.dscales[i3 + 2] = ds[2];
        }
        if (p.drots) *reinterpret_cast<float4*>(p.drots + 4 * (size_t)i) = make_float4(dr[0], dr[1], dr[2], dr[3]);
    } else {
        if (p.dscales)
            for (int k = 0; k < 3; k++) p.dscales[i3 + k] = 0.f;
        if (p.drots) *reinterpret_cast<float4*>(p.drots + 4 * (size_t)i) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

hipError_t launch_preprocess_backward(const PreprocessBwdParams& p, hipStream_t s)
{
    if (p.P == 0) return hipSuccess;
    const size_t lds = kPreThreads * (size_t)(3 * p.M + 1) * 4 * (p.shs ? 1 : 0);
    hipError_t e = allow_lds((const void*)k_preprocess_backward, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_preprocess_backward, dim3((p.P + kPreThreads - 1) / kPreThreads), dim3(kPreThreads),
                       lds, s, p);
    return hipGetLastError();
}

// Backward without geometry gradients (lsr_backward with every geometry output NULL): only the
// screen-space gradient (dmeans2D) and the language-feature gradient, straight from the render
// backward's per-Gaussian record -- what preprocess_backward_one writes for these two outputs.
__global__ __launch_bounds__(256) void k_grad_epilogue(int P, const int* __restrict__ radii,
                                                       const float* __restrict__ grad, int stride,
                                                       const float* __restrict__ lang, int raw_lang,
                                                       float* __restrict__ dmeans2D, float* __restrict__ dlang)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const size_t i3 = 3 * (size_t)i;
    // every load is issued up front (one memory round trip): the records of culled Gaussians are
    // zero (the backward zero-fills them and adds nothing), radii only selects the zero result
    const int rad = radii[i];
    // stride kGradStrideLang: the packed 20-B record {dx, dy, l0, l1, l2} (consecutive lanes read
    // consecutive records: 20 B per Gaussian of HBM traffic); kGradStride: the full 64-B record
    float4 ga, gb;
    if (stride == kGradStrideLang) {
        const float* r = grad + (size_t)i * kGradStrideLang;
        ga = make_float4(r[0], r[1], r[2], r[3]);
        gb = make_float4(r[4], 0.f, 0.f, 0.f);
    } else {
        const float4* g4 = reinterpret_cast<const float4*>(grad + (size_t)i * stride);
        ga = g4[0];
        gb = g4[2];
    }
    const bool raw = raw_lang && lang && dlang;
    const float l0 = raw ? lang[i3] : 0.f, l1 = raw ? lang[i3 + 1] : 0.f, l2 = raw ? lang[i3 + 2] : 0.f;
    const bool live = rad > 0;
    if (dmeans2D) {
        dmeans2D[i3] = live ? ga.x : 0.f;
        dmeans2D[i3 + 1] = live ? ga.y : 0.f;
        dmeans2D[i3 + 2] = 0.f;
    }
    if (dlang) {
        float3 d = make_float3(0.f, 0.f, 0.f);
        if (live) {
            const float3 gl = stride == kGradStrideLang ? make_float3(ga.z, ga.w, gb.x) : make_float3(gb.y, gb.z, gb.w);
            d = raw ? act_lang_backward(l0, l1, l2, gl.x, gl.y, gl.z) : gl;
        }
        dlang[i3] = d.x;
        dlang[i3 + 1] = d.y;
        dlang[i3 + 2] = d.z;
    }
}

hipError_t launch_grad_epilogue(int P, const int* radii, const float* grad, int stride, const float* lang,
                                int raw_lang, float* dmeans2D, float* dlang, hipStream_t s)
{
    if (P == 0 || (!dmeans2D && !dlang)) return hipSuccess;
    hipLaunchKernelGGL(k_grad_epilogue, dim3((P + 255) / 256), dim3(256), 0, s, P, radii, grad, stride, lang,
                       raw_lang, dmeans2D, dlang);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_mark_visible(int P, const float* means, const float* view,
                                                      const float* proj, uint8_t* visible)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float3 pv = xform4x3(view, means[3 * i], means[3 * i + 1], means[3 * i + 2]);
    (void)proj;
    visible[i] = pv.z > 0.2f ? 1 : 0;
}

hipError_t launch_mark_visible(int P, const float* means, const float* view, const float* proj,
                               uint8_t* visible, hipStream_t s)
{
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mark_visible, dim3((P + 255) / 256), dim3(256), 0, s, P, means, view, proj, visible);
    return hipGetLastError();
}

}  // namespace lsr
