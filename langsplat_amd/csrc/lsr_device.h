// lsr_device.h -- device math shared by the rasterizer kernels (gfx950).
//
// Every expression here has the same explicit evaluation order as the CPU oracle
// (oracle/lsr_oracle.c); the kernels are compiled with -ffp-contract=off, so preprocessing and
// compositing produce bit-identical values on both sides.  Algorithm: the published 3DGS
// rasterizer forked by submodules/langsplat-rasterization (absent from the reference snapshot,
// SURVEY.md §0); call-site contract gaussian_renderer/__init__.py:37-105.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lsr {

constexpr int kTile = 16;              // BLOCK_X = BLOCK_Y = 16
constexpr int kTilePixels = kTile * kTile;

// Four floats of a caller's tensor at a dword-aligned address.  A contiguous torch view may start at
// any float (and a 180-B _features_rest row at a 4-B boundary), so the type tells the compiler the
// real alignment; gfx950's global_load_dwordx4 needs only dword alignment, so it is still one load.
typedef float lsr_f4u __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ float4 load_f4u(const void* ptr)
{
    const lsr_f4u v = *reinterpret_cast<const lsr_f4u*>(ptr);
    return make_float4(v.x, v.y, v.z, v.w);
}
// load_f4u with the non-temporal hint (streamed-once data: the cache keeps what other kernels reuse)
__device__ __forceinline__ float4 load_f4u_nt(const void* ptr)
{
    const lsr_f4u v = __builtin_nontemporal_load(reinterpret_cast<const lsr_f4u*>(ptr));
    return make_float4(v.x, v.y, v.z, v.w);
}

// SH constants, utils/sh_utils.py:26-45
constexpr float SH_C0 = 0.28209479177387814f;
constexpr float SH_C1 = 0.4886025119029199f;
constexpr float SH_C2_0 = 1.0925484305920792f, SH_C2_1 = -1.0925484305920792f,
                SH_C2_2 = 0.31539156525252005f, SH_C2_3 = -1.0925484305920792f,
                SH_C2_4 = 0.5462742152960396f;
constexpr float SH_C3_0 = -0.5900435899266435f, SH_C3_1 = 2.890611442640554f,
                SH_C3_2 = -0.4570457994644658f, SH_C3_3 = 0.3731763325901154f,
                SH_C3_4 = -0.4570457994644658f, SH_C3_5 = 1.445305721320277f,
                SH_C3_6 = -0.5900435899266435f;

// exp restatement (Cody-Waite by ln2 + a degree-6 polynomial fitted for relative error, 3e-9 on
// the reduced range; < 1 ulp overall); identical op sequence to lso_expf.
// n = x / ln2 rounded to nearest through the 1.5 * 2^23 shifter t (one fused rounding of the
// exact product); bits(t) = 0x4B400000 + n, and since 0x4B400000 << 23 == 0 (mod 2^32) the scale
// 2^n has the bits (bits(t) << 23) + (127 << 23): one shift-add, no rint / int conversion.
constexpr float kExpShift = 12582912.0f;  // 1.5 * 2^23
__device__ __forceinline__ float exp_scale(float t)
{
    return __uint_as_float((__float_as_uint(t) << 23) + (127u << 23));
}

__device__ __forceinline__ float expf_exact(float x)
{
    if (x < -87.0f) return 0.0f;
    const float t = __builtin_fmaf(x, 1.44269504088896341f, kExpShift);
    const float n = t - kExpShift;
    float r = __builtin_fmaf(n, -0.693145751953125f, x);
    r = __builtin_fmaf(n, -1.42860682030941723212e-6f, r);
    float p = 1.38145383e-3f;  // degree 6 (oracle lso_expf): c0 = c1 = 1, c2..c6 fitted
    p = __builtin_fmaf(p, r, 8.36874545e-3f);
    p = __builtin_fmaf(p, r, 4.16683890e-2f);
    p = __builtin_fmaf(p, r, 1.66665211e-1f);
    p = __builtin_fmaf(p, r, 4.99999940e-1f);
    p = __builtin_fmaf(p, r, 1.0f);
    p = __builtin_fmaf(p, r, 1.0f);
    return p * exp_scale(t);
}

// The render loops' exp (oracle lso_expf_render): expf_exact's polynomial after a one-constant
// range reduction (one FMA instead of two; <= 2 ulp for x >= -20, and every alpha the loops use
// comes from a power >= the cutoff of power_cutoff, > -6 for opacities up to 1e30), and no
// underflow branch.  Lanes below the cutoff get a meaningless value that no test lets through (the
// cutoff test rejects them whatever the alpha), so there is no clamp either (it cost 3 VALU per
// pair of entries in the forward walk).  Branch-free, so the chains of neighbouring list entries
// interleave.
__device__ __forceinline__ float expf_exact_render(float x)
{
    const float t = __builtin_fmaf(x, 1.44269504088896341f, kExpShift);
    const float n = t - kExpShift;
    // one-constant reduction (oracle lso_expf_render): |n| <= 8 on the compositing domain
    const float r = __builtin_fmaf(n, -0.693147182464599609375f, x);
    float p = 1.38145383e-3f;  // degree 6 (oracle lso_expf): c0 = c1 = 1, c2..c6 fitted
    p = __builtin_fmaf(p, r, 8.36874545e-3f);
    p = __builtin_fmaf(p, r, 4.16683890e-2f);
    p = __builtin_fmaf(p, r, 1.66665211e-1f);
    p = __builtin_fmaf(p, r, 4.99999940e-1f);
    p = __builtin_fmaf(p, r, 1.0f);
    p = __builtin_fmaf(p, r, 1.0f);
    return p * exp_scale(t);
}

// expf_exact_render of two values at once: the polynomial as packed fp32 (v_pk_fma_f32), i.e. the
// same IEEE operations per element in about half the instructions.
typedef float lsr_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ lsr_f2 make_f2(float x, float y)
{
    lsr_f2 v;
    v.x = x;
    v.y = y;
    return v;
}
__device__ __forceinline__ lsr_f2 expf_exact_render2(lsr_f2 x)
{
    const lsr_f2 t = __builtin_elementwise_fma(x, (lsr_f2)(1.44269504088896341f), (lsr_f2)(kExpShift));
    const lsr_f2 n = t - kExpShift;
    const lsr_f2 r = __builtin_elementwise_fma(n, (lsr_f2)(-0.693147182464599609375f), x);
    lsr_f2 p = (lsr_f2)(1.38145383e-3f);
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(8.36874545e-3f));
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(4.16683890e-2f));
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(1.66665211e-1f));
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(4.99999940e-1f));
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(1.0f));
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(1.0f));
    lsr_f2 sc;
    sc.x = exp_scale(t.x);
    sc.y = exp_scale(t.y);
    return p * sc;
}

// expf_exact_render2's constants held in scalar registers across a loop: defined by asm, so the
// compiler cannot re-materialise them (it re-created each one with an s_mov, or a v_mov for the two it
// put in vector registers, at every use: 8 issue slots per pair of entries in the forward walk)
struct ExpK {
    float log2e, shift, nln2, c6, c5, c4, c3, c2;
};
__device__ __forceinline__ ExpK exp_consts()
{
    ExpK k;
    asm("s_mov_b32 %0, 0x3fb8aa3b" : "=s"(k.log2e));  // 1.44269504088896341f
    asm("s_mov_b32 %0, 0x4b400000" : "=s"(k.shift));  // kExpShift
    asm("s_mov_b32 %0, 0xbf317218" : "=s"(k.nln2));   // -0.693147182464599609375f
    asm("s_mov_b32 %0, 0x3ab511e6" : "=s"(k.c6));     // 1.38145383e-3f
    asm("s_mov_b32 %0, 0x3c091d10" : "=s"(k.c5));     // 8.36874545e-3f
    asm("s_mov_b32 %0, 0x3d2aac79" : "=s"(k.c4));     // 4.16683890e-2f
    asm("s_mov_b32 %0, 0x3e2aaa49" : "=s"(k.c3));     // 1.66665211e-1f
    asm("s_mov_b32 %0, 0x3efffffe" : "=s"(k.c2));     // 4.99999940e-1f
    return k;
}
// expf_exact_render2 with the constants of exp_consts() (the same operations)
__device__ __forceinline__ lsr_f2 expf_exact_render2(lsr_f2 x, const ExpK& k)
{
    const lsr_f2 t = __builtin_elementwise_fma(x, (lsr_f2)(k.log2e), (lsr_f2)(k.shift));
    const lsr_f2 n = t - k.shift;
    const lsr_f2 r = __builtin_elementwise_fma(n, (lsr_f2)(k.nln2), x);
    lsr_f2 p = (lsr_f2)(k.c6);
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(k.c5));
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(k.c4));
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(k.c3));
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(k.c2));
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(1.0f));
    p = __builtin_elementwise_fma(p, r, (lsr_f2)(1.0f));
    lsr_f2 sc;
    sc.x = exp_scale(t.x);
    sc.y = exp_scale(t.y);
    return p * sc;
}

__device__ __forceinline__ float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// ---- parameter activations of the fused path (lsr_raw_flags; oracle lso_act_* restate them) ----
// exp over the whole float range: expf_exact below 88, +inf above (exp(88) = 1.65e38).
__device__ __forceinline__ float act_expf(float x) { return x > 88.0f ? __builtin_inff() : expf_exact(x); }
__device__ __forceinline__ float act_sigmoid(float x) { return 1.0f / (1.0f + act_expf(-x)); }
// torch.nn.functional.normalize(q, dim=1): q / max(||q||, 1e-12)
__device__ __forceinline__ float4 act_normalize4(float4 q)
{
    const float d = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), 1e-12f);
    return make_float4(q.x / d, q.y / d, q.z / d, q.w / d);
}
// autograd of q / clamp_min(norm(q), 1e-12): div, clamp_min and norm backward composed
__device__ __forceinline__ float4 act_normalize4_backward(float4 q, float4 g)
{
    const float n = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    const float d = fmaxf(n, 1e-12f);
    const float gd = -(g.x * q.x + g.y * q.y + g.z * q.z + g.w * q.w) / (d * d);
    const float k = (n >= 1e-12f && n > 0.0f) ? gd / n : 0.0f;
    return make_float4(g.x / d + q.x * k, g.y / d + q.y * k, g.z / d + q.z * k, g.w / d + q.w * k);
}
// language feature: f / (||f|| + 1e-9) (gaussian_renderer/__init__.py:87)
__device__ __forceinline__ float3 act_lang(float x, float y, float z)
{
    const float d = sqrtf(x * x + y * y + z * z) + 1e-9f;
    return make_float3(x / d, y / d, z / d);
}
__device__ __forceinline__ float3 act_lang_backward(float x, float y, float z, float gx, float gy, float gz)
{
    const float n = sqrtf(x * x + y * y + z * z);
    const float d = n + 1e-9f;
    const float gd = -(gx * x + gy * y + gz * z) / (d * d);
    const float k = n > 0.0f ? gd / n : 0.0f;
    return make_float3(gx / d + x * k, gy / d + y * k, gz / d + z * k);
}

// 3-term dot in the oracle's order: fma(a2,b2, fma(a1,b1, a0*b0))
__device__ __forceinline__ float dot3(float a0, float a1, float a2, float b0, float b1, float b2)
{
    return fma_(a2, b2, fma_(a1, b1, a0 * b0));
}

// Row-vector point transforms over a row-major 4x4 (scene/cameras.py:54-56 memory layout).
__device__ __forceinline__ float3 xform4x3(const float* m, float px, float py, float pz)
{
    return make_float3(fma_(m[8], pz, fma_(m[4], py, m[0] * px)) + m[12],
                       fma_(m[9], pz, fma_(m[5], py, m[1] * px)) + m[13],
                       fma_(m[10], pz, fma_(m[6], py, m[2] * px)) + m[14]);
}

__device__ __forceinline__ float xform4w(const float* m, float px, float py, float pz)
{
    return fma_(m[11], pz, fma_(m[7], py, m[3] * px)) + m[15];
}

__device__ __forceinline__ float ndc2pix(float v, int S)
{
    return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

struct Mat3 { float m[3][3]; };

__device__ __forceinline__ Mat3 quat_to_rot(float r, float x, float y, float z)
{
    Mat3 R;
    R.m[0][0] = 1.f - 2.f * (y * y + z * z);
    R.m[0][1] = 2.f * (x * y - r * z);
    R.m[0][2] = 2.f * (x * z + r * y);
    R.m[1][0] = 2.f * (x * y + r * z);
    R.m[1][1] = 1.f - 2.f * (x * x + z * z);
    R.m[1][2] = 2.f * (y * z - r * x);
    R.m[2][0] = 2.f * (x * z - r * y);
    R.m[2][1] = 2.f * (y * z + r * x);
    R.m[2][2] = 1.f - 2.f * (x * x + y * y);
    return R;
}

// Sigma = (R S)(R S)^T, packed (xx, xy, xz, yy, yz, zz): scene/gaussian_model.py:27-31
__device__ __forceinline__ void cov3d(float sx, float sy, float sz, float mod, float4 q, float* cov)
{
    Mat3 R = quat_to_rot(q.x, q.y, q.z, q.w);
    float s[3] = {mod * sx, mod * sy, mod * sz};
    float M[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int k = 0; k < 3; k++) M[i][k] = R.m[i][k] * s[k];
    cov[0] = dot3(M[0][0], M[0][1], M[0][2], M[0][0], M[0][1], M[0][2]);
    cov[1] = dot3(M[0][0], M[0][1], M[0][2], M[1][0], M[1][1], M[1][2]);
    cov[2] = dot3(M[0][0], M[0][1], M[0][2], M[2][0], M[2][1], M[2][2]);
    cov[3] = dot3(M[1][0], M[1][1], M[1][2], M[1][0], M[1][1], M[1][2]);
    cov[4] = dot3(M[1][0], M[1][1], M[1][2], M[2][0], M[2][1], M[2][2]);
    cov[5] = dot3(M[2][0], M[2][1], M[2][2], M[2][0], M[2][1], M[2][2]);
}

struct Cov2D {
    float t[3];      // clamped camera-space mean
    float A[2][3];   // J W
    float a, b, c;   // 2D covariance (+0.3 low-pass on a, c)
    float txtz, tytz;
};

// EWA projection A = J W; cov2D = A Sigma A^T + 0.3 I.
__device__ __forceinline__ Cov2D cov2d(float px, float py, float pz, float fx, float fy,
                                       float tanfovx, float tanfovy, const float* cov,
                                       const float* view)
{
    Cov2D o;
    float3 t = xform4x3(view, px, py, pz);
    float limx = 1.3f * tanfovx, limy = 1.3f * tanfovy;
    float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    float tz2 = t.z * t.z;
    float j00 = fx / t.z;
    float j02 = -(fx * t.x) / tz2;
    float j11 = fy / t.z;
    float j12 = -(fy * t.y) / tz2;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        float w0 = view[4 * k + 0], w1 = view[4 * k + 1], w2 = view[4 * k + 2];
        o.A[0][k] = fma_(j02, w2, j00 * w0);
        o.A[1][k] = fma_(j12, w2, j11 * w1);
    }
    const float S[3][3] = {{cov[0], cov[1], cov[2]}, {cov[1], cov[3], cov[4]}, {cov[2], cov[4], cov[5]}};
    float u0[3], u1[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
        u0[r] = dot3(S[r][0], S[r][1], S[r][2], o.A[0][0], o.A[0][1], o.A[0][2]);
        u1[r] = dot3(S[r][0], S[r][1], S[r][2], o.A[1][0], o.A[1][1], o.A[1][2]);
    }
    o.a = dot3(o.A[0][0], o.A[0][1], o.A[0][2], u0[0], u0[1], u0[2]) + 0.3f;
    o.b = dot3(o.A[1][0], o.A[1][1], o.A[1][2], u0[0], u0[1], u0[2]);
    o.c = dot3(o.A[1][0], o.A[1][1], o.A[1][2], u1[0], u1[1], u1[2]) + 0.3f;
    o.t[0] = t.x;
    o.t[1] = t.y;
    o.t[2] = t.z;
    o.txtz = txtz;
    o.tytz = tytz;
    return o;
}

// SH -> RGB for one channel (utils/sh_utils.py:57-112).  c0 is coefficient 0 of the channel; rest
// points at the channel's coefficient 1, coefficients strided by 3 (the P x M x 3 layout of
// GaussianModel.get_features from column 3, or a _features_rest row).
__device__ __forceinline__ float sh_eval_channel(int deg, float c0, const float* rest, float x, float y, float z)
{
    float res = SH_C0 * c0;
    if (deg > 0) {
        res = res - (SH_C1 * y) * rest[0 * 3];
        res = res + (SH_C1 * z) * rest[1 * 3];
        res = res - (SH_C1 * x) * rest[2 * 3];
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            res = res + (SH_C2_0 * xy) * rest[3 * 3];
            res = res + (SH_C2_1 * yz) * rest[4 * 3];
            res = res + (SH_C2_2 * (2.0f * zz - xx - yy)) * rest[5 * 3];
            res = res + (SH_C2_3 * xz) * rest[6 * 3];
            res = res + (SH_C2_4 * (xx - yy)) * rest[7 * 3];
            if (deg > 2) {
                res = res + (SH_C3_0 * y * (3.0f * xx - yy)) * rest[8 * 3];
                res = res + (SH_C3_1 * xy * z) * rest[9 * 3];
                res = res + (SH_C3_2 * y * (4.0f * zz - xx - yy)) * rest[10 * 3];
                res = res + (SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy)) * rest[11 * 3];
                res = res + (SH_C3_4 * x * (4.0f * zz - xx - yy)) * rest[12 * 3];
                res = res + (SH_C3_5 * z * (xx - yy)) * rest[13 * 3];
                res = res + (SH_C3_6 * x * (xx - 3.0f * yy)) * rest[14 * 3];
            }
        }
    }
    return res;
}

// Tile rectangle of a projected Gaussian (upstream getRect; clamped to the tile grid).
__device__ __forceinline__ void tile_rect(float ix, float iy, int r, int gx, int gy, int* r4)
{
    int v0 = (int)((ix - (float)r) / (float)kTile);
    int v1 = (int)((iy - (float)r) / (float)kTile);
    int v2 = (int)((ix + (float)r + (float)kTile - 1.0f) / (float)kTile);
    int v3 = (int)((iy + (float)r + (float)kTile - 1.0f) / (float)kTile);
    r4[0] = min(gx, max(0, v0));
    r4[1] = min(gy, max(0, v1));
    r4[2] = min(gx, max(0, v2));
    r4[3] = min(gy, max(0, v3));
}

// Per-Gaussian record gathered by the render kernels (48 B = 3 x dwordx4).
struct Record {
    float4 a;  // x, y, conic.x, conic.y
    float4 b;  // conic.z, opacity, r, g
    float4 c;  // b, f0, f1, f2
};

}  // namespace lsr
