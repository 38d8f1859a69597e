/*
 * lsr_oracle.c -- CPU restatement of the LangSplat differentiable Gaussian rasterizer
 * (forward + backward of RasterizeGaussians).
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (langsplat_amd/, include/,
 * diff_gaussian_rasterization/) links, loads or calls this file.  It is used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the checker.
 *
 * What it restates
 * ----------------
 * The rasterizer itself is the un-vendored git submodule submodules/langsplat-rasterization
 * (/root/reference/.gitmodules:7-9; the directory is empty in the snapshot).
 * This file therefore restates the published 3DGS "diff-gaussian-rasterization" algorithm
 * that the fork extends with a 3-channel language feature, pinned by
 * the reference call sites:
 *   - gaussian_renderer/__init__.py:37-51   settings (13 fields)
 *   - gaussian_renderer/__init__.py:61-91   which inputs are populated
 *   - gaussian_renderer/__init__.py:96-105  call and the (color, language, radii) return
 *   - utils/sh_utils.py:26-112              SH basis (pinned by tests/golden fixtures)
 *   - scene/cameras.py:54-57                matrix conventions (row-vector, transposed)
 *   - scene/gaussian_model.py:27-31         covariance = R S S^T R^T
 *
 * Arithmetic contract
 * -------------------
 * Every floating-point expression is written with an explicit evaluation order and explicit
 * fmaf() where a fused operation is wanted; the file is compiled with -ffp-contract=off.
 * The HIP kernels (langsplat_amd/csrc/, .hip files) follow the same order and are compiled the same
 * way, and both use the same exp() restatement (lsr_expf below), so the FORWARD outputs
 * (images, radii, per-tile lists, final T, contributor counts) are bit-identical between this
 * oracle and the GPU.  Gradients are accumulated here in double (the GPU uses float atomics in
 * arbitrary order) so backward parity is a tolerance, not bit-exactness.
 *
 * Pinning: the SH basis and its backward, the camera matrices and the
 * covariance are pinned to the reference's own Python (tests/golden, generated from
 * /root/reference/utils); the compositing core is PARITY UNPINNED against the reference
 * implementation (its source is the absent submodule) and is pinned instead to the published
 * algorithm by analytic known-answer tests and by the independent autograd formulation in
 * oracle/torch_ref.py.
 *
 * Upstream-vs-fork decisions (SURVEY.md marks them <U?>) taken here and in the kernels:
 *   - language channel composited with the same weights as RGB, with NO background term;
 *   - language channel contributes to dL/dalpha (the mathematically exact gradient);
 *   - when include_feature == 0 the language image is all zeros and its gradient is zero.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define BLOCK_X 16
#define BLOCK_Y 16

/* ------------------------------------------------------------------------------------------ */
/* settings / state                                                                             */
/* ------------------------------------------------------------------------------------------ */

typedef struct lso_settings {
    int32_t image_height;
    int32_t image_width;
    float tanfovx;
    float tanfovy;
    float scale_modifier;
    int32_t sh_degree;
    int32_t include_feature;
    int32_t prefiltered;
    float bg[3];
    float viewmatrix[16];
    float projmatrix[16];
    float campos[3];
    /* arithmetic form (see "Upstream forms" below): 0 = the kernels' operation sequence (the
       bit-exact contract), 1 = upstream's source expressions, one rounding per operation,
       2 = the same expressions with nvcc-style multiply-add contraction */
    int32_t form;
} lso_settings;

#define LSO_FORM_KERNEL 0
#define LSO_FORM_UPSTREAM 1
#define LSO_FORM_UPSTREAM_FMA 2

typedef struct lso_state {
    lso_settings s;
    int form;
    int P, M, gx, gy;
    int has_shs, has_colors, has_cov, has_lang;
    /* private copies of the inputs (the backward re-reads them) */
    float *means, *shs, *colors, *lang, *opac, *scales, *rots, *cov_pre;
    /* per-Gaussian state */
    float *depth, *xy, *conic_o, *rgb;
    int32_t *radii;
    uint32_t *tiles;
    uint8_t *clamped;
    /* binning */
    int64_t R;
    uint32_t *point_list; /* R Gaussian ids, tile-major, depth-then-id ordered */
    uint32_t *ranges;     /* 2 per tile: [start, end) */
    /* per-pixel */
    float *final_T;
    uint32_t *n_contrib;
} lso_state;

/* SH constants: utils/sh_utils.py:26-45 (as float, the kernel's precision) */
static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

static inline float bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* exp restatement shared (as a specification, not as code) with the kernels:
 * Cody-Waite reduction by ln2 and a degree-6 polynomial (c0 = c1 = 1, c2..c6 fitted for relative
 * error: 3e-9 on |r| <= ln2 / 2, 0.82 ulp overall); exact for the image, since
 * both sides evaluate the identical sequence of correctly-rounded IEEE operations. */
float lso_expf(float x)
{
    if (x < -87.0f) return 0.0f;
    /* n = x / ln2 rounded to nearest by the 1.5 * 2^23 shifter (one fused rounding of the exact
       product); the shifted value's low mantissa bits are n, which also gives 2^n's exponent */
    const float t = fmaf(x, 1.44269504088896341f, 12582912.0f);
    const float n = t - 12582912.0f;
    float r = fmaf(n, -0.693145751953125f, x);
    r = fmaf(n, -1.42860682030941723212e-6f, r);
    /* degree 6 with c0 = c1 = 1, c2..c6 fitted for relative error (3e-9 on |r| <= ln2 / 2) */
    float p = 1.38145383e-3f;
    p = fmaf(p, r, 8.36874545e-3f);
    p = fmaf(p, r, 4.16683890e-2f);
    p = fmaf(p, r, 1.66665211e-1f);
    p = fmaf(p, r, 4.99999940e-1f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    /* bits(t) = 0x4B400000 + n and 0x4B400000 << 23 == 0 (mod 2^32): (n + 127) << 23 */
    return p * bits2f((f2bits(t) << 23) + (127u << 23));
}

/* The compositing loops' exp (render forward / backward and the kernels' expf_exact_render*): as
 * lso_expf with a one-constant range reduction, valid (<= 2 ulp) for x >= -20; every power the
 * render loops composite is >= ln(1/255) - 0.01. */
float lso_expf_render(float x)
{
    if (x < -87.0f) return 0.0f;
    /* n = x / ln2 rounded to nearest by the 1.5 * 2^23 shifter (one fused rounding of the exact
       product); the shifted value's low mantissa bits are n, which also gives 2^n's exponent */
    const float t = fmaf(x, 1.44269504088896341f, 12582912.0f);
    const float n = t - 12582912.0f;
    /* one-constant reduction: |n| <= 8 on the compositing domain (power >= ln(1/255) - 0.01), so
       n (ln2_f - ln2) stays below 1.4e-8 (0.2 ulp); one FMA instead of two */
    float r = fmaf(n, -0.693147182464599609375f, x);
    /* degree 6 with c0 = c1 = 1, c2..c6 fitted for relative error (3e-9 on |r| <= ln2 / 2) */
    float p = 1.38145383e-3f;
    p = fmaf(p, r, 8.36874545e-3f);
    p = fmaf(p, r, 4.16683890e-2f);
    p = fmaf(p, r, 1.66665211e-1f);
    p = fmaf(p, r, 4.99999940e-1f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    /* bits(t) = 0x4B400000 + n and 0x4B400000 << 23 == 0 (mod 2^32): (n + 127) << 23 */
    return p * bits2f((f2bits(t) << 23) + (127u << 23));
}

/* ------------------------------------------------------------------------------------------ */
/* point transforms (row-vector matrices stored row-major: scene/cameras.py:54-56)             */
/* ------------------------------------------------------------------------------------------ */

static inline void xform4x3(const float* m, const float* p, float* o)
{
    o[0] = fmaf(m[8], p[2], fmaf(m[4], p[1], m[0] * p[0])) + m[12];
    o[1] = fmaf(m[9], p[2], fmaf(m[5], p[1], m[1] * p[0])) + m[13];
    o[2] = fmaf(m[10], p[2], fmaf(m[6], p[1], m[2] * p[0])) + m[14];
}

static inline void xform4x4(const float* m, const float* p, float* o)
{
    xform4x3(m, p, o);
    o[3] = fmaf(m[11], p[2], fmaf(m[7], p[1], m[3] * p[0])) + m[15];
}

static inline float ndc2pix(float v, int S)
{
    /* the upstream helper computes in double ((v + 1.0) * S - 1.0) * 0.5 */
    return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

/* ------------------------------------------------------------------------------------------ */
/* covariance                                                                                  */
/* ------------------------------------------------------------------------------------------ */

/* Standard rotation matrix of quaternion (r,x,y,z), utils/general_utils.py:90-98, WITHOUT
 * renormalisation (the caller normalised it, scene/gaussian_model.py:139-140). */
static void quat_to_rot(const float* q, float R[3][3])
{
    float r = q[0], x = q[1], y = q[2], z = q[3];
    R[0][0] = 1.f - 2.f * (y * y + z * z);
    R[0][1] = 2.f * (x * y - r * z);
    R[0][2] = 2.f * (x * z + r * y);
    R[1][0] = 2.f * (x * y + r * z);
    R[1][1] = 1.f - 2.f * (x * x + z * z);
    R[1][2] = 2.f * (y * z - r * x);
    R[2][0] = 2.f * (x * z - r * y);
    R[2][1] = 2.f * (y * z + r * x);
    R[2][2] = 1.f - 2.f * (x * x + y * y);
}

/* Sigma = (R S)(R S)^T packed (xx, xy, xz, yy, yz, zz): scene/gaussian_model.py:27-31 */
void lso_cov3d(const float* scale, float mod, const float* rot, float* cov)
{
    float R[3][3], M[3][3];
    float s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    quat_to_rot(rot, R);
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) M[i][k] = R[i][k] * s[k];
#define DOT3(a, b) fmaf((a)[2], (b)[2], fmaf((a)[1], (b)[1], (a)[0] * (b)[0]))
    cov[0] = DOT3(M[0], M[0]);
    cov[1] = DOT3(M[0], M[1]);
    cov[2] = DOT3(M[0], M[2]);
    cov[3] = DOT3(M[1], M[1]);
    cov[4] = DOT3(M[1], M[2]);
    cov[5] = DOT3(M[2], M[2]);
}

/* EWA projection: A = J W (2x3); cov2D = A Sigma A^T + 0.3 I.  Returns the clamped camera-space
 * point in t and A for the backward. */
static void cov2d(const float* mean, float fx, float fy, float tanfovx, float tanfovy,
                  const float* cov, const float* view, float* t, float A[2][3], float* abc,
                  float* txtz_out, float* tytz_out)
{
    xform4x3(view, mean, t);
    float limx = 1.3f * tanfovx, limy = 1.3f * tanfovy;
    float txtz = t[0] / t[2], tytz = t[1] / t[2];
    t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
    t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
    float tz2 = t[2] * t[2];
    float j00 = fx / t[2];
    float j02 = -(fx * t[0]) / tz2;
    float j11 = fy / t[2];
    float j12 = -(fy * t[1]) / tz2;
    /* W = rotation block of the world->camera matrix: view is stored transposed */
    for (int k = 0; k < 3; k++) {
        float w0 = view[4 * k + 0], w1 = view[4 * k + 1], w2 = view[4 * k + 2];
        A[0][k] = fmaf(j02, w2, j00 * w0);
        A[1][k] = fmaf(j12, w2, j11 * w1);
    }
    float S[3][3] = {{cov[0], cov[1], cov[2]}, {cov[1], cov[3], cov[4]}, {cov[2], cov[4], cov[5]}};
    float u0[3], u1[3];
    for (int r = 0; r < 3; r++) {
        u0[r] = DOT3(S[r], A[0]);
        u1[r] = DOT3(S[r], A[1]);
    }
    abc[0] = DOT3(A[0], u0) + 0.3f;
    abc[1] = DOT3(A[1], u0);
    abc[2] = DOT3(A[1], u1) + 0.3f;
    if (txtz_out) *txtz_out = txtz;
    if (tytz_out) *tytz_out = tytz;
}

/* ------------------------------------------------------------------------------------------ */
/* Upstream forms (a number for the unpinned core)                          */
/* ------------------------------------------------------------------------------------------ */
/* The kernels and form 0 evaluate kernel-shaped expressions (the 4-op power, the shared exp
 * restatement, A = J W with b = A1 (S A0), f (alpha T)).  Forms 1 and 2 evaluate instead the
 * expressions of the published 3DGS rasterizer that the absent submodule forks, as its source
 * writes them:
 *   - transformPoint4x3/4x4: m[0] x + m[4] y + m[8] z + m[12], left to right;
 *   - computeCov3D with glm: R from the quaternion, M = S R, Sigma = M^T M (glm's column-major
 *     products, each a left-to-right sum over k);
 *   - computeCov2D with glm: T = W J, cov = T^T V^T T evaluated left to right, +0.3 on the diagonal;
 *     det = a c - b b, conic, mid, lambda, radius as written;
 *   - computeColorFromSH: dir / glm::length(dir) (length = sqrt of the left-to-right dot), the basis
 *     sums as written;
 *   - renderCUDA: power = -0.5f (c.x dx dx + c.z dy dy) - c.y dx dy, alpha = min(0.99, o exp(power))
 *     with exp correctly rounded ((float)exp((double)x): CUDA's expf is within 2 ulp, so the
 *     nearest float is the best single stand-in), C += f alpha T (as (f alpha) T);
 *   - the backward renderCUDA's power, G = exp(power) and dG/ddelta = -gdx c.x - gdy c.y as written.
 * Form 1 rounds every operation.  Form 2 contracts a*b+c / a*b-c into one fma where nvcc's
 * default -fmad=true would: following LLVM's DAG combiner, in x*y + u*v the LEFT product is fused
 * (fma(x, y, u*v)), in s + x*y and s - x*y the product is fused into the sum.  Which products
 * upstream's compiler really fused is not knowable here; the two forms bracket the plausible
 * arithmetic.  Everything else (the tile rectangle, ndc2Pix, the preprocess backward's chain rule,
 * the SH and covariance backward) is shared with form 0, whose sequence there already follows the
 * upstream source.  tests/test_gpu_upstream_form.py reports and bounds HIP vs forms 1 and 2. */

static inline float u_sum2(int f, float a0, float b0, float a1, float b1)
{
    return f == LSO_FORM_UPSTREAM_FMA ? fmaf(a0, b0, a1 * b1) : a0 * b0 + a1 * b1;
}

static inline float u_sum3(int f, float a0, float b0, float a1, float b1, float a2, float b2)
{
    return f == LSO_FORM_UPSTREAM_FMA ? fmaf(a2, b2, fmaf(a0, b0, a1 * b1)) : (a0 * b0 + a1 * b1) + a2 * b2;
}

/* a*b - c*d */
static inline float u_diffp(int f, float a, float b, float c, float d)
{
    return f == LSO_FORM_UPSTREAM_FMA ? fmaf(a, b, -(c * d)) : a * b - c * d;
}

/* a*b - s */
static inline float u_prodsub(int f, float a, float b, float s)
{
    return f == LSO_FORM_UPSTREAM_FMA ? fmaf(a, b, -s) : a * b - s;
}

/* s + a*b */
static inline float u_addp(int f, float s, float a, float b)
{
    return f == LSO_FORM_UPSTREAM_FMA ? fmaf(a, b, s) : s + a * b;
}

/* s - a*b */
static inline float u_subp(int f, float s, float a, float b)
{
    return f == LSO_FORM_UPSTREAM_FMA ? fmaf(-a, b, s) : s - a * b;
}

static inline float u_exp(float x) { return (float)exp((double)x); }

static inline void u_xform4x3(int f, const float* m, const float* p, float* o)
{
    for (int r = 0; r < 3; r++) o[r] = u_sum3(f, m[r], p[0], m[4 + r], p[1], m[8 + r], p[2]) + m[12 + r];
}

static inline void u_xform4x4(int f, const float* m, const float* p, float* o)
{
    for (int r = 0; r < 4; r++) o[r] = u_sum3(f, m[r], p[0], m[4 + r], p[1], m[8 + r], p[2]) + m[12 + r];
}

/* computeCov3D with glm (column-major g[c][r]): R's columns from the quaternion, M = S R,
 * Sigma = M^T M: Sigma[c][r] = sum_k M[r][k] M[c][k]. */
static void u_cov3d(int f, const float* scale, float mod, const float* q, float* cov)
{
    const float r = q[0], x = q[1], y = q[2], z = q[3];
    float R[3][3];
    R[0][0] = u_subp(f, 1.f, 2.f, u_sum2(f, y, y, z, z));
    R[0][1] = 2.f * u_diffp(f, x, y, r, z);
    R[0][2] = 2.f * u_sum2(f, x, z, r, y);
    R[1][0] = 2.f * u_sum2(f, x, y, r, z);
    R[1][1] = u_subp(f, 1.f, 2.f, u_sum2(f, x, x, z, z));
    R[1][2] = 2.f * u_diffp(f, y, z, r, x);
    R[2][0] = 2.f * u_diffp(f, x, z, r, y);
    R[2][1] = 2.f * u_sum2(f, y, z, r, x);
    R[2][2] = u_subp(f, 1.f, 2.f, u_sum2(f, x, x, y, y));
    const float s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    float M[3][3];
    for (int c = 0; c < 3; c++)
        for (int k = 0; k < 3; k++) M[c][k] = s[k] * R[c][k]; /* S diagonal: the zero terms add +-0 */
#define SIG(c, r) u_sum3(f, M[r][0], M[c][0], M[r][1], M[c][1], M[r][2], M[c][2])
    cov[0] = SIG(0, 0);
    cov[1] = SIG(0, 1);
    cov[2] = SIG(0, 2);
    cov[3] = SIG(1, 1);
    cov[4] = SIG(1, 2);
    cov[5] = SIG(2, 2);
#undef SIG
}

/* computeCov2D with glm.  Outputs as cov2d(): the clamped t, the T = W J columns 0/1 in A (the
 * 2x3 the preprocess backward uses: A[c][k] = T[c][k]) and abc = (a + 0.3, b, c + 0.3). */
static void u_cov2d(int f, const float* mean, float fx, float fy, float tanfovx, float tanfovy, const float* cov,
                    const float* view, float* t, float A[2][3], float* abc, float* txtz_out, float* tytz_out)
{
    u_xform4x3(f, view, mean, t);
    const float limx = 1.3f * tanfovx, limy = 1.3f * tanfovy;
    const float txtz = t[0] / t[2], tytz = t[1] / t[2];
    t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
    t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
    const float j00 = fx / t[2], j02 = -(fx * t[0]) / (t[2] * t[2]);
    const float j11 = fy / t[2], j12 = -(fy * t[1]) / (t[2] * t[2]);
    /* W[c][r] = view[4 r + c]; T[c][r] = W[0][r] J[c][0] + W[1][r] J[c][1] + W[2][r] J[c][2] with
       J[0] = (j00, 0, j02), J[1] = (0, j11, j12): the zero product adds +-0 to the first nonzero
       one, and the last product is the one contracted into the sum */
    for (int r = 0; r < 3; r++) {
        A[0][r] = u_addp(f, view[4 * r] * j00, view[4 * r + 2], j02);
        A[1][r] = u_addp(f, view[4 * r + 1] * j11, view[4 * r + 2], j12);
    }
    const float V[3][3] = {{cov[0], cov[1], cov[2]}, {cov[1], cov[3], cov[4]}, {cov[2], cov[4], cov[5]}};
    /* X = T^T V: X[k][r] = sum_j T[r][j] V[k][j];  cov2D[c][r] = sum_k X[k][r] T[c][k] */
    float X0[3], X1[3];
    for (int k = 0; k < 3; k++) {
        X0[k] = u_sum3(f, A[0][0], V[k][0], A[0][1], V[k][1], A[0][2], V[k][2]);
        X1[k] = u_sum3(f, A[1][0], V[k][0], A[1][1], V[k][1], A[1][2], V[k][2]);
    }
    abc[0] = u_sum3(f, X0[0], A[0][0], X0[1], A[0][1], X0[2], A[0][2]) + 0.3f;
    abc[1] = u_sum3(f, X1[0], A[0][0], X1[1], A[0][1], X1[2], A[0][2]);
    abc[2] = u_sum3(f, X1[0], A[1][0], X1[1], A[1][1], X1[2], A[1][2]) + 0.3f;
    if (txtz_out) *txtz_out = txtz;
    if (tytz_out) *tytz_out = tytz;
}

/* computeColorFromSH as written, including the + 0.5 (form 1: lso_sh_eval's sequence; form 2
 * contracted: at degree 0 the + 0.5 meets the product SH_C0 sh[0] itself, above it the first
 * subtraction does) */
static void u_sh_eval(int f, int deg, const float* sh, const float* mean, const float* campos, float* out)
{
    float d[3] = {mean[0] - campos[0], mean[1] - campos[1], mean[2] - campos[2]};
    const float len = sqrtf(u_sum3(f, d[0], d[0], d[1], d[1], d[2], d[2]));
    const float x = d[0] / len, y = d[1] / len, z = d[2] / len;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    for (int c = 0; c < 3; c++) {
        const float* s = sh + c;
        if (deg == 0) {
            out[c] = u_addp(f, 0.5f, SH_C0, s[0]);
            continue;
        }
        float res;
        {
            res = u_diffp(f, SH_C0, s[0], SH_C1 * y, s[1 * 3]);
            res = u_addp(f, res, SH_C1 * z, s[2 * 3]);
            res = u_subp(f, res, SH_C1 * x, s[3 * 3]);
            if (deg > 1) {
                res = u_addp(f, res, SH_C2[0] * xy, s[4 * 3]);
                res = u_addp(f, res, SH_C2[1] * yz, s[5 * 3]);
                res = u_addp(f, res, SH_C2[2] * (u_subp(f, -xx, -2.0f, zz) - yy), s[6 * 3]);
                res = u_addp(f, res, SH_C2[3] * xz, s[7 * 3]);
                res = u_addp(f, res, SH_C2[4] * (xx - yy), s[8 * 3]);
                if (deg > 2) {
                    res = u_addp(f, res, SH_C3[0] * y * u_subp(f, -yy, -3.0f, xx), s[9 * 3]);
                    res = u_addp(f, res, SH_C3[1] * xy * z, s[10 * 3]);
                    res = u_addp(f, res, SH_C3[2] * y * (u_subp(f, -xx, -4.0f, zz) - yy), s[11 * 3]);
                    res = u_addp(f, res, SH_C3[3] * z * u_subp(f, u_diffp(f, 2.0f, zz, 3.0f, xx), 3.0f, yy),
                                 s[12 * 3]);
                    res = u_addp(f, res, SH_C3[4] * x * (u_subp(f, -xx, -4.0f, zz) - yy), s[13 * 3]);
                    res = u_addp(f, res, SH_C3[5] * z * (xx - yy), s[14 * 3]);
                    res = u_addp(f, res, SH_C3[6] * x * u_subp(f, xx, 3.0f, yy), s[15 * 3]);
                }
            }
        }
        out[c] = res + 0.5f;
    }
}

/* renderCUDA's power as written: -0.5f * (c.x dx dx + c.z dy dy) - c.y dx dy */
static inline float u_power(int f, const float* co, float dx, float dy)
{
    const float inner = u_sum2(f, co[0] * dx, dx, co[2] * dy, dy);
    return u_diffp(f, -0.5f, inner, co[1] * dx, dy);
}

/* ------------------------------------------------------------------------------------------ */
/* SH -> RGB (utils/sh_utils.py:57-112; +0.5 and clamp as gaussian_renderer/__init__.py:80)   */
/* ------------------------------------------------------------------------------------------ */

void lso_sh_eval(int deg, const float* sh /* [K][3] */, const float* dir, float* out)
{
    float x = dir[0], y = dir[1], z = dir[2];
    for (int c = 0; c < 3; c++) {
        float res = SH_C0 * sh[0 * 3 + c];
        if (deg > 0) {
            res = res - (SH_C1 * y) * sh[1 * 3 + c];
            res = res + (SH_C1 * z) * sh[2 * 3 + c];
            res = res - (SH_C1 * x) * sh[3 * 3 + c];
            if (deg > 1) {
                float xx = x * x, yy = y * y, zz = z * z;
                float xy = x * y, yz = y * z, xz = x * z;
                res = res + (SH_C2[0] * xy) * sh[4 * 3 + c];
                res = res + (SH_C2[1] * yz) * sh[5 * 3 + c];
                res = res + (SH_C2[2] * (2.0f * zz - xx - yy)) * sh[6 * 3 + c];
                res = res + (SH_C2[3] * xz) * sh[7 * 3 + c];
                res = res + (SH_C2[4] * (xx - yy)) * sh[8 * 3 + c];
                if (deg > 2) {
                    res = res + (SH_C3[0] * y * (3.0f * xx - yy)) * sh[9 * 3 + c];
                    res = res + (SH_C3[1] * xy * z) * sh[10 * 3 + c];
                    res = res + (SH_C3[2] * y * (4.0f * zz - xx - yy)) * sh[11 * 3 + c];
                    res = res + (SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy)) * sh[12 * 3 + c];
                    res = res + (SH_C3[4] * x * (4.0f * zz - xx - yy)) * sh[13 * 3 + c];
                    res = res + (SH_C3[5] * z * (xx - yy)) * sh[14 * 3 + c];
                    res = res + (SH_C3[6] * x * (xx - 3.0f * yy)) * sh[15 * 3 + c];
                }
            }
        }
        out[c] = res;
    }
}

static void view_dir(const float* mean, const float* campos, float* dir_orig, float* dir)
{
    dir_orig[0] = mean[0] - campos[0];
    dir_orig[1] = mean[1] - campos[1];
    dir_orig[2] = mean[2] - campos[2];
    float len = sqrtf(DOT3(dir_orig, dir_orig));
    dir[0] = dir_orig[0] / len;
    dir[1] = dir_orig[1] / len;
    dir[2] = dir_orig[2] / len;
}

/* ------------------------------------------------------------------------------------------ */
/* forward                                                                                      */
/* ------------------------------------------------------------------------------------------ */

static void* xcopy(const void* src, size_t bytes)
{
    if (!src || bytes == 0) return NULL;
    void* d = malloc(bytes);
    memcpy(d, src, bytes);
    return d;
}

/* the per-Gaussian state's covariance inputs in the state's arithmetic form */
static void cov3d_of(const lso_state* st, int i, float* cov_local, const float** cov)
{
    if (st->has_cov) {
        *cov = st->cov_pre + 6 * i;
    } else if (st->form == LSO_FORM_KERNEL) {
        lso_cov3d(st->scales + 3 * i, st->s.scale_modifier, st->rots + 4 * i, cov_local);
        *cov = cov_local;
    } else {
        u_cov3d(st->form, st->scales + 3 * i, st->s.scale_modifier, st->rots + 4 * i, cov_local);
        *cov = cov_local;
    }
}

static void cov2d_of(const lso_state* st, const float* mean, float fx, float fy, const float* cov, float* t,
                     float A[2][3], float* abc, float* txtz, float* tytz)
{
    const lso_settings* s = &st->s;
    if (st->form == LSO_FORM_KERNEL)
        cov2d(mean, fx, fy, s->tanfovx, s->tanfovy, cov, s->viewmatrix, t, A, abc, txtz, tytz);
    else
        u_cov2d(st->form, mean, fx, fy, s->tanfovx, s->tanfovy, cov, s->viewmatrix, t, A, abc, txtz, tytz);
}

static void preprocess_one(lso_state* st, int i, float focal_x, float focal_y)
{
    const lso_settings* s = &st->s;
    const int W = s->image_width, H = s->image_height;
    const int f = st->form;
    st->radii[i] = 0;
    st->tiles[i] = 0;
    const float* p = st->means + 3 * i;
    float pv[3];
    if (f == LSO_FORM_KERNEL) xform4x3(s->viewmatrix, p, pv);
    else u_xform4x3(f, s->viewmatrix, p, pv);
    if (pv[2] <= 0.2f) return; /* near cull */
    float hom[4];
    if (f == LSO_FORM_KERNEL) xform4x4(s->projmatrix, p, hom);
    else u_xform4x4(f, s->projmatrix, p, hom);
    float p_w = 1.0f / (hom[3] + 0.0000001f);
    float proj_x = hom[0] * p_w, proj_y = hom[1] * p_w;

    float cov_local[6];
    const float* cov;
    cov3d_of(st, i, cov_local, &cov);
    float t[3], A[2][3], abc[3];
    cov2d_of(st, p, focal_x, focal_y, cov, t, A, abc, NULL, NULL);
    float a = abc[0], b = abc[1], c = abc[2];
    float det = f == LSO_FORM_KERNEL ? a * c - b * b : u_diffp(f, a, c, b, b);
    if (det == 0.0f) return;
    float det_inv = 1.f / det;
    float cx = c * det_inv, cy = -b * det_inv, cz = a * det_inv;
    float mid = 0.5f * (a + c);
    float disc = fmaxf(0.1f, f == LSO_FORM_KERNEL ? mid * mid - det : u_prodsub(f, mid, mid, det));
    float sq = sqrtf(disc);
    float l1 = mid + sq, l2 = mid - sq;
    float my_radius = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    float ix = ndc2pix(proj_x, W), iy = ndc2pix(proj_y, H);
    int r = (int)my_radius;
    int rminx = (int)((ix - (float)r) / (float)BLOCK_X);
    int rminy = (int)((iy - (float)r) / (float)BLOCK_Y);
    int rmaxx = (int)((ix + (float)r + (float)BLOCK_X - 1.0f) / (float)BLOCK_X);
    int rmaxy = (int)((iy + (float)r + (float)BLOCK_Y - 1.0f) / (float)BLOCK_Y);
    rminx = rminx < 0 ? 0 : (rminx > st->gx ? st->gx : rminx);
    rminy = rminy < 0 ? 0 : (rminy > st->gy ? st->gy : rminy);
    rmaxx = rmaxx < 0 ? 0 : (rmaxx > st->gx ? st->gx : rmaxx);
    rmaxy = rmaxy < 0 ? 0 : (rmaxy > st->gy ? st->gy : rmaxy);
    uint32_t area = (uint32_t)((rmaxx - rminx) * (rmaxy - rminy));
    if (area == 0) return;

    if (st->has_shs) {
        float dir_orig[3], dir[3], res[3];
        if (f == LSO_FORM_KERNEL) {
            view_dir(p, s->campos, dir_orig, dir);
            lso_sh_eval(s->sh_degree, st->shs + (size_t)i * st->M * 3, dir, res);
            for (int ch = 0; ch < 3; ch++) res[ch] = res[ch] + 0.5f;
        } else {
            u_sh_eval(f, s->sh_degree, st->shs + (size_t)i * st->M * 3, p, s->campos, res);
        }
        for (int ch = 0; ch < 3; ch++) {
            float v = res[ch];
            st->clamped[3 * i + ch] = v < 0.0f;
            st->rgb[3 * i + ch] = fmaxf(v, 0.0f);
        }
    } else {
        for (int ch = 0; ch < 3; ch++) st->rgb[3 * i + ch] = st->colors[3 * i + ch];
    }
    st->depth[i] = pv[2];
    st->radii[i] = r;
    st->xy[2 * i] = ix;
    st->xy[2 * i + 1] = iy;
    st->conic_o[4 * i + 0] = cx;
    st->conic_o[4 * i + 1] = cy;
    st->conic_o[4 * i + 2] = cz;
    st->conic_o[4 * i + 3] = st->opac[i];
    st->tiles[i] = area;
}

static void tile_rect(const lso_state* st, int i, int* r4)
{
    const float ix = st->xy[2 * i], iy = st->xy[2 * i + 1];
    int r = st->radii[i];
    int v[4] = {(int)((ix - (float)r) / (float)BLOCK_X), (int)((iy - (float)r) / (float)BLOCK_Y),
                (int)((ix + (float)r + (float)BLOCK_X - 1.0f) / (float)BLOCK_X),
                (int)((iy + (float)r + (float)BLOCK_Y - 1.0f) / (float)BLOCK_Y)};
    int lim[4] = {st->gx, st->gy, st->gx, st->gy};
    for (int k = 0; k < 4; k++) r4[k] = v[k] < 0 ? 0 : (v[k] > lim[k] ? lim[k] : v[k]);
}

/* Render one pixel front to back; returns the pixel's final T and contributor count. */
static void render_pixel(const lso_state* st, int tile, int px, int py, float* C, float* F,
                         float* T_out, uint32_t* last_out)
{
    const float pfx = (float)px, pfy = (float)py;
    float T = 1.0f;
    uint32_t contributor = 0, last = 0;
    C[0] = C[1] = C[2] = 0.f;
    F[0] = F[1] = F[2] = 0.f;
    for (uint32_t k = st->ranges[2 * tile]; k < st->ranges[2 * tile + 1]; k++) {
        contributor++;
        uint32_t g = st->point_list[k];
        const float* co = st->conic_o + 4 * g;
        float dx = st->xy[2 * g] - pfx, dy = st->xy[2 * g + 1] - pfy;
        float hx = -0.5f * co[0], hz = -0.5f * co[2];
        float power = fmaf(dx, fmaf(-co[1], dy, hx * dx), (hz * dy) * dy);
        if (power > 0.0f) continue;
        float alpha = fminf(0.99f, co[3] * lso_expf_render(power));
        if (alpha < 1.0f / 255.0f) continue;
        float test_T = T * (1.0f - alpha);
        if (test_T < 0.0001f) break; /* done: this Gaussian is not blended */
        float w = alpha * T;
        for (int ch = 0; ch < 3; ch++) C[ch] = fmaf(st->rgb[3 * g + ch], w, C[ch]);
        if (st->s.include_feature && st->has_lang)
            for (int ch = 0; ch < 3; ch++) F[ch] = fmaf(st->lang[3 * g + ch], w, F[ch]);
        T = test_T;
        last = contributor;
    }
    *T_out = T;
    *last_out = last;
}

/* render_pixel in an upstream form (see "Upstream forms") */
static void render_pixel_upstream(const lso_state* st, int tile, int px, int py, float* C, float* F,
                                  float* T_out, uint32_t* last_out)
{
    const int f = st->form;
    const float pfx = (float)px, pfy = (float)py;
    float T = 1.0f;
    uint32_t contributor = 0, last = 0;
    C[0] = C[1] = C[2] = 0.f;
    F[0] = F[1] = F[2] = 0.f;
    const int feat = st->s.include_feature && st->has_lang;
    for (uint32_t k = st->ranges[2 * tile]; k < st->ranges[2 * tile + 1]; k++) {
        contributor++;
        uint32_t g = st->point_list[k];
        const float* co = st->conic_o + 4 * g;
        const float dx = st->xy[2 * g] - pfx, dy = st->xy[2 * g + 1] - pfy;
        const float power = u_power(f, co, dx, dy);
        if (power > 0.0f) continue;
        const float alpha = fminf(0.99f, co[3] * u_exp(power));
        if (alpha < 1.0f / 255.0f) continue;
        const float test_T = T * (1 - alpha);
        if (test_T < 0.0001f) break;
        for (int ch = 0; ch < 3; ch++) C[ch] = u_addp(f, C[ch], st->rgb[3 * g + ch] * alpha, T);
        if (feat)
            for (int ch = 0; ch < 3; ch++) F[ch] = u_addp(f, F[ch], st->lang[3 * g + ch] * alpha, T);
        T = test_T;
        last = contributor;
    }
    *T_out = T;
    *last_out = last;
}

static int lso_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* threads the oracle's parallel loops use (OMP_NUM_THREADS; bench.py's cpu_baseline reports it) */
int lso_num_threads(void) { return lso_threads(); }

static int tile_inst_cmp(const void* a, const void* b)
{
    const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : (x > y);
}

lso_state* lso_forward(const lso_settings* s, int P, int M, const float* means3D,
                       const float* shs, const float* colors_precomp, const float* lang,
                       const float* opacities, const float* scales, const float* rotations,
                       const float* cov3D_precomp, float* out_color, float* out_lang,
                       int32_t* radii_out)
{
    lso_state* st = (lso_state*)calloc(1, sizeof(lso_state));
    st->s = *s;
    st->form = (s->form == LSO_FORM_UPSTREAM || s->form == LSO_FORM_UPSTREAM_FMA) ? s->form : LSO_FORM_KERNEL;
    st->P = P;
    st->M = M;
    const int W = s->image_width, H = s->image_height;
    st->gx = (W + BLOCK_X - 1) / BLOCK_X;
    st->gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    const int T_tiles = st->gx * st->gy;
    st->has_shs = shs != NULL;
    st->has_colors = colors_precomp != NULL;
    st->has_cov = cov3D_precomp != NULL;
    st->has_lang = lang != NULL;
    st->means = (float*)xcopy(means3D, sizeof(float) * 3 * (size_t)P);
    st->shs = (float*)xcopy(shs, sizeof(float) * 3 * (size_t)M * P);
    st->colors = (float*)xcopy(colors_precomp, sizeof(float) * 3 * (size_t)P);
    st->lang = (float*)xcopy(lang, sizeof(float) * 3 * (size_t)P);
    st->opac = (float*)xcopy(opacities, sizeof(float) * (size_t)P);
    st->scales = (float*)xcopy(scales, sizeof(float) * 3 * (size_t)P);
    st->rots = (float*)xcopy(rotations, sizeof(float) * 4 * (size_t)P);
    st->cov_pre = (float*)xcopy(cov3D_precomp, sizeof(float) * 6 * (size_t)P);
    st->depth = (float*)calloc((size_t)P + 1, sizeof(float));
    st->xy = (float*)calloc(2 * (size_t)P + 1, sizeof(float));
    st->conic_o = (float*)calloc(4 * (size_t)P + 1, sizeof(float));
    st->rgb = (float*)calloc(3 * (size_t)P + 1, sizeof(float));
    st->radii = (int32_t*)calloc((size_t)P + 1, sizeof(int32_t));
    st->tiles = (uint32_t*)calloc((size_t)P + 1, sizeof(uint32_t));
    st->clamped = (uint8_t*)calloc(3 * (size_t)P + 1, 1);
    st->ranges = (uint32_t*)calloc(2 * (size_t)T_tiles, sizeof(uint32_t));
    st->final_T = (float*)calloc((size_t)W * H, sizeof(float));
    st->n_contrib = (uint32_t*)calloc((size_t)W * H, sizeof(uint32_t));

    if (P == 0) { /* upstream skips everything: images stay zero (not background) */
        memset(out_color, 0, sizeof(float) * 3 * (size_t)W * H);
        memset(out_lang, 0, sizeof(float) * 3 * (size_t)W * H);
        return st;
    }

    const float focal_y = (float)H / (2.0f * s->tanfovy);
    const float focal_x = (float)W / (2.0f * s->tanfovx);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; i++) preprocess_one(st, i, focal_x, focal_y);
    memcpy(radii_out, st->radii, sizeof(int32_t) * (size_t)P);

    /* duplicate with keys (tile << 32 | depth bits) and sort (stable: equal keys keep id order),
       i.e. the (tile, depth, id) order: a counting sort by tile in id order, then each tile's run
       sorted on (depth bits << 32 | id) -- the same order as one sort of the 64-bit keys */
    int64_t R = 0;
    for (int i = 0; i < P; i++) R += st->tiles[i];
    st->R = R;
    uint32_t* tile_count = (uint32_t*)calloc((size_t)T_tiles + 1, sizeof(uint32_t));
    for (int i = 0; i < P; i++) {
        if (st->tiles[i] == 0) continue;
        int r4[4];
        tile_rect(st, i, r4);
        for (int y = r4[1]; y < r4[3]; y++)
            for (int x = r4[0]; x < r4[2]; x++) tile_count[y * st->gx + x]++;
    }
    int64_t acc = 0;
    for (int t = 0; t < T_tiles; t++) {
        st->ranges[2 * t] = (uint32_t)acc;
        acc += tile_count[t];
        st->ranges[2 * t + 1] = (uint32_t)acc;
        tile_count[t] = st->ranges[2 * t]; /* now the write cursor */
    }
    uint64_t* inst = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(R + 1));
    for (int i = 0; i < P; i++) {
        if (st->tiles[i] == 0) continue;
        int r4[4];
        tile_rect(st, i, r4);
        const uint64_t key = ((uint64_t)f2bits(st->depth[i]) << 32) | (uint32_t)i;
        for (int y = r4[1]; y < r4[3]; y++)
            for (int x = r4[0]; x < r4[2]; x++) inst[tile_count[y * st->gx + x]++] = key;
    }
    free(tile_count);
#pragma omp parallel for schedule(dynamic, 16)
    for (int t = 0; t < T_tiles; t++) {
        const uint32_t a = st->ranges[2 * t], b = st->ranges[2 * t + 1];
        if (b - a > 1) qsort(inst + a, b - a, sizeof(uint64_t), tile_inst_cmp);
    }
    st->point_list = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(R + 1));
    for (int64_t k = 0; k < R; k++) st->point_list[k] = (uint32_t)inst[k];
    free(inst);

    const size_t HW = (size_t)W * H;
    const int upstream = st->form != LSO_FORM_KERNEL;
#pragma omp parallel for schedule(dynamic, 4)
    for (int tile = 0; tile < T_tiles; tile++) {
        const int ty = tile / st->gx, tx = tile % st->gx;
        for (int py = ty * BLOCK_Y; py < ty * BLOCK_Y + BLOCK_Y && py < H; py++)
            for (int px = tx * BLOCK_X; px < tx * BLOCK_X + BLOCK_X && px < W; px++) {
                float C[3], F[3], T;
                uint32_t last;
                if (upstream) render_pixel_upstream(st, tile, px, py, C, F, &T, &last);
                else render_pixel(st, tile, px, py, C, F, &T, &last);
                size_t pix = (size_t)py * W + px;
                st->final_T[pix] = T;
                st->n_contrib[pix] = last;
                for (int ch = 0; ch < 3; ch++) {
                    out_color[ch * HW + pix] = upstream ? u_addp(st->form, C[ch], T, s->bg[ch])
                                                        : fmaf(T, s->bg[ch], C[ch]);
                    out_lang[ch * HW + pix] = F[ch];
                }
            }
    }
    return st;
}

/* ------------------------------------------------------------------------------------------ */
/* backward                                                                                     */
/* ------------------------------------------------------------------------------------------ */

/* d normalize(v) / dv applied to dv (upstream dnormvdv) */
static void dnormvdv(const float* v, const float* dv, float* out)
{
    float sum2 = DOT3(v, v);
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    out[0] = ((sum2 - v[0] * v[0]) * dv[0] - v[1] * v[0] * dv[1] - v[2] * v[0] * dv[2]) * invsum32;
    out[1] = (-v[0] * v[1] * dv[0] + (sum2 - v[1] * v[1]) * dv[1] - v[2] * v[1] * dv[2]) * invsum32;
    out[2] = (-v[0] * v[2] * dv[0] - v[1] * v[2] * dv[1] + (sum2 - v[2] * v[2]) * dv[2]) * invsum32;
}

/* SH backward: dL/dsh (all M coefficients written, zeros above the active degree) and the
 * view-direction contribution to dL/dmean.  dL_drgb is already masked by the clamp flags. */
void lso_sh_backward(int deg, int M, const float* sh, const float* dir_orig,
                     const float* dL_drgb, float* dL_dsh, float* dL_dmean)
{
    float len = sqrtf(DOT3(dir_orig, dir_orig));
    float x = dir_orig[0] / len, y = dir_orig[1] / len, z = dir_orig[2] / len;
    float basis[16];
    float dx[3] = {0, 0, 0}, dy[3] = {0, 0, 0}, dz[3] = {0, 0, 0}; /* dRGB/d(dir) per channel */
    int K = (deg + 1) * (deg + 1);
    basis[0] = SH_C0;
    if (deg > 0) {
        basis[1] = -SH_C1 * y;
        basis[2] = SH_C1 * z;
        basis[3] = -SH_C1 * x;
        for (int c = 0; c < 3; c++) {
            dx[c] = -SH_C1 * sh[3 * 3 + c];
            dy[c] = -SH_C1 * sh[1 * 3 + c];
            dz[c] = SH_C1 * sh[2 * 3 + c];
        }
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z;
            float xy = x * y, yz = y * z, xz = x * z;
            basis[4] = SH_C2[0] * xy;
            basis[5] = SH_C2[1] * yz;
            basis[6] = SH_C2[2] * (2.f * zz - xx - yy);
            basis[7] = SH_C2[3] * xz;
            basis[8] = SH_C2[4] * (xx - yy);
            for (int c = 0; c < 3; c++) {
                const float* s = sh + c;
                dx[c] = dx[c] + (SH_C2[0] * y * s[4 * 3] + SH_C2[2] * 2.f * -x * s[6 * 3] +
                                 SH_C2[3] * z * s[7 * 3] + SH_C2[4] * 2.f * x * s[8 * 3]);
                dy[c] = dy[c] + (SH_C2[0] * x * s[4 * 3] + SH_C2[1] * z * s[5 * 3] +
                                 SH_C2[2] * 2.f * -y * s[6 * 3] + SH_C2[4] * 2.f * -y * s[8 * 3]);
                dz[c] = dz[c] + (SH_C2[1] * y * s[5 * 3] + SH_C2[2] * 2.f * 2.f * z * s[6 * 3] +
                                 SH_C2[3] * x * s[7 * 3]);
            }
            if (deg > 2) {
                basis[9] = SH_C3[0] * y * (3.f * xx - yy);
                basis[10] = SH_C3[1] * xy * z;
                basis[11] = SH_C3[2] * y * (4.f * zz - xx - yy);
                basis[12] = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
                basis[13] = SH_C3[4] * x * (4.f * zz - xx - yy);
                basis[14] = SH_C3[5] * z * (xx - yy);
                basis[15] = SH_C3[6] * x * (xx - 3.f * yy);
                for (int c = 0; c < 3; c++) {
                    const float* s = sh + c;
                    dx[c] = dx[c] + (SH_C3[0] * s[9 * 3] * 3.f * 2.f * xy + SH_C3[1] * s[10 * 3] * yz +
                                     SH_C3[2] * s[11 * 3] * -2.f * xy +
                                     SH_C3[3] * s[12 * 3] * -3.f * 2.f * xz +
                                     SH_C3[4] * s[13 * 3] * (-3.f * xx + 4.f * zz - yy) +
                                     SH_C3[5] * s[14 * 3] * 2.f * xz +
                                     SH_C3[6] * s[15 * 3] * 3.f * (xx - yy));
                    dy[c] = dy[c] + (SH_C3[0] * s[9 * 3] * 3.f * (xx - yy) + SH_C3[1] * s[10 * 3] * xz +
                                     SH_C3[2] * s[11 * 3] * (-3.f * yy + 4.f * zz - xx) +
                                     SH_C3[3] * s[12 * 3] * -3.f * 2.f * yz +
                                     SH_C3[4] * s[13 * 3] * -2.f * xy +
                                     SH_C3[5] * s[14 * 3] * -2.f * yz +
                                     SH_C3[6] * s[15 * 3] * -3.f * 2.f * xy);
                    dz[c] = dz[c] + (SH_C3[1] * s[10 * 3] * xy + SH_C3[2] * s[11 * 3] * 4.f * 2.f * yz +
                                     SH_C3[3] * s[12 * 3] * 3.f * (2.f * zz - xx - yy) +
                                     SH_C3[4] * s[13 * 3] * 4.f * 2.f * xz +
                                     SH_C3[5] * s[14 * 3] * (xx - yy));
                }
            }
        }
    }
    for (int k = 0; k < M; k++)
        for (int c = 0; c < 3; c++) dL_dsh[3 * k + c] = k < K ? basis[k] * dL_drgb[c] : 0.0f;
    float dL_ddir[3] = {DOT3(dx, dL_drgb), DOT3(dy, dL_drgb), DOT3(dz, dL_drgb)};
    dnormvdv(dir_orig, dL_ddir, dL_dmean);
}

/* Covariance backward: dL/dSigma (packed 6) -> dL/dscale, dL/drot (unnormalised quaternion,
 * no normalisation backward: autograd of F.normalize handles it). */
void lso_cov3d_backward(const float* scale, float mod, const float* rot, const float* dcov,
                        float* dscale, float* drot)
{
    float R[3][3], M[3][3];
    float s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    quat_to_rot(rot, R);
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) M[i][k] = R[i][k] * s[k];
    /* Sigma = M M^T with M = R diag(s);  dL/dM = 2 * dSym * M,  dSym with halved off-diagonals */
    float D[3][3] = {{dcov[0], 0.5f * dcov[1], 0.5f * dcov[2]},
                     {0.5f * dcov[1], dcov[3], 0.5f * dcov[4]},
                     {0.5f * dcov[2], 0.5f * dcov[4], dcov[5]}};
    float G[3][3]; /* dL/dM */
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++)
            G[i][k] = 2.0f * fmaf(D[i][2], M[2][k], fmaf(D[i][1], M[1][k], D[i][0] * M[0][k]));
    /* dL/ds_k = sum_i G[i][k] R[i][k] */
    for (int k = 0; k < 3; k++)
        dscale[k] = fmaf(G[2][k], R[2][k], fmaf(G[1][k], R[1][k], G[0][k] * R[0][k]));
    /* dL/dR[i][k] = G[i][k] s_k */
    float dR[3][3];
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) dR[i][k] = G[i][k] * s[k];
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    drot[0] = 2.f * z * (dR[1][0] - dR[0][1]) + 2.f * y * (dR[0][2] - dR[2][0]) +
              2.f * x * (dR[2][1] - dR[1][2]);
    drot[1] = 2.f * y * (dR[0][1] + dR[1][0]) + 2.f * z * (dR[0][2] + dR[2][0]) +
              2.f * r * (dR[2][1] - dR[1][2]) - 4.f * x * (dR[2][2] + dR[1][1]);
    drot[2] = 2.f * x * (dR[0][1] + dR[1][0]) + 2.f * r * (dR[0][2] - dR[2][0]) +
              2.f * z * (dR[2][1] + dR[1][2]) - 4.f * y * (dR[2][2] + dR[0][0]);
    drot[3] = 2.f * r * (dR[1][0] - dR[0][1]) + 2.f * x * (dR[0][2] + dR[2][0]) +
              2.f * y * (dR[2][1] + dR[1][2]) - 4.f * z * (dR[1][1] + dR[0][0]);
}

/* Per-pixel backward contributions, back to front (upstream BACKWARD::renderCUDA).  g holds 12
 * doubles per Gaussian: dxy 0-1, dconic 2-4, dopacity 5, drgb 6-8, dlang 9-11.  Forms 1 and 2
 * evaluate upstream's power, G = exp(power) and sums as written ("Upstream forms"). */
static void backward_pixel(const lso_state* st, int tile, int px, int py, const float* dpix,
                           const float* dpixF, double* gacc)
{
    const lso_settings* s = &st->s;
    const int W = s->image_width, H = s->image_height;
    const int form = st->form;
    const int up = form != LSO_FORM_KERNEL;
    const size_t pix = (size_t)py * W + px;
    const float T_final = st->final_T[pix];
    float T = T_final;
    const uint32_t last = st->n_contrib[pix];
    const float pfx = (float)px, pfy = (float)py;
    const float ddelx_dx = 0.5f * (float)W, ddely_dy = 0.5f * (float)H;
    const int feat = s->include_feature && st->has_lang;
    float acc[3] = {0, 0, 0}, accF[3] = {0, 0, 0}, last_c[3] = {0, 0, 0}, last_f[3] = {0, 0, 0};
    float last_alpha = 0.0f;
    float bg_dot = up ? u_addp(form, u_addp(form, u_addp(form, 0.0f, s->bg[0], dpix[0]), s->bg[1], dpix[1]),
                               s->bg[2], dpix[2])
                      : fmaf(s->bg[2], dpix[2], fmaf(s->bg[1], dpix[1], s->bg[0] * dpix[0]));
    const uint32_t start = st->ranges[2 * tile];
    for (int64_t j = (int64_t)last - 1; j >= 0; j--) {
        uint32_t g = st->point_list[start + j];
        double* ga = gacc + 12 * (size_t)g;
        const float* co = st->conic_o + 4 * g;
        float dx = st->xy[2 * g] - pfx, dy = st->xy[2 * g + 1] - pfy;
        float power, G;
        if (up) {
            power = u_power(form, co, dx, dy);
            if (power > 0.0f) continue;
            G = u_exp(power);
        } else {
            float hx = -0.5f * co[0], hz = -0.5f * co[2];
            power = fmaf(dx, fmaf(-co[1], dy, hx * dx), (hz * dy) * dy);
            if (power > 0.0f) continue;
            G = lso_expf_render(power);
        }
        float alpha = fminf(0.99f, co[3] * G);
        if (alpha < 1.0f / 255.0f) continue;
        float one_m = 1.0f - alpha;
        T = T / one_m;
        float dchannel_dcolor = alpha * T;
        float dL_dalpha = 0.0f;
        float oml = 1.0f - last_alpha;
        for (int ch = 0; ch < 3; ch++) {
            float c = st->rgb[3 * g + ch];
            acc[ch] = up ? u_sum2(form, last_alpha, last_c[ch], oml, acc[ch])
                         : fmaf(last_alpha, last_c[ch], oml * acc[ch]);
            last_c[ch] = c;
            dL_dalpha = up ? u_addp(form, dL_dalpha, c - acc[ch], dpix[ch]) : fmaf(c - acc[ch], dpix[ch], dL_dalpha);
            ga[6 + ch] += (double)(dchannel_dcolor * dpix[ch]);
        }
        if (feat) {
            for (int ch = 0; ch < 3; ch++) {
                float f = st->lang[3 * g + ch];
                accF[ch] = up ? u_sum2(form, last_alpha, last_f[ch], oml, accF[ch])
                              : fmaf(last_alpha, last_f[ch], oml * accF[ch]);
                last_f[ch] = f;
                dL_dalpha = up ? u_addp(form, dL_dalpha, f - accF[ch], dpixF[ch])
                               : fmaf(f - accF[ch], dpixF[ch], dL_dalpha);
                ga[9 + ch] += (double)(dchannel_dcolor * dpixF[ch]);
            }
        }
        dL_dalpha = dL_dalpha * T;
        last_alpha = alpha;
        dL_dalpha = up ? u_addp(form, dL_dalpha, -T_final / one_m, bg_dot) : fmaf(-T_final / one_m, bg_dot, dL_dalpha);
        float dL_dG = co[3] * dL_dalpha;
        float gdx = G * dx, gdy = G * dy;
        float dG_ddelx = up ? u_diffp(form, -gdx, co[0], gdy, co[1]) : -gdx * co[0] - gdy * co[1];
        float dG_ddely = up ? u_diffp(form, -gdy, co[2], gdx, co[1]) : -gdy * co[2] - gdx * co[1];
        ga[0] += (double)(dL_dG * dG_ddelx * ddelx_dx);
        ga[1] += (double)(dL_dG * dG_ddely * ddely_dy);
        ga[2] += (double)(-0.5f * gdx * dx * dL_dG);
        ga[3] += (double)(-0.5f * gdx * dy * dL_dG);
        ga[4] += (double)(-0.5f * gdy * dy * dL_dG);
        ga[5] += (double)(G * dL_dalpha);
    }
}

/* Per-Gaussian backward (upstream computeCov2DCUDA + preprocessCUDA backward). */
static void preprocess_backward_one(const lso_state* st, int i, float focal_x, float focal_y,
                                    const float* dxy, const float* dconic, const float* drgb_in,
                                    float* dL_dmeans, float* dL_dcov_out, float* dL_dsh,
                                    float* dL_dscale, float* dL_drot)
{
    const lso_settings* s = &st->s;
    const float* p = st->means + 3 * i;
    /* ---- cov2D backward ---- */
    float cov_local[6];
    const float* cov;
    cov3d_of(st, i, cov_local, &cov);
    float t[3], A[2][3], abc[3], txtz, tytz;
    cov2d_of(st, p, focal_x, focal_y, cov, t, A, abc, &txtz, &tytz);
    const float limx = 1.3f * s->tanfovx, limy = 1.3f * s->tanfovy;
    const float x_grad_mul = (txtz < -limx || txtz > limx) ? 0.0f : 1.0f;
    const float y_grad_mul = (tytz < -limy || tytz > limy) ? 0.0f : 1.0f;
    const float a = abc[0], b = abc[1], c = abc[2];
    const float dcx = dconic[0], dcy = dconic[1], dcz = dconic[2];
    float denom = a * c - b * b;
    float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
    float denom2inv = 1.0f / (denom * denom + 0.0000001f);
    float dcov[6] = {0, 0, 0, 0, 0, 0};
    if (denom2inv != 0.0f) {
        dL_da = denom2inv * (-c * c * dcx + 2.f * b * c * dcy + (denom - a * c) * dcz);
        dL_dc = denom2inv * (-a * a * dcz + 2.f * a * b * dcy + (denom - a * c) * dcx);
        dL_db = denom2inv * 2.f * (b * c * dcx - (denom + 2.f * b * b) * dcy + a * b * dcz);
        /* dcov2D/dSigma for a = A0 S A0^T, b = A0 S A1^T, c = A1 S A1^T */
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
    for (int k = 0; k < 3; k++) {
        SA0[k] = DOT3(A[0], S[k]);
        SA1[k] = DOT3(A[1], S[k]);
    }
    float dA[2][3];
    for (int k = 0; k < 3; k++) {
        dA[0][k] = 2.f * SA0[k] * dL_da + SA1[k] * dL_db;
        dA[1][k] = 2.f * SA1[k] * dL_dc + SA0[k] * dL_db;
    }
    const float* v = s->viewmatrix;
    /* A0 = j00 W0 + j02 W2;  A1 = j11 W1 + j12 W2, W_r[k] = v[4k + r] */
    float dJ00 = fmaf(v[8], dA[0][2], fmaf(v[4], dA[0][1], v[0] * dA[0][0]));
    float dJ02 = fmaf(v[10], dA[0][2], fmaf(v[6], dA[0][1], v[2] * dA[0][0]));
    float dJ11 = fmaf(v[9], dA[1][2], fmaf(v[5], dA[1][1], v[1] * dA[1][0]));
    float dJ12 = fmaf(v[10], dA[1][2], fmaf(v[6], dA[1][1], v[2] * dA[1][0]));
    float tz = 1.f / t[2];
    float tz2 = tz * tz;
    float tz3 = tz2 * tz;
    float dtx = x_grad_mul * -focal_x * tz2 * dJ02;
    float dty = y_grad_mul * -focal_y * tz2 * dJ12;
    float dtz = -focal_x * tz2 * dJ00 - focal_y * tz2 * dJ11 + (2.f * focal_x * t[0]) * tz3 * dJ02 +
                (2.f * focal_y * t[1]) * tz3 * dJ12;
    float dmean[3];
    dmean[0] = fmaf(v[2], dtz, fmaf(v[1], dty, v[0] * dtx));
    dmean[1] = fmaf(v[6], dtz, fmaf(v[5], dty, v[4] * dtx));
    dmean[2] = fmaf(v[10], dtz, fmaf(v[9], dty, v[8] * dtx));

    /* ---- screen-space mean backward ---- */
    const float* m = s->projmatrix;
    float hom[4];
    if (st->form == LSO_FORM_KERNEL) xform4x4(m, p, hom);
    else u_xform4x4(st->form, m, p, hom);
    float m_w = 1.0f / (hom[3] + 0.0000001f);
    float mul1 = hom[0] * m_w * m_w;
    float mul2 = hom[1] * m_w * m_w;
    float gx = dxy[0], gy = dxy[1];
    dmean[0] += (m[0] * m_w - m[3] * mul1) * gx + (m[1] * m_w - m[3] * mul2) * gy;
    dmean[1] += (m[4] * m_w - m[7] * mul1) * gx + (m[5] * m_w - m[7] * mul2) * gy;
    dmean[2] += (m[8] * m_w - m[11] * mul1) * gx + (m[9] * m_w - m[11] * mul2) * gy;

    /* ---- SH backward ---- */
    if (st->has_shs) {
        float drgb[3];
        for (int ch = 0; ch < 3; ch++) drgb[ch] = st->clamped[3 * i + ch] ? 0.0f : drgb_in[ch];
        float dir_orig[3] = {p[0] - s->campos[0], p[1] - s->campos[1], p[2] - s->campos[2]};
        float dm_sh[3];
        lso_sh_backward(s->sh_degree, st->M, st->shs + (size_t)i * st->M * 3, dir_orig, drgb,
                        dL_dsh + (size_t)i * st->M * 3, dm_sh);
        for (int k = 0; k < 3; k++) dmean[k] += dm_sh[k];
    }
    for (int k = 0; k < 3; k++) dL_dmeans[3 * i + k] = dmean[k];
    if (dL_dcov_out)
        for (int k = 0; k < 6; k++) dL_dcov_out[6 * i + k] = dcov[k];
    if (!st->has_cov)
        lso_cov3d_backward(st->scales + 3 * i, s->scale_modifier, st->rots + 4 * i, dcov,
                           dL_dscale + 3 * i, dL_drot + 4 * i);
}

/* Outputs are fully written (zeros for culled Gaussians).  Optional outputs may be NULL:
 * dL_dsh when no SH, dL_dscales/dL_drot when cov3D was precomputed. */
void lso_backward(const lso_state* st, const float* dL_dcolor, const float* dL_dlang,
                  float* dL_dmeans2D, float* dL_dcolors, float* dL_dlang_out, float* dL_dopacity,
                  float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales,
                  float* dL_drot)
{
    const lso_settings* s = &st->s;
    const int P = st->P, W = s->image_width, H = s->image_height;
    const size_t HW = (size_t)W * H;
    memset(dL_dmeans2D, 0, sizeof(float) * 3 * (size_t)P);
    memset(dL_dcolors, 0, sizeof(float) * 3 * (size_t)P);
    memset(dL_dlang_out, 0, sizeof(float) * 3 * (size_t)P);
    memset(dL_dopacity, 0, sizeof(float) * (size_t)P);
    memset(dL_dmeans3D, 0, sizeof(float) * 3 * (size_t)P);
    if (dL_dcov3D) memset(dL_dcov3D, 0, sizeof(float) * 6 * (size_t)P);
    if (dL_dsh) memset(dL_dsh, 0, sizeof(float) * 3 * (size_t)st->M * P);
    if (dL_dscales) memset(dL_dscales, 0, sizeof(float) * 3 * (size_t)P);
    if (dL_drot) memset(dL_drot, 0, sizeof(float) * 4 * (size_t)P);
    if (P == 0) return;

    /* per-thread accumulators (12 doubles per Gaussian), tiles dealt round-robin (a fixed
       assignment for a given thread count), then summed over threads in thread order */
    const int nth = lso_threads();
    double* gacc = (double*)calloc((size_t)nth * 12 * (size_t)P, sizeof(double));
    const int T_tiles = st->gx * st->gy;
#pragma omp parallel for schedule(static, 1) num_threads(nth)
    for (int tile = 0; tile < T_tiles; tile++) {
#ifdef _OPENMP
        double* mine = gacc + (size_t)omp_get_thread_num() * 12 * (size_t)P;
#else
        double* mine = gacc;
#endif
        const int ty = tile / st->gx, tx = tile % st->gx;
        for (int py = ty * BLOCK_Y; py < ty * BLOCK_Y + BLOCK_Y && py < H; py++)
            for (int px = tx * BLOCK_X; px < tx * BLOCK_X + BLOCK_X && px < W; px++) {
                size_t pix = (size_t)py * W + px;
                float dpix[3] = {dL_dcolor[pix], dL_dcolor[HW + pix], dL_dcolor[2 * HW + pix]};
                float dpixF[3] = {0, 0, 0};
                if (dL_dlang) {
                    dpixF[0] = dL_dlang[pix];
                    dpixF[1] = dL_dlang[HW + pix];
                    dpixF[2] = dL_dlang[2 * HW + pix];
                }
                backward_pixel(st, tile, px, py, dpix, dpixF, mine);
            }
    }
    const float focal_y = (float)H / (2.0f * s->tanfovy);
    const float focal_x = (float)W / (2.0f * s->tanfovx);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; i++) {
        if (!(st->radii[i] > 0)) continue;
        double gsum[12];
        for (int k = 0; k < 12; k++) gsum[k] = gacc[12 * (size_t)i + k];
        for (int t = 1; t < nth; t++)
            for (int k = 0; k < 12; k++) gsum[k] += gacc[((size_t)t * P + i) * 12 + k];
        float dxy[2] = {(float)gsum[0], (float)gsum[1]};
        float dconic[3] = {(float)gsum[2], (float)gsum[3], (float)gsum[4]};
        float drgb[3] = {(float)gsum[6], (float)gsum[7], (float)gsum[8]};
        dL_dmeans2D[3 * i] = dxy[0];
        dL_dmeans2D[3 * i + 1] = dxy[1];
        for (int ch = 0; ch < 3; ch++) {
            dL_dcolors[3 * i + ch] = drgb[ch];
            dL_dlang_out[3 * i + ch] = (float)gsum[9 + ch];
        }
        dL_dopacity[i] = (float)gsum[5];
        preprocess_backward_one(st, i, focal_x, focal_y, dxy, dconic, drgb, dL_dmeans3D, dL_dcov3D,
                                dL_dsh, dL_dscales, dL_drot);
    }
    free(gacc);
}

/* ------------------------------------------------------------------------------------------ */
/* state accessors (for tests)                                                                  */
/* ------------------------------------------------------------------------------------------ */
/* fused parameter activation (include/lsr.h lsr_raw_flags)                  */
/* ------------------------------------------------------------------------------------------ */
/* GaussianModel's activations (scene/gaussian_model.py:33-41 setup_functions; getters :134-161)
 * and the language normalisation (gaussian_renderer/__init__.py:87), restated with the same
 * operation order as the kernels (langsplat_amd/csrc/lsr_device.h act_*), so a fused GPU
 * forward is bit-identical to this activation followed by lso_forward.  Versus torch's own
 * sigmoid/exp/normalize these agree to a few ulp (tests/test_oracle_activation.py).  The
 * backward follows torch autograd's formulas: sigmoid_backward grad*(1-y)*y, exp grad*result,
 * and the composed div / clamp_min / norm backward of F.normalize. */
#define LSO_RAW_OPACITY 1
#define LSO_RAW_SCALES 2
#define LSO_RAW_ROTATIONS 4
#define LSO_RAW_LANGUAGE 8

float lso_act_expf(float x) { return x > 88.0f ? INFINITY : lso_expf(x); }
static float act_sigmoid(float x) { return 1.0f / (1.0f + lso_act_expf(-x)); }

/* Activates in place-free form: each non-NULL input (P rows) is written activated to its output. */
void lso_activate(int P, int raw, const float* opac, const float* scales, const float* rots, const float* lang,
                  float* opac_out, float* scales_out, float* rots_out, float* lang_out)
{
    for (int i = 0; i < P; i++) {
        if ((raw & LSO_RAW_OPACITY) && opac) opac_out[i] = act_sigmoid(opac[i]);
        if ((raw & LSO_RAW_SCALES) && scales)
            for (int k = 0; k < 3; k++) scales_out[3 * i + k] = lso_act_expf(scales[3 * i + k]);
        if ((raw & LSO_RAW_ROTATIONS) && rots) {
            const float* q = rots + 4 * i;
            const float d = fmaxf(sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]), 1e-12f);
            for (int k = 0; k < 4; k++) rots_out[4 * i + k] = q[k] / d;
        }
        if ((raw & LSO_RAW_LANGUAGE) && lang) {
            const float* f = lang + 3 * i;
            const float d = sqrtf(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]) + 1e-9f;
            for (int k = 0; k < 3; k++) lang_out[3 * i + k] = f[k] / d;
        }
    }
}

/* Gradients w.r.t. the activated tensors (g_*) -> gradients w.r.t. the raw inputs (d_*). */
void lso_activate_backward(int P, int raw, const float* opac, const float* scales, const float* rots,
                           const float* lang, const float* g_opac, const float* g_scales, const float* g_rots,
                           const float* g_lang, float* d_opac, float* d_scales, float* d_rots, float* d_lang)
{
    for (int i = 0; i < P; i++) {
        if ((raw & LSO_RAW_OPACITY) && opac) {
            const float y = act_sigmoid(opac[i]);
            d_opac[i] = g_opac[i] * (1.0f - y) * y;
        }
        if ((raw & LSO_RAW_SCALES) && scales)
            for (int k = 0; k < 3; k++) d_scales[3 * i + k] = g_scales[3 * i + k] * lso_act_expf(scales[3 * i + k]);
        if ((raw & LSO_RAW_ROTATIONS) && rots) {
            const float* q = rots + 4 * i;
            const float* g = g_rots + 4 * i;
            const float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
            const float d = fmaxf(n, 1e-12f);
            const float gd = -(g[0] * q[0] + g[1] * q[1] + g[2] * q[2] + g[3] * q[3]) / (d * d);
            const float kk = (n >= 1e-12f && n > 0.0f) ? gd / n : 0.0f;
            for (int k = 0; k < 4; k++) d_rots[4 * i + k] = g[k] / d + q[k] * kk;
        }
        if ((raw & LSO_RAW_LANGUAGE) && lang) {
            const float* f = lang + 3 * i;
            const float* g = g_lang + 3 * i;
            const float n = sqrtf(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
            const float d = n + 1e-9f;
            const float gd = -(g[0] * f[0] + g[1] * f[1] + g[2] * f[2]) / (d * d);
            const float kk = n > 0.0f ? gd / n : 0.0f;
            for (int k = 0; k < 3; k++) d_lang[3 * i + k] = g[k] / d + f[k] * kk;
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* distCUDA2 (simple-knn, scene/gaussian_model.py:20,180)                     */
/* ------------------------------------------------------------------------------------------ */
/* Brute force O(N^2): for each point, the 3 smallest squared distances to OTHER points (by
 * index), each fmaf(dz, dz, fmaf(dy, dy, dx * dx)), mean (d0 + d1 + d2) / 3 with d0 <= d1 <= d2;
 * missing neighbours (N < 4) are FLT_MAX -- simple-knn's published semantics (exact 3-NN). */
#include <float.h>
void lso_knn_mean_dist3(int64_t N, const float* pts, float* out)
{
    for (int64_t i = 0; i < N; i++) {
        float b0 = FLT_MAX, b1 = FLT_MAX, b2 = FLT_MAX;
        const float px = pts[3 * i], py = pts[3 * i + 1], pz = pts[3 * i + 2];
        for (int64_t j = 0; j < N; j++) {
            if (j == i) continue;
            const float dx = px - pts[3 * j], dy = py - pts[3 * j + 1], dz = pz - pts[3 * j + 2];
            const float d = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
            if (d < b2) {
                if (d < b1) {
                    b2 = b1;
                    if (d < b0) { b1 = b0; b0 = d; } else { b1 = d; }
                } else {
                    b2 = d;
                }
            }
        }
        out[i] = (b0 + b1 + b2) / 3.0f;
    }
}

/* ------------------------------------------------------------------------------------------ */

int64_t lso_num_rendered(const lso_state* st) { return st->R; }

/* Copies a named state array into dst (caller sizes it); returns bytes copied or -1. */
int64_t lso_get(const lso_state* st, const char* name, void* dst)
{
    const size_t P = (size_t)st->P, HW = (size_t)st->s.image_width * st->s.image_height;
    const size_t T = (size_t)st->gx * st->gy;
    const void* src = NULL;
    size_t bytes = 0;
    if (!strcmp(name, "depth")) { src = st->depth; bytes = 4 * P; }
    else if (!strcmp(name, "xy")) { src = st->xy; bytes = 8 * P; }
    else if (!strcmp(name, "conic_opacity")) { src = st->conic_o; bytes = 16 * P; }
    else if (!strcmp(name, "rgb")) { src = st->rgb; bytes = 12 * P; }
    else if (!strcmp(name, "tiles_touched")) { src = st->tiles; bytes = 4 * P; }
    else if (!strcmp(name, "clamped")) { src = st->clamped; bytes = 3 * P; }
    else if (!strcmp(name, "point_list")) { src = st->point_list; bytes = 4 * (size_t)st->R; }
    else if (!strcmp(name, "ranges")) { src = st->ranges; bytes = 8 * T; }
    else if (!strcmp(name, "final_T")) { src = st->final_T; bytes = 4 * HW; }
    else if (!strcmp(name, "n_contrib")) { src = st->n_contrib; bytes = 4 * HW; }
    else return -1;
    if (bytes && src) memcpy(dst, src, bytes);
    return (int64_t)bytes;
}

void lso_free(lso_state* st)
{
    if (!st) return;
    void* ptrs[] = {st->means, st->shs, st->colors, st->lang, st->opac, st->scales, st->rots,
                    st->cov_pre, st->depth, st->xy, st->conic_o, st->rgb, st->radii, st->tiles,
                    st->clamped, st->point_list, st->ranges, st->final_T, st->n_contrib};
    for (size_t k = 0; k < sizeof(ptrs) / sizeof(ptrs[0]); k++) free(ptrs[k]);
    free(st);
}
