// lsr_knn.hip -- distCUDA2: mean squared distance of every point to its 3 nearest other points
// (simple-knn, called at scene/gaussian_model.py:20,180 to initialise the
// Gaussian scales from the SfM point cloud).
//
// Exact 3-NN on a uniform grid, instead of simple-knn's Morton sort + box scan:
//   1. bounding box (per-block partials, one-workgroup final reduction);
//   2. grid of cubic cells sized for ~2 points per cell (at most 2N + 64 cells);
//   3. counting sort of the points by cell (cell counts, one scan, scatter);
//   4. one thread per point, in cell order (neighbouring threads search neighbouring cells):
//      shells of cells at Chebyshev distance r = 0, 1, 2, ... are scanned until the 3rd-best squared
//      distance is no larger than the squared distance from the point to the faces of the searched
//      cube -- every point outside that cube is at least that far, so the result is exact.
// Squared distances are fma(dz, dz, fma(dy, dy, dx * dx)); the mean is (d0 + d1 + d2) / 3 with
// d0 <= d1 <= d2 -- the operation order of oracle/lsr_oracle.c lso_knn_mean_dist3, so results are
// bit-identical to the brute-force oracle.  The point itself is excluded by index (duplicates of it
// count, at distance 0); with fewer than 4 points the missing neighbours are FLT_MAX, as upstream.
#include <float.h>

#include "lsr_internal.h"

namespace lsr {

constexpr int kKnnThreads = 256;

struct KnnGrid {
    float x0, y0, z0, h, inv_h;
    int nx, ny, nz;
};

__device__ __forceinline__ float knn_d2(float px, float py, float pz, float qx, float qy, float qz)
{
    const float dx = px - qx, dy = py - qy, dz = pz - qz;
    return fma_(dz, dz, fma_(dy, dy, dx * dx));
}

__device__ __forceinline__ void knn_insert(float d, float& b0, float& b1, float& b2)
{
    if (d < b2) {
        if (d < b1) {
            b2 = b1;
            if (d < b0) {
                b1 = b0;
                b0 = d;
            } else {
                b1 = d;
            }
        } else {
            b2 = d;
        }
    }
}

// per-block min/max of the coordinates -> partial[6 * block]
__global__ __launch_bounds__(kKnnThreads) void k_knn_bbox_partial(int64_t N, const float* __restrict__ pts,
                                                                  float* __restrict__ partial)
{
    __shared__ float red[6][kKnnThreads / 64];
    float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int64_t i = (int64_t)blockIdx.x * kKnnThreads + threadIdx.x; i < N; i += (int64_t)gridDim.x * kKnnThreads) {
        const float x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
        v[0] = fminf(v[0], x);
        v[1] = fminf(v[1], y);
        v[2] = fminf(v[2], z);
        v[3] = fmaxf(v[3], x);
        v[4] = fmaxf(v[4], y);
        v[5] = fmaxf(v[5], z);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const float w = __shfl_xor(v[k], o, 64);
            v[k] = k < 3 ? fminf(v[k], w) : fmaxf(v[k], w);
        }
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 6; k++) red[k][threadIdx.x >> 6] = v[k];
    __syncthreads();
    if (threadIdx.x < 6) {
        const int k = threadIdx.x;
        float r = red[k][0];
        for (int w = 1; w < kKnnThreads / 64; w++) r = k < 3 ? fminf(r, red[k][w]) : fmaxf(r, red[k][w]);
        partial[6 * blockIdx.x + k] = r;
    }
}

// one workgroup: final bounding box -> grid (cell size for ~2 points per cell, <= max_cells cells)
__global__ __launch_bounds__(64) void k_knn_grid(int nb, const float* __restrict__ partial, int64_t N, int64_t max_cells,
                                                 KnnGrid* __restrict__ grid)
{
    float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int b = threadIdx.x; b < nb; b += 64)
        for (int k = 0; k < 6; k++) v[k] = k < 3 ? fminf(v[k], partial[6 * b + k]) : fmaxf(v[k], partial[6 * b + k]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const float w = __shfl_xor(v[k], o, 64);
            v[k] = k < 3 ? fminf(v[k], w) : fmaxf(v[k], w);
        }
    if (threadIdx.x != 0) return;
    const double ex = (double)v[3] - v[0], ey = (double)v[4] - v[1], ez = (double)v[5] - v[2];
    double ext = fmax(ex, fmax(ey, ez));
    if (!(ext > 0.0)) ext = 1.0;  // all points coincide (or N == 0)
    // volume of the box with degenerate axes widened to 1% of the largest extent
    const double fx = fmax(ex, 0.01 * ext), fy = fmax(ey, 0.01 * ext), fz = fmax(ez, 0.01 * ext);
    double h = cbrt(fx * fy * fz / fmax(0.5 * (double)N, 1.0));
    int nx, ny, nz;
    for (;;) {
        nx = (int)fmin(ex / h + 1.0, 1048576.0);
        ny = (int)fmin(ey / h + 1.0, 1048576.0);
        nz = (int)fmin(ez / h + 1.0, 1048576.0);
        if ((double)nx * ny * nz <= (double)max_cells) break;
        h *= 1.26;
    }
    KnnGrid g;
    g.x0 = v[0];
    g.y0 = v[1];
    g.z0 = v[2];
    g.h = (float)h;
    g.inv_h = (float)(1.0 / h);
    g.nx = nx;
    g.ny = ny;
    g.nz = nz;
    *grid = g;
}

__device__ __forceinline__ int knn_axis_cell(float p, float p0, float inv_h, int n)
{
    const int c = (int)((p - p0) * inv_h);
    return c < 0 ? 0 : (c >= n ? n - 1 : c);
}

__global__ __launch_bounds__(kKnnThreads) void k_knn_cell(int64_t N, const float* __restrict__ pts,
                                                          const KnnGrid* __restrict__ gp, uint32_t* __restrict__ cell,
                                                          uint32_t* __restrict__ count)
{
    const int64_t i = (int64_t)blockIdx.x * kKnnThreads + threadIdx.x;
    if (i >= N) return;
    const KnnGrid g = *gp;
    const int cx = knn_axis_cell(pts[3 * i], g.x0, g.inv_h, g.nx);
    const int cy = knn_axis_cell(pts[3 * i + 1], g.y0, g.inv_h, g.ny);
    const int cz = knn_axis_cell(pts[3 * i + 2], g.z0, g.inv_h, g.nz);
    const uint32_t c = (uint32_t)((cz * g.ny + cy) * g.nx + cx);
    cell[i] = c;
    atomicAdd(&count[c], 1u);
}

// points in cell order (order inside a cell is arbitrary; the result does not depend on it)
__global__ __launch_bounds__(kKnnThreads) void k_knn_scatter(int64_t N, const float* __restrict__ pts,
                                                             const uint32_t* __restrict__ cell,
                                                             uint32_t* __restrict__ cursor,
                                                             float4* __restrict__ sorted)
{
    const int64_t i = (int64_t)blockIdx.x * kKnnThreads + threadIdx.x;
    if (i >= N) return;
    const uint32_t o = atomicAdd(&cursor[cell[i]], 1u);
    sorted[o] = make_float4(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2], __uint_as_float((uint32_t)i));
}

__global__ __launch_bounds__(kKnnThreads) void k_knn_search(int64_t N, const KnnGrid* __restrict__ gp,
                                                            const uint32_t* __restrict__ cell_start,
                                                            const float4* __restrict__ sorted,
                                                            float* __restrict__ out)
{
    const int64_t s = (int64_t)blockIdx.x * kKnnThreads + threadIdx.x;
    if (s >= N) return;
    const KnnGrid g = *gp;
    const float4 P = sorted[s];
    const uint32_t self = __float_as_uint(P.w);
    const int cx = knn_axis_cell(P.x, g.x0, g.inv_h, g.nx);
    const int cy = knn_axis_cell(P.y, g.y0, g.inv_h, g.ny);
    const int cz = knn_axis_cell(P.z, g.z0, g.inv_h, g.nz);
    float b0 = FLT_MAX, b1 = FLT_MAX, b2 = FLT_MAX;
    const int rmax = max(g.nx, max(g.ny, g.nz));
    auto visit = [&](int x, int y, int z) {
        const uint32_t c = (uint32_t)((z * g.ny + y) * g.nx + x);
        for (uint32_t k = cell_start[c]; k < cell_start[c + 1]; k++) {
            const float4 Q = sorted[k];
            if (__float_as_uint(Q.w) == self) continue;
            knn_insert(knn_d2(P.x, P.y, P.z, Q.x, Q.y, Q.z), b0, b1, b2);
        }
    };
    // absolute slack for the rounding of cell boundaries / assignment
    const float slack = 1e-3f * g.h + 1e-6f * (fabsf(P.x) + fabsf(P.y) + fabsf(P.z) + fabsf(g.x0) + fabsf(g.y0) +
                                               fabsf(g.z0));
    for (int r = 0; r <= rmax; r++) {
        const int z0 = max(cz - r, 0), z1 = min(cz + r, g.nz - 1);
        const int y0 = max(cy - r, 0), y1 = min(cy + r, g.ny - 1);
        for (int z = z0; z <= z1; z++)
            for (int y = y0; y <= y1; y++) {
                if (r == 0 || z == cz - r || z == cz + r || y == cy - r || y == cy + r) {
                    for (int x = max(cx - r, 0); x <= min(cx + r, g.nx - 1); x++) visit(x, y, z);
                } else {  // interior row of the shell: only its two end cells
                    if (cx - r >= 0) visit(cx - r, y, z);
                    if (cx + r < g.nx) visit(cx + r, y, z);
                }
            }
        // every point outside the cube of cells [c - r, c + r] is at least this far (cells are
        // clamped at the grid edge, so only the inner faces count)
        float m = FLT_MAX;
        if (cx - r > 0) m = fminf(m, P.x - (g.x0 + (float)(cx - r) * g.h));
        if (cx + r < g.nx - 1) m = fminf(m, (g.x0 + (float)(cx + r + 1) * g.h) - P.x);
        if (cy - r > 0) m = fminf(m, P.y - (g.y0 + (float)(cy - r) * g.h));
        if (cy + r < g.ny - 1) m = fminf(m, (g.y0 + (float)(cy + r + 1) * g.h) - P.y);
        if (cz - r > 0) m = fminf(m, P.z - (g.z0 + (float)(cz - r) * g.h));
        if (cz + r < g.nz - 1) m = fminf(m, (g.z0 + (float)(cz + r + 1) * g.h) - P.z);
        if (m == FLT_MAX) break;  // the cube covers the whole grid
        m -= slack;
        if (m > 0.0f && b2 <= m * m) break;
    }
    out[self] = (b0 + b1 + b2) / 3.0f;
}

size_t knn_scratch_bytes(int64_t N)
{
    const size_t n = (size_t)(N > 0 ? N : 1);
    const size_t cells = 2 * n + 64;
    const size_t nb = (n + kKnnThreads - 1) / kKnnThreads;
    const size_t pb = nb < 1024 ? nb : 1024;
    return align_up(sizeof(KnnGrid)) + align_up(4 * 6 * pb) + align_up(4 * n) + align_up(4 * (cells + 1)) +
           align_up(4 * (cells + 1)) + align_up(16 * n) + align_up(4 * scan_region_words((int64_t)cells + 1));
}

hipError_t launch_knn_mean_dist3(int64_t N, const float* pts, float* out, void* scratch, uint32_t* stall,
                                 hipStream_t s)
{
    if (N <= 0) return hipSuccess;
    const size_t n = (size_t)N;
    const int64_t cells = 2 * (int64_t)n + 64;
    const int nb = (int)((n + kKnnThreads - 1) / kKnnThreads);
    const int pb = nb < 1024 ? nb : 1024;
    char* p = static_cast<char*>(scratch);
    size_t o = 0;
    auto take = [&](size_t bytes) { char* r = p + o; o += align_up(bytes); return r; };
    KnnGrid* grid = reinterpret_cast<KnnGrid*>(take(sizeof(KnnGrid)));
    float* partial = reinterpret_cast<float*>(take(4 * 6 * (size_t)pb));
    uint32_t* cell = reinterpret_cast<uint32_t*>(take(4 * n));
    uint32_t* count = reinterpret_cast<uint32_t*>(take(4 * ((size_t)cells + 1)));
    uint32_t* start = reinterpret_cast<uint32_t*>(take(4 * ((size_t)cells + 1)));
    float4* sorted = reinterpret_cast<float4*>(take(16 * n));
    uint32_t* region = reinterpret_cast<uint32_t*>(take(4 * scan_region_words(cells + 1)));
    hipError_t e;
    if ((e = hipMemsetAsync(count, 0, 4 * ((size_t)cells + 1), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(region, 0, 4 * scan_region_words(cells + 1), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_knn_bbox_partial, dim3(pb), dim3(kKnnThreads), 0, s, N, pts, partial);
    hipLaunchKernelGGL(k_knn_grid, dim3(1), dim3(64), 0, s, pb, (const float*)partial, N, cells, grid);
    hipLaunchKernelGGL(k_knn_cell, dim3(nb), dim3(kKnnThreads), 0, s, N, pts, (const KnnGrid*)grid, cell, count);
    if ((e = scan_exclusive_u32(count, start, (int)(cells + 1), region, stall, s)) != hipSuccess) return e;
    // the scatter advances a copy of the cell starts as per-cell cursors
    if ((e = hipMemcpyAsync(count, start, 4 * ((size_t)cells + 1), hipMemcpyDeviceToDevice, s)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(k_knn_scatter, dim3(nb), dim3(kKnnThreads), 0, s, N, pts, (const uint32_t*)cell, count, sorted);
    hipLaunchKernelGGL(k_knn_search, dim3(nb), dim3(kKnnThreads), 0, s, N, (const KnnGrid*)grid,
                       (const uint32_t*)start, (const float4*)sorted, out);
    return hipGetLastError();
}

}  // namespace lsr
