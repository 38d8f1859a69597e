// lsr_internal.h -- buffer layout and kernel launchers shared by the liblsr.so translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/lsr.h"
#include "lsr_device.h"

namespace lsr {

// counters[] slots in the image buffer
enum Counter : int {
    kCntVisible = 0,
    kCntRendered = 1,
    kCntError = 2,
    kCntOversize = 3,
    kCntSlots = 16
};

constexpr int kRadixThreads = 256;
constexpr int kRadixItems = 16;
constexpr int kRadixTile = kRadixThreads * kRadixItems;  // keys per block per pass
constexpr int kTileSortCap = 8192;                       // LDS bitonic capacity (32 KB)
constexpr int kBigSortThreads = 1024;
constexpr int kBitmapWords = 32768;                      // 1 Mi ranks per LDS window (128 KB)
constexpr int kGradStride = 16;                          // floats per Gaussian grad record

struct Layout {
    // geometry
    size_t depth_key, tiles_touched, rect, record, clamped, sorted_ids, depth_rank;
    size_t keys_a, keys_b, vals_b, radix_hist;
    size_t geom_bytes;
    // image
    size_t counters, tile_start, tile_cursor, oversize, final_T, n_contrib;
    size_t image_bytes;
    // binning
    size_t point_list, list_rank;
    size_t binning_bytes;
    int radix_blocks;
    int gx, gy, tiles;
};

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

inline Layout make_layout(int P, int W, int H, int64_t R)
{
    Layout L{};
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = align_up(o + bytes); return r; };
    const size_t p = (size_t)(P > 0 ? P : 1);
    L.radix_blocks = (int)((p + kRadixTile - 1) / kRadixTile);
    L.depth_key = take(4 * p);
    L.tiles_touched = take(4 * p);
    L.rect = take(8 * p);
    L.record = take(48 * p);
    L.clamped = take(4 * p);
    L.sorted_ids = take(4 * p);
    L.depth_rank = take(4 * p);
    L.keys_a = take(4 * p);
    L.keys_b = take(4 * p);
    L.vals_b = take(4 * p);
    L.radix_hist = take(4 * 256 * (size_t)L.radix_blocks);
    L.geom_bytes = o;

    L.gx = (W + kTile - 1) / kTile;
    L.gy = (H + kTile - 1) / kTile;
    L.tiles = L.gx * L.gy;
    const size_t T = (size_t)(L.tiles > 0 ? L.tiles : 1);
    const size_t HW = (size_t)W * (size_t)H;
    o = 0;
    L.counters = take(4 * kCntSlots);
    L.tile_start = take(4 * (T + 1));
    L.tile_cursor = take(4 * T);
    L.oversize = take(4 * T);
    L.final_T = take(4 * (HW > 0 ? HW : 1));
    L.n_contrib = take(4 * (HW > 0 ? HW : 1));
    L.image_bytes = o;

    o = 0;
    const size_t r = (size_t)(R > 0 ? R : 1);
    L.point_list = take(4 * r);
    L.list_rank = take(4 * r);
    L.binning_bytes = o;
    return L;
}

struct PreprocessParams {
    int P, M, D, W, H, gx, gy;
    float tanfovx, tanfovy, focal_x, focal_y, scale_modifier;
    int include_feature, prefiltered;
    const float *means, *shs, *colors, *lang, *opac, *scales, *rots, *cov_pre;
    const float *view, *proj, *campos;
    int32_t* radii;
    uint32_t *depth_key, *tiles, *rect, *clamped, *counters;
    float4* record;
};

struct PreprocessBwdParams {
    int P, M, D, W, H;
    float tanfovx, tanfovy, focal_x, focal_y, scale_modifier;
    const float *means, *shs, *scales, *rots, *cov_pre, *view, *proj, *campos;
    const int32_t* radii;
    const uint32_t* clamped;
    const float* grad;  // P x kGradStride
    float *dmeans2D, *dcolors, *dlang, *dopac, *dmeans3D, *dcov, *dsh, *dscales, *drots;
};

struct RenderParams {
    int W, H, gx, gy, include_feature;
    const uint32_t* tile_start;
    const uint32_t* point_list;
    const float4* record;
    const float* bg;
    float* final_T;
    uint32_t* n_contrib;
    float *out_color, *out_lang;
    // backward
    const float *dL_dcolor, *dL_dlang;
    float* grad;
};

hipError_t launch_preprocess(const PreprocessParams& p, hipStream_t s);
hipError_t launch_preprocess_backward(const PreprocessBwdParams& p, hipStream_t s);
hipError_t launch_mark_visible(int P, const float* means, const float* view, const float* proj,
                               uint8_t* visible, hipStream_t s);

// depth sort of all P Gaussians by (depth key, id) -> sorted_ids; and depth_rank inverse
hipError_t launch_depth_sort(int P, const Layout& L, char* geom, uint32_t* counters, hipStream_t s,
                             bool debug);
hipError_t launch_tile_count(int P, const Layout& L, char* geom, char* image, hipStream_t s);
hipError_t launch_tile_scan(const Layout& L, char* image, hipStream_t s);
hipError_t launch_emit(int P, const Layout& L, char* geom, char* image, char* binning, hipStream_t s);
hipError_t launch_tile_sort(const Layout& L, char* geom, char* image, char* binning, hipStream_t s,
                            bool debug);

hipError_t launch_render_forward(const RenderParams& p, int tiles, hipStream_t s);
hipError_t launch_render_backward(const RenderParams& p, int tiles, hipStream_t s);

}  // namespace lsr
