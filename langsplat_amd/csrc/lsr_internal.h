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
    kCntRendered = 1,
    kCntError = 2,
    kCntFwdFlags = 3,    // what the forward prepared for its backward: kFwdZeroedRecords | kFwdFusedLoss
    kCntSuper = 4,       // super-tile entries E (binning)
    kCntKeyMin = 5,      // smallest visible depth key (float bits)
    kCntKeyMax = 6,      // largest visible depth key
    kCntOverflow = 7,    // capacity mode: the view exceeds the caller's capacities (nothing is binned)
    kCntSlots = 16
};
constexpr uint32_t kFwdZeroedRecords = 1u;  // the language step's gradient records cleared (the render
                                            // backward clears this bit: only its first use is valid)
constexpr uint32_t kFwdFusedLoss = 2u;      // loss codes written (dL_dloss is valid)
constexpr uint32_t kFwdNoColorState = 4u;   // split-replay states without the colour sums (no colour
                                            // gradient may follow: LSR_FWD_NO_COLOR_GRAD)
constexpr uint32_t kFwdNoBackward = 8u;     // no backward state written (LSR_FWD_NO_BACKWARD)
// longest-first tile schedule (lsr_render.hip): tiles per work class, forward and backward,
// right after the counters so one memset clears both
constexpr int kWorkClasses = 64;
constexpr int kCntFwdClass = kCntSlots;
constexpr int kCntBwdClass = kCntSlots + kWorkClasses;
constexpr int kCntWords = kCntSlots + 2 * kWorkClasses;

// Split replay (lsr_render.hip): the render forward records each pixel's state (T and the colour /
// feature sums) before list entries kSplitChunk, 2 kSplitChunk, ... (up to entry 1024 - kSplitChunk)
// of a tile it is still compositing (in the tile's own kSplitMax slots), so the backward can replay
// a long tile as up to kSplitItems independent work items of <= kSplitChunk entries each (the last
// one: the rest) instead of one long serial chain.  LSR_SPLIT_CHUNK=128 (round 6, measured and not
// the default: each wave records the boundary inside a 256-entry batch mid-walk) halved the items
// but cost more than it saved -- C3 render backward 141 -> 152 us, forward 125 -> 132 us, pipelined
// step 0.400 -> 0.465 ms (profiles/r06_split128_ab.txt).
#ifndef LSR_SPLIT_CHUNK
#define LSR_SPLIT_CHUNK 256
#endif
constexpr int kSplitChunk = LSR_SPLIT_CHUNK;
static_assert(kSplitChunk == 128 || kSplitChunk == 256, "split chunks of 128 or 256 list entries");
constexpr int kSplitMax = 1024 / kSplitChunk - 1;  // recorded boundaries per tile
constexpr int kSplitItems = kSplitMax + 1;  // backward work items per tile
constexpr int kSplitVals = 8;               // per pixel {T, feature (3)}, {colour (3), -}
constexpr int kSplitSlots = kSplitMax + 1;  // per tile: the boundaries' states, then the final sums

constexpr int kRadixThreads = 256;
// preprocess workgroups: the SH staging takes 4 (3M + 1) bytes of LDS per thread, so 128-thread
// blocks let more of them share a CU and overlap one block's loads with another's arithmetic
#ifndef LSR_PRE_THREADS
#define LSR_PRE_THREADS 128
#endif
constexpr int kPreThreads = LSR_PRE_THREADS;
constexpr int kSuper = 8;          // super-tile = kSuper x kSuper tiles (64-bit tile masks)
constexpr int kSegEntries = 512;   // super-tile list entries per binning workgroup
constexpr int kGradStride = 16;                          // floats per Gaussian grad record
constexpr int kGradStrideLang = 5;  // without geometry gradients: {dxy, dlang}, packed 20-B records
// LSR_BWD_DEFER_TAIL's planar records: P x 3 language partials, the step's skip flag (one word: the
// all-reduce carries it with the partials), padding, then P x 2 screen-space partials at 3 P + 4
constexpr int kDeferXyOffset = 4;  // floats after the 3 P language partials
constexpr int kFusedEntries = 3;    // capacity of the fused super-tile emission, entries per Gaussian
constexpr int kSuperHistBlock = 1024;  // entries per block of the super-tile pass (k_radix_scatter<4>)

size_t radix_hist_words(int64_t n);   // per-block digit histograms for n keys
int msd_blocks(int P);                 // blocks of the MSD depth pass's histogram
// placed emission's count words (lsr_binning.hip): [super-tile][bucket] counts, per group of
// kSupGroup buckets the group sums, the group arrival counters
constexpr int kSupGroup = 16;
constexpr size_t sup_words(int buckets)  // with 256 or 512 depth-order buckets
{
    return 256 * (size_t)buckets + 256 * (size_t)(buckets / kSupGroup) + (size_t)(buckets / kSupGroup);
}
constexpr size_t kSupWords = sup_words(512);  // the allocation (either bucket count)
size_t scan_region_words(int64_t n);  // look-back status + ticket of one scan of n words
constexpr int kDepthScans = 5;         // 4 depth-sort passes + the instance-offset scan

struct Layout {
    // geometry (per Gaussian)
    size_t depth_key, tiles_touched, rect, record, clamped, sorted_ids, super_offset;
    size_t keys_a, keys_b, vals_b, radix_hist, radix_hist_scan, scan_regions, rect_ranked, pre_partial;
    size_t scan_region_geom;  // u32 words per depth-order scan region
    size_t loss_words;        // fused loss: per-workgroup / per-group words and tickets, after the scan regions
    size_t zero_words;        // u32 words preprocess clears from scan_regions (scan status + loss words)
    size_t bucket_totals;     // MSD depth order: super-tile entries per top-digit bucket (<= 512 u32)
    size_t bucket_status;     // MSD depth order with fused emission: <= 512 {flag, bucket total} u64 words
                              // + the bucket ticket, inside the range preprocess clears
    size_t fused_keys, fused_vals;  // the super-tile entries the bucket sort emits (fused_cap each)
    int64_t fused_cap;
    // with fused emission and <= 256 super-tiles: the super-tile radix pass's [super-tile][block]
    // histogram (blocks of kSuperHistBlock entries, row stride super_hist_stride), counted by the
    // bucket sort as it emits; its scan and that scan's status words
    size_t super_hist, super_hist_scan, super_hist_status;
    size_t super_hist_words, super_hist_status_words;
    int super_hist_stride;
    // placed emission (<= 256 super-tiles): the bucket sort's entry counts (kSupWords, cleared by
    // preprocess); the MSD histogram then also holds one row per super-tile after its 256 digit rows
    size_t sup_status;
    size_t grad_records;      // P x kGradStrideLang floats: the language step's gradient records (cleared
                              // by the render forward under LSR_FWD_ZERO_GRAD_RECORDS)
    size_t geom_bytes;
    // image (per pixel / tile)
    size_t counters, ranges, final_T, n_contrib, tile_lists, loss_partial, loss_code;
    size_t split_desc, split_pool;  // per tile {boundaries, -}; per tile kSplitSlots x kSplitVals x 256 floats
    size_t image_bytes;
    // binning (point_list per tile instance, the rest per super-tile entry / segment)
    size_t point_list, cover, super_keys, super_vals, alt_keys, alt_vals, bin_radix_hist, bin_radix_hist_scan;
    size_t bin_scan_regions, super_ranges, seg_base, col_prefix, row_prefix, seg_table, seg_table_scan;
    size_t scan_region_bin;   // u32 words per binning scan region
    size_t seg_table_words;   // (tile, segment) count table incl. one trailing slot
    int64_t super_entries;    // E
    int64_t seg_blocks;       // upper bound on segments = binning grid
    size_t binning_bytes;
    int gx, gy, tiles, sgx, sgy, supers, super_bits, super_passes;
};

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

inline Layout make_layout(int P, int W, int H, int64_t R, int64_t E)
{
    Layout L{};
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = align_up(o + bytes); return r; };
    const size_t p = (size_t)(P > 0 ? P : 1);
    L.depth_key = take(4 * p);
    L.tiles_touched = take(4 * p);
    L.rect = take(8 * p);
    L.record = take(48 * p);
    L.clamped = take(4 * p);
    L.sorted_ids = take(4 * p);
    L.super_offset = take(4 * (p + 1));
    L.keys_a = take(4 * p);
    L.keys_b = take(4 * p);
    L.vals_b = take(4 * p);
    // 256 or 512 digit rows, then (placed emission) <= 256 super-tile rows
    const size_t hw_p = 3 * radix_hist_words((int64_t)p);
    L.radix_hist = take(4 * hw_p);
    L.radix_hist_scan = take(4 * hw_p);  // scans are out-of-place (k_scan's stall fallback)
    L.scan_region_geom = scan_region_words((int64_t)(hw_p > p ? hw_p : p));
    L.scan_regions = take(4 * kDepthScans * L.scan_region_geom);
    {
        const size_t gx = (size_t)(W + kTile - 1) / kTile, gy = (size_t)(H + kTile - 1) / kTile;
        const size_t loss_bytes = 8 * gx * gy;  // one word per render forward workgroup
        L.loss_words = take(loss_bytes);
        L.bucket_status = take(8 * 513);
        L.zero_words = (L.bucket_status + 8 * 513 - L.scan_regions + 3) / 4;
    }
    L.rect_ranked = take(8 * p);
    // + padding: cleared as whole float4s, and the deferred form's flag slot (kDeferFlagSlot)
    L.grad_records = take(4 * kGradStrideLang * p + 32);
    L.bucket_totals = take(4 * 512);
    {
        const int gx = (W + kTile - 1) / kTile, gy = (H + kTile - 1) / kTile;
        const int supers = ((gx + kSuper - 1) / kSuper) * ((gy + kSuper - 1) / kSuper);
        const int64_t cap = (int64_t)kFusedEntries * (int64_t)p;
        L.super_hist_stride = (int)((cap + kSuperHistBlock - 1) / kSuperHistBlock);
        L.super_hist_words = supers <= 256 ? (size_t)supers * (size_t)L.super_hist_stride : 0;
        L.super_hist_status_words = L.super_hist_words ? scan_region_words((int64_t)L.super_hist_words) : 0;
        L.super_hist = take(4 * L.super_hist_words);
        L.super_hist_scan = take(4 * L.super_hist_words);
        L.super_hist_status = take(4 * L.super_hist_status_words);
        L.sup_status = take(4 * kSupWords);
    }
    // E is ~1.5 per visible Gaussian at 1080p; a view with more than kFusedEntries per Gaussian
    // falls back to k_emit_super after the host wait
    L.fused_cap = (int64_t)kFusedEntries * (int64_t)p;
    L.fused_keys = take(4 * (size_t)L.fused_cap);
    L.fused_vals = take(4 * (size_t)L.fused_cap);
    L.pre_partial = take(16 * ((p + kPreThreads - 1) / kPreThreads));
    L.geom_bytes = o;

    L.gx = (W + kTile - 1) / kTile;
    L.gy = (H + kTile - 1) / kTile;
    L.tiles = L.gx * L.gy;
    L.sgx = (L.gx + kSuper - 1) / kSuper;
    L.sgy = (L.gy + kSuper - 1) / kSuper;
    L.supers = L.sgx * L.sgy;
    L.super_bits = 1;  // <= 16: the entry key keeps the super-tile id in its low 16 bits
    while ((1 << L.super_bits) < L.supers) L.super_bits++;
    L.super_passes = (L.super_bits + 7) / 8;
    const size_t T = (size_t)(L.tiles > 0 ? L.tiles : 1);
    const size_t HW = (size_t)W * (size_t)H;
    o = 0;
    L.counters = take(4 * kCntWords);
    L.ranges = take(8 * T);
    L.final_T = take(4 * (HW > 0 ? HW : 1));
    L.n_contrib = take(4 * (HW > 0 ? HW : 1));
    // [fwd][class][T] tiles, then [bwd][class][kSplitItems T] split-replay items
    L.tile_lists = take(4 * kWorkClasses * T * (1 + kSplitItems));
    L.loss_partial = take(8 * T);                    // fused loss, P == 0: one double per workgroup
    L.loss_code = take(HW > 0 ? HW : 1);             // fused loss: per-pixel sign / mask code
    L.split_desc = take(16 * T);
    L.split_pool = take(4 * (size_t)kSplitSlots * kSplitVals * kTilePixels * T);
    L.image_bytes = o;

    o = 0;
    const size_t r = (size_t)(R > 0 ? R : 1);
    const size_t e = (size_t)(E > 0 ? E : 1);
    L.super_entries = E;
    L.seg_blocks = (int64_t)((e + kSegEntries - 1) / kSegEntries) + L.supers;
    L.seg_table_words = 64 * (size_t)L.seg_blocks + 1;
    L.point_list = take(4 * r);
    L.cover = take(r);  // right after point_list: its offset depends on R only (the backward has no E)
    L.super_keys = take(4 * e);
    L.super_vals = take(4 * e);
    L.alt_keys = take(4 * e);
    L.alt_vals = take(4 * e);
    const size_t hw_e = radix_hist_words((int64_t)e);
    L.bin_radix_hist = take(4 * hw_e);
    L.bin_radix_hist_scan = take(4 * hw_e);
    L.scan_region_bin = scan_region_words((int64_t)(hw_e > L.seg_table_words ? hw_e : L.seg_table_words));
    L.bin_scan_regions = take(4 * (L.super_passes + 1) * L.scan_region_bin);
    L.super_ranges = take(8 * (size_t)L.supers);
    L.seg_base = take(4 * ((size_t)L.supers + 1));
    L.col_prefix = take(4 * (size_t)L.supers);
    L.row_prefix = take(4 * ((size_t)L.gy + 1));
    L.seg_table = take(4 * L.seg_table_words);
    L.seg_table_scan = take(4 * L.seg_table_words);
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
    uint32_t* zero;   // depth-order scan status, cleared here
    int zero_words;
    uint32_t* zero2;  // placed emission: the bucket sort's [super-tile][bucket] counts, cleared here
    int zero2_words;
    uint4* partial;   // per block {tile instances, super-tile entries, min / max visible depth key}
    int raw;                  // lsr_raw_flags
    const float* shs_rest;    // split SH rows (shs = dc only) or null
    uint8_t* visible;         // optional radii > 0 bytes
    int lang_deferred;        // the records' language slots are filled later (launch_fill_language)
};

struct PreprocessBwdParams {
    int P, M, D, W, H;
    float tanfovx, tanfovy, focal_x, focal_y, scale_modifier;
    const float *means, *shs, *scales, *rots, *cov_pre, *view, *proj, *campos;
    const int32_t* radii;
    const uint32_t* clamped;
    const float* grad;  // P x kGradStride
    float *dmeans2D, *dcolors, *dlang, *dopac, *dmeans3D, *dcov, *dsh, *dscales, *drots;
    int raw;                  // lsr_raw_flags: chain the activation derivatives
    const float *opac, *lang, *shs_rest;
    float* dsh_rest;
};

struct RenderParams {
    int W, H, gx, gy, include_feature;
    const uint2* ranges;
    const uint32_t* point_list;
    // per list instance: the 4-bit mask of the tile's wave blocks it can reach (entry_cover), written
    // by the forward for every instance it loads and read by the backward instead of recomputing it
    uint8_t* cover;
    const float4* record;
    const float* bg;
    float* final_T;
    uint32_t* n_contrib;
    float *out_color, *out_lang;
    // longest-first schedule: class counts (counters + kCntFwdClass / kCntBwdClass) and lists (the
    // forward's tiles of class c at sched_lists[c * tiles], the backward's split-replay items at
    // sched_lists[kWorkClasses * tiles + c * kSplitItems * tiles]); null: launch order
    uint32_t* sched_counts;
    uint32_t* sched_lists;
    // split replay (scheduled launches only; null: off): per tile kSplitMax per-pixel state slots and
    // a descriptor {boundaries recorded below the replay length, -, -, -}
    float* split_pool;
    uint4* split_desc;
    int split_color;  // forward: store the colour sums' half of every state (off: LSR_FWD_NO_COLOR_GRAD)
    int no_bwd;       // forward: write no state for a backward (LSR_FWD_NO_BACKWARD)
    int prio;  // wave priority by launch position (longest tiles highest), 0: off
    int shared_cu;  // another stream runs beside it (backward: LSR_BWD_SHARED_CU; forward: a composite
                    // phase): fewer workgroups per CU (lsr_render.hip kSharedWgsBwd / kSharedWgsFwd)
    int geo;   // backward: the conic / opacity partials are needed (geometry gradients)
    float4* zero_records;  // forward: clear these zero_records_n4 float4s (grid-stride), or null
    int64_t zero_records_n4;
    // backward
    const float *dL_dcolor, *dL_dlang;
    float* grad;
    // the language step's planar records (LSR_BWD_DEFER_TAIL): grad = P x 3 language partials, grad_xy
    // = P x 2 screen-space partials; null: the packed 20-B records {dx, dy, l0, l1, l2} at grad
    float* grad_xy;
    // LSR_BWD_DEFER_TAIL: the first workgroup copies *flag_src (0 if null) to *flag_dst, the word after
    // the language partials, so the one all-reduce of the partials carries the skip flag too
    const int32_t* flag_src;
    int32_t* flag_dst;
    uint32_t* fwd_flags;  // counters[kCntFwdFlags] of the forward (its records bit is cleared)
    // fused language-feature loss (null: off).  forward: gt (3 x HW), mask (HW bool bytes) -> codes,
    // per-workgroup partials, out_loss; backward: dL_dloss (device scalar) with the forward's codes
    const float* loss_gt;
    const uint8_t* loss_mask;
    uint8_t* loss_code;
    double* loss_partial;     // P == 0 (k_loss_background): one double per workgroup
    uint64_t* loss_words;     // render forward: words and tickets of loss_block_publish (zeroed)
    float* out_loss;
    uint32_t spin_limit;      // loss_block_publish's poll bound (stall_spin_limit())
    uint32_t* stall;          // its stall flag (the calling thread's pinned host word)
    const float* dL_dloss;
};

hipError_t launch_preprocess(const PreprocessParams& p, hipStream_t s);
// the language slots of the visible Gaussians' records (after a deferred preprocess)
hipError_t launch_fill_language(int P, const float* lang, int raw, const int32_t* radii, float4* record,
                                hipStream_t s);
hipError_t launch_preprocess_backward(const PreprocessBwdParams& p, hipStream_t s);
hipError_t launch_grad_epilogue(int P, const int* radii, const float* grad, int stride, const float* lang,
                                int raw_lang, float* dmeans2D, float* dlang, hipStream_t s);
hipError_t launch_mark_visible(int P, const float* means, const float* view, const float* proj,
                               uint8_t* visible, hipStream_t s);

// depth sort of all P Gaussians by (depth key, id) on `passes` 8-bit digits of the key minus the
// smallest visible key (counters[kCntKeyMin/Max], from launch_preprocess) -> sorted_ids; per-Gaussian
// super-tile entry offsets in that order
// fused_emit (MSD path only): the bucket sort also writes the super-tile entries into L.fused_keys /
// fused_vals when they fit (E <= L.fused_cap), so k_emit_super is not launched
// emit_cap > 0: the fused emission writes at most that many entries (capacity mode), else L.fused_cap
hipError_t launch_depth_order(int P, int passes, const Layout& L, char* geom, uint32_t* counters, uint32_t* stall,
                              hipStream_t s, bool debug, bool fused_emit = false, uint32_t emit_cap = 0,
                              bool placed = false);
// false: the depth order reads its pass count on the device (MSD pass + per-bucket LDS sort) and
// ignores `passes`; true (large P): LSD passes, `passes` must cover the visible key range
bool depth_order_uses_pass_count(int P);
int msd_digits(int P);  // the depth order's MSD buckets (256 / 512), 0: LSD passes
// LSR_FUSED_EMIT=0 turns the fused super-tile emission off (measurement knob, read once)
bool fused_emit_enabled();
// placed emission: the fused emission writes every entry at its super-tile-major position, so the
// binning's super-tile pass (scan + scatter) is not launched.  Needs <= 256 super-tiles.  Default:
// on for a whole forward, off for the split geometry phase (whose kernels run beside the previous
// view's render kernels, where the narrow scan + scatter launches fill gaps better than the longer
// bucket kernel: measured) and for the 512-bucket depth order (2M..4.2M
// Gaussians: a bucket's ~6k Gaussians have more entries than one LDS list; listed from parked
// arrays they take C5's depth order from 140 to 189 us for 32 us less binning: measured);
// LSR_PLACED=1 / 0 forces it (read per call)
bool placed_emit(const Layout& L, bool geometry_phase, int buckets);
// super-tile lists, per-(tile, segment) counts, scanned bases -> point_list and tile ranges.
// emitted: the depth order's bucket sort already wrote the E entries into L.fused_keys / fused_vals
// (super-tile-major when `placed`, the depth order's choice, else in depth order).
// Device-read counts for launches sized from capacities: n = min(n, *n) when n is set; a set *abort
// (counters[kCntOverflow]) makes the kernel skip its work (after the clearing the binning's first
// launch does).  Both null: the host's counts.
struct DevCount {
    const uint32_t* n;
    const uint32_t* abort;
};
// capacity mode: dc = {counters + kCntSuper, counters + kCntOverflow}, R / L from the capacities
hipError_t launch_binning(int P, int64_t R, const Layout& L, char* geom, char* image, char* binning, uint32_t* stall,
                          hipStream_t s, bool debug, bool emitted = false, DevCount dc = DevCount{nullptr, nullptr},
                          bool placed = false);

// Look-back stall handling (k_scan, k_masked_l1_forward).  A single-pass look-back polls at most
// stall_spin_limit() times for a predecessor's value; past that it computes the value itself from
// the inputs (same result) and stores 1 into `stall`, a word of the calling thread's pinned host
// block (lsr_api.hip), which lsr_debug_scan_stalls reads.  set_stall_spin_limit returns the old
// limit; 0 = never wait (every look-back takes the fallback: tests).
uint32_t stall_spin_limit();
uint32_t set_stall_spin_limit(uint32_t v);
__device__ __forceinline__ void note_stall(uint32_t* stall)
{
    if (stall) __hip_atomic_store(stall, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// work class of a tile with w >= 1 units of work: quarter-octaves, monotone in w, 0..63 (w >= 2^16
// shares the top class)
__device__ __forceinline__ int work_class(uint32_t w)
{
    if (w >= 65536u) return kWorkClasses - 1;
    const int lg = 31 - __clz(w);
    const int frac = lg >= 2 ? (int)((w >> (lg - 2)) & 3u) : (lg == 1 ? (int)((w & 1u) << 1) : 0);
    return 4 * lg + frac;
}

// appends tile t with w >= 1 units of work to class lists (counts[c], lists[c * T + i])
__device__ __forceinline__ void schedule_tile(uint32_t* counts, uint32_t* lists, int T, int t, uint32_t w)
{
    const int c = work_class(w);
    lists[(size_t)c * T + atomicAdd(&counts[c], 1u)] = (uint32_t)t;
}

struct AdamScalars {
    float w1;             // 1 - beta1 (lerp weight)
    float beta2, w2;      // beta2, 1 - beta2
    float inv_bc2_sqrt;   // 1 / sqrt(1 - beta2^step)
    float eps;
    float neg_step_size;  // -lr / (1 - beta1^step)
};
hipError_t launch_adam(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                       const AdamScalars& a, hipStream_t s);
constexpr int kAdamMaxTensors = 16;
struct AdamSegment {
    float* param;
    const float* grad;
    float *m, *v;
    int64_t n, block0;
    AdamScalars a;
    int vec;
};
struct AdamHyper {
    double lr, beta1, beta2, eps;
    int64_t step_offset;  // with step_dev: this tensor's count minus the device count
};
struct AdamTable {
    int count;
    AdamSegment seg[kAdamMaxTensors];
    AdamHyper hyper[kAdamMaxTensors];  // used with step_dev: the scalars are formed on the device (lr
                                       // from step_dev[LSR_ADAM_WORD_LR + k])
    int64_t* step_dev;                 // null: the host's step counts (seg[].a)
    const int32_t* skip;               // *skip != 0: the launch is a no-op (null: never)
};
hipError_t launch_adam_multi(AdamTable& tab, float grad_scale, hipStream_t s);
// lsr_backward_args.update: k_adam_advance (one tensor, the skip flag), then one pass per Gaussian: the
// gradient epilogue (dmeans2D, dlang from the 20-B records and the raw feature), the Adam step of the
// raw feature (its device scalars; nothing on *skip) and, with fill, the activated updated feature
// into fill's language slots of every Gaussian.  deferred (lsr_language_tail): the records are planar
// and their language partials reduced over the ranks (no radius gate on dlang: a Gaussian this view
// culled may carry another view's partials)
hipError_t launch_language_tail(int P, const int32_t* radii, const float* grad, float* lang, float* exp_avg,
                                float* exp_avg_sq, float* dmeans2D, float* dlang, const AdamHyper& h, int64_t* step_dev,
                                const int32_t* skip, float4* fill, int deferred, hipStream_t s);
hipError_t launch_adam_fill(int P, const float* grad, float grad_scale, float* lang, float* exp_avg, float* exp_avg_sq,
                            const AdamHyper& h, int64_t* step_dev, const int32_t* skip, float4* fill, int raw,
                            hipStream_t s);
// zero `bytes` bytes at p with a kernel (no memset node in a captured graph)
hipError_t zero_fill(void* p, size_t bytes, hipStream_t s);
hipError_t launch_densification_stats(int P, const int* radii, const float* dmeans2D, float* max_radii, float* accum,
                                      float* denom, hipStream_t s);

// out[i] = sum(in[0..i)); region: scan_region_words(n) zeroed words (single-pass look-back scan)
hipError_t scan_exclusive_u32(const uint32_t* in, uint32_t* out, int n, uint32_t* region, uint32_t* fault,
                              hipStream_t s);
// reduces the preprocess block partials into counters and publishes counters[0..7], each with seq,
// to the host slots (8 x u64 pinned)
// capacity mode (r_cap > 0): no host slots; counters[kCntOverflow] (and *overflow) = R > r_cap || E > e_cap
// || the LSD depth order needs more than depth_passes passes (depth_passes 0: not checked)
hipError_t launch_publish_counters(int nb, const uint4* partial, uint32_t* counters, uint64_t* host_slots,
                                   uint32_t seq, uint32_t fwd_flags, uint32_t r_cap, uint32_t e_cap,
                                   int32_t* overflow, int depth_passes, hipStream_t s);
size_t knn_scratch_bytes(int64_t N);
hipError_t launch_knn_mean_dist3(int64_t N, const float* pts, float* out, void* scratch, uint32_t* stall,
                                 hipStream_t s);

size_t masked_l1_scratch_bytes();
hipError_t launch_masked_l1_forward(int C, int64_t HW, const float* pred, const float* gt, const void* mask,
                                    int mask_is_float, float* loss, void* scratch, uint32_t epoch, uint32_t* stall,
                                    hipStream_t s);
hipError_t launch_masked_l1_backward(int C, int64_t HW, const float* pred, const float* gt, const void* mask,
                                     int mask_is_float, const float* grad_loss, float* grad_pred, hipStream_t s);
hipError_t launch_decode_language_feature(int H, int W, const int64_t* seg_level, int N, int D,
                                          const float* feature_map, float* out, uint8_t* mask, uint32_t* bad,
                                          hipStream_t s);

hipError_t launch_render_forward(const RenderParams& p, int tiles, hipStream_t s);
hipError_t launch_render_backward(const RenderParams& p, int tiles, hipStream_t s);
// the fused loss of an empty scene (P == 0: no render forward runs) into p.out_loss
hipError_t launch_loss_background(const RenderParams& p, hipStream_t s);
hipError_t render_stats_read(unsigned long long* out, int n);  // reads and clears
hipError_t render_timeline_read(uint32_t* out, int kernel, int n);
hipError_t bucket_timeline_read(uint32_t* out, int n);  // LSR_BUCKET_TIMELINE=1 records (k_depth_bucket_sort)
hipError_t launch_clock_probe(uint64_t* out, hipStream_t s);  // lsr_debug_clock_probe
hipError_t launch_delay(uint32_t ticks, hipStream_t s);        // lsr_debug_delay

}  // namespace lsr
