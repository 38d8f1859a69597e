/*
 * lsr.h -- C ABI of the MI355X-native LangSplat Gaussian rasterizer (liblsr.so).
 *
 * This is the drop-in boundary for the hot path named in BASELINE.json "north_star": the
 * forward and backward of RasterizeGaussians.  Each entry point replaces one native entry of
 * the reference's (absent) submodules/langsplat-rasterization extension, whose Python face
 * is used at:
 *
 *   reference interface (call site)                              replaced by
 *   ------------------------------------------------------------ ---------------------------
 *   _C.rasterize_gaussians            (called via GaussianRasterizer.forward,
 *                                      gaussian_renderer/__init__.py:96-105)        lsr_forward
 *   _C.rasterize_gaussians_backward   (autograd backward of the same call;
 *                                      train.py:104 loss.backward())                lsr_backward
 *   _C.mark_visible                   (GaussianRasterizer.markVisible; upstream API,
 *                                      unused by the reference scripts)             lsr_mark_visible
 *   C++ exception text -> RuntimeError (upstream error path)        lsr_last_error
 *
 * Conventions:
 *   - All array pointers are DEVICE pointers to contiguous fp32/int32 data, borrowed for the
 *     duration of the call.  Outputs are written in full; callers never need to pre-zero.
 *   - Matrices are the reference's row-vector matrices stored row-major, exactly the memory of
 *     Camera.world_view_transform / full_proj_transform (scene/cameras.py:54-56).
 *   - Work is enqueued on `stream` (a hipStream_t; NULL = legacy default stream).  lsr_forward
 *     waits once for the device to learn num_rendered (as upstream does) -- except in capacity mode
 *     (lsr_forward_args.capacity_rendered > 0), which sizes everything from caller capacities and
 *     never waits, so that a whole train step can be captured into a HIP graph.
 *   - Scratch is owned by the caller and requested through `alloc` (upstream's resizable
 *     geometry/binning/image buffers).  The three forward buffers must be kept alive, unchanged,
 *     and passed back to lsr_backward.
 *   - Return value: LSR_OK or an error code; lsr_last_error() describes the last failure on the
 *     calling thread.  The only process-wide state is the opt-in kernel profiler below (off by
 *     default, mutex-protected); rasterization itself is re-entrant.
 */
#ifndef LSR_H
#define LSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSR_ABI_VERSION 17

enum lsr_status {
    LSR_OK = 0,
    LSR_ERR_INVALID = 1,     /* bad argument (null pointer, negative size, ...) */
    LSR_ERR_HIP = 2,         /* a HIP runtime call or kernel launch failed */
    LSR_ERR_ALLOC = 3,       /* the alloc callback returned NULL */
    LSR_ERR_PREFILTERED = 4  /* prefiltered=1 but a Gaussian failed the frustum test */
};

/* Scratch buffers requested through the allocator (upstream geomBuffer/binningBuffer/imgBuffer) */
enum lsr_buffer {
    LSR_BUF_GEOM = 0,     /* per Gaussian; forward -> backward */
    LSR_BUF_BINNING = 1,  /* per tile instance; forward -> backward */
    LSR_BUF_IMAGE = 2,    /* per pixel / per tile; forward -> backward */
    LSR_BUF_BACKWARD = 3  /* per Gaussian gradient scratch, backward only */
};

/* Returns device memory of at least `bytes` bytes, 256-byte aligned, valid until the caller
 * releases it; NULL on failure.  Called synchronously from the calling thread. */
typedef void* (*lsr_alloc_fn)(void* user, int32_t which, size_t bytes);

/* Fused parameter activation.  Each bit set in lsr_forward_args.raw /
 * lsr_backward_args.raw says the matching input is GaussianModel's RAW parameter; the kernels
 * apply the model's activation (scene/gaussian_model.py:33-41 setup_functions, getters :134-161;
 * language normalisation gaussian_renderer/__init__.py:87) and the backward returns the gradient
 * w.r.t. the raw tensor.  raw == 0 is the reference's API: every input already activated. */
enum lsr_raw_flags {
    LSR_RAW_OPACITY = 1,    /* opacities = _opacity:            sigmoid(x) = 1 / (1 + exp(-x))      */
    LSR_RAW_SCALES = 2,     /* scales = _scaling:               exp(x)                              */
    LSR_RAW_ROTATIONS = 4,  /* rotations = _rotation:           x / max(||x||, 1e-12) (F.normalize) */
    LSR_RAW_LANGUAGE = 8    /* language_feature = _language_feature: x / (||x|| + 1e-9)             */
};

/* The language step's backward (no geometry gradient, no colour gradient) accumulates 20-byte
 * per-Gaussian gradient records that must start at zero.  With LSR_FWD_ZERO_GRAD_RECORDS the
 * forward clears them inside its compositing kernel (stores beside a VALU-bound loop: no separate
 * memset launch) in the geometry buffer; the FIRST backward of that forward then passes
 * LSR_BWD_RECORDS_ZEROED and uses them as they are.  Any other backward clears its own records.
 * LSR_BWD_RECORDS_ZEROED is only valid for the first backward of a forward that passed
 * LSR_FWD_ZERO_GRAD_RECORDS, and lsr_backward_args.dL_dloss only for a forward that fused the loss
 * (out_loss set): the forward records both in its image buffer, and with settings.debug the
 * backward checks them and fails with LSR_ERR_INVALID instead of reading stale records or codes. */
/* LSR_FWD_NO_COLOR_GRAD: the caller promises that the backward of this forward gets no colour
 * gradient (lsr_backward_args.dL_dout_color == NULL), as in LangSplat's language step
 * (train.py:96-104: the loss reads the language image only).  The compositing kernel then stores
 * only the transmittance and feature sums of its split-replay states (half the state traffic).  A
 * backward with dL_dout_color after such a forward would start long tiles' replay chunks from
 * missing colour sums: it is invalid, and with settings.debug it fails with LSR_ERR_INVALID. */
/* LSR_FWD_NO_BACKWARD (ABI 13): the caller promises that no lsr_backward follows this forward
 * (inference: render.py:24-55 renders under torch.no_grad()).  The compositing kernel then writes
 * only the images (and the fused loss, if asked): not the state only the backward reads -- the
 * per-instance cover masks, the split-replay states, the backward's work lists, and the image
 * buffer's final transmittance and contributor counts.  With settings.debug a backward of such a
 * forward fails with LSR_ERR_INVALID. */
enum lsr_forward_flags { LSR_FWD_ZERO_GRAD_RECORDS = 1, LSR_FWD_NO_COLOR_GRAD = 2, LSR_FWD_NO_BACKWARD = 4 };
/* LSR_BWD_SHARED_CU (ABI 14): another stream's kernels run beside this backward (the pipelined step,
 * langsplat_amd/pipeline.py: the next view's preprocess, sort and binning).  The render backward
 * then runs at most 6 workgroups per CU instead of 8 (extra dynamic LDS), leaving wave slots and LDS
 * to the other stream's workgroups: measured at C3, 0.417-0.421 -> 0.400-0.401 ms per pipelined step
 * (DESIGN.md §5b).  Results are unchanged. */
/* LSR_BWD_DEFER_TAIL (ABI 16): the fused update (lsr_backward_args.update) split around a gradient
 * all-reduce (train.py:104 + 134-137 with the views of N ranks: langsplat_amd.pipeline at N > 1).
 * lsr_backward then runs the render backward only and leaves the language step's gradient records
 * in the geometry buffer (lsr_state_layout.grad_records) in planar form: float[3P] language partials
 * (dL/d of the activated feature, before the activation's chain rule), one word holding
 * *update_skip (0 when NULL), three padding words, then float[2P] screen-space partials.  The caller
 * reduces the first 3 P + 1 floats over the ranks -- an AVG: the chain rule and the Adam step are
 * linear / pointwise in the partials, a Gaussian another rank saw has partials here too, and the
 * skip word (0 or the bits of 1.0f) stays non-zero on every rank once one rank's view overflowed --
 * then calls lsr_language_tail with the same arguments: ONE pass writes dL_dmeans2D (this view's,
 * from the unreduced screen-space partials), dL_dlanguage_feature (from the reduced partials) and
 * the Adam step on the reduced skip word (+ the fill): what lsr_backward with update does at N = 1,
 * with no gradient epilogue before the collective.  The records need no LSR_BWD_RECORDS_ZEROED (they
 * are cleared here otherwise). */
enum lsr_backward_flags { LSR_BWD_RECORDS_ZEROED = 1, LSR_BWD_SHARED_CU = 2, LSR_BWD_DEFER_TAIL = 4 };

/* GaussianRasterizationSettings (gaussian_renderer/__init__.py:37-51), device-pointer form. */
typedef struct lsr_settings {
    int32_t image_height;
    int32_t image_width;
    float tanfovx;
    float tanfovy;
    float scale_modifier;
    int32_t sh_degree;        /* active SH degree D (0..3) */
    int32_t prefiltered;
    int32_t debug;            /* sync + check after every kernel */
    int32_t include_feature;  /* composite the 3-channel language feature */
    int32_t reserved;
    const float* bg;          /* [3] */
    const float* viewmatrix;  /* [16] world_view_transform */
    const float* projmatrix;  /* [16] full_proj_transform */
    const float* campos;      /* [3] camera_center */
} lsr_settings;

/* Inputs/outputs of _C.rasterize_gaussians.  Exactly one of {shs, colors_precomp} and one of
 * {scales+rotations, cov3D_precomp} is non-NULL (GaussianRasterizer.forward validates). */
typedef struct lsr_forward_args {
    int32_t P;                       /* number of Gaussians */
    int32_t M;                       /* SH coefficients stored per Gaussian (shs: P x M x 3) */
    const float* means3D;            /* P x 3 */
    const float* shs;                /* P x M x 3 or NULL */
    const float* colors_precomp;     /* P x 3 or NULL */
    const float* language_feature;   /* P x 3, or NULL when include_feature == 0 */
    const float* opacities;          /* P */
    const float* scales;             /* P x 3 or NULL */
    const float* rotations;          /* P x 4 (already normalised) or NULL */
    const float* cov3D_precomp;      /* P x 6 or NULL */
    float* out_color;                /* 3 x H x W */
    float* out_language_feature;     /* 3 x H x W */
    int32_t* radii;                  /* P */
    int32_t raw;                     /* lsr_raw_flags; 0 = activated inputs (reference API) */
    int32_t flags;                   /* lsr_forward_flags */
    const float* shs_rest;           /* NULL, or P x (M-1) x 3 (_features_rest) with shs = P x 1 x 3
                                        (_features_dc): the SH rows without torch.cat
                                        (scene/gaussian_model.py:146-150) */
    uint8_t* visible;                /* NULL, or P bytes: radii > 0 (render()'s visibility_filter,
                                        gaussian_renderer/__init__.py:99), written by preprocess */
    /* Fused language-feature loss (train.py:96-99):
     *     *out_loss = l1_loss(language_feature_image * mask, loss_target * mask)
     *               = sum |f m - gt m| / (3 H W)          (utils/loss_utils.py:17-18)
     * computed by the compositing kernel from the pixels it just produced (deterministic order).
     * out_loss NULL: off.  Needs include_feature and language_feature. */
    const float* loss_target;        /* 3 x H x W, or NULL */
    const uint8_t* loss_mask;        /* H x W bool bytes (scene/cameras.py:72 seg != -1), or NULL */
    float* out_loss;                 /* one float (device), or NULL */
    /* Capacity mode (graph capture): capacity_rendered > 0 bounds the tile instances and
     * capacity_entries (> 0) the super-tile entries of this view; the buffers and launch grids are
     * sized from them, the device reads the true counts, and the call enqueues its work without
     * waiting for the device.  *num_rendered then returns capacity_rendered (the value lsr_backward
     * needs).  A view that exceeds either capacity is not rasterized (background image, zero
     * gradients) and sets *overflow (device int32, written by every capacity-mode forward: 0, or
     * when set 0x3F800000 -- the bits of 1.0f, ABI 14 -- so the flag tests non-zero as an int and
     * can be all-reduced as a float beside the gradients: with a SUM or an average over ranks it is
     * non-zero on every rank as soon as one rank's view overflowed); the caller re-runs it with
     * larger capacities.  capacity_rendered == 0: the host reads the
     * counts after the preprocess (one wait) and sizes exactly. */
    int64_t capacity_rendered;
    int64_t capacity_entries;
    int32_t* overflow;               /* device int32 or NULL */
    int64_t* out_num_entries;        /* HOST pointer or NULL: the super-tile entry count (not in
                                        capacity mode), the capacity_entries a later call needs */
    /* Deferred language feature (the gradient all-reduce overlap).  NULL: off.
     * Otherwise a hipEvent_t: the preprocess, depth order and binning run without reading
     * language_feature, and the stream waits for this event only before a small kernel copies
     * (raw: activates) language_feature into the per-Gaussian records and the compositing starts.
     * A trainer records the event after the previous step's all-reduce and optimiser update of the
     * language feature on another stream, so that update overlaps this view's geometry work
     * (langsplat_amd.distributed.UpdateOverlap, langsplat_amd.pipeline).  Results are identical to a
     * call without it.  In capacity mode (a graph capture) the event is one recorded in the same
     * capture (a join of two branches). */
    void* language_ready;
    /* Forward in two calls (capacity mode only; the ABI 11 pipelined graph step): LSR_PHASE_GEOMETRY
     * enqueues the preprocess (language feature deferred), depth order and binning and returns;
     * LSR_PHASE_COMPOSITE, with the same arguments and an allocator that returns the same buffers,
     * enqueues the rest: the language feature into the records and the compositing (+ fused loss).
     * Whatever the caller orders between the two calls on the stream (e.g. a wait for the feature's
     * update) runs between them, so the two halves can be captured into two HIP graphs replayed on
     * different streams.  The compositing of a composite phase runs at fewer workgroups per CU (6,
     * leaving wave slots and registers to the other stream; LSR_FWD_SHARE=0: all that fit), which
     * changes no result.  LSR_PHASE_ALL (0): one call does everything. */
    int32_t phase;
} lsr_forward_args;
/* LSR_PHASE_COMPOSITE_FILLED (ABI 12): as LSR_PHASE_COMPOSITE, but the records' language slots already
 * hold the activated feature -- written by a fused update's fill_record (lsr_backward_args), which
 * may run before or while the geometry call runs: the geometry call of a split forward never writes
 * those slots. */
enum lsr_forward_phase { LSR_PHASE_ALL = 0, LSR_PHASE_GEOMETRY = 1, LSR_PHASE_COMPOSITE = 2, LSR_PHASE_COMPOSITE_FILLED = 3 };

/* Inputs/outputs of _C.rasterize_gaussians_backward.  Every non-NULL output is fully written
 * (zeros for culled Gaussians).  dL_dsh may be NULL when shs is NULL; dL_dscales/dL_drotations
 * may be NULL when cov3D_precomp is given; dL_dcov3D may be NULL when scales are given.
 * Geometry gradients are all-or-nothing: when dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D,
 * dL_dsh, dL_dsh_rest, dL_dscales and dL_drotations are ALL NULL (no geometry input needs a
 * gradient: ctx.needs_input_grad, e.g. LangSplat's language step, scene/gaussian_model.py:203-217),
 * only dL_dmeans2D and dL_dlanguage_feature (either may be NULL too) are computed and the
 * preprocess backward is not run. */
typedef struct lsr_backward_args {
    int32_t P;
    int32_t M;
    int64_t num_rendered;            /* value returned by lsr_forward */
    const float* means3D;
    const float* shs;
    const float* colors_precomp;
    const float* language_feature;
    const float* opacities;
    const float* scales;
    const float* rotations;
    const float* cov3D_precomp;
    const int32_t* radii;
    const float* dL_dout_color;             /* 3 x H x W or NULL (treated as zeros) */
    const float* dL_dout_language_feature;  /* 3 x H x W or NULL (treated as zeros) */
    void* geom_buffer;
    void* binning_buffer;
    void* image_buffer;
    float* dL_dmeans2D;              /* P x 3 (z = 0) */
    float* dL_dcolors;               /* P x 3 */
    float* dL_dlanguage_feature;     /* P x 3 */
    float* dL_dopacity;              /* P */
    float* dL_dmeans3D;              /* P x 3 */
    float* dL_dcov3D;                /* P x 6 or NULL */
    float* dL_dsh;                   /* P x M x 3 or NULL */
    float* dL_dscales;               /* P x 3 or NULL */
    float* dL_drotations;            /* P x 4 or NULL */
    int32_t raw;                     /* as in the forward; gradients are then w.r.t. the raw inputs */
    int32_t flags;                   /* lsr_backward_flags */
    const float* shs_rest;           /* as in the forward */
    float* dL_dsh_rest;              /* P x (M-1) x 3 when shs_rest is set (dL_dsh is then P x 1 x 3) */
    const float* dL_dloss;           /* NULL, or the device scalar dL/d(out_loss) of a forward that fused
                                        the loss: its gradient dL/dloss * sign(f m - gt m) * m / (3 H W)
                                        (autograd's) is added to dL_dout_language_feature (NULL = 0) */
    /* ABI 12: LangSplat's language step with its optimiser step fused into the backward's epilogue
     * (train.py:104 + 134-137 at N = 1, where nothing happens between the two: langsplat_amd.graph /
     * langsplat_amd.pipeline use it in their captured steps).  update != NULL needs the language-only
     * backward (every geometry output NULL, dL_dout_color NULL), raw & LSR_RAW_LANGUAGE and
     * update->param == language_feature.  Then, after the render backward, ONE pass per Gaussian reads
     * its gradient record, writes dL_dmeans2D and dL_dlanguage_feature as always, and applies the
     * Adam step of lsr_adam_multi (device form: update_step_dev is that call's step block, tensor 0;
     * update_skip its skip flag) to param / exp_avg / exp_avg_sq -- the same operations, so the same
     * values as lsr_backward followed by lsr_adam_multi.  fill_record (NULL: off) is the record array
     * (lsr_state_layout.record) of another forward's geometry buffer over the same P Gaussians: every
     * Gaussian's language slots there receive the activated updated feature (skipped or not), so that
     * forward's composite call (LSR_PHASE_COMPOSITE_FILLED) needs no fill of its own. */
    const struct lsr_adam_tensor* update;  /* (defined with lsr_adam_multi below) */
    int64_t* update_step_dev;
    const int32_t* update_skip;
    float* fill_record;
} lsr_backward_args;

/* Byte offsets of the internal state inside the forward buffers, for inspection by tests and
 * for debug dumps.  All arrays are tightly packed at the given offsets. */
typedef struct lsr_state_layout {
    /* geometry buffer */
    size_t depth_key;      /* uint32[P]  float bits of view depth, 0xFFFFFFFF if culled */
    size_t tiles_touched;  /* uint32[P] */
    size_t rect;           /* uint32[2P] (minx | miny << 16, maxx | maxy << 16) */
    size_t record;         /* float4[3P] {x, y, conic.x, conic.y}{conic.z, opacity, r, g}{b, f0, f1, f2} */
    size_t clamped;        /* uint32[P]  bit c = SH colour channel c clamped */
    size_t sorted_ids;     /* uint32[P]  Gaussians by (depth, id); culled ones tie with the farthest */
    size_t super_offset;   /* uint32[P]  first super-tile entry of the Gaussian of depth rank r */
    /* image buffer */
    size_t counters;       /* uint32[16] {reserved, num_rendered, error, forward flags, super entries, ...} */
    size_t ranges;         /* uint32[2T] [start, end) of each tile in point_list */
    size_t final_T;        /* float[H*W] */
    size_t n_contrib;      /* uint32[H*W] */
    /* binning buffer */
    size_t point_list;     /* uint32[num_rendered] Gaussian ids, tile-major, (depth, id) order;
                              entry k belongs to the tile t with ranges[t].x <= k < ranges[t].y */
    /* geometry buffer (ABI 16) */
    size_t grad_records;   /* float[5P] the language step's gradient records; after a backward with
                              LSR_BWD_DEFER_TAIL: float[3P] language partials, the skip word, 3 words,
                              then float[2P] dx, dy */
} lsr_state_layout;

int32_t lsr_abi_version(void);
const char* lsr_last_error(void);

/* Sizes (bytes) of the forward scratch buffers, exactly what lsr_forward requests for the geometry
 * and image buffers (the geometry buffer holds one fused-loss word per tile, so it depends on the
 * image size too); binning: an upper bound for any scene with num_rendered tile instances (the
 * forward requests the size its super-tile entry count needs, at most this). */
size_t lsr_geom_bytes(int32_t P, int32_t width, int32_t height);
size_t lsr_image_bytes(int32_t width, int32_t height);
size_t lsr_binning_bytes(int32_t width, int32_t height, int64_t num_rendered);
size_t lsr_backward_bytes(int32_t P);
int32_t lsr_state_layout_of(int32_t P, int32_t width, int32_t height, int64_t num_rendered,
                            lsr_state_layout* out);

/* _C.rasterize_gaussians: preprocess, depth sort, tile binning (super-tile lists + per-tile
 * ranks), front-to-back compositing.  Writes out_color, out_language_feature, radii and *num_rendered. */
int32_t lsr_forward(const lsr_settings* settings, const lsr_forward_args* args,
                    lsr_alloc_fn alloc, void* alloc_user, void* stream, int64_t* num_rendered);

/* _C.rasterize_gaussians_backward: back-to-front replay and per-Gaussian chain rule. */
int32_t lsr_backward(const lsr_settings* settings, const lsr_backward_args* args,
                     lsr_alloc_fn alloc, void* alloc_user, void* stream);

/* Per-stage device time, measured with HIP events recorded on the caller's stream around each
 * launch group while profiling is enabled (measurement support for bench.py; no reference
 * counterpart).  lsr_profile_enable(1) clears and starts, (0) stops; lsr_profile_report
 * synchronises the recorded events and returns the number of stages written to `out`. */
typedef struct lsr_kernel_stat {
    char name[32];
    int64_t launches;
    double total_ms;
} lsr_kernel_stat;

int32_t lsr_profile_enable(int32_t on);
int32_t lsr_profile_report(lsr_kernel_stat* out, int32_t capacity);
/* Restricts profiling to the comma-separated stage names (NULL or "" = every stage), so a timed
 * run can time its dominant kernel live without event overhead around the other stages. */
int32_t lsr_profile_select(const char* stages);
/* Records the events on every `every`-th launch of a selected stage only (default 1; reset by each
 * call): a timed run samples its dominant kernel's duration at a fraction of the events' cost. */
int32_t lsr_profile_sample(int32_t every);

/* _C.mark_visible: visible[i] = 1 iff Gaussian i passes the near-plane frustum test. */
int32_t lsr_mark_visible(int32_t P, const float* means3D, const float* viewmatrix,
                         const float* projmatrix, uint8_t* visible, void* stream);

/* The language slots of a forward's render records, from the parameter (ABI 14): for every Gaussian
 * with radii[i] > 0, record[i]'s three feature words receive language_feature[i] (activated as
 * the forward activates it when raw has LSR_RAW_LANGUAGE: normalised).  `record` is
 * lsr_state_layout.record of the geometry buffer of a forward made with phase LSR_PHASE_GEOMETRY
 * over the same P Gaussians, and radii that forward's radii.  What LSR_PHASE_COMPOSITE does before
 * compositing; a caller that changed the parameter after a fused update already filled the records
 * (lsr_backward_args.fill_record) refills them with this before a LSR_PHASE_COMPOSITE_FILLED call
 * (langsplat_amd/pipeline.py follow_caller). */
int32_t lsr_fill_language(int32_t P, const float* language_feature, int32_t raw, const int32_t* radii, float* record,
                          void* stream);

/* Measurement hook, not part of the reference interface: with LSR_RENDER_STATS=1 in the
 * environment the render backward counts, per wave-iteration over a culled list entry, [0]
 * entries, [1] entries passing the power test in some lane, [2] entries some lane blends, [3]
 * lanes blending, [8 + c] a histogram of lanes blending (c = 0..64).  Copies min(n, 73) counters
 * to host memory and clears them (synchronous). */
int32_t lsr_debug_render_stats(uint64_t* out, int32_t n);

/* Measurement hook, not part of the reference interface: with LSR_RENDER_STATS=1 the render
 * kernels (kernel 0 = forward, 1 = backward) record per workgroup b < n into out[11 b .. 11 b + 10]:
 * {start, end} (100 MHz wall clock, low 32 bits), the tile (-1: a workgroup that only filled empty
 * tiles), the hardware slot (XCC_ID << 16 | CU/SH/SE bits of HW_ID), and (forward) the ticks spent
 * loading, compacting and walking its batches, the batch count | the first batch's load ticks << 16,
 * and six milestones of the first batch in ticks after the start, two 16-bit fields per word
 * (begin, tile range loaded, first barrier, point-list ids loaded, records gathered, load phase
 * done; synchronous). */
int32_t lsr_debug_render_timeline(int32_t kernel, uint32_t* out, int32_t n);

/* Look-back stalls, not part of the reference interface.  The single-pass scans of the forward
 * (depth order, binning), of lsr_dist_cuda2 and the block-sum hand-off of lsr_masked_l1_forward wait
 * for values published by other workgroups.  A wait is bounded: after `limit` polls (default
 * 1 << 24) the waiting workgroup computes the value itself from the inputs -- the results are the
 * same, only slower -- and flags the event.  lsr_debug_scan_stalls returns 1 if a launch made by
 * the calling thread on the current device took that path since the last call (read it after the
 * work finished, e.g. after a stream synchronise), and clears the flag; negative on error.
 * lsr_debug_set_spin_limit sets the poll bound for launches made after it and returns the old one;
 * 0 makes every wait take the fallback at once (fault injection for tests). */
int32_t lsr_debug_scan_stalls(void);
uint32_t lsr_debug_set_spin_limit(uint32_t limit);

/* Measurement hook, not part of the reference interface: with LSR_BUCKET_TIMELINE=1 the MSD depth
 * sort's bucket kernel records per workgroup b < min(n, 256) into out[8 b .. 8 b + 7]: {start, end}
 * (100 MHz wall clock, low 32 bits), the hardware slot (XCC_ID << 16 | CU/SH/SE bits of HW_ID),
 * the bucket's key count, the end times of the first pass, of all passes and of the output gathers,
 * and the time the bucket's keys had arrived (synchronous). */
int32_t lsr_debug_bucket_timeline(uint32_t* out, int32_t n);
/* Measurement aid (ABI 14): a one-wave kernel on `stream` reads the shader-clock counter (s_memtime)
 * and the constant 100 MHz counter (s_memrealtime) before and after a ~20 us spin and stores the four
 * values into out_device[0..3] (a device array of 4 u64): the engine clock the chip ran at meanwhile
 * is 100 (out[3] - out[1]) / (out[2] - out[0]) MHz (tools/clock_probe.py). */
int32_t lsr_debug_clock_probe(uint64_t* out_device, void* stream);
/* Measurement aid (ABI 15): a one-wave kernel on `stream` that spins for `microseconds` (at most
 * 1e6) of the constant 100 MHz counter -- a delay between two launches of one stream (the
 * pipelined step's stream phase, LSR_PG_GEO_DELAY_US). */
int32_t lsr_debug_delay(uint32_t microseconds, void* stream);
/* Host runtime helper (ABI 17): `stream` waits for each of the n_waits events, then the
 * instantiated graph `graph_exec` (a hipGraphExec_t) is launched on it and, if record_event is not
 * null, that event recorded after it -- the stream-A half of a pipelined step's replay in one call
 * (langsplat_amd/pipeline.py PipelinedGraphStep.replay), replacing torch's stream context, event
 * waits and CUDAGraph.replay() in Python (~8 us of host time before every synced step's launch,
 * profiles/r06_sync_gap.txt).  No reference counterpart: the reference has no captured step. */
int32_t lsr_graph_launch(void* graph_exec, void* stream, void* const* wait_events, int32_t n_waits,
                         void* record_event);

/* ---- the language-feature loss around the rasterizer ----------------
 *
 * lsr_masked_l1_forward replaces, in LangSplat's include_feature step (train.py:97-98),
 *     Ll1 = l1_loss(language_feature * mask, gt_language_feature * mask)
 * with l1_loss = torch.abs(a - b).mean() (utils/loss_utils.py:17-18): one pass over
 * pred / gt (C x HW fp32) and mask (HW, bool bytes or fp32, broadcast over the C channels).
 * *loss (one float, device) = sum |pred*m - gt*m| / (C*HW), summed in a fixed order
 * (deterministic).  `scratch` holds lsr_masked_l1_scratch_bytes(C, HW) bytes, zeroed once
 * before its first use and then reused (one stream at a time per scratch).
 *
 * lsr_masked_l1_backward writes the gradient torch autograd produces for that expression:
 *     grad_pred = sign(pred*m - gt*m) * (grad_loss[0] / (C*HW)) * m
 * (grad_loss is the device scalar dL/dLl1), bit-identical to autograd's mean/abs/sub/mul chain.
 *
 * lsr_decode_language_feature restates Camera.get_language_feature (scene/cameras.py:58-92) on
 * the GPU: seg = seg_map[level] (L x H x W int64), mask = (seg != -1), feature = feature_map[seg]
 * (N x D fp32; index -1 reads the last row, as torch indexing does) written as D x H x W, and
 * mask as H x W bytes -- so a training loop can decode each view's map once and keep it in HBM
 * instead of np.load + CPU gather + H2D every step.  A segment id outside [-N, N) (the reference's
 * feature_map[seg] raises IndexError) returns LSR_ERR_INVALID; the call waits for its kernel to
 * find that out (once per view). */
/* ---- optimiser step --------------------------------------------------
 * One Adam step of torch.optim.Adam (amsgrad=False, weight_decay=0), the optimiser of
 * scene/gaussian_model.py:229 stepped at train.py:134-137, over one fp32 parameter tensor of n
 * elements: exp_avg / exp_avg_sq updated in place, then param.  `step` is the 1-based step count
 * after this update (torch's state["step"]); lr may change between calls (learning-rate
 * schedules, scene/gaussian_model.py:231-241). */
int32_t lsr_adam_step(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, double lr,
                      double beta1, double beta2, double eps, int64_t step, void* stream);

/* The same step for several tensors in ONE launch (RGB mode's six parameter groups,
 * scene/gaussian_model.py:219-226, each with its own lr, betas, eps and step count, i.e. torch's
 * per-parameter state).  Every gradient is multiplied by grad_scale first (e.g. the 1 / N of a
 * gradient all-reduced as a SUM over N ranks; 1 = none).
 * step_dev (device int64[LSR_ADAM_STEP_WORDS], ABI 12) replaces the tensors' step fields AND learning
 * rates for a step replayed from a HIP graph (at most 16 tensors then):
 *   step_dev[0]                      the step count;
 *   step_dev[1 .. 48]                scratch: a one-wave kernel first advances the count by one and
 *                                    writes that step's bias-corrected scalars of every tensor here,
 *                                    which the update reads;
 *   step_dev[LSR_ADAM_WORD_SKIPPED]  the number of steps skipped through `skip` (below);
 *   step_dev[LSR_ADAM_WORD_LR + k]   tensor k's learning rate (a double's bits), which the caller keeps
 *                                    current (a learning-rate schedule, scene/gaussian_model.py:231-241,
 *                                    changes it between replays without a re-capture); the table's lr
 *                                    is not read;
 *   a tensor's `step` field is then its OFFSET from the count (ABI 14): tensor k's step of a replay
 *   is step_dev[0] + 1 + tensors[k].step (0 when all counts are equal; torch's per-parameter counts
 *   differ after replace_tensor_to_optimizer, scene/gaussian_model.py:326-339, since the replaced
 *   group skips that iteration's step).  The offset must be > -2^40 and < 2^40.
 * step_dev NULL: the host's step counts and lrs.
 * skip (device int32, or NULL): when *skip != 0 at run time the launch changes nothing -- no
 * parameter, moment or step count -- and, with step_dev, adds one to the skipped count.  A captured
 * train step passes its rasterizer's capacity overflow flag (lsr_forward_args.overflow), so a view
 * that was not rasterized is a no-op for the optimiser, exactly as if it had been left out. */
#define LSR_ADAM_STEP_WORDS 66   /* count, 16 x 3 scalar words, skipped count, 16 lrs */
#define LSR_ADAM_WORD_SKIPPED 49
#define LSR_ADAM_WORD_LR 50
typedef struct lsr_adam_tensor {
    int64_t n;
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    double lr, beta1, beta2, eps;
    int64_t step;                /* 1-based, after this update */
} lsr_adam_tensor;
int32_t lsr_adam_multi(int32_t count, const lsr_adam_tensor* tensors, float grad_scale, int64_t* step_dev,
                       const int32_t* skip, void* stream);

/* The language step's update at N > 1 (ABI 15): lsr_adam_multi of ONE tensor -- the raw language
 * feature, P x 3 (tensor->n = 3 P), its gradient the all-reduced one (times grad_scale) -- in the
 * device form (step_dev and its learning-rate word 0 as lsr_adam_multi's; skip as there), which
 * also writes the updated feature (activated when raw has LSR_RAW_LANGUAGE) into the language
 * slots of fill_record, another forward's render records (lsr_state_layout.record; the same slots
 * lsr_backward_args.fill_record receives at N = 1), so that forward's composite phase runs as
 * LSR_PHASE_COMPOSITE_FILLED.  A skipped step still fills (with the unchanged feature).  Replaces
 * lsr_adam_multi + the fill of LSR_PHASE_COMPOSITE when the gradient all-reduce sits between the
 * backward and the update (langsplat_amd.pipeline.PipelinedGraphStep with a bucket). */
int32_t lsr_adam_fill_language(const lsr_adam_tensor* tensor, float grad_scale, int64_t* step_dev, const int32_t* skip,
                               void* fill_record, int32_t raw, void* stream);

/* The second half of a backward made with LSR_BWD_DEFER_TAIL (ABI 16): settings and args as passed
 * to that lsr_backward (same buffers, update, update_step_dev, update_skip, fill_record; flags may
 * keep LSR_BWD_DEFER_TAIL), after the caller reduced the records' language partials.  Launches the
 * Adam step advance and one pass per Gaussian: dL_dmeans2D, dL_dlanguage_feature, the Adam step and
 * the fill, as lsr_backward with update (not deferred) does after its render backward. */
int32_t lsr_language_tail(const lsr_settings* settings, const lsr_backward_args* args, void* stream);

/* Densification statistics of one rendered view, one pass (train.py:125-126 with
 * GaussianModel.add_densification_stats, scene/gaussian_model.py:480-482), for Gaussians with
 * radii > 0:  max_radii2D = max(max_radii2D, radii);  xyz_gradient_accum += ||dL_dmeans2D[:, :2]||;
 * denom += 1.  dL_dmeans2D is P x 3 (viewspace_points.grad); the three outputs are P floats each
 * (the reference's (P,) and (P, 1) tensors); any of them may be NULL (not updated). */
int32_t lsr_densification_stats(int32_t P, const int32_t* radii, const float* dL_dmeans2D, float* max_radii2D,
                                float* xyz_gradient_accum, float* denom, void* stream);

/* ---- point-cloud initialisation --------------------------------------
 * simple-knn's distCUDA2 (scene/gaussian_model.py:20,180): for each of the N points (N x 3 fp32),
 * the mean of the squared distances to its 3 nearest OTHER points (exact; a duplicate of a point
 * counts at distance 0; with N < 4 the missing neighbours count as FLT_MAX).  Scratch is requested
 * once through `alloc` (which = LSR_BUF_BACKWARD). */
int32_t lsr_dist_cuda2(int64_t N, const float* points, float* out_mean_dist, lsr_alloc_fn alloc, void* alloc_user,
                       void* stream);

size_t lsr_masked_l1_scratch_bytes(int32_t C, int64_t HW);
int32_t lsr_masked_l1_forward(int32_t C, int64_t HW, const float* pred, const float* gt, const void* mask,
                              int32_t mask_is_float, float* loss, void* scratch, void* stream);
int32_t lsr_masked_l1_backward(int32_t C, int64_t HW, const float* pred, const float* gt, const void* mask,
                               int32_t mask_is_float, const float* grad_loss, float* grad_pred, void* stream);
int32_t lsr_decode_language_feature(int32_t L, int32_t H, int32_t W, const int64_t* seg_map, int32_t level,
                                    int32_t N, int32_t D, const float* feature_map, float* out_feature,
                                    uint8_t* out_mask, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* LSR_H */
