// lsr_api.hip -- the extern "C" boundary of liblsr.so (declared in include/lsr.h).
//
// Orchestration mirrors the reference's two native entry points (see include/lsr.h for the
// call sites they replace): forward = preprocess -> depth sort -> tile counts/scan ->
// [one D2H read of num_rendered] -> emit -> per-tile order -> render; backward = render
// replay -> per-Gaussian chain rule.
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "lsr_internal.h"

using namespace lsr;

static thread_local std::string g_last_error;

// ------------------------------------------------------------------ host timeline (measurement)
// LSR_HOST_TRACE=1: host timestamps of each lsr_forward's phases, averaged and printed at exit
// (where the host spends the time between the counter hand-off and the next launches).
namespace {
struct HostTrace {
    bool on = false;
    static constexpr int kMarks = 7;
    const char* names[kMarks] = {"entry->preprocess", "->depth order", "->binning alloc", "->wait returned",
                                 "->binning enqueued", "->forward enqueued", "(unused)"};
    double acc[kMarks] = {};
    int64_t calls = 0;
    HostTrace()
    {
        const char* v = getenv("LSR_HOST_TRACE");
        on = v && v[0] == '1';
    }
    ~HostTrace()
    {
        if (!on || calls == 0) return;
        fprintf(stderr, "lsr host trace over %lld forwards (us):", (long long)calls);
        for (int i = 0; i < kMarks - 1; i++) fprintf(stderr, " %s %.2f", names[i], acc[i] / calls);
        fprintf(stderr, "\n");
    }
};
HostTrace g_host_trace;
inline double now_us()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}
struct HostMarks {
    double t[HostTrace::kMarks + 1];
    int n = 0;
    void mark()
    {
        if (g_host_trace.on && n <= HostTrace::kMarks) t[n++] = now_us();
    }
    ~HostMarks()
    {
        if (!g_host_trace.on || n < HostTrace::kMarks) return;
        for (int i = 0; i + 1 < n; i++) g_host_trace.acc[i] += t[i + 1] - t[i];
        g_host_trace.calls++;
    }
};
}  // namespace

// ------------------------------------------------------------------ opt-in event profiler
namespace {
// timing-only events: no system-scope fence (cache writeback + invalidate) when they are recorded,
// which would otherwise stall the stream around the measured launches (~6 us per step measured
// at C3 with the default flags)
constexpr unsigned kEventFlags = hipEventDisableSystemFence;
struct Pending {
    const char* name;
    hipEvent_t a, b;
};
struct Profiler {
    std::mutex mu;
    bool on = false;
    std::vector<std::string> select;  // empty: every stage
    int64_t every = 1, seen = 0;      // lsr_profile_sample: events on every `every`-th selected launch
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    std::map<std::string, std::pair<int64_t, double>> stats;

    hipEvent_t get()
    {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, kEventFlags) != hipSuccess) return nullptr;
        return e;
    }
    void drain()
    {
        for (auto& p : pending) {
            float ms = 0.f;
            if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
                auto& st = stats[p.name];
                st.first += 1;
                st.second += ms;
            }
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pending.clear();
    }
};
Profiler g_prof;

// Records an event pair around one launch group when profiling is on.
struct Scope {
    hipEvent_t a = nullptr, b = nullptr;
    const char* name;
    hipStream_t s;
    Scope(const char* n, hipStream_t st) : name(n), s(st)
    {
        std::lock_guard<std::mutex> g(g_prof.mu);
        if (!g_prof.on) return;
        if (!g_prof.select.empty()) {
            bool hit = false;
            for (const auto& x : g_prof.select) hit = hit || x == n;
            if (!hit) return;
        }
        if (g_prof.seen++ % g_prof.every != 0) return;
        a = g_prof.get();
        b = g_prof.get();
        if (a && b) (void)hipEventRecord(a, s);
    }
    ~Scope()
    {
        if (!a || !b) return;
        (void)hipEventRecord(b, s);
        std::lock_guard<std::mutex> g(g_prof.mu);
        g_prof.pending.push_back({name, a, b});
    }
};
}  // namespace

// ------------------------------------------------------------------ pinned host block
// Per (thread, device) pinned host memory the kernels write with system-scope stores:
//   slot[8]: the forward's one host wait -- a one-workgroup kernel publishes the counters, each with
//            the call's sequence number in one 64-bit store, and the host spins until all 8 slots
//            carry it (no pageable device-to-host copy, which is synchronous, and no
//            stream-synchronise wake-up latency);
//   stall:   set by a look-back that stopped waiting and took its fallback (lsr_debug_scan_stalls).
// Per thread, because a sequence number belongs to one caller; per device, because the block is
// written by that device's kernels.  Freed when the thread exits.
namespace {
struct HostBlock {
    uint64_t slot[8];  // {value, seq}: low word the counter, high word the sequence number
    uint32_t stall;
    uint32_t seq;      // the last sequence number used (host side)
    uint32_t bad_segment;  // lsr_decode_language_feature: a segment id outside [-N, N)
    int32_t depth_passes;  // depth-sort passes the last forward needed (0: none yet)
    // binning buffer size to request before the host wait (the last forward's, with headroom), for
    // the same P and image size; the exact size is requested after the wait if it is larger
    int32_t hint_P, hint_W, hint_H;
    size_t binning_hint;
};

struct HostBlocks {
    std::vector<std::pair<int, HostBlock*>> blocks;
    ~HostBlocks()
    {
        for (auto& b : blocks) (void)hipHostFree(b.second);
    }
    // the calling thread's block for the current device (allocated on first use); null on failure
    HostBlock* get(hipError_t* err)
    {
        int dev = 0;
        if ((*err = hipGetDevice(&dev)) != hipSuccess) return nullptr;
        for (auto& b : blocks)
            if (b.first == dev) return b.second;
        void* h = nullptr;
        if ((*err = hipHostMalloc(&h, sizeof(HostBlock), hipHostMallocCoherent)) != hipSuccess) return nullptr;
        memset(h, 0, sizeof(HostBlock));
        blocks.emplace_back(dev, static_cast<HostBlock*>(h));
        return static_cast<HostBlock*>(h);
    }
};
thread_local HostBlocks t_host;

bool counters_arrived(const HostBlock* hb, uint32_t seq)
{
    for (int i = 0; i < 8; i++)
        if ((uint32_t)(__atomic_load_n(&hb->slot[i], __ATOMIC_ACQUIRE) >> 32) != seq) return false;
    return true;
}

// Waits until the counters published with `seq` arrived; a HIP error on failure.  The stream is
// queried only after the first millisecond of waiting (then once per ~1 ms): a query costs tens of
// microseconds of host time, and counters landing during one were seen that much later.
hipError_t wait_counters(const HostBlock* hb, uint32_t seq, hipStream_t stream)
{
    if (counters_arrived(hb, seq)) return hipSuccess;
    double next_query = now_us() + 1000.0;
    for (uint64_t spin = 0;; spin++) {
        if (counters_arrived(hb, seq)) return hipSuccess;
        if ((spin & 255) == 255 && now_us() > next_query) {
            next_query = now_us() + 1000.0;
            const hipError_t q = hipStreamQuery(stream);
            if (q != hipSuccess && q != hipErrorNotReady) return q;
            if (q == hipSuccess) {  // stream idle: the stores must be visible now
                if (counters_arrived(hb, seq)) return hipSuccess;
                return hipErrorUnknown;
            }
        }
        __builtin_ia32_pause();
    }
}
}  // namespace

static int32_t fail(int32_t code, const char* what, hipError_t e = hipSuccess)
{
    char buf[512];
    if (e != hipSuccess)
        snprintf(buf, sizeof(buf), "%s: %s (%s)", what, hipGetErrorString(e), hipGetErrorName(e));
    else
        snprintf(buf, sizeof(buf), "%s", what);
    g_last_error = buf;
    return code;
}

#define LSR_TRY(expr, what)                                                  \
    do {                                                                     \
        hipError_t _e;                                                       \
        {                                                                    \
            Scope _scope(what, stream);                                      \
            _e = (expr);                                                     \
        }                                                                    \
        if (_e == hipSuccess && debug) _e = hipStreamSynchronize(stream);    \
        if (_e == hipSuccess && debug) _e = hipGetLastError();               \
        if (_e != hipSuccess) return fail(LSR_ERR_HIP, what, _e);            \
    } while (0)

static AdamScalars adam_scalars(double lr, double beta1, double beta2, double eps, int64_t step)
{
    // torch/optim/adam.py _single_tensor_adam: Python-float scalars, cast where they meet tensors
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    AdamScalars a;
    a.w1 = (float)(1.0 - beta1);
    a.beta2 = (float)beta2;
    a.w2 = (float)(1.0 - beta2);
    a.inv_bc2_sqrt = 1.0f / (float)sqrt(bc2);
    a.eps = (float)eps;
    a.neg_step_size = (float)(-(lr / bc1));
    return a;
}

// The render forward of lsr_forward (both modes), after the binning.
static int32_t render_forward_and_finish(const lsr_settings* s, const lsr_forward_args* a, const Layout& L, char* geom,
                                         char* image, char* binning, HostBlock* hb, hipStream_t stream, bool debug)
{
    const int P = a->P, W = s->image_width, H = s->image_height;
    (void)P;
    RenderParams rp{};
    rp.W = W;
    rp.H = H;
    rp.gx = L.gx;
    rp.gy = L.gy;
    rp.include_feature = (s->include_feature && a->language_feature) ? 1 : 0;
    rp.ranges = reinterpret_cast<const uint2*>(image + L.ranges);
    rp.point_list = reinterpret_cast<const uint32_t*>(binning + L.point_list);
    rp.cover = reinterpret_cast<uint8_t*>(binning + L.cover);
    rp.record = reinterpret_cast<const float4*>(geom + L.record);
    rp.bg = s->bg;
    rp.final_T = reinterpret_cast<float*>(image + L.final_T);
    rp.n_contrib = reinterpret_cast<uint32_t*>(image + L.n_contrib);
    rp.sched_counts = reinterpret_cast<uint32_t*>(image + L.counters);
    rp.sched_lists = reinterpret_cast<uint32_t*>(image + L.tile_lists);
    rp.split_pool = reinterpret_cast<float*>(image + L.split_pool);
    rp.split_desc = reinterpret_cast<uint4*>(image + L.split_desc);
    rp.out_color = a->out_color;
    rp.out_lang = a->out_language_feature;
    rp.split_color = (a->flags & LSR_FWD_NO_COLOR_GRAD) ? 0 : 1;
    // a composite phase runs beside another stream's geometry phase: fewer workgroups per CU
    rp.shared_cu = (a->phase == LSR_PHASE_COMPOSITE || a->phase == LSR_PHASE_COMPOSITE_FILLED) ? 1 : 0;
    if (a->flags & LSR_FWD_NO_BACKWARD) {  // inference: no split states, no backward work lists
        rp.no_bwd = 1;
        rp.split_pool = nullptr;
    }
    if (a->flags & LSR_FWD_ZERO_GRAD_RECORDS) {
        rp.zero_records = reinterpret_cast<float4*>(geom + L.grad_records);
        rp.zero_records_n4 = ((int64_t)P * kGradStrideLang + kDeferXyOffset + 3) / 4;
    }
    if (a->out_loss && rp.include_feature) {
        rp.loss_gt = a->loss_target;
        rp.loss_mask = a->loss_mask;
        rp.loss_code = reinterpret_cast<uint8_t*>(image + L.loss_code);
        rp.loss_words = reinterpret_cast<uint64_t*>(geom + L.loss_words);
        rp.out_loss = a->out_loss;
        rp.spin_limit = stall_spin_limit();
        rp.stall = &hb->stall;
    }
    LSR_TRY(launch_render_forward(rp, L.tiles, stream), "render forward");
    return LSR_OK;
}

extern "C" {

int32_t lsr_abi_version(void) { return LSR_ABI_VERSION; }

const char* lsr_last_error(void) { return g_last_error.c_str(); }

size_t lsr_geom_bytes(int32_t P, int32_t width, int32_t height) { return make_layout(P, width, height, 0, 0).geom_bytes; }

size_t lsr_image_bytes(int32_t width, int32_t height) { return make_layout(0, width, height, 0, 0).image_bytes; }

// every super-tile entry carries at least one tile instance, so E <= num_rendered
size_t lsr_binning_bytes(int32_t width, int32_t height, int64_t num_rendered)
{
    return make_layout(0, width, height, num_rendered, num_rendered).binning_bytes;
}

size_t lsr_backward_bytes(int32_t P) { return 4 * (size_t)kGradStride * (size_t)(P > 0 ? P : 1); }

int32_t lsr_state_layout_of(int32_t P, int32_t width, int32_t height, int64_t num_rendered, lsr_state_layout* out)
{
    if (!out || P < 0 || width < 0 || height < 0 || num_rendered < 0)
        return fail(LSR_ERR_INVALID, "lsr_state_layout_of: invalid argument");
    const Layout L = make_layout(P, width, height, num_rendered, 0);
    out->depth_key = L.depth_key;
    out->tiles_touched = L.tiles_touched;
    out->rect = L.rect;
    out->record = L.record;
    out->clamped = L.clamped;
    out->sorted_ids = L.sorted_ids;
    out->super_offset = L.super_offset;
    out->counters = L.counters;
    out->ranges = L.ranges;
    out->final_T = L.final_T;
    out->n_contrib = L.n_contrib;
    out->point_list = L.point_list;
    out->grad_records = L.grad_records;
    return LSR_OK;
}

// The deferred language feature (lsr_forward_args.language_ready): the feature's update (another
// stream) has overlapped everything enqueued so far; the stream waits for it, then the visible
// Gaussians' records receive the feature.  Inside a graph capture the event is one recorded in the
// same capture (a join of the two branches).
static hipError_t wait_and_fill_language(const lsr_forward_args* a, const Layout& L, char* geom, hipStream_t stream)
{
    hipError_t e = hipStreamWaitEvent(stream, static_cast<hipEvent_t>(a->language_ready), 0);
    if (e != hipSuccess) return e;
    return launch_fill_language(a->P, a->language_feature, a->raw, a->radii, reinterpret_cast<float4*>(geom + L.record),
                                stream);
}

int32_t lsr_forward(const lsr_settings* s, const lsr_forward_args* a, lsr_alloc_fn alloc, void* user,
                    void* stream_ptr, int64_t* num_rendered)
{
    if (!s || !a || !alloc || !num_rendered) return fail(LSR_ERR_INVALID, "lsr_forward: null argument");
    const int P = a->P, W = s->image_width, H = s->image_height;
    if (P < 0 || W <= 0 || H <= 0 || W > 65535 * kTile || H > 65535 * kTile)
        return fail(LSR_ERR_INVALID, "lsr_forward: invalid P or image size");
    if (s->sh_degree < 0 || s->sh_degree > 3) return fail(LSR_ERR_INVALID, "lsr_forward: sh_degree must be 0..3");
    if (!a->out_color || !a->out_language_feature || (P > 0 && (!a->radii || !a->means3D || !a->opacities)))
        return fail(LSR_ERR_INVALID, "lsr_forward: missing input/output pointer");
    if (P > 0 && (!a->shs) == (!a->colors_precomp))
        return fail(LSR_ERR_INVALID, "lsr_forward: provide exactly one of shs / colors_precomp");
    if (P > 0 && ((a->scales && a->rotations) ? 1 : 0) == (a->cov3D_precomp ? 1 : 0))
        return fail(LSR_ERR_INVALID, "lsr_forward: provide exactly one of scales+rotations / cov3D_precomp");
    if (a->shs && (a->M < (s->sh_degree + 1) * (s->sh_degree + 1)))
        return fail(LSR_ERR_INVALID, "lsr_forward: M smaller than (sh_degree+1)^2");
    if (!s->bg || !s->viewmatrix || !s->projmatrix || !s->campos)
        return fail(LSR_ERR_INVALID, "lsr_forward: settings tensors missing");
    if (a->raw & ~(LSR_RAW_OPACITY | LSR_RAW_SCALES | LSR_RAW_ROTATIONS | LSR_RAW_LANGUAGE))
        return fail(LSR_ERR_INVALID, "lsr_forward: unknown raw flag");
    if (a->flags & ~(LSR_FWD_ZERO_GRAD_RECORDS | LSR_FWD_NO_COLOR_GRAD | LSR_FWD_NO_BACKWARD))
        return fail(LSR_ERR_INVALID, "lsr_forward: unknown flag");
    if (a->shs_rest && (!a->shs || a->M < 2))
        return fail(LSR_ERR_INVALID, "lsr_forward: shs_rest needs shs (features_dc) and M >= 2");
    if (a->capacity_rendered < 0 || (a->capacity_rendered > 0 && a->capacity_entries <= 0) ||
        a->capacity_rendered > 0xFFFFFFFFll || a->capacity_entries > 0xFFFFFFFFll)
        return fail(LSR_ERR_INVALID, "lsr_forward: capacity mode needs capacity_rendered > 0 and capacity_entries > 0 "
                                     "(both < 2^32)");
    if (a->phase < LSR_PHASE_ALL || a->phase > LSR_PHASE_COMPOSITE_FILLED ||
        (a->phase != LSR_PHASE_ALL && (a->capacity_rendered <= 0 || a->language_ready)))
        return fail(LSR_ERR_INVALID, "lsr_forward: a forward phase needs capacity mode and no language_ready");
    if (a->out_num_entries) *a->out_num_entries = 0;
    if (a->out_loss && (!s->include_feature || (P > 0 && !a->language_feature) || !a->loss_target || !a->loss_mask))
        return fail(LSR_ERR_INVALID, "lsr_forward: the fused loss needs include_feature, language_feature, "
                                     "loss_target and loss_mask");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = s->debug != 0;
    *num_rendered = 0;
    const size_t HW = (size_t)W * H;
    if (P == 0) {
        // upstream leaves the images at their zero initialisation when there is nothing to draw
        LSR_TRY(zero_fill(a->out_color, 3 * HW * 4, stream), "memset color");
        LSR_TRY(zero_fill(a->out_language_feature, 3 * HW * 4, stream), "memset language");
        if (a->out_loss) {
            const Layout L0 = make_layout(0, W, H, 0, 0);
            char* image = static_cast<char*>(alloc(user, LSR_BUF_IMAGE, L0.image_bytes));
            if (!image) return fail(LSR_ERR_ALLOC, "lsr_forward: image buffer allocation failed");
            RenderParams rp{};
            rp.W = W;
            rp.H = H;
            rp.loss_gt = a->loss_target;
            rp.loss_mask = a->loss_mask;
            rp.loss_code = reinterpret_cast<uint8_t*>(image + L0.loss_code);
            rp.loss_partial = reinterpret_cast<double*>(image + L0.loss_partial);
            rp.out_loss = a->out_loss;
            LSR_TRY(launch_loss_background(rp, stream), "loss");
        }
        return LSR_OK;
    }

    HostMarks hm;
    hm.mark();
    Layout L = make_layout(P, W, H, 0, 0);
    if (L.supers > 65536) return fail(LSR_ERR_INVALID, "lsr_forward: image larger than 65536 super-tiles");
    hipError_t herr = hipSuccess;
    HostBlock* hb = t_host.get(&herr);
    if (!hb) return fail(LSR_ERR_HIP, "lsr_forward: pinned host block", herr);
    char* geom = static_cast<char*>(alloc(user, LSR_BUF_GEOM, L.geom_bytes));
    char* image = static_cast<char*>(alloc(user, LSR_BUF_IMAGE, L.image_bytes));
    if (!geom || !image) return fail(LSR_ERR_ALLOC, "lsr_forward: geometry/image buffer allocation failed");
    // no memset: k_publish_counters initialises every counter word before anything reads it
    uint32_t* counters = reinterpret_cast<uint32_t*>(image + L.counters);

    PreprocessParams pp{};
    pp.P = P;
    pp.M = a->M;
    pp.D = s->sh_degree;
    pp.W = W;
    pp.H = H;
    pp.gx = L.gx;
    pp.gy = L.gy;
    pp.tanfovx = s->tanfovx;
    pp.tanfovy = s->tanfovy;
    pp.focal_y = (float)H / (2.0f * s->tanfovy);
    pp.focal_x = (float)W / (2.0f * s->tanfovx);
    pp.scale_modifier = s->scale_modifier;
    pp.include_feature = s->include_feature;
    pp.prefiltered = s->prefiltered;
    pp.means = a->means3D;
    pp.shs = a->shs;
    pp.colors = a->colors_precomp;
    pp.lang = a->language_feature;
    pp.opac = a->opacities;
    pp.scales = a->scales;
    pp.rots = a->rotations;
    pp.cov_pre = a->cov3D_precomp;
    pp.view = s->viewmatrix;
    pp.proj = s->projmatrix;
    pp.campos = s->campos;
    pp.radii = a->radii;
    pp.visible = a->visible;
    pp.depth_key = reinterpret_cast<uint32_t*>(geom + L.depth_key);
    pp.tiles = reinterpret_cast<uint32_t*>(geom + L.tiles_touched);
    pp.rect = reinterpret_cast<uint32_t*>(geom + L.rect);
    pp.clamped = reinterpret_cast<uint32_t*>(geom + L.clamped);
    pp.record = reinterpret_cast<float4*>(geom + L.record);
    pp.counters = counters;
    pp.zero = reinterpret_cast<uint32_t*>(geom + L.scan_regions);
    pp.zero_words = (int)L.zero_words;  // depth-sort scan status and the fused loss's words
    // placed emission (the MSD depth order's fused emission at super-tile-major positions)
    const bool placed = !depth_order_uses_pass_count(P) && placed_emit(L, a->phase == LSR_PHASE_GEOMETRY, msd_digits(P));
    if (placed) {  // the bucket sort's count table
        pp.zero2 = reinterpret_cast<uint32_t*>(geom + L.sup_status);
        pp.zero2_words = (int)sup_words(msd_digits(P));
    }
    pp.raw = a->raw;
    pp.shs_rest = a->shs_rest;
    pp.partial = reinterpret_cast<uint4*>(geom + L.pre_partial);
    // deferred language feature: geometry first, the feature after the caller's event (or, split in
    // phases, in the composite call)
    const bool deferred = (a->language_ready || a->phase != LSR_PHASE_ALL) && s->include_feature && a->language_feature;
    pp.lang_deferred = deferred ? 1 : 0;
    if (a->phase == LSR_PHASE_COMPOSITE || a->phase == LSR_PHASE_COMPOSITE_FILLED) {
        // the geometry call's buffers (same allocator keys and sizes): the feature (unless a fused
        // update already wrote it, LSR_PHASE_COMPOSITE_FILLED), then the compositing
        const int64_t R_cap = a->capacity_rendered;
        const int64_t E_cap = !depth_order_uses_pass_count(P) ? std::min<int64_t>(a->capacity_entries, L.fused_cap)
                                                                : a->capacity_entries;
        L = make_layout(P, W, H, R_cap, E_cap);
        char* binning = static_cast<char*>(alloc(user, LSR_BUF_BINNING, L.binning_bytes));
        if (!binning) return fail(LSR_ERR_ALLOC, "lsr_forward: binning buffer allocation failed");
        *num_rendered = R_cap;
        if (deferred && a->phase == LSR_PHASE_COMPOSITE)
            LSR_TRY(launch_fill_language(P, a->language_feature, a->raw, a->radii,
                                         reinterpret_cast<float4*>(geom + L.record), stream),
                    "fill language");
        return render_forward_and_finish(s, a, L, geom, image, binning, hb, stream, debug);
    }
    LSR_TRY(launch_preprocess(pp, stream), "preprocess");
    hm.mark();

    // The one host wait: num_rendered R and the super-tile entries E size the binning buffer, and
    // the visible depth-key range fixes the number of depth-sort passes.  The depth sort is enqueued
    // BEFORE the wait, with this thread's last pass count: it reads the key range on the device, and
    // any pass count >= the needed one gives the same order (the extra digits are all 0), so the GPU
    // sorts while the host waits, instead of idling until the host has enqueued the next launch.
    // Should the range need more passes than guessed, the sort is run again below.
    const uint32_t fwd_flags = ((a->flags & LSR_FWD_ZERO_GRAD_RECORDS) ? kFwdZeroedRecords : 0u) |
                               ((a->out_loss && s->include_feature && a->language_feature) ? kFwdFusedLoss : 0u) |
                               ((a->flags & LSR_FWD_NO_COLOR_GRAD) ? kFwdNoColorState : 0u) |
                               ((a->flags & LSR_FWD_NO_BACKWARD) ? kFwdNoBackward : 0u);
    if (a->capacity_rendered > 0) {
        // Capacity mode: nothing waits for the device.  The counters stay on the device, the binning's
        // grids and buffers come from the capacities and its kernels read the true counts; a view over
        // capacity sets counters[kCntOverflow] (and *overflow) and is not binned.
        const int64_t R_cap = a->capacity_rendered;
        const bool fused = !depth_order_uses_pass_count(P);
        const int64_t E_cap = fused ? std::min<int64_t>(a->capacity_entries, L.fused_cap) : a->capacity_entries;
        // LSD order (large P): the passes this thread's last eager forward needed (its key range is
        // not read on the host here; a view that needs more is flagged as over capacity)
        const int passes = fused ? 0 : (hb->depth_passes > 0 ? hb->depth_passes : 4);
        LSR_TRY(launch_publish_counters((P + kPreThreads - 1) / kPreThreads, pp.partial, counters, nullptr, 0,
                                        fwd_flags, (uint32_t)R_cap, (uint32_t)E_cap, a->overflow, passes, stream),
                "publish counters");
        LSR_TRY(launch_depth_order(P, fused ? 4 : passes, L, geom, counters, &hb->stall, stream, debug, fused,
                                   (uint32_t)E_cap, placed),
                "depth order");
        L = make_layout(P, W, H, R_cap, E_cap);
        char* binning = static_cast<char*>(alloc(user, LSR_BUF_BINNING, L.binning_bytes));
        if (!binning) return fail(LSR_ERR_ALLOC, "lsr_forward: binning buffer allocation failed");
        LSR_TRY(launch_binning(P, R_cap, L, geom, image, binning, &hb->stall, stream, debug, fused,
                               DevCount{counters + kCntSuper, counters + kCntOverflow}, placed),
                "binning");
        *num_rendered = R_cap;
        if (a->phase == LSR_PHASE_GEOMETRY) return LSR_OK;
        if (deferred) LSR_TRY(wait_and_fill_language(a, L, geom, stream), "fill language");
        return render_forward_and_finish(s, a, L, geom, image, binning, hb, stream, debug);
    }
    const uint32_t seq = ++hb->seq == 0 ? ++hb->seq : hb->seq;
    LSR_TRY(launch_publish_counters((P + kPreThreads - 1) / kPreThreads, pp.partial, counters, hb->slot, seq,
                                    fwd_flags, 0u, 0u, nullptr, 0, stream),
            "publish counters");
    const int guess = hb->depth_passes > 0 ? hb->depth_passes : 4;
    // MSD path: the bucket sort also emits the super-tile entries (into geometry arrays of fixed
    // capacity, so no host value is needed); used below when they fitted
    const bool fused_emit = !depth_order_uses_pass_count(P) && fused_emit_enabled();
    LSR_TRY(launch_depth_order(P, guess, L, geom, counters, &hb->stall, stream, debug, fused_emit, 0, placed),
            "depth order");
    hm.mark();
    // the binning buffer from the last forward's size while the GPU works (the allocator callback
    // is host work that would otherwise sit between the wait and the binning launches)
    char* binning = nullptr;
    size_t binning_have = 0;
    if (hb->binning_hint && hb->hint_P == P && hb->hint_W == W && hb->hint_H == H) {
        binning = static_cast<char*>(alloc(user, LSR_BUF_BINNING, hb->binning_hint));
        binning_have = binning ? hb->binning_hint : 0;
    }
    hm.mark();
    LSR_TRY(wait_counters(hb, seq, stream), "wait counters");
    hm.mark();
    uint32_t host_cnt[8];
    for (int i = 0; i < 8; i++) host_cnt[i] = (uint32_t)hb->slot[i];
    if (host_cnt[kCntError] && s->prefiltered)
        return fail(LSR_ERR_PREFILTERED, "lsr_forward: prefiltered=True but a Gaussian is outside the frustum");
    const int64_t R = host_cnt[kCntRendered];
    *num_rendered = R;
    if (a->out_num_entries) *a->out_num_entries = (int64_t)host_cnt[kCntSuper];
    if (R > 0) {
        // sort only the bits the visible keys span (key - min <= max - min)
        const uint32_t span = host_cnt[kCntKeyMax] - host_cnt[kCntKeyMin];
        int bits = 0;
        while (bits < 32 && (span >> bits) != 0) bits++;
        const int passes = bits <= 8 ? 1 : (bits + 7) / 8;
        if (depth_order_uses_pass_count(P)) hb->depth_passes = passes;
        if (depth_order_uses_pass_count(P) && passes > guess) {  // short guess: clear the scan status, sort again
            LSR_TRY(zero_fill(geom + L.scan_regions, 4 * kDepthScans * L.scan_region_geom, stream),
                    "clear scan status");
            LSR_TRY(launch_depth_order(P, passes, L, geom, counters, &hb->stall, stream, debug), "depth order");
        }
    }

    const bool emitted = fused_emit && (int64_t)host_cnt[kCntSuper] <= L.fused_cap;
    if (fused_emit && !emitted) {  // entries beyond the fused capacity: the depth order again, unfused
        LSR_TRY(zero_fill(geom + L.scan_regions, 4 * L.zero_words, stream), "clear scan status");
        LSR_TRY(launch_depth_order(P, guess, L, geom, counters, &hb->stall, stream, debug, false), "depth order");
    }
    L = make_layout(P, W, H, R, (int64_t)host_cnt[kCntSuper]);
    if (!binning || L.binning_bytes > binning_have) {
        binning = static_cast<char*>(alloc(user, LSR_BUF_BINNING, L.binning_bytes));
        if (!binning) return fail(LSR_ERR_ALLOC, "lsr_forward: binning buffer allocation failed");
    }
    hb->hint_P = P;
    hb->hint_W = W;
    hb->hint_H = H;
    hb->binning_hint = L.binning_bytes + L.binning_bytes / 8;  // 12.5 % headroom for the next view
    LSR_TRY(launch_binning(P, R, L, geom, image, binning, &hb->stall, stream, debug, emitted, DevCount{nullptr, nullptr},
                           placed),
            "binning");
    if (deferred) LSR_TRY(wait_and_fill_language(a, L, geom, stream), "fill language");
    hm.mark();
    const int32_t rc = render_forward_and_finish(s, a, L, geom, image, binning, hb, stream, debug);
    hm.mark();
    return rc;
}

int32_t lsr_backward(const lsr_settings* s, const lsr_backward_args* a, lsr_alloc_fn alloc, void* user,
                     void* stream_ptr)
{
    if (!s || !a || !alloc) return fail(LSR_ERR_INVALID, "lsr_backward: null argument");
    const int P = a->P, W = s->image_width, H = s->image_height;
    if (P < 0 || W <= 0 || H <= 0) return fail(LSR_ERR_INVALID, "lsr_backward: invalid P or image size");
    // geometry outputs: all given (full backward) or all NULL (screen-space + language only)
    const bool geometry = a->dL_dcolors || a->dL_dopacity || a->dL_dmeans3D || a->dL_dcov3D || a->dL_dsh ||
                          a->dL_dsh_rest || a->dL_dscales || a->dL_drotations;
    if (geometry) {
        if (!a->dL_dmeans2D || !a->dL_dcolors || !a->dL_dlanguage_feature || !a->dL_dopacity || !a->dL_dmeans3D)
            return fail(LSR_ERR_INVALID, "lsr_backward: missing output pointer");
        if ((a->shs && !a->dL_dsh) || (a->cov3D_precomp && !a->dL_dcov3D))
            return fail(LSR_ERR_INVALID, "lsr_backward: missing dL_dsh / dL_dcov3D output");
    }
    if (a->raw & ~(LSR_RAW_OPACITY | LSR_RAW_SCALES | LSR_RAW_ROTATIONS | LSR_RAW_LANGUAGE))
        return fail(LSR_ERR_INVALID, "lsr_backward: unknown raw flag");
    if (a->flags & ~(LSR_BWD_RECORDS_ZEROED | LSR_BWD_SHARED_CU | LSR_BWD_DEFER_TAIL))
        return fail(LSR_ERR_INVALID, "lsr_backward: unknown flag");
    const bool defer = (a->flags & LSR_BWD_DEFER_TAIL) != 0;
    if (defer && !a->update) return fail(LSR_ERR_INVALID, "lsr_backward: LSR_BWD_DEFER_TAIL needs update");
    if (geometry && a->shs_rest && (!a->shs || a->M < 2 || !a->dL_dsh_rest))
        return fail(LSR_ERR_INVALID, "lsr_backward: shs_rest needs shs, M >= 2 and dL_dsh_rest");
    if ((a->raw & LSR_RAW_OPACITY) && P > 0 && !a->opacities)
        return fail(LSR_ERR_INVALID, "lsr_backward: raw opacities missing");
    if (a->update) {
        const lsr_adam_tensor& u = *a->update;
        if (geometry || a->dL_dout_color || !(a->raw & LSR_RAW_LANGUAGE) || !s->include_feature || !a->language_feature ||
            u.param != a->language_feature || u.n != 3 * (int64_t)P || !u.exp_avg || !u.exp_avg_sq ||
            !a->update_step_dev || !a->dL_dlanguage_feature)
            return fail(LSR_ERR_INVALID, "lsr_backward: a fused update needs the language-only backward of the raw "
                                         "language feature (update->param), its moments, a step block and "
                                         "dL_dlanguage_feature");
    } else if (a->fill_record || a->update_step_dev || a->update_skip) {
        return fail(LSR_ERR_INVALID, "lsr_backward: fill_record / update_step_dev / update_skip need update");
    }
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = s->debug != 0;
    if (P == 0) return LSR_OK;
    if (!a->geom_buffer || !a->image_buffer || !a->binning_buffer || !a->radii)
        return fail(LSR_ERR_INVALID, "lsr_backward: missing forward state");
    const Layout L = make_layout(P, W, H, a->num_rendered, 0);  // point_list sits at offset 0
    char* geom = static_cast<char*>(a->geom_buffer);
    char* image = static_cast<char*>(a->image_buffer);
    char* binning = static_cast<char*>(a->binning_buffer);
    if (debug) {
        // what the forward prepared (counters[kCntFwdFlags]; the render backward clears the records
        // bit, so a second backward cannot reuse accumulated records)
        uint32_t ff = 0;
        LSR_TRY(hipMemcpyAsync(&ff, image + L.counters + 4 * kCntFwdFlags, 4, hipMemcpyDeviceToHost, stream),
                "read forward flags");
        LSR_TRY(hipStreamSynchronize(stream), "read forward flags");
        if ((a->flags & LSR_BWD_RECORDS_ZEROED) && !(ff & kFwdZeroedRecords))
            return fail(LSR_ERR_INVALID, "lsr_backward: LSR_BWD_RECORDS_ZEROED, but the forward did not clear the "
                                         "records (LSR_FWD_ZERO_GRAD_RECORDS) or they were used by a backward");
        if (a->dL_dloss && !(ff & kFwdFusedLoss))
            return fail(LSR_ERR_INVALID, "lsr_backward: dL_dloss, but the forward did not fuse the loss");
        if (a->dL_dout_color && (ff & kFwdNoColorState))
            return fail(LSR_ERR_INVALID, "lsr_backward: dL_dout_color, but the forward was told no colour gradient "
                                         "follows (LSR_FWD_NO_COLOR_GRAD)");
        if (ff & kFwdNoBackward)
            return fail(LSR_ERR_INVALID, "lsr_backward: the forward was told no backward follows (LSR_FWD_NO_BACKWARD)");
    }
    // the render backward's 5-value form (no geometry, no colour gradient) keeps 20-B records; the
    // first backward of a forward that cleared them (LSR_FWD_ZERO_GRAD_RECORDS) uses them directly
    const bool compact = !geometry && !a->dL_dout_color;
    const int stride = compact ? kGradStrideLang : kGradStride;
    float* grad = nullptr;
    if (compact && (a->flags & LSR_BWD_RECORDS_ZEROED)) {
        grad = reinterpret_cast<float*>(geom + L.grad_records);
    } else if (defer) {  // (update implies the compact form) the records stay for lsr_language_tail
        grad = reinterpret_cast<float*>(geom + L.grad_records);
        LSR_TRY(zero_fill(grad, 4 * ((size_t)kGradStrideLang * (size_t)P + kDeferXyOffset), stream),
                "memset grad records");
    } else {
        grad = static_cast<float*>(alloc(user, LSR_BUF_BACKWARD, lsr_backward_bytes(P)));
        if (!grad) return fail(LSR_ERR_ALLOC, "lsr_backward: gradient scratch allocation failed");
        LSR_TRY(zero_fill(grad, 4 * (size_t)stride * (size_t)P, stream), "memset grad");
    }

    RenderParams rp{};
    rp.W = W;
    rp.H = H;
    rp.gx = L.gx;
    rp.gy = L.gy;
    rp.include_feature = (s->include_feature && a->language_feature) ? 1 : 0;
    rp.ranges = reinterpret_cast<const uint2*>(image + L.ranges);
    rp.point_list = reinterpret_cast<const uint32_t*>(binning + L.point_list);
    rp.cover = reinterpret_cast<uint8_t*>(binning + L.cover);
    rp.record = reinterpret_cast<const float4*>(geom + L.record);
    rp.bg = s->bg;
    rp.final_T = reinterpret_cast<float*>(image + L.final_T);
    rp.n_contrib = reinterpret_cast<uint32_t*>(image + L.n_contrib);
    rp.sched_counts = reinterpret_cast<uint32_t*>(image + L.counters);
    rp.sched_lists = reinterpret_cast<uint32_t*>(image + L.tile_lists);
    rp.split_pool = reinterpret_cast<float*>(image + L.split_pool);
    rp.split_desc = reinterpret_cast<uint4*>(image + L.split_desc);
    rp.dL_dcolor = a->dL_dout_color;
    rp.dL_dlang = a->dL_dout_language_feature;
    rp.dL_dloss = a->dL_dloss;
    rp.loss_code = reinterpret_cast<uint8_t*>(image + L.loss_code);
    rp.grad = grad;
    if (defer) {  // planar records (LSR_BWD_DEFER_TAIL), the skip flag after the language partials
        rp.grad_xy = grad + 3 * (size_t)P + kDeferXyOffset;
        rp.flag_src = a->update_skip;
        rp.flag_dst = reinterpret_cast<int32_t*>(grad + 3 * (size_t)P);
    }
    rp.fwd_flags = reinterpret_cast<uint32_t*>(image + L.counters) + kCntFwdFlags;
    rp.geo = geometry ? 1 : 0;
    rp.shared_cu = (a->flags & LSR_BWD_SHARED_CU) ? 1 : 0;
    if (a->num_rendered > 0) {
        LSR_TRY(launch_render_backward(rp, L.tiles, stream), "render backward");
    } else if (defer) {  // no render backward: the flag word by a copy
        if (a->update_skip)
            LSR_TRY(hipMemcpyAsync(rp.flag_dst, a->update_skip, 4, hipMemcpyDeviceToDevice, stream), "copy skip flag");
        else
            LSR_TRY(zero_fill(rp.flag_dst, 4, stream), "clear skip flag");
    }
    if (a->update) {
        if (defer) return LSR_OK;  // lsr_language_tail runs the rest after the caller's all-reduce
        // the language step's tail in one pass: epilogue + Adam (+ the next forward's feature slots)
        const lsr_adam_tensor& u = *a->update;
        AdamHyper h{u.lr, u.beta1, u.beta2, u.eps, u.step};
        LSR_TRY(launch_language_tail(P, a->radii, grad, const_cast<float*>(a->language_feature), u.exp_avg, u.exp_avg_sq,
                                     a->dL_dmeans2D, a->dL_dlanguage_feature, h, a->update_step_dev, a->update_skip,
                                     reinterpret_cast<float4*>(a->fill_record), 0, stream),
                "language tail");
        return LSR_OK;
    }
    if (!geometry) {
        LSR_TRY(launch_grad_epilogue(P, a->radii, grad, stride, a->language_feature,
                                     (a->raw & LSR_RAW_LANGUAGE) ? 1 : 0, a->dL_dmeans2D,
                                     rp.include_feature ? a->dL_dlanguage_feature : nullptr, stream),
                "gradient epilogue");
        if (!rp.include_feature && a->dL_dlanguage_feature)
            LSR_TRY(zero_fill(a->dL_dlanguage_feature, (size_t)P * 3 * 4, stream), "memset dlang");
        return LSR_OK;
    }

    PreprocessBwdParams bp{};
    bp.P = P;
    bp.M = a->M;
    bp.D = s->sh_degree;
    bp.W = W;
    bp.H = H;
    bp.tanfovx = s->tanfovx;
    bp.tanfovy = s->tanfovy;
    bp.focal_y = (float)H / (2.0f * s->tanfovy);
    bp.focal_x = (float)W / (2.0f * s->tanfovx);
    bp.scale_modifier = s->scale_modifier;
    bp.means = a->means3D;
    bp.shs = a->shs;
    bp.scales = a->scales;
    bp.rots = a->rotations;
    bp.cov_pre = a->cov3D_precomp;
    bp.view = s->viewmatrix;
    bp.proj = s->projmatrix;
    bp.campos = s->campos;
    bp.radii = a->radii;
    bp.clamped = reinterpret_cast<const uint32_t*>(geom + L.clamped);
    bp.grad = grad;
    bp.dmeans2D = a->dL_dmeans2D;
    bp.dcolors = a->dL_dcolors;
    bp.dlang = a->dL_dlanguage_feature;
    bp.dopac = a->dL_dopacity;
    bp.dmeans3D = a->dL_dmeans3D;
    bp.dcov = a->dL_dcov3D;
    bp.dsh = a->shs ? a->dL_dsh : nullptr;
    bp.dscales = a->dL_dscales;
    bp.drots = a->dL_drotations;
    bp.raw = a->raw;
    bp.opac = a->opacities;
    bp.lang = a->language_feature;
    bp.shs_rest = a->shs_rest;
    bp.dsh_rest = a->dL_dsh_rest;
    if (!a->shs && a->dL_dsh && a->M > 0)
        LSR_TRY(zero_fill(a->dL_dsh, (size_t)P * a->M * 3 * 4, stream), "memset dsh");
    LSR_TRY(launch_preprocess_backward(bp, stream), "preprocess backward");
    return LSR_OK;
}

int32_t lsr_profile_enable(int32_t on)
{
    std::lock_guard<std::mutex> g(g_prof.mu);
    g_prof.drain();
    if (on) {
        g_prof.stats.clear();
        // events come from a pool filled here, not created inside the measured launches
        while (g_prof.pool.size() < 512) {
            hipEvent_t e = nullptr;
            if (hipEventCreateWithFlags(&e, kEventFlags) != hipSuccess) break;
            g_prof.pool.push_back(e);
        }
    }
    g_prof.on = on != 0;
    return LSR_OK;
}

int32_t lsr_profile_sample(int32_t every)
{
    if (every < 1) return fail(LSR_ERR_INVALID, "lsr_profile_sample: every must be >= 1");
    std::lock_guard<std::mutex> g(g_prof.mu);
    g_prof.every = every;
    g_prof.seen = 0;
    return LSR_OK;
}

int32_t lsr_profile_select(const char* stages)
{
    std::lock_guard<std::mutex> g(g_prof.mu);
    g_prof.select.clear();
    if (!stages) return LSR_OK;
    std::string cur;
    for (const char* c = stages;; c++) {
        if (*c == ',' || *c == 0) {
            if (!cur.empty()) g_prof.select.push_back(cur);
            cur.clear();
            if (*c == 0) break;
        } else {
            cur.push_back(*c);
        }
    }
    return LSR_OK;
}

int32_t lsr_profile_report(lsr_kernel_stat* out, int32_t capacity)
{
    std::lock_guard<std::mutex> g(g_prof.mu);
    g_prof.drain();
    int32_t n = 0;
    for (auto& kv : g_prof.stats) {
        if (out && n < capacity) {
            memset(out[n].name, 0, sizeof(out[n].name));
            strncpy(out[n].name, kv.first.c_str(), sizeof(out[n].name) - 1);
            out[n].launches = kv.second.first;
            out[n].total_ms = kv.second.second;
        }
        n++;
    }
    return n;
}

int32_t lsr_debug_render_stats(uint64_t* out, int32_t n)
{
    if (!out || n <= 0) return fail(LSR_ERR_INVALID, "lsr_debug_render_stats: invalid argument");
    const bool debug = false;
    hipStream_t stream = nullptr;
    (void)stream;
    LSR_TRY(render_stats_read(reinterpret_cast<unsigned long long*>(out), n), "render stats");
    return LSR_OK;
}

int32_t lsr_debug_render_timeline(int32_t kernel, uint32_t* out, int32_t n)
{
    if (!out || n <= 0 || kernel < 0 || kernel > 1)
        return fail(LSR_ERR_INVALID, "lsr_debug_render_timeline: invalid argument");
    const bool debug = false;
    hipStream_t stream = nullptr;
    (void)stream;
    LSR_TRY(render_timeline_read(out, kernel, n), "render timeline");
    return LSR_OK;
}

int32_t lsr_debug_scan_stalls(void)
{
    hipError_t herr = hipSuccess;
    HostBlock* hb = t_host.get(&herr);
    if (!hb) return -fail(LSR_ERR_HIP, "lsr_debug_scan_stalls: pinned host block", herr);
    return (int32_t)__atomic_exchange_n(&hb->stall, 0u, __ATOMIC_ACQ_REL);
}

uint32_t lsr_debug_set_spin_limit(uint32_t limit) { return set_stall_spin_limit(limit); }

int32_t lsr_debug_bucket_timeline(uint32_t* out, int32_t n)
{
    if (!out || n <= 0) return fail(LSR_ERR_INVALID, "lsr_debug_bucket_timeline: invalid argument");
    const bool debug = false;
    hipStream_t stream = nullptr;
    (void)stream;
    LSR_TRY(bucket_timeline_read(out, n), "bucket timeline");
    return LSR_OK;
}

int32_t lsr_debug_clock_probe(uint64_t* out_device, void* stream_ptr)
{
    if (!out_device) return fail(LSR_ERR_INVALID, "lsr_debug_clock_probe: invalid argument");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    LSR_TRY(launch_clock_probe(out_device, stream), "clock probe");
    return LSR_OK;
}

int32_t lsr_debug_delay(uint32_t microseconds, void* stream_ptr)
{
    if (microseconds > 1000000u) return fail(LSR_ERR_INVALID, "lsr_debug_delay: at most one second");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    LSR_TRY(launch_delay(100u * microseconds, stream), "delay");
    return LSR_OK;
}

int32_t lsr_graph_launch(void* graph_exec, void* stream_ptr, void* const* wait_events, int32_t n_waits,
                         void* record_event)
{
    if (!graph_exec || n_waits < 0 || (n_waits > 0 && !wait_events))
        return fail(LSR_ERR_INVALID, "lsr_graph_launch: invalid argument");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    hipError_t e;
    for (int32_t i = 0; i < n_waits; i++)
        if ((e = hipStreamWaitEvent(stream, reinterpret_cast<hipEvent_t>(wait_events[i]), 0)) != hipSuccess)
            return fail(LSR_ERR_HIP, "lsr_graph_launch: stream wait", e);
    if ((e = hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(graph_exec), stream)) != hipSuccess)
        return fail(LSR_ERR_HIP, "lsr_graph_launch: graph launch", e);
    if (record_event && (e = hipEventRecord(reinterpret_cast<hipEvent_t>(record_event), stream)) != hipSuccess)
        return fail(LSR_ERR_HIP, "lsr_graph_launch: event record", e);
    return LSR_OK;
}

int32_t lsr_mark_visible(int32_t P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                         uint8_t* visible, void* stream_ptr)
{
    if (P < 0 || (P > 0 && (!means3D || !viewmatrix || !projmatrix || !visible)))
        return fail(LSR_ERR_INVALID, "lsr_mark_visible: invalid argument");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    LSR_TRY(launch_mark_visible(P, means3D, viewmatrix, projmatrix, visible, stream), "mark visible");
    return LSR_OK;
}

int32_t lsr_fill_language(int32_t P, const float* language_feature, int32_t raw, const int32_t* radii, float* record,
                          void* stream_ptr)
{
    if (P < 0 || (P > 0 && (!language_feature || !radii || !record)) ||
        (reinterpret_cast<uintptr_t>(record) & 15) != 0)
        return fail(LSR_ERR_INVALID, "lsr_fill_language: invalid argument");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    LSR_TRY(launch_fill_language(P, language_feature, raw, radii, reinterpret_cast<float4*>(record), stream),
            "fill language");
    return LSR_OK;
}

size_t lsr_masked_l1_scratch_bytes(int32_t C, int64_t HW)
{
    (void)C;
    (void)HW;
    return masked_l1_scratch_bytes();
}

int32_t lsr_masked_l1_forward(int32_t C, int64_t HW, const float* pred, const float* gt, const void* mask,
                              int32_t mask_is_float, float* loss, void* scratch, void* stream_ptr)
{
    if (C <= 0 || HW <= 0 || !pred || !gt || !mask || !loss || !scratch)
        return fail(LSR_ERR_INVALID, "lsr_masked_l1_forward: invalid argument");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    hipError_t herr = hipSuccess;
    HostBlock* hb = t_host.get(&herr);
    if (!hb) return fail(LSR_ERR_HIP, "lsr_masked_l1_forward: pinned host block", herr);
    // per-scratch launch epoch (never 0, the value of freshly zeroed scratch)
    uint32_t epoch = 0;
    {
        static std::mutex mu;
        static std::map<void*, uint32_t> epochs;
        std::lock_guard<std::mutex> g(mu);
        uint32_t& e = epochs[scratch];
        e = e + 1 == 0 ? 1 : e + 1;
        epoch = e;
    }
    LSR_TRY(launch_masked_l1_forward(C, HW, pred, gt, mask, mask_is_float, loss, scratch, epoch, &hb->stall, stream),
            "masked l1");
    return LSR_OK;
}

int32_t lsr_masked_l1_backward(int32_t C, int64_t HW, const float* pred, const float* gt, const void* mask,
                               int32_t mask_is_float, const float* grad_loss, float* grad_pred, void* stream_ptr)
{
    if (C <= 0 || HW <= 0 || !pred || !gt || !mask || !grad_loss || !grad_pred)
        return fail(LSR_ERR_INVALID, "lsr_masked_l1_backward: invalid argument");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    LSR_TRY(launch_masked_l1_backward(C, HW, pred, gt, mask, mask_is_float, grad_loss, grad_pred, stream),
            "masked l1 backward");
    return LSR_OK;
}

int32_t lsr_adam_step(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq, double lr,
                      double beta1, double beta2, double eps, int64_t step, void* stream_ptr)
{
    if (n < 0 || (n > 0 && (!param || !grad || !exp_avg || !exp_avg_sq)) || step < 1)
        return fail(LSR_ERR_INVALID, "lsr_adam_step: invalid argument");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    const AdamScalars a = adam_scalars(lr, beta1, beta2, eps, step);
    LSR_TRY(launch_adam(n, param, grad, exp_avg, exp_avg_sq, a, stream), "adam");
    return LSR_OK;
}

int32_t lsr_adam_multi(int32_t count, const lsr_adam_tensor* tensors, float grad_scale, int64_t* step_dev,
                       const int32_t* skip, void* stream_ptr)
{
    if (count < 0 || (count > 0 && !tensors)) return fail(LSR_ERR_INVALID, "lsr_adam_multi: invalid argument");
    if (step_dev && count > kAdamMaxTensors)
        return fail(LSR_ERR_INVALID, "lsr_adam_multi: step_dev allows at most 16 tensors");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    for (int32_t k0 = 0; k0 < count; k0 += kAdamMaxTensors) {
        AdamTable tab{};
        for (int32_t k = k0; k < count && k < k0 + kAdamMaxTensors; k++) {
            const lsr_adam_tensor& t = tensors[k];
            if (t.n < 0 || (t.n > 0 && (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq)) ||
                (t.step < 1 && !step_dev) || (step_dev && (t.step < -((int64_t)1 << 40) || t.step > ((int64_t)1 << 40))))
                return fail(LSR_ERR_INVALID, "lsr_adam_multi: invalid tensor entry");
            if (t.n == 0) continue;
            tab.hyper[tab.count] = AdamHyper{t.lr, t.beta1, t.beta2, t.eps, step_dev ? t.step : 0};
            AdamSegment& g = tab.seg[tab.count++];
            g.param = t.param;
            g.grad = t.grad;
            g.m = t.exp_avg;
            g.v = t.exp_avg_sq;
            g.n = t.n;
            g.a = adam_scalars(t.lr, t.beta1, t.beta2, t.eps, t.step < 1 ? 1 : t.step);
        }
        tab.step_dev = step_dev;
        tab.skip = skip;
        LSR_TRY(launch_adam_multi(tab, grad_scale, stream), "adam");
    }
    return LSR_OK;
}

int32_t lsr_adam_fill_language(const lsr_adam_tensor* t, float grad_scale, int64_t* step_dev, const int32_t* skip,
                               void* fill_record, int32_t raw, void* stream_ptr)
{
    if (!t || !step_dev || !fill_record || t->n < 0 || t->n % 3 != 0 || t->n / 3 > INT32_MAX ||
        (t->n > 0 && (!t->param || !t->grad || !t->exp_avg || !t->exp_avg_sq)) ||
        t->step < -((int64_t)1 << 40) || t->step > ((int64_t)1 << 40))
        return fail(LSR_ERR_INVALID, "lsr_adam_fill_language: invalid argument");
    if (reinterpret_cast<uintptr_t>(fill_record) & 15)
        return fail(LSR_ERR_INVALID, "lsr_adam_fill_language: fill_record must be 16-byte aligned");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    const AdamHyper h{t->lr, t->beta1, t->beta2, t->eps, t->step};
    LSR_TRY(launch_adam_fill((int)(t->n / 3), t->grad, grad_scale, t->param, t->exp_avg, t->exp_avg_sq, h, step_dev,
                             skip, reinterpret_cast<float4*>(fill_record), raw, stream),
            "adam fill");
    return LSR_OK;
}

int32_t lsr_language_tail(const lsr_settings* s, const lsr_backward_args* a, void* stream_ptr)
{
    if (!s || !a) return fail(LSR_ERR_INVALID, "lsr_language_tail: null argument");
    const int P = a->P, W = s->image_width, H = s->image_height;
    if (P < 0 || W <= 0 || H <= 0) return fail(LSR_ERR_INVALID, "lsr_language_tail: invalid P or image size");
    if (!a->update || !a->update_step_dev || !a->dL_dlanguage_feature || !(a->raw & LSR_RAW_LANGUAGE) ||
        !a->language_feature || a->update->param != a->language_feature || a->update->n != 3 * (int64_t)P ||
        !a->update->exp_avg || !a->update->exp_avg_sq)
        return fail(LSR_ERR_INVALID, "lsr_language_tail: the arguments of a fused update (lsr_backward_args.update) "
                                     "are needed");
    if (P > 0 && (!a->geom_buffer || !a->radii)) return fail(LSR_ERR_INVALID, "lsr_language_tail: missing forward state");
    if (a->fill_record && (reinterpret_cast<uintptr_t>(a->fill_record) & 15))
        return fail(LSR_ERR_INVALID, "lsr_language_tail: fill_record must be 16-byte aligned");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = s->debug != 0;
    const Layout L = make_layout(P, W, H, a->num_rendered, 0);
    float* grad = P > 0 ? reinterpret_cast<float*>(static_cast<char*>(a->geom_buffer) + L.grad_records) : nullptr;
    const lsr_adam_tensor& u = *a->update;
    AdamHyper h{u.lr, u.beta1, u.beta2, u.eps, u.step};
    // the skip flag the all-reduce carried (the word after the language partials): any rank's overflow
    const int32_t* skip = P > 0 ? reinterpret_cast<const int32_t*>(grad + 3 * (size_t)P) : a->update_skip;
    LSR_TRY(launch_language_tail(P, a->radii, grad, const_cast<float*>(a->language_feature), u.exp_avg, u.exp_avg_sq,
                                 a->dL_dmeans2D, a->dL_dlanguage_feature, h, a->update_step_dev, skip,
                                 reinterpret_cast<float4*>(a->fill_record), 1, stream),
            "language tail");
    return LSR_OK;
}

int32_t lsr_densification_stats(int32_t P, const int32_t* radii, const float* dL_dmeans2D, float* max_radii2D,
                                float* xyz_gradient_accum, float* denom, void* stream_ptr)
{
    if (P < 0 || (P > 0 && (!radii || !dL_dmeans2D)))
        return fail(LSR_ERR_INVALID, "lsr_densification_stats: invalid argument");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    LSR_TRY(launch_densification_stats(P, radii, dL_dmeans2D, max_radii2D, xyz_gradient_accum, denom, stream),
            "densification stats");
    return LSR_OK;
}

int32_t lsr_dist_cuda2(int64_t N, const float* points, float* out_mean_dist, lsr_alloc_fn alloc, void* user,
                       void* stream_ptr)
{
    if (N < 0 || (N > 0 && (!points || !out_mean_dist || !alloc)) || N > 0x3FFFFFFF)
        return fail(LSR_ERR_INVALID, "lsr_dist_cuda2: invalid argument");
    if (N == 0) return LSR_OK;
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    void* scratch = alloc(user, LSR_BUF_BACKWARD, knn_scratch_bytes(N));
    if (!scratch) return fail(LSR_ERR_ALLOC, "lsr_dist_cuda2: scratch allocation failed");
    hipError_t herr = hipSuccess;
    HostBlock* hb = t_host.get(&herr);
    if (!hb) return fail(LSR_ERR_HIP, "lsr_dist_cuda2: pinned host block", herr);
    LSR_TRY(launch_knn_mean_dist3(N, points, out_mean_dist, scratch, &hb->stall, stream), "dist_cuda2");
    return LSR_OK;
}

int32_t lsr_decode_language_feature(int32_t L, int32_t H, int32_t W, const int64_t* seg_map, int32_t level,
                                    int32_t N, int32_t D, const float* feature_map, float* out_feature,
                                    uint8_t* out_mask, void* stream_ptr)
{
    if (L <= 0 || H <= 0 || W <= 0 || level < 0 || level >= L || N <= 0 || D <= 0 || !seg_map || !feature_map ||
        !out_feature || !out_mask)
        return fail(LSR_ERR_INVALID, "lsr_decode_language_feature: invalid argument");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_ptr);
    const bool debug = false;
    hipError_t herr = hipSuccess;
    HostBlock* hb = t_host.get(&herr);
    if (!hb) return fail(LSR_ERR_HIP, "lsr_decode_language_feature: pinned host block", herr);
    __atomic_store_n(&hb->bad_segment, 0u, __ATOMIC_RELEASE);
    LSR_TRY(launch_decode_language_feature(H, W, seg_map + (int64_t)level * H * W, N, D, feature_map, out_feature,
                                           out_mask, &hb->bad_segment, stream),
            "decode language feature");
    // once per view: wait, so that an id the reference's feature_map[seg] would reject is reported
    LSR_TRY(hipStreamSynchronize(stream), "decode language feature (sync)");
    if (__atomic_exchange_n(&hb->bad_segment, 0u, __ATOMIC_ACQ_REL))
        return fail(LSR_ERR_INVALID, "lsr_decode_language_feature: segment id outside [-N, N) of the feature map");
    return LSR_OK;
}

}  // extern "C"
