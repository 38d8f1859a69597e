// lsr_binning.hip -- tile binning and ordering.
//
// The reference (upstream) emits one 64-bit key (tile << 32 | depth bits) per tile instance and
// radix-sorts all R instances on 32+msb(T) bits.  This file reaches the SAME per-tile order
// ((depth, Gaussian id) ascending inside each tile) without sorting instances at all:
//
//   1. depth sort of the P Gaussians (32-bit keys, stable LSD radix with wave64 ballot ranking;
//      equal depths keep id order) -> sorted_ids;
//   2. super-tiles of 8 x 8 tiles (128 x 128 px): each visible Gaussian, in depth order, emits
//      one entry per super-tile its tile rectangle meets (about 1.5 per Gaussian vs ~8.5 tile
//      instances), and one stable radix pass on the super-tile id (8 bits at 1080p) gives every
//      super-tile its depth-ordered entry list;
//   3. inside a super-tile an entry's coverage is a 64-bit tile mask.  Segments of 2048 entries
//      are processed by one workgroup in batches of 64 per wave: a 64 x 64 bit transpose across
//      the wave turns the batch's masks into per-tile lane columns, so a tile's stable rank
//      among the batch is popcount(column & lanes-below) -- no keys, no atomics;
//   4. counts per (tile, segment) are scanned once in tile-major order: that gives every
//      segment's base inside every tile list, the tile ranges, and a point_list laid out
//      exactly like the sorted instance list (tile, depth, id).
//
// Every step is deterministic, so point_list is bit-identical to the oracle's (tile, depth, id)
// sort.  Scans are single-pass chained scans with decoupled look-back (one launch each).
#include <stdlib.h>

#include <atomic>

#include "lsr_internal.h"

namespace lsr {

__device__ __forceinline__ uint64_t lanemask_lt()
{
    const uint32_t lane = threadIdx.x & 63;
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Lanes of the wave whose digit (nbits wide) equals mine (restricted to `valid` lanes).
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid, int nbits)
{
    uint64_t m = __ballot(valid);
    for (int b = 0; b < nbits; b++) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        m &= bit ? bal : ~bal;
    }
    return m;
}

static hipError_t post(bool debug, hipStream_t s)
{
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && debug) e = hipStreamSynchronize(s);
    return e;
}

// ---------------------------------------------------------------- multi-block exclusive scan

constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int kScanChunk = kScanThreads * kScanItems;  // 4096 elements per block

// Block-wide exclusive scan of one value per thread; returns the block total in *total.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* wsum, uint32_t* total)
{
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; w++) {
        const uint32_t s = wsum[w];
        before += w < wave ? s : 0u;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return before + x - v;
}

// Single-pass chained scan with decoupled look-back.  Chunk ids come from an atomic ticket, so
// every predecessor of a running chunk has already been scheduled (no dispatch-order assumption,
// no deadlock).  Each chunk publishes {flag, value} in ONE 64-bit word (one sc1 store), so the
// hand-off needs no fences: flag 1 = chunk aggregate, flag 2 = inclusive prefix.  Wave 0 looks
// back over a window of 64 predecessors per hop.  The status words and the ticket must be zero
// at launch; launch_preprocess / k_emit clear them (no memset launches).
constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagInc = 2ull << 62;
// Stall bound (stall_spin_limit(), lsr_internal.h): a look-back that has polled that many times
// without its predecessors becoming ready stops waiting and computes its exclusive prefix itself,
// straight from the input (scans are out-of-place, so in[] is never overwritten): the result is the
// same, only slower.  It notes the event in the calling thread's pinned stall word
// (lsr_debug_scan_stalls).  Limit 0 takes that path in every chunk (tests).  With chunk ids from a
// ticket the predecessors are always resident, so only a GPU that stops scheduling them gets here.
static std::atomic<uint32_t> g_spin_limit{1u << 24};
uint32_t stall_spin_limit() { return g_spin_limit.load(std::memory_order_relaxed); }
uint32_t set_stall_spin_limit(uint32_t v) { return g_spin_limit.exchange(v); }

__host__ __device__ inline int scan_blocks(int n) { return (n + kScanChunk - 1) / kScanChunk; }

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// in != out: the stall fallback re-reads predecessors' inputs.
__global__ __launch_bounds__(kScanThreads) void k_scan(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       int n, uint64_t* __restrict__ status,
                                                       uint32_t* __restrict__ total, uint32_t* stall,
                                                       uint32_t spin_limit)
{
    __shared__ uint32_t wsum[kScanThreads / 64];
    __shared__ uint32_t s_chunk, s_prefix;
    const int nchunks = scan_blocks(n);
    uint32_t* ticket = reinterpret_cast<uint32_t*>(status + nchunks);
    if (threadIdx.x == 0) s_chunk = atomicAdd(ticket, 1u);
    __syncthreads();
    const int c = (int)s_chunk;
    const int i0 = c * kScanChunk + threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    if (i0 + kScanItems <= n) {
        const uint4* src = reinterpret_cast<const uint4*>(in + i0);
#pragma unroll
        for (int q = 0; q < kScanItems / 4; q++) {
            const uint4 w = src[q];
            v[4 * q] = w.x;
            v[4 * q + 1] = w.y;
            v[4 * q + 2] = w.z;
            v[4 * q + 3] = w.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; k++) v[k] = (i0 + k < n) ? in[i0 + k] : 0u;
    }
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++) sum += v[k];
    uint32_t agg;
    const uint32_t ex = block_exclusive_scan(sum, wsum, &agg);
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        uint32_t prefix = 0;
        if (c == 0) {
            if (lane == 0) __hip_atomic_store(&status[0], kFlagInc | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(&status[c], kFlagAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int top = c - 1;
            uint32_t spins = 0;
            for (;;) {
                const int idx = top - lane;
                const uint64_t w = idx >= 0
                    ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagInc;
                const uint32_t flag = (uint32_t)(w >> 62);
                const uint64_t inc = __ballot(flag == 2u);
                const int k = inc ? __ffsll((unsigned long long)inc) - 1 : 63;  // nearest inclusive
                const uint64_t upto = k == 63 ? ~0ull : ((2ull << k) - 1ull);
                if (spin_limit == 0u || (__ballot(flag == 0u) & upto)) {      // a predecessor is not ready
                    if (++spins > spin_limit) {  // stop waiting: the exclusive prefix from the input
                        uint32_t part = 0;
                        for (int i = lane; i < c * kScanChunk; i += 64) part += in[i];
                        prefix = wave_sum(part);
                        if (lane == 0) note_stall(stall);
                        break;
                    }
                    continue;
                }
                prefix += wave_sum(lane <= k ? (uint32_t)w : 0u);
                if (inc) break;
                top -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(&status[c], kFlagInc | (uint64_t)(prefix + agg), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            s_prefix = prefix;
            if (total && c == nchunks - 1) *total = prefix + agg;
        }
    }
    __syncthreads();
    uint32_t run = s_prefix + ex;
    if (i0 + kScanItems <= n) {
        uint4* dst = reinterpret_cast<uint4*>(out + i0);
#pragma unroll
        for (int q = 0; q < kScanItems / 4; q++) {
            uint4 w;
            w.x = run; run += v[4 * q];
            w.y = run; run += v[4 * q + 1];
            w.z = run; run += v[4 * q + 2];
            w.w = run; run += v[4 * q + 3];
            dst[q] = w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; k++) {
            if (i0 + k < n) out[i0 + k] = run;
            run += v[k];
        }
    }
}

// out[i] = sum(in[0..i)); if total != null it receives the grand total.  `in` must not alias `out`.
// region: scan_region_words(n) zeroed words (status per chunk + ticket).
static hipError_t scan_exclusive(const uint32_t* in, uint32_t* out, int n, uint32_t* region, uint32_t* total,
                                 uint32_t* stall, hipStream_t s, bool debug)
{
    if (n <= 0) return hipSuccess;
    if (in == out) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_scan, dim3(scan_blocks(n)), dim3(kScanThreads), 0, s, in, out, n,
                       reinterpret_cast<uint64_t*>(region), total, stall, stall_spin_limit());
    return post(debug, s);
}

// One workgroup: reduces the preprocess block partials into the counters (R, E, visible depth-key
// min / max, the prefiltered error flag: bit 31 of the max key), clears the other counter words
// (scan fault, the tile schedule's class counts) -- so the counters need no memset before the
// forward -- then publishes counters[0..7] to pinned host memory (system scope) followed by the
// sequence number the host spins on (one {value, seq} 64-bit slot per counter).
#ifndef LSR_PUBLISH_THREADS  // the counter reduction's workgroup size (measurement knob): 256 threads find
#define LSR_PUBLISH_THREADS 256  // a CU beside the pipelined step's render workgroups sooner than 1024
#endif                           // (C3 step 0.3999-0.4007 vs 0.4008-0.4015 ms, profiles/r05_publish_threads.txt)
constexpr int kPublishThreads = LSR_PUBLISH_THREADS;

__global__ __launch_bounds__(kPublishThreads) void k_publish_counters(int nb, const uint4* __restrict__ partial,
                                                                      uint32_t* __restrict__ counters,
                                                                      uint64_t* host_slots, uint32_t seq,
                                                                      uint32_t fwd_flags, uint32_t r_cap, uint32_t e_cap,
                                                                      int32_t* overflow, int depth_passes)
{
    constexpr int kWaves = kPublishThreads / 64;
    __shared__ uint32_t red[4][kWaves];
    uint32_t t = 0, e = 0, kmin = 0xFFFFFFFFu, kmax = 0;
    // kPer loads in flight per thread before any is consumed (8k partials at 1M Gaussians: one round)
    constexpr int kPer = 8 * 1024 / kPublishThreads;
    for (int b0 = threadIdx.x; b0 < nb; b0 += kPublishThreads * kPer) {
        uint4 v[kPer];
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const int b = b0 + j * kPublishThreads;
            v[j] = b < nb ? partial[b] : make_uint4(0u, 0u, 0xFFFFFFFFu, 0u);
        }
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            t += v[j].x;
            e += v[j].y;
            kmin = min(kmin, v[j].z);
            kmax = max(kmax, v[j].w);  // the error bit, if set anywhere, survives the max
        }
    }
    for (int i = threadIdx.x; i < kCntWords; i += kPublishThreads)
        if (i != kCntRendered && i != kCntSuper && i != kCntKeyMin && i != kCntKeyMax && i != kCntError)
            counters[i] = i == kCntFwdFlags ? fwd_flags : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        t += __shfl_xor(t, o, 64);
        e += __shfl_xor(e, o, 64);
        kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o, 64));
        kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o, 64));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = t;
        red[1][w] = e;
        red[2][w] = kmin;
        red[3][w] = kmax;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int k = 1; k < kWaves; k++) {
        red[0][0] += red[0][k];
        red[1][0] += red[1][k];
        red[2][0] = min(red[2][0], red[2][k]);
        red[3][0] = max(red[3][0], red[3][k]);
    }
    counters[kCntRendered] = red[0][0];
    counters[kCntSuper] = red[1][0];
    counters[kCntKeyMin] = red[2][0];
    counters[kCntKeyMax] = red[3][0] & 0x7FFFFFFFu;
    counters[kCntError] = red[3][0] >> 31;
    if (r_cap) {  // capacity mode: nothing goes to the host; the binning reads the counts here
        // LSD depth order (depth_passes > 0): the passes the visible key range needs (as the host
        // computes them in the eager forward) must not exceed the ones enqueued
        const uint32_t span = (red[3][0] & 0x7FFFFFFFu) - red[2][0];
        const int bits = span ? 32 - __clz(span) : 0;
        const int need = red[0][0] == 0 ? 0 : (bits <= 8 ? 1 : (bits + 7) / 8);
        const uint32_t ovf = (red[0][0] > r_cap || red[1][0] > e_cap || (depth_passes > 0 && need > depth_passes))
            ? 1u : 0u;
        counters[kCntOverflow] = ovf;
        // the caller's flag holds the bits of 1.0f when set: non-zero as an int (the Adam skip test)
        // and 1.0 as a float, so ranks can all-reduce it with their gradients (include/lsr.h)
        if (overflow) *overflow = ovf ? (int32_t)0x3F800000 : 0;
        return;
    }
    // each value travels with the sequence number in one 64-bit store (single-copy atomic): the
    // host waits for all 8 slots to carry `seq`, so no release fence (L2 write-back) is needed
    for (int i = 0; i < 8; i++)
        __hip_atomic_store(&host_slots[i], (uint64_t)counters[i] | ((uint64_t)seq << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_publish_counters(int nb, const uint4* partial, uint32_t* counters, uint64_t* host_slots,
                                   uint32_t seq, uint32_t fwd_flags, uint32_t r_cap, uint32_t e_cap,
                                   int32_t* overflow, int depth_passes, hipStream_t s)
{
    hipLaunchKernelGGL(k_publish_counters, dim3(1), dim3(kPublishThreads), 0, s, nb, partial, counters, host_slots,
                       seq, fwd_flags, r_cap, e_cap, overflow, depth_passes);
    return hipGetLastError();
}

hipError_t scan_exclusive_u32(const uint32_t* in, uint32_t* out, int n, uint32_t* region, uint32_t* stall,
                              hipStream_t s)
{
    return scan_exclusive(in, out, n, region, nullptr, stall, s, false);
}

// ---------------------------------------------------------------- stable LSD radix sort

// super-tile rectangle [sx0, sx1) x [sy0, sy1) of a packed tile rectangle
__device__ __forceinline__ void super_rect(uint2 rc, int& sx0, int& sy0, int& sx1, int& sy1)
{
    const int x0 = rc.x & 0xFFFF, y0 = rc.x >> 16, x1 = rc.y & 0xFFFF, y1 = rc.y >> 16;
    sx0 = x0 / kSuper;
    sy0 = y0 / kSuper;
    sx1 = (x1 + kSuper - 1) / kSuper;
    sy1 = (y1 + kSuper - 1) / kSuper;
}

// super-tile entries of a tile rectangle (0 for the empty rectangle of a culled Gaussian)
__device__ __forceinline__ uint32_t super_count(uint2 rc)
{
    if (rc.x == rc.y) return 0u;
    int sx0, sy0, sx1, sy1;
    super_rect(rc, sx0, sy0, sx1, sy1);
    return (uint32_t)((sx1 - sx0) * (sy1 - sy0));
}

// Optional work of the depth sort's LAST scatter pass, per output rank r (= depth rank): the
// Gaussian's tile rectangle copied into depth order (the binning's one random gather) and its
// super-tile entry count (-> exclusive scan = entry offsets); the sorted keys are not stored.
// rect == null: a plain pass.
struct ScatterTail {
    const uint2* rect;
    uint2* rect_ranked;
    uint32_t* ns;
};


// Both radix kernels use a BLOCKED arrangement: wave w of a block owns the contiguous keys
// [w * 64 * kItems, (w + 1) * 64 * kItems) of the block's tile and walks them in rounds of 64
// consecutive keys, counting digits in its own LDS row.  Rounds of one wave are ordered by the
// wave's in-order LDS pipeline, so no block barrier is needed until all rounds are done; the
// stable order (wave, round, lane) is the input order.

// Per-block digit histogram; hist layout [digit][block] so one scan yields the scatter bases.
// kItems keys per thread: 16 for large sorts, 4 for P-sized ones (so that >= ~1000 blocks run).
// First pass of the depth sort only (kxf != null): key' = key - kxf[0] (the smallest visible depth
// key), and culled keys (0xFFFFFFFF) -> kxf[1] - kxf[0], the largest visible one (their position
// among equal keys is irrelevant: they emit nothing).  Order among visible keys is unchanged.
__device__ __forceinline__ uint32_t key_xf(uint32_t k, const uint32_t* kxf)
{
    return k == 0xFFFFFFFFu ? kxf[1] - kxf[0] : k - kxf[0];
}

// XCD-aware tile order: workgroups are dispatched round-robin over the 8 XCDs (workgroup i on XCD
// i % 8), so consecutive tiles would land on 8 different L2s and every output line (histogram
// column, digit run) would be assembled from partial writes of several XCDs.  Tile of workgroup i:
// XCD x = i % 8 takes the contiguous tile range [x q + min(x, r), ...) with q = nblk / 8, r = nblk % 8.
__device__ __forceinline__ int xcd_tile(int nblk, int remap)
{
    const int i = blockIdx.x;
    if (!remap) return i;
    const int x = i & 7, q = nblk >> 3, r = nblk & 7;
    return x * q + min(x, r) + (i >> 3);
}

// MSD depth sort (launch_depth_order, P <= kMsd512MaxKeys): one radix pass splits the keys into 256 (512)
// buckets by a monotone function of the key, read on the device from kxf (min / max visible key),
// so no host value is needed; each bucket then sorts its keys on their own range.  The key is the
// depth's float bits, and two bucket maps are used:
//   - a narrow depth range (max <= kMsdLinearRatio min): 256 buckets of EQUAL DEPTH WIDTH,
//     bucket = min(255, (depth - dmin) 256 / w) (a float subtraction, a multiplication by a
//     positive constant and a truncation are each monotone);
//   - a wide one: the top 8 bits of key - min, i.e. equal KEY intervals, which are logarithmic in
//     depth (every float octave gets the same share).
// Equal key intervals alone (round 2) double their depth width at every float exponent step: at C3
// (depths 3..5) the keys of [4, 5) fell into half as many buckets as those of [3, 4), 64 buckets
// held ~8k keys, 120 ~3k and 64 none, and the 8k buckets set the bucket kernel's span (equal depth
// widths: 3.7k..4.1k per bucket).  Over a wide range depth counts fall off with distance, where
// logarithmic buckets stay even.  Culled keys (key_xf: max - min) land in the last bucket.
constexpr float kMsdLinearRatio = 2.5f;
// Above kMsdMaxKeys (below) the pass makes 512 buckets (9-bit digits: the same two
// maps with twice the resolution), so the average bucket stays within one workgroup's LDS sort up
// to kMsd512MaxKeys; `bits` = 8 or 9 is the digit width.

struct MsdMap {
    uint32_t kmin;
    float dmin, scale;
    int shift;
    int top;  // 2^bits - 1
    bool linear;
};

__device__ __forceinline__ MsdMap msd_map(const uint32_t* kxf, int dbits = 8)
{
    MsdMap m;
    m.kmin = kxf[0];
    m.dmin = __uint_as_float(kxf[0]);
    const float dmax = __uint_as_float(kxf[1]);
    const float w = dmax - m.dmin;
    m.linear = m.dmin > 0.0f && dmax <= kMsdLinearRatio * m.dmin;  // false when none is visible
    m.scale = w > 1e-30f ? (float)(1 << dbits) / w : 0.0f;
    const uint32_t span = kxf[1] - kxf[0];
    const int bits = span ? 32 - __clz(span) : 0;
    m.shift = bits > dbits ? bits - dbits : 0;
    m.top = (1 << dbits) - 1;
    return m;
}

// bucket of a transformed key kx = key_xf(key)
__device__ __forceinline__ uint32_t msd_bucket(uint32_t kx, const MsdMap& m)
{
    if (!m.linear) return (kx >> m.shift) & (uint32_t)m.top;
    const float v = (__uint_as_float(kx + m.kmin) - m.dmin) * m.scale;
    return (uint32_t)min(m.top, max(0, (int)v));
}

// Word ranges a kernel clears with grid-stride stores besides its own work (n = 0: none).  The
// binning's first launch clears the tables its later kernels accumulate into or leave partly
// unwritten (tile / super-tile ranges, the segment count table, the scans' status words).
struct ZeroList {
    uint32_t* p[4];
    int n[4];
};

__device__ __forceinline__ void zero_words_strided(const ZeroList& z)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    const int stride = gridDim.x * blockDim.x;
#pragma unroll
    for (int k = 0; k < 4; k++)
        for (int w = r; w < z.n[k]; w += stride) z.p[k][w] = 0u;
}

// LSD depth passes in capacity mode run the most passes any view can need (the host cannot read the
// key range there): a pass whose shift is at or above the bits of this view's visible key range
// (krange = {min, max} visible depth key, published by the forward's counter reduction; key_xf maps
// every key into [0, max - min]) sees digit 0 for every key, so its stable scatter is the identity
// and its histogram is not needed.
__device__ __forceinline__ bool uniform_pass(const uint32_t* krange, int shift)
{
    return krange && shift < 32 && ((krange[1] - krange[0]) >> shift) == 0u;
}

// srect (MSD pass with placed emission): the keys' tile rectangles by index; the block's super-tile
// entry counts then also go to rows 256 + s (s < supers) of hist, so the scan that yields the
// bucket starts also yields every super-tile's base in the super-tile-major entry list (+ n).
// msd: 0, or the MSD pass's digit bits (8, or 9 with kDig = 512 digit rows)
template <int kItems, int kDig = 256>
__global__ __launch_bounds__(kRadixThreads) void k_radix_hist(const uint32_t* __restrict__ keys, int n, int shift,
                                                              int nbits, uint32_t* __restrict__ hist, int nblk,
                                                              const uint32_t* __restrict__ kxf, int remap, int msd,
                                                              ZeroList zero, DevCount dc,
                                                              const uint2* __restrict__ srect = nullptr,
                                                              int supers = 0, int sgx = 0,
                                                              const uint32_t* __restrict__ krange = nullptr)
{
    constexpr int kWaves = kRadixThreads / 64;
    static_assert(kDig % kRadixThreads == 0, "digit rows per thread");
    __shared__ uint32_t wcnt[kWaves][kDig];
    __shared__ uint32_t scnt[256];
    zero_words_strided(zero);
    if (dc.abort && *dc.abort) return;
    if (uniform_pass(krange, shift)) return;  // the scatter copies; its histogram is not read
    if (dc.n) n = min(n, (int)*dc.n);
    MsdMap mm{};
    if (msd) {
        mm = msd_map(kxf, msd);
        shift = 0;
        nbits = msd;
    }
    const int blk = xcd_tile(nblk, remap);
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const uint32_t mask = (1u << nbits) - 1u;
#pragma unroll
    for (int w = 0; w < kWaves; w++)
#pragma unroll
        for (int j = 0; j < kDig; j += kRadixThreads) wcnt[w][j + t] = 0;
    scnt[t] = 0;
    __syncthreads();
    const int base = blk * kRadixThreads * kItems + wave * 64 * kItems;
    uint32_t d[kItems];
    bool valid[kItems];
    uint2 rc[kItems];
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        const int idx = base + it * 64 + lane;
        valid[it] = idx < n;
        uint32_t k = valid[it] ? keys[idx] : 0u;
        rc[it] = srect && valid[it] ? srect[idx] : make_uint2(0u, 0u);
        if (kxf) k = key_xf(k, kxf);
        d[it] = valid[it] ? (msd ? msd_bucket(k, mm) : (k >> shift) & mask) : 0u;
    }
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        const uint64_t peers = match_digit(d[it], valid[it], nbits);
        if (valid[it] && (peers & lanemask_lt()) == 0) wcnt[wave][d[it]] += (uint32_t)__popcll(peers);
    }
    if (srect) {
#pragma unroll
        for (int it = 0; it < kItems; it++) {
            if (rc[it].x == rc[it].y) continue;  // culled or past n: no entries
            int sx0, sy0, sx1, sy1;
            super_rect(rc[it], sx0, sy0, sx1, sy1);
            for (int y = sy0; y < sy1; y++)
                for (int x = sx0; x < sx1; x++) atomicAdd(&scnt[y * sgx + x], 1u);
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kDig; j += kRadixThreads) {
        const int dg = j + t;
        if (dg <= (int)mask) {
            uint32_t c = 0;
#pragma unroll
            for (int w = 0; w < kWaves; w++) c += wcnt[w][dg];
            hist[(size_t)dg * nblk + blk] = c;
        }
    }
    if (srect && t < supers) hist[(size_t)(kDig + t) * nblk + blk] = scnt[t];
}

// Stable scatter of one block's tile.  Ranks: per wave, round by round (ballot match + the wave's
// running digit counts); then per digit the block-local start (scan over digits) and each wave's
// exclusive offset (sum over lower waves).  The tile is reordered by digit in LDS and written
// from LDS in digit-contiguous runs, so global stores coalesce (a direct scatter would send the
// 64 lanes of a store to up to 64 different buckets).
// kCarry (MSD depth pass, vals_in == null): the Gaussian's rectangle tail.rect[idx] rides along
// with its key into tail.rect_ranked, so the bucket sort permutes rectangles inside its bucket
// instead of gathering them across all of rect (tail.ns is not used).
// kDig = 512: the 9-bit MSD pass (msd = 9), thread t ranking digits 2t and 2t + 1.
template <int kItems, bool kCarry = false, int kDig = 256>
__global__ __launch_bounds__(kRadixThreads) void k_radix_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, int n, int shift, int nbits,
    const uint32_t* __restrict__ hist, int nblk, uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
    const uint32_t* __restrict__ kxf, ScatterTail tail, int remap, int msd, DevCount dc, int hstride = 0,
    int hrows = 256, ZeroList zero = ZeroList{}, const uint32_t* __restrict__ krange = nullptr)
{
    zero_words_strided(zero);
    if (dc.abort && *dc.abort) return;
    if (hstride == 0) hstride = nblk;  // histogram rows of nblk blocks (the hist kernel's layout)
    if (dc.n) n = min(n, (int)*dc.n);
    if (!msd && uniform_pass(krange, shift)) {  // every key's digit is 0: the stable pass is the identity
        const int blk = xcd_tile(nblk, remap);
        for (int i = blk * kRadixThreads * kItems + threadIdx.x; i < min(n, (blk + 1) * kRadixThreads * kItems);
             i += kRadixThreads) {
            const uint32_t k = kxf ? key_xf(keys_in[i], kxf) : keys_in[i];
            const uint32_t v = vals_in ? vals_in[i] : (uint32_t)i;
            if (kCarry || !tail.rect) {
                keys_out[i] = k;
                vals_out[i] = v;
                if (kCarry) tail.rect_ranked[i] = tail.rect[i];
            } else {  // the last depth pass's tail, as below
                const uint2 rc = tail.rect[v];
                vals_out[i] = v;
                tail.rect_ranked[i] = rc;
                tail.ns[i] = super_count(rc);
            }
        }
        return;
    }
    MsdMap mm{};
    if (msd) {
        mm = msd_map(kxf, msd);
        shift = 0;
        nbits = msd;
    }
    auto digit_of = [&](uint32_t k) { return msd ? msd_bucket(k, mm) : (k >> shift) & ((1u << nbits) - 1u); };
    const int blk = xcd_tile(nblk, remap);
    constexpr int kTile = kRadixThreads * kItems;
    constexpr int kWaves = kRadixThreads / 64;
    constexpr int kPerT = kDig / kRadixThreads;  // digits per thread in the digit loops
    static_assert(kDig % kRadixThreads == 0, "digit rows per thread");
    __shared__ uint32_t sk[kTile];
    __shared__ uint32_t sv[kTile];
    __shared__ uint32_t wcnt[kWaves][kDig];  // running counts, then each wave's offset within the digit
    __shared__ uint32_t gbase[kDig];         // global output position of this block's first key per digit
    __shared__ uint32_t dstart[kDig];        // block-local start of each digit in the reordered tile
    __shared__ uint32_t wsum[kWaves];
    __shared__ uint2 sr[kCarry ? kTile : 1];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const uint32_t mask = (1u << nbits) - 1u;
#pragma unroll
    for (int j = 0; j < kPerT; j++) {
        const int dg = kPerT * t + j;
#pragma unroll
        for (int w = 0; w < kWaves; w++) wcnt[w][dg] = 0;
        gbase[dg] = dg <= (int)mask && dg < hrows ? hist[(size_t)dg * hstride + blk] : 0u;
    }
    const int tile0 = blk * kTile;
    const int base = tile0 + wave * 64 * kItems;
    uint32_t key[kItems], val[kItems], rank[kItems];
    uint2 rcv[kCarry ? kItems : 1];
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        const int idx = base + it * 64 + lane;
        const bool valid = idx < n;
        key[it] = valid ? keys_in[idx] : 0u;
        if (kxf) key[it] = key_xf(key[it], kxf);
        val[it] = valid ? (vals_in ? vals_in[idx] : (uint32_t)idx) : 0u;
        if (kCarry) rcv[kCarry ? it : 0] = valid ? tail.rect[idx] : make_uint2(0u, 0u);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        const bool valid = base + it * 64 + lane < n;
        const uint32_t d = digit_of(key[it]);
        const uint64_t peers = match_digit(d, valid, nbits);
        const uint32_t r = (uint32_t)__popcll(peers & lanemask_lt());
        const uint32_t c = wcnt[wave][d];
        rank[it] = c + r;
        if (valid && r == 0) wcnt[wave][d] = c + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // per digit: waves' exclusive offsets and the block-local digit start (thread t: digits
    // kPerT t .. kPerT t + kPerT - 1, consecutive, so one scan of their sums orders them all)
    {
        uint32_t dt[kPerT], tot = 0;
#pragma unroll
        for (int j = 0; j < kPerT; j++) {
            const int dg = kPerT * t + j;
            uint32_t run = 0;
#pragma unroll
            for (int w = 0; w < kWaves; w++) {
                const uint32_t c = wcnt[w][dg];
                wcnt[w][dg] = run;
                run += c;
            }
            dt[j] = run;
            tot += run;
        }
        uint32_t x = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        uint32_t before = 0;
        for (int w = 0; w < wave; w++) before += wsum[w];
        uint32_t ex = before + x - tot;
#pragma unroll
        for (int j = 0; j < kPerT; j++) {
            dstart[kPerT * t + j] = ex;
            ex += dt[j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        if (base + it * 64 + lane < n) {
            const uint32_t d = digit_of(key[it]);
            const uint32_t pos = dstart[d] + wcnt[wave][d] + rank[it];
            sk[pos] = key[it];
            sv[pos] = val[it];
            if (kCarry) sr[pos] = rcv[kCarry ? it : 0];
        }
    }
    __syncthreads();
    const int cnt = min(kTile, n - tile0);
    if (kCarry || !tail.rect) {
        for (int i = t; i < cnt; i += kRadixThreads) {
            const uint32_t k = sk[i];
            const uint32_t d = digit_of(k);
            const uint32_t o = gbase[d] + (uint32_t)i - dstart[d];
            keys_out[o] = k;
            vals_out[o] = sv[i];
            if (kCarry) tail.rect_ranked[o] = sr[i];
        }
        return;
    }
    // last depth pass: all of this thread's rectangle gathers in flight at once
    uint32_t outp[kItems], vid[kItems];
    uint2 rc[kItems];
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        const int i = t + it * kRadixThreads;
        outp[it] = 0xFFFFFFFFu;
        if (i < cnt) {
            const uint32_t d = digit_of(sk[i]);
            outp[it] = gbase[d] + (uint32_t)i - dstart[d];
            vid[it] = sv[i];
        }
    }
#pragma unroll
    for (int it = 0; it < kItems; it++)
        if (outp[it] != 0xFFFFFFFFu) rc[it] = tail.rect[vid[it]];
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        if (outp[it] == 0xFFFFFFFFu) continue;
        const uint32_t o = outp[it];
        vals_out[o] = vid[it];
        tail.rect_ranked[o] = rc[it];
        tail.ns[o] = super_count(rc[it]);
    }
}

// Sorts (keys, vals) by key bits [0, total_bits) in passes of <= 8 bits.  The input is read
// from (k0, v0) (v0 == null: values are the input indices) and the result lands in
// (kA, vA) after an even number of passes, or in (kB, vB) after an odd number; returns which.
// Radix tile size: 4 keys per thread (>= ~1000 workgroups) up to 16M keys, else 16.  The 4-key
// tiles (14-22 KB of LDS, 40-50 VGPRs) fit beside the render kernels of the pipelined step where the
// 16-key ones (39-72 KB, 100-132 VGPRs) wait for them: at C5 (3M depth keys) the pipelined graph
// step 0.985 -> 0.948 ms with the same eager depth order (profiles/r05_c5_radix_tiles.txt).
// LSR_RADIX_SMALL_MAX=n moves the threshold (measurement aid).
static bool radix_small(int64_t n)
{
    static const int64_t lim = [] {
        const char* e = getenv("LSR_RADIX_SMALL_MAX");
        return e ? (int64_t)atoll(e) : (int64_t)(1 << 24);
    }();
    return n <= lim;
}

static hipError_t radix_sort(const uint32_t* k0, const uint32_t* v0, int n, int total_bits, uint32_t* kA,
                             uint32_t* vA, uint32_t* kB, uint32_t* vB, uint32_t* hist, uint32_t* hist_scan,
                             uint32_t* scan_regions, size_t region_words, uint32_t* stall, hipStream_t s, bool debug,
                             int* passes_out,
                             const uint32_t* kxf = nullptr, ScatterTail last = ScatterTail{nullptr, nullptr, nullptr},
                             ZeroList zero = ZeroList{}, DevCount dc = DevCount{nullptr, nullptr},
                             const uint32_t* krange = nullptr)
{
    const bool small = radix_small(n);
    const int tile = kRadixThreads * (small ? 4 : 16);
    const int nblk = (n + tile - 1) / tile;
    const int passes = (total_bits + 7) / 8;
    *passes_out = passes;
    static const int remap = [] {  // LSR_XCD_REMAP=0: tiles in dispatch order (measurement knob)
        const char* v = getenv("LSR_XCD_REMAP");
        return v && v[0] == '0' ? 0 : 1;
    }();
    const uint32_t* kin = k0;
    const uint32_t* vin = v0;
    hipError_t e;
    for (int pass = 0; pass < passes; pass++) {
        const int shift = 8 * pass;
        const int nbits = (total_bits - shift) < 8 ? (total_bits - shift) : 8;
        uint32_t* kout = (pass & 1) ? kA : kB;
        uint32_t* vout = (pass & 1) ? vA : vB;
        const ZeroList z = pass == 0 ? zero : ZeroList{};
        if (small)
            hipLaunchKernelGGL(k_radix_hist<4>, dim3(nblk), dim3(kRadixThreads), 0, s, kin, n, shift, nbits, hist, nblk,
                               pass == 0 ? kxf : nullptr, remap, 0, z, dc, (const uint2*)nullptr, 0, 0, krange);
        else
            hipLaunchKernelGGL(k_radix_hist<16>, dim3(nblk), dim3(kRadixThreads), 0, s, kin, n, shift, nbits, hist,
                               nblk, pass == 0 ? kxf : nullptr, remap, 0, z, dc, (const uint2*)nullptr, 0, 0, krange);
        if ((e = post(debug, s)) != hipSuccess) return e;
        if ((e = scan_exclusive(hist, hist_scan, (1 << nbits) * nblk, scan_regions + pass * region_words, nullptr,
                                stall, s, debug)) != hipSuccess)
            return e;
        const ScatterTail tail = pass == passes - 1 ? last : ScatterTail{nullptr, nullptr, nullptr};
        if (small)
            hipLaunchKernelGGL(k_radix_scatter<4>, dim3(nblk), dim3(kRadixThreads), 0, s, kin, vin, n, shift, nbits,
                               hist_scan, nblk, kout, vout, pass == 0 ? kxf : nullptr, tail, remap, 0, dc, 0, 256,
                               ZeroList{}, krange);
        else
            hipLaunchKernelGGL(k_radix_scatter<16>, dim3(nblk), dim3(kRadixThreads), 0, s, kin, vin, n, shift, nbits,
                               hist_scan, nblk, kout, vout, pass == 0 ? kxf : nullptr, tail, remap, 0, dc, 0, 256,
                               ZeroList{}, krange);
        if ((e = post(debug, s)) != hipSuccess) return e;
        kin = kout;
        vin = vout;
    }
    return hipSuccess;
}

// sized for the smallest tile (4 keys per thread) so either variant fits
size_t radix_hist_words(int64_t n) { return 256 * (size_t)((n + 4 * kRadixThreads - 1) / (4 * kRadixThreads)); }
// one u64 status word per chunk + the u64 ticket slot, in u32 words
size_t scan_region_words(int64_t n) { return 2 * (size_t)((n + kScanChunk - 1) / kScanChunk) + 2; }

// ---------------------------------------------------------------- super-tiles

// An entry key: super-tile id in the low 16 bits (the only bits sorted on), the Gaussian's tile
// rectangle clipped to the super-tile in the high 16 (lx0, lx1, ly0, ly1: 4 bits each).
__device__ __forceinline__ uint32_t entry_key(uint2 rc, int sx, int sy, int sgx)
{
    const int ox = sx * kSuper, oy = sy * kSuper;
    const int lx0 = max((int)(rc.x & 0xFFFF) - ox, 0), ly0 = max((int)(rc.x >> 16) - oy, 0);
    const int lx1 = min((int)(rc.y & 0xFFFF) - ox, kSuper), ly1 = min((int)(rc.y >> 16) - oy, kSuper);
    return (uint32_t)(sy * sgx + sx) | ((uint32_t)lx0 << 16) | ((uint32_t)lx1 << 20) | ((uint32_t)ly0 << 24) |
           ((uint32_t)ly1 << 28);
}

// 64-bit mask (bit = ly * 8 + lx) of the entry's tiles inside its super-tile
__device__ __forceinline__ uint64_t entry_mask(uint32_t key)
{
    const int lx0 = (key >> 16) & 15, lx1 = (key >> 20) & 15, ly0 = (key >> 24) & 15, ly1 = key >> 28;
    if (lx0 >= lx1 || ly0 >= ly1) return 0ull;
    const uint64_t row = (uint64_t)(((1u << (lx1 - lx0)) - 1u) << lx0);
    uint64_t m = 0ull;
    for (int ly = ly0; ly < ly1; ly++) m |= row << (8 * ly);
    return m;
}

// 64 x 64 bit-matrix transpose across the wave: bit j of lane i -> bit i of lane j
__device__ __forceinline__ uint64_t transpose64(uint64_t x)
{
    const int lane = threadIdx.x & 63;
    const uint64_t M[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                           0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
    for (int k = 0; k < 6; k++) {
        const int sft = 32 >> k;
        const uint64_t y = __shfl_xor(x, sft, 64);
        x = (lane & sft) ? (((y & ~M[k]) >> sft) | (x & ~M[k])) : ((x & M[k]) | ((y & M[k]) << sft));
    }
    return x;
}

// ---------------------------------------------------------------- MSD depth sort: bucket pass
//
// Depth order for P <= kMsd512MaxKeys: ONE stable radix pass on the top <= 8 bits of the key range
// (9 bits, 512 buckets, above kMsdMaxKeys; k_radix_hist / scan / k_radix_scatter with msd = the digit
// bits) puts every key in its bucket in id order;
// then one workgroup per bucket sorts the bucket on the remaining low bits in LDS (stable LSD
// passes of 8 bits, wave64 ballot ranking) and writes the depth-order outputs (sorted ids, the
// rectangle in depth order, super-tile entry counts).  Same (key, id) order as the LSD sort: four
// kernels instead of up to twelve.  A bucket larger than LDS (kBucketCap keys: a depth range
// dense far beyond the average) is sorted by its workgroup in global memory, 1024 keys at a time.
constexpr int kBucketThreads = 1024;
constexpr int kBucketWaves = kBucketThreads / 64;
#ifndef LSR_BUCKET_CAP  // keys a bucket sorts in LDS (a multiple of 1024 up to 8192; measurement knob):
#define LSR_BUCKET_CAP 8192  // the LDS a bucket workgroup takes, 8 B per key + 8 KB, sets how many
#endif                       // render workgroups can share its CU while it runs
constexpr int kBucketCap = LSR_BUCKET_CAP;
static_assert(kBucketCap % 1024 == 0 && kBucketCap <= 8192, "bucket capacity");
constexpr int kBucketRounds = kBucketCap / kBucketThreads;  // rounds of 64 keys per wave
constexpr int64_t kMsdMaxKeys = 2000000;                    // above: 512 buckets (msd_digits)

// A bucket in LDS is kBucketCap packed words {key bits not yet ranked, local index (13 bits)}:
// pass 0 ranks on the low 8 key bits held in registers and packs the rest (<= 16 bits) above the
// index, so the two ping-pong buffers take 64 KB and two workgroups share a CU.
constexpr int kIdxBits = 13;  // local index within a bucket (kBucketCap <= 1 << kIdxBits)
constexpr uint32_t kIdxMask = (1u << kIdxBits) - 1u;
static_assert((1 << kIdxBits) >= kBucketCap, "local index width");
struct BucketLds {
    uint32_t w[2][kBucketCap];
    uint16_t wcnt[kBucketWaves][256];  // per wave: running digit counts, then the wave's offset in the digit
    uint32_t dstart[256];              // digit starts (LDS passes) / running digit bases (global passes)
    uint32_t ctot[256];                // global passes: the chunk's digit totals
    uint32_t wsum[kBucketWaves];
    uint32_t scnt[256];                // placed emission: the bucket's entries per super-tile
    uint32_t run[256];                 // placed emission: per super-tile, the next entry's position
};
constexpr size_t kBucketLdsBytes = sizeof(BucketLds);

// exclusive scan of v over the first 256 threads (4 waves); every thread of the block must call it
__device__ __forceinline__ uint32_t scan256(uint32_t v, uint32_t* wsum)
{
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (t < 256 && lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t before = 0;
    for (int i = 0; i < w && i < 4; i++) before += wsum[i];
    __syncthreads();
    return before + x - v;
}

// Ranks of the digits dig[] (R <= kRounds per thread, wave w holding positions [w R 64,
// (w + 1) R 64) round by round): rank[r] within the wave's digit, and in LDS the digit starts
// (L.dstart) and each wave's offset in its digit (L.wcnt); position = dstart + wcnt + rank.
template <int kRounds>
__device__ __forceinline__ void rank_digits(BucketLds& L, const uint32_t (&dig)[kRounds], int nb, int nbits, int R,
                            uint32_t (&rank)[kRounds])
{
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    for (int i = t; i < kBucketWaves * 256; i += kBucketThreads) (&L.wcnt[0][0])[i] = 0;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRounds; r++) {
        if (r >= R) break;  // workgroup-uniform: the rounds in use
        const bool valid = (w * R + r) * 64 + lane < nb;
        const uint64_t peers = match_digit(dig[r], valid, nbits);
        const uint32_t rr = (uint32_t)__popcll(peers & lanemask_lt());
        const uint32_t c = L.wcnt[w][dig[r]];
        rank[r] = c + rr;
        if (valid && rr == 0) L.wcnt[w][dig[r]] = (uint16_t)(c + (uint32_t)__popcll(peers));
    }
    __syncthreads();
    uint32_t tot = 0;
    if (t < 256) {
        for (int i = 0; i < kBucketWaves; i++) {
            const uint32_t c = L.wcnt[i][t];
            L.wcnt[i][t] = (uint16_t)tot;
            tot += c;
        }
    }
    const uint32_t ex = scan256(tot, L.wsum);
    if (t < 256) L.dstart[t] = ex;
    __syncthreads();
}

// One stable pass of the LDS sort: the values val[] (R <= kBucketRounds per thread, wave w holding
// positions [w R 64, (w + 1) R 64) round by round; R = the rounds a bucket of nb keys needs, so a
// bucket half the capacity spreads over every wave in half the rounds) are placed by digit dig[] into out.  Ranks: per
// wave, round by round (ballot match + the wave's running digit counts); then per digit the wave
// offsets and the digit starts.
template <int kRounds = kBucketRounds>
__device__ __forceinline__ void bucket_rank_scatter(BucketLds& L, const uint32_t (&dig)[kRounds], const uint32_t (&val)[kRounds],
                                    int nb, int nbits, uint32_t* out, int R)
{
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t rank[kRounds];
    rank_digits(L, dig, nb, nbits, R, rank);
#pragma unroll
    for (int r = 0; r < kRounds; r++) {
        if (r >= R) break;
        if ((w * R + r) * 64 + lane < nb) out[L.dstart[dig[r]] + L.wcnt[w][dig[r]] + rank[r]] = val[r];
    }
    __syncthreads();
}

// Bucket too large for LDS: the same stable passes through global memory, 1024 keys at a time
// (digit bases from a histogram of the whole bucket, advanced chunk by chunk).  (k0, v0) holds the
// bucket; (k1, v1) is scratch of the same size.  Returns the buffer index holding the result.
__device__ __forceinline__ int bucket_global_sort(BucketLds& L, uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, int nb,
                                  int lowbits)
{
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    uint32_t* K[2] = {k0, k1};
    uint32_t* V[2] = {v0, v1};
    int src = 0;
    for (int sh = 0; sh < lowbits; sh += 8) {
        const int nbits = min(8, lowbits - sh);
        const uint32_t mask = (1u << nbits) - 1u;
        if (t < 256) L.ctot[t] = 0u;
        __syncthreads();
        for (int i = t; i < nb; i += kBucketThreads) atomicAdd(&L.ctot[(K[src][i] >> sh) & mask], 1u);
        __syncthreads();
        const uint32_t ex = scan256(t < 256 ? L.ctot[t] : 0u, L.wsum);
        if (t < 256) L.dstart[t] = ex;
        __syncthreads();
        for (int c0 = 0; c0 < nb; c0 += kBucketThreads) {
            const int idx = c0 + t;
            const bool valid = idx < nb;
            const uint32_t key = valid ? K[src][idx] : 0u, val = valid ? V[src][idx] : 0u;
            const uint32_t d = (key >> sh) & mask;
            const uint64_t peers = match_digit(d, valid, nbits);
            const uint32_t rr = (uint32_t)__popcll(peers & lanemask_lt());
            for (int i = t; i < kBucketWaves * 256; i += kBucketThreads) (&L.wcnt[0][0])[i] = 0u;
            __syncthreads();
            if (valid && rr == 0) L.wcnt[w][d] = (uint32_t)__popcll(peers);
            __syncthreads();
            if (t < 256) {
                uint32_t run = 0;
                for (int i = 0; i < kBucketWaves; i++) {
                    const uint32_t c = L.wcnt[i][t];
                    L.wcnt[i][t] = run;
                    run += c;
                }
                L.ctot[t] = run;
            }
            __syncthreads();
            if (valid) {
                const uint32_t pos = L.dstart[d] + L.wcnt[w][d] + rr;
                K[src ^ 1][pos] = key;
                V[src ^ 1][pos] = val;
            }
            __syncthreads();
            if (t < 256) L.dstart[t] += L.ctot[t];
            __syncthreads();
        }
        src ^= 1;
        (void)lane;
    }
    return src;
}

// Exclusive scan of one value per thread over a kBucketThreads workgroup (every thread calls it);
// *total receives the sum.
__device__ __forceinline__ uint32_t scan1024(uint32_t v, uint32_t* wsum, uint32_t* total)
{
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kBucketWaves; i++) {
        const uint32_t c = wsum[i];
        before += i < w ? c : 0u;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return before + x - v;
}

// Fused super-tile emission (round 2).  With `keys` set, the bucket workgroups also write what
// k_emit_super would: each visible Gaussian's super-tile entries, in depth order, at the exclusive
// prefix of the entry counts.  Every workgroup publishes its bucket's entry total ({flag, total} in
// one 64-bit word) as soon as it has it, then sums its predecessors' words into its base (an LDS
// bucket after its sort; a bucket sorted in global memory counts its entries before sorting).
// Buckets are taken by ticket, so every predecessor of a waiting workgroup is already running, and
// no workgroup waits before it has published.  A
// wait that reaches the spin bound computes the base from the inputs instead (same value) and flags
// the stall.  A workgroup whose entries would pass `cap` writes none: the host sees E > cap after
// its wait and runs the depth order again without emission, then k_emit_super.  With emission the
// depth-order arrays k_emit_super reads (sorted ids, ranked rectangles, local offsets) are not
// written.
struct BucketEmit {
    uint32_t* keys;  // null: no emission
    uint32_t* vals;
    uint32_t cap;
    uint64_t* status;  // one word per bucket + the ticket (status[buckets]), zero at launch
    int msd_bits;      // the bucket map's digit bits (stall fallbacks)
    int sgx;
    uint32_t* stall;
    uint32_t spin_limit;
    const uint32_t* depth_key;  // stall fallback: the entries of all Gaussians in lower buckets
    const uint2* rect;
    int P;
    // the super-tile pass's [super-tile][block] histogram (null: not counted here), blocks of
    // kSuperHistBlock entry positions, row stride hstride; zero at launch (the MSD histogram
    // launch clears it)
    uint32_t* shist;
    int hstride;
    int supers;
    // placed emission (sup_status != null, supers <= 256): every entry is written at its position
    // in the super-tile-major list the binning reads (super-tile, then depth order), so no
    // super-tile radix pass follows.  The k-th entry of super-tile s in bucket d goes to base(s)
    // (the MSD histogram's super-tile rows, scanned with its digit rows) + the entries of s in
    // buckets 0..d-1 (the sum of their published counts) + k.
    uint32_t* sup_status;       // [super-tile][bucket] {kSupAgg | count}, cleared by preprocess
    const uint32_t* sup_base;   // sup_base[s * sup_stride] = P + base(s)
    int sup_stride;
    const uint32_t* etotal;     // counters[kCntSuper]: all entries of the view (no emission above cap)
    int sbits;                  // super-tile id bits
    const uint32_t* kxf;        // stall fallback: the bucket map
};
constexpr uint32_t kSupAgg = 1u << 30;  // sup_status: the flag of a published count
constexpr uint32_t kSupVal = kSupAgg - 1u;
static_assert(kSuperHistBlock == 4 * kRadixThreads, "super-tile pass blocks: k_radix_scatter<4> tiles");

// Writes Gaussian g's entries from position o and counts them into the super-tile histogram:
// hl (LDS, [super-tile][block - b0], nbl blocks) or, without it, straight into em.shist.
__device__ __forceinline__ void emit_entries(const BucketEmit& em, uint32_t o, uint32_t g, uint2 rc,
                                             uint32_t* hl = nullptr, uint32_t b0 = 0, int nbl = 0)
{
    if (rc.x == rc.y) return;  // culled: no entries
    int sx0, sy0, sx1, sy1;
    super_rect(rc, sx0, sy0, sx1, sy1);
    for (int y = sy0; y < sy1; y++)
        for (int x = sx0; x < sx1; x++) {
            em.keys[o] = entry_key(rc, x, y, em.sgx);
            em.vals[o] = g;
            const int sid = y * em.sgx + x;
            const uint32_t blk = o / kSuperHistBlock;
            if (hl)
                atomicAdd(&hl[sid * nbl + (int)(blk - b0)], 1u);
            else if (em.shist)
                atomicAdd(&em.shist[(size_t)sid * em.hstride + blk], 1u);
            o++;
        }
}

__device__ __forceinline__ void publish_bucket_total(const BucketEmit& em, int d, uint32_t total)
{
    if (em.keys && threadIdx.x == 0)
        __hip_atomic_store(&em.status[d], kFlagAgg | (uint64_t)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The entry base of bucket d: the sum of the totals of buckets 0..d-1 (every thread calls it).
template <int kDig>
__device__ __forceinline__ uint32_t bucket_entry_base(const BucketEmit& em, int d, const uint32_t* kxf, uint32_t* wsum)
{
    __shared__ uint32_t s_base;
    __shared__ int s_ok;
    const int t = threadIdx.x;
    if (t < 64) {
        uint32_t part = 0, spins = 0;
        bool ok = true;
        // every predecessor's word requested at once (up to kDig / 64 per lane: one memory round trip
        // when they are all published, instead of one per 64 predecessors), then the missing ones polled
        constexpr int kPer = kDig / 64;
        uint64_t w[kPer];
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int b = k * 64 + t;
            w[k] = b < d ? __hip_atomic_load(&em.status[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagAgg;
        }
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            if (k * 64 >= d || !ok) break;  // wave-uniform
            const int b = k * 64 + t;
            while (em.spin_limit == 0u || __ballot((w[k] >> 62) == 0ull) != 0ull) {
                if (em.spin_limit == 0u || ++spins > em.spin_limit) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                if ((w[k] >> 62) == 0ull)
                    w[k] = __hip_atomic_load(&em.status[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            part += (uint32_t)w[k];
        }
        part = wave_sum(part);
        if (t == 0) {
            s_base = part;
            s_ok = ok ? 1 : 0;
        }
    }
    __syncthreads();
    if (s_ok) return s_base;
    // stalled: the entries of every Gaussian whose bucket is below d, from the inputs
    const MsdMap mm = msd_map(kxf, em.msd_bits);
    uint32_t part = 0;
    for (int g = t; g < em.P; g += kBucketThreads)
        if (msd_bucket(key_xf(em.depth_key[g], kxf), mm) < (uint32_t)d) part += super_count(em.rect[g]);
    uint32_t tot;
    scan1024(part, wsum, &tot);
    if (t == 0) note_stall(em.stall);
    return tot;
}

// Placed emission's counts, in em.sup_status (cleared by preprocess): [super-tile][bucket] words
// {kSupAgg | count} (row stride kDig buckets), then per group of 16 buckets [group][super-tile] words
// {kSupAgg | the group's count}, then kDig / 16 group arrival counters.  Every bucket publishes its
// counts as soon as its rectangles are loaded; the last of a group to arrive also publishes the
// group's sums.  A bucket's prefix for super-tile s is then < kDig / 16 group sums + <= 15 counts
// of its own group (30 words with 256 buckets, 46 with 512; not d), read once the bucket is sorted,
// when they are long published.
template <int kDig>
constexpr size_t sup_group_off() { return 256 * (size_t)kDig; }  // words: the group sums
template <int kDig>
constexpr size_t sup_arrive_off() { return sup_group_off<kDig>() + 256 * (size_t)(kDig / kSupGroup); }  // the counters
static_assert(sup_arrive_off<256>() + 256 / kSupGroup == sup_words(256), "placed emission's count words");
static_assert(sup_arrive_off<512>() + 512 / kSupGroup == kSupWords, "placed emission's count words");

template <int kDig>
__device__ __forceinline__ void publish_super_counts(const BucketLds& L, const BucketEmit& em, int d)
{
    constexpr size_t kSupGroupOff = sup_group_off<kDig>(), kSupArriveOff = sup_arrive_off<kDig>();
    const int t = threadIdx.x, g = d / kSupGroup;
    __shared__ int s_last;
    // relaxed atomics throughout (release / acquire at agent scope would write back / invalidate the
    // L2 per operation): every word carries its own flag, and readers poll for it
    if (t < em.supers)
        __hip_atomic_store(&em.sup_status[(size_t)t * kDig + d], kSupAgg | L.scnt[t], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (t == 0)
        s_last = __hip_atomic_fetch_add(&em.sup_status[kSupArriveOff + g], 1u, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT) == kSupGroup - 1;
    __syncthreads();
    if (!s_last || t >= em.supers || em.spin_limit == 0u) return;
    // the group's last arrival: every member has published (its flags are polled all the same)
    uint32_t v[kSupGroup];
#pragma unroll
    for (int j = 0; j < kSupGroup; j++)
        v[j] = __hip_atomic_load(&em.sup_status[(size_t)t * kDig + g * kSupGroup + j], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    uint32_t sum = 0, spins = 0;
#pragma unroll
    for (int j = 0; j < kSupGroup; j++) {
        while (!(v[j] & kSupAgg)) {
            // bounded: past it the group's sums are not published, and every later bucket's sum
            // takes its own bounded wait and then its fallback (the prefixes from the inputs)
            if (++spins > em.spin_limit) return;
            __builtin_amdgcn_s_sleep(1);
            v[j] = __hip_atomic_load(&em.sup_status[(size_t)t * kDig + g * kSupGroup + j], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
        }
        sum += v[j] & kSupVal;
    }
    __hip_atomic_store(&em.sup_status[kSupGroupOff + (size_t)g * 256 + t], kSupAgg | sum, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Adds to L.run[s] the entries of super-tile s in buckets 0..d-1 (s < S; every thread calls it):
// the group sums below d's group and the counts of d's group members below d, one word per
// thread and pair (s, j < kSlots) in flight at once; false when a wait passed the spin bound.
template <int kDig>
__device__ __forceinline__ bool super_sum(BucketLds& L, const BucketEmit& em, int d)
{
    if (em.spin_limit == 0u) return false;  // never wait: the fallback (tests)
    constexpr size_t kSupGroupOff = sup_group_off<kDig>();
    constexpr int kGroups = kDig / kSupGroup;
    constexpr int kSlots = kGroups + kSupGroup;  // per super-tile: group sums, then group members
    const int t = threadIdx.x;
    const int g = d / kSupGroup, r = d - g * kSupGroup;
    constexpr int kPer = 256 * kSlots / kBucketThreads;  // (s, j) pairs per thread, j < kSlots
    const int total = em.supers * kSlots;
    uint32_t v[kPer];
    int at[kPer];  // word index, -1: none
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const int f = k * kBucketThreads + t, sj = f / kSlots, j = f % kSlots;
        at[k] = -1;
        v[k] = kSupAgg;
        if (f < total) {
            if (j < g)
                at[k] = (int)(kSupGroupOff + (size_t)j * 256 + sj);
            else if (j >= kGroups && j - kGroups < r)
                at[k] = sj * kDig + g * kSupGroup + (j - kGroups);
            if (at[k] >= 0)
                v[k] = __hip_atomic_load(&em.sup_status[at[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    uint32_t spins = 0;
    for (;;) {
        bool wait = false;
#pragma unroll
        for (int k = 0; k < kPer; k++)
            if (at[k] >= 0 && !(v[k] & kSupAgg)) {
                wait = true;
                v[k] = __hip_atomic_load(&em.sup_status[at[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        if (!__syncthreads_or(wait)) break;
        if (em.spin_limit == 0u || ++spins > em.spin_limit) return false;  // workgroup-uniform
        __builtin_amdgcn_s_sleep(1);
    }
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if (at[k] >= 0 && (v[k] & kSupVal)) atomicAdd(&L.run[(k * kBucketThreads + t) / kSlots], v[k] & kSupVal);
    return true;
}

// Placed emission: the write cursors L.run[s] = base(s) (thread s holds it) + the entries of
// super-tile s in buckets 0..d-1 (every thread calls it).  A sum that waited past the spin bound
// is computed from the inputs instead (same values).
template <int kDig>
__device__ __forceinline__ void super_cursors(BucketLds& L, const BucketEmit& em, int d, uint32_t base_s)
{
    const int t = threadIdx.x;
    __shared__ int s_ok;
    if (t < 256) L.run[t] = 0u;
    __syncthreads();
    const bool ok = super_sum<kDig>(L, em, d);
    if (t == 0) s_ok = ok ? 1 : 0;
    __syncthreads();
    if (!s_ok) {  // stalled: per super-tile, the entries of every Gaussian whose bucket is below d
        if (t < 256) L.run[t] = 0u;
        __syncthreads();
        const MsdMap mm = msd_map(em.kxf, em.msd_bits);
        for (int gg = t; gg < em.P; gg += kBucketThreads) {
            const uint2 rc = em.rect[gg];
            if (rc.x == rc.y || msd_bucket(key_xf(em.depth_key[gg], em.kxf), mm) >= (uint32_t)d) continue;
            int sx0, sy0, sx1, sy1;
            super_rect(rc, sx0, sy0, sx1, sy1);
            for (int y = sy0; y < sy1; y++)
                for (int x = sx0; x < sx1; x++) atomicAdd(&L.run[y * em.sgx + x], 1u);
        }
        __syncthreads();
        if (t == 0) note_stall(em.stall);
    }
    if (t < em.supers) L.run[t] += base_s;
    __syncthreads();
}

// the bucket's entries per super-tile, into L.scnt
__device__ __forceinline__ void count_supers(BucketLds& L, const BucketEmit& em, uint2 rc)
{
    if (rc.x == rc.y) return;
    int sx0, sy0, sx1, sy1;
    super_rect(rc, sx0, sy0, sx1, sy1);
    for (int y = sy0; y < sy1; y++)
        for (int x = sx0; x < sx1; x++) atomicAdd(&L.scnt[y * em.sgx + x], 1u);
}

// Placed emission: a list of up to kBucketCap entries {key (L.w[0]), Gaussian id (L.w[1])} in
// LDS, in the bucket's entry order (depth order; a Gaussian's super-tiles row by row).
// list_entries writes the entries [e0, e0 + n) of this thread's Gaussians r (id gid[r],
// rectangle rc[r], first entry off[r] in the bucket's order; ~0u: none) at position - e0.
template <int kG>
__device__ __forceinline__ void list_entries(BucketLds& L, const BucketEmit& em, const uint32_t (&gid)[kG], const uint2 (&rc)[kG],
                             const uint32_t (&off)[kG], uint32_t e0, uint32_t n)
{
#pragma unroll
    for (int r = 0; r < kG; r++) {
        if (off[r] >= e0 + n || rc[r].x == rc[r].y) continue;  // none here / culled
        int sx0, sy0, sx1, sy1;
        super_rect(rc[r], sx0, sy0, sx1, sy1);
        uint32_t e = off[r];
        for (int y = sy0; y < sy1; y++)
            for (int x = sx0; x < sx1; x++, e++)
                if (e >= e0 && e < e0 + n) {
                    L.w[0][e - e0] = entry_key(rc[r], x, y, em.sgx);
                    L.w[1][e - e0] = gid[r];
                }
    }
}

// list_entries for the nb Gaussians of a bucket parked in global memory in depth order (ids, tile
// rectangles, first entry offsets), one thread per Gaussian.
__device__ __forceinline__ void list_entries_parked(BucketLds& L, const BucketEmit& em, const uint32_t* gid,
                                                    const uint2* grc, const uint32_t* goff, int nb, uint32_t e0,
                                                    uint32_t n)
{
    for (int i = threadIdx.x; i < nb; i += kBucketThreads) {
        const uint32_t o = goff[i];
        if (o >= e0 + n) continue;
        const uint2 rc = grc[i];
        if (rc.x == rc.y) continue;  // culled
        int sx0, sy0, sx1, sy1;
        super_rect(rc, sx0, sy0, sx1, sy1);
        if (o + (uint32_t)((sx1 - sx0) * (sy1 - sy0)) <= e0) continue;  // all before this list
        const uint32_t g = gid[i];
        uint32_t e = o;
        for (int y = sy0; y < sy1; y++)
            for (int x = sx0; x < sx1; x++, e++)
                if (e >= e0 && e < e0 + n) {
                    L.w[0][e - e0] = entry_key(rc, x, y, em.sgx);
                    L.w[1][e - e0] = g;
                }
    }
}

// Reorders the n listed entries stably by super-tile id (the key's low 8 bits), in place, with the
// sort's ballot ranking; leaves the chunk-local super-tile starts in L.dstart.
__device__ __forceinline__ void rank_entries(BucketLds& L, const BucketEmit& em, int n)
{
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int R = (n + kBucketThreads - 1) / kBucketThreads;
    uint32_t a[kBucketRounds], b[kBucketRounds], dig[kBucketRounds], rank[kBucketRounds];
#pragma unroll
    for (int r = 0; r < kBucketRounds; r++) {
        if (r >= R) break;  // workgroup-uniform
        const int p = (w * R + r) * 64 + lane;
        a[r] = p < n ? L.w[0][p] : 0u;
        b[r] = p < n ? L.w[1][p] : 0u;
        dig[r] = a[r] & 0xFFu;
    }
    rank_digits(L, dig, n, em.sbits, R, rank);  // its barriers: every load above has landed
#pragma unroll
    for (int r = 0; r < kBucketRounds; r++) {
        if (r >= R) break;
        if ((w * R + r) * 64 + lane < n) {
            const uint32_t pos = L.dstart[dig[r]] + L.wcnt[w][dig[r]] + rank[r];
            L.w[0][pos] = a[r];
            L.w[1][pos] = b[r];
        }
    }
    __syncthreads();
}

// Writes the n ranked entries super-tile by super-tile from the cursors L.run[s] (consecutive
// threads on consecutive positions) and advances each cursor by its super-tile's count.
__device__ __forceinline__ void write_entries(BucketLds& L, const BucketEmit& em, uint32_t n)
{
    const int t = threadIdx.x;
    for (uint32_t j = t; j < n; j += kBucketThreads) {
        const uint32_t k = L.w[0][j];
        const uint32_t s = k & 0xFFu;
        const uint32_t o = L.run[s] + j - L.dstart[s];
        em.keys[o] = k;
        em.vals[o] = L.w[1][j];
    }
    __syncthreads();
    if (t < 256) L.run[t] += (t < 255 ? L.dstart[t + 1] : n) - L.dstart[t];
    __syncthreads();
}

// Placed emission from global memory (a bucket beyond LDS, or one with more entries than
// kBucketCap): 1024 Gaussians at a time in depth order (ids rid[0, nb),
// rectangles by id), their entries listed, ranked and written kBucketCap at a time.
__device__ __forceinline__ void place_runs(BucketLds& L, const BucketEmit& em, const uint32_t* rid, int nb)
{
    const int t = threadIdx.x;
    for (int c0 = 0; c0 < nb; c0 += kBucketThreads) {
        const int i = c0 + t;
        uint32_t gid[1] = {0u}, off[1] = {~0u};
        uint2 rc[1] = {make_uint2(0u, 0u)};
        if (i < nb) {
            gid[0] = rid[i];
            rc[0] = em.rect[gid[0]];
        }
        uint32_t m;
        const uint32_t ex = scan1024(i < nb ? super_count(rc[0]) : 0u, L.wsum, &m);
        if (i < nb) off[0] = ex;
        for (uint32_t e0 = 0; e0 < m; e0 += kBucketCap) {
            const uint32_t n = min((uint32_t)kBucketCap, m - e0);
            list_entries(L, em, gid, rc, off, e0, n);
            __syncthreads();
            rank_entries(L, em, (int)n);
            write_entries(L, em, n);
        }
    }
}

// One workgroup per bucket (top-digit value).  keys / ids: the MSD pass's output (transformed keys,
// bucket-contiguous, id order inside a bucket; rect_ranked holds the rectangles in the same
// layout); hist_scan: its scanned [digit][block] histogram, whose digit starts are the bucket
// ranges.  rect: the rectangles by id (global fallback only).  Writes, for every position of the bucket, the sorted
// id, the depth-ordered rectangle and the BUCKET-LOCAL exclusive prefix of the super-tile entry
// counts (local_off), and the bucket's total entry count (totals[d], 0 for empty buckets):
// k_emit_super adds the scanned bucket totals, so no separate P-long scan is launched.  scratch_k
// is P words of scratch for the global fallback (whose ids go through sorted_ids itself).
// Measurement hook (LSR_BUCKET_TIMELINE=1): per bucket workgroup {start, end} (s_memrealtime,
// 100 MHz), its hardware slot (XCC_ID << 16 | HW_ID bits 8..15), its key count and the times at
// which the first pass, all passes and the output gathers ended.
__device__ uint32_t g_bucket_timeline[512 * 8];

#ifndef LSR_BUCKET_MARK_BASE  // measurement knob: the timeline's 4th mark when the entry base is known
                              // (placed emission: when the entries are listed and ranked)
#define LSR_BUCKET_MARK_BASE 0
#endif
#ifndef LSR_BUCKET_WAVES  // one bucket workgroup per CU: no need to squeeze registers for two
#define LSR_BUCKET_WAVES 4
#endif
#ifndef LSR_BUCKET_WAVES_512  // the 512-bucket sort (measurement knob): 8 = two workgroups per CU, all 512
#define LSR_BUCKET_WAVES_512 4  // at once, at 64 VGPRs + 56 B of scratch without placed emission: C5 depth
#endif                          // order 150.9-151.7 against 148.6-148.9 us at 4 (profiles/r05_c5_msd512.txt)
// kDig buckets (256, or 512 above kMsdMaxKeys).
template <int kDig>
__global__ __launch_bounds__(kBucketThreads)
__attribute__((amdgpu_waves_per_eu(kDig == 512 ? LSR_BUCKET_WAVES_512 : LSR_BUCKET_WAVES, 8)))
void k_depth_bucket_sort(
    int n, uint32_t* __restrict__ keys, uint32_t* __restrict__ ids, const uint32_t* __restrict__ hist_scan, int nblk,
    const uint32_t* __restrict__ kxf, const uint2* __restrict__ rect, uint32_t* __restrict__ sorted_ids,
    uint2* __restrict__ rect_ranked, uint32_t* __restrict__ local_off, uint32_t* __restrict__ totals,
    uint32_t* __restrict__ scratch_k, int timeline, BucketEmit em)
{
    const uint64_t t_start = timeline ? wall_clock64() : 0;
    struct TimelineGuard {  // written when the workgroup leaves, on every path
        int on;
        uint64_t t0;
        int nb;
        uint32_t ph[4];
        __device__ __forceinline__ void mark(int i)
        {
            if (on) ph[i] = (uint32_t)wall_clock64();
        }
        __device__ __forceinline__ ~TimelineGuard()
        {
            if (!on || threadIdx.x != 0) return;
            const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
            uint32_t* o = g_bucket_timeline + 8 * blockIdx.x;
            o[0] = (uint32_t)t0;
            o[1] = (uint32_t)wall_clock64();
            o[2] = ((xcc & 0xFu) << 16) | ((hw >> 8) & 0xFFu);
            o[3] = (uint32_t)nb;
            o[4] = ph[0];
            o[5] = ph[1];
            o[6] = ph[2];
            o[7] = ph[3];
        }
    } guard{timeline, t_start, 0, {0u, 0u, 0u, 0u}};
    extern __shared__ uint4 s_bucket_raw[];
    BucketLds& L = *reinterpret_cast<BucketLds*>(s_bucket_raw);
    const int t = threadIdx.x;
    int d = (int)blockIdx.x;
    // every bucket's start from the scanned [bucket][block] histogram, loaded while the ticket is
    // taken (the range no longer waits behind the ticket's round trip)
    static_assert(kDig <= kBucketThreads, "one bucket start per thread");
    __shared__ uint32_t s_start[kDig + 1];
    if (t < kDig) s_start[t] = hist_scan[(size_t)t * nblk];
    if (t == kDig) s_start[kDig] = (uint32_t)n;
    // placed emission: on when the view's entries fit (block-uniform); base(s) loaded early
    const bool placed = em.sup_status && *em.etotal <= em.cap;
    const uint32_t base_s = placed && t < em.supers ? em.sup_base[(size_t)t * em.sup_stride] - (uint32_t)em.P : 0u;
    if (t < 256) L.scnt[t] = 0u;
    if (em.keys) {  // fused emission: buckets by ticket (a waiting workgroup's predecessors run)
        __shared__ int s_d;
        if (t == 0) s_d = (int)atomicAdd(reinterpret_cast<uint32_t*>(em.status + kDig), 1u);
        __syncthreads();
        d = s_d;
    } else {
        __syncthreads();
    }
    const uint32_t start = s_start[d];
    const uint32_t end = s_start[d + 1];
    const int nb = (int)(end - start);
    guard.nb = nb;
    if (nb <= 0) {  // no key in this depth interval
        if (t == 0) totals[d] = 0u;
        if (placed) publish_super_counts<kDig>(L, em, d);  // zeros (L.scnt cleared before the ticket's barrier)
        if (!placed) publish_bucket_total(em, d, 0u);
        return;
    }
    // the bucket's own key range [lo, hi]: it sorts key - lo on the bits that span
    const int w = t >> 6, lane = t & 63;
    uint32_t kr[kBucketRounds];
    uint32_t klo = 0xFFFFFFFFu, khi = 0u;
    // rounds of 64 keys per wave in use: every wave holds a share of the bucket
    const int R = (nb + kBucketThreads - 1) / kBucketThreads;
    if (nb <= kBucketCap) {
#pragma unroll
        for (int r = 0; r < kBucketRounds; r++) {
            const int idx = (w * R + r) * 64 + lane;
            kr[r] = r < R && idx < nb ? keys[start + idx] : 0u;
            if (r < R && idx < nb) {
                klo = min(klo, kr[r]);
                khi = max(khi, kr[r]);
            }
        }
        if (placed) {  // the bucket's entries per super-tile (rectangles in the keys' layout)
            uint2 q[kBucketRounds];
#pragma unroll
            for (int r = 0; r < kBucketRounds; r++) {
                const int idx = (w * R + r) * 64 + lane;
                q[r] = r < R && idx < nb ? rect_ranked[start + idx] : make_uint2(0u, 0u);
            }
#pragma unroll
            for (int r = 0; r < kBucketRounds; r++) count_supers(L, em, q[r]);
        }
    } else {
        for (int i = t; i < nb; i += kBucketThreads) {
            const uint32_t k = keys[start + i];
            klo = min(klo, k);
            khi = max(khi, k);
            if (placed) count_supers(L, em, rect_ranked[start + i]);
        }
    }
    {
        __shared__ uint32_t s_lo[kBucketWaves], s_hi[kBucketWaves];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            klo = min(klo, (uint32_t)__shfl_xor((int)klo, o, 64));
            khi = max(khi, (uint32_t)__shfl_xor((int)khi, o, 64));
        }
        if (lane == 0) {
            s_lo[w] = klo;
            s_hi[w] = khi;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kBucketWaves; i++) {
            klo = min(klo, s_lo[i]);
            khi = max(khi, s_hi[i]);
        }
    }
    const uint32_t span = khi - klo;
    const int lowbits = span ? 32 - __clz(span) : 0;
    if (placed) publish_super_counts<kDig>(L, em, d);  // counts completed by the barrier above
    const uint32_t* place_rid = nullptr;  // placed tail: ids in depth order, and the entry total
    uint32_t place_etot = 0;
    // the LDS sort packs {key bits 8.., local index} in one word: at most 27 key bits
    if (nb <= kBucketCap && lowbits <= 32 - kIdxBits + 8) {
        uint32_t dig[kBucketRounds], val[kBucketRounds];
        // pass 0 from registers: the keys in wave-blocked order, digit = bits 0..7 of key - lo, and
        // the packed word {bits 8.., local index} as the value
#pragma unroll
        for (int r = 0; r < kBucketRounds; r++) {
            const int idx = (w * R + r) * 64 + lane;
            const uint32_t k = r < R && idx < nb ? kr[r] - klo : 0u;
            dig[r] = k & 0xFFu;
            val[r] = ((k >> 8) << kIdxBits) | ((uint32_t)idx & kIdxMask);
        }
        if (timeline && !LSR_BUCKET_MARK_BASE) {  // measurement only: the keys' arrival
            __builtin_amdgcn_s_waitcnt(0);
            guard.mark(3);
        }
        int src = 0;
        if (lowbits > 0) {
            bucket_rank_scatter(L, dig, val, nb, min(8, lowbits), L.w[0], R);
            guard.mark(0);
        } else {
#pragma unroll
            for (int r = 0; r < kBucketRounds; r++) {
                const int idx = (w * R + r) * 64 + lane;
                if (r < R && idx < nb) L.w[0][idx] = val[r];
            }
            __syncthreads();
        }
        for (int sh = 8; sh < lowbits; sh += 8) {  // later passes: the digit from the packed word
#pragma unroll
            for (int r = 0; r < kBucketRounds; r++) {
                const int idx = (w * R + r) * 64 + lane;
                val[r] = r < R && idx < nb ? L.w[src][idx] : 0u;
                dig[r] = (val[r] >> (kIdxBits + sh - 8)) & 0xFFu;
            }
            bucket_rank_scatter(L, dig, val, nb, min(8, lowbits - sh), L.w[src ^ 1], R);
            src ^= 1;
        }
        guard.mark(1);
        // outputs: ids and rectangles (carried into rect_ranked by the MSD pass) permuted inside the
        // bucket.  Global reads and writes stay coalesced: each array is loaded in bucket order,
        // staged in the two free 32 KB LDS buffers and gathered there through the local indices
        // (lidx).  rect_ranked is permuted in place: all of its loads have landed in LDS before the
        // barriers that precede the stores.  The entry counts then go through LDS so that each thread
        // scans a contiguous run of R of them.
        uint32_t* S = L.w[src];
        uint32_t* X = L.w[src ^ 1];
        uint32_t lidx[kBucketRounds], id[kBucketRounds], ry[kBucketRounds];
        uint2 rc[kBucketRounds];
#pragma unroll
        for (int r = 0; r < kBucketRounds; r++) {
            if (r >= R) break;  // workgroup-uniform
            const int i = t + r * kBucketThreads;
            lidx[r] = i < nb ? S[i] & kIdxMask : 0u;
            id[r] = i < nb ? ids[start + i] : 0u;
            rc[r] = i < nb ? rect_ranked[start + i] : make_uint2(0u, 0u);
        }
        __syncthreads();  // S read by everyone
#pragma unroll
        for (int r = 0; r < kBucketRounds; r++) {
            if (r >= R) break;  // workgroup-uniform
            const int i = t + r * kBucketThreads;
            if (i < nb) {
                X[i] = id[r];
                S[i] = rc[r].x;
            }
            ry[r] = rc[r].y;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kBucketRounds; r++) {
            if (r >= R) break;
            id[r] = X[lidx[r]];
            rc[r].x = S[lidx[r]];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kBucketRounds; r++) {
            if (r >= R) break;  // workgroup-uniform
            const int i = t + r * kBucketThreads;
            if (i < nb) X[i] = ry[r];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kBucketRounds; r++) {
            if (r >= R) break;
            rc[r].y = X[lidx[r]];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kBucketRounds; r++) {
            if (r >= R) break;  // workgroup-uniform
            const int i = t + r * kBucketThreads;
            if (i < nb) {
                if (!em.keys) {  // fused emission: no later kernel reads the depth-order arrays
                    const uint32_t o = start + (uint32_t)i;
                    sorted_ids[o] = id[r];
                    rect_ranked[o] = rc[r];
                }
                X[i] = super_count(rc[r]);
            }
        }
        __syncthreads();
        guard.mark(2);
        uint32_t c[kBucketRounds], run = 0;
#pragma unroll
        for (int k = 0; k < kBucketRounds; k++) {
            if (k >= R) break;
            const int j = R * t + k;
            c[k] = j < nb ? X[j] : 0u;
            run += c[k];
        }
        uint32_t tot;
        uint32_t acc = scan1024(run, L.wsum, &tot);
#pragma unroll
        for (int k = 0; k < kBucketRounds; k++) {
            if (k >= R) break;
            const int j = R * t + k;
            if (j < nb) X[j] = acc;
            acc += c[k];
        }
        if (t == 0) totals[d] = tot;
        __syncthreads();
        if (placed) {
            uint32_t off[kBucketRounds];
#pragma unroll
            for (int r = 0; r < kBucketRounds; r++) {
                const int i = t + r * kBucketThreads;
                off[r] = r < R && i < nb ? X[i] : ~0u;
            }
            __syncthreads();  // X read: both buffers now hold the entry list
            if (tot <= (uint32_t)kBucketCap) {
                list_entries(L, em, id, rc, off, 0u, tot);
                __syncthreads();
                rank_entries(L, em, (int)tot);
                if (LSR_BUCKET_MARK_BASE) guard.mark(3);  // measurement only: listed and ranked
                super_cursors<kDig>(L, em, d, base_s);
                write_entries(L, em, tot);
                return;
            }
            if constexpr (kDig == 512) {
                // more entries than one list (the 512 buckets' ~6k Gaussians): lists of kBucketCap
                // entries in the bucket's entry order, each listed from the sorted Gaussians parked
                // in the depth-order arrays this fused emission leaves unused (write_entries advances
                // the super-tile cursors, so a later list's entries follow an earlier one's in every
                // super-tile); the arrays' barrier-ordered stores and loads stay in this workgroup.
                // (256 buckets keep the global tail below: this path's registers, 127 instead of
                // 104, would keep the bucket workgroup from sharing a CU in the pipelined step)
#pragma unroll
                for (int r = 0; r < kBucketRounds; r++) {
                    if (r >= R) break;
                    const int i = t + r * kBucketThreads;
                    if (i < nb) {
                        sorted_ids[start + i] = id[r];
                        rect_ranked[start + i] = rc[r];
                        local_off[start + i] = off[r];
                    }
                }
                super_cursors<kDig>(L, em, d, base_s);  // its barriers order the stores before the loads
                for (uint32_t e0 = 0; e0 < tot; e0 += (uint32_t)kBucketCap) {
                    const uint32_t n = min((uint32_t)kBucketCap, tot - e0);
                    list_entries_parked(L, em, sorted_ids + start, rect_ranked + start, local_off + start, nb, e0,
                                        n);
                    __syncthreads();
                    rank_entries(L, em, (int)n);
                    write_entries(L, em, n);
                }
                return;
            }
            // more entries than one list: the Gaussians' ids in depth order through global memory
            // (the placed tail below, shared with the global path)
#pragma unroll
            for (int r = 0; r < kBucketRounds; r++) {
                if (r >= R) break;
                const int i = t + r * kBucketThreads;
                if (i < nb) sorted_ids[start + i] = id[r];
            }
            place_rid = sorted_ids + start;
            place_etot = tot;
            goto placed_tail;
        }
        if (!em.keys) {
#pragma unroll
            for (int r = 0; r < kBucketRounds; r++) {
                if (r >= R) break;
                const int i = t + r * kBucketThreads;
                if (i < nb) local_off[start + i] = X[i];
            }
            return;
        }
        // the total is published once known (after the sort): a workgroup waiting for its base waits
        // for the slowest predecessor's sort, which with buckets of similar size ends about when
        // its own does (publishing before the sort put a rectangle load and a scan on every
        // workgroup's critical path instead)
        publish_bucket_total(em, d, tot);
        const uint32_t ebase = bucket_entry_base<kDig>(em, d, kxf, L.wsum);
        if (LSR_BUCKET_MARK_BASE) guard.mark(3);  // measurement only: the entry base known
        if ((uint64_t)ebase + tot > (uint64_t)em.cap) return;  // over capacity: the host re-runs unfused
        // the bucket's entries [ebase, ebase + tot) meet nbl blocks of the super-tile pass: their
        // [super-tile][block] counts in LDS (the free buffer S), then one atomic per non-zero count
        // (blocks at the bucket's ends are shared with its neighbours)
        const uint32_t b0 = ebase / kSuperHistBlock;
        const int nbl = tot ? (int)((ebase + tot - 1) / kSuperHistBlock - b0) + 1 : 0;
        uint32_t* hl = em.shist && tot && nbl * em.supers <= kBucketCap ? S : nullptr;
        if (hl) {
            for (int i = t; i < nbl * em.supers; i += kBucketThreads) hl[i] = 0u;
            __syncthreads();
        }
#pragma unroll
        for (int r = 0; r < kBucketRounds; r++) {
            if (r >= R) break;  // workgroup-uniform
            const int i = t + r * kBucketThreads;
            if (i < nb) emit_entries(em, ebase + X[i], id[r], rc[r], hl, b0, nbl);
        }
        if (hl) {
            __syncthreads();
            for (int i = t; i < nbl * em.supers; i += kBucketThreads) {
                const uint32_t v = hl[i];
                if (v) atomicAdd(&em.shist[(size_t)(i / nbl) * em.hstride + b0 + (uint32_t)(i % nbl)], v);
            }
        }
        return;
    }
    {  // beyond LDS: global passes between (keys, ids) and (scratch_k, sorted_ids) over the bucket
    uint32_t etot = 0;
    if (em.keys) {  // the bucket's entry total first (bucket layout: any order gives the same sum)
        uint32_t part = 0;
        for (int i = t; i < nb; i += kBucketThreads) part += super_count(rect_ranked[start + i]);
        scan1024(part, L.wsum, &etot);
        if (!placed) publish_bucket_total(em, d, etot);
    }
    for (int i = t; i < nb; i += kBucketThreads) keys[start + i] -= klo;  // sort key - lo
    __syncthreads();
    const int res = bucket_global_sort(L, keys + start, ids + start, scratch_k + start, sorted_ids + start, nb,
                                       lowbits);
    const uint32_t* rid = res ? sorted_ids + start : ids + start;
    if (placed) {
        place_rid = rid;
        place_etot = etot;
        goto placed_tail;
    }
    const uint32_t ebase = em.keys ? bucket_entry_base<kDig>(em, d, kxf, L.wsum) : 0u;
    const bool emit = em.keys && (uint64_t)ebase + etot <= (uint64_t)em.cap;
    uint32_t carry = 0;
    for (int c0 = 0; c0 < nb; c0 += kBucketThreads) {  // in order, 1024 positions at a time
        const int i = c0 + t;
        uint32_t cnt = 0, g = 0;
        uint2 rc = make_uint2(0u, 0u);
        if (i < nb) {
            g = rid[i];
            rc = rect[g];
            if (!em.keys) {
                sorted_ids[start + i] = g;  // in place when rid aliases sorted_ids
                rect_ranked[start + i] = rc;
            }
            cnt = super_count(rc);
        }
        uint32_t tot;
        const uint32_t ex = scan1024(cnt, L.wsum, &tot);
        if (i < nb) {
            if (!em.keys) local_off[start + i] = carry + ex;
            if (emit) emit_entries(em, ebase + carry + ex, g, rc);
        }
        carry += tot;
    }
    if (t == 0) totals[d] = carry;
    return;
    }
placed_tail:  // placed emission from global memory: the Gaussians' ids in depth order at place_rid
    super_cursors<kDig>(L, em, d, base_s);  // its barriers also order the id stores before the reads
    place_runs(L, em, place_rid, nb);
    if (t == 0) totals[d] = place_etot;
}

static int bucket_timeline_on()
{
    static const int v = [] {
        const char* e = getenv("LSR_BUCKET_TIMELINE");
        return e && e[0] == '1' ? 1 : 0;
    }();
    return v;
}

hipError_t bucket_timeline_read(uint32_t* out, int n)
{
    if (n > 512) n = 512;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bucket_timeline), sizeof(uint32_t) * 8 * n, 0,
                               hipMemcpyDeviceToHost);
}

template <int kDig>
static hipError_t allow_bucket_lds()
{
    static const hipError_t e = hipFuncSetAttribute((const void*)k_depth_bucket_sort<kDig>,
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBucketLdsBytes);
    return e;
}

// The depth order of P keys: 0 = LSD passes, else the MSD pass's bucket count -- 256 up to
// kMsdMaxKeys, 512 up to kMsd512MaxKeys (about 8k keys per bucket on average: the LDS sort's
// capacity), LSD above.  Knobs (measurement / tests, read per call): LSR_DEPTH_LSD=1 forces the LSD
// passes; LSR_MSD_MAX_KEYS=n and LSR_MSD512_MAX_KEYS=n move the two limits; LSR_MSD_BUCKETS=512
// takes 512 buckets wherever the MSD pass runs.
constexpr int64_t kMsd512MaxKeys = 4200000;
int msd_digits(int P)
{
    const char* e = getenv("LSR_DEPTH_LSD");
    if (e && e[0] == '1') return 0;
    const char* m = getenv("LSR_MSD_MAX_KEYS");
    const char* m2 = getenv("LSR_MSD512_MAX_KEYS");
    const char* b = getenv("LSR_MSD_BUCKETS");
    const int64_t lim = m ? (int64_t)atoll(m) : kMsdMaxKeys;
    const int64_t lim2 = m2 ? (int64_t)atoll(m2) : kMsd512MaxKeys;
    if (P <= lim) return b && atoi(b) == 512 ? 512 : 256;
    return P <= lim2 ? 512 : 0;
}

bool depth_order_uses_pass_count(int P) { return msd_digits(P) == 0; }

// ---------------------------------------------------------------- depth order + super-tile counts

bool fused_emit_enabled()
{
    static const bool v = [] {
        const char* e = getenv("LSR_FUSED_EMIT");
        return !(e && e[0] == '0');
    }();
    return v;
}

// Keys per thread of the MSD pass's radix tiles: 16 above radix_small's limit, else 8 with 512
// buckets (C5 depth order 152 -> 139 us against 4, profiles/r05_c5_msd512.txt) and 4 with 256 (the
// tiles that fit beside the pipelined step's render kernels, radix_small); LSR_MSD_ITEMS=4 / 8
// (measurement knob, read per call) sets it for either bucket count.
static int msd_items(int P)
{
    if (!radix_small(P)) return 16;
    const char* e = getenv("LSR_MSD_ITEMS");
    if (e && (atoi(e) == 4 || atoi(e) == 8)) return atoi(e);
    return msd_digits(P) == 512 ? 8 : 4;
}

int msd_blocks(int P)
{
    const int tile = kRadixThreads * msd_items(P);
    return (P + tile - 1) / tile;
}

bool placed_emit(const Layout& L, bool geometry_phase, int buckets)
{
    if (L.supers > 256) return false;
    const char* e = getenv("LSR_PLACED");
    if (e && (e[0] == '0' || e[0] == '1')) return e[0] == '1';
    return !geometry_phase && buckets == 256;
}

hipError_t launch_depth_order(int P, int passes, const Layout& L, char* geom, uint32_t* counters, uint32_t* stall,
                              hipStream_t s, bool debug, bool fused_emit, uint32_t emit_cap, bool placed_req)
{
    if (P == 0) return hipSuccess;
    uint32_t* hist = reinterpret_cast<uint32_t*>(geom + L.radix_hist);
    uint32_t* hist_scan = reinterpret_cast<uint32_t*>(geom + L.radix_hist_scan);
    uint32_t* regions = reinterpret_cast<uint32_t*>(geom + L.scan_regions);
    uint32_t* ka = reinterpret_cast<uint32_t*>(geom + L.keys_a);
    uint32_t* kb = reinterpret_cast<uint32_t*>(geom + L.keys_b);
    uint32_t* va = reinterpret_cast<uint32_t*>(geom + L.sorted_ids);
    uint32_t* vb = reinterpret_cast<uint32_t*>(geom + L.vals_b);
    // radix_sort ends in its (kA, vA) pair after an even number of passes and in (kB, vB) after an
    // odd one: swap the roles so the ids always end in sorted_ids
    int done = 0;
    const uint32_t* keys = reinterpret_cast<const uint32_t*>(geom + L.depth_key);
    uint32_t* off = reinterpret_cast<uint32_t*>(geom + L.super_offset);
    // the last pass stores no keys, so its key output buffer (keys_a in both role assignments) is
    // free: the per-rank super-tile entry counts go there and are scanned into super_offset
    const ScatterTail tail{reinterpret_cast<const uint2*>(geom + L.rect), reinterpret_cast<uint2*>(geom + L.rect_ranked),
                           ka};
    const uint32_t* kxf = counters + kCntKeyMin;
    const int nd = msd_digits(P);
    if (nd) {  // MSD pass + per-bucket LDS sort; `passes` is not used
        hipError_t e = nd == 512 ? allow_bucket_lds<512>() : allow_bucket_lds<256>();
        if (e != hipSuccess) return e;
        static const int remap = [] {
            const char* v = getenv("LSR_XCD_REMAP");
            return v && v[0] == '0' ? 0 : 1;
        }();
        const int items = msd_items(P);
        const bool small = items == 4;
        const int nblk = (P + kRadixThreads * items - 1) / (kRadixThreads * items);
        const int dbits = nd == 512 ? 9 : 8;
        // placed emission: the MSD histogram also counts each block's super-tile entries (rows nd + s);
        // else the super-tile histogram the bucket sort counts into, and its scan's status words
        const bool placed = fused_emit && placed_req && L.supers <= 256;
        const bool shist_on = fused_emit && !placed && L.super_hist_words > 0;
        const ZeroList zmsd = shist_on
            ? ZeroList{{reinterpret_cast<uint32_t*>(geom + L.super_hist), reinterpret_cast<uint32_t*>(geom + L.super_hist_status),
                        nullptr, nullptr},
                       {(int)L.super_hist_words, (int)L.super_hist_status_words, 0, 0}}
            : ZeroList{};
        const uint2* srect = placed ? tail.rect : nullptr;
        const DevCount nodc{nullptr, nullptr};
        if (nd == 512) {
            if (small)
                hipLaunchKernelGGL((k_radix_hist<4, 512>), dim3(nblk), dim3(kRadixThreads), 0, s, keys, P, 0, 9, hist,
                                   nblk, kxf, remap, 9, zmsd, nodc, srect, L.supers, L.sgx, (const uint32_t*)nullptr);
            else if (items == 8)
                hipLaunchKernelGGL((k_radix_hist<8, 512>), dim3(nblk), dim3(kRadixThreads), 0, s, keys, P, 0, 9, hist,
                                   nblk, kxf, remap, 9, zmsd, nodc, srect, L.supers, L.sgx, (const uint32_t*)nullptr);
            else
                hipLaunchKernelGGL((k_radix_hist<16, 512>), dim3(nblk), dim3(kRadixThreads), 0, s, keys, P, 0, 9, hist,
                                   nblk, kxf, remap, 9, zmsd, nodc, srect, L.supers, L.sgx, (const uint32_t*)nullptr);
        } else if (small) {
            hipLaunchKernelGGL(k_radix_hist<4>, dim3(nblk), dim3(kRadixThreads), 0, s, keys, P, 0, 8, hist, nblk, kxf,
                               remap, 8, zmsd, nodc, srect, L.supers, L.sgx);
        } else if (items == 8) {
            hipLaunchKernelGGL(k_radix_hist<8>, dim3(nblk), dim3(kRadixThreads), 0, s, keys, P, 0, 8, hist, nblk, kxf,
                               remap, 8, zmsd, nodc, srect, L.supers, L.sgx);
        } else {
            hipLaunchKernelGGL(k_radix_hist<16>, dim3(nblk), dim3(kRadixThreads), 0, s, keys, P, 0, 8, hist, nblk, kxf,
                               remap, 8, zmsd, nodc, srect, L.supers, L.sgx);
        }
        if ((e = post(debug, s)) != hipSuccess) return e;
        if ((e = scan_exclusive(hist, hist_scan, (nd + (placed ? L.supers : 0)) * nblk, regions, nullptr, stall, s,
                                debug)) != hipSuccess)
            return e;
        // the rectangles ride along into rect_ranked (bucket layout); the bucket sort permutes them
        const ScatterTail carry{tail.rect, tail.rect_ranked, nullptr};
        if (nd == 512) {
            if (small)
                hipLaunchKernelGGL((k_radix_scatter<4, true, 512>), dim3(nblk), dim3(kRadixThreads), 0, s, keys,
                                   (const uint32_t*)nullptr, P, 0, 9, hist_scan, nblk, kb, vb, kxf, carry, remap, 9, nodc,
                                   0, 512, ZeroList{}, (const uint32_t*)nullptr);
            else if (items == 8)
                hipLaunchKernelGGL((k_radix_scatter<8, true, 512>), dim3(nblk), dim3(kRadixThreads), 0, s, keys,
                                   (const uint32_t*)nullptr, P, 0, 9, hist_scan, nblk, kb, vb, kxf, carry, remap, 9, nodc,
                                   0, 512, ZeroList{}, (const uint32_t*)nullptr);
            else
                hipLaunchKernelGGL((k_radix_scatter<16, true, 512>), dim3(nblk), dim3(kRadixThreads), 0, s, keys,
                                   (const uint32_t*)nullptr, P, 0, 9, hist_scan, nblk, kb, vb, kxf, carry, remap, 9, nodc,
                                   0, 512, ZeroList{}, (const uint32_t*)nullptr);
        } else if (small) {
            hipLaunchKernelGGL((k_radix_scatter<4, true>), dim3(nblk), dim3(kRadixThreads), 0, s, keys,
                               (const uint32_t*)nullptr, P, 0, 8, hist_scan, nblk, kb, vb, kxf, carry, remap, 8, nodc);
        } else if (items == 8) {
            hipLaunchKernelGGL((k_radix_scatter<8, true>), dim3(nblk), dim3(kRadixThreads), 0, s, keys,
                               (const uint32_t*)nullptr, P, 0, 8, hist_scan, nblk, kb, vb, kxf, carry, remap, 8, nodc);
        } else {
            hipLaunchKernelGGL((k_radix_scatter<16, true>), dim3(nblk), dim3(kRadixThreads), 0, s, keys,
                               (const uint32_t*)nullptr, P, 0, 8, hist_scan, nblk, kb, vb, kxf, carry, remap, 8, nodc);
        }
        if ((e = post(debug, s)) != hipSuccess) return e;
        // bucket-local offsets into super_offset, bucket totals for k_emit_super (no P-long scan);
        // with fused emission also the super-tile entries themselves
        BucketEmit em{};
        em.msd_bits = dbits;
        if (fused_emit) {
            em.keys = reinterpret_cast<uint32_t*>(geom + L.fused_keys);
            em.vals = reinterpret_cast<uint32_t*>(geom + L.fused_vals);
            em.cap = emit_cap > 0 && emit_cap < (uint32_t)L.fused_cap ? emit_cap : (uint32_t)L.fused_cap;
            em.status = reinterpret_cast<uint64_t*>(geom + L.bucket_status);
            em.sgx = L.sgx;
            em.stall = stall;
            em.spin_limit = stall_spin_limit();
            em.depth_key = keys;
            em.rect = tail.rect;
            em.P = P;
            em.shist = shist_on ? reinterpret_cast<uint32_t*>(geom + L.super_hist) : nullptr;
            em.hstride = L.super_hist_stride;
            em.supers = L.supers;
            if (placed) {
                em.sup_status = reinterpret_cast<uint32_t*>(geom + L.sup_status);
                em.sup_base = hist_scan + (size_t)nd * nblk;
                em.sup_stride = nblk;
                em.etotal = counters + kCntSuper;
                em.sbits = L.super_bits;
                em.kxf = kxf;
            }
        }
        if (nd == 512)
            hipLaunchKernelGGL(k_depth_bucket_sort<512>, dim3(512), dim3(kBucketThreads), kBucketLdsBytes, s, P, kb, vb,
                               (const uint32_t*)hist_scan, nblk, kxf, tail.rect, va, tail.rect_ranked, off,
                               reinterpret_cast<uint32_t*>(geom + L.bucket_totals), ka, bucket_timeline_on(), em);
        else
            hipLaunchKernelGGL(k_depth_bucket_sort<256>, dim3(256), dim3(kBucketThreads), kBucketLdsBytes, s, P, kb, vb,
                               (const uint32_t*)hist_scan, nblk, kxf, tail.rect, va, tail.rect_ranked, off,
                               reinterpret_cast<uint32_t*>(geom + L.bucket_totals), ka, bucket_timeline_on(), em);
        return post(debug, s);
    }
    hipError_t e = (passes & 1)
        ? radix_sort(keys, nullptr, P, 8 * passes, kb, vb, ka, va, hist, hist_scan, regions, L.scan_region_geom, stall,
                     s, debug, &done, counters + kCntKeyMin, tail, ZeroList{}, DevCount{nullptr, nullptr}, kxf)
        : radix_sort(keys, nullptr, P, 8 * passes, ka, va, kb, vb, hist, hist_scan, regions, L.scan_region_geom, stall,
                     s, debug, &done, counters + kCntKeyMin, tail, ZeroList{}, DevCount{nullptr, nullptr}, kxf);
    if (e != hipSuccess) return e;
    return scan_exclusive(ka, off, P, regions + passes * L.scan_region_geom, counters + kCntSuper, stall, s, debug);
}

// ---------------------------------------------------------------- binning

// Super-tile entries in depth order (keys = entry_key, vals = Gaussian id); also clears what the
// later kernels need cleared (tile and super-tile ranges, the segment count table, scan status).
// offset[r]: the entry offset of depth rank r; with the MSD depth order (msd.totals != null) only
// bucket-local, the bucket bases being the exclusive scan of msd.totals over the buckets.
struct MsdOffsets {
    const uint32_t* totals;     // per top-digit bucket: super-tile entries (k_depth_bucket_sort), or null
    const uint32_t* hist_scan;  // the MSD pass's scanned [digit][block] histogram: bucket starts
    int nblk;
    const uint32_t* kxf;        // visible depth-key min / max: the number of buckets
    int ndig;                   // buckets: 256 or 512
};

__global__ __launch_bounds__(256) void k_emit_super(int P, int sgx, const uint32_t* __restrict__ sorted_ids,
                                                    const uint32_t* __restrict__ offset,
                                                    const uint2* __restrict__ rect_ranked,
                                                    uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                    uint32_t* __restrict__ z0, int n0, uint32_t* __restrict__ z1,
                                                    int n1, uint32_t* __restrict__ z2, int n2,
                                                    uint32_t* __restrict__ z3, int n3, MsdOffsets msd, DevCount dc)
{
    __shared__ uint32_t s_start[512], s_base[512], s_wsum[4];
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    const int stride = gridDim.x * blockDim.x;
    // this rank's inputs first: their round trip overlaps the bucket bases' below
    uint2 rc = make_uint2(0u, 0u);
    uint32_t g = 0, o = 0;
    if (r < P) {
        rc = rect_ranked[r];
        g = sorted_ids[r];
        o = offset[r];
    }
    const int per = msd.ndig / 256;  // buckets per thread (1 or 2, consecutive)
    if (msd.totals) {  // bucket starts and bases (every workgroup, 256 threads)
        const int t = threadIdx.x;
        uint32_t v[2] = {0u, 0u}, x = 0;
        for (int j = 0; j < per; j++) {
            const int b = per * t + j;
            s_start[b] = msd.hist_scan[(size_t)b * msd.nblk];
            v[j] = msd.totals[b];
            x += v[j];
        }
        const uint32_t sum = x;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if ((t & 63) >= o) x += y;
        }
        if ((t & 63) == 63) s_wsum[t >> 6] = x;
        __syncthreads();
        uint32_t before = 0;
        for (int i = 0; i < (t >> 6); i++) before += s_wsum[i];
        uint32_t ex = before + x - sum;
        for (int j = 0; j < per; j++) {
            s_base[per * t + j] = ex;
            ex += v[j];
        }
        __syncthreads();
    }
    for (int w = r; w < n0; w += stride) z0[w] = 0u;
    for (int w = r; w < n1; w += stride) z1[w] = 0u;
    for (int w = r; w < n2; w += stride) z2[w] = 0u;
    for (int w = r; w < n3; w += stride) z3[w] = 0u;
    if (dc.abort && *dc.abort) return;    // capacity mode, view over capacity: nothing is binned
    if (r >= P || rc.x == rc.y) return;  // past the ranks, or culled (empty rectangle)
    int sx0, sy0, sx1, sy1;
    super_rect(rc, sx0, sy0, sx1, sy1);
    if (msd.totals) {  // + the base of the bucket holding rank r: the last bucket starting at or before r
        int lo = 0, hi = msd.ndig - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_start[mid] <= (uint32_t)r) lo = mid;
            else hi = mid - 1;
        }
        o += s_base[lo];
    }
    for (int y = sy0; y < sy1; y++)
        for (int x = sx0; x < sx1; x++) {
            keys[o] = entry_key(rc, x, y, sgx);
            vals[o] = g;
            o++;
        }
}

// [start, end) of every super-tile in the sorted entries (the low 16 key bits)
__global__ __launch_bounds__(256) void k_super_ranges(int64_t E, const uint32_t* __restrict__ keys,
                                                      uint2* __restrict__ ranges, DevCount dc)
{
    if (dc.abort && *dc.abort) return;
    if (dc.n) E = min(E, (int64_t)*dc.n);
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= E) return;
    const uint32_t t = keys[k] & 0xFFFFu;
    if (k == 0 || (keys[k - 1] & 0xFFFFu) != t) ranges[t].x = (uint32_t)k;
    if (k == E - 1 || (keys[k + 1] & 0xFFFFu) != t) ranges[t].y = (uint32_t)(k + 1);
}

__device__ __forceinline__ uint32_t super_segments(uint2 r) { return (r.y - r.x + kSegEntries - 1) / kSegEntries; }

// Positions in the tile-major (tile, segment) count table, in closed form: tile t = (tx, ty) of
// super-tile s = (sx, sy) starts at row_prefix[ty] + col_prefix[s] + (tx - 8 sx) * nseg(s), where
// col_prefix[s] sums nseg x width over the super-tiles left of s in its row and row_prefix[ty] sums
// whole tile rows above ty.  One workgroup builds seg_base (segment -> super-tile map) and both
// prefixes from the S super-tile ranges.
__global__ __launch_bounds__(kScanThreads) void k_seg_setup(int S, int sgx, int sgy, int gx, int gy,
                                                            const uint2* __restrict__ sranges,
                                                            uint32_t* __restrict__ seg_base,
                                                            uint32_t* __restrict__ col_prefix,
                                                            uint32_t* __restrict__ row_prefix, DevCount dc)
{
    if (dc.abort && *dc.abort) return;
    __shared__ uint32_t wsum[kScanThreads / 64];
    extern __shared__ uint32_t row_total[];  // per super-row: tiles-weighted segment count of one tile row
    uint32_t carry = 0;
    for (int b = 0; b < S; b += kScanThreads) {
        const int i = b + threadIdx.x;
        const uint32_t v = i < S ? super_segments(sranges[i]) : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(v, wsum, &tot);
        if (i < S) seg_base[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) seg_base[S] = carry;
    for (int sy = threadIdx.x; sy < sgy; sy += blockDim.x) {
        uint32_t run = 0;
        for (int sx = 0; sx < sgx; sx++) {
            const int s = sy * sgx + sx;
            col_prefix[s] = run;
            run += super_segments(sranges[s]) * (uint32_t)min(kSuper, gx - sx * kSuper);
        }
        row_total[sy] = run;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int ty = 0; ty < gy; ty++) {
            row_prefix[ty] = run;
            run += row_total[ty / kSuper];
        }
        row_prefix[gy] = run;
    }
}

// This workgroup's (super-tile, segment) and its context; false for the grid's spare blocks.  Every
// thread tests its share of the S intervals [seg_base[s], seg_base[s + 1]) and loads the
// interval's super-tile range and column prefix alongside: one memory round trip on every
// workgroup's critical path (a binary search by one thread, then the context loads, were ~13
// dependent loads).
struct SegmentCtx {
    int s, seg, ox, oy;
    uint32_t e0, e1, nseg, colpre;
};

__device__ __forceinline__ bool block_segment_ctx(int S, int sgx, const uint32_t* __restrict__ seg_base,
                                                  const uint2* __restrict__ sranges,
                                                  const uint32_t* __restrict__ col_prefix, SegmentCtx* out)
{
    __shared__ uint32_t sh[5];
    // XCD-aware segment order (xcd_tile): consecutive segments of a super-tile write adjacent runs of
    // the same tile lists, so they are given to workgroups of one XCD, whose L2 then assembles the
    // shared point_list lines (instead of 8 L2s each writing back partial lines).  Over the segments
    // that exist (seg_base[S], read in the same round trip as the lookup), not the grid, whose
    // capacity-mode size exceeds them.
    const uint32_t nseg_all = seg_base[S];
    constexpr int kMaxPer = 4;  // intervals per thread, loaded before the block index is known
    uint32_t lo[kMaxPer], hi[kMaxPer], cp[kMaxPer];
    uint2 rr[kMaxPer];
#pragma unroll
    for (int k = 0; k < kMaxPer; k++) {
        const int s = threadIdx.x + k * blockDim.x;
        if (s < S) {
            lo[k] = seg_base[s];
            hi[k] = seg_base[s + 1];
            rr[k] = sranges[s];
            cp[k] = col_prefix[s];
        }
    }
    if (threadIdx.x == 0) sh[0] = 0xFFFFFFFFu;
    __syncthreads();
    if (blockIdx.x >= nseg_all) return false;  // block-uniform
    const int i = (int)blockIdx.x, n = (int)nseg_all;
    const int x = i & 7, q = n >> 3, r = n & 7;  // as xcd_tile: XCD x takes [x q + min(x, r), ...)
    const uint32_t b = (uint32_t)(x * q + min(x, r) + (i >> 3));
#pragma unroll
    for (int k = 0; k < kMaxPer; k++) {
        const int s = threadIdx.x + k * blockDim.x;
        if (s < S && lo[k] <= b && b < hi[k]) {
            sh[0] = (uint32_t)s;
            sh[1] = b - lo[k];
            sh[2] = rr[k].x;
            sh[3] = rr[k].y;
            sh[4] = cp[k];
        }
    }
    for (int s = threadIdx.x + kMaxPer * blockDim.x; s < S; s += blockDim.x) {  // beyond 1024 super-tiles
        const uint32_t l = seg_base[s], h = seg_base[s + 1];
        if (l <= b && b < h) {
            const uint2 rs = sranges[s];
            sh[0] = (uint32_t)s;
            sh[1] = b - l;
            sh[2] = rs.x;
            sh[3] = rs.y;
            sh[4] = col_prefix[s];
        }
    }
    __syncthreads();
    if (sh[0] == 0xFFFFFFFFu) return false;
    SegmentCtx& c = *out;
    c.s = (int)sh[0];
    c.seg = (int)sh[1];
    c.ox = (c.s % sgx) * kSuper;
    c.oy = (c.s / sgx) * kSuper;
    const uint2 rg = make_uint2(sh[2], sh[3]);
    c.e0 = rg.x + (uint32_t)c.seg * kSegEntries;
    c.e1 = min(rg.y, c.e0 + (uint32_t)kSegEntries);
    c.nseg = super_segments(rg);
    c.colpre = sh[4];
    return true;
}

// count-table slot of (local tile l, segment 0) of the super-tile, -1 outside the image;
// *gt = its global tile id
__device__ __forceinline__ int64_t table_slot(const SegmentCtx& c, int l, int gx, int gy,
                                              const uint32_t* __restrict__ row_prefix, int* gt)
{
    const int x = c.ox + (l & 7), y = c.oy + (l >> 3);
    if (x >= gx || y >= gy) return -1;
    *gt = y * gx + x;
    return (int64_t)row_prefix[y] + c.colpre + (uint32_t)(l & 7) * c.nseg;
}

// Per (tile, segment) entry counts into the tile-major count table.
__global__ __launch_bounds__(256) void k_bin_count(int S, int sgx, int gx, int gy, const uint32_t* __restrict__ seg_base,
                                                   const uint2* __restrict__ sranges,
                                                   const uint32_t* __restrict__ col_prefix,
                                                   const uint32_t* __restrict__ row_prefix,
                                                   const uint32_t* __restrict__ keys, uint32_t* __restrict__ table,
                                                   DevCount dc)
{
    if (dc.abort && *dc.abort) return;
    __shared__ uint32_t cnt[64];
    SegmentCtx c;
    if (!block_segment_ctx(S, sgx, seg_base, sranges, col_prefix, &c)) return;
    const int seg = c.seg;
    if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t mine = 0;  // lane l: entries of this wave covering local tile l
    for (uint32_t b = c.e0 + (threadIdx.x & ~63u); b < c.e1; b += 256) {
        const uint32_t e = b + (threadIdx.x & 63);
        const uint64_t m = e < c.e1 ? entry_mask(keys[e]) : 0ull;
        mine += (uint32_t)__popcll(transpose64(m));
    }
    atomicAdd(&cnt[threadIdx.x & 63], mine);
    __syncthreads();
    if (threadIdx.x < 64) {
        int gt;
        const int64_t slot = table_slot(c, threadIdx.x, gx, gy, row_prefix, &gt);
        if (slot >= 0) table[slot + seg] = cnt[threadIdx.x];
    }
}

// Writes every (tile, Gaussian) pair of a segment at its final point_list position, and the tile
// ranges (segment 0 of each super-tile).  `table` holds the scanned counts.  Per batch of 256
// entries: each wave transposes its 64 masks (lane l <- column of local tile l), so an entry's
// rank in tile l is popcount(column & lanes below) past the lower waves' columns.  The batch's
// output is up to 64 contiguous runs (one per tile); it is staged in LDS tile-major and written
// with consecutive lanes on consecutive addresses (batches over kStage instances store directly).
#ifndef LSR_BIN_STAGE  // staging capacity in instances (LDS: 5 B each); measurement knob
#define LSR_BIN_STAGE 4096
#endif
constexpr int kStage = LSR_BIN_STAGE;

// k_bin_count with the segment setup folded in, for a super-tile sort of ONE radix pass (S <= 256
// super-tiles): the super-tile ranges are then the digit starts of the scanned [digit][block]
// histogram (digit s starts at hist[s * nblk]; digits >= S are empty), so k_super_ranges and the
// one-workgroup k_seg_setup are not launched.  Every workgroup rebuilds the segment map of the S
// super-tiles in LDS (S loads + a block scan), finds its own segment in it, and workgroup 0 also
// writes the map to global memory for k_bin_emit.  Same counts as k_seg_setup + k_bin_count.
constexpr int kFusedSupers = 256;

__global__ __launch_bounds__(256) void k_bin_count_fused(int S, int sgx, int sgy, int gx, int gy, int nblk, int ndig,
                                                         int64_t E, const uint32_t* __restrict__ hist,
                                                         uint2* __restrict__ g_sranges, uint32_t* __restrict__ g_seg_base,
                                                         uint32_t* __restrict__ g_colpre, uint32_t* __restrict__ g_rowpre,
                                                         const uint32_t* __restrict__ keys, uint32_t* __restrict__ table,
                                                         DevCount dc, uint32_t bias = 0, ZeroList zero = ZeroList{},
                                                         int64_t table_words = 0)
{
    // placed emission (no super-tile pass before this launch): hist = the MSD histogram's scanned
    // super-tile rows (bias = its key count), and this launch clears what the later kernels need
    // cleared (zero: tile ranges, the table scan's status words; table_words: the count table past
    // the slots written below)
    zero_words_strided(zero);
    if (dc.abort && *dc.abort) return;
    if (dc.n) E = min(E, (int64_t)*dc.n);
    // super-tile s's entries are [sstart[s], sstart[s + 1]) (ndig >= S at both call sites, so a
    // range's end is the next one's start): one word per super-tile keeps the launch under 6 KB of
    // LDS, i.e. beside the 7 pipelined backward workgroups a CU holds (lsr_render.hip kSharedWgsBwd)
    __shared__ uint32_t sstart[kFusedSupers + 1];
    __shared__ uint32_t sbase[kFusedSupers + 1];
    __shared__ uint32_t scol[kFusedSupers];
    __shared__ uint32_t srow_tot[kFusedSupers];      // per super-row: segment-weighted count of one tile row
    __shared__ uint32_t srow_pre[kFusedSupers + 1];  // whole tile rows above super-row sy
    __shared__ uint32_t wsum[4];
    __shared__ uint32_t cnt[64];
    __shared__ int sh[2];
    const int t = threadIdx.x;
    uint32_t nseg = 0;
    if (t < S) {
        const uint32_t a = hist[(size_t)t * nblk] - bias;
        const uint32_t b = t + 1 < ndig ? hist[(size_t)(t + 1) * nblk] - bias : (uint32_t)E;
        sstart[t] = a;
        if (t == S - 1) sstart[S] = b;
        nseg = super_segments(make_uint2(a, b));
    }
    auto sr = [&](int i) { return make_uint2(sstart[i], sstart[i + 1]); };
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan(nseg, wsum, &tot);
    if (t < S) sbase[t] = ex;
    if (t == 0) sbase[S] = tot;
    // column prefixes inside each super-row and the row totals from one scan of the
    // tile-weighted segment counts (a row's prefix = scan - scan at the row start)
    const int sy = t < S ? t / sgx : 0, sx = t - sy * sgx;
    const uint32_t wv = t < S ? nseg * (uint32_t)min(kSuper, gx - sx * kSuper) : 0u;
    uint32_t wtot;
    const uint32_t wex = block_exclusive_scan(wv, wsum, &wtot);
    scol[t] = wex;  // global exclusive scan for now
    __syncthreads();
    const uint32_t row0 = t < S ? scol[sy * sgx] : 0u;
    if (t < S && sx == sgx - 1) srow_tot[sy] = wex + wv - row0;
    __syncthreads();
    if (t < S) scol[t] = wex - row0;
    // whole tile rows above each super-row
    const uint32_t rv = t < sgy ? srow_tot[t] * (uint32_t)min(kSuper, gy - t * kSuper) : 0u;
    uint32_t rtot;
    const uint32_t rex = block_exclusive_scan(rv, wsum, &rtot);
    if (t < sgy) srow_pre[t] = rex;
    if (t == 0) {
        srow_pre[sgy] = rtot;
        sh[0] = -1;
        sh[1] = 0;
    }
    for (int64_t w = (int64_t)rtot + (int64_t)blockIdx.x * blockDim.x + t; w < table_words;
         w += (int64_t)gridDim.x * blockDim.x)
        table[w] = 0u;
    __syncthreads();
    // this workgroup's (super-tile, segment): the s with sbase[s] <= b < sbase[s + 1]
    {
        // XCD-aware segment order, as k_bin_emit (block_segment_ctx): adjacent count-table words
        // are written by one XCD
        const int i = (int)blockIdx.x, n = (int)sbase[S];
        const int x = i & 7, q = n >> 3, r = n & 7;
        const uint32_t b = i < n ? (uint32_t)(x * q + min(x, r) + (i >> 3)) : (uint32_t)i;
        if (t < S && sbase[t] <= b && b < sbase[t + 1]) {
            sh[0] = t;
            sh[1] = (int)(b - sbase[t]);
        }
    }
    __syncthreads();
    auto row_prefix = [&](int y) { return srow_pre[y / kSuper] + (uint32_t)(y % kSuper) * srow_tot[y / kSuper]; };
    if (blockIdx.x == 0) {  // the map for k_bin_emit
        for (int i = t; i < S; i += blockDim.x) {
            g_sranges[i] = sr(i);
            g_seg_base[i] = sbase[i];
            g_colpre[i] = scol[i];
        }
        if (t == 0) g_seg_base[S] = sbase[S];
        for (int y = t; y <= gy; y += blockDim.x) g_rowpre[y] = y < gy ? row_prefix(y) : srow_pre[sgy];
    }
    const int s = sh[0], seg = sh[1];
    if (s < 0) return;
    SegmentCtx c;
    c.s = s;
    c.seg = seg;
    c.ox = (s % sgx) * kSuper;
    c.oy = (s / sgx) * kSuper;
    c.e0 = sr(s).x + (uint32_t)seg * kSegEntries;
    c.e1 = min(sr(s).y, c.e0 + (uint32_t)kSegEntries);
    c.nseg = super_segments(sr(s));
    c.colpre = scol[s];
    // the segment's (at most 2 x 256) keys loaded together: one memory round trip
    constexpr int kBatches = kSegEntries / 256;
    uint32_t kq[kBatches];
#pragma unroll
    for (int q = 0; q < kBatches; q++) {
        const uint32_t e = c.e0 + (uint32_t)(q * 256 + t);
        kq[q] = e < c.e1 ? keys[e] : 0u;
    }
    if (t < 64) cnt[t] = 0;
    __syncthreads();
    uint32_t mine = 0;  // lane l: entries of this wave covering local tile l
#pragma unroll
    for (int q = 0; q < kBatches; q++) {
        const uint32_t e = c.e0 + (uint32_t)(q * 256 + t);
        mine += (uint32_t)__popcll(transpose64(e < c.e1 ? entry_mask(kq[q]) : 0ull));
    }
    atomicAdd(&cnt[t & 63], mine);
    __syncthreads();
    if (t < 64) {
        const int x = c.ox + (t & 7), y = c.oy + (t >> 3);
        if (x < gx && y < gy) table[(int64_t)row_prefix(y) + c.colpre + (uint32_t)(t & 7) * c.nseg + seg] = cnt[t];
    }
}

__global__ __launch_bounds__(256) void k_bin_emit(int S, int sgx, int gx, int gy, const uint32_t* __restrict__ seg_base,
                                                  const uint2* __restrict__ sranges,
                                                  const uint32_t* __restrict__ col_prefix,
                                                  const uint32_t* __restrict__ row_prefix,
                                                  const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                  const uint32_t* __restrict__ table, uint32_t* __restrict__ point_list,
                                                  uint2* __restrict__ ranges, uint32_t* __restrict__ sched_counts,
                                                  uint32_t* __restrict__ sched_lists, DevCount dc)
{
    if (dc.abort && *dc.abort) return;
    __shared__ uint64_t colw[4][64];
    __shared__ uint32_t pre[4][64];    // per wave: rank base of tile l inside the batch's staging
    __shared__ uint32_t cursor[64];    // global position of tile l's next instance
    __shared__ uint32_t toff[65];      // batch staging offset of tile l (exclusive scan), total
    __shared__ uint32_t stage_g[kStage];
    __shared__ uint8_t stage_t[kStage];
    __shared__ uint32_t sg[4][64];     // the batch's Gaussian ids, entry order
    SegmentCtx c;
    if (!block_segment_ctx(S, sgx, seg_base, sranges, col_prefix, &c)) return;
    const int seg = c.seg;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    // both batches' entries loaded up front (a segment is at most kSegEntries = 2 x 256 entries):
    // one memory round trip instead of one per batch
    constexpr int kBatches = kSegEntries / 256;
    uint32_t gq[kBatches], kq[kBatches];
#pragma unroll
    for (int q = 0; q < kBatches; q++) {
        const uint32_t e = c.e0 + (uint32_t)(q * 256 + t);
        gq[q] = e < c.e1 ? vals[e] : 0u;
        kq[q] = e < c.e1 ? keys[e] : 0u;
    }
    if (t < 64) {
        int gt = 0;
        const int64_t slot = table_slot(c, t, gx, gy, row_prefix, &gt);
        cursor[t] = slot >= 0 ? table[slot + seg] : 0u;
        if (seg == 0 && slot >= 0) {
            const uint2 r = make_uint2(table[slot], table[slot + c.nseg]);
            ranges[gt] = r;
            // the forward's longest-first schedule: work = list length
            if (r.y > r.x) schedule_tile(sched_counts, sched_lists, gx * gy, gt, r.y - r.x);
        }
    }
#pragma unroll
    for (int q = 0; q < kBatches; q++) {
        const uint32_t b = c.e0 + (uint32_t)(q * 256);
        if (b >= c.e1) break;  // block-uniform
        const uint32_t e = b + t;
        const uint32_t g = gq[q];
        const uint64_t m = e < c.e1 ? entry_mask(kq[q]) : 0ull;
        colw[wave][lane] = transpose64(m);
        sg[wave][lane] = g;
        __syncthreads();
        if (t < 64) {  // wave 0, lane l = tile l: per-wave bases and the tile-major staging scan
            uint32_t run = 0;
#pragma unroll
            for (int w = 0; w < 4; w++) {
                pre[w][t] = run;
                run += (uint32_t)__popcll(colw[w][t]);
            }
            uint32_t x = run;  // inclusive scan of the tile totals over the 64 lanes
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if (t >= o) x += y;
            }
            toff[t] = x - run;
            if (t == 63) toff[64] = x;
        }
        __syncthreads();
        const uint32_t total = toff[64];
        // thread (wave, lane = local tile l) places the wave's entries covering tile l, in entry
        // order: a loop over one column of the transposed masks, so the trip count is a tile's
        // share of the batch rather than the widest entry's tile count
        uint64_t col = colw[wave][lane];
        const uint32_t* gw = sg[wave];
        if (total <= (uint32_t)kStage) {
            uint32_t i = toff[lane] + pre[wave][lane];
            while (col) {
                const int j = __ffsll((unsigned long long)col) - 1;
                col &= col - 1ull;
                stage_g[i] = gw[j];
                stage_t[i] = (uint8_t)lane;
                i++;
            }
            __syncthreads();
            for (uint32_t i = t; i < total; i += 256) {
                const int l = stage_t[i];
                point_list[cursor[l] + (i - toff[l])] = stage_g[i];
            }
        } else {
            uint32_t o = cursor[lane] + pre[wave][lane];
            while (col) {
                const int j = __ffsll((unsigned long long)col) - 1;
                col &= col - 1ull;
                point_list[o++] = gw[j];
            }
        }
        __syncthreads();
        if (t < 64) cursor[t] += toff[t + 1] - toff[t];
    }
}

// the MSD depth order's offset parts for k_emit_super (null totals: LSD order, global offsets)
static MsdOffsets msd_offsets(int P, const Layout& L, char* geom, char* image)
{
    MsdOffsets m{nullptr, nullptr, 0, nullptr, 256};
    m.ndig = msd_digits(P);
    if (m.ndig == 0) return m;
    const int tile = kRadixThreads * msd_items(P);
    m.totals = reinterpret_cast<const uint32_t*>(geom + L.bucket_totals);
    m.hist_scan = reinterpret_cast<const uint32_t*>(geom + L.radix_hist_scan);
    m.nblk = (P + tile - 1) / tile;
    m.kxf = reinterpret_cast<const uint32_t*>(image + L.counters) + kCntKeyMin;
    return m;
}

hipError_t launch_binning(int P, int64_t R, const Layout& L, char* geom, char* image, char* binning, uint32_t* stall,
                          hipStream_t s, bool debug, bool emitted, DevCount dc, bool placed)
{
    uint2* ranges = reinterpret_cast<uint2*>(image + L.ranges);
    if (R == 0) return zero_fill(ranges, 8 * (size_t)L.tiles, s);
    const int64_t E = L.super_entries;
    uint32_t* regions = reinterpret_cast<uint32_t*>(binning + L.bin_scan_regions);
    uint32_t* kA = reinterpret_cast<uint32_t*>(binning + L.super_keys);
    uint32_t* vA = reinterpret_cast<uint32_t*>(binning + L.super_vals);
    uint32_t* kB = reinterpret_cast<uint32_t*>(binning + L.alt_keys);
    uint32_t* vB = reinterpret_cast<uint32_t*>(binning + L.alt_vals);
    uint2* sranges = reinterpret_cast<uint2*>(binning + L.super_ranges);
    uint32_t* seg_base = reinterpret_cast<uint32_t*>(binning + L.seg_base);
    uint32_t* colpre = reinterpret_cast<uint32_t*>(binning + L.col_prefix);
    uint32_t* rowpre = reinterpret_cast<uint32_t*>(binning + L.row_prefix);
    uint32_t* table = reinterpret_cast<uint32_t*>(binning + L.seg_table);
    uint32_t* pl = reinterpret_cast<uint32_t*>(binning + L.point_list);
    hipError_t e;
    // the tables the kernels below accumulate into or leave partly unwritten, cleared by
    // k_emit_super or (fused emission) by the super-tile sort's first histogram launch
    const ZeroList zero{{reinterpret_cast<uint32_t*>(ranges), reinterpret_cast<uint32_t*>(sranges), table, regions},
                        {2 * L.tiles, 2 * L.supers, (int)L.seg_table_words,
                         (int)((L.super_passes + 1) * L.scan_region_bin)}};
    const uint32_t* k0 = kA;
    const uint32_t* v0 = vA;
    if (emitted) {  // the depth order's bucket sort wrote the entries
        k0 = reinterpret_cast<const uint32_t*>(geom + L.fused_keys);
        v0 = reinterpret_cast<const uint32_t*>(geom + L.fused_vals);
    } else {
        hipLaunchKernelGGL(k_emit_super, dim3((P + 255) / 256), dim3(256), 0, s, P, L.sgx,
                           reinterpret_cast<const uint32_t*>(geom + L.sorted_ids),
                           reinterpret_cast<const uint32_t*>(geom + L.super_offset),
                           reinterpret_cast<const uint2*>(geom + L.rect_ranked), kA, vA, zero.p[0], zero.n[0],
                           zero.p[1], zero.n[1], zero.p[2], zero.n[2], zero.p[3], zero.n[3],
                           msd_offsets(P, L, geom, image), dc);
        if ((e = post(debug, s)) != hipSuccess) return e;
    }
    int passes = 0;
    uint32_t* bin_hist_scan = reinterpret_cast<uint32_t*>(binning + L.bin_radix_hist_scan);
    int hist_stride = 0, hist_rows = 1 << L.super_bits;  // of the scanned histogram count_fused reads
    if (emitted && placed && L.supers <= 256) {
        // the bucket sort wrote the entries super-tile-major; the super-tile starts are the MSD
        // histogram's scanned super-tile rows (minus its P keys)
        const int nblk = msd_blocks(P);
        const ZeroList zplaced{{reinterpret_cast<uint32_t*>(ranges), regions + L.super_passes * L.scan_region_bin,
                                nullptr, nullptr},
                               {2 * L.tiles, (int)L.scan_region_bin, 0, 0}};
        hipLaunchKernelGGL(k_bin_count_fused, dim3((unsigned)L.seg_blocks), dim3(256), 0, s, L.supers, L.sgx, L.sgy,
                           L.gx, L.gy, nblk, L.supers, E,
                           (const uint32_t*)(reinterpret_cast<uint32_t*>(geom + L.radix_hist_scan) +
                                             (size_t)msd_digits(P) * nblk),
                           sranges, seg_base, colpre, rowpre, k0, table, dc, (uint32_t)P, zplaced,
                           (int64_t)L.seg_table_words);
        if ((e = post(debug, s)) != hipSuccess) return e;
        uint32_t* table_scan = reinterpret_cast<uint32_t*>(binning + L.seg_table_scan);
        if ((e = scan_exclusive(table, table_scan, (int)L.seg_table_words, regions + L.super_passes * L.scan_region_bin,
                                nullptr, stall, s, debug)) != hipSuccess)
            return e;
        hipLaunchKernelGGL(k_bin_emit, dim3((unsigned)L.seg_blocks), dim3(256), 0, s, L.supers, L.sgx, L.gx, L.gy,
                           (const uint32_t*)seg_base, (const uint2*)sranges, (const uint32_t*)colpre,
                           (const uint32_t*)rowpre, k0, v0, (const uint32_t*)table_scan, pl, ranges,
                           reinterpret_cast<uint32_t*>(image + L.counters) + kCntFwdClass,
                           reinterpret_cast<uint32_t*>(image + L.tile_lists), dc);
        return post(debug, s);
    }
    if (emitted && L.super_hist_words > 0) {
        // the bucket sort counted the super-tile pass's [super-tile][block] histogram as it emitted
        // (blocks of kSuperHistBlock entries): no histogram launch; the scatter clears the tables
        // the later kernels need cleared
        bin_hist_scan = reinterpret_cast<uint32_t*>(geom + L.super_hist_scan);
        if ((e = scan_exclusive(reinterpret_cast<const uint32_t*>(geom + L.super_hist), bin_hist_scan,
                                (int)L.super_hist_words, reinterpret_cast<uint32_t*>(geom + L.super_hist_status),
                                nullptr, stall, s, debug)) != hipSuccess)
            return e;
        static const int remap = [] {
            const char* v = getenv("LSR_XCD_REMAP");
            return v && v[0] == '0' ? 0 : 1;
        }();
        const int nblk = (int)((E + kSuperHistBlock - 1) / kSuperHistBlock);
        hipLaunchKernelGGL((k_radix_scatter<4, false>), dim3(nblk), dim3(kRadixThreads), 0, s, k0, v0, (int)E, 0,
                           L.super_bits, (const uint32_t*)bin_hist_scan, nblk, kB, vB, (const uint32_t*)nullptr,
                           ScatterTail{nullptr, nullptr, nullptr}, remap, 0, dc, L.super_hist_stride, L.supers, zero);
        if ((e = post(debug, s)) != hipSuccess) return e;
        passes = 1;
        hist_stride = L.super_hist_stride;
        hist_rows = L.supers;
    } else {
        e = radix_sort(k0, v0, (int)E, L.super_bits, kA, vA, kB, vB, reinterpret_cast<uint32_t*>(binning + L.bin_radix_hist),
                       bin_hist_scan, regions, L.scan_region_bin, stall, s, debug, &passes, nullptr,
                       ScatterTail{nullptr, nullptr, nullptr}, emitted ? zero : ZeroList{}, dc);
        if (e != hipSuccess) return e;
        if (passes == 1) {
            const int tile = kRadixThreads * (radix_small(E) ? 4 : 16);
            hist_stride = (int)((E + tile - 1) / tile);
        }
    }
    const uint32_t* skeys = (passes & 1) ? kB : kA;
    const uint32_t* svals = (passes & 1) ? vB : vA;
    const unsigned grid = (unsigned)L.seg_blocks;
    if (passes == 1 && L.supers <= kFusedSupers) {
        // one pass: the scanned histogram of that pass holds the super-tile ranges (layout
        // [digit][block], hist_stride blocks per digit row, hist_rows rows)
        hipLaunchKernelGGL(k_bin_count_fused, dim3(grid), dim3(256), 0, s, L.supers, L.sgx, L.sgy, L.gx, L.gy,
                           hist_stride, hist_rows, E, (const uint32_t*)bin_hist_scan, sranges, seg_base, colpre, rowpre,
                           skeys, table, dc);
        if ((e = post(debug, s)) != hipSuccess) return e;
    } else {
        hipLaunchKernelGGL(k_super_ranges, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, E, skeys, sranges, dc);
        if ((e = post(debug, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_seg_setup, dim3(1), dim3(kScanThreads), 4 * (size_t)L.sgy, s, L.supers, L.sgx, L.sgy,
                           L.gx, L.gy, (const uint2*)sranges, seg_base, colpre, rowpre, dc);
        if ((e = post(debug, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_bin_count, dim3(grid), dim3(256), 0, s, L.supers, L.sgx, L.gx, L.gy,
                           (const uint32_t*)seg_base, (const uint2*)sranges, (const uint32_t*)colpre,
                           (const uint32_t*)rowpre, skeys, table, dc);
        if ((e = post(debug, s)) != hipSuccess) return e;
    }
    uint32_t* table_scan = reinterpret_cast<uint32_t*>(binning + L.seg_table_scan);
    if ((e = scan_exclusive(table, table_scan, (int)L.seg_table_words, regions + L.super_passes * L.scan_region_bin,
                            nullptr, stall, s, debug)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(k_bin_emit, dim3(grid), dim3(256), 0, s, L.supers, L.sgx, L.gx, L.gy, (const uint32_t*)seg_base,
                       (const uint2*)sranges, (const uint32_t*)colpre, (const uint32_t*)rowpre, skeys, svals,
                       (const uint32_t*)table_scan, pl, ranges,
                       reinterpret_cast<uint32_t*>(image + L.counters) + kCntFwdClass,
                       reinterpret_cast<uint32_t*>(image + L.tile_lists), dc);
    return post(debug, s);
}

}  // namespace lsr
