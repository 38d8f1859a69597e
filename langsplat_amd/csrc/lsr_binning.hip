// lsr_binning.hip -- tile binning and ordering.
//
// The reference (upstream) emits one 64-bit key (tile << 32 | depth bits) per tile instance and
// radix-sorts all I instances on 32+msb(T) bits.  This file reaches the SAME per-tile order
// ((depth, Gaussian id) ascending inside each tile) with far less integer traffic:
//
//   1. depth sort of the P Gaussians only (32-bit keys, stable LSD radix with wave64 ballot
//      ranking; equal depths keep id order) -> sorted_ids;
//   2. exclusive scan of tiles_touched in that depth order -> each Gaussian's instance offset;
//   3. emission of every (tile, Gaussian) instance in depth order (no atomics);
//   4. stable LSD radix sort of the instances on the TILE bits only (ceil(log2 T) bits:
//      13 at 1080p = 2 passes) -- stability keeps depth order inside each tile;
//   5. tile ranges from the boundaries of the sorted tile keys.
//
// Every step is deterministic, so point_list is bit-identical to the oracle's (tile, depth, id)
// sort.  Scans are single-pass chained scans with decoupled look-back (one launch each).
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
constexpr uint32_t kMaxSpins = 1u << 24;  // a safety bound only; a stalled look-back flags kCntScanFault

__host__ __device__ inline int scan_blocks(int n) { return (n + kScanChunk - 1) / kScanChunk; }

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(kScanThreads) void k_scan(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       int n, uint64_t* __restrict__ status,
                                                       uint32_t* __restrict__ total, uint32_t* __restrict__ fault)
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
                if (__ballot(flag == 0u) & upto) {                             // a predecessor is not ready
                    if (++spins > kMaxSpins) {
                        if (lane == 0) atomicOr(fault, 1u);
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

// out[i] = sum(in[0..i)); if total != null it receives the grand total.  `in` may equal `out`.
// region: scan_region_words(n) zeroed words (status per chunk + ticket).
static hipError_t scan_exclusive(const uint32_t* in, uint32_t* out, int n, uint32_t* region, uint32_t* total,
                                 uint32_t* fault, hipStream_t s, bool debug)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_scan, dim3(scan_blocks(n)), dim3(kScanThreads), 0, s, in, out, n,
                       reinterpret_cast<uint64_t*>(region), total, fault);
    return post(debug, s);
}

// ---------------------------------------------------------------- stable LSD radix sort

// Both radix kernels use a BLOCKED arrangement: wave w of a block owns the contiguous keys
// [w * 64 * kItems, (w + 1) * 64 * kItems) of the block's tile and walks them in rounds of 64
// consecutive keys, counting digits in its own LDS row.  Rounds of one wave are ordered by the
// wave's in-order LDS pipeline, so no block barrier is needed until all rounds are done; the
// stable order (wave, round, lane) is the input order.

// Per-block digit histogram; hist layout [digit][block] so one scan yields the scatter bases.
// kItems keys per thread: 16 for large sorts, 4 for P-sized ones (so that >= ~1000 blocks run).
template <int kItems>
__global__ __launch_bounds__(kRadixThreads) void k_radix_hist(const uint32_t* __restrict__ keys, int n, int shift,
                                                              int nbits, uint32_t* __restrict__ hist, int nblk)
{
    constexpr int kWaves = kRadixThreads / 64;
    __shared__ uint32_t wcnt[kWaves][256];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const uint32_t mask = (1u << nbits) - 1u;
#pragma unroll
    for (int w = 0; w < kWaves; w++) wcnt[w][t] = 0;
    __syncthreads();
    const int base = blockIdx.x * kRadixThreads * kItems + wave * 64 * kItems;
    uint32_t d[kItems];
    bool valid[kItems];
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        const int idx = base + it * 64 + lane;
        valid[it] = idx < n;
        d[it] = valid[it] ? (keys[idx] >> shift) & mask : 0u;
    }
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        const uint64_t peers = match_digit(d[it], valid[it], nbits);
        if (valid[it] && (peers & lanemask_lt()) == 0) wcnt[wave][d[it]] += (uint32_t)__popcll(peers);
    }
    __syncthreads();
    if (t <= (int)mask) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) c += wcnt[w][t];
        hist[t * nblk + blockIdx.x] = c;
    }
}

// Stable scatter of one block's tile.  Ranks: per wave, round by round (ballot match + the wave's
// running digit counts); then per digit the block-local start (scan over digits) and each wave's
// exclusive offset (sum over lower waves).  The tile is reordered by digit in LDS and written
// from LDS in digit-contiguous runs, so global stores coalesce (a direct scatter would send the
// 64 lanes of a store to up to 64 different buckets).
template <int kItems>
__global__ __launch_bounds__(kRadixThreads) void k_radix_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, int n, int shift, int nbits,
    const uint32_t* __restrict__ hist, int nblk, uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out)
{
    constexpr int kTile = kRadixThreads * kItems;
    constexpr int kWaves = kRadixThreads / 64;
    __shared__ uint32_t sk[kTile];
    __shared__ uint32_t sv[kTile];
    __shared__ uint32_t wcnt[kWaves][256];  // running counts, then each wave's offset within the digit
    __shared__ uint32_t gbase[256];         // global output position of this block's first key per digit
    __shared__ uint32_t dstart[256];        // block-local start of each digit in the reordered tile
    __shared__ uint32_t wsum[kWaves];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const uint32_t mask = (1u << nbits) - 1u;
#pragma unroll
    for (int w = 0; w < kWaves; w++) wcnt[w][t] = 0;
    gbase[t] = t <= (int)mask ? hist[t * nblk + blockIdx.x] : 0u;
    const int tile0 = blockIdx.x * kTile;
    const int base = tile0 + wave * 64 * kItems;
    uint32_t key[kItems], val[kItems], rank[kItems];
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        const int idx = base + it * 64 + lane;
        const bool valid = idx < n;
        key[it] = valid ? keys_in[idx] : 0u;
        val[it] = valid ? (vals_in ? vals_in[idx] : (uint32_t)idx) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        const bool valid = base + it * 64 + lane < n;
        const uint32_t d = (key[it] >> shift) & mask;
        const uint64_t peers = match_digit(d, valid, nbits);
        const uint32_t r = (uint32_t)__popcll(peers & lanemask_lt());
        const uint32_t c = wcnt[wave][d];
        rank[it] = c + r;
        if (valid && r == 0) wcnt[wave][d] = c + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // per digit: waves' exclusive offsets and the block-local digit start
    {
        uint32_t tot = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) {
            const uint32_t c = wcnt[w][t];
            wcnt[w][t] = tot;
            tot += c;
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
        dstart[t] = before + x - tot;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kItems; it++) {
        if (base + it * 64 + lane < n) {
            const uint32_t d = (key[it] >> shift) & mask;
            const uint32_t pos = dstart[d] + wcnt[wave][d] + rank[it];
            sk[pos] = key[it];
            sv[pos] = val[it];
        }
    }
    __syncthreads();
    const int cnt = min(kTile, n - tile0);
    for (int i = t; i < cnt; i += kRadixThreads) {
        const uint32_t k = sk[i];
        const uint32_t d = (k >> shift) & mask;
        const uint32_t o = gbase[d] + (uint32_t)i - dstart[d];
        keys_out[o] = k;
        vals_out[o] = sv[i];
    }
}

// Sorts (keys, vals) by key bits [0, total_bits) in passes of <= 8 bits.  The input is read
// from (k0, v0) (v0 == null: values are the input indices) and the result lands in
// (kA, vA) after an even number of passes, or in (kB, vB) after an odd number; returns which.
static hipError_t radix_sort(const uint32_t* k0, const uint32_t* v0, int n, int total_bits, uint32_t* kA,
                             uint32_t* vA, uint32_t* kB, uint32_t* vB, uint32_t* hist, uint32_t* scan_regions,
                             size_t region_words, uint32_t* fault, hipStream_t s, bool debug, int* passes_out)
{
    const bool small = n <= (1 << 21);
    const int tile = kRadixThreads * (small ? 4 : 16);
    const int nblk = (n + tile - 1) / tile;
    const int passes = (total_bits + 7) / 8;
    *passes_out = passes;
    const uint32_t* kin = k0;
    const uint32_t* vin = v0;
    hipError_t e;
    for (int pass = 0; pass < passes; pass++) {
        const int shift = 8 * pass;
        const int nbits = (total_bits - shift) < 8 ? (total_bits - shift) : 8;
        uint32_t* kout = (pass & 1) ? kA : kB;
        uint32_t* vout = (pass & 1) ? vA : vB;
        if (small)
            hipLaunchKernelGGL(k_radix_hist<4>, dim3(nblk), dim3(kRadixThreads), 0, s, kin, n, shift, nbits, hist, nblk);
        else
            hipLaunchKernelGGL(k_radix_hist<16>, dim3(nblk), dim3(kRadixThreads), 0, s, kin, n, shift, nbits, hist, nblk);
        if ((e = post(debug, s)) != hipSuccess) return e;
        if ((e = scan_exclusive(hist, hist, (1 << nbits) * nblk, scan_regions + pass * region_words, nullptr, fault,
                                s, debug)) != hipSuccess)
            return e;
        if (small)
            hipLaunchKernelGGL(k_radix_scatter<4>, dim3(nblk), dim3(kRadixThreads), 0, s, kin, vin, n, shift, nbits,
                               hist, nblk, kout, vout);
        else
            hipLaunchKernelGGL(k_radix_scatter<16>, dim3(nblk), dim3(kRadixThreads), 0, s, kin, vin, n, shift, nbits,
                               hist, nblk, kout, vout);
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

// ---------------------------------------------------------------- depth order + instance offsets

__global__ __launch_bounds__(256) void k_gather_tiles(int P, const uint32_t* __restrict__ sorted_ids,
                                                      const uint32_t* __restrict__ tiles,
                                                      uint32_t* __restrict__ tiles_ranked)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < P) tiles_ranked[r] = tiles[sorted_ids[r]];
}

hipError_t launch_depth_order(int P, const Layout& L, char* geom, uint32_t* counters, hipStream_t s, bool debug)
{
    if (P == 0) return hipSuccess;
    uint32_t* hist = reinterpret_cast<uint32_t*>(geom + L.radix_hist);
    uint32_t* regions = reinterpret_cast<uint32_t*>(geom + L.scan_regions);
    uint32_t* fault = counters + kCntScanFault;
    uint32_t* ka = reinterpret_cast<uint32_t*>(geom + L.keys_a);
    uint32_t* kb = reinterpret_cast<uint32_t*>(geom + L.keys_b);
    uint32_t* va = reinterpret_cast<uint32_t*>(geom + L.sorted_ids);
    uint32_t* vb = reinterpret_cast<uint32_t*>(geom + L.vals_b);
    int passes = 0;
    hipError_t e = radix_sort(reinterpret_cast<const uint32_t*>(geom + L.depth_key), nullptr, P, 32, ka, va, kb, vb,
                              hist, regions, L.scan_region_geom, fault, s, debug, &passes);
    if (e != hipSuccess) return e;
    // 4 passes: the ids are in sorted_ids (va)
    uint32_t* off = reinterpret_cast<uint32_t*>(geom + L.inst_offset);
    hipLaunchKernelGGL(k_gather_tiles, dim3((P + 255) / 256), dim3(256), 0, s, P, va,
                       reinterpret_cast<const uint32_t*>(geom + L.tiles_touched), off);
    if ((e = post(debug, s)) != hipSuccess) return e;
    return scan_exclusive(off, off, P, regions + passes * L.scan_region_geom, counters + kCntRendered, fault, s,
                          debug);
}

// ---------------------------------------------------------------- emit + tile sort + ranges

__global__ __launch_bounds__(256) void k_emit(int P, int gx, const uint32_t* __restrict__ sorted_ids,
                                              const uint32_t* __restrict__ inst_offset,
                                              const uint32_t* __restrict__ tiles, const uint32_t* __restrict__ rect,
                                              uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                              uint32_t* __restrict__ zero_a, int zero_a_words,
                                              uint32_t* __restrict__ zero_b, int zero_b_words)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    // clear the tile ranges and the tile-sort scan status (replaces two memset launches)
    for (int w = r; w < zero_a_words; w += gridDim.x * blockDim.x) zero_a[w] = 0u;
    for (int w = r; w < zero_b_words; w += gridDim.x * blockDim.x) zero_b[w] = 0u;
    if (r >= P) return;
    const uint32_t g = sorted_ids[r];
    if (tiles[g] == 0) return;
    uint32_t o = inst_offset[r];
    const uint32_t r0 = rect[2 * g], r1 = rect[2 * g + 1];
    const int x0 = r0 & 0xFFFF, y0 = r0 >> 16, x1 = r1 & 0xFFFF, y1 = r1 >> 16;
    for (int y = y0; y < y1; y++)
        for (int x = x0; x < x1; x++) {
            keys[o] = (uint32_t)(y * gx + x);
            vals[o] = g;
            o++;
        }
}

__global__ __launch_bounds__(256) void k_ranges(int64_t R, const uint32_t* __restrict__ keys, uint2* __restrict__ ranges)
{
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= R) return;
    const uint32_t t = keys[k];
    if (k == 0 || keys[k - 1] != t) ranges[t].x = (uint32_t)k;
    if (k == R - 1 || keys[k + 1] != t) ranges[t].y = (uint32_t)(k + 1);
}

hipError_t launch_binning(int P, int64_t R, const Layout& L, char* geom, char* image, char* binning, hipStream_t s,
                          bool debug)
{
    uint2* ranges = reinterpret_cast<uint2*>(image + L.ranges);
    if (R == 0) return hipMemsetAsync(ranges, 0, 8 * (size_t)L.tiles, s);
    const int tile_bits = L.tile_bits;
    const int passes = L.tile_passes;
    uint32_t* regions = reinterpret_cast<uint32_t*>(binning + L.bin_scan_regions);
    uint32_t* fault = reinterpret_cast<uint32_t*>(image + L.counters) + kCntScanFault;
    hipError_t e;
    uint32_t* pl_keys = reinterpret_cast<uint32_t*>(binning + L.list_keys);
    uint32_t* pl = reinterpret_cast<uint32_t*>(binning + L.point_list);
    uint32_t* alt_keys = reinterpret_cast<uint32_t*>(binning + L.alt_keys);
    uint32_t* alt_vals = reinterpret_cast<uint32_t*>(binning + L.alt_vals);
    // emit so that the sorted result lands in (list_keys, point_list): odd pass counts start in the
    // (list) buffers and end in alt... radix_sort writes pass 0 to B, so start in A for even passes
    uint32_t *ek, *ev, *kA, *vA, *kB, *vB;
    if (passes % 2 == 0) {
        ek = pl_keys; ev = pl;            // A -> B -> A
        kA = pl_keys; vA = pl; kB = alt_keys; vB = alt_vals;
    } else {
        ek = alt_keys; ev = alt_vals;     // A' -> B' with B' = list buffers
        kA = alt_keys; vA = alt_vals; kB = pl_keys; vB = pl;
    }
    hipLaunchKernelGGL(k_emit, dim3((P + 255) / 256), dim3(256), 0, s, P, L.gx,
                       reinterpret_cast<const uint32_t*>(geom + L.sorted_ids),
                       reinterpret_cast<const uint32_t*>(geom + L.inst_offset),
                       reinterpret_cast<const uint32_t*>(geom + L.tiles_touched),
                       reinterpret_cast<const uint32_t*>(geom + L.rect), ek, ev,
                       reinterpret_cast<uint32_t*>(ranges), 2 * L.tiles, regions,
                       (int)(passes * L.scan_region_bin));
    if ((e = post(debug, s)) != hipSuccess) return e;
    int done = 0;
    e = radix_sort(ek, ev, (int)R, tile_bits, kA, vA, kB, vB, reinterpret_cast<uint32_t*>(binning + L.bin_radix_hist),
                   regions, L.scan_region_bin, fault, s, debug, &done);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_ranges, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, s, R, pl_keys, ranges);
    return post(debug, s);
}

}  // namespace lsr
