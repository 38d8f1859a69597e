// lsr_binning.hip -- tile binning and ordering.
//
// The reference (upstream) emits one 64-bit key (tile << 32 | depth bits) per tile instance and
// radix-sorts all I instances globally on 32+msb(T) bits.  This file reaches the SAME per-tile
// order ((depth, Gaussian id) ascending inside each tile) with far less integer traffic:
//
//   1. depth sort of the P Gaussians only (32-bit keys, LSD radix, wave64 ballot ranking, stable,
//      so equal depths keep id order) -> sorted_ids, and depth_rank = inverse permutation;
//   2. per-tile instance counts (atomics) and one exclusive scan -> tile_start (= ranges);
//   3. emission of each instance's 32-bit depth RANK into its tile segment (atomic cursor);
//   4. per-tile ordering of the unique ranks inside LDS: bitonic sort for segments <= 8192, an
//      LDS bitmap (rank-window compaction) for larger segments; ranks map back to ids.
//
// Every step is deterministic in its output, so point_list is bit-identical to the oracle's
// (tile, depth, id) sort.
#include "lsr_internal.h"

namespace lsr {

__device__ __forceinline__ uint64_t lanemask_lt()
{
    const uint32_t lane = threadIdx.x & 63;
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Lanes of the wave whose 8-bit digit equals mine (restricted to `valid` lanes).
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid)
{
    uint64_t m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        m &= bit ? bal : ~bal;
    }
    return m;
}

// ---------------------------------------------------------------- depth radix sort (LSD, 8 bit)

__global__ __launch_bounds__(kRadixThreads) void k_radix_hist(const uint32_t* __restrict__ keys, int n,
                                                              int shift, uint32_t* __restrict__ hist,
                                                              int nblk)
{
    __shared__ uint32_t h[256];
    const int t = threadIdx.x;
    h[t] = 0;
    __syncthreads();
    const int base = blockIdx.x * kRadixTile;
    for (int it = 0; it < kRadixItems; it++) {
        const int idx = base + it * kRadixThreads + t;
        const bool valid = idx < n;
        const uint32_t d = valid ? (keys[idx] >> shift) & 255u : 0u;
        const uint64_t peers = match_digit(d, valid);
        if (valid && (peers & lanemask_lt()) == 0) atomicAdd(&h[d], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    hist[t * nblk + blockIdx.x] = h[t];
}

// Exclusive scan of n counters in place by one 1024-thread block (16 consecutive items per
// thread, wave64 shuffle scans); optionally stores the total.
constexpr int kScanItems = 16;
__global__ __launch_bounds__(1024) void k_scan_exclusive(uint32_t* __restrict__ data, int n,
                                                         uint32_t* __restrict__ total_out,
                                                         uint32_t* __restrict__ last_slot)
{
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry_s;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (t == 0) carry_s = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 1024 * kScanItems) {
        uint32_t v[kScanItems];
        uint32_t sum = 0;
        const int i0 = base + t * kScanItems;
#pragma unroll
        for (int k = 0; k < kScanItems; k++) {
            v[k] = (i0 + k < n) ? data[i0 + k] : 0u;
            sum += v[k];
        }
        uint32_t x = sum;  // inclusive wave scan of per-thread sums
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        if (wave == 0) {
            uint32_t s = lane < 16 ? wsum[lane] : 0u;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                const uint32_t y = __shfl_up(s, o, 64);
                if (lane >= o) s += y;
            }
            if (lane < 16) wsum[lane] = s;  // inclusive per-wave prefix
        }
        __syncthreads();
        uint32_t run = carry_s + (wave ? wsum[wave - 1] : 0u) + x - sum;
#pragma unroll
        for (int k = 0; k < kScanItems; k++) {
            if (i0 + k < n) data[i0 + k] = run;
            run += v[k];
        }
        __syncthreads();
        if (t == 0) carry_s += wsum[15];
        __syncthreads();
    }
    if (t == 0) {
        if (total_out) *total_out = carry_s;
        if (last_slot) *last_slot = carry_s;
    }
}

__global__ __launch_bounds__(kRadixThreads) void k_radix_scatter(
    const uint32_t* __restrict__ keys_in, const uint32_t* __restrict__ vals_in, int n, int shift,
    const uint32_t* __restrict__ hist, int nblk, uint32_t* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out)
{
    __shared__ uint32_t base_s[256];
    __shared__ uint32_t wcount[kRadixThreads / 64][256];
    const int t = threadIdx.x, wave = t >> 6;
    base_s[t] = hist[t * nblk + blockIdx.x];
    const int base = blockIdx.x * kRadixTile;
    for (int it = 0; it < kRadixItems; it++) {
#pragma unroll
        for (int w = 0; w < kRadixThreads / 64; w++) wcount[w][t] = 0;
        __syncthreads();
        const int idx = base + it * kRadixThreads + t;
        const bool valid = idx < n;
        const uint32_t key = valid ? keys_in[idx] : 0u;
        const uint32_t val = valid ? (vals_in ? vals_in[idx] : (uint32_t)idx) : 0u;
        const uint32_t d = (key >> shift) & 255u;
        const uint64_t peers = match_digit(d, valid);
        const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
        if (valid && rank == 0) wcount[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t off = base_s[d] + rank;
            for (int w = 0; w < wave; w++) off += wcount[w][d];
            keys_out[off] = key;
            vals_out[off] = val;
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < kRadixThreads / 64; w++) add += wcount[w][t];
        base_s[t] += add;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_depth_rank(const uint32_t* __restrict__ sorted_ids,
                                                    const uint32_t* __restrict__ counters,
                                                    uint32_t* __restrict__ depth_rank)
{
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < counters[kCntVisible]) depth_rank[sorted_ids[r]] = r;
}

static hipError_t post(bool debug, hipStream_t s)
{
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && debug) e = hipStreamSynchronize(s);
    return e;
}

hipError_t launch_depth_sort(int P, const Layout& L, char* geom, uint32_t* counters, hipStream_t s, bool debug)
{
    if (P == 0) return hipSuccess;
    const int nblk = L.radix_blocks;
    uint32_t* hist = reinterpret_cast<uint32_t*>(geom + L.radix_hist);
    uint32_t* ka = reinterpret_cast<uint32_t*>(geom + L.keys_a);
    uint32_t* kb = reinterpret_cast<uint32_t*>(geom + L.keys_b);
    uint32_t* va = reinterpret_cast<uint32_t*>(geom + L.sorted_ids);
    uint32_t* vb = reinterpret_cast<uint32_t*>(geom + L.vals_b);
    const uint32_t* kin = reinterpret_cast<const uint32_t*>(geom + L.depth_key);
    const uint32_t* vin = nullptr;  // pass 0: ids are implicit (identity), i.e. id order
    hipError_t e;
    for (int pass = 0; pass < 4; pass++) {
        uint32_t* kout = (pass & 1) ? ka : kb;
        uint32_t* vout = (pass & 1) ? va : vb;
        const int shift = 8 * pass;
        hipLaunchKernelGGL(k_radix_hist, dim3(nblk), dim3(kRadixThreads), 0, s, kin, P, shift, hist, nblk);
        if ((e = post(debug, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_scan_exclusive, dim3(1), dim3(1024), 0, s, hist, 256 * nblk,
                           (uint32_t*)nullptr, (uint32_t*)nullptr);
        if ((e = post(debug, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_radix_scatter, dim3(nblk), dim3(kRadixThreads), 0, s, kin, vin, P, shift,
                           hist, nblk, kout, vout);
        if ((e = post(debug, s)) != hipSuccess) return e;
        kin = kout;
        vin = vout;
    }
    // after 4 passes the ids are in sorted_ids (va)
    uint32_t* rank = reinterpret_cast<uint32_t*>(geom + L.depth_rank);
    hipLaunchKernelGGL(k_depth_rank, dim3((P + 255) / 256), dim3(256), 0, s, va, counters, rank);
    return post(debug, s);
}

// ---------------------------------------------------------------- tile counts / scan / emit

__global__ __launch_bounds__(256) void k_tile_count(int P, int gx, const uint32_t* __restrict__ tiles,
                                                    const uint32_t* __restrict__ rect,
                                                    uint32_t* __restrict__ count)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P || tiles[i] == 0) return;
    const uint32_t r0 = rect[2 * i], r1 = rect[2 * i + 1];
    const int x0 = r0 & 0xFFFF, y0 = r0 >> 16, x1 = r1 & 0xFFFF, y1 = r1 >> 16;
    for (int y = y0; y < y1; y++)
        for (int x = x0; x < x1; x++) atomicAdd(&count[y * gx + x], 1u);
}

hipError_t launch_tile_count(int P, const Layout& L, char* geom, char* image, hipStream_t s)
{
    uint32_t* count = reinterpret_cast<uint32_t*>(image + L.tile_start);
    hipError_t e = hipMemsetAsync(count, 0, 4 * ((size_t)L.tiles + 1), s);
    if (e != hipSuccess || P == 0) return e;
    hipLaunchKernelGGL(k_tile_count, dim3((P + 255) / 256), dim3(256), 0, s, P, L.gx,
                       reinterpret_cast<const uint32_t*>(geom + L.tiles_touched),
                       reinterpret_cast<const uint32_t*>(geom + L.rect), count);
    return hipGetLastError();
}

hipError_t launch_tile_scan(const Layout& L, char* image, hipStream_t s)
{
    uint32_t* start = reinterpret_cast<uint32_t*>(image + L.tile_start);
    uint32_t* counters = reinterpret_cast<uint32_t*>(image + L.counters);
    hipLaunchKernelGGL(k_scan_exclusive, dim3(1), dim3(1024), 0, s, start, L.tiles,
                       counters + kCntRendered, start + L.tiles);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipMemsetAsync(image + L.tile_cursor, 0, 4 * (size_t)L.tiles, s);
}

__global__ __launch_bounds__(256) void k_emit(int P, int gx, const uint32_t* __restrict__ tiles,
                                              const uint32_t* __restrict__ rect,
                                              const uint32_t* __restrict__ depth_rank,
                                              const uint32_t* __restrict__ tile_start,
                                              uint32_t* __restrict__ cursor,
                                              uint32_t* __restrict__ list_rank)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P || tiles[i] == 0) return;
    const uint32_t rk = depth_rank[i];
    const uint32_t r0 = rect[2 * i], r1 = rect[2 * i + 1];
    const int x0 = r0 & 0xFFFF, y0 = r0 >> 16, x1 = r1 & 0xFFFF, y1 = r1 >> 16;
    for (int y = y0; y < y1; y++)
        for (int x = x0; x < x1; x++) {
            const int t = y * gx + x;
            const uint32_t slot = atomicAdd(&cursor[t], 1u);
            list_rank[tile_start[t] + slot] = rk;
        }
}

hipError_t launch_emit(int P, const Layout& L, char* geom, char* image, char* binning, hipStream_t s)
{
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(k_emit, dim3((P + 255) / 256), dim3(256), 0, s, P, L.gx,
                       reinterpret_cast<const uint32_t*>(geom + L.tiles_touched),
                       reinterpret_cast<const uint32_t*>(geom + L.rect),
                       reinterpret_cast<const uint32_t*>(geom + L.depth_rank),
                       reinterpret_cast<const uint32_t*>(image + L.tile_start),
                       reinterpret_cast<uint32_t*>(image + L.tile_cursor),
                       reinterpret_cast<uint32_t*>(binning + L.list_rank));
    return hipGetLastError();
}

// ---------------------------------------------------------------- per-tile ordering

constexpr int kTileSortThreads = 512;

__global__ __launch_bounds__(kTileSortThreads) void k_tile_sort(const uint32_t* __restrict__ tile_start,
                                                               const uint32_t* __restrict__ list_rank,
                                                               const uint32_t* __restrict__ sorted_ids,
                                                               uint32_t* __restrict__ point_list,
                                                               uint32_t* __restrict__ counters,
                                                               uint32_t* __restrict__ oversize)
{
    __shared__ uint32_t s[kTileSortCap];
    const int tile = blockIdx.x, t = threadIdx.x;
    const uint32_t start = tile_start[tile], n = tile_start[tile + 1] - start;
    if (n == 0) return;
    if (n > (uint32_t)kTileSortCap) {
        if (t == 0) oversize[atomicAdd(&counters[kCntOversize], 1u)] = (uint32_t)tile;
        return;
    }
    if (n == 1) {
        if (t == 0) point_list[start] = sorted_ids[list_rank[start]];
        return;
    }
    uint32_t N = 2;
    while (N < n) N <<= 1;
    for (uint32_t k = t; k < N; k += kTileSortThreads) s[k] = k < n ? list_rank[start + k] : 0xFFFFFFFFu;
    __syncthreads();
    for (uint32_t k = 2; k <= N; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = t; i < N; i += kTileSortThreads) {
                const uint32_t ixj = i ^ j;
                if (ixj > i) {
                    const uint32_t a = s[i], b = s[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        s[i] = b;
                        s[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t k = t; k < n; k += kTileSortThreads) point_list[start + k] = sorted_ids[s[k]];
}

// Segments larger than the LDS sort capacity: ranks are unique integers in [0, visible), so a
// bitmap over a window of ranks, compacted by popcount prefix sums, emits them in order.
__global__ __launch_bounds__(kBigSortThreads) void k_tile_sort_big(const uint32_t* __restrict__ tile_start,
                                                                  const uint32_t* __restrict__ list_rank,
                                                                  const uint32_t* __restrict__ sorted_ids,
                                                                  uint32_t* __restrict__ point_list,
                                                                  const uint32_t* __restrict__ counters,
                                                                  const uint32_t* __restrict__ oversize)
{
    __shared__ uint32_t bm[kBitmapWords];
    __shared__ uint32_t wsum[kBigSortThreads / 64];
    constexpr int kWordsPerThread = kBitmapWords / kBigSortThreads;  // 32
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t n_over = counters[kCntOversize];
    const uint32_t visible = counters[kCntVisible];
    for (uint32_t o = blockIdx.x; o < n_over; o += gridDim.x) {
        const uint32_t tile = oversize[o];
        const uint32_t start = tile_start[tile], n = tile_start[tile + 1] - start;
        uint32_t written = 0;
        for (uint32_t wbase = 0; wbase < visible; wbase += 32u * kBitmapWords) {
            for (int k = t; k < kBitmapWords; k += kBigSortThreads) bm[k] = 0;
            __syncthreads();
            for (uint32_t k = t; k < n; k += kBigSortThreads) {
                const uint32_t r = list_rank[start + k];
                if (r >= wbase && r - wbase < 32u * kBitmapWords) {
                    const uint32_t rel = r - wbase;
                    atomicOr(&bm[rel >> 5], 1u << (rel & 31));
                }
            }
            __syncthreads();
            // per-thread popcount over a contiguous run of words
            uint32_t cnt = 0;
            for (int w = 0; w < kWordsPerThread; w++) cnt += __popc(bm[t * kWordsPerThread + w]);
            uint32_t x = cnt;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d, 64);
                if (lane >= d) x += y;
            }
            if (lane == 63) wsum[wave] = x;
            __syncthreads();
            uint32_t before = 0, total = 0;
            for (int w = 0; w < kBigSortThreads / 64; w++) {
                if (w < wave) before += wsum[w];
                total += wsum[w];
            }
            uint32_t pos = start + written + before + x - cnt;
            for (int w = 0; w < kWordsPerThread; w++) {
                uint32_t bits = bm[t * kWordsPerThread + w];
                while (bits) {
                    const int b = __ffs(bits) - 1;
                    bits &= bits - 1;
                    const uint32_t r = wbase + 32u * (uint32_t)(t * kWordsPerThread + w) + (uint32_t)b;
                    point_list[pos++] = sorted_ids[r];
                }
            }
            written += total;
            __syncthreads();
        }
    }
}

hipError_t launch_tile_sort(const Layout& L, char* geom, char* image, char* binning, hipStream_t s, bool debug)
{
    if (L.tiles == 0) return hipSuccess;
    const uint32_t* start = reinterpret_cast<const uint32_t*>(image + L.tile_start);
    const uint32_t* ranks = reinterpret_cast<const uint32_t*>(binning + L.list_rank);
    const uint32_t* sorted = reinterpret_cast<const uint32_t*>(geom + L.sorted_ids);
    uint32_t* plist = reinterpret_cast<uint32_t*>(binning + L.point_list);
    uint32_t* counters = reinterpret_cast<uint32_t*>(image + L.counters);
    uint32_t* over = reinterpret_cast<uint32_t*>(image + L.oversize);
    hipLaunchKernelGGL(k_tile_sort, dim3(L.tiles), dim3(kTileSortThreads), 0, s, start, ranks, sorted, plist,
                       counters, over);
    hipError_t e = post(debug, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_tile_sort_big, dim3(64), dim3(kBigSortThreads), 0, s, start, ranks, sorted, plist,
                       counters, over);
    return post(debug, s);
}

}  // namespace lsr
