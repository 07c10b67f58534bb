// sortbin.hip — per-tile Gaussian lists by binning then sorting each tile.
//
// An alternative to tilelists.hip (A/B option GSR_OPT_SORTBIN, off by
// default: slower at C3) replacing duplicateWithKeys +
// cub::DeviceRadixSort::SortPairs + identifyTileRanges
// (CR/rasterizer_impl.cu:70-161, 392-421) for grids of up to
// kMaxSortbinTiles tiles.  The reference sorts
// K 64-bit (tile << 32 | depth bits) keys globally (45 bits, 6 passes over
// 24M pairs at 1080p); its per-tile result is the tile's Gaussians in
// (depth bits, index) order.  Here:
//   count:    each workgroup takes a contiguous range of Gaussians and counts
//             their live tiles (tiles.h: rect + opacity-aware ellipse culling)
//             in an LDS histogram over all tiles -> hist[block][tile];
//   colscan:  per tile, the exclusive prefix of hist over the blocks (in
//             place);
//   tilescan: the tiles' start offsets (exclusive scan of the totals), the
//             ranges, and the longest list (read back with K);
//   emit:     each workgroup writes its (depth bits, Gaussian) pairs into its
//             slots of every tile (LDS slot counters, order within a
//             (block, tile) run unspecified);
//   sort:     one workgroup per tile sorts the tile's pairs in LDS (rocPRIM
//             block radix sort on the 32-bit depth pattern), puts runs of
//             equal depth in Gaussian-index order (the reference's stable
//             tie order) and writes the ids: the point list (tiles longer
//             than one LDS sort: a per-tile LSD sort over global memory).
// No sort of all instances, no global depth sort, no atomics outside LDS.
// Measured at C3 (rocprofv3): count 69 us, colscan 17, tilescan 10, emit 196
// (13M 8-B pairs scattered into 8160 buckets: partial-line writes), sort 161
// (rocPRIM block radix sort, 4 passes) = 0.47 ms, against 0.36 ms for the
// depth sort + the two stable counting passes.
#pragma clang fp contract(off)

#include <rocprim/block/block_radix_sort.hpp>

#include "gsr_kernels.h"
#include "tiles.h"

namespace gsr {

constexpr int kBinThreads = 512;
constexpr int kBinMinChunk = 2048;  // Gaussians per count/emit workgroup (at least)
constexpr int kBinMaxBlocks = 512;

int sortbin_blocks(int P) {
    const int n = (P + kBinMinChunk - 1) / kBinMinChunk;
    return n < 1 ? 1 : (n > kBinMaxBlocks ? kBinMaxBlocks : n);
}
static int sortbin_chunk(int P, int nblk) { return (P + nblk - 1) / nblk; }
bool sortbin_fits(uint32_t gx, uint32_t gy) { return (size_t)gx * gy <= (size_t)kMaxSortbinTiles; }

// Live tiles of Gaussian g (the same test and spans as tilelists.hip / binning.hip).
template <class F>
__device__ __forceinline__ void for_live_tiles(uint32_t g, const Splat* __restrict__ splats,
                                               const int* __restrict__ radii, uint32_t gx, uint32_t gy, float pad,
                                               F&& f) {
    const int r = radii[g];
    if (r <= 0) return;
    const float4 w0 = splats[g].w0, w1 = splats[g].w1;
    const Ellipse E = make_ellipse(w0, w1, pad);
    const TileRect R = tile_rect(w0.x, w0.y, r, gx, gy);
    if (E.mode == 2 || R.x1 <= R.x0 || R.y1 <= R.y0) return;
    for (uint32_t y = R.y0; y < R.y1; y++) {
        uint32_t lo, hi;
        if (!row_span(E, R, y, &lo, &hi)) continue;
        for (uint32_t x = lo; x <= hi; x++) f(y * gx + x);
    }
}

__global__ void __launch_bounds__(kBinThreads)
    sortbin_count_kernel(int P, int chunk, uint32_t gx, uint32_t gy, float pad, const Splat* __restrict__ splats,
                         const int* __restrict__ radii, uint32_t* __restrict__ hist) {
    extern __shared__ uint32_t s_h[];
    const uint32_t T = gx * gy;
    const int tid = threadIdx.x;
    for (uint32_t t = tid; t < T; t += kBinThreads) s_h[t] = 0u;
    __syncthreads();
    const int g0 = blockIdx.x * chunk, g1 = min(P, g0 + chunk);
    for (int g = g0 + tid; g < g1; g += kBinThreads)
        for_live_tiles((uint32_t)g, splats, radii, gx, gy, pad, [&](uint32_t t) { atomicAdd(&s_h[t], 1u); });
    __syncthreads();
    uint32_t* out = hist + (size_t)blockIdx.x * T;
    for (uint32_t t = tid; t < T; t += kBinThreads) out[t] = s_h[t];
}

// Per tile, the exclusive prefix of hist over the blocks, in place.  A
// workgroup takes 64 tiles (one per lane: coalesced rows of hist) and splits
// the blocks into kColParts parts, one wave each.
constexpr int kColParts = 16;
__global__ void __launch_bounds__(64 * kColParts)
    sortbin_colscan_kernel(uint32_t T, int nblk, uint32_t* __restrict__ hist, uint32_t* __restrict__ total) {
    __shared__ uint32_t s_part[kColParts][64];
    const int tl = threadIdx.x & 63, q = threadIdx.x >> 6;
    const uint32_t t = blockIdx.x * 64 + tl;
    const int b0 = (nblk * q) / kColParts, b1 = (nblk * (q + 1)) / kColParts;
    uint32_t s = 0;
    if (t < T)
        for (int b = b0; b < b1; b++) s += hist[(size_t)b * T + t];
    s_part[q][tl] = s;
    __syncthreads();
    uint32_t run = 0;
    for (int k = 0; k < q; k++) run += s_part[k][tl];
    if (t < T) {
        for (int b = b0; b < b1; b++) {
            const uint32_t h = hist[(size_t)b * T + t];
            hist[(size_t)b * T + t] = run;
            run += h;
        }
        if (q == kColParts - 1) total[t] = run;
    }
}

// One workgroup: start[t] = exclusive scan of total, ranges (empty tiles stay
// (0, 0) as in the reference), info[0] = longest list, info[1] = number of
// non-empty tiles up to kSortSmall entries.
constexpr int kScanBlock = 1024;
__global__ void __launch_bounds__(kScanBlock)
    sortbin_tilescan_kernel(uint32_t T, const uint32_t* __restrict__ total, uint32_t* __restrict__ start,
                            uint2* __restrict__ ranges, uint32_t* __restrict__ info) {
    __shared__ uint32_t s_w[kScanBlock / 64];
    __shared__ uint32_t s_carry;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_carry = 0u;
    uint32_t mx = 0, nsmall = 0;
    for (uint32_t base = 0; base < T; base += kScanBlock) {
        const uint32_t t = base + tid;
        const uint32_t v = t < T ? total[t] : 0u;
        mx = max(mx, v);
        nsmall += (v > 0u && v <= (uint32_t)kSortSmall) ? 1u : 0u;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_w[wave] = x;
        __syncthreads();
        uint32_t before = s_carry, all = 0;
#pragma unroll
        for (int w = 0; w < kScanBlock / 64; w++) {
            const uint32_t s = s_w[w];
            before += w < wave ? s : 0u;
            all += s;
        }
        const uint32_t st = before + x - v;
        if (t < T) {
            start[t] = st;
            ranges[t] = v ? make_uint2(st, st + v) : make_uint2(0u, 0u);
        }
        __syncthreads();
        if (tid == 0) s_carry += all;
    }
    __syncthreads();
    mx = wave_max_u(mx);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nsmall += __shfl_xor(nsmall, o, 64);
    __shared__ uint32_t s_mx[kScanBlock / 64], s_ns[kScanBlock / 64];
    if (lane == 0) {
        s_mx[wave] = mx;
        s_ns[wave] = nsmall;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t m = 0, n = 0;
        for (int w = 0; w < kScanBlock / 64; w++) {
            m = max(m, s_mx[w]);
            n += s_ns[w];
        }
        info[0] = m;
        info[1] = n;
        start[T] = s_carry;
    }
}

__global__ void __launch_bounds__(kBinThreads)
    sortbin_emit_kernel(int P, int chunk, uint32_t gx, uint32_t gy, float pad, const Splat* __restrict__ splats,
                        const int* __restrict__ radii, const float* __restrict__ depths,
                        const uint32_t* __restrict__ off, const uint32_t* __restrict__ start,
                        uint2* __restrict__ pairs) {
    extern __shared__ uint32_t s_run[];
    const uint32_t T = gx * gy;
    const int tid = threadIdx.x;
    const uint32_t* my_off = off + (size_t)blockIdx.x * T;
    for (uint32_t t = tid; t < T; t += kBinThreads) s_run[t] = start[t] + my_off[t];
    __syncthreads();
    const int g0 = blockIdx.x * chunk, g1 = min(P, g0 + chunk);
    for (int g = g0 + tid; g < g1; g += kBinThreads) {
        const uint32_t key = __float_as_uint(depths[g]);
        for_live_tiles((uint32_t)g, splats, radii, gx, gy, pad, [&](uint32_t t) {
            pairs[atomicAdd(&s_run[t], 1u)] = make_uint2(key, (uint32_t)g);
        });
    }
}

// One workgroup per tile with lo < length <= BS * IPT.  Depth patterns are
// positive floats (|p_view| >= the near plane), so unsigned order is depth
// order; padding keys 0xffffffff sort behind them.
// The LDS sort of one tile's n <= BS * IPT pairs into point_list[r.x, r.x + n).
template <int BS, int IPT, class Sort>
__device__ __forceinline__ void sort_tile(uint2 r, uint32_t n, const uint2* __restrict__ pairs,
                                          uint32_t* __restrict__ point_list, typename Sort::storage_type& sort_storage,
                                          uint32_t* sk, uint32_t* sv) {
    const int tid = threadIdx.x;
    uint32_t keys[IPT], vals[IPT];
#pragma unroll
    for (int i = 0; i < IPT; i++) {
        const uint32_t j = tid + i * BS;  // striped: coalesced (input order is immaterial)
        const uint2 p = j < n ? pairs[r.x + j] : make_uint2(0xffffffffu, 0xffffffffu);
        keys[i] = p.x;
        vals[i] = p.y;
    }
    Sort().sort_to_striped(keys, vals, sort_storage);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IPT; i++) {
        sk[tid + i * BS] = keys[i];
        sv[tid + i * BS] = vals[i];
    }
    __syncthreads();
    // equal depth patterns: ascending Gaussian index (each run sorted by the
    // thread holding its first element; runs are rare and short)
#pragma unroll
    for (int i = 0; i < IPT; i++) {
        const uint32_t j = tid + i * BS;
        if (j + 1 < n && sk[j + 1] == sk[j] && (j == 0 || sk[j - 1] != sk[j])) {
            uint32_t e = j + 1;
            while (e + 1 < n && sk[e + 1] == sk[j]) e++;
            for (uint32_t a = j + 1; a <= e; a++) {
                const uint32_t v = sv[a];
                uint32_t b = a;
                while (b > j && sv[b - 1] > v) {
                    sv[b] = sv[b - 1];
                    b--;
                }
                sv[b] = v;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < IPT; i++) {
        const uint32_t j = tid + i * BS;
        if (j < n) point_list[r.x + j] = sv[j];
    }
}

template <int BS, int IPT>
__global__ void __launch_bounds__(BS)
    sortbin_sort_kernel(uint32_t T, uint32_t lo, const uint2* __restrict__ ranges, const uint2* __restrict__ pairs,
                        uint32_t* __restrict__ point_list) {
    using Sort = rocprim::block_radix_sort<uint32_t, BS, IPT, uint32_t>;
    constexpr int N = BS * IPT;
    __shared__ union {
        typename Sort::storage_type sort;
        struct {
            uint32_t k[N], v[N];
        } x;
    } s;
    // a fixed grid walks the tiles (the class sizes are not known on the host)
    for (uint32_t tile = blockIdx.x; tile < T; tile += gridDim.x) {
        const uint2 r = ranges[tile];
        const uint32_t n = r.y - r.x;
        if (n <= lo || n > (uint32_t)N) continue;  // uniform over the workgroup
        __syncthreads();  // the previous tile's LDS reads are done
        sort_tile<BS, IPT, Sort>(r, n, pairs, point_list, s.sort, s.x.k, s.x.v);
    }
}

hipError_t launch_sortbin_count(const FwdParams& p, const GeomState& gs, const int* radii, const TileState& ts,
                                hipStream_t stream) {
    const uint32_t gx = p.grid_x, gy = p.grid_y, T = gx * gy;
    const int nblk = sortbin_blocks(p.P), chunk = sortbin_chunk(p.P, nblk);
    const size_t lds = sizeof(uint32_t) * T;
    hipLaunchKernelGGL(sortbin_count_kernel, dim3(nblk), dim3(kBinThreads), lds, stream, p.P, chunk, gx, gy,
                       p.cull_pad, gs.splats, radii, gs.bin_hist);
    hipLaunchKernelGGL(sortbin_colscan_kernel, dim3((T + 63) / 64), dim3(64 * kColParts), 0, stream, T, nblk,
                       gs.bin_hist, gs.bin_total);
    hipLaunchKernelGGL(sortbin_tilescan_kernel, dim3(1), dim3(kScanBlock), 0, stream, T,
                       (const uint32_t*)gs.bin_total, gs.bin_start, ts.ranges, gs.bin_info);
    return hipGetLastError();
}

// Tiles longer than one LDS sort (n > kSortLarge): one 1024-lane workgroup
// per tile runs a stable LSD radix sort over global memory, 4 passes of 8
// bits, ping-ponging Gaussian ids between the point list and the tile's
// (now consumed) pair region; keys are re-read from the depths.  Equal-depth
// runs end in index order as above.  Rare: only grids with > kSortLarge
// live instances in a 16x16 tile take it.
constexpr int kHugeThreads = 1024;
__global__ void __launch_bounds__(kHugeThreads)
    sortbin_huge_kernel(uint32_t T, const uint2* __restrict__ ranges, uint2* __restrict__ pairs,
                        const float* __restrict__ depths, uint32_t* __restrict__ point_list) {
    constexpr int W = kHugeThreads / 64;
    __shared__ uint32_t s_hist[256], s_run[256];
    __shared__ uint32_t s_cnt[W][256];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (uint32_t tile = blockIdx.x; tile < T; tile += gridDim.x) {
        const uint2 r = ranges[tile];
        const uint32_t n = r.y - r.x;
        if (n <= (uint32_t)kSortLarge) continue;  // uniform
        uint32_t* A = point_list + r.x;
        uint32_t* B = reinterpret_cast<uint32_t*>(pairs + r.x);  // first half of the tile's pair region
        auto key_of = [&](int pass, uint32_t i, uint32_t* v) -> uint32_t {
            const uint32_t* src = (pass & 1) ? A : B;
            if (pass == 0) {
                const uint2 pv = pairs[r.x + i];
                *v = pv.y;
                return pv.x;
            }
            *v = src[i];
            return __float_as_uint(depths[*v]);
        };
        for (int pass = 0; pass < 4; pass++) {
            const int shift = 8 * pass;
            uint32_t* dst = (pass & 1) ? B : A;
            __syncthreads();
            if (tid < 256) s_hist[tid] = 0u;
            __syncthreads();
            for (uint32_t i = tid; i < n; i += kHugeThreads) {
                uint32_t v;
                atomicAdd(&s_hist[(key_of(pass, i, &v) >> shift) & 255u], 1u);
            }
            __syncthreads();
            if (tid == 0) {  // exclusive scan of 256 counts
                uint32_t run = 0;
                for (int d = 0; d < 256; d++) {
                    const uint32_t c = s_hist[d];
                    s_run[d] = run;
                    run += c;
                }
            }
            __syncthreads();
            for (uint32_t c0 = 0; c0 < n; c0 += kHugeThreads) {
                const uint32_t i = c0 + tid;
                const bool on = i < n;
                uint32_t v = 0, d = 0;
                if (on) d = (key_of(pass, i, &v) >> shift) & 255u;
                // lanes of the wave with the same digit (match over 8 ballots)
                unsigned long long peers = __ballot(on);
#pragma unroll
                for (int bit = 0; bit < 8; bit++) {
                    const unsigned long long m = __ballot(on && ((d >> bit) & 1u));
                    peers &= ((d >> bit) & 1u) ? m : ~m;
                }
                for (int q = tid; q < W * 256; q += kHugeThreads) (&s_cnt[0][0])[q] = 0u;
                __syncthreads();
                if (on && (peers & lt) == 0ull) s_cnt[wave][d] = (uint32_t)__popcll(peers);
                __syncthreads();
                if (tid < 256) {  // per digit: offsets of the waves, in wave (= element) order
                    uint32_t base = s_run[tid];
                    for (int w = 0; w < W; w++) {
                        const uint32_t c = s_cnt[w][tid];
                        s_cnt[w][tid] = base;
                        base += c;
                    }
                    s_run[tid] = base;
                }
                __syncthreads();
                if (on) dst[s_cnt[wave][d] + (uint32_t)__popcll(peers & lt)] = v;
                __syncthreads();
            }
        }
        __threadfence_block();
        __syncthreads();
        // B holds the ids in depth order; equal-depth runs to index order while copying to A
        for (uint32_t i = tid; i < n; i += kHugeThreads) {
            const uint32_t k = __float_as_uint(depths[B[i]]);
            const bool prev_eq = i > 0 && __float_as_uint(depths[B[i - 1]]) == k;
            const bool next_eq = i + 1 < n && __float_as_uint(depths[B[i + 1]]) == k;
            if (prev_eq) continue;  // copied by its run's first element
            if (!next_eq) {
                A[i] = B[i];
                continue;
            }
            uint32_t e = i + 1;
            while (e + 1 < n && __float_as_uint(depths[B[e + 1]]) == k) e++;
            for (uint32_t a = i; a <= e; a++) {
                const uint32_t v = B[a];
                uint32_t b = a;
                while (b > i && A[b - 1] > v) {
                    A[b] = A[b - 1];
                    b--;
                }
                A[b] = v;
            }
        }
    }
}

// Emission and the per-tile sorts (after the host knows K).  The sort
// kernels take the tile classes themselves: a fixed grid per class walks the
// tiles and skips the others.
hipError_t launch_sortbin_lists(const FwdParams& p, const GeomState& gs, const int* radii, const BinningState& bs,
                                const TileState& ts, hipStream_t stream) {
    const uint32_t gx = p.grid_x, gy = p.grid_y, T = gx * gy;
    const int nblk = sortbin_blocks(p.P), chunk = sortbin_chunk(p.P, nblk);
    const size_t lds = sizeof(uint32_t) * T;
    hipLaunchKernelGGL(sortbin_emit_kernel, dim3(nblk), dim3(kBinThreads), lds, stream, p.P, chunk, gx, gy,
                       p.cull_pad, gs.splats, radii, (const float*)gs.depths, (const uint32_t*)gs.bin_hist,
                       (const uint32_t*)gs.bin_start, bs.pairs);
    hipLaunchKernelGGL((sortbin_sort_kernel<256, kSortSmall / 256>), dim3(T), dim3(256), 0, stream, T, 0u,
                       (const uint2*)ts.ranges, (const uint2*)bs.pairs, bs.point_list);
    const uint32_t big_grid = T < 256u ? T : 256u;
    hipLaunchKernelGGL((sortbin_sort_kernel<1024, kSortLarge / 1024>), dim3(big_grid), dim3(1024), 0, stream, T,
                       (uint32_t)kSortSmall, (const uint2*)ts.ranges, (const uint2*)bs.pairs, bs.point_list);
    hipLaunchKernelGGL(sortbin_huge_kernel, dim3(big_grid), dim3(kHugeThreads), 0, stream, T,
                       (const uint2*)ts.ranges, bs.pairs, (const float*)gs.depths, bs.point_list);
    return hipGetLastError();
}

}  // namespace gsr
