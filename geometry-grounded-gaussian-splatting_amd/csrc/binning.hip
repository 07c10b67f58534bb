// binning.hip — tile binning on gfx950: depth order, prefix sum of tiles
// touched, per-tile instance emission, stable tile sort, per-tile ranges.
//
// Replaces, in CR/rasterizer_impl.cu: cub::DeviceScan::InclusiveSum (:380),
// duplicateWithKeys (:70-107, 392-400), cub::DeviceRadixSort::SortPairs on
// bits [0, 32 + getHigherMsb(tiles)) (:37-50, 403-412), identifyTileRanges
// (:142-161, 414-421) and checkFrustum (:54-66).
//
// The reference sorts K (tile << 32 | depth bits) keys on 32 + msb(tiles)
// bits — 6 passes over 12-B pairs at 1080p.  The order it produces is
// (tile, depth bits, Gaussian index): the sort is stable and instances are
// emitted in index order.  Here the same order is built as
//   1. a stable sort of the P depth bit patterns (32 bits, P << K), giving
//      Gaussians in (depth bits, index) order;
//   2. emission of the instances in that order (scan of tiles touched taken
//      in depth order);
//   3. a stable sort of the K instances on the tile id alone (msb(tiles)
//      bits, 16-bit keys when the grid has <= 65536 tiles: 2 passes over
//      6-B pairs at 1080p).
// Within a tile the stable tile sort keeps emission order = (depth bits,
// index).
//
// Tile culling: a (Gaussian, tile) instance is emitted only when some pixel
// centre of the tile can reach alpha >= 1/255, i.e. the opacity-aware
// ellipse a dx^2 + 2 b dx dy + c dy^2 <= 2 ln(255 o) meets the tile's pixel
// rectangle (row_span: the exact span of the ellipse per tile row, with a
// margin above every rounding of the per-pixel test).  The dropped
// instances fail the power/alpha test at every pixel of the tile in the
// forward and the backward, so images and gradients are unchanged; the point
// list is the reference's with those instances removed (tested against the
// oracle), and num_rendered stays the reference's K (the rect count).
// No FMA contraction in this file: the live-tile spans are computed twice
// (count, then emission) and must agree bit for bit.
#pragma clang fp contract(off)

#include <algorithm>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "gsr_kernels.h"
#include "tiles.h"

namespace gsr {

struct Uint2Plus {
    __host__ __device__ uint2 operator()(const uint2& a, const uint2& b) const {
        return make_uint2(a.x + b.x, a.y + b.y);
    }
};

size_t scan_temp_bytes(int P) {
    size_t bytes = 0;
    (void)rocprim::inclusive_scan(nullptr, bytes, (const uint2*)nullptr, (uint2*)nullptr, (size_t)P, Uint2Plus());
    return bytes;
}

// rocPRIM picks a merge sort below 1M items for 32-bit keys (10 merge passes
// at P = 1M); a merge-sort limit of 0 keeps the 4-pass onesweep radix sort.
#ifndef GSR_DSORT_BITS
#define GSR_DSORT_BITS 8  // 0: rocPRIM's tuned onesweep config; measured at C3: 8 / 512 x 16 0.127 ms vs tuned 0.147 (11 bits: 0.145-0.173, 7: 0.177)
#endif
// Keys per onesweep block, measured at C3 (depth_order): 1024 x 4 0.104 ms, 512 x 8 0.112, 1024 x 3 0.117,
// 1024 x 8 0.117, 512 x 12 0.120, 512 x 16 0.126, 1024 x 2 0.129, 256 x 12 0.134, 1024 x 6 0.137, 512 x 20 0.142,
// 256 x 8 0.145, 256 x 16 0.148, 512 x 6 0.153.
#ifndef GSR_DSORT_BLOCK
#define GSR_DSORT_BLOCK 1024
#endif
#ifndef GSR_DSORT_ITEMS
#define GSR_DSORT_ITEMS 4
#endif
#if GSR_DSORT_BITS
using DepthOnesweep = rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>,
                                                          rocprim::kernel_config<GSR_DSORT_BLOCK, GSR_DSORT_ITEMS>,
                                                          GSR_DSORT_BITS, rocprim::block_radix_rank_algorithm::match>;
#else
using DepthOnesweep = rocprim::default_config;
#endif
using DepthSortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                   DepthOnesweep, 0>;

size_t depth_sort_temp_bytes(int P) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs<DepthSortConfig>(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                    rocprim::counting_iterator<uint32_t>(0), (uint32_t*)nullptr, (size_t)P, 0u, 32u);
    return std::max(bytes, dsort_temp_bytes(P));  // dsort.hip (default) or rocPRIM (GSR_OPT_ROCPRIM_DSORT)
}

size_t sort_temp_bytes(int K, int tile_bits) {
    size_t bytes = 0;
    if (tile_key_bytes(tile_bits) == 2)
        (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint16_t*)nullptr, (uint16_t*)nullptr,
                                        (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)K, 0u,
                                        (unsigned)tile_bits);
    else
        (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                        (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)K, 0u,
                                        (unsigned)tile_bits);
    return bytes;
}

__device__ __forceinline__ uint32_t live_count(const Ellipse& E, const TileRect& R) {
    uint32_t n = 0, lo, hi;
    for (uint32_t ty = R.y0; ty < R.y1; ty++)
        if (row_span(E, R, ty, &lo, &hi)) n += hi - lo + 1;
    return n;
}

// Live tiles per Gaussian, in index order (coalesced reads).
__global__ void __launch_bounds__(256)
    live_tiles_kernel(int P, const uint32_t* __restrict__ tiles_touched, const Splat* __restrict__ splats,
                      const int* __restrict__ radii, uint32_t gx, uint32_t gy, float pad,
                      uint32_t* __restrict__ tiles_live) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    uint32_t live = 0;
    if (tiles_touched[idx]) {
        const float4 w0 = splats[idx].w0, w1 = splats[idx].w1;
        live = live_count(make_ellipse(w0, w1, pad), tile_rect(w0.x, w0.y, radii[idx], gx, gy));
    }
    tiles_live[idx] = live;
}

__global__ void __launch_bounds__(256)
    gather_counts_kernel(int P, const uint32_t* __restrict__ order, const uint32_t* __restrict__ tiles_touched,
                         const uint32_t* __restrict__ tiles_live, uint2* __restrict__ counts) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const uint32_t idx = order[q];
    counts[q] = make_uint2(tiles_touched[idx], tiles_live[idx]);
}

hipError_t launch_depth_sort(const GeomState& gs, int P, bool prepared, hipStream_t stream) {
    if (P == 0) return hipSuccess;
    if (!option(kOptRocprimDsort)) return launch_dsort(gs, P, prepared, stream);
    size_t bytes = gs.dsort_tmp_bytes;
    return rocprim::radix_sort_pairs<DepthSortConfig>(gs.dsort_tmp, bytes, reinterpret_cast<const uint32_t*>(gs.depths),
                                                      gs.depth_keys_sorted, rocprim::counting_iterator<uint32_t>(0),
                                                      gs.order, (size_t)P, 0u, 32u, stream);
}

// (sort path) live-tile counts in q order, for the emission offsets
hipError_t launch_live_counts(const FwdParams& p, const GeomState& gs, const int* radii, hipStream_t stream) {
    const int P = p.P;
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(live_tiles_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, gs.tiles_touched,
                       gs.splats, radii, p.grid_x, p.grid_y, p.cull_pad, gs.tiles_live);
    hipLaunchKernelGGL(gather_counts_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, gs.order,
                       gs.tiles_touched, gs.tiles_live, gs.counts);
    return hipGetLastError();
}

hipError_t launch_scan(const GeomState& gs, int P, hipStream_t stream) {
    if (P == 0) return hipSuccess;
    size_t bytes = gs.scan_tmp_bytes;
    return rocprim::inclusive_scan(gs.scan_tmp, bytes, gs.counts, gs.offsets, (size_t)P, Uint2Plus(), stream);
}

// Gaussians with more live tiles than this are emitted by the whole wave,
// one tile row per lane.
constexpr uint32_t kCoopLive = 32;

__device__ __forceinline__ float bcast(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint32_t bcast(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
// every field of lane l's ellipse (word by word, so a new field cannot be missed)
__device__ __forceinline__ Ellipse bcast(const Ellipse& E, int l) {
    static_assert(sizeof(Ellipse) % 4 == 0, "Ellipse is broadcast as 32-bit words");
    constexpr int kWords = sizeof(Ellipse) / 4;
    int w[kWords];
    __builtin_memcpy(w, &E, sizeof(Ellipse));
#pragma unroll
    for (int i = 0; i < kWords; i++) w[i] = __builtin_amdgcn_readlane(w[i], l);
    Ellipse B;
    __builtin_memcpy(&B, w, sizeof(Ellipse));
    return B;
}

// One thread per Gaussian in depth order writes its live tiles, row by row
// (the order within one Gaussian is irrelevant: it lands once per tile).
template <typename KeyT>
__global__ void __launch_bounds__(256)
    emit_keys_kernel(int P, const uint32_t* __restrict__ order, const Splat* __restrict__ splats,
                     const uint2* __restrict__ offsets, const int* __restrict__ radii, uint32_t grid_x,
                     uint32_t grid_y, float pad, KeyT* __restrict__ keys, uint32_t* __restrict__ values) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool in = q < P;
    const uint32_t idx = in ? order[q] : 0u;
    const uint2 o1 = in ? offsets[q] : make_uint2(0u, 0u);
    const uint32_t off0 = (!in || q == 0) ? 0u : offsets[q - 1].y;
    const uint32_t n = o1.y - off0;  // live tiles of this Gaussian
    Ellipse E{};
    TileRect R{0, 0, 0, 0};
    if (n) {
        const float4 w0 = splats[idx].w0, w1 = splats[idx].w1;
        E = make_ellipse(w0, w1, pad);
        R = tile_rect(w0.x, w0.y, radii[idx], grid_x, grid_y);
    }
    const bool big = n > kCoopLive;
    if (n && !big) {
        uint32_t off = off0, lo, hi;
        const uint32_t end = off0 + n;  // spans are recomputed bit-identically; never write past the count
        for (uint32_t ty = R.y0; ty < R.y1; ty++) {
            if (!row_span(E, R, ty, &lo, &hi)) continue;
            for (uint32_t tx = lo; tx <= hi && off < end; tx++) {
                keys[off] = (KeyT)(ty * grid_x + tx);
                values[off] = idx;
                off++;
            }
        }
    }
    // large footprints: one Gaussian at a time, a tile row per lane, rows
    // placed by a wave prefix sum of their lengths
    unsigned long long pending = __ballot(big);
    while (pending) {
        const int l = __builtin_ctzll(pending);
        pending &= pending - 1ull;
        const Ellipse B = bcast(E, l);
        TileRect RB;
        RB.x0 = bcast(R.x0, l), RB.x1 = bcast(R.x1, l), RB.y0 = bcast(R.y0, l), RB.y1 = bcast(R.y1, l);
        const uint32_t g = bcast(idx, l);
        uint32_t base = bcast(off0, l);
        const uint32_t end = base + bcast(n, l);
        for (uint32_t ty0 = RB.y0; ty0 < RB.y1; ty0 += 64) {
            const uint32_t ty = ty0 + lane;
            uint32_t lo = 0, hi = 0, len = 0;
            if (ty < RB.y1 && row_span(B, RB, ty, &lo, &hi)) len = hi - lo + 1;
            // exclusive prefix of len over the wave
            uint32_t incl = len;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = __shfl_up(incl, o, 64);
                if (lane >= o) incl += v;
            }
            uint32_t off = base + incl - len;
            for (uint32_t tx = lo; tx < lo + len && off < end; tx++) {
                keys[off] = (KeyT)(ty * grid_x + tx);
                values[off] = g;
                off++;
            }
            base += (uint32_t)__shfl(incl, 63, 64);
        }
    }
}

hipError_t launch_emit_keys(const FwdParams& p, const GeomState& gs, const int* radii, const BinningState& bs,
                            hipStream_t stream) {
    if (p.P == 0) return hipSuccess;
    const dim3 grid((p.P + 255) / 256);
    if (bs.key_bytes == 2)
        hipLaunchKernelGGL(emit_keys_kernel<uint16_t>, grid, dim3(256), 0, stream, p.P, gs.order, gs.splats,
                           gs.offsets, radii, p.grid_x, p.grid_y, p.cull_pad, (uint16_t*)bs.keys_unsorted,
                           bs.values_unsorted);
    else
        hipLaunchKernelGGL(emit_keys_kernel<uint32_t>, grid, dim3(256), 0, stream, p.P, gs.order, gs.splats,
                           gs.offsets, radii, p.grid_x, p.grid_y, p.cull_pad, (uint32_t*)bs.keys_unsorted,
                           bs.values_unsorted);
    return hipGetLastError();
}

hipError_t launch_sort(const BinningState& bs, int K, int tile_bits, hipStream_t stream) {
    if (K == 0) return hipSuccess;
    size_t bytes = bs.sort_tmp_bytes;
    if (bs.key_bytes == 2)
        return rocprim::radix_sort_pairs(bs.sort_tmp, bytes, (const uint16_t*)bs.keys_unsorted, (uint16_t*)bs.keys,
                                         bs.values_unsorted, bs.point_list, (size_t)K, 0u, (unsigned)tile_bits,
                                         stream);
    return rocprim::radix_sort_pairs(bs.sort_tmp, bytes, (const uint32_t*)bs.keys_unsorted, (uint32_t*)bs.keys,
                                     bs.values_unsorted, bs.point_list, (size_t)K, 0u, (unsigned)tile_bits, stream);
}

template <typename KeyT>
__global__ void __launch_bounds__(256)
    tile_ranges_kernel(int K, const KeyT* __restrict__ keys, uint2* __restrict__ ranges) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= K) return;
    const uint32_t cur = keys[idx];
    if (idx == 0) {
        ranges[cur].x = 0;
    } else {
        const uint32_t prev = keys[idx - 1];
        if (cur != prev) {
            ranges[prev].y = idx;
            ranges[cur].x = idx;
        }
    }
    if (idx == K - 1) ranges[cur].y = K;
}

hipError_t launch_tile_ranges(const BinningState& bs, int K, const TileState& ts, int tiles, hipStream_t stream) {
    hipError_t e = hipMemsetAsync(ts.ranges, 0, sizeof(uint2) * (size_t)tiles, stream);
    if (e != hipSuccess || K == 0) return e;
    if (bs.key_bytes == 2)
        hipLaunchKernelGGL(tile_ranges_kernel<uint16_t>, dim3((K + 255) / 256), dim3(256), 0, stream, K,
                           (const uint16_t*)bs.keys, ts.ranges);
    else
        hipLaunchKernelGGL(tile_ranges_kernel<uint32_t>, dim3((K + 255) / 256), dim3(256), 0, stream, K,
                           (const uint32_t*)bs.keys, ts.ranges);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256)
    mark_visible_kernel(int P, const float* __restrict__ means3D, const float* __restrict__ V,
                        uint8_t* __restrict__ present) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const float x = means3D[3 * idx], y = means3D[3 * idx + 1], z = means3D[3 * idx + 2];
    present[idx] = (V[2] * x + V[6] * y + V[10] * z + V[14]) > kNearPlane;
}

// prefiltered = true promises that every Gaussian passes the near-plane test
// (in_frustum, CR/auxiliary.h:144-149, traps otherwise).  flag |= 1 when one
// does not; the host reads it with K and reports the reference's message.
__global__ void __launch_bounds__(256)
    near_violation_kernel(int P, const float* __restrict__ means3D, const float* __restrict__ V,
                          uint32_t* __restrict__ flag) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    bool culled = false;
    if (idx < P) {
        const float x = means3D[3 * idx], y = means3D[3 * idx + 1], z = means3D[3 * idx + 2];
        culled = !((V[2] * x + V[6] * y + V[10] * z + V[14]) > kNearPlane);
    }
    if (__ballot(culled) != 0ull && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

hipError_t launch_near_violation(int P, const float* means3D, const float* view, uint32_t* flag,
                                 hipStream_t stream) {
    hipError_t e = hipMemsetAsync(flag, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess || P == 0) return e;
    hipLaunchKernelGGL(near_violation_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, means3D, view, flag);
    return hipGetLastError();
}

hipError_t launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present,
                               hipStream_t stream) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(mark_visible_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, means3D, view, present);
    return hipGetLastError();
}

}  // namespace gsr
