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
// rectangle (tile_live; exact minimum of the quadratic over the rectangle,
// with a margin above every rounding of the per-pixel test).  The dropped
// instances fail the power/alpha test at every pixel of the tile in the
// forward and the backward, so images and gradients are unchanged; the point
// list is the reference's with those instances removed (tested against the
// oracle), and num_rendered stays the reference's K (the rect count).
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "gsr_kernels.h"

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
using DepthSortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                   rocprim::default_config, 0>;

size_t depth_sort_temp_bytes(int P) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs<DepthSortConfig>(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                    rocprim::counting_iterator<uint32_t>(0), (uint32_t*)nullptr, (size_t)P, 0u, 32u);
    return bytes;
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

// Tile rect of Gaussian idx, the getRect of the reference (auxiliary.h:42-49);
// identical to the one preprocess_fwd.hip counted tiles_touched with.
struct TileRect {
    uint32_t x0, y0, x1, y1;
};
__device__ __forceinline__ TileRect tile_rect(float mx, float my, int r, uint32_t gx, uint32_t gy) {
    TileRect t;
    t.x0 = min(gx, (uint32_t)max(0, (int)((mx - r) / kTile)));
    t.y0 = min(gy, (uint32_t)max(0, (int)((my - r) / kTile)));
    t.x1 = min(gx, (uint32_t)max(0, (int)((mx + r + kTile - 1) / kTile)));
    t.y1 = min(gy, (uint32_t)max(0, (int)((my + r + kTile - 1) / kTile)));
    return t;
}

// Per-Gaussian constants of the tile test: Q(d) = a dx^2 + 2 b dx dy + c dy^2
// (power = -Q/2, render_forward.cu:486-487) and the threshold tau: a pixel
// can pass alpha = min(0.99, o e^power) >= 1/255 only if Q <= tau = 2 ln(255 o).
struct LiveTest {
    float mx, my, a, b, c, tau, b_over_a, b_over_c;
    bool none, all;  // no tile can pass / keep every tile (not positive definite, NaN)
};
__device__ __forceinline__ LiveTest live_test(const Splat& sp) {
    LiveTest L;
    L.mx = sp.w0.x;
    L.my = sp.w0.y;
    L.a = sp.w0.z;
    L.b = sp.w0.w;
    L.c = sp.w1.x;
    const float o = sp.w1.y;
    L.none = !(255.f * o >= 1.f) && o == o;  // o < 1/255: o e^power < 1/255 everywhere
    L.tau = 2.f * logf(fmaxf(255.f * o, 1.f));
    L.all = !(L.a > 0.f && L.c > 0.f && L.a * L.c - L.b * L.b > 0.f) || !(L.tau == L.tau);
    L.b_over_a = L.b / L.a;
    L.b_over_c = L.b / L.c;
    return L;
}
// Exact minimum of the positive-definite Q over the tile's pixel-centre
// rectangle (on an edge when the mean lies outside), compared with tau plus
// a margin far above the rounding of the per-pixel power and exp.
__device__ __forceinline__ bool tile_live(const LiveTest& L, uint32_t tx, uint32_t ty) {
    if (L.all) return true;
    if (L.none) return false;
    const float dx_lo = L.mx - (float)(tx * kTile + kTile - 1), dx_hi = L.mx - (float)(tx * kTile);
    const float dy_lo = L.my - (float)(ty * kTile + kTile - 1), dy_hi = L.my - (float)(ty * kTile);
    if (dx_lo <= 0.f && dx_hi >= 0.f && dy_lo <= 0.f && dy_hi >= 0.f) return true;
    auto q = [&](float dx, float dy) { return (L.a * dx + 2.f * L.b * dy) * dx + L.c * dy * dy; };
    const float y0 = fminf(fmaxf(-L.b_over_c * dx_lo, dy_lo), dy_hi);
    const float y1 = fminf(fmaxf(-L.b_over_c * dx_hi, dy_lo), dy_hi);
    const float x0 = fminf(fmaxf(-L.b_over_a * dy_lo, dx_lo), dx_hi);
    const float x1 = fminf(fmaxf(-L.b_over_a * dy_hi, dx_lo), dx_hi);
    const float qmin = fminf(fminf(q(dx_lo, y0), q(dx_hi, y1)), fminf(q(x0, dy_lo), q(x1, dy_hi)));
    const float mxd = fmaxf(fabsf(dx_lo), fabsf(dx_hi)), myd = fmaxf(fabsf(dy_lo), fabsf(dy_hi));
    const float scale = L.a * mxd * mxd + 2.f * fabsf(L.b) * mxd * myd + L.c * myd * myd;
    return qmin <= L.tau * 1.001f + 1e-3f + 1e-4f * scale;
}

// Splats touching more than this many tiles are tested by the whole wave
// (one tile per lane) instead of by their own lane.
constexpr uint32_t kCoopArea = 16;

__device__ __forceinline__ float bcast(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ uint32_t bcast(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }

// Live-tile count of each Gaussian in depth order (and its rect count).
__global__ void __launch_bounds__(256)
    gather_counts_kernel(int P, const uint32_t* __restrict__ order, const uint32_t* __restrict__ tiles_touched,
                         const Splat* __restrict__ splats, const int* __restrict__ radii, uint32_t gx, uint32_t gy,
                         uint2* __restrict__ counts) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool in = q < P;
    const uint32_t idx = in ? order[q] : 0u;
    const uint32_t touched = in ? tiles_touched[idx] : 0u;
    LiveTest L{};
    TileRect R{0, 0, 0, 0};
    if (touched) {
        const Splat sp = splats[idx];
        L = live_test(sp);
        R = tile_rect(sp.w0.x, sp.w0.y, radii[idx], gx, gy);
    }
    uint32_t live = 0;
    const bool big = touched > kCoopArea;
    if (touched && !big) {
        for (uint32_t y = R.y0; y < R.y1; y++)
            for (uint32_t x = R.x0; x < R.x1; x++) live += tile_live(L, x, y);
    }
    // large footprints: the wave takes them one at a time, a tile per lane
    unsigned long long pending = __ballot(big);
    while (pending) {
        const int l = __builtin_ctzll(pending);
        pending &= pending - 1ull;
        LiveTest B;
        B.mx = bcast(L.mx, l), B.my = bcast(L.my, l), B.a = bcast(L.a, l), B.b = bcast(L.b, l);
        B.c = bcast(L.c, l), B.tau = bcast(L.tau, l), B.b_over_a = bcast(L.b_over_a, l);
        B.b_over_c = bcast(L.b_over_c, l);
        B.none = bcast((uint32_t)L.none, l) != 0u, B.all = bcast((uint32_t)L.all, l) != 0u;
        const uint32_t x0 = bcast(R.x0, l), y0 = bcast(R.y0, l), w = bcast(R.x1, l) - x0;
        const uint32_t n = bcast(touched, l);
        uint32_t tot = 0;
        for (uint32_t i0 = 0; i0 < n; i0 += 64) {
            const uint32_t i = i0 + lane;
            tot += (uint32_t)__popcll(__ballot(i < n && tile_live(B, x0 + i % w, y0 + i / w)));
        }
        if (lane == l) live = tot;
    }
    if (in) counts[q] = make_uint2(touched, live);
}

hipError_t launch_depth_order(const FwdParams& p, const GeomState& gs, const int* radii, hipStream_t stream) {
    const int P = p.P;
    if (P == 0) return hipSuccess;
    size_t bytes = gs.dsort_tmp_bytes;
    hipError_t e = rocprim::radix_sort_pairs<DepthSortConfig>(gs.dsort_tmp, bytes, reinterpret_cast<const uint32_t*>(gs.depths),
                                             gs.depth_keys_sorted, rocprim::counting_iterator<uint32_t>(0), gs.order,
                                             (size_t)P, 0u, 32u, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gather_counts_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, gs.order,
                       gs.tiles_touched, gs.splats, radii, p.grid_x, p.grid_y, gs.counts);
    return hipGetLastError();
}

hipError_t launch_scan(const GeomState& gs, int P, hipStream_t stream) {
    if (P == 0) return hipSuccess;
    size_t bytes = gs.scan_tmp_bytes;
    return rocprim::inclusive_scan(gs.scan_tmp, bytes, gs.counts, gs.offsets, (size_t)P, Uint2Plus(), stream);
}

// One thread per Gaussian in depth order; writes its live tiles row-major
// (the reference's emission order within one Gaussian is irrelevant here:
// a Gaussian lands once in each tile).
template <typename KeyT>
__global__ void __launch_bounds__(256)
    emit_keys_kernel(int P, const uint32_t* __restrict__ order, const Splat* __restrict__ splats,
                     const uint2* __restrict__ offsets, const int* __restrict__ radii, uint32_t grid_x,
                     uint32_t grid_y, KeyT* __restrict__ keys, uint32_t* __restrict__ values) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool in = q < P;
    const uint32_t idx = in ? order[q] : 0u;
    const int r = in ? radii[idx] : 0;
    uint32_t off = (!in || q == 0) ? 0u : offsets[q - 1].y;
    LiveTest L{};
    TileRect R{0, 0, 0, 0};
    uint32_t area = 0;
    if (r > 0) {
        const Splat sp = splats[idx];
        L = live_test(sp);
        R = tile_rect(sp.w0.x, sp.w0.y, r, grid_x, grid_y);
        area = (R.x1 - R.x0) * (R.y1 - R.y0);
    }
    const bool big = area > kCoopArea;
    if (area && !big) {
        for (uint32_t y = R.y0; y < R.y1; y++)
            for (uint32_t x = R.x0; x < R.x1; x++) {
                if (!tile_live(L, x, y)) continue;
                keys[off] = (KeyT)(y * grid_x + x);
                values[off] = idx;
                off++;
            }
    }
    // large footprints: the wave emits them one at a time, a tile per lane,
    // live tiles compacted in row-major order by ballot prefix counts
    unsigned long long pending = __ballot(big);
    while (pending) {
        const int l = __builtin_ctzll(pending);
        pending &= pending - 1ull;
        LiveTest B;
        B.mx = bcast(L.mx, l), B.my = bcast(L.my, l), B.a = bcast(L.a, l), B.b = bcast(L.b, l);
        B.c = bcast(L.c, l), B.tau = bcast(L.tau, l), B.b_over_a = bcast(L.b_over_a, l);
        B.b_over_c = bcast(L.b_over_c, l);
        B.none = bcast((uint32_t)L.none, l) != 0u, B.all = bcast((uint32_t)L.all, l) != 0u;
        const uint32_t x0 = bcast(R.x0, l), y0 = bcast(R.y0, l), w = bcast(R.x1, l) - x0;
        const uint32_t n = bcast(area, l), g = bcast(idx, l);
        uint32_t base = bcast(off, l);
        const unsigned long long below = (1ull << lane) - 1ull;
        for (uint32_t i0 = 0; i0 < n; i0 += 64) {
            const uint32_t i = i0 + lane;
            const uint32_t ty = y0 + i / w, tx = x0 + i % w;
            const bool live = i < n && tile_live(B, tx, ty);
            const unsigned long long m = __ballot(live);
            if (live) {
                const uint32_t o = base + (uint32_t)__popcll(m & below);
                keys[o] = (KeyT)(ty * grid_x + tx);
                values[o] = g;
            }
            base += (uint32_t)__popcll(m);
        }
    }
}

hipError_t launch_emit_keys(const FwdParams& p, const GeomState& gs, const int* radii, const BinningState& bs,
                            hipStream_t stream) {
    if (p.P == 0) return hipSuccess;
    const dim3 grid((p.P + 255) / 256);
    if (bs.key_bytes == 2)
        hipLaunchKernelGGL(emit_keys_kernel<uint16_t>, grid, dim3(256), 0, stream, p.P, gs.order, gs.splats,
                           gs.offsets, radii, p.grid_x, p.grid_y, (uint16_t*)bs.keys_unsorted, bs.values_unsorted);
    else
        hipLaunchKernelGGL(emit_keys_kernel<uint32_t>, grid, dim3(256), 0, stream, p.P, gs.order, gs.splats,
                           gs.offsets, radii, p.grid_x, p.grid_y, (uint32_t*)bs.keys_unsorted, bs.values_unsorted);
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

hipError_t launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present,
                               hipStream_t stream) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(mark_visible_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, means3D, view, present);
    return hipGetLastError();
}

}  // namespace gsr
