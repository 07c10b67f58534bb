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
// index): the point list is identical to the reference's, element for element.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "gsr_kernels.h"

namespace gsr {

size_t scan_temp_bytes(int P) {
    size_t bytes = 0;
    (void)rocprim::inclusive_scan(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)P,
                                  rocprim::plus<uint32_t>());
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

__global__ void __launch_bounds__(256)
    gather_counts_kernel(int P, const uint32_t* __restrict__ order, const uint32_t* __restrict__ tiles_touched,
                         uint32_t* __restrict__ counts) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < P) counts[q] = tiles_touched[order[q]];
}

hipError_t launch_depth_order(const GeomState& gs, int P, hipStream_t stream) {
    if (P == 0) return hipSuccess;
    size_t bytes = gs.dsort_tmp_bytes;
    hipError_t e = rocprim::radix_sort_pairs<DepthSortConfig>(gs.dsort_tmp, bytes, reinterpret_cast<const uint32_t*>(gs.depths),
                                             gs.depth_keys_sorted, rocprim::counting_iterator<uint32_t>(0), gs.order,
                                             (size_t)P, 0u, 32u, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gather_counts_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, gs.order,
                       gs.tiles_touched, gs.counts);
    return hipGetLastError();
}

hipError_t launch_scan(const GeomState& gs, int P, hipStream_t stream) {
    if (P == 0) return hipSuccess;
    size_t bytes = gs.scan_tmp_bytes;
    return rocprim::inclusive_scan(gs.scan_tmp, bytes, gs.counts, gs.offsets, (size_t)P,
                                   rocprim::plus<uint32_t>(), stream);
}

// One thread per Gaussian in depth order; writes its rect's tiles row-major
// (the reference's emission order within one Gaussian is irrelevant here:
// a Gaussian lands once in each tile).
template <typename KeyT>
__global__ void __launch_bounds__(256)
    emit_keys_kernel(int P, const uint32_t* __restrict__ order, const Splat* __restrict__ splats,
                     const uint32_t* __restrict__ offsets, const int* __restrict__ radii, uint32_t grid_x,
                     uint32_t grid_y, KeyT* __restrict__ keys, uint32_t* __restrict__ values) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const uint32_t idx = order[q];
    const int r = radii[idx];
    if (r <= 0) return;
    uint32_t off = q == 0 ? 0 : offsets[q - 1];
    const float4 w0 = splats[idx].w0;
    const uint32_t x0 = min(grid_x, (uint32_t)max(0, (int)((w0.x - r) / kTile)));
    const uint32_t y0 = min(grid_y, (uint32_t)max(0, (int)((w0.y - r) / kTile)));
    const uint32_t x1 = min(grid_x, (uint32_t)max(0, (int)((w0.x + r + kTile - 1) / kTile)));
    const uint32_t y1 = min(grid_y, (uint32_t)max(0, (int)((w0.y + r + kTile - 1) / kTile)));
    for (uint32_t y = y0; y < y1; y++)
        for (uint32_t x = x0; x < x1; x++) {
            keys[off] = (KeyT)(y * grid_x + x);
            values[off] = idx;
            off++;
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
