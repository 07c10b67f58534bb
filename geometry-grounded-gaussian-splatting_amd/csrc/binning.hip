// binning.hip — tile binning on gfx950: prefix sum of tiles touched, key
// emission, stable radix sort, per-tile ranges.
//
// Replaces, in CR/rasterizer_impl.cu: cub::DeviceScan::InclusiveSum (:380),
// duplicateWithKeys (:70-107, 392-400), cub::DeviceRadixSort::SortPairs on
// bits [0, 32 + getHigherMsb(tiles)) (:37-50, 403-412), identifyTileRanges
// (:142-161, 414-421) and checkFrustum (:54-66).
//
// Key = (tile id << 32) | float bits of the view distance; depth > 0.2 so the
// float bits order like the floats.  The sort is stable, so equal keys keep
// emission order = Gaussian index order, as the reference's LSD sort does.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "gsr_kernels.h"

namespace gsr {

size_t scan_temp_bytes(int P) {
    size_t bytes = 0;
    (void)rocprim::inclusive_scan(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)P,
                                  rocprim::plus<uint32_t>());
    return bytes;
}

size_t sort_temp_bytes(int K, int end_bit) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                    (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)K, 0u,
                                    (unsigned)end_bit);
    return bytes;
}

hipError_t launch_scan(const GeomState& gs, int P, hipStream_t stream) {
    if (P == 0) return hipSuccess;
    size_t bytes = gs.scan_tmp_bytes;
    return rocprim::inclusive_scan(gs.scan_tmp, bytes, gs.tiles_touched, gs.offsets, (size_t)P,
                                   rocprim::plus<uint32_t>(), stream);
}

__global__ void __launch_bounds__(256)
    emit_keys_kernel(int P, const Splat* __restrict__ splats, const float* __restrict__ depths,
                     const uint32_t* __restrict__ offsets, const int* __restrict__ radii, uint32_t grid_x,
                     uint32_t grid_y, uint64_t* __restrict__ keys, uint32_t* __restrict__ values) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const int r = radii[idx];
    if (r <= 0) return;
    uint32_t off = idx == 0 ? 0 : offsets[idx - 1];
    const float4 w0 = splats[idx].w0;
    const uint32_t x0 = min(grid_x, (uint32_t)max(0, (int)((w0.x - r) / kTile)));
    const uint32_t y0 = min(grid_y, (uint32_t)max(0, (int)((w0.y - r) / kTile)));
    const uint32_t x1 = min(grid_x, (uint32_t)max(0, (int)((w0.x + r + kTile - 1) / kTile)));
    const uint32_t y1 = min(grid_y, (uint32_t)max(0, (int)((w0.y + r + kTile - 1) / kTile)));
    const uint64_t dbits = (uint64_t)__float_as_uint(depths[idx]);
    for (uint32_t y = y0; y < y1; y++)
        for (uint32_t x = x0; x < x1; x++) {
            keys[off] = ((uint64_t)(y * grid_x + x) << 32) | dbits;
            values[off] = (uint32_t)idx;
            off++;
        }
}

hipError_t launch_emit_keys(const FwdParams& p, const GeomState& gs, const int* radii, const BinningState& bs,
                            hipStream_t stream) {
    if (p.P == 0) return hipSuccess;
    hipLaunchKernelGGL(emit_keys_kernel, dim3((p.P + 255) / 256), dim3(256), 0, stream, p.P, gs.splats, gs.depths,
                       gs.offsets, radii, p.grid_x, p.grid_y, bs.keys_unsorted, bs.values_unsorted);
    return hipGetLastError();
}

hipError_t launch_sort(const BinningState& bs, int K, int end_bit, hipStream_t stream) {
    if (K == 0) return hipSuccess;
    size_t bytes = bs.sort_tmp_bytes;
    return rocprim::radix_sort_pairs(bs.sort_tmp, bytes, bs.keys_unsorted, bs.keys, bs.values_unsorted,
                                     bs.point_list, (size_t)K, 0u, (unsigned)end_bit, stream);
}

__global__ void __launch_bounds__(256)
    tile_ranges_kernel(int K, const uint64_t* __restrict__ keys, uint2* __restrict__ ranges) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= K) return;
    const uint32_t cur = (uint32_t)(keys[idx] >> 32);
    if (idx == 0) {
        ranges[cur].x = 0;
    } else {
        const uint32_t prev = (uint32_t)(keys[idx - 1] >> 32);
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
    hipLaunchKernelGGL(tile_ranges_kernel, dim3((K + 255) / 256), dim3(256), 0, stream, K, bs.keys, ts.ranges);
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
