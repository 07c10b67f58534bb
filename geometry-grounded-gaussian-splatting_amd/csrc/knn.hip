// knn.hip — distCUDA2 on gfx950: per point, the mean squared distance to its
// 3 nearest other points (the initial Gaussian scales of create_from_pcd,
// scene/gaussian_model.py:323).
//
// Replaces SimpleKNN::knn (submodules/simple-knn/simple_knn.cu:175-220) and
// distCUDA2 (spatial.cu:15-25).  Same algorithm shape, so the pruning and the
// result are the reference's: bounds of the points and the origin (cub Reduce
// with init {0, 0, 0}, :190-197), 30-bit Morton codes (:44-70), a stable
// radix sort, boxes of 1024 consecutive sorted points (:76-111), a reject
// distance from the +-3 sorted neighbours, then every box within reject and
// the running 3rd best is scanned (:143-173).  The result is the exact 3-NN
// mean; the sort and the boxes only prune.
//
// MI355X shape: the sorted points are gathered once into a float4 array; a
// 256-lane workgroup owns 256 consecutive sorted points (spatially compact,
// so its lanes want mostly the same boxes).  Per box the workgroup decides
// with one barrier-OR whether any lane needs it; if so the box's 1024 points
// are staged into LDS (16 KB) once and every needing lane scans them with
// broadcast ds_read_b128 — one global read of a box per workgroup instead of
// one per point.
#pragma clang fp contract(off)

#include <float.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "gsr_kernels.h"

namespace gsr {

constexpr int kKnnBox = 1024;  // BOX_SIZE (simple_knn.cu:12)
constexpr int kKnnReduceBlocks = 512;

using KnnSortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                 rocprim::default_config, 0>;

size_t knn_sort_temp_bytes(int P) {
    size_t bytes = 0;
    (void)rocprim::radix_sort_pairs<KnnSortConfig>(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                   rocprim::counting_iterator<uint32_t>(0), (uint32_t*)nullptr,
                                                   (size_t)P, 0u, 30u);
    return bytes;
}

size_t carve_knn(void* base, int P, KnnState& s) {
    Carver c(base);
    s.partials = c.take<float>((size_t)kKnnReduceBlocks * 6);
    s.bounds = c.take<float>(8);
    s.codes = c.take<uint32_t>(P);
    s.codes_sorted = c.take<uint32_t>(P);
    s.order = c.take<uint32_t>(P);
    s.sorted = c.take<float4>(P);
    s.boxes = c.take<float4>(2 * (size_t)((P + kKnnBox - 1) / kKnnBox));
    s.sort_tmp_bytes = knn_sort_temp_bytes(P);
    s.sort_tmp = c.take<char>(s.sort_tmp_bytes);
    return c.off + 256;
}

// min / max of the six bound values over a 256-lane block (fminf/fmaxf are
// exact, so the reduction order does not matter)
__device__ inline void block_minmax6(float (&v)[6], float (*s)[6]) {
#pragma unroll
    for (int k = 0; k < 6; k++) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const float u = __shfl_xor(v[k], o, 64);
            v[k] = k < 3 ? fminf(v[k], u) : fmaxf(v[k], u);
        }
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < 6; k++) s[wave][k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 6; k++) {
        const float a = s[0][k], b = s[1][k], c = s[2][k], d = s[3][k];
        v[k] = k < 3 ? fminf(fminf(a, b), fminf(c, d)) : fmaxf(fmaxf(a, b), fmaxf(c, d));
    }
}

__global__ void __launch_bounds__(256) knn_bounds_kernel(int P, const float* __restrict__ pts,
                                                         float* __restrict__ partials) {
    __shared__ float s[4][6];
    float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = blockIdx.x * 256 + threadIdx.x; i < P; i += gridDim.x * 256) {
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const float x = pts[3 * i + c];
            v[c] = fminf(v[c], x);
            v[3 + c] = fmaxf(v[3 + c], x);
        }
    }
    block_minmax6(v, s);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < 6; k++) partials[6 * blockIdx.x + k] = v[k];
    }
}

// final bounds; the reference's reductions start from init = {0, 0, 0}
__global__ void __launch_bounds__(256) knn_bounds_final_kernel(int nparts, const float* __restrict__ partials,
                                                               float* __restrict__ bounds) {
    __shared__ float s[4][6];
    float v[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int i = threadIdx.x; i < nparts; i += 256) {
#pragma unroll
        for (int k = 0; k < 6; k++) v[k] = k < 3 ? fminf(v[k], partials[6 * i + k]) : fmaxf(v[k], partials[6 * i + k]);
    }
    block_minmax6(v, s);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < 6; k++) bounds[k] = v[k];
    }
}

__device__ inline uint32_t prep_morton(uint32_t x) {
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}

// coord2Morton (simple_knn.cu:54-70), IEEE division as the reference builds it
__global__ void __launch_bounds__(256) knn_morton_kernel(int P, const float* __restrict__ pts,
                                                         const float* __restrict__ bounds,
                                                         uint32_t* __restrict__ codes) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    uint32_t q[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const float mn = bounds[c], mx = bounds[3 + c];
        const float f = ((pts[3 * i + c] - mn) / (mx - mn)) * (float)((1 << 10) - 1);
        q[c] = prep_morton(f == f ? (uint32_t)f : 0u);  // 0/0 (a flat axis) -> 0, as the hardware conversion
    }
    codes[i] = q[0] | (q[1] << 1) | (q[2] << 2);
}

// gather the sorted points into float4 and the bounds of every 1024-point box (boxMinMax, :76-111)
__global__ void __launch_bounds__(256) knn_boxes_kernel(int P, const float* __restrict__ pts,
                                                        const uint32_t* __restrict__ order,
                                                        float4* __restrict__ sorted, float4* __restrict__ boxes) {
    __shared__ float s[4][6];
    float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    const int base = blockIdx.x * kKnnBox;
#pragma unroll
    for (int k = 0; k < kKnnBox / 256; k++) {
        const int i = base + k * 256 + threadIdx.x;
        if (i < P) {
            const uint32_t o = order[i];
            const float x = pts[3 * o], y = pts[3 * o + 1], z = pts[3 * o + 2];
            sorted[i] = make_float4(x, y, z, 0.f);
            v[0] = fminf(v[0], x);
            v[1] = fminf(v[1], y);
            v[2] = fminf(v[2], z);
            v[3] = fmaxf(v[3], x);
            v[4] = fmaxf(v[4], y);
            v[5] = fmaxf(v[5], z);
        }
    }
    block_minmax6(v, s);
    if (threadIdx.x == 0) {
        boxes[2 * blockIdx.x] = make_float4(v[0], v[1], v[2], 0.f);
        boxes[2 * blockIdx.x + 1] = make_float4(v[3], v[4], v[5], 0.f);
    }
}

// squared distance as nvcc contracts point - ref (updateKBest, :127-140)
__device__ __forceinline__ float knn_dist(float4 p, float4 q) {
    const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

// updateKBest<3>: insert into the ascending best three (a no-op unless dist < b2)
__device__ __forceinline__ void knn_update(float dist, float& b0, float& b1, float& b2) {
    if (dist < b2) {
        if (dist < b1) {
            b2 = b1;
            if (dist < b0) {
                b1 = b0;
                b0 = dist;
            } else {
                b1 = dist;
            }
        } else {
            b2 = dist;
        }
    }
}

// distBoxPoint (:113-124)
__device__ __forceinline__ float box_dist(float4 mn, float4 mx, float4 p) {
    float dx = 0.f, dy = 0.f, dz = 0.f;
    if (p.x < mn.x || p.x > mx.x) dx = fminf(fabsf(p.x - mn.x), fabsf(p.x - mx.x));
    if (p.y < mn.y || p.y > mx.y) dy = fminf(fabsf(p.y - mn.y), fabsf(p.y - mx.y));
    if (p.z < mn.z || p.z > mx.z) dz = fminf(fabsf(p.z - mn.z), fabsf(p.z - mx.z));
    return dx * dx + dy * dy + dz * dz;
}

// boxMeanDist (:143-173)
__global__ void __launch_bounds__(256) knn_mean_kernel(int P, const float4* __restrict__ sorted,
                                                       const float4* __restrict__ boxes,
                                                       const uint32_t* __restrict__ order,
                                                       float* __restrict__ mean_dists) {
    __shared__ float4 s_pts[kKnnBox];
    const int idx = blockIdx.x * 256 + threadIdx.x;
    const bool valid = idx < P;
    const float4 p = valid ? sorted[idx] : make_float4(0.f, 0.f, 0.f, 0.f);
    float b0 = FLT_MAX, b1 = FLT_MAX, b2 = FLT_MAX;
    if (valid) {
        for (int i = max(0, idx - 3); i <= min(P - 1, idx + 3); i++)
            if (i != idx) knn_update(knn_dist(p, sorted[i]), b0, b1, b2);
    }
    const float reject = b2;
    b0 = b1 = b2 = FLT_MAX;
    const int nb = (P + kKnnBox - 1) / kKnnBox;
    for (int b = 0; b < nb; b++) {
        const float4 mn = boxes[2 * b], mx = boxes[2 * b + 1];
        const float d = box_dist(mn, mx, p);
        const bool need = valid && !(d > reject || d > b2);
        if (!__syncthreads_or(need)) continue;
        const int first = b * kKnnBox;
        const int n = min(kKnnBox, P - first);
        for (int k = threadIdx.x; k < n; k += 256) s_pts[k] = sorted[first + k];
        __syncthreads();
        if (need) {
            const int self = idx - first;  // skip the point itself (by sorted position)
            for (int j = 0; j < n; j++) {
                const float dist = knn_dist(p, s_pts[j]);
                if (j != self) knn_update(dist, b0, b1, b2);
            }
        }
        // the next staging overwrites s_pts only after the next __syncthreads_or
    }
    if (valid) mean_dists[order[idx]] = (b0 + b1 + b2) / 3.0f;
}

hipError_t launch_knn(int P, const float* pts, const KnnState& s, float* mean_dists, hipStream_t stream) {
    if (P <= 0) return hipSuccess;
    const int nred = min(kKnnReduceBlocks, (P + 255) / 256);
    hipLaunchKernelGGL(knn_bounds_kernel, dim3(nred), dim3(256), 0, stream, P, pts, s.partials);
    hipLaunchKernelGGL(knn_bounds_final_kernel, dim3(1), dim3(256), 0, stream, nred, s.partials, s.bounds);
    hipLaunchKernelGGL(knn_morton_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, pts, s.bounds, s.codes);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t bytes = s.sort_tmp_bytes;
    e = rocprim::radix_sort_pairs<KnnSortConfig>(s.sort_tmp, bytes, s.codes, s.codes_sorted,
                                                 rocprim::counting_iterator<uint32_t>(0), s.order, (size_t)P, 0u,
                                                 30u, stream);
    if (e != hipSuccess) return e;
    const int nb = (P + kKnnBox - 1) / kKnnBox;
    hipLaunchKernelGGL(knn_boxes_kernel, dim3(nb), dim3(256), 0, stream, P, pts, s.order, s.sorted, s.boxes);
    hipLaunchKernelGGL(knn_mean_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, s.sorted, s.boxes, s.order,
                       mean_dists);
    return hipGetLastError();
}

}  // namespace gsr
