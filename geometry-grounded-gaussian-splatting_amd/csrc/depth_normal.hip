// depth_normal.hip — the depth-normal consistency input of the training loss
// on gfx950: the normal map of the rendered median
// depth by central differences of the back-projected points, and its
// backward to the depth.
//
// Replaces the torch function depth_to_normal (utils/graphics_utils.py:103-119,
// called at train.py:174): points P(u, v) = depth (x_u, y_v, 1) with
// x_u = (u - Cx) / Fx, y_v = (v - Cy) / Fy; for interior pixels
// n = normalize(dy x dx), dy = P(v+1) - P(v-1), dx = P(u+1) - P(u-1)
// (F.normalize: / max(|c|, 1e-12)); zero on the one-pixel border; valid =
// depth > 0 at the pixel and its four neighbours.  One lane per pixel, the
// four neighbours read through L1 (a wave covers 64 consecutive pixels of a
// row).  The backward is a gather: pixel q collects the terms of the four
// interior pixels whose differences use it, recomputing their normals
// (no scratch, no atomics).
#include "gsr_kernels.h"

namespace gsr {

struct D3 {
    float x, y, z;
};
__device__ __forceinline__ D3 d3sub(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ D3 d3cross(D3 a, D3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float d3dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

struct DnArgs {
    const float* depth;
    int H, W;
    float Fx, Fy, Cx, Cy;
};
__device__ __forceinline__ D3 dn_point(const DnArgs& a, int v, int u) {
    const float d = a.depth[(size_t)v * a.W + u];
    const float x = ((float)u - a.Cx) / a.Fx, y = ((float)v - a.Cy) / a.Fy;
    return {d * x, d * y, d};
}
// cross product c = dy x dx of interior pixel (v, u)
__device__ __forceinline__ void dn_diffs(const DnArgs& a, int v, int u, D3& dy, D3& dx) {
    dy = d3sub(dn_point(a, v + 1, u), dn_point(a, v - 1, u));
    dx = d3sub(dn_point(a, v, u + 1), dn_point(a, v, u - 1));
}

__global__ void __launch_bounds__(256)
    depth_normal_fwd_kernel(DnArgs a, float* __restrict__ normal, uint8_t* __restrict__ valid) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.H * a.W) return;
    const int v = i / a.W, u = i - v * a.W;
    const size_t HW = (size_t)a.H * a.W;
    D3 n = {0.f, 0.f, 0.f};
    bool ok = false;
    if (v >= 1 && v < a.H - 1 && u >= 1 && u < a.W - 1) {
        D3 dy, dx;
        dn_diffs(a, v, u, dy, dx);
        const D3 c = d3cross(dy, dx);
        const float inv = 1.f / fmaxf(sqrtf(d3dot(c, c)), 1e-12f);
        n = {c.x * inv, c.y * inv, c.z * inv};
        const float* D = a.depth;
        ok = D[i] > 0.f && D[i - a.W] > 0.f && D[i + a.W] > 0.f && D[i - 1] > 0.f && D[i + 1] > 0.f;
    }
    normal[i] = n.x;
    normal[HW + i] = n.y;
    normal[2 * HW + i] = n.z;
    valid[i] = ok ? 1 : 0;
}

// dL/d(dy), dL/d(dx) of interior pixel (v, u) for the upstream normal gradient
__device__ __forceinline__ void dn_pixel_grads(const DnArgs& a, const float* g, int v, int u, D3& g_dy, D3& g_dx) {
    const size_t HW = (size_t)a.H * a.W, i = (size_t)v * a.W + u;
    D3 dy, dx;
    dn_diffs(a, v, u, dy, dx);
    const D3 c = d3cross(dy, dx);
    const float len = sqrtf(d3dot(c, c));
    const D3 gn = {g[i], g[HW + i], g[2 * HW + i]};
    D3 gc;
    if (len > 1e-12f) {  // d/dc of c / |c|: (g - n (n . g)) / |c|
        const float inv = 1.f / len;
        const D3 n = {c.x * inv, c.y * inv, c.z * inv};
        const float ng = d3dot(n, gn);
        gc = {(gn.x - n.x * ng) * inv, (gn.y - n.y * ng) * inv, (gn.z - n.z * ng) * inv};
    } else {  // clamp_min(eps) active: c / eps
        gc = {gn.x * 1e12f, gn.y * 1e12f, gn.z * 1e12f};
    }
    g_dy = d3cross(dx, gc);  // d(a x b)/da^T g = b x g
    g_dx = d3cross(gc, dy);  // d(a x b)/db^T g = g x a
}

__global__ void __launch_bounds__(256)
    depth_normal_bwd_kernel(DnArgs a, const float* __restrict__ g, float* __restrict__ dL_ddepth) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.H * a.W) return;
    const int v = i / a.W, u = i - v * a.W;
    auto interior = [&](int vv, int uu) { return vv >= 1 && vv < a.H - 1 && uu >= 1 && uu < a.W - 1; };
    D3 gp = {0.f, 0.f, 0.f}, g_dy, g_dx;
    if (interior(v - 1, u)) {  // this pixel is the +1 row of (v-1, u)
        dn_pixel_grads(a, g, v - 1, u, g_dy, g_dx);
        gp = {gp.x + g_dy.x, gp.y + g_dy.y, gp.z + g_dy.z};
    }
    if (interior(v + 1, u)) {  // the -1 row of (v+1, u)
        dn_pixel_grads(a, g, v + 1, u, g_dy, g_dx);
        gp = {gp.x - g_dy.x, gp.y - g_dy.y, gp.z - g_dy.z};
    }
    if (interior(v, u - 1)) {  // the +1 column of (v, u-1)
        dn_pixel_grads(a, g, v, u - 1, g_dy, g_dx);
        gp = {gp.x + g_dx.x, gp.y + g_dx.y, gp.z + g_dx.z};
    }
    if (interior(v, u + 1)) {  // the -1 column of (v, u+1)
        dn_pixel_grads(a, g, v, u + 1, g_dy, g_dx);
        gp = {gp.x - g_dx.x, gp.y - g_dx.y, gp.z - g_dx.z};
    }
    const float x = ((float)u - a.Cx) / a.Fx, y = ((float)v - a.Cy) / a.Fy;
    dL_ddepth[i] = gp.x * x + gp.y * y + gp.z;
}

hipError_t launch_depth_normal(bool backward, const float* depth, int H, int W, float Fx, float Fy, float Cx, float Cy,
                               const float* g, float* out, uint8_t* valid, hipStream_t stream) {
    if (H <= 0 || W <= 0) return hipSuccess;
    const DnArgs a{depth, H, W, Fx, Fy, Cx, Cy};
    const dim3 grid((unsigned)(((size_t)H * W + 255) / 256));
    if (backward)
        hipLaunchKernelGGL(depth_normal_bwd_kernel, grid, dim3(256), 0, stream, a, g, out);
    else
        hipLaunchKernelGGL(depth_normal_fwd_kernel, grid, dim3(256), 0, stream, a, out, valid);
    return hipGetLastError();
}

}  // namespace gsr
