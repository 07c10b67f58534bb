// ncc.hip — the multi-view photometric term of training on gfx950 (SURVEY
// §8(f) rank 3): normalised cross-correlation of a 7x7 half-step patch
// around each reference pixel against its plane-induced homography warp into
// the neighbouring view, with d(NCC)/d(depth, normal) in forward mode.
//
// Replaces WarpPatchNCC / forward_mode_differentiation
// (submodules/warp-patch-ncc/warp_patch_ncc.cu:5-52,
// cuda_warp_patch_ncc/warp_patch_ncc_impl.cu:18-302), called by the
// reference's PatchMatch loss (utils/loss_utils.py:239-256).
//
// One lane per pixel.  The pixels are the valid ones of a view in raster
// order, so the 64 lanes of a wave read a 67 x 4-pixel strip of the
// reference image and a similar warped strip of the neighbour image: the
// 49 x (<= 4 + 4) gathers per pixel are served by L1/L2, and the kernel is
// bound by its per-tap arithmetic (homography, bilinear weights, gradient
// terms).  Divisions by the homogeneous coordinate are one v_rcp_f32 per tap
// (the reference builds with --use_fast_math, warp-patch-ncc/setup.py:18).
#include "gsr_kernels.h"

namespace gsr {

struct NccArgs {
    int P;
    const float* depths;
    const float* normals;
    const int* uvs;
    const float* R;  // [9] device, the reference's column-major float33 (r to n)
    const float* T;  // [3] device
    const float* image_r;
    const float* image_n;
    float fx_r, fy_r, cx_r, cy_r, fx_n, fy_n, cx_n, cy_n;
    int Hr, Wr, Hn, Wn;
    float* ncc;
    float* grad_depths;
    float* grad_normals;
    uint8_t* valid;
};

struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

constexpr int kNccRadius = 3;          // RADIUS of the reference's <3, true> instance
constexpr float kNccHalfExtent = 1.5f;  // RADIUS * 0.5 (half-pixel steps)

__global__ void __launch_bounds__(256) ncc_kernel(NccArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.P) return;
    const int ux = a.uvs[2 * idx], uy = a.uvs[2 * idx + 1];
    const float depth = a.depths[idx];
    const f3 normal = {a.normals[3 * idx], a.normals[3 * idx + 1], a.normals[3 * idx + 2]};
    const f3 pnr = {(ux - a.cx_r) / a.fx_r, (uy - a.cy_r) / a.fy_r, 1.f};
    const float distance = -dot3(pnr, normal) * depth;
    float out_ncc = 0.f, out_gd = 0.f;
    f3 out_gn = {0.f, 0.f, 0.f};
    bool ok = ux - kNccHalfExtent > 0 && ux + kNccHalfExtent < a.Wr - 1 && uy - kNccHalfExtent > 0 &&
              uy + kNccHalfExtent < a.Hr - 1;
    if (ok) {
        // H = K_n (R - T n^T / d) K_r^-1, columns (R is the reference's column-major float33)
        const f3 Tm = {a.T[0], a.T[1], a.T[2]};  // uniform loads
        const float nn[3] = {normal.x, normal.y, normal.z};
        f3 H[3];
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const f3 c = f3{a.R[3 * i], a.R[3 * i + 1], a.R[3 * i + 2]} - Tm * (nn[i] / distance);
            H[i] = {a.fx_n * c.x + a.cx_n * c.z, a.fy_n * c.y + a.cy_n * c.z, c.z};
        }
        H[2] = (H[0] * (-a.cx_r / a.fx_r) + H[1] * (-a.cy_r / a.fy_r)) + H[2];
        H[0] = H[0] * (1.f / a.fx_r);
        H[1] = H[1] * (1.f / a.fy_r);
        const f3 H_uc = (H[0] * (float)ux + H[1] * (float)uy) + H[2];
        const f3 aux = Tm * (1.f / distance);
        float s_r = 0.f, s_n = 0.f, s_r2 = 0.f, s_n2 = 0.f, s_rn = 0.f;
        f3 g_n = {0.f, 0.f, 0.f}, g_n2 = {0.f, 0.f, 0.f}, g_rn = {0.f, 0.f, 0.f};
        const float* Ir = a.image_r;
        const float* In = a.image_n;
        for (int dv = -kNccRadius; dv <= kNccRadius; dv++) {
            const float dv_f = 0.5f * dv;
            const bool odd_v = (dv & 1) != 0;
            const int v0r = uy + (dv >> 1), v1r = v0r + (odd_v ? 1 : 0);  // floor / ceil of dv/2
            const float w_v0 = odd_v ? 0.5f : 1.f, w_v1 = odd_v ? 0.5f : 0.f;
            const f3 H_uc_v = H_uc + H[1] * dv_f;
            const float right_y = (uy + dv_f - a.cy_r) / a.fy_r;
#pragma unroll
            for (int du = -kNccRadius; du <= kNccRadius; du++) {
                const float du_f = 0.5f * du;
                const bool odd_u = (du & 1) != 0;
                const int u0r = ux + (du >> 1), u1r = u0r + (odd_u ? 1 : 0);
                const float w_u0 = odd_u ? 0.5f : 1.f, w_u1 = odd_u ? 0.5f : 0.f;
                // reference image at (u + du/2, v + dv/2): the taps of the reference's line cache
                const float c00 = Ir[v0r * a.Wr + u0r];
                const float c01 = odd_u ? Ir[v0r * a.Wr + u1r] : c00;
                const float c10 = odd_v ? Ir[v1r * a.Wr + u0r] : 0.f;
                const float c11 = (odd_v && odd_u) ? Ir[v1r * a.Wr + u1r] : 0.f;
                const float c_r = (c00 * w_u0 + c01 * w_u1) * w_v0 + (c10 * w_u0 + c11 * w_u1) * w_v1;
                // neighbour image at the warped position
                const f3 H_uv = H_uc_v + H[0] * du_f;
                const float rz = __builtin_amdgcn_rcpf(H_uv.z);
                const float un = H_uv.x * rz, vn = H_uv.y * rz;
                ok = ok && un - kNccHalfExtent > 0 && un + kNccHalfExtent < a.Wn - 1 && vn - kNccHalfExtent > 0 &&
                     vn + kNccHalfExtent < a.Hn - 1;
                const float fu = floorf(un), fv = floorf(vn);
                const int u0 = min(max((int)fu, 0), a.Wn - 1), v0 = min(max((int)fv, 0), a.Hn - 1);
                const int u1 = min(max((int)ceilf(nextafterf(un, INFINITY)), 0), a.Wn - 1);
                const int v1 = min(max((int)ceilf(nextafterf(vn, INFINITY)), 0), a.Hn - 1);
                const float c00n = In[v0 * a.Wn + u0], c01n = In[v0 * a.Wn + u1];
                const float c10n = In[v1 * a.Wn + u0], c11n = In[v1 * a.Wn + u1];
                const float wv0 = v1 - vn, wv1 = vn - v0, wu0 = u1 - un, wu1 = un - u0;
                const float c_n = wv0 * (wu0 * c00n + wu1 * c01n) + wv1 * (wu0 * c10n + wu1 * c11n);
                s_r += c_r;
                s_n += c_n;
                s_r2 += c_r * c_r;
                s_n2 += c_n * c_n;
                s_rn += c_r * c_n;
                // d c_n / d(homography column combination) (warp_patch_ncc_impl.cu:208-224)
                const float dcx = -c00n * wv0 + c01n * wv0 - c10n * wv1 + c11n * wv1;
                const float dcy = -c00n * wu0 - c01n * wu1 + c10n * wu0 + c11n * wu1;
                const f3 dH = {dcx * rz, dcy * rz, (-dcx * un - dcy * vn) * rz};
                const f3 left = {dH.x * a.fx_n, dH.y * a.fy_n, dH.x * a.cx_n + dH.y * a.cy_n + dH.z};
                const f3 right = {(ux + du_f - a.cx_r) / a.fx_r, right_y, 1.f};
                const f3 ga = right * dot3(left, aux);
                g_n = g_n + ga;
                g_n2 = g_n2 + ga * (2.f * c_n);
                g_rn = g_rn + ga * c_r;
            }
        }
        constexpr float kInv = 1.f / 49.f;
        const float cross = s_rn - s_r * s_n * kInv;
        const float var_r = s_r2 - s_r * s_r * kInv;
        const float var_n = s_n2 - s_n * s_n * kInv;
        const float den = var_r * var_n + 1e-8f;
        const float ncc = cross * cross / den;
        const float g_cross = 2.f * cross / den;
        const float g_var_n = -ncc / (var_n + 1e-8f);
        const float g_sum_n = (-g_cross * s_r - g_var_n * 2.f * s_n) * kInv;
        const f3 gaux = (g_n * g_sum_n + g_n2 * g_var_n) + g_rn * g_cross;
        const float gdist = dot3(gaux, normal) / distance;
        out_gn = gaux * -1.f + pnr * (-depth * gdist);
        out_gd = -dot3(pnr, normal) * gdist;
        out_ncc = ncc;
        ok = ok && var_r > 5e-6f && var_n > 5e-6f;
    }
    a.ncc[idx] = ok ? out_ncc : 0.f;
    a.grad_depths[idx] = ok ? out_gd : 0.f;
    a.grad_normals[3 * idx] = ok ? out_gn.x : 0.f;
    a.grad_normals[3 * idx + 1] = ok ? out_gn.y : 0.f;
    a.grad_normals[3 * idx + 2] = ok ? out_gn.z : 0.f;
    a.valid[idx] = ok ? 1 : 0;
}

hipError_t launch_ncc(const NccParams& q, hipStream_t stream) {
    if (q.P <= 0) return hipSuccess;
    NccArgs a;
    a.P = q.P;
    a.depths = q.depths;
    a.normals = q.normals;
    a.uvs = q.uvs;
    a.R = q.R;
    a.T = q.T;
    a.image_r = q.image_r;
    a.image_n = q.image_n;
    a.fx_r = q.fx_r;
    a.fy_r = q.fy_r;
    a.cx_r = q.cx_r;
    a.cy_r = q.cy_r;
    a.fx_n = q.fx_n;
    a.fy_n = q.fy_n;
    a.cx_n = q.cx_n;
    a.cy_n = q.cy_n;
    a.Hr = q.Hr;
    a.Wr = q.Wr;
    a.Hn = q.Hn;
    a.Wn = q.Wn;
    a.ncc = q.ncc;
    a.grad_depths = q.grad_depths;
    a.grad_normals = q.grad_normals;
    a.valid = q.valid;
    hipLaunchKernelGGL(ncc_kernel, dim3((q.P + 255) / 256), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
