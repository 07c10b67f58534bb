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
// 49 x (<= 4 + 4) gathers per pixel are served by L1/L2.  Divisions by the
// homogeneous coordinate are one v_rcp_f32 per tap (the reference builds with
// --use_fast_math, warp-patch-ncc/setup.py:18).
// Round 5 (GSR_NCC_TAPS2): the taps' gathers are issued per group of 3-4 taps
// before their arithmetic (the per-tap version waited on every tap's loads at
// 2 waves per SIMD), the reference's per-tap division for K_r^-1 of the tap is
// hoisted out of the rows, the homography-gradient dot product is folded to
// five operations, the three gradient sums keep their y and z components per
// row, and the margin test is taken on the extremes of the warps: ~60 VALU per
// tap at 4 waves per SIMD (128 VGPRs; ncc.o is compiled without SLP
// vectorisation, which packed the scalar chains at the cost of ~400 moves).
// pm_terms_kernel at the e2e scene: 0.51-0.55 -> 0.21-0.24 ms.
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

#ifndef GSR_NCC_TAPS2
#define GSR_NCC_TAPS2 1  // the folded tap loop (ncc_pixel); 0: the per-tap restatement
#endif
#ifndef GSR_NCC_WAVES
#define GSR_NCC_WAVES 4  // waves per SIMD the NCC kernels are compiled for (<= 128 VGPRs)
#endif
constexpr int kNccRadius = 3;          // RADIUS of the reference's <3, true> instance
constexpr float kNccHalfExtent = 1.5f;  // RADIUS * 0.5 (half-pixel steps)

struct NccPix {
    bool ok;
    float ncc, gd;
    f3 gn;
};

// One reference pixel (ux, uy) with its depth and (unit) normal: the NCC of
// its patch against the warp and d(NCC)/d(depth, normal) (forward mode).
__device__ __forceinline__ NccPix ncc_pixel(const NccArgs& a, int ux, int uy, float depth, f3 normal) {
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
#if GSR_NCC_TAPS2
        if (a.Wn < 3 || a.Hn < 3) {
            ok = false;  // (no warp can lie inside the margin; the taps below assume two columns and rows)
        } else {
            // Per tap: the warp (un, vn) = H (u + du/2, v + dv/2, 1) / z, the bilinear sample c_n of the
            // neighbour image there and its gradient s right, right = K_r^-1 (u + du/2, v + dv/2, 1), with
            // s = left . aux folded to rz (dcx (kx - un kz) + dcy (ky - vn kz)).  The three gradient sums
            // sum_taps w s right (w = 1, 2 c_n, c_r) keep x per tap and y, z per row (right.y is the
            // row's, right.z = 1).  A warp inside the margin has u0 + 1 = ceil(nextafter(un)) (and
            // likewise v), so the four taps are base, base + 1, base + Wn, base + Wn + 1; the margin
            // test is taken once on the extremes of un and vn (their sum catches NaN).
            const float kx = a.fx_n * aux.x + a.cx_n * aux.z, ky = a.fy_n * aux.y + a.cy_n * aux.z, kz = aux.z;
            float rx[2 * kNccRadius + 1];
#pragma unroll
            for (int du = -kNccRadius; du <= kNccRadius; du++) rx[du + kNccRadius] = (ux + 0.5f * du - a.cx_r) / a.fx_r;
            float umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY, fin = 0.f;
            float X1 = 0.f, X2 = 0.f, X3 = 0.f, Y1 = 0.f, Y2 = 0.f, Y3 = 0.f, Z1 = 0.f, Z2 = 0.f, Z3 = 0.f;
            const int Wn = a.Wn, Hn = a.Hn, Wr = a.Wr;
            // taps du0..du1 of row dv: their warps and gathers first, then the arithmetic (one memory
            // round trip per group of taps, not per tap)
            auto taps = [&](int dv, const float* r0, const float* r1, const f3& H_uc_v, float& R1, float& R2,
                            float& R3, auto odd_tag, auto lo_tag, auto hi_tag) {
                constexpr bool odd_v = decltype(odd_tag)::value;
                constexpr int du0 = decltype(lo_tag)::value, du1 = decltype(hi_tag)::value, n = du1 - du0 + 1;
                float t_un[n], t_vn[n], t_rz[n], t_c[n][4], t_cr[n];
#pragma unroll
                for (int k = 0; k < n; k++) {
                    const int du = du0 + k;
                    const bool odd_u = (du & 1) != 0;
                    const int o = du >> 1;
                    // reference image at (u + du/2, v + dv/2) (the reference's line cache, its weights)
                    float c_r = odd_u ? 0.5f * (r0[o] + r0[o + 1]) : r0[o];
                    if constexpr (odd_v) c_r = odd_u ? 0.25f * ((r0[o] + r0[o + 1]) + (r1[o] + r1[o + 1]))
                                                     : 0.5f * (r0[o] + r1[o]);
                    t_cr[k] = c_r;
                    const f3 H_uv = H_uc_v + H[0] * (0.5f * du);
                    const float rz = __builtin_amdgcn_rcpf(H_uv.z);
                    const float un = H_uv.x * rz, vn = H_uv.y * rz;
                    t_un[k] = un;
                    t_vn[k] = vn;
                    t_rz[k] = rz;
                    const int u0 = min(max((int)floorf(un), 0), Wn - 2), v0 = min(max((int)floorf(vn), 0), Hn - 2);
                    const float* q = In + (v0 * Wn + u0);
                    t_c[k][0] = q[0];
                    t_c[k][1] = q[1];
                    t_c[k][2] = q[Wn];
                    t_c[k][3] = q[Wn + 1];
                }
#pragma unroll
                for (int k = 0; k < n; k++) {
                    const float c_r = t_cr[k], rz = t_rz[k], un = t_un[k], vn = t_vn[k];
                    umin = fminf(umin, un);
                    umax = fmaxf(umax, un);
                    vmin = fminf(vmin, vn);
                    vmax = fmaxf(vmax, vn);
                    fin += un + vn;
                    const float fu = floorf(un), fv = floorf(vn);
                    const float c00n = t_c[k][0], c01n = t_c[k][1], c10n = t_c[k][2], c11n = t_c[k][3];
                    const float wv0 = (fv + 1.f) - vn, wv1 = vn - fv, wu0 = (fu + 1.f) - un, wu1 = un - fu;
                    const float c_n = wv0 * (wu0 * c00n + wu1 * c01n) + wv1 * (wu0 * c10n + wu1 * c11n);
                    s_r += c_r;
                    s_n += c_n;
                    s_r2 += c_r * c_r;
                    s_n2 += c_n * c_n;
                    s_rn += c_r * c_n;
                    const float dcx = wv0 * (c01n - c00n) + wv1 * (c11n - c10n);
                    const float dcy = wu0 * (c10n - c00n) + wu1 * (c11n - c01n);
                    const float s = rz * (dcx * (kx - un * kz) + dcy * (ky - vn * kz));
                    const float s2 = s * c_n, s3 = s * c_r;
                    const float x = rx[du0 + k + kNccRadius];
                    R1 += s;
                    R2 += s2;
                    R3 += s3;
                    X1 += x * s;
                    X2 += x * s2;
                    X3 += x * s3;
                }
            };
            auto row = [&](int dv, auto odd_tag) {
                const float dv_f = 0.5f * dv;
                const float* r0 = Ir + (size_t)(uy + (dv >> 1)) * Wr + ux;
                const float* r1 = r0 + Wr;
                const f3 H_uc_v = H_uc + H[1] * dv_f;
                const float right_y = (uy + dv_f - a.cy_r) / a.fy_r;
                float R1 = 0.f, R2 = 0.f, R3 = 0.f;
                taps(dv, r0, r1, H_uc_v, R1, R2, R3, odd_tag, std::integral_constant<int, -kNccRadius>{},
                     std::integral_constant<int, 0>{});
                taps(dv, r0, r1, H_uc_v, R1, R2, R3, odd_tag, std::integral_constant<int, 1>{},
                     std::integral_constant<int, kNccRadius>{});
                Y1 += right_y * R1;
                Y2 += right_y * R2;
                Y3 += right_y * R3;
                Z1 += R1;
                Z2 += R2;
                Z3 += R3;
            };
#pragma unroll 1
            for (int dv = -kNccRadius; dv <= kNccRadius; dv++) {
                if (dv & 1) row(dv, std::true_type{});  // (uniform: a scalar branch)
                else row(dv, std::false_type{});
            }
            ok = umin - kNccHalfExtent > 0 && umax + kNccHalfExtent < Wn - 1 && vmin - kNccHalfExtent > 0 &&
                 vmax + kNccHalfExtent < Hn - 1 && fabsf(fin) < INFINITY;
            g_n = {X1, Y1, Z1};
            g_n2 = f3{X2, Y2, Z2} * 2.f;
            g_rn = {X3, Y3, Z3};
        }
#else
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
#endif
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
    return NccPix{ok, out_ncc, out_gd, out_gn};
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSR_NCC_WAVES, 8))) ncc_kernel(NccArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.P) return;
    const int ux = a.uvs[2 * idx], uy = a.uvs[2 * idx + 1];
    const NccPix r = ncc_pixel(a, ux, uy, a.depths[idx],
                               f3{a.normals[3 * idx], a.normals[3 * idx + 1], a.normals[3 * idx + 2]});
    a.ncc[idx] = r.ok ? r.ncc : 0.f;
    a.grad_depths[idx] = r.ok ? r.gd : 0.f;
    a.grad_normals[3 * idx] = r.ok ? r.gn.x : 0.f;
    a.grad_normals[3 * idx + 1] = r.ok ? r.gn.y : 0.f;
    a.grad_normals[3 * idx + 2] = r.ok ? r.gn.z : 0.f;
    a.valid[idx] = r.ok ? 1 : 0;
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

// ------------------------------------------------------------------ PatchMatch
// The multi-view loss around sample_depth (PatchMatch.__call__,
// utils/loss_utils.py:140-267) as three kernels, for the training step
// (gsr_train.PatchMatchFused): no boolean gather, no host synchronisation
// (the reference's argwhere of the valid pixels), no chain of broadcast
// elementwise ops and their autograd mirror images.
//  * lift: the view's median-depth points in world space (:147-153),
//  * terms: per pixel the reprojection of the point sample_depth returned
//    from the nearest view (:160-170), the geometric mask and weight
//    (:206-221), and at the masked pixels the NCC of the normalised rendered
//    normal's homography warp (ncc_pixel, :239-256 with warp_patch_ncc), with
//    per-block sums of both masked means (:222-226, :258-262);
//  * finish: the two losses from the block sums in a fixed order.
// Their backwards: d(loss)/d(point in the nearest view, median depth,
// rendered normal), the two masked means' gradients through the same chain.
constexpr uint8_t kPmGeo = 1u, kPmNcc = 2u, kPmNccGrad = 4u;  // d_mask, ncc_mask, clamp passes the gradient

struct PmArgs {
    int H, W;
    const float* md;        // [H*W] median depth of the view
    const float* normal;    // [3, H*W] rendered normal (not normalised)
    const float* pin;       // [H*W, 3] sampled points in the nearest camera
    const uint8_t* inside;  // [H*W]
    const float* Mv;        // [3][3] row-major: point in view = tv + pin @ Mv
    const float* tv;        // [3]
    float Fx, Fy, Cx, Cy;   // view intrinsics (the reprojection)
    float noise_th;         // multi-view pixel noise threshold
    NccArgs nc;             // the NCC's poses, images and intrinsics
    float* w;               // [H*W] geometric weight exp(-noise) on d_mask, else 0
    uint8_t* flags;         // [H*W] kPm*
    float* gd;              // [H*W] d(NCC)/d(depth) at ncc_mask pixels
    float* gn;              // [H*W, 3] d(NCC)/d(unit normal)
    float* partial;         // [blocks][4] sums: w * noise, d_mask, ncc * w, ncc_mask
};

struct PmReproj {
    f3 piv;
    float z, dx, dy, noise;
};

// pts_in_view = tv + pin @ Mv, proj = (Cx, Cy) + (Fx, Fy) * xy / max(z, 1e-7),
// noise = |proj - pixel + 1e-6| (torch.pairwise_distance, eps 1e-6)
__device__ __forceinline__ PmReproj pm_reproject(const PmArgs& a, f3 pin, int x, int y) {
#pragma clang fp contract(off)  // (one rounding per torch op of the reference's formulation)
    PmReproj r;
    float v[3];
#pragma unroll
    for (int j = 0; j < 3; j++) v[j] = a.tv[j] + ((pin.x * a.Mv[j] + pin.y * a.Mv[3 + j]) + pin.z * a.Mv[6 + j]);
    r.piv = f3{v[0], v[1], v[2]};
    r.z = fmaxf(v[2], 1e-7f);
    const float px = a.Cx + a.Fx * (v[0] / r.z), py = a.Cy + a.Fy * (v[1] / r.z);
    r.dx = px - (float)x + 1e-6f;
    r.dy = py - (float)y + 1e-6f;
    r.noise = sqrtf(r.dx * r.dx + r.dy * r.dy);
    return r;
}

__device__ __forceinline__ f3 pm_normal(const PmArgs& a, int p, int n, float& len) {
#pragma clang fp contract(off)
    const f3 q = {a.normal[p], a.normal[n + p], a.normal[2 * n + p]};
    len = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z);
    const float m = fmaxf(len, 1e-12f);  // F.normalize (eps 1e-12)
    return f3{q.x / m, q.y / m, q.z / m};
}

// four per-lane sums -> one row of the block's partials (fixed order)
__device__ __forceinline__ void pm_block_sums(float (&v)[4], float* out) {
    __shared__ float s[4][4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = wave_sum_f(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 4; k++) s[wave][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x < 4) out[threadIdx.x] = (s[0][threadIdx.x] + s[1][threadIdx.x]) + (s[2][threadIdx.x] + s[3][threadIdx.x]);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSR_NCC_WAVES, 8))) pm_terms_kernel(PmArgs a) {
    const int n = a.H * a.W;
    const int p = blockIdx.x * 256 + threadIdx.x;
    float sums[4] = {0.f, 0.f, 0.f, 0.f};
    if (p < n) {
        const int y = p / a.W, x = p - y * a.W;
        const f3 pin = {a.pin[3 * p], a.pin[3 * p + 1], a.pin[3 * p + 2]};
        const PmReproj r = pm_reproject(a, pin, x, y);
        const float depth = a.md[p];
        const bool dm = a.inside[p] != 0 && pin.z > 0.2f && r.piv.z > 0.2f && r.noise < a.noise_th && depth > 0.f;
        const float w = dm ? expf(-r.noise) : 0.f;
        uint8_t fl = dm ? kPmGeo : 0u;
        float gd = 0.f;
        f3 gn = {0.f, 0.f, 0.f};
        if (dm) {
            sums[0] = w * r.noise;
            sums[1] = 1.f;
            float len;
            const NccPix c = ncc_pixel(a.nc, x, y, depth, pm_normal(a, p, n, len));
            const float one_m = 1.f - (c.ok ? c.ncc : 0.f);
            const float ncc = fminf(fmaxf(one_m, 0.f), 2.f);  // torch.clamp(1 - cc, 0, 2)
            if (c.ok && ncc < 0.9f) {
                fl |= kPmNcc | ((one_m >= 0.f && one_m <= 2.f) ? kPmNccGrad : 0u);
                sums[2] = ncc * w;
                sums[3] = 1.f;
                gd = c.gd;
                gn = c.gn;
            }
        }
        a.w[p] = w;
        a.flags[p] = fl;
        a.gd[p] = gd;
        a.gn[3 * p] = gn.x;
        a.gn[3 * p + 1] = gn.y;
        a.gn[3 * p + 2] = gn.z;
    }
    pm_block_sums(sums, a.partial + 4 * blockIdx.x);
}

// out = {geo_loss, ncc_loss, d_mask count, ncc_mask count}; an empty mask gives 0 (loss_utils.py:223-224)
__global__ void __launch_bounds__(1024) pm_finish_kernel(const float* __restrict__ partial, int nb,
                                                         float* __restrict__ out) {
    __shared__ float s[16][4];
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int b = threadIdx.x; b < nb; b += 1024) {
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] += partial[4 * b + k];
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = wave_sum_f(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 4; k++) s[wave][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float t[4] = {0.f, 0.f, 0.f, 0.f};
        for (int w = 0; w < 16; w++)
#pragma unroll
            for (int k = 0; k < 4; k++) t[k] += s[w][k];
        out[0] = t[1] > 0.f ? t[0] / t[1] : 0.f;
        out[1] = t[3] > 0.f ? t[2] / t[3] : 0.f;
        out[2] = t[1];
        out[3] = t[3];
    }
}

// dL/d(pin, md, normal) for dL/d(geo_loss, ncc_loss) = g[0], g[1] (device scalars)
__global__ void __launch_bounds__(256) pm_terms_bwd_kernel(PmArgs a, const float* __restrict__ out,
                                                           const float* __restrict__ g, float* __restrict__ dpin,
                                                           float* __restrict__ dmd, float* __restrict__ dnormal) {
    const int n = a.H * a.W;
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const float cg = out[2] > 0.f ? g[0] / out[2] : 0.f;
    const float cn = out[3] > 0.f ? g[1] / out[3] : 0.f;
    const uint8_t fl = a.flags[p];
    f3 gp = {0.f, 0.f, 0.f}, gnrm = {0.f, 0.f, 0.f};
    float gmd = 0.f;
    if (fl & kPmGeo) {
        const int y = p / a.W, x = p - y * a.W;
        const f3 pin = {a.pin[3 * p], a.pin[3 * p + 1], a.pin[3 * p + 2]};
        const PmReproj r = pm_reproject(a, pin, x, y);
        const float gnoise = cg * a.w[p];  // d(masked mean of w * noise)/d noise, w under no_grad
        const float s = r.noise > 0.f ? gnoise / r.noise : 0.f;
        const float gx = s * r.dx * a.Fx, gy = s * r.dy * a.Fy;  // d/d(xy / z) of the projection
        const float iz = 1.f / r.z;
        const float gz = r.piv.z >= 1e-7f ? -(gx * r.piv.x + gy * r.piv.y) * iz * iz : 0.f;
        const float gv[3] = {gx * iz, gy * iz, gz};
        gp.x = (gv[0] * a.Mv[0] + gv[1] * a.Mv[1]) + gv[2] * a.Mv[2];
        gp.y = (gv[0] * a.Mv[3] + gv[1] * a.Mv[4]) + gv[2] * a.Mv[5];
        gp.z = (gv[0] * a.Mv[6] + gv[1] * a.Mv[7]) + gv[2] * a.Mv[8];
        if (fl & kPmNccGrad) {
            const float gcc = -cn * a.w[p];  // ncc = clamp(1 - cc): d/dcc = -1
            gmd = gcc * a.gd[p];
            const f3 gu = f3{a.gn[3 * p], a.gn[3 * p + 1], a.gn[3 * p + 2]} * gcc;
            float len;
            const f3 u = pm_normal(a, p, n, len);
            // F.normalize backward: (g - u (u . g)) / |n| (|n| clamped to eps: g / eps)
            gnrm = len > 1e-12f ? (gu - u * dot3(u, gu)) * (1.f / len) : gu * 1e12f;
        }
    }
    dpin[3 * p] = gp.x;
    dpin[3 * p + 1] = gp.y;
    dpin[3 * p + 2] = gp.z;
    dmd[p] = gmd;
    dnormal[p] = gnrm.x;
    dnormal[n + p] = gnrm.y;
    dnormal[2 * n + p] = gnrm.z;
}

// the median-depth points in world space (loss_utils.py:147-153):
// ((md * ray - T) @ M), ray = ((x - Cx) / Fx, (y - Cy) / Fy, 1); backward: dL/dmd
__global__ void __launch_bounds__(256) pm_lift_kernel(bool backward, int H, int W, float Fx, float Fy, float Cx,
                                                      float Cy, const float* __restrict__ T,
                                                      const float* __restrict__ M, const float* __restrict__ md,
                                                      const float* __restrict__ gpts, float* __restrict__ out) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= H * W) return;
    const int y = p / W, x = p - y * W;
    const float ray[3] = {((float)x - Cx) / Fx, ((float)y - Cy) / Fy, 1.f};
    if (!backward) {
        const float d = md[p];
        const float v[3] = {d * ray[0] - T[0], d * ray[1] - T[1], d * ray[2] - T[2]};
#pragma unroll
        for (int j = 0; j < 3; j++) out[3 * p + j] = (v[0] * M[j] + v[1] * M[3 + j]) + v[2] * M[6 + j];
    } else {
        const float g[3] = {gpts[3 * p], gpts[3 * p + 1], gpts[3 * p + 2]};
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 3; k++) acc += ((g[0] * M[3 * k] + g[1] * M[3 * k + 1]) + g[2] * M[3 * k + 2]) * ray[k];
        out[p] = acc;
    }
}

static NccArgs pm_ncc_args(const PatchMatchParams& q) {
    NccArgs a{};
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
    a.Hr = q.H;
    a.Wr = q.W;
    a.Hn = q.Hn;
    a.Wn = q.Wn;
    return a;
}

static PmArgs pm_args(const PatchMatchParams& q) {
    PmArgs a{};
    a.H = q.H;
    a.W = q.W;
    a.md = q.md;
    a.normal = q.normal;
    a.pin = q.pin;
    a.inside = q.inside;
    a.Mv = q.Mv;
    a.tv = q.tv;
    a.Fx = q.Fx;
    a.Fy = q.Fy;
    a.Cx = q.Cx;
    a.Cy = q.Cy;
    a.noise_th = q.noise_th;
    a.nc = pm_ncc_args(q);
    a.w = q.w;
    a.flags = q.flags;
    a.gd = q.gd;
    a.gn = q.gn;
    return a;
}

size_t patchmatch_partials(int H, int W) { return (size_t)4 * (((size_t)H * W + 255) / 256); }

hipError_t launch_patchmatch_terms(const PatchMatchParams& q, float* partial, float* out, hipStream_t stream) {
    const int n = q.H * q.W;
    const int nb = (n + 255) / 256;
    if (n <= 0) return hipErrorInvalidValue;
    PmArgs a = pm_args(q);
    a.partial = partial;
    hipLaunchKernelGGL(pm_terms_kernel, dim3(nb), dim3(256), 0, stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(pm_finish_kernel, dim3(1), dim3(1024), 0, stream, (const float*)partial, nb, out);
    return hipGetLastError();
}

hipError_t launch_patchmatch_terms_bwd(const PatchMatchParams& q, const float* out, const float* dL_dloss,
                                       float* dL_dpin, float* dL_dmd, float* dL_dnormal, hipStream_t stream) {
    const int n = q.H * q.W;
    if (n <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pm_terms_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, pm_args(q), out, dL_dloss,
                       dL_dpin, dL_dmd, dL_dnormal);
    return hipGetLastError();
}

hipError_t launch_patchmatch_lift(bool backward, int H, int W, float Fx, float Fy, float Cx, float Cy, const float* T,
                                  const float* M, const float* md, const float* gpts, float* out, hipStream_t stream) {
    const int n = H * W;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(pm_lift_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, backward, H, W, Fx, Fy, Cx, Cy, T,
                       M, md, gpts, out);
    return hipGetLastError();
}

}  // namespace gsr
