// preprocess_fwd.hip — per-Gaussian forward preprocess on gfx950.
//
// Replaces FORWARD::preprocess / preprocessCUDA (render_forward.cu:283-386,
// 710-774) together with computeCov2D (:81-243) and computeColorFromSHSG
// (:22-78).  One lane per Gaussian; every output a later kernel gathers is
// packed into one 64-B Splat record (gsr_common.h) so the render kernels
// fetch a Gaussian with four 16-B loads.
//
// Outputs per Gaussian: radii (int32, the extension output), tiles_touched,
// depth (= |p_view|, the sort key, render_forward.cu:380), clamped bits, and
// the Splat record (only for Gaussians with radius > 0; the others are never
// gathered).
// Bit-exact integer outputs (radii, tiles_touched, K, sort keys) need the
// same fp32 operation sequence as the oracle: no FMA contraction in this
// translation unit (set before the includes so the inlined helpers of
// gsr_math.h are covered too).
#pragma clang fp contract(off)

#include "gsr_kernels.h"
#include "gsr_math.h"

namespace gsr {

struct PreprocessArgs {
    int P, D, SHM, SGD, SGM, W, H;
    const float* means3D;
    const float* colors_precomp;
    const float* opacities;
    const float* scales;
    const float* rotations;
    const float* cov3D_precomp;
    const float* shs;
    const float* shs_rest;  // split rows (FwdParams::shs_rest) or null
    const float* sg_axis;
    const float* sg_sharpness;
    const float* sg_color;
    float scale_modifier;
    const float* view;
    const float* proj;
    const float* campos;
    float tan_fovx, tan_fovy, focal_x, focal_y, kernel_size;
    uint32_t grid_x, grid_y;
    int* radii;
    uint8_t* clamped;
    float* ddir;  // 9 planes of P: d(SH colour)/d(direction) for the backward (D > 0)
    float* depths;
    Splat* splats;
    uint32_t* tiles_touched;
    uint4* foot;  // [P][2] tile footprint for the rows pass (GeomState::foot); its rect is empty when culled
    bool no_color;
    uint32_t* zero_first;  // words zeroed for the next kernels (dsort state; dsort_zero_region)
    size_t zero_words;
    uint32_t* zero_K;      // K accumulator of count_k_hist_kernel
};

// ndc2Pix in double, as the reference (auxiliary.h:38-40)
__device__ inline float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

// The rows pass of the tile lists (tilelists.hip) gathers, per Gaussian in
// depth order, exactly the footprint written here: the splat's centre,
// conic and opacity coefficient (bit for bit the Splat record's) and the
// tile rect packed as x0 | y0 << 16, x1 | y1 << 16 — one 32-B piece instead
// of the splat's first half plus the radius (two sectors and two dependent
// round trips).  A culled Gaussian gets an empty rect.
__device__ __forceinline__ void cull_foot(const PreprocessArgs& a, int idx) {
    a.foot[2 * (size_t)idx + 1] = make_uint4(0u, 0u, 0u, 0u);
}

// HOIST (the SH 3 + SG 7 colour model, BASELINE C5): the colour rows (192-B
// SH row, 196-B SG lobe rows) are requested at the top with the geometry
// inputs, before the culling branches (one memory round trip instead of
// three); the plain instance loads them where they are used.
template <bool HOIST, bool SPLIT = false>
#ifndef GSR_PRE_WAVES
#define GSR_PRE_WAVES 1
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSR_PRE_WAVES, 8))) preprocess_fwd_kernel(PreprocessArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    for (size_t i = (size_t)idx; i < a.zero_words; i += (size_t)gridDim.x * blockDim.x) a.zero_first[i] = 0u;
    if (idx == 0) *a.zero_K = 0u;
    if (idx >= a.P) return;
    a.radii[idx] = 0;
    a.tiles_touched[idx] = 0;

    const float px = a.means3D[3 * idx], py = a.means3D[3 * idx + 1], pz = a.means3D[3 * idx + 2];
    float sh[48], ax[21], sc[21], sh7[7];
    float opacity = 0.f, sc_in[3] = {0.f, 0.f, 0.f}, q_in[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (HOIST) {
        opacity = a.opacities[idx];
        sc_in[0] = a.scales[3 * idx];
        sc_in[1] = a.scales[3 * idx + 1];
        sc_in[2] = a.scales[3 * idx + 2];
        const float4 q4 = *reinterpret_cast<const float4*>(a.rotations + 4 * idx);
        q_in[0] = q4.x;
        q_in[1] = q4.y;
        q_in[2] = q4.z;
        q_in[3] = q4.w;
        load_sh(a.shs + (size_t)idx * a.SHM * 3, a.SHM, sh_count(a.D), sh);
        const size_t o0 = (size_t)idx * 7;
#pragma unroll
        for (int k = 0; k < 21; k++) ax[k] = a.sg_axis[3 * o0 + k];
#pragma unroll
        for (int k = 0; k < 21; k++) sc[k] = a.sg_color[3 * o0 + k];
#pragma unroll
        for (int k = 0; k < 7; k++) sh7[k] = a.sg_sharpness[o0 + k];
    }
    const float* V = a.view;
    const ViewGeom g = view_geom(V, px, py, pz, a.tan_fovx, a.tan_fovy);
    if (g.t[2] <= kNearPlane) {  // in_frustum (auxiliary.h:133-153)
        cull_foot(a, idx);
        return;
    }

    const float* Pm = a.proj;
    const float hx = Pm[0] * px + Pm[4] * py + Pm[8] * pz + Pm[12];
    const float hy = Pm[1] * px + Pm[5] * py + Pm[9] * pz + Pm[13];
    const float hw = Pm[3] * px + Pm[7] * py + Pm[11] * pz + Pm[15];
    const float p_w = 1.0f / (hw + 0.0000001f);

    const float fx = a.focal_x, fy = a.focal_y;
    const float tz = g.tz, itz = 1.0f / tz;
    float A[9], Rq[9], s[3];
    float cinv[9];  // cov_cam_inv (row-major, symmetric)
    float cov00, cov01, cov11;
    bool well_conditioned = true;
    // T = W J in the reference's glm product order: Tc[j][i] is column j,
    // row i.  Only columns 0 and 1 are non-zero (J's third column is 0).
    // Evaluated with contraction off (file-level pragma) so the 2D covariance,
    // and with it det == 0, the radius and the tile rect, are bit-identical to
    // the oracle's glm-order restatement: radii / tiles_touched / K / the
    // sorted instance list are integer outputs and must match exactly.
    const float j00 = fx / tz, j02 = -(fx * g.tx) / (tz * tz);
    const float j11 = fy / tz, j12 = -(fy * g.ty) / (tz * tz);
    float Tc0[3], Tc1[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        // W column c = (V[c], V[4+c], V[8+c]) -> W.c[c][i] = V[4*i + c]
        Tc0[i] = V[4 * i] * j00 + V[4 * i + 2] * j02;
        Tc1[i] = V[4 * i + 1] * j11 + V[4 * i + 2] * j12;
    }
    if (a.scales) {
        if constexpr (!HOIST) {
            const float* q = a.rotations + 4 * idx;
            q_in[0] = q[0];
            q_in[1] = q[1];
            q_in[2] = q[2];
            q_in[3] = q[3];
            sc_in[0] = a.scales[3 * idx];
            sc_in[1] = a.scales[3 * idx + 1];
            sc_in[2] = a.scales[3 * idx + 2];
        }
        rot_view(V, q_in[0], q_in[1], q_in[2], q_in[3], A, Rq);
        s[0] = a.scale_modifier * sc_in[0];
        s[1] = a.scale_modifier * sc_in[1];
        s[2] = a.scale_modifier * sc_in[2];
        // glm R column j = row j of R_q: R.c[j][i] = Rq[3*j + i]; (S R).c[j][i] = s_i * R.c[j][i]
        // M = (S R) T: M.c[j][i] = SR.c[0][i] T.c[j][0] + SR.c[1][i] T.c[j][1] + SR.c[2][i] T.c[j][2]
        float M0[3], M1[3];
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const float sr0 = s[i] * Rq[i], sr1 = s[i] * Rq[3 + i], sr2 = s[i] * Rq[6 + i];
            M0[i] = sr0 * Tc0[0] + sr1 * Tc0[1] + sr2 * Tc0[2];
            M1[i] = sr0 * Tc1[0] + sr1 * Tc1[1] + sr2 * Tc1[2];
        }
        // cov = M^T M: cov.c[j][i] = sum_k M.c[i][k] M.c[j][k]
        cov00 = M0[0] * M0[0] + M0[1] * M0[1] + M0[2] * M0[2];
        cov01 = M1[0] * M0[0] + M1[1] * M0[1] + M1[2] * M0[2];
        cov11 = M1[0] * M1[0] + M1[1] * M1[1] + M1[2] * M1[2];
        const float is2[3] = {1.0f / (s[0] * s[0]), 1.0f / (s[1] * s[1]), 1.0f / (s[2] * s[2])};
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++)
                cinv[3 * i + j] = A[3 * i] * A[3 * j] * is2[0] + A[3 * i + 1] * A[3 * j + 1] * is2[1] +
                                  A[3 * i + 2] * A[3 * j + 2] * is2[2];
    } else {
        // cov3D_precomp path (render_forward.cu:162-189): Vrk given; the
        // camera-space inverse via the adjugate when Vrk is well conditioned,
        // else the projector onto the eigenvector of the smallest eigenvalue.
        const float* c = a.cov3D_precomp + 6 * idx;
        const float Vk[9] = {c[0], c[1], c[2], c[1], c[3], c[4], c[2], c[4], c[5]};
        float Vinv[9];
        well_conditioned = sym3_inverse_or_null_projector(Vk, Vinv);
        // cov2D = (T^T Vrk^T) T in glm order (render_forward.cu:168); cov_cam_inv = W_r Vinv W_r^T
        float Wr[9];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) Wr[3 * i + j] = V[4 * j + i];
        const float Tc[3][3] = {{Tc0[0], Tc0[1], Tc0[2]}, {Tc1[0], Tc1[1], Tc1[2]}, {0.f, 0.f, 0.f}};
        // Vrk.c[k] = column k (symmetric); C.c[k][i] = sum_m T.c[i][m] Vrk.c[k][m]
        float C[3][2];
#pragma unroll
        for (int kk = 0; kk < 3; kk++)
#pragma unroll
            for (int i = 0; i < 2; i++)
                C[kk][i] = Tc[i][0] * Vk[3 * kk] + Tc[i][1] * Vk[3 * kk + 1] + Tc[i][2] * Vk[3 * kk + 2];
        cov00 = C[0][0] * Tc[0][0] + C[1][0] * Tc[0][1] + C[2][0] * Tc[0][2];
        cov01 = C[0][1] * Tc[0][0] + C[1][1] * Tc[0][1] + C[2][1] * Tc[0][2];
        cov11 = C[0][1] * Tc[1][0] + C[1][1] * Tc[1][1] + C[2][1] * Tc[1][2];
        float WV[9];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++)
                WV[3 * i + j] = Wr[3 * i] * Vinv[j] + Wr[3 * i + 1] * Vinv[3 + j] + Wr[3 * i + 2] * Vinv[6 + j];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++)
                cinv[3 * i + j] = WV[3 * i] * Wr[3 * j] + WV[3 * i + 1] * Wr[3 * j + 1] + WV[3 * i + 2] * Wr[3 * j + 2];
    }
    const float k = a.kernel_size;
    const float det_0 = fmaxf(1e-6f, cov00 * cov11 - cov01 * cov01);
    const float det_1 = fmaxf(1e-6f, (cov00 + k) * (cov11 + k) - cov01 * cov01);
    const float coef = sqrtf(det_0 / det_1);
    const float ca = cov00 + k, cb = cov01, cc = cov11 + k;

    // ray-plane and normal (render_forward.cu:207-241)
    const float u = g.u, v = g.v;
    const float m0 = cinv[0] * u + cinv[1] * v + cinv[2];
    const float m1 = cinv[3] * u + cinv[4] * v + cinv[5];
    const float m2 = cinv[6] * u + cinv[7] * v + cinv[8];
    const float vb = m0 * u + m1 * v + m2;
    const float u2 = u * u, v2 = v * v, uv = u * v;
    const float l = sqrtf(g.tx * g.tx + g.ty * g.ty + tz * tz);
    const float rl2 = u2 + v2 + 1.f;
    const float fnorm = l / rl2;
    const float ivb = 1.0f / vb;
    const float plx = ((v2 + 1.f) * m0 - uv * m1 - u * m2) * ivb;
    const float ply = (-uv * m0 + (u2 + 1.f) * m1 - v * m2) * ivb;
    const float rsig = well_conditioned ? sqrtf(vb / rl2) : 0.f;
    const float rnx = -plx * fnorm, rny = -ply * fnorm;
    const float il = 1.0f / l;
    const float cnx = rnx * itz - g.tx * il;
    const float cny = rny * itz - g.ty * il;
    const float cnz = -(g.tx * itz * itz) * rnx - (g.ty * itz * itz) * rny - tz * il;
    const float inn = 1.0f / sqrtf(cnx * cnx + cny * cny + cnz * cnz);

    // conic, radius, rect (render_forward.cu:347-368)
    const float det = ca * cc - cb * cb;
    if (det == 0.0f) {
        cull_foot(a, idx);
        return;
    }
    const float det_inv = 1.f / det;
    const float mid = 0.5f * (ca + cc);
    const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float radius = ceilf(3.f * sqrtf(lambda1));
    const float xpix = ndc2pix(hx * p_w, a.W), ypix = ndc2pix(hy * p_w, a.H);
    const int r = (int)radius;
    const uint32_t rminx = min(a.grid_x, (uint32_t)max(0, (int)((xpix - r) / kTile)));
    const uint32_t rminy = min(a.grid_y, (uint32_t)max(0, (int)((ypix - r) / kTile)));
    const uint32_t rmaxx = min(a.grid_x, (uint32_t)max(0, (int)((xpix + r + kTile - 1) / kTile)));
    const uint32_t rmaxy = min(a.grid_y, (uint32_t)max(0, (int)((ypix + r + kTile - 1) / kTile)));
    const uint32_t area = (rmaxx - rminx) * (rmaxy - rminy);
    if (area == 0) {
        cull_foot(a, idx);
        return;
    }

    // colour (render_forward.cu:22-78)
    float col[3];
    if (a.no_color) {  // sample_depth (rasterizer_impl.cu:1080): colour unused
        col[0] = col[1] = col[2] = 0.f;
        a.clamped[idx] = 0;
    } else if (a.colors_precomp == nullptr) {
        float dx = px - a.campos[0], dy = py - a.campos[1], dz = pz - a.campos[2];
        const float dl = sqrtf(dx * dx + dy * dy + dz * dz);
        dx /= dl;
        dy /= dl;
        dz /= dl;
        float Y[16];
        sh_basis(a.D, dx, dy, dz, Y);
        const int n = sh_count(a.D);
        if constexpr (SPLIT)  // (its own instance: the one-row kernel keeps its 126 VGPRs, 4 waves per SIMD)
            load_sh_split(a.shs + (size_t)idx * 3, a.shs_rest + (size_t)idx * (a.SHM - 1) * 3, a.SHM, n, sh);
        else if constexpr (!HOIST)
            load_sh(a.shs + (size_t)idx * a.SHM * 3, a.SHM, n, sh);
        col[0] = Y[0] * sh[0];
        col[1] = Y[0] * sh[1];
        col[2] = Y[0] * sh[2];
        // with the colour, coefficient by coefficient: the backward's colour -> direction
        // Jacobian (gsr_math.h sh_basis_grad; GeomState::ddir), J[3 c + i] = d colour_c / d dir_i
        float J[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 1; kk < 16; kk++) {
            if (kk < n) {
                col[0] += Y[kk] * sh[3 * kk];
                col[1] += Y[kk] * sh[3 * kk + 1];
                col[2] += Y[kk] * sh[3 * kk + 2];
                float gx, gy, gz;
                sh_basis_grad(kk, dx, dy, dz, gx, gy, gz);
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    J[3 * c] += gx * sh[3 * kk + c];
                    J[3 * c + 1] += gy * sh[3 * kk + c];
                    J[3 * c + 2] += gz * sh[3 * kk + c];
                }
            }
        }
        if (a.D > 0) {
#pragma unroll
            for (int j = 0; j < 9; j++) a.ddir[(size_t)j * a.P + idx] = J[j];
        }
        if (a.SGM == 7 && a.SGD == 7) {
            // SG degree 7 (C5): every lobe's axis / colour / sharpness rows
            // loaded at once as wide contiguous accesses (preprocess_bwd.hip
            // sg7_bwd); same arithmetic and order as the loop below
            if constexpr (!HOIST) {
                const size_t o0 = (size_t)idx * 7;
#pragma unroll
                for (int k = 0; k < 21; k++) ax[k] = a.sg_axis[3 * o0 + k];
#pragma unroll
                for (int k = 0; k < 21; k++) sc[k] = a.sg_color[3 * o0 + k];
#pragma unroll
                for (int k = 0; k < 7; k++) sh7[k] = a.sg_sharpness[o0 + k];
            }
#pragma unroll
            for (int sg = 0; sg < 7; sg++) {
                const float gs =
                    expf(sh7[sg] * ((ax[3 * sg] * dx + ax[3 * sg + 1] * dy + ax[3 * sg + 2] * dz) - 1.0f));
                col[0] += sc[3 * sg] * gs;
                col[1] += sc[3 * sg + 1] * gs;
                col[2] += sc[3 * sg + 2] * gs;
            }
        } else
        for (int sg = 0; sg < a.SGD; sg++) {
            const size_t o = (size_t)idx * a.SGM + sg;
            const float* ax = a.sg_axis + 3 * o;
            const float* sc = a.sg_color + 3 * o;
            const float gs = expf(a.sg_sharpness[o] * ((ax[0] * dx + ax[1] * dy + ax[2] * dz) - 1.0f));
            col[0] += sc[0] * gs;
            col[1] += sc[1] * gs;
            col[2] += sc[2] * gs;
        }
        col[0] += 0.5f;
        col[1] += 0.5f;
        col[2] += 0.5f;
        a.clamped[idx] = (uint8_t)((col[0] < 0) | ((col[1] < 0) << 1) | ((col[2] < 0) << 2));
        col[0] = fmaxf(col[0], 0.f);
        col[1] = fmaxf(col[1], 0.f);
        col[2] = fmaxf(col[2], 0.f);
    } else {
        col[0] = a.colors_precomp[3 * idx];
        col[1] = a.colors_precomp[3 * idx + 1];
        col[2] = a.colors_precomp[3 * idx + 2];
        a.clamped[idx] = 0;
    }

    Splat sp;
    sp.w0 = make_float4(xpix, ypix, cc * det_inv, -cb * det_inv);
    sp.w1 = make_float4(ca * det_inv, (HOIST ? opacity : a.opacities[idx]) * coef, plx * fnorm / fx, ply * fnorm / fy);
    sp.w2 = make_float4(g.tc, rsig, col[0], col[1]);
    sp.w3 = make_float4(col[2], cnx * inn, cny * inn, cnz * inn);
    a.splats[idx] = sp;
    a.foot[2 * (size_t)idx] = make_uint4(__float_as_uint(sp.w0.x), __float_as_uint(sp.w0.y), __float_as_uint(sp.w0.z),
                                         __float_as_uint(sp.w0.w));
    a.foot[2 * (size_t)idx + 1] = make_uint4(__float_as_uint(sp.w1.x), __float_as_uint(sp.w1.y), rminx | (rminy << 16),
                                             rmaxx | (rmaxy << 16));
    a.depths[idx] = g.tc;
    a.radii[idx] = r;
    a.tiles_touched[idx] = area;
}

hipError_t launch_preprocess_fwd(const FwdParams& p, const GeomState& gs, int* radii, hipStream_t stream) {
    if (p.P == 0) return hipSuccess;
    PreprocessArgs a;
    a.P = p.P;
    a.D = p.D;
    a.SHM = p.SHM;
    a.SGD = p.SGD;
    a.SGM = p.SGM;
    a.W = p.W;
    a.H = p.H;
    a.means3D = p.means3D;
    a.colors_precomp = p.colors_precomp;
    a.no_color = p.no_color;
    a.opacities = p.opacities;
    a.scales = p.scales;
    a.rotations = p.rotations;
    a.cov3D_precomp = p.cov3D_precomp;
    a.shs = p.shs;
    a.shs_rest = p.shs_rest;
    a.sg_axis = p.sg_axis;
    a.sg_sharpness = p.sg_sharpness;
    a.sg_color = p.sg_color;
    a.scale_modifier = p.scale_modifier;
    a.view = p.view;
    a.proj = p.proj;
    a.campos = p.campos;
    a.tan_fovx = p.tan_fovx;
    a.tan_fovy = p.tan_fovy;
    a.focal_x = p.focal_x;
    a.focal_y = p.focal_y;
    a.kernel_size = p.kernel_size;
    a.grid_x = p.grid_x;
    a.grid_y = p.grid_y;
    a.radii = radii;
    a.clamped = gs.clamped;
    a.ddir = gs.ddir;
    a.depths = gs.depths;
    a.splats = gs.splats;
    a.tiles_touched = gs.tiles_touched;
    a.foot = gs.foot;
    dsort_zero_region(gs.dsort_tmp, p.P, &a.zero_first, &a.zero_words);
    a.zero_K = gs.offsets_K;
    // (the hoisted instance needs every colour row: SH + 7 SG lobes, scales / rotations, no precomputed colours)
    const bool hoist = p.SGM == 7 && p.SGD == 7 && p.shs && !p.shs_rest && p.scales && !p.colors_precomp && !p.no_color;
    if (hoist)
        hipLaunchKernelGGL(preprocess_fwd_kernel<true>, dim3((p.P + 255) / 256), dim3(256), 0, stream, a);
    else if (p.shs_rest)
        hipLaunchKernelGGL((preprocess_fwd_kernel<false, true>), dim3((p.P + 255) / 256), dim3(256), 0, stream, a);
    else
        hipLaunchKernelGGL(preprocess_fwd_kernel<false>, dim3((p.P + 255) / 256), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
