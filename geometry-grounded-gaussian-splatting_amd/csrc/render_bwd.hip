// render_bwd.hip — per-tile back-to-front gradient pass on gfx950.
//
// Replaces renderCUDA<3, GEOMETRY> backward (render_backward.cu:716-1069) and
// BACKWARD::render (:1164-1209).
//
// Same tile/workgroup geometry as render_fwd.hip.  Per (pixel, Gaussian) the
// kernel recomputes alpha and produces up to 17 gradient terms; they are
// summed over the 64 pixels of a wave with one transposed butterfly
// (wave_transpose_reduce16: v_permlane32_swap / v_permlane16_swap, then DPP
// mirrors and quad perms, all VALU), after which lanes 0, 4, ..., 60 hold the
// 16 field totals and issue ONE global_atomic_add_f32 whose 16 field lanes
// cover the Gaussian's 64-B accumulator record (a single 64-B atomic request)
// and whose 17th lane adds the |dmean2D| channel.  The reference (32-lane cg::reduce per field, then 17
// scalar atomics from lane 0) issues 17 single-lane atomic requests per warp
// and Gaussian.  Waves with no valid pixel for a Gaussian skip it (ballot),
// as the reference's warp.any does.
#include "gsr_kernels.h"

namespace gsr {

struct RenderBwdArgs {
    const uint2* ranges;
    const uint32_t* point_list;
    const Splat* splats;
    const uint32_t* n_contrib;
    const uint32_t* max_contrib;
    int W, H;
    uint32_t grid_x, num_tiles;
    float focal_x, focal_y;
    const float* bg;
    const float* alphas;
    const float* normalmap;
    const float* mdepth;
    const float* dL_dpix;
    const float* dL_dmdepth;
    const float* dL_dalpha;
    const float* dL_dnormal;
    float* acc;      // [P][16]
    float* acc_abs;  // [P]
};

template <bool GEOM>
__global__ void __launch_bounds__(256) render_bwd_kernel(RenderBwdArgs a) {
    __shared__ float4 s_w0[kTilePixels], s_w1[kTilePixels], s_w2[kTilePixels], s_w3[kTilePixels];
    __shared__ uint32_t s_id[kTilePixels];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t tile = xcd_remap(blockIdx.x, a.num_tiles);
    const uint32_t tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int px = tx * kTile + (tid & 15), py = ty * kTile + (tid >> 4);
    const bool inside = px < a.W && py < a.H;
    const float pixx = (float)px, pixy = (float)py;
    const uint2 range = a.ranges[tile];
    const int max_contrib = (int)a.max_contrib[tile];
    if (max_contrib == 0) return;  // uniform over the block
    const int HW = a.W * a.H;
    const int pix = a.W * py + px;

    const float w_final = inside ? a.alphas[pix] : 0.f;
    const float T_final = 1.f - w_final;
    float T = T_final;
    const uint32_t last = inside ? a.n_contrib[pix] : 0u;

    float dLp0 = 0.f, dLp1 = 0.f, dLp2 = 0.f, dL_dfinalT = 0.f;
    float dLn0 = 0.f, dLn1 = 0.f, dLn2 = 0.f, mDepth = 0.f, dL_dmt = 0.f;
    if (inside) {
        dLp0 = a.dL_dpix[pix];
        dLp1 = a.dL_dpix[HW + pix];
        dLp2 = a.dL_dpix[2 * HW + pix];
        dL_dfinalT = -a.dL_dalpha[pix] + a.bg[0] * dLp0 + a.bg[1] * dLp1 + a.bg[2] * dLp2;
        if constexpr (GEOM) {
            const float inv_w = 1.f / w_final;
            const float pnx = (pixx - (float)(a.W - 1) / 2.f) / a.focal_x;
            const float pny = (pixy - (float)(a.H - 1) / 2.f) / a.focal_y;
            const float nrm = sqrtf(pnx * pnx + pny * pny + 1.f);
            dL_dmt = a.dL_dmdepth[pix] * (1.0f / nrm);
            dLn0 = a.dL_dnormal[pix] * inv_w;
            dLn1 = a.dL_dnormal[HW + pix] * inv_w;
            dLn2 = a.dL_dnormal[2 * HW + pix] * inv_w;
            dL_dfinalT += dLn0 * a.normalmap[pix] + dLn1 * a.normalmap[HW + pix] + dLn2 * a.normalmap[2 * HW + pix];
            mDepth = a.mdepth[pix] * nrm;
        }
    }
    const int rounds = (max_contrib + kTilePixels - 1) / kTilePixels;

    // ---- median-depth implicit gradient pre-pass (render_backward.cu:835-880)
    float kappa = 0.f;
    if constexpr (GEOM) {
        float dT_dtm = 0.f;
        uint32_t c = 0;
        bool pdone = (mDepth == 0.f) || (last == 0) || !inside;
        int toDo = max_contrib;
        for (int i = 0; i < rounds; i++, toDo -= kTilePixels) {
            __syncthreads();
            const int k = i * kTilePixels + tid;
            if (k < max_contrib) {
                const Splat* sp = a.splats + a.point_list[range.x + k];
                s_w0[tid] = sp->w0;
                s_w1[tid] = sp->w1;
                s_w2[tid] = sp->w2;
            }
            __syncthreads();
            const int n = min(kTilePixels, toDo);
            for (int j = 0; !pdone && j < n; j++) {
                c++;
                pdone = c >= last;
                const float4 w0 = s_w0[j];
                const float dx = w0.x - pixx, dy = w0.y - pixy;
                const float4 w1 = s_w1[j];
                const float power = splat_power(w0, w1, dx, dy);
                if (power > 0.0f) continue;
                const float alpha = fminf(0.99f, w1.y * __expf(power));
                if (alpha < 1.0f / 255.0f) continue;
                const float4 w2 = s_w2[j];
                const float t_peak = splat_tpeak(w1, w2, dx, dy);
                const float rsig = w2.y;
                const float t_delta = (mDepth - t_peak) * rsig;
                const float G_exp = __expf(-0.5f * t_delta * t_delta);
                const float Gt = alpha * G_exp;
                dT_dtm += fast_div(-0.25f * Gt, 1.f - Gt) * fabsf(t_delta) * rsig;
            }
        }
        kappa = dL_dmt / fmaxf(-dT_dtm, 1e-7f);
    }

    // ---- main back-to-front pass (render_backward.cu:882-1068)
    uint32_t contributor = (uint32_t)max_contrib;
    float last_alpha = 0.f;
    float lc0 = 0.f, lc1 = 0.f, lc2 = 0.f, ar0 = 0.f, ar1 = 0.f, ar2 = 0.f;
    float ln0 = 0.f, ln1 = 0.f, ln2 = 0.f, an0 = 0.f, an1 = 0.f, an2 = 0.f;
    const float ddelx_dx = 0.5f * a.W, ddely_dy = 0.5f * a.H;
    int toDo = max_contrib;
    for (int i = 0; i < rounds; i++, toDo -= kTilePixels) {
        __syncthreads();
        const int k = i * kTilePixels + tid;
        if (k < max_contrib) {
            const uint32_t g = a.point_list[range.x + max_contrib - k - 1];
            const Splat sp = a.splats[g];
            s_id[tid] = g;
            s_w0[tid] = sp.w0;
            s_w1[tid] = sp.w1;
            s_w2[tid] = sp.w2;
            s_w3[tid] = sp.w3;
        }
        __syncthreads();
        const int n = min(kTilePixels, toDo);
        for (int j = 0; j < n; j++) {
            contributor--;
            const float4 w0 = s_w0[j];
            const float dx = w0.x - pixx, dy = w0.y - pixy;
            const float4 w1 = s_w1[j];
            const float power = splat_power(w0, w1, dx, dy);
            const float G = __expf(power);
            const float alpha = fminf(0.99f, w1.y * G);
            const bool valid = inside && !(contributor >= last || power > 0.0f || alpha < 1.0f / 255.0f);
            if (__ballot(valid) == 0ull) continue;  // wave-uniform skip (warp.any)

            float f[16];
#pragma unroll
            for (int q = 0; q < 16; q++) f[q] = 0.f;
            float fabs_sum = 0.f;
            if (valid) {
                const float4 w2 = s_w2[j];
                const float4 w3 = s_w3[j];
                const float r1a = fast_rcp(1.f - alpha);
                T = T * r1a;
                const float bw = alpha * T;
                float dL_dopa = 0.f;
                ar0 = last_alpha * lc0 + (1.f - last_alpha) * ar0;
                ar1 = last_alpha * lc1 + (1.f - last_alpha) * ar1;
                ar2 = last_alpha * lc2 + (1.f - last_alpha) * ar2;
                lc0 = w2.z;
                lc1 = w2.w;
                lc2 = w3.x;
                dL_dopa += (lc0 - ar0) * dLp0;
                dL_dopa += (lc1 - ar1) * dLp1;
                dL_dopa += (lc2 - ar2) * dLp2;
                f[kAccColor + 0] = bw * dLp0;
                f[kAccColor + 1] = bw * dLp1;
                f[kAccColor + 2] = bw * dLp2;
                float dL_dt = 0.f, dL_dopa_sigma = 0.f;
                if constexpr (GEOM) {
                    an0 = last_alpha * ln0 + (1.f - last_alpha) * an0;
                    an1 = last_alpha * ln1 + (1.f - last_alpha) * an1;
                    an2 = last_alpha * ln2 + (1.f - last_alpha) * an2;
                    ln0 = w3.y;
                    ln1 = w3.z;
                    ln2 = w3.w;
                    dL_dopa += (ln0 - an0) * dLn0;
                    dL_dopa += (ln1 - an1) * dLn1;
                    dL_dopa += (ln2 - an2) * dLn2;
                    f[kAccNormal + 0] = bw * dLn0;
                    f[kAccNormal + 1] = bw * dLn1;
                    f[kAccNormal + 2] = bw * dLn2;
                    const float t_peak = splat_tpeak(w1, w2, dx, dy);
                    const float rsig = w2.y;
                    const float t_delta = (mDepth - t_peak) * rsig;
                    const float G_exp = __expf(-0.5f * t_delta * t_delta);
                    const float Gt = alpha * G_exp;
                    float dL_dGt = fast_div(kappa * 0.25f, 1.f - Gt);
                    dL_dGt = mDepth > t_peak ? dL_dGt : -dL_dGt;
                    dL_dGt = rsig > 0.f ? dL_dGt : 0.f;
                    dL_dopa_sigma = dL_dGt * G_exp - kappa * (t_delta > 0.f ? 0.5f * r1a : 0.f);
                    const float dL_ddelta = -dL_dGt * Gt * t_delta;
                    dL_dt = -dL_ddelta * rsig;
                    f[kAccPlane + 0] = dL_dt * dx;
                    f[kAccPlane + 1] = dL_dt * dy;
                    f[kAccPlane + 2] = dL_dt;
                    f[kAccPlane + 3] = dL_ddelta * (mDepth - t_peak);
                }
                dL_dopa *= T;
                if constexpr (GEOM) dL_dopa += dL_dopa_sigma;
                dL_dopa += -T_final * r1a * dL_dfinalT;
                last_alpha = alpha;
                const float dL_dG = w1.y * dL_dopa;
                const float gdx = G * dx, gdy = G * dy;
                const float dG_ddelx = -gdx * w0.z - gdy * w0.w;
                const float dG_ddely = -gdy * w1.x - gdx * w0.w;
                float dL_ddelx = dL_dG * dG_ddelx;
                float dL_ddely = dL_dG * dG_ddely;
                if constexpr (GEOM) {
                    dL_ddelx += dL_dt * w1.z;
                    dL_ddely += dL_dt * w1.w;
                }
                f[kAccMean2D + 0] = dL_ddelx * ddelx_dx;
                f[kAccMean2D + 1] = dL_ddely * ddely_dy;
                fabs_sum = fabsf(f[kAccMean2D + 0]) + fabsf(f[kAccMean2D + 1]);
                f[kAccConic + 0] = -0.5f * gdx * dx * dL_dG;
                f[kAccConic + 1] = -0.5f * gdx * dy * dL_dG;
                f[kAccConic + 2] = -0.5f * gdy * dy * dL_dG;
                f[kAccConic + 3] = G * dL_dopa;
            }
            const float red = wave_transpose_reduce16(f);
            const float abs_red = wave_sum_dpp(fabs_sum);
            const uint32_t g = s_id[j];
            // one atomic instruction: lanes 0, 4, .., 60 add the 16 fields of
            // the record (one 64-B line), lane 1 adds |dmean2D|
            const bool field_lane = (lane & 3) == 0 && (GEOM || (lane >> 2) < kAccNormal);
            if (field_lane || lane == 1) {
                float* dst = field_lane ? a.acc + (size_t)g * kAccFields + (lane >> 2) : a.acc_abs + g;
                atomicAdd(dst, field_lane ? red : abs_red);
            }
        }
    }
}

hipError_t launch_render_bwd(const BwdParams& b, const GeomState& gs, const BinningState& bs, const ImageState& is,
                             const TileState& ts, const BwdState& ws, hipStream_t stream) {
    const FwdParams& p = b.f;
    RenderBwdArgs a;
    a.ranges = ts.ranges;
    a.point_list = bs.point_list;
    a.splats = gs.splats;
    a.n_contrib = is.n_contrib;
    a.max_contrib = ts.max_contrib;
    a.W = p.W;
    a.H = p.H;
    a.grid_x = p.grid_x;
    a.num_tiles = p.grid_x * p.grid_y;
    a.focal_x = p.focal_x;
    a.focal_y = p.focal_y;
    a.bg = p.background;
    a.alphas = b.alphas;
    a.normalmap = b.normalmap;
    a.mdepth = b.mdepth;
    a.dL_dpix = b.dL_dpix;
    a.dL_dmdepth = b.dL_dmdepth;
    a.dL_dalpha = b.dL_dalpha;
    a.dL_dnormal = b.dL_dnormal;
    a.acc = ws.acc;
    a.acc_abs = ws.acc_abs;
    if (a.num_tiles == 0) return hipSuccess;
    if (p.require_depth)
        hipLaunchKernelGGL(render_bwd_kernel<true>, dim3(a.num_tiles), dim3(kTilePixels), 0, stream, a);
    else
        hipLaunchKernelGGL(render_bwd_kernel<false>, dim3(a.num_tiles), dim3(kTilePixels), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
