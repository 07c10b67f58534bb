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
    const float* dT_dtm;
    const uint32_t* md_check;
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
    int skip_prepass;  // diagnostic (GSR_OPT_BWD_NO_PREPASS): time the kernel without the pre-pass
    int no_cache;      // GSR_OPT_BWD_NO_CACHE: recompute dT/dt_m everywhere
    const uint32_t* tile_order;  // [tiles] launch order (heaviest first) or null: XCD-contiguous
};

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kBwdThreads = 128;  // 2 wave64 per tile, two pixels per lane
constexpr int kBwdBatch = 256;    // splat records staged per LDS batch

__device__ __forceinline__ f2 sel2(bool ca, bool cb, f2 x, f2 y) { return f2{ca ? x.x : y.x, cb ? x.y : y.y}; }
__device__ __forceinline__ f2 splat2(float v) { return f2{v, v}; }
__device__ __forceinline__ float hsum(f2 v) { return v.x + v.y; }

// splat_power2 / splat_tpeak2 (gsr_common.h) for the two pixels of a lane,
// which share the column (dx) and differ in the row (dy.x, dy.y); the
// packed operations round exactly as the scalar helpers, so alpha and the
// contribute decision stay bit-identical to the forward.

// Per-pixel inputs of the backward (render_backward.cu:771-833).
struct PixIn {
    bool inside, cached;
    uint32_t last;
    float T_final, dLp0, dLp1, dLp2, dL_dfinalT, dLn0, dLn1, dLn2, mDepth, dL_dmt, dT_dtm;
};

template <bool GEOM>
__device__ __forceinline__ PixIn load_pixel(const RenderBwdArgs& a, int px, int py) {
    PixIn r{};
    r.inside = px < a.W && py < a.H;
    r.T_final = 1.f;
    if (!r.inside) return r;
    const int HW = a.W * a.H;
    const int pix = a.W * py + px;
    const float w_final = a.alphas[pix];
    r.T_final = 1.f - w_final;
    r.last = a.n_contrib[pix];
    if (r.last == 0) return r;  // blended nothing: no gradient terms (and 1/alpha would be inf)
    r.dLp0 = a.dL_dpix[pix];
    r.dLp1 = a.dL_dpix[HW + pix];
    r.dLp2 = a.dL_dpix[2 * HW + pix];
    r.dL_dfinalT = -a.dL_dalpha[pix] + a.bg[0] * r.dLp0 + a.bg[1] * r.dLp1 + a.bg[2] * r.dLp2;
    if constexpr (GEOM) {
        const float inv_w = 1.f / w_final;
        const float nrm = pixel_ray_norm((float)px, (float)py, a.W, a.H, a.focal_x, a.focal_y);
        r.dL_dmt = a.dL_dmdepth[pix] * (1.0f / nrm);
        r.dLn0 = a.dL_dnormal[pix] * inv_w;
        r.dLn1 = a.dL_dnormal[HW + pix] * inv_w;
        r.dLn2 = a.dL_dnormal[2 * HW + pix] * inv_w;
        r.dL_dfinalT += r.dLn0 * a.normalmap[pix] + r.dLn1 * a.normalmap[HW + pix] + r.dLn2 * a.normalmap[2 * HW + pix];
        const float md = a.mdepth[pix];
        r.mDepth = md * nrm;
        // the forward computed dT/dt_m for exactly this mdepth value
        r.cached = !a.no_cache && a.md_check[pix] == __float_as_uint(md);
        r.dT_dtm = a.dT_dtm[pix];
    }
    return r;
}

// One workgroup of 128 lanes (2 wave64) per 16x16 tile; lane l of wave w
// owns the pixel pair (x, y) and (x, y + 4) with x = l % 16,
// y = 8 w + l / 16.  The two pixels' state lives in the halves of packed
// fp32 registers (v_pk_{add,mul,fma}_f32), so one instruction stream serves
// two pixels, and the per-(wave, Gaussian) reduction and atomic cover 128
// pixels instead of 64.  Per-pixel validity is a select, not a branch.
template <bool GEOM>
__global__ void __launch_bounds__(kBwdThreads) render_bwd_kernel(RenderBwdArgs a) {
    __shared__ float4 s_w0[kBwdBatch], s_w1[kBwdBatch], s_w2[kBwdBatch], s_w3[kBwdBatch];
    __shared__ uint32_t s_id[kBwdBatch];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const uint32_t tile = a.tile_order ? a.tile_order[blockIdx.x] : xcd_remap(blockIdx.x, a.num_tiles);
    const uint32_t tx = tile % a.grid_x, ty = tile / a.grid_x;
    const uint2 range = a.ranges[tile];
    const int max_contrib = (int)a.max_contrib[tile];
    if (max_contrib == 0) return;  // uniform over the block

    const int px = tx * kTile + (lane & 15);
    const int pya = ty * kTile + wave * 8 + (lane >> 4), pyb = pya + 4;
    const PixIn pa = load_pixel<GEOM>(a, px, pya);
    const PixIn pb = load_pixel<GEOM>(a, px, pyb);
    const float pixx = (float)px;
    const f2 pixy = {(float)pya, (float)pyb};
    const bool ina = pa.inside, inb = pb.inside;
    const uint32_t last_a = pa.last, last_b = pb.last;
    const f2 T_final = {pa.T_final, pb.T_final};
    const f2 dLp0 = {pa.dLp0, pb.dLp0}, dLp1 = {pa.dLp1, pb.dLp1}, dLp2 = {pa.dLp2, pb.dLp2};
    const f2 dL_dfinalT = {pa.dL_dfinalT, pb.dL_dfinalT};
    const f2 dLn0 = {pa.dLn0, pb.dLn0}, dLn1 = {pa.dLn1, pb.dLn1}, dLn2 = {pa.dLn2, pb.dLn2};
    const f2 mDepth = {pa.mDepth, pb.mDepth};
    const int rounds = (max_contrib + kBwdBatch - 1) / kBwdBatch;

    auto stage_fwd = [&](int i) {
        for (int k = tid; k < kBwdBatch; k += kBwdThreads) {
            const int c = i * kBwdBatch + k;
            if (c < max_contrib) {
                const Splat* sp = a.splats + a.point_list[range.x + c];
                s_w0[k] = sp->w0;
                s_w1[k] = sp->w1;
                s_w2[k] = sp->w2;
            }
        }
    };

    // ---- median-depth implicit gradient pre-pass (render_backward.cu:835-880)
    // Pixels whose mdepth is the forward's own output take dT/dt_m from the
    // forward (render_fwd.hip); the others (an mdepth the caller changed, a
    // tile too long for the forward's LDS cache) recompute it here.
    f2 kappa = {0.f, 0.f};
    if (GEOM && !a.skip_prepass) {
        f2 dT_dtm = {pa.cached ? pa.dT_dtm : 0.f, pb.cached ? pb.dT_dtm : 0.f};
        const bool on_a = ina && pa.mDepth != 0.f && last_a != 0 && !pa.cached;
        const bool on_b = inb && pb.mDepth != 0.f && last_b != 0 && !pb.cached;
        const uint32_t wave_last = wave_max_u(max(on_a ? last_a : 0u, on_b ? last_b : 0u));
        const bool block_needs = __syncthreads_or(wave_last != 0u);
        uint32_t c = 0;
        int toDo = max_contrib;
        for (int i = 0; block_needs && i < rounds; i++, toDo -= kBwdBatch) {
            __syncthreads();
            stage_fwd(i);
            __syncthreads();
            const int n = min(kBwdBatch, toDo);
            for (int j = 0; j < n && c < wave_last; j++) {
                c++;
                const float4 w0 = s_w0[j];
                const float4 w1 = s_w1[j];
                const float dx = w0.x - pixx;
                const f2 dy = splat2(w0.y) - pixy;
                const f2 power = splat_power2(w0, w1, dx, dy);
                const f2 alpha = {fminf(0.99f, w1.y * __expf(power.x)), fminf(0.99f, w1.y * __expf(power.y))};
                const bool va = on_a && c <= last_a && !(power.x > 0.f) && !(alpha.x < 1.0f / 255.0f);
                const bool vb = on_b && c <= last_b && !(power.y > 0.f) && !(alpha.y < 1.0f / 255.0f);
                const float4 w2 = s_w2[j];
                const f2 t_peak = splat_tpeak2(w1, w2, dx, dy);
                const float rsig = w2.y;
                const f2 t_delta = (mDepth - t_peak) * rsig;
                const f2 G_exp = {__expf(-0.5f * t_delta.x * t_delta.x), __expf(-0.5f * t_delta.y * t_delta.y)};
                const f2 Gt = alpha * G_exp;
                const f2 term = f2{fast_div(-0.25f * Gt.x, 1.f - Gt.x), fast_div(-0.25f * Gt.y, 1.f - Gt.y)} *
                                f2{fabsf(t_delta.x), fabsf(t_delta.y)} * rsig;
                dT_dtm += sel2(va, vb, term, splat2(0.f));
            }
        }
        kappa = f2{pa.dL_dmt / fmaxf(-dT_dtm.x, 1e-7f), pb.dL_dmt / fmaxf(-dT_dtm.y, 1e-7f)};
    }

    // ---- main back-to-front pass (render_backward.cu:882-1068)
    // The reference carries (last_alpha, last_colour) one step and folds them
    // into accum_rec at the NEXT valid contributor; here a contributor is
    // folded in right after its own terms (same values; accum_rec's update is
    // written as one fma, a few ulp from the reference's rounding).  A pixel
    // for which the splat is not valid runs with alpha = 0, which leaves
    // T (x rcp(1) = 1), accum_rec (+ 0 x d) and the plane terms unchanged
    // exactly, so only G dL/dopacity needs a select.
    uint32_t contributor = (uint32_t)max_contrib;
    f2 T = T_final;
    const f2 tfd = -T_final * dL_dfinalT;  // dL/dopacity term of the final transmittance, / (1 - alpha)
    const f2 kappa_q = 0.25f * kappa;
    f2 ar0 = {0.f, 0.f}, ar1 = {0.f, 0.f}, ar2 = {0.f, 0.f};
    f2 an0 = {0.f, 0.f}, an1 = {0.f, 0.f}, an2 = {0.f, 0.f};
    const float ddelx_dx = 0.5f * a.W, ddely_dy = 0.5f * a.H;
    const f2 zero = {0.f, 0.f}, one = {1.f, 1.f};
    int toDo = max_contrib;
    for (int i = 0; i < rounds; i++, toDo -= kBwdBatch) {
        __syncthreads();
        for (int k = tid; k < kBwdBatch; k += kBwdThreads) {
            const int c = i * kBwdBatch + k;
            if (c < max_contrib) {
                const uint32_t g = a.point_list[range.x + max_contrib - c - 1];
                const Splat* sp = a.splats + g;
                s_id[k] = g;
                s_w0[k] = sp->w0;
                s_w1[k] = sp->w1;
                s_w2[k] = sp->w2;
                s_w3[k] = sp->w3;
            }
        }
        __syncthreads();
        const int n = min(kBwdBatch, toDo);
        for (int j = 0; j < n; j++) {
            contributor--;
            const float4 w0 = s_w0[j];
            const float4 w1 = s_w1[j];
            const float dx = w0.x - pixx;
            const f2 dy = splat2(w0.y) - pixy;
            const f2 power = splat_power2(w0, w1, dx, dy);
            const f2 G = {__expf(power.x), __expf(power.y)};
            const f2 alpha_raw = {fminf(0.99f, w1.y * G.x), fminf(0.99f, w1.y * G.y)};
            const bool va = ina && !(contributor >= last_a || power.x > 0.0f || alpha_raw.x < 1.0f / 255.0f);
            const bool vb = inb && !(contributor >= last_b || power.y > 0.0f || alpha_raw.y < 1.0f / 255.0f);
            if (__ballot(va || vb) == 0ull) continue;  // wave-uniform skip (warp.any)

            const float4 w2 = s_w2[j];
            const float4 w3 = s_w3[j];
            const f2 alpha = sel2(va, vb, alpha_raw, zero);
            const f2 one_m_alpha = one - alpha;
            const f2 r1a = {fast_rcp(one_m_alpha.x), fast_rcp(one_m_alpha.y)};
            T = T * r1a;
            const f2 bw = alpha * T;
            // accum_rec = alpha c + (1 - alpha) accum_rec as accum_rec + alpha (c - accum_rec)
            const f2 d0 = splat2(w2.z) - ar0, d1 = splat2(w2.w) - ar1, d2 = splat2(w3.x) - ar2;
            f2 dL_dopa = d0 * dLp0 + d1 * dLp1 + d2 * dLp2;
            ar0 = __builtin_elementwise_fma(alpha, d0, ar0);
            ar1 = __builtin_elementwise_fma(alpha, d1, ar1);
            ar2 = __builtin_elementwise_fma(alpha, d2, ar2);
            float f[16];
            f[kAccColor + 0] = hsum(bw * dLp0);
            f[kAccColor + 1] = hsum(bw * dLp1);
            f[kAccColor + 2] = hsum(bw * dLp2);
            f2 dL_dt = zero;
            if constexpr (GEOM) {
                const f2 e0 = splat2(w3.y) - an0, e1 = splat2(w3.z) - an1, e2 = splat2(w3.w) - an2;
                dL_dopa += e0 * dLn0 + e1 * dLn1 + e2 * dLn2;
                an0 = __builtin_elementwise_fma(alpha, e0, an0);
                an1 = __builtin_elementwise_fma(alpha, e1, an1);
                an2 = __builtin_elementwise_fma(alpha, e2, an2);
                f[kAccNormal + 0] = hsum(bw * dLn0);
                f[kAccNormal + 1] = hsum(bw * dLn1);
                f[kAccNormal + 2] = hsum(bw * dLn2);
                const f2 t_peak = splat_tpeak2(w1, w2, dx, dy);
                const float rsig = w2.y;
                const f2 dmt = mDepth - t_peak;
                const f2 t_delta = dmt * rsig;
                // exp(-delta^2 / 2) as exp2(delta^2 (-log2 e / 2))
                const f2 ge = (t_delta * t_delta) * splat2(-0.72134752044448170368f);
                const f2 G_exp = {__builtin_amdgcn_exp2f(ge.x), __builtin_amdgcn_exp2f(ge.y)};
                const f2 Gt = alpha * G_exp;  // 0 for a non-valid pixel -> no plane terms
                const f2 omGt = one - Gt;
                // 0.25 kappa / (1 - Gt), + in front of the peak, - behind; 0 for a non-ball splat
                f2 dL_dGt = (kappa_q * (rsig > 0.f ? 1.f : 0.f)) * f2{fast_rcp(omGt.x), fast_rcp(omGt.y)};
                dL_dGt = sel2(dmt.x > 0.f, dmt.y > 0.f, dL_dGt, -dL_dGt);
                const f2 half_r = sel2(t_delta.x > 0.f, t_delta.y > 0.f, 0.5f * r1a, zero);
                const f2 dL_dopa_sigma = dL_dGt * G_exp - kappa * half_r;
                const f2 dL_ddelta = -dL_dGt * Gt * t_delta;
                dL_dt = -dL_ddelta * rsig;
                const float hdt = hsum(dL_dt);
                f[kAccPlane + 0] = hdt * dx;
                f[kAccPlane + 1] = hsum(dL_dt * dy);
                f[kAccPlane + 2] = hdt;
                f[kAccPlane + 3] = hsum(dL_ddelta * dmt);
                dL_dopa = __builtin_elementwise_fma(dL_dopa, T, dL_dopa_sigma);
            } else {
                dL_dopa = dL_dopa * T;
            }
            dL_dopa = __builtin_elementwise_fma(tfd, r1a, dL_dopa);
            // p = G dL/dopacity on the valid pixels; every remaining term is a multiple of it:
            // dL/dG G = op p, dG/ddelx = -G (a dx + b dy), dG/ddely = -G (c dy + b dx),
            // dG/dconic = -G/2 (dx^2, dx dy, dy^2)
            const f2 p = sel2(va, vb, G * dL_dopa, zero);
            const f2 q = w1.y * p;
            const f2 nq = -q;
            f2 dL_ddelx = nq * __builtin_elementwise_fma(splat2(w0.w), dy, splat2(w0.z * dx));
            f2 dL_ddely = nq * __builtin_elementwise_fma(splat2(w1.x), dy, splat2(w0.w * dx));
            if constexpr (GEOM) {
                dL_ddelx = __builtin_elementwise_fma(dL_dt, splat2(w1.z), dL_ddelx);
                dL_ddely = __builtin_elementwise_fma(dL_dt, splat2(w1.w), dL_ddely);
            }
            const f2 mx = dL_ddelx * ddelx_dx, my = dL_ddely * ddely_dy;
            f[kAccMean2D + 0] = hsum(mx);
            f[kAccMean2D + 1] = hsum(my);
            const float fabs_sum = (fabsf(mx.x) + fabsf(my.x)) + (fabsf(mx.y) + fabsf(my.y));
            const f2 qdy = q * dy;
            f[kAccConic + 0] = hsum(q) * (-0.5f * dx * dx);
            f[kAccConic + 1] = hsum(qdy) * (-0.5f * dx);
            f[kAccConic + 2] = -0.5f * hsum(qdy * dy);
            f[kAccConic + 3] = hsum(p);
            if constexpr (!GEOM) {
#pragma unroll
                for (int q = kAccNormal; q < kAccFields; q++) f[q] = 0.f;
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
    a.dT_dtm = is.dT_dtm;
    a.md_check = is.md_check;
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
    a.skip_prepass = option(kOptBwdNoPrepass);
    a.no_cache = option(kOptBwdNoCache);
    a.tile_order = ws.tile_order;
    if (a.num_tiles == 0) return hipSuccess;
    if (p.require_depth)
        hipLaunchKernelGGL(render_bwd_kernel<true>, dim3(a.num_tiles), dim3(kBwdThreads), 0, stream, a);
    else
        hipLaunchKernelGGL(render_bwd_kernel<false>, dim3(a.num_tiles), dim3(kBwdThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
