// render_bwd.hip — per-tile back-to-front gradient pass on gfx950.
//
// Replaces renderCUDA<3, GEOMETRY> backward (render_backward.cu:716-1069) and
// BACKWARD::render (:1164-1209).
//
// One wave64 per 16x16 tile (four pixels per lane, in two packed pairs).  Per (pixel, Gaussian)
// the kernel recomputes alpha and produces up to 17 gradient terms; they are
// summed over the lane's pixels, then over the wave with one transposed butterfly
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
    const uint32_t* blend_mask;  // [tiles][kBlendWords]: entries some pixel blended in the forward
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
    int no_cache;      // GSR_OPT_BWD_NO_CACHE: recompute dT/dt_m everywhere
    const uint32_t* tile_order;  // [tiles] launch order (heaviest first) or null: XCD-contiguous
};

typedef float f2 __attribute__((ext_vector_type(2)));
#ifndef GSR_BWD_WAVES
#define GSR_BWD_WAVES 3
#endif
constexpr int kBwdBatch = 128;    // splat records staged per LDS batch (8.5 KB: 3 one-wave blocks per SIMD)

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
    // (a NULL upstream gradient is zero)
    r.dLp0 = a.dL_dpix ? a.dL_dpix[pix] : 0.f;
    r.dLp1 = a.dL_dpix ? a.dL_dpix[HW + pix] : 0.f;
    r.dLp2 = a.dL_dpix ? a.dL_dpix[2 * HW + pix] : 0.f;
    r.dL_dfinalT = -(a.dL_dalpha ? a.dL_dalpha[pix] : 0.f) + a.bg[0] * r.dLp0 + a.bg[1] * r.dLp1 + a.bg[2] * r.dLp2;
    if constexpr (GEOM) {
        const float inv_w = 1.f / w_final;
        const float nrm = pixel_ray_norm((float)px, (float)py, a.W, a.H, a.focal_x, a.focal_y);
        r.dL_dmt = (a.dL_dmdepth ? a.dL_dmdepth[pix] : 0.f) * (1.0f / nrm);
        r.dLn0 = (a.dL_dnormal ? a.dL_dnormal[pix] : 0.f) * inv_w;
        r.dLn1 = (a.dL_dnormal ? a.dL_dnormal[HW + pix] : 0.f) * inv_w;
        r.dLn2 = (a.dL_dnormal ? a.dL_dnormal[2 * HW + pix] : 0.f) * inv_w;
        r.dL_dfinalT += r.dLn0 * a.normalmap[pix] + r.dLn1 * a.normalmap[HW + pix] + r.dLn2 * a.normalmap[2 * HW + pix];
        const float md = a.mdepth[pix];
        r.mDepth = md * nrm;
        // the forward computed dT/dt_m for exactly this mdepth value
        r.cached = !a.no_cache && a.md_check[pix] == __float_as_uint(md);
        r.dT_dtm = a.dT_dtm[pix];
    }
    return r;
}

// Per-lane pixel pair: the pixels (x, y) and (x, y + 4) in the halves of
// packed fp32 registers (v_pk_{add,mul,fma}_f32), one instruction stream for
// both.  Per-pixel validity is a select, not a branch.
struct PixPair {
    f2 pixy, T_final, dLp0, dLp1, dLp2, dL_dfinalT, dLn0, dLn1, dLn2, mDepth, dL_dmt, dT_cached;
    bool ina, inb, ca, cb;
    uint32_t last_a, last_b;
};

template <bool GEOM>
__device__ __forceinline__ PixPair load_pair(const RenderBwdArgs& a, int px, int py) {
    const PixIn pa = load_pixel<GEOM>(a, px, py), pb = load_pixel<GEOM>(a, px, py + 4);
    PixPair r;
    r.pixy = f2{(float)py, (float)(py + 4)};
    r.T_final = f2{pa.T_final, pb.T_final};
    r.dLp0 = f2{pa.dLp0, pb.dLp0};
    r.dLp1 = f2{pa.dLp1, pb.dLp1};
    r.dLp2 = f2{pa.dLp2, pb.dLp2};
    r.dL_dfinalT = f2{pa.dL_dfinalT, pb.dL_dfinalT};
    r.dLn0 = f2{pa.dLn0, pb.dLn0};
    r.dLn1 = f2{pa.dLn1, pb.dLn1};
    r.dLn2 = f2{pa.dLn2, pb.dLn2};
    r.mDepth = f2{pa.mDepth, pb.mDepth};
    r.dL_dmt = f2{pa.dL_dmt, pb.dL_dmt};
    r.dT_cached = f2{pa.cached ? pa.dT_dtm : 0.f, pb.cached ? pb.dT_dtm : 0.f};
    r.ina = pa.inside;
    r.inb = pb.inside;
    r.ca = pa.cached;
    r.cb = pb.cached;
    r.last_a = pa.last;
    r.last_b = pb.last;
    return r;
}

// One workgroup of 128 / NP lanes per 16x16 tile; lane l of wave w owns NP
// pixel pairs, pair k at x = l % 16, y = 8 (NP w + k) + l / 16 (and y + 4).
// The per-(wave, Gaussian) field sums and the one atomic instruction then
// cover 128 NP pixels: NP = 2 (one wave per tile) halves the reductions and
// atomics per pixel and amortises the record's shared work over 4 pixels per
// lane, against a larger register file per wave.  Measured at C3: NP = 2 with
// 128-record batches (8.5 KB of LDS) at 3 waves per SIMD (154 VGPRs) 0.516 ms;
// with 256-record batches (17 KB: at most 9 blocks per CU) 0.540 at 180 VGPRs,
// 0.568 at 168, 0.619 with 2 spilled registers; 4 waves per SIMD spill 72;
// NP = 1 0.565.
template <bool GEOM, int NP>
__global__ void __launch_bounds__(128 / NP) __attribute__((amdgpu_waves_per_eu(NP == 1 ? 4 : GSR_BWD_WAVES, 8)))
    render_bwd_kernel(RenderBwdArgs a) {
    constexpr int kThreads = 128 / NP;
    __shared__ float4 s_w0[kBwdBatch], s_w1[kBwdBatch], s_w2[kBwdBatch], s_w3[kBwdBatch];
    __shared__ uint32_t s_id[kBwdBatch];
    __shared__ uint32_t s_bm[kBlendWords];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const uint32_t tile = a.tile_order ? a.tile_order[blockIdx.x] : xcd_remap(blockIdx.x, a.num_tiles);
    const uint32_t tx = tile % a.grid_x, ty = tile / a.grid_x;
    const uint2 range = a.ranges[tile];
    const int max_contrib = (int)a.max_contrib[tile];
    if (max_contrib == 0) return;  // uniform over the block

    const int px = tx * kTile + (lane & 15);
    const float pixx = (float)px;
    PixPair pp[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) pp[k] = load_pair<GEOM>(a, px, ty * kTile + 8 * (NP * wave + k) + (lane >> 4));
    const int rounds = (max_contrib + kBwdBatch - 1) / kBwdBatch;
    const f2 zero = {0.f, 0.f}, one = {1.f, 1.f};

    auto stage_fwd = [&](int i) {
        for (int k = tid; k < kBwdBatch; k += kThreads) {
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
    f2 kappa[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) kappa[k] = zero;
    if (GEOM) {
        f2 dT_dtm[NP];
        bool on_a[NP], on_b[NP];
        uint32_t mine = 0;
#pragma unroll
        for (int k = 0; k < NP; k++) {
            const PixPair& P = pp[k];
            dT_dtm[k] = P.dT_cached;
            on_a[k] = P.ina && P.mDepth.x != 0.f && P.last_a != 0 && !P.ca;
            on_b[k] = P.inb && P.mDepth.y != 0.f && P.last_b != 0 && !P.cb;
            mine = max(mine, max(on_a[k] ? P.last_a : 0u, on_b[k] ? P.last_b : 0u));
        }
        const uint32_t wave_last = wave_max_u(mine);
        const bool block_needs = NP == 2 ? wave_last != 0u : __syncthreads_or(wave_last != 0u);
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
                const float4 w2 = s_w2[j];
                const float dx = w0.x - pixx;
                const float rsig = w2.y;
#pragma unroll
                for (int k = 0; k < NP; k++) {
                    const PixPair& P = pp[k];
                    const f2 dy = splat2(w0.y) - P.pixy;
                    const f2 power = splat_power2(w0, w1, dx, dy);
                    const f2 alpha = {fminf(0.99f, w1.y * __expf(power.x)), fminf(0.99f, w1.y * __expf(power.y))};
                    const bool va = on_a[k] && c <= P.last_a && !(power.x > 0.f) && !(alpha.x < 1.0f / 255.0f);
                    const bool vb = on_b[k] && c <= P.last_b && !(power.y > 0.f) && !(alpha.y < 1.0f / 255.0f);
                    const f2 t_peak = splat_tpeak2(w1, w2, dx, dy);
                    const f2 t_delta = (P.mDepth - t_peak) * rsig;
                    const f2 G_exp = {__expf(-0.5f * t_delta.x * t_delta.x), __expf(-0.5f * t_delta.y * t_delta.y)};
                    const f2 Gt = alpha * G_exp;
                    const f2 term = f2{fast_div(-0.25f * Gt.x, 1.f - Gt.x), fast_div(-0.25f * Gt.y, 1.f - Gt.y)} *
                                    f2{fabsf(t_delta.x), fabsf(t_delta.y)} * rsig;
                    dT_dtm[k] += sel2(va, vb, term, zero);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < NP; k++)
            kappa[k] = f2{pp[k].dL_dmt.x / fmaxf(-dT_dtm[k].x, 1e-7f), pp[k].dL_dmt.y / fmaxf(-dT_dtm[k].y, 1e-7f)};
    }

    // ---- main back-to-front pass (render_backward.cu:882-1068)
    // The reference carries (last_alpha, last_colour) one step and folds them
    // into accum_rec at the NEXT valid contributor; here a contributor is
    // folded in right after its own terms.  accum_rec (and accum_normal) enter
    // the gradient only through sum_ch (c_ch - accum_rec_ch) dL/dpixel_ch
    // (render_backward.cu:946-957), so the pixel keeps the one running dot
    // product S = sum_ch accum_rec_ch dL/dpixel_ch instead of the three
    // channels: dL/dalpha = c.dL - S, then S += alpha (c.dL - S) — the same
    // recurrence, dotted with the pixel's constant dL/dpixel (5 operations per
    // pixel instead of 9, a few ulp of rounding apart).  A pixel for which the
    // splat is not valid runs with alpha = 0, which leaves T (x rcp(1) = 1), S
    // (+ 0 x d) and the plane terms unchanged exactly, so only G dL/dopacity
    // needs a select.
    uint32_t contributor = (uint32_t)max_contrib;
    f2 T[NP], tfd[NP], kh[NP], sc[NP], sn[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) {
        T[k] = pp[k].T_final;
        tfd[k] = -pp[k].T_final * pp[k].dL_dfinalT;  // dL/dopacity term of the final transmittance, / (1 - alpha)
        kh[k] = 0.5f * kappa[k];
        sc[k] = sn[k] = zero;
    }
    const float ddelx_dx = 0.5f * a.W, ddely_dy = 0.5f * a.H;
    // factor of field lane >> 2 after the reduction: the NDC scale of dL/dmean2D, -1/2 of dL/dconic's
    // three terms (exact: a power of two)
    const int field = lane >> 2;
    const float post_scale = field == kAccMean2D     ? ddelx_dx
                             : field == kAccMean2D + 1 ? ddely_dy
                             : (field >= kAccConic && field < kAccConic + 3) ? -0.5f
                                                                              : 1.f;
    // the entries no pixel of the tile blended in the forward: skipped without evaluation (entries past the
    // mask's kBlendWords * 32 are all walked)
    if (tid < kBlendWords) s_bm[tid] = a.blend_mask[(size_t)tile * kBlendWords + tid];
    __syncthreads();
    auto needed = [&](int e) { return e >= kBlendWords * 32 || ((s_bm[e >> 5] >> (e & 31)) & 1u) != 0u; };
    int toDo = max_contrib;
    static_assert(kBwdBatch == 128 && kThreads == 64, "one wave stages a 128-record batch, two ballots");
    for (int i = 0; i < rounds; i++, toDo -= kBwdBatch) {
        // this batch's entries (back to front: slot k holds entry max_contrib - 1 - (i * kBwdBatch + k))
        const int c0 = i * kBwdBatch + tid, c1 = c0 + kThreads;
        const bool need0 = c0 < max_contrib && needed(max_contrib - 1 - c0);
        const bool need1 = c1 < max_contrib && needed(max_contrib - 1 - c1);
        unsigned long long m0 = __ballot(need0), m1 = __ballot(need1);
        if ((m0 | m1) == 0ull) continue;  // (wave-uniform: one wave per tile)
        __syncthreads();
        {
            // every needed list entry of the batch, then every record, requested before
            // any is stored (left to itself the compiler waited on each of the
            // four record loads in turn, reusing one register quad)
            constexpr int kPer = kBwdBatch / kThreads;
            const bool need[kPer] = {need0, need1};
            uint32_t g[kPer];
#pragma unroll
            for (int u = 0; u < kPer; u++) {
                const int c = i * kBwdBatch + tid + u * kThreads;
                g[u] = need[u] ? a.point_list[range.x + max_contrib - c - 1] : 0u;
            }
            float4 r[kPer][4];
#pragma unroll
            for (int u = 0; u < kPer; u++) {
                const float4* sp = reinterpret_cast<const float4*>(a.splats + g[u]);
#pragma unroll
                for (int w = 0; w < 4; w++) r[u][w] = need[u] ? sp[w] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < kPer; u++) {
                const int k = tid + u * kThreads;
                if (need[u]) {
                    s_id[k] = g[u];
                    s_w0[k] = r[u][0];
                    s_w1[k] = r[u][1];
                    s_w2[k] = r[u][2];
                    s_w3[k] = r[u][3];
                }
            }
        }
        __syncthreads();
        while ((m0 | m1) != 0ull) {
            int j;
            if (m0) {
                j = __builtin_ctzll(m0);
                m0 &= m0 - 1ull;
            } else {
                j = 64 + __builtin_ctzll(m1);
                m1 &= m1 - 1ull;
            }
            contributor = (uint32_t)(max_contrib - 1 - (i * kBwdBatch + j));
            const float4 w0 = s_w0[j];
            const float4 w1 = s_w1[j];
            const float dx = w0.x - pixx;
            f2 dy[NP], G[NP], alpha_raw[NP];
            bool va[NP], vb[NP];
            bool any = false;
#pragma unroll
            for (int k = 0; k < NP; k++) {
                dy[k] = splat2(w0.y) - pp[k].pixy;
                const f2 power = splat_power2(w0, w1, dx, dy[k]);
                // __expf(x) = v_exp_f32(x log2 e) (the forward's rounding), the products packed
                const f2 pe = power * splat2(1.44269504088896340736f);
                G[k] = f2{__builtin_amdgcn_exp2f(pe.x), __builtin_amdgcn_exp2f(pe.y)};
                const f2 og = splat2(w1.y) * G[k];
                alpha_raw[k] = f2{fminf(0.99f, og.x), fminf(0.99f, og.y)};
                // (bitwise, not short-circuit: straight-line compares the ballot below reads directly)
                va[k] = pp[k].ina & (contributor < pp[k].last_a) & !(power.x > 0.0f) & !(alpha_raw[k].x < 1.0f / 255.0f);
                vb[k] = pp[k].inb & (contributor < pp[k].last_b) & !(power.y > 0.0f) & !(alpha_raw[k].y < 1.0f / 255.0f);
                any = any | va[k] | vb[k];
            }
            if (__ballot(any) == 0ull) continue;  // wave-uniform skip (warp.any)

            const float4 w2 = s_w2[j];
            const float4 w3 = s_w3[j];
            // (wave-uniform: in a scalar register, so the test is a scalar compare)
            const float rsig = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, w2.y)));
            const float ks = rsig > 0.f ? 0.5f : 0.f;  // 0.25 kappa = 0.5 kh; non-ball splat: no plane terms
            // field sums over the lane's pixels (the conic / plane terms keep
            // their per-lane factors dx out of the sums)
            f2 Fc0, Fc1, Fc2, Fn0, Fn1, Fn2, Fdt, Fdtdy, Fdd, Fmx, Fmy, Fq, Fqdy, Fqdy2, Fp;
            float fabs_sum = 0.f;
#pragma unroll
            for (int k = 0; k < NP; k++) {
                const PixPair& P = pp[k];
                const f2 alpha = sel2(va[k], vb[k], alpha_raw[k], zero);
                const f2 one_m_alpha = one - alpha;
                const f2 r1a = {fast_rcp(one_m_alpha.x), fast_rcp(one_m_alpha.y)};
                T[k] = T[k] * r1a;
                const f2 bw = alpha * T[k];
                // accum_rec . dL/dpixel as S + alpha (c . dL/dpixel - S)
                const f2 cdl = __builtin_elementwise_fma(
                    splat2(w3.x), P.dLp2, __builtin_elementwise_fma(splat2(w2.w), P.dLp1, splat2(w2.z) * P.dLp0));
                f2 dL_dopa = cdl - sc[k];
                sc[k] = __builtin_elementwise_fma(alpha, dL_dopa, sc[k]);
                const f2 c0 = bw * P.dLp0, c1 = bw * P.dLp1, c2 = bw * P.dLp2;
                Fc0 = k ? Fc0 + c0 : c0;
                Fc1 = k ? Fc1 + c1 : c1;
                Fc2 = k ? Fc2 + c2 : c2;
                f2 dL_dt = zero;
                if constexpr (GEOM) {
                    const f2 ndl = __builtin_elementwise_fma(
                        splat2(w3.w), P.dLn2, __builtin_elementwise_fma(splat2(w3.z), P.dLn1, splat2(w3.y) * P.dLn0));
                    const f2 e = ndl - sn[k];
                    dL_dopa += e;
                    sn[k] = __builtin_elementwise_fma(alpha, e, sn[k]);
                    const f2 n0 = bw * P.dLn0, n1 = bw * P.dLn1, n2 = bw * P.dLn2;
                    Fn0 = k ? Fn0 + n0 : n0;
                    Fn1 = k ? Fn1 + n1 : n1;
                    Fn2 = k ? Fn2 + n2 : n2;
                    const f2 t_peak = splat_tpeak2(w1, w2, dx, dy[k]);
                    const f2 dmt = P.mDepth - t_peak;
                    const f2 t_delta = dmt * rsig;
                    // exp(-delta^2 / 2) as exp2(delta^2 (-log2 e / 2))
                    const f2 ge = (t_delta * t_delta) * splat2(-0.72134752044448170368f);
                    const f2 G_exp = {__builtin_amdgcn_exp2f(ge.x), __builtin_amdgcn_exp2f(ge.y)};
                    const f2 Gt = alpha * G_exp;  // 0 for a non-valid pixel -> no plane terms
                    const f2 omGt = one - Gt;
                    // 0.25 kappa / (1 - Gt), + in front of the peak, - behind
                    f2 dL_dGt = (kh[k] * ks) * f2{fast_rcp(omGt.x), fast_rcp(omGt.y)};
                    dL_dGt = sel2(dmt.x > 0.f, dmt.y > 0.f, dL_dGt, -dL_dGt);
                    // kappa (0.5 / (1 - alpha)) behind the peak (kh = kappa / 2: the same rounding)
                    const f2 kr = sel2(t_delta.x > 0.f, t_delta.y > 0.f, kh[k] * r1a, zero);
                    const f2 dL_dopa_sigma = dL_dGt * G_exp - kr;
                    const f2 dL_ddelta = -dL_dGt * Gt * t_delta;
                    dL_dt = -dL_ddelta * rsig;
                    const f2 dtdy = dL_dt * dy[k], dd = dL_ddelta * dmt;
                    Fdt = k ? Fdt + dL_dt : dL_dt;
                    Fdtdy = k ? Fdtdy + dtdy : dtdy;
                    Fdd = k ? Fdd + dd : dd;
                    dL_dopa = __builtin_elementwise_fma(dL_dopa, T[k], dL_dopa_sigma);
                } else {
                    dL_dopa = dL_dopa * T[k];
                }
                dL_dopa = __builtin_elementwise_fma(tfd[k], r1a, dL_dopa);
                // p = G dL/dopacity on the valid pixels; every remaining term is a multiple of it:
                // dL/dG G = op p, dG/ddelx = -G (a dx + b dy), dG/ddely = -G (c dy + b dx),
                // dG/dconic = -G/2 (dx^2, dx dy, dy^2)
                const f2 p = sel2(va[k], vb[k], G[k] * dL_dopa, zero);
                const f2 q = w1.y * p;
                const f2 nq = -q;
                f2 dL_ddelx = nq * __builtin_elementwise_fma(splat2(w0.w), dy[k], splat2(w0.z * dx));
                f2 dL_ddely = nq * __builtin_elementwise_fma(splat2(w1.x), dy[k], splat2(w0.w * dx));
                if constexpr (GEOM) {
                    dL_ddelx = __builtin_elementwise_fma(dL_dt, splat2(w1.z), dL_ddelx);
                    dL_ddely = __builtin_elementwise_fma(dL_dt, splat2(w1.w), dL_ddely);
                }
                // (the NDC scale W/2, H/2 of dL/dmean2D applied to the sums; |.| per pixel, scaled)
                fabs_sum = __builtin_fmaf(fabsf(dL_ddelx.x), ddelx_dx, fabs_sum);
                fabs_sum = __builtin_fmaf(fabsf(dL_ddely.x), ddely_dy, fabs_sum);
                fabs_sum = __builtin_fmaf(fabsf(dL_ddelx.y), ddelx_dx, fabs_sum);
                fabs_sum = __builtin_fmaf(fabsf(dL_ddely.y), ddely_dy, fabs_sum);
                const f2 qdy = q * dy[k], qdy2 = qdy * dy[k];
                Fmx = k ? Fmx + dL_ddelx : dL_ddelx;
                Fmy = k ? Fmy + dL_ddely : dL_ddely;
                Fq = k ? Fq + q : q;
                Fqdy = k ? Fqdy + qdy : qdy;
                Fqdy2 = k ? Fqdy2 + qdy2 : qdy2;
                Fp = k ? Fp + p : p;
            }
            float f[16];
            f[kAccColor + 0] = hsum(Fc0);
            f[kAccColor + 1] = hsum(Fc1);
            f[kAccColor + 2] = hsum(Fc2);
            // (the wave-uniform factors W/2, H/2 and -1/2 applied after the reduction: post_scale)
            f[kAccMean2D + 0] = hsum(Fmx);
            f[kAccMean2D + 1] = hsum(Fmy);
            f[kAccConic + 0] = hsum(Fq) * (dx * dx);
            f[kAccConic + 1] = hsum(Fqdy) * dx;
            f[kAccConic + 2] = hsum(Fqdy2);
            f[kAccConic + 3] = hsum(Fp);
            if constexpr (GEOM) {
                f[kAccNormal + 0] = hsum(Fn0);
                f[kAccNormal + 1] = hsum(Fn1);
                f[kAccNormal + 2] = hsum(Fn2);
                const float hdt = hsum(Fdt);
                f[kAccPlane + 0] = hdt * dx;
                f[kAccPlane + 1] = hsum(Fdtdy);
                f[kAccPlane + 2] = hdt;
                f[kAccPlane + 3] = hsum(Fdd);
            } else {
#pragma unroll
                for (int q = kAccNormal; q < kAccFields; q++) f[q] = 0.f;
            }
#ifndef GSR_TIME_BWD_PROBE
#define GSR_TIME_BWD_PROBE 0  // (timing builds only, gradients wrong: 1 = no reductions, 2 = no atomics)
#endif
#if GSR_TIME_BWD_PROBE == 1
            float red = f[0];
#pragma unroll
            for (int q = 1; q < 16; q++) red = (lane & 15) == q ? f[q] : red;
            red *= post_scale;
            const float abs_red = fabs_sum;
#else
            const float red = wave_transpose_reduce16(f) * post_scale;
            const float abs_red = wave_sum_dpp(fabs_sum);
#endif
            // (wave-uniform: the record's address in scalar registers, each lane's field an offset)
            const uint32_t g = __builtin_amdgcn_readfirstlane(s_id[j]);
            // lanes 0, 4, .., 60 add the 16 fields of the record (one 64-B line, one atomic
            // instruction), lane 1 adds |dmean2D|
            const bool field_lane = (lane & 3) == 0 && (GEOM || (lane >> 2) < kAccNormal);
#if GSR_TIME_BWD_PROBE == 2
            if (field_lane && red == 1234.5f && abs_red == 1.f && g == 7u) a.acc[lane] = red;
#else
            // one atomic instruction for both: as two, the |dmean2D| lane's uniform address made the
            // compiler wrap its atomic in the atomic optimizer's scalar lane loop on every step
            if (field_lane || lane == 1)
                atomicAdd(lane == 1 ? a.acc_abs + g : a.acc + (size_t)g * kAccFields + (lane >> 2),
                          lane == 1 ? abs_red : red);
#endif
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
    a.blend_mask = ts.blend_mask;
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
    a.no_cache = option(kOptBwdNoCache);
    a.tile_order = ws.tile_order;
    if (a.num_tiles == 0) return hipSuccess;
    // NP = 2: one wave per tile (the two-wave NP = 1 layout measured slower, see the kernel)
    if (p.require_depth)
        hipLaunchKernelGGL((render_bwd_kernel<true, 2>), dim3(a.num_tiles), dim3(64), 0, stream, a);
    else
        hipLaunchKernelGGL((render_bwd_kernel<false, 2>), dim3(a.num_tiles), dim3(64), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
