// preprocess_bwd.hip — per-Gaussian backward on gfx950.
//
// One fused kernel replaces BACKWARD::preprocess (render_backward.cu:1071-1161):
//   computeCov2DCUDA   (:249-656)  conic / Mip coef / ray-plane / normal -> cov3D -> scale, rot, mean
//   computeCov3D bwd   (:193-244)
//   preprocessCUDA bwd (:661-713)  screen-space mean -> mean3D, SH/SG colour backward (:56-191)
// It also writes the dL/dmeans2D and dL/dcolors extension outputs from the
// render-backward accumulator, so every gradient tensor is written exactly once
// with plain stores (zeros for culled Gaussians) and the host never memsets
// them (the reference zero-fills 11 tensors per backward,
// rasterize_points.cu:190-200).
//
// Reproduced reference behaviour that differs from the exact derivative of
// the forward (tests/torch_ref.py Q1, Q4): the normal backward scales by
// 1/|normalize(n)| (== 1); d rsigma / d(u, v) through vb is not propagated.
#include "gsr_kernels.h"
#include "gsr_math.h"

namespace gsr {

struct PreprocessBwdArgs {
    int P, D, SHM, SGD, SGM;
    const float* means3D;
    const float* opacities;
    const float* scales;
    const float* rotations;
    const float* cov3D_precomp;
    const float* shs;
    const float* sg_axis;
    const float* sg_sharpness;
    const float* sg_color;
    float scale_modifier;
    const float* view;
    const float* proj;
    const float* campos;
    float tan_fovx, tan_fovy, focal_x, focal_y, kernel_size;
    const int* radii;
    const uint8_t* clamped;
    const float* ddir;  // the forward's SH colour -> direction Jacobian, 9 planes of P (GeomState::ddir)
    const float* acc;
    const float* acc_abs;
    float* dL_dmean3D;
    float* dL_dmean2D;
    float* dL_dcolor;
    float* dL_dopacity;
    float* dL_dscale;
    float* dL_drot;
    float* dL_dcov3D;
    float* dL_dsh;
    float* dL_dsh_rest;  // split rows (BwdParams::dL_dsh_rest) or null
    float* dL_dsg_axis;
    float* dL_dsg_sharpness;
    float* dL_dsg_color;
    int begin, end;  // the Gaussians of this launch: [begin, end)
    // factored view-parallel mode (gsr_dist.OverlappedViewGrads): the DC row
    // dL/dsh[:, 0, :] goes to dc_rows [P][3] and no SH / SG gradient row is
    // written (gsr_view_color_grads_chunked rebuilds them from every view's DC rows)
    float* dc_rows;
};

// a Gaussian's SH gradient rows zeroed (one row, or the DC and rest rows of the split layout)
__device__ __forceinline__ void zero_sh_rows(const PreprocessBwdArgs& a, int idx) {
    if (!a.dL_dsh) return;
    if (a.dL_dsh_rest) {
        for (int k = 0; k < 3; k++) a.dL_dsh[(size_t)idx * 3 + k] = 0.f;
        for (int k = 0; k < 3 * (a.SHM - 1); k++) a.dL_dsh_rest[(size_t)idx * 3 * (a.SHM - 1) + k] = 0.f;
    } else {
        for (int k = 0; k < 3 * a.SHM; k++) a.dL_dsh[(size_t)idx * 3 * a.SHM + k] = 0.f;
    }
}

template <bool ROWS = true>
__device__ inline void zero_outputs(const PreprocessBwdArgs& a, int idx) {
    for (int k = 0; k < 3; k++) a.dL_dmean3D[3 * idx + k] = 0.f;
    a.dL_dopacity[idx] = 0.f;
    if (a.dL_dscale)
        for (int k = 0; k < 3; k++) a.dL_dscale[3 * idx + k] = 0.f;
    if (a.dL_drot)
        for (int k = 0; k < 4; k++) a.dL_drot[4 * idx + k] = 0.f;
    if (a.dL_dcov3D)
        for (int k = 0; k < 6; k++) a.dL_dcov3D[6 * idx + k] = 0.f;
    if (a.dc_rows) {
        for (int c = 0; c < 3; c++) a.dc_rows[3 * idx + c] = 0.f;
        return;
    }
    if (!ROWS) return;
    zero_sh_rows(a, idx);
    for (int k = 0; k < a.SGM; k++) {
        const size_t o = (size_t)idx * a.SGM + k;
        if (a.dL_dsg_sharpness) a.dL_dsg_sharpness[o] = 0.f;
        for (int c = 0; c < 3; c++) {
            if (a.dL_dsg_axis) a.dL_dsg_axis[3 * o + c] = 0.f;
            if (a.dL_dsg_color) a.dL_dsg_color[3 * o + c] = 0.f;
        }
    }
}

#ifndef GSR_SG_UNROLL
#define GSR_SG_UNROLL 1
#endif
// SG degree 7 (the configuration with SG lobes, BASELINE C5), all lobes of
// a Gaussian at once: its axis / colour / sharpness rows (21 + 21 + 7
// consecutive floats) are loaded and its gradient rows stored as wide
// contiguous accesses issued together, instead of 7 dependent iterations of
// 3-float pieces.  Same arithmetic in the same order as the generic loop.
constexpr int kSG7 = 7;
// (lobe rows move as unaligned 16-B pieces: load_row / store_row, gsr_math.h)
struct SG7Rows {
    float ax[3 * kSG7], gc[3 * kSG7], sharp[kSG7];
};
__device__ __forceinline__ void sg7_load(const PreprocessBwdArgs& a, int idx, SG7Rows& r) {
    const size_t o0 = (size_t)idx * kSG7;
    load_row(a.sg_axis + 3 * o0, r.ax);
    load_row(a.sg_color + 3 * o0, r.gc);
    load_row(a.sg_sharpness + o0, r.sharp);
}
// Staged rows (GSR_OPT_PBWD_STAGE): per wave, LDS rows for its 64 Gaussians
// in the global layout — the SG-7 lobe rows (colour 21, sharpness 7, axis 21
// floats each), loaded by LDS-DMA, replaced in place by their gradient rows
// and written out by wave_store_rows; then, reusing the space, the SH
// gradient rows (48 floats each).
constexpr int kStageColor = 0, kStageSharp = 64 * 21, kStageAxis = 64 * 28, kStageFloats = 64 * 49;
__device__ __forceinline__ void sg7_bwd(const PreprocessBwdArgs& a, int idx, const SG7Rows& rows, float x, float y,
                                        float z, float dR0, float dR1, float dR2, float& ddx, float& ddy, float& ddz) {
    const size_t o0 = (size_t)idx * kSG7;
    const float* ax = rows.ax;
    const float* gc = rows.gc;
    const float* sharp = rows.sharp;
    float dcol[3 * kSG7], dax[3 * kSG7], dsh[kSG7];
#pragma unroll
    for (int sg = 0; sg < kSG7; sg++) {
        const float* axs = ax + 3 * sg;
        const float* gcs = gc + 3 * sg;
        const float auxs = (axs[0] * x + axs[1] * y + axs[2] * z) - 1.0f;
        const float gs = expf(sharp[sg] * auxs);
        dcol[3 * sg + 0] = dR0 * gs;
        dcol[3 * sg + 1] = dR1 * gs;
        dcol[3 * sg + 2] = dR2 * gs;
        const float dL_dgs = gcs[0] * dR0 + gcs[1] * dR1 + gcs[2] * dR2;
        const float dL_dexp = dL_dgs * gs;
        dsh[sg] = dL_dexp * auxs;
        const float dL_daux = dL_dexp * sharp[sg];
        dax[3 * sg + 0] = dL_daux * x;
        dax[3 * sg + 1] = dL_daux * y;
        dax[3 * sg + 2] = dL_daux * z;
        ddx += dL_daux * axs[0];
        ddy += dL_daux * axs[1];
        ddz += dL_daux * axs[2];
    }
    if (a.dc_rows) return;  // (rows rebuilt by the view exchange)
    store_row(a.dL_dsg_color + 3 * o0, dcol);
    store_row(a.dL_dsg_sharpness + o0, dsh);
    store_row(a.dL_dsg_axis + 3 * o0, dax);
}

// (STAGE) SG-7 backward on the wave's LDS rows: slot `slot` of the lobe rows
// loaded by wave_load_rows; the gradient rows replace them in place (every
// input is read before the first write, in the same lockstep instructions).
__device__ __forceinline__ void sg7_bwd_slots(float* stage, int slot, float x, float y, float z, float dR0, float dR1,
                                              float dR2, float& ddx, float& ddy, float& ddz) {
    float* col = stage + kStageColor + 3 * kSG7 * slot;
    float* shp = stage + kStageSharp + kSG7 * slot;
    float* axs = stage + kStageAxis + 3 * kSG7 * slot;
    float dcol[3 * kSG7], dax[3 * kSG7], dsh[kSG7];
#pragma unroll
    for (int sg = 0; sg < kSG7; sg++) {
        const float a0 = axs[3 * sg], a1 = axs[3 * sg + 1], a2 = axs[3 * sg + 2];
        const float sharp = shp[sg];
        const float auxs = (a0 * x + a1 * y + a2 * z) - 1.0f;
        const float gs = expf(sharp * auxs);
        dcol[3 * sg + 0] = dR0 * gs;
        dcol[3 * sg + 1] = dR1 * gs;
        dcol[3 * sg + 2] = dR2 * gs;
        const float dL_dgs = col[3 * sg] * dR0 + col[3 * sg + 1] * dR1 + col[3 * sg + 2] * dR2;
        const float dL_dexp = dL_dgs * gs;
        dsh[sg] = dL_dexp * auxs;
        const float dL_daux = dL_dexp * sharp;
        dax[3 * sg + 0] = dL_daux * x;
        dax[3 * sg + 1] = dL_daux * y;
        dax[3 * sg + 2] = dL_daux * z;
        ddx += dL_daux * a0;
        ddy += dL_daux * a1;
        ddz += dL_daux * a2;
    }
#pragma unroll
    for (int k = 0; k < 3 * kSG7; k++) col[k] = dcol[k];
#pragma unroll
    for (int k = 0; k < kSG7; k++) shp[k] = dsh[k];
#pragma unroll
    for (int k = 0; k < 3 * kSG7; k++) axs[k] = dax[k];
}

// A wave's nf consecutive floats (rows of its Gaussians) into LDS by LDS-DMA
// (global_load_lds_dwordx4: one instruction moves 1 KB of consecutive bytes,
// no VGPR destination); the tail past the last whole 16-B piece by plain loads.
__device__ __forceinline__ void wave_load_rows(const float* __restrict__ g, float* l, int nf, int lane) {
    const int n4 = nf >> 2;
    for (int c0 = 0; c0 < n4; c0 += 64) {
        if (c0 + lane < n4)
            __builtin_amdgcn_global_load_lds((const void*)(g + 4 * (c0 + lane)),
                                             (__attribute__((address_space(3))) void*)(l + 4 * c0), 16, 0, 0);
    }
    for (int c = (n4 << 2) + lane; c < nf; c += 64) l[c] = g[c];
}

// A wave's n consecutive rows of nf floats each, staged in LDS in the
// global layout, written out as whole-wave 16-B pieces: one store
// instruction covers 1 KB of consecutive bytes instead of 64 rows.
// (GSR_PBWD_NT: non-temporal stores — the gradient rows are read next by the optimizer step, after the
// whole backward has streamed through the caches)
#ifndef GSR_PBWD_NT
#define GSR_PBWD_NT 1
#endif
typedef float pbwd_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void wave_store_rows(float* __restrict__ g, const float* __restrict__ l, int nf, int lane) {
    const int n4 = nf >> 2;
    for (int c = lane; c < n4; c += 64) {
        if constexpr (GSR_PBWD_NT)
            __builtin_nontemporal_store(reinterpret_cast<const pbwd_f4*>(l)[c], reinterpret_cast<pbwd_f4*>(g) + c);
        else
            reinterpret_cast<float4*>(g)[c] = reinterpret_cast<const float4*>(l)[c];
    }
    for (int c = (n4 << 2) + lane; c < nf; c += 64) g[c] = l[c];
}

#ifndef GSR_PBWD_WAVES
#define GSR_PBWD_WAVES 0
#endif
#ifndef GSR_PBWD_STAGE_WAVES
#define GSR_PBWD_STAGE_WAVES 3
#endif
#ifndef GSR_PBWD_STAGE_DEFAULT
#define GSR_PBWD_STAGE_DEFAULT 1  // staged row stores: C5 preprocess_bwd 1.18-1.22 -> 0.91-0.93 ms, C3 0.151 -> 0.122
#endif
// STAGE (SH rows of 16 coefficients, launch ranges in whole workgroups): the
// SH and SG-7 gradient rows go out through LDS as whole-wave stores (and the
// SG-7 input rows come in by 16-B LDS-DMA).  Every lane of a wave then takes
// part, so a lane past the range computes the wave's first Gaussian (`wbase`)
// again (same values to the same addresses) and only its staged rows are left out.
template <bool STAGE>
#if GSR_PBWD_WAVES
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSR_PBWD_WAVES, 8)))
preprocess_bwd_kernel(PreprocessBwdArgs a) {
#else
// (STAGE: the lobe rows live in LDS, not VGPRs: 3 waves per SIMD fit (168 VGPRs, 6 spilled); LDS 49 KB
// per block, 3 blocks per CU)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(STAGE ? GSR_PBWD_STAGE_WAVES : 1, 8)))
preprocess_bwd_kernel(PreprocessBwdArgs a) {
#endif
    const int idx0 = a.begin + blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const int wbase = idx0 - lane;  // the wave's first Gaussian
    if (!STAGE && idx0 >= a.end) return;
    if (STAGE && wbase >= a.end) return;  // (a whole wave past the range takes no part in anything)
    // (STAGE: a lane past the range duplicates the wave's first Gaussian: same values, same addresses)
    const int idx = idx0 < a.end ? idx0 : (STAGE ? wbase : a.begin);
    const int slot = idx - wbase;  // (STAGE) the Gaussian's row slot in the wave's LDS rows
    __shared__ float s_stage[STAGE ? 4 * kStageFloats : 1];
    float* stage = s_stage + (STAGE ? (threadIdx.x >> 6) * kStageFloats : 0);
    // (STAGE) what the SH rows need, left by the visible-Gaussian body: direction and clamp-masked dL/dRGB
    float st_x = 0.f, st_y = 0.f, st_z = 0.f, st_d0 = 0.f, st_d1 = 0.f, st_d2 = 0.f;
    bool culled = false;
    // every per-Gaussian input row is requested up front, before the culled
    // test and the dependent chains (one memory round trip instead of one per
    // phase; the kernel is latency-bound)
    float acc[kAccFields];
    {
        const float4* a4 = reinterpret_cast<const float4*>(a.acc + (size_t)idx * kAccFields);  // 64-B records
#pragma unroll
        for (int k = 0; k < kAccFields / 4; k++) {
            const float4 v = a4[k];
            acc[4 * k] = v.x;
            acc[4 * k + 1] = v.y;
            acc[4 * k + 2] = v.z;
            acc[4 * k + 3] = v.w;
        }
    }
    const int radius = a.radii[idx];
    const float mx = a.means3D[3 * idx], my = a.means3D[3 * idx + 1], mz = a.means3D[3 * idx + 2];
    const float opacity = a.opacities[idx];
    float sc_in[3] = {0.f, 0.f, 0.f}, q_in[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.scales) {
        sc_in[0] = a.scales[3 * idx];
        sc_in[1] = a.scales[3 * idx + 1];
        sc_in[2] = a.scales[3 * idx + 2];
        const float4 q4 = *reinterpret_cast<const float4*>(a.rotations + 4 * idx);
        q_in[0] = q4.x;
        q_in[1] = q4.y;
        q_in[2] = q4.z;
        q_in[3] = q4.w;
    }
#if GSR_SG_UNROLL
    // (SG degree 7: the 196-B lobe rows as well; 2 waves per SIMD fit them)
    const bool sg7 = a.shs && a.SGM == kSG7 && a.SGD == kSG7;
    SG7Rows sgr;
    if (STAGE && sg7) {  // the wave's lobe rows into its LDS slots, by LDS-DMA (read after the geometry chain)
        const int n = min(64, a.end - wbase);
        const size_t o = (size_t)wbase * kSG7;
        wave_load_rows(a.sg_color + 3 * o, stage + kStageColor, n * 3 * kSG7, lane);
        wave_load_rows(a.sg_sharpness + o, stage + kStageSharp, n * kSG7, lane);
        wave_load_rows(a.sg_axis + 3 * o, stage + kStageAxis, n * 3 * kSG7, lane);
    } else if (sg7) {
        sg7_load(a, idx, sgr);
    }
#endif
    // extension outputs straight from the accumulator (zero for culled
    // Gaussians); sample_depth returns neither (rasterize_points.cu:633)
    if (a.dL_dmean2D) {
        a.dL_dmean2D[3 * idx + 0] = acc[kAccMean2D + 0];
        a.dL_dmean2D[3 * idx + 1] = acc[kAccMean2D + 1];
        a.dL_dmean2D[3 * idx + 2] = a.acc_abs[idx];
    }
    if (a.dL_dcolor) {
        a.dL_dcolor[3 * idx + 0] = acc[kAccColor + 0];
        a.dL_dcolor[3 * idx + 1] = acc[kAccColor + 1];
        a.dL_dcolor[3 * idx + 2] = acc[kAccColor + 2];
    }
    if (!(radius > 0)) {
        if constexpr (!STAGE) {
            zero_outputs(a, idx);
            return;
        }
        zero_outputs<false>(a, idx);  // (rows: zero slots in the staged stores below)
        culled = true;
    }
    auto visible = [&]() {
    const float fx = a.focal_x, fy = a.focal_y;
    const float* V = a.view;
    const float dconx = acc[kAccConic + 0], dcony = acc[kAccConic + 1], dconz = acc[kAccConic + 2],
                dconw = acc[kAccConic + 3];
    const float dnx = acc[kAccNormal + 0], dny = acc[kAccNormal + 1], dnz = acc[kAccNormal + 2];
    const float drpx = acc[kAccPlane + 0] / fx, drpy = acc[kAccPlane + 1] / fy;
    const float dL_dtc = acc[kAccPlane + 2], dL_drsig = acc[kAccPlane + 3];

    // ---------------- computeCov2DCUDA ----------------
    const ViewGeom g = view_geom(V, mx, my, mz, a.tan_fovx, a.tan_fovy);
    const float rtc = 1.0f / sqrtf(g.t[0] * g.t[0] + g.t[1] * g.t[1] + g.t[2] * g.t[2]);
    const float dtc_x = g.t[0] * rtc * dL_dtc, dtc_y = g.t[1] * rtc * dL_dtc, dtc_z = g.t[2] * rtc * dL_dtc;
    const float xgm = g.clamp_x ? 0.f : 1.f, ygm = g.clamp_y ? 0.f : 1.f;
    const float u = g.u, v = g.v, tz = g.tz, tx = g.tx, ty = g.ty;
    const float j00 = fx / tz, j02 = -(fx * tx) / (tz * tz);
    const float j11 = fy / tz, j12 = -(fy * ty) / (tz * tz);
    float Wr[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) Wr[3 * i + j] = V[4 * j + i];
    // Q = J W_r rows (glm T[0][k] = Q0[k], T[1][k] = Q1[k])
    float Q0[3], Q1[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        Q0[k] = j00 * Wr[k] + j02 * Wr[6 + k];
        Q1[k] = j11 * Wr[3 + k] + j12 * Wr[6 + k];
    }
    float Vrk[9], Vinv[9], Rq[9], s[3] = {0.f, 0.f, 0.f};
    float evl[3] = {0.f, 0.f, 0.f}, EV[9];
    bool well_conditioned = true;
    if (a.scales) {
        s[0] = a.scale_modifier * sc_in[0];
        s[1] = a.scale_modifier * sc_in[1];
        s[2] = a.scale_modifier * sc_in[2];
        const float* q = q_in;
        float A_unused[9];
        rot_view(V, q[0], q[1], q[2], q[3], A_unused, Rq);
        const float s2[3] = {s[0] * s[0], s[1] * s[1], s[2] * s[2]};
        const float is2[3] = {1.0f / s2[0], 1.0f / s2[1], 1.0f / s2[2]};
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) {
                Vrk[3 * i + j] = Rq[3 * i] * Rq[3 * j] * s2[0] + Rq[3 * i + 1] * Rq[3 * j + 1] * s2[1] +
                                 Rq[3 * i + 2] * Rq[3 * j + 2] * s2[2];
                Vinv[3 * i + j] = Rq[3 * i] * Rq[3 * j] * is2[0] + Rq[3 * i + 1] * Rq[3 * j + 1] * is2[1] +
                                  Rq[3 * i + 2] * Rq[3 * j + 2] * is2[2];
            }
    } else {
        const float* c = a.cov3D_precomp + 6 * idx;
        const float Vk[9] = {c[0], c[1], c[2], c[1], c[3], c[4], c[2], c[4], c[5]};
#pragma unroll
        for (int k = 0; k < 9; k++) Vrk[k] = Vk[k];
        sym3_eigen(Vk, evl, EV);
        well_conditioned = evl[0] > 1e-8f;
        if (well_conditioned) {
            const float il[3] = {1.0f / evl[0], 1.0f / evl[1], 1.0f / evl[2]};
#pragma unroll
            for (int i = 0; i < 3; i++)
#pragma unroll
                for (int j = 0; j < 3; j++)
                    Vinv[3 * i + j] = EV[i] * EV[j] * il[0] + EV[3 + i] * EV[3 + j] * il[1] + EV[6 + i] * EV[6 + j] * il[2];
        } else {
#pragma unroll
            for (int i = 0; i < 3; i++)
#pragma unroll
                for (int j = 0; j < 3; j++) Vinv[3 * i + j] = EV[i] * EV[j];
        }
    }
    // cov2D = Q Vrk Q^T (no kernel), cov_cam_inv = W_r Vinv W_r^T
    float VQ0[3], VQ1[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
        VQ0[i] = Vrk[3 * i] * Q0[0] + Vrk[3 * i + 1] * Q0[1] + Vrk[3 * i + 2] * Q0[2];
        VQ1[i] = Vrk[3 * i] * Q1[0] + Vrk[3 * i + 1] * Q1[1] + Vrk[3 * i + 2] * Q1[2];
    }
    const float c00 = Q0[0] * VQ0[0] + Q0[1] * VQ0[1] + Q0[2] * VQ0[2];
    const float c01 = Q0[0] * VQ1[0] + Q0[1] * VQ1[1] + Q0[2] * VQ1[2];
    const float c11 = Q1[0] * VQ1[0] + Q1[1] * VQ1[1] + Q1[2] * VQ1[2];
    float WV[9], cinv[9];
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
    const float ks = a.kernel_size;
    const float det_0 = fmaxf(1e-6f, c00 * c11 - c01 * c01);
    const float det_1 = fmaxf(1e-6f, (c00 + ks) * (c11 + ks) - c01 * c01);
    const float coef = sqrtf(det_0 / det_1);

    // ray-plane / normal backward (render_backward.cu:425-545)
    const float m0 = cinv[0] * u + cinv[1] * v + cinv[2];
    const float m1 = cinv[3] * u + cinv[4] * v + cinv[5];
    const float m2 = cinv[6] * u + cinv[7] * v + cinv[8];
    const float vb = m0 * u + m1 * v + m2;
    const float u2 = u * u, v2 = v * v, uv = u * v;
    const float l = sqrtf(tx * tx + ty * ty + tz * tz);
    const float clamp_vb = fmaxf(vb, 1e-7f);
    const float rl2 = u2 + v2 + 1.f;
    const float rl_inv = __builtin_amdgcn_rsqf(rl2);
    const float fn = l / rl2;
    const float mv0 = m0 / clamp_vb, mv1 = m1 / clamp_vb, mv2 = m2 / clamp_vb;  // uvh_m / vb
    const float plx = (v2 + 1.f) * mv0 - uv * mv1 - u * mv2;
    const float ply = -uv * mv0 + (u2 + 1.f) * mv1 - v * mv2;
    const float rn0 = -plx * fn, rn1 = -ply * fn, rn2 = -1.f;
    const float itz = 1.f / tz, il = 1.f / l;
    const float cn0 = rn0 * itz + tx * il * rn2;
    const float cn1 = rn1 * itz + ty * il * rn2;
    const float cn2 = -(tx * itz * itz) * rn0 - (ty * itz * itz) * rn1 + tz * il * rn2;
    const float icn = 1.0f / sqrtf(cn0 * cn0 + cn1 * cn1 + cn2 * cn2);
    const float nv0 = cn0 * icn, nv1 = cn1 * icn, nv2 = cn2 * icn;
    const float rlv = 1.0f / sqrtf(nv0 * nv0 + nv1 * nv1 + nv2 * nv2);  // == 1 (reference quirk Q1)
    const float ndot = nv0 * dnx + nv1 * dny + nv2 * dnz;
    const float dc0 = (dnx - nv0 * ndot) * rlv, dc1 = (dny - nv1 * ndot) * rlv, dc2 = (dnz - nv2 * ndot) * rlv;
    // dL/d rnv = nJ^T dL/dcam_n ; nJ rows (1/tz, 0, tx/l), (0, 1/tz, ty/l), (-tx/tz^2, -ty/tz^2, tz/l)
    const float drn0 = dc0 * itz - dc2 * tx * itz * itz;
    const float drn1 = dc1 * itz - dc2 * ty * itz * itz;
    // dL_dnJ (glm [i][j] = dc[j] * rn[i])
    const float aux_nJ = (-(dc0 * rn2) * u - (dc1 * rn2) * v - dc2 * rn2) / rl2 * rl_inv;
    const float du_nJ = -(dc2 * rn0) / tz + (dc0 * rn2) * rl_inv + aux_nJ * u;
    const float dv_nJ = -(dc2 * rn1) / tz + (dc1 * rn2) * rl_inv + aux_nJ * v;
    const float dz_nJ = ((dc0 * rn0) + (dc1 * rn1) - (dc2 * rn0) * u - (dc2 * rn1) * v) / (-tz * tz);
    const float e0 = -drn0 + drpx, e1 = -drn1 + drpy;
    const float dL_dfn = plx * e0 + ply * e1;
    const float dpx = e0 * fn, dpy = e1 * fn;
    const float aux = dpx * plx + dpy * ply;
    // nJ_inv^T dpa, nJ_inv rows (v2+1, -uv, -u), (-uv, u2+1, -v), 0
    const float nt0 = (v2 + 1.f) * dpx - uv * dpy;
    const float nt1 = -uv * dpx + (u2 + 1.f) * dpy;
    const float nt2 = -u * dpx - v * dpy;
    const float icvb = 1.0f / clamp_vb;
    const float duvh0 = 2.f * (-aux) * mv0 + (cinv[0] * nt0 + cinv[1] * nt1 + cinv[2] * nt2) * icvb;
    const float duvh1 = 2.f * (-aux) * mv1 + (cinv[3] * nt0 + cinv[4] * nt1 + cinv[5] * nt2) * icvb;
    const float rsigmat = sqrtf(vb / rl2);
    const float drl2_sig = -dL_drsig * rsigmat / rl2;
    // dL_dnJ_inv glm [i][j] = dpa[j] * mv[i]
    const float E01 = dpy * mv0, E10 = dpx * mv1, E11 = dpy * mv1, E20 = dpx * mv2, E00 = dpx * mv0, E21 = dpy * mv2;
    const float du_plane = duvh0 + (E01 + E10) * (-v) + 2.f * E11 * u - E20;
    const float dv_plane = duvh1 + (E01 + E10) * (-u) + 2.f * E00 * v - E21;
    const float aux_f = dL_dfn * (-tz / rl2 * rl_inv);
    const float dL_du = du_nJ + du_plane + aux_f * u + drl2_sig * u;
    const float dL_dv = dv_nJ + dv_plane + aux_f * v + drl2_sig * v;
    const float dL_dz = dz_nJ + dL_dfn * rl_inv;
    const float dvbx = -aux + dL_drsig * 0.5f * rsigmat;
    // W_uvh = W_r^T uvh ; W nJ_inv^T dpa = W_r^T nt
    float Wu[3], Wn[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        Wu[k] = Wr[k] * u + Wr[3 + k] * v + Wr[6 + k];
        Wn[k] = Wr[k] * nt0 + Wr[3 + k] * nt1 + Wr[6 + k] * nt2;
    }
    float dVrk[9];  // glm layout dVrk[3*i + j] = dL_dVrk[i][j]
    float dLr[3] = {0.f, 0.f, 0.f};
    if (well_conditioned) {
        float av[3], bv[3];
#pragma unroll
        for (int i = 0; i < 3; i++) {
            av[i] = Vinv[3 * i] * Wu[0] + Vinv[3 * i + 1] * Wu[1] + Vinv[3 * i + 2] * Wu[2];
            const float r0 = Wn[0] + Wu[0] * dvbx, r1 = Wn[1] + Wu[1] * dvbx, r2 = Wn[2] + Wu[2] * dvbx;
            bv[i] = Vinv[3 * i] * r0 + Vinv[3 * i + 1] * r1 + Vinv[3 * i + 2] * r2;
        }
        // -outerProduct(av, bv) / vb : glm [i][j] = -av[j] * bv[i] / vb
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) dVrk[3 * i + j] = -(av[j] * bv[i]) / vb;
    } else {
#pragma unroll
        for (int k = 0; k < 9; k++) dVrk[k] = 0.f;
        float rv[3];
#pragma unroll
        for (int k = 0; k < 3; k++) rv[k] = Wu[k] * dvbx + Wn[k];
        // S = dL_dVrk_inv + transpose (symmetric), dL_dv = S e_min
        const float* em = EV;  // eigenvector of the smallest eigenvalue
        float dLdv[3];
#pragma unroll
        for (int i = 0; i < 3; i++) {
            float acc_i = 0.f;
#pragma unroll
            for (int j = 0; j < 3; j++) acc_i += ((Wu[i] * rv[j] + Wu[j] * rv[i]) / vb) * em[j];
            dLdv[i] = acc_i;
        }
        if (a.scales) {
            // R[min_id] with well_conditioned always true on this path (kept for completeness)
        } else {
#pragma unroll
            for (int kk = 1; kk < 3; kk++) {
                const float* ek = EV + 3 * kk;
                const float sc = (ek[0] * dLdv[0] + ek[1] * dLdv[1] + ek[2] * dLdv[2]) / fminf(evl[0] - evl[kk], -1e-7f);
#pragma unroll
                for (int i = 0; i < 3; i++)
#pragma unroll
                    for (int j = 0; j < 3; j++) dVrk[3 * i + j] += (ek[j] * sc) * em[i];
            }
        }
    }
    // conic / coefficient backward (render_backward.cu:547-579)
    const float dL_dcoef = dconw * opacity;
    const float dL_dsqrtcoef = dL_dcoef * 0.5f / (coef + 1e-6f);
    const float dL_ddet0 = dL_dsqrtcoef / det_1;
    const float dL_ddet1 = -dL_ddet0 * coef;
    const float dcoef_da = dL_ddet0 * c11 + dL_ddet1 * (c11 + ks);
    const float dcoef_db = (-2.f * c01) * (dL_ddet0 + dL_ddet1);
    const float dcoef_dc = dL_ddet0 * c00 + dL_ddet1 * (c00 + ks);
    const float ca = c00 + ks, cb = c01, cc = c11 + ks;
    const float denom = ca * cc - cb * cb;
    const float denom2inv = 1.0f / ((denom * denom) + 1e-7f);
    float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
    float dcl[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float dopa = 0.f;
    if (denom2inv != 0.f) {
        dL_da = denom2inv * (-cc * cc * dconx + 2 * cb * cc * dcony + (denom - ca * cc) * dconz);
        dL_dc = denom2inv * (-ca * ca * dconz + 2 * ca * cb * dcony + (denom - ca * cc) * dconx);
        dL_db = denom2inv * 2 * (cb * cc * dconx - (denom + 2 * cb * cb) * dcony + ca * cb * dconz);
        dL_da += dcoef_da;
        dL_dc += dcoef_dc;
        dL_db += dcoef_db;
        dopa = dconw * coef;
        dcl[0] = Q0[0] * Q0[0] * dL_da + Q0[0] * Q1[0] * dL_db + Q1[0] * Q1[0] * dL_dc;
        dcl[3] = Q0[1] * Q0[1] * dL_da + Q0[1] * Q1[1] * dL_db + Q1[1] * Q1[1] * dL_dc;
        dcl[5] = Q0[2] * Q0[2] * dL_da + Q0[2] * Q1[2] * dL_db + Q1[2] * Q1[2] * dL_dc;
        dcl[1] = 2 * Q0[0] * Q0[1] * dL_da + (Q0[0] * Q1[1] + Q0[1] * Q1[0]) * dL_db + 2 * Q1[0] * Q1[1] * dL_dc;
        dcl[2] = 2 * Q0[0] * Q0[2] * dL_da + (Q0[0] * Q1[2] + Q0[2] * Q1[0]) * dL_db + 2 * Q1[0] * Q1[2] * dL_dc;
        dcl[4] = 2 * Q0[2] * Q0[1] * dL_da + (Q0[1] * Q1[2] + Q0[2] * Q1[1]) * dL_db + 2 * Q1[1] * Q1[2] * dL_dc;
    }
    a.dL_dopacity[idx] = dopa;
    dcl[0] += dVrk[0];
    dcl[3] += dVrk[4];
    dcl[5] += dVrk[8];
    dcl[1] += dVrk[1] + dVrk[3];
    dcl[2] += dVrk[2] + dVrk[6];
    dcl[4] += dVrk[5] + dVrk[7];

    if (a.scales) {
        // computeCov3D backward (render_backward.cu:193-244), math layout:
        // R_m = R_q^T, M = S R_m, dL/dM = 2 M G, d[i][j] = dL/dR_m[i][j]
        const float G[9] = {dcl[0], 0.5f * dcl[1], 0.5f * dcl[2], 0.5f * dcl[1], dcl[3],
                            0.5f * dcl[4], 0.5f * dcl[2], 0.5f * dcl[4], dcl[5]};
        float Rm[9];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) Rm[3 * i + j] = Rq[3 * j + i];
        float d[9], dsc[3];
#pragma unroll
        for (int i = 0; i < 3; i++) {
            float dM[3];
#pragma unroll
            for (int j = 0; j < 3; j++)
                dM[j] = 2.0f * s[i] * (Rm[3 * i] * G[j] + Rm[3 * i + 1] * G[3 + j] + Rm[3 * i + 2] * G[6 + j]);
            dsc[i] = Rm[3 * i] * dM[0] + Rm[3 * i + 1] * dM[1] + Rm[3 * i + 2] * dM[2];
#pragma unroll
            for (int j = 0; j < 3; j++) d[3 * i + j] = dM[j] * s[i];
        }
        (void)dLr;
        a.dL_dscale[3 * idx] = dsc[0];
        a.dL_dscale[3 * idx + 1] = dsc[1];
        a.dL_dscale[3 * idx + 2] = dsc[2];
        const float* q = q_in;
        const float r = q[0], x = q[1], y = q[2], z = q[3];
#define D_(i, j) d[3 * (i) + (j)]
        a.dL_drot[4 * idx + 0] = 2 * z * (D_(0, 1) - D_(1, 0)) + 2 * y * (D_(2, 0) - D_(0, 2)) + 2 * x * (D_(1, 2) - D_(2, 1));
        a.dL_drot[4 * idx + 1] = 2 * y * (D_(1, 0) + D_(0, 1)) + 2 * z * (D_(2, 0) + D_(0, 2)) +
                                 2 * r * (D_(1, 2) - D_(2, 1)) - 4 * x * (D_(2, 2) + D_(1, 1));
        a.dL_drot[4 * idx + 2] = 2 * x * (D_(1, 0) + D_(0, 1)) + 2 * r * (D_(2, 0) - D_(0, 2)) +
                                 2 * z * (D_(1, 2) + D_(2, 1)) - 4 * y * (D_(2, 2) + D_(0, 0));
        a.dL_drot[4 * idx + 3] = 2 * r * (D_(0, 1) - D_(1, 0)) + 2 * x * (D_(2, 0) + D_(0, 2)) +
                                 2 * y * (D_(1, 2) + D_(2, 1)) - 4 * z * (D_(1, 1) + D_(0, 0));
#undef D_
        if (a.dL_dcov3D)
            for (int k = 0; k < 6; k++) a.dL_dcov3D[6 * idx + k] = 0.f;
    } else {
        for (int k = 0; k < 6; k++) a.dL_dcov3D[6 * idx + k] = dcl[k];
        if (a.dL_dscale)
            for (int k = 0; k < 3; k++) a.dL_dscale[3 * idx + k] = 0.f;
        if (a.dL_drot)
            for (int k = 0; k < 4; k++) a.dL_drot[4 * idx + k] = 0.f;
    }

    // dL/dT -> dL/dJ -> dL/dt (render_backward.cu:613-646)
    float dQ0[3], dQ1[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float vq0 = Vrk[3 * k] * Q0[0] + Vrk[3 * k + 1] * Q0[1] + Vrk[3 * k + 2] * Q0[2];
        const float vq1 = Vrk[3 * k] * Q1[0] + Vrk[3 * k + 1] * Q1[1] + Vrk[3 * k + 2] * Q1[2];
        dQ0[k] = 2 * vq0 * dL_da + vq1 * dL_db;
        dQ1[k] = 2 * vq1 * dL_dc + vq0 * dL_db;
    }
    const float dJ00 = Wr[0] * dQ0[0] + Wr[1] * dQ0[1] + Wr[2] * dQ0[2];
    const float dJ02 = Wr[6] * dQ0[0] + Wr[7] * dQ0[1] + Wr[8] * dQ0[2];
    const float dJ11 = Wr[3] * dQ1[0] + Wr[4] * dQ1[1] + Wr[5] * dQ1[2];
    const float dJ12 = Wr[6] * dQ1[0] + Wr[7] * dQ1[1] + Wr[8] * dQ1[2];
    const float tz1 = 1.f / tz, tz2 = tz1 * tz1, tz3 = tz2 * tz1;
    const float dtx = xgm * (-fx * tz2 * dJ02 + dL_du * tz1);
    const float dty = ygm * (-fy * tz2 * dJ12 + dL_dv * tz1);
    const float dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + ((1 + xgm) * fx * tx) * tz3 * dJ02 +
                      ((1 + ygm) * fy * ty) * tz3 * dJ12 - (xgm * dL_du * tx + ygm * dL_dv * ty) * tz2 + dL_dz;
    const float gx_ = dtx + dtc_x, gy_ = dty + dtc_y, gz_ = dtz + dtc_z;
    float dm0 = V[0] * gx_ + V[1] * gy_ + V[2] * gz_;
    float dm1 = V[4] * gx_ + V[5] * gy_ + V[6] * gz_;
    float dm2 = V[8] * gx_ + V[9] * gy_ + V[10] * gz_;

    // ---------------- preprocessCUDA backward: screen-space mean ----------------
    const float* Pm = a.proj;
    const float hw = Pm[3] * mx + Pm[7] * my + Pm[11] * mz + Pm[15];
    const float m_w = 1.0f / (hw + 0.0000001f);
    const float mul1 = (Pm[0] * mx + Pm[4] * my + Pm[8] * mz + Pm[12]) * m_w * m_w;
    const float mul2 = (Pm[1] * mx + Pm[5] * my + Pm[9] * mz + Pm[13]) * m_w * m_w;
    const float g2x = acc[kAccMean2D + 0], g2y = acc[kAccMean2D + 1];
    dm0 += (Pm[0] * m_w - Pm[3] * mul1) * g2x + (Pm[1] * m_w - Pm[3] * mul2) * g2y;
    dm1 += (Pm[4] * m_w - Pm[7] * mul1) * g2x + (Pm[5] * m_w - Pm[7] * mul2) * g2y;
    dm2 += (Pm[8] * m_w - Pm[11] * mul1) * g2x + (Pm[9] * m_w - Pm[11] * mul2) * g2y;

    // ---------------- SH / SG colour backward ----------------
    if (a.shs) {
        // the forward's colour -> direction Jacobian (9 coalesced plane loads instead of the 192-B SH row)
        float jd[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (a.D > 0) {
#pragma unroll
            for (int j = 0; j < 9; j++) jd[j] = a.ddir[(size_t)j * a.P + idx];
        }
        const float dox = mx - a.campos[0], doy = my - a.campos[1], doz = mz - a.campos[2];
        const float dlen = sqrtf(dox * dox + doy * doy + doz * doz);
        const float x = dox / dlen, y = doy / dlen, z = doz / dlen;
        const uint8_t cl = a.clamped[idx];
        const float dR0 = (cl & 1) ? 0.f : acc[kAccColor + 0];
        const float dR1 = (cl & 2) ? 0.f : acc[kAccColor + 1];
        const float dR2 = (cl & 4) ? 0.f : acc[kAccColor + 2];
        float Y[16];
        sh_basis(a.D, x, y, z, Y);
        const int n = sh_count(a.D);
        if (STAGE) {  // the row is written by the staged stores
            st_x = x, st_y = y, st_z = z, st_d0 = dR0, st_d1 = dR1, st_d2 = dR2;
        } else if (a.dc_rows) {  // the DC row as store_sh_grad writes it (Y[0] dR)
            a.dc_rows[3 * idx] = Y[0] * dR0;
            a.dc_rows[3 * idx + 1] = Y[0] * dR1;
            a.dc_rows[3 * idx + 2] = Y[0] * dR2;
        } else if (a.dL_dsh_rest) {
            store_sh_grad_split(a.dL_dsh + (size_t)idx * 3, a.dL_dsh_rest + (size_t)idx * (a.SHM - 1) * 3, a.SHM, n, Y,
                                dR0, dR1, dR2);
        } else {
            store_sh_grad(a.dL_dsh + (size_t)idx * a.SHM * 3, a.SHM, n, Y, dR0, dR1, dR2);
        }
        // d(colour)/d(dir) per channel (render_backward.cu:94-153): the forward's
        // Jacobian planes (gsr_math.h sh_basis_grad)
        const float gdx[3] = {jd[0], jd[3], jd[6]}, gdy[3] = {jd[1], jd[4], jd[7]}, gdz[3] = {jd[2], jd[5], jd[8]};
        float ddx = gdx[0] * dR0 + gdx[1] * dR1 + gdx[2] * dR2;
        float ddy = gdy[0] * dR0 + gdy[1] * dR1 + gdy[2] * dR2;
        float ddz = gdz[0] * dR0 + gdz[1] * dR1 + gdz[2] * dR2;
#if GSR_SG_UNROLL
        if (sg7) {
            if constexpr (STAGE) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA row loads have landed
                sg7_bwd_slots(stage, slot, x, y, z, dR0, dR1, dR2, ddx, ddy, ddz);
            } else {
                sg7_bwd(a, idx, sgr, x, y, z, dR0, dR1, dR2, ddx, ddy, ddz);
            }
        } else
#endif
        for (int sg = 0; sg < a.SGM; sg++) {
            const size_t o = (size_t)idx * a.SGM + sg;
            if (sg >= a.SGD) {
                if (a.dc_rows) continue;
                a.dL_dsg_sharpness[o] = 0.f;
                for (int c = 0; c < 3; c++) {
                    a.dL_dsg_axis[3 * o + c] = 0.f;
                    a.dL_dsg_color[3 * o + c] = 0.f;
                }
                continue;
            }
            const float* ax = a.sg_axis + 3 * o;
            const float* gc = a.sg_color + 3 * o;
            const float sharp = a.sg_sharpness[o];
            const float auxs = (ax[0] * x + ax[1] * y + ax[2] * z) - 1.0f;
            const float gs = expf(sharp * auxs);
            const float dL_dgs = gc[0] * dR0 + gc[1] * dR1 + gc[2] * dR2;
            const float dL_dexp = dL_dgs * gs;
            const float dL_daux = dL_dexp * sharp;
            if (!a.dc_rows) {
                a.dL_dsg_color[3 * o + 0] = dR0 * gs;
                a.dL_dsg_color[3 * o + 1] = dR1 * gs;
                a.dL_dsg_color[3 * o + 2] = dR2 * gs;
                a.dL_dsg_sharpness[o] = dL_dexp * auxs;
                a.dL_dsg_axis[3 * o + 0] = dL_daux * x;
                a.dL_dsg_axis[3 * o + 1] = dL_daux * y;
                a.dL_dsg_axis[3 * o + 2] = dL_daux * z;
            }
            ddx += dL_daux * ax[0];
            ddy += dL_daux * ax[1];
            ddz += dL_daux * ax[2];
        }
        // dnormvdv (auxiliary.h:104-113)
        const float inv = 1.0f / dlen;
        const float vx = dox * inv, vy = doy * inv, vz = doz * inv;
        dm0 += ((1.f - vx * vx) * ddx - vy * vx * ddy - vz * vx * ddz) * inv;
        dm1 += (-vx * vy * ddx + (1.f - vy * vy) * ddy - vz * vy * ddz) * inv;
        dm2 += (-vx * vz * ddx - vy * vz * ddy + (1.f - vz * vz) * ddz) * inv;
    } else {
        for (int sg = 0; sg < a.SGM; sg++) {
            const size_t o = (size_t)idx * a.SGM + sg;
            if (a.dL_dsg_sharpness) a.dL_dsg_sharpness[o] = 0.f;
            for (int c = 0; c < 3; c++) {
                if (a.dL_dsg_axis) a.dL_dsg_axis[3 * o + c] = 0.f;
                if (a.dL_dsg_color) a.dL_dsg_color[3 * o + c] = 0.f;
            }
        }
        zero_sh_rows(a, idx);
    }
    a.dL_dmean3D[3 * idx] = dm0;
    a.dL_dmean3D[3 * idx + 1] = dm1;
    a.dL_dmean3D[3 * idx + 2] = dm2;
    };
    if (!culled) visible();
    if constexpr (STAGE) {
        // the wave's Gaussians [wbase, wbase + n): rows in LDS, then whole-wave stores
        const int n = min(64, a.end - wbase);
        if (sg7) {
            if (culled) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the DMA must not land after the zeros)
#pragma unroll
                for (int k = 0; k < 3 * kSG7; k++) {
                    stage[kStageColor + 3 * kSG7 * slot + k] = 0.f;
                    stage[kStageAxis + 3 * kSG7 * slot + k] = 0.f;
                }
#pragma unroll
                for (int k = 0; k < kSG7; k++) stage[kStageSharp + kSG7 * slot + k] = 0.f;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const size_t o = (size_t)wbase * kSG7;
            wave_store_rows(a.dL_dsg_color + 3 * o, stage + kStageColor, n * 3 * kSG7, lane);
            wave_store_rows(a.dL_dsg_sharpness + o, stage + kStageSharp, n * kSG7, lane);
            wave_store_rows(a.dL_dsg_axis + 3 * o, stage + kStageAxis, n * 3 * kSG7, lane);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // SH rows (Y_k dR, zero past the active degree; culled lanes have dR = 0)
        float Y[16];
        sh_basis(a.D, st_x, st_y, st_z, Y);
        const int nsh = sh_count(a.D);
        auto val = [&](int e) {
            const int k = e / 3, c = e - 3 * (e / 3);
            const float d = c == 0 ? st_d0 : (c == 1 ? st_d1 : st_d2);
            return k < nsh ? Y[k] * d : 0.f;
        };
        if (a.dL_dsh_rest) {  // the split layout: the wave's 45-float rest rows, then its 3-float DC rows
            float* rest = stage + 45 * slot;
            float* dc = stage + 45 * 64 + 3 * slot;
#pragma unroll
            for (int e = 0; e < 3; e++) dc[e] = val(e);
#pragma unroll
            for (int e = 0; e < 45; e++) rest[e] = val(3 + e);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            wave_store_rows(a.dL_dsh + (size_t)wbase * 3, stage + 45 * 64, n * 3, lane);
            wave_store_rows(a.dL_dsh_rest + (size_t)wbase * 45, stage, n * 45, lane);
        } else {
            float4* row = reinterpret_cast<float4*>(stage + 48 * slot);
#pragma unroll
            for (int i = 0; i < 12; i++)
                row[i] = make_float4(val(4 * i), val(4 * i + 1), val(4 * i + 2), val(4 * i + 3));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            wave_store_rows(a.dL_dsh + (size_t)wbase * 48, stage, n * 48, lane);
        }
    }
}

hipError_t launch_preprocess_bwd(const BwdParams& b, const GeomState& gs, const BwdState& ws, hipStream_t stream,
                                 int begin, int end, float* dc_rows) {
    const FwdParams& p = b.f;
    if (end < 0) end = p.P;
    if (end <= begin) return hipSuccess;
    PreprocessBwdArgs a;
    a.P = p.P;
    a.D = p.D;
    a.SHM = p.SHM;
    a.SGD = p.SGD;
    a.SGM = p.SGM;
    a.means3D = p.means3D;
    a.opacities = p.opacities;
    a.scales = p.scales;
    a.rotations = p.rotations;
    a.cov3D_precomp = p.cov3D_precomp;
    a.shs = p.shs;
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
    a.radii = b.radii;
    a.clamped = gs.clamped;
    a.ddir = gs.ddir;
    a.acc = ws.acc;
    a.acc_abs = ws.acc_abs;
    a.dL_dmean3D = b.dL_dmean3D;
    a.dL_dmean2D = b.dL_dmean2D;
    a.dL_dcolor = b.dL_dcolor;
    a.dL_dopacity = b.dL_dopacity;
    a.dL_dscale = b.dL_dscale;
    a.dL_drot = b.dL_drot;
    a.dL_dcov3D = b.dL_dcov3D;
    a.dL_dsh = b.dL_dsh;
    a.dL_dsh_rest = b.dL_dsh_rest;
    a.dL_dsg_axis = b.dL_dsg_axis;
    a.dL_dsg_sharpness = b.dL_dsg_sharpness;
    a.dL_dsg_color = b.dL_dsg_color;
    a.begin = begin;
    a.end = end;
    a.dc_rows = dc_rows;
    // staged row stores: the 16-coefficient SH layout, 16-B aligned rows, SG degree 0 or 7 (the
    // configurations with wide rows), whole-workgroup ranges; GSR_OPT_PBWD_STAGE 1 forces it, 2 turns it off.
    // Alignment of every row base the stage touches: the gradient rows it stores and, at SG 7, the lobe
    // input rows it loads by 16-B LDS-DMA (a tensor that is a view at a 4-B offset takes the per-lane path)
    const int so = option(kOptPbwdStage);
    auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    const bool stage_ok = p.shs && !dc_rows && (!b.dL_dsh_rest || al16(b.dL_dsh_rest)) && p.SHM == 16 && (begin & 255) == 0 && al16(b.dL_dsh) &&
                          (p.SGM == 0 || (p.SGM == kSG7 && p.SGD == kSG7 && al16(b.dL_dsg_color) &&
                                          al16(b.dL_dsg_sharpness) && al16(b.dL_dsg_axis) &&
                                          al16(p.sg_color) && al16(p.sg_sharpness) && al16(p.sg_axis)));
    const bool stage = stage_ok && (so == 1 || (so == 0 && GSR_PBWD_STAGE_DEFAULT));
    if (stage)
        hipLaunchKernelGGL(preprocess_bwd_kernel<true>, dim3((end - begin + 255) / 256), dim3(256), 0, stream, a);
    else
        hipLaunchKernelGGL(preprocess_bwd_kernel<false>, dim3((end - begin + 255) / 256), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
