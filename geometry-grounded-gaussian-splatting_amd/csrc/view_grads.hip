// view_grads.hip — the colour gradients of a view-parallel step, rebuilt from
// every view's DC row (gsr_dist.FactoredViewGrads).
//
// Per Gaussian and view v the colour backward (render_backward.cu:56-191,
// preprocess_bwd.hip) gives, with d_v = normalize(mean - campos_v) and dR_v
// the view's clamp-masked dL/dRGB:
//   dL/dsh[k][c]        = Y_k(d_v) dR_v[c]
//   dL/dsg_color[l][c]  = dR_v[c] g_l,         g_l = exp(lambda_l (a_l . d_v - 1))
//   dL/dsg_sharpness[l] = s_l g_l (a_l . d_v - 1),   s_l = sum_c sg_color[l][c] dR_v[c]
//   dL/dsg_axis[l][c]   = s_l g_l lambda_l d_v[c]
// Y_0 = SH_C0 is a constant, so dR_v = dL/dsh[0]_v / SH_C0: the step's summed
// SH and SG gradients are a function of the views' 3-float DC rows and camera
// centres.  All-gathering those (12 B per Gaussian and view) replaces
// all-reducing the 192-B (SH 3) or 388-B (SH 3 + SG 7) gradient rows; every
// rank then sums the views here, in view order, so the replicas stay
// bit-identical.  The DC row itself is summed as gathered (no division).
//
// Two layouts of the gathered rows:
//  * chunk = 0 (gsr_dist.FactoredViewGrads, one all-gather after the
//    backward): [n_views][P * 3 + 4], each view's DC rows then its camera centre;
//  * chunk > 0 (gsr_dist.OverlappedViewGrads, one all-gather per Gaussian
//    range as the backward produces it): the Gaussians in ranges of `chunk`
//    (the last one shorter); range r = [b, b + len) occupies
//    [3 n_views b, 3 n_views (b + len)) as [n_views][len][3], and the camera
//    centres are a separate [n_views][4] array.
#include "gsr_kernels.h"
#include "gsr_math.h"

namespace gsr {

struct ViewColorArgs {
    int P, D, SHM, SGD, SGM, n_views;
    const float* gathered;  // the views' dL/dsh[:, 0, :] (and camera centres), layout by `chunk` (header)
    const float* means3D;
    const float* sg_axis;
    const float* sg_sharpness;
    const float* sg_color;
    float* dL_dsh;
    float* dL_dsg_axis;
    float* dL_dsg_sharpness;
    float* dL_dsg_color;
    int chunk;
    const float* campos;  // [n_views][4] when chunk > 0
    float* dL_dsh_rest;   // split SH layout: dL_dsh is the DC rows [P][1][3], these the rest [P][SHM - 1][3]
};

constexpr int kMaxSG = 7;

__global__ void __launch_bounds__(256) view_color_grads_kernel(ViewColorArgs a) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= a.P) return;
    const size_t stride = (size_t)a.P * 3 + 4;
    const float mx = a.means3D[3 * idx], my = a.means3D[3 * idx + 1], mz = a.means3D[3 * idx + 2];
    const int n = sh_count(a.D);
    const int sgd = min(a.SGD, min(a.SGM, kMaxSG));
    float ax[3 * kMaxSG], gc[3 * kMaxSG], lam[kMaxSG];
#pragma unroll
    for (int l = 0; l < kMaxSG; l++) {
        if (l < sgd) {
            const size_t o = (size_t)idx * a.SGM + l;
#pragma unroll
            for (int c = 0; c < 3; c++) {
                ax[3 * l + c] = a.sg_axis[3 * o + c];
                gc[3 * l + c] = a.sg_color[3 * o + c];
            }
            lam[l] = a.sg_sharpness[o];
        } else {
#pragma unroll
            for (int c = 0; c < 3; c++) ax[3 * l + c] = gc[3 * l + c] = 0.f;
            lam[l] = 0.f;
        }
    }
    float dsh[48], dcol[3 * kMaxSG], dlam[kMaxSG], dax[3 * kMaxSG];
#pragma unroll
    for (int k = 0; k < 48; k++) dsh[k] = 0.f;
#pragma unroll
    for (int k = 0; k < 3 * kMaxSG; k++) dcol[k] = dax[k] = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxSG; k++) dlam[k] = 0.f;
    // (chunked layout: this Gaussian's range and its slot in it)
    const int rb = a.chunk > 0 ? idx / a.chunk * a.chunk : 0;
    const int rlen = a.chunk > 0 ? min(a.chunk, a.P - rb) : 0;
    for (int v = 0; v < a.n_views; v++) {
        const float* row;
        const float* cp;
        if (a.chunk > 0) {
            row = a.gathered + (size_t)3 * a.n_views * rb + (size_t)3 * v * rlen - (size_t)3 * rb;
            cp = a.campos + 4 * v;
        } else {
            row = a.gathered + (size_t)v * stride;
            cp = row + (size_t)a.P * 3;
        }
        const float g0 = row[3 * idx], g1 = row[3 * idx + 1], g2 = row[3 * idx + 2];
        // direction as the colour backward forms it (preprocess_bwd.hip)
        const float dox = mx - cp[0], doy = my - cp[1], doz = mz - cp[2];
        const float dlen = sqrtf(dox * dox + doy * doy + doz * doz);
        const float x = dox / dlen, y = doy / dlen, z = doz / dlen;
        const float dR0 = g0 / kSH_C0, dR1 = g1 / kSH_C0, dR2 = g2 / kSH_C0;
        float Y[16];
        sh_basis(a.D, x, y, z, Y);
        dsh[0] += g0;
        dsh[1] += g1;
        dsh[2] += g2;
#pragma unroll
        for (int k = 1; k < 16; k++) {
            if (k < n) {
                dsh[3 * k] += Y[k] * dR0;
                dsh[3 * k + 1] += Y[k] * dR1;
                dsh[3 * k + 2] += Y[k] * dR2;
            }
        }
#pragma unroll
        for (int l = 0; l < kMaxSG; l++) {
            if (l < sgd) {
                const float auxs = (ax[3 * l] * x + ax[3 * l + 1] * y + ax[3 * l + 2] * z) - 1.0f;
                const float gs = expf(lam[l] * auxs);
                dcol[3 * l] += dR0 * gs;
                dcol[3 * l + 1] += dR1 * gs;
                dcol[3 * l + 2] += dR2 * gs;
                const float dL_dexp = (gc[3 * l] * dR0 + gc[3 * l + 1] * dR1 + gc[3 * l + 2] * dR2) * gs;
                dlam[l] += dL_dexp * auxs;
                const float dL_daux = dL_dexp * lam[l];
                dax[3 * l] += dL_daux * x;
                dax[3 * l + 1] += dL_daux * y;
                dax[3 * l + 2] += dL_daux * z;
            }
        }
    }
    if (a.dL_dsh && a.dL_dsh_rest) {  // (the split layout: GaussianModel's features_dc / features_rest)
        float* dc = a.dL_dsh + (size_t)idx * 3;
        float* rest = a.dL_dsh_rest + (size_t)idx * (a.SHM - 1) * 3;
        dc[0] = dsh[0], dc[1] = dsh[1], dc[2] = dsh[2];
#pragma unroll
        for (int e = 3; e < 48; e++)
            if (e < 3 * a.SHM) rest[e - 3] = dsh[e];
        for (int e = 48; e < 3 * a.SHM; e++) rest[e - 3] = 0.f;
    } else if (a.dL_dsh) {
        float* out = a.dL_dsh + (size_t)idx * a.SHM * 3;
        if (sh_rows_vec4(out, a.SHM)) {
            float4* q = reinterpret_cast<float4*>(out);
#pragma unroll
            for (int i = 0; i < 12; i++) q[i] = make_float4(dsh[4 * i], dsh[4 * i + 1], dsh[4 * i + 2], dsh[4 * i + 3]);
        } else {
#pragma unroll
            for (int e = 0; e < 48; e++)
                if (e < 3 * a.SHM) out[e] = dsh[e];
            for (int e = 48; e < 3 * a.SHM; e++) out[e] = 0.f;
        }
    }
    for (int l = 0; l < a.SGM; l++) {
        const size_t o = (size_t)idx * a.SGM + l;
        float c3[3] = {0.f, 0.f, 0.f}, a3[3] = {0.f, 0.f, 0.f}, s1 = 0.f;
#pragma unroll
        for (int m = 0; m < kMaxSG; m++)
            if (m == l) {
                c3[0] = dcol[3 * m], c3[1] = dcol[3 * m + 1], c3[2] = dcol[3 * m + 2];
                a3[0] = dax[3 * m], a3[1] = dax[3 * m + 1], a3[2] = dax[3 * m + 2];
                s1 = dlam[m];
            }
        if (a.dL_dsg_sharpness) a.dL_dsg_sharpness[o] = s1;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            if (a.dL_dsg_color) a.dL_dsg_color[3 * o + c] = c3[c];
            if (a.dL_dsg_axis) a.dL_dsg_axis[3 * o + c] = a3[c];
        }
    }
}

hipError_t launch_view_color_grads(int P, int D, int SHM, int SGD, int SGM, int n_views, const float* gathered,
                                   const float* means3D, const float* sg_axis, const float* sg_sharpness,
                                   const float* sg_color, float* dL_dsh, float* dL_dsg_axis, float* dL_dsg_sharpness,
                                   float* dL_dsg_color, hipStream_t stream, int chunk, const float* campos,
                                   float* dL_dsh_rest) {
    if (P == 0) return hipSuccess;
    ViewColorArgs a{P, D, SHM, SGD, SGM, n_views, gathered, means3D, sg_axis, sg_sharpness, sg_color,
                    dL_dsh, dL_dsg_axis, dL_dsg_sharpness, dL_dsg_color, chunk, campos, dL_dsh_rest};
    hipLaunchKernelGGL(view_color_grads_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
