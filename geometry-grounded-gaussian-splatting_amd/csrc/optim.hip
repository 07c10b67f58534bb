// optim.hip — the per-iteration parameter update of training on gfx950
// (SURVEY §8(f) rank 2): a multi-tensor Adam step over all Gaussian
// parameter groups in one launch, and the densification statistics.
//
// Replaces, for the Gaussian parameters:
//   torch.optim.Adam(..., eps=1e-15).step()   (scene/gaussian_model.py:347-351,
//                                              train.py:259-261)
//     exp_avg    = lerp(exp_avg, g, 1 - beta1)
//     exp_avg_sq = beta2 exp_avg_sq + (1 - beta2) g^2
//     p         -= lr / (1 - beta1^t) * exp_avg / (sqrt(exp_avg_sq) / sqrt(1 - beta2^t) + eps)
//   (torch/optim/adam.py _single_tensor_adam, the published Adam of
//   Kingma & Ba with torch's rounding order);
//   GaussianModel.add_densification_stats + the max_radii2D update
//     (scene/gaussian_model.py:818-821, train.py:236-237).
// Both are pure HBM streams (28 B per parameter element, 24 B + 3 x 4 B per
// Gaussian for the statistics): float4 loads/stores, grid-stride over all
// groups, no LDS.
#include "gsr_kernels.h"

namespace gsr {

struct AdamArgs {
    int n_groups;
    float beta1, beta2, one_m_beta1, one_m_beta2;
    AdamGroup g[kMaxAdamGroups];
    float step_size[kMaxAdamGroups];   // lr / (1 - beta1^t)
    float bc2_sqrt[kMaxAdamGroups];    // sqrt(1 - beta2^t)
    unsigned long long vec_begin[kMaxAdamGroups + 1];  // prefix of float4 counts
};

__device__ __forceinline__ float adam_one(float& p, float g, float& m, float& v, float b2, float omb1, float omb2,
                                          float step_size, float bc2s, float eps) {
    // torch: exp_avg.lerp_(grad, 1 - beta1); exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
    m = m + omb1 * (g - m);           // lerp, weight < 0.5 branch (ATen Lerp.h)
    v = v * b2 + (omb2 * g) * g;      // addcmul: self + value * t1 * t2, left to right
    const float denom = sqrtf(v) / bc2s + eps;
    p = p - step_size * (m / denom);
    return p;
}

#ifndef GSR_ADAM_NT
// Non-temporal loads and stores (each element is touched once per step, and the step's 1-2 GB pass through
// the caches otherwise): bench_optim's full parameter set 0.576 -> 0.531 ms.  Two or four float4 per thread
// per grid-stride step with all loads issued first measured slower (0.541 / 0.623 ms with these hints).
#define GSR_ADAM_NT 1
#endif

typedef float adam_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_stream(const float4* p) {
    if constexpr (GSR_ADAM_NT) {
        const adam_f4 v = __builtin_nontemporal_load(reinterpret_cast<const adam_f4*>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}
__device__ __forceinline__ void st_stream(float4* p, float4 v) {
    if constexpr (GSR_ADAM_NT) __builtin_nontemporal_store(adam_f4{v.x, v.y, v.z, v.w}, reinterpret_cast<adam_f4*>(p));
    else *p = v;
}

__global__ void __launch_bounds__(256) adam_kernel(AdamArgs a, float eps) {
    const unsigned long long total = a.vec_begin[a.n_groups];
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    int gi = 0;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        while (i >= a.vec_begin[gi + 1]) gi++;  // groups are visited in increasing order per thread
        const AdamGroup& G = a.g[gi];
        const unsigned long long e0 = (i - a.vec_begin[gi]) * 4ull;
        const float ss = a.step_size[gi], bc = a.bc2_sqrt[gi];
        if (e0 + 4 <= (unsigned long long)G.n && G.aligned) {
            float4* const pp = reinterpret_cast<float4*>(G.param) + e0 / 4;
            float4* const mp = reinterpret_cast<float4*>(G.exp_avg) + e0 / 4;
            float4* const vp = reinterpret_cast<float4*>(G.exp_avg_sq) + e0 / 4;
            float4 p = ld_stream(pp);
            const float4 g = ld_stream(reinterpret_cast<const float4*>(G.grad) + e0 / 4);
            float4 m = ld_stream(mp);
            float4 v = ld_stream(vp);
            adam_one(p.x, g.x, m.x, v.x, a.beta2, a.one_m_beta1, a.one_m_beta2, ss, bc, eps);
            adam_one(p.y, g.y, m.y, v.y, a.beta2, a.one_m_beta1, a.one_m_beta2, ss, bc, eps);
            adam_one(p.z, g.z, m.z, v.z, a.beta2, a.one_m_beta1, a.one_m_beta2, ss, bc, eps);
            adam_one(p.w, g.w, m.w, v.w, a.beta2, a.one_m_beta1, a.one_m_beta2, ss, bc, eps);
            st_stream(pp, p);
            st_stream(mp, m);
            st_stream(vp, v);
        } else {
            for (unsigned long long e = e0; e < e0 + 4 && e < (unsigned long long)G.n; e++)
                adam_one(G.param[e], G.grad[e], G.exp_avg[e], G.exp_avg_sq[e], a.beta2, a.one_m_beta1,
                         a.one_m_beta2, ss, bc, eps);
        }
    }
}

hipError_t launch_adam(int n_groups, const AdamGroup* groups, const double* lr, double step, double beta1,
                       double beta2, double eps, hipStream_t stream) {
    if (n_groups <= 0) return hipSuccess;
    AdamArgs a;
    a.n_groups = n_groups;
    // as torch: Python-float (double) scalars, rounded to fp32 where they meet the tensors
    a.beta1 = (float)beta1;
    a.beta2 = (float)beta2;
    a.one_m_beta1 = (float)(1.0 - beta1);
    a.one_m_beta2 = (float)(1.0 - beta2);
    a.vec_begin[0] = 0;
    // bias corrections as torch computes them for a CPU float step (python floats, double)
    const double bc1 = 1.0 - pow(beta1, step);
    const double bc2 = 1.0 - pow(beta2, step);
    for (int k = 0; k < n_groups; k++) {
        a.g[k] = groups[k];
        a.step_size[k] = (float)(lr[k] / bc1);
        a.bc2_sqrt[k] = (float)sqrt(bc2);
        a.vec_begin[k + 1] = a.vec_begin[k] + (unsigned long long)((groups[k].n + 3) / 4);
    }
    const unsigned long long total = a.vec_begin[n_groups];
    if (total == 0) return hipSuccess;
    const unsigned long long blocks = (total + 255) / 256;
    const unsigned grid = (unsigned)(blocks < 256ull * 32ull ? blocks : 256ull * 32ull);  // 32 blocks per CU
    hipLaunchKernelGGL(adam_kernel, dim3(grid), dim3(256), 0, stream, a, (float)eps);
    return hipGetLastError();
}

// add_densification_stats + max_radii2D (scene/gaussian_model.py:818-821,
// train.py:236-237), for the Gaussians with radii > 0:
//   max_radii2D = max(max_radii2D, radii)
//   xyz_gradient_accum     += |grad[:2]|    (norm of the screen-space x, y gradient)
//   xyz_gradient_accum_abs += |grad[2:]|    (the |.|-sum channel, render_backward.cu:1028)
//   denom += 1
__global__ void __launch_bounds__(256)
    densify_stats_kernel(int P, const float* __restrict__ vgrad, const int* __restrict__ radii,
                         float* __restrict__ max_radii2D, float* __restrict__ accum, float* __restrict__ accum_abs,
                         float* __restrict__ denom) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int r = radii[i];
    if (!(r > 0)) return;
    const float gx = vgrad[3 * i], gy = vgrad[3 * i + 1], gz = vgrad[3 * i + 2];
    max_radii2D[i] = fmaxf(max_radii2D[i], (float)r);
    accum[i] += sqrtf(gx * gx + gy * gy);
    accum_abs[i] += fabsf(gz);
    denom[i] += 1.f;
}

hipError_t launch_densify_stats(int P, const float* vgrad, const int* radii, float* max_radii2D, float* accum,
                                float* accum_abs, float* denom, hipStream_t stream) {
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(densify_stats_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, vgrad, radii,
                       max_radii2D, accum, accum_abs, denom);
    return hipGetLastError();
}

// ------------------------------------------------------------------ getters
// GaussianModel's activation getters (scene/gaussian_model.py:146-212) that
// feed every render and sample_depth call of training, as one thread per
// Gaussian instead of ~10 broadcast torch ops (and ~20 in their autograd
// backward: prod / sqrt / division / zero checks):
//   get_scaling_n_opacity_with_3D_filter (and the separate
//   get_scaling_with_3D_filter / get_opacity_with_3D_filter):
//     q = exp(s)^2, a = q + f^2, scales = sqrt(a),
//     opacity = sigmoid(o) sqrt(q0 q1 q2) rsqrt(a0 a1 a2)
//   backward: dL/ds_k = gS_k q_k / sqrt(a_k) + gO opacity f^2 / a_k,
//             dL/do = gO opacity (1 - sigmoid(o));
//   get_rotation (F.normalize, eps 1e-12) and its backward
//     (g - y (y . g)) / max(|x|, eps) (|x| <= eps: g / eps).
// Pure HBM streams (20 B in, 16 B out per Gaussian).
__global__ void __launch_bounds__(256) scale_opacity_kernel(int P, const float* __restrict__ s,
                                                            const float* __restrict__ o,
                                                            const float* __restrict__ f, float* __restrict__ scales,
                                                            float* __restrict__ opac, const float* __restrict__ gS,
                                                            const float* __restrict__ gO, float* __restrict__ ds,
                                                            float* __restrict__ dop, bool backward) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const float f2 = f[i] * f[i];
    float q[3], a[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float e = expf(s[3 * i + k]);
        q[k] = e * e;
        a[k] = q[k] + f2;
    }
    const float sig = 1.f / (1.f + expf(-o[i]));
    const float coef = sqrtf((q[0] * q[1]) * q[2]) * (1.f / sqrtf((a[0] * a[1]) * a[2]));
    const float op = sig * coef;
    if (!backward) {
#pragma unroll
        for (int k = 0; k < 3; k++) scales[3 * i + k] = sqrtf(a[k]);
        opac[i] = op;
        return;
    }
    const float go = gO ? gO[i] : 0.f;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float g = gS ? gS[3 * i + k] : 0.f;
        ds[3 * i + k] = g * (q[k] / sqrtf(a[k])) + go * op * (f2 / a[k]);
    }
    dop[i] = go * op * (1.f - sig);
}

__global__ void __launch_bounds__(256) normalize_rows_kernel(int n, int D, const float* __restrict__ x,
                                                             const float* __restrict__ gy, float* __restrict__ out,
                                                             bool backward) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float* r = x + (size_t)i * D;
    float* o = out + (size_t)i * D;
    if (D == 4 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out) |
                    reinterpret_cast<uintptr_t>(gy)) & 15) == 0) {  // quaternions: one 16-B access each way
        const float4 v = *reinterpret_cast<const float4*>(r);
        const float len = sqrtf(((v.x * v.x + v.y * v.y) + v.z * v.z) + v.w * v.w), m = fmaxf(len, 1e-12f);
        const float4 u = make_float4(v.x / m, v.y / m, v.z / m, v.w / m);
        if (!backward) {
            *reinterpret_cast<float4*>(o) = u;
            return;
        }
        const float4 g = *reinterpret_cast<const float4*>(gy + (size_t)i * 4);
        float4 d;
        if (len > 1e-12f) {
            const float dot = ((u.x * g.x + u.y * g.y) + u.z * g.z) + u.w * g.w;
            d = make_float4((g.x - u.x * dot) / m, (g.y - u.y * dot) / m, (g.z - u.z * dot) / m, (g.w - u.w * dot) / m);
        } else {
            d = make_float4(g.x / m, g.y / m, g.z / m, g.w / m);
        }
        *reinterpret_cast<float4*>(o) = d;
        return;
    }
    float ss = 0.f;
    for (int k = 0; k < D; k++) ss += r[k] * r[k];
    const float len = sqrtf(ss), m = fmaxf(len, 1e-12f);
    if (!backward) {
        for (int k = 0; k < D; k++) o[k] = r[k] / m;
        return;
    }
    const float* g = gy + (size_t)i * D;
    if (len > 1e-12f) {
        float dot = 0.f;
        for (int k = 0; k < D; k++) dot += (r[k] / m) * g[k];
        for (int k = 0; k < D; k++) o[k] = (g[k] - (r[k] / m) * dot) / m;
    } else {
        for (int k = 0; k < D; k++) o[k] = g[k] / m;
    }
}

hipError_t launch_scale_opacity(int P, const float* s, const float* o, const float* f, float* scales, float* opac,
                                const float* gS, const float* gO, float* ds, float* dop, bool backward,
                                hipStream_t stream) {
    if (P <= 0) return hipSuccess;
    hipLaunchKernelGGL(scale_opacity_kernel, dim3((P + 255) / 256), dim3(256), 0, stream, P, s, o, f, scales, opac,
                       gS, gO, ds, dop, backward);
    return hipGetLastError();
}

hipError_t launch_normalize_rows(int n, int D, const float* x, const float* gy, float* out, bool backward,
                                 hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(normalize_rows_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, n, D, x, gy, out,
                       backward);
    return hipGetLastError();
}

}  // namespace gsr
