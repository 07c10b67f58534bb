// gsr_math.h — per-Gaussian projection math shared by the forward and
// backward preprocess kernels (gfx950).
//
// Written in math (row, col) convention.  The reference builds the same
// quantities with glm column-major matrices (render_forward.cu:81-243); the
// mapping used here is
//   A   = W_r * R_q        (world->camera rotation times the Gaussian rotation)
//   cov2D = (J A S)(J A S)^T              == glm transpose(S*R*T) * (S*R*T)
//   cov_cam_inv = (A S^-1)(A S^-1)^T      == glm transpose(S^-1*R*W) * (S^-1*R*W)
// with W_r[i][j] = view[4j+i], R_q the standard rotation of q = (r, x, y, z)
// (not renormalised) and J the EWA Jacobian at the
// clamped view ray.
#pragma once

#include "gsr_common.h"

namespace gsr {

struct ViewGeom {
    float t[3];    // view-space position (unclamped)
    float tc;      // |t|  (ray_plane.z, and the sort depth)
    float u, v;    // clamped ray slopes
    float tx, tz, ty;  // clamped view position (tx = u*tz, ty = v*tz)
    bool clamp_x, clamp_y;
};

__device__ inline void view_point(const float* __restrict__ V, float px, float py, float pz, float* t) {
    t[0] = V[0] * px + V[4] * py + V[8] * pz + V[12];
    t[1] = V[1] * px + V[5] * py + V[9] * pz + V[13];
    t[2] = V[2] * px + V[6] * py + V[10] * pz + V[14];
}

__device__ inline ViewGeom view_geom(const float* __restrict__ V, float px, float py, float pz, float tan_fovx,
                                     float tan_fovy) {
    ViewGeom g;
    view_point(V, px, py, pz, g.t);
    g.tc = sqrtf(g.t[0] * g.t[0] + g.t[1] * g.t[1] + g.t[2] * g.t[2]);
    const float limx = 1.3f * tan_fovx, limy = 1.3f * tan_fovy;
    const float u0 = g.t[0] / g.t[2], v0 = g.t[1] / g.t[2];
    g.clamp_x = u0 < -limx || u0 > limx;
    g.clamp_y = v0 < -limy || v0 > limy;
    g.tz = g.t[2];
    g.tx = fminf(limx, fmaxf(-limx, u0)) * g.tz;
    g.ty = fminf(limy, fmaxf(-limy, v0)) * g.tz;
    g.u = g.tx / g.tz;
    g.v = g.ty / g.tz;
    return g;
}

// A = W_r * R_q (row-major 3x3)
__device__ inline void rot_view(const float* __restrict__ V, float qr, float qx, float qy, float qz, float* A,
                                float* Rq) {
    Rq[0] = 1.f - 2.f * (qy * qy + qz * qz);
    Rq[1] = 2.f * (qx * qy - qr * qz);
    Rq[2] = 2.f * (qx * qz + qr * qy);
    Rq[3] = 2.f * (qx * qy + qr * qz);
    Rq[4] = 1.f - 2.f * (qx * qx + qz * qz);
    Rq[5] = 2.f * (qy * qz - qr * qx);
    Rq[6] = 2.f * (qx * qz - qr * qy);
    Rq[7] = 2.f * (qy * qz + qr * qx);
    Rq[8] = 1.f - 2.f * (qx * qx + qy * qy);
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            A[3 * i + j] = V[i] * Rq[j] + V[4 + i] * Rq[3 + j] + V[8 + i] * Rq[6 + j];
}

// SH constants (CR/auxiliary.h:21-36)
__device__ constexpr float kSH_C0 = 0.28209479177387814f;
__device__ constexpr float kSH_C1 = 0.4886025119029199f;
__device__ constexpr float kSH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                                        -1.0925484305920792f, 0.5462742152960396f};
__device__ constexpr float kSH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                                        0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                                        -0.5900435899266435f};

// SH basis values Y_k(dir) for k < (D+1)^2 (coefficient k multiplies Y_k).
__device__ inline void sh_basis(int D, float x, float y, float z, float* Y) {
    Y[0] = kSH_C0;
    if (D > 0) {
        Y[1] = -kSH_C1 * y;
        Y[2] = kSH_C1 * z;
        Y[3] = -kSH_C1 * x;
        if (D > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            Y[4] = kSH_C2[0] * xy;
            Y[5] = kSH_C2[1] * yz;
            Y[6] = kSH_C2[2] * (2.0f * zz - xx - yy);
            Y[7] = kSH_C2[3] * xz;
            Y[8] = kSH_C2[4] * (xx - yy);
            if (D > 2) {
                Y[9] = kSH_C3[0] * y * (3.0f * xx - yy);
                Y[10] = kSH_C3[1] * xy * z;
                Y[11] = kSH_C3[2] * y * (4.0f * zz - xx - yy);
                Y[12] = kSH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
                Y[13] = kSH_C3[4] * x * (4.0f * zz - xx - yy);
                Y[14] = kSH_C3[5] * z * (xx - yy);
                Y[15] = kSH_C3[6] * x * (xx - 3.0f * yy);
            }
        }
    }
}

__device__ inline int sh_count(int D) { return (D + 1) * (D + 1); }

// dY_k / d(x, y, z) of the SH basis above (k >= 1): the terms of the
// reference's dRGBdx / dRGBdy / dRGBdz (render_backward.cu:94-153), so that
// d colour_c / d dir_i = sum_k dY_k/d dir_i sh[k][c].  The forward preprocess
// accumulates that Jacobian coefficient by coefficient next to the colour
// (each SH entry used once, its register then free) and stores it as
// GeomState::ddir, so the backward does not read the 192-B row again
// (preprocess_bwd.hip).
__device__ __forceinline__ void sh_basis_grad(int k, float x, float y, float z, float& gx, float& gy, float& gz) {
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    gx = 0.f, gy = 0.f, gz = 0.f;
    switch (k) {
        case 1: gy = -kSH_C1; break;
        case 2: gz = kSH_C1; break;
        case 3: gx = -kSH_C1; break;
        case 4: gx = kSH_C2[0] * y; gy = kSH_C2[0] * x; break;
        case 5: gy = kSH_C2[1] * z; gz = kSH_C2[1] * y; break;
        case 6: gx = kSH_C2[2] * 2.f * -x; gy = kSH_C2[2] * 2.f * -y; gz = kSH_C2[2] * 2.f * 2.f * z; break;
        case 7: gx = kSH_C2[3] * z; gz = kSH_C2[3] * x; break;
        case 8: gx = kSH_C2[4] * 2.f * x; gy = kSH_C2[4] * 2.f * -y; break;
        case 9: gx = kSH_C3[0] * 3.f * 2.f * xy; gy = kSH_C3[0] * 3.f * (xx - yy); break;
        case 10: gx = kSH_C3[1] * yz; gy = kSH_C3[1] * xz; gz = kSH_C3[1] * xy; break;
        case 11: gx = kSH_C3[2] * -2.f * xy; gy = kSH_C3[2] * (-3.f * yy + 4.f * zz - xx); gz = kSH_C3[2] * 4.f * 2.f * yz; break;
        case 12: gx = kSH_C3[3] * -3.f * 2.f * xz; gy = kSH_C3[3] * -3.f * 2.f * yz; gz = kSH_C3[3] * 3.f * (2.f * zz - xx - yy); break;
        case 13: gx = kSH_C3[4] * (-3.f * xx + 4.f * zz - yy); gy = kSH_C3[4] * -2.f * xy; gz = kSH_C3[4] * 4.f * 2.f * xz; break;
        case 14: gx = kSH_C3[5] * 2.f * xz; gy = kSH_C3[5] * -2.f * yz; gz = kSH_C3[5] * (xx - yy); break;
        default: gx = kSH_C3[6] * 3.f * (xx - yy); gy = kSH_C3[6] * -3.f * 2.f * xy; break;
    }
}

// A lobe row (21 or 7 floats, 84 / 28 B) is only 4-B aligned; gfx950 serves
// unaligned dwordx4 accesses, so a row moves as 16-B pieces: 6 + 6 + 2 load
// instructions per Gaussian instead of 49 single dwords, each of which made
// the L1 look up 64 distinct lines (the rows of a wave's lanes are 84 B apart).
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
template <int N>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float (&v)[N]) {
#pragma unroll
    for (int k = 0; k + 4 <= N; k += 4) {
        const f4u t = *reinterpret_cast<const f4u*>(p + k);
        v[k] = t.x;
        v[k + 1] = t.y;
        v[k + 2] = t.z;
        v[k + 3] = t.w;
    }
#pragma unroll
    for (int k = N / 4 * 4; k < N; k++) v[k] = p[k];
}
template <int N>
__device__ __forceinline__ void store_row(float* __restrict__ p, const float (&v)[N]) {
#pragma unroll
    for (int k = 0; k + 4 <= N; k += 4) *reinterpret_cast<f4u*>(p + k) = f4u{v[k], v[k + 1], v[k + 2], v[k + 3]};
#pragma unroll
    for (int k = N / 4 * 4; k < N; k++) p[k] = v[k];
}
// One Gaussian's SH row ([SHM][3] floats, coefficient-major) in registers.
// The training layout (SHM = 16, 16-B aligned rows of 192 B) moves as 12
// dwordx4 per lane; other layouts element by element (entries >= 3 n read 0).
__device__ __forceinline__ bool sh_rows_vec4(const void* base, int SHM) {
    return SHM == 16 && (reinterpret_cast<uintptr_t>(base) & 15) == 0;
}
__device__ __forceinline__ void load_sh(const float* row, int SHM, int n, float (&v)[48]) {
    if (sh_rows_vec4(row, SHM)) {
        const float4* q = reinterpret_cast<const float4*>(row);
#pragma unroll
        for (int i = 0; i < 12; i++) {
            const float4 t = q[i];
            v[4 * i] = t.x;
            v[4 * i + 1] = t.y;
            v[4 * i + 2] = t.z;
            v[4 * i + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 48; k++) v[k] = k < 3 * n ? row[k] : 0.f;
    }
}
// The split layout of training (GaussianModel's _features_dc [P][1][3] and
// _features_rest [P][SHM-1][3] as two tensors, no concatenation): the DC row
// and the rest row (4-B aligned, 180 B at SHM 16) in 16-B pieces.
__device__ __forceinline__ void load_sh_split(const float* dc, const float* rest, int SHM, int n, float (&v)[48]) {
    v[0] = dc[0];
    v[1] = dc[1];
    v[2] = dc[2];
    if (SHM == 16) {  // straight into v (a staging array of its own raised the kernel's VGPRs 126 -> 147)
#pragma unroll
        for (int k = 0; k < 44; k += 4) {
            const f4u t = *reinterpret_cast<const f4u*>(rest + k);
            v[3 + k] = 3 + k < 3 * n ? t.x : 0.f;
            v[4 + k] = 4 + k < 3 * n ? t.y : 0.f;
            v[5 + k] = 5 + k < 3 * n ? t.z : 0.f;
            v[6 + k] = 6 + k < 3 * n ? t.w : 0.f;
        }
        v[47] = 47 < 3 * n ? rest[44] : 0.f;
    } else {
#pragma unroll
        for (int k = 3; k < 48; k++) v[k] = (k < 3 * n && k < 3 * SHM) ? rest[k - 3] : 0.f;
    }
}
// dL/dsh row: entry 3k + c = Y_k dL/dRGB_c for k < n, 0 beyond (all 3 * SHM
// entries written), generated straight into the stores.
__device__ __forceinline__ void store_sh_grad(float* row, int SHM, int n, const float (&Y)[16], float d0, float d1,
                                              float d2) {
    auto val = [&](int e) {
        const int k = e / 3, c = e - 3 * (e / 3);
        const float d = c == 0 ? d0 : (c == 1 ? d1 : d2);
        return k < n ? Y[k] * d : 0.f;
    };
    if (sh_rows_vec4(row, SHM)) {
        float4* q = reinterpret_cast<float4*>(row);
#pragma unroll
        for (int i = 0; i < 12; i++) q[i] = make_float4(val(4 * i), val(4 * i + 1), val(4 * i + 2), val(4 * i + 3));
    } else {
#pragma unroll
        for (int e = 0; e < 48; e++)
            if (e < 3 * SHM) row[e] = val(e);
        for (int e = 48; e < 3 * SHM; e++) row[e] = 0.f;
    }
}

// store_sh_grad for the split layout: the DC row and the rest row
__device__ __forceinline__ void store_sh_grad_split(float* dc, float* rest, int SHM, int n, const float (&Y)[16],
                                                    float d0, float d1, float d2) {
    auto val = [&](int e) {
        const int k = e / 3, c = e - 3 * (e / 3);
        const float d = c == 0 ? d0 : (c == 1 ? d1 : d2);
        return k < n ? Y[k] * d : 0.f;
    };
    dc[0] = val(0);
    dc[1] = val(1);
    dc[2] = val(2);
    if (SHM == 16) {
#pragma unroll
        for (int e = 0; e < 44; e += 4)
            *reinterpret_cast<f4u*>(rest + e) = f4u{val(3 + e), val(4 + e), val(5 + e), val(6 + e)};
        rest[44] = val(47);
    } else {
#pragma unroll
        for (int e = 3; e < 48; e++)
            if (e < 3 * SHM) rest[e - 3] = val(e);
        for (int e = 48; e < 3 * SHM; e++) rest[e - 3] = 0.f;
    }
}

// ---- symmetric 3x3 eigen-decomposition (cov3D_precomp path) --------------
// The reference's solver (glm_modification::findEigenvaluesSymReal,
// auxiliary.h:155-340): Householder reduction to tridiagonal form, then
// implicit QL iterations, in fp32 with its 1e-7 zero tests — restated here
// (as in oracle/gsr_oracle.c) because the inverse of a thin Gaussian's
// covariance is only as accurate as its smallest eigenvalue, and a closed-form
// (trigonometric) solver loses that one to cancellation: normals 4e-4 off the
// oracle's on tests/golden/cov3d.npz against 1e-4 for this solver.
// Every use is sign- and order-invariant (E diag(1/l) E^T, e e^T).
__device__ inline float sym3_pythag(float a, float b) {
    float aa = fabsf(a), ab = fabsf(b);
    if (aa > ab) {
        ab /= aa;
        ab *= ab;
        return aa * sqrtf(1.f + ab);
    }
    if (ab <= 1e-7f) return 0.f;
    aa /= ab;
    aa *= aa;
    return ab * sqrtf(1.f + aa);
}

// eigenvalues ascending in l[0..2], eigenvectors as rows of E (E[3k..3k+2] for l[k])
__device__ inline void sym3_eigen(const float* A, float* l, float* E) {
    constexpr float eps = 1e-7f;
    // a: row-major working copy (the matrix is symmetric, so glm's column order reads the same)
    float a[9], d[3], e[3];
#pragma unroll
    for (int k = 0; k < 9; k++) a[k] = A[k];
    // Householder: rows 2, 1 (tred2 with n = 3)
    for (int i = 2; i >= 1; i--) {
        const int lm = i - 1;  // last column of the row's sub-diagonal part
        float h = 0.f;
        if (lm > 0) {
            float scale = 0.f;
            for (int k = 0; k <= lm; k++) scale += fabsf(a[3 * i + k]);
            if (scale <= eps) {
                e[i] = a[3 * i + lm];
            } else {
                for (int k = 0; k <= lm; k++) {
                    a[3 * i + k] /= scale;
                    h += a[3 * i + k] * a[3 * i + k];
                }
                float f = a[3 * i + lm];
                float g = f >= 0.f ? -sqrtf(h) : sqrtf(h);
                e[i] = scale * g;
                h -= f * g;
                a[3 * i + lm] = f - g;
                f = 0.f;
                for (int j = 0; j <= lm; j++) {
                    a[3 * j + i] = a[3 * i + j] / h;
                    g = 0.f;
                    for (int k = 0; k <= j; k++) g += a[3 * j + k] * a[3 * i + k];
                    for (int k = j + 1; k <= lm; k++) g += a[3 * k + j] * a[3 * i + k];
                    e[j] = g / h;
                    f += e[j] * a[3 * i + j];
                }
                const float hh = f / (h + h);
                for (int j = 0; j <= lm; j++) {
                    f = a[3 * i + j];
                    e[j] = g = e[j] - hh * f;
                    for (int k = 0; k <= j; k++) a[3 * j + k] -= (f * e[k] + g * a[3 * i + k]);
                }
            }
        } else {
            e[i] = a[3 * i + lm];
        }
        d[i] = h;
    }
    d[0] = 0.f;
    e[0] = 0.f;
    // accumulate the transformations
    for (int i = 0; i < 3; i++) {
        if (!(fabsf(d[i]) <= eps)) {
            for (int j = 0; j < i; j++) {
                float g = 0.f;
                for (int k = 0; k < i; k++) g += a[3 * i + k] * a[3 * k + j];
                for (int k = 0; k < i; k++) a[3 * k + j] -= g * a[3 * k + i];
            }
        }
        d[i] = a[3 * i + i];
        a[3 * i + i] = 1.f;
        for (int j = 0; j < i; j++) a[3 * j + i] = a[3 * i + j] = 0.f;
    }
    // implicit QL on the tridiagonal (d, e)
    e[0] = e[1];
    e[1] = e[2];
    e[2] = 0.f;
    for (int ll = 0; ll < 3; ll++) {
        int iter = 0, m;
        do {
            for (m = ll; m < 2; m++)
                if (fabsf(e[m]) <= eps) break;
            if (m != ll) {
                if (iter++ == 30) break;
                float g = (d[ll + 1] - d[ll]) / (2.f * e[ll]);
                float r = sym3_pythag(g, 1.f);
                g = d[m] - d[ll] + e[ll] / (g + (g >= 0.f ? fabsf(r) : -fabsf(r)));
                float s = 1.f, c = 1.f, p = 0.f;
                int i;
                bool zero = false;
                for (i = m - 1; i >= ll; i--) {
                    const float f = s * e[i];
                    const float b = c * e[i];
                    e[i + 1] = r = sym3_pythag(f, g);
                    if (r <= eps) {
                        d[i + 1] -= p;
                        e[m] = 0.f;
                        zero = true;
                        break;
                    }
                    s = f / r;
                    c = g / r;
                    g = d[i + 1] - p;
                    r = (d[i] - g) * s + 2.f * c * b;
                    d[i + 1] = g + (p = s * r);
                    g = c * r - b;
                    for (int k = 0; k < 3; k++) {
                        const float fk = a[3 * k + i + 1];
                        a[3 * k + i + 1] = s * a[3 * k + i] + c * fk;
                        a[3 * k + i] = c * a[3 * k + i] - s * fk;
                    }
                }
                if (zero && i >= ll) continue;
                d[ll] -= p;
                e[ll] = g;
                e[m] = 0.f;
            }
        } while (m != ll);
    }
    // ascending, eigenvector k = column k of a
    int o[3] = {0, 1, 2};
    if (d[o[1]] < d[o[0]]) { const int t = o[0]; o[0] = o[1]; o[1] = t; }
    if (d[o[2]] < d[o[1]]) { const int t = o[1]; o[1] = o[2]; o[2] = t; }
    if (d[o[1]] < d[o[0]]) { const int t = o[0]; o[0] = o[1]; o[1] = t; }
    for (int k = 0; k < 3; k++) {
        l[k] = d[o[k]];
        for (int r = 0; r < 3; r++) E[3 * k + r] = a[3 * r + o[k]];
    }
}

// Vrk^-1 when the smallest eigenvalue exceeds 1e-8 (returns true), else the
// projector e_min e_min^T (returns false): render_forward.cu:170-187.
__device__ inline bool sym3_inverse_or_null_projector(const float* A, float* out) {
    float l[3], E[9];
    sym3_eigen(A, l, E);
    if (l[0] > 1e-8f) {
        const float il[3] = {1.0f / l[0], 1.0f / l[1], 1.0f / l[2]};
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++)
                out[3 * i + j] = E[i] * E[j] * il[0] + E[3 + i] * E[3 + j] * il[1] + E[6 + i] * E[6 + j] * il[2];
        return true;
    }
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) out[3 * i + j] = E[i] * E[j];
    return false;
}

}  // namespace gsr
