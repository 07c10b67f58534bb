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

// ---- symmetric 3x3 eigen-decomposition (cov3D_precomp path) --------------
// The reference runs glm's Householder + QL solver (auxiliary.h:155-340); any
// solver that returns the same eigen-pairs up to sign gives the same results,
// because every use is sign-invariant (Vrk^-1 = E diag(1/l) E^T, and
// projectors e e^T).  Closed form: trigonometric eigenvalues, eigenvectors
// from the largest cross product of two rows of (A - l I).
__device__ inline void sym3_eigvec(const float* A, float lam, float* e) {
    const float r0[3] = {A[0] - lam, A[1], A[2]};
    const float r1[3] = {A[3], A[4] - lam, A[5]};
    const float r2[3] = {A[6], A[7], A[8] - lam};
    float c[3][3];
    const float* rs[3][2] = {{r0, r1}, {r0, r2}, {r1, r2}};
    int best = 0;
    float bn = -1.f;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float* a = rs[k][0];
        const float* b = rs[k][1];
        c[k][0] = a[1] * b[2] - a[2] * b[1];
        c[k][1] = a[2] * b[0] - a[0] * b[2];
        c[k][2] = a[0] * b[1] - a[1] * b[0];
        const float n = c[k][0] * c[k][0] + c[k][1] * c[k][1] + c[k][2] * c[k][2];
        if (n > bn) { bn = n; best = k; }
    }
    if (bn <= 1e-30f) { e[0] = 1.f; e[1] = 0.f; e[2] = 0.f; return; }
    const float in = 1.0f / sqrtf(bn);
    e[0] = c[best][0] * in; e[1] = c[best][1] * in; e[2] = c[best][2] * in;
}

// eigenvalues ascending in l[0..2], eigenvectors as rows of E (E[3k..3k+2] for l[k])
__device__ inline void sym3_eigen(const float* A, float* l, float* E) {
    const float p1 = A[1] * A[1] + A[2] * A[2] + A[5] * A[5];
    const float q = (A[0] + A[4] + A[8]) * (1.0f / 3.0f);
    const float p2 = (A[0] - q) * (A[0] - q) + (A[4] - q) * (A[4] - q) + (A[8] - q) * (A[8] - q) + 2.f * p1;
    const float p = sqrtf(p2 * (1.0f / 6.0f));
    if (p <= 1e-30f) {
        l[0] = l[1] = l[2] = q;
        E[0] = 1; E[1] = 0; E[2] = 0; E[3] = 0; E[4] = 1; E[5] = 0; E[6] = 0; E[7] = 0; E[8] = 1;
        return;
    }
    const float ip = 1.0f / p;
    const float B[9] = {(A[0] - q) * ip, A[1] * ip, A[2] * ip, A[3] * ip, (A[4] - q) * ip, A[5] * ip,
                        A[6] * ip, A[7] * ip, (A[8] - q) * ip};
    float r = 0.5f * (B[0] * (B[4] * B[8] - B[5] * B[7]) - B[1] * (B[3] * B[8] - B[5] * B[6]) +
                      B[2] * (B[3] * B[7] - B[4] * B[6]));
    r = fminf(1.f, fmaxf(-1.f, r));
    const float phi = acosf(r) * (1.0f / 3.0f);
    const float hi = q + 2.f * p * cosf(phi);
    const float lo = q + 2.f * p * cosf(phi + 2.0943951023931953f);
    l[0] = lo;
    l[2] = hi;
    l[1] = 3.f * q - hi - lo;
    sym3_eigvec(A, l[0], E);
    sym3_eigvec(A, l[2], E + 6);
    // middle eigenvector orthogonal to the other two
    E[3] = E[7] * E[2] - E[8] * E[1];
    E[4] = E[8] * E[0] - E[6] * E[2];
    E[5] = E[6] * E[1] - E[7] * E[0];
    const float n = sqrtf(E[3] * E[3] + E[4] * E[4] + E[5] * E[5]);
    if (n > 0) { E[3] /= n; E[4] /= n; E[5] /= n; }
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
