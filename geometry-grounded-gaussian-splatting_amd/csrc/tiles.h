// tiles.h — tile rect and tile culling shared by the binning kernels
// (binning.hip, tilelists.hip).  Translation units including it compile with
// FMA contraction off: the spans are recomputed by several kernels and must
// agree bit for bit.
#pragma once

#include "gsr_common.h"

namespace gsr {

// Tile rect of Gaussian idx, the getRect of the reference (auxiliary.h:42-49);
// identical to the one preprocess_fwd.hip counted tiles_touched with.
struct TileRect {
    uint32_t x0, y0, x1, y1;
};
__device__ __forceinline__ TileRect tile_rect(float mx, float my, int r, uint32_t gx, uint32_t gy) {
    TileRect t;
    t.x0 = min(gx, (uint32_t)max(0, (int)((mx - r) / kTile)));
    t.y0 = min(gy, (uint32_t)max(0, (int)((my - r) / kTile)));
    t.x1 = min(gx, (uint32_t)max(0, (int)((mx + r + kTile - 1) / kTile)));
    t.y1 = min(gy, (uint32_t)max(0, (int)((my + r + kTile - 1) / kTile)));
    return t;
}

// Tile culling.  A pixel passes the reference's test alpha = min(0.99,
// o e^power) >= 1/255 only if Q(u, v) = a u^2 + 2 b u v + c v^2 <= tau =
// 2 ln(255 o), with (u, v) = mean - pixel centre and (a, b, c) the conic
// (power = -Q/2, render_forward.cu:486-487).  For a tile row (pixel centres
// v in [v_lo, v_hi]) the ellipse Q <= tau covers one interval of u: its ends
// are the concave/convex branches u = (-b v +- sqrt(a tau - det v^2)) / a,
// extremal at v = -+ b sqrt(tau / (c det)), so clamping that point into the
// band gives the exact interval; the row's live tiles are those whose pixel
// centres meet it — the same set as "the minimum of Q over the tile's pixel
// rectangle is <= tau", with tau raised by a margin (x1.001 + 0.01) far above
// the rounding of the per-pixel power and exp.  Non-positive-definite conics
// keep their whole rect; o < 1/255 keeps nothing.
// pad widens every tile by that many pixels on each side: 0 for the
// render path (pixel centres), 0.5 for sample_depth, whose points in tile tx
// lie anywhere in [16 tx - 0.5, 16 tx + 15.5) (createWithKeys,
// rasterizer_impl.cu:129-130).
struct Ellipse {
    float mx, my, a, b, c, det, tau, vmax, kst, ia, pad;
    int mode;  // 0 = interval test, 1 = whole rect, 2 = nothing
};
__device__ __forceinline__ Ellipse make_ellipse(const float4& w0, const float4& w1, float pad) {
    Ellipse E;
    E.pad = pad;
    E.mx = w0.x;
    E.my = w0.y;
    E.a = w0.z;
    E.b = w0.w;
    E.c = w1.x;
    const float o = w1.y;
    E.det = E.a * E.c - E.b * E.b;
    E.tau = 2.f * logf(fmaxf(255.f * o, 1.f)) * 1.001f + 0.01f;
    E.vmax = sqrtf(E.a * E.tau / E.det);
    E.kst = sqrtf(E.tau / (E.c * E.det));
    E.ia = 1.f / E.a;
    const bool pd = E.a > 0.f && E.c > 0.f && E.det > 0.f && E.vmax == E.vmax && E.kst == E.kst;
    E.mode = !(255.f * o >= 1.f) && o == o ? 2 : (pd ? 0 : 1);
    return E;
}
// Live tiles [*lo, *hi] of tile row ty inside rect R (false: none).
__device__ __forceinline__ bool row_span(const Ellipse& E, const TileRect& R, uint32_t ty, uint32_t* lo,
                                         uint32_t* hi) {
    if (E.mode == 2) return false;
    if (E.mode == 1) {
        *lo = R.x0;
        *hi = R.x1 - 1;
        return R.x1 > R.x0;
    }
    const float vlo = fmaxf(E.my - ((float)(ty * kTile + kTile - 1) + E.pad), -E.vmax);
    const float vhi = fminf(E.my - ((float)(ty * kTile) - E.pad), E.vmax);
    if (vlo > vhi) return false;
    const float vu = fminf(fmaxf(-E.b * E.kst, vlo), vhi);  // maximiser of the upper branch
    const float vl = fminf(fmaxf(E.b * E.kst, vlo), vhi);   // minimiser of the lower branch
    const float ia = E.ia;
    const float umax = (-E.b * vu + sqrtf(fmaxf(E.a * E.tau - E.det * vu * vu, 0.f))) * ia;
    const float umin = (-E.b * vl - sqrtf(fmaxf(E.a * E.tau - E.det * vl * vl, 0.f))) * ia;
    // pixel centres x in [mx - umax, mx - umin]; tile tx holds x in [16 tx - pad, 16 tx + 15 + pad]
    const float xlo = E.mx - umax, xhi = E.mx - umin;
    const int t0 = (int)ceilf((xlo - ((float)(kTile - 1) + E.pad)) * (1.f / kTile));
    const int t1 = (int)floorf((xhi + E.pad) * (1.f / kTile));
    const int l = max(t0, (int)R.x0), h = min(t1, (int)R.x1 - 1);
    if (l > h) return false;
    *lo = (uint32_t)l;
    *hi = (uint32_t)h;
    return true;
}
}  // namespace gsr
