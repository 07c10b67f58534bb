/*
 * median_sim.c — development tool (not product, not the oracle): simulates
 * median-depth root-finding strategies on real per-pixel contributor sets and
 * compares them with the reference's 5 x 8-way bisection
 * (render_forward.cu:549-645), counting per-wave walk steps so the GPU cost
 * of each strategy can be estimated before writing it in HIP.
 *
 * Input: the oracle's geometry (means2D, conic_opacity, ray_planes) and
 * binning (point_list, ranges) for the sampled tiles.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#define SPLIT 8
#define PASSES 5
#define RANGE 0.4f

typedef struct { float a, tp, rs; } contrib_t;

/* vacancy transmittance at t (reference formula, fp32) */
static float vac(const contrib_t* c, int n, float t) {
    float T = 1.f;
    for (int i = 0; i < n; i++) {
        const int ball = c[i].rs > 0;
        const float d = (t - c[i].tp) * c[i].rs;
        const float g = ball ? expf(-0.5f * d * d) : 0.f;
        const float omg = 1.f - c[i].a * g;
        T *= (t > c[i].tp ? 1.f - c[i].a : omg) * (1.f / sqrtf(omg));
    }
    return T;
}

/* log T and d log T / dt (h' as in the backward's dT/dtm / T, render_backward.cu:866-877) */
static void vac_d(const contrib_t* c, int n, float t, float* logT, float* dlog) {
    float A = 1.f, B = 1.f, D = 0.f;
    for (int i = 0; i < n; i++) {
        const int ball = c[i].rs > 0;
        const float d = (t - c[i].tp) * c[i].rs;
        const float g = ball ? expf(-0.5f * d * d) : 0.f;
        const float ag = c[i].a * g;
        const float omg = 1.f - ag;
        A *= t > c[i].tp ? 1.f - c[i].a : omg;
        B *= omg;
        if (ball) D += -0.5f * ag / omg * fabsf(d) * c[i].rs;
    }
    *logT = logf(A) - 0.5f * logf(B);
    *dlog = D;
}

static float ref_bisect(const contrib_t* c, int n, float m0, float Tfinal, int* in_range_out) {
    float Tp[SPLIT + 1];
    float lo = fmaxf(m0 - RANGE, 0.f), hi = fmaxf(m0 + RANGE, 0.f);
    int in_range = Tfinal <= 0.45f;
    for (int it = 0; it < PASSES; it++) {
        const int first = it == 0;
        const float iv = (hi - lo) * (1.f / SPLIT);
        for (int s = first ? 0 : 1; s < (first ? SPLIT + 1 : SPLIT); s++) Tp[s] = vac(c, n, lo + iv * s);
        if (first) in_range = Tp[0] >= 0.5f && Tp[SPLIT] <= 0.5f && in_range;
        int sid = 0;
        for (int p = 1; p < SPLIT; p++) sid = Tp[p] >= 0.5f ? p : sid;
        hi = lo + (sid + 1) * iv;
        lo = lo + sid * iv;
        Tp[0] = Tp[sid];
        Tp[SPLIT] = Tp[sid + 1];
    }
    float w = (Tp[0] - 0.5f) / (Tp[0] - Tp[SPLIT]);
    w = (w != w) ? 0.f : fminf(fmaxf(w, 0.f), 1.f);
    *in_range_out = in_range;
    return in_range ? w * hi + (1.f - w) * lo : 0.f;
}

/* Strategy: `npass` reference 8-way passes, then bracketed Newton on log T.
 * Returns the depth; *walks = Newton walks used; counts per-walk contributor
 * counts into wk[] (0 when the lane is done). */
static int g_halley = 0;
int g_dbg = 0;
static float g_sa, g_sb;
static int g_sel = 0;
static float g_smax = 1e30f;
static float g_hnoise = 0.f;
void sim_set_hnoise(float v) { g_hnoise = v; }
void sim_set_pred(int sel, float smax) { g_sel = sel; g_smax = smax; }
void sim_set_halley(int v) { g_halley = v; }
/* h, h', h'' of h = log T + ln 2 */
static float g_lastF = 0.f;  /* sum |e| of the last vac_d2 (a bound on |H''| either side of a splat peak) */
static float g_loose = 0.f, g_tolF = 0.f;
void sim_set_loose(float loose_rel, float tolF) { g_loose = loose_rel; g_tolF = tolF; }
static void vac_d2(const contrib_t* c, int n, float t, float* hv, float* d1, float* d2) {
    float A = 1.f, B = 1.f, D = 0.f, E = 0.f, F = 0.f;
    for (int i = 0; i < n; i++) {
        const int ball = c[i].rs > 0;
        const float d = (t - c[i].tp) * c[i].rs;
        const float g = ball ? expf(-0.5f * d * d) : 0.f;
        const float ag = c[i].a * g;
        const float omg = 1.f - ag;
        const int before = !(t > c[i].tp);
        A *= before ? omg : 1.f - c[i].a;
        B *= omg;
        if (ball) {
            const float x = ag / omg;
            D += -0.5f * x * fabsf(d) * c[i].rs;
            const float e = 0.5f * c[i].rs * c[i].rs * x * (1.f - d * d * (1.f + x));
            E += before ? e : -e;
            F += fabsf(e);
        }
    }
    g_lastF = F;
    *hv = logf(A) - 0.5f * logf(B) + 0.69314718f;
    *d1 = D;
    *d2 = E;
}
static float newton_strategy(const contrib_t* c, int n, float m0, float Tfinal, int npass, float tol_rel,
                             int maxit, int* walks, int* in_range_out, int* fell_back) {
    float Tp[SPLIT + 1];
    float lo = fmaxf(m0 - RANGE, 0.f), hi = fmaxf(m0 + RANGE, 0.f);
    int in_range = Tfinal <= 0.45f;
    *walks = 0;
    *fell_back = 0;
    for (int it = 0; it < npass; it++) {
        const int first = it == 0;
        const float iv = (hi - lo) * (1.f / SPLIT);
        for (int s = first ? 0 : 1; s < (first ? SPLIT + 1 : SPLIT); s++) Tp[s] = vac(c, n, lo + iv * s);
        if (first) in_range = Tp[0] >= 0.5f && Tp[SPLIT] <= 0.5f && in_range;
        int sid = 0;
        for (int p = 1; p < SPLIT; p++) sid = Tp[p] >= 0.5f ? p : sid;
        hi = lo + (sid + 1) * iv;
        lo = lo + sid * iv;
        Tp[0] = Tp[sid];
        Tp[SPLIT] = Tp[sid + 1];
    }
    *in_range_out = in_range;
    {
        float sa = 0.f, sb = 0.f;
        const float wl = lo - (hi - lo) * 3.5f, wh = hi + (hi - lo) * 3.5f; /* pass-2 window */
        for (int i = 0; i < n; i++) {
            if (c[i].rs <= 0.f) continue;
            const int near_cell = !((lo - c[i].tp) * c[i].rs > 6.f || (hi - c[i].tp) * c[i].rs < -6.f);
            const int near_win = !((wl - c[i].tp) * c[i].rs > 6.f || (wh - c[i].tp) * c[i].rs < -6.f);
            if (near_cell && c[i].rs > sa) sa = c[i].rs;
            if (near_win && c[i].rs > sb) sb = c[i].rs;
        }
        g_sa = sa * (hi - lo);
        g_sb = sb * (hi - lo);
    }
    if (!in_range) return 0.f;
    const float lo2 = lo, hi2 = hi;
    /* bracket [lo, hi]: T(lo) >= 0.5 >= T(hi) (h = log T + ln 2) */
    float t;
    if (npass == 0) {
        /* walk 1 also gives T at the window ends (in_range) */
        Tp[0] = vac(c, n, lo);
        Tp[SPLIT] = vac(c, n, hi);
        in_range = Tp[0] >= 0.5f && Tp[SPLIT] <= 0.5f && in_range;
        *in_range_out = in_range;
        if (!in_range) return 0.f;
        t = fminf(fmaxf(m0, lo), hi);
    } else {
        float hlo = logf(Tp[0]) + 0.69314718f, hhi = logf(Tp[SPLIT]) + 0.69314718f;
        float w = hlo / (hlo - hhi);
        w = (w != w) ? 0.5f : fminf(fmaxf(w, 0.f), 1.f);
        t = lo + w * (hi - lo);
    }
    const float tol = tol_rel * fmaxf(t, 1.f);
    for (int k = 0; k < maxit; k++) {
        float h, dh, d2 = 0.f;
        vac_d2(c, n, t, &h, &dh, &d2);
        (*walks)++;
        if (h >= 0.f) lo = t; else hi = t;
        float tn;
        if (g_halley) {
            const float den = 2.f * dh * dh - h * d2;
            tn = den != 0.f ? t - 2.f * h * dh / den : 0.5f * (lo + hi);
        } else {
            tn = dh < 0.f ? t - h / dh : 0.5f * (lo + hi);
        }
        int bis = 0;
        if (!(tn >= lo && tn <= hi)) { tn = 0.5f * (lo + hi); bis = 1; }
        const float step = fabsf(tn - t);
        t = tn;
        if (bis) *fell_back += 1;
        if (g_dbg) fprintf(stderr, "walk %d t=%.7f h=%g d1=%g d2=%g tn=%.7f lo=%.7f hi=%.7f\n", k, t, h, dh, d2, tn, lo, hi);
        if ((dh < 0.f && fabsf(h) <= tol * -dh) || hi - lo <= tol) {
            /* well-conditioned root only: ulp noise in log2 T (~kHNoise) must move it by < tol */
            if (-dh / 0.69314718f * tol >= g_hnoise) return t;
            break;
        }
    }
    lo = lo2; hi = hi2; /* fallback: the reference's remaining passes from the pass-2 cell */
    /* not converged: 8-way passes on the bracket down to the reference's final width */
    {
        const float wfinal = 2.f * RANGE / 32768.f;
        float Tlo = Tp[0], Thi = Tp[SPLIT];
        for (int it = npass; it < PASSES; it++) {
            const float iv = (hi - lo) * (1.f / SPLIT);
            float Tp[SPLIT + 1];
            Tp[0] = Tlo; Tp[SPLIT] = Thi;
            for (int s2 = 1; s2 < SPLIT; s2++) Tp[s2] = vac(c, n, lo + iv * s2);
            int sid = 0;
            for (int p = 1; p < SPLIT; p++) sid = Tp[p] >= 0.5f ? p : sid;
            hi = lo + (sid + 1) * iv;
            lo = lo + sid * iv;
            Tlo = Tp[sid]; Thi = Tp[sid + 1];
            if (g_dbg) fprintf(stderr, "fb sid %d lo=%.7f hi=%.7f Tlo=%g Thi=%g\n", sid, lo, hi, Tlo, Thi);
            *walks += 100;
        }
        float w = (Tlo - 0.5f) / (Tlo - Thi);
        w = (w != w) ? 0.f : fminf(fmaxf(w, 0.f), 1.f);
        return w * hi + (1.f - w) * lo;
    }
}

/* per-pixel composite over the tile list: blended set, T, m0 */
static int composite(const uint32_t* list, int cnt, const float* xy, const float* co, const float* rp, float px,
                     float py, contrib_t* out, float* Tfin, float* m0) {
    float T = 1.f, mi = 0.f;
    int n = 0;
    for (int k = 0; k < cnt; k++) {
        const uint32_t g = list[k];
        const float dx = xy[2 * g] - px, dy = xy[2 * g + 1] - py;
        const float* c4 = co + 4 * g;
        const float power = -0.5f * (c4[0] * dx * dx + c4[2] * dy * dy) - c4[1] * dx * dy;
        if (power > 0.f) continue;
        const float alpha = fminf(0.99f, c4[3] * expf(power));
        if (alpha < 1.f / 255.f) continue;
        const float tT = T * (1.f - alpha);
        if (tT < 1e-4f) break;
        const float* r = rp + 4 * g;
        const float t = r[0] * dx + r[1] * dy + r[2];
        mi = T > 0.5f ? t : mi;
        out[n].a = alpha;
        out[n].tp = t;
        out[n].rs = r[3];
        n++;
        T = tT;
    }
    *Tfin = T;
    *m0 = mi;
    return n;
}

/* stats: [0] pixels, [1] in_range, [2] max |d|, [4] sum walks, [5] ref cost, [6] strategy cost,
 * [7] bisect fallbacks inside the walk loop, [8] in_range mismatches, [9] lanes needing the pass fallback,
 * [10] sum blended, [11] non-ball, [12..27] walk histogram.
 * Cost model per contributor-step: first pass 1.2, later pass 1.0, walk `wcost`. */
void sim_run(int W, int H, int gx, int ntiles, const uint32_t* tiles, const uint32_t* ranges,
             const uint32_t* point_list, const float* xy, const float* co, const float* rp, int npass,
             float tol_rel, int maxit, float wcost, double* stats, float* md_ref_out, float* md_new_out) {
    contrib_t* buf = malloc(sizeof(contrib_t) * 65536);
    for (int ti = 0; ti < ntiles; ti++) {
        const uint32_t tile = tiles[ti];
        const uint32_t tx = tile % gx, ty = tile / gx;
        const uint32_t r0 = ranges[2 * tile], r1 = ranges[2 * tile + 1];
        for (int wv = 0; wv < 4; wv++) {
            int lane_n[64], lane_walks[64], lane_fb[64];
            float lane_s[64];
            int nmax = 0;
            for (int l = 0; l < 64; l++) {
                const int px = tx * 16 + (l & 15), py = ty * 16 + wv * 4 + (l >> 4);
                lane_n[l] = lane_walks[l] = lane_fb[l] = 0;
                lane_s[l] = 0.f;
                const int pidx = ti * 256 + wv * 64 + l;
                md_ref_out[pidx] = 0.f;
                md_new_out[pidx] = 0.f;
                if (px >= W || py >= H) continue;
                float Tf, m0;
                const int n = composite(point_list + r0, (int)(r1 - r0), xy, co, rp, (float)px, (float)py, buf,
                                        &Tf, &m0);
                stats[0] += 1;
                stats[10] += n;
                for (int i = 0; i < n; i++) stats[11] += buf[i].rs <= 0.f;
                int ir1, ir2, walks, fb;
                const float mr = ref_bisect(buf, n, m0, Tf, &ir1);
                g_dbg = (px == 394 && py == 792);
                const float mn = newton_strategy(buf, n, m0, Tf, npass, tol_rel, maxit, &walks, &ir2, &fb);
                md_ref_out[pidx] = mr;
                md_new_out[pidx] = mn;
                stats[1] += ir1;
                stats[8] += ir1 != ir2;
                const double d = fabs((double)mr - mn);
                if (d > stats[2]) stats[2] = d;
                stats[4] += walks % 100;
                stats[7] += fb;
                stats[9] += walks >= 100;
                stats[12 + (walks % 100 < 15 ? walks % 100 : 15)] += 1;
                if (ir1) {
                    const float sv = g_sel ? g_sb : g_sa;
                    int b = sv <= 0.25f ? 0 : sv <= 0.5f ? 1 : sv <= 1.f ? 2 : sv <= 2.f ? 3 : sv <= 4.f ? 4 : 5;
                    stats[32 + b * 3] += 1;
                    stats[32 + b * 3 + 1] += walks >= 100;
                    stats[32 + b * 3 + 2] += walks % 100;
                    lane_s[l] = sv;
                }
                if (ir1) {
                    lane_n[l] = n;
                    lane_walks[l] = walks % 100;
                    lane_fb[l] = walks / 100;
                }
                if (lane_n[l] > nmax) nmax = lane_n[l];
            }
            stats[5] += nmax * (1.2 + (PASSES - 1));
            {
                int smooth = 1;
                for (int l = 0; l < 64; l++) smooth &= lane_s[l] <= g_smax;
                stats[50] += smooth;
                stats[51] += 1;
                if (!smooth) {
                    stats[6] += nmax * (1.2 + (PASSES - 1));
                    continue;
                }
            }
            stats[6] += npass > 0 ? nmax * (1.2 + (npass - 1)) : 0;
            for (int k = 0; k < maxit; k++) {
                int m = 0;
                for (int l = 0; l < 64; l++)
                    if (lane_walks[l] > k && lane_n[l] > m) m = lane_n[l];
                stats[6] += m * wcost;
            }
            for (int k = 0; k < 4; k++) {
                int m = 0;
                for (int l = 0; l < 64; l++)
                    if (lane_fb[l] > k && lane_n[l] > m) m = lane_n[l];
                stats[6] += m;
            }
        }
    }
    free(buf);
}

/* near-set sizes: contributors within 6 sigma of the pass-1 window, of the
 * pass-1 cell (pass-2 window) and of the pass-2 cell, plus those wholly in
 * front of each (a (1 - a) factor).  out[0] pixels, [1] sum n, [2..4] near
 * counts, [5..7] in-front counts, [8..10] wave-max near counts. */
void sim_nearsets(int W, int H, int gx, int ntiles, const uint32_t* tiles, const uint32_t* ranges,
                  const uint32_t* point_list, const float* xy, const float* co, const float* rp, double* out) {
    contrib_t* buf = malloc(sizeof(contrib_t) * 65536);
    for (int ti = 0; ti < ntiles; ti++) {
        const uint32_t tile = tiles[ti];
        const uint32_t tx = tile % gx, ty = tile / gx;
        const uint32_t r0 = ranges[2 * tile], r1 = ranges[2 * tile + 1];
        for (int wv = 0; wv < 4; wv++) {
            int wmax[3] = {0, 0, 0};
            for (int l = 0; l < 64; l++) {
                const int px = tx * 16 + (l & 15), py = ty * 16 + wv * 4 + (l >> 4);
                if (px >= W || py >= H) continue;
                float Tf, m0;
                const int n = composite(point_list + r0, (int)(r1 - r0), xy, co, rp, (float)px, (float)py, buf, &Tf, &m0);
                out[0] += 1;
                out[1] += n;
                float lo = fmaxf(m0 - RANGE, 0.f), hi = fmaxf(m0 + RANGE, 0.f);
                float Tp[SPLIT + 1];
                for (int it = 0; it < 3; it++) {
                    int near = 0, front = 0;
                    for (int i = 0; i < n; i++) {
                        const float rs = buf[i].rs;
                        const int beh = rs > 0 && (lo - buf[i].tp) * rs > 6.f;
                        const int fr = rs > 0 && (hi - buf[i].tp) * rs < -6.f;
                        near += !(beh || fr);
                        front += beh;
                    }
                    out[2 + it] += near;
                    out[5 + it] += front;
                    if (near > wmax[it]) wmax[it] = near;
                    if (it == 2) break;
                    const float iv = (hi - lo) * (1.f / SPLIT);
                    for (int s = 0; s <= SPLIT; s++) Tp[s] = vac(buf, n, lo + iv * s);
                    int sid = 0;
                    for (int p = 1; p < SPLIT; p++) sid = Tp[p] >= 0.5f ? p : sid;
                    hi = lo + (sid + 1) * iv;
                    lo = lo + sid * iv;
                }
            }
            for (int k = 0; k < 3; k++) out[8 + k] += wmax[k];
            out[11] += 1;
        }
    }
    free(buf);
}

/* root - m0 per in-range pixel (out_d), the reference's median depth minus m0 */
void sim_root_offsets(int W, int H, int gx, int ntiles, const uint32_t* tiles, const uint32_t* ranges,
                      const uint32_t* point_list, const float* xy, const float* co, const float* rp, float* out_d,
                      float* out_sig) {
    contrib_t* buf = malloc(sizeof(contrib_t) * 65536);
    for (int ti = 0; ti < ntiles; ti++) {
        const uint32_t tile = tiles[ti];
        const uint32_t tx = tile % gx, ty = tile / gx;
        const uint32_t r0 = ranges[2 * tile], r1 = ranges[2 * tile + 1];
        for (int l = 0; l < 256; l++) {
            const int px = tx * 16 + (l & 15), py = ty * 16 + (l >> 4);
            out_d[ti * 256 + l] = NAN;
            if (px >= W || py >= H) continue;
            float Tf, m0;
            const int n = composite(point_list + r0, (int)(r1 - r0), xy, co, rp, (float)px, (float)py, buf, &Tf, &m0);
            int ir;
            const float md = ref_bisect(buf, n, m0, Tf, &ir);
            if (!ir) continue;
            out_d[ti * 256 + l] = md - m0;
            float sg = 0.f;
            for (int i = 0; i < n; i++) if (buf[i].tp == m0) sg = buf[i].rs;
            out_sig[ti * 256 + l] = sg;
        }
    }
    free(buf);
}

/* Strategy S2: walk 1 evaluates T at the window ends (in_range) and at m0 + off[k] (nk offsets, sorted,
 * one of them 0 where h, h', h'' are taken too); the bracket is the tightest pair of samples around the
 * crossing; then bracketed Halley walks (one point each) until |h / h'| <= tol or the bracket is <= tol.
 * Lanes not converged in maxit walks or ill-conditioned fall back to the reference's 5 passes.
 * out: [0] in-range lanes, [1] sum walks (after walk 1), [2] fallbacks, [3] max |d|, [4] waves,
 * [5] sum over waves of the max walks (fallback lanes counted as 100), [6..21] wave-max histogram,
 * [22..37] lane walk hist, [40] in_range mismatches */
void sim_s2(int W, int H, int gx, int ntiles, const uint32_t* tiles, const uint32_t* ranges,
            const uint32_t* point_list, const float* xy, const float* co, const float* rp, int nk, const float* off,
            float tol_rel, float tol_abs, int maxit, float hnoise, double* out) {
    contrib_t* buf = malloc(sizeof(contrib_t) * 65536);
    for (int ti = 0; ti < ntiles; ti++) {
        const uint32_t tile = tiles[ti];
        const uint32_t tx = tile % gx, ty = tile / gx;
        const uint32_t r0 = ranges[2 * tile], r1 = ranges[2 * tile + 1];
        for (int wv = 0; wv < 4; wv++) {
            int wmax = 0;
            for (int l = 0; l < 64; l++) {
                const int px = tx * 16 + (l & 15), py = ty * 16 + wv * 4 + (l >> 4);
                if (px >= W || py >= H) continue;
                float Tf, m0;
                const int n = composite(point_list + r0, (int)(r1 - r0), xy, co, rp, (float)px, (float)py, buf, &Tf, &m0);
                int ir;
                const float mr = ref_bisect(buf, n, m0, Tf, &ir);
                const float dmin = fmaxf(m0 - RANGE, 0.f), dmax = fmaxf(m0 + RANGE, 0.f);
                const float T0 = vac(buf, n, dmin), T8 = vac(buf, n, dmax);
                const int ir2 = T0 >= 0.5f && T8 <= 0.5f && Tf <= 0.45f;
                out[40] += ir != ir2;
                if (!ir2) continue;
                out[0] += 1;
                float lo = dmin, hi = dmax, hlo = logf(T0) + 0.69314718f, hhi = logf(T8) + 0.69314718f;
                float h0 = 0, d1 = 0, d2 = 0, tm = fminf(fmaxf(m0, dmin), dmax);
                for (int k = 0; k < nk; k++) {
                    const float t = m0 + off[k];
                    if (!(t > lo && t < hi)) continue;
                    float h;
                    if (off[k] == 0.f) { vac_d2(buf, n, t, &h, &d1, &d2); h0 = h; }
                    else h = logf(vac(buf, n, t)) + 0.69314718f;
                    if (h >= 0.f) { if (t > lo) { lo = t; hlo = h; } }
                    else { if (t < hi) { hi = t; hhi = h; } }
                }
                /* re-tighten: samples in increasing order, so lo/hi are the last >= 0 / first < 0 only if
                 * monotone; fine for the sim */
                float t;
                {
                    const float den = 2.f * d1 * d1 - h0 * d2;
                    t = den != 0.f ? tm - 2.f * h0 * d1 / den : 0.5f * (lo + hi);
                    if (getenv("SIM_INIT") && atoi(getenv("SIM_INIT")) == 1) t = -1.f;
                    if (!(t >= lo && t <= hi)) {
                        float w = hlo / (hlo - hhi);
                        w = (w != w) ? 0.5f : fminf(fmaxf(w, 0.f), 1.f);
                        t = lo + w * (hi - lo);
                    }
                }
                const float tol = fmaxf(tol_rel * fmaxf(t, 1.f), tol_abs);
                int walks = 0, ok = 0;
                float res = 0.f;
                for (int k = 0; k < maxit; k++) {
                    float h, dh, dd;
                    vac_d2(buf, n, t, &h, &dh, &dd);
                    walks++;
                    if (h >= 0.f) lo = t; else hi = t;
                    const float den = 2.f * dh * dh - h * dd;
                    float tn = den != 0.f ? t - 2.f * h * dh / den : 0.5f * (lo + hi);
                    if (!(tn >= lo && tn <= hi)) tn = 0.5f * (lo + hi);
                    if ((dh < 0.f && fabsf(h) <= tol * -dh) || hi - lo <= tol) {
                        if (-dh * tol >= hnoise) { ok = 1; res = tn; }
                        break;
                    }
                    t = tn;
                }
                if (!ok) { out[2] += 1; walks = 100; res = mr; }
                else out[1] += walks;
                out[22 + (walks < 15 ? walks : 15)] += 1;
                const double d = fabs((double)res - mr);
                if (d > out[3]) out[3] = d;
                if (walks > wmax) wmax = walks;
            }
            out[4] += 1;
            out[5] += wmax;
            out[6 + (wmax < 15 ? wmax : 15)] += 1;
        }
    }
    free(buf);
}

/* |secant estimate - reference depth| and |Halley-from-secant - reference| after the probe walk (S2's walk 1) */
void sim_secant_err(int W, int H, int gx, int ntiles, const uint32_t* tiles, const uint32_t* ranges,
                    const uint32_t* point_list, const float* xy, const float* co, const float* rp, int nk,
                    const float* off, float* out_sec, float* out_hal, float* out_quad) {
    contrib_t* buf = malloc(sizeof(contrib_t) * 65536);
    for (int ti = 0; ti < ntiles; ti++) {
        const uint32_t tile = tiles[ti];
        const uint32_t tx = tile % gx, ty = tile / gx;
        const uint32_t r0 = ranges[2 * tile], r1 = ranges[2 * tile + 1];
        for (int l = 0; l < 256; l++) {
            const int px = tx * 16 + (l & 15), py = ty * 16 + (l >> 4);
            const int o = ti * 256 + l;
            out_sec[o] = out_hal[o] = out_quad[o] = NAN;
            if (px >= W || py >= H) continue;
            float Tf, m0;
            const int n = composite(point_list + r0, (int)(r1 - r0), xy, co, rp, (float)px, (float)py, buf, &Tf, &m0);
            int ir;
            const float mr = ref_bisect(buf, n, m0, Tf, &ir);
            if (!ir) continue;
            float ts[32], hs[32];
            const float dmin = fmaxf(m0 - RANGE, 0.f), dmax = fmaxf(m0 + RANGE, 0.f);
            int m = 0;
            ts[m++] = dmin;
            for (int k = 0; k < nk; k++) ts[m++] = fminf(fmaxf(m0 + off[k], dmin), dmax);
            ts[m++] = dmax;
            for (int k = 0; k < m; k++) hs[k] = logf(vac(buf, n, ts[k])) + 0.69314718f;
            int k1 = 0;
            for (int k = 1; k < m - 1; k++) if (hs[k] >= 0.f) k1 = k;
            const float lo = ts[k1], hi = ts[k1 + 1];
            float w = hs[k1] / (hs[k1] - hs[k1 + 1]);
            w = (w != w) ? 0.5f : fminf(fmaxf(w, 0.f), 1.f);
            const float t = lo + w * (hi - lo);
            out_sec[o] = t - mr;
            float h, d1, d2;
            vac_d2(buf, n, t, &h, &d1, &d2);
            const float den = 2.f * d1 * d1 - h * d2;
            out_hal[o] = (den != 0.f ? t - 2.f * h * d1 / den : t) - mr;
            /* inverse quadratic through 3 probes around the crossing */
            int a0 = k1 > 0 ? k1 - 1 : 0;
            if (a0 + 2 >= m) a0 = m - 3;
            const float x0 = hs[a0], x1 = hs[a0 + 1], x2 = hs[a0 + 2];
            const float y0 = ts[a0], y1 = ts[a0 + 1], y2 = ts[a0 + 2];
            float q = y0 * x1 * x2 / ((x0 - x1) * (x0 - x2)) + y1 * x0 * x2 / ((x1 - x0) * (x1 - x2)) +
                      y2 * x0 * x1 / ((x2 - x0) * (x2 - x1));
            if (!(q >= lo && q <= hi)) q = t;
            out_quad[o] = q - mr;
        }
    }
    free(buf);
}

/* S3: probe walk, then alternating Halley walks (H, H', H'' at t -> tn) and verification walks (T at
 * tn -+ eps: the root bracketed within eps of tn -> done, result = log-secant in [tn - eps, tn + eps]);
 * a failed verification is followed by another Halley walk from tn.  maxit Halley walks.
 * out: [0] lanes, [1] max |d|, [2] fallbacks, [3] waves, [4] sum wave cost (walk units: halley 1,
 * verify vcost), [5..20] lane hist of halley walks */
void sim_s3(int W, int H, int gx, int ntiles, const uint32_t* tiles, const uint32_t* ranges,
            const uint32_t* point_list, const float* xy, const float* co, const float* rp, int nk, const float* off,
            float eps_rel, int maxit, float hnoise, double* out, float* dout) {
    contrib_t* buf = malloc(sizeof(contrib_t) * 65536);
    for (int ti = 0; ti < ntiles; ti++) {
        const uint32_t tile = tiles[ti];
        const uint32_t tx = tile % gx, ty = tile / gx;
        const uint32_t r0 = ranges[2 * tile], r1 = ranges[2 * tile + 1];
        for (int wv = 0; wv < 4; wv++) {
            int seq[64];  /* per lane: number of (halley, verify) rounds used */
            int nl = 0, wmax = 0;
            for (int l = 0; l < 64; l++) {
                const int px = tx * 16 + (l & 15), py = ty * 16 + wv * 4 + (l >> 4);
                dout[ti * 256 + wv * 64 + l] = 0.f;
                seq[l] = 0;
                if (px >= W || py >= H) continue;
                float Tf, m0;
                const int n = composite(point_list + r0, (int)(r1 - r0), xy, co, rp, (float)px, (float)py, buf, &Tf, &m0);
                int ir;
                const float mr = ref_bisect(buf, n, m0, Tf, &ir);
                if (!ir) continue;
                out[0] += 1;
                float ts[32], hs[32];
                const float dmin = fmaxf(m0 - RANGE, 0.f), dmax = fmaxf(m0 + RANGE, 0.f);
                int m = 0;
                ts[m++] = dmin;
                for (int k = 0; k < nk; k++) ts[m++] = fminf(fmaxf(m0 + off[k], dmin), dmax);
                ts[m++] = dmax;
                for (int k = 0; k < m; k++) hs[k] = logf(vac(buf, n, ts[k])) + 0.69314718f;
                int k1 = 0;
                for (int k = 1; k < m - 1; k++) if (hs[k] >= 0.f) k1 = k;
                float lo = ts[k1], hi = ts[k1 + 1];
                float w = hs[k1] / (hs[k1] - hs[k1 + 1]);
                w = (w != w) ? 0.5f : fminf(fmaxf(w, 0.f), 1.f);
                float t = lo + w * (hi - lo);
                const float eps = eps_rel * fmaxf(t, 1.f);
                int rounds = 0, ok = 0;
                float res = 0.f;
                for (int k = 0; k < maxit && !ok; k++) {
                    float h, dh, dd;
                    vac_d2(buf, n, t, &h, &dh, &dd);
                    rounds++;
                    if (h >= 0.f) lo = t; else hi = t;
                    const float den = 2.f * dh * dh - h * dd;
                    float tn = den != 0.f ? t - 2.f * h * dh / den : 0.5f * (lo + hi);
                    if (!(tn >= lo && tn <= hi)) tn = 0.5f * (lo + hi);
                    /* verification walk */
                    const float a = tn - eps, b = tn + eps;
                    const float ha = logf(vac(buf, n, a)) + 0.69314718f, hb = logf(vac(buf, n, b)) + 0.69314718f;
                    if (ha >= 0.f && hb < 0.f) {
                        if (-dh * 1e-6f * fmaxf(t, 1.f) >= hnoise) {
                            float ww = ha / (ha - hb);
                            ww = (ww != ww) ? 0.5f : fminf(fmaxf(ww, 0.f), 1.f);
                            res = a + ww * (b - a);
                            ok = 1;
                        }
                        break;
                    }
                    if (ha >= 0.f) lo = fmaxf(lo, a); else hi = fminf(hi, a);
                    if (hb >= 0.f) lo = fmaxf(lo, b); else hi = fminf(hi, b);
                    t = tn;
                }
                if (!ok) { out[2] += 1; rounds = 100; res = mr; }
                out[5 + (rounds < 15 ? rounds : 15)] += 1;
                const double d = fabs((double)res - mr);
                dout[ti * 256 + wv * 64 + l] = (float)d;
                if (d > out[1]) out[1] = d;
                seq[l] = rounds;
                if (rounds > wmax) wmax = rounds;
                nl++;
            }
            out[3] += 1;
            out[4] += wmax;
        }
    }
    free(buf);
}

/* Reference median depth of every pixel of the sampled tiles (0 where not in range): out[ti*256 + l]. */
void sim_ref_depths(int W, int H, int gx, int ntiles, const uint32_t* tiles, const uint32_t* ranges,
                    const uint32_t* point_list, const float* xy, const float* co, const float* rp, float* out,
                    float* out_m0) {
    contrib_t* buf = malloc(sizeof(contrib_t) * 65536);
    for (int ti = 0; ti < ntiles; ti++) {
        const uint32_t tile = tiles[ti];
        const uint32_t tx = tile % gx, ty = tile / gx;
        const uint32_t r0 = ranges[2 * tile], r1 = ranges[2 * tile + 1];
        for (int l = 0; l < 256; l++) {
            const int px = tx * 16 + (l & 15), py = ty * 16 + (l >> 4);
            out[ti * 256 + l] = 0.f;
            out_m0[ti * 256 + l] = 0.f;
            if (px >= W || py >= H) continue;
            float Tf, m0;
            const int n = composite(point_list + r0, (int)(r1 - r0), xy, co, rp, (float)px, (float)py, buf, &Tf, &m0);
            int ir;
            out[ti * 256 + l] = ref_bisect(buf, n, m0, Tf, &ir);
            out_m0[ti * 256 + l] = m0;
        }
    }
    free(buf);
}

/* S4: grid pixels (even x, even y of a tile: 64) find their root with S2 (probe walk + Halley from the
 * log-secant); the other 192 start bracketed Halley walks from the average of their tile's grid neighbours'
 * roots (walk 1 also samples the window ends for in_range).  out: [0] lanes, [1] max|d|, [2] fallbacks,
 * [3] sum of phase-1 wave max walks, [4] phase-1 waves, [5] sum of phase-2 wave max walks, [6] phase-2 waves,
 * [8..23] phase-2 lane walk hist, [24] lanes without a grid guess */
static long g_why_ill, g_why_nc, g_why_ok;  /* fallback reasons: ill-conditioned / not converged */
static double g_why_D[8];  /* ill-conditioned: histogram of log10(D * scale) */
void sim_why(long* o) { o[0] = g_why_ok; o[1] = g_why_ill; o[2] = g_why_nc; for (int i = 0; i < 8; i++) o[3 + i] = (long)g_why_D[i]; }
static float g_last_t, g_last_lo, g_last_hi;  /* the iterate and bracket a non-converged call stopped at */
static int halley_from(const contrib_t* c, int n, float t, float lo, float hi, float tol_rel, int maxit,
                       float hnoise, float* res) {
    const float tol = tol_rel * fmaxf(t, 1.f);
    int walks = 0;
    for (int k = 0; k < maxit; k++) {
        float h, dh, dd;
        vac_d2(c, n, t, &h, &dh, &dd);
        walks++;
        if (h >= 0.f) lo = t; else hi = t;
        const float den = 2.f * dh * dh - h * dd;
        float tn = den != 0.f ? t - 2.f * h * dh / den : 0.5f * (lo + hi);
        if (!(tn >= lo && tn <= hi)) tn = 0.5f * (lo + hi);
        const float sc = fmaxf(t, 1.f), D = -dh;
        const int loose = g_loose > 0.f && D > 0.f && fabsf(h) <= g_loose * sc * D &&
                          fabsf(h) * g_lastF <= g_tolF * D * D;  /* step x curvature (F / D) <= tolF */
        if ((dh < 0.f && fabsf(h) <= tol * -dh) || hi - lo <= tol || loose) {
            if (-dh * 1e-6f * fmaxf(t, 1.f) >= hnoise) { *res = tn; g_why_ok++; return walks; }
            g_why_ill++;
            { double v = log10(fmax(-dh * fmaxf(t, 1.f), 1e-30)); int b = (int)floor(v) + 4; b = b < 0 ? 0 : b > 7 ? 7 : b; g_why_D[b] += 1; }
            return -walks;
        }
        t = tn;
        g_last_t = t;
        g_last_lo = lo;
        g_last_hi = hi;
    }
    g_why_nc++;
    return -walks;
}
void sim_s4(int W, int H, int gx, int ntiles, const uint32_t* tiles, const uint32_t* ranges,
            const uint32_t* point_list, const float* xy, const float* co, const float* rp, int nk, const float* off,
            float tol_rel, int maxit, float hnoise, double* out) {
    contrib_t* buf = malloc(sizeof(contrib_t) * 65536);
    const int G = getenv("SIM_GRID") ? atoi(getenv("SIM_GRID")) : 2;  /* grid stride of phase 1 */
    for (int ti = 0; ti < ntiles; ti++) {
        const uint32_t tile = tiles[ti];
        const uint32_t tx = tile % gx, ty = tile / gx;
        const uint32_t r0 = ranges[2 * tile], r1 = ranges[2 * tile + 1];
        float root[256];
        int have[256], walksv[256];
        /* phase 1: grid pixels */
        int wmax1 = 0;
        for (int l = 0; l < 256; l++) {
            have[l] = 0;
            walksv[l] = 0;
            const int lx = l & 15, ly = l >> 4;
            if ((lx % G) || (ly % G)) continue;
            const int px = tx * 16 + lx, py = ty * 16 + ly;
            if (px >= W || py >= H) continue;
            float Tf, m0;
            const int n = composite(point_list + r0, (int)(r1 - r0), xy, co, rp, (float)px, (float)py, buf, &Tf, &m0);
            int ir;
            const float mr = ref_bisect(buf, n, m0, Tf, &ir);
            if (!ir) continue;
            out[0] += 1;
            float ts[32], hs[32];
            const float dmin = fmaxf(m0 - RANGE, 0.f), dmax = fmaxf(m0 + RANGE, 0.f);
            if (getenv("SIM_P1")) {  /* variant: Halley from m0 in the window, no probe walk */
                float res = mr;
                int wk = halley_from(buf, n, fminf(fmaxf(m0, dmin), dmax), dmin, dmax, tol_rel, maxit, hnoise, &res);
                if (wk < 0) { out[2] += 1; res = mr; wk = 100; }
                out[25 + (wk < 6 ? wk : 6)] += 1;
                root[l] = res;
                have[l] = 1;
                const double d = fabs((double)res - mr);
                if (d > out[1]) out[1] = d;
                if (wk > wmax1) wmax1 = wk;
                continue;
            }
            int m = 0;
            const int noends = getenv("SIM_NOENDS") != NULL;  /* the GPU's probe walk since round 4 */
            if (!noends) ts[m++] = dmin;
            for (int k = 0; k < nk; k++) ts[m++] = fminf(fmaxf(m0 + off[k], dmin), dmax);
            if (!noends) ts[m++] = dmax;
            for (int k = 0; k < m; k++) hs[k] = logf(vac(buf, n, ts[k])) + 0.69314718f;
            if (noends && !(hs[0] >= 0.f && hs[m - 1] <= 0.f)) {  /* unbracketed: left to the passes */
                out[2] += 1;
                out[42] += 1;
                root[l] = mr;
                have[l] = 0;
                continue;
            }
            int k1 = 0;
            for (int k = 1; k < m - 1; k++) if (hs[k] >= 0.f) k1 = k;
            float w = hs[k1] / (hs[k1] - hs[k1 + 1]);
            w = (w != w) ? 0.5f : fminf(fmaxf(w, 0.f), 1.f);
            float t0 = ts[k1] + w * (ts[k1 + 1] - ts[k1]);
            if (getenv("SIM_P1_INTERP")) {  /* variant: the root of the cubic through 4 probes around the bracket */
                int a0 = k1 - 1;
                if (a0 < 0) a0 = 0;
                if (a0 + 3 > m - 1) a0 = m - 4;
                if (a0 >= 0) {
                    const float* X = ts + a0;
                    const float* Y = hs + a0;
                    int ok = 1;
                    for (int q = 0; q < 3; q++) ok = ok && X[q + 1] > X[q];
                    if (ok) {
                        /* Newton on the Lagrange cubic from the secant guess, kept in the bracket */
                        float x = t0;
                        for (int it = 0; it < 8; it++) {
                            double P = 0, dP = 0;
                            for (int i = 0; i < 4; i++) {
                                double li = 1, dli = 0;
                                for (int j = 0; j < 4; j++) if (j != i) {
                                    const double den = X[i] - X[j];
                                    dli = dli * (x - X[j]) / den + li / den;
                                    li *= (x - X[j]) / den;
                                }
                                P += Y[i] * li; dP += Y[i] * dli;
                            }
                            if (dP == 0) break;
                            float xn = (float)(x - P / dP);
                            if (!(xn >= ts[k1] && xn <= ts[k1 + 1])) break;
                            x = xn;
                        }
                        t0 = x;
                    }
                }
            }
            if (getenv("SIM_P1H")) {  /* variant: a Halley step from m0 (h, h', h'' taken in the probe walk) */
                float h0, d1, d2;
                const float tm = fminf(fmaxf(m0, dmin), dmax);
                vac_d2(buf, n, tm, &h0, &d1, &d2);
                const float den = 2.f * d1 * d1 - h0 * d2;
                const float th = den != 0.f ? tm - 2.f * h0 * d1 / den : -1.f;
                if (th >= ts[k1] && th <= ts[k1 + 1]) t0 = th;
            }
            float res = mr;
            /* SIM_P1_MAXIT=k: phase 1 stops after k Halley walks; a grid pixel not converged by then
               publishes its current iterate as its neighbours' guess and continues in phase 2b */
            const int k1max = getenv("SIM_P1_MAXIT") ? atoi(getenv("SIM_P1_MAXIT")) : maxit;
            const long nc0 = g_why_nc;
            int wk = halley_from(buf, n, t0, ts[k1], ts[k1 + 1], tol_rel, k1max, hnoise, &res);
            if (wk < 0 && g_why_nc > nc0 && k1max < maxit) {
                out[40] += 1;  /* stragglers */
                const float tg = g_last_t;
                float res2 = mr;
                int wk2 = halley_from(buf, n, g_last_t, g_last_lo, g_last_hi, tol_rel, maxit - k1max, hnoise, &res2);
                out[41] += wk2 < 0 ? -wk2 : wk2;
                if (wk2 < 0) { out[2] += 1; res2 = mr; }
                root[l] = tg;  /* (the guess phase 2 sees) */
                have[l] = 1;
                const double d = fabs((double)res2 - mr);
                if (d > out[1]) out[1] = d;
                wk = k1max;
                if (wk > wmax1) wmax1 = wk;
                out[32 + (wk < 7 ? wk : 7)] += 1;
                continue;
            }
            if (wk < 0) { out[2] += 1; res = mr; wk = 100; }
            out[32 + (wk < 7 ? wk : 7)] += 1;
            root[l] = res;
            have[l] = 1;
            const double d = fabs((double)res - mr);
            if (d > out[1]) out[1] = d;
            if (wk > wmax1) wmax1 = wk;
        }
        out[3] += wmax1;
        out[4] += 1;
        /* phase 2: the others, in raster order, 64 per wave */
        int lane = 0, wmax2 = 0;
        for (int l = 0; l < 256; l++) {
            const int lx = l & 15, ly = l >> 4;
            if (!((lx % G) || (ly % G))) continue;
            const int px = tx * 16 + lx, py = ty * 16 + ly;
            int wk = 0;
            if (px < W && py < H) {
                float Tf, m0;
                const int n = composite(point_list + r0, (int)(r1 - r0), xy, co, rp, (float)px, (float)py, buf, &Tf, &m0);
                int ir;
                const float mr = ref_bisect(buf, n, m0, Tf, &ir);
                if (ir) {
                    out[0] += 1;
                    float sum = 0.f, cnt = 0.f;
                    /* bilinear over the surrounding grid pixels present (G = 2: the mean of the 1, 2 or 4 of them) */
                    const int x0g = lx - lx % G, y0g = ly - ly % G;
                    for (int yy = y0g; yy <= y0g + G; yy += G)
                        for (int xx = x0g; xx <= x0g + G; xx += G)
                            if (yy >= 0 && yy < 16 && xx >= 0 && xx < 16 && have[yy * 16 + xx]) {
                                const float wx = xx == x0g ? (float)(G - lx % G) : (float)(lx % G);
                                const float wy = yy == y0g ? (float)(G - ly % G) : (float)(ly % G);
                                const float wgt = wx * wy;
                                if (wgt <= 0.f) continue;
                                sum += wgt * root[yy * 16 + xx];
                                cnt += wgt;
                            }
                    const float dmin = fmaxf(m0 - RANGE, 0.f), dmax = fmaxf(m0 + RANGE, 0.f);
                    float res = mr;
                    if (!cnt) {
                        out[24] += 1;
                        wk = 100;
                    } else {
                        const float t0 = fminf(fmaxf(sum / cnt, dmin), dmax);
                        (void)0;
                        wk = halley_from(buf, n, t0, dmin, dmax, tol_rel, maxit, hnoise, &res);
                        if (wk < 0) { out[2] += 1; res = mr; wk = 100; }
                    }
                    const double d = fabs((double)res - mr);
                    if (d > out[1]) out[1] = d;
                    out[8 + (wk < 15 ? wk : 15)] += 1;
                }
            }
            if (wk > wmax2) wmax2 = wk;
            if (++lane == 64) {
                out[5] += wmax2;
                out[6] += 1;
                lane = 0;
                wmax2 = 0;
            }
        }
    }
    free(buf);
}

/* ---- round 5: the first guess of the median depth from the composite's crossing contributor ----
 * Single-splat model: contributors before the crossing one (the last with T_before > 1/2) are taken as
 * fully passed (factor 1 - a), those after as not reached (factor 1): T(t) = T_b f_k(t), f_k = sqrt(1 - a g)
 * in front of the peak and (1 - a) / sqrt(1 - a g) behind it, g = exp(-((t - tp) rs)^2 / 2), solved for
 * T(t) = 1/2 in closed form.  Reports how often ONE walk from the guess passes the kernel's acceptance
 * (Newton step <= tol max(t, 1), or <= loose max(t, 1) with |step| F <= curv |h'|), against the mean of
 * the grid neighbours' exact roots (the current phase-2 guess). */
static float guess_single(float Tb, float a, float tp, float rs) {
    if (!(rs > 0.f)) return tp;
    const float s = sqrtf(1.f - a);
    float g;
    int behind;
    if (Tb * s > 0.5f) {  /* root behind the peak */
        const float q = 2.f * Tb * (1.f - a);
        if (q >= 1.f) return tp;  /* never crosses */
        g = (1.f - q * q) / a;
        behind = 1;
    } else {
        g = (1.f - 0.25f / (Tb * Tb)) / a;
        behind = 0;
    }
    if (!(g > 0.f)) return tp;
    if (g > 1.f) g = 1.f;
    const float d = sqrtf(-2.f * logf(g)) / rs;
    return behind ? tp + d : tp - d;
}
static int composite_x(const uint32_t* list, int cnt, const float* xy, const float* co, const float* rp, float px,
                       float py, contrib_t* out, float* Tfin, float* m0, float* Tb_out, int* kx) {
    float T = 1.f, mi = 0.f, Tb = 1.f;
    int n = 0, kk = -1;
    for (int k = 0; k < cnt; k++) {
        const uint32_t g = list[k];
        const float dx = xy[2 * g] - px, dy = xy[2 * g + 1] - py;
        const float* c4 = co + 4 * g;
        const float power = -0.5f * (c4[0] * dx * dx + c4[2] * dy * dy) - c4[1] * dx * dy;
        if (power > 0.f) continue;
        const float alpha = fminf(0.99f, c4[3] * expf(power));
        if (alpha < 1.f / 255.f) continue;
        const float tT = T * (1.f - alpha);
        if (tT < 1e-4f) break;
        const float* r = rp + 4 * g;
        const float t = r[0] * dx + r[1] * dy + r[2];
        if (T > 0.5f) { mi = t; kk = n; Tb = T; }
        out[n].a = alpha;
        out[n].tp = t;
        out[n].rs = r[3];
        n++;
        T = tT;
    }
    *Tfin = T;
    *m0 = mi;
    *Tb_out = Tb;
    *kx = kk;
    return n;
}
/* exact root by bisection in double over [lo, hi] (T non-increasing) */
static double root_exact(const contrib_t* c, int n, double lo, double hi) {
    for (int it = 0; it < 60; it++) {
        const double mid = 0.5 * (lo + hi);
        double T = 1.0;
        for (int i = 0; i < n; i++) {
            const double d = (mid - c[i].tp) * c[i].rs;
            const double g = c[i].rs > 0 ? exp(-0.5 * d * d) : 0.0;
            const double omg = 1.0 - c[i].a * g;
            T *= (mid > c[i].tp ? 1.0 - c[i].a : omg) / sqrt(omg);
        }
        if (T >= 0.5) lo = mid; else hi = mid;
    }
    return 0.5 * (lo + hi);
}
static int accept_from(const contrib_t* c, int n, float t, float tol, float loose, float curv) {
    float h, d1, d2;
    vac_d2(c, n, t, &h, &d1, &d2);
    const float D = -d1, F = g_lastF, scale = fmaxf(t, 1.f);
    if (!(D > 0.f)) return 0;
    const float step = fabsf(h) / D;
    return step <= tol * scale || (step <= loose * scale && step * F <= curv * D);
}
/* out: [0] pixels in range, [1] single-guess accepted after one walk, [2] neighbour-mean accepted,
 * [3..10] hist of log10(|guess - root| / max(root, 1)) for the single guess (bins <-7, -7..-6, .., >=-1),
 * [11..18] the same for the neighbour mean, [19] either accepted, [20] single-guess within the window */
void sim_guess(int W, int H, int gx, int ntiles, const uint32_t* tiles, const uint32_t* ranges,
               const uint32_t* plist, const float* xy, const float* co, const float* rp, float tol, float loose,
               float curv, double* out) {
    static contrib_t cc[256][4096];
    static int nn[256], inr[256];
    static float gs[256], m0s[256], tfs[256];
    static double rt[256];
    for (int ti = 0; ti < ntiles; ti++) {
        const uint32_t tile = tiles[ti];
        const int tx = tile % gx, ty = tile / gx;
        const uint32_t b = ranges[2 * tile], e = ranges[2 * tile + 1];
        for (int p = 0; p < 256; p++) {
            const int px = tx * 16 + (p & 15), py = ty * 16 + (p >> 4);
            inr[p] = 0;
            if (px >= W || py >= H) continue;
            float Tf, m0, Tb;
            int kx;
            nn[p] = composite_x(plist + b, (int)(e - b), xy, co, rp, (float)px, (float)py, cc[p], &Tf, &m0, &Tb, &kx);
            m0s[p] = m0;
            tfs[p] = Tf;
            if (Tf > 0.45f || kx < 0) continue;
            const double lo = fmax(m0 - RANGE, 0.f), hi = fmax(m0 + RANGE, 0.f);
            /* in range as the reference decides it (window ends) */
            if (!(vac(cc[p], nn[p], (float)lo) >= 0.5f && vac(cc[p], nn[p], (float)hi) <= 0.5f)) continue;
            inr[p] = 1;
            rt[p] = root_exact(cc[p], nn[p], lo, hi);
            const contrib_t* k = &cc[p][kx];
            gs[p] = guess_single(Tb, k->a, k->tp, k->rs);
        }
        for (int p = 0; p < 256; p++) {
            if (!inr[p]) continue;
            const int lx = p & 15, ly = p >> 4;
            double sum = 0;
            int cnt = 0;
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    const int use = ((lx & 1) ? dx != 0 : dx == 0) && ((ly & 1) ? dy != 0 : dy == 0);
                    const int nx = lx + dx, ny = ly + dy;
                    if (use && nx >= 0 && nx < 16 && ny >= 0 && ny < 16 && inr[ny * 16 + nx] && !((nx | ny) & 1) &&
                        !(nx == lx && ny == ly)) {
                        sum += rt[ny * 16 + nx];
                        cnt++;
                    }
                }
            const double scale = fmax(rt[p], 1.0);
            {   /* higher-order guess: tensor-product Lagrange interpolation of the grid roots */
                double wxv[4], wyv[4];
                int xs[4], ys[4], nx_ = 0, ny_ = 0;
                for (int ax = 0; ax < 2; ax++) {
                    const int l = ax ? ly : lx;
                    double* wv = ax ? wyv : wxv;
                    int* cs = ax ? ys : xs;
                    int* nc = ax ? &ny_ : &nx_;
                    if (!(l & 1)) { cs[0] = l; wv[0] = 1; *nc = 1; continue; }
                    if (l >= 3 && l <= 11) { int o[4] = {-3, -1, 1, 3}; double w[4] = {-1/16., 9/16., 9/16., -1/16.};
                        for (int q = 0; q < 4; q++) { cs[q] = l + o[q]; wv[q] = w[q]; } *nc = 4; }
                    else if (l == 1) { int o[3] = {-1, 1, 3}; double w[3] = {3/8., 3/4., -1/8.};
                        for (int q = 0; q < 3; q++) { cs[q] = l + o[q]; wv[q] = w[q]; } *nc = 3; }
                    else if (l == 13) { int o[3] = {-3, -1, 1}; double w[3] = {-1/8., 3/4., 3/8.};
                        for (int q = 0; q < 3; q++) { cs[q] = l + o[q]; wv[q] = w[q]; } *nc = 3; }
                    else { int o[2] = {-3, -1}; double w[2] = {-0.5, 1.5};  /* l = 15: linear extrapolation */
                        for (int q = 0; q < 2; q++) { cs[q] = l + o[q]; wv[q] = w[q]; } *nc = 2; }
                }
                double gsum = 0; int ok = 1;
                for (int i = 0; i < nx_; i++) for (int j = 0; j < ny_; j++) {
                    const int q = ys[j] * 16 + xs[i];
                    if (!inr[q]) ok = 0; else gsum += wxv[i] * wyv[j] * rt[q];
                }
                if (ok && !(!(lx & 1) && !(ly & 1))) {
                    const float gh = (float)gsum;
                    out[21] += 1;
                    out[22] += accept_from(cc[p], nn[p], gh, tol, loose, curv);
                    double e3 = fabs(gh - rt[p]) / scale;
                    int b3 = e3 <= 0 ? 0 : (int)floor(log10(e3)) + 8;
                    b3 = b3 < 0 ? 0 : b3 > 7 ? 7 : b3;
                    out[23 + b3] += 1;
                }
            }
            {   /* two-level grid: an even-grid pixel not on the 4-grid, guessed from the 4-grid roots
                 * (coordinates / 2 on the 4-grid's half-resolution lattice: the same 1-D rules, h = 4) */
                if (!(lx & 1) && !(ly & 1) && ((lx | ly) & 2)) {
                    const int hx = lx >> 1, hy = ly >> 1;  /* 0..7, 4-grid at even h */
                    double wxv[4], wyv[4];
                    int xs[4], ys[4], nx_ = 0, ny_ = 0;
                    for (int ax = 0; ax < 2; ax++) {
                        const int l = ax ? hy : hx;
                        double* wv = ax ? wyv : wxv;
                        int* cs = ax ? ys : xs;
                        int* nc = ax ? &ny_ : &nx_;
                        if (!(l & 1)) { cs[0] = l; wv[0] = 1; *nc = 1; continue; }
                        if (l == 3) { int o[4] = {-3, -1, 1, 3}; double w[4] = {-1/16., 9/16., 9/16., -1/16.};
                            for (int q = 0; q < 4; q++) { cs[q] = l + o[q]; wv[q] = w[q]; } *nc = 4; }
                        else if (l == 1) { int o[3] = {-1, 1, 3}; double w[3] = {3/8., 3/4., -1/8.};
                            for (int q = 0; q < 3; q++) { cs[q] = l + o[q]; wv[q] = w[q]; } *nc = 3; }
                        else if (l == 5) { int o[3] = {-3, -1, 1}; double w[3] = {-1/8., 3/4., 3/8.};
                            for (int q = 0; q < 3; q++) { cs[q] = l + o[q]; wv[q] = w[q]; } *nc = 3; }
                        else { int o[2] = {-3, -1}; double w[2] = {-0.5, 1.5};
                            for (int q = 0; q < 2; q++) { cs[q] = l + o[q]; wv[q] = w[q]; } *nc = 2; }
                    }
                    double g4 = 0; int ok4 = 1;
                    for (int i = 0; i < nx_; i++) for (int j = 0; j < ny_; j++) {
                        const int q = (2 * ys[j]) * 16 + 2 * xs[i];
                        if (!inr[q]) ok4 = 0; else g4 += wxv[i] * wyv[j] * rt[q];
                    }
                    if (ok4) {
                        const float gh = (float)g4;
                        out[31] += 1;
                        const int acc = accept_from(cc[p], nn[p], gh, tol, loose, curv);
                        out[32] += acc;
                        {   /* by the tile's 4-grid root spread (max - min) / max(mean, 1): bins <1e-3, <1e-2, <3e-2, <0.1, >= */
                            double mn = 1e30, mx = -1e30, sm = 0; int nv = 0;
                            for (int q4 = 0; q4 < 16; q4++) {
                                const int qq = (4 * (q4 >> 2)) * 16 + 4 * (q4 & 3);
                                if (inr[qq]) { mn = fmin(mn, rt[qq]); mx = fmax(mx, rt[qq]); sm += rt[qq]; nv++; }
                            }
                            const double sp = nv ? (mx - mn) / fmax(sm / nv, 1.0) : 1.0;
                            const int sb = nv < 16 ? 5 : sp < 1e-3 ? 0 : sp < 1e-2 ? 1 : sp < 3e-2 ? 2 : sp < 0.1 ? 3 : 4;
                            out[34 + 2 * sb] += 1;
                            out[35 + 2 * sb] += acc;
                            /* the same by the spread of the 4-grid pixels' composite m0 (known before phase 1) */
                            double mn2 = 1e30, mx2 = -1e30, sm2 = 0; int nv2 = 0;
                            for (int q4 = 0; q4 < 16; q4++) {
                                const int qq = (4 * (q4 >> 2)) * 16 + 4 * (q4 & 3);
                                if (tfs[qq] <= 0.45f) { mn2 = fmin(mn2, m0s[qq]); mx2 = fmax(mx2, m0s[qq]); sm2 += m0s[qq]; nv2++; }
                            }
                            const double sp2 = nv2 ? (mx2 - mn2) / fmax(sm2 / nv2, 1.0) : 1.0;
                            const int sb2 = nv2 < 16 ? 5 : sp2 < 1e-2 ? 0 : sp2 < 2e-2 ? 1 : sp2 < 5e-2 ? 2 : sp2 < 0.1 ? 3 : 4;
                            out[46 + 2 * sb2] += 1;
                            out[47 + 2 * sb2] += acc;
                        }
                        if (!acc) {  /* a second walk from the Halley iterate */
                            float h, d1, d2;
                            vac_d2(cc[p], nn[p], gh, &h, &d1, &d2);
                            const float tn = gh - 2.f * h * d1 / (2.f * d1 * d1 - h * d2);
                            out[33] += accept_from(cc[p], nn[p], tn, tol, loose, curv);
                        }
                    }
                }
            }
            out[0] += 1;
            const int a1 = accept_from(cc[p], nn[p], gs[p], tol, loose, curv);
            out[1] += a1;
            double e1 = fabs(gs[p] - rt[p]) / scale;
            int b1 = e1 <= 0 ? 0 : (int)floor(log10(e1)) + 8;
            b1 = b1 < 0 ? 0 : b1 > 7 ? 7 : b1;
            out[3 + b1] += 1;
            out[20] += fabs(gs[p] - rt[p]) < 0.4;
            if (cnt) {
                const float gm = (float)(sum / cnt);
                const int a2 = accept_from(cc[p], nn[p], gm, tol, loose, curv);
                out[2] += a2;
                out[19] += a1 || a2;
                double e2 = fabs(gm - rt[p]) / scale;
                int b2 = e2 <= 0 ? 0 : (int)floor(log10(e2)) + 8;
                b2 = b2 < 0 ? 0 : b2 > 7 ? 7 : b2;
                out[11 + b2] += 1;
            }
        }
    }
}

/* round 5: blended contributors a median-depth walk must visit when the list is cut after the last one
 * that is not "far behind" the reference's whole first window (t_peak - K / rsigma > m0 + 0.4 for
 * contributors after the T = 1/2 crossing, whose factor is then exactly 1 at every depth of the window).
 * out: [0] in-range pixels, [1] blended contributors, [2] blended up to the cut, [3] blended before the
 * crossing, [4] far-behind contributors before the cut (still walked) */
void sim_cut(int W, int H, int gx, int ntiles, const uint32_t* tiles, const uint32_t* ranges, const uint32_t* plist,
             const float* xy, const float* co, const float* rp, float K, double* out) {
    static contrib_t cc[4096];
    for (int ti = 0; ti < ntiles; ti++) {
        const uint32_t tile = tiles[ti];
        const int tx = tile % gx, ty = tile / gx;
        const uint32_t b = ranges[2 * tile], e = ranges[2 * tile + 1];
        for (int p = 0; p < 256; p++) {
            const int px = tx * 16 + (p & 15), py = ty * 16 + (p >> 4);
            if (px >= W || py >= H) continue;
            float Tf, m0, Tb;
            int kx;
            const int n = composite_x(plist + b, (int)(e - b), xy, co, rp, (float)px, (float)py, cc, &Tf, &m0, &Tb, &kx);
            if (Tf > 0.45f || kx < 0) continue;
            int cut = kx, farb = 0;
            for (int i = kx + 1; i < n; i++) {
                const int far = cc[i].rs > 0 && cc[i].tp - K / cc[i].rs > m0 + RANGE;
                if (!far) cut = i;
            }
            for (int i = kx + 1; i <= cut; i++) farb += cc[i].rs > 0 && cc[i].tp - K / cc[i].rs > m0 + RANGE;
            out[0] += 1;
            out[1] += n;
            out[2] += cut + 1;
            out[3] += kx + 1;
            out[4] += farb;
        }
    }
}

/* round 5: the backward's walked (tile, entry) steps: entries before the tile's max contributor that some
 * pixel blended (TileState::blend_mask; entries past the first 256 are all walked).
 * out: [0] tiles, [1] sum max_contrib, [2] walked steps, [3] sum over walked steps of blending pixels */
void sim_bwd_steps(int W, int H, int gx, int ntiles, const uint32_t* tiles, const uint32_t* ranges,
                   const uint32_t* plist, const float* xy, const float* co, double* out) {
    static int cnt[65536];
    for (int ti = 0; ti < ntiles; ti++) {
        const uint32_t tile = tiles[ti];
        const int tx = tile % gx, ty = tile / gx;
        const uint32_t b = ranges[2 * tile], e = ranges[2 * tile + 1];
        const int n = (int)(e - b);
        for (int k = 0; k < n && k < 65536; k++) cnt[k] = 0;
        int maxc = 0;
        for (int p = 0; p < 256; p++) {
            const int px = tx * 16 + (p & 15), py = ty * 16 + (p >> 4);
            if (px >= W || py >= H) continue;
            float T = 1.f;
            int last = 0;
            for (int k = 0; k < n; k++) {
                const uint32_t g = plist[b + k];
                const float dx = xy[2 * g] - px, dy = xy[2 * g + 1] - py;
                const float* c4 = co + 4 * g;
                const float power = -0.5f * (c4[0] * dx * dx + c4[2] * dy * dy) - c4[1] * dx * dy;
                if (power > 0.f) continue;
                const float alpha = fminf(0.99f, c4[3] * expf(power));
                if (alpha < 1.f / 255.f) continue;
                const float tT = T * (1.f - alpha);
                if (tT < 1e-4f) break;
                cnt[k]++;
                T = tT;
                last = k + 1;
            }
            if (last > maxc) maxc = last;
        }
        out[0] += 1;
        out[1] += maxc;
        for (int k = 0; k < maxc; k++) {
            if (k >= 256 || cnt[k] > 0) { out[2] += 1; out[3] += cnt[k]; }
        }
    }
}
