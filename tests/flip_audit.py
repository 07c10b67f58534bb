"""Exact accounting of the pixels where two fp32 forwards (the GPU's and the
oracle's) take a different discrete decision ("what's weak" 1).

The reference's composite has three per-(pixel, contributor) tests —
power > 0, alpha < 1/255 and the saturation stop T (1 - alpha) < 1e-4
(render_forward.cu:487-502) — and the median depth picks bisection cells by
T(t_s) >= 1/2 and decides `in_range` by T(window ends) against 1/2 and the
final T against MIN_TRANSMITTANCE (:549-645).  Two fp32 evaluations of the
same products in different (but equally valid) orders can fall on opposite
sides of a threshold only when the exact value is within rounding of it.
This module re-evaluates every such decision of a pixel in float64 from the
oracle's own forward state and returns the margin to the nearest threshold,
so a test can prove that each differing pixel is such a near-tie instead of
allowing a budget of arbitrary differences.
"""
from __future__ import annotations

import math

import numpy as np

SPLIT, SAMPLE_RANGE, MIN_TRANSMITTANCE = 8, 0.4, 0.45


class PixelChains:
    """float64 composite chains of single pixels over the oracle's tile lists."""

    def __init__(self, o, W, H, tanx, tany):
        st = o["state"]
        self.W, self.H, self.tanx, self.tany = W, H, tanx, tany
        self.geo = st.geometry()
        self.plist = st.binning()["point_list"].astype(np.int64)
        self.ranges = st.tile_state()["ranges"].astype(np.int64)
        self.gx = (W + 15) // 16

    def contributors(self, x, y):
        """[(position 1.., power, alpha, t_peak, rsigma)] of every list entry of
        the pixel's tile, float64, with the reference's arithmetic."""
        t = (y // 16) * self.gx + (x // 16)
        a, b = self.ranges[t]
        g = self.plist[a:b]
        m = self.geo["means2D"][g].astype(np.float64)
        co = self.geo["conic_opacity"][g].astype(np.float64)
        rp = self.geo["ray_planes"][g].astype(np.float64)
        dx, dy = m[:, 0] - x, m[:, 1] - y
        power = -0.5 * (co[:, 0] * dx * dx + co[:, 2] * dy * dy) - co[:, 1] * dx * dy
        alpha = np.minimum(0.99, co[:, 3] * np.exp(np.minimum(power, 0.0)))
        t_peak = rp[:, 0] * dx + rp[:, 1] * dy + rp[:, 2]
        return power, alpha, t_peak, rp[:, 3]

    def composite(self, x, y, toggle=-1):
        """(last contributor, final T, m0, per-entry margins) of the float64
        composite; margins[k] = the smallest relative distance of entry k+1's
        three decisions to their thresholds.  `toggle` = k takes the other
        outcome of entry k's nearest decision (skip / blend / stop), as an fp32
        evaluation on the other side of that threshold would."""
        power, alpha, t_peak, _ = self.contributors(x, y)
        n = len(power)
        T, last, m0 = 1.0, 0, 0.0
        margins = np.full(n, np.inf)
        self.m0_margin = math.inf  # the T > 1/2 test that picks m0
        for k in range(n):
            mk = abs(power[k]) / max(1e-30, abs(power[k]) + 1.0) * 1e3  # power = 0 decides only at exactly 0
            ma = abs(alpha[k] * 255.0 - 1.0)
            test_T = T * (1.0 - alpha[k])
            ms = abs(test_T / 1e-4 - 1.0)
            skip = power[k] > 0 or alpha[k] < 1.0 / 255.0
            stop = not skip and test_T < 1e-4
            if k == toggle:
                if min(mk, ma) <= ms:
                    skip, stop = not skip, False
                    stop = not skip and test_T < 1e-4
                else:
                    skip, stop = False, not stop
            if power[k] > 0 and k != toggle:
                margins[k] = mk
                continue
            if skip:
                margins[k] = min(mk, ma)
                continue
            margins[k] = min(mk, ma, ms)
            if stop:
                break
            self.m0_margin = min(self.m0_margin, abs(T / 0.5 - 1.0))
            if T > 0.5:
                m0 = t_peak[k]
            T, last = test_T, k + 1
        return last, T, m0, margins

    def vacancy(self, x, y, last, ts):
        """T(t) of the median-depth search at depths `ts` over contributors
        1..last (render_forward.cu:566-611), float64."""
        power, alpha, t_peak, rsig = self.contributors(x, y)
        ts = np.atleast_1d(np.asarray(ts, np.float64))
        T = np.ones_like(ts)
        for k in range(min(last, len(power))):
            if power[k] > 0 or alpha[k] < 1.0 / 255.0:
                continue
            d = (ts - t_peak[k]) * rsig[k]
            g = np.exp(-0.5 * d * d) if rsig[k] > 0 else np.zeros_like(ts)
            omg = 1.0 - alpha[k] * g
            T *= np.where(ts > t_peak[k], 1.0 - alpha[k], omg) / np.sqrt(omg)
        return T

    def depth_of(self, x, y, mdepth_px):
        """The ray distance t of an mdepth output (mdepth = t * rln)."""
        fx = self.W / 2.0 / self.tanx
        fy = self.H / 2.0 / self.tany
        nx = (x - (self.W - 1) / 2.0) / fx
        ny = (y - (self.H - 1) / 2.0) / fy
        return mdepth_px * math.sqrt(nx * nx + ny * ny + 1.0)


def chain_margin(ch, x, y, upto):
    """The smallest float64 margin of the composite's decisions over the
    pixel's first `upto` list entries: a pixel whose images differ between
    two fp32 forwards without a near-tie there is not explained by rounding."""
    _, _, _, margins = ch.composite(x, y)
    return float(np.min(margins[:upto])) if upto > 0 and len(margins) else math.inf


def ncontrib_flip_explained(ch, x, y, last_gpu, tol=2e-4):
    """Whether the GPU's last contributor is the float64 composite's with one
    decision at most `tol` from its threshold taking its other outcome: the
    flip is then a rounding-level tie, directly (the decision between the two
    last contributors) or upstream (a weak contributor's alpha at 1/255 moves
    T by up to 1/255 relative, and a later saturation test with it)."""
    last, _, _, margins = ch.composite(x, y)
    if last == last_gpu:
        return True
    for k in np.flatnonzero(margins[:max(last, last_gpu) + 1] <= tol):
        if ch.composite(x, y, toggle=int(k))[0] == last_gpu:
            return True
    return False


def ncontrib_flip_margin(ch, x, y, a, b):
    """The decision that separates last contributor a from b (positions in
    the pixel's list): the smallest float64 margin among entries (min, max]."""
    _, _, _, margins = ch.composite(x, y)
    lo, hi = min(a, b), max(a, b)
    return float(np.min(margins[lo:hi])) if hi > lo else math.inf


def mdepth_flip_margin(ch, x, y, t_gpu, t_orc):
    """Why two median depths of a pixel differ: the distance of T to 1/2 (or
    of the final T to MIN_TRANSMITTANCE) at the decisions involved, float64.
    Both in range: T at both depths is within the returned margin of 1/2 —
    the root is ill-conditioned (T flat within rounding of 1/2 between them).
    One of them 0 (out of range): T at the window ends vs 1/2, the final T vs
    0.45."""
    last, T_final, m0, _ = ch.composite(x, y)
    if t_gpu > 0 and t_orc > 0:
        Tv = ch.vacancy(x, y, last, [t_gpu, t_orc])
        lo, hi = min(t_gpu, t_orc), max(t_gpu, t_orc)
        inner = ch.vacancy(x, y, last, np.linspace(lo, hi, 9))
        return float(max(np.abs(Tv - 0.5).max(), np.abs(inner - 0.5).max()))
    ends = ch.vacancy(x, y, last, [max(m0 - SAMPLE_RANGE, 0.0), max(m0 + SAMPLE_RANGE, 0.0)])
    return float(min(abs(T_final - MIN_TRANSMITTANCE), np.abs(ends - 0.5).min(), ch.m0_margin))
