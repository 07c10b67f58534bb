"""Independent float64 torch-autograd restatement of the rasterizer path.

Used only by the tests to pin the C oracle (oracle/gsr_oracle.c): it is
written as dense tensor math in *math* (row, col) matrix convention — not as
a transcription of the glm code — and its gradients come from autograd, so it
checks that the oracle's hand-written backward is the derivative of its
forward, exactly where the reference's backward is an exact derivative.

Where the reference's backward deliberately differs from the exact derivative
of its forward, this file reproduces the reference and says so:
  Q1  normal = normalize(cam_normal); the backward scales by 1/|normal| (== 1)
      instead of 1/|cam_normal| (render_backward.cu:468-470)
      -> `_quirk_normalize`.
  Q2  the median-depth gradient is the implicit-function derivative of the
      vacancy transmittance at T = 1/2 (render_backward.cu:835-880, 983-999)
      -> `_median_depth_surrogate` (uses the same T = 1/2 assumption).
  Q3  alpha = min(0.99, o*G) passes gradient through the clamp
      (render_backward.cu:931-933, 1012; sample_backward.cu:284-327): dL/dG
      = o * dL/dalpha even where alpha is clamped -> `_clamp_st`.
  Q4  rsigma = sqrt(vb / |uvh|^2): the backward omits d rsigma / d(u, v)
      through vb (render_backward.cu:484-490) -> `vb_rs` below.
  Q5  Mip-filter coefficient coef = sqrt(det0/det1): the backward uses
      dL/ddet1 = -dL/ddet0 * coef instead of * coef**2 (render_backward.cu:551)
      -> `_QuirkCoef`.  Exact when kernel_size = 0 (coef = 1).
Discrete decisions (culling, rect, skip/stop rules, bisection interval
choice) follow CR/render_forward.cu; their thresholds are evaluated in float64
here and in float32 in the oracle, so tests use scenes away from the edges.
"""
from __future__ import annotations

import math

import numpy as np
import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]


class _QuirkNormalize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        n = x / x.norm(dim=-1, keepdim=True)
        ctx.save_for_backward(n)
        return n

    @staticmethod
    def backward(ctx, g):
        (n,) = ctx.saved_tensors
        return g - n * (n * g).sum(-1, keepdim=True)


def _quirk_normalize(x):
    return _QuirkNormalize.apply(x)


class _QuirkCoef(torch.autograd.Function):
    """coef = sqrt(det0 / det1) with the reference's backward
    (render_backward.cu:548-551): dL/ddet1 = -dL/ddet0 * coef, where the exact
    derivative has coef**2; and the 1e-6 guard in 0.5 / (coef + 1e-6)."""

    @staticmethod
    def forward(ctx, det0, det1):
        coef = torch.sqrt(det0 / det1)
        ctx.save_for_backward(coef, det1)
        return coef

    @staticmethod
    def backward(ctx, g):
        coef, det1 = ctx.saved_tensors
        d0 = g * 0.5 / (coef + 1e-6) / det1
        return d0, -d0 * coef


def _clamp_st(x):
    """min(0.99, x) whose gradient is 1 everywhere (Q3: the reference
    differentiates alpha = o*G through the clamp)."""
    return x - (x - torch.clamp(x, max=0.99)).detach()


def _sh_color(shs, sg_axis, sg_sharp, sg_color, means, campos, deg, sgd):
    d = means - campos[None]
    d = d / d.norm(dim=1, keepdim=True)
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    sh = shs
    r = SH_C0 * sh[:, 0]
    if deg > 0:
        r = r - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            r = (r + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6]
                 + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
            if deg > 2:
                r = (r + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
                     + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11]
                     + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
                     + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
                     + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    for g in range(sgd):
        gauss = torch.exp(sg_sharp[:, g:g + 1] * ((sg_axis[:, g] * d).sum(1, keepdim=True) - 1.0))
        r = r + sg_color[:, g] * gauss
    r = r + 0.5
    return r.clamp_min(0.0)


def preprocess(means3D, scales, rotations, opacities, shs, sg_axis, sg_sharp, sg_color, means2D, view, proj, campos,
               W, H, tanx, tany, kernel_size, deg, sgd, colors_precomp=None, scale_modifier=1.0):
    """Per-Gaussian screen-space quantities (math of render_forward.cu:81-386)."""
    fx = W / (2.0 * tanx)
    fy = H / (2.0 * tany)
    Pn = means3D.shape[0]
    Wm = view[:3, :3]  # math W: p_view = Wm^T p + view[3,:3]
    t = means3D @ Wm + view[3, :3]
    visible = (t[:, 2] > 0.2).detach()
    tc = t.norm(dim=1)
    limx, limy = 1.3 * tanx, 1.3 * tany
    u = torch.clamp(t[:, 0] / t[:, 2], -limx, limx)
    v = torch.clamp(t[:, 1] / t[:, 2], -limy, limy)
    tz = t[:, 2]
    tx, ty = u * tz, v * tz
    zero = torch.zeros_like(tz)
    # J (math) = [[fx/tz, 0, -fx tx/tz^2], [0, fy/tz, -fy ty/tz^2], [0, 0, 0]];   T = W J^T ... in glm order
    Jm = torch.stack([torch.stack([fx / tz, zero, zero], 1),
                      torch.stack([zero, fy / tz, zero], 1),
                      torch.stack([-fx * tx / tz ** 2, -fy * ty / tz ** 2, zero], 1)], 1)  # math layout of glm J
    Tm = Wm[None] @ Jm
    q = rotations
    r_, x_, y_, z_ = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    # glm R columns -> math layout (R_math[:, c] = glm column c)
    Rm = torch.stack([
        torch.stack([1 - 2 * (y_ ** 2 + z_ ** 2), 2 * (x_ * y_ + r_ * z_), 2 * (x_ * z_ - r_ * y_)], 1),
        torch.stack([2 * (x_ * y_ - r_ * z_), 1 - 2 * (x_ ** 2 + z_ ** 2), 2 * (y_ * z_ + r_ * x_)], 1),
        torch.stack([2 * (x_ * z_ + r_ * y_), 2 * (y_ * z_ - r_ * x_), 1 - 2 * (x_ ** 2 + y_ ** 2)], 1)], 1)
    s = scales * scale_modifier
    S = torch.diag_embed(s)
    Sinv = torch.diag_embed(1.0 / s)
    M = S @ Rm @ Tm
    cov = M.transpose(1, 2) @ M
    Minv = Sinv @ Rm @ Wm[None]
    cov_cam_inv = Minv.transpose(1, 2) @ Minv
    a0, b0, c0 = cov[:, 0, 0], cov[:, 0, 1], cov[:, 1, 1]
    det0 = torch.clamp(a0 * c0 - b0 * b0, min=1e-6)
    det1 = torch.clamp((a0 + kernel_size) * (c0 + kernel_size) - b0 * b0, min=1e-6)
    coef = _QuirkCoef.apply(det0, det1)
    a, b, c = a0 + kernel_size, b0, c0 + kernel_size
    det = a * c - b * b
    conic = torch.stack([c / det, -b / det, a / det], 1)
    mid = 0.5 * (a + c)
    lam = mid + torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
    radius = torch.ceil(3.0 * torch.sqrt(lam)).detach()
    # ray plane and normal
    uvh = torch.stack([u, v, torch.ones_like(u)], 1)
    uvh_m = (cov_cam_inv @ uvh[..., None])[..., 0]
    u2, v2, uv = u * u, v * v, u * v
    l = torch.stack([tx, ty, tz], 1).norm(dim=1)
    nJinv = torch.stack([torch.stack([v2 + 1, -uv, -u], 1), torch.stack([-uv, u2 + 1, -v], 1),
                         torch.stack([zero, zero, zero], 1)], 1)  # rows of math matrix
    vb = (uvh_m * uvh).sum(1)
    rl2 = u2 + v2 + 1
    fn = l / rl2
    plane = (nJinv @ (uvh_m / vb[:, None])[..., None])[..., 0]
    # Q4: the reference backward drops d(rsigma)/d(u,v) through vb
    # (render_backward.cu:484-490 adds only the plane term to dL_duvh), so
    # rsigma sees vb with uvh held constant.
    uvh_c = uvh.detach()
    vb_rs = (((cov_cam_inv @ uvh_c[..., None])[..., 0]) * uvh_c).sum(1)
    rsig = torch.sqrt(vb_rs / rl2)
    ray_plane = torch.stack([plane[:, 0] * fn / fx, plane[:, 1] * fn / fy, tc, rsig], 1)
    rnv = torch.stack([-plane[:, 0] * fn, -plane[:, 1] * fn, -torch.ones_like(fn)], 1)
    nJ = torch.stack([torch.stack([1 / tz, zero, tx / l], 1), torch.stack([zero, 1 / tz, ty / l], 1),
                      torch.stack([-tx / tz ** 2, -ty / tz ** 2, tz / l], 1)], 1)  # rows of math matrix
    normal = _quirk_normalize((nJ @ rnv[..., None])[..., 0])
    # projection to pixels; means2D is the NDC-space dummy that receives dL/dndc
    p_hom = means3D @ proj[:3] + proj[3]
    ndc = p_hom[:, :2] / (p_hom[:, 3:4] + 1e-7) + means2D[:, :2]
    xy = torch.stack([((ndc[:, 0] + 1.0) * W - 1.0) * 0.5, ((ndc[:, 1] + 1.0) * H - 1.0) * 0.5], 1)
    if colors_precomp is None:
        rgb = _sh_color(shs, sg_axis, sg_sharp, sg_color, means3D, campos, deg, sgd)
    else:
        rgb = colors_precomp
    depth = t.norm(dim=1)
    opac = opacities[:, 0] * coef
    return dict(xy=xy, conic=conic, opac=opac, rgb=rgb, ray_plane=ray_plane, normal=normal, depth=depth,
                radius=radius, visible=visible & (det != 0).detach(), _tanx=tanx, _tany=tany)


def binning(pre, W, H):
    """Per-tile depth-sorted Gaussian lists (rasterizer_impl.cu:70-161)."""
    gx, gy = (W + 15) // 16, (H + 15) // 16
    xy = pre["xy"].detach().numpy()
    rad = pre["radius"].numpy()
    depth = pre["depth"].detach().numpy().astype(np.float32)
    vis = pre["visible"].numpy()
    lists = [[] for _ in range(gx * gy)]
    radii = np.zeros(len(rad), np.int32)
    for i in range(len(rad)):
        if not vis[i]:
            continue
        r = int(rad[i])
        x0 = min(gx, max(0, int((xy[i, 0] - r) / 16)))
        y0 = min(gy, max(0, int((xy[i, 1] - r) / 16)))
        x1 = min(gx, max(0, int((xy[i, 0] + r + 15) / 16)))
        y1 = min(gy, max(0, int((xy[i, 1] + r + 15) / 16)))
        if (x1 - x0) * (y1 - y0) == 0:
            continue
        radii[i] = r
        for ty in range(y0, y1):
            for tx in range(x0, x1):
                lists[ty * gx + tx].append(i)
    for t in range(len(lists)):
        lists[t].sort(key=lambda i: (depth[i], i))
    return lists, radii


def render(pre, lists, W, H, bg, require_depth=True, split=8, iters=5, sample_range=0.4, mdepth_override=None):
    """Dense composite per tile (render_forward.cu:412-670); returns outputs and
    the median-depth surrogate pieces for the implicit gradient."""
    gx = (W + 15) // 16
    dt = pre["xy"].dtype
    color = torch.zeros(3, H, W, dtype=dt)
    alpha_img = torch.zeros(1, H, W, dtype=dt)
    normal_img = torch.zeros(3, H, W, dtype=dt)
    mdepth = torch.zeros(1, H, W, dtype=dt)
    n_contrib = np.zeros((H, W), np.int64)
    surrogate_terms = []  # (pixel mask index, logT expression, dlogT/dt, t_m)
    fx = W / (2.0 * pre["_tanx"])
    fy = H / (2.0 * pre["_tany"])
    for tile, lst in enumerate(lists):
        tx0, ty0 = (tile % gx) * 16, (tile // gx) * 16
        xs = torch.arange(tx0, min(tx0 + 16, W), dtype=dt)
        ys = torch.arange(ty0, min(ty0 + 16, H), dtype=dt)
        py, px = torch.meshgrid(ys, xs, indexing="ij")
        px, py = px.reshape(-1), py.reshape(-1)
        npx = px.shape[0]
        T = torch.ones(npx, dtype=dt)
        C = torch.zeros(npx, 3, dtype=dt)
        N = torch.zeros(npx, 3, dtype=dt)
        m0 = torch.zeros(npx, dtype=dt)
        done = torch.zeros(npx, dtype=torch.bool)
        last = torch.zeros(npx, dtype=torch.long)
        used = []  # per list position: (alpha, t_peak, rsig, contributes-mask)
        for k, g in enumerate(lst):
            d = pre["xy"][g][None] - torch.stack([px, py], 1)
            co = pre["conic"][g]
            power = -0.5 * (co[0] * d[:, 0] ** 2 + co[2] * d[:, 1] ** 2) - co[1] * d[:, 0] * d[:, 1]
            G = torch.exp(power)
            al = _clamp_st(pre["opac"][g] * G)
            ok = (~done) & (power <= 0).detach() & (al >= 1.0 / 255.0).detach()
            test_T = T * (1 - al)
            stop = ok & (test_T < 1e-4).detach()
            done = done | stop
            ok = ok & ~stop
            w = torch.where(ok, al * T, torch.zeros_like(T))
            C = C + w[:, None] * pre["rgb"][g][None]
            rp = pre["ray_plane"][g]
            tp = rp[0] * d[:, 0] + rp[1] * d[:, 1] + rp[2]
            if require_depth:
                N = N + w[:, None] * pre["normal"][g][None]
                m0 = torch.where(ok & (T > 0.5).detach(), tp.detach(), m0)
            T = torch.where(ok, test_T, T)
            last = torch.where(ok, torch.full_like(last, k + 1), last)
            used.append((al, tp, rp[3], (power <= 0).detach() & (al >= 1.0 / 255.0).detach()))
        lin = (py.long() * W + px.long())
        color.view(3, -1)[:, lin] = (C + T[:, None] * bg[None]).T
        alpha_img.view(-1)[lin] = 1 - T
        n_contrib.reshape(-1)[lin.numpy()] = last.numpy()
        if not require_depth:
            continue
        lastf = last.clamp_min(1)
        nrm = torch.where((last > 0)[:, None], N / (1 - T)[:, None].clamp_min(1e-30), torch.zeros_like(N))
        normal_img.view(3, -1)[:, lin] = nrm.T
        # --- median depth: bisection (no grad), render_forward.cu:549-645 ---
        with torch.no_grad():
            Td = T.detach()
            dmin = torch.clamp(m0 - sample_range, min=0.0)
            dmax = torch.clamp(m0 + sample_range, min=0.0)
            in_range = Td <= 0.45
            Tp = torch.ones(npx, split + 1, dtype=dt)
            for it in range(iters):
                first = it == 0
                ids = range(0, split + 1) if first else range(1, split)
                for sidx in ids:
                    Tp[:, sidx] = 1.0
                interval = (dmax - dmin) / split
                for k, (al, tp, rs, mask) in enumerate(used):
                    m = mask & ((k + 1) <= last) & in_range
                    if not bool(m.any()):
                        continue
                    for sidx in ids:
                        ts = dmin + interval * sidx
                        delta = (ts - tp) * rs
                        gg = torch.exp(-0.5 * delta * delta) if float(rs) > 0 else torch.zeros_like(ts)
                        omg = 1 - al * gg
                        f = torch.where(ts > tp, 1 - al, omg) / torch.sqrt(omg)
                        Tp[:, sidx] = torch.where(m, Tp[:, sidx] * f, Tp[:, sidx])
                if first:
                    in_range = (Tp[:, 0] >= 0.5) & (Tp[:, split] <= 0.5) & in_range
                start = torch.zeros(npx, dtype=torch.long)
                for p_ in range(1, split):
                    start = torch.where(Tp[:, p_] >= 0.5, torch.full_like(start, p_), start)
                dmax = dmin + (start + 1) * interval
                dmin = dmin + start * interval
                Tp0 = Tp.gather(1, start[:, None])[:, 0]
                Tp8 = Tp.gather(1, (start + 1)[:, None])[:, 0]
                Tp[:, 0], Tp[:, split] = Tp0, Tp8
            wmax = ((Tp[:, 0] - 0.5) / (Tp[:, 0] - Tp[:, split])).nan_to_num(0.0).clamp(0, 1)
            tm = torch.where(in_range, wmax * dmax + (1 - wmax) * dmin, torch.zeros_like(dmin))
        pnx = (px - (W - 1) / 2.0) / fx
        pny = (py - (H - 1) / 2.0) / fy
        rln = 1.0 / torch.sqrt(pnx ** 2 + pny ** 2 + 1)
        mdepth.view(-1)[lin] = tm * rln
        if mdepth_override is not None:
            # evaluate the implicit gradient at a given median depth (the backward
            # receives mdepth as an input, render_backward.cu:828)
            tm = torch.as_tensor(mdepth_override, dtype=dt).reshape(-1)[lin] / rln
        # implicit-gradient surrogate pieces (render_backward.cu:835-880, 983-999)
        logT = torch.zeros(npx, dtype=dt)
        dlogT_dt = torch.zeros(npx, dtype=dt)
        valid_px = (tm != 0) & (last > 0)
        for k, (al, tp, rs, mask) in enumerate(used):
            m = mask & ((k + 1) <= last) & valid_px
            if not bool(m.any()):
                continue
            delta = (tm - tp) * rs
            ge = torch.exp(-0.5 * delta * delta)
            Gt = al * ge
            f = torch.where(tm > tp, torch.log(1 - al) - 0.5 * torch.log(1 - Gt), 0.5 * torch.log(1 - Gt))
            if float(rs.detach()) <= 0:
                f = torch.where(tm > tp, torch.log(1 - al), torch.zeros_like(f))
            logT = logT + torch.where(m, f, torch.zeros_like(f))
            with torch.no_grad():
                dd = -0.5 * Gt / (1 - Gt) * delta.abs() * rs
                dlogT_dt = dlogT_dt + torch.where(m, dd, torch.zeros_like(dd))
        surrogate_terms.append((lin, logT, dlogT_dt, rln, valid_px))
    return dict(color=color, alpha=alpha_img, normal=normal_img, mdepth=mdepth, n_contrib=n_contrib,
                _surrogate=surrogate_terms)


def median_depth_surrogate(out, dL_dmdepth):
    """Scalar whose gradient is the reference's implicit median-depth gradient."""
    tot = 0.0
    g = dL_dmdepth.reshape(-1)
    for lin, logT, dlogT_dt, rln, valid in out["_surrogate"]:
        dT_dtm = 0.5 * dlogT_dt  # T = 1/2 at the median
        kappa = (g[lin] * rln) / torch.clamp(-dT_dtm, min=1e-7)
        kappa = torch.where(valid, kappa, torch.zeros_like(kappa))
        tot = tot + (kappa.detach() * 0.5 * logT).sum()
    return tot


def sample(pre, lists, points3D, view, proj, W, H, split=8, iters=5, sample_range=0.4, mdepth_override=None):
    """Median depth at 3D points (sample_forward.cu:9-53, 430-657), float64.

    Returns output [N, 3] = (pnx, pny, 1) * mdepth * rln with the median depth
    held constant (its gradient comes from `sample_surrogate`, the implicit
    derivative the reference's sample backward computes,
    sample_backward.cu:170-354), the inside flags, the per-point median depth
    (along-ray) and the surrogate pieces."""
    dt = pre["xy"].dtype
    pts = points3D.reshape(-1, 3)
    N = pts.shape[0]
    gx, gy = (W + 15) // 16, (H + 15) // 16
    t = pts @ view[:3, :3] + view[3, :3]
    p_hom = pts @ proj[:3] + proj[3]
    ndc = p_hom[:, :2] / (p_hom[:, 3:4] + 1e-7)
    xy = torch.stack([((ndc[:, 0] + 1.0) * W - 1.0) * 0.5, ((ndc[:, 1] + 1.0) * H - 1.0) * 0.5], 1)
    xyd = xy.detach()
    valid = ((t[:, 2] > 0.2) & (xyd[:, 0] >= 0) & (xyd[:, 0] <= W - 1) & (xyd[:, 1] >= 0)
             & (xyd[:, 1] <= H - 1)).detach()
    tx = torch.clamp(((xyd[:, 0] + 0.5) / 16).floor().long(), 0, gx - 1)
    ty = torch.clamp(((xyd[:, 1] + 0.5) / 16).floor().long(), 0, gy - 1)
    tile = torch.where(valid, ty * gx + tx, torch.full_like(tx, -1))
    fx = W / (2.0 * pre["_tanx"])
    fy = H / (2.0 * pre["_tany"])
    pnx = (xy[:, 0] - (W - 1) / 2.0) / fx
    pny = (xy[:, 1] - (H - 1) / 2.0) / fy
    rln = 1.0 / torch.sqrt(pnx ** 2 + pny ** 2 + 1)
    tm_all = torch.zeros(N, dtype=dt)
    inside = torch.zeros(N, dtype=torch.bool)
    last_all = torch.zeros(N, dtype=torch.long)
    terms = []
    for tl in torch.unique(tile[tile >= 0]).tolist():
        idx = torch.nonzero(tile == tl)[:, 0]
        lst = lists[tl]
        n = idx.shape[0]
        pxy = xy[idx]
        T = torch.ones(n, dtype=dt)
        m0 = torch.zeros(n, dtype=dt)
        done = torch.zeros(n, dtype=torch.bool)
        last = torch.zeros(n, dtype=torch.long)
        used = []
        for k, g in enumerate(lst):
            d = pre["xy"][g][None] - pxy
            co = pre["conic"][g]
            power = -0.5 * (co[0] * d[:, 0] ** 2 + co[2] * d[:, 1] ** 2) - co[1] * d[:, 0] * d[:, 1]
            al = _clamp_st(pre["opac"][g] * torch.exp(power))
            ok = (~done) & (power <= 0).detach() & (al >= 1.0 / 255.0).detach()
            test_T = T * (1 - al)
            stop = ok & (test_T < 1e-4).detach()
            done = done | stop
            ok = ok & ~stop
            rp = pre["ray_plane"][g]
            tp = rp[0] * d[:, 0] + rp[1] * d[:, 1] + rp[2]
            m0 = torch.where(ok & (T > 0.5).detach(), tp.detach(), m0)
            T = torch.where(ok, test_T, T)
            last = torch.where(ok, torch.full_like(last, k + 1), last)
            used.append((al, tp, rp[3], (power <= 0).detach() & (al >= 1.0 / 255.0).detach()))
        with torch.no_grad():
            dmin = torch.clamp(m0 - sample_range, min=0.0)
            dmax = torch.clamp(m0 + sample_range, min=0.0)
            in_range = T.detach() <= 0.45
            Tp = torch.ones(n, split + 1, dtype=dt)
            for it in range(iters):
                first = it == 0
                ids = range(0, split + 1) if first else range(1, split)
                for sidx in ids:
                    Tp[:, sidx] = 1.0
                interval = (dmax - dmin) / split
                for k, (al, tp, rs, mask) in enumerate(used):
                    m = mask & ((k + 1) <= last) & in_range
                    if not bool(m.any()):
                        continue
                    for sidx in ids:
                        ts = dmin + interval * sidx
                        delta = (ts - tp) * rs
                        gg = torch.exp(-0.5 * delta * delta) if float(rs) > 0 else torch.zeros_like(ts)
                        omg = 1 - al * gg
                        f = torch.where(ts > tp, 1 - al, omg) / torch.sqrt(omg)
                        Tp[:, sidx] = torch.where(m, Tp[:, sidx] * f, Tp[:, sidx])
                if first:
                    in_range = (Tp[:, 0] >= 0.5) & (Tp[:, split] <= 0.5) & in_range
                start = torch.zeros(n, dtype=torch.long)
                for p_ in range(1, split):
                    start = torch.where(Tp[:, p_] >= 0.5, torch.full_like(start, p_), start)
                dmax = dmin + (start + 1) * interval
                dmin = dmin + start * interval
                Tp0 = Tp.gather(1, start[:, None])[:, 0]
                Tp8 = Tp.gather(1, (start + 1)[:, None])[:, 0]
                Tp[:, 0], Tp[:, split] = Tp0, Tp8
            wmax = ((Tp[:, 0] - 0.5) / (Tp[:, 0] - Tp[:, split])).nan_to_num(0.0).clamp(0, 1)
            tm = torch.where(in_range, wmax * dmax + (1 - wmax) * dmin, torch.zeros_like(dmin))
        tm_all[idx] = tm
        inside[idx] = in_range
        last_all[idx] = last
        if mdepth_override is not None:
            tm = torch.as_tensor(mdepth_override, dtype=dt).reshape(-1)[idx]
        logT = torch.zeros(n, dtype=dt)
        dlogT_dt = torch.zeros(n, dtype=dt)
        valid_pt = in_range & (last > 0)
        for k, (al, tp, rs, mask) in enumerate(used):
            m = mask & ((k + 1) <= last) & valid_pt
            if not bool(m.any()):
                continue
            delta = (tm - tp) * rs
            Gt = al * torch.exp(-0.5 * delta * delta)
            f = torch.where(tm > tp, torch.log(1 - al) - 0.5 * torch.log(1 - Gt), 0.5 * torch.log(1 - Gt))
            if float(rs.detach()) <= 0:
                f = torch.where(tm > tp, torch.log(1 - al), torch.zeros_like(f))
            logT = logT + torch.where(m, f, torch.zeros_like(f))
            with torch.no_grad():
                dd = -0.5 * Gt / (1 - Gt) * delta.abs() * rs
                dlogT_dt = dlogT_dt + torch.where(m, dd, torch.zeros_like(dd))
        terms.append((idx, logT, dlogT_dt, valid_pt))
    tm_used = tm_all if mdepth_override is None else torch.as_tensor(mdepth_override, dtype=dt).reshape(-1)
    depth = tm_used.detach() * rln
    out = torch.stack([pnx * depth, pny * depth, depth], 1)
    out = torch.where(valid[:, None], out, torch.zeros_like(out))
    return dict(output=out.reshape(points3D.shape), inside=inside.reshape(points3D.shape[:-1]), mdepth=tm_all,
                n_contrib=last_all, tile=tile, _terms=terms, _pn=(pnx.detach(), pny.detach(), rln.detach()))


def point_distance(points3D, view):
    """|p_view| of world points (preprocessPointsCUDA ts, sample_forward.cu:50)."""
    pts = points3D.reshape(-1, 3)
    t = pts @ view[:3, :3] + view[3, :3]
    return torch.sqrt((t * t).sum(1))


def integrate(pre, lists, points3D, view, proj, W, H):
    """Vacancy transmittance of the Gaussian field at world points
    (evaluateTransmittanceCUDA, sample_forward.cu:55-169), float64, no
    gradient: per point the tile's list front to back, the composite's
    power / alpha / early-stop tests, and per blended Gaussian
    T_point *= (t > t_peak ? 1 - a : 1 - a g) / sqrt(1 - a g),
    g = exp(-((t_peak - t) rsigma)^2 / 2) (0 for rsigma <= 0)."""
    dt = pre["xy"].dtype
    pts = points3D.reshape(-1, 3).to(dt)
    N = pts.shape[0]
    gx, gy = (W + 15) // 16, (H + 15) // 16
    tv = pts @ view[:3, :3] + view[3, :3]
    p_hom = pts @ proj[:3] + proj[3]
    ndc = p_hom[:, :2] / (p_hom[:, 3:4] + 1e-7)
    xy = torch.stack([((ndc[:, 0] + 1.0) * W - 1.0) * 0.5, ((ndc[:, 1] + 1.0) * H - 1.0) * 0.5], 1)
    valid = (tv[:, 2] > 0.2) & (xy[:, 0] >= 0) & (xy[:, 0] <= W - 1) & (xy[:, 1] >= 0) & (xy[:, 1] <= H - 1)
    tx = torch.clamp(((xy[:, 0] + 0.5) / 16).floor().long(), 0, gx - 1)
    ty = torch.clamp(((xy[:, 1] + 0.5) / 16).floor().long(), 0, gy - 1)
    tile = torch.where(valid, ty * gx + tx, torch.full_like(tx, -1))
    pt_t = torch.sqrt((tv * tv).sum(1))
    T_out = torch.zeros(N, dtype=dt)
    with torch.no_grad():
        for tl in torch.unique(tile[tile >= 0]).tolist():
            idx = torch.nonzero(tile == tl)[:, 0]
            pxy, tpt = xy[idx], pt_t[idx]
            n = idx.shape[0]
            T = torch.ones(n, dtype=dt)
            Tp = torch.ones(n, dtype=dt)
            done = torch.zeros(n, dtype=torch.bool)
            for g in lists[tl]:
                d = pre["xy"][g][None] - pxy
                co = pre["conic"][g]
                power = -0.5 * (co[0] * d[:, 0] ** 2 + co[2] * d[:, 1] ** 2) - co[1] * d[:, 0] * d[:, 1]
                al = _clamp_st(pre["opac"][g] * torch.exp(power))
                ok = (~done) & (power <= 0) & (al >= 1.0 / 255.0)
                test_T = T * (1 - al)
                stop = ok & (test_T < 1e-4)
                done = done | stop
                ok = ok & ~stop
                rp = pre["ray_plane"][g]
                tp = rp[0] * d[:, 0] + rp[1] * d[:, 1] + rp[2]
                gg = torch.exp(-0.5 * ((tp - tpt) * rp[3]) ** 2) if float(rp[3]) > 0 else torch.zeros_like(tp)
                omg = 1 - al * gg
                f = torch.where(tpt > tp, 1 - al, omg) / torch.sqrt(omg)
                Tp = torch.where(ok, Tp * f, Tp)
                T = torch.where(ok, test_T, T)
            T_out[idx] = Tp
    return dict(transmittance=T_out, inside=tile >= 0, tile=tile)


def sample_surrogate(out, dL_doutput):
    """Scalar whose gradient is the reference's implicit median-depth gradient
    of the sampled points (sample_backward.cu:138-215, 289-301)."""
    g = dL_doutput.reshape(-1, 3)
    pnx, pny, rln = out["_pn"]
    dL_dDepth = rln * (g[:, 0] * pnx + g[:, 1] * pny + g[:, 2])
    tot = 0.0
    for idx, logT, dlogT_dt, valid in out["_terms"]:
        kappa = dL_dDepth[idx] / torch.clamp(-0.5 * dlogT_dt, min=1e-7)
        kappa = torch.where(valid, kappa, torch.zeros_like(kappa))
        tot = tot + (kappa.detach() * 0.5 * logT).sum()
    return tot


def _bilinear(img, u, v):
    """Bilinear sample of img [H, W] at (u, v) with taps (floor, floor + 1),
    clamped to the image, differentiable in (u, v) (warp_patch_ncc_impl.cu:178-199)."""
    H, W = img.shape
    u0f, v0f = torch.floor(u.detach()), torch.floor(v.detach())
    u0 = u0f.long().clamp(0, W - 1)
    v0 = v0f.long().clamp(0, H - 1)
    u1 = (u0f + 1).long().clamp(0, W - 1)
    v1 = (v0f + 1).long().clamp(0, H - 1)
    wu1, wv1 = u - u0f, v - v0f
    wu0, wv0 = (u0f + 1) - u, (v0f + 1) - v
    c00, c01, c10, c11 = img[v0, u0], img[v0, u1], img[v1, u0], img[v1, u1]
    return wv0 * (wu0 * c00 + wu1 * c01) + wv1 * (wu0 * c10 + wu1 * c11)


def warp_patch_ncc(depths, normals, uvs, R, T, image_r, image_n, fx_r, fy_r, cx_r, cy_r, fx_n, fy_n, cx_n, cy_n):
    """Dense float64 restatement of the warp-patch NCC (warp_patch_ncc_impl.cu:18-266): the 7x7 half-step patch
    around each reference pixel is mapped by the plane-induced homography H = K_n (R - T n^T / d) K_r^-1 with
    d = -n . K_r^-1 (u, v, 1) * depth; NCC = cross^2 / (var_r var_n + 1e-8).  Returns (ncc, valid) with ncc
    differentiable in depths and normals (autograd replaces the reference's forward-mode derivative).
    R is indexed as the reference's column-major float33 (column i = R[3i:3i+3])."""
    dt = depths.dtype
    P = depths.shape[0]
    u = uvs[:, 0].to(dt)
    v = uvs[:, 1].to(dt)
    pnr = torch.stack([(u - cx_r) / fx_r, (v - cy_r) / fy_r, torch.ones_like(u)], 1)
    dist = -(pnr * normals).sum(1) * depths
    Rm = R.reshape(3, 3).T.to(dt)  # math matrix: column i = R[3i:3i+3]
    Kn = torch.tensor([[fx_n, 0, cx_n], [0, fy_n, cy_n], [0, 0, 1]], dtype=dt)
    Kr_inv = torch.tensor([[1 / fx_r, 0, -cx_r / fx_r], [0, 1 / fy_r, -cy_r / fy_r], [0, 0, 1]], dtype=dt)
    Hn = Rm[None] - T.to(dt)[None, :, None] * (normals / dist[:, None])[:, None, :]
    H = Kn[None] @ Hn @ Kr_inv[None]
    offs = torch.arange(-3, 4, dtype=dt) * 0.5
    dv, du = torch.meshgrid(offs, offs, indexing="ij")
    ur = u[:, None] + du.reshape(1, -1)
    vr = v[:, None] + dv.reshape(1, -1)
    c_r = _bilinear(image_r.to(dt), ur, vr)
    hom = torch.stack([ur, vr, torch.ones_like(ur)], -1)  # [P, 49, 3]
    w = hom @ H.transpose(1, 2)
    un, vn = w[..., 0] / w[..., 2], w[..., 1] / w[..., 2]
    Hn_img, Wn_img = image_n.shape
    inside_n = ((un - 1.5 > 0) & (un + 1.5 < Wn_img - 1) & (vn - 1.5 > 0) & (vn + 1.5 < Hn_img - 1)).all(1)
    Hr_img, Wr_img = image_r.shape
    inside_r = (u - 1.5 > 0) & (u + 1.5 < Wr_img - 1) & (v - 1.5 > 0) & (v + 1.5 < Hr_img - 1)
    c_n = _bilinear(image_n.to(dt), un, vn)
    n = 49.0
    s_r, s_n = c_r.sum(1), c_n.sum(1)
    cross = (c_r * c_n).sum(1) - s_r * s_n / n
    var_r = (c_r * c_r).sum(1) - s_r * s_r / n
    var_n = (c_n * c_n).sum(1) - s_n * s_n / n
    ncc = cross * cross / (var_r * var_n + 1e-8)
    valid = (inside_r & inside_n & (var_r > 5e-6) & (var_n > 5e-6)).detach()
    return torch.where(valid, ncc, torch.zeros_like(ncc)), valid
