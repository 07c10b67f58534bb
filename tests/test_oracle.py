"""CPU tests: pin the C oracle (oracle/gsr_oracle.c) before it is trusted as
the parity checker of the HIP path.

  * golden fixtures produced by the reference's own Python (tests/golden/):
    SH evaluation, camera matrices, GaussianModel getters;
  * an independent float64 torch-autograd restatement (tests/torch_ref.py):
    forward outputs and every gradient;
  * closed-form known-answer tests (single isotropic Gaussian, depth ties,
    tile-rect borders, getHigherMsb).
"""
from __future__ import annotations

import math
import os

import numpy as np
import pytest
import torch

import gsr_scene as S
import helpers as Hh
import torch_ref as R
import torch_ref as R_
from oracle import gsr_oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


# ---------------------------------------------------------------- fixtures
def test_sh_matches_reference_eval_sh():
    """oracle colour == reference utils/sh_utils.eval_sh + 0.5, clamped (render_forward.cu:22-78)."""
    d = np.load(os.path.join(GOLD, "sh_eval.npz"))
    for deg in range(4):
        sh, dirs, ref = d[f"sh_{deg}"], d[f"dirs_{deg}"], d[f"out_{deg}"]
        for i in range(sh.shape[0]):
            mean = dirs[i] * 3.0  # campos = 0 -> normalised direction == dirs[i]
            rgb, cl = O.eval_color(deg, mean, np.zeros(3), sh[i].T.copy())
            want = ref[i] + 0.5
            np.testing.assert_allclose(rgb, np.maximum(want, 0.0), rtol=2e-6, atol=2e-6)
            assert (cl == (want < 0)).all()


def test_cameras_match_reference():
    d = np.load(os.path.join(GOLD, "cameras.npz"))
    for i in range(3):
        W, H = (int(v) for v in d[f"wh_{i}"])
        fovx, fovy = d[f"fov_{i}"]
        cam = S.make_camera(W, H, R=d[f"R_{i}"], T=d[f"T_{i}"], fovx_deg=math.degrees(fovx))
        assert abs(cam.FoVy - fovy) < 1e-12
        np.testing.assert_allclose(cam.world_view_transform.numpy(), d[f"world_view_{i}"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(cam.full_proj_transform.numpy(), d[f"full_proj_{i}"], rtol=0, atol=1e-5)
        np.testing.assert_allclose(cam.camera_center.numpy(), d[f"center_{i}"], rtol=0, atol=1e-5)


def test_getters_and_filter3d_match_reference():
    d = np.load(os.path.join(GOLD, "getters.npz"))
    t = lambda k: torch.tensor(d["raw_" + k])  # noqa: E731

    class Cam:
        def __init__(self, R, T, whf):
            self.R, self.T = torch.tensor(R), torch.tensor(T)
            self.image_width, self.image_height, self.Fx = float(whf[0]), float(whf[1]), float(whf[2])
            self.Fy = self.Fx

    cams = [Cam(d["cam_R"][k], d["cam_T"][k], d["cam_WHF"][k]) for k in range(2)]
    filt = S.compute_filter_3D(t("xyz"), cams)
    np.testing.assert_allclose(filt.numpy(), d["filter_3D"], rtol=1e-6, atol=0)
    raw = S.RawGaussians(t("xyz"), t("features_dc"), t("features_rest"), t("scaling"), t("rotation"), t("opacity"),
                         t("sg_axis"), t("sg_sharpness"), t("sg_color"), torch.tensor(d["filter_3D"]))
    scales, opac = raw.get_scaling_n_opacity_with_3D_filter()
    np.testing.assert_array_equal(scales.numpy(), d["scales"])
    np.testing.assert_array_equal(opac.numpy(), d["opacity"])
    np.testing.assert_array_equal(raw.get_rotation().numpy(), d["rotation_out"])
    np.testing.assert_array_equal(raw.get_features().numpy(), d["features"])
    np.testing.assert_array_equal(raw.get_sg_axis().numpy(), d["sg_axis_out"])
    np.testing.assert_array_equal(raw.get_sg_sharpness().numpy(), d["sg_sharpness_out"])
    np.testing.assert_array_equal(raw.get_sg_color().numpy(), d["sg_color_out"])


# ------------------------------------------------- oracle vs float64 autograd
def _torch_ref(c, require_depth=True, colors_precomp=None, sgd=0, kernel_size=0.0, mdepth=None):
    P = c["inp"]["means3D"].shape[0]
    inp = {k: v.double().clone().requires_grad_(True) for k, v in c["inp"].items()}
    cp = None if colors_precomp is None else colors_precomp.double().clone().requires_grad_(True)
    m2d = torch.zeros(P, 3, dtype=torch.float64, requires_grad=True)
    cam = c["cam"]
    pre = R.preprocess(inp["means3D"], inp["scales"], inp["rotations"], inp["opacities"], inp["shs"],
                       inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"], m2d, cam.world_view_transform.double(),
                       cam.full_proj_transform.double(), cam.camera_center.double(), c["W"], c["H"], c["tanx"],
                       c["tany"], kernel_size, c["sh_degree"], sgd, colors_precomp=cp)
    lists, radii = R.binning(pre, c["W"], c["H"])
    out = R.render(pre, lists, c["W"], c["H"], c["bg"].double(), require_depth=require_depth,
                   mdepth_override=None if mdepth is None else torch.as_tensor(mdepth).double())
    return inp, m2d, cp, out, radii


CASES = [
    dict(P=40, W=40, H=24, seed=0),
    dict(P=60, W=48, H=40, seed=3, kernel_size=0.1),
    dict(P=50, W=37, H=29, seed=5, sgm=2, sg_degree=2),
    dict(P=45, W=40, H=24, seed=7, require_depth=False),
    dict(P=45, W=40, H=24, seed=9, bg=(0.2, 0.5, 1.0)),
    # the alpha = 0.99 clamp (logits up to 6: o up to 0.9975) with its pass-through gradient
    dict(P=60, W=40, H=32, seed=40, opacity_max_logit=6.0, opacity_std=3.0),
    # the SH warm-up layout (train.py:130): 16 SH rows rendered at active degree 0, 1, 2
    dict(P=45, W=40, H=24, seed=41, sh_degree=0, sh_max_degree=3),
    dict(P=45, W=40, H=24, seed=42, sh_degree=1, sh_max_degree=3),
    dict(P=45, W=40, H=24, seed=43, sh_degree=2, sh_max_degree=3),
]


def test_cov3d_matches_reference_fixture():
    """The covariance convention (the glm column-major hazard)
    pinned to the reference's own Python: scene/gaussian_model.py:46-50
    build_covariance_from_scaling_rotation over utils/general_utils.py:77-113
    (tests/golden/cov3d.npz), forward and fp32 autograd gradients.  The
    kernels' Sigma = (S R)^T (S R) (gsro_cov3d) equals the reference's
    L L^T (L = R S); computeCov3D's backward (render_backward.cu:193-244)
    gives dL/d(mod scale) (the Python gradient is mod times
    it) and dL/dq of the unnormalised quaternion (App. B.3: the Python,
    which normalises, sees its tangential part)."""
    d = np.load(os.path.join(GOLD, "cov3d.npz"))
    q = d["rotations"].astype(np.float64)
    for tag, mod in (("m1", 1.0), ("m07", 0.7)):
        cov = O.cov3d(d["scales"], mod, d["rotations"])
        ref = d["cov_" + tag]
        assert np.abs(cov - ref).max() <= 2e-6 * np.abs(ref).max(), tag
        ds, dq = O.cov3d_backward(d["scales"], mod, d["rotations"], d["upstream"])
        want_s = d["dscales_" + tag]
        assert np.abs(mod * ds - want_s).max() <= 1e-5 * np.abs(want_s).max(), tag
        dq = dq.astype(np.float64)
        tang = dq - q * (q * dq).sum(1, keepdims=True)
        want_q = d["drotations_" + tag]
        assert np.abs(tang - want_q).max() <= 1e-5 * np.abs(want_q).max(), tag
    # a transposed rotation (the classic mis-transpose) is caught by the fixture
    qt = d["rotations"].copy()
    qt[:, 1:] *= -1  # conjugate quaternion: R^T
    assert np.abs(O.cov3d(d["scales"], 1.0, qt) - d["cov_m1"]).max() > 1e-3 * np.abs(d["cov_m1"]).max()


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_oracle_matches_float64_autograd(case):
    case = dict(case)
    ks = case.pop("kernel_size", 0.0)
    geom = case.get("require_depth", True)
    c = Hh.small_case(kernel_size=ks, **case)
    o = O.forward(*Hh.oracle_args(c))
    # the median-depth gradient is evaluated at the oracle's own median depth
    # (it is an input of the backward); the forward mdepth is compared above
    inp, m2d, _, out, radii = _torch_ref(c, require_depth=geom, sgd=c["sg_degree"], kernel_size=ks,
                                         mdepth=o["mdepth"] if geom else None)
    assert (radii == o["radii"]).all()
    assert (out["n_contrib"] == o["state"].n_contrib()).all()
    for k in ("color", "alpha") + (("normal", "mdepth") if geom else ()):
        assert Hh.rel_err(o[k], out[k].detach().numpy()) < 5e-5, k
    g = S.upstream_grads(c["H"], c["W"])
    L = (out["color"] * g["color"].double()).sum() + (out["alpha"] * g["alpha"].double()).sum()
    if geom:
        L = L + (out["normal"] * g["normal"].double()).sum() + R.median_depth_surrogate(out, g["mdepth"].double())
    L.backward()
    b = O.backward(o["state"], *Hh.oracle_args(c)[:19], g["color"], g["mdepth"], g["alpha"], g["normal"], o["alpha"],
                   o["normal"], o["mdepth"], c["cam"].camera_center, o["radii"])
    q = c["inp"]["rotations"].double().numpy()
    tang = lambda v: v - q * (q * v).sum(1, keepdims=True)  # noqa: E731 - dL/dq is defined up to the radial part
    checks = {
        "dmeans3D": (b["dmeans3D"], inp["means3D"].grad.numpy()),
        "dscales": (b["dscales"], inp["scales"].grad.numpy()),
        "drotations": (tang(b["drotations"]), tang(inp["rotations"].grad.numpy())),
        "dopacity": (b["dopacity"], inp["opacities"].grad.numpy()),
        "dsh": (b["dsh"], inp["shs"].grad.numpy()),
        "dmeans2D": (b["dmeans2D"][:, :2], m2d.grad[:, :2].numpy()),
    }
    if c["sg_degree"]:
        checks.update(dsg_axis=(b["dsg_axis"], inp["sg_axis"].grad.numpy()),
                      dsg_sharpness=(b["dsg_sharpness"], inp["sg_sharpness"].grad.numpy()),
                      dsg_color=(b["dsg_color"], inp["sg_color"].grad.numpy()))
    for k, (mine, ref) in checks.items():
        assert Hh.rel_err(mine, ref) < 2e-4, (k, Hh.rel_err(mine, ref))
    if case.get("opacity_max_logit", 2.0) > 4.6:  # the case must reach the clamp
        assert int((c["inp"]["opacities"] > 0.99).sum()) > 0
    if case.get("sh_max_degree"):  # rows past the active degree get exactly zero
        n = (c["sh_degree"] + 1) ** 2
        assert not np.any(b["dsh"][:, n:]) and b["dsh"].shape[1] == 16


def test_oracle_colors_precomp_path():
    c = Hh.small_case(P=40, W=40, H=24, seed=11)
    cols = torch.rand(40, 3, generator=torch.Generator().manual_seed(1))
    o = O.forward(*Hh.oracle_args(c, colors_precomp=cols))
    inp, m2d, cp, out, _ = _torch_ref(c, colors_precomp=cols, mdepth=o["mdepth"])
    assert Hh.rel_err(o["color"], out["color"].detach().numpy()) < 5e-5
    g = S.upstream_grads(c["H"], c["W"])
    L = (out["color"] * g["color"].double()).sum() + (out["normal"] * g["normal"].double()).sum()
    L = L + R.median_depth_surrogate(out, g["mdepth"].double())
    L.backward()
    args = Hh.oracle_args(c, colors_precomp=cols)
    b = O.backward(o["state"], *args[:19], g["color"], g["mdepth"], g["alpha"], g["normal"], o["alpha"], o["normal"],
                   o["mdepth"], c["cam"].camera_center, o["radii"])
    assert Hh.rel_err(b["dcolors"], cp.grad.numpy()) < 1e-5
    assert Hh.rel_err(b["dmeans3D"], inp["means3D"].grad.numpy()) < 2e-4
    assert b["dsh"].size == 0


def test_median_depth_gradient_is_implicit_derivative():
    """The reference's median-depth gradient (render_backward.cu:835-880,
    983-999) equals the finite-difference derivative of the float64 bisection
    result w.r.t. a Gaussian's opacity (implicit-function theorem)."""
    c = Hh.small_case(P=30, W=32, H=32, seed=4)
    cam = c["cam"]

    def mdepth_sum(op_scale, idx):
        inp = {k: v.double().clone() for k, v in c["inp"].items()}
        inp["opacities"][idx] *= op_scale
        m2d = torch.zeros(30, 3, dtype=torch.float64)
        pre = R.preprocess(inp["means3D"], inp["scales"], inp["rotations"], inp["opacities"], inp["shs"],
                           inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"], m2d,
                           cam.world_view_transform.double(), cam.full_proj_transform.double(),
                           cam.camera_center.double(), 32, 32, c["tanx"], c["tany"], 0.0, 3, 0)
        lists, _ = R.binning(pre, 32, 32)
        return R.render(pre, lists, 32, 32, c["bg"].double(), iters=12)

    base = mdepth_sum(1.0, 0)
    md = base["mdepth"].detach()
    inp = {k: v.double().clone().requires_grad_(True) for k, v in c["inp"].items()}
    m2d = torch.zeros(30, 3, dtype=torch.float64)
    pre = R.preprocess(inp["means3D"], inp["scales"], inp["rotations"], inp["opacities"], inp["shs"], inp["sg_axis"],
                       inp["sg_sharpness"], inp["sg_color"], m2d, cam.world_view_transform.double(),
                       cam.full_proj_transform.double(), cam.camera_center.double(), 32, 32, c["tanx"], c["tany"],
                       0.0, 3, 0)
    lists, _ = R.binning(pre, 32, 32)
    out = R.render(pre, lists, 32, 32, c["bg"].double(), iters=12)
    w = (md > 0).double()  # pixels with a defined median depth
    R.median_depth_surrogate(out, w).backward()
    # pick the Gaussian with the largest analytic sensitivity
    g = inp["opacities"].grad[:, 0].abs()
    idx = int(torch.argmax(g))
    eps = 1e-5
    fp = mdepth_sum(1 + eps, idx)["mdepth"]
    fm = mdepth_sum(1 - eps, idx)["mdepth"]
    fd = float(((fp - fm) * w).sum() / (2 * eps * float(c["inp"]["opacities"][idx])))
    an = float(inp["opacities"].grad[idx, 0])
    assert abs(an) > 0
    assert abs(fd - an) <= 2e-2 * abs(an) + 1e-9, (fd, an)


# ------------------------------------------------------------------- KATs
def test_kat_single_isotropic_gaussian():
    """One isotropic Gaussian on the optical axis (SURVEY §8(c) KAT 1)."""
    W = H = 64
    cam = S.make_camera(W, H)
    z, s, o = 4.0, 0.05, 0.8
    means = torch.tensor([[0.0, 0.0, z]])
    scales = torch.full((1, 3), s)
    rot = torch.tensor([[1.0, 0.0, 0.0, 0.0]])
    op = torch.tensor([[o]])
    sh = torch.zeros(1, 16, 3)
    sh[0, 0] = torch.tensor([0.2, -0.1, 0.4]) / 0.28209479177387814  # colour = sh0*C0 + 0.5
    tanx = math.tan(cam.FoVx / 2)
    tany = math.tan(cam.FoVy / 2)
    bg = torch.tensor([0.1, 0.2, 0.3])
    out = O.forward(bg, means, None, op, scales, rot, None, sh, torch.zeros(1, 0, 3), torch.zeros(1, 0),
                    torch.zeros(1, 0, 3), 0, 0, 1.0, cam.world_view_transform, cam.full_proj_transform, tanx, tany, 0.0,
                    H, W, cam.camera_center, False, True)
    f = W / (2 * tanx)
    sigma_px = s * f / z
    lam = sigma_px ** 2 + 0.0
    assert out["radii"][0] == math.ceil(3 * math.sqrt(lam + math.sqrt(0.1)))  # mid^2-det clamped at 0.1
    # the centre ((W-1)/2) falls between pixels; check the 4 central pixels
    rgb = np.array([0.7, 0.4, 0.9])
    c = (W - 1) / 2
    for py in (31, 32):
        for px in (31, 32):
            d2 = (px - c) ** 2 + (py - c) ** 2
            a = min(0.99, o * math.exp(-0.5 * d2 / lam))
            np.testing.assert_allclose(out["color"][:, py, px], a * rgb + (1 - a) * bg.numpy(), rtol=2e-5)
            np.testing.assert_allclose(out["alpha"][0, py, px], a, rtol=2e-5)
            np.testing.assert_allclose(out["normal"][:, py, px], [0, 0, -1], atol=2e-3)
            if a >= 0.55:  # T <= 0.45 -> median depth defined: the Gaussian's depth along the pixel ray
                pnx, pny = (px - c) / f, (py - c) / f
                ray = math.sqrt(pnx ** 2 + pny ** 2 + 1)
                assert abs(out["mdepth"][0, py, px] * ray - z) < 3 * s


def test_kat_depth_ties_keep_index_order():
    """Equal sort keys keep emission (Gaussian index) order: stable LSD sort."""
    W = H = 32
    cam = S.make_camera(W, H)
    P = 4
    means = torch.tensor([[0.0, 0.0, 3.0]] * P)  # identical depth, identical tile
    scales = torch.full((P, 3), 0.03)
    rot = torch.tensor([[1.0, 0.0, 0.0, 0.0]] * P)
    op = torch.full((P, 1), 0.3)
    cols = torch.rand(P, 3, generator=torch.Generator().manual_seed(0))
    out = O.forward(torch.zeros(3), means, cols, op, scales, rot, None, None, None, None, None, 0, 0, 1.0,
                    cam.world_view_transform, cam.full_proj_transform, math.tan(cam.FoVx / 2),
                    math.tan(cam.FoVy / 2), 0.0, H, W, cam.camera_center, False, False)
    b = out["state"].binning()
    keys, plist = b["keys"], b["point_list"]
    for t in np.unique(keys >> np.uint64(32)):
        sel = plist[(keys >> np.uint64(32)) == t]
        assert list(sel) == sorted(sel)
    assert out["num_rendered"] == 4 * out["state"].geometry()["tiles_touched"][0]


def test_kat_rect_at_borders():
    """tiles_touched equals the getRect area (auxiliary.h:42-49), including
    Gaussians hanging over the image border and fully off-screen ones."""
    W, H = 50, 34  # ragged last tiles
    cam = S.make_camera(W, H)
    rng = np.random.default_rng(3)
    P = 400
    z = rng.uniform(1.5, 4.0, P)
    tx = math.tan(cam.FoVx / 2)
    ty = math.tan(cam.FoVy / 2)
    means = np.stack([rng.uniform(-1.6, 1.6, P) * z * tx, rng.uniform(-1.6, 1.6, P) * z * ty, z], 1)
    scales = np.exp(rng.normal(math.log(0.05), 0.5, (P, 3)))
    rot = rng.normal(size=(P, 4))
    rot /= np.linalg.norm(rot, axis=1, keepdims=True)
    cols = rng.uniform(size=(P, 3))
    out = O.forward(torch.zeros(3), means, cols, np.full((P, 1), 0.5), scales, rot, None, None, None, None, None,
                    0, 0, 1.0, cam.world_view_transform, cam.full_proj_transform, tx, ty, 0.0, H, W,
                    cam.camera_center, False, False)
    g = out["state"].geometry()
    gx, gy = (W + 15) // 16, (H + 15) // 16
    for i in range(P):
        r = int(out["radii"][i])
        if r == 0:
            assert g["tiles_touched"][i] == 0
            continue
        x, y = g["means2D"][i]
        x0 = min(gx, max(0, int((x - r) / 16)))
        y0 = min(gy, max(0, int((y - r) / 16)))
        x1 = min(gx, max(0, int((x + r + 15) / 16)))
        y1 = min(gy, max(0, int((y + r + 15) / 16)))
        assert g["tiles_touched"][i] == (x1 - x0) * (y1 - y0)
    assert (out["radii"] == 0).sum() > 0 and (out["radii"] > 0).sum() > 0


@pytest.mark.parametrize("n,want", [(1, 1), (2, 2), (255, 8), (256, 9), (2500, 12), (8160, 13), (65536, 17)])
def test_higher_msb(n, want):
    assert O.higher_msb(n) == want


def test_empty_and_all_culled():
    W, H = 32, 16
    cam = S.make_camera(W, H)
    out = O.forward(torch.zeros(3), np.zeros((0, 3)), None, np.zeros((0, 1)), np.zeros((0, 3)), np.zeros((0, 4)),
                    None, np.zeros((0, 16, 3)), None, None, None, 3, 0, 1.0, cam.world_view_transform,
                    cam.full_proj_transform, 0.5, 0.3, 0.0, H, W, cam.camera_center, False, True)
    assert out["num_rendered"] == 0 and out["color"].sum() == 0
    # every Gaussian behind the near plane
    means = np.array([[0.0, 0.0, 0.1], [0.0, 0.0, -2.0]])
    out = O.forward(torch.tensor([0.5, 0.5, 0.5]), means, np.ones((2, 3)), np.full((2, 1), 0.5),
                    np.full((2, 3), 0.1), np.array([[1.0, 0, 0, 0]] * 2), None, None, None, None, None, 0, 0, 1.0,
                    cam.world_view_transform, cam.full_proj_transform, 0.5, 0.3, 0.0, H, W, cam.camera_center, False,
                    True)
    assert out["num_rendered"] == 0 and (out["radii"] == 0).all()
    np.testing.assert_allclose(out["color"], 0.5)
    assert (out["alpha"] == 0).all() and (out["mdepth"] == 0).all() and (out["normal"] == 0).all()


def test_mark_visible():
    cam = S.make_camera(16, 16)
    means = np.array([[0, 0, 0.1], [0, 0, 0.3], [5, 5, 1.0], [0, 0, -1]], np.float32)
    assert list(O.mark_visible(means, cam.world_view_transform)) == [False, True, True, False]


# ------------------------------------------------------------ sample_depth
def sample_points(c, n, seed, z_range=(1.5, 4.5)):
    """Random 3D points in the camera's view (pixel position + depth), plus a
    few behind the near plane and a few projecting outside the image."""
    g = torch.Generator().manual_seed(seed)
    W, H = c["W"], c["H"]
    fx, fy = W / (2 * c["tanx"]), H / (2 * c["tany"])
    px = torch.rand(n, generator=g) * (W + 8) - 4
    py = torch.rand(n, generator=g) * (H + 8) - 4
    z = torch.rand(n, generator=g) * (z_range[1] - z_range[0]) + z_range[0]
    z[: max(1, n // 50)] = 0.1  # behind the near plane
    cam_pts = torch.stack([(px - (W - 1) / 2) / fx * z, (py - (H - 1) / 2) / fy * z, z], 1)
    V = c["cam"].world_view_transform  # p_view = p @ V[:3, :3] + V[3, :3]
    world = (cam_pts - V[3, :3]) @ torch.linalg.inv(V[:3, :3])
    return world.float().contiguous()


def sample_args(c, pts, kernel_size=0.0):
    inp = c["inp"]
    return (pts, inp["means3D"], inp["opacities"], inp["scales"], inp["rotations"], 1.0, None,
            c["cam"].world_view_transform, c["cam"].full_proj_transform, c["tanx"], c["tany"], kernel_size, c["H"],
            c["W"], c["cam"].camera_center, False)


@pytest.mark.parametrize("seed", [0, 1])
def test_sample_depth_matches_float64_autograd(seed):
    """sample_depth forward (median depth at points, sample_forward.cu:430-657)
    and every gradient of its backward (sample_backward.cu:42-359 + the
    Gaussian preprocess backward) against the float64 autograd restatement."""
    c = Hh.small_case(P=150, W=40, H=32, seed=seed)
    pts = sample_points(c, 300, seed + 10).reshape(20, 15, 3)
    o = O.sample_forward(*sample_args(c, pts))
    assert o["num_points"] > 150 and o["inside"].sum() > 50
    op = o["state"].points()
    cam = c["cam"]
    inp = {k: v.double().clone().requires_grad_(True) for k, v in c["inp"].items()}
    p64 = pts.double().clone().requires_grad_(True)
    m2d = torch.zeros(150, 3, dtype=torch.float64)
    pre = R.preprocess(inp["means3D"], inp["scales"], inp["rotations"], inp["opacities"], inp["shs"],
                       inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"], m2d, cam.world_view_transform.double(),
                       cam.full_proj_transform.double(), cam.camera_center.double(), c["W"], c["H"], c["tanx"],
                       c["tany"], 0.0, 3, 0)
    lists, _ = R.binning(pre, c["W"], c["H"])
    out = R.sample(pre, lists, p64, cam.world_view_transform.double(), cam.full_proj_transform.double(), c["W"],
                   c["H"], mdepth_override=op["median_depth"].astype(np.float64))
    assert np.array_equal(o["inside"], out["inside"].numpy())
    assert np.array_equal(op["n_contrib"], out["n_contrib"].numpy())
    ref_md = out["mdepth"].numpy()
    assert Hh.rel_err(op["median_depth"], ref_md) < 5e-5
    assert Hh.rel_err(o["output"], out["output"].detach().numpy()) < 5e-5
    g = torch.randn(pts.shape, generator=torch.Generator().manual_seed(seed)) * 1e-2
    L = (out["output"] * g.double()).sum() + R.sample_surrogate(out, g.double())
    L.backward()
    b = O.sample_backward(o["state"], *sample_args(c, pts)[:9], o["inside"], g, c["tanx"], c["tany"], 0.0)
    q = c["inp"]["rotations"].double().numpy()
    tang = lambda v: v - q * (q * v).sum(1, keepdims=True)  # noqa: E731
    checks = {"dmeans3D": (b["dmeans3D"], inp["means3D"].grad.numpy()),
              "dscales": (b["dscales"], inp["scales"].grad.numpy()),
              "drotations": (tang(b["drotations"]), tang(inp["rotations"].grad.numpy())),
              "dopacity": (b["dopacity"], inp["opacities"].grad.numpy()),
              "dpoints3D": (b["dpoints3D"], p64.grad.numpy())}
    for k, (mine, ref) in checks.items():
        assert np.abs(ref).max() > 0, k
        assert Hh.rel_err(mine, ref) < 2e-4, (k, Hh.rel_err(mine, ref))


def test_sample_depth_at_pixel_centres_equals_render():
    """A point placed on a pixel's ray samples the median depth the render
    forward computed for that pixel (same algorithm, same Gaussian lists)."""
    c = Hh.small_case(P=300, W=64, H=48, seed=1)
    o = O.forward(*Hh.oracle_args(c))
    md = o["mdepth"][0]
    md_in = np.zeros_like(md)
    md_in[1:-1, 1:-1] = md[1:-1, 1:-1]  # border centres may round outside [0, W-1] and be culled
    ys, xs = np.nonzero(md_in > 0)
    W, H = c["W"], c["H"]
    fx, fy = W / (2 * c["tanx"]), H / (2 * c["tany"])
    z = torch.tensor(md[ys, xs])
    cam_pts = torch.stack([(torch.tensor(xs, dtype=torch.float32) - (W - 1) / 2) / fx * z,
                           (torch.tensor(ys, dtype=torch.float32) - (H - 1) / 2) / fy * z, z], 1)
    V = c["cam"].world_view_transform
    pts = ((cam_pts - V[3, :3]) @ torch.linalg.inv(V[:3, :3])).float().contiguous()
    s = O.sample_forward(*sample_args(c, pts))
    zs = s["output"][:, 2]
    close = np.abs(zs - md[ys, xs]) <= 1e-4 * np.abs(md).max()
    assert close.mean() > 0.995, close.mean()  # points land within ~1e-5 px of the centre
    assert s["inside"].mean() > 0.995


# ------------------------------------------------- integrate / evaluate_sdf
def query_args(c, pts, cov3D=None):
    """The 18-argument tuple of _C.integrate_gaussians_to_points /
    evaluate_sdf_from_signle_view (DGR/__init__.py:369-388)."""
    inp = c["inp"]
    scales, rots = (inp["scales"], inp["rotations"]) if cov3D is None else (None, None)
    return (pts, inp["means3D"], inp["opacities"], scales, rots, 1.0, cov3D, None, c["cam"].world_view_transform,
            c["cam"].full_proj_transform, c["tanx"], c["tany"], 0.0, c["H"], c["W"], c["cam"].camera_center, False,
            False)


def _ref_pre(c):
    cam = c["cam"]
    inp = {k: v.double() for k, v in c["inp"].items()}
    pre = R.preprocess(inp["means3D"], inp["scales"], inp["rotations"], inp["opacities"], inp["shs"],
                       inp["sg_axis"], inp["sg_sharpness"], inp["sg_color"],
                       torch.zeros(inp["means3D"].shape[0], 3, dtype=torch.float64), cam.world_view_transform.double(),
                       cam.full_proj_transform.double(), cam.camera_center.double(), c["W"], c["H"], c["tanx"],
                       c["tany"], 0.0, 3, 0)
    lists, _ = R.binning(pre, c["W"], c["H"])
    return pre, lists


@pytest.mark.parametrize("seed", [0, 1])
def test_integrate_matches_float64(seed):
    """integrate (evaluateTransmittanceCUDA, sample_forward.cu:55-169) against
    the float64 restatement: inside flags exact, transmittance <= 1e-5."""
    c = Hh.small_case(P=150, W=40, H=32, seed=seed)
    pts = sample_points(c, 400, seed + 20)
    K, T, inside = O.integrate(*query_args(c, pts))
    assert K > 0 and inside.sum() > 200
    pre, lists = _ref_pre(c)
    cam = c["cam"]
    ref = R.integrate(pre, lists, pts.double(), cam.world_view_transform.double(), cam.full_proj_transform.double(),
                      c["W"], c["H"])
    assert np.array_equal(inside, ref["inside"].numpy())
    assert (T[~inside] == 0).all()  # culled points keep torch::full(0) (rasterize_points.cu:314)
    Tr = ref["transmittance"].numpy()
    assert 0.05 < Tr[inside].mean() < 0.95  # the scene occludes a fair share of the points
    assert np.abs(T - Tr).max() <= 1e-5, np.abs(T - Tr).max()


@pytest.mark.parametrize("seed", [0, 1])
def test_evaluate_sdf_matches_float64(seed):
    """evaluate_sdf (evaluateSDFCUDA, sample_forward.cu:171-427: a +-0.8 first
    window and 6 bisection passes) against the float64 restatement: inside
    exact, depth <= 5e-5 relative, sdf = depth - |p_view|."""
    c = Hh.small_case(P=150, W=40, H=32, seed=seed)
    pts = sample_points(c, 400, seed + 30)
    K, depth, sdf, inside = O.evaluate_sdf(*query_args(c, pts))
    assert inside.sum() > 50
    pre, lists = _ref_pre(c)
    cam = c["cam"]
    out = R.sample(pre, lists, pts.double(), cam.world_view_transform.double(), cam.full_proj_transform.double(),
                   c["W"], c["H"], iters=6, sample_range=0.8)
    assert np.array_equal(inside, out["inside"].numpy())
    md = out["mdepth"].numpy()
    assert Hh.rel_err(depth, md) < 5e-5
    dist = R.point_distance(pts.double(), cam.world_view_transform.double()).numpy()
    in_view = out["tile"].numpy() >= 0
    ref_sdf = np.where(in_view, md - dist, 0.0)
    assert np.abs(sdf - ref_sdf).max() <= 5e-5 * np.abs(md).max()
    # the 6-pass +-0.8 search differs from sample_depth's 5-pass +-0.4 one
    s = O.sample_forward(*sample_args(c, pts))
    assert not np.array_equal(s["inside"], inside) or Hh.rel_err(depth, s["state"].points()["median_depth"]) > 0


def test_point_queries_against_render():
    """Known answers linking the queries to the render path: a point on a
    pixel centre's ray far behind every Gaussian (g = 0 for all of them) has
    integrate's transmittance = the render's 1 - alpha; a point at the
    rendered median depth has |sdf| ~ 0 where the median is defined."""
    c = Hh.small_case(P=300, W=64, H=48, seed=1)
    o = O.forward(*Hh.oracle_args(c))
    md, alpha = o["mdepth"][0], o["alpha"][0]
    W, H = c["W"], c["H"]
    fx, fy = W / (2 * c["tanx"]), H / (2 * c["tany"])
    ys, xs = np.mgrid[1:H - 1, 1:W - 1]
    ys, xs = ys.ravel(), xs.ravel()
    V = c["cam"].world_view_transform

    def world(z):
        z = torch.as_tensor(z, dtype=torch.float32)
        cam_pts = torch.stack([(torch.tensor(xs, dtype=torch.float32) - (W - 1) / 2) / fx * z,
                               (torch.tensor(ys, dtype=torch.float32) - (H - 1) / 2) / fy * z, z], 1)
        return ((cam_pts - V[3, :3]) @ torch.linalg.inv(V[:3, :3])).float().contiguous()

    K, T, inside = O.integrate(*query_args(c, world(np.full(xs.shape, 60.0))))
    assert inside.all()
    assert np.abs((1 - T) - alpha[ys, xs]).max() <= 1e-4
    sel = md[ys, xs] > 0
    z = np.where(sel, md[ys, xs], 3.0)
    K, depth, sdf, inside = O.evaluate_sdf(*query_args(c, world(z)))
    ok = sel & inside
    assert ok.mean() > 0.5
    # both bisections bracket the same root of T(t) = 1/2 (measured: 99th percentile 1.2e-6 at depth 2.5)
    assert np.percentile(np.abs(sdf[ok]), 99) <= 1e-4 * np.median(md[ys, xs][ok])


def test_point_queries_degenerate():
    c = Hh.small_case(P=50, W=40, H=32, seed=3)
    K, T, inside = O.integrate(*query_args(c, torch.zeros(0, 3)))
    assert K == 0 and T.shape == (0,) and inside.shape == (0,)
    pts = torch.tensor([[0.0, 0.0, -5.0], [100.0, 0.0, 3.0]])  # behind the camera / outside the image
    K, depth, sdf, inside = O.evaluate_sdf(*query_args(c, pts))
    assert not inside.any() and (depth == 0).all() and (sdf == 0).all()


# ------------------------------------------------------------ simple_knn
@pytest.mark.parametrize("P", [4, 5, 1000, 1023, 1025, 30000])
def test_knn_matches_exact_kdtree(P):
    """distCUDA2 restatement (submodules/simple-knn/simple_knn.cu:44-220):
    the mean squared distance to the 3 nearest other points equals scipy's
    exact k-d tree in float64 (the box pruning never drops a neighbour)."""
    from scipy.spatial import cKDTree

    rng = np.random.default_rng(P)
    pts = rng.normal(size=(P, 3)).astype(np.float32)
    pts[P // 2:] *= 0.01  # two scales
    got, order = O.knn_mean_dist(pts)
    d, _ = cKDTree(pts.astype(np.float64)).query(pts.astype(np.float64), k=4)
    ref = (d[:, 1:] ** 2).mean(1)
    assert np.abs(got - ref).max() <= 1e-6 * ref.max()
    assert np.all(np.abs(got - ref) <= 1e-5 * ref + 1e-30)
    assert sorted(order.tolist()) == list(range(P))


def test_knn_small_counts_follow_reference():
    """P < 4: the missing neighbours stay FLT_MAX in the sum (simple_knn.cu:146,
    172): P = 1, 2 give inf (FLT_MAX + FLT_MAX overflows), P = 3 gives
    (d1 + d2 + FLT_MAX) / 3."""
    got, _ = O.knn_mean_dist(np.array([[0, 0, 0]], np.float32))
    assert np.isinf(got).all()
    got, _ = O.knn_mean_dist(np.array([[0, 0, 0], [1, 0, 0]], np.float32))
    assert np.isinf(got).all()
    got, _ = O.knn_mean_dist(np.array([[0, 0, 0], [1, 0, 0], [0, 2, 0]], np.float32))
    assert np.allclose(got, np.float32(np.finfo(np.float32).max) / np.float32(3), rtol=1e-6)


# ---------------------------------------------------------- warp_patch_ncc
def ncc_case(P, seed, Wr=48, Hr=40, Wn=52, Hn=44):
    """Two smooth textured images, a relative pose (r to n) and random
    pixels with depths and normals facing the camera."""
    g = torch.Generator().manual_seed(seed)

    def texture(H, W):
        base = torch.rand(1, 1, H // 4 + 2, W // 4 + 2, generator=g)
        img = torch.nn.functional.interpolate(base, size=(H, W), mode="bicubic", align_corners=True)[0, 0]
        return (img + 0.05 * torch.rand(H, W, generator=g)).float().contiguous()

    img_r, img_n = texture(Hr, Wr), texture(Hn, Wn)
    a = torch.randn(3, generator=g, dtype=torch.float64)
    a = a / a.norm()
    th = 0.08
    K = torch.tensor([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]], dtype=torch.float64)
    Rm = torch.eye(3, dtype=torch.float64) + math.sin(th) * K + (1 - math.cos(th)) * K @ K
    T = (torch.randn(3, generator=g) * 0.1).float()
    R = Rm.T.reshape(-1).float().contiguous()  # column-major float33: column i at [3i:3i+3]
    uvs = torch.stack([torch.randint(3, Wr - 3, (P,), generator=g), torch.randint(3, Hr - 3, (P,), generator=g)],
                      1).int().contiguous()
    depths = (torch.rand(P, generator=g) * 2 + 2).float()
    nrm = torch.randn(P, 3, generator=g) * 0.3
    nrm[:, 2] = -1.0
    normals = (nrm / nrm.norm(dim=1, keepdim=True)).float().contiguous()
    K = dict(fx_r=50.0, fy_r=52.0, cx_r=Wr / 2 - 0.3, cy_r=Hr / 2 + 0.2, fx_n=55.0, fy_n=54.0, cx_n=Wn / 2,
             cy_n=Hn / 2 - 0.4)
    return depths, normals, uvs, R, T, img_r, img_n, K


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_warp_patch_ncc_matches_float64_autograd(seed):
    """warp_patch_ncc (warp_patch_ncc_impl.cu:18-266): NCC values, valid flags
    and the forward-mode d(NCC)/d(depth, normal) against autograd of an
    independent float64 restatement (textured images, so var_r var_n >> 1e-8
    and the reference's -ncc / (var_n + 1e-8) term is the exact derivative)."""
    d, n, uv, R, T, ir, inn, K = ncc_case(400, seed)
    o = O.warp_patch_ncc(d, n, uv, R, T, ir, inn, *K.values())
    assert o["valid"].sum() > 100
    dd = d.double().clone().requires_grad_(True)
    nd = n.double().clone().requires_grad_(True)
    ncc, valid = R_.warp_patch_ncc(dd, nd, uv, R, T, ir, inn, *K.values())
    assert np.array_equal(valid.numpy(), o["valid"])
    assert Hh.rel_err(o["ncc"], ncc.detach().numpy()) < 5e-4  # fp32 one-pass variances cancel
    ncc.sum().backward()
    assert Hh.rel_err(o["grad_depths"], dd.grad.numpy()) < 1e-3
    assert Hh.rel_err(o["grad_normals"], nd.grad.numpy()) < 1e-3


# ------------------------------------- loss restatements vs the reference's own Python
def _losses():
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "losses.npz"))


@pytest.mark.parametrize("i", [0, 1, 2])
@pytest.mark.parametrize("padding", ["same", "valid"])
def test_ssim_ref_matches_reference_fixture(i, padding):
    """oracle/ssim_ref.ssim (float64) against utils/loss_utils.py:36-72 _ssim
    run by the reference itself (fp32 torch; "valid" = its SSIM map cropped
    by 5): mean within 1e-6, dSSIM/dimg1 within 1e-5 relative L2."""
    from oracle import ssim_ref

    d = _losses()
    a = torch.tensor(d[f"ssim_img1_{i}"]).double().requires_grad_(True)
    b = torch.tensor(d[f"ssim_img2_{i}"]).double()
    v = ssim_ref.ssim(a, b, padding=padding)
    v.backward()
    want, gwant = float(d[f"ssim_{padding}_{i}"]), d[f"ssim_{padding}_grad_{i}"].astype(np.float64)
    assert abs(v.item() - want) <= 1e-6, (v.item(), want)
    assert np.linalg.norm(a.grad.numpy() - gwant) / np.linalg.norm(gwant) <= 1e-5


@pytest.mark.parametrize("i", [0, 1])
def test_depth_to_normal_ref_matches_reference_fixture(i):
    """oracle/ssim_ref.depth_to_normal against utils/graphics_utils.py:103-119
    run by the reference itself: valid exact, normals within 1e-5, the
    gradient of <normal, upstream> within 1e-5 relative L2 (the reference
    computes in fp32, the restatement here in float64)."""
    from oracle import ssim_ref

    d = _losses()
    W, H, Fx, Fy, Cx, Cy = d[f"dn_view_{i}"]
    depth = torch.tensor(d[f"dn_depth_{i}"]).double().requires_grad_(True)
    n, valid = ssim_ref.depth_to_normal(depth, Fx, Fy, Cx, Cy)
    (n * torch.tensor(d[f"dn_upstream_{i}"]).double()).sum().backward()
    assert np.array_equal(valid.numpy(), d[f"dn_valid_{i}"])
    assert np.abs(n.detach().numpy() - d[f"dn_normal_{i}"]).max() <= 1e-5
    g = d[f"dn_grad_{i}"].astype(np.float64)
    assert np.linalg.norm(depth.grad.numpy() - g) / np.linalg.norm(g) <= 1e-5
