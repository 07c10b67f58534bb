"""Generate golden fixtures by importing the reference's own Python code.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py
The reference never travels: only the small .npz/.json DATA files written
next to this script are committed (inputs and the reference's outputs).

What is captured (all on CPU; `.cuda()` is monkey-patched to identity and
the CUDA-only / unavailable imports are stubbed — nothing here runs the
reference's CUDA rasterizer, which cannot build in this image):
  sh_eval.npz      utils/sh_utils.py:57-112 eval_sh on random coefficients
  cameras.npz      scene/cameras.py:20-73 Camera matrices built by
                   utils/graphics_utils.py:44-92
  getters.npz      scene/gaussian_model.py:146-262 activations + compute_3D_filter
  boundary.json    DGR/diff_gaussian_rasterization/__init__.py:23-336 — the
                   exact _C argument tuples (order, kinds, dtypes, shapes) and
                   the 12-gradient routing, recorded with a stub `_C`.
  boundary_sample.json  DGR/diff_gaussian_rasterization/__init__.py:470-655 —
                   the same for GaussianRasterizer.sample_depth / _SampleDepth
                   (_C.sample_rasterized_depth{,_backward}).
  boundary_query.json   DGR/diff_gaussian_rasterization/__init__.py:338-468 —
                   the same for GaussianRasterizer.integrate / evaluate_sdf
                   (_C.integrate_gaussians_to_points, _C.evaluate_sdf_from_signle_view).
  losses.npz       utils/loss_utils.py:36-72 create_window / _ssim (the SSIM
                   map the reference defines, captured from inside _ssim; its
                   mean in "same" padding and cropped by 5 for "valid", the
                   mode loss_utils.ssim asks fused_ssim for, :48-49) and
                   utils/graphics_utils.py:103-119 depth_to_normal, with the
                   reference's own fp32 torch autograd gradients (CPU).
  cov3d.npz        scene/gaussian_model.py:46-50 build_covariance_from_scaling_rotation
                   over utils/general_utils.py:77-113 (build_rotation,
                   build_scaling_rotation, strip_symmetric): the 3D covariance
                   of (scale, quaternion, scaling_modifier) — the glm
                   column-major hazard of SURVEY §7 — and its fp32 autograd
                   gradients w.r.t. scale and quaternion for random upstream
                   gradients of the six covariance entries.

    python tests/golden/make_golden.py [fixture ...]   (default: all)
"""
from __future__ import annotations

import importlib
import json
import math
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def _install_stubs():
    _stub("cv2")
    _stub("trimesh")
    _stub("plyfile", PlyData=object, PlyElement=object)
    _stub("simple_knn")
    _stub("simple_knn._C", distCUDA2=lambda *a, **k: None)
    _stub("open3d")
    # import the reference's `scene` as a namespace so scene/__init__.py
    # (dataset readers, open3d) is not executed
    scene = types.ModuleType("scene")
    scene.__path__ = [os.path.join(REF, "scene")]
    sys.modules["scene"] = scene
    sys.path.insert(0, REF)
    torch.Tensor.cuda = lambda self, *a, **k: self  # CPU-only container


def sh_fixture(rng):
    sh_utils = importlib.import_module("utils.sh_utils")
    out = {}
    for deg in range(4):
        n = 64
        sh = rng.standard_normal((n, 3, 16)).astype(np.float32) * 0.5
        d = rng.standard_normal((n, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        res = sh_utils.eval_sh(deg, torch.tensor(sh), torch.tensor(d)).numpy()
        out[f"sh_{deg}"] = sh
        out[f"dirs_{deg}"] = d
        out[f"out_{deg}"] = res
    np.savez(os.path.join(OUT, "sh_eval.npz"), **out)


def camera_fixture(rng):
    cams = importlib.import_module("scene.cameras")
    out = {}
    cases = [(np.eye(3), np.zeros(3), 60.0, 64, 48), (None, None, 45.0, 96, 64), (None, None, 75.0, 40, 40)]
    for i, (R, T, fovx_deg, W, H) in enumerate(cases):
        if R is None:
            a = rng.standard_normal(3)
            a /= np.linalg.norm(a)
            th = rng.uniform(-0.6, 0.6)
            K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
            R = np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K
            T = rng.standard_normal(3) * 0.5
        fovx = math.radians(fovx_deg)
        fovy = 2 * math.atan(math.tan(fovx / 2) * H / W)
        img = torch.zeros(3, H, W)
        cam = cams.Camera(colmap_id=0, R=R, T=T, FoVx=fovx, FoVy=fovy, image=img, gt_alpha_mask=None, gt_mask=None,
                          image_name="x", uid=0, data_device="cpu")
        out[f"R_{i}"] = R
        out[f"T_{i}"] = T
        out[f"fov_{i}"] = np.array([fovx, fovy])
        out[f"wh_{i}"] = np.array([W, H])
        out[f"world_view_{i}"] = cam.world_view_transform.numpy()
        out[f"full_proj_{i}"] = cam.full_proj_transform.numpy()
        out[f"center_{i}"] = cam.camera_center.numpy()
    np.savez(os.path.join(OUT, "cameras.npz"), **out)


def getters_fixture(rng):
    gm = importlib.import_module("scene.gaussian_model")
    P, sh_deg, sg_deg = 64, 3, 2
    g = gm.GaussianModel(sh_deg, sg_deg)
    xyz = rng.standard_normal((P, 3)).astype(np.float32)
    xyz[:, 2] = rng.uniform(1.0, 6.0, P)
    raw = dict(
        xyz=xyz,
        features_dc=rng.standard_normal((P, 1, 3)).astype(np.float32),
        features_rest=rng.standard_normal((P, 15, 3)).astype(np.float32) * 0.1,
        scaling=(rng.standard_normal((P, 3)) * 0.5 + math.log(0.02)).astype(np.float32),
        rotation=rng.standard_normal((P, 4)).astype(np.float32),
        opacity=rng.standard_normal((P, 1)).astype(np.float32),
        sg_axis=rng.standard_normal((P, sg_deg, 3)).astype(np.float32),
        sg_sharpness=rng.standard_normal((P, sg_deg)).astype(np.float32),
        sg_color=rng.standard_normal((P, sg_deg, 3)).astype(np.float32) * 0.1,
    )
    for k, v in raw.items():
        setattr(g, "_" + k, torch.tensor(v))

    class _Cam:  # the attributes compute_3D_filter reads (gaussian_model.py:225-262)
        def __init__(self, R, T, W, H, F):
            self.R, self.T = torch.tensor(R, dtype=torch.float32), torch.tensor(T, dtype=torch.float32)
            self.image_width, self.image_height, self.Fx, self.Fy = W, H, F, F

    cams = [_Cam(np.eye(3), np.zeros(3), 64, 48, 55.0), _Cam(np.eye(3), np.array([0.1, 0.0, 0.5]), 64, 48, 70.0)]
    g.compute_3D_filter(cams)
    filt = g.filter_3D.numpy()
    scales, opac = g.get_scaling_n_opacity_with_3D_filter
    out = {f"raw_{k}": v for k, v in raw.items()}
    out.update(filter_3D=filt, scales=scales.numpy(), opacity=opac.numpy(), rotation_out=g.get_rotation.numpy(),
               features=g.get_features.numpy(), sg_axis_out=g.get_sg_axis.numpy(),
               sg_sharpness_out=g.get_sg_sharpness.numpy(), sg_color_out=g.get_sg_color.numpy(),
               cam_R=np.stack([c.R.numpy() for c in cams]), cam_T=np.stack([c.T.numpy() for c in cams]),
               cam_WHF=np.array([[c.image_width, c.image_height, c.Fx] for c in cams], np.float32))
    np.savez(os.path.join(OUT, "getters.npz"), **out)


def boundary_fixture():
    calls = {}

    def describe(a):
        if isinstance(a, torch.Tensor):
            return {"kind": "tensor", "dtype": str(a.dtype).replace("torch.", ""), "shape": list(a.shape)}
        return {"kind": type(a).__name__, "value": a if isinstance(a, (int, float, bool)) else None}

    P, H, W, SHM, SGM = 5, 8, 12, 16, 2

    def rasterize_gaussians(*args):
        calls["forward"] = [describe(a) for a in args]
        color = torch.full((3, H, W), 1.0)
        alpha = torch.full((1, H, W), 2.0)
        normal = torch.full((3, H, W), 3.0)
        mdepth = torch.full((1, H, W), 4.0)
        radii = torch.arange(P, dtype=torch.int32)
        bufs = [torch.zeros(7, dtype=torch.uint8) for _ in range(4)]
        return (17, color, alpha, normal, mdepth, radii, *bufs)

    def rasterize_gaussians_backward(*args):
        calls["backward"] = [describe(a) for a in args]
        calls["backward_num_rendered"] = args[29]
        # tag every returned grad with its C++ position so routing is visible
        shapes = [(P, 3), (P, 3), (P, 1), (P, 3), (P, 6), (P, SHM, 3), (P, SGM, 3), (P, SGM), (P, SGM, 3), (P, 3),
                  (P, 4)]
        return tuple(torch.full(s, float(i + 1)) for i, s in enumerate(shapes))

    def mark_visible(*args):
        calls["mark_visible"] = [describe(a) for a in args]
        return torch.ones(P, dtype=torch.bool)

    scalls = {}
    PTS = (4, 6, 3)

    def sample_rasterized_depth(*args):
        scalls["forward"] = [describe(a) for a in args]
        out = torch.full(PTS, 5.0)
        inside = torch.ones(PTS[:-1], dtype=torch.bool)
        bufs = [torch.zeros(3, dtype=torch.uint8) for _ in range(6)]
        return (11, 7, 3, out, inside, *bufs)

    def sample_rasterized_depth_backward(*args):
        scalls["backward"] = [describe(a) for a in args]
        scalls["backward_counts"] = [args[23], args[24], args[25]]
        shapes = [(P, 1), (P, 3), (P, 6), (P, 3), (P, 4), PTS]
        return tuple(torch.full(s, float(i + 1)) for i, s in enumerate(shapes))

    qcalls = {}
    QN = 9

    def integrate_gaussians_to_points(*args):
        qcalls["integrate"] = [describe(a) for a in args]
        return (13, torch.full((QN,), 0.25), torch.ones(QN, dtype=torch.bool))

    def evaluate_sdf_from_signle_view(*args):
        qcalls["evaluate_sdf"] = [describe(a) for a in args]
        return (13, torch.full((QN,), 2.5), torch.full((QN,), -0.5), torch.ones(QN, dtype=torch.bool))

    _stub("diff_gaussian_rasterization._C", rasterize_gaussians=rasterize_gaussians,
          rasterize_gaussians_backward=rasterize_gaussians_backward, mark_visible=mark_visible,
          sample_rasterized_depth=sample_rasterized_depth,
          sample_rasterized_depth_backward=sample_rasterized_depth_backward,
          integrate_gaussians_to_points=integrate_gaussians_to_points,
          evaluate_sdf_from_signle_view=evaluate_sdf_from_signle_view)
    pkg = types.ModuleType("diff_gaussian_rasterization")
    pkg.__path__ = [os.path.join(REF, "submodules/diff-gaussian-rasterization/diff_gaussian_rasterization")]
    sys.modules["diff_gaussian_rasterization"] = pkg
    spec = importlib.util.spec_from_file_location(
        "diff_gaussian_rasterization",
        os.path.join(REF, "submodules/diff-gaussian-rasterization/diff_gaussian_rasterization/__init__.py"),
        submodule_search_locations=pkg.__path__)
    dgr = importlib.util.module_from_spec(spec)
    sys.modules["diff_gaussian_rasterization"] = dgr
    spec.loader.exec_module(dgr)
    settings = dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=0.5, tanfovy=0.4, kernel_size=0.1, bg=torch.zeros(3),
        scale_modifier=1.0, viewmatrix=torch.eye(4), projmatrix=torch.eye(4), sh_degree=3, sg_degree=1,
        campos=torch.zeros(3), prefiltered=False, require_depth=True, debug=False)
    rz = dgr.GaussianRasterizer(settings)
    inputs = dict(means3D=torch.zeros(P, 3), means2D=torch.zeros(P, 3), opacities=torch.zeros(P, 1),
                  shs=torch.zeros(P, SHM, 3), sg_axis=torch.zeros(P, SGM, 3), sg_sharpness=torch.zeros(P, SGM),
                  sg_color=torch.zeros(P, SGM, 3), scales=torch.zeros(P, 3), rotations=torch.zeros(P, 4))
    for v in inputs.values():
        v.requires_grad_(True)
    outs = rz(**inputs)
    calls["forward_outputs"] = [describe(o) for o in outs]
    calls["forward_output_values"] = [float(o.flatten()[0]) for o in outs]
    loss = sum((o.float() * (i + 1)).sum() for i, o in enumerate(outs) if o.dtype.is_floating_point)
    loss.backward()
    calls["grad_routing"] = {k: (None if v.grad is None else float(v.grad.flatten()[0])) for k, v in inputs.items()}
    rz.markVisible(torch.zeros(P, 3))
    # argument-validation behaviour (DGR/__init__.py:302-308)
    errs = {}
    for name, kw in [("no_colors", dict(shs=None)), ("both_colors", dict(colors_precomp=torch.zeros(P, 3))),
                     ("no_cov", dict(scales=None)), ("both_cov", dict(cov3D_precomp=torch.zeros(P, 6)))]:
        args = dict(inputs)
        args.update(kw)
        try:
            rz(**args)
            errs[name] = None
        except Exception as e:  # noqa: BLE001 - record the reference's behaviour
            errs[name] = type(e).__name__ + ": " + str(e)
    calls["errors"] = errs
    calls["settings_fields"] = list(dgr.GaussianRasterizationSettings._fields)
    with open(os.path.join(OUT, "boundary.json"), "w") as f:
        json.dump(calls, f, indent=1)

    # sample_depth (DGR/__init__.py:470-655)
    sin = dict(points3D=torch.zeros(PTS), means3D=torch.zeros(P, 3), opacities=torch.zeros(P, 1),
               scales=torch.zeros(P, 3), rotations=torch.zeros(P, 4))
    for v in sin.values():
        v.requires_grad_(True)
    depth, inside = rz.sample_depth(**sin)
    scalls["forward_outputs"] = [describe(depth), describe(inside)]
    (depth * 2.0).sum().backward()
    scalls["grad_routing"] = {k: (None if v.grad is None else float(v.grad.flatten()[0])) for k, v in sin.items()}
    errs = {}
    for name, kw in [("no_cov", dict(scales=None)), ("both_cov", dict(cov3D_precomp=torch.zeros(P, 6)))]:
        args = dict(sin)
        args.update(kw)
        try:
            rz.sample_depth(**args)
            errs[name] = None
        except Exception as e:  # noqa: BLE001 - record the reference's behaviour
            errs[name] = type(e).__name__ + ": " + str(e)
    scalls["errors"] = errs
    scalls["settings_kernel_size"] = 0.1
    with open(os.path.join(OUT, "boundary_sample.json"), "w") as f:
        json.dump(scalls, f, indent=1)

    # integrate / evaluate_sdf (DGR/__init__.py:338-468): forward-only queries
    qin = dict(points3D=torch.zeros(QN, 3), means3D=torch.zeros(P, 3), opacities=torch.zeros(P, 1),
               scales=torch.zeros(P, 3), rotations=torch.zeros(P, 4))
    a, ins = rz.integrate(**qin)
    qcalls["integrate_outputs"] = [describe(a), describe(ins), float(a[0])]
    d, s, ins = rz.evaluate_sdf(**qin)
    qcalls["evaluate_sdf_outputs"] = [describe(d), describe(s), describe(ins), float(d[0]), float(s[0])]
    errs = {}
    for fn in ("integrate", "evaluate_sdf"):
        for name, kw in [("no_cov", dict(scales=None)), ("both_cov", dict(cov3D_precomp=torch.zeros(P, 6)))]:
            args = dict(qin)
            args.update(kw)
            try:
                getattr(rz, fn)(**args)
                errs[fn + "_" + name] = None
            except Exception as e:  # noqa: BLE001 - record the reference's behaviour
                errs[fn + "_" + name] = type(e).__name__ + ": " + str(e)
    qcalls["errors"] = errs
    qcalls["settings_kernel_size"] = 0.1
    with open(os.path.join(OUT, "boundary_query.json"), "w") as f:
        json.dump(qcalls, f, indent=1)


def loss_fixture(rng):
    """SSIM and depth->normal from the reference's own functions (fp32 torch, CPU)."""
    scene = sys.modules["scene"]
    scene.GaussianModel, scene.Camera = object, object  # `from scene import GaussianModel, Camera`
    _stub("fused_ssim", fused_ssim=lambda *a, **k: None)
    _stub("warp_patch_ncc")
    _stub("gaussian_renderer", sample_depth=lambda *a, **k: None, render=lambda *a, **k: None)
    lu = importlib.import_module("utils.loss_utils")
    gu = importlib.import_module("utils.graphics_utils")
    out = {}
    for i, (n, c, h, w) in enumerate([(1, 3, 37, 53), (1, 3, 64, 80), (2, 1, 17, 11)]):
        a = rng.random((n, c, h, w)).astype(np.float32)
        b = np.clip(a + 0.1 * rng.standard_normal(a.shape), 0, 1).astype(np.float32)
        maps = []
        real_mean = torch.Tensor.mean

        def capture(self, *args, **kw):  # the first .mean() of _ssim is ssim_map.mean()
            if not maps and not args and not kw:
                maps.append(self)
            return real_mean(self, *args, **kw)

        x = torch.tensor(a, requires_grad=True)
        torch.Tensor.mean = capture
        try:
            same = lu._ssim(x, torch.tensor(b), lu.create_window(11, c), 11, c)
        finally:
            torch.Tensor.mean = real_mean
        (g_same,) = torch.autograd.grad(same, x, retain_graph=True)
        valid = maps[0][:, :, 5:-5, 5:-5].mean()
        (g_valid,) = torch.autograd.grad(valid, x)
        out.update({f"ssim_img1_{i}": a, f"ssim_img2_{i}": b, f"ssim_same_{i}": same.detach().numpy(),
                    f"ssim_same_grad_{i}": g_same.numpy(), f"ssim_valid_{i}": valid.detach().numpy(),
                    f"ssim_valid_grad_{i}": g_valid.numpy()})

    real_arange = torch.arange

    def arange_cpu(*args, **kw):  # depth_to_normal builds its pixel grid on "cuda"
        kw.pop("device", None)
        return real_arange(*args, **kw)

    class _View:
        def __init__(self, W, H):
            self.image_width, self.image_height = W, H
            self.Fx, self.Fy, self.Cx, self.Cy = 0.9 * W, 0.85 * W, W / 2 - 0.5, H / 2 + 0.25

    for i, (W, H) in enumerate([(40, 30), (64, 48)]):
        base = torch.tensor(rng.random((1, 1, H // 8 + 2, W // 8 + 2)).astype(np.float32)) * 3 + 2
        depth = torch.nn.functional.interpolate(base, size=(H, W), mode="bicubic", align_corners=True)[0]
        depth[:, : H // 7, : W // 5] = 0.0  # holes (median depth 0 where undefined)
        depth = depth.contiguous()
        v = _View(W, H)
        d = depth.clone().requires_grad_(True)
        torch.arange = arange_cpu
        try:
            normal, valid = gu.depth_to_normal(v, d)
        finally:
            torch.arange = real_arange
        gn = torch.tensor(rng.standard_normal((3, H, W)).astype(np.float32)) * valid
        (normal * gn).sum().backward()
        out.update({f"dn_depth_{i}": depth.numpy(), f"dn_view_{i}": np.array([W, H, v.Fx, v.Fy, v.Cx, v.Cy]),
                    f"dn_normal_{i}": normal.detach().numpy(), f"dn_valid_{i}": valid.numpy(),
                    f"dn_upstream_{i}": gn.numpy(), f"dn_grad_{i}": d.grad.numpy()})
    np.savez(os.path.join(OUT, "losses.npz"), **out)


def cov3d_fixture(rng):
    gm = importlib.import_module("scene.gaussian_model")
    g = gm.GaussianModel(3, 0)  # setup_functions: covariance_activation (gaussian_model.py:46-55)
    P = 96
    scales = np.exp(rng.standard_normal((P, 3)) * 0.8 + math.log(0.05)).astype(np.float32)
    rot = rng.standard_normal((P, 4)).astype(np.float32)
    rot[:8] = np.eye(4, dtype=np.float32)[np.arange(8) % 4]  # axis-aligned: identity and half-turns
    rot /= np.linalg.norm(rot, axis=1, keepdims=True)
    up = rng.standard_normal((P, 6)).astype(np.float32)
    zeros = torch.zeros  # build_rotation / build_scaling_rotation allocate with device="cuda"

    def cpu_zeros(*a, **k):
        k.pop("device", None)
        return zeros(*a, **k)

    out = dict(scales=scales, rotations=rot, upstream=up)
    torch.zeros = cpu_zeros
    try:
        for tag, mod in (("m1", 1.0), ("m07", 0.7)):
            s = torch.tensor(scales, requires_grad=True)
            q = torch.tensor(rot, requires_grad=True)
            cov = g.covariance_activation(s, mod, q)
            (cov * torch.tensor(up)).sum().backward()
            out.update({f"cov_{tag}": cov.detach().numpy(), f"dscales_{tag}": s.grad.numpy(),
                        f"drotations_{tag}": q.grad.numpy()})
    finally:
        torch.zeros = zeros
    np.savez(os.path.join(OUT, "cov3d.npz"), **out)


def main():
    _install_stubs()
    which = set(sys.argv[1:]) or {"sh", "boundary", "loss", "cov3d"}
    if "sh" in which:  # sh_eval, cameras and getters share one random stream
        rng = np.random.default_rng(1234)
        sh_fixture(rng)
        camera_fixture(rng)
        getters_fixture(rng)
    if "boundary" in which:
        boundary_fixture()
    if "loss" in which:
        loss_fixture(np.random.default_rng(4321))
    if "cov3d" in which:
        cov3d_fixture(np.random.default_rng(2468))
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
