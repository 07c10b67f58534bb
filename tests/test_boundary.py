"""CPU tests of the drop-in boundary (no GPU needed).

* The Python surface marshals exactly the reference's `_C` argument tuples
  (order, kinds, dtypes, shapes), routes the 11 C++ gradients to the same 12
  autograd slots and raises the same errors — pinned by tests/golden/boundary.json,
  recorded from the reference's own diff_gaussian_rasterization/__init__.py.
* libgsr.so loads and exports every function include/gsr.h declares
  (no compute call without a GPU).
* The product fails loudly on CPU tensors (no CPU fallback).
"""
from __future__ import annotations

import ctypes
import json
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "boundary.json")))
GOLD_SAMPLE = json.load(open(os.path.join(ROOT, "tests", "golden", "boundary_sample.json")))
GOLD_QUERY = json.load(open(os.path.join(ROOT, "tests", "golden", "boundary_query.json")))


def _describe(a):
    if isinstance(a, torch.Tensor):
        return {"kind": "tensor", "dtype": str(a.dtype).replace("torch.", ""), "shape": list(a.shape)}
    return {"kind": type(a).__name__, "value": a if isinstance(a, (int, float, bool)) else None}


def test_wrapper_marshals_reference_tuples(monkeypatch):
    import diff_gaussian_rasterization as dgr

    calls = {}
    P, H, W, SHM, SGM = 5, 8, 12, 16, 2

    def fwd(*args):
        calls["forward"] = [_describe(a) for a in args]
        return (17, torch.full((3, H, W), 1.0), torch.full((1, H, W), 2.0), torch.full((3, H, W), 3.0),
                torch.full((1, H, W), 4.0), torch.arange(P, dtype=torch.int32),
                *[torch.zeros(7, dtype=torch.uint8) for _ in range(4)])

    def bwd(*args):
        calls["backward"] = [_describe(a) for a in args]
        calls["backward_num_rendered"] = args[29]
        shapes = [(P, 3), (P, 3), (P, 1), (P, 3), (P, 6), (P, SHM, 3), (P, SGM, 3), (P, SGM), (P, SGM, 3), (P, 3),
                  (P, 4)]
        return tuple(torch.full(s, float(i + 1)) for i, s in enumerate(shapes))

    def mv(*args):
        calls["mark_visible"] = [_describe(a) for a in args]
        return torch.ones(P, dtype=torch.bool)

    monkeypatch.setattr(dgr._C, "rasterize_gaussians", fwd)
    monkeypatch.setattr(dgr._C, "rasterize_gaussians_backward", bwd)
    monkeypatch.setattr(dgr._C, "mark_visible", mv)
    settings = dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=0.5, tanfovy=0.4, kernel_size=0.1, bg=torch.zeros(3),
        scale_modifier=1.0, viewmatrix=torch.eye(4), projmatrix=torch.eye(4), sh_degree=3, sg_degree=1,
        campos=torch.zeros(3), prefiltered=False, require_depth=True, debug=False)
    assert list(settings._fields) == GOLD["settings_fields"]
    rz = dgr.GaussianRasterizer(settings)
    inputs = dict(means3D=torch.zeros(P, 3), means2D=torch.zeros(P, 3), opacities=torch.zeros(P, 1),
                  shs=torch.zeros(P, SHM, 3), sg_axis=torch.zeros(P, SGM, 3), sg_sharpness=torch.zeros(P, SGM),
                  sg_color=torch.zeros(P, SGM, 3), scales=torch.zeros(P, 3), rotations=torch.zeros(P, 4))
    for v in inputs.values():
        v.requires_grad_(True)
    outs = rz(**inputs)
    assert [_describe(o) for o in outs] == GOLD["forward_outputs"]
    assert [float(o.flatten()[0]) for o in outs] == GOLD["forward_output_values"]
    loss = sum((o.float() * (i + 1)).sum() for i, o in enumerate(outs) if o.dtype.is_floating_point)
    loss.backward()
    assert calls["forward"] == GOLD["forward"]
    assert calls["backward"] == GOLD["backward"]
    assert calls["backward_num_rendered"] == GOLD["backward_num_rendered"]
    routing = {k: (None if v.grad is None else float(v.grad.flatten()[0])) for k, v in inputs.items()}
    assert routing == GOLD["grad_routing"]
    rz.markVisible(torch.zeros(P, 3))
    assert calls["mark_visible"] == GOLD["mark_visible"]
    for name, kw in [("no_colors", dict(shs=None)), ("both_colors", dict(colors_precomp=torch.zeros(P, 3))),
                     ("no_cov", dict(scales=None)), ("both_cov", dict(cov3D_precomp=torch.zeros(P, 6)))]:
        args = dict(inputs)
        args.update(kw)
        with pytest.raises(Exception) as ei:
            rz(**args)
        assert type(ei.value).__name__ + ": " + str(ei.value) == GOLD["errors"][name]


def test_sample_depth_marshals_reference_tuples(monkeypatch):
    """GaussianRasterizer.sample_depth / _SampleDepth: the reference's
    _C.sample_rasterized_depth{,_backward} tuples (kernel_size 0.0 forward,
    the settings' value backward), output kinds, gradient routing and errors
    (tests/golden/boundary_sample.json, DGR/__init__.py:470-655)."""
    import diff_gaussian_rasterization as dgr

    calls = {}
    P, H, W = 5, 8, 12
    PTS = (4, 6, 3)

    def fwd(*args):
        calls["forward"] = [_describe(a) for a in args]
        return (11, 7, 3, torch.full(PTS, 5.0), torch.ones(PTS[:-1], dtype=torch.bool),
                *[torch.zeros(3, dtype=torch.uint8) for _ in range(6)])

    def bwd(*args):
        calls["backward"] = [_describe(a) for a in args]
        calls["backward_counts"] = [args[23], args[24], args[25]]
        shapes = [(P, 1), (P, 3), (P, 6), (P, 3), (P, 4), PTS]
        return tuple(torch.full(s, float(i + 1)) for i, s in enumerate(shapes))

    monkeypatch.setattr(dgr._C, "sample_rasterized_depth", fwd)
    monkeypatch.setattr(dgr._C, "sample_rasterized_depth_backward", bwd)
    settings = dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=0.5, tanfovy=0.4, kernel_size=GOLD_SAMPLE["settings_kernel_size"],
        bg=torch.zeros(3), scale_modifier=1.0, viewmatrix=torch.eye(4), projmatrix=torch.eye(4), sh_degree=3,
        sg_degree=1, campos=torch.zeros(3), prefiltered=False, require_depth=True, debug=False)
    rz = dgr.GaussianRasterizer(settings)
    sin = dict(points3D=torch.zeros(PTS), means3D=torch.zeros(P, 3), opacities=torch.zeros(P, 1),
               scales=torch.zeros(P, 3), rotations=torch.zeros(P, 4))
    for v in sin.values():
        v.requires_grad_(True)
    depth, inside = rz.sample_depth(**sin)
    assert [_describe(depth), _describe(inside)] == GOLD_SAMPLE["forward_outputs"]
    (depth * 2.0).sum().backward()
    assert calls["forward"] == GOLD_SAMPLE["forward"]
    assert calls["backward"] == GOLD_SAMPLE["backward"]
    assert calls["backward_counts"] == GOLD_SAMPLE["backward_counts"]
    routing = {k: (None if v.grad is None else float(v.grad.flatten()[0])) for k, v in sin.items()}
    assert routing == GOLD_SAMPLE["grad_routing"]
    for name, kw in [("no_cov", dict(scales=None)), ("both_cov", dict(cov3D_precomp=torch.zeros(P, 6)))]:
        args = dict(sin)
        args.update(kw)
        with pytest.raises(Exception) as ei:
            rz.sample_depth(**args)
        assert type(ei.value).__name__ + ": " + str(ei.value) == GOLD_SAMPLE["errors"][name]


def test_sample_depth_no_cpu_fallback():
    from diff_gaussian_rasterization import _C

    with pytest.raises(RuntimeError, match="HIP device tensor"):
        _C.sample_rasterized_depth(torch.zeros(4, 3), torch.zeros(2, 3), torch.zeros(2, 1), torch.ones(2, 3),
                                   torch.zeros(2, 4), 1.0, torch.Tensor([]), torch.eye(4), torch.eye(4), 0.5, 0.5,
                                   0.0, 8, 8, torch.zeros(3), False, False)
    with pytest.raises(RuntimeError, match="points3D must have shape"):
        _C.sample_rasterized_depth(torch.zeros(4, 2), torch.zeros(2, 3), *([None] * 15))


def test_point_queries_marshal_reference_tuples(monkeypatch):
    """GaussianRasterizer.integrate / evaluate_sdf: the reference's 18-argument
    _C tuples (kernel size 0.0 whatever the settings hold, an empty
    view2gaussian_precomp), the returned values (integrate returns
    1 - transmittance) and the argument errors (tests/golden/boundary_query.json,
    DGR/__init__.py:338-468)."""
    import diff_gaussian_rasterization as dgr

    calls = {}
    P, H, W, QN = 5, 8, 12, 9

    def integ(*args):
        calls["integrate"] = [_describe(a) for a in args]
        return (13, torch.full((QN,), 0.25), torch.ones(QN, dtype=torch.bool))

    def sdf(*args):
        calls["evaluate_sdf"] = [_describe(a) for a in args]
        return (13, torch.full((QN,), 2.5), torch.full((QN,), -0.5), torch.ones(QN, dtype=torch.bool))

    monkeypatch.setattr(dgr._C, "integrate_gaussians_to_points", integ)
    monkeypatch.setattr(dgr._C, "evaluate_sdf_from_signle_view", sdf)
    settings = dgr.GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=0.5, tanfovy=0.4, kernel_size=GOLD_QUERY["settings_kernel_size"],
        bg=torch.zeros(3), scale_modifier=1.0, viewmatrix=torch.eye(4), projmatrix=torch.eye(4), sh_degree=3,
        sg_degree=1, campos=torch.zeros(3), prefiltered=False, require_depth=True, debug=False)
    rz = dgr.GaussianRasterizer(settings)
    qin = dict(points3D=torch.zeros(QN, 3), means3D=torch.zeros(P, 3), opacities=torch.zeros(P, 1),
               scales=torch.zeros(P, 3), rotations=torch.zeros(P, 4))
    a, ins = rz.integrate(**qin)
    assert [_describe(a), _describe(ins), float(a[0])] == GOLD_QUERY["integrate_outputs"]
    d, s, ins = rz.evaluate_sdf(**qin)
    assert [_describe(d), _describe(s), _describe(ins), float(d[0]), float(s[0])] == GOLD_QUERY["evaluate_sdf_outputs"]
    assert calls["integrate"] == GOLD_QUERY["integrate"]
    assert calls["evaluate_sdf"] == GOLD_QUERY["evaluate_sdf"]
    for fn in ("integrate", "evaluate_sdf"):
        for name, kw in [("no_cov", dict(scales=None)), ("both_cov", dict(cov3D_precomp=torch.zeros(P, 6)))]:
            args = dict(qin)
            args.update(kw)
            with pytest.raises(Exception) as ei:
                getattr(rz, fn)(**args)
            assert type(ei.value).__name__ + ": " + str(ei.value) == GOLD_QUERY["errors"][fn + "_" + name]


def test_point_queries_no_cpu_fallback():
    from diff_gaussian_rasterization import _C

    args = (torch.zeros(4, 3), torch.zeros(2, 3), torch.zeros(2, 1), torch.ones(2, 3), torch.zeros(2, 4), 1.0,
            torch.Tensor([]), torch.Tensor([]), torch.eye(4), torch.eye(4), 0.5, 0.5, 0.0, 8, 8, torch.zeros(3),
            False, False)
    for fn in (_C.integrate_gaussians_to_points, _C.evaluate_sdf_from_signle_view):
        with pytest.raises(RuntimeError, match="HIP device tensor"):
            fn(*args)
        with pytest.raises(RuntimeError, match="points3D must have dimensions"):
            fn(torch.zeros(4, 2), *args[1:])


def test_distcuda2_no_cpu_fallback():
    """simple_knn._C.distCUDA2 (scene/gaussian_model.py:20) resolves to gsr
    and refuses CPU tensors."""
    from simple_knn._C import distCUDA2

    with pytest.raises(RuntimeError, match="HIP device tensor"):
        distCUDA2(torch.zeros(8, 3))


def test_library_exports_header_symbols():
    header = open(os.path.join(ROOT, "include", "gsr.h")).read()
    names = sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(gsr_\w+)\s*\(", header, re.M)))
    assert "gsr_rasterize_forward" in names and "gsr_rasterize_backward" in names and "gsr_mark_visible" in names
    from diff_gaussian_rasterization import _C

    lib = ctypes.CDLL(_C.loaded_library_path())
    for n in names:
        assert hasattr(lib, n), n
    lib.gsr_abi_version.restype = ctypes.c_int
    assert lib.gsr_abi_version() == _C.ABI_VERSION == 20
    lib.gsr_stage_name.restype = ctypes.c_char_p
    assert lib.gsr_stage_name(5) == b"render_fwd"


def test_retired_options_are_rejected():
    """Option ids 0, 2-4, 7, 8 (retired variants and diagnostics) and
    out-of-range ids fail loudly instead of being silently ignored (host-only
    call, no GPU); the test-oracle paths remain."""
    from diff_gaussian_rasterization import _C

    for opt in (0, 2, 3, 4, 7, 8, 11, -1):
        with pytest.raises(RuntimeError, match="unknown option"):
            _C.set_option(opt, 1)
    for opt in (_C.OPT_RENDER_STATS, _C.OPT_NO_REFINE, _C.OPT_BWD_NO_CACHE, _C.OPT_ROCPRIM_DSORT, _C.OPT_PBWD_STAGE):
        _C.set_option(opt, 0)


def test_library_targets_gfx950():
    from diff_gaussian_rasterization import _C

    blob = open(_C.loaded_library_path(), "rb").read()
    assert b"gfx950" in blob


def test_no_cpu_fallback():
    from diff_gaussian_rasterization import _C

    P = 4
    t = torch.zeros(P, 3)
    with pytest.raises(RuntimeError, match="HIP device tensor"):
        _C.rasterize_gaussians(torch.zeros(3), t, torch.Tensor([]), torch.zeros(P, 1), torch.ones(P, 3),
                               torch.zeros(P, 4), torch.Tensor([]), torch.zeros(P, 16, 3), torch.zeros(P, 0, 3),
                               torch.zeros(P, 0), torch.zeros(P, 0, 3), 3, 0, 1.0, torch.eye(4), torch.eye(4), 0.5,
                               0.5, 0.0, 8, 8, torch.zeros(3), False, True, False)
    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        _C.rasterize_gaussians(torch.zeros(3), torch.zeros(P, 2), *([None] * 23))


def test_empty_scene_matches_reference_semantics():
    """P == 0 returns zero images and num_rendered 0 without touching the GPU
    (rasterize_points.cu:77-95)."""
    from diff_gaussian_rasterization import _C

    out = _C.rasterize_gaussians(torch.zeros(3), torch.zeros(0, 3), torch.Tensor([]), torch.zeros(0, 1),
                                 torch.zeros(0, 3), torch.zeros(0, 4), torch.Tensor([]), torch.zeros(0, 16, 3),
                                 torch.zeros(0, 0, 3), torch.zeros(0, 0), torch.zeros(0, 0, 3), 3, 0, 1.0,
                                 torch.eye(4), torch.eye(4), 0.5, 0.5, 0.0, 6, 10, torch.zeros(3), False, True, False)
    assert out[0] == 0
    assert out[1].shape == (3, 6, 10) and float(out[1].abs().sum()) == 0.0
    assert out[5].shape == (0,)
