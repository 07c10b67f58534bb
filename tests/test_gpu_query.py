"""GPU parity tests for the point queries of the offline mesh extraction
(SURVEY §8(f) rank 4): integrate and evaluate_sdf through
`_C.integrate_gaussians_to_points` / `_C.evaluate_sdf_from_signle_view`
(libgsr.so, render_fwd.hip in SAMPLE mode) against the C oracle's
restatement of sample_forward.cu:55-427 on identical seeded inputs.

Tolerances (north star: 1e-4 relative):
  * integer outputs (num_rendered, inside flags): exact;
  * integrate transmittance (in [0, 1]): max|a-b| <= 1e-4 (products of up to
    a few hundred factors, each carrying v_exp / v_rsq rounding);
  * evaluate_sdf depth: max|a-b| / max|b| <= 1e-4; sdf: max|a-b| <= 1e-4 max|depth|.
At full size (1M Gaussians, 1080p, the tetra points of every Gaussian, the
call of mesh_extract_tetrahedra.py:75): determinism, and exact agreement of a
20k-point subsample with the oracle run on those points alone (a point's
result does not depend on the other points).
"""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

import gsr_scene as S
import helpers as Hh
from oracle import gsr_oracle as O
from test_oracle import query_args, sample_points

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _gpu(x):
    if isinstance(x, torch.Tensor):
        return x.to(DEV)
    return torch.Tensor([]) if x is None else x


def _check(c, pts, cov3D=None):
    from diff_gaussian_rasterization import _C

    a = query_args(c, pts, cov3D)
    ga = [_gpu(x) for x in a]
    K, T, inside = O.integrate(*a)
    gK, gT, gin = _C.integrate_gaussians_to_points(*ga)
    assert gK == K
    assert np.array_equal(gin.cpu().numpy(), inside)
    margins = {"integrate 1 - T (absolute)": (float(np.abs(gT.cpu().numpy() - T).max()), 1e-4)}
    assert np.abs(gT.cpu().numpy() - T).max() <= 1e-4, np.abs(gT.cpu().numpy() - T).max()
    assert 0.0 < T[inside].mean() < 1.0
    K, depth, sdf, inside = O.evaluate_sdf(*a)
    gK, gd, gs, gin = _C.evaluate_sdf_from_signle_view(*ga)
    assert gK == K
    assert np.array_equal(gin.cpu().numpy(), inside)
    assert inside.sum() > 0
    margins["evaluate_sdf depth / max"] = (Hh.rel_err(gd.cpu().numpy(), depth), 1e-4)
    margins["evaluate_sdf sdf / max depth"] = (float(np.abs(gs.cpu().numpy() - sdf).max() / np.abs(depth).max()), 1e-4)
    Hh.record_margins(margins, "point queries vs oracle")
    assert Hh.rel_err(gd.cpu().numpy(), depth) <= 1e-4, Hh.rel_err(gd.cpu().numpy(), depth)
    assert np.abs(gs.cpu().numpy() - sdf).max() <= 1e-4 * np.abs(depth).max()


CASES = [
    dict(P=150, W=40, H=32, seed=0, n=400),
    dict(P=600, W=96, H=64, seed=1, n=3000),
    dict(P=2000, W=160, H=96, seed=2, n=20000, log_scale=math.log(0.05)),
    dict(P=300, W=61, H=53, seed=3, n=2500),  # ragged tiles at the image border
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_query_parity(case):
    case = dict(case)
    n = case.pop("n")
    c = Hh.small_case(**case)
    _check(c, sample_points(c, n, case["seed"] + 200))


def test_query_parity_cov3D_precomp():
    c = Hh.small_case(P=400, W=64, H=48, seed=6)
    s = c["inp"]["scales"].double()
    q = c["inp"]["rotations"].double()
    r, x, y, z = q.unbind(1)
    Rm = torch.stack([torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], 1),
                      torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], 1),
                      torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1)], 1)
    Sig = Rm @ torch.diag_embed(s * s) @ Rm.transpose(1, 2)
    cov = torch.stack([Sig[:, 0, 0], Sig[:, 0, 1], Sig[:, 0, 2], Sig[:, 1, 1], Sig[:, 1, 2], Sig[:, 2, 2]], 1)
    _check(c, sample_points(c, 2000, 8), cov3D=cov.float().contiguous())


def test_query_points_on_tile_borders():
    """Points within half a pixel of tile borders (the tile lists are culled
    over [16 t - 0.5, 16 t + 15.5], where the points of a tile live)."""
    c = Hh.small_case(P=800, W=96, H=64, seed=9, log_scale=math.log(0.05))
    g = torch.Generator().manual_seed(4)
    n = 4000
    W, H = c["W"], c["H"]
    px = torch.randint(1, W // 16, (n,), generator=g) * 16.0 + (torch.rand(n, generator=g) - 0.5) * 0.999 - 0.5
    py = torch.randint(1, H // 16, (n,), generator=g) * 16.0 + (torch.rand(n, generator=g) - 0.5) * 0.999 - 0.5
    z = torch.rand(n, generator=g) * 2.5 + 1.5
    fx, fy = W / (2 * c["tanx"]), H / (2 * c["tany"])
    cam_pts = torch.stack([(px - (W - 1) / 2) / fx * z, (py - (H - 1) / 2) / fy * z, z], 1)
    V = c["cam"].world_view_transform
    _check(c, ((cam_pts - V[3, :3]) @ torch.linalg.inv(V[:3, :3])).float().contiguous())


def test_query_wide_grid_sort_path():
    """> 1024 tiles across: the Gaussian lists come from binning.hip's sort path."""
    c = Hh.small_case(P=600, W=16400, H=40, seed=10, log_scale=math.log(0.01))
    _check(c, sample_points(c, 5000, 11))


def test_query_degenerate():
    from diff_gaussian_rasterization import _C

    c = Hh.small_case(P=100, W=40, H=32, seed=12)
    pts = torch.tensor([[0.0, 0.0, -5.0], [100.0, 0.0, 3.0]])  # behind the camera / outside the image
    K, T, inside = _C.integrate_gaussians_to_points(*[_gpu(x) for x in query_args(c, pts)])
    assert float(T.abs().max()) == 0 and not bool(inside.any())
    K, d, s, inside = _C.evaluate_sdf_from_signle_view(*[_gpu(x) for x in query_args(c, pts)])
    assert float(d.abs().max()) == 0 and float(s.abs().max()) == 0 and not bool(inside.any())
    empty = torch.zeros(0, 3)
    K, T, inside = _C.integrate_gaussians_to_points(*[_gpu(x) for x in query_args(c, empty)])
    assert K == 0 and T.shape == (0,) and inside.shape == (0,)
    with pytest.raises(RuntimeError, match="points3D must have dimensions"):
        _C.evaluate_sdf_from_signle_view(*[_gpu(x) for x in query_args(c, torch.zeros(4, 2))])


class _Pipe:
    debug = False
    compute_cov3D_python = False


class _Model:
    """The GaussianModel getters the reference's integrate / evaluate_sdf read
    (gaussian_renderer/__init__.py:131-143)."""

    def __init__(self, inp):
        self.get_xyz = inp["means3D"]
        self.get_opacity_with_3D_filter = inp["opacities"]
        self.get_scaling_with_3D_filter = inp["scales"]
        self.get_rotation = inp["rotations"]
        self.active_sh_degree = 3
        self.active_sg_degree = 0


def test_renderer_integrate_and_evaluate_sdf():
    """gaussian_renderer.integrate / evaluate_sdf (gaussian_renderer/__init__.py:
    101-222): the reference's returned dicts, alpha_integrated = 1 - T."""
    import gaussian_renderer as GR

    c = Hh.small_case(P=600, W=96, H=64, seed=13)
    pts = sample_points(c, 3000, 14)
    K, T, inside = O.integrate(*query_args(c, pts))
    _, depth, sdf, sin = O.evaluate_sdf(*query_args(c, pts))
    cam = c["cam"].to(DEV)
    pc = _Model({k: v.to(DEV) for k, v in c["inp"].items()})
    r = GR.integrate(pts.to(DEV), cam, pc, _Pipe(), kernel_size=0.1)
    assert set(r) == {"alpha_integrated", "inside"}
    assert np.array_equal(r["inside"].cpu().numpy(), inside)
    assert np.abs(r["alpha_integrated"].cpu().numpy() - (1 - T)).max() <= 1e-4
    r = GR.evaluate_sdf(pts.to(DEV), cam, pc, _Pipe(), kernel_size=0.1)
    assert set(r) == {"depth", "sdf", "inside"}
    assert np.array_equal(r["inside"].cpu().numpy(), sin)
    assert Hh.rel_err(r["depth"].cpu().numpy(), depth) <= 1e-4


def test_query_full_size():
    """1M Gaussians (C3 scene), 1080p, the 15M tetra points: deterministic,
    and a 20k-point subsample equals the oracle on those points alone."""
    from diff_gaussian_rasterization import _C

    W, H, P = 1920, 1080, 1_000_000
    cam = S.make_camera(W, H)
    inp = {k: v.contiguous() for k, v in S.activated_inputs(S.make_gaussians(P, aspect=H / W)).items()}
    c = dict(inp=inp, cam=cam, W=W, H=H, tanx=math.tan(cam.FoVx * 0.5), tany=math.tan(cam.FoVy * 0.5))
    gin = {k: v.to(DEV) for k, v in inp.items()}
    pts = S.tetra_points(gin)
    ga = [_gpu(x) for x in query_args(dict(c, inp=gin), pts)]
    K1, T1, in1 = _C.integrate_gaussians_to_points(*ga)
    K2, T2, in2 = _C.integrate_gaussians_to_points(*ga)
    assert K1 == K2 and torch.equal(T1, T2) and torch.equal(in1, in2)
    assert float(in1.float().mean()) > 0.5
    Ks, d1, s1, sin1 = _C.evaluate_sdf_from_signle_view(*ga)
    _, d2, s2, sin2 = _C.evaluate_sdf_from_signle_view(*ga)
    assert torch.equal(d1, d2) and torch.equal(s1, s2) and torch.equal(sin1, sin2)
    sub = torch.randperm(pts.shape[0], generator=torch.Generator().manual_seed(0))[:20000]
    psub = pts[sub.to(DEV)].cpu()
    K, T, inside = O.integrate(*query_args(c, psub))
    assert K == K1
    assert np.array_equal(in1[sub.to(DEV)].cpu().numpy(), inside)
    assert np.abs(T1[sub.to(DEV)].cpu().numpy() - T).max() <= 1e-4
    K, depth, sdf, sinside = O.evaluate_sdf(*query_args(c, psub))
    mine = sin1[sub.to(DEV)].cpu().numpy()
    assert (mine != sinside).mean() <= 1e-3  # a bracket decision within float noise of T = 1/2 may flip
    both = mine & sinside
    assert both.sum() > 1000
    dm = d1[sub.to(DEV)].cpu().numpy()
    bad = np.abs(dm - depth)[both] > 1e-4 * np.abs(depth).max()
    assert bad.mean() <= 1e-3, bad.mean()
