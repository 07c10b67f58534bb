"""GPU parity tests for sample_depth: the HIP path
(libgsr.so through `_C.sample_rasterized_depth{,_backward}` and
GaussianRasterizer.sample_depth) against the C oracle's restatement of
sample_forward.cu / sample_backward.cu on identical seeded inputs.

Tolerances (north star: 1e-4 relative):
  * integer outputs (num_rendered, num_points, the reference's block count,
    inside flags): exact;
  * sampled points: max|a-b| / max|b| <= 1e-4;
  * gradients: ||a-b|| / ||b|| <= 1e-4 and max|a-b| / max|b| <= 1e-3 (float
    atomics on the GPU, double sums in the oracle).
At full size (1M Gaussians, 1080p, one point per pixel of a second view, the
training call pattern of utils/loss_utils.py:147-166): determinism, exact
counts against the oracle, point parity on a sample, backward linearity.
"""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

import gsr_scene as S
import helpers as Hh
from oracle import gsr_oracle as O
from test_oracle import sample_args, sample_points

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
GRADS = ["dopacity", "dmeans3D", "dcov3D", "dscales", "drotations", "dpoints3D"]


def _gpu(x):
    if isinstance(x, torch.Tensor):
        return x.to(DEV)
    return torch.Tensor([]) if x is None else x


def _run(c, pts, kernel_size=0.0, bwd_kernel_size=None, cov3D=None, check_bwd=True, strict=True):
    from diff_gaussian_rasterization import _C

    a = list(sample_args(c, pts, kernel_size))
    if cov3D is not None:
        a[3], a[4], a[6] = None, None, cov3D
    o = O.sample_forward(*a)
    ga = [_gpu(x) for x in a] + [False]
    out = _C.sample_rasterized_depth(*ga)
    K, RN, TN, output, inside = out[:5]
    assert (K, RN, TN) == (o["num_rendered"], o["num_points"], o["num_duplicated_tiles"])
    ins = inside.cpu().numpy()
    if strict:
        assert np.array_equal(ins, o["inside"])
        assert Hh.rel_err(output.cpu().numpy(), o["output"]) <= 1e-4
    else:
        assert (ins != o["inside"]).mean() <= 1e-4
        bad = np.abs(output.cpu().numpy() - o["output"]) > 1e-4 * np.abs(o["output"]).max()
        assert bad.mean() <= 1e-4
    if not check_bwd:
        return out, o
    bks = kernel_size if bwd_kernel_size is None else bwd_kernel_size
    g = torch.randn(pts.shape, generator=torch.Generator().manual_seed(3)) * 1e-2
    # the backward reads the forward's per-point median depth; feed the GPU's
    # to the oracle so the comparison isolates the backward (the implicit
    # gradient is steep in it near thin Gaussians)
    md, _ = _C.debug_sample_points(out[7], pts.numel() // 3)
    o["state"].set_median_depth(md)
    b = O.sample_backward(o["state"], *a[:9], o["inside"], g, c["tanx"], c["tany"], bks)
    gb = _C.sample_rasterized_depth_backward(*ga[:9], inside, _gpu(g), c["tanx"], c["tany"], bks, c["H"], c["W"],
                                             _gpu(c["cam"].camera_center), *out[5:11], K, RN, TN, False, False)
    margins = {}
    try:
        for name, t in zip(GRADS, gb):
            mine, ref = t.cpu().numpy().astype(np.float64), b[name]
            assert mine.shape == ref.shape, name
            if not np.any(ref):
                assert not np.any(mine), name
                continue
            l2 = np.linalg.norm(mine - ref) / np.linalg.norm(ref)
            margins[f"{name} L2"] = (l2, 1e-4)
            margins[f"{name} max"] = (Hh.rel_err(mine, ref), 1e-3)
            assert l2 <= 1e-4, (name, l2)
            assert Hh.rel_err(mine, ref) <= 1e-3, (name, Hh.rel_err(mine, ref))
    finally:
        Hh.record_margins(margins, "sample_depth gradients vs oracle backward")
    return out, o


CASES = [
    dict(P=150, W=40, H=32, seed=0, n=400),
    dict(P=600, W=96, H=64, seed=1, n=3000),
    dict(P=2000, W=160, H=96, seed=2, n=20000, log_scale=math.log(0.05)),
    dict(P=300, W=61, H=53, seed=3, n=2500),  # ragged tiles at the image border
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_sample_parity(case):
    case = dict(case)
    n = case.pop("n")
    c = Hh.small_case(**case)
    pts = sample_points(c, n, case["seed"] + 100)
    _run(c, pts)


def test_sample_scratch_split_is_exact(monkeypatch):
    """gsr_sample_depth_forward_ex (the binding's forward) with its
    forward-only scratch outside the saved buffers against
    gsr_sample_depth_forward's layout (a NULL scratch allocator): the same
    points, flags and counts bit for bit, the same gradients to the atomics'
    summation order, and smaller geometry / binning buffers."""
    from diff_gaussian_rasterization import _C

    c = Hh.small_case(P=2000, W=160, H=96, seed=2, log_scale=math.log(0.05))
    pts = sample_points(c, 20000, 102)
    ga = [_gpu(x) for x in sample_args(c, pts)] + [False]
    g = _gpu(torch.randn(pts.shape, generator=torch.Generator().manual_seed(3)) * 1e-2)

    def run():
        out = _C.sample_rasterized_depth(*ga)
        K, RN, TN, _, inside = out[:5]
        gb = _C.sample_rasterized_depth_backward(*ga[:9], inside, g, c["tanx"], c["tany"], 0.0, c["H"], c["W"],
                                                 _gpu(c["cam"].camera_center), *out[5:11], K, RN, TN, False, False)
        return out, gb

    split = run()

    class _NoScratch:  # a NULL scratch allocator: gsr_sample_depth_forward's layout
        def __init__(self, _dev):
            self.cb = _C._ALLOC()

    monkeypatch.setattr(_C, "_ScratchBlocks", _NoScratch)
    whole = run()
    assert split[0][:3] == whole[0][:3]
    assert torch.equal(split[0][3], whole[0][3]) and torch.equal(split[0][4], whole[0][4])
    for name, a, b in zip(GRADS, split[1], whole[1]):
        if b.numel():
            assert float((a - b).abs().max()) <= 1e-5 * max(float(b.abs().max()), 1e-30), name
    assert split[0][5].numel() < whole[0][5].numel()  # geometry buffer
    assert split[0][6].numel() < whole[0][6].numel()  # binning buffer


def test_sample_parity_batched_shape_and_kernel_size():
    """points3D of shape [H, W, 3] (the training call); forward with kernel
    size 0.0 and backward with the settings' 0.1, as the reference wrapper
    passes them (DGR/__init__.py:500-518, 598)."""
    c = Hh.small_case(P=600, W=96, H=64, seed=5)
    pts = sample_points(c, 64 * 96, 7).reshape(64, 96, 3)
    _run(c, pts, kernel_size=0.0, bwd_kernel_size=0.1)


def test_sample_parity_cov3D_precomp():
    c = Hh.small_case(P=400, W=64, H=48, seed=6)
    s = c["inp"]["scales"].double()
    q = c["inp"]["rotations"].double()
    r, x, y, z = q.unbind(1)
    Rm = torch.stack([torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], 1),
                      torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], 1),
                      torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1)], 1)
    Sig = Rm @ torch.diag_embed(s * s) @ Rm.transpose(1, 2)
    cov = torch.stack([Sig[:, 0, 0], Sig[:, 0, 1], Sig[:, 0, 2], Sig[:, 1, 1], Sig[:, 1, 2], Sig[:, 2, 2]], 1)
    _run(c, sample_points(c, 2000, 8), cov3D=cov.float().contiguous())


def test_sample_points_on_tile_borders():
    """Points within half a pixel of tile borders: the tile lists are culled
    over [16 t - 0.5, 16 t + 15.5] (tiles.h pad), where the points of a tile
    live (createWithKeys, rasterizer_impl.cu:129-130)."""
    c = Hh.small_case(P=800, W=96, H=64, seed=9, log_scale=math.log(0.05))
    g = torch.Generator().manual_seed(4)
    n = 4000
    W, H = c["W"], c["H"]
    bx = torch.randint(1, W // 16, (n,), generator=g) * 16.0 + (torch.rand(n, generator=g) - 0.5) * 0.999 - 0.5
    by = torch.rand(n, generator=g) * (H - 1)
    swap = torch.rand(n, generator=g) < 0.5
    px = torch.where(swap, torch.rand(n, generator=g) * (W - 1), bx)
    py = torch.where(swap, torch.randint(1, H // 16, (n,), generator=g) * 16.0
                     + (torch.rand(n, generator=g) - 0.5) * 0.999 - 0.5, by)
    z = torch.rand(n, generator=g) * 2.5 + 1.5
    fx, fy = W / (2 * c["tanx"]), H / (2 * c["tany"])
    cam_pts = torch.stack([(px - (W - 1) / 2) / fx * z, (py - (H - 1) / 2) / fy * z, z], 1)
    V = c["cam"].world_view_transform
    pts = ((cam_pts - V[3, :3]) @ torch.linalg.inv(V[:3, :3])).float().contiguous()
    _run(c, pts)


def test_sample_points_crowded_tiles():
    """Most points in two tiles (several 256-point chunks each, whole waves of
    one tile: the scatter's per-wave runs), culled points interleaved (behind
    the camera: key = tiles, in no range) and a point count that is not a
    multiple of 256: the grouping is order-free, every point's result and the
    gradients as the oracle's."""
    c = Hh.small_case(P=800, W=96, H=64, seed=9, log_scale=math.log(0.05))
    g = torch.Generator().manual_seed(21)
    n = 3333
    W, H = c["W"], c["H"]
    tile_x = torch.where(torch.rand(n, generator=g) < 0.5, 1.0, 3.0)
    px = tile_x * 16.0 + torch.rand(n, generator=g) * 15.0
    py = 16.0 + torch.rand(n, generator=g) * 15.0
    z = torch.rand(n, generator=g) * 2.5 + 1.5
    z = torch.where(torch.rand(n, generator=g) < 0.1, -z, z)  # (behind the camera: culled)
    fx, fy = W / (2 * c["tanx"]), H / (2 * c["tany"])
    cam_pts = torch.stack([(px - (W - 1) / 2) / fx * z.abs(), (py - (H - 1) / 2) / fy * z.abs(), z], 1)
    V = c["cam"].world_view_transform
    pts = ((cam_pts - V[3, :3]) @ torch.linalg.inv(V[:3, :3])).float().contiguous()
    out, o = _run(c, pts)
    assert 0 < o["num_points"] < n


def test_sample_tile_borders_ragged_grid():
    """The sample pad at tile borders, and a ragged grid."""
    c = Hh.small_case(P=800, W=96, H=64, seed=9, log_scale=math.log(0.05))
    _run(c, sample_points(c, 4000, 12))
    c = Hh.small_case(P=300, W=61, H=53, seed=3)
    _run(c, sample_points(c, 2500, 103))


def test_sample_wide_grid_sort_path():
    """> 1024 tiles across: the Gaussian lists come from binning.hip's sort path."""
    c = Hh.small_case(P=600, W=16400, H=40, seed=10, log_scale=math.log(0.01))
    _run(c, sample_points(c, 5000, 11))


def test_sample_degenerate():
    from diff_gaussian_rasterization import _C

    c = Hh.small_case(P=100, W=40, H=32, seed=12)
    # no point in view: everything culled, zero outputs
    pts = torch.tensor([[0.0, 0.0, -5.0], [100.0, 0.0, 3.0]])
    out = _C.sample_rasterized_depth(*[_gpu(x) for x in sample_args(c, pts)], False)
    assert out[1] == 0 and out[2] == 0
    assert float(out[3].abs().max()) == 0 and not bool(out[4].any())
    # no points at all
    pts = torch.zeros(0, 3)
    out = _C.sample_rasterized_depth(*[_gpu(x) for x in sample_args(c, pts)], False)
    assert out[0] == 0 and out[3].shape == (0, 3) and out[4].shape == (0,)
    with pytest.raises(RuntimeError):
        _C.sample_rasterized_depth(*[_gpu(x) for x in sample_args(c, torch.zeros(4, 2))], False)


def test_sample_depth_autograd_matches_direct_call():
    """GaussianRasterizer.sample_depth -> _SampleDepth: same values and the
    gradient routing of DGR/__init__.py:640-655 (points3D, means3D,
    opacities, scales, rotations)."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

    c = Hh.small_case(P=600, W=96, H=64, seed=13)
    pts = sample_points(c, 3000, 14)
    o = O.sample_forward(*sample_args(c, pts))
    cam = c["cam"].to(DEV)
    settings = GaussianRasterizationSettings(
        image_height=c["H"], image_width=c["W"], tanfovx=c["tanx"], tanfovy=c["tany"], kernel_size=0.0, bg=0,
        scale_modifier=1.0, viewmatrix=cam.world_view_transform, projmatrix=cam.full_proj_transform, sh_degree=3,
        sg_degree=0, campos=cam.camera_center, prefiltered=False, require_depth=True, debug=False)
    leaves = {k: v.to(DEV).requires_grad_(True) for k, v in dict(
        points3D=pts, means3D=c["inp"]["means3D"], opacities=c["inp"]["opacities"], scales=c["inp"]["scales"],
        rotations=c["inp"]["rotations"]).items()}
    depth, inside = GaussianRasterizer(settings).sample_depth(**leaves)
    assert Hh.rel_err(depth.detach().cpu().numpy(), o["output"]) <= 1e-4
    assert np.array_equal(inside.cpu().numpy(), o["inside"])
    g = torch.randn(pts.shape, generator=torch.Generator().manual_seed(3)) * 1e-2
    (depth * g.to(DEV)).sum().backward()
    # the forward is deterministic: a direct call yields the median depths the
    # autograd ctx's point buffer holds; the oracle backward uses them
    from diff_gaussian_rasterization import _C

    direct = _C.sample_rasterized_depth(*[_gpu(x) for x in sample_args(c, pts)], False)
    assert torch.equal(direct[3], depth.detach())
    o["state"].set_median_depth(_C.debug_sample_points(direct[7], pts.shape[0])[0])
    b = O.sample_backward(o["state"], *sample_args(c, pts)[:9], o["inside"], g, c["tanx"], c["tany"], 0.0)
    for name, key in (("points3D", "dpoints3D"), ("means3D", "dmeans3D"), ("opacities", "dopacity"),
                      ("scales", "dscales"), ("rotations", "drotations")):
        mine = leaves[name].grad.cpu().numpy().astype(np.float64)
        assert np.linalg.norm(mine - b[key]) <= 1e-4 * np.linalg.norm(b[key]), name


def test_sample_depth_at_pixel_centres_equals_render():
    """GPU consistency of the two rasters: a point on a pixel's ray samples
    the median depth render_fwd computed for that pixel."""
    from diff_gaussian_rasterization import _C

    c = Hh.small_case(P=3000, W=160, H=96, seed=15, log_scale=math.log(0.05))
    fo = _C.rasterize_gaussians(*[_gpu(x) for x in Hh.oracle_args(c)], False)
    md = fo[4][0].cpu().numpy()
    md_in = np.zeros_like(md)
    md_in[1:-1, 1:-1] = md[1:-1, 1:-1]
    ys, xs = np.nonzero(md_in > 0)
    W, H = c["W"], c["H"]
    fx, fy = W / (2 * c["tanx"]), H / (2 * c["tany"])
    z = torch.tensor(md[ys, xs])
    cam_pts = torch.stack([(torch.tensor(xs, dtype=torch.float32) - (W - 1) / 2) / fx * z,
                           (torch.tensor(ys, dtype=torch.float32) - (H - 1) / 2) / fy * z, z], 1)
    V = c["cam"].world_view_transform
    pts = ((cam_pts - V[3, :3]) @ torch.linalg.inv(V[:3, :3])).float().contiguous()
    out = _C.sample_rasterized_depth(*[_gpu(x) for x in sample_args(c, pts)], False)
    zs = out[3][:, 2].cpu().numpy()
    close = np.abs(zs - md[ys, xs]) <= 1e-4 * np.abs(md).max()
    assert close.mean() > 0.995, close.mean()


# ------------------------------------------------------------- full size
def test_sample_full_size():
    """1M Gaussians, 1080p; the points are the C3 view's median-depth points
    re-observed by an orbit camera (the multi-view loss's call)."""
    from diff_gaussian_rasterization import _C

    W, H, P = 1920, 1080, 1_000_000
    cam0 = S.make_camera(W, H)
    raw = S.make_gaussians(P, aspect=H / W)
    inp = {k: v.detach().contiguous() for k, v in S.activated_inputs(raw).items()}
    c0 = dict(bg=torch.zeros(3), inp=inp, cam=cam0, W=W, H=H, sh_degree=3, sg_degree=0, kernel_size=0.0,
              require_depth=True, tanx=math.tan(cam0.FoVx / 2), tany=math.tan(cam0.FoVy / 2))
    fo = _C.rasterize_gaussians(*[_gpu(x) for x in Hh.oracle_args(c0)], False)
    md = fo[4][0]
    fx, fy = W / (2 * c0["tanx"]), H / (2 * c0["tany"])
    ys, xs = torch.meshgrid(torch.arange(H, device=DEV, dtype=torch.float32),
                            torch.arange(W, device=DEV, dtype=torch.float32), indexing="ij")
    pts = torch.stack([(xs - (W - 1) / 2) / fx * md, (ys - (H - 1) / 2) / fy * md, md], -1)  # [H, W, 3], camera 0 = world
    cam1 = S.orbit_cameras(8, W, H)[1]
    c1 = dict(c0, cam=cam1)
    a = [_gpu(x) for x in sample_args(c1, pts.cpu())] + [False]
    out1 = _C.sample_rasterized_depth(*a)
    out2 = _C.sample_rasterized_depth(*a)
    assert torch.equal(out1[3], out2[3]) and torch.equal(out1[4], out2[4])
    O.set_threads(16)
    o = O.sample_forward(*sample_args(c1, pts.cpu()))
    assert (out1[0], out1[1], out1[2]) == (o["num_rendered"], o["num_points"], o["num_duplicated_tiles"])
    assert out1[1] > 1_000_000 and int(out1[4].sum()) > 500_000
    ins = out1[4].cpu().numpy()
    assert (ins != o["inside"]).mean() <= 1e-4
    got = out1[3].cpu().numpy()
    bad = np.abs(got - o["output"]) > 1e-4 * np.abs(o["output"]).max()
    Hh.record_margins({"inside flips (fraction)": (float((ins != o["inside"]).mean()), 1e-4),
                       "points beyond 1e-4 of max (fraction)": (float(bad.mean()), 1e-4)}, "full-size forward")
    assert bad.mean() <= 1e-4, bad.mean()
    del o
    K, RN, TN, output, inside = out1[:5]
    g1 = torch.randn(pts.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1)) * 1e-2
    g2 = torch.randn(pts.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(2)) * 1e-2

    def bwd(g):
        return _C.sample_rasterized_depth_backward(*a[:9], inside, g, c1["tanx"], c1["tany"], 0.0, H, W,
                                                   _gpu(cam1.camera_center), *out1[5:11], K, RN, TN, False, False)

    b1, b2, b12 = bwd(g1), bwd(g2), bwd(g1 + 2 * g2)
    lin = {}
    for name, x, y, z in zip(GRADS, b1, b2, b12):
        assert torch.isfinite(z).all(), name
        want = (x + 2 * y).double()
        if float(want.norm()) == 0:
            continue
        err = float((z.double() - want).norm() / want.norm())
        lin[name] = (err, 1e-4)
    Hh.record_margins(lin, "full-size backward linearity")
    for name, (err, _) in lin.items():
        assert err <= 1e-4, (name, err)
