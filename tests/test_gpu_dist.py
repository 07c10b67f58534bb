"""RCCL leg of the view-parallel gradient exchange (gsr_dist).

A one-rank "nccl" (RCCL) group on cuda:0: the in-place coalesced all-reduce
and the bucketed one run through RCCL on device tensors and leave the sums
(here: the rank's own gradients) in the .grad tensors, in place for the
default path.  The two-rank arithmetic is covered by test_dist.py (gloo);
multi-GPU runs are bench.py --gpus N under torchrun.
"""
import os
import sys

import pytest
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]

pytestmark = pytest.mark.gpu


def test_rccl_inplace_and_bucketed_allreduce(tmp_path):
    from gsr_dist import ViewParallelGrads

    dev = torch.device("cuda", 0)
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        g = torch.Generator().manual_seed(0)
        shapes = [(1000, 3), (1000, 16, 3), (1000, 0, 3), (1000, 1), (1000, 4)]
        want = [torch.randn(s, generator=g) for s in shapes]
        for inplace in (True, False):
            params = [torch.zeros(s, device=dev, requires_grad=True) for s in shapes]
            for p, w in zip(params, want):
                p.grad = w.to(dev)
            ptrs = [p.grad.data_ptr() for p in params]
            red = ViewParallelGrads(params, bucket_mb=0.01, inplace=inplace)
            red.all_reduce(async_op=True)
            red.finish()
            torch.cuda.synchronize()
            for p, w in zip(params, want):
                assert torch.equal(p.grad.cpu(), w)
            if inplace:
                assert [p.grad.data_ptr() for p in params] == ptrs
    finally:
        dist.destroy_process_group()


def _views_backward(P, W, H, sh_degree, sg_degree, n_views, seed):
    """Per-view gradients of one shared scene seen by n orbit views (the
    C4 / C5 view-parallel setting), through the product autograd path."""
    import math

    import gsr_scene as S
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer

    dev = torch.device("cuda", 0)
    raw = S.make_gaussians(P, sh_degree=3, sg_degree=sg_degree, seed=seed, aspect=H / W, z_range=(4.0, 8.0))
    inp = {k: v.detach().contiguous().to(dev) for k, v in S.activated_inputs(raw).items()}
    cams = S.orbit_cameras(n_views, W, H)
    per_view, campos = [], []
    for v, cam_cpu in enumerate(cams):
        cam = cam_cpu.to(dev)
        ps = {k: t.clone().requires_grad_(True) for k, t in inp.items()}
        settings = GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2),
            kernel_size=0.0, bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam.world_view_transform,
            projmatrix=cam.full_proj_transform, sh_degree=sh_degree, sg_degree=sg_degree, campos=cam.camera_center,
            prefiltered=False, require_depth=True, debug=False)
        color, radii, mdepth, alpha, normal = GaussianRasterizer(settings)(
            means3D=ps["means3D"], means2D=torch.zeros(P, 3, device=dev, requires_grad=True),
            opacities=ps["opacities"], shs=ps["shs"], sg_axis=ps["sg_axis"], sg_sharpness=ps["sg_sharpness"],
            sg_color=ps["sg_color"], scales=ps["scales"], rotations=ps["rotations"])
        g = S.upstream_grads(H, W, seed=20 + v)
        torch.autograd.backward([color, mdepth, normal], [g["color"].to(dev), g["mdepth"].to(dev),
                                                          g["normal"].to(dev)])
        per_view.append({k: t.grad for k, t in ps.items()})
        campos.append(cam.camera_center.float())
    torch.cuda.synchronize()
    return inp, per_view, campos


@pytest.mark.parametrize("sh_degree,sg_degree", [(3, 0), (3, 7), (1, 0), (2, 3)])
def test_view_color_grads_match_summed_views(sh_degree, sg_degree):
    """gsr_view_color_grads (view_grads.hip) rebuilds the SH / SG gradient
    rows of a view-parallel step from each view's DC row and camera centre:
    against the sum over 3 views of the rows the backward itself produced
    (clamped colour channels included), within fp32 rounding."""
    from diff_gaussian_rasterization import _C

    P, W, H, n = 20000, 320, 240, 3
    inp, per_view, campos = _views_backward(P, W, H, sh_degree, sg_degree, n, seed=sh_degree + sg_degree)
    dev = inp["means3D"].device
    gathered = torch.cat([torch.cat([pv["shs"][:, 0, :].reshape(-1), c.reshape(3), torch.zeros(1, device=dev)])
                          for pv, c in zip(per_view, campos)])
    out = {k: torch.full_like(inp[k], float("nan")) for k in ("shs", "sg_axis", "sg_sharpness", "sg_color")}
    _C.view_color_grads(gathered, n, inp["means3D"], sh_degree, out["shs"], sg_degree, inp["sg_axis"],
                        inp["sg_sharpness"], inp["sg_color"], out["sg_axis"], out["sg_sharpness"], out["sg_color"])
    torch.cuda.synchronize()
    for k in ("shs", "sg_axis", "sg_sharpness", "sg_color"):
        want = sum(pv[k].double() for pv in per_view)
        got = out[k].double()
        if want.numel() == 0:
            continue
        assert bool(torch.isfinite(got).all()), k
        if not bool(want.any()):
            assert not bool(got.any()), k
            continue
        err = float((got - want).norm() / want.norm())
        assert err <= 1e-5, (k, err)
        assert float((got - want).abs().max() / want.abs().max()) <= 1e-4, k
    # the DC row is summed as gathered
    assert torch.equal(out["shs"][:, 0, :], per_view[0]["shs"][:, 0, :] + per_view[1]["shs"][:, 0, :]
                       + per_view[2]["shs"][:, 0, :])


def test_rccl_factored_exchange_one_rank(tmp_path):
    """FactoredViewGrads through RCCL on a one-rank group: the all-gather,
    the geometry all-reduce and the kernel rebuild this view's own SH / SG
    rows from its DC row (the two-rank sums: test_dist.py on gloo, and the
    kernel against summed views above)."""
    from gsr_dist import FactoredViewGrads

    dev = torch.device("cuda", 0)
    inp, per_view, campos = _views_backward(8000, 256, 192, 3, 7, 1, seed=5)
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        ps = {k: t.clone().requires_grad_(True) for k, t in inp.items()}
        for k in ps:
            ps[k].grad = per_view[0][k].clone()
        # (the backward ran before this exchanger existed: its count guard is off, its verify check on)
        ex = FactoredViewGrads(ps["means3D"], ps["opacities"], ps["scales"], ps["rotations"], ps["shs"],
                               ps["sg_axis"], ps["sg_sharpness"], ps["sg_color"], guard=False, verify=True)
        ex.exchange(campos[0], 3, 7)
        torch.cuda.synchronize()
        for k in ps:
            want, got = per_view[0][k].double(), ps[k].grad.double()
            err = float((got - want).norm() / want.norm().clamp_min(1e-30))
            assert err <= 1e-5, (k, err)
    finally:
        dist.destroy_process_group()


def test_factored_exchange_contract_guards(tmp_path):
    """FactoredViewGrads refuses a step whose SH rows are not those of
    exactly one rasterizer backward: two renders per step (the backward-count
    guard, on by default) and an extra SH-row gradient (verify)."""
    import math

    import gsr_scene as S
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from gsr_dist import FactoredViewGrads

    dev = torch.device("cuda", 0)
    P, W, H = 4000, 128, 96
    raw = S.make_gaussians(P, seed=3, aspect=H / W, z_range=(2.0, 6.0))
    ps = {k: v.detach().contiguous().to(dev).requires_grad_(True) for k, v in S.activated_inputs(raw).items()}
    cam = S.make_camera(W, H).to(dev)
    settings = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2),
        kernel_size=0.0, bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam.world_view_transform,
        projmatrix=cam.full_proj_transform, sh_degree=3, sg_degree=0, campos=cam.camera_center, prefiltered=False,
        require_depth=True, debug=False)

    def render_backward():
        color = GaussianRasterizer(settings)(
            means3D=ps["means3D"], means2D=torch.zeros(P, 3, device=dev, requires_grad=True),
            opacities=ps["opacities"], shs=ps["shs"], sg_axis=ps["sg_axis"], sg_sharpness=ps["sg_sharpness"],
            sg_color=ps["sg_color"], scales=ps["scales"], rotations=ps["rotations"])[0]
        color.square().sum().backward()

    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        ex = FactoredViewGrads(ps["means3D"], ps["opacities"], ps["scales"], ps["rotations"], ps["shs"],
                               verify=True)
        render_backward()
        ex.exchange(cam.camera_center, 3)  # one render: accepted
        for t in ps.values():
            t.grad = None
        render_backward()
        render_backward()
        with pytest.raises(RuntimeError, match="2 rasterizer SH backwards"):
            ex.exchange(cam.camera_center, 3)
        for t in ps.values():
            t.grad = None
        render_backward()
        ps["shs"].grad[:, 4] += 1e-3  # another loss on the SH rest rows
        with pytest.raises(RuntimeError, match="verify"):
            ex.exchange(cam.camera_center, 3)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sg_degree,chunks", [(0, 3), (7, 4), (0, 1)])
def test_overlapped_exchange_one_rank_matches_plain_backward(tmp_path, sg_degree, chunks):
    """gsr_dist.OverlappedViewGrads through RCCL on a one-rank group: the
    rasterizer backward runs its per-Gaussian tail in Gaussian ranges (the
    DC-row mode of gsr_rasterize_backward_ex), every range's geometry rows
    all-reduced and DC rows all-gathered as it is queued, the SH / SG rows
    rebuilt at the end — and the parameters' gradients equal those of the
    plain backward (geometry to the render backward's atomic order, colour
    rows to fp32 rounding of the rebuild)."""
    import math

    import gsr_scene as S
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from gsr_dist import OverlappedViewGrads

    dev = torch.device("cuda", 0)
    P, W, H = 20000, 320, 240
    raw = S.make_gaussians(P, sg_degree=sg_degree, seed=7, aspect=H / W, z_range=(2.0, 6.0))
    inp = {k: v.detach().contiguous().to(dev) for k, v in S.activated_inputs(raw).items()}
    cam = S.make_camera(W, H).to(dev)
    settings = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2),
        kernel_size=0.0, bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam.world_view_transform,
        projmatrix=cam.full_proj_transform, sh_degree=3, sg_degree=sg_degree, campos=cam.camera_center,
        prefiltered=False, require_depth=True, debug=False)
    g = {k: v.to(dev) for k, v in S.upstream_grads(H, W, seed=4).items()}

    def step():
        ps = {k: t.clone().requires_grad_(True) for k, t in inp.items()}
        color, radii, mdepth, alpha, normal = GaussianRasterizer(settings)(
            means3D=ps["means3D"], means2D=torch.zeros(P, 3, device=dev, requires_grad=True),
            opacities=ps["opacities"], shs=ps["shs"], sg_axis=ps["sg_axis"], sg_sharpness=ps["sg_sharpness"],
            sg_color=ps["sg_color"], scales=ps["scales"], rotations=ps["rotations"])
        torch.autograd.backward([color, mdepth, normal], [g["color"], g["mdepth"], g["normal"]])
        torch.cuda.synchronize()
        return {k: t.grad for k, t in ps.items()}

    plain = step()
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        with OverlappedViewGrads(chunks=chunks):
            over = step()
    finally:
        dist.destroy_process_group()
    for k in plain:
        want, got = plain[k].double(), over[k].double()
        if want.numel() == 0:
            continue
        assert bool(torch.isfinite(got).all()), k
        err = float((got - want).norm() / want.norm().clamp_min(1e-30))
        assert err <= 1e-5, (k, err)


# ---- two ranks through the real HIP backward (one GPU shared, gloo) ----
def _two_rank_worker(rank, world, port, outdir, sg_degree):
    import math
    import socket  # noqa: F401  (spawned interpreter: nothing is imported yet)
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [root, os.path.join(root, "geometry-grounded-gaussian-splatting_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gsr_scene as S
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from gsr_dist import FactoredViewGrads, OverlappedViewGrads

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    P, W, H = 20000, 320, 240
    raw = S.make_gaussians(P, sg_degree=sg_degree, seed=7, aspect=H / W, z_range=(2.0, 6.0))
    inp = {k: v.detach().contiguous().to(dev) for k, v in S.activated_inputs(raw).items()}
    cam = S.orbit_cameras(2, W, H, center_z=4.0, max_deg=8.0)[rank].to(dev)
    settings = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2),
        kernel_size=0.0, bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam.world_view_transform,
        projmatrix=cam.full_proj_transform, sh_degree=3, sg_degree=sg_degree, campos=cam.camera_center,
        prefiltered=False, require_depth=True, debug=False)
    g = {k: v.to(dev) for k, v in S.upstream_grads(H, W, seed=4 + rank).items()}

    def step(ps=None):
        ps = ps or {k: t.clone().requires_grad_(True) for k, t in inp.items()}
        color, radii, mdepth, alpha, normal = GaussianRasterizer(settings)(
            means3D=ps["means3D"], means2D=torch.zeros(P, 3, device=dev, requires_grad=True),
            opacities=ps["opacities"], shs=ps["shs"], sg_axis=ps["sg_axis"], sg_sharpness=ps["sg_sharpness"],
            sg_color=ps["sg_color"], scales=ps["scales"], rotations=ps["rotations"])
        torch.autograd.backward([color, mdepth, normal], [g["color"], g["mdepth"], g["normal"]])
        torch.cuda.synchronize()
        return ps

    plain = {k: t.grad.cpu() for k, t in step().items()}
    with OverlappedViewGrads(chunks=3):
        over = {k: t.grad.cpu() for k, t in step().items()}
    ps = {k: t.clone().requires_grad_(True) for k, t in inp.items()}
    ex = FactoredViewGrads(ps["means3D"], ps["opacities"], ps["scales"], ps["rotations"], ps["shs"], ps["sg_axis"],
                           ps["sg_sharpness"], ps["sg_color"])  # (its guard counts the backwards from here)
    step(ps)
    ex.exchange(cam.camera_center, 3, sg_degree)
    torch.cuda.synchronize()
    fact = {k: t.grad.cpu() for k, t in ps.items()}
    torch.save({"plain": plain, "over": over, "fact": fact}, os.path.join(outdir, f"g{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sg_degree", [0, 3])
def test_two_ranks_exchange_sums_views_on_gpu(tmp_path, sg_degree):
    """bench.py's N > 1 step with two ranks (two processes sharing cuda:0;
    gloo, since RCCL refuses two ranks on one device): each rank renders its
    own orbit view through the HIP forward and backward, and the overlapped
    (inside the backward, range by range) and factored (after it) exchanges
    give both ranks the same gradients, equal to the sum of the two views'
    plain gradients (rel. L2 <= 1e-5: the geometry rows are sums in another
    order, the colour rows are rebuilt from the gathered DC rows)."""
    import socket
    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.start_processes(_two_rank_worker, args=(2, port, str(tmp_path), sg_degree), nprocs=2, join=True,
                       start_method="spawn")
    r0 = torch.load(tmp_path / "g0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "g1.pt", weights_only=True)
    for k, p0 in r0["plain"].items():
        want = (p0.double() + r1["plain"][k].double())
        if want.numel() == 0:
            continue
        for form in ("over", "fact"):
            a, b = r0[form][k], r1[form][k]
            assert torch.equal(a, b), (form, k)  # the replicas stay bit-identical
            assert bool(torch.isfinite(a).all()), (form, k)
            err = float((a.double() - want).norm() / want.norm().clamp_min(1e-30))
            assert err <= 1e-5, (form, k, err)
