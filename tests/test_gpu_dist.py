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
    import torch.multiprocessing as mp

    import helpers as Hh
    port = Hh.free_port()
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


# ---- C4 / C5 at their full workload: N ranks sharing cuda:0 (gloo) ----
def _checksum(t: torch.Tensor) -> int:
    """A position-weighted checksum of a float32 tensor's bit patterns (equal
    checksums on every rank: the replicas are bit-identical, up to a hash
    collision)."""
    bits = t.detach().contiguous().view(-1).view(torch.int32).to(torch.int64)
    n = bits.numel()
    w = (torch.arange(n, device=bits.device, dtype=torch.int64) * 2654435761 + 97) % 1000003 + 1
    return int((bits * w).sum())


def _range_sums(t: torch.Tensor, ranges) -> torch.Tensor:
    """[n_ranges, 2] float64: the sum and the absolute sum of t's rows in each
    Gaussian range (queued on the stream, no host synchronisation)."""
    return torch.stack([torch.stack([t[b:e].double().sum(), t[b:e].double().abs().sum()]) for b, e in ranges])


def _full_rank_worker(rank, world, port, outdir, P, sg_degree, views, forms, chunks):
    """One rank of the view-parallel step at full workload (bench.py's N > 1
    step): its own 1080p orbit view of the shared scene, forward
    + backward through the HIP rasterizer, then each exchange form on fresh
    parameters; the float64 sum over the ranks of the plain per-view
    gradients is the yardstick, formed in float64 by an all-reduce.

    Self-diagnosing: per Gaussian range of the overlapped form,
    every tensor's error against the yardstick, and the range sums of what
    this rank posted (taken right after each range's collectives are posted,
    so the posting itself is not delayed) beside the same sums of its plain
    gradients — _run_full_ranks prints them on failure, which tells a wrong
    kernel output on one rank (posted != plain there) from a wrong transport
    (the posted sums add up to something other than the result)."""
    import json
    import math
    import sys
    import time

    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [root, os.path.join(root, "geometry-grounded-gaussian-splatting_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gsr_scene as S
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from gsr_dist import FactoredViewGrads, OverlappedViewGrads, ViewParallelGrads

    t_start = time.time()
    torch.set_num_threads(max(1, 16 // world))  # (the ranks share the box's 16-core CPU share)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    W, H = 1920, 1080
    raw = S.make_gaussians(P, sh_degree=3, sg_degree=sg_degree, aspect=H / W)  # bench.py's scene (seed 0)
    inp = {k: v.detach().contiguous().to(dev) for k, v in S.activated_inputs(raw).items()}
    del raw
    cam = S.orbit_cameras(views, W, H)[rank].to(dev)
    settings = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=math.tan(cam.FoVx / 2), tanfovy=math.tan(cam.FoVy / 2),
        kernel_size=0.0, bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam.world_view_transform,
        projmatrix=cam.full_proj_transform, sh_degree=3, sg_degree=sg_degree, campos=cam.camera_center,
        prefiltered=False, require_depth=True, debug=False)
    g = {k: v.to(dev) for k, v in S.upstream_grads(H, W, seed=11 + rank).items()}
    keys = ["means3D", "opacities", "scales", "rotations", "shs", "sg_axis", "sg_sharpness", "sg_color"]

    def fresh():
        return {k: inp[k].clone().requires_grad_(True) for k in keys}

    def step(ps):
        color, radii, mdepth, alpha, normal = GaussianRasterizer(settings)(
            means3D=ps["means3D"], means2D=torch.zeros(P, 3, device=dev, requires_grad=True),
            opacities=ps["opacities"], shs=ps["shs"], sg_axis=ps["sg_axis"], sg_sharpness=ps["sg_sharpness"],
            sg_color=ps["sg_color"], scales=ps["scales"], rotations=ps["rotations"])
        torch.autograd.backward([color, mdepth, normal], [g["color"], g["mdepth"], g["normal"]])
        torch.cuda.synchronize()
        n_vis = int((radii > 0).sum())
        return {k: (t.grad if t.grad is not None else torch.zeros_like(t)) for k, t in ps.items()}, n_vis

    plain, n_vis = step(fresh())
    from diff_gaussian_rasterization import _C as _gsr_C
    cs_ = _gsr_C.backward_chunk_size(P, chunks)
    ranges = [(b, min(P, b + cs_)) for b in range(0, P, cs_)]
    dkeys = ["means3D", "opacities", "scales", "rotations", "shs"]
    plain_sums = {k: _range_sums(plain[k] if k != "shs" else plain[k][:, 0], ranges).cpu().tolist() for k in dkeys}
    want = {}
    for k in keys:  # the yardstick: sum over the views in float64 (reduced on host copies: gloo's own staging
        w = plain[k].double().cpu()  # of device tensors is what the round-5 wrong sum was)
        if w.numel():
            dist.all_reduce(w)
        want[k] = w.to(dev)
    del plain
    res = {"rank": rank, "visible": n_vis, "forms": {}}
    for form in forms:
        ps = fresh()
        if form == "overlap":
            ex = OverlappedViewGrads(chunks=chunks)
            posted = []
            orig_on_chunk = ex.on_chunk

            def on_chunk(b, e, grads, ex=ex, orig=orig_on_chunk, posted=posted):
                orig(b, e, grads)
                g11 = grads[:11]
                rows = {"means3D": g11[3], "opacities": g11[2], "scales": g11[9], "rotations": g11[10]}
                sums = {k: _range_sums(v, [(b, e)])[0] for k, v in rows.items()}
                sums["shs"] = _range_sums(ex._dc.view(-1, 3), [(b, e)])[0]  # the DC rows all-gathered
                posted.append(sums)
            ex.on_chunk = on_chunk
            with ex:
                got, _ = step(ps)
        elif form == "factored":
            ex = FactoredViewGrads(ps["means3D"], ps["opacities"], ps["scales"], ps["rotations"], ps["shs"],
                                   ps["sg_axis"], ps["sg_sharpness"], ps["sg_color"])
            step(ps)
            ex.exchange(cam.camera_center, 3, sg_degree)
            torch.cuda.synchronize()
            got = {k: t.grad for k, t in ps.items()}
        else:
            step(ps)
            ViewParallelGrads([ps[k] for k in keys]).all_reduce()
            torch.cuda.synchronize()
            got = {k: t.grad for k, t in ps.items()}
        out = {}
        for k in keys:
            if want[k].numel() == 0:
                continue
            a = got[k]
            err = float((a.double() - want[k]).norm() / want[k].norm().clamp_min(1e-30))
            cs = torch.tensor([_checksum(a), -_checksum(a)], dtype=torch.int64)
            dist.all_reduce(cs, op=dist.ReduceOp.MAX)  # max and -min over the ranks
            out[k] = {"rel_l2": err, "finite": bool(torch.isfinite(a).all()),
                      "replicas_identical": int(cs[0]) == -int(cs[1])}
            if k in dkeys:  # per range: error, the result's range sums
                a2 = a if k != "shs" else a[:, 0]
                w2 = want[k] if k != "shs" else want[k][:, 0]
                out[k]["ranges"] = [float((a2[b:e].double() - w2[b:e]).norm() / w2[b:e].norm().clamp_min(1e-30))
                                    for b, e in ranges]
                out[k]["got_sums"] = _range_sums(a2, ranges).cpu().tolist()
        if form == "overlap":
            out["_posted"] = {k: [p[k].cpu().tolist() for p in posted] for k in dkeys}
            out["_plain"] = plain_sums
        res["forms"][form] = out
        del got, ps
    res["seconds"] = round(time.time() - t_start, 1)
    with open(os.path.join(outdir, f"full{rank}.json"), "w") as f:
        json.dump(res, f)
    print(f"[rank {rank}] done in {res['seconds']} s", flush=True)
    dist.barrier()
    dist.destroy_process_group()


def _print_overlap_diagnosis(rs) -> None:
    """On a failure: per range and tensor of the overlapped form, the error
    against the yardstick; each rank's posted range sums against its plain
    gradients' (a rank whose kernel output was wrong); and the posted sums
    over the ranks against the result's (a transport that lost rows)."""
    for form, d0 in rs[0]["forms"].items():
        for k, v in d0.items():
            if k.startswith("_") or "ranges" not in v:
                continue
            print(f"[diag] {form} {k}: per-range rel L2 " + " ".join(f"{x:.2e}" for x in v["ranges"]))
    if "overlap" not in rs[0]["forms"]:
        return
    for k in rs[0]["forms"]["overlap"]["_posted"]:
        n_ranges = len(rs[0]["forms"]["overlap"]["_posted"][k])
        for i in range(n_ranges):
            posted = [r["forms"]["overlap"]["_posted"][k][i] for r in rs]
            plain = [r["forms"]["overlap"]["_plain"][k][i] for r in rs]
            got = rs[0]["forms"]["overlap"][k]["got_sums"][i]
            rel = [abs(p[0] - q[0]) / max(q[1], 1e-30) for p, q in zip(posted, plain)]
            tot = sum(p[0] for p in posted)
            print(f"[diag] overlap {k} range {i}: posted-vs-plain per rank " + " ".join(f"{x:.1e}" for x in rel)
                  + f"; sum of posted {tot:.6e} vs result {got[0]:.6e} (abs-sum scale {got[1]:.3e})")


def _run_full_ranks(tmp_path, world, P, sg_degree, views, forms, chunks=4):
    import json
    import torch.multiprocessing as mp

    import helpers as Hh
    port = Hh.free_port()
    mp.start_processes(_full_rank_worker, args=(world, port, str(tmp_path), P, sg_degree, views, forms, chunks),
                       nprocs=world, join=True, start_method="spawn")
    rs = [json.load(open(tmp_path / f"full{r}.json")) for r in range(world)]
    bad = any(not v["finite"] or not v["replicas_identical"] or v["rel_l2"] > 1e-5
              for r in rs for d in r["forms"].values() for k, v in d.items() if not k.startswith("_"))
    if bad:
        _print_overlap_diagnosis(rs)
    for r in rs:
        print(f"rank {r['rank']}: {r['visible']} visible Gaussians, {r['seconds']} s, "
              + ", ".join(f"{f}: max rel L2 {max(v['rel_l2'] for k, v in d.items() if not k.startswith('_')):.2e}"
                          for f, d in r["forms"].items()))
        assert r["visible"] > 0.3 * P, r["visible"]  # every view sees a large part of the scene
        for form, d in r["forms"].items():
            for k, v in d.items():
                if k.startswith("_"):
                    continue
                assert v["finite"], (r["rank"], form, k)
                assert v["replicas_identical"], (r["rank"], form, k)  # bit-identical on every rank
                assert v["rel_l2"] <= 1e-5, (r["rank"], form, k, v["rel_l2"])
    return rs


@pytest.mark.timeout(600)
def test_c4_eight_ranks_full_workload(tmp_path):
    """C4 (BASELINE.json configs[3]) at its workload: 8 ranks — 8 processes
    sharing cuda:0 over gloo, since RCCL refuses two ranks on one device —
    each rendering its own 1920x1080 orbit view of the same 1M Gaussians (SH
    3) forward + backward through the HIP rasterizer.  For the overlapped
    (inside the backward, 4 Gaussian ranges), factored and all-reduce
    exchanges: every rank's gradients are bit-identical and within 1e-5
    relative L2 of the float64 sum over the 8 views of each view's plain
    gradients (train.py:142-262 sharded per SURVEY §8(e)).  The RCCL/xGMI
    timing itself is the driver's 8-GPU run."""
    _run_full_ranks(tmp_path, 8, 1_000_000, 0, 8, ["overlap", "factored", "allreduce"])


@pytest.mark.timeout(600)
def test_c5_two_ranks_full_workload(tmp_path):
    """C5's multi-GPU leg at its workload, on two ranks sharing cuda:0 (gloo):
    5M Gaussians with SH 3 + SG 7 at 1920x1080, two orbit views; the
    overlapped (7 ranges) and factored exchanges against the float64 sum of
    the two views' plain gradients (bit-identical replicas, rel. L2 <= 1e-5)."""
    _run_full_ranks(tmp_path, 2, 5_000_000, 7, 8, ["overlap", "factored"], chunks=7)


@pytest.mark.timeout(900)
def test_c5_eight_ranks_full_workload(tmp_path):
    """C5's 8-GPU leg (BASELINE.json configs[4]) at its workload, rehearsed
    as 8 ranks sharing cuda:0 over gloo: 5M Gaussians with
    SH 3 + SG 7 at 1920x1080, 8 orbit views — the 8-view range-major DC-row
    gather (8 x 5M x 12 B) and 8 replicas of the SG-7 state — for the
    overlapped (7 ranges) and factored exchanges against the float64 sum of
    the 8 views' plain gradients (bit-identical replicas, rel. L2 <= 1e-5).
    RCCL over xGMI itself stays the driver's 8-GPU run."""
    _run_full_ranks(tmp_path, 8, 5_000_000, 7, 8, ["overlap", "factored"], chunks=7)


# ---- the training step's split SH layout through the overlapped exchange ----
def _train_rank_worker(rank, world, port, outdir):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [root, os.path.join(root, "geometry-grounded-gaussian-splatting_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gsr_train
    from gaussian_renderer import render
    from gsr_dist import OverlappedViewGrads

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    step, view, nearest = gsr_train.synthetic_training_setup(20_000, 320, 240, device="cuda", seed=3)
    g = step.g
    mine = gsr_train.orbit_views(8, 320, 240, dev)[2 + 3 * rank]  # this rank's view
    gen = torch.Generator().manual_seed(40 + rank)
    w = {k: torch.randn(s, generator=gen).to(dev) for k, s in
         (("render", (3, 240, 320)), ("median_depth", (1, 240, 320)), ("normal", (3, 240, 320)))}
    params = {n: p for n, p in g.named_parameters() if p.numel()}

    def render_grads():
        """A loss on the render outputs alone (no other term on the parameters):
        the raw parameters' gradients through the fused getters and the split
        SH pair, as TrainStep's render call forms them."""
        g.optimizer.zero_grad(set_to_none=True)
        g.begin_step()
        try:
            pkg = render(mine, g, step.pipe, step.bg, 0.0, require_depth=True)
            assert isinstance(g.get_features, tuple)  # the split layout is what the exchange sees
            loss = sum((pkg[k] * w[k]).sum() for k in w)
            loss.backward()
        finally:
            g.end_step()
        torch.cuda.synchronize()
        return {n: p.grad.detach().clone() for n, p in params.items()}

    plain = render_grads()
    with OverlappedViewGrads(chunks=3) as ex:
        over = render_grads()
        ex.check()
        # a whole TrainStep (render + depth-normal + PatchMatch + L1/SSIM + backward + densify + Adam) with the
        # exchange installed: the render backward exchanges its split-SH gradients, the step completes
        loss = step.step(view, nearest)
        ex.check()
    finite = bool(torch.isfinite(loss)) and all(bool(torch.isfinite(p).all()) for p in params.values())
    torch.save({"plain": {k: v.cpu() for k, v in plain.items()}, "over": {k: v.cpu() for k, v in over.items()},
                "finite": finite}, os.path.join(outdir, f"t{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_train_step_split_sh_through_overlapped_exchange(tmp_path):
    """TrainGaussians.get_features hands the rasterizer the split
    SH pair (features_dc, features_rest), and the overlapped exchange now
    rebuilds both gradient tensors (gsr_view_color_grads_chunked's split
    output, ABI 20).  Two ranks on cuda:0 (gloo), each with its own view: a
    loss on the render outputs gives every raw parameter (through the fused
    getters) the sum over the two views of its plain gradient, identically on
    both ranks; and a whole TrainStep runs with the exchange installed."""
    import torch.multiprocessing as mp

    import helpers as Hh
    port = Hh.free_port()
    mp.start_processes(_train_rank_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    r = [torch.load(tmp_path / f"t{k}.pt", weights_only=True) for k in range(2)]
    assert r[0]["finite"] and r[1]["finite"]
    for k, p0 in r[0]["plain"].items():
        want = p0.double() + r[1]["plain"][k].double()
        a, b = r[0]["over"][k], r[1]["over"][k]
        assert torch.equal(a, b), k  # the replicas stay bit-identical
        err = float((a.double() - want).norm() / want.norm().clamp_min(1e-30))
        print(f"{k}: rel L2 {err:.2e}")
        assert err <= 1e-5, (k, err)
