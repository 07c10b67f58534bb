"""Multi-process CPU test (gloo, world size 2) of the view-parallel step
(gsr_dist.ViewParallelGrads): after the all-reduce every rank
holds sum over views of the per-view gradients, identical on both ranks and
equal to a single-process sum."""
from __future__ import annotations

import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    import helpers as Hh
    return Hh.free_port()  # (outside the ephemeral range: see helpers.free_port)


def _view_grads(view):
    """float64 autograd gradients of one view of a small shared scene."""
    import gsr_scene as S
    import torch_ref as R
    import helpers as Hh

    cam = S.orbit_cameras(2, 32, 24, center_z=3.0, max_deg=10.0)[view]
    c = Hh.small_case(P=30, W=32, H=24, seed=2, cam=cam, z_range=(2.0, 4.0))
    inp = {k: v.double().clone().requires_grad_(True) for k, v in c["inp"].items()}
    m2d = torch.zeros(30, 3, dtype=torch.float64, requires_grad=True)
    pre = R.preprocess(inp["means3D"], inp["scales"], inp["rotations"], inp["opacities"], inp["shs"], inp["sg_axis"],
                       inp["sg_sharpness"], inp["sg_color"], m2d, cam.world_view_transform.double(),
                       cam.full_proj_transform.double(), cam.camera_center.double(), 32, 24, c["tanx"], c["tany"],
                       0.0, 3, 0)
    lists, _ = R.binning(pre, 32, 24)
    out = R.render(pre, lists, 32, 24, c["bg"].double(), require_depth=False)
    g = S.upstream_grads(24, 32, seed=10 + view)
    (out["color"] * g["color"].double()).sum().backward()
    return inp


def _worker(rank, world, port, outdir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gsr_dist import ViewParallelGrads, reduce_densification_stats

    inp = _view_grads(rank)
    params = [inp[k] for k in ("means3D", "shs", "opacities", "scales", "rotations")]
    red = ViewParallelGrads([p.float().detach().requires_grad_(True) for p in params], bucket_mb=0.002,
                            inplace=False)
    for p, src in zip(red.params, params):
        p.grad = src.grad.float().clone()
    assert len(red.buckets) >= 2  # small buckets exercise the bucketing path
    red.all_reduce(async_op=(rank == 0))
    if rank == 0:
        red.finish() if red._work else None
    # the default: .grad tensors summed in place by one coalesced all-reduce
    ipl = ViewParallelGrads([p.float().detach().requires_grad_(True) for p in params])
    for p, src in zip(ipl.params, params):
        p.grad = src.grad.float().clone()
    ptrs = [p.grad.data_ptr() for p in ipl.params]
    ipl.all_reduce(async_op=(rank == 1))
    if rank == 1:
        ipl.finish()
    assert [p.grad.data_ptr() for p in ipl.params] == ptrs  # no copies
    for a, b in zip(ipl.params, red.params):
        assert torch.equal(a.grad, b.grad)
    gn = torch.arange(30, dtype=torch.float32) * (rank + 1)
    den = torch.ones(30) * (rank + 1)
    mr = torch.arange(30, dtype=torch.int32) * (1 if rank == 0 else -1) + rank * 100
    reduce_densification_stats(gn, den, mr)
    torch.save({"grads": [p.grad for p in red.params], "gn": gn, "den": den, "mr": mr},
               os.path.join(outdir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_view_parallel_allreduce_sums_views(tmp_path):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    g0, g1 = _view_grads(0), _view_grads(1)
    for k, name in enumerate(("means3D", "shs", "opacities", "scales", "rotations")):
        want = (g0[name].grad + g1[name].grad).float()
        assert torch.equal(r0["grads"][k], r1["grads"][k])
        torch.testing.assert_close(r0["grads"][k], want, rtol=1e-5, atol=1e-7)
    assert torch.equal(r0["gn"], torch.arange(30, dtype=torch.float32) * 3)
    assert torch.equal(r0["den"], torch.full((30,), 3.0))
    assert torch.equal(r0["mr"], torch.maximum(torch.arange(30, dtype=torch.int32),
                                               100 - torch.arange(30, dtype=torch.int32)))


# ---- factored colour exchange (gsr_dist.FactoredViewGrads) ----------------
_C0, _C1 = 0.28209479177387814, 0.4886025119029199
_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
       1.445305721320277, -0.5900435899266435)


def _sh_basis(d):
    """SH basis [P, 16] of unit directions [P, 3] (CR/auxiliary.h:21-36, render_forward.cu:22-78)."""
    x, y, z = d[:, 0], d[:, 1], d[:, 2]
    xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
    return torch.stack([torch.full_like(x, _C0), -_C1 * y, _C1 * z, -_C1 * x,
                        _C2[0] * xy, _C2[1] * yz, _C2[2] * (2 * zz - xx - yy), _C2[3] * xz, _C2[4] * (xx - yy),
                        _C3[0] * y * (3 * xx - yy), _C3[1] * xy * z, _C3[2] * y * (4 * zz - xx - yy),
                        _C3[3] * z * (2 * zz - 3 * xx - 3 * yy), _C3[4] * x * (4 * zz - xx - yy),
                        _C3[5] * z * (xx - yy), _C3[6] * x * (xx - 3 * yy)], dim=1)


def _expand_ref(gathered, n_views, means3D, sh_degree, dL_dsh, sg_degree=0, *_sg):
    """float64 torch restatement of gsr_view_color_grads (view_grads.hip) for
    SH only: dL/dsh[k] = sum_v Y_k(d_v) dsh0_v / SH_C0, the DC row summed as is."""
    P = means3D.shape[0]
    g = gathered.double().view(n_views, 3 * P + 4)
    n = (sh_degree + 1) ** 2
    out = torch.zeros(P, dL_dsh.shape[1], 3, dtype=torch.float64)
    for v in range(n_views):
        dsh0 = g[v, :3 * P].view(P, 3)
        d = means3D.double() - g[v, 3 * P:3 * P + 3]
        Y = _sh_basis(d / d.norm(dim=1, keepdim=True))
        out[:, 0] += dsh0
        out[:, 1:n] += Y[:, 1:n, None] * (dsh0 / _C0)[:, None, :]
    dL_dsh.copy_(out.to(dL_dsh.dtype))


def _factored_worker(rank, world, port, outdir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gsr_scene as S
    from gsr_dist import FactoredViewGrads

    inp = _view_grads(rank)
    names = ("means3D", "opacities", "scales", "rotations", "shs")
    ps = {k: inp[k].float().detach().requires_grad_(True) for k in names}
    for k in names:
        ps[k].grad = inp[k].grad.float().clone()
    campos = S.orbit_cameras(2, 32, 24, center_z=3.0, max_deg=10.0)[rank].camera_center.float()
    # the contract guards (gsr_dist.FactoredViewGrads docstring), checked on both ranks before any collective:
    # no rasterizer backward ran in this process -> the backward-count guard refuses the exchange
    import pytest
    with pytest.raises(RuntimeError, match="rasterizer SH backwards"):
        FactoredViewGrads(ps["means3D"], ps["opacities"], ps["scales"], ps["rotations"], ps["shs"],
                          expand=_expand_ref, guard=True).exchange(campos, sh_degree=3)
    # an extra contribution to the SH rest rows (a stale .grad / another loss) -> verify refuses it
    stale = ps["shs"].detach().clone().requires_grad_(True)
    stale.grad = ps["shs"].grad.clone()
    stale.grad[:, 5] += 1e-3
    with pytest.raises(RuntimeError, match="verify"):
        FactoredViewGrads(ps["means3D"], ps["opacities"], ps["scales"], ps["rotations"], stale,
                          expand=_expand_ref, verify=True).exchange(campos, sh_degree=3)
    ex = FactoredViewGrads(ps["means3D"], ps["opacities"], ps["scales"], ps["rotations"], ps["shs"],
                           expand=_expand_ref, verify=True)
    # the reference's split SH parameters (features_dc, features_rest) before the exchange above overwrites shs.grad
    dc = ps["shs"][:, :1].detach().clone().requires_grad_(True)
    rest = ps["shs"][:, 1:].detach().clone().requires_grad_(True)
    dc.grad = ps["shs"].grad[:, :1].clone()
    rest.grad = ps["shs"].grad[:, 1:].clone()
    ex.exchange(campos, sh_degree=3)
    geo = [t.detach().clone().requires_grad_(True) for t in (ps["means3D"], ps["opacities"], ps["scales"],
                                                           ps["rotations"])]
    for t, k in zip(geo, ("means3D", "opacities", "scales", "rotations")):
        t.grad = inp[k].grad.float().clone()
    FactoredViewGrads(*geo, (dc, rest), expand=_expand_ref).exchange(campos, sh_degree=3)
    assert torch.equal(torch.cat([dc.grad, rest.grad], dim=1), ps["shs"].grad)
    torch.save({k: ps[k].grad for k in names}, os.path.join(outdir, f"f{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_factored_exchange_sums_views(tmp_path):
    """The factored exchange (geometry rows all-reduced, colour rows rebuilt
    from the all-gathered DC rows + camera centres) gives every rank the sum
    over views of the per-view gradients — the SH rows included — identically
    on both ranks."""
    port = _free_port()
    mp.start_processes(_factored_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    f0 = torch.load(tmp_path / "f0.pt", weights_only=True)
    f1 = torch.load(tmp_path / "f1.pt", weights_only=True)
    g0, g1 = _view_grads(0), _view_grads(1)
    for name in ("means3D", "opacities", "scales", "rotations", "shs"):
        want = (g0[name].grad + g1[name].grad).float()
        assert torch.equal(f0[name], f1[name]), name
        torch.testing.assert_close(f0[name], want, rtol=1e-5, atol=1e-7)


# ---- the exchange inside the backward, range by range (gsr_dist.OverlappedViewGrads) ----
def _expand_chunked_ref(gathered, campos, n_views, chunk, means3D, sh_degree, dL_dsh, sg_degree=0, *_sg):
    """_expand_ref for the range-by-range gathered layout (include/gsr.h
    gsr_view_color_grads_chunked): range [b, b+len) holds [n_views][len][3]."""
    P = means3D.shape[0]
    dc = torch.empty(n_views, P, 3, dtype=gathered.dtype)
    for b in range(0, P, chunk):
        e = min(P, b + chunk)
        dc[:, b:e] = gathered[3 * n_views * b:3 * n_views * e].view(n_views, e - b, 3)
    legacy = torch.cat([torch.cat([dc[v].reshape(-1), campos[v]]) for v in range(n_views)])
    _expand_ref(legacy, n_views, means3D, sh_degree, dL_dsh)


def _overlap_worker(rank, world, port, outdir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gsr_scene as S
    from gsr_dist import OverlappedViewGrads

    inp = _view_grads(rank)
    P = 30
    campos = S.orbit_cameras(2, 32, 24, center_z=3.0, max_deg=10.0)[rank].camera_center.float()
    g = {k: inp[k].grad.float().clone() for k in ("means3D", "opacities", "scales", "rotations", "shs")}
    z = lambda *s: torch.zeros(*s)  # noqa: E731
    # the rasterizer's 11 outputs as _C.rasterize_gaussians_backward returns them (dsh left for the rebuild)
    grads = (z(P, 3), z(P, 3), g["opacities"].clone(), g["means3D"].clone(), z(P, 6), torch.full((P, 16, 3), 7.0),
             z(P, 0, 3), z(P, 0), z(P, 0, 3), g["scales"].clone(), g["rotations"].clone())
    ex = OverlappedViewGrads(chunks=4, expand=_expand_chunked_ref)
    ex.chunk_size = lambda P_: 8  # (the HIP backward's ranges are whole 256-Gaussian workgroups; 30 Gaussians here)
    ex.begin(campos, P, True, True)
    ex.dc_rows(P, "cpu").copy_(g["shs"][:, 0, :].reshape(-1))  # what the kernel writes in DC-row mode
    cs = ex.chunk_size(P)
    for b in range(0, P, cs):  # as gsr_rasterize_backward_ex calls on_chunk
        ex.on_chunk(b, min(P, b + cs), grads)
    ex.finish(grads, inp["means3D"].detach().float(), None, None, None, 3, 0)
    torch.save({"means3D": grads[3], "opacities": grads[2], "scales": grads[9], "rotations": grads[10],
                "shs": grads[5]}, os.path.join(outdir, f"o{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_overlapped_exchange_sums_views(tmp_path):
    """OverlappedViewGrads' range-by-range protocol (geometry rows all-reduced
    and DC rows all-gathered per Gaussian range, colour rows rebuilt at the
    end) gives both ranks the sum over views of every gradient, identically."""
    port = _free_port()
    mp.start_processes(_overlap_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    o0 = torch.load(tmp_path / "o0.pt", weights_only=True)
    o1 = torch.load(tmp_path / "o1.pt", weights_only=True)
    g0, g1 = _view_grads(0), _view_grads(1)
    for name in ("means3D", "opacities", "scales", "rotations", "shs"):
        want = (g0[name].grad + g1[name].grad).float()
        assert torch.equal(o0[name], o1[name]), name
        torch.testing.assert_close(o0[name], want, rtol=1e-5, atol=1e-7)


def test_coalescing_choice_by_backend_and_device(tmp_path):
    """gsr_dist._coalescing: the coalesced all-reduce where the backend has it
    for the tensors (gloo on host tensors; RCCL always), one all-reduce per
    tensor for gloo with device tensors (the one-GPU rehearsal of the N > 1
    path: gloo has no allreduce_coalesced for them)."""
    sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
    from gsr_dist import _coalescing

    class Dev:  # a stand-in device tensor: only .is_cuda is read
        is_cuda = True

    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("gloo", store=store, rank=0, world_size=1)
    try:
        assert _coalescing(None, [torch.zeros(3), torch.zeros(2)]) is getattr(dist, "_coalescing_manager", None)
        assert _coalescing(None, [torch.zeros(3), Dev()]) is None
    finally:
        dist.destroy_process_group()


# ---- OverlappedViewGrads on its error paths -------------------
def _overlap_grads(P, seed):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g)  # noqa: E731
    return (torch.zeros(P, 3), torch.zeros(P, 3), r(P, 1), r(P, 3), torch.zeros(P, 6), torch.zeros(P, 16, 3),
            torch.zeros(P, 0, 3), torch.zeros(P, 0), torch.zeros(P, 0, 3), r(P, 3), r(P, 4))


def _error_worker(rank, world, port, outdir, sync_check=None):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gsr_dist import OverlappedViewGrads

    P = 30

    class Failing(OverlappedViewGrads):
        def on_chunk(self, b, e, grads):
            if rank == 0 and b == 8:
                raise ValueError("injected failure in range [8, 16)")
            super().on_chunk(b, e, grads)

    ex = Failing(chunks=4, expand=_expand_chunked_ref, sync_check=sync_check)
    ex.chunk_size = lambda P_: 8
    grads = _overlap_grads(P, seed=rank)
    mine = [t.clone() for t in grads]
    ex.begin(torch.zeros(3), P, True, True)
    ex.dc_rows(P, "cpu").copy_(torch.arange(3 * P, dtype=torch.float32) * (rank + 1))
    cb = ex.hook(grads)
    for b in range(0, P, 8):  # as gsr_rasterize_backward_ex calls its callback: every range, after a failure too
        cb(b, min(P, b + 8))
    raised = None
    try:
        ex.settle(True)
        ex.finish(grads, torch.randn(P, 3), None, None, None, 3, 0)
    except (ValueError, RuntimeError) as e:
        raised = str(e)
    out = {"raised": raised, "works_left": len(ex._works), "active": ex._active,
           "means3D": grads[3], "mine": mine[3]}
    if sync_check is False:  # deferred: the flag is read by the next begin() (or check()), before any collective
        out["raised_in_backward"] = raised
        try:
            ex.begin(torch.zeros(3), P, True, True)
            out["raised"] = None
            ex.abort()
        except RuntimeError as e:
            out["raised"] = str(e) if raised is None else raised
        out["active_after_begin"] = ex._active
    # the next backward runs normally after the failed one: the group is still in lockstep
    ex2 = OverlappedViewGrads(chunks=4, expand=_expand_chunked_ref)
    ex2.chunk_size = lambda P_: 8
    g2 = _overlap_grads(P, seed=10 + rank)
    ex2.begin(torch.zeros(3), P, True, False)
    cb2 = ex2.hook(g2)
    for b in range(0, P, 8):
        cb2(b, min(P, b + 8))
    ex2.settle(True)
    ex2.finish(g2, None, None, None, None, 3, 0)
    out["next_step"] = g2[3]
    torch.save(out, os.path.join(outdir, f"e{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sync_check", [None, False])
def test_overlapped_exchange_failure_keeps_ranks_in_lockstep(tmp_path, sync_check):
    """A range whose exchange raises on one rank: that rank still
    posts every remaining range's collectives — on NaN rows — waits for all of
    its works and re-raises; the peer's backward completes its collectives (no
    deadlock) and then raises too (the failure flag all-reduced at
    the end of every backward), so no rank hands NaN-summed gradients to its
    optimizer; the next step runs normally on both."""
    port = _free_port()
    mp.start_processes(_error_worker, args=(2, port, str(tmp_path), sync_check), nprocs=2, join=True,
                       start_method="spawn")
    e0 = torch.load(tmp_path / "e0.pt", weights_only=True)
    e1 = torch.load(tmp_path / "e1.pt", weights_only=True)
    assert e0["raised"] == "injected failure in range [8, 16)"
    assert e1["raised"] is not None and "a peer rank's rasterizer backward failed" in e1["raised"]
    assert e0["works_left"] == 0 and not e0["active"] and not e1["active"]
    if sync_check is False:  # deferred: the peer's backward returns; its next begin() raises
        assert e1["raised_in_backward"] is None and not e1["active_after_begin"]
    m1 = e1["means3D"]
    torch.testing.assert_close(m1[:8], e0["mine"][:8] + e1["mine"][:8])  # posted before the failure: summed
    assert torch.isnan(m1[8:]).all()  # the failed rank's remaining ranges: NaN, not silently one view
    want = _overlap_grads(30, 10)[3] + _overlap_grads(30, 11)[3]
    torch.testing.assert_close(e0["next_step"], want)
    torch.testing.assert_close(e1["next_step"], want)


def _layout_worker(rank, world, port, outdir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd"), HERE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gsr_dist import OverlappedViewGrads
    import pytest

    P = 30
    ex = OverlappedViewGrads(chunks=4, expand=_expand_chunked_ref)
    ex.chunk_size = lambda P_: 8
    g = _overlap_grads(P, seed=rank)
    # a backward whose ranges do not follow the layout the gathered rows assume (a range size of 10, not 8)
    ex.begin(torch.zeros(3), P, True, False)
    cb = ex.hook(g)
    for b in range(0, P, 10):
        cb(b, min(P, b + 10))
    with pytest.raises(RuntimeError, match="does not follow the range layout"):
        ex.settle(True)
    # a backward that stopped part-way (the C call failed after range 1) is settled by abort()
    ex.begin(torch.zeros(3), P, True, False)
    cb = ex.hook(g)
    cb(0, 8)
    cb(8, 16)
    ex.settle(False)
    assert not ex._works and not ex._active
    # ranges that do not cover [0, P): finish refuses
    ex.begin(torch.zeros(3), P, True, False)
    cb = ex.hook(g)
    cb(0, 8)
    with pytest.raises(RuntimeError, match=r"covered \[0, 8\) of 30"):
        ex.finish(g, None, None, None, None, 3, 0)
    # verify_replicas: identical gradients pass, a rank-local extra term is caught
    ps = [torch.ones(4, 3).requires_grad_(True), torch.ones(4, 1).requires_grad_(True)]
    for p in ps:
        p.grad = torch.full_like(p, 2.0)
    ex.verify_replicas(ps)
    if rank == 1:
        ps[1].grad[0] += 1e-3
    with pytest.raises(RuntimeError, match="parameter 1's gradients differ"):
        ex.verify_replicas(ps)
    dist.barrier()
    dist.destroy_process_group()


def test_overlapped_exchange_layout_and_replica_guards(tmp_path):
    """Ranges that do not follow gsr_backward_chunk_size's layout are refused
    (the DC rows would be rebuilt from the wrong views' rows); a backward that
    failed part-way is settled with every range posted; ranges that stop
    short are refused by finish; verify_replicas catches drifting replicas."""
    port = _free_port()
    mp.start_processes(_layout_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")


def test_backward_chunk_size_is_the_library_s():
    """One source for the range size: gsr_backward_chunk_size (host
    only) and OverlappedViewGrads.chunk_size agree with the layout
    view_color_grads_chunked reads."""
    sys.path[:0] = [os.path.join(ROOT, "geometry-grounded-gaussian-splatting_amd")]
    from diff_gaussian_rasterization import _C
    import pytest

    for P, c in [(0, 1), (1, 1), (255, 4), (256, 1), (1000, 4), (1_000_000, 4), (5_000_000, 7), (2**31 - 1, 3)]:
        assert _C.backward_chunk_size(P, c) == ((P + c - 1) // c + 255) // 256 * 256
    with pytest.raises(RuntimeError, match="chunks >= 1"):
        _C.backward_chunk_size(10, 0)
