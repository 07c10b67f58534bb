"""Multi-process CPU test (gloo, world size 2) of the view-parallel step
(gsr_dist.ViewParallelGrads): after the all-reduce every rank
holds sum over views of the per-view gradients, identical on both ranks and
equal to a single-process sum."""
from __future__ import annotations

import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


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
