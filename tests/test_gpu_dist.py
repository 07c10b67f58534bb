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
