"""GPU parity tests of distCUDA2 (the initial scales of
create_from_pcd, scene/gaussian_model.py:323) — simple_knn._C.distCUDA2 over
libgsr.so (csrc/knn.hip) against the C oracle's restatement of
submodules/simple-knn/simple_knn.cu (itself pinned to scipy's exact k-d tree
in tests/test_oracle.py).

Both compute the exact 3-nearest-neighbour mean with the same squared-distance
rounding, so the bar is bit-exact equality; at 1M points (a DTU-scale
initial cloud) the check is against scipy's exact k-d tree (relative 1e-6).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import gsr_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _clouds():
    rng = np.random.default_rng(7)
    yield "gauss", rng.normal(size=(20000, 3))
    yield "uniform_offset", rng.uniform(3, 5, size=(5000, 3))  # bounds include the origin (init {0,0,0})
    surf = rng.normal(size=(30000, 3))
    yield "sphere_shell", surf / np.linalg.norm(surf, axis=1, keepdims=True) * 2 + 0.001 * rng.normal(size=surf.shape)
    dup = rng.normal(size=(3000, 3))
    yield "duplicates", np.concatenate([dup, dup[:1000], dup[:10]])
    yield "flat_z", np.concatenate([rng.normal(size=(4000, 2)), np.zeros((4000, 1))], 1)  # a 0/0 Morton axis
    yield "ragged_box", rng.normal(size=(1025, 3))
    for n in (1, 2, 3, 4, 7):
        yield f"tiny{n}", rng.normal(size=(n, 3))


@pytest.mark.parametrize("name,pts", list(_clouds()), ids=lambda x: x if isinstance(x, str) else "")
def test_distcuda2_bit_exact(name, pts):
    from simple_knn._C import distCUDA2

    pts = np.ascontiguousarray(pts, np.float32)
    ref, _ = O.knn_mean_dist(pts)
    got = distCUDA2(torch.from_numpy(pts).to(DEV)).cpu().numpy()
    assert got.shape == ref.shape
    assert np.array_equal(got, ref), (name, np.abs(got - ref).max())


def test_distcuda2_full_size_and_errors():
    from scipy.spatial import cKDTree
    from simple_knn._C import distCUDA2

    rng = np.random.default_rng(3)
    # a clustered 1M-point cloud (surfaces + noise), the shape of an SfM initialisation
    centers = rng.uniform(-5, 5, size=(2000, 3))
    pts = (centers[rng.integers(0, 2000, 1_000_000)] + 0.05 * rng.normal(size=(1_000_000, 3))).astype(np.float32)
    t = torch.from_numpy(pts).to(DEV)
    a = distCUDA2(t)
    b = distCUDA2(t)
    assert torch.equal(a, b)
    d, _ = cKDTree(pts.astype(np.float64)).query(pts.astype(np.float64), k=4, workers=16)
    ref = (d[:, 1:] ** 2).mean(1)
    got = a.cpu().numpy().astype(np.float64)
    assert np.abs(got - ref).max() <= 1e-6 * ref.max() + 1e-12
    assert (np.abs(got - ref) <= 1e-5 * ref + 1e-12).mean() > 0.9999
    assert distCUDA2(torch.zeros(0, 3, device=DEV)).shape == (0,)
    with pytest.raises(RuntimeError):
        distCUDA2(torch.zeros(5, 2, device=DEV))
    with pytest.raises(RuntimeError):
        distCUDA2(torch.zeros(5, 3))
