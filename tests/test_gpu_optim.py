"""GPU tests of the training update (csrc/optim.hip):
FusedAdam against torch.optim.Adam (the reference's optimizer,
scene/gaussian_model.py:347-351) and the densification statistics against
the reference's own torch statements (gaussian_model.py:818-821,
train.py:236-237).  The oracle here is torch on the CPU, fp32.

Tolerances: Adam state and parameters max|a-b| <= 2e-6 * max|b| + 1e-12
(same fp32 formula, different rounding of sqrt/division); statistics exact
except the x/y norm (<= 1 ulp).
"""
from __future__ import annotations

import math

import pytest
import torch

import gsr_optim

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)

# the Gaussian parameter groups of GaussianModel (xyz, f_dc, f_rest, opacity, scaling, rotation, sg_*)
SHAPES = {"xyz": (3,), "f_dc": (1, 3), "f_rest": (15, 3), "opacity": (1,), "scaling": (3,), "rotation": (4,),
          "sg_axis": (7, 3), "sg_sharpness": (7,), "sg_color": (7, 3)}
LRS = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 1.25e-4, "opacity": 5e-2, "scaling": 5e-3, "rotation": 1e-3,
       "sg_axis": 1e-3, "sg_sharpness": 1e-3, "sg_color": 1e-4}


def _groups(P, seed, device):
    g = torch.Generator().manual_seed(seed)
    return [{"params": [torch.nn.Parameter(torch.randn((P,) + s, generator=g).to(device))], "lr": LRS[k], "name": k}
            for k, s in SHAPES.items()]


def _pair(P, seed):
    ref = _groups(P, seed, "cpu")
    mine = _groups(P, seed, DEV)
    o_ref = torch.optim.Adam(ref, lr=0.0, eps=1e-15, foreach=False)
    o_mine = gsr_optim.FusedAdam(mine, lr=0.0, eps=1e-15)
    return ref, mine, o_ref, o_mine


def _close(a, b, rtol=2e-6):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    return float((a - b).abs().max()) <= rtol * float(b.abs().max()) + 1e-12


@pytest.mark.parametrize("P", [1, 7, 10007])
def test_fused_adam_matches_torch_adam(P):
    ref, mine, o_ref, o_mine = _pair(P, 0)
    g = torch.Generator().manual_seed(1)
    for it in range(4):
        for gr, gm in zip(ref, mine):
            grad = torch.randn(gr["params"][0].shape, generator=g) * 10 ** (-it)
            if it == 2:
                grad[: max(1, P // 3)] = 0.0  # zero gradients still decay the moments
            gr["params"][0].grad = grad.clone()
            gm["params"][0].grad = grad.to(DEV)
        if it == 1:  # the reference's xyz learning-rate schedule edits param_groups in place
            for o in (o_ref, o_mine):
                for grp in o.param_groups:
                    if grp["name"] == "xyz":
                        grp["lr"] = 1.1e-4
        o_ref.step()
        o_mine.step()
        for gr, gm in zip(ref, mine):
            pr, pm = gr["params"][0], gm["params"][0]
            assert _close(pm, pr), (gr["name"], it)
            sr, sm = o_ref.state[pr], o_mine.state[pm]
            assert set(sm) == set(sr) and float(sm["step"]) == float(sr["step"])
            assert _close(sm["exp_avg"], sr["exp_avg"]) and _close(sm["exp_avg_sq"], sr["exp_avg_sq"])


def test_fused_adam_survives_densification_state_edits():
    """cat_tensors_to_optimizer / _prune_optimizer (gaussian_model.py) replace
    params and their exp_avg/exp_avg_sq in the state dict; the next step
    must use the new tensors (here: a pruned, non-16-B-aligned view too)."""
    ref, mine, o_ref, o_mine = _pair(1000, 2)
    for gr, gm in zip(ref, mine):
        gr["params"][0].grad = torch.ones_like(gr["params"][0]) * 0.1
        gm["params"][0].grad = torch.ones_like(gm["params"][0]) * 0.1
    o_ref.step()
    o_mine.step()
    keep = torch.arange(1000) % 3 != 0
    for o, dev in ((o_ref, "cpu"), (o_mine, DEV)):
        for grp in o.param_groups:
            old = grp["params"][0]
            st = o.state.pop(old)
            new = torch.nn.Parameter(old.detach()[keep.to(dev)].contiguous())
            st["exp_avg"] = st["exp_avg"][keep.to(dev)].contiguous()
            st["exp_avg_sq"] = st["exp_avg_sq"][keep.to(dev)].contiguous()
            grp["params"][0] = new
            o.state[new] = st
            new.grad = torch.full_like(new, -0.05)
    o_ref.step()
    o_mine.step()
    for gr, gm in zip(o_ref.param_groups, o_mine.param_groups):
        assert _close(gm["params"][0], gr["params"][0]), gr["name"]
    # an unaligned (offset-1) but contiguous parameter takes the scalar path
    base = torch.zeros(1001, device=DEV)
    p = torch.nn.Parameter(base[1:])
    o = gsr_optim.FusedAdam([p], lr=0.1)
    p.grad = torch.ones(1000, device=DEV)
    o.step()
    assert torch.allclose(p.detach(), torch.full((1000,), -0.1, device=DEV), rtol=1e-6)


def test_densify_stats_matches_reference_statements():
    P = 5003
    g = torch.Generator().manual_seed(3)
    vgrad = torch.randn(P, 3, generator=g)
    radii = torch.randint(-1, 4, (P,), generator=g, dtype=torch.int32)
    state = {k: torch.rand(P, 1, generator=g) for k in ("accum", "accum_abs", "denom")}
    max_r = torch.rand(P, generator=g) * 3
    # reference (train.py:236-237, gaussian_model.py:818-821), on CPU
    vis = radii > 0
    r_max = max_r.clone()
    r_max[vis] = torch.max(r_max[vis], radii[vis])
    r_acc, r_abs, r_den = state["accum"].clone(), state["accum_abs"].clone(), state["denom"].clone()
    r_acc[vis] += torch.norm(vgrad[vis, :2], dim=-1, keepdim=True)
    r_abs[vis] += torch.norm(vgrad[vis, 2:], dim=-1, keepdim=True)
    r_den[vis] += 1

    class G:
        pass

    gm = G()
    gm.max_radii2D = max_r.to(DEV)
    gm.xyz_gradient_accum, gm.xyz_gradient_accum_abs, gm.denom = (state[k].to(DEV) for k in ("accum", "accum_abs",
                                                                                               "denom"))
    vp = torch.zeros(P, 3, device=DEV, requires_grad=True)
    vp.grad = vgrad.to(DEV)
    gsr_optim.add_densification_stats(gm, vp, radii.to(DEV))
    assert torch.equal(gm.max_radii2D.cpu(), r_max)
    assert torch.equal(gm.denom.cpu(), r_den) and torch.equal(gm.xyz_gradient_accum_abs.cpu(), r_abs)
    assert torch.allclose(gm.xyz_gradient_accum.cpu(), r_acc, rtol=2e-7, atol=0)
