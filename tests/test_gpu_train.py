"""The training iteration's PatchMatch losses (gsr_train.patchmatch): the
sync-free masked means against the reference's boolean-gather means
(utils/loss_utils.py:140-267: ((weights * pixel_noise)[d_mask]).mean() and
(ncc * weights)[ncc_mask].mean()), values and gradients, on one small
synthetic scene; and one whole TrainStep runs with finite losses."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    import gsr_train
    step, view, nearest = gsr_train.synthetic_training_setup(20_000, 320, 240, device="cuda", seed=3)
    return gsr_train, step, view, nearest


def _grads(loss, params):
    return torch.autograd.grad(loss, params, retain_graph=True, allow_unused=True)


def test_patchmatch_masked_means_match_gathers(setup):
    gsr_train, step, view, nearest = setup
    from gaussian_renderer import render
    g = step.g
    pkg = render(view, g, step.pipe, step.bg, step.kernel_size, require_depth=True)
    t = gsr_train.patchmatch_terms(g, pkg, view, nearest, step.kernel_size, step.pipe)
    assert int(t["d_mask"].sum()) > 100 and int(t["ncc_mask"].sum()) > 100, "scene too sparse to test"
    geo_ref = ((t["weights"] * t["pixel_noise"])[t["d_mask"]]).mean()
    ncc_ref = (t["ncc"] * t["w_sel"])[t["ncc_mask"]].mean()
    geo = gsr_train.masked_mean(t["weights"] * t["pixel_noise"], t["d_mask"])
    ncc = gsr_train.masked_mean(t["ncc"] * t["w_sel"], t["ncc_mask"], empty=0.0)
    torch.testing.assert_close(geo, geo_ref, rtol=1e-5, atol=0.0)
    torch.testing.assert_close(ncc, ncc_ref, rtol=1e-5, atol=0.0)
    params = [g._xyz, g._opacity, g._scaling, g._rotation]
    for a, b in ((geo, geo_ref), (ncc, ncc_ref)):
        for ga, gb in zip(_grads(a, params), _grads(b, params)):
            assert (ga is None) == (gb is None)
            if ga is not None:
                assert torch.isfinite(ga).all()
                assert float((ga - gb).norm()) <= 1e-5 * float(gb.norm()) + 1e-12


def test_masked_mean_empty_mask():
    import gsr_train
    x = torch.randn(64, device="cuda", requires_grad=True)
    m = torch.zeros(64, dtype=torch.bool, device="cuda")
    assert torch.isnan(gsr_train.masked_mean(x, m))
    z = gsr_train.masked_mean(x, m, empty=0.0)
    assert float(z) == 0.0
    (gx,) = torch.autograd.grad(z, x)
    assert torch.equal(gx, torch.zeros_like(gx))


def test_patchmatch_empty_mask_returns_zero(setup):
    """No pixel passes d_mask (every median depth 0): the reference returns
    (0, 0) (utils/loss_utils.py:223-224); here both losses are 0, not NaN, and
    their gradients are zero."""
    gsr_train, step, view, nearest = setup
    from gaussian_renderer import render
    g = step.g
    pkg = render(view, g, step.pipe, step.bg, step.kernel_size, require_depth=True)
    pkg = dict(pkg, median_depth=pkg["median_depth"] * 0.0)
    from gsr_patchmatch import patchmatch_fused
    params = [g._xyz, g._opacity, g._scaling, g._rotation]
    for fn in (gsr_train.patchmatch, patchmatch_fused):
        ncc, geo = fn(g, pkg, view, nearest, step.kernel_size, step.pipe)
        assert float(ncc) == 0.0 and float(geo) == 0.0
        for ga in _grads(geo + ncc, params):
            assert ga is None or (torch.isfinite(ga).all() and float(ga.abs().max()) == 0.0)


def _rel(a, b):
    return float((a - b).norm()) / max(float(b.norm()), 1e-30)


def _close(a, b, name=""):
    """Gradient agreement for fp32-sensitive terms: relative L2 <= 1e-3 and
    99% of the entries within 1e-4 of the largest magnitude."""
    assert _rel(a, b) <= 1e-3, (name, _rel(a, b))
    tol = 1e-4 * float(b.abs().max())
    frac = float(((a - b).abs() <= tol).float().mean())
    assert frac >= 0.99, (name, frac)


def _pm_inputs(setup):
    gsr_train, step, view, nearest = setup
    from gaussian_renderer import render
    pkg = render(view, step.g, step.pipe, step.bg, step.kernel_size, require_depth=True)
    md = pkg["median_depth"].detach().requires_grad_(True)
    nrm = pkg["normal"].detach().requires_grad_(True)
    return gsr_train, step, view, nearest, dict(pkg, median_depth=md, normal=nrm), md, nrm


def test_fused_patchmatch_lift_matches_torch(setup):
    """The lift kernel against the reference's (md * ray - T) @ R^T
    (loss_utils.py:147-153): points and dL/dmd to fp32 rounding."""
    gsr_train, step, view, nearest, pkg, md, nrm = _pm_inputs(setup)
    import gsr_patchmatch as PM
    rays, _, _ = gsr_train._pixel_grids(view, md.device)
    ref = gsr_train._mat3(md.squeeze().unsqueeze(-1) * rays - view.T, view.R.T)
    got = PM._Lift.apply(md, view.T, view.R.T.contiguous(), (view.Fx, view.Fy, view.Cx, view.Cy))
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=1e-6 * float(ref.abs().max()))
    g = torch.randn_like(ref)
    assert _rel(torch.autograd.grad(got, md, g)[0], torch.autograd.grad(ref, md, g)[0]) <= 1e-6


def test_fused_patchmatch_geo_terms_match_torch(setup):
    """The terms kernel's geometric loss from one set of sampled points
    against the reference's reprojection, pairwise distance and masked mean
    (loss_utils.py:160-226): the loss to 1e-5 and dL/d(sampled point) to 1e-3
    relative L2 (99% of the pixels within 1e-4 of the largest) at the pixels
    whose reprojection error is >= 0.1 px.  The gradient's direction is that
    of proj - pixel + 1e-6 over its length: at a point that reprojects onto
    its own pixel (consistent median depths) that is the pairwise distance's
    eps plus fp32 rounding of a ~300 px coordinate (ulp 3e-5) in either
    formulation, and it converges as 1 / error — there only the count of such
    pixels and finiteness are compared."""
    gsr_train, step, view, nearest, pkg, md, nrm = _pm_inputs(setup)
    import gsr_patchmatch as PM
    from gaussian_renderer import sample_depth
    rays, pixels, pixels_f = gsr_train._pixel_grids(view, md.device)
    pts = gsr_train._mat3(md.detach().squeeze().unsqueeze(-1) * rays - view.T, view.R.T)
    smp = sample_depth(pts, nearest, step.g, step.pipe, step.kernel_size)
    pin = smp["sampled_depth"].detach().requires_grad_(True)
    inside = smp["inside"]
    with torch.no_grad():
        wv = view.world_view_transform
        tv = -wv[:3, :3].T @ nearest.R @ nearest.T + wv[3, :3]
        Mv = nearest.R.transpose(1, 0) @ wv[:3, :3]
    piv = tv + gsr_train._mat3(pin, Mv)
    proj = piv[..., :2] / torch.clamp_min(piv[..., 2:], 1e-7)
    proj = torch.addcmul(proj.new_tensor([view.Cx, view.Cy]), proj.new_tensor([view.Fx, view.Fy]), proj)
    noise = torch.pairwise_distance(proj, pixels_f)
    with torch.no_grad():
        dm = inside & (pin[..., -1] > 0.2) & (piv[..., -1] > 0.2) & (noise < 1.0) & (md.squeeze() > 0)
        w = torch.exp(-noise).masked_fill_(~dm, 0.0)
    ref = gsr_train.masked_mean(w * noise, dm, empty=0.0)
    got, _ = PM._Terms.apply(md, nrm, pin, inside, PM._Consts(view, nearest))
    assert int(dm.sum()) > 100
    assert abs(float(got) - float(ref)) <= 1e-5 * float(ref)
    (ga,) = torch.autograd.grad(got, pin)
    (gb,) = torch.autograd.grad(ref, pin)
    good = (noise >= 0.1) & dm
    assert int(good.sum()) > 100
    _close(ga[good], gb[good])
    kink = dm & ~good
    assert torch.isfinite(ga).all()
    assert int((ga[kink] != 0).any(-1).sum()) == int((gb[kink] != 0).any(-1).sum())
    assert not (ga[~dm] != 0).any()


def test_fused_patchmatch_ncc_matches_torch(setup):
    """The NCC loss on the full chain (lift, sample_depth, terms) against the
    reference's (gather, warp_patch_ncc, clamp, masked mean; loss_utils.py:
    228-262): the loss to 1e-4 relative and its gradients into the median
    depth and the rendered normals on the same pixels, 99% of them within 1e-4
    of the largest and 1e-3 relative L2 overall: the NCC's forward-mode
    derivatives divide by the plane's distance along the ray (ncc.hip), so the
    last-bit differences between torch's F.normalize and the kernel's (and
    between the compacted and the dense kernel's instruction schedules) reach
    ~3% at a few near-grazing pixels (measured: relative L2 1.9e-4, the top 10
    pixels 60% of it)."""
    gsr_train, step, view, nearest, pkg, md, nrm = _pm_inputs(setup)
    from gsr_patchmatch import patchmatch_fused
    g = step.g
    t = gsr_train.patchmatch_terms(g, pkg, view, nearest, step.kernel_size, step.pipe)
    assert int(t["ncc_mask"].sum()) > 100, "scene too sparse to test"
    ref = gsr_train.patchmatch(g, pkg, view, nearest, step.kernel_size, step.pipe)[0]
    got = patchmatch_fused(g, pkg, view, nearest, step.kernel_size, step.pipe)[0]
    assert float(ref) > 0.0
    assert abs(float(got) - float(ref)) <= 1e-4 * abs(float(ref)), (float(got), float(ref))
    for name, ga, gb in zip(["median_depth", "normal"], _grads(got, [md, nrm]), _grads(ref, [md, nrm])):
        assert torch.isfinite(ga).all(), name
        assert torch.equal(ga != 0, gb != 0), name
        _close(ga, gb, name)


def test_train_step_fused_and_torch_patchmatch_agree(setup):
    """One whole iteration's loss with either PatchMatch (fresh copies of the
    same Gaussians, so both start from the same state)."""
    import gsr_train
    out = []
    for fused in (True, False):
        step, view, nearest = gsr_train.synthetic_training_setup(20_000, 320, 240, device="cuda", seed=3)
        step = gsr_train.TrainStep(step.g, fused_patchmatch=fused)
        out.append(float(step.step(view, nearest)))
    assert abs(out[0] - out[1]) <= 1e-5 * abs(out[1]), out


def test_train_step_runs(setup):
    _, step, view, nearest = setup
    losses = [float(step.step(view, nearest)) for _ in range(2)]
    assert all(torch.isfinite(torch.tensor(losses)))


def test_mat3_and_rays_match_the_reference_products():
    """The broadcast forms of the PatchMatch glue equal the reference's cat and
    (H, W, 3) @ (3, 3) products (loss_utils.py:148-156) to fp32 rounding."""
    import gsr_train
    gen = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(48, 64, 3, generator=gen).cuda()
    M = torch.randn(3, 3, generator=gen).cuda()
    torch.testing.assert_close(gsr_train._mat3(x, M), x @ M, rtol=1e-6, atol=1e-6)
    from types import SimpleNamespace
    view = SimpleNamespace(image_width=64, image_height=48, Fx=50.0, Fy=52.0, Cx=31.5, Cy=23.5)
    rays, pixels, pixels_f = gsr_train._pixel_grids(view, torch.device("cuda"))
    depth = torch.rand(48, 64, 1, generator=gen).cuda()
    ix = (torch.arange(64, device="cuda", dtype=torch.float32) - view.Cx) / view.Fx
    iy = (torch.arange(48, device="cuda", dtype=torch.float32) - view.Cy) / view.Fy
    ref = torch.cat([depth * ix[None, :, None], depth * iy[:, None, None], depth], dim=-1)
    assert torch.equal(depth * rays, ref)
    assert pixels.dtype == torch.int32 and torch.equal(pixels[..., 0][0], torch.arange(64, device="cuda", dtype=torch.int32))
    assert torch.equal(pixels_f, pixels.float())


def test_fused_getters_match_torch(setup):
    """The fused activation getters (gsr_optim: scale / opacity with the 3D
    filter, get_rotation's normalisation) against the reference's torch
    expressions (gaussian_model.py:146-212): values to 2e-6 relative and
    their gradients for random upstream gradients to 1e-5 relative L2."""
    _, step, _, _ = setup
    g = step.g
    gen = torch.Generator(device="cuda").manual_seed(7)
    saved_filter = g.filter_3D.clone()
    # a filter of the scales' size (the synthetic scene's is zero: the f^2 terms would go unchecked)
    g.filter_3D.copy_(torch.exp(g._scaling.detach()).mean(1, keepdim=True)
                      * torch.rand(g.filter_3D.shape, device="cuda", generator=gen))
    try:
        _check_getters(g, gen)
    finally:
        g.filter_3D.copy_(saved_filter)


def _check_getters(g, gen):
    outs = {}
    for torch_getters in (True, False):
        g.torch_getters = torch_getters
        try:
            sc, op = g.get_scaling_n_opacity_with_3D_filter
            vals = [sc, op, g.get_scaling_with_3D_filter, g.get_opacity_with_3D_filter, g.get_rotation]
        finally:
            g.torch_getters = False
        outs[torch_getters] = vals
    ups = [torch.randn(v.shape, device="cuda", generator=gen) for v in outs[True]]
    for k, (a, b) in enumerate(zip(outs[False], outs[True])):
        torch.testing.assert_close(a, b, rtol=2e-6, atol=0.0, msg=f"getter {k}")
        leaves = [g._scaling, g._opacity, g._rotation]
        ga = torch.autograd.grad(a, leaves, ups[k], retain_graph=True, allow_unused=True)
        gb = torch.autograd.grad(b, leaves, ups[k], retain_graph=True, allow_unused=True)
        ga = [torch.zeros_like(lf) if x is None else x for x, lf in zip(ga, leaves)]  # (unused: None or zeros)
        gb = [torch.zeros_like(lf) if y is None else y for y, lf in zip(gb, leaves)]
        scale = max(float(y.norm()) for y in gb)
        for j, (x, y) in enumerate(zip(ga, gb)):
            assert float((x - y).norm()) <= 1e-5 * max(float(y.norm()), 1e-2 * scale), (k, j, _rel(x, y))


def test_split_sh_layout_matches_concatenated(setup):
    """The split SH layout (features_dc, features_rest handed to the
    rasterizer as a pair: gsr_rasterize_{forward,backward}_ex2) against the
    reference's concatenated get_features: images bit-identical, every
    gradient (the DC and rest rows against the two slices of the
    concatenated gradient) equal up to the float atomics' order."""
    gsr_train, step, view, nearest = setup
    from gaussian_renderer import render
    g = step.g
    class _Cat:  # the same model with the reference's concatenating get_features (all else delegated)
        def __getattr__(self, name):
            return getattr(g, name)

        @property
        def get_features(self):
            return torch.cat((g._features_dc, g._features_rest), dim=1)

    outs = {}
    for torch_getters, pc in ((True, _Cat()), (False, g)):
        pkg = render(view, pc, step.pipe, step.bg, step.kernel_size, require_depth=True)
        gen = torch.Generator(device="cuda").manual_seed(11)
        loss = (pkg["render"] * torch.randn(pkg["render"].shape, device="cuda", generator=gen)).sum() + \
            (pkg["median_depth"] * torch.randn(pkg["median_depth"].shape, device="cuda", generator=gen)).sum()
        leaves = [g._features_dc, g._features_rest, g._xyz, g._opacity]
        outs[torch_getters] = (pkg, torch.autograd.grad(loss, leaves))
    (pa, ga), (pb, gb) = outs[False], outs[True]
    for k in ("render", "median_depth", "normal", "mask"):
        assert torch.equal(pa[k], pb[k]), k
    for x, y in zip(ga, gb):  # (the accumulated dL/dcolour the SH rows derive from is summed by atomics)
        assert x.shape == y.shape and _rel(x, y) <= 1e-5, _rel(x, y)


def test_patchmatch_no_nearest_camera_and_inplace_losses(setup):
    """without a nearest camera both PatchMatch forms return the
    reference's two [1]-shaped zeros (utils/loss_utils.py:141-142); and the
    fused form's losses may be changed in place before the backward (they are
    not the tensor its backward saves)."""
    gsr_train, step, view, nearest = setup
    from gaussian_renderer import render
    from gsr_patchmatch import patchmatch_fused
    g = step.g
    pkg = render(view, g, step.pipe, step.bg, step.kernel_size, require_depth=True)
    for fn in (patchmatch_fused, gsr_train.patchmatch):
        ncc, geo = fn(g, pkg, view, None, step.kernel_size, step.pipe)
        assert ncc.shape == (1,) and geo.shape == (1,) and float(ncc) == 0.0 and float(geo) == 0.0
    ncc, geo = patchmatch_fused(g, pkg, view, nearest, step.kernel_size, step.pipe)
    ref = torch.autograd.grad(0.6 * ncc + 0.02 * geo, [g._xyz], retain_graph=True)[0]
    ncc, geo = patchmatch_fused(g, pkg, view, nearest, step.kernel_size, step.pipe)
    ncc *= 0.6
    geo *= 0.02
    got = torch.autograd.grad(ncc + geo, [g._xyz])[0]
    assert float((got - ref).norm()) <= 1e-6 * float(ref.norm()) + 1e-12
