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
    ncc, geo = gsr_train.patchmatch(g, pkg, view, nearest, None, step.kernel_size, step.pipe)
    assert float(ncc) == 0.0 and float(geo) == 0.0
    params = [g._xyz, g._opacity, g._scaling, g._rotation]
    for ga in _grads(geo + ncc, params):
        assert ga is None or (torch.isfinite(ga).all() and float(ga.abs().max()) == 0.0)


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
