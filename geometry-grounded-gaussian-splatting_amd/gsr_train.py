"""One training iteration of the reference after the regularisation kick-in
(train.py:142-262, iteration >= regularization_from_iter = 7000), on the HIP
kernels of this package: the end-to-end variant of SURVEY §8(d).

Per iteration, in the reference's order:
  getters (gaussian_model.py:146-212, torch)  -> render() with require_depth
  (gaussian_renderer.render -> GaussianRasterizer, render_fwd.hip)
  -> L1 (loss_utils.py:28-29; app_model NO)  -> depth_to_normal + normal loss
  (train.py:171-176; depth_normal.hip)  -> PatchMatch (loss_utils.py:140-267:
  the median-depth points re-observed from the nearest camera through
  sample_depth (sample.hip), the geometric loss, warp_patch_ncc (ncc.hip) on
  the consistent pixels)  -> fused SSIM (ssim.hip)  -> loss.backward()
  (render_bwd / preprocess_bwd / sample_bwd ...)  -> densification statistics
  (train.py:236-237, optim.hip)  -> Adam step + zero_grad (train.py:262-263,
  FusedAdam, optim.hip).
Out of the step, as in the reference's steady state: densify/prune (every 100
iterations until 15000), the 3D filter recomputation and logging.

The torch glue between the kernels (loss arithmetic, the PatchMatch
projections and masks) is the reference's own torch code restated; the hot
ops are the package's HIP kernels.  Synthetic data (no datasets here): the
ground-truth images are renders of a perturbed copy of the Gaussians.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

import gsr_scene as S
from fused_ssim import fused_ssim
from gaussian_renderer import render, sample_depth
from gsr_geometry import depth_to_normal
from gsr_optim import FusedAdam, add_densification_stats, normalize_rows, scaling_n_opacity_with_3D_filter
from gsr_patchmatch import patchmatch_fused
import warp_patch_ncc


@dataclass
class TrainView:
    """The attributes of scene/cameras.py::Camera a training iteration reads
    (R, T in the reference's convention: world_view_transform = [R^T | T]^T)."""

    image_width: int
    image_height: int
    FoVx: float
    FoVy: float
    world_view_transform: torch.Tensor
    full_proj_transform: torch.Tensor
    camera_center: torch.Tensor
    R: torch.Tensor
    T: torch.Tensor
    Fx: float
    Fy: float
    Cx: float
    Cy: float
    original_image: torch.Tensor | None = None
    gray_image: torch.Tensor | None = None


def train_view(W: int, H: int, R: np.ndarray, T: np.ndarray, device) -> TrainView:
    c = S.make_camera(W, H, R, T).to(device)
    Fx = W / (2 * math.tan(c.FoVx / 2.0))
    Fy = H / (2 * math.tan(c.FoVy / 2.0))
    return TrainView(W, H, c.FoVx, c.FoVy, c.world_view_transform, c.full_proj_transform, c.camera_center,
                     torch.tensor(R, dtype=torch.float32, device=device), torch.tensor(T, dtype=torch.float32,
                                                                                        device=device),
                     Fx, Fy, float(W - 1) / 2, float(H - 1) / 2)


def orbit_views(n: int, W: int, H: int, device, center_z: float = 6.0, max_deg: float = 20.0):
    """C4's orbit (gsr_scene.orbit_cameras) as training views."""
    views = []
    c = np.array([0.0, 0.0, center_z])
    for a in (np.linspace(-max_deg, max_deg, n) if n > 1 else np.zeros(1)):
        th = math.radians(float(a))
        Rc = np.array([[math.cos(th), 0, math.sin(th)], [0, 1, 0], [-math.sin(th), 0, math.cos(th)]])
        pos = c - Rc @ np.array([0.0, 0.0, center_z])
        views.append(train_view(W, H, Rc, -Rc.T @ pos, device))
    return views


class TrainGaussians(torch.nn.Module):
    """GaussianModel's trained state (gaussian_model.py): raw parameters,
    the 3D filter, Adam (FusedAdam with the reference's parameter groups and
    eps = 1e-15, gaussian_model.py:342-351) and the densification statistics."""

    def __init__(self, raw: S.RawGaussians, spatial_lr_scale: float = 1.0, sh_degree: int = 3, sg_degree: int = 0):
        super().__init__()
        P = lambda t: torch.nn.Parameter(t.detach().clone().contiguous())  # noqa: E731
        self._xyz, self._features_dc, self._features_rest = P(raw.xyz), P(raw.features_dc), P(raw.features_rest)
        self._scaling, self._rotation, self._opacity = P(raw.scaling), P(raw.rotation), P(raw.opacity)
        self._sg_axis, self._sg_sharpness, self._sg_color = P(raw.sg_axis), P(raw.sg_sharpness), P(raw.sg_color)
        self.register_buffer("filter_3D", raw.filter_3D.detach().clone())
        self.active_sh_degree, self.active_sg_degree = sh_degree, sg_degree
        self.torch_getters = False
        self._step_cache = None  # (TrainStep: the fused getters' outputs shared by render and sample_depth)
        n = raw.xyz.shape[0]
        dev = raw.xyz.device
        self.max_radii2D = torch.zeros(n, device=dev)
        self.xyz_gradient_accum = torch.zeros(n, 1, device=dev)
        self.xyz_gradient_accum_abs = torch.zeros(n, 1, device=dev)
        self.denom = torch.zeros(n, 1, device=dev)
        # OptimizationParams defaults (arguments/__init__.py:85-99)
        groups = [("xyz", self._xyz, 0.00016 * spatial_lr_scale), ("f_dc", self._features_dc, 0.0013),
                  ("f_rest", self._features_rest, 0.00011), ("opacity", self._opacity, 0.05),
                  ("scaling", self._scaling, 0.005), ("rotation", self._rotation, 0.001)]
        if raw.sg_color.shape[1]:
            groups += [("sg_axis", self._sg_axis, 0.002), ("sg_sharpness", self._sg_sharpness, 0.095),
                       ("sg_color", self._sg_color, 0.00064)]
        self.optimizer = FusedAdam([{"params": [p], "lr": lr, "name": nm} for nm, p, lr in groups], lr=0.0,
                                   eps=1e-15)

    # ---- getters (gaussian_model.py:146-212) ----
    def _cached(self, key, fn):
        # within a TrainStep (begin_step .. end_step) each fused getter runs once: render and the PatchMatch
        # sample_depth take the same outputs (the parameters do not change between them), so one kernel
        # each way instead of two or three, and the two consumers' gradients meet at the outputs
        c = self._step_cache
        if c is None:
            return fn()
        if key not in c:
            c[key] = fn()
        return c[key]

    def begin_step(self):
        self._step_cache = {}

    def end_step(self):
        self._step_cache = None

    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    # (the three 3D-filter getters and get_rotation on the fused kernels of gsr_optim; torch_getters=True
    # keeps the reference's torch expressions, which tests/test_gpu_train.py compares them with)
    @property
    def get_scaling_with_3D_filter(self):
        if not self.torch_getters:
            return self._cached("so", lambda: scaling_n_opacity_with_3D_filter(self._scaling, self._opacity, self.filter_3D))[0]
        return torch.sqrt(torch.square(self.get_scaling) + torch.square(self.filter_3D))

    @property
    def get_opacity_with_3D_filter(self):
        if not self.torch_getters:
            return self._cached("so", lambda: scaling_n_opacity_with_3D_filter(self._scaling, self._opacity, self.filter_3D))[1]
        sq = torch.square(self.get_scaling)
        coef = torch.sqrt(sq.prod(dim=1) / (sq + torch.square(self.filter_3D)).prod(dim=1))
        return torch.sigmoid(self._opacity) * coef[..., None]

    @property
    def get_scaling_n_opacity_with_3D_filter(self):
        if not self.torch_getters:
            return self._cached("so", lambda: scaling_n_opacity_with_3D_filter(self._scaling, self._opacity, self.filter_3D))
        sq = torch.square(self.get_scaling)
        after = sq + torch.square(self.filter_3D)
        coef = sq.prod(dim=1).sqrt() * after.prod(dim=1).rsqrt()
        return after.sqrt(), torch.sigmoid(self._opacity) * coef[..., None]

    @property
    def get_rotation(self):
        if not self.torch_getters:
            return self._cached("rot", lambda: normalize_rows(self._rotation))
        return F.normalize(self._rotation)

    @property
    def get_features(self):
        # the pair as GaussianModel keeps it: GaussianRasterizer takes the split SH layout without the
        # concatenation (192 MB at 1M Gaussians, and the gradient's split); torch_getters: the reference's cat
        if not self.torch_getters:
            return self._features_dc, self._features_rest
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_sg_axis(self):
        return F.normalize(self._sg_axis, dim=2)

    @property
    def get_sg_sharpness(self):
        return F.softplus(self._sg_sharpness)

    @property
    def get_sg_color(self):
        return self._sg_color


class _Pipe:
    debug = False
    compute_cov3D_python = False


# loss weights and PatchMatch settings (arguments/__init__.py:106-118)
LAMBDA_DSSIM, LAMBDA_DEPTH_NORMAL, LAMBDA_NCC, LAMBDA_GEO = 0.2, 0.05, 0.6, 0.02
PATCH_SIZE, PIXEL_NOISE_TH = 3, 1.0


_GRIDS: dict = {}


def _pixel_grids(view, dev):
    """Per camera (cached): the rays (ix, iy, 1) of the reference's pixel
    grid (loss_utils.py:148-152), and its (H, W, 2) int32 / float pixel
    coordinates."""
    key = (view.image_width, view.image_height, view.Fx, view.Fy, view.Cx, view.Cy, str(dev))
    if key not in _GRIDS:
        W, H = view.image_width, view.image_height
        ix = (torch.arange(W, device=dev, dtype=torch.float32) - view.Cx) / view.Fx
        iy = (torch.arange(H, device=dev, dtype=torch.float32) - view.Cy) / view.Fy
        rays = torch.stack([ix[None, :].expand(H, W), iy[:, None].expand(H, W), torch.ones(H, W, device=dev)], -1)
        gx, gy = torch.meshgrid(torch.arange(W, device=dev, dtype=torch.int32),
                                torch.arange(H, device=dev, dtype=torch.int32), indexing="xy")
        pixels = torch.stack([gx, gy], dim=-1)
        if len(_GRIDS) > 8:
            _GRIDS.clear()
        _GRIDS[key] = (rays.contiguous(), pixels, pixels.float())
    return _GRIDS[key]


def _mat3(x: torch.Tensor, M: torch.Tensor) -> torch.Tensor:
    """x @ M for x [..., 3] and a 3x3 M, as three broadcast multiply-adds."""
    return torch.addcmul(torch.addcmul(x[..., 0:1] * M[0], x[..., 1:2], M[1]), x[..., 2:3], M[2])


def patchmatch_terms(gaussians, render_pkg, view, nearest, kernel_size, pipe) -> dict:
    """PatchMatch.__call__ (utils/loss_utils.py:140-267) without its debug
    image dumps, up to its two masked means: the median-depth points of `view`
    re-observed from `nearest` (sample_depth), the per-pixel reprojection error
    and weights of the geometric loss with its mask, and the multi-view NCC of
    7x7 half-step patches (warp_patch_ncc) at the consistent pixels with its
    weights and mask."""
    dev = render_pkg["median_depth"].device
    rays, pixels, pixels_f = _pixel_grids(view, dev)
    with torch.no_grad():
        view_to_nearest_T = (-view.world_view_transform[:3, :3].T @ nearest.R @ nearest.T
                             + view.world_view_transform[3, :3])
        nearest_to_view_R = nearest.R.transpose(1, 0) @ view.world_view_transform[:3, :3]
    depth_reshape = render_pkg["median_depth"].squeeze().unsqueeze(-1)
    # (the reference's cat of depth * (ix, iy, 1) and its two (H, W, 3) @ (3, 3) products; as broadcast
    # multiply-adds — a K = 3 matmul took a 130-us library GEMM each way)
    pts = _mat3(depth_reshape * rays - view.T, view.R.T)
    sampled = sample_depth(pts, nearest, gaussians, pipe, kernel_size)
    pts_in_nearest = sampled["sampled_depth"]
    pts_in_view = view_to_nearest_T + _mat3(pts_in_nearest, nearest_to_view_R)
    proj = pts_in_view[..., :2] / torch.clamp_min(pts_in_view[..., 2:], 1e-7)
    proj = torch.addcmul(proj.new_tensor([view.Cx, view.Cy]), proj.new_tensor([view.Fx, view.Fy]), proj)
    pixel_noise = torch.pairwise_distance(proj, pixels_f)
    with torch.no_grad():
        d_mask = (sampled["inside"] & (pts_in_nearest[..., -1] > 0.2) & (pts_in_view[..., -1] > 0.2)
                  & (pixel_noise < PIXEL_NOISE_TH) & (render_pkg["median_depth"].squeeze() > 0))
        weights = torch.exp(-pixel_noise).masked_fill_(~d_mask, 0.0)
    with torch.no_grad():
        d_flat = torch.flatten(d_mask)
        valid = torch.argwhere(d_flat).squeeze(1)
        w_sel = torch.flatten(weights)[valid]
        px = torch.index_select(pixels.view(-1, 2), dim=0, index=valid)
        r_rel = nearest.world_view_transform[:3, :3].transpose(-1, -2) @ view.world_view_transform[:3, :3]
        t_rel = -r_rel @ view.world_view_transform[3, :3] + nearest.world_view_transform[3, :3]
    depth_sel = torch.index_select(render_pkg["median_depth"].view(-1), dim=0, index=valid)
    normal_sel = F.normalize(torch.index_select(render_pkg["normal"].view(3, -1), dim=1, index=valid).T, dim=-1)
    cc, valid_mask = warp_patch_ncc.warp_patch_ncc(
        depth_sel, normal_sel, px, r_rel.T, t_rel, view.gray_image.squeeze(), nearest.gray_image.squeeze(),
        view.Fx, view.Fy, view.Cx, view.Cy, nearest.Fx, nearest.Fy, nearest.Cx, nearest.Cy, False)
    ncc = torch.clamp(1 - cc, 0.0, 2.0)
    ncc_mask = (ncc < 0.9) & valid_mask
    return {"pixel_noise": pixel_noise, "weights": weights, "d_mask": d_mask, "ncc": ncc.squeeze(), "w_sel": w_sel,
            "ncc_mask": ncc_mask.squeeze()}


def masked_mean(x: torch.Tensor, mask: torch.Tensor, empty: float | None = None) -> torch.Tensor:
    """x[mask].mean() without the boolean gather's device-to-host sync: the
    masked sum over the mask's count (NaN for an empty mask as the gather's
    mean, or `empty` when given).  Same value up to summation order, same
    gradient (mask / count on the selected entries)."""
    cnt = mask.sum()
    mean = torch.where(mask, x, torch.zeros((), device=x.device, dtype=x.dtype)).sum() / cnt
    return mean if empty is None else torch.where(cnt > 0, mean, torch.full_like(mean, empty))


def patchmatch(gaussians, render_pkg, view, nearest, kernel_size, pipe):
    """PatchMatch.__call__ (utils/loss_utils.py:140-267): (ncc_loss, geo_loss).
    The reference's means over boolean gathers ((weights * pixel_noise)[d_mask],
    (ncc * weights)[ncc_mask]) are taken as masked sums (`masked_mean`), so the
    only host synchronisation left is the valid-pixel count warp_patch_ncc
    needs (tests/test_gpu_train.py checks both forms agree)."""
    if nearest is None:  # loss_utils.py:141-142
        z = lambda: torch.zeros(1, dtype=torch.float32, device=render_pkg["median_depth"].device)  # noqa: E731
        return z(), z()
    t = patchmatch_terms(gaussians, render_pkg, view, nearest, kernel_size, pipe)
    # The reference returns (0, 0) when no pixel passes d_mask (loss_utils.py:223-224) and its NCC mean is
    # over a non-empty set otherwise; the mean of an empty set would be NaN, so both means take empty=0.
    geo_loss = masked_mean(t["weights"] * t["pixel_noise"], t["d_mask"], empty=0.0)
    ncc_loss = masked_mean(t["ncc"] * t["w_sel"], t["ncc_mask"], empty=0.0)
    return ncc_loss, geo_loss


class TrainStep:
    """The iteration; `step(view, nearest)` runs it, `stamps` (when timing)
    holds CUDA events at the component boundaries of the last call."""

    COMPONENTS = ("render", "depth_normal", "patchmatch", "rgb_loss", "backward", "densify_stats", "adam")

    def __init__(self, gaussians: TrainGaussians, kernel_size: float = 0.0, bg=None, densify: bool = True,
                 fused_patchmatch: bool = True):
        self.g = gaussians
        # PatchMatch on the fused kernels (gsr_patchmatch), or the reference's torch formulation (patchmatch)
        self.patchmatch = patchmatch_fused if fused_patchmatch else patchmatch
        self.kernel_size = kernel_size
        dev = gaussians._xyz.device
        self.bg = torch.zeros(3, device=dev) if bg is None else bg
        self.pipe = _Pipe()
        self.densify = densify
        self.timing = False
        self.stamps = []

    def _mark(self):
        if self.timing:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.stamps.append(e)

    def step(self, view: TrainView, nearest: TrainView) -> torch.Tensor:
        g = self.g
        self.stamps = []
        self._mark()
        g.begin_step()
        try:
            return self._step(g, view, nearest)
        finally:
            g.end_step()

    def _step(self, g, view, nearest):
        pkg = render(view, g, self.pipe, self.bg, self.kernel_size, require_depth=True)
        image = pkg["render"]
        self._mark()
        depth_normal, valid_points = depth_to_normal(view, pkg["median_depth"])
        err = 1 - torch.linalg.vecdot(pkg["normal"], depth_normal, dim=0)
        normal_loss = torch.where(valid_points.squeeze(), err, 0.0).mean()  # (a scalar 0: no zero-filled map)
        self._mark()
        ncc_loss, geo_loss = self.patchmatch(g, pkg, view, nearest, self.kernel_size, self.pipe)
        self._mark()
        gt = view.original_image
        l1 = torch.abs(image - gt).mean()
        rgb_loss = (1.0 - LAMBDA_DSSIM) * l1 + LAMBDA_DSSIM * (1.0 - fused_ssim(image.unsqueeze(0), gt.unsqueeze(0),
                                                                                 padding="valid"))
        loss = rgb_loss + LAMBDA_DEPTH_NORMAL * normal_loss + LAMBDA_NCC * ncc_loss + LAMBDA_GEO * geo_loss
        self._mark()
        loss.backward()
        self._mark()
        with torch.no_grad():
            if self.densify:  # train.py:236-237 (iterations < densify_until_iter)
                add_densification_stats(g, pkg["viewspace_points"], pkg["radii"])
            self._mark()
            g.optimizer.step()
            g.optimizer.zero_grad(set_to_none=True)
        self._mark()
        return loss.detach()

    def component_ms(self) -> dict:
        """Milliseconds per component of the last timed step (synchronises)."""
        torch.cuda.synchronize()
        e = self.stamps
        return {name: e[k].elapsed_time(e[k + 1]) for k, name in enumerate(self.COMPONENTS)}


def synthetic_training_setup(P: int, W: int, H: int, sh_degree: int = 3, sg_degree: int = 0, device="cuda",
                             seed: int = 0):
    """(TrainStep, view, nearest view): the bench scene's Gaussians as the
    trained state, two orbit views 5.7 degrees apart, and ground-truth images
    rendered from a copy of the Gaussians with perturbed colours and positions."""
    raw = S.make_gaussians(P, sh_degree=sh_degree, sg_degree=sg_degree, seed=seed, aspect=H / W).to(device)
    views = orbit_views(8, W, H, device)
    view, nearest = views[3], views[4]
    gen = torch.Generator(device="cpu").manual_seed(seed + 1)
    gt_raw = S.RawGaussians(*[getattr(raw, f).clone() for f in raw.__dataclass_fields__])
    gt_raw.features_dc += (torch.randn(gt_raw.features_dc.shape, generator=gen) * 0.1).to(device)
    gt_raw.xyz += (torch.randn(gt_raw.xyz.shape, generator=gen) * 0.01).to(device)
    gt = TrainGaussians(gt_raw, sh_degree=sh_degree, sg_degree=sg_degree)
    with torch.no_grad():
        for v in (view, nearest):
            img = render(v, gt, _Pipe(), torch.zeros(3, device=device), 0.0, require_depth=False)["render"]
            v.original_image = img.clamp(0.0, 1.0).contiguous()
            v.gray_image = (0.299 * img[0] + 0.587 * img[1] + 0.114 * img[2])[None].contiguous()
    del gt
    return TrainStep(TrainGaussians(raw, sh_degree=sh_degree, sg_degree=sg_degree)), view, nearest
