"""ctypes front end of the CPU oracle (gsr_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product never does.  It mirrors the two entry points
of the reference extension (DGR/rasterize_points.cu:39-258):

  forward(...)  -> dict(color, alpha, normal, mdepth, radii, num_rendered, state)
  backward(...) -> dict(dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh,
                        dsg_axis, dsg_sharpness, dsg_color, dscales, drotations)

All arrays are float32/int32 numpy arrays (torch CPU tensors are accepted and
converted).  Outputs are allocated zero-filled like torch::full / torch::zeros.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libgsr_oracle.so")
_lib = None

_f = ctypes.POINTER(ctypes.c_float)
_i = ctypes.POINTER(ctypes.c_int)
_u32 = ctypes.POINTER(ctypes.c_uint32)
_u64 = ctypes.POINTER(ctypes.c_uint64)
_u8 = ctypes.POINTER(ctypes.c_uint8)
_d = ctypes.POINTER(ctypes.c_double)


def build() -> str:
    """Compile the oracle with its Makefile (gcc) if needed."""
    src = os.path.join(_HERE, "gsr_oracle.c")
    if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        L.gsro_forward.restype = ctypes.c_void_p
        L.gsro_forward.argtypes = (
            [ctypes.c_int] * 5 + [_f, ctypes.c_int, ctypes.c_int] + [_f] * 10 + [ctypes.c_float] + [_f] * 3
            + [ctypes.c_float] * 3 + [ctypes.c_int] + [_f] * 4 + [_i, ctypes.c_int, _i])
        L.gsro_backward.restype = ctypes.c_int
        L.gsro_backward.argtypes = (
            [ctypes.c_void_p] + [_f] * 11 + [ctypes.c_float] + [_f] * 3 + [ctypes.c_float] * 3 + [_i]
            + [_f] * 7 + [_f] * 11)
        L.gsro_free.argtypes = [ctypes.c_void_p]
        L.gsro_set_threads.argtypes = [ctypes.c_int]
        L.gsro_set_tile_stride.argtypes = [ctypes.c_int]
        L.gsro_last_times.argtypes = [_d]
        L.gsro_eval_color.argtypes = [ctypes.c_int] * 4 + [_f] * 6 + [_f, _u8]
        L.gsro_max_threads.restype = ctypes.c_int
        L.gsro_higher_msb.argtypes = [ctypes.c_uint32]
        L.gsro_higher_msb.restype = ctypes.c_uint32
        L.gsro_mark_visible.argtypes = [ctypes.c_int, _f, _f, _u8]
        L.gsro_num_rendered.argtypes = [ctypes.c_void_p]
        L.gsro_num_rendered.restype = ctypes.c_int
        L.gsro_get_geometry.argtypes = [ctypes.c_void_p, _f, _f, _f, _f, _f, _f, _u32, _u8]
        L.gsro_get_binning.argtypes = [ctypes.c_void_p, _u64, _u32]
        L.gsro_get_tiles.argtypes = [ctypes.c_void_p, _u32, _u32]
        L.gsro_get_n_contrib.argtypes = [ctypes.c_void_p, _u32]
        L.gsro_set_n_contrib.argtypes = [ctypes.c_void_p, _u32]
        L.gsro_set_exp_mode.argtypes = [ctypes.c_int]
        L.gsro_get_bwd_accum.argtypes = [ctypes.c_void_p, _d, _d, _d]
        L.gsro_sample_forward.restype = ctypes.c_void_p
        L.gsro_sample_forward.argtypes = ([ctypes.c_int] * 4 + [_f] * 4 + [ctypes.c_float] + [_f] * 5
                                          + [ctypes.c_float] * 3 + [_f, _u8, _i, _i, _i])
        L.gsro_sample_backward.restype = ctypes.c_int
        L.gsro_sample_backward.argtypes = ([ctypes.c_void_p] + [_f] * 4 + [ctypes.c_float] + [_f] * 4
                                           + [ctypes.c_float] * 3 + [_u8, _f] + [_f] * 6)
        L.gsro_sample_free.argtypes = [ctypes.c_void_p]
        L.gsro_sample_set_median_depth.argtypes = [ctypes.c_void_p, _f]
        L.gsro_sample_get_points.argtypes = [ctypes.c_void_p, _f, _u32, _u32, _f]
        L.gsro_warp_patch_ncc.argtypes = ([ctypes.c_int, _f, _f, _i, _f, _f, _f, _f] + [ctypes.c_float] * 8
                                          + [ctypes.c_int] * 4 + [_f, _f, _f, _u8])
        L.gsro_point_query.restype = ctypes.c_int
        L.gsro_point_query.argtypes = ([ctypes.c_int] * 5 + [_f] * 4 + [ctypes.c_float] + [_f] * 5
                                       + [ctypes.c_float] * 3 + [_f, _f, _u8, _i])
        L.gsro_knn_mean_dist.restype = ctypes.c_int
        L.gsro_knn_mean_dist.argtypes = [ctypes.c_int, _f, _f, _u32]
        L.gsro_cov3d.argtypes = [ctypes.c_int, _f, ctypes.c_float, _f, _f]
        L.gsro_cov3d_bwd.argtypes = [ctypes.c_int, _f, ctypes.c_float, _f, _f, _f, _f]
        L.gsro_sample_gaussians.restype = ctypes.c_void_p
        L.gsro_sample_gaussians.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


def set_threads(n: int) -> None:
    lib().gsro_set_threads(int(n))


def set_exp_mode(mode: int) -> None:
    """1 (default): exp2f(x * log2e) in fp32, the form the reference's
    --use_fast_math build compiles expf to; 0: libm expf (gsr_oracle.c header)."""
    lib().gsro_set_exp_mode(int(mode))


def set_tile_stride(n: int) -> None:
    """Bounded-sample mode: render/backpropagate only every n-th tile."""
    lib().gsro_set_tile_stride(int(n))


def last_times() -> dict:
    """Seconds spent in the last forward/backward: per-Gaussian + binning,
    tile render, backward tile render, per-Gaussian backward."""
    t = np.zeros(4)
    lib().gsro_last_times(_p(t, _d))
    return dict(preprocess_binning=t[0], render=t[1], render_bwd=t[2], preprocess_bwd=t[3])


def max_threads() -> int:
    return lib().gsro_max_threads()


def _np(x, dtype=np.float32):
    if x is None:
        return None
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    a = np.ascontiguousarray(np.asarray(x, dtype=dtype))
    return None if a.size == 0 else a


def _p(a, ty=_f):
    return None if a is None else a.ctypes.data_as(ty)


class State:
    """Owns the oracle's forward state (geometry/binning/tile/image buffers)."""

    def __init__(self, ptr, P, W, H, K):
        self.ptr, self.P, self.W, self.H, self.K = ptr, P, W, H, K

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None and not hasattr(self, "_borrowed_from"):
            _lib.gsro_free(self.ptr)
        self.ptr = None

    @property
    def tiles(self):
        return ((self.W + 15) // 16) * ((self.H + 15) // 16)

    def geometry(self) -> dict:
        P = self.P
        out = dict(depths=np.zeros(P, np.float32), means2D=np.zeros((P, 2), np.float32),
                   conic_opacity=np.zeros((P, 4), np.float32), rgb=np.zeros((P, 3), np.float32),
                   ray_planes=np.zeros((P, 4), np.float32), normals=np.zeros((P, 3), np.float32),
                   tiles_touched=np.zeros(P, np.uint32), clamped=np.zeros((P, 3), np.uint8))
        lib().gsro_get_geometry(self.ptr, _p(out["depths"]), _p(out["means2D"]), _p(out["conic_opacity"]),
                                _p(out["rgb"]), _p(out["ray_planes"]), _p(out["normals"]),
                                _p(out["tiles_touched"], _u32), _p(out["clamped"], _u8))
        return out

    def binning(self) -> dict:
        keys = np.zeros(self.K, np.uint64)
        plist = np.zeros(self.K, np.uint32)
        lib().gsro_get_binning(self.ptr, _p(keys, _u64), _p(plist, _u32))
        return dict(keys=keys, point_list=plist)

    def tile_state(self) -> dict:
        ranges = np.zeros((self.tiles, 2), np.uint32)
        mc = np.zeros(self.tiles, np.uint32)
        lib().gsro_get_tiles(self.ptr, _p(ranges, _u32), _p(mc, _u32))
        return dict(ranges=ranges, max_contributor=mc)

    def n_contrib(self) -> np.ndarray:
        n = np.zeros(self.W * self.H, np.uint32)
        lib().gsro_get_n_contrib(self.ptr, _p(n, _u32))
        return n.reshape(self.H, self.W)

    def set_n_contrib(self, n_contrib) -> None:
        """Make the backward run with these per-pixel last contributors
        (positions in THIS state's per-tile lists; per-tile max recomputed)."""
        n = np.ascontiguousarray(np.asarray(n_contrib, np.uint32).reshape(-1))
        assert n.size == self.W * self.H
        lib().gsro_set_n_contrib(self.ptr, _p(n, _u32))

    def bwd_accum(self) -> dict:
        P = self.P
        out = dict(conic=np.zeros((P, 4)), ray_plane=np.zeros((P, 4)), normal=np.zeros((P, 3)))
        lib().gsro_get_bwd_accum(self.ptr, _p(out["conic"], _d), _p(out["ray_plane"], _d), _p(out["normal"], _d))
        return out


def forward(bg, means3D, colors_precomp, opacities, scales, rotations, cov3D_precomp, sh, sg_axis, sg_sharpness,
            sg_color, sh_degree, sg_degree, scale_modifier, viewmatrix, projmatrix, tan_fovx, tan_fovy,
            kernel_size, image_height, image_width, campos, prefiltered=False, require_depth=True) -> dict:
    """Same argument list as _C.rasterize_gaussians (DGR/rasterize_points.h:18-43)."""
    L = lib()
    means3D = _np(means3D)
    P = 0 if means3D is None else means3D.shape[0]
    sh_a = _np(sh)
    sgc = _np(sg_color)
    SHM = 0 if sh_a is None else sh_a.shape[1]
    SGM = 0 if sgc is None else sgc.shape[1]
    H, W = int(image_height), int(image_width)
    color = np.zeros((3, H, W), np.float32)
    mdepth = np.zeros((1, H, W), np.float32)
    alpha = np.zeros((1, H, W), np.float32)
    normal = np.zeros((3, H, W), np.float32)
    radii = np.zeros(P, np.int32)
    K = ctypes.c_int(0)
    keep = [_np(bg), means3D, _np(colors_precomp), _np(opacities), _np(scales), _np(rotations), _np(cov3D_precomp),
            sh_a, _np(sg_axis), _np(sg_sharpness), sgc, _np(viewmatrix), _np(projmatrix), _np(campos)]
    if P == 0:
        return dict(num_rendered=0, color=color, alpha=alpha, normal=normal, mdepth=mdepth, radii=radii, state=None)
    ptr = L.gsro_forward(P, int(sh_degree), SHM, int(sg_degree), SGM, _p(keep[0]), W, H, _p(keep[1]), _p(keep[2]),
                         _p(keep[3]), _p(keep[4]), _p(keep[5]), _p(keep[6]), _p(keep[7]), _p(keep[8]), _p(keep[9]),
                         _p(keep[10]), float(scale_modifier), _p(keep[11]), _p(keep[12]), _p(keep[13]),
                         float(tan_fovx), float(tan_fovy), float(kernel_size), int(bool(prefiltered)), _p(color),
                         _p(mdepth), _p(alpha), _p(normal), _p(radii, _i), int(bool(require_depth)),
                         ctypes.byref(K))
    st = State(ptr, P, W, H, K.value)
    return dict(num_rendered=K.value, color=color, alpha=alpha, normal=normal, mdepth=mdepth, radii=radii,
                state=st)


def backward(state: State, bg, means3D, colors_precomp, opacities, scales, rotations, cov3D_precomp, sh, sg_axis,
             sg_sharpness, sg_color, sh_degree, sg_degree, scale_modifier, viewmatrix, projmatrix, tan_fovx,
             tan_fovy, kernel_size, dL_dcolor, dL_dmdepth, dL_dalpha, dL_dnormal, alpha, normal, mdepth, campos,
             radii) -> dict:
    """Same meaning as _C.rasterize_gaussians_backward (DGR/rasterize_points.h:45-80)."""
    L = lib()
    means3D = _np(means3D)
    P = means3D.shape[0]
    sh_a = _np(sh)
    sgc = _np(sg_color)
    SHM = 0 if sh_a is None else sh_a.shape[1]
    SGM = 0 if sgc is None else sgc.shape[1]
    out = dict(dmeans2D=np.zeros((P, 3), np.float32), dcolors=np.zeros((P, 3), np.float32),
               dopacity=np.zeros((P, 1), np.float32), dmeans3D=np.zeros((P, 3), np.float32),
               dcov3D=np.zeros((P, 6), np.float32), dsh=np.zeros((P, SHM, 3), np.float32),
               dsg_axis=np.zeros((P, SGM, 3), np.float32), dsg_sharpness=np.zeros((P, SGM), np.float32),
               dsg_color=np.zeros((P, SGM, 3), np.float32), dscales=np.zeros((P, 3), np.float32),
               drotations=np.zeros((P, 4), np.float32))
    if P == 0 or state is None:
        return out
    keep = [_np(bg), means3D, _np(colors_precomp), _np(opacities), _np(scales), _np(rotations), _np(cov3D_precomp),
            sh_a, _np(sg_axis), _np(sg_sharpness), sgc, _np(viewmatrix), _np(projmatrix), _np(campos),
            _np(radii, np.int32), _np(alpha), _np(normal), _np(mdepth), _np(dL_dcolor), _np(dL_dmdepth),
            _np(dL_dalpha), _np(dL_dnormal)]
    zeros_hw = np.zeros(state.W * state.H * 3, np.float32)
    for k in (15, 16, 17, 18, 19, 20, 21):  # never pass NULL pixel planes
        if keep[k] is None:
            keep[k] = zeros_hw
    rc = L.gsro_backward(state.ptr, _p(keep[0]), _p(keep[1]), _p(keep[2]), _p(keep[3]), _p(keep[4]), _p(keep[5]),
                         _p(keep[6]), _p(keep[7]), _p(keep[8]), _p(keep[9]), _p(keep[10]), float(scale_modifier),
                         _p(keep[11]), _p(keep[12]), _p(keep[13]), float(tan_fovx), float(tan_fovy),
                         float(kernel_size), _p(keep[14], _i), _p(keep[15]), _p(keep[16]), _p(keep[17]),
                         _p(keep[18]), _p(keep[19]), _p(keep[20]), _p(keep[21]), _p(out["dmeans3D"]),
                         _p(out["dmeans2D"]), _p(out["dcolors"]), _p(out["dopacity"]), _p(out["dscales"]),
                         _p(out["drotations"]), _p(out["dcov3D"]), _p(out["dsh"]), _p(out["dsg_axis"]),
                         _p(out["dsg_sharpness"]), _p(out["dsg_color"]))
    if rc != 0:
        raise RuntimeError(f"oracle backward failed: {rc}")
    return out


def mark_visible(means3D, viewmatrix) -> np.ndarray:
    m = _np(means3D)
    P = 0 if m is None else m.shape[0]
    out = np.zeros(P, np.uint8)
    if P:
        lib().gsro_mark_visible(P, _p(m), _p(_np(viewmatrix)), _p(out, _u8))
    return out.astype(bool)


def eval_color(D, mean, campos, sh, sg_axis=None, sg_sharpness=None, sg_color=None, sgd=0):
    """Colour of one Gaussian: sh [SHM,3], sg_* [SGM,3]/[SGM]. Returns (rgb, clamped)."""
    sh = np.ascontiguousarray(sh, np.float32)
    SHM = sh.shape[0]
    SGM = 0 if sg_color is None else np.asarray(sg_color).shape[0]
    rgb = np.zeros(3, np.float32)
    cl = np.zeros(3, np.uint8)
    m, c = np.ascontiguousarray(mean, np.float32), np.ascontiguousarray(campos, np.float32)
    ax = None if sg_axis is None else np.ascontiguousarray(sg_axis, np.float32)
    shp = None if sg_sharpness is None else np.ascontiguousarray(sg_sharpness, np.float32)
    col = None if sg_color is None else np.ascontiguousarray(sg_color, np.float32)
    lib().gsro_eval_color(int(D), SHM, int(sgd), SGM, _p(m), _p(c), _p(sh), _p(ax), _p(shp), _p(col), _p(rgb),
                          _p(cl, _u8))
    return rgb, cl.astype(bool)


def higher_msb(n: int) -> int:
    return int(lib().gsro_higher_msb(int(n)))


class SampleState:
    """Owns the oracle's sample_depth state (Gaussian binning + per-point results)."""

    def __init__(self, ptr, P, PN, W, H, K):
        self.ptr, self.P, self.PN, self.W, self.H, self.K = ptr, P, PN, W, H, K

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.gsro_sample_free(self.ptr)
            self.ptr = None

    def points(self) -> dict:
        PN = self.PN
        out = dict(points2D=np.zeros((PN, 2), np.float32), tile=np.zeros(PN, np.uint32),
                   n_contrib=np.zeros(PN, np.uint32), median_depth=np.zeros(PN, np.float32))
        lib().gsro_sample_get_points(self.ptr, _p(out["points2D"]), _p(out["tile"], _u32),
                                     _p(out["n_contrib"], _u32), _p(out["median_depth"]))
        return out

    def set_median_depth(self, md) -> None:
        """Make the backward use these per-point median depths (e.g. the GPU forward's)."""
        md = np.ascontiguousarray(np.asarray(md, np.float32).reshape(-1))
        assert md.size == self.PN
        lib().gsro_sample_set_median_depth(self.ptr, _p(md))

    def gaussians(self) -> State:
        """The Gaussian side as a borrowed State (binning, geometry accessors)."""
        st = State.__new__(State)
        st.ptr, st.P, st.W, st.H, st.K = lib().gsro_sample_gaussians(self.ptr), self.P, self.W, self.H, self.K
        st._borrowed_from = self
        return st


def sample_forward(points3D, means3D, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
                   projmatrix, tan_fovx, tan_fovy, kernel_size, image_height, image_width, campos,
                   prefiltered=False) -> dict:
    """Same argument list as _C.sample_rasterized_depth (DGR/rasterize_points.cu:459-476)."""
    L = lib()
    pts = _np(points3D)
    shape = tuple(points3D.shape) if hasattr(points3D, "shape") else np.asarray(points3D).shape
    PN = 0 if pts is None else pts.size // 3
    means3D = _np(means3D)
    P = 0 if means3D is None else means3D.shape[0]
    H, W = int(image_height), int(image_width)
    output = np.zeros(shape, np.float32)
    inside = np.zeros(shape[:-1], np.uint8)
    if P == 0 or PN == 0:
        return dict(num_rendered=0, num_points=0, num_duplicated_tiles=0, output=output, inside=inside.astype(bool),
                    state=None)
    keep = [pts, means3D, _np(opacity), _np(scales), _np(rotations), _np(cov3D_precomp), _np(viewmatrix),
            _np(projmatrix), _np(campos)]
    K, RN, TN = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    ptr = L.gsro_sample_forward(PN, P, W, H, _p(keep[0]), _p(keep[1]), _p(keep[2]), _p(keep[3]),
                                float(scale_modifier), _p(keep[4]), _p(keep[5]), _p(keep[6]), _p(keep[7]),
                                _p(keep[8]), float(tan_fovx), float(tan_fovy), float(kernel_size), _p(output),
                                _p(inside, _u8), ctypes.byref(K), ctypes.byref(RN), ctypes.byref(TN))
    st = SampleState(ptr, P, PN, W, H, K.value)
    return dict(num_rendered=K.value, num_points=RN.value, num_duplicated_tiles=TN.value, output=output,
                inside=inside.astype(bool), state=st)


def _point_query(mode, points3D, means3D, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                 view2gaussian_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, kernel_size, image_height,
                 image_width, campos, prefiltered, debug):
    del view2gaussian_precomp, prefiltered, debug  # unused by the reference (rasterizer_impl.cu:594-1040)
    L = lib()
    pts = _np(points3D)
    PN = 0 if pts is None else pts.size // 3
    means3D = _np(means3D)
    P = 0 if means3D is None else means3D.shape[0]
    out0, out1 = np.zeros(PN, np.float32), np.zeros(PN, np.float32)
    inside = np.zeros(PN, np.uint8)
    K = ctypes.c_int(0)
    if P and PN:
        keep = [pts, means3D, _np(opacity), _np(scales), _np(rotations), _np(cov3D_precomp), _np(viewmatrix),
                _np(projmatrix), _np(campos)]
        rc = L.gsro_point_query(mode, PN, P, int(image_width), int(image_height), _p(keep[0]), _p(keep[1]),
                                _p(keep[2]), _p(keep[3]), float(scale_modifier), _p(keep[4]), _p(keep[5]),
                                _p(keep[6]), _p(keep[7]), _p(keep[8]), float(tan_fovx), float(tan_fovy),
                                float(kernel_size), _p(out0), _p(out1), _p(inside, _u8), ctypes.byref(K))
        if rc != 0:
            raise RuntimeError(f"oracle point query failed: {rc}")
    return K.value, out0, out1, inside.astype(bool)


def integrate(*args):
    """Same 18 arguments and return tuple as _C.integrate_gaussians_to_points
    (DGR/rasterize_points.cu:279-366): (num_rendered, transmittance, inside)."""
    K, T, _, inside = _point_query(0, *args)
    return K, T, inside


def evaluate_sdf(*args):
    """Same 18 arguments and return tuple as _C.evaluate_sdf_from_signle_view
    (DGR/rasterize_points.cu:368-457): (num_rendered, depth, sdf, inside)."""
    return _point_query(1, *args)


def sample_backward(state: SampleState, points3D, means3D, opacity, scales, rotations, scale_modifier,
                    cov3D_precomp, viewmatrix, projmatrix, inside, dL_doutput, tan_fovx, tan_fovy,
                    kernel_size) -> dict:
    """Same meaning as _C.sample_rasterized_depth_backward (DGR/rasterize_points.cu:555-633):
    returns dopacity, dmeans3D, dcov3D, dscales, drotations, dpoints3D."""
    L = lib()
    pts = _np(points3D)
    shape = tuple(points3D.shape) if hasattr(points3D, "shape") else np.asarray(points3D).shape
    means3D = _np(means3D)
    P = means3D.shape[0]
    out = dict(dopacity=np.zeros((P, 1), np.float32), dmeans3D=np.zeros((P, 3), np.float32),
               dcov3D=np.zeros((P, 6), np.float32), dscales=np.zeros((P, 3), np.float32),
               drotations=np.zeros((P, 4), np.float32), dpoints3D=np.zeros(shape, np.float32))
    if state is None:
        return out
    keep = [pts, means3D, _np(opacity), _np(scales), _np(rotations), _np(cov3D_precomp), _np(viewmatrix),
            _np(projmatrix), _np(inside, np.uint8), _np(dL_doutput)]
    rc = L.gsro_sample_backward(state.ptr, _p(keep[0]), _p(keep[1]), _p(keep[2]), _p(keep[3]),
                                float(scale_modifier), _p(keep[4]), _p(keep[5]), _p(keep[6]), _p(keep[7]),
                                float(tan_fovx), float(tan_fovy), float(kernel_size), _p(keep[8], _u8),
                                _p(keep[9]), _p(out["dopacity"]), _p(out["dmeans3D"]), _p(out["dcov3D"]),
                                _p(out["dscales"]), _p(out["drotations"]), _p(out["dpoints3D"]))
    if rc != 0:
        raise RuntimeError(f"oracle sample backward failed: {rc}")
    return out


def warp_patch_ncc(depths, normals, uvs, R, T, image_r, image_n, fx_r, fy_r, cx_r, cy_r, fx_n, fy_n, cx_n, cy_n):
    """Same meaning as the reference's _C.warp_patch_ncc (submodules/warp-patch-ncc/warp_patch_ncc.cu:5-52):
    returns dict(ncc [P], grad_depths [P], grad_normals [P,3], valid [P] bool)."""
    d = _np(depths)
    P = 0 if d is None else d.size
    out = dict(ncc=np.zeros(P, np.float32), grad_depths=np.zeros(P, np.float32),
               grad_normals=np.zeros((P, 3), np.float32), valid=np.zeros(P, np.uint8))
    if P == 0:
        out["valid"] = out["valid"].astype(bool)
        return out
    ir, inn = _np(image_r), _np(image_n)
    Hr, Wr = np.asarray(image_r.shape if hasattr(image_r, "shape") else ir.shape)[-2:]
    Hn, Wn = np.asarray(image_n.shape if hasattr(image_n, "shape") else inn.shape)[-2:]
    keep = [d, _np(normals), _np(uvs, np.int32), _np(R), _np(T), ir, inn]
    lib().gsro_warp_patch_ncc(P, _p(keep[0]), _p(keep[1]), _p(keep[2], _i), _p(keep[3]), _p(keep[4]), _p(keep[5]),
                              _p(keep[6]), float(fx_r), float(fy_r), float(cx_r), float(cy_r), float(fx_n),
                              float(fy_n), float(cx_n), float(cy_n), int(Hr), int(Wr), int(Hn), int(Wn),
                              _p(out["ncc"]), _p(out["grad_depths"]), _p(out["grad_normals"]), _p(out["valid"], _u8))
    out["valid"] = out["valid"].astype(bool)
    return out


def cov3d(scales, scale_modifier, rotations):
    """[P, 6] 3D covariance (xx, xy, xz, yy, yz, zz) of the scale/rotation
    path, (S R)^T (S R) in the kernels' glm convention (gsro_cov3d)."""
    s = np.ascontiguousarray(_np(scales), np.float32).reshape(-1, 3)
    q = np.ascontiguousarray(_np(rotations), np.float32).reshape(-1, 4)
    out = np.zeros((s.shape[0], 6), np.float32)
    lib().gsro_cov3d(s.shape[0], _p(s), float(scale_modifier), _p(q), _p(out))
    return out


def cov3d_backward(scales, scale_modifier, rotations, dL_dcov3D):
    """(dL/d(mod scale) [P, 3], dL/dq [P, 4]) of computeCov3D's backward
    (render_backward.cu:193-244) alone (gsro_cov3d_bwd)."""
    s = np.ascontiguousarray(_np(scales), np.float32).reshape(-1, 3)
    q = np.ascontiguousarray(_np(rotations), np.float32).reshape(-1, 4)
    g = np.ascontiguousarray(_np(dL_dcov3D), np.float32).reshape(-1, 6)
    ds = np.zeros_like(s)
    dq = np.zeros_like(q)
    lib().gsro_cov3d_bwd(s.shape[0], _p(s), float(scale_modifier), _p(q), _p(g), _p(ds), _p(dq))
    return ds, dq


def knn_mean_dist(points):
    """distCUDA2 (submodules/simple-knn/spatial.cu:15-25): [P] mean squared
    distance to the 3 nearest other points.  Returns (dists, Morton order)."""
    pts = np.ascontiguousarray(_np(points), np.float32).reshape(-1, 3)
    P = pts.shape[0]
    out = np.zeros(P, np.float32)
    order = np.zeros(P, np.uint32)
    if P:
        lib().gsro_knn_mean_dist(P, _p(pts), _p(out), _p(order, _u32))
    return out, order
