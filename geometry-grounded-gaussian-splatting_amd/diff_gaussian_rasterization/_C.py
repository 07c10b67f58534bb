"""`_C` — the extension entry points of the reference, bound to libgsr.so.

Mirrors the pybind module of the reference (DGR/ext.cpp:15-23) with the same
names, argument order, return tuples and error behaviour:

  rasterize_gaussians(25 args)           -> (num_rendered, color, alpha, normal, mdepth, radii,
                                             geomBuffer, binningBuffer, imgBuffer, tileBuffer)
                                             (DGR/rasterize_points.cu:39-139)
  rasterize_gaussians_backward(35 args)  -> (dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh,
                                             dsg_axis, dsg_sharpness, dsg_color, dscales, drotations)
                                             (DGR/rasterize_points.cu:141-258)
  mark_visible(means3D, view, proj)      -> bool[P]  (DGR/rasterize_points.cu:260-277)
  sample_rasterized_depth(17 args)       -> (num_rendered, num_points, num_duplicated_tiles, output, inside,
                                             geomBuffer, binningBuffer, pointBuffer, pointBinningBuffer,
                                             tileBuffer, duplicatedTileBuffer)  (DGR/rasterize_points.cu:459-553)
  sample_rasterized_depth_backward(28)   -> (dopacity, dmeans3D, dcov3D, dscales, drotations, dpoints3D)
                                             (DGR/rasterize_points.cu:555-633)

The C ABI (include/gsr.h) takes raw device pointers and allocation callbacks;
here torch provides the memory (caching allocator), the current HIP stream and
the uint8 scratch tensors that autograd keeps alive between forward and
backward.  There is no CPU fallback: inputs must be HIP (cuda) tensors and the
shared library must load, otherwise these functions raise.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSR_LIB") or os.path.join(_HERE, "libgsr.so")  # GSR_LIB: development A/B builds

_ALLOC = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
_CHUNK = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.c_int)  # gsr_chunk_fn
_lib = None


class AdamGroup(ctypes.Structure):
    """gsr_adam_group (include/gsr.h)."""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("n", ctypes.c_longlong), ("lr", ctypes.c_double)]


# include/gsr.h ABI these bindings are written for (gsr_abi_version)
ABI_VERSION = 20


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libgsr.so not built ({LIB_PATH}); run `make -C geometry-grounded-gaussian-splatting_amd` "
                           "or __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    L.gsr_abi_version.restype = i
    if L.gsr_abi_version() != ABI_VERSION:  # the argtypes below are written for this ABI
        raise RuntimeError(f"{LIB_PATH}: ABI {L.gsr_abi_version()}, expected {ABI_VERSION} (stale build? "
                           "run `make -C geometry-grounded-gaussian-splatting_amd`)")
    L.gsr_rasterize_forward.restype = i
    L.gsr_rasterize_forward.argtypes = ([_ALLOC, vp] * 4 + [i] * 5 + [vp, i, i] + [vp] * 10 + [f] + [vp] * 3
                                        + [f] * 3 + [i] + [vp] * 5 + [i, i, vp, ctypes.POINTER(i)])
    L.gsr_rasterize_forward_ex.restype = i
    L.gsr_rasterize_forward_ex.argtypes = L.gsr_rasterize_forward.argtypes + [_ALLOC, vp]
    L.gsr_rasterize_backward.restype = i
    L.gsr_rasterize_backward.argtypes = ([_ALLOC, vp] + [i] * 6 + [vp, i, i] + [vp] * 10 + [f] + [vp] * 3
                                         + [f] * 3 + [vp] * 4 + [vp] * 4 + [vp] * 4 + [vp] * 11 + [i, i, vp])
    L.gsr_rasterize_backward_ex.restype = i
    L.gsr_rasterize_backward_ex.argtypes = L.gsr_rasterize_backward.argtypes[:-1] + [i, _CHUNK, vp, vp, vp]
    L.gsr_rasterize_forward_ex2.restype = i
    L.gsr_rasterize_forward_ex2.argtypes = L.gsr_rasterize_forward_ex.argtypes + [vp]
    L.gsr_rasterize_backward_ex2.restype = i
    L.gsr_rasterize_backward_ex2.argtypes = L.gsr_rasterize_backward_ex.argtypes + [vp, vp]
    L.gsr_sample_depth_forward.restype = i
    L.gsr_sample_depth_forward.argtypes = ([_ALLOC, vp] * 6 + [i] * 4 + [vp] * 4 + [f] + [vp] * 5 + [f] * 3 + [i]
                                           + [vp, vp, i, vp] + [ctypes.POINTER(i)] * 3)
    L.gsr_sample_depth_forward_ex.restype = i
    L.gsr_sample_depth_forward_ex.argtypes = L.gsr_sample_depth_forward.argtypes + [_ALLOC, vp]
    L.gsr_integrate_forward.restype = i
    L.gsr_integrate_forward.argtypes = ([_ALLOC, vp] * 6 + [i] * 4 + [vp] * 4 + [f] + [vp] * 6 + [f] * 3 + [i]
                                        + [vp, vp, i, vp, ctypes.POINTER(i)])
    L.gsr_evaluate_sdf_forward.restype = i
    L.gsr_evaluate_sdf_forward.argtypes = ([_ALLOC, vp] * 6 + [i] * 4 + [vp] * 4 + [f] + [vp] * 6 + [f] * 3 + [i]
                                           + [vp, vp, vp, i, vp, ctypes.POINTER(i)])
    L.gsr_sample_depth_backward.restype = i
    L.gsr_sample_depth_backward.argtypes = ([_ALLOC, vp] + [i] * 7 + [vp] * 4 + [f] + [vp] * 5 + [f] * 3
                                            + [vp] * 6 + [vp] * 2 + [vp] * 6 + [i, vp])
    L.gsr_adam_step.restype = i
    L.gsr_adam_step.argtypes = [i, ctypes.POINTER(AdamGroup), ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                ctypes.c_double, vp]
    L.gsr_densify_stats.restype = i
    L.gsr_densify_stats.argtypes = [i] + [vp] * 7
    L.gsr_view_color_grads.restype = i
    L.gsr_view_color_grads.argtypes = [i] * 6 + [vp] * 10
    L.gsr_view_color_grads_chunked.restype = i
    L.gsr_view_color_grads_chunked.argtypes = [i] * 7 + [vp] * 12
    L.gsr_backward_chunk_size.restype = i
    L.gsr_backward_chunk_size.argtypes = [i, i]
    L.gsr_mark_visible.restype = i
    L.gsr_mark_visible.argtypes = [i, vp, vp, vp, vp, vp]
    L.gsr_set_option.argtypes = [i, i]
    L.gsr_debug_binning.argtypes = [vp, vp, i, i, i, vp, vp, vp]
    L.gsr_debug_image.argtypes = [vp, i, i, vp, vp]
    L.gsr_debug_tile_stats.argtypes = [vp, i, i, vp, vp]
    L.gsr_debug_sample_points.argtypes = [vp, i, vp, vp, vp]
    L.gsr_debug_render_stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), i]
    L.gsr_timing_enable.argtypes = [i]
    L.gsr_timing_stage_mask.argtypes = [ctypes.c_uint]
    L.gsr_timing_collect.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i)]
    L.gsr_stage_name.restype = ctypes.c_char_p
    L.gsr_stage_name.argtypes = [i]
    L.gsr_last_error.restype = ctypes.c_char_p
    _lib = L
    return L


def loaded_library_path() -> str:
    _load()
    return LIB_PATH


NUM_STAGES = 14
# debugging aid: keep the last backward's accumulator buffer (gsr_api.hip
# carve_bwd layout: 256-B aligned base, float acc[P][16], then float acc_abs[P])
KEEP_BWD_SCRATCH = False
last_bwd_scratch = None
# (ids 0, 2-4, 7, 8: retired variants and diagnostics, rejected by gsr_set_option)
OPT_RENDER_STATS = 1
OPT_NO_REFINE = 5
OPT_BWD_NO_CACHE = 6
OPT_ROCPRIM_DSORT = 9
OPT_PBWD_STAGE = 10


def backward_chunk_size(P: int, chunks: int) -> int:
    """The Gaussian range size of a backward run in `chunks` ranges
    (gsr_backward_chunk_size; host only, no GPU needed)."""
    n = _load().gsr_backward_chunk_size(int(P), int(chunks))
    if n < 0:
        raise RuntimeError(f"gsr: backward_chunk_size({P}, {chunks}): P must be >= 0 and chunks >= 1")
    return n


def debug_render_stats(reset: bool = True) -> list:
    """Counters of forward launches made with OPT_RENDER_STATS (render_fwd.hip)."""
    out = (ctypes.c_ulonglong * 20)()
    _check(_load().gsr_debug_render_stats(out, int(bool(reset))))
    return list(out)


def debug_binning(binningBuffer, tileBuffer, R: int, image_height: int, image_width: int, with_list: bool = True):
    """(point_list [R] uint32, ranges [tiles, 2] uint32) of a forward's buffers
    (gsr_debug_binning), as numpy arrays.  The per-tile lists hold only the
    instances that survive tile culling: their count is ranges[:, 1].max(),
    R (= num_rendered, the reference's K) is the capacity."""
    import numpy as np

    tiles = ((image_width + 15) // 16) * ((image_height + 15) // 16)
    plist = np.zeros(max(R, 0) if with_list else 0, np.uint32)
    ranges = np.zeros((tiles, 2), np.uint32)
    stream = torch.cuda.current_stream(binningBuffer.device).cuda_stream
    _check(_load().gsr_debug_binning(ctypes.c_void_p(binningBuffer.data_ptr()),
                                     ctypes.c_void_p(tileBuffer.data_ptr()), int(R), int(image_width),
                                     int(image_height), plist.ctypes.data_as(ctypes.c_void_p) if with_list else None,
                                     ranges.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(stream)))
    return plist, ranges


def debug_n_contrib(imgBuffer, image_height: int, image_width: int):
    """Per-pixel last contributor [H, W] uint32 of a forward's image buffer
    (gsr_debug_image): 1-based positions in the culled per-tile lists of
    debug_binning."""
    import numpy as np

    out = np.zeros((image_height, image_width), np.uint32)
    stream = torch.cuda.current_stream(imgBuffer.device).cuda_stream
    _check(_load().gsr_debug_image(ctypes.c_void_p(imgBuffer.data_ptr()), int(image_width), int(image_height),
                                   out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(stream)))
    return out


def debug_max_contrib(tileBuffer, image_height: int, image_width: int):
    """Per-tile max contributor [tiles] uint32 of a forward's tile buffer
    (gsr_debug_tile_stats): how far into each culled tile list the forward's
    pixels blended, the range the backward walks."""
    import numpy as np

    tiles = ((image_width + 15) // 16) * ((image_height + 15) // 16)
    out = np.zeros(tiles, np.uint32)
    stream = torch.cuda.current_stream(tileBuffer.device).cuda_stream
    _check(_load().gsr_debug_tile_stats(ctypes.c_void_p(tileBuffer.data_ptr()), int(image_width), int(image_height),
                                        out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(stream)))
    return out


def debug_sample_points(pointBuffer, PN: int):
    """(median depth along the ray [PN] float32, last contributor [PN] uint32)
    of a sample_rasterized_depth forward's point buffer (gsr_debug_sample_points)."""
    import numpy as np

    md = np.zeros(PN, np.float32)
    last = np.zeros(PN, np.uint32)
    stream = torch.cuda.current_stream(pointBuffer.device).cuda_stream
    _check(_load().gsr_debug_sample_points(ctypes.c_void_p(pointBuffer.data_ptr()), int(PN),
                                           md.ctypes.data_as(ctypes.c_void_p), last.ctypes.data_as(ctypes.c_void_p),
                                           ctypes.c_void_p(stream)))
    return md, last


def set_option(opt: int, value: int) -> None:
    """Select an A/B kernel variant (gsr_set_option); variants are bit-identical."""
    _check(_load().gsr_set_option(int(opt), int(value)))


def timing_enable(on: bool = True) -> None:
    """Bracket every kernel stage with hipEvents on its stream (gsr_timing_enable)."""
    _load().gsr_timing_enable(int(bool(on)))


def timing_stages(names=None) -> None:
    """Time only the named stages (None: all), gsr_timing_stage_mask."""
    L = _load()
    if names is None:
        mask = 0xFFFFFFFF
    else:
        idx = {L.gsr_stage_name(k).decode(): k for k in range(NUM_STAGES)}
        mask = sum(1 << idx[n] for n in set(names))
    _check(L.gsr_timing_stage_mask(mask))


def timing_collect() -> dict:
    """{stage name: (total ms, launches)} since the last collect (gsr_timing_collect)."""
    L = _load()
    ms = (ctypes.c_double * NUM_STAGES)()
    n = (ctypes.c_int * NUM_STAGES)()
    _check(L.gsr_timing_collect(ms, n))
    return {L.gsr_stage_name(k).decode(): (ms[k], n[k]) for k in range(NUM_STAGES)}


class _ByteBuffer:
    """A resizable torch.uint8 device tensor handed to the C ABI as a callback
    (replaces resizeFunctional, DGR/rasterize_points.cu:27-37)."""

    def __init__(self, device, zero: bool = False):
        self.device = device
        self.zero = zero
        self.tensor = torch.empty(0, dtype=torch.uint8, device=device)

        def _cb(_ctx, n):
            try:
                self.tensor = (torch.zeros if self.zero else torch.empty)(int(n), dtype=torch.uint8,
                                                                           device=self.device)
                return self.tensor.data_ptr() if n else self.tensor.data_ptr() or 1
            except Exception:  # noqa: BLE001 - allocation failure is reported as NULL
                return None

        self.cb = _ALLOC(_cb)


class _ScratchBlocks:
    """Forward-only scratch for gsr_rasterize_forward_ex: every block the
    callback hands out is kept until the forward returns, then dropped (the
    caching allocator reuses it in stream order), so it is not saved for the
    backward as the binning buffer is."""

    def __init__(self, device):
        self.device = device
        self.blocks = []

        def _cb(_ctx, n):
            try:
                t = torch.empty(max(int(n), 1), dtype=torch.uint8, device=self.device)
                self.blocks.append(t)
                return t.data_ptr()
            except Exception:  # noqa: BLE001 - allocation failure is reported as NULL
                return None

        self.cb = _ALLOC(_cb)


def _ptr(t):
    if t is None or t.numel() == 0:
        return None
    return ctypes.c_void_p(t.data_ptr())


def _dev_contig(t, name):
    if t is None:
        return None
    if t.numel() == 0:
        return t
    if not t.is_cuda:
        raise RuntimeError(f"gsr: `{name}` must be a HIP device tensor (got {t.device})")
    if t.dtype != torch.float32 and name not in ("radii",):
        raise RuntimeError(f"gsr: `{name}` must be float32 (got {t.dtype})")
    return t.contiguous()


def _split_rest(sh, sh_rest, P):
    """The rest rows of the split SH layout, checked, or None (one [P, M, 3] tensor)."""
    if sh_rest is None:
        return None
    if sh is None or sh.numel() == 0 or tuple(sh.shape) != (P, 1, 3) or sh_rest.dim() != 3 or \
            sh_rest.size(0) != P or sh_rest.size(2) != 3 or sh_rest.size(1) < 1:
        raise RuntimeError("gsr: split SH rows are sh [P, 1, 3] and sh_rest [P, M-1, 3]")
    return _dev_contig(sh_rest, "sh_rest")


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _check(rc):
    if rc != 0:
        raise RuntimeError("gsr: " + _lib.gsr_last_error().decode())


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, cov3D_precomp, sh, sg_axis,
                        sg_sharpness, sg_color, sh_degree, sg_degree, scale_modifier, viewmatrix, projmatrix,
                        tan_fovx, tan_fovy, kernel_size, image_height, image_width, campos, prefiltered,
                        require_depth, debug, sh_rest=None):
    """The reference's 25 arguments (rasterize_points.cu:36-139).  `sh_rest`
    (not in the reference): the split SH layout of training — `sh` the DC
    rows [P, 1, 3] and `sh_rest` the rest [P, M-1, 3] as GaussianModel keeps
    them, without their concatenation (gsr_rasterize_forward_ex2)."""
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    L = _load()
    P = means3D.size(0)
    H, W = int(image_height), int(image_width)
    dev = means3D.device
    fopt = dict(dtype=torch.float32, device=dev)
    if P == 0:  # rasterize_points.cu:77-95: zero outputs, nothing rendered
        bufs = [torch.empty(0, dtype=torch.uint8, device=dev) for _ in range(4)]
        return (0, torch.zeros(3, H, W, **fopt), torch.zeros(1, H, W, **fopt), torch.zeros(3, H, W, **fopt),
                torch.zeros(1, H, W, **fopt), torch.zeros(0, dtype=torch.int32, device=dev), *bufs)
    args = {k: _dev_contig(v, k) for k, v in dict(
        background=background, means3D=means3D, colors=colors, opacity=opacity, scales=scales,
        rotations=rotations, cov3D_precomp=cov3D_precomp, sh=sh, sg_axis=sg_axis, sg_sharpness=sg_sharpness,
        sg_color=sg_color, viewmatrix=viewmatrix, projmatrix=projmatrix, campos=campos).items()}
    SHM = sh.size(1) if sh is not None and sh.size(0) != 0 else 0
    SGM = sg_color.size(1) if sg_color is not None and sg_color.size(0) != 0 else 0
    rest = _split_rest(sh, sh_rest, P)
    if rest is not None:
        SHM = 1 + sh_rest.size(1)
    color = torch.empty(3, H, W, **fopt)
    mdepth = torch.empty(1, H, W, **fopt)
    alpha = torch.empty(1, H, W, **fopt)
    normal = torch.empty(3, H, W, **fopt)
    radii = torch.empty(P, dtype=torch.int32, device=dev)
    bufs = [_ByteBuffer(dev) for _ in range(4)]
    scratch = _ScratchBlocks(dev)
    K = ctypes.c_int(0)
    with torch.cuda.device(dev):
        rc = L.gsr_rasterize_forward_ex2(
            bufs[0].cb, None, bufs[1].cb, None, bufs[2].cb, None, bufs[3].cb, None,
            P, int(sh_degree), SHM, int(sg_degree), SGM, _ptr(args["background"]), W, H, _ptr(args["means3D"]),
            _ptr(args["colors"]), _ptr(args["opacity"]), _ptr(args["scales"]), _ptr(args["rotations"]),
            _ptr(args["cov3D_precomp"]), _ptr(args["sh"]), _ptr(args["sg_axis"]), _ptr(args["sg_sharpness"]),
            _ptr(args["sg_color"]), float(scale_modifier), _ptr(args["viewmatrix"]), _ptr(args["projmatrix"]),
            _ptr(args["campos"]), float(tan_fovx), float(tan_fovy), float(kernel_size), int(bool(prefiltered)),
            _ptr(color), _ptr(mdepth), _ptr(alpha), _ptr(normal), _ptr(radii), int(bool(require_depth)),
            int(bool(debug)), _stream(dev), ctypes.byref(K), scratch.cb, None, _ptr(rest))
    del scratch
    _check(rc)
    return (K.value, color, alpha, normal, mdepth, radii, bufs[0].tensor, bufs[1].tensor, bufs[2].tensor,
            bufs[3].tensor)


def rasterize_gaussians_backward(background, means3D, colors, opacity, scales, rotations, cov3D_precomp, sh,
                                 sg_axis, sg_sharpness, sg_color, sh_degree, sg_degree, scale_modifier, viewmatrix,
                                 projmatrix, tan_fovx, tan_fovy, kernel_size, dL_dout_color, dL_dout_mdepth,
                                 dL_dout_alpha, dL_dout_normal, alphas, normalmap, mdepth, campos, radii,
                                 geomBuffer, R, binningBuffer, imageBuffer, tileBuffer, require_depth, debug,
                                 exchange=None, sh_rest=None):
    """The reference's 35 arguments and 11 gradients (rasterize_points.cu:141-258).
    `exchange` (not in the reference; gsr_dist.OverlappedViewGrads) runs the
    per-Gaussian backward in exchange.chunks Gaussian ranges through
    gsr_rasterize_backward_ex and calls exchange.on_chunk(begin, end, grads)
    after each range is queued; with exchange.dc_rows(...) a buffer, only the
    DC gradient rows are written there (the SH / SG rows are the exchange's to
    rebuild before the gradients are used).  `sh_rest` (the split SH layout,
    see rasterize_gaussians): dsh is then [P, 1, 3] and a 12th gradient,
    dsh_rest [P, M-1, 3], is returned (gsr_rasterize_backward_ex2)."""
    L = _load()
    P = means3D.size(0)
    img = dL_dout_color if dL_dout_color is not None else alphas  # (a None upstream gradient is zero)
    H, W = img.size(1), img.size(2)
    SHM = sh.size(1) if sh is not None and sh.size(0) != 0 else 0
    SGM = sg_color.size(1) if sg_color is not None and sg_color.size(0) != 0 else 0
    rest = _split_rest(sh, sh_rest, P)
    dev = means3D.device
    fopt = dict(dtype=torch.float32, device=dev)
    alloc = torch.zeros if P == 0 else torch.empty  # the kernels overwrite every element
    outs = dict(dmeans3D=alloc(P, 3, **fopt), dmeans2D=alloc(P, 3, **fopt), dcolors=alloc(P, 3, **fopt),
                dopacity=alloc(P, 1, **fopt), dcov3D=alloc(P, 6, **fopt), dsh=alloc(P, SHM, 3, **fopt),
                dsg_axis=alloc(P, SGM, 3, **fopt), dsg_sharpness=alloc(P, SGM, **fopt),
                dsg_color=alloc(P, SGM, 3, **fopt), dscales=alloc(P, 3, **fopt), drotations=alloc(P, 4, **fopt))
    if rest is not None:
        outs["dsh_rest"] = alloc(*sh_rest.shape, **fopt)
        SHM = 1 + sh_rest.size(1)
    if P != 0:
        a = {k: _dev_contig(v, k) for k, v in dict(
            background=background, means3D=means3D, colors=colors, opacity=opacity, scales=scales,
            rotations=rotations, cov3D_precomp=cov3D_precomp, sh=sh, sg_axis=sg_axis, sg_sharpness=sg_sharpness,
            sg_color=sg_color, viewmatrix=viewmatrix, projmatrix=projmatrix, campos=campos, alphas=alphas,
            normalmap=normalmap, mdepth=mdepth, dL_dout_color=dL_dout_color, dL_dout_mdepth=dL_dout_mdepth,
            dL_dout_alpha=dL_dout_alpha, dL_dout_normal=dL_dout_normal).items()}
        radii = radii.contiguous()
        scratch = _ByteBuffer(dev)
        grads = (outs["dmeans2D"], outs["dcolors"], outs["dopacity"], outs["dmeans3D"], outs["dcov3D"], outs["dsh"],
                 outs["dsg_axis"], outs["dsg_sharpness"], outs["dsg_color"], outs["dscales"], outs["drotations"])
        chunks, dc = 1, None
        hook = _CHUNK()  # NULL
        if exchange is not None:
            chunks = max(1, int(exchange.chunks))
            dc = exchange.dc_rows(P, dev) if SHM else None
            cb = exchange.hook(grads)  # (errors held by the exchange, raised by settle below)
            hook = _CHUNK(lambda _ctx, b, e: cb(b, e))
        with torch.cuda.device(dev):
            rc = L.gsr_rasterize_backward_ex2(
                scratch.cb, None, P, int(sh_degree), SHM, int(sg_degree), SGM, int(R), _ptr(a["background"]), W, H,
                _ptr(a["means3D"]), _ptr(a["colors"]), _ptr(a["opacity"]), _ptr(a["scales"]), _ptr(a["rotations"]),
                _ptr(a["cov3D_precomp"]), _ptr(a["sh"]), _ptr(a["sg_axis"]), _ptr(a["sg_sharpness"]),
                _ptr(a["sg_color"]), float(scale_modifier), _ptr(a["viewmatrix"]), _ptr(a["projmatrix"]),
                _ptr(a["campos"]), float(tan_fovx), float(tan_fovy), float(kernel_size), _ptr(radii),
                _ptr(a["alphas"]), _ptr(a["normalmap"]), _ptr(a["mdepth"]), _ptr(geomBuffer), _ptr(binningBuffer),
                _ptr(imageBuffer), _ptr(tileBuffer), _ptr(a["dL_dout_color"]), _ptr(a["dL_dout_mdepth"]),
                _ptr(a["dL_dout_alpha"]), _ptr(a["dL_dout_normal"]), _ptr(outs["dmeans3D"]), _ptr(outs["dmeans2D"]),
                _ptr(outs["dcolors"]), _ptr(outs["dopacity"]), _ptr(outs["dscales"]), _ptr(outs["drotations"]),
                _ptr(outs["dcov3D"]), _ptr(outs["dsh"]), _ptr(outs["dsg_axis"]), _ptr(outs["dsg_sharpness"]),
                _ptr(outs["dsg_color"]), int(bool(require_depth)), int(bool(debug)), chunks, hook, None,
                None if dc is None else _ptr(dc), _stream(dev), _ptr(rest), _ptr(outs.get("dsh_rest")))
        if exchange is not None:  # a failed backward still posts every range's collectives (no peer blocks)
            exchange.settle(rc == 0)
        _check(rc)
        if KEEP_BWD_SCRATCH:
            global last_bwd_scratch
            last_bwd_scratch = scratch.tensor
    g = (outs["dmeans2D"], outs["dcolors"], outs["dopacity"], outs["dmeans3D"], outs["dcov3D"], outs["dsh"],
         outs["dsg_axis"], outs["dsg_sharpness"], outs["dsg_color"], outs["dscales"], outs["drotations"])
    return g if rest is None else g + (outs["dsh_rest"],)


def mark_visible(means3D, viewmatrix, projmatrix):
    L = _load()
    P = means3D.size(0)
    present = torch.zeros(P, dtype=torch.bool, device=means3D.device)
    if P != 0:
        m = _dev_contig(means3D, "means3D")
        v = _dev_contig(viewmatrix, "viewmatrix")
        p = _dev_contig(projmatrix, "projmatrix")
        with torch.cuda.device(means3D.device):
            _check(L.gsr_mark_visible(P, _ptr(m), _ptr(v), _ptr(p), _ptr(present), _stream(means3D.device)))
    return present


def _point_query(fn, points3D, means3D, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                 view2gaussian_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, kernel_size, image_height,
                 image_width, campos, prefiltered, debug):
    """IntegrateGaussiansToPointsCUDA / evaluateSDFfromSingleView
    (DGR/rasterize_points.cu:279-457): outputs zero-filled (torch::full 0),
    the scratch buffers are local to the call."""
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    if points3D.ndimension() != 2 or points3D.size(1) != 3:
        raise RuntimeError("points3D must have dimensions (num_points, 3)")
    L = _load()
    PN, P = points3D.size(0), means3D.size(0)
    dev = means3D.device
    out0 = torch.zeros(PN, dtype=torch.float32, device=dev)
    out1 = torch.zeros(PN, dtype=torch.float32, device=dev)
    inside = torch.zeros(PN, dtype=torch.bool, device=dev)
    K = ctypes.c_int(0)
    if P != 0 and PN != 0:
        a = {k: _dev_contig(v, k) for k, v in dict(
            points3D=points3D, means3D=means3D, opacity=opacity, scales=scales, rotations=rotations,
            cov3D_precomp=cov3D_precomp, view2gaussian_precomp=view2gaussian_precomp, viewmatrix=viewmatrix,
            projmatrix=projmatrix, campos=campos).items()}
        bufs = [_ByteBuffer(dev) for _ in range(6)]
        head = [bufs[0].cb, None, bufs[1].cb, None, bufs[2].cb, None, bufs[3].cb, None, bufs[4].cb, None,
                bufs[5].cb, None, PN, P, int(image_width), int(image_height), _ptr(a["points3D"]),
                _ptr(a["means3D"]), _ptr(a["opacity"]), _ptr(a["scales"]), float(scale_modifier),
                _ptr(a["rotations"]), _ptr(a["cov3D_precomp"]), _ptr(a["view2gaussian_precomp"]),
                _ptr(a["viewmatrix"]), _ptr(a["projmatrix"]), _ptr(a["campos"]), float(tan_fovx), float(tan_fovy),
                float(kernel_size), int(bool(prefiltered))]
        outs = [_ptr(out0)] if fn == "integrate" else [_ptr(out0), _ptr(out1)]
        with torch.cuda.device(dev):
            entry = L.gsr_integrate_forward if fn == "integrate" else L.gsr_evaluate_sdf_forward
            rc = entry(*head, *outs, _ptr(inside), int(bool(debug)), _stream(dev), ctypes.byref(K))
        _check(rc)
    return K.value, out0, out1, inside


def integrate_gaussians_to_points(points3D, means3D, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                                  view2gaussian_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, kernel_size,
                                  image_height, image_width, campos, prefiltered, debug):
    """-> (num_rendered, transmittance [PN], inside [PN] bool), rasterize_points.cu:279-366."""
    K, T, _, inside = _point_query("integrate", points3D, means3D, opacity, scales, rotations, scale_modifier,
                                   cov3D_precomp, view2gaussian_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy,
                                   kernel_size, image_height, image_width, campos, prefiltered, debug)
    return K, T, inside


def evaluate_sdf_from_signle_view(points3D, means3D, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                                  view2gaussian_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, kernel_size,
                                  image_height, image_width, campos, prefiltered, debug):
    """-> (num_rendered, depth [PN], sdf [PN], inside [PN] bool), rasterize_points.cu:368-457
    (the reference's spelling of the binding name, DGR/ext.cpp)."""
    return _point_query("sdf", points3D, means3D, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        view2gaussian_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, kernel_size,
                        image_height, image_width, campos, prefiltered, debug)


# (measurement hook, bench.py --e2e: the last sample_rasterized_depth call's points, camera and outputs, for
# the SAMPLE raster's algorithmic bytes)
CAPTURE_SAMPLE = False
last_sample = None


def sample_rasterized_depth(points3D, means3D, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                            viewmatrix, projmatrix, tan_fovx, tan_fovy, kernel_size, image_height, image_width,
                            campos, prefiltered, debug):
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    if points3D.ndimension() < 1 or points3D.size(-1) != 3:
        raise RuntimeError("points3D must have shape (..., 3) with last dimension == 3")
    L = _load()
    PN = points3D.numel() // 3
    P = means3D.size(0)
    H, W = int(image_height), int(image_width)
    dev = means3D.device
    output = torch.zeros_like(points3D)
    inside = torch.zeros(points3D.shape[:-1], dtype=torch.bool, device=points3D.device)
    bufs = [_ByteBuffer(dev) for _ in range(6)]
    scratch = _ScratchBlocks(dev)
    K, RN, TN = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    if P != 0 and PN != 0:
        a = {k: _dev_contig(v, k) for k, v in dict(
            points3D=points3D, means3D=means3D, opacity=opacity, scales=scales, rotations=rotations,
            cov3D_precomp=cov3D_precomp, viewmatrix=viewmatrix, projmatrix=projmatrix, campos=campos).items()}
        with torch.cuda.device(dev):
            rc = L.gsr_sample_depth_forward_ex(
                bufs[0].cb, None, bufs[1].cb, None, bufs[2].cb, None, bufs[3].cb, None, bufs[4].cb, None,
                bufs[5].cb, None, PN, P, W, H, _ptr(a["points3D"]), _ptr(a["means3D"]), _ptr(a["opacity"]),
                _ptr(a["scales"]), float(scale_modifier), _ptr(a["rotations"]), _ptr(a["cov3D_precomp"]),
                _ptr(a["viewmatrix"]), _ptr(a["projmatrix"]), _ptr(a["campos"]), float(tan_fovx), float(tan_fovy),
                float(kernel_size), int(bool(prefiltered)), _ptr(output), _ptr(inside), int(bool(debug)),
                _stream(dev), ctypes.byref(K), ctypes.byref(RN), ctypes.byref(TN), scratch.cb, None)
        del scratch
        _check(rc)
    res = (K.value, RN.value, TN.value, output, inside, *[b.tensor for b in bufs])
    if CAPTURE_SAMPLE:
        global last_sample
        last_sample = dict(points3D=points3D, projmatrix=projmatrix, H=H, W=W, out=res)
    return res


def sample_rasterized_depth_backward(points3D, means3D, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                                     viewmatrix, projmatrix, inside, dL_doutput, tan_fovx, tan_fovy, kernel_size,
                                     image_height, image_width, campos, geomBuffer, binningBuffer, pointBuffer,
                                     pointBinningBuffer, tileBuffer, duplicatedTileBuffer, R, RN, TN, prefiltered,
                                     debug):
    L = _load()
    PN = points3D.numel() // 3
    P = means3D.size(0)
    dev = means3D.device
    fopt = dict(dtype=torch.float32, device=dev)
    alloc = torch.zeros if (P == 0 or PN == 0) else torch.empty  # the kernels overwrite every element
    outs = dict(dopacity=alloc(P, 1, **fopt), dmeans3D=alloc(P, 3, **fopt), dcov3D=alloc(P, 6, **fopt),
                dscales=alloc(P, 3, **fopt), drotations=alloc(P, 4, **fopt), dpoints3D=torch.zeros_like(points3D))
    if P != 0 and PN != 0:
        a = {k: _dev_contig(v, k) for k, v in dict(
            points3D=points3D, means3D=means3D, opacity=opacity, scales=scales, rotations=rotations,
            cov3D_precomp=cov3D_precomp, viewmatrix=viewmatrix, projmatrix=projmatrix, campos=campos,
            dL_doutput=dL_doutput).items()}
        ins = inside.contiguous()
        if not ins.is_cuda or ins.dtype != torch.bool:
            raise RuntimeError("gsr: `inside` must be the forward's bool device tensor")
        scratch = _ByteBuffer(dev)
        with torch.cuda.device(dev):
            rc = L.gsr_sample_depth_backward(
                scratch.cb, None, PN, P, int(RN), int(R), int(TN), int(image_width), int(image_height),
                _ptr(a["points3D"]), _ptr(a["means3D"]), _ptr(a["opacity"]), _ptr(a["scales"]), float(scale_modifier),
                _ptr(a["rotations"]), _ptr(a["cov3D_precomp"]), _ptr(a["viewmatrix"]), _ptr(a["projmatrix"]),
                _ptr(a["campos"]), float(tan_fovx), float(tan_fovy), float(kernel_size), _ptr(geomBuffer),
                _ptr(binningBuffer), _ptr(pointBuffer), _ptr(pointBinningBuffer), _ptr(tileBuffer),
                _ptr(duplicatedTileBuffer), _ptr(ins), _ptr(a["dL_doutput"]), _ptr(outs["dopacity"]),
                _ptr(outs["dmeans3D"]), _ptr(outs["dcov3D"]), _ptr(outs["dscales"]), _ptr(outs["drotations"]),
                _ptr(outs["dpoints3D"]), int(bool(debug)), _stream(dev))
        _check(rc)
    return (outs["dopacity"], outs["dmeans3D"], outs["dcov3D"], outs["dscales"], outs["drotations"],
            outs["dpoints3D"])


MAX_ADAM_GROUPS = 16


def adam_step(tensors, lrs, step: float, beta1: float, beta2: float, eps: float) -> None:
    """One Adam update (gsr_adam_step) of up to 16 (param, grad, exp_avg,
    exp_avg_sq) fp32 device tensors, contiguous, each with its learning rate,
    all at step count `step` (after increment)."""
    L = _load()
    if not tensors:
        return
    arr = (AdamGroup * len(tensors))()
    dev = None
    for k, ((p, g, m, v), lr) in enumerate(zip(tensors, lrs)):
        for t, name in ((p, "param"), (g, "grad"), (m, "exp_avg"), (v, "exp_avg_sq")):
            if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous() or t.numel() != p.numel():
                raise RuntimeError(f"gsr adam: `{name}` must be a contiguous fp32 HIP tensor shaped like its param")
        dev = p.device
        arr[k] = AdamGroup(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), float(lr))
    with torch.cuda.device(dev):
        _check(L.gsr_adam_step(len(tensors), arr, float(step), float(beta1), float(beta2), float(eps), _stream(dev)))


def densify_stats(viewspace_grad, radii, max_radii2D, accum, accum_abs, denom) -> None:
    """add_densification_stats + max_radii2D (gsr_densify_stats), in place."""
    L = _load()
    P = radii.numel()
    for t, name in ((viewspace_grad, "viewspace_grad"), (max_radii2D, "max_radii2D"), (accum, "accum"),
                    (accum_abs, "accum_abs"), (denom, "denom")):
        if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
            raise RuntimeError(f"gsr densify_stats: `{name}` must be a contiguous fp32 HIP tensor")
    if radii.dtype != torch.int32 or not radii.is_cuda:
        raise RuntimeError("gsr densify_stats: `radii` must be an int32 HIP tensor")
    if viewspace_grad.numel() != 3 * P or max_radii2D.numel() != P or accum.numel() != P or accum_abs.numel() != P \
            or denom.numel() != P:
        raise RuntimeError("gsr densify_stats: shape mismatch")
    dev = radii.device
    r = radii.contiguous()
    with torch.cuda.device(dev):
        _check(L.gsr_densify_stats(P, _ptr(viewspace_grad), _ptr(r), _ptr(max_radii2D), _ptr(accum), _ptr(accum_abs),
                                   _ptr(denom), _stream(dev)))


def view_color_grads_chunked(gathered, campos, n_views: int, chunk: int, means3D, sh_degree: int, dL_dsh,
                             sg_degree: int = 0, sg_axis=None, sg_sharpness=None, sg_color=None, dL_dsg_axis=None,
                             dL_dsg_sharpness=None, dL_dsg_color=None, dL_dsh_rest=None) -> None:
    """gsr_view_color_grads_chunked: view_color_grads for the range-by-range
    gathered layout (include/gsr.h): gathered [n_views * P * 3] DC rows in
    ranges of `chunk` Gaussians, campos [n_views, 4].  With `dL_dsh_rest` (the
    split SH layout) dL_dsh is the DC rows [P, 1, 3] and dL_dsh_rest the rest
    [P, SHM - 1, 3]."""
    L = _load()
    P = means3D.shape[0]
    SHM = dL_dsh.shape[1] if dL_dsh_rest is None else 1 + dL_dsh_rest.shape[1]
    SGM = dL_dsg_color.shape[1] if dL_dsg_color is not None and dL_dsg_color.numel() else 0
    if gathered.numel() != n_views * P * 3 or campos.numel() != 4 * n_views or chunk < 1:
        raise RuntimeError("gsr view_color_grads_chunked: `gathered` must hold n_views * 3 P floats, `campos` "
                           "n_views * 4, chunk >= 1")
    want = {"means3D": (means3D, (P, 3)), "dL_dsh": (dL_dsh, (P, SHM, 3) if dL_dsh_rest is None else (P, 1, 3))}
    if dL_dsh_rest is not None:
        if SHM < 2:
            raise RuntimeError("gsr view_color_grads_chunked: the split SH layout needs SHM >= 2")
        want["dL_dsh_rest"] = (dL_dsh_rest, (P, SHM - 1, 3))
    if SGM:
        want.update(dL_dsg_axis=(dL_dsg_axis, (P, SGM, 3)), dL_dsg_sharpness=(dL_dsg_sharpness, (P, SGM)),
                    dL_dsg_color=(dL_dsg_color, (P, SGM, 3)))
    if sg_degree:
        want.update(sg_axis=(sg_axis, (P, SGM, 3)), sg_sharpness=(sg_sharpness, (P, SGM)),
                    sg_color=(sg_color, (P, SGM, 3)))
    for name, (t, shape) in list(want.items()) + [("gathered", (gathered, tuple(gathered.shape))),
                                                  ("campos", (campos, tuple(campos.shape)))]:
        if tuple(t.shape) != shape or not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
            raise RuntimeError(f"gsr view_color_grads_chunked: `{name}` must be a contiguous fp32 HIP tensor "
                               f"of shape {shape}")
    dev = means3D.device
    p = lambda t: _ptr(t) if t is not None and t.numel() else None  # noqa: E731
    with torch.cuda.device(dev):
        _check(L.gsr_view_color_grads_chunked(P, int(sh_degree), SHM, int(sg_degree), SGM, int(n_views), int(chunk),
                                              _ptr(gathered), _ptr(campos), _ptr(means3D), p(sg_axis),
                                              p(sg_sharpness), p(sg_color), _ptr(dL_dsh), p(dL_dsg_axis),
                                              p(dL_dsg_sharpness), p(dL_dsg_color), p(dL_dsh_rest), _stream(dev)))


def view_color_grads(gathered, n_views: int, means3D, sh_degree: int, dL_dsh, sg_degree: int = 0, sg_axis=None,
                     sg_sharpness=None, sg_color=None, dL_dsg_axis=None, dL_dsg_sharpness=None,
                     dL_dsg_color=None) -> None:
    """gsr_view_color_grads (view_grads.hip): the SH / SG gradient rows of a
    view-parallel step summed over `n_views` views, from the gathered
    [n_views, P * 3 + 4] DC rows + camera centres; outputs written in place."""
    L = _load()
    P = means3D.shape[0]
    SHM = dL_dsh.shape[1]
    SGM = dL_dsg_color.shape[1] if dL_dsg_color is not None and dL_dsg_color.numel() else 0
    need = [(gathered, "gathered"), (means3D, "means3D"), (dL_dsh, "dL_dsh")]
    if SGM:
        need += [(dL_dsg_axis, "dL_dsg_axis"), (dL_dsg_sharpness, "dL_dsg_sharpness"), (dL_dsg_color, "dL_dsg_color")]
    if sg_degree:
        need += [(sg_axis, "sg_axis"), (sg_sharpness, "sg_sharpness"), (sg_color, "sg_color")]
    for t, name in need:
        if t is None or not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
            raise RuntimeError(f"gsr view_color_grads: `{name}` must be a contiguous fp32 HIP tensor")
    if gathered.numel() != n_views * (3 * P + 4):
        raise RuntimeError("gsr view_color_grads: `gathered` must hold n_views * (3 P + 4) floats")
    want = {"means3D": (means3D, (P, 3)), "dL_dsh": (dL_dsh, (P, SHM, 3))}
    if SGM:
        want.update(dL_dsg_axis=(dL_dsg_axis, (P, SGM, 3)), dL_dsg_sharpness=(dL_dsg_sharpness, (P, SGM)),
                    dL_dsg_color=(dL_dsg_color, (P, SGM, 3)))
    if sg_degree:
        want.update(sg_axis=(sg_axis, (P, SGM, 3)), sg_sharpness=(sg_sharpness, (P, SGM)),
                    sg_color=(sg_color, (P, SGM, 3)))
    for name, (t, shape) in want.items():
        if tuple(t.shape) != shape:
            raise RuntimeError(f"gsr view_color_grads: `{name}` has shape {tuple(t.shape)}, expected {shape}")
    if not 0 <= int(sh_degree) <= 3 or SHM < (int(sh_degree) + 1) ** 2 or not 0 <= int(sg_degree) <= SGM:
        raise RuntimeError(f"gsr view_color_grads: degrees (SH {sh_degree}, SG {sg_degree}) do not fit "
                           f"{SHM} SH rows and {SGM} SG lobes")
    dev = means3D.device
    p = lambda t: _ptr(t) if t is not None and t.numel() else None  # noqa: E731
    with torch.cuda.device(dev):
        _check(L.gsr_view_color_grads(P, int(sh_degree), SHM, int(sg_degree), SGM, int(n_views), _ptr(gathered),
                                      _ptr(means3D), p(sg_axis), p(sg_sharpness), p(sg_color), _ptr(dL_dsh),
                                      p(dL_dsg_axis), p(dL_dsg_sharpness), p(dL_dsg_color), _stream(dev)))
