/*
 * gsr.h — C ABI of the MI355X (gfx950) differentiable Gaussian-splatting
 * rasterizer (libgsr.so).
 *
 * This is the drop-in boundary for the reference's hot path
 *   gaussian_renderer.render() -> GaussianRasterizer -> _C.rasterize_gaussians{,_backward}
 * The three entry points replace, one for one, the reference's C++ ABI
 *   CudaRasterizer::Rasterizer::forward / backward / markVisible
 *   (submodules/diff-gaussian-rasterization/cuda_rasterizer/rasterizer.h:21-129)
 * which its pybind layer binds as _C.rasterize_gaussians, _C.rasterize_gaussians_backward
 * and _C.mark_visible (DGR/ext.cpp:15-23, DGR/rasterize_points.cu:39-277).
 *
 * Differences from the reference ABI, all mechanical:
 *   - std::function<char*(size_t)> resize callbacks become (gsr_alloc_fn, ctx)
 *     pairs; a callback returns device memory of at least the requested size,
 *     valid until the backward of the same call has run (the reference keeps it
 *     alive in torch uint8 tensors saved by autograd, DGR/__init__.py:114-133).
 *     A NULL return makes the call fail with GSR_ERR_ALLOC.
 *   - every call takes the hipStream_t to launch on (the reference uses the
 *     legacy default stream); the forward synchronises that stream once, to read
 *     the instance count K (as the reference's cudaMemcpy does,
 *     rasterizer_impl.cu:384);
 *   - bool -> int, and a status code is returned (0 = success); the instance
 *     count is written to *num_rendered;
 *   - gradient outputs are fully written by the backward (no pre-zeroing
 *     needed); forward image outputs are written for every pixel
 *     (mdepth/normal are written as 0 when require_depth == 0).
 * All pointers are DEVICE pointers to contiguous fp32 / int32 arrays with the
 * reference's layouts: means3D [P,3], opacities [P,1], scales [P,3],
 * rotations [P,4] (r,x,y,z), shs [P,SHM,3], sg_axis [P,SGM,3],
 * sg_sharpness [P,SGM], sg_color [P,SGM,3], colors_precomp [P,3],
 * cov3D_precomp [P,6], viewmatrix/projmatrix [16] column-major, campos [3],
 * background [3]; images are planar [C,H,W].  Optional inputs may be NULL
 * (colors_precomp xor shs; scales+rotations xor cov3D_precomp).
 */
#ifndef GSR_H_INCLUDED
#define GSR_H_INCLUDED

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum gsr_status {
    GSR_OK = 0,
    GSR_ERR_ARGS = 1,   /* invalid argument combination or shape */
    GSR_ERR_ALLOC = 2,  /* an allocation callback returned NULL */
    GSR_ERR_HIP = 3,    /* a HIP runtime / launch error (message: gsr_last_error) */
};

/* Replaces std::function<char*(size_t)> (rasterizer.h:30-33, rasterize_points.cu:27-37). */
typedef void* (*gsr_alloc_fn)(void* ctx, size_t bytes);

/*
 * Replaces CudaRasterizer::Rasterizer::forward (rasterizer.h:29-61,
 * rasterizer_impl.cu:285-448).  radii may be NULL (kept internally).
 */
int gsr_rasterize_forward(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                          gsr_alloc_fn image_alloc, void* image_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                          int P, int sh_degree, int SHM, int sg_degree, int SGM, const float* background, int width,
                          int height, const float* means3D, const float* colors_precomp, const float* opacities,
                          const float* scales, const float* rotations, const float* cov3D_precomp,
                          const float* shs, const float* sg_axis, const float* sg_sharpness, const float* sg_color,
                          float scale_modifier, const float* viewmatrix, const float* projmatrix,
                          const float* cam_pos, float tan_fovx, float tan_fovy, float kernel_size, int prefiltered,
                          float* out_color, float* out_mdepth, float* out_alpha, float* out_normal, int* radii,
                          int require_depth, int debug, void* stream, int* num_rendered);

/*
 * Replaces CudaRasterizer::Rasterizer::backward (rasterizer.h:63-109,
 * rasterizer_impl.cu:452-592).  geom/binning/image/tile buffers are the ones
 * the forward obtained from its callbacks; R is the forward's num_rendered.
 * Output gradients (all fully overwritten): dL_dmean3D [P,3],
 * dL_dmean2D [P,3] (x, y, and the |.|-sum channel, render_backward.cu:1028),
 * dL_dcolor [P,3], dL_dopacity [P,1], dL_dscale [P,3], dL_drot [P,4],
 * dL_dcov3D [P,6], dL_dsh [P,SHM,3], dL_dsg_axis [P,SGM,3],
 * dL_dsg_sharpness [P,SGM], dL_dsg_color [P,SGM,3].
 */
int gsr_rasterize_backward(gsr_alloc_fn geom_bwd_alloc, void* geom_bwd_ctx, int P, int sh_degree, int SHM,
                           int sg_degree, int SGM, int R, const float* background, int width, int height,
                           const float* means3D, const float* colors_precomp, const float* opacities,
                           const float* scales, const float* rotations, const float* cov3D_precomp,
                           const float* shs, const float* sg_axis, const float* sg_sharpness,
                           const float* sg_color, float scale_modifier, const float* viewmatrix,
                           const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                           float kernel_size, const int* radii, const float* alphas, const float* normalmap,
                           const float* mdepth, const void* geom_buffer, const void* binning_buffer,
                           const void* image_buffer, const void* tile_buffer, const float* dL_dpix,
                           const float* dL_dpix_mdepth, const float* dL_dalphas, const float* dL_dpixel_normals,
                           float* dL_dmean3D, float* dL_dmean2D, float* dL_dcolor, float* dL_dopacity,
                           float* dL_dscale, float* dL_drot, float* dL_dcov3D, float* dL_dsh, float* dL_dsg_axis,
                           float* dL_dsg_sharpness, float* dL_dsg_color, int require_depth, int debug,
                           void* stream);

/* Replaces CudaRasterizer::Rasterizer::markVisible (rasterizer.h:21-27,
 * rasterizer_impl.cu:186-197): present[i] = (view-space z > 0.2). */
int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream);

/*
 * Per-stage GPU timing (no reference equivalent; SURVEY §5 "tracing").  While
 * enabled, every kernel stage of the calls above is bracketed by two hipEvents
 * on the call's stream.  gsr_timing_collect() waits for the recorded events,
 * adds each stage's total milliseconds and launch count into the caller's
 * arrays (length GSR_NUM_STAGES, indexed by enum gsr_stage) and clears the
 * record.  Process-wide, thread-safe.
 */
enum gsr_stage {
    GSR_STAGE_PREPROCESS = 0,
    GSR_STAGE_SCAN,
    GSR_STAGE_EMIT_KEYS, /* (grids > 1024 tiles a side) instance emission for the tile-id sort */
    GSR_STAGE_SORT,      /* (grids > 1024 tiles a side) stable tile-id sort */
    GSR_STAGE_TILE_RANGES, /* (grids > 1024 tiles a side) */
    GSR_STAGE_RENDER_FWD,
    GSR_STAGE_BWD_CLEAR,
    GSR_STAGE_RENDER_BWD,
    GSR_STAGE_PREPROCESS_BWD,
    GSR_STAGE_DEPTH_ORDER, /* stable depth sort of the Gaussians (binning.hip) */
    GSR_STAGE_TILE_LISTS,  /* per-tile lists without an instance sort (tilelists.hip; grids <= 1024^2 tiles) */
    GSR_NUM_STAGES
};
int gsr_timing_enable(int on);
int gsr_timing_collect(double* ms, int* launches);
const char* gsr_stage_name(int stage);

/*
 * Process-wide switches selecting A/B variants of a kernel, for measuring one
 * against the other in the same process (all variants give bit-identical
 * results).  GSR_OPT_BISECT_SKIP (default 0): exact shortcut for bisection
 * samples far from a Gaussian's ray peak (render_fwd.hip; slower on the
 * fog-like benchmark scene, where most samples are near a peak).
 */
/* GSR_OPT_BISECT_PASSES (diagnostic, default 0 = all 5): run only n median-depth
 * bisection passes (n < 0: none) to time them; median depth is then wrong. */
/* GSR_OPT_BWD_NO_PREPASS (diagnostic): skip the backward's median-depth pre-pass
 * (its gradient terms are then wrong), to time it. */
enum gsr_option {
    GSR_OPT_BISECT_SKIP = 0,
    GSR_OPT_RENDER_STATS = 1,
    GSR_OPT_BISECT_PASSES = 2,
    GSR_OPT_BWD_NO_PREPASS = 3
};
int gsr_set_option(int opt, int value);
/* Diagnostic counters of GSR_OPT_RENDER_STATS forward launches (8 values, see render_fwd.hip). */
int gsr_debug_render_stats(unsigned long long* out8, int reset);

/*
 * Introspection of a forward's opaque buffers (test hook, no reference
 * equivalent): copies the per-tile depth-ordered Gaussian list (R entries,
 * R = num_rendered) and the tile ranges (2 x tiles uint32, tiles =
 * ceil(W/16) * ceil(H/16)) to host memory; synchronises `stream`.
 */
int gsr_debug_binning(const void* binning_buffer, const void* tile_buffer, int R, int width, int height,
                      uint32_t* point_list_out, uint32_t* ranges_out, void* stream);

/* Human-readable message for the last non-OK status on this thread. */
const char* gsr_last_error(void);

/* ABI version of this header (bumped on any signature or enum change). */
int gsr_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H_INCLUDED */
