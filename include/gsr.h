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
/* Host callback of gsr_rasterize_backward_ex after each Gaussian range [begin, end) of the
 * per-Gaussian backward has been queued on the call's stream. */
typedef void (*gsr_chunk_fn)(void* ctx, int begin, int end);

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
 * gsr_rasterize_forward with a fifth allocator for the forward-only scratch
 * (the depth-sort / scan temporaries and the tile-list building state: at 1M
 * Gaussians and 1080p about 0.25 GB that the reference keeps inside the saved
 * geometry / binning buffers until the backward).  scratch_alloc may be called
 * more than once per call; every block it returns must stay valid until the
 * call returns, and may be released then (stream-ordered: the kernels that use
 * it are queued on `stream`).  scratch_alloc == NULL is gsr_rasterize_forward.
 * The buffers the backward reads have the same layout either way.
 */
int gsr_rasterize_forward_ex(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                             gsr_alloc_fn image_alloc, void* image_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                             int P, int sh_degree, int SHM, int sg_degree, int SGM, const float* background, int width,
                             int height, const float* means3D, const float* colors_precomp, const float* opacities,
                             const float* scales, const float* rotations, const float* cov3D_precomp,
                             const float* shs, const float* sg_axis, const float* sg_sharpness, const float* sg_color,
                             float scale_modifier, const float* viewmatrix, const float* projmatrix,
                             const float* cam_pos, float tan_fovx, float tan_fovy, float kernel_size, int prefiltered,
                             float* out_color, float* out_mdepth, float* out_alpha, float* out_normal, int* radii,
                             int require_depth, int debug, void* stream, int* num_rendered,
                             gsr_alloc_fn scratch_alloc, void* scratch_ctx);

/*
 * Replaces CudaRasterizer::Rasterizer::backward (rasterizer.h:63-109,
 * rasterizer_impl.cu:452-592).  geom/binning/image/tile buffers are the ones
 * the forward obtained from its callbacks; R is the forward's num_rendered.
 * Output gradients (all fully overwritten): dL_dmean3D [P,3],
 * dL_dmean2D [P,3] (x, y, and the |.|-sum channel, render_backward.cu:1028),
 * dL_dcolor [P,3], dL_dopacity [P,1], dL_dscale [P,3], dL_drot [P,4],
 * dL_dcov3D [P,6], dL_dsh [P,SHM,3], dL_dsg_axis [P,SGM,3],
 * dL_dsg_sharpness [P,SGM], dL_dsg_color [P,SGM,3].
 * An upstream image gradient (dL_dpix, dL_dpix_mdepth, dL_dalphas,
 * dL_dpixel_normals) may be NULL for an output the loss does not use: it is
 * then zero (no reference equivalent; the autograd wrapper passes None
 * instead of materialising zero images).
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

/*
 * gsr_rasterize_backward with the per-Gaussian backward split into `chunks`
 * consecutive Gaussian ranges (no reference equivalent: the view-parallel
 * training step).  After each range's kernel is queued on
 * `stream`, on_chunk(chunk_ctx, begin, end) runs on the calling thread, so
 * the caller can post that range's gradient exchange on another stream while
 * the next range computes (gsr_dist.OverlappedViewGrads).  The ranges hold
 * ceil(ceil(P / chunks) / 256) * 256 Gaussians each (the last one fewer).  With dc_rows
 * non-NULL ([P][3] floats, SH colour path only) the kernel writes each
 * Gaussian's DC gradient row dL/dsh[:, 0, :] there and leaves dL_dsh and the
 * SG gradient rows unwritten: gsr_view_color_grads_chunked rebuilds them from
 * every view's DC rows.  chunks = 1, on_chunk = NULL, dc_rows = NULL is
 * gsr_rasterize_backward.
 */
int gsr_rasterize_backward_ex(gsr_alloc_fn geom_bwd_alloc, void* geom_bwd_ctx, int P, int sh_degree, int SHM,
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
                              int chunks, gsr_chunk_fn on_chunk, void* chunk_ctx, float* dc_rows, void* stream);

/*
 * The split SH layout of training (round 5): GaussianModel keeps the DC and
 * the higher-order SH coefficients as two tensors (_features_dc [P,1,3],
 * _features_rest [P,SHM-1,3]) and get_features concatenates them every call
 * (scene/gaussian_model.py:165-169: 192 MB at 1M Gaussians, and the
 * gradient's split in the backward).  These two entry points take them as
 * they are: `shs` is then the DC rows [P][3] and `shs_rest` the rest
 * [P][SHM-1][3] (SHM counts all coefficients, as before); the backward writes
 * dL_dsh [P][3] and dL_dsh_rest [P][SHM-1][3].  NULL shs_rest is exactly
 * the _ex call.  With dc_rows (the overlapped exchange, ABI 20) neither SH
 * gradient tensor is written: gsr_view_color_grads_chunked rebuilds both.
 */
int gsr_rasterize_forward_ex2(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                              gsr_alloc_fn image_alloc, void* image_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                              int P, int sh_degree, int SHM, int sg_degree, int SGM, const float* background,
                              int width, int height, const float* means3D, const float* colors_precomp,
                              const float* opacities, const float* scales, const float* rotations,
                              const float* cov3D_precomp, const float* shs, const float* sg_axis,
                              const float* sg_sharpness, const float* sg_color, float scale_modifier,
                              const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                              float tan_fovy, float kernel_size, int prefiltered, float* out_color, float* out_mdepth,
                              float* out_alpha, float* out_normal, int* radii, int require_depth, int debug,
                              void* stream, int* num_rendered, gsr_alloc_fn scratch_alloc, void* scratch_ctx,
                              const float* shs_rest);
int gsr_rasterize_backward_ex2(gsr_alloc_fn geom_bwd_alloc, void* geom_bwd_ctx, int P, int sh_degree, int SHM,
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
                               int chunks, gsr_chunk_fn on_chunk, void* chunk_ctx, float* dc_rows, void* stream,
                               const float* shs_rest, float* dL_dsh_rest);

/* The Gaussian range size gsr_rasterize_backward_ex uses for `chunks` ranges
 * of P Gaussians: ceil(ceil(P / chunks) / 256) * 256 (whole 256-Gaussian
 * workgroups; the last range holds the rest).  The range-major layout of the
 * gathered DC rows (gsr_view_color_grads_chunked) depends on it, so callers
 * take it from here.  -1 for P < 0 or chunks < 1.  Host only. */
int gsr_backward_chunk_size(int P, int chunks);

/* Replaces CudaRasterizer::Rasterizer::markVisible (rasterizer.h:21-27,
 * rasterizer_impl.cu:186-197): present[i] = (view-space z > 0.2). */
int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream);

/*
 * sample_depth: the median depth of the Gaussian field
 * at PN arbitrary world points seen from one camera — the multi-view
 * geometric-consistency term of the reference's training loss
 * (utils/loss_utils.py:160, gaussian_renderer/__init__.py:225-278).
 *
 * Replaces CudaRasterizer::Rasterizer::sampleDepth (rasterizer.h:170-195,
 * rasterizer_impl.cu:1042-1245), bound as _C.sample_rasterized_depth
 * (DGR/ext.cpp:21, rasterize_points.cu:459-553).  The six resize callbacks
 * are the reference's geometry, binning, point, point-binning, tile and
 * duplicated-tile buffers.  points3D [PN,3]; output [PN,3] is the
 * camera-space point (x, y, z) at the median depth along its ray and
 * inside [PN] (uint8) whether the median is defined; both are written for the
 * points that project into the image and left untouched for the others (the
 * reference zero-initialises them, so callers pass zeroed buffers).
 * kernel_size is whatever the caller passes: the reference's Python wrapper
 * passes 0.0 here (DGR/__init__.py:500-518) and the settings' value to the
 * backward.  Synchronises `stream` once (K, valid points, block count).
 * *num_points = points that project into the image, *num_duplicated_tiles =
 * the reference's count of 512-point blocks (both opaque to callers; the
 * backward ignores them).
 */
int gsr_sample_depth_forward(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                             gsr_alloc_fn point_alloc, void* point_ctx, gsr_alloc_fn point_binning_alloc,
                             void* point_binning_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                             gsr_alloc_fn dup_tile_alloc, void* dup_tile_ctx, int PN, int P, int width, int height,
                             const float* points3D, const float* means3D, const float* opacities,
                             const float* scales, float scale_modifier, const float* rotations,
                             const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                             const float* cam_pos, float tan_fovx, float tan_fovy, float kernel_size,
                             int prefiltered, float* output, uint8_t* inside, int debug, void* stream,
                             int* num_rendered, int* num_points, int* num_duplicated_tiles);

/* gsr_sample_depth_forward with the forward-only scratch allocator of
 * gsr_rasterize_forward_ex (same contract; the saved buffers keep their layout). */
int gsr_sample_depth_forward_ex(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc,
                                void* binning_ctx, gsr_alloc_fn point_alloc, void* point_ctx,
                                gsr_alloc_fn point_binning_alloc, void* point_binning_ctx, gsr_alloc_fn tile_alloc,
                                void* tile_ctx, gsr_alloc_fn dup_tile_alloc, void* dup_tile_ctx, int PN, int P,
                                int width, int height, const float* points3D, const float* means3D,
                                const float* opacities, const float* scales, float scale_modifier,
                                const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                                const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                                float kernel_size, int prefiltered, float* output, uint8_t* inside, int debug,
                                void* stream, int* num_rendered, int* num_points, int* num_duplicated_tiles,
                                gsr_alloc_fn scratch_alloc, void* scratch_ctx);

/*
 * integrate / evaluate_sdf: forward-only queries of the
 * Gaussian field at PN world points, used by the offline tetrahedral mesh
 * extraction (mesh_extract_tetrahedra.py:75, gaussian_renderer/__init__.py:
 * 101-222).  Same six resize callbacks, arguments and point binning as
 * gsr_sample_depth_forward; view2gaussian_precomp is accepted and ignored, as
 * in the reference.  Outputs are written for the points that project into
 * the image and left untouched for the others (callers pass zeroed buffers,
 * as the reference's torch::full(0)).  Synchronises `stream` once.
 *
 * gsr_integrate_forward replaces CudaRasterizer::Rasterizer::
 * evaluateTransmittance (rasterizer.h:111-138, rasterizer_impl.cu:594-815),
 * bound as _C.integrate_gaussians_to_points (DGR/rasterize_points.cu:279-366):
 * out_transmittance [PN] = the vacancy transmittance at each point's distance
 * from the camera (sample_forward.cu:55-169), inside [PN] = 1.
 *
 * gsr_evaluate_sdf_forward replaces Rasterizer::evaluateSDF (rasterizer.h:
 * 140-168, rasterizer_impl.cu:817-1040), bound as
 * _C.evaluate_sdf_from_signle_view (rasterize_points.cu:368-457):
 * out_depth [PN] = the median depth along the point's ray (+-0.8 first
 * window, 6 bisection passes, sample_forward.cu:171-427), out_sdf [PN] =
 * out_depth - |p_view|, inside [PN] = whether the median is defined.
 */
int gsr_integrate_forward(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                          gsr_alloc_fn point_alloc, void* point_ctx, gsr_alloc_fn point_binning_alloc,
                          void* point_binning_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                          gsr_alloc_fn dup_tile_alloc, void* dup_tile_ctx, int PN, int P, int width, int height,
                          const float* points3D, const float* means3D, const float* opacities, const float* scales,
                          float scale_modifier, const float* rotations, const float* cov3D_precomp,
                          const float* view2gaussian_precomp, const float* viewmatrix, const float* projmatrix,
                          const float* cam_pos, float tan_fovx, float tan_fovy, float kernel_size, int prefiltered,
                          float* out_transmittance, uint8_t* inside, int debug, void* stream, int* num_rendered);
int gsr_evaluate_sdf_forward(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                             gsr_alloc_fn point_alloc, void* point_ctx, gsr_alloc_fn point_binning_alloc,
                             void* point_binning_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                             gsr_alloc_fn dup_tile_alloc, void* dup_tile_ctx, int PN, int P, int width, int height,
                             const float* points3D, const float* means3D, const float* opacities,
                             const float* scales, float scale_modifier, const float* rotations,
                             const float* cov3D_precomp, const float* view2gaussian_precomp,
                             const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                             float tan_fovy, float kernel_size, int prefiltered, float* out_depth, float* out_sdf,
                             uint8_t* inside, int debug, void* stream, int* num_rendered);

/*
 * Replaces CudaRasterizer::Rasterizer::sampleDepthBackward (rasterizer.h:197-233,
 * rasterizer_impl.cu:1247-1394), bound as _C.sample_rasterized_depth_backward
 * (rasterize_points.cu:555-633).  The six buffers are the forward's; R, RN, TN
 * its three counts.  Gradients written: dL_dopacity [P,1], dL_dmean3D [P,3],
 * dL_dscale [P,3] + dL_drot [P,4] (scale/rotation path) or dL_dcov3D [P,6]
 * (precomputed covariance), all fully overwritten; dL_dpoints3D [PN,3] is
 * written for the points that project into the image only (callers pass a
 * zeroed buffer, as the reference's torch::zeros_like).
 */
int gsr_sample_depth_backward(gsr_alloc_fn geom_bwd_alloc, void* geom_bwd_ctx, int PN, int P, int RN, int R, int TN,
                              int width, int height, const float* points3D, const float* means3D,
                              const float* opacities, const float* scales, float scale_modifier,
                              const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                              const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                              float kernel_size, const void* geom_buffer, const void* binning_buffer,
                              const void* point_buffer, const void* point_binning_buffer, const void* tile_buffer,
                              const void* dup_tile_buffer, const uint8_t* inside, const float* dL_doutput,
                              float* dL_dopacity, float* dL_dmean3D, float* dL_dcov3D, float* dL_dscale,
                              float* dL_drot, float* dL_dpoints3D, int debug, void* stream);

/*
 * Training update.  One Adam step over up to 16
 * parameter groups in a single launch — torch.optim.Adam's update with its
 * rounding order (scene/gaussian_model.py:347-351 builds it with eps 1e-15;
 * train.py:259-261 steps it), every group at the same step count `step`
 * (>= 1, the value after increment) with its own learning rate.  Groups are
 * flat fp32 arrays of n elements; param, exp_avg and exp_avg_sq are updated
 * in place.
 */
typedef struct {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    long long n;
    double lr;
} gsr_adam_group;
/* lr, betas and eps are doubles, like the Python floats torch combines them
 * in before rounding to fp32 (e.g. 1 - beta2). */
int gsr_adam_step(int n_groups, const gsr_adam_group* groups, double step, double beta1, double beta2, double eps,
                  void* stream);

/*
 * GaussianModel.add_densification_stats + the max_radii2D update
 * (scene/gaussian_model.py:818-821, train.py:236-237) for the P Gaussians
 * with radii > 0: max_radii2D = max(max_radii2D, radii), accum += |vgrad.xy|,
 * accum_abs += |vgrad.z|, denom += 1.  vgrad [P,3] is the viewspace-points
 * gradient (dL/dmeans2D of the backward); the four statistics are [P] fp32.
 */
int gsr_densify_stats(int P, const float* vgrad, const int* radii, float* max_radii2D, float* accum,
                      float* accum_abs, float* denom, void* stream);

/*
 * View-parallel training (no reference equivalent: the
 * reference trains one view per step on one GPU).  The SH / SG gradient rows
 * of a step summed over n_views views, rebuilt from each view's DC gradient
 * row and camera centre (view_grads.hip): per view the colour backward
 * (CR/render_backward.cu:56-191) makes every row a function of the
 * clamp-masked dL/dRGB = dL/dsh[:, 0, :] / SH_C0 and the view direction.
 * gathered: [n_views][P * 3 + 4] fp32, view v's dL/dsh[:, 0, :] (P x 3)
 * followed by its camera centre (3) and one pad float.  Outputs are
 * overwritten: dL_dsh [P, SHM, 3] (rows past (sh_degree + 1)^2 zero), and
 * when SGM > 0 dL_dsg_axis [P, SGM, 3], dL_dsg_sharpness [P, SGM],
 * dL_dsg_color [P, SGM, 3] (lobes past sg_degree zero); sg_degree <= 7.
 */
/*
 * gsr_view_color_grads for the layout gsr_dist.OverlappedViewGrads gathers
 * range by range: the Gaussians in ranges of `chunk` (the last shorter);
 * range [b, b + len) occupies gathered[3 n_views b, 3 n_views (b + len)) as
 * [n_views][len][3] DC rows; the camera centres are campos [n_views][4].
 * dL_dsh_rest (ABI 20; NULL: the one-tensor layout): the split SH layout of
 * gsr_rasterize_backward_ex2 — dL_dsh is then the DC rows [P, 1, 3] and
 * dL_dsh_rest the other SHM - 1 rows [P, SHM - 1, 3].
 */
int gsr_view_color_grads_chunked(int P, int sh_degree, int SHM, int sg_degree, int SGM, int n_views, int chunk,
                                 const float* gathered, const float* campos, const float* means3D,
                                 const float* sg_axis, const float* sg_sharpness, const float* sg_color,
                                 float* dL_dsh, float* dL_dsg_axis, float* dL_dsg_sharpness, float* dL_dsg_color,
                                 float* dL_dsh_rest, void* stream);

int gsr_view_color_grads(int P, int sh_degree, int SHM, int sg_degree, int SGM, int n_views, const float* gathered,
                         const float* means3D, const float* sg_axis, const float* sg_sharpness, const float* sg_color,
                         float* dL_dsh, float* dL_dsg_axis, float* dL_dsg_sharpness, float* dL_dsg_color,
                         void* stream);

/*
 * Multi-view photometric term: replaces WarpPatchNCC /
 * forward_mode_differentiation (submodules/warp-patch-ncc/warp_patch_ncc.cu:5-52,
 * cuda_warp_patch_ncc/warp_patch_ncc_impl.cu:18-302), bound as
 * warp_patch_ncc._C.warp_patch_ncc.  For P reference pixels uvs [P,2] (int32)
 * with depths [P], normals [P,3]: the NCC of the 7x7 half-step patch against
 * its homography warp into image_n, and d(NCC)/d(depth) [P],
 * d(NCC)/d(normal) [P,3]; valid [P] (uint8).  R [9] is the r-to-n rotation
 * as the reference's column-major float33, T [3]; images are [H,W] fp32
 * (grey).  Every output element is written.
 */
int gsr_warp_patch_ncc(int P, const float* depths, const float* normals, const int* uvs, const float* R,
                       const float* T, const float* image_r, const float* image_n, float fx_r, float fy_r,
                       float cx_r, float cy_r, float fx_n, float fy_n, float cx_n, float cy_n, int image_height_r,
                       int image_width_r, int image_height_n, int image_width_n, float* ncc, float* grad_depths,
                       float* grad_normals, uint8_t* valid, void* stream);

/*
 * GaussianModel's activation getters (the callers of the
 * rasterizer in training; scene/gaussian_model.py:146-212), one thread per
 * Gaussian.  scale/opacity with the 3D filter
 * (get_scaling_n_opacity_with_3D_filter): scaling [P,3] and opacity [P]
 * are the raw parameters, filter_3D [P]; scales [P,3] = sqrt(exp(s)^2 +
 * f^2), opacities [P] = sigmoid(o) * sqrt(prod exp(s)^2 / prod(exp(s)^2 +
 * f^2)).  The backward writes dL/dscaling, dL/dopacity for dL/dscales,
 * dL/dopacities (either may be NULL: zero).  normalize_rows: y = x /
 * max(|x|, 1e-12) per row of D (get_rotation's F.normalize) and its
 * backward.
 */
int gsr_scale_opacity_3d_filter(int P, const float* scaling, const float* opacity, const float* filter_3D,
                                float* scales, float* opacities, void* stream);
int gsr_scale_opacity_3d_filter_backward(int P, const float* scaling, const float* opacity, const float* filter_3D,
                                         const float* dL_dscales, const float* dL_dopacities, float* dL_dscaling,
                                         float* dL_dopacity, void* stream);
int gsr_normalize_rows(int n, int D, const float* x, float* y, void* stream);
int gsr_normalize_rows_backward(int n, int D, const float* x, const float* dL_dy, float* dL_dx, void* stream);

/*
 * PatchMatch multi-view loss, fused (the training
 * step's caller of sample_depth and warp_patch_ncc): replaces the torch body
 * of PatchMatch.__call__ (utils/loss_utils.py:140-267) around its two
 * extension calls, for one view of H x W pixels and its nearest view.
 *  - lift: points [H*W,3] = (median_depth * ray - T) @ M, ray = ((x - Cx) / Fx,
 *    (y - Cy) / Fy, 1) (:147-153; T = view.T, M = view.R^T, row-major);
 *    backward: dL/dmedian_depth [H*W] for dL/dpoints.
 *  - terms forward: from points_nearest [H*W,3] (sample_depth of the lifted
 *    points in the nearest view) and inside [H*W] (uint8): the reprojection
 *    into the view (point in view = tv + p @ Mv, Mv row-major), the pixel
 *    noise, the geometric mask (inside, both depths > 0.2, noise < noise_th,
 *    median depth > 0) and weight exp(-noise) (:160-221), and at the masked
 *    pixels the NCC (as gsr_warp_patch_ncc, R/T/intrinsics/images likewise) of
 *    the normalised normal [3,H*W] (:228-256).  out4 (device) = {geo_loss,
 *    ncc_loss, d_mask count, ncc_mask count}; a loss over an empty mask is 0
 *    (:223-224).  saved_* ([H*W] w, flags, gd; [H*W,3] gn) are for the
 *    backward.  One scratch allocation (16 B per 256 pixels); no host
 *    synchronisation.
 *  - terms backward: dL/d(points_nearest, median_depth, normal) for
 *    dL/d(geo_loss, ncc_loss) = dL_dloss2 (device, 2 floats).  Every output
 *    element is written.
 */
int gsr_patchmatch_lift(int H, int W, float Fx, float Fy, float Cx, float Cy, const float* T, const float* M,
                        const float* median_depth, float* points, void* stream);
int gsr_patchmatch_lift_backward(int H, int W, float Fx, float Fy, float Cx, float Cy, const float* M,
                                 const float* dL_dpoints, float* dL_dmedian_depth, void* stream);
int gsr_patchmatch_terms_forward(gsr_alloc_fn scratch_alloc, void* scratch_ctx, int H, int W,
                                 const float* median_depth, const float* normal, const float* points_nearest,
                                 const uint8_t* inside, const float* Mv, const float* tv, float Fx, float Fy, float Cx,
                                 float Cy, float noise_th, const float* R, const float* T, const float* image_r,
                                 const float* image_n, float fx_r, float fy_r, float cx_r, float cy_r, float fx_n,
                                 float fy_n, float cx_n, float cy_n, int image_height_n, int image_width_n,
                                 float* saved_w, uint8_t* saved_flags, float* saved_gd, float* saved_gn,
                                 float* out4, void* stream);
int gsr_patchmatch_terms_backward(int H, int W, const float* median_depth, const float* normal,
                                  const float* points_nearest, const uint8_t* inside, const float* Mv, const float* tv,
                                  float Fx, float Fy, float Cx, float Cy, float noise_th, const float* R,
                                  const float* T, const float* image_r, const float* image_n, float fx_r, float fy_r,
                                  float cx_r, float cy_r, float fx_n, float fy_n, float cx_n, float cy_n,
                                  int image_height_n, int image_width_n, const float* saved_w,
                                  const uint8_t* saved_flags, const float* saved_gd, const float* saved_gn,
                                  const float* out4, const float* dL_dloss2, float* dL_dpoints_nearest,
                                  float* dL_dmedian_depth, float* dL_dnormal, void* stream);

/*
 * D-SSIM term: replaces the external fused_ssim(img1,
 * img2, padding) that utils/loss_utils.py:48-49 calls (padding "valid") with
 * the SSIM of the reference's own _ssim (loss_utils.py:36-72): 11 x 11
 * Gaussian window, sigma 1.5, C1 = 1e-4, C2 = 9e-4, zero padding.  Images
 * are NC planes of H x W fp32 (e.g. [1,3,H,W]).  valid != 0 averages over
 * the positions whose window lies inside the image (needs H, W > 10).
 * *out_mean (device) receives the mean SSIM.  factors (device, 3*NC*H*W
 * floats, may be NULL when no gradient is wanted) receives what the backward
 * reads.  The backward writes dL/dimg1 (NC*H*W) for dL/dmean at dL_dmean
 * (device scalar).
 */
int gsr_fused_ssim_forward(gsr_alloc_fn scratch_alloc, void* scratch_ctx, int NC, int H, int W, int valid,
                           const float* img1, const float* img2, float* out_mean, float* factors, void* stream);
int gsr_fused_ssim_backward(int NC, int H, int W, int valid, const float* img1, const float* img2,
                            const float* factors, const float* dL_dmean, float* dL_dimg1, void* stream);

/*
 * Depth-normal consistency input: replaces the torch
 * function depth_to_normal (utils/graphics_utils.py:103-119).  depth [H,W];
 * forward: normal [3,H,W] (zero on the border), valid [H,W] uint8;
 * backward: dL/ddepth [H,W] for dL/dnormal [3,H,W].  Fx, Fy, Cx, Cy are the
 * camera's (scene/cameras.py).
 */
int gsr_depth_to_normal_forward(const float* depth, int H, int W, float Fx, float Fy, float Cx, float Cy,
                                float* normal, uint8_t* valid, void* stream);
int gsr_depth_to_normal_backward(const float* depth, int H, int W, float Fx, float Fy, float Cx, float Cy,
                                 const float* dL_dnormal, float* dL_ddepth, void* stream);

/*
 * Initial scales: replaces distCUDA2 / SimpleKNN::knn
 * (submodules/simple-knn/spatial.cu:15-25, simple_knn.cu:175-220), bound as
 * simple_knn._C.distCUDA2 (scene/gaussian_model.py:20, 323).  points [P,3]
 * fp32; mean_dists [P] = the mean of the squared distances to the 3 nearest
 * other points (inf / FLT_MAX-based values when P < 4, as the reference).
 * scratch_alloc is called once (about 48 B per point plus the sort's
 * temporary).  No host synchronisation.
 */
int gsr_knn_mean_dist(gsr_alloc_fn scratch_alloc, void* scratch_ctx, int P, const float* points, float* mean_dists,
                      void* stream);

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
    GSR_STAGE_SAMPLE_POINTS, /* sample_depth: point projection, per-tile point lists and chunks (sample.hip) */
    GSR_STAGE_SAMPLE_FWD,    /* sample_depth forward raster (render_fwd.hip, SAMPLE mode) */
    GSR_STAGE_SAMPLE_BWD,    /* sample_depth backward raster + point projection backward (sample.hip) */
    GSR_NUM_STAGES
};
int gsr_timing_enable(int on);
/* Restrict the timing to the stages whose bit (1 << enum gsr_stage) is set
 * (default: all).  Each recorded event costs the stream ~10 us of idle time,
 * so a throughput measurement times only the stage it reports. */
int gsr_timing_stage_mask(unsigned int mask);
int gsr_timing_collect(double* ms, int* launches);
const char* gsr_stage_name(int stage);

/*
 * Process-wide switches selecting the alternative kernel paths the parity
 * tests use as references for the default ones (all but GSR_OPT_NO_REFINE
 * give bit-identical results) and the forward's diagnostic counters.  Ids 0,
 * 2-4, 7 and 8 belonged to retired variants and diagnostics (a bisection
 * shortcut, bisection-pass and pre-pass timing switches, an unordered tile
 * launch, per-tile sort binning, a two-wave backward layout) and are rejected
 * with GSR_ERR_ARGS.
 */
/* GSR_OPT_BWD_NO_CACHE (A/B, default 0): the backward recomputes dT/dt_m at every
 * pixel in its pre-pass (render_backward.cu:835-880) instead of taking the
 * forward's cached value. */
/* GSR_OPT_ROCPRIM_DSORT (A/B, default 0): the depth order by rocPRIM's onesweep
 * radix sort instead of dsort.hip's (same order). */
/* GSR_OPT_PBWD_STAGE (A/B): the per-Gaussian backward's SH / SG-7 gradient rows
 * written through LDS as whole-wave stores (1) or per lane (2); 0 = the build's
 * default (GSR_PBWD_STAGE_DEFAULT). */
/* GSR_OPT_NO_REFINE (A/B, default 0): find the median depth with the reference's
 * five bisection passes only, instead of two passes plus the bracketed Halley
 * refinement (render_fwd.hip; results agree to ~1e-7 of the depth, not bitwise). */
enum gsr_option {
    GSR_OPT_RENDER_STATS = 1,
    GSR_OPT_NO_REFINE = 5,
    GSR_OPT_BWD_NO_CACHE = 6,
    GSR_OPT_ROCPRIM_DSORT = 9,
    GSR_OPT_PBWD_STAGE = 10
};
int gsr_set_option(int opt, int value);
/* Diagnostic counters of GSR_OPT_RENDER_STATS forward launches (20 values, see render_fwd.hip). */
int gsr_debug_render_stats(unsigned long long* out20, int reset);

/*
 * Introspection of a forward's opaque buffers (test hook, no reference
 * equivalent): copies the per-tile depth-ordered Gaussian list (R entries,
 * R = num_rendered) and the tile ranges (2 x tiles uint32, tiles =
 * ceil(W/16) * ceil(H/16)) to host memory; synchronises `stream`.
 */
int gsr_debug_binning(const void* binning_buffer, const void* tile_buffer, int R, int width, int height,
                      uint32_t* point_list_out, uint32_t* ranges_out, void* stream);

/*
 * Introspection of a forward's image buffer (test hook): the per-pixel last
 * contributor (1-based index into the pixel's tile list, which holds only the
 * instances that survive tile culling, see gsr_debug_binning), W x H uint32
 * row-major; synchronises `stream`.
 */
int gsr_debug_image(const void* image_buffer, int width, int height, uint32_t* n_contrib_out, void* stream);

/*
 * Introspection of a sample_depth forward's point buffer (test hook): the
 * per-point median depth along the ray and last contributor (index into the
 * culled per-tile list) for PN points; synchronises `stream`.
 */
int gsr_debug_sample_points(const void* point_buffer, int PN, float* median_depth_out, uint32_t* last_out,
                            void* stream);

/*
 * Introspection of a forward's tile buffer (test / measurement hook): the
 * per-tile max contributor (the last list position any pixel of the tile
 * blended, 1-based; the backward walks each tile's list up to it), one
 * uint32 per tile; synchronises `stream`.
 */
int gsr_debug_tile_stats(const void* tile_buffer, int width, int height, uint32_t* max_contrib_out, void* stream);

/* Human-readable message for the last non-OK status on this thread. */
const char* gsr_last_error(void);

/* ABI version of this header (bumped on any signature or enum change). */
int gsr_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H_INCLUDED */
