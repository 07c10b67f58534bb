// gsr_kernels.h — internal launch interface between the C-ABI host code
// (gsr_api.hip) and the kernels.  Not part of the public ABI (include/gsr.h).
#pragma once

#include "gsr_common.h"

namespace gsr {

// Run-time switches for A/B variants of one kernel in one process
// (gsr_set_option in include/gsr.h); defaults are the shipped paths.
// ids 0, 7 and 8 belonged to retired A/B variants (bisection shortcut, per-tile
// sort binning, two-wave backward); gsr_set_option rejects them
enum Option : int { kOptRenderStats = 1, kOptNoRefine = 5, kOptBwdNoCache = 6, kOptRocprimDsort = 9, kOptPbwdStage = 10, kNumOptions = 11 };
inline bool option_retired(int opt) { return opt == 0 || (opt >= 2 && opt <= 4) || opt == 7 || opt == 8; }
int option(int which);
hipError_t read_render_stats(unsigned long long* out, bool reset);

struct FwdParams {
    int P, D, SHM, SGD, SGM, W, H;
    const float* background;
    const float* means3D;
    const float* colors_precomp;
    const float* opacities;
    const float* scales;
    const float* rotations;
    const float* cov3D_precomp;
    const float* shs;
    const float* sg_axis;
    const float* sg_sharpness;
    const float* sg_color;
    const float* shs_rest = nullptr;  // split SH rows: shs holds [P][3] DC rows, shs_rest [P][SHM-1][3]
    float scale_modifier;
    const float* view;
    const float* proj;
    const float* campos;
    float tan_fovx, tan_fovy, focal_x, focal_y, kernel_size;
    uint32_t grid_x, grid_y;
    bool require_depth;
    bool no_color;   // sample_depth: preprocess skips the colour (rasterizer_impl.cu:1080)
    float cull_pad;  // tile-culling pad in pixels (tiles.h): 0 render, 0.5 sample_depth
};

struct BwdParams {
    FwdParams f;
    int R;
    const int* radii;
    const float* alphas;
    const float* normalmap;
    const float* mdepth;
    const float* dL_dpix;
    const float* dL_dmdepth;
    const float* dL_dalpha;
    const float* dL_dnormal;
    float* dL_dmean3D;
    float* dL_dmean2D;
    float* dL_dcolor;
    float* dL_dopacity;
    float* dL_dscale;
    float* dL_drot;
    float* dL_dcov3D;
    float* dL_dsh;
    float* dL_dsg_axis;
    float* dL_dsg_sharpness;
    float* dL_dsg_color;
    float* dL_dsh_rest = nullptr;  // split SH rows (f.shs_rest): dL_dsh [P][3], dL_dsh_rest [P][SHM-1][3]
};

// preprocess_fwd.hip
hipError_t launch_preprocess_fwd(const FwdParams& p, const GeomState& gs, int* radii, hipStream_t stream);

// binning.hip
size_t scan_temp_bytes(int P);
size_t depth_sort_temp_bytes(int P);
size_t sort_temp_bytes(int K, int tile_bits);
hipError_t launch_depth_sort(const GeomState& gs, int P, bool prepared, hipStream_t stream);
// dsort.hip
size_t dsort_temp_bytes(int P);
void dsort_zero_region(void* base, int P, uint32_t** first, size_t* words);
// K into gs.offsets_K and, with `hist`, the depth-key digit histograms (both zeroed by the preprocess)
hipError_t launch_count_k_hist(const GeomState& gs, int P, bool hist, hipStream_t stream);
// `prepared`: state zeroed and histograms counted by the two kernels above
hipError_t launch_dsort(const GeomState& gs, int P, bool prepared, hipStream_t stream);
hipError_t launch_live_counts(const FwdParams& p, const GeomState& gs, const int* radii, hipStream_t stream);
hipError_t launch_scan(const GeomState& gs, int P, hipStream_t stream);
hipError_t launch_emit_keys(const FwdParams& p, const GeomState& gs, const int* radii, const BinningState& bs,
                            hipStream_t stream);
hipError_t launch_sort(const BinningState& bs, int K, int tile_bits, hipStream_t stream);
hipError_t launch_tile_ranges(const BinningState& bs, int K, const TileState& ts, int tiles, hipStream_t stream);

// tilelists.hip
bool list_binning(uint32_t gx, uint32_t gy);
ListLayout list_layout(int P, int K, uint32_t gx, uint32_t gy);
size_t reduce_temp_bytes(int P);
hipError_t launch_list_binning(const FwdParams& p, const GeomState& gs, const int* radii, const BinningState& bs,
                               const TileState& ts, int K, hipStream_t stream);


// render_fwd.hip
hipError_t launch_render_fwd(const FwdParams& p, const GeomState& gs, const BinningState& bs, const ImageState& is,
                             const TileState& ts, float* out_color, float* out_alpha, float* out_normal,
                             float* out_mdepth, hipStream_t stream);

// render_bwd.hip
hipError_t launch_render_bwd(const BwdParams& b, const GeomState& gs, const BinningState& bs, const ImageState& is,
                             const TileState& ts, const BwdState& ws, hipStream_t stream);

// preprocess_bwd.hip
// Gaussians [begin, end) (end < 0: all P); dc_rows non-null: factored view-parallel mode
// (preprocess_bwd.hip PreprocessBwdArgs::dc_rows)
hipError_t launch_preprocess_bwd(const BwdParams& b, const GeomState& gs, const BwdState& ws, hipStream_t stream,
                                 int begin = 0, int end = -1, float* dc_rows = nullptr);

// render_fwd.hip: the forward raster in SAMPLE mode (median depth at points)
// point queries answered by the forward raster in SAMPLE mode
enum { kQuerySample = 0, kQueryIntegrate = 1, kQuerySDF = 2 };
// sample_depth: out0 = points [PN][3]; integrate: out0 = transmittance [PN];
// evaluate_sdf: out0 = median depth [PN], out1 = sdf [PN]
hipError_t launch_point_fwd(int query, const FwdParams& p, const GeomState& gs, const BinningState& bs,
                            const TileState& ts, const PointState& ps, const PointBinState& pb, const SampleTiles& st,
                            const ChunkState& cs, uint32_t num_chunks, float* out0, float* out1, uint8_t* out_inside,
                            hipStream_t stream);

// sample.hip
size_t point_sort_temp_bytes(int PN, uint32_t tiles);
hipError_t launch_sample_points(const FwdParams& p, int PN, const float* points3D, const PointState& ps,
                                const PointBinState& pb, const SampleTiles& st, hipStream_t stream);
hipError_t launch_sample_setup(int PN, uint32_t tiles, const PointBinState& pb, const SampleTiles& st,
                               hipStream_t stream);
struct SampleBwdParams {
    FwdParams f;
    int PN;
    const float* points3D;
    const uint8_t* inside;
    const float* dL_doutput;
    float* dL_dpoints3D;
};
hipError_t launch_sample_bwd(const SampleBwdParams& b, const GeomState& gs, const BinningState& bs,
                             const TileState& ts, const PointState& ps, const PointBinState& pb,
                             const SampleTiles& st, const ChunkState& cs, const BwdState& ws, hipStream_t stream);

// optim.hip: multi-tensor Adam step and densification statistics
constexpr int kMaxAdamGroups = 16;
struct AdamGroup {
    float* param;
    const float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    long long n;
    int aligned;  // all four pointers 16-B aligned: float4 path
};
hipError_t launch_adam(int n_groups, const AdamGroup* groups, const double* lr, double step, double beta1,
                       double beta2, double eps, hipStream_t stream);
// view_grads.hip: a view-parallel step's SH / SG gradients from the gathered DC rows
hipError_t launch_view_color_grads(int P, int D, int SHM, int SGD, int SGM, int n_views, const float* gathered,
                                   const float* means3D, const float* sg_axis, const float* sg_sharpness,
                                   const float* sg_color, float* dL_dsh, float* dL_dsg_axis, float* dL_dsg_sharpness,
                                   float* dL_dsg_color, hipStream_t stream, int chunk = 0,
                                   const float* campos = nullptr, float* dL_dsh_rest = nullptr);
hipError_t launch_densify_stats(int P, const float* vgrad, const int* radii, float* max_radii2D, float* accum,
                                float* accum_abs, float* denom, hipStream_t stream);

// ncc.hip: warp-patch NCC with forward-mode gradients
struct NccParams {
    int P;
    const float* depths;
    const float* normals;
    const int* uvs;
    const float* R;
    const float* T;
    const float* image_r;
    const float* image_n;
    float fx_r, fy_r, cx_r, cy_r, fx_n, fy_n, cx_n, cy_n;
    int Hr, Wr, Hn, Wn;
    float* ncc;
    float* grad_depths;
    float* grad_normals;
    uint8_t* valid;
};
hipError_t launch_ncc(const NccParams& q, hipStream_t stream);

// optim.hip: the activation getters of training (gsr_scale_opacity_3d_filter*, gsr_normalize_rows*)
hipError_t launch_scale_opacity(int P, const float* s, const float* o, const float* f, float* scales, float* opac,
                                const float* gS, const float* gO, float* ds, float* dop, bool backward,
                                hipStream_t stream);
hipError_t launch_normalize_rows(int n, int D, const float* x, const float* gy, float* out, bool backward,
                                 hipStream_t stream);

// ncc.hip: the fused PatchMatch terms of training (gsr_patchmatch_*)
struct PatchMatchParams {
    int H, W;               // the view (reference image of the NCC)
    const float* md;        // [H*W]
    const float* normal;    // [3, H*W]
    const float* pin;       // [H*W, 3]
    const uint8_t* inside;  // [H*W]
    const float* Mv;        // [9] row-major
    const float* tv;        // [3]
    float Fx, Fy, Cx, Cy;
    float noise_th;
    const float* R;  // [9] NCC rotation (the reference's column-major float33), T [3]
    const float* T;
    const float* image_r;
    const float* image_n;
    float fx_r, fy_r, cx_r, cy_r, fx_n, fy_n, cx_n, cy_n;
    int Hn, Wn;
    float* w;
    uint8_t* flags;
    float* gd;
    float* gn;
};
size_t patchmatch_partials(int H, int W);
hipError_t launch_patchmatch_terms(const PatchMatchParams& q, float* partial, float* out, hipStream_t stream);
hipError_t launch_patchmatch_terms_bwd(const PatchMatchParams& q, const float* out, const float* dL_dloss,
                                       float* dL_dpin, float* dL_dmd, float* dL_dnormal, hipStream_t stream);
hipError_t launch_patchmatch_lift(bool backward, int H, int W, float Fx, float Fy, float Cx, float Cy, const float* T,
                                  const float* M, const float* md, const float* gpts, float* out, hipStream_t stream);

// ssim.hip: fused SSIM forward / backward
size_t ssim_partials(int NC, int H, int W);
hipError_t launch_ssim_fwd(int NC, int H, int W, int valid, const float* img1, const float* img2, float* fA,
                           float* fB, float* fC, float* partial, float* out, hipStream_t stream);
hipError_t launch_ssim_bwd(int NC, int H, int W, int valid, const float* img1, const float* img2, const float* fA,
                           const float* fB, const float* fC, const float* dL_dloss, float* dL_dimg1,
                           hipStream_t stream);

// depth_normal.hip: normal map of a depth map and its backward
hipError_t launch_depth_normal(bool backward, const float* depth, int H, int W, float Fx, float Fy, float Cx, float Cy,
                               const float* g, float* out, uint8_t* valid, hipStream_t stream);

// mark visible
hipError_t launch_near_violation(int P, const float* means3D, const float* view, uint32_t* flag,
                                 hipStream_t stream);
hipError_t launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present,
                               hipStream_t stream);

// distCUDA2 (knn.hip): scratch carved from one caller buffer
struct KnnState {
    float* partials;
    float* bounds;
    uint32_t* codes;
    uint32_t* codes_sorted;
    uint32_t* order;
    float4* sorted;
    float4* boxes;
    char* sort_tmp;
    size_t sort_tmp_bytes;
};
size_t carve_knn(void* base, int P, KnnState& s);
hipError_t launch_knn(int P, const float* pts, const KnnState& s, float* mean_dists, hipStream_t stream);

// Launch order of the per-tile raster kernels, heaviest tile first (longest-
// processing-time-first list scheduling: the tail of a launch is then made
// of short tiles).  Cost = the tile's list length (ranges, forward) or its
// max contributor (backward); one 1024-lane workgroup.
hipError_t launch_tile_order(uint32_t num_tiles, const uint2* ranges, const uint32_t* max_contrib, uint32_t* order,
                             hipStream_t stream);
// the tile order (workgroup 0) and the clearing of [zero, zero + zero_bytes)
// (16-B aligned and sized) in one launch
hipError_t launch_bwd_prepare(void* zero, size_t zero_bytes, uint32_t num_tiles, const uint32_t* max_contrib,
                              uint32_t* order, hipStream_t stream);
// the same for sample_depth's point chunks (count *n_dev <= bound, cost = chunk max contributor)
hipError_t launch_chunk_order(uint32_t bound, const uint32_t* n_dev, const uint32_t* chunk_max, uint32_t* order,
                              hipStream_t stream);
uint32_t sample_chunk_bound(int PN, uint32_t tiles);

}  // namespace gsr
