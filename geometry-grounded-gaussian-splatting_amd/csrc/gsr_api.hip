// gsr_api.hip — the C ABI (include/gsr.h): host orchestration of the gfx950
// kernels, replacing CudaRasterizer::Rasterizer::{forward, backward,
// markVisible} (CR/rasterizer_impl.cu:186-592).
//
// Everything is enqueued on the caller's stream.  The forward synchronises
// that stream exactly once, to read K (the number of Gaussian/tile instances)
// and size the binning buffer, like the reference's cudaMemcpy at
// rasterizer_impl.cu:384.  No other host<->device traffic, no device
// allocation (all scratch comes from the caller's allocation callbacks).
#include <stdio.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/gsr.h"
#include "gsr_kernels.h"

namespace {

thread_local std::string g_last_error;

// The forward's one host synchronisation (K sizes the binning buffer, as
// rasterizer_impl.cu:384) waits on an event recorded right after the counts
// are copied into pinned host memory, not on the whole stream: work queued
// behind the event (the depth sort) keeps the GPU busy while the host reads
// K and allocates.  The pinned words and the event come from a process-wide
// per-device pool: a forward leases a slot for its readback and returns it,
// so slots are created only up to the number of concurrent forwards and are
// reused by every thread (no per-thread slots left behind by short-lived
// threads; no hipHostMalloc / hipHostFree, which synchronise, per call).
struct HostReadback {
    uint32_t* pinned = nullptr;  // 8 words
    hipEvent_t ev = nullptr;
    int dev = 0;
};
constexpr int kMaxReadbackDevices = 64;

class ReadbackPool {
  public:
    hipError_t acquire(HostReadback*& rb) {
        rb = nullptr;
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        if (dev < 0 || dev >= kMaxReadbackDevices) return hipErrorInvalidDevice;
        {
            std::lock_guard<std::mutex> lock(m_);
            if (!free_[dev].empty()) {
                rb = free_[dev].back();
                free_[dev].pop_back();
                return hipSuccess;
            }
        }
        auto* slot = new HostReadback();
        slot->dev = dev;
        if ((e = hipHostMalloc(reinterpret_cast<void**>(&slot->pinned), 8 * sizeof(uint32_t),
                               hipHostMallocDefault)) != hipSuccess) {
            delete slot;
            return e;
        }
        if ((e = hipEventCreateWithFlags(&slot->ev, hipEventDisableTiming)) != hipSuccess) {
            (void)hipHostFree(slot->pinned);
            delete slot;
            return e;
        }
        rb = slot;
        return hipSuccess;
    }
    void release(HostReadback* rb) {
        std::lock_guard<std::mutex> lock(m_);
        free_[rb->dev].push_back(rb);
    }

  private:
    std::mutex m_;
    std::vector<HostReadback*> free_[kMaxReadbackDevices];
};
ReadbackPool g_readback_pool;

// a slot leased for one forward's readback, returned on every exit path.  Copies into the
// slot are queued on `stream` (arm() before the first); the slot's event is recorded after
// the last one (recorded()).  An exit between the two has no event covering the copies, so
// the stream is drained instead; a slot whose copies cannot be proven finished is never
// returned to the pool (another forward could otherwise lease it while a late copy lands).
struct ReadbackLease {
    HostReadback* rb = nullptr;
    hipStream_t stream = nullptr;
    bool armed = false, has_event = false;
    ReadbackLease() = default;
    ReadbackLease(const ReadbackLease&) = delete;
    ReadbackLease& operator=(const ReadbackLease&) = delete;
    void arm(hipStream_t s) { stream = s; armed = true; }
    void recorded() { has_event = true; }
    ~ReadbackLease() {
        if (!rb) return;
        hipError_t e = hipSuccess;
        if (has_event) e = hipEventSynchronize(rb->ev);
        else if (armed) e = hipStreamSynchronize(stream);
        if (e == hipSuccess) g_readback_pool.release(rb);  // (else the slot is leaked, not reused)
    }
};

int fail(int code, const char* what, hipError_t e = hipSuccess) {
    char buf[512];
    if (e != hipSuccess)
        snprintf(buf, sizeof(buf), "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
    else
        snprintf(buf, sizeof(buf), "%s", what);
    g_last_error = buf;
    return code;
}

// getHigherMsb, CR/rasterizer_impl.cu:37-50
uint32_t higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

using namespace gsr;

// Binning path: the tile lists of tilelists.hip where the grid allows, else
// the instance sort of binning.hip.
int bin_path(uint32_t gx, uint32_t gy) {
    return list_binning(gx, gy) ? kBinLists : kBinInstanceSort;
}

// `tmp`: where the forward-only scratch (scan / depth-sort temporaries) goes; NULL keeps it at the end of the buffer itself.  The
// fields the backward reads come first either way, so it re-carves without
// knowing which layout the forward used.
size_t carve_geom(void* base, int P, uint32_t gx, uint32_t gy, GeomState& g, Carver* tmp = nullptr) {
    Carver c(base);
    Carver& t = tmp ? *tmp : c;
    g.splats = c.take<Splat>(P);
    g.depths = c.take<float>(P);
    g.tiles_touched = c.take<uint32_t>(P);
    g.order = c.take<uint32_t>(P);
    g.depth_keys_sorted = c.take<uint32_t>(P);
    g.tiles_live = c.take<uint32_t>(P);
    g.counts = c.take<uint2>(P);
    g.offsets = c.take<uint2>(P);
    g.radii = c.take<int>(P);
    g.clamped = c.take<uint8_t>(P);
    g.ddir = c.take<float>((size_t)9 * P);
    g.offsets_K = c.take<uint32_t>(1);
    g.near_flag = c.take<uint32_t>(1);
    g.scan_tmp_bytes = scan_temp_bytes(P) > reduce_temp_bytes(P) ? scan_temp_bytes(P) : reduce_temp_bytes(P);
    g.scan_tmp = t.take<char>(g.scan_tmp_bytes);
    g.dsort_tmp_bytes = depth_sort_temp_bytes(P);
    g.dsort_tmp = t.take<char>(g.dsort_tmp_bytes);
    g.foot = t.take<uint4>((size_t)2 * P);
    return c.off + 256;
}

// Binning buffer.  The point list comes first, so its offset depends only on
// the base (gsr_debug_binning carves it knowing K alone); the rest depends
// on the path: tile lists (tilelists.hip) or emit + tile-id sort.
// `tmp` as in carve_geom: the list-building (or key-sort) scratch, dead once
// the point list is written, goes there instead of into the saved buffer.
size_t carve_binning(void* base, int K, int P, uint32_t gx, uint32_t gy, int path, BinningState& b,
                     Carver* tmp = nullptr) {
    Carver c(base);
    Carver& t = tmp ? *tmp : c;
    b.point_list = c.take<uint32_t>(K);
    const int tiles = (int)(gx * gy);
    const int tile_bits = (int)higher_msb((uint32_t)tiles);
    b.path = path;
    b.use_lists = path == kBinLists;
    b.key_bytes = tile_key_bytes(tile_bits);
    if (b.use_lists) {
        b.lists = list_layout(P, K, gx, gy);
        b.rows = t.take<uint2>(K);
        b.qrec = t.take<uint4>((size_t)2 * P);
        b.rows_count = t.take<uint32_t>((size_t)gy * b.lists.nseg_rows);
        b.rows_off = t.take<uint32_t>((size_t)gy * b.lists.nseg_rows);
        b.segbase = t.take<uint32_t>(gy + 1);
        b.tiles_count = t.take<uint32_t>((size_t)gx * b.lists.nseg_tiles_max + 1);
        b.tiles_off = t.take<uint32_t>((size_t)gx * b.lists.nseg_tiles_max + 1);
        b.list_tmp = t.take<char>(b.lists.tmp_bytes);
        b.keys_unsorted = b.keys = nullptr;
        b.values_unsorted = nullptr;
        b.sort_tmp = nullptr;
        b.sort_tmp_bytes = 0;
    } else {
        b.keys_unsorted = t.take<char>((size_t)K * b.key_bytes);
        b.keys = t.take<char>((size_t)K * b.key_bytes);
        b.values_unsorted = t.take<uint32_t>(K);
        b.sort_tmp_bytes = sort_temp_bytes(K, tile_bits);
        b.sort_tmp = t.take<char>(b.sort_tmp_bytes);
    }
    return c.off + 256;
}

size_t carve_image(void* base, int HW, ImageState& s) {
    Carver c(base);
    s.n_contrib = c.take<uint32_t>(HW);
    s.dT_dtm = c.take<float>(HW);
    s.md_check = c.take<uint32_t>(HW);
    return c.off + 256;
}

size_t carve_tiles(void* base, int T, TileState& s) {
    Carver c(base);
    s.ranges = c.take<uint2>(T);
    s.max_contrib = c.take<uint32_t>(T);
    s.order = c.take<uint32_t>(T);
    s.blend_mask = c.take<uint32_t>((size_t)T * kBlendWords);
    s.bwd_cost = c.take<uint32_t>(T);
    return c.off + 256;
}

size_t carve_bwd(void* base, int P, BwdState& s, int T = 0) {
    Carver c(base);
    s.acc = c.take<float>((size_t)P * kAccFields);
    s.acc_abs = c.take<float>(P);
    s.tile_order = c.take<uint32_t>(T);
    return c.off;
}

// sample_depth buffers (the reference's pointBuffer, point_binningBuffer,
// tileBuffer<true> and duplicatedTileBuffer, rasterizer_impl.h)
size_t carve_points(void* base, int PN, PointState& s) {
    Carver c(base);
    s.xy = c.take<float2>(PN);
    s.last = c.take<uint32_t>(PN);
    s.mdepth = c.take<float>(PN);
    s.dT = c.take<float>(PN);
    s.cached = c.take<uint8_t>(PN);
    s.t = c.take<float>(PN);
    return c.off + 256;
}

size_t carve_point_binning(void* base, int PN, uint32_t tiles, PointBinState& s) {
    Carver c(base);
    s.keys_unsorted = c.take<uint32_t>(PN);
    s.keys = c.take<uint32_t>(PN);
    s.pt_list = c.take<uint32_t>(PN);
    s.sort_tmp_bytes = point_sort_temp_bytes(PN, tiles);
    s.sort_tmp = c.take<char>(s.sort_tmp_bytes);
    return c.off + 256;
}

size_t carve_sample_tiles(void* base, int T, TileState& ts, SampleTiles& st) {
    Carver c(base);
    ts.ranges = c.take<uint2>(T);
    ts.max_contrib = c.take<uint32_t>(T);
    st.counts = c.take<uint32_t>(T);
    st.pt_ranges = c.take<uint2>(T);
    st.chunk_off = c.take<uint32_t>((size_t)T + 1);
    st.totals = c.take<uint32_t>(4);
    return c.off + 256;
}

size_t carve_chunks(void* base, uint32_t n, ChunkState& s) {
    Carver c(base);
    s.chunk_max = c.take<uint32_t>(n ? n : 1);
    return c.off + 256;
}

// 256-B alignment of the carve base (callbacks may return any alignment)
void* aligned_base(void* p) {
    return reinterpret_cast<void*>(align_up(reinterpret_cast<uintptr_t>(p), 256));
}

FwdParams make_params(int P, int D, int SHM, int SGD, int SGM, const float* background, int W, int H,
                      const float* means3D, const float* colors_precomp, const float* opacities,
                      const float* scales, const float* rotations, const float* cov3D_precomp, const float* shs,
                      const float* sg_axis, const float* sg_sharpness, const float* sg_color, float scale_modifier,
                      const float* view, const float* proj, const float* campos, float tan_fovx, float tan_fovy,
                      float kernel_size, int require_depth) {
    FwdParams p;
    p.P = P;
    p.D = D;
    p.SHM = SHM;
    p.SGD = SGD;
    p.SGM = SGM;
    p.W = W;
    p.H = H;
    p.background = background;
    p.means3D = means3D;
    p.colors_precomp = colors_precomp;
    p.opacities = opacities;
    p.scales = scales;
    p.rotations = rotations;
    p.cov3D_precomp = cov3D_precomp;
    p.shs = shs;
    p.sg_axis = sg_axis;
    p.sg_sharpness = sg_sharpness;
    p.sg_color = sg_color;
    p.scale_modifier = scale_modifier;
    p.view = view;
    p.proj = proj;
    p.campos = campos;
    p.tan_fovx = tan_fovx;
    p.tan_fovy = tan_fovy;
    p.focal_y = H / (2.0f * tan_fovy);
    p.focal_x = W / (2.0f * tan_fovx);
    p.kernel_size = kernel_size;
    p.grid_x = (W + kTile - 1) / kTile;
    p.grid_y = (H + kTile - 1) / kTile;
    p.require_depth = require_depth != 0;
    p.no_color = false;
    p.cull_pad = 0.f;
    return p;
}

const char* check_params(const FwdParams& p) {
    if (p.P < 0 || p.W <= 0 || p.H <= 0) return "invalid P / image size";
    if (p.P == 0) return nullptr;
    if (!p.means3D || !p.opacities || !p.view || !p.proj || !p.background) return "missing required input";
    if ((p.colors_precomp == nullptr) == (p.shs == nullptr))
        return "Please provide excatly one of either SHs or precomputed colors!";
    const bool have_sr = p.scales && p.rotations;
    if (have_sr == (p.cov3D_precomp != nullptr))
        return "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!";
    if (p.shs && (p.D < 0 || p.D > 3 || p.SHM < (p.D + 1) * (p.D + 1))) return "sh_degree / SH size mismatch";
    if (p.shs && !p.campos) return "campos required for SH colours";
    if (p.SGD < 0 || p.SGD > p.SGM) return "sg_degree exceeds SG lobes";
    if (p.SGD > 0 && (!p.sg_axis || !p.sg_sharpness || !p.sg_color)) return "missing SG tensors";
    return nullptr;
}

// ---- per-stage timing (gsr_timing_*) -------------------------------------
struct TimingRec {
    int stage;
    hipEvent_t e0, e1;
};
std::mutex g_tmu;
bool g_timing = false;
unsigned g_stage_mask = ~0u;
std::vector<TimingRec> g_recs;
std::vector<hipEvent_t> g_pool;

hipEvent_t pool_event() {
    if (!g_pool.empty()) {
        hipEvent_t e = g_pool.back();
        g_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

struct StageTimer {
    hipStream_t stream;
    int stage;
    hipEvent_t e0 = nullptr;
    StageTimer(int st, hipStream_t s) : stream(s), stage(st) {
        std::lock_guard<std::mutex> lk(g_tmu);
        if (!g_timing || !((g_stage_mask >> st) & 1u)) return;
        e0 = pool_event();
        if (e0) (void)hipEventRecord(e0, stream);
    }
    ~StageTimer() {
        if (!e0) return;
        std::lock_guard<std::mutex> lk(g_tmu);
        hipEvent_t e1 = pool_event();
        if (!e1) return;
        (void)hipEventRecord(e1, stream);
        g_recs.push_back({stage, e0, e1});
    }
};

#define GSR_TRY(expr, what)                                   \
    do {                                                      \
        hipError_t _e = (expr);                               \
        if (_e != hipSuccess) return fail(GSR_ERR_HIP, what, _e); \
        if (debug) {                                          \
            _e = hipStreamSynchronize(stream);                \
            if (_e != hipSuccess) return fail(GSR_ERR_HIP, what, _e); \
        }                                                     \
    } while (0)

#define GSR_STAGE(stage, expr, what)                          \
    do {                                                      \
        StageTimer _t(stage, stream);                         \
        GSR_TRY(expr, what);                                  \
    } while (0)

}  // namespace

namespace gsr {
static int g_options[kNumOptions] = {};
int option(int which) { return (which >= 0 && which < kNumOptions) ? g_options[which] : 0; }
}  // namespace gsr

extern "C" {

int gsr_debug_render_stats(unsigned long long* out20, int reset) {
    hipError_t e = gsr::read_render_stats(out20, reset != 0);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "render stats", e);
}

int gsr_debug_binning(const void* binning_buffer, const void* tile_buffer, int R, int width, int height,
                      uint32_t* point_list_out, uint32_t* ranges_out, void* stream_ptr) {
    if (!binning_buffer || !tile_buffer || R < 0 || width <= 0 || height <= 0)
        return fail(GSR_ERR_ARGS, "invalid arguments");
    const uint32_t gx = (width + kTile - 1) / kTile, gy = (height + kTile - 1) / kTile;
    const int tiles = (int)(gx * gy);
    BinningState bs;
    {
        Carver c(aligned_base(const_cast<void*>(binning_buffer)));
        bs.point_list = c.take<uint32_t>(R);  // first in every layout (carve_binning)
    }
    TileState ts{};
    carve_tiles(aligned_base(const_cast<void*>(tile_buffer)), tiles, ts);
    hipStream_t stream = (hipStream_t)stream_ptr;
    hipError_t e = hipSuccess;
    if (point_list_out && R > 0)
        e = hipMemcpyAsync(point_list_out, bs.point_list, sizeof(uint32_t) * R, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess && ranges_out)
        e = hipMemcpyAsync(ranges_out, ts.ranges, sizeof(uint2) * tiles, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "debug binning", e);
}

int gsr_debug_sample_points(const void* point_buffer, int PN, float* median_depth_out, uint32_t* last_out,
                            void* stream_ptr) {
    if (!point_buffer || PN < 0) return fail(GSR_ERR_ARGS, "invalid arguments");
    PointState ps;
    carve_points(aligned_base(const_cast<void*>(point_buffer)), PN, ps);
    hipStream_t stream = (hipStream_t)stream_ptr;
    hipError_t e = hipSuccess;
    if (median_depth_out && PN)
        e = hipMemcpyAsync(median_depth_out, ps.mdepth, sizeof(float) * PN, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess && last_out && PN)
        e = hipMemcpyAsync(last_out, ps.last, sizeof(uint32_t) * PN, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "debug sample points", e);
}

int gsr_debug_image(const void* image_buffer, int width, int height, uint32_t* n_contrib_out, void* stream_ptr) {
    if (!image_buffer || width <= 0 || height <= 0 || !n_contrib_out) return fail(GSR_ERR_ARGS, "invalid arguments");
    ImageState is;
    carve_image(aligned_base(const_cast<void*>(image_buffer)), width * height, is);
    hipStream_t stream = (hipStream_t)stream_ptr;
    hipError_t e = hipMemcpyAsync(n_contrib_out, is.n_contrib, sizeof(uint32_t) * (size_t)width * height,
                                  hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "debug image", e);
}

int gsr_debug_tile_stats(const void* tile_buffer, int width, int height, uint32_t* max_contrib_out, void* stream_ptr) {
    if (!tile_buffer || width <= 0 || height <= 0 || !max_contrib_out) return fail(GSR_ERR_ARGS, "invalid arguments");
    const int tiles = (int)(((width + kTile - 1) / kTile) * ((height + kTile - 1) / kTile));
    TileState ts{};
    carve_tiles(aligned_base(const_cast<void*>(tile_buffer)), tiles, ts);
    hipStream_t stream = (hipStream_t)stream_ptr;
    hipError_t e = hipMemcpyAsync(max_contrib_out, ts.max_contrib, sizeof(uint32_t) * (size_t)tiles,
                                  hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "debug tile stats", e);
}

int gsr_set_option(int opt, int value) {
    if (opt < 0 || opt >= gsr::kNumOptions || gsr::option_retired(opt)) return fail(GSR_ERR_ARGS, "unknown option");
    gsr::g_options[opt] = value;
    return GSR_OK;
}


int gsr_abi_version(void) { return 20; }

int gsr_backward_chunk_size(int P, int chunks) {
    if (P < 0 || chunks < 1) return -1;
    const long long per = ((long long)P + chunks - 1) / chunks;
    return (int)((per + 255) / 256 * 256);
}

int gsr_timing_enable(int on) {
    std::lock_guard<std::mutex> lk(g_tmu);
    g_timing = on != 0;
    return GSR_OK;
}

int gsr_timing_stage_mask(unsigned int mask) {
    std::lock_guard<std::mutex> lk(g_tmu);
    g_stage_mask = mask;
    return GSR_OK;
}

int gsr_timing_collect(double* ms, int* launches) {
    std::vector<TimingRec> recs;
    {
        std::lock_guard<std::mutex> lk(g_tmu);
        recs.swap(g_recs);
    }
    int rc = GSR_OK;
    for (const TimingRec& r : recs) {
        float t = 0.f;
        hipError_t e = hipEventSynchronize(r.e1);
        if (e == hipSuccess) e = hipEventElapsedTime(&t, r.e0, r.e1);
        if (e != hipSuccess) rc = fail(GSR_ERR_HIP, "timing", e);
        if (ms) ms[r.stage] += t;
        if (launches) launches[r.stage] += 1;
    }
    std::lock_guard<std::mutex> lk(g_tmu);
    for (const TimingRec& r : recs) {
        g_pool.push_back(r.e0);
        g_pool.push_back(r.e1);
    }
    return rc;
}

const char* gsr_stage_name(int stage) {
    static const char* names[GSR_NUM_STAGES] = {"preprocess", "scan", "emit_keys", "sort", "tile_ranges",
                                                 "render_fwd", "bwd_clear", "render_bwd", "preprocess_bwd",
                                                 "depth_order", "tile_lists", "sample_points", "sample_fwd",
                                                 "sample_bwd"};
    return (stage >= 0 && stage < GSR_NUM_STAGES) ? names[stage] : "?";
}

const char* gsr_last_error(void) { return g_last_error.c_str(); }

// CR/auxiliary.h:146-148 (the reference traps the kernel)
static const char* kPrefilteredMsg = "Point is filtered although prefiltered is set. This shouldn't happen!";

int gsr_rasterize_forward_ex2(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                             gsr_alloc_fn image_alloc, void* image_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                             int P, int sh_degree, int SHM, int sg_degree, int SGM, const float* background, int width,
                             int height, const float* means3D, const float* colors_precomp, const float* opacities,
                             const float* scales, const float* rotations, const float* cov3D_precomp,
                             const float* shs, const float* sg_axis, const float* sg_sharpness, const float* sg_color,
                             float scale_modifier, const float* viewmatrix, const float* projmatrix,
                             const float* cam_pos, float tan_fovx, float tan_fovy, float kernel_size, int prefiltered,
                             float* out_color, float* out_mdepth, float* out_alpha, float* out_normal, int* radii,
                             int require_depth, int debug, void* stream_ptr, int* num_rendered,
                             gsr_alloc_fn scratch_alloc, void* scratch_ctx, const float* shs_rest) {
    hipStream_t stream = (hipStream_t)stream_ptr;
    if (num_rendered) *num_rendered = 0;
    FwdParams p = make_params(P, sh_degree, SHM, sg_degree, SGM, background, width, height, means3D, colors_precomp,
                              opacities, scales, rotations, cov3D_precomp, shs, sg_axis, sg_sharpness, sg_color,
                              scale_modifier, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, kernel_size,
                              require_depth);
    p.shs_rest = shs_rest;
    if (shs_rest && (!shs || SHM < 2)) return fail(GSR_ERR_ARGS, "split SH rows need the DC rows and SHM >= 2");
    if (const char* msg = check_params(p)) return fail(GSR_ERR_ARGS, msg);
    if (!out_color || !out_alpha || !out_mdepth || !out_normal) return fail(GSR_ERR_ARGS, "missing output buffer");
    if (!geom_alloc || !binning_alloc || !image_alloc || !tile_alloc) return fail(GSR_ERR_ARGS, "missing allocator");
    const int tiles = (int)(p.grid_x * p.grid_y);

    // forward-only scratch from scratch_alloc when given (two blocks: the
    // per-Gaussian sort/scan temporaries now, the list-building scratch once
    // K is known), else inside the geometry / binning buffers
    GeomState gs;
    Carver gtmp(nullptr);
    void* gbuf = geom_alloc(geom_ctx, carve_geom(nullptr, P, p.grid_x, p.grid_y, gs, scratch_alloc ? &gtmp : nullptr));
    if (!gbuf) return fail(GSR_ERR_ALLOC, "geometry buffer allocation failed");
    if (scratch_alloc) {
        void* sbuf = scratch_alloc(scratch_ctx, gtmp.off + 256);
        if (!sbuf) return fail(GSR_ERR_ALLOC, "scratch allocation failed");
        gtmp = Carver(aligned_base(sbuf));
    }
    carve_geom(aligned_base(gbuf), P, p.grid_x, p.grid_y, gs, scratch_alloc ? &gtmp : nullptr);
    TileState ts{};
    void* tbuf = tile_alloc(tile_ctx, carve_tiles(nullptr, tiles, ts));
    if (!tbuf) return fail(GSR_ERR_ALLOC, "tile buffer allocation failed");
    carve_tiles(aligned_base(tbuf), tiles, ts);
    ImageState is;
    void* ibuf = image_alloc(image_ctx, carve_image(nullptr, width * height, is));
    if (!ibuf) return fail(GSR_ERR_ALLOC, "image buffer allocation failed");
    carve_image(aligned_base(ibuf), width * height, is);
    if (radii == nullptr) radii = gs.radii;

    if (P == 0) {
        // empty scene: background image, zero geometry (rasterize_points.cu:95)
        hipError_t e = hipMemsetAsync(ts.ranges, 0, sizeof(uint2) * tiles, stream);
        if (e == hipSuccess) e = hipMemsetAsync(ts.max_contrib, 0, sizeof(uint32_t) * tiles, stream);
        if (e != hipSuccess) return fail(GSR_ERR_HIP, "memset", e);
        BinningState bs;
        void* bbuf = binning_alloc(binning_ctx, carve_binning(nullptr, 0, 0, p.grid_x, p.grid_y, kBinLists, bs));
        if (!bbuf) return fail(GSR_ERR_ALLOC, "binning buffer allocation failed");
        carve_binning(aligned_base(bbuf), 0, 0, p.grid_x, p.grid_y, kBinLists, bs);
        GSR_TRY(launch_render_fwd(p, gs, bs, is, ts, out_color, out_alpha, out_normal, out_mdepth, stream), "render");
        return GSR_OK;
    }

    GSR_STAGE(GSR_STAGE_PREPROCESS, launch_preprocess_fwd(p, gs, radii, stream), "preprocess");
    if (prefiltered) GSR_TRY(launch_near_violation(P, means3D, viewmatrix, gs.near_flag, stream), "prefiltered check");
    uint32_t near_flag = 0;
    const int path = bin_path(p.grid_x, p.grid_y);
    // K = the reference's instance count (rect tiles): returned as
    // num_rendered and the capacity of the binning buffer.  The instance-sort
    // path also needs K_live, the instances that survive tile culling.
    uint2 Ks = make_uint2(0u, 0u);
    if (path != kBinInstanceSort) {
        // K depends on preprocess only: one readback
        ReadbackLease lease;
        GSR_TRY(g_readback_pool.acquire(lease.rb), "pinned readback buffer");
        HostReadback* rb = lease.rb;
        GSR_STAGE(GSR_STAGE_SCAN, launch_count_k_hist(gs, P, path == kBinLists, stream), "count K");
        lease.arm(stream);
        GSR_TRY(hipMemcpyAsync(rb->pinned, gs.offsets_K, sizeof(uint32_t), hipMemcpyDeviceToHost, stream), "memcpy K");
        if (prefiltered)
            GSR_TRY(hipMemcpyAsync(rb->pinned + 1, gs.near_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, stream),
                    "memcpy prefiltered flag");
        GSR_TRY(hipEventRecord(rb->ev, stream), "event record");
        lease.recorded();
        // the GPU counts the tile lists (or sorts by depth) while the host waits
        if (path == kBinLists) GSR_STAGE(GSR_STAGE_DEPTH_ORDER, launch_depth_sort(gs, P, true, stream), "depth order");
        GSR_TRY(hipEventSynchronize(rb->ev), "event sync");
        Ks.x = rb->pinned[0];
        if (prefiltered) near_flag = rb->pinned[1];
    } else {
        GSR_STAGE(GSR_STAGE_DEPTH_ORDER, launch_depth_sort(gs, P, false, stream), "depth order");
        GSR_STAGE(GSR_STAGE_DEPTH_ORDER, launch_live_counts(p, gs, radii, stream), "live counts");
        GSR_STAGE(GSR_STAGE_SCAN, launch_scan(gs, P, stream), "scan");
        GSR_TRY(hipMemcpyAsync(&Ks, gs.offsets + (P - 1), sizeof(uint2), hipMemcpyDeviceToHost, stream), "memcpy K");
        if (prefiltered)
            GSR_TRY(hipMemcpyAsync(&near_flag, gs.near_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, stream),
                    "memcpy prefiltered flag");
        hipError_t e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return fail(GSR_ERR_HIP, "stream sync", e);
    }
    if (near_flag) return fail(GSR_ERR_ARGS, kPrefilteredMsg);
    const uint32_t K = Ks.x, K_live = Ks.y;
    BinningState bs;
    Carver btmp(nullptr);
    void* bbuf = binning_alloc(binning_ctx, carve_binning(nullptr, (int)K, P, p.grid_x, p.grid_y, path, bs,
                                                          scratch_alloc ? &btmp : nullptr));
    if (!bbuf) return fail(GSR_ERR_ALLOC, "binning buffer allocation failed");
    if (scratch_alloc) {
        void* sbuf = scratch_alloc(scratch_ctx, btmp.off + 256);
        if (!sbuf) return fail(GSR_ERR_ALLOC, "scratch allocation failed");
        btmp = Carver(aligned_base(sbuf));
    }
    carve_binning(aligned_base(bbuf), (int)K, P, p.grid_x, p.grid_y, path, bs, scratch_alloc ? &btmp : nullptr);
    if (path == kBinLists) {
        GSR_STAGE(GSR_STAGE_TILE_LISTS, launch_list_binning(p, gs, radii, bs, ts, (int)K, stream), "tile lists");
    } else {
        const int tile_bits = (int)higher_msb((uint32_t)tiles);
        GSR_STAGE(GSR_STAGE_EMIT_KEYS, launch_emit_keys(p, gs, radii, bs, stream), "emit keys");
        GSR_STAGE(GSR_STAGE_SORT, launch_sort(bs, (int)K_live, tile_bits, stream), "sort");
        GSR_STAGE(GSR_STAGE_TILE_RANGES, launch_tile_ranges(bs, (int)K_live, ts, tiles, stream), "tile ranges");
    }
    // Heaviest tile first (LPT, cost = list length) when the grid fills the
    // chip only a few times over: then the last round of long tiles sets the
    // launch's length.  At C3 (8160 tiles, ~5 rounds of 6 blocks per CU) the
    // order saved 8 us of render_fwd for a 12 us ordering launch, so larger
    // grids keep the XCD-contiguous order.
#ifndef GSR_FWD_LPT_MAX_TILES
#define GSR_FWD_LPT_MAX_TILES 4096
#endif
    const bool lpt = tiles <= GSR_FWD_LPT_MAX_TILES;
    if (!lpt) ts.order = nullptr;
    // (one stage: the ordering launch is part of the forward raster's time)
    GSR_STAGE(GSR_STAGE_RENDER_FWD, [&]() {
        if (lpt) {
            const hipError_t e = launch_tile_order((uint32_t)tiles, ts.ranges, nullptr, ts.order, stream);
            if (e != hipSuccess) return e;
        }
        return launch_render_fwd(p, gs, bs, is, ts, out_color, out_alpha, out_normal, out_mdepth, stream);
    }(), "render");
    if (num_rendered) *num_rendered = (int)K;
    return GSR_OK;
}

int gsr_rasterize_forward_ex(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                             gsr_alloc_fn image_alloc, void* image_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                             int P, int sh_degree, int SHM, int sg_degree, int SGM, const float* background, int width,
                             int height, const float* means3D, const float* colors_precomp, const float* opacities,
                             const float* scales, const float* rotations, const float* cov3D_precomp,
                             const float* shs, const float* sg_axis, const float* sg_sharpness, const float* sg_color,
                             float scale_modifier, const float* viewmatrix, const float* projmatrix,
                             const float* cam_pos, float tan_fovx, float tan_fovy, float kernel_size, int prefiltered,
                             float* out_color, float* out_mdepth, float* out_alpha, float* out_normal, int* radii,
                             int require_depth, int debug, void* stream_ptr, int* num_rendered,
                             gsr_alloc_fn scratch_alloc, void* scratch_ctx) {
    return gsr_rasterize_forward_ex2(geom_alloc, geom_ctx, binning_alloc, binning_ctx, image_alloc, image_ctx,
                                     tile_alloc, tile_ctx, P, sh_degree, SHM, sg_degree, SGM, background, width,
                                     height, means3D, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                                     shs, sg_axis, sg_sharpness, sg_color, scale_modifier, viewmatrix, projmatrix,
                                     cam_pos, tan_fovx, tan_fovy, kernel_size, prefiltered, out_color, out_mdepth,
                                     out_alpha, out_normal, radii, require_depth, debug, stream_ptr, num_rendered,
                                     scratch_alloc, scratch_ctx, nullptr);
}

int gsr_rasterize_forward(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                          gsr_alloc_fn image_alloc, void* image_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                          int P, int sh_degree, int SHM, int sg_degree, int SGM, const float* background, int width,
                          int height, const float* means3D, const float* colors_precomp, const float* opacities,
                          const float* scales, const float* rotations, const float* cov3D_precomp,
                          const float* shs, const float* sg_axis, const float* sg_sharpness, const float* sg_color,
                          float scale_modifier, const float* viewmatrix, const float* projmatrix,
                          const float* cam_pos, float tan_fovx, float tan_fovy, float kernel_size, int prefiltered,
                          float* out_color, float* out_mdepth, float* out_alpha, float* out_normal, int* radii,
                          int require_depth, int debug, void* stream_ptr, int* num_rendered) {
    return gsr_rasterize_forward_ex(geom_alloc, geom_ctx, binning_alloc, binning_ctx, image_alloc, image_ctx,
                                    tile_alloc, tile_ctx, P, sh_degree, SHM, sg_degree, SGM, background, width,
                                    height, means3D, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                                    shs, sg_axis, sg_sharpness, sg_color, scale_modifier, viewmatrix, projmatrix,
                                    cam_pos, tan_fovx, tan_fovy, kernel_size, prefiltered, out_color, out_mdepth,
                                    out_alpha, out_normal, radii, require_depth, debug, stream_ptr, num_rendered,
                                    nullptr, nullptr);
}

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
                           int chunks, gsr_chunk_fn on_chunk, void* chunk_ctx, float* dc_rows,
                              void* stream_ptr, const float* shs_rest, float* dL_dsh_rest) {
    hipStream_t stream = (hipStream_t)stream_ptr;
    BwdParams b;
    b.f = make_params(P, sh_degree, SHM, sg_degree, SGM, background, width, height, means3D, colors_precomp,
                      opacities, scales, rotations, cov3D_precomp, shs, sg_axis, sg_sharpness, sg_color,
                      scale_modifier, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, kernel_size, require_depth);
    if (P == 0) return GSR_OK;
    if (const char* msg = check_params(b.f)) return fail(GSR_ERR_ARGS, msg);
    // (a NULL upstream image gradient is zero: gsr.h)
    if (!geom_buffer || !binning_buffer || !image_buffer || !tile_buffer || !radii || !alphas || !dL_dmean3D ||
        !dL_dmean2D || !dL_dcolor || !dL_dopacity)
        return fail(GSR_ERR_ARGS, "missing backward buffer");
    if (b.f.require_depth && (!normalmap || !mdepth))
        return fail(GSR_ERR_ARGS, "missing geometry buffers for require_depth");
    if (scales && (!dL_dscale || !dL_drot)) return fail(GSR_ERR_ARGS, "missing scale/rotation gradients");
    if (cov3D_precomp && !dL_dcov3D) return fail(GSR_ERR_ARGS, "missing cov3D gradient");
    if (shs && !dL_dsh) return fail(GSR_ERR_ARGS, "missing SH gradient");
    if (SGM > 0 && shs && (!dL_dsg_axis || !dL_dsg_sharpness || !dL_dsg_color))
        return fail(GSR_ERR_ARGS, "missing SG gradients");
    if (chunks < 1) return fail(GSR_ERR_ARGS, "chunks must be >= 1");
    if (dc_rows && !shs) return fail(GSR_ERR_ARGS, "dc_rows needs the SH colour path");
    if (shs_rest && (!shs || SHM < 2 || !dL_dsh_rest))
        return fail(GSR_ERR_ARGS, "split SH rows need the DC rows, SHM >= 2 and both gradients");
    b.f.shs_rest = shs_rest;
    b.dL_dsh_rest = dL_dsh_rest;
    b.R = R;
    b.radii = radii;
    b.alphas = alphas;
    b.normalmap = normalmap;
    b.mdepth = mdepth;
    b.dL_dpix = dL_dpix;
    b.dL_dmdepth = dL_dpix_mdepth;
    b.dL_dalpha = dL_dalphas;
    b.dL_dnormal = dL_dpixel_normals;
    b.dL_dmean3D = dL_dmean3D;
    b.dL_dmean2D = dL_dmean2D;
    b.dL_dcolor = dL_dcolor;
    b.dL_dopacity = dL_dopacity;
    b.dL_dscale = dL_dscale;
    b.dL_drot = dL_drot;
    b.dL_dcov3D = dL_dcov3D;
    b.dL_dsh = dL_dsh;
    b.dL_dsg_axis = dL_dsg_axis;
    b.dL_dsg_sharpness = dL_dsg_sharpness;
    b.dL_dsg_color = dL_dsg_color;

    const int tiles = (int)(b.f.grid_x * b.f.grid_y);
    GeomState gs;
    carve_geom(aligned_base(const_cast<void*>(geom_buffer)), P, b.f.grid_x, b.f.grid_y, gs);
    BinningState bs;  // (the backward reads the point list only: first in every layout)
    carve_binning(aligned_base(const_cast<void*>(binning_buffer)), R, P, b.f.grid_x, b.f.grid_y,
                  bin_path(b.f.grid_x, b.f.grid_y), bs);
    ImageState is;
    carve_image(aligned_base(const_cast<void*>(image_buffer)), width * height, is);
    TileState ts{};
    carve_tiles(aligned_base(const_cast<void*>(tile_buffer)), tiles, ts);
    BwdState ws{};
    const size_t wbytes = carve_bwd(nullptr, P, ws, tiles);
    void* wbuf = geom_bwd_alloc(geom_bwd_ctx, wbytes + 256);
    if (!wbuf) return fail(GSR_ERR_ALLOC, "backward buffer allocation failed");
    void* wb = aligned_base(wbuf);
    carve_bwd(wb, P, ws, tiles);
    if (tiles > 0) {
        // heaviest tiles first (cost: the forward's per-tile max contributor),
        // ordered by one workgroup while the others clear the accumulators
        const size_t zbytes = (size_t)(reinterpret_cast<char*>(ws.tile_order) - static_cast<char*>(wb));
        GSR_STAGE(GSR_STAGE_BWD_CLEAR,
                  launch_bwd_prepare(wb, zbytes, (uint32_t)tiles, ts.bwd_cost, ws.tile_order, stream),
                  "clear accumulators + tile order");
    } else {
        GSR_STAGE(GSR_STAGE_BWD_CLEAR, hipMemsetAsync(wb, 0, wbytes, stream), "memset accumulators");
        ws.tile_order = nullptr;
    }
    GSR_STAGE(GSR_STAGE_RENDER_BWD, launch_render_bwd(b, gs, bs, is, ts, ws, stream), "render backward");
    // the per-Gaussian backward over `chunks` consecutive Gaussian ranges; after each range's launch
    // the host callback may post work on other streams that waits for it (gsr_dist.OverlappedViewGrads:
    // the range's gradient exchange runs while the next range computes)
    // (ranges of whole 256-Gaussian workgroups; gsr_dist.OverlappedViewGrads reads the size from
    // gsr_backward_chunk_size and checks the ranges it is called with against it)
    const int cs = gsr_backward_chunk_size(P, chunks);
    for (int b0 = 0; b0 < P; b0 += cs) {
        const int b1 = min(P, b0 + cs);
        GSR_STAGE(GSR_STAGE_PREPROCESS_BWD, launch_preprocess_bwd(b, gs, ws, stream, b0, b1, dc_rows),
                  "preprocess backward");
        if (on_chunk) on_chunk(chunk_ctx, b0, b1);
    }
    return GSR_OK;
}

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
                           int chunks, gsr_chunk_fn on_chunk, void* chunk_ctx, float* dc_rows,
                              void* stream_ptr) {
    return gsr_rasterize_backward_ex2(geom_bwd_alloc, geom_bwd_ctx, P, sh_degree, SHM, sg_degree, SGM, R, background, width, height, means3D, colors_precomp, opacities, scales, rotations, cov3D_precomp, shs, sg_axis, sg_sharpness, sg_color, scale_modifier, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, kernel_size, radii, alphas, normalmap, mdepth, geom_buffer, binning_buffer, image_buffer, tile_buffer, dL_dpix, dL_dpix_mdepth, dL_dalphas, dL_dpixel_normals, dL_dmean3D, dL_dmean2D, dL_dcolor, dL_dopacity, dL_dscale, dL_drot, dL_dcov3D, dL_dsh, dL_dsg_axis, dL_dsg_sharpness, dL_dsg_color, require_depth, debug, chunks, on_chunk, chunk_ctx, dc_rows, stream_ptr, nullptr, nullptr);
}

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
                           void* stream_ptr) {
    return gsr_rasterize_backward_ex(geom_bwd_alloc, geom_bwd_ctx, P, sh_degree, SHM, sg_degree, SGM, R, background,
                                     width, height, means3D, colors_precomp, opacities, scales, rotations,
                                     cov3D_precomp, shs, sg_axis, sg_sharpness, sg_color, scale_modifier, viewmatrix,
                                     projmatrix, campos, tan_fovx, tan_fovy, kernel_size, radii, alphas, normalmap,
                                     mdepth, geom_buffer, binning_buffer, image_buffer, tile_buffer, dL_dpix,
                                     dL_dpix_mdepth, dL_dalphas, dL_dpixel_normals, dL_dmean3D, dL_dmean2D, dL_dcolor,
                                     dL_dopacity, dL_dscale, dL_drot, dL_dcov3D, dL_dsh, dL_dsg_axis,
                                     dL_dsg_sharpness, dL_dsg_color, require_depth, debug, 1, nullptr, nullptr,
                                     nullptr, stream_ptr);
}

// The point-query forwards (sample_depth, integrate, evaluate_sdf) share
// everything but the raster's mode and outputs: Rasterizer::sampleDepth
// (rasterizer_impl.cu:1042-1261), evaluateTransmittance (:594-815) and
// evaluateSDF (:817-1040) run the same preprocess, Gaussian binning, point
// preprocess and point binning.
static int point_query_forward(int query, gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc,
                               void* binning_ctx, gsr_alloc_fn point_alloc, void* point_ctx,
                               gsr_alloc_fn point_binning_alloc, void* point_binning_ctx, gsr_alloc_fn tile_alloc,
                               void* tile_ctx, gsr_alloc_fn dup_tile_alloc, void* dup_tile_ctx, int PN, int P,
                               int width, int height, const float* points3D, const float* means3D,
                               const float* opacities, const float* scales, float scale_modifier,
                               const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                               const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                               float kernel_size, int prefiltered, float* output, float* output2, uint8_t* inside,
                               int debug, void* stream_ptr, int* num_rendered, int* num_points,
                               int* num_duplicated_tiles, gsr_alloc_fn scratch_alloc = nullptr,
                               void* scratch_ctx = nullptr) {
    hipStream_t stream = (hipStream_t)stream_ptr;
    if (num_rendered) *num_rendered = 0;
    if (num_points) *num_points = 0;
    if (num_duplicated_tiles) *num_duplicated_tiles = 0;
    if (P < 0 || PN < 0 || width <= 0 || height <= 0) return fail(GSR_ERR_ARGS, "invalid P / PN / image size");
    if (P == 0 || PN == 0) return GSR_OK;  // rasterize_points.cu:517: nothing sampled, zero outputs
    static const float kZeroBg[3] = {0.f, 0.f, 0.f};
    FwdParams p = make_params(P, 0, 0, 0, 0, kZeroBg, width, height, means3D, nullptr, opacities, scales, rotations,
                              cov3D_precomp, nullptr, nullptr, nullptr, nullptr, scale_modifier, viewmatrix,
                              projmatrix, cam_pos, tan_fovx, tan_fovy, kernel_size, 1);
    p.no_color = true;
    p.cull_pad = 0.5f;
    if (!means3D || !opacities || !viewmatrix || !projmatrix || !points3D) return fail(GSR_ERR_ARGS, "missing input");
    if ((scales && rotations) == (cov3D_precomp != nullptr))
        return fail(GSR_ERR_ARGS, "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    if (!output || !inside || (query == kQuerySDF && !output2)) return fail(GSR_ERR_ARGS, "missing output buffer");
    if (!geom_alloc || !binning_alloc || !point_alloc || !point_binning_alloc || !tile_alloc || !dup_tile_alloc)
        return fail(GSR_ERR_ARGS, "missing allocator");
    const uint32_t tiles = p.grid_x * p.grid_y;

    // forward-only scratch as in gsr_rasterize_forward_ex
    GeomState gs;
    Carver gtmp(nullptr);
    void* gbuf = geom_alloc(geom_ctx, carve_geom(nullptr, P, p.grid_x, p.grid_y, gs, scratch_alloc ? &gtmp : nullptr));
    if (!gbuf) return fail(GSR_ERR_ALLOC, "geometry buffer allocation failed");
    if (scratch_alloc) {
        void* sbuf = scratch_alloc(scratch_ctx, gtmp.off + 256);
        if (!sbuf) return fail(GSR_ERR_ALLOC, "scratch allocation failed");
        gtmp = Carver(aligned_base(sbuf));
    }
    carve_geom(aligned_base(gbuf), P, p.grid_x, p.grid_y, gs, scratch_alloc ? &gtmp : nullptr);
    TileState ts{};
    SampleTiles st;
    void* tbuf = tile_alloc(tile_ctx, carve_sample_tiles(nullptr, (int)tiles, ts, st));
    if (!tbuf) return fail(GSR_ERR_ALLOC, "tile buffer allocation failed");
    carve_sample_tiles(aligned_base(tbuf), (int)tiles, ts, st);
    PointState ps;
    void* pbuf = point_alloc(point_ctx, carve_points(nullptr, PN, ps));
    if (!pbuf) return fail(GSR_ERR_ALLOC, "point buffer allocation failed");
    carve_points(aligned_base(pbuf), PN, ps);
    PointBinState pb;
    void* pbbuf = point_binning_alloc(point_binning_ctx, carve_point_binning(nullptr, PN, tiles, pb));
    if (!pbbuf) return fail(GSR_ERR_ALLOC, "point binning buffer allocation failed");
    carve_point_binning(aligned_base(pbbuf), PN, tiles, pb);

    GSR_STAGE(GSR_STAGE_PREPROCESS, launch_preprocess_fwd(p, gs, gs.radii, stream), "preprocess");
    if (prefiltered) GSR_TRY(launch_near_violation(P, means3D, viewmatrix, gs.near_flag, stream), "prefiltered check");
    uint32_t near_flag = 0;
    const int path = bin_path(p.grid_x, p.grid_y);  // as the render forward
    uint2 Ks = make_uint2(0u, 0u);
    uint32_t totals[4] = {0, 0, 0, 0};
    if (path != kBinInstanceSort) {
        // K, the tile list sizes and the point totals depend on preprocess and
        // the points only: one readback (HostReadback)
        ReadbackLease lease;
        GSR_TRY(g_readback_pool.acquire(lease.rb), "pinned readback buffer");
        HostReadback* rb = lease.rb;
        GSR_STAGE(GSR_STAGE_SCAN, launch_count_k_hist(gs, P, path == kBinLists, stream), "count K");
        GSR_STAGE(GSR_STAGE_SAMPLE_POINTS, launch_sample_points(p, PN, points3D, ps, pb, st, stream), "sample points");
        GSR_STAGE(GSR_STAGE_SAMPLE_POINTS, launch_sample_setup(PN, tiles, pb, st, stream), "sample setup");
        lease.arm(stream);
        GSR_TRY(hipMemcpyAsync(rb->pinned, gs.offsets_K, sizeof(uint32_t), hipMemcpyDeviceToHost, stream), "memcpy K");
        GSR_TRY(hipMemcpyAsync(rb->pinned + 4, st.totals, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost, stream),
                "memcpy totals");
        if (prefiltered)
            GSR_TRY(hipMemcpyAsync(rb->pinned + 1, gs.near_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, stream),
                    "memcpy prefiltered flag");
        GSR_TRY(hipEventRecord(rb->ev, stream), "event record");
        lease.recorded();
        // the GPU counts the tile lists (or sorts by depth) while the host waits
        if (path == kBinLists) GSR_STAGE(GSR_STAGE_DEPTH_ORDER, launch_depth_sort(gs, P, true, stream), "depth order");
        GSR_TRY(hipEventSynchronize(rb->ev), "event sync");
        Ks.x = rb->pinned[0];
        if (prefiltered) near_flag = rb->pinned[1];
        for (int k = 0; k < 4; k++) totals[k] = rb->pinned[4 + k];
    } else {
        GSR_STAGE(GSR_STAGE_DEPTH_ORDER, launch_depth_sort(gs, P, false, stream), "depth order");
        GSR_STAGE(GSR_STAGE_DEPTH_ORDER, launch_live_counts(p, gs, gs.radii, stream), "live counts");
        GSR_STAGE(GSR_STAGE_SCAN, launch_scan(gs, P, stream), "scan");
        GSR_STAGE(GSR_STAGE_SAMPLE_POINTS, launch_sample_points(p, PN, points3D, ps, pb, st, stream), "sample points");
        GSR_STAGE(GSR_STAGE_SAMPLE_POINTS, launch_sample_setup(PN, tiles, pb, st, stream), "sample setup");
        GSR_TRY(hipMemcpyAsync(&Ks, gs.offsets + (P - 1), sizeof(uint2), hipMemcpyDeviceToHost, stream), "memcpy K");
        GSR_TRY(hipMemcpyAsync(totals, st.totals, sizeof(totals), hipMemcpyDeviceToHost, stream), "memcpy totals");
        if (prefiltered)
            GSR_TRY(hipMemcpyAsync(&near_flag, gs.near_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, stream),
                    "memcpy prefiltered flag");
        hipError_t e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return fail(GSR_ERR_HIP, "stream sync", e);
    }
    if (near_flag) return fail(GSR_ERR_ARGS, kPrefilteredMsg);
    const uint32_t K = Ks.x, K_live = Ks.y, n_chunks = totals[2];
    BinningState bs;
    Carver btmp(nullptr);
    void* bbuf = binning_alloc(binning_ctx, carve_binning(nullptr, (int)K, P, p.grid_x, p.grid_y, path, bs,
                                                          scratch_alloc ? &btmp : nullptr));
    if (!bbuf) return fail(GSR_ERR_ALLOC, "binning buffer allocation failed");
    if (scratch_alloc) {
        void* sbuf = scratch_alloc(scratch_ctx, btmp.off + 256);
        if (!sbuf) return fail(GSR_ERR_ALLOC, "scratch allocation failed");
        btmp = Carver(aligned_base(sbuf));
    }
    carve_binning(aligned_base(bbuf), (int)K, P, p.grid_x, p.grid_y, path, bs, scratch_alloc ? &btmp : nullptr);
    ChunkState cs{};
    void* cbuf = dup_tile_alloc(dup_tile_ctx, carve_chunks(nullptr, n_chunks, cs));
    if (!cbuf) return fail(GSR_ERR_ALLOC, "duplicated-tile buffer allocation failed");
    carve_chunks(aligned_base(cbuf), n_chunks, cs);
    if (path == kBinLists) {
        GSR_STAGE(GSR_STAGE_TILE_LISTS, launch_list_binning(p, gs, gs.radii, bs, ts, (int)K, stream), "tile lists");
    } else {
        const int tile_bits = (int)higher_msb(tiles);
        GSR_STAGE(GSR_STAGE_EMIT_KEYS, launch_emit_keys(p, gs, gs.radii, bs, stream), "emit keys");
        GSR_STAGE(GSR_STAGE_SORT, launch_sort(bs, (int)K_live, tile_bits, stream), "sort");
        GSR_STAGE(GSR_STAGE_TILE_RANGES, launch_tile_ranges(bs, (int)K_live, ts, (int)tiles, stream), "tile ranges");
    }
    // (heaviest-first chunk order with the tile's list length as the cost
    // was measured for this forward: no change, 1.52 vs 1.51 ms at 1.27M points)
    GSR_STAGE(GSR_STAGE_SAMPLE_FWD,
              launch_point_fwd(query, p, gs, bs, ts, ps, pb, st, cs, n_chunks, output, output2, inside, stream),
              "point query");
    if (num_rendered) *num_rendered = (int)K;
    if (num_points) *num_points = (int)totals[0];
    if (num_duplicated_tiles) *num_duplicated_tiles = (int)totals[1];
    return GSR_OK;
}

int gsr_sample_depth_forward(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                             gsr_alloc_fn point_alloc, void* point_ctx, gsr_alloc_fn point_binning_alloc,
                             void* point_binning_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                             gsr_alloc_fn dup_tile_alloc, void* dup_tile_ctx, int PN, int P, int width, int height,
                             const float* points3D, const float* means3D, const float* opacities,
                             const float* scales, float scale_modifier, const float* rotations,
                             const float* cov3D_precomp, const float* viewmatrix, const float* projmatrix,
                             const float* cam_pos, float tan_fovx, float tan_fovy, float kernel_size,
                             int prefiltered, float* output, uint8_t* inside, int debug, void* stream_ptr,
                             int* num_rendered, int* num_points, int* num_duplicated_tiles) {
    return point_query_forward(kQuerySample, geom_alloc, geom_ctx, binning_alloc, binning_ctx, point_alloc,
                               point_ctx, point_binning_alloc, point_binning_ctx, tile_alloc, tile_ctx,
                               dup_tile_alloc, dup_tile_ctx, PN, P, width, height, points3D, means3D, opacities,
                               scales, scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos,
                               tan_fovx, tan_fovy, kernel_size, prefiltered, output, nullptr, inside, debug,
                               stream_ptr, num_rendered, num_points, num_duplicated_tiles);
}

int gsr_sample_depth_forward_ex(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc,
                                void* binning_ctx, gsr_alloc_fn point_alloc, void* point_ctx,
                                gsr_alloc_fn point_binning_alloc, void* point_binning_ctx, gsr_alloc_fn tile_alloc,
                                void* tile_ctx, gsr_alloc_fn dup_tile_alloc, void* dup_tile_ctx, int PN, int P,
                                int width, int height, const float* points3D, const float* means3D,
                                const float* opacities, const float* scales, float scale_modifier,
                                const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                                const float* projmatrix, const float* cam_pos, float tan_fovx, float tan_fovy,
                                float kernel_size, int prefiltered, float* output, uint8_t* inside, int debug,
                                void* stream_ptr, int* num_rendered, int* num_points, int* num_duplicated_tiles,
                                gsr_alloc_fn scratch_alloc, void* scratch_ctx) {
    return point_query_forward(kQuerySample, geom_alloc, geom_ctx, binning_alloc, binning_ctx, point_alloc,
                               point_ctx, point_binning_alloc, point_binning_ctx, tile_alloc, tile_ctx,
                               dup_tile_alloc, dup_tile_ctx, PN, P, width, height, points3D, means3D, opacities,
                               scales, scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos,
                               tan_fovx, tan_fovy, kernel_size, prefiltered, output, nullptr, inside, debug,
                               stream_ptr, num_rendered, num_points, num_duplicated_tiles, scratch_alloc,
                               scratch_ctx);
}

int gsr_integrate_forward(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                          gsr_alloc_fn point_alloc, void* point_ctx, gsr_alloc_fn point_binning_alloc,
                          void* point_binning_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                          gsr_alloc_fn dup_tile_alloc, void* dup_tile_ctx, int PN, int P, int width, int height,
                          const float* points3D, const float* means3D, const float* opacities, const float* scales,
                          float scale_modifier, const float* rotations, const float* cov3D_precomp,
                          const float* view2gaussian_precomp, const float* viewmatrix, const float* projmatrix,
                          const float* cam_pos, float tan_fovx, float tan_fovy, float kernel_size, int prefiltered,
                          float* out_transmittance, uint8_t* inside, int debug, void* stream_ptr,
                          int* num_rendered) {
    (void)view2gaussian_precomp;  // unused by the reference (rasterizer_impl.cu:610)
    return point_query_forward(kQueryIntegrate, geom_alloc, geom_ctx, binning_alloc, binning_ctx, point_alloc,
                               point_ctx, point_binning_alloc, point_binning_ctx, tile_alloc, tile_ctx,
                               dup_tile_alloc, dup_tile_ctx, PN, P, width, height, points3D, means3D, opacities,
                               scales, scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos,
                               tan_fovx, tan_fovy, kernel_size, prefiltered, out_transmittance, nullptr, inside,
                               debug, stream_ptr, num_rendered, nullptr, nullptr);
}

int gsr_evaluate_sdf_forward(gsr_alloc_fn geom_alloc, void* geom_ctx, gsr_alloc_fn binning_alloc, void* binning_ctx,
                             gsr_alloc_fn point_alloc, void* point_ctx, gsr_alloc_fn point_binning_alloc,
                             void* point_binning_ctx, gsr_alloc_fn tile_alloc, void* tile_ctx,
                             gsr_alloc_fn dup_tile_alloc, void* dup_tile_ctx, int PN, int P, int width, int height,
                             const float* points3D, const float* means3D, const float* opacities,
                             const float* scales, float scale_modifier, const float* rotations,
                             const float* cov3D_precomp, const float* view2gaussian_precomp,
                             const float* viewmatrix, const float* projmatrix, const float* cam_pos, float tan_fovx,
                             float tan_fovy, float kernel_size, int prefiltered, float* out_depth, float* out_sdf,
                             uint8_t* inside, int debug, void* stream_ptr, int* num_rendered) {
    (void)view2gaussian_precomp;  // unused by the reference (rasterizer_impl.cu:833)
    return point_query_forward(kQuerySDF, geom_alloc, geom_ctx, binning_alloc, binning_ctx, point_alloc, point_ctx,
                               point_binning_alloc, point_binning_ctx, tile_alloc, tile_ctx, dup_tile_alloc,
                               dup_tile_ctx, PN, P, width, height, points3D, means3D, opacities, scales,
                               scale_modifier, rotations, cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx,
                               tan_fovy, kernel_size, prefiltered, out_depth, out_sdf, inside, debug, stream_ptr,
                               num_rendered, nullptr, nullptr);
}

int gsr_sample_depth_backward(gsr_alloc_fn geom_bwd_alloc, void* geom_bwd_ctx, int PN, int P, int RN, int R, int TN,
                              int width, int height, const float* points3D, const float* means3D,
                              const float* opacities, const float* scales, float scale_modifier,
                              const float* rotations, const float* cov3D_precomp, const float* viewmatrix,
                              const float* projmatrix, const float* campos, float tan_fovx, float tan_fovy,
                              float kernel_size, const void* geom_buffer, const void* binning_buffer,
                              const void* point_buffer, const void* point_binning_buffer, const void* tile_buffer,
                              const void* dup_tile_buffer, const uint8_t* inside, const float* dL_doutput,
                              float* dL_dopacity, float* dL_dmean3D, float* dL_dcov3D, float* dL_dscale,
                              float* dL_drot, float* dL_dpoints3D, int debug, void* stream_ptr) {
    (void)RN;
    (void)TN;
    hipStream_t stream = (hipStream_t)stream_ptr;
    if (P == 0 || PN == 0) return GSR_OK;
    if (P < 0 || PN < 0 || width <= 0 || height <= 0) return fail(GSR_ERR_ARGS, "invalid P / PN / image size");
    static const float kZeroBg[3] = {0.f, 0.f, 0.f};
    SampleBwdParams b;
    b.f = make_params(P, 0, 0, 0, 0, kZeroBg, width, height, means3D, nullptr, opacities, scales, rotations,
                      cov3D_precomp, nullptr, nullptr, nullptr, nullptr, scale_modifier, viewmatrix, projmatrix,
                      campos, tan_fovx, tan_fovy, kernel_size, 1);
    b.f.no_color = true;
    b.f.cull_pad = 0.5f;
    b.PN = PN;
    b.points3D = points3D;
    b.inside = inside;
    b.dL_doutput = dL_doutput;
    b.dL_dpoints3D = dL_dpoints3D;
    if (!geom_buffer || !binning_buffer || !point_buffer || !point_binning_buffer || !tile_buffer ||
        !dup_tile_buffer || !inside || !dL_doutput || !dL_dopacity || !dL_dmean3D || !dL_dpoints3D || !points3D)
        return fail(GSR_ERR_ARGS, "missing backward buffer");
    if (scales && (!dL_dscale || !dL_drot)) return fail(GSR_ERR_ARGS, "missing scale/rotation gradients");
    if (cov3D_precomp && !dL_dcov3D) return fail(GSR_ERR_ARGS, "missing cov3D gradient");
    const uint32_t tiles = b.f.grid_x * b.f.grid_y;
    GeomState gs;
    carve_geom(aligned_base(const_cast<void*>(geom_buffer)), P, b.f.grid_x, b.f.grid_y, gs);
    BinningState bs;  // (the backward reads the point list only: first in every layout)
    carve_binning(aligned_base(const_cast<void*>(binning_buffer)), R, P, b.f.grid_x, b.f.grid_y,
                  bin_path(b.f.grid_x, b.f.grid_y), bs);
    PointState ps;
    carve_points(aligned_base(const_cast<void*>(point_buffer)), PN, ps);
    PointBinState pb;
    carve_point_binning(aligned_base(const_cast<void*>(point_binning_buffer)), PN, tiles, pb);
    TileState ts{};
    SampleTiles st;
    carve_sample_tiles(aligned_base(const_cast<void*>(tile_buffer)), (int)tiles, ts, st);
    ChunkState cs;
    {
        Carver c(aligned_base(const_cast<void*>(dup_tile_buffer)));
        cs.chunk_max = c.take<uint32_t>(1);  // first in the buffer (carve_chunks)
    }
    BwdState ws{};
    const uint32_t bound = PN > 0 ? sample_chunk_bound(PN, tiles) : 0u;
    const size_t wbytes = carve_bwd(nullptr, P, ws, (int)bound);
    void* wbuf = geom_bwd_alloc(geom_bwd_ctx, wbytes + 256);
    if (!wbuf) return fail(GSR_ERR_ALLOC, "backward buffer allocation failed");
    void* wb = aligned_base(wbuf);
    carve_bwd(wb, P, ws, (int)bound);
    GSR_STAGE(GSR_STAGE_BWD_CLEAR, hipMemsetAsync(wb, 0, wbytes, stream), "memset accumulators");
    if (bound)  // heaviest chunks first (cost: the forward's chunk max contributor)
        GSR_STAGE(GSR_STAGE_BWD_CLEAR, launch_chunk_order(bound, st.totals + 2, cs.chunk_max, ws.tile_order, stream),
                  "chunk order");
    else
        ws.tile_order = nullptr;
    GSR_STAGE(GSR_STAGE_SAMPLE_BWD, launch_sample_bwd(b, gs, bs, ts, ps, pb, st, cs, ws, stream), "sample backward");
    BwdParams pbw{};
    pbw.f = b.f;
    pbw.R = R;
    pbw.radii = gs.radii;
    pbw.dL_dmean3D = dL_dmean3D;
    pbw.dL_dopacity = dL_dopacity;
    pbw.dL_dscale = dL_dscale;
    pbw.dL_drot = dL_drot;
    pbw.dL_dcov3D = dL_dcov3D;
    GSR_STAGE(GSR_STAGE_PREPROCESS_BWD, launch_preprocess_bwd(pbw, gs, ws, stream), "preprocess backward");
    return GSR_OK;
}

int gsr_adam_step(int n_groups, const gsr_adam_group* groups, double step, double beta1, double beta2, double eps,
                  void* stream_ptr) {
    if (n_groups < 0 || n_groups > kMaxAdamGroups || (n_groups > 0 && !groups) || !(step >= 1.0))
        return fail(GSR_ERR_ARGS, "adam: 0..16 groups and step >= 1");
    AdamGroup g[kMaxAdamGroups];
    double lr[kMaxAdamGroups];
    for (int k = 0; k < n_groups; k++) {
        const gsr_adam_group& s = groups[k];
        if (s.n < 0 || (s.n > 0 && (!s.param || !s.grad || !s.exp_avg || !s.exp_avg_sq)))
            return fail(GSR_ERR_ARGS, "adam: missing group buffer");
        g[k].param = s.param;
        g[k].grad = s.grad;
        g[k].exp_avg = s.exp_avg;
        g[k].exp_avg_sq = s.exp_avg_sq;
        g[k].n = s.n;
        const uintptr_t bits = (uintptr_t)s.param | (uintptr_t)s.grad | (uintptr_t)s.exp_avg | (uintptr_t)s.exp_avg_sq;
        g[k].aligned = (bits & 15u) == 0;
        lr[k] = s.lr;
    }
    hipError_t e = launch_adam(n_groups, g, lr, step, beta1, beta2, eps, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "adam", e);
}

int gsr_densify_stats(int P, const float* vgrad, const int* radii, float* max_radii2D, float* accum,
                      float* accum_abs, float* denom, void* stream_ptr) {
    if (P < 0 || (P > 0 && (!vgrad || !radii || !max_radii2D || !accum || !accum_abs || !denom)))
        return fail(GSR_ERR_ARGS, "densify stats: invalid arguments");
    hipError_t e = launch_densify_stats(P, vgrad, radii, max_radii2D, accum, accum_abs, denom, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "densify stats", e);
}

int gsr_view_color_grads_chunked(int P, int sh_degree, int SHM, int sg_degree, int SGM, int n_views, int chunk,
                                 const float* gathered, const float* campos, const float* means3D,
                                 const float* sg_axis, const float* sg_sharpness, const float* sg_color,
                                 float* dL_dsh, float* dL_dsg_axis, float* dL_dsg_sharpness, float* dL_dsg_color,
                                 float* dL_dsh_rest, void* stream_ptr) {
    if (P < 0 || n_views < 1 || chunk < 1 || sh_degree < 0 || sh_degree > 3 ||
        SHM < (sh_degree + 1) * (sh_degree + 1) || SGM < 0 || sg_degree < 0 || sg_degree > 7 || sg_degree > SGM ||
        (dL_dsh_rest && SHM < 2))
        return fail(GSR_ERR_ARGS, "view colour grads: invalid arguments");
    if (P > 0 && (!gathered || !campos || !means3D || !dL_dsh ||
                  (SGM > 0 && (!dL_dsg_axis || !dL_dsg_sharpness || !dL_dsg_color)) ||
                  (sg_degree > 0 && (!sg_axis || !sg_sharpness || !sg_color))))
        return fail(GSR_ERR_ARGS, "view colour grads: missing buffer");
    hipError_t e = launch_view_color_grads(P, sh_degree, SHM, sg_degree, SGM, n_views, gathered, means3D, sg_axis,
                                           sg_sharpness, sg_color, dL_dsh, dL_dsg_axis, dL_dsg_sharpness,
                                           dL_dsg_color, (hipStream_t)stream_ptr, chunk, campos, dL_dsh_rest);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "view colour grads", e);
}

int gsr_view_color_grads(int P, int sh_degree, int SHM, int sg_degree, int SGM, int n_views, const float* gathered,
                         const float* means3D, const float* sg_axis, const float* sg_sharpness, const float* sg_color,
                         float* dL_dsh, float* dL_dsg_axis, float* dL_dsg_sharpness, float* dL_dsg_color,
                         void* stream_ptr) {
    if (P < 0 || n_views < 1 || sh_degree < 0 || sh_degree > 3 || SHM < (sh_degree + 1) * (sh_degree + 1) ||
        SGM < 0 || sg_degree < 0 || sg_degree > 7 || sg_degree > SGM)
        return fail(GSR_ERR_ARGS, "view colour grads: invalid arguments");
    if (P > 0 && (!gathered || !means3D || !dL_dsh ||
                  (SGM > 0 && (!dL_dsg_axis || !dL_dsg_sharpness || !dL_dsg_color)) ||
                  (sg_degree > 0 && (!sg_axis || !sg_sharpness || !sg_color))))
        return fail(GSR_ERR_ARGS, "view colour grads: missing buffer");
    hipError_t e = launch_view_color_grads(P, sh_degree, SHM, sg_degree, SGM, n_views, gathered, means3D, sg_axis,
                                           sg_sharpness, sg_color, dL_dsh, dL_dsg_axis, dL_dsg_sharpness,
                                           dL_dsg_color, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "view colour grads", e);
}

int gsr_warp_patch_ncc(int P, const float* depths, const float* normals, const int* uvs, const float* R,
                       const float* T, const float* image_r, const float* image_n, float fx_r, float fy_r,
                       float cx_r, float cy_r, float fx_n, float fy_n, float cx_n, float cy_n, int image_height_r,
                       int image_width_r, int image_height_n, int image_width_n, float* ncc, float* grad_depths,
                       float* grad_normals, uint8_t* valid, void* stream_ptr) {
    if (P < 0 || image_height_r <= 0 || image_width_r <= 0 || image_height_n <= 0 || image_width_n <= 0)
        return fail(GSR_ERR_ARGS, "warp_patch_ncc: invalid sizes");
    if (P > 0 && (!depths || !normals || !uvs || !R || !T || !image_r || !image_n || !ncc || !grad_depths ||
                  !grad_normals || !valid))
        return fail(GSR_ERR_ARGS, "warp_patch_ncc: missing buffer");
    NccParams q{P, depths, normals, uvs, R, T, image_r, image_n, fx_r, fy_r, cx_r, cy_r, fx_n, fy_n, cx_n, cy_n,
                image_height_r, image_width_r, image_height_n, image_width_n, ncc, grad_depths, grad_normals, valid};
    hipError_t e = launch_ncc(q, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "warp_patch_ncc", e);
}

int gsr_scale_opacity_3d_filter(int P, const float* scaling, const float* opacity, const float* filter_3D,
                                float* scales, float* opacities, void* stream_ptr) {
    if (P < 0 || (P > 0 && (!scaling || !opacity || !filter_3D || !scales || !opacities)))
        return fail(GSR_ERR_ARGS, "scale/opacity getter: invalid arguments");
    hipError_t e = launch_scale_opacity(P, scaling, opacity, filter_3D, scales, opacities, nullptr, nullptr, nullptr,
                                        nullptr, false, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "scale/opacity getter", e);
}

int gsr_scale_opacity_3d_filter_backward(int P, const float* scaling, const float* opacity, const float* filter_3D,
                                         const float* dL_dscales, const float* dL_dopacities, float* dL_dscaling,
                                         float* dL_dopacity, void* stream_ptr) {
    if (P < 0 || (P > 0 && (!scaling || !opacity || !filter_3D || !dL_dscaling || !dL_dopacity)))
        return fail(GSR_ERR_ARGS, "scale/opacity getter backward: invalid arguments");
    hipError_t e = launch_scale_opacity(P, scaling, opacity, filter_3D, nullptr, nullptr, dL_dscales, dL_dopacities,
                                        dL_dscaling, dL_dopacity, true, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "scale/opacity getter backward", e);
}

int gsr_normalize_rows(int n, int D, const float* x, float* y, void* stream_ptr) {
    if (n < 0 || D <= 0 || (n > 0 && (!x || !y))) return fail(GSR_ERR_ARGS, "normalize: invalid arguments");
    hipError_t e = launch_normalize_rows(n, D, x, nullptr, y, false, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "normalize", e);
}

int gsr_normalize_rows_backward(int n, int D, const float* x, const float* dL_dy, float* dL_dx, void* stream_ptr) {
    if (n < 0 || D <= 0 || (n > 0 && (!x || !dL_dy || !dL_dx)))
        return fail(GSR_ERR_ARGS, "normalize backward: invalid arguments");
    hipError_t e = launch_normalize_rows(n, D, x, dL_dy, dL_dx, true, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "normalize backward", e);
}

int gsr_patchmatch_lift(int H, int W, float Fx, float Fy, float Cx, float Cy, const float* T, const float* M,
                        const float* median_depth, float* points, void* stream_ptr) {
    if (H < 0 || W < 0 || (H * W > 0 && (!T || !M || !median_depth || !points)))
        return fail(GSR_ERR_ARGS, "patchmatch lift: invalid arguments");
    hipError_t e = launch_patchmatch_lift(false, H, W, Fx, Fy, Cx, Cy, T, M, median_depth, nullptr, points,
                                          (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "patchmatch lift", e);
}

int gsr_patchmatch_lift_backward(int H, int W, float Fx, float Fy, float Cx, float Cy, const float* M,
                                 const float* dL_dpoints, float* dL_dmedian_depth, void* stream_ptr) {
    if (H < 0 || W < 0 || (H * W > 0 && (!M || !dL_dpoints || !dL_dmedian_depth)))
        return fail(GSR_ERR_ARGS, "patchmatch lift backward: invalid arguments");
    hipError_t e = launch_patchmatch_lift(true, H, W, Fx, Fy, Cx, Cy, nullptr, M, nullptr, dL_dpoints,
                                          dL_dmedian_depth, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "patchmatch lift backward", e);
}

static const char* pm_check(int H, int W, const float* md, const float* normal, const float* pin,
                            const uint8_t* inside, const float* Mv, const float* tv, const float* R, const float* T,
                            const float* image_r, const float* image_n, int Hn, int Wn, const float* saved_w,
                            const uint8_t* saved_flags, const float* saved_gd, const float* saved_gn) {
    if (H <= 0 || W <= 0 || Hn <= 0 || Wn <= 0) return "patchmatch: invalid sizes";
    if (!md || !normal || !pin || !inside || !Mv || !tv || !R || !T || !image_r || !image_n || !saved_w ||
        !saved_flags || !saved_gd || !saved_gn)
        return "patchmatch: missing buffer";
    return nullptr;
}

int gsr_patchmatch_terms_forward(gsr_alloc_fn scratch_alloc, void* scratch_ctx, int H, int W,
                                 const float* median_depth, const float* normal, const float* points_nearest,
                                 const uint8_t* inside, const float* Mv, const float* tv, float Fx, float Fy, float Cx,
                                 float Cy, float noise_th, const float* R, const float* T, const float* image_r,
                                 const float* image_n, float fx_r, float fy_r, float cx_r, float cy_r, float fx_n,
                                 float fy_n, float cx_n, float cy_n, int image_height_n, int image_width_n,
                                 float* saved_w, uint8_t* saved_flags, float* saved_gd, float* saved_gn,
                                 float* out4, void* stream_ptr) {
    if (const char* m = pm_check(H, W, median_depth, normal, points_nearest, inside, Mv, tv, R, T, image_r, image_n,
                                 image_height_n, image_width_n, saved_w, saved_flags, saved_gd, saved_gn))
        return fail(GSR_ERR_ARGS, m);
    if (!out4 || !scratch_alloc) return fail(GSR_ERR_ARGS, "patchmatch: missing buffer");
    void* buf = scratch_alloc(scratch_ctx, patchmatch_partials(H, W) * sizeof(float) + 256);
    if (!buf) return fail(GSR_ERR_ALLOC, "patchmatch: scratch allocation failed");
    PatchMatchParams q{H, W, median_depth, normal, points_nearest, inside, Mv, tv, Fx, Fy, Cx, Cy, noise_th, R, T,
                       image_r, image_n, fx_r, fy_r, cx_r, cy_r, fx_n, fy_n, cx_n, cy_n, image_height_n,
                       image_width_n, saved_w, saved_flags, saved_gd, saved_gn};
    hipError_t e = launch_patchmatch_terms(q, reinterpret_cast<float*>(aligned_base(buf)), out4,
                                           (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "patchmatch terms", e);
}

int gsr_patchmatch_terms_backward(int H, int W, const float* median_depth, const float* normal,
                                  const float* points_nearest, const uint8_t* inside, const float* Mv, const float* tv,
                                  float Fx, float Fy, float Cx, float Cy, float noise_th, const float* R,
                                  const float* T, const float* image_r, const float* image_n, float fx_r, float fy_r,
                                  float cx_r, float cy_r, float fx_n, float fy_n, float cx_n, float cy_n,
                                  int image_height_n, int image_width_n, const float* saved_w,
                                  const uint8_t* saved_flags, const float* saved_gd, const float* saved_gn,
                                  const float* out4, const float* dL_dloss2, float* dL_dpoints_nearest,
                                  float* dL_dmedian_depth, float* dL_dnormal, void* stream_ptr) {
    if (const char* m = pm_check(H, W, median_depth, normal, points_nearest, inside, Mv, tv, R, T, image_r, image_n,
                                 image_height_n, image_width_n, saved_w, saved_flags, saved_gd, saved_gn))
        return fail(GSR_ERR_ARGS, m);
    if (!out4 || !dL_dloss2 || !dL_dpoints_nearest || !dL_dmedian_depth || !dL_dnormal)
        return fail(GSR_ERR_ARGS, "patchmatch backward: missing buffer");
    PatchMatchParams q{H, W, median_depth, normal, points_nearest, inside, Mv, tv, Fx, Fy, Cx, Cy, noise_th, R, T,
                       image_r, image_n, fx_r, fy_r, cx_r, cy_r, fx_n, fy_n, cx_n, cy_n, image_height_n,
                       image_width_n, const_cast<float*>(saved_w), const_cast<uint8_t*>(saved_flags),
                       const_cast<float*>(saved_gd), const_cast<float*>(saved_gn)};
    hipError_t e = launch_patchmatch_terms_bwd(q, out4, dL_dloss2, dL_dpoints_nearest, dL_dmedian_depth, dL_dnormal,
                                               (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "patchmatch terms backward", e);
}

int gsr_fused_ssim_forward(gsr_alloc_fn scratch_alloc, void* scratch_ctx, int NC, int H, int W, int valid,
                           const float* img1, const float* img2, float* out_mean, float* factors, void* stream_ptr) {
    if (NC <= 0 || H <= 0 || W <= 0 || (valid && (H <= 10 || W <= 10)))
        return fail(GSR_ERR_ARGS, "fused_ssim: invalid sizes (valid padding needs H, W > 10)");
    if (!img1 || !img2 || !out_mean || !scratch_alloc) return fail(GSR_ERR_ARGS, "fused_ssim: missing buffer");
    const size_t n = ssim_partials(NC, H, W);
    void* buf = scratch_alloc(scratch_ctx, n * sizeof(float) + 256);
    if (!buf) return fail(GSR_ERR_ALLOC, "fused_ssim: scratch allocation failed");
    float* partial = reinterpret_cast<float*>(aligned_base(buf));
    const size_t plane = (size_t)NC * H * W;
    hipError_t e = launch_ssim_fwd(NC, H, W, valid, img1, img2, factors, factors ? factors + plane : nullptr,
                                   factors ? factors + 2 * plane : nullptr, partial, out_mean, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "fused_ssim forward", e);
}

int gsr_fused_ssim_backward(int NC, int H, int W, int valid, const float* img1, const float* img2,
                            const float* factors, const float* dL_dmean, float* dL_dimg1, void* stream_ptr) {
    if (NC <= 0 || H <= 0 || W <= 0 || (valid && (H <= 10 || W <= 10)))
        return fail(GSR_ERR_ARGS, "fused_ssim: invalid sizes");
    if (!img1 || !img2 || !factors || !dL_dmean || !dL_dimg1) return fail(GSR_ERR_ARGS, "fused_ssim: missing buffer");
    const size_t plane = (size_t)NC * H * W;
    hipError_t e = launch_ssim_bwd(NC, H, W, valid, img1, img2, factors, factors + plane, factors + 2 * plane,
                                   dL_dmean, dL_dimg1, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "fused_ssim backward", e);
}

int gsr_depth_to_normal_forward(const float* depth, int H, int W, float Fx, float Fy, float Cx, float Cy,
                                float* normal, uint8_t* valid, void* stream_ptr) {
    if (H < 0 || W < 0 || (H * W > 0 && (!depth || !normal || !valid)))
        return fail(GSR_ERR_ARGS, "depth_to_normal: invalid arguments");
    hipError_t e = launch_depth_normal(false, depth, H, W, Fx, Fy, Cx, Cy, nullptr, normal, valid,
                                       (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "depth_to_normal", e);
}

int gsr_depth_to_normal_backward(const float* depth, int H, int W, float Fx, float Fy, float Cx, float Cy,
                                 const float* dL_dnormal, float* dL_ddepth, void* stream_ptr) {
    if (H < 0 || W < 0 || (H * W > 0 && (!depth || !dL_dnormal || !dL_ddepth)))
        return fail(GSR_ERR_ARGS, "depth_to_normal backward: invalid arguments");
    hipError_t e = launch_depth_normal(true, depth, H, W, Fx, Fy, Cx, Cy, dL_dnormal, dL_ddepth, nullptr,
                                       (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "depth_to_normal backward", e);
}

int gsr_knn_mean_dist(gsr_alloc_fn scratch_alloc, void* scratch_ctx, int P, const float* points,
                      float* mean_dists, void* stream_ptr) {
    if (P < 0) return fail(GSR_ERR_ARGS, "distCUDA2: P < 0");
    if (P == 0) return GSR_OK;
    if (!points || !mean_dists || !scratch_alloc) return fail(GSR_ERR_ARGS, "distCUDA2: missing buffer");
    KnnState ks;
    void* buf = scratch_alloc(scratch_ctx, carve_knn(nullptr, P, ks));
    if (!buf) return fail(GSR_ERR_ALLOC, "distCUDA2: scratch allocation failed");
    carve_knn(aligned_base(buf), P, ks);
    hipError_t e = launch_knn(P, points, ks, mean_dists, (hipStream_t)stream_ptr);
    return e == hipSuccess ? GSR_OK : fail(GSR_ERR_HIP, "distCUDA2", e);
}

int gsr_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, void* stream_ptr) {
    (void)projmatrix;
    if (P < 0 || (P > 0 && (!means3D || !viewmatrix || !present))) return fail(GSR_ERR_ARGS, "invalid arguments");
    hipError_t e = launch_mark_visible(P, means3D, viewmatrix, present, (hipStream_t)stream_ptr);
    if (e != hipSuccess) return fail(GSR_ERR_HIP, "mark_visible", e);
    return GSR_OK;
}

}  // extern "C"
