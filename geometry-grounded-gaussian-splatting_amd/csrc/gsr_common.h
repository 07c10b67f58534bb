// gsr_common.h — shared constants, HBM layouts and wave64 helpers for the
// gfx950 rasterizer kernels.
//
// Semantics follow the reference's compile-time configuration
// (DGR/cuda_rasterizer/config.h:21-40): 16x16 tiles are semantic (they decide
// which Gaussians a pixel sees), SPLIT = 8 samples x 5 bisection iterations
// over +-0.4 around the initial median depth, MIN_TRANSMITTANCE = 0.45.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsr {

constexpr int kTile = 16;                 // BLOCK_X = BLOCK_Y
constexpr int kTilePixels = kTile * kTile;  // one workgroup (4 wave64) per tile
constexpr int kSplit = 8;
constexpr int kSplitIterations = 5;
constexpr float kSampleRange = 0.4f;
constexpr float kMinTransmittance = 0.45f;
constexpr float kNearPlane = 0.2f;

// --------------------------------------------------------------------------
// Per-Gaussian render record ("splat"), written by the preprocess and
// gathered by both render kernels.  64 B = four 16-B words, one aligned
// 64-B segment per Gaussian:
//   w0 = (x_pix, y_pix, conic.x, conic.y)
//   w1 = (conic.z, opacity*coef, plane.x, plane.y)
//   w2 = (plane.z = |t|, plane.w = rsigma, r, g)
//   w3 = (b, n.x, n.y, n.z)
// The median-depth bisection needs only w0, w1, w2.xy (48 B).
// --------------------------------------------------------------------------
struct alignas(16) Splat {
    float4 w0, w1, w2, w3;
};

// Per-Gaussian gradient accumulator written by the backward render with
// wave-wide atomics: 16 fields in one 64-B record + the |dmean2D| channel in
// a separate dense array.
//   0..2  dL/dcolor          3..4  dL/dmean2D (x, y; NDC units)
//   5..8  dL/dconic (x, y, z) and dL/d(opacity-weighted) w
//   9..11 dL/dnormal         12..15 dL/dray_plane (x, y, tc, rsigma)
enum AccField : int {
    kAccColor = 0, kAccMean2D = 3, kAccConic = 5, kAccNormal = 9, kAccPlane = 12, kAccFields = 16
};

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Carves a byte buffer into typed arrays, 256-B aligned.
struct Carver {
    char* base;
    size_t off;
    __host__ explicit Carver(void* b) : base(static_cast<char*>(b)), off(0) {}
    template <class T>
    __host__ T* take(size_t count) {
        off = align_up(off, 256);
        T* p = reinterpret_cast<T*>(base + off);
        off += count * sizeof(T);
        return p;
    }
};

// ---- per-Gaussian forward state (replaces GeometryState, rasterizer_impl.h) ----
struct GeomState {
    Splat* splats;
    float* depths;
    uint32_t* tiles_touched;
    uint32_t* order;              // Gaussian indices in (depth bits, index) order
    uint32_t* depth_keys_sorted;  // sorted depth bit patterns (sort output, unused after)
    uint32_t* tiles_live;         // tiles of the rect that pass the tile test (binning.hip)
    uint2* counts;                // per Gaussian in depth order: (tiles_touched, live tiles)
    uint2* offsets;               // inclusive scan of counts: .x -> K (reference count), .y -> live instances
    uint32_t* offsets_K;          // (tile-list path) K = sum of tiles_touched
    uint32_t* near_flag;          // prefiltered check: 1 if a Gaussian fails the near-plane test
    int* radii;                   // internal copy when the caller passes radii == NULL
    uint8_t* clamped;             // bit c set: colour channel c was clamped at 0
    float* ddir;                  // SH colour's direction Jacobian (gsr_math.h sh_basis_grad): 9 planes of P floats
    void* scan_tmp;
    size_t scan_tmp_bytes;
    void* dsort_tmp;
    size_t dsort_tmp_bytes;
    uint4* foot;  // forward-only: [P][2] tile footprint (x, y, conic.a, conic.b), (conic.c, opacity coef, rect) (tilelists.hip)
};
// ---- per-instance state (replaces BinningState) ----
// tile ids as 16-bit sort keys when the grid allows (<= 65536 tiles)
inline int tile_key_bytes(int tile_bits) { return tile_bits <= 16 ? 2 : 4; }
// Tile-list binning (tilelists.hip): grids up to kMaxGrid x kMaxGrid tiles.
constexpr int kMaxGrid = 1024;
enum BinPath : int { kBinInstanceSort = 0, kBinLists = 1 };
struct ListLayout {
    int nseg_rows = 0, nseg_tiles_max = 0, rowseg = 64;
    size_t tmp_bytes = 0;
};
struct BinningState {
    uint32_t* point_list;  // first in the buffer: its offset depends on nothing else
    int path;              // BinPath
    bool use_lists;        // tilelists.hip path
    ListLayout lists;
    uint2* rows;           // (Gaussian, column span) per tile row, q order
    uint4* qrec;           // [P][2] per Gaussian in q order: id, rows y0 | y1 << 16, spans of rows y0 .. y0 + 5
    uint32_t *rows_count, *rows_off, *segbase, *tiles_count, *tiles_off;
    void* list_tmp;
    int key_bytes;        // 2 or 4 (tile_key_bytes)
    void* keys_unsorted;  // tile id per instance, emission (depth) order
    void* keys;           // tile ids sorted
    uint32_t* values_unsorted;
    void* sort_tmp;
    size_t sort_tmp_bytes;
};
// ---- per-pixel / per-tile state (ImageState, TileState<false>) ----
struct ImageState {
    uint32_t* n_contrib;
    float* dT_dtm;       // GEOM: median-depth implicit derivative, computed by the forward
    uint32_t* md_check;  // bits of the mdepth output it belongs to (NaN pattern: not cached)
};
constexpr uint32_t kNoCache = 0x7fffffffu;
// The first kBlendWords * 32 entries of a tile's list: bit set where at least
// one pixel of the tile blended the entry in the forward composite (render_fwd).
// For an entry before a pixel's last contributor, "blended" is exactly the
// backward's per-pixel validity (power <= 0, alpha >= 1/255 with the same
// rounding), so the backward skips the unset entries without evaluating them.
constexpr int kBlendWords = 8;
struct TileState {
    uint2* ranges;
    uint32_t* max_contrib;
    uint32_t* order;       // launch order of the tiles, heaviest first (tile_order_kernel)
    uint32_t* blend_mask;  // [T][kBlendWords]
    uint32_t* bwd_cost;    // [T] entries the backward walks: set bits of blend_mask + entries past it
};
// ---- sample_depth state (PointState / DuplicatedTileState, rasterizer_impl.h) ----
constexpr uint32_t kNoTile = 0xffffffffu;
struct PointState {  // per point (point buffer)
    float2* xy;        // projected position (pixels)
    uint32_t* last;    // last contributor
    float* mdepth;     // median depth along the ray (the reference's pointState.median_depth)
    float* dT;         // dT/dt_m at mdepth, computed by the forward when `cached`
    uint8_t* cached;
    float* t;          // |p_view| (preprocessPointsCUDA ts, sample_forward.cu:50; integrate / evaluate_sdf)
};
struct PointBinState {  // point binning buffer
    uint32_t* keys_unsorted;  // tile of each point (num_tiles when culled: sorts last)
    uint32_t* keys;
    uint32_t* pt_list;        // point indices stably sorted by tile
    void* sort_tmp;
    size_t sort_tmp_bytes;
};
struct SampleTiles {  // per tile, after TileState in the tile buffer
    uint32_t* counts;     // valid points per tile
    uint2* pt_ranges;     // [first, end) in pt_list
    uint32_t* chunk_off;  // [tiles + 1]: exclusive scan of ceil(count / 256)
    uint32_t* totals;     // [4]: valid points, reference blocks (512 points each), chunks, 0
};
struct ChunkState {  // duplicated-tile buffer: one entry per 256-point chunk
    uint32_t* chunk_max;  // max contributor over the chunk's points
};

// ---- backward scratch (replaces GeometryBwdState) ----
struct BwdState {
    float* acc;      // [P][16]
    float* acc_abs;  // [P]
    uint32_t* tile_order;  // [tiles] backward launch order, heaviest first
};

// --------------------------------------------------------------------------
// wave64 helpers
// --------------------------------------------------------------------------
__device__ inline float wave_max_f(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ inline uint32_t wave_max_u(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t w = __shfl_xor(v, o, 64);
        v = v > w ? v : w;
    }
    return v;
}
__device__ inline float wave_sum_f(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// DPP lane moves (VOP_DPP, folded into the consuming v_add by the compiler):
// quad_perm xor 1 / xor 2 within quads, row_half_mirror (l ^ 7 within 8
// lanes) and row_mirror (l ^ 15 within a 16-lane row).  No LDS traffic,
// unlike __shfl_xor (ds_bpermute_b32).
enum : int { kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppRowMirror = 0x140, kDppRowHalfMirror = 0x141 };
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// a_l + a_{l ^ 16} and a_l + a_{l ^ 32} through gfx950's permlane swaps
__device__ __forceinline__ float add_lane_xor16(float a) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(a), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float add_lane_xor32(float a) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(a), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// OR over the 64 lanes of a wave, result in every lane; VALU only (as wave_sum_dpp)
__device__ __forceinline__ uint32_t wave_or_dpp(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppRowMirror, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppRowHalfMirror, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppXor2, 0xF, 0xF, false);
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppXor1, 0xF, 0xF, false);
    auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = r[0] | r[1];
    r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return r[0] | r[1];
}

// Sum over the 64 lanes of a wave, result in every lane; VALU only.  Within
// a 16-lane row the partners are l^15, l^7 (mirrors: each stage pairs the two
// halves of a group bijectively, so each lane is counted once), then l^2, l^1.
__device__ __forceinline__ float wave_sum_dpp(float v) {
    v += dpp_mov<kDppRowMirror>(v);
    v += dpp_mov<kDppRowHalfMirror>(v);
    v += dpp_mov<kDppXor2>(v);
    v += dpp_mov<kDppXor1>(v);
    return add_lane_xor32(add_lane_xor16(v));
}

// Transposed butterfly reduction of 16 per-lane values over the 64 lanes of
// a wave.  Stage 1/2 use gfx950's v_permlane32_swap / v_permlane16_swap (one
// swap moves half of a pair across the 32- or 16-lane boundary, so each stage
// halves the number of live values); stages 3/4 pair the halves of 16- and
// 8-lane groups with DPP mirrors (keep/send select: field bit 1 <- lane bit 3,
// field bit 0 <- lane bit 2); the last two stages are DPP quad adds.  On
// return lane l (all four lanes of each quad) holds the full wave sum of field
// (l >> 2); every cross-lane move is a VALU op.
__device__ inline float wave_transpose_reduce16(const float (&v)[16]) {
    const int lane = threadIdx.x & 63;
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 8]), false, false);
        a[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    // lanes 0..31 hold fields 0..7, lanes 32..63 fields 8..15 (sums over l, l^32)
    float b[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[i]), __float_as_uint(a[i + 4]), false, false);
        b[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    // field bit 1 <- lane bit 3 (partner l ^ 15: opposite bit 3, same row)
    const bool hi8 = (lane & 8) != 0;
    float c[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const float keep = hi8 ? b[i + 2] : b[i];
        const float send = hi8 ? b[i] : b[i + 2];
        c[i] = keep + dpp_mov<kDppRowMirror>(send);
    }
    // field bit 0 <- lane bit 2 (partner l ^ 7: opposite bit 2, same 8 lanes)
    const bool hi4 = (lane & 4) != 0;
    const float keep = hi4 ? c[1] : c[0];
    const float send = hi4 ? c[0] : c[1];
    float d = keep + dpp_mov<kDppRowHalfMirror>(send);
    d += dpp_mov<kDppXor2>(d);
    d += dpp_mov<kDppXor1>(d);
    return d;
}

// XCD-aware tile order: blocks are dealt round-robin over the 8 XCDs, so map
// the blocks one XCD receives onto a contiguous run of tiles (rows of tiles
// that share Gaussians then share that XCD's L2).  Bijective for any count.
__device__ inline uint32_t xcd_remap(uint32_t b, uint32_t n) {
    const uint32_t q = n / 8, r = n % 8, xcd = b % 8, local = b / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// The tile of a 256-point chunk: the last t in [0, n) with off[t] <= chunk
// (off non-decreasing, off[0] = 0), searched 64-wide — each lane tests one of
// 64 evenly spaced candidates and the ballot narrows the span 64-fold — so
// 8160 tiles take 3 dependent loads, against 13 for a binary search (the
// chain sat in front of every SAMPLE workgroup's first batch).  Call with
// every lane of the wave active; the result is wave-uniform.
__device__ inline uint32_t wave_find_chunk_tile(const uint32_t* __restrict__ off, uint32_t n, uint32_t chunk) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t lo = 0, span = n;
    while (span > 1) {
        const uint32_t step = (span + 63u) >> 6;
        const uint32_t t = lo + lane * step;
        const bool ok = lane == 0u || (t < lo + span && off[t] <= chunk);
        const unsigned long long b = __ballot(ok);
        const uint32_t L = 63u - (uint32_t)__builtin_clzll(b);
        const uint32_t end = lo + span;
        lo += L * step;
        span = min(step, end - lo);
    }
    return __builtin_amdgcn_readfirstlane(lo);
}

// Division as the reference compiles it: CR is built with --use_fast_math
// (DGR/setup.py), where a / b is the approximate div.approx.f32, i.e.
// a * rcp(b).  Here: v_rcp_f32 (1 ulp) and one multiply, instead of the
// ~10-instruction IEEE division sequence.  Used in the per-(pixel, splat)
// backward loops; per-Gaussian code keeps IEEE division (its integer
// outputs are checked bit-exactly against the oracle).
__device__ __forceinline__ float fast_rcp(float b) { return __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ float fast_div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }

// Length of the ray (pnx, pny, 1) through pixel (px, py): the median depth
// is stored divided by it (render_forward.cu:651-653) and multiplied back in
// the backward (render_backward.cu:813-816); one rounding sequence for both.
__device__ __forceinline__ float pixel_ray_norm(float px, float py, int W, int H, float fx, float fy) {
#pragma clang fp contract(off)
    const float pnx = (px - (float)(W - 1) / 2.f) / fx;
    const float pny = (py - (float)(H - 1) / 2.f) / fy;
    return sqrtf(pnx * pnx + pny * pny + 1.f);
}

// Footprint of a splat record at a pixel offset (dx, dy) = (mean - pixel):
//   power  = -0.5 (a dx^2 + c dy^2) - b dx dy   (render_forward.cu:486-487)
//   t_peak = plane.x dx + plane.y dy + |t|      (render_forward.cu:513, 603)
// Every rounding is spelled out (explicit fma, contraction off) so the
// composite, the median-depth bisection and the backward — compiled in
// different contexts — agree bit for bit on alpha and on which
// (pixel, splat) pairs contribute.
__device__ __forceinline__ float splat_power(const float4& w0, const float4& w1, float dx, float dy) {
#pragma clang fp contract(off)
    const float q = __builtin_fmaf(w1.x * dy, dy, (w0.z * dx) * dx);
    return __builtin_fmaf(-0.5f, q, -((w0.w * dx) * dy));
}
__device__ __forceinline__ float splat_tpeak(const float4& w1, const float4& w2, float dx, float dy) {
#pragma clang fp contract(off)
    return __builtin_fmaf(w1.w, dy, w1.z * dx) + w2.x;
}

// The same for two pixels of one column (shared dx, dy in the halves of a
// packed register): the packed operations round exactly as the scalar ones.
typedef float pf32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pf32x2 splat_power2(const float4& w0, const float4& w1, float dx, pf32x2 dy) {
#pragma clang fp contract(off)
    const float ax = (w0.z * dx) * dx;
    const pf32x2 q = __builtin_elementwise_fma(pf32x2{w1.x, w1.x} * dy, dy, pf32x2{ax, ax});
    const float bx = w0.w * dx;
    return __builtin_elementwise_fma(pf32x2{-0.5f, -0.5f}, q, -(pf32x2{bx, bx} * dy));
}
__device__ __forceinline__ pf32x2 splat_tpeak2(const float4& w1, const float4& w2, float dx, pf32x2 dy) {
#pragma clang fp contract(off)
    const float cx = w1.z * dx;
    return __builtin_elementwise_fma(pf32x2{w1.w, w1.w}, dy, pf32x2{cx, cx}) + pf32x2{w2.x, w2.x};
}

}  // namespace gsr
