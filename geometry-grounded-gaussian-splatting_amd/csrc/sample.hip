// sample.hip — sample_depth on gfx950: the median depth of the Gaussian
// field at arbitrary 3D points (the multi-view geometric-consistency term of
// the reference's training loss, utils/loss_utils.py:160), and its backward.
//
// Replaces, in CR/rasterizer_impl.cu:1042-1394 (Rasterizer::sampleDepth /
// sampleDepthBackward): preprocessPointsCUDA (sample_forward.cu:9-53),
// createWithKeys + SortPairs + identifyTileRanges on the points (:109-137,
// 745-779), countPointBatches + InclusiveSum + setBlockId (:163-183,
// 781-790), sampleDepthCUDA backward (sample_backward.cu:77-359) and
// preprocessPointsCUDA backward (:42-75).  The forward raster itself is
// render_fwd.hip in SAMPLE mode; the Gaussian side reuses preprocess_fwd,
// the binning and preprocess_bwd.
//
// Points are grouped per tile and cut into chunks of 256 points, one 256-lane workgroup each
// (the reference uses 512-point blocks, 2 points per thread: a point's result
// does not depend on the grouping, every point stops at its own last
// contributor).  No host synchronisation besides the forward's one: the
// chunk count is derived on the device (sample_setup_kernel) and read
// together with K.
// The grouping (round 5, GSR_POINT_SCATTER): the reference sorts the points
// by tile id (SortPairs, stable).  No result depends on the order of a tile's
// points, so they are scattered instead: the per-tile counts the points
// kernel already takes are scanned into the tile ranges (sample_setup) and
// each wave reserves a run of its tile's range with one atomic per distinct
// tile (sample_scatter_kernel) — one pass over 4 B per point instead of the
// radix sort's histogram and two onesweep passes (62 + 16 us for 2.07M points
// at the e2e scene).  Within a wave the points keep their order.
#pragma clang fp contract(off)

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "gsr_kernels.h"

namespace gsr {

#ifndef GSR_POINT_SCATTER
#define GSR_POINT_SCATTER 1  // 0: the reference's stable sort by tile id (rocprim radix sort)
#endif
using PointSortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                   rocprim::default_config, 0>;

// bits to hold 0..tiles (culled points carry key = tiles and sort last).
// (A (tile, Morton cell) key that makes each wave's points spatially compact
// was measured: no gain at the benchmark scale, one more sort pass.)
static unsigned point_key_bits(uint32_t tiles) { return 32u - (unsigned)__builtin_clz(tiles | 1u); }

size_t point_sort_temp_bytes(int PN, uint32_t tiles) {
    size_t bytes = 0;
    if (GSR_POINT_SCATTER) return 0;
    (void)rocprim::radix_sort_pairs<PointSortConfig>(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                     rocprim::counting_iterator<uint32_t>(0), (uint32_t*)nullptr,
                                                     (size_t)PN, 0u, point_key_bits(tiles));
    return bytes;
}

// ndc2Pix in double, as the reference (auxiliary.h:38-40)
__device__ inline float ndc2pix_d(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

// preprocessPointsCUDA (sample_forward.cu:9-53) + the point's tile
// (createWithKeys, rasterizer_impl.cu:127-131) + per-tile counts.
__global__ void __launch_bounds__(256)
    sample_points_kernel(int PN, const float* __restrict__ pts, const float* __restrict__ V,
                         const float* __restrict__ M, int W, int H, uint32_t gx, uint32_t gy,
                         float2* __restrict__ xy_out, float* __restrict__ t_out, uint32_t* __restrict__ keys,
                         uint32_t* __restrict__ counts) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= PN) return;
    const uint32_t tiles = gx * gy;
    keys[idx] = tiles;
    const float x = pts[3 * idx], y = pts[3 * idx + 1], z = pts[3 * idx + 2];
    const float vz = V[2] * x + V[6] * y + V[10] * z + V[14];
    if (vz <= kNearPlane) return;  // in_frustum (auxiliary.h:133-153)
    const float vx = V[0] * x + V[4] * y + V[8] * z + V[12];
    const float vy = V[1] * x + V[5] * y + V[9] * z + V[13];
    const float hx = M[0] * x + M[4] * y + M[8] * z + M[12];
    const float hy = M[1] * x + M[5] * y + M[9] * z + M[13];
    const float hw = M[3] * x + M[7] * y + M[11] * z + M[15];
    const float p_w = 1.0f / (hw + 0.0000001f);
    const float px = ndc2pix_d(hx * p_w, W), py = ndc2pix_d(hy * p_w, H);
    if (px < 0 || px > W - 1 || py < 0 || py > H - 1) return;
    xy_out[idx] = make_float2(px, py);
    t_out[idx] = sqrtf(vx * vx + vy * vy + vz * vz);  // norm3df(p_view), sample_forward.cu:50
    const uint32_t tx = (uint32_t)min((int)gx - 1, max(0, (int)((px + 0.5f) / kTile)));
    const uint32_t ty = (uint32_t)min((int)gy - 1, max(0, (int)((py + 0.5f) / kTile)));
    const uint32_t t = ty * gx + tx;
    keys[idx] = t;
    // neighbouring points mostly share a tile: one atomic per distinct tile of the wave
    bool pending = true;
    while (pending) {
        const uint32_t lead = __builtin_amdgcn_readfirstlane(t);
        const unsigned long long same = __ballot(t == lead);
        if (t == lead) {
            pending = false;
            if ((threadIdx.x & 63) == (unsigned)__builtin_ctzll(same)) atomicAdd(&counts[t], (uint32_t)__popcll(same));
        }
    }
}

hipError_t launch_sample_points(const FwdParams& p, int PN, const float* points3D, const PointState& ps,
                                const PointBinState& pb, const SampleTiles& st, hipStream_t stream) {
    const uint32_t tiles = p.grid_x * p.grid_y;
    hipError_t e = hipMemsetAsync(st.counts, 0, sizeof(uint32_t) * tiles, stream);
    if (e != hipSuccess || PN == 0) return e;
    hipLaunchKernelGGL(sample_points_kernel, dim3((PN + 255) / 256), dim3(256), 0, stream, PN, points3D, p.view,
                       p.proj, p.W, p.H, p.grid_x, p.grid_y, ps.xy, ps.t, pb.keys_unsorted, st.counts);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (GSR_POINT_SCATTER) return hipSuccess;  // (sample_scatter_kernel, after the setup's scan)
    size_t bytes = pb.sort_tmp_bytes;
    return rocprim::radix_sort_pairs<PointSortConfig>(pb.sort_tmp, bytes, pb.keys_unsorted, pb.keys,
                                                      rocprim::counting_iterator<uint32_t>(0), pb.pt_list,
                                                      (size_t)PN, 0u, point_key_bits(tiles), stream);
}

// Block-wide exclusive scan of three counters (1024 lanes = 16 waves).
struct Scan3 {
    uint32_t a, b, c;
};
__device__ inline Scan3 block_exclusive_scan3(Scan3 v, Scan3* s_wave, Scan3& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Scan3 inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t ua = __shfl_up(inc.a, o, 64), ub = __shfl_up(inc.b, o, 64), uc = __shfl_up(inc.c, o, 64);
        if (lane >= o) {
            inc.a += ua;
            inc.b += ub;
            inc.c += uc;
        }
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    Scan3 base{0, 0, 0};
    total = Scan3{0, 0, 0};
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) {
        const Scan3 t = s_wave[w];
        if (w < wave) {
            base.a += t.a;
            base.b += t.b;
            base.c += t.c;
        }
        total.a += t.a;
        total.b += t.b;
        total.c += t.c;
    }
    __syncthreads();
    return Scan3{base.a + inc.a - v.a, base.b + inc.b - v.b, base.c + inc.c - v.c};
}

// countPointBatches + InclusiveSum + the point ranges: per tile, its points
// [first, end) in pt_list, its first 256-point chunk, and the totals
// (valid points, the reference's 512-point block count, chunks).
__global__ void __launch_bounds__(1024)
    sample_setup_kernel(uint32_t tiles, const uint32_t* __restrict__ counts, uint2* __restrict__ pt_ranges,
                        uint32_t* __restrict__ chunk_off, uint32_t* __restrict__ totals) {
    __shared__ Scan3 s_wave[16];
    Scan3 carry{0, 0, 0};
    for (uint32_t base = 0; base < tiles; base += blockDim.x) {
        const uint32_t t = base + threadIdx.x;
        const uint32_t n = t < tiles ? counts[t] : 0u;
        Scan3 tot;
        const Scan3 ex = block_exclusive_scan3(Scan3{n, (n + kTilePixels - 1) / kTilePixels, (n + 511u) / 512u},
                                               s_wave, tot);
        if (t < tiles) {
            const uint32_t first = carry.a + ex.a;
            pt_ranges[t] = make_uint2(first, first + n);
            chunk_off[t] = carry.b + ex.b;
        }
        carry.a += tot.a;
        carry.b += tot.b;
        carry.c += tot.c;
    }
    if (threadIdx.x == 0) {
        chunk_off[tiles] = carry.b;
        totals[0] = carry.a;
        totals[1] = carry.c;
        totals[2] = carry.b;
        totals[3] = 0u;
    }
}

// Each point into its tile's range (GSR_POINT_SCATTER): a wave takes one run of
// slots per distinct tile among its lanes from the end of that tile's range
// (counts[t] counts down to 0), its lanes in lane order within the run.
__global__ void __launch_bounds__(256)
    sample_scatter_kernel(int PN, uint32_t tiles, const uint32_t* __restrict__ keys, uint32_t* __restrict__ counts,
                          const uint2* __restrict__ pt_ranges, uint32_t* __restrict__ pt_list) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t t = idx < PN ? keys[idx] : tiles;
    const uint32_t lane = threadIdx.x & 63;
    bool pending = t < tiles;  // (culled points carry t = tiles: in no range)
    for (unsigned long long pm = __ballot(pending); pm != 0ull; pm = __ballot(pending)) {
        // (every lane stays in the loop: the leader is the first still-pending lane, read by lane index)
        const uint32_t lead = (uint32_t)__builtin_amdgcn_readlane((int)t, __builtin_ctzll(pm));
        const unsigned long long same = __ballot(pending && t == lead);
        uint32_t base = 0u;
        if (lane == (uint32_t)__builtin_ctzll(same)) base = atomicSub(&counts[lead], (uint32_t)__popcll(same));
        // (the leader's lane id is wave-uniform, so the run's base is a lane read)
        base = __shfl(base, __builtin_ctzll(same), 64);
        if (pending && t == lead) {
            const uint32_t rank = (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
            pt_list[pt_ranges[t].x + base - (uint32_t)__popcll(same) + rank] = (uint32_t)idx;
            pending = false;
        }
    }
}

hipError_t launch_sample_setup(int PN, uint32_t tiles, const PointBinState& pb, const SampleTiles& st,
                               hipStream_t stream) {
    hipLaunchKernelGGL(sample_setup_kernel, dim3(1), dim3(1024), 0, stream, tiles, st.counts, st.pt_ranges,
                       st.chunk_off, st.totals);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !GSR_POINT_SCATTER || PN == 0) return e;
    hipLaunchKernelGGL(sample_scatter_kernel, dim3((PN + 255) / 256), dim3(256), 0, stream, PN, tiles,
                       pb.keys_unsorted, st.counts, st.pt_ranges, pb.pt_list);
    return hipGetLastError();
}

// ------------------------------------------------------------------ backward
#ifndef GSR_SAMPLE_BWD_PAIRS
#define GSR_SAMPLE_BWD_PAIRS 1
#endif
struct SampleBwdArgs {
    const uint2* ranges;
    const uint32_t* point_list;
    const Splat* splats;
    const uint32_t* chunk_off;
    const uint2* pt_ranges;
    const uint32_t* pt_list;
    const uint32_t* totals;
    const uint32_t* chunk_max;
    const float2* pt_xy;
    const uint32_t* pt_last;
    const float* pt_mdepth;
    const float* pt_dT;
    const uint8_t* pt_cached;
    const float* points3D;
    const uint8_t* inside;
    const float* dL_doutput;
    float* dL_dpoints3D;
    const float* proj;
    int W, H;
    uint32_t num_tiles;
    float focal_x, focal_y;
    float* acc;  // [P][16] (gsr_common.h AccField): mean2D, conic, ray-plane
    const uint32_t* chunk_order;  // launch order of the chunks (heaviest first) or null
};

// sampleDepthCUDA backward (sample_backward.cu:77-359), one 256-lane
// workgroup per chunk, one point per lane.  Per (wave, Gaussian) the 10
// gradient terms are summed by the wave transpose reduction of render_bwd
// (wave_transpose_reduce16) and added with one atomic instruction into the
// Gaussian's accumulator record; the point's own gradient (through its
// projected position) stays in registers, and the projection backward of
// the point (preprocessPointsCUDA bwd, sample_backward.cu:42-75) is fused at
// the end.  The grid is an upper bound on the chunk count (read on the
// device); surplus workgroups exit at once.
__global__ void __launch_bounds__(256) sample_bwd_kernel(SampleBwdArgs a) {
    __shared__ float4 s_w0[kTilePixels], s_w1[kTilePixels], s_w2[kTilePixels];
    __shared__ uint32_t s_id[kTilePixels];

    if (blockIdx.x >= a.totals[2]) return;  // uniform over the block
    const uint32_t chunk = a.chunk_order ? a.chunk_order[blockIdx.x] : xcd_remap(blockIdx.x, a.totals[2]);
    const int tid = threadIdx.x, lane = tid & 63;
    const uint32_t tile = wave_find_chunk_tile(a.chunk_off, a.num_tiles, chunk);
    const uint2 range = a.ranges[tile];
    const int max_contrib = (int)a.chunk_max[chunk];
    const uint2 pr = a.pt_ranges[tile];
    const uint32_t slot = pr.x + (chunk - a.chunk_off[tile]) * kTilePixels + tid;
    const bool in = slot < pr.y;
    const uint32_t pid = in ? a.pt_list[slot] : 0u;

    // per-point seed (sample_backward.cu:138-158)
    float pixx = 0.f, pixy = 0.f, mDepth = 0.f, dL_dDepth = 0.f, dpx = 0.f, dpy = 0.f, dT = 0.f;
    uint32_t last = 0;
    bool on = false, cached = false;
    if (in) {
        const float2 xy = a.pt_xy[pid];
        pixx = xy.x;
        pixy = xy.y;
        last = a.pt_last[pid];
        mDepth = a.pt_mdepth[pid];
        const bool in_r = a.inside[pid] != 0;
        const float g0 = a.dL_doutput[3 * pid], g1 = a.dL_doutput[3 * pid + 1], g2 = a.dL_doutput[3 * pid + 2];
        const float pnx = (pixx - (float)(a.W - 1) / 2.f) / a.focal_x;
        const float pny = (pixy - (float)(a.H - 1) / 2.f) / a.focal_y;
        const float rln = 1.0f / sqrtf(pnx * pnx + pny * pny + 1.f);
        const float rln2 = 1.f / (pnx * pnx + pny * pny + 1.f);
        const float depth = mDepth * rln;
        const float dL_ddepth = g0 * pnx + g1 * pny + g2;
        dL_dDepth = rln * dL_ddepth;
        const float aux = dL_ddepth * rln2;
        dpx = (g0 - aux * pnx) * depth / a.focal_x;
        dpy = (g1 - aux * pny) * depth / a.focal_y;
        on = last != 0 && in_r;
        cached = a.pt_cached[pid] != 0;
        dT = cached ? a.pt_dT[pid] : 0.f;
    }
    const int rounds = (max_contrib + kTilePixels - 1) / kTilePixels;
    auto stage = [&](int i, bool ids) {
        const int c = i * kTilePixels + tid;
        if (c < max_contrib) {
            const uint32_t g = a.point_list[range.x + c];
            const Splat* sp = a.splats + g;
            s_w0[tid] = sp->w0;
            s_w1[tid] = sp->w1;
            s_w2[tid] = sp->w2;
            if (ids) s_id[tid] = g;
        }
    };

    // pre-pass dT/dt_m (sample_backward.cu:170-215) unless the forward cached it
    {
        const bool need = on && !cached;
        const uint32_t wave_last = wave_max_u(need ? last : 0u);
        const bool block_needs = __syncthreads_or(wave_last != 0u);
        uint32_t c = 0;
        int toDo = max_contrib;
        for (int i = 0; block_needs && i < rounds; i++, toDo -= kTilePixels) {
            __syncthreads();
            stage(i, false);
            __syncthreads();
            const int n = min(kTilePixels, toDo);
            for (int j = 0; j < n && c < wave_last; j++) {
                c++;
                const float4 w0 = s_w0[j], w1 = s_w1[j];
                const float dx = w0.x - pixx, dy = w0.y - pixy;
                const float power = splat_power(w0, w1, dx, dy);
                const float alpha = fminf(0.99f, w1.y * __expf(power));
                if (!(need && c <= last && !(power > 0.f) && !(alpha < 1.0f / 255.0f))) continue;
                const float4 w2 = s_w2[j];
                const float t_peak = splat_tpeak(w1, w2, dx, dy);
                const float t_delta = (mDepth - t_peak) * w2.y;
                const float Gt = alpha * __expf(-0.5f * t_delta * t_delta);
                dT += fast_div(-0.25f * Gt, 1.f - Gt) * fabsf(t_delta) * w2.y;
            }
        }
    }
    const float kappa = on ? dL_dDepth / fmaxf(-dT, 1e-7f) : 0.f;
    // contributors past the wave's last are invalid for every lane of it
    const uint32_t wave_last = wave_max_u(on ? last : 0u);

    // main pass, front to back (sample_backward.cu:228-354)
    const float ddelx_dx = 0.5f * a.W, ddely_dy = 0.5f * a.H;
    uint32_t contributor = 0;
    int toDo = max_contrib;
    for (int i = 0; i < rounds; i++, toDo -= kTilePixels) {
        __syncthreads();
        stage(i, true);
        __syncthreads();
        const int n = min(kTilePixels, toDo);
        for (int j = 0; j < n && contributor < wave_last; j++) {
            contributor++;
            const float4 w0 = s_w0[j], w1 = s_w1[j];
            const float dx = w0.x - pixx, dy = w0.y - pixy;
            const float power = splat_power(w0, w1, dx, dy);
            const float G = __expf(power);
            const bool valid = on && contributor <= last && !(power > 0.f) && !(w1.y * G < 1.0f / 255.0f);
            if (__ballot(valid) == 0ull) continue;  // wave-uniform skip (warp.any)
            const float4 w2 = s_w2[j];
            const float alpha = fminf(0.99f, w1.y * G);
            const float t_peak = splat_tpeak(w1, w2, dx, dy);
            const float rsig = w2.y;
            const float t_delta = (mDepth - t_peak) * rsig;
            const float G_exp = __expf(-0.5f * t_delta * t_delta);
            const float Gt = alpha * G_exp;
            float dL_dGt = kappa * 0.25f * fast_rcp(1.f - Gt);
            dL_dGt = mDepth > t_peak ? dL_dGt : -dL_dGt;
            dL_dGt = rsig > 0.f ? dL_dGt : 0.f;
            const float dL_dopa = dL_dGt * G_exp - kappa * (t_delta > 0.f ? 0.5f * fast_rcp(1.f - alpha) : 0.f);
            const float dL_ddelta = -dL_dGt * Gt * t_delta;
            const float dL_drsig = dL_ddelta * (mDepth - t_peak);
            const float dL_dt = -dL_ddelta * rsig;
            const float dL_dG = w1.y * dL_dopa;
            const float gdx = G * dx, gdy = G * dy;
            const float dG_ddelx = -gdx * w0.z - gdy * w0.w;
            const float dG_ddely = -gdy * w1.x - gdx * w0.w;
            float dL_ddelx = dL_dG * dG_ddelx + dL_dt * w1.z;
            float dL_ddely = dL_dG * dG_ddely + dL_dt * w1.w;
            float f[16];
#pragma unroll
            for (int q = 0; q < 16; q++) f[q] = 0.f;
            if (valid) {
                dpx -= dL_ddelx;
                dpy -= dL_ddely;
                f[kAccMean2D + 0] = dL_ddelx * ddelx_dx;
                f[kAccMean2D + 1] = dL_ddely * ddely_dy;
                f[kAccConic + 0] = -0.5f * gdx * dx * dL_dG;
                f[kAccConic + 1] = -0.5f * gdx * dy * dL_dG;
                f[kAccConic + 2] = -0.5f * gdy * dy * dL_dG;
                f[kAccConic + 3] = G * dL_dopa;
                f[kAccPlane + 0] = dL_dt * dx;
                f[kAccPlane + 1] = dL_dt * dy;
                f[kAccPlane + 2] = dL_dt;
                f[kAccPlane + 3] = dL_drsig;
            }
            const float red = wave_transpose_reduce16(f);
            // lanes 4k hold field k; colour (0-2) and normal (9-11) are zero here
            const int field = lane >> 2;
            const bool field_lane = (lane & 3) == 0 && field >= kAccMean2D &&
                                    (field < kAccNormal || field >= kAccPlane);
            if (field_lane) atomicAdd(a.acc + (size_t)s_id[j] * kAccFields + field, red);
        }
    }
    if (in) {
        // dL/dpoints2D in NDC units, then the projection backward
        // (preprocessPointsCUDA bwd, sample_backward.cu:42-75)
        const float gx2 = dpx * ddelx_dx, gy2 = dpy * ddely_dy;
        const float* Pm = a.proj;
        const float mx = a.points3D[3 * pid], my = a.points3D[3 * pid + 1], mz = a.points3D[3 * pid + 2];
        const float hw = Pm[3] * mx + Pm[7] * my + Pm[11] * mz + Pm[15];
        const float m_w = 1.0f / (hw + 0.0000001f);
        const float mul1 = (Pm[0] * mx + Pm[4] * my + Pm[8] * mz + Pm[12]) * m_w * m_w;
        const float mul2 = (Pm[1] * mx + Pm[5] * my + Pm[9] * mz + Pm[13]) * m_w * m_w;
        a.dL_dpoints3D[3 * pid + 0] = (Pm[0] * m_w - Pm[3] * mul1) * gx2 + (Pm[1] * m_w - Pm[3] * mul2) * gy2;
        a.dL_dpoints3D[3 * pid + 1] = (Pm[4] * m_w - Pm[7] * mul1) * gx2 + (Pm[5] * m_w - Pm[7] * mul2) * gy2;
        a.dL_dpoints3D[3 * pid + 2] = (Pm[8] * m_w - Pm[11] * mul1) * gx2 + (Pm[9] * m_w - Pm[11] * mul2) * gy2;
    }
}

// The same with 2 NPR points per lane (GSR_SAMPLE_BWD_PAIRS): a workgroup of
// 128 / NPR lanes per 256-point chunk, the lane's points in NPR packed pairs
// (pair k: points lane + 2k L and lane + (2k + 1) L, L the lane count).  Per
// (wave, Gaussian) step the record reads, the skip ballot, the transpose
// reduction and the atomic serve 2 NPR points per lane instead of one, and
// the per-point arithmetic runs as v_pk_* pairs; every packed operation
// rounds as the scalar one, so alpha and the contribute decisions stay
// bit-identical to the forward's.  NPR = 2 (round 5): one wave per chunk, as
// render_bwd's one wave per tile.
typedef float sf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ sf2 ssplat(float v) { return sf2{v, v}; }
__device__ __forceinline__ sf2 ssel(bool ca, bool cb, sf2 x, sf2 y) { return sf2{ca ? x.x : y.x, cb ? x.y : y.y}; }

#ifndef GSR_SAMPLE_BWD_NPR
#define GSR_SAMPLE_BWD_NPR 2
#endif

template <int NPR>
__global__ void __launch_bounds__(kTilePixels / (2 * NPR)) sample_bwd_pairs_kernel(SampleBwdArgs a) {
    constexpr int L = kTilePixels / (2 * NPR);  // lanes
    constexpr int NQ = 2 * NPR;                 // points per lane
    constexpr int B = kTilePixels / NPR;        // records per LDS batch (2 per lane; NPR = 2: 6.5 KB, 6 waves per SIMD)
    constexpr int RL = B / L;
    __shared__ float4 s_w0[B], s_w1[B], s_w2[B];
    __shared__ uint32_t s_id[B];

    if (blockIdx.x >= a.totals[2]) return;  // uniform over the block
    const uint32_t chunk = a.chunk_order ? a.chunk_order[blockIdx.x] : xcd_remap(blockIdx.x, a.totals[2]);
    const int tid = threadIdx.x, lane = tid & 63;
    const uint32_t tile = wave_find_chunk_tile(a.chunk_off, a.num_tiles, chunk);
    const uint2 range = a.ranges[tile];
    const int max_contrib = (int)a.chunk_max[chunk];
    const uint2 pr = a.pt_ranges[tile];
    const uint32_t base = pr.x + (chunk - a.chunk_off[tile]) * kTilePixels + tid;

    // per-point seed (sample_backward.cu:138-158), point q at slot base + q L
    float px[NQ], py[NQ], md[NQ], dLD[NQ], dT[NQ], gpx[NQ], gpy[NQ];
    uint32_t last[NQ], pid[NQ];
    bool in[NQ], on[NQ], cached[NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) {
        px[q] = py[q] = md[q] = dLD[q] = dT[q] = gpx[q] = gpy[q] = 0.f;
        last[q] = pid[q] = 0u;
        on[q] = cached[q] = false;
        const uint32_t slot = base + q * L;
        in[q] = slot < pr.y;
        if (!in[q]) continue;
        pid[q] = a.pt_list[slot];
        const uint32_t id = pid[q];
        const float2 xy = a.pt_xy[id];
        px[q] = xy.x;
        py[q] = xy.y;
        last[q] = a.pt_last[id];
        md[q] = a.pt_mdepth[id];
        const bool in_r = a.inside[id] != 0;
        const float g0 = a.dL_doutput[3 * id], g1 = a.dL_doutput[3 * id + 1], g2 = a.dL_doutput[3 * id + 2];
        const float pnx = (px[q] - (float)(a.W - 1) / 2.f) / a.focal_x;
        const float pny = (py[q] - (float)(a.H - 1) / 2.f) / a.focal_y;
        const float rln = 1.0f / sqrtf(pnx * pnx + pny * pny + 1.f);
        const float rln2 = 1.f / (pnx * pnx + pny * pny + 1.f);
        const float depth = md[q] * rln;
        const float dL_ddepth = g0 * pnx + g1 * pny + g2;
        dLD[q] = rln * dL_ddepth;
        const float aux = dL_ddepth * rln2;
        gpx[q] = (g0 - aux * pnx) * depth / a.focal_x;
        gpy[q] = (g1 - aux * pny) * depth / a.focal_y;
        on[q] = last[q] != 0 && in_r;
        cached[q] = a.pt_cached[id] != 0;
        dT[q] = cached[q] ? a.pt_dT[id] : 0.f;
    }
    const int rounds = (max_contrib + B - 1) / B;
    // every list entry, then every record, requested before any is stored
    auto stage = [&](int i, bool ids) {
        uint32_t g[RL];
        float4 r[RL][3];
#pragma unroll
        for (int h = 0; h < RL; h++) {
            const int c = i * B + tid + h * L;
            g[h] = c < max_contrib ? a.point_list[range.x + c] : 0u;
        }
#pragma unroll
        for (int h = 0; h < RL; h++) {
            const int c = i * B + tid + h * L;
            const Splat* sp = a.splats + g[h];
            const bool ok = c < max_contrib;
            r[h][0] = ok ? sp->w0 : make_float4(0.f, 0.f, 0.f, 0.f);
            r[h][1] = ok ? sp->w1 : make_float4(0.f, 0.f, 0.f, 0.f);
            r[h][2] = ok ? sp->w2 : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int h = 0; h < RL; h++) {
            const int k = tid + h * L;
            if (i * B + k < max_contrib) {
                s_w0[k] = r[h][0];
                s_w1[k] = r[h][1];
                s_w2[k] = r[h][2];
                if (ids) s_id[k] = g[h];
            }
        }
    };

    // pre-pass dT/dt_m (sample_backward.cu:170-215) for points the forward did not cache
    {
        bool need[NQ];
        uint32_t mine = 0u;
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            need[q] = on[q] && !cached[q];
            mine = max(mine, need[q] ? last[q] : 0u);
        }
        const uint32_t wave_last = wave_max_u(mine);
        const bool block_needs = __syncthreads_or(wave_last != 0u);
        uint32_t c = 0;
        int toDo = max_contrib;
        for (int i = 0; block_needs && i < rounds; i++, toDo -= B) {
            __syncthreads();
            stage(i, false);
            __syncthreads();
            const int n = min(B, toDo);
            for (int j = 0; j < n && c < wave_last; j++) {
                c++;
                const float4 w0 = s_w0[j], w1 = s_w1[j], w2 = s_w2[j];
#pragma unroll
                for (int q = 0; q < NQ; q++) {
                    const float dx = w0.x - px[q], dy = w0.y - py[q];
                    const float power = splat_power(w0, w1, dx, dy);
                    const float alpha = fminf(0.99f, w1.y * __expf(power));
                    if (!(need[q] && c <= last[q] && !(power > 0.f) && !(alpha < 1.0f / 255.0f))) continue;
                    const float t_peak = splat_tpeak(w1, w2, dx, dy);
                    const float t_delta = (md[q] - t_peak) * w2.y;
                    const float Gt = alpha * __expf(-0.5f * t_delta * t_delta);
                    dT[q] += fast_div(-0.25f * Gt, 1.f - Gt) * fabsf(t_delta) * w2.y;
                }
            }
        }
    }
    sf2 kappa[NPR], pixx[NPR], pixy[NPR], mDepth[NPR], dpx[NPR], dpy[NPR];
    uint32_t mine = 0u;
#pragma unroll
    for (int k = 0; k < NPR; k++) {
        const int q0 = 2 * k, q1 = 2 * k + 1;
        kappa[k] = {on[q0] ? dLD[q0] / fmaxf(-dT[q0], 1e-7f) : 0.f, on[q1] ? dLD[q1] / fmaxf(-dT[q1], 1e-7f) : 0.f};
        pixx[k] = {px[q0], px[q1]};
        pixy[k] = {py[q0], py[q1]};
        mDepth[k] = {md[q0], md[q1]};
        dpx[k] = {gpx[q0], gpx[q1]};
        dpy[k] = {gpy[q0], gpy[q1]};
        mine = max(mine, max(on[q0] ? last[q0] : 0u, on[q1] ? last[q1] : 0u));
    }
    const uint32_t wave_last = wave_max_u(mine);

    // main pass, front to back (sample_backward.cu:228-354)
    const float ddelx_dx = 0.5f * a.W, ddely_dy = 0.5f * a.H;
    constexpr float kLog2e = 1.44269504088896340736f;
    uint32_t contributor = 0;
    int toDo = max_contrib;
    for (int i = 0; i < rounds; i++, toDo -= B) {
        __syncthreads();
        stage(i, true);
        __syncthreads();
        const int n = min(B, toDo);
        for (int j = 0; j < n && contributor < wave_last; j++) {
            contributor++;
            const float4 w0 = s_w0[j], w1 = s_w1[j];
            sf2 dx[NPR], dy[NPR], G[NPR], og[NPR];
            bool va[NPR], vb[NPR];
            bool any = false;
#pragma unroll
            for (int k = 0; k < NPR; k++) {
                dx[k] = ssplat(w0.x) - pixx[k];
                dy[k] = ssplat(w0.y) - pixy[k];
                sf2 power;
                {
#pragma clang fp contract(off)
                    const sf2 ax = (ssplat(w0.z) * dx[k]) * dx[k];  // splat_power, per half
                    const sf2 qq = __builtin_elementwise_fma(ssplat(w1.x) * dy[k], dy[k], ax);
                    power = __builtin_elementwise_fma(ssplat(-0.5f), qq, -((ssplat(w0.w) * dx[k]) * dy[k]));
                }
                const sf2 pe = power * ssplat(kLog2e);  // __expf(x) = v_exp_f32(x log2 e)
                G[k] = sf2{__builtin_amdgcn_exp2f(pe.x), __builtin_amdgcn_exp2f(pe.y)};
                og[k] = ssplat(w1.y) * G[k];
                va[k] = on[2 * k] & (contributor <= last[2 * k]) & !(power.x > 0.f) & !(og[k].x < 1.0f / 255.0f);
                vb[k] = on[2 * k + 1] & (contributor <= last[2 * k + 1]) & !(power.y > 0.f) &
                        !(og[k].y < 1.0f / 255.0f);
                any = any | va[k] | vb[k];
            }
            if (__ballot(any) == 0ull) continue;  // wave-uniform skip (warp.any)
            const float4 w2 = s_w2[j];
            const float rsig = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, w2.y)));
            sf2 Fmx, Fmy, Fcx, Fcy, Fcz, Fops, Ftx, Fty, Fdt, Fdr;
#pragma unroll
            for (int k = 0; k < NPR; k++) {
                // (an invalid half: offsets 0 keep its terms finite, its gradient factors are zeroed below)
                const sf2 dxk = ssel(va[k], vb[k], dx[k], ssplat(0.f));
                const sf2 dyk = ssel(va[k], vb[k], dy[k], ssplat(0.f));
                const sf2 alpha = {fminf(0.99f, og[k].x), fminf(0.99f, og[k].y)};
                sf2 t_peak;
                {
#pragma clang fp contract(off)
                    t_peak = __builtin_elementwise_fma(ssplat(w1.w), dyk, ssplat(w1.z) * dxk) + ssplat(w2.x);
                }
                const sf2 md_tp = mDepth[k] - t_peak;
                const sf2 t_delta = md_tp * ssplat(rsig);
                const sf2 ge = ((ssplat(-0.5f) * t_delta) * t_delta) * ssplat(kLog2e);
                const sf2 G_exp = {__builtin_amdgcn_exp2f(ge.x), __builtin_amdgcn_exp2f(ge.y)};
                const sf2 Gt = alpha * G_exp;
                const sf2 omg = ssplat(1.f) - Gt, oma = ssplat(1.f) - alpha;
                sf2 dL_dGt = (kappa[k] * ssplat(0.25f)) * sf2{fast_rcp(omg.x), fast_rcp(omg.y)};
                dL_dGt = ssel(md_tp.x > 0.f, md_tp.y > 0.f, dL_dGt, -dL_dGt);
                dL_dGt = ssel(va[k] && rsig > 0.f, vb[k] && rsig > 0.f, dL_dGt, ssplat(0.f));
                const sf2 kr = ssel(va[k] && t_delta.x > 0.f, vb[k] && t_delta.y > 0.f,
                                    ssplat(0.5f) * sf2{fast_rcp(oma.x), fast_rcp(oma.y)}, ssplat(0.f));
                const sf2 dL_dopa = dL_dGt * G_exp - kappa[k] * kr;
                const sf2 dL_ddelta = -dL_dGt * Gt * t_delta;
                const sf2 dL_drsig = dL_ddelta * md_tp;
                const sf2 dL_dt = -dL_ddelta * ssplat(rsig);
                const sf2 dL_dG = ssplat(w1.y) * dL_dopa;
                const sf2 Gv = ssel(va[k], vb[k], G[k], ssplat(0.f));  // (power > 0 may have overflowed G)
                const sf2 gdx = Gv * dxk, gdy = Gv * dyk;
                const sf2 dG_ddelx = -gdx * ssplat(w0.z) - gdy * ssplat(w0.w);
                const sf2 dG_ddely = -gdy * ssplat(w1.x) - gdx * ssplat(w0.w);
                const sf2 dL_ddelx = dL_dG * dG_ddelx + dL_dt * ssplat(w1.z);
                const sf2 dL_ddely = dL_dG * dG_ddely + dL_dt * ssplat(w1.w);
                dpx[k] -= dL_ddelx;
                dpy[k] -= dL_ddely;
                const sf2 c0 = ssplat(-0.5f) * gdx * dL_dG, c2 = ssplat(-0.5f) * gdy * dL_dG;
                const sf2 cx = c0 * dxk, cy = c0 * dyk, cz = c2 * dyk, ops = Gv * dL_dopa;
                const sf2 tx = dL_dt * dxk, ty = dL_dt * dyk;
                Fmx = k ? Fmx + dL_ddelx : dL_ddelx;
                Fmy = k ? Fmy + dL_ddely : dL_ddely;
                Fcx = k ? Fcx + cx : cx;
                Fcy = k ? Fcy + cy : cy;
                Fcz = k ? Fcz + cz : cz;
                Fops = k ? Fops + ops : ops;
                Ftx = k ? Ftx + tx : tx;
                Fty = k ? Fty + ty : ty;
                Fdt = k ? Fdt + dL_dt : dL_dt;
                Fdr = k ? Fdr + dL_drsig : dL_drsig;
            }
            float f[16];
#pragma unroll
            for (int q = 0; q < 16; q++) f[q] = 0.f;
            f[kAccMean2D + 0] = (Fmx.x + Fmx.y) * ddelx_dx;
            f[kAccMean2D + 1] = (Fmy.x + Fmy.y) * ddely_dy;
            f[kAccConic + 0] = Fcx.x + Fcx.y;
            f[kAccConic + 1] = Fcy.x + Fcy.y;
            f[kAccConic + 2] = Fcz.x + Fcz.y;
            f[kAccConic + 3] = Fops.x + Fops.y;
            f[kAccPlane + 0] = Ftx.x + Ftx.y;
            f[kAccPlane + 1] = Fty.x + Fty.y;
            f[kAccPlane + 2] = Fdt.x + Fdt.y;
            f[kAccPlane + 3] = Fdr.x + Fdr.y;
            const float red = wave_transpose_reduce16(f);
            // lanes 4k hold field k; colour (0-2) and normal (9-11) are zero here
            const int field = lane >> 2;
            const bool field_lane = (lane & 3) == 0 && field >= kAccMean2D &&
                                    (field < kAccNormal || field >= kAccPlane);
            const uint32_t g = __builtin_amdgcn_readfirstlane(s_id[j]);
            if (field_lane) atomicAdd(a.acc + (size_t)g * kAccFields + field, red);
        }
    }
    const float* Pm = a.proj;
#pragma unroll
    for (int q = 0; q < NQ; q++) {
        if (!in[q]) continue;
        // dL/dpoints2D in NDC units, then the projection backward
        // (preprocessPointsCUDA bwd, sample_backward.cu:42-75)
        const uint32_t id = pid[q];
        const sf2 gxp = dpx[q >> 1], gyp = dpy[q >> 1];
        const float gx2 = ((q & 1) ? gxp.y : gxp.x) * ddelx_dx, gy2 = ((q & 1) ? gyp.y : gyp.x) * ddely_dy;
        const float mx = a.points3D[3 * id], my = a.points3D[3 * id + 1], mz = a.points3D[3 * id + 2];
        const float hw = Pm[3] * mx + Pm[7] * my + Pm[11] * mz + Pm[15];
        const float m_w = 1.0f / (hw + 0.0000001f);
        const float mul1 = (Pm[0] * mx + Pm[4] * my + Pm[8] * mz + Pm[12]) * m_w * m_w;
        const float mul2 = (Pm[1] * mx + Pm[5] * my + Pm[9] * mz + Pm[13]) * m_w * m_w;
        a.dL_dpoints3D[3 * id + 0] = (Pm[0] * m_w - Pm[3] * mul1) * gx2 + (Pm[1] * m_w - Pm[3] * mul2) * gy2;
        a.dL_dpoints3D[3 * id + 1] = (Pm[4] * m_w - Pm[7] * mul1) * gx2 + (Pm[5] * m_w - Pm[7] * mul2) * gy2;
        a.dL_dpoints3D[3 * id + 2] = (Pm[8] * m_w - Pm[11] * mul1) * gx2 + (Pm[9] * m_w - Pm[11] * mul2) * gy2;
    }
}

// chunks <= ceil(points / 256) + tiles holding points
uint32_t sample_chunk_bound(int PN, uint32_t tiles) {
    return (uint32_t)((PN + kTilePixels - 1) / kTilePixels) + min(tiles, (uint32_t)PN);
}

hipError_t launch_sample_bwd(const SampleBwdParams& b, const GeomState& gs, const BinningState& bs,
                             const TileState& ts, const PointState& ps, const PointBinState& pb,
                             const SampleTiles& st, const ChunkState& cs, const BwdState& ws, hipStream_t stream) {
    const FwdParams& p = b.f;
    const uint32_t tiles = p.grid_x * p.grid_y;
    if (b.PN == 0 || p.P == 0) return hipSuccess;
    SampleBwdArgs a;
    a.ranges = ts.ranges;
    a.point_list = bs.point_list;
    a.splats = gs.splats;
    a.chunk_off = st.chunk_off;
    a.pt_ranges = st.pt_ranges;
    a.pt_list = pb.pt_list;
    a.totals = st.totals;
    a.chunk_max = cs.chunk_max;
    a.pt_xy = ps.xy;
    a.pt_last = ps.last;
    a.pt_mdepth = ps.mdepth;
    a.pt_dT = ps.dT;
    a.pt_cached = ps.cached;
    a.points3D = b.points3D;
    a.inside = b.inside;
    a.dL_doutput = b.dL_doutput;
    a.dL_dpoints3D = b.dL_dpoints3D;
    a.proj = p.proj;
    a.W = p.W;
    a.H = p.H;
    a.num_tiles = tiles;
    a.focal_x = p.focal_x;
    a.focal_y = p.focal_y;
    a.acc = ws.acc;
    a.chunk_order = ws.tile_order;
    const uint32_t bound = sample_chunk_bound(b.PN, tiles);
    constexpr int kNpr = GSR_SAMPLE_BWD_NPR;
    if (GSR_SAMPLE_BWD_PAIRS)
        hipLaunchKernelGGL(sample_bwd_pairs_kernel<kNpr>, dim3(bound), dim3(kTilePixels / (2 * kNpr)), 0, stream, a);
    else
        hipLaunchKernelGGL(sample_bwd_kernel, dim3(bound), dim3(kTilePixels), 0, stream, a);
    return hipGetLastError();
}

}  // namespace gsr
