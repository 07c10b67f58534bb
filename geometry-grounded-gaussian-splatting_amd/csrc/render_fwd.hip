// render_fwd.hip — per-tile front-to-back alpha compositing on gfx950, with
// the geometry outputs (normal, median depth) of the reference.
//
// Replaces renderCUDA<3, GEOMETRY, 8, 5> (render_forward.cu:391-671) and its
// dispatch FORWARD::render (:674-708).
//
// One 256-lane workgroup (4 wave64) per 16x16 tile; a wave covers a 16x4
// strip of pixels.  Workgroups are remapped so the tiles one XCD receives are
// contiguous (neighbouring tiles share Gaussians, hence that XCD's L2).
// The tile's depth-sorted list is gathered through LDS in batches of 256
// Splat records (4 x 16 B per record, broadcast ds_read_b128 in the hot
// loop).  The block-wide early exit of the reference (__syncthreads_and) is a
// per-wave ballot written to LDS before the staging barrier.
//
// GEOM: after the composite the tile's max contributor is reduced across the
// block and the median depth is found by the reference's 5 x 8-way bisection
// of the vacancy transmittance (render_forward.cu:549-645).  When the tile's
// contributing prefix fits (<= kResident records) it is staged into LDS once
// (48 B per record: w0, w1, w2) and all five bisection passes run out of LDS
// with no further barriers; longer lists are restaged per pass.
#include "gsr_kernels.h"

namespace gsr {

constexpr int kResident = 512;

struct RenderFwdArgs {
    const uint2* ranges;
    const uint32_t* point_list;
    const Splat* splats;
    int W, H;
    uint32_t grid_x, num_tiles;
    float focal_x, focal_y;
    const float* bg;
    uint32_t* n_contrib;
    uint32_t* max_contrib;
    float* out_color;
    float* out_alpha;
    float* out_normal;
    float* out_mdepth;
    float one;  // 1.0f, passed at run time so rsq(1.0) is evaluated by the hardware
};

// One contributor's factor on the bisection samples (render_forward.cu:610-621):
//   T_p[s] *= (ts > t_peak ? 1 - a : 1 - a g) * rsqrt(1 - a g),  g = exp(-delta^2 / 2)
// Exact shortcut (SKIP): when every sample of the window has |delta| > 7,
// a*g < e^-24.5 < 2^-25, so 1 - a*g rounds to exactly 1.0f and the factor is
// exactly (1 - a) * rsq(1) in front of the window or rsq(1) behind it (the
// samples are monotone in s, so the two window ends decide).  rsq1 is the
// hardware's rsq(1.0) so the shortcut is bit-identical to the full path.
template <bool FIRST, bool SKIP>
__device__ __forceinline__ void bisect_step(float (&Tp)[kSplit + 1], float dmin, float interval, float alpha,
                                            float t_peak, float rsig, float rsq1) {
    constexpr int START = FIRST ? 0 : 1;
    constexpr int END = FIRST ? kSplit + 1 : kSplit;
    const bool ball = rsig > 0.f;
    if constexpr (SKIP) {
        const float d_lo = ((dmin + interval * START) - t_peak) * rsig;
        const float d_hi = ((dmin + interval * (END - 1)) - t_peak) * rsig;
        if (ball && d_lo > 7.f) {
            const float f = (1.f - alpha) * rsq1;
#pragma unroll
            for (int s = START; s < END; s++) Tp[s] *= f;
            return;
        }
        if (ball && d_hi < -7.f) {
#pragma unroll
            for (int s = START; s < END; s++) Tp[s] *= rsq1;
            return;
        }
    }
#pragma unroll
    for (int s = START; s < END; s++) {
        const float ts = dmin + interval * s;
        const float delta = (ts - t_peak) * rsig;
        const float gg = ball ? __expf(-0.5f * delta * delta) : 0.f;
        const float omg = 1.f - alpha * gg;
        const float rv = __builtin_amdgcn_rsqf(omg);
        Tp[s] *= (ts > t_peak ? (1.f - alpha) : omg) * rv;
    }
}

// Diagnostic counters (STATS builds only, option GSR_OPT_RENDER_STATS):
// [0] bisection wave-visits, [1] lanes reaching a bisection step,
// [2] wave-visits with any lane on the full path, [3] lanes on the full path,
// [4] composite wave-visits, [5] composite active lanes.
__device__ unsigned long long g_render_stats[8];

template <bool GEOM, bool SKIP, bool STATS = false>
__global__ void __launch_bounds__(256) render_fwd_kernel(RenderFwdArgs a) {
    // LDS: composite staging (4 x 256 x 16 B = 16 KB) aliased with the
    // bisection cache (3 x 512 x 16 B = 24 KB).
    __shared__ float4 s_rec[3 * kResident];
    __shared__ int s_alive[2][4];
    __shared__ uint32_t s_max[4];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const uint32_t tile = xcd_remap(blockIdx.x, a.num_tiles);
    const uint32_t tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int px = tx * kTile + (tid & 15), py = ty * kTile + (tid >> 4);
    const bool inside = px < a.W && py < a.H;
    const float pixx = (float)px, pixy = (float)py;

    const uint2 range = a.ranges[tile];
    const int total = (int)(range.y - range.x);
    const int rounds = (total + kTilePixels - 1) / kTilePixels;

    float4* s_w0 = s_rec;
    float4* s_w1 = s_rec + kTilePixels;
    float4* s_w2 = s_rec + 2 * kTilePixels;
    float4* s_w3 = s_rec + 3 * kTilePixels;  // within the 24 KB (3*512 float4 >= 4*256)

    float T = 1.0f;
    uint32_t contributor = 0, last = 0;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f;
    float N0 = 0.f, N1 = 0.f, N2 = 0.f, m_init = 0.f;
    bool done = !inside;

    int toDo = total;
    for (int i = 0; i < rounds; i++, toDo -= kTilePixels) {
        // block-wide early exit: every wave publishes whether any lane is live
        const bool wave_alive = __ballot(!done) != 0ull;
        if ((tid & 63) == 0) s_alive[i & 1][wave] = wave_alive;
        __syncthreads();  // also: everyone finished reading the previous batch
        if (!(s_alive[i & 1][0] | s_alive[i & 1][1] | s_alive[i & 1][2] | s_alive[i & 1][3])) break;
        const int k = i * kTilePixels + tid;
        if (k < total) {
            const Splat sp = a.splats[a.point_list[range.x + k]];
            s_w0[tid] = sp.w0;
            s_w1[tid] = sp.w1;
            s_w2[tid] = sp.w2;
            s_w3[tid] = sp.w3;
        }
        __syncthreads();
        const int n = min(kTilePixels, toDo);
        for (int j = 0; !done && j < n; j++) {
            contributor++;
            const float4 w0 = s_w0[j];
            const float dx = w0.x - pixx, dy = w0.y - pixy;
            const float4 w1 = s_w1[j];
            const float power = -0.5f * (w0.z * dx * dx + w1.x * dy * dy) - w0.w * dx * dy;
            if (power > 0.0f) continue;
            const float alpha = fminf(0.99f, w1.y * __expf(power));
            if (alpha < 1.0f / 255.0f) continue;
            const float test_T = T * (1.f - alpha);
            if (test_T < 0.0001f) {
                done = true;
                continue;
            }
            const float aT = alpha * T;
            const float4 w2 = s_w2[j];
            const float4 w3 = s_w3[j];
            C0 += w2.z * aT;
            C1 += w2.w * aT;
            C2 += w3.x * aT;
            if constexpr (GEOM) {
                const float t = w1.z * dx + w1.w * dy + w2.x;
                N0 += w3.y * aT;
                N1 += w3.z * aT;
                N2 += w3.w * aT;
                m_init = T > 0.5f ? t : m_init;
            }
            T = test_T;
            last = contributor;
        }
    }

    // block max of last contributor (cub BlockReduce in the reference)
    const uint32_t wmax = wave_max_u(last);
    if ((tid & 63) == 0) s_max[wave] = wmax;
    __syncthreads();
    const uint32_t max_contrib = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));

    float mDepth = 0.f;
    if constexpr (GEOM) {
        unsigned long long st[4] = {0, 0, 0, 0};
        float Tp[kSplit + 1];
        const float rsq1 = __builtin_amdgcn_rsqf(a.one);  // hardware rsq(1.0) (kept opaque to the compiler)
        float dmin = fmaxf(m_init - kSampleRange, 0.f);
        float dmax = fmaxf(m_init + kSampleRange, 0.f);
        bool in_range = T <= kMinTransmittance;
        const bool resident = max_contrib <= (uint32_t)kResident;
        float4* c_w0 = s_rec;
        float4* c_w1 = s_rec + kResident;
        float4* c_w2 = s_rec + 2 * kResident;
        const int chunk = resident ? kResident : kTilePixels;
        const int chunks = ((int)max_contrib + chunk - 1) / chunk;
        auto stage = [&](int c0) {
            for (int k = tid; k < chunk && c0 + k < (int)max_contrib; k += kTilePixels) {
                const Splat* sp = a.splats + a.point_list[range.x + c0 + k];
                c_w0[k] = sp->w0;
                c_w1[k] = sp->w1;
                c_w2[k] = sp->w2;
            }
        };
        if (resident && max_contrib > 0) {
            __syncthreads();
            stage(0);
            __syncthreads();
        }
#pragma unroll 1
        for (int it = 0; it < kSplitIterations; it++) {
            const bool first = it == 0;
            if (first) {
#pragma unroll
                for (int s = 0; s <= kSplit; s++) Tp[s] = 1.f;
            } else {
#pragma unroll
                for (int s = 1; s < kSplit; s++) Tp[s] = 1.f;
            }
            const float interval = (dmax - dmin) * (1.f / (float)kSplit);
            bool bdone = !in_range;
            uint32_t c = 0;
            for (int ch = 0; ch < chunks; ch++) {
                if (!resident) {
                    __syncthreads();
                    stage(ch * chunk);
                    __syncthreads();
                }
                const int n = min(chunk, (int)max_contrib - ch * chunk);
                for (int j = 0; !bdone && j < n; j++) {
                    c++;
                    bdone = c >= last;
                    if constexpr (STATS) {
                        const unsigned long long m = __ballot(1);
                        if ((tid & 63) == __builtin_ctzll(m)) st[0] += 1;
                    }
                    const float4 w0 = c_w0[j];
                    const float dx = w0.x - pixx, dy = w0.y - pixy;
                    const float4 w1 = c_w1[j];
                    const float power = -0.5f * (w0.z * dx * dx + w1.x * dy * dy) - w0.w * dx * dy;
                    if (power > 0.0f) continue;
                    const float alpha = fminf(0.99f, w1.y * __expf(power));
                    if (alpha < 1.0f / 255.0f) continue;
                    const float4 w2 = c_w2[j];
                    const float t_peak = w1.z * dx + w1.w * dy + w2.x;
                    if constexpr (STATS) {
                        const int START = first ? 0 : 1, END = first ? kSplit + 1 : kSplit;
                        const float d_lo = ((dmin + interval * START) - t_peak) * w2.y;
                        const float d_hi = ((dmin + interval * (END - 1)) - t_peak) * w2.y;
                        const bool full = !(w2.y > 0.f && (d_lo > 7.f || d_hi < -7.f));
                        const unsigned long long m = __ballot(1);
                        const unsigned long long f = __ballot(full);
                        if ((tid & 63) == __builtin_ctzll(m)) {
                            st[1] += __popcll(m);
                            st[2] += f != 0ull;
                            st[3] += __popcll(f);
                        }
                    }
                    if (first) bisect_step<true, SKIP>(Tp, dmin, interval, alpha, t_peak, w2.y, rsq1);
                    else bisect_step<false, SKIP>(Tp, dmin, interval, alpha, t_peak, w2.y, rsq1);
                }
            }
            if (first) in_range = (Tp[0] >= 0.5f) && (Tp[kSplit] <= 0.5f) && in_range;
            int start_id = 0;
#pragma unroll
            for (int p = 1; p < kSplit; p++) start_id = Tp[p] >= 0.5f ? p : start_id;
            // select Tp[start_id], Tp[start_id + 1] with constant register indices
            float lo = Tp[0], hi = Tp[1];
#pragma unroll
            for (int p = 1; p < kSplit; p++) {
                lo = start_id == p ? Tp[p] : lo;
                hi = start_id == p ? Tp[p + 1] : hi;
            }
            dmax = dmin + (start_id + 1) * interval;
            dmin = dmin + (start_id + 0) * interval;
            Tp[0] = lo;
            Tp[kSplit] = hi;
        }
        if constexpr (STATS) {
            for (int q = 0; q < 4; q++)
                if (st[q]) atomicAdd(&g_render_stats[q], st[q]);
        }
        float w_max = (Tp[0] - 0.5f) / (Tp[0] - Tp[kSplit]);
        w_max = fminf(fmaxf(w_max, 0.f), 1.f);  // __saturatef (NaN -> 0)
        const float w_min = 1.f - w_max;
        mDepth = in_range ? w_max * dmax + w_min * dmin : 0.f;
    }

    if (inside) {
        const int HW = a.H * a.W;
        const int pix = a.W * py + px;
        a.n_contrib[pix] = last;
        a.out_color[pix] = C0 + T * a.bg[0];
        a.out_color[HW + pix] = C1 + T * a.bg[1];
        a.out_color[2 * HW + pix] = C2 + T * a.bg[2];
        a.out_alpha[pix] = 1.f - T;
        if constexpr (GEOM) {
            const float pnx = (pixx - (float)(a.W - 1) / 2.f) / a.focal_x;
            const float pny = (pixy - (float)(a.H - 1) / 2.f) / a.focal_y;
            const float rln = 1.0f / sqrtf(pnx * pnx + pny * pny + 1.f);
            a.out_mdepth[pix] = mDepth * rln;
            const float len = 1.f - T;
            a.out_normal[pix] = last ? N0 / len : 0.f;
            a.out_normal[HW + pix] = last ? N1 / len : 0.f;
            a.out_normal[2 * HW + pix] = last ? N2 / len : 0.f;
        } else {
            a.out_mdepth[pix] = 0.f;
            a.out_normal[pix] = 0.f;
            a.out_normal[HW + pix] = 0.f;
            a.out_normal[2 * HW + pix] = 0.f;
        }
    }
    if (tid == 0) a.max_contrib[tile] = max_contrib;
}

hipError_t launch_render_fwd(const FwdParams& p, const GeomState& gs, const BinningState& bs, const ImageState& is,
                             const TileState& ts, float* out_color, float* out_alpha, float* out_normal,
                             float* out_mdepth, hipStream_t stream) {
    RenderFwdArgs a;
    a.ranges = ts.ranges;
    a.point_list = bs.point_list;
    a.splats = gs.splats;
    a.W = p.W;
    a.H = p.H;
    a.grid_x = p.grid_x;
    a.num_tiles = p.grid_x * p.grid_y;
    a.focal_x = p.focal_x;
    a.focal_y = p.focal_y;
    a.bg = p.background;
    a.n_contrib = is.n_contrib;
    a.max_contrib = ts.max_contrib;
    a.out_color = out_color;
    a.out_alpha = out_alpha;
    a.out_normal = out_normal;
    a.out_mdepth = out_mdepth;
    a.one = 1.0f;
    if (a.num_tiles == 0) return hipSuccess;
    if (p.require_depth) {
        if (option(kOptRenderStats))
            hipLaunchKernelGGL((render_fwd_kernel<true, true, true>), dim3(a.num_tiles), dim3(kTilePixels), 0, stream, a);
        else if (option(kOptBisectSkip))
            hipLaunchKernelGGL((render_fwd_kernel<true, true>), dim3(a.num_tiles), dim3(kTilePixels), 0, stream, a);
        else
            hipLaunchKernelGGL((render_fwd_kernel<true, false>), dim3(a.num_tiles), dim3(kTilePixels), 0, stream, a);
    } else {
        hipLaunchKernelGGL((render_fwd_kernel<false, false>), dim3(a.num_tiles), dim3(kTilePixels), 0, stream, a);
    }
    return hipGetLastError();
}

hipError_t read_render_stats(unsigned long long* out, bool reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_render_stats), sizeof(unsigned long long) * 8);
    if (e == hipSuccess && reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_render_stats), z, sizeof(z));
    }
    return e;
}

}  // namespace gsr
