// tilelists.hip — per-tile Gaussian lists without sorting the instances.
//
// Replaces duplicateWithKeys + cub::DeviceRadixSort::SortPairs +
// identifyTileRanges (CR/rasterizer_impl.cu:70-161, 392-421) for grids of
// up to kMaxGrid x kMaxGrid tiles (binning.hip keeps the sort path for larger
// ones).  Input: the Gaussians in q order = (depth bits, index), the stable
// depth sort of binning.hip.  Output: for every tile, the Gaussians whose
// live tile set (tiles.h: rect + opacity-aware ellipse culling) contains it,
// in q order — exactly the reference's per-tile (depth, index) order with
// the culled instances removed — and the tile ranges.
//
// Two stable counting passes, each a deterministic rank-and-scatter:
//   rows:  q order -> per tile row, the (Gaussian, column span) entries in
//          q order;
//   tiles: per row -> per tile of the row, the Gaussians in q order.
// Each pass: (1) one wave per segment counts its entries per bucket (LDS
// histogram); (2) an exclusive scan of the [bucket][segment] counts gives
// every (bucket, segment) its first output slot; (3) the same wave walks its
// segment again 64 entries at a time: every entry ORs its lane bit into a
// 64-bit LDS mask per bucket it lands in, its rank among the 64 is the
// popcount of the lower lanes' bits, and the bucket's first entry advances
// the bucket's running slot.  One wave per segment and in-order LDS make
// this barrier-free; rows and tile columns are few (<= kMaxGrid), so the
// LDS per wave is small and many segments run per CU.
#pragma clang fp contract(off)

#include <rocprim/device/device_reduce.hpp>
#include <rocprim/device/device_scan.hpp>

#include "gsr_kernels.h"
#include "tiles.h"

namespace gsr {

#ifndef GSR_ROW_SEG
#define GSR_ROW_SEG 64  // measured at C3: tile_lists 0.248 ms vs 0.256 (128), 0.277 (96), 0.31 (256), 0.39 (512)
#endif
#ifndef GSR_ROW_SEG_BIG
#define GSR_ROW_SEG_BIG GSR_ROW_SEG  // row-pass segment for P > kRowSegBigP (multiple of 64)
#endif
#ifndef GSR_TILE_SEG
#define GSR_TILE_SEG 512
#endif
constexpr int kRowSeg = GSR_ROW_SEG;    // Gaussians per row-pass segment
constexpr int kRowSegBig = GSR_ROW_SEG_BIG;
constexpr int kRowSegBigP = 2000000;
static_assert(kRowSeg % 64 == 0 && kRowSegBig % 64 == 0, "row-pass segments are whole 64-entry chunks");
constexpr int kTileSeg = GSR_TILE_SEG;  // row entries per tile-pass segment
#ifndef GSR_ROW_WAVES
#define GSR_ROW_WAVES 1
#endif
// Row-pass waves per workgroup: each wave still owns one segment and its own
// LDS share (no cross-wave step), so a wave orders its LDS phases with a
// wave-scope fence instead of a workgroup barrier; more than one wave per
// workgroup only changes how many segments a CU can hold at once.
constexpr int kRowWaves = GSR_ROW_WAVES;

// orders one wave's LDS phases (LDS instructions of a wave execute in issue
// order; this keeps the compiler from moving them across the point)
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void row_lds_order() {
    if constexpr (kRowWaves == 1) __syncthreads();
    else wave_lds_order();
}

// ------------------------------------------- exclusive scan, device-sized
// The counting passes' [bucket][segment] count arrays are scanned by a
// two-kernel reduce-then-scan whose length n is read on the device (the
// tile pass's segment count, gx * segbase[gy], is known there only): the
// grid covers the host's upper bound, blocks past n exit at once, no input
// beyond n is read (so the count array needs no clearing) and out[n] gets
// the total.  (rocPRIM's lookback scan over the host bound scanned ~6x the
// live length at C3 behind a memset: 46 us of the tile-list stage.)
constexpr int kScanThreads = 256, kScanItems = 16, kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ uint32_t scan_len(uint32_t n_host, const uint32_t* n_dev, uint32_t mul) {
    return n_dev ? mul * *n_dev : n_host;
}

// exclusive scan of one value per thread over the block; *total = block sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; w++) {
        const uint32_t t = s_w[w];
        before += w < wave ? t : 0u;
        all += t;
    }
    *total = all;
    return before + x - v;
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* s_w) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) s_w[wave] = v;
    __syncthreads();
    uint32_t all = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; w++) all += s_w[w];
    __syncthreads();  // s_w is reused
    return all;
}

__device__ __forceinline__ void scan_load(const uint32_t* in, uint32_t i0, uint32_t n, uint32_t (&v)[kScanItems]) {
    if (i0 + kScanItems <= n) {
        const uint4* q = reinterpret_cast<const uint4*>(in + i0);  // i0 is a multiple of 16: 16-B aligned
#pragma unroll
        for (int k = 0; k < kScanItems / 4; k++) {
            const uint4 u = q[k];
            v[4 * k] = u.x;
            v[4 * k + 1] = u.y;
            v[4 * k + 2] = u.z;
            v[4 * k + 3] = u.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; k++) v[k] = i0 + k < n ? in[i0 + k] : 0u;
    }
}

__global__ void __launch_bounds__(kScanThreads)
    scan_sums_kernel(const uint32_t* __restrict__ in, uint32_t n_host, const uint32_t* __restrict__ n_dev, uint32_t mul,
                     uint32_t* __restrict__ sums) {
    __shared__ uint32_t s_w[kScanThreads / 64];
    const uint32_t n = scan_len(n_host, n_dev, mul);
    const uint32_t base = blockIdx.x * (uint32_t)kScanTile;
    if (base >= n) {
        if (threadIdx.x == 0) sums[blockIdx.x] = 0u;
        return;
    }
    uint32_t v[kScanItems];
    scan_load(in, base + threadIdx.x * kScanItems, n, v);
    uint32_t t = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++) t += v[k];
    uint32_t total;
    (void)block_excl_scan(t, s_w, &total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ void __launch_bounds__(kScanThreads)
    scan_out_kernel(const uint32_t* __restrict__ in, uint32_t n_host, const uint32_t* __restrict__ n_dev, uint32_t mul,
                    const uint32_t* __restrict__ sums, uint32_t* __restrict__ out) {
    __shared__ uint32_t s_w[kScanThreads / 64];
    const uint32_t n = scan_len(n_host, n_dev, mul);
    const uint32_t base = blockIdx.x * (uint32_t)kScanTile;
    if (base > n) return;  // (the block holding index n writes the total there)
    const uint32_t i0 = base + threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    scan_load(in, i0, n, v);
    uint32_t t = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++) t += v[k];
    // this block's offset: the sum of the earlier blocks' sums (<= a few
    // thousand words from L2; cheaper than a separate launch scanning them)
    uint32_t pre = 0;
    for (uint32_t j = threadIdx.x; j < blockIdx.x; j += kScanThreads) pre += sums[j];
    pre = block_sum(pre, s_w);
    uint32_t total;
    uint32_t run = pre + block_excl_scan(t, s_w, &total);
    if (i0 + kScanItems <= n) {
        uint4* q = reinterpret_cast<uint4*>(out + i0);
#pragma unroll
        for (int k = 0; k < kScanItems / 4; k++) {
            uint4 u;
            u.x = run;
            run += v[4 * k];
            u.y = run;
            run += v[4 * k + 1];
            u.z = run;
            run += v[4 * k + 2];
            u.w = run;
            run += v[4 * k + 3];
            q[k] = u;
        }
        if (i0 + kScanItems == n) out[n] = run;
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; k++) {
            if (i0 + k <= n) out[i0 + k] = run;
            run += v[k];
        }
    }
}

// exclusive scan of in[0, n) into out[0, n], n = n_dev ? mul * *n_dev : n;
// cap >= n is the host's bound, sums holds scan_sums_count(cap) words
uint32_t scan_sums_count(size_t cap) { return (uint32_t)(cap / kScanTile + 1); }

hipError_t launch_scan_excl(const uint32_t* in, uint32_t* out, size_t cap, uint32_t n_host, const uint32_t* n_dev,
                            uint32_t mul, uint32_t* sums, hipStream_t stream) {
    const uint32_t nb = scan_sums_count(cap);
    hipLaunchKernelGGL(scan_sums_kernel, dim3(nb), dim3(kScanThreads), 0, stream, in, n_host, n_dev, mul, sums);
    hipLaunchKernelGGL(scan_out_kernel, dim3(nb), dim3(kScanThreads), 0, stream, in, n_host, n_dev, mul,
                       (const uint32_t*)sums, out);
    return hipGetLastError();
}

bool list_binning(uint32_t gx, uint32_t gy) { return gx <= (uint32_t)kMaxGrid && gy <= (uint32_t)kMaxGrid; }

ListLayout list_layout(int P, int K, uint32_t gx, uint32_t gy) {
    ListLayout L;
    L.rowseg = P > kRowSegBigP ? kRowSegBig : kRowSeg;
    L.nseg_rows = (P + L.rowseg - 1) / L.rowseg;
    L.nseg_tiles_max = (K + kTileSeg - 1) / kTileSeg + (int)gy;
    size_t a = 0, b = 0, c = 0;
    (void)rocprim::exclusive_scan(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u,
                                  (size_t)gy * L.nseg_rows, rocprim::plus<uint32_t>());
    (void)rocprim::exclusive_scan(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u,
                                  (size_t)gx * L.nseg_tiles_max + 1, rocprim::plus<uint32_t>());
    (void)rocprim::reduce(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)P,
                          rocprim::plus<uint32_t>());
    L.tmp_bytes = a > b ? a : b;
    L.tmp_bytes = L.tmp_bytes > c ? L.tmp_bytes : c;
    // the device-sized scans' block sums
    const size_t d = 4 * (size_t)scan_sums_count((size_t)gx * L.nseg_tiles_max + (size_t)gy * L.nseg_rows);
    L.tmp_bytes = L.tmp_bytes > d ? L.tmp_bytes : d;
    return L;
}

size_t reduce_temp_bytes(int P) {
    size_t c = 0;
    (void)rocprim::reduce(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)P,
                          rocprim::plus<uint32_t>());
    return c;
}


// --------------------------------------------------------------- rows pass
struct QGauss {  // one Gaussian in q order, as the row kernels need it
    bool on;
    uint32_t g;
    Ellipse E;
    TileRect R;
};
// the Gaussian at q: its footprint (GeomState::foot, written by the
// preprocess: the Splat record's centre, conic and opacity coefficient bit
// for bit, and the tile_rect of its radius; an empty rect when culled)
__device__ __forceinline__ QGauss load_q(int q, int q1, const uint32_t* order, const uint4* foot, float pad) {
    QGauss G{};
    if (q >= q1) return G;
    G.g = order[q];
    const uint4 f0 = foot[2 * (size_t)G.g], f1 = foot[2 * (size_t)G.g + 1];
    G.R.x0 = f1.z & 0xffffu;
    G.R.y0 = f1.z >> 16;
    G.R.x1 = f1.w & 0xffffu;
    G.R.y1 = f1.w >> 16;
    if (!(G.R.x1 > G.R.x0 && G.R.y1 > G.R.y0)) return G;
    const float4 w0 = make_float4(__uint_as_float(f0.x), __uint_as_float(f0.y), __uint_as_float(f0.z),
                                  __uint_as_float(f0.w));
    const float4 w1 = make_float4(__uint_as_float(f1.x), __uint_as_float(f1.y), 0.f, 0.f);
    G.E = make_ellipse(w0, w1, pad);
    G.on = G.E.mode != 2;
    return G;
}

// rows_count writes, per Gaussian in q order, a 32-B record: its id (or
// kNoSpan when it has no live tile), its rect rows y0 | y1 << 16 and the
// column spans of rows y0 .. y0 + kRecSpans - 1 (kNoSpan where not live).
// rows_emit streams the records instead of gathering the splat by id and
// recomputing the spans; it falls back to both only for rows past the
// record's (Gaussians taller than kRecSpans tile rows).
constexpr int kRecSpans = 6;
constexpr uint32_t kNoSpan = 0xffffffffu;  // (spans are lo | hi << 16 with hi < 1024)

__global__ void __launch_bounds__(64 * kRowWaves)
    rows_count_kernel(int P, int nseg, int rowseg, uint32_t gy, float pad, const uint32_t* __restrict__ order,
                      const uint4* __restrict__ foot, uint32_t* __restrict__ M, uint4* __restrict__ qrec) {
    extern __shared__ unsigned long long s_dyn[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* s_cnt = reinterpret_cast<uint32_t*>(s_dyn) + wave * gy;
    const int seg = (int)xcd_remap(blockIdx.x, gridDim.x) * kRowWaves + wave;  // XCD-contiguous segments
    if (seg >= nseg) return;
    for (uint32_t y = lane; y < gy; y += 64) s_cnt[y] = 0u;
    row_lds_order();
    const int q0 = seg * rowseg, q1 = min(P, q0 + rowseg);
    for (int q = q0 + lane; q < q1; q += 64) {
        const QGauss G = load_q(q, q1, order, foot, pad);
        uint32_t lo, hi;
        // the record rows_emit reads instead of re-gathering and re-spanning
        uint32_t sp[kRecSpans];
#pragma unroll
        for (int k = 0; k < kRecSpans; k++) {
            const uint32_t y = G.R.y0 + (uint32_t)k;
            sp[k] = kNoSpan;
            if (G.on && y < G.R.y1 && row_span(G.E, G.R, y, &lo, &hi)) {
                sp[k] = lo | (hi << 16);
                atomicAdd(&s_cnt[y], 1u);
            }
        }
        qrec[2 * (size_t)q] = make_uint4(G.on ? G.g : kNoSpan, G.R.y0 | (G.R.y1 << 16), sp[0], sp[1]);
        qrec[2 * (size_t)q + 1] = make_uint4(sp[2], sp[3], sp[4], sp[5]);
        if (!G.on) continue;
        for (uint32_t y = G.R.y0 + kRecSpans; y < G.R.y1; y++)
            if (row_span(G.E, G.R, y, &lo, &hi)) atomicAdd(&s_cnt[y], 1u);
    }
    row_lds_order();
    for (uint32_t y = lane; y < gy; y += 64) M[(size_t)y * nseg + seg] = s_cnt[y];
}


// Ranking within a 64-entry chunk: every entry ORs its lane bit into its
// bucket's mask; its slot is the bucket's running slot plus the popcount of
// the lower lanes' bits, and the bucket's lowest lane advances the running
// slot into the other half of a ping-pong pair, so one walk over the
// entries does rank, write and advance.  The row-wide prologue of each chunk
// carries the untouched running slots over and clears the next chunk's masks.
__global__ void __launch_bounds__(64 * kRowWaves)
    rows_emit_kernel(int P, int nseg, int rowseg, uint32_t gy, float pad, const uint32_t* __restrict__ order,
                     const uint4* __restrict__ foot, const uint32_t* __restrict__ O, const uint4* __restrict__ qrec,
                     uint2* __restrict__ rows) {
    extern __shared__ unsigned long long s_dyn[];  // per wave: 2 x [gy] masks, then 2 x [gy] running slots
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long* s_cov = s_dyn + (size_t)wave * 3 * gy;
    uint32_t* s_run = reinterpret_cast<uint32_t*>(s_cov + 2 * gy);
    const int seg = (int)xcd_remap(blockIdx.x, gridDim.x) * kRowWaves + wave;  // XCD-contiguous segments
    if (seg >= nseg) return;
    const int q0 = seg * rowseg, q1 = min(P, q0 + rowseg);
    // the first chunk's records are requested before the strided running-slot
    // loads, so the two round trips overlap; later chunks' one chunk ahead
    uint4 n0 = make_uint4(kNoSpan, 0u, kNoSpan, kNoSpan), n1 = make_uint4(kNoSpan, kNoSpan, kNoSpan, kNoSpan);
    if (q0 + lane < q1) {
        n0 = qrec[2 * (size_t)(q0 + lane)];
        n1 = qrec[2 * (size_t)(q0 + lane) + 1];
    }
    for (uint32_t y = lane; y < gy; y += 64) {
        s_run[y] = O[(size_t)y * nseg + seg];
        s_cov[y] = 0ull;
    }
    row_lds_order();
    const unsigned long long bit = 1ull << lane, below = bit - 1ull;
    uint32_t cur = 0;
    for (int c0 = q0; c0 < q1; c0 += 64, cur ^= 1u) {
        unsigned long long* cov = s_cov + cur * gy;
        const uint32_t* run = s_run + cur * gy;
        uint32_t* run_next = s_run + (cur ^ 1u) * gy;
        const int q = c0 + lane;
        const uint4 r0 = n0, r1 = n1;
        n0 = make_uint4(kNoSpan, 0u, kNoSpan, kNoSpan);
        n1 = make_uint4(kNoSpan, kNoSpan, kNoSpan, kNoSpan);
        if (q + 64 < q1) {
            n0 = qrec[2 * (size_t)(q + 64)];
            n1 = qrec[2 * (size_t)(q + 64) + 1];
        }
        for (uint32_t y = lane; y < gy; y += 64) {
            run_next[y] = run[y];
            s_cov[(cur ^ 1u) * gy + y] = 0ull;
        }
        const bool on = r0.x != kNoSpan;
        const uint32_t y0 = r0.y & 0xffffu, y1 = r0.y >> 16;
        const uint32_t span[kRecSpans] = {r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
        // rows past the record: the splat's ellipse, as rows_count had it
        const bool tall = on && y1 > y0 + kRecSpans;
        QGauss G{};
        if (tall) G = load_q(q, q1, order, foot, pad);
        uint32_t lo, hi;
#pragma unroll
        for (int k = 0; k < kRecSpans; k++)
            if (span[k] != kNoSpan) atomicOr(&cov[y0 + (uint32_t)k], bit);
        if (tall)
            for (uint32_t y = y0 + kRecSpans; y < y1; y++)
                if (row_span(G.E, G.R, y, &lo, &hi)) atomicOr(&cov[y], bit);
        row_lds_order();
        auto emit = [&](uint32_t y, uint32_t sp) {
            const unsigned long long m = cov[y];
            const uint32_t rs = run[y];
            rows[rs + (uint32_t)__popcll(m & below)] = make_uint2(r0.x, sp);
            if ((m & below) == 0ull) run_next[y] = rs + (uint32_t)__popcll(m);
        };
#pragma unroll
        for (int k = 0; k < kRecSpans; k++)
            if (span[k] != kNoSpan) emit(y0 + (uint32_t)k, span[k]);
        if (tall)
            for (uint32_t y = y0 + kRecSpans; y < y1; y++)
                if (row_span(G.E, G.R, y, &lo, &hi)) emit(y, lo | (hi << 16));
        row_lds_order();
    }
}

// Coalesced emission helper (the tiles pass below).  (The rows
// pass with the staged emission measured 0.234 -> 0.239 ms at C3, 1.018 -> 1.008
// at C5: not adopted; its 8-B entries land in only ~5 rows per Gaussian.)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// --------------------------------------------------------------- tiles pass
// Row y's entries are [O_rows[y * nseg_rows], O_rows[(y + 1) * nseg_rows]);
// it is cut into ceil(len / kTileSeg) segments; segbase[y] is the exclusive
// prefix of the segment counts (segbase[gy] = total).  The tile-pass counts
// of row y live at [gx * segbase[y], gx * segbase[y + 1]), column-major
// (x * nk + k), so one exclusive scan orders them (row, column, segment).
__device__ __forceinline__ uint32_t row_begin(const uint32_t* O_rows, int nseg_rows, uint32_t y, uint32_t gy,
                                              uint32_t total) {
    return y < gy ? O_rows[(size_t)y * nseg_rows] : total;
}

struct TileSeg {
    bool on;
    uint32_t y, k, nk, e0, e1;
};
__device__ __forceinline__ TileSeg find_seg(uint32_t b, uint32_t gy, const uint32_t* segbase, const uint32_t* O_rows,
                                            int nseg_rows, uint32_t total) {
    TileSeg S{};
    if (b >= segbase[gy]) return S;
    uint32_t lo = 0, hi = gy;  // largest y with segbase[y] <= b
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (segbase[mid] <= b) lo = mid;
        else hi = mid;
    }
    S.on = true;
    S.y = lo;
    S.k = b - segbase[lo];
    S.nk = segbase[lo + 1] - segbase[lo];
    const uint32_t rb = row_begin(O_rows, nseg_rows, lo, gy, total), re = row_begin(O_rows, nseg_rows, lo + 1, gy, total);
    S.e0 = rb + S.k * kTileSeg;
    S.e1 = min(re, S.e0 + kTileSeg);
    return S;
}

// The segment table in LDS: segbase[0..gy] and every row's first entry
// (row_begin), so locating a segment is a binary search over LDS instead of
// ~log2(gy) + 3 dependent global round trips per segment.
__device__ __forceinline__ void stage_seg_table(uint32_t gy, int nseg_rows, const uint32_t* O_rows,
                                                const uint32_t* M_rows_last, const uint32_t* segbase, uint32_t* s_sb,
                                                uint32_t* s_rb) {
    const uint32_t total = O_rows[(size_t)gy * nseg_rows - 1] + M_rows_last[0];
    for (uint32_t y = threadIdx.x; y <= gy; y += blockDim.x) {
        s_sb[y] = segbase[y];
        s_rb[y] = row_begin(O_rows, nseg_rows, y, gy, total);
    }
    __syncthreads();
}
// The segment table built from the rows pass's scan by one wave (the work a
// separate one-workgroup launch did before): every row's first entry, its
// segment count ceil(len / kTileSeg), their exclusive scan in s_sb; `out`
// (one block) gets segbase for the kernels after.  One 64-lane block.
__device__ __forceinline__ void build_seg_table(uint32_t gy, int nseg_rows, const uint32_t* O_rows,
                                                const uint32_t* M_rows_last, uint32_t* s_sb, uint32_t* s_rb,
                                                uint32_t* out) {
    const uint32_t lane = threadIdx.x;
    // total row entries = last exclusive offset + last count
    const uint32_t total = O_rows[(size_t)gy * nseg_rows - 1] + M_rows_last[0];
    for (uint32_t y = lane; y <= gy; y += 64) s_rb[y] = row_begin(O_rows, nseg_rows, y, gy, total);
    __syncthreads();
    uint32_t carry = 0;
    for (uint32_t y0 = 0; y0 < gy; y0 += 64) {
        const uint32_t y = y0 + lane;
        const uint32_t nk = y < gy ? (s_rb[y + 1] - s_rb[y] + kTileSeg - 1) / kTileSeg : 0u;
        const uint32_t incl = wave_incl_scan(nk);
        if (y < gy) s_sb[y + 1] = carry + incl;
        carry += __shfl(incl, 63, 64);
    }
    if (lane == 0) s_sb[0] = 0u;
    __syncthreads();
    if (out)
        for (uint32_t y = lane; y <= gy; y += 64) out[y] = s_sb[y];
}

__device__ __forceinline__ TileSeg find_seg_lds(uint32_t b, uint32_t gy, const uint32_t* s_sb, const uint32_t* s_rb) {
    TileSeg S{};
    if (b >= s_sb[gy]) return S;
    uint32_t lo = 0, hi = gy;  // largest y with segbase[y] <= b
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_sb[mid] <= b) lo = mid;
        else hi = mid;
    }
    S.on = true;
    S.y = lo;
    S.k = b - s_sb[lo];
    S.nk = s_sb[lo + 1] - s_sb[lo];
    S.e0 = s_rb[lo] + S.k * kTileSeg;
    S.e1 = min(s_rb[lo + 1], S.e0 + kTileSeg);
    return S;
}

// The tile-pass kernels run a fixed grid that walks the actual segments
// (segbase[gy], known on the device only).  Blocks are dealt round-robin over
// the 8 XCDs; XCD x takes the x-th eighth of the segments, and its blocks
// walk that range in lockstep strides, so the rows an XCD works on at any
// moment are one or two, and their point-list region (~1 MB at C3) stays in
// that XCD's L2 while the partial lines written by successive segments fill
// up (write-back of whole lines instead of ~16-B pieces).
#ifndef GSR_TILE_BLOCKS
#define GSR_TILE_BLOCKS (8 * 1024)
#endif
constexpr int kTileBlocks = GSR_TILE_BLOCKS;

template <typename F>
__device__ __forceinline__ void for_xcd_segments(uint32_t n, F&& f) {
    const uint32_t xcd = blockIdx.x % 8u, slot = blockIdx.x / 8u, nslots = gridDim.x / 8u;
    const uint32_t lo = (uint32_t)(((unsigned long long)n * xcd) / 8u);
    const uint32_t hi = (uint32_t)(((unsigned long long)n * (xcd + 1u)) / 8u);
    for (uint32_t l = lo + slot; l < hi; l += nslots) f(l);
}

__global__ void __launch_bounds__(64)
    tiles_count_kernel(uint32_t gx, uint32_t gy, int nseg_rows, const uint32_t* __restrict__ O_rows,
                       const uint32_t* __restrict__ M_rows_last, uint32_t* __restrict__ segbase,
                       const uint2* __restrict__ rows, uint32_t* __restrict__ M) {
    // (segbase: written here by block 0 for the kernels after; every block builds its own copy in LDS)
    extern __shared__ unsigned long long s_dyn[];  // [gx] counts, then the segment table (2 x [gy + 1])
    uint32_t* s_cnt = reinterpret_cast<uint32_t*>(s_dyn);
    uint32_t* s_sb = s_cnt + gx;
    uint32_t* s_rb = s_sb + gy + 1;
    const int lane = threadIdx.x;
    build_seg_table(gy, nseg_rows, O_rows, M_rows_last, s_sb, s_rb, blockIdx.x == 0 ? segbase : nullptr);
    for_xcd_segments(s_sb[gy], [&](uint32_t l) {
        const TileSeg S = find_seg_lds(l, gy, s_sb, s_rb);
        __syncthreads();  // previous segment's counts read out
        for (uint32_t x = lane; x < gx; x += 64) s_cnt[x] = 0u;
        __syncthreads();
        for (uint32_t e = S.e0 + lane; e < S.e1; e += 64) {
            const uint32_t sp = rows[e].y;
            for (uint32_t x = sp & 0xffffu; x <= (sp >> 16); x++) atomicAdd(&s_cnt[x], 1u);
        }
        __syncthreads();
        const size_t base = (size_t)gx * s_sb[S.y];
        for (uint32_t x = lane; x < gx; x += 64) M[base + (size_t)x * S.nk + S.k] = s_cnt[x];
    });
}

#ifndef GSR_TILES_EMIT_SORTED
#define GSR_TILES_EMIT_SORTED 3  // 3: tiles_emit_coop_kernel (default, grids <= 256 tiles wide), 2: tiles_emit_wide_kernel
#endif

// tiles_emit_sorted with chunks of 64 NPL entries (NPL per lane: entries
// c0 + 64 h + lane, h < NPL, with a mask plane each), so the per-chunk work —
// the bucket scan of chunk_bases, the mask clearing and the barriers — is
// shared by NPL times the instances.  A bucket's plane-h entries rank after
// all of its entries in planes < h (they precede them in the row), so the
// slots and values are those of the 64-entry kernel.
#ifndef GSR_EMIT_PLANES
#define GSR_EMIT_PLANES 2
#endif
constexpr int kEmitPlanes = GSR_EMIT_PLANES;
#ifndef GSR_EMIT_CAP
#define GSR_EMIT_CAP (512 * GSR_EMIT_PLANES)
#endif
constexpr int kEmitCapW = GSR_EMIT_CAP;  // instances staged per chunk (more: direct writes)

template <int NPL>
__global__ void __launch_bounds__(64)
    tiles_emit_wide_kernel(uint32_t gx, uint32_t gy, int nseg_rows, const uint32_t* __restrict__ O_rows,
                           const uint32_t* __restrict__ M_rows_last, const uint32_t* __restrict__ segbase,
                           const uint2* __restrict__ rows, const uint32_t* __restrict__ O,
                           uint32_t* __restrict__ point_list) {
    constexpr uint32_t kCap = kEmitCapW;
    // LDS: NPL x [gx] masks, [gx] running slots, [gx] chunk offsets, [gx] write bases, kCap ids and tiles
    extern __shared__ unsigned long long s_dyn[];
    unsigned long long* s_cov = s_dyn;
    uint32_t* s_run = reinterpret_cast<uint32_t*>(s_dyn + NPL * gx);
    uint32_t* s_off = s_run + gx;
    uint32_t* s_base = s_off + gx;
    uint32_t* s_id = s_base + gx;
    uint16_t* s_x = reinterpret_cast<uint16_t*>(s_id + kCap);
    const int lane = threadIdx.x;
    const uint32_t total = O_rows[(size_t)gy * nseg_rows - 1] + M_rows_last[0];
    const unsigned long long bit = 1ull << lane, below = bit - 1ull;
    for_xcd_segments(segbase[gy], [&](uint32_t l) {
        const TileSeg S = find_seg(l, gy, segbase, O_rows, nseg_rows, total);
        const size_t base = (size_t)gx * segbase[S.y];
        __syncthreads();  // previous segment done with the LDS
        for (uint32_t x = lane; x < gx; x += 64) s_run[x] = O[base + (size_t)x * S.nk + S.k];
        for (uint32_t x = lane; x < NPL * gx; x += 64) s_cov[x] = 0ull;
        __syncthreads();
        for (uint32_t c0 = S.e0; c0 < S.e1; c0 += 64 * NPL) {
            bool on[NPL];
            uint32_t id[NPL], lo[NPL], hi[NPL];
#pragma unroll
            for (int h = 0; h < NPL; h++) {
                const uint32_t e = c0 + 64 * h + lane;
                on[h] = e < S.e1;
                const uint2 ent = on[h] ? rows[e] : make_uint2(0u, 1u);  // empty span when off
                id[h] = ent.x;
                lo[h] = ent.y & 0xffffu;
                hi[h] = on[h] ? (ent.y >> 16) : 0u;
            }
#pragma unroll
            for (int h = 0; h < NPL; h++)
                for (uint32_t x = lo[h]; on[h] && x <= hi[h]; x++) atomicOr(&s_cov[h * gx + x], bit);
            __syncthreads();
            // per tile: count (all planes), base among the chunk's instances, write base (chunk_bases)
            uint32_t carry = 0;
            for (uint32_t b0 = 0; b0 < gx; b0 += 64) {
                const uint32_t b = b0 + lane;
                uint32_t cnt = 0;
                if (b < gx) {
#pragma unroll
                    for (int h = 0; h < NPL; h++) cnt += (uint32_t)__popcll(s_cov[h * gx + b]);
                }
                const uint32_t incl = wave_incl_scan(cnt);
                if (b < gx) {
                    const uint32_t o = carry + incl - cnt;
                    const uint32_t r = s_run[b];
                    s_off[b] = o;
                    s_base[b] = r - o;
                    s_run[b] = r + cnt;
                }
                carry += __shfl(incl, 63, 64);
            }
            __syncthreads();
            // rank of plane h's entry at tile x: the chunk's earlier planes, then the lower lanes
            auto rank = [&](int h, uint32_t x) {
                uint32_t r = (uint32_t)__popcll(s_cov[h * gx + x] & below);
                for (int k = 0; k < h; k++) r += (uint32_t)__popcll(s_cov[k * gx + x]);
                return r;
            };
            if (carry <= kCap) {
#pragma unroll
                for (int h = 0; h < NPL; h++)
                    for (uint32_t x = lo[h]; on[h] && x <= hi[h]; x++) {
                        const uint32_t p = s_off[x] + rank(h, x);
                        s_id[p] = id[h];
                        s_x[p] = (uint16_t)x;
                    }
                __syncthreads();
                for (uint32_t p = lane; p < carry; p += 64) point_list[s_base[s_x[p]] + p] = s_id[p];
            } else {
#pragma unroll
                for (int h = 0; h < NPL; h++)
                    for (uint32_t x = lo[h]; on[h] && x <= hi[h]; x++)
                        point_list[s_base[x] + s_off[x] + rank(h, x)] = id[h];
            }
            __syncthreads();
            for (uint32_t x = lane; x < NPL * gx; x += 64) s_cov[x] = 0ull;
            __syncthreads();
        }
    });
}

// tiles_emit with whole-workgroup segments (round 3).  The single-wave
// emission runs ~1000 blocks per XCD, so every segment of the XCD's share is
// in flight at once and the point-list region being written (~6.5 MB per XCD
// at C3) exceeds its 4 MB L2: partial lines leave the L2 before they are
// complete (WRITE_SIZE 158 MB per C3 launch against 52 MB of point list;
// with 128 single-wave blocks per XCD the writes fall to 53 MB, but then the
// launch is latency-bound).  Here NW waves work one segment together, its
// 64 NW NPL entries ranked at once (entry c0 + 64 (NPL w + h) + lane is wave
// w's plane h; a tile's rank counts the planes before, then the lower
// lanes), staged in LDS by (tile, rank) and written by consecutive lanes; and
// kCoopBlocks / 8 blocks per XCD walk its segments in lockstep strides, so
// the region in flight is a row or two.  Same slots, same values.
#ifndef GSR_COOP_BLOCKS
#define GSR_COOP_BLOCKS (8 * 128)
#endif
#ifndef GSR_COOP_CAP
#define GSR_COOP_CAP 2048
#endif
constexpr int kCoopBlocks = GSR_COOP_BLOCKS;
constexpr int kCoopWaves = 4, kCoopPlanes = 2;  // 512 entries per segment: one round
static_assert(64 * kCoopWaves * kCoopPlanes == kTileSeg, "a tile-pass segment is one coop round");
constexpr uint32_t kCoopCap = GSR_COOP_CAP;     // instances staged per round (more: direct writes)
constexpr int kCoopMaxGx = 64 * kCoopWaves;     // one running slot per thread; wider grids keep tiles_emit_wide_kernel
size_t coop_lds_bytes(uint32_t gx, uint32_t gy) {
    constexpr int kPl = kCoopWaves * kCoopPlanes;
    return (size_t)2 * 8 * kPl * gx + (size_t)4 * (3 + kPl) * gx + (size_t)6 * kCoopCap + (size_t)8 * (gy + 1);
}

// One segment's inputs, requested a segment ahead: its entries (NPL per lane)
// and its running slots (one tile per thread).
template <int NW, int NPL>
struct CoopSeg {
    TileSeg S;
    uint32_t run;
    uint2 ent[NPL];
};
template <int NW, int NPL>
__device__ __forceinline__ CoopSeg<NW, NPL> coop_fetch(uint32_t l, uint32_t hi, uint32_t gx, uint32_t gy,
                                                       const uint32_t* s_sb, const uint32_t* s_rb, const uint2* rows,
                                                       const uint32_t* O) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    CoopSeg<NW, NPL> c;
    c.S = l < hi ? find_seg_lds(l, gy, s_sb, s_rb) : TileSeg{};
    c.run = 0u;
    if (c.S.on && (uint32_t)tid < gx) c.run = O[(size_t)gx * s_sb[c.S.y] + (size_t)tid * c.S.nk + c.S.k];
#pragma unroll
    for (int h = 0; h < NPL; h++) {
        const uint32_t e = c.S.e0 + 64 * (NPL * wave + h) + lane;
        c.ent[h] = c.S.on && e < c.S.e1 ? rows[e] : make_uint2(0u, 1u);  // (lo 1 > hi 0: empty span)
    }
    return c;
}

// tiles_emit with whole-workgroup segments (round 3).  The single-wave
// emission runs ~1000 blocks per XCD, so every segment of the XCD's share is
// in flight at once and the point-list region being written (~6.5 MB per XCD
// at C3) exceeds its 4 MB L2: partial lines leave the L2 before they are
// complete (WRITE_SIZE 158 MB per C3 launch against 52 MB of point list;
// with 128 single-wave blocks per XCD the writes fall to 53 MB, but then the
// launch is latency-bound).  Here NW waves work one segment (one round of
// 64 NW NPL entries) together: entry e0 + 64 (NPL w + h) + lane is wave w's
// plane h, and a tile's rank counts the planes before, then the lower lanes;
// the round's instances are staged in LDS by (tile, rank) and written by
// consecutive lanes; kCoopBlocks / 8 blocks per XCD walk its segments in
// lockstep strides, so the region in flight is a row or two.  Same slots,
// same values.  Per segment the block is a chain of dependent steps, so:
// the segment table sits in LDS (find_seg_lds); the next segment's entries
// and running slots are requested before this one is worked; and the mask
// planes are double-buffered (a buffer is cleared while the round's ids are
// written out, and reused two segments later), which leaves three barriers
// per segment.
template <int NW, int NPL>
__global__ void __launch_bounds__(64 * NW)
    tiles_emit_coop_kernel(uint32_t gx, uint32_t gy, int nseg_rows, const uint32_t* __restrict__ O_rows,
                           const uint32_t* __restrict__ M_rows_last, const uint32_t* __restrict__ segbase,
                           const uint2* __restrict__ rows, const uint32_t* __restrict__ O,
                           uint32_t* __restrict__ point_list, uint2* __restrict__ ranges) {
    constexpr int kPl = NW * NPL;
    constexpr int kThreads = 64 * NW;
    // LDS: 2 x kPl x [gx] masks; [gx] running slots, chunk offsets, write bases; kPl x [gx] plane prefixes;
    // kCoopCap ids and tiles; the segment table
    extern __shared__ unsigned long long s_dyn[];
    unsigned long long* s_cov2 = s_dyn;
    uint32_t* s_run = reinterpret_cast<uint32_t*>(s_dyn + 2 * kPl * gx);
    uint32_t* s_off = s_run + gx;
    uint32_t* s_base = s_off + gx;
    uint32_t* s_pl = s_base + gx;
    uint32_t* s_id = s_pl + kPl * gx;
    uint16_t* s_x = reinterpret_cast<uint16_t*>(s_id + kCoopCap);
    uint32_t* s_sb = reinterpret_cast<uint32_t*>(s_x + kCoopCap);
    uint32_t* s_rb = s_sb + gy + 1;
    __shared__ uint32_t s_carry;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned long long bit = 1ull << lane, below = bit - 1ull;
    for (uint32_t x = tid; x < 2 * kPl * gx; x += kThreads) s_cov2[x] = 0ull;
    stage_seg_table(gy, nseg_rows, O_rows, M_rows_last, segbase, s_sb, s_rb);  // (ends with a barrier)
    const uint32_t n = s_sb[gy];
    // the tile ranges (list_ranges_kernel's work) depend only on the scan this kernel starts from: every
    // block writes a share of them first, so they need no launch of their own
    for (uint32_t t = blockIdx.x * kThreads + tid; t < gx * gy; t += gridDim.x * kThreads) {
        const uint32_t y = t / gx, x = t - y * gx;
        const uint32_t nk = s_sb[y + 1] - s_sb[y];
        uint2 r = make_uint2(0u, 0u);
        if (nk) {
            const size_t base = (size_t)gx * s_sb[y];
            const uint32_t b = O[base + (size_t)x * nk], e = O[base + (size_t)(x + 1) * nk];
            if (e > b) r = make_uint2(b, e);  // empty tiles stay (0, 0) as in the reference
        }
        ranges[t] = r;
    }
    const uint32_t xcd = blockIdx.x % 8u, slot0 = blockIdx.x / 8u, nslots = gridDim.x / 8u;
    const uint32_t lo_l = (uint32_t)(((unsigned long long)n * xcd) / 8u);
    const uint32_t hi_l = (uint32_t)(((unsigned long long)n * (xcd + 1u)) / 8u);
    uint32_t l = lo_l + slot0, buf = 0;
    CoopSeg<NW, NPL> cur = coop_fetch<NW, NPL>(l, hi_l, gx, gy, s_sb, s_rb, rows, O);
    while (cur.S.on) {
        const CoopSeg<NW, NPL> nxt = coop_fetch<NW, NPL>(l + nslots, hi_l, gx, gy, s_sb, s_rb, rows, O);
        unsigned long long* s_cov = s_cov2 + buf * kPl * gx;
        // (s_run is read only by wave 0's scan below, after the barrier that ends the previous segment's writes)
        if ((uint32_t)tid < gx) s_run[tid] = cur.run;
        uint32_t id[NPL], lo[NPL], hi[NPL];
#pragma unroll
        for (int h = 0; h < NPL; h++) {
            id[h] = cur.ent[h].x;
            lo[h] = cur.ent[h].y & 0xffffu;
            hi[h] = cur.ent[h].y >> 16;
            unsigned long long* cov = s_cov + (NPL * wave + h) * gx;
            for (uint32_t x = lo[h]; x <= hi[h]; x++) atomicOr(&cov[x], bit);
        }
        __syncthreads();
        // per tile (wave 0): plane prefixes, count, base among the round's instances, write base
        if (wave == 0) {
            uint32_t carry = 0;
            for (uint32_t b0 = 0; b0 < gx; b0 += 64) {
                const uint32_t b = b0 + lane;
                uint32_t cnt = 0;
                if (b < gx) {
#pragma unroll
                    for (int p = 0; p < kPl; p++) {
                        s_pl[p * gx + b] = cnt;
                        cnt += (uint32_t)__popcll(s_cov[p * gx + b]);
                    }
                }
                const uint32_t incl = wave_incl_scan(cnt);
                if (b < gx) {
                    const uint32_t o = carry + incl - cnt;
                    s_off[b] = o;
                    s_base[b] = s_run[b] - o;
                }
                carry += __shfl(incl, 63, 64);
            }
            if (lane == 0) s_carry = carry;
        }
        __syncthreads();
        const uint32_t carry = s_carry;
        auto slot = [&](int p, uint32_t x) {
            return s_off[x] + s_pl[p * gx + x] + (uint32_t)__popcll(s_cov[p * gx + x] & below);
        };
        if (carry <= kCoopCap) {
#pragma unroll
            for (int h = 0; h < NPL; h++) {
                const int p = NPL * wave + h;
                for (uint32_t x = lo[h]; x <= hi[h]; x++) {
                    const uint32_t q = slot(p, x);
                    s_id[q] = id[h];
                    s_x[q] = (uint16_t)x;
                }
            }
            __syncthreads();
            for (uint32_t x = tid; x < kPl * gx; x += kThreads) s_cov[x] = 0ull;
            for (uint32_t q = tid; q < carry; q += kThreads) point_list[s_base[s_x[q]] + q] = s_id[q];
        } else {
#pragma unroll
            for (int h = 0; h < NPL; h++) {
                const int p = NPL * wave + h;
                for (uint32_t x = lo[h]; x <= hi[h]; x++) point_list[s_base[x] + slot(p, x)] = id[h];
            }
            __syncthreads();
            for (uint32_t x = tid; x < kPl * gx; x += kThreads) s_cov[x] = 0ull;
        }
        // The next segment's mask atomics use the other buffer (cleared one segment ago, before this
        // segment's first barrier); its scan rewrites s_off / s_base / s_pl / s_carry only after its
        // first barrier, which every wave reaches after finishing the writes above.
        cur = nxt;
        l += nslots;
        buf ^= 1u;
    }
}

__global__ void __launch_bounds__(256)
    list_ranges_kernel(uint32_t gx, uint32_t gy, const uint32_t* __restrict__ segbase, const uint32_t* __restrict__ O,
                       uint2* __restrict__ ranges) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= gx * gy) return;
    const uint32_t y = t / gx, x = t - y * gx;
    const uint32_t nk = segbase[y + 1] - segbase[y];
    uint2 r = make_uint2(0u, 0u);
    if (nk) {
        const size_t base = (size_t)gx * segbase[y];
        const uint32_t b = O[base + (size_t)x * nk], e = O[base + (size_t)(x + 1) * nk];
        if (e > b) r = make_uint2(b, e);  // empty tiles stay (0, 0) as in the reference
    }
    ranges[t] = r;
}

hipError_t launch_list_binning(const FwdParams& p, const GeomState& gs, const int* radii, const BinningState& bs,
                               const TileState& ts, int K, hipStream_t stream) {
    const uint32_t gx = p.grid_x, gy = p.grid_y;
    const ListLayout& L = bs.lists;
    hipError_t e;
    // rows pass
    const uint32_t row_blocks = (uint32_t)((L.nseg_rows + kRowWaves - 1) / kRowWaves);
    hipLaunchKernelGGL(rows_count_kernel, dim3(row_blocks), dim3(64 * kRowWaves), 4 * gy * kRowWaves, stream, p.P, L.nseg_rows, L.rowseg, gy,
                       p.cull_pad, gs.order, (const uint4*)gs.foot, bs.rows_count, bs.qrec);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    uint32_t* sums = reinterpret_cast<uint32_t*>(bs.list_tmp);
    const size_t nrows = (size_t)gy * L.nseg_rows;
    // (rows_off holds gy * nseg_rows words: the scan writes the total at [n] only up to n - 1 here)
    if ((e = launch_scan_excl(bs.rows_count, bs.rows_off, nrows - 1, (uint32_t)(nrows - 1), nullptr, 1u, sums,
                              stream)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(rows_emit_kernel, dim3(row_blocks), dim3(64 * kRowWaves), 24 * gy * kRowWaves, stream, p.P, L.nseg_rows, L.rowseg, gy,
                       p.cull_pad, gs.order, (const uint4*)gs.foot, bs.rows_off, bs.qrec, bs.rows);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // tiles pass
    const uint32_t* last = bs.rows_count + (size_t)gy * L.nseg_rows - 1;
    hipLaunchKernelGGL(tiles_count_kernel, dim3(kTileBlocks), dim3(64), 4 * gx + 8 * (gy + 1), stream, gx, gy, L.nseg_rows,
                       bs.rows_off, last, bs.segbase, bs.rows, bs.tiles_count);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // counts of the live segments only: gx * segbase[gy] of them (tiles_count_kernel writes every one)
    if ((e = launch_scan_excl(bs.tiles_count, bs.tiles_off, (size_t)gx * L.nseg_tiles_max, 0u, bs.segbase + gy, gx,
                              sums, stream)) != hipSuccess)
        return e;
    if (GSR_TILES_EMIT_SORTED == 3 && gx <= (uint32_t)kCoopMaxGx && coop_lds_bytes(gx, gy) <= 65536) {
        // (the coop kernel writes the tile ranges too)
        hipLaunchKernelGGL((tiles_emit_coop_kernel<kCoopWaves, kCoopPlanes>), dim3(kCoopBlocks), dim3(64 * kCoopWaves),
                           coop_lds_bytes(gx, gy), stream, gx, gy, L.nseg_rows, bs.rows_off, last, bs.segbase, bs.rows,
                           bs.tiles_off, bs.point_list, ts.ranges);
    } else {
        hipLaunchKernelGGL(tiles_emit_wide_kernel<kEmitPlanes>, dim3(kTileBlocks), dim3(64),
                           (8 * kEmitPlanes + 12) * gx + 6 * kEmitCapW, stream, gx,
                           gy, L.nseg_rows, bs.rows_off, last, bs.segbase, bs.rows, bs.tiles_off, bs.point_list);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL(list_ranges_kernel, dim3((gx * gy + 255) / 256), dim3(256), 0, stream, gx, gy, bs.segbase,
                           bs.tiles_off, ts.ranges);
    }
    (void)K;
    return hipGetLastError();
}

}  // namespace gsr
