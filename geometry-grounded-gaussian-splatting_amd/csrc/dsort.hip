// dsort.hip — the depth order of the Gaussians (a stable sort of the P depth
// bit patterns, values = Gaussian index) as a 4-pass onesweep LSD radix sort
// on gfx950.
//
// Replaces the reference's depth part of the (tile | depth) key sort
// (CR/rasterizer_impl.cu:403-412; binning.hip header: the Gaussians in
// (depth bits, index) order, then stable counting passes per tile).  rocPRIM's
// onesweep sort (GSR_OPT_ROCPRIM_DSORT) clears its look-back state with a
// memset per pass: at P = 1M the depth order took 16 launches, 9 of them
// fills (~45 us of 0.12 ms).  Here: one zeroing kernel, one histogram kernel
// and one kernel per 8-bit digit, and the look-back state of all four passes
// is zeroed once.
//
// Pass kernel (one 1024-lane workgroup per tile of 6144 keys, 12288 above 2M
// keys — 16 waves per CU
// for latency; tiles numbered in the order workgroups start, by an atomic
// counter, so every look-back target is running or done):
//  1. each wave ranks its 384 / 768 keys (6 / 12 per lane, position i*64 + lane) by
//     digit with 8 ballots per item (peer lanes), a per-wave digit counter in
//     LDS giving the stable rank among the wave's earlier items;
//  2. per digit (lanes 0-255): the wave counts combined into the tile's
//     digit counts, published at once with flag AGG, and the in-tile prefix;
//  3. keys and values go to LDS in tile-sorted order;
//  4. the decoupled look-back over the preceding tiles (4 lanes per digit,
//     32 status words each per round: 128 tiles per round, consumed newest
//     first up to the first INC or not-ready word)
//     gives the tile's exclusive prefix, published with flag INC, and the
//     keys are written out striped: consecutive lanes write consecutive
//     output positions of a digit run.
// Stability: within a digit, tile order, then wave, item and lane order,
// which is position order; so the result is the (key, index) order of the
// reference's stable sort.
#include <type_traits>

#include "gsr_kernels.h"

namespace gsr {

#ifndef GSR_DS_THREADS
#define GSR_DS_THREADS 1024
#endif
#ifndef GSR_DS_ITEMS
#define GSR_DS_ITEMS 6  // keys per lane up to kDsBigP keys (round 3: 4 -> 8, C5 depth order 0.294 -> 0.222 ms; round 5: 8 -> 6 at C3, 123 -> 163 tiles for 256 CUs: 0.0805 -> 0.0774 ms; 4: 0.083, 512 lanes x 8: 0.088)
#endif
#ifndef GSR_DS_ITEMS_BIG
#define GSR_DS_ITEMS_BIG 12  // above kDsBigP (C5: 0.221 -> 0.188 ms; 12 at C3: 0.080 -> 0.088, 16: 0.207 / 0.098)
#endif
constexpr int kDsThreads = GSR_DS_THREADS;
constexpr int kDsWaves = kDsThreads / 64;
constexpr int kDsItems = GSR_DS_ITEMS, kDsItemsBig = GSR_DS_ITEMS_BIG;
constexpr int kDsBigP = 2000000;
// keys per lane for P keys: fewer, larger tiles for large P (fewer look-back steps; one block per CU)
static int dsort_items(int P) { return P > kDsBigP ? kDsItemsBig : kDsItems; }
static_assert(kDsThreads >= 256 && kDsThreads % 64 == 0, "a digit per lane of the first 256 lanes");
constexpr int kDsLook = 32;                     // status words read per look-back round
constexpr uint32_t kDsAgg = 1u << 30, kDsInc = 2u << 30, kDsVal = (1u << 30) - 1u;

struct DsortState {
    uint32_t* keys_alt;
    uint32_t* vals_alt;
    uint32_t* hist;    // [4][256] digit counts of the whole input
    uint32_t* ctr;     // [4] tile counters
    uint32_t* status;  // [4][tiles][256] flag | count
    int tiles;
};

static int dsort_tiles(int P) {
    const int tile = kDsThreads * dsort_items(P);
    return (P + tile - 1) / tile;
}

static DsortState carve_dsort(void* base, int P) {
    Carver c(base);
    DsortState s;
    s.tiles = dsort_tiles(P);
    s.keys_alt = c.take<uint32_t>(P);
    s.vals_alt = c.take<uint32_t>(P);
    s.hist = c.take<uint32_t>(4 * 256);
    s.ctr = c.take<uint32_t>(64);
    s.status = c.take<uint32_t>((size_t)4 * s.tiles * 256);
    return s;
}

// the words the preprocess zeroes before the histogram (hist, counters, status)
void dsort_zero_region(void* base, int P, uint32_t** first, size_t* words) {
    DsortState s = carve_dsort(base, P);
    *first = s.hist;
    *words = (size_t)(s.status + (size_t)4 * s.tiles * 256 - s.hist);
}

size_t dsort_temp_bytes(int P) {
    DsortState s = carve_dsort(nullptr, P);
    return reinterpret_cast<size_t>(s.status + (size_t)4 * s.tiles * 256) + 256;
}

// zero the histogram, the tile counters and every pass's status words
__global__ void __launch_bounds__(256) dsort_zero_kernel(DsortState s) {
    const size_t n = (size_t)4 * s.tiles * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s.status[i] = 0u;
    if (blockIdx.x == 0) {
        for (int i = threadIdx.x; i < 4 * 256; i += 256) s.hist[i] = 0u;
        if (threadIdx.x < 4) s.ctr[threadIdx.x] = 0u;
    }
}

// the four digit histograms in one read of the keys
__global__ void __launch_bounds__(256) dsort_hist_kernel(const uint32_t* __restrict__ keys, int P, DsortState s) {
    __shared__ uint32_t h[4][256];
    for (int i = threadIdx.x; i < 4 * 256; i += 256) (&h[0][0])[i] = 0u;
    __syncthreads();
    const int per = (P + gridDim.x - 1) / gridDim.x;
    const int i0 = blockIdx.x * per, i1 = min(P, i0 + per);
    for (int i = i0 + threadIdx.x; i < i1; i += 256) {
        const uint32_t k = keys[i];
        atomicAdd(&h[0][k & 255u], 1u);
        atomicAdd(&h[1][(k >> 8) & 255u], 1u);
        atomicAdd(&h[2][(k >> 16) & 255u], 1u);
        atomicAdd(&h[3][k >> 24], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * 256; i += 256) {
        const uint32_t v = (&h[0][0])[i];
        if (v) atomicAdd(&s.hist[i], v);
    }
}

// K (the sum of tiles touched, into a word the preprocess zeroed) and, with
// `hist`, the four digit histograms of the depth keys: one read of both
// arrays, replacing a 2-kernel reduce plus this file's zero and histogram
// kernels on the render path.
__global__ void __launch_bounds__(256) count_k_hist_kernel(int P, const uint32_t* __restrict__ tiles_touched,
                                                           const uint32_t* __restrict__ keys, uint32_t* K,
                                                           int hist, DsortState s) {
    __shared__ uint32_t h[4][256];
    __shared__ uint32_t s_sum[4];
    if (hist)
        for (int i = threadIdx.x; i < 4 * 256; i += 256) (&h[0][0])[i] = 0u;
    __syncthreads();
    const int per = (P + gridDim.x - 1) / gridDim.x;
    const int i0 = blockIdx.x * per, i1 = min(P, i0 + per);
    uint32_t sum = 0;
    for (int i = i0 + threadIdx.x; i < i1; i += 256) {
        sum += tiles_touched[i];
        if (hist) {
            const uint32_t k = keys[i];
            atomicAdd(&h[0][k & 255u], 1u);
            atomicAdd(&h[1][(k >> 8) & 255u], 1u);
            atomicAdd(&h[2][(k >> 16) & 255u], 1u);
            atomicAdd(&h[3][k >> 24], 1u);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(K, s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3]);
    if (hist)
        for (int i = threadIdx.x; i < 4 * 256; i += 256) {
            const uint32_t v = (&h[0][0])[i];
            if (v) atomicAdd(&s.hist[i], v);
        }
}

hipError_t launch_count_k_hist(const GeomState& gs, int P, bool hist, hipStream_t stream) {
    if (P == 0) return hipMemsetAsync(gs.offsets_K, 0, sizeof(uint32_t), stream);
    DsortState s = carve_dsort(gs.dsort_tmp, P);
#ifndef GSR_KHIST_BLOCKS
#define GSR_KHIST_BLOCKS 512  // round 3: 256 -> 512 blocks, C5 count + histograms 47 -> 36 us (1024: 39)
#endif
    hipLaunchKernelGGL(count_k_hist_kernel, dim3(min(GSR_KHIST_BLOCKS, (P + 4095) / 4096)), dim3(256), 0, stream, P,
                       gs.tiles_touched, reinterpret_cast<const uint32_t*>(gs.depths), gs.offsets_K, hist ? 1 : 0, s);
    return hipGetLastError();
}

__device__ __forceinline__ uint32_t ds_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ds_store(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// exclusive scan of one value per lane over the first 256 lanes of the
// block (every lane calls it: it holds a barrier); s_w: 4 words
__device__ __forceinline__ uint32_t ds_digit_excl(uint32_t v, uint32_t* s_w) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63 && wave < 4) s_w[wave] = x;
    __syncthreads();
    uint32_t before = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) before += w < wave ? s_w[w] : 0u;
    return before + x - v;
}

template <int PASS, int ITEMS>
__global__ void __launch_bounds__(kDsThreads) dsort_pass_kernel(const uint32_t* __restrict__ keys_in,
                                                                const uint32_t* __restrict__ vals_in, int P,
                                                                DsortState s, uint32_t* __restrict__ keys_out,
                                                                uint32_t* __restrict__ vals_out) {
    constexpr int kShift = 8 * PASS;
    constexpr int kItems = ITEMS, kTile = kDsThreads * ITEMS;
    __shared__ uint32_t s_wcnt[kDsWaves][256];  // per-wave digit counters, then the waves' exclusive offsets
    __shared__ uint32_t s_goff[256];     // digit start in the output: global prefix + preceding tiles
    __shared__ uint32_t s_pre[256];      // in-tile exclusive digit prefix
    __shared__ uint32_t s_cnt[256], s_excl[256];  // the tile's digit counts; the preceding tiles' sums
    __shared__ uint32_t s_keys[kTile], s_vals[kTile];
    __shared__ uint32_t s_w[4];
    __shared__ uint32_t s_tile;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(&s.ctr[PASS], 1u);
    for (int i = tid; i < kDsWaves * 256; i += kDsThreads) (&s_wcnt[0][0])[i] = 0u;
    __syncthreads();
    const int tile = (int)s_tile;
    const int base = tile * kTile + wave * (kTile / kDsWaves);

    uint32_t k[kItems], v[kItems], r[kItems];
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        const int p = base + i * 64 + lane;
        const bool ok = p < P;
        k[i] = ok ? keys_in[p] : 0xffffffffu;  // padding: digit 255, after every real key of the tile
        v[i] = PASS == 0 ? (uint32_t)p : (ok ? vals_in[p] : 0u);
    }
    // 1. stable rank of each item among the wave's keys of its digit
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        const uint32_t d = (k[i] >> kShift) & 255u;
        uint64_t peers = ~0ull;
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint64_t bal = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? bal : ~bal;
        }
        const uint32_t below = (uint32_t)__popcll(peers & lt);
        const uint32_t c0 = s_wcnt[wave][d];
        r[i] = c0 + below;
        if ((peers & lt) == 0ull) s_wcnt[wave][d] = c0 + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // 2. per digit (lane d < 256): the tile's count, published at once (AGG), and the in-tile prefix
    const int d = tid & 255;
    const bool dl = tid < 256;
    uint32_t cnt = 0;
    uint32_t* st = s.status + ((size_t)PASS * s.tiles) * 256 + d;
    if (dl) {
        for (int w = 0; w < kDsWaves; w++) {
            const uint32_t c = s_wcnt[w][d];
            s_wcnt[w][d] = cnt;  // wave's exclusive offset within the digit
            cnt += c;
        }
        if (tile == s.tiles - 1 && d == 255) cnt -= (uint32_t)(s.tiles * kTile - P);  // not the padding keys
        ds_store(st + (size_t)tile * 256, (tile == 0 ? kDsInc : kDsAgg) | cnt);
    }
    // (digit 255's count, with or without the padding, enters no prefix)
    const uint32_t pre = ds_digit_excl(cnt, s_w);
    if (dl) s_pre[d] = pre;
    __syncthreads();
    // 3. keys and values to LDS in tile-sorted order (while the preceding tiles publish)
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        const uint32_t dd = (k[i] >> kShift) & 255u;
        const uint32_t rank = s_pre[dd] + s_wcnt[wave][dd] + r[i];
        s_keys[rank] = k[i];
        s_vals[rank] = v[i];
    }
    // 4. look-back over the preceding tiles for the digit's exclusive prefix: 4 lanes per digit
    //    (one quad of a wave), each reading kDsLook status words per round, so a round covers
    //    4 kDsLook tiles; the quad's parts are consumed newest first up to the first INC or
    //    not-ready word
    if (dl) s_cnt[d] = cnt;
    __syncthreads();
    for (int dq0 = 0; dq0 < 256; dq0 += kDsThreads / 4) {  // (one round with 1024 lanes)
        const int dq = dq0 + (tid >> 2), part = tid & 3, quad = lane & ~3;
        const uint32_t* sq = s.status + ((size_t)PASS * s.tiles) * 256 + dq;
        uint32_t excl = 0;
        int j = tile - 1;
        while (j >= 0) {
            const int j0 = j - part * kDsLook;
            uint32_t w[kDsLook];
#pragma unroll
            for (int q = 0; q < kDsLook; q++) w[q] = j0 - q >= 0 ? ds_load(sq + (size_t)(j0 - q) * 256) : kDsInc;
            uint32_t sum = 0;
            int used = 0, kind = 0;  // kind: 0 every word an aggregate, 1 INC reached, 2 a word not ready
#pragma unroll
            for (int q = 0; q < kDsLook; q++) {
                if (kind != 0) continue;
                if ((w[q] & ~kDsVal) == 0u) {
                    kind = 2;
                    continue;
                }
                sum += w[q] & kDsVal;
                used = q + 1;
                if ((w[q] & ~kDsVal) == kDsInc) kind = 1;
            }
            int consumed = 0, fin = 0, stop = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t sp = __shfl(sum, quad + q, 64);
                const int up = __shfl(used, quad + q, 64), kp = __shfl(kind, quad + q, 64);
                if (stop) continue;
                excl += sp;
                consumed += up;
                if (kp != 0) {
                    stop = 1;
                    fin = kp == 1;
                }
            }
            if (fin) break;
            j -= consumed;  // (0 when the newest word is not ready yet: read it again)
        }
        if (part == 0) {
            if (tile > 0) ds_store(s.status + ((size_t)PASS * s.tiles + tile) * 256 + dq, kDsInc | (excl + s_cnt[dq]));
            s_excl[dq] = excl;
        }
    }
    __syncthreads();
    // global digit start: exclusive scan of the whole-input histogram, plus the preceding tiles
    const uint32_t gpre = ds_digit_excl(dl ? s.hist[PASS * 256 + d] : 0u, s_w);
    if (dl) s_goff[d] = gpre + s_excl[d];
    __syncthreads();
    const int nvalid = min(kTile, P - tile * kTile);
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        const int rank = i * kDsThreads + tid;
        if (rank < nvalid) {
            const uint32_t key = s_keys[rank];
            const uint32_t d = (key >> kShift) & 255u;
            const uint32_t pos = s_goff[d] + (uint32_t)rank - s_pre[d];
            keys_out[pos] = key;
            vals_out[pos] = s_vals[rank];
        }
    }
}

hipError_t launch_dsort(const GeomState& gs, int P, bool prepared, hipStream_t stream) {
    if (P == 0) return hipSuccess;
    DsortState s = carve_dsort(gs.dsort_tmp, P);
    const uint32_t* keys = reinterpret_cast<const uint32_t*>(gs.depths);
    if (!prepared) {  // (render / sample paths: zeroed by the preprocess, histograms by count_k_hist_kernel)
        const int zblocks = min(1024, (4 * s.tiles * 256 + 255) / 256);
        hipLaunchKernelGGL(dsort_zero_kernel, dim3(zblocks), dim3(256), 0, stream, s);
        hipLaunchKernelGGL(dsort_hist_kernel, dim3(min(256, (P + 4095) / 4096)), dim3(256), 0, stream, keys, P, s);
    }
    const dim3 grid(s.tiles), block(kDsThreads);
    auto passes = [&](auto items_c) {
        constexpr int I = decltype(items_c)::value;
        hipLaunchKernelGGL((dsort_pass_kernel<0, I>), grid, block, 0, stream, keys, nullptr, P, s, s.keys_alt,
                           s.vals_alt);
        hipLaunchKernelGGL((dsort_pass_kernel<1, I>), grid, block, 0, stream, s.keys_alt, s.vals_alt, P, s,
                           gs.depth_keys_sorted, gs.order);
        hipLaunchKernelGGL((dsort_pass_kernel<2, I>), grid, block, 0, stream, gs.depth_keys_sorted, gs.order, P, s,
                           s.keys_alt, s.vals_alt);
        hipLaunchKernelGGL((dsort_pass_kernel<3, I>), grid, block, 0, stream, s.keys_alt, s.vals_alt, P, s,
                           gs.depth_keys_sorted, gs.order);
    };
    if (dsort_items(P) == kDsItems) passes(std::integral_constant<int, kDsItems>{});
    else passes(std::integral_constant<int, kDsItemsBig>{});
    return hipGetLastError();
}

}  // namespace gsr
