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
// of the vacancy transmittance (render_forward.cu:549-645).  The bisection
// only multiplies in the contributors a pixel actually blended (the others
// fail the same power/alpha test in every pass), so the composite records
// them as a per-pixel bitmask in LDS.  When the tile's contributing prefix
// fits (<= kResident records) it is staged into LDS once (48 B per record:
// w0, w1, w2) and every lane walks its own bitmask in increasing order —
// the lanes of a wave then do useful work on every step instead of idling
// on the ~2/3 of (pixel, contributor) pairs that fail the test (measured on
// C3 with GSR_OPT_RENDER_STATS).  Longer lists keep the wave-uniform walk
// with the records restaged per pass.
// Contraction is off for this file: every fma below is written out, so each
// template instance (plain, GSR_OPT_RENDER_STATS, the sample queries) rounds
// identically.
#ifndef GSR_FWD_CONTRACT
#define GSR_FWD_CONTRACT 0  // (development: 1 = contract(fast) outside the shared footprint helpers)
#endif
#if GSR_FWD_CONTRACT
#pragma clang fp contract(fast)
#else
#pragma clang fp contract(off)
#endif

#include <type_traits>

#include <algorithm>

#include "gsr_kernels.h"
#include "tiles.h"

namespace gsr {

#ifndef GSR_RESIDENT
#define GSR_RESIDENT 256
#endif
#ifndef GSR_BATCH
#define GSR_BATCH 128
#endif
constexpr int kResident = GSR_RESIDENT;  // LDS-resident contributing prefix (C3: every tile's max contributor <= 184)
constexpr int kMaskWords = kResident / 32;
constexpr int kBatch = GSR_BATCH;        // records per composite staging batch
// The median-depth walks take a step's two contributors' fields in the halves of packed register pairs.
// GSR_WALK_SOA = 1: the staged records are 12 SoA planes of kPlane floats and a field pair is two
// ds_read_b32 straight into the pair's halves (no moves; kPlane = kResident + 1 keeps the compiler from
// merging two fields of one record into a ds_read2); 0: the float4 records (three ds_read_b128 each) and
// the pairs built by moves.
#ifndef GSR_WALK_SOA
#define GSR_WALK_SOA 1
#endif
constexpr bool kWalkSoA = GSR_WALK_SOA;
#ifndef GSR_SAMPLE_WALK_SOA
#define GSR_SAMPLE_WALK_SOA GSR_WALK_SOA  // (the SAMPLE instance's own choice: A/B)
#endif
constexpr bool kSampleWalkSoA = GSR_SAMPLE_WALK_SOA;
constexpr int kPlane = kResident + 1;
constexpr int kPlanes = 12;  // x, y, conic a, b, c, opacity, plane x, y, |t|, rsigma, sc, ball
constexpr int kRecSlots = 3 * kPlane > 4 * kBatch ? 3 * kPlane : 4 * kBatch;
// the non-resident median-depth path stages kTilePixels-record chunks at offsets 0, kResident and
// 2 kResident of s_rec: a resident cache smaller than a chunk would overlap them and overrun s_rec
static_assert(kResident >= kTilePixels, "GSR_RESIDENT must be >= kTilePixels (256)");

struct RenderFwdArgs {
    const uint2* ranges;
    const uint32_t* point_list;
    const Splat* splats;
    int W, H;
    uint32_t grid_x, num_tiles;
    float focal_x, focal_y;
    const float* bg;
    uint32_t* n_contrib;
    float* dT_dtm;
    uint32_t* md_check;
    uint32_t* max_contrib;
    uint32_t* blend_mask;  // [tiles][kBlendWords] (render path)
    uint32_t* bwd_cost;    // [tiles] (render path) the backward's walk length, its LPT launch order's cost
    float* out_color;
    float* out_alpha;
    float* out_normal;
    float* out_mdepth;
    int passes;  // bisection passes (kSplitIterations; evaluate_sdf: kSplitIterations + 1)
    int refine;  // root refinement after pass 2 (GSR_OPT_NO_REFINE = 0 for the reference's passes only)
    float sample_range;  // half-width of the first bisection window (kSampleRange; 2 kSampleRange for evaluate_sdf)
    // SAMPLE mode (sample_depth, sample.hip): a workgroup is one chunk of
    // kTilePixels points of one tile instead of the tile's pixels
    uint32_t num_chunks;
    const uint32_t* chunk_off;  // [tiles + 1] exclusive scan of chunks per tile
    const uint2* pt_ranges;     // [tiles] points of each tile in pt_list
    const uint32_t* pt_list;    // point indices grouped by tile
    const float2* pt_xy;        // projected point positions
    int query;                  // kQuerySample / kQueryIntegrate / kQuerySDF
    const float* pt_t;          // [PN] |p_view| of each point
    float* out_points;          // [PN][3] camera-space point at the median depth (sample_depth);
                                // [PN] transmittance (integrate) or median depth (evaluate_sdf)
    float* out_sdf;             // [PN] median depth - |p_view| (evaluate_sdf)
    uint8_t* out_inside;        // [PN]
    uint32_t* pt_last;          // [PN] last contributor
    float* pt_mdepth;           // [PN] median depth along the ray
    float* pt_dT;               // [PN] dT/dt_m at pt_mdepth (valid where pt_cached)
    uint8_t* pt_cached;         // [PN]
    uint32_t* chunk_max;        // [chunks] max contributor of the chunk
    const uint32_t* tile_order; // [tiles] launch order (heaviest first) or null: XCD-contiguous
};

// One contributor's factor on the bisection samples (render_forward.cu:610-621):
//   T_p[s] *= (ts > t_peak ? 1 - a : 1 - a g) * rsqrt(1 - a g),  g = exp(-delta^2 / 2)
// The product over contributors is kept as two products,
//   A[s] = prod (ts > t_peak ? 1 - a : 1 - a g),   B[s] = prod (1 - a g),
// and T_p[s] = A[s] * rsqrt(B[s]) once per pass: one rsqrt per sample and
// pass instead of one per contributor (the reassociation moves T_p by a few
// ulp; both products stay >= the pixel's final transmittance >= 1e-4, so
// nothing underflows).  Samples are evaluated two at a time with packed
// fp32 (v_pk_{add,mul,fma}_f32), and
//  * exp(-delta^2/2) = exp2(-u u) with u = ts sc - t_peak sc and
//    sc = rsigma sqrt(0.5 log2e) per contributor: one packed fma gives a
//    sample pair's u and the negation rides on v_exp's source modifier (the
//    rounding differs from the reference's ((ts - t_peak) rsigma)^2 by a
//    few ulp of u, i.e. an absolute error of ~1e-7 in g);
//  * a non-ball splat (rsigma <= 0, g = 0 in the reference) runs with
//    alpha_g = 0 and sc = 0: u = 0, g = 1, 1 - 0*g = 1 exactly.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 ld4(const float4* p) { return *reinterpret_cast<const f32x4*>(p); }
constexpr float kSqrtHalfLog2e = 0.84932180028801904272f;  // sqrt(0.5 log2 e)
constexpr float kLog2e = 1.44269504088896340736f;          // (__expf(x) = v_exp_f32(x * kLog2e))

// Samples live in packed register pairs (pair k holds samples START + 2k and
// START + 2k + 1, so every v_pk_* operand is an aligned pair and no lane
// moves feed them); an odd count leaves one scalar sample (A1, B1 at T1).
// Per contributor the staged record supplies sc = rsigma sqrt(0.5 log2e)
// and the ball flag bm (1 or 0), so a_g = alpha bm and u = fma(ts, sc, -t_peak sc).
template <int NP, bool HAS1>
__device__ __forceinline__ void bisect_step(f32x2 (&A)[NP], f32x2 (&B)[NP], const f32x2 (&TS)[NP], float& A1,
                                            float& B1, float T1, float alpha, float t_peak, float rsig, float sc,
                                            float bm) {
    const float om = 1.f - alpha;
    const float ag = alpha * bm;
    const float q = -t_peak * sc;
    const f32x2 ag2 = {ag, ag}, sc2 = {sc, sc}, q2 = {q, q};
    const f32x2 one2 = {1.f, 1.f};
#pragma unroll
    for (int k = 0; k < NP; k++) {
        const f32x2 t = TS[k];
        const f32x2 u = __builtin_elementwise_fma(t, sc2, q2);
        const f32x2 e = u * u;
        const f32x2 g = {__builtin_amdgcn_exp2f(-e.x), __builtin_amdgcn_exp2f(-e.y)};
        const f32x2 omg = __builtin_elementwise_fma(-ag2, g, one2);
        const f32x2 sel = {t.x > t_peak ? om : omg.x, t.y > t_peak ? om : omg.y};
        A[k] *= sel;
        B[k] *= omg;
    }
    if constexpr (HAS1) {
        const float u = __builtin_fmaf(T1, sc, q);
        const float g = __builtin_amdgcn_exp2f(-(u * u));
        const float omg = __builtin_fmaf(-ag, g, 1.f);
        A1 *= T1 > t_peak ? om : omg;
        B1 *= omg;
    }
}

// Root refinement.  The vacancy transmittance T(t) is continuous and
// non-increasing in t (each factor is sqrt(1 - a g) in front of the splat's
// peak and (1 - a) / sqrt(1 - a g) behind it), so the reference's 5-pass
// 8-way bisection converges on the root of T(t) = 1/2 and returns it within
// its final cell (0.8 / 8^5 = 2.4e-5 wide, linearly interpolated: ~1e-8 from
// the root where T is smooth).  Here the root is found directly:
//  1. one walk evaluates T at kProbes depths: the reference's window ends
//     (its in_range test) and m0 + kProbeOffsets * SAMPLE_RANGE, which
//     bracket the root tightly (on C3 the root is within 0.05 of m0 for 97%
//     of pixels, within 0.2 for all);
//  2. bracketed Halley steps on H(t) = log2 T(t) + 1 from the secant root of
//     H in that bracket:
//       H'  = -sum x sc |u|,                    x = a g / (1 - a g)
//       H'' = sum (+-) x sc^2 (1 - 2 ln2 u^2 (1 + x))   (+ in front of the peak)
//     with u = (t - t_peak) sc and g = exp2(-u^2) as in bisect_step.  A lane
//     is done when the Newton step |H / H'| <= kRefineTol max(t, 1) (the
//     Halley iterate after it is then ~(step / sigma)^2 closer still), and
//     keeps the result where the root is well conditioned (|H'| kCondTol
//     max(t, 1) >= kHNoise).
// Lanes not done after kRefineWalks walks and ill-conditioned lanes run the
// reference's 5 passes from its first window (the root of a T that stays
// within rounding of 1/2 over a stretch is decided by rounding: there only
// the reference's own sample grid reproduces its answer).  Measured on C3
// contributor sets (tools/sim/s2_sim.py): 2.0 walks per lane, 2.27 per wave
// (the slowest lane), max |refined - bisected| = 2.4e-7, no lane left to the
// passes.  (The previous scheme ran the reference's first two passes and
// refined from the pass-2 cell: one more 7-sample walk per contributor.)
#ifndef GSR_PROBES
#define GSR_PROBES 7  // (11 -> 9 -> 7: render_fwd 0.769 -> 0.758 -> (later build) 0.683 -> 0.671 ms at C3, profiles/r4_ab_probes.txt)
#endif
constexpr int kProbes = GSR_PROBES;  // 11 (the window ends, m0 and 8 offsets around it); 9 or 7 (no ends)
// With 9 probes the window ends are not sampled: T is non-increasing in t, so a bracket between the
// inner probes (m0 -/+ SAMPLE_RANGE / 2) implies the reference's in_range test (T(e0) >= 1/2 >= T(e8));
// a pixel whose root lies outside them is left to the reference's passes.
constexpr bool kProbeEnds = kProbes == 11;
#if GSR_PROBES == 7
__constant__ constexpr float kProbeOffsets[kProbes] = {-0.25f, -0.125f, -0.0625f, 0.f, 0.0625f, 0.125f, 0.25f};
#elif GSR_PROBES == 9
__constant__ constexpr float kProbeOffsets[kProbes] = {-0.5f, -0.25f, -0.125f, -0.0625f, 0.f,
                                                        0.0625f, 0.125f, 0.25f, 0.5f};
#else
__constant__ constexpr float kProbeOffsets[kProbes] = {0.f,    -0.5f,   -0.25f, -0.125f, -0.0625f, 0.f,
                                                        0.0625f, 0.125f, 0.25f,  0.5f,    0.f};
#endif
constexpr uint32_t kPubRefined = 1u, kPubOut = 2u, kPubIll = 4u;  // phase results: root found / not in range /
                                                                   // root found, ill-conditioned (below)
constexpr uint32_t kPubBracket = 128u;  // left to the passes with an evaluated bracket [lo, hi] of the root
constexpr uint32_t kLastMask = 0x3fffffffu, kLoEv = 1u << 30, kHiEv = 1u << 31;  // (s_pub_last of a phase-2b pixel)
#ifndef GSR_REFINE_WALKS
#define GSR_REFINE_WALKS 4
#endif
constexpr int kRefineWalks = GSR_REFINE_WALKS;
// SAMPLE mode: Halley walks from the query point's own distance (GSR_SAMPLE_GUESS, in the kernel)
#ifndef GSR_SAMPLE_GUESS
#define GSR_SAMPLE_GUESS 1
#endif
#ifndef GSR_SAMPLE_WALKS
#define GSR_SAMPLE_WALKS 5
#endif
constexpr int kSampleWalks = GSR_SAMPLE_WALKS;
#ifndef GSR_SAMPLE_DT_TOL
#define GSR_SAMPLE_DT_TOL 0.004f  // (SAMPLE) longest step, relative to the curvature length, dT/dt_m is continued over
#endif
constexpr float kSampleDtTol = GSR_SAMPLE_DT_TOL;
#ifndef GSR_SAMPLE_PASS_GROUP
#define GSR_SAMPLE_PASS_GROUP 1  // (SAMPLE) the passes and the exact dT/dt_m walk of left points in lane groups
#endif
#ifndef GSR_SAMPLE_NO_ENDS
#define GSR_SAMPLE_NO_ENDS 1  // (round 5: sample_fwd 0.839-0.844 -> 0.792-0.812 ms at the sample bench; 2 more of 1.27M points to the passes)
#endif
constexpr bool kSampleNoEnds = GSR_SAMPLE_NO_ENDS;
#ifndef GSR_REFINE_TOL
#define GSR_REFINE_TOL 3e-5f
#endif
constexpr float kRefineTol = GSR_REFINE_TOL;
// A longer Newton step is accepted too when it is short against the local
// curvature length of H: |H / H'| <= kLooseTol max(t, 1) and |H / H'| F / |H'|
// <= kCurvTol, F = sum |H'' terms| (bounds H'' across the splat peaks where it
// jumps).  The Halley iterate is then within ~step kCurvTol^2 of the root, and
// dT/dt_m continued over that step keeps a relative error ~kCurvTol^2
// (tools/sim/s4_sim.py, SIM_LOOSE / SIM_TOLF: on C3 phase-2 second walks
// 11.2k -> 3.9k of 50.8k lanes, phase-1 wave walks 2.41 -> 2.14, max
// |refined - bisected| 2.4e-7 -> 9.5e-7).
#ifndef GSR_LOOSE_TOL
#define GSR_LOOSE_TOL 2e-4f
#endif
#ifndef GSR_CURV_TOL
#define GSR_CURV_TOL 0.02f
#endif
constexpr float kLooseTol = GSR_LOOSE_TOL;
constexpr float kCurvTol = GSR_CURV_TOL;
constexpr float kCondTol = 1e-6f;   // conditioning threshold (as the previous scheme's tolerance)
constexpr float kTwoLn2 = 1.38629436111989061883f;
#ifndef GSR_ILL_NEWTON
#define GSR_ILL_NEWTON 1
#endif
#ifndef GSR_HNOISE
#define GSR_HNOISE 1e-5f
#endif
// A converged root whose noise-induced uncertainty kHNoise / |H'| is above the
// kCondTol bar but below kIllTol max(t, 1) (T flat near 1/2 between two
// splats' peaks: C2 leaves 98k of 640k pixels so) is kept as the median depth
// (within kIllTol of the reference's own noise-decided bisection answer) and
// its dT/dt_m is computed exactly by the reference's pre-pass formula at that
// depth in one more walk — instead of the reference's five passes plus that
// walk.  (The continued H'' value refined lanes use would be off by ~kCurvTol^2
// relative, which the implicit gradient's 1 / dT/dt_m amplifies at such pixels.)
#ifndef GSR_ILL_ACCEPT
#define GSR_ILL_ACCEPT 1
#endif
constexpr float kIllTol = 1e-5f;
constexpr float kHNoise = GSR_HNOISE;  // rounding noise assumed in log2 T (~10x a 64-factor product's; 2e-6 measured: C2 render_fwd 0.763 -> 0.717 ms, but a small scene's dL/dmeans2D drifts to 1.3e-4 of the oracle through the implicit median-depth gradient)

__device__ __forceinline__ void refine_step(float& A, float& B, float& D, float& E, float& F, float t, float alpha,
                                            float t_peak, float sc, float bm) {
    const float om = 1.f - alpha;
    const float u = __builtin_fmaf(t, sc, -t_peak * sc);
    const float u2 = u * u;
    const float ag = (alpha * bm) * __builtin_amdgcn_exp2f(-u2);
    const float omg = 1.f - ag;
    const bool behind = t > t_peak;
    A *= behind ? om : omg;
    B *= omg;
    const float x = ag * __builtin_amdgcn_rcpf(omg);
    const float xs = x * sc;
    D = __builtin_fmaf(xs, fabsf(u), D);
    const float xsc = xs * sc;
    const float p = __builtin_fmaf(-kTwoLn2 * u2, 1.f + x, 1.f);
    E = __builtin_fmaf(behind ? -xsc : xsc, p, E);
    F = __builtin_fmaf(xsc, fabsf(p), F);  // bounds |H''| on either side of every splat peak (where H'' jumps)
}

// refine_step for the walk's two contributors at once, in the halves of packed registers: every product
// and sum chain is kept per half (A, B, D, E, F pairs, combined after the walk), so the two chains are
// independent and each op is one v_pk_* instruction; the transcendentals, compares and selects stay
// per half.  Same per-contributor arithmetic as refine_step (a lone contributor's partner has alpha = 0:
// factors exactly 1, terms exactly 0).
__device__ __forceinline__ void refine_step2(f32x2& A, f32x2& B, f32x2& D, f32x2& E, f32x2& F, f32x2 t2,
                                             f32x2 alpha, f32x2 t_peak, f32x2 sc, f32x2 bm) {
    const f32x2 one = {1.f, 1.f};
    const f32x2 om = one - alpha;
    const f32x2 u = __builtin_elementwise_fma(t2, sc, -(t_peak * sc));
    const f32x2 u2 = u * u;
    const f32x2 g = {__builtin_amdgcn_exp2f(-u2.x), __builtin_amdgcn_exp2f(-u2.y)};
    const f32x2 ag = (alpha * bm) * g;
    const f32x2 omg = one - ag;
    const bool bx = t2.x > t_peak.x, by = t2.y > t_peak.y;
    A *= f32x2{bx ? om.x : omg.x, by ? om.y : omg.y};
    B *= omg;
    const f32x2 x = ag * f32x2{__builtin_amdgcn_rcpf(omg.x), __builtin_amdgcn_rcpf(omg.y)};
    const f32x2 xs = x * sc;
    D = f32x2{__builtin_fmaf(xs.x, fabsf(u.x), D.x), __builtin_fmaf(xs.y, fabsf(u.y), D.y)};
    // the H'' term e = xsc p, fused into its two sums (xsc >= 0: |e| = xsc |p|)
    const f32x2 xsc = xs * sc;
    const f32x2 p = __builtin_elementwise_fma(f32x2{-kTwoLn2, -kTwoLn2} * u2, one + x, one);
    E = __builtin_elementwise_fma(f32x2{bx ? -xsc.x : xsc.x, by ? -xsc.y : xsc.y}, p, E);
    F = f32x2{__builtin_fmaf(xsc.x, fabsf(p.x), F.x), __builtin_fmaf(xsc.y, fabsf(p.y), F.y)};
}

// An opaque copy of v: the compiler cannot prove it equal to v, so values
// derived from it are recomputed at the use instead of kept live (or spilled)
// from an earlier, identical expression.
__device__ __forceinline__ int opaque_int(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// What a walk over one pixel's blended set needs: its mask column, last
// contributor, coordinates and the contributor filter of a lane group.  The
// refinement takes it from a functor called at every walk, which recomputes
// it (from an opaque lane id and LDS) instead of holding it across the walks.
struct PixSrc {
    const uint32_t* mask;
    uint32_t plast;
    float x, y;
    uint32_t filter;
};

// Diagnostic counters (STATS builds only, option GSR_OPT_RENDER_STATS):
// [0] per-lane walk wave-steps and [1] their active lanes; [2] composite
// wave-steps and [3] their blending lanes;
// [4] waves running the refinement, [5] waves sending a lane to the
// reference's passes, [6] refinement lane-walks, [7] lanes left to the passes;
// [8 + 2 f], [9 + 2 f]: walk wave-steps and their active lanes of render-path
// phase f = 0 (1: grid pixels), 1 (2: first walk), 2 (2b: grouped), 3 (3: passes / dT walks);
// [16] ill-conditioned roots kept (phase 3 computes their dT/dt_m only), [17] lanes phase 3 gives its
// listed pixels (render path); [18] reference passes skipped by phase-3 pixels' brackets, [19] pixels that
// skipped at least one.
constexpr int kRenderStats = 20;
__device__ unsigned long long g_render_stats[kRenderStats];

// SAMPLE: queries at arbitrary points — lanes hold points of one tile's
// chunk and the outputs are per point.  Everything else (batching,
// bisection) is shared with the render path.
//  * GEOM (sample_depth, sampleDepthCUDA, sample_forward.cu:430-657; and
//    evaluate_sdf, evaluateSDFCUDA, :171-427, which differs only in a twice
//    as wide first window, one more pass and its outputs): the composite
//    keeps only T / last / m0 / blended set, then the bisection runs.
//  * !GEOM (integrate, evaluateTransmittanceCUDA, :55-169): the composite
//    also carries the vacancy transmittance at the point's own distance.
// Occupancy (C3, GSR_* build variants through tools/ab_libs.sh): 24.3 KB of
// LDS per block (a 256-record resident cache, 128-record composite batches)
// fits 6 blocks per CU, and 6 waves per SIMD (80 VGPRs): 0.812 ms (round 2,
// with 28 registers spilled around the median-depth phases: 216 MB of
// scratch written per C3 launch; round 3 recomputes what was spilled — the
// pixel coordinates, mask column, LDS indices and bisection window — from an
// opaque lane id at each walk (PixSrc, opaque_int), and the lane groups
// combine through DPP quad moves instead of ds_bpermute: one spilled
// register, WRITE_SIZE 303 -> 93 MiB per launch, 0.783 -> 0.760 ms); the same at 5 waves per SIMD (96 VGPRs) 0.823; a
// 352-record cache with 256-record batches (31.8 KB: the LDS granule left 4
// blocks per CU) 0.893; a 192-record cache 0.820; 64-record batches 0.825.
// Tiles whose contributing prefix exceeds the cache take the wave-uniform
// walk (C3's largest per-tile max contributor is 184).
// Development: -DGSR_DBG_PX=x -DGSR_DBG_PY=y prints the median-depth phases' results for one pixel.
#ifdef GSR_DBG_PX
#define GSR_DBG(p, ...) \
    do { if (x0 + ((p) & 15) == GSR_DBG_PX && y0 + ((p) >> 4) == GSR_DBG_PY) printf(__VA_ARGS__); } while (0)
#define GSR_DBG_NEAR(p, ...) \
    do { if (abs(x0 + ((p) & 15) - GSR_DBG_PX) <= 1 && abs(y0 + ((p) >> 4) - GSR_DBG_PY) <= 1) printf(__VA_ARGS__); } while (0)
#else
#define GSR_DBG(p, ...) do { } while (0)
#define GSR_DBG_NEAR(p, ...) do { } while (0)
#endif
#ifndef GSR_FWD_WAVES
#define GSR_FWD_WAVES 6
#endif
#ifndef GSR_SAMPLE_WAVES
#define GSR_SAMPLE_WAVES 7  // (the SAMPLE instance: 72 VGPRs; the grouped exact dT/dt_m walk took it to 74 = 6 waves)
#endif

// Median-depth phases 2b and 3 (render path) give each listed pixel as many
// lanes as one round of the block allows (up to 16), instead of 4 and 1.
#ifndef GSR_ADAPT_GROUPS
#define GSR_ADAPT_GROUPS 1
#endif
constexpr bool kAdaptGroups = GSR_ADAPT_GROUPS;
// Phase 2 without the window-end samples (in_range implied by a root well inside the window).
#ifndef GSR_P2_NOENDS
#define GSR_P2_NOENDS 1  // (0: ends sampled in the first walk; render_fwd 0.738 -> 0.682 ms at C3 with 1, profiles/r4_ab_p2_noends.txt)
#endif
constexpr bool kP2NoEnds = GSR_P2_NOENDS;
// Phase 1 with one Halley walk: a grid pixel that needs more continues in phase 2 on its own lane
// (whose fourth wave was idle) from its iterate, which its neighbours take as their guess.
#ifndef GSR_P1_ONE
#define GSR_P1_ONE 1  // (0: up to 4 Halley walks in phase 1; render_fwd 0.672 -> 0.628 ms at C3 with 1, profiles/r4_ab_p1_one.txt)
#endif
constexpr bool kP1One = GSR_P1_ONE;
// Phase 2b: Halley walks of a straggler before it is left to the passes (3: C2 render_fwd 0.500 -> 0.490 ms,
// C3 unchanged, profiles/r4_ab_p2b_walks.txt; the sample path keeps kRefineWalks)
#ifndef GSR_P2B_WALKS
#define GSR_P2B_WALKS 2
#endif
constexpr int kP2bWalks = GSR_P2B_WALKS;
#ifndef GSR_P3_ILL_SHIFT
#define GSR_P3_ILL_SHIFT 3  // phase 3: an ill-conditioned root's group is at least G_p >> this (2 and 4: the same within noise, profiles/r4_ab_p3_ill_floor.txt)
#endif
#ifndef GSR_PASS_SKIP
#define GSR_PASS_SKIP 1  // phase 3 skips the reference passes a pixel's evaluated bracket decides
#endif
#ifndef GSR_LEFT_STATS
#define GSR_LEFT_STATS 0  // (development: render stats slots 12..15 count why pixels are left to the passes)
#endif
// Phase 2b group size: the largest (at most 16 lanes) that runs every straggler in one round, down to
// GSR_P2B_ONE_ROUND - 1 as log2 (0: 16 / 8 / 4 lanes by count, more rounds above 64 stragglers)
#ifndef GSR_P2B_ONE_ROUND
#define GSR_P2B_ONE_ROUND 1  // (C2 render_fwd 0.523 -> 0.503 ms, C3 unchanged; profiles/r4_ab_p2b_one_round.txt)
#endif

template <bool GEOM, bool STATS = false, bool SAMPLE = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((SAMPLE && GEOM && !STATS) ? GSR_SAMPLE_WAVES : GSR_FWD_WAVES, 8))) render_fwd_kernel(RenderFwdArgs a) {
    // LDS: composite staging (4 x 128 x 16 B = 8 KB) aliased with the
    // resident cache (3 x 256 x 16 B = 12 KB), the 8 KB of masks and the
    // phase exchange: 24.3 KB per block, 6 blocks (24 waves) per CU.
    __shared__ float4 s_rec[kRecSlots];
    // blended contributors per pixel, word-major (word w of lane t at w * 256 + t: conflict-free)
    __shared__ uint32_t s_mask[GEOM ? kTilePixels * kMaskWords : 1];
    __shared__ int s_alive[2][4];
    __shared__ uint32_t s_union[kBlendWords];  // (render path) entries some pixel of the tile blended
    __shared__ uint32_t s_max[4];
    // (render path, GEOM) the median-depth phases: per pixel the composite's last contributor,
    // m0 and T, then the worker's result (flags, md_out, dT/dt_m); the grid pixels' roots
    constexpr int kPub = (GEOM && !SAMPLE) ? kTilePixels : 1;
    __shared__ uint32_t s_pub_last[kPub];
    __shared__ float s_pub_m0[kPub], s_pub_T[kPub];
    __shared__ float s_groot[(GEOM && !SAMPLE) ? 64 : 1];  // then the compacted phase-2 list (bytes)
    __shared__ uint8_t s_glive[(GEOM && !SAMPLE) ? 64 : 1];  // (kP1One) grid pixel continued in phase 2
    __shared__ float s_pub_hi[kPub];

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    // (development, STATS builds with -DGSR_PHASE_CLOCK=1: shader clocks at the render path's phase
    // boundaries, summed per wave into render stats [8..13] in place of the per-phase walk counts)
#ifndef GSR_PHASE_CLOCK
#define GSR_PHASE_CLOCK 0
#endif
    constexpr bool kClock = GSR_PHASE_CLOCK && STATS;
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    auto stamp = [&](int k) {
        if constexpr (kClock) ph[k] = clock64();
    };
    stamp(0);
    uint32_t tile, chunk = 0, pid = 0;
    int px = 0, py = 0;
    bool inside;
    float pixx, pixy, pt_t = 0.f;
    if constexpr (SAMPLE) {
        // chunks of one tile are consecutive: XCD-contiguous runs of chunks share Gaussian lists
        chunk = xcd_remap(blockIdx.x, a.num_chunks);
        tile = wave_find_chunk_tile(a.chunk_off, a.num_tiles, chunk);
        const uint2 pr = a.pt_ranges[tile];
        const uint32_t slot = pr.x + (chunk - a.chunk_off[tile]) * kTilePixels + tid;
        inside = slot < pr.y;
        pid = inside ? a.pt_list[slot] : 0u;
        const float2 xy = inside ? a.pt_xy[pid] : make_float2(0.f, 0.f);
        pixx = xy.x;
        pixy = xy.y;
        pt_t = inside ? a.pt_t[pid] : 0.f;  // (GEOM: the refinement's start, GSR_SAMPLE_GUESS)
#ifndef GSR_SAMPLE_SORT
#define GSR_SAMPLE_SORT 1
#endif
        if constexpr (GEOM && GSR_SAMPLE_SORT) {
            // The chunk's points reordered by their pixel cell in the tile (row-major 16 x 16), so each wave
            // holds a compact patch of the tile as the render path's 16 x 4 strips: neighbouring points
            // blend similar sets, which makes a wave's composite and walks less divergent (the scatter into
            // the tile ranges leaves the points in arbitrary order).  A counting sort in LDS, before any
            // staging uses it; no output depends on which lane works a point.
            uint32_t* s_cnt = reinterpret_cast<uint32_t*>(s_rec);  // [256] counts, then offsets
            uint32_t* s_sp = s_cnt + kTilePixels;                  // [256] point id, x, y, |p_view| by rank
            float* s_sx = reinterpret_cast<float*>(s_sp + kTilePixels);
            float* s_sy = s_sx + kTilePixels;
            float* s_st = s_sy + kTilePixels;
            uint32_t* s_wt = reinterpret_cast<uint32_t*>(s_st + kTilePixels);  // [4] wave totals
            s_cnt[tid] = 0u;
            __syncthreads();
            const int tx0 = (int)(tile % a.grid_x) * kTile, ty0 = (int)(tile / a.grid_x) * kTile;
            const int lx = min(max((int)floorf(pixx + 0.5f) - tx0, 0), kTile - 1);
            const int ly = min(max((int)floorf(pixy + 0.5f) - ty0, 0), kTile - 1);
            const uint32_t key = (uint32_t)(ly * kTile + lx);
            const uint32_t rk = inside ? atomicAdd(&s_cnt[key], 1u) : 0u;
            __syncthreads();
            const uint32_t c = s_cnt[tid];
            uint32_t incl = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if ((tid & 63) >= o) incl += y;
            }
            if ((tid & 63) == 63) s_wt[tid >> 6] = incl;
            __syncthreads();
            uint32_t off = 0;
            for (int w = 0; w < (tid >> 6); w++) off += s_wt[w];
            s_cnt[tid] = off + incl - c;  // (each lane rewrites only its own count, read above)
            __syncthreads();
            if (inside) {
                const uint32_t d = s_cnt[key] + rk;
                s_sp[d] = pid;
                s_sx[d] = pixx;
                s_sy[d] = pixy;
                s_st[d] = pt_t;
            }
            const uint32_t n_in = s_wt[0] + s_wt[1] + s_wt[2] + s_wt[3];
            __syncthreads();
            inside = (uint32_t)tid < n_in;
            pid = inside ? s_sp[tid] : 0u;
            pixx = inside ? s_sx[tid] : 0.f;
            pixy = inside ? s_sy[tid] : 0.f;
            pt_t = inside ? s_st[tid] : 0.f;
            __syncthreads();  // (the staging below reuses s_rec)
        }
    } else {
        tile = a.tile_order ? a.tile_order[blockIdx.x] : xcd_remap(blockIdx.x, a.num_tiles);
        const uint32_t tx = tile % a.grid_x, ty = tile / a.grid_x;
        px = tx * kTile + (tid & 15);
        py = ty * kTile + (tid >> 4);
        inside = px < a.W && py < a.H;
        pixx = (float)px;
        pixy = (float)py;
    }

    const uint2 range = a.ranges[tile];
    unsigned long long t_pro = 0, n_rounds = 0, n_idle = 0;  // (phase-clock builds, SAMPLE) prologue end, batches
#if GSR_SAMPLE_PROLOGUE_ONLY  // (timing build: the SAMPLE raster's prologue alone; its outputs are wrong)
    if constexpr (SAMPLE) {
        if (inside && pixx == -1234.f && range.y == 7u) a.out_inside[pid] = 7;
        if (tid == 0) a.chunk_max[chunk] = 0u;
        return;
    }
#endif
    if constexpr (kClock && SAMPLE) t_pro = clock64() + (unsigned long long)(range.x & 0u);
    const int total = (int)(range.y - range.x);
    const int rounds = (total + kBatch - 1) / kBatch;

    float4* s_w0 = s_rec;
    float4* s_w1 = s_rec + kBatch;
    float4* s_w2 = s_rec + 2 * kBatch;
    float4* s_w3 = s_rec + 3 * kBatch;

    // each lane owns one mask column: no barrier needed between init, writes and reads
    uint32_t* my_mask = s_mask + (GEOM ? tid : 0);
    uint32_t mask_cur = 0;
    int mask_w = 0;
    if constexpr (GEOM) {
#pragma unroll
        for (int q = 0; q < kMaskWords; q++) my_mask[q * kTilePixels] = 0u;
    }

    if constexpr (!SAMPLE) {
        if (tid < kBlendWords) s_union[tid] = 0u;  // (ordered by the first batch's barrier)
    }
    uint32_t wbits = 0u;  // (render path, no depth) the lane's blended entries of the current 32-entry word
    float T = 1.0f, T_pt = 1.0f;
    uint32_t last = 0;
    float C0 = 0.f, C1 = 0.f, C2 = 0.f;
    float N0 = 0.f, N1 = 0.f, N2 = 0.f, m_init = 0.f;
    bool done = !inside;

    unsigned long long cst[2] = {0, 0};  // (STATS) composite wave-steps, blending lanes
    // One list entry g (0-based) at this lane, the reference's per-pixel loop
    // body: w0, w1 are the record's footprint words, w2f / w3f fetch the rest
    // only when the lane blends.
    // (step_pre: with the footprint terms dx, dy, power and alpha evaluated by the caller)
    auto step_pre = [&](const float4& w0, const float4& w1, auto&& w2f, auto&& w3f, int g, float dx, float dy,
                        float power, float alpha) {
        if constexpr (STATS) {
            const unsigned long long m = __ballot(1);
            if ((tid & 63) == __builtin_ctzll(m)) cst[0] += 1;
        }
        // the reference's three early-outs (power > 0, alpha < 1/255,
        // saturation) as one branch: every lane evaluates alpha and test_T
        const float test_T = T * (1.f - alpha);
        const bool pass = !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
        const bool sat = test_T < 0.0001f;
        if (!pass || sat) {
            done = done || (pass && sat);
            return;
        }
        if constexpr (STATS) {
            const unsigned long long m = __ballot(1);
            if ((tid & 63) == __builtin_ctzll(m)) cst[1] += __popcll(m);
        }
        const float aT = alpha * T;
        if constexpr (!SAMPLE && !GEOM) wbits |= 1u << (g & 31);  // (GEOM: from the blended-set masks)
        const float4 w2 = w2f();
        if constexpr (SAMPLE && !GEOM) {
            // vacancy transmittance at the point (sample_forward.cu:152-160)
            const float t_peak = splat_tpeak(w1, w2, dx, dy);
            const float rsigma = w2.y;
            const float delta = (t_peak - pt_t) * rsigma;
            const float gg = rsigma > 0.f ? __expf(-0.5f * delta * delta) : 0.f;
            const float omg = 1.f - alpha * gg;
            T_pt *= (pt_t > t_peak ? 1.f - alpha : omg) * __builtin_amdgcn_rsqf(omg);
        }
        if constexpr (!SAMPLE) {
            const float4 w3 = w3f();
            C0 = __builtin_fmaf(w2.z, aT, C0);
            C1 = __builtin_fmaf(w2.w, aT, C1);
            C2 = __builtin_fmaf(w3.x, aT, C2);
            if constexpr (GEOM) {
                N0 = __builtin_fmaf(w3.y, aT, N0);
                N1 = __builtin_fmaf(w3.z, aT, N1);
                N2 = __builtin_fmaf(w3.w, aT, N2);
            }
        }
        if constexpr (GEOM) {
            const float t = splat_tpeak(w1, w2, dx, dy);
            m_init = T > 0.5f ? t : m_init;
            if (g < kResident) {
                if ((g >> 5) != mask_w) {
                    my_mask[mask_w * kTilePixels] = mask_cur;
                    mask_cur = 0u;
                    mask_w = g >> 5;
                }
                mask_cur |= 1u << (g & 31);
            }
        }
        T = test_T;
        last = (uint32_t)g + 1u;  // the reference's 1-based contributor index
    };
    auto step = [&](const float4& w0, const float4& w1, auto&& w2f, auto&& w3f, int g) {
        const float dx = w0.x - pixx, dy = w0.y - pixy;
        const float power = splat_power(w0, w1, dx, dy);
        step_pre(w0, w1, w2f, w3f, g, dx, dy, power, fminf(0.99f, w1.y * __expf(power)));
    };
    int toDo = total;
    for (int i = 0; i < rounds; i++, toDo -= kBatch) {
        // block-wide early exit: every wave publishes whether any lane is live
        const bool wave_alive = __ballot(!done) != 0ull;
        if ((tid & 63) == 0) s_alive[i & 1][wave] = wave_alive;
        __syncthreads();  // also: everyone finished reading the previous batch
        if (!(s_alive[i & 1][0] | s_alive[i & 1][1] | s_alive[i & 1][2] | s_alive[i & 1][3])) break;
        if constexpr (kClock && SAMPLE) {
            n_rounds++;
            n_idle += wave_alive ? 0ull : 1ull;
        }
        const int k = i * kBatch + tid;
        if (tid < kBatch && k < total) {
            const Splat* sp = a.splats + a.point_list[range.x + k];
            const float4 w0 = sp->w0, w1 = sp->w1;
            s_w0[tid] = w0;
            s_w1[tid] = w1;
            s_w2[tid] = sp->w2;
            if constexpr (!SAMPLE) s_w3[tid] = sp->w3;
        }
        __syncthreads();
        const int n = min(kBatch, toDo);
        if constexpr (!GEOM && !SAMPLE) {
            // no depth: the batch in 32-entry words, each word's blended bits ORed over the wave
            // (DPP) and set by one lane (one atomic per blending step: render_fwd 0.214 -> 0.181 ms
            // without depth at C3; with no mask at all the backward walks every entry: 0.34 -> 0.40 ms)
            for (int j0 = 0; j0 < n; j0 += 32) {
                wbits = 0u;
                const int j1 = min(n, j0 + 32);
                for (int j = j0; !done && j < j1; j++)
                    step(s_w0[j], s_w1[j], [&] { return s_w2[j]; }, [&] { return s_w3[j]; }, i * kBatch + j);
                const int word = (i * kBatch + j0) >> 5;
                if (word < kBlendWords) {
                    const uint32_t v = wave_or_dpp(wbits);
                    if ((tid & 63) == 0 && v) atomicOr(&s_union[word], v);
                }
            }
        } else {
            for (int j = 0; !done && j < n; j++)
                step(s_w0[j], s_w1[j], [&] { return s_w2[j]; }, [&] { return s_w3[j]; }, i * kBatch + j);
        }
    }

    stamp(1);
    if constexpr (GEOM) {
        my_mask[mask_w * kTilePixels] = mask_cur;
        if constexpr (!SAMPLE) {  // the tile's union of the blended sets (the lane's own column: no barrier)
            static_assert(kMaskWords >= kBlendWords, "the blended-set masks cover the blend mask");
            // OR over the wave first (DPP, VALU only), then one lane per wave: 64 lanes' atomics on
            // one LDS word would serialize
            // (per-lane atomics instead: render_fwd 0.766 -> 0.821 ms at C3)
#pragma unroll
            for (int q = 0; q < kBlendWords; q++) {
                const uint32_t v = wave_or_dpp(my_mask[q * kTilePixels]);
                if ((tid & 63) == 0 && v) atomicOr(&s_union[q], v);
            }
        }
    }
    if constexpr (!SAMPLE) {
        // the composite's outputs are final: written before the median depth
        // (their registers are free for it)
        if (inside) {
            const int HW = a.H * a.W;
            const int pix = a.W * py + px;
            a.n_contrib[pix] = last;
            a.out_color[pix] = __builtin_fmaf(T, a.bg[0], C0);
            a.out_color[HW + pix] = __builtin_fmaf(T, a.bg[1], C1);
            a.out_color[2 * HW + pix] = __builtin_fmaf(T, a.bg[2], C2);
            a.out_alpha[pix] = 1.f - T;
            if constexpr (GEOM) {
                const float len = 1.f - T;
                a.out_normal[pix] = last ? N0 / len : 0.f;
                a.out_normal[HW + pix] = last ? N1 / len : 0.f;
                a.out_normal[2 * HW + pix] = last ? N2 / len : 0.f;
            }
        }
    }

    // block max of last contributor (cub BlockReduce in the reference)
    const uint32_t wmax = wave_max_u(last);
    if ((tid & 63) == 0) s_max[wave] = wmax;
    __syncthreads();
    if constexpr (!SAMPLE) {
        if (tid < kBlendWords) a.blend_mask[(size_t)tile * kBlendWords + tid] = s_union[tid];
    }
    const uint32_t max_contrib = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));

    // (render path) the pixel's coordinates recomputed where they are needed
    // after the composite, from the wave-uniform tile origin and an opaque
    // copy of the lane id: through the median-depth phases they would
    // otherwise stay live, with the LDS addresses derived from them, and spill
    const int tile_x0 = SAMPLE ? 0 : (int)(tile % a.grid_x) * kTile;
    const int tile_y0 = SAMPLE ? 0 : (int)(tile / a.grid_x) * kTile;
    auto lane_px = [&]() -> int { return tile_x0 + (opaque_int(tid) & 15); };
    auto lane_py = [&]() -> int { return tile_y0 + (opaque_int(tid) >> 4); };
    auto lane_fx = [&]() -> float {
        if constexpr (SAMPLE) return pixx;
        else return (float)lane_px();
    };
    auto lane_fy = [&]() -> float {
        if constexpr (SAMPLE) return pixy;
        else return (float)lane_py();
    };
    auto lane_mask = [&]() -> const uint32_t* { return s_mask + (GEOM ? opaque_int(tid) : 0); };
    float mDepth = 0.f, md_out = 0.f, md_dT = 0.f;
    bool md_ok = false, md_in_range = false;
#ifndef GSR_TIME_COMPOSITE_ONLY
#define GSR_TIME_COMPOSITE_ONLY 0  // (timing builds only: skip the median depth, its outputs are then wrong)
#endif
#ifndef GSR_TIME_SAMPLE_COMPOSITE_ONLY
#define GSR_TIME_SAMPLE_COMPOSITE_ONLY 0  // (timing builds only: the SAMPLE raster without its median depth)
#endif
    if constexpr (GEOM && !(GSR_TIME_COMPOSITE_ONLY && !SAMPLE) && !(GSR_TIME_SAMPLE_COMPOSITE_ONLY && SAMPLE)) {
        unsigned long long st[kRenderStats] = {0, 0, cst[0], cst[1]};
        int st_phase = 0;  // (STATS) render-path phase of the walks below
        float Tp[kSplit + 1];
        // the reference's first window (render_forward.cu:560-562)
        // (set where the passes start: only m_init stays live until then)
        auto win_lo = [&] { return fmaxf(m_init - a.sample_range, 0.f); };
        auto win_hi = [&] { return fmaxf(m_init + a.sample_range, 0.f); };
        float dmin = 0.f, dmax = 0.f;
        bool in_range = T <= kMinTransmittance;
        const bool resident = max_contrib <= (uint32_t)kResident;
        float4* c_w0 = s_rec;
        float4* c_w1 = s_rec + kResident;
        float4* c_w2 = s_rec + 2 * kResident;
        constexpr bool kSoA = SAMPLE ? kSampleWalkSoA : kWalkSoA;
        float* const s_pl = reinterpret_cast<float*>(s_rec);  // (kSoA) kPlanes planes of kPlane floats
        auto pl = [&](int f, int j) -> float { return s_pl[f * kPlane + j]; };
        auto pl2 = [&](int f, int j1, int j2) -> f32x2 { return f32x2{s_pl[f * kPlane + j1], s_pl[f * kPlane + j2]}; };
        // one staged record as the three float4 words (w2 = |t|, rsigma, sc, ball)
        auto rec = [&](int j, float4& w0, float4& w1, float4& w2) {
            if constexpr (kSoA) {
                w0 = make_float4(pl(0, j), pl(1, j), pl(2, j), pl(3, j));
                w1 = make_float4(pl(4, j), pl(5, j), pl(6, j), pl(7, j));
                w2 = make_float4(pl(8, j), pl(9, j), pl(10, j), pl(11, j));
            } else {
                w0 = c_w0[j];
                w1 = c_w1[j];
                w2 = c_w2[j];
            }
        };
        const int chunk = resident ? kResident : kTilePixels;
        const int chunks = ((int)max_contrib + chunk - 1) / chunk;
        auto stage = [&](int c0) {
            for (int k = tid; k < chunk && c0 + k < (int)max_contrib; k += kTilePixels) {
                const Splat* sp = a.splats + a.point_list[range.x + c0 + k];
                const float4 w0 = sp->w0, w1 = sp->w1, w2s = sp->w2;
                const bool ball = w2s.y > 0.f;  // non-ball splats: g = 0 (bisect_step)
                const float4 w2 = make_float4(w2s.x, w2s.y, ball ? w2s.y * kSqrtHalfLog2e : 0.f, ball ? 1.f : 0.f);
                if constexpr (kSoA) {
                    const float v[kPlanes] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x, w2.y, w2.z, w2.w};
#pragma unroll
                    for (int f = 0; f < kPlanes; f++) s_pl[f * kPlane + k] = v[f];
                } else {
                    c_w0[k] = w0;
                    c_w1[k] = w1;
                    c_w2[k] = w2;
                }
            }
        };
        if (resident && max_contrib > 0) {
            __syncthreads();
            stage(0);
            __syncthreads();
        }
        // Per-lane walk over the LDS-resident records of the contributors the
        // lane blended, in increasing index order (the reference's c = 1..last
        // multiplication order); each lane advances through its own mask words.
        // Two contributors per iteration (halving the per-step control and
        // exec-mask work; two independent dependency chains): when a word has
        // one left, the second is a dummy with alpha = 0, for which every walk
        // body multiplies by exactly 1 and adds exactly 0.
        auto walk = [&](const uint32_t* mask, uint32_t plast, float ppx, float ppy, uint32_t filter, bool active,
                        auto&& body) {
            const int nwords = active ? (int)((plast + 31) >> 5) : 0;
            int w = 0;
            uint32_t bits = nwords ? (mask[0] & filter) : 0u;
            // (the search for the next word with bits ends the loop body, so the loop-carried sums of the
            // body stay in one register set: a search at the top left ten v_mov copies per step)
            auto next_word = [&] {
                while (bits == 0u && w + 1 < nwords) bits = mask[++w * kTilePixels] & filter;
            };
            next_word();
            while (bits != 0u) {
                const int j1 = (w << 5) + __builtin_ctz(bits);
                bits &= bits - 1u;
                const bool two = bits != 0u;
                const int j2 = two ? (w << 5) + __builtin_ctz(bits) : j1;
                bits &= bits - 1u;
                if constexpr (STATS) {
                    const unsigned long long m = __ballot(1);
                    if ((tid & 63) == __builtin_ctzll(m)) {
                        st[0] += 1;
                        st[1] += __popcll(m);
                        if (!GSR_LEFT_STATS || st_phase < 2) {
                            st[8 + 2 * st_phase] += 1;
                            st[9 + 2 * st_phase] += __popcll(m);
                        }
                    }
                }
                // both contributors' footprint in packed halves, with splat_power / splat_tpeak's
                // roundings (packed fp32 rounds as the scalar ops: alpha stays bit-identical to the
                // composite's and the backward's); __expf(x) = v_exp_f32(x log2 e)
                f32x2 X, Y, CA, CB, CC, OP, PX, PY, TT, RS, SC, BM;
                if constexpr (kSoA) {
                    X = pl2(0, j1, j2), Y = pl2(1, j1, j2), CA = pl2(2, j1, j2), CB = pl2(3, j1, j2);
                    CC = pl2(4, j1, j2), OP = pl2(5, j1, j2), PX = pl2(6, j1, j2), PY = pl2(7, j1, j2);
                    TT = pl2(8, j1, j2), RS = pl2(9, j1, j2), SC = pl2(10, j1, j2), BM = pl2(11, j1, j2);
                } else {
                    const f32x4 a0 = ld4(c_w0 + j1), b0 = ld4(c_w0 + j2);
                    const f32x4 a1 = ld4(c_w1 + j1), b1 = ld4(c_w1 + j2);
                    const f32x4 a2 = ld4(c_w2 + j1), b2 = ld4(c_w2 + j2);
                    X = __builtin_shufflevector(a0, b0, 0, 4), Y = __builtin_shufflevector(a0, b0, 1, 5);
                    CA = __builtin_shufflevector(a0, b0, 2, 6), CB = __builtin_shufflevector(a0, b0, 3, 7);
                    CC = __builtin_shufflevector(a1, b1, 0, 4), OP = __builtin_shufflevector(a1, b1, 1, 5);
                    PX = __builtin_shufflevector(a1, b1, 2, 6), PY = __builtin_shufflevector(a1, b1, 3, 7);
                    TT = __builtin_shufflevector(a2, b2, 0, 4), RS = __builtin_shufflevector(a2, b2, 1, 5);
                    SC = __builtin_shufflevector(a2, b2, 2, 6), BM = __builtin_shufflevector(a2, b2, 3, 7);
                }
                const f32x2 dx = X - f32x2{ppx, ppx}, dy = Y - f32x2{ppy, ppy};
                const f32x2 q = __builtin_elementwise_fma(CC * dy, dy, (CA * dx) * dx);
                const f32x2 power = __builtin_elementwise_fma(f32x2{-0.5f, -0.5f}, q, -((CB * dx) * dy));
                const f32x2 pe = power * f32x2{kLog2e, kLog2e};
                const f32x2 og = OP * f32x2{__builtin_amdgcn_exp2f(pe.x), __builtin_amdgcn_exp2f(pe.y)};
                const f32x2 alpha = {fminf(0.99f, og.x), two ? fminf(0.99f, og.y) : 0.f};
                const f32x2 t_peak = __builtin_elementwise_fma(PY, dy, PX * dx) + TT;
                body(alpha, t_peak, RS, SC, BM);
                next_word();
            }
        };
        // a body taking one contributor at a time (alpha, t_peak, rsigma, sc, ball), first then second
        auto each = [](auto&& body1) {
            return [&body1](f32x2 al, f32x2 tp, f32x2 rs, f32x2 sc, f32x2 bm) {
                body1(al.x, tp.x, rs.x, sc.x, bm.x);
                body1(al.y, tp.y, rs.y, sc.y, bm.y);
            };
        };
        auto lane_walk = [&](bool active, auto&& body) {
            walk(lane_mask(), last, lane_fx(), lane_fy(), ~0u, active, body);
        };
        auto own_src = [&] { return PixSrc{lane_mask(), last, lane_fx(), lane_fy(), ~0u}; };
        bool refined = false;   // median depth found by the root refinement
        float t_ref = 0.f;
        float ref_t = 0.f, ref_D = 0.f, ref_E = 0.f;  // the last refinement walk's depth, -H', H''
        bool dt_loose = false;  // (SAMPLE) refined, but dT/dt_m continued over too long a step: walked exactly
        float dT_pre = 0.f;  // (SAMPLE, GSR_SAMPLE_GUESS) a refined root's continued dT/dt_m
        bool passed_grp = false;  // (SAMPLE) left to the passes, which ran in lane groups: median depth in t_ref
        // one pass of the reference's bisection (render_forward.cu:560-645) over
        // the lanes still in range and not refined; FIRST evaluates all 9
        // samples, later passes reuse the bracketing ends
        // (src: the pixel whose blended set the resident walk uses, PixSrc)
        // A pixel may be worked by a group of G = 1, 2, 4, 8 or 16 aligned lanes (uniform over
        // the wave): lane q walks the contributors with index % G == q (gfilter), and the group's
        // products and sums are combined by DPP moves (xor 1, xor 2, half mirror, mirror: each
        // step pairs the two halves of a doubled group), identical in the G lanes as float * and
        // + commute — the same values, a different association than one lane's product.
        auto gprod = [&](float v, int G) {
            if (G >= 2) v *= dpp_mov<kDppXor1>(v);  // (DPP moves: no LDS addresses to keep)
            if (G >= 4) v *= dpp_mov<kDppXor2>(v);
            if (G >= 8) v *= dpp_mov<kDppRowHalfMirror>(v);
            if (G >= 16) v *= dpp_mov<kDppRowMirror>(v);
            return v;
        };
        auto gsum = [&](float v, int G) {
            if (G >= 2) v += dpp_mov<kDppXor1>(v);
            if (G >= 4) v += dpp_mov<kDppXor2>(v);
            if (G >= 8) v += dpp_mov<kDppRowHalfMirror>(v);
            if (G >= 16) v += dpp_mov<kDppRowMirror>(v);
            return v;
        };
        // (the G lanes' share of a blended-set word, lane q of the group)
        auto gfilter = [](int G, int q) -> uint32_t {
            return G == 1 ? ~0u : G == 2 ? 0x55555555u << q : G == 4 ? 0x11111111u << q
                 : G == 8 ? 0x01010101u << q : 0x00010001u << q;
        };
        auto pass = [&](auto first_c, auto&& src, int G, bool on) {
            constexpr bool FIRST = decltype(first_c)::value;
            constexpr int START = FIRST ? 0 : 1;
            constexpr int END = FIRST ? kSplit + 1 : kSplit;
            constexpr int NP = (END - START) / 2;
            constexpr bool HAS1 = ((END - START) & 1) != 0;
            const float interval = (dmax - dmin) * (1.f / (float)kSplit);
            float ts[kSplit + 1];
#pragma unroll
            for (int s = 0; s <= kSplit; s++) ts[s] = __builtin_fmaf(interval, (float)s, dmin);
            f32x2 A[NP], B[NP], TS[NP];
#pragma unroll
            for (int k = 0; k < NP; k++) {
                TS[k] = f32x2{ts[START + 2 * k], ts[START + 2 * k + 1]};
                A[k] = f32x2{1.f, 1.f};
                B[k] = f32x2{1.f, 1.f};
            }
            float A1 = 1.f, B1 = 1.f;
            const float T1 = ts[END - 1];
            if (resident) {
                const PixSrc ps = src();
                walk(ps.mask, ps.plast, ps.x, ps.y, ps.filter, in_range && !refined && on,
                     each([&](float alpha, float t_peak, float rs, float sc, float bm) {
                         bisect_step<NP, HAS1>(A, B, TS, A1, B1, T1, alpha, t_peak, rs, sc, bm);
                     }));
            } else {
                bool bdone = !in_range || !on;
                uint32_t c = 0;
                for (int ch = 0; ch < chunks; ch++) {
                    __syncthreads();
                    stage(ch * chunk);
                    __syncthreads();
                    const int n = min(chunk, (int)max_contrib - ch * chunk);
                    for (int j = 0; !bdone && j < n; j++) {
                        c++;
                        bdone = c >= last;
                        float4 w0, w1, w2;
                        rec(j, w0, w1, w2);
                        const float dx = w0.x - lane_fx(), dy = w0.y - lane_fy();
                        const float power = splat_power(w0, w1, dx, dy);
                        if (power > 0.0f) continue;
                        const float alpha = fminf(0.99f, w1.y * __expf(power));
                        if (alpha < 1.0f / 255.0f) continue;
                        const float t_peak = splat_tpeak(w1, w2, dx, dy);
                        bisect_step<NP, HAS1>(A, B, TS, A1, B1, T1, alpha, t_peak, w2.y, w2.z, w2.w);
                    }
                }
            }
            if (!on) return;  // (a lane whose passes are done keeps its cell; a group shares `on`)
#pragma unroll
            for (int k = 0; k < NP; k++) {
                Tp[START + 2 * k] = gprod(A[k].x, G) * __builtin_amdgcn_rsqf(gprod(B[k].x, G));
                Tp[START + 2 * k + 1] = gprod(A[k].y, G) * __builtin_amdgcn_rsqf(gprod(B[k].y, G));
            }
            if constexpr (HAS1) Tp[END - 1] = gprod(A1, G) * __builtin_amdgcn_rsqf(gprod(B1, G));
            // (refined lanes did not walk: their in_range stands)
            if (FIRST && !refined) in_range = (Tp[0] >= 0.5f) && (Tp[kSplit] <= 0.5f) && in_range;
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
            dmax = __builtin_fmaf((float)(start_id + 1), interval, dmin);
            dmin = __builtin_fmaf((float)start_id, interval, dmin);
            Tp[0] = lo;
            Tp[kSplit] = hi;
        };
        // Root refinement for one pixel, shared by the phases below: probe
        // walk + bracketed Halley walks.
        // Up to `walks` Halley walks from t in the bracket [lo, hi] (H(lo) >= 0 >= H(hi)),
        // tolerances relative to `scale`.  With `ends`, the first walk also evaluates T at the
        // window ends e0, e8 and sets in_range.  A lane still live on return continues from
        // (t, lo, hi).
        struct Refine {
            bool refined, ill, in_range, live, newton_done;
            float t_ref, ref_t, ref_D, ref_E;
            float t, lo, hi;
            bool lo_ev, hi_ev;  // lo / hi set by an evaluation of T (not the window's unevaluated ends)
            float ref_F;        // the last walk's curvature bound F (sum |H'' terms|)
        };
#ifdef GSR_DBG_ROOT
        // (development: the walked pixel is the traced one.  Build the trace with -DGSR_FWD_WAVES=5: at 6 waves
        // per SIMD the printf call spills registers, and that build loses values in unrelated tiles — DESIGN §5)
        bool dbg_here = false;
#endif
        // One walk's update of a live pixel: log2 T, its derivatives -D, E and the curvature bound F at t
        // (the products and sums of the walk), the bracket, the Halley iterate, and acceptance.
        auto root_update = [&](Refine& r, bool& live, float& t, float& lo, float& hi, float A, float B, float D, float E,
                               float F, float scale) {
#ifdef GSR_DBG_ROOT
            if (dbg_here)
                printf("root_update lane %d t %.7f H %g D %g E %g F %g [%.7f %.7f]\n", (int)(threadIdx.x & 63), t,
                       __builtin_fmaf(-0.5f, __builtin_amdgcn_logf(B), __builtin_amdgcn_logf(A)) + 1.f, D, E, F, lo, hi);
#endif
            const float tol = kRefineTol * scale, tol_cond = kCondTol * scale, tol_loose = kLooseTol * scale;
            if constexpr (STATS) st[6] += 1;
            const float H = __builtin_fmaf(-0.5f, __builtin_amdgcn_logf(B), __builtin_amdgcn_logf(A)) + 1.f;
            if (H >= 0.f) {
                lo = t;
                r.lo_ev = true;
            } else {
                hi = t;
                r.hi_ev = true;
            }
            // Halley step t - 2 H H' / (2 H'^2 - H H''), H' = -D, H'' = E; bisection if it leaves the bracket
            const float th = t + fast_div(2.f * H * D, __builtin_fmaf(2.f * D, D, -H * E));
            const bool halley_in = th >= lo && th <= hi;
            float tn = halley_in ? th : 0.5f * (lo + hi);
            // (converged by the Newton step, or by the bracket closing — the latter also at a jump of T
            // across 1/2, where H need not be small)
            const bool newton = (D > 0.f && fabsf(H) <= tol * D) ||
                                (D > 0.f && fabsf(H) <= tol_loose * D && fabsf(H) * F <= kCurvTol * D * D);
            const bool done = newton || hi - lo <= tol;
            if (done) {
                // accepted only where the root is well conditioned: rounding noise of
                // ~kHNoise in log2 T moves it by less than tol_cond (T flat near 1/2 — a
                // pixel between two splats' peaks — leaves it to the reference's passes)
                // (converged by the Newton test with the Halley iterate out of the bracket — H'' large
                // against H' near a splat's peak — the root is the Newton iterate, not the midpoint)
                r.t_ref = newton && !halley_in ? fminf(fmaxf(t + fast_div(H, D), lo), hi) : tn;
                // dT/dt_m is continued from t to the root with H'' (publish): only over a step short
                // against the curvature length of H — a thin splat's peak next to the root makes the
                // continuation meaningless (a surfel scene had H' change sign across a 8.5e-5 step) —
                // else the root is kept as an ill-conditioned one and dT/dt_m computed exactly (phase 3)
                const bool smooth = fabsf(r.t_ref - t) * F <= kCurvTol * D;
                r.refined = D * tol_cond >= kHNoise && smooth;
                // (an ill-conditioned root only where T itself is at 1/2: converged by the Newton step)
                bool ill = GSR_ILL_ACCEPT && !r.refined && newton && D * (kIllTol * scale) >= kHNoise;
                if (GSR_ILL_NEWTON && ill && !smooth) {
                    // A Halley step long against the curvature length crossed a splat's peak, where H''
                    // flips sign: its iterate is not the root (W16400 case, px (14729, 10): t 5.6e-5
                    // Newton steps before the root next to a peak, H H'' / H'^2 = 0.76, the Halley
                    // iterate 1.8e-4 past the root).  The Newton iterate is within F (H / H')^2 / (2 |H'|)
                    // of it; kept where that is within kIllTol, else the lane takes the reference's passes.
                    const float sN = fast_div(H, D);
                    r.t_ref = fminf(fmaxf(t + sN, lo), hi);
                    ill = F * sN * sN <= 2.f * D * (kIllTol * scale);
                }
                r.ill = ill;
                r.newton_done = newton;
                live = false;
                r.ref_t = t;
                r.ref_D = D;
                r.ref_E = E;
                r.ref_F = F;
            }
            t = tn;
        };
        auto halley = [&](auto&& src, int grouped, bool live, float t, float lo, float hi, bool ends, float e0, float e8, bool in_range0,
                          int walks, float scale, bool lo_ev, bool hi_ev) {
            Refine r{false, false, in_range0, false, false, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, lo_ev, hi_ev};
            const f32x2 TSE[1] = {f32x2{e0, e8}};
            for (int k = 0; k < walks && a.passes > 1; k++) {
                if (__ballot(live) == 0ull) break;
                if constexpr (STATS && SAMPLE && !kClock) st_phase = k < 3 ? k : 3;  // (walk stats per walk index)
                float A = 1.f, B = 1.f, D = 0.f, E = 0.f, F = 0.f;
                f32x2 AE[1] = {f32x2{1.f, 1.f}}, BE[1] = {f32x2{1.f, 1.f}};
                float unusedA = 1.f, unusedB = 1.f;
                const PixSrc ps = src();
#ifdef GSR_DBG_ROOT
#ifndef GSR_DBG_ROOT_PX
#define GSR_DBG_ROOT_PX GSR_DBG_PX
#define GSR_DBG_ROOT_PY GSR_DBG_PY
#endif
                dbg_here = ps.x == (float)GSR_DBG_ROOT_PX && ps.y == (float)GSR_DBG_ROOT_PY;
#endif
                if (ends && k == 0) {
                    walk(ps.mask, ps.plast, ps.x, ps.y, ps.filter, live,
                         each([&](float alpha, float t_peak, float rs, float sc, float bm) {
                             refine_step(A, B, D, E, F, t, alpha, t_peak, sc, bm);
                             bisect_step<1, false>(AE, BE, TSE, unusedA, unusedB, 0.f, alpha, t_peak, rs, sc, bm);
                         }));
                } else {
                    // the two contributor chains of a walk step in packed halves (refine_step2)
                    f32x2 A2 = {1.f, 1.f}, B2 = {1.f, 1.f}, D2 = {0.f, 0.f}, E2 = {0.f, 0.f}, F2 = {0.f, 0.f};
                    const f32x2 t2 = {t, t};
                    walk(ps.mask, ps.plast, ps.x, ps.y, ps.filter, live,
                         [&](f32x2 alpha, f32x2 t_peak, f32x2 rs, f32x2 sc, f32x2 bm) {
                             refine_step2(A2, B2, D2, E2, F2, t2, alpha, t_peak, sc, bm);
                         });
                    A = A2.x * A2.y;
                    B = B2.x * B2.y;
                    D = D2.x + D2.y;
                    E = E2.x + E2.y;
                    F = F2.x + F2.y;
                }
                A = gprod(A, grouped);
                B = gprod(B, grouped);
                D = gsum(D, grouped);
                E = gsum(E, grouped);
                F = gsum(F, grouped);
                if (ends && k == 0) {
                    const float T0 = gprod(AE[0].x, grouped) * __builtin_amdgcn_rsqf(gprod(BE[0].x, grouped));
                    const float T8 = gprod(AE[0].y, grouped) * __builtin_amdgcn_rsqf(gprod(BE[0].y, grouped));
                    r.in_range = r.in_range && T0 >= 0.5f && T8 <= 0.5f;
                    live = live && r.in_range;
                }
                if (live) root_update(r, live, t, lo, hi, A, B, D, E, F, scale);
            }
            if (a.passes == 1 && r.in_range) {  // diagnostic timing of the probe walk alone
                r.refined = true;
                r.t_ref = t;
                live = false;
            }
            r.live = live;
            r.t = t;
            r.lo = lo;
            r.hi = hi;
            return r;
        };
        // Probe walk (window ends + m0 + kProbeOffsets * SAMPLE_RANGE), then the
        // Halley walks from the log-secant root of the bracketing probes.
        auto probe_refine = [&](auto&& src, float pm0, float pT, int grouped, int walks) {
            bool pin = pT <= kMinTransmittance;
            const float lo_w = fmaxf(pm0 - a.sample_range, 0.f), hi_w = fmaxf(pm0 + a.sample_range, 0.f);
            const float interval = (hi_w - lo_w) * (1.f / (float)kSplit);
            const float e0 = lo_w, e8 = __builtin_fmaf(interval, (float)kSplit, lo_w);
            float tp[kProbes];
#pragma unroll
            for (int s = 0; s < kProbes; s++) {
                const float off = kProbeOffsets[s] * a.sample_range;
                tp[s] = kProbeEnds && s == 0 ? e0 : kProbeEnds && s == kProbes - 1 ? e8 : fminf(fmaxf(pm0 + off, e0), e8);
            }
            // the m0 probe is the scalar sample, the others go in packed pairs
            constexpr int NP = (kProbes - 1) / 2, MID = (kProbes - 1) / 2;
            f32x2 A[NP], B[NP], TS[NP];
#pragma unroll
            for (int k = 0; k < NP; k++) {
                const int s0 = 2 * k < MID ? 2 * k : 2 * k + 1, s1 = 2 * k + 1 < MID ? 2 * k + 1 : 2 * k + 2;
                TS[k] = f32x2{tp[s0], tp[s1]};
                A[k] = f32x2{1.f, 1.f};
                B[k] = f32x2{1.f, 1.f};
            }
            float A1 = 1.f, B1 = 1.f;
            const PixSrc ps = src();
            walk(ps.mask, ps.plast, ps.x, ps.y, ps.filter, pin,
                 each([&](float alpha, float t_peak, float rs, float sc, float bm) {
                     bisect_step<NP, true>(A, B, TS, A1, B1, tp[MID], alpha, t_peak, rs, sc, bm);
                 }));
            stamp(3);
            float Tv[kProbes];
#pragma unroll
            for (int k = 0; k < NP; k++) {
                const int s0 = 2 * k < MID ? 2 * k : 2 * k + 1, s1 = 2 * k + 1 < MID ? 2 * k + 1 : 2 * k + 2;
                Tv[s0] = gprod(A[k].x, grouped) * __builtin_amdgcn_rsqf(gprod(B[k].x, grouped));
                Tv[s1] = gprod(A[k].y, grouped) * __builtin_amdgcn_rsqf(gprod(B[k].y, grouped));
            }
            Tv[MID] = gprod(A1, grouped) * __builtin_amdgcn_rsqf(gprod(B1, grouped));
            const bool bracketed = (Tv[0] >= 0.5f) && (Tv[kProbes - 1] <= 0.5f);
            if constexpr (kProbeEnds) pin = bracketed && pin;
            // bracket: the last probe with T >= 1/2 and the next one
            int k1 = 0;
#pragma unroll
            for (int s = 1; s < kProbes - 1; s++) k1 = Tv[s] >= 0.5f ? s : k1;
            float lo = tp[0], hi = tp[1], Tlo = Tv[0], Thi = Tv[1];
#pragma unroll
            for (int s = 1; s < kProbes - 1; s++) {
                lo = k1 == s ? tp[s] : lo;
                hi = k1 == s ? tp[s + 1] : hi;
                Tlo = k1 == s ? Tv[s] : Tlo;
                Thi = k1 == s ? Tv[s + 1] : Thi;
            }
            // bracketed Halley on H(t) = log2 T(t) + 1 from the secant root of H in the bracket
            const float Hlo = __builtin_amdgcn_logf(Tlo) + 1.f;
            const float Hhi = __builtin_amdgcn_logf(Thi) + 1.f;
            float wsec = Hlo / (Hlo - Hhi);
            wsec = wsec != wsec ? 0.5f : fminf(fmaxf(wsec, 0.f), 1.f);
            const float t = __builtin_fmaf(wsec, hi - lo, lo);
            return halley(src, grouped, pin && bracketed, t, lo, hi, false, 0.f, 0.f, pin, walks, fmaxf(t, 1.f), bracketed,
                          bracketed);
        };
        bool have_out = false;  // (render path) md_out and dT/dt_m published by the pixel's worker
        if (a.refine && resident && a.passes > 0) {
            if constexpr (STATS) {
                if ((tid & 63) == 0) st[4] += 1;
            }
            if constexpr (!SAMPLE) {
                // Two phases over the tile (render_fwd.hip header, tools/sim/s4_sim.py):
                //  1. the 64 pixels of the even grid (x, y even), 4 lanes each: probe walk + Halley;
                //  2. the other 192, one lane each on 3 of the 4 waves: a Halley walk from the mean of
                //     their grid neighbours' roots (the median depth varies slowly: the guess is within
                //     2e-4 of the root for 90% of pixels at C3, against ~1e-3 for the probe bracket),
                //     also sampling the window ends for in_range; the ~30% not converged after it are
                //     compacted and continued by groups of 4 lanes (walk wave-steps at C3 3.08M with
                //     42 active lanes per step -> 2.53M with 51).
                // The owner lane then takes the result, or runs the reference's passes where there is
                // none (not converged, ill-conditioned, no grid neighbour with a root).
                const int x0 = tile_x0, y0 = tile_y0;
                s_pub_last[tid] = last;
                s_pub_m0[tid] = m_init;
                s_pub_T[tid] = T;
                __syncthreads();
                stamp(2);
                auto publish = [&](int p, const Refine& r) {
                    p = opaque_int(p);  // (the LDS addresses at the store, not kept from the reads)
                    uint32_t flags = r.in_range ? 0u : kPubOut;
                    float mo = 0.f, dt = 0.f;
                    if (r.in_range && (r.refined || r.ill)) {
                        flags = r.refined ? kPubRefined : kPubIll;
                        const float nrm = pixel_ray_norm((float)(x0 + (p & 15)), (float)(y0 + (p >> 4)), a.W, a.H,
                                                         a.focal_x, a.focal_y);
                        mo = r.t_ref * (1.0f / nrm);
                        const float mb = mo * nrm;
                        if (r.refined && mb != 0.f)
                            dt = (0.5f * 0.69314718055994530942f) * __builtin_fmaf(r.ref_E, mb - r.ref_t, -r.ref_D);
                    }
                    if (GSR_PASS_SKIP && r.in_range && !r.refined && !r.ill && r.lo_ev && r.hi_ev) {
                        flags = kPubBracket;  // (the reference's passes whose cell holds the bracket are skipped)
                        mo = r.lo;
                        s_pub_hi[p] = r.hi;
                    }
                    if (GSR_LEFT_STATS && r.in_range && !r.refined && !r.ill) flags = r.live ? 16u : r.newton_done ? 32u : 64u;
#ifdef GSR_DBG_DT
                    if ((flags & kPubRefined) && !(dt < -1e-4f))
                        printf("dbgdt publish (%d,%d) t_ref %.7f ref_t %.7f D %g E %g dt %g\n", x0 + (p & 15), y0 + (p >> 4),
                               r.t_ref, r.ref_t, r.ref_D, r.ref_E, dt);
#endif
                    s_pub_last[p] = flags;
                    s_pub_T[p] = mo;
                    s_pub_m0[p] = dt;
                };
                // Two-level phase 1 (round 5): the 16 pixels of the 4-spaced grid run the probe walk and a Halley
                // walk on 16 lanes each (1a); the other 48 even-grid pixels start a Halley walk from the
                // 4-grid roots interpolated (1b, 4 lanes each) instead of running the probe walk
                // themselves.  tools/sim/guess_sim.py (C3 contributor sets): 89% of them are accepted after
                // that one walk, 99.9% within two; the probe walk (7 samples per contributor) they skip
                // cost about 1.75 Halley walks.  A pixel with no root among its taps starts from its own
                // m0.  Those not converged continue in phase 2 on their own lane (as the grid pixels do).
#ifndef GSR_P1_TWO_LEVEL
#define GSR_P1_TWO_LEVEL 1
#endif
#ifndef GSR_INTERP_SPREAD
#define GSR_INTERP_SPREAD 0.05f
#endif
                constexpr float kInterpSpread = GSR_INTERP_SPREAD;
                // (block-uniform) the two-level scheme needs a smooth root field: every 4-grid pixel in range
                // (T <= MIN_TRANSMITTANCE) and their composite m0 within kInterpSpread of their mean (m0, the
                // crossing contributor's depth, is known before phase 1; the roots follow it within ~0.05).
                // tools/sim/guess_sim.py: C3 tiles under 5e-2 hold 97% of the pixels (82-93% of the 1b pixels
                // accepted after one walk); the sparse C2 scene's median depth is rough (17% of its tiles, 25%
                // accepted), and there a tile takes phase 1 as before: its 64 grid pixels probe-walked at once
                // (a two-level tile that falls back after 1a leaves a wave idle in 1b: C2 0.48 -> 0.505 ms).
                bool two_level = GSR_P1_TWO_LEVEL;
                if (two_level) {
                    float g_min = 3.4e38f, g_max = -3.4e38f, g_sum = 0.f;
                    bool all_in = true;
#pragma unroll
                    for (int i = 0; i < 16; i++) {
                        const int q = (i >> 2) * 64 + (i & 3) * 4;
                        const float gm = s_pub_m0[q];
                        all_in = all_in && s_pub_T[q] <= kMinTransmittance;
                        g_min = fminf(g_min, gm);
                        g_max = fmaxf(g_max, gm);
                        g_sum += gm;
                    }
                    two_level = all_in && g_max - g_min <= kInterpSpread * fmaxf(g_sum * (1.f / 16.f), 1.f);
                }
                if (two_level) {
                    {  // phase 1a: (4 (g / 4), 4 (g % 4)), g = lane / 16
                        auto grid4_pixel = [&](int lane) { return ((lane >> 4) >> 2) * 64 + ((lane >> 4) & 3) * 4; };
                        const int gp = grid4_pixel(tid), q = tid & 15;
                        const float gm0 = s_pub_m0[gp], gT = s_pub_T[gp];
                        auto src = [&] {
                            const int lane = opaque_int(tid), gq = grid4_pixel(lane);
                            return PixSrc{s_mask + gq, s_pub_last[gq], (float)(x0 + (gq & 15)), (float)(y0 + (gq >> 4)),
                                          0x00010001u << (lane & 15)};
                        };
                        const Refine r = probe_refine(src, gm0, gT, 16, 1);
                        if (q == 0) {
                            const int lane = opaque_int(tid), g4 = grid4_pixel(lane);
                            const bool cont = r.live;
                            const int gi = (g4 >> 5) * 8 + ((g4 & 15) >> 1);  // s_groot index (y / 2) 8 + x / 2
                            s_groot[gi] = (r.in_range && r.refined) ? r.t_ref : cont ? r.t : -1.f;
                            s_glive[gi] = cont ? 1 : 0;
                            if (!cont) publish(g4, r);
                        }
                    }
                    __syncthreads();
                    stamp(3);
                    {  // phase 1b: the 48 even-grid pixels off the 4-grid, 4 lanes each (waves 0-2)
                        // k = lane / 4: rows of the half-resolution grid in pairs (2 r, 2 r + 1): 4 pixels (odd
                        // half-res x) then 8
                        auto half_xy = [](int k, int& hx, int& hy) {
                            const int r = k / 12, m = k - 12 * (k / 12);
                            hx = m < 4 ? 2 * m + 1 : m - 4;
                            hy = m < 4 ? 2 * r : 2 * r + 1;
                        };
                        const int k = tid >> 2;
                        // (block-uniform) a 4-grid pixel without a root (1a did not find it in range): these 48
                        // run the probe walk instead
                        const bool v16 = s_groot[((tid & 15) >> 2) * 16 + (tid & 3) * 2] >= 0.f;
                        const bool interp_tile = (__ballot(v16) & 0xFFFFull) == 0xFFFFull;
                        if (k < 48) {
                            int hx, hy;
                            half_xy(k, hx, hy);
                            const int p = (2 * hy) * 16 + 2 * hx;
                            // the 4-grid roots interpolated on the half-resolution lattice (the phase-2 rules)
                            auto rule = [](int l, int* o, float* w, int& n) {
                                if (!(l & 1)) {
                                    o[0] = l; w[0] = 1.f; n = 1;
                                } else if (l == 1) {
                                    o[0] = 0; o[1] = 2; o[2] = 4; w[0] = 0.375f; w[1] = 0.75f; w[2] = -0.125f; n = 3;
                                } else if (l == 5) {
                                    o[0] = 2; o[1] = 4; o[2] = 6; w[0] = -0.125f; w[1] = 0.75f; w[2] = 0.375f; n = 3;
                                } else if (l == 7) {
                                    o[0] = 4; o[1] = 6; w[0] = -0.5f; w[1] = 1.5f; n = 2;
                                } else {
                                    o[0] = 0; o[1] = 2; o[2] = 4; o[3] = 6;
                                    w[0] = -0.0625f; w[1] = 0.5625f; w[2] = 0.5625f; w[3] = -0.0625f; n = 4;
                                }
                            };
                            int ox[4], oy[4], nx, ny;
                            float wx[4], wy[4];
                            rule(hx, ox, wx, nx);
                            rule(hy, oy, wy, ny);
                            float acc = 0.f;
                            bool ok = true;
#pragma unroll
                            for (int j = 0; j < 4; j++) {
                                if (j >= ny) break;
                                float row = 0.f;
#pragma unroll
                                for (int i = 0; i < 4; i++) {
                                    if (i >= nx) break;
                                    const float gr = s_groot[oy[j] * 8 + ox[i]];
                                    ok = ok && gr >= 0.f;
                                    row = __builtin_fmaf(wx[i], gr, row);
                                }
                                acc = __builtin_fmaf(wy[j], row, acc);
                            }
                            const float qm0 = s_pub_m0[p], qT = s_pub_T[p];
                            const bool qin = qT <= kMinTransmittance;
                            const float lo_w = fmaxf(qm0 - a.sample_range, 0.f), hi_w = fmaxf(qm0 + a.sample_range, 0.f);
                            const float e0 = lo_w, e8 = __builtin_fmaf((hi_w - lo_w) * (1.f / (float)kSplit), (float)kSplit, lo_w);
                            const float t0 = fminf(fmaxf(ok ? acc : qm0, e0), e8);
                            auto src = [&] {
                                int hx2, hy2;
                                half_xy(opaque_int(tid) >> 2, hx2, hy2);
                                const int pp = (2 * hy2) * 16 + 2 * hx2;
                                return PixSrc{s_mask + pp, s_pub_last[pp], (float)(x0 + (pp & 15)), (float)(y0 + (pp >> 4)),
                                              0x11111111u << (opaque_int(tid) & 3)};
                            };
                            const Refine r = interp_tile
                                                 ? halley(src, 4, qin, t0, e0, e8, false, 0.f, 0.f, qin, 1, fmaxf(t0, 1.f),
                                                          false, false)
                                                 : probe_refine(src, qm0, qT, 4, 1);
                            if ((tid & 3) == 0) {
                                const bool cont = r.live;
                                s_groot[hy * 8 + hx] = (r.in_range && r.refined) ? r.t_ref : cont ? r.t : -1.f;
                                s_glive[hy * 8 + hx] = cont ? 1 : 0;
                                if (!cont) publish(p, r);
                            }
                        }
                    }
                } else {  // phase 1
                    // (2 (g / 8), 2 (g % 8)) in the tile, g = lane / 4; recomputed for the publish
                    auto grid_pixel = [&](int lane) { return ((lane >> 2) >> 3) * 32 + ((lane >> 2) & 7) * 2; };
                    const int gp = grid_pixel(tid), q = tid & 3;
                    const float gm0 = s_pub_m0[gp], gT = s_pub_T[gp];
                    auto src = [&] {
                        const int lane = opaque_int(tid), gq = grid_pixel(lane);
                        return PixSrc{s_mask + gq, s_pub_last[gq], (float)(x0 + (gq & 15)), (float)(y0 + (gq >> 4)),
                                      0x11111111u << (lane & 3)};
                    };
                    const Refine r = probe_refine(src, gm0, gT, 4, kP1One ? 1 : kRefineWalks);
                    if (q == 0) {
                        const int lane = opaque_int(tid);
                        // (kP1One: a grid pixel not converged after its one Halley walk hands its iterate to its
                        // neighbours as their guess and continues in phase 2 on its own lane)
                        const bool cont = kP1One && r.live;
                        s_groot[lane >> 2] = (r.in_range && r.refined) ? r.t_ref : cont ? r.t : -1.f;
                        if constexpr (kP1One) s_glive[lane >> 2] = cont ? 1 : 0;
                        GSR_DBG_NEAR(grid_pixel(lane), "p1 (%d,%d): m0 %.7f -> live %d in %d ref %d ill %d t_ref %.7f D %g\n",
                                     x0 + (grid_pixel(lane) & 15), y0 + (grid_pixel(lane) >> 4), gm0, (int)r.live,
                                     (int)r.in_range, (int)r.refined, (int)r.ill, r.t_ref, r.ref_D);
                        if (!cont) publish(grid_pixel(lane), r);
                    }
                }
                __syncthreads();
                stamp(4);
                const int skip = (int)(blockIdx.x & 3u);  // the wave left idle (rotated over the SIMDs)
                if constexpr (STATS) st_phase = 1;
                bool live2 = false;  // phase-2 pixel not converged after its first walk
                int p2 = 0;
                // the grid neighbours' mean root of a phase-2 pixel: the pixel itself on even coordinates,
                // both sides on odd ones
                auto guess = [&](int lx, int ly, float& sum, int& cnt) {
                    sum = 0.f;
                    cnt = 0;
#pragma unroll
                    for (int dy = -1; dy <= 1; dy++)
#pragma unroll
                        for (int dx = -1; dx <= 1; dx++) {
                            const int nx = lx + dx, ny = ly + dy;
                            const bool use = ((lx & 1) ? dx != 0 : dx == 0) && ((ly & 1) ? dy != 0 : dy == 0);
                            if (use && nx >= 0 && nx < 16 && ny >= 0 && ny < 16) {
                                const float gr = s_groot[(ny >> 1) * 8 + (nx >> 1)];
                                if (gr >= 0.f) {
                                    sum += gr;
                                    cnt++;
                                }
                            }
                        }
                };
                // Higher-order guess (round 5): the root varies smoothly over a tile, so the grid roots are
                // interpolated by a tensor product of 1-D Lagrange rules on the grid coordinates — cubic
                // (-1, 9, 9, -1) / 16 over the grid points at -3, -1, +1, +3 inside the tile, quadratic
                // next to its edges, linear extrapolation at the last column / row; a coordinate on the
                // grid takes its grid point.  On C3 contributor sets (tools/sim/guess_sim.py) one walk
                // from it is accepted for 98% of the off-grid pixels, against 90% from the neighbours'
                // mean.  Any tap without a root (out of range): the mean above.
#ifndef GSR_P2_INTERP
#define GSR_P2_INTERP 1
#endif
                auto guess_interp = [&](int lx, int ly, float& out) -> bool {
                    int ox[4], oy[4];
                    float wx[4], wy[4];
                    int nx = 0, ny = 0;
                    auto rule = [](int l, int* o, float* w, int& n) {
                        if (!(l & 1)) {
                            o[0] = l; w[0] = 1.f; n = 1;
                        } else if (l == 1) {
                            o[0] = 0; o[1] = 2; o[2] = 4; w[0] = 0.375f; w[1] = 0.75f; w[2] = -0.125f; n = 3;
                        } else if (l == 13) {
                            o[0] = 10; o[1] = 12; o[2] = 14; w[0] = -0.125f; w[1] = 0.75f; w[2] = 0.375f; n = 3;
                        } else if (l == 15) {
                            o[0] = 12; o[1] = 14; w[0] = -0.5f; w[1] = 1.5f; n = 2;
                        } else {
                            o[0] = l - 3; o[1] = l - 1; o[2] = l + 1; o[3] = l + 3;
                            w[0] = -0.0625f; w[1] = 0.5625f; w[2] = 0.5625f; w[3] = -0.0625f; n = 4;
                        }
                    };
                    rule(lx, ox, wx, nx);
                    rule(ly, oy, wy, ny);
                    float acc = 0.f;
                    bool ok = true;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        if (j >= ny) break;
                        float row = 0.f;
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            if (i >= nx) break;
                            const float gr = s_groot[(oy[j] >> 1) * 8 + (ox[i] >> 1)];
                            ok = ok && gr >= 0.f;
                            row = __builtin_fmaf(wx[i], gr, row);
                        }
                        acc = __builtin_fmaf(wy[j], row, acc);
                    }
                    out = acc;
                    return ok;
                };
                // (kP1One: every lane takes its own pixel — the 192 off-grid ones and the grid pixels phase 1
                // left live, from their own iterate; otherwise 3 of the 4 waves take the 192 off-grid ones)
                const int k = kP1One ? tid : (wave < skip ? wave : wave - 1) * 64 + (tid & 63);
                const int pair = k / 24, r24 = k - pair * 24;
                const int lx = kP1One ? (tid & 15) : r24 < 8 ? 2 * r24 + 1 : r24 - 8;
                const int ly = kP1One ? (tid >> 4) : r24 < 8 ? 2 * pair : 2 * pair + 1;
                const bool on_grid = !(lx & 1) && !(ly & 1);
                const bool p2_todo = kP1One ? (!on_grid || s_glive[(ly >> 1) * 8 + (lx >> 1)] != 0) : wave != skip;
                if (p2_todo) {  // phase 2, first walk
                    const int p = ly * 16 + lx;
                    p2 = p;
                    const float qx = (float)(x0 + lx), qy = (float)(y0 + ly);
                    const uint32_t ql = s_pub_last[p];
                    const float qm0 = s_pub_m0[p], qT = s_pub_T[p];
                    float sum;
                    int cnt;
                    guess(lx, ly, sum, cnt);  // (a live grid pixel: its own iterate, the one grid neighbour it has)
                    const bool qin = qT <= kMinTransmittance;
                    const float lo_w = fmaxf(qm0 - a.sample_range, 0.f), hi_w = fmaxf(qm0 + a.sample_range, 0.f);
                    const float interval = (hi_w - lo_w) * (1.f / (float)kSplit);
                    const float e0 = lo_w, e8 = __builtin_fmaf(interval, (float)kSplit, lo_w);
                    float ti = 0.f;
                    const bool interp = GSR_P2_INTERP && !on_grid && guess_interp(lx, ly, ti);
                    const float t0 = cnt ? fminf(fmaxf(interp ? ti : sum / (float)cnt, e0), e8) : e0;
                    auto src = [&] { return PixSrc{s_mask + p, ql, qx, qy, ~0u}; };  // (one walk)
                    const Refine r = halley(src, 1, qin && cnt > 0, t0, e0, e8, !kP2NoEnds, e0, e8, qin, 1, fmaxf(t0, 1.f),
                                            false, false);
                    GSR_DBG(p, "p2: m0 %.7f cnt %d t0 %.7f -> live %d in %d ref %d ill %d t_ref %.7f t %.7f [%.7f %.7f] D %g\n",
                            qm0, cnt, t0, (int)r.live, (int)r.in_range, (int)r.refined, (int)r.ill, r.t_ref, r.t, r.lo,
                            r.hi, r.ref_D);
                    live2 = r.live;
                    if (live2) {  // continued by a lane group below (which ends of its bracket are evaluated: high bits)
                        s_pub_last[p] = ql | (r.lo_ev ? kLoEv : 0u) | (r.hi_ev ? kHiEv : 0u);
                        s_pub_T[p] = r.t;
                        s_pub_m0[p] = r.lo;
                        s_pub_hi[p] = r.hi;
                    } else if (cnt > 0 || !qin) {
                        publish(p, r);
                    } else {
                        s_pub_last[p] = GSR_LEFT_STATS ? 8u : 0u;  // no guess: the owner runs the passes
                    }
                }
                // The pixels not converged after one walk (~30% at C3), compacted and continued by
                // groups of 4 lanes (as phase 1): their second walk no longer holds every lane of
                // the three phase-2 waves.
                stamp(5);
                const unsigned long long bl = __ballot(live2);
                if ((tid & 63) == 0) s_max[wave] = (uint32_t)__popcll(bl);
                __syncthreads();  // also: every phase-2 lane has read s_groot
                uint32_t before = 0, n_live = 0;
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    before += w < wave ? s_max[w] : 0u;
                    n_live += s_max[w];
                }
                uint8_t* s_list = reinterpret_cast<uint8_t*>(s_groot);
                if constexpr (STATS) st_phase = 2;
                if (live2) s_list[before + __popcll(bl & ((1ull << (tid & 63)) - 1ull))] = (uint8_t)p2;
                __syncthreads();
                // group size: as many lanes per pixel as one round of the block allows (4 .. 16)
#if GSR_P2B_ONE_ROUND
                int lg2b = 4;
                while (lg2b > GSR_P2B_ONE_ROUND - 1 && (n_live << lg2b) > (uint32_t)kTilePixels) lg2b--;
#else
                const int lg2b = kAdaptGroups ? (n_live <= 16 ? 4 : n_live <= 32 ? 3 : 2) : 2;
#endif
                const int G2b = 1 << lg2b;
                for (uint32_t e = (uint32_t)(tid >> lg2b); e < n_live; e += (uint32_t)(kTilePixels >> lg2b)) {
                    const int p = s_list[e];
                    const float t = s_pub_T[p];
                    const uint32_t sl = s_pub_last[p];
                    auto src = [&] {
                        const int pp = s_list[opaque_int((int)e)];
                        return PixSrc{s_mask + pp, s_pub_last[pp] & kLastMask, (float)(x0 + (pp & 15)), (float)(y0 + (pp >> 4)),
                                      gfilter(G2b, opaque_int(tid) & (G2b - 1))};
                    };
                    const Refine r = halley(src, G2b, true, t, s_pub_m0[p], s_pub_hi[p], false, 0.f, 0.f, true,
                                            kP2bWalks, fmaxf(t, 1.f), (sl & kLoEv) != 0u, (sl & kHiEv) != 0u);
                    if ((tid & (G2b - 1)) == 0)
                        GSR_DBG(p, "p2b: from %.7f -> live %d in %d ref %d ill %d t_ref %.7f t %.7f [%.7f %.7f] D %g\n", t,
                                (int)r.live, (int)r.in_range, (int)r.refined, (int)r.ill, r.t_ref, r.t, r.lo, r.hi, r.ref_D);
                    if ((tid & (G2b - 1)) == 0) publish(s_list[opaque_int((int)e)], r);
                }
                __syncthreads();
                stamp(6);
                const int me = opaque_int(tid);
                uint32_t flags = s_pub_last[me];
                if constexpr (kP2NoEnds) {
                    // phase 2 did not sample the window ends: a root found well inside the reference's
                    // first window implies its in_range test (T is non-increasing); one near or past an
                    // end is left to the passes, which decide in_range with their own samples
                    if (flags & (kPubRefined | kPubIll)) {
                        const float t_pub = s_pub_T[me] * pixel_ray_norm(lane_fx(), lane_fy(), a.W, a.H, a.focal_x,
                                                                         a.focal_y);
                        const float e0 = win_lo(), hi_w = win_hi();
                        const float e8 = __builtin_fmaf((hi_w - e0) * (1.f / (float)kSplit), (float)kSplit, e0);
                        const float margin = 1e-4f * fmaxf(t_pub, 1.f);
                        if (!(t_pub > e0 + margin && t_pub < e8 - margin)) flags = 0u;
                    }
                }
                const bool ill = (flags & kPubIll) != 0u;  // root in s_pub_T[me]; dT/dt_m by the walk below
                if (flags & kPubRefined) {
                    refined = true;
                    have_out = true;
                    md_out = s_pub_T[me];
                    md_dT = s_pub_m0[me];
                } else if (flags & kPubOut) {
                    in_range = false;
                }
                // Phase 3: the pixels left to the reference's passes (not converged, ill-conditioned, no
                // guess) compacted, lane e of the block working the e-th of them: a wave holding one such
                // pixel no longer runs the passes with all of its lanes (C2, a sparse 800x800 scene: 134k
                // of 640k pixels left, in 85% of the waves).  Per pixel the same walks in the same order
                // as its owner lane would run them: the same outputs.
                // The list holds the pixels that need the passes first, then the ill-conditioned roots
                // (one walk each), so the waves working the latter skip the passes.
                const bool left3 = in_range && !refined;
                const bool left3p = left3 && !ill;
                if constexpr (STATS) st_phase = 3;
                const unsigned long long bl3 = __ballot(left3p), bl3i = __ballot(left3 && ill);
                if ((tid & 63) == 0) {
                    s_max[wave] = (uint32_t)__popcll(bl3);
                    s_alive[0][wave] = __popcll(bl3i);
                }
                __syncthreads();  // (every owner has read its flags)
                uint32_t before3 = 0, n_pass = 0, before3i = 0, n_ill = 0;
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    before3 += w < wave ? s_max[w] : 0u;
                    n_pass += s_max[w];
                    before3i += w < wave ? (uint32_t)s_alive[0][w] : 0u;
                    n_ill += (uint32_t)s_alive[0][w];
                }
                const uint32_t n_left = n_pass + n_ill;
                if constexpr (STATS) {
                    st[7] += left3p ? 1 : 0;
                    st[16] += (left3 && ill) ? 1 : 0;
                }
#if GSR_LEFT_STATS
                // (development) why a pixel is left to the passes: no guess / still live after its walks /
                // converged by the Newton test but not well conditioned (the rest: the bracket closed
                // without it, or a root near a window end); ill roots
                if constexpr (STATS) {
                    const bool ng = left3p && (s_pub_last[me] & 8u) != 0u;
                    const bool mr = left3p && !ng && (s_pub_last[me] & 16u) != 0u;
                    const bool cn = left3p && !ng && (s_pub_last[me] & 32u) != 0u;  // converged by the Newton test, conditioning
                    const unsigned long long b0 = __ballot(ng), b1 = __ballot(mr), b2 = __ballot(cn),
                                             b3 = __ballot(left3 && ill);
                    if ((tid & 63) == 0) {
                        st[12] += __popcll(b0);
                        st[13] += __popcll(b1);
                        st[14] += __popcll(b2);
                        st[15] += __popcll(b3);
                    }
                }
#endif
                if (n_left > 0) {  // (block-uniform)
                    if (left3) {
                        const unsigned long long lower = (1ull << (tid & 63)) - 1ull;
                        const uint32_t slot = ill ? n_pass + before3i + __popcll(bl3i & lower)
                                                  : before3 + __popcll(bl3 & lower);
                        s_list[slot] = (uint8_t)me;
                        s_pub_last[me] = last;
                        s_pub_m0[me] = m_init;  // (an ill root stays in s_pub_T[me]; a bracket's lo too, its hi in s_pub_hi)
                        if (!ill && !(flags & kPubBracket)) s_pub_hi[me] = -1.f;
                    }
                    __syncthreads();
                    const bool own_in = in_range, own_refined = refined;  // (the worker role reuses them)
                    // lane groups: the pixels that need the passes (five walks and the dT/dt_m walk) get
                    // G_p lanes each, the ill-conditioned roots (the dT/dt_m walk only) G_i <= G_p, the
                    // largest powers of two with n_pass G_p + n_ill G_i <= 256 and G_i >= G_p / 8; a
                    // pixel's group is aligned (the pass groups first), so its DPP combine stays inside it
                    int lgp = kAdaptGroups ? 4 : 0;
                    while (lgp > 0 && (n_pass << lgp) + n_ill * (uint32_t)max(1, (1 << lgp) >> GSR_P3_ILL_SHIFT) > (uint32_t)kTilePixels)
                        lgp--;
                    int lgi = lgp;
                    while (lgi > 0 && (n_pass << lgp) + (n_ill << lgi) > (uint32_t)kTilePixels) lgi--;
                    const uint32_t np_lanes = n_pass << lgp;
                    if constexpr (STATS) st[17] += tid == 0 ? np_lanes + (n_ill << lgi) : 0u;
                    auto lane_group = [&](uint32_t t, int& lg) -> uint32_t {  // (listed pixel of lane t, its group log2)
                        const bool is_p = t < np_lanes;
                        lg = is_p ? lgp : lgi;
                        return is_p ? (t >> lgp) : n_pass + ((t - np_lanes) >> lgi);
                    };
                    int lg3;
                    const uint32_t e3 = lane_group((uint32_t)tid, lg3);
                    const int G3 = 1 << lg3;
                    const bool work = e3 < n_left;
                    const bool work_pass = e3 < n_pass;
                    if (__ballot(work) != 0ull) {  // (waves past the list skip)
                        auto wsrc = [&] {
                            int lgw;
                            const uint32_t ew = lane_group((uint32_t)opaque_int(tid), lgw);
                            const int pp = s_list[ew];
                            return PixSrc{s_mask + pp, s_pub_last[pp], (float)(x0 + (pp & 15)), (float)(y0 + (pp >> 4)),
                                          gfilter(1 << lgw, opaque_int(tid) & ((1 << lgw) - 1))};
                        };
                        const int pw = work ? (int)s_list[e3] : 0;
                        const float wm0 = s_pub_m0[pw];
                        in_range = work_pass;
                        refined = false;
                        if (__ballot(work_pass) != 0ull) {
                            if constexpr (STATS) {
                                if ((tid & 63) == 0) st[5] += 1;
                            }
                            dmin = fmaxf(wm0 - a.sample_range, 0.f);
                            dmax = fmaxf(wm0 + a.sample_range, 0.f);
                            const int npass = max(a.passes, kSplitIterations);
                            // Passes decided by the bracket (round 5): where the pixel's walks left an evaluated
                            // bracket lo < root < hi (T(lo) >= 1/2 > T(hi)) that lies inside one cell of a pass,
                            // T being non-increasing that pass picks exactly that cell, so it is not evaluated:
                            // the first evaluated pass starts in the deepest such cell (all 9 of its samples, as
                            // the reference's first pass; the same depths bit for bit, so the same values as if
                            // the skipped passes had run).  A decision within rounding of the bracket's ends is a
                            // float64 near-tie either way (tests/flip_audit.py).
                            int skip = 0;
                            const float bhi = work_pass ? s_pub_hi[pw] : -1.f;
                            if (GSR_PASS_SKIP && bhi >= 0.f) {
                                const float blo = s_pub_T[pw];
                                const float mg = 1e-6f * fmaxf(bhi, 1.f);
#pragma unroll 1
                                for (int lv = 0; lv < npass - 1; lv++) {
                                    const float iv = (dmax - dmin) * (1.f / (float)kSplit);
                                    int kc = -1;
#pragma unroll
                                    for (int c = 0; c < kSplit; c++) {
                                        const float c0 = __builtin_fmaf(iv, (float)c, dmin);
                                        const float c1 = __builtin_fmaf(iv, (float)(c + 1), dmin);
                                        kc = (c0 <= blo - mg && c1 >= bhi + mg) ? c : kc;
                                    }
                                    if (kc < 0) break;
                                    dmax = __builtin_fmaf((float)(kc + 1), iv, dmin);
                                    dmin = __builtin_fmaf((float)kc, iv, dmin);
                                    skip++;
                                }
                            }
                            if constexpr (STATS) {
                                if (work_pass && (tid & (G3 - 1)) == 0) {
                                    st[18] += (unsigned long long)skip;
                                    st[19] += skip > 0 ? 1ull : 0ull;
                                }
                            }
                            pass(std::true_type{}, wsrc, G3, true);
#pragma unroll 1
                            for (int it = 1; it < npass; it++) {
                                const bool on = it < npass - skip;
                                if (__ballot(on) == 0ull) break;
                                pass(std::false_type{}, wsrc, G3, on);
                            }
                        }
                        // the median depth and dT/dt_m as the owner path below computes them
                        float w_max = (Tp[0] - 0.5f) / (Tp[0] - Tp[kSplit]);
                        w_max = fminf(fmaxf(w_max, 0.f), 1.f);
                        const float w_min = 1.f - w_max;
                        const float md = in_range ? __builtin_fmaf(w_max, dmax, w_min * dmin) : 0.f;
                        const PixSrc ps = wsrc();
                        const float nrm = pixel_ray_norm(ps.x, ps.y, a.W, a.H, a.focal_x, a.focal_y);
                        // (an ill-conditioned root: published as the output already)
                        const bool wi = work && !work_pass;
                        const float mo = wi ? s_pub_T[pw] : md * (1.0f / nrm);
                        in_range = in_range || wi;
                        const float mb = mo * nrm;
                        float dT = 0.f;
                        walk(ps.mask, ps.plast, ps.x, ps.y, ps.filter, work && mb != 0.f && ps.plast != 0,
                             each([&](float alpha, float t_peak, float rs, float, float) {
                                 const float t_delta = (mb - t_peak) * rs;
                                 const float Gt = alpha * __expf(-0.5f * t_delta * t_delta);
                                 dT += fast_div(-0.25f * Gt, 1.f - Gt) * fabsf(t_delta) * rs;
                             }));
                        dT = gsum(dT, G3);
                        if (work) GSR_DBG(pw, "p3: pass %d m0 %.7f [%.7f %.7f] Tp0 %.7f Tp8 %.7f in %d mo %.7f dT %g\n",
                                          (int)work_pass, wm0, dmin, dmax, Tp[0], Tp[kSplit], (int)in_range, mo, dT);
                        if (work && (tid & (G3 - 1)) == 0) {
                            int lgw;
                            const int q = s_list[lane_group((uint32_t)opaque_int(tid), lgw)];
                            s_pub_T[q] = mo;
                            s_pub_m0[q] = dT;
                            s_pub_last[q] = in_range ? 1u : 0u;
                        }
                    }
                    in_range = own_in;
                    refined = own_refined;
                    __syncthreads();
                    if (left3) {
                        have_out = true;
                        md_out = s_pub_T[me];
                        md_dT = s_pub_m0[me];
                        in_range = s_pub_last[me] != 0u;
                    }
                }
            } else if (GSR_SAMPLE_GUESS) {
                stamp(2);
                // SAMPLE (round 5): the query point lies on the other view's median-depth surface, so where
                // that surface is seen from this view the root is near the point's own distance |p_view|
                // (pt_t).  The Halley walks start there — the first one also samples the window ends for
                // the reference's in_range test, as phase 2 of the render path — instead of behind a
                // 7-probe walk; the bisection fallback of root_update keeps an occluded point's far-off
                // start inside the window's bracket.
                const bool pin = T <= kMinTransmittance;
                const float lo_w = win_lo(), hi_w = win_hi();
                const float e0 = lo_w, e8 = __builtin_fmaf((hi_w - lo_w) * (1.f / (float)kSplit), (float)kSplit, lo_w);
                const float t0 = fminf(fmaxf(pt_t, e0), e8);
                // (GSR_SAMPLE_NO_ENDS: every walk the packed two-contributor walk, no window-end samples; a
                // root found well inside the first window implies the reference's in_range test, T being
                // non-increasing — the render path's phase-2 argument — and one near or past an end is left
                // to the passes, which decide in_range with their own samples)
                const Refine r = halley(own_src, 1, pin, t0, e0, e8, !kSampleNoEnds, e0, e8, pin, kSampleWalks,
                                        fmaxf(t0, 1.f), false, false);
                in_range = r.in_range;
                refined = r.refined;
                if (kSampleNoEnds && refined) {
                    const float margin = 1e-4f * fmaxf(r.t_ref, 1.f);
                    refined = r.t_ref > e0 + margin && r.t_ref < e8 - margin;
                }
                t_ref = r.t_ref;
                ref_t = r.ref_t;
                ref_D = r.ref_D;
                ref_E = r.ref_E;
                // dT/dt_m continued from the last walk over the step to the root keeps a relative error
                // ~(|step| F / D)^2 (up to kCurvTol^2 = 4e-4 by the acceptance test); the sample backward's
                // implicit gradient scales with 1 / dT/dt_m, and its parity against the exact pre-pass
                // (sample_backward.cu:77-140) sat at the 1e-4 bar (drotations, P600-W96-H64-seed1) — so a
                // root whose step is longer than kSampleDtTol of the curvature length gets the exact walk
                dt_loose = refined && fabsf(r.t_ref - r.ref_t) * r.ref_F > kSampleDtTol * r.ref_D;
                // (the continued dT/dt_m of the other refined roots taken here, as below: the passes' lane
                // groups then need no continuation state; in_range and t_ref of a refined lane stand)
                const float mb_r = in_range ? t_ref : 0.f;
                dT_pre = refined && mb_r != 0.f
                             ? (0.5f * 0.69314718055994530942f) * __builtin_fmaf(ref_E, mb_r - ref_t, -ref_D) : 0.f;
                if constexpr (STATS && !kClock) st[19] += dt_loose ? 1 : 0;
                stamp(4);
            } else {
                stamp(2);
                const Refine r = probe_refine(own_src, m_init, T, 1, kRefineWalks);
                in_range = r.in_range;
                refined = r.refined;
                t_ref = r.t_ref;
                ref_t = r.ref_t;
                ref_D = r.ref_D;
                ref_E = r.ref_E;
                stamp(4);
            }
            // lanes left: the reference's passes from its first window (render path: phase 3 above)
            const bool left = SAMPLE && in_range && !refined;
            if constexpr (STATS && SAMPLE) st[7] += left ? 1 : 0;
            if (SAMPLE && __ballot(left) != 0ull) {
                if constexpr (STATS && !kClock) st_phase = 3;  // (the passes' walks counted with walk4+)
                if constexpr (STATS) {
                    if ((tid & 63) == 0) st[5] += 1;
                }
                const int npass = max(a.passes, kSplitIterations);
                if (GSR_SAMPLE_PASS_GROUP && resident) {
                    // The wave's left points dealt to groups of 16 lanes, 4 points a round: lane q of a group
                    // walks the contributors of index % 16 == q of its point (gfilter) and the group combines
                    // by DPP (gprod) — a fixed group size, so a point's values do not depend on how many
                    // other points of its wave are left (the scratch-split test holds them bit for bit);
                    // the results go back to the owners by __shfl.  Instead of 5 passes with ~5 lanes live.
                    // (few registers stay live across the rounds: the lanes' flags as wave masks, each left
                    // point's median depth returned into its t_ref, which only refined lanes use)
                    const unsigned long long bl = __ballot(left);
                    const unsigned long long m_in = __ballot(in_range), m_ref = __ballot(refined);
                    unsigned long long m_rin = 0ull;
                    const int n = __popcll(bl);
                    const int lane = tid & 63;
#pragma unroll 1
                    for (int base = 0; base < n; base += 4) {  // (wave-uniform)
                        // (the owner of lane's group: the e-th left lane, found again at each use)
                        auto owner_of = [&](int ln) {
                            const int e = base + (ln >> 4);
                            int owner = ln;
                            unsigned long long m = bl;
                            for (int i = 0; i < n; i++) {  // (scalar loop: the i-th left lane of the wave)
                                const int o = __builtin_ctzll(m);
                                m &= m - 1ull;
                                owner = e == i ? o : owner;
                            }
                            return owner;
                        };
                        const int e = base + (lane >> 4);
                        const int owner = owner_of(lane);
                        auto gsrc = [&] {
                            const int o = owner_of(opaque_int(lane));
                            return PixSrc{s_mask + ((tid & ~63) + o), (uint32_t)__shfl((int)last, o, 64),
                                          __shfl(lane_fx(), o, 64), __shfl(lane_fy(), o, 64), gfilter(16, lane & 15)};
                        };
                        const float om = __shfl(m_init, owner, 64);
                        dmin = fmaxf(om - a.sample_range, 0.f);  // (win_lo, win_hi of the owner)
                        dmax = fmaxf(om + a.sample_range, 0.f);
                        in_range = e < n;
                        refined = false;
                        pass(std::true_type{}, gsrc, 16, true);
#pragma unroll 1
                        for (int it = 1; it < npass; it++) pass(std::false_type{}, gsrc, 16, true);
                        // the median depth as the owner path below computes it
                        float w_max = (Tp[0] - 0.5f) / (Tp[0] - Tp[kSplit]);
                        w_max = fminf(fmaxf(w_max, 0.f), 1.f);
                        const float md = in_range ? __builtin_fmaf(w_max, dmax, (1.f - w_max) * dmin) : 0.f;
                        const int rank = __popcll(bl & ((1ull << lane) - 1ull));
                        const int from = ((rank - base) << 4) & 63;
                        const float md_o = __shfl(md, from, 64);
                        const bool mine = ((bl >> lane) & 1ull) && rank >= base && rank < base + 4;
                        const bool in_o = __shfl((int)in_range, from, 64) != 0;
                        m_rin |= __ballot(mine && in_o);
                        if (mine) t_ref = md_o;
                    }
                    refined = ((m_ref >> lane) & 1ull) != 0ull;
                    in_range = ((((bl >> lane) & 1ull) ? m_rin : m_in) >> lane) & 1ull;
                    passed_grp = left;
                } else {
                    dmin = win_lo();
                    dmax = win_hi();
                    pass(std::true_type{}, own_src, 1, true);
#pragma unroll 1
                    for (int it = 1; it < npass; it++) pass(std::false_type{}, own_src, 1, true);
                }
            }
            if constexpr (SAMPLE) stamp(5);
        } else {
            dmin = win_lo();
            dmax = win_hi();
            if (a.passes > 0) pass(std::true_type{}, own_src, 1, true);
#pragma unroll 1
            for (int it = 1; it < a.passes; it++) pass(std::false_type{}, own_src, 1, true);
        }
        if constexpr (STATS) {
            stamp(7);
            if constexpr (kClock) {
#pragma unroll
                for (int k = 1; k < 8; k++) ph[k] = ph[k] ? ph[k] : ph[k - 1];  // (SAMPLE: stamps 3, 6 unset)
#pragma unroll
                for (int k = 0; k < 7; k++) st[8 + k] = (tid & 63) == 0 ? ph[k + 1] - ph[k] : 0ull;
                if constexpr (SAMPLE) {  // prologue clocks, batches, batches with the wave's lanes all done
                    st[16] = (tid & 63) == 0 ? t_pro - ph[0] : 0ull;
                    st[17] = (tid & 63) == 0 ? n_rounds : 0ull;
                    st[18] = (tid & 63) == 0 ? n_idle : 0ull;
                }
                st[15] = (tid & 63) == 0 ? ph[7] - ph[0] : 0ull;
            }
            for (int q = 0; q < kRenderStats; q++)
                if (st[q]) atomicAdd(&g_render_stats[q], st[q]);
        }
        md_in_range = in_range;
        if (!have_out) {
            float w_max = (Tp[0] - 0.5f) / (Tp[0] - Tp[kSplit]);
            w_max = fminf(fmaxf(w_max, 0.f), 1.f);  // __saturatef (NaN -> 0)
            const float w_min = 1.f - w_max;
            mDepth = in_range ? (refined || passed_grp ? t_ref : __builtin_fmaf(w_max, dmax, w_min * dmin)) : 0.f;

            // The backward's median-depth pre-pass (render_backward.cu:835-880),
            // done here while the blended set is still in LDS: dT/dt_m at the
            // depth the backward will reconstruct from the mdepth output.  The
            // backward uses it when it receives that same mdepth (md_check) and
            // recomputes it otherwise.
            float mDepth_b;
            if constexpr (SAMPLE) {
                mDepth_b = mDepth;  // the sample backward reads the median depth itself (sample_backward.cu:135)
            } else {
                const float nrm = pixel_ray_norm(lane_fx(), lane_fy(), a.W, a.H, a.focal_x, a.focal_y);
                md_out = mDepth * (1.0f / nrm);
                mDepth_b = md_out * nrm;
            }
            float dT_dtm = 0.f;
            const bool want_dT = !SAMPLE || a.query == kQuerySample;
            if (SAMPLE && GSR_SAMPLE_GUESS && refined && !dt_loose) {
                dT_dtm = dT_pre;
            } else if (refined && !dt_loose) {
                // the reference's dT/dt_m (render_backward.cu:876) is T H' ln2 = H' ln2 / 2 at T = 1/2;
                // continued to mDepth_b from the last walk: H'(t) = -D + E (t - ref_t) (|t - ref_t| <= a
                // Newton step of kRefineTol max(t, 1); the next term is ~(step / sigma)^2 relative)
                if (mDepth_b != 0.f)
                    dT_dtm = (0.5f * 0.69314718055994530942f) * __builtin_fmaf(ref_E, mDepth_b - ref_t, -ref_D);
            }
            // (SAMPLE) the exact dT/dt_m of the loose-continuation roots, per wave: those lanes' points
            // compacted into groups of G lanes (the largest power of two up to 16 that fits them all in
            // the wave), lane q of a group walking the contributors of index % G == q of its point's
            // blended set, combined by DPP (gsum) and sent back to the owner — instead of every lane of
            // the wave waiting while the few loose ones walk their whole sets (a quarter of the points
            // are loose at the sample bench, in almost every wave)
            // (GSR_SAMPLE_PASS_GROUP: the points the passes decided, whose dT/dt_m is the exact walk too)
            float dT_grp = 0.f;
            const bool grp_dT = SAMPLE && (dt_loose || (GSR_SAMPLE_PASS_GROUP && !refined));
            bool need = false;
            if constexpr (SAMPLE) {
                need = grp_dT && resident && want_dT && inside && mDepth_b != 0.f && last != 0;
                const unsigned long long bl = __ballot(need);
                if (bl != 0ull) {  // (wave-uniform)
                    const int lane = tid & 63;
                    const int n = __popcll(bl);
                    int lg = 4;
                    while (lg > 0 && (n << lg) > 64) lg--;
                    const int G = 1 << lg;
                    const int e = lane >> lg;
                    const bool work = e < n;
                    int owner = lane;
                    unsigned long long m = bl;
                    for (int i = 0; i < n; i++) {  // (scalar loop: the i-th loose lane of the wave)
                        const int o = __builtin_ctzll(m);
                        m &= m - 1ull;
                        owner = e == i ? o : owner;
                    }
                    const float ot = __shfl(mDepth_b, owner, 64);
                    const float ox = __shfl(lane_fx(), owner, 64), oy = __shfl(lane_fy(), owner, 64);
                    const uint32_t ol = (uint32_t)__shfl((int)last, owner, 64);
                    float d = 0.f;
                    if constexpr (STATS && !kClock) st_phase = 4;  // (the grouped dT walk: slots 16, 17)
                    walk(s_mask + ((tid & ~63) + owner), ol, ox, oy, gfilter(G, lane & (G - 1)), work,
                         each([&](float alpha, float t_peak, float rs, float, float) {
                             const float t_delta = (ot - t_peak) * rs;
                             const float Gt = alpha * __expf(-0.5f * t_delta * t_delta);
                             d += fast_div(-0.25f * Gt, 1.f - Gt) * fabsf(t_delta) * rs;
                         }));
                    d = gsum(d, G);
                    dT_grp = __shfl(d, __popcll(bl & ((1ull << lane) - 1ull)) << lg, 64);
                }
            }
            if (grp_dT) {
                dT_dtm = need ? dT_grp : 0.f;  // (a tile past the LDS cache: 0, and md_ok tells the backward to recompute)
            } else if (!refined && resident) {
                lane_walk(want_dT && inside && mDepth_b != 0.f && last != 0,
                          each([&](float alpha, float t_peak, float rs, float, float) {
                              const float t_delta = (mDepth_b - t_peak) * rs;
                              const float Gt = alpha * __expf(-0.5f * t_delta * t_delta);
                              dT_dtm += fast_div(-0.25f * Gt, 1.f - Gt) * fabsf(t_delta) * rs;
                          }));
            }
            md_dT = dT_dtm;
        } else {
            mDepth = 1.f;  // (render path: only md_out is used; nonzero = in range)
        }
        md_ok = resident;
    }

    if constexpr (SAMPLE && !GEOM) {
        if (inside) {  // sample_forward.cu:165-168
            a.out_points[pid] = T_pt;
            a.out_inside[pid] = 1;
        }
        if (tid == 0) a.chunk_max[chunk] = max_contrib;
        return;
    }
    if constexpr (SAMPLE) {
        if (inside && a.query == kQuerySDF) {
            // sample_forward.cu:420-427
            a.out_points[pid] = mDepth;
            a.out_sdf[pid] = mDepth - a.pt_t[pid];
            a.out_inside[pid] = (uint8_t)(md_in_range ? 1 : 0);
        } else if (inside) {
            // sample_forward.cu:647-657
            const float pnx = (pixx - (float)(a.W - 1) / 2.f) / a.focal_x;
            const float pny = (pixy - (float)(a.H - 1) / 2.f) / a.focal_y;
            const float rln = 1.0f / sqrtf(pnx * pnx + pny * pny + 1.f);
            const float depth = mDepth * rln;
            a.out_points[3 * pid + 0] = pnx * depth;
            a.out_points[3 * pid + 1] = pny * depth;
            a.out_points[3 * pid + 2] = depth;
            a.out_inside[pid] = (uint8_t)(md_in_range ? 1 : 0);
            a.pt_last[pid] = last;
            a.pt_mdepth[pid] = mDepth;
            a.pt_dT[pid] = md_dT;
            a.pt_cached[pid] = (uint8_t)(md_ok ? 1 : 0);
        }
        if (tid == 0) a.chunk_max[chunk] = max_contrib;
        return;
    }
    if (inside) {
        const int pix = a.W * lane_py() + lane_px();
        if constexpr (GEOM) {
            a.out_mdepth[pix] = md_out;
            a.dT_dtm[pix] = md_dT;
            a.md_check[pix] = md_ok ? __float_as_uint(md_out) : kNoCache;
        } else {
            const int HW = a.H * a.W;
            a.md_check[pix] = kNoCache;
            a.out_mdepth[pix] = 0.f;
            a.out_normal[pix] = 0.f;
            a.out_normal[HW + pix] = 0.f;
            a.out_normal[2 * HW + pix] = 0.f;
        }
    }
    if (tid == 0) {
        a.max_contrib[tile] = max_contrib;
        // the backward walks the blended entries of the mask plus every entry past it
        uint32_t n = max_contrib > (uint32_t)(kBlendWords * 32) ? max_contrib - (uint32_t)(kBlendWords * 32) : 0u;
#pragma unroll
        for (int q = 0; q < kBlendWords; q++) n += (uint32_t)__popc(s_union[q]);
        a.bwd_cost[tile] = n;
    }
}

hipError_t launch_render_fwd(const FwdParams& p, const GeomState& gs, const BinningState& bs, const ImageState& is,
                             const TileState& ts, float* out_color, float* out_alpha, float* out_normal,
                             float* out_mdepth, hipStream_t stream) {
    RenderFwdArgs a{};
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
    a.dT_dtm = is.dT_dtm;
    a.md_check = is.md_check;
    a.max_contrib = ts.max_contrib;
    a.blend_mask = ts.blend_mask;
    a.bwd_cost = ts.bwd_cost;
    a.tile_order = ts.order;
    a.out_color = out_color;
    a.out_alpha = out_alpha;
    a.out_normal = out_normal;
    a.out_mdepth = out_mdepth;
    a.sample_range = kSampleRange;
    a.refine = option(kOptNoRefine) ? 0 : 1;
    a.passes = kSplitIterations;
    if (a.num_tiles == 0) return hipSuccess;
    if (p.require_depth) {
        if (option(kOptRenderStats))
            hipLaunchKernelGGL((render_fwd_kernel<true, true>), dim3(a.num_tiles), dim3(kTilePixels), 0, stream, a);
        else
            hipLaunchKernelGGL((render_fwd_kernel<true>), dim3(a.num_tiles), dim3(kTilePixels), 0, stream, a);
    } else {
        hipLaunchKernelGGL((render_fwd_kernel<false>), dim3(a.num_tiles), dim3(kTilePixels), 0, stream, a);
    }
    return hipGetLastError();
}

hipError_t launch_point_fwd(int query, const FwdParams& p, const GeomState& gs, const BinningState& bs,
                            const TileState& ts, const PointState& ps, const PointBinState& pb, const SampleTiles& st,
                            const ChunkState& cs, uint32_t num_chunks, float* out0, float* out1, uint8_t* out_inside,
                            hipStream_t stream) {
    RenderFwdArgs a{};
    a.ranges = ts.ranges;
    a.point_list = bs.point_list;
    a.splats = gs.splats;
    a.W = p.W;
    a.H = p.H;
    a.grid_x = p.grid_x;
    a.num_tiles = p.grid_x * p.grid_y;
    a.focal_x = p.focal_x;
    a.focal_y = p.focal_y;
    // evaluateSDF: SPLIT_ITERATIONS + 1 passes over a +-2 SAMPLE_RANGE window (sample_forward.cu:319-320, 792)
    a.passes = query == kQuerySDF ? kSplitIterations + 1 : kSplitIterations;
    a.sample_range = query == kQuerySDF ? kSampleRange * 2.f : kSampleRange;
    a.query = query;
    a.refine = option(kOptNoRefine) ? 0 : 1;
    a.pt_t = ps.t;
    a.out_sdf = out1;
    a.num_chunks = num_chunks;
    a.chunk_off = st.chunk_off;
    a.pt_ranges = st.pt_ranges;
    a.pt_list = pb.pt_list;
    a.pt_xy = ps.xy;
    a.out_points = out0;
    a.out_inside = out_inside;
    a.pt_last = ps.last;
    a.pt_mdepth = ps.mdepth;
    a.pt_dT = ps.dT;
    a.pt_cached = ps.cached;
    a.chunk_max = cs.chunk_max;
    if (num_chunks == 0) return hipSuccess;
    if (query == kQueryIntegrate)
        hipLaunchKernelGGL((render_fwd_kernel<false, false, true>), dim3(num_chunks), dim3(kTilePixels), 0,
                           stream, a);
    else if (option(kOptRenderStats))
        hipLaunchKernelGGL((render_fwd_kernel<true, true, true>), dim3(num_chunks), dim3(kTilePixels), 0,
                           stream, a);
    else
        hipLaunchKernelGGL((render_fwd_kernel<true, false, true>), dim3(num_chunks), dim3(kTilePixels), 0,
                           stream, a);
    return hipGetLastError();
}

// LPT order: the tiles bucketed by cost (1024 buckets over [0, max cost]),
// heaviest bucket first.  The order within a bucket is whatever the LDS
// atomics give: a tile's outputs do not depend on when it runs.
__device__ __forceinline__ void tile_order_body(uint32_t n, const uint32_t* __restrict__ n_dev,
                                                const uint2* __restrict__ ranges,
                                                const uint32_t* __restrict__ max_contrib,
                                                uint32_t* __restrict__ order) {
    constexpr uint32_t kB = 1024;
    if (n_dev) n = min(n, *n_dev);  // chunk counts known on the device only
    __shared__ uint32_t s_cnt[kB];
    __shared__ uint32_t s_max[kB / 64];
    const uint32_t tid = threadIdx.x;
    auto cost = [&](uint32_t t) { return ranges ? ranges[t].y - ranges[t].x : max_contrib[t]; };
    uint32_t m = 0;
    for (uint32_t t = tid; t < n; t += kB) m = max(m, cost(t));
    m = wave_max_u(m);
    if ((tid & 63) == 0) s_max[tid >> 6] = m;
    s_cnt[tid] = 0u;
    __syncthreads();
    m = 0;
    for (uint32_t w = 0; w < kB / 64; w++) m = max(m, s_max[w]);
    const unsigned long long scale = (unsigned long long)m + 1ull;
    auto bucket = [&](uint32_t c) { return kB - 1u - (uint32_t)(((unsigned long long)c * kB) / scale); };
    for (uint32_t t = tid; t < n; t += kB) atomicAdd(&s_cnt[bucket(cost(t))], 1u);
    __syncthreads();
    // exclusive scan of the bucket counts (Hillis-Steele in LDS)
    const uint32_t own = s_cnt[tid];
    uint32_t v = own;
    for (uint32_t o = 1; o < kB; o <<= 1) {
        const uint32_t u = tid >= o ? s_cnt[tid - o] : 0u;
        __syncthreads();
        v += u;
        s_cnt[tid] = v;
        __syncthreads();
    }
    s_cnt[tid] = v - own;
    __syncthreads();
    for (uint32_t t = tid; t < n; t += kB) order[atomicAdd(&s_cnt[bucket(cost(t))], 1u)] = t;
}

__global__ void __launch_bounds__(1024) tile_order_kernel(uint32_t n, const uint32_t* __restrict__ n_dev,
                                                          const uint2* __restrict__ ranges,
                                                          const uint32_t* __restrict__ max_contrib,
                                                          uint32_t* __restrict__ order) {
    tile_order_body(n, n_dev, ranges, max_contrib, order);
}

// The backward's preparation in one launch: workgroup 0 builds the LPT tile
// order while the others clear the accumulators (a memset and the
// single-workgroup ordering kernel were two serial launches, ~23 us).
__global__ void __launch_bounds__(1024) bwd_prepare_kernel(uint4* __restrict__ zero, size_t n16, uint32_t n_tiles,
                                                           const uint32_t* __restrict__ max_contrib,
                                                           uint32_t* __restrict__ order) {
    if (blockIdx.x == 0) {
        tile_order_body(n_tiles, nullptr, nullptr, max_contrib, order);
        return;
    }
    const size_t stride = (size_t)(gridDim.x - 1) * blockDim.x;
    for (size_t i = (size_t)(blockIdx.x - 1) * blockDim.x + threadIdx.x; i < n16; i += stride)
        zero[i] = make_uint4(0u, 0u, 0u, 0u);
}

hipError_t launch_tile_order(uint32_t num_tiles, const uint2* ranges, const uint32_t* max_contrib, uint32_t* order,
                             hipStream_t stream) {
    if (num_tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, stream, num_tiles, (const uint32_t*)nullptr, ranges,
                       max_contrib, order);
    return hipGetLastError();
}

hipError_t launch_bwd_prepare(void* zero, size_t zero_bytes, uint32_t num_tiles, const uint32_t* max_contrib,
                              uint32_t* order, hipStream_t stream) {
    if (zero_bytes % 16 != 0 || ((uintptr_t)zero & 15u) != 0) return hipErrorInvalidValue;
    const size_t n16 = zero_bytes / 16;
    const uint32_t zblocks = (uint32_t)std::min<size_t>((n16 + 1023) / 1024, 1024);
    hipLaunchKernelGGL(bwd_prepare_kernel, dim3(1 + zblocks), dim3(1024), 0, stream, reinterpret_cast<uint4*>(zero),
                       n16, num_tiles, max_contrib, order);
    return hipGetLastError();
}

hipError_t launch_chunk_order(uint32_t bound, const uint32_t* n_dev, const uint32_t* chunk_max, uint32_t* order,
                              hipStream_t stream) {
    if (bound == 0) return hipSuccess;
    hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, stream, bound, n_dev, (const uint2*)nullptr,
                       chunk_max, order);
    return hipGetLastError();
}

hipError_t read_render_stats(unsigned long long* out, bool reset) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_render_stats), sizeof(unsigned long long) * kRenderStats);
    if (e == hipSuccess && reset) {
        unsigned long long z[kRenderStats] = {};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_render_stats), z, sizeof(z));
    }
    return e;
}

}  // namespace gsr
