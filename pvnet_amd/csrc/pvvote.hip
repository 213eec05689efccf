// pvvote.hip -- MI355X (gfx950, CDNA4) implementation of PVNet's pixel-wise
// RANSAC keypoint voting, exported through the C ABI in include/pvvote.h.
//
// Reference (kennege/pvnet):
//   KU  lib/ransac_voting_gpu_layer/src/ransac_voting_kernel.cu
//   BND lib/ransac_voting_gpu_layer/src/ransac_voting.cpp
//   RV  lib/ransac_voting_gpu_layer/ransac_voting_gpu.py
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared
// (see pvnet_amd/build.py).  -ffp-contract=off matters: every expression that
// restates reference arithmetic must round after each operation.  The few
// fused multiply-adds this file wants (the approximate vote test) are written
// as explicit fmaf() calls.
//
// Design notes (DESIGN.md has the long form):
//   * The (hypothesis, pixel) vote test runs in the pixel's rotated frame:
//     5 FMAs and a compare, no sqrt or division.  A rigorous error bound
//     puts a guard band around the threshold; pairs inside it, and
//     hypotheses / pixels outside the bound's domain, are re-decided with
//     the reference's exact IEEE sequence (KU:116-125), so every decision is
//     bit-identical to the reference's.
//   * v3 / EVD never materialise the [hn,vn,tn] inlier mask: the fused
//     vote/count kernel keeps per-hypothesis counts in registers (lane =
//     hypothesis, pixels broadcast from LDS).  The byte mask is produced only
//     by the API entry point voting_for_hypothesis, as coalesced 8-byte
//     stores (lane = 8 pixels, hypotheses broadcast from LDS).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <array>

#include <algorithm>
#include <type_traits>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pvvote.h"

#define PV_VERSION "pvvote 0.2 (gfx950)"

// Per-wave timestamp traces (tools/vote_trace.py, tools/compact_trace.py)
// exist only in trace builds (-DPVV_TRACE); the product kernels carry none.
#ifdef PVV_TRACE
#define PVV_TRACE_ON(a) ((a).trace != nullptr)
#else
#define PVV_TRACE_ON(a) false
#endif

namespace {

constexpr int kWave = 64;
constexpr int kCompactChunk = 256;           // pixels per compaction block (one per thread)
constexpr int kVoteChunk = 256;              // pixels per LDS-staged sub-chunk of the vote waves
// refine blocks per (image, keypoint); measured with the gathering hand-off
// (tools/ab_libs.sh, two rounds, stream images/s and sequential latency):
// 16 -> 53.8-54.0k / 47.7-48.6 us, 32 -> 53.2-53.3k / 47.5-48.2 us; with the
// round-4 ticket hand-off 8 -> 52.7k / 50.9-51.8 us, 16 -> 53.0k / 50.8-51.2,
// 32 -> 52.5-52.7k / 51.1-51.6 (the round-4 kernel itself: 52.5-52.7k / 52.1)
#ifndef PVV_REFINE_NJ
#define PVV_REFINE_NJ 16
#endif
constexpr int kRefineNJ = PVV_REFINE_NJ;
#ifndef PVV_REFINE_T
#define PVV_REFINE_T 256
#endif
// refine block threads (round 5, 16 blocks per keypoint: 256 -> 53.6-53.9k
// images/s, 512 -> 52.7-53.6k, 1024 -> 44.5k / 50.5 us; round 4, same threads
// per keypoint: 8 x 256 43.3-43.8k / 51.9 us, 16 x 128 43.0k / 53.6-53.9 us,
// 32 x 64 41.6k / 59.5 us)
constexpr int kRT = PVV_REFINE_T;
// a refine block's published partial: 5 least-squares sums (fp64) + its winner
// (ratio, index), each value as one 16-B pair of tagged 8-B granules
constexpr int kRefineGran = 6;
constexpr int kRefineLdsHyp = 1024;          // hypotheses per keypoint kept in LDS (more: k_refine_solve<true>)
// domain of the fast test's error bound
constexpr float kHypMax = 1.0e17f;           // |hx|,|hy| above -> exact-only hypothesis
constexpr float kLattice = 2.5e-6f;          // |h - round(h)| below (both axes) -> exact-only
constexpr float kN1Max = 1.0e18f;            // |direction| above -> exact-only pixel

__host__ __device__ inline int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// --------------------------------------------------------------------------
// exact reference arithmetic (contraction is off for the whole file)
// --------------------------------------------------------------------------

// KU's guards compare a float against the double 1e-6: (double)x < 1e-6 holds
// exactly when x <= 1e-6f (the float nearest 1e-6 lies below it), so the
// guard runs in f32 without the two f64 conversions (NaN: false either way)
__device__ __forceinline__ bool below_1e6(float x) { return x <= 1e-6f; }

// KU:107-125: one (h, v, t) decision.
__device__ __forceinline__ bool exact_vote(float nx, float ny, float cx, float cy, float hx, float hy,
                                           float thr) {
    float dx = hx - cx;
    float dy = hy - cy;
    float norm1 = sqrtf(nx * nx + ny * ny);
    float norm2 = sqrtf(dx * dx + dy * dy);
    if (below_1e6(norm1) || below_1e6(norm2)) return false;
    float angle_dist = (dx * nx + dy * ny) / (norm1 * norm2);
    return angle_dist > thr;
}

// exact_vote's decision for K6's one hypothesis per keypoint, settled by a
// squared comparison where that is provably the same (*und: not settled, the
// exact sequence must decide): on the domain below
// (squared norms in [1e-11, 1e18]: KU's 1e-6 guards pass, nothing over- or
// underflows) the exact sequence's angle is dot / (|n| |d|) within 4 roundings
// (2.4e-7 relative) and dot^2 / (thr^2 |n|^2 |d|^2) is within 5 roundings of
// its square, so outside a 2e-6 band around equality both decide alike;
// inside the band, outside the domain, or for thr outside [1e-3, 1] (`fast`
// false), the exact sequence decides.  `thr2` = thr * thr.
__device__ __forceinline__ void refine_vote_pre(float nx, float ny, float cx, float cy, float hx, float hy,
                                                float thr2, bool fast, bool *inl, bool *und) {
    const float dx = hx - cx, dy = hy - cy;
    const float nn1 = nx * nx + ny * ny;
    const float nn2 = dx * dx + dy * dy;
    const float dot = dx * nx + dy * ny;   // the exact sequence's numerator, bit for bit
    const bool dom = fast && nn1 >= 1e-11f && nn1 <= 1e18f && nn2 >= 1e-11f && nn2 <= 1e18f;
    const float l = dot * dot, r = thr2 * nn1 * nn2;
    const bool pos = dot > 0.f;            // else angle <= 0 < thr (or NaN): outlier
    const bool in = pos && l > r * (1.f + 2e-6f);
    const bool out = !pos || l < r * (1.f - 2e-6f);
    *inl = dom && in;
    *und = !dom || !(in || out);
}

// KU:28-48: intersection of the lines through two pixels. false = degenerate.
__device__ __forceinline__ bool exact_intersect(float dx0, float dy0, float cx0, float cy0, float dx1, float dy1,
                                                float cx1, float cy1, float *ox, float *oy) {
    float nx0 = dy0, ny0 = -dx0;
    float nx1 = dy1, ny1 = -dx1;
    float d0 = nx1 * ny0 - nx0 * ny1;
    if (below_1e6(fabsf(d0))) return false;
    float d1 = ny1 * nx0 - ny0 * nx1;
    if (below_1e6(fabsf(d1))) return false;
    float p0 = nx0 * cx0 + ny0 * cy0;
    float p1 = nx1 * cx1 + ny1 * cy1;
    *oy = (nx1 * p0 - nx0 * p1) / d0;
    *ox = (ny1 * p0 - ny0 * p1) / d1;
    return true;
}

// Is hypothesis (hx, hy) outside the fast test's domain?  Non-finite, huge, or
// within 2.5e-6 of an integer lattice point (pixel centres are integers, so
// only such hypotheses can come within the reference's norm2 < 1e-6 guard).
__device__ __forceinline__ bool hyp_exact_only(float hx, float hy) {
    bool big = !(fabsf(hx) <= kHypMax) || !(fabsf(hy) <= kHypMax);   // also NaN/inf
    bool lat = fabsf(hx - rintf(hx)) < kLattice && fabsf(hy - rintf(hy)) < kLattice;
    return big || lat;
}

__device__ __forceinline__ uint64_t ballot(bool x) { return __ballot(x); }

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

// --------------------------------------------------------------------------
// RNG (counter based; the reference uses torch's device RNG, which cannot be
// reproduced -- parity tests inject idxs / keep-masks instead)
// --------------------------------------------------------------------------
__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// 32-bit avalanche (lowbias32 constants); two rounds keyed by the seed
__host__ __device__ inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du;
    x ^= x >> 15; x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ inline int32_t rand_index(uint64_t seed, uint64_t key, int32_t n) {
    uint32_t r = hash32(hash32((uint32_t)key ^ (uint32_t)seed) + (uint32_t)(key >> 32) + (uint32_t)(seed >> 32));
    return (int32_t)(((uint64_t)r * (uint32_t)n) >> 32);
}

__device__ inline float rand_unit(uint64_t seed, uint64_t key) {
    return (float)(mix64(seed ^ mix64(key ^ 0x5bd1e995ull)) >> 40) * (1.0f / 16777216.0f);
}

// --------------------------------------------------------------------------
// masks
// --------------------------------------------------------------------------
struct MaskView {
    const void *p;
    int64_t s0, s1, s2, s3;
};

// foreground predicate.  V3: RV:533 `mask.byte()` != 0.  EVD: RV:340 `mask == 1`.
// SEG: argmax over 2 logits == 1 (torch.argmax: first max wins, NaN is max).
template <int KIND, bool EVD>
__device__ __forceinline__ bool is_fg(const MaskView &m, int b, int r, int c) {
    if constexpr (KIND == PV_MASK_SEG_F32 || KIND == PV_MASK_SEG_F16) {
        int64_t o = b * m.s0 + r * m.s2 + c * m.s3;
        float s0, s1;
        if constexpr (KIND == PV_MASK_SEG_F32) {
            s0 = ((const float *)m.p)[o];
            s1 = ((const float *)m.p)[o + m.s1];
        } else {
            s0 = __half2float(((const __half *)m.p)[o]);
            s1 = __half2float(((const __half *)m.p)[o + m.s1]);
        }
        if (isnan(s0)) return false;
        if (isnan(s1)) return true;
        return s1 > s0;
    } else {
        int64_t o = b * m.s0 + r * m.s1 + c * m.s2;
        int64_t v;
        if constexpr (KIND == PV_MASK_I64) v = ((const int64_t *)m.p)[o];
        else if constexpr (KIND == PV_MASK_I32) v = ((const int32_t *)m.p)[o];
        else v = ((const uint8_t *)m.p)[o];
        if constexpr (EVD) return v == 1;
        else return (uint8_t)v != 0;
    }
}

// --------------------------------------------------------------------------
// workspace
// --------------------------------------------------------------------------
struct Workspace {
    int32_t *counts;    // [b][vn][nh]   zeroed by k_fg_count
    uint4 *refslot;     // [b][vn][kRefineNJ][kRefineGran] zeroed by k_fg_count: k_refine_solve's tagged partials
    int32_t *dsagg;     // [b][nblk]     zeroed by k_fg_count: downsampled count + 1 per block (look-back)
    int32_t *confc;     // [b][vn][2]    zeroed by k_fg_count: v5 confidence count, ticket
    int64_t zero_words; // counts + refslot + dsagg + confc (contiguous)
    int32_t *tn;        // [b] compacted pixels (0 = image skipped)
    int32_t *fgtot;     // [b] foreground before downsampling
    int32_t *blkcnt;    // [b][nblk]
    int32_t *grpcnt;    // [b][ceil(nblk / kFgWideCPB)]: the wide k_fg_count blocks' sums (large grids only)
    uint64_t *fgbits;   // [b][nblk][4] foreground ballot of each wave of a k_fg_count block
    uint64_t *keptbits; // [b][nblk][4] downsampled images: k_compact's kept ballots (for compact_hyp)
    float4 *pex;        // [b][vn][P]   exact pixel data (cx, cy, nx, ny): reference operands
    float2 *hyp;        // [b][nh][vn]  (reference layout)
    float2 *hypv;       // [b][vn][nh]  keypoint-major copy (pre-generated hypotheses)
    size_t total;
};

Workspace carve(void *base, int b, int H, int W, int vn, int nh) {
    Workspace w{};
    int64_t P = (int64_t)H * W;
    int64_t nblk = (P + kCompactChunk - 1) / kCompactChunk;
    char *p = (char *)base;
    int64_t off = 0;
    auto take = [&](int64_t bytes) { char *q = p ? p + off : nullptr; off = align_up(off + bytes, 256); return q; };
    const int64_t ncnt = align_up((int64_t)b * vn * nh, 4);            // refslot 16-B aligned
    const int64_t nslot = (int64_t)b * vn * kRefineNJ * kRefineGran;
    w.zero_words = ncnt + 4 * nslot + b * nblk + 2 * (int64_t)b * vn;
    w.counts = (int32_t *)take(4 * w.zero_words);
    w.refslot = w.counts ? (uint4 *)(w.counts + ncnt) : nullptr;
    w.dsagg = w.counts ? (int32_t *)(w.refslot + nslot) : nullptr;
    w.confc = w.counts ? w.dsagg + b * nblk : nullptr;
    w.tn = (int32_t *)take(4 * b);
    w.fgtot = (int32_t *)take(4 * b);
    w.blkcnt = (int32_t *)take(4 * b * nblk);
    w.grpcnt = (int32_t *)take(4 * b * ((nblk + 7) / 8));
    w.fgbits = (uint64_t *)take(8 * 4 * b * nblk);
    w.keptbits = (uint64_t *)take(8 * 4 * b * nblk);
    w.pex = (float4 *)take(16 * b * vn * P);
    w.hyp = (float2 *)take(8 * (int64_t)b * nh * vn);
    w.hypv = (float2 *)take(8 * (int64_t)b * nh * vn);
    w.total = (size_t)off;
    return w;
}

// agent-scope (device-wide) relaxed atomics for the in-kernel hand-offs
template <typename T>
__device__ __forceinline__ void st_agent(T *p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename T>
__device__ __forceinline__ T ld_agent(const T *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// --------------------------------------------------------------------------
// block helpers (256 threads = 4 waves)
// --------------------------------------------------------------------------
// wave sums (every lane gets the sum): DPP within each 16-lane row, then
// v_permlane16_swap / v_permlane32_swap across rows -- no ds_bpermute round
// trips (six serial LDS latencies in the __shfl_xor form)
template <int CTRL>
__device__ __forceinline__ int dpp_i(int x) { return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, true); }
__device__ __forceinline__ int wave_sum_i(int x) {
    x += dpp_i<0xB1>(x);
    x += dpp_i<0x4E>(x);
    x += dpp_i<0x141>(x);
    x += dpp_i<0x140>(x);
    const auto r16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    x = (int)(r16[0] + r16[1]);
    const auto r32 = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return (int)(r32[0] + r32[1]);
}
// inclusive prefix sum over the wave by DPP: row_shr 1/2/4/8 within each
// 16-lane row (bound_ctrl: lanes past the row start add 0), then row_bcast15
// (rows 1, 3) and row_bcast31 (rows 2, 3) -- no ds_bpermute round trips
// (the __shfl_up form is six serial LDS latencies)
__device__ __forceinline__ int wave_incl_scan_i(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);
    return x;
}
__device__ __forceinline__ double wave_sum_d(double x) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}
// sum over each 16-lane row of the wave (every lane of a row gets its row's
// sum) by DPP moves: xor 1, xor 2, half-row mirror, row mirror -- VALU
// operations, not the LDS-routed ds_bpermute of __shfl_xor
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t u) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, true);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t row_max_u64(uint64_t x) {
    uint64_t o;
    o = dpp_u64<0xB1>(x); x = o > x ? o : x;
    o = dpp_u64<0x4E>(x); x = o > x ? o : x;
    o = dpp_u64<0x141>(x); x = o > x ? o : x;
    o = dpp_u64<0x140>(x); x = o > x ? o : x;
    return x;
}
__device__ __forceinline__ double row_sum_d(double x) {
    x += dpp_d<0xB1>(x);    // quad_perm [1,0,3,2]
    x += dpp_d<0x4E>(x);    // quad_perm [2,3,0,1]
    x += dpp_d<0x141>(x);   // row_half_mirror: quad q <-> 1-q within each half row
    x += dpp_d<0x140>(x);   // row_mirror: half rows swapped
    return x;
}
// sum over the block of (x, y); `sh` holds >= 8 ints
__device__ __forceinline__ int2 block_sum2(int x, int y, int *sh) {
    x = wave_sum_i(x);
    y = wave_sum_i(y);
    __syncthreads();
    if (lane_id() == 0) { sh[threadIdx.x / 64] = x; sh[4 + threadIdx.x / 64] = y; }
    __syncthreads();
    return make_int2(sh[0] + sh[1] + sh[2] + sh[3], sh[4] + sh[5] + sh[6] + sh[7]);
}

// ==========================================================================
// K1: foreground count per 256-pixel chunk (one pixel per thread and chunk)
// and the chunk's four wave ballots (k_compact reads 32 B instead of the mask
// again); zeroes the pipeline's counters.  A block takes CPB consecutive
// chunks, their mask loads issued together (clamped to the image, so no
// branch sits between them).  One chunk per block for grids that fit the
// chip at once (a one-image call: tools/lat_ab.sh, 1 chunk 52.1-52.4 us
// sequential latency, 2 chunks 52.8-53.1, 4 chunks 54.3); kFgWideCPB for
// larger grids, where one-chunk blocks -- one mask round trip each, eight
// per CU at a time -- left the kernel bound by block turnover (configs[2],
// 32 frames: 70 us).
// ==========================================================================
#ifndef PVV_FG_WIDE_ABOVE
#define PVV_FG_WIDE_ABOVE 4096
#endif
constexpr int kFgWideCPB = 8;
constexpr int64_t kFgWideAbove = PVV_FG_WIDE_ABOVE;   // blocks of one chunk above which the wide form runs
template <int KIND, bool EVD, int CPB>
__global__ __launch_bounds__(256) void k_fg_count(MaskView m, int H, int W, int32_t *blkcnt, uint64_t *fgbits,
                                                  int32_t *grpcnt, int nblk, int32_t *zero, int64_t zero_words) {
    static_assert(kCompactChunk == 256, "one pixel per thread");
    const int b = blockIdx.y, wid = threadIdx.x / 64;
    const int64_t P = (int64_t)H * W;
    {   // zero counts + tickets (read only by later kernels of this pipeline)
        int64_t g = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x;
        int64_t G = (int64_t)gridDim.x * gridDim.y * 256;
        for (int64_t i = g; i < zero_words; i += G) zero[i] = 0;
    }
    __shared__ int sh[CPB][4];
    bool f[CPB];
#pragma unroll
    for (int k = 0; k < CPB; ++k) {
        const int blk = blockIdx.x * CPB + k;
        const int64_t p = (int64_t)blk * kCompactChunk + threadIdx.x;
        const uint32_t pc = (uint32_t)min(p, P - 1);   // every load in range: none behind a branch
        const bool v = is_fg<KIND, EVD>(m, b, (int)(pc / (uint32_t)W), (int)(pc % (uint32_t)W));
        f[k] = blk < nblk && p < P && v;
    }
#pragma unroll
    for (int k = 0; k < CPB; ++k) {
        const int blk = blockIdx.x * CPB + k;   // block-uniform
        if (blk >= nblk) break;
        const uint64_t bal = ballot(f[k]);
        if (lane_id() == 0) {
            fgbits[((int64_t)b * nblk + blk) * 4 + wid] = bal;
            sh[k][wid] = __popcll(bal);
        }
    }
    __syncthreads();
    const int blk = blockIdx.x * CPB + (int)threadIdx.x;
    if (threadIdx.x < CPB && blk < nblk)
        blkcnt[b * nblk + blk] = sh[threadIdx.x][0] + sh[threadIdx.x][1] + sh[threadIdx.x][2] + sh[threadIdx.x][3];
    if (CPB > 1 && threadIdx.x == 0) {   // the block's sum: k_compact's image totals read these
        int g = 0;
#pragma unroll
        for (int k = 0; k < CPB; ++k)
            if (blockIdx.x * CPB + k < nblk) g += sh[k][0] + sh[k][1] + sh[k][2] + sh[k][3];
        grpcnt[b * gridDim.x + blockIdx.x] = g;
    }
}

// foreground total of image b from the per-block counts (every block of K1b/K2 does this)
__device__ __forceinline__ int2 image_totals(const int32_t *cnt, int nblk, int upto, int *sh) {
    int all = 0, pre = 0;
    for (int j = threadIdx.x; j < nblk; j += 256) {
        int v = cnt[j];
        all += v;
        pre += j < upto ? v : 0;
    }
    return block_sum2(all, pre, sh);
}

// ==========================================================================
// K2: row-major stream compaction (RV:548-552): coords (x=col, y=row) and the
// per-keypoint raw directions, keypoint-major so the vote waves read them
// contiguously.  Reads the [b,H,W,vn,2] view through its strides, so the
// network's NCHW vertex_pred is gathered directly (no permute copy).
// ==========================================================================
// debug-only phase stamps (s_memrealtime) of the compaction blocks; see
// pv_debug_compact_trace
#ifdef PVV_TRACE
__device__ uint64_t g_ctrace[4096 * 4];
__device__ int g_ctrace_on;
__device__ __forceinline__ void cstamp(int blk, int k) {
    if (g_ctrace_on && threadIdx.x == 0 && blk < 4096) g_ctrace[blk * 4 + k] = __builtin_amdgcn_s_memrealtime();
}
#else
__device__ __forceinline__ void cstamp(int, int) {}
#endif

struct VertexView {
    const void *p;
    int kind;
    int64_t s[5];
    int32_t extent;     // bytes spanned by one image's [h,w,vn,2] view (< 2^31: buffer-load range)
};

#ifndef PVV_COMPACT_SKIP
#define PVV_COMPACT_SKIP 1   // k_compact blocks without foreground exit at once
#endif
constexpr int kCompactKp = 12;   // keypoints whose vertex loads a compaction thread keeps in flight at once
constexpr uint64_t kLookbackSpin = 20000;   // s_memrealtime ticks (100 MHz): 200 us
__device__ int g_lb_self;   // debug (pv_debug_lookback_self): every look-back count worked out by the waiter

// one chunk (256 pixels) of image b: the whole of a k_compact block
// (block-uniform early returns; sh holds 8 ints, wcnt 4, pos 256 with TASKS)
template <int KIND, bool EVD, int VK, bool TASKS>
__device__ __forceinline__ void compact_chunk(const VertexView &vx, int H, int W, int vn, const int32_t *blkcnt,
                                              const int32_t *grpcnt, const uint64_t *fgbits, int32_t *dsagg,
                                              int nblk, int min_num, int max_num, uint64_t seed, const uint8_t *keep,
                                              int32_t *tn, int32_t *fgtot, float4 *pex, const int b, const int blk,
                                              int *sh, int *wcnt, uint16_t *pos, uint64_t *keptbits) {
    static_assert(kCompactChunk == 256, "one pixel per thread");
    const int64_t P = (int64_t)H * W;
    const int wid = threadIdx.x / 64, lane = lane_id();
    cstamp(blk, 0);
#if PVV_COMPACT_SKIP
    // a block without foreground has nothing to store; only blocks 0 and
    // nblk - 1 (which write tn / fgtot) run on.  The downsampling look-back
    // below takes such a predecessor's kept count as 0 from its k_fg_count
    // count, without waiting for it.
    if (blk != 0 && blk != nblk - 1 && blkcnt[b * nblk + blk] == 0) return;
#endif
    // one round trip: this wave's foreground ballot (k_fg_count) beside the
    // image's per-block counts (the total and this block's row-major offset)
    const uint64_t fw = fgbits[((int64_t)b * nblk + blk) * 4 + wid];
    int2 tot;
    if constexpr (TASKS) {
        // the image's total and this chunk's prefix from the wide k_fg_count
        // blocks' sums (8 chunks each) and the chunks before it in its group
        const int ng = (nblk + 7) / 8, g0 = blk / 8;
        int all = 0, pre = 0;
        for (int j = threadIdx.x; j < ng; j += 256) {
            const int v = grpcnt[b * ng + j];
            all += v;
            pre += j < g0 ? v : 0;
        }
        if (threadIdx.x < 8 && g0 * 8 + (int)threadIdx.x < blk) pre += blkcnt[b * nblk + g0 * 8 + threadIdx.x];
        tot = block_sum2(all, pre, sh);
    } else {
        tot = image_totals(blkcnt + b * nblk, nblk, blk, sh);
    }
    cstamp(blk, 1);
    const int fgb = tot.x;
    if (fgb < min_num) {
        if (blk == 0 && threadIdx.x == 0) { tn[b] = 0; fgtot[b] = fgb; }
        return;
    }
    const bool ds = fgb > max_num;
    int base = tot.y;
    if (!ds && blk == 0 && threadIdx.x == 0) {
        tn[b] = fgb;
        fgtot[b] = fgb;
    }
    const uint32_t p = (uint32_t)blk * kCompactChunk + threadIdx.x;   // H, W <= 65535: fits
    bool f = (fw >> lane) & 1;
    if (ds && f) f = keep ? keep[b * P + p] != 0 : rand_unit(seed, (uint64_t)b * P + p) < (float)max_num / (float)fgb;
    const uint64_t bal = ds ? ballot(f) : fw;
    const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
    if (lane == 0) wcnt[wid] = __popcll(bal);
    if (ds && keptbits && lane == 0) {
        // the kept ballots for compact_hyp, stored before this block's
        // look-back value is published (the barrier below orders them)
        st_agent(&keptbits[((int64_t)b * nblk + blk) * 4 + wid], bal);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // this pixel's vertex loads (all keypoints of a group in flight together),
    // issued before the block's offsets are known: buffer loads through a
    // per-image descriptor, one VGPR offset for the pixel and the keypoint /
    // component plane offsets in SGPRs (host check: the image's view spans
    // < 2 GiB)
    const int r = (int)(p / (uint32_t)W), c = (int)(p - (uint32_t)r * W);
    constexpr int ES = VK == PV_VERTEX_F32 ? 4 : 2;
    const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)((const char *)vx.p + (int64_t)b * vx.s[0] * ES), (short)0, vx.extent, 0x00020000);
    const int voff = (int)((r * vx.s[1] + c * vx.s[2]) * ES);
    float nx[kCompactKp], ny[kCompactKp];
    auto load_group = [&](int v0) {
#pragma unroll
        for (int u = 0; u < kCompactKp; ++u) {
            nx[u] = ny[u] = 0.f;
            if (f && v0 + u < vn) {
                const int so = uniform((int)((v0 + u) * vx.s[3] * ES));
                const int s4 = uniform((int)(vx.s[4] * ES));
                if constexpr (VK == PV_VERTEX_F32) {
                    nx[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vr, voff, so, 0));
                    ny[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vr, voff, so + s4, 0));
                } else {
                    nx[u] = __half2float(__ushort_as_half(__builtin_amdgcn_raw_buffer_load_b16(vr, voff, so, 0)));
                    ny[u] = __half2float(__ushort_as_half(__builtin_amdgcn_raw_buffer_load_b16(vr, voff, so + s4, 0)));
                }
            }
        }
    };
    if constexpr (!TASKS) load_group(0);
    __syncthreads();
    const int nsel = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    int off = below;
    for (int q = 0; q < wid; ++q) off += wcnt[q];
    if constexpr (TASKS) {
        if (f) pos[off] = (uint16_t)threadIdx.x;   // the block's selected pixels in rank order
    }
    if (ds) {
        // Downsampled offsets by look-back: publish this block's kept count
        // (+1, so 0 = not yet; k_fg_count zeroed the array), then add up the
        // earlier blocks' counts, waiting for each.  No dispatch order is
        // assumed: a count not seen within kLookbackSpin (a block not yet
        // scheduled) is worked out by the waiting thread itself from the
        // foreground ballots and the keep decisions, so every wait ends.
        int32_t *agg = dsagg + (int64_t)b * nblk;
        if (threadIdx.x == 0) {
            st_agent(&agg[blk], nsel + 1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const bool self_all = g_lb_self != 0;
        int pre = 0;
        // one deadline per thread (not per predecessor): after kLookbackSpin
        // the thread stops waiting and counts every unseen predecessor itself,
        // so no thread waits longer than kLookbackSpin in all
        const uint64_t t_dead = __builtin_amdgcn_s_memrealtime() + kLookbackSpin;
        for (int j = threadIdx.x; j < blk; j += 256) {
#if PVV_COMPACT_SKIP
            if (blkcnt[b * nblk + j] == 0) continue;   // no foreground: kept 0 (the block may not publish)
#endif
            int v = self_all ? 0 : ld_agent(&agg[j]);
            if (v == 0 && !self_all)
                while ((v = ld_agent(&agg[j])) == 0 && __builtin_amdgcn_s_memrealtime() < t_dead)
                    __builtin_amdgcn_s_sleep(1);
            if (v == 0) {   // block j's kept count from its ballots
                for (int q = 0; q < 4; ++q) {
                    uint64_t w = fgbits[((int64_t)b * nblk + j) * 4 + q];
                    while (w) {
                        const uint32_t pj = (uint32_t)j * kCompactChunk + q * 64 + __builtin_ctzll(w);
                        w &= w - 1;
                        v += keep ? keep[b * P + pj] != 0
                                  : rand_unit(seed, (uint64_t)b * P + pj) < (float)max_num / (float)fgb;
                    }
                }
                ++v;
            }
            pre += v - 1;
        }
        base = block_sum2(pre, 0, sh).x;
        if (blk == nblk - 1 && threadIdx.x == 0) { tn[b] = base + nsel; fgtot[b] = fgb; }
    }
    cstamp(blk, 2);
    // the selected pixel's records at t = base + its rank: consecutive
    // selected pixels write consecutive records of each keypoint
    float4 *eb = pex + (int64_t)b * vn * P;
    if constexpr (TASKS) {
        // one (selected pixel, keypoint) record per thread and pass, keypoint
        // major: the block's nsel x vn records spread over all its lanes (with
        // a sparse mask a lane-per-pixel store pass runs ~8 % of its lanes)
        __syncthreads();   // pos written
        const int n = nsel * vn;
        const int s4 = uniform((int)(vx.s[4] * ES));
        for (int i = (int)threadIdx.x; i < n; i += 256) {
            const int v = (int)((uint32_t)i / (uint32_t)nsel), k = i - v * nsel;
            const uint32_t pp = (uint32_t)blk * kCompactChunk + pos[k];
            const int rr = (int)(pp / (uint32_t)W), cc = (int)(pp - (uint32_t)rr * W);
            const int vo = (int)((rr * vx.s[1] + cc * vx.s[2] + v * vx.s[3]) * ES);
            float x, y;
            if constexpr (VK == PV_VERTEX_F32) {
                x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vr, vo, 0, 0));
                y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vr, vo, s4, 0));
            } else {
                x = __half2float(__ushort_as_half(__builtin_amdgcn_raw_buffer_load_b16(vr, vo, 0, 0)));
                y = __half2float(__ushort_as_half(__builtin_amdgcn_raw_buffer_load_b16(vr, vo, s4, 0)));
            }
            const int64_t t = base + k;   // (bounded as below)
            if (t < P) eb[(int64_t)v * P + t] = make_float4((float)cc, (float)rr, x, y);
        }
        cstamp(blk, 3);
        return;
    }
    const int64_t t = base + off;
    // t < fg <= P whenever the counts are this call's own; the bound keeps a
    // workspace shared by two calls in flight (a caller error) from writing
    // past the image's records
    const bool store = f && t < P;
    for (int v0 = 0; v0 < vn; v0 += kCompactKp) {
        if (v0 > 0) load_group(v0);
        if (store) {
#pragma unroll
            for (int u = 0; u < kCompactKp; ++u) {
                if (v0 + u >= vn) break;
                const int64_t o = (int64_t)(v0 + u) * P + t;
                // the reference's operands only: the vote kernel makes the fast
                // test's (prep_compacted) while it stages them
                eb[o] = make_float4((float)c, (float)r, nx[u], ny[u]);
            }
        }
    }
    cstamp(blk, 3);
}

// ==========================================================================
// K3 inside K2 (round 6): the hypotheses (KU:11-49, RV:553-557) made by the
// first `nhb` blocks of k_compact's grid, beside the compaction, instead of a
// k_hyp_gen launch after it.  Everything they need is k_fg_count's (the
// kernel before): the image's chunk counts give tn and a chunk prefix (LDS),
// a pair index t finds its chunk by binary search and its pixel by a bit
// select in that chunk's four wave ballots, and the pixel's direction is read
// from the input view -- the same (col, row, nx, ny) k_compact stores as its
// record, so the hypotheses are bit-identical to k_hyp_gen's.  Downsampled
// images (fg > max_num) rank the kept pixels: kept counts from the
// compaction blocks' look-back values (a count not seen within kLookbackSpin
// is worked out from the ballots and keep decisions), kept bits by the same
// keep decision.  One dependent trip more than a compaction block (the
// ballots), one kernel fewer in the call's chain: a k_hyp_gen launch costs
// the batch-1 stream ~9 % (profiles/r06/ablation.txt).
// ==========================================================================
#ifndef PVV_HYP_FASTSEARCH
#define PVV_HYP_FASTSEARCH 0   // 1: compact_hyp with a DPP wave scan and an 8-ary chunk search (bit-identical; measured neutral)
#endif
constexpr int kHypMaxChunks = 1536;   // chunks per image the fused hypotheses handle (LDS prefix); more: k_hyp_gen
struct HypGen {
    int nhb;                    // hypothesis blocks per image (0: none, k_hyp_gen runs)
    int nh, vn, min_num, max_num;
    uint64_t seed;              // the hypotheses' counter RNG (VoteArgs::seed)
    uint64_t kseed;             // the downsampling keep decisions' (k_compact's seed)
    const int32_t *idxs;        // [b][nh][vn][2] pixel pairs, or nullptr (counter RNG)
    const uint8_t *keep;
    float2 *hyp_out;            // [b][nh][vn]
    float2 *hypv_out;           // [b][vn][nh]
    float *diag_hyp;            // [b][nh][vn][2] or nullptr
    uint64_t *keptbits;         // downsampled images: the compaction blocks' kept ballots [b][nblk][4]
};

template <int VK>
__device__ __forceinline__ void read_dir(const __amdgpu_buffer_rsrc_t &vr, int voff, int s4, float &x, float &y) {
    if constexpr (VK == PV_VERTEX_F32) {
        x = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vr, voff, 0, 0));
        y = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(vr, voff, s4, 0));
    } else {
        x = __half2float(__ushort_as_half(__builtin_amdgcn_raw_buffer_load_b16(vr, voff, 0, 0)));
        y = __half2float(__ushort_as_half(__builtin_amdgcn_raw_buffer_load_b16(vr, voff, s4, 0)));
    }
}

// the q-th set bit (0-based) of the 256-bit mask w[0..3]; q < popcount
__device__ __forceinline__ int select_bit(const uint64_t (&w)[4], int q) {
    int base = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = __popcll(w[k]);
        if (q < c) {
            uint64_t x = w[k];
            uint32_t lo = (uint32_t)x;
            int off = 0;
            if (q >= __popc(lo)) { q -= __popc(lo); lo = (uint32_t)(x >> 32); off = 32; }
            // binary descent on the 32-bit half
            int pos = 0;
#pragma unroll
            for (int sh = 16; sh >= 1; sh >>= 1) {
                const int c2 = __popc(lo & ((1u << sh) - 1u));
                if (q >= c2) { q -= c2; lo >>= sh; pos += sh; }
            }
            return base + off + pos;
        }
        q -= c;
        base += 64;
    }
    return 255;
}

template <int KIND, bool EVD, int VK>
__device__ void compact_hyp(const VertexView &vx, int H, int W, int nblk, const int32_t *blkcnt,
                            const uint64_t *fgbits, const int32_t *dsagg, int32_t *pre, int *sh, const HypGen &g,
                            int b, int hb) {
    const int64_t P = (int64_t)H * W;
    const int per = (nblk + 255) / 256;            // consecutive chunks per thread (<= 6)
    // ---- the image's chunk counts and their exclusive prefix (one trip)
    int c[6];
    const int j0 = (int)threadIdx.x * per;
#pragma unroll
    for (int k = 0; k < 6; ++k) c[k] = k < per && j0 + k < nblk ? blkcnt[b * nblk + j0 + k] : 0;
    auto scan = [&](int (&v)[6]) -> int {        // block exclusive scan into pre[], returns the total
        int run = 0;
#pragma unroll
        for (int k = 0; k < 6; ++k) run += v[k];
        // inclusive wave scan of run (row shifts + row broadcasts)
#if PVV_HYP_FASTSEARCH
        const int x = wave_incl_scan_i(run);
#else
        int x = run;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane_id() >= o) x += y;
        }
#endif
        __syncthreads();
        if (lane_id() == 63) sh[threadIdx.x / 64] = x;
        __syncthreads();
        int wpre = 0;
        for (int w = 0; w < (int)threadIdx.x / 64; ++w) wpre += sh[w];
        const int total = sh[0] + sh[1] + sh[2] + sh[3];
        int e = wpre + x - run;
#pragma unroll
        for (int k = 0; k < 6; ++k)
            if (k < per && j0 + k < nblk) { pre[j0 + k] = e; e += v[k]; }
        if (threadIdx.x == 0) pre[nblk] = total;
        __syncthreads();
        return total;
    };
    const int fgb = scan(c);
    if (fgb < g.min_num) return;                   // tn = 0: no hypotheses (as k_hyp_gen)
    const bool ds = fgb > g.max_num;
    const float pk = (float)g.max_num / (float)fgb;
    auto kept = [&](int64_t p) -> bool {
        return g.keep ? g.keep[b * P + p] != 0 : rand_unit(g.kseed, (uint64_t)b * P + p) < pk;
    };
    int n = fgb;
    uint32_t seen = 0;                             // ds: chunks whose kept count (and ballots) were published
    if (ds) {
        // kept counts from the compaction blocks' look-back values (count + 1)
        const uint64_t t_dead = __builtin_amdgcn_s_memrealtime() + kLookbackSpin;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int j = j0 + k;
            if (!(k < per && j < nblk) || c[k] == 0) { c[k] = 0; continue; }
            int v = g_lb_self ? 0 : ld_agent(&dsagg[b * nblk + j]);
            while (v == 0 && !g_lb_self && __builtin_amdgcn_s_memrealtime() < t_dead) {
                __builtin_amdgcn_s_sleep(1);
                v = ld_agent(&dsagg[b * nblk + j]);
            }
            if (v != 0) seen |= 1u << k;
            if (v == 0) {                          // worked out from the ballots and keep decisions
                for (int q = 0; q < 4; ++q) {
                    uint64_t w = fgbits[((int64_t)b * nblk + j) * 4 + q];
                    while (w) {
                        v += kept((int64_t)j * kCompactChunk + q * 64 + __builtin_ctzll(w));
                        w &= w - 1;
                    }
                }
                ++v;
            }
            c[k] = v - 1;
        }
        n = scan(c);
        // which chunks' kept ballots are published: bit j of the LDS words
        // after pre[] (pre[nblk + 1 ...]); the rest are worked out below
        int32_t *pub = pre + nblk + 1;
        for (int q = (int)threadIdx.x; q < (nblk + 31) / 32; q += 256) pub[q] = 0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 6; ++k)
            if ((seen >> k) & 1u) atomicOr(&pub[(j0 + k) >> 5], 1 << ((j0 + k) & 31));
        __syncthreads();
    }
    n = min(n, (int)P);
    if (n <= 0) return;
    // ---- this thread's hypothesis: item i = (h, v) of image b
    const int i = hb * 256 + (int)threadIdx.x;
    if (i >= g.nh * g.vn) return;
    const int h = i / g.vn, v = i - h * g.vn;
    const int64_t gid = ((int64_t)b * g.nh + h) * g.vn + v;
    int t[2];
    if (g.idxs) {
        t[0] = min(max(g.idxs[gid * 2], 0), n - 1);
        t[1] = min(max(g.idxs[gid * 2 + 1], 0), n - 1);
    } else {
        const uint64_t key = (uint64_t)gid;
        t[0] = rand_index(g.seed, key * 2, n);
        t[1] = rand_index(g.seed, key * 2 + 1, n);
    }
    int jj[2], rr[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {                  // the last chunk with pre <= t (never an empty one)
        int lo = 0, hi = nblk - 1;
#if PVV_HYP_FASTSEARCH
        // 8-ary: seven pivots read together per step (4 dependent LDS trips
        // for 1,200 chunks instead of 11); the same index as the bisection
        while (hi - lo >= 8) {
            int pv[7], cnt = 0;
#pragma unroll
            for (int k = 0; k < 7; ++k) pv[k] = lo + (int)(((int64_t)(hi - lo) * (k + 1) + 7) / 8);
            int vv[7];
#pragma unroll
            for (int k = 0; k < 7; ++k) vv[k] = pre[pv[k]];
#pragma unroll
            for (int k = 0; k < 7; ++k) cnt += vv[k] <= t[e] ? 1 : 0;
            int nlo = lo, nhi = hi;
#pragma unroll
            for (int k = 0; k < 7; ++k) {
                if (cnt == k + 1) nlo = pv[k];
                if (cnt == k) nhi = pv[k] - 1;
            }
            lo = nlo; hi = nhi;
        }
#endif
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (pre[mid] <= t[e]) lo = mid; else hi = mid - 1;
        }
        jj[e] = lo;
        rr[e] = t[e] - pre[lo];
    }
    uint64_t w0[4], w1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        w0[q] = fgbits[((int64_t)b * nblk + jj[0]) * 4 + q];
        w1[q] = fgbits[((int64_t)b * nblk + jj[1]) * 4 + q];
    }
    if (ds) {                                      // keep only the kept pixels' bits
        const int32_t *pub = pre + nblk + 1;
        const bool p0 = g.keptbits && ((pub[jj[0] >> 5] >> (jj[0] & 31)) & 1);
        const bool p1 = g.keptbits && ((pub[jj[1] >> 5] >> (jj[1] & 31)) & 1);
        // published: the compaction block's own kept ballots (one load)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (p0) w0[q] = ld_agent(&g.keptbits[((int64_t)b * nblk + jj[0]) * 4 + q]);
            if (p1) w1[q] = ld_agent(&g.keptbits[((int64_t)b * nblk + jj[1]) * 4 + q]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (p0 && p1) break;
            uint64_t m0 = w0[q], m1 = w1[q], x0 = p0 ? 0 : w0[q], x1 = p1 ? 0 : w1[q];
            if (!p0) m0 = 0;
            if (!p1) m1 = 0;
            while (x0) { const int z = __builtin_ctzll(x0); x0 &= x0 - 1;
                         if (kept((int64_t)jj[0] * kCompactChunk + q * 64 + z)) m0 |= 1ull << z; }
            while (x1) { const int z = __builtin_ctzll(x1); x1 &= x1 - 1;
                         if (kept((int64_t)jj[1] * kCompactChunk + q * 64 + z)) m1 |= 1ull << z; }
            w0[q] = m0; w1[q] = m1;
        }
    }
    constexpr int ES = VK == PV_VERTEX_F32 ? 4 : 2;
    const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)((const char *)vx.p + (int64_t)b * vx.s[0] * ES), (short)0, vx.extent, 0x00020000);
    const int s4 = (int)(vx.s[4] * ES);
    float cx[2], cy[2], nx[2], ny[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int q = select_bit(e == 0 ? w0 : w1, rr[e]);
        const uint32_t p = (uint32_t)jj[e] * kCompactChunk + (uint32_t)q;
        const int r = (int)(p / (uint32_t)W), col = (int)(p - (uint32_t)r * W);
        cx[e] = (float)col;
        cy[e] = (float)r;
        read_dir<VK>(vr, (int)((r * vx.s[1] + col * vx.s[2] + v * vx.s[3]) * ES), s4, nx[e], ny[e]);
    }
    float x = 0.f, y = 0.f, ox, oy;
    if (exact_intersect(nx[0], ny[0], cx[0], cy[0], nx[1], ny[1], cx[1], cy[1], &ox, &oy)) { x = ox; y = oy; }
    g.hyp_out[gid] = make_float2(x, y);
    if (g.diag_hyp) { g.diag_hyp[gid * 2] = x; g.diag_hyp[gid * 2 + 1] = y; }
    g.hypv_out[((int64_t)b * g.vn + v) * g.nh + h] = make_float2(x, y);
}

// TASKS (grids above kFgWideAbove blocks, i.e. batches): the records are
// written by (pixel, keypoint) tasks spread over the block instead of by the
// pixel's own lane (configs[2]'s 32 network frames, ~8 % foreground: 69 us).
// With g.nhb > 0 the grid's first g.nhb blocks per image make the hypotheses.
template <int KIND, bool EVD, int VK, bool TASKS>
__global__ __launch_bounds__(256) void k_compact(MaskView, VertexView vx, int H, int W, int vn,
                                                 const int32_t *blkcnt, const int32_t *grpcnt,
                                                 const uint64_t *fgbits, int32_t *dsagg,
                                                 int nblk, int min_num, int max_num, uint64_t seed,
                                                 const uint8_t *keep, int32_t *tn, int32_t *fgtot, float4 *pex,
                                                 HypGen g) {
    __shared__ int sh[8];
    __shared__ int wcnt[4];
    __shared__ uint16_t pos[TASKS ? kCompactChunk : 1];
    __shared__ int32_t pre[kHypMaxChunks + 1 + (kHypMaxChunks + 31) / 32];
    if ((int)blockIdx.x < g.nhb) {
        compact_hyp<KIND, EVD, VK>(vx, H, W, nblk, blkcnt, fgbits, dsagg, pre, sh, g, (int)blockIdx.y, (int)blockIdx.x);
        return;
    }
    compact_chunk<KIND, EVD, VK, TASKS>(vx, H, W, vn, blkcnt, grpcnt, fgbits, dsagg, nblk, min_num, max_num, seed, keep, tn,
                                        fgtot, pex, (int)blockIdx.y, (int)blockIdx.x - g.nhb, sh, wcnt, pos,
                                        g.nhb > 0 ? g.keptbits : nullptr);
}

// ==========================================================================
// K4: hypotheses (KU:11-49) + fused vote/count.
// counts[b][v][h] += #{t : inlier(h, v, t)}.
//
// In the pipeline the vote kernel makes its own hypotheses (pixel pairs from
// the caller or the counter RNG, RV:553; item_hyp) in its prologue, beside
// its first pixel loads; the unit whose range starts at pixel 0 of a (b, v,
// group) stores them in the reference layout (refine stage, diagnostics).
//
// k_vote_count: lane = hypothesis (kHypLane = 2 per lane, groups of 128 per
// wave); the (image, keypoint, group, pixel) space is cut into equal
// contiguous ranges over persistent units.  With hn a multiple of 512 a unit
// is a block whose four waves take four groups against the same pixels, which
// the block stages once per 256-pixel sub-chunk in LDS; every wave then reads
// a pixel's four fast operands with one broadcast ds_read_b128, and the
// per-lane inlier count is one v_addc on the compare's VCC.
//
// The test (fast path) works in the pixel's rotated frame: with u the unit
// predicted direction and d = h - c,
//     x' = u.d,  y' = u x d,    cos(u,d) > thr  <=>  x' tau - |y'| > 0,
//     tau = sqrt(1 - thr^2) / thr   (0 < thr < 1),
// i.e. 2 subs + 4 mul/fma + 1 fma + compare: no sqrt, rsq or division.
// A pair is decided by the fast path only when |z| = |x' tau - |y'|| exceeds
// gz * D, where D >= |d| bounds the distance to every pixel of the chunk and
// gz covers both the fast path's rounding and the reference's own (<= 8 ulp
// on the cosine, KU:119-123); the rest (and hypotheses / pixels outside the
// bound's domain) are re-decided with the reference's exact sequence.  See
// DESIGN.md "Exactness of the fast vote test" for the derivation.
// ==========================================================================
// plain PODs read through the constant address space -> s_load (scalar) loads
struct alignas(16) F4 { float x, y, z, w; };
struct alignas(8) F2 { float x, y; };
// a pointer the compiler can see is wave-uniform (so loads through it become s_load)
template <typename T>
__device__ __forceinline__ T *uptr(T *p) {
    uint64_t v = (uint64_t)p;
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (T *)(((uint64_t)hi << 32) | lo);
}

struct VoteArgs {
    const float4 *pex;          // PREPPED: exact data (cx, cy, nx, ny), same layout
    const float2 *coords;       // !PREPPED: coords[b*P + t]
    const float2 *raw;          // !PREPPED: raw[b*vn*P + v*raw_v + t*raw_t]
    const float2 *hyp;          // !GEN: hyp[b*hyp_sb + v*hyp_sv + h*hyp_sh]
    float2 *hyp_out;            // GEN: generated hypotheses [b][nh][vn]
    float2 *hypv_out;           // k_hyp_gen: keypoint-major copy [b][vn][nh]
    int64_t hyp_sb, hyp_sv, hyp_sh;
    float *diag_hyp;            // GEN: optional copy [b][nh][vn][2]
    const int32_t *idxs;        // GEN: pixel pairs [b][nh][vn][2], or nullptr (counter RNG)
    int32_t *counts;            // counts[b*cnt_bs + v*cnt_v + h*cnt_h]
    const int32_t *tn_dev;      // [b] pixels per image, or nullptr (tn_host)
    uint64_t seed;
    int32_t P, raw_v, raw_t, cnt_v, cnt_h, cnt_bs;
    int32_t tn_host, b, vn, nh, hgn, fast;
    int32_t b0;                 // GEN: batch index of image 0 of this launch (RNG key: the same pairs in any chunking)
    float thr, tau, gzf, gzr;
    uint64_t *trace;            // debug: per-wave (start, end) s_memrealtime stamps, or nullptr
    int32_t rw[4];              // SH, four resident rounds of blocks: work weights per round (0: even)
};

// Share of unit w when the units come in four dispatch rounds of B = n / 4
// blocks each weighted rw[r]: a SIMD issues age-first, so a CU's first-
// dispatched block runs ahead of its later ones; weighting the earlier
// rounds more makes the four end together.  Contiguous and exact: unit w
// starts at total * (B * sum(rw[<r]) + i * rw[r]) / (B * sum(rw)).
// (rw[3] == 0: three rounds of n / 3 blocks)
__device__ __forceinline__ void round_share(uint32_t total, uint32_t n, uint32_t w, const int32_t *rw, uint32_t *lo,
                                            uint32_t *hi) {
    const uint32_t nr = rw[3] > 0 ? 4u : 3u;
    const uint64_t B = n / nr, W = (uint64_t)rw[0] + rw[1] + rw[2] + rw[3];
    auto pos = [&](uint32_t u) -> uint32_t {
        if (u >= n) return total;
        const uint32_t r = u / (uint32_t)B, i = u % (uint32_t)B;
        uint64_t pre = 0;
        for (uint32_t k = 0; k < r; ++k) pre += (uint64_t)rw[k];
        return (uint32_t)((uint64_t)total * (B * pre + (uint64_t)i * rw[r]) / (B * W));
    };
    *lo = pos(w);
    *hi = pos(w + 1);
}

// image b's compacted pixel count, clamped to [0, P]: the vote kernels size
// and index their work from it, so whatever the workspace holds (a caller
// that hands one workspace to two calls in flight), every pex / hypothesis
// index stays inside the image's P records
__device__ __forceinline__ int tn_at(const VoteArgs &a, int b) {
    const int n = a.tn_dev ? a.tn_dev[b] : a.tn_host;
    return min(max(n, 0), a.P);
}

// the reference's operands of pixel t: (cx, cy, nx, ny)
template <bool PREPPED>
__device__ __forceinline__ F4 pixel_exact(const VoteArgs &a, int b, int v, int t) {
    if (PREPPED) {
        const float4 e = a.pex[((int64_t)b * a.vn + v) * a.P + t];
        return F4{e.x, e.y, e.z, e.w};
    }
    const float2 c = a.coords[(int64_t)b * a.P + t];
    const float2 d = a.raw[(int64_t)b * a.vn * a.P + (int64_t)v * a.raw_v + (int64_t)t * a.raw_t];
    return F4{c.x, c.y, d.x, d.y};
}

// the hypothesis of lane h (exact value; (0, 0) for a degenerate pair, KU:33-41)
template <bool GEN, bool PREPPED>
__device__ __forceinline__ float2 item_hyp(const VoteArgs &a, int b, int v, int h, bool hl, int n, bool store) {
    float x = 0.f, y = 0.f;
    if (GEN) {
        if (hl) {
            int64_t gid = ((int64_t)b * a.nh + h) * a.vn + v;
            int t0, t1;
            if (a.idxs) {
                t0 = min(max(a.idxs[gid * 2], 0), n - 1);
                t1 = min(max(a.idxs[gid * 2 + 1], 0), n - 1);
            } else {
                const uint64_t key = (uint64_t)((((int64_t)a.b0 + b) * a.nh + h) * a.vn + v);
                t0 = rand_index(a.seed, key * 2, n);
                t1 = rand_index(a.seed, key * 2 + 1, n);
            }
            const F4 e0 = pixel_exact<PREPPED>(a, b, v, t0), e1 = pixel_exact<PREPPED>(a, b, v, t1);
            float ox, oy;
            if (exact_intersect(e0.z, e0.w, e0.x, e0.y, e1.z, e1.w, e1.x, e1.y, &ox, &oy)) { x = ox; y = oy; }
            if (store) {
                a.hyp_out[gid] = make_float2(x, y);
                if (a.diag_hyp) { a.diag_hyp[gid * 2] = x; a.diag_hyp[gid * 2 + 1] = y; }
            }
        }
    } else if (hl) {
        float2 q = a.hyp[b * a.hyp_sb + v * a.hyp_sv + h * a.hyp_sh];
        x = q.x; y = q.y;
    }
    return make_float2(x, y);
}

// wave w's share [lo, hi) of `total` items cut evenly over `nwaves` (32-bit: the callers keep total < 2^31)
__device__ __forceinline__ void even_share(uint32_t total, uint32_t nwaves, uint32_t w, uint32_t *lo, uint32_t *hi) {
    const uint32_t q = total / nwaves, rem = total - q * nwaves;
    *lo = w * q + min(w, rem);
    *hi = *lo + q + (w < rem ? 1u : 0u);
}

__device__ __forceinline__ float bcast(float x, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), lane));
}

// Wave-wide min / max (result in every lane), all on the VALU: DPP within
// each row of 16 lanes (quad xor 1, quad xor 2, half-row mirror, row
// mirror), then v_permlane16_swap and v_permlane32_swap across the rows
// (no LDS round trips, unlike ds_swizzle / ds_bpermute).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}
template <bool MAX>
__device__ __forceinline__ float wave_reduce(float x) {
    auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : fminf(a, b); };
    x = op(x, dpp_f<0xB1>(x));    // quad_perm [1,0,3,2]
    x = op(x, dpp_f<0x4E>(x));    // quad_perm [2,3,0,1]
    x = op(x, dpp_f<0x141>(x));   // row_half_mirror
    x = op(x, dpp_f<0x140>(x));   // row_mirror
    const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_int(x), __float_as_int(x), false, false);
    x = op(__int_as_float(r16[0]), __int_as_float(r16[1]));
    const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_int(x), __float_as_int(x), false, false);
    return op(__int_as_float(r32[0]), __int_as_float(r32[1]));
}
__device__ __forceinline__ float wave_min(float x) { return wave_reduce<false>(x); }
__device__ __forceinline__ float wave_max(float x) { return wave_reduce<true>(x); }

// fast data of one pixel from its raw direction (API path without a prepped array)
__device__ __forceinline__ float4 prep_pixel(float cx, float cy, float nx, float ny) {
    float n1 = sqrtf(nx * nx + ny * ny);                 // exactly the reference's norm1
    bool ok = !below_1e6(n1);
    double N = sqrt((double)nx * nx + (double)ny * ny);
    return make_float4(ok ? cx : __builtin_nanf(""), cy, (float)(nx / N), (float)(ny / N));
}

// fast data of a compacted pipeline pixel (cx, cy, nx, ny), made while the
// vote kernel stages it: validity by the reference's own norm1 (KU:119-121),
// the direction rounded per component after scaling by rsq (the fast test
// needs only its direction); *exo: votes, but outside the fast domain
__device__ __forceinline__ float4 prep_compacted(const F4 &e, bool *exo) {
    const float n1 = sqrtf(e.z * e.z + e.w * e.w);
    const bool valid = !below_1e6(n1);
    const float rs = __builtin_amdgcn_rsqf(fmaf(e.z, e.z, e.w * e.w));
    *exo = valid && !(n1 <= kN1Max);
    return make_float4(valid ? e.x : __builtin_nanf(""), e.y, e.z * rs, e.w * rs);
}

__device__ __forceinline__ bool pixel_exotic(float nx, float ny) {
    float n1 = sqrtf(nx * nx + ny * ny);
    return !below_1e6(n1) && !(n1 <= kN1Max);     // votes, but outside the fast domain
}

// One segment = pixels [ts, te) of one (image b, keypoint v, hypothesis group
// hg) against the group's kGroup hypotheses (kHypLane per lane).
//
// Pixels are staged per sub-chunk of 256 in two LDS slabs of the wave: the
// fast operands (ux, uy, -k1, -k2) with k1 = u.c', k2 = u x c' and c' = c - o
// relative to the sub-chunk origin o (an integer corner of its bounding box,
// so c' is exact for pixel centres), and the reference's operands (cx, cy,
// nx, ny) for the rare exact decisions.  For h' = h - o:
//     x' = u.h' - k1,  y' = u x h' - k2,  z = x' tau - |y'|
// = 4 fma + 1 fma, a compare for the count and a min for the guard band.
// The band is gzf * B + gzr * D: B >= |h'| + |c'| bounds the fast path's own
// rounding (per sub-chunk), D >= |h - c| the reference's (per 64-pixel
// quarter, from the quarter's bounding box).
constexpr int kHypLane = 2;
constexpr int kGroup = kWave * kHypLane;

// The wave's slab of exact operands.  Pipeline pixels are integer centres
// below 65536 (check_desc), packed as cx | cy << 16: 12 B per pixel keeps a
// block at 28 KiB of LDS (5 blocks per CU); API coordinates are any floats.
template <bool PACKED, int N = kVoteChunk>
struct ExactSlab {
    float2 n[N];
    uint32_t c[N];
    __device__ __forceinline__ void put(int j, const F4 &e) {
        n[j] = make_float2(e.z, e.w);
        c[j] = (uint32_t)e.x | ((uint32_t)e.y << 16);
    }
    __device__ __forceinline__ F4 get(int j) const {
        const float2 d = n[j];
        const uint32_t q = c[j];
        return F4{(float)(q & 0xffffu), (float)(q >> 16), d.x, d.y};
    }
};
template <int N>
struct ExactSlab<false, N> {
    F4 e[N];
    __device__ __forceinline__ void put(int j, const F4 &x) { e[j] = x; }
    __device__ __forceinline__ F4 get(int j) const { return e[j]; }
};

// LDS of one sub-chunk: fast operands and exact operands
template <bool PREPPED>
struct VoteSlab {
    F4 stage[kVoteChunk];
    ExactSlab<PREPPED> x;
};
// block-shared staging: the four quarter bounding boxes and exotic flags
struct QuarterBoxes {
    float4 box[4];
    uint32_t exo[4];
};

//
// SH (block-shared staging): the block's four waves take the same pixels
// against four different hypothesis groups, so a sub-chunk is loaded and
// staged once per block (one pixel per thread, double-buffered slabs, one
// barrier per sub-chunk) instead of once per wave.  Its origin is the
// sub-chunk's first pixel (known to every wave without a reduction); the
// quarter boxes come through LDS.
template <bool PREPPED, bool SH>
__device__ __forceinline__ void vote_segment(const VoteArgs &a, VoteSlab<PREPPED> *slabs, QuarterBoxes *qbs, float2 *hlds, int &buf, int b, int v, int hg,
                                             int ts, int te, int n, uint32_t rem_after, uint32_t prio_hi, uint32_t prio_mid, int &nfix,
                                             uint64_t &tloop) {
    const int lane = lane_id();
    const int wid = SH ? (int)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave) : 0;
    // Issue priority from the work this wave still has (0..3): the SIMD's
    // arbiter otherwise favours the oldest wave, so equal shares finish
    // staggered and the last waves run alone; this keeps them level.
    // (levels 0..2: 3 is the prologue's, above every hot loop; the caller's
    // thresholds are ceil(2 (total + 1) / 3) and ceil((total + 1) / 3), so
    // the comparisons need no 64-bit products: 32-bit, wave-uniform)
    auto set_prio = [&](uint32_t remaining) {
        if (remaining >= prio_hi) __builtin_amdgcn_s_setprio(2);
        else if (remaining >= prio_mid) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    };
    const float tau = a.tau;
    constexpr float kBig = 3.0e38f;

    // SH: the loads of a sub-chunk (this thread's pixel, the first pixel for
    // the origin); the first sub-chunk's are issued before the hypothesis
    // generation so that the two memory round trips overlap
    struct SubLoad {
        F4 f0, e;
    };
    auto load_sub = [&](int s0, int np) {
        SubLoad L;
        const int t = wid * kWave + lane;
        L.f0 = pixel_exact<PREPPED>(a, b, v, s0);
        L.e = F4{0.f, 0.f, 0.f, 0.f};
        if (t < np) L.e = pixel_exact<PREPPED>(a, b, v, s0 + t);
        return L;
    };
    SubLoad L;               // (loaded at the end of the previous sub-chunk: not live across its hot loop)
    if (SH) L = load_sub(ts, min(kVoteChunk, te - ts));

    // exact hypotheses (the reference's operands): SH keeps them in the wave's
    // LDS row (read per sub-chunk and by the rare exact decisions), which
    // frees their registers for the hot loop
    float2 he_r[kHypLane];
    auto he_set = [&](int i, float2 x) {
        if (SH) hlds[i * kWave + lane] = x;
        else he_r[i] = x;
    };
    auto he = [&](int i) -> float2 { return SH ? hlds[i * kWave + lane] : he_r[i]; };
    bool hf[kHypLane];       // decided by the fast test
    bool hxo[kHypLane];      // outside the fast test's domain: exact only
    int cnt[kHypLane];
#pragma unroll
    for (int i = 0; i < kHypLane; ++i) {
        const int h = hg * kGroup + i * kWave + lane;
        const bool hl = h < a.nh;
#ifndef PVVOTE_ABLATE_HYP
        // the pipeline (PREPPED) makes its hypotheses here: every block of
        // (b, v, group) intersects the same pixel pairs, the one whose range
        // starts at pixel 0 stores them (reference layout, for the refine /
        // EVD stages and the diagnostics); the API path reads the caller's
        const float2 hv = item_hyp<PREPPED, PREPPED>(a, b, v, h, hl, n, PREPPED && ts == 0);
#else
        const float2 hv = make_float2(300.f + 0.37f * lane + 0.11f * v, 200.f + 0.23f * i + 0.5f * hg);
#endif
        he_set(i, hv);
        const bool fin = isfinite(hv.x) && isfinite(hv.y);    // non-finite: never an inlier
        hxo[i] = hl && fin && hyp_exact_only(hv.x, hv.y);
        hf[i] = hl && fin && !hxo[i];
        cnt[i] = 0;
    }

    for (int s0 = ts; s0 < te; s0 += kVoteChunk) {
        const int np = min(kVoteChunk, te - s0);
        VoteSlab<PREPPED> &S = slabs[SH ? buf : 0];
        F4 *stage = S.stage;
        ExactSlab<PREPPED> &stagex = S.x;
        QuarterBoxes &QB = qbs[SH ? buf : 0];
        if (SH) buf ^= 1;
        float qxl = kBig, qxh = -kBig, qyl = kBig, qyh = -kBig;
        float cxl = kBig, cxh = -kBig, cyl = kBig, cyh = -kBig;
        float ox, oy, R;
        bool slow = !a.fast;
        if (SH) {
            const int t = wid * kWave + lane;
            ox = floorf(L.f0.x);
            oy = floorf(L.f0.y);
            if (!(fabsf(ox) <= 1.6e7f && fabsf(oy) <= 1.6e7f)) { ox = 0.f; oy = 0.f; }
            F4 q{__builtin_nanf(""), 0.f, 0.f, 0.f};
            float xl = kBig, xh = -kBig;
            bool exo_p = false;
            if (t < np) {
                const F4 e = L.e;
                if (PREPPED) {
                    const float4 f = prep_compacted(e, &exo_p);
                    q = F4{f.x, f.y, f.z, f.w};
                } else {
                    const float4 f = prep_pixel(e.x, e.y, e.z, e.w);
                    q = F4{f.x, f.y, f.z, f.w};
                    exo_p = pixel_exotic(e.z, e.w);
                }
                stagex.put(t, e);
                xl = e.x;
                xh = e.x;
            }
            {
                const float cx = q.x - ox, cy = q.y - oy;
                const float k1 = fmaf(q.z, cx, q.w * cy);
                const float k2 = fmaf(q.z, cy, -(q.w * cx));
                // a pixel that never votes (prep: cx NaN; the slab's padding):
                // u = 0, -k1 = -1e30 -> z = -1e30 tau < 0 and far outside the band
                stage[t] = q.x == q.x ? F4{q.z, q.w, -k1, -k2} : F4{0.f, 0.f, -1.0e30f, 0.f};
            }
            if (wid * kWave < np) {
                const float mn = wave_min(xl), mx = wave_max(xh);
                float yn, yx;
                if (PREPPED) {
                    yn = bcast(q.y, 0);
                    yx = bcast(q.y, min(kWave - 1, np - 1 - wid * kWave));
                } else {
                    const bool in = t < np;
                    yn = wave_min(in ? q.y : kBig);
                    yx = wave_max(in ? q.y : -kBig);
                }
                const uint32_t ex = __builtin_amdgcn_ballot_w64(exo_p) != 0;
                if (lane == 0) {
                    QB.box[wid] = make_float4(mn, mx, yn, yx);
                    QB.exo[wid] = ex;
                }
            } else if (lane == 0) {
                QB.box[wid] = make_float4(kBig, -kBig, kBig, -kBig);
                QB.exo[wid] = 0;
            }
            __syncthreads();
            uint32_t ex = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 Q = QB.box[k];
                cxl = fminf(cxl, Q.x); cxh = fmaxf(cxh, Q.y);
                cyl = fminf(cyl, Q.z); cyh = fmaxf(cyh, Q.w);
                ex |= QB.exo[k];
            }
            slow |= ex != 0;
            slow = __builtin_amdgcn_readfirstlane(slow);
            const float ax = fmaxf(cxh - ox, ox - cxl), ay = fmaxf(cyh - oy, oy - cyl);
            R = __builtin_amdgcn_sqrtf(fmaf(ax, ax, ay * ay)) * 1.00001f;
        } else {
        F4 q4[kVoteChunk / kWave];
        float xl[kVoteChunk / kWave], xh[kVoteChunk / kWave];
        bool exo_p = false;
#pragma unroll
        for (int k = 0; k < kVoteChunk / kWave; ++k) {
            const int j = k * kWave + lane;
            F4 q{__builtin_nanf(""), 0.f, 0.f, 0.f};
            xl[k] = kBig;
            xh[k] = -kBig;
            if (j < np) {
                const F4 e = pixel_exact<PREPPED>(a, b, v, s0 + j);
                if (PREPPED) {
                    bool xo;
                    const float4 f = prep_compacted(e, &xo);
                    q = F4{f.x, f.y, f.z, f.w};
                    exo_p |= xo;
                } else {
                    const float4 f = prep_pixel(e.x, e.y, e.z, e.w);
                    q = F4{f.x, f.y, f.z, f.w};
                    exo_p |= pixel_exotic(e.z, e.w);
                }
                stagex.put(j, e);
                xl[k] = e.x;
                xh[k] = e.x;
            }
            q4[k] = q;
        }
        slow |= __builtin_amdgcn_ballot_w64(exo_p) != 0;
        slow = __builtin_amdgcn_readfirstlane(slow);
        // per-quarter bounding boxes (lane k of qxl..qyh holds quarter k); the
        // compacted pixels are row-major, so a quarter's rows run from its
        // first pixel to its last (the API path takes arbitrary coordinates)
#pragma unroll
        for (int k = 0; k < kVoteChunk / kWave; ++k) {
            if (k * kWave < np) {
                const float mn = wave_min(xl[k]), mx = wave_max(xh[k]);
                float yn, yx;
                if (PREPPED) {
                    yn = bcast(q4[k].y, 0);
                    yx = bcast(q4[k].y, min(kWave - 1, np - 1 - k * kWave));
                } else {
                    const bool in = k * kWave + lane < np;
                    yn = wave_min(in ? q4[k].y : kBig);
                    yx = wave_max(in ? q4[k].y : -kBig);
                }
                if (lane == k) { qxl = mn; qxh = mx; qyl = yn; qyh = yx; }
                cxl = fminf(cxl, mn); cxh = fmaxf(cxh, mx);
                cyl = fminf(cyl, yn); cyh = fmaxf(cyh, yx);
            }
        }
        const bool empty = !(cxl <= cxh) || !(cyl <= cyh);
        ox = empty ? 0.f : floorf(cxl);
        oy = empty ? 0.f : floorf(cyl);
        R = empty ? 0.f : __builtin_amdgcn_sqrtf(fmaf(cxh - ox, cxh - ox, (cyh - oy) * (cyh - oy))) * 1.00001f;
        // stage the fast operands (ux, uy, -k1, -k2)
#pragma unroll
        for (int k = 0; k < kVoteChunk / kWave; ++k) {
            const F4 q = q4[k];
            const float cx = q.x - ox, cy = q.y - oy;          // exact for pixel centres
            const float k1 = fmaf(q.z, cx, q.w * cy);          // NaN for invalid pixels
            const float k2 = fmaf(q.z, cy, -(q.w * cx));
            stage[k * kWave + lane] = q.x == q.x ? F4{q.z, q.w, -k1, -k2} : F4{0.f, 0.f, -1.0e30f, 0.f};
        }
        __builtin_amdgcn_wave_barrier();
        }
        // lane constants of this sub-chunk
        float hx[kHypLane], hy[kHypLane], Bv[kHypLane], gd[kHypLane];
#pragma unroll
        for (int i = 0; i < kHypLane; ++i) {
            const float2 hv = he(i);
            hx[i] = hf[i] ? hv.x - ox : __builtin_nanf("");
            hy[i] = hf[i] ? hv.y - oy : __builtin_nanf("");
            Bv[i] = (__builtin_amdgcn_sqrtf(fmaf(hx[i], hx[i], hy[i] * hy[i])) + R) * 1.00001f + 1e-30f;
            gd[i] = 0.f;
        }
        // band of quarter k
        auto set_band = [&](int k) {
            float xn, xx, yn, yx;
            if (SH) {   // the block's quarter boxes are still in LDS: no registers held across the loop
                const float4 Q = QB.box[k];
                xn = Q.x - ox; xx = Q.y - ox; yn = Q.z - oy; yx = Q.w - oy;
            } else {
                xn = bcast(qxl, k) - ox; xx = bcast(qxh, k) - ox;
                yn = bcast(qyl, k) - oy; yx = bcast(qyh, k) - oy;
            }
#pragma unroll
            for (int i = 0; i < kHypLane; ++i) {
                const float ax = fmaxf(fabsf(hx[i] - xn), fabsf(hx[i] - xx));
                const float ay = fmaxf(fabsf(hy[i] - yn), fabsf(hy[i] - yx));
                const float D = fmaf(__builtin_amdgcn_sqrtf(fmaf(ax, ax, ay * ay)), 1.00001f, Bv[i] * 1e-6f);
                const float g = fmaf(a.gzr, D, a.gzf * Bv[i]);
                // a hypothesis outside the fast test (hx, hy NaN -> g NaN) gets
                // -1: its z is NaN, never counted, and it must never trigger
                // the band (the exact-only loop below decides it)
                gd[i] = g >= 0.f ? g : -1.f;
            }
        };
        if (!slow) {
            auto zval = [&](const F4 &q, float hxi, float hyi) {
                const float xr = fmaf(q.x, hxi, fmaf(q.y, hyi, q.z));      // u.h' - k1
                const float yr = fmaf(q.x, hyi, fmaf(-q.y, hxi, q.w));     // u x h' - k2
                return fmaf(xr, tau, -fabsf(yr));
            };
            // rare: some pair of pixels [j, j+4) is inside the band.  One (pixel,
            // hypothesis) pair per iteration, not unrolled, so the hot loop's
            // registers stay free; the exact operands come from the LDS slab.
            auto fix_step = [&](int j) {
#pragma unroll 1
                for (int pi = 0; pi < 4 * kHypLane; ++pi) {
                    const int p = pi / kHypLane, i = pi % kHypLane;
                    const float2 h0 = he(0);
                    float hxi = hx[0], hyi = hy[0], gdi = gd[0], ex = h0.x, ey = h0.y;
#pragma unroll
                    for (int k = 1; k < kHypLane; ++k) {
                        if (i == k) { const float2 hk = he(k); hxi = hx[k]; hyi = hy[k]; gdi = gd[k]; ex = hk.x; ey = hk.y; }
                    }
                    const float zz = zval(stage[j + p], hxi, hyi);
                    const bool u = fabsf(zz) <= gdi;
                    if (__builtin_amdgcn_ballot_w64(u)) {
                        const F4 e = stagex.get(j + p);
                        const int r = (u && exact_vote(e.z, e.w, e.x, e.y, ex, ey, a.thr)) ? 1 : 0;
                        const int f = (u && !signbit(zz)) ? 1 : 0;   // what the sign count took
#pragma unroll
                        for (int k = 0; k < kHypLane; ++k) cnt[k] += i == k ? r - f : 0;
                    }
                }
            };
            // 4 pixels x kHypLane hypotheses per step, LDS reads one step ahead
            // into two named buffers (no register copies).  The band is checked
            // once per step on min |z| per hypothesis (v_min ignores NaN, so
            // non-fast hypotheses never trigger it).
            // The fast count is a sign count: v_perm gathers the sign bytes
            // (0xff / 0x00) of 4 z values and v_sad_u8 adds them, 255 per
            // negative z -- 1 VALU op per pair instead of a compare and an
            // add-with-carry.  Pairs inside the band are re-decided by
            // fix_step, which also takes back what the sign count gave them.
            uint32_t neg[kHypLane];
#pragma unroll
            for (int i = 0; i < kHypLane; ++i) neg[i] = 0;
            uint64_t hitmask = 0;    // steps (4 pixels each) with a pair in the band
            auto step = [&](F4 q0, F4 q1, F4 q2, F4 q3, int j) {
                float m[kHypLane];
#pragma unroll
                for (int i = 0; i < kHypLane; ++i) m[i] = kBig;
                const F4 *qs[4] = {&q0, &q1, &q2, &q3};
                float z[4][kHypLane];
#pragma unroll
                for (int p = 0; p < 4; ++p) {
#pragma unroll
                    for (int i = 0; i < kHypLane; ++i) {
                        z[p][i] = zval(*qs[p], hx[i], hy[i]);
                        m[i] = fminf(m[i], fabsf(z[p][i]));
                    }
                }
#pragma unroll
                for (int i = 0; i < kHypLane; ++i) {
                    const uint32_t p01 = __builtin_amdgcn_perm(__float_as_uint(z[1][i]), __float_as_uint(z[0][i]), 0x0c0c0b09u);
                    const uint32_t p23 = __builtin_amdgcn_perm(__float_as_uint(z[3][i]), __float_as_uint(z[2][i]), 0x0b090c0cu);
                    // p01 and p23 have no byte in common: sum |p01 - p23| = sum of both
                    neg[i] = __builtin_amdgcn_sad_u8(p01, p23, neg[i]);
                }
                // (one ballot per compare: the compare's VCC is the ballot)
                uint64_t hit = 0;
#pragma unroll
                for (int i = 0; i < kHypLane; ++i) hit |= __builtin_amdgcn_ballot_w64(m[i] <= gd[i]);
                // a step with a pair in the band is only noted here (bit j / 4 of
                // a wave-uniform mask) and re-decided after the loop: the exact
                // sequence's registers are then not live beside the hot loop's
                if (hit) hitmask |= 1ull << (j >> 2);
            };
            // the slab past np holds never-voting pixels (negative z, never in
            // the band), so the loop runs whole 8-pixel iterations
#ifdef PVVOTE_ABLATE_LOOP
            const int nit = 0;
#else
            const int nit = (np + 7) >> 3;
#endif
            F4 a0 = stage[0], a1 = stage[1], a2 = stage[2], a3 = stage[3];
            if (PVV_TRACE_ON(a) && tloop == 0) tloop = __builtin_amdgcn_s_memrealtime();   // (debug traces only)
            for (int it = 0; it < nit; ++it) {
                const int j = it * 8;
                if ((j & (kWave - 1)) == 0) {
                    set_band(j / kWave);
                    set_prio(rem_after + (uint32_t)(te - s0 - j));
                }
                const F4 b0 = stage[j + 4], b1 = stage[j + 5], b2 = stage[j + 6], b3 = stage[j + 7];
                step(a0, a1, a2, a3, j);
                const int jn = (j + 8) & (kVoteChunk - 1);
                a0 = stage[jn]; a1 = stage[jn + 1]; a2 = stage[jn + 2]; a3 = stage[jn + 3];
                step(b0, b1, b2, b3, j + 4);
            }
            // the band pairs, by the reference's sequence, under the band of
            // their own quarter (set_band is deterministic: the same gd as in the loop)
            {
                uint64_t hm = hitmask;
                int kq = -1;
                while (hm) {
                    const int j = __builtin_ctzll(hm) * 4;
                    hm &= hm - 1;
                    if ((j >> 6) != kq) { kq = j >> 6; set_band(kq); }
                    ++nfix;
#ifndef PVVOTE_ABLATE_FIX   // (profiling ablation: band pairs keep the sign count's guess)
                    fix_step(j);
#endif
                }
            }
            // positives = pairs stepped - negatives (never-voting pixels and the
            // padding are negative); hypotheses outside the fast test count 0 here
#pragma unroll
            for (int i = 0; i < kHypLane; ++i) cnt[i] += hf[i] ? 8 * nit - (int)(neg[i] / 255u) : 0;
            // exact-only hypotheses (rare): lane = pixel, one hypothesis at a time
#pragma unroll
            for (int i = 0; i < kHypLane; ++i) {
                uint64_t m = __builtin_amdgcn_ballot_w64(hxo[i]);
                while (m) {
                    const int l = __builtin_ctzll(m);
                    m &= m - 1;
                    float ex, ey;
                    if (SH) { const float2 hl2 = hlds[i * kWave + l]; ex = hl2.x; ey = hl2.y; }
                    else { ex = bcast(he_r[i].x, l); ey = bcast(he_r[i].y, l); }
                    int c = 0;
#pragma unroll
                    for (int k = 0; k < kVoteChunk / kWave; ++k) {
                        const int jj = k * kWave + lane;
                        bool e = false;
                        if (jj < np) {
                            const F4 x = stagex.get(jj);
                            e = exact_vote(x.z, x.w, x.x, x.y, ex, ey, a.thr);
                        }
                        c += __popcll(__builtin_amdgcn_ballot_w64(e));
                    }
                    if (lane == l) cnt[i] += c;
                }
            }
        } else {
            // every pair through the reference sequence
#pragma unroll 1
            for (int j = 0; j < np; ++j) {
                const F4 e = stagex.get(j);
#pragma unroll
                for (int i = 0; i < kHypLane; ++i) {
                    const float2 hv = he(i);
                    cnt[i] += exact_vote(e.z, e.w, e.x, e.y, hv.x, hv.y, a.thr);
                }
            }
        }
        if (!SH) __builtin_amdgcn_wave_barrier();
        if (SH && s0 + kVoteChunk < te) L = load_sub(s0 + kVoteChunk, min(kVoteChunk, te - s0 - kVoteChunk));
    }
    int32_t *cp = a.counts + (int64_t)b * a.cnt_bs + (int64_t)v * a.cnt_v;
#pragma unroll
    for (int i = 0; i < kHypLane; ++i) {
        const int h = hg * kGroup + i * kWave + lane;
#ifndef PVVOTE_ABLATE_ATOMIC
        if (h < a.nh && cnt[i]) atomicAdd(&cp[(int64_t)h * a.cnt_h], cnt[i]);
#else
        if (h < a.nh && cnt[i] == 0x7fffffff) cp[0] = 1;
#endif
    }
}

// Balanced persistent waves: the (image, keypoint, hypothesis group, pixel)
// work space is linearised with pixels fastest and cut into equal contiguous
// ranges, one per wave, so every wave does the same number of pixel steps and
// generates each group's hypotheses once per range.  SH: the unit is a block
// (its four waves = four consecutive hypothesis groups on the same pixels),
// the space is (image, keypoint, group of four groups, pixel); needs
// hgn % 4 == 0 (hn a multiple of 512).
template <bool PREPPED, bool SH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 5))) void k_vote_count(VoteArgs a) {
    const int wave = uniform((int)(blockIdx.x * 4 + threadIdx.x / 64));
    const int unit = SH ? (int)blockIdx.x : wave;
    const int64_t nunits = SH ? (int64_t)gridDim.x : (int64_t)gridDim.x * 4;
    const int gpu = SH ? 4 : 1;           // hypothesis groups per unit
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    // the prologue (hypotheses, first sub-chunk) at the top issue priority:
    // the hot loops rank 0..2 by the work they have left (set_prio), and a
    // wave still in its prologue would otherwise wait behind them
    __builtin_amdgcn_s_setprio(3);
    __shared__ VoteSlab<PREPPED> slab_all[SH ? 2 : 4];
    __shared__ QuarterBoxes qb_all[SH ? 2 : 1];
    __shared__ float2 hyp_all[SH ? 4 * kGroup : 1];   // SH: each wave's exact hypotheses
    VoteSlab<PREPPED> *slabs = SH ? slab_all : slab_all + threadIdx.x / 64;
    int buf = 0;
    const int ggn = a.hgn / gpu;          // unit groups per keypoint
    // 32-bit index math (the host splits launches so that the work stays < 2^31)
    uint32_t total = 0;
    for (int b = 0; b < a.b; ++b) total += (uint32_t)(a.vn * ggn) * (uint32_t)tn_at(a, b);
    uint32_t lo, hi;
    if (SH && a.rw[0] > 0 && nunits % 4 == 0)
        round_share(total, (uint32_t)nunits, (uint32_t)unit, a.rw, &lo, &hi);
    else
        even_share(total, (uint32_t)nunits, (uint32_t)unit, &lo, &hi);
    // issue-priority thresholds of the wave's share (vote_segment set_prio)
    const uint32_t w1 = hi - lo + 1u;
    const uint32_t prio_hi = uniform((int)((2ull * w1 + 2) / 3)), prio_mid = uniform((int)((w1 + 2) / 3));
    int nfix = 0, nseg = 0;   // diagnostics (trace)
    uint64_t tloop = 0;       // (trace) first hot-loop entry
    // walk the segments of [lo, hi)
    int b = 0;
    uint32_t base = 0;
    while (lo < hi && b < a.b) {
        const int n = tn_at(a, b);
        const uint32_t span = (uint32_t)(a.vn * ggn) * (uint32_t)n;
        if (lo >= base + span) { base += span; ++b; continue; }
        const uint32_t r = lo - base;
        const int g = (int)(r / (uint32_t)n);               // (v, unit group) index
        const int ts = (int)(r - (uint32_t)g * n);
        const int te = (int)min((uint32_t)n, ts + (hi - lo));
        const int v = g / ggn, gg = g - v * ggn;
        const int hg = SH ? gg * 4 + (int)__builtin_amdgcn_readfirstlane(threadIdx.x / 64) : gg;
        vote_segment<PREPPED, SH>(a, slabs, qb_all, SH ? hyp_all + (threadIdx.x / 64) * kGroup : hyp_all, buf, uniform(b), uniform(v), uniform(hg), uniform(ts), uniform(te), n,
                                       uniform((int)((hi - lo) - (uint32_t)(te - ts))), prio_hi, prio_mid, nfix, tloop);
        lo += te - ts;
        ++nseg;
    }
    if (PVV_TRACE_ON(a) && lane_id() == 0) {
        uint32_t hw;
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        a.trace[wave * 8] = t_start;
        a.trace[wave * 8 + 1] = __builtin_amdgcn_s_memrealtime();
        a.trace[wave * 8 + 2] = ((uint64_t)xcc << 32) | hw;
        a.trace[wave * 8 + 3] = ((uint64_t)nseg << 32) | (uint32_t)nfix;
        a.trace[wave * 8 + 4] = tloop;
    }
}

// Hypotheses once per launch (pipeline, hyp_pregen), one thread per
// (image, hypothesis, keypoint): the pixel pair (the caller's idxs or the
// counter RNG, RV:553) and its intersection (KU:11-49), stored in the
// reference layout and keypoint-major; images without a vote are left alone.
// profiling ablations only (pv_debug_set_ablation bit 32): a launch that does nothing
__global__ void k_abl_empty(int) {}

__global__ __launch_bounds__(256) void k_hyp_gen(VoteArgs a) {
    const int64_t per = (int64_t)a.nh * a.vn;
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= per * a.b) return;
    const int b = (int)(gid / per);
    const int r = (int)(gid - b * per);
    const int h = r / a.vn, v = r - h * a.vn;
    const int n = tn_at(a, b);
    if (n > 0) a.hypv_out[((int64_t)b * a.vn + v) * a.nh + h] = item_hyp<true, true>(a, b, v, h, true, n, true);
}

// ==========================================================================
// K5m: the fused vote/count on the matrix cores (block-shared layout, hn a
// multiple of 512).  The rotated-frame test's two forms are linear in the
// hypothesis:
//     X = tau (u.h' - u.c') = a_X . h' - b_X,   a_X = tau u
//     Y =      u x h' - u x c' = a_Y . h' - b_Y,   a_Y = (-u_y, u_x)
// and z = X - |Y| (= x' tau - |y'| of the VALU kernel above).  One
// v_mfma_f32_32x32x8_f16 evaluates both forms for 16 pixels x 32 hypotheses
// (rows = (pixel, form), columns = hypotheses) from hi/lo-split fp16
// operands, K = 8:
//     row (pixel form): [ax_hi, ax_hi, ax_lo, ay_hi | ay_hi, ay_lo, -b_hi, -b_lo]
//     col (hypothesis): [hx_hi, hx_lo, hx_hi, hy_hi | hy_lo, hy_hi,  s,     s   ]
// (products of fp16 are exact in the f32 accumulation; the lo x lo terms are
// dropped; s = 2^-k keeps |h' s| < 2^14 in fp16 range).  The VALU is left with
// z = X - |Y| (one fast-rate v_sub), the sign count (v_perm + v_sad_u8) and
// the band check (v_minimum3 of |z|): ~18 instructions per 8 pairs per lane
// instead of ~54 (tools/valu_rates.hip: add/fma/or issue at ~2.7 cycles per
// wave64 instruction, min/perm/sad at ~4.3).
//
// Exactness: the MFMA path's error is bounded by gzm * |a| * B with
// B >= |h'| + |c'| (fp16 splits, the f32 sum of the
// matrix core's 8 exact products -- bounded by 16 u sum|terms| for any
// order of roundings (mfma_gz), measured within 5.2 u on 2M random sums
// (tools/mfma_probe.hip) and tested on crafted cancellation sums --, the
// rounded h', c', b and tau u); a pair is decided by the fast sign only if
// |z| > (gzm + gzr) B s (cheap per hypothesis and sub-chunk); the few that
// are not are re-checked after the sub-chunk against gzm B + gzr D with the
// pair's own distance D, and decided by the reference's sequence when
// inside it -- every decision equals KU:116-125's.
// ==========================================================================
typedef _Float16 h4f __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMB = 16;                        // pixels per MFMA batch (32 rows: 16 pixels x (X, Y))
#ifndef PVM_CHUNK
#define PVM_CHUNK 352
#endif
#ifndef PVM_QUEUE
#define PVM_QUEUE 128
#endif
#ifndef PVM_DMAX
// 1: the hot-loop band's reference-error term against the sub-chunk box's
// farthest pixel instead of B (6 % fewer flagged MFMAs on S(1234), but the
// stream measured 2 % slower: profiles/r06/vote_band_ab.txt)
#define PVM_DMAX 0
#endif
#ifndef PVM_BANDV
#define PVM_BANDV 2     // band re-check: 2 one FMA a pair to find candidates (round 6), 1 the full per-pair bound (round 5)
#endif
#if PVM_DMAX && PVM_BANDV >= 2
#error "PVM_BANDV 2 derives G from the hot-loop bound, which PVM_DMAX changes"
#endif
#ifndef PVM_ONEBAR
#define PVM_ONEBAR 0    // 1: k_vote_mfma<PREPPED> stages a sub-chunk with one barrier (origin = its first / last records' midpoint)
#endif
#ifndef PVM_HOTPRIO
#define PVM_HOTPRIO 3   // k_vote_mfma's hot-loop issue priority (the rest of the kernel runs at 3)
#endif
#ifndef PVM_BANDK
#define PVM_BANDK 1     // flagged MFMAs re-checked this many at a time (2 measured the same as 1)
#endif
// pixels per sub-chunk: a unit's range (~350 px at configs[1]) in one; 352
// (with a 128-entry band queue) keeps the block's LDS under 40 KiB, so a
// fourth block -- the next image's -- fits beside a launch's three per CU
constexpr int kMChunk = PVM_CHUNK;
constexpr int kMSlots = (kMChunk + 255) / 256; // pixels per thread in the block's staging (2)
constexpr int kMBatch = kMChunk / kMB;         // batches per sub-chunk (24)
static_assert(kMChunk % kMB == 0 && kMBatch <= 32 && kMChunk <= 512, "hit masks: 2 x 64 bits; queue: 9-bit pixel");
constexpr int kMSet = 4;                       // 32-hypothesis column sets per wave (128 hypotheses)
constexpr float kMHypMax = 8.0e6f;             // |hx|, |hy| above -> exact-only (keeps s >= 2^-9)
constexpr float kMRMax = 30000.f;              // sub-chunk radius above -> exact sub-chunk (fp16 range of b)
constexpr int kMQueue = PVM_QUEUE;             // band pairs queued per wave before a reference pass

template <bool PREPPED>
struct MSlab {
    uint4 rows[kMBatch][2 * kMB];              // [batch][row = 2 pixel + form (X, Y)]: k 0..7 as 8 halves (12 KiB)
    ExactSlab<PREPPED, kMChunk> x;
};

__device__ __forceinline__ uint32_t pack_h2(_Float16 lo, _Float16 hi) {
    return (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
}

// a row of the A operand: features of one pixel form (ax, ay, b) as 8 halves
__device__ __forceinline__ uint4 form_row(float ax, float ay, float b) {
    const _Float16 axh = (_Float16)ax, axl = (_Float16)(ax - (float)axh);
    const _Float16 ayh = (_Float16)ay, ayl = (_Float16)(ay - (float)ayh);
    const float nb = -b;
    const _Float16 bh = (_Float16)nb, bl = (_Float16)(nb - (float)bh);
    return make_uint4(pack_h2(axh, axh), pack_h2(axl, ayh), pack_h2(ayh, ayl), pack_h2(bh, bl));
}

#ifndef PVM_ALIGNED
// 1: one-image launches split along (keypoint, group) segments -- no block
// pays a second segment's prologue: the launch alone 28.1 -> 25.4 us span
// (tools/vote_trace.py), but sequential latency only 48.3-48.7 -> 48.0-48.2 us
// and the stream 54.2k -> 53.3-53.6k images/s (tools/ab_libs.sh, two rounds)
#define PVM_ALIGNED 0
#endif
#ifndef PVM_WPE
// waves per SIMD the registers are sized for.  Round 2: 3 (152 VGPRs; 4 then
// spilled across the hot loop): 40.4k -> 41.5k images/s.  Round 6: the kernel
// needs 129 at 3 -- one over the 128 that lets a fourth wave, the next
// frame's block, share the SIMD -- and fits 122 without spills at 4: the
// batch-1 stream 53.2-53.5k -> 54.2-54.6k images/s, latency unchanged
// (profiles/r06/vote_wpe_ab.txt)
#define PVM_WPE 4
#endif
#define PVM_WPE_STR2(x) #x
#define PVM_WPE_STR3(x) PVM_WPE_STR2(x)
#define PVM_WPE_STR PVM_WPE_STR3(PVM_WPE)
template <bool PREPPED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PVM_WPE, PVM_WPE))) void k_vote_mfma(VoteArgs a) {
    const int lane = lane_id();
    const int wid = (int)__builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int col = lane & 31, half = lane >> 5;
    const int unit = (int)blockIdx.x;
    const uint32_t nunits = gridDim.x;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_setprio(3);
    __shared__ MSlab<PREPPED> slab[2];
    __shared__ QuarterBoxes qb_all[2];
    __shared__ float2 hyp_all[4 * kGroup];     // each wave's 128 exact hypotheses, [set][column]
    __shared__ uint32_t bq_all[4][kMQueue];     // each wave's band pairs awaiting the reference sequence
    __shared__ int32_t corr_all[4][kGroup];     // each wave's count corrections, [set][column]
    float2 *hlds = hyp_all + wid * kGroup;
    uint32_t *bq = bq_all[wid];
    int32_t *corr = corr_all[wid];
    const int ggn = a.hgn / 4;
    uint32_t total = 0;
    for (int b = 0; b < a.b; ++b) total += (uint32_t)(a.vn * ggn) * (uint32_t)tn_at(a, b);
    uint32_t lo, hi;
    const uint32_t nsegs = (uint32_t)(a.vn * ggn);
    if (PVM_ALIGNED && a.b == 1 && a.rw[0] == 0 && nunits >= nsegs) {
        // one image: every block inside one (keypoint, 512-hypothesis group)
        // segment -- nunits / nsegs blocks per segment, the first nunits % nsegs
        // segments one more -- so that no block pays a second segment's
        // prologue (the launch's last waves were such blocks); the shares
        // differ by at most one block's part of a segment (< 1 %)
        const uint32_t base = nunits / nsegs, extra = nunits - base * nsegs;
        uint32_t sg, k, nb;
        if ((uint32_t)unit < extra * (base + 1)) {
            sg = (uint32_t)unit / (base + 1); k = (uint32_t)unit - sg * (base + 1); nb = base + 1;
        } else {
            const uint32_t u2 = (uint32_t)unit - extra * (base + 1);
            sg = extra + u2 / base; k = u2 - (u2 / base) * base; nb = base;
        }
        const uint64_t n = (uint64_t)tn_at(a, 0);
        lo = sg * (uint32_t)n + (uint32_t)(k * n / nb);
        hi = sg * (uint32_t)n + (uint32_t)((k + 1) * n / nb);
    } else if (a.rw[0] > 0 && nunits % (a.rw[3] > 0 ? 4 : 3) == 0) {
        round_share(total, nunits, (uint32_t)unit, a.rw, &lo, &hi);
    } else {
        even_share(total, nunits, (uint32_t)unit, &lo, &hi);
    }
    int buf = 0, nfix = 0, nseg = 0, nslow = 0, nxo = 0, nqd = 0;   // (nqd: band pairs queued, trace builds)
    uint64_t tloop = 0, t_total = 0, t_hyp = 0;
    uint64_t c_stage = 0, c_hot = 0, c_fix = 0, c_seg = 0, c_mark = 0;   // debug: shader cycles per phase
    uint64_t c_band = 0, c_flush = 0, c_xo = 0;                            // (trace builds: parts of c_fix)
    auto cyc = [&]() -> uint64_t { return PVV_TRACE_ON(a) ? __builtin_amdgcn_s_memtime() : 0; };
    if (PVV_TRACE_ON(a)) t_total = __builtin_amdgcn_s_memrealtime();
    const float tau = a.tau;
    constexpr float kBig = 3.0e38f;
    int b = 0;
    uint32_t base = 0;
    while (lo < hi && b < a.b) {
        const int n = tn_at(a, b);
        const uint32_t span = (uint32_t)(a.vn * ggn) * (uint32_t)n;
        if (lo >= base + span) { base += span; ++b; continue; }
        const uint32_t r0 = lo - base;
        const int g = (int)(r0 / (uint32_t)n);
        const int ts = uniform((int)(r0 - (uint32_t)g * n));
        const int te = uniform((int)min((uint32_t)n, ts + (hi - lo)));
        const int v = uniform(g / ggn), gg = g - (g / ggn) * ggn;
        const int hg = uniform(gg * 4 + wid);
        // ---- segment: pixels [ts, te) of (b, v) against hypotheses hg*128 .. +127 ----
        c_mark = cyc();
        F4 L[kMSlots];
        // (PVM_ONEBAR: the sub-chunk's first and last records, whose midpoint is
        // the origin -- row-major compacted records: a strip of rows)
        float fx0 = 0.f, fy0 = 0.f, fx1 = 0.f, fy1 = 0.f;
        auto load_px = [&](int s0, int np) {
#pragma unroll
            for (int k = 0; k < kMSlots; ++k) {
                const int t = k * 256 + wid * kWave + lane;
                L[k] = F4{0.f, 0.f, 0.f, 0.f};
                if (t < np) L[k] = pixel_exact<PREPPED>(a, b, v, s0 + t);
            }
            if (PVM_ONEBAR && PREPPED) {
                const F4 e0 = pixel_exact<PREPPED>(a, b, v, s0), e1 = pixel_exact<PREPPED>(a, b, v, s0 + np - 1);
                fx0 = e0.x; fy0 = e0.y; fx1 = e1.x; fy1 = e1.y;
            }
        };
        load_px(ts, min(kMChunk, te - ts));
        // hypotheses: lane makes h = hg*128 + i*64 + lane (i = 0, 1), stored at
        // [set 2i + half][col] -- the same linear index
        uint32_t hfm = 0, hxm = 0;              // per set: fast / exact-only (bit j)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int h = hg * kGroup + i * kWave + lane;
            const bool hl = h < a.nh;
            // pre-generated (k_hyp_gen, a.hyp keypoint-major) or made here
            const float2 hv = a.hyp ? item_hyp<false, PREPPED>(a, b, v, h, hl, n, false)
                                    : item_hyp<PREPPED, PREPPED>(a, b, v, h, hl, n, PREPPED && ts == 0);
            hlds[i * kWave + lane] = hv;
        }
        __builtin_amdgcn_wave_barrier();
        // (the exact hypotheses stay in LDS, hlds[set * 32 + col]: read where
        // needed rather than held in registers across the hot loop)
#pragma unroll
        for (int j = 0; j < kMSet; ++j) {
            const int h = hg * kGroup + j * 32 + col;
            const float2 hv = hlds[j * 32 + col];
            const bool fin = isfinite(hv.x) && isfinite(hv.y);
            const bool xo = h < a.nh && fin &&
                            (hyp_exact_only(hv.x, hv.y) || !(fabsf(hv.x) < kMHypMax && fabsf(hv.y) < kMHypMax));
            hxm |= xo ? 1u << j : 0u;
            hfm |= (h < a.nh && fin && !xo) ? 1u << j : 0u;
        }
        int cnt[kMSet] = {0, 0, 0, 0};
        corr[lane] = 0;
        corr[64 + lane] = 0;
        if (PVV_TRACE_ON(a) && t_hyp == 0) t_hyp = __builtin_amdgcn_s_memrealtime();
        for (int s0 = ts; s0 < te; s0 += kMChunk) {
            {
                const uint64_t t = cyc();
                if (s0 == ts) c_seg += t - c_mark; else c_fix += t - c_mark;
                c_mark = t;
            }
            const int np = uniform(min(kMChunk, te - s0));
            MSlab<PREPPED> &S = slab[buf];
            QuarterBoxes &QB = qb_all[buf];
            buf ^= 1;
            // ---- stage: pixels t and 256 + t of thread t; the origin is the
            // centre of the sub-chunk's bounding box (block reduce), so |c'| <= R
            // is small ----
            const int t = wid * kWave + lane;
            bool exo_p = false;
            float xl = kBig, xh = -kBig;
            float4 q[kMSlots];
            float yq[kMSlots];
#pragma unroll
            for (int k = 0; k < kMSlots; ++k) {
                const int tt = k * 256 + t;
                q[k] = make_float4(__builtin_nanf(""), 0.f, 0.f, 0.f);
                yq[k] = 0.f;
                if (tt < np) {
                    const F4 e = L[k];
                    bool ex = false;
                    if (PREPPED) q[k] = prep_compacted(e, &ex);
                    else { q[k] = prep_pixel(e.x, e.y, e.z, e.w); ex = pixel_exotic(e.z, e.w); }
                    exo_p |= ex;
                    S.x.put(tt, e);
                    xl = fminf(xl, e.x); xh = fmaxf(xh, e.x); yq[k] = q[k].y;
                }
            }
            if (wid * kWave < np) {
                const float mn = wave_min(xl), mx = wave_max(xh);
                float yn, yx;
                if (PREPPED) {
                    // rows never decrease along the compacted order: the wave's
                    // first pixel (64 wid) and its last (slot 1 when it has one)
                    yn = bcast(yq[0], 0);
                    const bool s1 = kMSlots > 1 && 256 + wid * kWave < np;
                    yx = s1 ? bcast(yq[kMSlots - 1], min(kWave - 1, np - 1 - 256 - wid * kWave))
                            : bcast(yq[0], min(kWave - 1, np - 1 - wid * kWave));
                } else {
                    float mnq = kBig, mxq = -kBig;
#pragma unroll
                    for (int k = 0; k < kMSlots; ++k)
                        if (k * 256 + t < np) { mnq = fminf(mnq, yq[k]); mxq = fmaxf(mxq, yq[k]); }
                    yn = wave_min(mnq);
                    yx = wave_max(mxq);
                }
                const uint32_t ex = __builtin_amdgcn_ballot_w64(exo_p) != 0;
                if (lane == 0) { QB.box[wid] = make_float4(mn, mx, yn, yx); QB.exo[wid] = ex; }
            } else if (lane == 0) {
                QB.box[wid] = make_float4(kBig, -kBig, kBig, -kBig);
                QB.exo[wid] = 0;
            }
            // the form rows of the sub-chunk's pixels against origin (ox, oy)
            auto put_rows = [&](float ox, float oy, bool slow) {
#pragma unroll
                for (int k = 0; k < kMSlots; ++k) {
                    const int tt = k * 256 + t;
                    if (tt >= kMChunk) break;
                    uint4 rx = make_uint4(0u, 0u, pack_h2((_Float16)0.f, (_Float16)0.f),
                                          pack_h2((_Float16)(-60000.f), (_Float16)0.f));   // never votes: X = -6e4 s
                    uint4 ry = make_uint4(0u, 0u, 0u, 0u);
                    if (q[k].x == q[k].x && !slow) {
                        const float cx = q[k].x - ox, cy = q[k].y - oy;      // exact for pixel centres
                        const float axX = tau * q[k].z, ayX = tau * q[k].w;
                        rx = form_row(axX, ayX, fmaf(axX, cx, ayX * cy));
                        ry = form_row(-q[k].w, q[k].z, fmaf(-q[k].w, cx, q[k].z * cy));
                    }
                    S.rows[tt >> 4][2 * (tt & 15)] = rx;
                    S.rows[tt >> 4][2 * (tt & 15) + 1] = ry;
                }
            };
            constexpr bool onebar = PVM_ONEBAR && PREPPED;
            float ox = 0.f, oy = 0.f;
            if constexpr (onebar) {
                // One barrier per sub-chunk: the origin is the midpoint of the
                // sub-chunk's first and last records (known to every thread
                // before any reduction), the rows are written against it
                // before the barrier, and the box reduction after it only
                // measures R about that origin (an origin anywhere keeps every
                // decision exact; a central one keeps R, so the band, small)
                ox = floorf(0.5f * fx0 + 0.5f * fx1);
                oy = floorf(0.5f * fy0 + 0.5f * fy1);
                if (!(fabsf(ox) <= 1.6e7f && fabsf(oy) <= 1.6e7f)) { ox = 0.f; oy = 0.f; }
                ox = __builtin_amdgcn_readfirstlane(ox);
                oy = __builtin_amdgcn_readfirstlane(oy);
                put_rows(ox, oy, !a.fast);
            }
            // next sub-chunk's loads, in flight across the barriers and the hot loop
            if (s0 + kMChunk < te) load_px(s0 + kMChunk, min(kMChunk, te - s0 - kMChunk));
            __syncthreads();
            float cxl = kBig, cxh = -kBig, cyl = kBig, cyh = -kBig;
            uint32_t exq = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 Q = QB.box[k];
                cxl = fminf(cxl, Q.x); cxh = fmaxf(cxh, Q.y);
                cyl = fminf(cyl, Q.z); cyh = fmaxf(cyh, Q.w);
                exq |= QB.exo[k];
            }
            if constexpr (!onebar) {
                ox = floorf(0.5f * cxl + 0.5f * cxh), oy = floorf(0.5f * cyl + 0.5f * cyh);
                if (!(fabsf(ox) <= 1.6e7f && fabsf(oy) <= 1.6e7f)) { ox = 0.f; oy = 0.f; }
            }
            const float axr = fmaxf(cxh - ox, ox - cxl), ayr = fmaxf(cyh - oy, oy - cyl);
            const float R = __builtin_amdgcn_sqrtf(fmaf(axr, axr, ayr * ayr)) * 1.00001f;
            // (the fp16 b operands reach max(tau, 1) R: tau u.c' for X, u x c' for Y)
            bool slow = !a.fast || exq != 0 || !(R * fmaxf(tau, 1.f) <= kMRMax);
            slow = __builtin_amdgcn_readfirstlane(slow);
            nslow += slow ? 1 : 0;
            if constexpr (!onebar) {
                put_rows(ox, oy, slow);
                __syncthreads();
            }
            if (!slow) {
                // ---- the hypotheses' B fragments and bands for this origin ----
                // hypothesis j's scale s = 2^-k (|h' s| < 2^14) and bound B >=
                // |h'| + |c'| + 1 (the +1 covers the fp16 subnormal terms) for
                // this origin; made again for the band pairs (not held across
                // the hot loop)
                auto hscale = [&](int j, float &hx, float &hy, float &s, float &Bv) {
                    const bool fj = (hfm >> j) & 1u;
                    const float2 hv = hlds[j * 32 + col];
                    hx = hv.x - ox;
                    hy = hv.y - oy;
                    const float mag = fmaxf(fabsf(hx), fabsf(hy));
                    const int e = __builtin_amdgcn_frexp_expf(mag);       // mag < 2^e
                    const int k = fj ? max(0, e - 14) : 0;
                    s = __builtin_ldexpf(1.f, -k);
                    Bv = (__builtin_amdgcn_sqrtf(fmaf(hx, hx, hy * hy)) * 1.00001f + R) * 1.00001f + 1.f;
                };
                h4f bf[kMSet];
                float gb[kMSet];
#pragma unroll
                for (int j = 0; j < kMSet; ++j) {
                    const bool fj = (hfm >> j) & 1u;
                    float hx, hy, s, Bv;
                    hscale(j, hx, hy, s, Bv);
                    const float hxs = hx * s, hys = hy * s;               // exact
                    const _Float16 xh_ = (_Float16)hxs, xl_ = (_Float16)(hxs - (float)xh_);
                    const _Float16 yh_ = (_Float16)hys, yl_ = (_Float16)(hys - (float)yh_);
                    const _Float16 sh = (_Float16)s;
                    h4f f = half ? h4f{yl_, yh_, sh, sh} : h4f{xh_, xl_, xh_, yh_};
                    if (!fj) f = h4f{(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
                    bf[j] = f;
#if PVM_DMAX
                    // the reference-error term against the farthest pixel the
                    // sub-chunk's box allows, not B: D <= |(|h'x| + axr, |h'y| + ayr)|
                    // <= |h'| + R (a strip of rows is wide, not tall: 15-30 %
                    // smaller for hypotheses above or below it)
                    const float ex = fabsf(hx) + axr, ey = fabsf(hy) + ayr;
                    const float Dm = __builtin_amdgcn_sqrtf(fmaf(ex, ex, ey * ey)) * 1.0001f;
                    gb[j] = fj ? (a.gzf * Bv + a.gzr * Dm) * s * 1.00001f : -1.f;
#else
                    gb[j] = fj ? (a.gzf + a.gzr) * Bv * s * 1.00001f : -1.f;
#endif
                }
                uint32_t neg[kMSet] = {0u, 0u, 0u, 0u};
                uint64_t hm0 = 0, hm1 = 0;              // band hits: bit 4 p + set, batches 0-15 / 16-31
#ifdef PVM_ABL_HOT
                const int nb = 0;
#else
                const int nb = (np + kMB - 1) / kMB;
#endif
                const uint2 *arow = (const uint2 *)&S.rows[0][0];
                // the lane's A fragment of batch p: row (col) of the batch's 32
                // rows (pixel col>>1, form col&1), k half `half`
                auto afrag = [&](int p) -> h4f {
                    const uint2 w = arow[(p * kMB * 2 + col) * 2 + half];
                    return __builtin_bit_cast(h4f, w);
                };
                auto zvals = [&](const f32x16 &c, float z[8]) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) z[q] = c[2 * q] - fabsf(c[2 * q + 1]);
                };
                // z of the lane's 8 pairs -> sign count into neg, returns min |z|
                auto proc = [&](const f32x16 &c, uint32_t &ng) -> float {
                    float z[8];
                    zvals(c, z);
#pragma unroll
                    for (int q = 0; q < 8; q += 4) {
                        const uint32_t p01 = __builtin_amdgcn_perm(__float_as_uint(z[q + 1]), __float_as_uint(z[q]), 0x0c0c0b09u);
                        const uint32_t p23 = __builtin_amdgcn_perm(__float_as_uint(z[q + 3]), __float_as_uint(z[q + 2]), 0x0b090c0cu);
                        ng = __builtin_amdgcn_sad_u8(p01, p23, ng);
                    }
                    float mb = __builtin_elementwise_minimum(__builtin_elementwise_minimum(fabsf(z[0]), fabsf(z[1])), fabsf(z[2]));
                    mb = __builtin_elementwise_minimum(__builtin_elementwise_minimum(mb, fabsf(z[3])), fabsf(z[4]));
                    mb = __builtin_elementwise_minimum(__builtin_elementwise_minimum(mb, fabsf(z[5])), fabsf(z[6]));
                    return __builtin_elementwise_minimum(mb, fabsf(z[7]));
                };
                // software pipelined: the next MFMA is in flight while the
                // previous one's results are processed, the next batch's A
                // fragment is read one batch ahead, and the band ballots of a
                // batch are taken together at its end
                const f32x16 zero = {};
                if (PVV_TRACE_ON(a) && tloop == 0) tloop = __builtin_amdgcn_s_memrealtime();
                { const uint64_t t = cyc(); c_stage += t - c_mark; c_mark = t; }
#if PVM_HOTPRIO < 3
                // the hot loop below the kernel's other phases: a wave in its
                // prologue, staging or band re-check (latency-bound chains of a
                // few instructions) issues ahead of the co-resident hot loops
                __builtin_amdgcn_s_setprio(PVM_HOTPRIO);
#endif
                h4f A = afrag(0);
                f32x16 c0 = __builtin_amdgcn_mfma_f32_32x32x8f16(A, bf[0], zero, 0, 0, 0);
#pragma unroll 1
                for (int p = 0; p < nb; ++p) {
                    const h4f An = afrag(min(p + 1, kMBatch - 1));
                    const f32x16 c1 = __builtin_amdgcn_mfma_f32_32x32x8f16(A, bf[1], zero, 0, 0, 0);
                    const float m0 = proc(c0, neg[0]);
                    const f32x16 c2 = __builtin_amdgcn_mfma_f32_32x32x8f16(A, bf[2], zero, 0, 0, 0);
                    const float m1 = proc(c1, neg[1]);
                    const f32x16 c3 = __builtin_amdgcn_mfma_f32_32x32x8f16(A, bf[3], zero, 0, 0, 0);
                    const float m2 = proc(c2, neg[2]);
                    c0 = __builtin_amdgcn_mfma_f32_32x32x8f16(An, bf[0], zero, 0, 0, 0);   // (unused after the last batch)
                    const float m3 = proc(c3, neg[3]);
                    const uint32_t hb = (__builtin_amdgcn_ballot_w64(m0 <= gb[0]) != 0 ? 1u : 0u) |
                                        (__builtin_amdgcn_ballot_w64(m1 <= gb[1]) != 0 ? 2u : 0u) |
                                        (__builtin_amdgcn_ballot_w64(m2 <= gb[2]) != 0 ? 4u : 0u) |
                                        (__builtin_amdgcn_ballot_w64(m3 <= gb[3]) != 0 ? 8u : 0u);
                    const uint64_t hbs = (uint64_t)hb << ((p & 15) * kMSet);
                    if (p < 16) hm0 |= hbs; else hm1 |= hbs;
                    A = An;
                }
#if PVM_HOTPRIO < 3
                __builtin_amdgcn_s_setprio(3);
#endif
                // positives = slots - negatives (padding and never-voting rows are negative)
#pragma unroll
                for (int j = 0; j < kMSet; ++j) cnt[j] += ((hfm >> j) & 1u) ? 8 * nb - (int)(neg[j] / 255u) : 0;
                { const uint64_t t = cyc(); c_hot += t - c_mark; c_mark = t; }
                // ---- band pairs: the same MFMA again (bit-identical); each pair
                // against its own distance, bounded from the MFMA's own forms:
                // D = |h - c| <= |x'| + |y'| = |X| / tau + |Y| (scaled by s;
                // the forms' own errors, < gzm B s, add < 1e-3 of G), and the
                // reference's sequence inside the band ----
#ifdef PVM_ABL_FIX
                nfix += __popcll(hm0) + __popcll(hm1);
                hm0 = hm1 = 0;
#endif
#ifdef PVM_ABL_FIX_RT   // the same, decided at run time (the band code stays in the kernel)
                if (a.rw[3] == 7777) hm0 = hm1 = 0;
#endif
                const float kx = a.gzr / tau * 1.0001f, ky = a.gzr * 1.0001f;
                // the queued pairs by the reference's sequence, one pair per lane;
                // a decision the sign count got wrong corrects (set, column)
                int nq = 0;
                auto flush = [&]() {
                    for (int k0 = 0; k0 < nq; k0 += kWave) {
                        if (k0 + lane < nq) {
                            const uint32_t en = bq[k0 + lane];
                            const int pix = (int)(en & 0x1ffu), jj = (int)((en >> 9) & 3u), cl = (int)((en >> 11) & 31u);
                            const int f = (int)(en >> 16) & 1;
                            const F4 e = S.x.get(pix);
                            const float2 hj = hlds[jj * 32 + cl];
                            const int r = exact_vote(e.z, e.w, e.x, e.y, hj.x, hj.y, a.thr) ? 1 : 0;
                            if (r != f) atomicAdd(&corr[jj * 32 + cl], r - f);
                        }
                    }
                    nq = 0;
                };
#if PVM_BANDV >= 2
                // Each set's per-pair constant G = gzf B s (1.001), once: from
                // the hot-loop bound gb = (gzf + gzr) B s (1.00001) with the
                // same B and s, gb gzf / (gzf + gzr) 1.0011 >= gzf B s 1.001 --
                // not an hscale (LDS read, sqrt) per flagged MFMA.
                //
                // Round 5 tested each pair against g = G + kx |X| + ky |Y|
                // (~7 VALU a pair, ~90 per flagged MFMA: the band phase was
                // 12 % of the batch-1 stream, its VALU issued beside three
                // other waves' hot loops).  Now one FMA a pair decides whether
                // any pair of the lane can be inside: |Y| <= |X| + |z| for z =
                // X - |Y| (X >= 0: |Y| = X - z; X < 0: |Y| <= |z|), so |z| <= g
                // implies |z| (1 - ky) <= G + (kx + ky) |X|, i.e. t = |z| - K |X|
                // <= G' with K = (kx + ky) / (1 - ky) and G' = G / (1 - ky)
                // (both with a 2e-4 margin that also covers t's rounding;
                // tests/test_band_filter.py checks the inclusion in float32).  The pairs with t <= G' are queued for the
                // reference's sequence: a superset of round 5's queue, so every
                // decision still equals KU's.
                // (1 / (1 - ky): ky reaches 8e-4 at thr 0.999999 -- gzr grows with 1/tau)
                const float inv1k = 1.0002f / (1.f - ky * 1.0001f);
                float Gs[kMSet];
                const float gq = a.gzf / (a.gzf + a.gzr) * 1.0011f * inv1k;
#pragma unroll
                for (int j = 0; j < kMSet; ++j) Gs[j] = gb[j] * gq;
                const float Kb = (kx + ky) * inv1k;
                auto band_test = [&](const f32x16 &c, int p, int j) {
                    const bool fj = (hfm >> j) & 1u;
                    // (selects on the wave-uniform j: a dynamic index would put Gs / bf in scratch)
                    const float G = j == 0 ? Gs[0] : j == 1 ? Gs[1] : j == 2 ? Gs[2] : Gs[3];
                    float zs[8], ts[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const float X = c[2 * q], Y = c[2 * q + 1];
                        zs[q] = X - fabsf(Y);
                        ts[q] = fmaf(-Kb, fabsf(X), fabsf(zs[q]));
                    }
                    float mt = __builtin_elementwise_minimum(__builtin_elementwise_minimum(ts[0], ts[1]), ts[2]);
                    mt = __builtin_elementwise_minimum(__builtin_elementwise_minimum(mt, ts[3]), ts[4]);
                    mt = __builtin_elementwise_minimum(__builtin_elementwise_minimum(mt, ts[5]), ts[6]);
                    mt = __builtin_elementwise_minimum(mt, ts[7]);
#ifdef PVM_ABL_Q_RT   // profiling: the candidates found but never queued (counts wrong)
                    if (a.rw[3] == 7778) mt = 3.0e38f;
#endif
                    if (__builtin_amdgcn_ballot_w64(fj && mt <= G)) {
#pragma unroll
                        for (int q = 0; q < 8; ++q) {
                            const int pix = p * kMB + (q & 1) + 4 * (q >> 1) + 2 * half;
                            const bool u = fj && pix < np && ts[q] <= G;
                            const uint64_t m = __builtin_amdgcn_ballot_w64(u);
                            if (m) {
                                if (nq > kMQueue - kWave) flush();
                                const int at = nq + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                                if (u) bq[at] = (uint32_t)pix | ((uint32_t)j << 9) | ((uint32_t)col << 11) | ((signbit(zs[q]) ? 0u : 1u) << 16);
                                nq += __popcll(m);
                                nqd += __popcll(m);
                            }
                        }
                    }
                };
                static_assert(kMSet == 4, "band selects");
                auto bsel = [&](int j) -> h4f { return j == 0 ? bf[0] : j == 1 ? bf[1] : j == 2 ? bf[2] : bf[3]; };
                while (hm0 | hm1) {
                    int pk[PVM_BANDK], jk[PVM_BANDK], nk = 0;
#pragma unroll
                    for (int k = 0; k < PVM_BANDK; ++k) {
                        pk[k] = 0; jk[k] = 0;
                        if (hm0 | hm1) {
                            int bit;
                            if (hm0) { bit = __builtin_ctzll(hm0); hm0 &= hm0 - 1; }
                            else { bit = 64 + __builtin_ctzll(hm1); hm1 &= hm1 - 1; }
                            pk[k] = bit / kMSet; jk[k] = bit % kMSet;
                            nk = k + 1;
                        }
                    }
                    nfix += nk;
                    h4f ak[PVM_BANDK];
#pragma unroll
                    for (int k = 0; k < PVM_BANDK; ++k) ak[k] = afrag(pk[k]);
                    f32x16 ck[PVM_BANDK];
#pragma unroll
                    for (int k = 0; k < PVM_BANDK; ++k)
                        ck[k] = __builtin_amdgcn_mfma_f32_32x32x8f16(ak[k], bsel(jk[k]), zero, 0, 0, 0);
#pragma unroll
                    for (int k = 0; k < PVM_BANDK; ++k)
                        if (k < nk) band_test(ck[k], pk[k], jk[k]);
                }
#else
                while (hm0 | hm1) {
                    int bit;
                    if (hm0) { bit = __builtin_ctzll(hm0); hm0 &= hm0 - 1; }
                    else { bit = 64 + __builtin_ctzll(hm1); hm1 &= hm1 - 1; }
                    const int p = bit / kMSet, j = bit % kMSet;
                    ++nfix;
                    h4f bj = bf[0];
#pragma unroll
                    for (int k = 1; k < kMSet; ++k)
                        if (j == k) bj = bf[k];
                    float hxj, hyj, sj, gBj;
                    hscale(j, hxj, hyj, sj, gBj);
                    const bool fj = (hfm >> j) & 1u;
                    const float G = a.gzf * gBj * sj * 1.001f;
                    const f32x16 c = __builtin_amdgcn_mfma_f32_32x32x8f16(afrag(p), bj, zero, 0, 0, 0);
                    // register pair (2q, 2q + 1) = rows 2m, 2m + 1 with
                    // m = (q & 1) + 4 (q >> 1) + 2 half: pixel m of the batch.
                    // Every pair's test first, one ballot for the lot: most
                    // flagged MFMAs hold no pair inside its own bound, and
                    // then the per-pair ballots and queue writes are skipped
                    uint32_t um = 0;
                    float zs[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const float X = c[2 * q], Y = c[2 * q + 1];
                        const float zq = X - fabsf(Y);
                        const float g = fmaf(kx, fabsf(X), fmaf(ky, fabsf(Y), G));
                        const int pix = p * kMB + (q & 1) + 4 * (q >> 1) + 2 * half;
                        zs[q] = zq;
                        um |= (fj && pix < np && fabsf(zq) <= g) ? 1u << q : 0u;
                    }
                    if (__builtin_amdgcn_ballot_w64(um != 0)) {
#pragma unroll
                        for (int q = 0; q < 8; ++q) {
                            const bool u = (um >> q) & 1u;
                            const uint64_t m = __builtin_amdgcn_ballot_w64(u);
                            if (m) {
                                const int pix = p * kMB + (q & 1) + 4 * (q >> 1) + 2 * half;
                                if (nq > kMQueue - kWave) flush();
                                const int at = nq + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                                if (u) bq[at] = (uint32_t)pix | ((uint32_t)j << 9) | ((uint32_t)col << 11) | ((signbit(zs[q]) ? 0u : 1u) << 16);
                                nq += __popcll(m);
                                nqd += __popcll(m);
                            }
                        }
                    }
                }
#endif
                { const uint64_t t = cyc(); c_band += t - c_mark; c_fix += t - c_mark; c_mark = t; }
                flush();
                __builtin_amdgcn_wave_barrier();
                { const uint64_t t = cyc(); c_flush += t - c_mark; c_fix += t - c_mark; c_mark = t; }
                // exact-only hypotheses (rare): lane = pixel, one hypothesis at a time
#pragma unroll
                for (int j = 0; j < kMSet; ++j) {
                    uint64_t mm = __builtin_amdgcn_ballot_w64(((hxm >> j) & 1u) && half == 0);
                    nxo += __popcll(mm);
#ifdef PVM_ABL_XO
                    mm = 0;
#endif
                    while (mm) {
                        const int l = __builtin_ctzll(mm);
                        mm &= mm - 1;
                        const float2 hx2 = hlds[j * 32 + l];
                        int c = 0;
#pragma unroll
                        for (int k = 0; k < (kMChunk + kWave - 1) / kWave; ++k) {
                            const int jj = k * kWave + lane;
                            bool e = false;
                            if (jj < np) {
                                const F4 x = S.x.get(jj);
                                e = exact_vote(x.z, x.w, x.x, x.y, hx2.x, hx2.y, a.thr);
                            }
                            c += __popcll(__builtin_amdgcn_ballot_w64(e));
                        }
                        if (lane == l) cnt[j] += c;
                    }
                }
                { const uint64_t t = cyc(); c_xo += t - c_mark; c_fix += t - c_mark; c_mark = t; }
            } else {
                // every pair through the reference sequence (lane = hypothesis column;
                // the two lane halves take alternate pixels)
#pragma unroll 1
                for (int jj = half; jj < np; jj += 2) {
                    const F4 e = S.x.get(jj);
#pragma unroll
                    for (int j = 0; j < kMSet; ++j)
                        if ((hfm | hxm) >> j & 1u) {
                            const float2 hv = hlds[j * 32 + col];
                            cnt[j] += exact_vote(e.z, e.w, e.x, e.y, hv.x, hv.y, a.thr);
                        }
                }
            }
        }
        // the reference pass's corrections (LDS atomics of this wave), then
        // the two lane halves hold the same hypotheses
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < kMSet; ++j) cnt[j] += half == 0 ? corr[j * 32 + col] : 0;
        int32_t *cp = a.counts + (int64_t)b * a.cnt_bs + (int64_t)v * a.cnt_v;
#pragma unroll
        for (int j = 0; j < kMSet; ++j) {
            const auto sw = __builtin_amdgcn_permlane32_swap(cnt[j], cnt[j], false, false);
            const int tot = (int)(sw[0] + sw[1]);   // both halves, VALU only
            const int h = hg * kGroup + j * 32 + col;
            if (half == 0 && h < a.nh && tot) atomicAdd(&cp[(int64_t)h * a.cnt_h], tot);
        }
        lo += te - ts;
        ++nseg;
        { const uint64_t t = cyc(); c_fix += t - c_mark; c_mark = t; }
    }
    if (PVV_TRACE_ON(a) && lane == 0) {
        const int wave = (int)(blockIdx.x * 4 + wid);
        uint64_t *q = a.trace + 65536 + wave * 8;
        q[0] = c_seg; q[1] = c_stage; q[2] = c_hot; q[3] = c_fix;
        q[4] = c_band; q[5] = c_flush; q[6] = c_xo; q[7] = (uint64_t)nqd;
    }
    if (PVV_TRACE_ON(a) && lane == 0) {
        const int wave = (int)(blockIdx.x * 4 + wid);
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        a.trace[wave * 8] = t_start;
        a.trace[wave * 8 + 1] = __builtin_amdgcn_s_memrealtime();
        a.trace[wave * 8 + 2] = ((uint64_t)xcc << 32) | hw;
        a.trace[wave * 8 + 3] = ((uint64_t)nseg << 32) | (uint32_t)nfix;
        a.trace[wave * 8 + 4] = tloop;
        a.trace[wave * 8 + 5] = ((uint64_t)nslow << 32) | (uint32_t)nxo;
        a.trace[wave * 8 + 6] = t_total;
        a.trace[wave * 8 + 7] = t_hyp;
    }
}

// f32 2x2 inverse as LAPACK sgesv(A, I) (partial pivoting); false if a pivot is 0.
__device__ inline bool lu2_inv(float a00, float a01, float a10, float a11, float inv[4]) {
    bool sw = fabsf(a10) > fabsf(a00);
    if (sw) { float t0 = a00, t1 = a01; a00 = a10; a01 = a11; a10 = t0; a11 = t1; }
    if (a00 == 0.f) return false;
    float l = a10 / a00;
    float u11 = a11 - l * a01;
    if (u11 == 0.f) return false;
    for (int jc = 0; jc < 2; ++jc) {
        float e0 = (jc == 0) ? 1.f : 0.f, e1 = (jc == 1) ? 1.f : 0.f;
        float b0 = sw ? e1 : e0, b1 = sw ? e0 : e1;
        float y1 = b1 - l * b0;
        float x1 = y1 / u11;
        float x0 = (b0 - a01 * x1) / a00;
        inv[0 * 2 + jc] = x0;
        inv[1 * 2 + jc] = x1;
    }
    return true;
}


// ==========================================================================
// K6: winner per (image, keypoint) (RV:567-575) + least-squares partial sums
// over the winner's inliers (RV:584-599, fp64), kRefineNJ blocks per
// keypoint; the last block of each image gathers its image's partials, sums
// them per keypoint in a fixed order, solves (pts = b_inv(ATA) @ ATb, RV:600)
// with b_inv's batch-wide identity fallback (RV:503-518).
// Hand-off (cdna_hip_programming.md Guideline 16, R2: the data is the flag):
// every value travels as 8-B granules {32-bit half, tag}, a pair per 16-B
// sc1 store; the gathering block re-reads them with 16-B sc1 loads until
// every tag is set.  The granules are zeroed by k_fg_count every call; no
// ticket, no drain before a signal, one memory trip from publish to use.
// ==========================================================================
#ifdef PVV_TRACE
__device__ uint64_t *g_refine_trace;   // trace builds only: per-block phase stamps of k_refine_solve
#define PVR_STAMP(k)                                                                                      \
    if (g_refine_trace && threadIdx.x == 0)                                                               \
        g_refine_trace[(((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 8 + (k)] = \
            __builtin_amdgcn_s_memrealtime()
#else
#define PVR_STAMP(k)
#endif
constexpr uint32_t kRefineTag = 1u;           // granule tag (slots zeroed every call)
constexpr uint32_t kRefineSpinMax = 1u << 21;  // gather polls before giving up (~seconds): outputs NaN
// BIG: nh > 1024 hypotheses (the winner's is fetched, not kept in LDS; the
// counts beyond the first 1024 read in a loop) -- its own instantiation, so
// the common one has no loop whose loads would make the compiler drain every
// load in flight before the argmax
template <bool BIG>
__global__ __launch_bounds__(kRT) void k_refine_solve(const int32_t *counts, const float2 *hyp, int64_t hsb, int hsv,
                                                      int hsh, const float4 *pex, const int32_t *tn, int64_t P, int vn,
                                                      int nh, float thr, uint4 *slot, float confidence, int max_iter,
                                                      float *out, pv_v3_diag diag) {
    const int j = blockIdx.x, v = blockIdx.y, b = blockIdx.z;
    PVR_STAMP(0);
    __shared__ uint64_t skey[kRT / 16];
    __shared__ double sacc[kRT / 16][5];   // row sums (16-lane rows)
    constexpr int HC = kRefineLdsHyp / kRT;         // counts / hypotheses per thread, in registers
    static_assert(kRefineLdsHyp % kRT == 0, "PVV_REFINE_T divides the LDS hypothesis capacity");
    __shared__ float2 shyp[kRefineLdsHyp];
    // Loads are issued in the order they are needed and return in that order:
    // the pixel count, the keypoint's vote counts and hypotheses (the argmax
    // needs only those), then this block's pixels (the winner's votes).
    const int n = min(max(tn[b], 0), (int)P);   // clamped like tn_at: loads stay inside the P records
    const int32_t *cnt = counts + ((int64_t)b * vn + v) * nh;
    const float2 *hb = hyp + b * hsb + (int64_t)v * hsv;
    constexpr bool lds_hyp = !BIG;
    int32_t c[HC];
    float2 hh[HC];
    // (every load unconditional, its index clamped into range, so that no
    // branch makes the compiler wait for all of them before the first use)
#pragma unroll
    for (int q = 0; q < HC; ++q) c[q] = cnt[min((int)threadIdx.x + q * kRT, nh - 1)];
#pragma unroll
    for (int q = 0; q < HC; ++q) hh[q] = hb[(int64_t)min((int)threadIdx.x + q * kRT, nh - 1) * hsh];
    constexpr int U = 32768 / (kRefineNJ * kRT);    // 32768 pixels per keypoint preloaded
    static_assert(U >= 1, "PVV_REFINE_NJ * PVV_REFINE_T must not exceed 32768 (preload depth)");
    static_assert(kRT % 64 == 0 && kRT <= 1024, "PVV_REFINE_T: whole waves, at most 1024 threads");
    // (guarded by the buffer's extent P, not by tn: the loads do not wait for
    // tn's; records at t >= tn are read but never used)
    const float4 *eb = pex + ((int64_t)b * vn + v) * P;
    const int t0 = j * kRT + threadIdx.x, tstep = kRefineNJ * kRT;
    float4 e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) e[u] = eb[min(t0 + u * tstep, (int)P - 1)];
    // argmax over h, first index on ties: key = count << 32 | ~h
    uint64_t key = 0;
    auto take = [&](int32_t cv, int h) {
        const uint64_t k2 = ((uint64_t)(uint32_t)cv << 32) | (uint32_t)(0xffffffffu - (uint32_t)h);
        key = k2 > key ? k2 : key;
    };
#pragma unroll
    for (int q = 0; q < HC; ++q) {
        const int h = (int)threadIdx.x + q * kRT;
        take(h < nh ? c[q] : 0, h < nh ? h : -1);   // out of range: key 0 (the initial value)
    }
    if constexpr (BIG)
        for (int h = (int)threadIdx.x + kRefineLdsHyp; h < nh; h += kRT) take(cnt[h], h);
    if constexpr (lds_hyp)
#pragma unroll
        for (int q = 0; q < HC; ++q)
            if ((int)threadIdx.x + q * kRT < nh) shyp[threadIdx.x + q * kRT] = hh[q];
    key = row_max_u64(key);                      // DPP within 16-lane rows, rows through LDS
    if ((lane_id() & 15) == 0) skey[threadIdx.x / 16] = key;
    __syncthreads();
    PVR_STAMP(1);
    key = skey[0];
#pragma unroll
    for (int q = 1; q < kRT / 16; ++q) key = skey[q] > key ? skey[q] : key;
    const int win = (int)(0xffffffffu - (uint32_t)key);
    const int wcnt = (int)(key >> 32);
    // RV:570-575: ratio = count / tn; best starts at 0 and is replaced only on a strict increase
    const float ratio = n > 0 ? (float)wcnt / (float)n : 0.f;
    float2 best = make_float2(0.f, 0.f);
    if (n > 0 && 0.f < ratio) best = lds_hyp ? shyp[win] : hb[(int64_t)win * hsh];
#ifdef PVV_TRACE
    if (g_refine_trace) {   // trace builds: when the block's pixels have arrived
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PVR_STAMP(7);
    }
#endif
    double acc[5] = {0, 0, 0, 0, 0};
    const bool fast = thr >= 1e-3f && thr <= 1.f;
    const float thr2 = thr * thr;
    // branch-free: the squared pre-test decides by selects; the exact sequence
    // runs only when some lane of the wave is undecided; an outlier adds zeros
    auto accum = [&](const float4 &q, bool valid) {   // (cx, cy, nx, ny)
        bool inl, und;
        refine_vote_pre(q.z, q.w, q.x, q.y, best.x, best.y, thr2, fast, &inl, &und);
        und = und && valid;
        if (__ballot(und)) {
            if (und) inl = exact_vote(q.z, q.w, q.x, q.y, best.x, best.y, thr);
        }
        inl = inl && valid;
        const float n0 = inl ? q.w : 0.f, n1 = inl ? -q.z : 0.f;   // RV:585-587 normal = (d_y, -d_x)
        const float bb = inl ? q.w * q.x + -q.z * q.y : 0.f;       // RV:597 (2-term fp32 sum)
        // f32 x f32 is exact in f64, so each fma equals the product-then-add
        const double d0 = n0, d1 = n1, db = bb;
        acc[0] = __fma_rn(d0, d0, acc[0]);
        acc[1] = __fma_rn(d0, d1, acc[1]);
        acc[2] = __fma_rn(d1, d1, acc[2]);
        acc[3] = __fma_rn(d0, db, acc[3]);
        acc[4] = __fma_rn(d1, db, acc[4]);
    };
#pragma unroll
    for (int u = 0; u < U; ++u) accum(e[u], t0 + u * tstep < n);
    for (int t = t0 + U * tstep; t < n; t += tstep) accum(eb[t], true);   // images larger than U * tstep
    PVR_STAMP(2);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const double sr = row_sum_d(acc[k]);
        if ((lane_id() & 15) == 0) sacc[threadIdx.x / 16][k] = sr;
    }
    __syncthreads();
    PVR_STAMP(3);
    // ---- publish: this block's partial, the data as its own flag ----
    const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(slot + (int64_t)b * vn * kRefineNJ * kRefineGran), (short)0, 0x7fffffff, 0x00020000);
    static_assert(kRefineNJ <= 32, "gather: one pending bit per partial");
    if (threadIdx.x < kRefineGran) {
        const int k = threadIdx.x;
        uint64_t bits;
        if (k < 5) {
            double sk = sacc[0][k];
#pragma unroll
            for (int q = 1; q < kRT / 16; ++q) sk += sacc[q][k];
            bits = __builtin_bit_cast(uint64_t, sk);
        } else {
            bits = ((uint64_t)(uint32_t)(n > 0 ? win : 0) << 32) | __float_as_uint(ratio);
        }
        typedef int v4i __attribute__((ext_vector_type(4)));
        const v4i g = {(int)(uint32_t)bits, (int)kRefineTag, (int)(uint32_t)(bits >> 32), (int)kRefineTag};
        __builtin_amdgcn_raw_buffer_store_b128(g, sr, ((v * kRefineNJ + j) * kRefineGran + k) * 16, 0, 16);   // sc1
    }
    if (j == 0 && threadIdx.x == 0) {
        if (diag.win_ratio) diag.win_ratio[b * vn + v] = n > 0 ? ratio : 0.f;
        if (diag.win_idx) diag.win_idx[b * vn + v] = n > 0 ? win : 0;
    }
    PVR_STAMP(4);
    // the image's highest block gathers: dispatched last (in practice: only
    // speed depends on it), it mostly finds every partial already there
    if (j != kRefineNJ - 1 || v != vn - 1) return;
    // ---- gather.  Thread p polls value k of keypoint vv in a quarter of the
    // kRefineNJ partials (its loads in flight together); sums in partial
    // order, quarters then in order: deterministic ----
    constexpr int kGQ = kRefineNJ >= 4 ? 4 : kRefineNJ, kGJ = kRefineNJ / kGQ;
    __shared__ double sks[64][5];
    __shared__ double sq[64 * kRefineGran * kGQ];
    __shared__ float srat[64];
    __shared__ int sflag;   // bit 0: some matrix singular, bit 1: gather gave up
    if (threadIdx.x == 0) sflag = 0;
    __syncthreads();
    bool gave_up = false;
    for (int p = threadIdx.x; p < vn * kRefineGran * kGQ; p += kRT) {
        const int vk = p / kGQ, jq = p - vk * kGQ;
        const int vv = vk / kRefineGran, k = vk - vv * kRefineGran;
        const int base = (vv * kRefineNJ + jq * kGJ) * kRefineGran + k;
        uint64_t val[kGJ];
        uint32_t pend = (1u << kGJ) - 1;
        for (uint32_t spins = 0; pend; ++spins) {
            typedef int v4i __attribute__((ext_vector_type(4)));
            v4i g[kGJ];
#pragma unroll
            for (int jj = 0; jj < kGJ; ++jj)
                if (pend >> jj & 1) g[jj] = __builtin_amdgcn_raw_buffer_load_b128(sr, (base + jj * kRefineGran) * 16, 0, 16);
#pragma unroll
            for (int jj = 0; jj < kGJ; ++jj)
                if ((pend >> jj & 1) && (uint32_t)g[jj].y == kRefineTag && (uint32_t)g[jj].w == kRefineTag) {
                    val[jj] = ((uint64_t)(uint32_t)g[jj].z << 32) | (uint32_t)g[jj].x;
                    pend &= ~(1u << jj);
                }
            if (pend && spins >= kRefineSpinMax) { gave_up = true; break; }
            if (pend) __builtin_amdgcn_s_sleep(2);
        }
        if (gave_up) break;
        if (k < 5) {
            double sum = __builtin_bit_cast(double, val[0]);
#pragma unroll
            for (int jj = 1; jj < kGJ; ++jj) sum += __builtin_bit_cast(double, val[jj]);
            sq[p] = sum;
        } else if (jq == 0) {
            srat[vv] = __uint_as_float((uint32_t)val[0]);   // every block of a keypoint finds the same winner
        }
    }
    if (gave_up) sflag = 2;   // benign race: every writer stores 2
    __syncthreads();
    for (int q = threadIdx.x; q < vn * 5; q += kRT) {
        const int vv = q / 5, k = q - vv * 5;
        const double *sp = &sq[(vv * kRefineGran + k) * kGQ];
        double sum = sp[0];
#pragma unroll
        for (int jq = 1; jq < kGQ; ++jq) sum += sp[jq];
        sks[vv][k] = sum;
    }
    __syncthreads();
    PVR_STAMP(5);
    // ---- solve, one thread per keypoint (vn <= 64: wave 0) ----
    const int vv = threadIdx.x;
    const bool act = vv < vn;
    float A00 = 0, A01 = 0, A11 = 0, B0 = 0, B1 = 0, rat = 3.0e38f;
    float inv[4] = {1.f, 0.f, 0.f, 1.f};
    if (act) {
        A00 = (float)sks[vv][0]; A01 = (float)sks[vv][1]; A11 = (float)sks[vv][2];
        B0 = (float)sks[vv][3]; B1 = (float)sks[vv][4];
        rat = srat[vv];
        if (!lu2_inv(A00, A01, A01, A11, inv)) atomicOr(&sflag, 1);
    }
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const int flag = sflag;
    if (flag & 1) { inv[0] = 1.f; inv[1] = 0.f; inv[2] = 0.f; inv[3] = 1.f; }   // RV:514-517
    if (act) {
        float x = inv[0] * B0 + inv[1] * B1;
        float y = inv[2] * B0 + inv[3] * B1;
        if (n == 0) { x = 0.f; y = 0.f; }
        if (flag & 2) { x = __int_as_float(0x7fc00000); y = x; }   // gather gave up: loud
        out[((int64_t)b * vn + vv) * 2] = x;
        out[((int64_t)b * vn + vv) * 2 + 1] = y;
        if (diag.ata) {
            float *q = diag.ata + ((int64_t)b * vn + vv) * 4;
            q[0] = A00; q[1] = A01; q[2] = A01; q[3] = A11;
        }
        if (diag.atb) { diag.atb[((int64_t)b * vn + vv) * 2] = B0; diag.atb[((int64_t)b * vn + vv) * 2 + 1] = B1; }
    }
    if (diag.tn && vv == 0) diag.tn[b] = n;
    if (diag.iters) {
        // min ratio over keypoints -> iterations the reference's `while True` would run
        float r = rat;
        for (int o = 32; o > 0; o >>= 1) r = fminf(r, __shfl_xor(r, o));
        if (vv == 0) {
            int it = 0;
            if (n > 0) {
                long long hyp_num = 0;
                while (true) {
                    hyp_num += nh;
                    ++it;
                    float val = 1.f - powf(1.f - r * r, (float)hyp_num);
                    if (val > confidence || it > max_iter) break;
                }
            }
            diag.iters[b] = it;
        }
    }
    PVR_STAMP(6);
}

// ==========================================================================
// ransac_motion_voting (RV:966-987): per image and keypoint, the mean over
// the foreground (mask.byte() != 0) of vertex + (col, row) -- the vertex
// field holds offsets here.  fp64 sums (torch.mean's fp32 order is
// unspecified), block-local in LDS, then one device-scope add per block; the
// last block of each image divides.  Empty foreground -> zeros (RV:977-979).
// ==========================================================================
template <int KIND>
__global__ __launch_bounds__(256) void k_motion_vote(MaskView m, VertexView vx, int H, int W, int vn, double *acc,
                                                     int32_t *cnt, int32_t *ticket, float *out) {
    const int b = blockIdx.y, nblk = gridDim.x;
    __shared__ double sacc[64 * 2];
    __shared__ int scnt;
    for (int i = threadIdx.x; i < vn * 2; i += 256) sacc[i] = 0.0;
    if (threadIdx.x == 0) scnt = 0;
    __syncthreads();
    const uint32_t p = (uint32_t)blockIdx.x * 256 + threadIdx.x;
    if (p < (uint32_t)H * W) {
        const int r = (int)(p / (uint32_t)W), c = (int)(p - (uint32_t)r * W);
        if (is_fg<KIND, false>(m, b, r, c)) {
            atomicAdd(&scnt, 1);
            const int64_t vo = b * vx.s[0] + r * vx.s[1] + c * vx.s[2];
            for (int v = 0; v < vn; ++v) {
                float dx, dy;
                if (vx.kind == PV_VERTEX_F32) {
                    dx = ((const float *)vx.p)[vo + v * vx.s[3]];
                    dy = ((const float *)vx.p)[vo + v * vx.s[3] + vx.s[4]];
                } else {
                    dx = __half2float(((const __half *)vx.p)[vo + v * vx.s[3]]);
                    dy = __half2float(((const __half *)vx.p)[vo + v * vx.s[3] + vx.s[4]]);
                }
                atomicAdd(&sacc[v * 2], (double)(dx + (float)c));       // RV:983 vertex + coords (fp32 add)
                atomicAdd(&sacc[v * 2 + 1], (double)(dy + (float)r));
            }
        }
    }
    __syncthreads();
    if (scnt) {
        for (int i = threadIdx.x; i < vn * 2; i += 256) atomicAdd(&acc[(int64_t)b * vn * 2 + i], sacc[i]);
        if (threadIdx.x == 0) atomicAdd(&cnt[b], scnt);
    }
    __syncthreads();
    __shared__ int slast;
    if (threadIdx.x == 0) {
        __threadfence();
        slast = __hip_atomic_fetch_add(&ticket[b], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1;
    }
    __syncthreads();
    if (!slast) return;
    const int n = ld_agent(&cnt[b]);
    for (int i = threadIdx.x; i < vn * 2; i += 256)
        out[(int64_t)b * vn * 2 + i] = n > 0 ? (float)(ld_agent(&acc[(int64_t)b * vn * 2 + i]) / n) : 0.f;
}

template <int KIND, bool EVD>
struct MotionStage {
    static int run(const MaskView *m, const VertexView *vx, int b, int H, int W, int vn, double *acc, int32_t *cnt,
                   int32_t *ticket, float *out, hipStream_t s) {
        dim3 grid((unsigned)(((int64_t)H * W + 255) / 256), (unsigned)b);
        k_motion_vote<KIND><<<grid, 256, 0, s>>>(*m, *vx, H, W, vn, acc, cnt, ticket, out);
        return PV_OK;
    }
};

// ==========================================================================
// v5 confidence (RV:856-858): the inlier ratio of each refined keypoint at
// a second threshold (0.999), counted over the image's compacted pixels.
// ==========================================================================
__global__ __launch_bounds__(256) void k_point_conf(const float *pts, const float4 *pex, const int32_t *tn, int64_t P,
                                                    int vn, float thr, int32_t *confc, float *conf) {
    const int j = blockIdx.x, v = blockIdx.y, b = blockIdx.z;
    const int n = min(max(tn[b], 0), (int)P);   // clamped like tn_at: loads stay inside the P records
    __shared__ int sh[8];
    const float px = pts[((int64_t)b * vn + v) * 2], py = pts[((int64_t)b * vn + v) * 2 + 1];
    const float4 *eb = pex + ((int64_t)b * vn + v) * P;
    int c = 0;
    for (int t = j * 256 + threadIdx.x; t < n; t += kRefineNJ * 256) {
        const float4 e = eb[t];   // (cx, cy, nx, ny)
        c += exact_vote(e.z, e.w, e.x, e.y, px, py, thr) ? 1 : 0;
    }
    c = block_sum2(c, 0, sh).x;
    if (threadIdx.x == 0) {
        int32_t *cc = confc + ((int64_t)b * vn + v) * 2;
        if (c) atomicAdd(&cc[0], c);
        __threadfence();
        const int t = __hip_atomic_fetch_add(&cc[1], 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (t == kRefineNJ - 1) {
            const int total = ld_agent(&cc[0]);
            conf[(int64_t)b * vn + v] = n > 0 ? (float)total / (float)n : 0.f;   // RV:858 float division
        }
    }
}

// ==========================================================================
// EVD (RV:333-406, RV:263-331): per (image, keypoint) over all hypotheses.
// ==========================================================================
__global__ __launch_bounds__(256) void k_evd_with_mean(const int32_t *counts, const float2 *hyp, const int32_t *fg,
                                                       const int32_t *tn, int vn, int nh, int min_num,
                                                       int min_hyp_num, const float *mean, float *cov) {
    const int v = blockIdx.x, b = blockIdx.y;
    const int fgb = fg[b];
    const float mx = mean[(b * vn + v) * 2], my = mean[(b * vn + v) * 2 + 1];
    __shared__ double sacc[4][4];
    __shared__ float smax[4];
    float *cv = cov + ((int64_t)b * vn + v) * 4;
    if (fgb < min_num) {
        // RV:343-348: min_hyp_num zero hypotheses with ratio 1 (all kept by the max-0.1 rule)
        if (threadIdx.x == 0) {
            double dx = (double)(0.f - mx), dy = (double)(0.f - my);
            double w = (double)min_hyp_num;
            float den = (float)w + 1e-3f;
            cv[0] = (float)(w * dx * dx) / den;
            cv[1] = (float)(w * dx * dy) / den;
            cv[2] = (float)(w * dy * dx) / den;
            cv[3] = (float)(w * dy * dy) / den;
        }
        return;
    }
    const float fgf = (float)tn[b];   // RV:355 foreground re-counted after downsampling == tn
    const int32_t *cnt = counts + ((int64_t)b * vn + v) * nh;
    float m = -1.f;
    for (int h = threadIdx.x; h < nh; h += 256) m = fmaxf(m, (float)cnt[h] / fgf);
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane_id() == 0) smax[threadIdx.x / 64] = m;
    __syncthreads();
    m = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
    const float thresh = m - 0.1f;                                   // RV:394
    double a[4] = {0, 0, 0, 0};
    for (int h = threadIdx.x; h < nh; h += 256) {
        float w = (float)cnt[h] / fgf;
        if (w < thresh) w = 0.f;                                     // RV:395
        float2 q = hyp[((int64_t)b * nh + h) * vn + v];
        float dx = q.x - mx, dy = q.y - my;                          // RV:398
        float wx = dx * w, wy = dy * w;                              // RV:399
        a[0] += (double)dx * wx;
        a[1] += (double)dx * wy;
        a[2] += (double)dy * wy;
        a[3] += (double)w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        double s = wave_sum_d(a[k]);
        if (lane_id() == 0) sacc[threadIdx.x / 64][k] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s[4];
        for (int k = 0; k < 4; ++k) s[k] = sacc[0][k] + sacc[1][k] + sacc[2][k] + sacc[3][k];
        float den = (float)s[3] + 1e-3f;                             // RV:401
        cv[0] = (float)s[0] / den;
        cv[1] = (float)s[1] / den;
        cv[2] = (float)s[1] / den;
        cv[3] = (float)s[2] / den;
    }
}

// RV:320-329: top-k (ties: lowest index first) then weighted mean / covariance.
__global__ __launch_bounds__(256) void k_evd_topk(const int32_t *counts, const float2 *hyp, const int32_t *fg,
                                                  const int32_t *tn, int vn, int nh, int min_num, int topk,
                                                  float *mean, float *cov) {
    const int v = blockIdx.x, b = blockIdx.y;
    const int fgb = fg[b];
    float *mo = mean + ((int64_t)b * vn + v) * 2;
    float *cv = cov + ((int64_t)b * vn + v) * 4;
    if (fgb < min_num) {   // RV:276-281: zero hypotheses -> mean 0, cov 0
        if (threadIdx.x == 0) { mo[0] = 0.f; mo[1] = 0.f; cv[0] = cv[1] = cv[2] = cv[3] = 0.f; }
        return;
    }
    const float fgf = (float)tn[b];
    const int32_t *cnt = counts + ((int64_t)b * vn + v) * nh;
    __shared__ int sred[4];
    __shared__ double sacc[4][6];
    auto block_sum = [&](int x) {
        x = wave_sum_i(x);
        __syncthreads();
        if (lane_id() == 0) sred[threadIdx.x / 64] = x;
        __syncthreads();
        return sred[0] + sred[1] + sred[2] + sred[3];
    };
    // k-th largest count T: largest T with #{count >= T} >= k (binary search on the value)
    int k = min(topk, nh);
    int lo = 0, hi = 0;
    for (int h = threadIdx.x; h < nh; h += 256) hi = max(hi, cnt[h]);
    for (int o = 32; o > 0; o >>= 1) hi = max(hi, __shfl_xor(hi, o));
    __syncthreads();
    if (lane_id() == 0) sred[threadIdx.x / 64] = hi;
    __syncthreads();
    hi = max(max(sred[0], sred[1]), max(sred[2], sred[3]));
    while (lo < hi) {   // invariant: #{>= lo} >= k
        int mid = (lo + hi + 1) / 2;
        int c = 0;
        for (int h = threadIdx.x; h < nh; h += 256) c += cnt[h] >= mid;
        c = block_sum(c);
        if (c >= k) lo = mid; else hi = mid - 1;
    }
    const int T = lo;
    int ngt = 0;
    for (int h = threadIdx.x; h < nh; h += 256) ngt += cnt[h] > T;
    ngt = block_sum(ngt);
    const int need_eq = k - ngt;   // take the first `need_eq` hypotheses with count == T (index order)
    double a[6] = {0, 0, 0, 0, 0, 0};
    // pass 1: weights, weighted sums of x, y (mean, RV:323-324)
    int eq_base = 0;
    for (int h0 = 0; h0 < nh; h0 += 256) {
        int h = h0 + threadIdx.x;
        int c = h < nh ? cnt[h] : -1;
        bool eq = c == T;
        // exclusive prefix of eq inside this 256-slab
        uint64_t bal = ballot(eq);
        int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
        __syncthreads();
        if (lane_id() == 0) sred[threadIdx.x / 64] = __popcll(bal);
        __syncthreads();
        int woff = 0;
        for (int q = 0; q < (int)(threadIdx.x / 64); ++q) woff += sred[q];
        int slab = sred[0] + sred[1] + sred[2] + sred[3];
        bool sel = (c > T) || (eq && eq_base + woff + below < need_eq);
        if (h < nh && sel) {
            float w = (float)c / fgf;
            float2 q = hyp[((int64_t)b * nh + h) * vn + v];
            a[0] += (double)w;
            a[1] += (double)(w * q.x);
            a[2] += (double)(w * q.y);
        }
        eq_base += slab;
    }
    for (int kk = 0; kk < 3; ++kk) {
        double s = wave_sum_d(a[kk]);
        if (lane_id() == 0) sacc[threadIdx.x / 64][kk] = s;
    }
    __syncthreads();
    double W = sacc[0][0] + sacc[1][0] + sacc[2][0] + sacc[3][0];
    double SX = sacc[0][1] + sacc[1][1] + sacc[2][1] + sacc[3][1];
    double SY = sacc[0][2] + sacc[1][2] + sacc[2][2] + sacc[3][2];
    const float wsum = (float)W;
    const float mx = (float)SX / wsum, my = (float)SY / wsum;
    // pass 2: covariance about the mean (RV:326-329), every hypothesis, zero weight if not selected
    eq_base = 0;
    double c3[3] = {0, 0, 0};
    for (int h0 = 0; h0 < nh; h0 += 256) {
        int h = h0 + threadIdx.x;
        int c = h < nh ? cnt[h] : -1;
        bool eq = c == T;
        uint64_t bal = ballot(eq);
        int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
        __syncthreads();
        if (lane_id() == 0) sred[threadIdx.x / 64] = __popcll(bal);
        __syncthreads();
        int woff = 0;
        for (int q = 0; q < (int)(threadIdx.x / 64); ++q) woff += sred[q];
        int slab = sred[0] + sred[1] + sred[2] + sred[3];
        bool sel = (c > T) || (eq && eq_base + woff + below < need_eq);
        if (h < nh && sel) {
            float w = (float)c / fgf;
            float2 q = hyp[((int64_t)b * nh + h) * vn + v];
            float dx = q.x - mx, dy = q.y - my;
            c3[0] += (double)dx * (dx * w);
            c3[1] += (double)dx * (dy * w);
            c3[2] += (double)dy * (dy * w);
        }
        eq_base += slab;
    }
    __syncthreads();
    for (int kk = 0; kk < 3; ++kk) {
        double s = wave_sum_d(c3[kk]);
        if (lane_id() == 0) sacc[threadIdx.x / 64][3 + kk] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s0 = sacc[0][3] + sacc[1][3] + sacc[2][3] + sacc[3][3];
        double s1 = sacc[0][4] + sacc[1][4] + sacc[2][4] + sacc[3][4];
        double s2 = sacc[0][5] + sacc[1][5] + sacc[2][5] + sacc[3][5];
        mo[0] = mx; mo[1] = my;
        cv[0] = (float)s0 / wsum;
        cv[1] = (float)s1 / wsum;
        cv[2] = (float)s1 / wsum;
        cv[3] = (float)s2 / wsum;
    }
}

// ==========================================================================
// drop-in kernels on the reference layouts
// ==========================================================================

// KU:11-86
__global__ __launch_bounds__(256) void k_generate_api(const float *direct, const float *coords, const int32_t *idxs,
                                                      float *hypo, int tn, int vn, int hn) {
    int hv = blockIdx.x * 256 + threadIdx.x;
    if (hv >= hn * vn) return;
    int hi = hv / vn, vi = hv - hi * vn;
    int t0 = idxs[hi * vn * 2 + vi * 2], t1 = idxs[hi * vn * 2 + vi * 2 + 1];
    float x = 0.f, y = 0.f, ox, oy;
    if (t0 >= 0 && t0 < tn && t1 >= 0 && t1 < tn &&
        exact_intersect(direct[t0 * vn * 2 + vi * 2], direct[t0 * vn * 2 + vi * 2 + 1], coords[t0 * 2],
                        coords[t0 * 2 + 1], direct[t1 * vn * 2 + vi * 2], direct[t1 * vn * 2 + vi * 2 + 1],
                        coords[t1 * 2], coords[t1 * 2 + 1], &ox, &oy)) {
        x = ox; y = oy;
    }
    hypo[hi * vn * 2 + vi * 2] = x;
    hypo[hi * vn * 2 + vi * 2 + 1] = y;
}

// KU:88-167 with byte outputs: inliers[h][v][t] (U1, store-bound: hn*vn*tn
// bytes).  Mode OR writes only the inlier bytes (reference semantics: the
// caller's buffer keeps its other bytes), DENSE writes every byte.
//
// A wave takes one item: keypoint v, a window of 512 pixels w and 64
// consecutive hypotheses; lane l owns pixels t = 512w + 8l + j, j < 8, and
// writes their 8 bytes of each row (h, v) at R = (h*vn + v)*tn + t with one
// 8-byte store, unaligned as the rows are (measured as fast as aligned
// stores on gfx950).  One item per wave, every item's operand loads at the
// start of the launch, before the store stream fills the memory system.
// There is no prepass: with hn a multiple of 256 a block's four waves take
// four hypothesis groups of one window and stage the window once (raw
// operands, fast operands and the window's frame, in LDS); the grid is
// CU-balanced (full blocks a multiple of the CU count, the rest as quarter
// blocks).  The vote test is vote_segment's rotated-frame test (5 FMAs per
// pair); the inlier bytes are the signs of -z gathered with v_perm.  Pairs
// inside the guard band go to a per-wave LDS queue decided by the
// reference's sequence at the wave's end; hypotheses / pixels outside the
// fast domain take it for their whole row.
constexpr int kBytePix = 8;
constexpr int kByteWin = kWave * kBytePix;      // bytes of a row per segment
#ifndef PVV_BYTE_HB
#define PVV_BYTE_HB 64
#endif
constexpr int kByteHB = PVV_BYTE_HB;             // hypothesis records per batch (rows per wave, <= 64)
static_assert(kByteHB <= 64 && kByteHB % 16 == 0, "row masks are 64-bit; quarter blocks take 16 rows");
constexpr uint32_t kQueuePerWave = 128;          // band pairs a wave queues for its end (LDS)

#ifdef PVVOTE_TRACE_U1
__device__ uint64_t *g_btrace;      // debug build only: per-wave phase stamps of k_vote_bytes
#endif

struct ByteArgs {
    const float *direct;   // [tn][vn][2]
    const float *coords;   // [tn][2]
    const float *hypo;     // [hn][vn][2]
    uint8_t *out;          // [hn][vn][tn]
    int tn, vn, hn, nwin, nhg, fast;
    float thr, tau, gzf, gzr;
    int dbg;               // test hook (pv_debug_set_bytes_mode): 4 = one-entry band queue
    int xcd;               // XCD-contiguous item ranges (grid a multiple of 8)
    // CU-balanced grid (bal_nt > 0): bal_t full blocks, then bal_nt quarter
    // blocks; per XCD bal_tnx / bal_ttx of each (see k_vote_bytes)
    int bal_t, bal_nt, bal_tnx, bal_ttx;
};

// Operands of pixel (t, v) in the byte-output kernel, made where they are
// staged (no prepass): (ux, uy, cx, cy) with u the direction rounded per
// component; (0, 0) for a pixel that never votes (norm1 < 1e-6 or NaN,
// KU:119-121, or non-finite coordinates) and ux = NaN for one outside the
// fast domain.
__device__ __forceinline__ float4 api_pixel(const float2 c, const float2 d) {
    const float n1 = sqrtf(d.x * d.x + d.y * d.y);
    const bool ok = !below_1e6(n1) && n1 == n1 && isfinite(c.x) && isfinite(c.y);
    const float rs = __builtin_amdgcn_rsqf(fmaf(d.x, d.x, d.y * d.y));
    float4 q = make_float4(0.f, 0.f, c.x, c.y);
    if (ok)
        q = (n1 <= kN1Max) ? make_float4(d.x * rs, d.y * rs, c.x, c.y)
                           : make_float4(__builtin_nanf(""), 0.f, c.x, c.y);
    return q;
}
__device__ __forceinline__ float2 api_coords(const ByteArgs &a, int t) {
    return *(const float2 *)(a.coords + (int64_t)t * 2);
}
__device__ __forceinline__ float2 api_direct(const ByteArgs &a, int t, int v) {
    return *(const float2 *)(a.direct + ((int64_t)t * a.vn + v) * 2);
}

// Issue priority from the rows a wave still has (0..3), as in vote_segment:
// otherwise the SIMD favours its oldest wave, equal shares finish staggered
// and the last waves of each SIMD run alone at a fraction of the issue rate.
// (levels 0..2: 3 is the setup's, above every hot loop)
__device__ __forceinline__ void prio_by_remaining(uint32_t remaining, uint32_t total) {
    const uint64_t r3 = (uint64_t)remaining * 3, w1 = (uint64_t)total + 1;
    if (r3 >= 2 * w1) __builtin_amdgcn_s_setprio(2);
    else if (r3 >= w1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

// A window's fast-test frame, shared by the waves that vote it: origin o
// (an integer point), the voting pixels' bounding box relative to o and its
// radius R >= |c - o|; slow = some pixel is outside the fast domain.
struct WinInfo {
    float ox, oy, bxl, bxh, byl, byh, Rw;
    int slow;
};

// rows h0 + i, i < nh (<= kByteHB), of keypoint v, pixels of window w
template <int MODE>
__device__ __forceinline__ void vote_bytes_seg(const ByteArgs &a, F4 *recs, uint8_t *band8, int v, int w, int h0,
                                               int nh, uint32_t rem_after, uint32_t wave_total, uint16_t *wq,
                                               uint32_t &qn, uint64_t *tsetup, const float4 *stage, float2 hq,
                                               const float4 *raw, const float2 *hraw, const WinInfo *win) {
    const uint32_t qcap = a.dbg == 4 ? 1u : kQueuePerWave;   // (dbg 4: test hook, a full queue)
    const int lane = lane_id();
    const float ntau = -a.tau;
    const int tb = kByteWin * w + kBytePix * lane;              // lane's first pixel
    const int64_t rstep = (int64_t)a.vn * a.tn;                 // R(h + 1) - R(h)
    // row i's bytes of this lane: wave-uniform offset (SGPRs) + 32-bit lane offset
    int64_t obase = ((int64_t)h0 * a.vn + v) * a.tn + (int64_t)kByteWin * w;
    obase = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(obase >> 32)) << 32 |
                      (uint32_t)__builtin_amdgcn_readfirstlane((int)obase));   // (SGPRs for the asm below)
    const uint32_t loff = kBytePix * lane;

    // ---- operands ----
    // hq: lane's hypothesis (row h0 + lane), loaded by the caller with the pixels
    uint32_t vmask = 0;
    float fu[kBytePix], fv[kBytePix], fk1[kBytePix], fk2[kBytePix];
    float ox = 0.f, oy = 0.f, Rw = 0.f, bxl = 0.f, bxh = 0.f, byl = 0.f, byh = 0.f;
    bool slow;
    if (stage) {
        // block-staged window: the fast operands and the window's bounds are
        // made once per block (stage_window); pixels past tn never vote
#pragma unroll
        for (int j = 0; j < kBytePix; ++j) {
            fu[j] = fv[j] = fk2[j] = 0.f;
            fk1[j] = -1.0e30f;
            if (tb + j < a.tn) {
                const float4 q = stage[j * kWave + lane];
                fu[j] = q.x; fv[j] = q.y; fk1[j] = q.z; fk2[j] = q.w;
                vmask |= 1u << j;
            }
        }
        slow = __builtin_amdgcn_readfirstlane(!a.fast || win->slow);
        ox = win->ox; oy = win->oy; Rw = win->Rw;
        bxl = win->bxl; bxh = win->bxh; byl = win->byl; byh = win->byh;
        __syncthreads();   // the staging area is the block's band masks from here on
    } else {
        // from the caller's arrays: all 16 loads in flight, then the operands
        uint32_t okmask = 0;
        bool exo = false;
        float2 c[kBytePix], d[kBytePix];
#pragma unroll
        for (int j = 0; j < kBytePix; ++j) {
            const int t = tb + j;
            c[j] = d[j] = make_float2(0.f, 0.f);
            if (t < a.tn) {
                c[j] = api_coords(a, t);
                d[j] = api_direct(a, t, v);
                vmask |= 1u << j;
            }
        }
#pragma unroll
        for (int j = 0; j < kBytePix; ++j) {
            const float4 q = api_pixel(c[j], d[j]);
            const bool in = vmask >> j & 1;
            fu[j] = in ? q.x : 0.f; fv[j] = in ? q.y : 0.f; fk1[j] = in ? q.z : 0.f; fk2[j] = in ? q.w : 0.f;
        }
#pragma unroll
        for (int j = 0; j < kBytePix; ++j) {
            exo |= fu[j] != fu[j];                                  // outside the fast domain
            if (fu[j] != 0.f || fv[j] != 0.f) okmask |= 1u << j;    // votes at all
        }
        slow = __builtin_amdgcn_readfirstlane(!a.fast || __builtin_amdgcn_ballot_w64(exo) != 0);
        // origin: an integer point at the first voting pixel; the voting pixels'
        // bounding box relative to it (R >= |c - o|, and D >= |h - c| per row)
        const uint64_t anyok = __builtin_amdgcn_ballot_w64(okmask != 0);
        if (anyok) {
            const int l0 = __builtin_ctzll(anyok);
            const int j0 = __builtin_ctz(__builtin_amdgcn_readlane(okmask, l0));
            float fx = fk1[0], fy = fk2[0];
#pragma unroll
            for (int j = 1; j < kBytePix; ++j)
                if (j == j0) { fx = fk1[j]; fy = fk2[j]; }
            ox = floorf(bcast(fx, l0));
            oy = floorf(bcast(fy, l0));
            float xl = 3.0e38f, xh = -3.0e38f, yl = 3.0e38f, yh = -3.0e38f;
#pragma unroll
            for (int j = 0; j < kBytePix; ++j)
                if (okmask >> j & 1) {
                    xl = fminf(xl, fk1[j] - ox); xh = fmaxf(xh, fk1[j] - ox);
                    yl = fminf(yl, fk2[j] - oy); yh = fmaxf(yh, fk2[j] - oy);
                }
            bxl = wave_min(xl); bxh = wave_max(xh);
            byl = wave_min(yl); byh = wave_max(yh);
            const float ax = fmaxf(-bxl, bxh), ay = fmaxf(-byl, byh);
            Rw = __builtin_amdgcn_sqrtf(fmaf(ax, ax, ay * ay)) * 1.00001f;
        }
        // fast operands (ux, uy, -k1, -k2) relative to the origin, in place;
        // pixels that never vote get u = 0, -k1 = -1e30: -z = 1e30 tau, far
        // above the band, for every finite h'
#pragma unroll
        for (int j = 0; j < kBytePix; ++j) {
            const bool ok = okmask >> j & 1;
            const float ux = fu[j], uy = fv[j];
            const float cx = fk1[j] - ox, cy = fk2[j] - oy;
            fu[j] = ok ? ux : 0.f;
            fv[j] = ok ? uy : 0.f;
            fk1[j] = ok ? -fmaf(ux, cx, uy * cy) : -1.0e30f;
            fk2[j] = ok ? -fmaf(ux, cy, -(uy * cx)) : 0.f;
        }
    }
    // hypothesis records (lane i -> row h0 + 8i): h - o, band, exact flag
    uint64_t flagged;                                   // rows the exact pass decides whole
    {
        // (flagged rows carry an infinite band, so the hot loop defers them
        // without testing the flag)
        F4 rec{0.f, 0.f, __builtin_inff(), 1.f};
        if (lane < nh) {
            // non-finite or outside the fast domain: the exact sequence decides
            const bool xo = !(isfinite(hq.x) && isfinite(hq.y)) || hyp_exact_only(hq.x, hq.y);
            if (!xo && !slow) {
                const float hx = hq.x - ox, hy = hq.y - oy;
                const float B = (__builtin_amdgcn_sqrtf(fmaf(hx, hx, hy * hy)) + Rw) * 1.00001f + 1e-30f;
                const float dx = fmaxf(fabsf(hx - bxl), fabsf(hx - bxh));
                const float dy = fmaxf(fabsf(hy - byl), fabsf(hy - byh));
                const float D = fmaf(__builtin_amdgcn_sqrtf(fmaf(dx, dx, dy * dy)), 1.00001f, B * 1e-6f);
                rec = F4{hx, hy, fmaf(a.gzr, D, a.gzf * B) * 1.00001f, 0.f};
            }
        }
        flagged = __builtin_amdgcn_ballot_w64(lane < nh && rec.w != 0.f);
        __builtin_amdgcn_wave_barrier();
        if (lane < kByteHB) recs[lane] = rec;
        __builtin_amdgcn_wave_barrier();
    }

    typedef uint64_t u64a1 __attribute__((aligned(1)));   // rows start at any byte
    auto store = [&](uint8_t *p, uint32_t lo, uint32_t hi, auto partial) {
        if (!decltype(partial)::value || vmask == 0xffu) {
            const uint64_t x = (uint64_t)hi << 32 | lo;
            if (MODE == PV_VOTE_DENSE) {
                *(u64a1 *)p = x;
            } else {
                // KU:125 sets inlier bytes to 1 and leaves the others
                const uint64_t old = *(const u64a1 *)p;
                *(u64a1 *)p = (old & ~(x * 0xffu)) | x;
            }
        } else if (vmask) {
            // a row's last pixels (vmask is a prefix): 4 + 2 + 1 bytes at most
            typedef uint32_t u32a1 __attribute__((aligned(1)));
            typedef uint16_t u16a1 __attribute__((aligned(1)));
            const int n = __builtin_popcount(vmask);
            uint64_t x = (uint64_t)hi << 32 | lo;
            int o = 0;
            if (n & 4) {
                const uint32_t y = (uint32_t)x;
                if (MODE == PV_VOTE_DENSE) *(u32a1 *)(p + o) = y;
                else *(u32a1 *)(p + o) = (*(const u32a1 *)(p + o) & ~(y * 0xffu)) | y;
                x >>= 32;
                o += 4;
            }
            if (n & 2) {
                const uint16_t y = (uint16_t)x;
                if (MODE == PV_VOTE_DENSE) *(u16a1 *)(p + o) = y;
                else *(u16a1 *)(p + o) = (uint16_t)((*(const u16a1 *)(p + o) & ~(y * 0xffu)) | y);
                x >>= 16;
                o += 2;
            }
            if (n & 1) {
                const uint8_t y = (uint8_t)x;
                if (MODE == PV_VOTE_DENSE) p[o] = y;
                else if (y) p[o] = 1;
            }
        }
    };
    // inlier bytes from the signs of nz = -z: v_perm's selectors 9 / 11
    // replicate the sign bit of its second / first operand into a byte, 12 is 0
    constexpr uint32_t kSgn01 = 0x0c0c0b09u;   // sign(z0) -> b0, sign(z1) -> b1
    constexpr uint32_t kSgn23 = 0x0b090c0cu;   // sign(z2) -> b2, sign(z3) -> b3
    auto pack4 = [&](float z0, float z1, float z2, float z3) {
        const uint32_t p01 = __builtin_amdgcn_perm(__float_as_uint(z1), __float_as_uint(z0), kSgn01);
        const uint32_t p23 = __builtin_amdgcn_perm(__float_as_uint(z3), __float_as_uint(z2), kSgn23);
        return (p01 | p23) & 0x01010101u;   // 1 where z > 0 (band pairs fixed below); one v_bitop3
    };
    // nz = -z = x' (-tau) + |y'|, and min |nz| for the band check
    auto zrow = [&](const F4 &rec, float nz[kBytePix]) {
        float m = 3.0e38f;
#pragma unroll
        for (int j = 0; j < kBytePix; ++j) {
            const float xr = fmaf(fu[j], rec.x, fmaf(fv[j], rec.y, fk1[j]));
            const float yr = fmaf(fu[j], rec.y, fmaf(-fv[j], rec.x, fk2[j]));
            nz[j] = fmaf(xr, ntau, fabsf(yr));
            m = fminf(m, fabsf(nz[j]));
        }
        return m;
    };

    if (tsetup && *tsetup == 0) *tsetup = __builtin_amdgcn_s_memrealtime();   // (trace builds only)
    // Hot loop: the fast decision of every pair, one 8-byte store per row.
    // A row with a pair inside the band records which (an 8-bit mask per lane
    // in LDS) and its word is stored with those bytes as the fast guess
    // (dense) or left out (OR); the exact pass rewrites just those bytes.
    // Flagged rows (outside the fast domain) are decided whole by the exact
    // pass.  Waves holding a partial word (row ends) use byte stores.
    // Queue this lane's band pairs of row i (bits of bm) in the wave's LDS
    // queue, decided at the wave's end (fix_queued): a wave prefix of the
    // per-lane counts (<= 8, four ballots).  False when the queue is full
    // (entries that fit are still written: deciding a pair twice is harmless,
    // both give the reference's byte).
    auto enqueue = [&](uint32_t bm, int i) {
        const uint32_t n = __builtin_popcount(bm);
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t m = __builtin_amdgcn_ballot_w64((n >> k) & 1u);
            pre += (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) << k;
            tot += (uint32_t)__builtin_popcountll(m) << k;
        }
        const uint32_t base = qn;
        qn = min(base + tot, qcap);
        uint32_t k = base + pre;
#pragma unroll
        for (int j = 0; j < kBytePix; ++j) {
            if (bm >> j & 1) {
                // (row in the wave's batch, pixel in the window): 6 + 9 bits
                if (k < qcap) wq[k] = (uint16_t)(i << 9 | (kBytePix * lane + j));
                ++k;
            }
        }
        return base + tot <= qcap;
    };
    uint64_t dmask = 0;                                 // rows with exact work in this kernel (nh <= 64)
    uint32_t lof = loff;                                // (loop-carried through the asm below: no copies)
    auto row = [&](const F4 &rec, int i, uint32_t &lo, uint32_t &hi) {
        float nz[kBytePix];
#ifdef PVVOTE_ABLATE_U1_COMPUTE
        float m = 3e38f;
        for (int j = 0; j < kBytePix; ++j) nz[j] = rec.x + (float)j;
#else
        const float m = zrow(rec, nz);
#endif
        const uint64_t hit = __builtin_amdgcn_ballot_w64(m <= rec.z);   // flagged rows: rec.z = inf
        lo = pack4(nz[0], nz[1], nz[2], nz[3]);
        hi = pack4(nz[4], nz[5], nz[6], nz[7]);
        bool skip = false;
        if (hit) {
            dmask |= 1ull << i;
            if ((flagged >> i) & 1) {
                skip = MODE != PV_VOTE_DENSE;
            } else {
                uint32_t bm = 0;
#pragma unroll
                for (int j = 0; j < kBytePix; ++j) bm |= (fabsf(nz[j]) <= rec.z ? 1u : 0u) << j;
                int io = i;
                asm volatile("" : "+s"(io));   // address math here, not an induction variable of the hot loop
                band8[io * kWave + lane] = (uint8_t)bm;
                if (MODE != PV_VOTE_DENSE) {
                    lo &= ~((bm & 1u) | (bm & 2u) << 7 | (bm & 4u) << 14 | (bm & 8u) << 21);
                    hi &= ~((bm >> 4 & 1u) | (bm >> 4 & 2u) << 7 | (bm >> 4 & 4u) << 14 | (bm >> 4 & 8u) << 21);
                }
            }
        }
#ifdef PVVOTE_ABLATE_U1_STORE
        if (lo == 0x12345678u && hi == 0x9abcdef0u) skip = false; else skip = true;
#endif
        return skip;
    };
    using gbyte = __attribute__((address_space(1))) uint8_t;
    // (the row offset is made opaque so that the address stays a scalar
    // base + 32-bit lane offset instead of a strength-reduced 64-bit VGPR pointer)
    auto store_row = [&](int i, uint32_t lo, uint32_t hi, bool skip, auto partial) {
        uint64_t rp = (uint64_t)(a.out + (obase + rstep * i));
        rp = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(rp >> 32)) << 32 |
             (uint32_t)__builtin_amdgcn_readfirstlane((int)rp);
        gbyte *rowp = (gbyte *)rp;
        asm volatile("" : "+s"(rowp), "+v"(lof));
        if (!skip) store((uint8_t *)(rowp + lof), lo, hi, partial);
    };
    auto rows = [&](auto partial) {
        F4 ra = recs[0];
        int i = 0;
        for (; i + 1 < nh; i += 2) {
            const F4 rb = recs[i + 1];
            if ((i & 7) == 0) prio_by_remaining(rem_after + (uint32_t)(nh - i), wave_total);
            uint32_t lo0, hi0, lo1, hi1;
            const bool s0 = row(ra, i, lo0, hi0);
            ra = recs[min(i + 2, kByteHB - 1)];
            const bool s1 = row(rb, i + 1, lo1, hi1);
            store_row(i, lo0, hi0, s0, partial);
            store_row(i + 1, lo1, hi1, s1, partial);
        }
        if (i < nh) {
            uint32_t lo, hi;
            const bool sk = row(ra, i, lo, hi);
            store_row(i, lo, hi, sk, partial);
        }
    };
    if (__builtin_amdgcn_ballot_w64(vmask != 0xffu)) rows(std::true_type{});
    else rows(std::false_type{});

    // Band rows: their pairs go to k_fix_bytes' queue (outside the hot loop:
    // the queue's masks and atomics would crowd its registers).
    {
        uint64_t m = dmask & ~flagged;
        while (m) {
            const int i = __builtin_ctzll(m);
            m &= m - 1;
            if (enqueue(band8[i * kWave + lane], i)) dmask &= ~(1ull << i);
        }
    }
    // Exact pass over what is left -- flagged rows, and band rows that found
    // the queue full: the lane's pixels' reference operands are loaded once
    // (one memory round trip), then the reference's sequence decides.
#ifdef PVVOTE_ABLATE_U1_EXACT
    dmask = 0;   // profiling ablation only
#endif
    if (dmask) {
        float2 ec[kBytePix], ed[kBytePix];
#pragma unroll
        for (int j = 0; j < kBytePix; ++j) {
            const int t = tb + j;
            ec[j] = ed[j] = make_float2(0.f, 0.f);
            if (vmask >> j & 1) {
                if (raw) {
                    const float4 r = raw[j * kWave + lane];
                    ec[j] = make_float2(r.x, r.y);
                    ed[j] = make_float2(r.z, r.w);
                } else {
                    ec[j] = *(const float2 *)(a.coords + (int64_t)t * 2);
                    ed[j] = *(const float2 *)(a.direct + ((int64_t)t * a.vn + v) * 2);
                }
            }
        }
        while (dmask) {
            const int i = __builtin_ctzll(dmask);
            dmask &= dmask - 1;
            const float2 q = hraw[i];
            uint8_t *p = a.out + (obase + rstep * i) + loff;
            if ((flagged >> i) & 1) {
                uint32_t lo = 0, hi = 0;
#pragma unroll
                for (int j = 0; j < kBytePix; ++j) {
                    const uint32_t bit =
                        ((vmask >> j & 1) && exact_vote(ed[j].x, ed[j].y, ec[j].x, ec[j].y, q.x, q.y, a.thr)) ? 1u : 0u;
                    if (j < 4) lo |= bit << (8 * j);
                    else hi |= bit << (8 * (j - 4));
                }
                store(p, lo, hi, std::true_type{});
            } else {
                const uint32_t bm = band8[i * kWave + lane];
#pragma unroll
                for (int j = 0; j < kBytePix; ++j) {
                    if (bm >> j & 1) {
                        const bool e = exact_vote(ed[j].x, ed[j].y, ec[j].x, ec[j].y, q.x, q.y, a.thr);
                        if (MODE == PV_VOTE_DENSE) p[j] = e ? 1 : 0;
                        else if (e) p[j] = 1;
                    }
                }
            }
        }
    }
}

// A wave's queued band pairs, decided by the reference's sequence at its
// end: lane = entry; the operands are the reference's own (c, d, h) -- from
// the block's raw window in LDS when it is staged (no memory round trip at
// the wave's end), else loaded, up to 64 pairs in flight at once; the byte
// goes over the wave's own earlier fast guess (dense, program order) or is
// set (OR).
template <int MODE>
__device__ __forceinline__ void fix_queued(const ByteArgs &a, const uint16_t *wq, uint32_t qn, int v, int w, int h0,
                                           const float4 *raw, const float2 *hraw) {
    for (uint32_t k = lane_id(); k < qn; k += kWave) {
        const uint32_t e = wq[k];
        const uint32_t i = e >> 9, p = e & (kByteWin - 1);
        const uint32_t t = (uint32_t)(kByteWin * w) + p;
        const float2 q = hraw[i];
        float2 c, d;
        if (raw) {
            const float4 r = raw[(p % kBytePix) * kWave + p / kBytePix];
            c = make_float2(r.x, r.y);
            d = make_float2(r.z, r.w);
        } else {
            c = *(const float2 *)(a.coords + (int64_t)t * 2);
            d = *(const float2 *)(a.direct + ((int64_t)t * a.vn + v) * 2);
        }
        const bool in = exact_vote(d.x, d.y, c.x, c.y, q.x, q.y, a.thr);
        uint8_t *o = a.out + ((int64_t)(h0 + (int)i) * a.vn + v) * a.tn + t;
        if (MODE == PV_VOTE_DENSE) *o = in ? 1 : 0;
        else if (in) *o = 1;
    }
}

// One item per wave: (keypoint v, window w, hypothesis group g of kByteHB
// rows, or of 16 rows in a quarter block of the balanced grid), g fastest;
// a wave beyond the items exits.
template <int MODE, int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(5, 8))) void k_vote_bytes(ByteArgs a) {
    __shared__ F4 recs_all[WPB][kByteHB];
    __shared__ alignas(16) uint8_t band_all[WPB][kByteHB * kWave];   // per deferred row: each lane's band-pair mask
    __shared__ uint16_t queue_all[WPB][kQueuePerWave];     // per wave: queued band pairs (row, pixel)
    __shared__ float2 hraw_all[WPB][kByteHB];              // per wave: its rows' hypotheses
    __shared__ float4 raw_win[WPB == 4 ? kByteWin : 1];    // block-staged window: (c, d) as given
    __shared__ float4 win_part[WPB];                       // per wave: its pixels' bounds (staging)
    __shared__ int win_exo[WPB];
    F4 *recs = recs_all[threadIdx.x / 64];
    uint8_t *band8 = band_all[threadIdx.x / 64];
    uint16_t *wq = queue_all[threadIdx.x / 64];
    float2 *hraw = hraw_all[threadIdx.x / 64];
    // setup at the top issue priority, above every hot loop (whose waves
    // rank 0..2 by the rows they have left, prio_by_remaining): a wave still
    // in its setup would otherwise wait for them -- and then finish last
    __builtin_amdgcn_s_setprio(3);
    int blk = (int)blockIdx.x;
#ifdef PVVOTE_TRACE_U1
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    uint64_t t_setup = 0;
    uint64_t *tsetup = &t_setup;
#else
    uint64_t *tsetup = nullptr;
#endif
    // Every load of the wave is issued at the launch's start, in one round
    // trip: the item's hypotheses, and the window's pixels.  With the
    // hypothesis groups in fours (hn a multiple of 256) a block's four items
    // share (v, w): the block stages the window's pixels in LDS once (the
    // band-mask area, free until the hot loop) instead of four times.
    const bool shared = WPB == 4 && a.nhg % 4 == 0;
    int wave, v, w, h0, nh;
    if (WPB == 4 && a.bal_nt > 0) {
        // CU-balanced grid (shared staging only): the bal_t full blocks (64
        // rows per wave) are a multiple of the CU count; the remaining units
        // are split four ways into quarter blocks (16 rows per wave),
        // dispatched after the full ones -- at most one beside a CU's full
        // blocks, so every CU carries the same rows to within a quarter block
        // instead of a whole fifth block on some.  Each XCD (blocks i, i + 8,
        // ... under round-robin dispatch) takes a contiguous share of both
        // kinds, full ones first.  (Speed only: any placement is correct.)
        const int x = blk % 8, k = blk / 8;
        int u, part = -1;
        if (k < a.bal_tnx) {
            u = x * a.bal_tnx + k;
            if (u >= a.bal_t) return;                     // (whole blocks)
        } else {
            const int i = x * a.bal_ttx + (k - a.bal_tnx);
            if (i >= a.bal_nt) return;
            u = a.bal_t + i / 4;
            part = i % 4;
        }
        const int G = a.nhg / 4, q = (int)(threadIdx.x / 64);
        const int gq = u % G, rest = u / G;
        v = rest % a.vn;
        w = (rest / a.vn + a.nwin - 1) % a.nwin;
        h0 = part < 0 ? gq * 4 * kByteHB + q * kByteHB : gq * 4 * kByteHB + part * kByteHB + q * (kByteHB / 4);
        nh = part < 0 ? kByteHB : kByteHB / 4;
        wave = uniform(blk * 4 + q);
    } else {
        if (a.xcd) {
            // blocks i, i + 8, ... run on one XCD (round-robin dispatch; speed
            // only, nothing depends on it): give each XCD a contiguous range of
            // items, whose windows' pixels its L2 then fetches once
            const int per = (int)gridDim.x / 8;   // (the host pads the grid to a multiple of 8)
            blk = (blk % 8) * per + blk / 8;
        }
        wave = uniform(blk * WPB + (int)(threadIdx.x / 64));
        const uint32_t nitems = (uint32_t)a.vn * a.nwin * a.nhg;   // < 2^31 (host-checked)
        // (shared: nitems is a multiple of 4, every wave of a block has an item)
        if ((uint32_t)wave >= nitems) return;
        // items (w, v, g), g fastest: a window's items are adjacent; the last
        // (partial) window first, so that its slower byte-store rows are not the
        // launch's tail
        const uint32_t g = (uint32_t)wave % a.nhg, rest = (uint32_t)wave / a.nhg;
        v = (int)(rest % (uint32_t)a.vn);
        w = (int)((rest / (uint32_t)a.vn + (uint32_t)a.nwin - 1) % (uint32_t)a.nwin);
        h0 = (int)g * kByteHB;
        nh = min(kByteHB, a.hn - h0);
    }
    v = uniform(v); w = uniform(w); h0 = uniform(h0); nh = uniform(nh);
    float2 hq = make_float2(0.f, 0.f);
    if (lane_id() < nh) hq = *(const float2 *)(a.hypo + ((int64_t)(h0 + lane_id()) * a.vn + v) * 2);
    if (lane_id() < kByteHB) hraw[lane_id()] = hq;
    const float4 *stage = nullptr, *raw = nullptr;
    WinInfo wi{};
    if (WPB == 4 && shared) {
        // the block's window, once: raw (c, d) for the exact decisions, the
        // fast operands (ux, uy, -k1, -k2) relative to the window's origin
        // (the floor of its first pixel), and the voting pixels' bounds
        float4 *st = (float4 *)&band_all[0][0];
        constexpr int kPer = kByteWin / 256;   // pixels per thread; loads first, then the operands
        const int t0 = kByteWin * w;
        float2 c[kPer], d[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int t = t0 + k * 256 + (int)threadIdx.x;
            if (t < a.tn) { c[k] = api_coords(a, t); d[k] = api_direct(a, t, v); }
        }
        const float2 c0 = api_coords(a, t0);
        const bool obad = !(isfinite(c0.x) && isfinite(c0.y));
        const float ox = obad ? 0.f : floorf(c0.x), oy = obad ? 0.f : floorf(c0.y);
        float xl = 3.0e38f, xh = -3.0e38f, yl = 3.0e38f, yh = -3.0e38f;
        bool exo = false;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int t = t0 + k * 256 + (int)threadIdx.x;
            // lane-interleaved: lane l's pixel j (k = 8l + j) at j * 64 + l, so
            // that each of the waves' eight reads is 64 consecutive float4
            const int kk = k * 256 + (int)threadIdx.x;
            if (t < a.tn) {
                const float4 q = api_pixel(c[k], d[k]);
                const bool ok = q.x != 0.f || q.y != 0.f;   // votes at all (NaN: outside the fast domain)
                exo |= q.x != q.x;
                const float cx = q.z - ox, cy = q.w - oy;
                float4 f = make_float4(0.f, 0.f, -1.0e30f, 0.f);   // never votes: -z = 1e30 tau
                if (ok) {
                    f = make_float4(q.x, q.y, -fmaf(q.x, cx, q.y * cy), -fmaf(q.x, cy, -(q.y * cx)));
                    xl = fminf(xl, cx); xh = fmaxf(xh, cx);
                    yl = fminf(yl, cy); yh = fmaxf(yh, cy);
                }
                st[(kk % kBytePix) * kWave + kk / kBytePix] = f;
                raw_win[(kk % kBytePix) * kWave + kk / kBytePix] = make_float4(c[k].x, c[k].y, d[k].x, d[k].y);
            }
        }
        xl = wave_min(xl); xh = wave_max(xh);
        yl = wave_min(yl); yh = wave_max(yh);
        const bool wexo = __builtin_amdgcn_ballot_w64(exo) != 0;
        if (lane_id() == 0) {
            win_part[threadIdx.x / 64] = make_float4(xl, xh, yl, yh);
            win_exo[threadIdx.x / 64] = wexo;
        }
        __syncthreads();
        float4 p = win_part[0];
        int ex = win_exo[0];
#pragma unroll
        for (int k = 1; k < 4; ++k) {
            const float4 q = win_part[k];
            p.x = fminf(p.x, q.x); p.y = fmaxf(p.y, q.y);
            p.z = fminf(p.z, q.z); p.w = fmaxf(p.w, q.w);
            ex |= win_exo[k];
        }
        wi.slow = ex | obad;
        wi.ox = ox; wi.oy = oy;
        if (p.x <= p.y) {   // some pixel votes
            wi.bxl = p.x; wi.bxh = p.y; wi.byl = p.z; wi.byh = p.w;
            const float ax = fmaxf(-p.x, p.y), ay = fmaxf(-p.z, p.w);
            wi.Rw = __builtin_amdgcn_sqrtf(fmaf(ax, ax, ay * ay)) * 1.00001f;
        }
        stage = st;
        raw = raw_win;
    }
#ifdef PVVOTE_TRACE_U1
    const uint64_t t_staged = __builtin_amdgcn_s_memrealtime();
#endif
    uint32_t qn = 0;
    vote_bytes_seg<MODE>(a, recs, band8, uniform(v), uniform(w), uniform(h0), uniform(nh), 0u, (uint32_t)nh, wq, qn,
                         tsetup, stage, hq, raw, hraw, &wi);
#ifdef PVVOTE_TRACE_U1
    const uint64_t t_first = __builtin_amdgcn_s_memrealtime();
#endif
    __builtin_amdgcn_wave_barrier();
    fix_queued<MODE>(a, wq, qn, v, w, h0, raw, hraw);
#ifdef PVVOTE_TRACE_U1
    if (g_btrace && lane_id() == 0) {
        g_btrace[wave * 8] = t_start;
        g_btrace[wave * 8 + 1] = t_first;
        g_btrace[wave * 8 + 2] = __builtin_amdgcn_s_memrealtime();
        g_btrace[wave * 8 + 3] = t_setup;
        g_btrace[wave * 8 + 4] = t_staged;
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_btrace[wave * 8 + 5] = ((uint64_t)xcc << 32) | hw;
    }
#endif
}

// test hook of the matrix-core sums the vote kernel's error bound rests on
// (pv_debug_mfma_sums): tile i = A [32][8] fp16 x B [8][32] fp16 -> D
// [32][32] f32 by the instruction k_vote_mfma issues, with a zero accumulator
// as there; lane l holds A[l & 31][4 (l >> 5) + j] and B[4 (l >> 5) + j][l & 31]
__global__ __launch_bounds__(64) void k_debug_mfma_sums(const uint16_t *A, const uint16_t *B, float *D) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    const uint16_t *At = A + (int64_t)blockIdx.x * 256, *Bt = B + (int64_t)blockIdx.x * 256;
    h4f a, b;
    for (int j = 0; j < 4; ++j) {
        a[j] = __builtin_bit_cast(_Float16, At[r * 8 + 4 * h + j]);
        b[j] = __builtin_bit_cast(_Float16, Bt[(4 * h + j) * 32 + r]);
    }
    const f32x16 zero = {};
    const f32x16 c = __builtin_amdgcn_mfma_f32_32x32x8f16(a, b, zero, 0, 0, 0);
    float *Dt = D + (int64_t)blockIdx.x * 1024;
    for (int i = 0; i < 16; ++i) Dt[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}

// test hook of wave_min / wave_max (pv_debug_wave_minmax)
__global__ __launch_bounds__(64) void k_debug_minmax(const float *in, float *out) {
    const float x = in[blockIdx.x * 64 + threadIdx.x];
    const float mn = wave_min(x), mx = wave_max(x);
    // every lane must hold the result
    const bool agree = __builtin_amdgcn_ballot_w64(mn != bcast(mn, 0) || mx != bcast(mx, 0)) == 0;
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = agree ? mn : __builtin_nanf("");
        out[2 * blockIdx.x + 1] = agree ? mx : __builtin_nanf("");
    }
}

// KU:170-229
__global__ __launch_bounds__(256) void k_generate_vp(const float *direct, const float *coords, const int32_t *idxs,
                                                     float *hypo, int tn, int vn, int hn) {
    int hv = blockIdx.x * 256 + threadIdx.x;
    if (hv >= hn * vn) return;
    int hi = hv / vn, vi = hv - hi * vn;
    int id0 = idxs[hi * vn * 2 + vi * 2], id1 = idxs[hi * vn * 2 + vi * 2 + 1];
    float x = 0.f, y = 0.f, z = 0.f;
    if (id0 >= 0 && id0 < tn && id1 >= 0 && id1 < tn) {
        float dx0 = direct[id0 * vn * 2 + vi * 2], dy0 = direct[id0 * vn * 2 + vi * 2 + 1];
        float cx0 = coords[id0 * 2], cy0 = coords[id0 * 2 + 1];
        float dx1 = direct[id1 * vn * 2 + vi * 2], dy1 = direct[id1 * vn * 2 + vi * 2 + 1];
        float cx1 = coords[id1 * 2], cy1 = coords[id1 * 2 + 1];
        float lx0 = dy0, ly0 = -dx0, lz0 = cy0 * dx0 - cx0 * dy0;
        float lx1 = dy1, ly1 = -dx1, lz1 = cy1 * dx1 - cx1 * dy1;
        x = ly0 * lz1 - lz0 * ly1;
        y = lz0 * lx1 - lx0 * lz1;
        z = lx0 * ly1 - ly0 * lx1;
        float vx0 = dx0 * (x - z * cx0), vx1 = dx1 * (x - z * cx1);
        float vy0 = dy0 * (y - z * cy0), vy1 = dy1 * (y - z * cy1);
        if (vx0 < 0 && vx1 < 0 && vy0 < 0 && vy1 < 0) { z = -z; x = -x; y = -y; }
        if (vx0 * vx1 < 0 || vy0 * vy1 < 0) { x = 0.f; y = 0.f; z = 0.f; }
    }
    hypo[hi * vn * 3 + vi * 3] = x;
    hypo[hi * vn * 3 + vi * 3 + 1] = y;
    hypo[hi * vn * 3 + vi * 3 + 2] = z;
}

// KU:268-310
__global__ __launch_bounds__(256) void k_vote_vp(const float *direct, const float *coords, const float *hypo,
                                                 uint8_t *inliers, int tn, int vn, int hn, float thr) {
    int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    int64_t tot = (int64_t)hn * vn * tn;
    if (gid >= tot) return;
    int ti = (int)(gid % tn);
    int vi = (int)((gid / tn) % vn);
    int hi = (int)(gid / ((int64_t)tn * vn));
    float cx = coords[ti * 2], cy = coords[ti * 2 + 1];
    float hx = hypo[(hi * vn + vi) * 3], hy = hypo[(hi * vn + vi) * 3 + 1], hz = hypo[(hi * vn + vi) * 3 + 2];
    float ddx = direct[(int64_t)ti * vn * 2 + vi * 2], ddy = direct[(int64_t)ti * vn * 2 + vi * 2 + 1];
    float fx = hx - cx * hz, fy = hy - cy * hz;
    float n1 = sqrtf(ddx * ddx + ddy * ddy);
    float n2 = sqrtf(fx * fx + fy * fy);
    if (below_1e6(n1) || below_1e6(n2)) return;
    float ad = (ddx * fx + ddy * fy) / (n1 * n2);
    float vx = fx * ddx, vy = fy * ddy;
    if (vx < 0 || vy < 0) return;
    if (fabsf(ad) > thr) inliers[gid] = 1;
}

// --------------------------------------------------------------------------
// host helpers
// --------------------------------------------------------------------------
int cu_count() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
            n = prop.multiProcessorCount;
        if (n <= 0) n = 256;
    }
    return n;
}

inline int rc(hipError_t e) { return e == hipSuccess ? PV_OK : (int)e; }
inline int last() { return rc(hipGetLastError()); }

// Constants of the rotated-frame test (DESIGN.md "Exactness of the fast vote
// test"): tau = sqrt(1-thr^2)/thr; band = gzf * B + gzr * D with
// B >= |h - o| + |c - o| and D >= |h - c|:
//   gzf = 2 * (9 tau + 8) * 2^-24   the fast path's rounding (7 tau + 6, plus
//                                   2 (tau + 1) for a rounded c - o when the
//                                   coordinates are not integers)
//   gzr = 2 * 9.5 (tau + 1/tau) * 2^-24   the reference's 8-ulp cosine error
//                                   (+1.5 ulp for its rounded d) mapped
//                                   through dz/dcos = |d| (tau + 1/tau)
// both with 2x margin.
void fast_constants(float thr, VoteArgs *va) {
    va->thr = thr;
    const double t = (double)thr;
    if (t >= 0.05 && t <= 0.999999) {
        const double tau = sqrt(1.0 - t * t) / t;
        const double u = 1.0 / 16777216.0;
        va->tau = (float)tau;
        va->gzf = (float)(2.0 * (9.0 * tau + 8.0) * u * 1.0001);
        va->gzr = (float)(2.0 * 9.5 * (tau + 1.0 / tau) * u * 1.0001);
        va->fast = 1;
    } else {   // outside the derivation's range: every pair takes the exact sequence
        va->tau = 0.f;
        va->gzf = 0.f;
        va->gzr = 0.f;
        va->fast = 0;
    }
}

// The matrix-core vote (k_vote_mfma): its own fast-path constant (DESIGN.md
// section 5a): per form F the error is <= u |a_F| (37.7 + [X] 2 sqrt 2 tau) B
// (h', c' and b roundings 5.7, fp16 splits 12, b split 4, the matrix core's
// f32 sum of 8 exact products 16: any order of its 7 additions, each off by
// less than one f32 ulp of a partial sum <= sum|terms| -- truncating,
// k-ordered, or aligned to the largest product and truncated -- stays within
// 14 u sum|terms|, +1 u for the final rounding, +1 u margin; tested with
// crafted cancellation sums, test_mfma_sum_error_bound), z = X - |Y| adds
// u (tau + 1) B:
//   gzm = 2 (41.5 tau + 38.7) 2^-24 (2x margin);  gzr as above.
float mfma_gz(float tau) { return (float)(2.0 * (41.5 * (double)tau + 38.7) / 16777216.0 * 1.0001); }

// persistent vote grid: every block resident at once (the occupancy limit of
// the kernel: LDS slabs, registers), fewer when the work is small (>= ~128
// pixel steps per wave)
int vote_grid_steps(int64_t pixel_steps, const void *kernel, int max_per_cu = 1 << 30) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu <= 0) per_cu = 4;
    per_cu = std::min(per_cu, max_per_cu);
    int64_t cap = (int64_t)cu_count() * per_cu;
    int64_t need = (pixel_steps / 128 + 3) / 4;
    return (int)(need < 1 ? 1 : (need < cap ? need : cap));
}

#ifdef PVV_TRACE
uint64_t *g_vote_trace = nullptr;   // trace builds only (pv_debug_set_vote_trace)
#endif

// Kernel selection and grid shapes are compile-time constants of the build
// (pvnet_amd/build.py; pv_build_config() reports them): no environment
// variable changes what the library runs.  The A/B measurements behind each
// default are in the comments and DESIGN.md section 7.
#ifndef PVV_ABL
#define PVV_ABL 0           // profiling ablations only (outputs wrong): 1 no k_compact, 2 no k_hyp_gen, 4 no vote, 8 no refine, 16 no k_fg_count
#endif
// the ablation bits in effect (pv_debug_set_ablation; set between captures by profiling tools only)
int g_abl = PVV_ABL;
#ifndef PVV_VM_BPC
#define PVV_VM_BPC 3        // k_vote_mfma blocks per CU (tools/vm_ab.sh, 8 in flight: 4 -> 36.6k images/s, 3 -> 40.2k, 2 -> 39.7k)
#endif
#ifndef PVV_HYPGEN
#define PVV_HYPGEN 1        // hypotheses by k_hyp_gen before the vote: 34.6k -> 36.6k images/s, vote 35.2 -> 31.8 us
#endif
#ifndef PVV_HYPFUSE
#define PVV_HYPFUSE 1       // ... made by k_compact's first blocks instead of a k_hyp_gen launch (round 6)
#endif
#ifndef PVV_BYTES_XCD
#define PVV_BYTES_XCD 1     // k_vote_bytes: XCD-contiguous item ranges (31.1 vs 31.9 us interleaved)
#endif
#ifndef PVV_BYTES_BAL
#define PVV_BYTES_BAL 1     // k_vote_bytes: CU-balanced grid of full + quarter blocks (33.0 -> 31.1 us)
#endif
static_assert(PVV_VM_BPC >= 1 && PVV_VM_BPC <= 4, "k_vote_mfma: 1..4 blocks per CU");
#ifndef PVV_VM_RW3_0
#define PVV_VM_RW3_0 0      // k_vote_mfma work weights of its three dispatch rounds (0: even shares)
#define PVV_VM_RW3_1 0
#define PVV_VM_RW3_2 0
#endif

// Test hooks (not in pvvote.h, set only by explicit calls between launches,
// never during a capture): which fused vote/count kernel the pipeline runs
// (pv_debug_set_vote_kernel: the tests check both in one process) and the
// byte kernel's band-queue capacity (pv_debug_set_bytes_mode 4: a queue of
// one entry, so the in-kernel exact pass runs).
int g_vote_kernel = 0;    // 0: k_vote_mfma (hn a multiple of 512), 1: k_vote_count
int g_bytes_dbg = 0;
bool vote_old() { return g_vote_kernel == 1; }
// does front_half pre-generate the hypotheses (k_hyp_gen, keypoint-major in w.hypv)?
bool hyp_pregen_used(int vn, int nh) {
    (void)vn;
    return PVV_HYPGEN && ((nh + kGroup - 1) / kGroup) % 4 == 0 && !vote_old();
}

template <bool PREPPED>
void launch_vote(const VoteArgs &va, int64_t pixel_steps, hipStream_t s) {
    if (va.hgn % 4 == 0 && !vote_old()) {
        // blocks per CU of the persistent grid: with 3 of the 4 wave slots
        // of every SIMD one launch leaves room for the next image's blocks,
        // whose prologue (dependent loads) then overlaps this one's
        // matrix/VALU work; the work is cut evenly over the blocks
        const int grid = vote_grid_steps(pixel_steps, (const void *)k_vote_mfma<PREPPED>, PVV_VM_BPC);
        VoteArgs vr = va;
        vr.gzf = va.fast ? mfma_gz(va.tau) : 0.f;
        for (int k = 0; k < 4; ++k) vr.rw[k] = 0;
#ifdef PVM_ABL_FIX_RT
        vr.rw[3] = 7777;
#endif
#ifdef PVM_ABL_Q_RT
        vr.rw[3] = 7778;
#endif
        // a SIMD issues age-first: with one resident block per CU per dispatch
        // round, the rounds' waves end in start order (tools/vote_trace.py:
        // 0 / 3.8 / 7.7 us apart with equal shares); weight the rounds' work
        if (grid == 3 * cu_count() && PVV_VM_RW3_0 > 0) {
            vr.rw[0] = PVV_VM_RW3_0; vr.rw[1] = PVV_VM_RW3_1; vr.rw[2] = PVV_VM_RW3_2;
        }
        k_vote_mfma<PREPPED><<<grid, 256, 0, s>>>(vr);
    } else if (va.hgn % 4 == 0) {
        const int grid = vote_grid_steps(pixel_steps, (const void *)k_vote_count<PREPPED, true>, 4);
        VoteArgs vr = va;
        if (grid == 4 * cu_count()) {
            // four resident rounds: weight the earlier-dispatched ones (round_share;
            // measured: the rounds' mean ends 28.1/30.6/32.9/35.3 us with equal
            // shares, within ~2 us with 1080/1024/976/920, vote kernel -6 %;
            // these a further -1.5 %)
            constexpr int w[4] = {1110, 1035, 965, 890};
            for (int k = 0; k < 4; ++k) vr.rw[k] = w[k];
        }
        k_vote_count<PREPPED, true><<<grid, 256, 0, s>>>(vr);
    } else
        k_vote_count<PREPPED, false>
            <<<vote_grid_steps(pixel_steps, (const void *)k_vote_count<PREPPED, false>), 256, 0, s>>>(va);
}

struct Launch {
    int kind;
    bool evd;
};


template <template <int, bool> class F, typename... A>
int dispatch_mask(int kind, bool evd, A... args) {
    switch (kind) {
#define PV_CASE(K)                                                    \
    case K:                                                           \
        return evd ? F<K, true>::run(args...) : F<K, false>::run(args...);
        PV_CASE(PV_MASK_I64)
        PV_CASE(PV_MASK_U8)
        PV_CASE(PV_MASK_I32)
        PV_CASE(PV_MASK_SEG_F32)
        PV_CASE(PV_MASK_SEG_F16)
#undef PV_CASE
    default:
        return PV_EINVAL;
    }
}

struct CompactArgs {
    MaskView m;
    VertexView vx;
    int b, H, W, vn, nblk, min_num, max_num;
    uint64_t seed;
    const uint8_t *keep;
    Workspace ws;
    HypGen hg;          // hg.nhb > 0: k_compact's first blocks make the hypotheses
    hipStream_t s;
};

template <int KIND, bool EVD>
struct CompactStage {
    static int run(const CompactArgs *a) {
        dim3 grid(a->nblk + a->hg.nhb, a->b);
        static_assert(kFgWideCPB == 8, "grpcnt: groups of 8 chunks");
        if (g_abl & 16) {
        } else if ((int64_t)a->nblk * a->b > kFgWideAbove)
            k_fg_count<KIND, EVD, kFgWideCPB><<<dim3((a->nblk + kFgWideCPB - 1) / kFgWideCPB, a->b), 256, 0, a->s>>>(
                a->m, a->H, a->W, a->ws.blkcnt, a->ws.fgbits, a->ws.grpcnt, a->nblk, a->ws.counts, a->ws.zero_words);
        else
            k_fg_count<KIND, EVD, 1><<<dim3(a->nblk, a->b), 256, 0, a->s>>>(a->m, a->H, a->W, a->ws.blkcnt, a->ws.fgbits,
                                                                          nullptr, a->nblk, a->ws.counts,
                                                                          a->ws.zero_words);
        if (g_abl & 1) return last();
        if ((int64_t)a->nblk * a->b > kFgWideAbove) {
            if (a->vx.kind == PV_VERTEX_F32)
                k_compact<KIND, EVD, PV_VERTEX_F32, true><<<grid, 256, 0, a->s>>>(
                    a->m, a->vx, a->H, a->W, a->vn, a->ws.blkcnt, a->ws.grpcnt, a->ws.fgbits, a->ws.dsagg, a->nblk, a->min_num,
                    a->max_num, a->seed, a->keep, a->ws.tn, a->ws.fgtot, a->ws.pex, a->hg);
            else
                k_compact<KIND, EVD, PV_VERTEX_F16, true><<<grid, 256, 0, a->s>>>(
                    a->m, a->vx, a->H, a->W, a->vn, a->ws.blkcnt, a->ws.grpcnt, a->ws.fgbits, a->ws.dsagg, a->nblk, a->min_num,
                    a->max_num, a->seed, a->keep, a->ws.tn, a->ws.fgtot, a->ws.pex, a->hg);
            return last();
        }
        if (a->vx.kind == PV_VERTEX_F32)
            k_compact<KIND, EVD, PV_VERTEX_F32, false><<<grid, 256, 0, a->s>>>(a->m, a->vx, a->H, a->W, a->vn, a->ws.blkcnt, a->ws.grpcnt, a->ws.fgbits, a->ws.dsagg,
                                                     a->nblk, a->min_num, a->max_num, a->seed, a->keep, a->ws.tn,
                                                     a->ws.fgtot, a->ws.pex, a->hg);
        else
            k_compact<KIND, EVD, PV_VERTEX_F16, false><<<grid, 256, 0, a->s>>>(a->m, a->vx, a->H, a->W, a->vn, a->ws.blkcnt, a->ws.grpcnt, a->ws.fgbits, a->ws.dsagg,
                                                     a->nblk, a->min_num, a->max_num, a->seed, a->keep, a->ws.tn,
                                                     a->ws.fgtot, a->ws.pex, a->hg);
        return last();
    }
};

int check_desc(const pv_image_desc *img) {
    if (!img || !img->mask || !img->vertex) return PV_EINVAL;
    if (img->b <= 0 || img->H <= 0 || img->W <= 0 || img->vn <= 0 || img->vn > 64) return PV_EINVAL;
    if (img->H > 65535 || img->W > 65535) return PV_EINVAL;   // pixel centres pack into 16 bits
    if (img->mask_kind < PV_MASK_I64 || img->mask_kind > PV_MASK_SEG_F16) return PV_EINVAL;
    if (img->vertex_kind != PV_VERTEX_F32 && img->vertex_kind != PV_VERTEX_F16) return PV_EINVAL;
    return PV_OK;
}

// compaction + hypotheses + fused vote/count, shared by v3 and EVD
int front_half(const pv_image_desc *img, const pv_vote_params *prm, int nh, bool evd, const Workspace &w,
               const pv_v3_diag &dg, hipStream_t s) {
    const int b = img->b, H = img->H, W = img->W, vn = img->vn;
    const int64_t P = (int64_t)H * W;
    const int nblk = (int)((P + kCompactChunk - 1) / kCompactChunk);
    CompactArgs ca;
    ca.m = MaskView{img->mask, img->mask_strides[0], img->mask_strides[1], img->mask_strides[2],
                    img->mask_strides[3]};
    ca.vx.p = img->vertex;
    ca.vx.kind = img->vertex_kind;
    for (int i = 0; i < 5; ++i) ca.vx.s[i] = img->vertex_strides[i];
    {   // bytes one image's view spans (the compaction's buffer-load range)
        const int64_t es = img->vertex_kind == PV_VERTEX_F32 ? 4 : 2;
        int64_t hi = 0;
        const int64_t dims[5] = {1, H, W, vn, 2};
        for (int i = 1; i < 5; ++i) {
            if (ca.vx.s[i] < 0) return PV_EINVAL;
            hi += (dims[i] - 1) * ca.vx.s[i];
        }
        if ((hi + 1) * es > INT32_MAX) return PV_EINVAL;
        ca.vx.extent = (int32_t)((hi + 1) * es);
    }
    ca.b = b; ca.H = H; ca.W = W; ca.vn = vn; ca.nblk = nblk;
    ca.min_num = prm->min_num; ca.max_num = prm->max_num;
    ca.seed = mix64(prm->seed ^ 0xd1b54a32d192ed03ull);
    ca.keep = prm->keep;
    ca.ws = w;
    ca.s = s;
    if ((int64_t)vn * ((nh + kGroup - 1) / kGroup) * P >= (1ll << 31)) return PV_EINVAL;
    // the hypotheses by k_compact's first blocks (compact_hyp) instead of a k_hyp_gen launch
    const bool hfuse = PVV_HYPFUSE && hyp_pregen_used(vn, nh) && nblk <= kHypMaxChunks && !(g_abl & 2);
    ca.hg = HypGen{};
    if (hfuse) {
        ca.hg.nhb = (int)(((int64_t)nh * vn + 255) / 256);
        ca.hg.nh = nh; ca.hg.vn = vn; ca.hg.min_num = prm->min_num; ca.hg.max_num = prm->max_num;
        ca.hg.seed = mix64(prm->seed); ca.hg.kseed = ca.seed;
        ca.hg.idxs = prm->idxs; ca.hg.keep = prm->keep;
        ca.hg.hyp_out = w.hyp; ca.hg.hypv_out = w.hypv; ca.hg.diag_hyp = dg.hyp;
        ca.hg.keptbits = w.keptbits;
    }
    int r = dispatch_mask<CompactStage>(img->mask_kind, evd, (const CompactArgs *)&ca);
    if (r) return r;
    if (dg.ev_compact_end) {
        hipError_t e = hipEventRecord((hipEvent_t)dg.ev_compact_end, s);
        if (e != hipSuccess) return rc(e);
    }
    VoteArgs va{};
    va.pex = w.pex; va.P = (int32_t)P;
    va.hyp = nullptr;
    va.hyp_out = w.hyp; va.diag_hyp = dg.hyp;
    va.idxs = prm->idxs; va.seed = mix64(prm->seed);
    va.counts = w.counts; va.cnt_bs = vn * nh; va.cnt_v = nh; va.cnt_h = 1;
    va.tn_dev = w.tn; va.tn_host = 0;
    va.b = b; va.vn = vn; va.nh = nh; va.hgn = (nh + kGroup - 1) / kGroup;
    fast_constants(prm->inlier_thresh, &va);
#ifdef PVV_TRACE
    va.trace = g_vote_trace;
#endif
    // the vote kernel generates the hypotheses itself (item_hyp in its
    // prologue, overlapped with its first pixel loads) and stores them in
    // the reference layout; by default (hyp_pregen) one k_hyp_gen launch makes
    // them first and the vote kernel (k_vote_mfma) reads them keypoint-major
    if (hyp_pregen_used(vn, nh)) {
        va.hypv_out = w.hypv;
        const int64_t nt = (int64_t)b * nh * vn;
        if (hfuse) {
        } else if (!(g_abl & 2)) k_hyp_gen<<<(unsigned)((nt + 255) / 256), 256, 0, s>>>(va);
        else if (g_abl & 32) k_abl_empty<<<1, 64, 0, s>>>(0);
        if ((r = last())) return r;
        va.hyp = w.hypv; va.hyp_sb = (int64_t)vn * nh; va.hyp_sv = nh; va.hyp_sh = 1;
    }
    if (dg.ev_vote_begin) {
        hipError_t e = hipEventRecord((hipEvent_t)dg.ev_vote_begin, s);
        if (e != hipSuccess) return rc(e);
    }
    // the kernel indexes its work in 32 bits: images per launch such that the
    // upper bound (every pixel of every image in the foreground) stays < 2^31
    const int64_t per_img = (int64_t)vn * va.hgn * P;
    const int chunk = (int)std::max<int64_t>(1, std::min<int64_t>(b, ((1ll << 31) - 1) / per_img));
    if (per_img >= (1ll << 31)) return PV_EINVAL;
    for (int b0 = 0; b0 < b; b0 += chunk) {
        VoteArgs vc = va;
        const int nb = std::min(chunk, b - b0);
        vc.b = nb;
        vc.b0 = b0;
        vc.pex += (int64_t)b0 * vn * P;
        vc.hyp_out += (int64_t)b0 * nh * vn;
        if (vc.hyp) vc.hyp += (int64_t)b0 * nh * vn;
        if (vc.diag_hyp) vc.diag_hyp += (int64_t)b0 * nh * vn * 2;
        if (vc.idxs) vc.idxs += (int64_t)b0 * nh * vn * 2;
        vc.counts += (int64_t)b0 * va.cnt_bs;
        vc.tn_dev += b0;
        if (!(g_abl & 4)) launch_vote<true>(vc, nb * per_img, s);
        if ((r = last())) return r;
    }
    if (dg.ev_vote_end) return rc(hipEventRecord((hipEvent_t)dg.ev_vote_end, s));
    return PV_OK;
}

}  // namespace


// ==========================================================================
// C ABI
// ==========================================================================
extern "C" {

const char *pv_version(void) { return PV_VERSION; }

#define PVV_STR2(x) #x
#define PVV_STR(x) PVV_STR2(x)
const char *pv_build_config(void) {
    return "vote=k_vote_mfma(bpc=" PVV_STR(PVV_VM_BPC) ",wpe=" PVM_WPE_STR ",chunk=" PVV_STR(PVM_CHUNK) ",queue=" PVV_STR(PVM_QUEUE) ",band=" PVV_STR(PVM_BANDV) ",rw=" PVV_STR(PVV_VM_RW3_0) "/"
           PVV_STR(PVV_VM_RW3_1) "/" PVV_STR(PVV_VM_RW3_2) ")"
           " hypgen=" PVV_STR(PVV_HYPGEN) " hypfuse=" PVV_STR(PVV_HYPFUSE)
           " refine=" PVV_STR(PVV_REFINE_NJ) "x" PVV_STR(PVV_REFINE_T)
           " fg_cpb=1/" PVV_STR(8) " compact_skip=" PVV_STR(PVV_COMPACT_SKIP)
           " bytes=k_vote_bytes(rows=" PVV_STR(PVV_BYTE_HB) ",xcd=" PVV_STR(PVV_BYTES_XCD) ",bal=" PVV_STR(PVV_BYTES_BAL) ")"
#ifdef PVV_TRACE
           " TRACE"
#endif
        ;
}

const char *pv_error_string(int code) {
    switch (code) {
    case PV_OK: return "ok";
    case PV_EINVAL: return "invalid argument";
    case PV_EWORKSPACE: return "workspace missing or too small";
    case PV_EALIGN: return "misaligned pointer";
    default: return code > 0 ? hipGetErrorString((hipError_t)code) : "unknown error";
    }
}

int pv_device_arch(char *buf, int len) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return rc(e);
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) return rc(e);
    if (buf && len > 0) {
        strncpy(buf, prop.gcnArchName, (size_t)len - 1);
        buf[len - 1] = 0;
    }
    return PV_OK;
}

int pv_stream_create(int32_t priority, pv_stream_t *out) {
    if (!out) return PV_EINVAL;
    hipStream_t s = nullptr;
    const hipError_t e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority);
    if (e != hipSuccess) return rc(e);
    *out = (pv_stream_t)s;
    return PV_OK;
}

int pv_stream_destroy(pv_stream_t stream) {
    if (!stream) return PV_EINVAL;
    return rc(hipStreamDestroy((hipStream_t)stream));
}

int pv_stream_capture_id(pv_stream_t stream, uint64_t *id) {
    if (!id) return PV_EINVAL;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    unsigned long long cid = 0;
    const hipError_t e = hipStreamGetCaptureInfo((hipStream_t)stream, &st, &cid);
    if (e != hipSuccess) return rc(e);
    *id = st == hipStreamCaptureStatusActive ? (uint64_t)cid : 0;
    return PV_OK;
}

int pv_generate_hypothesis(const float *direct, const float *coords, const int32_t *idxs, float *hypo, int32_t tn,
                           int32_t vn, int32_t hn, pv_stream_t stream) {
    if (!direct || !coords || !idxs || !hypo || tn <= 0 || vn <= 0 || hn < 0) return PV_EINVAL;
    if (hn == 0) return PV_OK;
    int64_t n = (int64_t)hn * vn;
    k_generate_api<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(direct, coords, idxs, hypo, tn, vn,
                                                                                  hn);
    return last();
}


int pv_voting_for_hypothesis(const float *direct, const float *coords, const float *hypo, uint8_t *inliers,
                             int32_t tn, int32_t vn, int32_t hn, float inlier_thresh, int32_t mode,
                             pv_stream_t stream) {
    if (!direct || !coords || !hypo || !inliers || tn < 0 || vn <= 0 || hn < 0) return PV_EINVAL;
    if (mode != PV_VOTE_OR && mode != PV_VOTE_DENSE) return PV_EINVAL;
    if (tn == 0 || hn == 0) return PV_OK;
    VoteArgs fc{};
    fast_constants(inlier_thresh, &fc);
    ByteArgs ba{};
    ba.direct = direct; ba.coords = coords; ba.hypo = hypo; ba.out = inliers;
    ba.tn = tn; ba.vn = vn; ba.hn = hn;
    ba.fast = fc.fast; ba.thr = fc.thr; ba.tau = fc.tau; ba.gzf = fc.gzf; ba.gzr = fc.gzr;
    ba.nwin = (tn + kByteWin - 1) / kByteWin;
    ba.nhg = (hn + kByteHB - 1) / kByteHB;
    ba.dbg = g_bytes_dbg;
    const int64_t items = (int64_t)vn * ba.nwin * ba.nhg;
    if (items >= (1ll << 31)) return PV_EINVAL;   // the kernel's 32-bit item index
    // one launch, no scratch: the operands are made where the blocks stage them
    unsigned grid = (unsigned)((items + 3) / 4);
    ba.xcd = PVV_BYTES_XCD;
    if (ba.xcd) grid = (grid + 7) / 8 * 8;
    if (PVV_BYTES_BAL && ba.nhg % 4 == 0 && ba.xcd) {
        // CU-balanced grid: full blocks a multiple of the CU count, the rest
        // as quarter blocks, when that leaves at most one quarter block per CU
        // beside four full ones (one resident round; see k_vote_bytes)
        const int64_t units = items / 4, cus = cu_count();
        const int64_t T = units / cus * cus, E = units - T;
        if (T > 0 && T <= 4 * cus && E > 0 && 4 * E <= cus) {
            ba.bal_t = (int)T;
            ba.bal_nt = (int)(4 * E);
            ba.bal_tnx = (int)((T + 7) / 8);
            ba.bal_ttx = (int)((4 * E + 7) / 8);
            grid = (unsigned)(8 * (ba.bal_tnx + ba.bal_ttx));
        }
    }
    hipStream_t s = (hipStream_t)stream;
    if (mode == PV_VOTE_DENSE)
        k_vote_bytes<PV_VOTE_DENSE, 4><<<grid, 256, 0, s>>>(ba);
    else
        k_vote_bytes<PV_VOTE_OR, 4><<<grid, 256, 0, s>>>(ba);
    return last();
}

int pv_generate_hypothesis_vp(const float *direct, const float *coords, const int32_t *idxs, float *hypo,
                              int32_t tn, int32_t vn, int32_t hn, pv_stream_t stream) {
    if (!direct || !coords || !idxs || !hypo || tn <= 0 || vn <= 0 || hn < 0) return PV_EINVAL;
    if (hn == 0) return PV_OK;
    int64_t n = (int64_t)hn * vn;
    k_generate_vp<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(direct, coords, idxs, hypo, tn, vn,
                                                                                 hn);
    return last();
}

int pv_voting_for_hypothesis_vp(const float *direct, const float *coords, const float *hypo, uint8_t *inliers,
                                int32_t tn, int32_t vn, int32_t hn, float inlier_thresh, pv_stream_t stream) {
    if (!direct || !coords || !hypo || !inliers || tn < 0 || vn <= 0 || hn < 0) return PV_EINVAL;
    int64_t n = (int64_t)hn * vn * tn;
    if (n == 0) return PV_OK;
    k_vote_vp<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(direct, coords, hypo, inliers, tn, vn, hn,
                                                                            inlier_thresh);
    return last();
}

int pv_vote_counts(const float *direct, const float *coords, const float *hypo, int32_t *counts, int32_t tn,
                   int32_t vn, int32_t hn, float inlier_thresh, pv_stream_t stream) {
    if (!direct || !coords || !hypo || !counts || tn < 0 || vn <= 0 || hn < 0) return PV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (hn == 0) return PV_OK;
    // counts[h][v] (the layout of torch.sum(inliers, 2)): zero, then accumulate
    hipError_t e = hipMemsetAsync(counts, 0, sizeof(int32_t) * (size_t)hn * vn, s);
    if (e != hipSuccess) return rc(e);
    VoteArgs va{};
    va.coords = (const float2 *)coords; va.P = tn;
    va.raw = (const float2 *)direct; va.raw_v = 1; va.raw_t = vn;
    va.hyp = (const float2 *)hypo; va.hyp_sb = 0; va.hyp_sv = 1; va.hyp_sh = vn;
    va.counts = counts; va.cnt_bs = 0; va.cnt_v = 1; va.cnt_h = vn;
    va.tn_dev = nullptr; va.tn_host = tn;
    va.b = 1; va.vn = vn; va.nh = hn; va.hgn = (hn + kGroup - 1) / kGroup;
    fast_constants(inlier_thresh, &va);
    if (tn == 0) return PV_OK;
    if ((int64_t)vn * va.hgn * tn >= (1ll << 31)) return PV_EINVAL;   // the kernel's 32-bit work index
    launch_vote<false>(va, (int64_t)vn * va.hgn * tn, s);
    return last();
}

// debug only (not in pvvote.h): wave min / max of 64 floats per wave -> out[2 * wave + {0, 1}]
// debug only (not in pvvote.h): ntiles products A[i] (32 x 8 fp16) x B[i] (8 x 32 fp16) -> D[i]
// (32 x 32 f32) on v_mfma_f32_32x32x8_f16 with a zero accumulator (the vote kernel's sums)
int pv_debug_mfma_sums(const uint16_t *A, const uint16_t *B, float *D, int32_t ntiles, pv_stream_t stream) {
    if (!A || !B || !D || ntiles <= 0) return PV_EINVAL;
    k_debug_mfma_sums<<<(unsigned)ntiles, 64, 0, (hipStream_t)stream>>>(A, B, D);
    return last();
}

int pv_debug_wave_minmax(const float *in, float *out, int32_t nwaves, pv_stream_t stream) {
    if (!in || !out || nwaves <= 0) return PV_EINVAL;
    k_debug_minmax<<<(unsigned)nwaves, 64, 0, (hipStream_t)stream>>>(in, out);
    return last();
}

// debug only (not in pvvote.h): the downsampling look-back counts every earlier
// block itself instead of reading its count (tests of the fallback path)
int pv_debug_lookback_self(int32_t on) {
    return rc(hipMemcpyToSymbol(HIP_SYMBOL(g_lb_self), &on, sizeof(on)));
}

// debug only (profiling tools, never during a capture): pipeline kernels left out of the next
// launches (bits: 1 k_compact, 2 k_hyp_gen, 4 vote, 8 refine, 16 k_fg_count; 32 with 2: an empty
// kernel in k_hyp_gen's place); outputs are wrong
int pv_debug_set_ablation(int32_t m) {
    g_abl = m;
    return PV_OK;
}

#ifdef PVV_TRACE
// trace builds only: per-wave timestamps of the next pipeline vote launches
void pv_debug_set_vote_trace(uint64_t *buf) { g_vote_trace = buf; }
// trace builds only: per-block phase stamps of the next k_refine_solve launches
int pv_debug_set_refine_trace(uint64_t *buf) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_refine_trace), &buf, sizeof(buf)); }
#endif
// test hook (not in pvvote.h): which fused vote/count kernel the pipeline runs
// (0 matrix-core k_vote_mfma, 1 VALU k_vote_count); returns the previous
int pv_debug_set_vote_kernel(int32_t which) {
    const int prev = g_vote_kernel;
    g_vote_kernel = which == 1 ? 1 : 0;
    return prev;
}
// test hook (not in pvvote.h): the byte kernel's band-queue mode (4: one-entry
// queue, so band rows take the in-kernel exact pass); returns the previous
int pv_debug_set_bytes_mode(int32_t dbg) {
    const int prev = g_bytes_dbg;
    g_bytes_dbg = dbg == 4 ? 4 : 0;
    return prev;
}
#ifdef PVVOTE_TRACE_U1
int pv_debug_set_bytes_trace(uint64_t *buf) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_btrace), &buf, sizeof(buf)); }
#endif
#ifdef PVV_TRACE
int pv_debug_compact_trace(int on, uint64_t *host, int n) {
    if (host) return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ctrace), sizeof(uint64_t) * (size_t)n);
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ctrace_on), &on, sizeof(int));
}
#endif

size_t pv_v3_workspace_size(int32_t b, int32_t H, int32_t W, int32_t vn, int32_t n_hyp) {
    if (b <= 0 || H <= 0 || W <= 0 || vn <= 0 || n_hyp <= 0) return 0;
    return carve(nullptr, b, H, W, vn, n_hyp).total;
}

int pv_v3_kernel_launches(int32_t b, int32_t H, int32_t W, int32_t vn, int32_t n_hyp) {
    if (b <= 0 || H <= 0 || W <= 0 || vn <= 0 || n_hyp <= 0) return 0;
    const int64_t P = (int64_t)H * W;
    const int nblk = (int)((P + kCompactChunk - 1) / kCompactChunk);
    const int64_t per_img = (int64_t)vn * ((n_hyp + kGroup - 1) / kGroup) * P;
    if (per_img >= (1ll << 31)) return 0;
    const int chunk = (int)std::max<int64_t>(1, std::min<int64_t>(b, ((1ll << 31) - 1) / per_img));
    const bool pre = hyp_pregen_used(vn, n_hyp);
    const bool fuse = PVV_HYPFUSE && pre && nblk <= kHypMaxChunks;
    return 2 + (pre && !fuse ? 1 : 0) + (b + chunk - 1) / chunk + 1;
}

int pv_ransac_voting_v3(const pv_image_desc *img, const pv_vote_params *prm, float *out, void *workspace,
                        size_t workspace_bytes, const pv_v3_diag *diag, pv_stream_t stream) {
    int r = check_desc(img);
    if (r) return r;
    if (!prm || !out || prm->round_hyp_num <= 0) return PV_EINVAL;
    const int nh = prm->round_hyp_num;
    Workspace w = carve(workspace, img->b, img->H, img->W, img->vn, nh);
    if (!workspace || workspace_bytes < w.total) return PV_EWORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    pv_v3_diag dg{};
    if (diag) dg = *diag;
    if ((r = front_half(img, prm, nh, false, w, dg, s))) return r;
    const int b = img->b, vn = img->vn;
    const int64_t P = (int64_t)img->H * img->W;
    // hypotheses keypoint-major when the pipeline pre-generated them (coalesced), else the reference layout
    const bool hv = hyp_pregen_used(vn, nh);
    auto *kref = nh > kRefineLdsHyp ? k_refine_solve<true> : k_refine_solve<false>;
    if (!(g_abl & 8)) kref<<<dim3(kRefineNJ, vn, b), kRT, 0, s>>>(w.counts, hv ? w.hypv : w.hyp, (int64_t)nh * vn,
                                                          hv ? nh : 1, hv ? 1 : vn, w.pex, w.tn, P, vn, nh,
                                                          prm->inlier_thresh, w.refslot,
                                                          prm->confidence, prm->max_iter, out, dg);
    if ((r = last())) return r;
    if (dg.counts) {
        hipError_t e = hipMemcpyAsync(dg.counts, w.counts, sizeof(int32_t) * (size_t)b * vn * nh,
                                      hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return rc(e);
    }
    return PV_OK;
}

int pv_ransac_voting_v5(const pv_image_desc *img, const pv_vote_params *prm, float conf_thresh, float *out,
                        float *conf, void *workspace, size_t workspace_bytes, const pv_v3_diag *diag,
                        pv_stream_t stream) {
    if (!conf) return PV_EINVAL;
    int r = pv_ransac_voting_v3(img, prm, out, workspace, workspace_bytes, diag, stream);
    if (r) return r;
    Workspace w = carve(workspace, img->b, img->H, img->W, img->vn, prm->round_hyp_num);
    const int64_t P = (int64_t)img->H * img->W;
    k_point_conf<<<dim3(kRefineNJ, img->vn, img->b), 256, 0, (hipStream_t)stream>>>(out, w.pex, w.tn, P, img->vn,
                                                                                     conf_thresh, w.confc, conf);
    return last();
}

int pv_ransac_motion_voting(const pv_image_desc *img, float *out, pv_stream_t stream) {
    int r = check_desc(img);
    if (r) return r;
    if (!out || img->mask_kind == PV_MASK_SEG_F32 || img->mask_kind == PV_MASK_SEG_F16) return PV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int b = img->b, vn = img->vn;
    // stream-ordered, zeroed scratch: sums [b][vn][2] f64, counts [b], tickets [b]
    const size_t acc_bytes = sizeof(double) * 2 * (size_t)b * vn, bytes = acc_bytes + sizeof(int32_t) * 2 * b;
    char *scr = nullptr;
    hipError_t e = hipMallocAsync((void **)&scr, bytes, s);
    if (e != hipSuccess) return rc(e);
    e = hipMemsetAsync(scr, 0, bytes, s);
    if (e != hipSuccess) return rc(e);
    MaskView m{img->mask, img->mask_strides[0], img->mask_strides[1], img->mask_strides[2], img->mask_strides[3]};
    VertexView vx;
    vx.p = img->vertex;
    vx.kind = img->vertex_kind;
    for (int i = 0; i < 5; ++i) vx.s[i] = img->vertex_strides[i];
    int32_t *cnt = (int32_t *)(scr + acc_bytes);
    r = dispatch_mask<MotionStage>(img->mask_kind, false, (const MaskView *)&m, (const VertexView *)&vx, b, img->H,
                                   img->W, vn, (double *)scr, cnt, cnt + b, out, s);
    if (r) return r;
    r = last();
    e = hipFreeAsync(scr, s);
    return r ? r : rc(e);
}

static int evd_front(const pv_image_desc *img, const pv_vote_params *prm, void *workspace, size_t workspace_bytes,
                     Workspace *w, int *nh, hipStream_t s, const pv_v3_diag *diag = nullptr) {
    int r = check_desc(img);
    if (r) return r;
    if (!prm || prm->round_hyp_num <= 0 || prm->min_hyp_num <= 0) return PV_EINVAL;
    int rounds = (prm->min_hyp_num + prm->round_hyp_num - 1) / prm->round_hyp_num;
    *nh = rounds * prm->round_hyp_num;
    *w = carve(workspace, img->b, img->H, img->W, img->vn, *nh);
    if (!workspace || workspace_bytes < w->total) return PV_EWORKSPACE;
    pv_v3_diag ev{};     // the diag's timing events only (bench.py's U4 line)
    if (diag) {
        ev.ev_vote_begin = diag->ev_vote_begin;
        ev.ev_vote_end = diag->ev_vote_end;
        ev.ev_compact_end = diag->ev_compact_end;
    }
    return front_half(img, prm, *nh, true, *w, ev, s);
}

int pv_estimate_voting_distribution_with_mean_diag(const pv_image_desc *img, const pv_vote_params *prm,
                                                   const float *mean, float *cov, void *workspace,
                                                   size_t workspace_bytes, const pv_v3_diag *diag,
                                                   pv_stream_t stream) {
    if (!mean || !cov) return PV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    Workspace w;
    int nh = 0;
    int r = evd_front(img, prm, workspace, workspace_bytes, &w, &nh, s, diag);
    if (r) return r;
    k_evd_with_mean<<<dim3(img->vn, img->b), 256, 0, s>>>(w.counts, w.hyp, w.fgtot, w.tn, img->vn, nh, prm->min_num,
                                                          prm->min_hyp_num, mean, cov);
    return last();
}

int pv_estimate_voting_distribution_with_mean(const pv_image_desc *img, const pv_vote_params *prm,
                                              const float *mean, float *cov, void *workspace,
                                              size_t workspace_bytes, pv_stream_t stream) {
    return pv_estimate_voting_distribution_with_mean_diag(img, prm, mean, cov, workspace, workspace_bytes, nullptr,
                                                          stream);
}

int pv_estimate_voting_distribution(const pv_image_desc *img, const pv_vote_params *prm, float *mean, float *cov,
                                    void *workspace, size_t workspace_bytes, pv_stream_t stream) {
    if (!mean || !cov || !prm || prm->topk <= 0) return PV_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    Workspace w;
    int nh = 0;
    int r = evd_front(img, prm, workspace, workspace_bytes, &w, &nh, s);
    if (r) return r;
    k_evd_topk<<<dim3(img->vn, img->b), 256, 0, s>>>(w.counts, w.hyp, w.fgtot, w.tn, img->vn, nh, prm->min_num,
                                                     prm->topk, mean, cov);
    return last();
}

}  // extern "C"
