// PVNet's full-resolution decoder tail on the matrix cores (gfx950, fp16):
//
//   out = conv1x1(leaky(conv3x3(cat(up2(fm), img, 0-pad)) + b1)) + b2
//
// i.e. MR:51-58 (lib/networks/model_repository.py): up2storaw (x2 bilinear,
// align_corners), torch.cat([fm, x], 1), convraw = [3x3 conv, BN, LeakyReLU
// (0.1), 1x1 conv to seg_dim + ver_dim], with the BN folded into the 3x3
// convolution's bias.  The unfused inference form writes the 40-channel cat
// (786 MB at batch 32), reads it back for MIOpen's 3x3 convolution, writes
// its 32 channels (629 MB) and reads them for the head; here one launch reads
// the low-resolution map and the image and writes the 20 (44) output
// channels.  Exported through include/pvvote.h (pv_decoder_tail_f16).
//
// Work unit: an 8 x 32 tile of output pixels of one image; persistent blocks
// (4 waves, 2 per CU) loop over the tiles, the next tile's inputs (a 7 x 19
// pixel patch of fm, 10 rows of the image) loaded into registers while this
// tile convolves.  Per tile the block builds the convolution's input halo
// (10 x 34 pixels x 40 channels fp16: 32 upsampled, the image's 3, 5 zero) in
// LDS -- the x2 bilinear blend per halo pixel straight from the patch, two
// column blends then a row blend in packed fp16 -- and each wave computes two
// rows of 32 pixels: a 3x3 convolution as [32 out x 368 k] x [368 k x 32
// pixels] on v_mfma_f32_32x32x16_f16 (k = tap x 40 channels, 23 MFMAs per row;
// the A fragments -- the weights -- stay in registers for the whole launch,
// a B fragment is one 16-byte LDS read of 8 channels of one halo pixel).
// Then in registers: the f32 sums rounded to fp16 (a fp16 convolution's
// output), + b1, LeakyReLU as ATen rounds it (y * slope in f32), and that
// 32 x 32 tile -- its rows on the lane's registers, its column on the lane --
// is directly the B operand of the 1x1 convolution (K = the 32 conv channels
// in the accumulator's row order; the 1x1 weights are permuted to match on
// the host), 2 MFMAs per 32 outputs; fp16, + b2, 4-channel runs stored.
//
// Rounding against ATen's unfused fp16 ops: the blend's weights and
// intermediate are fp16 here (ATen: f32, rounded once), the convolutions sum
// in another order; everything else rounds where ATen does.  Tolerance-level
// parity: tests/test_backbone.py::test_decoder_tail_matches_torch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/pvvote.h"

#ifndef PVC_PT_MAJOR
#define PVC_PT_MAJOR 1      // k_conv3x3 tile order within an XCD's range: 1 pixel tile major (5.41-5.45 -> 5.29 ms backbone), 0 cout tile major
#endif
#ifndef PVC_DEC_V1
#define PVC_DEC_V1 0        // 1: the decoder steps on the round-4 kernels (k_dec_conv2s / 4s: halo build and MFMAs in sequence; A/B)
#endif
#ifndef PVC_DEC_AHEAD
#define PVC_DEC_AHEAD 3     // k_dec_conv consumers: fragment reads this many k-steps ahead of their MFMAs
#endif
#ifndef PVC_DEC_2ROW
#define PVC_DEC_2ROW 0      // 1: 4 consumer waves of 2 output rows (measured slower: conv4s 191 vs 160 us, conv2s 315 vs 250)
#endif
#ifndef PVC_L1_AHEAD
#define PVC_L1_AHEAD 2      // halo kernels (k_conv64, k_dec_conv2s / 4s): fragment reads this many k-steps ahead of their MFMAs
#endif
#ifndef PVC_DEC_BAL
#define PVC_DEC_BAL 0       // conv2s (k_dec_conv<32, 2>): three halo buffers, each blend spread over two phases (0: one phase each)
#endif

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f16x __attribute__((ext_vector_type(16)));

constexpr int kTR = 8, kTC = 32;                  // output tile: rows x columns
constexpr int kHR = kTR + 2, kHC = kTC + 2;       // halo
constexpr int kCP = 40;                           // halo channels per pixel (32 + 3 + 5 zero)
constexpr int kKS = 23;                           // MFMA k-steps: ceil(9 taps x 40 / 16)
constexpr int kK = kKS * 16;                      // 368 (the last 8 zero)
constexpr int kHaloPx = kHR * kHC;                // 340
// the low-resolution rows / columns one tile's halo reads: rh, rw < 1/2, so
// 10 halo rows reach at most 7 rows of fm (with the +1 neighbour), 34 columns 19
constexpr int kPR = 7, kPC = 19;
constexpr int kPatchChunks = kPR * kPC * 4;       // 16-byte chunks (32 channels fp16 = 4 per pixel)
constexpr int kPatchIt = (kPatchChunks + 255) / 256;
// the image rows of the halo as dwords: halo columns x0-1 .. x0+32 are bytes
// 6 (x0 - 1) .. 6 (x0 + 33) of the row; from the dword at 6 x0 - 8 (x0 is a
// multiple of 32, so 4-aligned), 52 dwords cover them
constexpr int kImgDw = 52;
constexpr int kImgWords = kHR * kImgDw;
constexpr int kImgIt = (kImgWords + 255) / 256;

struct TailArgs {
    const _Float16 *fm;    // [N][Hin][Win][32]
    const _Float16 *img;   // [N][H][W][3]
    const _Float16 *w1;    // [32][368]: k = tap * 40 + channel (tap = 3 ky + kx)
    const float *b1;       // [32]
    const _Float16 *w2;    // [MT][2][32][16]: the 1x1 weights in the accumulator's row order (host-permuted)
    const float *b2;       // [cout]
    _Float16 *out;         // [N][H][W][cout]; split: the vertex channels [N][H][W][cout - 2]
    _Float16 *seg;         // split: the two segmentation channels [N][H][W][2]; else null
    int N, Hin, Win, H, W, tiles_r, tiles_c, ntiles;
    float rh, rw, slope;
#ifdef PVT_TRACE
    unsigned long long *trace;   // [block][tile iteration < 8][wave][8 phase stamps] (s_memtime)
#endif
};

#ifdef PVT_TRACE
#define PVT_STAMP(k)                                                                                      \
    if (a.trace && it < 8 && lane == 0)                                                                 \
        a.trace[(((int64_t)blockIdx.x * 8 + it) * 4 + wid) * 8 + (k)] = __builtin_amdgcn_s_memtime()
#else
#define PVT_STAMP(k)
#endif

#ifndef PVC_XCD_TILES
#define PVC_XCD_TILES 1     // persistent halo kernels: each XCD takes a contiguous range of a round's tiles (0: block-cyclic)
#endif
// Blocks b, b + 8, ... run on one XCD (the dispatcher deals blocks round
// robin over the 8 XCDs).  Renumbered so that XCD x holds a contiguous range
// of [0, nb): in a round of a persistent grid its blocks take neighbouring
// tiles, whose shared halo rows and columns then meet in that XCD's L2.
__device__ __forceinline__ int xcd_block(int bid, int nb) {
#if PVC_XCD_TILES
    const int q = nb / 8, r = nb % 8, x = bid % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
#else
    (void)nb;
    return bid;
#endif
}

__device__ __forceinline__ void tile_coords(const TailArgs &a, int tile, int &b, int &y0, int &x0, int &ly0,
                                            int &lx0) {
    const int tc = tile % a.tiles_c, rest = tile / a.tiles_c;
    const int tr = rest % a.tiles_r;
    b = rest / a.tiles_r;
    y0 = tr * kTR;
    x0 = tc * kTC;
    ly0 = (int)(a.rh * (float)max(y0 - 1, 0));
    lx0 = (int)(a.rw * (float)max(x0 - 1, 0));
}

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef unsigned int u2 __attribute__((ext_vector_type(2)));

// buffer descriptor over one image's map: offsets past `bytes` (and, as
// unsigned, negative ones) read 0 / drop the store -- the fetches need no clamps
__device__ __forceinline__ __amdgpu_buffer_rsrc_t image_rsrc(const void *base, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes, 0x00020000);
}

// a tile's fm patch and image rows, straight to LDS (buffer loads to LDS, 16
// and 4 bytes a lane at lane-linear addresses: patch chunk c at byte 16 c,
// image dword w at byte 4 w; rows past the map read 0, columns past it read
// the next row -- the halo build never uses either).  Issued once the halo
// is built, so they land during this tile's convolution and nothing holds
// registers for them (round 4; before: loads into 15 VGPRs and an LDS store
// phase, which kept the kernel at 2 blocks per CU).
[[maybe_unused]] __device__ __forceinline__ void fetch(const TailArgs &a, int tile, _Float16 *patch, uint32_t *imgs) {
    int b, y0, x0, ly0, lx0;
    tile_coords(a, tile, b, y0, x0, ly0, lx0);
    const int lane = (int)(threadIdx.x & 63), wid = (int)(threadIdx.x >> 6);
    const int64_t fbytes = (int64_t)a.Hin * a.Win * 64;
    const __amdgpu_buffer_rsrc_t fr = image_rsrc(a.fm + (int64_t)b * a.Hin * a.Win * 32, fbytes);
    const int base = (ly0 * a.Win + lx0) * 64;
#pragma unroll
    for (int i = 0; i < kPatchIt; ++i) {
        const int c0 = 256 * i + 64 * wid, c = c0 + lane;     // the wave's first chunk, the lane's
        if (c0 < kPatchChunks && c < kPatchChunks) {
            const int pp = c >> 2, pr = pp / kPC;
            const int off = base + pr * a.Win * 64 + (pp - pr * kPC) * 64 + 16 * (c & 3);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(fr, (__attribute__((address_space(3))) void *)(patch + 8 * c0),
                                                     16, off, 0, 0, 0);
        }
    }
    const int64_t ibytes = (int64_t)a.H * a.W * 6;
    const __amdgpu_buffer_rsrc_t ir = image_rsrc(a.img + (int64_t)b * a.H * a.W * 3, ibytes);
    const int ibase = ((y0 - 1) * a.W * 3 / 2 + x0 * 3 / 2 - 2) * 4;
#pragma unroll
    for (int i = 0; i < kImgIt; ++i) {
        const int w0 = 256 * i + 64 * wid, w = w0 + lane;
        if (w0 < kImgWords && w < kImgWords) {
            const int r = w / kImgDw;
            const int off = ibase + r * a.W * 6 + (w - r * kImgDw) * 4;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ir, (__attribute__((address_space(3))) void *)(imgs + w0), 4,
                                                     off, 0, 0, 0);
        }
    }
}

// per-thread fixed task geometry of the halo build (tile independent): the
// 136 (halo column, 8-channel group) pairs c = 4 hx + q over the halo's 10 rows
struct Geo {
    int rc0, rhy0, rc1, rhy1;    // rows rhy0 .. rhy0 + 4 of column task rc0; + (rc1, rhy1) if rx
    bool rx;
};

__device__ __forceinline__ Geo make_geo(int t) {
    Geo g;
    const bool lo = t < 136;
    g.rc0 = lo ? t : t - 136;          // 136 + 120 threads x 5 rows; the last 16 columns of rows 5..9
    g.rhy0 = lo ? 0 : 5;               // by threads 0..79
    g.rx = t < 80;
    g.rc1 = 120 + (t & 15);
    g.rhy1 = 5 + (t >> 4);
    return g;
}

// column blend for task column c of the tile: the patch offset of its left
// source pixel, the right one's distance, and the weights (fp16)
struct ColW {
    int poff, dp;
    _Float16 w0, w1;
};

__device__ __forceinline__ ColW col_weights(const TailArgs &a, int c, int x0, int lx0) {
    const int hx = c >> 2;
    const int ox = min(max(x0 - 1 + hx, 0), a.W - 1);
    const float w1r = a.rw * (float)ox;
    const int w1 = (int)w1r;
    const float w1l = w1r - (float)w1;
    ColW r;
    r.poff = (w1 - lx0) * 32 + 8 * (c & 3);
    r.dp = w1 < a.Win - 1 ? 32 : 0;
    r.w0 = (_Float16)(1.f - w1l);
    r.w1 = (_Float16)w1l;
    return r;
}

// halo pixel (row hy, column task c = 4 hx + q): the column blends of its
// two source rows of the patch, then the row blend (zero outside the image).
// Round 4: straight from the patch -- a column blend is recomputed for each
// of the ~3 halo rows that use it (1.8x the blend arithmetic) instead of
// going through an LDS intermediate with its own phase and barrier; the
// fp16 expressions, and so the values, are those of the separable form.
// (Measured: a branch-free form sharing a thread's four column blends over
// its five rows, with bit-mask picks, was 6 % slower -- the picks cost more
// VALU than the reads they save.)
#ifndef PVT_BLEND4
#define PVT_BLEND4 0        // 1: the tail's blend with one fp16 weight per source (backbone 4.949-4.960 vs 4.954-4.963 ms: no gain)
#endif
__device__ __forceinline__ void halo_blend(const TailArgs &a, const _Float16 *patch, _Float16 *halo, const ColW &w,
                                           int c, int hy, bool colok, int y0, int ly0) {
    const int oy = y0 - 1 + hy;
    h8 v = {};
    if (colok && oy >= 0 && oy < a.H) {
        const float h1r = a.rh * (float)oy;
        const int h1 = (int)h1r;
        const int dh = h1 < a.Hin - 1 ? kPC * 32 : 0;
        const float h1l = h1r - (float)h1;
        const _Float16 *p = patch + (h1 - ly0) * (kPC * 32) + w.poff;
        const h8 A = *(const h8 *)p, B = *(const h8 *)(p + w.dp);
        const h8 C = *(const h8 *)(p + dh), D = *(const h8 *)(p + dh + w.dp);
#if PVT_BLEND4
        // one weight per source (f32 products rounded once to fp16): 4 packed
        // ops per 2 channels instead of the separable form's 6
        const float cw0 = (float)w.w0, cw1 = (float)w.w1;
        const _Float16 q00 = (_Float16)(cw0 * (1.f - h1l)), q01 = (_Float16)(cw1 * (1.f - h1l));
        const _Float16 q10 = (_Float16)(cw0 * h1l), q11 = (_Float16)(cw1 * h1l);
        v = __builtin_elementwise_fma(D, (h8)q11, __builtin_elementwise_fma(C, (h8)q10,
                __builtin_elementwise_fma(B, (h8)q01, A * (h8)q00)));
#else
        const h8 c0 = __builtin_elementwise_fma(B, (h8)w.w1, A * (h8)w.w0);
        const h8 c1 = __builtin_elementwise_fma(D, (h8)w.w1, C * (h8)w.w0);
        v = __builtin_elementwise_fma(c1, (h8)(_Float16)h1l, c0 * (h8)(_Float16)(1.f - h1l));
#endif
    }
    *(h8 *)(halo + hy * (kHC * kCP) + (c >> 2) * kCP + 8 * (c & 3)) = v;
}

#ifndef PVT_V1
#define PVT_V1 1             // 1: k_decoder_tail (3 blocks per CU); 0: k_decoder_tail2, warp-specialised (A/B: measured slower)
#endif
#ifndef PVT_AHEAD
#define PVT_AHEAD 3          // k_decoder_tail2 consumers: B fragments this many k-steps ahead
#endif
#ifndef PVT_WPE
#define PVT_WPE 3            // waves per SIMD the tail's registers are sized for (blocks of 4 waves per CU)
#endif
#ifndef PVT_WREG
#define PVT_WREG 12          // k-steps whose weights stay in registers (cout <= 32; 2 fewer above); the rest in LDS
#endif

// The head's output stores: 4 channels o0 .. o0 + 3 of one pixel (8 bytes).
// Unsplit, [N][H][W][cout] at 2 * (cout pix + o0).  Split (pv_decoder_tail_split_f16),
// channels 0-1 go to seg [N][H][W][2] and the rest to the vertex map [N][H][W][cout - 2]:
// group 0 is one 4-byte store to each, a later group one 8-byte store (4-byte
// aligned) to the vertex map.  Buffer descriptors per image; pix < 0 (outside
// the image) gives an offset past the range, so the store is dropped.
struct TailOut {
    __amdgpu_buffer_rsrc_t o, sg;
    bool split;
};
template <int COUT>
__device__ __forceinline__ TailOut tail_out(const TailArgs &a, int b) {
    const int64_t hw = (int64_t)a.H * a.W;
    TailOut t;
    t.split = a.seg != nullptr;
    const int oc = t.split ? COUT - 2 : COUT;
    t.o = image_rsrc(a.out + b * hw * oc, hw * oc * 2);
    t.sg = image_rsrc(t.split ? a.seg + b * hw * 2 : a.out, t.split ? hw * 4 : 0);
    return t;
}
template <int COUT>
__device__ __forceinline__ void tail_store(const TailOut &t, int pix, int o0, h4 v) {
    const u2 w = __builtin_bit_cast(u2, v);
    if (!t.split) {
        const int po = pix >= 0 ? pix * (COUT * 2) + 2 * o0 : (int)0x80000000;
        __builtin_amdgcn_raw_buffer_store_b64(w, t.o, po, 0, 0);
    } else if (o0 == 0) {
        __builtin_amdgcn_raw_buffer_store_b32(w.x, t.sg, pix >= 0 ? pix * 4 : (int)0x80000000, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(w.y, t.o, pix >= 0 ? pix * ((COUT - 2) * 2) : (int)0x80000000, 0, 0);
    } else {
        const int po = pix >= 0 ? pix * ((COUT - 2) * 2) + 2 * (o0 - 2) : (int)0x80000000;
        __builtin_amdgcn_raw_buffer_store_b64(w, t.o, po, 0, 0);
    }
}

#if PVT_V1
template <int COUT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PVT_WPE, PVT_WPE))) void k_decoder_tail(TailArgs a) {
    constexpr int MT = (COUT + 31) / 32;
    constexpr int kWReg = MT == 1 ? PVT_WREG : PVT_WREG - 2, kWLds = kKS - kWReg;
    static_assert(kWReg >= 1 && kWLds >= 0, "PVT_WREG in 3 .. 23");
    __shared__ alignas(16) _Float16 halo[kHaloPx * kCP];
    __shared__ alignas(16) _Float16 patch[kPatchChunks * 8];
    __shared__ alignas(16) uint32_t imgs[kImgWords];
    __shared__ alignas(16) _Float16 bias[32 + 32 * MT];
    __shared__ alignas(16) h8 wlds[kWLds > 0 ? kWLds * 64 : 1];   // k-steps kWReg.. : [s][lane]
    const int lane = (int)(threadIdx.x & 63), wid = (int)(threadIdx.x >> 6);
    const int n = lane & 31, h = lane >> 5;
    // the A fragments for the whole launch: lane (out r = n, half h) takes
    // w1[r][16 s + 8 h .. + 8] for k-step s -- the first kWReg k-steps' from
    // the wave's registers, the rest from LDS (one conflict-free ds_read_b128
    // per k-step, shared by the wave's two rows).  All 23 in registers held the
    // kernel at 2 blocks per CU (224 VGPRs); 12 (10 for the 44-output head: 5 spilled VGPRs)
    // leave it 3 (round 4).
    h8 wa[kWReg];
#pragma unroll
    for (int s = 0; s < kWReg; ++s) wa[s] = *(const h8 *)(a.w1 + n * kK + 16 * s + 8 * h);
    for (int i = (int)threadIdx.x; i < kWLds * 64; i += 256) {
        const int s = kWReg + (i >> 6), l = i & 63;
        wlds[i] = *(const h8 *)(a.w1 + (l & 31) * kK + 16 * s + 8 * (l >> 5));
    }
    h8 wb[MT][2];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) wb[t][s2] = *(const h8 *)(a.w2 + ((t * 2 + s2) * 32 + n) * 16 + 8 * h);
    // the weights are in registers before the tile loop (vmcnt 0)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    // the biases, fp16: conv rows [0, 32), head outputs [32, 32 + 32 MT)
    for (int i = (int)threadIdx.x; i < 32 + 32 * MT; i += 256)
        bias[i] = i < 32 ? (_Float16)a.b1[i] : (i - 32 < COUT ? (_Float16)a.b2[i - 32] : (_Float16)0.f);
    const Geo g = make_geo((int)threadIdx.x);
    // the next tile's inputs are fetched during this tile's convolution
    int tile = xcd_block((int)blockIdx.x, (int)gridDim.x);
    if (tile < a.ntiles) fetch(a, tile, patch, imgs);
    __builtin_amdgcn_s_waitcnt(0x0F70);                // the first tile's inputs have landed
    for (int it = 0; tile < a.ntiles; tile += (int)gridDim.x, ++it) {
        (void)it;
        PVT_STAMP(0);
        int b, y0, x0, ly0, lx0;
        tile_coords(a, tile, b, y0, x0, ly0, lx0);
        // this wave's patch / image loads landed before its last epilogue
        // (whose stores may still be in flight); the barrier: every wave's,
        // and every wave is past the previous tile's convolution (halo reads)
        PVT_STAMP(1);
        __syncthreads();
        PVT_STAMP(2);
        PVT_STAMP(3);
        PVT_STAMP(4);
        // ---- halo: pixel (y0 - 1 + hy, x0 - 1 + hx).  x2 bilinear, align_corners:
        // column blends t = w0l A + w1l B of fm rows h1, h1 + 1, then h0l t(h1) + h1l t(h1 + 1) ----
#ifndef PVT_SKIP_HALO
        {
            const int ox0 = x0 - 1 + (g.rc0 >> 2), ox1 = x0 - 1 + (g.rc1 >> 2);
            const bool ok0 = ox0 >= 0 && ox0 < a.W, ok1 = ox1 >= 0 && ox1 < a.W;
            const ColW w0 = col_weights(a, g.rc0, x0, lx0);
#pragma unroll
            for (int i = 0; i < 5; ++i) halo_blend(a, patch, halo, w0, g.rc0, g.rhy0 + i, ok0, y0, ly0);
            if (g.rx) halo_blend(a, patch, halo, col_weights(a, g.rc1, x0, lx0), g.rc1, g.rhy1, ok1, y0, ly0);
            // the image's channels 32..39 (3 + 5 zero)
            for (int p = (int)threadIdx.x; p < kHaloPx; p += 256) {
                const int hy = p / kHC, hx = p - hy * kHC;
                const int oy = y0 - 1 + hy, ox = x0 - 1 + hx;
                h8 v = {};
                if (oy >= 0 && oy < a.H && ox >= 0 && ox < a.W) {
                    const uint16_t *ip = (const uint16_t *)(imgs + hy * kImgDw) + 3 * hx + 1;
                    v[0] = __builtin_bit_cast(_Float16, ip[0]);
                    v[1] = __builtin_bit_cast(_Float16, ip[1]);
                    v[2] = __builtin_bit_cast(_Float16, ip[2]);
                }
                *(h8 *)(halo + p * kCP + 32) = v;
            }
        }
#endif
        PVT_STAMP(5);
        __syncthreads();
        PVT_STAMP(6);
        // patch / imgs are free (read only by the halo build)
        if (tile + (int)gridDim.x < a.ntiles) fetch(a, tile + (int)gridDim.x, patch, imgs);
        // ---- the wave's two output rows: 3x3 convolution on the matrix cores ----
        f16x acc[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) acc[r] = f16x{};
#ifndef PVT_SKIP_CONV
#pragma unroll
        for (int s = 0; s < kKS; ++s) {
            const int G = 2 * s + h;                      // 8-channel group of this lane half
            h8 bf[2];
            if (G < 45) {
                const int tap = G / 5, q = G - 5 * tap;
                const int ky = tap / 3, kx = tap - 3 * ky;
#pragma unroll
                for (int r = 0; r < 2; ++r)
                    bf[r] = *(const h8 *)(halo + ((2 * wid + r + ky) * kHC + n + kx) * kCP + 8 * q);
            } else {
                bf[0] = bf[1] = h8{};
            }
            const h8 af = s < kWReg ? wa[s < kWReg ? s : 0] : wlds[(s - kWReg) * 64 + lane];
#pragma unroll
            for (int r = 0; r < 2; ++r) acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, bf[r], acc[r], 0, 0, 0);
        }
#else
        acc[0][0] = (float)halo[threadIdx.x];
#endif
        // the next tile's fetch (issued before the convolution) has landed, and
        // the previous tile's stores are out; this tile's stay in flight
        __builtin_amdgcn_s_waitcnt(0x0F70);
        PVT_STAMP(7);
        // ---- epilogue + head, per row ----
        const TailOut to = tail_out<COUT>(a, b);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int oy = y0 + 2 * wid + r, ox = x0 + n;
            // conv rows of acc[i]: (i & 3) + 8 (i >> 2) + 4 h -- 4 consecutive rows per i >> 2
            h8 act[2];
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const h4 bq = *(const h4 *)(bias + 8 * gq + 4 * h);
                h4 y;
#pragma unroll
                for (int j = 0; j < 4; ++j) y[j] = (_Float16)acc[r][4 * gq + j];   // the conv's fp16 output
                y = y + bq;
                h4 ys;
#pragma unroll
                for (int j = 0; j < 4; ++j) ys[j] = (_Float16)((float)y[j] * a.slope);
                y = __builtin_elementwise_max(y, ys);          // LeakyReLU, slope < 1
#pragma unroll
                for (int j = 0; j < 4; ++j) act[gq >> 1][4 * (gq & 1) + j] = y[j];
            }
            // the pixel; -1 outside the image (its stores dropped)
            const int pix = (oy < a.H && ox < a.W) ? oy * a.W + ox : -1;
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                f16x d = {};
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) d = __builtin_amdgcn_mfma_f32_32x32x16_f16(wb[t][s2], act[s2], d, 0, 0, 0);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int o0 = 32 * t + 8 * q + 4 * h;
                    if (o0 + 3 < COUT) {
                        h4 v;
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] = (_Float16)d[4 * q + j];
                        v = v + *(const h4 *)(bias + 32 + o0);
#ifdef PVT_SKIP_STORE
                        if (v[0] == (_Float16)1234.5f)
#endif
                        tail_store<COUT>(to, pix, o0, v);
                    }
                }
            }
        }
    }
}

#endif  // PVT_V1

#ifdef PVT_TRACE
unsigned long long *g_tail_trace = nullptr;
#endif

// The tail, warp-specialised (round 5): one block of 8 waves per CU, waves
// 0-3 consumers (two output rows each: 46 MFMAs per tile, A fragments -- all
// 23 k-steps of the 3x3 weights -- in registers for the launch, the 1x1
// head's too), waves 4-7 producers: per tile they LDS-DMA the fm patch and
// image rows of the tile two ahead and build the halo of the next tile into
// the other of two halo buffers (k_decoder_tail's blend, make_geo's task
// split: the same values), so the halo build runs beside the MFMAs instead
// of between them.  One barrier per tile.  LDS: 2 halos (54.4 KB), 2 patch +
// image buffers (21 KB).
template <int COUT>
__global__ __launch_bounds__(512) void k_decoder_tail2(TailArgs a) {
    constexpr int MT = (COUT + 31) / 32;
    __shared__ alignas(16) _Float16 halo2[2][kHaloPx * kCP];
    __shared__ alignas(16) _Float16 patch2[3][kPatchChunks * 8];
    __shared__ alignas(16) uint32_t imgs2[3][kImgWords];
    __shared__ alignas(16) _Float16 bias[32 + 32 * MT];
    const int t = (int)threadIdx.x, lane = t & 63, wid = t >> 6;
    const int n = lane & 31, h = lane >> 5;
    const bool consumer = wid < 4;
    const int G = (int)gridDim.x;
    for (int i = t; i < 32 + 32 * MT; i += 512)
        bias[i] = i < 32 ? (_Float16)a.b1[i] : (i - 32 < COUT ? (_Float16)a.b2[i - 32] : (_Float16)0.f);
    int tile = (int)blockIdx.x;
    if (tile >= a.ntiles) return;
    if (consumer) {
        h8 wa[kKS], wb[MT][2];
#pragma unroll
        for (int s = 0; s < kKS; ++s) wa[s] = *(const h8 *)(a.w1 + n * kK + 16 * s + 8 * h);
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) wb[m][s2] = *(const h8 *)(a.w2 + ((m * 2 + s2) * 32 + n) * 16 + 8 * h);
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();                               // (prologue: the producers' first halo)
        __syncthreads();
        for (int k = 0;; ++k) {
            int b, y0, x0, ly0, lx0;
            tile_coords(a, tile, b, y0, x0, ly0, lx0);
            const _Float16 *halo = halo2[k & 1];
            f16x acc[2] = {f16x{}, f16x{}};
            auto bfrag = [&](int s, int r) -> h8 {
                const int Gq = 2 * s + h;
                if (Gq >= 45) return h8{};
                const int tap = Gq / 5, q = Gq - 5 * tap, ky = tap / 3, kx = tap - 3 * ky;
                return *(const h8 *)(halo + ((2 * wid + r + ky) * kHC + n + kx) * kCP + 8 * q);
            };
            // B fragments PVT_AHEAD k-steps ahead of their MFMAs (one consumer
            // wave per SIMD: nothing else hides a fragment's LDS latency)
            constexpr int AH = PVT_AHEAD;
            h8 fb[AH + 1][2];
#pragma unroll
            for (int s = 0; s < AH; ++s) { fb[s][0] = bfrag(s, 0); fb[s][1] = bfrag(s, 1); }
#pragma unroll
            for (int s = 0; s < kKS; ++s) {
                if (s + AH < kKS) {
                    fb[(s + AH) % (AH + 1)][0] = bfrag(s + AH, 0);
                    fb[(s + AH) % (AH + 1)][1] = bfrag(s + AH, 1);
                }
                const int c = s % (AH + 1);
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wa[s], fb[c][0], acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wa[s], fb[c][1], acc[1], 0, 0, 0);
            }
            const TailOut to = tail_out<COUT>(a, b);
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int oy = y0 + 2 * wid + r, ox = x0 + n;
                h8 act[2];
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const h4 bq = *(const h4 *)(bias + 8 * gq + 4 * h);
                    h4 y;
#pragma unroll
                    for (int j = 0; j < 4; ++j) y[j] = (_Float16)acc[r][4 * gq + j];
                    y = y + bq;
                    h4 ys;
#pragma unroll
                    for (int j = 0; j < 4; ++j) ys[j] = (_Float16)((float)y[j] * a.slope);
                    y = __builtin_elementwise_max(y, ys);
#pragma unroll
                    for (int j = 0; j < 4; ++j) act[gq >> 1][4 * (gq & 1) + j] = y[j];
                }
                const int pix = (oy < a.H && ox < a.W) ? oy * a.W + ox : -1;
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    f16x d = {};
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) d = __builtin_amdgcn_mfma_f32_32x32x16_f16(wb[m][s2], act[s2], d, 0, 0, 0);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int o0 = 32 * m + 8 * q + 4 * h;
                        if (o0 + 3 < COUT) {
                            h4 v;
#pragma unroll
                            for (int j = 0; j < 4; ++j) v[j] = (_Float16)d[4 * q + j];
                            v = v + *(const h4 *)(bias + 32 + o0);
                            tail_store<COUT>(to, pix, o0, v);
                        }
                    }
                }
            }
            __syncthreads();                           // this halo's reads are done; the next one is built
            tile += G;
            if (tile >= a.ntiles) break;
        }
        return;
    }
    // producers: wave pw = wid - 4 issues the DMA pieces a 4-wave block would
    // (fetch's lane-linear layout); thread pt builds make_geo(pt)'s halo tasks
    const int pw = wid - 4, pt = t - 256;
    auto fetch2 = [&](int tl, _Float16 *patch, uint32_t *imgs) {
        int b, y0, x0, ly0, lx0;
        tile_coords(a, tl, b, y0, x0, ly0, lx0);
        const __amdgpu_buffer_rsrc_t fr = image_rsrc(a.fm + (int64_t)b * a.Hin * a.Win * 32, (int64_t)a.Hin * a.Win * 64);
        const int base = (ly0 * a.Win + lx0) * 64;
#pragma unroll
        for (int i = 0; i < kPatchIt; ++i) {
            const int c0 = 256 * i + 64 * pw, c = c0 + lane;
            if (c0 < kPatchChunks && c < kPatchChunks) {
                const int pp = c >> 2, pr = pp / kPC;
                const int off = base + pr * a.Win * 64 + (pp - pr * kPC) * 64 + 16 * (c & 3);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(fr, (__attribute__((address_space(3))) void *)(patch + 8 * c0),
                                                         16, off, 0, 0, 0);
            }
        }
        const __amdgpu_buffer_rsrc_t ir = image_rsrc(a.img + (int64_t)b * a.H * a.W * 3, (int64_t)a.H * a.W * 6);
        const int ibase = ((y0 - 1) * a.W * 3 / 2 + x0 * 3 / 2 - 2) * 4;
#pragma unroll
        for (int i = 0; i < kImgIt; ++i) {
            const int w0 = 256 * i + 64 * pw, w = w0 + lane;
            if (w0 < kImgWords && w < kImgWords) {
                const int r = w / kImgDw;
                const int off = ibase + r * a.W * 6 + (w - r * kImgDw) * 4;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(ir, (__attribute__((address_space(3))) void *)(imgs + w0), 4,
                                                         off, 0, 0, 0);
            }
        }
    };
    const Geo g = make_geo(pt);
    auto build = [&](int tl, const _Float16 *patch, const uint32_t *imgs, _Float16 *halo) {
        int b, y0, x0, ly0, lx0;
        tile_coords(a, tl, b, y0, x0, ly0, lx0);
        const int ox0 = x0 - 1 + (g.rc0 >> 2), ox1 = x0 - 1 + (g.rc1 >> 2);
        const bool ok0 = ox0 >= 0 && ox0 < a.W, ok1 = ox1 >= 0 && ox1 < a.W;
        const ColW w0 = col_weights(a, g.rc0, x0, lx0);
#pragma unroll
        for (int i = 0; i < 5; ++i) halo_blend(a, patch, halo, w0, g.rc0, g.rhy0 + i, ok0, y0, ly0);
        if (g.rx) halo_blend(a, patch, halo, col_weights(a, g.rc1, x0, lx0), g.rc1, g.rhy1, ok1, y0, ly0);
        for (int p = pt; p < kHaloPx; p += 256) {
            const int hy = p / kHC, hx = p - hy * kHC;
            const int oy = y0 - 1 + hy, ox = x0 - 1 + hx;
            h8 v = {};
            if (oy >= 0 && oy < a.H && ox >= 0 && ox < a.W) {
                const uint16_t *ip = (const uint16_t *)(imgs + hy * kImgDw) + 3 * hx + 1;
                v[0] = __builtin_bit_cast(_Float16, ip[0]);
                v[1] = __builtin_bit_cast(_Float16, ip[1]);
                v[2] = __builtin_bit_cast(_Float16, ip[2]);
            }
            *(h8 *)(halo + p * kCP + 32) = v;
        }
    };
    // tile i's patch and image rows in buffer i % 3: fetched in phase i - 2
    // (after that phase's build), read in phase i - 1; a phase waits only for
    // the previous phase's pieces (a counted vmcnt: wave 0 issues 6 pieces
    // per tile, waves 1-3 four)
    fetch2(tile, patch2[0], imgs2[0]);
    if (tile + G < a.ntiles) fetch2(tile + G, patch2[1], imgs2[1]);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();                                   // every producer's pieces have landed
    build(tile, patch2[0], imgs2[0], halo2[0]);
    __syncthreads();
    for (int k = 0;; ++k) {
        const int t1 = tile + G, t2 = tile + 2 * G;
        if (t1 < a.ntiles) build(t1, patch2[(k + 1) % 3], imgs2[(k + 1) % 3], halo2[(k + 1) & 1]);
        if (t2 < a.ntiles) {
            fetch2(t2, patch2[(k + 2) % 3], imgs2[(k + 2) % 3]);
            if (pw == 0) __builtin_amdgcn_s_waitcnt(0x0F76);   // vmcnt(6): tile k + 2's in flight, k + 1's landed
            else __builtin_amdgcn_s_waitcnt(0x0F74);           // vmcnt(4)
        } else {
            __builtin_amdgcn_s_waitcnt(0x0F70);
        }
        __syncthreads();
        tile = t1;
        if (tile >= a.ntiles) break;
    }
}



// ==========================================================================
// The backbone's wide 3x3 convolutions (layer2 / layer3 / layer4 / fc /
// conv8s: Cin a multiple of 64, Cout of 128, stride 1, padding = dilation;
// RN:21-38, 167-198, MR:22-35) as an implicit GEMM on v_mfma_f32_16x16x32_f16, with
// the conv epilogue (folded BN bias, residual, ReLU; k_epilogue's roundings)
// fused.  D[cout][pixel] = sum_k W[cout][k] X[k][pixel], k = tap * Cin + c.
//
// Block: 16 waves, a 256-cout x 256-pixel tile (wave = 64 couts x 64 pixels:
// 4 x 4 accumulator tiles of 16 x 16; 111 VGPRs, 4 waves per SIMD).  K-step = 64 (one tap, 64
// input channels): the weights' and the pixels' 256 rows x 128 bytes each go
// to LDS by buffer loads straight to LDS (16 bytes a lane; rows outside the
// image or past the map read as zeros -- the convolution's zero padding),
// two stages (128 KiB), the next step's loads in flight while this step's
// 64 MFMAs per wave run; one barrier per step.  LDS image: row r's 16-byte
// segment s at granule 8 r + (s ^ (r & 7)) (the XOR swizzle is applied to
// the loads' source addresses; the LDS side is lane-linear), which keeps the
// fragments' ds_read_b128 conflict-free.  The accumulator's 4 registers are
// 4 consecutive output channels of one pixel: an 8-byte store per lane.
// Cout a multiple of 128 but not 256 (layer2, conv8s): 128-cout tiles (wave =
// 32 couts x 64 pixels, 2 x 4 accumulators; 96 KiB of LDS).
// ==========================================================================
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kCT = 256;                   // couts per tile (128 for Cout a multiple of 128 only)
constexpr int kPT = 256;                   // pixels per tile

struct ConvArgs {
    const _Float16 *x;      // [N][Hin][Win][Cin]
    const _Float16 *x2;     // second input or null: [N][H][W][Cin2] (cat) or [N][H2][W2][Cin2] (1x1)
    const _Float16 *w;      // [Cout][ksteps][64]: tap-major [9][Cin (+ Cin2)], then (1x1) [Cin2]
    const _Float16 *bias;   // [Cout]
    const _Float16 *res;    // [N][H][W][Cout] or null
    const _Float16 *rbias;  // [Cout] or null
    _Float16 *out;          // [N][H][W][ldo]
    int N, H, W, Cin, Cout, ldo, dil, act, ntp, nct, ntiles, ksteps, cblocks;
    int Hin, Win, stride;   // the main input's geometry (output pixel (y, x) reads (stride y + dy, stride x + dx))
    int mode2, Cin2, H2, W2, s2, cb1, nmain;   // PV_CONV_X2_*; cb1 = Cin / 64; nmain = 9 cblocks
    int nfull, nsplit;      // tiles run whole (blocks 0 .. nfull-1); each later tile in nsplit K parts
    u4 *slab;               // split tiles' f32 partials [tail][part][f][1024 threads] (16 B each)
    int *tick;              // [tail] arrival counters (zeroed per call)
    float slope;
    int64_t M;              // output pixels
};

// LDS image of a stage: row r's 16-byte segment s at granule 8 r + (s ^ (r & 7))
[[maybe_unused]] __device__ __forceinline__ int conv_granule(int row, int seg) { return row * 8 + (seg ^ (row & 7)); }

// 16 bytes a lane from a buffer straight to LDS (wave-uniform LDS base + 16 x lane)
__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, uint8_t *lds_base, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)lds_base, 16, voff, soff, 0,
                                             0);
}

#ifndef PVC_NW
#define PVC_NW 16
#endif
#ifndef PVC_CB_MAJOR
#define PVC_CB_MAJOR 1
#endif
#ifndef PVC_WINDOW
#define PVC_WINDOW 0             // 1: stride-1 convolutions on k_conv3x3w (A/B variant; measured slower)
#endif
#ifndef PVC_FRAG_AHEAD
#define PVC_FRAG_AHEAD 0         // 1: a step's fragments all read before its MFMAs (A/B, with PVC_NW=8)
#endif
#ifndef PVC_RING4
#define PVC_RING4 0              // 1: k_conv3x3r, 32-channel half steps in a ring of four stages (A/B: bit-identical, measured ~25 % slower)
#endif
#ifndef PVC_XRING3
#define PVC_XRING3 0             // 1: k_conv3x3's pixel stages in a ring of three (issued two steps ahead), weights in two
#endif
#ifndef PVC_PRIO
#define PVC_PRIO 0               // 1: s_setprio(1) around each MFMA cluster (A/B)
#endif
#ifndef PVC_ISSUE_MID
#define PVC_ISSUE_MID 2          // 0 before the step's MFMAs, 1 after its first half, 2 = 1 for 256-cout tiles only
#endif
#ifndef PVC_REGSTAGE
// 1: k_conv3x3's operands staged through registers (buffer_load to VGPRs,
// ds_write_b128 into the stage) instead of buffer loads to LDS.  A step's
// loads are issued two steps ahead and written into the free stage in the
// middle of the step before their use, so each load has a whole step
// (~3k cycles) to arrive.  The LDS-DMA form cannot keep loads in flight
// across a barrier: the compiler waits for every outstanding LDS-DMA
// (vmcnt(0)) before the next ds_read of the LDS it may alias -- which also
// drained PVC_XRING3's third stage at every step.  Measured 7-9 % slower on
// every wide shape (profiles/r06/conv_regstage_ab.txt); kept off.
#define PVC_REGSTAGE 0
#endif
constexpr int kNW = PVC_NW;                   // waves per block: 16 (4 cout x 4 pixel groups; 8 = 2 x 4 measured 5-8 % slower)

// The end of a k_conv3x3 / k_conv3x3w tile: a split tile's part hands its
// f32 partials over (the last part to arrive sums them in part order), then
// the epilogue (bias, residual (+ its bias), activation; k_epilogue's
// roundings) and the channels-last stores.
template <int CT, int MI, int WC>
__device__ __forceinline__ void conv_finish(const ConvArgs &a, f4v (&acc)[MI][4], int tail, int part, int n0,
                                            int64_t p0, int wn, int wm, int lane, uint8_t *lds) {
    if (tail >= 0) {
        // Hand-off (MI355X_MICROARCH.md, "Valid forms", sc1 row): sc1
        // (write-through) partial stores, every wave's vmcnt(0), a barrier,
        // one agent-scope ticket add; the last arriver reads every other
        // part's partials with sc1 loads.
        constexpr int NF = MI * 4;                    // 16-byte accumulator groups per thread
        const int64_t slab_bytes = (int64_t)a.nsplit * NF * (64 * kNW) * 16;
        const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
            (void *)((uint8_t *)a.slab + (int64_t)tail * slab_bytes), 0, (int)slab_bytes, 0x00020000);
        const int tbase = (int)threadIdx.x * 16;
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const int f = mi * 4 + ni;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, acc[mi][ni]), sr,
                                                       ((part * NF + f) * (64 * kNW)) * 16 + tbase, 0, 16);
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int *flag = (int *)lds;                       // the stages are free: the loop's reads are done
        if (threadIdx.x == 0) {
            const int t = __hip_atomic_fetch_add(&a.tick[tail], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            flag[0] = t == a.nsplit - 1;
        }
        __syncthreads();
        if (!flag[0]) return;
        if (threadIdx.x == 0) a.tick[tail] = 0;       // zero again for the next call on this ws
        // every part's partials from the slabs (this block's own included), in
        // part order: the sum does not depend on which part arrived last, and
        // the accumulators are reused (no second register set)
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const int f = mi * 4 + ni;
                f4v t = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(sr, f * (64 * kNW) * 16 + tbase, 0, 16));
                for (int p = 1; p < a.nsplit; ++p)
                    t += __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(
                                                     sr, ((p * NF + f) * (64 * kNW)) * 16 + tbase, 0, 16));
                acc[mi][ni] = t;
            }
    }
    // ---- epilogue: lane's accumulator (mi, ni) = couts c .. c+3 of pixel p;
    // k_epilogue's roundings (bias add, residual (+ its bias), activation) ----
    h4 bq[MI], rbq[MI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
        const int c = n0 + wn * (MI * 16) + mi * 16 + 4 * (lane >> 4);
        bq[mi] = *(const h4 *)(a.bias + c);
        rbq[mi] = a.rbias ? *(const h4 *)(a.rbias + c) : h4{};
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
        const int64_t p = p0 + wm * 64 + ni * 16 + (lane & 15);
        const bool pv = p < a.M;
        const int64_t pc = pv ? p : 0;
        h4 r[MI];
        if (a.res) {
#pragma unroll
            for (int mi = 0; mi < MI; ++mi)
                r[mi] = *(const h4 *)(a.res + pc * a.Cout + n0 + wn * (MI * 16) + mi * 16 + 4 * (lane >> 4));
        }
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
            const int c = n0 + wn * (MI * 16) + mi * 16 + 4 * (lane >> 4);
            h4 y;
#pragma unroll
            for (int j = 0; j < 4; ++j) y[j] = (_Float16)((float)(_Float16)acc[mi][ni][j] + (float)bq[mi][j]);
            if (a.res) {
                h4 rr = r[mi];
                if (a.rbias) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) rr[j] = (_Float16)((float)rr[j] + (float)rbq[mi][j]);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) y[j] = (_Float16)((float)y[j] + (float)rr[j]);
            } else if (a.rbias) {
                // the downsample's bias (its convolution summed in the accumulator)
#pragma unroll
                for (int j = 0; j < 4; ++j) y[j] = (_Float16)((float)y[j] + (float)rbq[mi][j]);
            }
            if (a.act == 1) {
#pragma unroll
                for (int j = 0; j < 4; ++j) y[j] = (float)y[j] > 0.f ? y[j] : (_Float16)0.f;
            } else if (a.act == 2) {
#pragma unroll
                for (int j = 0; j < 4; ++j) y[j] = (float)y[j] > 0.f ? y[j] : (_Float16)((float)y[j] * a.slope);
            }
            if (pv) *(h4 *)(a.out + p * a.ldo + c) = y;
        }
    }
}

#ifdef PVC_CLOCK_TRACE
// diagnostic builds only: per block, s_memtime and s_memrealtime (100 MHz)
// before the K loop and after it -- the in-kernel shader clock (MI355X_MICROARCH
// "DVFS give-back": MFMA-dense loops hold the clock well below 2.4 GHz)
__device__ unsigned long long *g_conv_clk;
#endif
template <int CT>
__global__ __launch_bounds__(64 * kNW) void k_conv3x3(ConvArgs a) {
#ifdef PVC_CLOCK_TRACE
    const unsigned long long ck0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    constexpr int KB = 64;                                 // K-step: one tap x 64 input channels
    constexpr int RB = KB * 2;                             // bytes per LDS row
    constexpr int STAGE = (CT + kPT) * RB;                 // 64 KiB (CT 256), 48 KiB (CT 128)
    constexpr int GPR = RB / 16;                           // 16-byte granules per row
    constexpr int NI = (kPT * RB) / (1024 * kNW);          // pixel buffer-to-LDS loads per wave per stage
    constexpr int NW = (CT * RB) / (1024 * kNW);           // weight loads per wave per stage
    constexpr int WC = kNW / 4;                            // cout groups of waves
    constexpr int MI = CT / WC / 16;                       // 16-cout accumulator tiles per wave
#if PVC_XRING3
    // weights in a ring of two stages, pixels in a ring of three: a step's
    // pixel loads are issued two steps ahead (their L2 / HBM latency exceeds
    // the ~half step the two-stage form leaves them); 160 KiB at CT 256
    constexpr int WST = CT * RB, XST = kPT * RB;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WST + 3 * XST];
#else
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE];
#endif
    const int lane = (int)(threadIdx.x & 63), wid = (int)(threadIdx.x >> 6);
    // XCD-aware tile order: blocks i, i + 8, ... share an XCD; give each XCD a
    // contiguous range of tiles, pixel tile major (PVC_PT_MAJOR)
    // The last partial round of tiles (ntiles mod CUs) is cut into nsplit K
    // parts run by nsplit blocks each (dispatched last), so that round ends
    // nsplit x sooner; the part that arrives last sums the others' f32
    // partials (in part order: deterministic) and runs the epilogue.
    int bid = (int)blockIdx.x, part = 0, tail = -1;
    if (bid < a.nfull) {
        const int nb = a.nfull, q = nb / 8, r = nb % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    } else {
        const int j = bid - a.nfull;
        tail = j / a.nsplit;
        part = j - tail * a.nsplit;
        bid = a.nfull + tail;
    }
#if PVC_PT_MAJOR
    const int ct = bid % a.nct, pt = bid / a.nct;     // a pixel tile's cout tiles adjacent (same XCD, same time)
#else
    const int ct = bid / a.ntp, pt = bid % a.ntp;
#endif
    const int n0 = ct * CT;
    const int64_t p0 = (int64_t)pt * kPT;
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.w, 0, (int)((int64_t)a.Cout * a.ksteps * 128), 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.x, 0, (int)((int64_t)a.N * a.Hin * a.Win * a.Cin * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t x2r = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.x2, 0,
        a.mode2 == PV_CONV_X2_1X1 ? (int)((int64_t)a.N * a.H2 * a.W2 * a.Cin2 * 2)
                                  : (int)((int64_t)a.N * a.Hin * a.Win * a.Cin2 * 2),
        0x00020000);
    const int K2 = a.ksteps * RB;            // bytes per weight row
    const int cbk = a.cblocks;               // channel blocks per tap (both inputs' for a cat)
    const int ksteps = a.ksteps;
    // this lane's NW weight and NI pixel granules per stage: granule g = (N wid + i) 64 + lane
    int woff[NW];
    // per pixel granule: its output pixel's input position (stride applied;
    // far out of range for rows past the map) and its byte offset in x (and in
    // x2: the same pixel of the cat's second map, or the 1x1 input's pixel),
    // segment included -- a step adds one wave-uniform tap / channel delta
    int pyb[NI], pxb[NI];
    uint32_t pb1[NI], pb2[NI];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const int g = (NW * wid + i) * 64 + lane, row = g / GPR, pseg = g % GPR;
        const int seg = conv_granule(row, pseg) - row * GPR;   // the swizzle is an involution per row
        woff[i] = (n0 + row) * K2 + seg * 16;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int g = (NI * wid + i) * 64 + lane, row = g / GPR, pseg = g % GPR;
        const int seg = conv_granule(row, pseg) - row * GPR;
        const int64_t p = p0 + row;
        const bool pin = p < a.M;
        const int64_t pc = pin ? p : 0;
        const int img = (int)(pc / ((int64_t)a.H * a.W)), rem = (int)(pc - (int64_t)img * a.H * a.W);
        const int py = rem / a.W, px = rem - py * a.W;
        pyb[i] = pin ? py * a.stride : -(1 << 28);
        pxb[i] = px * a.stride;
        const int pix = (img * a.Hin + py * a.stride) * a.Win + px * a.stride;
        pb1[i] = (uint32_t)(pix * a.Cin * 2 + seg * 16);
        if (a.mode2 == PV_CONV_X2_1X1)
            pb2[i] = pin ? (uint32_t)(((img * a.H2 + py * a.s2) * a.W2 + px * a.s2) * a.Cin2 * 2 + seg * 16)
                         : 0x80000000u;
        else
            pb2[i] = (uint32_t)(pix * a.Cin2 * 2 + seg * 16);
    }
#if PVC_CB_MAJOR
    // K order: step s of the 3x3 part is (channel block s / 9, tap s % 9): a
    // tile's nine taps read the same channel block of its (dilated) halo
    // within nine consecutive steps, while those lines are still in the XCD's
    // L2 (tap-major, a line came back one channel sweep -- cbk steps of every
    // tile on the XCD -- later, after the 4 MB L2 had turned over: layer4's
    // 512 -> 512 launches fetched 1.9x the bytes they fetch now).
    auto step_tap = [&](int s) { return s % 9; };
    auto step_cb = [&](int s) { return s / 9; };
#else
    auto step_tap = [&](int s) { return s / cbk; };
    auto step_cb = [&](int s) { return s % cbk; };
#endif
    // the K index (tap * cbk + cb: the weights' memory order) of step s
    auto kidx = [&](int s) { return s < a.nmain ? step_tap(s) * cbk + step_cb(s) : s; };
    auto issue_w = [&](int s, int buf) {
#if PVC_XRING3
        uint8_t *st = lds + buf * WST;
#else
        uint8_t *st = lds + buf * STAGE;
#endif
        const int ks = kidx(s);
#pragma unroll
        for (int i = 0; i < NW; ++i) glds16(wr, st + (NW * wid + i) * 1024, woff[i], ks * RB);
    };
    auto issue_x = [&](int s, int buf) {
#if PVC_XRING3
        uint8_t *st = lds + 2 * WST + buf * XST;
#else
        uint8_t *st = lds + buf * STAGE + CT * RB;
#endif
        if (a.mode2 == PV_CONV_X2_1X1 && s >= a.nmain) {
            // the 1x1 second input (the BasicBlock's downsample): centre tap at stride s2
            const uint32_t cbo = (uint32_t)(s - a.nmain) * RB;
#pragma unroll
            for (int i = 0; i < NI; ++i) glds16(x2r, st + (NI * wid + i) * 1024, pb2[i] + cbo, 0);
            return;
        }
        const int tap = step_tap(s), cb = step_cb(s);
        const int dy = (tap / 3 - 1) * a.dil, dx = (tap % 3 - 1) * a.dil;
        const bool second = a.mode2 == PV_CONV_X2_CAT && cb >= a.cb1;   // the concatenation's second part
        const int C = second ? a.Cin2 : a.Cin, cbo = (second ? cb - a.cb1 : cb) * RB;
        const uint32_t delta = (uint32_t)((dy * a.Win + dx) * C * 2 + cbo);
        uint32_t off[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const bool ok = (unsigned)(pyb[i] + dy) < (unsigned)a.Hin && (unsigned)(pxb[i] + dx) < (unsigned)a.Win;
            off[i] = ok ? (second ? pb2[i] : pb1[i]) + delta : 0x80000000u;
        }
        if (second) {
#pragma unroll
            for (int i = 0; i < NI; ++i) glds16(x2r, st + (NI * wid + i) * 1024, off[i], 0);
        } else {
#pragma unroll
            for (int i = 0; i < NI; ++i) glds16(xr, st + (NI * wid + i) * 1024, off[i], 0);
        }
    };
    auto issue = [&](int s, int buf) { issue_w(s, buf); issue_x(s, buf); };
    const int wn = wid % WC, wm = wid / WC;  // wave: couts wn*(256/WC) .., pixels wm*64 .. +63
    f4v acc[MI][4];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f4v{0.f, 0.f, 0.f, 0.f};
    // a step half's fragments (kc: 32 of its 64 channels) and its MFMAs
    auto read_frags = [&](const uint8_t *st, int kc, h8v (&af)[MI], h8v (&bf)[4]) {
        const int sg = kc * 4 + (lane >> 4);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
            const int r = wn * (MI * 16) + mi * 16 + (lane & 15);
            af[mi] = *(const h8v *)(st + conv_granule(r, sg) * 16);
        }
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int r = wm * 64 + ni * 16 + (lane & 15);
            bf[ni] = *(const h8v *)(st + CT * RB + conv_granule(r, sg) * 16);
        }
    };
    auto mfma_frags = [&](const h8v (&af)[MI], const h8v (&bf)[4]) {
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
    };
    (void)read_frags;
    (void)mfma_frags;
    // kc-th half of a step (32 of its 64 channels)
    auto compute_kx = [&](const uint8_t *st, const uint8_t *xst, int kc) {
        {
            const int sg = kc * 4 + (lane >> 4);
            h8v af[MI], bf[4];
#pragma unroll
            for (int mi = 0; mi < MI; ++mi) {
                const int r = wn * (MI * 16) + mi * 16 + (lane & 15);
                af[mi] = *(const h8v *)(st + conv_granule(r, sg) * 16);
            }
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const int r = wm * 64 + ni * 16 + (lane & 15);
                bf[ni] = *(const h8v *)(xst + conv_granule(r, sg) * 16);
            }
#ifdef PVC_NO_MFMA
#pragma unroll
            for (int mi = 0; mi < MI; ++mi) acc[mi][0][0] += (float)af[mi][0] + (float)bf[mi & 3][1];
#else
#if PVC_PRIO
            __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
            for (int mi = 0; mi < MI; ++mi)
#pragma unroll
                for (int ni = 0; ni < 4; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
#if PVC_PRIO
            __builtin_amdgcn_s_setprio(0);
#endif
#endif
        }
    };
    auto compute_kc = [&](const uint8_t *st, int kc) { compute_kx(st, st + CT * RB, kc); };
    const int k0 = tail < 0 ? 0 : part * ksteps / a.nsplit;
    const int k1 = tail < 0 ? ksteps : (part + 1) * ksteps / a.nsplit;
#if PVC_REGSTAGE && !PVC_XRING3
    (void)issue;
    // the same source offsets and LDS image as issue_w / issue_x (granule g of
    // the stage <- the lane's swizzled 16-byte source segment), by way of
    // registers: rw / rx hold step s + 1's operands while step s computes
    u4 rw[NW], rx[NI];
    auto load_regs = [&](int s) {
        const int ks = kidx(s);
#pragma unroll
        for (int i = 0; i < NW; ++i) rw[i] = __builtin_amdgcn_raw_buffer_load_b128(wr, woff[i], ks * RB, 0);
        if (a.mode2 == PV_CONV_X2_1X1 && s >= a.nmain) {
            const uint32_t cbo = (uint32_t)(s - a.nmain) * RB;
#pragma unroll
            for (int i = 0; i < NI; ++i) rx[i] = __builtin_amdgcn_raw_buffer_load_b128(x2r, pb2[i] + cbo, 0, 0);
            return;
        }
        const int tap = step_tap(s), cb = step_cb(s);
        const int dy = (tap / 3 - 1) * a.dil, dx = (tap % 3 - 1) * a.dil;
        const bool second = a.mode2 == PV_CONV_X2_CAT && cb >= a.cb1;
        const int C = second ? a.Cin2 : a.Cin, cbo = (second ? cb - a.cb1 : cb) * RB;
        const uint32_t delta = (uint32_t)((dy * a.Win + dx) * C * 2 + cbo);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const bool ok = (unsigned)(pyb[i] + dy) < (unsigned)a.Hin && (unsigned)(pxb[i] + dx) < (unsigned)a.Win;
            const uint32_t off = ok ? (second ? pb2[i] : pb1[i]) + delta : 0x80000000u;
            rx[i] = __builtin_amdgcn_raw_buffer_load_b128(second ? x2r : xr, off, 0, 0);
        }
    };
    auto store_regs = [&](int buf) {
        uint8_t *st = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < NW; ++i) *(u4 *)(st + (NW * wid + i) * 1024 + lane * 16) = rw[i];
#pragma unroll
        for (int i = 0; i < NI; ++i) *(u4 *)(st + CT * RB + (NI * wid + i) * 1024 + lane * 16) = rx[i];
    };
    load_regs(k0);
    store_regs(0);
    if (k0 + 1 < k1) load_regs(k0 + 1);
    for (int s = k0; s < k1; ++s) {
        const int buf = (s - k0) & 1;
        __syncthreads();                              // stage buf written by every wave; step s-1's reads done
        compute_kc(lds + buf * STAGE, 0);
        if (s + 1 < k1) {
            store_regs(buf ^ 1);                      // step s + 1's operands (loaded a step ago)
            if (s + 2 < k1) load_regs(s + 2);
        }
        compute_kc(lds + buf * STAGE, 1);
    }
#elif PVC_XRING3
    (void)compute_kc;
    (void)issue;
    issue_x(k0, 0);
    issue_w(k0, 0);
    if (k0 + 1 < k1) issue_x(k0 + 1, 1);
    for (int s = k0; s < k1; ++s) {
        const int i = s - k0, wb = i & 1, xb = i % 3;
        // this wave's weights(s) and pixels(s) have landed: only pixels(s + 1),
        // issued after weights(s), may still be in flight
        if (s + 1 < k1) __builtin_amdgcn_s_waitcnt(0x0F70 | NI);
        else __builtin_amdgcn_s_waitcnt(0x0F70);
        // ... every wave's; step s-1's reads are done.  A bare s_barrier:
        // __syncthreads' workgroup release fence would wait for every
        // outstanding LDS-DMA (vmcnt(0)), pixels(s + 1) included
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const uint8_t *wst = lds + wb * WST, *xst = lds + 2 * WST + xb * XST;
        compute_kx(wst, xst, 0);
        if (s + 1 < k1) issue_w(s + 1, wb ^ 1);
        if (s + 2 < k1) issue_x(s + 2, (i + 2) % 3);
        compute_kx(wst, xst, 1);
    }
#else
    issue(k0, 0);
    for (int s = k0; s < k1; ++s) {
        const int buf = (s - k0) & 1;
        __builtin_amdgcn_s_waitcnt(0x0F70);          // this wave's loads of step s have landed (vmcnt 0)
#ifdef PVC_NO_BARRIER
        if (s == k0)
#endif
        __syncthreads();                              // ... and every wave's; step s-1's reads are done
#ifdef PVC_NO_LOADS
        const bool nx = s == k0 && k1 - k0 > 1;
#else
        const bool nx = s + 1 < k1;
#endif
#if PVC_FRAG_AHEAD
        if (true) {
            // both halves' fragments read before the step's MFMAs (the
            // second half's reads in flight under the first half's MFMAs;
            // registers for 8-wave blocks), the next step's loads between
            const uint8_t *st = lds + buf * STAGE;
            h8v a0[MI], b0[4], a1[MI], b1[4];
            read_frags(st, 0, a0, b0);
            read_frags(st, 1, a1, b1);
            mfma_frags(a0, b0);
            if (nx) issue(s + 1, buf ^ 1);
            mfma_frags(a1, b1);
        } else
#endif
        if (PVC_ISSUE_MID == 1 || (PVC_ISSUE_MID == 2 && CT == 256)) {
            // the next step's loads after this step's first 16 MFMAs: the MFMA
            // pipe starts right after the barrier instead of behind every
            // wave's address arithmetic and load issue (256-cout tiles: layer4
            // 625-645 -> 584-630 us; the 128-cout tiles measured 4-7 % slower)
            compute_kc(lds + buf * STAGE, 0);
            if (nx) issue(s + 1, buf ^ 1);
            compute_kc(lds + buf * STAGE, 1);
        } else {
            if (nx) issue(s + 1, buf ^ 1);
            compute_kc(lds + buf * STAGE, 0);
            compute_kc(lds + buf * STAGE, 1);
        }
    }
#endif
#ifdef PVC_CLOCK_TRACE
    if (g_conv_clk && threadIdx.x == 0 && tail < 0) {
        unsigned long long *q = g_conv_clk + (int64_t)blockIdx.x * 4;
        q[0] = ck0; q[1] = rt0; q[2] = __builtin_amdgcn_s_memtime(); q[3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    conv_finish<CT, MI, WC>(a, acc, tail, part, n0, p0, wn, wm, lane, lds);
}


// --------------------------------------------------------------------------
// k_conv3x3 with a four-stage ring of half steps (round 5): the same tiles,
// tile order, split-K, epilogue and MFMA sequence (so the same sums, bit for
// bit), but each 64-channel step's two 32-channel halves are staged
// separately -- a stage is CT + 256 rows x 64 bytes (32 KiB at CT 256) -- in a
// ring of four, and a half step's loads are issued three half steps before
// it is consumed, right after the barrier that frees their stage.  The wait
// before a half step is for its own loads only (a counted vmcnt: the two
// newer half steps' stay in flight), so the loads' latency is covered by
// three half steps of MFMAs instead of half a step (the 2-stage form issued
// the next step's loads mid-step and waited for them at the next barrier).
// LDS image: row r's 16-byte granule g at 4 r + (g ^ ((r >> 1) & 3))
// (conflict-free for the 16x16x32 fragments' ds_read_b128).
// --------------------------------------------------------------------------
[[maybe_unused]] __device__ __forceinline__ int ring_granule(int row, int seg) { return row * 4 + (seg ^ ((row >> 1) & 3)); }

template <int CT>
__global__ __launch_bounds__(64 * kNW) void k_conv3x3r(ConvArgs a) {
    constexpr int RB = 64;                                 // bytes per LDS row (32 channels)
    constexpr int STAGE = (CT + kPT) * RB;                 // 32 KiB (CT 256), 24 KiB (CT 128)
    constexpr int GPR = RB / 16;                           // 4 granules per row
    constexpr int NI = (kPT * RB) / (1024 * kNW);          // pixel pieces per wave per stage: 1
    constexpr int WPW = CT * RB / 1024;                    // weight pieces per stage: 16 (CT 256), 8 (CT 128)
    constexpr int WC = kNW / 4;                            // cout groups of waves
    constexpr int MI = CT / WC / 16;                       // 16-cout accumulator tiles per wave
    static_assert(NI == 1 && WPW <= kNW, "one pixel piece per wave, at most one weight piece");
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * STAGE];
    const int lane = (int)(threadIdx.x & 63), wid = (int)(threadIdx.x >> 6);
    const bool wload = wid < WPW;                          // this wave stages one weight piece per half step
    int bid = (int)blockIdx.x, part = 0, tail = -1;
    if (bid < a.nfull) {
        const int nb = a.nfull, q = nb / 8, r = nb % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    } else {
        const int j = bid - a.nfull;
        tail = j / a.nsplit;
        part = j - tail * a.nsplit;
        bid = a.nfull + tail;
    }
#if PVC_PT_MAJOR
    const int ct = bid % a.nct, pt = bid / a.nct;
#else
    const int ct = bid / a.ntp, pt = bid % a.ntp;
#endif
    const int n0 = ct * CT;
    const int64_t p0 = (int64_t)pt * kPT;
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.w, 0, (int)((int64_t)a.Cout * a.ksteps * 128), 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.x, 0, (int)((int64_t)a.N * a.Hin * a.Win * a.Cin * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t x2r = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.x2, 0,
        a.mode2 == PV_CONV_X2_1X1 ? (int)((int64_t)a.N * a.H2 * a.W2 * a.Cin2 * 2)
                                  : (int)((int64_t)a.N * a.Hin * a.Win * a.Cin2 * 2),
        0x00020000);
    const int K2 = a.ksteps * 128;           // bytes per weight row
    const int cbk = a.cblocks;
    const int nmain2 = 2 * a.nmain;          // half steps of the 3x3 part
    // this wave's weight piece (rows 16 wid .. +15) and pixel piece (rows 16 wid .. +15)
    int woff = 0, pyb, pxb;
    uint32_t pb1, pb2;
    {
        const int g = wid * 64 + lane, row = g / GPR, pseg = g % GPR;
        const int seg = pseg ^ ((row >> 1) & 3);
        woff = (n0 + row) * K2 + seg * 16;
        const int64_t p = p0 + row;
        const bool pin = p < a.M;
        const int64_t pc = pin ? p : 0;
        const int img = (int)(pc / ((int64_t)a.H * a.W)), rem = (int)(pc - (int64_t)img * a.H * a.W);
        const int py = rem / a.W, px = rem - py * a.W;
        pyb = pin ? py * a.stride : -(1 << 28);
        pxb = px * a.stride;
        const int pix = (img * a.Hin + py * a.stride) * a.Win + px * a.stride;
        pb1 = (uint32_t)(pix * a.Cin * 2 + seg * 16);
        if (a.mode2 == PV_CONV_X2_1X1)
            pb2 = pin ? (uint32_t)(((img * a.H2 + py * a.s2) * a.W2 + px * a.s2) * a.Cin2 * 2 + seg * 16) : 0x80000000u;
        else
            pb2 = (uint32_t)(pix * a.Cin2 * 2 + seg * 16);
    }
    // half step h: 64-channel step s = h / 2 (channel block s / 9, tap s % 9, as
    // k_conv3x3's PVC_CB_MAJOR order; the 1x1 part after it), channels
    // 32 (h % 2) .. of it
    auto issue = [&](int h, int buf) {
        uint8_t *st = lds + buf * STAGE;
        const int s = h >> 1, hf = h & 1;
        if (wload) {
            const int ks = s < a.nmain ? (s % 9) * cbk + s / 9 : s;
            glds16(wr, st + wid * 1024, (uint32_t)woff, (uint32_t)(ks * 128 + hf * 64));
        }
        uint8_t *px = st + CT * RB + wid * 1024;
        if (a.mode2 == PV_CONV_X2_1X1 && s >= a.nmain) {
            glds16(x2r, px, pb2 + (uint32_t)((h - nmain2) * 64), 0);
            return;
        }
        const int tap = s % 9, cb = s / 9;
        const int dy = (tap / 3 - 1) * a.dil, dx = (tap % 3 - 1) * a.dil;
        const bool second = a.mode2 == PV_CONV_X2_CAT && cb >= a.cb1;
        const int C = second ? a.Cin2 : a.Cin, cbo = (second ? cb - a.cb1 : cb) * 128 + hf * 64;
        const uint32_t delta = (uint32_t)((dy * a.Win + dx) * C * 2 + cbo);
        const bool ok = (unsigned)(pyb + dy) < (unsigned)a.Hin && (unsigned)(pxb + dx) < (unsigned)a.Win;
        const uint32_t off = ok ? (second ? pb2 : pb1) + delta : 0x80000000u;
        glds16(second ? x2r : xr, px, off, 0);
    };
    const int wn = wid % WC, wm = wid / WC;
    f4v acc[MI][4];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f4v{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](const uint8_t *st) {
        const int sg = lane >> 4;
        h8v af[MI], bf[4];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
            const int r = wn * (MI * 16) + mi * 16 + (lane & 15);
            af[mi] = *(const h8v *)(st + ring_granule(r, sg) * 16);
        }
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int r = wm * 64 + ni * 16 + (lane & 15);
            bf[ni] = *(const h8v *)(st + CT * RB + ring_granule(r, sg) * 16);
        }
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
    };
    const int ksteps = a.ksteps;
    const int k0 = 2 * (tail < 0 ? 0 : part * ksteps / a.nsplit);
    const int k1 = 2 * (tail < 0 ? ksteps : (part + 1) * ksteps / a.nsplit);
#pragma unroll
    for (int u = 0; u < 3; ++u)
        if (k0 + u < k1) issue(k0 + u, u);
    for (int h = k0; h < k1; ++h) {
        // this wave's pieces of half step h have landed; those of the (up to)
        // two half steps issued after it may still be in flight
        const int ahead = min(2, k1 - 1 - h);
        if (wload) {
            if (ahead == 2) __builtin_amdgcn_s_waitcnt(0x0F74);        // vmcnt(4)
            else if (ahead == 1) __builtin_amdgcn_s_waitcnt(0x0F72);   // vmcnt(2)
            else __builtin_amdgcn_s_waitcnt(0x0F70);
        } else {
            if (ahead == 2) __builtin_amdgcn_s_waitcnt(0x0F72);        // vmcnt(2)
            else if (ahead == 1) __builtin_amdgcn_s_waitcnt(0x0F71);   // vmcnt(1)
            else __builtin_amdgcn_s_waitcnt(0x0F70);
        }
        __syncthreads();                       // ... and every wave's; half step h - 1's reads are done
        if (h + 3 < k1) issue(h + 3, (h + 3 - k0) & 3);
        compute(lds + ((h - k0) & 3) * STAGE);
    }
    conv_finish<CT, MI, WC>(a, acc, tail, part, n0, p0, wn, wm, lane, lds);
}

// --------------------------------------------------------------------------
// The window form (stride 1, dilation <= kMaxDil): the same tiles, K order
// (channel block, ky, kx) and epilogue as k_conv3x3, but a tile's pixel
// operand for the three taps of one kernel row ky comes from ONE window of
// 256 + 2d consecutive pixels (the tile's, shifted by the row offset dy and
// widened by d on both sides) staged once in LDS: tap kx reads the window's
// rows shifted by (kx - 1) d, and the lanes whose pixel x + dx leaves its
// image row (where the linear shift wraps into the next row) take zeros, the
// convolution's padding.  A step's loads drop from 32 KiB of weights + 32 KiB
// of pixels to 32 KiB + a third of a 33 KiB window (layer4: ~2/3 of the
// bytes, and 2 + 1 instead of 4 LDS-DMA pieces per wave and step).  A
// window's 33 pieces are issued in thirds during the three steps of the
// window before it; the downsample's 1x1 steps (PV_CONV_X2_1X1) are
// one-step windows of the tile's own 256 pixels.
// LDS: 2 weight stages (CT rows x 128 B) + 2 windows (264 rows x 128 B).
// Measured (round 4, tools/r04_gpu5.sh): correct (the conv3x3 parity cases)
// but slower than k_conv3x3 on every layer (layer4 640-690 against 583-630
// us): the kernel is not bound by its bytes; the masking and the longer
// path from the barrier to the first MFMA cost more than the loads saved.
// Kept as an A/B build (PVC_WINDOW=1), not in the product library.
// --------------------------------------------------------------------------
#if PVC_WINDOW
constexpr int kMaxDil = 4;
constexpr int kWinRows = kPT + 2 * kMaxDil;          // 264
constexpr int kWinPieces = kWinRows * 128 / 1024;    // 33 LDS-DMA pieces (1 KiB) per window
constexpr int kWinThird = (kWinPieces + 2) / 3;      // 11: pieces per step, one per wave 0..10

template <int CT>
__global__ __launch_bounds__(64 * kNW) void k_conv3x3w(ConvArgs a) {
    constexpr int RB = 128;                                // bytes per LDS row (64 channels)
    constexpr int GPR = RB / 16;
    constexpr int WST = CT * RB;                           // weight stage: 32 KiB (CT 256)
    constexpr int XST = kWinRows * RB;                     // window: 33 KiB
    constexpr int NW = (CT * RB) / (1024 * kNW);           // weight pieces per wave per step
    constexpr int WC = kNW / 4;
    constexpr int MI = CT / WC / 16;
    static_assert(kWinThird <= kNW, "one window piece per wave and step");
    // + a 128-byte zero block: the B rows of lanes whose shifted tap leaves its image row
    __shared__ __attribute__((aligned(128))) uint8_t lds[2 * WST + 2 * XST + 128];
    if (threadIdx.x < 8) *(uint4 *)(lds + 2 * WST + 2 * XST + 16 * threadIdx.x) = make_uint4(0u, 0u, 0u, 0u);
    const int lane = (int)(threadIdx.x & 63), wid = (int)(threadIdx.x >> 6);
    int bid = (int)blockIdx.x, part = 0, tail = -1;
    if (bid < a.nfull) {
        const int nb = a.nfull, q = nb / 8, r = nb % 8, x = bid % 8;
        bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    } else {
        const int j = bid - a.nfull;
        tail = j / a.nsplit;
        part = j - tail * a.nsplit;
        bid = a.nfull + tail;
    }
    const int ct = bid % a.nct, pt = bid / a.nct;
    const int n0 = ct * CT;
    const int64_t p0 = (int64_t)pt * kPT;
    const int d = a.dil;
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.w, 0, (int)((int64_t)a.Cout * a.ksteps * 128), 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.x, 0, (int)((int64_t)a.N * a.H * a.W * a.Cin * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t x2r = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.x2, 0,
        a.mode2 == PV_CONV_X2_1X1 ? (int)((int64_t)a.N * a.H2 * a.W2 * a.Cin2 * 2)
                                  : (int)((int64_t)a.N * a.H * a.W * a.Cin2 * 2),
        0x00020000);
    const int K2 = a.ksteps * RB;
    const int cbk = a.cblocks;
    const int64_t HW = (int64_t)a.H * a.W;
    int woff[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const int g = (NW * wid + i) * 64 + lane, row = g / GPR, pseg = g % GPR;
        woff[i] = (n0 + row) * K2 + (pseg ^ (row & 7)) * 16;
    }
    // this lane's window granules: piece u * kWinThird + wid (u = 0..2, waves
    // 0..10), row = piece * 8 + lane / 8, segment (lane & 7) ^ (row & 7); for
    // the 3x3 windows the pixel q = p0 - d + row (its index and row y, or far
    // out of range past the window / the map), for the 1x1 windows the byte
    // offset of pixel p0 + row's input in x2
    const uint32_t seg16 = (uint32_t)(((lane & 7) ^ (lane >> 3)) * 16);
    int qpix[3], qy[3];
    uint32_t qds[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
        const int piece = u * kWinThird + wid, row = piece * 8 + (lane >> 3);
        const int64_t q = p0 - d + row;
        const bool in = wid < kWinThird && piece < kWinPieces && row < kPT + 2 * d && q >= 0 && q < a.M;
        const int64_t qc = in ? q : 0;
        const int img = (int)(qc / HW), rem = (int)(qc - img * HW), y = rem / a.W;
        qpix[u] = (int)qc;
        qy[u] = in ? y : -(1 << 28);
        const int64_t q1 = p0 + row;
        const bool in1 = wid < kWinThird && row < kPT && q1 < a.M;
        const int64_t qc1 = in1 ? q1 : 0;
        const int img1 = (int)(qc1 / HW), rem1 = (int)(qc1 - img1 * HW), y1 = rem1 / a.W, x1 = rem1 - y1 * a.W;
        qds[u] = a.mode2 == PV_CONV_X2_1X1 && in1
                     ? (uint32_t)(((img1 * a.H2 + y1 * a.s2) * a.W2 + x1 * a.s2) * a.Cin2 * 2) + seg16
                     : 0x80000000u;
    }
    const int wn = wid % WC, wm = wid / WC;
    // x of this lane's B-operand pixel in each 16-pixel group (zero padding of shifted taps)
    int xp[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
        const int64_t p = p0 + wm * 64 + ni * 16 + (lane & 15);
        const int64_t pc = p < a.M ? p : 0;
        xp[ni] = (int)((pc % HW) % a.W);
    }
    // step s -> window j, its first step and length; 3x3 part: (cb s / 9, ky, kx)
    auto win_of = [&](int s) { return s < a.nmain ? s / 3 : a.nmain / 3 + (s - a.nmain); };
    auto win_first = [&](int j) { return j < a.nmain / 3 ? 3 * j : a.nmain + (j - a.nmain / 3); };
    auto issue_w = [&](int s, int buf) {
        // K index of step s: (cb, tap) -> tap * cbk + cb (the weights' memory order)
        const int ks = s < a.nmain ? (s % 9) * cbk + s / 9 : s;
        uint8_t *st = lds + buf * WST;
#pragma unroll
        for (int i = 0; i < NW; ++i) glds16(wr, st + (NW * wid + i) * 1024, woff[i], ks * RB);
    };
    // third u of window j (its piece u * kWinThird + wid) into window buffer j & 1
    auto issue_third = [&](int j, int u) {
        if (wid >= kWinThird) return;
        const int piece = u * kWinThird + wid;
        if (piece >= kWinPieces) return;
        uint8_t *st = lds + 2 * WST + (j & 1) * XST + piece * 1024;
        if (j >= a.nmain / 3) {                       // the downsample's 1x1 input, channel block j - nmain/3
            const uint32_t cbo = (uint32_t)(j - a.nmain / 3) * RB;
            glds16(x2r, st, qds[u] + cbo, 0);
            return;
        }
        const int cb = j / 3, ky = j - 3 * cb;
        const int dy = (ky - 1) * d;
        const bool second = a.mode2 == PV_CONV_X2_CAT && cb >= a.cb1;
        const int C = second ? a.Cin2 : a.Cin;
        const uint32_t cbo = (uint32_t)((second ? cb - a.cb1 : cb) * RB);
        const bool ok = (unsigned)(qy[u] + dy) < (unsigned)a.H;
        const uint32_t off = ok ? (uint32_t)((qpix[u] + dy * a.W) * C * 2) + cbo + seg16 : 0x80000000u;
        glds16(second ? x2r : xr, st, off, 0);
    };
    f4v acc[MI][4];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f4v{0.f, 0.f, 0.f, 0.f};
    // kc-th half of step s (32 of its 64 channels): A from weight stage wst, B
    // from the LDS byte offsets boff[ni] of this step's kc 0 granules (kc 1's
    // are boff ^ 64: segment 4 + q of a row lies at granule (4 + q) ^ (r & 7)
    // = that of q, xor 4); a lane outside its image row points at the zero block
    auto compute_kc = [&](const uint8_t *wst, const uint32_t (&boff)[4], int kc) {
        const int sg = kc * 4 + (lane >> 4);
        h8v af[MI], bf[4];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
            const int r = wn * (MI * 16) + mi * 16 + (lane & 15);
            af[mi] = *(const h8v *)(wst + conv_granule(r, sg) * 16);
        }
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) bf[ni] = *(const h8v *)(lds + (boff[ni] ^ (uint32_t)(kc * 64)));
#ifdef PVC_NO_MFMA
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) acc[mi][0][0] += (float)af[mi][0] + (float)bf[mi & 3][1];
#else
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)
                acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mi], bf[ni], acc[mi][ni], 0, 0, 0);
#endif
    };
    const int ksteps = a.ksteps;
    const int k0 = tail < 0 ? 0 : part * ksteps / a.nsplit;
    const int k1 = tail < 0 ? ksteps : (part + 1) * ksteps / a.nsplit;
    issue_w(k0, 0);
    {
        const int j0 = win_of(k0);
        for (int u = 0; u < 3; ++u) issue_third(j0, u);
    }
    for (int s = k0; s < k1; ++s) {
        const int wbuf = (s - k0) & 1;
        const int j = win_of(s), f = win_first(j), len = j < a.nmain / 3 ? 3 : 1, t = s - f;
        __builtin_amdgcn_s_waitcnt(0x0F70);          // this wave's loads for step s have landed (vmcnt 0)
        __syncthreads();                              // ... and every wave's; step s-1's reads are done
        // B rows of this step: window row = tile row + d + dx (3x3) or the tile row (1x1)
        int sh = 0;
        unsigned msk = 0xF;
        if (j < a.nmain / 3) {
            const int dx = (t - 1) * d;               // kx = t
            sh = d + dx;
            if (dx != 0) {
                msk = 0;
#pragma unroll
                for (int ni = 0; ni < 4; ++ni) msk |= ((unsigned)(xp[ni] + dx) < (unsigned)a.W ? 1u : 0u) << ni;
            }
        }
        const uint8_t *wst = lds + wbuf * WST;
        uint32_t boff[4];
        {
            const int r0 = wm * 64 + (lane & 15) + sh;
            const uint32_t b0 = (uint32_t)(2 * WST + (j & 1) * XST + conv_granule(r0, lane >> 4) * 16);
#pragma unroll
            for (int ni = 0; ni < 4; ++ni)          // + ni * 16 rows keeps the swizzle
                boff[ni] = (msk >> ni) & 1 ? b0 + (uint32_t)(ni * 16 * RB) : (uint32_t)(2 * WST + 2 * XST);
        }
        compute_kc(wst, boff, 0);
        if (s + 1 < k1) issue_w(s + 1, wbuf ^ 1);
        // the next window's thirds: this step's own, plus the earlier ones when
        // the part started inside window j, plus the rest at the window's last step
        if (win_first(j + 1) < k1) {
            const int lo = s == k0 ? 0 : t, hi = t == len - 1 ? 2 : t;
            for (int u = lo; u <= hi; ++u) issue_third(j + 1, u);
        }
        compute_kc(wst, boff, 1);
    }
    conv_finish<CT, MI, WC>(a, acc, tail, part, n0, p0, wn, wm, lane, lds);
}
#endif  // PVC_WINDOW


// ==========================================================================
// conv2s with the upsampling and concatenation before it (MR:43-51,75-78:
// up4sto2s, torch.cat([fm, x2s], 1), conv2s = 3x3 conv + BN + LeakyReLU):
// out = leaky(conv3x3(cat(up2(fm), skip)) + b), fp16, channels-last, in one
// pass: fm [N][Hin][Win][64] (conv4s's output), skip [N][H][W][64] (x2s),
// out [N][H][W][32].  The unfused form writes the 128-channel cat (629 MB
// at batch 32), reads it back nine times over for MIOpen's convolution and
// passes its output through an epilogue.
//
// Persistent blocks of 8 waves (one per CU: 144 KiB LDS); an 8 x 32 output
// tile; per tile the 10 x 34 halo is built twice in one LDS buffer -- first
// the 64 upsampled channels (separable blend from a 7 x 19 fm patch, packed
// fp16, as pv_decoder_tail), then the 64 skip channels (copied) -- and each
// time every wave runs its 32-pixel output row's half of the convolution:
// 36 v_mfma_f32_32x32x16_f16, A = the weights (all 73.7 KB of them resident
// in LDS for the launch, read as one 16-byte row fragment per MFMA), B = one
// 16-byte LDS read of 8 channels of one halo pixel (XOR-swizzled within the
// pixel's 128 bytes: conflict-free).  The next tile's patch and skip pixels
// are loaded into registers (buffer loads, zero outside the maps) while this
// tile convolves.  Epilogue in registers: fp16 round of the f32 sums, + b,
// LeakyReLU (y * slope in f32), 8-byte stores of 4 consecutive channels.
// ==========================================================================
[[maybe_unused]] constexpr int kDCo = 32, kDC1 = 64, kDC2 = 64;
[[maybe_unused]] constexpr int kDOct = 9 * (kDC1 + kDC2) / 8;          // weight octets (16 bytes of 8 channels): 144
constexpr int kDPatch = kPR * kPC * (kDC1 / 8);       // fm patch chunks: 1064
[[maybe_unused]] constexpr int kDPatchIt = (kDPatch + 511) / 512;
[[maybe_unused]] constexpr int kDTcol = kPR * kHC * (kDC1 / 8);        // column blends: 1904
constexpr int kDHalo = kHaloPx * 8;                   // halo chunks per part: 2720
constexpr int kDSkipIt = (kDHalo + 511) / 512;

struct DecConvArgs {
    const _Float16 *fm, *skip;
    const _Float16 *w;      // [2 parts][9 taps][8 octets][32 couts][8]: the LDS image of the weights
    const _Float16 *bias;   // [32]
    _Float16 *out;
    int N, Hin, Win, H, W, tiles_r, tiles_c, ntiles;
    float rh, rw, slope;
};

__device__ __forceinline__ int halo_granule(int hp, int q) { return hp * 8 + (q ^ (hp & 7)); }

constexpr int kEC1 = 128, kECo = 64;                  // conv4s: fm channels, couts

#if PVC_DEC_V1
__global__ __launch_bounds__(512) void k_dec_conv2s(DecConvArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kDOct * kDCo * 16 + kDHalo * 16 + kDTcol * 16];
    uint8_t *wl = lds;                                  // 73,728 B
    uint8_t *halo = lds + kDOct * kDCo * 16;            // 43,520 B (the fm patch aliases its front)
    uint8_t *tcol = halo + kDHalo * 16;                 // 30,464 B
    const int t = (int)threadIdx.x, lane = t & 63, wid = t >> 6;
    const int n = lane & 31, h = lane >> 5;
    // the weights, once per launch
    for (int i = t; i < kDOct * kDCo; i += 512) *(h8 *)(wl + i * 16) = *(const h8 *)(a.w + i * 8);
    const h4 bq[4] = {*(const h4 *)(a.bias + 0 + 4 * h), *(const h4 *)(a.bias + 8 + 4 * h),
                      *(const h4 *)(a.bias + 16 + 4 * h), *(const h4 *)(a.bias + 24 + 4 * h)};
    auto coords = [&](int tile, int &b, int &y0, int &x0, int &ly0, int &lx0) {
        const int tc = tile % a.tiles_c, rest = tile / a.tiles_c;
        b = rest / a.tiles_r;
        y0 = (rest % a.tiles_r) * kTR;
        x0 = tc * kTC;
        ly0 = (int)(a.rh * (float)max(y0 - 1, 0));
        lx0 = (int)(a.rw * (float)max(x0 - 1, 0));
    };
    // prefetch of a tile's fm patch and skip halo into registers
    h8 ppre[kDPatchIt], spre[kDSkipIt];
    auto fetch = [&](int tile) {
        int b, y0, x0, ly0, lx0;
        coords(tile, b, y0, x0, ly0, lx0);
        const __amdgpu_buffer_rsrc_t fr = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.fm + (int64_t)b * a.Hin * a.Win * kDC1), 0, a.Hin * a.Win * kDC1 * 2, 0x00020000);
#pragma unroll
        for (int i = 0; i < kDPatchIt; ++i) {
            const int c = min(t + 512 * i, kDPatch - 1), pp = c >> 3, q = c & 7;
            const int pr = pp / kPC, pc = pp - pr * kPC;
            const int off = ((ly0 + pr) * a.Win + lx0 + pc) * (kDC1 * 2) + q * 16;   // rows past fm read 0
            ppre[i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(fr, off, 0, 0));
        }
        const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.skip + (int64_t)b * a.H * a.W * kDC2), 0, a.H * a.W * kDC2 * 2, 0x00020000);
#pragma unroll
        for (int i = 0; i < kDSkipIt; ++i) {
            const int c = min(t + 512 * i, kDHalo - 1), hp = c >> 3, q = c & 7;
            const int hy = hp / kHC, hx = hp - hy * kHC;
            const int oy = y0 - 1 + hy, ox = x0 - 1 + hx;
            const bool ok = oy >= 0 && oy < a.H && ox >= 0 && ox < a.W;
            const uint32_t off = ok ? (uint32_t)((oy * a.W + ox) * (kDC2 * 2) + q * 16) : 0x80000000u;
            spre[i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(sr, off, 0, 0));
        }
    };
    __builtin_amdgcn_s_waitcnt(0x0F70);
    int tile = xcd_block((int)blockIdx.x, (int)gridDim.x);
    if (tile < a.ntiles) fetch(tile);
    __builtin_amdgcn_s_waitcnt(0x0F70);                // (every tile starts with its halo registers landed)
    for (; tile < a.ntiles; tile += (int)gridDim.x) {
        int b, y0, x0, ly0, lx0;
        coords(tile, b, y0, x0, ly0, lx0);
        __syncthreads();                      // the previous tile's skip-part reads of the halo are done
#pragma unroll
        for (int i = 0; i < kDPatchIt; ++i)
            if (t + 512 * i < kDPatch) *(h8 *)(halo + (t + 512 * i) * 16) = ppre[i];   // patch, at the halo's front
        __syncthreads();
        // column blends: (fm row r, halo column hx, octet q) -> tcol [r][hx][q]
        for (int task = t; task < kDTcol; task += 512) {
            const int q = task & 7, rc = task >> 3;
            const int r = rc / kHC, hx = rc - r * kHC;
            const int ox = min(max(x0 - 1 + hx, 0), a.W - 1);
            const float w1r = a.rw * (float)ox;
            const int w1 = (int)w1r, w1p = w1 < a.Win - 1 ? 8 : 0;
            const float w1l = w1r - (float)w1;
            const uint8_t *pp = halo + ((r * kPC + (w1 - lx0)) * 8 + q) * 16;
            const h8 A = *(const h8 *)pp, B = *(const h8 *)(pp + w1p * 16);
            *(h8 *)(tcol + task * 16) =
                __builtin_elementwise_fma(B, (h8)(_Float16)w1l, A * (h8)(_Float16)(1.f - w1l));
        }
        __syncthreads();                      // the patch is dead: the halo may be written
        // row blends -> halo (upsampled channels, zero outside the image)
        for (int task = t; task < kDHalo; task += 512) {
            const int q = task & 7, hp = task >> 3;
            const int hy = hp / kHC, hx = hp - hy * kHC;
            const int oy = y0 - 1 + hy, ox = x0 - 1 + hx;
            h8 v = {};
            if (oy >= 0 && oy < a.H && ox >= 0 && ox < a.W) {
                const float h1r = a.rh * (float)oy;
                const int h1 = (int)h1r;
                const int dh = h1 < a.Hin - 1 ? kHC * 8 * 16 : 0;
                const float h1l = h1r - (float)h1;
                const uint8_t *tp = tcol + (((h1 - ly0) * kHC + hx) * 8 + q) * 16;
                const h8 c0 = *(const h8 *)tp, c1 = *(const h8 *)(tp + dh);
                v = __builtin_elementwise_fma(c1, (h8)(_Float16)h1l, c0 * (h8)(_Float16)(1.f - h1l));
            }
            *(h8 *)(halo + halo_granule(hp, q) * 16) = v;
        }
        __syncthreads();
        if (tile + (int)gridDim.x < a.ntiles) {
            // the next tile's patch now (its skip pixels are still needed below)
            int nb, ny0, nx0, nly0, nlx0;
            coords(tile + (int)gridDim.x, nb, ny0, nx0, nly0, nlx0);
            const __amdgpu_buffer_rsrc_t fr = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(a.fm + (int64_t)nb * a.Hin * a.Win * kDC1), 0, a.Hin * a.Win * kDC1 * 2, 0x00020000);
#pragma unroll
            for (int i = 0; i < kDPatchIt; ++i) {
                const int c = min(t + 512 * i, kDPatch - 1), pp = c >> 3, q = c & 7;
                const int pr = pp / kPC, pc = pp - pr * kPC;
                const int off = ((nly0 + pr) * a.Win + nlx0 + pc) * (kDC1 * 2) + q * 16;
                ppre[i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(fr, off, 0, 0));
            }
        }
        // ---- the convolution, part by part: wave = output row wid, 32 pixels ----
        f16x acc = {};
        auto conv_part = [&](int part) {
            // fragments read PVC_L1_AHEAD k-steps ahead of their MFMAs (k_conv64)
            auto frag = [&](int s, h8 &af, h8 &bf) {
                const int o = 2 * s + h;                  // octet of this lane half: tap o / 8, channels 8 (o % 8)
                const int tap = o >> 3, q = o & 7;
                const int ky = tap / 3, kx = tap - 3 * ky;
                af = *(const h8 *)(wl + ((part * 72 + o) * kDCo + n) * 16);
                bf = *(const h8 *)(halo + halo_granule((wid + ky) * kHC + n + kx, q) * 16);
            };
            constexpr int AH = PVC_L1_AHEAD;
            h8 fa[AH + 1], fb[AH + 1];
#pragma unroll
            for (int s = 0; s < AH; ++s) frag(s, fa[s], fb[s]);
#pragma unroll
            for (int s = 0; s < 36; ++s) {
                if (s + AH < 36) frag(s + AH, fa[(s + AH) % (AH + 1)], fb[(s + AH) % (AH + 1)]);
                const int c = s % (AH + 1);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[c], fb[c], acc, 0, 0, 0);
            }
        };
        conv_part(0);
        __syncthreads();                      // every wave is done with the upsampled halo
#pragma unroll
        for (int i = 0; i < kDSkipIt; ++i) {
            const int c = t + 512 * i;
            if (c < kDHalo) *(h8 *)(halo + halo_granule(c >> 3, c & 7) * 16) = spre[i];
        }
        __syncthreads();
        if (tile + (int)gridDim.x < a.ntiles) {
            int nb, ny0, nx0, nly0, nlx0;
            coords(tile + (int)gridDim.x, nb, ny0, nx0, nly0, nlx0);
            const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(a.skip + (int64_t)nb * a.H * a.W * kDC2), 0, a.H * a.W * kDC2 * 2, 0x00020000);
#pragma unroll
            for (int i = 0; i < kDSkipIt; ++i) {
                const int c = min(t + 512 * i, kDHalo - 1), hp = c >> 3, q = c & 7;
                const int hy = hp / kHC, hx = hp - hy * kHC;
                const int oy = ny0 - 1 + hy, ox = nx0 - 1 + hx;
                const bool ok = oy >= 0 && oy < a.H && ox >= 0 && ox < a.W;
                const uint32_t off = ok ? (uint32_t)((oy * a.W + ox) * (kDC2 * 2) + q * 16) : 0x80000000u;
                spre[i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(sr, off, 0, 0));
            }
        }
        conv_part(1);
        // ---- epilogue: rows (i & 3) + 8 (i >> 2) + 4 h of acc = couts, column n = pixel ----
        const int oy = y0 + wid, ox = x0 + n;
        if (oy < a.H && ox < a.W) {
            _Float16 *op = a.out + (((int64_t)b * a.H + oy) * a.W + ox) * kDCo;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                h4 y;
#pragma unroll
                for (int j = 0; j < 4; ++j) y[j] = (_Float16)acc[4 * g + j];
                y = y + bq[g];
                h4 ys;
#pragma unroll
                for (int j = 0; j < 4; ++j) ys[j] = (_Float16)((float)y[j] * a.slope);
                *(h4 *)(op + 8 * g + 4 * h) = __builtin_elementwise_max(y, ys);
            }
        }
    }
}


// ==========================================================================
// conv4s with the upsampling and concatenation before it (MR:35-43,75-77:
// up8sto4s, torch.cat([fm, x4s], 1), conv4s = 3x3 conv + BN + LeakyReLU):
// fm [N][Hin][Win][128] (conv8s's output), skip [N][H][W][64] (x4s), out
// [N][H][W][64], fp16 channels-last, one pass.  k_dec_conv2s's structure
// with 192 input channels in three 64-channel parts (upsampled 0..63,
// upsampled 64..127, skip) and 64 output channels (two 32 x 32 accumulators
// per wave); the 221 KB of weights do not fit in LDS beside the halo, so each
// part's 73.7 KB are loaded straight to LDS (buffer loads) while its halo is
// built.
// ==========================================================================
constexpr int kEWPart = 9 * 8 * kECo;                 // weight octets (16 B) per part: 4608
constexpr int kEWIt = kEWPart * 16 / (1024 * 8);      // buffer-to-LDS loads per wave per part: 9

__global__ __launch_bounds__(512) void k_dec_conv4s(DecConvArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kEWPart * 16 + kDHalo * 16 + kDTcol * 16];
    uint8_t *wl = lds;                                  // 73,728 B: this part's weights
    uint8_t *halo = lds + kEWPart * 16;                 // 43,520 B (the fm patch aliases its front)
    uint8_t *tcol = halo + kDHalo * 16;                 // 30,464 B
    const int t = (int)threadIdx.x, lane = t & 63, wid = t >> 6;
    const int n = lane & 31, h = lane >> 5;
    h4 bq[2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) bq[m][g] = *(const h4 *)(a.bias + 32 * m + 8 * g + 4 * h);
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.w, 0, 3 * kEWPart * 16, 0x00020000);
    auto load_w = [&](int part) {   // this part's LDS image, 1 KB per wave instruction
#pragma unroll
        for (int i = 0; i < kEWIt; ++i)
            glds16(wr, wl + (kEWIt * wid + i) * 1024, (uint32_t)(((kEWIt * wid + i) * 64 + lane) * 16),
                   (uint32_t)(part * kEWPart * 16));
    };
    auto coords = [&](int tile, int &b, int &y0, int &x0, int &ly0, int &lx0) {
        const int tc = tile % a.tiles_c, rest = tile / a.tiles_c;
        b = rest / a.tiles_r;
        y0 = (rest % a.tiles_r) * kTR;
        x0 = tc * kTC;
        ly0 = (int)(a.rh * (float)max(y0 - 1, 0));
        lx0 = (int)(a.rw * (float)max(x0 - 1, 0));
    };
    h8 ppre[kDPatchIt], spre[kDSkipIt];
    // 64-channel slice `half` of a tile's fm patch
    auto fetch_patch = [&](int tile, int half) {
        int b, y0, x0, ly0, lx0;
        coords(tile, b, y0, x0, ly0, lx0);
        const __amdgpu_buffer_rsrc_t fr = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.fm + (int64_t)b * a.Hin * a.Win * kEC1), 0, a.Hin * a.Win * kEC1 * 2, 0x00020000);
#pragma unroll
        for (int i = 0; i < kDPatchIt; ++i) {
            const int c = min(t + 512 * i, kDPatch - 1), pp = c >> 3, q = c & 7;
            const int pr = pp / kPC, pc = pp - pr * kPC;
            const int off = ((ly0 + pr) * a.Win + lx0 + pc) * (kEC1 * 2) + half * 128 + q * 16;
            ppre[i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(fr, off, 0, 0));
        }
    };
    auto fetch_skip = [&](int tile) {
        int b, y0, x0, ly0, lx0;
        coords(tile, b, y0, x0, ly0, lx0);
        const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.skip + (int64_t)b * a.H * a.W * kDC2), 0, a.H * a.W * kDC2 * 2, 0x00020000);
#pragma unroll
        for (int i = 0; i < kDSkipIt; ++i) {
            const int c = min(t + 512 * i, kDHalo - 1), hp = c >> 3, q = c & 7;
            const int hy = hp / kHC, hx = hp - hy * kHC;
            const int oy = y0 - 1 + hy, ox = x0 - 1 + hx;
            const bool ok = oy >= 0 && oy < a.H && ox >= 0 && ox < a.W;
            const uint32_t off = ok ? (uint32_t)((oy * a.W + ox) * (kDC2 * 2) + q * 16) : 0x80000000u;
            spre[i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(sr, off, 0, 0));
        }
    };
    // the upsampled halo of the patch in ppre (64 channels)
    auto build_up = [&](int y0, int x0, int ly0, int lx0) {
#pragma unroll
        for (int i = 0; i < kDPatchIt; ++i)
            if (t + 512 * i < kDPatch) *(h8 *)(halo + (t + 512 * i) * 16) = ppre[i];
        __syncthreads();
        for (int task = t; task < kDTcol; task += 512) {
            const int q = task & 7, rc = task >> 3;
            const int r = rc / kHC, hx = rc - r * kHC;
            const int ox = min(max(x0 - 1 + hx, 0), a.W - 1);
            const float w1r = a.rw * (float)ox;
            const int w1 = (int)w1r, w1p = w1 < a.Win - 1 ? 8 : 0;
            const float w1l = w1r - (float)w1;
            const uint8_t *pp = halo + ((r * kPC + (w1 - lx0)) * 8 + q) * 16;
            const h8 A = *(const h8 *)pp, B = *(const h8 *)(pp + w1p * 16);
            *(h8 *)(tcol + task * 16) =
                __builtin_elementwise_fma(B, (h8)(_Float16)w1l, A * (h8)(_Float16)(1.f - w1l));
        }
        __syncthreads();
        for (int task = t; task < kDHalo; task += 512) {
            const int q = task & 7, hp = task >> 3;
            const int hy = hp / kHC, hx = hp - hy * kHC;
            const int oy = y0 - 1 + hy, ox = x0 - 1 + hx;
            h8 v = {};
            if (oy >= 0 && oy < a.H && ox >= 0 && ox < a.W) {
                const float h1r = a.rh * (float)oy;
                const int h1 = (int)h1r;
                const int dh = h1 < a.Hin - 1 ? kHC * 8 * 16 : 0;
                const float h1l = h1r - (float)h1;
                const uint8_t *tp = tcol + (((h1 - ly0) * kHC + hx) * 8 + q) * 16;
                const h8 c0 = *(const h8 *)tp, c1 = *(const h8 *)(tp + dh);
                v = __builtin_elementwise_fma(c1, (h8)(_Float16)h1l, c0 * (h8)(_Float16)(1.f - h1l));
            }
            *(h8 *)(halo + halo_granule(hp, q) * 16) = v;
        }
    };
    f16x acc[2];
    auto conv_part = [&]() {
        // fragments read PVC_L1_AHEAD k-steps ahead of their MFMAs (k_conv64)
        auto frag = [&](int s, h8 &bf, h8 &a0, h8 &a1) {
            const int o = 2 * s + h;
            const int tap = o >> 3, q = o & 7;
            const int ky = tap / 3, kx = tap - 3 * ky;
            bf = *(const h8 *)(halo + halo_granule((wid + ky) * kHC + n + kx, q) * 16);
            a0 = *(const h8 *)(wl + ((o * 2 + 0) * 32 + n) * 16);
            a1 = *(const h8 *)(wl + ((o * 2 + 1) * 32 + n) * 16);
        };
        constexpr int AH = PVC_L1_AHEAD;
        h8 fb[AH + 1], f0[AH + 1], f1[AH + 1];
#pragma unroll
        for (int s = 0; s < AH; ++s) frag(s, fb[s], f0[s], f1[s]);
#pragma unroll
        for (int s = 0; s < 36; ++s) {
            if (s + AH < 36) frag(s + AH, fb[(s + AH) % (AH + 1)], f0[(s + AH) % (AH + 1)], f1[(s + AH) % (AH + 1)]);
            const int c = s % (AH + 1);
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f0[c], fb[c], acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f1[c], fb[c], acc[1], 0, 0, 0);
        }
    };
    int tile = (int)blockIdx.x;
    if (tile < a.ntiles) { fetch_patch(tile, 0); fetch_skip(tile); }
    for (; tile < a.ntiles; tile += (int)gridDim.x) {
        int b, y0, x0, ly0, lx0;
        coords(tile, b, y0, x0, ly0, lx0);
        const bool more = tile + (int)gridDim.x < a.ntiles;
        acc[0] = acc[1] = f16x{};
#pragma unroll 1
        for (int part = 0; part < 3; ++part) {
            __syncthreads();                  // the previous part's convolution is done with halo and weights
            load_w(part);                     // lands while the halo is built
            if (part < 2) {
                build_up(y0, x0, ly0, lx0);
            } else {
#pragma unroll
                for (int i = 0; i < kDSkipIt; ++i) {
                    const int c = t + 512 * i;
                    if (c < kDHalo) *(h8 *)(halo + halo_granule(c >> 3, c & 7) * 16) = spre[i];
                }
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);   // this wave's weight loads have landed
            __syncthreads();
            // the next part's inputs, in flight during this part's convolution
            if (part == 0) fetch_patch(tile, 1);
            else if (part == 1 && more) fetch_patch(tile + (int)gridDim.x, 0);
            else if (part == 2 && more) fetch_skip(tile + (int)gridDim.x);
            conv_part();
        }
        // ---- epilogue: acc[m] rows (i & 3) + 8 (i >> 2) + 4 h = couts 32 m + .., column n = pixel ----
        const int oy = y0 + wid, ox = x0 + n;
        if (oy < a.H && ox < a.W) {
            _Float16 *op = a.out + (((int64_t)b * a.H + oy) * a.W + ox) * kECo;
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    h4 y;
#pragma unroll
                    for (int j = 0; j < 4; ++j) y[j] = (_Float16)acc[m][4 * g + j];
                    y = y + bq[m][g];
                    h4 ys;
#pragma unroll
                    for (int j = 0; j < 4; ++j) ys[j] = (_Float16)((float)y[j] * a.slope);
                    *(h4 *)(op + 32 * m + 8 * g + 4 * h) = __builtin_elementwise_max(y, ys);
                }
        }
    }
}

#endif  // PVC_DEC_V1

// ==========================================================================
// The decoder steps conv4s / conv2s, warp-specialised (round 5): the same
// operation as k_dec_conv4s / k_dec_conv2s above (up2(fm) + cat(., skip) + 3x3
// conv + bias + LeakyReLU, fp16 channels-last), with the halo build and the
// global loads no longer in sequence with the MFMAs.
//
// A tile (8 x 32 outputs of one image) is convolved in 32-channel parts: NUP
// upsampled parts (fm channels 32p ..), then 2 skip parts.  Persistent blocks
// of 16 waves, one per CU: waves 0-7 are consumers (wave = output row, 32
// pixels x CO couts, 18 v_mfma_f32_32x32x16_f16 per part and 32 couts), waves
// 8-15 producers.  One part per phase, one barrier per phase:
//   consumers: LDS-DMA the NEXT part's weights (36 x CO x 16 B, from the
//              host's [p64][9][8][CO][8] image) into the other weight buffer,
//              the MFMAs of this part, the epilogue after the last part;
//   producers: build the next part's halo (10 x 34 pixels x 32 channels,
//              64 B a pixel, granule q ^ ((hp >> 2) & 3): conflict-free) in
//              the other halo buffer -- an upsampled part blended from its
//              7 x 19 fm patch (in one of two patch buffers, written two
//              phases ahead from registers), a skip part copied from
//              registers -- and issue the next tile's global loads.
// The blend is pv_decoder_tail's / k_dec_conv2s's packed-fp16 separable
// blend (two column blends, one row blend), bit for bit; the summation order
// of the convolution is per 32-channel part (the former kernels: per 64).
// LDS: 2 weight + 2 halo + 2 patch buffers = 97 KB (conv2s) / 134 KB (conv4s).
// ==========================================================================
constexpr int kXHalo = kHaloPx * 4;                   // halo chunks (16 B) per 32-channel part: 1360
constexpr int kXHaloB = kXHalo * 16;                  // 21,760 B
constexpr int kXPatch = kPR * kPC * 4;                // fm patch chunks per part: 532
constexpr int kXPatchB = kXPatch * 16;                // 8,512 B
constexpr int kXSkipIt = (kXHalo + 511) / 512;        // chunks per producer thread: 3
constexpr int kXPatchIt = (kXPatch + 511) / 512;      // 2
constexpr int kXBlendIt = (kXHalo + 511) / 512;       // 3

__device__ __forceinline__ int halo32(int hp, int q) { return hp * 4 + (q ^ ((hp >> 2) & 3)); }

#ifdef PVC_DEC_TRACE
// trace builds only: per block, tile iteration < 4, phase < 6: s_memtime stamps
// [0] consumer phase start, [1] consumer MFMAs issued/done, [2] consumer wait
// done, [4] producer phase start, [5] producer loads issued, [6] producer
// build done, [7] producer patch writes done
__device__ unsigned long long *g_dec_trace;
#define PVD_STAMP(it, j, k)                                                                                 \
    if (g_dec_trace && (it) < 4 && lane == 0 && (wid == 0 || wid == kDecCW))                                  \
        g_dec_trace[(((int64_t)blockIdx.x * 4 + (it)) * 6 + (j)) * 8 + (k)] = __builtin_amdgcn_s_memtime()
#else
#define PVD_STAMP(it, j, k)
#endif

// Consumer waves (PVC_DEC_2ROW): 4, each two output rows -- a weight fragment
// read from LDS feeds both rows' MFMAs (half the weight reads of one row per
// wave; LDS bandwidth, not the matrix cores, bounded the one-row form) -- one
// per SIMD; or 8 of one row.  Producer waves: 8.
constexpr int kDecCW = PVC_DEC_2ROW ? 4 : 8;           // consumer waves
constexpr int kDecRows = kTR / kDecCW;                 // output rows per consumer wave
constexpr int kDecThreads = (kDecCW + 8) * 64;
template <int CO, int NUP>
__global__ __launch_bounds__(kDecThreads) void k_dec_conv(DecConvArgs a) {
    constexpr int C1 = 32 * NUP;                       // fm channels
    constexpr int P = NUP + 2;                         // parts per tile (even: buffer parity = part parity)
    constexpr int WB = 36 * CO * 16;                   // one part's weights in LDS
    constexpr int PIECES = WB / 1024;                  // LDS-DMA pieces per part (18 / 36)
    constexpr int MT = CO / 32;                        // 32-cout accumulators per consumer
    // the next tile's patch loads at phase 0 (conv2s) / 2 (conv4s: after this
    // tile's parts 2, 3 are written), its skip loads at the last phase (after
    // this tile's are consumed): one register set each
    constexpr int LP = NUP == 2 ? 0 : 2, LS = P - 1, SS = 1;
    static_assert(P % 2 == 0 && PIECES * 1024 == WB, "part parity and whole DMA pieces");
    // BAL (conv2s): parts in the order up0, skip0, up1, skip1, each in halo
    // buffer (part count) mod 3, so that part k can be built over phases k - 2
    // and k - 1: an upsampled part's blend is split in two halves, one per
    // phase, and every phase's producer work is half a blend (+ a skip copy in
    // phases 0 and 2) instead of a whole blend in two phases of four and a
    // copy in the other two (the blend phases were producer-bound, the copy
    // phases consumer-bound).
    constexpr bool BAL = PVC_DEC_BAL && NUP == 2;
    constexpr int NH = BAL ? 3 : 2;                    // halo buffers
    // the weight part (32-channel block of cat([up(fm), skip])) of phase j
    auto wpart = [](int j) { return BAL ? ((j >> 1) | ((j & 1) << 1)) : j; };
    // store instructions of a tile's epilogue (every one issued, out-of-range
    // pixels' dropped by the buffer range): the last phase's wait leaves them
    // in flight and waits for the weight DMA issued before them
    constexpr int NST = kDecRows * MT * 4;
    static_assert(NST <= 15, "vmcnt immediate");
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WB + NH * kXHaloB + 2 * kXPatchB + CO * 2];
    uint8_t *const wbuf = lds, *const hbuf = lds + 2 * WB, *const pbuf = lds + 2 * WB + NH * kXHaloB;
    _Float16 *const bl = (_Float16 *)(lds + 2 * WB + NH * kXHaloB + 2 * kXPatchB);   // the bias (consumers)
    const int t = (int)threadIdx.x, lane = t & 63, wid = t >> 6;
    [[maybe_unused]] const int n = lane & 31, h = lane >> 5;
    const bool consumer = wid < kDecCW;
    const int pt = t - kDecCW * 64;                    // producer thread (0..511)
    const int G = (int)gridDim.x;
    auto coords = [&](int tile, int &b, int &y0, int &x0, int &ly0, int &lx0) {
        const int tc = tile % a.tiles_c, rest = tile / a.tiles_c;
        b = rest / a.tiles_r;
        y0 = (rest % a.tiles_r) * kTR;
        x0 = tc * kTC;
        ly0 = (int)(a.rh * (float)max(y0 - 1, 0));
        lx0 = (int)(a.rw * (float)max(x0 - 1, 0));
    };
    // ---- consumers: weights by LDS-DMA, MFMAs, epilogue ----
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void *)a.w, 0, (P / 2) * 9 * 8 * CO * 16, 0x00020000);
    auto dma_weights = [&](int part, int buf) {        // consumer waves: pieces wid, wid + kDecCW, ...
        uint8_t *dst = wbuf + buf * WB;
        const int p64 = part >> 1, q0 = (part & 1) * 4;
        for (int i = wid; i < PIECES; i += kDecCW) {
            const int byte = i * 1024 + lane * 16;
            const int blk = byte / (CO * 16), within = byte - blk * (CO * 16);
            const int tap = blk >> 2, q = blk & 3;
            glds16(wr, dst + i * 1024, (uint32_t)(((p64 * 9 + tap) * 8 + q0 + q) * (CO * 16) + within), 0u);
        }
    };
    f16x acc[kDecRows][MT];
    // k-step s (tap s >> 1, channel half s & 1 of the part): the weight
    // fragments once, the halo fragment of each of the wave's rows; the
    // summation order of every output is the one-row form's
    auto mfma_part = [&](int wb, int hb) {
        const uint8_t *W = wbuf + wb * WB, *Hb = hbuf + hb * kXHaloB;
        auto frag = [&](int s, h8 (&bf)[kDecRows], h8 (&af)[MT]) {
            const int o = 2 * s + h, tap = o >> 2, q = o & 3;
            const int ky = tap / 3, kx = tap - 3 * ky;
#pragma unroll
            for (int r = 0; r < kDecRows; ++r)
                bf[r] = *(const h8 *)(Hb + halo32((kDecRows * wid + r + ky) * kHC + n + kx, q) * 16);
#pragma unroll
            for (int m = 0; m < MT; ++m) af[m] = *(const h8 *)(W + ((tap * 4 + q) * CO + 32 * m + n) * 16);
        };
        // (two rows of conv4s' 64 couts: 64 accumulator registers; fragments 2 steps ahead)
        constexpr int AH = kDecRows * MT > 2 ? 2 : PVC_DEC_AHEAD;
        h8 fb[AH + 1][kDecRows], fa[AH + 1][MT];
#pragma unroll
        for (int s = 0; s < AH; ++s) frag(s, fb[s], fa[s]);
#pragma unroll
        for (int s = 0; s < 18; ++s) {
            if (s + AH < 18) frag(s + AH, fb[(s + AH) % (AH + 1)], fa[(s + AH) % (AH + 1)]);
            const int c = s % (AH + 1);
#pragma unroll
            for (int r = 0; r < kDecRows; ++r)
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    acc[r][m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fa[c][m], fb[c][r], acc[r][m], 0, 0, 0);
        }
    };
    auto epilogue = [&](int tile) {
        int b, y0, x0, ly0, lx0;
        coords(tile, b, y0, x0, ly0, lx0);
        const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.out + (int64_t)b * a.H * a.W * CO), 0, a.H * a.W * CO * 2, 0x00020000);
#pragma unroll
        for (int r = 0; r < kDecRows; ++r) {
            const int oy = y0 + kDecRows * wid + r, ox = x0 + n;
            const uint32_t po = oy < a.H && ox < a.W ? (uint32_t)((oy * a.W + ox) * CO * 2) : 0x80000000u;
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    h4 y;
#pragma unroll
                    for (int j = 0; j < 4; ++j) y[j] = (_Float16)acc[r][m][4 * g + j];
                    y = y + *(const h4 *)(bl + 32 * m + 8 * g + 4 * h);
                    h4 ys;
#pragma unroll
                    for (int j = 0; j < 4; ++j) ys[j] = (_Float16)((float)y[j] * a.slope);
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, __builtin_elementwise_max(y, ys)), orr,
                                                          po + (32 * m + 8 * g + 4 * h) * 2, 0, 0);
                }
        }
    };
    // ---- producers: loads into registers, patch writes, halo builds ----
    h8 preg[2][kXPatchIt], sreg[SS][2][kXSkipIt];
    // a tile's fm patches of up parts [u0, u1) (part u into slot u & 1) / skip
    // halo (both parts) into registers; a tile past the last reads nothing
    // (out-of-range offsets)
    auto load_patch = [&](int tile, int u0, int u1) {
        int b, y0, x0, ly0, lx0;
        coords(min(tile, a.ntiles - 1), b, y0, x0, ly0, lx0);
        const __amdgpu_buffer_rsrc_t fr = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.fm + (int64_t)b * a.Hin * a.Win * C1), 0, a.Hin * a.Win * C1 * 2, 0x00020000);
#pragma unroll
        for (int i = 0; i < kXPatchIt; ++i) {
            const int c = min(pt + 512 * i, kXPatch - 1), pp = c >> 2, q = c & 3;
            const int pr = pp / kPC, pc = pp - pr * kPC;
            const uint32_t off = tile < a.ntiles ? (uint32_t)(((ly0 + pr) * a.Win + lx0 + pc) * (C1 * 2) + q * 16)
                                                 : 0x80000000u;   // rows past fm read 0
            for (int u = u0; u < u1; ++u)
                preg[u & 1][i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(fr, off, u * 64, 0));
        }
    };
    auto load_skip = [&](int tile, h8 (&sr)[2][kXSkipIt]) {
        int b, y0, x0, ly0, lx0;
        coords(min(tile, a.ntiles - 1), b, y0, x0, ly0, lx0);
        const __amdgpu_buffer_rsrc_t sr_ = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.skip + (int64_t)b * a.H * a.W * 64), 0, a.H * a.W * 64 * 2, 0x00020000);
#pragma unroll
        for (int i = 0; i < kXSkipIt; ++i) {
            const int c = min(pt + 512 * i, kXHalo - 1), hp = c >> 2, q = c & 3;
            const int hy = hp / kHC, hx = hp - hy * kHC;
            const int oy = y0 - 1 + hy, ox = x0 - 1 + hx;
            const bool ok = tile < a.ntiles && oy >= 0 && oy < a.H && ox >= 0 && ox < a.W;
            const uint32_t off = ok ? (uint32_t)((oy * a.W + ox) * 128 + q * 16) : 0x80000000u;
#pragma unroll
            for (int u = 0; u < 2; ++u)
                sr[u][i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(sr_, off, u * 64, 0));
        }
    };
    auto write_patch = [&](int up) {                   // up part `up`'s patch -> patch buffer up & 1
        uint8_t *pb = pbuf + (up & 1) * kXPatchB;
#pragma unroll
        for (int i = 0; i < kXPatchIt; ++i)
            if (pt + 512 * i < kXPatch) *(h8 *)(pb + (pt + 512 * i) * 16) = preg[up & 1][i];
    };
    auto build_skip = [&](int sp, int hidx, const h8 (&sr)[2][kXSkipIt]) {
        uint8_t *hb = hbuf + hidx * kXHaloB;
#pragma unroll
        for (int i = 0; i < kXSkipIt; ++i) {
            const int c = pt + 512 * i;
            if (c < kXHalo) *(h8 *)(hb + halo32(c >> 2, c & 3) * 16) = sr[sp][i];
        }
    };
    // the blend tasks of this producer thread: halo chunks pt + 512 i, i < 3
    // (the last only for pt < 336) -- pixel (thy[i], thx[i]), octet pt & 3;
    // tile independent
    int thy[kXBlendIt], thx[kXBlendIt];
#pragma unroll
    for (int i = 0; i < kXBlendIt; ++i) {
        const int hp = (pt + 512 * i) >> 2;
        thy[i] = hp / kHC;
        thx[i] = hp - thy[i] * kHC;
    }
    auto build_up = [&](int tile, int part) {          // blend of patch buffer part & 1 -> halo buffer part & 1
        int b, y0, x0, ly0, lx0;
        coords(tile, b, y0, x0, ly0, lx0);
        const uint8_t *pb = pbuf + (part & 1) * kXPatchB;
        uint8_t *hb = hbuf + (part & 1) * kXHaloB;
        const int q = pt & 3;
        // tasks [i0, i1): their four patch reads each first (their LDS
        // latencies overlap), then the blends; a halo pixel outside the image
        // reads a clamped one and stores zero
        auto tasks = [&](auto I0, auto I1) {
            constexpr int i0 = decltype(I0)::value, i1 = decltype(I1)::value;
            h8 A[i1 - i0], B[i1 - i0], C[i1 - i0], D[i1 - i0];
            float wl[i1 - i0], hl[i1 - i0];
            bool in[i1 - i0];
#pragma unroll
            for (int i = i0; i < i1; ++i) {
                const int k = i - i0;
                const int oy = y0 - 1 + thy[i], ox = x0 - 1 + thx[i];
                in[k] = oy >= 0 && oy < a.H && ox >= 0 && ox < a.W;
                const int oyc = min(max(oy, 0), a.H - 1), oxc = min(max(ox, 0), a.W - 1);
                const float w1r = a.rw * (float)oxc, h1r = a.rh * (float)oyc;
                const int w1 = (int)w1r, h1 = (int)h1r;
                const int dw = w1 < a.Win - 1 ? 4 : 0, dh = h1 < a.Hin - 1 ? kPC * 4 : 0;
                wl[k] = w1r - (float)w1;
                hl[k] = h1r - (float)h1;
                const uint8_t *pp = pb + (((h1 - ly0) * kPC + (w1 - lx0)) * 4 + q) * 16;
                A[k] = *(const h8 *)pp;
                B[k] = *(const h8 *)(pp + dw * 16);
                C[k] = *(const h8 *)(pp + dh * 16);
                D[k] = *(const h8 *)(pp + (dh + dw) * 16);
            }
#pragma unroll
            for (int i = i0; i < i1; ++i) {
                const int k = i - i0;
                const int c = pt + 512 * i;
                if (c >= kXHalo) break;
                const h8 ww = (h8)(_Float16)wl[k], w0 = (h8)(_Float16)(1.f - wl[k]);
                const h8 c0 = __builtin_elementwise_fma(B[k], ww, A[k] * w0);
                const h8 c1 = __builtin_elementwise_fma(D[k], ww, C[k] * w0);
                h8 v = __builtin_elementwise_fma(c1, (h8)(_Float16)hl[k], c0 * (h8)(_Float16)(1.f - hl[k]));
                if (!in[k]) v = h8{};
                *(h8 *)(hb + halo32(c >> 2, q) * 16) = v;
            }
        };
        static_assert(kXBlendIt == 3, "tasks 0-1, then 2");
        tasks(std::integral_constant<int, 0>{}, std::integral_constant<int, 2>{});
        tasks(std::integral_constant<int, 2>{}, std::integral_constant<int, 3>{});
    };

    int tile = xcd_block((int)blockIdx.x, G);
    if (tile >= a.ntiles) return;
    // The two roles run separate loops (so that their registers -- the
    // accumulators and fragments, the prefetched inputs -- share the file)
    // with the same barriers: two in the prologue, one per phase.
    if (consumer) {
        if (wid == 0 && lane < CO / 4) *(h4 *)(bl + 4 * lane) = *(const h4 *)(a.bias + 4 * lane);
        dma_weights(wpart(0), 0);                      // phase 0's weights
        int hk = 0;                                    // this phase's halo buffer
        __builtin_amdgcn_s_waitcnt(0x0F70);            // vmcnt(0)
        __syncthreads();
        __syncthreads();
        for (int it = 0;; ++it) {
            (void)it;
            const bool more = tile + G < a.ntiles;
#pragma unroll
            for (int r = 0; r < kDecRows; ++r)
#pragma unroll
                for (int m = 0; m < MT; ++m) acc[r][m] = f16x{};
#pragma unroll 1     // (unrolled, the phases' fragment and DMA registers overlap: spills at MT = 2)
            for (int j = 0; j < P; ++j) {
                PVD_STAMP(it, j, 0);
                if (j + 1 < P || more) dma_weights(wpart((j + 1) % P), (j + 1) & 1);
                mfma_part(j & 1, BAL ? hk : (j & 1));
                hk = hk == NH - 1 ? 0 : hk + 1;
                PVD_STAMP(it, j, 1);
                // this wave's weight pieces have landed, then every wave's (and
                // every wave's fragment reads of this part are done).  A plain
                // barrier: through __syncthreads' fence the compiler waits for
                // the epilogue's stores too (vmcnt(0)), ~4k cycles a tile
                if (j == P - 1) {
                    epilogue(tile);
                    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(NST) : "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
                }
                PVD_STAMP(it, j, 2);
            }
            tile += G;
            if (!more) break;
        }
        return;
    }
    if constexpr (BAL) {
        // one skip part's halo chunks into sreg[0][u] (a tile past the last reads nothing)
        auto load_skip1 = [&](int tile, int u) {
            int b, y0, x0, ly0, lx0;
            coords(min(tile, a.ntiles - 1), b, y0, x0, ly0, lx0);
            const __amdgpu_buffer_rsrc_t sr_ = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(a.skip + (int64_t)b * a.H * a.W * 64), 0, a.H * a.W * 64 * 2, 0x00020000);
#pragma unroll
            for (int i = 0; i < kXSkipIt; ++i) {
                const int c = min(pt + 512 * i, kXHalo - 1), hp = c >> 2, q = c & 3;
                const int hy = hp / kHC, hx = hp - hy * kHC;
                const int oy = y0 - 1 + hy, ox = x0 - 1 + hx;
                const bool ok = tile < a.ntiles && oy >= 0 && oy < a.H && ox >= 0 && ox < a.W;
                const uint32_t off = ok ? (uint32_t)((oy * a.W + ox) * 128 + q * 16) : 0x80000000u;
                sreg[0][u][i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(sr_, off, u * 64, 0));
            }
        };
        // half hf of an upsampled part's blend (halo chunks [680 hf, 680 hf + 680):
        // this thread's pt + 680 hf and, for pt < 168, + 512) from patch slot
        // `slot` into halo buffer hidx; the same arithmetic as build_up
        auto build_half = [&](int tile, int slot, int hidx, int hf) {
            int b, y0, x0, ly0, lx0;
            coords(tile, b, y0, x0, ly0, lx0);
            const uint8_t *pb = pbuf + slot * kXPatchB;
            uint8_t *hb = hbuf + hidx * kXHaloB;
            const int q = pt & 3;
            constexpr int kHalf = kXHalo / 2;
            static_assert(kHalf % 4 == 0 && kHalf > 512 && kHalf <= 1024, "two tasks per thread and half");
            const int cs[2] = {kHalf * hf + pt, kHalf * hf + pt + 512};
            h8 A[2], B[2], C[2], D[2];
            float wl[2], hl[2];
            bool in[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int hp = min(cs[k], kXHalo - 1) >> 2, hy = hp / kHC, hx = hp - hy * kHC;
                const int oy = y0 - 1 + hy, ox = x0 - 1 + hx;
                in[k] = oy >= 0 && oy < a.H && ox >= 0 && ox < a.W;
                const int oyc = min(max(oy, 0), a.H - 1), oxc = min(max(ox, 0), a.W - 1);
                const float w1r = a.rw * (float)oxc, h1r = a.rh * (float)oyc;
                const int w1 = (int)w1r, h1 = (int)h1r;
                const int dw = w1 < a.Win - 1 ? 4 : 0, dh = h1 < a.Hin - 1 ? kPC * 4 : 0;
                wl[k] = w1r - (float)w1;
                hl[k] = h1r - (float)h1;
                const uint8_t *pp = pb + (((h1 - ly0) * kPC + (w1 - lx0)) * 4 + q) * 16;
                A[k] = *(const h8 *)pp;
                B[k] = *(const h8 *)(pp + dw * 16);
                C[k] = *(const h8 *)(pp + dh * 16);
                D[k] = *(const h8 *)(pp + (dh + dw) * 16);
            }
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (k == 1 && pt + 512 >= kHalf) break;
                const h8 ww = (h8)(_Float16)wl[k], w0 = (h8)(_Float16)(1.f - wl[k]);
                const h8 c0 = __builtin_elementwise_fma(B[k], ww, A[k] * w0);
                const h8 c1 = __builtin_elementwise_fma(D[k], ww, C[k] * w0);
                h8 v = __builtin_elementwise_fma(c1, (h8)(_Float16)hl[k], c0 * (h8)(_Float16)(1.f - hl[k]));
                if (!in[k]) v = h8{};
                *(h8 *)(hb + halo32(cs[k] >> 2, q) * 16) = v;
            }
        };
        auto hnext = [](int h, int d) { h += d; return h >= 3 ? h - 3 : h; };
        // prologue: tile 0's patches (slots 0, 1) and skip parts; up0 built
        // whole into halo buffer 0 (phase 0's); up0 of the next tile loading
        load_patch(tile, 0, 2);
        load_skip1(tile, 0);
        load_skip1(tile, 1);
        write_patch(0);
        write_patch(1);
        __syncthreads();
        build_half(tile, 0, 0, 0);
        build_half(tile, 0, 0, 1);
        load_patch(tile + G, 0, 1);
        __syncthreads();
        // phase j: the consumers read halo buffer hk; this phase finishes part
        // k + 1 (buffer hk + 1) and starts part k + 2 (hk + 2), mod 3
        int hk = 0;
        [[maybe_unused]] int it = 0;                   // (trace builds: the tile iteration)
        for (;;) {
            const int nxt = tile + G;
            const bool more = nxt < a.ntiles;
            // phase 0: skip0 copied, up1's first half; slot 0 <- up0(nxt); loads up1(nxt)
            PVD_STAMP(it, 0, 4);
            build_skip(0, hnext(hk, 1), sreg[0]);
            build_half(tile, 1, hnext(hk, 2), 0);
            PVD_STAMP(it, 0, 5);
            write_patch(0);
            PVD_STAMP(it, 0, 6);
            load_patch(nxt, 1, 2);
            PVD_STAMP(it, 0, 7);
            __syncthreads();
            hk = hnext(hk, 1);
            // phase 1: up1's second half; loads skip0(nxt), up0(nxt + G)
            PVD_STAMP(it, 1, 4);
            build_half(tile, 1, hnext(hk, 1), 1);
            PVD_STAMP(it, 1, 5);
            PVD_STAMP(it, 1, 6);
            load_skip1(nxt, 0);
            load_patch(nxt + G, 0, 1);
            PVD_STAMP(it, 1, 7);
            __syncthreads();
            hk = hnext(hk, 1);
            // phase 2: skip1 copied, up0(nxt)'s first half; slot 1 <- up1(nxt)
            PVD_STAMP(it, 2, 4);
            build_skip(1, hnext(hk, 1), sreg[0]);
            if (more) build_half(nxt, 0, hnext(hk, 2), 0);
            PVD_STAMP(it, 2, 5);
            write_patch(1);
            PVD_STAMP(it, 2, 6);
            PVD_STAMP(it, 2, 7);
            __syncthreads();
            hk = hnext(hk, 1);
            // phase 3: up0(nxt)'s second half; loads skip1(nxt)
            PVD_STAMP(it, 3, 4);
            if (more) build_half(nxt, 0, hnext(hk, 1), 1);
            PVD_STAMP(it, 3, 5);
            PVD_STAMP(it, 3, 6);
            load_skip1(nxt, 1);
            PVD_STAMP(it, 3, 7);
            __syncthreads();
            hk = hnext(hk, 1);
            tile = nxt;
            ++it;
            if (!more) break;
        }
        return;
    }
    // producers.  Prologue: tile 0's inputs, its patches 0 and 1 written,
    // part 0 built
    load_patch(tile, 0, 2);
    load_skip(tile, sreg[0]);
    write_patch(0);
    write_patch(1);
    if (NUP == 4) load_patch(tile, 2, 3);              // (part 3: at this tile's phase 0)
    __syncthreads();
    build_up(tile, 0);
    __syncthreads();
    // one tile: P phases (part j consumed, part j + 1 built), one barrier each
    [[maybe_unused]] int it = 0;                       // (trace builds: the tile iteration)
    auto tile_body = [&](auto SET) {
        constexpr int S = decltype(SET)::value;        // this tile's skip register set
        constexpr int SN = (S + 1) % SS;               // the next tile's
        const int nxt = tile + G;
        const bool more = nxt < a.ntiles;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            PVD_STAMP(it, j, 4);
            const int m = j + 1;                       // the part this phase builds
            if (m < NUP) build_up(tile, m);
            else if (m < P) build_skip(m - NUP, m & 1, sreg[S]);
            else if (more) build_up(nxt, 0);
            PVD_STAMP(it, j, 5);
            // patches two phases ahead of their builds
            if (j + 2 < NUP) write_patch(j + 2);
            else if (j >= P - 2) write_patch(j - (P - 2));
            PVD_STAMP(it, j, 6);
            // global loads last: a wave's instructions issue in order, and a
            // load waiting for room in the memory pipeline would hold the build
            // behind it.  Patch registers, two slots: conv2s the next tile's
            // parts 0-1 at phase 0; conv4s its parts 0-1 at phase 2, its part 2
            // at phase 5 (once this tile's parts are written), this tile's part
            // 3 at phase 0 (used at phase 1)
            if (j == LP) load_patch(nxt, 0, 2);        // (past the last tile: no access)
            if (NUP == 4 && j == P - 1) load_patch(nxt, 2, 3);
            if (NUP == 4 && j == 0) load_patch(tile, 3, 4);
            if (j == LS) load_skip(nxt, sreg[SN]);
            PVD_STAMP(it, j, 7);
            __syncthreads();
        }
        tile = nxt;
        ++it;
        return more;
    };
    if constexpr (SS == 2) {
        while (tile_body(std::integral_constant<int, 0>{}) && tile_body(std::integral_constant<int, 1>{})) {
        }
    } else {
        while (tile_body(std::integral_constant<int, 0>{})) {
        }
    }
}

// ==========================================================================
// layer1's convolutions (RN:21-70 BasicBlock, 64 -> 64 channels, 3x3, stride
// 1, pad 1, at quarter resolution) with their epilogue (folded BN bias, the
// residual, ReLU; k_epilogue's roundings), fp16 channels-last, one pass.  An
// implicit GEMM would read each pixel nine times over for 64 output
// channels; here the decoder kernels' halo structure: persistent blocks of 8
// waves, one per CU; the weights (73.7 KB, [9 taps][8 octets][64][8]) resident
// in LDS for the launch; an 8 x 32 output tile per step, its 10 x 34 x 64
// halo copied into LDS (XOR-swizzled per pixel) from registers loaded during
// the previous tile's convolution; per wave one output row: 36 k-steps x 2
// v_mfma_f32_32x32x16_f16 (64 output channels).
// ==========================================================================
struct L1Args {
    const _Float16 *x, *w, *bias, *res;   // res: [N][H][W][64] or null
    _Float16 *out;
    int N, H, W, tiles_r, tiles_c, ntiles, act;
};

__global__ __launch_bounds__(512) void k_conv64(L1Args a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[72 * 64 * 16 + kDHalo * 16];
    uint8_t *wl = lds;                                  // 73,728 B
    uint8_t *halo = lds + 72 * 64 * 16;                 // 43,520 B
    const int t = (int)threadIdx.x, lane = t & 63, wid = t >> 6;
    const int n = lane & 31, h = lane >> 5;
    for (int i = t; i < 72 * 64; i += 512) *(h8 *)(wl + i * 16) = *(const h8 *)(a.w + i * 8);
    h4 bq[2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int g = 0; g < 4; ++g) bq[m][g] = *(const h4 *)(a.bias + 32 * m + 8 * g + 4 * h);
    auto coords = [&](int tile, int &b, int &y0, int &x0) {
        const int tc = tile % a.tiles_c, rest = tile / a.tiles_c;
        b = rest / a.tiles_r;
        y0 = (rest % a.tiles_r) * kTR;
        x0 = tc * kTC;
    };
    h8 pre[kDSkipIt];
    auto fetch = [&](int tile) {
        int b, y0, x0;
        coords(tile, b, y0, x0);
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.x + (int64_t)b * a.H * a.W * 64), 0, a.H * a.W * 128, 0x00020000);
#pragma unroll
        for (int i = 0; i < kDSkipIt; ++i) {
            const int c = min(t + 512 * i, kDHalo - 1), hp = c >> 3, q = c & 7;
            const int hy = hp / kHC, hx = hp - hy * kHC;
            const int oy = y0 - 1 + hy, ox = x0 - 1 + hx;
            const bool ok = oy >= 0 && oy < a.H && ox >= 0 && ox < a.W;
            const uint32_t off = ok ? (uint32_t)((oy * a.W + ox) * 128 + q * 16) : 0x80000000u;
            pre[i] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
        }
    };
    __builtin_amdgcn_s_waitcnt(0x0F70);
    int tile = xcd_block((int)blockIdx.x, (int)gridDim.x);
    if (tile < a.ntiles) fetch(tile);
    __builtin_amdgcn_s_waitcnt(0x0F70);                // (every tile starts with its halo registers landed)
    for (; tile < a.ntiles; tile += (int)gridDim.x) {
        int b, y0, x0;
        coords(tile, b, y0, x0);
        __syncthreads();                      // the previous tile's halo reads (and the weights) are done
#pragma unroll
        for (int i = 0; i < kDSkipIt; ++i) {
            const int c = t + 512 * i;
            if (c < kDHalo) *(h8 *)(halo + halo_granule(c >> 3, c & 7) * 16) = pre[i];
        }
        __syncthreads();
        if (tile + (int)gridDim.x < a.ntiles) fetch(tile + (int)gridDim.x);
        // this lane's residual, loaded now so its latency hides behind the convolution
        const int oy = y0 + wid, ox = x0 + n;
        const bool pix_ok = oy < a.H && ox < a.W;
        const int64_t po = (((int64_t)b * a.H + (pix_ok ? oy : 0)) * a.W + (pix_ok ? ox : 0)) * 64;
        h4 r[2][4];
        if (a.res) {
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int g = 0; g < 4; ++g) r[m][g] = *(const h4 *)(a.res + po + 32 * m + 8 * g + 4 * h);
        }
        f16x acc[2] = {};
        // k-step s's fragments: the halo pixel's 8 channels (B) and the two
        // 32-cout weight rows (A).  Read PVC_L1_AHEAD steps ahead of their
        // MFMAs: at 2 waves per SIMD a read issued right before its MFMA
        // leaves the LDS latency exposed on every step.
        auto frag = [&](int s, h8 &bf, h8 &a0, h8 &a1) {
            const int o = 2 * s + h;          // octet of this lane half: tap o / 8, channels 8 (o % 8)
            const int tap = o >> 3, q = o & 7;
            const int ky = tap / 3, kx = tap - 3 * ky;
            bf = *(const h8 *)(halo + halo_granule((wid + ky) * kHC + n + kx, q) * 16);
            a0 = *(const h8 *)(wl + ((o * 2 + 0) * 32 + n) * 16);
            a1 = *(const h8 *)(wl + ((o * 2 + 1) * 32 + n) * 16);
        };
        constexpr int AH = PVC_L1_AHEAD;
        h8 fb[AH + 1], f0[AH + 1], f1[AH + 1];
#pragma unroll
        for (int s = 0; s < AH; ++s) frag(s, fb[s], f0[s], f1[s]);
#pragma unroll
        for (int s = 0; s < 36; ++s) {
            if (s + AH < 36) frag(s + AH, fb[(s + AH) % (AH + 1)], f0[(s + AH) % (AH + 1)], f1[(s + AH) % (AH + 1)]);
            const int c = s % (AH + 1);
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f0[c], fb[c], acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f1[c], fb[c], acc[1], 0, 0, 0);
        }
        // the next tile's halo registers and the residual have landed (and the
        // previous tile's stores are out): the stores below stay in flight
        // through the next tile's halo write instead of being waited for there
        __builtin_amdgcn_s_waitcnt(0x0F70);
        // ---- epilogue: acc[m] rows (i & 3) + 8 (i >> 2) + 4 h = couts 32 m + .., column n = pixel ----
        if (pix_ok) {
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    h4 y;
#pragma unroll
                    for (int j = 0; j < 4; ++j) y[j] = (_Float16)((float)(_Float16)acc[m][4 * g + j] + (float)bq[m][g][j]);
                    if (a.res) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) y[j] = (_Float16)((float)y[j] + (float)r[m][g][j]);
                    }
                    if (a.act == 1) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) y[j] = (float)y[j] > 0.f ? y[j] : (_Float16)0.f;
                    }
                    *(h4 *)(a.out + po + 32 * m + 8 * g + 4 * h) = y;
                }
        }
    }
}

int cu_count_dec() {
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

}  // namespace

static int decoder_tail(const void *fm, const void *img, const void *w1, const float *b1, const void *w2,
                        const float *b2, void *out, void *seg, int32_t n, int32_t hin, int32_t win, int32_t cout,
                        float slope, pv_stream_t stream) {
    if (!fm || !img || !w1 || !b1 || !w2 || !b2 || !out || n < 0 || hin < 2 || win < 2) return PV_EINVAL;
    if (cout != 20 && cout != 44) return PV_EINVAL;
    if (!(slope >= 0.f && slope < 1.f)) return PV_EINVAL;          // LeakyReLU as max(y, slope y)
    if (((uintptr_t)fm | (uintptr_t)w1 | (uintptr_t)w2) % 16 || (uintptr_t)img % 4) return PV_EALIGN;
    if (seg ? ((uintptr_t)out | (uintptr_t)seg) % 4 : (uintptr_t)out % 8) return PV_EALIGN;
    if (n == 0) return PV_OK;
    TailArgs a;
    a.seg = (_Float16 *)seg;
    a.fm = (const _Float16 *)fm;
    a.img = (const _Float16 *)img;
    a.w1 = (const _Float16 *)w1;
    a.b1 = b1;
    a.w2 = (const _Float16 *)w2;
    a.b2 = b2;
    a.out = (_Float16 *)out;
    a.N = n; a.Hin = hin; a.Win = win; a.H = 2 * hin; a.W = 2 * win;
    if ((int64_t)n * a.H * a.W * 40 >= (1ll << 31) * 16) return PV_EINVAL;
    // one image's map per buffer descriptor (32-bit byte offsets)
    if ((int64_t)a.H * a.W * 2 * cout >= (1ll << 31) || (int64_t)hin * win * 64 >= (1ll << 31)) return PV_EINVAL;
    a.tiles_r = (a.H + kTR - 1) / kTR;
    a.tiles_c = (a.W + kTC - 1) / kTC;
    const int64_t nt = (int64_t)n * a.tiles_r * a.tiles_c;
    if (nt >= (1ll << 31)) return PV_EINVAL;
    a.ntiles = (int)nt;
    // ATen's area_pixel_compute_scale with align_corners: (in - 1) / (out - 1) in f32
    a.rh = (float)(hin - 1) / (float)(a.H - 1);
    a.rw = (float)(win - 1) / (float)(a.W - 1);
    a.slope = slope;
#ifdef PVT_TRACE
    a.trace = g_tail_trace;
#endif
    hipStream_t s = (hipStream_t)stream;
#if PVT_V1
    const int64_t grid = std::min<int64_t>(nt, (int64_t)PVT_WPE * cu_count_dec());   // persistent: PVT_WPE blocks per CU
    if (cout == 20) k_decoder_tail<20><<<(unsigned)grid, 256, 0, s>>>(a);
    else k_decoder_tail<44><<<(unsigned)grid, 256, 0, s>>>(a);
#else
    const int64_t grid2 = std::min<int64_t>(nt, cu_count_dec());   // persistent: one block per CU
    if (cout == 20) k_decoder_tail2<20><<<(unsigned)grid2, 512, 0, s>>>(a);
    else k_decoder_tail2<44><<<(unsigned)grid2, 512, 0, s>>>(a);
#endif
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}

extern "C" int pv_decoder_tail_f16(const void *fm, const void *img, const void *w1, const float *b1, const void *w2,
                                   const float *b2, void *out, int32_t n, int32_t hin, int32_t win, int32_t cout,
                                   float slope, pv_stream_t stream) {
    return decoder_tail(fm, img, w1, b1, w2, b2, out, nullptr, n, hin, win, cout, slope, stream);
}

extern "C" int pv_decoder_tail_split_f16(const void *fm, const void *img, const void *w1, const float *b1,
                                         const void *w2, const float *b2, void *seg, void *ver, int32_t n, int32_t hin,
                                         int32_t win, int32_t cout, float slope, pv_stream_t stream) {
    if (!seg) return PV_EINVAL;
    return decoder_tail(fm, img, w1, b1, w2, b2, ver, seg, n, hin, win, cout, slope, stream);
}

#ifdef PVT_TRACE
extern "C" void pv_debug_set_tail_trace(void *p) { g_tail_trace = (unsigned long long *)p; }
#endif

namespace {
// The split of the last partial round (k_conv3x3): tiles run whole, parts per
// later tile, and the workspace it needs (counters, then the f32 partials).
struct ConvSplit {
    int nfull, nsplit;
    int64_t tick_bytes, bytes;
};
ConvSplit conv_split(int64_t pixels, int32_t cout, int32_t ksteps) {
    const bool wide = cout % kCT == 0;
    const int64_t ntiles = (pixels + kPT - 1) / kPT * (cout / (wide ? kCT : 128));
    const int cus = cu_count_dec();
    const int64_t rem = ntiles % cus;
    int S = rem > 0 ? (int)std::min<int64_t>(4, cus / rem) : 1;
    while (S > 1 && ksteps / S < 4) --S;          // parts of at least 4 K-steps
    if (S < 2) return ConvSplit{(int)ntiles, 1, 0, 0};
    // the counters' region has one size for every call (4 KiB: up to 1,024
    // split tiles), so that a scratch shared by calls of different shapes
    // never has one call's partials over another's counters
    const int64_t tb = std::max<int64_t>(4096, (rem * 4 + 255) / 256 * 256);
    // one tile's partials: its CT x 256 f32 sums (each of the 64 kNW threads
    // holds CT / kNW 16-byte groups), per part
    const int64_t per = (int64_t)S * (wide ? kCT : 128) * kPT * 4;
    return ConvSplit{(int)(ntiles - rem), S, tb, tb + rem * per};
}
}  // namespace

extern "C" int64_t pv_conv3x3_workspace_bytes(int64_t pixels, int32_t cout, int32_t ksteps) {
    if (pixels <= 0 || cout <= 0 || cout % 128 || ksteps <= 0) return 0;
    return conv_split(pixels, cout, ksteps).bytes;
}

extern "C" int64_t pv_conv3x3_workspace_counter_bytes(int64_t pixels, int32_t cout, int32_t ksteps) {
    if (pixels <= 0 || cout <= 0 || cout % 128 || ksteps <= 0) return 0;
    return conv_split(pixels, cout, ksteps).tick_bytes;
}

extern "C" int pv_conv3x3_ex_f16(const void *x, int32_t hin, int32_t win, int32_t stride, const void *x2,
                                 int32_t mode2, int32_t cin2, int32_t h2, int32_t w2, int32_t s2, const void *w,
                                 const void *bias, const void *res, const void *rbias, void *out, int32_t ldo,
                                 int32_t n, int32_t h, int32_t wd, int32_t cin, int32_t cout, int32_t dil, int32_t act,
                                 float slope, void *ws, int64_t ws_bytes, pv_stream_t stream) {
    if (!x || !w || !bias || !out || n < 0 || h <= 0 || wd <= 0 || dil < 1 || act < 0 || act > 2) return PV_EINVAL;
    if (cin <= 0 || cin % 64 || cout <= 0 || cout % 128 || (rbias && !res && mode2 != PV_CONV_X2_1X1))
        return PV_EINVAL;
    if (stride != 1 && stride != 2) return PV_EINVAL;
    // the output's geometry is the convolution's: padding = dilation, kernel 3
    if (hin <= 0 || win <= 0 || h != (hin - 1) / stride + 1 || wd != (win - 1) / stride + 1) return PV_EINVAL;
    if (mode2 != PV_CONV_X2_NONE && mode2 != PV_CONV_X2_CAT && mode2 != PV_CONV_X2_1X1) return PV_EINVAL;
    if (mode2 != PV_CONV_X2_NONE && (!x2 || cin2 <= 0 || cin2 % 64 || ((uintptr_t)x2 % 16))) return PV_EINVAL;
    if (mode2 == PV_CONV_X2_1X1 && (s2 < 1 || h2 <= 0 || w2 <= 0 || (int64_t)(h - 1) * s2 >= h2 ||
                                    (int64_t)(wd - 1) * s2 >= w2 || res))
        return PV_EINVAL;
    if (ldo == 0) ldo = cout;
    if (ldo < cout || ldo % 4) return PV_EINVAL;
    if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)out | (uintptr_t)res) % 16 || ((uintptr_t)bias | (uintptr_t)rbias) % 8)
        return PV_EALIGN;
    if (out == x || (res && out == res) || (x2 && out == x2)) return PV_EINVAL;
    if (n == 0) return PV_OK;
    ConvArgs a;
    a.x = (const _Float16 *)x; a.w = (const _Float16 *)w; a.bias = (const _Float16 *)bias;
    a.x2 = mode2 != PV_CONV_X2_NONE ? (const _Float16 *)x2 : (const _Float16 *)x;
    a.res = (const _Float16 *)res; a.rbias = (const _Float16 *)rbias; a.out = (_Float16 *)out;
    a.N = n; a.H = h; a.W = wd; a.Cin = cin; a.Cout = cout; a.ldo = ldo; a.dil = dil; a.act = act; a.slope = slope;
    a.Hin = hin; a.Win = win; a.stride = stride;
    a.mode2 = mode2; a.Cin2 = mode2 != PV_CONV_X2_NONE ? cin2 : 0; a.H2 = h2; a.W2 = w2; a.s2 = s2;
    a.M = (int64_t)n * h * wd;
    a.cb1 = cin / 64;
    a.cblocks = (cin + (mode2 == PV_CONV_X2_CAT ? cin2 : 0)) / 64;
    a.nmain = 9 * a.cblocks;
    a.ksteps = a.nmain + (mode2 == PV_CONV_X2_1X1 ? cin2 / 64 : 0);
    // 32-bit buffer offsets (+ the 0x80000000 out-of-range marker): the maps under 2 GiB
    const int64_t in1 = (int64_t)n * hin * win * cin * 2;
    const int64_t in2 = mode2 == PV_CONV_X2_1X1 ? (int64_t)n * h2 * w2 * cin2 * 2
                        : mode2 == PV_CONV_X2_CAT ? (int64_t)n * hin * win * cin2 * 2 : 0;
    if (in1 >= (1ll << 31) || in2 >= (1ll << 31) || (int64_t)cout * a.ksteps * 128 >= (1ll << 31) ||
        a.M * ldo >= (1ll << 31))
        return PV_EINVAL;
    a.ntp = (int)((a.M + kPT - 1) / kPT);
    const bool wide = cout % kCT == 0;       // 256-cout tiles, else 128
    a.nct = cout / (wide ? kCT : 128);
    a.ntiles = a.ntp * a.nct;
    a.nfull = a.ntiles;
    a.nsplit = 1;
    a.slab = nullptr;
    a.tick = nullptr;
    if (ws) {
        if ((uintptr_t)ws % 256) return PV_EALIGN;
        const ConvSplit sp = conv_split(a.M, cout, a.ksteps);
        if (sp.nsplit > 1 && ws_bytes >= sp.bytes) {
            a.nfull = sp.nfull;
            a.nsplit = sp.nsplit;
            // the counters start zeroed (the caller's zero-filled ws) and every
            // split tile's last part returns its counter to zero: no memset node
            a.tick = (int *)ws;
            a.slab = (u4 *)((uint8_t *)ws + sp.tick_bytes);
        }
    }
    const unsigned grid = (unsigned)(a.nfull + (a.ntiles - a.nfull) * a.nsplit);
#if PVC_WINDOW
    if (stride == 1 && dil <= kMaxDil) {
        if (wide) k_conv3x3w<kCT><<<grid, 64 * kNW, 0, (hipStream_t)stream>>>(a);
        else k_conv3x3w<128><<<grid, 64 * kNW, 0, (hipStream_t)stream>>>(a);
    } else
#endif
    {
#if PVC_RING4
        if (wide) k_conv3x3r<kCT><<<grid, 64 * kNW, 0, (hipStream_t)stream>>>(a);
        else k_conv3x3r<128><<<grid, 64 * kNW, 0, (hipStream_t)stream>>>(a);
#else
        if (wide) k_conv3x3<kCT><<<grid, 64 * kNW, 0, (hipStream_t)stream>>>(a);
        else k_conv3x3<128><<<grid, 64 * kNW, 0, (hipStream_t)stream>>>(a);
#endif
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}

extern "C" int pv_conv3x3_f16(const void *x, const void *w, const void *bias, const void *res, const void *rbias,
                              void *out, int32_t ldo, int32_t n, int32_t h, int32_t wd, int32_t cin, int32_t cout,
                              int32_t dil, int32_t act, float slope, pv_stream_t stream) {
    if (rbias && !res) return PV_EINVAL;
    return pv_conv3x3_ex_f16(x, h, wd, 1, nullptr, PV_CONV_X2_NONE, 0, 0, 0, 0, w, bias, res, rbias, out, ldo, n, h,
                             wd, cin, cout, dil, act, slope, nullptr, 0, stream);
}

extern "C" int pv_decoder_conv2s_f16(const void *fm, const void *skip, const void *w, const void *bias, void *out,
                                     int32_t n, int32_t hin, int32_t win, float slope, pv_stream_t stream) {
    if (!fm || !skip || !w || !bias || !out || n < 0 || hin < 2 || win < 2) return PV_EINVAL;
    if (!(slope >= 0.f && slope < 1.f)) return PV_EINVAL;
    if (((uintptr_t)fm | (uintptr_t)skip | (uintptr_t)w | (uintptr_t)out) % 16 || (uintptr_t)bias % 8)
        return PV_EALIGN;
    if (n == 0) return PV_OK;
    DecConvArgs a;
    a.fm = (const _Float16 *)fm; a.skip = (const _Float16 *)skip; a.w = (const _Float16 *)w;
    a.bias = (const _Float16 *)bias; a.out = (_Float16 *)out;
    a.N = n; a.Hin = hin; a.Win = win; a.H = 2 * hin; a.W = 2 * win;
    if ((int64_t)a.H * a.W * kDC2 * 2 >= (1ll << 31) || (int64_t)hin * win * kDC1 * 2 >= (1ll << 31)) return PV_EINVAL;
    a.tiles_r = (a.H + kTR - 1) / kTR;
    a.tiles_c = (a.W + kTC - 1) / kTC;
    const int64_t nt = (int64_t)n * a.tiles_r * a.tiles_c;
    if (nt >= (1ll << 31)) return PV_EINVAL;
    a.ntiles = (int)nt;
    a.rh = (float)(hin - 1) / (float)(a.H - 1);
    a.rw = (float)(win - 1) / (float)(a.W - 1);
    a.slope = slope;
    const int64_t grid = std::min<int64_t>(nt, cu_count_dec());   // persistent: one block per CU
#if PVC_DEC_V1
    k_dec_conv2s<<<(unsigned)grid, 512, 0, (hipStream_t)stream>>>(a);
#else
    k_dec_conv<32, 2><<<(unsigned)grid, kDecThreads, 0, (hipStream_t)stream>>>(a);
#endif
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}

#ifdef PVC_CLOCK_TRACE
extern "C" int pv_debug_set_conv_clk(void *p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_conv_clk), &p, sizeof(p));
}
#endif
#ifdef PVC_DEC_TRACE
extern "C" int pv_debug_set_dec_trace(void *p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_dec_trace), &p, sizeof(p));
}
#endif

extern "C" int pv_decoder_conv4s_f16(const void *fm, const void *skip, const void *w, const void *bias, void *out,
                                     int32_t n, int32_t hin, int32_t win, float slope, pv_stream_t stream) {
    if (!fm || !skip || !w || !bias || !out || n < 0 || hin < 2 || win < 2) return PV_EINVAL;
    if (!(slope >= 0.f && slope < 1.f)) return PV_EINVAL;
    if (((uintptr_t)fm | (uintptr_t)skip | (uintptr_t)w | (uintptr_t)out) % 16 || (uintptr_t)bias % 8)
        return PV_EALIGN;
    if (n == 0) return PV_OK;
    DecConvArgs a;
    a.fm = (const _Float16 *)fm; a.skip = (const _Float16 *)skip; a.w = (const _Float16 *)w;
    a.bias = (const _Float16 *)bias; a.out = (_Float16 *)out;
    a.N = n; a.Hin = hin; a.Win = win; a.H = 2 * hin; a.W = 2 * win;
    if ((int64_t)a.H * a.W * kECo * 2 >= (1ll << 31) || (int64_t)hin * win * kEC1 * 2 >= (1ll << 31)) return PV_EINVAL;
    a.tiles_r = (a.H + kTR - 1) / kTR;
    a.tiles_c = (a.W + kTC - 1) / kTC;
    const int64_t nt = (int64_t)n * a.tiles_r * a.tiles_c;
    if (nt >= (1ll << 31)) return PV_EINVAL;
    a.ntiles = (int)nt;
    a.rh = (float)(hin - 1) / (float)(a.H - 1);
    a.rw = (float)(win - 1) / (float)(a.W - 1);
    a.slope = slope;
    const int64_t grid = std::min<int64_t>(nt, cu_count_dec());   // persistent: one block per CU
#if PVC_DEC_V1
    k_dec_conv4s<<<(unsigned)grid, 512, 0, (hipStream_t)stream>>>(a);
#else
    k_dec_conv<64, 4><<<(unsigned)grid, kDecThreads, 0, (hipStream_t)stream>>>(a);
#endif
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}


// ==========================================================================
// The stem (RN:139-142, 201-204): conv1 7x7 / 2 / pad 3, 3 -> 64 channels,
// BN folded, ReLU -> x2s, and maxpool 3x3 / 2 / pad 1 of x2s, on the matrix
// cores, in one pass.  A stride-2 7x7 convolution is a stride-1 4x4 one over
// the image folded 2 x 2 into its channels (space-to-depth): s2d pixel (Y, X)
// holds image pixels (2Y + dy, 2X + dx) as channels dy*6 + dx*3 + c (12,
// padded to 16), and
//     x2s(y, x) = relu(b + sum_{ty,tx} W2[ty][tx] . s2d(y - 2 + ty, x - 2 + tx)),
//     W2[ty][tx][dy*6 + dx*3 + c] = W[c][2ty + dy - 1][2tx + dx - 1]
// (zero outside 0..6).  One tap = 16 channels = one v_mfma_f32_32x32x16_f16
// per 32 output channels: 32 per wave and tile.  In the image's channels-last
// fp16 layout the 6 channels of an s2d pixel's row dy are 12 contiguous bytes,
// so a pixel is two 12-byte loads.
// Tiles: 8 x2s rows (wave = row) x 32 computed columns x0 - 1 .. x0 + 30, of
// which 30 are the tile's own (x0 = 30 tc): pool columns 15 tc .. 15 tc + 14
// need x2s columns x0 - 1 .. x0 + 29, so the left neighbour column is
// computed again (and the 32nd is computed unused) -- 7 % more matrix work
// than 32-column tiles, for no halo exchange between tiles of a row.  Pool
// rows 4 tr .. 4 tr + 3 need x2s rows y0 - 1 .. y0 + 7: row y0 - 1 is the
// previous tile's last row, kept in LDS (two output buffers, alternating),
// so tiles run top to bottom through a column strip: tile index = (image,
// strip, row tile), row tile fastest, and a block takes a contiguous range
// (when its range starts below a strip's top it first computes the tile
// above, keeping only that row).  The pool's padding is 0, not -inf: x2s is a
// ReLU output (>= 0, never NaN) and every window holds a valid pixel, so the
// max is the same.  An 8 x 32 tile reads an 11 x 35 s2d halo (12.3 KB in
// LDS, double buffered; its two 16-byte granules per pixel swapped on odd
// 8-pixel groups: conflict-free); halo pixels are loaded into registers two
// tiles ahead; the weights (32 KB) stay in registers for the launch.
// Epilogue: fp16 round, + b, ReLU (as k_relu_pool), through LDS to 16-byte
// x2s stores.  A tile's pool runs one tile later, between the next tile's
// barrier and its MFMAs (one 8-channel output per thread, its 9 LDS reads in
// flight together, v_pk_max_u16 on the bits), to 16-byte stores: no barrier
// of its own.  pool NULL: x2s only.  (tools/stem_probe.py, configs[2]'s
// shape, one box, two rounds: conv + separate pool pass 228-232 us, this
// kernel 137-140 us; with a barrier before the pool 143 us, with the pool's
// reads one at a time 146-150 us, its 32-column form without the pool 108 us.)
// ==========================================================================
#ifndef PVC_STEM_ZH
#define PVC_STEM_ZH 1
#endif
#ifndef PVC_STEM_POOLPOS
#define PVC_STEM_POOLPOS 0  // where a tile's step runs the previous tile's pool: 0 before its MFMAs, 1 at its end (2: none, timing only)
#endif
constexpr int kSR = 8, kSC = 32;                      // tile: 8 rows x 32 computed columns
#ifndef PVC_STEM_NEW
#define PVC_STEM_NEW 30     // (32: a timing diagnostic only -- the pool and the last column are then wrong)
#endif
constexpr int kSNew = PVC_STEM_NEW;                   // ... of which the tile's own (pool-aligned)
constexpr int kSHR = kSR + 3, kSHC = kSC + 3;         // s2d halo: 11 x 35
constexpr int kSHalo = kSHR * kSHC;                   // 385 pixels
constexpr int kSCo = 64;
typedef unsigned int u3 __attribute__((ext_vector_type(3)));

struct StemArgs {
    const _Float16 *img;    // [N][H][W][3]
    const _Float16 *w;      // [2 cout halves][16 taps][2 k halves][32 couts][8]: the lanes' A fragments
    const _Float16 *bias;   // [64]
    _Float16 *out;          // [N][H/2][W/2][64]
    _Float16 *pool;         // [N][Hp][Wp][64] or NULL
    int N, H, W, Ho, Wo, Hp, Wp, tiles_r, tiles_c, ntiles;
};

__device__ __forceinline__ int stem_slot(int hp, int g) { return hp * 2 + (g ^ ((hp >> 3) & 1)); }

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_stem(StemArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t halo2[2][kSHalo * 32];
    __shared__ __attribute__((aligned(16))) uint8_t obuf[2][kSR][kSC * kSCo * 2];   // two tiles' 8 x 32 x 64 outputs
    __shared__ __attribute__((aligned(16))) uint8_t carry[3][kSC * kSCo * 2];        // three tiles' last rows
    __shared__ __attribute__((aligned(16))) uint8_t zchunk[16];                       // zeros: the pool's padding
    const int t = (int)threadIdx.x, lane = t & 63, wid = t >> 6;
    const int n = lane & 31, h = lane >> 5;
    // this block's tiles: a contiguous range of (image, strip, row tile)
    const int G = (int)gridDim.x, per = a.ntiles / G, rem = a.ntiles % G, bi = (int)blockIdx.x;
    const int t0 = bi * per + min(bi, rem), t1 = t0 + per + (bi < rem ? 1 : 0);
    if (t0 >= t1) return;
    h8 wf[2][16];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int tap = 0; tap < 16; ++tap) wf[m][tap] = *(const h8 *)(a.w + (((m * 16 + tap) * 2 + h) * 32 + n) * 8);
    // the bias in LDS, read by the epilogue (registers are full: weights, halo
    // addresses, two prefetch sets)
    __shared__ _Float16 sbias[kSCo];
    if (t < kSCo) sbias[t] = a.bias[t];
    if (t < 4) ((uint32_t *)zchunk)[t] = 0u;
    __builtin_amdgcn_s_waitcnt(0x0F70);     // vmcnt(0): no weight waits inside the tile loop
    auto coords = [&](int tile, int &b, int &tr, int &y0, int &x0) {
#ifdef PVC_STEM_DIAG_ORDER   // timing diagnostic only (the pool is wrong): blocks' k-th tiles side by side
        if (tile < per * G) tile = (tile % per) * G + tile / per;
#endif
        tr = tile % a.tiles_r;
        const int rest = tile / a.tiles_r;
        b = rest / a.tiles_c;
        y0 = tr * kSR;
        x0 = (rest % a.tiles_c) * kSNew;
    };
    // this thread's halo pixel (t < 385): rows 2Y and 2Y + 1, 12 bytes each;
    // two tiles ahead (a tile's MFMAs are shorter than a load's latency), in
    // two register sets A and B that alternate
    const int hy = t / kSHC, hx = t - hy * kSHC;
    u3 a0 = {}, a1 = {}, b0 = {}, b1 = {};
    // (issued for every tile, past the last as well -- with no access -- so the
    // count of loads in flight is the same on every path)
    auto fetch = [&](int tile, u3 &r0, u3 &r1) {
        int b, tr, y0, x0;
        coords(min(tile, t1 - 1), b, tr, y0, x0);
        const __amdgpu_buffer_rsrc_t ir = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.img + (int64_t)b * a.H * a.W * 3), 0, a.H * a.W * 6, 0x00020000);
        // computed column c of the tile is x2s column x0 - 1 + c: s2d columns x0 - 3 + hx
        const int Y = y0 - 2 + hy, X = x0 - 3 + hx;
        const bool ok = tile < t1 && t < kSHalo && Y >= 0 && 2 * Y < a.H && X >= 0 && 2 * X < a.W;
        const uint32_t off = ok ? (uint32_t)((2 * Y * a.W + 2 * X) * 6) : 0x80000000u;
        const uint32_t off1 = ok ? off + (uint32_t)(a.W * 6) : 0x80000000u;
        r0 = __builtin_bit_cast(u3, __builtin_amdgcn_raw_buffer_load_b96(ir, off, 0, 0));
        r1 = __builtin_bit_cast(u3, __builtin_amdgcn_raw_buffer_load_b96(ir, off1, 0, 0));
    };
    auto put = [&](uint8_t *halo, const u3 &r0, const u3 &r1) {
        if (t < kSHalo) {
            *(u4 *)(halo + stem_slot(t, 0) * 16) = u4{r0.x, r0.y, r0.z, r1.x};
            *(u4 *)(halo + stem_slot(t, 1) * 16) = u4{r1.y, r1.z, 0u, 0u};
        }
    };
    const __amdgpu_buffer_rsrc_t prr = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a.pool, 0, a.pool ? 0x7fffffff : 0, 0x00020000);
    // pool of tile `pt` (a tile of the range), run one tile behind, between the
    // next tile's barrier and its MFMAs: its rows are `rows` (that tile's
    // buffer, complete since the barrier), the row above is carry[(pt - 1) % 3]
    // (the copy wave 7 made of the tile above's last row; three copies, so the
    // one read here is not the one being written).  Output (py, px), channels
    // 8q .. 8q + 7 = max over x2s rows 2py - 1 .. 2py + 1 = this tile's rows
    // 2j - 1 .. 2j + 1, computed columns 2i .. 2i + 2; waves 2j and 2j + 1 take
    // pool row j, their lanes the 120 (i, q).  Past the range (pt < t0 or
    // pt >= t1) the store is dropped.
    auto pool_tile = [&](int pt, uint8_t (*rows)[kSC * kSCo * 2], const uint8_t *above) {
        int b, tr, y0, x0;
        coords(max(pt, 0), b, tr, y0, x0);
        // (the lane index through an opaque copy: everything below is made
        // here, not hoisted out of the tile loop -- the registers are full)
        int ol;
        asm volatile("v_mov_b32 %0, %1" : "=v"(ol) : "v"(lane));
        const int j = wid >> 1, e = (wid & 1) * 64 + ol, i = e >> 3, q = e & 7;
        const int py = (y0 >> 1) + j, px = (x0 >> 1) + i;
        // x2s is >= +0 and never NaN: its fp16 bit patterns order as unsigned
        // integers, so the max is v_pk_max_u16 on the bits
        typedef unsigned short us8 __attribute__((ext_vector_type(8)));
        // all nine reads in flight together (no branches: a window pixel
        // outside the map reads the zero chunk instead), then the maxima.
        // (Measured: the same work on waves 4-7 only, two outputs per lane, so
        // that waves 0-3 start their MFMAs at once: 142-146 against 137-140 us.)
        us8 v[9];
#pragma unroll
        for (int dr = 0; dr < 3; ++dr) {
            const int lr = 2 * j + dr - 1, yy = y0 + lr;
            const bool rok = yy >= 0 && yy < a.Ho;
            const uint8_t *row = lr < 0 ? above : rows[lr < 0 ? 0 : lr];
#pragma unroll
            for (int dc = 0; dc < 3; ++dc) {
                const int c = 2 * i + dc, xx = x0 - 1 + c;
                const bool ok = rok && xx >= 0 && xx < a.Wo && e < (kSNew / 2) * 8;
                v[dr * 3 + dc] = *(const us8 *)(ok ? row + (c * 128 + ((q ^ (c & 7)) * 16)) : zchunk);
            }
        }
        us8 mx = v[0];
#pragma unroll
        for (int k = 1; k < 9; ++k) mx = __builtin_elementwise_max(mx, v[k]);
        const bool own = pt >= t0 && pt < t1 && e < (kSNew / 2) * 8 && py < a.Hp && px < a.Wp;
        const uint32_t po = own ? ((uint32_t)((b * a.Hp + py) * a.Wp + px) * kSCo) * 2u + (uint32_t)q * 16u
                                : 0x80000000u;   // (< 2^31: checked at launch)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, mx), prr, po, 0, 0);
    };
    // Tile i: the barrier (tile i - 1's rows complete, this halo written), tile
    // i + 2's loads, tile i - 1's pool, tile i's MFMAs, tile i + 1's halo into
    // the other buffer (its loads issued a tile earlier), tile i's outputs
    // through LDS to 16-byte x2s stores (wave 7 also keeps a copy of its row
    // for tile i + 1's pool).  `keep`: the tile above the range, computed for
    // its last row only (no stores).
    auto step = [&](int tile, const uint8_t *halo, uint8_t *next, u3 &f0, u3 &f1, const u3 &p0, const u3 &p1,
                    uint8_t (*cur)[kSC * kSCo * 2], uint8_t (*prev)[kSC * kSCo * 2]) {
        int b, tr, y0, x0;
        coords(tile, b, tr, y0, x0);
        const bool keep = tile < t0;
        __syncthreads();                      // this halo written; the reads of the other done
        fetch(tile + 2, f0, f1);
#if PVC_STEM_POOLPOS == 0
        pool_tile(tile - 1, prev, carry[(tile + 1) % 3]);   // ((tile - 2) mod 3)
#endif
        f16x acc0 = {}, acc1 = {};
        // (the halo base through an opaque zero: the 16 per-tap offsets are then
        // shared by both halo buffers instead of hoisted once for each)
#if PVC_STEM_ZH
        int zh;
        asm volatile("v_mov_b32 %0, 0" : "=v"(zh));
        const uint8_t *hb = halo + zh;
#else
        const uint8_t *hb = halo;
#endif
#pragma unroll
        for (int tap = 0; tap < 16; ++tap) {
            const int ty = tap >> 2, tx = tap & 3;
            const h8 bf = *(const h8 *)(hb + stem_slot((wid + ty) * kSHC + n + tx, h) * 16);
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[0][tap], bf, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wf[1][tap], bf, acc1, 0, 0, 0);
        }
        if (tile + 1 < t1) put(next, p0, p1);
        // rows (i & 3) + 8 (i >> 2) + 4 h of acc = channels, column n = pixel:
        // 8-byte pieces into the wave's LDS row (16-byte chunk c of pixel n at
        // c ^ (n & 7): conflict-free both ways), read back as 16 bytes per lane
        uint8_t *ob = cur[wid];
        uint8_t *cb = carry[tile % 3];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                h4 y;
                const h4 bq = *(const h4 *)(sbias + 32 * m + 8 * g + 4 * h);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const _Float16 v = (_Float16)((float)(_Float16)(m ? acc1 : acc0)[4 * g + j] + (float)bq[j]);
                    y[j] = (float)v > 0.f ? v : (_Float16)0.f;
                }
                const int off = n * 128 + (((4 * m + g) ^ (n & 7)) * 16) + 8 * h;
                *(h4 *)(ob + off) = y;
                if (wid == kSR - 1) *(h4 *)(cb + off) = y;
            }
        __builtin_amdgcn_wave_barrier();
        const int oy = y0 + wid;
        const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.out + (int64_t)b * a.Ho * a.Wo * kSCo), 0, a.Ho * a.Wo * kSCo * 2, 0x00020000);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int p = 8 * r + (lane >> 3), q = lane & 7, ox = x0 - 1 + p;   // computed column p
            const u4 v = *(const u4 *)(ob + p * 128 + ((q ^ (p & 7)) * 16));
            const bool own = !keep && p >= 1 && p <= kSNew && oy < a.Ho && ox < a.Wo;
            const uint32_t po = own ? (uint32_t)(((oy * a.Wo + ox) * kSCo) * 2 + q * 16) : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b128(v, orr, po, 0, 0);
        }
#if PVC_STEM_POOLPOS == 1
        pool_tile(tile - 1, prev, carry[(tile + 1) % 3]);   // ((tile - 2) mod 3)
#endif
    };
    // the tile above the range's first, when that is not a strip's top: its last
    // row is the first pool rows' row y0 - 1
    const int first = (t0 % a.tiles_r) > 0 ? t0 - 1 : t0;
    fetch(first, a0, a1);
    fetch(first + 1, b0, b1);
    {   // five dropped stores (out-of-range offset), as a step ends with: the
        // loop is entered with the same memory operations in flight as it
        // repeats with, so the compiler's wait before the first put() is for
        // that tile's loads only, not for the last stores as well
        const __amdgpu_buffer_rsrc_t orr = __builtin_amdgcn_make_buffer_rsrc((void *)a.out, 0, 0, 0x00020000);
#pragma unroll
        for (int r = 0; r < 5; ++r) __builtin_amdgcn_raw_buffer_store_b128(u4{0u, 0u, 0u, 0u}, orr, 0x80000000u + 16u * r, 0, 0);
    }
    put(halo2[0], a0, a1);
    int tile = first;
    while (true) {
        step(tile, halo2[0], halo2[1], a0, a1, b0, b1, obuf[0], obuf[1]);
        if (++tile >= t1) break;
        step(tile, halo2[1], halo2[0], b0, b1, a0, a1, obuf[1], obuf[0]);
        if (++tile >= t1) break;
    }
    // the last tile's pool: its rows are in obuf[(t1 - 1 - first) & 1]
    __syncthreads();
    pool_tile(t1 - 1, obuf[(t1 - 1 - first) & 1], carry[(t1 - 2 + 3) % 3]);
}

static int stem_launch(const void *img, const void *w, const void *bias, void *out, void *pool, int32_t n, int32_t h,
                       int32_t wd, pv_stream_t stream) {
    if (!img || !w || !bias || !out || n < 0 || h < 2 || wd < 2 || h % 2 || wd % 2) return PV_EINVAL;
    if (((uintptr_t)w | (uintptr_t)out | (uintptr_t)pool) % 16 || (uintptr_t)bias % 8 || (uintptr_t)img % 4)
        return PV_EALIGN;
    if (out == pool) return PV_EINVAL;
    if (n == 0) return PV_OK;
    if ((int64_t)h * wd * 6 >= (1ll << 31) || (int64_t)h * wd * kSCo / 2 >= (1ll << 31)) return PV_EINVAL;
    StemArgs a;
    a.img = (const _Float16 *)img; a.w = (const _Float16 *)w; a.bias = (const _Float16 *)bias;
    a.out = (_Float16 *)out; a.pool = (_Float16 *)pool;
    a.N = n; a.H = h; a.W = wd; a.Ho = h / 2; a.Wo = wd / 2;
    a.Hp = (a.Ho - 1) / 2 + 1; a.Wp = (a.Wo - 1) / 2 + 1;
    if (pool && (int64_t)n * a.Hp * a.Wp * kSCo * 2 >= (1ll << 31)) return PV_EINVAL;
    a.tiles_r = (a.Ho + kSR - 1) / kSR;
    a.tiles_c = (a.Wo + kSNew - 1) / kSNew;
    const int64_t nt = (int64_t)n * a.tiles_r * a.tiles_c;
    if (nt >= (1ll << 31)) return PV_EINVAL;
    a.ntiles = (int)nt;
    const int64_t grid = std::min<int64_t>(nt, cu_count_dec());   // persistent: one block per CU
    k_stem<<<(unsigned)grid, 512, 0, (hipStream_t)stream>>>(a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}

extern "C" int pv_stem_conv_f16(const void *img, const void *w, const void *bias, void *out, int32_t n, int32_t h,
                                int32_t wd, pv_stream_t stream) {
    return stem_launch(img, w, bias, out, nullptr, n, h, wd, stream);
}

extern "C" int pv_stem_pool_f16(const void *img, const void *w, const void *bias, void *x2s, void *pool, int32_t n,
                                int32_t h, int32_t wd, pv_stream_t stream) {
    if (!pool) return PV_EINVAL;
    return stem_launch(img, w, bias, x2s, pool, n, h, wd, stream);
}

extern "C" int pv_conv64_f16(const void *x, const void *w, const void *bias, const void *res, void *out, int32_t n,
                             int32_t h, int32_t wd, int32_t act, pv_stream_t stream) {
    if (!x || !w || !bias || !out || n < 0 || h <= 0 || wd <= 0 || act < 0 || act > 1) return PV_EINVAL;
    if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)out | (uintptr_t)res) % 16 || (uintptr_t)bias % 8) return PV_EALIGN;
    if (out == x || (res && out == res)) return PV_EINVAL;
    if (n == 0) return PV_OK;
    if ((int64_t)h * wd * 128 >= (1ll << 31)) return PV_EINVAL;
    L1Args a;
    a.x = (const _Float16 *)x; a.w = (const _Float16 *)w; a.bias = (const _Float16 *)bias;
    a.res = (const _Float16 *)res; a.out = (_Float16 *)out;
    a.N = n; a.H = h; a.W = wd; a.act = act;
    a.tiles_r = (h + kTR - 1) / kTR;
    a.tiles_c = (wd + kTC - 1) / kTC;
    const int64_t nt = (int64_t)n * a.tiles_r * a.tiles_c;
    if (nt >= (1ll << 31)) return PV_EINVAL;
    a.ntiles = (int)nt;
    const int64_t grid = std::min<int64_t>(nt, cu_count_dec());   // persistent: one block per CU
    k_conv64<<<(unsigned)grid, 512, 0, (hipStream_t)stream>>>(a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}
