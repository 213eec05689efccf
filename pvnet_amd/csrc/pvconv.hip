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
// LDS -- the x2 bilinear blend separably, column blends once per (fm row,
// halo column), then row blends, in packed fp16 -- and each wave computes two
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

#include "../../include/pvvote.h"

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
constexpr int kTcolTasks = kPR * kHC * 4;         // column blends: (fm row, halo column, 8 channels)

struct TailArgs {
    const _Float16 *fm;    // [N][Hin][Win][32]
    const _Float16 *img;   // [N][H][W][3]
    const _Float16 *w1;    // [32][368]: k = tap * 40 + channel (tap = 3 ky + kx)
    const float *b1;       // [32]
    const _Float16 *w2;    // [MT][2][32][16]: the 1x1 weights in the accumulator's row order (host-permuted)
    const float *b2;       // [cout]
    _Float16 *out;         // [N][H][W][cout]
    int N, Hin, Win, H, W, tiles_r, tiles_c, ntiles;
    float rh, rw, slope;
};

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

// global loads of a tile's fm patch and image rows into registers, branch-free:
// addresses are clamped into the maps (the halo build never reads a patch
// pixel outside fm, and writes zeros itself for halo pixels outside the
// image), so nothing waits on the loads until the next tile's halo build.
// pk / ik: the thread's tile-independent chunk coordinates (hoisted).
__device__ __forceinline__ void fetch(const TailArgs &a, int tile, const int (&pk)[kPatchIt],
                                      const int (&ik)[kImgIt], h8 (&pre)[kPatchIt], uint32_t (&pimg)[kImgIt]) {
    int b, y0, x0, ly0, lx0;
    tile_coords(a, tile, b, y0, x0, ly0, lx0);
    const _Float16 *fmb = a.fm + (int64_t)b * a.Hin * a.Win * 32;
#pragma unroll
    for (int i = 0; i < kPatchIt; ++i) {
        const int row = min(ly0 + (pk[i] >> 16), a.Hin - 1), col = min(lx0 + ((pk[i] >> 8) & 255), a.Win - 1);
        pre[i] = *(const h8 *)(fmb + (row * a.Win + col) * 32 + 8 * (pk[i] & 3));
    }
    const uint32_t *imb = (const uint32_t *)(a.img + (int64_t)b * a.H * a.W * 3);
    const int rowdw = a.W * 3 / 2;                 // dwords per image row (W even)
#pragma unroll
    for (int i = 0; i < kImgIt; ++i) {
        const int oy = min(max(y0 - 1 + (ik[i] >> 8), 0), a.H - 1);
        const int j = min(max(x0 * 3 / 2 - 2 + (ik[i] & 255), 0), rowdw - 1);
        pimg[i] = imb[oy * rowdw + j];
    }
}

template <int COUT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_decoder_tail(TailArgs a) {
    constexpr int MT = (COUT + 31) / 32;
    __shared__ alignas(16) _Float16 halo[kHaloPx * kCP];
    __shared__ alignas(16) _Float16 patch[kPatchChunks * 8];
    __shared__ alignas(16) _Float16 tcol[kTcolTasks * 8];
    __shared__ alignas(16) uint32_t imgs[kImgWords];
    __shared__ alignas(16) _Float16 bias[32 + 32 * MT];
    const int lane = (int)(threadIdx.x & 63), wid = (int)(threadIdx.x >> 6);
    const int n = lane & 31, h = lane >> 5;
    // the wave's A fragments for the whole launch: lane (out r = n, half h)
    // holds w1[r][16 s + 8 h .. + 8] for k-step s
    h8 wa[kKS];
#pragma unroll
    for (int s = 0; s < kKS; ++s) wa[s] = *(const h8 *)(a.w1 + n * kK + 16 * s + 8 * h);
    h8 wb[MT][2];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) wb[t][s2] = *(const h8 *)(a.w2 + ((t * 2 + s2) * 32 + n) * 16 + 8 * h);
    // the weights are in registers before the tile loop (vmcnt 0): the loop's
    // only outstanding loads are then the next tile's prefetch, which nothing
    // waits for until the next iteration
    __builtin_amdgcn_s_waitcnt(0x0F70);
    // the biases, fp16: conv rows [0, 32), head outputs [32, 32 + 32 MT)
    for (int i = (int)threadIdx.x; i < 32 + 32 * MT; i += 256)
        bias[i] = i < 32 ? (_Float16)a.b1[i] : (i - 32 < COUT ? (_Float16)a.b2[i - 32] : (_Float16)0.f);
    int pk[kPatchIt], ik[kImgIt];
#pragma unroll
    for (int i = 0; i < kPatchIt; ++i) {
        const int c = min((int)threadIdx.x + 256 * i, kPatchChunks - 1);
        const int pp = c >> 2, pr = pp / kPC;
        pk[i] = (pr << 16) | ((pp - pr * kPC) << 8) | (c & 3);
    }
#pragma unroll
    for (int i = 0; i < kImgIt; ++i) {
        const int w = min((int)threadIdx.x + 256 * i, kImgWords - 1);
        const int r = w / kImgDw;
        ik[i] = (r << 8) | (w - r * kImgDw);
    }
    // next tile's inputs, fetched during this tile's convolution
    h8 pre[kPatchIt];
    uint32_t pimg[kImgIt];
    int tile = (int)blockIdx.x;
    if (tile < a.ntiles) fetch(a, tile, pk, ik, pre, pimg);
    for (; tile < a.ntiles; tile += (int)gridDim.x) {
        int b, y0, x0, ly0, lx0;
        tile_coords(a, tile, b, y0, x0, ly0, lx0);
        __syncthreads();   // the previous tile's halo reads are done
#pragma unroll
        for (int i = 0; i < kPatchIt; ++i) {
            const int c = (int)threadIdx.x + 256 * i;
            if (c < kPatchChunks) *(h8 *)(patch + 8 * c) = pre[i];
        }
#pragma unroll
        for (int i = 0; i < kImgIt; ++i) {
            const int w = (int)threadIdx.x + 256 * i;
            if (w < kImgWords) imgs[w] = pimg[i];
        }
        __syncthreads();
        // ---- halo: pixel (y0 - 1 + hy, x0 - 1 + hx) ----
#ifndef PVT_SKIP_HALO
        // column blends t = w0l A + w1l B per (fm row r, halo column hx, 8 channels)
        for (int task = (int)threadIdx.x; task < kTcolTasks; task += 256) {
            const int q = task & 3, rc = task >> 2;
            const int r = rc / kHC, hx = rc - r * kHC;
            const int ox = min(max(x0 - 1 + hx, 0), a.W - 1);
            const float w1r = a.rw * (float)ox;
            const int w1 = (int)w1r, w1p = w1 < a.Win - 1 ? 32 : 0;
            const float w1l = w1r - (float)w1;
            const _Float16 *p = patch + (r * kPC + (w1 - lx0)) * 32 + 8 * q;
            const h8 A = *(const h8 *)p, B = *(const h8 *)(p + w1p);
            *(h8 *)(tcol + 8 * task) =
                __builtin_elementwise_fma(B, (h8)(_Float16)w1l, A * (h8)(_Float16)(1.f - w1l));
        }
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
        __syncthreads();
        // row blends h0l t(h1) + h1l t(h1 + 1) per (halo pixel, 8 channels)
        for (int task = (int)threadIdx.x; task < kHaloPx * 4; task += 256) {
            const int q = task & 3, px = task >> 2;
            const int hy = px / kHC, hx = px - hy * kHC;
            const int oy = y0 - 1 + hy, ox = x0 - 1 + hx;
            h8 v = {};
            if (oy >= 0 && oy < a.H && ox >= 0 && ox < a.W) {
                const float h1r = a.rh * (float)oy;
                const int h1 = (int)h1r, h1p = h1 < a.Hin - 1 ? kHC * 32 : 0;
                const float h1l = h1r - (float)h1;
                const _Float16 *tp = tcol + ((h1 - ly0) * kHC + hx) * 32 + 8 * q;
                const h8 c0 = *(const h8 *)tp, c1 = *(const h8 *)(tp + h1p);
                v = __builtin_elementwise_fma(c1, (h8)(_Float16)h1l, c0 * (h8)(_Float16)(1.f - h1l));
            }
            *(h8 *)(halo + px * kCP + 8 * q) = v;
        }
#endif
        __syncthreads();
        if (tile + (int)gridDim.x < a.ntiles) fetch(a, tile + (int)gridDim.x, pk, ik, pre, pimg);
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
#pragma unroll
            for (int r = 0; r < 2; ++r) acc[r] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wa[s], bf[r], acc[r], 0, 0, 0);
        }
#else
        acc[0][0] = (float)halo[threadIdx.x];
#endif
        // ---- epilogue + head, per row ----
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int oy = y0 + 2 * wid + r, ox = x0 + n;
            // conv rows of acc[i]: (i & 3) + 8 (i >> 2) + 4 h -- 4 consecutive rows per i >> 2
            h8 act[2];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const h4 bq = *(const h4 *)(bias + 8 * g + 4 * h);
                h4 y;
#pragma unroll
                for (int j = 0; j < 4; ++j) y[j] = (_Float16)acc[r][4 * g + j];   // the conv's fp16 output
                y = y + bq;
                h4 ys;
#pragma unroll
                for (int j = 0; j < 4; ++j) ys[j] = (_Float16)((float)y[j] * a.slope);
                y = __builtin_elementwise_max(y, ys);          // LeakyReLU, slope < 1
#pragma unroll
                for (int j = 0; j < 4; ++j) act[g >> 1][4 * (g & 1) + j] = y[j];
            }
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                f16x d = {};
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) d = __builtin_amdgcn_mfma_f32_32x32x16_f16(wb[t][s2], act[s2], d, 0, 0, 0);
#ifdef PVT_SKIP_STORE
                if (oy < a.H && ox < a.W && d[0] == 1234.5f) {
#else
                if (oy < a.H && ox < a.W) {
#endif
                    _Float16 *op = a.out + (((int64_t)b * a.H + oy) * a.W + ox) * COUT;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int o0 = 32 * t + 8 * q + 4 * h;
                        if (o0 + 3 < COUT) {
                            h4 v;
#pragma unroll
                            for (int j = 0; j < 4; ++j) v[j] = (_Float16)d[4 * q + j];
                            *(h4 *)(op + o0) = v + *(const h4 *)(bias + 32 + o0);
                        }
                    }
                }
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

extern "C" int pv_decoder_tail_f16(const void *fm, const void *img, const void *w1, const float *b1, const void *w2,
                                   const float *b2, void *out, int32_t n, int32_t hin, int32_t win, int32_t cout,
                                   float slope, pv_stream_t stream) {
    if (!fm || !img || !w1 || !b1 || !w2 || !b2 || !out || n < 0 || hin < 2 || win < 2) return PV_EINVAL;
    if (cout != 20 && cout != 44) return PV_EINVAL;
    if (!(slope >= 0.f && slope < 1.f)) return PV_EINVAL;          // LeakyReLU as max(y, slope y)
    if (((uintptr_t)fm | (uintptr_t)w1 | (uintptr_t)w2) % 16 || (uintptr_t)out % 8 || (uintptr_t)img % 4)
        return PV_EALIGN;
    if (n == 0) return PV_OK;
    TailArgs a;
    a.fm = (const _Float16 *)fm;
    a.img = (const _Float16 *)img;
    a.w1 = (const _Float16 *)w1;
    a.b1 = b1;
    a.w2 = (const _Float16 *)w2;
    a.b2 = b2;
    a.out = (_Float16 *)out;
    a.N = n; a.Hin = hin; a.Win = win; a.H = 2 * hin; a.W = 2 * win;
    if ((int64_t)n * a.H * a.W * 40 >= (1ll << 31) * 16) return PV_EINVAL;
    if ((int64_t)a.H * a.W * 3 >= (1ll << 31) || (int64_t)hin * win * 32 >= (1ll << 31)) return PV_EINVAL;
    a.tiles_r = (a.H + kTR - 1) / kTR;
    a.tiles_c = (a.W + kTC - 1) / kTC;
    const int64_t nt = (int64_t)n * a.tiles_r * a.tiles_c;
    if (nt >= (1ll << 31)) return PV_EINVAL;
    a.ntiles = (int)nt;
    // ATen's area_pixel_compute_scale with align_corners: (in - 1) / (out - 1) in f32
    a.rh = (float)(hin - 1) / (float)(a.H - 1);
    a.rw = (float)(win - 1) / (float)(a.W - 1);
    a.slope = slope;
    const int64_t grid = std::min<int64_t>(nt, 2ll * cu_count_dec());   // persistent: 2 blocks per CU
    hipStream_t s = (hipStream_t)stream;
    if (cout == 20) k_decoder_tail<20><<<(unsigned)grid, 256, 0, s>>>(a);
    else k_decoder_tail<44><<<(unsigned)grid, 256, 0, s>>>(a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}
