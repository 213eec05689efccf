// PVNet decoder step on gfx950: the x2 bilinear upsampling (align_corners,
// nn.UpsamplingBilinear2d) of a channels-last fp16 or f32 feature map fused with
// the concatenation that follows it (torch.cat([up(fm), skip], 1)) and a
// zero channel pad, in one memory pass -- MR:66-75
// (lib/networks/model_repository.py), where the decoder runs the upsampling
// and the cat as two full-resolution passes and the last cat has 35 channels
// (no 16-byte vector path for the convolution after it).  Exported through
// include/pvvote.h.
//
// Thread = one output pixel x 16 bytes of channels (8 fp16 / 4 f32), a block
// 256 of them along one output row (32-bit index math); the upsampled
// channels come from four 16-byte loads of the input's neighbours, blended
// in f32 as ATen's upsample_bilinear2d_nhwc_out_frame does
// (rheight = (Hin-1)/(Hout-1), src = r * dst, lambdas in f32, the same
// association), then rounded to the map's type; skip channels are copied; channels past
// C1 + C2 are zero.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/pvvote.h"

namespace {

// V lanes of T in one 16-byte vector (8 fp16 or 4 f32 channels)
template <typename T, int V>
struct Vec { typedef T type __attribute__((ext_vector_type(V))); };

template <typename T>
__global__ __launch_bounds__(256) void k_up2_cat(const T *__restrict__ x, const T *__restrict__ skip,
                                                 T *__restrict__ out, int N, int Hin, int Win, int C1, int C2,
                                                 int Cpad, float rh, float rw) {
    constexpr int V = 16 / sizeof(T);
    typedef typename Vec<T, V>::type vT;
    const int Hout = 2 * Hin, Wout = 2 * Win, cpv = Cpad / V, c1v = C1 / V;
    // block (x, y): 256 chunks of output row y (n * Hout + oy); 32-bit index math
    const int j = (int)(blockIdx.x * 256 + threadIdx.x);
    if (j >= Wout * cpv) return;
    const int k = j % cpv, ox = j / cpv;
    for (int row = (int)blockIdx.y; row < N * Hout; row += (int)gridDim.y) {
        const int oy = row % Hout, n = row / Hout;
        const int64_t pix = (int64_t)row * Wout + ox;
        vT v;
        if (k < c1v) {
            const float h1r = rh * (float)oy;
            const int h1 = (int)h1r, h1p = h1 < Hin - 1 ? 1 : 0;
            const float h1l = h1r - (float)h1, h0l = 1.f - h1l;
            const float w1r = rw * (float)ox;
            const int w1 = (int)w1r, w1p = w1 < Win - 1 ? 1 : 0;
            const float w1l = w1r - (float)w1, w0l = 1.f - w1l;
            const T *p = x + (((int64_t)n * Hin + h1) * Win + w1) * C1 + V * k;
            const int64_t dw = (int64_t)w1p * C1, dh = (int64_t)h1p * Win * C1;
            const vT a = *(const vT *)p, b = *(const vT *)(p + dw), c = *(const vT *)(p + dh),
                     d = *(const vT *)(p + dh + dw);
#pragma unroll
            for (int q = 0; q < V; ++q)
                v[q] = (T)(h0l * (w0l * (float)a[q] + w1l * (float)b[q]) + h1l * (w0l * (float)c[q] + w1l * (float)d[q]));
        } else {
            const int c0 = V * (k - c1v);
            const T *q = skip + pix * C2 + c0;
            if (C2 % V == 0 && c0 + V <= C2) {
                v = *(const vT *)q;
            } else {
#pragma unroll
                for (int e = 0; e < V; ++e) v[e] = c0 + e < C2 ? q[e] : (T)0.f;
            }
        }
        *(vT *)(out + pix * Cpad + V * k) = v;
    }
}

template <typename T>
int up2_cat(const void *x, const void *skip, void *out, int32_t n, int32_t hin, int32_t win, int32_t c1, int32_t c2,
            int32_t cpad, pv_stream_t stream) {
    constexpr int V = 16 / sizeof(T);
    if (!x || !out || n < 0 || hin <= 0 || win <= 0 || c1 <= 0 || c2 < 0 || (c2 > 0 && !skip)) return PV_EINVAL;
    if (c1 % V || cpad % V || cpad < c1 + c2) return PV_EINVAL;
    // 16-byte vectors: every pixel's channels start 16-byte aligned
    if (((uintptr_t)x | (uintptr_t)out) % 16 || (c2 % V == 0 && c2 > 0 && (uintptr_t)skip % 16)) return PV_EINVAL;
    if (n == 0) return PV_OK;
    const int hout = 2 * hin, wout = 2 * win;
    // ATen's area_pixel_compute_scale with align_corners: (in - 1) / (out - 1) in f32
    const float rh = (float)(hin - 1) / (float)(hout - 1), rw = (float)(win - 1) / (float)(wout - 1);
    if ((int64_t)wout * (cpad / V) >= (1ll << 31) || (int64_t)n * hout >= (1ll << 31)) return PV_EINVAL;
    const int rows = n * hout;
    const dim3 grid((unsigned)((wout * (cpad / V) + 255) / 256), (unsigned)(rows < 65535 ? rows : 65535));
    k_up2_cat<T><<<grid, 256, 0, (hipStream_t)stream>>>((const T *)x, (const T *)skip, (T *)out, n, hin, win, c1, c2,
                                                        cpad, rh, rw);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}

// --------------------------------------------------------------------------
// Convolution epilogues (the inference form's only passes besides MIOpen's
// convolutions): the folded BatchNorm's bias, the residual add and the
// activation of a BasicBlock (RN:41-70) or a conv-BN-(Leaky)ReLU stage
// (MR:22-58), in one pass over a channels-last map, optionally writing the
// result beside a skip map (the torch.cat that follows fc, MR:66-67).
// Roundings follow ATen's sequence for the unfused modules: y = x + b
// rounded to T, then + (r + rb) with (r + rb) rounded to T, then the
// activation (relu exact; leaky: y > 0 ? y : y * slope, rounded).
// Thread = 16 bytes of channels of one pixel (8 fp16 / 4 f32).
// --------------------------------------------------------------------------
enum { kActNone = 0, kActRelu = 1, kActLeaky = 2 };

template <typename T>
__global__ __launch_bounds__(256) void k_epilogue(const T *__restrict__ x, const T *__restrict__ bias,
                                                  const T *__restrict__ res, const T *__restrict__ rbias,
                                                  const T *__restrict__ skip, T *out, int64_t P, int C1, int C2,
                                                  int act, float slope) {
    constexpr int V = 16 / sizeof(T);
    typedef typename Vec<T, V>::type vT;
    const int c1v = C1 / V, cv = (C1 + C2) / V, Co = C1 + C2;
    const uint32_t n = (uint32_t)(P * cv);        // < 2^31 (host): 32-bit division, not 64-bit
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const uint32_t p32 = i / (uint32_t)cv;
        const int k = (int)(i - p32 * (uint32_t)cv);
        const int64_t p = p32;
        vT v;
        if (k < c1v) {
            v = *(const vT *)(x + p * C1 + V * k);
            const vT b = *(const vT *)(bias + V * k);
            vT r, rb;
            if (res) {
                r = *(const vT *)(res + p * C1 + V * k);
                if (rbias) rb = *(const vT *)(rbias + V * k);
            }
#pragma unroll
            for (int q = 0; q < V; ++q) {
                T y = (T)((float)v[q] + (float)b[q]);
                if (res) {
                    const T rr = rbias ? (T)((float)r[q] + (float)rb[q]) : r[q];
                    y = (T)((float)y + (float)rr);
                }
                if (act == kActRelu) y = (float)y > 0.f ? y : (T)0.f;
                else if (act == kActLeaky) y = (float)y > 0.f ? y : (T)((float)y * slope);
                v[q] = y;
            }
        } else {
            v = *(const vT *)(skip + p * C2 + V * (k - c1v));
        }
        *(vT *)(out + p * Co + V * k) = v;
    }
}

template <typename T>
int epilogue(const void *x, const void *bias, const void *res, const void *rbias, const void *skip, void *out,
             int64_t P, int32_t c1, int32_t c2, int32_t act, float slope, pv_stream_t stream) {
    constexpr int V = 16 / sizeof(T);
    if (!x || !bias || !out || P < 0 || c1 <= 0 || c2 < 0 || (c2 > 0 && !skip) || (rbias && !res)) return PV_EINVAL;
    if (act < kActNone || act > kActLeaky || c1 % V || c2 % V) return PV_EINVAL;
    if (((uintptr_t)x | (uintptr_t)bias | (uintptr_t)res | (uintptr_t)rbias | (uintptr_t)skip | (uintptr_t)out) % 16)
        return PV_EALIGN;
    if (c2 > 0 && out == x) return PV_EINVAL;     // in place only without the skip channels
    if (P == 0) return PV_OK;
    const int64_t n = P * ((c1 + c2) / V);
    if (n >= (1ll << 31)) return PV_EINVAL;       // the kernel's 32-bit element index
    const int64_t blocks = (n + 255) / 256;
    k_epilogue<T><<<(unsigned)(blocks < 256 * 64 ? blocks : 256 * 64), 256, 0, (hipStream_t)stream>>>(
        (const T *)x, (const T *)bias, (const T *)res, (const T *)rbias, (const T *)skip, (T *)out, P, c1, c2, act,
        slope);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}

// --------------------------------------------------------------------------
// The stem's tail (RN:139-142 conv1 -> bn1 -> relu = x2s, then maxpool
// 3x3 / 2 / pad 1; RN:201-204): x2s = relu(x + b) written once and the pooled
// map from it in the same pass.  Thread = 16 bytes of channels of one pooled
// pixel: it reads its 3x3 window of the conv output, writes the 2x2 of x2s it
// owns (rows 2py, 2py + 1, columns 2px, 2px + 1 -- the owned blocks tile x2s)
// and the window's max.  Roundings as k_epilogue; the max is exact, so both
// maps equal ATen's bias add + ReLU + max_pool2d bit for bit.  Pool-only form
// (bias and x2s NULL: x is x2s already, from pv_stem_conv_f16): the max alone.
// --------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_relu_pool(const T *__restrict__ x, const T *__restrict__ bias,
                                                   T *__restrict__ x2s, T *__restrict__ pool, int N, int H, int W,
                                                   int C, int Ho, int Wo) {
    constexpr int V = 16 / sizeof(T);
    typedef typename Vec<T, V>::type vT;
    // 32-bit index arithmetic (the host keeps total < 2^31): a 64-bit
    // division is a long software sequence on the GPU, three of them per
    // element made this pass index-bound
    const uint32_t cv = (uint32_t)(C / V);
    const uint32_t total = (uint32_t)N * Ho * Wo * cv;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
        const uint32_t p = i / cv, k = i - p * cv;
        const uint32_t q = p / (uint32_t)Wo, px = p - q * (uint32_t)Wo;
        const uint32_t b = q / (uint32_t)Ho, py = q - b * (uint32_t)Ho;
        vT bv = {};
        if (bias) bv = *(const vT *)(bias + V * k);
        vT m;
#pragma unroll
        for (int e = 0; e < V; ++e) m[e] = (T)(-INFINITY);
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy) {
            const int iy = 2 * (int)py + dy;
            if (iy < 0 || iy >= H) continue;
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const int ix = 2 * (int)px + dx;
                if (ix < 0 || ix >= W) continue;
                const int64_t off = (((int64_t)b * H + iy) * W + ix) * C + V * k;
                vT v = *(const vT *)(x + off);
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    if (bias) {
                        const T y = (T)((float)v[e] + (float)bv[e]);
                        v[e] = (float)y > 0.f ? y : (T)0.f;
                    }
                    m[e] = (float)v[e] > (float)m[e] ? v[e] : m[e];
                }
                if (bias && dy >= 0 && dx >= 0) *(vT *)(x2s + off) = v;
            }
        }
        *(vT *)(pool + (int64_t)p * C + V * k) = m;
    }
}

template <typename T>
int relu_pool(const void *x, const void *bias, void *x2s, void *pool, int32_t n, int32_t h, int32_t w, int32_t c,
              pv_stream_t stream) {
    constexpr int V = 16 / sizeof(T);
    if (!x || !pool || n < 0 || h <= 0 || w <= 0 || c <= 0 || c % V) return PV_EINVAL;
    if (!bias != !x2s) return PV_EINVAL;   // both NULL: pool-only
    if (((uintptr_t)x | (uintptr_t)bias | (uintptr_t)x2s | (uintptr_t)pool) % 16) return PV_EALIGN;
    if (x2s == x || pool == x || (x2s && pool == x2s)) return PV_EINVAL;
    if (n == 0) return PV_OK;
    const int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;     // kernel 3, stride 2, pad 1
    const int64_t total = (int64_t)n * ho * wo * (c / V);
    if (total >= (1ll << 31)) return PV_EINVAL;   // the kernel's 32-bit element index
    const int64_t blocks = (total + 255) / 256;
    k_relu_pool<T><<<(unsigned)(blocks < 256 * 64 ? blocks : 256 * 64), 256, 0, (hipStream_t)stream>>>(
        (const T *)x, (const T *)bias, (T *)x2s, (T *)pool, n, h, w, c, ho, wo);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}

// --------------------------------------------------------------------------
// The network's head, convraw after its 3x3 convolution (MR:53-58): the
// folded BN bias + LeakyReLU(0.1) and the 1x1 convolution to seg_dim +
// ver_dim channels with its bias, in one pass -- 32 channels in, 20 (or 44,
// PVnet(42, 2)) out per pixel, instead of three passes over the full-
// resolution map and a separate 1x1 convolution.
// The 1x1 convolution is a [cout x 32] x [32 x pixels] product on the matrix
// cores: a wave takes 32 pixels, A = the weights (outputs x channels, fixed
// per lane for the whole kernel), B = the pixels' activations, D = [32
// outputs x 32 pixels]; fp16 maps use v_mfma_f32_32x32x8_f16 (fp16 weights
// and activations, exact products, f32 sums: MIOpen's fp16 convolution
// arithmetic up to summation order), f32 maps v_mfma_f32_32x32x2_f32.  The
// K order is permuted so that lane half h holds channels 16h .. 16h + 15 of
// its pixel (two / four 16-byte loads of contiguous channels); lane l's
// results are 4-channel runs of pixel l % 32 (8- / 16-byte stores).
// Roundings: t = leaky(x + b1) as k_epilogue; the sum rounded to T, + b2
// rounded to T (ATen's bias add).
// --------------------------------------------------------------------------
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f16x __attribute__((ext_vector_type(16)));

template <typename T, int COUT>
__global__ __launch_bounds__(256) void k_head(const T *__restrict__ x, const float *__restrict__ b1,
                                              const float *__restrict__ w2, const float *__restrict__ b2,
                                              T *__restrict__ out, int64_t P, float slope) {
    constexpr int CIN = 32;
    constexpr bool F16 = sizeof(T) == 2;
    constexpr int MT = (COUT + 31) / 32;             // 32-output tiles
    constexpr int KS = F16 ? 4 : 16;                 // MFMA K steps over the 32 channels
    const int lane = (int)(threadIdx.x & 63), m = lane & 31, h = lane >> 5;
    // channel of (lane half h, step s, j): 16 h + 4 s + j (fp16), 16 h + s (f32)
    // A fragments (weights): output m + 32 t, the lane's channels
    typedef typename std::conditional<F16, h4, float>::type AF;
    AF wa[MT][KS];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int s2 = 0; s2 < KS; ++s2) {
            const int o = m + 32 * t;
            if constexpr (F16) {
                h4 v;
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = o < COUT ? (_Float16)w2[o * CIN + 16 * h + 4 * s2 + j] : (_Float16)0.f;
                wa[t][s2] = v;
            } else {
                wa[t][s2] = o < COUT ? w2[o * CIN + 16 * h + s2] : 0.f;
            }
        }
    float bb[16], bo[MT][16];
#pragma unroll
    for (int c = 0; c < 16; ++c) bb[c] = (float)(T)b1[16 * h + c];
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int o = 32 * t + 8 * (i / 4) + 4 * h + i % 4;
            bo[t][i] = o < COUT ? (float)(T)b2[o] : 0.f;
        }
    const int64_t ngroups = (P + 31) / 32;
    const int wave = (int)(blockIdx.x * 4 + (threadIdx.x >> 6)), nwaves = (int)(gridDim.x * 4);
    for (int64_t g = wave; g < ngroups; g += nwaves) {
        const int64_t p = g * 32 + m;
        const bool ok = p < P;
        // the pixel's 16 channels of this lane half, activated (B fragments)
        constexpr int V = 16 / sizeof(T);
        typedef typename Vec<T, V>::type vT;
        float act[16];
#pragma unroll
        for (int q = 0; q < 16 / V; ++q) {
            vT v = {};
            if (ok) v = *(const vT *)(x + p * CIN + 16 * h + V * q);
#pragma unroll
            for (int j = 0; j < V; ++j) {
                const T y = (T)((float)v[j] + bb[V * q + j]);
                act[V * q + j] = (float)((float)y > 0.f ? y : (T)((float)y * slope));
            }
        }
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            f16x d = {};
#pragma unroll
            for (int s2 = 0; s2 < KS; ++s2) {
                if constexpr (F16) {
                    const h4 bv = {(_Float16)act[4 * s2], (_Float16)act[4 * s2 + 1], (_Float16)act[4 * s2 + 2],
                                   (_Float16)act[4 * s2 + 3]};
                    d = __builtin_amdgcn_mfma_f32_32x32x8f16(wa[t][s2], bv, d, 0, 0, 0);
                } else {
                    d = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[t][s2], act[s2], d, 0, 0, 0);
                }
            }
            // d[i]: output (i % 4) + 8 (i / 4) + 4 h of tile t, pixel g * 32 + (lane & 31)
            if (ok) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int o0 = 32 * t + 8 * q + 4 * h;
                    if (o0 + 3 < COUT) {
                        typedef typename Vec<T, 4>::type v4;
                        v4 r;
#pragma unroll
                        for (int j = 0; j < 4; ++j) r[j] = (T)((float)(T)d[4 * q + j] + bo[t][4 * q + j]);
                        *(v4 *)(out + p * COUT + o0) = r;
                    }
                }
            }
        }
    }
}

template <typename T>
int head(const void *x, const float *b1, const float *w2, const float *b2, void *out, int64_t P, int32_t cin,
         int32_t cout, float slope, pv_stream_t stream) {
    if (!x || !b1 || !w2 || !b2 || !out || P < 0) return PV_EINVAL;
    if ((uintptr_t)x % 16 || (uintptr_t)out % 8) return PV_EALIGN;
    if (P == 0) return PV_OK;
    const int64_t blocks = (P + 127) / 128;          // 4 waves x 32 pixels per block and pass
    const unsigned g = (unsigned)(blocks < 256 * 8 ? blocks : 256 * 8);
    hipStream_t s = (hipStream_t)stream;
    if (cin == 32 && cout == 20)
        k_head<T, 20><<<g, 256, 0, s>>>((const T *)x, b1, w2, b2, (T *)out, P, slope);
    else if (cin == 32 && cout == 44)
        k_head<T, 44><<<g, 256, 0, s>>>((const T *)x, b1, w2, b2, (T *)out, P, slope);
    else
        return PV_EINVAL;
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}

}  // namespace

extern "C" int pv_conv_epilogue_f16(const void *x, const void *bias, const void *res, const void *rbias,
                                    const void *skip, void *out, int64_t P, int32_t c1, int32_t c2, int32_t act,
                                    float slope, pv_stream_t stream) {
    return epilogue<_Float16>(x, bias, res, rbias, skip, out, P, c1, c2, act, slope, stream);
}

extern "C" int pv_conv_epilogue_f32(const void *x, const void *bias, const void *res, const void *rbias,
                                    const void *skip, void *out, int64_t P, int32_t c1, int32_t c2, int32_t act,
                                    float slope, pv_stream_t stream) {
    return epilogue<float>(x, bias, res, rbias, skip, out, P, c1, c2, act, slope, stream);
}

extern "C" int pv_head_f16(const void *x, const float *b1, const float *w2, const float *b2, void *out, int64_t P,
                           int32_t cin, int32_t cout, float slope, pv_stream_t stream) {
    return head<_Float16>(x, b1, w2, b2, out, P, cin, cout, slope, stream);
}

extern "C" int pv_head_f32(const void *x, const float *b1, const float *w2, const float *b2, void *out, int64_t P,
                           int32_t cin, int32_t cout, float slope, pv_stream_t stream) {
    return head<float>(x, b1, w2, b2, out, P, cin, cout, slope, stream);
}

extern "C" int pv_upsample2x_cat_f16(const void *x, const void *skip, void *out, int32_t n, int32_t hin,
                                     int32_t win, int32_t c1, int32_t c2, int32_t cpad, pv_stream_t stream) {
    return up2_cat<_Float16>(x, skip, out, n, hin, win, c1, c2, cpad, stream);
}

extern "C" int pv_upsample2x_cat_f32(const void *x, const void *skip, void *out, int32_t n, int32_t hin,
                                     int32_t win, int32_t c1, int32_t c2, int32_t cpad, pv_stream_t stream) {
    return up2_cat<float>(x, skip, out, n, hin, win, c1, c2, cpad, stream);
}

extern "C" int pv_relu_maxpool_f16(const void *x, const void *bias, void *x2s, void *pool, int32_t n, int32_t h,
                                   int32_t w, int32_t c, pv_stream_t stream) {
    return relu_pool<_Float16>(x, bias, x2s, pool, n, h, w, c, stream);
}

extern "C" int pv_relu_maxpool_f32(const void *x, const void *bias, void *x2s, void *pool, int32_t n, int32_t h,
                                   int32_t w, int32_t c, pv_stream_t stream) {
    return relu_pool<float>(x, bias, x2s, pool, n, h, w, c, stream);
}
