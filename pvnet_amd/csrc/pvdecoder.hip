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

}  // namespace

extern "C" int pv_upsample2x_cat_f16(const void *x, const void *skip, void *out, int32_t n, int32_t hin,
                                     int32_t win, int32_t c1, int32_t c2, int32_t cpad, pv_stream_t stream) {
    return up2_cat<_Float16>(x, skip, out, n, hin, win, c1, c2, cpad, stream);
}

extern "C" int pv_upsample2x_cat_f32(const void *x, const void *skip, void *out, int32_t n, int32_t hin,
                                     int32_t win, int32_t c1, int32_t c2, int32_t cpad, pv_stream_t stream) {
    return up2_cat<float>(x, skip, out, n, hin, win, c1, c2, cpad, stream);
}
