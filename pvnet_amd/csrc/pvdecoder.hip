// PVNet decoder step on gfx950: the x2 bilinear upsampling (align_corners,
// nn.UpsamplingBilinear2d) of a channels-last fp16 feature map fused with
// the concatenation that follows it (torch.cat([up(fm), skip], 1)) and a
// zero channel pad, in one memory pass -- MR:66-75
// (lib/networks/model_repository.py), where the decoder runs the upsampling
// and the cat as two full-resolution passes and the last cat has 35 channels
// (no 16-byte vector path for the convolution after it).  Exported through
// include/pvvote.h.
//
// Thread = one output pixel x 8 channels (one 16-byte store); the upsampled
// channels come from four 16-byte loads of the input's neighbours, blended
// in f32 exactly as ATen's upsample_bilinear2d_nhwc_out_frame does
// (rheight = (Hin-1)/(Hout-1), src = r * dst, lambdas in f32, the same
// association), then rounded to fp16; skip channels are copied; channels past
// C1 + C2 are zero.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pvvote.h"

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(256) void k_up2_cat_f16(const _Float16 *__restrict__ x, const _Float16 *__restrict__ skip,
                                                     _Float16 *__restrict__ out, int N, int Hin, int Win, int C1,
                                                     int C2, int Cpad, float rh, float rw) {
    const int Hout = 2 * Hin, Wout = 2 * Win, cp8 = Cpad / 8, c18 = C1 / 8;
    const int64_t total = (int64_t)N * Hout * Wout * cp8;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int k = (int)(i % cp8);
        const int64_t pix = i / cp8;                       // n * Hout * Wout + oy * Wout + ox
        const int ox = (int)(pix % Wout);
        const int64_t r = pix / Wout;
        const int oy = (int)(r % Hout), n = (int)(r / Hout);
        h8 v;
        if (k < c18) {
            const float h1r = rh * (float)oy;
            const int h1 = (int)h1r, h1p = h1 < Hin - 1 ? 1 : 0;
            const float h1l = h1r - (float)h1, h0l = 1.f - h1l;
            const float w1r = rw * (float)ox;
            const int w1 = (int)w1r, w1p = w1 < Win - 1 ? 1 : 0;
            const float w1l = w1r - (float)w1, w0l = 1.f - w1l;
            const _Float16 *p = x + (((int64_t)n * Hin + h1) * Win + w1) * C1 + 8 * k;
            const int64_t dw = (int64_t)w1p * C1, dh = (int64_t)h1p * Win * C1;
            const h8 a = *(const h8 *)p, b = *(const h8 *)(p + dw), c = *(const h8 *)(p + dh),
                     d = *(const h8 *)(p + dh + dw);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                v[j] = (_Float16)(h0l * (w0l * (float)a[j] + w1l * (float)b[j]) +
                                  h1l * (w0l * (float)c[j] + w1l * (float)d[j]));
        } else {
            const int c0 = 8 * (k - c18);
            const _Float16 *q = skip + (((int64_t)n * Hout + oy) * Wout + ox) * C2 + c0;
            if (C2 % 8 == 0 && c0 + 8 <= C2) {
                v = *(const h8 *)q;
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = c0 + j < C2 ? q[j] : (_Float16)0.f;
            }
        }
        *(h8 *)(out + pix * Cpad + 8 * k) = v;
    }
}

}  // namespace

extern "C" int pv_upsample2x_cat_f16(const void *x, const void *skip, void *out, int32_t n, int32_t hin,
                                     int32_t win, int32_t c1, int32_t c2, int32_t cpad, pv_stream_t stream) {
    if (!x || !out || n < 0 || hin <= 0 || win <= 0 || c1 <= 0 || c2 < 0 || (c2 > 0 && !skip)) return PV_EINVAL;
    if (c1 % 8 || cpad % 8 || cpad < c1 + c2) return PV_EINVAL;
    // 16-byte vectors: every pixel's channels start 16-byte aligned
    if (((uintptr_t)x | (uintptr_t)out) % 16 || (c2 % 8 == 0 && c2 > 0 && (uintptr_t)skip % 16)) return PV_EINVAL;
    if (n == 0) return PV_OK;
    const int hout = 2 * hin, wout = 2 * win;
    // ATen's area_pixel_compute_scale with align_corners: (in - 1) / (out - 1) in f32
    const float rh = (float)(hin - 1) / (float)(hout - 1), rw = (float)(win - 1) / (float)(wout - 1);
    const int64_t total = (int64_t)n * hout * wout * (cpad / 8);
    const int64_t blocks = (total + 255) / 256;
    const unsigned grid = (unsigned)(blocks < 262144 ? blocks : 262144);
    k_up2_cat_f16<<<grid, 256, 0, (hipStream_t)stream>>>((const _Float16 *)x, (const _Float16 *)skip, (_Float16 *)out,
                                                         n, hin, win, c1, c2, cpad, rh, rw);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}
