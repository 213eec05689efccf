// Probe of v_mfma_f32_32x32x16_f16 on gfx950: operand / result lane maps,
// accumulation numerics (vs exact sums and vs a k-ordered fmaf chain) and
// fp16 subnormal inputs.  The vote kernels' fast test evaluates its two
// half-plane forms per (pixel, hypothesis) pair with this instruction on
// hi/lo-split fp16 operands; its error bound needs these facts.
//   hipcc --offload-arch=gfx950 -O2 -o tools/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

// A [32][16], B [16][32] row-major fp16; D [32][32] f32
__global__ __launch_bounds__(64) void k_mfma(const _Float16 *A, const _Float16 *B, const float *C, float *D) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    h8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = A[r * 16 + 8 * h + j];
        b[j] = B[(8 * h + j) * 32 + r];
    }
    f16v c;
    for (int i = 0; i < 16; ++i) c[i] = C[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r];
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    for (int i = 0; i < 16; ++i) D[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
// K = 8 form: lane l holds A[l&31][4h + j], B[4h + j][l&31], j = 0..3
__global__ __launch_bounds__(64) void k_mfma8(const _Float16 *A, const _Float16 *B, const float *C, float *D) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    h4 a, b;
    for (int j = 0; j < 4; ++j) {
        a[j] = A[r * 8 + 4 * h + j];
        b[j] = B[(4 * h + j) * 32 + r];
    }
    f16v c;
    for (int i = 0; i < 16; ++i) c[i] = C[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r];
    c = __builtin_amdgcn_mfma_f32_32x32x8f16(a, b, c, 0, 0, 0);
    for (int i = 0; i < 16; ++i) D[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}

// throughput: NM independent MFMAs per iteration, plus NV VALU ops per MFMA
// that consume its result the way the vote loop does (min, perm, sad, min3)
template <int K8, int NV>
__global__ __launch_bounds__(256) void k_rate(float *out, int iters, const _Float16 *src) {
    const int l = threadIdx.x & 63;
    h4 a4 = {src[l], src[l + 1], src[l + 2], src[l + 3]};
    h4 b4[4];
    h8 b8[4];
    for (int j = 0; j < 4; ++j) {
        b4[j] = h4{src[l + 4 + j], src[l + 5], src[l + 6], src[l + 7]};
        b8[j] = h8{src[l + 4 + j], src[l + 5], src[l + 6], src[l + 7], src[l], src[l + 1], src[l + 2], src[l + 3]};
    }
    h8 a8 = {src[l], src[l + 1], src[l + 2], src[l + 3], src[l + 4], src[l + 5], src[l + 6], src[l + 7]};
    uint32_t neg = 0;
    float mb = 1e30f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            f16v z = {};
            f16v c;
            if (K8) c = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, b4[j], z, 0, 0, 0);
            else c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, b8[j], z, 0, 0, 0);
            if (NV) {
                float m[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) m[q] = __builtin_elementwise_minimum(c[2 * q], c[2 * q + 1]);
#pragma unroll
                for (int q = 0; q < 8; q += 4) {
                    const uint32_t p01 = __builtin_amdgcn_perm(__float_as_uint(m[q + 1]), __float_as_uint(m[q]), 0x0c0c0b09u);
                    const uint32_t p23 = __builtin_amdgcn_perm(__float_as_uint(m[q + 3]), __float_as_uint(m[q + 2]), 0x0b090c0cu);
                    neg = __builtin_amdgcn_sad_u8(p01, p23, neg);
                }
#pragma unroll
                for (int q = 0; q < 8; q += 2)
                    mb = __builtin_elementwise_minimum(__builtin_elementwise_minimum(mb, fabsf(m[q])), fabsf(m[q + 1]));
            } else {
                mb = __builtin_elementwise_minimum(mb, c[j]);
            }
        }
        a4[0] = a4[0] + (_Float16)1.0f;
        a8[0] = a4[0];
    }
    out[blockIdx.x * 256 + threadIdx.x] = mb + (float)neg;
}

static float h2f(_Float16 x) { return (float)x; }

int main() {
    _Float16 *A, *B;
    float *C, *D;
    hipMallocManaged(&A, 32 * 16 * 2);
    hipMallocManaged(&B, 16 * 32 * 2);
    hipMallocManaged(&C, 32 * 32 * 4);
    hipMallocManaged(&D, 32 * 32 * 4);
    int bad = 0;
    // 1. lane maps: small integers, asymmetric B, nonzero C
    for (int r = 0; r < 32; ++r)
        for (int k = 0; k < 16; ++k) A[r * 16 + k] = (_Float16)((r * 3 + k * 7) % 11 - 5);
    for (int k = 0; k < 16; ++k)
        for (int c = 0; c < 32; ++c) B[k * 32 + c] = (_Float16)((k * 5 + c * 2) % 13 - 6);
    for (int i = 0; i < 1024; ++i) C[i] = (float)(i % 17);
    hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, A, B, C, D);
    hipDeviceSynchronize();
    for (int r = 0; r < 32; ++r)
        for (int c = 0; c < 32; ++c) {
            double s = C[r * 32 + c];
            for (int k = 0; k < 16; ++k) s += (double)h2f(A[r * 16 + k]) * h2f(B[k * 32 + c]);
            if (s != D[r * 32 + c]) ++bad;
        }
    printf("layout: %d mismatches of 1024\n", bad);

    // 2. numerics on random operands with wide magnitude spread
    srand(1);
    double worst = 0, worst_chain = 0;
    long eq_exact = 0, eq_chain = 0, eq_rev = 0, n = 0;
    for (int trial = 0; trial < 2000; ++trial) {
        for (int i = 0; i < 512; ++i) {
            float m = ldexpf(1.f, rand() % 24 - 14);
            A[i] = (_Float16)(m * ((rand() / (float)RAND_MAX) * 2.f - 1.f));
        }
        for (int i = 0; i < 512; ++i) {
            float m = ldexpf(1.f, rand() % 20 - 8);
            B[i] = (_Float16)(m * ((rand() / (float)RAND_MAX) * 2.f - 1.f));
        }
        for (int i = 0; i < 1024; ++i) C[i] = (trial & 1) ? ((rand() / (float)RAND_MAX) * 2.f - 1.f) * 1000.f : 0.f;
        hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, A, B, C, D);
        hipDeviceSynchronize();
        for (int r = 0; r < 32; ++r)
            for (int c = 0; c < 32; ++c) {
                double s = C[r * 32 + c], mag = fabs((double)C[r * 32 + c]);
                float chain = C[r * 32 + c], rev = C[r * 32 + c];
                for (int k = 0; k < 16; ++k) {
                    const double p = (double)h2f(A[r * 16 + k]) * h2f(B[k * 32 + c]);
                    s += p;
                    mag += fabs(p);
                    chain = fmaf(h2f(A[r * 16 + k]), h2f(B[k * 32 + c]), chain);
                }
                for (int k = 15; k >= 0; --k) rev = fmaf(h2f(A[r * 16 + k]), h2f(B[k * 32 + c]), rev);
                const float d = D[r * 32 + c];
                if (mag > 0) {
                    worst = fmax(worst, fabs(d - s) / mag / ldexp(1.0, -24));
                    worst_chain = fmax(worst_chain, fabs((double)chain - s) / mag / ldexp(1.0, -24));
                }
                eq_exact += d == (float)s;
                eq_chain += d == chain;
                eq_rev += d == rev;
                ++n;
            }
    }
    printf("numerics: max |D - exact| / sum|terms| = %.3f u (fmaf chain: %.3f u); D == round(exact) %.4f, "
           "== k-ordered fmaf chain %.4f, == reversed chain %.4f (n=%ld)\n",
           worst, worst_chain, eq_exact / (double)n, eq_chain / (double)n, eq_rev / (double)n, n);

    // 3. fp16 subnormal inputs (2^-24 .. 2^-15) times normals: flushed or kept?
    memset(A, 0, 32 * 16 * 2);
    memset(B, 0, 16 * 32 * 2);
    for (int r = 0; r < 32; ++r) A[r * 16 + 0] = (_Float16)ldexpf((float)(r + 1), -24);
    for (int c = 0; c < 32; ++c) B[0 * 32 + c] = (_Float16)(float)(c + 1);
    for (int i = 0; i < 1024; ++i) C[i] = 0.f;
    hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, A, B, C, D);
    hipDeviceSynchronize();
    bad = 0;
    for (int r = 0; r < 32; ++r)
        for (int c = 0; c < 32; ++c)
            if (D[r * 32 + c] != ldexpf((float)(r + 1), -24) * (float)(c + 1)) ++bad;
    printf("subnormal fp16 A operands: %d of 1024 wrong (0 = kept exactly)%s\n", bad,
           bad ? "" : "");
    printf("D[0][0] = %g (expect %g)\n", D[0], ldexpf(1.f, -24));

    // 4. K = 8 lane map
    for (int r = 0; r < 32; ++r)
        for (int k = 0; k < 8; ++k) A[r * 8 + k] = (_Float16)((r * 3 + k * 7) % 11 - 5);
    for (int k = 0; k < 8; ++k)
        for (int c = 0; c < 32; ++c) B[k * 32 + c] = (_Float16)((k * 5 + c * 2) % 13 - 6);
    for (int i = 0; i < 1024; ++i) C[i] = (float)(i % 17);
    hipLaunchKernelGGL(k_mfma8, dim3(1), dim3(64), 0, 0, A, B, C, D);
    hipDeviceSynchronize();
    bad = 0;
    for (int r = 0; r < 32; ++r)
        for (int c = 0; c < 32; ++c) {
            double s = C[r * 32 + c];
            for (int k = 0; k < 8; ++k) s += (double)h2f(A[r * 8 + k]) * h2f(B[k * 32 + c]);
            if (s != D[r * 32 + c]) ++bad;
        }
    printf("layout 32x32x8f16: %d mismatches of 1024\n", bad);

    // 5. rates: 256 CUs x 4 blocks of 4 waves, 4 MFMAs per iteration
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *out;
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 2000;
    auto run = [&](const char *name, void (*kern)(float *, int, const _Float16 *), int bpc) {
        hipLaunchKernelGGL(kern, dim3(cus * bpc), dim3(256), 0, 0, out, 10, A);
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(cus * bpc), dim3(256), 0, 0, out, iters, A);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        // per SIMD: bpc waves, iters * 4 MFMAs each; cycles at 2.4 GHz
        const double mfma_per_simd = (double)bpc * iters * 4;
        printf("%-34s %2d waves/SIMD: %.3f ms, %.1f cyc per MFMA per SIMD (2.4 GHz)\n", name, bpc, ms,
               ms * 1e-3 * 2.4e9 / mfma_per_simd);
    };
    for (int bpc : {1, 4}) {
        run("32x32x16 f16 alone", k_rate<0, 0>, bpc);
        run("32x32x8 f16 alone", k_rate<1, 0>, bpc);
        run("32x32x16 f16 + vote VALU", k_rate<0, 1>, bpc);
        run("32x32x8 f16 + vote VALU", k_rate<1, 1>, bpc);
    }
    return 0;
}
