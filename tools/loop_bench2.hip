// Microbenchmark: the byte-output vote row loop with the real kernel's rare
// paths switched in one at a time (synthetic operands, same store pattern).
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ bool exact_vote(float nx, float ny, float cx, float cy, float hx, float hy, float thr) {
    float dx = hx - cx, dy = hy - cy;
    float norm1 = sqrtf(nx * nx + ny * ny), norm2 = sqrtf(dx * dx + dy * dy);
    if ((double)norm1 < 1e-6 || (double)norm2 < 1e-6) return false;
    return (dx * nx + dy * ny) / (norm1 * norm2) > thr;
}

template <int F>   // bit0: band fix path, bit1: per-row exact-flag branch, bit2: vmask store lambda
__global__ __launch_bounds__(256) void k_loop(uint8_t *out, const float *direct, const float *coords,
                                              const float *hypo, int64_t rstep, int nwin, float tau, float gd0,
                                              int tn, int vn) {
    const int wave = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x & 63;
    __shared__ float4 recs_all[4][64];
    float4 *recs = recs_all[threadIdx.x / 64];
    recs[lane] = make_float4(lane * 0.37f, lane * 0.11f, gd0, 0.f);
    __builtin_amdgcn_wave_barrier();
    float fu[8], fv[8], fk1[8], fk2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float a = (lane * 8 + j) * 0.01f;
        fu[j] = __cosf(a); fv[j] = __sinf(a); fk1[j] = -a * 3.f; fk2[j] = a * 0.5f;
    }
    const int w = wave % nwin, vc = wave / nwin, v = vc % 9;
    const int tb = w * 512 + lane * 8;
    const uint32_t vmask = tb + 8 <= tn ? 0xffu : 0x0fu;
    uint8_t *p = out + (int64_t)vc * 29861 + (int64_t)w * 512 + lane * 8;
    auto exact_at = [&](int j, int h) {
        int t = tb + j;
        asm volatile("" : "+v"(t));
        const float2 q = *(const float2 *)(hypo + ((int64_t)h * vn + v) * 2);
        const float2 cc = *(const float2 *)(coords + (int64_t)t * 2);
        const float2 d = *(const float2 *)(direct + ((int64_t)t * vn + v) * 2);
        return exact_vote(d.x, d.y, cc.x, cc.y, q.x, q.y, 0.99f);
    };
    float4 rec = recs[0];
    for (int i = 0; i < 64; ++i) {
        float4 nrec = recs[(i + 1) & 63];
        uint32_t lo = 0, hi = 0;
        const int h = (vc / 9) + 8 * i;
        if ((F & 2) && __builtin_amdgcn_readfirstlane(__float_as_uint(rec.w))) {
#pragma unroll 1
            for (int j = 0; j < 8; ++j) {
                const uint32_t bit = ((vmask >> j & 1) && exact_at(j, h)) ? 1u : 0u;
                if (j < 4) lo |= bit << (8 * j);
                else hi |= bit << (8 * (j - 4));
            }
        } else {
            float z[8];
            float m = 3e38f;
            const float gd = rec.z;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float xr = fmaf(fu[j], rec.x, fmaf(fv[j], rec.y, fk1[j]));
                float yr = fmaf(fu[j], rec.y, fmaf(-fv[j], rec.x, fk2[j]));
                z[j] = fmaf(xr, tau, -fabsf(yr));
                m = fminf(m, fabsf(z[j]));
            }
            auto pack4 = [&](float z0, float z1, float z2, float z3) {
                uint32_t p01 = __builtin_amdgcn_perm(__float_as_uint(z1), __float_as_uint(z0), 0x0c0c0703u);
                uint32_t p23 = __builtin_amdgcn_perm(__float_as_uint(z3), __float_as_uint(z2), 0x0c0c0703u);
                uint32_t sg = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
                return (~sg & 0x80808080u) >> 7;
            };
            lo = pack4(z[0], z[1], z[2], z[3]);
            hi = pack4(z[4], z[5], z[6], z[7]);
            if (__builtin_amdgcn_ballot_w64(m <= gd)) {
                if (F & 1) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const bool u = fabsf(z[j]) <= gd;
                        if (__builtin_amdgcn_ballot_w64(u)) {
                            if (u) {
                                const uint32_t bit = 1u << (8 * (j & 3));
                                const bool e = exact_at(j, h);
                                if (j < 4) lo = e ? (lo | bit) : (lo & ~bit);
                                else hi = e ? (hi | bit) : (hi & ~bit);
                            }
                        }
                    }
                } else {
                    lo ^= 1;
                }
            }
        }
        uint8_t *q = p + rstep * i;
        if (F & 4) {
            if (vmask == 0xffu) {
                *(uint2 *)q = make_uint2(lo, hi);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (vmask >> j & 1) q[j] = (uint8_t)(((j < 4 ? lo : hi) >> (8 * (j & 3))) & 1u);
            }
        } else {
            *(uint2 *)q = make_uint2(lo, hi);
        }
        rec = nrec;
    }
}

int main() {
    const int64_t tn = 29861, vn = 9, hn = 512;
    uint8_t *out;
    float *direct, *coords, *hypo;
    if (hipMalloc(&out, hn * vn * tn + 4096) != hipSuccess) return 1;
    if (hipMalloc(&direct, tn * vn * 8) != hipSuccess || hipMalloc(&coords, tn * 8) != hipSuccess ||
        hipMalloc(&hypo, hn * vn * 8) != hipSuccess)
        return 1;
    (void)hipMemset(direct, 0, tn * vn * 8);
    (void)hipMemset(coords, 0, tn * 8);
    (void)hipMemset(hypo, 0, hn * vn * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int nwin = (int)((tn + 7 + 511) / 512);
    const int64_t rstep = 8 * vn * tn;
    const int waves = 72 * nwin;
    const int blocks = (waves + 3) / 4;
    for (int f = 0; f < 8; ++f) {
        auto go = [&]() {
            switch (f) {
#define L(F) case F: k_loop<F><<<blocks, 256>>>(out, direct, coords, hypo, rstep, nwin, 0.1425f, 1e-6f, (int)tn, (int)vn); break;
                L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7)
#undef L
            }
        };
        go();
        (void)hipEventRecord(e0);
        for (int k = 0; k < 10; ++k) go();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("features %d (fix=%d flag=%d vmask=%d): %.1f us per launch\n", f, f & 1, (f >> 1) & 1, (f >> 2) & 1,
               ms * 100);
    }
    return 0;
}
