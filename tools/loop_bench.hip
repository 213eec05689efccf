// Microbenchmark: the byte-output vote loop in isolation (synthetic operands):
// per row 8 pixels x (5 FMAs, |z| min, sign-byte pack) + one 8-byte store.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int MODE>   // 0 compute+store, 1 compute only, 2 store only
__global__ __launch_bounds__(256) void k_loop(uint8_t *out, int64_t rstep, int nrows, int nwin, float tau, float gd0) {
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
    const int w = wave % nwin, vc = wave / nwin;
    uint8_t *p = out + (int64_t)vc * 29861 + (int64_t)w * 512 + lane * 8;
    float4 rec = recs[0];
    for (int i = 0; i < nrows; ++i) {
        float4 nrec = recs[(i + 1) & 63];
        uint32_t lo = i, hi = i;
        float m = 3e38f;
        if (MODE != 2) {
            float z[8];
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
            if (__builtin_amdgcn_ballot_w64(m <= rec.z)) { lo ^= 1; }
        }
        if (MODE != 1 || lo == 0x12345678u) *(uint2 *)(p + rstep * i) = make_uint2(lo, hi);
        rec = nrec;
    }
}

int main() {
    const int64_t tn = 29861, vn = 9, hn = 512;
    uint8_t *out;
    if (hipMalloc(&out, hn * vn * tn + 4096) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int nwin = (int)((tn + 7 + 511) / 512);
    const int64_t rstep = 8 * vn * tn;
    const int waves = 72 * nwin;
    const int blocks = (waves + 3) / 4;
    for (int mode = 0; mode < 3; ++mode) {
        for (int r = 0; r < 2; ++r) {
            auto go = [&]() {
                if (mode == 0) k_loop<0><<<blocks, 256>>>(out, rstep, 64, nwin, 0.1425f, 1e-6f);
                if (mode == 1) k_loop<1><<<blocks, 256>>>(out, rstep, 64, nwin, 0.1425f, 1e-6f);
                if (mode == 2) k_loop<2><<<blocks, 256>>>(out, rstep, 64, nwin, 0.1425f, 1e-6f);
            };
            go();
            (void)hipEventRecord(e0);
            for (int k = 0; k < 10; ++k) go();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r) printf("mode %d (%s): %.1f us per launch\n", mode,
                          mode == 0 ? "compute+store" : mode == 1 ? "compute only" : "store only", ms * 100);
        }
    }
    return 0;
}
